# Fused pair timing only (tools/convbench x3f, ABL 0 / 64), Mode N shapes: quick A/B of epilogue forms.
# usage: bash tools/archive/cb_f67q.sh <tag>
export TMPDIR=/tmp
T=${1:-f67q}; O=gpurun_out/$T; mkdir -p $O
for shp in "1 384 512" "1 288 256"; do
  for abl in 0 64 0; do
    echo "== $shp ABL=$abl" >> $O/cb.txt
    ISLPOSE_X3_ABL=$abl timeout -k 10 60 tools/convbench $shp 46 82 32 100 x3f 2 >> $O/cb.txt 2>&1 || exit 1
  done
done
grep -E "^==|round 1" $O/cb.txt
