# wino_f16 vs conv_x3 per shape, and the Winograd kernel's stage ablations (ISLPOSE_W2_ABL:
# 1 no MFMA, 2 no transform, 4 no filter loads, 8 no raw DMA, 16 no epilogue).
# usage: bash tools/w2_abl.sh <tag>   (gpurun_out/<tag>)
export TMPDIR=/tmp
T=${1:-w2abl}; O=gpurun_out/$T; mkdir -p $O
run() { echo "== $*" >> $O/abl.txt; timeout -k 10 120 "$@" >> $O/abl.txt 2>&1; }
for shape in "3 128 128 46 82 32" "3 384 128 46 82 32" "3 256 256 92 164 32" "3 512 512 46 82 32"; do
  run tools/convbench $shape 10 x3,w2 2 || exit 1
  for k in 1 2 4 8 16 6 12 14 3 31; do
    ISLPOSE_W2_ABL=$k run tools/convbench $shape 10 w2 1 || exit 1
  done
done
cat $O/abl.txt | grep -E "==|round"
