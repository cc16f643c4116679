# Fixed cost of a small-grid x3 launch (development build, ISLPOSE_X3_ABL): 7 = no K-loop
# work (prologue + epilogue + launch), + 16 no prologue staging, + 32 no bias load, + 64 no
# epilogue.  usage: bash tools/archive/gpu_abl2.sh <tag>
T=${1:-abl2}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for s in "3 128 128 23 41 32" "3 128 128 23 41 1" "3 128 128 46 82 32"; do
  for a in 0 7 23 39 71 87 119; do
    echo "== $s abl=$a" >> $O/abl.txt
    ISLPOSE_X3_ABL=$a ISLPOSE_X3_UNION=0 timeout -k 10 60 tools/convbench $s 40 x3 2 >> $O/abl.txt 2>&1 || { tail $O/abl.txt; exit 1; }
  done
done
grep "==\|round 1" $O/abl.txt
