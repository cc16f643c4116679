# A/B of x3 kernel variants (ISLPOSE_X3_VAR) on the conv microbenchmark. usage: bash tools/gpu_cbvar.sh <tag> <vars...>
set -o pipefail
export TMPDIR=/tmp
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
for s in "3 128 128 46 82 32" "3 384 128 46 82 32" "3 96 96 46 82 32" "3 256 256 92 164 32" "3 64 64 368 656 32" "1 384 512 46 82 32" "3 512 512 46 82 32"; do
  for v in "$@"; do
    echo "VAR=$v" >> $O/cb.txt
    ISLPOSE_X3_VAR=$v timeout -k 10 120 tools/convbench $s 20 x3 3 >> $O/cb.txt 2>&1 || { echo "convbench failed: $s var $v"; cat $O/cb.txt; exit 1; }
  done
done
cat $O/cb.txt
