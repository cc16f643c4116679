set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for s in "3 96 96 46 82 32" "3 288 96 46 82 32" "3 64 64 368 656 32" "3 64 128 184 328 32" "1 512 52 46 82 32" "1 512 26 46 82 32"; do
  for v in "$@"; do
    echo "VAR=$v" >> $O/cb.txt
    ISLPOSE_X3_VAR=$v timeout -k 10 120 tools/convbench $s 20 x3 3 >> $O/cb.txt 2>&1 || { echo "convbench failed: $s"; cat $O/cb.txt; exit 1; }
  done
done
grep -E "VAR|conv|round 2" $O/cb.txt
