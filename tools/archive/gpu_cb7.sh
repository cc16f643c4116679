set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for s in "7 128 128 46 46 32" "7 128 128 92 92 32" "7 152 128 69 69 32" "3 512 512 92 92 32" "3 64 64 736 736 8" "1 128 128 92 92 32"; do
  timeout -k 10 120 tools/convbench $s 10 x3,direct 2 >> $O/cb.txt 2>&1 || { echo "convbench failed: $s"; cat $O/cb.txt; exit 1; }
done
grep -E "conv|round 1" $O/cb.txt
