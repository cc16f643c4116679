# A/B of balanced tiles (ISLPOSE_X3_BAL=1: equal 32-px-aligned tiles, dead column groups
# skipped, 4x4 wave layout), the 4x4 layout alone (2) and the default (0), per layer shape.
set -o pipefail
O=gpurun_out/bal; mkdir -p $O; : > $O/b.txt
for s in "3 128 128 46 82 32" "3 384 128 46 82 32" "3 256 256 92 164 32" "3 128 256 92 164 32" "3 512 512 46 82 32" "3 512 256 46 82 32"; do
  for r in 1 2; do
    for m in 0 1 2; do
      echo "shape $s bal $m" >> $O/b.txt
      ISLPOSE_X3_BAL=$m timeout -k 10 120 tools/convbench $s 20 x3 2 >> $O/b.txt 2>&1 || { echo "convbench failed: $s $m"; tail $O/b.txt; exit 1; }
    done
  done
  echo "done $s"
done
grep -E "^shape|round 1" $O/b.txt
