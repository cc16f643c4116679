# 3x3 layers off the row union (full-resolution, short K): 16-wave 512-pixel blocks (default)
# vs other block shapes (ISLPOSE_X3_MID, see launch_ks)
set -o pipefail
O=gpurun_out/mid; mkdir -p $O; : > $O/m.txt
run() {   # shape, modes
  for r in 1 2; do
    for m in $2; do
      echo "shape $1 mid $m" >> $O/m.txt
      ISLPOSE_X3_MID=$m timeout -k 10 120 tools/convbench $1 10 x3 2 >> $O/m.txt 2>&1 || { echo "convbench failed: $1"; tail $O/m.txt; exit 1; }
    done
  done
}
run "3 64 64 368 656 32" "0 2 3 5 8" && run "3 64 64 552 552 16" "0 2 3 5 8" &&
run "3 64 128 184 328 32" "0 6 7" && run "3 128 128 184 328 32" "0 6 7" && run "3 128 128 368 368 16" "0 6 7" &&
grep -E "^shape|round 1" $O/m.txt
