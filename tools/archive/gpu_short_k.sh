# short-K full-resolution layers: big 512-pixel tiles (default) vs the 128-pixel family
set -o pipefail
O=gpurun_out/shortk; mkdir -p $O; : > $O/s.txt
for s in "3 64 64 368 656 32" "3 64 128 184 328 32" "3 128 128 184 328 32" "3 3 64 368 656 32"; do
  for m in big small; do
    echo "shape $s tiles $m" >> $O/s.txt
    if [ $m = small ]; then export ISLPOSE_X3_TILES=small; else unset ISLPOSE_X3_TILES; fi
    timeout -k 10 120 tools/convbench $s 10 x3 2 >> $O/s.txt 2>&1 || { echo "convbench failed: $s"; tail $O/s.txt; exit 1; }
  done
done
unset ISLPOSE_X3_TILES
grep -E "^shape|round 1" $O/s.txt
