# 7x7 tile families: output-channel tile 128 (128-pixel family, current) vs 64 (512-pixel
# 16-wave family on large grids, 128-pixel 2-blocks-per-CU family on small ones).
export TMPDIR=/tmp
O=gpurun_out/${1:-ab7}; mkdir -p $O
for s in "7 128 128 23 23 32" "7 128 128 46 46 32" "7 128 128 69 69 32" "7 128 128 92 92 32" "7 150 128 92 92 32" \
         "7 128 128 23 41 32" "7 185 128 23 41 1" "7 128 128 46 46 2"; do
  for b in 128 64; do
    echo "== $s bco=$b" >> $O/h.txt
    CONVBENCH_BCO=$b timeout -k 10 120 tools/convbench $s 10 x3 3 >> $O/h.txt 2>&1 || { tail $O/h.txt; exit 1; }
  done
done
grep -E "==|round 2" $O/h.txt
