# 7x7 layers: 128-pixel tiles (ISLPOSE_X3_WIDE7=0) vs 256-pixel tiles (=1), interleaved, per launch size
# (the data behind X3_WIDE7_COST in conv_x3.hip).
export TMPDIR=/tmp
O=gpurun_out/${1:-w7}; mkdir -p $O
for s in "7 128 128 92 92 32" "7 128 128 69 69 32" "7 128 128 46 46 32" "7 150 128 92 92 32" "7 150 128 69 69 32" \
         "7 128 128 92 92 13" "7 128 128 69 69 13" "7 128 128 46 82 32" "7 185 128 46 82 32" "7 128 128 92 92 64"; do
  for m in 0 1; do
    echo "== $s wide7=$m" >> $O/w.txt
    ISLPOSE_X3_WIDE7=$m timeout -k 10 120 tools/convbench $s 10 x3 3 >> $O/w.txt 2>&1 || { tail $O/w.txt; exit 1; }
  done
done
grep -E "==|round 2" $O/w.txt
