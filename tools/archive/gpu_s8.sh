# 128-pixel family: 4-wave blocks vs 8-wave (128-ch) / 12-wave (96-ch) blocks (ISLPOSE_X3_S8), Mode R and hand shapes.
export TMPDIR=/tmp
O=gpurun_out/${1:-s8}; mkdir -p $O
for s in "3 128 128 23 41 32" "3 384 128 23 41 32" "3 96 96 23 41 32" "3 288 96 23 41 32" "3 512 512 23 41 32" \
         "3 128 128 23 41 8" "3 384 128 23 41 1" "3 512 512 23 23 32" "3 256 256 46 46 13"; do
  for m in 0 1; do
    echo "== $s s8=$m" >> $O/s.txt
    CONVBENCH_SPLIT=1 ISLPOSE_X3_S8=$m timeout -k 10 120 tools/convbench $s 20 x3 3 >> $O/s.txt 2>&1 || { tail $O/s.txt; exit 1; }
  done
done
grep -E "==|round 2" $O/s.txt
