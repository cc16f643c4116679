# 8-wave 128-pixel layouts for 1x1 and ranged 7x7 layers (default) vs 4-wave (ISLPOSE_X3_S8=0).
export TMPDIR=/tmp
O=gpurun_out/${1:-s8b}; mkdir -p $O
for s in "1 384 512 23 41 32" "1 288 256 23 41 32" "1 512 52 23 41 32" "7 128 128 23 23 32" "7 150 128 23 23 32" "7 128 128 23 41 32" "7 128 128 23 23 13" "1 128 512 23 23 32"; do
  for m in 0 1; do
    echo "== $s s8=$m" >> $O/s.txt
    CONVBENCH_SPLIT=1 ISLPOSE_X3_S8=$m timeout -k 10 120 tools/convbench $s 20 x3 3 >> $O/s.txt 2>&1 || { tail $O/s.txt; exit 1; }
  done
done
grep -E "==|round 2" $O/s.txt
