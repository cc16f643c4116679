# Canonical K ranges: in one block (ISLPOSE_X3_ACROSS=0) vs across blocks (=1), per launch size.
export TMPDIR=/tmp
O=gpurun_out/${1:-acr}; mkdir -p $O
for s in "7 128 128 23 23 32" "7 150 128 23 23 32" "3 512 512 23 23 32" "3 256 512 23 23 32" "3 512 128 23 23 32" \
         "3 128 128 23 41 32" "3 384 128 23 41 32" "3 288 96 23 41 32" "1 384 512 23 41 32" "3 512 512 23 41 32" \
         "3 128 128 23 41 8" "3 384 128 23 41 8" "7 128 128 23 23 13" "3 512 512 23 23 13"; do
  for m in 0 1; do
    echo "== $s across=$m" >> $O/a.txt
    CONVBENCH_SPLIT=1 ISLPOSE_X3_ACROSS=$m timeout -k 10 120 tools/convbench $s 20 x3 3 >> $O/a.txt 2>&1 || { tail $O/a.txt; exit 1; }
  done
done
grep -E "==|round 2" $O/a.txt
