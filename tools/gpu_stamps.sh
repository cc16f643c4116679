# s_memtime phase stamps of the union loop variants (ISLPOSE_X3_UNION=4 full, 6 no DMA,
# 7 no input loads, 8 neither -- the ablations are timing only), per shape.
export TMPDIR=/tmp
O=gpurun_out/${1:-stamps}; mkdir -p $O
for s in "3 128 128 46 82 32" "3 384 128 46 82 32"; do
  for u in 4 6 7 8; do
    echo "== $s union=$u" >> $O/s.txt
    ISLPOSE_X3_UNION=$u timeout -k 10 120 tools/convbench $s 10 x3 2 >> $O/s.txt 2>&1 || { tail $O/s.txt; exit 1; }
  done
done
grep -E "==|round 1|stamps" $O/s.txt
