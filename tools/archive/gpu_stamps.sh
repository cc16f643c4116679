# s_memtime phase stamps of the row-union loop (ISLPOSE_X3_UNION=4, development build), per shape.
export TMPDIR=/tmp
O=gpurun_out/${1:-stamps}; mkdir -p $O
for s in "3 128 128 46 82 32" "3 384 128 46 82 32"; do
  echo "== $s union=4" >> $O/s.txt
  ISLPOSE_X3_UNION=4 timeout -k 10 120 tools/convbench $s 10 x3 2 >> $O/s.txt 2>&1 || { tail $O/s.txt; exit 1; }
done
cat $O/s.txt
