# In-kernel clock of the union loop (stamp build) over several rounds of back-to-back launches.
export TMPDIR=/tmp
O=gpurun_out/${1:-clk}; mkdir -p $O
for s in "3 128 128 46 82 32" "3 384 128 46 82 32"; do
  echo "== $s" >> $O/c.txt
  ISLPOSE_X3_UNION=4 timeout -k 10 120 tools/convbench $s 200 x3 4 >> $O/c.txt 2>&1 || { tail $O/c.txt; exit 1; }
done
grep -E "==|round|clock|stamps" $O/c.txt
