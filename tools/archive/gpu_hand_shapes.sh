# conv microbenchmarks of the hand net's layer shapes (32 crops per scale, configs[2]).
export TMPDIR=/tmp
O=gpurun_out/${1:-hand}; mkdir -p $O
for s in "7 128 128 23 23 32" "7 128 128 46 46 32" "7 128 128 69 69 32" "7 128 128 92 92 32" "7 150 128 92 92 32" \
         "3 512 512 92 92 32" "3 512 512 46 46 32" "3 256 256 184 184 32" "3 64 64 736 736 8" "1 128 512 92 92 32" "1 512 22 92 92 32"; do
  echo "== $s" >> $O/h.txt
  timeout -k 10 120 tools/convbench $s 10 x3 2 >> $O/h.txt 2>&1 || { tail $O/h.txt; exit 1; }
done
grep -E "==|round 1" $O/h.txt
