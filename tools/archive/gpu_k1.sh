# 1x1 layers: 128-channel tiles (CONVBENCH_BCO=128, the old packing) vs 256-channel, two pairs per step (256).
export TMPDIR=/tmp
O=gpurun_out/${1:-k1}; mkdir -p $O
for s in "1 384 512 46 82 32" "1 288 256 46 82 32" "1 128 512 46 46 32" "1 512 512 92 92 32" "1 384 512 23 41 32" "1 384 512 23 41 1"; do
  for b in 128 256; do
    echo "== $s bco=$b" >> $O/k.txt
    CONVBENCH_SPLIT=1 CONVBENCH_BCO=$b timeout -k 10 120 tools/convbench $s 20 x3 3 >> $O/k.txt 2>&1 || { tail $O/k.txt; exit 1; }
  done
done
grep -E "==|round 2" $O/k.txt
