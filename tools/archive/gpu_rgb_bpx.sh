# conv1_1 (conv_x3_rgb) tile width A/B: 512 (default) / 256 / 128 pixels per block
set -o pipefail
O=gpurun_out/rgbbpx; mkdir -p $O; : > $O/r.txt
for r in 1 2; do
  for b in 512 256 128; do
    echo "bpx $b" >> $O/r.txt
    ISLPOSE_RGB_BPX=$b timeout -k 10 120 python3 tools/net_layers.py body25 32 368x656 2>&1 | grep -E "c3->64|total" >> $O/r.txt || exit 1
  done
done
cat $O/r.txt
