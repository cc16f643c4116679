# C3 evidence at HEAD: hand-net per-layer table (engine HIP events) at the four crop scales,
# then a rocprofv3 kernel trace + stats of one C3 step.
# usage: bash tools/archive/gpu_c3prof.sh <tag>   (outputs under gpurun_out/<tag>)
export TMPDIR=/tmp
T=${1:-c3prof}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python3 -u tools/net_layers.py hand 32 184 368 552 736 > $O/hand_layers.txt 2> $O/hand_layers.json &&
timeout -k 10 300 python3 -u tools/net_layers.py body25 16 184x328 > $O/body_r16_layers.txt 2> $O/body_r16_layers.json &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config c3 --steps 1 --warmup 1 > $O/trace.log 2>&1
rc=$?
cat $O/hand_layers.txt
echo rc=$rc
exit $rc
