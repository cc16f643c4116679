# Kernel trace of the default bench (+ per-layer table) and the union-loop stamps.
export TMPDIR=/tmp
T=${1:-tr}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --e2e-steps 0 --steps 5 --warmup 2 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python tools/layer_times.py $f > $O/layers.txt && cat $O/layers.txt
bash tools/archive/gpu_stamps.sh $T
