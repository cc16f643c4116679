# C5 overlapped run under a kernel trace (per-kernel totals of the last pass).
export TMPDIR=/tmp
O=gpurun_out/${1:-c5t}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config c5 --c5-batch 32 --c5-frames 96 --c5-videos 2 --c5-overlap-only > $O/trace.log 2>&1
rc=$?
tail -2 $O/trace.log
exit $rc
