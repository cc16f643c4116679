# The per-frame call (FRAME leg, tools/bench_configs.py --config frame): throughput, a kernel
# trace, and a host profile (cProfile) of the same loop.  usage: bash tools/profile_frame.sh <tag>
export TMPDIR=/tmp
T=${1:-frp}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame.json 2> $O/frame.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config frame --frame-count 16 > $O/trace.log 2>&1 &&
timeout -k 10 300 python3 -m cProfile -o $O/frame.prof tools/bench_configs.py --config frame --frame-count 32 > $O/cprof.log 2>&1 &&
python3 -c "
import pstats; p = pstats.Stats('$O/frame.prof'); p.sort_stats('cumulative').print_stats(45)" > $O/cprof.txt 2>&1
rc=$?
cat $O/frame.json
echo rc=$rc
exit $rc
