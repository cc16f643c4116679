# Per-frame path profile: phases (synchronised laps), kernel trace of 16 frames, host cProfile.
# usage: bash tools/frame_prof6.sh <tag>   (gpurun_out/<tag>)
export TMPDIR=/tmp
T=${1:-fr6}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python3 tools/frame_phases.py --frames 48 > $O/phases.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config frame --frame-count 16 > $O/trace.log 2>&1 &&
timeout -k 10 300 python3 -m cProfile -o $O/frame.prof tools/bench_configs.py --config frame --frame-count 32 > $O/cprof.log 2>&1 &&
python3 -c "
import pstats; p = pstats.Stats('$O/frame.prof'); p.sort_stats('tottime').print_stats(30)" > $O/cprof.txt 2>&1
rc=$?
cat $O/phases.txt
exit $rc
