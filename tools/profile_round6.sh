# Round-6 profile at HEAD (the bench legs under the profiler without the frame leg): the bench line (with the CPU baseline), kernel trace + FETCH / WRITE /
# SQ passes of Mode N (profiles/conv_traffic.json, post_traffic.json), a kernel trace of Mode R
# batch 32, the per-layer table.  usage: bash tools/profile_round6.sh <tag>  (gpurun_out/<tag>)
export TMPDIR=/tmp
T=${1:-r6p}; O=gpurun_out/$T; mkdir -p $O
B="python3 bench.py --no-cpu --no-mode-r --e2e-steps 0 --frame-count 0 --steps 3 --warmup 1"
R="python3 bench.py --no-cpu --no-mode-r --e2e-steps 0 --frame-count 0 --steps 3 --warmup 1 --scale 0.5"
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- $B > $O/sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/traceR -o run -- $R > $O/traceR.log 2>&1
rc=$?
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 tools/layer_times.py $f > $O/layers.txt; fr=$(find $O/traceR -name "*kernel_trace.csv" | head -1); [ -n "$fr" ] && python3 -c "import sys; sys.argv=[\"x\", \"$fr\"]; sys.path.insert(0, \"tools\"); import layer_times; layer_times.main(\"$fr\", 184, 328, 32)" > $O/layersR.txt
st=$(find $O/trace -name "*kernel_stats.csv" | head -1)
[ -n "$st" ] && python3 tools/pmc_summary.py $O/fetch $O/write --steps 4 --out $O/pmc_summary.json --sq $O/sq --stats $st \
  --traffic-out $O/conv_traffic.json --post-out $O/post_traffic.json > $O/pmc_summary.txt 2>&1
echo rc=$rc
python3 -c "
import json
d=json.load(open('$O/bench.json'))
print('N', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_us'], 'post', d['post']['ms_per_step'], 'R32', d['mode_r']['batch32']['frames_per_s'], d['mode_r']['batch32']['roofline']['frac'], 'R1', d['mode_r']['batch1']['frames_per_s'], 'cpu', d['cpu_baseline']['value'])
"
exit $rc
