# C3 / C4 throughput (tools/bench_configs.py) + a kernel trace and an SQ pass of C3.
# usage: bash tools/profile_configs.sh <tag>
export TMPDIR=/tmp
T=${1:-cfg}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python3 tools/bench_configs.py --config c3 --steps 3 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 600 python3 tools/bench_configs.py --config c4 --steps 3 > $O/c4.json 2> $O/c4.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config c3 --steps 1 --warmup 1 > $O/trace.log 2>&1 &&
timeout -s KILL 600 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- python3 tools/bench_configs.py --config c3 --steps 1 --warmup 1 > $O/sq.log 2>&1
rc=$?
cat $O/c3.json $O/c4.json
echo rc=$rc
exit $rc
