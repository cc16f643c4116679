# Round profile: bench (with CPU baseline), kernel trace, HBM traffic (FETCH/WRITE), SQ pass,
# per-layer table, and the in-kernel clock of the dominant conv shape (stamp build).
# usage: bash tools/profile_round.sh <tag>      (outputs under gpurun_out/<tag>)
export TMPDIR=/tmp
T=${1:-r2p}; O=gpurun_out/$T; mkdir -p $O
B="python3 bench.py --no-cpu --no-mode-r --e2e-steps 0 --steps 3 --warmup 1"
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- $B > $O/sq.log 2>&1 &&
ISLPOSE_X3_UNION=4 timeout -k 10 120 tools/convbench 3 384 128 46 82 32 200 x3 3 > $O/clock.txt 2>&1
rc=$?
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 tools/layer_times.py $f > $O/layers.txt
echo rc=$rc
grep clock $O/clock.txt
cat $O/bench.json
exit $rc
