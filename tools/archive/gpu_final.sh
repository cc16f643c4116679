# Round profile at HEAD (tools/profile_round.sh) + pmc summary, then C3 kernel trace and SQ pass.
export TMPDIR=/tmp
T=${1:-final}; O=gpurun_out/$T
bash tools/profile_round.sh $T || exit $?
python3 tools/pmc_summary.py $O/fetch $O/write --steps 4 --out $O/pmc_summary.json --sq $O/sq --stats $(find $O/trace -name "*kernel_stats.csv" | head -1) > $O/pmc_summary.txt 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3trace -o run -- python3 tools/bench_configs.py --config c3 --steps 1 --warmup 1 > $O/c3trace.log 2>&1 &&
timeout -s KILL 600 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/c3sq -o run -- python3 tools/bench_configs.py --config c3 --steps 1 --warmup 1 > $O/c3sq.log 2>&1
rc=$?
f=$(find $O/c3trace -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 tools/trace_summary.py $f $O/c3sq --out $O/c3_kernels.json > /dev/null 2>&1
echo rc=$rc
exit $rc
