# Round 4: HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the Mode R batch-32 post kernels.
T=${1:-r4ab}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
P="python3 tools/post_prof.py --batch 32 --iters 3"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $P > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $P > $O/write.log 2>&1
rc=$?
st=$(find $O/trace -name "*kernel_stats.csv" | head -1)
[ -n "$st" ] && python3 tools/pmc_summary.py $O/fetch $O/write --steps 4 --out $O/pmc_summary.json --stats $st --post-out $O/post_traffic_modeR.json > $O/pmc_summary.txt 2>&1
cat $O/post_traffic_modeR.json
exit $rc
