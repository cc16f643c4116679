# Batch-1 Mode R kernel trace (CSV stats + trace) of a short bench run.
T=${1:-b1trace}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o b1 -- python3 $GRAFT_REPO_ROOT/bench.py --scale 0.5 --batch 1 --steps 30 --warmup 3 --no-cpu --no-mode-r --e2e-steps 0 --no-op-timing > $GRAFT_REPO_ROOT/$O/prof_bench.json 2>> $GRAFT_REPO_ROOT/$O/bench.err
rc=$?
cd $GRAFT_REPO_ROOT
find $O/prof -name '*.csv' | head
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -c1-150 $f | head -30
exit $rc
