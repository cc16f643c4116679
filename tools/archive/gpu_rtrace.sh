# Mode R batch-32 kernel trace (CSV) of a short bench run: the post kernels of one step, in order.
T=${1:-rtrace}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o r32 -- python3 $GRAFT_REPO_ROOT/bench.py --scale 0.5 --steps 5 --warmup 2 --no-cpu --no-mode-r --e2e-steps 0 --no-op-timing > $GRAFT_REPO_ROOT/$O/prof_bench.json 2>> $GRAFT_REPO_ROOT/$O/bench.err
