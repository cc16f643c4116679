# Round 4: smoke(), and kernel traces of the batch-1 Mode R post and forward.
T=${1:-r4q}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t1 -o run -- python3 tools/post_prof.py --batch 1 --iters 20 > $O/t1.log 2>&1
rc=$?
tail -1 $O/smoke.log
exit $rc
