# Split-K reduce rewrite (ranges' loads in flight, contiguous halves): parity (canonical ranges across vs in
# blocks, split-K, hand scales), batch-1 / batch-32 Mode R bench, then a batch-1 kernel trace (reduce avg us).
T=${1:-reduce}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py tests/test_gpu_hand.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "canonical or splitk or halfco or deep or pps2 or fold or graph or hand or timed or vs_oracle" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_$i.json 2>> $O/bench.err &&
  timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/b32_$i.json 2>> $O/bench.err || exit 1
done
python3 -c "
import json
for i in (1,2):
  for b in ('b1','b32'):
    x=json.load(open('$O/%s_%d.json'%(b,i))); print(b, x['value'], 'ms', x['ms_per_step'], 'net', x['roofline']['net_ms_per_step'])
"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o b1 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --scale 0.5 --batch 1 --steps 30 --warmup 3 --no-cpu --no-mode-r --e2e-steps 0 --no-op-timing > $GRAFT_REPO_ROOT/$O/prof_bench.json 2>> $GRAFT_REPO_ROOT/$O/bench.err
rc=$?
cd $GRAFT_REPO_ROOT
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && grep -h "splitk_reduce\|Name" $f | cut -c1-160
exit $rc
