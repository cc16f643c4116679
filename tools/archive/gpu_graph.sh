# Graph replay of the conv chain: full -m gpu suite (replay is the default), batch-1 host vs GPU
# time with replay on / off, then bench A/B (ISLPOSE_NET_GRAPH=0 vs default) at batch 1, Mode R b32, Mode N.
T=${1:-graph}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
tail -3 $O/gputest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/b1_host.py > $O/host_on.txt 2>&1 && cat $O/host_on.txt &&
ISLPOSE_NET_GRAPH=0 timeout -k 10 200 python -u tools/b1_host.py > $O/host_off.txt 2>&1 && cat $O/host_off.txt || exit 1
for i in 1 2; do
  for v in 0 1; do
    if [ $v = 0 ]; then export ISLPOSE_NET_GRAPH=0; else unset ISLPOSE_NET_GRAPH; fi
    timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_g$v$i.json 2>> $O/bench.err &&
    timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/b32_g$v$i.json 2>> $O/bench.err || exit 1
  done
done
unset ISLPOSE_NET_GRAPH
timeout -k 10 300 python -u bench.py > $O/bench.json 2>> $O/bench.err || exit 1
python3 -c "
import json
for i in (1,2):
  for v in (0,1):
    for b in ('b1','b32'):
      x=json.load(open('$O/%s_g%d%d.json'%(b,v,i)))
      print(b, 'graph' if v else 'eager', x['value'], 'ms', x['ms_per_step'], 'net', x['roofline']['net_ms_per_step'])
x=json.load(open('$O/bench.json')); print('ModeN', x['value'], x['roofline']['frac'], x['mode_r']['batch32']['frames_per_s'], x['mode_r']['batch1']['frames_per_s'])
"
