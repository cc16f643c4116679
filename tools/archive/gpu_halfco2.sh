# HALFCO by default on across-block split layers: parity (bit identity, canonical ranges, batch-1 paths), then
# Mode R batch 1 / 32 with ISLPOSE_X3_HALFCO=0 (old default) vs unset (new default), interleaved twice; C3 once each.
T=${1:-halfco2}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py tests/test_gpu_hand.py -x -v --timeout 300 --timeout-method thread \
  -k "halfco or canonical or splitk or deep or estimate or hand" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 0 d; do
    if [ $v = 0 ]; then export ISLPOSE_X3_HALFCO=0; else unset ISLPOSE_X3_HALFCO; fi
    timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_$v$i.json 2>> $O/bench.err &&
    timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/b32_$v$i.json 2>> $O/bench.err || exit 1
  done
done
for v in 0 d; do
  if [ $v = 0 ]; then export ISLPOSE_X3_HALFCO=0; else unset ISLPOSE_X3_HALFCO; fi
  timeout -k 10 600 python -u tools/bench_configs.py --config c3 --steps 5 > $O/c3_$v.log 2>&1 || exit 1
done
unset ISLPOSE_X3_HALFCO
python3 -c "
import json
for i in (1,2):
  for v in ('0','d'):
    for b in ('b1','b32'):
      x=json.load(open('$O/%s_%s%d.json'%(b,v,i)))
      print(b, 'old' if v=='0' else 'new', x['value'], 'net', x['roofline']['net_ms_per_step'])
"
grep -h frames_per_s $O/c3_*.log | cut -c1-160
