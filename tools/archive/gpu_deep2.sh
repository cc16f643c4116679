# DEEP by default on single-round 3x3 small grids: parity (bit-identity, batch invariance), then
# Mode R batch 32 / batch 1 and Mode N with the default vs ISLPOSE_X3_DEEP=0, interleaved twice.
T=${1:-deep2}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py -x -v --timeout 300 --timeout-method thread \
  -k "deep or canonical or timed_config or splitk" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for d in "" 0; do
    ISLPOSE_X3_DEEP=$d timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/b32_d${d}_$i.json 2>> $O/bench.err &&
    ISLPOSE_X3_DEEP=$d timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_d${d}_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for d in ('','0'):
    for b in ('b32','b1'):
      x=json.load(open('$O/%s_d%s_%d.json'%(b,d,i)))
      print(b, 'deep=%s'%(d or 'default'), x['value'], 'frac', x['roofline']['frac'], 'net_ms', x['roofline']['net_ms_per_step'])
"
