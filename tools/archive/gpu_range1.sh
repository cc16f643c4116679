# A/B of one-pair canonical K ranges (ISLPOSE_X3_RANGE1, a temporary switch since removed): neutral, see profiles/r03/range1.
T=${1:-rng1}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
ISLPOSE_X3_RANGE1=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py -x -v --timeout 300 --timeout-method thread \
  -k "canonical or deep or splitk or algo" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 1 0; do
    ISLPOSE_X3_RANGE1=$v timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_v${v}_$i.json 2>> $O/bench.err &&
    ISLPOSE_X3_RANGE1=$v timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/b32_v${v}_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for v in (1,0):
    for b in ('b1','b32'):
      x=json.load(open('$O/%s_v%d_%d.json'%(b,v,i)))
      print(b, 'S=pairs' if v else 'S=pairs/2', x['value'], 'net', x['roofline']['net_ms_per_step'])
"
