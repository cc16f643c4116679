# Split-K reduce A/B: ISLPOSE_X3_REDUCE_V1=1 (the previous kernel; a temporary switch, since removed) vs the new one, batch-1
# Mode R interleaved three times; parity of the new one first (plus the body post goldens: assemble staging).
T=${1:-reduce_ab}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py tests/test_gpu_hand.py -x -v --timeout 300 --timeout-method thread \
  -k "canonical or splitk or halfco or graph or hand_net or post or golden or estimate or fused or coco or timed" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    ISLPOSE_X3_REDUCE_V1=$v timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_v${v}_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2,3):
  for v in (1,0):
    x=json.load(open('$O/b1_v%d_%d.json'%(v,i))); print('old' if v else 'new', x['value'], 'ms', x['ms_per_step'])
"
