# A/B of the resize kernel (ISLPOSE_RESIZE_V1=1 selected the previous one, since removed): the body / hand post
# parity tests, then Mode R batch-32 bench (post_ms) interleaved twice.
T=${1:-rsab}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_body.py tests/test_gpu_hand.py tests/test_gpu_compat.py -x -v --timeout 300 --timeout-method thread \
  -k "post or golden or fused or estimate or hand or pyramid or designed" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 1 0; do
    ISLPOSE_RESIZE_V1=$v timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/R32_v${v}_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for v in (1,0):
    x=json.load(open('$O/R32_v%d_%d.json'%(v,i)))
    print('v1' if v else 'new', x['value'], 'ms', x['ms_per_step'], 'post', x['post']['ms_per_step'])
"
