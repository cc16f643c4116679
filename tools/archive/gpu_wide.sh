# Wide fused-blur window (Mode R two-stage frames, stage-2 x2 resized on the fly): body post parity (fused /
# unfused / oracle, goldens, Mode R estimates), then Mode R batch 32 / batch 1 with ISLPOSE_FUSED_WIDE=0 vs 1.
T=${1:-wide}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py tests/test_gpu_compat.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "post or golden or fused or estimate or blur or coco or c5 or launch or two_stage" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 0 1; do
    ISLPOSE_FUSED_WIDE=$v timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/R32_w${v}_$i.json 2>> $O/bench.err &&
    ISLPOSE_FUSED_WIDE=$v timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_w${v}_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for v in (0,1):
    for b in ('R32','b1'):
      x=json.load(open('$O/%s_w%d_%d.json'%(b,v,i))); print(b, 'wide' if v else 'materialised', x['value'], 'ms', x['ms_per_step'], 'post', x['post']['ms_per_step'])
"
