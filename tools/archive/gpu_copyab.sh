# Batch-1 step: records D2H on the post stream (default for small records) vs the copy stream
# (ISLPOSE_BENCH_COPY_STREAM=1), with the preprocess table upload skipped when unchanged; parity first.
T=${1:-copyab}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py tests/test_gpu_hand.py tests/test_gpu_configs.py tests/test_gpu_compat.py -x -v --timeout 300 --timeout-method thread \
  -k "preprocess or crop or estimate or call or c5 or pipeline or golden or pyramid or launch" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    ISLPOSE_BENCH_COPY_STREAM=$v timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_c${v}_$i.json 2>> $O/bench.err || exit 1
  done
done
timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/b32.json 2>> $O/bench.err || exit 1
python3 -c "
import json
for i in (1,2,3):
  for v in (1,0):
    x=json.load(open('$O/b1_c%d_%d.json'%(v,i))); print('copy-stream' if v else 'same-stream', x['value'], 'ms', x['ms_per_step'])
x=json.load(open('$O/b32.json')); print('b32', x['value'])
"
