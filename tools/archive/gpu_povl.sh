# Post overlap (--post-overlap: the post of batch k on its own stream beside the net of batch k+1) vs
# post on the net's stream (default): the launch(post_stream) parity test, then Mode N,
# Mode R batch 32 and batch 1, interleaved twice.  usage: bash tools/archive/gpu_povl.sh <tag>
T=${1:-povl}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py -x -v --timeout 300 --timeout-method thread \
  -k "post_stream or end_to_end or designed" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for o in "--post-overlap" ""; do
    tag=$([ -n "$o" ] && echo ovl || echo seq)
    timeout -k 10 300 python -u bench.py --no-cpu --no-mode-r --e2e-steps 0 $o > $O/N_${tag}_$i.json 2>> $O/bench.err &&
    timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 $o > $O/R32_${tag}_$i.json 2>> $O/bench.err &&
    timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 $o > $O/R1_${tag}_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for t in ('ovl','seq'):
    for b in ('N','R32','R1'):
      x=json.load(open('$O/%s_%s_%d.json'%(b,t,i)))
      print(b, t, x['value'], 'ms', x['ms_per_step'], 'net', x['roofline']['net_ms_per_step'], 'post', x['post']['ms_per_step'], 'frac', x['roofline']['frac'])
"
