# Resize block shape A/B on Mode R batch 32 (post_ms): rows per block (ISLPOSE_RS_TY) x 128-column blocks
# (ISLPOSE_RS_TX128); temporary switches, since removed (128 columns adopted); post parity with the non-default shape.
T=${1:-rsty}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
ISLPOSE_RS_TY=32 ISLPOSE_RS_TX128=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py tests/test_gpu_hand.py -x -q --timeout 300 --timeout-method thread \
  -k "post or golden or estimate or two_stage or hand_post or pyramid" > $O/test.log 2>&1; rc=$?
tail -2 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for cfg in "64 0" "32 0" "64 1" "32 1" "16 1"; do
    set -- $cfg
    ISLPOSE_RS_TY=$1 ISLPOSE_RS_TX128=$2 timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/R_$1_$2_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for c in ('64_0','32_0','64_1','32_1','16_1'):
    x=json.load(open('$O/R_%s_%d.json'%(c,i))); print(c, x['value'], 'post', x['post']['ms_per_step'])
"
