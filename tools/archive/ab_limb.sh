# limb_kernel: large pair sets in LDS and the split scoring of small batches: GPU tests, then the
# FRAME leg and the bench line with the split on / off (ISLPOSE_LIMB_SPLIT=0).
# usage: bash tools/ab_limb.sh <tag>
export TMPDIR=/tmp
T=${1:-limb}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_body.py -k "limb_large or assemble_register or designed_maps or launch_post or golden_bit_exact or end_to_end" > $O/tests.log 2>&1 &&
timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_on.json 2> $O/frame_on.err &&
ISLPOSE_LIMB_SPLIT=0 timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_off.json 2> $O/frame_off.err &&
timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_on2.json 2> $O/frame_on2.err &&
bash tools/ab_bench.sh $T on: off:ISLPOSE_LIMB_SPLIT=0 on2:
rc=$?
for f in frame_on frame_off frame_on2; do python3 -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])"; done
exit $rc
