# Small 7x7 grids on 64-channel x 64-pixel blocks (x3_small7): hand GPU tests, then the FRAME
# leg with it on / off and C3.  usage: bash tools/ab_small7.sh <tag>
export TMPDIR=/tmp
T=${1:-s7}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_hand.py tests/test_gpu_configs.py -k "small7 or c3_crop or estimate_crops or per_frame or split_k" > $O/tests.log 2>&1 &&
timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_on.json 2> $O/frame_on.err &&
ISLPOSE_X3_SMALL7=0 timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_off.json 2> $O/frame_off.err &&
timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_on2.json 2> $O/frame_on2.err &&
timeout -k 10 300 python3 tools/bench_configs.py --config c3 --steps 5 > $O/c3.json 2> $O/c3.err
rc=$?
for f in frame_on frame_off frame_on2; do python3 -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])"; done
cat $O/c3.json
exit $rc
