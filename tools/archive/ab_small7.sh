# Small 7x7 grids (x3_small7): hand GPU tests, then the FRAME leg with ISLPOSE_X3_SMALL7=2
# (default: deep prefetch within one round) / 1 / 3 (always deep), and single-crop hand op tables.  usage: bash tools/ab_small7.sh <tag>
export TMPDIR=/tmp
T=${1:-s7}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_hand.py tests/test_gpu_configs.py -k "small7 or c3_crop or estimate_crops or per_frame or split_k" > $O/tests.log 2>&1 &&
for m in 2 1 2b 3; do
  ISLPOSE_X3_SMALL7=${m:0:1} timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_$m.json 2> $O/frame_$m.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/frame_$m.json')); print('$m', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])"
done &&
for s in 368 736; do
  timeout -k 10 200 python3 tools/op_table.py --kind hand --batch 1 --h $s --w $s --runs 5 > $O/ops_hand_b1_$s.txt 2>&1 || exit 1
done
