# The streaming (non-fused) blur filter: post GPU tests, then the bench line (Mode R batch 32 post).
# usage: bash tools/ab_blurstream.sh <tag>
export TMPDIR=/tmp
T=${1:-bs}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_blur_filter.py tests/test_gpu_body.py tests/test_gpu_hand.py -k "blur or post or golden or designed or limb or fused_resize or two_stage or hand_post or end_to_end" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
bash tools/ab_bench.sh $T a: b: c:
