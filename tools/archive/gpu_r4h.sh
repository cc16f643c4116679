# Round 4: the blur's fp32 filter -- its tests, the post tests, and kernel traces of the Mode R
# post with and without it (ISLPOSE_BLUR_EXACT=1).
T=${1:-r4h}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_blur_filter.py \
  tests/test_gpu_hand.py "tests/test_gpu_body.py::test_body_post_golden_bit_exact" \
  "tests/test_gpu_body.py::test_designed_maps_batch_bit_exact" "tests/test_gpu_body.py::test_fused_resize_blur_matches_unfused" \
  "tests/test_gpu_body.py::test_fused_two_stage_post_matches_unfused" > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; fi
P="python3 tools/post_prof.py --batch 32 --iters 5"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tf -o run -- $P > $O/tf.log 2>&1 &&
ISLPOSE_BLUR_EXACT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tx -o run -- $P > $O/tx.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tn -o run -- python3 tools/post_prof.py --batch 32 --iters 5 --scale 1.0 > $O/tn.log 2>&1 &&
ISLPOSE_BLUR_EXACT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tnx -o run -- python3 tools/post_prof.py --batch 32 --iters 5 --scale 1.0 > $O/tnx.log 2>&1
rc=$?
grep post_ms $O/tf.log $O/tx.log $O/tn.log $O/tnx.log
exit $rc
