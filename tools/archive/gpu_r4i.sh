# Round 4: the nested PAF samples and the blur filter under the post tests, per-tile phase
# profile of the blur (development library), post timings.
T=${1:-r4i}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_blur_filter.py \
  "tests/test_gpu_body.py::test_body_post_golden_bit_exact" "tests/test_gpu_body.py::test_body_estimate_end_to_end" \
  "tests/test_gpu_body.py::test_designed_maps_batch_bit_exact" "tests/test_gpu_body.py::test_fused_resize_blur_matches_unfused" \
  "tests/test_gpu_body.py::test_fused_two_stage_post_matches_unfused" "tests/test_gpu_body.py::test_launch_post_stream_equals_estimate" tests/test_gpu_hand.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; fi
timeout -k 10 200 python3 tools/tile_prof.py --scale 0.5 > $O/tile_r.json 2> $O/tile.err &&
ISLPOSE_BLUR_LIST=0 timeout -k 10 200 python3 tools/tile_prof.py --scale 0.5 > $O/tile_r0.json 2>> $O/tile.err &&
ISLPOSE_BLUR_LIST=0 timeout -k 10 200 python3 tools/post_prof.py --batch 32 --iters 10 > $O/post_r0.txt 2>&1 &&
timeout -k 10 200 python3 tools/tile_prof.py --scale 1.0 > $O/tile_n.json 2>> $O/tile.err &&
timeout -k 10 200 python3 tools/post_prof.py --batch 32 --iters 10 > $O/post_r.txt 2>&1 &&
timeout -k 10 200 python3 tools/post_prof.py --batch 32 --iters 10 --scale 1.0 > $O/post_n.txt 2>&1 &&
timeout -k 10 200 python3 tools/post_prof.py --batch 1 --iters 20 > $O/post_r1.txt 2>&1 &&
ISLPOSE_RESIZE_V4=0 timeout -k 10 200 python3 tools/post_prof.py --batch 32 --iters 10 > $O/post_r_v40.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/post_prof.py --batch 32 --iters 5 > $O/tr.log 2>&1 &&
ISLPOSE_LIB=tools/libislpose_dev.so timeout -k 10 200 python3 tools/post_prof.py --batch 32 --iters 10 > $O/post_r_dev.txt 2>&1 &&
ISLPOSE_LIB=tools/libislpose_dev.so ISLPOSE_FUSED_WIDE=1 timeout -k 10 200 python3 tools/post_prof.py --batch 32 --iters 10 > $O/post_r_wide.txt 2>&1 &&
ISLPOSE_LIB=tools/libislpose_dev.so ISLPOSE_FUSED_WIDE=1 timeout -k 10 200 python3 tools/tile_prof.py --scale 0.5 > $O/tile_r_wide.json 2>> $O/tile.err
rc=$?
cat $O/tile_r.json $O/tile_r0.json $O/tile_n.json $O/post_r0.txt $O/post_r.txt $O/post_r_v40.txt $O/post_n.txt $O/post_r1.txt $O/post_r_dev.txt $O/post_r_wide.txt $O/tile_r_wide.json; tail -3 $O/tile.err
exit $rc
