# Round 4: blur NMS / window / XCD-list changes -- the post tests, tile profile, post timings, trace.
T=${1:-r4j}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_blur_filter.py \
  "tests/test_gpu_body.py::test_body_post_golden_bit_exact" "tests/test_gpu_body.py::test_designed_maps_batch_bit_exact" \
  "tests/test_gpu_body.py::test_fused_resize_blur_matches_unfused" "tests/test_gpu_body.py::test_fused_two_stage_post_matches_unfused" \
  tests/test_gpu_hand.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; fi
timeout -k 10 200 python3 tools/tile_prof.py --scale 0.5 > $O/tile_r.json 2> $O/tile.err &&
timeout -k 10 200 python3 tools/tile_prof.py --scale 1.0 > $O/tile_n.json 2>> $O/tile.err &&
timeout -k 10 200 python3 tools/post_prof.py --batch 32 --iters 10 > $O/post_r.txt 2>&1 &&
ISLPOSE_RESIZE_SKIP=0 timeout -k 10 200 python3 tools/post_prof.py --batch 32 --iters 10 > $O/post_rx.txt 2>&1 &&
timeout -k 10 200 python3 tools/post_prof.py --batch 32 --iters 10 --scale 1.0 > $O/post_n.txt 2>&1 &&
ISLPOSE_BLUR_EXACT=1 timeout -k 10 200 python3 tools/post_prof.py --batch 32 --iters 10 --scale 1.0 > $O/post_nx.txt 2>&1 &&
timeout -k 10 200 python3 tools/post_prof.py --batch 1 --iters 20 > $O/post_r1.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/post_prof.py --batch 32 --iters 5 > $O/tr.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tn -o run -- python3 tools/post_prof.py --batch 32 --iters 5 --scale 1.0 > $O/tn.log 2>&1
rc=$?
cat $O/tile_r.json $O/tile_n.json; grep -h post_ms $O/post_*.txt; tail -3 $O/tile.err
exit $rc
