# Round 4: post correctness tests (goldens, designed batches, configs) and batch-1 / 32 post traces.
T=${1:-r4s}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_blur_filter.py \
  "tests/test_gpu_body.py::test_body_post_golden_bit_exact" "tests/test_gpu_body.py::test_designed_maps_batch_bit_exact" \
  "tests/test_gpu_body.py::test_body_estimate_end_to_end" "tests/test_gpu_body.py::test_launch_post_stream_equals_estimate" \
  tests/test_gpu_configs.py tests/test_gpu_compat.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t1 -o run -- python3 tools/post_prof.py --batch 1 --iters 20 > $O/t1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t32 -o run -- python3 tools/post_prof.py --batch 32 --iters 5 > $O/t32.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tn -o run -- python3 tools/post_prof.py --batch 32 --iters 5 --scale 1.0 > $O/tn.log 2>&1
