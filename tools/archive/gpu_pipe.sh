# Pipelined C5 (ISLSignPos.call_batches): the affected -m gpu tests, C5 host timeline, C5 at batch 16 / 32.
export TMPDIR=/tmp
T=${1:-pipe}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_compat.py tests/test_pipeline.py tests/test_gpu_configs.py tests/test_gpu_hand.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/c5_timeline.py 96 2 32 > $O/c5tl.txt 2>&1 &&
timeout -k 10 600 python3 -u tools/bench_configs.py --config c5 --c5-overlap-only --c5-batch 16 > $O/c5_b16.json 2> $O/c5.err &&
timeout -k 10 600 python3 -u tools/bench_configs.py --config c5 --c5-overlap-only --c5-batch 32 > $O/c5_b32.json 2>> $O/c5.err
rc=$?
cat $O/c5tl.txt $O/c5_b16.json $O/c5_b32.json
exit $rc
