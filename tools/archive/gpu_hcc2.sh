# Hand post check: hand GPU tests (bit-exact), hand post timing, C5 host timeline and C5 / C3.
export TMPDIR=/tmp
T=${1:-hcc}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_hand.py tests/test_gpu_configs.py -v --timeout 200 --timeout-method thread > $O/hand_tests.log 2>&1
rc=$?
tail -3 $O/hand_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/hand_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python3 -u tools/hand_post_timing.py 150 600 1000 > $O/hand_post_timing.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/c5_timeline.py 96 2 32 > $O/c5tl.txt 2>&1 &&
timeout -k 10 600 python3 -u tools/bench_configs.py --config c5 --c5-overlap-only > $O/c5.json 2> $O/c5.err &&
timeout -k 10 600 python3 -u tools/bench_configs.py --config c3 > $O/c3.json 2>> $O/c5.err
rc=$?
cat $O/hand_post_timing.txt $O/c5tl.txt $O/c5.json $O/c3.json
exit $rc
