export TMPDIR=/tmp
O=gpurun_out/${1:-lk2}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_body.py tests/test_gpu_configs.py tests/test_gpu_compat.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.txt | head; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d -o run -- python3 tools/bench_configs.py --config frame --frame-count 16 --frame-repeat 1 > $O/d.log 2>&1 &&
grep -E "limb_kernel|compact_kernel" $O/d/run_kernel_stats.csv | awk -F, '{printf "%s calls %s avg %.1f us\n", substr($1,1,50), $2, $4/1000}' &&
for i in 1 2; do timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_$i.json 2>>$O/frame.err && python3 -c "import json; d=json.load(open('$O/frame_$i.json')); print('frame', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])" || exit 1; done
