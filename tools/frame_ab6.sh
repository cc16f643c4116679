# Frame path after the stream fork fix: hand/pyramid GPU tests, FRAME/C3/C4 with the default
# hardware queues and with GPU_MAX_HW_QUEUES=8, a kernel trace of 16 frames.
# usage: bash tools/frame_ab6.sh <tag>   (gpurun_out/<tag>)
export TMPDIR=/tmp
T=${1:-fr6b}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hand.py tests/test_gpu_configs.py tests/test_gpu_compat.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python3 tools/bench_configs.py --config frame --frame-count 64 > $O/frame_q4.json 2>$O/frame_q4.err &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 tools/bench_configs.py --config frame --frame-count 64 > $O/frame_q8.json 2>$O/frame_q8.err &&
timeout -k 10 300 python3 tools/bench_configs.py --config c3 > $O/c3_q4.json 2>$O/c3.err &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 tools/bench_configs.py --config c3 > $O/c3_q8.json 2>>$O/c3.err &&
timeout -k 10 300 python3 tools/bench_configs.py --config c4 > $O/c4_q4.json 2>$O/c4.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config frame --frame-count 16 > $O/trace.log 2>&1
rc=$?
tail -3 $O/tests.txt; cat $O/frame_q4.json $O/frame_q8.json $O/c3_q4.json $O/c3_q8.json $O/c4_q4.json 2>/dev/null
exit $rc
