export TMPDIR=/tmp
O=gpurun_out/${1:-lz2}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_body.py tests/test_gpu_configs.py tests/test_gpu_compat.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.txt | head; exit $rc; }
for i in 1 2; do timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_$i.json 2>>$O/frame.err && python3 -c "import json; d=json.load(open('$O/frame_$i.json')); print('frame', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])" || exit 1; done
timeout -k 10 400 python3 bench.py --no-cpu --frame-count 0 --e2e-steps 0 > $O/bench.json 2>$O/bench.err && python3 -c "
import json; d=json.load(open('$O/bench.json')); print('N', d['value'], 'post', d['post']['ms_per_step'], 'R32', d['mode_r']['batch32']['frames_per_s'], d['mode_r']['batch32']['post_ms_per_step'], 'R1', d['mode_r']['batch1']['frames_per_s'], d['mode_r']['batch1']['post_ms_per_step'])"
