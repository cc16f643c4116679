export TMPDIR=/tmp
O=gpurun_out/${1:-s96}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hand.py tests/test_gpu_configs.py tests/test_gpu_wino2.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.txt | head; exit $rc; }
timeout -k 10 200 python3 tools/op_table.py --kind hand --batch 1 --h 736 --w 736 --runs 5 > $O/ops_736_new.txt 2>&1 &&
ISLPOSE_X3_S7W96=0 timeout -k 10 200 python3 tools/op_table.py --kind hand --batch 1 --h 736 --w 736 --runs 5 > $O/ops_736_old.txt 2>&1 &&
for v in 1 0 1 0; do
  ISLPOSE_X3_S7W96=$v timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_$v.json 2>>$O/frame.err || exit 1
  python3 -c "import json; d=json.load(open('$O/frame_$v.json')); print('s7w96 $v', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])"
done
sed -n 2,4p $O/ops_736_new.txt; sed -n 2,4p $O/ops_736_old.txt
