export TMPDIR=/tmp
O=gpurun_out/${1:-np1}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hand.py tests/test_gpu_configs.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.txt | head; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pt -o run -- python3 tools/post_trace.py > $O/pt.log 2>&1 &&
python3 -c "
import csv
for r in csv.DictReader(open('$O/pt/run_kernel_stats.csv')):
    if 'hand_cc' in r['Name'] or 'bufsum' in r['Name']: print(r['Name'][:45], r['Calls'], '%.1f' % (float(r['AverageNs'])/1e3))
" &&
for i in 1 2; do timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_$i.json 2>>$O/frame.err && python3 -c "import json; d=json.load(open('$O/frame_$i.json')); print('frame', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])" || exit 1; done
