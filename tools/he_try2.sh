export TMPDIR=/tmp
O=gpurun_out/${1:-cp2}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_body.py tests/test_gpu_configs.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.txt | head; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d -o run -- python3 tools/bench_configs.py --config frame --frame-count 16 --frame-repeat 1 > $O/d.log 2>&1 &&
python3 -c "
import csv
for r in csv.DictReader(open('$O/d/run_kernel_stats.csv')):
    if 'compact' in r['Name']: print(r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3)
"
