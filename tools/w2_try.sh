# Winograd (wino_f16) first GPU check: parity tests, then op tables and the bench with and without it.
# usage: bash tools/w2_try.sh <tag>   (gpurun_out/<tag>)
export TMPDIR=/tmp
T=${1:-w2a}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wino2.py -x -v -s --timeout 200 --timeout-method thread > $O/w2test.log 2>&1
rc=$?
tail -15 $O/w2test.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 tools/op_table.py --batch 32 > $O/ops_w2.txt 2>&1 &&
ISLPOSE_X3_W2=0 timeout -k 10 300 python3 tools/op_table.py --batch 32 > $O/ops_x3.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_w2.json 2> $O/bench_w2.err &&
ISLPOSE_X3_W2=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_x3.json 2> $O/bench_x3.err
rb=$?
head -30 $O/ops_w2.txt; head -30 $O/ops_x3.txt
python3 -c "
import json
for f in ('bench_w2', 'bench_x3'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'])
"
exit $rb
