# Round-3 first checkpoint: -m gpu suite, bench Mode N / Mode R (b32, b1), per-op tables.
T=${1:-r3a}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -3 $O/gputest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --e2e-steps 0 > $O/bench_modeR_b32.json 2>> $O/bench.err &&
timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 50 --warmup 5 --no-cpu --e2e-steps 0 > $O/bench_modeR_b1.json 2>> $O/bench.err &&
timeout -k 10 200 python -u tools/op_table.py --batch 32 --h 368 --w 656 > $O/ops_N_b32.txt 2>&1 &&
timeout -k 10 200 python -u tools/op_table.py --batch 32 --h 184 --w 328 > $O/ops_R_b32.txt 2>&1 &&
timeout -k 10 200 python -u tools/op_table.py --batch 1 --h 184 --w 328 --runs 20 > $O/ops_R_b1.txt 2>&1
rb=$?
python3 -c "
import json
for f in ['bench','bench_modeR_b32','bench_modeR_b1']:
    try:
        d=json.load(open('$O/'+f+'.json'))
        print(f, d['value'], d['unit'], 'frac', d['roofline']['frac'], d.get('range_guard'))
    except Exception as e: print(f, 'n/a', e)
"
echo "pytest rc=$rc bench rc=$rb"
exit $rb
