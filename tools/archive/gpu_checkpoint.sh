# Checkpoint: the -m gpu suite, the default bench line, Mode R at batch 1 and 32, and the C3/C4/C5 configs.
# usage: bash tools/archive/gpu_checkpoint.sh <tag>   (outputs under gpurun_out/<tag>)
T=${1:-ck}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -3 $O/gputest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 50 --warmup 5 --no-cpu --e2e-steps 0 > $O/bench_modeR_b1.json 2>> $O/bench.err &&
timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --e2e-steps 0 > $O/bench_modeR_b32.json 2>> $O/bench.err &&
timeout -k 10 600 python -u tools/bench_configs.py --config c3 > $O/c3.json 2>> $O/bench.err &&
timeout -k 10 600 python -u tools/bench_configs.py --config c4 > $O/c4.json 2>> $O/bench.err &&
timeout -k 10 600 python -u tools/bench_configs.py --config c5 > $O/c5.json 2>> $O/bench.err
rb=$?
python3 -c "
import json,sys
for f in ['bench','bench_modeR_b1','bench_modeR_b32']:
    try:
        d=json.load(open('$O/'+f+'.json'))
        print(f, d['value'], d['unit'], 'frac', d['roofline']['frac'])
    except Exception as e: print(f, 'n/a', e)
"
cat $O/c3.json $O/c4.json $O/c5.json 2>/dev/null
echo "pytest rc=$rc bench rc=$rb"
exit $rb
