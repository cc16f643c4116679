# Round-6 checkpoint: the whole -m gpu suite, smoke(), then the bench line and the C3 / C4 / C5 /
# FRAME configs.  usage: bash tools/checkpoint_r6.sh <tag>   (gpurun_out/<tag>)
export TMPDIR=/tmp
T=${1:-ck6}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -3 $O/gputest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|error" $O/gputest.log | head -20; echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 600 python3 tools/bench_configs.py --config c3 > $O/c3.json 2>> $O/cfg.err &&
timeout -k 10 600 python3 tools/bench_configs.py --config c4 > $O/c4.json 2>> $O/cfg.err &&
timeout -k 10 600 python3 tools/bench_configs.py --config c5 > $O/c5.json 2>> $O/cfg.err
rb=$?
python3 -c "
import json
d=json.load(open('$O/bench.json')); r=d['mode_r']
print('N', d['value'], d['roofline']['frac'], 'post', d['post']['ms_per_step'], 'R32', r['batch32']['frames_per_s'], r['batch32']['roofline']['frac'], 'post', r['batch32']['post_ms_per_step'], 'R1', r['batch1']['frames_per_s'], 'cpu', d['cpu_baseline']['value'])
print('frame', d.get('frame'))
for c in ('c3', 'c4', 'c5'):
    try: j = json.load(open('$O/' + c + '.json')); print(c, j.get('frames_per_s', j.get('overlap_frames_per_s')))
    except Exception as e: print(c, 'n/a', e)
"
echo "pytest rc=$rc bench rc=$rb"
exit $rb
