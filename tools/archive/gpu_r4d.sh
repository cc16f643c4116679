# Round 4: resize / blur-band A/B, the whole -m gpu suite, the bench line, configs C3-C5.
T=${1:-r4d}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/resize_ab.py > $O/resize_ab.json 2>&1 || { echo "resize_ab failed"; tail -5 $O/resize_ab.json; exit 1; }
tail -1 $O/resize_ab.json
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -3 $O/gputest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err &&
timeout -k 10 600 python -u tools/bench_configs.py --config c3 > $O/c3.json 2>> $O/bench.err &&
timeout -k 10 600 python -u tools/bench_configs.py --config c5 > $O/c5.json 2>> $O/bench.err
rb=$?
python3 -c "
import json
d=json.load(open('$O/bench.json'))
print('N', d['value'], d['roofline']['frac'], 'post', d['post']['ms_per_step'], 'R32', d['mode_r']['batch32']['frames_per_s'], d['mode_r']['batch32']['roofline']['frac'], d['mode_r']['batch32']['post_ms_per_step'], 'R1', d['mode_r']['batch1']['frames_per_s'], d['mode_r']['batch1']['post_ms_per_step'])
"
cat $O/c3.json $O/c5.json
exit $rb
