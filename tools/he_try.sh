export TMPDIR=/tmp
O=gpurun_out/${1:-he15}; mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.json 2>$O/bench.err
rc=$?
python3 -c "
import json
d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['mode_r']['batch1']['frames_per_s'], d['frame'])
"
exit $rc
