# Round 4: graph replay A/B on the bench line (twice each, interleaved).
T=${1:-r4v}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/g1_$i.json 2>> $O/err.log || exit 1
  ISLPOSE_NET_GRAPH=0 timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/g0_$i.json 2>> $O/err.log || exit 1
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/r4v/g*.json')):
    d = json.load(open(f))
    print(f, 'N', d['value'], d['roofline']['frac'], 'R32', d['mode_r']['batch32']['frames_per_s'], 'R1', d['mode_r']['batch1']['frames_per_s'])
PY
