# Round 4: the small-grid forms (x3_px64, x3_halfsmall) on vs off, interleaved on one box: the
# bench line and C3 (hand crops at small batch take them too), twice each.
T=${1:-r4ak}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/on_$i.json 2>> $O/err.log || exit 1
  ISLPOSE_X3_PX64=0 ISLPOSE_X3_HALFSMALL=0 timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/off_$i.json 2>> $O/err.log || exit 1
  timeout -k 10 300 python -u tools/bench_configs.py --config c3 > $O/c3on_$i.json 2>> $O/err.log || exit 1
  ISLPOSE_X3_PX64=0 ISLPOSE_X3_HALFSMALL=0 timeout -k 10 300 python -u tools/bench_configs.py --config c3 > $O/c3off_$i.json 2>> $O/err.log || exit 1
done
python3 - "$O" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/*.json')):
    d = json.load(open(f))
    if 'mode_r' in d:
        print(f, 'N', d['value'], 'R32', d['mode_r']['batch32']['frames_per_s'], 'R1', d['mode_r']['batch1']['frames_per_s'])
    else:
        print(f, 'C3', d['frames_per_s'])
PY
