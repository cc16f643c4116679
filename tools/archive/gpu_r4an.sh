# Round 4 (A/B): the bench line with the post beside the next batch's net (--post-overlap) vs
# serial (default), interleaved, twice -- after the fp32 blur filter made the post cheaper.
T=${1:-r4an}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/ser_$i.json 2>> $O/err.log || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 --post-overlap > $O/ovl_$i.json 2>> $O/err.log || exit 1
done
python3 - "$O" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/*.json')):
    d = json.load(open(f))
    r = d['mode_r']
    print(f, 'N', d['value'], d['roofline']['frac'], 'R32', r['batch32']['frames_per_s'], r['batch32']['roofline']['frac'], 'R1', r['batch1']['frames_per_s'], r['batch1']['roofline']['frac'])
PY
