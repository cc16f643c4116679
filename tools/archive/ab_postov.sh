# The post beside the next batch's net (--post-overlap) vs in line, interleaved, Mode N and
# Mode R batch 32.  usage: bash tools/ab_postov.sh <tag>
export TMPDIR=/tmp
T=${1:-po}; O=gpurun_out/$T; mkdir -p $O
for k in off on offb onb; do
  f=""; [ "${k:0:2}" = "on" ] && f="--post-overlap"
  timeout -k 10 300 python3 bench.py --no-cpu --e2e-steps 0 $f > $O/bench_$k.json 2> $O/bench_$k.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/bench_$k.json')); r=d['mode_r']
print('$k', 'N', d['value'], d['roofline']['frac'], 'post', d['post']['ms_per_step'], 'R32', r['batch32']['frames_per_s'], r['batch32']['roofline']['frac'], 'R1', r['batch1']['frames_per_s'])"
done
