# Mode N with the batch split over 1 / 2 streams (lanes), interleaved.  usage: bash tools/ab_streams.sh <tag>
export TMPDIR=/tmp
T=${1:-st}; O=gpurun_out/$T; mkdir -p $O
for k in s1 s2 s1b s2b; do
  n=${k:1:1}
  timeout -k 10 300 python3 bench.py --no-cpu --no-mode-r --e2e-steps 0 --streams $n > $O/bench_$k.json 2> $O/bench_$k.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/bench_$k.json')); print('$k', d['value'], d['roofline']['frac'], d['post']['ms_per_step'])"
done
