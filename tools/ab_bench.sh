#!/bin/bash
# A/B of the whole bench line (Mode N headline + Mode R batch 32 / batch 1 legs) on one box: for
# each "NAME:ENV=V,ENV=V" argument, bench.py without the CPU baseline into gpurun_out/<tag>/.
# usage: bash tools/ab_bench.sh <tag> base: c12off:ISLPOSE_C12=0 ...
export TMPDIR=/tmp
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 300 python3 bench.py --no-cpu --e2e-steps 0 > $O/bench_$name.json 2> $O/bench_$name.err ) || exit 1
  python3 -c "
import json; d=json.load(open('$O/bench_$name.json')); r=d['mode_r']
print('$name', 'N', d['value'], d['roofline']['frac'], 'post', d['post']['ms_per_step'], 'R32', r['batch32']['frames_per_s'], r['batch32']['roofline']['frac'], 'R1', r['batch1']['frames_per_s'])"
done
