#!/bin/bash
# A/B of batch-1 Mode R forms on one box: for each "NAME:ENV=V,ENV=V" argument, the op table
# (tools/op_table.py, HIP events per op) and the bench's batch-1 step (200 timed steps), into
# gpurun_out/<tag>/.  usage: bash tools/ab_b1.sh <tag> base: wr0:ISLPOSE_X3_WR=0 ...
export TMPDIR=/tmp
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 120 python3 tools/op_table.py --batch 1 --h 184 --w 328 --runs 20 > $O/ops_$name.txt 2>&1 &&
    timeout -k 10 180 python3 bench.py --batch 1 --scale 0.5 --no-mode-r --no-cpu --e2e-steps 0 --no-op-timing \
        --steps 200 --warmup 10 > $O/b1_$name.json 2> $O/b1_$name.err ) || exit 1
  python3 -c "import json; d=json.load(open('$O/b1_$name.json')); print('$name', d['value'], d['ms_per_step'])"
done
