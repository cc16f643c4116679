#!/bin/bash
# Op tables (tools/op_table.py, HIP events per op) of one net size for several switch settings.
# usage: bash tools/ab_ops.sh <tag> <batch> <h> <w> NAME:ENV=V,ENV=V ...
export TMPDIR=/tmp
T=$1; B=$2; H=$3; W=$4; shift 4; O=gpurun_out/$T; mkdir -p $O
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 180 python3 tools/op_table.py --batch $B --h $H --w $W --runs 10 > $O/ops_${name}_b$B.txt 2>&1 ) || exit 1
done
