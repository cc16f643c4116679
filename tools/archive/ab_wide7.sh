# 7x7 tile width A/B on the hand scales of C3 (batch 32 crops): default (by grid estimate) vs
# forced 128 / 256 / 384-pixel tiles.  usage: bash tools/ab_wide7.sh <tag>
export TMPDIR=/tmp
T=${1:-w7}; O=gpurun_out/$T; mkdir -p $O
for s in 552 368; do
  for m in d 1 3 0; do
    if [ $m = d ]; then unset ISLPOSE_X3_WIDE7; else export ISLPOSE_X3_WIDE7=$m; fi
    timeout -k 10 200 python3 tools/op_table.py --kind hand --batch 32 --h $s --w $s --runs 3 > $O/ops_${s}_$m.txt 2>&1 || exit 1
    grep -m1 "net" $O/ops_${s}_$m.txt | sed "s/^/$s $m /"
  done
done
