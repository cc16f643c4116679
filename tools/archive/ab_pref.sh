# L2 prefetch at the start of the generic conv loops (ISLPOSE_X3_PREF=1) vs off: Mode R batch-32
# op tables and the bench line, interleaved.  usage: bash tools/ab_pref.sh <tag>
export TMPDIR=/tmp
T=${1:-pf}; O=gpurun_out/$T; mkdir -p $O
for m in 0 1 0b 1b; do
  ISLPOSE_X3_PREF=${m:0:1} timeout -k 10 200 python3 tools/op_table.py --batch 32 --h 184 --w 328 --runs 5 > $O/ops_R32_$m.txt 2>&1 || exit 1
  grep -m1 "net" $O/ops_R32_$m.txt | sed "s/^/$m /"
done
bash tools/ab_bench.sh $T off:ISLPOSE_X3_PREF=0 on:ISLPOSE_X3_PREF=1
