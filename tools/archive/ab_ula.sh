# Row-union loaders at the step's top (ISLPOSE_X3_ULA=1) vs after the kx = 0 group: Mode N op
# tables and bench, interleaved.  usage: bash tools/ab_ula.sh <tag>
export TMPDIR=/tmp
T=${1:-ula}; O=gpurun_out/$T; mkdir -p $O
for m in 0 1 0b 1b; do
  ISLPOSE_X3_ULA=${m:0:1} timeout -k 10 200 python3 tools/op_table.py --batch 32 --runs 5 > $O/ops_N_$m.txt 2>&1 || exit 1
  grep -m1 "net" $O/ops_N_$m.txt | sed "s/^/$m /"
done
bash tools/ab_bench.sh $T off:ISLPOSE_X3_ULA=0 on:ISLPOSE_X3_ULA=1 offb:ISLPOSE_X3_ULA=0 onb:ISLPOSE_X3_ULA=1
