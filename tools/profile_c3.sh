# C3 at HEAD: throughput (tools/bench_configs.py), a kernel trace of one C3 step, and per-op
# tables of the hand net at its four crop scales (batch 32 = C3's crops per step) and of the
# Mode R body at batch 16.  usage: bash tools/profile_c3.sh <tag>   (gpurun_out/<tag>)
export TMPDIR=/tmp
T=${1:-c3p}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python3 tools/bench_configs.py --config c3 --steps 5 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config c3 --steps 1 --warmup 1 > $O/trace.log 2>&1 &&
for s in 184 368 552 736; do
  timeout -k 10 200 python3 tools/op_table.py --kind hand --batch 32 --h $s --w $s --runs 3 > $O/ops_hand_$s.txt 2>&1 || exit 1
done &&
timeout -k 10 200 python3 tools/op_table.py --kind body25 --batch 16 --h 184 --w 328 --runs 5 > $O/ops_body_b16.txt 2>&1
rc=$?
cat $O/c3.json
echo rc=$rc
exit $rc
