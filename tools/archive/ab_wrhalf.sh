# Wave-range blocks of 16 pixels at batch 1 (default) vs 32 (ISLPOSE_X3_WR_HALF=0): WR tests,
# batch-1 op tables and the bench's batch-1 leg, interleaved.  usage: bash tools/ab_wrhalf.sh <tag>
export TMPDIR=/tmp
T=${1:-wrh}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wr.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for m in 1 0 1b 0b; do
  ISLPOSE_X3_WR_HALF=${m:0:1} timeout -k 10 200 python3 tools/op_table.py --batch 1 --h 184 --w 328 --runs 20 > $O/ops_b1_$m.txt 2>&1 || exit 1
  grep -m1 "net" $O/ops_b1_$m.txt | sed "s/^/$m /"
done
for m in 1 0 1b 0b; do
  ISLPOSE_X3_WR_HALF=${m:0:1} timeout -k 10 300 python3 bench.py --no-cpu --e2e-steps 0 --scale 0.5 --batch 1 --steps 200 --warmup 10 > $O/b1_$m.json 2> $O/b1_$m.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b1_$m.json')); print('$m b1', d['value'], d['ms_per_step'])"
done
