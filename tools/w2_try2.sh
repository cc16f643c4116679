# wino_f16 (8-wave form) parity tests, then per-shape convbench vs conv_x3 with ablations,
# then the op table and bench with and without it.  usage: bash tools/w2_try2.sh <tag>
export TMPDIR=/tmp
T=${1:-w2b}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wino2.py -x -v -s --timeout 200 --timeout-method thread > $O/w2test.log 2>&1
rc=$?
tail -12 $O/w2test.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
run() { echo "== $*" >> $O/abl.txt; timeout -k 10 120 "$@" >> $O/abl.txt 2>&1; }
for shape in "3 128 128 46 82 32" "3 384 128 46 82 32" "3 256 256 92 164 32" "3 512 512 46 82 32"; do
  run tools/convbench $shape 10 x3,w2 2 || exit 1
  for k in 16 2 1 3 31; do
    ISLPOSE_W2_ABL=$k run tools/convbench $shape 10 w2 1 || exit 1
  done
done
grep -E "==|round" $O/abl.txt | sed 's/tools.convbench //'
timeout -k 10 300 python3 tools/op_table.py --batch 32 > $O/ops_w2.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --frame-count 0 > $O/bench_w2.json 2> $O/bench_w2.err &&
ISLPOSE_X3_W2=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --frame-count 0 > $O/bench_x3.json 2> $O/bench_x3.err
rb=$?
head -24 $O/ops_w2.txt
python3 -c "
import json
for f in ('bench_w2', 'bench_x3'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('ms_per_step_by_kind'))
"
exit $rb
