# Round 3: split-K fold A/B at batch 1 (Mode R), then the 16x16x32 union A/B (tools/archive/gpu_m16.sh).
T=${1:-r3b}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_body.py -x -q --timeout 120 --timeout-method thread \
  -k "fold or canonical or splitk_small" > $O/fold_test.log 2>&1 || { tail -20 $O/fold_test.log; exit 1; }
tail -2 $O/fold_test.log
for i in 1 2; do
  for f in 0 1; do
    ISLPOSE_X3_FOLD=$f timeout -k 10 200 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --e2e-steps 0 \
      > $O/b1_fold${f}_$i.json 2>> $O/bench.err || exit 1
  done
done
ISLPOSE_X3_FOLD=1 timeout -k 10 200 python -u tools/op_table.py --batch 1 --h 184 --w 328 --runs 20 > $O/ops_R_b1_fold1.txt 2>&1
ISLPOSE_X3_FOLD=0 timeout -k 10 200 python -u tools/op_table.py --batch 1 --h 184 --w 328 --runs 20 > $O/ops_R_b1_fold0.txt 2>&1
python3 -c "
import json
for i in (1,2):
  for f in (0,1):
    d=json.load(open('$O/b1_fold%d_%d.json'%(f,i)))
    print('fold=%d'%f, d['value'], 'frac', d['roofline']['frac'])
"
bash tools/archive/gpu_m16.sh $T
