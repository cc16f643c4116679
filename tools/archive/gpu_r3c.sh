# Round 3: half-channel-tile small grids (VAR 256) A/B: convbench per Mode R layer shape at
# batch 32 (in-block canonical ranges) and batch 1 (across blocks), parity, Mode R bench.
T=${1:-r3c}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
CB=tools/convbench
for n in 32 1; do
  for s in "3 128 128 23 41 $n" "3 384 128 23 41 $n" "3 96 96 23 41 $n" "3 288 96 23 41 $n" "1 384 512 23 41 $n" "3 512 512 23 41 $n"; do
    echo "== $s" >> $O/ab.txt
    CONVBENCH_SPLIT=1 timeout -k 10 120 $CB $s 50 x3,x3h 3 >> $O/ab.txt 2>&1 || { echo "convbench failed: $s"; tail $O/ab.txt; exit 1; }
  done
done
grep -E "==|round 2" $O/ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_body.py -x -q --timeout 120 --timeout-method thread \
  -k "halfco or canonical" > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
tail -2 $O/test.log
for i in 1 2; do
  for h in 0 1; do
    ISLPOSE_X3_HALFCO=$h timeout -k 10 200 python -u bench.py --scale 0.5 --no-cpu --e2e-steps 0 > $O/b32_h${h}_$i.json 2>> $O/bench.err || exit 1
    ISLPOSE_X3_HALFCO=$h timeout -k 10 200 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --e2e-steps 0 > $O/b1_h${h}_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for h in (0,1):
    for b in ('b32','b1'):
      d=json.load(open('$O/%s_h%d_%d.json'%(b,h,i)))
      print(b, 'halfco=%d'%h, d['value'], 'frac', d['roofline']['frac'])
"
