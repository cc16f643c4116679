# A/B: small grids with inputs and weights two K steps ahead (x3d, ISLPOSE_X3_DEEP=1) vs the
# default 128-pixel loop (x3): bit-identity test, per-layer timings (Mode R 23x41, batch 32
# and 1), then Mode R bench at batch 32 and 1.  usage: bash tools/archive/gpu_deep.sh <tag> [bench]
T=${1:-deep}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py -x -v --timeout 300 --timeout-method thread \
  -k "deep or canonical" > $O/test.log 2>&1; rc=$?
tail -5 $O/test.log
[ $rc -ne 0 ] && exit $rc
CB=tools/convbench
for s in "3 128 128 23 41 32" "3 384 128 23 41 32" "3 96 96 23 41 32" "1 384 512 23 41 32" "3 128 128 23 41 1" "3 384 128 23 41 1"; do
  echo "== $s" >> $O/ab.txt
  timeout -k 10 120 $CB $s 40 x3,x3d 3 >> $O/ab.txt 2>&1 || { echo "convbench failed: $s"; tail $O/ab.txt; exit 1; }
done
grep "==\|round [12]" $O/ab.txt
[ "$2" = "bench" ] || exit 0
for i in 1 2; do
  for d in 0 1; do
    ISLPOSE_X3_DEEP=$d timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/b32_d${d}_$i.json 2>> $O/bench.err &&
    ISLPOSE_X3_DEEP=$d timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_d${d}_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for d in (0,1):
    for b in ('b32','b1'):
      x=json.load(open('$O/%s_d%d_%d.json'%(b,d,i)))
      print(b, 'deep=%d'%d, x['value'], 'frac', x['roofline']['frac'])
"
