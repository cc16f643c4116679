# A/B: the row union on 16x16x32 (x3m) vs 32x32x16 (x3), interleaved per layer shape, then the
# M16 parity test and the bench with ISLPOSE_X3_M16=0/1.
# usage: bash tools/archive/gpu_m16.sh <tag>
T=${1:-m16}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
CB=tools/convbench
for s in "3 128 128 46 82 32" "3 384 128 46 82 32" "3 512 512 46 82 32" "3 256 512 46 82 32" \
         "3 256 256 92 164 32" "3 128 256 92 164 32"; do
  echo "== $s" >> $O/ab.txt
  timeout -k 10 120 $CB $s 20 x3,x3m 3 >> $O/ab.txt 2>&1 || { echo "convbench failed: $s"; tail $O/ab.txt; exit 1; }
done
cat $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py -x -v --timeout 300 --timeout-method thread \
  -k "m16 or timed_config" > $O/test.log 2>&1; rc=$?
tail -4 $O/test.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  ISLPOSE_X3_M16=0 timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/bench0_$i.json 2>> $O/bench.err &&
  ISLPOSE_X3_M16=1 timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/bench1_$i.json 2>> $O/bench.err || exit 1
done
python3 -c "
import json
for i in (1,2):
  for m in (0,1):
    d=json.load(open('$O/bench%d_%d.json'%(m,i)))
    print('m16=%d'%m, d['value'], 'frac', d['roofline']['frac'], 'avg_us', d['roofline']['avg_launch_us'])
"
