# Round 3: PPS2 (canonical-range layers) parity + Mode R A/B; Mode R kernel trace (post breakdown).
T=${1:-r3e}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py -x -q --timeout 200 --timeout-method thread \
  > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
for i in 1 2; do
  for h in 0 1; do
    ISLPOSE_X3_PPS2=$h timeout -k 10 200 python -u bench.py --scale 0.5 --no-cpu --e2e-steps 0 > $O/b32_p${h}_$i.json 2>> $O/bench.err || exit 1
    ISLPOSE_X3_PPS2=$h timeout -k 10 200 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --e2e-steps 0 > $O/b1_p${h}_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for h in (0,1):
    for b in ('b32','b1'):
      d=json.load(open('$O/%s_p%d_%d.json'%(b,h,i)))
      print(b, 'pps2=%d'%h, d['value'], 'frac', d['roofline']['frac'], 'post_ms', d['post']['ms_per_step'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_R -o run -- python3 bench.py --scale 0.5 --no-cpu --e2e-steps 0 --steps 3 --warmup 1 > $O/trace_R.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_R1 -o run -- python3 bench.py --scale 0.5 --batch 1 --no-cpu --e2e-steps 0 --steps 20 --warmup 3 > $O/trace_R1.log 2>&1
f=$(find $O/trace_R -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -30 $f
