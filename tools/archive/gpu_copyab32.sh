# Batch-32 steps: records D2H on the copy stream (ISLPOSE_BENCH_COPY_STREAM=1, the default above 1 MB) vs on
# the post stream (=0); Mode N and Mode R, interleaved twice.
T=${1:-copyab32}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for v in 1 0; do
    ISLPOSE_BENCH_COPY_STREAM=$v timeout -k 10 300 python -u bench.py --no-cpu --no-mode-r --e2e-steps 0 > $O/N_c${v}_$i.json 2>> $O/bench.err &&
    ISLPOSE_BENCH_COPY_STREAM=$v timeout -k 10 300 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/R_c${v}_$i.json 2>> $O/bench.err || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for v in (1,0):
    for m in ('N','R'):
      x=json.load(open('$O/%s_c%d_%d.json'%(m,v,i))); print(m, 'copy-stream' if v else 'same-stream', x['value'], 'ms', x['ms_per_step'], 'frac', x['roofline']['frac'])
"
