# Mode R (net 184x328) at batch 32 with the batch split over 1 / 2 / 4 streams, interleaved twice
T=${1:-strr}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for s in 1 2 4; do
    timeout -k 10 200 python -u bench.py --scale 0.5 --streams $s --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/b32_s${s}_$i.json 2>> $O/err.txt || exit 1
  done
done
python3 -c "
import json
for i in (1,2):
  for s in (1,2,4):
    d=json.load(open('$O/b32_s%d_%d.json'%(s,i)))
    print('streams', s, d['value'], 'frac', d['roofline']['frac'], 'ms', d['ms_per_step'])
"
