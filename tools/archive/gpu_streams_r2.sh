# Mode R batch 32 split over 2 streams with the small grids' K ranges kept in one block
# (ISLPOSE_X3_ACROSS=0): do two half-batch chains overlap each other's fixed costs?
T=${1:-strr2}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/s1_$i.json 2>> $O/err.txt &&
  ISLPOSE_X3_ACROSS=0 timeout -k 10 200 python -u bench.py --scale 0.5 --streams 2 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/s2_$i.json 2>> $O/err.txt &&
  ISLPOSE_X3_ACROSS=0 timeout -k 10 200 python -u bench.py --scale 0.5 --streams 4 --no-cpu --no-mode-r --e2e-steps 0 --steps 20 > $O/s4_$i.json 2>> $O/err.txt || exit 1
done
python3 -c "
import json
for i in (1,2):
  for s in (1,2,4):
    d=json.load(open('$O/s%d_%d.json'%(s,i)))
    print('streams', s, d['value'], 'ms', d['ms_per_step'], 'net', d['roofline']['net_ms_per_step'], 'frac', d['roofline']['frac'])
"
