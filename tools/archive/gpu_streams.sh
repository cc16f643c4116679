set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for s in 1 2 4; do
  timeout -k 10 200 python -u bench.py --no-cpu --streams $s > $O/bench_s$s.json 2> $O/bench_s$s.err || { cat $O/bench_s$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_s$s.json'));r=d['roofline'];print('streams $s fps',d['value'],'net_ms',r['net_ms_per_step'])"
done
