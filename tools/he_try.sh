export TMPDIR=/tmp
O=gpurun_out/${1:-lz1}; mkdir -p $O
for z in d 32 64; do
  if [ $z = d ]; then timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/z$z -o run -- python3 tools/bench_configs.py --config frame --frame-count 16 --frame-repeat 1 > $O/z$z.log 2>&1 || exit 1
  else ISLPOSE_LIMB_Z=$z timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/z$z -o run -- python3 tools/bench_configs.py --config frame --frame-count 16 --frame-repeat 1 > $O/z$z.log 2>&1 || exit 1; fi
  python3 -c "
import csv
for r in csv.DictReader(open('$O/z$z/run_kernel_stats.csv')):
    if 'limb' in r['Name']: print('$z', r['Name'][:40], r['Calls'], '%.1f' % (float(r['AverageNs'])/1e3))
"
done
