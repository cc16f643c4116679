set -o pipefail
export TMPDIR=/tmp
T=$1; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 ; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('fps',d['value'],'ms',d['ms_per_step'],'net_ms',r['net_ms_per_step'],'TF',r['achieved'],'frac',r['frac'], r['ms_per_step_by_kind'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/trace.log 2>&1
