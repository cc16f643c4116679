set -o pipefail
export TMPDIR=/tmp
T=$1; O=gpurun_out/$T; mkdir -p $O
for s in "3 128 128 46 82 32" "3 384 128 46 82 32" "3 96 96 46 82 32" "3 256 256 92 164 32" "3 64 64 368 656 32" "3 512 512 46 82 32"; do
  timeout -k 10 120 tools/convbench $s 20 x3,wx3 3 >> $O/cb.txt 2>&1 || { echo "convbench failed: $s"; cat $O/cb.txt; exit 1; }
done
grep -E "conv|round 2" $O/cb.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_body.py -m gpu -x -q -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 ; rc=$?
grep -E "rel err|passed|failed|Error" $O/pytest.log | head -20
[ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit $rc; }
timeout -k 10 200 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('fps',d['value'],'net_ms',r['net_ms_per_step'],'TF',r['achieved'],'frac',r['frac'],'fp32eq',r['fp32_equiv_tflops'], r['ms_per_step_by_kind'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/trace.log 2>&1
