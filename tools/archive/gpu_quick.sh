# parity tests (body) + bench (x3) + kernel trace.  usage: bash tools/archive/gpu_quick.sh <tag>
set -o pipefail
export TMPDIR=/tmp
T=${1:-q}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_body.py -m gpu -x -q -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 ; rc=$?
grep -E "rel err|passed|failed|Error" $O/pytest.log | head -20
[ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit $rc; }
timeout -k 10 200 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('fps',d['value'],'net_ms',r['net_ms_per_step'],'conv TF(fp16 alg)',r['achieved'],'frac',r['frac'],'fp32eq',r['fp32_equiv_tflops'], r['ms_per_step_by_kind'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/trace.log 2>&1
