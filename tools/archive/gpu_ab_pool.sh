# Fused 2x2 pools (pair-max conv epilogue + row-pair pool) vs conv + maxpool2: parity tests, then the bench interleaved.
export TMPDIR=/tmp
O=gpurun_out/${1:-abp}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_body.py tests/test_gpu_configs.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for f in 0 1; do
    ISLPOSE_FUSED_POOL=$f timeout -k 10 300 python3 bench.py --no-cpu --e2e-steps 0 > $O/b_${f}_$r.json 2>> $O/bench.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${f}_$r.json')); print('fused=$f', d['value'], d['ms_per_step'], d['roofline']['ms_per_step_by_kind'])"
  done
done
