# First split-fp16 conv check: parity tests then A/B bench of the three conv algorithms.
set -o pipefail
export TMPDIR=/tmp
T=${1:-x3}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_body.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 ; rc=$?
echo pytest rc=$rc
tail -25 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for a in x3 wino; do
  timeout -k 10 200 python -u bench.py --no-cpu --algo $a > $O/bench_$a.json 2> $O/bench_$a.err || exit 1
  cat $O/bench_$a.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/trace.log 2>&1
