# One GPU call: parity tests, smoke, bench (with CPU baseline), kernel-trace profile.
# usage: bash tools/archive/gpu_check.sh <tag>
set -o pipefail
export TMPDIR=/tmp
T=${1:-chk}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 python -u bench.py --scale 0.5 --no-cpu > $O/bench_r.json 2> $O/bench_r.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/trace.log 2>&1
rc=$?
echo rc=$rc
tail -3 $O/pytest.log; cat $O/smoke.log $O/bench.json $O/bench_r.json
exit $rc
