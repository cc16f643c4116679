# One GPU call: the -m gpu suite, then the default bench line.
# usage: bash tools/archive/gpu_tests_bench.sh <tag>   (outputs under gpurun_out/<tag>)
# A test failure (pytest rc 1) still runs the bench; a fault, abort or timeout stops.
T=${1:-r2}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
rb=$?
cat $O/bench.json
echo "pytest rc=$rc bench rc=$rb"
exit $rb
