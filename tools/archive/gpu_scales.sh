# Pyramid scales on their own streams: the -m gpu suite, then C3 / C4 / C5 and the default bench.
export TMPDIR=/tmp
T=${1:-scales}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -3 $O/gputest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $O/gputest.log | head -30; exit $rc; fi
timeout -k 10 600 python3 -u tools/bench_configs.py --config c3 > $O/c3.json 2> $O/cfg.err &&
timeout -k 10 600 python3 -u tools/bench_configs.py --config c4 > $O/c4.json 2>> $O/cfg.err &&
timeout -k 10 600 python3 -u tools/bench_configs.py --config c5 --c5-overlap-only > $O/c5.json 2>> $O/cfg.err
rc=$?
cat $O/c3.json $O/c4.json $O/c5.json
exit $rc
