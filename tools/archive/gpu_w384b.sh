# 7x7 tile choice by grid quantisation (128 / 256 / 384 px): the -m gpu suite, hand layer table,
# C3 / C4 / C5 and the default bench.
export TMPDIR=/tmp
T=${1:-w384b}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -3 $O/gputest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $O/gputest.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/net_layers.py hand 32 184 368 552 736 > $O/hand_layers.txt 2>/dev/null &&
timeout -k 10 600 python3 -u tools/bench_configs.py --config c3 > $O/c3.json 2> $O/cfg.err &&
timeout -k 10 600 python3 -u tools/bench_configs.py --config c4 > $O/c4.json 2>> $O/cfg.err &&
timeout -k 10 600 python3 -u tools/bench_configs.py --config c5 --c5-overlap-only > $O/c5.json 2>> $O/cfg.err &&
timeout -k 10 300 python3 -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
grep "==\|k7" $O/hand_layers.txt; cat $O/c3.json $O/c4.json $O/c5.json; python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'])"
exit $rc
