export TMPDIR=/tmp
O=gpurun_out/${1:-fx1}; mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; tail -3 $O/gputest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/gputest.log | head; exit $rc; }
R="python3 bench.py --scale 0.5 --batch 1 --steps 300 --warmup 20 --no-cpu --no-mode-r --e2e-steps 0 --frame-count 0 --no-op-timing"
for v in 1 0 1 0; do
  ISLPOSE_X3_FIXUP=$v timeout -k 10 200 $R > $O/r1_$v.json 2>>$O/r1.err || exit 1
  python3 -c "import json; print('fixup $v', json.load(open('$O/r1_$v.json'))['value'])"
done
timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame.json 2>$O/frame.err && python3 -c "import json; print('frame', json.load(open('$O/frame.json'))['frames_per_s'])"
