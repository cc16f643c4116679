# GPU suite, bench (Mode N default), Mode R batch 1 / 32 latency + throughput.
T=${1:-r2b}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -3 $O/gputest.log; grep -E "FAILED|ERROR" $O/gputest.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json;d=json.load(open('$O/bench.json'));print('modeN b32', d['value'], d['roofline']['frac'], d['e2e']['frames_per_s'])"
for b in 1 32; do
  timeout -k 10 300 python -u bench.py --no-cpu --scale 0.5 --batch $b --steps 20 > $O/bench_r_b$b.json 2>> $O/bench.err || exit 1
  python -c "import json;d=json.load(open('$O/bench_r_b$b.json'));print('modeR b$b', d['value'], d['ms_per_step'], d['e2e']['frames_per_s'])"
done
timeout -k 10 300 python -u bench.py --no-cpu --scale 0.5 --batch 1 --steps 20 --split-k > $O/bench_r_b1_sk2.json 2>> $O/bench.err || exit 1
python -c "import json;d=json.load(open('$O/bench_r_b1_sk2.json'));print('modeR b1 latency-mode', d['value'], d['ms_per_step'])"
echo "pytest rc=$rc"
