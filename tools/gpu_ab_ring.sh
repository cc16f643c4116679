# A/B: 3-buffer weight ring on the short-run union layers (default) vs 2 buffers (ISLPOSE_X3_RING=0).
export TMPDIR=/tmp
T=${1:-ring}; O=gpurun_out/$T; mkdir -p $O
for s in "3 128 128 46 82 32" "3 384 128 46 82 32" "3 96 96 46 82 32" "3 288 96 46 82 32" "3 512 512 46 82 32" "3 180 128 46 82 32"; do
  for r in 1 0; do
    echo "== $s ring=$r" >> $O/u.txt
    ISLPOSE_X3_RING=$r timeout -k 10 120 tools/convbench $s 20 x3 3 >> $O/u.txt 2>&1 || { echo "convbench failed: $s"; tail $O/u.txt; exit 1; }
  done
done
grep -E "==|round 2" $O/u.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py -m gpu -x -q --timeout 300 --timeout-method thread -k "forward or golden or estimate or invariant" > $O/parity.log 2>&1 || { echo parity failed; tail -20 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2; do
  for r in 1 0; do
    ISLPOSE_X3_RING=$r timeout -k 10 300 python bench.py --no-cpu --e2e-steps 0 > $O/bench_r$r.$i.json 2>> $O/bench.err || exit 1
    python -c "import json;d=json.load(open('$O/bench_r$r.$i.json'));print('ring=$r', d['value'], d['roofline']['frac'])"
  done
done
