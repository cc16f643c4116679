# Round 4: 96-channel split-K layers on 64-pixel blocks (x3_px64) -- parity tests, then the bench
# line A/B (ISLPOSE_X3_PX64=0), twice each, interleaved.
T=${1:-r4ag}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_body.py::test_x3_px64_c96_split_bit_identical" "tests/test_gpu_body.py::test_canonical_ranges_batch_invariant" \
  "tests/test_gpu_body.py::test_x3_halfco_default_selection" "tests/test_gpu_body.py::test_body25_forward_vs_oracle" \
  tests/test_gpu_configs.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/p1_$i.json 2>> $O/err.log || exit 1
  ISLPOSE_X3_PX64=0 timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/p0_$i.json 2>> $O/err.log || exit 1
done
python3 - "$O" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/p*.json')):
    d = json.load(open(f))
    print(f, 'N', d['value'], d['roofline']['frac'], 'R32', d['mode_r']['batch32']['frames_per_s'], 'R1', d['mode_r']['batch1']['frames_per_s'])
PY
