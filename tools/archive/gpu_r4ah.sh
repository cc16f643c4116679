# Round 4: small-grid block forms at batch 1 -- parity, then the bench line A/B (interleaved, twice):
# ISLPOSE_X3_PX64 in {1 (default), 2} x ISLPOSE_X3_HALFSMALL in {0 (default), 1, 2}.
T=${1:-r4ah}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_body.py::test_x3_px64_c96_split_bit_identical" "tests/test_gpu_body.py::test_canonical_ranges_batch_invariant" \
  "tests/test_gpu_body.py::test_x3_halfco_default_selection" > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; fi
for i in 1 2; do
  for p in 1 2; do for h in 0 1 2; do
    ISLPOSE_X3_PX64=$p ISLPOSE_X3_HALFSMALL=$h timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/p${p}h${h}_$i.json 2>> $O/err.log || exit 1
  done; done
done
python3 - "$O" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/p*.json')):
    d = json.load(open(f))
    print(f, 'N', d['value'], d['roofline']['frac'], 'R32', d['mode_r']['batch32']['frames_per_s'], 'R1', d['mode_r']['batch1']['frames_per_s'])
PY
