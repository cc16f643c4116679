# Round 4 (A/B, done): Mode R batch 32's ranged c96 deep layers on 64-pixel blocks (ISLPOSE_X3_PX64B=1;
# measured 38-45 % slower per layer, profiles/r04/r4am/, and removed: the switch no longer exists).
T=${1:-r4am}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
ISLPOSE_X3_PX64B=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_body.py::test_canonical_ranges_batch_invariant" > $O/tests.log 2>&1 || exit 1
for p in 0 1; do
  ISLPOSE_X3_PX64B=$p timeout -k 10 120 python -u tools/op_table.py --batch 32 --h 184 --w 328 --runs 10 > $O/ops_b32_p$p.txt 2>&1 || exit 1
done
for i in 1 2; do for p in 0 1; do
  ISLPOSE_X3_PX64B=$p timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/p${p}_$i.json 2>> $O/err.log || exit 1
done; done
grep -h "net " $O/ops_b32_*.txt
python3 - "$O" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/p*.json')):
    d = json.load(open(f))
    print(f, 'N', d['value'], 'R32', d['mode_r']['batch32']['frames_per_s'], d['mode_r']['batch32']['roofline']['frac'], 'R1', d['mode_r']['batch1']['frames_per_s'])
PY
