# Round 4 (A/B, done): the split small-grid blocks on 32 pixels (ISLPOSE_X3_PX64=3) vs 64 (default);
# measured level, profiles/r04/r4al/, and not built: =3 now runs the 64-pixel blocks.
T=${1:-r4al}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
ISLPOSE_X3_PX64=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_body.py::test_canonical_ranges_batch_invariant" > $O/tests.log 2>&1 || exit 1
for p in 2 3; do
  ISLPOSE_X3_PX64=$p timeout -k 10 120 python -u tools/op_table.py --batch 1 --h 184 --w 328 --runs 20 > $O/ops_b1_p$p.txt 2>&1 || exit 1
done
for i in 1 2; do for p in 2 3; do
  ISLPOSE_X3_PX64=$p timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/p${p}_$i.json 2>> $O/err.log || exit 1
done; done
grep -h "net " $O/ops_b1_*.txt
python3 - "$O" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/p*.json')):
    d = json.load(open(f))
    print(f, 'N', d['value'], 'R32', d['mode_r']['batch32']['frames_per_s'], 'R1', d['mode_r']['batch1']['frames_per_s'])
PY
