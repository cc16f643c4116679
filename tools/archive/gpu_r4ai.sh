# Round 4: batch-1 Mode R op tables for the small-grid block forms, then the bench line A/B
# (interleaved, three times): default vs ISLPOSE_X3_PX64=2 with ISLPOSE_X3_HALFSMALL=0/1/2.
T=${1:-r4ai}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for cfg in "0 0" "1 0" "2 0" "2 1" "2 2"; do
  set -- $cfg
  ISLPOSE_X3_PX64=$1 ISLPOSE_X3_HALFSMALL=$2 timeout -k 10 120 python -u tools/op_table.py --batch 1 --h 184 --w 328 --runs 20 > $O/ops_b1_p$1h$2.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  for cfg in "1 0" "2 0" "2 1" "2 2"; do
    set -- $cfg
    ISLPOSE_X3_PX64=$1 ISLPOSE_X3_HALFSMALL=$2 timeout -k 10 300 python -u bench.py --no-cpu --e2e-steps 0 > $O/p$1h$2_$i.json 2>> $O/err.log || exit 1
  done
done
grep -h "net " $O/ops_b1_*.txt
python3 - "$O" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/p*.json')):
    d = json.load(open(f))
    print(f, 'N', d['value'], 'R32', d['mode_r']['batch32']['frames_per_s'], 'R1', d['mode_r']['batch1']['frames_per_s'])
PY
