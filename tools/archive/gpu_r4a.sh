# Round 4: the fused Mconv6 -> Mconv7 pair -- its parity tests, per-op tables fused vs two
# launches (Mode N batch 32, Mode R batch 32 / 1), then the bench line.
T=${1:-r4a}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_body.py -x -v --timeout 300 --timeout-method thread \
  -k "fused or timed_config or canonical or halfco or graph" > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for F in 1 0; do
  ISLPOSE_X3_FUSE67=$F timeout -k 10 200 python -u tools/op_table.py --batch 32 > $O/ops_N_b32_f$F.txt 2>&1 &&
  ISLPOSE_X3_FUSE67=$F timeout -k 10 200 python -u tools/op_table.py --batch 32 --h 184 --w 328 > $O/ops_R_b32_f$F.txt 2>&1 &&
  ISLPOSE_X3_FUSE67=$F timeout -k 10 200 python -u tools/op_table.py --batch 1 --h 184 --w 328 --runs 20 > $O/ops_R_b1_f$F.txt 2>&1 || exit 1
done
grep -h "Mconv6\|Mconv7\|convs:" $O/ops_*.txt
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err
rb=$?
python3 -c "
import json
d=json.load(open('$O/bench.json'))
print('N', d['value'], d['roofline']['frac'], 'R32', d['mode_r']['batch32']['frames_per_s'], d['mode_r']['batch32']['roofline']['frac'], d['mode_r']['batch32']['post_ms_per_step'], 'R1', d['mode_r']['batch1']['frames_per_s'])
"
exit $rb
