# Round 4: fused pair forms (fused / permuted two launches) + G2 (128-channel only) -- parity
# tests, per-op tables (F67PPS A/B), batch-1 A/B, then the bench line.
T=${1:-r4c}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_body.py tests/test_gpu_hand.py -x -v --timeout 300 --timeout-method thread \
  -k "fused or timed_config or canonical or halfco or graph or g2 or splitk or deep or c3 or estimate_crops" > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for F in 0 1; do
  ISLPOSE_X3_F67PPS=$F timeout -k 10 200 python -u tools/op_table.py --batch 32 > $O/ops_N_b32_pps$F.txt 2>&1 &&
  ISLPOSE_X3_F67PPS=$F timeout -k 10 200 python -u tools/op_table.py --batch 32 --h 184 --w 328 > $O/ops_R_b32_pps$F.txt 2>&1 || exit 1
done
timeout -k 10 200 python -u tools/op_table.py --batch 1 --h 184 --w 328 --runs 20 > $O/ops_R_b1.txt 2>&1 || exit 1
grep -h "k1\|net " $O/ops_*.txt
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err
rb=$?
[ $rb -eq 0 ] && timeout -k 10 200 python -u bench.py --scale 0.5 --batch 1 --steps 50 --warmup 5 --no-cpu --e2e-steps 0 --no-mode-r > $O/b1_default.json 2>> $O/bench.err
rb=$?
python3 -c "
import json
d=json.load(open('$O/bench.json'))
print('N', d['value'], d['roofline']['frac'], 'post', d['post']['ms_per_step'], 'R32', d['mode_r']['batch32']['frames_per_s'], d['mode_r']['batch32']['roofline']['frac'], d['mode_r']['batch32']['post_ms_per_step'], 'R1', d['mode_r']['batch1']['frames_per_s'])
d=json.load(open('$O/b1_default.json')); print('b1 standalone', d['value'])
"
exit $rb
