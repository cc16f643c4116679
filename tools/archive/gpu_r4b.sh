# Round 4: fused Mconv6 -> Mconv7 + two K groups (VAR 32) -- parity tests, per-op tables
# (G2 on / off, fused on / off), then the bench line.
T=${1:-r4b}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_body.py tests/test_gpu_hand.py -x -v --timeout 300 --timeout-method thread \
  -k "fused or timed_config or canonical or halfco or graph or g2 or splitk or deep or c3" > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for V in "G2=1 FUSE67=1" "G2=0 FUSE67=1" "G2=1 FUSE67=0"; do
  set -- $V; tag=${1}_${2}
  env ISLPOSE_X3_$1 ISLPOSE_X3_$2 timeout -k 10 200 python -u tools/op_table.py --batch 32 --h 184 --w 328 > $O/ops_R_b32_$tag.txt 2>&1 || exit 1
done
ISLPOSE_X3_FUSE67=0 timeout -k 10 200 python -u tools/op_table.py --batch 32 > $O/ops_N_b32_FUSE0.txt 2>&1 &&
timeout -k 10 200 python -u tools/op_table.py --batch 32 > $O/ops_N_b32.txt 2>&1 &&
timeout -k 10 200 python -u tools/op_table.py --batch 1 --h 184 --w 328 --runs 20 > $O/ops_R_b1.txt 2>&1 || exit 1
head -12 $O/ops_R_b32_*.txt $O/ops_N_b32*.txt $O/ops_R_b1.txt
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err
rb=$?
[ $rb -eq 0 ] && ISLPOSE_X3_ACROSS=0 timeout -k 10 200 python -u bench.py --scale 0.5 --batch 1 --steps 50 --warmup 5 --no-cpu --e2e-steps 0 --no-mode-r > $O/b1_across0.json 2>> $O/bench.err
rb=$?
[ $rb -eq 0 ] && timeout -k 10 200 python -u bench.py --scale 0.5 --batch 1 --steps 50 --warmup 5 --no-cpu --e2e-steps 0 --no-mode-r > $O/b1_default.json 2>> $O/bench.err
rb=$?
[ $rb -eq 0 ] && ISLPOSE_X3_FUSE67=0 timeout -k 10 200 python -u bench.py --scale 0.5 --batch 1 --steps 50 --warmup 5 --no-cpu --e2e-steps 0 --no-mode-r > $O/b1_fuse0.json 2>> $O/bench.err
rb=$?
python3 -c "
import json
for f in ('b1_across0','b1_default','b1_fuse0'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['value'], d['roofline']['frac'])
"
python3 -c "
import json
d=json.load(open('$O/bench.json'))
print('N', d['value'], d['roofline']['frac'], 'R32', d['mode_r']['batch32']['frames_per_s'], d['mode_r']['batch32']['roofline']['frac'], d['mode_r']['batch32']['post_ms_per_step'], 'R1', d['mode_r']['batch1']['frames_per_s'])
"
exit $rb
