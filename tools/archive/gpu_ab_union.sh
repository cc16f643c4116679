# A/B of the union-path variants per layer shape (ISLPOSE_X3_UNION=1 old loop,
# 2 role-split loop + LDS epilogue, 4 = 2 with s_memtime stamps), parity with mode 2, bench A/B.
# usage: bash tools/archive/gpu_ab_union.sh <tag> [bench]
export TMPDIR=/tmp
T=${1:-ab}; O=gpurun_out/$T; mkdir -p $O
CB=tools/convbench
for s in "3 128 128 46 82 32" "3 384 128 46 82 32" "3 96 96 46 82 32" "3 288 96 46 82 32" "3 512 512 46 82 32" \
         "3 256 256 92 164 32" "3 128 256 92 164 32"; do
  for u in ${MODES:-1 2}; do
    echo "== $s union=$u" >> $O/u.txt
    ISLPOSE_X3_UNION=$u timeout -k 10 120 $CB $s 20 x3 3 >> $O/u.txt 2>&1 || { echo "convbench failed: $s"; tail $O/u.txt; exit 1; }
  done
done
for s in "3 128 128 46 82 32" "3 384 128 46 82 32"; do
  echo "== $s union=4" >> $O/u.txt
  ISLPOSE_X3_UNION=4 timeout -k 10 120 $CB $s 10 x3 2 >> $O/u.txt 2>&1 || { echo "convbench failed: $s"; tail $O/u.txt; exit 1; }
done
grep -E "==|round 2|stamps" $O/u.txt
ISLPOSE_X3_UNION=${PMODE:-2} timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py -m gpu -x -q --timeout 300 --timeout-method thread -k "forward or golden or estimate" > $O/parity.log 2>&1 || { echo parity failed; tail -20 $O/parity.log; exit 1; }
tail -2 $O/parity.log
[ "$2" = "bench" ] || exit 0
for i in 1 2; do
  for u in ${BMODES:-1 2}; do
    ISLPOSE_X3_UNION=$u timeout -k 10 300 python bench.py --no-cpu --e2e-steps 0 > $O/bench_u$u.$i.json 2>> $O/bench.err || exit 1
    python -c "import json;d=json.load(open('$O/bench_u$u.$i.json'));print('union=$u', d['value'], d['roofline']['frac'])"
  done
done
