# A/B of library variants built into build_ab/libislpose_<v>.so (VARIANTS="..."; first used for the x3 input split: base / pk / sub),
# sub: packed converts + scalar subs), interleaved on one box: Mode N bench x3 rounds each.
export TMPDIR=/tmp
VARIANTS=${VARIANTS:-base pk sub}
O=gpurun_out/${1:-split_ab}; mkdir -p $O
for v in $VARIANTS; do
  ISLPOSE_LIB=build_ab/libislpose_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_body.py -m gpu -q --timeout 200 -k "forward or ranges or fused_pool" > $O/t_$v.log 2>&1 || { tail -5 $O/t_$v.log; exit 1; }
  tail -1 $O/t_$v.log
done
for r in 1 2 3; do for v in $VARIANTS; do
  ISLPOSE_LIB=build_ab/libislpose_$v.so timeout -k 10 300 python3 -u bench.py --no-cpu --e2e-steps 0 --steps 20 > $O/b_$v.$r.json 2>> $O/err || exit 1
done; done
python3 - <<PY
import json,glob,collections
d=collections.defaultdict(list)
for f in sorted(glob.glob('$O/b_*.json')):
    v=f.split('/b_')[1].split('.')[0]; j=json.load(open(f)); d[v].append((j['value'], j['roofline']['frac']))
for v,x in d.items(): print(v, x)
PY
