# Tail tiles (x3_tail_plan) vs one tiling (ISLPOSE_X3_TAIL=0): bits (body_25 Mode N batch 32, the
# hand net at its C3 scales, batch 32), Mode N op tables, the bench line and C3, interleaved.
# usage: bash tools/ab_tail.sh <tag>
export TMPDIR=/tmp
T=${1:-tail}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python3 - > $O/bits.txt 2>&1 <<'PY' || { cat $O/bits.txt; exit 1; }
import os, sys
sys.path.insert(0, "isl-signlanguage-translation_amd")
import numpy as np, torch
from islpose import runtime as rt, synth
ok = True
for kind, code, n, h, w in (("body25", rt.ISL_BODY25, 32, 368, 656), ("hand", rt.ISL_HAND, 32, 736, 736),
                            ("hand", rt.ISL_HAND, 32, 552, 552), ("hand", rt.ISL_HAND, 32, 368, 368)):
    net = rt.Net(code); net.load_weights(synth.synth_weights(code))
    x = torch.from_numpy(np.random.RandomState(h).uniform(-0.5, 0.5, (n, 3, h, w)).astype(np.float32)).cuda()
    outs = []
    for m in ("0", "1"):
        os.environ["ISLPOSE_X3_TAIL"] = m
        o = net.forward(x); o = o if isinstance(o, tuple) else (o,)
        torch.cuda.synchronize(); outs.append([t.clone() for t in o])
    eq = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    ok &= eq
    print(kind, h, w, "equal", eq, flush=True)
    del net, x, outs
print("ALL_EQUAL", ok)
PY
cat $O/bits.txt
grep -q "ALL_EQUAL True" $O/bits.txt || exit 1
for m in 0 1 0b 1b; do
  ISLPOSE_X3_TAIL=${m:0:1} timeout -k 10 200 python3 tools/op_table.py --batch 32 --runs 5 > $O/ops_N_$m.txt 2>&1 || exit 1
  grep -m1 "net" $O/ops_N_$m.txt | sed "s/^/$m /"
done
bash tools/ab_bench.sh $T off:ISLPOSE_X3_TAIL=0 on:ISLPOSE_X3_TAIL=1 offb:ISLPOSE_X3_TAIL=0 onb:ISLPOSE_X3_TAIL=1 offc:ISLPOSE_X3_TAIL=0 onc:ISLPOSE_X3_TAIL=1 || exit 1
for m in 0 1; do
  ISLPOSE_X3_TAIL=$m timeout -k 10 300 python3 tools/bench_configs.py --config c3 --steps 5 > $O/c3_$m.json 2> $O/c3_$m.err || exit 1
  python3 -c "import json; print('c3 tail=$m', json.load(open('$O/c3_$m.json'))['frames_per_s'])"
done
