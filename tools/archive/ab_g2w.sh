# Two K groups of 4 waves of 64co x 64px (ISLPOSE_X3_G2W=1) vs 8 waves of 64co x 32px: bits
# (Mode R batch 32 forward equal), op tables, bench.  usage: bash tools/ab_g2w.sh <tag>
export TMPDIR=/tmp
T=${1:-g2w}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 200 python3 - > $O/bits.txt 2>&1 <<'PY' || exit 1
import os, sys
sys.path.insert(0, "isl-signlanguage-translation_amd")
import numpy as np, torch
from islpose import runtime as rt, synth
net = rt.Net(rt.ISL_BODY25); net.load_weights(synth.synth_weights(0))
x = torch.from_numpy(np.random.RandomState(1).uniform(-0.5, 0.5, (32, 3, 184, 328)).astype(np.float32)).cuda()
outs = []
for m in ("0", "1"):
    os.environ["ISLPOSE_X3_G2W"] = m
    p, h = net.forward(x); torch.cuda.synchronize(); outs.append((p.clone(), h.clone()))
    print(m, sum(1 for _, v in net.op_variants() if rt.decode_variant(v).get("g2")))
print("equal", all(torch.equal(a, b) for a, b in zip(outs[0], outs[1])))
PY
cat $O/bits.txt
for m in 0 1 0b 1b; do
  ISLPOSE_X3_G2W=${m:0:1} timeout -k 10 200 python3 tools/op_table.py --batch 32 --h 184 --w 328 --runs 5 > $O/ops_R32_$m.txt 2>&1 || exit 1
  grep -m1 "net" $O/ops_R32_$m.txt | sed "s/^/$m /"
done
bash tools/ab_bench.sh $T off:ISLPOSE_X3_G2W=0 on:ISLPOSE_X3_G2W=1
