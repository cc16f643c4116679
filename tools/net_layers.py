"""Per-layer-shape conv times of one network from the engine's own HIP events
(isl_net_set_timing), for any kind and input size: the hand net at its four crop
scales, COCO, or body_25 at a given batch.

  python3 tools/net_layers.py hand 32 184 368 552 736      (batch, then sides)
  python3 tools/net_layers.py body25 32 368x656
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))

import torch  # noqa: E402

from islpose import netspec, synth  # noqa: E402
from islpose import runtime as rt  # noqa: E402

KINDS = {"body25": (rt.ISL_BODY25, 0), "coco": (rt.ISL_COCO, 1), "hand": (rt.ISL_HAND, 2)}   # (runtime, netspec)


def layer_table(kind_name, n, h, w, runs=3):
    kind, spec = KINDS[kind_name]
    net = rt.Net(kind)
    net.load_weights(synth.synth_weights(spec))
    x = torch.rand(n, 3, h, w, device="cuda") - 0.5
    net.forward(x)
    torch.cuda.synchronize()
    net.set_timing(True)
    for _ in range(runs):
        net.forward(x)
    torch.cuda.synchronize()
    t = net.timing()
    net.set_timing(False)
    convs = netspec.convs_for(spec)
    groups, ci, H, W, tot = {}, 0, h, w, 0.0
    for ms, k, fl in zip(t["ms"], t["kind"], t["flops"]):
        ms /= max(t["n_runs"], 1)
        tot += ms
        if k == 0:
            key = "maxpool"
            g = groups.setdefault(key, [0, 0.0, 0.0])
            g[0] += 1
            g[1] += ms
            continue
        c = convs[ci]
        key = "%dx%d c%d->%d k%d" % (H, W, c.cin, c.cout, c.k)
        g = groups.setdefault(key, [0, 0.0, 0.0])
        g[0] += 1
        g[1] += ms
        g[2] += 2.0 * c.cout * c.cin * c.k * c.k * H * W * n
        if c.name in ("conv1_2", "conv2_2", "conv3_4"):
            H, W = H // 2, W // 2
        ci += 1
    rows = []
    for key, (cnt, ms, fl) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        rows.append({"layer": key, "count": cnt, "ms": round(ms, 4), "share": round(ms / tot, 4),
                     "tflops_fp32_eq": round(fl / (ms * 1e-3) / 1e12, 1) if fl else None})
    return {"net": kind_name, "batch": n, "hw": [h, w], "net_ms": round(tot, 3), "layers": rows}


def main():
    kind_name, n = sys.argv[1], int(sys.argv[2])
    for s in sys.argv[3:]:
        h, w = (int(v) for v in s.split("x")) if "x" in s else (int(s), int(s))
        r = layer_table(kind_name, n, h, w)
        print("== %s batch %d %dx%d: %.3f ms" % (kind_name, n, h, w, r["net_ms"]))
        for L in r["layers"]:
            print("  %-28s x%-3d %9.3f ms %5.1f%%  %s" % (L["layer"], L["count"], L["ms"], 100 * L["share"],
                                                        "%.1f TF" % L["tflops_fp32_eq"] if L["tflops_fp32_eq"] else ""))
        print(json.dumps(r), file=sys.stderr)


if __name__ == "__main__":
    main()
