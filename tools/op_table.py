"""Per-op table of one net run from the library's own HIP events (isl_net_set_timing) and
the variant each conv ran (isl_net_op_info): ms, TF-eq (direct-conv FLOPs x 3 / time, the
split-fp16 MFMA work), fraction of the dense FP16 peak, and the kernel variant.

usage: python tools/op_table.py [--kind body25|coco|hand] [--batch N] [--h H] [--w W] [--runs R]
Groups layers of the same shape and variant; prints the per-group totals, largest first.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from islpose import runtime as rt, synth  # noqa: E402

PEAK = 2516.6


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kind", default="body25")
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--h", type=int, default=368)
    p.add_argument("--w", type=int, default=656)
    p.add_argument("--runs", type=int, default=5)
    p.add_argument("--json", default="")
    a = p.parse_args()
    kind = {"body25": rt.ISL_BODY25, "coco": rt.ISL_COCO, "hand": rt.ISL_HAND}[a.kind]
    w = synth.synth_weights(kind)
    net = rt.Net(kind)
    net.load_weights(w)
    x = torch.from_numpy(np.random.RandomState(0).uniform(-0.5, 0.5, (a.batch, 3, a.h, a.w)).astype(np.float32)).cuda()
    for _ in range(3):
        net.forward(x)
    torch.cuda.synchronize()
    net.set_timing(True)
    for _ in range(a.runs):
        net.forward(x)
    torch.cuda.synchronize()
    net.set_timing(False)
    t = net.timing()
    var = net.op_variants()
    runs = max(1, t["n_runs"])
    groups = {}
    rows = []
    tot = float(t["ms"].sum()) / runs
    for k, (name, v) in enumerate(var):
        ms = float(t["ms"][k]) / runs
        fl = float(t["flops"][k]) / runs
        d = rt.decode_variant(v)
        tag = "pool" if name == "maxpool2" else "var%d/%dpx/%dco/k%d" % (d.get("var", 0), d.get("bpx", 0),
                                                                         d.get("bco", 0), d.get("ks", 0))
        rows.append({"op": name, "ms": ms, "gflop": fl / 1e9, "variant": v, "tag": tag})
        key = (tag, round(fl / 1e9, 3))
        g = groups.setdefault(key, {"n": 0, "ms": 0.0, "fl": 0.0, "names": []})
        g["n"] += 1
        g["ms"] += ms
        g["fl"] += fl
        g["names"].append(name)
    print("batch %d  %dx%d  %s  net %.3f ms (HIP events, %d runs)" % (a.batch, a.h, a.w, a.kind, tot, runs))
    for (tag, _), g in sorted(groups.items(), key=lambda kv: -kv[1]["ms"]):
        tf = 3 * g["fl"] / (g["ms"] * 1e-3) / 1e12 if g["ms"] > 0 and g["fl"] > 0 else 0.0
        print("%-34s x%-3d %8.3f ms %5.1f%%  %7.1f TF-eq  frac %.3f  e.g. %s" % (
            tag, g["n"], g["ms"], 100 * g["ms"] / tot, tf, tf / PEAK, g["names"][0]))
    conv_ms = sum(r["ms"] for r in rows if r["gflop"] > 0)
    conv_fl = sum(r["gflop"] for r in rows)
    print("convs: %.3f ms, %.1f TF-eq, frac %.4f" % (conv_ms, 3 * conv_fl / conv_ms, 3 * conv_fl / conv_ms / PEAK))
    if a.json:
        json.dump({"batch": a.batch, "h": a.h, "w": a.w, "kind": a.kind, "net_ms": tot, "ops": rows}, open(a.json, "w"))


if __name__ == "__main__":
    main()
