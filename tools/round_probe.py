"""Probe: per-layer time of the body net at several batch sizes (HIP events per op), to see
whether a layer's time follows its rounds of one block per CU or its block count.
usage: python tools/round_probe.py [--batches 24,26,28,30,32] [--layers conv3_2,conv2_2]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from islpose import runtime as rt, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="24,26,28,30,32")
    ap.add_argument("--layers", default="conv3_2,conv3_3,conv2_2,conv4_2,Mconv1_stage1_L2_1")
    ap.add_argument("--h", type=int, default=368)
    ap.add_argument("--w", type=int, default=656)
    a = ap.parse_args()
    net = rt.Net(rt.ISL_BODY25)
    net.load_weights(synth.synth_weights(0))
    names = a.layers.split(",")
    for b in [int(x) for x in a.batches.split(",")]:
        x = torch.from_numpy(np.random.RandomState(0).uniform(-0.5, 0.5, (b, 3, a.h, a.w)).astype(np.float32)).cuda()
        for _ in range(2):
            net.forward(x)
        torch.cuda.synchronize()
        net.set_timing(True)
        for _ in range(5):
            net.forward(x)
        torch.cuda.synchronize()
        net.set_timing(False)
        t = net.timing()
        runs = max(1, t["n_runs"])
        ops = [n for n, _ in net.op_variants()]
        row = []
        for nm in names:
            k = ops.index(nm)
            row.append("%s %.1f us" % (nm, float(t["ms"][k]) / runs * 1e3))
        print("batch %d: %s" % (b, ", ".join(row)), flush=True)
        del x


if __name__ == "__main__":
    main()
