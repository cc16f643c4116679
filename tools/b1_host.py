"""Batch-1 Mode R: is the GPU waiting for the host?  Times (a) the host-side enqueue of one
isl_net_forward (GPU idle before; the C call without Net.forward's synchronous range check),
(b) the GPU time of one forward (events), (c) back-to-back forwards per iteration.
usage: python tools/b1_host.py [--h 184 --w 328 --batch 1 --iters 200]"""
import argparse
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from islpose import runtime as rt, synth  # noqa: E402
from islpose.runtime import lib, ptr  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--h", type=int, default=184)
    p.add_argument("--w", type=int, default=328)
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--iters", type=int, default=200)
    a = p.parse_args()
    net = rt.Net(rt.ISL_BODY25)
    net.load_weights(synth.synth_weights(rt.ISL_BODY25))
    x = torch.from_numpy(np.random.RandomState(0).uniform(-0.5, 0.5, (a.batch, 3, a.h, a.w)).astype(np.float32)).cuda()
    o0 = torch.empty((a.batch, 52, a.h // 8, a.w // 8), device="cuda")
    o1 = torch.empty((a.batch, 26, a.h // 8, a.w // 8), device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def fwd():
        rc = lib().isl_net_forward(net.h, ptr(x), a.batch, a.h, a.w, ptr(o0), ptr(o1), s)
        assert rc == 0, rc

    for _ in range(10):
        fwd()
    torch.cuda.synchronize()
    host = []
    gpu = []
    for _ in range(50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        t0 = time.perf_counter()
        fwd()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        host.append((t1 - t0) * 1e3)
        gpu.append(e0.elapsed_time(e1))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        fwd()
    torch.cuda.synchronize()
    loop = (time.perf_counter() - t0) * 1e3 / a.iters
    print("host enqueue %.3f ms (median), GPU per forward %.3f ms (median, idle start), back-to-back %.3f ms/forward"
          % (np.median(host), np.median(gpu), loop))


if __name__ == "__main__":
    main()
