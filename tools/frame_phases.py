"""Host-side phases of the per-frame call (FRAME leg, ISLSignPos.call on 1080x1920 frames):
wall time of each step with a device synchronisation at its end, so the GPU work lands in the
phase that enqueued it.  usage: python tools/frame_phases.py [--frames N]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from islpose import synth  # noqa: E402
from islpose.body import BodyEstimator  # noqa: E402
from src import util  # noqa: E402
from src.body import Body  # noqa: E402
from src.hand import Hand  # noqa: E402
from src.ISL_Model_parameter import ISLSignPos  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    a = ap.parse_args()
    T, H, W = a.frames, 1080, 1920
    rgb = synth.synth_frames(T, H, W, seed=57)
    wb = synth.synth_weights(0)
    cal = BodyEstimator(wb, "body25", scale_search=(0.5,))
    _, _, heats = cal.run_scales(torch.from_numpy(np.ascontiguousarray(rgb[:1, ..., ::-1])).cuda(), keep_maps=True)
    wb = synth.tame_heat_layer(wb, heats[0].cpu().numpy(), "body25", gain=0.05)
    del cal
    tw = lambda d: {k: torch.from_numpy(v) for k, v in d.items()}  # noqa: E731
    isl = ISLSignPos(Body(tw(wb), "body25").model, Hand(tw(synth.synth_weights(2))).model)
    body, hand = isl._estimators()
    for i in range(min(5, T)):
        isl.call(rgb[i][:, :, ::-1])
    torch.cuda.synchronize()
    ph = {k: 0.0 for k in ("upload", "nets", "post+D2H", "range_check", "decode", "handDetect", "hands", "assemble")}

    def lap(k, t0):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ph[k] += t1 - t0
        return t1

    crops = 0
    t_all = time.perf_counter()
    for i in range(T):
        t = time.perf_counter()
        x = isl._upload(rgb[i][:, :, ::-1])
        t = lap("upload", t)
        n, fh, fw, _ = x.shape
        geoms, pafs, hts = body.run_scales(x)
        t = lap("nets", t)
        host, lay, caps = body.post(n, fh, fw, geoms, pafs, hts)
        t = lap("post+D2H", t)
        ok = body.net.range_ok()
        t = lap("range_check", t)
        assert ok
        (c, s), = [(r.candidate, r.subset) for r in body.decode(host, lay, caps, n, False)]
        t = lap("decode", t)
        boxes = [(0, bx, by, bw) for bx, by, bw, _l in util.handDetect(c, s, x[0])]
        t = lap("handDetect", t)
        peaks = hand.estimate_crops(x, boxes)
        crops += len(boxes)
        t = lap("hands", t)
        isl._assemble([(c, s)], boxes, peaks)
        lap("assemble", t)
    tot = time.perf_counter() - t_all
    print("frames %d  ms/frame %.3f  crops/frame %.2f" % (T, tot / T * 1e3, crops / T))
    for k, v in ph.items():
        print("  %-12s %7.3f ms" % (k, v / T * 1e3))
    hand_detail(isl, body, hand, rgb)


def hand_detail(isl, body, hand, rgb):
    """The hand phase of the frames with crops, split: the four scales' nets side by side
    (run_crops), each scale alone, the post + D2H; eager and graph replay."""
    from islpose.hand import BOXSIZE
    jobs = []
    for i in range(len(rgb)):
        x = isl._upload(rgb[i][:, :, ::-1])
        (c, s), = body.estimate(x)
        boxes = [(0, bx, by, bw) for bx, by, bw, _l in util.handDetect(c, s, x[0])]
        if boxes:
            jobs.append((x, boxes))
    if not jobs:
        return
    for graph in ("0", "1"):
        os.environ["ISLPOSE_NET_GRAPH"] = graph
        for x, boxes in jobs[:2]:                 # warm-up (graph capture)
            for _ in range(2):
                hand.post_crops(boxes, hand.run_crops(x, boxes))
        torch.cuda.synchronize()
        tn = tp = 0.0
        ta = [0.0] * len(hand.scale_search)
        for x, boxes in jobs:
            t0 = time.perf_counter()
            heats = hand.run_crops(x, boxes)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            hand.post_crops(boxes, heats)
            t2 = time.perf_counter()
            tn += t1 - t0
            tp += t2 - t1
            crops = [(f, bx, by, w, w) for (f, bx, by, w) in boxes]
            for k, sc in enumerate(hand.scale_search):
                t3 = time.perf_counter()
                gh, gw = hand.net.preprocess_crops(x, crops, sc * BOXSIZE)
                heat = torch.empty((len(crops), 22, gh // 8, gw // 8), device=x.device)
                hand.net.run(heat)
                torch.cuda.synchronize()
                ta[k] += time.perf_counter() - t3
        J = len(jobs)
        print("hand frames %d (graph=%s): nets side by side %.3f ms, post+D2H %.3f ms; alone %s (sum %.3f)" % (
            J, graph, tn / J * 1e3, tp / J * 1e3, " ".join("%.3f" % (v / J * 1e3) for v in ta), sum(ta) / J * 1e3))
    os.environ.pop("ISLPOSE_NET_GRAPH")


if __name__ == "__main__":
    main()
