"""The four hand scales side by side, timed with HIP events on their own streams (no profiler:
rocprofv3's per-dispatch interception delays each stream's enqueue by ~1 ms and hides the
overlap).  Prints each scale's start / end relative to the fork, graph replay on."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "isl-signlanguage-translation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from islpose import runtime as rt, synth  # noqa: E402
from islpose.hand import HandEstimator, BOXSIZE  # noqa: E402


def main():
    frames = torch.from_numpy(np.ascontiguousarray(synth.synth_frames(1, 1080, 1920, seed=5))).cuda()
    hand = HandEstimator(synth.synth_weights(2))
    hand.net.set_graph(os.environ.get("GRAPH", "1") == "1")
    order = [int(c) for c in os.environ.get("ORDER", "0123")]
    crops = [(0, 700, 100, 640, 640)]
    pre = os.environ.get("PRE", "")
    if "h" in pre:     # a hand post first (its C++ lane streams)
        hand.post_crops([(0, 700, 100, 640)], hand.run_crops(frames, [(0, 700, 100, 640)]))
    if "b" in pre:     # a body estimate first (its net, graph capture stream, post)
        from islpose.body import BodyEstimator
        body = BodyEstimator(synth.synth_weights(0), "body25", scale_search=(0.5,))
        body.net.set_graph(True)
        for _ in range(3):
            body.estimate(frames)
    cur = torch.cuda.current_stream()
    # LANES: the lane (stream) of each scale, e.g. "0122": 184 px on lane 0, 368 on 1, 552 and
    # 736 on lane 2 (in scale order); default one lane per scale
    lanes = [int(c) for c in os.environ.get("LANES", "0123")]
    pool = rt.scale_streams(hand, frames.device, max(lanes) + 1)
    streams = [pool[k] for k in lanes]
    res = []
    for it in range(12):
        t0 = torch.cuda.Event(enable_timing=True)
        t0.record(cur)
        rt.fork_streams(cur, streams)
        ev = {}
        for k in order:
            st, s = streams[k], hand.scale_search[k]
            with torch.cuda.stream(st):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                gh, gw = hand.net.preprocess_crops(frames, crops, s * BOXSIZE)
                heat = torch.empty((1, 22, gh // 8, gw // 8), device="cuda")
                hand.net.run(heat)
                b.record(st)
                ev[k] = (a, b)
        rt.join_streams(cur, streams)
        t1 = torch.cuda.Event(enable_timing=True)
        t1.record(cur)
        torch.cuda.synchronize()
        if it >= 4:
            res.append([t0.elapsed_time(t1)] + [x for k in range(4) for x in (t0.elapsed_time(ev[k][0]), t0.elapsed_time(ev[k][1]))])
    r = np.median(np.array(res), axis=0)
    print("pre %s lanes %s order %s graph %s  total %.3f ms  " % (pre, os.environ.get("LANES", "0123"), os.environ.get("ORDER", "0123"), os.environ.get("GRAPH", "1"), r[0]) +
          "  ".join("s%d %.2f-%.2f" % (k, r[1 + 2 * k], r[2 + 2 * k]) for k in range(4)))


if __name__ == "__main__":
    main()
