"""Where the C5 overlapped pipeline's wall time goes, per thread: wraps the host-side
phases (prefetch copy into pinned memory, frame H2D enqueue, preprocess, net runs, the
body / hand posts with their result copies, record decode, handDetect, JSON writing)
with wall-clock spans and prints the totals per (thread, phase) over one timed pass.

  python3 tools/c5_timeline.py [frames_per_video] [videos] [batch]
"""
import collections
import functools
import os
import shutil
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

SPANS = collections.defaultdict(float)
COUNT = collections.defaultdict(int)
ON = [False]


def wrap(obj, name, label):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            if ON[0]:
                key = (threading.current_thread().name, label)
                SPANS[key] += time.perf_counter() - t
                COUNT[key] += 1
    setattr(obj, name, g)


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    V = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    from islpose import pipeline, synth, runtime as rt
    from islpose import body as ibody, hand as ihand
    from islpose.body import BodyEstimator
    from src import util
    from src.body import Body
    from src.hand import Hand
    from src.ISL_Model_parameter import ISLSignPos
    rgb = synth.synth_frames(T, 1080, 1920, seed=57)
    wb = synth.synth_weights(0)
    cal = BodyEstimator(wb, "body25", scale_search=(0.5,))
    _, _, heats = cal.run_scales(torch.from_numpy(np.ascontiguousarray(rgb[:1, ..., ::-1])).cuda(), keep_maps=True)
    wb = synth.tame_heat_layer(wb, heats[0].cpu().numpy(), "body25", gain=0.05)
    del cal
    tw = lambda d: {k: torch.from_numpy(v) for k, v in d.items()}  # noqa: E731
    isl = ISLSignPos(Body(tw(wb), "body25").model, Hand(tw(synth.synth_weights(2))).model)
    clips = {"v%d.mp4" % k: rgb for k in range(V)}
    rows = [{"Filepath": f, "type": "Greetings", "expression": "hello"} for f in clips]

    wrap(np, "copyto", "prefetch: copy into pinned")
    wrap(rt.Net, "preprocess", "preprocess (body)")
    wrap(rt.Net, "preprocess_crops", "preprocess_crops (hand)")
    wrap(rt.Net, "run", "net run enqueue")
    wrap(ibody.BodyEstimator, "post", "body post + result copy")
    wrap(ibody.BodyEstimator, "decode", "body record decode")
    wrap(ihand.HandEstimator, "post_crops", "hand post + result copy")
    wrap(util, "handDetect", "handDetect")
    wrap(pipeline.KeypointExtractor, "_write", "writer: JSON + rows")
    wrap(ISLSignPos, "call_batch", "call_batch (total)")

    out = tempfile.mkdtemp(prefix="c5t_")
    try:
        pipeline.extract_dataset(rows[:1], clips.__getitem__, isl, out, batch=B, export=False, overlap=True)
        shutil.rmtree(out)
        torch.cuda.synchronize()
        ON[0] = True
        t0 = time.perf_counter()
        feats, ex = pipeline.extract_dataset(rows, clips.__getitem__, isl, out, batch=B, export=False, overlap=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ON[0] = False
    finally:
        shutil.rmtree(out, ignore_errors=True)
    print("frames %d in %.3f s: %.1f frames/s" % (ex.frames_done, dt, ex.frames_done / dt))
    for (th, lab), s in sorted(SPANS.items(), key=lambda kv: (kv[0][0], -kv[1])):
        print("  %-12s %-30s x%-4d %8.1f ms  (%4.1f%% of wall)" % (th[:12], lab, COUNT[(th, lab)], s * 1e3,
                                                                100 * s / dt))


if __name__ == "__main__":
    main()
