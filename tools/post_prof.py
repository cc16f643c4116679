"""Mode R post alone (scale 0.5, 368x656 frames, designed 3-person maps) for kernel traces and
counter passes: `python tools/post_prof.py [--batch 32] [--iters 10]` (dev tool; the
switches of the run come from the environment)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from islpose import synth  # noqa: E402
from islpose.body import BodyEstimator, scale_geometry  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--scale", type=float, default=0.5)
    a = ap.parse_args()
    H, W, B = 368, 656, a.batch
    est = BodyEstimator(synth.synth_weights(0), "body25")
    geoms = [g[1:] for g in scale_geometry(H, W, (a.scale,))]
    nh, nw = geoms[0][0] // 8, geoms[0][1] // 8
    des = [synth.designed_pose_maps(nh, nw, 3, seed=i) for i in range(B)]
    paf = torch.from_numpy(np.stack([p for p, _ in des])).cuda()
    heat = torch.from_numpy(np.stack([h for _, h in des])).cuda()
    res = est.post_maps(H, W, geoms, [paf], [heat])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        est.post(B, H, W, geoms, [paf], [heat])
    e1.record()
    torch.cuda.synchronize()
    print("post_ms %.4f peaks %d" % (e0.elapsed_time(e1) / a.iters, sum(len(r.candidate) for r in res)))


if __name__ == "__main__":
    main()
