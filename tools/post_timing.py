"""Kernel-time breakdown of the single-scale body post (dev tool).

Runs BodyEstimator.post on batch-32 low-res maps of three kinds -- all zero,
designed 3-person maps, dense noise -- with the fused resize+blur on and off
(ISLPOSE_FUSED_BLUR), and prints the average wall time of the post call with
HIP events (the post launches are on the current stream)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from islpose import synth  # noqa: E402
from islpose.body import BodyEstimator, scale_geometry  # noqa: E402


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 368          # frame size (e.g. 1080 1920)
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 656
    B = 32
    est = BodyEstimator(synth.synth_weights(0), "body25")
    geoms = [g[1:] for g in scale_geometry(H, W, (scale,))]
    nh, nw = geoms[0][0] // 8, geoms[0][1] // 8
    des = [synth.designed_pose_maps(nh, nw, 3, seed=i) for i in range(B)]
    paf = torch.from_numpy(np.stack([a for a, _ in des])).cuda()
    kinds = {
        "zero": torch.zeros(B, 26, nh, nw, device="cuda"),
        "designed": torch.from_numpy(np.stack([b for _, b in des])).cuda(),
        "dense": torch.from_numpy(np.random.RandomState(0).uniform(0, 0.12, (B, 26, nh, nw)).astype(np.float32)).cuda(),
    }
    out = {}
    for name, heat in kinds.items():
        for fused in ("1", "0"):
            os.environ["ISLPOSE_FUSED_BLUR"] = fused
            for _ in range(2):
                est.post(B, H, W, geoms, [paf], [heat])
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                est.post(B, H, W, geoms, [paf], [heat])
            e1.record()
            torch.cuda.synchronize()
            out["%s_fused%s_ms" % (name, fused)] = round(e0.elapsed_time(e1) / 5, 3)
    print(json.dumps(dict(out, scale=scale)))


if __name__ == "__main__":
    main()
