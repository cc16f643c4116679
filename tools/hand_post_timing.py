"""Hand post (isl_hand_post) alone, per crop side and map kind: designed blobs
(trained-net-like) vs dense random maps (random-weight nets: giant components).
Prints ms per call from HIP events; run under rocprofv3 --kernel-trace --stats for
the per-kernel split.   usage: python3 tools/hand_post_timing.py [sides...]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from islpose import synth  # noqa: E402
from islpose.body import scale_geometry  # noqa: E402
from islpose.hand import HandEstimator, HAND_SCALES  # noqa: E402


def main():
    sides = [int(v) for v in sys.argv[1:]] or [150, 300, 600]
    hest = HandEstimator(synth.synth_weights(2))
    rng = np.random.RandomState(0)
    for side in sides:
        geoms = [g[1:] for g in scale_geometry(side, side, HAND_SCALES)]
        for kind in ("designed", "dense"):
            heats = []
            for (nh, nw, vh, vw) in geoms:
                if kind == "dense":
                    m = rng.uniform(0.02, 1.0, (1, 22, nh // 8, nw // 8)).astype(np.float32)
                else:
                    m = synth.designed_hand_maps(nh // 8, nw // 8, seed=nh, n_blobs=3)[None]
                heats.append(torch.from_numpy(m).cuda())
            hest.post_maps(side, side, geoms, heats)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                hest.post_maps(side, side, geoms, heats)
            torch.cuda.synchronize()
            print("side %d %-8s %.2f ms per crop" % (side, kind, (time.perf_counter() - t0) / 5 * 1e3), flush=True)


if __name__ == "__main__":
    main()
