"""A/B of the blur's band-maxima early out (ISLPOSE_BLUR_BANDS=0|1; round 4 also used it for the
resize variants, profiles/r04/r4d/resize_ab.json) on the Mode R post (scale 0.5: the two-stage resizes), batch 32 and batch 1, designed maps:
HIP-event time per post call, and the records equal across variants (dev tool)."""
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
    H, W = 368, 656
    est = BodyEstimator(synth.synth_weights(0), "body25")
    geoms = [g[1:] for g in scale_geometry(H, W, (0.5,))]
    nh, nw = geoms[0][0] // 8, geoms[0][1] // 8
    out = {}
    for B in (32, 1):
        des = [synth.designed_pose_maps(nh, nw, 3, seed=i) for i in range(B)]
        paf = torch.from_numpy(np.stack([a for a, _ in des])).cuda()
        heat = torch.from_numpy(np.stack([b for _, b in des])).cuda()
        ref = None
        for rounds in range(4):
            for v in ("B1", "B0"):
                os.environ["ISLPOSE_BLUR_BANDS"] = v[1]
                res = est.post_maps(H, W, geoms, [paf], [heat])
                if ref is None:
                    ref = res
                for a, b in zip(res, ref):
                    assert np.array_equal(a.candidate, b.candidate) and np.array_equal(a.subset, b.subset), v
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    est.post(B, H, W, geoms, [paf], [heat])
                e1.record()
                torch.cuda.synchronize()
                out.setdefault("b%d_%s_ms" % (B, v), []).append(round(e0.elapsed_time(e1) / 10, 4))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
