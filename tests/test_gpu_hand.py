"""Hand path on the GPU: post-processing bit-exact vs the reference goldens and the
oracle, and the full crop -> peaks pipeline vs the oracle post on the GPU's maps."""
import os

import numpy as np
import pytest
import torch

from oracle import cpu_ref
from islpose import synth
from islpose.body import scale_geometry
from islpose.hand import HandEstimator, HAND_SCALES

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def hest():
    return HandEstimator(synth.synth_weights(2))


def test_hand_post_golden(hest):
    z = np.load(os.path.join(GOLDEN, "g4_hand_post.npz"))
    for c in sorted({k.split("/")[0] for k in z.files}):
        crop = int(z[c + "/crop"])
        geoms = [g[1:] for g in scale_geometry(crop, crop, HAND_SCALES)]
        heats = [torch.from_numpy(z[c + "/heat%d" % i][None]).cuda() for i in range(4)]
        peaks = hest.post_maps(crop, crop, geoms, heats)[0]
        assert np.array_equal(peaks, z[c + "/peaks"]), c


@pytest.mark.parametrize("h,w", [(64, 64), (150, 150), (90, 120)])
def test_hand_post_designed_batch(hest, h, w):
    n = 3
    geoms = [g[1:] for g in scale_geometry(h, w, HAND_SCALES)]
    heats, per = [], []
    for (nh, nw, vh, vw) in geoms:
        maps = [synth.designed_hand_maps(nh // 8, nw // 8, seed=7 * i + nh, n_blobs=3) for i in range(n)]
        per.append(maps)
        heats.append(torch.from_numpy(np.stack(maps)).cuda())
    got = hest.post_maps(h, w, geoms, heats)
    for i in range(n):
        it = iter([per[s][i] for s in range(4)])
        ref = cpu_ref.hand_call(np.zeros((h, w, 3), np.uint8), lambda im: next(it)[None])
        assert np.array_equal(got[i], ref), i


def test_hand_estimate_end_to_end(hest):
    crops = synth.synth_frames(2, 96, 96, seed=11)
    t = torch.from_numpy(crops).cuda()
    geoms, heats = hest.run_scales(t)
    got = hest.post_maps(96, 96, geoms, heats)
    for i in range(2):
        maps = iter([h[i].cpu().numpy() for h in heats])
        ref = cpu_ref.hand_call(crops[i], lambda im: next(maps)[None])
        assert np.array_equal(got[i], ref)
    assert np.array_equal(hest.estimate(crops[0]), got[0])
