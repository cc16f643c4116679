"""The blur + NMS fp32 filter (blur_tile in csrc/post.hip; body.py:86-100, hand.py:58-62): the
packed-fp32 passes decide every pixel whose comparisons clear the error margin and hand the
rest of the tile to the fp64 passes, so the masks -- hence the peak lists -- equal the fp64
passes' (ISLPOSE_BLUR_EXACT=1), the forced fallback's (=2: nearly every live tile re-run in
fp64 after the filter wrote its words) and the oracle's, bit for bit.  Maps: noise around the
thresholds and exact plateaus (ties: the fallback), on the Mode N fused path, the Mode R
materialised planes, the multi-scale fp64 average and the hand planes.  GPU only."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref
from islpose import synth
from islpose.body import BodyEstimator, scale_geometry
from islpose.hand import HandEstimator, HAND_SCALES

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def est25():
    return BodyEstimator(synth.synth_weights(0), "body25")


def _heat(nh, nw, seed, kind):
    """Designed 2-person maps plus noise around 0.1 (kind "noise") or, in parts 0, 4 and 9,
    a 6 x 6 low-resolution plateau of 0.6 whose full-resolution interior blurs to exactly
    equal values (kind "plateau": tied neighbours, every such pixel a peak)."""
    rng = np.random.RandomState(seed)
    pl, hl = synth.designed_pose_maps(nh, nw, 2, seed)
    if kind == "noise":
        hl = hl + (rng.uniform(0.0, 0.16, hl.shape) * (rng.rand(*hl.shape) < 0.15)).astype(np.float32)
    else:
        for k, part in enumerate((0, 4, 9)):
            y, x = 1 + (k * 5) % max(nh - 7, 1), 1 + (k * 11) % max(nw - 7, 1)
            hl[part, y:y + 6, x:x + 6] = np.float32(0.6)
    return pl, hl


def _post(est, H, W, geoms, pafs, heats, monkeypatch, mode):
    if mode is None:
        monkeypatch.delenv("ISLPOSE_BLUR_EXACT", raising=False)
    else:
        monkeypatch.setenv("ISLPOSE_BLUR_EXACT", mode)
    return est.post_maps(H, W, geoms, pafs, heats)


@pytest.mark.parametrize("kind", ["noise", "plateau"])
@pytest.mark.parametrize("H,W,scales", [(368, 656, (1.0,)), (368, 656, (0.5,)), (240, 328, (0.5, 1.0)),
                                        (368, 131, (1.0,))])
def test_body_filter_matches_fp64_and_oracle(est25, monkeypatch, H, W, scales, kind):
    """Body planes: single scale fused (1.0) and materialised (0.5), two scales (the fp64
    average), a narrow frame; two frames each, frame 0 against the oracle."""
    geoms = [g[1:] for g in scale_geometry(H, W, scales)]
    per = [[_heat(g[0] // 8, g[1] // 8, 17 * i + si, kind) for i in range(2)] for si, g in enumerate(geoms)]
    pafs = [torch.from_numpy(np.stack([m[0] for m in ms])).cuda() for ms in per]
    heats = [torch.from_numpy(np.stack([m[1] for m in ms])).cuda() for ms in per]
    got = _post(est25, H, W, geoms, pafs, heats, monkeypatch, None)
    for mode in ("1", "2"):
        ref = _post(est25, H, W, geoms, pafs, heats, monkeypatch, mode)
        for a, b in zip(got, ref):
            assert np.array_equal(a.candidate, b.candidate) and np.array_equal(a.subset, b.subset), mode
    it = iter([(ms[0][0][None], ms[0][1][None]) for ms in per])
    heat_avg, paf_avg = cpu_ref.body_maps(np.zeros((H, W, 3), np.uint8), lambda im: next(it), "body25", scales)
    cand, subset, _, _ = cpu_ref.body_post(heat_avg, paf_avg, "body25", H)
    assert np.array_equal(got[0].candidate, cand) and np.array_equal(got[0].subset, subset)
    assert len(cand) > 0


@pytest.mark.parametrize("kind", ["noise", "plateau"])
def test_hand_filter_matches_fp64_and_oracle(monkeypatch, kind):
    """Hand planes (the fp64 average of four scales, the 0.05 binary map)."""
    hest = HandEstimator(synth.synth_weights(2))
    h = w = 184
    geoms = [g[1:] for g in scale_geometry(h, w, HAND_SCALES)]
    rng = np.random.RandomState(5)
    heats, per = [], []
    for (nh, nw, _, _) in geoms:
        m = synth.designed_hand_maps(nh // 8, nw // 8, seed=nh, n_blobs=3)
        if kind == "noise":
            m = m + (rng.uniform(0.0, 0.08, m.shape) * (rng.rand(*m.shape) < 0.15)).astype(np.float32)
        else:
            m[3, 2:8, 2:8] = np.float32(0.3)
        per.append(m)
        heats.append(torch.from_numpy(m[None]).cuda())
    monkeypatch.delenv("ISLPOSE_BLUR_EXACT", raising=False)
    got = hest.post_maps(h, w, geoms, heats)[0]
    for mode in ("1", "2"):
        monkeypatch.setenv("ISLPOSE_BLUR_EXACT", mode)
        assert np.array_equal(hest.post_maps(h, w, geoms, heats)[0], got), mode
    it = iter(per)
    ref = cpu_ref.hand_call(np.zeros((h, w, 3), np.uint8), lambda im: next(it)[None])
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("H,W", [(368, 656), (400, 520), (1080, 1920)])
def test_stage2_skip_matches_full_resize(est25, monkeypatch, H, W):
    """Mode R geometry (scale 0.5: stage 1 to the net's valid crop, stage 2 to the frame): the
    stage-2 resize tiles that no live blur window can read are skipped (stage2_need_kernel, from
    the stage-1 band maxima) -- the same peaks and persons as resizing every tile
    (ISLPOSE_RESIZE_SKIP=0) and as the oracle, on noisy maps around the threshold, batch 3."""
    geoms = [g[1:] for g in scale_geometry(H, W, (0.5,))]
    ms = [_heat(geoms[0][0] // 8, geoms[0][1] // 8, 50 + i, "noise" if i != 1 else "plateau") for i in range(3)]
    pafs = [torch.from_numpy(np.stack([m[0] for m in ms])).cuda()]
    heats = [torch.from_numpy(np.stack([m[1] for m in ms])).cuda()]
    monkeypatch.delenv("ISLPOSE_RESIZE_SKIP", raising=False)
    got = est25.post_maps(H, W, geoms, pafs, heats)
    monkeypatch.setenv("ISLPOSE_RESIZE_SKIP", "0")
    ref = est25.post_maps(H, W, geoms, pafs, heats)
    for a, b in zip(got, ref):
        assert np.array_equal(a.candidate, b.candidate) and np.array_equal(a.subset, b.subset)
    heat_avg, paf_avg = cpu_ref.body_maps(np.zeros((H, W, 3), np.uint8), lambda im: (ms[0][0][None], ms[0][1][None]),
                                          "body25", (0.5,))
    cand, subset, _, _ = cpu_ref.body_post(heat_avg, paf_avg, "body25", H)
    assert np.array_equal(got[0].candidate, cand) and np.array_equal(got[0].subset, subset) and len(cand) > 0
