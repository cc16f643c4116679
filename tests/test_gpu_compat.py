"""Drop-in `src` package on the GPU: module seam, Body/Hand calls, ISLSignPos, pyramid."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref
from islpose import synth
from islpose.body import BodyEstimator, scale_geometry

pytestmark = pytest.mark.gpu


def _w(kind):
    return {k: torch.from_numpy(v) for k, v in synth.synth_weights(kind).items()}


@pytest.fixture(scope="module")
def body():
    from src.body import Body
    return Body(_w(0), "body25")


@pytest.fixture(scope="module")
def hand():
    from src.hand import Hand
    return Hand(_w(2))


def test_module_forward_cpu_and_cuda_inputs(body):
    x = np.ascontiguousarray(np.transpose(synth.synth_frames(1, 64, 80, seed=2).astype(np.float32),
                                          (0, 3, 1, 2)) / 256 - 0.5)
    paf_c, heat_c = body.model(torch.from_numpy(x))          # CPU in -> CPU out
    assert not paf_c.is_cuda and paf_c.shape == (1, 52, 8, 10)
    paf_g, heat_g = body.model(torch.from_numpy(x).cuda())
    assert paf_g.is_cuda and torch.equal(paf_g.cpu(), paf_c)
    rp, rh = cpu_ref.make_net_fn("body25", synth.synth_weights(0))(x)
    assert np.max(np.abs(heat_c.numpy() - rh)) / np.max(np.abs(rh)) < 1e-4


def test_body_call_types_and_equivalence(body):
    frame = synth.synth_frames(1, 240, 320, seed=4)[0]
    cand, subset = body(frame)
    assert cand.dtype == np.float64 and subset.dtype == np.float64
    assert subset.ndim == 2 and subset.shape[1] == 27
    assert cand.shape == (0,) or (cand.ndim == 2 and cand.shape[1] == 4)
    est = BodyEstimator(synth.synth_weights(0), "body25")
    c2, s2 = est.estimate(frame)
    assert np.array_equal(cand, c2) and np.array_equal(subset, s2)
    batch = body.estimate_batch(synth.synth_frames(3, 240, 320, seed=4))
    assert np.array_equal(batch[0][0], cand) and np.array_equal(batch[0][1], subset)


def test_pyramid_bit_exact_vs_oracle_post(body):
    """scale_search [0.5, 1, 1.5, 2] (the commented list of body.py:40): doubling quirk included."""
    scales = (0.5, 1.0, 1.5, 2.0)
    est = BodyEstimator(model_type="body25", scale_search=scales, net=body.model.native(0))
    H, W = 200, 256
    maps = [synth.designed_pose_maps(g[1] // 8, g[2] // 8, 2, seed=50 + i) for i, g in
            enumerate(scale_geometry(H, W, scales))]
    geoms = [g[1:] for g in scale_geometry(H, W, scales)]
    res = est.post_maps(H, W, geoms, [torch.from_numpy(m[0][None]).cuda() for m in maps],
                        [torch.from_numpy(m[1][None]).cuda() for m in maps])[0]
    it = iter(maps)
    cand, subset = cpu_ref.body_call(np.zeros((H, W, 3), np.uint8), lambda im: tuple(a[None] for a in next(it)),
                                     "body25", scales)
    assert np.array_equal(res.candidate, cand) and np.array_equal(res.subset, subset)


def test_hand_call(hand):
    crop = synth.synth_frames(1, 120, 120, seed=9)[0]
    peaks = hand(crop)
    assert peaks.dtype == np.int64 and peaks.shape == (21, 2)
    t = torch.from_numpy(crop[None]).cuda()
    est = hand.estimator()
    geoms, heats = est.run_scales(t)
    maps = iter([h[0].cpu().numpy() for h in heats])
    ref = cpu_ref.hand_call(crop, lambda im: next(maps)[None])
    assert np.array_equal(peaks, ref)


def test_isl_sign_pos_matches_composition(body, hand):
    from src.ISL_Model_parameter import ISLSignPos
    from src import util
    isl = ISLSignPos(body.model, hand.model)
    frame = synth.synth_frames(1, 368, 656, seed=12)[0]
    cand, subset, hands = isl.call(torch.from_numpy(frame))
    c2, s2 = body(frame)
    assert np.array_equal(cand, c2) and np.array_equal(subset, s2)
    boxes = util.handDetect(c2, s2, frame)
    assert len(hands) == len(boxes)
    for (x, y, w, _), pk in zip(boxes, hands):
        ref = hand(frame[y:y + w, x:x + w])
        ref[:, 0] = np.where(ref[:, 0] == 0, ref[:, 0], ref[:, 0] + x)
        ref[:, 1] = np.where(ref[:, 1] == 0, ref[:, 1], ref[:, 1] + y)
        assert np.array_equal(pk, ref)
    out = isl.call_batch(np.stack([frame, frame]))
    assert np.array_equal(out[1][0], cand) and len(out[1][2]) == len(hands)


def test_call_batches_pipelined_equals_call_batch(body, hand):
    """ISLSignPos.call_batches (the body of batch k on one stream beside the hands of
    batch k-1 on another) yields, in order, exactly what call_batch gives per batch:
    ragged batches, frames with and without hand crops."""
    from src.ISL_Model_parameter import ISLSignPos
    isl = ISLSignPos(body.model, hand.model)
    frames = synth.synth_frames(7, 240, 368, seed=21)
    sizes = [3, 1, 3]
    ref, batches, o = [], [], 0
    for k, n in enumerate(sizes):
        ref.append(isl.call_batch(frames[o:o + n]))
        batches.append((k, torch.from_numpy(frames[o:o + n]).cuda()))
        o += n
    got = list(isl.call_batches(iter(batches)))
    assert [k for k, _ in got] == list(range(len(sizes)))
    n_hands = 0
    for (_, res), exp in zip(got, ref):
        assert len(res) == len(exp)
        for (c, s, hs), (c2, s2, hs2) in zip(res, exp):
            assert np.array_equal(c, c2) and np.array_equal(s, s2) and len(hs) == len(hs2)
            n_hands += len(hs)
            for a, b in zip(hs, hs2):
                assert np.array_equal(a, b)
    assert n_hands > 0
