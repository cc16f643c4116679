"""The BASELINE configs end to end on the GPU, against the oracle.

* C4 (configs[3]): body_25 with scale_search [0.5, 1, 1.5, 2] (the commented list
  of /root/reference/src/body.py:40) on 368x656 frames: every scale's net output
  (184x328 ... 736x1312) within 1e-4 of the oracle network, and candidate / subset /
  connection_all bit-exact against the oracle post on the GPU's own maps (the
  doubling quirk of body.py:80 included).
* Hand nets at 552^2 and 736^2 (the upper two of Hand.__call__'s scales,
  hand.py:25-56) within 1e-4 of the oracle.
* C5 (configs[4]): the extract_features_mp.py:122-132 pipeline on 1080x1920 RGB frames:
  the per-frame JSON text equals the oracle composition (oracle pre/post for the body,
  handDetect, the 4-scale hand path per crop) on the GPU's own maps; the nets
  themselves are checked against the oracle networks separately.

The post comparisons replay the GPU's low-res maps through the oracle: the nets are
fp32 computations with a 1e-4 tolerance, the post is bit-exact on identical maps.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import cpu_ref
from islpose import synth
from islpose import runtime as rt
from islpose.body import BodyEstimator, scale_geometry
from islpose.hand import HandEstimator, HAND_SCALES

import _tame

pytestmark = pytest.mark.gpu
TOL = 1e-4
C4_SCALES = (0.5, 1.0, 1.5, 2.0)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.fixture(scope="module")
def c4():
    frames = synth.synth_frames(2, 368, 656, seed=41)
    w = _tame.tame_body(synth.synth_weights(0), frames[0], scale=0.5, gain=0.02)
    est = BodyEstimator(w, "body25", scale_search=C4_SCALES)
    t = torch.from_numpy(frames).cuda()
    geoms, pafs, heats = est.run_scales(t, keep_maps=True)
    torch.cuda.synchronize()
    return {"frames": frames, "w": w, "est": est, "t": t, "geoms": geoms,
            "pafs": [p.cpu().numpy() for p in pafs], "heats": [h.cpu().numpy() for h in heats]}


@pytest.mark.parametrize("si", range(4))
def test_c4_pyramid_nets_vs_oracle(c4, si):
    """Scale si of the pyramid: net input round8(s * 368 * 656/368 ...) -> 184x328,
    368x656, 552x984, 736x1312; both frames within 1e-4 of the oracle network."""
    fn = cpu_ref.make_net_fn("body25", c4["w"])
    (m, nh, nw, _, _) = scale_geometry(368, 656, C4_SCALES)[si]
    assert c4["geoms"][si][:2] == (nh, nw)
    for i in range(2):
        im, _, _ = cpu_ref.net_input(c4["frames"][i], m)
        assert im.shape[2:] == (nh, nw)
        rp, rh = fn(im)
        ep, eh = _rel(c4["pafs"][si][i:i + 1], rp), _rel(c4["heats"][si][i:i + 1], rh)
        print("scale %.1f net %dx%d frame %d: rel err paf %.3g heat %.3g" % (C4_SCALES[si], nh, nw, i, ep, eh))
        assert ep < TOL and eh < TOL


def test_c4_pyramid_post_bit_exact(c4):
    """candidate / subset / connection_all of the 4-scale frame == the oracle post on the
    same maps; the estimate() path (maps read back from the arena per scale) agrees."""
    est, frames = c4["est"], c4["frames"]
    res = est.post_maps(368, 656, c4["geoms"], [torch.from_numpy(p).cuda() for p in c4["pafs"]],
                        [torch.from_numpy(h).cuda() for h in c4["heats"]])
    direct = est.estimate(c4["t"], details=True)
    for i in range(2):
        it = iter([(c4["pafs"][s][i:i + 1], c4["heats"][s][i:i + 1]) for s in range(4)])
        hm, pm = cpu_ref.body_maps(frames[i], lambda im: next(it), "body25", C4_SCALES)
        cand, subset, _, conn = cpu_ref.body_post(hm, pm, "body25", 368)
        assert len(subset) >= 2, "the tamed weights should find persons"
        assert np.array_equal(res[i].candidate, cand), i
        assert np.array_equal(res[i].subset, subset), i
        for a, b in zip(res[i].connection_all, conn):
            assert np.array_equal(np.asarray(a).reshape(-1, 5), np.asarray(b).reshape(-1, 5)), i
        assert np.array_equal(direct[i].candidate, cand) and np.array_equal(direct[i].subset, subset), i


@pytest.fixture(scope="module")
def hand_w():
    return synth.synth_weights(2)


@pytest.mark.parametrize("side", [552, 736])
def test_hand_net_large_scales_vs_oracle(hand_w, side):
    net = rt.Net(rt.ISL_HAND)
    net.load_weights(hand_w)
    x = np.ascontiguousarray(np.transpose(synth.synth_frames(1, side, side, seed=side).astype(np.float32),
                                          (0, 3, 1, 2)) / 256 - 0.5)
    out = net.forward(torch.from_numpy(x).cuda()).cpu().numpy()
    ref = cpu_ref.make_net_fn("hand", hand_w)(x)
    assert out.shape == ref.shape == (1, 22, side // 8, side // 8)
    e = _rel(out, ref)
    print("hand %d: rel err %.3g" % (side, e))
    assert e < TOL


def test_c5_pipeline_1080p_json_vs_oracle(tmp_path, hand_w):
    """Two 1080x1920 RGB frames through islpose.pipeline (ISLSignPos.call_batch: Mode R
    body net 184x328, batched hand crops): each frame's JSON == json.dumps of the oracle
    composition (extract_features_mp.py:79-84) on the GPU's own maps."""
    from islpose import pipeline
    from src.body import Body
    from src.hand import Hand
    from src.ISL_Model_parameter import ISLSignPos
    rgb = synth.synth_frames(2, 1080, 1920, seed=57)
    bgr = np.ascontiguousarray(rgb[..., ::-1])
    wb = _tame.tame_body(synth.synth_weights(0), bgr[0], scale=0.5 * 368 / 1080, gain=0.05)
    tw = lambda d: {k: torch.from_numpy(v) for k, v in d.items()}  # noqa: E731
    body, hand = Body(tw(wb), "body25"), Hand(tw(hand_w))
    isl = ISLSignPos(body.model, hand.model)
    base = tmp_path / "data"
    os.makedirs(base)
    np.save(base / "clip.npy", rgb)
    rows = [{"Filepath": "clip.npy", "type": "Greetings", "expression": "hello"}]
    feats, ex = pipeline.extract_dataset(rows, pipeline.npy_decoder(str(base)), isl, str(tmp_path / "out"),
                                         batch=2, export=False)
    assert len(feats) == 2 and ex.frames_done == 2
    # the GPU's maps for the same batch (deterministic: same batch, same kernels)
    best = BodyEstimator(model_type="body25", scale_search=(0.5,), net=body.model.native(0))
    hest = HandEstimator(net=hand.model.native(0))
    t = torch.from_numpy(bgr).cuda()
    geoms, pafs, heats = best.run_scales(t, keep_maps=True)
    n_hands = 0
    for i in range(2):
        pl, hl = pafs[0][i:i + 1].cpu().numpy(), heats[0][i:i + 1].cpu().numpy()
        cand, subset = cpu_ref.body_call(bgr[i], lambda im: (pl, hl), "body25", (0.5,))
        boxes = cpu_ref.hand_detect(cand, subset, bgr[i].shape[:2])
        hands = []
        if boxes:
            hh = [h.cpu().numpy() for h in hest.run_crops(t, [(i, x, y, w) for x, y, w, _ in boxes])]
            for j, (x, y, w, _) in enumerate(boxes):
                it = iter([h[j:j + 1] for h in hh])
                pk = cpu_ref.hand_call(np.ascontiguousarray(bgr[i, y:y + w, x:x + w]), lambda im: next(it))
                pk[:, 0] = np.where(pk[:, 0] == 0, pk[:, 0], pk[:, 0] + x)    # ISL_Model_parameter.py:56-59
                pk[:, 1] = np.where(pk[:, 1] == 0, pk[:, 1], pk[:, 1] + y)
                hands.append(pk)
        n_hands += len(hands)
        ref = json.dumps({'candidate': cand.tolist(), 'subset': subset.tolist(),
                          'all_hand_peaks': [p.tolist() for p in hands]})
        with open(feats[i]['filepath']) as fh:
            assert fh.read() == ref, i
    assert n_hands >= 1, "the tamed weights should produce hand crops"
    # the body net at this frame size against the oracle network
    im, _, _ = cpu_ref.net_input(bgr[0], 0.5 * 368 / 1080)
    rp, rh = cpu_ref.make_net_fn("body25", wb)(im)
    assert _rel(pafs[0][0:1].cpu().numpy(), rp) < TOL and _rel(heats[0][0:1].cpu().numpy(), rh) < TOL


def test_isl_call_per_frame_1080p_equals_batch_and_per_crop(hand_w):
    """The unchanged scripts' per-frame call (extract_features_mp.py:125-130:
    model(frame[:, :, ::-1]) on one 1080x1920 frame at a time) == call_batch over the same frames
    == the reference's composition (Body, handDetect, Hand per crop, offsets;
    ISL_Model_parameter.py:51-60) bit for bit, with hand crops present."""
    from src import util
    from src.body import Body
    from src.hand import Hand
    from src.ISL_Model_parameter import ISLSignPos
    rgb = synth.synth_frames(3, 1080, 1920, seed=58)
    bgr = np.ascontiguousarray(rgb[..., ::-1])
    wb = _tame.tame_body(synth.synth_weights(0), bgr[0], scale=0.5 * 368 / 1080, gain=0.05)
    tw = lambda d: {k: torch.from_numpy(v) for k, v in d.items()}  # noqa: E731
    body, hand = Body(tw(wb), "body25"), Hand(tw(hand_w))
    isl = ISLSignPos(body.model, hand.model)
    batch = isl.call_batch(bgr)
    n_hands = 0
    for i in range(3):
        cand, subset, hands = isl.call(rgb[i][:, :, ::-1])       # a non-contiguous view, as the script
        c2, s2, h2 = batch[i]
        assert np.array_equal(cand, c2) and np.array_equal(subset, s2) and len(hands) == len(h2)
        boxes = util.handDetect(cand, subset, bgr[i])
        assert len(boxes) == len(hands)
        for (x, y, w, _), pk, pb in zip(boxes, hands, h2):
            ref = hand(bgr[i, y:y + w, x:x + w])
            ref[:, 0] = np.where(ref[:, 0] == 0, ref[:, 0], ref[:, 0] + x)
            ref[:, 1] = np.where(ref[:, 1] == 0, ref[:, 1], ref[:, 1] + y)
            assert np.array_equal(pk, ref) and np.array_equal(pk, pb)
        n_hands += len(hands)
    assert n_hands >= 1, "the tamed weights should produce hand crops"
