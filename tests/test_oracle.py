"""Pin the CPU oracle against the reference's own outputs (tests/golden, made by
tests/golden/make_golden.py from /root/reference) and against scipy."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import cpu_ref, cv_resize
from islpose import synth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _frame_input(h, w, seed):
    f = synth.synth_frames(1, h, w, seed=seed)[0]
    return np.ascontiguousarray(np.transpose(np.float32(f[:, :, :, None]), (3, 2, 0, 1)) / 256 - 0.5)


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.fixture(scope="module")
def g1():
    return np.load(os.path.join(GOLDEN, "g1_networks.npz"))


def test_body25_forward_matches_reference(g1):
    w = synth.synth_weights(0)
    torch.set_num_threads(8)
    for h, wd in ((184, 328), (50, 70)):
        x = _frame_input(h, wd, int(g1["body25_%dx%d_seed" % (h, wd)]))
        paf, heat = cpu_ref.make_net_fn("body25", w)(x)
        assert paf.shape == g1["body25_%dx%d_paf" % (h, wd)].shape
        assert _rel(paf, g1["body25_%dx%d_paf" % (h, wd)]) < 1e-6
        assert _rel(heat, g1["body25_%dx%d_heat" % (h, wd)]) < 1e-6


def test_coco_forward_on_ski_matches_reference(g1):
    ski = np.load(os.path.join(GOLDEN, "ski_bgr.npz"))["img"]
    im, padded_hw, pad = cpu_ref.net_input(ski, 0.5 * 368 / ski.shape[0])
    assert im.shape == (1, 3, 184, 200)
    paf, heat = cpu_ref.make_net_fn("coco", synth.synth_weights(1))(im)
    assert _rel(paf, g1["coco_ski_paf"]) < 1e-6
    assert _rel(heat, g1["coco_ski_heat"]) < 1e-6
    assert heat.min() >= 0          # the Mconv7_stage6_L2 ReLU quirk (model.py:218)


def test_hand_forward_matches_reference(g1):
    w = synth.synth_weights(2)
    for s in (184, 368):
        x = _frame_input(s, s, int(g1["hand_%d_seed" % s]))
        out = cpu_ref.make_net_fn("hand", w)(x)
        assert _rel(out, g1["hand_%d" % s]) < 1e-6


def test_hand_output_size_table():
    """hand_model_output_size.json: net output side == floor(i / 8) (floor-mode pooling)."""
    table = json.load(open(os.path.join(GOLDEN, "hand_model_output_size.json")))
    assert len(table) == 990
    for k, v in table.items():
        assert v == int(k) // 8


def test_gaussian_blur_bit_exact_vs_scipy():
    from scipy.ndimage import gaussian_filter
    rng = np.random.RandomState(0)
    for shape in ((46, 82), (37, 19), (13, 13), (200, 31)):
        a = rng.rand(*shape) ** 4
        assert np.array_equal(cpu_ref.gaussian_blur(a), gaussian_filter(a, sigma=3))


def test_gaussian_weights_match_scipy():
    from scipy.ndimage import _filters
    assert np.array_equal(cpu_ref.gaussian_weights(), _filters._gaussian_kernel1d(3, 0, 12)[::-1])


@pytest.fixture(scope="module")
def g2():
    z = np.load(os.path.join(GOLDEN, "g2_body_post.npz"))
    names = sorted({k.split("/")[0] for k in z.files})
    return z, names


def _replay(z, name):
    n = len(z[name + "/scales"])
    outs = [(z[name + "/paf%d" % i], z[name + "/heat%d" % i]) for i in range(n)]
    it = iter(outs)

    def net(im):
        paf, heat = next(it)
        return paf[None], heat[None]
    return net


def test_body_post_matches_reference(g2):
    z, names = g2
    assert len(names) >= 9
    for name in names:
        mt = str(z[name + "/model_type"])
        H, W = (int(v) for v in z[name + "/frame_hw"])
        scales = tuple(float(s) for s in z[name + "/scales"])
        cand, subset = cpu_ref.body_call(np.zeros((H, W, 3), np.uint8), _replay(z, name), mt, scales)
        ref_c, ref_s = z[name + "/candidate"], z[name + "/subset"]
        assert cand.shape == ref_c.shape, name
        assert np.array_equal(cand, ref_c), name
        assert subset.shape == ref_s.shape, name
        assert np.array_equal(subset, ref_s), name


def test_hand_post_matches_reference():
    z = np.load(os.path.join(GOLDEN, "g4_hand_post.npz"))
    cases = sorted({k.split("/")[0] for k in z.files})
    for c in cases:
        crop = int(z[c + "/crop"])
        maps = iter([z[c + "/heat%d" % i] for i in range(4)])
        peaks = cpu_ref.hand_call(np.zeros((crop, crop, 3), np.uint8), lambda im: next(maps)[None])
        assert peaks.dtype == z[c + "/peaks"].dtype
        assert np.array_equal(peaks, z[c + "/peaks"]), c


def test_hand_detect_matches_reference():
    z = np.load(os.path.join(GOLDEN, "g5_hand_detect.npz"))
    cases = sorted({k.split("/")[0] for k in z.files})
    assert len(cases) >= 4
    for c in cases:
        res = cpu_ref.hand_detect(z[c + "/candidate"], z[c + "/subset"], tuple(z[c + "/img_hw"]))
        got = np.array([[x, y, w, int(l)] for x, y, w, l in res], np.int64).reshape(-1, 4)
        assert np.array_equal(got, z[c + "/result"]), c


def test_resize_identity_and_shapes():
    img = synth.synth_frames(1, 37, 53)[0]
    assert np.array_equal(cv_resize.resize(img, (53, 37)), img)
    out = cv_resize.resize(img, (0, 0), fx=0.5, fy=0.5)
    assert out.shape == (18, 26, 3) and out.dtype == np.uint8      # cvRound(18.5) = 18 (half-even)
    f = np.random.RandomState(1).rand(5, 7, 3).astype(np.float32)
    up = cv_resize.resize(f, (0, 0), fx=8, fy=8)
    assert up.shape == (40, 56, 3) and up.dtype == np.float32
    # constant images stay constant up to rounding of the coefficient sums
    c = np.full((6, 9, 26), 0.25, np.float32)
    assert np.allclose(cv_resize.resize(c, (0, 0), fx=8, fy=8), 0.25, atol=1e-6)
