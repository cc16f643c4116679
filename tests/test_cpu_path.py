"""The product's GPU-less path (islpose.cpu + the CPU forwards of src/model.py; the reference
runs Body / Hand on the CPU without a CUDA device, /root/reference/src/body.py:31-32,
hand.py:18-20) pinned against the reference's own outputs: the networks against G1, the
body post against G2, the hand post against G4 (tests/golden, made from /root/reference),
and the resize against the oracle restatement (the checker only; the product path does not
import it)."""
import os

import numpy as np
import pytest
import torch

from oracle import cpu_ref, cv_resize
from islpose import cpu, synth
from src import util
from src.model import bodypose_25_model, bodypose_model, handpose_model

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def _module(cls, seed):
    m = cls()
    w = {k: torch.from_numpy(v) for k, v in synth.synth_weights(seed).items()}
    m.load_state_dict(util.transfer(m, w))
    return m.eval()


def _frame_input(h, w, seed):
    f = synth.synth_frames(1, h, w, seed=seed)[0]
    return np.ascontiguousarray(np.transpose(np.float32(f[:, :, :, None]), (3, 2, 0, 1)) / 256 - 0.5)


@pytest.fixture(scope="module")
def g1():
    return np.load(os.path.join(GOLDEN, "g1_networks.npz"))


def test_cpu_forward_matches_reference(g1):
    torch.set_num_threads(8)
    with torch.no_grad():
        m = _module(bodypose_25_model, 0)
        x = _frame_input(50, 70, int(g1["body25_50x70_seed"]))
        paf, heat = m.cpu_forward(torch.from_numpy(x))
        assert _rel(paf.numpy(), g1["body25_50x70_paf"]) < 1e-6 and _rel(heat.numpy(), g1["body25_50x70_heat"]) < 1e-6
        ski = np.load(os.path.join(GOLDEN, "ski_bgr.npz"))["img"]
        im, _, _ = cpu_ref.net_input(ski, 0.5 * 368 / ski.shape[0])
        paf, heat = _module(bodypose_model, 1).cpu_forward(torch.from_numpy(im))
        assert _rel(paf.numpy(), g1["coco_ski_paf"]) < 1e-6 and _rel(heat.numpy(), g1["coco_ski_heat"]) < 1e-6
        x = _frame_input(184, 184, int(g1["hand_184_seed"]))
        out = _module(handpose_model, 2).cpu_forward(torch.from_numpy(x))
        assert _rel(out.numpy(), g1["hand_184"]) < 1e-6


@pytest.mark.parametrize("dtype,shape,kw", [(np.uint8, (37, 53, 3), dict(fx=0.7)), (np.uint8, (40, 64, 3), dict(fx=1.6)),
                                            (np.float32, (23, 41, 26), dict(fx=8)),
                                            (np.float32, (184, 328, 5), dict(dsize=(656, 368))),
                                            (np.float32, (61, 45, 3), dict(dsize=(30, 100)))])
def test_cpu_resize_matches_restatement(dtype, shape, kw):
    rng = np.random.RandomState(sum(shape))
    img = (rng.randint(0, 256, shape) if dtype == np.uint8 else rng.randn(*shape)).astype(dtype)
    got = cpu.resize(img, **kw)
    ref = cv_resize.resize(img, **(dict(fx=kw["fx"], fy=kw["fx"]) if "fx" in kw else kw))
    assert got.dtype == ref.dtype and np.array_equal(got, ref)


def test_cpu_body_post_matches_reference():
    z = np.load(os.path.join(GOLDEN, "g2_body_post.npz"))
    names = sorted({k.split("/")[0] for k in z.files})
    for name in names:
        mt = str(z[name + "/model_type"])
        H, W = (int(v) for v in z[name + "/frame_hw"])
        scales = tuple(float(s) for s in z[name + "/scales"])
        it = iter([(z[name + "/paf%d" % i][None], z[name + "/heat%d" % i][None]) for i in range(len(scales))])
        cand, subset = cpu.body_call(np.zeros((H, W, 3), np.uint8), lambda im: next(it), mt, scales)
        assert cand.shape == z[name + "/candidate"].shape and np.array_equal(cand, z[name + "/candidate"]), name
        assert subset.shape == z[name + "/subset"].shape and np.array_equal(subset, z[name + "/subset"]), name


def test_cpu_hand_post_matches_reference():
    z = np.load(os.path.join(GOLDEN, "g4_hand_post.npz"))
    for c in sorted({k.split("/")[0] for k in z.files}):
        crop = int(z[c + "/crop"])
        maps = iter([z[c + "/heat%d" % i] for i in range(4)])
        peaks = cpu.hand_call(np.zeros((crop, crop, 3), np.uint8), lambda im: next(maps)[None])
        assert peaks.dtype == z[c + "/peaks"].dtype and np.array_equal(peaks, z[c + "/peaks"]), c


def test_cpu_assemble_third_match_raises_index_error():
    """body.py:193-196: a connection matching three subset rows stores subset_idx[2] and raises
    IndexError.  Crafted connections reach it: limb 1 (neck -> r-shoulder) makes rows R0 / R1,
    a third connection overlapping both takes the found == 2 'as found == 1' branch and leaves
    shoulder 3 in two rows; limb 2 (r-shoulder -> r-elbow) makes R2 with elbow 5, and (3, 5)
    then matches R0, R1 and R2.  The GPU assembly flags the same case (ISL_E_INDEX)."""
    all_peaks = [[(i, i, 0.5 + 0.01 * i, i) for i in range(8)]] + [[] for _ in range(24)]
    conns = [np.zeros((0, 5)) for _ in range(24)]
    conns[1] = np.array([[0, 2, 0.5, 0, 0], [1, 3, 0.5, 1, 1], [0, 3, 0.4, 0, 1]], np.float64)
    conns[2] = np.array([[4, 5, 0.5, 0, 0], [3, 5, 0.4, 1, 0]], np.float64)
    with pytest.raises(IndexError):
        cpu._assemble(all_peaks, conns, [], "body25", 26)
    with pytest.raises(IndexError):
        cpu_ref.assemble(all_peaks, conns, [], "body25")
    # without the last connection both return the same rows
    conns[2] = conns[2][:1]
    cand, subset = cpu._assemble(all_peaks, conns, [], "body25", 26)
    rc, rs = cpu_ref.assemble(all_peaks, conns, [], "body25")
    assert np.array_equal(cand, rc) and np.array_equal(subset, rs)


@pytest.mark.skipif(torch.cuda.is_available(), reason="the GPU-less seam (with a device Body runs on it)")
def test_body_and_hand_without_gpu_match_oracle():
    """src.body.Body / src.hand.Hand on a GPU-less host: frame in, (candidate, subset) / peaks
    out, equal to the oracle's composition of the reference's call on the same weights."""
    from src.body import Body
    from src.hand import Hand
    torch.set_num_threads(8)
    ski = np.load(os.path.join(GOLDEN, "ski_bgr.npz"))["img"]
    w1 = synth.synth_weights(1)
    b = Body({k: torch.from_numpy(v) for k, v in w1.items()}, "coco")
    cand, subset = b(ski)
    rc, rs = cpu_ref.body_call(ski, cpu_ref.make_net_fn("coco", w1), "coco", (0.5,))
    assert np.array_equal(cand, rc) and np.array_equal(subset, rs)
    w2 = synth.synth_weights(2)
    h = Hand({k: torch.from_numpy(v) for k, v in w2.items()})
    crop = np.ascontiguousarray(ski[:96, :96])
    assert np.array_equal(h(crop), cpu_ref.hand_call(crop, cpu_ref.make_net_fn("hand", w2)))
