"""The wave-range kernel (conv_x3_wr, VAR 8; csrc/conv_x3.hip): small grids whose canonical K
ranges would run across blocks (batch-1 Mode R, reference callers' one-frame-per-call pattern,
/root/reference/extract_features_mp.py:125-130 -> src/model.py:171-207) sum each range in one
wave straight from L2 and add the ranges in LDS in x3_canonical_order.  It must give the bits of
the split-K launches + x3_splitk_reduce (ISLPOSE_X3_WR=0) and of the in-block ranges of large
batches, and stay within the oracle tolerance."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref
from islpose import synth
from islpose import runtime as rt

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def _inputs(n, h, w, seed):
    f = synth.synth_frames(n, h, w, seed=seed)
    return np.ascontiguousarray(np.transpose(f.astype(np.float32), (0, 3, 1, 2)) / 256 - 0.5)


@pytest.fixture(scope="module")
def w25():
    return synth.synth_weights(0)


@pytest.fixture(scope="module")
def net25(w25):
    n = rt.Net(rt.ISL_BODY25)
    n.load_weights(w25)
    return n


def _run(net, x, env, monkeypatch):
    for k in ("ISLPOSE_X3_WR", "ISLPOSE_X3_WR_WN"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    out = net.forward(x)
    torch.cuda.synchronize()
    var = [rt.decode_variant(v) for _, v in net.op_variants()]
    return out, var


@pytest.mark.parametrize("n", [1, 2])
def test_wr_equals_split_reduce_body25(net25, w25, n, monkeypatch):
    """Mode R (net 184x328) at batch 1 and 2: the default (wave ranges on the layers with at most
    4 K ranges, split-K on the others) == the split-K launches + reduce everywhere bit for bit, and
    so do every layer with ranges on the wave ranges (ISLPOSE_X3_WR=3) in both tile widths (32 / 64
    pixels per wave) and the small grids without ranges on one wave per block (ISLPOSE_X3_WR=2);
    batch-1 frames equal the oracle."""
    x = torch.from_numpy(_inputs(n, 184, 328, seed=410 + n)).cuda()
    (p0, h0), v0 = _run(net25, x, {"ISLPOSE_X3_WR": "0"}, monkeypatch)
    assert not any(v.get("var", 0) & 8 and not v.get("rgb") for v in v0)
    (p1, h1), v1 = _run(net25, x, {}, monkeypatch)
    wr = [v for v in v1 if v.get("var", 0) & 8 and not v.get("rgb")]
    assert len(wr) >= 40, len(wr)
    assert all(v["bco"] == 32 and v["bpx"] == 32 for v in wr)
    assert torch.equal(p0, p1) and torch.equal(h0, h1)
    (p4, h4), v4 = _run(net25, x, {"ISLPOSE_X3_WR": "3"}, monkeypatch)
    assert sum(1 for v in v4 if v.get("var", 0) & 8 and not v.get("rgb")) >= 90
    assert not any(v.get("split") for v in v4)
    assert torch.equal(p0, p4) and torch.equal(h0, h4)
    (p2, h2), v2 = _run(net25, x, {"ISLPOSE_X3_WR": "3", "ISLPOSE_X3_WR_WN": "2"}, monkeypatch)
    assert sum(1 for v in v2 if v.get("var", 0) & 8 and v["bpx"] == 64) >= 90
    assert torch.equal(p0, p2) and torch.equal(h0, h2)
    (p3, h3), v3 = _run(net25, x, {"ISLPOSE_X3_WR": "2"}, monkeypatch)
    assert sum(1 for v in v3 if v.get("var", 0) & 8 and not v.get("ranged")) >= 1
    assert torch.equal(p0, p3) and torch.equal(h0, h3)
    rp, rh = cpu_ref.make_net_fn("body25", w25)(x[:1].cpu().numpy())
    assert _rel(p1[:1].cpu().numpy(), rp) < TOL and _rel(h1[:1].cpu().numpy(), rh) < TOL


def test_wr_batch_invariant(net25, monkeypatch):
    """A frame alone (wave ranges) == the same frame inside a batch of 24 (in-block ranges on the
    two-K-group / deep loops): the canonical order is the same."""
    for k in ("ISLPOSE_X3_WR", "ISLPOSE_X3_WR_WN"):
        monkeypatch.delenv(k, raising=False)
    x = torch.from_numpy(_inputs(24, 184, 328, seed=4242)).cuda()
    pb, hb = net25.forward(x)
    for i in (0, 11, 23):
        p1, h1 = net25.forward(x[i:i + 1].contiguous())
        assert torch.equal(p1, pb[i:i + 1]) and torch.equal(h1, hb[i:i + 1]), i


@pytest.mark.parametrize("kind,h,w,n", [("hand", 184, 184, 2), ("coco", 184, 200, 1)])
def test_wr_7x7_equals_split_reduce(kind, h, w, n, monkeypatch):
    """7x7 stage layers at 23x23 / 23x25 (the hand's 184-pixel scale for two crops, COCO on
    ski.jpg's net size) on the wave ranges == the split-K form, and within the oracle tolerance."""
    code = {"hand": rt.ISL_HAND, "coco": rt.ISL_COCO}[kind]
    wts = synth.synth_weights(code)
    net = rt.Net(code)
    net.load_weights(wts)
    x = torch.from_numpy(_inputs(n, h, w, seed=h * n + 1)).cuda()
    o0, v0 = _run(net, x, {"ISLPOSE_X3_WR": "0"}, monkeypatch)
    o1, v1 = _run(net, x, {"ISLPOSE_X3_WR": "3"}, monkeypatch)
    assert sum(1 for v in v1 if v.get("var", 0) & 8 and v.get("ks") == 7 and not v.get("rgb")) >= 10
    o0 = o0 if isinstance(o0, tuple) else (o0,)
    o1 = o1 if isinstance(o1, tuple) else (o1,)
    for a, b in zip(o0, o1):
        assert torch.equal(a, b)
    ref = cpu_ref.make_net_fn(kind, wts)(x.cpu().numpy())
    ref = ref if isinstance(ref, tuple) else (ref,)
    for a, r in zip(o1, ref):
        assert _rel(a.cpu().numpy(), r) < TOL

