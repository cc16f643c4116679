"""The split-fp16 Winograd F(2x2, 3x3) kernel (csrc/wino_f16.hip, the 3x3 layers of
src/model.py:25-64 on chip-filling grids) against conv_x3 (ISLPOSE_X3_W2=0) and the oracle.
Runs on an MI355X only (-m gpu)."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref
from islpose import synth
from islpose import runtime as rt

pytestmark = pytest.mark.gpu
TOL = 1e-4   # north_star: heatmap/PAF tensors within 1e-4 relative (max|d| / max|ref|) in fp32


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def _inputs(n, h, w, seed):
    f = synth.synth_frames(n, h, w, seed=seed)
    return np.ascontiguousarray(np.transpose(f.astype(np.float32), (0, 3, 1, 2)) / 256 - 0.5)


@pytest.fixture(scope="module")
def w25():
    return synth.synth_weights(rt.ISL_BODY25)


@pytest.fixture(autouse=True)
def _w2_everywhere(monkeypatch):
    """Every eligible launch on the Winograd kernel (the default takes layers with >= 256 input
    channels only), so the parity checks cover the 128-channel stage layers too."""
    monkeypatch.setenv("ISLPOSE_X3_W2", "1")


@pytest.fixture(scope="module")
def net25(w25):
    n = rt.Net(rt.ISL_BODY25)
    n.load_weights(w25)
    return n


def _w2_layers(net):
    return [name for name, v in net.op_variants() if rt.decode_variant(v).get("wino2")]


# (n, h, w): the bench's 368x656 (46x82 / 92x164 levels, even), an odd level-3 plane
# (376x664 -> 47x83: odd tile rows and columns, a half band at the bottom), and a frame whose
# level-3 rows are exactly 32 tiles wide (W = 63 -> 504 px)
@pytest.mark.parametrize("n,h,w", [(2, 368, 656), (1, 376, 664), (2, 264, 504)])
def test_wino2_vs_x3_and_oracle(net25, w25, n, h, w, monkeypatch):
    x = _inputs(n, h, w, seed=h + 3 * w)
    xt = torch.from_numpy(x).cuda()
    paf, heat = net25.forward(xt)
    torch.cuda.synchronize()
    used = _w2_layers(net25)
    assert "conv4_2" in used and "conv4_3_CPM" in used and "conv4_4_CPM" in used, used
    assert any(k.startswith("Mconv2_stage1") for k in used), used
    monkeypatch.setenv("ISLPOSE_X3_W2", "0")
    paf0, heat0 = net25.forward(xt)
    torch.cuda.synchronize()
    assert not _w2_layers(net25)
    ep, eh = _rel(paf.cpu().numpy(), paf0.cpu().numpy()), _rel(heat.cpu().numpy(), heat0.cpu().numpy())
    print("wino2 vs x3: paf %.3g heat %.3g (%d layers)" % (ep, eh, len(used)))
    assert ep < 2e-5 and eh < 2e-5, (ep, eh)
    rp, rh = cpu_ref.make_net_fn("body25", w25)(x[:1])
    ep, eh = _rel(paf[:1].cpu().numpy(), rp), _rel(heat[:1].cpu().numpy(), rh)
    print("wino2 vs oracle: paf %.3g heat %.3g" % (ep, eh))
    assert ep < TOL and eh < TOL, (ep, eh)


def test_wino2_hand_736_vs_x3():
    """The hand net at its 736 px scale (92^2 at level 3: the VGG front's conv4/conv5 layers
    on the Winograd kernel) against conv_x3, and within the bar of the oracle."""
    w = synth.synth_weights(rt.ISL_HAND)
    net = rt.Net(rt.ISL_HAND)
    net.load_weights(w)
    x = _inputs(1, 736, 736, seed=11)
    xt = torch.from_numpy(x).cuda()
    out = net.forward(xt)
    torch.cuda.synchronize()
    used = _w2_layers(net)
    assert "conv5_2" in used, used
    import os
    os.environ["ISLPOSE_X3_W2"] = "0"
    try:
        out0 = net.forward(xt)
        torch.cuda.synchronize()
    finally:
        os.environ["ISLPOSE_X3_W2"] = "1"
    assert _rel(out.cpu().numpy(), out0.cpu().numpy()) < 2e-5
    ref = cpu_ref.make_net_fn("hand", w)(x)
    assert _rel(out.cpu().numpy(), ref) < TOL


def test_wino2_graph_replay_bit_identical(net25):
    """Graph replay of a chain with Winograd launches gives the eager bits."""
    xt = torch.from_numpy(_inputs(2, 368, 656, seed=8)).cuda()
    p0, h0 = net25.forward(xt)
    net25.set_graph(True)
    try:
        for _ in range(3):
            p1, h1 = net25.forward(xt)
    finally:
        net25.set_graph(False)
    torch.cuda.synchronize()
    assert torch.equal(p0, p1) and torch.equal(h0, h1)


def test_wino2_deterministic_and_batch_position(net25):
    """Same frame alone and inside a batch (at another position) gives the same bits: the
    Winograd blocks never span frames and sum in a fixed order."""
    x = _inputs(3, 368, 656, seed=21)
    xt = torch.from_numpy(x).cuda()
    p3, h3 = net25.forward(xt)
    p1, h1 = net25.forward(xt[2:3].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(p3[2:3], p1) and torch.equal(h3[2:3], h1)


def test_wino2_default_rule(net25, monkeypatch):
    """The default (ISLPOSE_X3_W2 unset): the Winograd kernel on the eligible layers with >= 256
    input channels (the 384-channel stage inputs, conv3_2/3_3, conv4_2 .. conv4_4), conv_x3 on
    the 128-channel stage layers, where it is faster."""
    monkeypatch.delenv("ISLPOSE_X3_W2", raising=False)
    xt = torch.from_numpy(_inputs(1, 368, 656, seed=5)).cuda()
    net25.forward(xt)
    torch.cuda.synchronize()
    used = set(_w2_layers(net25))
    assert {"conv3_2", "conv3_3", "conv4_2", "conv4_3_CPM", "conv4_4_CPM"} <= used, used
    assert "Mconv2_stage1_L2_0" in used and "Mconv2_stage1_L2_1" not in used, used
