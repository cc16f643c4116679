"""The fused 1x1 pair (conv_x3 VAR 16): Mconv6 -> Mconv7 of every body_25 stage
(/root/reference/src/model.py:108-109, 125-126, make_layers_Mconv :48-64) and the hand's
conv6_1/6_2 and Mconv6/7 pairs (:360-392) in one launch, the Mconv6 output never written.
Checked against the oracle at the tolerance of the north star, against the two-launch path
(ISLPOSE_X3_FUSE67=0) at fp32 round-off, and for batch-invariant bits.  GPU only."""
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
    return synth.synth_weights(0)


@pytest.fixture(scope="module")
def net25(w25):
    n = rt.Net(rt.ISL_BODY25)
    n.load_weights(w25)
    return n


def _assert_fused(net, n_pairs):
    var = net.op_variants()
    fused = [(k, rt.decode_variant(v)) for k, (_, v) in enumerate(var) if rt.decode_variant(v).get("fused67")]
    assert len(fused) == n_pairs, [var[k][0] for k, _ in fused]
    for k, d in fused:
        assert d["ks"] == 1 and d["bco"] in (128, 256, 512), (var[k], d)
        assert var[k + 1][1] == -2, var[k + 1]          # the second layer ran inside the first
    return [var[k][0] for k, _ in fused]


@pytest.mark.parametrize("n,h,w", [(1, 184, 328), (2, 92, 164), (3, 64, 200)])
def test_body25_fused_pair_vs_oracle(net25, w25, monkeypatch, n, h, w):
    """Mode R's net size at batch 1 and two awkward sizes: all six Mconv6 -> Mconv7 pairs fused
    (forced, ISLPOSE_X3_FUSE67=2, and asserted through isl_net_op_info), the maps within the bar
    of the oracle; bit-identical to the pair's permuted two-launch form (=3: these stage planes
    have canonical K ranges) that small grids run by default; within fp32 round-off of the
    plain two launches (=0)."""
    x = _inputs(n, h, w, seed=7 * h + w + n)
    xt = torch.from_numpy(x).cuda()
    monkeypatch.setenv("ISLPOSE_X3_FUSE67", "2")
    paf, heat = net25.forward(xt)
    torch.cuda.synchronize()
    names = _assert_fused(net25, 6)
    assert all(nm.startswith("Mconv6") for nm in names), names
    monkeypatch.setenv("ISLPOSE_X3_FUSE67", "3")
    pp, hp = net25.forward(xt)
    torch.cuda.synchronize()
    var = net25.op_variants()
    assert not any(rt.decode_variant(v).get("fused67") for _, v in var)
    m7 = [rt.decode_variant(v) for name, v in var if name.startswith("Mconv7")]
    assert len(m7) == 6 and all(d.get("split") or d.get("ranged") for d in m7), m7
    assert torch.equal(pp, paf) and torch.equal(hp, heat)
    monkeypatch.delenv("ISLPOSE_X3_FUSE67")
    pd, hd = net25.forward(xt)
    torch.cuda.synchronize()
    assert torch.equal(pd, paf) and torch.equal(hd, heat)
    monkeypatch.setenv("ISLPOSE_X3_FUSE67", "0")
    paf0, heat0 = net25.forward(xt)
    torch.cuda.synchronize()
    assert not any(rt.decode_variant(v).get("fused67") for _, v in net25.op_variants())
    assert _rel(paf.cpu().numpy(), paf0.cpu().numpy()) < 1e-5
    assert _rel(heat.cpu().numpy(), heat0.cpu().numpy()) < 1e-5
    rp, rh = cpu_ref.make_net_fn("body25", w25)(x)
    assert _rel(paf.cpu().numpy(), rp) < TOL and _rel(heat.cpu().numpy(), rh) < TOL


def test_body25_fused_pair_timed_config(net25, w25):
    """The bench's configuration (32 frames of 368x656, net input 368x656): the six pairs on
    the fused variant (512- and 256-channel tiles), frames 0 and 31 against the oracle."""
    n, h, w = 32, 368, 656
    x = _inputs(n, h, w, seed=31337)
    paf, heat = net25.forward(torch.from_numpy(x).cuda())
    torch.cuda.synchronize()
    _assert_fused(net25, 6)
    bcos = sorted(rt.decode_variant(v)["bco"] for _, v in net25.op_variants()
                  if rt.decode_variant(v).get("fused67"))
    assert bcos == [256, 256, 512, 512, 512, 512], bcos
    fn = cpu_ref.make_net_fn("body25", w25)
    for f in (0, 31):
        rp, rh = fn(x[f:f + 1])
        assert _rel(paf[f:f + 1].cpu().numpy(), rp) < TOL and _rel(heat[f:f + 1].cpu().numpy(), rh) < TOL, f


def test_fused_pair_batch_invariant(net25):
    """A Mode R frame gives the same bits alone (the pairs as their permuted two launches)
    and inside a batch of 16 (the four 512-channel pairs fused, the two 256-channel ones --
    half the blocks -- still as two launches)."""
    x = torch.from_numpy(_inputs(16, 184, 328, seed=404)).cuda()
    pb, hb = net25.forward(x)
    assert sum(1 for _, v in net25.op_variants() if rt.decode_variant(v).get("fused67")) == 4
    for i in (0, 15):
        p1, h1 = net25.forward(x[i:i + 1].contiguous())
        assert torch.equal(p1, pb[i:i + 1]) and torch.equal(h1, hb[i:i + 1]), i


@pytest.mark.parametrize("n,side", [(1, 184), (5, 368)])
def test_hand_fused_pairs_vs_oracle(monkeypatch, n, side):
    """The hand net: conv6_1_CPM -> conv6_2_CPM (128 -> 512 -> 22) and the five Mconv6 ->
    Mconv7 pairs (128 -> 128 -> 22) fused (forced); maps vs the oracle and the two-launch
    paths (the permuted one bit-identical where the planes have canonical K ranges: 23x23)."""
    wh = synth.synth_weights(2)
    net = rt.Net(rt.ISL_HAND)
    net.load_weights(wh)
    x = _inputs(n, side, side, seed=side + n)
    xt = torch.from_numpy(x).cuda()
    monkeypatch.setenv("ISLPOSE_X3_FUSE67", "2")
    hm = net.forward(xt)
    torch.cuda.synchronize()
    names = _assert_fused(net, 6)
    assert "conv6_1_CPM" in names, names
    if side == 184:
        monkeypatch.setenv("ISLPOSE_X3_FUSE67", "3")
        hp = net.forward(xt)
        torch.cuda.synchronize()
        assert torch.equal(hp, hm)
    monkeypatch.setenv("ISLPOSE_X3_FUSE67", "0")
    h0 = net.forward(xt)
    torch.cuda.synchronize()
    assert _rel(hm.cpu().numpy(), h0.cpu().numpy()) < 1e-5
    rh = cpu_ref.make_net_fn("hand", wh)(x)
    rh = rh[0] if isinstance(rh, tuple) else rh
    assert _rel(hm.cpu().numpy(), rh) < TOL


def test_fused_pair_range_guard(w25, monkeypatch):
    """An Mconv6 output beyond the split range (|x| >= 65504 cannot be split into the fp16
    operand of Mconv7) raises the range flag inside the fused launch; Net.forward then
    recomputes on the fp32 kernels and still matches the oracle."""
    monkeypatch.setenv("ISLPOSE_X3_FUSE67", "2")
    w = dict(w25)
    for k in list(w):
        if k.startswith("Mconv6_stage0_L2") and k.endswith(".bias"):
            w[k] = w[k] + np.float32(1e5)
    net = rt.Net(rt.ISL_BODY25)
    net.load_weights(w)
    x = _inputs(1, 64, 96, seed=5)
    xt = torch.from_numpy(x).cuda()
    o0 = torch.empty((1, 52, 8, 12), device="cuda")
    o1 = torch.empty((1, 26, 8, 12), device="cuda")
    rt.check(rt.lib().isl_net_forward(net.h, rt.ptr(xt), 1, 64, 96, rt.ptr(o0), rt.ptr(o1), rt.stream_handle()))
    assert not net.range_ok()
    paf, heat = net.forward(xt)
    rp, rh = cpu_ref.make_net_fn("body25", w)(x)
    assert _rel(paf.cpu().numpy(), rp) < TOL and _rel(heat.cpu().numpy(), rh) < TOL


@pytest.mark.parametrize("n", [1, 8, 32])
def test_fused_pair_default_form_by_grid(net25, monkeypatch, n):
    """Default choice (x3_fused67_grid): Mode R frames fuse the pairs from half a block per CU
    up (batch 32), smaller batches run the permuted two launches; both forms give the same
    bits (so a frame's maps do not depend on its batch)."""
    x = torch.from_numpy(_inputs(n, 184, 328, seed=77 + n)).cuda()
    monkeypatch.delenv("ISLPOSE_X3_FUSE67", raising=False)
    pd, hd = net25.forward(x)
    torch.cuda.synchronize()
    fused = sum(1 for _, v in net25.op_variants() if rt.decode_variant(v).get("fused67"))
    assert fused == (6 if n >= 32 else 0), fused
    monkeypatch.setenv("ISLPOSE_X3_FUSE67", "3" if n >= 32 else "2")
    po, ho = net25.forward(x)
    torch.cuda.synchronize()
    assert torch.equal(po, pd) and torch.equal(ho, hd)


def _c12_run(net, x, mode, monkeypatch):
    monkeypatch.setenv("ISLPOSE_C12", mode)
    out = net.forward(x)
    torch.cuda.synchronize()
    var = net.op_variants()
    return (out if isinstance(out, tuple) else (out,)), var


@pytest.mark.parametrize("kind,n,h,w", [("body25", 2, 368, 656), ("body25", 1, 184, 328), ("body25", 3, 62, 94),
                                        ("body25", 1, 61, 94), ("hand", 2, 184, 184), ("hand", 1, 368, 368),
                                        ("coco", 1, 184, 200)])
def test_c12_conv1_pair_bit_identical(kind, n, h, w, monkeypatch):
    """conv1_1 -> conv1_2 -> pool1 in one launch (conv_c12.hip: conv1_1 recomputed on each 8 x 32
    tile's halo into LDS, the 2 x 2 pool in the epilogue; model.py:25-45's first layers of every
    net) == the rgb kernel + conv1_2 on the generic loop + the pool (ISLPOSE_C12=0) == the fused
    launch writing the pair-max buffer that conv2_1's staging finishes (=2), bit for bit, at the
    bench's size, Mode R, sizes with partial row and column tiles (an odd height: floor-mode pool),
    the hand scales and COCO; asserted to run (isl_net_op_info), and within the tolerance of the
    oracle."""
    code = {"body25": rt.ISL_BODY25, "hand": rt.ISL_HAND, "coco": rt.ISL_COCO}[kind]
    wts = synth.synth_weights(code)
    net = rt.Net(code)
    net.load_weights(wts)
    x = _inputs(n, h, w, seed=h * 3 + w + n)
    xt = torch.from_numpy(x).cuda()
    o0, v0 = _c12_run(net, xt, "0", monkeypatch)
    o2, v2 = _c12_run(net, xt, "2", monkeypatch)
    o1, v1 = _c12_run(net, xt, "1", monkeypatch)
    for v in (v1, v2):
        d = dict((name, rt.decode_variant(c)) for name, c in v)
        assert d["conv1_1"].get("var", 0) & 4 and d["conv1_2"].get("fused_into_prev"), (d["conv1_1"], d["conv1_2"])
    i12 = [name for name, _ in v1].index("conv1_2")
    assert v1[i12 + 1][0] == "maxpool2" and v1[i12 + 1][1] == -2 and v2[i12 + 1][1] != -2, (v1[i12 + 1], v2[i12 + 1])
    assert not rt.decode_variant(v1[i12 + 2][1]).get("vin"), v1[i12 + 2]
    assert not any(rt.decode_variant(v).get("var", 0) & 4 and not rt.decode_variant(v).get("rgb") for _, v in v0)
    for a, b, c in zip(o0, o1, o2):
        assert torch.equal(a, b) and torch.equal(a, c)
    ref = cpu_ref.make_net_fn(kind, wts)(x[:1])
    ref = ref if isinstance(ref, tuple) else (ref,)
    for a, r in zip(o1, ref):
        assert _rel(a[:1].cpu().numpy(), r) < TOL


@pytest.mark.parametrize("kind,n,h,w", [("body25", 32, 368, 656), ("hand", 32, 368, 368), ("hand", 32, 736, 736)])
def test_tail_tiles_bit_identical(kind, n, h, w, monkeypatch):
    """Tail tiles (conv_x3.hip x3_tail_plan: whole rounds of full 512-pixel tiles, then each
    frame's remaining pixels as tail tiles whose dead waves skip their MFMAs -- Mode N's 92x164
    layers, the hand's VGG layers at the C3 scales) == one tiling (ISLPOSE_X3_TAIL=0) bit for
    bit, and within the tolerance of the oracle on a frame."""
    code = {"body25": rt.ISL_BODY25, "hand": rt.ISL_HAND}[kind]
    wts = synth.synth_weights(code)
    net = rt.Net(code)
    net.load_weights(wts)
    x = _inputs(n, h, w, seed=h + n)
    xt = torch.from_numpy(x).cuda()
    outs = []
    for m in ("0", "1"):
        monkeypatch.setenv("ISLPOSE_X3_TAIL", m)
        o = net.forward(xt)
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (o if isinstance(o, tuple) else (o,))])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    ref = cpu_ref.make_net_fn(kind, wts)(x[n - 1:n])
    ref = ref if isinstance(ref, tuple) else (ref,)
    for a, r in zip(outs[1], ref):
        assert _rel(a[n - 1:n].cpu().numpy(), r) < TOL
