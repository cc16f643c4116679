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


@pytest.mark.parametrize("h,w,dense", [(256, 256, False), (200, 330, False), (192, 192, True), (260, 240, True)])
def test_hand_post_large_and_dense(hest, h, w, dense):
    """Planes above the LDS parent array (> 36864 px: the multi-block union-find
    pre-pass) and dense maps (random-weight-like: a few giant components, every pixel
    over the threshold) against the oracle, bit for bit."""
    n = 2
    geoms = [g[1:] for g in scale_geometry(h, w, HAND_SCALES)]
    rng = np.random.RandomState(h + w)
    heats, per = [], []
    for (nh, nw, vh, vw) in geoms:
        if dense:
            maps = [rng.uniform(0.02, 1.0, (22, nh // 8, nw // 8)).astype(np.float32) for _ in range(n)]
        else:
            maps = [synth.designed_hand_maps(nh // 8, nw // 8, seed=5 * i + nh, n_blobs=3) for i in range(n)]
        per.append(maps)
        heats.append(torch.from_numpy(np.stack(maps)).cuda())
    got = hest.post_maps(h, w, geoms, heats)
    for i in range(n):
        it = iter([per[s][i] for s in range(4)])
        ref = cpu_ref.hand_call(np.zeros((h, w, 3), np.uint8), lambda im: next(it)[None])
        assert np.array_equal(got[i], ref), i


@pytest.mark.parametrize("n", [1, 7, 8, 100, 128, 129, 1000, 8192, 8193, 16384 + 77, 50000, 360000])
def test_np_sum_association_bit_exact(n):
    """The device np.sum that ranks tied hand components (hand.py:68) against numpy's
    own np.sum, bit for bit, on values spread over 16 decades (where the association
    of the additions shows in the result): partial trees, full 8192-element buffers
    summed eight lanes per leaf, several buffers added left to right."""
    import ctypes
    from islpose import runtime as rt
    rng = np.random.RandomState(n)
    a = rng.standard_normal(n) * 10.0 ** rng.uniform(-8, 8, n)
    d = torch.from_numpy(a).cuda()
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    rt.check(rt.lib().isl_debug_np_sum(rt.ptr(d), n, rt.ptr(out), rt.stream_handle()), "isl_debug_np_sum")
    got = out.cpu().numpy()[0]
    assert got.tobytes() == np.sum(a).tobytes(), (n, got, np.sum(a), float(np.sum(a.astype(np.longdouble))))


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


def test_crop_preprocess_bit_exact(hest):
    """isl_net_preprocess_crops: each crop resized as its own image (borders replicated at
    the crop edge) == the oracle's net_input on the cut-out crop, bit for bit."""
    frames = synth.synth_frames(2, 120, 160, seed=17)
    t = torch.from_numpy(frames).cuda()
    boxes = [(0, 10, 5, 60), (1, 100, 60, 60), (0, 0, 0, 37), (1, 123, 83, 37)]
    for s in HAND_SCALES:
        same = [b for b in boxes if b[3] == 60]
        nh, nw = hest.net.preprocess_crops(t, [(f, x, y, w, w) for f, x, y, w in same], s * 368)
        got = hest.net.debug_input(len(same), nh, nw).cpu().numpy()
        for i, (f, x, y, w) in enumerate(same):
            ref, _, _ = cpu_ref.net_input(np.ascontiguousarray(frames[f, y:y + w, x:x + w]), s * 368 / w)
            assert ref.shape[2:] == (nh, nw)
            assert np.array_equal(got[i:i + 1], ref), (s, i)


def test_estimate_crops_matches_per_crop(hest):
    """Batched crops of different sizes (one batch per scale) == estimate() per crop."""
    frames = synth.synth_frames(3, 160, 200, seed=23)
    boxes = [(0, 20, 30, 96), (1, 0, 0, 40), (2, 104, 64, 96), (0, 150, 100, 50), (1, 33, 71, 77)]
    got = hest.estimate_crops(frames, boxes)
    assert got.shape == (5, 21, 2) and got.dtype == np.int64
    for (f, x, y, w), pk in zip(boxes, got):
        ref = hest.estimate(np.ascontiguousarray(frames[f, y:y + w, x:x + w]))
        assert np.array_equal(pk, ref), (f, x, y, w)
    assert hest.estimate_crops(frames, []).shape == (0, 21, 2)


def test_run_crops_concurrent_scales_bit_identical(hest):
    """run_crops forks all four scale streams before joining any, so the scales' nets run
    side by side on their own arenas; their maps equal each scale run alone on the current
    stream with the device drained in between, bit for bit (repeated: stream interleavings
    vary from call to call)."""
    from islpose.hand import BOXSIZE
    frames = torch.from_numpy(synth.synth_frames(2, 400, 600, seed=41)).cuda()
    boxes = [(0, 40, 30, 200), (1, 300, 150, 200)]
    crops = [(f, x, y, w, w) for f, x, y, w in boxes]
    alone = []
    for s in HAND_SCALES:
        gh, gw = hest.net.preprocess_crops(frames, crops, s * BOXSIZE)
        heat = torch.empty((len(crops), 22, gh // 8, gw // 8), device="cuda")
        hest.net.run(heat)
        torch.cuda.synchronize()
        alone.append(heat.clone())
    for _ in range(3):
        got = hest.run_crops(frames, boxes)
        torch.cuda.synchronize()
        for s, a, g in zip(HAND_SCALES, alone, got):
            assert torch.equal(a, g), s


def test_hand_net_split_k(hest):
    """A single crop at the 184/736 px scales (grids far below the CU count) in the
    latency mode (adaptive split-K on top of the canonical ranges): deterministic and
    within 1e-5 of the default net."""
    for s in (184, 736):
        x = torch.from_numpy(np.ascontiguousarray(
            np.transpose(synth.synth_frames(1, s, s, seed=s).astype(np.float32), (0, 3, 1, 2)) / 256 - 0.5)).cuda()
        h0 = hest.net.forward(x)
        hest.net.set_split_k(2)
        try:
            h1 = hest.net.forward(x)
            h2 = hest.net.forward(x)
        finally:
            hest.net.set_split_k(1)
        assert torch.equal(h1, h2)
        d = (h1 - h0).abs().max().item() / max(h0.abs().max().item(), 1e-30)
        assert d < 1e-5, d


@pytest.mark.parametrize("side", [184, 368, 552, 736])
def test_small7_half_channel_bit_identical(hest, side, monkeypatch):
    """A frame's single hand crop (the per-frame call of the reference scripts): the 7x7 stage
    layers' grids are under one 128-pixel block per CU, so they run as 64-channel blocks on
    64-pixel tiles with their operands two steps ahead (conv_x3.hip x3_small7, VAR 256 | 128;
    the 23^2 scale with its across-block K ranges) == the same blocks one step ahead
    (ISLPOSE_X3_SMALL7=1) == the 128-pixel blocks (=0) bit for bit, and the crop alone == the
    crop inside a batch of 8.  (92^2: 266 64-pixel blocks, past one round: 96-pixel tiles two
    steps ahead, 178 blocks, x3_small7_96; ISLPOSE_X3_S7W96=0 gives the 64-pixel blocks one
    step ahead, the same bits.)"""
    from islpose import runtime as rt
    x = torch.from_numpy(np.ascontiguousarray(
        np.transpose(synth.synth_frames(8, side, side, seed=side + 1).astype(np.float32), (0, 3, 1, 2)) / 256 - 0.5)).cuda()
    monkeypatch.delenv("ISLPOSE_X3_SMALL7", raising=False)
    h1 = hest.net.forward(x[:1]).clone()
    var = [rt.decode_variant(v) for name, v in hest.net.op_variants()
           if name.startswith("Mconv") and "Mconv6" not in name and "Mconv7" not in name]
    want_bpx = 96 if side == 736 else 64
    assert len(var) == 25 and all(d["ks"] == 7 and d["var"] & 256 and d["bpx"] == want_bpx for d in var), var[:2]
    # operands two steps ahead where the grid fits one block per CU (x3_small7_deep / _96)
    assert all(d["var"] & 128 for d in var), var[:2]
    h8 = hest.net.forward(x).clone()
    monkeypatch.setenv("ISLPOSE_X3_S7W96", "0")
    h64 = hest.net.forward(x[:1]).clone()
    monkeypatch.delenv("ISLPOSE_X3_S7W96")
    monkeypatch.setenv("ISLPOSE_X3_SMALL7", "1")
    hs = hest.net.forward(x[:1]).clone()
    monkeypatch.setenv("ISLPOSE_X3_SMALL7", "0")
    h0 = hest.net.forward(x[:1]).clone()
    torch.cuda.synchronize()
    assert torch.equal(h1, h0) and torch.equal(h1, hs) and torch.equal(h1, h64)
    assert torch.equal(h1[0], h8[0])


def test_arena_bounded_over_crop_counts():
    """estimate_crops with a different crop count per batch keeps one arena
    per hand scale, sized by the largest count seen -- not one per (count, scale)."""
    from islpose import runtime as rt
    est = HandEstimator(synth.synth_weights(2))
    frames = synth.synth_frames(2, 160, 200, seed=29)
    counts = [3, 1, 5, 2, 4, 5, 1]
    for c in counts:
        boxes = [(i % 2, 10 + 7 * i, 5 + 3 * i, 60) for i in range(c)]
        est.estimate_crops(frames, boxes)
    used, n = est.net.arena_info()
    assert n == len(HAND_SCALES), n
    ref = HandEstimator(net=rt.Net(rt.ISL_HAND))
    ref.net.load_weights(synth.synth_weights(2))
    ref.estimate_crops(frames, [(i % 2, 10 + 7 * i, 5 + 3 * i, 60) for i in range(max(counts))])
    assert used == ref.net.arena_info()[0]


def _x3_7x7_bpx(n, side):
    """conv_x3.hip x3_7x7_bpx for the hand's 7x7 stage layers (128 outputs, input ring 3) on
    a side x side level-3 grid at batch n: canonical K ranges (<= 1024 pixels) keep 128-pixel
    tiles, else the tile with the fewest rounds of one block per CU, a round of 256- / 384-
    pixel blocks costing 1.52 / 2.38 rounds of 128 (ties keep the smaller tile)."""
    if side * side <= 1024:
        return 128

    def tile_pixels(bpx):
        for t in range(bpx, 1, -1):
            if t - 1 + 2 * 3 * ((side + t - 2) // side) + 2 * 3 + 1 <= bpx + 64:
                return t
        return 1
    best, best_t = 128, None
    for bpx, cost in ((128, 1.0), (256, 1.52), (384, 2.38)):
        blocks = n * -(-side * side // tile_pixels(bpx))
        tt = -(-blocks // 256) * cost
        if best_t is None or tt < best_t:
            best, best_t = bpx, tt
    return best


def test_c3_crop_batch_vs_oracle():
    """configs[2] (C3) at its own batch: 16 frames of 368x656 with 2 hand crops each (120-200
    px, as tools/bench_configs.py c3), 32 crops per scale through the batched hand net at all
    four scales (reference src/hand.py:25-56 per crop).  Crops 0, 15 and 31: maps within 1e-4 of
    the oracle's net on the oracle's own crop input, peaks bit-exact with the oracle's post on
    those maps; the 7x7 tile size every scale ran (isl_net_op_info) is the grid-quantisation
    choice for 32 crops."""
    from islpose import runtime as rt
    B, H, W = 16, 368, 656
    frames = synth.synth_frames(B, H, W, seed=5)
    rng = np.random.RandomState(0)
    boxes = []
    for f in range(B):
        for _ in range(2):
            w = int(rng.randint(120, 201))
            boxes.append((f, int(rng.randint(0, W - w)), int(rng.randint(0, H - w)), w))
    wh = synth.synth_weights(2)
    net = rt.Net(rt.ISL_HAND)
    net.load_weights(wh)
    t = torch.from_numpy(frames).cuda()
    heats = []
    for s in HAND_SCALES:
        one = HandEstimator(net=net, scale_search=(s,))
        heats += one.run_crops(t, boxes)
        torch.cuda.synchronize()
        side = int(round(s * 368)) // 8
        want = _x3_7x7_bpx(len(boxes), side)
        var = [rt.decode_variant(v) for name, v in net.op_variants() if name.startswith("Mconv") and "Mconv6" not in name
               and "Mconv7" not in name]
        assert len(var) == 25 and all(d["ks"] == 7 and d["bpx"] == want for d in var), (s, want, var[:2])
    peaks = HandEstimator(net=net).post_crops(boxes, heats)
    fn = cpu_ref.make_net_fn("hand", wh)
    for i in (0, 15, 31):
        f, x, y, w = boxes[i]
        crop = np.ascontiguousarray(frames[f, y:y + w, x:x + w])
        for si, s in enumerate(HAND_SCALES):
            im, _, _ = cpu_ref.net_input(crop, s * 368 / w)
            ref = fn(im)
            ref = ref[0] if isinstance(ref, tuple) else ref
            got = heats[si][i:i + 1].cpu().numpy()
            assert got.shape == ref.shape, (i, s)
            d = float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-30))
            assert d < 1e-4, (i, s, d)
        maps = iter([h[i].cpu().numpy() for h in heats])
        assert np.array_equal(peaks[i], cpu_ref.hand_call(crop, lambda im: next(maps)[None])), i
