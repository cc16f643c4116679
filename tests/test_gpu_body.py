"""Parity of the HIP path (libislpose.so) against the CPU oracle and the golden
vectors.  Runs on an MI355X only (-m gpu)."""
import os

import numpy as np
import pytest
import torch

from oracle import cpu_ref
from islpose import synth
from islpose import runtime as rt
from islpose.body import BodyEstimator, scale_geometry

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-4   # north_star: heatmap/PAF tensors within 1e-4 relative (max|d| / max|ref|) in fp32


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.fixture(scope="module")
def w25():
    return synth.synth_weights(0)


@pytest.fixture(scope="module")
def net25(w25):
    n = rt.Net(rt.ISL_BODY25)
    n.load_weights(w25)
    return n


def _inputs(n, h, w, seed):
    f = synth.synth_frames(n, h, w, seed=seed)
    return np.ascontiguousarray(np.transpose(f.astype(np.float32), (0, 3, 1, 2)) / 256 - 0.5)


@pytest.mark.parametrize("n,h,w", [(1, 50, 70), (2, 184, 328), (1, 368, 656)])
def test_body25_forward_vs_oracle(net25, w25, n, h, w):
    x = _inputs(n, h, w, seed=h + w)
    paf, heat = net25.forward(torch.from_numpy(x).cuda())
    torch.cuda.synchronize()
    rp, rh = cpu_ref.make_net_fn("body25", w25)(x)
    assert paf.shape == rp.shape and heat.shape == rh.shape
    assert _rel(paf.cpu().numpy(), rp) < TOL
    assert _rel(heat.cpu().numpy(), rh) < TOL


@pytest.mark.parametrize("algo", ["x3", "direct", "wino"])
def test_body25_forward_algo_vs_oracle(net25, w25, algo):
    """Every conv arithmetic (split-fp16 x3, direct fp32 implicit GEMM, Winograd
    F(2x2,3x3)) against the oracle; 2 x 184x328 puts odd sizes (23x41) on the stage layers."""
    x = _inputs(2, 184, 328, seed=77)
    with net25.algo_scope(algo):
        paf, heat = net25.forward(torch.from_numpy(x).cuda())
    torch.cuda.synchronize()
    rp, rh = cpu_ref.make_net_fn("body25", w25)(x)
    ep, eh = _rel(paf.cpu().numpy(), rp), _rel(heat.cpu().numpy(), rh)
    print("algo %s: rel err paf %.3g heat %.3g" % (algo, ep, eh))
    assert ep < TOL and eh < TOL, (ep, eh)


@pytest.mark.parametrize("n,h,w", [(2, 184, 328), (1, 368, 656), (2, 50, 70), (3, 96, 136), (8, 368, 656),
                                   (16, 184, 328), (8, 372, 656), (4, 100, 104)])
def test_fused_pool_bit_identical(net25, n, h, w, monkeypatch):
    """conv1_2 / conv2_2 / conv3_4 writing horizontal pair maxima (ConvLaunch::hpool) +
    the row-pair max inside the next conv's staging (ConvLaunch::vin, on chip-filling
    grids: 8 x 368x656 takes it after all three pools, 16 x 184x328 after two and
    vpool2_kernel for the third) or in vpool2_kernel (ISLPOSE_POOL_INPUT=0) == conv +
    maxpool2, bit for bit (max is exact); odd widths (50x70's 25x35 level) take the plain
    path.  8 x 372x656 and 4 x 100x104 have an odd pre-pool height (93 / 25 rows before
    pool3) with an even width: that pool must not hand its pair-max buffer to the next
    conv's staging, whose chunk stride assumes 2H rows."""
    x = torch.from_numpy(_inputs(n, h, w, seed=h + w)).cuda()
    paf0, heat0 = net25.forward(x)
    monkeypatch.setenv("ISLPOSE_POOL_INPUT", "0")
    paf2, heat2 = net25.forward(x)
    monkeypatch.setenv("ISLPOSE_FUSED_POOL", "0")
    paf1, heat1 = net25.forward(x)
    torch.cuda.synchronize()
    assert torch.equal(paf0, paf1) and torch.equal(heat0, heat1)
    assert torch.equal(paf2, paf1) and torch.equal(heat2, heat1)


@pytest.mark.parametrize("n,h,w", [(2, 184, 328), (1, 50, 70)])
def test_rgb_first_layer_kernel(net25, w25, n, h, w, monkeypatch):
    """conv1_1 through conv_x3_rgb (K = the 27 real (ky, kx, c) products) against the
    generic split-fp16 kernel (ISLPOSE_RGB_CONV=0) and the oracle: the same fp32-accurate
    sums in another order, so within 1e-5 of each other and the 1e-4 bar vs the oracle."""
    x = _inputs(n, h, w, seed=5 * h + w)
    xt = torch.from_numpy(x).cuda()
    paf1, heat1 = net25.forward(xt)
    monkeypatch.setenv("ISLPOSE_RGB_CONV", "0")
    paf0, heat0 = net25.forward(xt)
    torch.cuda.synchronize()
    assert _rel(paf1.cpu().numpy(), paf0.cpu().numpy()) < 1e-5
    assert _rel(heat1.cpu().numpy(), heat0.cpu().numpy()) < 1e-5
    rp, rh = cpu_ref.make_net_fn("body25", w25)(x)
    assert _rel(paf1.cpu().numpy(), rp) < TOL and _rel(heat1.cpu().numpy(), rh) < TOL


def test_body25_forward_lds_dma_staging(net25, w25, monkeypatch):
    """The LDS-DMA staging variant of the conv kernel gives the same results."""
    x = torch.from_numpy(_inputs(2, 50, 70, seed=9)).cuda()
    with net25.algo_scope("direct"):
        paf0, heat0 = net25.forward(x)
        monkeypatch.setenv("ISLPOSE_CONV_STAGING", "glds")
        paf1, heat1 = net25.forward(x)
    torch.cuda.synchronize()
    assert torch.equal(paf0, paf1) and torch.equal(heat0, heat1)


def test_body25_forward_golden(net25):
    g1 = np.load(os.path.join(GOLDEN, "g1_networks.npz"))
    x = _inputs(1, 184, 328, int(g1["body25_184x328_seed"]))
    paf, heat = net25.forward(torch.from_numpy(x).cuda())
    assert _rel(paf.cpu().numpy(), g1["body25_184x328_paf"]) < TOL
    assert _rel(heat.cpu().numpy(), g1["body25_184x328_heat"]) < TOL


def test_coco_forward_golden():
    g1 = np.load(os.path.join(GOLDEN, "g1_networks.npz"))
    net = rt.Net(rt.ISL_COCO)
    net.load_weights(synth.synth_weights(1))
    ski = np.load(os.path.join(GOLDEN, "ski_bgr.npz"))["img"]
    im, _, _ = cpu_ref.net_input(ski, 0.5 * 368 / ski.shape[0])
    paf, heat = net.forward(torch.from_numpy(im).cuda())
    assert _rel(paf.cpu().numpy(), g1["coco_ski_paf"]) < TOL
    assert _rel(heat.cpu().numpy(), g1["coco_ski_heat"]) < TOL


def test_hand_forward_golden():
    g1 = np.load(os.path.join(GOLDEN, "g1_networks.npz"))
    net = rt.Net(rt.ISL_HAND)
    net.load_weights(synth.synth_weights(2))
    for s in (184, 368):
        x = _inputs(1, s, s, int(g1["hand_%d_seed" % s]))
        out = net.forward(torch.from_numpy(x).cuda())
        assert _rel(out.cpu().numpy(), g1["hand_%d" % s]) < TOL


@pytest.mark.parametrize("H,W,scale", [(368, 656, 0.5), (368, 656, 1.0), (300, 500, 368 / 300 * 0.5),
                                       (97, 131, 1.7), (674, 712, 0.5 * 368 / 674)])
def test_preprocess_bit_exact(net25, H, W, scale):
    frames = synth.synth_frames(2, H, W, seed=7)
    nh, nw = net25.preprocess(torch.from_numpy(frames).cuda(), scale)
    got = net25.debug_input(2, nh, nw).cpu().numpy()
    for i in range(2):
        ref, _, _ = cpu_ref.net_input(frames[i], scale)
        assert ref.shape[2:] == (nh, nw)
        assert np.array_equal(got[i:i + 1], ref)


def _golden_cases():
    z = np.load(os.path.join(GOLDEN, "g2_body_post.npz"))
    return z, sorted({k.split("/")[0] for k in z.files})


@pytest.fixture(scope="module")
def est25(w25):
    return BodyEstimator(w25, "body25")


@pytest.fixture(scope="module")
def estcoco():
    return BodyEstimator(synth.synth_weights(1), "coco")


@pytest.mark.parametrize("kind,persons,drop", [("body25", 3, ()), ("body25", 80, ()), ("coco", 40, (12,)),
                                               ("coco", 70, (12,))])
def test_assemble_register_merge_equals_table(est25, estcoco, monkeypatch, kind, persons, drop):
    """Person assembly with the subset rows in lane registers (the default) == the table merge
    (ISLPOSE_ASM_REG=0) == the oracle (body.py:164-232).  368 x 4096 frames (46 x 512 low-res)
    with up to 80 designed persons: more than 64 subset rows spill the registers to the table
    mid-merge; COCO with the neck -> nose limb dropped makes every head its own row until the ear
    limbs merge it into its body (the found == 2 branch and its row delete)."""
    est = est25 if kind == "body25" else estcoco
    H, W = 368, 4096
    geoms = [g[1:] for g in scale_geometry(H, W, (1.0,))]
    nh, nw = geoms[0][0] // 8, geoms[0][1] // 8
    ms = [synth.designed_pose_maps(nh, nw, persons, seed=300 + i, model_type=kind, drop_limbs=drop) for i in range(2)]
    pafs = [torch.from_numpy(np.stack([m[0] for m in ms])).cuda()]
    heats = [torch.from_numpy(np.stack([m[1] for m in ms])).cuda()]
    monkeypatch.delenv("ISLPOSE_ASM_REG", raising=False)
    got = est.post_maps(H, W, geoms, pafs, heats)
    monkeypatch.setenv("ISLPOSE_ASM_REG", "0")
    ref = est.post_maps(H, W, geoms, pafs, heats)
    for a, b in zip(got, ref):
        assert np.array_equal(a.candidate, b.candidate) and np.array_equal(a.subset, b.subset)
    if persons > 64:
        assert len(got[0].subset) > 64
    heat_avg, paf_avg = cpu_ref.body_maps(np.zeros((H, W, 3), np.uint8), lambda im: (ms[0][0][None], ms[0][1][None]),
                                          kind, (1.0,))
    cand, subset, _, _ = cpu_ref.body_post(heat_avg, paf_avg, kind, H)
    assert np.array_equal(got[0].candidate, cand) and np.array_equal(got[0].subset, subset)


@pytest.mark.parametrize("H,W,scale,persons", [(368, 4096, 1.0, 20), (368, 4096, 1.0, 45), (1080, 1920, 0.5, 16)])
def test_limb_large_pair_sets(est25, monkeypatch, H, W, scale, persons):
    """Limbs with more than LIMB_ITEMS / 10 candidate pairs (body.py:142-175; hundreds per limb on
    crowded or noisy frames, e.g. 1080p frames through the two-stage resize): the chunked scoring
    with the rank sort and the greedy in LDS (default) == the per-thread pair loop
    (ISLPOSE_LIMB_LDS=0), with the scoring spread over blocks (small batches, the default) and in
    the limb's own block (ISLPOSE_LIMB_SPLIT=0) == the oracle, connections included."""
    geoms = [g[1:] for g in scale_geometry(H, W, (scale,))]
    nh, nw = geoms[0][0] // 8, geoms[0][1] // 8
    ms = [synth.designed_pose_maps(nh, nw, persons, seed=500 + persons + i) for i in range(2)]
    pafs = [torch.from_numpy(np.stack([m[0] for m in ms])).cuda()]
    heats = [torch.from_numpy(np.stack([m[1] for m in ms])).cuda()]
    monkeypatch.delenv("ISLPOSE_LIMB_LDS", raising=False)
    monkeypatch.delenv("ISLPOSE_LIMB_SPLIT", raising=False)
    got = est25.post_maps(H, W, geoms, pafs, heats)
    refs = []
    for lds, split in (("0", "1"), ("1", "0"), ("0", "0")):
        monkeypatch.setenv("ISLPOSE_LIMB_LDS", lds)
        monkeypatch.setenv("ISLPOSE_LIMB_SPLIT", split)
        refs.append(est25.post_maps(H, W, geoms, pafs, heats))
    for ref in refs:
        for a, b in zip(got, ref):
            assert np.array_equal(a.candidate, b.candidate) and np.array_equal(a.subset, b.subset)
            for x, y in zip(a.connection_all, b.connection_all):
                assert np.array_equal(np.asarray(x).reshape(-1, 5), np.asarray(y).reshape(-1, 5))
    heat_avg, paf_avg = cpu_ref.body_maps(np.zeros((H, W, 3), np.uint8), lambda im: (ms[0][0][None], ms[0][1][None]),
                                          "body25", (scale,))
    cand, subset, peaks, conn = cpu_ref.body_post(heat_avg, paf_avg, "body25", H)
    assert max(len(p) for p in peaks) ** 2 > 204     # some limb takes the large-pair path
    assert np.array_equal(got[0].candidate, cand) and np.array_equal(got[0].subset, subset)
    for x, y in zip(got[0].connection_all, conn):
        assert np.array_equal(np.asarray(x).reshape(-1, 5), np.asarray(y).reshape(-1, 5))


def test_body_post_golden_bit_exact(est25, estcoco):
    """Designed low-res maps replayed through the GPU post kernels == reference Body.__call__."""
    z, names = _golden_cases()
    for name in names:
        mt = str(z[name + "/model_type"])
        est = est25 if mt == "body25" else estcoco
        H, W = (int(v) for v in z[name + "/frame_hw"])
        scales = tuple(float(s) for s in z[name + "/scales"])
        geoms = [g[1:] for g in scale_geometry(H, W, scales)]
        pafs = [torch.from_numpy(z[name + "/paf%d" % i][None]).cuda() for i in range(len(scales))]
        heats = [torch.from_numpy(z[name + "/heat%d" % i][None]).cuda() for i in range(len(scales))]
        r = est.post_maps(H, W, geoms, pafs, heats)[0]
        assert r.candidate.shape == z[name + "/candidate"].shape, name
        assert np.array_equal(r.candidate, z[name + "/candidate"]), name
        assert np.array_equal(r.subset, z[name + "/subset"]), name


def test_body_estimate_end_to_end(est25, w25):
    """Frames -> GPU pre-proc + net + post; the GPU's own low-res maps replayed through
    the oracle post must give identical candidate / subset / connections."""
    frames = synth.synth_frames(2, 368, 656, seed=3)
    t = torch.from_numpy(frames).cuda()
    geoms, pafs, heats = est25.run_scales(t, keep_maps=True)
    res = est25.post_maps(368, 656, geoms, pafs, heats)
    for i in range(2):
        pl, hl = pafs[0][i].cpu().numpy(), heats[0][i].cpu().numpy()
        heat_avg, paf_avg = cpu_ref.body_maps(frames[i], lambda im: (pl[None], hl[None]), "body25", (0.5,))
        cand, subset, all_peaks, conn = cpu_ref.body_post(heat_avg, paf_avg, "body25", 368)
        assert np.array_equal(res[i].candidate, cand)
        assert np.array_equal(res[i].subset, subset)
        for a, b in zip(res[i].connection_all, conn):
            assert np.array_equal(np.asarray(a).reshape(-1, 5), np.asarray(b).reshape(-1, 5))
    # and the net outputs themselves are within tolerance of the oracle network
    for i in range(2):
        im, _, _ = cpu_ref.net_input(frames[i], 0.5)
        rp, rh = cpu_ref.make_net_fn("body25", w25)(im)
        assert _rel(pafs[0][i:i + 1].cpu().numpy(), rp) < TOL
        assert _rel(heats[0][i:i + 1].cpu().numpy(), rh) < TOL


def test_launch_post_stream_equals_estimate(est25):
    """BodyEstimator.launch(post_stream=...): the nets of three batches run back to back on
    the current stream while each batch's post and records' copy run on a post stream beside
    the next batch's nets (the maps in tensors of the batch, the range check on the net's
    stream); finish() of each gives exactly estimate()'s candidate / subset, capacity re-runs
    included (random-weight maps are dense)."""
    ps = torch.cuda.Stream()
    batches = [torch.from_numpy(synth.synth_frames(2, 368, 656, seed=40 + k)).cuda() for k in range(3)]
    jobs = [est25.launch(b, post_stream=ps) for b in batches]
    got = [est25.finish(j) for j in jobs]
    for b, g in zip(batches, got):
        ref = est25.estimate(b)
        for (c0, s0), (c1, s1) in zip(ref, g):
            assert np.array_equal(c0, c1) and np.array_equal(s0, s1)


def test_designed_maps_batch_bit_exact(est25):
    """A batch of designed maps (P = 0..6 persons) through the GPU post == oracle post."""
    H, W = 368, 656
    geoms = [g[1:] for g in scale_geometry(H, W, (1.0,))]
    maps = [synth.designed_pose_maps(46, 82, p, 100 + p) for p in range(7)]
    paf = torch.from_numpy(np.stack([m[0] for m in maps])).cuda()
    heat = torch.from_numpy(np.stack([m[1] for m in maps])).cuda()
    res = est25.post_maps(H, W, geoms, [paf], [heat])
    for i, (pl, hl) in enumerate(maps):
        heat_avg, paf_avg = cpu_ref.body_maps(np.zeros((H, W, 3), np.uint8), lambda im: (pl[None], hl[None]),
                                              "body25", (1.0,))
        cand, subset, _, _ = cpu_ref.body_post(heat_avg, paf_avg, "body25", H)
        assert np.array_equal(res[i].candidate, cand), i
        assert np.array_equal(res[i].subset, subset), i
        assert len(subset) == i, i


@pytest.mark.parametrize("H,W", [(368, 656), (368, 131), (368, 45)])
def test_fused_resize_blur_matches_unfused(est25, monkeypatch, H, W):
    """Single-scale post with the resize fused into blur_nms (no full-res planes, exact
    early-out of dead tiles) == the two-kernel path == the oracle, on maps with noise
    just around the 0.1 threshold (many live and borderline tiles) and odd sizes."""
    geoms = [g[1:] for g in scale_geometry(H, W, (1.0,))]
    nh, nw = geoms[0][0] // 8, geoms[0][1] // 8
    rng = np.random.RandomState(H)
    maps = [synth.designed_pose_maps(nh, nw, p, 200 + p) for p in (1, 2, 3)]
    heat_np = np.stack([m[1] for m in maps])
    noise = rng.uniform(0.0, 0.16, heat_np.shape).astype(np.float32) * (rng.rand(*heat_np.shape) < 0.15)
    heat_np = heat_np + noise
    paf = torch.from_numpy(np.stack([m[0] for m in maps])).cuda()
    heat = torch.from_numpy(heat_np).cuda()
    monkeypatch.setenv("ISLPOSE_FUSED_BLUR", "1")
    fused = est25.post_maps(H, W, geoms, [paf], [heat])
    monkeypatch.setenv("ISLPOSE_FUSED_BLUR", "0")
    plain = est25.post_maps(H, W, geoms, [paf], [heat])
    for i in range(len(maps)):
        assert np.array_equal(fused[i].candidate, plain[i].candidate), i
        assert np.array_equal(fused[i].subset, plain[i].subset), i
        hl, pl = heat_np[i], maps[i][0]
        heat_avg, paf_avg = cpu_ref.body_maps(np.zeros((H, W, 3), np.uint8), lambda im: (pl[None], hl[None]),
                                              "body25", (1.0,))
        cand, subset, _, _ = cpu_ref.body_post(heat_avg, paf_avg, "body25", H)
        assert np.array_equal(fused[i].candidate, cand), i
        assert np.array_equal(fused[i].subset, subset), i


@pytest.mark.parametrize("H,W", [(1000, 1000), (1080, 1920), (368, 656), (400, 520)])
def test_fused_two_stage_post_matches_unfused(est25, monkeypatch, H, W):
    """Mode R (scale 0.5: net 184 px tall, then the second resize: >5x on large frames, the
    small LDS window; ~2x at 368 x 656 / 400 x 520, the wide window): the second resize fused
    into blur_nms (no full-resolution planes) == the materialised two-kernel path == the
    oracle, on noisy maps around the 0.1 threshold.  (The wide window for the ~2x stage-2
    scales measured slower than the materialised planes and lives in the development build
    only, so 368 x 656 / 400 x 520 check the materialised path against the oracle.)"""
    geoms = [g[1:] for g in scale_geometry(H, W, (0.5,))]
    nh, nw = geoms[0][0] // 8, geoms[0][1] // 8
    rng = np.random.RandomState(H + W)
    pl, hl = synth.designed_pose_maps(nh, nw, 2, 300)
    hl = hl + (rng.uniform(0.0, 0.16, hl.shape) * (rng.rand(*hl.shape) < 0.15)).astype(np.float32)
    paf, heat = torch.from_numpy(pl[None]).cuda(), torch.from_numpy(hl[None]).cuda()
    monkeypatch.setenv("ISLPOSE_FUSED_BLUR", "1")
    fused = est25.post_maps(H, W, geoms, [paf], [heat])[0]
    monkeypatch.setenv("ISLPOSE_FUSED_BLUR", "0")
    plain = est25.post_maps(H, W, geoms, [paf], [heat])[0]
    assert np.array_equal(fused.candidate, plain.candidate) and np.array_equal(fused.subset, plain.subset)
    heat_avg, paf_avg = cpu_ref.body_maps(np.zeros((H, W, 3), np.uint8), lambda im: (pl[None], hl[None]),
                                          "body25", (0.5,))
    cand, subset, _, _ = cpu_ref.body_post(heat_avg, paf_avg, "body25", H)
    assert np.array_equal(fused.candidate, cand) and np.array_equal(fused.subset, subset)
    assert len(cand) > 0


def test_fused_post_reads_the_arena(est25, monkeypatch):
    """Mode N estimate (scale 1.0: the fused resize + blur) reading the net's own arena
    output == the same maps handed over as caller tensors == the unfused kernels."""
    from islpose.body import BodyEstimator
    est = BodyEstimator(model_type="body25", scale_search=(1.0,), net=est25.net)
    frames = torch.from_numpy(synth.synth_frames(2, 368, 200, seed=21)).cuda()
    arena = est.estimate(frames, details=True)
    geoms, pafs, heats = est.run_scales(frames, keep_maps=True)
    caller = est.post_maps(368, 200, geoms, pafs, heats)
    monkeypatch.setenv("ISLPOSE_FUSED_BLUR", "0")
    plain = est.post_maps(368, 200, geoms, pafs, heats)
    for a, b, c in zip(arena, caller, plain):
        assert np.array_equal(a.candidate, b.candidate) and np.array_equal(a.subset, b.subset)
        assert np.array_equal(a.candidate, c.candidate) and np.array_equal(a.subset, c.subset)


def test_x3_range_guard_falls_back_to_fp32(w25):
    """Activations beyond the fp16 split range (|x| >= 65504) raise the net's range
    flag; Net.forward then recomputes on the fp32 kernels, so the result still
    matches the oracle, and the net keeps its split-fp16 default afterwards."""
    w = dict(w25)
    w["conv1_1.weight"] = w["conv1_1.weight"] * np.float32(2.0 ** 20)   # conv1_1 outputs ~1e5-1e6
    w["conv1_1.bias"] = w["conv1_1.bias"] * np.float32(2.0 ** 20)
    net = rt.Net(rt.ISL_BODY25)
    net.load_weights(w)
    assert net.algo == "x3"
    x = _inputs(1, 64, 96, seed=21)
    xt = torch.from_numpy(x).cuda()
    o0 = torch.empty((1, 52, 8, 12), device="cuda")
    o1 = torch.empty((1, 26, 8, 12), device="cuda")
    rt.check(rt.lib().isl_net_forward(net.h, rt.ptr(xt), 1, 64, 96, rt.ptr(o0), rt.ptr(o1), rt.stream_handle()))
    assert not net.range_ok()             # raw x3 run flagged
    assert net.range_ok()                 # and the flag was cleared
    paf, heat = net.forward(xt)           # guarded seam: falls back
    rp, rh = cpu_ref.make_net_fn("body25", w)(x)
    assert _rel(paf.cpu().numpy(), rp) < TOL and _rel(heat.cpu().numpy(), rh) < TOL
    assert net.algo == "x3"


@pytest.mark.parametrize("n,h,w", [(1, 184, 328), (1, 368, 656), (2, 92, 164)])
def test_x3_splitk_small_grids(net25, w25, n, h, w):
    """K-range modes on small grids: 1 (default, canonical ranges on the <= 1024-pixel
    layers, split across blocks at this batch), 2 (latency: also an adaptive split of
    the other small grids) and 0 (no ranges) are each deterministic and within 1e-5
    of each other and within the tolerance of the oracle."""
    x = torch.from_numpy(_inputs(n, h, w, seed=n * h + w)).cuda()
    outs = {}
    try:
        for mode in (0, 2, 1):
            net25.set_split_k(mode)
            a = net25.forward(x)
            b = net25.forward(x)
            assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), mode
            outs[mode] = [t.cpu().numpy() for t in a]
    finally:
        net25.set_split_k(1)
    for mode in (1, 2):
        assert _rel(outs[mode][0], outs[0][0]) < 1e-5 and _rel(outs[mode][1], outs[0][1]) < 1e-5, mode
    if h <= 184:
        rp, rh = cpu_ref.make_net_fn("body25", w25)(x.cpu().numpy())
        for mode in (0, 1, 2):
            assert _rel(outs[mode][0], rp) < TOL and _rel(outs[mode][1], rh) < TOL, mode


def test_canonical_ranges_batch_invariant(net25):
    """Default mode: a Mode R frame (net 184x328: 23x41 stages with canonical K ranges)
    gives the same bits alone (ranges split across blocks) and inside a batch of 20
    (ranges summed in one block) -- the per-frame callers' fast path does not change
    the maps of batched runs."""
    x = torch.from_numpy(_inputs(20, 184, 328, seed=5)).cuda()
    pb, hb = net25.forward(x)
    for i in (0, 7, 19):
        p1, h1 = net25.forward(x[i:i + 1].contiguous())
        assert torch.equal(p1, pb[i:i + 1]) and torch.equal(h1, hb[i:i + 1]), i


def test_x3_matches_direct_small_shapes(net25):
    """Split-fp16 vs fp32 direct on awkward shapes (narrow images, one-row tiles,
    odd chunk counts) -- both within the tolerance of each other."""
    for (n, h, w) in [(1, 16, 200), (3, 40, 16), (1, 64, 24), (1, 8, 8)]:
        x = torch.from_numpy(_inputs(n, h, w, seed=h * w)).cuda()
        with net25.algo_scope("direct"):
            p0, h0 = net25.forward(x)
        p1, h1 = net25.forward(x)
        assert _rel(p1.cpu().numpy(), p0.cpu().numpy()) < TOL
        assert _rel(h1.cpu().numpy(), h0.cpu().numpy()) < TOL


def test_timed_config_forward_vs_oracle(net25, w25):
    """The bench's own configuration (configs[1]: body_25, 32 frames of 368x656, net input
    368x656; reference src/model.py:171-207) checked against the oracle on frames 0, 17 and
    31, with the kernel variants the bench times asserted through isl_net_op_info: the
    46x82 stage 3x3 layers on the 512-pixel row union, conv2_1 / conv3_1 / conv4_1 staging
    their pooled input (the pools folded away), every Mconv6 -> Mconv7 pair fused into
    one launch (VAR 16), conv1_1 -> conv1_2 -> pool1 in one launch (conv_c12.hip)."""
    n, h, w = 32, 368, 656
    x = _inputs(n, h, w, seed=2024)
    paf, heat = net25.forward(torch.from_numpy(x).cuda())
    torch.cuda.synchronize()
    var = {name: rt.decode_variant(v) for name, v in net25.op_variants()}
    stage3 = [k for k in var if k.startswith("Mconv") and k[5] in "12345"]
    assert len(stage3) == 90
    # the first conv of blocks 2-5 of the 128-wide stages reads 384 channels: the split-fp16
    # Winograd kernel (wino_f16, the default for >= 256 input channels); the rest the row union
    w2 = [k for k in stage3 if var[k].get("wino2")]
    assert sorted(w2) == sorted(k for k in stage3 if k[5] in "2345" and k.endswith("_0") and "stage0" not in k), w2
    for k in stage3:
        if k not in w2:
            assert var[k].get("union") and var[k]["bpx"] == 512, (k, var[k])
    for k in ("conv3_2", "conv3_3", "conv4_2", "conv4_3_CPM", "conv4_4_CPM"):
        assert var[k].get("wino2"), (k, var[k])
    for k in ("conv3_1", "conv4_1"):
        assert var[k].get("vin"), (k, var[k])
    assert var["conv2_1"]["bpx"] == 512 and not var["conv2_1"].get("vin"), var["conv2_1"]   # pool1 in conv_c12
    assert var["conv4_1"].get("union"), var["conv4_1"]   # (pooled input: not eligible for wino_f16)
    m6 = [k for k in var if k.startswith("Mconv6")]
    assert len(m6) == 6 and all(var[k].get("fused67") and var[k]["bco"] in (256, 512) for k in m6), m6
    assert all(var[k].get("fused_into_prev") for k in var if k.startswith("Mconv7"))
    assert var["conv1_1"].get("c12") and var["conv1_2"].get("fused_into_prev")   # conv_c12.hip
    ops = net25.op_variants()
    i12 = [name for name, _ in ops].index("conv1_2")
    assert ops[i12 + 1][0] == "maxpool2" and ops[i12 + 1][1] == -2, ops[i12 + 1]   # ... with pool1
    assert sum(1 for _, v in net25.op_variants() if v == -1) == 2      # the other two pools folded
    fn = cpu_ref.make_net_fn("body25", w25)
    for f in (0, 17, 31):
        rp, rh = fn(x[f:f + 1])
        ep = _rel(paf[f:f + 1].cpu().numpy(), rp)
        eh = _rel(heat[f:f + 1].cpu().numpy(), rh)
        assert ep < TOL and eh < TOL, (f, ep, eh)


def test_colliding_pyramid_scales_serialised(w25):
    """Two pyramid scales that pad to the same net size (0.505 and 0.51 -> 192 x 336) share
    the net's arena for that size; run_scales must run them in order on one stream (ADVICE
    r02).  Each scale's maps must equal the same scale run alone."""
    frames = torch.from_numpy(synth.synth_frames(2, 368, 656, seed=77)).cuda()
    est = BodyEstimator(w25, "body25", scale_search=(0.505, 0.51, 1.0))
    geoms, pafs, heats = est.run_scales(frames)
    torch.cuda.synchronize()
    assert geoms[0][:2] == geoms[1][:2]
    for i, s in enumerate((0.505, 0.51, 1.0)):
        one = BodyEstimator(w25, "body25", scale_search=(s,))
        _, p1, h1 = one.run_scales(frames, keep_maps=True)
        torch.cuda.synchronize()
        assert torch.equal(pafs[i], p1[0]) and torch.equal(heats[i], h1[0]), s


@pytest.mark.parametrize("n", [1, 2, 32])
def test_x3_deep_small_grids_bit_identical(net25, n, monkeypatch):
    """Small grids (Mode R's 23x41 stage layers on the 128-pixel family: canonical K ranges in
    one block at batch 32, across blocks at batch 1-2) with inputs and weights staged two K
    steps ahead (VAR 128, ISLPOSE_X3_DEEP=1: loader / DMA role split, unconditional loads so
    the waits are counted, raw barriers) run the same MFMA sequence as the default loop:
    bit-identical maps, with the stage layers on the variant (isl_net_op_info)."""
    x = torch.from_numpy(_inputs(n, 184, 328, seed=600 + n)).cuda()
    monkeypatch.setenv("ISLPOSE_X3_WR", "0")     # the split-K form (wave ranges take precedence)
    monkeypatch.setenv("ISLPOSE_X3_G2", "0")     # two K groups take precedence over the deep loop
    monkeypatch.setenv("ISLPOSE_X3_DEEP", "0")
    paf0, heat0 = net25.forward(x)
    torch.cuda.synchronize()
    monkeypatch.setenv("ISLPOSE_X3_DEEP", "1")
    paf1, heat1 = net25.forward(x)
    torch.cuda.synchronize()
    var = [rt.decode_variant(v) for _, v in net25.op_variants()]
    assert sum(1 for v in var if v.get("var", 0) & 128) >= 60
    assert torch.equal(paf0, paf1) and torch.equal(heat0, heat1)


@pytest.mark.parametrize("n", [1, 4])
def test_graph_replay_bit_identical(w25, n, monkeypatch):
    """The conv chain replayed as a HIP graph (isl_net_set_graph, opt-in): the first run
    of a key is eager, the second captures, later runs replay -- every run's maps equal the
    eager net's bit for bit, the op variants are those of the eager run, a changed ISLPOSE_*
    switch is a new key, and new weights drop the captured launches (their scales are kernel
    arguments)."""
    monkeypatch.delenv("ISLPOSE_NET_GRAPH", raising=False)
    eager = rt.Net(rt.ISL_BODY25)
    eager.load_weights(w25)
    eager.set_graph(False)
    g = rt.Net(rt.ISL_BODY25)
    g.load_weights(w25)
    g.set_graph(True)
    xs = [torch.from_numpy(_inputs(n, 184, 328, seed=300 + k)).cuda() for k in range(4)]
    ref = [eager.forward(x) for x in xs]
    var0 = eager.op_variants()
    for k, x in enumerate(xs):   # eager, capture, replay, replay
        paf, heat = g.forward(x)
        assert torch.equal(paf, ref[k][0]) and torch.equal(heat, ref[k][1]), k
        assert g.op_variants() == var0, k
    # another switch value: a new key (eager, then captured) with its own variants
    monkeypatch.setenv("ISLPOSE_X3_DEEP", "0")
    e2 = [eager.forward(x) for x in xs[:3]]
    for k in range(3):
        paf, heat = g.forward(xs[k])
        assert torch.equal(paf, e2[k][0]) and torch.equal(heat, e2[k][1]), k
    assert g.op_variants() == eager.op_variants()
    monkeypatch.delenv("ISLPOSE_X3_DEEP")
    # new weights (other power-of-two scales): the old graphs are dropped
    w2 = {k: v * 0.5 for k, v in w25.items()}
    eager.load_weights(w2)
    g.load_weights(w2)
    for k in range(3):
        r = eager.forward(xs[k])
        paf, heat = g.forward(xs[k])
        assert torch.equal(paf, r[0]) and torch.equal(heat, r[1]), k
    torch.cuda.synchronize()


@pytest.mark.parametrize("n", [1, 32])
def test_x3_halfco_default_selection(net25, n, monkeypatch):
    """Half-channel blocks (VAR 256: two 64-channel blocks per 128-channel tile) are the
    default of the split-K form (ISLPOSE_X3_WR=0) where the canonical K ranges run across blocks
    (batch-1 Mode R) and on the 3x3 grids of at most half a block per CU (x3_halfsmall); at batch
    32 none.  Same bits either way: the batch-invariance test compares the two executions."""
    monkeypatch.setenv("ISLPOSE_X3_WR", "0")
    x = torch.from_numpy(_inputs(n, 184, 328, seed=91 + n)).cuda()
    net25.forward(x)
    torch.cuda.synchronize()
    var = [rt.decode_variant(v) for _, v in net25.op_variants()]
    halves = sum(1 for v in var if v.get("var", 0) & 256)
    assert halves >= 40 if n == 1 else halves == 0
    # without ranges only on the small 3x3 grids (x3_halfsmall: batch-1 conv2_x / conv3_x)
    assert all(v.get("var", 0) & 2048 or v["ks"] == 3 for v in var if v.get("var", 0) & 256)


@pytest.mark.parametrize("n", [1, 2])
@pytest.mark.parametrize("env", [None, ("ISLPOSE_X3_PX64", "1"), ("ISLPOSE_X3_HALFSMALL", "0")])
def test_x3_px64_c96_split_bit_identical(net25, n, env, monkeypatch):
    """Small-grid block forms == the 128-pixel full-channel blocks (ISLPOSE_X3_PX64=0,
    ISLPOSE_X3_HALFSMALL=0) bit for bit, by default and in the A/B forms: where the canonical K
    ranges run across blocks (the 23x41 stage layers at small batch) the 96-channel tiles and
    the half-channel blocks on 64 pixels (x3_px64; =1 the 96-channel ones only), and the small
    3x3 grids without ranges on half-channel blocks (x3_halfsmall) -- same K order per output."""
    x = torch.from_numpy(_inputs(n, 184, 328, seed=77 + n)).cuda()
    monkeypatch.setenv("ISLPOSE_X3_WR", "0")      # the split-K form's block shapes
    monkeypatch.setenv("ISLPOSE_X3_PX64", "0")
    monkeypatch.setenv("ISLPOSE_X3_HALFSMALL", "0")
    paf0, heat0 = net25.forward(x)
    torch.cuda.synchronize()
    var0 = [rt.decode_variant(v) for _, v in net25.op_variants()]
    monkeypatch.delenv("ISLPOSE_X3_PX64")
    monkeypatch.delenv("ISLPOSE_X3_HALFSMALL")
    if env:
        monkeypatch.setenv(*env)
    paf1, heat1 = net25.forward(x)
    torch.cuda.synchronize()
    var1 = [rt.decode_variant(v) for _, v in net25.op_variants()]
    px64 = [v for v in var1 if v.get("bco") == 96 and v.get("bpx") == 64]
    assert len(px64) >= 10 and all(v["split"] for v in px64)
    assert not any(v.get("bco") == 96 and v.get("bpx") == 64 for v in var0)
    half64 = sum(1 for v in var1 if v.get("var", 0) & 256 and v["bpx"] == 64)
    assert half64 >= 20 if env != ("ISLPOSE_X3_PX64", "1") else half64 == 0
    if n == 1:
        small = sum(1 for v in var1 if v.get("var", 0) & 256 and not v["split"])
        assert small >= 2 if env != ("ISLPOSE_X3_HALFSMALL", "0") else small == 0
    assert torch.equal(paf0, paf1) and torch.equal(heat0, heat1)


def test_graph_drop_waits_for_queued_replays(w25):
    """Replays queued on a non-default stream, then new weights and a forward with no
    synchronisation in between: the weight upload drops the instantiated graphs while those
    replays may still be in flight, so the drop must drain the device first.  The
    maps of the last forward equal an eager net's on the new weights."""
    g = rt.Net(rt.ISL_BODY25)
    g.load_weights(w25)
    g.set_graph(True)
    s = torch.cuda.Stream()
    x = torch.from_numpy(_inputs(2, 184, 328, seed=17)).cuda()
    o0 = torch.empty((2, 52, 23, 41), device="cuda")
    o1 = torch.empty((2, 26, 23, 41), device="cuda")
    sh = rt.stream_handle(s)
    s.wait_stream(torch.cuda.current_stream())
    for _ in range(6):   # eager, capture, then replays left queued
        rt.check(rt.lib().isl_net_forward(g.h, rt.ptr(x), 2, 184, 328, rt.ptr(o0), rt.ptr(o1), sh))
    w2 = {k: v * 0.5 for k, v in w25.items()}
    g.load_weights(w2)
    rt.check(rt.lib().isl_net_forward(g.h, rt.ptr(x), 2, 184, 328, rt.ptr(o0), rt.ptr(o1), sh))
    s.synchronize()
    assert g.range_ok()
    eager = rt.Net(rt.ISL_BODY25)
    eager.load_weights(w2)
    eager.set_graph(False)
    rp, rh = eager.forward(x)
    torch.cuda.synchronize()
    assert torch.equal(o0, rp) and torch.equal(o1, rh)


def test_graph_cap_evicts_without_draining(w25):
    """More run keys than the per-arena cap (8 instantiated graphs): each new capture retires the
    least recently launched exec behind the event of its last replay instead of a device-wide
    synchronisation; the retired execs are freed once those events have passed.
    Ten batch sizes, each captured and replayed on a non-default stream with no host wait, then
    every size again: all maps equal an eager net's."""
    g = rt.Net(rt.ISL_BODY25)
    g.load_weights(w25)
    g.set_graph(True)
    eager = rt.Net(rt.ISL_BODY25)
    eager.load_weights(w25)
    eager.set_graph(False)
    s = torch.cuda.Stream()
    sh = rt.stream_handle(s)
    x = torch.from_numpy(_inputs(10, 64, 96, seed=23)).cuda()
    outs = {}
    s.wait_stream(torch.cuda.current_stream())
    for rnd in range(2):
        for n in range(1, 11):
            o0 = torch.empty((n, 52, 8, 12), device="cuda")
            o1 = torch.empty((n, 26, 8, 12), device="cuda")
            for _ in range(3):   # eager, capture + replay, replay
                rt.check(rt.lib().isl_net_forward(g.h, rt.ptr(x), n, 64, 96, rt.ptr(o0), rt.ptr(o1), sh))
            outs[(rnd, n)] = (o0, o1)
    s.synchronize()
    assert g.range_ok()
    for n in range(1, 11):
        rp, rh = eager.forward(x[:n])
        torch.cuda.synchronize()
        for rnd in range(2):
            assert torch.equal(outs[(rnd, n)][0], rp) and torch.equal(outs[(rnd, n)][1], rh), (rnd, n)


@pytest.mark.parametrize("n", [32, 40])   # >= one block per CU: the ranges run in one block
def test_x3_g2_two_k_groups_bit_identical(net25, w25, n, monkeypatch):
    """Two K groups per block (VAR 32: the first group of waves sums the first half of a layer's
    canonical K ranges, the second group the second half, the halves meet in LDS) == one group walking every range
    (ISLPOSE_X3_G2=0: three accumulator sets) bit for bit -- both add each half's range sums
    in order and then the halves (x3_canonical_order), as x3_splitk_reduce does for the
    ranges split across blocks.  The 23x41 stage layers take the variant (isl_net_op_info);
    frame 0 matches the oracle."""
    x = _inputs(n, 184, 328, seed=900 + n)
    xt = torch.from_numpy(x).cuda()
    monkeypatch.delenv("ISLPOSE_X3_G2", raising=False)
    paf1, heat1 = net25.forward(xt)
    torch.cuda.synchronize()
    var = [rt.decode_variant(v) for _, v in net25.op_variants()]
    assert sum(1 for v in var if v.get("g2")) >= 60, sum(1 for v in var if v.get("g2"))
    assert all(v.get("ranged") and v["bco"] == 128 for v in var if v.get("g2"))
    monkeypatch.setenv("ISLPOSE_X3_G2", "0")
    paf0, heat0 = net25.forward(xt)
    torch.cuda.synchronize()
    assert not any(v.get("g2") for v in (rt.decode_variant(c) for _, c in net25.op_variants()))
    assert torch.equal(paf0, paf1) and torch.equal(heat0, heat1)
    rp, rh = cpu_ref.make_net_fn("body25", w25)(x[:1])
    assert _rel(paf1[:1].cpu().numpy(), rp) < TOL and _rel(heat1[:1].cpu().numpy(), rh) < TOL


def _forward_async(net, x, stream):
    """isl_net_forward on `stream` without the synchronous range check (Net.forward's), so the
    host enqueues and returns at once."""
    n, _, h, w = x.shape
    o0 = torch.empty((n, 52, h // 8, w // 8), device=x.device)
    o1 = torch.empty((n, 26, h // 8, w // 8), device=x.device)
    rt.check(rt.lib().isl_net_forward(net.h, rt.ptr(x), n, h, w, rt.ptr(o0), rt.ptr(o1), rt.stream_handle(stream)),
             "isl_net_forward")
    return o0, o1


def test_first_arena_on_nonblocking_stream_while_another_is_busy(w25):
    """VERDICT r05 #4 (order, don't drain): a new arena is zeroed with hipMemsetAsync on the
    caller's stream instead of a null-stream memset plus a device-wide drain.  While one
    non-blocking stream is busy with a batch-8 368x656 forward, a second non-blocking stream
    runs the first forward of two new sizes (new arenas: their rings and gap channels must be
    zero before any conv reads them); each equals the same forward run alone, bit for bit.
    The synchronous range check then waits on the two streams' events only."""
    net = rt.Net(rt.ISL_BODY25)
    net.load_weights(w25)
    ref = rt.Net(rt.ISL_BODY25)
    ref.load_weights(w25)
    xa = torch.from_numpy(_inputs(8, 368, 656, seed=3)).cuda()
    xb = torch.from_numpy(_inputs(2, 200, 264, seed=4)).cuda()
    xc = torch.from_numpy(_inputs(3, 96, 136, seed=5)).cuda()
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    pa, ha = _forward_async(net, xa, sa)        # long: ~6 ms of convs on sa
    pb, hb = _forward_async(net, xb, sb)        # new arenas, first runs, on sb
    pc, hc = _forward_async(net, xc, sb)
    assert net.range_ok()                       # waits for sa's and sb's events, not the device
    torch.cuda.synchronize()
    for x, p, hh in ((xb, pb, hb), (xc, pc, hc), (xa, pa, ha)):
        rp, rh = ref.forward(x)
        torch.cuda.synchronize()
        assert torch.equal(p, rp) and torch.equal(hh, rh)
