"""Throughput of the other BASELINE.json configs on one GPU (bench.py measures configs[1]).

  C3  body_25 + handpose, batch 16 frames, 1 person and 2 hand crops per frame
      (crop widths 120-200 px, Hand.__call__'s 4-scale pyramid 184/368/552/736):
      body net (Mode R, scale 0.5 like the ISL scripts) + body post on designed
      1-person maps + one batched hand pass over the 32 crops per step.
  C4  body_25 4-scale pyramid (scale_search 0.5/1/1.5/2 -> nets 184x328 ... 736x1312),
      batch 16 frames per GPU (128 over 8 GPUs, sharded), post on designed maps.

  C5  the video -> JSON pipeline (islpose.pipeline) on 1080x1920 RGB frames, body
      (Mode R) + batched hand crops + per-frame JSON files, sequential vs overlapped.
  FRAME  the unchanged scripts' per-frame path: ISLSignPos.call on one 1080x1920 frame at a
      time (extract_features_mp.py:125-130, model(frame[:, :, ::-1])), with the C5 tamed body
      weights (hand crops up to ~1000 px); wall time per call, split into the body part
      (bodypos + handDetect on the same frames) and the hand part (the rest).
  C6  translator head: the HIP sign classifier (csrc/sign.hip) on [B, 20, 156]
      windows -- latency of one window (the demo's per-frame call) and throughput
      of a batch of 4096 windows; plus translate_stream over a 64-frame clip
      (body + hands once per frame, 45 windows classified in one launch).

Prints one JSON line per config: frames/s, ms per step and the conv TFLOP/s of the
step (direct-conv FLOP count, HIP events around the whole step).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def conv_gflop(kind, h, w):
    from islpose import netspec
    g, H, W = 0.0, h, w
    for c in netspec.convs_for(kind):
        g += 2.0 * c.cout * c.cin * c.k * c.k * H * W / 1e9
        if c.name in ("conv1_2", "conv2_2", "conv3_4"):
            H, W = H // 2, W // 2
    return g


def timed(step, steps, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def c3(args):
    from islpose import synth
    from islpose.body import BodyEstimator, scale_geometry
    from islpose.hand import HandEstimator, HAND_SCALES
    B, H, W = args.batch, 368, 656
    body = BodyEstimator(synth.synth_weights(0), "body25", scale_search=(0.5,))
    hand = HandEstimator(synth.synth_weights(2))
    frames = torch.from_numpy(synth.synth_frames(B, H, W, seed=5)).cuda()
    (m, nh, nw, vh, vw), = scale_geometry(H, W, (0.5,))
    maps = [synth.designed_pose_maps(nh // 8, nw // 8, 1, seed=i) for i in range(B)]
    paf = torch.from_numpy(np.stack([a for a, _ in maps])).cuda()
    heat = torch.from_numpy(np.stack([b for _, b in maps])).cuda()
    rng = np.random.RandomState(0)
    boxes = []
    for f in range(B):
        for _ in range(2):
            w = int(rng.randint(120, 201))
            boxes.append((f, int(rng.randint(0, W - w)), int(rng.randint(0, H - w)), w))

    # designed hand maps for the post (random weights give dense maps: one giant component
    # per plane, unlike real footage); the hand nets still run in full on every crop
    hgeo = [(s * 368 // 8, s * 368 // 8) for s in (0.5, 1.0, 1.5, 2.0)]
    hmaps = [torch.from_numpy(np.stack([synth.designed_hand_maps(int(hh), int(ww), seed=31 * i + k)
                                        for i in range(len(boxes))])).cuda()
             for k, (hh, ww) in enumerate(hgeo)]

    def step():
        body.net.preprocess(frames, m)
        body.net.run()
        body.post_maps(H, W, [(nh, nw, vh, vw)], [paf], [heat], details=False)
        heats = hand.run_crops(frames, boxes)
        hand.post_crops(boxes, hmaps if args.designed_hands else heats)

    sec = timed(step, args.steps, args.warmup)
    gf = B * conv_gflop(0, nh, nw) + len(boxes) * sum(conv_gflop(2, s, s) for s in (184, 368, 552, 736))
    return {"config": "C3 body_25 + hand (2 crops/frame, 4 scales)", "batch": B, "crops": len(boxes),
            "frames_per_s": round(B / sec, 2), "ms_per_step": round(sec * 1e3, 2),
            "conv_gflop_per_step": round(gf, 1), "conv_tflops_fp32_equiv_wall": round(gf / sec / 1e3, 1),
            "hand_scales": list(HAND_SCALES),
            "hand_post_on": "designed maps" if args.designed_hands else "raw net output (random weights: dense maps)"}


def c4(args):
    from islpose import synth
    from islpose.body import BodyEstimator, scale_geometry
    B, H, W = args.batch, 368, 656
    scales = (0.5, 1.0, 1.5, 2.0)
    body = BodyEstimator(synth.synth_weights(0), "body25", scale_search=scales)
    frames = torch.from_numpy(synth.synth_frames(B, H, W, seed=6)).cuda()
    geo = scale_geometry(H, W, scales)
    pafs, heats = [], []
    for i, g in enumerate(geo):
        mp = [synth.designed_pose_maps(g[1] // 8, g[2] // 8, 3, seed=10 * i + k) for k in range(B)]
        pafs.append(torch.from_numpy(np.stack([a for a, _ in mp])).cuda())
        heats.append(torch.from_numpy(np.stack([b for _, b in mp])).cuda())
    geoms = [g[1:] for g in geo]

    def step():
        for (m, nh, nw, vh, vw) in geo:
            body.net.preprocess(frames, m)
            body.net.run()
        body.post_maps(H, W, geoms, pafs, heats, details=False)

    sec = timed(step, args.steps, args.warmup)
    gf = B * sum(conv_gflop(0, g[1], g[2]) for g in geo)
    return {"config": "C4 body_25 4-scale pyramid", "batch_per_gpu": B, "nets": [[g[1], g[2]] for g in geo],
            "frames_per_s": round(B / sec, 2), "ms_per_step": round(sec * 1e3, 2),
            "conv_gflop_per_step": round(gf, 1), "conv_tflops_fp32_equiv_wall": round(gf / sec / 1e3, 1)}


def c5(args):
    """configs[4]: the extract_features_mp.py:122-132 pipeline on 1080x1920 RGB frames
    (Mode R body net 184x327 -> 184x328, batched hand crops, per-frame JSON files),
    sequential vs overlapped (prefetch + async H2D + GPU flip + writer thread)."""
    import shutil
    import tempfile
    from islpose import pipeline, synth
    from islpose.body import BodyEstimator
    from src.body import Body
    from src.hand import Hand
    from src.ISL_Model_parameter import ISLSignPos
    T, H, W = args.c5_frames, 1080, 1920
    B = args.c5_batch
    rgb = synth.synth_frames(T, H, W, seed=57)
    # heat layer tamed on the GPU net's own output for frame 0 (a few persons per frame)
    wb = synth.synth_weights(0)
    cal = BodyEstimator(wb, "body25", scale_search=(0.5,))
    _, _, heats = cal.run_scales(torch.from_numpy(np.ascontiguousarray(rgb[:1, ..., ::-1])).cuda(), keep_maps=True)
    wb = synth.tame_heat_layer(wb, heats[0].cpu().numpy(), "body25", gain=0.05)
    del cal
    tw = lambda d: {k: torch.from_numpy(v) for k, v in d.items()}  # noqa: E731
    isl = ISLSignPos(Body(tw(wb), "body25").model, Hand(tw(synth.synth_weights(2))).model)
    clips = {"v%d.mp4" % k: rgb for k in range(args.c5_videos)}
    rows = [{"Filepath": f, "type": "Greetings", "expression": "hello"} for f in clips]
    res = {"config": "C5 video -> per-frame JSON, 1080x1920 RGB frames", "frames": T * len(rows),
           "videos": len(rows), "batch": B, "export": False,
           "decode": "frames already decoded in host memory (pims/ffmpeg absent); the pipeline reads them as "
                     "slices of the [T,H,W,3] array"}
    for ov in ((True,) if args.c5_overlap_only else (False, True)):
        out = tempfile.mkdtemp(prefix="c5_")
        try:
            # warm-up (arenas, hand scales) on the first video, then the timed pass over all
            pipeline.extract_dataset(rows[:1], clips.__getitem__, isl, out, batch=B, export=False, overlap=ov)
            shutil.rmtree(out)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            feats, ex = pipeline.extract_dataset(rows, clips.__getitem__, isl, out, batch=B,
                                                 export=False, overlap=ov)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            hands = 0
            for f in feats:
                hands += len(f["all_hand_peaks"])
        finally:
            shutil.rmtree(out, ignore_errors=True)
        key = "overlap" if ov else "sequential"
        res[key + "_frames_per_s"] = round(ex.frames_done / dt, 2)
        res[key + "_s"] = round(dt, 3)
        res["hand_crops_per_frame"] = round(hands / max(len(feats), 1), 2)
    return res


def frame(args):
    """ISLSignPos.call per frame, 1080x1920 RGB frames flipped to BGR as a view (the script's
    frame[:, :, ::-1]); every call returns to the host (numpy results), as in the script."""
    from islpose import runtime as rt, synth
    from islpose.body import BodyEstimator
    from src import util
    from src.body import Body
    from src.hand import Hand
    from src.ISL_Model_parameter import ISLSignPos
    T, H, W = args.frame_count, 1080, 1920
    rgb = synth.synth_frames(T, H, W, seed=57)
    wb = synth.synth_weights(0)
    cal = BodyEstimator(wb, "body25", scale_search=(0.5,))
    _, _, heats = cal.run_scales(torch.from_numpy(np.ascontiguousarray(rgb[:1, ..., ::-1])).cuda(), keep_maps=True)
    wb = synth.tame_heat_layer(wb, heats[0].cpu().numpy(), "body25", gain=0.05)
    del cal
    tw = lambda d: {k: torch.from_numpy(v) for k, v in d.items()}  # noqa: E731
    isl = ISLSignPos(Body(tw(wb), "body25").model, Hand(tw(synth.synth_weights(2))).model)
    body = isl._estimators()[0]
    for i in range(min(5, T)):          # warm-up: arenas of the body and of the hand crop sizes
        isl.call(rgb[i][:, :, ::-1])
    torch.cuda.synchronize()
    crops, widths = 0, []
    # the T frames REPEAT times over (a pass is ~0.35 s: one pass read +-4 % run to run)
    R = max(1, getattr(args, "frame_repeat", 1))
    t0 = time.perf_counter()
    for _ in range(R):
        for i in range(T):
            _, _, hands = isl.call(rgb[i][:, :, ::-1])
            crops += len(hands)
    dt = (time.perf_counter() - t0) / R
    crops /= R
    t0 = time.perf_counter()
    for i in range(T):
        f = rgb[i][:, :, ::-1]
        (c, sb), = body.estimate(isl._upload(f))
        widths += [w for _, _, w, _ in util.handDetect(c, sb, f)]
    db = time.perf_counter() - t0
    # conv launches per frame: the body net (one run) and the hand net (one run per scale of the
    # frame's crop batch), from the op variants of their last runs; a split-K layer adds its reduce
    hand = isl._estimators()[1]

    def launches(net):
        codes = [v for _, v in net.op_variants()]
        return sum(1 for v in codes if v not in (-1, -2)) + sum(1 for v in codes if rt.decode_variant(v).get("split"))
    body_launches = launches(body.net)
    # the hand net's conv launches over its four scales for one crop of a frame with hands (each
    # scale run once more, after the timed passes, to read its op variants)
    hand_launches = 0
    if widths:
        from islpose.hand import BOXSIZE
        f = rgb[0][:, :, ::-1]
        x = isl._upload(f)
        w0 = widths[0]
        crop = [(0, 0, 0, w0, w0)]
        for s in hand.scale_search:
            gh, gw = hand.net.preprocess_crops(x, crop, s * BOXSIZE)
            hand.net.run(torch.empty((1, 22, gh // 8, gw // 8), device=x.device))
            torch.cuda.synchronize()
            hand_launches += launches(hand.net)
    return {"config": "FRAME ISLSignPos.call per 1080x1920 frame (extract_features_mp.py:130 pattern)",
            "body_conv_launches_per_frame": body_launches,
            "hand_conv_launches_per_crop_4_scales": hand_launches,
            "frames": T, "passes": R, "frames_per_s": round(T / dt, 2), "ms_per_frame": round(dt / T * 1e3, 3),
            "body_ms_per_frame": round(db / T * 1e3, 3), "hand_ms_per_frame": round((dt - db) / T * 1e3, 3),
            "hand_crops_per_frame": round(crops / T, 2),
            "crop_width_px": [int(min(widths)), int(max(widths))] if widths else [],
            "basis": "wall time of T sequential calls (host frame -> pinned H2D -> GPU flip -> body net + post -> "
                     "handDetect -> hand crops batched per scale -> peaks on the host); body = upload + estimate + "
                     "handDetect on the same frames, hand = the rest"}


def c6(args):
    from islpose import synth, translate
    from src.body import Body
    from src.hand import Hand
    from src.ISL_Model_parameter import ISLSignPosTranslator
    clf = translate.SignClassifier()
    rng = np.random.RandomState(0)
    res = {"config": "C6 translator head (sign classifier + translate_stream)"}
    for B in (1, 4096):
        x = torch.from_numpy(rng.uniform(0, 600, (B, 20, 156)).astype(np.float32)).cuda()
        out = torch.empty(B, clf.n_classes, device="cuda")
        sec = timed(lambda: clf(x), args.steps * 10, args.warmup)
        res["windows_%d_us" % B] = round(sec * 1e6, 1)
        res["windows_%d_per_s" % B] = round(B / sec, 1)
        del out
    print(json.dumps(res), flush=True)
    wts = lambda k: {n: torch.from_numpy(v) for n, v in synth.synth_weights(k).items()}  # noqa: E731
    t = ISLSignPosTranslator(Body(wts(0), "body25").model, Hand(wts(2)).model, clf)
    full = t.call_batch
    n_hands = []

    def two_hands(f):      # random weights detect many people; keep <= 2 hands per frame for the export
        r = full(f)
        n_hands.append(sum(len(h) for _, _, h in r))
        return [(c, s, h[:2]) for c, s, h in r]
    t.call_batch = two_hands
    frames = synth.synth_frames(64, 368, 656, seed=4)
    sec = timed(lambda: t.translate_stream(frames), args.steps, args.warmup)
    res.update({"stream_frames": 64, "stream_windows": 45, "stream_ms": round(sec * 1e3, 1),
                "stream_frames_per_s": round(64 / sec, 1),
                "stream_hand_crops_per_clip": int(sum(n_hands) / (args.steps + args.warmup)),
                "stream_note": "synthetic weights: hand crops per clip is set by the random body net"})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["c3", "c4", "c5", "c6", "frame", "all"], default="all")
    ap.add_argument("--frame-count", type=int, default=64, help="FRAME: sequential per-frame calls timed")
    ap.add_argument("--frame-repeat", type=int, default=4, help="FRAME: timed passes over the frames")
    ap.add_argument("--batch", type=int, default=16, help="C3 / C4 frames per step")
    ap.add_argument("--c5-batch", type=int, default=32, help="C5 frames per pipeline batch")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--c5-frames", type=int, default=96, help="C5: frames per (synthetic 1080p) video")
    ap.add_argument("--c5-videos", type=int, default=3)
    ap.add_argument("--c5-overlap-only", action="store_true")
    ap.add_argument("--raw-hand-maps", dest="designed_hands", action="store_false",
                    help="C3: run the hand post on the raw net maps instead of designed maps")
    a = ap.parse_args()
    for name, fn in (("c3", c3), ("c4", c4), ("c5", c5), ("c6", c6), ("frame", frame)):
        if a.config in (name, "all"):
            print(json.dumps(fn(a)), flush=True)


if __name__ == "__main__":
    main()
