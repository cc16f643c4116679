"""Benchmark: frames/s of body_25 forward + NMS + PAF grouping (BASELINE.json metric).

One step = the whole hot path over one batch of synthetic 368x656 uint8 frames
resident in HBM:
    isl_net_preprocess   (cubic resize / pad / normalise -> padded NHWC)
    isl_net_run          (body_25: 114 convolutions + 3 pools; split-fp16 x3 on the
                          FP16 matrix cores by default, fp32-accurate)
    isl_body_post        (x8 cubic resize, fp64 blur + NMS, peak lists, PAF line
                          integrals, greedy matching, person assembly)
    + async D2H of the per-frame result records (copy stream, overlapping the next step).
The post stage is fed designed pose maps (3 persons per frame) so that its cost
is that of real footage (raw outputs of random weights produce ~4k peaks, see
SURVEY.md §8d); the network still runs in full every step.

Multi-GPU: one process per GPU, frames sharded across ranks with no collective
on the data path (weak scaling).  `--gpus N` without a WORLD_SIZE in the
environment starts the N rank processes itself (islpose.parallel.spawn_ranks);
under torch.distributed.run the ranks come from the environment.  A barrier +
device sync brackets the timed region; rank 0 reports the max-over-ranks time.
The barrier and the timing reductions run on gloo over the host: nothing on the
data path needs RCCL.  `--dry-run` exercises that whole launch / shard / gather
structure on the CPU (tests/test_bench_launch.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from islpose import parallel  # noqa: E402

METRIC = "frames/sec body_25 368×656 fwd+NMS+PAF at 1/8 MI355X; conv MFMA util %"
PEAK_FP32_MFMA_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 matrix peak (spec) = 256 CU x 4 SIMD x 64 FLOP/clk x 2.4 GHz
PEAK_FP16_MFMA_TFLOPS = 2516.6     # dense FP16/BF16 MFMA: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz (~2.5 PF, no sparsity)
PEAK_HBM_GBPS = 8000.0             # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
MFMA_LOOP_CEILING_TF = 1549.0      # measured: bare x3 3x3 step loop, 32x32x16, all CUs (profiles/r02/mfma_shape/)
KIND = {0: "maxpool2_kernel", 1: "conv_mfma_f32 (direct fp32)", 2: "wino_f23_mfma (Winograd F(2x2,3x3) fp32)",
        3: "conv_x3_f16 (split-fp16 x3, fp32-accurate)",
        4: "wino_x3_f16 (Winograd F(2x2,3x3), split-fp16 x3, fp32-accurate)",
        5: "wino_f16 (Winograd F(2x2,3x3), split-fp16 x3, fp32-accurate)"}
# MFMA FLOPs the algorithm of each kind needs per direct-conv FLOP (2*Cout*Cin*k*k*H*W), tile padding excluded
ALG_FACTOR = {1: 1.0, 2: 16.0 / 36.0, 3: 3.0, 4: 3.0 * 16.0 / 36.0, 5: 3.0 * 16.0 / 36.0}
KIND_PEAK = {1: PEAK_FP32_MFMA_TFLOPS, 2: PEAK_FP32_MFMA_TFLOPS, 3: PEAK_FP16_MFMA_TFLOPS, 4: PEAK_FP16_MFMA_TFLOPS,
             5: PEAK_FP16_MFMA_TFLOPS}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=32, help="frames per GPU per step")
    p.add_argument("--height", type=int, default=368)
    p.add_argument("--width", type=int, default=656)
    p.add_argument("--scale", type=float, default=1.0,
                   help="scale_search entry: 1.0 = net at 368x656 (metric shape); 0.5 = reference default")
    p.add_argument("--persons", type=int, default=3)
    p.add_argument("--streams", type=int, default=1,
                   help="split the per-GPU batch over this many HIP streams (own arena each) so one "
                        "sub-batch's layer tail overlaps the other's next layer (+2-3 %% frames/s); the "
                        "per-kernel roofline is then taken over overlapping launches and reads low")
    p.add_argument("--algo", default="x3", choices=["x3", "wino", "direct"],
                   help="conv arithmetic: split-fp16 x3 on the FP16 matrix cores (default), Winograd or direct fp32")
    p.add_argument("--cpu-frames", type=int, default=6, help="frames for the CPU baseline sample (0 = skip)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-op-timing", action="store_true",
                   help="A/B only: no per-op HIP events in the timed region (roofline fields then absent)")
    p.add_argument("--e2e-steps", type=int, default=3,
                   help="batches timed through the caller path (host frames in, Python results out); 0 = skip")
    p.add_argument("--split-k", action="store_true",
                   help="latency mode of the conv K ranges (isl_net_set_split_k mode 2: also an adaptive, "
                        "batch-dependent split of small grids); the default is mode 1 (canonical ranges)")
    p.add_argument("--dry-run", action="store_true",
                   help="no GPU: run the rank launch, shard and max-over-ranks timing structure only")
    p.add_argument("--fail-rank", type=int, default=-1,
                   help="test only (with --dry-run): this rank exits 1 after the group is up, so the "
                        "launcher's fail-fast path is exercised (tests/test_bench_launch.py)")
    p.add_argument("--post-overlap", action="store_true",
                   help="the post of batch k on its own stream beside the net of batch k+1 "
                        "(BodyEstimator.launch(post_stream=...)); measured +0.8 %% Mode N, +0-5 %% Mode R, "
                        "+5 %% at batch 1, but the post then slows the concurrent convs (Mode N frac 0.446 -> "
                        "0.439, Mode R 0.34 -> 0.29), so off by default (profiles/r03/post_overlap/)")
    p.add_argument("--frame-count", type=int, default=64,
                   help="the unchanged scripts' per-frame path (ISLSignPos.call on sequential 1080x1920 frames, "
                        "extract_features_mp.py:125-130) timed over this many frames after the headline, reported "
                        "as the 'frame' sub-object (rank 0; 0 = skip)")
    p.add_argument("--frame-repeat", type=int, default=4,
                   help="frame leg: timed passes over the --frame-count frames (one pass read +-4 %% run to run)")
    p.add_argument("--no-mode-r", dest="mode_r", action="store_false",
                   help="skip the Mode R sub-measurement (net 184x328 at batch 32 and batch 1)")
    p.add_argument("--pg-timeout", type=float, default=120.0,
                   help="seconds a gloo collective (init, barrier, gather) may block before the rank fails")
    return p.parse_args(argv)


def rank_env():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init_group(world, timeout_s=120.0):
    """Host-side (gloo) group for the barrier and the timing reductions only.  gloo
    prints its connection lines on the process's stdout: they go to stderr here, so
    rank 0's stdout carries only the JSON line.  An explicit timeout bounds every
    collective: a rank whose peer died fails instead of blocking for torch's default."""
    if world > 1:
        import datetime
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            torch.distributed.init_process_group("gloo", timeout=datetime.timedelta(seconds=timeout_s))
            torch.distributed.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        assert torch.distributed.get_world_size() == world


def gather_floats(vals, world):
    """All ranks' float vectors (host gloo all_gather) -> [world, len(vals)] numpy."""
    t = torch.tensor(vals, dtype=torch.float64)
    if world == 1:
        return t[None].numpy()
    parts = [torch.zeros_like(t) for _ in range(world)]
    torch.distributed.all_gather(parts, t)
    return torch.stack(parts).numpy()


def frame_shard(rank, batch):
    """Frame indices of one rank's per-step batch: disjoint across ranks (weak scaling)."""
    return rank * batch, (rank + 1) * batch


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launcher: N rank processes, this process never touches the GPU
        codes, out0 = parallel.spawn_ranks([os.path.abspath(__file__)] + sys.argv[1:], args.gpus)
        sys.stdout.write(out0 or "")
        sys.stdout.flush()
        # a rank's own failure (positive code) wins over the signal codes of the siblings
        # the launcher terminated after it
        bad = [c for c in codes if c > 0] or [1 for c in codes if c]
        if bad:
            print("bench.py: rank exit codes %s" % codes, file=sys.stderr)
        sys.exit(bad[0] if bad else 0)
    rank, local, world = rank_env()
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    init_group(world, args.pg_timeout)
    try:
        if args.dry_run:
            dry_run(args, rank, world)
        else:
            gpu_main(args, rank, local, world)
    finally:
        if world > 1:
            torch.distributed.destroy_process_group()


def dry_run(args, rank, world):
    """The launch / shard / timing skeleton of gpu_main without a GPU: every rank
    'processes' its own frame shard per step; rank 0 prints what the real run
    would report about ranks and shards."""
    lo, hi = frame_shard(rank, args.batch)
    if rank == args.fail_rank:
        print("bench.py: rank %d failing on request (--fail-rank)" % rank, file=sys.stderr, flush=True)
        os._exit(1)
    for _ in range(args.warmup):
        pass
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    g = gather_floats([elapsed, lo, hi], world)
    if rank != 0:
        return
    print(json.dumps({"dry_run": True, "n_gpus": world,
                      "world_observed": torch.distributed.get_world_size() if world > 1 else 1,
                      "shards": [[int(a), int(b)] for a, b in g[:, 1:]],
                      "elapsed_max_s": float(g[:, 0].max()), "steps": args.steps, "warmup": args.warmup}))


def gpu_main(args, rank, local, world):
    import ctypes

    from islpose import runtime as rt
    from islpose import synth
    from islpose.body import BodyEstimator, scale_geometry

    # one GPU per rank; more ranks than visible GPUs share them round-robin (a rehearsal
    # of the multi-rank path on a smaller box -- the line then says so in "ranks")
    ndev = torch.cuda.device_count()
    local = local % ndev if ndev > 0 else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    H, W = args.height, args.width
    weights = synth.synth_weights(0)
    L = rt.lib()
    main_stream = torch.cuda.current_stream(dev)

    def measure(scale, B, steps, warmup, S, op_timing):
        """One configuration: B frames per rank per step at `scale`, S lanes (streams); warmup
        steps, then `steps` timed steps between barriers; per-op HIP events on the last."""
        assert B % S == 0, "batch must split evenly over the streams"
        lo, hi = frame_shard(rank, B)
        # frames of this rank: indices [lo, hi), disjoint shards
        frames_h = synth.synth_frames(B, H, W, seed=1000 + rank)
        frames = torch.from_numpy(frames_h).to(dev)
        (mult, nh, nw, vh, vw), = scale_geometry(H, W, (scale,))
        geoms = [(nh, nw, vh, vw)]
        maps = [synth.designed_pose_maps(nh // 8, nw // 8, args.persons, seed=i) for i in range(lo, hi)]
        d_paf = torch.from_numpy(np.stack([m[0] for m in maps])).to(dev)
        d_heat = torch.from_numpy(np.stack([m[1] for m in maps])).to(dev)

        class Lane:
            """One sub-batch on its own stream with its own net arena; lanes overlap on the GPU."""

            def __init__(self, s):
                self.est = BodyEstimator(weights, "body25", device=local, scale_search=(scale,))
                self.net = self.est.net
                self.net.set_algo(args.algo)
                if args.split_k:
                    self.net.set_split_k(2)
                self.b = B // S
                sl = slice(s * self.b, (s + 1) * self.b)
                self.frames, self.paf, self.heat = frames[sl], d_paf[sl], d_heat[sl]
                self.caps = rt.IslCaps(**self.est.caps)
                self.lay = rt.body_layout(self.est.kind, self.caps)
                self.d_res = torch.empty(self.b * self.lay.record_bytes, dtype=torch.uint8, device=dev)
                self.h_res = torch.empty(self.b * self.lay.record_bytes, dtype=torch.uint8, pin_memory=True)
                self.g = (rt.IslScaleGeom * 1)(rt.IslScaleGeom(*geoms[0]))
                self.pp = (ctypes.c_void_p * 1)(self.paf.data_ptr())
                self.hp = (ctypes.c_void_p * 1)(self.heat.data_ptr())
                self.stream = main_stream if S == 1 else torch.cuda.Stream(dev)
                self.sh = rt.stream_handle(self.stream)
                # post overlap: the net writes this batch's low-res maps into one of two NCHW
                # buffers (what BodyEstimator.launch(post_stream=...) keeps for the post), and
                # the post of batch k runs on its own stream beside the net of batch k+1.  The
                # post here reads the designed maps (see `data`); the unpack into the buffers
                # and the buffer hand-over events are the product's own cost and ordering.
                self.pstream = torch.cuda.Stream(dev) if args.post_overlap else self.stream
                self.psh = rt.stream_handle(self.pstream)
                nh8, nw8 = nh // 8, nw // 8
                self.maps = [(torch.empty((self.b, 52, nh8, nw8), device=dev),
                              torch.empty((self.b, 26, nh8, nw8), device=dev)) for _ in range(2)] \
                    if args.post_overlap else None
                self.maps_free = [None, None]
                self.k = 0
                # D2H of the records on a copy stream: it overlaps the next step's preprocess and
                # net; the next post (which rewrites d_res) waits for it, and the timed region's
                # closing device synchronize includes it.  Small records (batch 1: ~0.1 MB, a
                # ~5 us blit) are copied on the post's own stream instead: the cross-queue wait
                # the copy stream needs costs more (~14 us between the net and the post)
                cs_env = os.environ.get("ISLPOSE_BENCH_COPY_STREAM")   # 1 / 0: force either (A/B)
                use_cs = cs_env == "1" if cs_env in ("0", "1") else self.d_res.numel() > (1 << 20)
                self.cs = torch.cuda.Stream(dev) if use_cs else None
                self.copied = None

        lanes = [Lane(s) for s in range(S)]
        ev = []

        def step(timed):
            # timed: stage events (net / post windows) on this step; timing events are kept
            # off the other steps, like the per-op events (each costs a dispatch gap)
            def mark(stream):
                e = torch.cuda.Event(enable_timing=timed)
                e.record(stream)
                return e
            ref = mark(main_stream)
            marks = []
            for ln in lanes:
                if ln.stream is not main_stream:
                    ln.stream.wait_event(ref)
                ln.net.preprocess(ln.frames, mult, stream=ln.stream)
                e0 = mark(ln.stream) if timed else None
                if ln.maps is not None:
                    slot = ln.k & 1
                    if ln.maps_free[slot] is not None:        # the post two batches back is done with it
                        ln.stream.wait_event(ln.maps_free[slot])
                    ln.net.run(ln.maps[slot][0], ln.maps[slot][1], stream=ln.stream)
                else:
                    ln.net.run(stream=ln.stream)
                e1 = mark(ln.stream)
                if ln.pstream is not ln.stream:   # (a wait on the stream's own event is a barrier packet)
                    ln.pstream.wait_event(e1)
                if ln.copied is not None:
                    ln.pstream.wait_event(ln.copied)
                rt.check(L.isl_body_post(ln.net.h, ln.b, H, W, 1, ln.g, ln.pp, ln.hp, ctypes.byref(ln.caps),
                                         rt.ptr(ln.d_res), ln.psh), "post")
                e2 = mark(ln.pstream)
                if ln.maps is not None:
                    ln.maps_free[ln.k & 1] = e2
                    ln.k += 1
                marks.append((e0, e1, e2))
                if ln.cs is None:
                    with torch.cuda.stream(ln.pstream):
                        ln.h_res.copy_(ln.d_res, non_blocking=True)
                else:
                    ln.cs.wait_event(e2)
                    with torch.cuda.stream(ln.cs):
                        ln.h_res.copy_(ln.d_res, non_blocking=True)
                    ln.copied = torch.cuda.Event()
                    ln.copied.record(ln.cs)
            for ln in lanes:
                if ln.stream is not main_stream:
                    main_stream.wait_stream(ln.stream)
            if timed:
                ev.append((ref, marks))

        def net_window_ms(ref, marks):
            # conv stage wall time of one step: first net start -> last net end over all lanes
            return max(ref.elapsed_time(m[1]) for m in marks) - min(ref.elapsed_time(m[0]) for m in marks)

        def post_window_ms(ref, marks):
            # post kernels of one step (isl_body_post: resize/blur/NMS, peaks, PAF scoring, assembly)
            return max(ref.elapsed_time(m[2]) for m in marks) - min(ref.elapsed_time(m[1]) for m in marks)

        for _ in range(warmup):
            step(False)
        torch.cuda.synchronize(dev)
        # validate one step's records (no overflow / errors) outside the timed region, and
        # count the (A, B) candidate pairs the PAF kernel scores (sum over limbs of nA * nB)
        pairs = 0
        for ln in lanes:
            host = ln.h_res.numpy()
            for f in range(ln.b):
                o = f * ln.lay.record_bytes + ln.lay.status
                st = int(host[o:o + 4].view(np.int32)[0])
                assert st == 0, "post status %d on frame %d" % (st, f)
                o = f * ln.lay.record_bytes + ln.lay.n_peaks
                npk = host[o:o + 128].view(np.int32)
                pairs += sum(int(npk[a]) * int(npk[b]) for a, b in synth.BODY25_LIMBS)
            assert ln.net.range_ok(), "split-fp16 range exceeded in warmup"
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        t0 = time.perf_counter()
        # the net / post window events sit on the step before the last: an un-instrumented
        # step like the others (the instrumented step differs; with graph replay
        # opted in, ISLPOSE_NET_GRAPH=1, it is the one eager step); with a single timed step
        # they share it
        win = steps - 2 if steps >= 2 else steps - 1
        for i in range(steps):
            # per-op HIP events (each lane's stream) on the last timed step only: an event
            # between every launch costs ~8 us of dispatch gap (1.8 % of the step when every
            # step carried them, tools/archive/gpu_optiming.sh); one instrumented step of K still gives
            # the per-launch averages of every kernel, inside the timed region
            last = i == steps - 1
            if last and op_timing:
                for ln in lanes:
                    ln.net.set_timing(True)
            step(i == win)
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        elapsed = time.perf_counter() - t0
        for ln in lanes:
            ln.net.set_timing(False)
        # range guard over the timed steps (outside the timed region): a set flag would mean a
        # batch needed the fp32 recompute the timed loop did not do
        range_timed = sum(0 if ln.net.range_ok() else 1 for ln in lanes)
        range_trips = sum(ln.net.range_trips() for ln in lanes)
        ops = [ln.net.timing() for ln in lanes] if op_timing else None
        net_ms = float(np.mean([net_window_ms(r, m) for r, m in ev]))
        post_ms = float(np.mean([post_window_ms(r, m) for r, m in ev]))
        g = gather_floats([elapsed, net_ms, post_ms, B * steps / elapsed, lo, hi, local], world)
        return {"elapsed": float(g[:, 0].max()), "net_ms": float(g[:, 1].max()), "post_ms": float(g[:, 2].max()),
                "g": g, "ops": ops, "pairs": pairs, "range_timed": range_timed, "range_trips": range_trips,
                "lanes": lanes, "frames_h": frames_h, "maps": maps, "mult": mult, "nh": nh, "nw": nw,
                "B": B, "steps": steps, "fps": B * world * steps / float(g[:, 0].max())}

    B, S = args.batch, args.streams
    # one GPU: the per-frame leg first, on a fresh process -- after the batch-32 legs (their
    # arenas, Mode R's 200 timed batch-1 steps) the same leg read 3-6 % lower (171-177 vs
    # 182 frames/s alone, profiles/r06/fr6/); the headline's timed steps do not depend on it
    frame_first = args.frame_count > 0 and world == 1
    frame = frame_leg(args) if frame_first else None
    m = measure(args.scale, B, args.steps, args.warmup, S, not args.no_op_timing)
    e2e = e2e_rate(args, m["lanes"][0].est, m["frames_h"], m["maps"], dev) if args.e2e_steps > 0 else None
    # Mode R (the reference scripts' net size, scale_search=[0.5], body.py:41): the
    # same step at batch 32 and at batch 1 (the scripts' one-frame-per-call pattern), in the
    # same invocation, with their own roofline -- a sub-object, not the headline value
    mode_r = None
    if args.mode_r and args.scale == 1.0 and not args.no_op_timing:
        mode_r = {}
        for key, bb, st, wu in (("batch32", 32, args.steps, max(1, args.warmup)),
                                # (batch 1: 200 timed steps, ~0.35 s, so that one host hiccup does not
                                # decide the rate; 30 steps read 467-575 frames/s box to box, r4ax)
                                ("batch1", 1, max(200, args.steps), max(10, args.warmup))):
            mr = measure(0.5, bb, st, wu, 1, True)
            rf = roofline_of(mr["ops"])
            mode_r[key] = {"frames_per_s": round(mr["fps"], 2), "batch_per_gpu": bb, "steps": st, "warmup": wu,
                           "ms_per_step": round(mr["elapsed"] / st * 1e3, 3), "net_hw": [mr["nh"], mr["nw"]],
                           "net_ms_per_step": round(mr["net_ms"], 3), "post_ms_per_step": round(mr["post_ms"], 3),
                           "roofline": {k: rf[k] for k in ("bound", "kernel", "achieved", "peak", "unit", "frac",
                                                           "launches", "avg_launch_us", "all_convs_tflops",
                                                           "ms_per_step_by_kind")},
                           "range_guard_trips_in_timed_steps": mr["range_timed"]}
            del mr
        mode_r["basis"] = ("scale_search=[0.5] (net 184x328), same step as the headline (preprocess + body_25 + "
                           "post on designed maps + D2H), timed in this invocation after it; frac as the headline's")
    if rank != 0:
        return
    g = m["g"]
    elapsed, net_ms, post_ms, ops = m["elapsed"], m["net_ms"], m["post_ms"], m["ops"]
    nh, nw, mult = m["nh"], m["nw"], m["mult"]
    fps = m["fps"]
    if args.no_op_timing:
        print(json.dumps({"metric": METRIC, "value": round(fps, 2), "unit": "frames/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 3), "op_timing": False}))
        return
    rf = roofline_of(ops)
    rf["op_timing"] = "per-op HIP events on the last of the %d timed steps (lane streams)" % args.steps
    rf["net_ms_per_step"] = round(net_ms, 3)
    out = {
        "metric": METRIC,
        "value": round(fps, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {3: "fp32 (split-fp16 x3 MFMA, fp32 accumulate)",
                  4: "fp32 (split-fp16 x3 MFMA, fp32 accumulate)"}.get(rf.pop("_dom"), "fp32"),
        "data": "synthetic (seeded uint8 frames, counter-hash weights; post fed designed %d-person maps)"
                % args.persons,
        "config": {"workload": "configs[1]: body_25 single-scale %dx%d frames, batch %d per GPU, net input %dx%d"
                               % (H, W, B, nh, nw),
                   "batch_per_gpu": B, "frame_hw": [H, W], "scale_search": [args.scale], "net_hw": [nh, nw],
                   "streams_per_gpu": S, "post_overlap": bool(args.post_overlap),
                   "conv_algo": args.algo, "split_k": bool(args.split_k),
                   "parallelism": "frame-sharded x%d (no collective)" % world},
        "ranks": {"world_observed": torch.distributed.get_world_size() if world > 1 else 1,
                  "per_rank_frames_per_s": [round(float(v), 2) for v in g[:, 3]],
                  "frame_shards": [[int(a), int(b)] for a, b in g[:, 4:6]],
                  "rank_devices": [int(d) for d in g[:, 6]],
                  "devices_shared": bool(len(set(int(d) for d in g[:, 6])) < world),
                  "timing_collectives": "gloo (host): barrier + all_gather of per-rank times; no data-path collective"},
        "roofline": rf,
        "mode_r": mode_r,
        "range_guard": {"trips_in_timed_steps": m["range_timed"], "trips_total": m["range_trips"],
                        "basis": "split-fp16 range flag (|x| >= 65504 in any conv output) checked after the "
                                 "timed steps; a trip means a batch must be recomputed on the fp32 kernels "
                                 "(isl_net_range_info counts them per net)"},
        "post": post_fields(H, W, B, post_ms, m["pairs"]),
        "e2e": e2e,
        "cpu_baseline": None,
    }
    if args.frame_count > 0:
        out["frame"] = frame if frame_first else frame_leg(args)
    if not args.no_cpu and args.cpu_frames > 0 and world == 1:
        out["cpu_baseline"] = cpu_baseline(args, mult, nh, nw)
    print(json.dumps(out))
    sys.stdout.flush()


def frame_leg(args):
    """The unchanged reference scripts' per-frame path: ISLSignPos.call on
    sequential 1080x1920 frames (extract_features_mp.py:125-130), body and hand ms per frame
    and the conv launches per frame -- tools/bench_configs.py's FRAME leg, run in this
    invocation after the headline (rank 0)."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import bench_configs
    ns = argparse.Namespace(frame_count=args.frame_count, frame_repeat=args.frame_repeat)
    try:
        return bench_configs.frame(ns)
    except Exception as e:   # never lose the headline line to the sub-measurement
        return {"error": "%s: %s" % (type(e).__name__, e)}


def conv_stage(kinds, runs):
    """All split-fp16 conv launches (kinds 3 + 5): executed MFMA TF/s and frac, the direct-conv
    equivalent (3 x 2*Cout*Cin*k*k*H*W) TF/s and frac, and each algorithm's share."""
    ks = [k for k in kinds if k in (3, 5)]
    if not ks:
        return None
    ms = sum(kinds[k]["ms"] for k in ks)
    sec = ms * 1e-3
    executed = sum(kinds[k]["mfma_flops"] for k in ks) / sec / 1e12
    alg = sum(ALG_FACTOR[k] * kinds[k]["flops"] for k in ks) / sec / 1e12
    deq = 3.0 * sum(kinds[k]["flops"] for k in ks) / sec / 1e12
    return {"ms_per_step": round(ms / runs, 3), "launches_per_step": sum(kinds[k]["launches"] for k in ks) // runs,
            "executed_mfma_tflops": round(executed, 2), "executed_frac": round(executed / PEAK_FP16_MFMA_TFLOPS, 4),
            "algorithmic_mfma_tflops": round(alg, 2), "algorithmic_frac": round(alg / PEAK_FP16_MFMA_TFLOPS, 4),
            "direct_equiv_tflops": round(deq, 2), "direct_equiv_frac": round(deq / PEAK_FP16_MFMA_TFLOPS, 4),
            "basis": "executed = MFMA FLOPs the kernels ran (tile padding included); algorithmic = split-fp16 "
                     "direct x3 / Winograd 3 x 16/36 of the direct count; direct_equiv = 3 x the direct-conv count "
                     "for every layer (the rate the round-5 frac measured), all over the summed conv launch time",
            "share_ms": {KIND[k]: round(kinds[k]["ms"] / runs, 3) for k in ks}}


def roofline_of(ops):
    """Roofline fields of the dominant kernel class from per-op HIP-event timings (summed
    over lanes and recorded runs): achieved = the MFMA FLOPs its algorithm needs / summed
    launch time, against the dense peak of the dtype the matrix cores run."""
    kinds = {}
    for o in ops:
        for k in set(o["kind"].tolist()):
            msk = o["kind"] == k
            d = kinds.setdefault(int(k), {"ms": 0.0, "flops": 0.0, "mfma_flops": 0.0, "launches": 0})
            d["ms"] += float(o["ms"][msk].sum())
            d["flops"] += float(o["flops"][msk].sum())
            d["mfma_flops"] += float(o["mfma_flops"][msk].sum())
            d["launches"] += int(msk.sum()) * o["n_runs"]
    dom = max(kinds, key=lambda k: kinds[k]["ms"])
    dk = kinds[dom]
    peak = KIND_PEAK.get(dom, PEAK_FP32_MFMA_TFLOPS)
    sec = dk["ms"] * 1e-3
    fp32_equiv = dk["flops"] / sec / 1e12                      # direct-conv FLOPs per second
    achieved = ALG_FACTOR.get(dom, 1.0) * dk["flops"] / sec / 1e12   # MFMA work the algorithm needs, no padding
    executed = dk["mfma_flops"] / sec / 1e12                   # what the matrix cores ran (tile padding included)
    conv_ms = sum(v["ms"] for k, v in kinds.items() if k in (1, 2, 3, 4, 5))
    conv_flops = sum(v["flops"] for k, v in kinds.items() if k in (1, 2, 3, 4, 5))
    key = {1: "direct", 2: "wino", 3: "x3", 4: "wino_x3", 5: "w2"}.get(dom, "x3")
    traffic = mfma_busy = clk = busy_s = clk_s = stage_busy = stage_busy_s = src = None
    prof = os.path.join(REPO, "profiles", "conv_traffic.json")
    if os.path.exists(prof):
        pj = json.load(open(prof))
        traffic = pj.get(key + "_hbm_bytes_per_launch")
        mfma_busy, clk = pj.get(key + "_mfma_busy_frac"), pj.get(key + "_effective_clock_ghz")
        busy_s, clk_s = pj.get(key + "_mfma_busy_frac_at_stamp_clock"), pj.get(key + "_stamp_clock_ghz")
        stage_busy = pj.get("conv_stage_mfma_busy_frac")
        stage_busy_s = pj.get("conv_stage_mfma_busy_frac_at_stamp_clock")
        src = pj.get("source")
    runs = max(1, ops[0]["n_runs"])
    return {"bound": "mfma", "kernel": KIND[dom], "_dom": dom,
            "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": traffic,
            "achieved_basis": "MFMA FLOPs the kernel's algorithm needs (direct-conv count 2*Cout*Cin*k*k*H*W "
                              "x %.4g: split-fp16 = 3 fp16 products per fp32 MAC, Winograd = 16/36, tile "
                              "padding excluded) / summed launch time; peak = dense MFMA peak of the dtype the "
                              "matrix cores run (fp16 2516.6 / fp32 157.3 TF)" % ALG_FACTOR.get(dom, 1.0),
            "fp32_equiv_tflops": round(fp32_equiv, 2),
            "fp32_equiv_vs_fp32_peak": round(fp32_equiv / PEAK_FP32_MFMA_TFLOPS, 4),
            "executed_tflops": round(executed, 2),
            "executed_frac": round(executed / peak, 4),
            "launches": dk["launches"], "avg_launch_us": round(dk["ms"] * 1e3 / dk["launches"], 2),
            "algorithmic_gflop_per_launch": round(dk["flops"] / dk["launches"] / 1e9, 3),
            "all_convs_tflops": round(conv_flops / (conv_ms * 1e-3) / 1e12, 2),
            "ms_per_step_by_kind": {KIND[k]: round(v["ms"] / runs, 3) for k, v in kinds.items()},
            # every conv of the step together (split-fp16 direct + Winograd): the MFMA work the
            # matrix cores executed and the direct-conv-equivalent rate (3 x the direct count, the
            # work the x3 direct form would need: comparable across rounds), side by side
            "conv_stage": conv_stage(kinds, runs),
            # PMC (profiles/conv_traffic.json, from tools/profile_round.sh): MFMA pipe busy
            # fraction of the dominant kernel's wall cycles, and the DVFS clock it ran at; the
            # conv stage adds conv1_1's write-bound conv_x3_rgb
            "mfma_busy_pmc": mfma_busy,
            "conv_stage_mfma_busy_pmc": stage_busy,
            "conv_stage_mfma_busy_pmc_at_stamp_clock": stage_busy_s,
            "effective_clock_ghz": clk,
            "frac_at_effective_clock": round(achieved / (peak * clk / 2.4), 4) if clk else None,
            # the GRBM-based clock reads high on sub-10 ms dispatches (MI355X_MICROARCH.md DVFS item 6);
            # the in-kernel clock of a stamp build (s_memtime / s_memrealtime) of the dominant shape:
            "mfma_busy_pmc_at_stamp_clock": busy_s,
            "stamp_clock_ghz": clk_s,
            "frac_at_stamp_clock": round(achieved / (peak * clk_s / 2.4), 4) if clk_s else None,
            "pmc_source": src or "profiles/conv_traffic.json (tools/profile_round.sh + tools/pmc_summary.py)",
            # the bare x3 inner loop (LDS fragment reads + 3 MFMAs per product, no staging,
            # no barriers) on every CU: what the chip sustains with this MFMA shape under its
            # power limit (the clock settles at ~1.55 GHz)
            "mfma_loop_ceiling_tflops": MFMA_LOOP_CEILING_TF if key == "x3" else None,
            "frac_of_mfma_loop_ceiling": round(achieved / MFMA_LOOP_CEILING_TF, 4) if key == "x3" else None,
            "ceiling_source": "tools/mfma_shape_bench.hip step32, profiles/r02/mfma_shape/mfma_shape_bench.txt"}


def post_fields(H, W, B, post_ms, pairs):
    """The metric's "NMS and PAF" part: live post time (HIP events around isl_body_post),
    plus the counter-backed HBM traffic and rocprof durations of the NMS / PAF kernels
    from the last committed profile (profiles/post_traffic.json)."""
    out = {
        "ms_per_step": round(post_ms, 3),
        "frames_per_s": round(B / (post_ms * 1e-3), 1),
        "nms_algorithmic_bytes_per_frame": 25 * H * W * 4,
        "nms_effective_GBps": round(25 * H * W * 4 * B / (post_ms * 1e-3) / 1e9, 1),
        "paf_pairs_per_frame": round(pairs / B, 1),
        "paf_pairs_per_s": round(pairs / (post_ms * 1e-3), 1),
        "basis": "HIP events around isl_body_post on the post stream (with post_overlap it runs beside the next "
                 "batch's net, so this window can stretch; fused resize+blur+NMS, peak lists, PAF "
                 "scoring, greedy matching, assembly; D2H excluded). nms_effective_GBps = SURVEY 8(d)'s NMS "
                 "bytes (25 x H x W x 4 B f32 heat per frame) / whole post time: the fused kernel never "
                 "materialises those planes, so this is an effective rate, not HBM traffic",
    }
    prof = os.path.join(REPO, "profiles", "post_traffic.json")
    if os.path.exists(prof):
        pj = json.load(open(prof))
        out["pmc"] = {k: pj[k] for k in ("blur_nms_kernel", "blur_nms_exact", "limb_kernel", "tile_live_kernel",
                                         "band_live_kernel", "compact_kernel", "assemble_kernel") if k in pj}
        out["pmc_source"] = pj.get("source")
        out["pmc_peak_GBps"] = PEAK_HBM_GBPS
        out["pmc_basis"] = pj.get("note")
    return out


def e2e_rate(args, est, frames_h, maps, dev):
    """Caller-path rate (what Body.estimate_batch users get): host uint8 frames -> H2D ->
    preprocess + net -> post on the designed maps -> D2H of the records -> Python decode
    into (candidate, subset) per frame.  Timed per batch, after the main timed region."""
    from islpose.body import scale_geometry
    H, W = frames_h.shape[1:3]
    geoms = [g[1:] for g in scale_geometry(H, W, (args.scale,))]
    paf = torch.from_numpy(np.stack([m[0] for m in maps])).to(dev)
    heat = torch.from_numpy(np.stack([m[1] for m in maps])).to(dev)

    def once():
        t = torch.from_numpy(frames_h).to(dev)
        est.run_scales(t)
        return est.post_maps(H, W, geoms, [paf], [heat], details=False)

    once()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.e2e_steps):
        res = once()
    dt = (time.perf_counter() - t0) / args.e2e_steps
    assert len(res) == len(frames_h)
    return {"frames_per_s": round(len(frames_h) / dt, 2), "ms_per_batch": round(dt * 1e3, 3),
            "batch": len(frames_h), "batches_timed": args.e2e_steps,
            "basis": "host frames -> H2D -> preprocess + body_25 -> isl_body_post (designed maps) -> D2H -> "
                     "BodyEstimator.decode to the reference's (candidate, subset); wall time per batch, rank 0"}


def cpu_baseline(args, mult, nh, nw):
    """The oracle (torch-CPU conv graph + numpy post, parity-pinned against the
    reference) timed per frame on this host's cores: forward + post, designed maps
    for the post exactly as on the GPU."""
    from oracle import cpu_ref
    from islpose import synth
    affinity = len(os.sched_getaffinity(0))
    # the GPU box exports OMP_NUM_THREADS = its CPU share per GPU; the forward is also
    # timed on every core of the affinity set and the faster one is the baseline
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    share = min(affinity, omp) if omp > 0 else affinity
    w = synth.synth_weights(0)
    fwd = cpu_ref.make_net_fn("body25", w)
    frames = synth.synth_frames(args.cpu_frames, args.height, args.width, seed=1000)
    med = lambda t: float(np.median(t[1:] if len(t) > 2 else t))
    t_fwd, t_post = [], []
    torch.set_num_threads(share)
    for i in range(args.cpu_frames):
        print("cpu_baseline: frame %d/%d" % (i + 1, args.cpu_frames), file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        im, _, _ = cpu_ref.net_input(frames[i], mult)
        fwd(im)
        t1 = time.perf_counter()
        pl, hl = synth.designed_pose_maps(nh // 8, nw // 8, args.persons, seed=i)
        cpu_ref.body_call(frames[i], lambda x: (pl[None], hl[None]), "body25", (args.scale,))
        t2 = time.perf_counter()
        t_fwd.append(t1 - t0)
        t_post.append(t2 - t1)
    fwd_by_threads = {share: med(t_fwd)}
    # every affinity core too, unless the affinity set is far larger than the CPU share
    # (the GPU box: 256 visible, 16 granted -- 256 torch threads there ran > 3 minutes)
    oversubscribed = affinity > 2 * share
    if share < affinity and not oversubscribed:
        torch.set_num_threads(affinity)
        t_all = []
        for i in range(min(3, args.cpu_frames)):
            t0 = time.perf_counter()
            im, _, _ = cpu_ref.net_input(frames[i], mult)
            fwd(im)
            t_all.append(time.perf_counter() - t0)
        fwd_by_threads[affinity] = med(t_all)
        torch.set_num_threads(share)
    cores = min(fwd_by_threads, key=fwd_by_threads.get)
    per = fwd_by_threads[cores] + med(t_post)
    return {"value": round(1.0 / per, 4), "unit": "frames/s", "cores": cores, "kind": "port",
            "affinity_cores": affinity,
            "fwd_s_by_threads": {str(k): round(v, 4) for k, v in fwd_by_threads.items()},
            "threads_basis": "forward timed with torch.set_num_threads(t) for t in {min(affinity, OMP_NUM_THREADS=%s), "
                             "len(sched_getaffinity)=%d}; the faster is used (cores). The post is numpy/scipy, one thread"
                             % (omp or "unset", affinity) +
                             ("; all-affinity timing skipped: %d visible cores > 2x the %d-CPU share (oversubscribed)"
                              % (affinity, share) if oversubscribed else ""),
            "sample": "%d frames %dx%d (scale %.2f, net %dx%d), median of frames 2..N: fwd %.3f s + post %.3f s per frame"
                      % (args.cpu_frames, args.height, args.width, args.scale, nh, nw,
                         fwd_by_threads[cores], med(t_post))}


if __name__ == "__main__":
    main()
