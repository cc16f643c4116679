"""ctypes binding of libislpose.so (include/islpose.h).

The HIP library is the only compute path: if it is missing or a call fails,
this module raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

ISL_OK, ISL_E_ARG, ISL_E_PARAM, ISL_E_HIP, ISL_E_CAPACITY, ISL_E_STATE, ISL_E_INDEX = 0, -1, -2, -3, -4, -5, -6
ISL_E_RANGE = -7
ISL_BODY25, ISL_COCO, ISL_HAND = 0, 1, 2
# conv arithmetic (isl_algo): split-fp16 x3 (default), Winograd fp32, direct fp32
ISL_ALGO_X3, ISL_ALGO_WINO, ISL_ALGO_DIRECT = 0, 1, 2
ALGOS = {"x3": ISL_ALGO_X3, "wino": ISL_ALGO_WINO, "direct": ISL_ALGO_DIRECT}

LIB_PATH = os.environ.get("ISLPOSE_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libislpose.so"))

# every symbol include/islpose.h declares
EXPORTS = ["isl_abi_version", "isl_last_error", "isl_net_create", "isl_net_destroy", "isl_net_param_count",
           "isl_net_param_info", "isl_net_set_param", "isl_net_forward", "isl_net_preprocess", "isl_net_run", "isl_net_debug_input",
           "isl_net_set_timing", "isl_net_timing", "isl_body_layout", "isl_body_post", "isl_hand_post",
           "isl_net_set_algo", "isl_net_get_algo", "isl_net_check", "isl_net_preprocess_crops",
           "isl_sign_param_count", "isl_sign_classify", "isl_net_set_split_k", "isl_net_arena_info",
           "isl_debug_np_sum", "isl_hand_post_crops", "isl_net_check_async", "isl_net_range_info",
           "isl_net_op_info", "isl_net_set_graph", "isl_lane_stream_create", "isl_lane_stream_destroy"]


class IslCaps(ctypes.Structure):
    _fields_ = [("max_peaks", ctypes.c_int32), ("max_pairs", ctypes.c_int32),
                ("max_conns", ctypes.c_int32), ("max_rows", ctypes.c_int32)]


class IslLayout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in
                ("status", "n_peaks", "n_conns", "n_rows", "peaks", "conns", "subset", "record_bytes")]


class IslScaleGeom(ctypes.Structure):
    _fields_ = [("net_h", ctypes.c_int32), ("net_w", ctypes.c_int32),
                ("valid_h", ctypes.c_int32), ("valid_w", ctypes.c_int32)]


class IslCrop(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("frame", "x", "y", "w", "h")]


class IslError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libislpose.so once; raise loudly if it is absent (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libislpose.so not found at %s -- build it with `make` (or __graft_entry__.build())"
                          % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
    L.isl_abi_version.restype = i32
    L.isl_last_error.restype = ctypes.c_char_p
    L.isl_net_create.argtypes = [i32, i32, ctypes.POINTER(vp)]
    L.isl_net_destroy.argtypes = [vp]
    L.isl_net_param_count.argtypes = [vp]
    L.isl_net_param_info.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(i64)]
    L.isl_net_set_param.argtypes = [vp, ctypes.c_char_p, vp, i64]
    L.isl_net_forward.argtypes = [vp, vp, i32, i32, i32, vp, vp, vp]
    L.isl_net_preprocess.argtypes = [vp, vp, i32, i32, i32, dbl, ctypes.POINTER(i32), ctypes.POINTER(i32), vp]
    L.isl_net_run.argtypes = [vp, vp, vp, vp]
    L.isl_net_debug_input.argtypes = [vp, vp, vp]
    L.isl_net_set_timing.argtypes = [vp, i32]
    L.isl_net_preprocess_crops.argtypes = [vp, vp, i32, i32, i32, ctypes.POINTER(IslCrop), i32, dbl,
                                           ctypes.POINTER(i32), ctypes.POINTER(i32), vp]
    L.isl_net_set_algo.argtypes = [vp, i32]
    L.isl_net_get_algo.argtypes = [vp]
    L.isl_net_check.argtypes = [vp, i32]
    L.isl_net_check_async.argtypes = [vp, vp, vp]
    L.isl_net_range_info.argtypes = [vp, ctypes.POINTER(i64)]
    L.isl_net_op_info.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(i32)]
    pi, pd = ctypes.POINTER(i32), ctypes.POINTER(dbl)
    L.isl_net_timing.argtypes = [vp, i32, pi, pi, pd, pi, pd, pd]
    L.isl_body_layout.argtypes = [i32, ctypes.POINTER(IslCaps), ctypes.POINTER(IslLayout)]
    L.isl_body_post.argtypes = [vp, i32, i32, i32, i32, ctypes.POINTER(IslScaleGeom), ctypes.POINTER(vp),
                                ctypes.POINTER(vp), ctypes.POINTER(IslCaps), vp, vp]
    L.isl_hand_post.argtypes = [vp, i32, i32, i32, i32, ctypes.POINTER(IslScaleGeom), ctypes.POINTER(vp), vp, vp]
    L.isl_sign_param_count.argtypes = [i32, i32, ctypes.POINTER(i64)]
    L.isl_net_set_split_k.argtypes = [vp, i32]
    L.isl_net_set_graph.argtypes = [vp, i32]
    L.isl_lane_stream_create.argtypes = [i32, i32, ctypes.POINTER(vp)]
    L.isl_lane_stream_destroy.argtypes = [vp]
    L.isl_net_arena_info.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(i32)]
    L.isl_sign_classify.argtypes = [vp, i32, i32, i32, vp, i32, vp, vp]
    L.isl_debug_np_sum.argtypes = [vp, i64, vp, vp]
    L.isl_hand_post_crops.argtypes = [vp, i32, ctypes.POINTER(i32), i32, ctypes.POINTER(IslScaleGeom),
                                      ctypes.POINTER(vp), vp, vp]
    for name in EXPORTS[2:]:
        getattr(L, name).restype = i32
    if L.isl_abi_version() != 1:
        raise ImportError("libislpose ABI mismatch")
    _lib = L
    return L


def check(rc: int, what: str = ""):
    if rc == ISL_OK:
        return
    msg = lib().isl_last_error().decode(errors="replace")
    if rc == ISL_E_PARAM:
        raise KeyError(msg)
    if rc == ISL_E_INDEX:
        raise IndexError("list assignment index out of range")
    raise IslError("%s failed (%d): %s" % (what or "libislpose", rc, msg))


def body_layout(kind: int, caps: IslCaps) -> IslLayout:
    lay = IslLayout()
    check(lib().isl_body_layout(kind, ctypes.byref(caps), ctypes.byref(lay)), "isl_body_layout")
    return lay


def stream_handle(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def flag_slot(owner, ring: int = 4):
    """A pinned int32 slot for Net.check_async, from a ring kept on `owner` for its life
    (the copy into it is issued outside torch, so the buffer must never go back to torch's
    pinned cache while a copy may be in flight); at most `ring` launches in flight."""
    import torch
    slots = getattr(owner, "_flag_slots", None)
    if slots is None:
        slots = owner._flag_slots = [torch.zeros(1, dtype=torch.int32, pin_memory=True) for _ in range(ring)]
        owner._flag_next = 0
    f = slots[owner._flag_next % len(slots)]
    owner._flag_next += 1
    f.zero_()
    return f


_LANES = {}   # device index -> [torch.cuda.ExternalStream], lane k of every estimator


def lane_priorities(k):
    """Priority class of each of k lanes (isl_lane_stream_create): lane 0 (the largest scale,
    the critical path) high, lane 1 low, the rest normal -- three classes, three queue pools.
    ISLPOSE_LANE_PRIO=0: every lane normal (A/B)."""
    if os.environ.get("ISLPOSE_LANE_PRIO", "1") == "0":
        return [0] * k
    return [(-1, 1)[j] if j < 2 else 0 for j in range(k)]


def scale_streams(owner, device, k):
    """k non-blocking streams for a pyramid's scales (isl_lane_stream_create with the classes
    of lane_priorities).  One pool per device, shared by every estimator (work on one stream
    stays in order) and never destroyed: torch's allocator may still hold events on a stream
    that a tensor was recorded on.  `owner` is unused (kept for the callers' signature)."""
    import torch
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    prios = lane_priorities(k)
    key = (idx, tuple(prios[:3]))
    pool = _LANES.setdefault(key, [])
    while len(pool) < k:
        h = ctypes.c_void_p()
        check(lib().isl_lane_stream_create(idx, prios[len(pool)], ctypes.byref(h)), "isl_lane_stream_create")
        pool.append(torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx)))
    return pool[:k]


SCALE_LANES = 4   # streams a pyramid's scales share (lane_plan)


def lane_plan(owner, device, keys, lanes=None):
    """Streams for a pyramid's scales (keys: their net sizes) and the order to enqueue them:
    the distinct sizes go largest first onto the least loaded of SCALE_LANES streams (load =
    net area), and the scales are enqueued largest first.  One stream per scale ran the two
    largest hand scales one after the other (a process has 4 hardware queues, the current
    stream holds one, so the fourth scale stream shared one with the third): 6.70 ms for one
    crop's four scales; [736] [552] [368 -> 184] on three lanes: 5.48 ms
    (tools/hand_conc_events.py, profiles/r06/fr6/lanes.txt).  Scales of one size share a
    lane, in their order (they share that size's arena)."""
    lane, order, n = lane_assign(keys, SCALE_LANES if lanes is None else lanes)
    ss = scale_streams(owner, device, n)
    return [ss[j] for j in lane], order


def lane_assign(keys, lanes):
    """lane_plan without the streams: (lane index per key, enqueue order, lanes used)."""
    distinct = list(dict.fromkeys(keys))
    area = {k: k[0] * k[1] for k in distinct}
    n = max(1, min(lanes, len(distinct)))
    load, lane = [0] * n, {}
    for k in sorted(distinct, key=lambda k: -area[k]):
        j = min(range(n), key=lambda i: load[i])
        lane[k] = j
        load[j] += area[k]
    order = sorted(range(len(keys)), key=lambda i: (-area[keys[i]], i))
    return [lane[k] for k in keys], order, n


def fork_streams(cur, streams):
    """Every distinct stream of `streams` waits for the work queued so far on `cur`.  All
    forks come before any join: a stream forked after `cur` joined an earlier one would wait
    for that one's whole chain, and the scales would run one after another."""
    for st in dict.fromkeys(streams):
        st.wait_stream(cur)


def join_streams(cur, streams):
    """`cur` waits for everything queued on `streams` (after fork_streams and the launches)."""
    for st in dict.fromkeys(streams):
        cur.wait_stream(st)


def crop_net_size(crop_h: int, crop_w: int, scale_times_box: float):
    """Padded net size isl_net_preprocess_crops gives a crop (runtime.cpp: fx = fy =
    scale_times_box / h, cvRound, then padRightDownCorner to a multiple of 8)."""
    m = scale_times_box / crop_h
    rh, rw = int(np.rint(crop_h * m)), int(np.rint(crop_w * m))
    return (rh + 7) // 8 * 8, (rw + 7) // 8 * 8


def ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def decode_variant(code: int) -> dict:
    """isl_net_op_info's variant code -> dict(var=VAR bits, bpx, bco, ks, rgb, pool_fused, ...):
    wave_ranges (conv_x3_wr, VAR 8), c12 (conv1_1 -> conv1_2 in one launch, 4), wino2 (the
    split-fp16 Winograd kernel wino_f16, 64)."""
    if code == -1:
        return {"pool_fused": True}
    if code == -2:
        return {"fused_into_prev": True}     # the second layer of a fused 1x1 pair (VAR 16)
    if code <= 0:
        return {}
    f67 = bool(code & 16)   # the fused pair records its all-channel tile halved (4-bit field)
    return {"var": code & 0xfffff, "bpx": ((code >> 20) & 31) * 32,
            "bco": ((code >> 25) & 15) * 32 * (2 if f67 else 1), "fused67": f67, "g2": bool(code & 32),
            "ks": 2 * ((code >> 29) & 3) + 1, "rgb": bool(code & (1 << 18)),
            "union": bool(code & 512), "ranged": bool(code & 1024), "split": bool(code & 2048),
            "pairs2": bool(code & 4096), "vin": bool(code & 32768), "sib": bool(code & 65536),
            "fold": bool(code & 8192), "m16": bool(code & 131072), "fold_out": bool(code & (1 << 19)),
            "wave_ranges": bool(code & 8), "c12": bool(code & 4), "wino2": bool(code & 64)}


class Net:
    """One network (body25 / coco / hand) on one device, owned by libislpose."""

    def __init__(self, kind: int, device: int = 0):
        self.kind = kind
        self.device = device
        h = ctypes.c_void_p()
        check(lib().isl_net_create(kind, device, ctypes.byref(h)), "isl_net_create")
        self.h = h
        self.loaded = False
        e = os.environ.get("ISLPOSE_X3_SPLITK", "")[:1]
        self.split_k = int(e) if e in ("0", "2") else 1      # isl_net_create's default

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and _lib is not None:
            _lib.isl_net_destroy(h)
            self.h = None

    def param_names(self):
        out = []
        n = lib().isl_net_param_count(self.h)
        for i in range(n):
            name = ctypes.c_char_p()
            numel = ctypes.c_int64()
            check(lib().isl_net_param_info(self.h, i, ctypes.byref(name), ctypes.byref(numel)))
            out.append((name.value.decode(), numel.value))
        return out

    def load_weights(self, weights: dict):
        """weights: flat {caffe_name: array/tensor} (the dict util.transfer reads).
        A missing name raises KeyError like util.transfer (src/util.py:39-43)."""
        for name, numel in self.param_names():
            v = weights[name]
            if hasattr(v, "detach"):
                v = v.detach().cpu().numpy()
            a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
            if a.size != numel:
                raise KeyError("%s: expected %d elements, got %d" % (name, numel, a.size))
            check(lib().isl_net_set_param(self.h, name.encode(), a.ctypes.data_as(ctypes.c_void_p), a.size),
                  "isl_net_set_param")
        self.loaded = True

    def forward(self, x, out0=None, out1=None, stream=None):
        """Module seam: x float32 NCHW cuda tensor -> (paf, heat) or heat."""
        import torch
        assert x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.shape[1] == 3
        x = x.contiguous()
        n, _, h, w = x.shape
        h8, w8 = h // 8, w // 8
        if self.kind == ISL_HAND:
            o0 = out0 if out0 is not None else torch.empty((n, 22, h8, w8), device=x.device)
            o1 = None
        else:
            npaf, nj = (52, 26) if self.kind == ISL_BODY25 else (38, 19)
            o0 = out0 if out0 is not None else torch.empty((n, npaf, h8, w8), device=x.device)
            o1 = out1 if out1 is not None else torch.empty((n, nj, h8, w8), device=x.device)
        check(lib().isl_net_forward(self.h, ptr(x), n, h, w, ptr(o0), ptr(o1), stream_handle(stream)),
              "isl_net_forward")
        if not self.range_ok():
            # an activation left the split-fp16 range: recompute on the fp32 kernels
            with self.algo_scope("direct"):
                check(lib().isl_net_forward(self.h, ptr(x), n, h, w, ptr(o0), ptr(o1), stream_handle(stream)),
                      "isl_net_forward")
        return o0 if o1 is None else (o0, o1)

    # -- conv arithmetic -----------------------------------------------------------
    @property
    def algo(self) -> str:
        a = lib().isl_net_get_algo(self.h)
        return {v: k for k, v in ALGOS.items()}[a]

    def set_algo(self, algo: str):
        """'x3' (split-fp16 on the FP16 matrix cores, fp32-accurate; default), 'wino'
        (Winograd F(2x2,3x3), FP32 MFMA) or 'direct' (implicit GEMM, FP32 MFMA)."""
        check(lib().isl_net_set_algo(self.h, ALGOS[algo]), "isl_net_set_algo")

    def set_split_k(self, mode):
        """K-range mode of the x3 convs (isl_net_set_split_k): 1 canonical ranges (default,
        batch-invariant bits), 0 none, 2 latency (also an adaptive, batch-dependent split
        of the other small grids).  True/False map to 2/0."""
        mode = {True: 2, False: 0}.get(mode, mode) if isinstance(mode, bool) else int(mode)
        check(lib().isl_net_set_split_k(self.h, mode), "isl_net_set_split_k")
        self.split_k = mode

    def set_graph(self, on: bool):
        """Replay the conv chain as a HIP graph after its first runs (isl_net_set_graph;
        default off, env ISLPOSE_NET_GRAPH=0|1 overrides): the same kernels and bits, without
        the per-launch host cost that bounds batch-1 frames."""
        check(lib().isl_net_set_graph(self.h, 1 if on else 0), "isl_net_set_graph")

    def algo_scope(self, algo: str):
        import contextlib

        @contextlib.contextmanager
        def scope():
            prev = self.algo
            self.set_algo(algo)
            try:
                yield
            finally:
                self.set_algo(prev)
        return scope()

    def range_ok(self, clear: bool = True) -> bool:
        """Synchronous check of the split-fp16 range flag (isl_net_check; it waits for the
        streams this net's runs were queued on, not the whole device): False if any conv
        output since the last clear reached |x| >= 65504."""
        rc = lib().isl_net_check(self.h, 1 if clear else 0)
        if rc == ISL_E_RANGE:
            return False
        check(rc, "isl_net_check")
        return True

    def check_async(self, flag_host, stream=None):
        """Stream-ordered range check (isl_net_check_async): flag_host, a pinned int32
        tensor of one element, holds the flag (then cleared on the device) once `stream`
        has reached this point."""
        assert flag_host.is_pinned() and flag_host.dtype.itemsize == 4
        check(lib().isl_net_check_async(self.h, ptr(flag_host), stream_handle(stream)), "isl_net_check_async")

    def range_trips(self) -> int:
        """Range-guard trips so far (isl_net_range_info): batches whose split-fp16 range
        check failed and that the caller recomputed on the fp32 kernels.  Synchronising."""
        t = ctypes.c_int64()
        check(lib().isl_net_range_info(self.h, ctypes.byref(t)), "isl_net_range_info")
        return t.value

    def preprocess(self, frames_u8, scale: float, stream=None):
        """frames uint8 [n,H,W,3] cuda -> fills the net input; returns (net_h, net_w)."""
        n, H, W, _ = frames_u8.shape
        nh, nw = ctypes.c_int32(), ctypes.c_int32()
        check(lib().isl_net_preprocess(self.h, ptr(frames_u8), n, H, W, float(scale), ctypes.byref(nh),
                                       ctypes.byref(nw), stream_handle(stream)), "isl_net_preprocess")
        return nh.value, nw.value

    def preprocess_crops(self, frames_u8, crops, scale_times_box: float, stream=None):
        """frames uint8 [n,H,W,3] cuda; crops [(frame, x, y, w, h)] -> fills one net-input
        slot per crop (Hand.__call__'s resize of each crop); returns (net_h, net_w)."""
        n, H, W, _ = frames_u8.shape
        arr = (IslCrop * len(crops))(*[IslCrop(*map(int, c)) for c in crops])
        nh, nw = ctypes.c_int32(), ctypes.c_int32()
        check(lib().isl_net_preprocess_crops(self.h, ptr(frames_u8), n, H, W, arr, len(crops), float(scale_times_box),
                                             ctypes.byref(nh), ctypes.byref(nw), stream_handle(stream)),
              "isl_net_preprocess_crops")
        return nh.value, nw.value

    def debug_input(self, n, h, w, stream=None):
        import torch
        x = torch.empty((n, 3, h, w), device="cuda:%d" % self.device)
        check(lib().isl_net_debug_input(self.h, ptr(x), stream_handle(stream)), "isl_net_debug_input")
        return x

    def run(self, out0=None, out1=None, stream=None):
        check(lib().isl_net_run(self.h, ptr(out0), ptr(out1), stream_handle(stream)), "isl_net_run")

    def arena_info(self):
        """(bytes, arenas) of the net's activation arenas (isl_net_arena_info)."""
        b, k = ctypes.c_int64(), ctypes.c_int32()
        check(lib().isl_net_arena_info(self.h, ctypes.byref(b), ctypes.byref(k)), "isl_net_arena_info")
        return b.value, k.value

    def op_variants(self):
        """[(op name, variant code)] of the last run (isl_net_op_info): the conv kernel
        variant of every op; decode with decode_variant."""
        L = lib()
        n_ops, n_runs = ctypes.c_int32(), ctypes.c_int32()
        check(L.isl_net_timing(self.h, 0, ctypes.byref(n_ops), ctypes.byref(n_runs), None, None, None, None),
              "isl_net_timing")
        out = []
        for k in range(n_ops.value):
            name, var = ctypes.c_char_p(), ctypes.c_int32()
            check(L.isl_net_op_info(self.h, k, ctypes.byref(name), ctypes.byref(var)), "isl_net_op_info")
            out.append((name.value.decode(), var.value))
        return out

    def set_timing(self, on: bool):
        """Record HIP events around every op of the following runs (isl_net_set_timing)."""
        check(lib().isl_net_set_timing(self.h, 1 if on else 0), "isl_net_set_timing")

    def timing(self):
        """Per-op sums over the recorded runs: dict of numpy arrays ms, kind (0 pool,
        1 direct conv, 2 Winograd conv), flops (algorithmic), mfma_flops; plus n_runs."""
        import numpy as np
        L = lib()
        n_ops, n_runs = ctypes.c_int32(), ctypes.c_int32()
        check(L.isl_net_timing(self.h, 0, ctypes.byref(n_ops), ctypes.byref(n_runs), None, None, None, None),
              "isl_net_timing")
        k = n_ops.value
        ms, fl, mf = np.zeros(k), np.zeros(k), np.zeros(k)
        kind = np.zeros(k, np.int32)
        dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
        check(L.isl_net_timing(self.h, k, ctypes.byref(n_ops), ctypes.byref(n_runs), dp(ms),
                               kind.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), dp(fl), dp(mf)), "isl_net_timing")
        return {"ms": ms, "kind": kind, "flops": fl, "mfma_flops": mf, "n_runs": n_runs.value}
