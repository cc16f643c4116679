"""Batched body-pose estimation on the HIP path (frame seam of src/body.py).

``BodyEstimator.estimate(frames)`` runs, for every scale of ``scale_search``
(body.py:41, default ``[0.5]``), the fused pre-processing kernel and the
body_25 / COCO network, then the post-processing kernels (resize, fp64 blur +
NMS, PAF scoring, greedy matching, assembly), and decodes the per-frame result
records into the reference's return values ``(candidate, subset)``
(body.py:235): ``candidate`` float64 [N,4] (x, y, score, id) or shape (0,),
``subset`` float64 [P, njoint+1].
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import runtime as rt

BOXSIZE, STRIDE = 368, 8
NJOINT = {rt.ISL_BODY25: 26, rt.ISL_COCO: 19}
NPAF = {rt.ISL_BODY25: 52, rt.ISL_COCO: 38}
NLIMBS = {rt.ISL_BODY25: 24, rt.ISL_COCO: 19}
KINDS = {"body25": rt.ISL_BODY25, "coco": rt.ISL_COCO}
DEFAULT_CAPS = dict(max_peaks=128, max_pairs=4096, max_conns=128, max_rows=128)


def cv_round(x: float) -> int:
    return int(np.rint(x))


def scale_geometry(H: int, W: int, scale_search):
    """Per scale: (multiplier, net_h, net_w, valid_h, valid_w) as body.py:47-54 computes them."""
    out = []
    for s in scale_search:
        m = s * BOXSIZE / H
        vh, vw = cv_round(H * m), cv_round(W * m)
        out.append((m, -(-vh // STRIDE) * STRIDE, -(-vw // STRIDE) * STRIDE, vh, vw))
    return out


class FrameResult:
    __slots__ = ("candidate", "subset", "all_peaks", "connection_all", "special_k")

    def __init__(self, candidate, subset, all_peaks, connection_all, special_k):
        self.candidate, self.subset = candidate, subset
        self.all_peaks, self.connection_all, self.special_k = all_peaks, connection_all, special_k


class BodyEstimator:
    def __init__(self, weights: dict = None, model_type: str = "body25", device: int = 0, scale_search=(0.5,),
                 caps=None, net: "rt.Net" = None):
        self.kind = KINDS[model_type]
        self.model_type = model_type
        self.device = device
        self.scale_search = tuple(scale_search)
        self.caps = dict(DEFAULT_CAPS, **(caps or {}))
        if net is None:
            net = rt.Net(self.kind, device)
            net.load_weights(weights)
        assert net.kind == self.kind
        self.net = net
        self.njoint, self.npaf = NJOINT[self.kind], NPAF[self.kind]

    # -- network -----------------------------------------------------------------
    def run_scales(self, frames, keep_maps=False):
        """frames: torch uint8 cuda [n,H,W,3]. Returns (geoms, pafs, heats); maps are None
        (read from the arena by the post kernels) for a single scale unless keep_maps."""
        import torch
        n, H, W, _ = frames.shape
        geoms, pafs, heats = [], [], []
        multi = len(self.scale_search) > 1 or keep_maps
        if len(self.scale_search) > 1:
            # pyramid: the scales side by side on the lanes of rt.lane_plan (per-size arenas),
            # as HandEstimator.run_crops; two scales that pad to the same size share one arena,
            # preprocess table and split-K workspace, so they run in order on one lane
            cur = torch.cuda.current_stream(frames.device)
            sg = scale_geometry(H, W, self.scale_search)
            streams, order = rt.lane_plan(self, frames.device, [(g[1], g[2]) for g in sg])
            rt.fork_streams(cur, streams)
            pafs, heats = [None] * len(sg), [None] * len(sg)
            for i in order:
                st, (m, nh, nw, vh, vw) = streams[i], sg[i]
                with torch.cuda.stream(st):
                    gh, gw = self.net.preprocess(frames, m)
                    assert (gh, gw) == (nh, nw)
                    paf = torch.empty((n, self.npaf, nh // 8, nw // 8), device=frames.device)
                    heat = torch.empty((n, self.njoint, nh // 8, nw // 8), device=frames.device)
                    self.net.run(paf, heat)
                frames.record_stream(st)
                paf.record_stream(cur)
                heat.record_stream(cur)
                pafs[i], heats[i] = paf, heat
            geoms = [(nh, nw, vh, vw) for (m, nh, nw, vh, vw) in sg]
            rt.join_streams(cur, streams)
            return geoms, pafs, heats
        for (m, nh, nw, vh, vw) in scale_geometry(H, W, self.scale_search):
            gh, gw = self.net.preprocess(frames, m)
            assert (gh, gw) == (nh, nw)
            if multi:
                paf = torch.empty((n, self.npaf, nh // 8, nw // 8), device=frames.device)
                heat = torch.empty((n, self.njoint, nh // 8, nw // 8), device=frames.device)
                self.net.run(paf, heat)
            else:
                paf = heat = None
                self.net.run()
            geoms.append((nh, nw, vh, vw))
            pafs.append(paf)
            heats.append(heat)
        return geoms, pafs, heats

    # -- post-processing ---------------------------------------------------------
    def post(self, n, H, W, geoms, pafs, heats, caps=None):
        """Run isl_body_post and return the raw result records (numpy uint8) + layout."""
        import torch
        caps = dict(self.caps, **(caps or {}))
        while True:
            c = rt.IslCaps(**caps)
            lay = rt.body_layout(self.kind, c)
            res = torch.empty(n * lay.record_bytes, dtype=torch.uint8, device="cuda:%d" % self.device)
            ns = len(geoms)
            g = (rt.IslScaleGeom * ns)(*[rt.IslScaleGeom(*gg) for gg in geoms])
            pp = (ctypes.c_void_p * ns)(*[rt.ptr(p).value for p in pafs])
            hp = (ctypes.c_void_p * ns)(*[rt.ptr(h).value for h in heats])
            rt.check(rt.lib().isl_body_post(self.net.h, n, H, W, ns, g, pp, hp, ctypes.byref(c), rt.ptr(res),
                                           rt.stream_handle()), "isl_body_post")
            host = res.cpu().numpy()
            grow = self._grow(host, lay, n, caps)
            if grow is None:
                return host, lay, caps
            caps = grow          # capacity overflow: re-run the post kernels with larger buffers (GPU)

    def _grow(self, host, lay, n, caps):
        need = None
        for f in range(n):
            rec = host[f * lay.record_bytes:(f + 1) * lay.record_bytes]
            st = int(rec[lay.status:lay.status + 4].view(np.int32)[0])
            if st == rt.ISL_E_INDEX:
                raise IndexError("list assignment index out of range")
            if st == rt.ISL_E_CAPACITY:
                npk = rec[lay.n_peaks:lay.n_peaks + 128].view(np.int32)[:self.njoint - 1]
                mp = int(npk.max())
                need = need or dict(caps)
                need["max_peaks"] = max(need["max_peaks"], 2 * mp, 2 * caps["max_peaks"] if mp <= caps["max_peaks"] else 0)
                need["max_conns"] = max(need["max_conns"], need["max_peaks"])
                need["max_pairs"] = max(need["max_pairs"], mp * mp)
                need["max_rows"] = max(need["max_rows"], 2 * caps["max_rows"], need["max_conns"] * 4)
            elif st != rt.ISL_OK:
                raise rt.IslError("body post: frame %d status %d" % (f, st))
        return need

    def decode(self, host, lay, caps, n, details=True):
        """Per-frame result records -> FrameResult.  candidate rows are the peaks of parts
        0..nparts-1 in order, ids consecutive (body.py:101-107, 183); all_peaks,
        connection_all and special_k are built only with details (the reference's
        __call__ returns candidate and subset)."""
        out = []
        nparts, nl = self.njoint - 1, NLIMBS[self.kind]
        mpk, mcn, rw = caps["max_peaks"], caps["max_conns"], self.njoint + 1
        slot = np.arange(mpk)
        for f in range(n):
            rec = host[f * lay.record_bytes:(f + 1) * lay.record_bytes]
            npk = rec[lay.n_peaks:lay.n_peaks + 128].view(np.int32)[:nparts]
            nrows = int(rec[lay.n_rows:lay.n_rows + 4].view(np.int32)[0])
            pk = rec[lay.peaks:lay.peaks + nparts * mpk * 24].view(np.float64).reshape(nparts, mpk, 3)
            sel = pk[slot[None, :] < npk[:, None]]               # [N, 3] (x, y, score), part-major
            if len(sel):
                candidate = np.empty((len(sel), 4), np.float64)
                candidate[:, :3] = sel
                candidate[:, 3] = np.arange(len(sel), dtype=np.float64)
            else:
                candidate = np.array([])
            sb = rec[lay.subset:lay.subset + caps["max_rows"] * rw * 8].view(np.float64).reshape(-1, rw)
            subset = sb[:nrows].copy()
            if not details:
                out.append(FrameResult(candidate, subset, None, None, None))
                continue
            ncn = rec[lay.n_conns:lay.n_conns + 128].view(np.int32)[:nl]
            cn = rec[lay.conns:lay.conns + nl * mcn * 40].view(np.float64).reshape(nl, mcn, 5)
            all_peaks, pid = [], 0
            for p in range(nparts):
                lst = []
                for i in range(int(npk[p])):
                    x, y, sc = pk[p, i]
                    lst.append((np.int64(x), np.int64(y), np.float64(sc), pid))
                    pid += 1
                all_peaks.append(lst)
            conn_all, special = [], []
            for k in range(nl):
                if ncn[k] < 0:
                    special.append(k)
                    conn_all.append([])
                else:
                    conn_all.append(cn[k, :ncn[k]].copy())
            out.append(FrameResult(candidate, subset, all_peaks, conn_all, special))
        return out

    def estimate(self, frames, details=False):
        """frames: uint8 [n,H,W,3] (numpy or torch) or one [H,W,3] frame -> list of (candidate, subset)."""
        import torch
        single = frames.ndim == 3
        t = torch.as_tensor(frames)
        if single:
            t = t[None]
        t = t.to("cuda:%d" % self.device).contiguous()
        n, H, W, _ = t.shape
        geoms, pafs, heats = self.run_scales(t)
        host, lay, caps = self.post(n, H, W, geoms, pafs, heats)
        if not self.net.range_ok():
            # split-fp16 range exceeded somewhere in the batch: recompute it on the fp32 kernels
            with self.net.algo_scope("direct"):
                geoms, pafs, heats = self.run_scales(t)
                host, lay, caps = self.post(n, H, W, geoms, pafs, heats)
        res = self.decode(host, lay, caps, n, details)
        if details:
            return res
        out = [(r.candidate, r.subset) for r in res]
        return out[0] if single else out

    # -- pipelined (stream-ordered) form of estimate --------------------------------
    def launch(self, frames_t, post_stream=None):
        """Enqueue estimate() on the current stream without waiting: nets, post, the
        records' copy to pinned host memory and a stream-ordered range check.  frames_t:
        cuda uint8 [n,H,W,3].  finish(job) completes it.

        Without post_stream the net must not run again before finish (its arena holds the
        maps the post and a capacity re-run read).  With post_stream the nets write this
        batch's low-res maps into tensors of its own, the range check follows them on the
        current stream, and the post and the records' copy run on post_stream: the next
        launch's nets may start on the current stream at once, beside this post (the body
        of a video's batch k+1 beside the post of batch k).  post_stream is opt-in: it
        measured as a slowdown of the convs beside the fp64 blur; bench.py's
        --post-overlap times the same overlap on its own step loop."""
        import torch
        n, H, W, _ = frames_t.shape
        geoms, pafs, heats = self.run_scales(frames_t, keep_maps=post_stream is not None)
        flag = rt.flag_slot(self)
        self.net.check_async(flag)
        caps = dict(self.caps)
        c = rt.IslCaps(**caps)
        lay = rt.body_layout(self.kind, c)
        cur = torch.cuda.current_stream(frames_t.device)
        ps = post_stream if post_stream is not None else cur
        if ps is not cur:
            ps.wait_stream(cur)
        with torch.cuda.stream(ps):
            res = torch.empty(n * lay.record_bytes, dtype=torch.uint8, device=frames_t.device)
            ns = len(geoms)
            g = (rt.IslScaleGeom * ns)(*[rt.IslScaleGeom(*gg) for gg in geoms])
            pp = (ctypes.c_void_p * ns)(*[rt.ptr(p).value for p in pafs])
            hp = (ctypes.c_void_p * ns)(*[rt.ptr(h).value for h in heats])
            rt.check(rt.lib().isl_body_post(self.net.h, n, H, W, ns, g, pp, hp, ctypes.byref(c), rt.ptr(res),
                                           rt.stream_handle(ps)), "isl_body_post")
            host = torch.empty(res.shape, dtype=torch.uint8, pin_memory=True)
            host.copy_(res, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(ps)
        if ps is not cur:
            for m in pafs + heats:
                if m is not None:
                    m.record_stream(ps)
        return dict(t=frames_t, n=n, H=H, W=W, geoms=geoms, pafs=pafs, heats=heats, caps=caps, lay=lay, res=res,
                    host=host, flag=flag, ev=ev, ps=post_stream)

    def finish(self, job, details=False):
        """Wait for a launch() and decode it: the same results as estimate(), including
        the fp32 re-run of a batch that left the split-fp16 range and the post re-run
        with larger buffers on a capacity overflow."""
        import contextlib
        import torch
        job["ev"].synchronize()
        n, H, W = job["n"], job["H"], job["W"]
        # a re-run's post goes where the launch's post went: the posts of later launches on a
        # post stream share the net's post scratch with it
        ps = job.get("ps")
        on_ps = (lambda: torch.cuda.stream(ps)) if ps is not None else contextlib.nullcontext
        if int(job["flag"][0]) != 0:
            with self.net.algo_scope("direct"):
                geoms, pafs, heats = self.run_scales(job["t"], keep_maps=ps is not None)
                if ps is not None:
                    ps.wait_stream(torch.cuda.current_stream(job["t"].device))
                with on_ps():
                    host, lay, caps = self.post(n, H, W, geoms, pafs, heats)
        else:
            host, lay, caps = job["host"].numpy(), job["lay"], job["caps"]
            grow = self._grow(host, lay, n, caps)
            if grow is not None:
                with on_ps():
                    host, lay, caps = self.post(n, H, W, job["geoms"], job["pafs"], job["heats"], caps=grow)
        res = self.decode(host, lay, caps, n, details)
        return res if details else [(r.candidate, r.subset) for r in res]

    def post_maps(self, H, W, geoms, pafs, heats, details=True):
        """Post-processing only, on caller low-res maps (NCHW cuda tensors per scale)."""
        n = pafs[0].shape[0]
        host, lay, caps = self.post(n, H, W, geoms, pafs, heats)
        res = self.decode(host, lay, caps, n, details)
        return res if details else [(r.candidate, r.subset) for r in res]
