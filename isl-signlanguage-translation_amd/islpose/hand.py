"""Batched hand keypoints on the HIP path (frame seam of src/hand.py).

``HandEstimator.estimate(crops)`` runs the 4-scale pyramid of Hand.__call__
(hand.py:25, scales 0.5/1/1.5/2 of 368 px) through the fused pre-processing
kernel and the hand network, then isl_hand_post: cubic resize of every scale
back to the crop, fp64 averaging, fp64 blur, 8-connected components of the
thresholded map, largest-mass component and its first maximum.  Returns int64
[21, 2] (x, y) per crop exactly like the reference (hand.py:74).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import runtime as rt
from .body import BOXSIZE, scale_geometry

HAND_SCALES = (0.5, 1.0, 1.5, 2.0)


CROP_CHUNK = 64     # hand crops per batched pass of estimate_crops


class HandEstimator:
    def __init__(self, weights: dict = None, device: int = 0, scale_search=HAND_SCALES, net: "rt.Net" = None):
        self.device = device
        self.scale_search = tuple(scale_search)
        if net is None:
            net = rt.Net(rt.ISL_HAND, device)
            net.load_weights(weights)
        assert net.kind == rt.ISL_HAND
        self.net = net

    def run_scales(self, crops):
        import torch
        n, h, w, _ = crops.shape
        cur = torch.cuda.current_stream(crops.device)
        # the scales side by side on the lanes of rt.lane_plan, as run_crops
        sg = scale_geometry(h, w, self.scale_search)
        streams, order = rt.lane_plan(self, crops.device, [(g[1], g[2]) for g in sg])
        rt.fork_streams(cur, streams)
        heats = [None] * len(sg)
        for i in order:
            st, (m, nh, nw, vh, vw) = streams[i], sg[i]
            with torch.cuda.stream(st):
                gh, gw = self.net.preprocess(crops, m)
                assert (gh, gw) == (nh, nw)
                heat = torch.empty((n, 22, nh // 8, nw // 8), device=crops.device)
                self.net.run(heat)
            crops.record_stream(st)
            heat.record_stream(cur)
            heats[i] = heat
        rt.join_streams(cur, streams)
        geoms = [(nh, nw, vh, vw) for (m, nh, nw, vh, vw) in sg]
        return geoms, heats

    def post_maps(self, h, w, geoms, heats, out=None):
        """isl_hand_post on low-res maps [n,22,h8,w8] per scale -> int64 [n,21,2]; with
        `out` (a cuda tensor) the result is written there and not synchronised."""
        import torch
        n = heats[0].shape[0]
        ns = len(geoms)
        dst = out if out is not None else torch.empty((n, 21, 2), dtype=torch.int64, device=heats[0].device)
        g = (rt.IslScaleGeom * ns)(*[rt.IslScaleGeom(*gg) for gg in geoms])
        hp = (ctypes.c_void_p * ns)(*[rt.ptr(t).value for t in heats])
        rt.check(rt.lib().isl_hand_post(self.net.h, n, h, w, ns, g, hp, rt.ptr(dst), rt.stream_handle()),
                 "isl_hand_post")
        return None if out is not None else dst.cpu().numpy()

    def estimate_crops(self, frames, boxes):
        """Batched Hand.__call__ over crops of different sizes: frames uint8 [n,H,W,3]
        (numpy or torch), boxes [(frame_index, x, y, w)] (util.handDetect's square boxes,
        oriImg[y:y+w, x:x+w]) -> int64 [len(boxes), 21, 2] in crop coordinates, equal to
        estimate() on each crop.  The 4 scales run as one batch of all crops each (every
        crop resizes to round(s*368) px); the post runs per crop (its resize-back target
        is the crop size)."""
        import torch
        if len(boxes) == 0:
            return np.zeros((0, 21, 2), np.int64)
        t = torch.as_tensor(np.ascontiguousarray(frames) if isinstance(frames, np.ndarray) else frames)
        t = t.to("cuda:%d" % self.device).contiguous()
        out = []
        # bounded batches: the 736 px scale costs ~0.4 GB of activations per crop
        for c in range(0, len(boxes), CROP_CHUNK):
            part = boxes[c:c + CROP_CHUNK]
            peaks = self.post_crops(part, self.run_crops(t, part))
            if not self.net.range_ok():
                with self.net.algo_scope("direct"):
                    peaks = self.post_crops(part, self.run_crops(t, part))
            out.append(peaks)
        return np.concatenate(out)

    def run_crops(self, frames_t, boxes):
        """The hand net over all crops, one batch per scale -> low-res heat [n,22,h8,w8] per
        scale.  The scales run side by side on the streams of rt.lane_plan (three lanes, the
        largest scales first), forked from the current stream and joined back (every scale
        has its own arena, table and split-K workspace in the net): the small scales' grids
        fill the CUs the large ones leave idle."""
        import torch
        crops = [(f, x, y, w, w) for (f, x, y, w) in boxes]
        cur = torch.cuda.current_stream(frames_t.device)
        # one lane per net size at most (scales that pad to one size share its arena)
        keys = [rt.crop_net_size(crops[0][4], crops[0][3], s * BOXSIZE) for s in self.scale_search]
        streams, order = rt.lane_plan(self, frames_t.device, keys)
        rt.fork_streams(cur, streams)
        heats = [None] * len(keys)
        for i in order:
            st, s = streams[i], self.scale_search[i]
            with torch.cuda.stream(st):
                gh, gw = self.net.preprocess_crops(frames_t, crops, s * BOXSIZE)
                heat = torch.empty((len(crops), 22, gh // 8, gw // 8), device=frames_t.device)
                self.net.run(heat)
            frames_t.record_stream(st)
            heat.record_stream(cur)
            heats[i] = heat
        rt.join_streams(cur, streams)
        return heats

    def launch_crops(self, frames_t, boxes):
        """Enqueue estimate_crops() on the current stream without waiting (nets, posts,
        peaks to pinned host memory, stream-ordered range check); finish_crops(job)
        completes it."""
        import torch
        if not boxes:      # nothing to enqueue (and no flag copy left in flight into a freed buffer)
            return dict(t=frames_t, boxes=boxes, parts=[], flag=None, ev=None)
        parts = []
        for c in range(0, len(boxes), CROP_CHUNK):
            part = boxes[c:c + CROP_CHUNK]
            heats = self.run_crops(frames_t, part)
            out = self._post_crops_dev(part, heats)
            host = torch.empty(out.shape, dtype=torch.int64, pin_memory=True)
            host.copy_(out, non_blocking=True)
            parts.append((part, heats, out, host))
        flag = rt.flag_slot(self)
        self.net.check_async(flag)
        ev = torch.cuda.Event()
        ev.record()
        return dict(t=frames_t, boxes=boxes, parts=parts, flag=flag, ev=ev)

    def finish_crops(self, job):
        if not job["boxes"]:
            return np.zeros((0, 21, 2), np.int64)
        job["ev"].synchronize()
        if int(job["flag"][0]) != 0:     # split-fp16 range left: the whole call again on fp32
            with self.net.algo_scope("direct"):
                return np.concatenate([self.post_crops(part, self.run_crops(job["t"], part))
                                       for part, _, _, _ in job["parts"]])
        return np.concatenate([host.numpy() for _, _, _, host in job["parts"]])

    def post_crops(self, boxes, heats):
        """isl_hand_post per crop (its resize-back target is the crop size) -> int64 [n,21,2]."""
        return self._post_crops_dev(boxes, heats).cpu().numpy()

    def _post_crops_dev(self, boxes, heats):
        import torch
        n, ns = len(boxes), len(heats)
        out = torch.empty((n, 21, 2), dtype=torch.int64, device=heats[0].device)
        # one call: the crops' kernel chains run side by side on the net's post streams
        ws = (ctypes.c_int32 * n)(*[b[3] for b in boxes])
        g = (rt.IslScaleGeom * (n * ns))()
        for i, b in enumerate(boxes):
            geoms = [gg[1:] for gg in scale_geometry(b[3], b[3], self.scale_search)]
            assert all((gg[0], gg[1]) == (hh.shape[2] * 8, hh.shape[3] * 8) for gg, hh in zip(geoms, heats))
            for si, gg in enumerate(geoms):
                g[i * ns + si] = rt.IslScaleGeom(*gg)
        assert all(hh.is_contiguous() for hh in heats)
        hp = (ctypes.c_void_p * ns)(*[rt.ptr(hh).value for hh in heats])
        rt.check(rt.lib().isl_hand_post_crops(self.net.h, n, ws, ns, g, hp, rt.ptr(out), rt.stream_handle()),
                 "isl_hand_post_crops")
        return out

    def estimate(self, crops):
        """crops: uint8 [n,h,w,3] or one [h,w,3] (numpy or torch) -> int64 [n,21,2] / [21,2]."""
        import torch
        single = crops.ndim == 3
        t = torch.as_tensor(np.ascontiguousarray(crops) if isinstance(crops, np.ndarray) else crops)
        if single:
            t = t[None]
        t = t.to("cuda:%d" % self.device).contiguous()
        n, h, w, _ = t.shape
        geoms, heats = self.run_scales(t)
        peaks = self.post_maps(h, w, geoms, heats)
        if not self.net.range_ok():
            # split-fp16 range exceeded: recompute the crops on the fp32 kernels
            with self.net.algo_scope("direct"):
                geoms, heats = self.run_scales(t)
                peaks = self.post_maps(h, w, geoms, heats)
        return peaks[0] if single else peaks
