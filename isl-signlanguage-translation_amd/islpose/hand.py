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
from .body import scale_geometry

HAND_SCALES = (0.5, 1.0, 1.5, 2.0)


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
        geoms, heats = [], []
        for (m, nh, nw, vh, vw) in scale_geometry(h, w, self.scale_search):
            gh, gw = self.net.preprocess(crops, m)
            assert (gh, gw) == (nh, nw)
            heat = torch.empty((n, 22, nh // 8, nw // 8), device=crops.device)
            self.net.run(heat)
            geoms.append((nh, nw, vh, vw))
            heats.append(heat)
        return geoms, heats

    def post_maps(self, h, w, geoms, heats):
        import torch
        n = heats[0].shape[0]
        ns = len(geoms)
        out = torch.empty((n, 21, 2), dtype=torch.int64, device=heats[0].device)
        g = (rt.IslScaleGeom * ns)(*[rt.IslScaleGeom(*gg) for gg in geoms])
        hp = (ctypes.c_void_p * ns)(*[rt.ptr(t).value for t in heats])
        rt.check(rt.lib().isl_hand_post(self.net.h, n, h, w, ns, g, hp, rt.ptr(out), rt.stream_handle()),
                 "isl_hand_post")
        return out.cpu().numpy()

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
