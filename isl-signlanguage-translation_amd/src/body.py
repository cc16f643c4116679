"""Drop-in for the reference's src/body.py: ``Body(model_path, model_type)``.

Same constructor (body.py:16-37: model_type 'coco' | 'body25', anything else
prints a message and falls back to COCO; weights through util.transfer) and
the same call (body.py:39-235): ``Body(...)(oriImg) -> (candidate, subset)``
with identical dtypes, shapes and values.  The whole call runs on the GPU
(pre-processing, network, resize, blur/NMS, PAF, assembly) -- on a host without a
visible HIP device, on the CPU instead (islpose.cpu, as the reference); ``scale_search``
defaults to the reference's [0.5] and can be changed per instance.
``estimate_batch(frames)`` processes a batch of frames in one pass.
"""
from __future__ import annotations

import numpy as np
import torch

from islpose import cpu
from islpose.body import BodyEstimator

from . import util
from .model import bodypose_25_model, bodypose_model


class Body(object):
    def __init__(self, model_path, model_type="coco"):
        if model_type == "coco":
            self.model, self.njoint, self.npaf = bodypose_model(), 19, 38
        elif model_type == "body25":
            self.model, self.njoint, self.npaf = bodypose_25_model(), 26, 52
        else:
            print("not right model_type, use coco")
            self.model, self.njoint, self.npaf = bodypose_model(), 19, 38
        self.model_type = model_type
        if torch.cuda.is_available():
            self.model = self.model.cuda()
        weights = model_path if isinstance(model_path, dict) else torch.load(model_path, map_location="cpu",
                                                                            weights_only=True)
        self.model.load_state_dict(util.transfer(self.model, weights))
        self.model.eval()
        self.scale_search = [0.5]          # body.py:41
        self._est = None

    def estimator(self) -> BodyEstimator:
        dev = torch.cuda.current_device()
        net = self.model.native(dev)
        kind = "body25" if self.model_type == "body25" else "coco"
        if self._est is None or self._est.net is not net or self._est.scale_search != tuple(self.scale_search):
            self._est = BodyEstimator(model_type=kind, device=dev, scale_search=self.scale_search, net=net)
        return self._est

    def __call__(self, oriImg):
        img = oriImg.cpu().numpy() if isinstance(oriImg, torch.Tensor) else np.asarray(oriImg)
        img = np.ascontiguousarray(img, dtype=np.uint8)
        if not torch.cuda.is_available():   # GPU-less host: the product's CPU path (body.py:31-32)
            return cpu.body_call(img, self._cpu_net, "body25" if self.model_type == "body25" else "coco",
                                 tuple(self.scale_search))
        return self.estimator().estimate(img)

    def _cpu_net(self, im):
        with torch.no_grad():
            return tuple(o.numpy() for o in self.model(torch.from_numpy(im)))

    def estimate_batch(self, frames):
        """frames: uint8 [n, H, W, 3] (numpy or torch, BGR) -> [(candidate, subset)] * n."""
        if not torch.cuda.is_available():
            return [self(f) for f in frames]
        return self.estimator().estimate(frames)
