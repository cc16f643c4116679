"""Drop-in for the reference's src/hand.py: ``Hand(model_path)(oriImg) -> int64 [21, 2]``.

Same constructor (hand.py:16-22) and call (hand.py:24-74): 4-scale pyramid,
fp64 averaging, blur, connected components, largest-mass component, first
maximum -- all on the GPU (on a host without a visible HIP device, on the CPU: islpose.cpu).  ``estimate_batch(crops)`` takes equal-size crops.
"""
from __future__ import annotations

import numpy as np
import torch

from islpose import cpu
from islpose.hand import HandEstimator

from . import util
from .model import handpose_model


class Hand(object):
    def __init__(self, model_path):
        self.model = handpose_model()
        if torch.cuda.is_available():
            self.model = self.model.cuda()
        weights = model_path if isinstance(model_path, dict) else torch.load(model_path, map_location="cpu",
                                                                            weights_only=True)
        self.model.load_state_dict(util.transfer(self.model, weights))
        self.model.eval()
        self._est = None

    def estimator(self) -> HandEstimator:
        dev = torch.cuda.current_device()
        net = self.model.native(dev)
        if self._est is None or self._est.net is not net:
            self._est = HandEstimator(device=dev, net=net)
        return self._est

    def __call__(self, oriImg):
        img = oriImg.cpu().numpy() if isinstance(oriImg, torch.Tensor) else np.asarray(oriImg)
        img = np.ascontiguousarray(img, dtype=np.uint8)
        if not torch.cuda.is_available():   # GPU-less host: the product's CPU path (hand.py:18-20)
            return cpu.hand_call(img, self._cpu_net)
        return self.estimator().estimate(img)

    def _cpu_net(self, im):
        with torch.no_grad():
            return self.model(torch.from_numpy(im)).numpy()

    def estimate_batch(self, crops):
        if not torch.cuda.is_available():
            return [self(c) for c in crops]
        return self.estimator().estimate(crops)
