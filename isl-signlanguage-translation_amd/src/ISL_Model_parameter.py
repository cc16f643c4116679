"""Keras-free drop-in for the reference's ISLSignPos (src/ISL_Model_parameter.py:41-306).

``ISLSignPos(pt_body_model, pt_hand_model)`` takes the networks of ``Body(...).model``
and ``Hand(...).model`` exactly like the reference (extract_features_mp.py:162-164)
and ``call(oriImg)`` returns ``(candidate, subset, all_hand_peaks)``:
body pose (body25, scale_search [0.5], ISL_Model_parameter.py:62-254), handDetect,
then hand peaks per crop offset into frame coordinates (:51-60, 256-306).
Everything runs on the GPU through libislpose; there is no keras dependency.

``call_batch(frames)`` runs the body path for a whole batch of frames at once.

Out of scope: ``ISLSignPosTranslator`` (the Keras BiLSTM sign
classifier, :308-689) and the ffmpeg ``Writer`` -- constructing them raises.
"""
from __future__ import annotations

import numpy as np
import torch

from islpose.body import BodyEstimator
from islpose.hand import HandEstimator

from . import util


def _as_numpy(img):
    return img.cpu().numpy() if isinstance(img, torch.Tensor) else np.asarray(img)


class ISLSignPos(object):
    def __init__(self, pt_body_model, pt_hand_model):
        self.pt_body = pt_body_model
        self.pt_hand = pt_hand_model
        self.njoint_body = 26
        self.npaf_body = 52
        self._body = None
        self._hand = None

    def _estimators(self):
        dev = torch.cuda.current_device()
        bnet, hnet = self.pt_body.native(dev), self.pt_hand.native(dev)
        if self._body is None or self._body.net is not bnet:
            self._body = BodyEstimator(model_type="body25", device=dev, scale_search=(0.5,), net=bnet)
        if self._hand is None or self._hand.net is not hnet:
            self._hand = HandEstimator(device=dev, net=hnet)
        return self._body, self._hand

    def bodypos(self, oriImg):
        return self._estimators()[0].estimate(np.ascontiguousarray(_as_numpy(oriImg), dtype=np.uint8))

    def handpos(self, oriImg):
        return self._estimators()[1].estimate(np.ascontiguousarray(_as_numpy(oriImg), dtype=np.uint8))

    def _hands(self, img, candidate, subset):
        out = []
        for x, y, w, is_left in util.handDetect(candidate, subset, img):
            peaks = self.handpos(img[y:y + w, x:x + w, :])
            peaks[:, 0] = np.where(peaks[:, 0] == 0, peaks[:, 0], peaks[:, 0] + x)
            peaks[:, 1] = np.where(peaks[:, 1] == 0, peaks[:, 1], peaks[:, 1] + y)
            out.append(peaks)
        return out

    def call(self, oriImg):
        img = _as_numpy(oriImg)
        candidate, subset = self.bodypos(img)
        return (candidate, subset, self._hands(img, candidate, subset))

    __call__ = call

    def call_batch(self, frames):
        """frames uint8 [n, H, W, 3] -> [(candidate, subset, all_hand_peaks)] * n, equal to
        call() per frame.  The body runs as one batch; every hand crop of the batch
        (util.handDetect boxes, in the reference's order) runs as one batch per scale."""
        frames = np.ascontiguousarray(_as_numpy(frames), dtype=np.uint8)
        body, hand = self._estimators()
        t = torch.from_numpy(frames).to("cuda:%d" % body.device)
        res = body.estimate(t)
        boxes, owner = [], []
        for i, (c, s) in enumerate(res):
            for x, y, w, _is_left in util.handDetect(c, s, frames[i]):
                boxes.append((i, x, y, w))
                owner.append(i)
        peaks = hand.estimate_crops(t, boxes)
        out = [(c, s, []) for (c, s) in res]
        for (i, x, y, _w), pk in zip(boxes, peaks):
            pk = pk.copy()
            pk[:, 0] = np.where(pk[:, 0] == 0, pk[:, 0], pk[:, 0] + x)   # ISL_Model_parameter.py:56-59
            pk[:, 1] = np.where(pk[:, 1] == 0, pk[:, 1], pk[:, 1] + y)
            out[i][2].append(pk)
        return out


class ISLSignPosTranslator(object):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("ISLSignPosTranslator (Keras BiLSTM sign classifier) is outside the MI355X "
                                  "keypoint engine; use ISLSignPos for the keypoints")


class Writer(object):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("ffmpeg video writing is out of scope")
