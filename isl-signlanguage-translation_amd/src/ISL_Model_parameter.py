"""Keras-free drop-in for the reference's ISLSignPos (src/ISL_Model_parameter.py:41-306).

``ISLSignPos(pt_body_model, pt_hand_model)`` takes the networks of ``Body(...).model``
and ``Hand(...).model`` exactly like the reference (extract_features_mp.py:162-164)
and ``call(oriImg)`` returns ``(candidate, subset, all_hand_peaks)``:
body pose (body25, scale_search [0.5], ISL_Model_parameter.py:62-254), handDetect,
then hand peaks per crop offset into frame coordinates (:51-60, 256-306).
Everything runs on the GPU through libislpose; there is no keras dependency.

``call_batch(frames)`` runs the body path for a whole batch of frames at once.

``ISLSignPosTranslator(body_model, hand_model, translation_model)`` (:308-443)
turns a 20-frame window into [1, 20, 156] ``populate_features`` rows and applies
``translation_model`` -- a keras-free ``islpose.translate.SignClassifier`` (one
HIP launch, csrc/sign.hip) or any callable taking that array.
``translate_stream(frames)`` is the batched form of the demo's rolling-window loop
(demo_isl_translate.py:170-197): keypoints once per frame, every window classified
in one launch.

Out of scope: the ffmpeg ``Writer`` -- constructing it raises.
"""
from __future__ import annotations

import collections
import os

import numpy as np
import torch
import xxhash

from islpose import translate
from islpose.body import BodyEstimator
from islpose.hand import HandEstimator

from . import util

# the per-frame calls replay each net's conv chain as a HIP graph (bit-identical to the eager
# launches, tests/test_gpu_wino2.py, test_gpu_body.py): one host call per run instead of
# ~50-150 kernel launches, so the four hand scales' streams start together.  (body, hand);
# ISLPOSE_FRAME_GRAPH="10" etc. overrides (A/B)
_fg = os.environ.get("ISLPOSE_FRAME_GRAPH", "11")
GRAPH_REPLAY = (_fg[:1] == "1", _fg[1:2] == "1")


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
        self._device = None          # pinned by .to(); default: the current HIP device

    def to(self, device):
        """Pin the HIP device the keypoint nets run on and return self: the reference
        class is a keras.Model, and extract_features_mp.py:150 / extract_featuressingle.py
        :150 call ``model.to(device)``.  A CPU device leaves the placement unchanged
        (the engine runs on the GPU only)."""
        d = torch.device(device)
        if d.type == "cuda":
            self._device = d.index if d.index is not None else torch.cuda.current_device()
        return self

    def _estimators(self):
        dev = self._device if self._device is not None else torch.cuda.current_device()
        bnet, hnet = self.pt_body.native(dev), self.pt_hand.native(dev)
        if self._body is None or self._body.net is not bnet:
            self._body = BodyEstimator(model_type="body25", device=dev, scale_search=(0.5,), net=bnet)
            bnet.set_graph(GRAPH_REPLAY[0])
        if self._hand is None or self._hand.net is not hnet:
            self._hand = HandEstimator(device=dev, net=hnet)
            hnet.set_graph(GRAPH_REPLAY[1])
        return self._body, self._hand

    def state_key(self):
        """Identity of what produces the keypoints: the two modules, their current
        parameters (storage and in-place version, as _NativeNet.native() tracks them)
        and the native nets' split-K state."""
        def part(m):
            if m is None:
                return (None,)
            net = getattr(m, "_native_net", None)
            return (id(m), tuple((p.data_ptr(), p._version) for p in m.parameters()),
                    getattr(net, "split_k", None))
        return part(self.pt_body) + part(self.pt_hand)

    def bodypos(self, oriImg):
        return self._estimators()[0].estimate(np.ascontiguousarray(_as_numpy(oriImg), dtype=np.uint8))

    def handpos(self, oriImg):
        return self._estimators()[1].estimate(np.ascontiguousarray(_as_numpy(oriImg), dtype=np.uint8))

    def call(self, oriImg):
        """ISL_Model_parameter.py:51-60 on one frame (the extract_features_mp.py:125-130 /
        demo pattern): body pose, handDetect, hand peaks per crop offset into the frame.  The
        frame goes to the GPU once (_upload) and every hand crop of it runs as one batch per
        scale (HandEstimator.estimate_crops) instead of one 4-scale chain per crop in turn; the
        results equal the reference's per-crop handpos (tests/test_gpu_configs.py)."""
        ests = self._estimators()   # (once per call: it checks both modules' parameters)
        return self.call_batch(self._upload(oriImg, ests), ests)[0]

    def _upload(self, img, ests=None):
        """One host frame [H, W, 3] -> cuda uint8 [1, H, W, 3] BGR.  The scripts pass
        frame[:, :, ::-1] of a decoded RGB frame (extract_features_mp.py:130): that view is
        uploaded as the contiguous RGB buffer it reverses and flipped on the GPU, not copied
        into a contiguous BGR array on the host first; the copy goes through a reused pinned
        buffer (one memcpy, then a DMA) instead of a pageable upload."""
        body = (ests or self._estimators())[0]
        dev = torch.device("cuda:%d" % body.device)
        if isinstance(img, torch.Tensor) and img.is_cuda:
            # any dtype, as the host path's np.ascontiguousarray(..., dtype=np.uint8)
            return img.to(dev).to(torch.uint8).contiguous()[None]
        a = _as_numpy(img)
        flip = a.ndim == 3 and a.shape[2] == 3 and a.strides[2] < 0 and a[:, :, ::-1].flags.c_contiguous
        src = np.ascontiguousarray(a[:, :, ::-1] if flip else a, dtype=np.uint8)
        buf = getattr(self, "_pinned", None)
        if buf is None or buf.numel() < src.size:
            buf = self._pinned = torch.empty(src.size, dtype=torch.uint8, pin_memory=True)
            self._pinned_ev = None
        if self._pinned_ev is not None:
            self._pinned_ev.synchronize()          # the previous upload has left the buffer
        host = buf[:src.size].view(src.shape)
        host.copy_(torch.from_numpy(src))          # (torch's copy runs on the host's threads)
        # (in row bands, each band's DMA beside the next band's copy: measured level, 268 vs
        # 287 us for 1 / 4 bands of a 1080p frame, tools/upload_micro.py -- the copy is 16 us)
        t = host.to(dev, non_blocking=True)
        self._pinned_ev = torch.cuda.Event()
        self._pinned_ev.record(torch.cuda.current_stream(dev))
        return (t.flip(-1) if flip else t)[None]

    __call__ = call

    def call_batch(self, frames, ests=None):
        """frames uint8 [n, H, W, 3] -> [(candidate, subset, all_hand_peaks)] * n, equal to
        call() per frame.  The body runs as one batch; every hand crop of the batch
        (util.handDetect boxes, in the reference's order) runs as one batch per scale."""
        body, hand = ests or self._estimators()
        if isinstance(frames, torch.Tensor) and frames.is_cuda:
            # already resident (islpose.pipeline's prefetch: async H2D on a copy stream)
            if frames.dtype != torch.uint8 or frames.ndim != 4 or frames.shape[3] != 3:
                raise ValueError("frames: uint8 [n, H, W, 3] expected, got %s %s" % (frames.dtype, tuple(frames.shape)))
            t = frames.contiguous()
        else:
            t = torch.from_numpy(np.ascontiguousarray(_as_numpy(frames), dtype=np.uint8)).to("cuda:%d" % body.device)
        res = body.estimate(t)
        boxes = []
        for i, (c, s) in enumerate(res):
            # handDetect reads only the frame's shape (util.py:245)
            for x, y, w, _is_left in util.handDetect(c, s, t[i]):
                boxes.append((i, x, y, w))
        peaks = hand.estimate_crops(t, boxes)
        return self._assemble(res, boxes, peaks)

    @staticmethod
    def _assemble(res, boxes, peaks):
        out = [(c, s, []) for (c, s) in res]
        for (i, x, y, _w), pk in zip(boxes, peaks):
            pk = pk.copy()
            pk[:, 0] = np.where(pk[:, 0] == 0, pk[:, 0], pk[:, 0] + x)   # ISL_Model_parameter.py:56-59
            pk[:, 1] = np.where(pk[:, 1] == 0, pk[:, 1], pk[:, 1] + y)
            out[i][2].append(pk)
        return out

    def call_batches(self, batches):
        """call_batch over an iterable of (key, frames) -- frames cuda uint8 [n, H, W, 3]
        BGR, ready on the current stream -- yielding (key, results) in order, the same
        results as call_batch.  Software-pipelined across batches on two streams: the
        body net and post of batch k run while the hand nets and posts of batch k-1 do,
        so one phase's small grids fill the CUs the other leaves idle."""
        body, hand = self._estimators()
        dev = torch.device("cuda:%d" % body.device)
        cur = torch.cuda.current_stream(dev)
        if getattr(self, "_pipe_streams", None) is None:
            self._pipe_streams = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
        sb, sh = self._pipe_streams
        prev = None                                  # (key, body results, boxes, hand job)
        for key, t in batches:
            sb.wait_stream(cur)
            with torch.cuda.stream(sb):
                bjob = body.launch(t)
            t.record_stream(sb)
            if prev is not None:                     # its hands ran beside this body
                yield prev[0], self._assemble(prev[1], prev[2], hand.finish_crops(prev[3]))
            res = body.finish(bjob)
            boxes = [(i, x, y, w) for i, (c, s) in enumerate(res) for x, y, w, _l in util.handDetect(c, s, t[i])]
            sh.wait_stream(cur)
            with torch.cuda.stream(sh):
                hjob = hand.launch_crops(t, boxes)
            t.record_stream(sh)
            prev = (key, res, boxes, hjob)
        if prev is not None:
            yield prev[0], self._assemble(prev[1], prev[2], hand.finish_crops(prev[3]))


class ISLSignPosTranslator(ISLSignPos):
    window_size = translate.WINDOW

    cache_frames = 64   # per-frame feature rows kept for overlapping windows

    def __init__(self, body_model, hand_model, translation_model):
        super().__init__(body_model, hand_model)
        self.model_type = 'body25'
        self.translation_layer = translation_model
        self._rows = collections.OrderedDict()
        self._rows_key = None

    def populate_features(self, bodypose_circles, handpose_peaks):
        return translate.populate_features(bodypose_circles, handpose_peaks)

    def frame_features(self, candidate, subset, all_hand_peaks):
        """One frame's 156-d row (ISL_Model_parameter.py:320-329): export tuples, then
        populate_features.  More than two hands raises IndexError (get_handpose), as in
        the reference."""
        circles, _ = util.get_bodypose(candidate, subset, self.model_type)
        _, peaks = util.get_handpose(all_hand_peaks)
        return self.populate_features(circles, peaks)

    def features(self, frames, batch: int = 32):
        """[T, H, W, 3] uint8 BGR frames -> [T, 156] rows (body + hand keypoints in GPU batches)."""
        frames = _as_numpy(frames)
        rows = []
        for s in range(0, len(frames), batch):
            rows.extend(self.frame_features(*r) for r in self.call_batch(frames[s:s + batch]))
        return np.array(rows, dtype=np.float64).reshape(len(rows), translate.N_FEATURES)

    def cached_features(self, frames):
        """Feature rows of frames, reusing the rows of frames seen in recent calls (keyed by
        a 128-bit hash of the pixels): the demo's rolling window (demo_isl_translate.py:
        183-190) shares 19 of its 20 frames with the previous call, so only the new frame
        goes through the keypoint nets.  The cache is dropped whenever the nets, their
        weights or their split-K state change (ISLSignPos.state_key), so rows are those of
        computing them afresh (up to the range guard: a batch recomputed on the fp32
        kernels gives rows within the fp32 tolerance, not the same bits)."""
        state = self.state_key()
        if self._rows_key != state:
            self._rows.clear()
            self._rows_key = state
        keys = [(f.shape, xxhash.xxh3_128_digest(np.ascontiguousarray(f))) for f in frames]
        miss = [i for i, k in enumerate(keys) if k not in self._rows]
        if miss:
            res = self.call_batch(np.stack([frames[i] for i in miss]))
            for i, r in zip(miss, res):
                self._rows[keys[i]] = self.frame_features(*r)
        rows = []
        for k in keys:
            self._rows.move_to_end(k)
            rows.append(self._rows[k])
        while len(self._rows) > max(self.cache_frames, len(frames)):
            self._rows.popitem(last=False)
        return rows

    def call(self, window):
        """ISL_Model_parameter.py:318-337: window [20, H, W, 3] -> translation_model of the
        [1, 20, 156] feature window.  Shorter windows fail as in the reference, whose
        padding branch reads ``.shape`` of a list (:331-333); longer ones fail its reshape."""
        frames = _as_numpy(window)
        feats = self.cached_features(frames) if len(frames) else []
        if len(feats) < self.window_size:
            raise AttributeError("'list' object has no attribute 'shape'")
        return self.translation_layer(np.array(feats).reshape(1, self.window_size, translate.N_FEATURES))

    __call__ = call

    def translate_stream(self, frames, batch: int = 32):
        """Every full window of a clip: row s = translation_model(features[s:s+20]), the
        result call(frames[s:s+20]) gives, for s = 0 .. T-20.  Keypoints run once per
        frame instead of 20 times, and all windows go to the classifier together.
        (The demo's loop classifies s >= 1: it fills the window before its first call.)"""
        wins = translate.sliding_windows(self.features(frames, batch), self.window_size)
        if len(wins) == 0:
            return wins
        return self.translation_layer(wins)

    def frame_to_window(self, frame):
        """ISL_Model_parameter.py:353-374: shift self.window by one and append frame
        (self.window must have been set by the caller, as in the reference)."""
        self.window[:-1] = self.window[1:]
        self.window[-1] = frame


class Writer(object):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("ffmpeg video writing is out of scope")
