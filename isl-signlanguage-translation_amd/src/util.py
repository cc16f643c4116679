"""Drop-in for the reference's src/util.py: the helpers on and around the hot path.

Follows /root/reference/src/util.py:
  padRightDownCorner 12-32, transfer 35-44, get_bodypose 99-151,
  get_handpose 187-219, handDetect 242-306, npmax 394-399.
The drawing helpers (draw_bodypose, draw_handpose, draw_handpose_by_opencv,
drawStickmodel, crop_to_drawing; util.py:47-96,154-185,222-238,308-391) render with
OpenCV/matplotlib after the path and are out of scope of the engine (SURVEY §2 row
5): they call the reference's own util.py (the original ``src`` this package falls
through to, see src/__init__.py), so extract_features_mp.py's ``test = True``
rendering (:57, :90) works where the reference's dependencies are installed.
Without the original ``src`` they raise NotImplementedError.
"""
from __future__ import annotations

import math

import numpy as np

BODY25_LIMBS = [[1, 0], [1, 2], [2, 3], [3, 4], [1, 5], [5, 6], [6, 7], [1, 8], [8, 9], [9, 10],
                [10, 11], [8, 12], [12, 13], [13, 14], [0, 15], [0, 16], [15, 17], [16, 18],
                [11, 24], [11, 22], [14, 21], [14, 19], [22, 23], [19, 20]]
COCO_LIMBS = [[1, 2], [1, 5], [2, 3], [3, 4], [5, 6], [6, 7], [1, 8], [8, 9], [9, 10], [1, 11],
              [11, 12], [12, 13], [1, 0], [0, 14], [14, 16], [0, 15], [15, 17], [2, 16], [5, 17]]
HAND_EDGES = [[0, 1], [1, 2], [2, 3], [3, 4], [0, 5], [5, 6], [6, 7], [7, 8], [0, 9], [9, 10], [10, 11],
              [11, 12], [0, 13], [13, 14], [14, 15], [15, 16], [0, 17], [17, 18], [18, 19], [19, 20]]


def padRightDownCorner(img, stride, padValue):
    """Pad bottom/right to a multiple of `stride` with `padValue`; returns (img_padded, pad[4])."""
    h, w = img.shape[0], img.shape[1]
    pad = [0, 0, 0 if h % stride == 0 else stride - h % stride, 0 if w % stride == 0 else stride - w % stride]
    out = np.empty((h + pad[2], w + pad[3]) + img.shape[2:], dtype=img.dtype)
    out[...] = padValue
    out[:h, :w] = img
    return out, pad


def transfer(model, model_weights):
    """Map the flat caffe-named weight dict onto model.state_dict() keys (KeyError if absent)."""
    out = {}
    for k in model.state_dict().keys():
        parts = k.split(".")
        out[k] = model_weights[".".join(parts[3:]) if len(parts) > 4 else ".".join(parts[1:])]
    return out


def npmax(array):
    """(row, col) of the first raster-order maximum."""
    arrayindex = array.argmax(1)
    arrayvalue = array.max(1)
    i = arrayvalue.argmax()
    return i, arrayindex[i]


def handDetect(candidate, subset, oriImg):
    """Hand boxes [[x, y, w, is_left], ...] from arm keypoints (left hand first per person)."""
    ratio = 0.33
    H, W = oriImg.shape[0:2]
    result = []
    for person in subset.astype(int):
        has_left = np.sum(person[[5, 6, 7]] == -1) == 0
        has_right = np.sum(person[[2, 3, 4]] == -1) == 0
        if not (has_left or has_right):
            continue
        arms = []
        if has_left:
            arms.append((person[[5, 6, 7]], True))
        if has_right:
            arms.append((person[[2, 3, 4]], False))
        for (i1, i2, i3), is_left in arms:
            x1, y1 = candidate[i1][:2]
            x2, y2 = candidate[i2][:2]
            x3, y3 = candidate[i3][:2]
            x = x3 + ratio * (x3 - x2)
            y = y3 + ratio * (y3 - y2)
            d_we = math.sqrt((x3 - x2) ** 2 + (y3 - y2) ** 2)
            d_es = math.sqrt((x2 - x1) ** 2 + (y2 - y1) ** 2)
            width = 1.5 * max(d_we, 0.9 * d_es)
            x -= width / 2
            y -= width / 2
            if x < 0:
                x = 0
            if y < 0:
                y = 0
            w1 = w2 = width
            if x + width > W:
                w1 = W - x
            if y + width > H:
                w2 = H - y
            width = min(w1, w2)
            if width >= 20:
                result.append([int(x), int(y), int(width), is_left])
    return result


def get_bodypose(candidate, subset, model_type="coco"):
    """Export tuples: ([(x, y) per present joint], [(mY, mX, angle, length) per present limb])."""
    limbs, njoint = (BODY25_LIMBS, 25) if model_type == "body25" else (COCO_LIMBS, 18)
    circles = []
    for i in range(njoint):
        for n in range(len(subset)):
            index = int(subset[n][i])
            if index == -1:
                continue
            x, y = candidate[index][0:2]
            circles.append((x, y))
    sticks = []
    for i in range(njoint - 1):
        for n in range(len(subset)):
            index = subset[n][np.array(limbs[i])]
            if -1 in index:
                continue
            Y = candidate[index.astype(int), 0]
            X = candidate[index.astype(int), 1]
            mX = np.mean(X)
            mY = np.mean(Y)
            length = ((X[0] - X[1]) ** 2 + (Y[0] - Y[1]) ** 2) ** 0.5
            angle = math.degrees(math.atan2(X[0] - X[1], Y[0] - Y[1]))
            sticks.append((mY, mX, angle, length))
    return (circles, sticks)


def get_handpose(all_hand_peaks, show_number=False):
    """Export tuples for (at most two) hands: (edges, peaks); a third hand raises IndexError
    exactly like the reference (its export lists have two slots)."""
    export_edges, export_peaks = [[], []], [[], []]
    for idx, peaks in enumerate(all_hand_peaks):
        for ie, e in enumerate(HAND_EDGES):
            if np.sum(np.all(peaks[e], axis=1) == 0) == 0:
                x1, y1 = peaks[e[0]]
                x2, y2 = peaks[e[1]]
                export_edges[idx].append((ie, (x1, y1), (x2, y2)))
        for i, kp in enumerate(peaks):
            x, y = kp
            export_peaks[idx].append((x, y, str(i)))
    return (export_edges, export_peaks)


_reference_util = None


def reference_util():
    """The reference's own util module (drawing helpers), loaded from the original
    ``src`` directory under a private name; None when the original is not found."""
    global _reference_util
    if _reference_util is None:
        import importlib.util
        import os
        from . import reference_src
        d = reference_src()
        if d is None or not os.path.isfile(os.path.join(d, "util.py")):
            return None
        spec = importlib.util.spec_from_file_location("src._reference_util", os.path.join(d, "util.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _reference_util = mod
    return _reference_util


def _drawing(name):
    def fn(*args, **kwargs):
        ref = reference_util()
        if ref is None:
            raise NotImplementedError(
                "%s renders with OpenCV/matplotlib and is out of scope of the MI355X engine; it runs from the "
                "reference's own src/util.py, which was not found (set ISLPOSE_REFERENCE_SRC or keep the original "
                "src as src.orig)" % name)
        return getattr(ref, name)(*args, **kwargs)
    fn.__name__ = name
    return fn


draw_bodypose = _drawing("draw_bodypose")
draw_handpose = _drawing("draw_handpose")
draw_handpose_by_opencv = _drawing("draw_handpose_by_opencv")
drawStickmodel = _drawing("drawStickmodel")
crop_to_drawing = _drawing("crop_to_drawing")
