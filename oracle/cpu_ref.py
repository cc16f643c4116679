"""CPU restatement of the reference hot path (networks + body/hand post-processing).

ORACLE — test infrastructure only (see oracle/__init__.py).  The product path
never imports this module.

Follows, function by function:
  * networks            /root/reference/src/model.py:66-407
  * Body.__call__       /root/reference/src/body.py:39-235
  * Hand.__call__       /root/reference/src/hand.py:24-74
  * padRightDownCorner  /root/reference/src/util.py:12-32
  * handDetect          /root/reference/src/util.py:242-306
  * npmax               /root/reference/src/util.py:394-399
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from . import cv_resize

# ---------------------------------------------------------------------------
# networks (torch CPU fp32), restating src/model.py
# ---------------------------------------------------------------------------


class _Params:
    """caffe-named weight dict -> torch tensors (the flat format util.transfer reads)."""

    def __init__(self, weights: dict):
        self.t = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in weights.items()}

    def conv(self, x, name, act):
        w = self.t[name + ".weight"]
        y = F.conv2d(x, w, self.t[name + ".bias"], stride=1, padding=w.shape[-1] // 2)
        if act == "relu":
            return F.relu(y)
        if act is None:
            return y
        return F.prelu(y, self.t[act + ".weight"])      # act = PReLU parameter name


def _vgg(p: _Params, x, names, prelu=()):
    # make_layers: ReLU unless in no_relu, PReLU named 'prelu'+name[4:] (model.py:25-45)
    for n in names:
        if n == "pool":
            x = F.max_pool2d(x, 2, 2, 0)
        else:
            x = p.conv(x, n, ("prelu" + n[4:]) if n in prelu else "relu")
    return x


_FRONT = ["conv1_1", "conv1_2", "pool", "conv2_1", "conv2_2", "pool", "conv3_1", "conv3_2",
          "conv3_3", "conv3_4", "pool", "conv4_1", "conv4_2"]


def forward_body25(weights: dict, x: torch.Tensor):
    """bodypose_25_model.forward (model.py:179-207) -> (paf[N,52,h,w], heat[N,26,h,w])."""
    p = weights if isinstance(weights, _Params) else _Params(weights)
    no_act = {"Mconv7_stage0_L1", "Mconv7_stage0_L2", "Mconv7_stage1_L1", "Mconv7_stage1_L2",
              "Mconv7_stage2_L2", "Mconv7_stage3_L2"}

    def mc(t, name):
        return p.conv(t, name, None if name in no_act else "Mprelu" + name[5:])

    def stage(t, tag):
        # five dense blocks: out of each conv kept, the block output is their concat
        for b in range(1, 6):
            outs = []
            for j in range(3):
                t = mc(t, "Mconv%d_%s_%d" % (b, tag, j))
                outs.append(t)
            t = torch.cat(outs, 1)
        t = mc(t, "Mconv6_%s" % tag)
        return mc(t, "Mconv7_%s" % tag)

    out0 = _vgg(p, x, _FRONT + ["conv4_3_CPM", "conv4_4_CPM"],
                prelu=("conv4_2", "conv4_3_CPM", "conv4_4_CPM"))
    t = out0
    for s in range(4):
        paf = stage(t, "stage%d_L2" % s)
        t = torch.cat([out0, paf], 1)
    heat0 = stage(t, "stage0_L1")
    heat1 = stage(torch.cat([out0, heat0, paf], 1), "stage1_L1")
    return paf, heat1


def forward_coco(weights: dict, x: torch.Tensor):
    """bodypose_model.forward (model.py:302-329) -> (L1 paf[N,38], L2 heat[N,19])."""
    p = weights if isinstance(weights, _Params) else _Params(weights)
    # model.py:215-218 lists Mconv7_stage6_L1 twice, never Mconv7_stage6_L2 (its ReLU stays)
    no_relu = {"conv5_5_CPM_L1", "conv5_5_CPM_L2"} | {
        "Mconv7_stage%d_L%d" % (i, b) for i in range(2, 6) for b in (1, 2)} | {"Mconv7_stage6_L1"}

    def seq(t, names):
        for n in names:
            t = p.conv(t, n, None if n in no_relu else "relu")
        return t

    out1 = _vgg(p, x, _FRONT + ["conv4_3_CPM", "conv4_4_CPM"])
    b1 = seq(out1, ["conv5_%d_CPM_L1" % j for j in range(1, 6)])
    b2 = seq(out1, ["conv5_%d_CPM_L2" % j for j in range(1, 6)])
    for i in range(2, 7):
        t = torch.cat([b1, b2, out1], 1)
        b1 = seq(t, ["Mconv%d_stage%d_L1" % (j, i) for j in range(1, 8)])
        b2 = seq(t, ["Mconv%d_stage%d_L2" % (j, i) for j in range(1, 8)])
    return b1, b2


def forward_hand(weights: dict, x: torch.Tensor):
    """handpose_model.forward (model.py:394-407) -> heat[N,22,h,w]."""
    p = weights if isinstance(weights, _Params) else _Params(weights)
    no_relu = {"conv6_2_CPM"} | {"Mconv7_stage%d" % i for i in range(2, 7)}

    def seq(t, names):
        for n in names:
            t = p.conv(t, n, None if n in no_relu else "relu")
        return t

    out1_0 = _vgg(p, x, _FRONT + ["conv4_3", "conv4_4", "conv5_1", "conv5_2", "conv5_3_CPM"])
    t = seq(out1_0, ["conv6_1_CPM", "conv6_2_CPM"])
    for i in range(2, 7):
        t = seq(torch.cat([t, out1_0], 1), ["Mconv%d_stage%d" % (j, i) for j in range(1, 8)])
    return t


FORWARDS = {"body25": forward_body25, "coco": forward_coco, "hand": forward_hand}


def make_net_fn(model_type: str, weights: dict):
    """numpy NCHW f32 -> tuple of numpy outputs, like `self.model(data)` + `.numpy()`."""
    fwd = FORWARDS[model_type]
    p = _Params(weights)

    def run(im: np.ndarray):
        with torch.no_grad():
            out = fwd(p, torch.from_numpy(np.ascontiguousarray(im, np.float32)))
        if isinstance(out, tuple):
            return tuple(o.numpy() for o in out)
        return out.numpy()
    return run


# ---------------------------------------------------------------------------
# pre-processing (body.py:47-58, util.py:12-32)
# ---------------------------------------------------------------------------

BOXSIZE, STRIDE, PADVALUE = 368, 8, 128


def pad_right_down(img: np.ndarray, stride: int = STRIDE, pad_value: int = PADVALUE):
    """util.padRightDownCorner: pad bottom/right with pad_value to a multiple of stride."""
    h, w = img.shape[:2]
    pad = [0, 0, 0 if h % stride == 0 else stride - h % stride,
           0 if w % stride == 0 else stride - w % stride]
    out = np.full((h + pad[2], w + pad[3]) + img.shape[2:], pad_value, dtype=img.dtype)
    out[:h, :w] = img
    return out, pad


def net_input(img_u8: np.ndarray, scale: float):
    """resize -> pad -> float32/256 - 0.5 -> NCHW (body.py:53-56); returns (im, padded_hw, pad)."""
    small = cv_resize.resize(img_u8, (0, 0), fx=scale, fy=scale)
    padded, pad = pad_right_down(small)
    im = np.ascontiguousarray(np.transpose(np.float32(padded[:, :, :, None]), (3, 2, 0, 1)) / 256 - 0.5)
    return im, padded.shape[:2], pad


def upsample_map(lowres_chw: np.ndarray, padded_hw, pad, out_hw):
    """body.py:69-72: CHW f32 -> x8 cubic -> crop padding -> cubic to frame size (HWC f32)."""
    m = np.transpose(lowres_chw, (1, 2, 0))
    m = cv_resize.resize(m, (0, 0), fx=STRIDE, fy=STRIDE)
    m = m[:padded_hw[0] - pad[2], :padded_hw[1] - pad[3], :]
    return cv_resize.resize(m, (out_hw[1], out_hw[0]))


# ---------------------------------------------------------------------------
# fp64 gaussian blur (scipy.ndimage.gaussian_filter, sigma=3, mode='reflect')
# ---------------------------------------------------------------------------


def gaussian_weights(sigma: float = 3, truncate: float = 4.0) -> np.ndarray:
    """scipy _gaussian_kernel1d(sigma, 0, radius); radius = int(truncate*sigma + 0.5)."""
    radius = int(truncate * float(sigma) + 0.5)
    x = np.arange(-radius, radius + 1)
    phi = np.exp(-0.5 / (sigma * sigma) * x ** 2)
    return phi / phi.sum()


_GW = gaussian_weights()


def _blur_axis(a: np.ndarray, axis: int, w: np.ndarray = _GW) -> np.ndarray:
    # NI_Correlate1D, symmetric branch: o = c*w0; for j = r..1: o += (a[-j] + a[+j]) * w[j]
    r = len(w) // 2
    n = a.shape[axis]
    padw = [(0, 0)] * a.ndim
    padw[axis] = (r, r)
    p = np.pad(a, padw, mode="symmetric")            # scipy 'reflect' = d c b a | a b c d | d c b a

    def sl(off):
        idx = [slice(None)] * a.ndim
        idx[axis] = slice(r + off, r + off + n)
        return p[tuple(idx)]
    out = sl(0) * w[r]
    for j in range(r, 0, -1):
        out = out + (sl(-j) + sl(j)) * w[r - j]
    return out


def gaussian_blur(a: np.ndarray) -> np.ndarray:
    """gaussian_filter(a, sigma=3) on a float64 plane: axis 0 then axis 1."""
    return _blur_axis(_blur_axis(np.asarray(a, np.float64), 0), 1)


# ---------------------------------------------------------------------------
# body post-processing (body.py:83-235)
# ---------------------------------------------------------------------------

LIMBS = {
    "body25": ([[1, 0], [1, 2], [2, 3], [3, 4], [1, 5], [5, 6], [6, 7], [1, 8], [8, 9], [9, 10],
                [10, 11], [8, 12], [12, 13], [13, 14], [0, 15], [0, 16], [15, 17], [16, 18],
                [11, 24], [11, 22], [14, 21], [14, 19], [22, 23], [19, 20]],
               [[30, 31], [14, 15], [16, 17], [18, 19], [22, 23], [24, 25], [26, 27], [0, 1], [6, 7],
                [2, 3], [4, 5], [8, 9], [10, 11], [12, 13], [32, 33], [34, 35], [36, 37], [38, 39],
                [50, 51], [46, 47], [44, 45], [40, 41], [48, 49], [42, 43]]),
    "coco": ([[1, 2], [1, 5], [2, 3], [3, 4], [5, 6], [6, 7], [1, 8], [8, 9], [9, 10], [1, 11],
              [11, 12], [12, 13], [1, 0], [0, 14], [14, 16], [0, 15], [15, 17], [2, 16], [5, 17]],
             [[12, 13], [20, 21], [14, 15], [16, 17], [22, 23], [24, 25], [0, 1], [2, 3], [4, 5],
              [6, 7], [8, 9], [10, 11], [28, 29], [30, 31], [34, 35], [32, 33], [36, 37], [18, 19],
              [26, 27]]),
}
NJOINT = {"body25": 26, "coco": 19}
NPAF = {"body25": 52, "coco": 38}


def find_peaks(heatmap_avg: np.ndarray, njoint: int, thre1: float = 0.1):
    """body.py:83-107 -> all_peaks: per part list of (x, y, score, id)."""
    all_peaks, counter = [], 0
    for part in range(njoint - 1):
        map_ori = heatmap_avg[:, :, part]
        g = gaussian_blur(map_ori)
        ok = g > thre1
        ok[1:, :] &= g[1:, :] >= g[:-1, :]
        ok[:-1, :] &= g[:-1, :] >= g[1:, :]
        ok[:, 1:] &= g[:, 1:] >= g[:, :-1]
        ok[:, :-1] &= g[:, :-1] >= g[:, 1:]
        ok[0, :] &= g[0, :] >= 0          # out-of-image neighbours compare against 0
        ok[-1, :] &= g[-1, :] >= 0
        ok[:, 0] &= g[:, 0] >= 0
        ok[:, -1] &= g[:, -1] >= 0
        ys, xs = np.nonzero(ok)
        peaks = [(xs[i], ys[i], map_ori[ys[i], xs[i]], counter + i) for i in range(len(xs))]
        all_peaks.append(peaks)
        counter += len(peaks)
    return all_peaks


def score_limb(candA, candB, paf_x, paf_y, img_h, thre2=0.05, mid_num=10):
    """PAF line integral for every (i, j) pair of one limb (body.py:141-164), vectorised.

    Returns the connection_candidate list [i, j, score, score + sA + sB] in
    (i, j) order, keeping only pairs meeting both criteria.
    """
    nA, nB = len(candA), len(candB)
    ax = np.array([c[0] for c in candA], np.int64)[:, None]
    ay = np.array([c[1] for c in candA], np.int64)[:, None]
    bx = np.array([c[0] for c in candB], np.int64)[None, :]
    by = np.array([c[1] for c in candB], np.int64)[None, :]
    vx, vy = bx - ax, by - ay                                     # int64
    norm = np.sqrt((vx * vx + vy * vy).astype(np.float64))        # == math.sqrt(int)
    norm = np.maximum(0.001, norm)
    ux, uy = vx / norm, vy / norm
    # np.linspace(a, b, 10): i*step + a (step = (b-a)/9), last sample = b
    step_x = (bx.astype(np.float64) - ax.astype(np.float64)) / 9
    step_y = (by.astype(np.float64) - ay.astype(np.float64)) / 9
    total = None
    count = np.zeros((nA, nB), np.int64)
    for I in range(mid_num):
        if I == mid_num - 1:
            sx = np.broadcast_to(bx.astype(np.float64), (nA, nB))
            sy = np.broadcast_to(by.astype(np.float64), (nA, nB))
        else:
            sx = float(I) * step_x + ax.astype(np.float64)
            sy = float(I) * step_y + ay.astype(np.float64)
        xi = np.rint(sx).astype(np.int64)                        # int(round(.)): half to even
        yi = np.rint(sy).astype(np.int64)
        s = paf_x[yi, xi] * ux + paf_y[yi, xi] * uy
        total = s if total is None else total + s                 # builtin sum(): left to right
        count += s > thre2
    score = total / mid_num + np.minimum(0.5 * img_h / norm - 1, 0)
    keep = (count > 0.8 * mid_num) & (score > 0)
    out = []
    for i, j in zip(*np.nonzero(keep)):
        sc = score[i, j]
        out.append([int(i), int(j), sc, sc + candA[i][2] + candB[j][2]])
    return out


def connect_limbs(all_peaks, paf_avg, model_type, img_h, thre2=0.05):
    """body.py:128-178 -> (connection_all, special_k)."""
    limbSeq, mapIdx = LIMBS[model_type]
    connection_all, special_k = [], []
    for k in range(len(mapIdx)):
        candA, candB = all_peaks[limbSeq[k][0]], all_peaks[limbSeq[k][1]]
        nA, nB = len(candA), len(candB)
        if nA == 0 or nB == 0:
            special_k.append(k)
            connection_all.append([])
            continue
        cands = score_limb(candA, candB, paf_avg[:, :, mapIdx[k][0]], paf_avg[:, :, mapIdx[k][1]],
                           img_h, thre2)
        cands = sorted(cands, key=lambda c: c[2], reverse=True)   # stable
        used_i, used_j, rows = set(), set(), []
        for i, j, s, _ in cands:
            if i in used_i or j in used_j:
                continue
            rows.append([candA[i][3], candB[j][3], s, i, j])
            used_i.add(i)
            used_j.add(j)
            if len(rows) >= min(nA, nB):
                break
        connection_all.append(np.array(rows, np.float64).reshape(-1, 5))
    return connection_all, special_k


def assemble(all_peaks, connection_all, special_k, model_type):
    """body.py:180-235 -> (candidate, subset)."""
    limbSeq, mapIdx = LIMBS[model_type]
    njoint = NJOINT[model_type]
    subset = -1 * np.ones((0, njoint + 1))
    candidate = np.array([pk for part in all_peaks for pk in part])
    for k in range(len(mapIdx)):
        if k in special_k:
            continue
        conn = connection_all[k]
        A, B = limbSeq[k]
        for i in range(len(conn)):
            idA, idB, s = conn[i, 0], conn[i, 1], conn[i, 2]
            hits = [r for r in range(len(subset)) if subset[r][A] == idA or subset[r][B] == idB]
            if len(hits) > 2:
                # body.py:196 assigns subset_idx[found] with found == 2
                raise IndexError("list assignment index out of range")
            if len(hits) == 1:
                r = hits[0]
                if subset[r][B] != idB:
                    subset[r][B] = idB
                    subset[r][-1] += 1
                    subset[r][-2] += candidate[int(idB), 2] + s
            elif len(hits) == 2:
                r1, r2 = hits
                both = ((subset[r1] >= 0).astype(int) + (subset[r2] >= 0).astype(int))[:-2]
                if not np.any(both == 2):
                    subset[r1][:-2] += subset[r2][:-2] + 1
                    subset[r1][-2:] += subset[r2][-2:]
                    subset[r1][-2] += s
                    subset = np.delete(subset, r2, 0)
                else:
                    subset[r1][B] = idB
                    subset[r1][-1] += 1
                    subset[r1][-2] += candidate[int(idB), 2] + s
            elif k < njoint - 2:
                row = -1 * np.ones(njoint + 1)
                row[A], row[B] = idA, idB
                row[-1] = 2
                row[-2] = (candidate[int(idA), 2] + candidate[int(idB), 2]) + s
                subset = np.vstack([subset, row])
    drop = [r for r in range(len(subset)) if subset[r][-1] < 4 or subset[r][-2] / subset[r][-1] < 0.4]
    return candidate, np.delete(subset, drop, axis=0)


def body_post(heatmap_avg, paf_avg, model_type, img_h):
    """body.py:83-235 on accumulated full-resolution maps."""
    all_peaks = find_peaks(heatmap_avg, NJOINT[model_type])
    connection_all, special_k = connect_limbs(all_peaks, paf_avg, model_type, img_h)
    candidate, subset = assemble(all_peaks, connection_all, special_k, model_type)
    return candidate, subset, all_peaks, connection_all


def body_maps(oriImg, net_fn, model_type="body25", scale_search=(0.5,)):
    """body.py:39-81: multi-scale forward + resize + (quirky) fp64 accumulation."""
    H, W = oriImg.shape[:2]
    njoint, npaf = NJOINT[model_type], NPAF[model_type]
    multiplier = [x * BOXSIZE / H for x in scale_search]
    heatmap_avg = np.zeros((H, W, njoint))
    paf_avg = np.zeros((H, W, npaf))
    for scale in multiplier:
        im, padded_hw, pad = net_input(oriImg, scale)
        paf_lr, heat_lr = net_fn(im)
        heat = upsample_map(np.squeeze(heat_lr, 0), padded_hw, pad, (H, W))
        paf = upsample_map(np.squeeze(paf_lr, 0), padded_hw, pad, (H, W))
        heatmap_avg += heatmap_avg + heat / len(multiplier)       # body.py:80 (doubling quirk)
        paf_avg += + paf / len(multiplier)
    return heatmap_avg, paf_avg


def body_call(oriImg, net_fn, model_type="body25", scale_search=(0.5,)):
    """Body.__call__ -> (candidate, subset)."""
    heatmap_avg, paf_avg = body_maps(oriImg, net_fn, model_type, scale_search)
    candidate, subset, _, _ = body_post(heatmap_avg, paf_avg, model_type, oriImg.shape[0])
    return candidate, subset


# ---------------------------------------------------------------------------
# hand (hand.py:24-74) and handDetect (util.py:242-306)
# ---------------------------------------------------------------------------

HAND_SCALES = (0.5, 1.0, 1.5, 2.0)


def label8(binary: np.ndarray):
    """8-connected component labels in raster order of first pixel (skimage.measure.label
    with connectivity=2; scipy.ndimage.label with a 3x3 structure numbers identically)."""
    from scipy import ndimage
    return ndimage.label(binary, structure=np.ones((3, 3), np.int32))


def npmax(array):
    """util.npmax: first raster-order maximum -> (row, col)."""
    idx = array.argmax(1)
    val = array.max(1)
    i = val.argmax()
    return i, idx[i]


def hand_maps(oriImg, net_fn, scale_search=HAND_SCALES):
    """hand.py:31-56 -> heatmap_avg [h, w, 22] f64."""
    H, W = oriImg.shape[:2]
    multiplier = [x * BOXSIZE / H for x in scale_search]
    heatmap_avg = np.zeros((H, W, 22))
    for scale in multiplier:
        im, padded_hw, pad = net_input(oriImg, scale)
        out = net_fn(im)
        heat = upsample_map(np.squeeze(out, 0), padded_hw, pad, (H, W))
        heatmap_avg += heat / len(multiplier)
    return heatmap_avg


def hand_post(heatmap_avg, thre=0.05):
    """hand.py:58-74 -> int64 [21, 2] of (x, y); modifies heatmap_avg like the reference."""
    peaks = []
    for part in range(21):
        map_ori = heatmap_avg[:, :, part]
        g = gaussian_blur(map_ori)
        binary = np.ascontiguousarray(g > thre, dtype=np.uint8)
        if np.sum(binary) == 0:
            peaks.append([0, 0])
            continue
        lab, n = label8(binary)
        best = np.argmax([np.sum(map_ori[lab == i]) for i in range(1, n + 1)]) + 1
        lab[lab != best] = 0
        map_ori[lab == 0] = 0
        y, x = npmax(map_ori)
        peaks.append([x, y])
    return np.array(peaks)


def hand_call(oriImg, net_fn):
    return hand_post(hand_maps(oriImg, net_fn))


def hand_detect(candidate, subset, img_hw):
    """util.handDetect -> [[x, y, w, is_left], ...]."""
    ratio = 0.33
    H, W = img_hw
    out = []
    for person in subset.astype(int):
        has_left = np.sum(person[[5, 6, 7]] == -1) == 0
        has_right = np.sum(person[[2, 3, 4]] == -1) == 0
        if not (has_left or has_right):
            continue
        hands = []
        if has_left:
            s, e, w = person[[5, 6, 7]]
            hands.append((candidate[s][:2], candidate[e][:2], candidate[w][:2], True))
        if has_right:
            s, e, w = person[[2, 3, 4]]
            hands.append((candidate[s][:2], candidate[e][:2], candidate[w][:2], False))
        for (x1, y1), (x2, y2), (x3, y3), is_left in hands:
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
                out.append([int(x), int(y), int(width), is_left])
    return out
