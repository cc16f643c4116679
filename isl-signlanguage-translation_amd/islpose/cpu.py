"""GPU-less execution of the drop-in seams (src/body.py, src/hand.py, src/model.py).

The reference runs ``Body`` / ``Hand`` on the CPU when no CUDA device is visible
(/root/reference/src/body.py:31-32,56-57, hand.py:18-20,42-43); BASELINE configs[0]
(demo.py on one image) is exactly that.  This module is the product's CPU path for those
callers: the networks through the torch CPU modules of src/model.py (``cpu_forward``, the
reference's dataflow), the cubic resizes in numpy with the arithmetic of the GPU kernels
(``preprocess_kernel`` for the uint8 frame, ``resize_sep_kernel`` for the maps: OpenCV's
INTER_CUBIC operation order), scipy's ``gaussian_filter`` for the blur (the reference's own
call), the peaks, PAF scoring and assembly of body.py:84-235 and the hand peaks of
hand.py:58-74 (scipy's 8-connected ``label``).  It does not import the test oracle.

It is slow (seconds per 368-row frame on a few cores) and exists so that GPU-less hosts
run; the GPU path is the product's fast path.  Pinned against the reference's own outputs
(tests/golden G1/G2/G4) in tests/test_cpu_path.py.
"""
from __future__ import annotations

import math

import numpy as np

BOXSIZE, STRIDE, PADVALUE = 368, 8, 128
_F = np.float32

# limb tables (body.py:114-131), 0-based joints and PAF channel indices
LIMBS = {
    "body25": ([[1, 0], [1, 2], [2, 3], [3, 4], [1, 5], [5, 6], [6, 7], [1, 8], [8, 9], [9, 10], [10, 11], [8, 12],
                [12, 13], [13, 14], [0, 15], [0, 16], [15, 17], [16, 18], [11, 24], [11, 22], [14, 21], [14, 19],
                [22, 23], [19, 20]],
               [[30, 31], [14, 15], [16, 17], [18, 19], [22, 23], [24, 25], [26, 27], [0, 1], [6, 7], [2, 3],
                [4, 5], [8, 9], [10, 11], [12, 13], [32, 33], [34, 35], [36, 37], [38, 39], [50, 51], [46, 47],
                [44, 45], [40, 41], [48, 49], [42, 43]]),
    "coco": ([[1, 2], [1, 5], [2, 3], [3, 4], [5, 6], [6, 7], [1, 8], [8, 9], [9, 10], [1, 11], [11, 12], [12, 13],
              [1, 0], [0, 14], [14, 16], [0, 15], [15, 17], [2, 16], [5, 17]],
             [[12, 13], [20, 21], [14, 15], [16, 17], [22, 23], [24, 25], [0, 1], [2, 3], [4, 5], [6, 7], [8, 9],
              [10, 11], [28, 29], [30, 31], [34, 35], [32, 33], [36, 37], [18, 19], [26, 27]]),
}


# ---------------------------------------------------------------------------
# cubic resize (the GPU kernels' arithmetic: taps() / cubic_coeffs_f, HResizeCubic then
# VResizeCubic; uint8 frames in fixed point as preprocess_kernel)
# ---------------------------------------------------------------------------

def _taps(dst_n: int, src_n: int, scale: float):
    """Per output index the 4 clamped source indices [4, n] and float32 coefficients [4, n]."""
    f = ((np.arange(dst_n, dtype=np.float64) + 0.5) * scale - 0.5).astype(_F)
    s = np.floor(f)
    t = (f - s).astype(_F)
    s = s.astype(np.int64)
    A = _F(-0.75)
    tp1 = t + _F(1)
    c0 = ((A * tp1 - _F(5) * A) * tp1 + _F(8) * A) * tp1 - _F(4) * A
    c1 = ((A + _F(2)) * t - (A + _F(3))) * t * t + _F(1)
    u = _F(1) - t
    c2 = ((A + _F(2)) * u - (A + _F(3))) * u * u + _F(1)
    c3 = _F(1) - c0 - c1 - c2
    idx = np.stack([np.clip(s + k - 1, 0, src_n - 1) for k in range(4)])
    return idx, np.stack([c0, c1, c2, c3]).astype(_F)


def _geometry(src_hw, dsize=None, fx=None):
    """cv::resize's destination size and per-axis scale (fx == fy here)."""
    sh, sw = src_hw
    if dsize is None:
        dh, dw = int(np.rint(sh * fx)), int(np.rint(sw * fx))
        return dh, dw, 1.0 / fx, 1.0 / fx
    dw, dh = dsize
    return dh, dw, 1.0 / (dh / sh), 1.0 / (dw / sw)


def resize(img: np.ndarray, dsize=None, fx=None) -> np.ndarray:
    """INTER_CUBIC resize of an H x W x C uint8 or float32 image to dsize = (W, H), or by fx."""
    sh, sw, cn = img.shape
    dh, dw, sy, sx = _geometry((sh, sw), dsize, fx)
    if (dh, dw) == (sh, sw):
        return img.copy()
    xi, xc = _taps(dw, sw, sx)
    yi, yc = _taps(dh, sh, sy)
    flat = np.arange(dw)[:, None] * cn + np.arange(cn)[None, :]   # element index within a row
    if img.dtype == np.uint8:
        ia = (xc * _F(2048)).astype(np.float64).round().astype(np.int64)   # saturate_cast<short>(c * 2048)
        ib = (yc * _F(2048)).astype(np.float64).round().astype(np.int64)
        src = img.astype(np.int64)
        hz = sum(src[:, xi[k], :] * ia[k][None, :, None] for k in range(4))   # int sums, exact
        rows = [hz[yi[k]] for k in range(4)]
        fixed = np.clip((sum(rows[k] * ib[k][:, None, None] for k in range(4)) + (1 << 21)) >> 22, 0, 255)
        bf = [(ib[k].astype(_F) * _F(1.0 / (2048 * 2048)))[:, None, None] for k in range(4)]
        r = [x.astype(_F) for x in rows]
        v = r[0] * bf[0] + (r[1] * bf[1] + (r[2] * bf[2] + r[3] * bf[3]))
        vec = np.clip(np.clip(np.rint(v), -32768, 32767), 0, 255)
        body = dw * cn - (dw * cn) % 8
        return np.where((flat < body)[None], vec, fixed).astype(np.uint8)
    img = img.astype(_F, copy=False)
    hz = img[:, xi[0], :] * xc[0][None, :, None]
    for k in (1, 2, 3):
        hz = hz + img[:, xi[k], :] * xc[k][None, :, None]
    r = [hz[yi[k]] for k in range(4)]
    b = [yc[k][:, None, None] for k in range(4)]
    vec = r[0] * b[0] + (r[1] * b[1] + (r[2] * b[2] + r[3] * b[3]))     # VResizeCubicVec_32f body
    tail = ((r[0] * b[0] + r[1] * b[1]) + r[2] * b[2]) + r[3] * b[3]   # scalar tail
    body = dw * cn - (dw * cn) % 4
    return np.where((flat < body)[None], vec, tail).astype(_F)


def pad_right_down(img: np.ndarray):
    """util.padRightDownCorner(img, 8, 128): pad the bottom / right to multiples of 8."""
    h, w = img.shape[:2]
    pd, pr = (-h) % STRIDE, (-w) % STRIDE
    out = np.full((h + pd, w + pr) + img.shape[2:], PADVALUE, img.dtype)
    out[:h, :w] = img
    return out, [0, 0, pd, pr]


def _scale_maps(ori_hw, frame, scale, net_fn):
    """One scale of body.py:51-78 / hand.py:36-56: the net's outputs resized to the frame."""
    H, W = ori_hw
    test = resize(frame, fx=scale)
    padded, pad = pad_right_down(test)
    im = np.ascontiguousarray(np.transpose(np.float32(padded[:, :, :, None]), (3, 2, 0, 1)) / 256 - 0.5)
    outs = net_fn(im)
    res = []
    for o in (outs if isinstance(outs, tuple) else (outs,)):
        m = np.transpose(np.squeeze(np.asarray(o, np.float32), 0), (1, 2, 0))
        m = resize(np.ascontiguousarray(m), fx=STRIDE)
        m = m[:padded.shape[0] - pad[2], :padded.shape[1] - pad[3], :]
        res.append(resize(np.ascontiguousarray(m), dsize=(W, H)))
    return res


# ---------------------------------------------------------------------------
# body (body.py:39-235)
# ---------------------------------------------------------------------------

def _peaks(heatmap_avg, njoint, thre1=0.1):
    from scipy.ndimage import gaussian_filter
    all_peaks, counter = [], 0
    for part in range(njoint - 1):
        map_ori = heatmap_avg[:, :, part]
        g = gaussian_filter(map_ori, sigma=3)
        nb = np.zeros((4,) + g.shape)
        nb[0, 1:, :], nb[1, :-1, :] = g[:-1, :], g[1:, :]
        nb[2, :, 1:], nb[3, :, :-1] = g[:, :-1], g[:, 1:]
        ys, xs = np.nonzero((g >= nb).all(0) & (g > thre1))
        all_peaks.append([(int(x), int(y), map_ori[y, x], counter + i) for i, (x, y) in enumerate(zip(xs, ys))])
        counter += len(xs)
    return all_peaks


def _connect(all_peaks, paf_avg, model_type, img_h, thre2=0.05, mid_num=10):
    limbs, mapidx = LIMBS[model_type]
    connection_all, special_k = [], []
    for k, (la, lb) in enumerate(limbs):
        candA, candB = all_peaks[la], all_peaks[lb]
        if not candA or not candB:
            special_k.append(k)
            connection_all.append([])
            continue
        px, py = paf_avg[:, :, mapidx[k][0]], paf_avg[:, :, mapidx[k][1]]
        cands = []
        for i, a in enumerate(candA):
            for j, b in enumerate(candB):
                vx, vy = b[0] - a[0], b[1] - a[1]
                norm = max(0.001, math.sqrt(vx * vx + vy * vy))
                sx = np.linspace(a[0], b[0], num=mid_num)
                sy = np.linspace(a[1], b[1], num=mid_num)
                xi, yi = np.rint(sx).astype(np.int64), np.rint(sy).astype(np.int64)   # int(round(.))
                s = px[yi, xi] * (vx / norm) + py[yi, xi] * (vy / norm)
                score = sum(s.tolist()) / len(s) + min(0.5 * img_h / norm - 1, 0)   # builtin sum, in order
                if np.count_nonzero(s > thre2) > 0.8 * len(s) and score > 0:
                    cands.append((i, j, score))
        cands.sort(key=lambda c: c[2], reverse=True)   # stable, as sorted(..., reverse=True)
        conn, usedA, usedB = [], set(), set()
        for i, j, s in cands:
            if i not in usedA and j not in usedB:
                conn.append([candA[i][3], candB[j][3], s, i, j])
                usedA.add(i)
                usedB.add(j)
                if len(conn) >= min(len(candA), len(candB)):
                    break
        connection_all.append(np.array(conn, np.float64).reshape(-1, 5))
    return connection_all, special_k


def _assemble(all_peaks, connection_all, special_k, model_type, njoint):
    limbs, _ = LIMBS[model_type]
    candidate = np.array([p for peaks in all_peaks for p in peaks])
    subset = -1 * np.ones((0, njoint + 1))
    for k, (ia, ib) in enumerate(limbs):
        if k in special_k:
            continue
        conn = connection_all[k]
        for c in conn:
            pa, pb = c[0], c[1]
            hits = [r for r in range(len(subset)) if subset[r][ia] == pa or subset[r][ib] == pb]
            if len(hits) > 2:
                # body.py:193-196: subset_idx has two slots, the third match's store raises
                # (the GPU path flags it as ISL_E_INDEX and raises the same)
                raise IndexError("list assignment index out of range")
            if len(hits) == 1 or (len(hits) == 2 and
                                  ((subset[hits[0]] >= 0).astype(int) + (subset[hits[1]] >= 0).astype(int))[:-2]
                                  .max() == 2):
                r = hits[0]
                if len(hits) == 2 or subset[r][ib] != pb:
                    subset[r][ib] = pb
                    subset[r][-1] += 1
                    subset[r][-2] += candidate[int(pb), 2] + c[2]
            elif len(hits) == 2:   # disjoint rows: merge the second into the first
                r1, r2 = hits
                subset[r1][:-2] += subset[r2][:-2] + 1
                subset[r1][-2:] += subset[r2][-2:]
                subset[r1][-2] += c[2]
                subset = np.delete(subset, r2, 0)
            elif not hits and k < njoint - 2:
                row = -1 * np.ones(njoint + 1)
                row[ia], row[ib], row[-1] = pa, pb, 2
                row[-2] = sum(candidate[c[:2].astype(int), 2]) + c[2]
                subset = np.vstack([subset, row])
    keep = [r for r in range(len(subset)) if not (subset[r][-1] < 4 or subset[r][-2] / subset[r][-1] < 0.4)]
    return candidate, subset[keep] if len(keep) != len(subset) else subset


def body_call(frame: np.ndarray, net_fn, model_type: str = "body25", scale_search=(0.5,)):
    """Body.__call__ on the CPU: frame uint8 H x W x 3 (BGR); net_fn(NCHW float32) -> (paf, heat)."""
    njoint, npaf = (26, 52) if model_type == "body25" else (19, 38)
    H, W = frame.shape[:2]
    mult = [s * BOXSIZE / H for s in scale_search]
    heat_avg = np.zeros((H, W, njoint))
    paf_avg = np.zeros((H, W, npaf))
    for scale in mult:
        paf, heat = _scale_maps((H, W), frame, scale, net_fn)
        heat_avg += heat_avg + heat / len(mult)     # body.py:80 (the doubling quirk)
        paf_avg += + paf / len(mult)
    all_peaks = _peaks(heat_avg, njoint)
    conns, special_k = _connect(all_peaks, paf_avg, model_type, H)
    return _assemble(all_peaks, conns, special_k, model_type, njoint)


# ---------------------------------------------------------------------------
# hand (hand.py:24-74)
# ---------------------------------------------------------------------------

HAND_SCALES = (0.5, 1.0, 1.5, 2.0)


def hand_call(frame: np.ndarray, net_fn, scale_search=HAND_SCALES, thre=0.05):
    """Hand.__call__ on the CPU: frame uint8 H x W x 3; net_fn(NCHW float32) -> heat [1,22,h,w]."""
    from scipy.ndimage import gaussian_filter, label
    H, W = frame.shape[:2]
    mult = [s * BOXSIZE / H for s in scale_search]
    heat_avg = np.zeros((H, W, 22))
    for scale in mult:
        heat_avg += _scale_maps((H, W), frame, scale, net_fn)[0] / len(mult)
    peaks = []
    for part in range(21):
        map_ori = heat_avg[:, :, part]
        binary = gaussian_filter(map_ori, sigma=3) > thre
        if not binary.any():
            peaks.append([0, 0])
            continue
        lab, n = label(binary, structure=np.ones((3, 3), np.int32))   # 8-connected, raster-order labels
        best = int(np.argmax([np.sum(map_ori[lab == i]) for i in range(1, n + 1)])) + 1
        m = np.where(lab == best, map_ori, 0.0)
        i = int(m.max(1).argmax())            # util.npmax: row of the first maximal row maximum
        peaks.append([int(m[i].argmax()), i])
    return np.array(peaks)
