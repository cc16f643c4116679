"""Deterministic synthetic inputs: weights, frames and designed pose maps.

The reference's pretrained weights are not available offline,
so every test and benchmark runs on *synthetic* weights produced here by a
counter-hash generator.  The generator is pure integer arithmetic on uint64
(splitmix64), so the same seed yields bit-identical tensors on every machine
(this container, the GPU box) without committing any weight file.

``designed_pose_maps`` builds low-resolution network outputs with a controlled
number of people (Gaussian keypoint blobs + unit-vector PAF strips).  Raw
outputs of random-weight networks explode to thousands of peaks (SURVEY.md
§8d), so post-processing is fed these maps wherever its cost must be
meaningful.
"""
from __future__ import annotations

import zlib

import numpy as np

from . import netspec

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 finaliser over a uint64 array (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return z ^ (z >> np.uint64(31))


def hash_uniform(key: int, n: int) -> np.ndarray:
    """n float64 values uniform in [0, 1), a pure function of (key, index)."""
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = np.uint64(key & 0xFFFFFFFFFFFFFFFF) * np.uint64(0x2545F4914F6CDD1D)
    h = splitmix64(idx ^ base)
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def _key(seed: int, name: str) -> int:
    return (seed * 1000003 + zlib.crc32(name.encode())) & 0xFFFFFFFFFFFFFFFF


def synth_weights(kind: int, seed: int = 0) -> dict:
    """Flat caffe-named weight dict {name: float32 ndarray} (the format util.transfer reads).

    conv weights: He-uniform U(-a, a), a = sqrt(6 / fan_in); biases U(-0.05, 0.05);
    PReLU slopes U(0.05, 0.25).
    """
    out = {}
    for c in netspec.convs_for(kind):
        fan_in = c.cin * c.k * c.k
        a = np.sqrt(6.0 / fan_in)
        w = hash_uniform(_key(seed, c.name + ".weight"), c.cout * fan_in)
        out[c.name + ".weight"] = ((w * 2.0 - 1.0) * a).astype(np.float32).reshape(c.cout, c.cin, c.k, c.k)
        b = hash_uniform(_key(seed, c.name + ".bias"), c.cout)
        out[c.name + ".bias"] = ((b * 2.0 - 1.0) * 0.05).astype(np.float32)
        if c.prelu is not None:
            p = hash_uniform(_key(seed, c.prelu + ".weight"), c.cout)
            out[c.prelu + ".weight"] = (0.05 + 0.2 * p).astype(np.float32)
    return out


HEAT_LAYER = {"body25": "Mconv7_stage1_L1", "coco": "Mconv7_stage6_L2"}


def tame_heat_layer(weights: dict, heat: np.ndarray, model_type: str = "body25", gain: float = 0.05) -> dict:
    """Synthetic weights whose heat output behaves like a trained net's.

    Raw outputs of the seeded He-init weights put thousands of peaks on a frame
    (SURVEY §8d).  Given the net's heat output on one calibration frame (low-res
    [1, C, h, w], from any implementation of the net), the heat output layer is
    rescaled per channel: heat_k = gain * (z_k - mean_k) / std_k, so a part map
    crosses the 0.1 peak threshold where its field is ~0.1/gain standard deviations
    high -- a handful of peaks per part, a few persons per frame.  The PAF layers are
    untouched."""
    z = np.asarray(heat)[0].reshape(heat.shape[1], -1).astype(np.float64)
    m, s = z.mean(1), np.maximum(z.std(1), 1e-6)
    a = gain / s
    layer = HEAT_LAYER[model_type]
    out = dict(weights)
    out[layer + ".weight"] = (weights[layer + ".weight"] * a[:, None, None, None]).astype(np.float32)
    out[layer + ".bias"] = ((weights[layer + ".bias"] - m) * a).astype(np.float32)
    return out


def synth_frames(n: int, h: int, w: int, seed: int = 0) -> np.ndarray:
    """uint8 [n, h, w, 3] BGR frames; frame i depends only on (seed, i)."""
    frames = np.empty((n, h, w, 3), np.uint8)
    for i in range(n):
        u = hash_uniform(_key(seed, "frame%d" % i), h * w * 3)
        frames[i] = (u * 256.0).astype(np.uint8).reshape(h, w, 3)
    return frames


# ---------------------------------------------------------------------------
# designed pose maps
# ---------------------------------------------------------------------------

# body_25 keypoint template (x, y) in units of person height, origin at MidHip.
_BODY25_TEMPLATE = np.array([
    (0.00, -0.42), (0.00, -0.32), (-0.11, -0.31), (-0.15, -0.15), (-0.17, 0.00),
    (0.11, -0.31), (0.15, -0.15), (0.17, 0.00), (0.00, 0.00), (-0.07, 0.00),
    (-0.08, 0.22), (-0.08, 0.44), (0.07, 0.00), (0.08, 0.22), (0.08, 0.44),
    (-0.03, -0.45), (0.03, -0.45), (-0.06, -0.43), (0.06, -0.43), (0.12, 0.50),
    (0.14, 0.49), (0.07, 0.47), (-0.12, 0.50), (-0.14, 0.49), (-0.07, 0.47)])

# COCO-18 keypoint template.
_COCO_TEMPLATE = np.array([
    (0.00, -0.42), (0.00, -0.32), (-0.11, -0.31), (-0.15, -0.15), (-0.17, 0.00),
    (0.11, -0.31), (0.15, -0.15), (0.17, 0.00), (-0.07, 0.00), (-0.08, 0.22),
    (-0.08, 0.44), (0.07, 0.00), (0.08, 0.22), (0.08, 0.44), (-0.03, -0.45),
    (0.03, -0.45), (-0.06, -0.43), (0.06, -0.43)])

# Limb tables, /root/reference/src/body.py:111-126.
BODY25_LIMBS = [[1, 0], [1, 2], [2, 3], [3, 4], [1, 5], [5, 6], [6, 7], [1, 8], [8, 9], [9, 10],
                [10, 11], [8, 12], [12, 13], [13, 14], [0, 15], [0, 16], [15, 17], [16, 18],
                [11, 24], [11, 22], [14, 21], [14, 19], [22, 23], [19, 20]]
BODY25_MAPIDX = [[30, 31], [14, 15], [16, 17], [18, 19], [22, 23], [24, 25], [26, 27], [0, 1], [6, 7],
                 [2, 3], [4, 5], [8, 9], [10, 11], [12, 13], [32, 33], [34, 35], [36, 37], [38, 39],
                 [50, 51], [46, 47], [44, 45], [40, 41], [48, 49], [42, 43]]
COCO_LIMBS = [[1, 2], [1, 5], [2, 3], [3, 4], [5, 6], [6, 7], [1, 8], [8, 9], [9, 10], [1, 11],
              [11, 12], [12, 13], [1, 0], [0, 14], [14, 16], [0, 15], [15, 17], [2, 16], [5, 17]]
COCO_MAPIDX = [[12, 13], [20, 21], [14, 15], [16, 17], [22, 23], [24, 25], [0, 1], [2, 3], [4, 5],
               [6, 7], [8, 9], [10, 11], [28, 29], [30, 31], [34, 35], [32, 33], [36, 37], [18, 19],
               [26, 27]]


def designed_pose_maps(h8: int, w8: int, n_persons: int, seed: int, model_type: str = "body25",
                       sigma: float = 1.0, strip: float = 1.0, drop_limbs=()):
    """Low-resolution (paf, heat) maps, NCHW without batch: ([npaf,h8,w8], [njoint,h8,w8]) f32.

    Persons are placed left to right with seeded jitter; each keypoint is a
    Gaussian blob (std ``sigma`` low-res px), each limb a strip of unit vectors
    (half-width ``strip``) in its two PAF channels, except the limbs listed in
    ``drop_limbs`` (indices into the limb table): e.g. COCO limb 12 (neck -> nose)
    dropped makes every head its own subset row until the redundant ear limbs 17/18
    merge it into the body (the found == 2 branch of body.py:204-218).  The last
    heat channel is the background (1 - max of parts).
    """
    if model_type == "body25":
        tmpl, limbs, mapidx, njoint, npaf = _BODY25_TEMPLATE, BODY25_LIMBS, BODY25_MAPIDX, 26, 52
    else:
        tmpl, limbs, mapidx, njoint, npaf = _COCO_TEMPLATE, COCO_LIMBS, COCO_MAPIDX, 19, 38
    rng = np.random.RandomState(seed)
    heat = np.zeros((njoint, h8, w8), np.float64)
    paf = np.zeros((npaf, h8, w8), np.float64)
    cnt = np.zeros((npaf // 2, h8, w8), np.float64)
    yy, xx = np.mgrid[0:h8, 0:w8].astype(np.float64)
    slot = w8 / max(n_persons, 1)
    for p in range(n_persons):
        height = h8 * rng.uniform(0.65, 0.85)
        cx = slot * (p + 0.5) + rng.uniform(-0.1, 0.1) * slot
        cy = h8 * 0.5 + rng.uniform(-0.05, 0.05) * h8
        kp = np.empty_like(tmpl)
        kp[:, 0] = cx + tmpl[:, 0] * height * min(1.0, slot / (0.45 * height)) + rng.normal(0, 0.3, len(tmpl))
        kp[:, 1] = cy + tmpl[:, 1] * height + rng.normal(0, 0.3, len(tmpl))
        amp = rng.uniform(0.7, 1.0, len(tmpl))
        for k in range(len(tmpl)):
            g = amp[k] * np.exp(-((xx - kp[k, 0]) ** 2 + (yy - kp[k, 1]) ** 2) / (2 * sigma * sigma))
            g[g < 1e-3] = 0.0          # truncated tails keep the maps sparse
            heat[k] = np.maximum(heat[k], g)
        for li, (a, b) in enumerate(limbs):
            if li in drop_limbs:
                continue
            pa, pb = kp[a], kp[b]
            d = pb - pa
            ln = np.hypot(d[0], d[1])
            if ln < 1e-6:
                continue
            u = d / ln
            rx, ry = xx - pa[0], yy - pa[1]
            t = rx * u[0] + ry * u[1]
            perp = np.abs(rx * u[1] - ry * u[0])
            m = (t >= -strip) & (t <= ln + strip) & (perp <= strip)
            cx_, cy_ = mapidx[li]
            paf[cx_][m] += u[0]
            paf[cy_][m] += u[1]
            cnt[li][m] += 1
    for li, (cx_, cy_) in enumerate(mapidx):
        nz = cnt[li] > 0
        paf[cx_][nz] /= cnt[li][nz]
        paf[cy_][nz] /= cnt[li][nz]
    heat[njoint - 1] = 1.0 - heat[:njoint - 1].max(axis=0)
    return paf.astype(np.float32), heat.astype(np.float32)


def designed_hand_maps(h8: int, w8: int, seed: int, sigma: float = 1.0, n_blobs: int = 2):
    """Low-resolution hand heatmaps [22, h8, w8] f32: each of the 21 parts gets
    ``n_blobs`` Gaussian blobs of different amplitude (so the connected-component
    selection in Hand.__call__ has a choice to make); channel 21 = background."""
    rng = np.random.RandomState(seed)
    yy, xx = np.mgrid[0:h8, 0:w8].astype(np.float64)
    heat = np.zeros((22, h8, w8), np.float64)
    for k in range(21):
        for b in range(n_blobs):
            if rng.uniform() < 0.15:
                continue
            cx, cy = rng.uniform(1, w8 - 1), rng.uniform(1, h8 - 1)
            amp = rng.uniform(0.2, 1.0)
            s = sigma * rng.uniform(0.8, 1.6)
            g = amp * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * s * s))
            g[g < 1e-3] = 0.0
            heat[k] += g
    heat[21] = 1.0 - np.clip(heat[:21].max(axis=0), 0, 1)
    return heat.astype(np.float32)
