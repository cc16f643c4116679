"""Restatement of OpenCV ``cv2.resize(..., interpolation=cv2.INTER_CUBIC)``.

ORACLE — test infrastructure only (see oracle/__init__.py).

The reference calls cv2.resize at src/body.py:53,70,72,76,78 and
src/hand.py:37,52,54 (copies in src/ISL_Model_parameter.py).  opencv-python is
an unpinned dependency (requirements.txt:3) absent from this environment, so
this is a restatement of OpenCV 4.x's generic resize path
(modules/imgproc/src/resize.cpp: cv::resize -> hal::resize -> resizeGeneric_
with HResizeCubic / VResizeCubic), x86-64 SSE-baseline build:

* dsize from fx/fy: (cvRound(W*fx), cvRound(H*fy)); scale_x = 1/fx.
  dsize given: inv_scale_x = dW/sW, scale_x = 1/inv_scale_x.  dsize == ssize
  -> plain copy.
* per output index d: f = (float)((d+0.5)*scale - 0.5); s = floor(f); f -= s;
  taps s-1..s+2 clamped to [0, n-1]; coefficients interpolateCubic(f), A=-0.75,
  all in float32.
* float images: horizontal D = ((S0*a0 + S1*a1) + S2*a2) + S3*a3 (float32,
  no FMA); vertical, SIMD body (VResizeCubicVec_32f, v_muladd = mul+add on
  SSE): S0*b0 + (S1*b1 + (S2*b2 + S3*b3)) for row elements
  x < rowlen - rowlen % 4, scalar tail ((S0*b0 + S1*b1) + S2*b2) + S3*b3.
* uint8 images: coefficients saturate_cast<short>(c*2048); horizontal sums in
  int; vertical SIMD body (VResizeCubicVec_32s8u): float math with beta/2^22,
  round-half-even, saturate; scalar tail (x >= rowlen - rowlen % 8) fixed
  point (sum + 2^21) >> 22, saturate.

The GPU kernels (csrc/post_kernels.hip) implement the same arithmetic; the
golden vectors use this module as their cv2 shim, so the resize arithmetic is
"parity unpinned" against real OpenCV while everything around it is pinned.
"""
from __future__ import annotations

import numpy as np

_F = np.float32


def cubic_coeffs(t: np.ndarray) -> np.ndarray:
    """interpolateCubic (resize.cpp), float32 arithmetic. t: float32 array -> [4, len]."""
    t = t.astype(_F)
    A = _F(-0.75)
    one = _F(1.0)
    tp1 = t + one
    c0 = ((A * tp1 - _F(5.0) * A) * tp1 + _F(8.0) * A) * tp1 - _F(4.0) * A
    c1 = ((A + _F(2.0)) * t - (A + _F(3.0))) * t * t + one
    u = one - t
    c2 = ((A + _F(2.0)) * u - (A + _F(3.0))) * u * u + one
    c3 = one - c0 - c1 - c2
    return np.stack([c0, c1, c2, c3]).astype(_F)


def axis_table(dst_n: int, src_n: int, scale: float):
    """Per output index: 4 clamped source indices and 4 float32 coefficients."""
    d = np.arange(dst_n, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(_F)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(_F)).astype(_F)
    idx = np.stack([np.clip(s + k - 1, 0, src_n - 1) for k in range(4)])
    return idx, cubic_coeffs(f)


def _cv_round(x: float) -> int:
    return int(np.rint(x))


def dst_size(src_hw, dsize=None, fx=None, fy=None):
    """(dst_h, dst_w, scale_y, scale_x) as cv::resize computes them."""
    sh, sw = src_hw
    if dsize is None or dsize == (0, 0):
        dw, dh = _cv_round(sw * fx), _cv_round(sh * fy)
        inv_x, inv_y = float(fx), float(fy)
    else:
        dw, dh = dsize
        inv_x, inv_y = dw / sw, dh / sh
    return dh, dw, 1.0 / inv_y, 1.0 / inv_x


def resize(img: np.ndarray, dsize=None, fx=None, fy=None) -> np.ndarray:
    """cv2.resize(img, dsize, fx=fx, fy=fy, interpolation=INTER_CUBIC) for uint8 / float32 HxW[xC]."""
    squeeze = img.ndim == 2
    if squeeze:
        img = img[:, :, None]
    sh, sw, cn = img.shape
    dh, dw, scale_y, scale_x = dst_size((sh, sw), dsize, fx, fy)
    if (dh, dw) == (sh, sw):
        out = img.copy()
        return out[:, :, 0] if squeeze else out
    xi, xc = axis_table(dw, sw, scale_x)
    yi, yc = axis_table(dh, sh, scale_y)
    if img.dtype == np.uint8:
        out = _resize_u8(img, xi, xc, yi, yc)
    elif img.dtype == np.float32:
        out = _resize_f32(img, xi, xc, yi, yc)
    else:
        raise TypeError("resize restatement covers uint8 and float32 only, got %s" % img.dtype)
    return out[:, :, 0] if squeeze else out


def _resize_f32(img, xi, xc, yi, yc):
    sh, sw, cn = img.shape
    dh, dw = yi.shape[1], xi.shape[1]
    # horizontal pass over every source row: [sh, dw, cn]
    a = xc[:, :, None]
    hz = img[:, xi[0], :] * a[0]
    hz = hz + img[:, xi[1], :] * a[1]
    hz = hz + img[:, xi[2], :] * a[2]
    hz = hz + img[:, xi[3], :] * a[3]
    hz = hz.astype(_F)
    b = yc[:, :, None, None]
    S0, S1, S2, S3 = (hz[yi[k]] for k in range(4))       # [dh, dw, cn]
    vec = S0 * b[0] + (S1 * b[1] + (S2 * b[2] + S3 * b[3]))
    sca = ((S0 * b[0] + S1 * b[1]) + S2 * b[2]) + S3 * b[3]
    rowlen = dw * cn
    body = rowlen - rowlen % 4
    flat_idx = (np.arange(dw)[:, None] * cn + np.arange(cn)[None, :])
    out = np.where((flat_idx < body)[None], vec, sca)
    return out.astype(_F)


def _resize_u8(img, xi, xc, yi, yc):
    sh, sw, cn = img.shape
    dh, dw = yi.shape[1], xi.shape[1]
    ia = np.rint(xc.astype(np.float64) * 2048.0).astype(np.int64)   # saturate_cast<short>(c*2048)
    ib = np.rint(yc.astype(np.float64) * 2048.0).astype(np.int64)
    # note: c*2048 is computed in float32 in OpenCV; scaling by a power of two is exact.
    src = img.astype(np.int64)
    hz = (src[:, xi[0], :] * ia[0][:, None] + src[:, xi[1], :] * ia[1][:, None]
          + src[:, xi[2], :] * ia[2][:, None] + src[:, xi[3], :] * ia[3][:, None])  # int sums
    S = [hz[yi[k]] for k in range(4)]
    # scalar tail: fixed point
    acc = S[0] * ib[0][:, None, None] + S[1] * ib[1][:, None, None] + S[2] * ib[2][:, None, None] \
        + S[3] * ib[3][:, None, None]
    fixed = np.clip((acc + (1 << 21)) >> 22, 0, 255)
    # SIMD body: float32 with beta * 2^-22
    scale = _F(1.0 / (2048 * 2048))
    bf = [(ib[k].astype(_F) * scale)[:, None, None] for k in range(4)]
    Sf = [s.astype(_F) for s in S]
    v = Sf[0] * bf[0] + (Sf[1] * bf[1] + (Sf[2] * bf[2] + Sf[3] * bf[3]))
    v = np.clip(np.rint(v.astype(_F)), -32768, 32767)
    simd = np.clip(v, 0, 255)
    rowlen = dw * cn
    body = rowlen - rowlen % 8
    flat_idx = (np.arange(dw)[:, None] * cn + np.arange(cn)[None, :])
    out = np.where((flat_idx < body)[None], simd, fixed)
    return out.astype(np.uint8)
