"""Sign translation head: keypoint features of a frame window -> expression probabilities.

The reference's ISLSignPosTranslator (src/ISL_Model_parameter.py:308-443) turns
every frame of a 20-frame window into a 156-d feature row (``populate_features``,
:376-443) and feeds the [1, 20, 156] window to a keras classifier built in
demo_isl_translate.py:72-100:

    Masking(0) -> BatchNormalization -> Bidirectional(LSTM(32, return_sequences))
    -> Dropout -> Bidirectional(LSTM(32)) -> elu -> Dense(32, no bias) -> BN
    -> Dropout -> elu -> Dense(32, no bias) -> BN -> elu -> Dropout
    -> Dense(len(expression_mapping) = 167, softmax)

``SignClassifier`` runs that stack at inference on the GPU as ONE HIP launch per
batch of windows (csrc/sign.hip, ``isl_sign_classify``): one workgroup per window.
Weights are the keras ``model.get_weights()`` list (Sequential order), e.g. saved
with ``np.savez(path, *model.get_weights())``; without weights the layers get
keras' default initialisers from a seed (synthetic runs -- the reference's
``isl_model_final.keras`` is not in the repository).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .runtime import check, lib, ptr, stream_handle

N_FEATURES = 156        # 15 body x + 15 body y + 2 hands x (21 x + 21 y + 21 peak index)
WINDOW = 20             # frames per window (ISL_Model_parameter.py:324, :337)
UNITS = 32              # LSTM(32)
DENSE = 32              # Dense(32)
N_CLASSES = 167         # len(expression_mapping) (src/expression_mapping.py)


def populate_features(bodypose_circles, handpose_peaks) -> np.ndarray:
    """ISL_Model_parameter.py:376-443: the first 15 body circles' x then y, then for
    each of the two hand slots 21 x, 21 y and 21 peak labels (float(str(i))), zero
    padded.  Like the reference, the row is int64 zeros when nothing at all was
    detected (every entry is the int 0) and float64 otherwise."""
    circles = list(bodypose_circles)[:15]
    n_any = len(circles) + sum(min(len(handpose_peaks[h]), 21) for h in range(2))
    out = np.zeros(N_FEATURES, np.float64 if n_any else np.int64)
    for i, c in enumerate(circles):
        out[i] = c[0]
        out[15 + i] = c[1]
    base = 30
    for h in range(2):
        pk = handpose_peaks[h][:21]
        for i, p in enumerate(pk):
            out[base + i] = float(p[0])
            out[base + 21 + i] = float(p[1])
            out[base + 42 + i] = float(p[2])
        base += 63
    return out


def keras_weight_shapes(n_features: int = N_FEATURES, n_classes: int = N_CLASSES):
    """Shapes of ``model.get_weights()`` for the reference's Sequential, in order."""
    g = 4 * UNITS
    lstm = lambda fin: [(fin, g), (UNITS, g), (g,)]  # noqa: E731  kernel, recurrent_kernel, bias
    bn = lambda n: [(n,)] * 4                        # noqa: E731  gamma, beta, moving_mean, moving_variance
    return (bn(n_features) + lstm(n_features) + lstm(n_features) + lstm(2 * UNITS) + lstm(2 * UNITS)
            + [(2 * UNITS, DENSE)] + bn(DENSE) + [(DENSE, DENSE)] + bn(DENSE) + [(DENSE, n_classes), (n_classes,)])


def keras_default_weights(n_features: int = N_FEATURES, n_classes: int = N_CLASSES, seed: int = 0):
    """Keras' default initialisers for the reference's layers: LSTM kernel glorot_uniform,
    recurrent orthogonal, bias zeros with unit_forget_bias; Dense(32) he_normal
    (truncated); the softmax Dense glorot_uniform + zero bias; BN identity."""
    rng = np.random.RandomState(seed)
    g = 4 * UNITS

    def glorot(fi, fo):
        lim = np.sqrt(6.0 / (fi + fo))
        return rng.uniform(-lim, lim, (fi, fo))

    def orth(n, m):
        q, r = np.linalg.qr(rng.normal(size=(m, n)))
        return (q * np.sign(np.diag(r))).T[:n, :m]

    def he(fi, fo):
        sd = np.sqrt(2.0 / fi) / 0.87962566103423978
        return np.clip(rng.normal(0, 1, (fi, fo)), -2, 2) * sd

    def bn(n):
        return [np.ones(n), np.zeros(n), np.zeros(n), np.ones(n)]

    def lstm(fin):
        b = np.zeros(g)
        b[UNITS:2 * UNITS] = 1.0
        return [glorot(fin, g), orth(UNITS, g), b]

    w = bn(n_features) + lstm(n_features) + lstm(n_features) + lstm(2 * UNITS) + lstm(2 * UNITS)
    w += [he(2 * UNITS, DENSE)] + bn(DENSE) + [he(DENSE, DENSE)] + bn(DENSE)
    w += [glorot(DENSE, n_classes), np.zeros(n_classes)]
    return [a.astype(np.float32) for a in w]


def load_keras_weights(path: str):
    """``np.savez(path, *model.get_weights())`` -> list (arr_0, arr_1, ...); no pickles."""
    with np.load(path, allow_pickle=False) as z:
        return [z["arr_%d" % i] for i in range(len(z.files))]


class SignClassifier:
    """The reference's translation model on one GPU (csrc/sign.hip).

    ``clf(windows)`` with float [B, T, F] (or one [T, F] window; numpy or torch) returns
    a torch float32 tensor [B, n_classes] of softmax probabilities on the device,
    like the keras model's ``__call__`` (demo_isl_translate.py:190-193 then takes
    ``[0].cpu().detach().numpy()``)."""

    def __init__(self, weights=None, n_features: int = N_FEATURES, n_classes: int = N_CLASSES, device=None,
                 seed: int = 0):
        import torch
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        if isinstance(weights, str):
            weights = load_keras_weights(weights)
        if weights is None:
            weights = keras_default_weights(n_features, n_classes, seed)
        shapes = keras_weight_shapes(n_features, n_classes)
        if len(weights) != len(shapes):
            raise ValueError("expected %d weight arrays (keras get_weights order), got %d" % (len(shapes), len(weights)))
        for i, (w, s) in enumerate(zip(weights, shapes)):
            if tuple(np.shape(w)) != s:
                raise ValueError("weight %d: shape %s, expected %s" % (i, tuple(np.shape(w)), s))
        n = ctypes.c_int64()
        check(lib().isl_sign_param_count(n_features, n_classes, ctypes.byref(n)), "isl_sign_param_count")
        flat = np.concatenate([np.asarray(w, np.float32).ravel() for w in weights])
        assert flat.size == n.value
        self.params = torch.from_numpy(flat).to(self.device)
        self.n_features, self.n_classes = n_features, n_classes

    def __call__(self, windows, stream=None):
        import torch
        x = windows if isinstance(windows, torch.Tensor) else torch.from_numpy(np.asarray(windows, np.float32))
        if x.dim() == 2:
            x = x.unsqueeze(0)
        if x.dim() != 3 or x.shape[2] != self.n_features:
            raise ValueError("windows must be [B, T, %d], got %s" % (self.n_features, tuple(x.shape)))
        x = x.to(self.device, torch.float32).contiguous()
        out = torch.empty(x.shape[0], self.n_classes, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(lib().isl_sign_classify(ptr(self.params), self.n_features, x.shape[1], self.n_classes, ptr(x),
                                          x.shape[0], ptr(out), stream_handle(stream)), "isl_sign_classify")
        return out


def sliding_windows(features: np.ndarray, window: int = WINDOW) -> np.ndarray:
    """[T, F] per-frame rows -> [T - window + 1, window, F]: every full window, stride 1."""
    f = np.asarray(features)
    if f.shape[0] < window:
        return np.zeros((0, window, f.shape[1]), f.dtype)
    return np.lib.stride_tricks.sliding_window_view(f, window, axis=0).transpose(0, 2, 1).copy()
