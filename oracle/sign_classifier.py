"""ORACLE — test infrastructure only (see oracle/__init__.py).

float64 numpy restatement of the reference's translation model at inference,
demo_isl_translate.py:72-100 (keras Sequential), applied by
ISLSignPosTranslator.call (src/ISL_Model_parameter.py:337):

    Masking(mask_value=0.)                  a step is masked when all its features == 0
    BatchNormalization()                    (x - mean) / sqrt(var + 1e-3) * gamma + beta
    Bidirectional(LSTM(32, return_sequences=True), merge concat)
        masked steps carry (h, c) and output 0 (zero_output_for_mask = return_sequences);
        the backward LSTM reads the window reversed, its outputs are flipped back
    Dropout(0.2)                            identity at inference
    Bidirectional(LSTM(32))                 last carried h of each direction, concat
    elu -> Dense(32, no bias) -> BN -> Dropout -> elu -> Dense(32, no bias) -> BN -> elu
    -> Dropout -> Dense(n_classes) -> softmax

LSTM cell (keras, gate order i, f, c, o): z = x K + h R + b; i, f, o = sigmoid;
c' = f c + i tanh(z_c); h' = o tanh(c').

Parity: keras is not installed here and the trained weights
(model/isl_model_final.keras) are not in the reference checkout, so this
restatement is "parity unpinned" against keras itself; it pins the HIP kernel
(csrc/sign.hip) to the published layer semantics above.
"""
from __future__ import annotations

import numpy as np

UNITS = 32


def _sigmoid(z):
    return 1.0 / (1.0 + np.exp(-z))


def _elu(v):
    return np.where(v > 0, v, np.expm1(np.minimum(v, 0)))


def _bn(v, p):
    gamma, beta, mean, var = p
    return (v - mean) / np.sqrt(var + 1e-3) * gamma + beta


def _lstm(x, mask, K, R, b, reverse):
    """x [T, Fin] -> (sequence [T, U] with zeros at masked steps, last carried h)."""
    T = x.shape[0]
    h = np.zeros(UNITS)
    c = np.zeros(UNITS)
    seq = np.zeros((T, UNITS))
    for s in range(T):
        t = T - 1 - s if reverse else s
        if not mask[t]:
            continue
        z = x[t] @ K + h @ R + b
        i, f, g, o = (z[k * UNITS:(k + 1) * UNITS] for k in range(4))
        c = _sigmoid(f) * c + _sigmoid(i) * np.tanh(g)
        h = _sigmoid(o) * np.tanh(c)
        seq[t] = h
    return seq, h


def classify(weights, window):
    """weights: keras get_weights() list; window [T, F] -> probabilities [n_classes] (float64)."""
    w = [np.asarray(a, np.float64) for a in weights]
    x = np.asarray(window, np.float64)
    mask = np.any(x != 0, axis=1)
    x = _bn(x, w[0:4])
    f1, _ = _lstm(x, mask, *w[4:7], reverse=False)
    b1, _ = _lstm(x, mask, *w[7:10], reverse=True)
    y = np.concatenate([f1, b1], axis=1)
    _, hf = _lstm(y, mask, *w[10:13], reverse=False)
    _, hb = _lstm(y, mask, *w[13:16], reverse=True)
    v = _elu(np.concatenate([hf, hb]))
    v = _elu(_bn(v @ w[16], w[17:21]))
    v = _elu(_bn(v @ w[21], w[22:26]))
    logits = v @ w[26] + w[27]
    e = np.exp(logits - logits.max())
    return e / e.sum()


def classify_batch(weights, windows):
    return np.stack([classify(weights, wnd) for wnd in windows])


def populate_features(bodypose_circles, handpose_peaks):
    """ISL_Model_parameter.py:376-443 as the reference writes it: a Python list of
    15 body x, 15 body y, then per hand slot 21 x, 21 y, 21 peak labels, 0-padded."""
    feature = []
    for k in (0, 1):
        for idx in range(15):
            feature.append(bodypose_circles[idx][k] if idx < len(bodypose_circles) else 0)
    for hand in range(2):
        for k in (0, 1, 2):
            for idx in range(21):
                feature.append(float(handpose_peaks[hand][idx][k]) if idx < len(handpose_peaks[hand]) else 0)
    return np.array(feature)
