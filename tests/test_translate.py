"""Translator head (§8f#4): populate_features against the reference's own method
(tests/golden/g9_translator_features.json, made by make_golden.py g9), the
ISLSignPosTranslator window logic, and -- with -m gpu -- the HIP sign classifier
(csrc/sign.hip) against the float64 keras-semantics oracle (oracle/sign_classifier.py).

Classifier tolerance: |p_gpu - p_oracle| <= 1e-5 + 1e-4 * p_oracle (fp32 arithmetic
vs float64, 40 sequential LSTM steps).  Keras itself is absent, so the oracle's
layer semantics are "parity unpinned" against keras."""
import ctypes
import json
import os

import numpy as np
import pytest

from islpose import translate
from oracle import sign_classifier as ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL_ABS, TOL_REL = 1e-5, 1e-4


def test_populate_features_matches_reference_golden():
    from src import util
    z = np.load(os.path.join(GOLDEN, "g2_body_post.npz"))
    cases = json.load(open(os.path.join(GOLDEN, "g9_translator_features.json")))
    assert len(cases) >= 12
    for c in cases:
        cand, subset = z[c["case"] + "/candidate"], z[c["case"] + "/subset"]
        circles, _ = util.get_bodypose(cand, subset, "body25")
        _, peaks = util.get_handpose([np.array(h, np.int64) for h in c["hands"]])
        got = translate.populate_features(circles, peaks)
        exp = np.array(c["features"])
        assert got.shape == (156,) and str(got.dtype) == c["dtype"]
        np.testing.assert_array_equal(got, exp)
        np.testing.assert_array_equal(ref.populate_features(circles, peaks), exp)


def test_populate_features_edge_cases():
    # nothing detected: the reference's list holds only the int 0 -> int64 zeros
    z = translate.populate_features([], [[], []])
    assert z.dtype == np.int64 and not z.any()
    assert ref.populate_features([], [[], []]).dtype == np.int64
    # more than 15 body circles: only the first 15 are kept; one hand in slot 1
    circles = [(float(i), float(100 + i)) for i in range(40)]
    peaks = [[], [(i, 2 * i, str(i)) for i in range(21)]]
    f = translate.populate_features(circles, peaks)
    np.testing.assert_array_equal(f, ref.populate_features(circles, peaks))
    assert f[14] == 14 and f[29] == 114 and not f[30:93].any() and f[93 + 21 + 5] == 10 and f[-1] == 20


def test_keras_weight_layout_matches_native_count():
    import ctypes as C
    from islpose import runtime as rt
    if not os.path.exists(rt.LIB_PATH):
        pytest.skip("libislpose.so not built")
    for F, K in ((156, 167), (10, 3)):
        n = C.c_int64()
        rt.check(rt.lib().isl_sign_param_count(F, K, C.byref(n)))      # host-only call
        assert n.value == sum(int(np.prod(s)) for s in translate.keras_weight_shapes(F, K))
    assert rt.lib().isl_sign_param_count(300, 5, C.byref(n)) == rt.ISL_E_ARG
    w = translate.keras_default_weights()
    assert [a.shape for a in w] == translate.keras_weight_shapes()
    assert len(w) == 28


def test_keras_weights_npz_round_trip(tmp_path):
    """np.savez(path, *model.get_weights()) -> load_keras_weights: same arrays, same order."""
    w = translate.keras_default_weights(seed=5)
    p = str(tmp_path / "w.npz")
    np.savez(p, *w)
    back = translate.load_keras_weights(p)
    assert len(back) == len(w) == 28
    for a, b in zip(w, back):
        np.testing.assert_array_equal(a, b)


def _trained_like_weights(F=156, K=167, seed=3):
    """Keras default init plus BN statistics of pixel-scale features, so the LSTMs see
    unit-scale inputs (as with trained weights) instead of saturating."""
    w = translate.keras_default_weights(F, K, seed)
    rng = np.random.RandomState(seed + 1)
    w[0] = rng.uniform(0.5, 1.5, F).astype(np.float32)
    w[1] = rng.uniform(-0.2, 0.2, F).astype(np.float32)
    w[2] = rng.uniform(0, 300, F).astype(np.float32)
    w[3] = rng.uniform(50, 200, F).astype(np.float32) ** 2
    for base in (17, 22):
        w[base:base + 4] = [rng.uniform(0.5, 1.5, 32).astype(np.float32), rng.uniform(-.2, .2, 32).astype(np.float32),
                            rng.uniform(-.3, .3, 32).astype(np.float32), rng.uniform(0.5, 2, 32).astype(np.float32)]
    return w


def _windows(B, T=20, F=156, seed=0, masked=0.25):
    rng = np.random.RandomState(seed)
    x = rng.uniform(0, 600, (B, T, F)).astype(np.float32)
    lo = min(30, F // 2)
    x[:, :, lo:] = np.where(rng.rand(B, T, F - lo) < 0.3, 0, x[:, :, lo:])   # missing joints
    x[rng.rand(B, T) < masked] = 0                                            # frames with nothing detected
    return x


def test_oracle_masking_semantics():
    """Keras masking: a masked (all-zero) frame is skipped by both directions, so where
    the empty frames sit in the window does not change the prediction."""
    w = _trained_like_weights(F=12, K=7)
    rng = np.random.RandomState(1)
    real = rng.uniform(0, 600, (13, 12))
    a = np.zeros((20, 12))
    a[:13] = real
    b = np.zeros((20, 12))
    b[[0, 2, 3, 5, 8, 9, 10, 11, 13, 15, 16, 18, 19]] = real
    pa, pb = ref.classify(w, a), ref.classify(w, b)
    np.testing.assert_allclose(pa, pb, rtol=1e-12, atol=1e-14)
    assert abs(pa.sum() - 1) < 1e-12
    c = a.copy()
    c[13] = real[0]                      # one more real frame does change it
    assert np.abs(ref.classify(w, c) - pa).max() > 1e-6


class _FakePose:
    """call_batch stand-in (no GPU): frame i -> one body joint at (i, 2i) and one hand."""

    def call_batch(self, frames):
        out = []
        for f in frames:
            v = float(f[0, 0, 0])
            cand = np.array([[v, 2 * v, 0.9, 0.0]])
            subset = np.full((1, 27), -1.0)
            subset[0, 0], subset[0, -2], subset[0, -1] = 0, 0.9, 1
            hand = np.zeros((21, 2), np.int64)
            hand[3] = (int(v) + 1, 7)
            out.append((cand, subset, [hand]))
        return out


def _fake_translator(layer):
    from src.ISL_Model_parameter import ISLSignPosTranslator
    t = ISLSignPosTranslator(None, None, layer)
    t.call_batch = _FakePose().call_batch
    return t


def test_translator_window_logic():
    seen = []

    def layer(x):
        seen.append(np.array(x))
        return np.asarray(x).reshape(len(x), -1).sum(axis=1)

    t = _fake_translator(layer)
    frames = np.zeros((23, 4, 4, 3), np.uint8)
    frames[:, 0, 0, 0] = np.arange(23) + 1
    with pytest.raises(AttributeError):              # reference: list has no .shape (:331-333)
        t.call(frames[:19])
    with pytest.raises(ValueError):                  # reference: reshape(1, 20, 156) of 23 rows
        t.call(frames)
    r = t.call(frames[2:22])
    x = seen[-1]
    assert x.shape == (1, 20, 156) and x.dtype == np.float64
    assert x[0, 0, 0] == 3 and x[0, 0, 15] == 6 and x[0, 0, 30 + 3] == 4 and x[0, 0, 30 + 42 + 3] == 3
    stream = t.translate_stream(frames, batch=5)
    assert seen[-1].shape == (4, 20, 156)
    assert stream[2] == r[0]
    for s in range(4):
        np.testing.assert_array_equal(seen[-1][s], t.features(frames[s:s + 20]))
    assert len(t.translate_stream(frames[:10])) == 0


def test_translator_rolling_window_reuses_rows():
    """The demo's rolling window: after the first call only the new frame is computed,
    and every result equals a fresh computation."""
    seen = []
    t = _fake_translator(lambda x: (seen.append(np.array(x)), np.asarray(x).sum())[1])
    counted = []
    inner = t.call_batch
    t.call_batch = lambda f: (counted.append(len(f)), inner(f))[1]
    frames = np.zeros((25, 4, 4, 3), np.uint8)
    frames[:, 0, 0, 0] = np.arange(25) + 1
    for s in range(6):
        t.call(frames[s:s + 20])
    assert counted == [20, 1, 1, 1, 1, 1]
    fresh = _fake_translator(lambda x: np.asarray(x).sum())
    for s in range(6):
        np.testing.assert_array_equal(seen[s][0], fresh.features(frames[s:s + 20]))
    assert len(t._rows) <= t.cache_frames


# ---------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_sign_classifier_matches_oracle():
    w = _trained_like_weights()
    clf = translate.SignClassifier(w)
    x = _windows(37)
    x[5] = 0                                          # a window with nothing detected
    got = clf(x).cpu().numpy()
    exp = ref.classify_batch(w, x)
    assert got.shape == (37, 167)
    err = np.abs(got - exp) - (TOL_ABS + TOL_REL * exp)
    assert err.max() <= 0, "max excess %g" % err.max()
    np.testing.assert_allclose(got.sum(axis=1), 1, atol=1e-5)
    assert (got.argmax(1) == exp.argmax(1)).all()
    # batch invariance: one window alone gives the same bits
    np.testing.assert_array_equal(clf(x[7]).cpu().numpy()[0], got[7])


@pytest.mark.gpu
@pytest.mark.parametrize("T,F,K", [(1, 156, 167), (7, 10, 3), (32, 256, 1024), (20, 156, 2)])
def test_sign_classifier_shapes(T, F, K):
    w = _trained_like_weights(F, K, seed=T)
    clf = translate.SignClassifier(w, n_features=F, n_classes=K)
    x = _windows(5, T, F, seed=T, masked=0.2)
    got = clf(x).cpu().numpy()
    exp = ref.classify_batch(w, x)
    assert (np.abs(got - exp) <= TOL_ABS + TOL_REL * exp).all()


@pytest.mark.gpu
def test_sign_classifier_bad_args():
    from islpose import runtime as rt
    clf = translate.SignClassifier()
    with pytest.raises(rt.IslError):
        clf(np.zeros((1, 33, 156), np.float32))       # window > 32
    with pytest.raises(ValueError):
        clf(np.zeros((1, 20, 155), np.float32))
    assert clf(np.zeros((0, 20, 156), np.float32)).shape == (0, 167)
    with pytest.raises(ValueError):
        translate.SignClassifier(translate.keras_default_weights()[:-1])


@pytest.mark.gpu
def test_translator_end_to_end():
    """Synthetic-weight body + hand nets -> features -> HIP classifier; translate_stream
    rows equal call() on each window and the oracle on the same feature windows."""
    import torch
    from islpose import synth
    from src.body import Body
    from src.hand import Hand
    from src.ISL_Model_parameter import ISLSignPosTranslator
    wts = lambda k: {n: torch.from_numpy(v) for n, v in synth.synth_weights(k).items()}  # noqa: E731
    w = _trained_like_weights()
    clf = translate.SignClassifier(w)
    t = ISLSignPosTranslator(Body(wts(0), "body25").model, Hand(wts(2)).model, clf)
    frames = synth.synth_frames(22, 184, 240, seed=12)
    # random weights detect many people; get_handpose (as in the reference) raises on a
    # third hand, so keep the first two hands of each frame for this test
    full = t.call_batch
    t.call_batch = lambda f: [(c, s, h[:2]) for c, s, h in full(f)]
    feats = t.features(frames)
    assert feats.shape == (22, 156) and np.count_nonzero(feats) > 0
    probs = t.translate_stream(frames).cpu().numpy()
    assert probs.shape == (3, 167)
    one = t.call(frames[1:21]).cpu().numpy()
    np.testing.assert_array_equal(one[0], probs[1])
    exp = ref.classify_batch(w, translate.sliding_windows(feats).astype(np.float32))
    assert (np.abs(probs - exp) <= TOL_ABS + TOL_REL * exp).all()
