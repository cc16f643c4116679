"""BodyEstimator.decode on hand-built result records (CPU: isl_body_layout is a host
function): the vectorised candidate / subset equal the reference's construction
(body.py:101-107, 183: peaks of parts 0..24 in order, consecutive ids, shape (0,)
when empty), with and without the detail lists."""
import numpy as np

from islpose import runtime as rt
from islpose.body import BodyEstimator, DEFAULT_CAPS


def _records(est, caps, n, rng):
    lay = rt.body_layout(est.kind, rt.IslCaps(**caps))
    host = np.zeros(n * lay.record_bytes, np.uint8)
    nparts, nl, mpk = est.njoint - 1, 24, caps["max_peaks"]
    truth = []
    for f in range(n):
        rec = host[f * lay.record_bytes:(f + 1) * lay.record_bytes]
        npk = rng.randint(0, 4, nparts).astype(np.int32) if f % 3 else np.zeros(nparts, np.int32)
        rec[lay.n_peaks:lay.n_peaks + 4 * nparts] = npk.view(np.uint8)
        pk = rec[lay.peaks:lay.peaks + nparts * mpk * 24].view(np.float64).reshape(nparts, mpk, 3)
        pk[:] = rng.uniform(0, 600, pk.shape).round()
        pk[:, :, 2] = rng.uniform(0, 1, (nparts, mpk))
        nrows = f % 4
        rec[lay.n_rows:lay.n_rows + 4] = np.array([nrows], np.int32).view(np.uint8)
        sb = rec[lay.subset:lay.subset + caps["max_rows"] * 27 * 8].view(np.float64).reshape(-1, 27)
        sb[:] = rng.uniform(-1, 30, sb.shape)
        rec[lay.n_conns:lay.n_conns + 4 * 32] = np.array([1] * nl + [-1] * (32 - nl), np.int32).view(np.uint8)
        rows, pid = [], 0
        for p in range(nparts):
            for i in range(int(npk[p])):
                x, y, s = pk[p, i]
                rows.append((x, y, s, float(pid)))
                pid += 1
        truth.append((np.array(rows, np.float64) if rows else np.array([]), sb[:nrows].copy(), npk.copy()))
    return host, lay, truth


def test_decode_vectorised_matches_reference_construction():
    est = BodyEstimator.__new__(BodyEstimator)
    est.kind, est.njoint, est.npaf = rt.ISL_BODY25, 26, 52
    caps = dict(DEFAULT_CAPS)
    host, lay, truth = _records(est, caps, 7, np.random.RandomState(3))
    for details in (False, True):
        res = est.decode(host, lay, caps, 7, details)
        for r, (cand, subset, npk) in zip(res, truth):
            assert r.candidate.dtype == np.float64 and r.candidate.shape == cand.shape
            assert np.array_equal(r.candidate, cand)
            assert np.array_equal(r.subset, subset)
            if details:
                assert [len(p) for p in r.all_peaks] == list(npk)
                flat = [q for p in r.all_peaks for q in p]
                assert [q[3] for q in flat] == list(range(len(flat)))
                if len(flat):
                    assert np.array_equal(np.array([q[:3] for q in flat], np.float64), cand[:, :3])
            else:
                assert r.all_peaks is None
