"""Test helper: synthetic weights whose heat output behaves like a trained net's.

Raw outputs of the seeded He-init weights put thousands of peaks on a frame (SURVEY
§8d: 40 s of reference post per frame).  For the end-to-end config tests the heat
output layer is rescaled per channel, from the oracle net's statistics on one
calibration frame: heat_k = gain * (z_k - mean_k) / std_k, so a part map crosses the
0.1 peak threshold where its field is ~0.1/gain standard deviations high (a handful
of peaks per part, a few persons per frame).  Both the GPU path and the oracle use
the same tamed weights; the PAF and hand layers are untouched."""
import numpy as np

from oracle import cpu_ref

HEAT_LAYER = {"body25": "Mconv7_stage1_L1", "coco": "Mconv7_stage6_L2"}


def tame_body(weights, frame, scale=0.5, gain=0.05, model_type="body25"):
    fn = cpu_ref.make_net_fn(model_type, weights)
    im, _, _ = cpu_ref.net_input(frame, scale)
    _, heat = fn(im)
    z = heat[0].reshape(heat.shape[1], -1).astype(np.float64)
    m, s = z.mean(1), np.maximum(z.std(1), 1e-6)
    a = gain / s
    layer = HEAT_LAYER[model_type]
    out = dict(weights)
    out[layer + ".weight"] = (weights[layer + ".weight"] * a[:, None, None, None]).astype(np.float32)
    out[layer + ".bias"] = ((weights[layer + ".bias"] - m) * a).astype(np.float32)
    return out
