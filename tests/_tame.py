"""Test helper: tamed synthetic body weights (islpose.synth.tame_heat_layer), with the
calibration heat map computed by the oracle network.  Both the GPU path and the
oracle then use the same tamed weights; the PAF and hand layers are untouched."""
from islpose import synth
from oracle import cpu_ref


def tame_body(weights, frame, scale=0.5, gain=0.05, model_type="body25"):
    fn = cpu_ref.make_net_fn(model_type, weights)
    im, _, _ = cpu_ref.net_input(frame, scale)
    _, heat = fn(im)
    return synth.tame_heat_layer(weights, heat, model_type, gain)
