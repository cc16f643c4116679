"""Peaks and persons per frame of the frame leg's workload (1080x1920 synthetic frames, tamed
body heat layer): how large the limb scoring's pair sets are."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "isl-signlanguage-translation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from islpose import synth  # noqa: E402
from islpose.body import BodyEstimator  # noqa: E402
from src.body import Body  # noqa: E402
from src.hand import Hand  # noqa: E402
from src.ISL_Model_parameter import ISLSignPos  # noqa: E402


def main():
    T = 16
    rgb = synth.synth_frames(T, 1080, 1920, seed=57)
    wb = synth.synth_weights(0)
    cal = BodyEstimator(wb, "body25", scale_search=(0.5,))
    _, _, heats = cal.run_scales(torch.from_numpy(np.ascontiguousarray(rgb[:1, ..., ::-1])).cuda(), keep_maps=True)
    wb = synth.tame_heat_layer(wb, heats[0].cpu().numpy(), "body25", gain=0.05)
    tw = lambda d: {k: torch.from_numpy(v) for k, v in d.items()}  # noqa: E731
    isl = ISLSignPos(Body(tw(wb), "body25").model, Hand(tw(synth.synth_weights(2))).model)
    for i in range(T):
        c, s, hands = isl.call(rgb[i][:, :, ::-1])
        print("frame %d peaks %d persons %d hands %d" % (i, len(c), len(s), len(hands)))


if __name__ == "__main__":
    main()
