"""Kernel mix of the frame path's posts (run under rocprofv3 --kernel-trace): the hand post of
one crop of 500 / 800 / 1080 px (four scales), then the body post of a 1080x1920 frame with
the frame leg's tamed heat layer.  Markers: a tiny torch fill between the sections."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "isl-signlanguage-translation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from islpose import synth  # noqa: E402
from islpose.hand import HandEstimator  # noqa: E402
from islpose.body import BodyEstimator  # noqa: E402


def main():
    rgb = synth.synth_frames(2, 1080, 1920, seed=57)
    frames = torch.from_numpy(np.ascontiguousarray(rgb[..., ::-1])).cuda()
    hand = HandEstimator(synth.synth_weights(2))
    mark = torch.zeros(1, device="cuda")
    for w in (500, 800, 1080):
        boxes = [(0, 1920 - w - 10, 0, w)]
        heats = hand.run_crops(frames, boxes)
        for _ in range(4):
            hand.post_crops(boxes, heats)
        mark.fill_(float(w))
    wb = synth.synth_weights(0)
    cal = BodyEstimator(wb, "body25", scale_search=(0.5,))
    _, _, hm = cal.run_scales(frames[:1], keep_maps=True)
    wb = synth.tame_heat_layer(wb, hm[0].cpu().numpy(), "body25", gain=0.05)
    body = BodyEstimator(wb, "body25", scale_search=(0.5,))
    for i in range(4):
        body.estimate(frames[i % 2:i % 2 + 1])
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
