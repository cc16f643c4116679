"""Probe: peak counts of the FRAME leg's 1080p frames and the body time with the limb LDS path on / off."""
import sys, os, time, json
sys.path.insert(0, "isl-signlanguage-translation_amd"); sys.path.insert(0, "tools")
import numpy as np, torch
from islpose import synth
from islpose.body import BodyEstimator
from src.body import Body
from src.hand import Hand
from src.ISL_Model_parameter import ISLSignPos
T, H, W = 8, 1080, 1920
rgb = synth.synth_frames(T, H, W, seed=57)
wb = synth.synth_weights(0)
cal = BodyEstimator(wb, "body25", scale_search=(0.5,))
_, _, heats = cal.run_scales(torch.from_numpy(np.ascontiguousarray(rgb[:1, ..., ::-1])).cuda(), keep_maps=True)
wb = synth.tame_heat_layer(wb, heats[0].cpu().numpy(), "body25", gain=0.05)
tw = lambda d: {k: torch.from_numpy(v) for k, v in d.items()}
isl = ISLSignPos(Body(tw(wb), "body25").model, Hand(tw(synth.synth_weights(2))).model)
body = isl._estimators()[0]
for i in range(T):
    (c, sb), = body.estimate(isl._upload(rgb[i][:, :, ::-1]))
    print("frame", i, "peaks", len(c), "subset", len(sb), "caps", body.caps)
torch.cuda.synchronize()
for mode in ("1", "0", "1"):
    os.environ["ISLPOSE_LIMB_LDS"] = mode
    t0 = time.perf_counter()
    for i in range(T):
        body.estimate(isl._upload(rgb[i][:, :, ::-1]))
    torch.cuda.synchronize()
    print("LIMB_LDS", mode, "ms/frame", (time.perf_counter() - t0) / T * 1e3)
