"""Isolate the C4 pyramid failure: the fixture's exact setup, repeated, per switch setting; and
with the scales serialised (a sync after each scale's launches)."""
import os, sys
sys.path.insert(0, "isl-signlanguage-translation_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np, torch
from islpose import synth, runtime as rt
from islpose.body import BodyEstimator, scale_geometry
from oracle import cpu_ref
import _tame

frames = synth.synth_frames(2, 368, 656, seed=41)
w = _tame.tame_body(synth.synth_weights(0), frames[0], scale=0.5, gain=0.02)
t = torch.from_numpy(frames).cuda()
S = (0.5, 1.0, 1.5, 2.0)
fn = cpu_ref.make_net_fn("body25", w)
refs = []
for si in range(4):
    (m, nh, nw, _, _) = scale_geometry(368, 656, S)[si]
    im, _, _ = cpu_ref.net_input(frames[0], m)
    refs.append(fn(im)[0])
def check(pafs):
    return ["%.2g" % (np.abs(pafs[i][:1].cpu().numpy() - refs[i]).max() / np.abs(refs[i]).max()) for i in range(4)]
for name, env in (("default", {}), ("c12=0", {"ISLPOSE_C12": "0"}), ("wr=0", {"ISLPOSE_X3_WR": "0"}),
                  ("both0", {"ISLPOSE_C12": "0", "ISLPOSE_X3_WR": "0"})):
    for k in ("ISLPOSE_C12", "ISLPOSE_X3_WR"):
        os.environ.pop(k, None)
    os.environ.update(env)
    for rep in range(2):
        est = BodyEstimator(w, "body25", scale_search=S)
        geoms, pafs, heats = est.run_scales(t, keep_maps=True)
        torch.cuda.synchronize()
        a = check(pafs)
        geoms, pafs, heats = est.run_scales(t, keep_maps=True)   # same net, arenas warm
        torch.cuda.synchronize()
        b = check(pafs)
        print(name, rep, "fresh", a, "again", b, flush=True)
        del est
