"""Per-frame latency of the unchanged-script path (batch 1): Body(...)(frame),
Hand(...)(crop) and ISLSignPos.call(frame), synthetic weights, 368x656 frames."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "isl-signlanguage-translation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, n=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    from islpose import synth
    from src.body import Body
    from src.hand import Hand
    from src.ISL_Model_parameter import ISLSignPos
    w = lambda k: {n: torch.from_numpy(v) for n, v in synth.synth_weights(k).items()}  # noqa: E731
    body, hand = Body(w(0), "body25"), Hand(w(2))
    frame = synth.synth_frames(1, 368, 656, seed=3)[0]
    crop = synth.synth_frames(1, 160, 160, seed=4)[0]
    isl = ISLSignPos(body.model, hand.model)
    out = {"body_call_ms": round(timed(lambda: body(frame)), 3),
           "hand_call_ms": round(timed(lambda: hand(crop)), 3)}
    # the ISL wrapper: body (scale 0.5) + handDetect + hands of that frame
    out["isl_sign_pos_call_ms"] = round(timed(lambda: isl.call(frame)), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
