"""Upload of one 1080x1920x3 frame: host copy into pinned memory, the DMA, and ISLSignPos._upload
with a synchronisation at the end; median microseconds."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "isl-signlanguage-translation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def med(fn, reps=30):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return 1e6 * float(np.median(ts))


def main():
    import src.ISL_Model_parameter as P
    from islpose import synth
    from src.body import Body
    from src.hand import Hand
    rgb = synth.synth_frames(1, 1080, 1920, seed=1)[0]
    src = np.ascontiguousarray(rgb)
    pin = torch.empty(src.shape, dtype=torch.uint8, pin_memory=True)
    dev = torch.empty(src.shape, dtype=torch.uint8, device="cuda")
    print("torch threads", torch.get_num_threads())
    print("host copy_ into pinned  %8.1f us" % med(lambda: pin.copy_(torch.from_numpy(src))))
    print("np.copyto into pinned   %8.1f us" % med(lambda: np.copyto(pin.numpy(), src)))
    print("DMA pinned -> device    %8.1f us" % med(lambda: dev.copy_(pin, non_blocking=True)))
    print("pageable -> device      %8.1f us" % med(lambda: dev.copy_(torch.from_numpy(src))))
    tw = lambda d: {k: torch.from_numpy(v) for k, v in d.items()}  # noqa: E731
    isl = P.ISLSignPos(Body(tw(synth.synth_weights(0)), "body25").model, Hand(tw(synth.synth_weights(2))).model)
    print("ISLSignPos._upload       %8.1f us" % med(lambda: isl._upload(rgb[:, :, ::-1])))


if __name__ == "__main__":
    main()
