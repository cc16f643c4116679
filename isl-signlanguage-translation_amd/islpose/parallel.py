"""Frame sharding across GPUs (one process per GPU, no collective on the data path).

Frames are independent units: each rank takes a contiguous shard
of the frame index range, runs the whole hot path on its own device, and the
per-frame keypoints (a few KB) are gathered on rank 0 on the host -- the
MI355X counterpart of the reference's mp.Process + mp.Queue pipeline
(extract_features_mp.py:183-239), which ran every worker on cuda:0.
"""
from __future__ import annotations

import os


def shard_bounds(n_items: int, rank: int, world: int):
    """Contiguous [start, end) of `rank`'s shard; sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    q, r = divmod(n_items, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def dist_env():
    """(rank, local_rank, world) from the torch.distributed.run environment (1 process = 1 GPU)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(argv, world: int, env=None, poll_s: float = 0.2):
    """Start `world` child processes running `argv` (one per GPU: RANK = LOCAL_RANK =
    r, WORLD_SIZE = world, rendezvous on 127.0.0.1) -- the launcher the reference
    builds from mp.Process (extract_features_mp.py:205-220), with every child on its
    own device instead of cuda:0.  The caller must not have touched the GPU (children
    are separate processes, never an exec of this one).  Returns (exit codes, rank-0
    stdout); the other ranks' stdout and every stderr pass through.

    Fail-fast: every child is polled; the first one to exit non-zero gets its siblings
    terminated (SIGTERM, then SIGKILL after a grace period), so one rank dying during
    init or the timed loop never leaves the others blocked at a gloo barrier until
    torch's default timeout.  Terminated siblings report their signal exit codes."""
    import subprocess
    import sys
    import threading
    import time
    port = free_port()
    procs = []
    for r in range(world):
        e = dict(os.environ if env is None else env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=e,
                                      stdout=subprocess.PIPE if r == 0 else None, text=True))
    # rank 0's stdout is drained by a thread so polling never blocks on a full pipe
    chunks = []
    reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    failed = False
    while True:
        codes = [p.poll() for p in procs]
        if any(c not in (None, 0) for c in codes):
            failed = True
            break
        if all(c is not None for c in codes):
            break
        time.sleep(poll_s)
    if failed:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 10.0
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    reader.join(timeout=10.0)
    codes = [p.wait() for p in procs]
    return codes, "".join(c for c in chunks if c)


def run_sharded(n_frames, get_frames, estimate, batch: int, rank: int, world: int):
    """Process this rank's shard in batches: get_frames(start, end) -> frames,
    estimate(frames) -> list of per-frame results. Returns [(frame_index, result)]."""
    start, end = shard_bounds(n_frames, rank, world)
    out = []
    for s in range(start, end, batch):
        e = min(s + batch, end)
        res = estimate(get_frames(s, e))
        out.extend(zip(range(s, e), res))
    return out


def gather_to_rank0(local, rank: int, world: int, group=None):
    """Host-side gather of per-frame results (no device collective); rank 0 gets
    them ordered by frame index, other ranks get None."""
    if world == 1:
        return [r for _, r in sorted(local, key=lambda t: t[0])]
    import torch.distributed as dist
    bucket = [None] * world if rank == 0 else None
    dist.gather_object(local, bucket, dst=0, group=group)
    if rank != 0:
        return None
    merged = [item for part in bucket for item in part]
    return [r for _, r in sorted(merged, key=lambda t: t[0])]
