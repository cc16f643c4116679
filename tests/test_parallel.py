"""Multi-process frame sharding (world_size 2, gloo, CPU)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from islpose.parallel import shard_bounds, run_sharded, gather_to_rank0


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 32, 33, 128):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_frames, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # stand-in for the GPU estimator: a per-frame result that identifies the frame
    local = run_sharded(n_frames, lambda s, e: list(range(s, e)), lambda fr: [("frame", f, f * f) for f in fr],
                        batch=4, rank=rank, world=world)
    out = gather_to_rank0(local, rank, world)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_frames", [11, 32])
def test_gather_two_ranks_gloo(n_frames):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_frames, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert out == [("frame", f, f * f) for f in range(n_frames)]
