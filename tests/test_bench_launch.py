"""bench.py's multi-rank launch on the CPU: `--gpus N` without a torch.distributed.run
environment starts N rank processes itself (islpose.parallel.spawn_ranks), the ranks
meet over gloo, shard the frames disjointly and rank 0 reports (extract_features_mp.py:
183-239 is the reference's process launcher).  --dry-run keeps the GPU out of it."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    e = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    e["HIP_VISIBLE_DEVICES"] = ""
    return e


def _run(*argv):
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + list(argv), env=_env(),
                          capture_output=True, text=True, timeout=240)


def test_bench_spawns_two_ranks_dry_run():
    r = _run("--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1", "--batch", "4")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert len(lines) == 1, r.stdout          # rank 0's JSON line only (gloo's connection lines go to stderr)
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["world_observed"] == 2
    assert out["shards"] == [[0, 4], [4, 8]]  # disjoint frame shards
    assert out["steps"] == 3 and out["elapsed_max_s"] > 0


def test_bench_single_rank_dry_run():
    r = _run("--dry-run", "--steps", "1", "--warmup", "0", "--batch", "2")
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 1 and out["shards"] == [[0, 2]]


def test_bench_rejects_world_mismatch():
    e = _env()
    e.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"], env=e,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_bench_launch_fails_fast_when_a_rank_dies():
    """One rank exits 1 right after the group is up; its sibling would block at the next
    gloo barrier.  The launcher must notice the failure, terminate the sibling and exit
    non-zero long before the collective timeout (--pg-timeout 120 s here)."""
    import time
    t0 = time.time()
    r = _run("--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1", "--batch", "4", "--fail-rank", "1")
    dt = time.time() - t0
    assert r.returncode == 1, (r.returncode, r.stderr[-2000:])
    assert "failing on request" in r.stderr
    assert dt < 60, dt


def test_spawn_ranks_kills_siblings_on_first_failure():
    """parallel.spawn_ranks: child 0 sleeps far longer than the test, child 1 exits 3;
    the launcher returns promptly with child 1's code and child 0 terminated."""
    import time
    from islpose import parallel
    prog = ("import os, sys, time\n"
            "r = int(os.environ['RANK'])\n"
            "print('rank', r, flush=True)\n"
            "time.sleep(300) if r == 0 else sys.exit(3)\n")
    t0 = time.time()
    codes, out0 = parallel.spawn_ranks(["-c", prog], 2, env=_env())
    assert time.time() - t0 < 30
    assert codes[1] == 3 and codes[0] != 0
    assert "rank 0" in out0
