"""bench.py's multi-rank control flow on CPU (gloo, world_size 2): the env ranges the ranks own,
the barrier-bracketed timed loop and the slowest-rank elapsed time every rank reports.

The driver launches `bench.py --gpus N` under torchrun, one rank per GPU; the GPU parts are the
engine's (test_sharding_gpu.py), what is checked here is the plumbing around them."""
import os
import socket
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        strong = bench.env_range(rank, world, 65537, 0)
        weak = bench.env_range(rank, world, 65536, 8192)
        calls = {"steps": 0, "sync": 0, "hook": 0}

        def one_step():
            calls["steps"] += 1
            time.sleep(0.002 * (rank + 1))  # rank 1 is the slow one

        def sync():
            calls["sync"] += 1

        def hook():
            calls["hook"] += 1

        elapsed = bench.timed_loop(one_step, 20, 3, sync, True, before_timing=hook)
        slowest = bench.max_over_ranks(elapsed, torch.device("cpu"))
        out = [None] * world
        dist.all_gather_object(out, (strong, weak, elapsed, slowest, dict(calls)))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def test_env_range_is_shard_range():
    """bench.env_range and vector.shard_range give the same ranges for non-divisible totals."""
    import bench
    from libzombsole_amd.vector import shard_range
    for total in (65537, 65536, 8191, 10, 3):
        for world in (1, 2, 3, 4, 7, 8):
            covered = 0
            for rank in range(world):
                n, env0, kind, tot = bench.env_range(rank, world, total)
                assert (env0, n) == shard_range(total, rank, world) and kind == "strong" and tot == total
                assert env0 == covered
                covered += n
            assert covered == total


def test_bench_two_rank_control_flow():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (s0, w0, e0, m0, c0), (s1, w1, e1, m1, c1) = res
    # strong scaling: contiguous ranges covering [0, total) exactly, sizes differ by at most one
    assert s0[1] == 0 and s0[1] + s0[0] == s1[1] and s1[1] + s1[0] == 65537
    assert abs(s0[0] - s1[0]) <= 1 and s0[2] == s1[2] == "strong" and s0[3] == s1[3] == 65537
    # ... and exactly vector.shard_range's partition (the batched API's): the extra env goes to rank 0
    assert (s0[0], s0[1]) == (32769, 0) and (s1[0], s1[1]) == (32768, 32769)
    # weak scaling: a fixed count per rank, node total = count x ranks
    assert (w0[0], w0[1], w1[1], w0[2], w0[3]) == (8192, 0, 8192, "weak", 16384)
    # exactly W + K steps, the device synced around the warmup and both sides of the timed window
    assert c0 == c1 == {"steps": 23, "sync": 3, "hook": 1}
    # every rank reports the slowest rank's time; the closing barrier already stretches the fast rank's
    # window over the slow rank's 20 steps of 4 ms
    assert m0 == m1 == max(e0, e1) and min(e0, e1) >= 20 * 0.004


def _bench(argv, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "TORCHELASTIC_RUN_ID")):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + argv, cwd=root, env=env,
                          capture_output=True, text=True, timeout=240)


def test_bench_gpus_flag_spawns_the_ranks():
    """`bench.py --gpus 2` with no launcher starts the two rank processes itself (RANK / WORLD_SIZE /
    MASTER_* as torchrun sets them); rank 0's JSON line reports both ranks' env ranges and n_gpus 2."""
    import json
    r = _bench(["--gpus", "2", "--dry-run", "--steps", "6", "--warmup", "2", "--envs", "65537"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["dry_run"] and out["total_envs"] == 65537
    assert [tuple(x) for x in out["rank_env_ranges"]] == [(0, 32769), (32769, 32768)]


def test_bench_gpus_flag_must_match_launcher():
    """Under a launcher (WORLD_SIZE set) a different --gpus is an error, not a silent 1-rank run."""
    r = _bench(["--gpus", "4", "--dry-run", "--steps", "2", "--warmup", "0"],
               {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
    r = _bench(["--gpus", "1", "--dry-run", "--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
