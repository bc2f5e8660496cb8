"""Multi-rank env sharding on CPU (gloo, world_size 2), SURVEY.md §8(e).

Envs are independent and env i is seeded base+i, so a node's results must not depend on
how envs are split over ranks: each rank runs its `shard_range` of the bench workload
through the C oracle (test infrastructure) and the all-reduced checksum must equal the
single-rank run.  The optional observation gather (`gather_observations`) is checked with
rank-tagged tensors, on shards of unequal size (25 envs over 2 ranks: 13 + 12), and C5's
per-step, double-buffered `StepGather` (rewards / done / truncated / listed / was_reset in one flat byte
buffer beside the observations, padded output sets) over several steps, each step's gathered values checked.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from libzombsole_amd import _abi


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _builder():
    return _abi.multi_env_config(1, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                 max_episode_steps=1000, obs_dtype=_abi.DTYPE_I64)


TOTAL, STEPS = 25, 60


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from libzombsole_amd.vector import gather_observations, shard_range
        from oracle.oracle import run_batch
        e0, n = shard_range(TOTAL, rank, world)
        cnt, csum = run_batch(_builder(), e0, n, STEPS, 7, threads=1)
        parts = [None] * world
        dist.all_gather_object(parts, (cnt, csum))
        from libzombsole_amd.engine import StepOutputs
        from libzombsole_amd.vector import StepGather
        obs = torch.full((n, 2, 3, 5, 5), rank, dtype=torch.int32)
        g = gather_observations(obs)
        g2 = gather_observations(obs, sizes=[shard_range(TOTAL, r, world)[1] for r in range(world)])
        # a stand-in engine (CPU tensors) for the per-step exchange: its step writes step-tagged values
        gl = torch.arange(e0, e0 + n)

        class Fake(object):
            N, A, multi, obs_shape, obs_dtype, device, torch = n, 2, True, (2, 3, 5, 5), torch.int32, \
                torch.device("cpu"), torch

            def outputs(self, rows=None, obs=None, flat=None):
                return StepOutputs(self, max(rows or n, n), obs, flat)

        def run(t):
            def fill(out):
                out.obs[:n] = 10 * gl.view(-1, 1, 1, 1, 1).int() + 1000 * t
                out.rewards[:n] = ((gl.double() / 4) + t).view(-1, 1).repeat(1, 2)
                out.done[:n] = ((gl + t) % 2).to(torch.uint8)
                out.trunc[:n] = ((gl + t) % 3 == 0).to(torch.uint8)
                out.listed[:n] = torch.stack([(gl + t) % 5 != 0, (gl + 2 * t) % 7 != 0], 1).to(torch.uint8)
                out.was_reset[:n] = ((gl * 3 + t) % 4 == 0).to(torch.uint8)
            return fill

        sg = StepGather(Fake())
        ok = torch.equal(g, g2) and len(sg.sets) == 2 and all(s.obs.shape[0] == 13 for s in sg.sets)
        # the output sets are this rank's slices of the gather buffers (in-place collectives)
        ok = ok and all(s.obs.data_ptr() == sg.g_obs[k][13 * rank:].data_ptr() for k, s in enumerate(sg.sets))
        ga = torch.arange(TOTAL)
        for t in range(5):
            used = sg.step(run(t))
            ok = ok and used is sg.sets[t % 2]
            ok = ok and (torch.equal(sg.obs()[:, 0, 0, 0, 0], ga.int() * 10 + 1000 * t)
                         and torch.equal(sg.rewards()[:, 1], ga.double() / 4 + t)
                         and torch.equal(sg.done(), ((ga + t) % 2).to(torch.uint8))
                         and torch.equal(sg.truncated(), ((ga + t) % 3 == 0).to(torch.uint8))
                         and torch.equal(sg.listed(), torch.stack([(ga + t) % 5 != 0, (ga + 2 * t) % 7 != 0],
                                                                  1).to(torch.uint8))
                         and torch.equal(sg.was_reset(), ((ga * 3 + t) % 4 == 0).to(torch.uint8)))
        if rank == 0:
            q.put((sum(c for c, _ in parts), sum(s for _, s in parts) % (1 << 64), g[:, 0, 0, 0, 0].tolist(), ok))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_match_single_rank():
    from oracle.oracle import run_batch
    cnt1, csum1 = run_batch(_builder(), 0, TOTAL, STEPS, 7, threads=1)
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
    cnt2, csum2, tags, ok = res
    assert cnt2 == cnt1 == TOTAL * STEPS
    assert csum2 == csum1  # checksums add over envs (oracle/zs_oracle.c zo_run_batch)
    assert tags == [0] * 13 + [1] * 12
    assert ok
