"""Env sharding and the RCCL exchange on one MI355X.

- Two engine handles owning global env ranges [0, N/2) and [N/2, N) (seeds = global index, as
  bench.py's ranks do) produce exactly the observations, rewards and flags of one handle over
  [0, N): trajectories do not depend on how the envs are split over GPUs.
- A world_size-1 RCCL ("nccl") process group runs `gather_observations` and C5's per-step
  `StepGather` (the bench's pack + all-gather) on the engine's device tensors; the gathered
  tensors equal the local ones.
"""
import os
import socket

import pytest

from libzombsole_amd import _abi

pytestmark = pytest.mark.gpu


def _c2(n):
    return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                 minimum_zombies=0, max_episode_steps=25)


def _c5(n):
    return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1", "2", "3"], initial_zombies=20,
                                 minimum_zombies=0, max_episode_steps=1000, obs_dtype=_abi.DTYPE_I16)


@pytest.mark.parametrize("total", [4096, 4097])
def test_two_handles_equal_one(total):
    import torch

    from libzombsole_amd.engine import Engine
    from libzombsole_amd.vector import shard_range

    whole = Engine(_c2(total))
    whole.seed(list(range(total)))
    whole.reset()
    parts = []
    for r in range(2):
        e0, n = shard_range(total, r, 2)
        eng = Engine(_c2(n))
        eng.seed([e0 + i for i in range(n)])
        eng.reset()
        parts.append(eng)
    for t in range(1, 61):  # TimeLimit 25: two autoreset waves
        for eng in [whole] + parts:
            eng.step_graph(t, 7)
        torch.cuda.synchronize()
        for name in ("obs", "rewards", "done", "trunc", "listed", "was_reset"):
            cat = torch.cat([getattr(p, name) for p in parts], dim=0)
            assert torch.equal(cat, getattr(whole, name)), (name, t)
    for eng in [whole] + parts:
        eng.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("self_exchange", [True, False])
def test_rccl_world1_gather(self_exchange):
    """World size 1: with self_exchange the in-place RCCL all-gathers run (the exchange's code path at one
    rank); without, StepGather skips them (its output sets are the whole buffers) and the results are
    the same."""
    import torch
    import torch.distributed as dist

    from libzombsole_amd.engine import Engine
    from libzombsole_amd.vector import StepGather, gather_observations

    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        eng = Engine(_c5(2048))
        eng.seed(list(range(2048)))
        eng.reset()
        g = StepGather(eng, self_exchange=self_exchange)
        assert g.skip == (not self_exchange)
        ref = Engine(_c5(2048))  # the same envs stepped without the exchange, default outputs
        ref.seed(list(range(2048)))
        ref.reset()
        for t in range(1, 9):
            out = g.step(lambda o: eng.step_graph(t, 7, out=o))
            assert out is g.sets[(t - 1) % 2]  # double-buffered outputs, graphs cached per set
            ref.step_graph(t, 7)
            torch.cuda.synchronize()
            assert torch.equal(g.obs(), ref.obs)
            assert torch.equal(out.obs, ref.obs)
            assert torch.equal(g.rewards(), ref.rewards)
            assert torch.equal(g.done(), ref.done)
            assert torch.equal(g.truncated(), ref.trunc)
            assert torch.equal(g.listed(), ref.listed)
            assert torch.equal(g.was_reset(), ref.was_reset)
            assert torch.equal(gather_observations(ref.obs), ref.obs)
            assert torch.equal(gather_observations(ref.obs, sizes=[2048]), ref.obs)
        ref.close()
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("self_exchange", [True, False])
def test_rccl_world1_gather_in_flight(self_exchange):
    """C5's exchange with steps in flight: 8 gathered steps issued back to back with no host sync and no
    wait on the caller's stream, so step t + 1 computes while step t's collectives run, and a set is
    written again only after the collectives of two steps earlier.  A consumer on the communication stream
    (StepGather.step(after=...)) hashes every step's gathered observations, rewards and flags (done, truncated, listed,
    was_reset) there; the
    hashes, and the last two sets' gathered tensors, equal those of a reference engine stepped alone
    (gym/multiagent_env.py:111-171)."""
    import torch
    import torch.distributed as dist

    from libzombsole_amd.engine import Engine
    from libzombsole_amd.vector import StepGather

    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1,
                            device_id=dev)
    try:
        n, steps = 8192, 8
        eng = Engine(_c5(n))
        eng.seed(list(range(n)))
        eng.reset()
        g = StepGather(eng, self_exchange=self_exchange)
        hashes = torch.zeros((steps, 2), dtype=torch.int64, device=dev)
        wts = torch.arange(1, g.g_obs[0].numel() + 1, dtype=torch.int64, device=dev) % 1000003

        def hash_into(t):
            def after(k):  # runs on the communication stream, after the collectives filling set k
                hashes[t - 1, 0] = (g.g_obs[k].reshape(-1).to(torch.int64) * wts).sum()
                hashes[t - 1, 1] = (g.g_flat[k].to(torch.int64) * wts[:g.g_flat[k].numel()]).sum()
            return after

        for t in range(1, steps + 1):
            g.step(lambda o: eng.step_graph(t, 7, out=o), after=hash_into(t))
        ref = Engine(_c5(n))
        ref.seed(list(range(n)))
        ref.reset()
        exp = torch.zeros_like(hashes)
        last = {}
        for t in range(1, steps + 1):
            ref.step_graph(t, 7)
            exp[t - 1, 0] = (ref.obs.reshape(-1).to(torch.int64) * wts).sum()
            exp[t - 1, 1] = (ref.out.flat.to(torch.int64) * wts[:ref.out.flat.numel()]).sum()
            if t > steps - 2:
                last[t] = (ref.obs.clone(), ref.out.flat.clone())
        torch.cuda.synchronize()
        g.wait()
        torch.cuda.synchronize()
        assert torch.equal(hashes, exp), (hashes - exp).abs().sum(dim=1).tolist()
        for t in (steps - 1, steps):
            k = (t - 1) % g.depth
            assert torch.equal(g.g_obs[k], last[t][0]), t
            # rewards, done, truncated, listed, was_reset (engine.StepOutputs)
            assert torch.equal(g.g_flat[k], last[t][1]), t
        assert torch.equal(g.obs(copy=True), last[steps][0])
        ref.close()
        eng.close()
    finally:
        dist.destroy_process_group()
