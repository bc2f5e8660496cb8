"""The learner's step as a graph: caller-supplied actions replayed through zs_step_graph with
n_discrete = 0 (`Engine.step_graphed`, `BatchedZombsole.step`), against the oracle.

The reference takes the caller's actions every tick (`zombsole/gym/multiagent_env.py:111-171`,
`zombsole/gym_env.py:99-145`).  Here those actions are written into the engine's action buffer on
the engine's stream before each graph launch:
  * at full size, by zs_gen_actions (the counter-based stream the oracle's run_hashes replays), so every
    env and step is compared through the per-env step hashes;
  * on a small batch, by `bench.external_policy` (torch ops on the previous step's observations, the
    loop `bench.py --policy external` times), every step's observations, rewards and flags compared with
    one oracle env per batch env driven by the same actions.
"""
import numpy as np
import pytest

from libzombsole_amd import _abi

pytestmark = pytest.mark.gpu


def c3(n, max_steps=1000):
    return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                 minimum_zombies=0, max_episode_steps=max_steps)


def c5(n, max_steps=1000):
    return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1", "2", "3"], initial_zombies=20,
                                 minimum_zombies=0, max_episode_steps=max_steps, obs_dtype=_abi.DTYPE_I16)


def c4(n, max_steps=1000):
    return _abi.multi_env_config(n, "safehouse", [], "city128", ["0", "1", "2", "3"], initial_zombies=50,
                                 minimum_zombies=50, max_episode_steps=max_steps)


def run_external_hashes(make_builder, n, steps, seed0=0, nd=7, min_resets=1):
    from libzombsole_amd.engine import Engine
    from oracle.oracle import run_hashes
    from parity_hash import StepHasher

    eng = Engine(make_builder(n))
    eng.seed([seed0 + i for i in range(n)])
    eng.reset()
    hs = StepHasher(eng)
    got = np.zeros((n, steps + 1), dtype=np.uint64)
    got[:, 0] = hs.obs_hash().cpu().numpy().view(np.uint64)
    resets = 0
    for t in range(1, steps + 1):
        eng.gen_actions(t, nd)  # the caller's actions, written into the buffer the graph reads
        eng.step_graphed()
        got[:, t] = hs.step_hash().cpu().numpy().view(np.uint64)
        resets += int(eng.was_reset.sum().item())
    exp = run_hashes(make_builder(1), seed0, n, steps, nd, threads=0)
    bad = np.argwhere(got != exp)
    assert bad.size == 0, "%d of %d env-steps differ; first (env, step): %s" % (len(bad), got.size, bad[:12].tolist())
    assert resets >= min_resets, resets
    desc = eng.describe()
    eng.close()
    return desc


def test_external_graph_c3_65536():
    """The headline size with TimeLimit 16 (autoreset waves on the reset side stream) through the
    caller-actions graph."""
    d = run_external_hashes(lambda n: c3(n, max_steps=16), 65536, 36, min_resets=2 * 65536)
    assert d["step_kernel"] == "k_tick", d


def test_external_graph_c3_8192_shard():
    """The N=8 shard size: the fused step launch (k_step) reading the caller's actions."""
    d = run_external_hashes(lambda n: c3(n, max_steps=20), 8192, 45, seed0=3 * 8192)
    assert d["step_kernel"] == "k_step", d


def test_external_graph_c5_65536_int16():
    run_external_hashes(lambda n: c5(n, max_steps=12), 65536, 26, min_resets=65536)


def test_external_graph_c4_16384():
    """C4 (k_respawn after every tick), TimeLimit 15: autoreset waves at steps 16 and 32."""
    run_external_hashes(lambda n: c4(n, max_steps=15), 16384, 34, min_resets=2 * 16384)


@pytest.mark.parametrize("maker,n", [(c3, 48), (c5, 40)])
def test_batched_step_obs_policy_against_oracle(maker, n):
    """BatchedZombsole.step on actions a torch policy derives from the previous step's observations
    (bench.external_policy, written straight into the engine's action buffer): each env against an
    oracle env stepped with the same actions, every step's observations, listed rewards, done and
    truncated compared exactly; next-step autoresets included (TimeLimit 12)."""
    import torch

    from bench import external_policy
    from libzombsole_amd.vector import BatchedZombsole
    from oracle.oracle import OracleEnv

    A = 2 if maker is c3 else 4
    venv = BatchedZombsole("multi", n, "extermination", [], "bridge64", agent_ids=[str(a) for a in range(A)],
                           initial_zombies=10 if A == 2 else 20, max_episode_steps=12, base_seed=500,
                           obs_dtype=maker(1).cfg.obs_dtype)
    eng = venv.engine
    obs = venv.reset()
    policy = external_policy(eng)
    orc = []
    for i in range(n):
        o = OracleEnv(maker(1, max_steps=12))
        o.seed(500 + i)
        o.reset()
        orc.append(o)
    assert np.array_equal(obs.cpu().numpy(), np.stack([o.obs() for o in orc]))
    need = [False] * n
    resets = 0
    for t in range(1, 31):
        policy(t)
        acts = venv.actions.cpu().numpy().copy()
        obs, rew, done, trunc = venv.step(venv.actions)  # the buffer itself: no copy, graph replay
        torch.cuda.synchronize()
        g_obs, g_rew = obs.cpu().numpy(), rew.cpu().numpy()
        g_done, g_trunc, g_listed = done.cpu().numpy(), trunc.cpu().numpy(), venv.listed.cpu().numpy()
        g_reset = venv.was_reset.cpu().numpy()
        for i, o in enumerate(orc):
            if need[i]:
                e_obs = o.reset()
                need[i] = False
                resets += 1
                assert g_reset[i] == 1
                assert not g_done[i] and not g_trunc[i]
            else:
                e_obs, e_rew, d, tr, listed = o.step(acts[i])
                assert bool(g_done[i]) == d and bool(g_trunc[i]) == tr, (t, i)
                assert np.array_equal(g_listed[i].astype(bool), listed), (t, i)
                for a in range(A):
                    if listed[a]:
                        assert g_rew[i, a].hex() == e_rew[a].hex(), (t, i, a)
                need[i] = d or tr
            assert np.array_equal(g_obs[i], e_obs), (t, i)
    assert resets >= n, resets
    assert eng.describe()["envs"] == n
    venv.close()
