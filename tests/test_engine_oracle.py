"""HIP engine vs the C oracle on many seeded envs (bit-exact), through the C ABI.

Covers the configs of BASELINE.json at reduced env counts, step by step with
full observations and periodic state, plus bots / rules / encodings the golden
fixtures touch only briefly.  The configs at the sizes bench.py times them
(4 096 .. 65 536 envs) are checked every env and every step in
test_fullsize_parity.py.
"""
import numpy as np
import pytest

from libzombsole_amd import _abi
from libzombsole_amd import actions as A

pytestmark = pytest.mark.gpu


def _rich_triples(seed, step, n_agents):
    return np.array([A.encode_action(A.rich_action(seed, step, a)) for a in range(n_agents)], dtype=np.int32)


def run_parity(make_builder, n_envs, steps, stream="discrete", seed0=1000, n_discrete=7, check_state_every=25,
               graph=False, launch=None, lanes=0):
    import torch
    from libzombsole_amd.engine import Engine
    from oracle.oracle import OracleEnv

    b = make_builder(n_envs).set_launch(launch)
    if lanes:
        b.cfg.lanes_per_env = lanes
    eng = Engine(b)
    kinds = [o[2] for o in eng.builder.map.obstacles]
    seeds = [seed0 + i for i in range(n_envs)]
    eng.seed(seeds)
    obs0 = eng.reset().cpu().numpy()
    refs = []
    for k, s in enumerate(seeds):
        o = OracleEnv(make_builder(1))
        o.seed(s)
        exp = o.reset()
        assert np.array_equal(obs0[k], exp), ("reset obs", k)
        refs.append(o)
    need = [False] * n_envs
    for t in range(1, steps + 1):
        if graph:  # actions generated inside the replayed step graph
            assert stream == "discrete"
            eng.step_graph(t, n_discrete)
            acts = eng.actions.cpu().numpy()
        elif stream == "discrete":
            eng.gen_actions(t, n_discrete)
            acts = eng.actions.cpu().numpy()
            eng.step()
        else:
            acts = np.stack([_rich_triples(s, t, eng.A) for s in seeds])
            eng.actions.copy_(torch.from_numpy(acts))
            eng.step()
        torch.cuda.synchronize()
        obs = eng.obs.cpu().numpy()
        rew = eng.rewards.cpu().numpy()
        done = eng.done.cpu().numpy()
        trunc = eng.trunc.cpu().numpy()
        was_reset = eng.was_reset.cpu().numpy()
        for k, o in enumerate(refs):
            if need[k]:
                assert was_reset[k], ("expected autoreset", k, t)
                exp = o.reset()
                need[k] = False
            else:
                assert not was_reset[k], ("unexpected reset", k, t)
                exp, r, d, tr, lb = o.step(acts[k])
                assert bool(done[k]) == d and bool(trunc[k]) == tr, ("flags", k, t)
                if eng.multi:
                    assert np.array_equal(rew[k][lb], r[:eng.A][lb]), ("rew", k, t, rew[k], r)
                else:
                    assert rew[k][0] == r[0], ("rew", k, t, rew[k][0], r[0])
                need[k] = d or tr
            assert np.array_equal(obs[k], exp), ("obs", k, t)
            if check_state_every and t % check_state_every == 0:
                assert eng.get_state(k).canonical(kinds) == o.state(), ("state", k, t)
    eng.close()


def c2(n):
    return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                 minimum_zombies=0, max_episode_steps=1000)


def test_c2_bridge64_multi_discrete():
    run_parity(c2, 192, 160)


def test_single_bridge_world_simple():
    run_parity(lambda n: _abi.single_env_config(n, "extermination", [], "bridge", 0, initial_zombies=10,
                                                observation_scope="world", observation_position_encoding="simple",
                                                max_episode_steps=1000),
               128, 120, n_discrete=6)


def test_city128_safehouse_respawn():
    run_parity(lambda n: _abi.multi_env_config(n, "safehouse", [], "city128", ["0", "1", "2", "3"],
                                               initial_zombies=50, minimum_zombies=50),
               48, 60)


def test_city_for_safehouse_long_shuffles():
    run_parity(lambda n: _abi.multi_env_config(n, "safehouse", [], "city_for_safehouse", ["0", "1", "2", "3"],
                                               initial_zombies=50, minimum_zombies=50),
               32, 40)


def test_bots_rules_rich_actions():
    run_parity(lambda n: _abi.single_env_config(n, "evacuation", ["terminator", "randoman", "hamster", "troll"],
                                                "easy_exit", "0", initial_zombies=8, minimum_zombies=6,
                                                observation_scope="surroundings:9",
                                                observation_position_encoding="channels", agent_weapon="random",
                                                max_episode_steps=80),
               96, 150, stream="rich")


def test_multi_bots_survival_rich_int16():
    run_parity(lambda n: _abi.multi_env_config(n, "survival", ["sniper", "randoman"], "fort",
                                               ["0", "1", "2"], initial_zombies=30, minimum_zombies=20,
                                               agent_weapons=["random", "gun"], observation_surroundings_width=11,
                                               obs_dtype=_abi.DTYPE_I16, max_episode_steps=70),
               64, 140, stream="rich")


# Alternative kernel paths the engine picks by map / size (or that the config's launch overrides force,
# zs_launch: 1 = on, -1 = off): each must be bit-exact too.
PATHS = {
    "unfused": {"fused": -1},                  # separate k_reset launch
    "fused": {"fused": 1},                    # reset work inside the step launch
    "obs_in_step": {"fobs": 1},               # observations written by the step / reset launches
    "obs_in_step_unfused": {"fobs": 1, "fused": -1},
    "obs_k_obs": {"fobs": -1, "obs_pipe": -1, "obs_gather": -1},  # one-env-per-wave k_obs
    "obs_gather": {"fobs": -1, "obs_pipe": -1, "obs_ring": -1},  # window-only fetches (k_obs_gather)
    "obs_gather_scell": {"fobs": -1, "obs_pipe": -1, "obs_ring": -1, "obs_gather_stat": -1},  # ... global static words
    "obs_pbring": {"fobs": -1, "obs_pipe": -1},  # window-only encoders + writer waves (k_obs_pbring)
    "obs_pipe_cells": {"obs_lds": -1},          # k_obs_pipe's per-cell stores instead of the staged flush
    "obs_lds": {"obs_lds": 1},                 # the LDS-staged store kernels at any env count
    "obs_lds_select": {"obs_lds": 1, "obs_patch": -1},  # ... without the padded-table encoder
    "obs_ring": {"obs_lds": 1, "obs_ring": 1},  # encoder / writer waves through an LDS ring
    "obs_ring_select": {"obs_lds": 1, "obs_ring": 1, "obs_ring_patch": -1},  # ... select-chain encoders
    "obs_scan": {"obs_win": -1},                # per-cell entity scan instead of the window map
    "obs_scan_in_step": {"obs_win": -1, "fobs": 1},
    "obs_scell": {"obs_stat": -1},              # per-cell static words instead of LDS bitmaps
    "obs_scell_in_step": {"obs_stat": -1, "fobs": 1},
    "no_lds_budget": {"lds_budget": -1},        # largest LDS copies instead of occupancy-first
    "serial_exec": {"par_exec": -1},               # the leader's serial shuffle + execution (core.py:76,103-119)
}


@pytest.mark.parametrize("path", sorted(PATHS))
def test_kernel_paths(path):
    run_parity(c2, 96, 60, check_state_every=30, launch=PATHS[path])
    run_parity(lambda n: _abi.single_env_config(n, "safehouse", ["terminator"], "city_for_safehouse", "0",
                                                initial_zombies=20, minimum_zombies=20,
                                                observation_scope="world", observation_position_encoding="channels",
                                                max_episode_steps=50),
               16, 60, check_state_every=30, launch=PATHS[path])


# Zombie respawn in the tick's leader or deferred to k_respawn (wave per env): both bit-exact, on a
# long candidate list (city128, 439 spawns), on every-cell candidates (city_for_safehouse) and on a
# short list under Extermination, where a respawn decides whether the game ends (boxed: 1 zombie,
# minimum 1), and on a map without obstacles.
RESPAWN = {
    "leader": {"defer_respawn": -1},
    "deferred": {"defer_respawn": 1},
    "deferred_fused": {"defer_respawn": 1, "fused": 1},
    "deferred_unfused_serial_reset": {"defer_respawn": 1, "fused": -1, "reset_stream": -1},
    "deferred_unfused_side_reset": {"defer_respawn": 1, "fused": -1},
}


@pytest.mark.parametrize("path", sorted(RESPAWN))
def test_respawn_paths(path):
    lo = RESPAWN[path]
    run_parity(lambda n: _abi.single_env_config(n, "extermination", ["terminator"], "boxed", "0",
                                                initial_zombies=1, minimum_zombies=1,
                                                observation_scope="world", observation_position_encoding="channels",
                                                agent_weapon="shotgun", max_episode_steps=60),
               64, 100, stream="rich", check_state_every=20, launch=lo)
    run_parity(lambda n: _abi.multi_env_config(n, "safehouse", [], "city128", ["0", "1", "2", "3"],
                                               initial_zombies=50, minimum_zombies=50),
               24, 40, check_state_every=20, launch=lo)
    run_parity(lambda n: _abi.multi_env_config(n, "extermination", [], "city_for_safehouse", ["0", "1"],
                                               initial_zombies=3, minimum_zombies=2, max_episode_steps=40),
               32, 60, stream="rich", check_state_every=20, launch=lo)
    # a map without obstacles (easy_exit: no obstacle-present words to stage)
    run_parity(lambda n: _abi.single_env_config(n, "evacuation", ["terminator"], "easy_exit", "0",
                                                initial_zombies=8, minimum_zombies=6, max_episode_steps=60),
               32, 60, stream="rich", check_state_every=20, launch=lo)


# The bench loop as a replayed hipGraph (zs_step_graph): same trajectories, for both pending-list
# parities and every launch layout the graph may capture (fused step launch, separate reset launch on
# the side stream, deferred respawn).
GRAPH = {
    "default": {},
    "unfused_side_stream": {"fused": -1},
    "unfused_serial": {"fused": -1, "reset_stream": -1},
}


@pytest.mark.parametrize("path", sorted(GRAPH))
def test_step_graph(path):
    run_parity(c2, 128, 80, check_state_every=40, graph=True, launch=GRAPH[path])
    run_parity(lambda n: _abi.multi_env_config(n, "safehouse", [], "city128", ["0", "1", "2", "3"],
                                               initial_zombies=50, minimum_zombies=50),
               16, 30, check_state_every=15, graph=True, launch=GRAPH[path])


@pytest.mark.parametrize("kernel", ["patch", "ring_select"])
def test_store_stream_every_phase(kernel):
    """k_obs_patch and k_obs_ring (here with its select-chain encoders) write each observation block from an
    LDS slot kept at the destination's 16-B phase: int16 blocks of 4 agents (2646 B: every even phase), int32
    single-agent blocks (5292 B)."""
    lo = {"patch": {"obs_lds": 1, "obs_patch": 1, "obs_ring": -1},
          "ring_select": {"obs_lds": 1, "obs_ring": 1, "obs_ring_patch": -1}}[kernel]
    run_parity(lambda n: _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1", "2", "3"],
                                               initial_zombies=20, obs_dtype=_abi.DTYPE_I16, max_episode_steps=200),
               64, 60, check_state_every=30, launch=lo)
    run_parity(lambda n: _abi.single_env_config(n, "extermination", [], "bridge64", 0, initial_zombies=10,
                                                observation_scope="surroundings:21",
                                                observation_position_encoding="channels", max_episode_steps=200),
               64, 60, n_discrete=6, check_state_every=30, launch=lo)


CITY128_OBS = {"pbring": {}, "gather": {"obs_ring": -1},
               "gather_scell": {"obs_ring": -1, "obs_gather_stat": -1}}


@pytest.mark.parametrize("path", sorted(CITY128_OBS))
def test_city128_obs_paths(path):
    """C4's observation kernels: k_obs_pbring (default: window-only encoders, the things written over the
    windows, writer waves), k_obs_gather with static words from the LDS tables or one global load per window
    cell."""
    run_parity(lambda n: _abi.multi_env_config(n, "safehouse", [], "city128", ["0", "1", "2", "3"],
                                               initial_zombies=50, minimum_zombies=50),
               24, 30, check_state_every=15, launch=CITY128_OBS[path])


@pytest.mark.parametrize("lanes", [4, 8, 16, 32, 64])
def test_lanes_per_env(lanes):
    """k_tick / k_step at every lanes-per-env count: the lanes' parallel execution in chunks of G actions
    (chunks of 4 and 8 on 12-actor envs; more lanes than actions), and the leader's serial loop where an
    action list exceeds 2G (G = 4); rich actions on a multi-bot map exercise heals, obstacle hits and
    the deferred (RNG-drawing) decisions that keep the serial path."""
    run_parity(c2, 64, 60, check_state_every=30, launch=None, lanes=lanes)
    run_parity(lambda n: _abi.multi_env_config(n, "survival", ["sniper", "terminator", "troll"], "fort",
                                               ["0", "1", "2"], initial_zombies=12, minimum_zombies=8,
                                               agent_weapons=["shotgun", "gun", "axe"], max_episode_steps=60,
                                               lanes_per_env=lanes),
               48, 80, stream="rich", check_state_every=40)


def test_rng_window_reload():
    """A 32-word RNG window on 54-actor envs (median 82 draws per step): the tick runs its window dry and
    reloads it from the ring several times per step (core.py:76 shuffle, :168-202 attack / heal draws),
    by the env's lanes or its leader, bit-exact."""
    run_parity(lambda n: _abi.multi_env_config(n, "safehouse", [], "city128", ["0", "1", "2", "3"],
                                               initial_zombies=50, minimum_zombies=50),
               24, 30, check_state_every=15, launch={"rw_need": 32})
    run_parity(c2, 128, 60, check_state_every=30, graph=True, launch={"rw_need": 32})
    # 24 actors (C5's shape) on a 32-word window: the lanes' shuffle and damage draws run the window dry
    # and reload it themselves (grp_reload) mid-shuffle and mid-chunk
    run_parity(lambda n: _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1", "2", "3"],
                                               initial_zombies=20, obs_dtype=_abi.DTYPE_I16, max_episode_steps=200),
               64, 80, check_state_every=40, launch={"rw_need": 32})


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("fused", [-1, 1])
def test_masked_reset_of_pending_envs(fused, graph):
    """Next-step autoreset, reset work on the side stream (unfused) or inside the step launch: between
    calls a pending env still shows its terminal world (state records against the oracle's, which resets
    only at the next call); a masked zs_reset of pending and running envs alike resets each once (the
    oracle's env.reset() draws) and takes the pending ones off the list, and the unmasked pending envs
    still autoreset at the next step."""
    import torch
    from libzombsole_amd.engine import Engine
    from oracle.oracle import OracleEnv

    def b(n):
        return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                     minimum_zombies=0, max_episode_steps=6)
    n, steps = 256, 30
    eng = Engine(b(n).set_launch({"fused": fused}))
    assert eng.describe()["reset_side_stream"] == (fused < 0)
    kinds = [o[2] for o in eng.builder.map.obstacles]
    eng.seed([700 + i for i in range(n)])
    eng.reset()
    refs = []
    for k in range(n):
        o = OracleEnv(b(1))
        o.seed(700 + k)
        o.reset()
        refs.append(o)
    need = [False] * n
    masked_pending = 0
    for t in range(1, steps + 1):
        if t in (7, 9, 20):  # masked reset of every other env, pending ones included
            mask = (torch.arange(n, device=eng.device) % 2 == 0).to(torch.uint8)
            obs = eng.reset(mask).cpu().numpy()
            for k in range(0, n, 2):
                assert np.array_equal(obs[k], refs[k].reset()), ("masked reset obs", k, t)
                masked_pending += need[k]
                need[k] = False
        if graph:  # replayed step graphs between masked resets (the reset flips the list parity)
            eng.step_graph(t, 7)
        else:
            eng.gen_actions(t, 7)
            eng.step()
        acts = eng.actions.cpu().numpy()
        torch.cuda.synchronize()
        obs = eng.obs.cpu().numpy()
        rew = eng.rewards.cpu().numpy()
        was_reset = eng.was_reset.cpu().numpy()
        for k, o in enumerate(refs):
            if need[k]:
                assert was_reset[k], (k, t)
                exp = o.reset()
                need[k] = False
            else:
                assert not was_reset[k], (k, t)
                exp, r, d, tr, lb = o.step(acts[k])
                assert np.array_equal(rew[k][lb], r[:2][lb]), ("rew", k, t)
                need[k] = d or tr
            assert np.array_equal(obs[k], exp), ("obs", k, t)
        for k in range(0, n, 17):  # pending envs included: the terminal world until the next call
            assert eng.get_state(k).canonical(kinds) == refs[k].state(), ("state", k, t)
    assert masked_pending > 0  # the masked resets met envs whose autoreset was pending
    eng.close()
