"""Coverage of the lanes' chunked execution (zs_tick.hpp grp_execute) by the parity runs.

The engine's G lanes of an env execute its shuffled action list (core.py:103-119) in chunks of G
consecutive actions and resolve, by ballots inside a chunk, the cases where an action depends on an
earlier one of the same chunk.  The oracle counts those cases while it executes the list serially
(zs_oracle.c census_*, oracle.run_hashes(chunk_g=G) / OracleEnv.set_census):

  enter_vacated  a valid move into the source cell of an earlier valid move of the chunk
  same_dest      a valid move onto the destination of an earlier valid move
  target_moved   an attack / heal whose thing target moved earlier in the chunk
  target_later   an attack / heal whose thing target has a valid move later in the chunk
  multi_hit      an in-range hit on a target an earlier action of the chunk already hit
  hit_dead       an in-range hit on a target an earlier hit of the chunk took to life <= 0
  heal_clamp     an in-range heal clamped at MAX_LIFE (core.py:186-202)
  obst_int16     a hit leaving an obstacle's life below -32768 (a12: lives carried over resets)

CPU: the bench workloads (C2/C3 at G = 8, C5 at 16, C4 at 32) reach every case but obst_int16 on the
lanes' path alone; the melee workload below (obstacle lives poked near the int16 floor, fixed agent
actions on a crowded 12 x 6 map, one chunk per list at G = 32) reaches all eight and chunks holding six at
once.  GPU: that melee workload through zs_set_state pokes, every step against the oracle.
"""
import numpy as np
import pytest

from libzombsole_amd import _abi
from libzombsole_amd import actions as A
from libzombsole_amd.maps import Map

MELEE_MAP = ("wwwwwwwwwwww\n"
             "w..pppp....w\n"
             "w.zzzzzzzz.w\n"
             "w.zzzzzzzz.w\n"
             "w..........w\n"
             "wwwwwwwwwwww\n")
# agent 0 shoots the (poked) border wall above it, agents 1 and 2 walk right along the spawn row (each
# may enter the cell the other one leaves), agent 3 heals itself at full life (clamped)
MELEE_ACTIONS = np.array([[A.ACT_ATTACK, 0, -1], [A.ACT_MOVE, 1, 0], [A.ACT_MOVE, 1, 0], [A.ACT_HEAL, 0, 0]],
                         dtype=np.int32)
MELEE_LIFE = -32760
CASES = ("enter_vacated", "same_dest", "target_moved", "target_later", "multi_hit", "hit_dead", "heal_clamp",
         "obst_int16")


def melee(n, lanes=32, max_steps=2):
    return _abi.multi_env_config(n, "survival", [], Map.from_text(MELEE_MAP, name="melee"), ["0", "1", "2", "3"],
                                 initial_zombies=14, minimum_zombies=14, max_episode_steps=max_steps,
                                 lanes_per_env=lanes)


def bench_builder(cfg):
    if cfg == "c4":
        return _abi.multi_env_config(1, "safehouse", [], "city128", ["0", "1", "2", "3"], initial_zombies=50,
                                     minimum_zombies=50, max_episode_steps=1000)
    if cfg == "c5":
        return _abi.multi_env_config(1, "extermination", [], "bridge64", ["0", "1", "2", "3"], initial_zombies=20,
                                     max_episode_steps=1000, obs_dtype=_abi.DTYPE_I16)
    return _abi.multi_env_config(1, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                 max_episode_steps=1000)


@pytest.mark.parametrize("cfg,G", [("c3", 8), ("c3", 16), ("c5", 16), ("c4", 32)])
def test_bench_workloads_reach_every_lane_case(cfg, G):
    """The random-policy workloads the full-size parity tests compare (tests/test_fullsize_parity.py):
    every list on the lanes' path, every case but obst_int16 (no obstacle is poked there) occurring."""
    from oracle.oracle import run_hashes
    _, c = run_hashes(bench_builder(cfg), 0, 256, 60, 7, chunk_g=G)
    assert c["lists_serial"] == 0 and c["lists"] > 0, c
    for k in CASES:
        if k != "obst_int16":
            assert c[k] > 0, (k, c)
    assert c["obst_int16"] == 0


def melee_oracles(n, seed0=0, lanes=32):
    from oracle.oracle import OracleEnv
    m = Map.from_text(MELEE_MAP, name="melee")
    out = []
    for i in range(n):
        o = OracleEnv(melee(1, lanes))
        for k in range(len(m.obstacles)):
            o.poke_obstacle(k, MELEE_LIFE)
        o.seed(seed0 + i)
        o.reset()
        o.set_census(lanes)
        out.append(o)
    return out


def census_sum(oracles):
    tot = {}
    for o in oracles:
        for k, v in o.census().items():
            tot[k] = max(tot.get(k, 0), v) if k == "max_in_chunk" else tot.get(k, 0) + v
    return tot


def test_melee_reaches_every_case_in_one_chunk():
    orc = melee_oracles(64)
    need = [False] * len(orc)
    for _ in range(12):
        for i, o in enumerate(orc):
            if need[i]:
                o.reset()
                need[i] = False
            else:
                _, _, d, tr, _ = o.step(MELEE_ACTIONS)
                need[i] = d or tr
    c = census_sum(orc)
    assert c["lists_serial"] == 0
    for k in CASES:
        if k != "hit_dead":
            assert c[k] > 0, (k, c)
    assert c["chunks_all6"] > 0, c


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [32, 16])
def test_engine_melee_poked_against_oracle(lanes):
    """256 melee envs, border walls poked to -32 760 through zs_set_state (the reference's map objects
    carry their life over resets), TimeLimit 2 so every other step is an episode's first tick with those
    walls still standing: 24 steps, every env's observations, listed rewards and flags against the oracle
    each step, the full state of every env at the end, and the oracle's census of the same run showing
    every case (at G = 32 all in one chunk, at G = 16 across two chunks)."""
    import torch

    from libzombsole_amd.engine import Engine

    n, steps = 256, 24
    eng = Engine(melee(n, lanes))
    desc = eng.describe()
    assert desc["lanes_per_env"] == lanes and desc["par_exec"] == 1, desc
    kinds = [o[2] for o in eng.builder.map.obstacles]
    eng.seed(list(range(n)))
    for k in range(n):
        st = eng.get_state(k)
        st.obst_life[:] = MELEE_LIFE
        eng.set_state(k, st)
    obs = eng.reset().cpu().numpy()
    orc = melee_oracles(n, 0, lanes)
    for k, o in enumerate(orc):
        assert np.array_equal(obs[k], o.obs()), ("reset obs", k)
    eng.actions.copy_(torch.from_numpy(np.broadcast_to(MELEE_ACTIONS, (n, 4, 3)).copy()))
    need = [False] * n
    for t in range(1, steps + 1):
        eng.step()
        torch.cuda.synchronize()
        obs, rew = eng.obs.cpu().numpy(), eng.rewards.cpu().numpy()
        done, trunc, was_reset = eng.done.cpu().numpy(), eng.trunc.cpu().numpy(), eng.was_reset.cpu().numpy()
        for k, o in enumerate(orc):
            if need[k]:
                assert was_reset[k], (k, t)
                exp = o.reset()
                need[k] = False
            else:
                exp, r, d, tr, lb = o.step(MELEE_ACTIONS)
                assert bool(done[k]) == d and bool(trunc[k]) == tr, (k, t)
                for a in range(4):
                    if lb[a]:
                        assert rew[k, a].hex() == r[a].hex(), (k, t, a)
                need[k] = d or tr
            assert np.array_equal(obs[k], exp), ("obs", k, t)
    for k, o in enumerate(orc):
        assert eng.get_state(k).canonical(kinds) == o.state(), ("state", k)
    c = census_sum(orc)
    for k in CASES:
        if k != "hit_dead":
            assert c[k] > 0, (k, c)
    if lanes == 32:
        assert c["chunks_all6"] > 0, c
    assert eng.overflow() & _abi.OVF_INT16
    eng.close()
