"""Obstacle life carried over resets without a floor.

The reference's Box/Wall objects belong to the map and are re-spawned at every reset with the life
they had (game.py:151-155); a destroyed one is back in the world until the first cleanup of the
episode (core.py:72-78) and can be hit again on tick 1 (core.py:168-184), so its life falls across
episodes with no lower bound (a Python int).  The engine holds it in int32 (exact down to
-2**31 + 1, then saturating with ZS_OVF_INT32), and its int16 observation form saturates a life
below -32768 (ZS_OVF_INT16).  The reference fixture `multi_wallhp_carryover_a2` (make_golden.py)
pins the same map and actions through test_engine_golden / test_dropin_golden / test_oracle_golden.
"""
import numpy as np
import pytest

from libzombsole_amd import _abi
from libzombsole_amd import actions as A
from libzombsole_amd.maps import Map

WALL_HP_MAP = "wwwww\nwpwpw\nw...w\nwwwww\n"
# agent 0 shoots one cell right, agent 1 one cell left: both hit the centre wall (obstacle 6) when the
# spawn shuffle puts them either side of it, else each hits a border wall (obstacles 5 and 7)
FIXED = np.array([[A.ACT_ATTACK, 1, 0], [A.ACT_ATTACK, -1, 0]], dtype=np.int32)


def _builder(n, dtype=_abi.DTYPE_I64, agents=("0", "1")):
    return _abi.multi_env_config(n, "extermination", [], Map.from_text(WALL_HP_MAP, name="wall_hp"), list(agents),
                                 initial_zombies=0, minimum_zombies=0, obs_dtype=dtype)


def test_fixed_action_is_attack():
    assert tuple(A.encode_action({"action_type": "attack", "parameter": [1, 0]})) == tuple(FIXED[0])
    assert tuple(A.encode_action({"action_type": "attack", "parameter": [-1, 0]})) == tuple(FIXED[1])


def test_oracle_life_falls_across_resets():
    """CPU: the oracle alone, the int16 floor crossed within a few episodes."""
    from oracle.oracle import OracleEnv
    o = OracleEnv(_builder(1))
    for i, life in ((5, -32700), (6, -32720), (7, -32760)):
        assert o.poke_obstacle(i, life) == 0
    o.seed(3)
    o.reset()
    lows = []
    for _ in range(20):
        _, _, done, _, _ = o.step(FIXED)
        assert done  # no zombies: Extermination ends every episode at its first step
        lows.append(min(r[1] for r in o.state()["obst"]))
        o.reset()
    assert lows[-1] < -32768 - 500 and all(b <= a for a, b in zip(lows, lows[1:]))


def _poke_all(eng, pokes):
    for k in range(eng.N):
        st = eng.get_state(k)
        for i, life in pokes:
            st.obst_life[i] = life
        eng.set_state(k, st)


# observation kernels: the engine's pick for the size (int16: k_obs_ring, int32: k_obs_patch), the
# store streams forced at 64 envs (int64 too: k_obs_patch, k_obs_ring), and k_obs_pipe's per-cell stores
OBS_PATHS = {"default": {}, "patch": {"obs_lds": 1, "obs_ring": -1},
             "ring": {"obs_lds": 1, "obs_ring": 1},
             "pipe_cells": {"obs_lds": -1}}


@pytest.mark.gpu
@pytest.mark.parametrize("path", sorted(OBS_PATHS))
@pytest.mark.parametrize("dtype", [_abi.DTYPE_I64, _abi.DTYPE_I32, _abi.DTYPE_I16])
def test_engine_matches_oracle_across_resets(dtype, path):
    """64 envs x 160 calls (80 episodes), every call's obs / rewards / flags and the obstacle state
    against the oracle; int16 observations saturate like the oracle's int16 form and raise
    ZS_OVF_INT16, never ZS_OVF_INT32.  The 5 x 4 map puts most of every 21 x 21 window out of bounds,
    and the walls the agents shoot are damaged, destroyed and re-spawned at negative life."""
    import torch
    from libzombsole_amd.engine import Engine
    from oracle.oracle import OracleEnv
    n, calls = 64, 160
    pokes = [(5, -32700), (6, -32720), (7, -32760)]
    eng = Engine(_builder(n, dtype).set_launch(OBS_PATHS[path]))
    kinds = [o[2] for o in eng.builder.map.obstacles]
    seeds = [500 + i for i in range(n)]
    eng.seed(seeds)
    _poke_all(eng, pokes)
    obs = eng.reset().cpu().numpy()
    refs = []
    for k, s in enumerate(seeds):
        o = OracleEnv(_builder(1, dtype))
        for i, life in pokes:
            o.poke_obstacle(i, life)
        o.seed(s)
        assert np.array_equal(obs[k], o.reset()), ("reset obs", k)
        refs.append(o)
    need = [False] * n
    acts = np.broadcast_to(FIXED, (n, 2, 3)).copy()
    eng.actions.copy_(torch.from_numpy(acts))
    for t in range(1, calls):
        eng.step()
        torch.cuda.synchronize()
        obs = eng.obs.cpu().numpy()
        rew = eng.rewards.cpu().numpy()
        done = eng.done.cpu().numpy()
        was_reset = eng.was_reset.cpu().numpy()
        for k, o in enumerate(refs):
            if need[k]:
                assert was_reset[k], (k, t)
                exp = o.reset()
                need[k] = False
            else:
                exp, r, d, tr, lb = o.step(FIXED)
                assert bool(done[k]) == d, (k, t)
                assert np.array_equal(rew[k][lb], r[:2][lb]), (k, t)
                need[k] = d or tr
            assert np.array_equal(obs[k], exp), ("obs", k, t)
            if t % 40 == 0 or t == calls - 1:
                assert eng.get_state(k).canonical(kinds) == o.state(), ("state", k, t)
    lows = [min(r[1] for r in o.state()["obst"]) for o in refs]
    assert max(lows) < -32768 - 1000  # every env crossed the int16 floor long ago
    flags = eng.overflow()
    assert flags == _abi.OVF_INT16, flags
    if dtype == _abi.DTYPE_I16:
        with pytest.raises(OverflowError):
            eng.check_lossless()
    else:
        eng.check_lossless()
    eng.close()


@pytest.mark.gpu
def test_int32_floor_saturates_and_flags():
    """A life poked just above -2**31 + 1: the next hits saturate it there (no wrap to a positive
    life that would bring the wall back) and raise ZS_OVF_INT32; INT32_MIN itself is refused."""
    import torch
    from libzombsole_amd.engine import Engine, EngineError
    eng = Engine(_builder(8))
    eng.seed(list(range(8)))
    _poke_all(eng, [(5, -2147483630), (6, -2147483630), (7, -2147483630)])  # any hit (>= 25) passes the floor
    eng.reset()
    assert eng.overflow(clear=True) == _abi.OVF_INT16  # the poke itself left the int16 range
    eng.actions.copy_(torch.from_numpy(np.broadcast_to(FIXED, (8, 2, 3)).copy()))
    for _ in range(12):
        eng.step()
    torch.cuda.synchronize()
    assert eng.overflow() == _abi.OVF_INT16 | _abi.OVF_INT32
    for k in range(8):
        st = eng.get_state(k)
        hit = [int(st.obst_life[i]) for i in (5, 6, 7) if int(st.obst_life[i]) != -2147483630]
        assert hit and all(v == -2147483647 for v in hit), (k, list(st.obst_life[5:8]))
    with pytest.raises(OverflowError):
        eng.check_lossless()
    st = eng.get_state(0)
    st.obst_life[6] = -2147483648
    with pytest.raises((ValueError, EngineError)):
        eng.set_state(0, st)
    eng.close()


@pytest.mark.gpu
def test_set_state_refuses_pending_flag_change():
    """zs_set_state does not move an env on or off the engine's pending-reset lists: a record whose
    needs_reset word differs from the engine's is refused and nothing is written."""
    import torch
    from libzombsole_amd.engine import Engine, EngineError
    eng = Engine(_builder(4))
    eng.seed([1, 2, 3, 4])
    eng.reset()
    eng.actions.copy_(torch.from_numpy(np.broadcast_to(FIXED, (4, 2, 3)).copy()))
    eng.step()  # every episode ends: all four envs are pending reset now
    st = eng.get_state(2)
    assert int(st.buf[5]) in (1, 2)  # pending: rebuilt by the next call, or already into its shadow record
    before = st.buf.copy()
    st.buf[5] = 0
    st.buf[0] = 777
    with pytest.raises((ValueError, EngineError)):
        eng.set_state(2, st)
    assert np.array_equal(eng.get_state(2).buf, before)
    eng.set_state(2, eng.get_state(2))  # the engine's own record round-trips
    # a present thing placed outside the map is refused (the kernels index the map by its cell)
    st = eng.get_state(1)
    before = st.buf.copy()
    s0 = int(np.nonzero(st.ent[:, 1])[0][0])
    for x, y in ((-1, 0), (0, -1), (st.W, 0), (0, st.H)):
        st.ent[s0, 2], st.ent[s0, 3] = x, y
        with pytest.raises(ValueError):
            eng.set_state(1, st)
    assert np.array_equal(eng.get_state(1).buf, before)
    eng.close()


@pytest.mark.gpu
def test_raise_kind_only_in_debug_envs():
    """Action kind 7 (ZS_ACT_RAISE) stops World.step only with ZS_FLAG_DEBUG; in other envs it is
    an unknown kind and the agent idles — engine and oracle alike."""
    import torch
    from libzombsole_amd.engine import Engine
    from oracle.oracle import OracleEnv

    def b(n, debug):
        return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                     minimum_zombies=0, debug=debug)
    acts = np.array([[A.ACT_RAISE, 0, 0], [A.ACT_MOVE, 0, 1]], dtype=np.int32)
    for debug in (False, True):
        eng = Engine(b(16, debug))
        eng.seed(list(range(16)))
        obs0 = eng.reset().cpu().numpy()
        eng.actions.copy_(torch.from_numpy(np.broadcast_to(acts, (16, 2, 3)).copy()))
        eng.step()
        torch.cuda.synchronize()
        t = [eng.get_state(k).t for k in range(16)]
        for k in range(16):
            o = OracleEnv(b(1, debug))
            o.seed(k)
            assert np.array_equal(o.reset(), obs0[k])
            if debug:
                from oracle.oracle import OracleRaised
                with pytest.raises(OracleRaised):
                    o.step(acts)
            else:
                exp, r, d, tr, lb = o.step(acts)
                assert np.array_equal(eng.obs[k].cpu().numpy(), exp)
                assert eng.get_state(k).canonical([x[2] for x in eng.builder.map.obstacles]) == o.state()
        assert all(v == 0 for v in t)  # World.t advanced once from -1 either way
        eng.close()


BIG_ENCODERS = {"k_obs_pbring": {}, "k_obs_gather": {"obs_ring": -1}}


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", sorted(BIG_ENCODERS))
@pytest.mark.parametrize("dtype", [_abi.DTYPE_I64, _abi.DTYPE_I16])
def test_big_map_encoders_on_poked_states(dtype, kernel):
    """The big-map observation kernels (C4's city128: 3689 obstacles, 512 dead-body words, past the register
    prefetch of the store-stream kernels) against the oracle's encoder (gym/observation.py:57-173) on poked
    states: dead bodies in every dead-body chunk (clean chunks read the shared zero row), damaged and
    cleaned-up obstacles in several HP chunks (clean chunks read hp_init), lives below the int16 range.
    1536 envs: k_obs_pbring's 256 workgroups walk six envs each, so its ring slots are reused."""
    from libzombsole_amd.engine import Engine
    from oracle.oracle import OracleEnv
    n = 1536

    def cfg(k):
        return _abi.multi_env_config(k, "safehouse", [], "city128", ["0", "1", "2", "3"], initial_zombies=50,
                                     minimum_zombies=50, obs_dtype=dtype)

    eng = Engine(cfg(n).set_launch(BIG_ENCODERS[kernel]))
    assert eng.describe()["obs_kernel"] == kernel
    eng.seed([1300 + i for i in range(n)])
    eng.reset()
    rng = np.random.default_rng(12)
    st0 = eng.get_state(0)
    W, cells = st0.W, st0.W * st0.H
    refs = {}
    for e in range(n):
        if e % 3 and e % 97:  # every third env and a scattered set poked; the others as reset
            continue
        o = OracleEnv(cfg(1))
        o.seed(1300 + e)
        o.reset()
        st = eng.get_state(e)
        dw = st.dead_words.view(np.uint32)
        for c in rng.choice(cells, size=(0, 30, 400, 3000)[e % 4], replace=False):
            dw[int(c) >> 5] |= np.uint32(1 << (int(c) & 31))
            o.poke_dead(int(c) % W, int(c) // W)
        for i in rng.choice(st.O, size=(0, 5, 40, 200)[(e // 3) % 4], replace=False):
            st.obst_life[i] = int(rng.integers(-40000, 199))
            o.poke_obstacle(int(i), int(st.obst_life[i]))
            if st.obst_life[i] <= 0 and rng.integers(2):
                st.obst_present[i] = 0
                o.poke_obstacle_gone(int(i))
        eng.set_state(e, st)
        refs[e] = o
    got = eng.observe().cpu().numpy()
    for e, o in refs.items():
        assert np.array_equal(got[e], o.obs()), ("obs", kernel, e)
    # envs left as reset: the reset observation of the same seed
    for e in (1, 2, 4, 1535):
        if e in refs:
            continue
        o = OracleEnv(cfg(1))
        o.seed(1300 + e)
        assert np.array_equal(got[e], o.reset()), ("reset obs", kernel, e)
    eng.close()


# name -> (launch overrides, the kernel they select)
ENCODERS = {"k_obs_patch": ({"obs_lds": 1, "obs_ring": -1, "obs_patch": 1}, "k_obs_patch"),
            "k_obs_pipe": ({"obs_lds": -1}, "k_obs_pipe"),
            "k_obs_ring": ({"obs_lds": 1, "obs_ring": 1}, "k_obs_ring"),
            "k_obs_ring_select": ({"obs_lds": 1, "obs_ring": 1, "obs_ring_patch": -1}, "k_obs_ring")}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,kernel", [(_abi.DTYPE_I16, k) for k in sorted(ENCODERS)] +
                         [(_abi.DTYPE_I64, "k_obs_pipe"), (_abi.DTYPE_I64, "k_obs_patch")])
def test_observation_encoders_on_poked_states(dtype, kernel):
    """The store-stream observation kernels (the padded-table encoder of k_obs_patch and k_obs_ring, the
    per-cell select chains of k_obs_pipe and of k_obs_ring's fallback encoders) against the oracle's encoder
    (gym/observation.py:57-173) on the
    same poked states of bridge64 with 4 agents: 40 to 900 dead-body cells per env (more than
    PATCH_DEAD_CAP = 256 cells takes the per-word scan), bodies under map obstacles and under things,
    damaged and cleaned-up obstacles, lives below the int16 range (int16 saturates in both).  (k_obs_ring's
    LDS ring does not fit four int64 blocks: the engine does not pick it there.)"""
    from libzombsole_amd.engine import Engine
    from oracle.oracle import OracleEnv
    n = 64

    def cfg(k):
        return _abi.multi_env_config(k, "extermination", [], "bridge64", ["0", "1", "2", "3"], initial_zombies=20,
                                     obs_dtype=dtype)

    eng = Engine(cfg(n).set_launch(ENCODERS[kernel][0]))
    assert eng.describe()["obs_kernel"] == ENCODERS[kernel][1]
    eng.seed([900 + i for i in range(n)])
    eng.reset()
    rng = np.random.default_rng(11)
    W = eng.get_state(0).W
    cells = W * eng.get_state(0).H
    refs = []
    for e in range(n):
        o = OracleEnv(cfg(1))
        o.seed(900 + e)
        o.reset()
        st = eng.get_state(e)
        dw = st.dead_words.view(np.uint32)  # writes through to the record
        for c in rng.choice(cells, size=(40, 200, 300, 900)[e % 4], replace=False):
            dw[int(c) >> 5] |= np.uint32(1 << (int(c) & 31))
            o.poke_dead(int(c) % W, int(c) // W)
        for i in rng.choice(st.O, size=12, replace=False):
            st.obst_life[i] = int(rng.integers(-40000, 199))
            o.poke_obstacle(int(i), int(st.obst_life[i]))
            if st.obst_life[i] <= 0 and rng.integers(2):
                st.obst_present[i] = 0
                o.poke_obstacle_gone(int(i))
        eng.set_state(e, st)
        refs.append(o)
    got = eng.observe().cpu().numpy()
    for e, o in enumerate(refs):
        assert np.array_equal(got[e], o.obs()), ("obs", kernel, e)
    eng.close()
