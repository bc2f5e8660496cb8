"""Shared helpers for replaying golden fixtures (tests/golden/*.json.gz).

A fixture holds, per seed, the reference's outputs for a sequence of calls
(reset / step) under the next-step autoreset protocol of make_golden.py.
`replay_*` functions drive a backend through the same calls and yield, per
call, what it produced in the fixture's canonical form so tests can compare
field by field.
"""
import glob
import gzip
import hashlib
import json
import os

import numpy as np

from libzombsole_amd import _abi
from libzombsole_amd import actions as A

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_names():
    return sorted(os.path.basename(p)[:-len(".json.gz")] for p in glob.glob(os.path.join(GOLDEN, "*.json.gz"))
                  if not os.path.basename(p).startswith("stdio_"))  # stdio transcripts: test_stdio_json.py


def load_fixture(name):
    with gzip.open(os.path.join(GOLDEN, name + ".json.gz"), "rt", encoding="utf-8") as f:
        return json.load(f)


def map_path(name):
    """A fixture's map: the test-only maps of tests/golden/maps by path, else a bundled map name."""
    p = os.path.join(GOLDEN, "maps", name + ".txt")
    return p if os.path.isfile(p) else name


def obstacle_pokes(fx):
    """[[obstacle index, life], ...] set on the map's Box/Wall objects before the first reset."""
    return (fx.get("extras") or {}).get("poke_obstacles", [])


def builder_for(fx, num_envs=1, dtype=None):
    kw = dict(fx["kwargs"])
    ms = fx.get("max_steps", 0)
    debug = bool(kw.get("debug", False))
    if fx["surface"] == "single":
        return _abi.single_env_config(
            num_envs, kw["rules_name"], kw.get("player_names", []), map_path(kw["map_name"]), kw["agent_id"],
            initial_zombies=kw.get("initial_zombies", 0), minimum_zombies=kw.get("minimum_zombies", 0),
            observation_scope=kw.get("observation_scope", "world"),
            observation_position_encoding=kw.get("observation_position_encoding", "simple"),
            agent_weapon=kw.get("agent_weapon", "rifle"), max_episode_steps=ms,
            obs_dtype=_abi.DTYPE_I32 if dtype is None else dtype, debug=debug)
    return _abi.multi_env_config(
        num_envs, kw["rules_name"], kw.get("player_names", []), map_path(kw["map_name"]), kw["agent_ids"],
        initial_zombies=kw.get("initial_zombies", 0), minimum_zombies=kw.get("minimum_zombies", 0),
        observation_surroundings_width=kw.get("observation_surroundings_width", 21),
        observation_position_encoding_style=kw.get("observation_position_encoding_style", "channels"),
        agent_weapons=kw.get("agent_weapons", "rifle"), max_episode_steps=ms,
        obs_dtype=_abi.DTYPE_I64 if dtype is None else dtype, debug=debug)


def action_triples(fx, rec, n_agents):
    """Engine triples for one recorded step."""
    if fx["surface"] == "single":
        acts = [rec["act"]]
    else:
        acts = rec["act"]
    out = np.zeros((max(n_agents, 1), 3), dtype=np.int32)
    debug = bool(fx["kwargs"].get("debug", False))
    for i, a in enumerate(acts[:n_agents]):
        if fx["stream"] == "discrete":
            out[i] = A.DISCRETE_TRIPLES[int(a)]
        else:
            try:
                out[i] = A.encode_action(a)
            except A.ActionError:  # next_step raises: World.step re-raises (debug) or the agent idles
                out[i] = (A.ACT_RAISE, 0, 0) if debug else (A.ACT_IDLE, 0, 0)
    return out


def obs_sha(fx, obs, listed=None):
    """sha256 of the reference's obs bytes: single int32 [C,H,W]; multi: int64 per listed agent."""
    if fx["surface"] == "single":
        return hashlib.sha256(np.ascontiguousarray(obs.reshape(obs.shape[1:]), dtype="<i4").tobytes()).hexdigest()
    parts = [np.ascontiguousarray(obs[i], dtype="<i8").tobytes() for i in range(obs.shape[0])
             if listed is None or listed[i]]
    return hashlib.sha256(b"".join(parts)).hexdigest()


def rewards_record(fx, rew, listed):
    if fx["surface"] == "single":
        return float(rew[0]).hex()
    return [[i, float(rew[i]).hex()] for i in range(len(listed)) if listed[i]]


def compare_call(fx, rec, got, where):
    """Assert one call's outputs equal the fixture's.  `got` has keys obs_sha, state and,
    for steps, rew, done, trunc, listed (multi)."""
    assert got["kind"] == rec["kind"], where
    if "raised" in rec:  # the step re-raised an agent's error: only the state it left is defined
        assert got.get("raised"), (where, "expected the step to raise", rec["raised"])
        if isinstance(got["raised"], list):
            assert got["raised"] == rec["raised"], (where, "raised", got["raised"], rec["raised"])
        for k in ("ctr", "agents", "players", "dyn", "obst", "dead"):
            assert got["state"][k] == rec["state"][k], (where, k, got["state"][k], rec["state"][k])
        return
    assert not got.get("raised"), (where, "raised", got.get("raised"))
    if rec["kind"] == "step":
        assert got["done"] == rec["done"], (where, "done")
        assert got["trunc"] == rec["trunc"], (where, "trunc")
        if fx["surface"] == "multi":
            assert got["listed"] == rec["before"], (where, "listed", got["listed"], rec["before"])
        assert got["rew"] == rec["rew"], (where, "rew", got["rew"], rec["rew"])
    st = got["state"]
    for k in ("ctr", "agents", "players", "dyn", "obst", "dead"):
        if st is not None and k in st:
            assert st[k] == rec["state"][k], (where, k, st[k], rec["state"][k])
    if "obs" in rec and got.get("obs_full") is not None:
        exp = rec["obs"]
        if fx["surface"] == "single":
            assert list(np.asarray(got["obs_full"]).ravel()) == exp, (where, "obs")
        else:
            assert [list(np.asarray(o).ravel()) for o in got["obs_full"]] == exp, (where, "obs")
    assert got["obs_sha"] == rec["obs_sha"], (where, "obs_sha")
