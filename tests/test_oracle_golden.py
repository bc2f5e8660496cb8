"""Pin the C oracle against the reference's own outputs (tests/golden).

The fixtures were produced by running the real reference (make_golden.py); a
failure here means the CPU restatement diverged from jvstinian/libzombsole.
"""
import pytest

import golden_util as G
from oracle.oracle import OracleEnv, OracleRaised


def replay_oracle(fx, run):
    b = G.builder_for(fx)
    env = OracleEnv(b)
    for i, life in G.obstacle_pokes(fx):
        assert env.poke_obstacle(i, life) == 0
    env.seed(run["seed"])
    listed = None
    for i, rec in enumerate(run["calls"]):
        where = (fx["name"], run["seed"], i)
        got = {"kind": rec["kind"]}
        if rec["kind"] == "reset":
            obs = env.reset()
            listed = [True] * b.num_agents
        else:
            acts = G.action_triples(fx, rec, b.num_agents)
            try:
                obs, rew, done, trunc, lb = env.step(acts)
            except OracleRaised:
                got.update(raised=True, state=env.state())
                G.compare_call(fx, rec, got, where)
                continue
            got.update(done=done, trunc=trunc, listed=[j for j in range(len(lb)) if lb[j]],
                       rew=G.rewards_record(fx, rew, lb))
            listed = lb
        got["obs_sha"] = G.obs_sha(fx, obs, listed if fx["surface"] == "multi" else None)
        got["state"] = env.state()
        if "obs" in rec:
            got["obs_full"] = obs if fx["surface"] == "single" else [obs[j] for j in range(len(listed)) if listed[j]]
        G.compare_call(fx, rec, got, where)


@pytest.mark.parametrize("name", G.fixture_names())
def test_oracle_matches_reference(name):
    fx = G.load_fixture(name)
    for run in fx["runs"]:
        replay_oracle(fx, run)
