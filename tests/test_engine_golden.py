"""HIP engine vs the reference's golden vectors (and the C oracle), through the C ABI.

Every seed of a fixture runs as one env of a single batched engine, stepped in
lock-step with the engine's next-step autoreset — the same call protocol the
fixtures were recorded under (tests/golden/make_golden.py).  Bit-exact on
obs, state and float64 rewards.
"""
import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu


def _engine(fx, n):
    from libzombsole_amd.engine import Engine
    return Engine(G.builder_for(fx, num_envs=n))


def replay_engine(fx):
    import torch
    runs = fx["runs"]
    n = len(runs)
    eng = _engine(fx, n)
    kinds = [o[2] for o in eng.builder.map.obstacles]
    eng.seed([r["seed"] for r in runs])
    pokes = G.obstacle_pokes(fx)
    for k in range(n if pokes else 0):  # the map's Box/Wall life before the first reset (carried over)
        st = eng.get_state(k)
        for i, life in pokes:
            st.obst_life[i] = life
        eng.set_state(k, st)
    eng.reset()
    ncalls = len(runs[0]["calls"])
    for i in range(ncalls):
        if i > 0:
            acts = np.zeros((n, eng.A, 3), dtype=np.int32)
            for k, r in enumerate(runs):
                rec = r["calls"][i]
                if rec["kind"] == "step":
                    acts[k] = G.action_triples(fx, rec, eng.A)[:eng.A]
            eng.actions.copy_(torch.from_numpy(acts))
            eng.step()
        torch.cuda.synchronize()
        obs = eng.obs.cpu().numpy()
        rew = eng.rewards.cpu().numpy()
        done = eng.done.cpu().numpy()
        trunc = eng.trunc.cpu().numpy()
        listed = eng.listed.cpu().numpy()
        was_reset = eng.was_reset.cpu().numpy()
        for k, r in enumerate(runs):
            rec = r["calls"][i]
            where = (fx["name"], r["seed"], i)
            kind = "reset" if (i == 0 or was_reset[k]) else "step"
            got = {"kind": kind}
            if "raised" in rec:  # the step stopped at a ZS_ACT_RAISE agent: only the state is defined
                got.update(raised=True, state=eng.get_state(k).canonical(kinds))
                G.compare_call(fx, rec, got, where)
                continue
            lst = listed[k].astype(bool) if kind == "step" else np.ones(eng.A, bool)
            if kind == "step":
                got.update(done=bool(done[k]), trunc=bool(trunc[k]),
                           listed=[j for j in range(eng.A) if lst[j]],
                           rew=G.rewards_record(fx, rew[k], lst))
            got["obs_sha"] = G.obs_sha(fx, obs[k], lst if fx["surface"] == "multi" else None)
            got["state"] = eng.get_state(k).canonical(kinds)
            if "obs" in rec:
                got["obs_full"] = obs[k] if fx["surface"] == "single" else [obs[k][j] for j in range(eng.A) if lst[j]]
            G.compare_call(fx, rec, got, where)
    eng.close()


@pytest.mark.parametrize("name", G.fixture_names())
def test_engine_matches_reference(name):
    replay_engine(G.load_fixture(name))
