"""The drop-in classes (ZombsoleGymEnv*, MultiagentZombsoleEnv*) replayed through the very
driver that recorded the golden fixtures from the reference (tests/golden_driver.py):
same constructor calls, `random.seed(s); env.reset()`, same action streams, same records.
Every record must equal the reference's — obs sha256 (and full obs for the first calls),
float64 reward hex, done/truncated, the canonical state read through `env.game`.
"""
import pytest

import golden_util as G
from golden_driver import run_config

pytestmark = pytest.mark.gpu


class K:
    from libzombsole_amd.things import Agent, Box, DeadBody, Player, Wall, Zombie
    from libzombsole_amd.gym_env import ZombsoleGymEnv, ZombsoleGymEnvDiscreteAction
    from libzombsole_amd.gym.multiagent_env import MultiagentZombsoleEnv, MultiagentZombsoleEnvDiscreteAction

    @staticmethod
    def map_arg(name):
        return G.map_path(name)


def _cfg(fx):
    runs = fx["runs"]
    calls = len(runs[0]["calls"])
    full = sum(1 for r in runs[0]["calls"] if "obs" in r)
    return (fx["name"], fx["surface"], fx["stream"], fx["kwargs"], [r["seed"] for r in runs], calls, full,
            fx["max_steps"], fx.get("extras") or {})


# the 32-agent fort fixture is covered through the batched ABI (test_engine_golden)
NAMES = [n for n in G.fixture_names() if n != "multi_fort_a32_z100"]


@pytest.mark.parametrize("name", NAMES)
def test_dropin_matches_reference(name):
    fx = G.load_fixture(name)
    got = run_config(_cfg(fx), K)
    for r_exp, r_got in zip(fx["runs"], got["runs"]):
        assert r_exp["seed"] == r_got["seed"]
        for i, (a, b) in enumerate(zip(r_exp["calls"], r_got["calls"])):
            for k in a:
                assert b.get(k) == a[k], (name, r_exp["seed"], i, k)
