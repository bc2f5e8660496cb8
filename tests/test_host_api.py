"""Host-side logic of the drop-in surface that runs without a GPU: constructor argument
validation (the reference's exceptions), action encoding, spaces, registration, sharding."""
import numpy as np
import pytest

from libzombsole_amd import _abi
from libzombsole_amd import actions as A
from libzombsole_amd.spaces import Box, Dict, Discrete, Text, registry
from libzombsole_amd.vector import shard_range


def test_registry():
    import libzombsole_amd.gym_env  # noqa: F401  (registers, gym_env.py:382-414)
    assert "jvstinian/Zombsole-v0" in registry
    assert "jvstinian/Zombsole-SurroundingsView-v0" in registry
    spec = registry["jvstinian/Zombsole-SurroundingsView-v0"]
    assert spec.max_episode_steps == 1000 and spec.nondeterministic
    assert spec.kwargs["observation_scope"] == "surroundings:21"


@pytest.mark.parametrize("kw,exc", [
    (dict(rules_name="nope"), ValueError),                         # rules/factory.py:19
    (dict(observation_scope="surroundings:4"), ValueError),        # observation.py:185-188
    (dict(observation_scope="planet"), ValueError),                # observation.py:189-192
    (dict(observation_position_encoding="fancy"), ValueError),     # observation.py:199-201
    (dict(agent_weapon="banana"), ValueError),                     # weapons.py:45
    (dict(player_names=["nobody"]), ModuleNotFoundError),          # game.py:30 __import__
    (dict(map_name="no_such_map"), FileNotFoundError),             # game.py Map.from_file
    (dict(render_mode="rgb_array"), ValueError),                   # gym_env.py:58-59
])
def test_single_env_constructor_errors(kw, exc):
    from libzombsole_amd.gym_env import ZombsoleGymEnv
    args = dict(rules_name="extermination", player_names=[], map_name="boxed", agent_id=0)
    args.update(kw)
    with pytest.raises(exc):
        ZombsoleGymEnv(**args)


@pytest.mark.parametrize("kw,exc", [
    (dict(observation_surroundings_width=20), ValueError),
    (dict(observation_position_encoding_style="fancy"), ValueError),
    (dict(agent_weapons=3), ValueError),                           # game.py:149
    (dict(rules_name="nope"), ValueError),
])
def test_multi_env_constructor_errors(kw, exc):
    from libzombsole_amd.gym.multiagent_env import MultiagentZombsoleEnv
    args = dict(rules_name="extermination", player_names=[], map_name="boxed", agent_ids=["0"])
    args.update(kw)
    with pytest.raises(exc):
        MultiagentZombsoleEnv(**args)


def test_weapon_cycling():
    # game.py:142-149: a str repeats, a list cycles, and zip() truncates agents to the weapons
    assert _abi.expand_weapons("axe", 3) == ["axe"] * 3
    assert _abi.expand_weapons(["axe", "gun"], 3) == ["axe", "gun", "axe"]
    b = _abi.multi_env_config(1, "extermination", [], "boxed", ["0", "1"], agent_weapons=[])
    assert b.num_agents == 0


def test_encode_action_branches():
    assert A.encode_action({}) == (A.ACT_IDLE, 0, 0)
    assert A.encode_action({"action_type": "move", "parameter": [1, -1]}) == (A.ACT_MOVE, 1, -1)
    assert A.encode_action({"action_type": "attack", "parameter": (0, 0)}) == (A.ACT_ATTACK, 0, 0)
    assert A.encode_action({"action_type": "heal"}) == (A.ACT_HEAL, 0, 0)
    assert A.encode_action({"action_type": "heal", "parameter": [0, 0]}) == (A.ACT_HEAL, 0, 0)
    assert A.encode_action({"action_type": "heal", "parameter": [2, 1]}) == (A.ACT_HEAL, 2, 1)
    assert A.encode_action({"action_type": "heal_closest"}) == (A.ACT_HEAL_CLOSEST, 0, 0)
    assert A.encode_action({"action_type": "dance"}) == (A.ACT_CONFUSED, 0, 0)
    with pytest.raises(A.ActionError):
        A.encode_action({"action_type": "move"})          # None + tuple -> TypeError in agent.py:35
    with pytest.raises(A.ActionError):
        A.encode_action({"action_type": "heal", "parameter": np.array([1, 0])})  # ambiguous truth value


def test_discrete_tables_match_reference_order():
    from libzombsole_amd.gym.multiagent_env import MultiagentZombsoleEnvDiscreteAction
    from libzombsole_amd.gym_env import ZombsoleGymEnvDiscreteAction
    assert ZombsoleGymEnvDiscreteAction.game_actions == A.SINGLE_DISCRETE_ACTIONS
    assert MultiagentZombsoleEnvDiscreteAction.game_actions == A.MULTI_DISCRETE_ACTIONS
    for i, act in enumerate(A.MULTI_DISCRETE_ACTIONS):
        assert tuple(A.DISCRETE_TRIPLES[i]) == A.encode_action(dict(act, parameter=act.get("parameter", [0, 0])))


def test_spaces_shim():
    d = Discrete(7, seed=3)
    vals = {d.sample() for _ in range(200)}
    assert vals <= set(range(7)) and len(vals) == 7
    assert d.contains(6) and not d.contains(7)
    b = Box(low=-10, high=10, shape=(2,), dtype=np.int32)
    s = b.sample()
    assert s.shape == (2,) and s.dtype == np.int32 and b.contains(s)
    sp = Dict({"action_type": Text(15), "parameter": b})
    x = sp.sample()
    assert sp.contains(x) and 1 <= len(x["action_type"]) <= 15


@pytest.mark.parametrize("total,world", [(65536, 8), (10, 3), (7, 8), (8192, 1)])
def test_shard_range_partitions(total, world):
    cover = []
    for r in range(world):
        e0, n = shard_range(total, r, world)
        cover.extend(range(e0, e0 + n))
    assert cover == list(range(total))


def test_obs_shapes():
    b = _abi.single_env_config(4, "extermination", [], "bridge", 0, observation_scope="surroundings:11",
                               observation_position_encoding="channels")
    assert b.obs_shape() == (1, 3, 11, 11)
    b = _abi.single_env_config(4, "extermination", [], "bridge", 0)
    assert b.obs_shape() == (1, 1, 12, 111)
    b = _abi.multi_env_config(4, "extermination", [], "bridge64", ["0", "1", "2"])
    assert b.obs_shape() == (3, 3, 21, 21)
