"""Scripted request sessions for the JSON-over-stdio server (zombsole/interactive_json.py).

Shared by tests/golden/make_stdio_golden.py (which records the reference's transcripts) and
tests/test_stdio_json.py (which replays them against libzombsole_amd.interactive_json).
"""
import json

from libzombsole_amd import actions as A


def _req(tag, parameters=None, with_params=True):
    d = {"tag": tag}
    if with_params:
        d["parameters"] = parameters
    return json.dumps(d)


def _config(**kw):
    return _req("GameConfigUpdate", kw)


def _single_actions(seed, n):
    return [_req("GameAction", A.rich_action(seed, t, 0)) for t in range(1, n + 1)]


def _multi_actions(seed, n, ids):
    return [_req("GameAction", {aid: A.rich_action(seed, t, i) for i, aid in enumerate(ids)}) for t in range(1, n + 1)]


_PROTOCOL_ERRORS = [
    "this is not json",
    _req("Bogus", None, with_params=False),
    _req("GameAction", None, with_params=False),
    _req("GameConfigUpdate", None, with_params=False),
    _config(rules_name="extermination"),  # GameConfig(**d) raises TypeError: missing arguments
    _config(rules_name="extermination", map_name="bridge", players=[], agent_ids=["0"], colour="red"),
]

SESSIONS = [
    dict(name="single_surr_channels", multi=False, seed=21, requests=(
        [_req("GameStatus", with_params=False)] + _PROTOCOL_ERRORS +
        [_config(rules_name="extermination", map_name="bridge", players=[], agent_ids=["0"], initial_zombies=10,
                 minimum_zombies=2, observation_scope="surroundings:11", observation_position_encoding="channels"),
         _req("GameStatus", with_params=False), _req("StartGame", with_params=False)] +
        _single_actions(21, 40) +
        [_req("GameStatus", with_params=False), _req("Exit", with_params=False)])),
    dict(name="single_world_simple_bots", multi=False, seed=22, requests=(
        [_config(rules_name="safehouse", map_name="to_the_closet", players=["terminator", "sniper"],
                 agent_ids=["0"], initial_zombies=6, minimum_zombies=6),
         _req("StartGame", with_params=False)] + _single_actions(22, 25) +
        # a second game on a new config, then a restart of it
        [_config(rules_name="survival", map_name="boxed", players=[], agent_ids=["7"], initial_zombies=2,
                 minimum_zombies=0, observation_scope="world", observation_position_encoding="channels"),
         _req("StartGame", with_params=False)] + _single_actions(23, 10) +
        [_req("StartGame", with_params=False)] + _single_actions(24, 5) + [_req("Exit", with_params=False)])),
    dict(name="multi_bridge", multi=True, seed=23, requests=(
        [_req("GameStatus", with_params=False),
         _config(rules_name="extermination", map_name="bridge", players=[], agent_ids=["0", "1"],
                 initial_zombies=12, minimum_zombies=4, observation_scope="surroundings:9"),
         _req("StartGame", with_params=False)] + _multi_actions(23, 40, ["0", "1"]) +
        [_req("GameStatus", with_params=False), _req("Exit", with_params=False)])),
    dict(name="multi_default_width", multi=True, seed=24, requests=(
        [_config(rules_name="evacuation", map_name="easy_exit", players=["troll"], agent_ids=["0", "1", "2"],
                 initial_zombies=5, minimum_zombies=5),
         _req("StartGame", with_params=False)] + _multi_actions(24, 20, ["0", "1", "2"]) +
        [_req("Exit", with_params=False)])),
    # sessions the reference's server does not survive
    dict(name="no_tag", multi=False, seed=25, requests=[json.dumps({"parameters": 1})]),
    # channel observations encode agents as 8 + int(agent_id) (observation.py:74): ValueError
    dict(name="multi_nonint_ids", multi=True, seed=28, requests=[
        _config(rules_name="extermination", map_name="bridge", players=[], agent_ids=["a", "b"],
                initial_zombies=3, minimum_zombies=0),
        _req("StartGame", with_params=False)]),
    dict(name="start_before_config", multi=False, seed=26, requests=[_req("StartGame", with_params=False)]),
    dict(name="eof", multi=True, seed=27, requests=[_req("GameStatus", with_params=False)]),
]
