"""Action vocabulary shared by the host wrappers, the tests and the device bench.

The reference's agents take an action dict ``{"action_type": str, "parameter": [dx, dy]}``
(`zombsole/gym_env.py:43-46`, consumed by `zombsole/players/agent.py:22-96`).  The
engine's C-ABI takes the same information as an int32 triple ``(kind, dx, dy)``
per agent (`include/zombsole_mi355x.h`, ``ZS_ACT_*``).

Also defines the counter-based action streams used for parity runs and for the
benchmark: every action is a pure function of
``(env seed, step index, agent index)`` through splitmix64, so the identical
stream can be produced in Python (for the reference / oracle) and on the GPU
(``zs_gen_actions``).
"""
import numpy as np

# --- engine action kinds (must match include/zombsole_mi355x.h) -------------
ACT_IDLE = 0            # falsy action_type -> next_step returns None   (agent.py:30-32)
ACT_MOVE = 1            # pos + parameter                               (agent.py:33-37)
ACT_ATTACK = 2          # thing at pos + parameter                      (agent.py:49-58)
ACT_ATTACK_CLOSEST = 3  # closest zombie in dict order                  (agent.py:38-48)
ACT_HEAL = 4            # self if parameter falsy/(0,0) else Player/Box/Wall at pos+parameter (agent.py:59-75)
ACT_HEAL_CLOSEST = 5    # closest other Player, else self               (agent.py:76-88)
ACT_CONFUSED = 6        # unknown action_type -> None                   (agent.py:89-91)
ACT_RAISE = 7           # next_step raises (debug=True): World.step stops at this actor (core.py:96-99)

_KIND_BY_NAME = {
    "move": ACT_MOVE,
    "attack": ACT_ATTACK,
    "attack_closest": ACT_ATTACK_CLOSEST,
    "heal": ACT_HEAL,
    "heal_closest": ACT_HEAL_CLOSEST,
}

# Discrete action tables, in the reference's order.
# ZombsoleGymEnvDiscreteAction.game_actions  (gym_env.py:328-351)
SINGLE_DISCRETE_ACTIONS = [
    {"action_type": "move", "parameter": [0, 1]},
    {"action_type": "move", "parameter": [-1, 0]},
    {"action_type": "move", "parameter": [0, -1]},
    {"action_type": "move", "parameter": [1, 0]},
    {"action_type": "attack_closest"},
    {"action_type": "heal"},
]
# MultiagentZombsoleEnvDiscreteAction.game_actions  (gym/multiagent_env.py:259-285)
MULTI_DISCRETE_ACTIONS = SINGLE_DISCRETE_ACTIONS + [{"action_type": "heal_closest"}]

# The same tables as engine triples.  The multi-agent env fills a missing
# parameter with [0, 0] (multiagent_env.py:99-104); the single env leaves it
# None, which agent.py:61 treats exactly like (0, 0) for 'heal'.
DISCRETE_TRIPLES = np.array([
    [ACT_MOVE, 0, 1],
    [ACT_MOVE, -1, 0],
    [ACT_MOVE, 0, -1],
    [ACT_MOVE, 1, 0],
    [ACT_ATTACK_CLOSEST, 0, 0],
    [ACT_HEAL, 0, 0],
    [ACT_HEAL_CLOSEST, 0, 0],
], dtype=np.int32)


class ActionError(Exception):
    """An action the reference's Agent.next_step would raise on."""


def _target_offset(param):
    """The offset `Agent.next_step` adds to the position, evaluated as the reference does
    (``self.position[0] + self.action_parameter[0]``, agent.py:36-37 / 51-52 / 67-68), so a bad
    parameter raises the reference's own exception (None -> TypeError, short -> IndexError,
    str -> TypeError)."""
    try:
        ox, oy = 0 + param[0], 0 + param[1]
        return int(ox), int(oy)
    except Exception as err:
        raise ActionError(err)


def encode_action(action):
    """Map one reference action dict to an engine triple.

    Mirrors the branches of `Agent.next_step` (`zombsole/players/agent.py:28-96`), in its order
    of evaluation.  Raises ActionError (carrying the exception the reference would raise) for
    inputs on which the reference raises inside next_step; the caller decides, like
    `World.get_actions` (`core.py:96-99`), whether to re-raise (debug) or to treat the agent as
    idle.
    """
    atype = action.get("action_type", None)
    param = action.get("parameter", None)
    if not atype:
        return (ACT_IDLE, 0, 0)
    kind = _KIND_BY_NAME.get(atype, ACT_CONFUSED) if isinstance(atype, str) else ACT_CONFUSED
    if kind in (ACT_MOVE, ACT_ATTACK):
        dx, dy = _target_offset(param)
        return (kind, dx, dy)
    if kind == ACT_HEAL:
        try:  # (not param) or (tuple(param) == (0, 0))  (agent.py:61)
            self_heal = (not param) or (tuple(param) == (0, 0))
        except Exception as err:  # numpy truth value, tuple(int)...
            raise ActionError(err)
        if self_heal:
            return (ACT_HEAL, 0, 0)
        dx, dy = _target_offset(param)
        return (ACT_HEAL, dx, dy)
    return (kind, 0, 0)


# --- counter-based action streams -------------------------------------------
_M64 = (1 << 64) - 1


def splitmix64(x):
    """splitmix64 finaliser (same constants as zs_gen_actions in engine.hip)."""
    x = (x + 0x9E3779B97F4A7C15) & _M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def action_hash(seed, step, agent):
    return splitmix64(splitmix64(splitmix64(seed & _M64) ^ (step & _M64)) ^ (agent & _M64))


def discrete_action_id(seed, step, agent, n_actions):
    """Uniform discrete action id (bench / parity stream)."""
    return action_hash(seed, step, agent) % n_actions


RICH_TYPES = [None, "move", "attack", "attack_closest", "heal", "heal_closest", "dance", "move"]


def rich_action(seed, step, agent):
    """A dict action covering every Agent.next_step branch, incl. bad inputs.

    kind = h % 8 over RICH_TYPES; parameter = two values in [-2, 2] so that
    adjacent targets (and (0, 0) = self) are hit often.
    """
    h = action_hash(seed, step, agent)
    atype = RICH_TYPES[h % 8]
    dx = int((h >> 8) % 5) - 2
    dy = int((h >> 16) % 5) - 2
    return {"action_type": atype, "parameter": [dx, dy]}


BAD_PARAMETERS = [None, [1], 5, ["a", 1]]


def bad_action(seed, step, agent):
    """rich_action, with one in eight actions carrying a parameter on which Agent.next_step raises
    for move / attack / heal (None, a short list, an int, a str coordinate: agent.py:36-68)."""
    act = rich_action(seed, step, agent)
    h = action_hash(seed ^ 0x5A5A, step, agent)
    if h % 8 == 0:
        act = {"action_type": ("move", "attack", "heal")[(h >> 3) % 3],
               "parameter": BAD_PARAMETERS[(h >> 5) % len(BAD_PARAMETERS)]}
    return act
