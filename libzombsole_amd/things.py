"""Host-side views of the things of one engine env (`env.game.world.things` & co.).

The reference keeps every game object as a Python instance (`zombsole/core.py:211-251`,
`zombsole/things.py`, `zombsole/players/agent.py`); here the state lives in HBM and these
classes are thin views over one env's `zs_get_state` record, so code written against the
reference (`isinstance(thing, Zombie)`, `thing.life`, `agent.position`,
`env.game.agents[0].life = 25`) keeps working:

  * class names, `name`, `MAX_LIFE`, `ask_for_actions`, `is_decoration` and `weapon`
    follow the reference (`things.py:10-160`, `weapons.py:18-25`, `players/*.py` create());
  * reads come from a state record cached until the env next steps or resets;
  * `life` is writable (the tests' pokes, `tests/test_game.py:55,105`,
    `tests/test_multiagent_env.py:108`) and goes to the device through `zs_set_state`.

A thing removed by a step's cleanup keeps its values at removal, as the reference object does once
it is out of the world: the drop-in env hands each step's removals (the engine's death log) to the
views, so a zombie view reports its final position and life even when the same step's respawn
reuses its slot (GameView.after_step).
"""
from . import _abi


class Weapon(object):
    """`core.Weapon` (core.py:236-241) with the classes of weapons.py:18-25."""

    def __init__(self, name, max_range, damage_range):
        self.name = name
        self.max_range = max_range
        self.damage_range = damage_range

    def __repr__(self):
        return "<%s>" % self.name


_WEAPONS = {
    _abi.WEAPON_CLAWS: ("ZombieClaws", 1.5, (5, 10)),
    _abi.WEAPON_KNIFE: ("Knife", 1.5, (5, 10)),
    _abi.WEAPON_AXE: ("Axe", 1.5, (75, 100)),
    _abi.WEAPON_GUN: ("Gun", 6, (10, 50)),
    _abi.WEAPON_RIFLE: ("Rifle", 10, (25, 75)),
    _abi.WEAPON_SHOTGUN: ("Shotgun", 3, (75, 100)),
}


def weapon_for_code(code):
    w = _WEAPONS.get(int(code))
    return Weapon(*w) if w else None


class Thing(object):
    """`core.Thing` (core.py:211-233)."""
    MAX_LIFE = 1
    ICON_BASIC = "?"
    ask_for_actions = False
    is_decoration = False
    dead_decoration = None

    name = "thing"

    def next_step(self, things, t):
        return None

    def __repr__(self):
        return "<%s %s at %s life %s>" % (type(self).__name__, self.name, self.position, self.life)


class FightingThing(Thing):
    ask_for_actions = True


class _Static(object):
    """Fixed position / life (decorations, map-file things)."""

    def __init__(self, position, life=0):
        self.position = tuple(position)
        self.life = life


class DeadBody(_Static, Thing):
    ICON_BASIC = "="
    is_decoration = True

    def __init__(self, name, position):
        _Static.__init__(self, position, 0)
        self.name = name


class ObjectiveLocation(_Static, Thing):
    ICON_BASIC = "*"
    is_decoration = True
    name = "objective"


class _ObstacleView(object):
    """A Box or Wall.  Bound to an engine env, life and presence come from the state
    record (the reference shares one map object across episodes, so the HP carries over,
    `game.py:154-155`); unbound (`Map.things` of a parsed map) it is a plain full-life thing."""

    def __init__(self, position, game=None, index=-1):
        self._game = game
        self._index = index
        self.position = tuple(position)
        self._life = self.MAX_LIFE

    @property
    def life(self):
        if self._game is None:
            return self._life
        return int(self._game._state().obst_life[self._index])

    @life.setter
    def life(self, value):
        if self._game is None:
            self._life = int(value)
        else:
            self._game._poke_obstacle(self._index, int(value))


class Box(_ObstacleView, Thing):
    MAX_LIFE = 10
    ICON_BASIC = "@"
    name = "box"


class Wall(_ObstacleView, Thing):
    MAX_LIFE = 200
    ICON_BASIC = "#"
    name = "wall"


class _EntityView(object):
    """An agent / bot / zombie slot of the engine env (entity record of include/zombsole_mi355x.h)."""

    def __init__(self, game, slot, row=None):
        self._game = game
        self._slot = slot
        r = game._state().ent[slot] if row is None else row
        self._serial = int(r[7])
        self._last = [int(v) for v in r]  # always holds a row of this thing (see _finalize)
        self._gone = False

    def _row(self):
        if self._gone:
            return self._last
        r = self._game._state().ent[self._slot]
        if int(r[7]) == self._serial:
            self._last = [int(v) for v in r]
        return self._last

    def _finalize(self, x, y, life):
        """Removed from the world with these values (core.py:121-138).  The slot may already hold the
        same step's respawned zombie (a new serial): the row kept from this thing's last read (every
        poke refreshes it) supplies the fields the death log does not carry (kind, weapon)."""
        r = list(self._row())
        r[1], r[2], r[3], r[4] = 0, int(x), int(y), int(life)
        self._last = r
        self._gone = True

    @property
    def position(self):
        r = self._row()
        return (r[2], r[3])

    @position.setter
    def position(self, value):
        raise NotImplementedError("moving a thing by assigning .position is not supported by the engine "
                                  "(the reference would leave World.things keyed by the old position)")

    @property
    def life(self):
        return self._row()[4]

    @life.setter
    def life(self, value):
        if self._gone:  # no longer in the world: the reference object just holds the value
            self._last = list(self._last)
            self._last[4] = int(value)
            return
        self._game._poke_entity(self._slot, int(value))
        self._last = None
        self._row()  # re-read now, while the slot still holds this thing

    @property
    def weapon(self):
        return weapon_for_code(self._row()[5])

    @property
    def alive_in_world(self):
        return bool(self._row()[1])


def weapon_r2(code):
    """The largest squared distance a weapon's max_range reaches (weapons.py:18-25; `distance > max_range`
    in core.py:177 on integer positions)."""
    return {_abi.WEAPON_GUN: 36, _abi.WEAPON_RIFLE: 100, _abi.WEAPON_SHOTGUN: 9}.get(int(code), 2)


class Zombie(_EntityView, FightingThing):
    """`things.Zombie` (things.py:60-107)."""
    MAX_LIFE = 100
    ICON_BASIC = "x"
    name = "zombie"

    @property
    def dead_decoration(self):
        return DeadBody("zombie remains", self.position)  # things.py:64


class Player(_EntityView, FightingThing):
    """`things.Player` (things.py:110-128) — a scripted bot (players/*.py)."""
    MAX_LIFE = 100
    ICON_BASIC = "P"

    def __init__(self, game, slot, name):
        _EntityView.__init__(self, game, slot)
        self.name = name

    @property
    def dead_decoration(self):
        return DeadBody("dead " + self.name, self.position)


class Agent(Player):
    """`players/agent.Agent` (players/agent.py:9-20)."""
    ICON_BASIC = "A"

    def __init__(self, game, slot, agent_id):
        Player.__init__(self, game, slot, "agent")
        self.agent_id = agent_id
        self.thing_type = "agent"
        self.action = None
        self.action_type = None
        self.action_parameter = None

    def set_action(self, action):
        """players/agent.py:22-26: stored here; encoded to the engine triple by the env."""
        self.action = action
        self.action_type = action.get("action_type", None)
        self.action_parameter = action.get("parameter", None)


OBSTACLE_CLASSES = {_abi.THING_BOX: Box, _abi.THING_WALL: Wall}
