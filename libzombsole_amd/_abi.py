"""ctypes mirror of include/zombsole_mi355x.h (constants, structs) and the
host-side translation of the reference's constructor arguments into a
`zs_config` (rules / weapon / observation / player-name factories).

Pure host code: importable without torch or a GPU.
"""
import ctypes as C

import numpy as np

from .maps import Map, load_map

# status codes
ZS_OK, ZS_EINVAL, ZS_ENOSPACE, ZS_EHIP, ZS_ESTATE = 0, 1, 2, 3, 4
# things
THING_NONE, THING_BOX, THING_DEADBODY, THING_OBJECTIVE, THING_WALL = 0, 1, 2, 3, 4
THING_ZOMBIE, THING_PLAYER, THING_AGENT = 5, 6, 7
# weapons (observation codes, gym/observation.py:27-34)
WEAPON_NONE, WEAPON_CLAWS, WEAPON_KNIFE, WEAPON_AXE = 0, 1, 10, 11
WEAPON_GUN, WEAPON_RIFLE, WEAPON_SHOTGUN, WEAPON_RANDOM = 12, 13, 14, 255
# bots
BOT_TERMINATOR, BOT_SNIPER, BOT_TROLL, BOT_HAMSTER, BOT_RANDOMAN = 1, 2, 3, 4, 5
# rules
RULES_EXTERMINATION, RULES_SURVIVAL, RULES_EVACUATION, RULES_SAFEHOUSE = 0, 1, 2, 3
REWARD_SINGLE, REWARD_MULTI = 0, 1
OBS_WORLD, OBS_SURROUNDINGS = 0, 1
ENC_SIMPLE, ENC_CHANNELS = 0, 1
DTYPE_I32, DTYPE_I64, DTYPE_I16 = 0, 1, 2
FLAG_AUTORESET = 1
FLAG_DEBUG = 2
FLAG_DEATH_LOG = 4  # zs_death_log: the drop-in views' decoration order and removed zombies' final values
OVF_INT16, OVF_INT32 = 1, 2  # zs_overflow range flags
STATE_HEADER, STATE_ENTITY_WORDS = 16, 8

DTYPE_NP = {DTYPE_I32: np.int32, DTYPE_I64: np.int64, DTYPE_I16: np.int16}

_RULES = {"extermination": RULES_EXTERMINATION, "survival": RULES_SURVIVAL,
          "evacuation": RULES_EVACUATION, "safehouse": RULES_SAFEHOUSE}
_WEAPONS = {"knife": WEAPON_KNIFE, "axe": WEAPON_AXE, "gun": WEAPON_GUN, "rifle": WEAPON_RIFLE,
            "shotgun": WEAPON_SHOTGUN, "random": WEAPON_RANDOM}
_BOTS = {"terminator": BOT_TERMINATOR, "sniper": BOT_SNIPER, "troll": BOT_TROLL,
         "hamster": BOT_HAMSTER, "randoman": BOT_RANDOMAN}


class zs_map_desc(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32),
                ("n_obstacles", C.c_int32), ("obstacle_xy", C.POINTER(C.c_int32)),
                ("obstacle_kind", C.POINTER(C.c_uint8)),
                ("n_objectives", C.c_int32), ("objective_xy", C.POINTER(C.c_int32)),
                ("n_player_spawns", C.c_int32), ("player_spawn_xy", C.POINTER(C.c_int32)),
                ("n_zombie_spawns", C.c_int32), ("zombie_spawn_xy", C.POINTER(C.c_int32))]


LAUNCH_FIELDS = ["fused", "fobs", "tick_waves", "lds_budget", "rw_need", "reset_wgs", "reset_stream", "reset_lists",
                 "reset_grid", "defer_respawn", "respawn_grid", "obs_pipe", "obs_lds", "obs_patch", "obs_ring",
                 "obs_ring_patch", "obs_gather", "obs_gather_stat", "obs_stat", "obs_win", "obs_wgs", "par_exec"]


class zs_launch(C.Structure):
    """Launch overrides (include/zombsole_mi355x.h): 0 = automatic; switches 1 = on, -1 = off."""
    _fields_ = [(f, C.c_int32) for f in LAUNCH_FIELDS] + [("reserved", C.c_int32 * 10)]


class zs_config(C.Structure):
    _fields_ = [("num_envs", C.c_int32), ("map", zs_map_desc), ("rules", C.c_int32),
                ("num_agents", C.c_int32), ("agent_weapons", C.POINTER(C.c_int32)),
                ("agent_codes", C.POINTER(C.c_int32)),
                ("num_bots", C.c_int32), ("bot_types", C.POINTER(C.c_int32)),
                ("initial_zombies", C.c_int32), ("minimum_zombies", C.c_int32),
                ("reward_mode", C.c_int32), ("obs_scope", C.c_int32), ("obs_encoding", C.c_int32),
                ("obs_width", C.c_int32), ("obs_dtype", C.c_int32),
                ("max_episode_steps", C.c_int32), ("flags", C.c_uint32), ("lanes_per_env", C.c_int32),
                ("launch", C.POINTER(zs_launch))]


def rules_id(rules_name):
    """RulesFactory.create_rules (rules/factory.py:9-19)."""
    if rules_name in _RULES:
        return _RULES[rules_name]
    raise ValueError(f"{rules_name} is not a valid rule name.  Valid options are extermination, "
                     "survival, evacuation, and safehouse")


def weapon_id(weapon_name):
    """WeaponFactory.create_player_weapon (weapons.py:28-45)."""
    w = _WEAPONS.get(str(weapon_name).lower())
    if w is None:
        raise ValueError(f"{weapon_name} is not a valid player weapon name.  Valid options are knife, "
                         "axe, gun, rifle, shotgun, and random.")
    return w


def bot_id(name):
    """create_player -> __import__('zombsole.players.' + name) (game.py:17-32)."""
    if name in _BOTS:
        return _BOTS[name]
    if name == "me":
        raise NotImplementedError("the interactive keyboard player 'me' blocks on input() and "
                                  "cannot run in a batched engine (SURVEY.md §2)")
    raise ModuleNotFoundError("No module named 'zombsole.players.%s'" % name)


def expand_weapons(agent_weapons, n_agents):
    """Game.__process_weapon_name_inputs__ (game.py:142-149)."""
    if isinstance(agent_weapons, str):
        names = [agent_weapons] * n_agents
    elif isinstance(agent_weapons, list):
        names = [agent_weapons[i % len(agent_weapons)] for i in range(n_agents)] if agent_weapons else []
        if len(names) < n_agents:
            names = names  # islice(cycle([])) yields nothing; zip() then truncates agents
    else:
        raise ValueError(f"{agent_weapons} is not a valid value for argument agent_weapons.  Value must "
                         "be the weapon name as a string or a list of weapon names.")
    return names


def parse_scope(scope):
    """build_observation scope parsing (gym/observation.py:176-192) -> (OBS_*, width)."""
    lscope = scope.lower()
    if lscope in ["world", "map"]:
        return OBS_WORLD, 0
    if lscope.startswith("surroundings"):
        width = int(lscope[len("surroundings:"):])
        if (width % 2 == 0) or (width <= 1):
            raise ValueError("surroundings width must be an odd number greater than 1")
        return OBS_SURROUNDINGS, width
    raise ValueError(f"{scope} is not a valid observation scope, must be \"world\", \"map\", or of the "
                     "form \"surroundings:i\" where i is an integer")


def parse_encoding(style):
    lpes = style.lower()
    if lpes not in ["simple", "channels"]:
        raise ValueError(f"{lpes} must be \"simple\" or \"channels\"")
    return ENC_SIMPLE if lpes == "simple" else ENC_CHANNELS


def agent_code(agent_id):
    """Channels code of an agent: 8 + int(agent_id) (gym/observation.py:59-60).

    The reference evaluates int(agent_id) lazily in the encoder; ids that do
    not convert get code -1 here and the wrapper raises the reference's
    ValueError when a channels observation is produced."""
    try:
        return 8 + int(agent_id)
    except (TypeError, ValueError):
        return -1


class ConfigBuilder(object):
    """Owns the numpy arrays a zs_config points into."""

    def __init__(self, num_envs, map_, rules, agent_weapons, agent_codes, bot_types, initial_zombies,
                 minimum_zombies, reward_mode, obs_scope, obs_encoding, obs_width, obs_dtype,
                 max_episode_steps=0, autoreset=True, lanes_per_env=0, debug=False):
        m = map_ if isinstance(map_, Map) else load_map(map_)
        self.map = m

        def xy(lst):
            a = np.asarray(lst, dtype=np.int32).reshape(-1, 2)
            return np.ascontiguousarray(a)

        self._obst_xy = xy([o[:2] for o in m.obstacles])
        self._obst_kind = np.ascontiguousarray(np.asarray([o[2] for o in m.obstacles], dtype=np.uint8))
        self._obj = xy(m.objectives)
        self._ps = xy(m.player_spawns)
        self._zs = xy(m.zombie_spawns)
        self._aw = np.ascontiguousarray(np.asarray(agent_weapons, dtype=np.int32))
        self._ac = np.ascontiguousarray(np.asarray(agent_codes, dtype=np.int32))
        self._bt = np.ascontiguousarray(np.asarray(bot_types, dtype=np.int32))
        p32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
        md = zs_map_desc(m.size[0], m.size[1], len(m.obstacles), p32(self._obst_xy),
                         self._obst_kind.ctypes.data_as(C.POINTER(C.c_uint8)),
                         len(m.objectives), p32(self._obj), len(m.player_spawns), p32(self._ps),
                         len(m.zombie_spawns), p32(self._zs))
        self.cfg = zs_config(int(num_envs), md, int(rules), len(self._aw), p32(self._aw), p32(self._ac),
                             len(self._bt), p32(self._bt), int(initial_zombies), int(minimum_zombies),
                             int(reward_mode), int(obs_scope), int(obs_encoding), int(obs_width),
                             int(obs_dtype), int(max_episode_steps),
                             (FLAG_AUTORESET if autoreset else 0) | (FLAG_DEBUG if debug else 0),
                             int(lanes_per_env))
        self._launch = None

    def set_launch(self, overrides):
        """Force launch alternatives for the handles built from this config: a dict of zs_launch fields
        (LAUNCH_FIELDS), e.g. {"fused": -1, "obs_ring": 1}; None or {} = every choice automatic."""
        if not overrides:
            self._launch = None
            self.cfg.launch = C.POINTER(zs_launch)()
            return self
        unknown = set(overrides) - set(LAUNCH_FIELDS)
        if unknown:
            raise ValueError("unknown launch overrides: %s" % sorted(unknown))
        self._launch = zs_launch(**{k: int(v) for k, v in overrides.items()})
        self.cfg.launch = C.pointer(self._launch)
        return self

    @property
    def launch(self):
        """The overrides set on this config, as a dict of the non-zero fields."""
        if self._launch is None:
            return {}
        return {f: getattr(self._launch, f) for f in LAUNCH_FIELDS if getattr(self._launch, f)}

    @property
    def num_agents(self):
        return len(self._aw)

    @property
    def num_bots(self):
        return len(self._bt)

    def obs_shape(self):
        """(obs per env, C, H, W) — mirrors zs_obs_shape."""
        c = self.cfg
        chans = 3 if c.obs_encoding == ENC_CHANNELS else 1
        if c.obs_scope == OBS_WORLD:
            h, w = c.map.height, c.map.width
        else:
            h = w = c.obs_width
        n = c.num_agents if (c.reward_mode == REWARD_MULTI and c.obs_scope == OBS_SURROUNDINGS) else 1
        return (n, chans, h, w)

    def ptr(self):
        return C.byref(self.cfg)


def single_env_config(num_envs, rules_name, player_names, map_name, agent_id, initial_zombies=0,
                      minimum_zombies=0, observation_scope="world", observation_position_encoding="simple",
                      agent_weapon="rifle", max_episode_steps=0, obs_dtype=DTYPE_I32, autoreset=True,
                      lanes_per_env=0, debug=False):
    """zs_config for the ZombsoleGymEnv surface (gym_env.py:49-83): one agent + bots."""
    m = load_map(map_name)
    rules = rules_id(rules_name)
    bots = [bot_id(n) for n in player_names]
    weapons = [weapon_id(w) for w in expand_weapons([agent_weapon], 1)]
    scope, width = parse_scope(observation_scope)
    enc = parse_encoding(observation_position_encoding)
    return ConfigBuilder(num_envs, m, rules, weapons, [agent_code(agent_id)], bots, initial_zombies,
                         minimum_zombies, REWARD_SINGLE, scope, enc, width, obs_dtype, max_episode_steps,
                         autoreset, lanes_per_env, debug)


def multi_env_config(num_envs, rules_name, player_names, map_name, agent_ids, initial_zombies=0,
                     minimum_zombies=0, observation_surroundings_width=21,
                     observation_position_encoding_style="channels", agent_weapons="rifle",
                     max_episode_steps=0, obs_dtype=DTYPE_I64, autoreset=True, lanes_per_env=0, debug=False):
    """zs_config for the MultiagentZombsoleEnv surface (gym/multiagent_env.py:25-78)."""
    w = int(observation_surroundings_width)
    if (w % 2 == 0) or (w <= 1):
        raise ValueError("surroundings width must be an odd number greater than 1")
    enc = parse_encoding(observation_position_encoding_style)
    m = load_map(map_name)
    rules = rules_id(rules_name)
    bots = [bot_id(n) for n in player_names]
    names = expand_weapons(agent_weapons, len(agent_ids))
    ids = list(agent_ids)[:len(names)]  # zip(agent_ids, agent_weapons) truncates (game.py:162-163)
    weapons = [weapon_id(n) for n in names]
    return ConfigBuilder(num_envs, m, rules, weapons, [agent_code(a) for a in ids], bots, initial_zombies,
                         minimum_zombies, REWARD_MULTI, OBS_SURROUNDINGS, enc, w, obs_dtype,
                         max_episode_steps, autoreset, lanes_per_env, debug)
