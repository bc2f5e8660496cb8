"""The golden-vector driver shared by tests/golden/make_golden.py (run against the real
reference, this container only) and tests/test_dropin_golden.py (run against the drop-in
classes of libzombsole_amd on the GPU).

`K` is a namespace with the env classes (ZombsoleGymEnv, ZombsoleGymEnvDiscreteAction,
MultiagentZombsoleEnv, MultiagentZombsoleEnvDiscreteAction), the thing classes used to build
the canonical state (Box, Wall, Agent, Player, Zombie, DeadBody) and `map_arg(name)`.
The same call protocol and the same record format come out of both, so a drop-in
replay can be compared with a fixture record for record.
"""
import hashlib
import random

import numpy as np

from libzombsole_amd import actions as A

WEAPON_CODE = {"ZombieClaws": 1, "Knife": 10, "Axe": 11, "Gun": 12, "Rifle": 13, "Shotgun": 14}


def h256(b):
    return hashlib.sha256(b).hexdigest()


def weapon_code(t):
    w = getattr(t, "weapon", None)
    return WEAPON_CODE.get(w.name, 0) if w is not None else 0


def canonical_state(game, obstacles, K):
    w = game.world
    dyn = []
    for t in w.things.values():
        if isinstance(t, (K.Box, K.Wall)):
            continue
        if isinstance(t, K.Agent):
            kind, extra = 7, game.agents.index(t)
        elif isinstance(t, K.Player):
            kind, extra = 6, game.players.index(t)
        elif isinstance(t, K.Zombie):
            kind, extra = 5, 0
        else:
            raise RuntimeError("unexpected thing %r" % t)
        dyn.append([kind, t.position[0], t.position[1], t.life, weapon_code(t), extra])
    obst = []
    for i, t in enumerate(obstacles):
        present = int(w.things.get(t.position) is t)
        if t.life != t.MAX_LIFE or not present:
            obst.append([i, t.life, present])
    W = w.size[0]
    dead = sorted(p[1] * W + p[0] for p, d in w.decoration.items() if isinstance(d, K.DeadBody))
    agents = [[a.position[0], a.position[1], a.life, weapon_code(a)] for a in game.agents]
    players = [[p.position[0], p.position[1], p.life, weapon_code(p)] for p in game.players]
    return {"dyn": dyn, "obst": obst, "dead": dead, "ctr": [w.t, w.deaths, w.zombie_deaths],
            "agents": agents, "players": players}


class ViewTracker(object):
    """extras["views"]: per call, World.decoration in its dict order ([x, y, class, name]), the zombies
    of World.things in dict order with a stable identity ([ident, x, y, life]; the same object keeps
    its ident, a respawned zombie is a new one), and after a step the zombies that left the world
    since the previous call, read through the objects the driver still holds ([ident, x, y, life]:
    the reference object keeps its values at removal, core.py:121-138)."""

    def __init__(self, K):
        self.K = K
        self.held = {}  # ident -> object
        self.ids = {}   # id(object) -> ident
        self.next = 0

    def new_world(self):
        self.held, self.ids = {}, {}

    def record(self, game, rec, step):
        K = self.K
        w = game.world
        rec["deco"] = [[p[0], p[1], type(d).__name__, getattr(d, "name", "")] for p, d in w.decoration.items()]
        zs, seen = [], set()
        for t in w.things.values():
            if isinstance(t, K.Zombie):
                k = self.ids.get(id(t))
                if k is None:
                    k = self.ids[id(t)] = self.next
                    self.held[k] = t
                    self.next += 1
                seen.add(k)
                zs.append([k, t.position[0], t.position[1], t.life])
        rec["zid"] = zs
        if step:
            rec["zgone"] = [[k, t.position[0], t.position[1], t.life] for k, t in sorted(self.held.items())
                            if k not in seen]
        for k in [k for k in self.held if k not in seen]:
            del self.ids[id(self.held[k])]
            del self.held[k]


def thing_kind(K, t):
    """The family of an event's thing: zombie, agent, player (a bot), wall, box."""
    for cls, name in ((K.Zombie, "zombie"), (K.Agent, "agent"), (K.Player, "player"), (K.Wall, "wall"),
                      (K.Box, "box")):
        if isinstance(t, cls):
            return name
    return type(t).__name__


class EventTracker(object):
    """extras["events"]: after a step, the World.event records it appended (core.py:68-70), each
    [t, the thing's family, its name, the message]; a reset starts a new World (and log)."""

    def __init__(self, K):
        self.K = K
        self.n = 0

    def new_world(self, game):
        self.n = len(game.world.events)

    def record(self, game, rec):
        evs = game.world.events
        rec["events"] = [[int(t), thing_kind(self.K, th), getattr(th, "name", ""), msg] for t, th, msg in evs[self.n:]]
        self.n = len(evs)


def obs_bytes_single(obs):
    return np.ascontiguousarray(obs, dtype="<i4").tobytes()


def obs_bytes_multi(obs, agent_ids):
    keys = [a for a in agent_ids if a in obs]
    return keys, b"".join(np.ascontiguousarray(obs[a], dtype="<i8").tobytes() for a in keys)


def run_config(cfg, K):
    name, surface, stream, kw, seeds, calls, full_calls, max_steps = cfg[:8]
    # extras: poke_obstacles [[i, life], ...] set on the map's Box/Wall objects before the first reset
    # (the reference shares them across resets, game.py:151-155); stream "fixed": `actions`, one dict
    # action per agent, every step
    extras = cfg[8] if len(cfg) > 8 else {}
    kw = dict(kw)
    kw["map_name"] = K.map_arg(kw["map_name"])
    out = []
    for seed in seeds:
        if surface == "single":
            env = (K.ZombsoleGymEnvDiscreteAction if stream == "discrete" else K.ZombsoleGymEnv)(**kw)
            base = env.env if stream == "discrete" else env
            n_act = 6
        else:
            ctor = K.MultiagentZombsoleEnvDiscreteAction if stream == "discrete" else K.MultiagentZombsoleEnv
            ckw = dict(kw)
            if stream == "discrete":
                ckw.pop("observation_position_encoding_style", None)
            env = ctor(**ckw)
            base = env.env if stream == "discrete" else env
            n_act = 7
        game = base.game
        obstacles = [t for t in game.map.things if isinstance(t, (K.Box, K.Wall))]
        agent_ids = list(base.possible_agents) if surface == "multi" else [kw["agent_id"]]
        for i, life in extras.get("poke_obstacles", []):
            obstacles[i].life = life
        recs = []
        views = ViewTracker(K) if extras.get("views") else None
        events = EventTracker(K) if extras.get("events") else None
        random.seed(seed)
        obs, _ = env.reset()
        need_reset = False
        elapsed = 0
        for call in range(calls):
            rec = {}
            if call == 0 or need_reset:
                if call > 0:
                    obs, _ = env.reset()
                if views:
                    views.new_world()
                if events:
                    events.new_world(game)
                rec["kind"] = "reset"
                need_reset = False
                elapsed = 0
            else:
                rec["kind"] = "step"
                dict_act = A.bad_action if stream == "bad" else A.rich_action
                try:
                    if surface == "single":
                        if stream == "discrete":
                            act = A.discrete_action_id(seed, call, 0, n_act)
                            rec["act"] = int(act)
                        elif stream == "fixed":
                            act = dict(extras["actions"][0])
                            rec["act"] = act
                        else:
                            act = dict_act(seed, call, 0)
                            rec["act"] = act
                        obs, rew, done, trunc, _ = env.step(act)
                        rec["rew"] = float(rew).hex()
                    else:
                        if stream == "discrete":
                            act = {aid: int(A.discrete_action_id(seed, call, i, n_act))
                                   for i, aid in enumerate(agent_ids)}
                        elif stream == "fixed":
                            act = {aid: dict(extras["actions"][i]) for i, aid in enumerate(agent_ids)}
                        else:
                            act = {aid: dict_act(seed, call, i) for i, aid in enumerate(agent_ids)}
                        rec["act"] = [act[a] for a in agent_ids]
                        before = list(base.agents)
                        obs, rews, dones, truncs, _ = env.step(act)
                except Exception as err:
                    if stream != "bad":
                        raise
                    # a debug env re-raises an agent's next_step error from inside World.step
                    # (core.py:96-99): record it and the state it left, then go on stepping
                    rec["raised"] = [type(err).__name__, str(err)]
                    rec["state"] = canonical_state(game, obstacles, K)
                    recs.append(rec)
                    continue
                if surface != "single":
                    rec["before"] = [agent_ids.index(a) for a in before]
                    rec["rew"] = [[agent_ids.index(a), float(r).hex()] for a, r in rews.items()]
                    done = bool(all(dones.values())) if dones else False
                    trunc = bool(all(truncs.values())) if truncs else False
                    assert set(dones.values()) <= {done} and set(truncs.values()) <= {trunc}
                elapsed += 1
                if max_steps and elapsed >= max_steps:
                    trunc = True
                rec["done"] = bool(done)
                rec["trunc"] = bool(trunc)
                if done or trunc:
                    need_reset = True
            if surface == "single":
                ob = obs_bytes_single(obs)
                rec["obs_shape"] = list(np.asarray(obs).shape)
                if call < full_calls:
                    rec["obs"] = np.asarray(obs, dtype=np.int64).ravel().tolist()
            else:
                keys, ob = obs_bytes_multi(obs, agent_ids)
                rec["obs_keys"] = [agent_ids.index(k) for k in keys]
                if call < full_calls:
                    rec["obs"] = [np.asarray(obs[k], dtype=np.int64).ravel().tolist() for k in keys]
            rec["obs_sha"] = h256(ob)
            rec["state"] = canonical_state(game, obstacles, K)
            if views:
                views.record(game, rec, rec["kind"] == "step")
            if events and rec["kind"] == "step":
                events.record(game, rec)
            recs.append(rec)
        out.append({"seed": seed, "calls": recs})
    res = {"name": name, "surface": surface, "stream": stream, "kwargs": dict(cfg[3]),
           "max_steps": max_steps, "runs": out}
    if extras:
        res["extras"] = extras
    return res
