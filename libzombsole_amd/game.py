"""`env.game` of the drop-in envs: a host view of one engine env shaped like the
reference's `Game` / `World` (`zombsole/game.py:109-201`, `zombsole/core.py:10-22`).

Nothing here runs game logic — the tick, respawn, rules and rewards all run in the HIP
engine.  `GameView` reads the env's state record (`zs_get_state`) lazily, caches it until
the env next changes, and writes pokes back through `zs_set_state`.  The rules objects
re-evaluate the reference's predicates (`rules/*.py`) on that state so that
`env.game.rules.game_won()` answers like the reference after a step.
"""
from . import _abi
from .engine import StateView
from .maps import Map, load_map  # noqa: F401  (reference: zombsole.game.Map)
from .things import OBSTACLE_CLASSES, Agent, DeadBody, ObjectiveLocation, Player, Zombie, weapon_for_code, weapon_r2

BOT_NAMES = {v: k for k, v in _abi._BOTS.items()}


class MapView(object):
    """`game.map`: the parsed map, whose `things` are this env's (shared, HP-carrying)
    obstacle objects — the same objects `world.things` holds (game.py:154-155)."""

    def __init__(self, map_, obstacles):
        self._map = map_
        self._obstacles = obstacles

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self._map, name)

    @property
    def things(self):
        return list(self._obstacles) + [ObjectiveLocation(p) for p in self._map.objectives]


class WorldView(object):
    """`core.World` attributes read by user code: size, t, deaths, zombie_deaths, things,
    decoration (core.py:12-22).  `things` is a fresh dict in the reference's insertion
    order: present obstacles in map-file order, then dynamic things in dict order.
    `decoration` is in the reference's insertion order too: the map's objectives, then every
    cell in the order a body first landed on it (core.py:24-31,121-128), the value the last body
    placed there; the order comes from the engine's per-step death log (ZS_FLAG_DEATH_LOG)."""

    def __init__(self, game):
        self._game = game
        self.size = tuple(game.map.size)
        self.debug = game.debug
        # World.event's log (core.py:68-70): (t, thing, message) per idle actor, next_step error, executed
        # action and death.  GameView.after_step queues each step's logs; the messages are formed when the
        # log is read
        self._events = []
        self._pending = []

    @property
    def events(self):
        if self._pending:
            for p in self._pending:
                self._events.extend(self._game._step_events(*p))
            self._pending = []
        return self._events

    @events.setter
    def events(self, value):
        self._pending = []
        self._events = value

    t = property(lambda s: s._game._state().t)
    deaths = property(lambda s: s._game._state().deaths)
    zombie_deaths = property(lambda s: s._game._state().zombie_deaths)

    @property
    def things(self):
        g = self._game
        st = g._state()
        out = {}
        for i, ob in enumerate(g._obstacles):
            if st.obst_present[i]:
                out[ob.position] = ob
        for slot in st.order[:st.n_order]:
            v = g._entity(int(slot))
            out[v.position] = v
        return out

    @property
    def decoration(self):
        g = self._game
        st = g._state()
        W = self.size[0]
        dead = set(st.dead_cells())
        out = {}
        for p, name in g._deco.items():
            c = p[1] * W + p[0]
            if name is None:  # an objective no body has landed on
                out[p] = ObjectiveLocation(p)
            elif c in dead:
                out[p] = DeadBody(name, p)
            dead.discard(c)
        for c in sorted(dead):  # bodies the log did not see (zs_set_state pokes)
            p = (c % W, c // W)
            out[p] = DeadBody("dead body", p)
        return out


class _Rules(object):
    """`rules/rules.py:6-18` predicates over the view."""

    def __init__(self, game):
        self.game = game

    def players_alive(self):
        return any(p.life > 0 for p in self.game.get_all_players())

    def agents_alive(self):
        return any(p.life > 0 for p in self.game.agents)


class ExterminationRules(_Rules):
    """rules/extermination.py:11-26"""

    def zombies_alive(self):
        return any(isinstance(t, Zombie) and t.life > 0 for t in self.game.world.things.values())

    def game_ended(self):
        return not self.players_alive() or not self.zombies_alive()

    def game_won(self):
        if self.players_alive():
            return True, 'zombies exterminated! :)'
        return False, 'players exterminated! :('


class SurvivalRules(_Rules):
    """rules/survival.py:5-15"""

    def game_ended(self):
        return not self.players_alive()

    def game_won(self):
        if self.players_alive():
            return True, u'you won a game that never ends (?!)'
        return False, u'everybody is dead :('


class SafeHouseRules(_Rules):
    """rules/safehouse.py:10-32"""

    def alive_players_in_house(self):
        obj = set(map(tuple, self.game.map.objectives))
        return all(p.position in obj for p in self.game.get_all_players() if p.life > 0)

    def game_ended(self):
        if self.players_alive():
            return self.alive_players_in_house()
        return True

    def game_won(self):
        if self.players_alive():
            return True, u'everybody made it into the safehouse :)'
        return False, u'nobody made it into the safehouse :('


class EvacuationRules(_Rules):
    """rules/evacuation.py:13-57"""

    def get_alive_players(self):
        return [p for p in self.game.get_all_players() if p.life > 0]

    def alive_players_together(self):
        alive = self.get_alive_players()
        by_pos = dict((p.position, p) for p in alive)
        together = set()
        pending = [alive[0]]
        while pending:
            p = pending.pop()
            together.add(id(p))
            x, y = p.position
            for q in ((x, y + 1), (x, y - 1), (x + 1, y), (x - 1, y)):
                if q in by_pos and id(by_pos[q]) not in together:
                    pending.append(by_pos[q])
        return len(together) == len(alive)

    def half_team_alive(self):
        return len(self.get_alive_players()) >= len(self.game.get_all_players()) / 2.0

    def game_ended(self):
        if self.half_team_alive():
            return self.alive_players_together()
        return True

    def game_won(self):
        if self.half_team_alive():
            return True, u'players got together and were evacuated :)'
        return False, u'too few survivors to send a rescue helicopter :('


_RULES = {"extermination": ExterminationRules, "survival": SurvivalRules,
          "evacuation": EvacuationRules, "safehouse": SafeHouseRules}


class GameView(object):
    """`game.Game` attributes (game.py:115-140): rules_name, rules, map, initial_zombies,
    minimum_zombies, debug, player_names, agent_ids, agent_weapons, world, players, agents.

    `engine` is a `libzombsole_amd.engine.Engine`; `env` the env index inside it."""

    def __init__(self, engine, env, map_, rules_name, player_names, agent_ids, agent_weapons,
                 initial_zombies, minimum_zombies, debug):
        self.engine = engine
        self.env = env
        self._obstacles = [OBSTACLE_CLASSES[k]((x, y), self, i) for i, (x, y, k) in enumerate(map_.obstacles)]
        self.map = MapView(map_, self._obstacles)
        self.rules_name = rules_name
        self.rules = _RULES[rules_name](self)
        self.player_names = list(player_names)
        self.agent_ids = list(agent_ids)
        self.agent_weapons = list(agent_weapons)
        self.initial_zombies = initial_zombies
        self.minimum_zombies = minimum_zombies
        self.debug = debug
        self._cache = None
        self.new_episode()

    # -- state cache ---------------------------------------------------------
    def invalidate(self):
        self._cache = None

    def _state(self):
        if self._cache is None:
            self._cache = self.engine.get_state(self.env)
        return self._cache

    def _poke_entity(self, slot, life):
        st = self.engine.get_state(self.env)
        st.ent[slot][4] = life
        self.engine.set_state(self.env, st)
        self._cache = None

    def _poke_obstacle(self, index, life):
        st = self.engine.get_state(self.env)
        st.obst_life[index] = life
        self.engine.set_state(self.env, st)
        self._cache = None

    # -- objects ---------------------------------------------------------------
    def end_episode(self):
        """Before a reset: every object of the ending episode keeps the values it has now.  The reference
        builds a new World and new player objects (game.py:151-169); the old objects are out of any world
        and hold their last position and life, whatever the new episode puts in the same engine slot."""
        views = getattr(self, "_views", None)
        if not views:
            return
        st = self._state()
        for slot, v in views.items():
            if v._gone:
                continue
            r = st.ent[slot]
            if int(r[7]) == v._serial:
                v._last = [int(x) for x in r]
            v._gone = True
        self._views = {}

    def new_episode(self, state_buf=None):
        """Fresh objects after a reset (the reference builds a new World and new players,
        game.py:151-169); `state_buf` is the reset's state record, when the caller has it."""
        self._cache = None if state_buf is None else StateView(self.engine, state_buf)
        # World.decoration's keys in insertion order -> the name of the body on the cell (None: the
        # objective spawned there by the map, game.py:151-155)
        self._deco = {tuple(p): None for p in self.map.objectives}
        A = len(self.agent_ids)
        self.agents = [Agent(self, i, self.agent_ids[i]) for i in range(A)]
        self.players = [Player(self, A + j, self.player_names[j]) for j in range(len(self.player_names))]
        self._views = {}
        for i, a in enumerate(self.agents):
            self._views[i] = a
        for j, p in enumerate(self.players):
            self._views[A + j] = p
        self.world = WorldView(self)

    def after_step(self, pre, rec, errors=None, raising=None):
        """Book-keeping of a step the env took (EnvCore.tick), from the state record `pre` of the world the
        step started from and the step's host record `rec`: the bodies its cleanup left, in the order it
        removed the things (core.py:121-128), the final values of the removed things into their views (a
        removed zombie's slot may be reused by the same step's respawn), the state after the step, and the
        step's World.events, queued (`errors`: the agents' next_step errors by slot; `raising`: the slot whose
        error a debug env re-raised)."""
        actors = {}
        for slot in pre.order[:pre.n_order]:  # the objects in the world while the step ran
            slot = int(slot)
            v = self._views.get(slot)
            if v is None or v._serial != int(pre.ent[slot][7]):
                v = Zombie(self, slot, row=pre.ent[slot])
                self._views[slot] = v
            actors[slot] = v
        deaths = rec.death_log()
        for slot, serial, x, y, life in deaths:
            v = self._views.get(slot)
            if v is not None and v._serial == serial:
                v._finalize(x, y, life)
            # things.py:64,118 (agents and bots always have a view; a zombie slot may have none)
            self._deco[(x, y)] = ("dead " + v.name) if isinstance(v, Player) else "zombie remains"
        post = StateView(self.engine, rec.state_buf)
        self._cache = post
        self.world._pending.append((pre, post, actors, deaths, rec.action_log(), errors or {}, raising))

    def _step_events(self, pre, post, actors, deaths, alog, errors, raising):
        """One step's World.event records (core.py:68-70) in the reference's order: for every actor in dict
        order whose next_step gave no action, 'idle', or 'error with next_step: <err>' when it raised
        (core.py:80-101; a debug env stops at the first error, core.py:96-99); each executed action's result
        in execution order (core.py:103-119, the messages of thing_move / thing_attack / thing_heal,
        core.py:140-202), with positions and occupancy followed through the step's moves; 'died' for every
        thing the cleanup removed, obstacles first in map order, then the others in dict order
        (core.py:121-138).  The actions and their order come from the engine (zs_action_log); the messages
        are their outcomes against the state from before the step."""
        t = pre.t + 1
        W, H = self.world.size
        acts, _ = alog
        ev = []
        acted = set(a[0] for a in acts)
        for slot in pre.order[:pre.n_order]:
            slot = int(slot)
            if slot in errors:
                ev.append((t, actors[slot], u"error with next_step: %s" % str(errors[slot].args[0])))
                if slot == raising:
                    return ev
            elif slot not in acted:
                ev.append((t, actors[slot], u"idle"))
        pos, occ = {}, {}
        for i, ob in enumerate(self._obstacles):
            if pre.obst_present[i]:
                occ[ob.position] = ob
        for slot, v in actors.items():
            r = pre.ent[slot]
            pos[slot] = (int(r[2]), int(r[3]))
            occ[pos[slot]] = v

        def target(tgt):
            return (self._obstacles[-1 - tgt], self._obstacles[-1 - tgt].position) if tgt < 0 else (actors[tgt], pos[tgt])

        for slot, kind, tgt in acts:
            me, (x, y) = actors[slot], pos[slot]
            if kind == 1:  # thing_move (core.py:140-166)
                dx, dy = tgt & 0xffff, tgt >> 16
                dx = dx - 0x10000 if dx >= 0x8000 else dx
                if 0 <= dx < W and 0 <= dy < H:
                    if (dx, dy) in occ:
                        msg = u"hit %s with his head" % occ[(dx, dy)].name
                    elif (dx - x) ** 2 + (dy - y) ** 2 > 1:
                        msg = u"tried to walk too fast, but physics forbade it"
                    else:
                        del occ[(x, y)]
                        occ[(dx, dy)] = me
                        pos[slot] = (dx, dy)
                        msg = u"moved to " + str((dx, dy))
                else:
                    msg = u"Tried to move out of bounds to %s" % str((dx, dy))
            elif kind == 2:  # thing_attack (core.py:168-184)
                tg, (tx, ty) = target(tgt)
                code = int(pre.ent[slot][5])
                if (tx - x) ** 2 + (ty - y) ** 2 > weapon_r2(code):
                    msg = u"tried to attack %s, but it is too far for a %s" % (tg.name, weapon_for_code(code).name)
                else:
                    msg = u"injured %s with a %s" % (tg.name, weapon_for_code(code).name)
            else:  # thing_heal (core.py:186-202), HEALING_RANGE = 3
                tg, (tx, ty) = target(tgt)
                if (tx - x) ** 2 + (ty - y) ** 2 > 9:
                    msg = u"tried to heal %s, but it is too far away" % tg.name
                else:
                    msg = u"healed " + tg.name
            ev.append((t, me, msg))
        for i, ob in enumerate(self._obstacles):
            if pre.obst_present[i] and not post.obst_present[i]:
                ev.append((t, ob, u"died"))
        for slot, serial, x, y, life in deaths:
            v = actors.get(slot)
            if v is not None and v._serial == serial:
                ev.append((t, v, u"died"))
        return ev

    def _entity(self, slot):
        v = self._views.get(slot)
        st = self._state()
        if v is not None and isinstance(v, Zombie) and v._serial != int(st.ent[slot][7]):
            v = None
        if v is None:
            v = Zombie(self, slot)
            self._views[slot] = v
        return v

    def get_all_players(self):
        return self.players + self.agents

    def get_agents_health(self):
        return sum(t.life for t in self.agents)

    def get_players_health(self):
        return sum(t.life for t in self.players)

    def draw(self):
        raise NotImplementedError("rendering is out of scope for the MI355X engine (SURVEY.md §8)")
