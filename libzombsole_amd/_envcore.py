"""Shared plumbing of the drop-in envs: one engine env on the GPU driven with the
process-global `random` stream.

The reference's game draws every random number from CPython's module-global `random`
(`zombsole/core.py:2`, `things.py:2`, `weapons.py:2`, `players/*.py`), so two envs in one
process interleave on one stream and `random.seed(s)` before construction / `reset()`
fixes an episode.  `EnvCore` keeps exactly that contract: every engine call takes
`random.getstate()` into the env's MT19937 stream and hands the advanced stream back
(`random.setstate`).  The tick itself always runs in the HIP engine; there is no host
fallback.

A call is one `zs_host_step` / `zs_host_reset` / `zs_host_observe` (include/zombsole_mi355x.h):
the actions and the `random` state go in with one copy, and one record comes back with one
copy and one synchronisation — the observation, rewards and flags, the advanced stream, the
step's action and death logs and the env's state record, which `env.game` then reads without
another device round trip.
"""
import random
import struct

import numpy as np

from . import _abi
from .actions import ACT_RAISE, ActionError, encode_action
from .engine import Engine, decode_action_log, decode_death_log
from .game import GameView

HOST_FLAGS, HOST_ERR, HOST_ALOG_N, HOST_DLOG_N, HOST_RNG = 0, 1, 2, 3, 4  # ZS_HOST_* header words
MT_WORDS = 625
_MT = struct.Struct("<625I")  # random.getstate()[1] <-> the engine's 625 uint32 words


class HostRecord(object):
    """One env's zs_host_* record (layout: zs_host_layout)."""

    def __init__(self, eng, rec, lay, obs_dtype):
        self.rec = rec
        self.lay = lay
        self.E = eng.E
        self.flags = int(rec[HOST_FLAGS])
        self.done = bool(self.flags & 1)
        self.trunc = bool(self.flags & 2)
        self.rewards = rec[lay["rew"]:lay["rew"] + 2 * lay["R"]].view(np.float64)
        ob = lay["obs"]
        nbytes = lay["obs_bytes"]
        self.obs = rec[ob:ob + (nbytes + 3) // 4].view(np.uint8)[:nbytes].view(obs_dtype).reshape(eng.obs_shape)
        self.state_buf = rec[lay["state"]:lay["state"] + eng.state_words]

    def rng_state(self):
        """The env's stream after the call, as a random.setstate() argument."""
        return (3, _MT.unpack_from(self.rec, 4 * HOST_RNG), None)

    def rng_bytes(self):
        """The same stream as the packed words EnvCore._rng_in produces."""
        return self.rec[HOST_RNG:HOST_RNG + MT_WORDS].tobytes()

    def action_log(self):
        return decode_action_log(self.rec[self.lay["alog"]:], int(self.rec[HOST_ALOG_N]), self.E)

    def death_log(self):
        return decode_death_log(self.rec[self.lay["dlog"]:], int(self.rec[HOST_DLOG_N]), self.E)


class EnvCore(object):
    def __init__(self, builder, map_, rules_name, player_names, agent_ids, agent_weapons, initial_zombies,
                 minimum_zombies, debug, device=None):
        # the per-step death / action logs feed the views' decoration order, removed things and World.events
        builder.cfg.flags |= _abi.FLAG_DEATH_LOG
        self.engine = Engine(builder, device=device)
        self.torch = self.engine.torch
        self.debug = debug
        self._lay = self.engine.host_layout()
        self._np_obs = _abi.DTYPE_NP[builder.cfg.obs_dtype]
        self._actions = np.zeros((1, self.engine.A, 3), dtype=np.int32)
        self.last = None  # the last call's HostRecord
        self._rng_last = None  # its stream, packed
        self.game = GameView(self.engine, 0, map_, rules_name, player_names, agent_ids, agent_weapons,
                             initial_zombies, minimum_zombies, debug)
        self.new_world(first=True)

    @staticmethod
    def _rng_in():
        return _MT.pack(*random.getstate()[1])

    def _record(self, rec):
        self.last = HostRecord(self.engine, rec[0], self._lay, self._np_obs)
        self._rng_last = self.last.rng_bytes()
        return self.last

    # Game.__initialize_world__ (game.py:151-169) on the engine, drawing from `random`
    def new_world(self, first=False):
        eng = self.engine
        if not first:
            self.game.end_episode()  # objects of the ending episode keep their values
        rec = eng.host_record()
        try:
            eng.host_reset(self._rng_in(), rec)
        except Exception as err:
            if type(err) is not Exception:
                raise
            # ZS_ENOSPACE: the draws were taken, as in the reference, which raises naming the first thing it
            # could not place (core.py:58-64): players spawn first, then agents, on the same spawn cells
            random.setstate(HostRecord(eng, rec[0], self._lay, self._np_obs).rng_state())
            raise Exception("Not enough space to spawn %s" % self._unplaced()) from None
        r = self._record(rec)
        random.setstate(r.rng_state())
        self.game.new_episode(r.state_buf)
        return r

    def _unplaced(self):
        """The name of the first thing a reset cannot place (game.py:181-187, core.py:40-66): every spawn cell
        is free at a reset (the map's obstacles stand on other cells; with no spawn cells listed, every cell
        but an obstacle's), the players take them first, then the agents."""
        m = self.game.map
        free = len(m.player_spawns) if m.player_spawns else m.size[0] * m.size[1] - len(m.obstacles)
        names = self.game.player_names
        return names[free] if free < len(names) else "agent"

    def encode(self, action):
        """Agent.next_step's parse of one action dict: an engine triple, or the ActionError the reference's
        next_step raises for it (World.get_actions then logs it and, with debug, re-raises it;
        core.py:96-99)."""
        try:
            return encode_action(action)
        except ActionError as err:
            return err

    def tick(self, triples):
        """One World.step + env glue for the single engine env; returns the call's HostRecord (obs
        [n_obs, C, H, W], rewards [R], done, trunc).

        An entry of `triples` may be the ActionError `encode` returned.  Without debug the agent idles and
        World.events logs its error (core.py:96-97).  With debug the engine runs World.step up to the first
        such agent in dict order — t += 1 and the decisions (RNG draws included) of the actors before it —
        and this re-raises that agent's exception, as the reference's World.step does (core.py:72-78,
        96-99).  Agents that are not in the world are never asked for an action, so their errors do not
        raise."""
        eng = self.engine
        errors = {i: t for i, t in enumerate(triples) if isinstance(t, ActionError)}
        pre = self.game._state()  # the world the step starts from (its World.events are derived from it)
        raising = None
        if errors and self.debug:
            for slot in pre.order[:pre.n_order]:
                if int(slot) in errors:
                    raising = int(slot)
                    break
        act = self._actions[0]
        for i, t in enumerate(triples):
            act[i] = (ACT_RAISE if self.debug else 0, 0, 0) if i in errors else t
        rec = eng.host_record()
        rng = self._rng_in()
        # the stream the engine already holds (nothing drew from `random` since the last call): not moved in
        eng.host_step(self._actions, None if rng == self._rng_last else rng, rec)
        r = self._record(rec)
        random.setstate(r.rng_state())
        self.game.after_step(pre, r, errors, raising)
        if raising is not None:
            raise errors[raising].args[0]
        return r

    def observe(self):
        rec = self.engine.host_record()
        self.engine.host_observe(rec)
        return HostRecord(self.engine, rec[0], self._lay, self._np_obs).obs

    def close(self):
        self.engine.close()


def obs_np_dtype(builder):
    return _abi.DTYPE_NP[builder.cfg.obs_dtype]
