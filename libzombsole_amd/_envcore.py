"""Shared plumbing of the drop-in envs: one engine env on the GPU driven with the
process-global `random` stream.

The reference's game draws every random number from CPython's module-global `random`
(`zombsole/core.py:2`, `things.py:2`, `weapons.py:2`, `players/*.py`), so two envs in one
process interleave on one stream and `random.seed(s)` before construction / `reset()`
fixes an episode.  `EnvCore` keeps exactly that contract: around every engine call it
moves `random.getstate()` into the env's MT19937 slot (`zs_set_rng`) and the advanced
state back out (`zs_get_rng` -> `random.setstate`).  The tick itself always runs in the
HIP engine; there is no host fallback.
"""
import random

import numpy as np

from . import _abi
from .actions import ACT_RAISE, ActionError, encode_action
from .engine import Engine
from .game import GameView


class EnvCore(object):
    def __init__(self, builder, map_, rules_name, player_names, agent_ids, agent_weapons, initial_zombies,
                 minimum_zombies, debug, device=None):
        # the per-step death log feeds the views' decoration order and removed things (game.py)
        builder.cfg.flags |= _abi.FLAG_DEATH_LOG
        self.engine = Engine(builder, device=device)
        self.torch = self.engine.torch
        self.debug = debug
        self.game = GameView(self.engine, 0, map_, rules_name, player_names, agent_ids, agent_weapons,
                             initial_zombies, minimum_zombies, debug)
        self._host_actions = np.zeros((1, self.engine.A, 3), dtype=np.int32)
        self.new_world(first=True)

    # Game.__initialize_world__ (game.py:151-169) on the engine, drawing from `random`
    def new_world(self, first=False):
        eng = self.engine
        if not first:
            self.game.end_episode()  # objects of the ending episode keep their values
        eng.load_python_random(0)
        try:
            eng.reset()
        finally:
            eng.store_python_random(0)
        self.game.new_episode()

    def encode(self, action):
        """Agent.next_step's parse of one action dict; errors as World.get_actions treats them
        (core.py:96-99): with debug the agent's action becomes ZS_ACT_RAISE (the tick stops there
        and `tick` re-raises the exception), otherwise the agent idles."""
        try:
            return encode_action(action)
        except ActionError as err:
            if self.debug:
                return err
            return (0, 0, 0)

    def tick(self, triples):
        """One World.step + env glue for the single engine env; returns host copies of
        (obs[n_obs, C, H, W], rewards[A], done, truncated).

        An entry of `triples` may be the ActionError `encode` returned for a debug env: the engine
        then runs World.step up to the first such agent in dict order — t += 1 and the decisions
        (RNG draws included) of the actors before it — and this re-raises that agent's exception,
        as the reference's World.step does (core.py:72-78, 96-99).  Agents that are not in the
        world are never asked for an action, so their errors do not raise."""
        eng = self.engine
        errors = {i: t for i, t in enumerate(triples) if isinstance(t, ActionError)}
        raising = None
        if errors:
            st = eng.get_state(0)
            for slot in st.order[:st.n_order]:
                if int(slot) in errors:
                    raising = errors[int(slot)]
                    break
        rows = [(ACT_RAISE, 0, 0) if isinstance(t, ActionError) else t for t in triples]
        self._host_actions[0, :len(rows)] = np.asarray(rows, dtype=np.int32).reshape(-1, 3)
        eng.actions.copy_(self.torch.from_numpy(self._host_actions))
        pre = self.game._state()  # the world the step starts from (its World.events are derived from it)
        eng.load_python_random(0)
        try:
            eng.step()
        finally:
            eng.store_python_random(0)
            self.game.invalidate()
        # a debug raise stops World.step inside get_actions: no action ran, nothing died (core.py:96-99)
        self.game.after_step(None if raising is not None else pre)
        if raising is not None:
            raise raising.args[0]
        obs = eng.obs[0].cpu().numpy()
        rew = eng.rewards[0].cpu().numpy()
        return obs, rew, bool(eng.done[0].item()), bool(eng.trunc[0].item())

    def observe(self):
        eng = self.engine
        eng.observe()
        return eng.obs[0].cpu().numpy()

    def close(self):
        self.engine.close()


def obs_np_dtype(builder):
    return _abi.DTYPE_NP[builder.cfg.obs_dtype]
