"""Drop-in `MultiagentZombsoleEnv` / `MultiagentZombsoleEnvDiscreteAction`
(zombsole/gym/multiagent_env.py) on the MI355X engine.

Constructor, attributes (`agents`, `possible_agents`, `action_spaces`,
`observation_spaces`, `game`), dict-shaped step/reset results and exceptions follow the
reference (`gym/multiagent_env.py:15-319`).  The world is one env of a `zs_handle`; the
tick, rewards (`gym/reward.py:67-98`), respawn, observations (int64 [3, w, w] per agent that
was alive before the step) and rules run in the HIP engine.  Randomness comes from the
process-global `random` module exactly as in the reference (see `_envcore.EnvCore`).
"""
import numpy as np

from .. import _abi
from .._envcore import EnvCore
from ..maps import load_map
from ..spaces import Box, Dict, Discrete, Text


class MultiagentZombsoleEnv(object):
    """gym/multiagent_env.py:15-205"""
    metadata = {'render.modes': ['human']}
    reward_range = (-float('inf'), float('inf'))

    def __init__(self, rules_name, player_names, map_name, agent_ids, initial_zombies=0,
                 minimum_zombies=0, render_mode=None,
                 observation_surroundings_width=21,
                 observation_position_encoding_style="channels",
                 agent_weapons="rifle",
                 debug=False, device=None):
        self.position_encoding_style = observation_position_encoding_style
        self.surroundings_width = observation_surroundings_width
        # build_surroundings_observation (gym/observation.py:205-214) validates width and style
        w = int(observation_surroundings_width)
        if (w % 2 == 0) or (w <= 1):
            raise ValueError("surroundings width must be an odd number greater than 1")
        enc = _abi.parse_encoding(observation_position_encoding_style)

        self.agents = agent_ids
        self.possible_agents = agent_ids
        self.action_spaces = {
            agent_id: Dict({
                "action_type": Text(15),
                "parameter": Box(low=-10, high=10, shape=(2,), dtype=np.int32)
            })
            for agent_id in self.possible_agents
        }
        high = 8 * 16 * 16 if enc == _abi.ENC_SIMPLE else 128
        self.observation_spaces = {
            agent_id: Box(low=0, high=high, shape=(3 if enc == _abi.ENC_CHANNELS else 1, w, w), dtype=np.int32)
            for agent_id in self.possible_agents
        }

        map_ = load_map(map_name)
        if render_mode is not None and (render_mode not in self.metadata['render.modes']):
            raise ValueError("render_mode={} is not supported".format(render_mode))
        self.render_mode = render_mode

        builder = _abi.multi_env_config(1, rules_name, player_names, map_, agent_ids,
                                        initial_zombies=initial_zombies, minimum_zombies=minimum_zombies,
                                        observation_surroundings_width=w,
                                        observation_position_encoding_style=observation_position_encoding_style,
                                        agent_weapons=agent_weapons, max_episode_steps=0,
                                        obs_dtype=_abi.DTYPE_I64, autoreset=False, debug=debug)
        names = _abi.expand_weapons(agent_weapons, len(agent_ids))
        self._simple = enc == _abi.ENC_SIMPLE
        self._ids = list(agent_ids)[:len(names)]
        self._bad_ids = [a for a, c in zip(self._ids, builder._ac) if c < 0]
        self._core = EnvCore(builder, builder.map, rules_name, player_names, self._ids, names,
                             initial_zombies, minimum_zombies, debug, device)
        self.frames_per_second = None

    @property
    def game(self):
        return self._core.game

    @property
    def engine(self):
        return self._core.engine

    def _observations(self, obs):
        if self._simple:
            # SurroundingsSimpleObservation has no get_observation_at_position
            raise AttributeError("'SurroundingsSimpleObservation' object has no attribute "
                                 "'get_observation_at_position'")
        for a in self._bad_ids:
            if a in self.agents:
                int(a)  # gym/observation.py:59-60 raises this ValueError
        ret = {}
        for i, aid in enumerate(self._ids):
            if aid in self.agents:  # alive before the step (multiagent_env.py:87-96)
                ret[aid] = obs[i]
        return ret

    def get_observation(self):
        return self._observations(self._core.observe())

    def _process_single_agent_action(self, sp_action):
        coords = sp_action.get("parameter", [0, 0])
        return {"action_type": sp_action["action_type"], "parameter": coords}

    def _process_action(self, actions):
        return {agent_id: self._process_single_agent_action(v) for agent_id, v in actions.items()}

    def step(self, action):
        """gym/multiagent_env.py:111-171"""
        agent_actions = self._process_action(action)
        triples = []
        for agent in self.game.agents:
            agent_action = agent_actions.get(agent.agent_id, {"action_type": "heal", "parameter": [0, 0]})
            agent.set_action(agent_action)
            triples.append(self._core.encode(agent_action))
        r = self._core.tick(triples)

        rewards = {}
        for i, aid in enumerate(self._ids):
            if aid in self.agents:
                rewards[aid] = float(r.rewards[i])
        observations = self._observations(r.obs)
        done = {agent_id: r.done for agent_id in self.agents}
        truncated = {agent_id: r.trunc for agent_id in self.agents}
        self.agents = [agent.agent_id for agent in self.game.agents if agent.life > 0]
        return observations, rewards, done, truncated, {}

    def reset(self, seed=None, options=None):
        """gym/multiagent_env.py:173-184"""
        self.agents = self.possible_agents
        r = self._core.new_world()
        return self._observations(r.obs), {}

    def render(self):
        if self.render_mode == 'human':
            raise NotImplementedError("rendering is out of scope for the MI355X engine (SURVEY.md §8)")
        raise ValueError("mode={} is not supported".format(self.render_mode))

    def close(self):
        self._core.close()

    def __str__(self):
        return '<{} instance>'.format(type(self).__name__)

    def __enter__(self):
        return self

    def __exit__(self, *args):
        self.close()
        return False


class MultiAgentWrapper(object):
    """gym/multiagent_env.py:207-254"""

    def __init__(self, env):
        self.env = env
        self.action_spaces = self.env.action_spaces
        self.observation_spaces = self.env.observation_spaces
        self.reward_range = self.env.reward_range
        self.metadata = self.env.metadata
        self.render_mode = self.env.render_mode

    @classmethod
    def class_name(cls):
        return cls.__name__

    def step(self, action):
        return self.env.step(action)

    def reset(self, seed=None, options=None):
        return self.env.reset(seed=seed, options=options)

    def render(self):
        return self.env.render()

    def close(self):
        self.env.close()

    def __str__(self):
        return '<{}{}>'.format(type(self).__name__, self.env)


class MultiagentZombsoleEnvDiscreteAction(MultiAgentWrapper):
    """gym/multiagent_env.py:256-319: Discrete(7), adds heal_closest."""
    game_actions = [
        {'action_type': 'move', 'parameter': [0, 1]},
        {'action_type': 'move', 'parameter': [-1, 0]},
        {'action_type': 'move', 'parameter': [0, -1]},
        {'action_type': 'move', 'parameter': [1, 0]},
        {'action_type': 'attack_closest'},
        {'action_type': 'heal'},
        {'action_type': 'heal_closest'},
    ]

    def __init__(self, rules_name, player_names, map_name, agent_ids,
                 initial_zombies=0, minimum_zombies=0,
                 render_mode=None,
                 observation_surroundings_width=21,
                 agent_weapons="rifle",
                 debug=False, device=None):
        env = MultiagentZombsoleEnv(
            rules_name, player_names, map_name, agent_ids,
            initial_zombies=initial_zombies, minimum_zombies=minimum_zombies,
            render_mode=render_mode,
            observation_surroundings_width=observation_surroundings_width,
            agent_weapons=agent_weapons,
            debug=debug, device=device
        )
        super().__init__(env)
        self.action_spaces = {
            agent_id: Discrete(len(MultiagentZombsoleEnvDiscreteAction.game_actions))
            for agent_id in self.env.possible_agents
        }

    def step(self, actions):
        return super().step(self.actions(actions))

    def actions(self, actions):
        return {agent_id: self.game_actions[action] for agent_id, action in actions.items()}

    def reverse_actions(self, actions):
        return {agent_id: self.game_actions.index(action) for agent_id, action in actions.items()}
