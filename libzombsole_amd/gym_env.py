"""Drop-in `ZombsoleGymEnv` / `ZombsoleGymEnvDiscreteAction` (zombsole/gym_env.py) on the
MI355X engine.

Same constructor arguments, attributes, return values and exceptions as the reference
(`gym_env.py:49-164`, `:327-414`); the world is one env of a `zs_handle` on the GPU and
`env.game` is a view of it (`libzombsole_amd.game`).  Every step runs in the HIP engine
(`libzombsole_amd/_build/libzombsole_mi355x.so`); constructing an env without the built
library or a visible GPU raises `EngineUnavailable`.

Randomness: like the reference, the game draws from the process-global `random` module
(see `_envcore.EnvCore`), so `random.seed(s); env.reset()` replays the reference's episode
bit for bit.  `reset(seed=...)` seeds only `self.np_random`, as gymnasium's Env.reset does in
the reference (`gym_env.py:162`).
"""
import numpy as np

from . import _abi
from ._envcore import EnvCore
from .maps import load_map
from .spaces import Box, Dict, Discrete, Env, Text, make, register, registry  # noqa: F401


class ZombsoleGymEnv(Env):
    """gym_env.py:16-233"""
    metadata = {'render.modes': ['human']}
    reward_range = (-float('inf'), float('inf'))
    action_space = Dict({
        "action_type": Text(15),
        "parameter": Box(low=-10, high=10, shape=(2,), dtype=np.int32)
    })

    def __init__(self, rules_name, player_names, map_name, agent_id, initial_zombies=0,
                 minimum_zombies=0, render_mode=None,
                 observation_scope="world", observation_position_encoding="simple",
                 agent_weapon="rifle",
                 debug=False, device=None):
        map_ = load_map(map_name)
        if render_mode is not None and (render_mode not in self.metadata['render.modes']):
            raise ValueError("render_mode={} is not supported".format(render_mode))
        self.render_mode = render_mode
        builder = _abi.single_env_config(1, rules_name, player_names, map_, agent_id,
                                         initial_zombies=initial_zombies, minimum_zombies=minimum_zombies,
                                         observation_scope=observation_scope,
                                         observation_position_encoding=observation_position_encoding,
                                         agent_weapon=agent_weapon, max_episode_steps=0,
                                         obs_dtype=_abi.DTYPE_I32, autoreset=False, debug=debug)
        cfg = builder.cfg
        # a channels observation encodes 8 + int(agent_id): the reference raises that ValueError
        # whenever it builds an observation (gym/observation.py:59-60), not at construction
        self._bad_agent_id = cfg.obs_encoding == _abi.ENC_CHANNELS and builder._ac[0] < 0
        self._agent_id = agent_id
        self._core = EnvCore(builder, builder.map, rules_name, player_names, [agent_id], [agent_weapon],
                             initial_zombies, minimum_zombies, debug, device)
        _, C, H, W = builder.obs_shape()
        high = 8 * 16 * 16 if cfg.obs_encoding == _abi.ENC_SIMPLE else 128
        # gym/observation.py:130-169
        self.observation_space = Box(low=0, high=high, shape=(C, H, W), dtype=np.int32)
        self._obs_scope = observation_scope

    @property
    def game(self):
        return self._core.game

    @property
    def engine(self):
        return self._core.engine

    def _check_id(self):
        if self._bad_agent_id:
            int(self._agent_id)

    def get_observation(self):
        self._check_id()
        return self._core.observe()[0]

    def get_frame_size(self):
        return tuple(self.observation_space.shape[1:3])

    def step(self, action):
        """gym_env.py:99-145: set_action, World.step, reward, respawn, obs, rules, end reward."""
        self.game.agents[0].set_action(action)
        r = self._core.tick([self._core.encode(action)])
        self._check_id()
        return r.obs[0], float(r.rewards[0]), r.done, r.trunc, {}

    def reset(self, seed=None, options=None):
        """gym_env.py:148-164"""
        super().reset(seed=seed)
        r = self._core.new_world()
        self._check_id()
        return r.obs[0], {}

    def render(self):
        if self.render_mode == 'human':
            raise NotImplementedError("rendering is out of scope for the MI355X engine (SURVEY.md §8)")
        raise ValueError("mode={} is not supported".format(self.render_mode))

    def close(self):
        self._core.close()

    @property
    def unwrapped(self):
        return self

    def __str__(self):
        if getattr(self, "spec", None) is None:
            return '<{} instance>'.format(type(self).__name__)
        return '<{}<{}>>'.format(type(self).__name__, self.spec.id)

    def __enter__(self):
        return self

    def __exit__(self, *args):
        self.close()
        return False


class Wrapper(Env):
    """gym_env.py:236-300"""

    def __init__(self, env):
        self.env = env
        self.action_space = self.env.action_space
        self.observation_space = self.env.observation_space
        self.reward_range = self.env.reward_range
        self.metadata = self.env.metadata
        self.render_mode = self.env.render_mode

    def __getattr__(self, name):
        if name.startswith('_'):
            raise AttributeError("attempted to get missing private attribute '{}'".format(name))
        return getattr(self.env, name)

    @property
    def spec(self):
        return self.env.spec

    @spec.setter
    def spec(self, value):
        self.env.spec = value

    @classmethod
    def class_name(cls):
        return cls.__name__

    def step(self, action):
        return self.env.step(action)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def render(self, **kwargs):
        return self.env.render(**kwargs)

    def close(self):
        return self.env.close()

    def __str__(self):
        return '<{}{}>'.format(type(self).__name__, self.env)

    def __repr__(self):
        return str(self)

    @property
    def unwrapped(self):
        return self.env.unwrapped


class ZombsoleGymEnvDiscreteAction(Wrapper):
    """gym_env.py:327-379: Discrete(6) over the moves, attack_closest and heal."""
    game_actions = [
        {'action_type': 'move', 'parameter': [0, 1]},
        {'action_type': 'move', 'parameter': [-1, 0]},
        {'action_type': 'move', 'parameter': [0, -1]},
        {'action_type': 'move', 'parameter': [1, 0]},
        {'action_type': 'attack_closest'},
        {'action_type': 'heal'},
    ]

    def __init__(self, rules_name, player_names, map_name, agent_id,
                 initial_zombies=0, minimum_zombies=0,
                 render_mode=None,
                 observation_scope="world", observation_position_encoding="simple",
                 debug=False, device=None):
        env = ZombsoleGymEnv(
            rules_name, player_names, map_name, agent_id,
            initial_zombies=initial_zombies, minimum_zombies=minimum_zombies,
            render_mode=render_mode,
            observation_scope=observation_scope, observation_position_encoding=observation_position_encoding,
            debug=debug, device=device
        )
        super().__init__(env)
        self.action_space = Discrete(len(ZombsoleGymEnvDiscreteAction.game_actions))

    def reset(self, **kwargs):
        return super().reset(**kwargs)

    def step(self, action):
        return super().step(self.action(action))

    def action(self, action):
        return self.game_actions[action]

    def reverse_action(self, action):
        return self.game_actions.index(action)


# gym_env.py:382-414
register(
    id='jvstinian/Zombsole-v0',
    entry_point='libzombsole_amd.gym_env:ZombsoleGymEnvDiscreteAction',
    max_episode_steps=1000,
    nondeterministic=True,
    kwargs={
        'rules_name': 'extermination',
        'player_names': [],
        'map_name': 'bridge',
        'agent_id': 0,
        'initial_zombies': 10,
        'minimum_zombies': 0,
        'debug': False
    }
)

register(
    id='jvstinian/Zombsole-SurroundingsView-v0',
    entry_point='libzombsole_amd.gym_env:ZombsoleGymEnvDiscreteAction',
    max_episode_steps=1000,
    nondeterministic=True,
    kwargs={
        'rules_name': 'extermination',
        'player_names': [],
        'map_name': 'bridge',
        'agent_id': 0,
        'initial_zombies': 10,
        'minimum_zombies': 0,
        'observation_scope': 'surroundings:21',
        'observation_position_encoding': 'simple',
        'debug': False
    }
)
