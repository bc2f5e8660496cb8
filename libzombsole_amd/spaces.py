"""gymnasium spaces / Env / registry, or a minimal local stand-in when gymnasium is absent.

The reference's envs subclass `gymnasium.core.Env` and use `Text`, `Box`, `Dict`,
`Discrete` and `register` (`zombsole/gym_env.py:4-7`, `gym/multiagent_env.py:3-5`).
When gymnasium is importable it is used as-is; otherwise (this image) the classes below
provide the parts of that API the envs and their users touch: `sample()`, `seed()`,
`contains()`, `n`, `shape`, `dtype`, `low`/`high`, plus a registry with `make()` that
applies the registration's `max_episode_steps` through a TimeLimit wrapper.
"""
import numpy as np

try:  # pragma: no cover - gymnasium is not installed in this image
    import gymnasium as _gym
    from gymnasium.core import Env
    from gymnasium.envs.registration import register as _gym_register
    from gymnasium.spaces import Box, Dict, Discrete, Sequence, Text
    HAVE_GYMNASIUM = True
except ImportError:
    _gym = None
    HAVE_GYMNASIUM = False

    class Space(object):
        def __init__(self, shape=None, dtype=None, seed=None):
            self.shape = shape
            self.dtype = None if dtype is None else np.dtype(dtype)
            self._np_random = None
            if seed is not None:
                self.seed(seed)

        @property
        def np_random(self):
            if self._np_random is None:
                self.seed()
            return self._np_random

        def seed(self, seed=None):
            self._np_random = np.random.default_rng(seed)
            return [seed]

        def __contains__(self, x):
            return self.contains(x)

    class Discrete(Space):
        def __init__(self, n, seed=None, start=0):
            super().__init__((), np.int64, seed)
            self.n = int(n)
            self.start = int(start)

        def sample(self, mask=None):
            return int(self.start + self.np_random.integers(self.n))

        def contains(self, x):
            try:
                v = int(x)
            except (TypeError, ValueError):
                return False
            return v == x and self.start <= v < self.start + self.n

        def __repr__(self):
            return "Discrete(%d)" % self.n

        def __eq__(self, other):
            return isinstance(other, Discrete) and other.n == self.n and other.start == self.start

    class Box(Space):
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            shape = tuple(shape) if shape is not None else np.shape(low)
            super().__init__(shape, dtype, seed)
            self.low = np.full(shape, low, dtype=self.dtype)
            self.high = np.full(shape, high, dtype=self.dtype)

        def sample(self, mask=None):
            if np.issubdtype(self.dtype, np.integer):
                return self.np_random.integers(self.low, self.high.astype(np.int64) + 1, size=self.shape).astype(
                    self.dtype)
            return self.np_random.uniform(self.low, self.high, size=self.shape).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

        def __repr__(self):
            return "Box(%s, %s, %s, %s)" % (self.low.min(), self.high.max(), self.shape, self.dtype)

    class Text(Space):
        CHARSET = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_"

        def __init__(self, max_length, min_length=1, charset=None, seed=None):
            super().__init__((), str, seed)
            self.max_length = int(max_length)
            self.min_length = int(min_length)
            self.charset = charset or self.CHARSET

        def sample(self, mask=None):
            n = int(self.np_random.integers(self.min_length, self.max_length + 1))
            return "".join(self.charset[int(i)] for i in self.np_random.integers(len(self.charset), size=n))

        def contains(self, x):
            return isinstance(x, str) and self.min_length <= len(x) <= self.max_length

    class Dict(Space):
        def __init__(self, spaces=None, seed=None, **kw):
            super().__init__(None, None, None)
            self.spaces = dict(spaces or {}, **kw)
            if seed is not None:
                self.seed(seed)

        def seed(self, seed=None):
            super().seed(seed)
            for i, sp in enumerate(self.spaces.values()):
                sp.seed(None if seed is None else seed + i)
            return [seed]

        def sample(self, mask=None):
            return {k: sp.sample() for k, sp in self.spaces.items()}

        def contains(self, x):
            return isinstance(x, dict) and all(k in x and sp.contains(x[k]) for k, sp in self.spaces.items())

        def __getitem__(self, k):
            return self.spaces[k]

    class Sequence(Space):
        def __init__(self, space, seed=None):
            super().__init__(None, None, seed)
            self.feature_space = space

        def sample(self, mask=None):
            return tuple(self.feature_space.sample() for _ in range(int(self.np_random.integers(0, 5))))

        def contains(self, x):
            return isinstance(x, tuple) and all(self.feature_space.contains(v) for v in x)

    class Env(object):
        """The subset of gymnasium.core.Env the envs rely on."""
        metadata = {"render_modes": []}
        render_mode = None
        reward_range = (-float("inf"), float("inf"))
        spec = None
        _np_random = None

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = np.random.default_rng()
            return self._np_random

        def reset(self, *, seed=None, options=None):
            if seed is not None:
                self._np_random = np.random.default_rng(seed)

        @property
        def unwrapped(self):
            return self

        def close(self):
            pass

    _gym_register = None


class EnvSpec(object):
    def __init__(self, id, entry_point, max_episode_steps=None, nondeterministic=False, kwargs=None):
        self.id = id
        self.entry_point = entry_point
        self.max_episode_steps = max_episode_steps
        self.nondeterministic = nondeterministic
        self.kwargs = dict(kwargs or {})


registry = {}


def register(id, entry_point, max_episode_steps=None, nondeterministic=False, kwargs=None):
    """`gymnasium.envs.registration.register` (local registry when gymnasium is absent)."""
    if _gym_register is not None:  # pragma: no cover
        _gym_register(id=id, entry_point=entry_point, max_episode_steps=max_episode_steps,
                      nondeterministic=nondeterministic, kwargs=kwargs)
    registry[id] = EnvSpec(id, entry_point, max_episode_steps, nondeterministic, kwargs)


class TimeLimit(object):
    """gymnasium.wrappers.TimeLimit: truncated=True once `max_episode_steps` steps ran."""

    def __init__(self, env, max_episode_steps):
        self.env = env
        self._max_episode_steps = max_episode_steps
        self._elapsed_steps = None

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    def step(self, action):
        obs, rew, term, trunc, info = self.env.step(action)
        self._elapsed_steps += 1
        if self._elapsed_steps >= self._max_episode_steps:
            trunc = True
        return obs, rew, term, trunc, info

    def reset(self, **kwargs):
        self._elapsed_steps = 0
        return self.env.reset(**kwargs)

    @property
    def unwrapped(self):
        return self.env.unwrapped


def make(id, **kwargs):
    """`gymnasium.make` for the ids registered here."""
    if HAVE_GYMNASIUM:  # pragma: no cover
        return _gym.make(id, **kwargs)
    spec = registry[id]
    mod, _, attr = spec.entry_point.partition(":")
    import importlib
    cls = getattr(importlib.import_module(mod), attr)
    kw = dict(spec.kwargs)
    kw.update(kwargs)
    env = cls(**kw)
    env.spec = spec
    if spec.max_episode_steps:
        env = TimeLimit(env, spec.max_episode_steps)
    return env
