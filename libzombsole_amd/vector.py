"""Batched device API: N lock-step envs of one surface on one GPU, env-sharded across ranks.

This is the throughput path (`bench.py`).  The drop-in classes in
`gym_env` / `gym.multiagent_env` drive one env each through the same engine; here the
caller hands whole-batch device tensors in and gets device tensors back:

    venv = BatchedZombsole("multi", 8192, rules_name="extermination", player_names=[],
                           map_name="bridge64", agent_ids=["0", "1"], initial_zombies=10,
                           max_episode_steps=1000, base_seed=0, env0=rank * 8192)
    obs = venv.reset()                                  # [N, A, 3, 21, 21] on the GPU
    obs, rew, done, trunc = venv.step(actions)          # actions int32 [N, A, 3] or ids [N, A]

Envs are independent: rank r of G owns global envs [r*N/G, (r+1)*N/G) and env i is seeded
`base_seed + i` (CPython random.seed semantics per env), so every env's trajectory is the
same whatever G is.  Done/truncated envs are reset by the next step (autoreset); the
`was_reset` tensor flags them.  The only collective is the optional observation gather
for a centralised learner (`gather_observations`, RCCL all-gather over xGMI).
"""
from . import _abi
from .actions import DISCRETE_TRIPLES
from .engine import Engine


def shard_range(total_envs, rank, world):
    """(first global env, count) of `rank`'s shard; contiguous, sizes differ by <= 1."""
    base, extra = divmod(int(total_envs), int(world))
    n = base + (1 if rank < extra else 0)
    env0 = rank * base + min(rank, extra)
    return env0, n


class BatchedZombsole(object):
    def __init__(self, surface, num_envs, rules_name, player_names, map_name, agent_ids=None, agent_id=0,
                 initial_zombies=0, minimum_zombies=0, max_episode_steps=0, base_seed=0, env0=0,
                 observation_scope="world", observation_position_encoding="simple", agent_weapon="rifle",
                 observation_surroundings_width=21, observation_position_encoding_style="channels",
                 agent_weapons="rifle", obs_dtype=None, autoreset=True, device=None, lanes_per_env=0):
        if surface == "single":
            b = _abi.single_env_config(num_envs, rules_name, player_names, map_name, agent_id, initial_zombies,
                                       minimum_zombies, observation_scope, observation_position_encoding,
                                       agent_weapon, max_episode_steps,
                                       _abi.DTYPE_I32 if obs_dtype is None else obs_dtype, autoreset, lanes_per_env)
        elif surface == "multi":
            b = _abi.multi_env_config(num_envs, rules_name, player_names, map_name, agent_ids, initial_zombies,
                                      minimum_zombies, observation_surroundings_width,
                                      observation_position_encoding_style, agent_weapons, max_episode_steps,
                                      _abi.DTYPE_I64 if obs_dtype is None else obs_dtype, autoreset, lanes_per_env)
        else:
            raise ValueError("surface must be 'single' or 'multi'")
        self.surface = surface
        self.engine = Engine(b, device=device)
        self.torch = self.engine.torch
        self.num_envs = int(num_envs)
        self.env0 = int(env0)
        self.base_seed = int(base_seed)
        self.engine.seed([self.base_seed + self.env0 + i for i in range(self.num_envs)])
        self._triples = self.torch.from_numpy(DISCRETE_TRIPLES).to(self.engine.device)
        self.n_discrete = 7 if surface == "multi" else 6

    @property
    def obs(self):
        return self.engine.obs

    @property
    def was_reset(self):
        return self.engine.was_reset

    @property
    def listed(self):
        return self.engine.listed

    def reset(self, mask=None):
        return self.engine.reset(mask)

    def discrete_to_triples(self, ids):
        """Discrete(6)/(7) ids [N, A] (gym_env.py:328-351, gym/multiagent_env.py:259-285) -> [N, A, 3]."""
        return self._triples[ids.long()]

    def step(self, actions):
        t = self.torch
        if actions.dim() == 2:
            actions = self.discrete_to_triples(actions)
        if actions.dtype != t.int32 or not actions.is_contiguous():
            actions = actions.to(t.int32).contiguous()
        return self.engine.step(actions)

    def sample_actions(self, step):
        """The bench/parity uniform policy, generated on device (zs_gen_actions)."""
        return self.engine.gen_actions(step, self.n_discrete)

    def close(self):
        self.engine.close()


def gather_observations(obs, group=None):
    """All-gather every rank's observation shard into one [G*N, ...] tensor.

    Over RCCL on MI355X this is one all_gather_into_tensor of the compact obs; with gloo
    (CPU tests) the same call runs on host tensors."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty((world * obs.shape[0],) + tuple(obs.shape[1:]), dtype=obs.dtype, device=obs.device)
    if dist.get_backend(group) == "gloo":
        parts = list(out.chunk(world, dim=0))
        dist.all_gather(parts, obs.contiguous(), group=group)
        out = torch.cat(parts, dim=0)
    else:
        dist.all_gather_into_tensor(out, obs.contiguous(), group=group)
    return out
