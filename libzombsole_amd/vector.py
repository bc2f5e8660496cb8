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

    @property
    def actions(self):
        """The engine's action buffer, int32 [N, A, 3]: a caller that writes its actions here (e.g.
        `torch.index_select(..., out=venv.actions.view(-1, 3))`) saves step()'s copy."""
        return self.engine.actions

    def step(self, actions, graph=True):
        """One tick of every env on the caller's actions (int32 [N, A, 3] triples, or Discrete ids
        [N, A]), as MultiagentZombsoleEnv.step / ZombsoleGymEnv.step do per env
        (gym/multiagent_env.py:111-171, gym_env.py:99-145).  graph=True replays the step as one hipGraph
        launch reading the engine's action buffer (Engine.step_graphed); graph=False dispatches its
        kernels one by one (zs_step)."""
        t = self.torch
        if actions.dim() == 2:
            actions = self.discrete_to_triples(actions)
        if not graph:
            if actions.dtype != t.int32 or not actions.is_contiguous():
                actions = actions.to(t.int32).contiguous()
            return self.engine.step(actions)
        buf = self.engine.actions
        if actions.data_ptr() != buf.data_ptr():
            buf.copy_(actions)
        return self.engine.step_graphed(buf)

    def sample_actions(self, step):
        """The bench/parity uniform policy, generated on device (zs_gen_actions)."""
        return self.engine.gen_actions(step, self.n_discrete)

    def close(self):
        self.engine.close()


def _gather_sizes(n_local, device, group):
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    t = torch.tensor([int(n_local)], dtype=torch.int64, device=device)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    return [int(p.item()) for p in parts]


def _all_gather_rows(out, x, group):
    """out[r*m:(r+1)*m] = rank r's x (every rank's x has m rows).

    RCCL has no int16 type (the compact C5 observations): such tensors travel as their bytes."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo":
        dist.all_gather(list(out.chunk(dist.get_world_size(group), dim=0)), x, group=group)
        return
    if x.dtype in (torch.int16, torch.uint16, torch.bool):
        out, x = out.view(torch.uint8), x.view(torch.uint8)
    dist.all_gather_into_tensor(out, x, group=group)


def gather_observations(obs, group=None, sizes=None):
    """All-gather every rank's observation shard into one [sum(N_r), ...] tensor in global env
    order.

    Shards from `shard_range` differ by at most one env: short shards are padded to the longest, so
    every rank issues one equal-sized collective.  `sizes` (every rank's shard size, e.g. from
    shard_range) saves a size exchange and its host sync per call; per-step callers should use
    StepGather, which also overlaps the exchange with the next step.  Over RCCL on MI355X it is one
    all_gather_into_tensor; with gloo (CPU tests) the same call on host tensors."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if sizes is None:
        sizes = _gather_sizes(obs.shape[0], obs.device, group)
    sizes = [int(v) for v in sizes]
    m = max(sizes)
    x = obs.contiguous()
    if x.shape[0] < m:
        x = torch.cat([x, x.new_zeros((m - x.shape[0],) + tuple(x.shape[1:]))], dim=0)
    out = torch.empty((world * m,) + tuple(obs.shape[1:]), dtype=obs.dtype, device=obs.device)
    _all_gather_rows(out, x, group)
    if all(n == m for n in sizes):
        return out
    return torch.cat([out[r * m:r * m + n] for r, n in enumerate(sizes)], dim=0)


class StepGather(object):
    """C5's per-step exchange for a centralised learner, overlapped with the next
    step's compute.

    Every rank's observation shard plus its rewards / done / truncated / listed / was_reset are
    all-gathered into node-wide tensors (obs + reward + done/trunc/alive; `listed` says
    which agents' rewards and observations are valid — the agents alive before the step, whose keys the
    reference's dicts carry, gym/multiagent_env.py:156-169 — and `was_reset` which observations are a reset's).
    The engine writes each step into one of `depth` output sets (Engine.outputs) whose storage
    is this rank's slice of that set's gather buffers, padded to the longest shard, so the exchange copies
    nothing: the collectives run in place (a rank receives the other ranks' slices only), the observations
    one collective and the rest (one flat byte tensor per set, engine.StepOutputs) a second.  Step t
    writes set t % depth on the caller's stream; its collectives are issued on a communication stream
    that waits for that step only, so they run while step t + 1 computes into the next set; before a
    set is written again the caller's stream waits for the collectives that read it.  With gloo (CPU
    tensors) everything is synchronous.

        g = StepGather(eng)
        g.step(lambda out: eng.step_graph(t, 7, out=out))   # per step
        g.obs(), g.rewards(), g.done(), g.truncated()      # the last step's node-wide tensors
        g.listed(), g.was_reset()

    The tensors obs() returns are the exchange buffers themselves when every shard has the same size
    (no copy): they hold step t's values until the exchange of step t + depth overwrites them, and are
    ordered on the current stream only (obs(copy=True) returns a copy).  A consumer that reads a step's
    gathered values on the communication stream instead (a learner overlapping with the next step)
    passes after=fn to step(): fn(k) runs there right after the collectives that fill set k.
    """

    def __init__(self, engine, group=None, depth=2, self_exchange=False):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.eng = engine
        self.group = group
        self.world = dist.get_world_size(group)
        self.n = engine.N
        self.sizes = _gather_sizes(self.n, engine.device, group)  # once: shards keep their size
        self.m = max(self.sizes)
        self.R = engine.A if engine.multi else 1
        self.depth = int(depth)
        dev = engine.device
        rank = dist.get_rank(group)
        shape = tuple(engine.obs_shape)
        self.A = engine.A
        # a rank's segment of the flat exchange buffer (engine.StepOutputs); the float64 rewards 8-B aligned
        nflat = (self.m * (8 * self.R + 3 + self.A) + 15) // 16 * 16
        self.g_obs = [torch.zeros((self.world * self.m,) + shape, dtype=engine.obs_dtype, device=dev)
                      for _ in range(self.depth)]
        self.g_flat = [torch.zeros(self.world * nflat, dtype=torch.uint8, device=dev) for _ in range(self.depth)]
        # the engine's output sets are this rank's slices of the gather buffers (in-place collectives)
        self.sets = [engine.outputs(rows=self.m, obs=self.g_obs[k][rank * self.m:(rank + 1) * self.m],
                                    flat=self.g_flat[k][rank * nflat:(rank + 1) * nflat]) for k in range(self.depth)]
        cuda = dev.type == "cuda"
        self.comm = torch.cuda.Stream(device=dev) if cuda else None
        self.pending = [None] * self.depth  # per set: event after the collectives that read it
        # world size 1: the output sets are the whole gather buffers, so the gathered tensors are already
        # complete and the collectives are skipped (self_exchange=True issues them anyway: diagnostics of
        # the exchange's fixed cost)
        self.skip = self.world == 1 and not self_exchange
        self.t = 0
        self.last = None

    def step(self, run, after=None):
        """run(out) issues one engine step into output set `out` on the current stream; the step's
        exchange follows on the communication stream, then after(k) (if given) on that stream, with
        g_obs[k] / g_flat[k] holding the step's gathered values.  Returns the set used."""
        torch = self.torch
        k = self.t % self.depth
        out = self.sets[k]
        if self.pending[k] is not None:
            torch.cuda.current_stream(self.eng.device).wait_event(self.pending[k])
        run(out)
        if self.skip:
            if after is not None:
                after(k)
        elif self.comm is not None:
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(self.eng.device))
            self.comm.wait_event(done)
            with torch.cuda.stream(self.comm):
                _all_gather_rows(self.g_obs[k], out.obs, self.group)
                _all_gather_rows(self.g_flat[k], out.flat, self.group)
                if after is not None:
                    after(k)
                ev = torch.cuda.Event()
                ev.record(self.comm)
            self.pending[k] = ev
        else:
            _all_gather_rows(self.g_obs[k], out.obs, self.group)
            _all_gather_rows(self.g_flat[k], out.flat, self.group)
            if after is not None:
                after(k)
        self.last = k
        self.t += 1
        return out

    def wait(self):
        """Make the current stream wait for the last step's exchange (before reading its results)."""
        if self.last is not None and self.pending[self.last] is not None:
            self.torch.cuda.current_stream(self.eng.device).wait_event(self.pending[self.last])

    def _rows(self, t):
        if all(s == self.m for s in self.sizes):
            return t
        return self.torch.cat([t[r * self.m:r * self.m + s] for r, s in enumerate(self.sizes)], dim=0)

    def _flat(self, lo, hi):
        """Rows [lo, hi) of every rank's flat buffer segment (units: bytes per row), ranks in order."""
        self.wait()
        f = self.g_flat[self.last].view(self.world, -1)
        m = self.m
        return self.torch.cat([f[r, lo * m:hi * m].view(m, hi - lo)[:s] for r, s in enumerate(self.sizes)], dim=0)

    def obs(self, copy=False):
        """The last step's node-wide observations (see the class note on their lifetime)."""
        self.wait()
        o = self._rows(self.g_obs[self.last])
        return o.clone() if copy and o is self.g_obs[self.last] else o

    def rewards(self):
        R = self.R
        return self._flat(0, 8 * R).contiguous().view(self.torch.float64).view(-1, R)

    def done(self):
        return self._flat(8 * self.R, 8 * self.R + 1).view(-1)

    def truncated(self):
        return self._flat(8 * self.R + 1, 8 * self.R + 2).view(-1)

    def listed(self):
        """[N, A] uint8: agent a of env e was alive before the step (its reward and observation are valid)."""
        o = 8 * self.R + 2
        return self._flat(o, o + self.A)

    def was_reset(self):
        """[N] uint8: env e's observation is the one its autoreset produced this step."""
        o = 8 * self.R + 2 + self.A
        return self._flat(o, o + 1).view(-1)
