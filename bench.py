#!/usr/bin/env python3
"""Benchmark: batched zombsole env-steps/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json metric: "65 536 parallel 64x64 envs at 1/2/4/8 MI355X";
configs[2], "C3", at 8 GPUs): synthetic 64x64 `bridge64` map, extermination
rules, MultiagentZombsoleEnv semantics with 2 agents + 10 zombies per env,
21x21x3 int64 channel observations for every agent written to HBM each step,
uniform Discrete(7) policy generated on device (splitmix64(seed, step, agent)),
gym TimeLimit 1000, next-step autoreset.  The 65 536 envs are split over the N
GPUs ("strong" scaling: 65 536 on 1 GPU, 8 192 per GPU on 8); envs are
independent, so each rank owns a contiguous global env range (seeds = global
index) and no data-path collective runs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 65536]
    torchrun --nproc-per-node N bench.py --gpus N ...

--gpus N decides the world size: without a launcher, N > 1 starts N rank processes of the same
command (one per GPU, rendezvous on 127.0.0.1); under torchrun, WORLD_SIZE must equal N.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import libzombsole_amd  # noqa: E402

libzombsole_amd.plain_graph_dispatch()  # HIP's plain dispatch for the step graphs, before the first HIP call

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node), 65 536 parallel 64×64 envs at 1/2/4/8 MI355X"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


# C2 4 096 envs on 1 GPU; C3 (headline) 65 536 envs over the node's GPUs; C4
# synthetic city128 safehouse, 4 agents + 50 zombies (minimum 50), 16 384 envs; C5 Multiagent 4
# agents + 20 zombies, 65 536 envs, observations all-gathered every step.
PRESETS = {
    "c2": dict(envs=4096, map="bridge64", agents=2, zombies=10, min_zombies=0, rules="extermination", gather=False,
               obs_dtype="int64"),
    "c3": dict(envs=65536, map="bridge64", agents=2, zombies=10, min_zombies=0, rules="extermination", gather=False,
               obs_dtype="int64"),
    "c4": dict(envs=16384, map="city128", agents=4, zombies=50, min_zombies=50, rules="safehouse", gather=False,
               obs_dtype="int64"),
    # C5 gathers compact int16 observations (lossless, 1/4 of the xGMI bytes)
    "c5": dict(envs=65536, map="bridge64", agents=4, zombies=20, min_zombies=0, rules="extermination", gather=True,
               obs_dtype="int16"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--envs", type=int, default=None, help="total envs over all ranks (strong scaling)")
    p.add_argument("--envs-per-gpu", type=int, default=0, help="fixed envs per rank instead (weak scaling)")
    p.add_argument("--config", default="c3", choices=sorted(PRESETS),
                   help="BASELINE.json configs[1..4] (SURVEY.md §8(d) C2..C5); c3 = the headline metric")
    p.add_argument("--map", default=None)
    p.add_argument("--agents", type=int, default=None)
    p.add_argument("--zombies", type=int, default=None)
    p.add_argument("--min-zombies", type=int, default=None)
    p.add_argument("--rules", default=None)
    p.add_argument("--gather", action="store_true", default=None,
                   help="all-gather the observation shards every step (C5's RCCL exchange)")
    p.add_argument("--gather-self", action="store_true",
                   help="(diagnostics) issue the exchange's collectives at world size 1 too (StepGather "
                        "self_exchange; by default they are skipped there: the output sets are the whole buffers)")
    p.add_argument("--max-episode-steps", type=int, default=1000)
    p.add_argument("--obs-dtype", default=None, choices=["int64", "int32", "int16"])
    p.add_argument("--lanes-per-env", type=int, default=0, help="k_tick lanes per env (0 = engine default)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-graph", action="store_true",
                   help="launch every step's kernels from the host instead of replaying the step as a hipGraph")
    p.add_argument("--graph-steps", type=int, default=1,
                   help="steps per graph launch at most (zs_step_graph_n; the largest count dividing --steps; "
                        "--warmup rounded up to whole launches); 1 (default) = one graph launch per step, every "
                        "step's outputs visible to the caller")
    p.add_argument("--multi-steps", type=int, default=8,
                   help="after the timed loop, time the same steps again with up to this many steps per graph "
                        "launch and report them in the separate 'multi_step_graph' field (0 = skip); the "
                        "intermediate steps' outputs are overwritten there, so it is not the headline value")
    p.add_argument("--policy", default="device", choices=["device", "external"],
                   help="device: the uniform Discrete(7) policy generated on device inside the step graph "
                        "(SURVEY.md §8(d)); external: a caller-side policy, torch ops on the engine's stream "
                        "that derive every step's actions from the previous step's observations, then the "
                        "graphed step on those actions (zs_step_graph with n_discrete = 0; a learner's loop)")
    p.add_argument("--cpu-steps", type=int, default=2000)
    p.add_argument("--launch", default="",
                   help="launch overrides for A/B runs, 'field=v,...' (zs_launch fields; 1 = on, -1 = off, n = size)")
    p.add_argument("--engine-lib", default=None, help="(tools) another build of the engine's sources, e.g. an A/B build")
    p.add_argument("--dry-run", action="store_true",
                   help="(tests) the multi-rank control flow only: rank processes, gloo rendezvous, env ranges, the "
                        "barrier-bracketed timed loop on a no-op step and the slowest-rank time; no engine, no GPU")
    a = p.parse_args()
    a.launch = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.launch.split(",") if kv)
    for k, v in PRESETS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


# mean MT19937 words drawn per env-step of each preset's workload (oracle/zs_oracle.c, uniform Discrete(7)
# agents, 24 envs x 300 steps: C2/C3 12.2, C5 23.2; C4 median 82)
MT_WORDS = {"c2": 12, "c3": 12, "c4": 82, "c5": 23}


def algorithmic_bytes(E, A, OW, obs_bytes_per_env, mt_words):
    """Algorithmic HBM bytes per env-step, split by kernel.

    tick: entity SoA read + write (E x (pos 4 + life 4 + weapon 1 + present 1 + order 1) x 2)
          + per-env scalars read + write (9 x 4 x 2) + reward tracker / env.agents rows (A x 5 x 2)
          + RNG stream state (4 x 2) + obstacle-present bits read (4 x OW)
          + MT words drawn x 12 (the word read, and its share of the twist that made it: 4 read + 4 write)
          + actions (12 A) + rewards (8 A) + done / truncated / listed (2 + A)
    obs : observation bytes written (A x 3 x 21 x 21 x 8 B for int64)
    The step launch (k_step) carries both when it writes the observations itself (fobs).
    """
    tick = 22 * E + 72 + 10 * A + 8 + 4 * OW + 12 * mt_words + 12 * A + 8 * A + 2 + A
    return tick, obs_bytes_per_env


def host_cpu():
    """nproc, the affinity set, the cgroup CPU quota and the CPU model of this host."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = info["nproc"]
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            info["cgroup_cpu_quota"] = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        info["cgroup_cpu_quota"] = None
    model, sockets, cores = None, set(), None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name") and model is None:
                    model = line.split(":", 1)[1].strip()
                elif line.startswith("physical id"):
                    sockets.add(line.split(":", 1)[1].strip())
                elif line.startswith("cpu cores") and cores is None:
                    cores = int(line.split(":", 1)[1])
    except (OSError, ValueError):
        pass
    info["model"] = model
    info["sockets"] = len(sockets) or None
    info["physical_cores"] = cores * len(sockets) if cores and sockets else None
    return info


def cpu_baseline(args, builder_fn):
    """The C oracle (bit-exact CPU restatement, "port") on this host, bounded sample, OpenMP over every
    CPU of the affinity set, plus a 1-thread figure."""
    from oracle.oracle import run_batch
    host = host_cpu()
    # every CPU of the affinity set, unless a cgroup CPU quota caps the process below that (the GPU
    # box: 256 CPUs visible, a 16-CPU quota; oversubscribing the quota only adds preemption)
    threads = host["affinity"] or 1
    if host["cgroup_cpu_quota"]:
        threads = max(1, min(threads, int(host["cgroup_cpu_quota"] + 0.5)))
    b = builder_fn(1)

    def timed(n_envs, steps, th):
        t0 = time.perf_counter()
        n, _ = run_batch(b, 0, n_envs, steps, 7, threads=th)
        return n, time.perf_counter() - t0

    # size the samples from a short probe: ~1.5 s wall on one thread, ~3 s on all of them
    n1, dt1 = timed(64, 20, 1)
    rate1 = n1 / dt1
    steps1 = max(20, min(args.cpu_steps, int(1.5 * rate1 / 64)))
    n1, dt1 = timed(64, steps1, 1)
    rate1 = n1 / dt1
    steps = args.cpu_steps
    eff = min(threads, host["cgroup_cpu_quota"] or threads)
    n_envs = max(threads * 4, int(3.0 * rate1 * eff / steps))
    n, dt = timed(n_envs, steps, threads)
    cores = host["physical_cores"] or host["nproc"]
    return {"value": n / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "host": host, "one_thread_value": rate1,
            # not measured: the 1-thread rate times the host's physical cores (linear scaling, no SMT
            # gain), the figure the whole host could reach without the quota
            "all_cores_linear_estimate": rate1 * cores,
            "sample": "C oracle (oracle/zs_oracle.c, OpenMP over envs, %d threads = the CPUs of the affinity set "
                      "within the cgroup quota; "
                      "host %s, %s socket(s), %s cores, nproc %s, cgroup CPU quota %s), %d envs x %d steps of the same "
                      "workload (same map/agents/zombies/policy/obs, autoreset, TimeLimit), %.2f s wall; "
                      "1 thread: %.0f env-steps/s over 64 envs x %d steps" % (
                          threads, host["model"], host["sockets"], host["physical_cores"], host["nproc"], host["cgroup_cpu_quota"],
                          n_envs, steps, dt, rate1, steps1)}


def external_policy(eng, n_discrete=7):
    """A learner-side policy with a true per-step dependency: every agent's Discrete(n) id is taken from
    its own window-centre cell of the previous step's observations (code + life + weapon channels) plus
    the step number, by torch ops on the engine's stream, and written as triples into the engine's
    action buffer, which the graphed step then reads (Engine.step_graphed).  Four small kernels."""
    import torch
    from libzombsole_amd.actions import DISCRETE_TRIPLES
    assert eng.multi, "the external policy reads the multi-agent [N, A, 3, w, w] observations"
    triples = torch.from_numpy(DISCRETE_TRIPLES[:n_discrete].copy()).to(eng.device)
    N, (nobs, C, H, W) = eng.N, eng.obs_shape
    centre = (H // 2) * W + W // 2
    cells = eng.obs.view(N, nobs, C, H * W)[:, :, :, centre]  # [N, A, 3] strided view
    dst = eng.actions.view(-1, 3)

    def policy(t):
        ids = cells.sum(-1, dtype=torch.int64)
        ids.add_(t).remainder_(n_discrete)
        torch.index_select(triples, 0, ids.view(-1), out=dst)
    return policy


def env_range(rank, world, total_envs, envs_per_gpu=0):
    """(envs on this rank, first global env, scaling, node-wide envs): a fixed count per rank (weak
    scaling) or the node's total split into contiguous ranges by vector.shard_range, the partition
    the batched API documents (strong)."""
    from libzombsole_amd.vector import shard_range
    if envs_per_gpu:
        return envs_per_gpu, rank * envs_per_gpu, "weak", envs_per_gpu * world
    env0, n = shard_range(total_envs, rank, world)
    return n, env0, "strong", total_envs


def timed_loop(one_step, steps, warmup, sync, distributed, before_timing=None):
    """W untimed steps, then exactly K steps bracketed by sync() (the device) and a barrier on both
    sides; returns this rank's wall time of the K steps."""
    import torch.distributed as dist
    for _ in range(warmup):
        one_step()
    sync()
    if distributed:
        dist.barrier()
    if before_timing:
        before_timing()
    sync()
    if distributed:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_step()
    sync()
    if distributed:
        dist.barrier()
    return time.perf_counter() - t0


def max_over_ranks(elapsed, device):
    """The slowest rank's time (every rank gets it)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`--gpus N` without a launcher: N rank processes of this same command (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* as torchrun sets them, rendezvous on 127.0.0.1), started before this process
    makes any HIP call, one per GPU.  Rank 0 prints the JSON line.  A rank that fails ends the others;
    the exit status is the first failing rank's."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code and not rc:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


def dry_run(args, world, rank, distributed):
    """--dry-run: the control flow of a multi-rank bench run on CPU (gloo), reported in the same JSON shape."""
    import torch
    import torch.distributed as dist
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    n_local, env0, scaling, total_envs = env_range(rank, world, args.envs, args.envs_per_gpu)
    elapsed = timed_loop(lambda: time.sleep(0.001), args.steps, args.warmup, lambda: None, distributed)
    ranges = [(env0, n_local)]
    if distributed:
        elapsed = max_over_ranks(elapsed, torch.device("cpu"))
        ranges = [None] * world
        dist.all_gather_object(ranges, (env0, n_local))
    out = {"metric": METRIC, "value": total_envs * args.steps / elapsed, "unit": "env-steps/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
           "scaling": scaling, "dry_run": True, "rank_env_ranges": ranges, "total_envs": total_envs}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


def main():
    args = parse()
    # --gpus N decides the world size: N > 1 without a launcher spawns the N ranks here (before any HIP
    # call in this process); under a launcher (torchrun: WORLD_SIZE set) the two must agree
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but the launcher's WORLD_SIZE is %s\n" % (args.gpus, env_world))
        sys.exit(2)
    if args.dry_run:
        world = int(os.environ.get("WORLD_SIZE", "1"))
        dry_run(args, world, int(os.environ.get("RANK", "0")), world > 1)
        return
    # ONE JSON line on stdout: anything else the process prints there (RCCL's version banner at its first
    # communicator, library notices) goes to stderr; the line itself is written to the saved stdout
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    from libzombsole_amd import _abi
    from libzombsole_amd import engine as engine_mod
    from libzombsole_amd.engine import Engine
    if args.engine_lib:
        engine_mod.use_library(args.engine_lib)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    # under torchrun (even --nproc-per-node 1) the ranks form an RCCL group: C5's gather then runs
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if distributed:
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    dtype = {"int64": _abi.DTYPE_I64, "int32": _abi.DTYPE_I32, "int16": _abi.DTYPE_I16}[args.obs_dtype]
    agent_ids = [str(i) for i in range(args.agents)]

    def builder(n):
        return _abi.multi_env_config(n, args.rules, [], args.map, agent_ids, initial_zombies=args.zombies,
                                     minimum_zombies=args.min_zombies, max_episode_steps=args.max_episode_steps,
                                     obs_dtype=dtype, lanes_per_env=args.lanes_per_env).set_launch(args.launch)

    n_local, env0, scaling, total_envs = env_range(rank, world, args.envs, args.envs_per_gpu)
    eng = Engine(builder(n_local), device=dev)
    launch = eng.describe()
    launch["step_graph"] = not args.no_graph
    if args.launch:
        launch["overrides"] = args.launch
    eng.seed([env0 + i for i in range(n_local)])
    eng.reset()
    torch.cuda.synchronize()

    gather = None
    if args.gather and distributed:
        # C5: every step's observation shards + rewards / done / truncated, all-gathered over RCCL into
        # node-wide tensors (a centralised learner's input) on a second stream while the next step runs
        from libzombsole_amd.vector import StepGather
        gather = StepGather(eng, self_exchange=args.gather_self)
        launch["exchange"] = "skipped (world size 1)" if gather.skip else "RCCL all-gathers (in place)"

    step = 0
    use_graph = not args.no_graph
    # steps per graph launch: every step still runs its policy, tick and observation launches; only the
    # graph launches are fewer (the outputs of a launch's earlier steps are overwritten, as they are by
    # the next launch with one step per graph).  Not with the per-step exchange.
    # the timed region covers exactly --steps steps: the largest count up to --graph-steps that divides it
    # (warmup rounded up to whole launches, so the timed launches replay an already captured graph)
    external = args.policy == "external"
    policy = external_policy(eng) if external else None
    gsteps = 1
    if use_graph and not gather and not external:
        gsteps = max(d for d in range(1, max(1, args.graph_steps) + 1) if args.steps % d == 0)
    args.warmup = -(-args.warmup // gsteps) * gsteps
    launch["graph_steps"] = gsteps
    launch["policy"] = "external: torch ops on the previous step's observations" if external else "on device"

    def one_step(gs=None):
        # the bench loop's step: the on-device policy's actions for step t, then zs_step; with graphs
        # both are one replayed hipGraph whose step counter advances on the device.  external: the
        # caller's policy writes the engine's action buffer from the last observations, then the step
        nonlocal step
        gs = gsteps if gs is None else gs
        if gs > 1:
            eng.step_graph(step + 1, 7, steps=gs)
            step += gs
            return
        step += 1
        if external:
            policy(step)
            if gather:
                gather.step(lambda out: eng.step_graphed(out=out) if use_graph else eng.step(out=out))
            elif use_graph:
                eng.step_graphed()
            else:
                eng.step()
        elif gather:
            if use_graph:
                gather.step(lambda out: eng.step_graph(step, 7, out=out))
            else:
                eng.gen_actions(step, 7)
                gather.step(lambda out: eng.step(out=out))
        elif use_graph:
            eng.step_graph(step, 7)
        else:
            eng.gen_actions(step, 7)
            eng.step()

    elapsed = timed_loop(one_step, args.steps // gsteps, args.warmup // gsteps, torch.cuda.synchronize, distributed,
                         before_timing=None if use_graph else (lambda: eng.profile(True)))
    # the same workload with several steps per graph launch (the launch gap paid once per launch; the
    # outputs of a launch's earlier steps are overwritten): reported beside the headline, never as it
    multi = None
    if use_graph and not gather and not external and gsteps == 1 and args.multi_steps > 1:
        ms = max(d for d in range(1, args.multi_steps + 1) if args.steps % d == 0)
        if ms > 1:
            el = timed_loop(lambda: one_step(ms), args.steps // ms, max(1, -(-args.warmup // ms)),
                            torch.cuda.synchronize, distributed)
            if distributed:
                el = max_over_ranks(el, torch.device("cuda", local))
            multi = {"graph_steps": ms, "value": total_envs * args.steps / el, "ms_per_step": el * 1e3 / args.steps,
                     "note": "%d steps per graph launch: only every %d-th step's outputs are visible to the caller; "
                             "not the headline" % (ms, ms)}
    prof_steps = args.steps
    if use_graph:
        # per-kernel HIP-event durations: the same steps launched one kernel at a time right after
        # the timed replays (events cannot bracket the kernels inside a graph)
        prof_steps = min(args.steps, 50)
        eng.profile(True)
        for _ in range(prof_steps):
            step += 1
            eng.gen_actions(step, 7)
            eng.step()
        torch.cuda.synchronize()
    prof = eng.profile_read()
    # the mix of the timed window: episodes ending per step (each is an autoreset at the next step,
    # on the reset side stream), sampled over a few untimed steps that continue the same trajectories
    mix_steps = 20
    eng.profile(False)
    ends = torch.zeros(2, dtype=torch.int64, device=eng.device)
    for _ in range(mix_steps):
        step += 1
        eng.gen_actions(step, 7)
        eng.step()
        ends[0] += eng.done.sum()
        ends[1] += eng.trunc.sum()
    torch.cuda.synchronize()
    ends = ends.tolist()
    if distributed:
        elapsed = max_over_ranks(elapsed, torch.device("cuda", local))
    value = total_envs * args.steps / elapsed

    # roofline of the dominant kernel (HIP-event durations on the engine's stream)
    m = eng.builder.map
    E = args.agents + args.zombies
    obs_per_env = eng.obs[0].numel() * eng.obs.element_size()
    n_obst = len(m.obstacles)
    tick_b, obs_b = algorithmic_bytes(E, args.agents, (n_obst + 31) // 32, obs_per_env, MT_WORDS.get(args.config, 12))
    # per-step kernel time (a step may run its tick and observation kernels in several env chunks
    # on two streams: sum the launches of each kind per step)
    tick_ms = prof["tick_ms"] / prof_steps
    obs_ms = prof["obs_ms"] / prof_steps
    reset_ms = prof["reset_ms"] / prof_steps
    fused = prof["reset_n"] == 0  # reset work runs inside the step launch (k_step)
    fobs = prof["obs_n"] == 0      # the step launch writes the observations itself (zs_launch.fobs)
    step_name = launch["step_kernel"]
    step_b = tick_b + (obs_b if fobs else 0)
    if fobs or tick_ms >= obs_ms:
        dom, dom_ms, dom_b = step_name, tick_ms, step_b
    else:
        dom, dom_ms, dom_b = launch["obs_kernel"], obs_ms, obs_b
    achieved = dom_b * n_local / (dom_ms * 1e-3) / 1e9
    # profiled workload key: the preset, or "n8" for C3's 8 192-env shard (the 8-GPU headline's per-GPU run)
    wkey = "n8" if (args.config == "c3" and n_local == 8192) else args.config
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                wls = json.load(f).get("workloads", {})
            wl = wls.get(wkey) or wls.get(args.config)
            # profiled bytes per launch, scaled to this run's envs per GPU (per-env work is fixed)
            t = wl["kernels"].get(dom, {}).get("hbm_bytes_per_launch") if wl else None
            traffic = t * n_local / wl["envs_per_gpu"] if t is not None else None
        except Exception:
            traffic = None
    # issue figures of the dominant and the step kernel from the SQ / GRBM counter passes (SURVEY.md §8(d):
    # the path is latency / issue bound; tools/pmc_sq.py defines them)
    issue = None
    sqp = os.path.join(ROOT, "profiles", "pmc_sq.json")
    if os.path.exists(sqp):
        try:
            with open(sqp) as f:
                wl = json.load(f).get("workloads", {}).get(wkey)
            if wl:
                keep = ("valu_busy", "waves_per_cu", "wait_frac", "stall_frac", "active_frac", "valu_per_wave")
                issue = {"profile": wl["profile"], "source": "profiles/pmc_sq.json"}
                for k in {dom, step_name, launch["obs_kernel"]}:
                    if k in wl["kernels"]:
                        issue[k] = {n: round(v, 4) for n, v in wl["kernels"][k].items() if n in keep}
        except Exception:
            issue = None
    out = {
        "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "int32", "data": "synthetic",
        "config": {"workload": "%s: %d parallel %dx%d '%s' envs over %d GPU(s) (%d per GPU), %s, %d agents + "
                               "%d zombies (minimum %d), MultiagentZombsoleEnv rewards, %s, 21x21x3 %s obs per "
                               "agent written to HBM every step%s, TimeLimit %d, next-step autoreset, one step per "
                               "graph launch%s" % (
                                   args.config.upper(), total_envs, m.size[0], m.size[1], args.map, world, n_local,
                                   args.rules, args.agents, args.zombies, args.min_zombies,
                                   "a caller-side torch policy on the previous step's observations" if external
                                   else "uniform Discrete(7) policy on device", args.obs_dtype,
                                   " and all-gathered over RCCL with rewards/done/truncated" if gather else "",
                                   args.max_episode_steps,
                                   "" if gsteps == 1 else " (here %d: only every %d-th step's outputs visible)" % (
                                       gsteps, gsteps)),
                   "preset": args.config, "envs_per_gpu": n_local, "total_envs": total_envs, "map": args.map,
                   "rules": args.rules, "agents": args.agents, "zombies": args.zombies,
                   "minimum_zombies": args.min_zombies, "obs_dtype": args.obs_dtype,
                   "parallelism": "env-sharded x%d (%s)" % (
                       world, "RCCL all-gather of obs + rewards/done per step" if gather
                       else "no data-path collective"), "launch": launch,
                   "episode_ends_per_step": {"done": ends[0] / mix_steps, "truncated": ends[1] / mix_steps,
                                             # done or truncated: each is an autoreset at the next step
                                             "fraction_of_envs": (ends[0] + ends[1]) / mix_steps / n_local,
                                             "sample": "%d untimed steps after the timed window, rank 0" % mix_steps}},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_step": dom_b * n_local,
                     "kernel_ms_per_step": dom_ms, "launches_per_step": {
                         "tick": prof["tick_n"] / prof_steps, "obs": prof["obs_n"] / prof_steps,
                         "reset": prof["reset_n"] / prof_steps, "respawn": prof["respawn_n"] / prof_steps},
                     "step_launch_ms": tick_ms, "k_obs_ms": obs_ms,
                     "k_reset_ms": reset_ms, "k_respawn_ms": prof["respawn_ms"] / prof_steps,
                     "step_launch_writes_obs": bool(fobs),
                     "step_launch_resets": bool(fused),
                     "issue": issue},
        "cpu_baseline": None,
    }
    if multi:
        out["multi_step_graph"] = multi
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, builder)
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    eng.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
