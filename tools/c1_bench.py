#!/usr/bin/env python3
"""C1 timing: the drop-in envs' per-call rate on one env (BASELINE.json configs[0]).

C1 is the reference's plumbing config: one env on the real `bridge` map (111x12), extermination, 10
zombies, driven through the reference's own class surface.  This times the drop-ins exactly as a
caller of the reference would use them, one call at a time:

  * `MultiagentZombsoleEnvDiscreteAction`, agents ["0", "1"], 21x21 channels (int64) observations
    (reference: 973 env-steps/s on one core);
  * `ZombsoleGymEnvDiscreteAction`, agent 0, world / simple observations
    (reference: 1 012 env-steps/s on one core).

Protocol of BASELINE.md §2: uniform random discrete actions (the counter-based stream of
`libzombsole_amd.actions`), `env.reset()` when an episode ends, reset time counted.  Also reported:
the mean time of a `step()` and of a `reset()` call alone, and the engine's share of a step (one
zs_host_step call: one copy in, one copy out, one synchronisation).

    python tools/c1_bench.py [--steps 3000] [--out profiles/r06_c1.json]
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import libzombsole_amd  # noqa: E402

libzombsole_amd.plain_graph_dispatch()
from libzombsole_amd import actions as A  # noqa: E402

REFERENCE = {"multi": 973.0, "single": 1012.0}  # BASELINE.md §2, env-steps/s on one core


def make(surface, events):
    from libzombsole_amd.gym_env import ZombsoleGymEnvDiscreteAction
    from libzombsole_amd.gym.multiagent_env import MultiagentZombsoleEnvDiscreteAction
    if surface == "multi":
        return MultiagentZombsoleEnvDiscreteAction("extermination", [], "bridge", ["0", "1"], initial_zombies=10,
                                                   minimum_zombies=0)
    return ZombsoleGymEnvDiscreteAction("extermination", [], "bridge", 0, initial_zombies=10, minimum_zombies=0,
                                        observation_scope="world", observation_position_encoding="simple")


def run(surface, steps, seed, events):
    env = make(surface, events)
    base = env.env
    random.seed(seed)
    env.reset()
    ids = list(base.possible_agents) if surface == "multi" else [0]
    n_act = 7 if surface == "multi" else 6
    t_step = t_reset = 0.0
    n_reset = 0
    n_events = 0
    t0 = time.perf_counter()
    for k in range(steps):
        if surface == "multi":
            act = {aid: int(A.discrete_action_id(seed, k, i, n_act)) for i, aid in enumerate(ids)}
        else:
            act = int(A.discrete_action_id(seed, k, 0, n_act))
        a = time.perf_counter()
        out = env.step(act)
        t_step += time.perf_counter() - a
        if events:
            n_events += len(base.game.world.events)
        if surface == "multi":
            done = bool(out[2]) and all(out[2].values())
            trunc = bool(out[3]) and all(out[3].values())
        else:
            done, trunc = out[2], out[3]
        if done or trunc or (surface == "multi" and not base.agents):
            a = time.perf_counter()
            env.reset()
            t_reset += time.perf_counter() - a
            n_reset += 1
    wall = time.perf_counter() - t0
    env.close()
    return {"surface": surface, "steps": steps, "resets": n_reset, "wall_s": wall, "env_steps_per_s": steps / wall,
            "step_us": 1e6 * t_step / steps, "reset_us": 1e6 * t_reset / max(1, n_reset),
            "reference_env_steps_per_s": REFERENCE[surface], "vs_reference": (steps / wall) / REFERENCE[surface],
            "events_read": bool(events)}


def raw_calls(steps):
    """The engine's share of a call: zs_host_step alone on the multi-agent C1 env (no env glue)."""
    env = make("multi", False)
    core = env.env._core
    eng = core.engine
    acts = core._actions
    acts[:] = 0
    out = {}
    for key, rng in (("host_step_rng_us", core._rng_in()), ("host_step_us", None)):
        rec = eng.host_record()
        for _ in range(50):
            eng.host_step(acts, rng, rec)
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.host_step(acts, rng, rec)
        out[key] = 1e6 * (time.perf_counter() - t0) / steps
    env.close()
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=3000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--out", default=None)
    p.add_argument("--events", action="store_true", help="also read World.events after every step")
    p.add_argument("--profile", action="store_true", help="cProfile the multi-agent run (top functions by own time)")
    args = p.parse_args()
    import torch
    res = {"metric": "drop-in env-steps/s, one env per call (C1: real bridge, extermination, 10 zombies)",
           "device": torch.cuda.get_device_name(0), "host_threads": 1, "runs": []}
    for surface in ("multi", "single"):
        run(surface, args.warmup, args.seed + 1, args.events)  # warm-up (first captures, allocations)
        r = run(surface, args.steps, args.seed, args.events)
        res["runs"].append(r)
        print("%-6s %8.0f env-steps/s  step %7.1f us  reset %8.1f us  (%d resets)  reference %5.0f -> x%.1f" % (
            surface, r["env_steps_per_s"], r["step_us"], r["reset_us"], r["resets"], r["reference_env_steps_per_s"],
            r["vs_reference"]), flush=True)
    res["engine_call"] = raw_calls(args.steps)
    print("engine alone: zs_host_step %.1f us (with the random state moved in), %.1f us (without)" % (
        res["engine_call"]["host_step_rng_us"], res["engine_call"]["host_step_us"]), flush=True)
    if args.profile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        run("multi", args.steps, args.seed, args.events)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    line = json.dumps(res)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(line + "\n")
    print(line)


if __name__ == "__main__":
    main()
