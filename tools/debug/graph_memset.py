#!/usr/bin/env python3
"""Diagnostic: the step graph with the pending-list counters zeroed by captured hipMemsetAsync nodes
(ZS_GRAPH_MEMSET=1) against the product graph (k_zero2), side by side on the same seeds: per step the
list counters of both handles and whether their outputs agree.  Never used by the product."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    from libzombsole_amd import _abi
    from libzombsole_amd.engine import Engine
    n = int(os.environ.get("N_ENVS", "128"))
    steps = int(os.environ.get("STEPS", "60"))
    if os.environ.get("MAP") == "city128":  # deferred respawn: a second counter zeroed per step
        mk = lambda: _abi.multi_env_config(n, "safehouse", [], "city128", ["0", "1", "2", "3"], initial_zombies=50,
                                           minimum_zombies=50, max_episode_steps=int(os.environ.get("MAXSTEPS", "1000")))
    else:
        mk = lambda: _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                           minimum_zombies=0, max_episode_steps=int(os.environ.get("MAXSTEPS", "1000")))
    os.environ["ZS_GRAPH_MEMSET"] = "1"
    a = Engine(mk())
    os.environ["ZS_GRAPH_MEMSET"] = "0"
    b = Engine(mk())
    print("memset handle:", a.describe())
    for e in (a, b):
        e.seed(list(range(1000, 1000 + n)))
        e.reset()
    torch.cuda.synchronize()
    print("after reset: memset", a.debug_lists(), "k_zero2", b.debug_lists(), flush=True)
    for t in range(1, steps + 1):
        a.step_graph(t, 7)
        la = a.debug_lists()
        b.step_graph(t, 7)
        lb = b.debug_lists()
        same = all(torch.equal(getattr(a, k), getattr(b, k)) for k in ("obs", "rewards", "done", "trunc", "was_reset"))
        print("step %3d memset %s k_zero2 %s outputs %s ended %d" % (
            t, la, lb, "same" if same else "DIFFER", int(b.done.sum() + b.trunc.sum())), flush=True)
    a.close()
    b.close()


if __name__ == "__main__":
    main()
