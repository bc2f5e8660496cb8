#!/usr/bin/env python3
"""Diagnostic (not the product): does C3's step get shorter when one half of the envs ticks while the other
half's observations stream?  Two handles of N/2 envs each (the same seeds as one handle of N) on one GPU:

  single   one handle of N: policy, zs_step (tick, side-stream reset, observations)
  seq      the two halves one after the other on one stream
  stagger  tick(A) on s1; tick(B) on s2 after tick(A); obs(A) on s1 beside tick(B); obs(B) after both
           (zs_step without observations, then zs_observe)

Eager launches (no graphs), 200 timed steps after 20 warmup, HIP events on s1."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import libzombsole_amd
    libzombsole_amd.plain_graph_dispatch()
    import torch

    from libzombsole_amd import _abi
    from libzombsole_amd.engine import Engine, _ptr
    cfg = os.environ.get("CFG", "c3")
    n = int(os.environ.get("N_ENVS", "65536"))
    steps, warm = int(os.environ.get("STEPS", "200")), 20
    if cfg == "c5":
        mk = lambda k: _abi.multi_env_config(k, "extermination", [], "bridge64", ["0", "1", "2", "3"], initial_zombies=20,
                                             minimum_zombies=0, max_episode_steps=1000, obs_dtype=_abi.DTYPE_I16)
    else:
        mk = lambda k: _abi.multi_env_config(k, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                             minimum_zombies=0, max_episode_steps=1000, obs_dtype=_abi.DTYPE_I64)
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    res = {}

    def timeit(name, one):
        t = [0]
        with torch.cuda.stream(s1):
            for _ in range(warm):
                t[0] += 1
                one(t[0])
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s1)
            for _ in range(steps):
                t[0] += 1
                one(t[0])
            e1.record(s1)
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
        res[name] = {"ms_per_step": round(ms, 4), "Menv_steps_per_s": round(n / ms / 1e3, 2)}
        print(name, res[name], flush=True)

    one = Engine(mk(n))
    one.seed(list(range(n)))
    one.reset()
    print("single:", json.dumps(one.describe()), flush=True)

    def single(t):
        one.gen_actions(t, 7)
        one.step()
    timeit("single", single)
    one.close()
    del one

    h = n // 2
    # launch overrides for the halves (e.g. HALF_LAUNCH=fused=-1: k_tick with the side-stream reset, as at N)
    hl = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in os.environ.get("HALF_LAUNCH", "").split(",") if kv)
    ha, hb = Engine(mk(h).set_launch(hl)), Engine(mk(n - h).set_launch(hl))
    ha.seed(list(range(h)))
    hb.seed(list(range(h, n)))
    ha.reset()
    hb.reset()
    print("half:", json.dumps(ha.describe()), flush=True)

    def seq(t):
        for e in (ha, hb):
            e.gen_actions(t, 7)
            e.step()
    timeit("seq", seq)

    def tick_only(e):
        o = e.out
        rc = e.L.zs_step(e.h, _ptr(e.actions), None, _ptr(o.rewards), _ptr(o.done), _ptr(o.trunc), _ptr(o.listed),
                         _ptr(o.was_reset), e._stream())
        assert rc == 0

    ev_a, ev_b = torch.cuda.Event(), torch.cuda.Event()

    def stagger(t):
        # s1: gen(A) tick(A) | s2: gen(B) (waits nothing), then tick(B) after tick(A)
        ha.gen_actions(t, 7)
        tick_only(ha)
        ev_a.record(s1)
        with torch.cuda.stream(s2):
            hb.gen_actions(t, 7)
            s2.wait_event(ev_a)
            tick_only(hb)
            ev_b.record(s2)
        ha.observe()
        s1.wait_event(ev_b)
        hb.observe()
    timeit("stagger", stagger)

    # parity of the staggered halves against the single handle: every step's observations at the end
    one = Engine(mk(n))
    one.seed(list(range(n)))
    one.reset()
    with torch.cuda.stream(s1):
        for rep in range(2):  # the halves ran steps 1..warm+steps twice (seq, then stagger)
            for t in range(1, warm + steps + 1):
                one.gen_actions(t, 7)
                one.step()
        torch.cuda.synchronize()
    same = bool(torch.equal(one.obs[:h], ha.obs) and torch.equal(one.obs[h:], hb.obs))
    res["halves_equal_single"] = same
    print("halves equal single handle:", same, flush=True)
    out = os.environ.get("OUT")
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
