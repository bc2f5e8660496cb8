#!/usr/bin/env python3
"""Diagnostic: where do k_tick's cycles go?  Builds a -DZS_STAMPS copy of the engine and
reports, per phase, the mean and max s_memtime cycles per workgroup launch for the bench
workload at several lanes-per-env settings.  Never used by the product or the bench."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "libzombsole_amd", "_build", "libzombsole_mi355x_stamps.so")
PHASES = ["stage-in", "decide", "grp-exec", "leader", "mt-refill", "stage-out", "obs-write",
          "  L:defer+shuffle", "  L:execute", "  L:order+cleanup", "  L:reward+rules", "  S:to round 1", "  S:to window",
          "R:setup+rng", "R:weapons", "R:spawn p+a", "R:zombie lives", "R:spawn z", "R:twist+out", "-",
          "  G:shuffle draws", "  G:shuffle track", "  G:chunk loads", "  G:chunk scan", "  G:resolve+range",
          "  G:damage draws", "  G:lives+commit", "  leader-exec envs"]


def main():
    import __graft_entry__ as ge
    if not os.path.exists(SO) or "--rebuild" in sys.argv:
        ge.build_engine(extra=["-DZS_STAMPS"], out=SO, tag="stamps")
    if "--build-only" in sys.argv:
        return
    import torch
    from libzombsole_amd import _abi
    from libzombsole_amd import engine as engine_mod
    from libzombsole_amd.engine import Engine
    engine_mod.use_library(SO)
    # launch overrides of the run, 'field=v,...' (zs_launch fields)
    launch = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in os.environ.get("LAUNCH", "").split(",") if kv)
    n_envs = int(os.environ.get("N_ENVS", "8192"))
    for G in [int(g) for g in os.environ.get("GS", "1,2,4,8,16").split(",")]:
        A = int(os.environ.get("AGENTS", "2"))
        b = _abi.multi_env_config(n_envs, os.environ.get("RULES", "extermination"), [],
                                  os.environ.get("MAP", "bridge64"), [str(i) for i in range(A)],
                                  initial_zombies=int(os.environ.get("ZOMBIES", "10")),
                                  minimum_zombies=int(os.environ.get("MINZ", "0")), max_episode_steps=1000,
                                  lanes_per_env=G).set_launch(launch)
        eng = Engine(b)
        eng.seed(list(range(n_envs)))
        eng.reset()
        for t in range(1, 31):
            eng.gen_actions(t, 7)
            eng.step()
        torch.cuda.synchronize()
        eng.debug_stamps()
        eng.profile(True)
        steps = 50
        nres_t = torch.zeros((), dtype=torch.int64, device=eng.device)
        for t in range(31, 31 + steps):
            eng.gen_actions(t, 7)
            eng.step()
            nres_t += eng.was_reset.sum()
        torch.cuda.synchronize()
        prof = eng.profile_read()
        nres = int(nres_t.item())
        print("resets per step: %.1f" % (nres / steps))
        ssum, smax = eng.debug_stamps(len(PHASES))
        wgs = (n_envs + 64 // G - 1) // (64 // G)
        print("G=%2d  k_tick %.1f us  k_obs %.1f us  k_reset %.1f us" % (
            G, 1e3 * prof["tick_ms"] / max(prof["tick_n"], 1), 1e3 * prof["obs_ms"] / max(prof["obs_n"], 1),
            1e3 * prof["reset_ms"] / max(prof["reset_n"], 1)))
        for k, name in enumerate(PHASES):
            if name == "-":
                continue
            if name.startswith("R:"):  # per reset performed
                print("   %-10s per-reset %9.0f cyc" % (name, ssum[k] / max(1, nres)))
            else:
                print("   %-10s mean %9.0f cyc   max %9d cyc" % (name, ssum[k] / (wgs * steps), smax[k]))
        if ssum[19]:  # k_respawn (its phases share the R: slots; resets are few where respawns are many)
            nr = float(int(ssum[19]) & 0xffffffff)
            print("respawns per step: %.1f (with zombies to place: %.1f)" % (nr / steps, (int(ssum[19]) >> 32) / steps))
            for i, name in enumerate(["loads+rows", "occupancy+rng", "lives draws", "spawn", "finish+out"]):
                print("   P:%-14s per-respawn %9.0f cyc" % (name, ssum[13 + i] / nr))
        desc = eng.describe()
        if desc.get("step_kernel") == "k_step":
            # workgroup timeline of one more fused step launch (s_memrealtime, 10 ns)
            import numpy as np
            n_reset = min(n_envs, launch.get("reset_wgs", 256))
            eng.debug_stamps(len(PHASES))  # clears: the next read is this one launch's
            eng.gen_actions(31 + steps, 7)
            eng.step()
            torch.cuda.synchronize()
            tl = eng.debug_timeline(n_reset + wgs).astype(np.int64)
            t0 = tl[:, 0].min()
            st, en = (tl[:, 0] - t0) / 100.0, (tl[:, 1] - t0) / 100.0  # us
            dur = en - st
            q = lambda a: " ".join("p%d %.1f" % (p, np.percentile(a, p)) for p in (10, 50, 90, 99, 100))
            print("   timeline (us from the first workgroup start): launch span %.1f" % en.max())
            print("     tick wg start  %s" % q(st[n_reset:]))
            print("     tick wg end    %s" % q(en[n_reset:]))
            print("     tick wg life   %s" % q(dur[n_reset:]))
            if n_reset:
                print("     reset wg end   %s" % q(en[:n_reset]))
            # phase cycles of that launch's slowest 1 % tick workgroups against its median ones
            ph = eng.debug_stamps_wg(n_reset + wgs, len(PHASES)).astype(np.float64)[n_reset:]
            life = dur[n_reset:]
            order = np.argsort(life)
            slow = order[-max(1, len(order) // 100):]
            mid = order[len(order) // 2 - len(order) // 20: len(order) // 2 + len(order) // 20]
            print("     phases of the slowest 1%% (%d wgs, life %.1f us) vs the median 10%% (life %.1f us):" % (
                len(slow), life[slow].mean(), life[mid].mean()))
            top = order[-3:][::-1]
            print("       %-18s %9s  %9s  | slowest three: %s us" % ("", "slowest1%", "median", " ".join("%.1f" % life[w] for w in top)))
            for k, name in enumerate(PHASES):
                if name == "-" or name.startswith("R:"):
                    continue
                a, b = ph[slow, k].mean(), ph[mid, k].mean()
                if a or b:
                    print("       %-18s %9.0f  %9.0f  | %s" % (name.strip(), a, b, " ".join("%9.0f" % ph[w, k] for w in top)))
        eng.close()


if __name__ == "__main__":
    main()
