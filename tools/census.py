#!/usr/bin/env python3
"""Conflict census of the full-size parity runs (CPU, the oracle only; tests/test_conflict_census.py
defines the cases).  For every run of tests/test_fullsize_parity.py and tests/test_step_graphed.py the
oracle replays the same envs, seeds and steps with the census on at the engine's lanes per env G for
that size, and the summed counts go to one JSON file (default profiles/r05_census.json).

    python tools/census.py [--out profiles/r05_census.json] [--threads 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from libzombsole_amd import _abi  # noqa: E402


def c3(n=1, max_steps=1000):
    return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                 minimum_zombies=0, max_episode_steps=max_steps)


def c4(n=1, max_steps=1000):
    return _abi.multi_env_config(n, "safehouse", [], "city128", ["0", "1", "2", "3"], initial_zombies=50,
                                 minimum_zombies=50, max_episode_steps=max_steps)


def c5(n=1, max_steps=1000):
    return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1", "2", "3"], initial_zombies=20,
                                 minimum_zombies=0, max_episode_steps=max_steps, obs_dtype=_abi.DTYPE_I16)


# (test, builder, envs, steps, seed0, masked-reset modulus, G the engine picks at that size)
RUNS = [
    ("test_c3_65536_graph", c3, 65536, 40, 0, 0, 8),
    ("test_c3_65536_truncation_waves", lambda: c3(max_steps=16), 65536, 40, 0, 3, 8),
    ("test_c3_65536_multistep_graph_side_reset", lambda: c3(max_steps=14), 65536, 40, 0, 0, 8),
    ("test_c2_4096_graph", c3, 4096, 60, 4242, 0, 16),
    ("test_c3_8192_shard_graph", c3, 8192, 60, 6 * 8192, 0, 16),
    ("test_c3_8192_shard_multistep_graph", lambda: c3(max_steps=15), 8192, 48, 4 * 8192, 0, 16),
    ("test_c5_65536_int16_graph", c5, 65536, 40, 0, 0, 16),
    ("test_c5_65536_multistep_graph_side_reset", lambda: c5(max_steps=15), 65536, 32, 0, 0, 16),
    ("test_c5_8192_int16_shard_graph", c5, 8192, 48, 5 * 8192, 0, 16),
    ("test_c4_16384_graph", c4, 16384, 80, 0, 0, 32),
    ("test_c4_16384_multistep_graph_respawn", lambda: c4(max_steps=15), 16384, 48, 0, 0, 32),
    ("test_external_graph_c3_65536", lambda: c3(max_steps=16), 65536, 36, 0, 0, 8),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_census.json"))
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    a = ap.parse_args()
    from oracle.oracle import CENSUS_CASES, run_hashes
    res = {}
    for name, mk, n, steps, seed0, twice, G in RUNS:
        t0 = time.time()
        _, cen = run_hashes(mk(), seed0, n, steps, 7, threads=a.threads, reset_twice_mod=twice, chunk_g=G)
        res[name] = dict(envs=n, steps=steps, seed0=seed0, lanes_per_env=G, census=cen)
        print("%-45s G=%-2d %s  (%.1f s)" % (name, G, " ".join("%s=%d" % (k, cen[k]) for k in CENSUS_CASES),
                                            time.time() - t0), flush=True)
    with open(a.out, "w") as f:
        json.dump({"source": "tools/census.py (oracle/zs_oracle.c census_*, the cases of zs_tick.hpp grp_execute)",
                   "runs": res}, f, indent=1)


if __name__ == "__main__":
    main()
