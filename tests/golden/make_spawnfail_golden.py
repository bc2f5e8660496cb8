#!/usr/bin/env python3
"""Golden vectors for a reset that cannot place every player / agent (core.py:40-66, game.py:151-187), from
the REAL reference (this container only; no-op shims for gymnasium / termcolor / cv2 as make_golden.py).

For each case: `random.seed(s)`, construct the env (its constructor builds the first world), catch the bare
Exception the reference raises, and record its message and the `random` state it leaves (sha256 of
getstate()'s words: the spawn shuffles' draws are taken before the failure).  Writes
tests/golden/spawn_failure.json.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_spawnfail_golden.py
"""
import hashlib
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, "shims"))
sys.path.insert(0, "/root/reference")

from zombsole.gym_env import ZombsoleGymEnv  # noqa: E402
from zombsole.gym.multiagent_env import MultiagentZombsoleEnv  # noqa: E402

WALL_HP = os.path.join(HERE, "maps", "wall_hp.txt")  # two player spawn cells
# name, surface, kwargs
CASES = [
    ("agents_past_spawns", "multi", dict(rules_name="extermination", player_names=[], map_name=WALL_HP,
                                         agent_ids=["0", "1", "2"], initial_zombies=0)),
    ("bots_take_spawns", "single", dict(rules_name="extermination", player_names=["troll", "sniper"],
                                        map_name=WALL_HP, agent_id=0, initial_zombies=0)),
    ("bot_past_spawns", "single", dict(rules_name="survival", player_names=["terminator", "sniper", "troll"],
                                       map_name=WALL_HP, agent_id=0, initial_zombies=0)),
]


def state_sha():
    return hashlib.sha256(struct.pack("<625I", *random.getstate()[1])).hexdigest()


def main():
    out = []
    for name, surface, kw in CASES:
        for seed in (3, 4):
            random.seed(seed)
            try:
                (ZombsoleGymEnv if surface == "single" else MultiagentZombsoleEnv)(**dict(kw))
                raise RuntimeError("expected a spawn failure: %s" % name)
            except Exception as err:
                if type(err) is not Exception:
                    raise
                out.append({"case": name, "surface": surface, "seed": seed,
                            "kwargs": dict(kw, map_name="wall_hp"), "message": str(err), "rng_sha": state_sha()})
    with open(os.path.join(HERE, "spawn_failure.json"), "w") as f:
        json.dump(out, f, indent=1)
    for r in out:
        print(r["case"], r["seed"], r["message"], r["rng_sha"][:12])


if __name__ == "__main__":
    main()
