#!/usr/bin/env python3
"""Import the reference's named maps as parsed JSON layouts (build container only).

Reads the map text files of the read-only reference (/root/reference/zombsole/maps)
with this package's own parser (libzombsole_amd/maps.py, a restatement of
`zombsole/game.py:45-97`) and writes their parsed content — size, obstacles in
file order, spawn and objective lists — to libzombsole_amd/maps/<name>.json, so
the drop-in wrappers accept the reference's map names (e.g. the registered
envs' "bridge", gym_env.py:382-414) on machines without the reference.

    python tools/import_maps.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from libzombsole_amd.maps import Map, MAPS_DIR  # noqa: E402

SRC = "/root/reference/zombsole/maps"


def main():
    for name in sorted(os.listdir(SRC)):
        m = Map.from_file(os.path.join(SRC, name))
        m.name = name
        out = os.path.join(MAPS_DIR, name + ".json")
        with open(out, "w", encoding="utf-8") as f:
            json.dump(m.to_json(), f, separators=(",", ":"))
        print("%-24s %3dx%-3d obstacles=%4d objectives=%3d pspawn=%3d zspawn=%3d" % (
            name, m.size[0], m.size[1], len(m.obstacles), len(m.objectives),
            len(m.player_spawns), len(m.zombie_spawns)))


if __name__ == "__main__":
    main()
