"""Map loading — host side of the boundary.

`Map.from_file` restates the reference's map text parser
(`zombsole/game.py:45-97`): one character per cell, column = x, row = y;
`▓`/`w`/`W` wall, `☒`/`b`/`B` box, `p` player spawn, `z` zombie spawn, `o`
objective (case-insensitive), anything else empty.  Width/height are the
largest column/row index seen (+1), where every character of a non-empty line
counts (spaces included) and empty lines are skipped but keep their row index.

Bundled maps live in ``libzombsole_amd/maps``: the synthetic benchmark maps
(`bridge64.txt`, `city128.txt`, written by tools/gen_maps.py in the reference
format) and the reference's named maps in parsed form (`<name>.json`, written
by tools/import_maps.py: size, obstacles in file order, spawn and objective
lists).  A map name that is an existing file path is parsed as text, exactly
like `os.path.join(fdir, 'maps', abs_path)` passes absolute paths through in
the reference (`gym_env.py:54-56`).
"""
import json
import os

MAPS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "maps")

BOX, WALL = 1, 4  # ZS_THING_BOX / ZS_THING_WALL
_BOX_CHARS = ("☒", "b", "B")   # Box.ICON (things.py:14), 'b', 'B'
_WALL_CHARS = ("▓", "w", "W")  # Wall.ICON (things.py:49), 'w', 'W'


class Map(object):
    """Parsed map: the same content as the reference's `Map` (game.py:34-42).

    `obstacles` is the ordered list of (x, y, kind) for the Box/Wall entries of
    the reference's `map.things` (file order = the order they enter the world's
    dict, game.py:154-155); objectives, player and zombie spawns are (x, y)
    lists in file order.
    """

    def __init__(self, size, obstacles, player_spawns, zombie_spawns, objectives, name=None):
        self.size = tuple(size)
        self.obstacles = [tuple(o) for o in obstacles]
        self.player_spawns = [tuple(p) for p in player_spawns]
        self.zombie_spawns = [tuple(p) for p in zombie_spawns]
        self.objectives = [tuple(p) for p in objectives]
        self.name = name

    @classmethod
    def from_text(cls, text, name=None):
        zombie_spawns, player_spawns, objectives, obstacles = [], [], [], []
        max_row = 0
        max_col = 0
        for row_index, line in enumerate(text.split("\n")):
            if not line:
                continue
            max_row = row_index
            for col_index, char in enumerate(line):
                max_col = max(col_index, max_col)
                position = (col_index, row_index)
                if char in _BOX_CHARS:
                    obstacles.append(position + (BOX,))
                elif char in _WALL_CHARS:
                    obstacles.append(position + (WALL,))
                elif char.lower() == "p":
                    player_spawns.append(position)
                elif char.lower() == "z":
                    zombie_spawns.append(position)
                elif char.lower() == "o":
                    objectives.append(position)
        return cls((max_col + 1, max_row + 1), obstacles, player_spawns, zombie_spawns, objectives, name)

    @classmethod
    def from_file(cls, path):
        with open(path, encoding="utf-8") as f:
            return cls.from_text(f.read(), name=os.path.basename(path))

    @classmethod
    def from_json(cls, path):
        with open(path, encoding="utf-8") as f:
            d = json.load(f)
        return cls(d["size"], d["obstacles"], d["player_spawns"], d["zombie_spawns"], d["objectives"],
                   name=d.get("name"))

    def to_json(self):
        return {"name": self.name, "size": list(self.size),
                "obstacles": [list(o) for o in self.obstacles],
                "player_spawns": [list(p) for p in self.player_spawns],
                "zombie_spawns": [list(p) for p in self.zombie_spawns],
                "objectives": [list(p) for p in self.objectives]}

    @classmethod
    def from_map_name(cls, map_name):
        return load_map(map_name)

    @property
    def things(self):
        """Box/Wall then ObjectiveLocation objects (the reference's `Map.things`, game.py:38-97,
        which interleaves them in file order; only the obstacles' relative order matters)."""
        from .things import OBSTACLE_CLASSES, ObjectiveLocation
        out = [OBSTACLE_CLASSES[k]((x, y)) for (x, y, k) in self.obstacles]
        out += [ObjectiveLocation((x, y)) for (x, y) in self.objectives]
        return out

    # counts used by the reference's tests/test_map.py
    @property
    def n_walls(self):
        return sum(1 for o in self.obstacles if o[2] == WALL)

    @property
    def n_boxes(self):
        return sum(1 for o in self.obstacles if o[2] == BOX)


def available_maps():
    names = set()
    for f in os.listdir(MAPS_DIR):
        base, ext = os.path.splitext(f)
        if ext in (".json", ".txt"):
            names.add(base)
    return sorted(names)


def load_map(map_name):
    """Resolve a reference-style map name or path."""
    if isinstance(map_name, Map):
        return map_name
    if os.path.isfile(map_name) and (os.path.isabs(map_name) or not os.path.exists(
            os.path.join(MAPS_DIR, map_name + ".json"))):
        return Map.from_file(map_name)
    js = os.path.join(MAPS_DIR, map_name + ".json")
    if os.path.isfile(js):
        return Map.from_json(js)
    txt = os.path.join(MAPS_DIR, map_name + ".txt")
    if os.path.isfile(txt):
        m = Map.from_file(txt)
        m.name = map_name
        return m
    raise FileNotFoundError("[Errno 2] No such file or directory: %r" % os.path.join(MAPS_DIR, map_name))
