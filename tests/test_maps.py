"""Map loading (host side): the reference's tests/test_map.py facts plus the synthetic maps."""
import pytest

from libzombsole_amd.game import Map
from libzombsole_amd.maps import available_maps, load_map
from libzombsole_amd.things import Box, ObjectiveLocation, Wall


# tests/test_map.py:5-24 of the reference
@pytest.mark.parametrize("map_name,exp_map_size,exp_walls_count,exp_objs_count", [
    ("bridge", (111, 12), 182, 28),
    ("boxed", (15, 8), 14, 0),
    ("fort", (73, 21), 210, 0),
])
def test_map_read(map_name, exp_map_size, exp_walls_count, exp_objs_count):
    lmap = Map.from_map_name(map_name)
    assert lmap.size == exp_map_size
    objectives_count = 0
    walls_count = 0
    for thing in lmap.things:
        if isinstance(thing, (Wall,)):
            walls_count += 1
        elif isinstance(thing, (ObjectiveLocation,)):
            objectives_count += 1
    assert walls_count == exp_walls_count
    assert objectives_count == exp_objs_count


def test_reference_maps_bundled():
    names = set(available_maps())
    for n in ("arduino", "boxed", "bridge", "city_for_evacuation", "city_for_safehouse", "easy_exit",
              "easy_exit_v2", "fort", "hallway", "maze_for_safehouse", "to_the_closet",
              "village_for_evacuation", "village_for_safehouse", "bridge64", "city128"):
        assert n in names


def test_synthetic_maps_shape():
    b = load_map("bridge64")
    assert b.size == (64, 64)
    assert b.player_spawns and b.zombie_spawns and b.objectives
    c = load_map("city128")
    assert c.size == (128, 128)
    # obstacles never overlap and stay in bounds
    for m in (b, c):
        cells = [(x, y) for x, y, _ in m.obstacles]
        assert len(set(cells)) == len(cells)
        assert all(0 <= x < m.size[0] and 0 <= y < m.size[1] for x, y in cells)


def test_map_text_parser_rules():
    # game.py:45-97: column = x, row = y; empty lines keep their row index; spaces count
    m = Map.from_text("#w b\n\n p z o\nB")
    assert m.size == (6, 4)
    assert m.obstacles == [(1, 0, 4), (3, 0, 1), (0, 3, 1)]
    assert m.player_spawns == [(1, 2)] and m.zombie_spawns == [(3, 2)] and m.objectives == [(5, 2)]
    assert all(isinstance(t, (Box, Wall, ObjectiveLocation)) for t in m.things)


def test_missing_map():
    with pytest.raises(FileNotFoundError):
        load_map("no_such_map")
