"""C-ABI library: loads without a GPU and exports every entry point include/ declares."""
import ctypes
import os
import re

from libzombsole_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "zombsole_mi355x.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(zs_\w+)\s*\(", src, re.M)))


def test_header_declares_the_binding_list():
    assert declared_symbols() == sorted(engine.SYMBOLS)


def test_library_loads_and_exports_all_symbols():
    L = engine.load_library()
    for s in declared_symbols():
        assert hasattr(L, s), s
        assert ctypes.cast(getattr(L, s), ctypes.c_void_p).value


def test_library_is_gfx950_code_object():
    data = open(engine.LIB_PATH, "rb").read()
    assert b"gfx950" in data
