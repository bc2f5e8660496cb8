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


def test_struct_layout_matches_header(tmp_path):
    """The ctypes mirrors of zs_map_desc / zs_launch / zs_config (libzombsole_amd/_abi.py) have the
    header's sizes and field offsets (gcc on the header itself)."""
    import subprocess

    from libzombsole_amd import _abi
    structs = {"zs_map_desc": _abi.zs_map_desc, "zs_launch": _abi.zs_launch, "zs_config": _abi.zs_config}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "zombsole_mi355x.h"', 'int main(void) {']
    for name, cls in structs.items():
        lines.append('printf("%s sizeof %%zu\\n", sizeof(%s));' % (name, name))
        for f in cls._fields_:
            lines.append('printf("%s %s %%zu\\n", offsetof(%s, %s));' % (name, f[0], name, f[0]))
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    got = dict((" ".join(l.split()[:2]), int(l.split()[2])) for l in subprocess.check_output([str(exe)]).decode().splitlines())
    for name, cls in structs.items():
        assert got["%s sizeof" % name] == ctypes.sizeof(cls), name
        for f in cls._fields_:
            assert got["%s %s" % (name, f[0])] == getattr(cls, f[0]).offset, (name, f[0])


def test_checked_launder_build_compiles(tmp_path):
    """The kernels that reload their Dev from kernarg offset 0 (zs_launder_dev: k_reset, k_respawn here) build
    with the contract check on (-DZS_CHECK_LAUNDER: the reloaded fields against the kernel's argument)."""
    import subprocess
    import __graft_entry__ as ge
    subprocess.check_call([ge._hipcc()] + ge.HIPCC_FLAGS + ["-DZS_CHECK_LAUNDER", "-c", "-o", str(tmp_path / "k_reset.o"),
                                                         os.path.join(ge.CSRC, "k_reset.hip")])
