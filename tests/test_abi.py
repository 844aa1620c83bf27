"""CPU: libdgs_hip.so loads and exports every entry point include/dgs.h declares (no compute calls)."""
import ctypes
import os
import re

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "dgs.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dgs_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    from deformgs import _lib
    lib = _lib.load()
    names = _declared()
    assert len(names) >= 18
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/dgs.h but not exported"
    # and the Python binding declares a signature for every one of them
    assert set(names) == set(_lib.EXPORTED)


def test_host_only_queries():
    from deformgs import _lib
    lib = _lib.load()
    assert b"gfx950" in lib.dgs_version()
    # blender: 26 tensors, 522,280 parameters packed with padding
    assert lib.dgs_deform_num_params(1) == 26
    assert lib.dgs_deform_num_params(0) == 22
    assert lib.dgs_deform_num_params(3) == 28
    assert lib.dgs_deform_outputs(1) == 10 and lib.dgs_deform_outputs(3) == 13
    # activations, relu bits (2 blocks + room for 3 more 16-point tail slots each), timenet
    assert lib.dgs_deform_saved_floats(1, 100) == 2416 * 128 + 2304 * 2 * (2 + 3 * 2) + 1024  # TC_FLOATS: t0 | TIN | TE | TH | C0 | C5
    assert lib.dgs_deform_packed_floats(1) > 522280


def test_library_is_gfx950_code_object():
    from deformgs import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert ctypes.CDLL(_lib.LIB_PATH)
