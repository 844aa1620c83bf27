"""The ctypes mirrors of include/dgs.h's argument structs have the C layout (CPU, no GPU): a small C
program built with gcc against the header prints sizeof and every field's offsetof, which must equal
the ctypes Structure's. A field added on one side only (e.g. dgs_train_step_args.phase) fails here
instead of as garbage arguments on the GPU."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

STRUCTS = [
    ("dgs_raster_settings", "deformgs._lib", "RasterSettings"),
    ("dgs_adam_tensor", "deformgs._lib", "AdamTensor"),
    ("dgs_row_job", "deformgs._lib", "RowJob"),
    ("dgs_train_step_args", "deformgs.native_step", "TrainStepArgs"),
]


def _ctypes_cls(mod, name):
    import importlib
    return getattr(importlib.import_module(mod), name)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_ctypes_mirrors_match_the_header(tmp_path):
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "dgs.h"', "int main(void) {"]
    for cname, mod, cls in STRUCTS:
        C = _ctypes_cls(mod, cls)
        lines.append(f'  printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f, _ in C._fields_:
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {}
    for line in out:
        if line.strip():
            s, f, v = line.split()
            got[(s, f)] = int(v)
    for cname, mod, cls in STRUCTS:
        C = _ctypes_cls(mod, cls)
        import ctypes
        assert got[(cname, "sizeof")] == ctypes.sizeof(C), cname
        for f, _ in C._fields_:
            assert got[(cname, f)] == getattr(C, f).offset, (cname, f)
