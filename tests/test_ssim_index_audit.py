"""Host audit of the fused SSIM kernels' addressing (tools/ssim_index_audit.cpp): every thread of every
workgroup of k_ssim_fwd / k_ssim_final / k_ssim_bwd replayed on the CPU with the kernels' index
expressions, each global and LDS address checked against its buffer's extent, for the shapes the GPU
loss tests use (tests/test_gpu_loss.py, among them the (3,61,83) run that preceded the r4v abort) and
ragged / degenerate ones. No GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_ssim_addresses_in_bounds(tmp_path):
    exe = tmp_path / "ssim_index_audit"
    subprocess.run(["g++", "-O2", "-Wall", "-o", str(exe), os.path.join(ROOT, "tools", "ssim_index_audit.cpp")],
                   check=True)
    shapes = [(3, 61, 83), (1, 16, 16), (3, 5, 200), (3, 256, 256), (3, 400, 400), (1, 1, 1), (2, 33, 31),
              (3, 32, 32), (3, 31, 65)]
    args = [str(v) for s in shapes for v in s]
    r = subprocess.run([str(exe)] + args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("0 out of bounds") == len(shapes), r.stdout
