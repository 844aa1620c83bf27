"""bench.py's output line keeps the driver's contract (task README / DESIGN.md §5): one JSON line on
stdout with the required keys, a whole-job value consistent with ms_per_step, and the roofline
object of the dominant kernel (frac = achieved / peak). A short run (one child process, small
scene, no CPU leg) — the numbers are not checked, the shape is."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

REQUIRED = {"metric": str, "value": float, "unit": str, "n_gpus": int, "steps": int, "warmup": int,
            "ms_per_step": float, "higher_is_better": bool, "scaling": str, "dtype": str, "data": str,
            "config": dict, "roofline": dict}


def test_bench_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "8", "--warmup", "2", "--n", "20000",
           "--res", "256", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    for k, t in REQUIRED.items():
        assert k in d, k
        assert isinstance(d[k], t) or (t is float and isinstance(d[k], int)), (k, type(d[k]))
    assert d["n_gpus"] == 1 and d["steps"] == 8 and d["warmup"] == 2
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    assert "vs_baseline" in d
    # whole-job throughput: iterations per second of the timed steps
    assert d["value"] == pytest.approx(1000.0 / d["ms_per_step"], rel=1e-6)
    assert "workload" in d["config"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] in ("hbm", "mfma") and r["unit"] in ("GB/s", "TFLOP/s")
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-6)
    assert 0.0 < r["frac"] < 1.0


def test_bench_self_launches_two_ranks_gloo_rehearsal():
    """`bench.py --gpus 2` invoked directly (no WORLD_SIZE) launches its own two ranks through
    torch.distributed.run; on a one-GPU box both ranks share cuda:0 over gloo (DGS_DEVICE=0,
    DGS_DIST_BACKEND=gloo: RCCL refuses two ranks on one GPU). Rank 0's single line reports n_gpus 2, the
    backend and what every rank saw."""
    env = dict(os.environ, DGS_DEVICE="0", DGS_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--n", "20000", "--res", "256", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2
    assert d["dist"]["world_size"] == 2 and d["dist"]["backend"] == "gloo"
    assert sorted(r["rank"] for r in d["dist"]["ranks"]) == [0, 1]
    assert all(r["world_seen"] == 2 for r in d["dist"]["ranks"])
    assert d["value"] == pytest.approx(2 * 1000.0 / d["ms_per_step"], rel=1e-6)
