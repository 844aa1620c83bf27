"""bench.py --gpus N launches its own ranks: without WORLD_SIZE and N > 1 the parent
makes no GPU call and runs `python -m torch.distributed.run --nproc-per-node N bench.py <same args>` as a
child process (subprocess, never exec), exiting with its return code. CPU only: the command is checked,
the child is stubbed."""
import os
import subprocess
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)


def test_launcher_command():
    import bench
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd = bench.launcher_cmd(argv, 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    j = cmd.index("--master-port")
    assert cmd[j + 1] == "29511"
    assert cmd[j + 2] == os.path.join(ROOT, "bench.py")
    assert cmd[j + 3:] == argv


def test_maybe_launch_runs_child_and_returns_its_code(monkeypatch):
    import bench
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 3

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    args = bench.parse(["--gpus", "2", "--steps", "4"])
    assert bench.maybe_launch(args, ["--gpus", "2", "--steps", "4"]) == 3
    assert "--nproc-per-node=2" in seen["cmd"] and seen["cmd"][-4:] == ["--gpus", "2", "--steps", "4"]
    # one GPU, or already a rank of a launched job: no child
    assert bench.maybe_launch(bench.parse(["--gpus", "1"]), []) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.maybe_launch(args, []) is None
