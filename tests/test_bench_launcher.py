"""bench.py --gpus N launches its own ranks: without WORLD_SIZE and N > 1 the parent
makes no GPU call and runs `python -m torch.distributed.run --nproc-per-node N bench.py <same args>` as a
child process (subprocess, never exec), exiting with its return code. CPU only: the command is checked,
the child is stubbed."""
import json
import os
import subprocess
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)


def test_launcher_command():
    import bench
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd, env = bench.launcher_cmd(argv, 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    j = cmd.index("--master-port")
    assert cmd[j + 1] == "29511"
    assert cmd[j + 2:] == [os.path.join(ROOT, "bench.py")]
    # the bench's own arguments travel in the environment (torch.distributed.run matches option prefixes
    # such as --n even after the script name)
    assert json.loads(env[bench.ARGV_ENV]) == argv
    assert bench.parse(json.loads(env[bench.ARGV_ENV])).gpus == 8


def test_torchrun_accepts_the_command():
    """torch.distributed.run's own parser takes the launcher's command (with the bench arguments that
    broke it on the command line, e.g. --n)."""
    import bench
    from torch.distributed.run import get_args_parser
    cmd, _ = bench.launcher_cmd(["--n", "20000", "--res", "256"], 2, 29512)
    a = get_args_parser().parse_args(cmd[3:])
    assert a.nproc_per_node == "2" and a.training_script == os.path.join(ROOT, "bench.py")
    assert a.training_script_args == []


def test_maybe_launch_runs_child_and_returns_its_code(monkeypatch):
    import bench
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 3

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    args = bench.parse(["--gpus", "2", "--steps", "4"])
    assert bench.maybe_launch(args, ["--gpus", "2", "--steps", "4"]) == 3
    assert "--nproc-per-node=2" in seen["cmd"]
    assert json.loads(seen["env"][bench.ARGV_ENV]) == ["--gpus", "2", "--steps", "4"]
    # one GPU, or already a rank of a launched job: no child
    assert bench.maybe_launch(bench.parse(["--gpus", "1"]), []) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.maybe_launch(args, []) is None
