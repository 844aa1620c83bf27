"""Frame-parallel training step with 2 ranks on the one GPU of the box: two fresh
child processes (DGS_DEVICE=0, DGS_DIST_BACKEND=gloo) each render their own camera through
train_step (deferred pair count, overlapped gradient all-reduce, overflow redo), then
Adam. Checks: the averaged gradients equal the mean of the two single-rank steps computed here (the
blend backward sums float atomics in arrival order: 1e-4 relative + 1e-6 of the tensor's max), and the
post-Adam parameters are bitwise identical on both ranks. "overflow": rank 1's speculative pair
capacity is forced to overflow: on the autograd path BOTH ranks must redo (the agreement), on the native
path (NativeStep.step_data_parallel) rank 1 redoes alone, its count being known before any collective;
the result is unchanged either way.
RCCL refuses two ranks on one GPU, so these carry the collectives over gloo; RCCL itself runs with a
one-rank group in test_rccl_group_runs_the_data_parallel_step.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

from conftest import ROOT, gpu_available

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _single_rank_grads(six=False):
    sys.path.insert(0, HERE)
    from dist_step_worker import build, params_of
    from deformgs.arguments import PipelineParams
    from deformgs.train_step import train_step
    dev = torch.device("cuda", 0)
    out = []
    for k in range(2):
        gs, deform, cams, gts = build(dev, six=six)
        train_step(gs, deform, cams[k], gts[k], PipelineParams(), torch.zeros(3, device=dev), six, deferred_count=False)
        out.append([p.grad.detach().clone().cpu() for p in params_of(gs, deform)])
    return out


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("path", ["native", "autograd"])
@pytest.mark.parametrize("mode", ["plain", "overflow", "6dof"])
def test_two_rank_step_averages_gradients(tmp_path, mode, path):
    """mode 6dof: config 4's screw deformation head (trex --is_6dof), plain deferred step. path: the
    native step's two calls around the Gaussian gradient all-reduce (NativeStep.step_data_parallel) or
    the autograd step with the post-accumulate-grad hooks (DGS_NATIVE_STEP=0)."""
    six = mode == "6dof"
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), DGS_DEVICE="0", DGS_DIST_BACKEND="gloo",
                   DGS_NATIVE_STEP="1" if path == "native" else "0")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_step_worker.py"), str(tmp_path),
                                       "plain" if six else mode] + (["6dof"] if six else []), env=env, cwd=ROOT))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=100))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(-9)
    assert rcs == [0, 0], rcs
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert r0["native"] == r1["native"] == (path == "native")
    if mode == "overflow" and path == "native":  # the overflowing rank redoes alone, before any collective
        assert r1["redone"] and not r0["redone"]
    elif mode == "overflow":
        assert r0["redone"] and r1["redone"], "an overflow on one rank must be redone on every rank"
    else:
        assert not r0["redone"] and not r1["redone"]
    single = _single_rank_grads(six)
    for i, (a, b, s0, s1) in enumerate(zip(r0["grads"], r1["grads"], *single)):
        assert torch.equal(a, b), f"reduced gradient {i} differs between ranks"
        want = (s0 + s1) / 2
        tol = 1e-6 * float(want.abs().max()) + 1e-4 * want.abs()
        assert bool(((a - want).abs() <= tol).all()), (i, float((a - want).abs().max()))
    for i, (a, b) in enumerate(zip(r0["params"], r1["params"])):
        assert torch.equal(a, b), f"parameter {i} differs between ranks after Adam"


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("variant", ["blender", "nonblender"])
def test_two_rank_loop_stays_replicated_through_densification(tmp_path, variant):
    """The training LOOP (deformgs/train.py training(), train_baseline.py:56-182) with 2 ranks on the one
    GPU (gloo): 34 iterations across the warm-up boundary, three densify_and_prune calls, an opacity
    reset and the stack refill (tests/dist_loop_worker.py). Replicas must stay IDENTICAL (SURVEY.md
    §8e): at every densify / reset iteration and at the end, the Gaussian count and every Gaussian and
    network parameter are bitwise equal on both ranks (the per-rank densification statistics are summed /
    maxed across ranks right before densify_and_prune, and the split noise is rank-identical). The loop must actually densify (the count changes)."""
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), DGS_DEVICE="0", DGS_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_loop_worker.py"), str(tmp_path),
                                       variant], env=env, cwd=ROOT))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=110))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(-9)
    assert rcs == [0, 0], rcs
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert r0["n"] == r1["n"], (r0["n"], r1["n"])
    n = r0["n"]
    assert n[9] != n[8], "the first densify_and_prune (iteration 10) must change the count"
    assert r0["expiries"] == 0 and r1["expiries"] == 0
    for it in sorted(r0["snaps"]):
        a, b = r0["snaps"][it], r1["snaps"][it]
        assert a["n"] == b["n"], it
        for i, (x, y) in enumerate(zip(a["params"], b["params"])):
            assert torch.equal(x, y), f"iteration {it}: parameter {i} differs between ranks"
    for i, (x, y) in enumerate(zip(r0["end"]["params"], r1["end"]["params"])):
        assert torch.equal(x, y), f"end: parameter {i} differs between ranks"
    # the ranks rendered different frames: their local losses differ (the test is not vacuous)
    assert r0["loss"] != r1["loss"]


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("reserve", [False, True])
def test_rccl_group_runs_the_data_parallel_step(tmp_path, reserve):
    """RCCL itself on the box's one GPU (tests/rccl1_worker.py): a "nccl" process group of one rank,
    AVG / SUM / MAX and an async all-reduce on a side stream leave the values bitwise unchanged, and the
    data-parallel step's RCCL-only branches (native step_data_parallel, the autograd path's overlapped
    reducer, the device-side path agreement; reserve: the opt-in CU reserve and channel cap) run and give
    the gradients of an un-reduced step (blend atomics: 1e-4 relative + 1e-6 of the tensor's max)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    for k in ("NCCL_MAX_NCHANNELS", "DGS_MLP_RESERVE_CUS", "DGS_NATIVE_STEP"):
        env.pop(k, None)
    p = subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "rccl1_worker.py"), str(tmp_path)]
                         + (["reserve"] if reserve else []), env=env, cwd=ROOT)
    try:
        rc = p.wait(timeout=100)
    except subprocess.TimeoutExpired:
        p.kill()
        rc = -9
    assert rc == 0, rc
    r = torch.load(tmp_path / "rccl.pt", weights_only=True)
    assert r["backend"] == "nccl" and r["avg"], r
    assert all(r["ops"].values()), r["ops"]
    assert r["nchannels"] == ("32" if reserve else None)
    assert r["reserved_cus"] == (32 if reserve else 0)
    steps = r["steps"]
    for path in ("native", "autograd"):
        local, red = steps[f"{path}-local"], steps[f"{path}-rccl"]
        assert local["native"] == red["native"] == (path == "native")
        assert not local["redone"] and not red["redone"]
        # the local steps issue no collective; the reduced ones go through the RCCL branches: native =
        # two step_data_parallel calls, each with async Gaussian + network all-reduces (warm) after
        # the path agreement (one sync MIN); autograd = the hooks' async early reduce + the late one
        assert local["calls"] == {"allreduce_async": 0, "allreduce_sync": 0, "dp_steps": 0}, local["calls"]
        c = red["calls"]
        if path == "native":
            assert c["dp_steps"] == 2 and c["allreduce_async"] == 4 and c["allreduce_sync"] == 1, c
        else:
            assert c["dp_steps"] == 0 and c["allreduce_async"] == 2 and c["allreduce_sync"] >= 2, c
        assert abs(local["loss"] - red["loss"]) <= 1e-6 * abs(local["loss"])
        for i, (a, want) in enumerate(zip(red["grads"], local["grads"])):
            tol = 1e-6 * float(want.abs().max()) + 1e-4 * want.abs()
            assert bool(((a - want).abs() <= tol).all()), (path, i, float((a - want).abs().max()))
