"""Frame-parallel data parallelism on CPU (gloo, world_size 2): the same code the bench runs over
RCCL, exercised without a GPU."""
import os
import socket
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deformgs.dist import (GradAllReduce, OverlappedGradAllReduce, init_from_env, rank_identical_generator,
                           sync_densification_stats)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _to_np(v):
    """Tensors cross the queue as numpy arrays: a tensor travels as a shared-memory fd that the
    parent can only fetch while the (already exiting) worker still serves it."""
    if isinstance(v, torch.Tensor):
        return ("__t__", v.detach().cpu().numpy())
    if isinstance(v, (list, tuple)):
        return type(v)(_to_np(x) for x in v)
    return v


def _from_np(v):
    if isinstance(v, tuple) and len(v) == 2 and v[0] == "__t__":
        return torch.from_numpy(v[1])
    if isinstance(v, (list, tuple)):
        return type(v)(_from_np(x) for x in v)
    return v


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        r, w, _ = init_from_env("gloo")
        assert (r, w) == (rank, world)
        q.put((rank, _to_np(fn(rank, world))))
    except Exception as e:  # surfaced in the parent
        q.put((rank, e))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, v = q.get(timeout=120)
        out[r] = _from_np(v)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, v in out.items():
        if isinstance(v, Exception):
            raise v
    return out


def _grad_case(rank, world):
    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(s)) for s in [(7, 3), (100,), (5, 5, 2), (3,)]]
    frozen = torch.nn.Parameter(torch.randn(4), requires_grad=False)
    for i, p in enumerate(params[:3]):  # last param: no grad on this step
        p.grad = torch.full_like(p, float(rank + 1) * (i + 1))
    # tiny buckets force several collectives; identical on both ranks
    GradAllReduce(lambda: params + [frozen], bucket_bytes=256)()
    return [None if p.grad is None else p.grad.clone() for p in params], frozen.grad


def _grad_uneven_case(rank, world):
    p = torch.nn.Parameter(torch.zeros(10))
    q = torch.nn.Parameter(torch.zeros(6))
    # rank 0 has q.grad, rank 1 does not: the missing grad contributes zeros
    p.grad = torch.arange(10.0) * (rank + 1)
    if rank == 0:
        q.grad = torch.ones(6) * 4.0
    GradAllReduce(lambda: [p, q])()
    return p.grad.clone(), q.grad.clone()


def _stats_case(rank, world):
    g = types.SimpleNamespace(
        xyz_gradient_accum=torch.full((5, 1), float(rank + 1)),
        denom=torch.full((5, 1), 2.0),
        max_radii2D=torch.tensor([1.0, 5.0, 3.0, 0.0, 2.0]) * (1 if rank == 0 else -1) + rank * 4,
    )
    sync_densification_stats(g)
    return g.xyz_gradient_accum.clone(), g.denom.clone(), g.max_radii2D.clone()


def _gen_case(rank, world):
    gen = rank_identical_generator("cpu", seed=77)
    return torch.randn(16, generator=gen), torch.rand(8, generator=gen)


def test_grad_allreduce_average():
    out = _run(_grad_case)
    grads0, fz0 = out[0]
    grads1, _ = out[1]
    for i in range(3):
        want = torch.full_like(grads0[i], 1.5 * (i + 1))  # mean of (1, 2) * (i + 1)
        torch.testing.assert_close(grads0[i], want)
        torch.testing.assert_close(grads1[i], want)
    # no grad anywhere -> zeros (never None after the step, so the optimizer sees the same on all ranks)
    assert torch.count_nonzero(grads0[3]) == 0 and torch.count_nonzero(grads1[3]) == 0
    assert fz0 is None  # frozen params are skipped


def test_grad_allreduce_missing_grad_counts_as_zero():
    out = _run(_grad_uneven_case)
    for r in (0, 1):
        pg, qg = out[r]
        torch.testing.assert_close(pg, torch.arange(10.0) * 1.5)
        torch.testing.assert_close(qg, torch.full((6,), 2.0))


def test_sync_densification_stats():
    out = _run(_stats_case)
    for r in (0, 1):
        acc, den, rad = out[r]
        torch.testing.assert_close(acc, torch.full((5, 1), 3.0))
        torch.testing.assert_close(den, torch.full((5, 1), 4.0))
        torch.testing.assert_close(rad, torch.tensor([3.0, 5.0, 3.0, 4.0, 2.0]))


def test_rank_identical_generator():
    out = _run(_gen_case)
    torch.testing.assert_close(out[0][0], out[1][0], rtol=0, atol=0)
    torch.testing.assert_close(out[0][1], out[1][1], rtol=0, atol=0)


def test_single_process_is_noop():
    p = torch.nn.Parameter(torch.ones(3))
    p.grad = torch.full((3,), 2.0)
    GradAllReduce(lambda: [p])()
    torch.testing.assert_close(p.grad, torch.full((3,), 2.0))
    sync_densification_stats(types.SimpleNamespace())  # not initialised -> untouched


def _overlap_case(rank, world):
    """Early group (a, b) reduced by the post-accumulate hooks during backward, late group (c) after;
    step 2: on rank 1 `b` gets no gradient, so its hook group never completes there (fallback)."""
    a = torch.nn.Parameter(torch.zeros(7))
    b = torch.nn.Parameter(torch.zeros(3, 2))
    c = torch.nn.Parameter(torch.zeros(5))
    ar = OverlappedGradAllReduce(lambda: [a, b], lambda: [c])
    out = []
    for step in range(2):
        for p in (a, b, c):
            p.grad = None
        ar.arm()
        s = (rank + 1.0)
        loss = (s * torch.arange(7.0) * a).sum() + (2 * s * c).sum()
        if not (step == 1 and rank == 1):
            loss = loss + (3 * s * b).sum()
        loss.backward()
        fired = ar._pending is not None
        ar()
        out.append((fired, a.grad.clone(), None if b.grad is None else b.grad.clone(), c.grad.clone()))
    return out


def test_overlapped_grad_allreduce():
    out = _run(_overlap_case)
    for rank in (0, 1):
        (f0, a0, b0, c0), (f1, a1, b1, c1) = out[rank]
        assert f0, "the early group's hook must start the collective during backward"
        torch.testing.assert_close(a0, 1.5 * torch.arange(7.0))
        torch.testing.assert_close(b0, torch.full((3, 2), 4.5))
        torch.testing.assert_close(c0, torch.full((5,), 3.0))
        assert f1 == (rank == 0)  # rank 1 had no b gradient in step 2: reduced in __call__ instead
        torch.testing.assert_close(a1, 1.5 * torch.arange(7.0))
        torch.testing.assert_close(b1, torch.full((3, 2), 1.5))  # (3 * 1 + 0) / 2
        torch.testing.assert_close(c1, torch.full((5,), 3.0))


def _agreement_case(rank, world):
    """OverflowAgreement: any rank's overflow makes every rank redo; an early collective of the
    discarded step completes on every rank and the redone step's reduction is the one kept."""
    from deformgs.dist import OverflowAgreement
    agree = OverflowAgreement()
    votes = [agree(False), agree(rank == 1), agree(rank == 0), agree(True)]
    a = torch.nn.Parameter(torch.zeros(4))
    c = torch.nn.Parameter(torch.zeros(2))
    ar = OverlappedGradAllReduce(lambda: [a], lambda: [c])
    ar.arm()
    ((rank + 1.0) * 100 * a).sum().backward()  # the overflowed step's gradients: discarded
    started = ar._pending is not None
    if agree(rank == 1):
        ar.discard()
        a.grad = None
        ar.arm()
        ((rank + 1.0) * a).sum().backward()
    (c * (rank + 1.0)).sum().backward()
    ar()
    return votes, started, a.grad.clone(), c.grad.clone()


def test_overflow_agreement_and_discard():
    out = _run(_agreement_case)
    for rank in (0, 1):
        votes, started, ag, cg = out[rank]
        assert votes == [False, True, True, True]
        assert started
        torch.testing.assert_close(ag, torch.full((4,), 1.5))
        torch.testing.assert_close(cg, torch.full((2,), 1.5))


def test_viewpoint_stack_matches_reference_formula():
    """train_baseline.py:80-89: sorted by fid, int(round(i * (total - 1) / (sequence_length - 1)))."""
    from deformgs.train import build_viewpoint_stack
    cams = [types.SimpleNamespace(fid=torch.tensor([f])) for f in torch.rand(47, generator=torch.Generator().manual_seed(1))]
    st = build_viewpoint_stack(cams, 30)
    srt = sorted(cams, key=lambda c: float(c.fid))
    step = (47 - 1) / (30 - 1)
    assert [id(c) for c in st] == [id(srt[int(round(i * step))]) for i in range(30)]
    assert [float(c.fid) for c in st] == sorted(float(c.fid) for c in st)
    # more frames asked for than exist: indices repeat, as upstream
    st2 = build_viewpoint_stack(cams[:5], 9)
    assert len(st2) == 9 and len({id(c) for c in st2}) == 5


def _agreement_uneven_case(rank, world):
    """The discarded step: on rank 1 the early parameter b gets no gradient, so its hook group never
    completes there and no early collective starts; discard() must issue the throwaway early
    reduction on rank 1 to pair with rank 0's, then the redone step reduces normally."""
    from deformgs.dist import OverflowAgreement
    agree = OverflowAgreement()
    a = torch.nn.Parameter(torch.zeros(4))
    b = torch.nn.Parameter(torch.zeros(3))
    c = torch.nn.Parameter(torch.zeros(2))
    ar = OverlappedGradAllReduce(lambda: [a, b], lambda: [c])
    ar.arm()
    loss = ((rank + 1.0) * 100 * a).sum()
    if rank == 0:
        loss = loss + (7.0 * b).sum()
    loss.backward()
    started = ar._pending is not None
    assert agree(rank == 0)
    ar.discard()
    for p in (a, b, c):
        p.grad = None
    ar.arm()
    ((rank + 1.0) * a).sum().backward()
    ((rank + 1.0) * 2 * b).sum().backward()
    (c * (rank + 1.0)).sum().backward()
    ar()
    # one more plain step: collectives still paired
    for p in (a, b, c):
        p.grad = None
    ar.arm()
    ((rank + 1.0) * (a.sum() + b.sum())).backward()
    (c * 3.0).sum().backward()
    ar()
    return started, a.grad.clone(), b.grad.clone(), c.grad.clone()


def test_overflow_discard_when_one_rank_missed_the_early_hook():
    out = _run(_agreement_uneven_case)
    assert out[0][0] and not out[1][0]
    for rank in (0, 1):
        _, ag, bg, cg = out[rank]
        torch.testing.assert_close(ag, torch.full((4,), 1.5))
        torch.testing.assert_close(bg, torch.full((3,), 1.5))
        torch.testing.assert_close(cg, torch.full((2,), 3.0))


def _warmup_late_case(rank, world):
    """A warm-up iteration: the late group (the network) has no gradient on any rank; it is not
    reduced and keeps .grad None (Adam skips it, as on one rank); the early group is reduced."""
    a = torch.nn.Parameter(torch.zeros(4))
    c = torch.nn.Parameter(torch.zeros(2))
    ar = OverlappedGradAllReduce(lambda: [a], lambda: [c])
    ar.arm()
    ((rank + 1.0) * a).sum().backward()
    ar()
    return a.grad.clone(), c.grad


def test_warmup_network_gradients_stay_none():
    out = _run(_warmup_late_case)
    for rank in (0, 1):
        ag, cg = out[rank]
        torch.testing.assert_close(ag, torch.full((4,), 1.5))
        assert cg is None


def _native_dp_case(rank, world):
    """NativeStep.step_data_parallel's collective sequence with the C calls stubbed (CPU tensors):
    phase 1, the redo of an overflowed pair count by that rank ALONE (rank 1: no agreement, no host
    collective), the Gaussian all-reduce, phase 2, the network all-reduce; a warm-up step has no
    network collective."""
    from deformgs.native_step import NativeStep, _flat_views

    class Stub(NativeStep):
        def __init__(self):
            self.calls = []
            self.gflat, self.gviews = _flat_views([torch.zeros(3, 2), torch.zeros(5)])
            self.mflat, self.mviews = _flat_views([torch.zeros(4)])

        def __call__(self, cam, gt, bg, warm, noise, lam, deferred, phase=0):
            self.calls.append(("p1", deferred))
            self._warm = warm
            self.gflat.fill_((rank + 1.0) * (10.0 if deferred else 1.0))
            return torch.tensor(float(rank)), {}, bool(deferred and rank == 1)

        def network_backward(self):
            self.calls.append(("p2",))
            self.mviews[0].copy_(torch.arange(4.0) * (rank + 1))

    ns = Stub()
    out = []
    for warm, deferred in ((True, True), (False, False)):
        ns.calls.clear()
        ns.mflat.fill_(-1.0)
        loss, _, redone = ns.step_data_parallel(None, None, None, warm, 0.0, 0.2, deferred)
        out.append((list(ns.calls), redone, ns.gviews[0].clone(), ns.gviews[1].clone(), ns.mviews[0].clone()))
    return out


def test_native_data_parallel_step_sequence():
    out = _run(_native_dp_case)
    for rank in (0, 1):
        (c0, r0, g0a, g0b, m0), (c1, r1, g1a, g1b, m1) = out[rank]
        if rank == 1:  # its overflow is redone (synchronously) by this rank alone
            assert c0 == [("p1", True), ("p1", False), ("p2",)] and r0
        else:
            assert c0 == [("p1", True), ("p2",)] and not r0
        torch.testing.assert_close(g0a, torch.full((3, 2), 6.0))  # mean of rank 0's 10 and rank 1's redone 2
        torch.testing.assert_close(g0b, torch.full((5,), 6.0))
        torch.testing.assert_close(m0, 1.5 * torch.arange(4.0))
        assert c1 == [("p1", False)] and not r1  # warm-up: no phase 2, no network collective
        torch.testing.assert_close(g1a, torch.full((3, 2), 1.5))
        torch.testing.assert_close(m1, torch.full((4,), -1.0))


def _path_agreement_case(rank, world):
    """train_step's native-vs-autograd choice with several ranks: the ranks MIN-reduce
    their local native_step.usable flag when a rank-invariant key changes (Gaussian count, image size,
    configuration) and reuse it otherwise; a rank forced onto the fallback pulls every rank onto the
    autograd path (matching collectives) instead of splitting them; a rank that loses the native path
    without a key change raises instead of issuing mismatched collectives. C calls stubbed (CPU)."""
    from deformgs import native_step, train_step as ts
    usable = {"v": rank == 0}
    calls = []
    native_step.usable = lambda *a, **k: usable["v"]

    class StubNative:
        def __init__(self, gs, deform):
            self.deform = deform

        def step_data_parallel(self, *a, **k):
            calls.append("native")
            return torch.tensor(0.0), {}, False

    native_step.NativeStep = StubNative

    def stub_fb(*a, **k):
        calls.append("autograd")
        return torch.tensor(0.0), {}

    ts.forward_backward = stub_fb

    class AR:
        group = None

        def world(self):
            return world

        def arm(self):
            pass

        def __call__(self):
            pass

    net = types.SimpleNamespace(is_6dof=False, flags=0, exact_fp32=False)
    deform = types.SimpleNamespace(deform=net)
    gt = torch.zeros(3, 8, 8)

    def gaussians(n):
        return types.SimpleNamespace(_xyz=torch.zeros(n, 3), _features_rest=torch.zeros(n, 15, 3))

    gs = gaussians(10)
    out = []
    for _ in range(2):  # rank 1 cannot: both take the autograd path; the second step reuses the choice
        ts.train_step(gs, deform, None, gt, types.SimpleNamespace(), None, deferred_count=False, allreduce=AR())
    out.append(list(calls))
    calls.clear()
    usable["v"] = True  # both could now, but the key is unchanged: the agreed choice stays
    ts.train_step(gs, deform, None, gt, types.SimpleNamespace(), None, deferred_count=False, allreduce=AR())
    out.append(list(calls))
    calls.clear()
    gs = gaussians(12)  # densification (same count on every rank): agreed again, both native
    ts.train_step(gs, deform, None, gt, types.SimpleNamespace(), None, deferred_count=False, allreduce=AR())
    out.append(list(calls))
    calls.clear()
    # each rank renders its own camera, whose size may change on one rank only (the reference's
    # readers allow a per-camera width / height): not a key change, so no lone 1-int collective that
    # would pair with another rank's gradient all-reduce
    gt_r = torch.zeros(3, 8, 8 + 4 * rank)
    for _ in range(2):
        ts.train_step(gs, deform, None, gt_r, types.SimpleNamespace(), None, deferred_count=False, allreduce=AR())
    out.append(list(calls))
    calls.clear()
    usable["v"] = rank == 0  # rank 1 loses the path without a key change: it raises
    try:
        ts.train_step(gs, deform, None, gt, types.SimpleNamespace(), None, deferred_count=False, allreduce=AR())
        out.append(list(calls))
    except RuntimeError as e:
        out.append("raised" if "collectives would not match" in str(e) else repr(e))
    return out


def test_native_path_choice_is_agreed_across_ranks():
    out = _run(_path_agreement_case)
    for rank in (0, 1):
        a, b, c, e, d = out[rank]
        assert a == ["autograd", "autograd"]
        assert b == ["autograd"]
        assert c == ["native"]
        assert e == ["native", "native"]
        assert d == (["native"] if rank == 0 else "raised")


def test_rccl_group_reserves_cus_for_the_collective(monkeypatch):
    """reserve_cus_for_collectives (opt-in: DGS_OVERLAP_RESERVE=1 before an RCCL group): NCCL_MAX_NCHANNELS
    defaults to OVERLAP_CUS and the MLP kernels leave that many CUs free (the library knob; a host-side
    setter, no GPU needed); explicit settings win. By default nothing is reserved."""
    import inspect
    from deformgs import dist as dgs_dist
    assert 'os.environ.get("DGS_OVERLAP_RESERVE", "0") == "1"' in inspect.getsource(dgs_dist.init_from_env)
    from deformgs import _lib
    from deformgs.dist import OVERLAP_CUS, reserve_cus_for_collectives
    lib = _lib.load()
    monkeypatch.delenv("NCCL_MAX_NCHANNELS", raising=False)
    monkeypatch.delenv("DGS_MLP_RESERVE_CUS", raising=False)
    try:
        reserve_cus_for_collectives()
        assert os.environ["NCCL_MAX_NCHANNELS"] == str(OVERLAP_CUS)
        assert lib.dgs_mlp_reserved_cus() == OVERLAP_CUS
        monkeypatch.setenv("NCCL_MAX_NCHANNELS", "16")
        reserve_cus_for_collectives()
        assert lib.dgs_mlp_reserved_cus() == 16
        lib.dgs_mlp_set_reserved_cus(3)
        monkeypatch.setenv("DGS_MLP_RESERVE_CUS", "3")
        reserve_cus_for_collectives()
        assert lib.dgs_mlp_reserved_cus() == 3  # an explicit reserve is left alone
    finally:
        lib.dgs_mlp_set_reserved_cus(0)
