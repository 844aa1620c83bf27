"""Host-side glue of the HIP training path, checked on the CPU (no kernel launches):
Adam's shared per-optimizer step tensors keep torch.optim.Adam's per-parameter step counts, and
render() recognises the deformation outputs it can hand to the fused input launches."""
import types

import torch

from deformgs import adam as dgs_adam
from deformgs import renderer


def test_adam_shared_step_counts_match_torch():
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(5, 3)) for _ in range(4)]
    rs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    ours = dgs_adam.Adam([{"params": [p], "lr": 1e-3} for p in ps], lr=0.0, eps=1e-15)
    ours._hip = True  # exercise the HIP path's bookkeeping (_collect) on CPU tensors, no launch
    ref = torch.optim.Adam([{"params": [p], "lr": 1e-3} for p in rs], lr=0.0, eps=1e-15, foreach=False)
    for it in range(9):
        for i, (a, b) in enumerate(zip(ps, rs)):
            idle = (i == 1 and it % 3 == 0) or (i == 3 and it in (4, 5))
            a.grad = None if idle else torch.ones_like(a)
            b.grad = None if idle else torch.ones_like(b)
        entries = []
        ours._collect(entries)
        ref.step()
        assert len(entries) == sum(p.grad is not None for p in ps)
        for a, b in zip(ps, rs):
            sa, sb = ours.state.get(a), ref.state.get(b)
            assert (sa is None) == (sb is None)
            if sa is not None:
                assert float(sa["step"]) == float(sb["step"]), (it, float(sa["step"]), float(sb["step"]))
    # parameters that always step together share one step tensor
    assert ours.state[ps[0]]["step"] is ours.state[ps[2]]["step"]


def _pc(N):
    return types.SimpleNamespace(_xyz=torch.zeros(N, 3))


def test_fused_deform_rows_detection():
    N = 7
    out = torch.randn(N, 10)
    pc = _pc(N)
    assert renderer._fused_deform_rows(pc, out[:, 0:3], out[:, 3:7], out[:, 7:10]) is out
    assert renderer._fused_deform_rows(pc, out[:, 0:3] * 1, out[:, 3:7], out[:, 7:10]) is None
    assert renderer._fused_deform_rows(pc, 0.0, 0.0, 0.0) == 0
    assert renderer._fused_deform_rows(pc, 0.5, 0.0, 0.0) is None
    assert renderer._fused_deform_rows(_pc(N + 1), out[:, 0:3], out[:, 3:7], out[:, 7:10]) is None


def test_fused_se3_rows_detection():
    N = 6
    raw = torch.randn(N, 13)
    dx = torch.zeros(N, 4, 4)
    dx._dgs_se3_raw = raw
    pc = _pc(N)
    assert renderer._fused_se3_rows(pc, dx, raw[:, 6:10], raw[:, 10:13]) is raw
    assert renderer._fused_se3_rows(pc, dx, raw[:, 6:10] * 1, raw[:, 10:13]) is None
    assert renderer._fused_se3_rows(pc, torch.zeros(N, 4, 4), raw[:, 6:10], raw[:, 10:13]) is None
    assert renderer._fused_se3_rows(pc, dx, raw[:, 5:9], raw[:, 10:13]) is None


def test_split_sh_needs_cuda():
    from diff_gaussian_rasterization import split_sh_ok
    # the split-SH rasterizer entry is a HIP path: CPU tensors always take the generic one
    assert split_sh_ok(torch.zeros(4, 1, 3), torch.zeros(4, 15, 3)) is False
