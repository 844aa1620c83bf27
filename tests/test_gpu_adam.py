"""Multi-tensor HIP Adam (dgs_adam_step) against torch.optim.Adam (fp32 reference of the same op)."""
import pytest
import torch

from conftest import gpu_available

pytestmark = pytest.mark.gpu


def _params(dev, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    shapes = [(1000, 3), (1000, 1, 3), (1000, 15, 3), (1000, 1), (1000, 4), (256, 63), (256,), (7,)]
    return [torch.nn.Parameter(torch.randn(s, generator=g).to(dev)) for s in shapes]


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_adam_matches_torch():
    from deformgs.adam import Adam, step_all
    dev = torch.device("cuda")
    pa, pb = _params(dev, 0), _params(dev, 0)
    lrs = [1.6e-4, 2.5e-3, 1.25e-4, 0.05, 1e-3, 8e-4, 8e-4, 0.0]
    ga = [{"params": [p], "lr": lr, "name": f"g{i}"} for i, (p, lr) in enumerate(zip(pa, lrs))]
    gb = [{"params": [p], "lr": lr, "name": f"g{i}"} for i, (p, lr) in enumerate(zip(pb, lrs))]
    ours = Adam(ga, lr=0.0, eps=1e-15)
    ref = torch.optim.Adam(gb, lr=0.0, eps=1e-15, foreach=False)
    assert ours._hip
    gen = torch.Generator(device="cpu").manual_seed(1)
    for it in range(12):
        for i, (a, b) in enumerate(zip(pa, pb)):
            if i == 4 and it % 3 == 0:  # a parameter without a gradient on some steps
                a.grad = b.grad = None
                continue
            g = torch.randn(a.shape, generator=gen).to(dev) * (10.0 ** (i % 3 - 1))
            if i == 2:  # non-contiguous gradient
                g = g.transpose(1, 2).contiguous().transpose(1, 2)
            a.grad = g.clone()
            b.grad = g.clone()
        if it % 2:
            step_all(ours)
        else:
            ours.step()
        ref.step()
        # learning-rate schedule changes between steps, as update_learning_rate does
        for go, gr in zip(ours.param_groups, ref.param_groups):
            go["lr"] *= 0.97
            gr["lr"] *= 0.97
    torch.cuda.synchronize()
    for a, b in zip(pa, pb):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)
        sa, sb = ours.state[a], ref.state[b]
        assert float(sa["step"]) == float(sb["step"])
        torch.testing.assert_close(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-4, atol=1e-8)


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_adam_two_optimizers_one_launch():
    from deformgs.adam import Adam, step_all
    dev = torch.device("cuda")
    a1, b1 = _params(dev, 3)[:3], _params(dev, 3)[:3]
    a2, b2 = _params(dev, 4)[5:], _params(dev, 4)[5:]
    o1, o2 = Adam(a1, lr=1e-2, eps=1e-15), Adam(a2, lr=5e-3, eps=1e-15)
    r1 = torch.optim.Adam(b1, lr=1e-2, eps=1e-15, foreach=False)
    r2 = torch.optim.Adam(b2, lr=5e-3, eps=1e-15, foreach=False)
    for _ in range(3):
        for a, b in zip(a1 + a2, b1 + b2):
            g = torch.randn_like(a)
            a.grad, b.grad = g.clone(), g.clone()
        step_all(o1, o2)
        r1.step()
        r2.step()
    for a, b in zip(a1 + a2, b1 + b2):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_adam_persistent_gradient_buffers_fast_path():
    """The native training step keeps each parameter's gradient in the same buffer every iteration;
    step_all then reuses its launch tables and only updates the step counts and bias corrections
    (deformgs/adam.py: the tables cached on the optimizer, `_dgs_fast`). With the learning rates changing every step and the gradients rewritten
    in place, the result must still be torch.optim.Adam's; a replaced parameter (densification)
    drops back to the full path."""
    from deformgs import adam as adam_mod
    from deformgs.adam import Adam, step_all
    dev = torch.device("cuda")
    pa, pb = _params(dev, 5), _params(dev, 5)
    ga = [{"params": [p], "lr": 1e-3 * (i + 1), "name": f"g{i}"} for i, p in enumerate(pa)]
    gb = [{"params": [p], "lr": 1e-3 * (i + 1), "name": f"g{i}"} for i, p in enumerate(pb)]
    ours = Adam(ga, lr=0.0, eps=1e-15)
    ref = torch.optim.Adam(gb, lr=0.0, eps=1e-15, foreach=False)
    bufs = [torch.empty_like(p) for p in pa]
    gen = torch.Generator(device="cpu").manual_seed(2)
    hits = 0
    for it in range(8):
        for a, b, buf in zip(pa, pb, bufs):
            buf.copy_(torch.randn(a.shape, generator=gen).to(dev))
            a.grad = buf
            b.grad = buf.clone()
        before = getattr(ours, "_dgs_fast", None)
        step_all(ours)
        hits += int(before is not None and getattr(ours, "_dgs_fast", None) is before)
        ref.step()
        for go, gr in zip(ours.param_groups, ref.param_groups):
            go["lr"] *= 0.9
            gr["lr"] *= 0.9
    assert hits >= 6, hits  # every step after the first reused the tables
    # the cache refers to the optimizer's own groups only; clearing it (end of training()) drops it
    adam_mod.clear_fast_cache(ours)
    assert ours._dgs_fast is None
    torch.cuda.synchronize()
    for a, b in zip(pa, pb):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)
        assert float(ours.state[a]["step"]) == float(ref.state[b]["step"]) == 8.0
