"""HIP row selection (dgs_select_rows, deformgs/compact.py) vs torch boolean indexing, alone and
inside densification (densify_and_clone / _split / prune_points edit six parameters, both Adam
moments and the statistics): bit-exact (pure data movement)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 255, 256, 1000, 70001])
def test_select_rows_matches_indexing(n):
    from deformgs.compact import select_rows
    g = torch.Generator(device="cuda").manual_seed(n)
    ts = [torch.randn((n,) + s, device="cuda", generator=g) for s in [(), (1,), (3,), (4,), (1, 3), (15, 3)]]
    for p in (0.0, 0.3, 0.97, 1.0):
        mask = torch.rand(n, device="cuda", generator=g) < p
        got = select_rows(mask, ts)
        for a, t in zip(got, ts):
            want = t[mask]
            assert a.shape == want.shape
            assert torch.equal(a, want)


def _model(n, dev):
    from deformgs.arguments import OptimizationParams
    from deformgs.gaussian_model import GaussianModel
    from deformgs.synthetic import synth_gaussians
    torch.manual_seed(0)
    g = synth_gaussians(n, seed=1, device=dev)
    m = GaussianModel(3)
    m.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    m.training_setup(OptimizationParams())
    # one Adam step so every parameter has moments to compact
    for p in (m._xyz, m._features_dc, m._features_rest, m._scaling, m._rotation, m._opacity):
        p.grad = torch.randn_like(p) * 1e-3
    m.optimizer.step()
    gen = torch.Generator(device=dev).manual_seed(3)
    m.xyz_gradient_accum = torch.rand((n, 1), device=dev, generator=gen) * 0.002
    m.denom = torch.randint(0, 3, (n, 1), device=dev, generator=gen).float()
    m.max_radii2D = torch.rand(n, device=dev, generator=gen) * 30
    return m


def _snapshot(m):
    out = {k: getattr(m, k).detach().clone() for k in
           ("_xyz", "_features_dc", "_features_rest", "_scaling", "_rotation", "_opacity",
            "xyz_gradient_accum", "denom", "max_radii2D")}
    for gi, group in enumerate(m.optimizer.param_groups):
        st = m.optimizer.state[group["params"][0]]
        out[f"m{gi}"] = st["exp_avg"].clone()
        out[f"v{gi}"] = st["exp_avg_sq"].clone()
    return out


def test_densify_and_prune_matches_torch_indexing(monkeypatch):
    """The same densify_and_prune with select_rows replaced by torch indexing (the upstream
    operations) must give bitwise the same model and optimizer state."""
    import deformgs.gaussian_model as gm
    res = []
    for mode in ("hip", "torch"):
        if mode == "torch":
            monkeypatch.setattr(gm, "select_rows", lambda mask, ts: [t[mask] for t in ts])
        m = _model(20000, "cuda")
        gen = torch.Generator(device="cuda").manual_seed(11)
        m.densify_and_prune(0.0007, 0.1, 2.0, 20, generator=gen)
        res.append(_snapshot(m))
    a, b = res
    assert a["_xyz"].shape[0] != 20000  # something was cloned / split / pruned
    for k in a:
        assert a[k].shape == b[k].shape, k
        assert torch.equal(a[k], b[k]), k
