"""CPU: densify_and_prune (clone, split, prune through deformgs/compact.select_rows) keeps every
parameter, both Adam moments and the statistics row-aligned, and reproduces the upstream counts
(scene/gaussian_model.py:242-292 semantics): clones are appended, each split source is replaced by
N = 2 samples, pruning removes low-opacity / oversized points."""
import torch

from deformgs.arguments import OptimizationParams
from deformgs.gaussian_model import GaussianModel
from deformgs.synthetic import synth_gaussians


def test_densify_and_prune_host():
    n = 3000
    torch.manual_seed(0)
    g = synth_gaussians(n, seed=2, device="cpu")
    m = GaussianModel(3)
    m.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    m.training_setup(OptimizationParams())
    for p in (m._xyz, m._features_dc, m._features_rest, m._scaling, m._rotation, m._opacity):
        p.grad = torch.randn_like(p) * 1e-3
    m.optimizer.step()
    gen = torch.Generator().manual_seed(5)
    m.xyz_gradient_accum = torch.rand((n, 1), generator=gen) * 0.002
    m.denom = torch.ones((n, 1))
    m.max_radii2D = torch.zeros(n)
    extent, thr, min_op = 2.0, 0.0007, 0.1  # percent_dense * extent = 0.02 ~ the median scale
    grads = (m.xyz_gradient_accum / m.denom).squeeze(1)
    big = m.get_scaling.max(dim=1).values > m.percent_dense * extent
    n_clone = int(((grads >= thr) & ~big).sum())
    n_split = int(((grads >= thr) & big).sum())
    assert n_clone > 0 and n_split > 0
    m.densify_and_prune(thr, min_op, extent, None, generator=torch.Generator().manual_seed(9))
    n1 = m._xyz.shape[0]
    # after clone + split (n + n_clone + n_split) every point with opacity < min_op is pruned; the
    # clones / split samples copy their source opacity, so count them on the final model
    assert n1 <= n + n_clone + n_split
    assert (m.get_opacity >= min_op).all()
    for gi, group in enumerate(m.optimizer.param_groups):
        p = group["params"][0]
        st = m.optimizer.state[p]
        assert p.shape[0] == n1 and st["exp_avg"].shape == p.shape and st["exp_avg_sq"].shape == p.shape
    assert m.xyz_gradient_accum.shape == (n1, 1) and m.denom.shape == (n1, 1) and m.max_radii2D.shape == (n1,)
    assert m._features_rest.shape[1:] == (15, 3)
