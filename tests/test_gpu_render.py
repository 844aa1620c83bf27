"""render(): the fused rasterizer-input kernels (dgs_gaussian_inputs_*) against the generic torch glue
of gaussian_renderer/__init__.py:70-112 (fp32 reference of the same ops), values and gradients."""
import pytest
import torch

from conftest import gpu_available

pytestmark = pytest.mark.gpu


def _setup(seed, warm=True):
    from deformgs.arguments import PipelineParams
    from deformgs.gaussian_model import GaussianModel
    from deformgs.synthetic import synth_camera, synth_gaussians
    dev = torch.device("cuda")
    g = synth_gaussians(3000, seed=seed, device=dev)
    gm = GaussianModel(3)
    gm.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    cam = synth_camera(160, 128, index=seed, fid=0.3, device=dev)
    gen = torch.Generator(device="cpu").manual_seed(seed)
    out = (torch.randn(3000, 10, generator=gen) * 0.01).to(dev).requires_grad_(True)
    return gm, cam, PipelineParams(), out


def _grads(gm, out, pkg, gt):
    loss = (pkg["render"] - gt).abs().mean() + 0.1 * pkg["depth"].mean()
    ps = [gm._xyz, gm._features_dc, gm._features_rest, gm._scaling, gm._rotation, gm._opacity]
    for p in ps + [out]:
        p.grad = None
    loss.backward()
    return [p.grad.clone() for p in ps] + [out.grad.clone() if out.grad is not None else None]


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("warm", [True, False])
def test_fused_inputs_match_torch_glue(warm):
    from deformgs import renderer
    gm, cam, pipe, out = _setup(5)
    bg = torch.tensor([0.1, 0.2, 0.3], device="cuda")
    gt = torch.rand(3, 128, 160, device="cuda")
    if warm:
        dx, dr, ds = out[:, 0:3], out[:, 3:7], out[:, 7:10]
        assert torch.is_tensor(renderer._fused_deform_rows(gm, dx, dr, ds))
        # clones are not views of one (N, 10) tensor -> the generic torch glue
        cx, cr, cs = out[:, 0:3] * 1.0, out[:, 3:7] * 1.0, out[:, 7:10] * 1.0
        assert renderer._fused_deform_rows(gm, cx, cr, cs) is None
    else:
        dx = dr = ds = 0.0
        cx = cr = cs = torch.zeros((), device="cuda")
    a = renderer.render(cam, gm, pipe, bg, dx, dr, ds)
    ga = _grads(gm, out, a, gt)
    b = renderer.render(cam, gm, pipe, bg, cx, cr, cs)
    gb = _grads(gm, out, b, gt)
    torch.testing.assert_close(a["render"], b["render"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a["depth"], b["depth"], rtol=1e-5, atol=1e-5)
    assert torch.equal(a["radii"], b["radii"])
    names = ["xyz", "f_dc", "f_rest", "scaling", "rotation", "opacity", "deform"]
    for n, x, y in zip(names, ga, gb):
        if y is None:
            assert x is None or torch.count_nonzero(x) == 0, n
            continue
        scale = y.abs().max().clamp_min(1e-12)
        assert ((x - y).abs().max() / scale) < 2e-4, n
