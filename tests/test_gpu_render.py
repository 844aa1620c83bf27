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


def _raw13(n, seed, dev):
    """(n, 13) raw 6-DoF head rows [w_r v_r d_rot d_scale] of the magnitudes a trained network emits."""
    gen = torch.Generator(device="cpu").manual_seed(seed)
    w = torch.randn(n, 3, generator=gen) * 0.3
    v = torch.randn(n, 3, generator=gen) * 0.01
    rs = torch.randn(n, 7, generator=gen) * 0.01
    return torch.cat([w, v, rs], 1).to(dev).requires_grad_(True)


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_se3_matrices_match_rigid_utils():
    """dgs_se3_*: exp_se3 of the screw head (utils/time_utils.py:114-121, rigid_utils.py:4-83) and its
    gradient vs the torch statement (deformgs/rigid.py) in float64 on the CPU. Tolerance: values 2e-6
    absolute (|M| <= ~2), gradients 1e-4 of the tensor's max."""
    from deformgs.deform_network import _ScrewSE3
    from deformgs.rigid import screw_from_raw
    raw = _raw13(5000, 3, "cuda")
    M = _ScrewSE3.apply(raw[:, 0:6])
    r64 = raw.detach().cpu().double().requires_grad_(True)
    M64 = screw_from_raw(r64[:, 0:3], r64[:, 3:6])
    assert (M.detach().cpu().double() - M64.detach()).abs().max() < 2e-6
    gM = torch.randn(5000, 4, 4, generator=torch.Generator().manual_seed(4))
    (M * gM.cuda()).sum().backward()
    (M64 * gM.double()).sum().backward()
    g, g64 = raw.grad.cpu().double(), r64.grad
    assert torch.count_nonzero(g[:, 6:]) == 0
    err = (g[:, :6] - g64[:, :6]).abs().max() / g64[:, :6].abs().max()
    assert err < 1e-4, err


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_fused_se3_inputs_match_torch_glue():
    """render(..., is_6dof=True): the screw applied inside the input launch (dgs_gaussian_inputs_se3_*)
    vs the reference's glue (bmm of the (N, 4, 4) torch screw with homogeneous xyz,
    gaussian_renderer/__init__.py:71-76) — images, radii and every gradient, the raw head's included."""
    from deformgs import renderer
    from deformgs.deform_network import _ScrewSE3
    from deformgs.rigid import screw_from_raw
    gm, cam, pipe, _ = _setup(6)
    raw = _raw13(3000, 6, "cuda")
    bg = torch.tensor([0.1, 0.2, 0.3], device="cuda")
    gt = torch.rand(3, 128, 160, device="cuda")
    dx = _ScrewSE3.apply(raw[:, 0:6])
    dx._dgs_se3_raw = raw
    dr, ds = raw[:, 6:10], raw[:, 10:13]
    assert renderer._fused_se3_rows(gm, dx, dr, ds) is raw
    a = renderer.render(cam, gm, pipe, bg, dx, dr, ds, is_6dof=True)
    ga = _grads(gm, raw, a, gt)
    cx = screw_from_raw(raw[:, 0:3], raw[:, 3:6])
    assert renderer._fused_se3_rows(gm, cx, dr, ds) is None
    b = renderer.render(cam, gm, pipe, bg, cx, raw[:, 6:10] * 1.0, raw[:, 10:13] * 1.0, is_6dof=True)
    gb = _grads(gm, raw, b, gt)
    assert a["radii"].gt(0).sum() > 500
    torch.testing.assert_close(a["render"], b["render"], rtol=1e-4, atol=1e-5)
    assert (a["radii"] != b["radii"]).float().mean() < 1e-3
    names = ["xyz", "f_dc", "f_rest", "scaling", "rotation", "opacity", "raw"]
    for n, x, y in zip(names, ga, gb):
        scale = y.abs().max().clamp_min(1e-12)
        frac_ok = (((x - y).abs() / scale) < 2e-3).float().mean()
        assert frac_ok > 0.999, (n, frac_ok)


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("degree", [3, 1])
def test_split_sh_raster_matches_concatenated(degree, monkeypatch):
    """render()'s training path with the split-SH rasterizer (features_dc / features_rest read and
    written in place, dgs_raster_*_split_sh) vs the same path on the concatenated (N, 16, 3) SH rows
    of the plain rasterizer: identical images and radii, gradients equal up to the blend backward's
    float-atomic ordering (tolerance 1e-5 of each tensor's max)."""
    from deformgs import renderer
    gm, cam, pipe, out = _setup(7)
    gm.active_sh_degree = degree
    bg = torch.tensor([0.0, 0.1, 0.2], device="cuda")
    gt = torch.rand(3, 128, 160, device="cuda")
    dx, dr, ds = out[:, 0:3], out[:, 3:7], out[:, 7:10]
    res = []
    for split in (True, False):
        monkeypatch.setattr(renderer, "_SPLIT_SH", split)
        pkg = renderer.render(cam, gm, pipe, bg, dx, dr, ds)
        res.append((pkg, _grads(gm, out, pkg, gt)))
    (a, ga), (b, gb) = res
    assert torch.equal(a["render"], b["render"]) and torch.equal(a["radii"], b["radii"])
    assert torch.equal(a["depth"], b["depth"])
    # visibility_filter: written by the preprocess kernel on the split path, radii > 0 on the other
    assert a["visibility_filter"].dtype == torch.bool and torch.equal(a["visibility_filter"], b["visibility_filter"])
    assert torch.equal(a["visibility_filter"], a["radii"] > 0)
    for n, x, y in zip(["xyz", "f_dc", "f_rest", "scaling", "rotation", "opacity", "deform"], ga, gb):
        scale = y.abs().max().clamp_min(1e-12)
        assert ((x - y).abs().max() / scale) < 1e-5, n
