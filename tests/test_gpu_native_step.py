"""The native training step (dgs_train_step, deformgs/native_step.py: one C call, no autograd engine)
against the autograd step it replaces (deformgs/train_step.forward_backward) on the same inputs.

Both issue the same kernels in the same order, so the forward (image, depth, radii, visibility, loss)
must be bitwise equal; gradients go through the blend backward's float atomics (arrival order), so
they are compared to 1e-4 relative + 1e-6 of each tensor's max. Variants: the blender network
(configs 1-3), the 6-DoF screw head (config 4), the non-blender network with an ast_noise frame-time
offset (config 5), a warm-up iteration (no deformation network), and a forced overflow of the deferred
pair count (redone synchronously by train_step). Edge cases: nothing rendered (every Gaussian behind the
camera) and a single Gaussian."""
import numpy as np
import pytest
import torch

from conftest import gpu_available

pytestmark = pytest.mark.gpu


def _model(N, is_blender, is_6dof, seed=0):
    from deformgs.arguments import OptimizationParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.synthetic import synth_gaussians
    dev = torch.device("cuda", 0)
    g = synth_gaussians(N, seed=seed, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    gs.training_setup(OptimizationParams())
    torch.manual_seed(seed)
    deform = DeformModelBaseline(is_blender=is_blender, is_6dof=is_6dof, device=dev)
    net = deform.deform
    heads = (net.branch_w, net.branch_v) if is_6dof else (net.gaussian_warp,)
    with torch.no_grad():
        for h in heads + (net.gaussian_rotation, net.gaussian_scaling):
            h.weight.mul_(0.01)
            h.bias.mul_(0.01)
    deform.train_setting(OptimizationParams())
    return gs, deform


def _params(gs, deform):
    return [gs._xyz, gs._features_dc, gs._features_rest, gs._scaling, gs._rotation, gs._opacity] + \
        list(deform.deform.parameters())


CASES = [
    # name, N, res, is_blender, is_6dof, ast_noise, warm
    ("blender", 16000, 400, True, False, 0.0, True),
    ("6dof", 12000, 320, True, True, 0.0, True),
    ("nonblender-noise", 12000, 320, False, False, -0.021, True),
    ("warmup", 8000, 256, True, False, 0.0, False),
    ("blender-1M", 1_000_000, 800, True, False, 0.0, True),  # 10x the bench's Gaussians, ~10 M pairs
]


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("name,N,res,is_blender,is_6dof,ast_noise,warm", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("deferred", [False, True])
def test_native_step_matches_autograd_step(name, N, res, is_blender, is_6dof, ast_noise, warm, deferred):
    from deformgs import _lib, native_step
    from deformgs.arguments import PipelineParams
    from deformgs.synthetic import synth_camera
    from deformgs.train_step import drop_grads, forward_backward, train_step
    dev = torch.device("cuda", 0)
    gs, deform = _model(N, is_blender, is_6dof)
    cam = synth_camera(res, res, index=3, fid=0.43, device=dev)
    gt = torch.rand((3, res, res), generator=torch.Generator().manual_seed(5)).to(dev)
    pipe, bg = PipelineParams(), torch.zeros(3, device=dev)
    noise = torch.full((1, 1), ast_noise, device=dev) if ast_noise else 0.0
    assert native_step.usable(gs, deform, pipe, gt)
    # autograd reference (synchronous pair count; also teaches the speculative capacity)
    loss_a, pkg_a = forward_backward(gs, deform, cam, gt, pipe, bg, is_6dof=is_6dof, warm=warm, ast_noise=noise)
    torch.cuda.synchronize()
    ref = dict(loss=float(loss_a), image=pkg_a["render"].detach().clone(), depth=pkg_a["depth"].detach().clone(),
               radii=pkg_a["radii"].clone(), vis=pkg_a["visibility_filter"].clone(),
               nr=int(pkg_a["render"].grad_fn.num_rendered),
               dens=pkg_a["viewspace_points_densify"].grad.clone(),
               grads=[None if p.grad is None else p.grad.clone() for p in _params(gs, deform)])
    drop_grads(gs, deform)
    loss_n, pkg_n, redone = train_step(gs, deform, cam, gt, pipe, bg, is_6dof, warm=warm, ast_noise=noise,
                                       deferred_count=deferred)
    torch.cuda.synchronize()
    assert getattr(gs, "_dgs_native", None) is not None, "train_step must take the native path here"
    assert not redone
    assert float(loss_n) == ref["loss"]
    assert torch.equal(pkg_n["render"], ref["image"]) and torch.equal(pkg_n["depth"], ref["depth"])
    assert torch.equal(pkg_n["radii"], ref["radii"]) and torch.equal(pkg_n["visibility_filter"], ref["vis"])
    assert pkg_n["num_rendered"] == ref["nr"] > 0  # also with the deferred count (resolved at the end)
    torch.testing.assert_close(pkg_n["viewspace_points_densify"].grad, ref["dens"], rtol=1e-4,
                               atol=1e-6 * float(ref["dens"].abs().max()))
    for i, (p, want) in enumerate(zip(_params(gs, deform), ref["grads"])):
        if want is None:  # warm-up: the network did not run
            assert p.grad is None, i
            continue
        torch.testing.assert_close(p.grad, want, rtol=1e-4, atol=1e-6 * max(float(want.abs().max()), 1e-30),
                                   msg=lambda m: f"param {i}: {m}")
    assert _lib.load().dgs_debug_guard_expiries() == 0


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("deferred", [False, True])
def test_native_step_nothing_rendered(deferred):
    """Every Gaussian behind the camera (num_rendered = 0: empty tile lists, no pair to sort, blend or
    replay): the native step and the autograd step give the background image, the same loss, radii 0,
    nothing visible, and all-zero gradients for every Gaussian and network parameter."""
    from deformgs.arguments import PipelineParams
    from deformgs.synthetic import synth_camera
    from deformgs.train_step import drop_grads, forward_backward, train_step
    dev = torch.device("cuda", 0)
    gs, deform = _model(3000, True, False, seed=2)
    cam = synth_camera(96, 80, index=1, fid=0.2, device=dev)
    with torch.no_grad():
        gs._xyz.copy_(cam.camera_center[None] * 1.5 + 0.01 * gs._xyz)
    gt = torch.rand((3, 80, 96), generator=torch.Generator().manual_seed(3)).to(dev)
    pipe, bg = PipelineParams(), torch.tensor([0.3, 0.2, 0.1], device=dev)
    loss_a, pkg_a = forward_backward(gs, deform, cam, gt, pipe, bg)
    torch.cuda.synchronize()
    assert int(pkg_a["render"].grad_fn.num_rendered) == 0
    ref = [None if p.grad is None else p.grad.clone() for p in _params(gs, deform)]
    drop_grads(gs, deform)
    loss_n, pkg_n, redone = train_step(gs, deform, cam, gt, pipe, bg, False, deferred_count=deferred)
    torch.cuda.synchronize()
    assert getattr(gs, "_dgs_native", None) is not None and not redone
    assert pkg_n["num_rendered"] == 0
    assert float(loss_n) == float(loss_a)
    want = bg[:, None, None].expand(3, 80, 96)
    assert torch.equal(pkg_n["render"], want) and torch.equal(pkg_a["render"].detach(), want)
    assert int(pkg_n["radii"].abs().sum()) == 0 and not bool(pkg_n["visibility_filter"].any())
    for i, (p, r) in enumerate(zip(_params(gs, deform), ref)):
        assert p.grad is not None and r is not None, i
        assert float(p.grad.abs().max()) == 0.0 and float(r.abs().max()) == 0.0, i


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_native_step_single_gaussian():
    """N = 1 (one 16-point tail block of the network kernels, one short tile list per covered tile): one
    Gaussian at the scene origin, in view; the native step equals the autograd step (image and loss
    bitwise, gradients to the atomics' 1e-4)."""
    from deformgs.arguments import PipelineParams
    from deformgs.synthetic import synth_camera
    from deformgs.train_step import drop_grads, forward_backward, train_step
    dev = torch.device("cuda", 0)
    gs, deform = _model(1, True, False, seed=4)
    with torch.no_grad():
        gs._xyz.zero_()
        gs._scaling.fill_(-2.0)
        gs._opacity.fill_(1.0)
    cam = synth_camera(96, 80, index=2, fid=0.6, device=dev)
    gt = torch.rand((3, 80, 96), generator=torch.Generator().manual_seed(8)).to(dev)
    pipe, bg = PipelineParams(), torch.zeros(3, device=dev)
    loss_a, pkg_a = forward_backward(gs, deform, cam, gt, pipe, bg)
    torch.cuda.synchronize()
    nr = int(pkg_a["render"].grad_fn.num_rendered)
    image = pkg_a["render"].detach().clone()
    ref = [p.grad.clone() for p in _params(gs, deform)]
    drop_grads(gs, deform)
    loss_n, pkg_n, redone = train_step(gs, deform, cam, gt, pipe, bg, False)
    torch.cuda.synchronize()
    assert getattr(gs, "_dgs_native", None) is not None and not redone
    assert pkg_n["num_rendered"] == nr > 0
    assert float(loss_n) == float(loss_a) and torch.equal(pkg_n["render"], image)
    assert float(image.abs().max()) > 0  # the Gaussian is drawn
    for i, (p, want) in enumerate(zip(_params(gs, deform), ref)):
        torch.testing.assert_close(p.grad, want, rtol=1e-4, atol=1e-6 * max(float(want.abs().max()), 1e-30),
                                   msg=lambda m: f"param {i}: {m}")
    assert float(gs._xyz.grad.abs().max()) > 0


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_native_step_overflow_redo_and_adam():
    """A forced overflow of the deferred pair count is redone synchronously (the result equals the
    plain native step); several steps with Adam and a densify-style reallocation in between follow the
    autograd path's losses to 1e-5 and parameters to 2e-4 relative (Adam moves near-zero-gradient elements by lr-sized steps of either sign)."""
    from deformgs import _lib
    from deformgs.arguments import PipelineParams
    from deformgs.synthetic import synth_camera
    from deformgs.train_step import optimizer_step, train_step
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    pipe, bg = PipelineParams(), torch.zeros(3, device=dev)
    cams = [synth_camera(240, 200, index=k, fid=0.1 * k, device=dev) for k in range(3)]
    gts = [torch.rand((3, 200, 240), generator=torch.Generator().manual_seed(k)).to(dev) for k in range(3)]
    runs = {}
    for native in (True, False):
        import deformgs.native_step as ns_mod
        old = ns_mod.enabled
        ns_mod.enabled = (lambda: True) if native else (lambda: False)
        try:
            gs, deform = _model(6000, True, False, seed=1)
            losses = []
            for it in range(6):
                if native and it == 2:
                    lib.dgs_debug_set_pair_cap(0, 300)
                loss, pkg, redone = train_step(gs, deform, cams[it % 3], gts[it % 3], pipe, bg, False)
                if native and it == 2:
                    assert redone, "the forced overflow must be redone"
                losses.append(float(loss))
                optimizer_step(gs, deform, 3000 + it)
                if it == 3:  # a prune, as densify_and_prune does: every tensor is replaced
                    keep = torch.ones(gs._xyz.shape[0], dtype=torch.bool, device=dev)
                    keep[::7] = False
                    gs.prune_points(~keep)
            torch.cuda.synchronize()
            runs[native] = (losses, [p.detach().clone() for p in _params(gs, deform)])
        finally:
            ns_mod.enabled = old
    la, lb = np.array(runs[True][0]), np.array(runs[False][0])
    assert np.all(np.abs(la - lb) <= 1e-5 * np.abs(lb)), (la, lb)
    for a, b in zip(runs[True][1], runs[False][1]):
        assert a.shape == b.shape
        assert float((a - b).norm()) <= 2e-4 * max(float(b.norm()), 1e-30)
