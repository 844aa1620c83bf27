"""The hot path at full size and as one composed training step, against the oracle chain.

(a) HIP rasterizer forward + backward vs oracle/raster_ref.c on synth-100k at 800x800 (the bench
    workload, P ~ 1e6 tile pairs), with the tolerances of tests/test_gpu_raster.py.
(b) One whole training step — fused MLP -> fused render inputs -> split-SH rasterizer -> fused L1+SSIM
    -> backward, deferred pair count on (deformgs/train_step.forward_backward) — against the oracle
    chain bench.py's cpu_baseline composes: oracle/mlp_ref.py (float64) -> render() glue in numpy ->
    oracle/raster_ref.c -> the reference's L1/SSIM in torch float64 on the CPU -> raster_ref backward
    -> glue chain rule -> mlp_ref backward. At config-1/2/3 sizes on synthetic scenes (5k @ 256^2,
    16k @ 400^2, 55k @ 800^2: BASELINE.json configs, whose datasets are absent here).
Tolerances (floating point, fp32 kernels vs an fp64/fp32 oracle): loss within 2e-6 relative; image
as test_gpu_raster; Gaussian gradients: >= 99.5 % of elements within 2e-3 of the tensor's max + 1e-3
relative (float atomics, alpha thresholds); MLP gradients (sums over all points): max error within
2e-3 of the tensor's max. The MLP oracle uses the kernel's own relu' masks (a pre-activation within an
ulp of 0 can take either sign in fp32; tests/test_gpu_mlp.py).
"""
import math

import numpy as np
import pytest
import torch

from conftest import gpu_available
from helpers import frac_close, mlp_relu_masks, oracle_run, rel_err, scene, settings_for_gpu

pytestmark = pytest.mark.gpu


def _guard_ok():
    from deformgs import _lib
    assert _lib.load().dgs_debug_guard_expiries() == 0


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_raster_bench_size_vs_oracle():
    from test_gpu_raster import _check, _run_gpu
    N, H, W = 100_000, 800, 800
    inputs, rs, _ = scene(N, H, W, cam_index=0)
    rng = np.random.default_rng(5)
    dcolor = rng.standard_normal((3, H, W)).astype(np.float32)
    o, g = oracle_run(inputs, rs, dcolor, None)
    assert o.num_rendered > 500_000, o.num_rendered  # the bench's pair-count regime
    color, radii, depth, grads = _run_gpu(inputs, rs, dcolor, None)
    _check(o, g, color, radii, depth, grads,
           [("means3D", "means3D"), ("shs", "shs"), ("opacities", "opacities"), ("scales", "scales"),
            ("rotations", "rotations"), ("means2D", "means2D"), ("means2D_densify", "means2D_densify")])


def _oracle_step(w, g, cam, gt, N, H, W, masks, lambda_dssim=0.2):
    """The step in the oracle chain; returns (loss, {param: grad})."""
    from deformgs.loss import l1_loss, ssim
    from oracle import mlp_ref
    from oracle.raster import OracleRaster, make_settings
    xyz = g["xyz"].cpu().numpy().astype(np.float64)
    t = np.full((N, 1), float(cam.fid.item()), np.float64)
    out, c = mlp_ref.forward(w, xyz, t, True, False)
    sc_raw = g["scaling"].cpu().numpy().astype(np.float64)
    q = g["rotation"].cpu().numpy().astype(np.float64)
    qn_norm = np.maximum(np.linalg.norm(q, axis=1, keepdims=True), 1e-12)
    qn = q / qn_norm
    op_raw = g["opacity"].cpu().numpy().astype(np.float64)
    sig = 1.0 / (1.0 + np.exp(-op_raw))
    means = xyz + out["d_xyz"]
    scales = np.exp(sc_raw) + out["d_scale"]
    rots = qn + out["d_rot"]
    shs = torch.cat([g["features_dc"], g["features_rest"]], 1).cpu().numpy()
    s = make_settings(H, W, math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), [0, 0, 0], 1.0,
                      cam.world_view_transform.cpu().numpy(), cam.full_proj_transform.cpu().numpy(), 3,
                      cam.camera_center.cpu().numpy())
    o = OracleRaster(s, means, shs=shs, opacities=sig, scales=scales, rotations=rots)
    img = torch.from_numpy(o.color.astype(np.float64)).requires_grad_(True)
    gtc = gt.cpu().double()
    loss = (1.0 - lambda_dssim) * l1_loss(img, gtc) + lambda_dssim * (1.0 - ssim(img, gtc))
    loss.backward()
    gr = o.backward(img.grad.numpy().astype(np.float32))
    gm, gs, grt = (gr[k].astype(np.float64) for k in ("means3D", "scales", "rotations"))
    grads = {
        "_xyz": gm,
        "_scaling": gs * np.exp(sc_raw),
        "_rotation": (grt - qn * (qn * grt).sum(1, keepdims=True)) / qn_norm,
        "_opacity": gr["opacities"].astype(np.float64) * sig * (1.0 - sig),
        "_features_dc": gr["shs"][:, :1].astype(np.float64),
        "_features_rest": gr["shs"][:, 1:].astype(np.float64),
    }
    mg = mlp_ref.backward(w, c, out, {"d_xyz": gm, "d_rot": grt, "d_scale": gs}, True, False, relu_masks=masks)
    grads.update({"mlp." + k: v for k, v in mg.items()})
    return float(loss), grads, o


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("N,res", [(5000, 256), (16000, 400), (55000, 800)])
def test_training_step_vs_oracle_chain(N, res):
    from deformgs.arguments import OptimizationParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.synthetic import synth_camera, synth_gaussians
    from deformgs.train_step import deferred_overflowed, drop_grads, forward_backward
    from oracle import mlp_ref
    from weights import mlp_weights
    dev = torch.device("cuda", 0)
    g = synth_gaussians(N, seed=2, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    gs.training_setup(OptimizationParams())
    deform = DeformModelBaseline(is_blender=True, is_6dof=False, device=dev)
    w = mlp_weights(mlp_ref.param_shapes(True, False), seed=4)
    for k in w:  # steady-state head scale (bench.py)
        if k.startswith(("gaussian_warp", "gaussian_rotation", "gaussian_scaling")):
            w[k] = (w[k] * 0.01).astype(np.float32)
    deform.deform.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    deform.train_setting(OptimizationParams())
    cam = synth_camera(res, res, index=1, fid=0.37, device=dev)
    gt = torch.rand((3, res, res), generator=torch.Generator().manual_seed(9)).to(dev)
    pipe, bg = PipelineParams(), torch.zeros(3, device=dev)
    # the kernel's relu' masks for this input (a separate, bitwise identical forward)
    raw = deform.deform.raw(gs.get_xyz.detach(), cam.fid.unsqueeze(0).expand(N, -1))
    masks = mlp_relu_masks(raw, N, True, False, th_saved=False)
    del raw
    # a synchronous step teaches the speculative pair capacity, then the deferred one is checked
    forward_backward(gs, deform, cam, gt, pipe, bg)
    drop_grads(gs, deform)
    loss, pkg = forward_backward(gs, deform, cam, gt, pipe, bg, deferred_count=True)
    assert not deferred_overflowed()
    torch.cuda.synchronize()
    want_loss, want, o = _oracle_step(w, g, cam, gt, N, res, res, masks)
    assert abs(float(loss) - want_loss) <= 2e-6 * abs(want_loss), (float(loss), want_loss)
    img = pkg["render"].detach().cpu().numpy()
    err = np.abs(img - o.color)
    assert err.mean() <= 1e-5 and (err <= 1e-4).mean() >= 0.999, err.mean()
    assert (pkg["radii"].cpu().numpy() == o.radii).mean() >= 0.9999
    params = {"_xyz": gs._xyz, "_scaling": gs._scaling, "_rotation": gs._rotation, "_opacity": gs._opacity,
              "_features_dc": gs._features_dc, "_features_rest": gs._features_rest}
    params.update({"mlp." + k: p for k, p in deform.deform.named_parameters()})
    for k, p in params.items():
        a = p.grad.detach().cpu().numpy().astype(np.float64).reshape(-1)
        b = want[k].reshape(-1)
        if k.startswith("mlp."):
            assert np.abs(a - b).max() <= 2e-3 * max(np.abs(b).max(), 1e-12), (k, rel_err(a, b))
        else:
            assert frac_close(a, b, atol=2e-3 * np.abs(b).max(), rtol=1e-3) >= 0.995, (k, rel_err(a, b))
    _guard_ok()
