"""Shared test helpers: scenes, camera settings, and HIP-vs-oracle comparisons."""
import math

import numpy as np
import torch

from deformgs.synthetic import synth_camera, synth_gaussians
from oracle.raster import OracleRaster, make_settings


def scene(N, H, W, seed=0, cam_index=0, scale_boost=0.0, device="cpu", bg=(0.0, 0.0, 0.0), sh_degree=3):
    g = synth_gaussians(N, seed=seed, device="cpu")
    g["scaling"] = g["scaling"] + scale_boost
    cam = synth_camera(W, H, index=cam_index, device="cpu")
    inputs = dict(
        means3D=g["xyz"],
        shs=torch.cat([g["features_dc"], g["features_rest"]], 1),
        opacities=torch.sigmoid(g["opacity"]),
        scales=torch.exp(g["scaling"]),
        rotations=torch.nn.functional.normalize(g["rotation"]),
    )
    rs = dict(H=H, W=W, tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2),
              bg=torch.tensor(bg, dtype=torch.float32), scale_modifier=1.0,
              viewmatrix=cam.world_view_transform, projmatrix=cam.full_proj_transform, sh_degree=sh_degree,
              campos=cam.camera_center)
    return inputs, rs, cam


def oracle_run(inputs, rs, dcolor=None, ddepth=None, use_cov=False, use_colors=False):
    s = make_settings(rs["H"], rs["W"], rs["tanfovx"], rs["tanfovy"], rs["bg"].numpy(), rs["scale_modifier"],
                      rs["viewmatrix"].numpy(), rs["projmatrix"].numpy(), rs["sh_degree"], rs["campos"].numpy())
    kw = dict(means3D=inputs["means3D"].numpy(), opacities=inputs["opacities"].numpy())
    if use_colors:
        kw["colors_precomp"] = inputs["colors"].numpy()
    else:
        kw["shs"] = inputs["shs"].numpy()
    if use_cov:
        kw["cov3D_precomp"] = inputs["cov3D"].numpy()
    else:
        kw["scales"] = inputs["scales"].numpy()
        kw["rotations"] = inputs["rotations"].numpy()
    o = OracleRaster(s, **kw)
    g = o.backward(dcolor, ddepth) if dcolor is not None else None
    return o, g


def settings_for_gpu(rs, device="cuda"):
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    return GaussianRasterizationSettings(
        image_height=rs["H"], image_width=rs["W"], tanfovx=rs["tanfovx"], tanfovy=rs["tanfovy"],
        bg=rs["bg"].to(device), scale_modifier=rs["scale_modifier"], viewmatrix=rs["viewmatrix"].to(device),
        projmatrix=rs["projmatrix"].to(device), sh_degree=rs["sh_degree"], campos=rs["campos"].to(device),
        prefiltered=False, debug=False)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def frac_close(a, b, atol, rtol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    ok = np.abs(a - b) <= atol + rtol * np.abs(b)
    return float(ok.mean())


# saved-activation rows of the fused MLP (csrc/mlp_shared.h: S_H0.., S_H4.., S_TH), feature-major [rows][Ns]
_S_H = [0, 256, 512, 768, 1120, 1376, 1632, 1888]
_S_TH = 2160


def mlp_relu_masks(output, N, blender, exact, th_saved=True):
    """The fused MLP kernel's own relu' masks {layer: bool (N, 256), "th": ...} read back from the
    activations it saved for backward (autograd ctx of the fused node reached from `output`).
    th_saved=False: the forward ran with DGS_MLP_UNIFORM_T (one-element or stride-0 t), which keeps
    no per-point TH rows; the oracle then uses its own TH masks."""
    seen, todo, node = set(), [output.grad_fn], None
    while todo:
        fn = todo.pop()
        if fn is None or fn in seen:
            continue
        seen.add(fn)
        if "FusedDeformMLP" in type(fn).__name__:
            node = fn
            break
        todo.extend(f for f, _ in fn.next_functions)
    assert node is not None, "fused MLP node not found in the autograd graph"
    _, saved = node.saved_tensors
    block = 32 if exact else 64
    Ns = (N + block - 1) // block * block
    rows = 2416 if blender else 2144
    sv = saved[: rows * Ns].view(rows, Ns)[:, :N].cpu().numpy()
    masks = {i: (sv[r:r + 256] > 0).T for i, r in enumerate(_S_H)}
    if blender and th_saved:
        masks["th"] = (sv[_S_TH:_S_TH + 256] > 0).T
    return masks
