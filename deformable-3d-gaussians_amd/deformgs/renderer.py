"""render() — same signature and return dict as gaussian_renderer/__init__.py:32-133.

The rasterizer underneath is this repo's diff_gaussian_rasterization (libdgs_hip.so). Glue math
(means3D = xyz + d_xyz or the 6-DoF transform, scales = exp(_scaling) + d_scale, rotations =
normalize(_rotation) + d_rot without re-normalisation, opacity = sigmoid) is unchanged; on the
training path (no 6-DoF, SHs and covariance in the rasterizer, deltas straight from the fused
deformation network or absent) it runs as one HIP launch each way (dgs_gaussian_inputs_*), whose
backward writes the deformation network's (N, 10) output gradient directly.
"""
import math
import os

import torch

from diff_gaussian_rasterization import (GaussianRasterizationSettings, GaussianRasterizer,
                                         rasterize_gaussians_split_sh, split_sh_ok)

from . import _lib
from .rigid import from_homogenous, to_homogenous
from .sh import eval_sh


class _GaussianInputs(torch.autograd.Function):
    """(xyz, f_dc, f_rest, scaling, rotation, opacity, deform (N, 10) | None) ->
    (means3D, shs, opacities, scales, rotations) of gaussian_renderer/__init__.py:70-112."""

    @staticmethod
    def forward(ctx, xyz, f_dc, f_rest, scaling, rotation, opacity, deform, se3=False, with_sh=True):
        lib = _lib.load()
        P = xyz.shape[0]
        M_rest = f_rest.shape[1]
        dev = xyz.device
        e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)  # noqa: E731
        means3D, scales, rots, opac = e(P, 3), e(P, 3), e(P, 4), e(P, 1)
        # with_sh False: the split-SH rasterizer reads features_dc / features_rest itself (no cat)
        shs = e(P, 1 + M_rest, 3) if with_sh else None
        ds = deform.stride(0) if deform is not None else 0
        fwd = lib.dgs_gaussian_inputs_se3_forward if se3 else lib.dgs_gaussian_inputs_forward
        _lib.check(fwd(
            P, M_rest, _lib.ptr(xyz), _lib.ptr(f_dc), _lib.ptr(f_rest), _lib.ptr(scaling), _lib.ptr(rotation),
            _lib.ptr(opacity), _lib.ptr(deform), ds, _lib.ptr(means3D), _lib.ptr(shs), _lib.ptr(scales),
            _lib.ptr(rots), _lib.ptr(opac), _lib.stream_ptr(dev)), "gaussian_inputs_forward")
        if se3:  # the screw rows and xyz are read again by the backward
            ctx.save_for_backward(scaling, rotation, opacity, xyz, deform)
        else:
            ctx.save_for_backward(scaling, rotation, opacity)
        ctx.M_rest = M_rest
        ctx.has_deform = deform is not None
        ctx.se3 = se3
        ctx.with_sh = with_sh
        return means3D, shs, opac, scales, rots

    @staticmethod
    def backward(ctx, g_means, g_shs, g_opac, g_scales, g_rots):
        lib = _lib.load()
        scaling, rotation, opacity = ctx.saved_tensors[:3]
        P, M_rest = scaling.shape[0], ctx.M_rest
        dev = scaling.device
        z = lambda t, *shape: (torch.zeros(shape, dtype=torch.float32, device=dev) if t is None  # noqa: E731
                               else t.contiguous())
        g_means, g_opac = z(g_means, P, 3), z(g_opac, P, 1)
        g_shs = z(g_shs, P, 1 + M_rest, 3) if ctx.with_sh else None
        g_scales, g_rots = z(g_scales, P, 3), z(g_rots, P, 4)
        need = ctx.needs_input_grad
        e = lambda ok, *shape: torch.empty(shape, dtype=torch.float32, device=dev) if ok else None  # noqa: E731
        o_xyz = e(need[0], P, 3)
        o_dc, o_rest = e(need[1] and ctx.with_sh, P, 1, 3), e(need[2] and ctx.with_sh, P, M_rest, 3)
        o_sc, o_rot, o_op = e(need[3], P, 3), e(need[4], P, 4), e(need[5], P, 1)
        if ctx.se3:
            xyz, deform = ctx.saved_tensors[3:]
            o_def = e(need[6], P, deform.shape[1])
            _lib.check(lib.dgs_gaussian_inputs_se3_backward(
                P, M_rest, _lib.ptr(xyz), _lib.ptr(deform), deform.stride(0), _lib.ptr(scaling), _lib.ptr(rotation),
                _lib.ptr(opacity), _lib.ptr(g_means), _lib.ptr(g_shs), _lib.ptr(g_scales), _lib.ptr(g_rots),
                _lib.ptr(g_opac), _lib.ptr(o_xyz), _lib.ptr(o_dc), _lib.ptr(o_rest), _lib.ptr(o_sc), _lib.ptr(o_rot),
                _lib.ptr(o_op), _lib.ptr(o_def), _lib.stream_ptr(dev)), "gaussian_inputs_se3_backward")
            return o_xyz, o_dc, o_rest, o_sc, o_rot, o_op, o_def, None, None, None
        o_def = e(ctx.has_deform and need[6], P, 10)
        _lib.check(lib.dgs_gaussian_inputs_backward(
            P, M_rest, _lib.ptr(scaling), _lib.ptr(rotation), _lib.ptr(opacity), _lib.ptr(g_means), _lib.ptr(g_shs),
            _lib.ptr(g_scales), _lib.ptr(g_rots), _lib.ptr(g_opac), _lib.ptr(o_xyz), _lib.ptr(o_dc), _lib.ptr(o_rest),
            _lib.ptr(o_sc), _lib.ptr(o_rot), _lib.ptr(o_op), _lib.ptr(o_def), 10, _lib.stream_ptr(dev)),
            "gaussian_inputs_backward")
        return o_xyz, o_dc, o_rest, o_sc, o_rot, o_op, o_def, None, None


# DGS_SPLIT_SH=0 (A/B diagnostic): the fused path concatenates the SH rows for the plain rasterizer
_SPLIT_SH = os.environ.get("DGS_SPLIT_SH", "1") not in ("", "0")

# override_color: the reference accepts it but never uses it (gaussian_renderer/__init__.py:101-113 test
# `colors_precomp is None`, which always holds, so SHs are rasterized), and so does render() here by
# default. DGS_HONOR_OVERRIDE_COLOR=1 / set_honor_override_color(True) rasterizes override_color as the
# precomputed colours instead (what the argument evidently intends; a different image from the reference).
_HONOR_OVERRIDE = {"on": os.environ.get("DGS_HONOR_OVERRIDE_COLOR", "0") not in ("", "0")}


def set_honor_override_color(on):
    _HONOR_OVERRIDE["on"] = bool(on)


# the fused render-input launches on the training path; off: the reference's torch glue for every call
# (deformgs/train.py fused=False, the comparison loop)
_FUSED = {"on": True}


def set_fused(on):
    _FUSED["on"] = bool(on)


def set_deterministic(on):
    """Bitwise-reproducible rasterizer gradients (libdgs: dgs_raster_set_deterministic; also
    DGS_DETERMINISTIC=1): the blend backward sums every Gaussian's per-tile terms in a fixed order instead
    of the reference's float atomics. Off by default (it costs the per-pair slot traffic). Returns the
    previous setting."""
    from . import _lib
    lib = _lib.load()
    before = bool(lib.dgs_raster_get_deterministic())
    lib.dgs_raster_set_deterministic(1 if on else 0)
    return before


def _fused_deform_rows(pc, d_xyz, d_rotation, d_scaling):
    """The (N, 10) deformation output the three deltas are column views of, 0 for no deformation,
    or None when the deltas have any other form (then the generic torch glue runs)."""
    if not torch.is_tensor(d_xyz) and not torch.is_tensor(d_rotation) and not torch.is_tensor(d_scaling):
        return 0 if (d_xyz == 0 and d_rotation == 0 and d_scaling == 0) else None
    if not (torch.is_tensor(d_xyz) and torch.is_tensor(d_rotation) and torch.is_tensor(d_scaling)):
        return None
    b = d_xyz._base
    if b is None or d_rotation._base is not b or d_scaling._base is not b:
        return None
    N = pc._xyz.shape[0]
    if b.dim() != 2 or tuple(b.shape) != (N, 10) or not b.is_contiguous() or b.dtype != torch.float32:
        return None
    off = b.storage_offset()
    for t, col, w in ((d_xyz, 0, 3), (d_rotation, 3, 4), (d_scaling, 7, 3)):
        if tuple(t.shape) != (N, w) or t.stride() != (10, 1) or t.storage_offset() - off != col:
            return None
    return b


def _fused_se3_rows(pc, d_xyz, d_rotation, d_scaling):
    """The (N, 13) raw 6-DoF deformation output [w_r v_r d_rot d_scale] behind d_xyz (the (N, 4, 4)
    screw matrices DeformNetwork returns, tagged with their source) when d_rotation / d_scaling are
    its column views, else None (then the generic torch glue runs on the matrices)."""
    b = getattr(d_xyz, "_dgs_se3_raw", None) if torch.is_tensor(d_xyz) else None
    if b is None or not (torch.is_tensor(d_rotation) and torch.is_tensor(d_scaling)):
        return None
    if d_rotation._base is not b or d_scaling._base is not b:
        return None
    N = pc._xyz.shape[0]
    if b.dim() != 2 or tuple(b.shape) != (N, 13) or not b.is_contiguous() or b.dtype != torch.float32:
        return None
    off = b.storage_offset()
    for t, col, w in ((d_rotation, 6, 4), (d_scaling, 10, 3)):
        if tuple(t.shape) != (N, w) or t.stride() != (13, 1) or t.storage_offset() - off != col:
            return None
    return b


def _fused_ok(pc):
    ts = (pc._xyz, pc._features_dc, pc._features_rest, pc._scaling, pc._rotation, pc._opacity)
    return (all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in ts)
            and pc._features_dc.dim() == 3 and pc._features_dc.shape[1] == 1
            and pc.scaling_activation is torch.exp and pc.opacity_activation is torch.sigmoid
            and pc.rotation_activation is torch.nn.functional.normalize)


def render(viewpoint_camera, pc, pipe, bg_color, d_xyz, d_rotation, d_scaling, is_6dof=False,
           scaling_modifier=1.0, override_color=None, direct_compute=False):
    dev = pc.get_xyz.device
    if not _HONOR_OVERRIDE["on"]:
        override_color = None  # the reference's behaviour (see _HONOR_OVERRIDE)
    # gaussian_renderer/__init__.py:41-47 builds these as zeros + 0 with retain_grad; the rasterizer never
    # reads their values (only .grad is delivered), so uninitialised leaf tensors serve: their .grad is
    # populated directly and no fill / add kernels run per render
    screenspace_points = torch.empty_like(pc.get_xyz, device=dev).requires_grad_(True)
    screenspace_points_densify = torch.empty_like(pc.get_xyz, device=dev).requires_grad_(True)
    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=pc.active_sh_degree, campos=viewpoint_camera.camera_center, prefiltered=False,
        debug=getattr(pipe, "debug", False))
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    rows, se3 = None, False
    if (_FUSED["on"] and not direct_compute and override_color is None and not getattr(pipe, "compute_cov3D_python", False)
            and not getattr(pipe, "convert_SHs_python", False) and _fused_ok(pc)):
        if not is_6dof:
            rows = _fused_deform_rows(pc, d_xyz, d_rotation, d_scaling)
        elif not torch.is_tensor(d_xyz):  # 6-DoF warm-up: means3D = xyz (no screw yet)
            rows = _fused_deform_rows(pc, 0.0, d_rotation, d_scaling)
        else:
            rows = _fused_se3_rows(pc, d_xyz, d_rotation, d_scaling)
            se3 = rows is not None
    if rows is not None:
        split = _SPLIT_SH and split_sh_ok(pc._features_dc, pc._features_rest)
        means3D, shs, opacity, scales, rotations = _GaussianInputs.apply(
            pc._xyz, pc._features_dc, pc._features_rest, pc._scaling, pc._rotation, pc._opacity,
            rows if torch.is_tensor(rows) else None, se3, not split)
        if split:  # SH rows read / written in place by the rasterizer (no (N, 16, 3) cat either way)
            rendered_image, radii, depth, visible = rasterize_gaussians_split_sh(
                means3D, screenspace_points, screenspace_points_densify, pc._features_dc, pc._features_rest, opacity,
                scales, rotations, raster_settings)
        else:
            rendered_image, radii, depth = rasterizer(
                means3D=means3D, means2D=screenspace_points, means2D_densify=screenspace_points_densify, shs=shs,
                colors_precomp=None, opacities=opacity, scales=scales, rotations=rotations, cov3D_precomp=None)
            visible = radii > 0
        return {"render": rendered_image, "viewspace_points": screenspace_points,
                "viewspace_points_densify": screenspace_points_densify, "visibility_filter": visible,
                "radii": radii, "depth": depth}
    if direct_compute:
        means3D = d_xyz
    elif is_6dof:
        if torch.is_tensor(d_xyz) is False:
            means3D = pc.get_xyz
        else:
            means3D = from_homogenous(torch.bmm(d_xyz, to_homogenous(pc.get_xyz).unsqueeze(-1)).squeeze(-1))
    else:
        means3D = pc.get_xyz + d_xyz
    opacity = pc.get_opacity
    scales = rotations = cov3D_precomp = None
    if getattr(pipe, "compute_cov3D_python", False):
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    elif d_scaling is None and d_rotation is None:
        scales = pc.get_scaling
        rotations = pc.get_rotation
    elif direct_compute:
        scales, rotations = d_scaling, d_rotation
    else:
        scales = pc.get_scaling + d_scaling
        rotations = pc.get_rotation + d_rotation
    shs = colors_precomp = None
    if override_color is None:
        if getattr(pipe, "convert_SHs_python", False):
            shs_view = pc.get_features.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
            dir_pp = pc.get_xyz - viewpoint_camera.camera_center.repeat(pc.get_features.shape[0], 1)
            dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
            sh2rgb = eval_sh(pc.active_sh_degree, shs_view, dir_pp_normalized)
            colors_precomp = torch.clamp_min(sh2rgb + 0.5, 0.0)
        else:
            shs = pc.get_features
    else:
        colors_precomp = override_color
    rendered_image, radii, depth = rasterizer(
        means3D=means3D, means2D=screenspace_points, means2D_densify=screenspace_points_densify, shs=shs,
        colors_precomp=colors_precomp, opacities=opacity, scales=scales, rotations=rotations,
        cov3D_precomp=cov3D_precomp)
    return {"render": rendered_image, "viewspace_points": screenspace_points,
            "viewspace_points_densify": screenspace_points_densify, "visibility_filter": radii > 0,
            "radii": radii, "depth": depth}
