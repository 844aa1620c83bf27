"""render() — same signature and return dict as gaussian_renderer/__init__.py:32-133.

The rasterizer underneath is this repo's diff_gaussian_rasterization (libdgs_hip.so). Glue math
(means3D = xyz + d_xyz or the 6-DoF transform, scales = exp(_scaling) + d_scale, rotations =
normalize(_rotation) + d_rot without re-normalisation, opacity = sigmoid) is unchanged.
"""
import math

import torch

from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

from .rigid import from_homogenous, to_homogenous
from .sh import eval_sh


def render(viewpoint_camera, pc, pipe, bg_color, d_xyz, d_rotation, d_scaling, is_6dof=False,
           scaling_modifier=1.0, override_color=None, direct_compute=False):
    dev = pc.get_xyz.device
    screenspace_points = torch.zeros_like(pc.get_xyz, dtype=pc.get_xyz.dtype, requires_grad=True, device=dev) + 0
    screenspace_points_densify = torch.zeros_like(pc.get_xyz, dtype=pc.get_xyz.dtype, requires_grad=True,
                                                  device=dev) + 0
    try:
        screenspace_points.retain_grad()
        screenspace_points_densify.retain_grad()
    except Exception:
        pass
    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=pc.active_sh_degree, campos=viewpoint_camera.camera_center, prefiltered=False,
        debug=getattr(pipe, "debug", False))
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
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
