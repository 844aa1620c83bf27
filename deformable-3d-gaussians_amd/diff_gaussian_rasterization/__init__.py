"""Drop-in `diff_gaussian_rasterization` for MI355X, backed by libdgs_hip.so (hand-written HIP).

Same Python surface as the module the reference imports at gaussian_renderer/__init__.py:14 and
calls at :53-68 and :115-124 (the un-vendored submodule of .gitmodules:4-7, branch filter-norm):

  GaussianRasterizationSettings  NamedTuple, 12 fields (image_height ... debug)
  GaussianRasterizer(nn.Module)  forward(means3D, means2D, opacities, means2D_densify=None, shs=None,
                                 colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None)
                                 -> (color (3,H,W), radii (N,) int32, depth (1,H,W))
                                 markVisible(positions) -> bool (N,)
  rasterize_gaussians(...)       functional form

means2D / means2D_densify are dummy tensors whose .grad receives dL/d(mean2D) (NDC units) and the
densification statistic (per-pixel |dL/dmean2D| summed per axis).
"""
from typing import NamedTuple

import torch
import torch.nn as nn

from deformgs import _lib


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


# Set by deformgs.train_step during a deferred-pair-count step: the backward leaves the context
# alive (freeing it resolves the pair count, a host wait) and the training step frees it once the
# whole backward has been issued (release_context).
_KEEP_CTX = {"on": False}


def release_context(color):
    """Free the rasterizer context behind a rendered image (resolving a deferred pair count)."""
    fn = getattr(color, "grad_fn", None)
    r = getattr(fn, "raster", None) if fn is not None else None
    if isinstance(r, _Ctx):
        r.free()


class _Ctx:
    """Owns one dgs_raster_ctx (geometry/binning/image buffers kept for backward)."""

    def __init__(self, handle):
        self.handle = handle

    def free(self):
        if self.handle:
            _lib.load().dgs_raster_ctx_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _require_ctx(ctx):
    if ctx.raster.handle is None:
        raise RuntimeError("rasterize_gaussians: a second backward through the same render needs its rasterizer "
                           "context, which the first backward released; keep it with "
                           "diff_gaussian_rasterization._KEEP_CTX['on'] = True (the accumulators are re-zeroed)")


def _f32(t):
    if t is None:
        return None
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _settings_struct(rs, keep):
    bg = _f32(rs.bg)
    view = _f32(rs.viewmatrix)
    proj = _f32(rs.projmatrix)
    campos = _f32(rs.campos)
    _lib.require_cuda(bg, view, proj, campos)
    keep.extend([bg, view, proj, campos])
    s = _lib.RasterSettings()
    s.image_height = int(rs.image_height)
    s.image_width = int(rs.image_width)
    s.tanfovx = float(rs.tanfovx)
    s.tanfovy = float(rs.tanfovy)
    s.bg = _lib.ptr(bg)
    s.scale_modifier = float(rs.scale_modifier)
    s.viewmatrix = _lib.ptr(view)
    s.projmatrix = _lib.ptr(proj)
    s.sh_degree = int(rs.sh_degree)
    s.campos = _lib.ptr(campos)
    s.prefiltered = int(bool(rs.prefiltered))
    s.debug = int(bool(rs.debug))
    return s


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, means2D_densify, shs, colors_precomp, opacities, scales, rotations,
                cov3D_precomp, raster_settings):
        lib = _lib.load()
        keep = []
        s = _settings_struct(raster_settings, keep)
        means3D = _f32(means3D)
        opacities = _f32(opacities)
        # GaussianRasterizer passes torch.Tensor([]) for an absent input (1-D, empty)
        given = lambda t: t is not None and not (t.dim() == 1 and t.numel() == 0)  # noqa: E731
        shs = _f32(shs) if given(shs) else None
        colors_precomp = _f32(colors_precomp) if given(colors_precomp) else None
        scales = _f32(scales) if given(scales) else None
        rotations = _f32(rotations) if given(rotations) else None
        cov3D_precomp = _f32(cov3D_precomp) if given(cov3D_precomp) else None
        if (shs is None) == (colors_precomp is None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if cov3D_precomp is None and (scales is None or rotations is None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        _lib.require_cuda(means3D, opacities, shs, colors_precomp, scales, rotations, cov3D_precomp)
        P = means3D.shape[0]
        if shs is None:
            M = 0
        elif shs.dim() == 3:
            M = shs.shape[1]
        else:
            M = shs.numel() // (3 * P) if P else 0
        H, W = int(raster_settings.image_height), int(raster_settings.image_width)
        dev = means3D.device
        color = torch.empty((3, H, W), dtype=torch.float32, device=dev)
        depth = torch.empty((1, H, W), dtype=torch.float32, device=dev)
        radii = torch.empty((P,), dtype=torch.int32, device=dev)
        handle = _lib.P()
        nr = _lib.I(0)
        rc = lib.dgs_raster_forward(s, P, M, _lib.ptr(means3D), _lib.ptr(shs), _lib.ptr(colors_precomp),
                                    _lib.ptr(opacities), _lib.ptr(scales), _lib.ptr(rotations),
                                    _lib.ptr(cov3D_precomp), _lib.ptr(color), _lib.ptr(depth), _lib.ptr(radii),
                                    handle, nr, _lib.stream_ptr(dev))
        _lib.check(rc, "rasterize_gaussians")
        ctx.raster = _Ctx(handle)
        ctx.raster_hw = (H, W)
        ctx.keep = keep
        ctx.num_rendered = nr.value
        ctx.M = M
        ctx.flags = (shs is not None, colors_precomp is not None, cov3D_precomp is not None)
        ctx.shapes = (shs.shape if shs is not None else None, None if scales is None else scales.shape,
                      None if rotations is None else rotations.shape)
        ctx.save_for_backward(means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, radii)
        ctx.mark_non_differentiable(radii)
        # an unused depth output (every training loss here) arrives as None: no zero-fill kernel
        ctx.set_materialize_grads(False)
        return color, radii, depth

    @staticmethod
    def backward(ctx, grad_color, grad_radii, grad_depth):
        lib = _lib.load()
        _require_ctx(ctx)
        means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, radii = ctx.saved_tensors
        P = means3D.shape[0]
        dev = means3D.device
        has_sh, has_col, has_cov = ctx.flags
        e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)  # noqa: E731
        d_means3D = e(P, 3)
        d_means2D = e(P, 3)
        d_dens = e(P, 3)
        d_opac = e(P, 1)
        d_col = e(P, 3) if has_col else None
        d_cov = e(P, 6) if has_cov else None
        d_shs = e(*shs.shape) if has_sh else None
        d_scales = e(P, 3) if not has_cov else None
        d_rots = e(P, 4) if not has_cov else None
        if grad_color is None:
            grad_color = torch.zeros((3, ctx.raster_hw[0], ctx.raster_hw[1]), dtype=torch.float32, device=dev)
        gc = _f32(grad_color)
        gd = _f32(grad_depth) if grad_depth is not None else None
        rc = lib.dgs_raster_backward(ctx.raster.handle, _lib.ptr(gc), _lib.ptr(gd), _lib.ptr(d_means3D),
                                     _lib.ptr(d_means2D), _lib.ptr(d_dens), _lib.ptr(d_col), _lib.ptr(d_opac),
                                     _lib.ptr(d_cov), _lib.ptr(d_shs), _lib.ptr(d_scales), _lib.ptr(d_rots),
                                     _lib.stream_ptr(dev))
        _lib.check(rc, "rasterize_gaussians_backward")
        if not _KEEP_CTX["on"]:
            ctx.raster.free()
        return (d_means3D, d_means2D, d_dens, d_shs, d_col, d_opac.view_as(opacities), d_scales, d_rots, d_cov, None)


class _RasterizeGaussiansSplitSH(torch.autograd.Function):
    """The same op with the SH rows read from (features_dc (P,1,3), features_rest (P,15,3)) and their
    gradients written back to both (dgs_raster_*_split_sh): render()'s training path, where the
    reference concatenates them every call (scene/gaussian_model.py:71-74). Not part of the upstream
    module's interface; results are those of shs = cat(features_dc, features_rest)."""

    @staticmethod
    def forward(ctx, means3D, means2D, means2D_densify, f_dc, f_rest, opacities, scales, rotations, raster_settings):
        lib = _lib.load()
        keep = []
        s = _settings_struct(raster_settings, keep)
        P = means3D.shape[0]
        H, W = int(raster_settings.image_height), int(raster_settings.image_width)
        dev = means3D.device
        color = torch.empty((3, H, W), dtype=torch.float32, device=dev)
        depth = torch.empty((1, H, W), dtype=torch.float32, device=dev)
        radii = torch.empty((P,), dtype=torch.int32, device=dev)
        visible = torch.empty((P,), dtype=torch.bool, device=dev)  # radii > 0, written by the preprocess
        handle = _lib.P()
        nr = _lib.I(0)
        rc = lib.dgs_raster_forward_split_sh(s, P, _lib.ptr(means3D), _lib.ptr(f_dc), _lib.ptr(f_rest),
                                             _lib.ptr(opacities), _lib.ptr(scales), _lib.ptr(rotations),
                                             _lib.ptr(color), _lib.ptr(depth), _lib.ptr(radii), _lib.ptr(visible),
                                             handle, nr, _lib.stream_ptr(dev))
        _lib.check(rc, "rasterize_gaussians")
        ctx.raster = _Ctx(handle)
        ctx.raster_hw = (H, W)
        ctx.keep = keep
        ctx.num_rendered = nr.value
        ctx.P = P
        # the saved C context points at these inputs: keep them alive (and version-checked) until backward
        ctx.save_for_backward(radii, means3D, f_dc, f_rest, opacities, scales, rotations)
        ctx.mark_non_differentiable(radii, visible)
        ctx.set_materialize_grads(False)
        return color, radii, depth, visible

    @staticmethod
    def backward(ctx, grad_color, grad_radii, grad_depth, grad_visible):
        lib = _lib.load()
        _require_ctx(ctx)
        radii = ctx.saved_tensors[0]
        P, dev = ctx.P, radii.device
        e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)  # noqa: E731
        d_means3D, d_means2D, d_dens, d_opac = e(P, 3), e(P, 3), e(P, 3), e(P, 1)
        d_dc, d_rest, d_scales, d_rots = e(P, 1, 3), e(P, 15, 3), e(P, 3), e(P, 4)
        if grad_color is None:
            grad_color = torch.zeros((3, ctx.raster_hw[0], ctx.raster_hw[1]), dtype=torch.float32, device=dev)
        gc = _f32(grad_color)
        gd = _f32(grad_depth) if grad_depth is not None else None
        rc = lib.dgs_raster_backward_split_sh(ctx.raster.handle, _lib.ptr(gc), _lib.ptr(gd), _lib.ptr(d_means3D),
                                              _lib.ptr(d_means2D), _lib.ptr(d_dens), _lib.ptr(d_opac),
                                              _lib.ptr(d_dc), _lib.ptr(d_rest), _lib.ptr(d_scales),
                                              _lib.ptr(d_rots), _lib.stream_ptr(dev))
        _lib.check(rc, "rasterize_gaussians_backward")
        if not _KEEP_CTX["on"]:
            ctx.raster.free()
        return d_means3D, d_means2D, d_dens, d_dc, d_rest, d_opac, d_scales, d_rots, None


def split_sh_ok(f_dc, f_rest):
    """(features_dc, features_rest) the split-SH op takes: fp32 CUDA, contiguous (P,1,3) / (P,15,3),
    16-byte aligned."""
    return (f_dc.is_cuda and f_dc.dtype == torch.float32 and f_rest.dtype == torch.float32 and f_dc.is_contiguous()
            and f_rest.is_contiguous() and f_dc.dim() == 3 and tuple(f_dc.shape[1:]) == (1, 3)
            and f_rest.dim() == 3 and tuple(f_rest.shape[1:]) == (15, 3) and f_rest.shape[0] == f_dc.shape[0]
            and f_dc.data_ptr() % 16 == 0 and f_rest.data_ptr() % 16 == 0)


def rasterize_gaussians_split_sh(means3D, means2D, means2D_densify, f_dc, f_rest, opacities, scales, rotations,
                                 raster_settings):
    """-> (color, radii, depth, visible = radii > 0)"""
    return _RasterizeGaussiansSplitSH.apply(means3D, means2D, means2D_densify, f_dc, f_rest, opacities, scales,
                                            rotations, raster_settings)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings, means2D_densify=None):
    if means2D_densify is None:
        means2D_densify = torch.zeros_like(means3D)
    return _RasterizeGaussians.apply(means3D, means2D, means2D_densify, sh, colors_precomp, opacities, scales,
                                     rotations, cov3Ds_precomp, raster_settings)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            rs = self.raster_settings
            pos = _f32(positions)
            view = _f32(rs.viewmatrix)
            proj = _f32(rs.projmatrix)
            _lib.require_cuda(pos, view, proj)
            vis = torch.empty((pos.shape[0],), dtype=torch.uint8, device=pos.device)
            rc = _lib.load().dgs_mark_visible(pos.shape[0], _lib.ptr(pos), _lib.ptr(view), _lib.ptr(proj),
                                              _lib.ptr(vis), _lib.stream_ptr(pos.device))
            _lib.check(rc, "mark_visible")
        return vis.bool()

    def forward(self, means3D, means2D, opacities, means2D_densify=None, shs=None, colors_precomp=None, scales=None,
                rotations=None, cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        empty = torch.Tensor([])
        shs = empty if shs is None else shs
        colors_precomp = empty if colors_precomp is None else colors_precomp
        scales = empty if scales is None else scales
        rotations = empty if rotations is None else rotations
        cov3D_precomp = empty if cov3D_precomp is None else cov3D_precomp
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, rs, means2D_densify=means2D_densify)
