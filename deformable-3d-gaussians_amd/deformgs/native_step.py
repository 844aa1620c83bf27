"""One training iteration through dgs_train_step (csrc/step.hip): the fused path of
train_step.forward_backward (train_baseline.py:104-128) issued from C++ in one call, without the
PyTorch autograd engine.

Same kernels, same order, same stream as the autograd path (tests/test_gpu_native_step.py holds the
two to the same loss, image and gradients); what changes is the host: one ctypes call with a prebuilt
argument block instead of ~0.85 ms of Python, autograd bookkeeping and tensor allocation per step,
which set the speed of the small configurations (BASELINE config 2, 16k Gaussians at 400x400).
Buffers are allocated once per Gaussian count (densification reallocates them); the parameter
gradients live in persistent buffers handed to the parameters as .grad, overwritten every step.

Used by train_step() on the fused path (DGS_NATIVE_STEP=0 turns it off). Data-parallel steps
(`step_data_parallel`) split the call in two: phase 1 runs up to the Gaussian parameter gradients and
resolves the pair count (an overflow is redone by that rank alone, before any collective); ONE async
all-reduce of the Gaussian gradients (a flat buffer the parameters' .grad tensors are views of: no
concatenation, no copy back) is started and overlaps phase 2, the network backward; then the network
gradients' all-reduce. The autograd path's hooks (dist.OverlappedGradAllReduce) do the same
overlap with a concatenation per step.
"""
import ctypes
import math
import os

import torch

from . import _lib

P_ = ctypes.c_void_p
I_ = ctypes.c_int
F_ = ctypes.c_float


class TrainStepArgs(ctypes.Structure):
    """dgs_train_step_args (include/dgs.h)."""
    _fields_ = [
        ("P", I_), ("xyz", P_), ("f_dc", P_), ("f_rest", P_), ("scaling", P_), ("rotation", P_), ("opacity", P_),
        ("deform", I_), ("mlp_flags", I_), ("mlp_params", P_), ("mlp_grads", P_),
        ("mlp_packed", P_), ("mlp_saved", P_), ("mlp_scratch", P_), ("mlp_out", P_), ("mlp_dout", P_),
        ("t", P_), ("t_full", P_), ("rs", _lib.RasterSettings), ("gt", P_), ("lambda_dssim", F_),
        ("means3D", P_), ("scales", P_), ("rotations", P_), ("opacities", P_),
        ("image", P_), ("depth", P_), ("radii", P_), ("visible", P_),
        ("loss3", P_), ("loss_scratch", P_), ("dimage", P_),
        ("d_means3D", P_), ("d_means2D", P_), ("d_means2D_densify", P_), ("d_opacities", P_), ("d_scales", P_),
        ("d_rotations", P_),
        ("g_xyz", P_), ("g_dc", P_), ("g_rest", P_), ("g_scaling", P_), ("g_rotation", P_), ("g_opacity", P_),
        ("deferred_count", I_), ("phase", I_),
    ]


def enabled():
    return os.environ.get("DGS_NATIVE_STEP", "1") not in ("", "0")


class _GradHolder:
    """Stands in for render()'s screen-space point tensors: only .grad is read (add_densification_stats)."""

    def __init__(self, grad):
        self.grad = grad


def usable(gaussians, deform, pipe, gt_image):
    """The native step covers render()'s fused training path: fused render inputs, split-SH raster,
    SHs and covariance in the rasterizer, the baseline network (rotation / scaling heads on)."""
    from diff_gaussian_rasterization import split_sh_ok
    from .deform_network import _DeformBase
    from .renderer import _FUSED, _HONOR_OVERRIDE, _SPLIT_SH, _fused_ok
    net = getattr(deform, "deform", None)
    return (enabled() and _FUSED["on"] and _SPLIT_SH and not _HONOR_OVERRIDE["on"] and isinstance(net, _DeformBase)
            and net._rotscale and not getattr(pipe, "compute_cov3D_python", False)
            and not getattr(pipe, "convert_SHs_python", False) and not getattr(pipe, "debug", False)
            and _fused_ok(gaussians) and split_sh_ok(gaussians._features_dc, gaussians._features_rest)
            and gaussians._features_rest.shape[1] == 15 and gt_image.is_cuda and gt_image.dtype == torch.float32
            and gt_image.is_contiguous() and gt_image.dim() == 3 and gt_image.shape[0] == 3)


class NativeStep:
    def __init__(self, gaussians, deform):
        self.gs, self.deform = gaussians, deform
        self.key = None
        self.lib = _lib.load()

    def _params(self):
        g = self.gs
        return [g._xyz, g._features_dc, g._features_rest, g._scaling, g._rotation, g._opacity]

    def _ensure(self, H, W):
        """(Re)build buffers and the argument block when the Gaussian set, the network or the image
        size changed (densification replaces the parameter tensors)."""
        gp = self._params()
        net = self.deform.deform
        mp = net.kernel_params()
        key = (tuple(p.data_ptr() for p in gp), tuple(p.data_ptr() for p in mp), gp[0].shape[0], H, W, net.flags,
               net.exact_fp32)
        if key == self.key:
            return
        lib, dev, N = self.lib, gp[0].device, gp[0].shape[0]
        # release the previous set first (densification / opacity resets would otherwise briefly hold
        # two sets of the several-KB-per-Gaussian MLP buffers); the parameters' .grad views of the old
        # flat buffers are dropped with them (the next step hands out the new ones)
        if self.key is not None:
            for p in getattr(self, "params", []):
                if p.grad is not None and any(p.grad is g for g in self.grads):
                    p.grad = None
        self.buf = self.gflat = self.mflat = self.ggrads = self.mgrads = self.grads = self.args = None
        self.key = None
        e = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)  # noqa: E731
        from .deform_network import FLAG_EXACT_FP32
        flags = net.flags | (FLAG_EXACT_FP32 if net.exact_fp32 else 0)
        nout = lib.dgs_deform_outputs(flags)
        b = self.buf = {
            "means3D": e(N, 3), "scales": e(N, 3), "rotations": e(N, 4), "opacities": e(N, 1),
            "depth": e(1, H, W), "radii": torch.empty((N,), dtype=torch.int32, device=dev),
            "visible": torch.empty((N,), dtype=torch.bool, device=dev),
            "loss_scratch": e(lib.dgs_l1_ssim_scratch_floats(3, H, W)), "dimage": e(3, H, W),
            "d_means3D": e(N, 3), "d_means2D": e(N, 3), "d_means2D_densify": e(N, 3), "d_opacities": e(N, 1),
            "d_scales": e(N, 3), "d_rotations": e(N, 4),
            "mlp_packed": e(lib.dgs_deform_packed_floats(flags | 16)),
            "mlp_saved": e(lib.dgs_deform_saved_floats(flags | 16, N)),
            "mlp_scratch": e(lib.dgs_deform_scratch_floats(flags | 16, N)),
            "mlp_out": e(N, nout), "mlp_dout": e(N, nout), "t_full": e(max(N, 1)),
        }
        # persistent parameter gradients (handed to the parameters as .grad; overwritten every step),
        # views of one flat buffer per group (the data-parallel all-reduce runs on it in place)
        self.gflat, self.ggrads = _flat_views(gp)
        self.mflat, self.mgrads = _flat_views(mp)
        self.params = gp + mp
        self.grads = self.ggrads + self.mgrads
        self._mp_arr = (P_ * len(mp))(*[p.data_ptr() for p in mp])
        self._mg_arr = (P_ * len(mp))(*[g.data_ptr() for g in self.mgrads])
        a = self.args = TrainStepArgs()
        a.P = N
        a.xyz, a.f_dc, a.f_rest, a.scaling, a.rotation, a.opacity = (p.data_ptr() for p in gp)
        a.mlp_flags = flags
        a.mlp_params = ctypes.cast(self._mp_arr, P_)
        a.mlp_grads = ctypes.cast(self._mg_arr, P_)
        for k in ("mlp_packed", "mlp_saved", "mlp_scratch", "mlp_out", "mlp_dout", "t_full", "means3D", "scales",
                  "rotations", "opacities", "depth", "radii", "visible", "loss_scratch", "dimage", "d_means3D",
                  "d_means2D", "d_means2D_densify", "d_opacities", "d_scales", "d_rotations"):
            setattr(a, k, b[k].data_ptr())
        a.g_xyz, a.g_dc, a.g_rest, a.g_scaling, a.g_rotation, a.g_opacity = (g.data_ptr() for g in self.ggrads)
        self.key = key

    def __call__(self, cam, gt_image, background, warm=True, ast_noise=0.0, lambda_dssim=0.2, deferred_count=False,
                 phase=0):
        """-> (loss (0-d tensor), render package as render() returns it, overflowed). phase 0: the whole
        step; 1: up to the Gaussian gradients (network_backward() issues the rest)."""
        H, W = int(cam.image_height), int(cam.image_width)
        self._ensure(H, W)
        a, b, lib = self.args, self.buf, self.lib
        dev = self.params[0].device
        keep = []
        # frame time fid + ast_noise (train_baseline.py:107-112), one value for every Gaussian
        t = cam.fid
        if torch.is_tensor(ast_noise) or ast_noise != 0.0:
            t = t.reshape(1) + (ast_noise.reshape(-1)[:1] if torch.is_tensor(ast_noise) else ast_noise)
            keep.append(t)
        a.t = t.data_ptr()
        a.deform = 1 if warm else 0
        bg, view, proj, campos = (x if x.is_contiguous() else x.contiguous() for x in
                                  (background, cam.world_view_transform, cam.full_proj_transform, cam.camera_center))
        keep += [bg, view, proj, campos]
        rs = a.rs
        rs.image_height, rs.image_width = H, W
        rs.tanfovx, rs.tanfovy = math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5)
        rs.bg, rs.scale_modifier = bg.data_ptr(), 1.0
        rs.viewmatrix, rs.projmatrix, rs.campos = view.data_ptr(), proj.data_ptr(), campos.data_ptr()
        rs.sh_degree, rs.prefiltered, rs.debug = int(self.gs.active_sh_degree), 0, 0
        a.gt = gt_image.data_ptr()
        a.lambda_dssim = float(lambda_dssim)
        # outputs a caller may keep past the next step: fresh each step (allocation only, no kernel)
        image = torch.empty((3, H, W), dtype=torch.float32, device=dev)
        loss3 = torch.empty((3,), dtype=torch.float32, device=dev)
        a.image, a.loss3 = image.data_ptr(), loss3.data_ptr()
        a.deferred_count = 1 if deferred_count else 0
        a.phase = phase
        self._warm = warm
        over, nr = I_(0), I_(0)
        _lib.check(lib.dgs_train_step(ctypes.byref(a), ctypes.byref(over), ctypes.byref(nr), _lib.stream_ptr(dev)),
                   "train_step")
        for p, g in zip(self.params, self.grads):
            if p.grad is not g:
                p.grad = g
        if not warm:  # the network did not run: no gradient (autograd leaves .grad None)
            for p in self.params[6:]:
                p.grad = None
        pkg = {"render": image, "viewspace_points": _GradHolder(b["d_means2D"]),
               "viewspace_points_densify": _GradHolder(b["d_means2D_densify"]), "visibility_filter": b["visible"],
               "radii": b["radii"], "depth": b["depth"], "num_rendered": int(nr.value)}
        return loss3[0], pkg, bool(over.value)

    def network_backward(self):
        """Phase 2 of the preceding phase-1 call: the network's dX / dW (nothing in the warm-up)."""
        if not self._warm:
            return
        a = self.args
        a.phase = 2
        _lib.check(self.lib.dgs_train_step(ctypes.byref(a), None, None, _lib.stream_ptr(self.params[0].device)),
                   "train_step")

    def step_data_parallel(self, cam, gt_image, background, warm, ast_noise, lambda_dssim, deferred_count,
                           agreement=None, group=None):
        """One data-parallel step (frame parallelism): phase 1, this rank's own redo of
        an overflowed deferred pair count, the Gaussian gradient all-reduce overlapped with the network
        backward, the network gradient all-reduce. Collectives are issued in the same order on every rank
        (warm is the same on every rank: it depends on the iteration only). -> (loss, pkg, redone).

        No rank agreement is needed (`agreement` is accepted and unused): the pair count is resolved at
        the end of phase 1, BEFORE this step issues any collective, so a rank whose speculative capacity
        overflowed redoes its own phase 1 synchronously and then joins the same collectives as every
        other rank (which simply wait for it inside the all-reduce). Only the autograd path, whose hooks
        may start the early collective before the count is known, needs dist.OverflowAgreement: the
        native path has no per-step host collective at all."""
        import torch.distributed as dist
        from .dist import _avg_op
        loss, pkg, over = self(cam, gt_image, background, warm, ast_noise, lambda_dssim, deferred_count, phase=1)
        redone = False
        if deferred_count and over:
            redone = True
            loss, pkg, _ = self(cam, gt_image, background, warm, ast_noise, lambda_dssim, False, phase=1)
        op = _avg_op(group)
        # the collective stream waits for the compute stream as of here (the Gaussian gradients are
        # final), so the all-reduce runs under the network backward issued next
        works = [dist.all_reduce(self.gflat, op=op, group=group, async_op=True)]
        if warm:
            self.network_backward()
            works.append(dist.all_reduce(self.mflat, op=op, group=group, async_op=True))
        for w in works:
            w.wait()  # a stream dependency (RCCL): the optimizer step queued next runs after both
        if op == dist.ReduceOp.SUM:
            ws = dist.get_world_size(group)
            self.gflat.div_(ws)
            if warm:
                self.mflat.div_(ws)
        return loss, pkg, redone


_ALIGN = 64  # floats: every view starts on a 256-byte boundary (the SH gradient rows need >= 16 B)


def _flat_views(params):
    """One flat fp32 buffer and a view of it shaped like each parameter, each view aligned to _ALIGN
    floats (the padding between views is zero and stays zero: it is all-reduced along, never written)."""
    offs, n = [], 0
    for p in params:
        offs.append(n)
        n += -(-p.numel() // _ALIGN) * _ALIGN
    flat = torch.zeros((max(n, 1),), dtype=torch.float32, device=params[0].device)
    views = [flat[o:o + p.numel()].view(p.shape) for o, p in zip(offs, params)]
    return flat[:n], views
