"""Deformation networks on the fused HIP MLP (libdgs_hip.so: dgs_deform_*).

DeformNetworkBaseline / DeformNetwork keep the reference's module tree, parameter names, shapes
and init (utils/time_utils.py:56-201), so `state_dict()` / `load_state_dict()` and
deform/iteration_k/deform.pth files are interchangeable with the reference. forward(x, t) runs
PE + timenet + 8x256 trunk + heads in one MFMA kernel; backward runs the dX chain kernel and the
split-N dW GEMM. Only the reference's shape is supported (D=8, W=256, multires=10): other shapes
raise. Gradients flow to the parameters only — every reference call site detaches x
(train_baseline.py:115, render*.py) and t never requires grad; asking for d/dx raises.
"""
import os

import torch
import torch.nn as nn

from . import _lib

FLAG_BLENDER = 1
FLAG_6DOF = 2
FLAG_NO_ROTSCALE = 4
FLAG_EXACT_FP32 = 8  # v_mfma_f32_32x32x2_f32 kernels instead of the split-f16 (f16x3) default
FLAG_UNIFORM_T = 16  # every point carries t[0] (set when t is one value or a stride-0 expand)


# DGS_SE3_GLUE=1 (A/B diagnostic): render() applies the 6-DoF matrices with the reference's torch glue
_SE3_GLUE = os.environ.get("DGS_SE3_GLUE", "0") not in ("", "0")


def _exact_default():
    return os.environ.get("DGS_MLP_EXACT_FP32", "0") not in ("", "0")


def get_embedder_out_dim(multires, i=1):
    return i + i * 2 * multires


class _FusedDeformMLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flags, x, t, *params):
        lib = _lib.load()
        dev = x.device
        N = x.shape[0]
        stream = _lib.stream_ptr(dev)
        packed = torch.empty(lib.dgs_deform_packed_floats(flags), dtype=torch.float32, device=dev)
        params_c = [p.detach().contiguous() for p in params]
        _lib.check(lib.dgs_deform_pack(flags, _lib.ptr_array(params_c), _lib.ptr(packed), stream), "deform_pack")
        nout = lib.dgs_deform_outputs(flags)
        out = torch.empty((N, nout), dtype=torch.float32, device=dev)
        need_grad = any(ctx.needs_input_grad[3:])
        saved = (torch.empty(lib.dgs_deform_saved_floats(flags, N), dtype=torch.float32, device=dev)
                 if need_grad else None)
        rc = lib.dgs_deform_forward(flags, N, _lib.ptr(x), _lib.ptr(t), _lib.ptr(packed), _lib.ptr(out),
                                    _lib.ptr(saved), stream)
        _lib.check(rc, "deform_forward")
        ctx.flags = flags
        ctx.N = N
        ctx.param_shapes = [p.shape for p in params]
        if need_grad:
            ctx.save_for_backward(packed, saved)
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = _lib.load()
        packed, saved = ctx.saved_tensors
        dev = packed.device
        flags, N = ctx.flags, ctx.N
        grads = [torch.empty(s, dtype=torch.float32, device=dev) for s in ctx.param_shapes]
        scratch = torch.empty(lib.dgs_deform_scratch_floats(flags, N), dtype=torch.float32, device=dev)
        dout = dout.contiguous().float()
        rc = lib.dgs_deform_backward(flags, N, _lib.ptr(packed), _lib.ptr(saved), _lib.ptr(dout), _lib.ptr(scratch),
                                     _lib.ptr_array(grads), _lib.stream_ptr(dev))
        _lib.check(rc, "deform_backward")
        return (None, None, None, *grads)


class _ScrewSE3(torch.autograd.Function):
    """Raw screw head (w_r, v_r) -> d_xyz (N, 4, 4) = rp_to_se3(exp_se3(...)) (utils/time_utils.py:114-121,
    utils/rigid_utils.py:4-83) in one HIP launch each way (dgs_se3_*); rigid.screw_from_raw is the torch
    statement of the same map."""

    @staticmethod
    def forward(ctx, wv):
        lib = _lib.load()
        N = wv.shape[0]
        assert wv.dim() == 2 and wv.shape[1] == 6 and wv.stride(1) == 1 and wv.dtype == torch.float32
        M = torch.empty((N, 4, 4), dtype=torch.float32, device=wv.device)
        _lib.check(lib.dgs_se3_forward(N, _lib.ptr(wv), wv.stride(0), _lib.ptr(M), _lib.stream_ptr(wv.device)),
                   "se3_forward")
        ctx.save_for_backward(wv)
        return M

    @staticmethod
    def backward(ctx, dM):
        lib = _lib.load()
        (wv,) = ctx.saved_tensors
        N = wv.shape[0]
        g = torch.empty((N, 6), dtype=torch.float32, device=wv.device)
        dM = dM.contiguous().float()
        _lib.check(lib.dgs_se3_backward(N, _lib.ptr(wv), wv.stride(0), _lib.ptr(dM), _lib.ptr(g), 6,
                                        _lib.stream_ptr(wv.device)), "se3_backward")
        return g


class _DeformBase(nn.Module):
    _rotscale = True

    def __init__(self, D=8, W=256, input_ch=3, output_ch=59, multires=10, is_blender=False, is_6dof=False,
                 exact_fp32=None):
        super().__init__()
        if D != 8 or W != 256 or multires != 10:
            raise NotImplementedError("fused deformation MLP supports the reference shape D=8, W=256, multires=10")
        self.D, self.W = D, W
        self.input_ch, self.output_ch = input_ch, output_ch
        self.t_multires = 6 if is_blender else 10
        self.skips = [D // 2]
        time_input_ch = get_embedder_out_dim(self.t_multires, 1)
        xyz_input_ch = get_embedder_out_dim(multires, 3)
        self.input_ch = xyz_input_ch + time_input_ch
        if is_blender:
            self.time_out = 30
            self.timenet = nn.Sequential(nn.Linear(time_input_ch, 256), nn.ReLU(inplace=True),
                                         nn.Linear(256, self.time_out))
            self.linear = nn.ModuleList(
                [nn.Linear(xyz_input_ch + self.time_out, W)] + [
                    nn.Linear(W, W) if i not in self.skips else nn.Linear(W + xyz_input_ch + self.time_out, W)
                    for i in range(D - 1)])
        else:
            self.linear = nn.ModuleList(
                [nn.Linear(self.input_ch, W)] + [
                    nn.Linear(W, W) if i not in self.skips else nn.Linear(W + self.input_ch, W)
                    for i in range(D - 1)])
        self.is_blender = is_blender
        self.is_6dof = is_6dof
        if is_6dof:
            self.branch_w = nn.Linear(W, 3)
            self.branch_v = nn.Linear(W, 3)
        else:
            self.gaussian_warp = nn.Linear(W, 3)
        self.gaussian_rotation = nn.Linear(W, 4)
        self.gaussian_scaling = nn.Linear(W, 3)
        self.flags = (FLAG_BLENDER if is_blender else 0) | (FLAG_6DOF if is_6dof else 0) | (
            0 if self._rotscale else FLAG_NO_ROTSCALE)
        # GEMM arithmetic: fp32 on f16 MFMA over a scaled hi/lo split (default) or fp32-input MFMA;
        # both are fp32-accurate (include/dgs.h), the flag is not part of the state_dict
        self.exact_fp32 = _exact_default() if exact_fp32 is None else bool(exact_fp32)

    def kernel_params(self):
        """Parameters in the order of the C ABI's table (include/dgs.h)."""
        ps = []
        if self.is_blender:
            ps += [self.timenet[0].weight, self.timenet[0].bias, self.timenet[2].weight, self.timenet[2].bias]
        for l in self.linear:
            ps += [l.weight, l.bias]
        heads = [self.branch_w, self.branch_v] if self.is_6dof else [self.gaussian_warp]
        heads += [self.gaussian_rotation, self.gaussian_scaling]
        for h in heads:
            ps += [h.weight, h.bias]
        return ps

    def raw(self, x, t):
        """(N, 10) [d_xyz, d_rot, d_scale] or (N, 13) [w, v, d_rot, d_scale] from the fused kernel."""
        if (x.requires_grad or t.requires_grad) and torch.is_grad_enabled():
            raise NotImplementedError("fused deformation MLP does not differentiate w.r.t. its inputs; "
                                      "detach xyz / t as every reference call site does")
        _lib.require_cuda(x, t)
        N = x.shape[0]
        # one frame time for every Gaussian (train_baseline.py:107-110: fid.unsqueeze(0).expand(N, -1),
        # ast_noise likewise expanded from (1, 1)): recognisable without a device read as a single value
        # or a stride-0 expand; the kernels then form the timenet gradients from the bias gradients
        uniform = t.numel() == 1 or (t.dim() >= 1 and t.shape[0] == N and t.stride(0) == 0)
        x = x.detach().float().contiguous()
        params = self.kernel_params()
        saves = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        if uniform and saves and self.is_blender and not self.exact_fp32 and t.dtype == torch.float32:
            # a training forward of the split path of a blender network (timenet) with one frame time
            # reads t[0] only (k_timenet): pass the (stride-0) column as is, no per-step copy kernel
            t = t.detach()
        else:
            t = t.detach().float().reshape(-1, 1).expand(N, 1).contiguous()
        flags = self.flags | (FLAG_EXACT_FP32 if self.exact_fp32 else 0) | (FLAG_UNIFORM_T if uniform else 0)
        return _FusedDeformMLP.apply(flags, x, t, *params)

    def glue_forward(self, x, t):
        """The reference's own torch forward (utils/time_utils.py:102-127: PE by cat of sin / cos bands,
        timenet, 8 x Linear + ReLU with the skip cat after layer 4, heads) on these parameters: the
        torch-glue comparison path of the training loop (deformgs/train.py fused=False), not the product
        path. rocBLAS fp32 GEMMs; gradients by autograd."""
        import torch.nn.functional as F
        from .rigid import screw_from_raw

        def embed(v, L):
            bands = [v]
            for i in range(L):
                f = 2.0 ** i
                bands += [torch.sin(v * f), torch.cos(v * f)]
            return torch.cat(bands, -1)

        t_emb = embed(t, self.t_multires)
        if self.is_blender:
            t_emb = self.timenet(t_emb)
        x_emb = embed(x, 10)
        h = torch.cat([x_emb, t_emb], dim=-1)
        for i, lin in enumerate(self.linear):
            h = F.relu(lin(h))
            if i in self.skips:
                h = torch.cat([x_emb, t_emb, h], -1)
        if self.is_6dof:
            d_xyz = screw_from_raw(self.branch_w(h), self.branch_v(h))
        else:
            d_xyz = self.gaussian_warp(h)
        if not self._rotscale:
            return d_xyz, 0, 0
        return d_xyz, self.gaussian_rotation(h), self.gaussian_scaling(h)

    def forward(self, x, t):
        out = self.raw(x, t)
        if self.is_6dof:
            d_xyz = _ScrewSE3.apply(out[:, 0:6])
            # render(..., is_6dof=True) recognises this and applies the screw to xyz inside its own input
            # launch (dgs_gaussian_inputs_se3_*), reading the raw rows instead of the (N, 4, 4) matrices
            if not _SE3_GLUE:
                d_xyz._dgs_se3_raw = out
            rot, scale = out[:, 6:10], out[:, 10:13]
        else:
            d_xyz = out[:, 0:3]
            rot, scale = out[:, 3:7], out[:, 7:10]
        if not self._rotscale:
            return d_xyz, 0, 0
        return d_xyz, rot, scale


class DeformNetworkBaseline(_DeformBase):
    """utils/time_utils.py:56-127."""
    _rotscale = True


class DeformNetwork(_DeformBase):
    """utils/time_utils.py:129-201 (fork variant: rotation = scaling = 0)."""
    _rotscale = False
