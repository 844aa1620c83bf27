// One training iteration in one C call: dgs_train_step (include/dgs.h).
//
// The fused path of deformgs/train_step.forward_backward (train_baseline.py:104-128: deform.step ->
// render -> (1 - l) L1 + l (1 - SSIM) -> backward) issued from C++ instead of through the PyTorch
// autograd engine: the same entry points in the same order on the same stream, so the results are
// those of the autograd path (tests/test_gpu_native_step.py), and the host cost of a step is the ~12
// launches' issue (~0.1 ms) instead of ~0.85 ms of Python, autograd and tensor allocation — the part
// that bounds the small configurations (BASELINE config 2: 16k Gaussians at 400x400, a GPU step
// under 0.9 ms). Every buffer is the caller's (allocated once per Gaussian count); the gradients are
// written in place, ready for dgs_adam_step.
#include <hip/hip_runtime.h>

#include "dgs_common.h"

namespace dgs {
namespace {

__global__ void k_fill_scalar(int n, const float *__restrict__ v, float *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = v[0];
}

constexpr int M_REST = 15;

}  // namespace
}  // namespace dgs

extern "C" int dgs_train_step(const dgs_train_step_args *a, int *overflowed, int *num_rendered, void *stream_) {
    using namespace dgs;
    hipStream_t stream = (hipStream_t)stream_;
    if (!a || a->P < 0 || !a->gt || !a->image || !a->depth || !a->radii || !a->loss3 || !a->loss_scratch ||
        !a->dimage || !a->means3D || !a->scales || !a->rotations || !a->opacities) {
        set_error("dgs_train_step: null argument");
        return DGS_ERR_ARGS;
    }
    const int P = a->P;
    const bool warm = a->deform != 0;
    const bool six = (a->mlp_flags & DGS_MLP_6DOF) != 0;
    const int nout = dgs_deform_outputs(a->mlp_flags);
    if (warm && (!a->mlp_params || !a->mlp_grads || !a->mlp_packed || !a->mlp_saved || !a->mlp_scratch ||
                 !a->mlp_out || !a->mlp_dout || !a->t)) {
        set_error("dgs_train_step: the deformation network needs its parameter / gradient tables and buffers");
        return DGS_ERR_ARGS;
    }
    const int phase = a->phase ? a->phase : 3;
    if (phase < 1 || phase > 3) {
        set_error("dgs_train_step: phase must be 0..3");
        return DGS_ERR_ARGS;
    }
    const int flags = a->mlp_flags | DGS_MLP_UNIFORM_T;
    if (phase == 2)  // the network backward of the preceding phase-1 call
        return warm ? dgs_deform_backward(flags, P, a->mlp_packed, a->mlp_saved, a->mlp_dout, a->mlp_scratch,
                                          a->mlp_grads, stream)
                    : DGS_OK;
    long long over0 = dgs_raster_deferred_overflows();
    // ---- deform.step(xyz.detach(), t) (scene/deform_model.py:323-324) with one frame time ----
    if (warm) {
        // the split path of a blender network reads t[0] only (k_timenet); every other kernel a column
        const float *t = a->t;
        if (!(a->mlp_flags & DGS_MLP_BLENDER) || (a->mlp_flags & DGS_MLP_EXACT_FP32)) {
            if (!a->t_full) {
                set_error("dgs_train_step: t_full (P floats) is needed by this network's kernels");
                return DGS_ERR_ARGS;
            }
            if (P > 0) hipLaunchKernelGGL(k_fill_scalar, dim3(div_up(P, 256)), dim3(256), 0, stream, P, a->t, a->t_full);
            DGS_LAUNCH_CHECK("k_fill_scalar", false, stream);
            t = a->t_full;
        }
        // pack + forward (k_pack, k_timenet, the forward: mlp_split.hip pack_forward)
        if (int rc = dgs_deform_pack_forward(flags, a->mlp_params, P, a->xyz, t, a->mlp_packed, a->mlp_out,
                                             a->mlp_saved, stream))
            return rc;
    }
    // ---- render(): input glue, then the split-SH rasterizer (gaussian_renderer/__init__.py:32-133) ----
    // (6-DoF warm-up: means3D = xyz, gaussian_renderer/__init__.py:71-74: the plain input launch)
    const float *rows = warm ? a->mlp_out : nullptr;
    if (warm && six) {
        if (int rc = dgs_gaussian_inputs_se3_forward(P, M_REST, a->xyz, a->f_dc, a->f_rest, a->scaling, a->rotation,
                                                     a->opacity, rows, nout, a->means3D, nullptr, a->scales,
                                                     a->rotations, a->opacities, stream))
            return rc;
    } else {
        if (int rc = dgs_gaussian_inputs_forward(P, M_REST, a->xyz, a->f_dc, a->f_rest, a->scaling, a->rotation,
                                                 a->opacity, rows, warm ? nout : 0, a->means3D, nullptr, a->scales,
                                                 a->rotations, a->opacities, stream))
            return rc;
    }
    dgs_raster_set_deferred_count(a->deferred_count ? 1 : 0);
    dgs_raster_ctx *ctx = nullptr;
    int nr = 0;
    int rc = dgs_raster_forward_split_sh(&a->rs, P, a->means3D, a->f_dc, a->f_rest, a->opacities, a->scales,
                                         a->rotations, a->image, a->depth, a->radii, a->visible, &ctx, &nr, stream);
    if (rc) {
        dgs_raster_set_deferred_count(0);
        return rc;
    }
    // ---- (1 - l) L1 + l (1 - SSIM) and its gradient (train_baseline.py:126-128) ----
    const int H = a->rs.image_height, W = a->rs.image_width;
    rc = dgs_l1_ssim_forward(3, H, W, a->image, a->gt, a->lambda_dssim, a->loss3, a->loss_scratch, stream);
    if (!rc) rc = dgs_l1_ssim_backward(3, H, W, a->image, a->gt, a->lambda_dssim, a->loss_scratch, nullptr, a->dimage,
                                       stream);
    // ---- backward: rasterizer (SH gradients straight into the parameters'), input glue, network ----
    if (!rc) rc = dgs_raster_backward_split_sh(ctx, a->dimage, nullptr, a->d_means3D, a->d_means2D,
                                               a->d_means2D_densify, a->d_opacities, a->g_dc, a->g_rest, a->d_scales,
                                               a->d_rotations, stream);
    if (!rc) {
        if (warm && six)
            rc = dgs_gaussian_inputs_se3_backward(P, M_REST, a->xyz, rows, nout, a->scaling, a->rotation, a->opacity,
                                                  a->d_means3D, nullptr, a->d_scales, a->d_rotations, a->d_opacities,
                                                  a->g_xyz, nullptr, nullptr, a->g_scaling, a->g_rotation, a->g_opacity,
                                                  a->mlp_dout, stream);
        else
            rc = dgs_gaussian_inputs_backward(P, M_REST, a->scaling, a->rotation, a->opacity, a->d_means3D, nullptr,
                                              a->d_scales, a->d_rotations, a->d_opacities, a->g_xyz, nullptr, nullptr,
                                              a->g_scaling, a->g_rotation, a->g_opacity, warm ? a->mlp_dout : nullptr,
                                              warm ? nout : 10, stream);
    }
    if (!rc && warm && phase == 3) rc = dgs_deform_backward(flags, P, a->mlp_packed, a->mlp_saved, a->mlp_dout, a->mlp_scratch,
                                              a->mlp_grads, stream);
    // the whole step (phase 1: up to the Gaussian gradients) is queued: now the deferred pair count may
    // be resolved (a host wait at most)
    if (num_rendered) *num_rendered = nr >= 0 ? nr : dgs_raster_ctx_num_rendered(ctx);
    dgs_raster_ctx_free(ctx);
    dgs_raster_set_deferred_count(0);
    if (overflowed) *overflowed = dgs_raster_deferred_overflows() != over0;
    return rc;
}
