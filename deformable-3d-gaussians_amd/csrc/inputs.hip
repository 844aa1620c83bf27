// Rasterizer inputs of render() in one launch each way.
//
// Forward (gaussian_renderer/__init__.py:70-112 with the activations of scene/gaussian_model.py:39-50):
//   means3D   = xyz + d_xyz
//   scales    = exp(scaling) + d_scaling
//   rotations = normalize(rotation) + d_rotation        (no re-normalisation, as upstream)
//   opacities = sigmoid(opacity)
//   shs       = cat(features_dc, features_rest, dim=1)
// Backward: the gradients of the five rasterizer inputs mapped back to the six Gaussian tensors and
// written straight into the (P, 10) deformation-output gradient (columns 0 / 3 / 7), replacing ~25
// small torch kernels (add/exp/norm/div/sigmoid/cat and their backward, slice-backward assembly).
// One thread per (Gaussian, SH coefficient): the coefficient copies are coalesced 12-byte rows;
// coefficient 0's thread also does the per-Gaussian activations.
#include <hip/hip_runtime.h>

#include "dgs_common.h"

namespace dgs {
namespace inputs {

constexpr float NORM_EPS = 1e-12f;  // torch.nn.functional.normalize default

__global__ __launch_bounds__(256) void k_inputs_fwd(int P, int C, const float *__restrict__ xyz,
                                                    const float *__restrict__ f_dc, const float *__restrict__ f_rest,
                                                    const float *__restrict__ scaling, const float *__restrict__ rotation,
                                                    const float *__restrict__ opacity, const float *__restrict__ deform,
                                                    int ds, float *__restrict__ means3D, float *__restrict__ shs,
                                                    float *__restrict__ scales, float *__restrict__ rots,
                                                    float *__restrict__ opac) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)P * C) return;
    const int p = (int)(idx / C), k = (int)(idx - (long long)p * C);
    const float *src = k == 0 ? f_dc + 3ll * p : f_rest + (3ll * (C - 1)) * p + 3 * (k - 1);
    float *dst = shs + 3 * idx;
    dst[0] = src[0];
    dst[1] = src[1];
    dst[2] = src[2];
    if (k != 0) return;
    const float *d = deform ? deform + (long long)ds * p : nullptr;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        means3D[3ll * p + j] = xyz[3ll * p + j] + (d ? d[j] : 0.f);
        scales[3ll * p + j] = expf(scaling[3ll * p + j]) + (d ? d[7 + j] : 0.f);
    }
    const float4 q = *reinterpret_cast<const float4 *>(rotation + 4ll * p);
    const float n = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), NORM_EPS);
    rots[4ll * p + 0] = q.x / n + (d ? d[3] : 0.f);
    rots[4ll * p + 1] = q.y / n + (d ? d[4] : 0.f);
    rots[4ll * p + 2] = q.z / n + (d ? d[5] : 0.f);
    rots[4ll * p + 3] = q.w / n + (d ? d[6] : 0.f);
    opac[p] = 1.f / (1.f + expf(-opacity[p]));
}

__global__ __launch_bounds__(256) void k_inputs_bwd(int P, int C, const float *__restrict__ scaling,
                                                    const float *__restrict__ rotation, const float *__restrict__ opacity,
                                                    const float *__restrict__ g_means, const float *__restrict__ g_shs,
                                                    const float *__restrict__ g_scales, const float *__restrict__ g_rots,
                                                    const float *__restrict__ g_opac, float *__restrict__ o_xyz,
                                                    float *__restrict__ o_dc, float *__restrict__ o_rest,
                                                    float *__restrict__ o_scaling, float *__restrict__ o_rotation,
                                                    float *__restrict__ o_opacity, float *__restrict__ o_deform, int ds) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)P * C) return;
    const int p = (int)(idx / C), k = (int)(idx - (long long)p * C);
    float *dst = k == 0 ? o_dc : o_rest;
    if (dst) {
        dst += k == 0 ? 3ll * p : (3ll * (C - 1)) * p + 3 * (k - 1);
        const float *src = g_shs + 3 * idx;
        dst[0] = src[0];
        dst[1] = src[1];
        dst[2] = src[2];
    }
    if (k != 0) return;
    float *dd = o_deform ? o_deform + (long long)ds * p : nullptr;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const float gm = g_means[3ll * p + j], gs = g_scales[3ll * p + j];
        if (o_xyz) o_xyz[3ll * p + j] = gm;
        if (o_scaling) o_scaling[3ll * p + j] = gs * expf(scaling[3ll * p + j]);
        if (dd) {
            dd[j] = gm;
            dd[7 + j] = gs;
        }
    }
    const float4 g = *reinterpret_cast<const float4 *>(g_rots + 4ll * p);
    if (dd) {
        dd[3] = g.x;
        dd[4] = g.y;
        dd[5] = g.z;
        dd[6] = g.w;
    }
    if (o_rotation) {
        const float4 q = *reinterpret_cast<const float4 *>(rotation + 4ll * p);
        const float nn = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
        float4 r;
        if (nn > NORM_EPS) {  // d(q/|q|) = (g - y (y.g)) / |q|
            const float yx = q.x / nn, yy = q.y / nn, yz = q.z / nn, yw = q.w / nn;
            const float yg = yx * g.x + yy * g.y + yz * g.z + yw * g.w;
            r = make_float4((g.x - yx * yg) / nn, (g.y - yy * yg) / nn, (g.z - yz * yg) / nn, (g.w - yw * yg) / nn);
        } else {  // clamped norm: q / eps, the clamp passes no gradient
            r = make_float4(g.x / NORM_EPS, g.y / NORM_EPS, g.z / NORM_EPS, g.w / NORM_EPS);
        }
        *reinterpret_cast<float4 *>(o_rotation + 4ll * p) = r;
    }
    if (o_opacity) {
        const float s = 1.f / (1.f + expf(-opacity[p]));
        o_opacity[p] = g_opac[p] * (1.f - s) * s;
    }
}

}  // namespace inputs
}  // namespace dgs

using namespace dgs;

extern "C" int dgs_gaussian_inputs_forward(int P, int M_rest, const float *xyz, const float *f_dc, const float *f_rest,
                                           const float *scaling, const float *rotation, const float *opacity,
                                           const float *deform, int deform_stride, float *means3D, float *shs,
                                           float *scales, float *rotations, float *opacities, void *stream_) {
    if (P < 0 || M_rest < 0 || (deform && deform_stride < 10)) {
        set_error("dgs_gaussian_inputs_forward: bad sizes");
        return DGS_ERR_ARGS;
    }
    if (P == 0) return DGS_OK;
    if (!xyz || !f_dc || (M_rest > 0 && !f_rest) || !scaling || !rotation || !opacity || !means3D || !shs || !scales ||
        !rotations || !opacities) {
        set_error("dgs_gaussian_inputs_forward: null argument");
        return DGS_ERR_ARGS;
    }
    hipStream_t stream = (hipStream_t)stream_;
    const int C = 1 + M_rest;
    const long long n = (long long)P * C;
    hipLaunchKernelGGL(inputs::k_inputs_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, P, C, xyz, f_dc,
                       f_rest, scaling, rotation, opacity, deform, deform_stride, means3D, shs, scales, rotations,
                       opacities);
    DGS_LAUNCH_CHECK("k_inputs_fwd", false, stream);
    return DGS_OK;
}

extern "C" int dgs_gaussian_inputs_backward(int P, int M_rest, const float *scaling, const float *rotation,
                                            const float *opacity, const float *d_means3D, const float *d_shs,
                                            const float *d_scales, const float *d_rotations, const float *d_opacities,
                                            float *g_xyz, float *g_dc, float *g_rest, float *g_scaling,
                                            float *g_rotation, float *g_opacity, float *g_deform, int deform_stride,
                                            void *stream_) {
    if (P < 0 || M_rest < 0 || (g_deform && deform_stride < 10)) {
        set_error("dgs_gaussian_inputs_backward: bad sizes");
        return DGS_ERR_ARGS;
    }
    if (P == 0) return DGS_OK;
    if (!scaling || !rotation || !opacity || !d_means3D || !d_shs || !d_scales || !d_rotations || !d_opacities) {
        set_error("dgs_gaussian_inputs_backward: null argument");
        return DGS_ERR_ARGS;
    }
    hipStream_t stream = (hipStream_t)stream_;
    const int C = 1 + M_rest;
    const long long n = (long long)P * C;
    hipLaunchKernelGGL(inputs::k_inputs_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, P, C, scaling,
                       rotation, opacity, d_means3D, d_shs, d_scales, d_rotations, d_opacities, g_xyz, g_dc, g_rest,
                       g_scaling, g_rotation, g_opacity, g_deform, deform_stride);
    DGS_LAUNCH_CHECK("k_inputs_bwd", false, stream);
    return DGS_OK;
}
