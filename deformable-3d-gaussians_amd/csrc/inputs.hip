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
// The SH concatenation moves 16-byte units (coalesced vector stores / loads on the (P, C, 3) side);
// separate threads do the per-Gaussian activations.
#include <hip/hip_runtime.h>

#include "dgs_common.h"

namespace dgs {
namespace inputs {

constexpr float NORM_EPS = 1e-12f;  // torch.nn.functional.normalize default

// Threads [0, P * C * 3 / 4) move one 16-byte unit of the (P, C, 3) SH rows each (C * 3 is a
// multiple of 4 for C = 16 and C = 4 / 9 / 1 are handled by the scalar tail path); threads
// [Pu, Pu + P) do the per-Gaussian activations, consecutive Gaussians on consecutive lanes.
// the Gaussian of the first float of unit idx (32-bit division while the array fits in 2^31 floats)
__device__ inline long long unit_row(long long idx, int row, int P) {
    return (long long)P * row < 0x7fffffffll ? (long long)((uint32_t)(4 * idx) / (uint32_t)row) : (4 * idx) / row;
}

__device__ inline float sh_src(const float *f_dc, const float *f_rest, int C, long long p, int e) {
    return e < 3 ? f_dc[3 * p + e] : f_rest[(3ll * (C - 1)) * p + (e - 3)];
}

__global__ __launch_bounds__(256) void k_inputs_fwd(int P, int C, const float *__restrict__ xyz,
                                                    const float *__restrict__ f_dc, const float *__restrict__ f_rest,
                                                    const float *__restrict__ scaling, const float *__restrict__ rotation,
                                                    const float *__restrict__ opacity, const float *__restrict__ deform,
                                                    int ds, float *__restrict__ means3D, float *__restrict__ shs,
                                                    float *__restrict__ scales, float *__restrict__ rots,
                                                    float *__restrict__ opac) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int row = 3 * C;                          // floats per Gaussian
    const long long nu = ((long long)P * row + 3) / 4;  // 16-byte units of shs
    if (idx < nu) {
        float v[4];
        long long p = unit_row(idx, row, P);  // one division per unit, then carry into the next row
        int e = (int)(4 * idx - p * row);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            v[j] = p < P ? sh_src(f_dc, f_rest, C, p, e) : 0.f;
            if (++e == row) {
                e = 0;
                p++;
            }
        }
        if (4 * idx + 3 < (long long)P * row) {
            *reinterpret_cast<float4 *>(shs + 4 * idx) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (4 * idx + j < (long long)P * row) shs[4 * idx + j] = v[j];
        }
        return;
    }
    const long long p = idx - nu;
    if (p >= P) return;
    const float *d = deform ? deform + (long long)ds * p : nullptr;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        means3D[3 * p + j] = xyz[3 * p + j] + (d ? d[j] : 0.f);
        scales[3 * p + j] = expf(scaling[3 * p + j]) + (d ? d[7 + j] : 0.f);
    }
    const float4 q = *reinterpret_cast<const float4 *>(rotation + 4 * p);
    const float n = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), NORM_EPS);
    *reinterpret_cast<float4 *>(rots + 4 * p) = make_float4(q.x / n + (d ? d[3] : 0.f), q.y / n + (d ? d[4] : 0.f),
                                                           q.z / n + (d ? d[5] : 0.f), q.w / n + (d ? d[6] : 0.f));
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
    const int row = 3 * C;
    const long long nu = ((long long)P * row + 3) / 4;
    if (idx < nu) {  // one 16-byte unit of the (P, C, 3) SH gradient -> the dc / rest gradients
        float v[4];
        if (4 * idx + 3 < (long long)P * row) {
            const float4 g = *reinterpret_cast<const float4 *>(g_shs + 4 * idx);
            v[0] = g.x; v[1] = g.y; v[2] = g.z; v[3] = g.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = 4 * idx + j < (long long)P * row ? g_shs[4 * idx + j] : 0.f;
        }
        long long p = unit_row(idx, row, P);
        int e = (int)(4 * idx - p * row);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (p < P) {
                if (e < 3) {
                    if (o_dc) o_dc[3 * p + e] = v[j];
                } else if (o_rest) {
                    o_rest[(3ll * (C - 1)) * p + (e - 3)] = v[j];
                }
            }
            if (++e == row) {
                e = 0;
                p++;
            }
        }
        return;
    }
    const long long p = idx - nu;
    if (p >= P) return;
    float *dd = o_deform ? o_deform + (long long)ds * p : nullptr;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const float gm = g_means[3 * p + j], gs = g_scales[3 * p + j];
        if (o_xyz) o_xyz[3 * p + j] = gm;
        if (o_scaling) o_scaling[3 * p + j] = gs * expf(scaling[3 * p + j]);
        if (dd) {
            dd[j] = gm;
            dd[7 + j] = gs;
        }
    }
    const float4 g = *reinterpret_cast<const float4 *>(g_rots + 4 * p);
    if (dd) {
        dd[3] = g.x;
        dd[4] = g.y;
        dd[5] = g.z;
        dd[6] = g.w;
    }
    if (o_rotation) {
        const float4 q = *reinterpret_cast<const float4 *>(rotation + 4 * p);
        const float nn = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
        float4 r;
        if (nn > NORM_EPS) {  // d(q/|q|) = (g - y (y.g)) / |q|
            const float yx = q.x / nn, yy = q.y / nn, yz = q.z / nn, yw = q.w / nn;
            const float yg = yx * g.x + yy * g.y + yz * g.z + yw * g.w;
            r = make_float4((g.x - yx * yg) / nn, (g.y - yy * yg) / nn, (g.z - yz * yg) / nn, (g.w - yw * yg) / nn);
        } else {  // clamped norm: q / eps, the clamp passes no gradient
            r = make_float4(g.x / NORM_EPS, g.y / NORM_EPS, g.z / NORM_EPS, g.w / NORM_EPS);
        }
        *reinterpret_cast<float4 *>(o_rotation + 4 * p) = r;
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
    const long long n = ((long long)P * 3 * C + 3) / 4 + P;  // SH units + activation threads
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
    const long long n = ((long long)P * 3 * C + 3) / 4 + P;  // SH units + activation threads
    hipLaunchKernelGGL(inputs::k_inputs_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, P, C, scaling,
                       rotation, opacity, d_means3D, d_shs, d_scales, d_rotations, d_opacities, g_xyz, g_dc, g_rest,
                       g_scaling, g_rotation, g_opacity, g_deform, deform_stride);
    DGS_LAUNCH_CHECK("k_inputs_bwd", false, stream);
    return DGS_OK;
}
