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
// 6-DoF (is_6dof): the deformation row holds the raw screw head [w_r v_r] instead of d_xyz and the
// launch forms exp_se3 and applies it (means3D = R xyz + p), backward included; dgs_se3_* build the
// (P, 4, 4) d_xyz the reference's DeformNetwork returns, for callers outside render().
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

// ---- 6-DoF deformation (utils/time_utils.py:114-121, utils/rigid_utils.py:4-83) ----
// From the raw head outputs (w_r, v_r): theta = |w_r|; w = w_r / theta + 1e-5; v = v_r / theta + 1e-5
// (the add after the division is the reference's); W = skew(w), W2 = W W;
// R = I + sin(theta) W + (1 - cos(theta)) W2; p = (theta I + (1 - cos(theta)) W + (theta - sin(theta)) W2) v.
// render() applies [[R, p], [0, 0, 0, 1]] to [xyz; 1] and divides by the last row (== 1):
// means3D = R xyz + p (gaussian_renderer/__init__.py:71-76).
struct Se3 {
    float th, s, c;
    float w[3], v[3];
    float W[9], W2[9], R[9], A[9];
};

__device__ inline Se3 se3_build(const float *wr, const float *vr) {
    Se3 e;
    e.th = sqrtf(wr[0] * wr[0] + wr[1] * wr[1] + wr[2] * wr[2]);
#pragma unroll
    for (int i = 0; i < 3; i++) {
        e.w[i] = wr[i] / e.th + 1e-5f;
        e.v[i] = vr[i] / e.th + 1e-5f;
    }
    const float W[9] = {0.f, -e.w[2], e.w[1], e.w[2], 0.f, -e.w[0], -e.w[1], e.w[0], 0.f};
    sincosf(e.th, &e.s, &e.c);
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const float w2 = W[3 * i] * W[j] + W[3 * i + 1] * W[3 + j] + W[3 * i + 2] * W[6 + j];
            const float id = i == j ? 1.f : 0.f;
            e.W[3 * i + j] = W[3 * i + j];
            e.W2[3 * i + j] = w2;
            e.R[3 * i + j] = id + e.s * W[3 * i + j] + (1.f - e.c) * w2;
            e.A[3 * i + j] = e.th * id + (1.f - e.c) * W[3 * i + j] + (e.th - e.s) * w2;
        }
    return e;
}

// (R, p) of se3_build -> gradients of (w_r, v_r), given dL/dR (GR, row-major) and dL/dp (gp).
__device__ inline void se3_grad(const float *wr, const float *vr, const Se3 &e, const float *GR, const float *gp,
                                float *gw, float *gv) {
    float GA[9], G2[9], gvv[3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) GA[3 * i + j] = gp[i] * e.v[j];  // p = A v
#pragma unroll
    for (int j = 0; j < 3; j++) gvv[j] = e.A[j] * gp[0] + e.A[3 + j] * gp[1] + e.A[6 + j] * gp[2];
    float dRW = 0.f, dRW2 = 0.f, dAW = 0.f, dAW2 = 0.f;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        G2[k] = (1.f - e.c) * GR[k] + (e.th - e.s) * GA[k];  // dL/dW2
        dRW += GR[k] * e.W[k];
        dRW2 += GR[k] * e.W2[k];
        dAW += GA[k] * e.W[k];
        dAW2 += GA[k] * e.W2[k];
    }
    // dL/dW = s GR + (1 - c) GA + G2 W^T + W^T G2  (W2 = W W)
    float GW[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            float t = e.s * GR[3 * i + j] + (1.f - e.c) * GA[3 * i + j];
#pragma unroll
            for (int k = 0; k < 3; k++) t += G2[3 * i + k] * e.W[3 * j + k] + e.W[3 * k + i] * G2[3 * k + j];
            GW[3 * i + j] = t;
        }
    const float dw[3] = {GW[7] - GW[5], GW[2] - GW[6], GW[3] - GW[1]};  // skew(w) entries
    float dth = e.c * dRW + e.s * (dRW2 + dAW) + (GA[0] + GA[4] + GA[8]) + (1.f - e.c) * dAW2;
    // w = w_r / theta + 1e-5, v = v_r / theta + 1e-5
    const float ith = 1.f / e.th;
    dth -= (dw[0] * wr[0] + dw[1] * wr[1] + dw[2] * wr[2] + gvv[0] * vr[0] + gvv[1] * vr[1] + gvv[2] * vr[2]) *
           ith * ith;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        gw[i] = dw[i] * ith + dth * wr[i] * ith;  // theta = |w_r|
        gv[i] = gvv[i] * ith;
    }
}

// raw rows [w_r(3) v_r(3) ...] (stride ds) -> M (P, 4, 4) = [[R, p], [0, 0, 0, 1]] (rp_to_se3)
__global__ __launch_bounds__(256) void k_se3_fwd(int P, const float *__restrict__ raw, int ds, float *__restrict__ M) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const float *d = raw + (long long)ds * p;
    const float wr[3] = {d[0], d[1], d[2]}, vr[3] = {d[3], d[4], d[5]};
    const Se3 e = se3_build(wr, vr);
    float4 *m = reinterpret_cast<float4 *>(M + 16 * p);
    const float p0 = e.A[0] * e.v[0] + e.A[1] * e.v[1] + e.A[2] * e.v[2];
    const float p1 = e.A[3] * e.v[0] + e.A[4] * e.v[1] + e.A[5] * e.v[2];
    const float p2 = e.A[6] * e.v[0] + e.A[7] * e.v[1] + e.A[8] * e.v[2];
    m[0] = make_float4(e.R[0], e.R[1], e.R[2], p0);
    m[1] = make_float4(e.R[3], e.R[4], e.R[5], p1);
    m[2] = make_float4(e.R[6], e.R[7], e.R[8], p2);
    m[3] = make_float4(0.f, 0.f, 0.f, 1.f);
}

// dL/dM (P, 4, 4) -> dL/d(w_r, v_r) rows (stride gs); the constant last row passes no gradient
__global__ __launch_bounds__(256) void k_se3_bwd(int P, const float *__restrict__ raw, int ds,
                                                 const float *__restrict__ dM, float *__restrict__ g, int gs) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const float *d = raw + (long long)ds * p;
    const float wr[3] = {d[0], d[1], d[2]}, vr[3] = {d[3], d[4], d[5]};
    const Se3 e = se3_build(wr, vr);
    const float4 *m = reinterpret_cast<const float4 *>(dM + 16 * p);
    const float4 m0 = m[0], m1 = m[1], m2 = m[2];
    const float GR[9] = {m0.x, m0.y, m0.z, m1.x, m1.y, m1.z, m2.x, m2.y, m2.z};
    const float gp[3] = {m0.w, m1.w, m2.w};
    float gw[3], gv[3];
    se3_grad(wr, vr, e, GR, gp, gw, gv);
    float *o = g + (long long)gs * p;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        o[i] = gw[i];
        o[3 + i] = gv[i];
    }
}

// Deformation row layout: SE3 = false: [d_xyz(3) d_rotation(4) d_scaling(3)];
// SE3 = true (6-DoF head): [w_r(3) v_r(3) d_rotation(4) d_scaling(3)], means3D = R xyz + p.
template <bool SE3>
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
    constexpr int ROT = SE3 ? 6 : 3, SCL = SE3 ? 10 : 7;
    const float *d = deform ? deform + (long long)ds * p : nullptr;
    if constexpr (SE3) {  // deform != nullptr (checked by the entry point)
        const float wr[3] = {d[0], d[1], d[2]}, vr[3] = {d[3], d[4], d[5]};
        const Se3 e = se3_build(wr, vr);
        const float x[3] = {xyz[3 * p], xyz[3 * p + 1], xyz[3 * p + 2]};
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const float pp = e.A[3 * i] * e.v[0] + e.A[3 * i + 1] * e.v[1] + e.A[3 * i + 2] * e.v[2];
            means3D[3 * p + i] = e.R[3 * i] * x[0] + e.R[3 * i + 1] * x[1] + e.R[3 * i + 2] * x[2] + pp;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 3; j++) means3D[3 * p + j] = xyz[3 * p + j] + (d ? d[j] : 0.f);
    }
#pragma unroll
    for (int j = 0; j < 3; j++) scales[3 * p + j] = expf(scaling[3 * p + j]) + (d ? d[SCL + j] : 0.f);
    const float4 q = *reinterpret_cast<const float4 *>(rotation + 4 * p);
    const float n = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), NORM_EPS);
    *reinterpret_cast<float4 *>(rots + 4 * p) =
        make_float4(q.x / n + (d ? d[ROT] : 0.f), q.y / n + (d ? d[ROT + 1] : 0.f), q.z / n + (d ? d[ROT + 2] : 0.f),
                    q.w / n + (d ? d[ROT + 3] : 0.f));
    opac[p] = 1.f / (1.f + expf(-opacity[p]));
}

template <bool SE3>
__global__ __launch_bounds__(256) void k_inputs_bwd(int P, int C, const float *__restrict__ xyz,
                                                    const float *__restrict__ deform, int dsi,
                                                    const float *__restrict__ scaling,
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
    constexpr int ROT = SE3 ? 6 : 3, SCL = SE3 ? 10 : 7;
    float *dd = o_deform ? o_deform + (long long)ds * p : nullptr;
    const float gm[3] = {g_means[3 * p], g_means[3 * p + 1], g_means[3 * p + 2]};
    if constexpr (SE3) {  // means3D = R xyz + p: dL/dR = g xyz^T, dL/dp = g, dL/dxyz = R^T g
        const float *d = deform + (long long)dsi * p;
        const float wr[3] = {d[0], d[1], d[2]}, vr[3] = {d[3], d[4], d[5]};
        const Se3 e = se3_build(wr, vr);
        const float x[3] = {xyz[3 * p], xyz[3 * p + 1], xyz[3 * p + 2]};
        if (o_xyz) {
#pragma unroll
            for (int j = 0; j < 3; j++) o_xyz[3 * p + j] = e.R[j] * gm[0] + e.R[3 + j] * gm[1] + e.R[6 + j] * gm[2];
        }
        if (dd) {
            float GR[9], gw[3], gv[3];
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int j = 0; j < 3; j++) GR[3 * i + j] = gm[i] * x[j];
            se3_grad(wr, vr, e, GR, gm, gw, gv);
#pragma unroll
            for (int i = 0; i < 3; i++) {
                dd[i] = gw[i];
                dd[3 + i] = gv[i];
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < 3; j++) {
            if (o_xyz) o_xyz[3 * p + j] = gm[j];
            if (dd) dd[j] = gm[j];
        }
    }
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const float gs = g_scales[3 * p + j];
        if (o_scaling) o_scaling[3 * p + j] = gs * expf(scaling[3 * p + j]);
        if (dd) dd[SCL + j] = gs;
    }
    const float4 g = *reinterpret_cast<const float4 *>(g_rots + 4 * p);
    if (dd) {
        dd[ROT] = g.x;
        dd[ROT + 1] = g.y;
        dd[ROT + 2] = g.z;
        dd[ROT + 3] = g.w;
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

namespace {

template <bool SE3>
int inputs_forward(const char *name, int P, int M_rest, const float *xyz, const float *f_dc, const float *f_rest,
                   const float *scaling, const float *rotation, const float *opacity, const float *deform,
                   int deform_stride, float *means3D, float *shs, float *scales, float *rotations, float *opacities,
                   hipStream_t stream) {
    if (P < 0 || M_rest < 0 || (deform && deform_stride < (SE3 ? 13 : 10)) || (SE3 && !deform)) {
        set_error(std::string(name) + ": bad sizes");
        return DGS_ERR_ARGS;
    }
    if (P == 0) return DGS_OK;
    if (!xyz || (shs && (!f_dc || (M_rest > 0 && !f_rest))) || !scaling || !rotation || !opacity || !means3D ||
        !scales || !rotations || !opacities) {
        set_error(std::string(name) + ": null argument");
        return DGS_ERR_ARGS;
    }
    const int C = shs ? 1 + M_rest : 0;  // shs == NULL: no SH concatenation (split-SH rasterizer)
    const long long n = ((long long)P * 3 * C + 3) / 4 + P;  // SH units + activation threads
    ScopedTimer tm("inputs_fwd", stream);
    hipLaunchKernelGGL(inputs::k_inputs_fwd<SE3>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, P, C, xyz,
                       f_dc, f_rest, scaling, rotation, opacity, deform, deform_stride, means3D, shs, scales, rotations,
                       opacities);
    DGS_LAUNCH_CHECK("k_inputs_fwd", false, stream);
    return DGS_OK;
}

template <bool SE3>
int inputs_backward(const char *name, int P, int M_rest, const float *xyz, const float *deform, int deform_stride,
                    const float *scaling, const float *rotation, const float *opacity, const float *d_means3D,
                    const float *d_shs, const float *d_scales, const float *d_rotations, const float *d_opacities,
                    float *g_xyz, float *g_dc, float *g_rest, float *g_scaling, float *g_rotation, float *g_opacity,
                    float *g_deform, int g_stride, hipStream_t stream) {
    const int minw = SE3 ? 13 : 10;
    if (P < 0 || M_rest < 0 || (g_deform && g_stride < minw) || (SE3 && deform_stride < minw)) {
        set_error(std::string(name) + ": bad sizes");
        return DGS_ERR_ARGS;
    }
    if (P == 0) return DGS_OK;
    if (!scaling || !rotation || !opacity || !d_means3D || !d_scales || !d_rotations || !d_opacities ||
        (SE3 && (!xyz || !deform))) {
        set_error(std::string(name) + ": null argument");
        return DGS_ERR_ARGS;
    }
    const int C = d_shs ? 1 + M_rest : 0;  // d_shs == NULL: the SH gradients are written elsewhere
    const long long n = ((long long)P * 3 * C + 3) / 4 + P;  // SH units + activation threads
    ScopedTimer tm("inputs_bwd", stream);
    hipLaunchKernelGGL(inputs::k_inputs_bwd<SE3>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, P, C, xyz,
                       deform, deform_stride, scaling, rotation, opacity, d_means3D, d_shs, d_scales, d_rotations,
                       d_opacities, g_xyz, g_dc, g_rest, g_scaling, g_rotation, g_opacity, g_deform, g_stride);
    DGS_LAUNCH_CHECK("k_inputs_bwd", false, stream);
    return DGS_OK;
}

}  // namespace

extern "C" int dgs_gaussian_inputs_forward(int P, int M_rest, const float *xyz, const float *f_dc, const float *f_rest,
                                           const float *scaling, const float *rotation, const float *opacity,
                                           const float *deform, int deform_stride, float *means3D, float *shs,
                                           float *scales, float *rotations, float *opacities, void *stream) {
    return inputs_forward<false>("dgs_gaussian_inputs_forward", P, M_rest, xyz, f_dc, f_rest, scaling, rotation,
                                 opacity, deform, deform_stride, means3D, shs, scales, rotations, opacities,
                                 (hipStream_t)stream);
}

extern "C" int dgs_gaussian_inputs_backward(int P, int M_rest, const float *scaling, const float *rotation,
                                            const float *opacity, const float *d_means3D, const float *d_shs,
                                            const float *d_scales, const float *d_rotations, const float *d_opacities,
                                            float *g_xyz, float *g_dc, float *g_rest, float *g_scaling,
                                            float *g_rotation, float *g_opacity, float *g_deform, int deform_stride,
                                            void *stream) {
    return inputs_backward<false>("dgs_gaussian_inputs_backward", P, M_rest, nullptr, nullptr, 0, scaling, rotation,
                                  opacity, d_means3D, d_shs, d_scales, d_rotations, d_opacities, g_xyz, g_dc, g_rest,
                                  g_scaling, g_rotation, g_opacity, g_deform, deform_stride, (hipStream_t)stream);
}

extern "C" int dgs_gaussian_inputs_se3_forward(int P, int M_rest, const float *xyz, const float *f_dc,
                                               const float *f_rest, const float *scaling, const float *rotation,
                                               const float *opacity, const float *deform, int deform_stride,
                                               float *means3D, float *shs, float *scales, float *rotations,
                                               float *opacities, void *stream) {
    return inputs_forward<true>("dgs_gaussian_inputs_se3_forward", P, M_rest, xyz, f_dc, f_rest, scaling, rotation,
                                opacity, deform, deform_stride, means3D, shs, scales, rotations, opacities,
                                (hipStream_t)stream);
}

extern "C" int dgs_gaussian_inputs_se3_backward(int P, int M_rest, const float *xyz, const float *deform,
                                                int deform_stride, const float *scaling, const float *rotation,
                                                const float *opacity, const float *d_means3D, const float *d_shs,
                                                const float *d_scales, const float *d_rotations,
                                                const float *d_opacities, float *g_xyz, float *g_dc, float *g_rest,
                                                float *g_scaling, float *g_rotation, float *g_opacity, float *g_deform,
                                                void *stream) {
    return inputs_backward<true>("dgs_gaussian_inputs_se3_backward", P, M_rest, xyz, deform, deform_stride, scaling,
                                 rotation, opacity, d_means3D, d_shs, d_scales, d_rotations, d_opacities, g_xyz, g_dc,
                                 g_rest, g_scaling, g_rotation, g_opacity, g_deform, deform_stride,
                                 (hipStream_t)stream);
}

extern "C" int dgs_se3_forward(int P, const float *raw, int raw_stride, float *M, void *stream) {
    if (P < 0 || raw_stride < 6) {
        set_error("dgs_se3_forward: bad sizes");
        return DGS_ERR_ARGS;
    }
    if (P == 0) return DGS_OK;
    if (!raw || !M) {
        set_error("dgs_se3_forward: null argument");
        return DGS_ERR_ARGS;
    }
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(inputs::k_se3_fwd, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P, raw, raw_stride, M);
    DGS_LAUNCH_CHECK("k_se3_fwd", false, s);
    return DGS_OK;
}

extern "C" int dgs_se3_backward(int P, const float *raw, int raw_stride, const float *dM, float *g_raw, int g_stride,
                                void *stream) {
    if (P < 0 || raw_stride < 6 || g_stride < 6) {
        set_error("dgs_se3_backward: bad sizes");
        return DGS_ERR_ARGS;
    }
    if (P == 0) return DGS_OK;
    if (!raw || !dM || !g_raw) {
        set_error("dgs_se3_backward: null argument");
        return DGS_ERR_ARGS;
    }
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(inputs::k_se3_bwd, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P, raw, raw_stride, dM,
                       g_raw, g_stride);
    DGS_LAUNCH_CHECK("k_se3_bwd", false, s);
    return DGS_OK;
}
