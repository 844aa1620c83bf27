// Multi-tensor Adam: every parameter of an optimizer (or of several) updated by ONE launch.
//
// Replaces torch.optim.Adam(..., eps=1e-15).step() of scene/gaussian_model.py:136 and
// scene/deform_model.py:332 (train_baseline.py:176-182). torch's multi_tensor_apply gives a
// 100k x 3 tensor five workgroups (65536-element chunks), so each of the 7 groups of a step took
// ~42 us of latency-bound time; here every tensor is cut into 2048-element blocks and the whole
// step is one HBM-bound grid (28 B per element: p, g, m, v read; p, m, v written).
//
// Update (torch.optim.Adam single-tensor/foreach rule, amsgrad and weight decay off):
//   m = m + (1 - b1) (g - m)                    (lerp, weight < 0.5 branch)
//   v = b2 v + (1 - b2) g g
//   p = p - step_size * m / (sqrt(v) / bc2_sqrt + eps)
#include <hip/hip_runtime.h>

#include "dgs_common.h"

namespace dgs {
namespace adam {

constexpr int THREADS = 256;
constexpr int PER_THREAD = 8;
constexpr int BLOCK_ELEMS = THREADS * PER_THREAD;
constexpr int MAXT = 40;

struct Job {
    float *p;
    const float *g;
    float *m;
    float *v;
    long long n;
    long long block0;
    float step_size, bc2_sqrt;
};
struct Jobs {
    Job j[MAXT];
    int n;
    float omb1, b2, omb2, eps;  // 1 - beta1, beta2, 1 - beta2 (differences taken in double, as torch)
};

__device__ __forceinline__ void adam1(float &p, float g, float &m, float &v, float c1, float b2, float c2, float eps,
                                      float step_size, float bc2_sqrt) {
    m = m + c1 * (g - m);
    v = v * b2 + c2 * (g * g);
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p + (-step_size) * (m / denom);
}

// Each thread updates PER_THREAD / 4 float4 units (16-byte loads and stores of p, g, m, v) when the
// tensor's four pointers are 16-byte aligned; otherwise (or for a ragged tail) element by element.
// Same arithmetic per element either way.
__global__ __launch_bounds__(THREADS) void k_adam(Jobs J) {
    const long long b = blockIdx.x;
    int q = 0;
    for (int k = 1; k < J.n; k++)  // uniform scan of the kernel-argument table
        if (b >= J.j[k].block0) q = k;
    const Job &T = J.j[q];
    const float c1 = J.omb1, c2 = J.omb2, b2 = J.b2, eps = J.eps, ss = T.step_size, bc = T.bc2_sqrt;
    const bool vec = ((reinterpret_cast<uintptr_t>(T.p) | reinterpret_cast<uintptr_t>(T.g) |
                       reinterpret_cast<uintptr_t>(T.m) | reinterpret_cast<uintptr_t>(T.v)) & 15) == 0;
    const long long e0 = (b - T.block0) * BLOCK_ELEMS;
    if (vec && e0 + BLOCK_ELEMS <= T.n) {
        constexpr int U = PER_THREAD / 4;
        float4 p[U], g[U], m[U], v[U];
        // every load of the thread first (the stores could alias other tensors' loads for the
        // compiler), then the updates, then the stores
#pragma unroll
        for (int k = 0; k < U; k++) {
            const long long i = e0 + 4ll * (threadIdx.x + k * THREADS);
            p[k] = *reinterpret_cast<const float4 *>(T.p + i);
            g[k] = *reinterpret_cast<const float4 *>(T.g + i);
            m[k] = *reinterpret_cast<const float4 *>(T.m + i);
            v[k] = *reinterpret_cast<const float4 *>(T.v + i);
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            adam1(p[k].x, g[k].x, m[k].x, v[k].x, c1, b2, c2, eps, ss, bc);
            adam1(p[k].y, g[k].y, m[k].y, v[k].y, c1, b2, c2, eps, ss, bc);
            adam1(p[k].z, g[k].z, m[k].z, v[k].z, c1, b2, c2, eps, ss, bc);
            adam1(p[k].w, g[k].w, m[k].w, v[k].w, c1, b2, c2, eps, ss, bc);
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const long long i = e0 + 4ll * (threadIdx.x + k * THREADS);
            *reinterpret_cast<float4 *>(T.p + i) = p[k];
            *reinterpret_cast<float4 *>(T.m + i) = m[k];
            *reinterpret_cast<float4 *>(T.v + i) = v[k];
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < PER_THREAD; k++) {
        const long long i = e0 + threadIdx.x + (long long)k * THREADS;
        if (i < T.n) {
            float p = T.p[i], m = T.m[i], v = T.v[i];
            adam1(p, T.g[i], m, v, c1, b2, c2, eps, ss, bc);
            T.p[i] = p;
            T.m[i] = m;
            T.v[i] = v;
        }
    }
}

}  // namespace adam
}  // namespace dgs

using namespace dgs;

extern "C" int dgs_adam_step(int n, const dgs_adam_tensor *t, double beta1, double beta2, double eps, void *stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    if (n < 0 || (n > 0 && !t)) {
        set_error("dgs_adam_step: bad tensor list");
        return DGS_ERR_ARGS;
    }
    int k = 0;
    while (k < n) {
        adam::Jobs J{};
        J.omb1 = (float)(1.0 - beta1);
        J.b2 = (float)beta2;
        J.omb2 = (float)(1.0 - beta2);
        J.eps = (float)eps;
        long long blocks = 0;
        for (; k < n && J.n < adam::MAXT; k++) {
            const dgs_adam_tensor &d = t[k];
            if (d.numel <= 0) continue;
            if (!d.param || !d.grad || !d.exp_avg || !d.exp_avg_sq) {
                set_error("dgs_adam_step: null tensor pointer");
                return DGS_ERR_ARGS;
            }
            adam::Job &j = J.j[J.n++];
            j.p = d.param; j.g = d.grad; j.m = d.exp_avg; j.v = d.exp_avg_sq;
            j.n = d.numel; j.block0 = blocks;
            j.step_size = d.step_size; j.bc2_sqrt = d.bc2_sqrt;
            blocks += (d.numel + adam::BLOCK_ELEMS - 1) / adam::BLOCK_ELEMS;
        }
        if (J.n == 0) continue;
        if (blocks > 0x7fffffffLL) {
            set_error("dgs_adam_step: tensor list too large for one grid");
            return DGS_ERR_ARGS;
        }
        ScopedTimer tm("adam", stream);
        hipLaunchKernelGGL(adam::k_adam, dim3((unsigned)blocks), dim3(adam::THREADS), 0, stream, J);
        DGS_LAUNCH_CHECK("k_adam", false, stream);
    }
    return DGS_OK;
}
