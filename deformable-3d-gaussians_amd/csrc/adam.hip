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

__global__ __launch_bounds__(THREADS) void k_adam(Jobs J) {
    const long long b = blockIdx.x;
    int q = 0;
    for (int k = 1; k < J.n; k++)  // uniform scan of the kernel-argument table
        if (b >= J.j[k].block0) q = k;
    const Job &T = J.j[q];
    const long long base = (b - T.block0) * BLOCK_ELEMS + threadIdx.x;
    const float c1 = J.omb1, c2 = J.omb2;
#pragma unroll
    for (int k = 0; k < PER_THREAD; k++) {
        const long long i = base + (long long)k * THREADS;
        if (i < T.n) {
            const float g = T.g[i];
            float m = T.m[i], v = T.v[i];
            m = m + c1 * (g - m);
            v = v * J.b2 + c2 * (g * g);
            const float denom = sqrtf(v) / T.bc2_sqrt + J.eps;
            T.p[i] = T.p[i] + (-T.step_size) * (m / denom);
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
        hipLaunchKernelGGL(adam::k_adam, dim3((unsigned)blocks), dim3(adam::THREADS), 0, stream, J);
        DGS_LAUNCH_CHECK("k_adam", false, stream);
    }
    return DGS_OK;
}
