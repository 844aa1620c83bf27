// Accuracy of long-K dot products (K = 4096) on MFMA, vs float64:
//  (a) split-bf16, 6 products per k-step accumulated into one running C
//  (b) split-bf16, each k-step's 6 products into a fresh T (C = 0), then acc += T (fp32 VALU, RNE)
//  (c) split-bf16 as (b) but flushing every 4 k-steps
//  (d) fp32-input MFMA (v_mfma_f32_32x32x2_f32, exact fma chain)
// One wave, 32x32 output, A (32 x K) signed normal, B (K x 32) = relu(normal) (activations).
// hipcc --offload-arch=gfx950 -O2 tools/mfma_accum_probe.hip -o tools/mfma_accum_probe.bin
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
#define MF(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

struct S3 { bf16x8 h, m, l; };
__device__ S3 split8(const float *x) {
    S3 s;
    for (int j = 0; j < 8; j++) {
        __bf16 hb = (__bf16)x[j]; float r = x[j] - (float)hb; __bf16 mb = (__bf16)r;
        s.h[j] = hb; s.m[j] = mb; s.l[j] = (__bf16)(r - (float)mb);
    }
    return s;
}
__device__ void six(const S3 &a, const S3 &b, f32x16 &c) {
    c = MF(a.m, b.m, c); c = MF(a.h, b.l, c); c = MF(a.l, b.h, c); c = MF(a.h, b.m, c); c = MF(a.m, b.h, c); c = MF(a.h, b.h, c);
}
// A: [32][K] row-major, B: [K][32] row-major; out: 4 x [32][32]
__global__ void k(const float *A, const float *B, int K, float *out) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    f32x16 ca = {}, cb = {}, cc = {}, cd = {}, tc = {};
    for (int s = 0; s < K / 16; s++) {
        float av[8], bv[8];
        for (int j = 0; j < 8; j++) { av[j] = A[r * K + 16 * s + 8 * h + j]; bv[j] = B[(16 * s + 8 * h + j) * 32 + r]; }
        const S3 a = split8(av), b = split8(bv);
        six(a, b, ca);
        f32x16 t = {};
        six(a, b, t);
        for (int i = 0; i < 16; i++) cb[i] += t[i];
        six(a, b, tc);
        if ((s & 3) == 3) { for (int i = 0; i < 16; i++) { cc[i] += tc[i]; tc[i] = 0.f; } }
        for (int kk = 0; kk < 16; kk += 2) {  // f32 32x32x2: lane holds A[r][k0 + h], B[k0 + h][r]
            const float a1 = A[r * K + 16 * s + kk + h], b1 = B[(16 * s + kk + h) * 32 + r];
            cd = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, cd, 0, 0, 0);
        }
    }
    for (int i = 0; i < 16; i++) {
        const int row = 8 * (i >> 2) + 4 * h + (i & 3);
        out[0 * 1024 + row * 32 + r] = ca[i];
        out[1 * 1024 + row * 32 + r] = cb[i];
        out[2 * 1024 + row * 32 + r] = cc[i];
        out[3 * 1024 + row * 32 + r] = cd[i];
    }
}

int main() {
    const int K = 4096;
    std::mt19937 g(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<float> A(32 * K), B(K * 32), o(4096);
    for (auto &v : A) v = 0.01f * nd(g);
    for (auto &v : B) v = std::max(0.f, nd(g));
    float *dA, *dB, *dO;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dO, o.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, K, dO);
    hipMemcpy(o.data(), dO, o.size() * 4, hipMemcpyDeviceToHost);
    const char *nm[4] = {"split, one running C", "split, fresh T per k-step + fp32 add", "split, T flushed every 4 k-steps", "fp32 MFMA (fma chain)"};
    for (int m = 0; m < 4; m++) {
        double maxe = 0, maxrel = 0, sum_e = 0, scale = 0;
        for (int i = 0; i < 32; i++)
            for (int j = 0; j < 32; j++) {
                double ex = 0, ab = 0;
                for (int kk = 0; kk < K; kk++) { ex += (double)A[i * K + kk] * B[kk * 32 + j]; ab += fabs((double)A[i * K + kk] * B[kk * 32 + j]); }
                const double e = o[m * 1024 + i * 32 + j] - ex;
                maxe = fmax(maxe, fabs(e)); sum_e += e; scale = fmax(scale, fabs(ex));
                maxrel = fmax(maxrel, fabs(e) / ab);
            }
        printf("%-40s max|err| %.3e (%.2e of max|ref|)  max err/sum|terms| %.3e  mean err %.3e\n", nm[m], maxe, maxe / scale, maxrel, sum_e / 1024);
    }
    return 0;
}
