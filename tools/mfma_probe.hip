// Micro-benchmark: fp32 MFMA (v_mfma_f32_32x32x2_f32) issue rate for the MLP GEMM's inner-loop
// pattern on gfx950. Variants: pure MFMA chains; + two ds_read_b128 of B per 8 MFMAs (the k_mlp_*
// chunk); + a global A-fragment load per chunk. Prints TFLOP/s per variant and waves per SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

template <int MODE>
__global__ __launch_bounds__(512) void k_probe(const float4 *__restrict__ A, float *out, int iters) {
    __shared__ float4 lds[16 * 64 * 2];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 16 * 64 * 2; i += 512) lds[i] = make_float4(1e-3f * i, 1.f, 0.5f, 0.25f);
    __syncthreads();
    f32x16 acc0 = {}, acc1 = {};
    float4 a = make_float4(0.001f * lane, 0.002f, 0.003f, 0.004f);
    float4 b0 = lds[lane], b1 = lds[64 + lane];
    const float4 *Ap = A + lane;
    for (int it = 0; it < iters; it++) {
        if (MODE >= 1) {
            const int g = (it & 15) * 64;
            b0 = lds[g + lane];
            b1 = lds[g + 32 + ((lane + 1) & 31)];
        }
        if (MODE >= 2) a = Ap[(it & 31) * 64];
        acc0 = MFMA(a.x, b0.x, acc0);
        acc1 = MFMA(a.x, b1.x, acc1);
        acc0 = MFMA(a.y, b0.y, acc0);
        acc1 = MFMA(a.y, b1.y, acc1);
        acc0 = MFMA(a.z, b0.z, acc0);
        acc1 = MFMA(a.z, b1.z, acc1);
        acc0 = MFMA(a.w, b0.w, acc0);
        acc1 = MFMA(a.w, b1.w, acc1);
    }
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 16; r++) s += acc0[r] + acc1[r];
    if (s == 1234.5f) out[0] = s;
}

template <int MODE>
static void run(const char *name, int blocks_per_cu, int lds_extra, int threads = 512) {
    const int cus = 256, iters = 4096;
    float4 *A;
    float *out;
    hipMalloc(&A, 32 * 64 * sizeof(float4));
    hipMemset(A, 0, 32 * 64 * sizeof(float4));
    hipMalloc(&out, 4);
    const int blocks = cus * blocks_per_cu;
    hipLaunchKernelGGL(k_probe<MODE>, dim3(blocks), dim3(threads), lds_extra, 0, A, out, iters);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_probe<MODE>, dim3(blocks), dim3(threads), lds_extra, 0, A, out, iters);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 5.0 * blocks * (threads / 64.0) * iters * 8.0 /*mfma*/ * 32 * 32 * 2 * 2;
    printf("%-28s blocks/CU=%d waves/block=%d  %.1f TFLOP/s\n", name, blocks_per_cu, threads / 64,
           flop / (ms * 1e-3) / 1e12);
    hipFree(A);
    hipFree(out);
}

int main() {
    run<0>("mfma only", 1, 0);
    run<1>("mfma + 2 ds_read_b128", 1, 0);
    run<2>("mfma + ds_read + global A", 1, 0);
    run<0>("mfma only", 2, 0);
    run<1>("mfma + 2 ds_read_b128", 2, 0);
    run<2>("mfma + ds_read + global A", 2, 0);
    run<0>("mfma only", 1, 0, 256);
    run<1>("mfma + 2 ds_read_b128", 1, 0, 256);
    run<2>("mfma + ds_read + global A", 1, 0, 256);
    return 0;
}
