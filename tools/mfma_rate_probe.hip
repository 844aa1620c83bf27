// MFMA issue-rate probe for the split-bf16 MLP k-step shape: 512-thread workgroups (2 waves/SIMD),
// one per CU, each wave running NK k-steps of 12 v_mfma_f32_32x32x16_bf16 (2 accumulators x 6),
// with (mode 0) operands in registers, (1) + 6 ds_read_b128 B reloads per k-step, (2) + 3 global
// A loads per k-step from a 3 MiB L2-resident image (4-deep ring), (3) = 2 with 16 waves/workgroup.
// Prints cycles per k-step per SIMD (ideal 2 x 12 x 32 = 768 with 2 waves/SIMD).
// hipcc --offload-arch=gfx950 -O3 tools/mfma_rate_probe.hip -o tools/mfma_rate_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
#define MF(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)
struct F3 { bf16x8 h, m, l; };
__device__ inline void six(const F3 &a, const F3 &b, f32x16 &c) {
    c = MF(a.m, b.m, c); c = MF(a.h, b.l, c); c = MF(a.l, b.h, c); c = MF(a.h, b.m, c); c = MF(a.m, b.h, c); c = MF(a.h, b.h, c);
}
template <int MODE>
__global__ __launch_bounds__(1024) void k(const bf16x8 *img, float *out, unsigned long long *cyc, int NK) {
    __shared__ bf16x8 lds[46 * 192];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 46 * 192; i += blockDim.x) lds[i] = img[i];
    __syncthreads();
    f32x16 acc[2] = {};
    F3 a = {img[lane], img[lane + 64], img[lane + 128]};
    F3 b[2];
    const bf16x8 *Bp = lds + (lane >> 5) * 192 + (lane & 31);
    for (int ct = 0; ct < 2; ct++) b[ct] = F3{Bp[32 * ct], Bp[64 + 32 * ct], Bp[128 + 32 * ct]};
    const bf16x8 *Ap = img + (size_t)(blockIdx.x % 8) * 8 * 1024 * 192 / 8 + wave * 16 * 192 + lane;
    F3 ring[4];
    for (int r = 0; r < 4; r++) ring[r] = F3{Ap[r * 192], Ap[r * 192 + 64], Ap[r * 192 + 128]};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < NK; it += 4) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const F3 &aa = MODE >= 2 ? ring[k] : a;
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int ct = 0; ct < 2; ct++) {
                six(aa, b[ct], acc[ct]);
                if (MODE >= 1) {
                    const bf16x8 *p = Bp + ((it + k + 1) % 22) * 384;
                    b[ct] = F3{p[32 * ct], p[64 + 32 * ct], p[128 + 32 * ct]};
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            if (MODE >= 2) {
                const bf16x8 *p = Ap + ((it + k + 4) % 512) * 192;
                ring[k] = F3{p[0], p[64], p[128]};
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int i = 0; i < 16; i++) s += acc[0][i] + acc[1][i];
    out[blockIdx.x * blockDim.x + tid] = s;
    if (lane == 0) cyc[blockIdx.x * 16 + wave] = t1 - t0;
}

int main() {
    const int CUs = 256, NK = 1024;
    const size_t nimg = (size_t)8 * 1024 * 192 + 46 * 192 + 4096;  // 8 x 3 MiB images (one per XCD group)
    std::vector<__bf16> h(nimg * 8);
    for (size_t i = 0; i < h.size(); i++) h[i] = (__bf16)(((i * 2654435761u) >> 16 & 1023) / 1024.f - 0.5f);
    bf16x8 *img; float *out; unsigned long long *cyc;
    hipMalloc(&img, nimg * 16); hipMalloc(&out, CUs * 1024 * 4); hipMalloc(&cyc, CUs * 16 * 8);
    hipMemcpy(img, h.data(), nimg * 16, hipMemcpyHostToDevice);
    auto run = [&](auto kern, int threads, const char *name) {
        for (int rep = 0; rep < 2; rep++) {
            hipLaunchKernelGGL(kern, dim3(CUs), dim3(threads), 0, 0, img, out, cyc, NK);
            hipDeviceSynchronize();
        }
        std::vector<unsigned long long> c(CUs * 16);
        hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
        double s = 0; int n = 0;
        for (int b = 0; b < CUs; b++) for (int w = 0; w < threads / 64; w++) { s += c[b * 16 + w]; n++; }
        const double per_ks = s / n / NK;  // cycles per k-step per wave
        const double waves_per_simd = threads / 64 / 4.0;
        printf("%-44s %.0f cycles per wave k-step; %.0f per SIMD k-step-slot (ideal %d) -> MFMA busy %.0f%%\n", name, per_ks,
               per_ks / waves_per_simd, 384, 100.0 * 384 * waves_per_simd / per_ks);
    };
    run(k<0>, 512, "regs only, 2 waves/SIMD");
    run(k<1>, 512, "+ LDS B reloads, 2 waves/SIMD");
    run(k<2>, 512, "+ L2 A ring, 2 waves/SIMD");
    run(k<2>, 1024, "+ L2 A ring, 4 waves/SIMD");
    return 0;
}
