// Diagnostic: per-phase cycle split of k_mlp_fwd (built with -DDGS_MLP_PROFILE, which compiles
// s_memtime stamps into the kernel; the product library never has them).
// Build: hipcc -O3 --offload-arch=gfx950 -DDGS_MLP_PROFILE -munsafe-fp-atomics -I include \
//        tools/mlp_phase.cpp deformable-3d-gaussians_amd/csrc/mlp.hip deformable-3d-gaussians_amd/csrc/api.hip \
//        -o tools/mlp_phase.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "dgs.h"

extern "C" void dgs_mlp_set_prof(unsigned long long *p);

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 100000;
    const int flags = DGS_MLP_BLENDER;
    const size_t npk = dgs_deform_packed_floats(flags);
    const size_t nsv = dgs_deform_saved_floats(flags, N);
    std::vector<float> h(npk);
    for (size_t i = 0; i < npk; i++) h[i] = ((float)rand() / RAND_MAX - 0.5f) * 0.1f;
    std::vector<float> hx(3 * (size_t)N), ht(N);
    for (auto &v : hx) v = (float)rand() / RAND_MAX * 2.f - 1.f;
    for (auto &v : ht) v = (float)rand() / RAND_MAX;
    float *pk, *x, *t, *out, *saved;
    hipMalloc(&pk, npk * 4);
    hipMalloc(&x, hx.size() * 4);
    hipMalloc(&t, ht.size() * 4);
    hipMalloc(&out, (size_t)N * 16 * 4);
    hipMalloc(&saved, nsv * 4);
    hipMemcpy(pk, h.data(), npk * 4, hipMemcpyHostToDevice);
    hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(t, ht.data(), ht.size() * 4, hipMemcpyHostToDevice);
    const int blocks = (N + 31) / 32;  // BM = 32
    unsigned long long *prof;
    hipMalloc(&prof, (size_t)blocks * 256 * 8);
    hipMemset(prof, 0, (size_t)blocks * 256 * 8);
    dgs_mlp_set_prof(prof);
    for (int w = 0; w < 3; w++) dgs_deform_forward(flags, N, x, t, pk, out, saved, nullptr);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    const int reps = 5;
    for (int r = 0; r < reps; r++) dgs_deform_forward(flags, N, x, t, pk, out, saved, nullptr);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> hp((size_t)blocks * 256);
    hipMemcpy(hp.data(), prof, hp.size() * 8, hipMemcpyDeviceToHost);
    printf("k_mlp_fwd N=%d: %.3f ms/launch (%s)\n", N, ms / reps, dgs_last_error());
    const char *names[30] = {"PE", "T1", "T2", 0};
    double sum[30] = {0};
    double total = 0;
    for (int b = 0; b < blocks; b++) {
        const unsigned long long *s = &hp[(size_t)b * 256];
        for (int k = 1; k < 30; k++) sum[k] += (double)(s[k] - s[k - 1]);
        total += (double)(s[29] - s[0]);
    }
    printf("mean cycles per block: %.0f\n", total / blocks);
    {
        double rt = 0, ck = 0;
        for (int b = 0; b < blocks; b++) {
            const unsigned long long *s = &hp[(size_t)b * 256];
            rt += (double)(s[254] - s[252]);
            ck += (double)(s[255] - s[253]);
        }
        printf("s_memtime rate: %.3f GHz (vs 100 MHz s_memrealtime)\n", 0.1 * ck / rt);
    }
    for (int k = 1; k < 30; k++) {
        char buf[32];
        const char *nm = names[k - 1];
        if (k >= 4 && k < 28) {
            int L = (k - 4) / 3, ph = (k - 4) % 3;
            snprintf(buf, sizeof buf, "L%d %s", L, ph == 0 ? "gemm" : ph == 1 ? "flush+sync" : "epilogue");
            nm = buf;
        } else if (k == 28) {
            nm = "L7 next->heads";
        } else if (k == 29) {
            nm = "out";
        }
        printf("  %-16s %9.0f  (%4.1f%%)\n", nm ? nm : "?", sum[k] / blocks, 100.0 * sum[k] / total);
    }
    // per-wave L1 GEMM duration (start = after L0 epilogue barrier) by SIMD
    double wsum[8] = {0}, wmax = 0;
    int simd_hist[8][4] = {{0}};
    double spread = 0;
    for (int b = 0; b < blocks; b++) {
        const unsigned long long *s = &hp[(size_t)b * 256];
        double mn = 1e30, mx = 0;
        for (int w = 0; w < 8; w++) {
            double d = (double)(s[40 + w] - s[32 + w]);
            wsum[w] += d;
            mn = d < mn ? d : mn;
            mx = d > mx ? d : mx;
            simd_hist[w][s[48 + w] & 3]++;
        }
        spread += mx - mn;
        wmax += mx;
    }
    // per-chunk progress of waves 0 and 4 (same SIMD) in L1, relative to the L0 epilogue end
    printf("L1 chunk end times (cycles after L1 start), wave 0 | wave 4:\n");
    for (int k = 0; k < 32; k++) {
        double a0 = 0, a4 = 0;
        for (int b = 0; b < blocks; b++) {
            const unsigned long long *s = &hp[(size_t)b * 256];
            a0 += (double)(s[64 + k] - s[32]);
            a4 += (double)(s[128 + k] - s[36]);
        }
        printf("  %2d %8.0f %8.0f\n", k, a0 / blocks, a4 / blocks);
    }
    printf("L1 GEMM per wave (cycles, mean over blocks): ");
    for (int w = 0; w < 8; w++) printf("%.0f ", wsum[w] / blocks);
    printf("\n  mean (max - min) over waves %.0f, mean max %.0f\n", spread / blocks, wmax / blocks);
    for (int w = 0; w < 8; w++)
        printf("  wave %d SIMD histogram: %d %d %d %d\n", w, simd_hist[w][0], simd_hist[w][1], simd_hist[w][2],
               simd_hist[w][3]);
    return 0;
}
