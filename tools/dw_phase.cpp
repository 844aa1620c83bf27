// Diagnostic: per-wave timing of k_dw chunks (built with -DDGS_MLP_PROFILE).
// Build: hipcc -O3 --offload-arch=gfx950 -DDGS_MLP_PROFILE -munsafe-fp-atomics -I include \
//        tools/dw_phase.cpp deformable-3d-gaussians_amd/csrc/mlp.hip deformable-3d-gaussians_amd/csrc/api.hip -o tools/dw_phase.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "dgs.h"

extern "C" void dgs_mlp_set_prof(unsigned long long *p);

int main() {
    const int N = 100000, flags = DGS_MLP_BLENDER;
    const size_t npk = dgs_deform_packed_floats(flags), nsv = dgs_deform_saved_floats(flags, N);
    const size_t nsc = dgs_deform_scratch_floats(flags, N);
    float *pk, *x, *t, *out, *saved, *dout, *scratch, *gbuf;
    hipMalloc(&pk, npk * 4);
    hipMalloc(&x, 3 * (size_t)N * 4);
    hipMalloc(&t, (size_t)N * 4);
    hipMalloc(&out, (size_t)N * 16 * 4);
    hipMalloc(&saved, nsv * 4);
    hipMalloc(&dout, (size_t)N * 16 * 4);
    hipMalloc(&scratch, nsc * 4);
    const int np = dgs_deform_num_params(flags);
    hipMalloc(&gbuf, (size_t)np * 256 * 352 * 4);
    std::vector<float *> grads(np);
    for (int k = 0; k < np; k++) grads[k] = gbuf + (size_t)k * 256 * 352;
    hipMemset(pk, 0, npk * 4);
    hipMemset(x, 0, 3 * (size_t)N * 4);
    hipMemset(t, 0, (size_t)N * 4);
    hipMemset(dout, 0, (size_t)N * 16 * 4);
    unsigned long long *prof;
    hipMalloc(&prof, (size_t)4096 * 256 * 8);
    hipMemset(prof, 0, (size_t)4096 * 256 * 8);
    dgs_mlp_set_prof(prof);
    dgs_deform_forward(flags, N, x, t, pk, out, saved, nullptr);
    for (int r = 0; r < 3; r++) dgs_deform_backward(flags, N, pk, saved, dout, scratch, grads.data(), nullptr);
    hipDeviceSynchronize();
    std::vector<unsigned long long> hp((size_t)256 * 256);
    hipMemcpy(hp.data(), prof, hp.size() * 8, hipMemcpyDeviceToHost);  // first 256 dW blocks
    double chunk = 0, spread = 0, lastend = 0;
    int nb = 0;
    double wsum[16] = {0};
    for (int b = 0; b < 250; b++) {
        const unsigned long long *s = &hp[(size_t)b * 256];
        if (!s[160] || !s[164]) continue;
        nb++;
        chunk += (double)(s[164] - s[160]) / 4;
        for (int c = 0; c < 4; c++) {
            const double bar = (double)s[160 + c];  // barrier end of the previous chunk
            double mn = 1e30, mx = 0;
            for (int w = 0; w < 8; w++) {
                double d = (double)s[64 + c * 16 + w] - bar;
                mn = d < mn ? d : mn;
                mx = d > mx ? d : mx;
                wsum[w] += d / 4;
            }
            spread += (mx - mn) / 4;
            lastend += ((double)s[161 + c] - bar - mx) / 4;
        }
    }
    printf("k_dw blocks sampled %d: chunk %.0f cycles (MFMA ideal 16384)\n", nb, chunk / nb);
    printf("  MFMA-loop end per wave after chunk start: ");
    for (int w = 0; w < 8; w++) printf("%.0f ", wsum[w] / nb);
    printf("\n  spread (last - first wave) %.0f; last wave's MFMA end -> barrier exit %.0f\n", spread / nb, lastend / nb);
    // per workgroup duration by job
    unsigned long long t0 = ~0ull, t1 = 0;
    int last = -1;
    double jsum = 0;
    int jn = 0;
    for (int b = 0; b < 256; b++) {
        const unsigned long long *s = &hp[(size_t)b * 256];
        if (!s[200]) continue;
        t0 = s[200] < t0 ? s[200] : t0;
        t1 = s[201] > t1 ? s[201] : t1;
    }
    for (int b = 0; b <= 256; b++) {
        const unsigned long long *s = &hp[(size_t)(b < 256 ? b : 255) * 256];
        int job = b < 256 && s[200] ? (int)s[202] : -2;
        if (job != last && jn) {
            printf("  job z%d x%d nsplit %d: mean WG %.0f cycles\n", last / 10000, last % 10000, (int)hp[(size_t)(b - 1) * 256 + 203], jsum / jn);
            jsum = 0;
            jn = 0;
        }
        if (job < 0) break;
        last = job;
        jsum += (double)(s[201] - s[200]);
        jn++;
    }
    printf("kernel span (first start -> last end) %.0f cycles\n", (double)(t1 - t0));
    return 0;
}
