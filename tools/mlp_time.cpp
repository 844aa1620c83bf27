// Diagnostic: event-timed k_mlp_fwd / k_mlp_bwd / k_dw at N points (argv[1], default 100k).
// Build: hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -I include tools/mlp_time.cpp \
//        deformable-3d-gaussians_amd/csrc/mlp.hip deformable-3d-gaussians_amd/csrc/api.hip -o tools/mlp_time.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "dgs.h"

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 100000, flags = DGS_MLP_BLENDER;
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
    std::vector<float> h(npk);
    for (size_t i = 0; i < npk; i++) h[i] = (float)((i * 2654435761u) % 1000) * 1e-4f - 0.05f;
    hipMemcpy(pk, h.data(), npk * 4, hipMemcpyHostToDevice);
    hipMemset(x, 0, 3 * (size_t)N * 4);
    hipMemset(t, 0, (size_t)N * 4);
    hipMemset(dout, 0, (size_t)N * 16 * 4);
    dgs_timing_enable(1);
    for (int r = 0; r < 10; r++) {
        dgs_deform_forward(flags, N, x, t, pk, out, saved, nullptr);
        dgs_deform_backward(flags, N, pk, saved, dout, scratch, grads.data(), nullptr);
    }
    hipDeviceSynchronize();
    dgs_timing_reset();
    for (int r = 0; r < 20; r++) {
        dgs_deform_forward(flags, N, x, t, pk, out, saved, nullptr);
        dgs_deform_backward(flags, N, pk, saved, dout, scratch, grads.data(), nullptr);
    }
    hipDeviceSynchronize();
    const char *names[] = {"mlp_fwd", "mlp_bwd", "mlp_dw", "mlp_dw_reduce"};
    for (const char *n : names) {
        int l = 0;
        double ms = dgs_timing_query(n, &l);
        printf("N=%-7d %-14s %.4f ms\n", N, n, l ? ms / l : 0.0);
    }
    return 0;
}
