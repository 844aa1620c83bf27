// Probe: how v_mfma_f32_32x32x16_bf16 rounds C + sum(a_k b_k) (RNE vs truncation, internal width).
// Element (0,0) of the output gets C + sum_k A[0][k] B[k][0]; every other element is 0 + 0.
// hipcc --offload-arch=gfx950 -O2 tools/mfma_round_probe.hip -o tools/mfma_round_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cmath>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct Case { float c; float a[16]; float b[16]; };

__global__ void k(const Case *cs, float *out, int n) {
    const int lane = threadIdx.x;
    for (int q = 0; q < n; q++) {
        bf16x8 a, b;
        for (int j = 0; j < 8; j++) {
            const int kk = 8 * (lane >> 5) + j;
            a[j] = (__bf16)((lane & 31) == 0 ? cs[q].a[kk] : 0.f);
            b[j] = (__bf16)((lane & 31) == 0 ? cs[q].b[kk] : 0.f);
        }
        f32x16 c = {};
        if (lane == 0) c[0] = cs[q].c;
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
        if (lane == 0) out[q] = c[0];
    }
}

int main() {
    const float u = ldexpf(1.f, -23);  // ulp(1)
    Case h[8];
    memset(h, 0, sizeof(h));
    const char *name[8];
    int n = 0;
    auto add = [&](const char *nm, float c, float a0, float b0, float a1 = 0, float b1 = 0, float a2 = 0, float b2 = 0) {
        h[n].c = c; h[n].a[0] = a0; h[n].b[0] = b0; h[n].a[1] = a1; h[n].b[1] = b1; h[n].a[2] = a2; h[n].b[2] = b2;
        name[n++] = nm;
    };
    add("C=1 + 0.75ulp (RNE: 1+ulp, RTZ: 1)", 1.f, 1.f, 0.75f * u);
    add("C=1 - 0.25ulp (RNE: 1, RTZ: 1-ulp/2)", 1.f, 1.f, -0.25f * u);
    add("C=1 + 0.5ulp tie (RNE: 1)", 1.f, 1.f, 0.5f * u);
    add("C=0: 1 + 2^-30 - 1 (exact: 2^-30)", 0.f, 1.f, 1.f, 1.f, ldexpf(1.f, -30), -1.f, 1.f);
    add("C=2^-30: 1 - 1 (exact: 2^-30)", ldexpf(1.f, -30), 1.f, 1.f, -1.f, 1.f);
    add("C=1: 0.3ulp + 0.3ulp (exact 1+0.6ulp, RNE 1+ulp)", 1.f, 1.f, 0.375f * u, 1.f, 0.375f * u);
    add("C=-1 - 0.75ulp (RNE: -1-ulp, RTZ: -1)", -1.f, 1.f, -0.75f * u);
    add("C=1 + 3*2^-26 (RNE: 1 (0.375ulp), RTZ: 1)", 1.f, 1.f, 0.375f * u);
    Case *d; float *o;
    hipMalloc(&d, sizeof(h)); hipMalloc(&o, sizeof(float) * 8);
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, n);
    float r[8];
    hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    for (int q = 0; q < n; q++) {
        double ex = h[q].c;
        for (int j = 0; j < 16; j++) ex += (double)h[q].a[j] * h[q].b[j];
        printf("%-50s got %.10e (1+%.3f ulp) exact %.10e\n", name[q], r[q], (r[q] - 1.0) / u, ex);
    }
    return 0;
}
