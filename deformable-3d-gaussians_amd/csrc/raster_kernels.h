// Device-side math shared by the rasterizer kernels (gfx950). Conventions follow the call site
// gaussian_renderer/__init__.py:53-124 and SURVEY.md §8a R1-R7; see oracle/raster_ref.c for the
// plain-C statement of the same math (the tests compare the two).
#pragma once
#include "dgs_common.h"

namespace dgs {

__constant__ constexpr float SH_C0 = 0.28209479177387814f;
__constant__ constexpr float SH_C1 = 0.4886025119029199f;
__constant__ constexpr float SH_C2_0 = 1.0925484305920792f, SH_C2_1 = -1.0925484305920792f,
                             SH_C2_2 = 0.31539156525252005f, SH_C2_3 = -1.0925484305920792f,
                             SH_C2_4 = 0.5462742152960396f;
__constant__ constexpr float SH_C3_0 = -0.5900435899266435f, SH_C3_1 = 2.890611442640554f,
                             SH_C3_2 = -0.4570457994644658f, SH_C3_3 = 0.3731763325901154f,
                             SH_C3_4 = -0.4570457994644658f, SH_C3_5 = 1.445305721320277f,
                             SH_C3_6 = -0.5900435899266435f;

// Camera block loaded once per thread from device memory (uniform address -> scalar loads).
struct Cam {
    float v[16];  // viewmatrix (transposed W2C, row-vector convention)
    float p[16];  // full projection
    float c[3];   // camera centre
};

__device__ inline void load_cam(Cam &cam, const float *view, const float *proj, const float *campos) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
        cam.v[i] = view[i];
        cam.p[i] = proj[i];
    }
    cam.c[0] = campos[0];
    cam.c[1] = campos[1];
    cam.c[2] = campos[2];
}

__device__ inline float3 xform43(const float *m, float3 p) {
    return make_float3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                       m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}

__device__ inline float4 xform44(const float *m, float3 p) {
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                       m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14],
                       m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}

// R (row-major, math convention of utils/general_utils.py:130-151) from the RAW quaternion
// (r, x, y, z); like the CUDA op, the quaternion is not normalised here.
__device__ inline void quat_to_R(float4 q, float R[9]) {
    float r = q.x, x = q.y, y = q.z, z = q.w;
    R[0] = 1.f - 2.f * (y * y + z * z); R[1] = 2.f * (x * y - r * z); R[2] = 2.f * (x * z + r * y);
    R[3] = 2.f * (x * y + r * z); R[4] = 1.f - 2.f * (x * x + z * z); R[5] = 2.f * (y * z - r * x);
    R[6] = 2.f * (x * z - r * y); R[7] = 2.f * (y * z + r * x); R[8] = 1.f - 2.f * (x * x + y * y);
}

// Sigma = L L^T, L = R diag(mod*s); 6-vector [00,01,02,11,12,22] (general_utils.py:114-163).
__device__ inline void cov3d(float3 s, float mod, float4 q, float cov[6]) {
    float R[9];
    quat_to_R(q, R);
    float sx = mod * s.x, sy = mod * s.y, sz = mod * s.z;
    float L[9] = {R[0] * sx, R[1] * sy, R[2] * sz, R[3] * sx, R[4] * sy, R[5] * sz,
                  R[6] * sx, R[7] * sy, R[8] * sz};
    cov[0] = L[0] * L[0] + L[1] * L[1] + L[2] * L[2];
    cov[1] = L[0] * L[3] + L[1] * L[4] + L[2] * L[5];
    cov[2] = L[0] * L[6] + L[1] * L[7] + L[2] * L[8];
    cov[3] = L[3] * L[3] + L[4] * L[4] + L[5] * L[5];
    cov[4] = L[3] * L[6] + L[4] * L[7] + L[5] * L[8];
    cov[5] = L[6] * L[6] + L[7] * L[7] + L[8] * L[8];
}

// T = J W (2x3) for the EWA projection; t is p_view. Returns the clamp masks for backward.
struct Ewa {
    float T[6];
    float tx, ty, tz;
    float mx, my;
};

__device__ inline void ewa_T(float3 tv, float fx, float fy, float tanx, float tany, const float *vm, Ewa &e) {
    float limx = 1.3f * tanx, limy = 1.3f * tany;
    float txtz = tv.x / tv.z, tytz = tv.y / tv.z;
    e.tx = fminf(limx, fmaxf(-limx, txtz)) * tv.z;
    e.ty = fminf(limy, fmaxf(-limy, tytz)) * tv.z;
    e.tz = tv.z;
    e.mx = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    e.my = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    float J00 = fx / e.tz, J02 = -(fx * e.tx) / (e.tz * e.tz);
    float J11 = fy / e.tz, J12 = -(fy * e.ty) / (e.tz * e.tz);
    // W[r][c] = vm[c*4 + r]
    e.T[0] = J00 * vm[0] + J02 * vm[2];
    e.T[1] = J00 * vm[4] + J02 * vm[6];
    e.T[2] = J00 * vm[8] + J02 * vm[10];
    e.T[3] = J11 * vm[1] + J12 * vm[2];
    e.T[4] = J11 * vm[5] + J12 * vm[6];
    e.T[5] = J11 * vm[9] + J12 * vm[10];
}

__device__ inline float3 cov2d(const Ewa &e, const float c[6]) {
    const float *T = e.T;
    // TV = T * V (V symmetric from c)
    float tv0 = T[0] * c[0] + T[1] * c[1] + T[2] * c[2];
    float tv1 = T[0] * c[1] + T[1] * c[3] + T[2] * c[4];
    float tv2 = T[0] * c[2] + T[1] * c[4] + T[2] * c[5];
    float tv3 = T[3] * c[0] + T[4] * c[1] + T[5] * c[2];
    float tv4 = T[3] * c[1] + T[4] * c[3] + T[5] * c[4];
    float tv5 = T[3] * c[2] + T[4] * c[4] + T[5] * c[5];
    float a = tv0 * T[0] + tv1 * T[1] + tv2 * T[2];
    float b = tv0 * T[3] + tv1 * T[4] + tv2 * T[5];
    float cc = tv3 * T[3] + tv4 * T[4] + tv5 * T[5];
    return make_float3(a + 0.3f, b, cc + 0.3f);
}

__device__ inline void tile_rect(float px, float py, int r, int gx, int gy, int &x0, int &y0, int &x1, int &y1) {
    x0 = min(gx, max(0, (int)((px - r) / TILE_X)));
    y0 = min(gy, max(0, (int)((py - r) / TILE_Y)));
    x1 = min(gx, max(0, (int)((px + r + TILE_X - 1) / TILE_X)));
    y1 = min(gy, max(0, (int)((py + r + TILE_Y - 1) / TILE_Y)));
}

// Per-Gaussian backward accumulator layout (floats), filled by the blend backward.
enum AccField {
    ACC_MX = 0, ACC_MY, ACC_CX, ACC_CY, ACC_CZ, ACC_OP, ACC_R, ACC_G, ACC_B, ACC_DEPTH, ACC_DX, ACC_DY,
    ACC_STRIDE = 12
};

}  // namespace dgs
