/*
 * ORACLE (test infrastructure only) — plain-C restatement of the differentiable Gaussian
 * rasterizer that gaussian_renderer/__init__.py:53-124 calls through `diff_gaussian_rasterization`.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / CPU baseline; the product path never links or calls it.
 *
 * PARITY UNPINNED for the projection / binning / blending math: the CUDA rasterizer is an
 * un-vendored git submodule (.gitmodules:4-7, ingra14m/diff-gaussian-rasterization-extentions,
 * branch filter-norm, commit unpinned) that is absent from /root/reference, and the reference
 * ships no rasterizer test or fixture. This file restates the public 3DGS algorithm (Kerbl et al.,
 * cited README.md:202-212) as the reference's call site uses it:
 *   - camera conventions: scene/cameras.py:55-61, utils/graphics_utils.py:42-76 (row-vector,
 *     transposed matrices: p_view = p * viewmatrix, p_hom = p * projmatrix);
 *   - SH basis / +0.5 / clamp: utils/sh_utils.py:26-112 and gaussian_renderer/__init__.py:105-109
 *     (pinned by tests/golden/sh.npz);
 *   - covariance Sigma = R S S^T R^T, 6-vector [00,01,02,11,12,22]: utils/general_utils.py:130-163
 *     (pinned by tests/golden/cov_lr.npz for unit quaternions; like the CUDA path, the quaternion
 *     is used un-normalised here);
 *   - depth output D = sum depth*alpha*T (fork extension, R5); means2D_densify grad = per-pixel
 *     |dL/dmean2D| accumulated per axis (R8: the fork's semantics are not visible; this build's
 *     documented choice).
 * It is self-checked by finite differences and a dense torch autograd restatement (tests/).
 *
 * Build: oracle/Makefile -> oracle/liboracle_raster.so (gcc -O2 -fopenmp).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BX 16
#define BY 16

typedef struct {
    int image_height, image_width;
    float tanfovx, tanfovy;
    float bg[3];
    float scale_modifier;
    float viewmatrix[16];
    float projmatrix[16];
    int sh_degree;
    float campos[3];
    int prefiltered;
} ORSettings;

static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

typedef struct {
    ORSettings s;
    int N, M, P;
    int grid_x, grid_y;
    /* inputs (copies) */
    float *means3D, *shs, *colors_in, *opac, *scales, *rots, *cov_in;
    /* per-Gaussian geometry */
    float *depth, *xy, *conic_o, *rgb, *cov3D;
    float *radf, *vz, *pxy; /* 3 sqrt(lambda_max) before the ceil; view-space z; pixel centre */
    int *radii, *tiles;
    uint8_t *clamped;
    float *rgb_raw; /* SH colour + 0.5 before the clamp at 0 (tests: or_preprocess_flags) */
    /* binning */
    uint64_t *keys;
    uint32_t *vals;
    int *range_lo, *range_hi;
    /* per-pixel */
    float *final_T;
    int *n_contrib;
} ORState;

static float *dupf(const float *p, size_t n) {
    if (!p) return NULL;
    float *q = (float *)malloc(n * sizeof(float));
    memcpy(q, p, n * sizeof(float));
    return q;
}

static void xform43(const float *m, const float *p, float *o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}

static void xform44(const float *m, const float *p, float *o) {
    xform43(m, p, o);
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}

/* rotation matrix R (row-major, math convention of general_utils.build_rotation) from raw q */
static void quat_to_R(const float *q, float R[9]) {
    float r = q[0], x = q[1], y = q[2], z = q[3];
    R[0] = 1.f - 2.f * (y * y + z * z); R[1] = 2.f * (x * y - r * z); R[2] = 2.f * (x * z + r * y);
    R[3] = 2.f * (x * y + r * z); R[4] = 1.f - 2.f * (x * x + z * z); R[5] = 2.f * (y * z - r * x);
    R[6] = 2.f * (x * z - r * y); R[7] = 2.f * (y * z + r * x); R[8] = 1.f - 2.f * (x * x + y * y);
}

/* Sigma = L L^T, L = R diag(mod*s) ; out 6-vector [00,01,02,11,12,22] */
static void cov3d_from(const float *s, float mod, const float *q, float *cov) {
    float R[9];
    quat_to_R(q, R);
    float L[9];
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) L[i * 3 + k] = R[i * 3 + k] * (mod * s[k]);
    float S[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            float a = 0.f;
            for (int k = 0; k < 3; k++) a += L[i * 3 + k] * L[j * 3 + k];
            S[i * 3 + j] = a;
        }
    cov[0] = S[0]; cov[1] = S[1]; cov[2] = S[2]; cov[3] = S[4]; cov[4] = S[5]; cov[5] = S[8];
}

/* EWA: cov2D = J W Sigma W^T J^T (+0.3 on the diagonal); t = p_view */
static void cov2d_from(const float *tv, float fx, float fy, float tanx, float tany, const float *cov3,
                       const float *vm, float *out) {
    float limx = 1.3f * tanx, limy = 1.3f * tany;
    float txtz = tv[0] / tv[2], tytz = tv[1] / tv[2];
    float tx = fminf(limx, fmaxf(-limx, txtz)) * tv[2];
    float ty = fminf(limy, fmaxf(-limy, tytz)) * tv[2];
    float tz = tv[2];
    float J00 = fx / tz, J02 = -(fx * tx) / (tz * tz);
    float J11 = fy / tz, J12 = -(fy * ty) / (tz * tz);
    /* W (math) rows: view rotation; vm stored transposed: W[r][c] = vm[c*4+r] */
    float Wm[9] = {vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]};
    float T[6];
    for (int c = 0; c < 3; c++) {
        T[c] = J00 * Wm[0 * 3 + c] + J02 * Wm[2 * 3 + c];
        T[3 + c] = J11 * Wm[1 * 3 + c] + J12 * Wm[2 * 3 + c];
    }
    float V[9] = {cov3[0], cov3[1], cov3[2], cov3[1], cov3[3], cov3[4], cov3[2], cov3[4], cov3[5]};
    float TV[6];
    for (int r = 0; r < 2; r++)
        for (int c = 0; c < 3; c++) {
            float a = 0.f;
            for (int k = 0; k < 3; k++) a += T[r * 3 + k] * V[k * 3 + c];
            TV[r * 3 + c] = a;
        }
    float a = 0.f, b = 0.f, cc = 0.f;
    for (int k = 0; k < 3; k++) {
        a += TV[0 * 3 + k] * T[0 * 3 + k];
        b += TV[0 * 3 + k] * T[1 * 3 + k];
        cc += TV[1 * 3 + k] * T[1 * 3 + k];
    }
    out[0] = a + 0.3f;
    out[1] = b;
    out[2] = cc + 0.3f;
}

static void sh_to_rgb(int deg, int M, const float *sh, const float *dir, float *rgb, uint8_t *cl, float *raw) {
    float x = dir[0], y = dir[1], z = dir[2];
    for (int c = 0; c < 3; c++) {
#define S(k) sh[(k) * 3 + c]
        float r = SH_C0 * S(0);
        if (deg > 0) {
            r = r - SH_C1 * y * S(1) + SH_C1 * z * S(2) - SH_C1 * x * S(3);
            if (deg > 1) {
                float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                r = r + SH_C2[0] * xy * S(4) + SH_C2[1] * yz * S(5) + SH_C2[2] * (2.f * zz - xx - yy) * S(6) +
                    SH_C2[3] * xz * S(7) + SH_C2[4] * (xx - yy) * S(8);
                if (deg > 2) {
                    r = r + SH_C3[0] * y * (3.f * xx - yy) * S(9) + SH_C3[1] * xy * z * S(10) +
                        SH_C3[2] * y * (4.f * zz - xx - yy) * S(11) +
                        SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy) * S(12) +
                        SH_C3[4] * x * (4.f * zz - xx - yy) * S(13) + SH_C3[5] * z * (xx - yy) * S(14) +
                        SH_C3[6] * x * (xx - 3.f * yy) * S(15);
                }
            }
        }
#undef S
        r += 0.5f;
        if (raw) raw[c] = r;
        cl[c] = r < 0.f;
        rgb[c] = r < 0.f ? 0.f : r;
    }
    (void)M;
}

int or_forward(const ORSettings *s, int N, int M, const float *means3D, const float *shs,
               const float *colors_precomp, const float *opac, const float *scales,
               const float *rots, const float *cov3D_precomp, float *out_color, float *out_depth,
               int *out_radii, void **state_out) {
    if ((shs == NULL) == (colors_precomp == NULL)) return -1;
    if (cov3D_precomp == NULL && (scales == NULL || rots == NULL)) return -2;
    ORState *st = (ORState *)calloc(1, sizeof(ORState));
    st->s = *s;
    st->N = N;
    st->M = M;
    const int H = s->image_height, W = s->image_width;
    st->grid_x = (W + BX - 1) / BX;
    st->grid_y = (H + BY - 1) / BY;
    const int T = st->grid_x * st->grid_y;
    st->means3D = dupf(means3D, (size_t)N * 3);
    st->shs = dupf(shs, (size_t)N * M * 3);
    st->colors_in = dupf(colors_precomp, (size_t)N * 3);
    st->opac = dupf(opac, (size_t)N);
    st->scales = cov3D_precomp ? NULL : dupf(scales, (size_t)N * 3);
    st->rots = cov3D_precomp ? NULL : dupf(rots, (size_t)N * 4);
    st->cov_in = dupf(cov3D_precomp, (size_t)N * 6);
    st->depth = (float *)calloc(N, sizeof(float));
    st->xy = (float *)calloc((size_t)N * 2, sizeof(float));
    st->conic_o = (float *)calloc((size_t)N * 4, sizeof(float));
    st->rgb = (float *)calloc((size_t)N * 3, sizeof(float));
    st->cov3D = (float *)calloc((size_t)N * 6, sizeof(float));
    st->radii = (int *)calloc(N, sizeof(int));
    st->tiles = (int *)calloc(N, sizeof(int));
    st->clamped = (uint8_t *)calloc((size_t)N * 3, 1);
    st->rgb_raw = (float *)calloc((size_t)N * 3, sizeof(float));
    st->radf = (float *)calloc(N, sizeof(float));
    st->vz = (float *)calloc(N, sizeof(float));
    st->pxy = (float *)calloc((size_t)N * 2, sizeof(float));

    const float fx = W / (2.f * s->tanfovx), fy = H / (2.f * s->tanfovy);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < N; i++) {
        const float *p = st->means3D + 3 * i;
        float pv[3];
        xform43(s->viewmatrix, p, pv);
        st->vz[i] = pv[2];
        if (pv[2] <= 0.2f) continue;
        float *cov = st->cov3D + 6 * i;
        if (st->cov_in)
            memcpy(cov, st->cov_in + 6 * i, 6 * sizeof(float));
        else
            cov3d_from(st->scales + 3 * i, s->scale_modifier, st->rots + 4 * i, cov);
        float c2[3];
        cov2d_from(pv, fx, fy, s->tanfovx, s->tanfovy, cov, s->viewmatrix, c2);
        float det = c2[0] * c2[2] - c2[1] * c2[1];
        if (det == 0.f) continue;
        float di = 1.f / det;
        float con[3] = {c2[2] * di, -c2[1] * di, c2[0] * di};
        float mid = 0.5f * (c2[0] + c2[2]);
        float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        st->radf[i] = 3.f * sqrtf(fmaxf(l1, l2));
        int rad = (int)ceilf(st->radf[i]);
        float ph[4];
        xform44(s->projmatrix, p, ph);
        float pw = 1.f / (ph[3] + 0.0000001f);
        float px = ((ph[0] * pw + 1.f) * W - 1.f) * 0.5f;
        float py = ((ph[1] * pw + 1.f) * H - 1.f) * 0.5f;
        st->pxy[2 * i] = px; /* also for Gaussians culled by an empty rect (tests: rect margins) */
        st->pxy[2 * i + 1] = py;
        int rminx = (int)fminf(st->grid_x, fmaxf(0, (int)((px - rad) / BX)));
        int rminy = (int)fminf(st->grid_y, fmaxf(0, (int)((py - rad) / BY)));
        int rmaxx = (int)fminf(st->grid_x, fmaxf(0, (int)((px + rad + BX - 1) / BX)));
        int rmaxy = (int)fminf(st->grid_y, fmaxf(0, (int)((py + rad + BY - 1) / BY)));
        int area = (rmaxx - rminx) * (rmaxy - rminy);
        if (area == 0) continue;
        if (st->colors_in) {
            memcpy(st->rgb + 3 * i, st->colors_in + 3 * i, 3 * sizeof(float));
        } else {
            float d[3] = {p[0] - s->campos[0], p[1] - s->campos[1], p[2] - s->campos[2]};
            float n = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            d[0] /= n; d[1] /= n; d[2] /= n;
            sh_to_rgb(s->sh_degree, M, st->shs + (size_t)i * M * 3, d, st->rgb + 3 * i, st->clamped + 3 * i,
                      st->rgb_raw + 3 * i);
        }
        st->depth[i] = pv[2];
        st->radii[i] = rad;
        st->xy[2 * i] = px;
        st->xy[2 * i + 1] = py;
        st->conic_o[4 * i] = con[0];
        st->conic_o[4 * i + 1] = con[1];
        st->conic_o[4 * i + 2] = con[2];
        st->conic_o[4 * i + 3] = st->opac[i];
        st->tiles[i] = area;
    }
    /* binning: per tile, visible Gaussians sorted by (depth bits, index) — equals a stable radix
       sort of (tile<<32 | depth_bits) keys emitted in index order */
    size_t P = 0;
    for (int i = 0; i < N; i++) P += st->tiles[i];
    st->P = (int)P;
    st->keys = (uint64_t *)malloc((P ? P : 1) * sizeof(uint64_t));
    st->vals = (uint32_t *)malloc((P ? P : 1) * sizeof(uint32_t));
    size_t off = 0;
    for (int i = 0; i < N; i++) {
        if (!st->tiles[i]) continue;
        float px = st->xy[2 * i], py = st->xy[2 * i + 1];
        int rad = st->radii[i];
        int rminx = (int)fminf(st->grid_x, fmaxf(0, (int)((px - rad) / BX)));
        int rminy = (int)fminf(st->grid_y, fmaxf(0, (int)((py - rad) / BY)));
        int rmaxx = (int)fminf(st->grid_x, fmaxf(0, (int)((px + rad + BX - 1) / BX)));
        int rmaxy = (int)fminf(st->grid_y, fmaxf(0, (int)((py + rad + BY - 1) / BY)));
        uint32_t db;
        memcpy(&db, &st->depth[i], 4);
        for (int y = rminy; y < rmaxy; y++)
            for (int x = rminx; x < rmaxx; x++) {
                st->keys[off] = ((uint64_t)(y * st->grid_x + x) << 32) | db;
                st->vals[off] = (uint32_t)i;
                off++;
            }
    }
    /* LSD radix sort (stable), 8 bits per pass */
    {
        uint64_t *k2 = (uint64_t *)malloc((P ? P : 1) * sizeof(uint64_t));
        uint32_t *v2 = (uint32_t *)malloc((P ? P : 1) * sizeof(uint32_t));
        for (int shift = 0; shift < 64; shift += 8) {
            size_t cnt[257] = {0};
            for (size_t j = 0; j < P; j++) cnt[((st->keys[j] >> shift) & 255) + 1]++;
            for (int b = 0; b < 256; b++) cnt[b + 1] += cnt[b];
            for (size_t j = 0; j < P; j++) {
                size_t d = cnt[(st->keys[j] >> shift) & 255]++;
                k2[d] = st->keys[j];
                v2[d] = st->vals[j];
            }
            uint64_t *tk = st->keys; st->keys = k2; k2 = tk;
            uint32_t *tv = st->vals; st->vals = v2; v2 = tv;
        }
        free(k2);
        free(v2);
    }
    st->range_lo = (int *)calloc(T, sizeof(int));
    st->range_hi = (int *)calloc(T, sizeof(int));
    for (size_t j = 0; j < P; j++) {
        int t = (int)(st->keys[j] >> 32);
        if (j == 0 || (int)(st->keys[j - 1] >> 32) != t) st->range_lo[t] = (int)j;
        if (j == P - 1 || (int)(st->keys[j + 1] >> 32) != t) st->range_hi[t] = (int)j + 1;
    }
    st->final_T = (float *)calloc((size_t)H * W, sizeof(float));
    st->n_contrib = (int *)calloc((size_t)H * W, sizeof(int));
    /* front-to-back blend per pixel */
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < T; t++) {
        int tx = t % st->grid_x, ty = t / st->grid_x;
        for (int ly = 0; ly < BY; ly++)
            for (int lx = 0; lx < BX; lx++) {
                int px = tx * BX + lx, py = ty * BY + ly;
                if (px >= W || py >= H) continue;
                float pfx = (float)px, pfy = (float)py;
                float Tt = 1.f, C[3] = {0, 0, 0}, Dd = 0.f;
                int contributor = 0, last = 0;
                for (int j = st->range_lo[t]; j < st->range_hi[t]; j++) {
                    contributor++;
                    int g = st->vals[j];
                    float dx = st->xy[2 * g] - pfx, dy = st->xy[2 * g + 1] - pfy;
                    const float *co = st->conic_o + 4 * g;
                    float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > 0.f) continue;
                    float alpha = fminf(0.99f, co[3] * expf(power));
                    if (alpha < 1.f / 255.f) continue;
                    float testT = Tt * (1.f - alpha);
                    if (testT < 0.0001f) break;
                    for (int c = 0; c < 3; c++) C[c] += st->rgb[3 * g + c] * alpha * Tt;
                    Dd += st->depth[g] * alpha * Tt;
                    Tt = testT;
                    last = contributor;
                }
                int pid = py * W + px;
                st->final_T[pid] = Tt;
                st->n_contrib[pid] = last;
                for (int c = 0; c < 3; c++) out_color[c * H * W + pid] = C[c] + Tt * s->bg[c];
                out_depth[pid] = Dd;
            }
    }
    memcpy(out_radii, st->radii, N * sizeof(int));
    *state_out = st;
    return 0;
}

int or_num_rendered(void *p) { return ((ORState *)p)->P; }

/* dL/dq for R(q) built un-normalised (quat_to_R), given dL/dR (row-major) */
static void dR_dq(const float *q, const float *dR, float *dq) {
    float r = q[0], x = q[1], y = q[2], z = q[3];
    /* R entries as functions of q, differentiated term by term */
    dq[0] = 2.f * (-z * dR[1] + y * dR[2] + z * dR[3] - x * dR[5] - y * dR[6] + x * dR[7]);
    dq[1] = 2.f * (y * dR[1] + z * dR[2] + y * dR[3] - r * dR[5] + z * dR[6] + r * dR[7]) -
            4.f * x * (dR[4] + dR[8]);
    dq[2] = 2.f * (x * dR[1] + r * dR[2] + x * dR[3] + z * dR[5] - r * dR[6] + z * dR[7]) -
            4.f * y * (dR[0] + dR[8]);
    dq[3] = 2.f * (-r * dR[1] + x * dR[2] + r * dR[3] + y * dR[5] + x * dR[6] + y * dR[7]) -
            4.f * z * (dR[0] + dR[4]);
}

int or_backward(void *p, const float *dL_dpix, const float *dL_ddepth, float *dL_dmeans3D,
                float *dL_dmeans2D, float *dL_dmeans2D_densify, float *dL_dcolors,
                float *dL_dopac, float *dL_dcov3D, float *dL_dshs, float *dL_dscales,
                float *dL_drots) {
    ORState *st = (ORState *)p;
    const ORSettings *s = &st->s;
    const int N = st->N, M = st->M, H = s->image_height, W = s->image_width;
    const int T = st->grid_x * st->grid_y;
    /* per-Gaussian accumulators (render backward). The tiles are split into NCH fixed contiguous
       chunks, each with its own accumulators, summed per Gaussian in chunk order afterwards: the float
       sums depend on (N, tiles) only, never on the thread count, so the result is reproducible and the
       chunks run in parallel (OpenMP). */
    enum { NF = 12 }; /* m2 xy, |m2| xy, conic xyz, opacity, rgb, depth */
    int NCH = T < 32 ? (T > 0 ? T : 1) : 32;
    while (NCH > 1 && (size_t)NCH * N * NF * sizeof(float) > ((size_t)768 << 20)) NCH /= 2;
    float *chunk_acc = (float *)calloc((size_t)NCH * N * NF + 1, sizeof(float));
    if (!chunk_acc) return -1; /* out of host memory: the caller raises */
    const float hx = 0.5f * W, hy = 0.5f * H;
#pragma omp parallel for schedule(dynamic, 1)
    for (int ch = 0; ch < NCH; ch++) {
        float *A = chunk_acc + (size_t)ch * N * NF;
        const int t_lo = (int)((long long)T * ch / NCH), t_hi = (int)((long long)T * (ch + 1) / NCH);
        for (int t = t_lo; t < t_hi; t++) {
        int tx = t % st->grid_x, ty = t / st->grid_x;
        for (int ly = 0; ly < BY; ly++)
            for (int lx = 0; lx < BX; lx++) {
                int px = tx * BX + lx, py = ty * BY + ly;
                if (px >= W || py >= H) continue;
                int pid = py * W + px;
                float pfx = (float)px, pfy = (float)py;
                const float Tfinal = st->final_T[pid];
                float Tt = Tfinal;
                int last = st->n_contrib[pid];
                float dpix[3], acc[3] = {0, 0, 0}, lastc[3] = {0, 0, 0};
                for (int c = 0; c < 3; c++) dpix[c] = dL_dpix[c * H * W + pid];
                float ddep = dL_ddepth ? dL_ddepth[pid] : 0.f;
                float accd = 0.f, lastd = 0.f, last_alpha = 0.f;
                float bgdot = 0.f;
                for (int c = 0; c < 3; c++) bgdot += s->bg[c] * dpix[c];
                int lo = st->range_lo[t];
                for (int j = lo + last - 1; j >= lo; j--) {
                    int g = st->vals[j];
                    float *a = A + (size_t)g * NF;
                    float dx = st->xy[2 * g] - pfx, dy = st->xy[2 * g + 1] - pfy;
                    const float *co = st->conic_o + 4 * g;
                    float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > 0.f) continue;
                    float G = expf(power);
                    float alpha = fminf(0.99f, co[3] * G);
                    if (alpha < 1.f / 255.f) continue;
                    Tt = Tt / (1.f - alpha);
                    float dchdcol = alpha * Tt;
                    float dL_dalpha = 0.f;
                    for (int c = 0; c < 3; c++) {
                        float col = st->rgb[3 * g + c];
                        acc[c] = last_alpha * lastc[c] + (1.f - last_alpha) * acc[c];
                        lastc[c] = col;
                        dL_dalpha += (col - acc[c]) * dpix[c];
                        a[8 + c] += dchdcol * dpix[c];
                    }
                    float dg = st->depth[g];
                    accd = last_alpha * lastd + (1.f - last_alpha) * accd;
                    lastd = dg;
                    dL_dalpha += (dg - accd) * ddep;
                    a[11] += dchdcol * ddep;
                    dL_dalpha *= Tt;
                    last_alpha = alpha;
                    dL_dalpha += (-Tfinal / (1.f - alpha)) * bgdot;
                    /* alpha = min(0.99, o*G): like the upstream kernel, the clamp is not
                       differentiated (treated as alpha = o*G) */
                    float dL_dG = co[3] * dL_dalpha;
                    float gdx = G * dx, gdy = G * dy;
                    float dGdx = -gdx * co[0] - gdy * co[1];
                    float dGdy = -gdy * co[2] - gdx * co[1];
                    float gmx = dL_dG * dGdx * hx, gmy = dL_dG * dGdy * hy;
                    a[0] += gmx;
                    a[1] += gmy;
                    a[2] += fabsf(gmx);
                    a[3] += fabsf(gmy);
                    a[4] += -0.5f * gdx * dx * dL_dG;
                    a[5] += -0.5f * gdx * dy * dL_dG;
                    a[6] += -0.5f * gdy * dy * dL_dG;
                    a[7] += G * dL_dalpha;
                }
            }
        }
    }
    float *g_m2 = (float *)calloc((size_t)N * 2 + 1, sizeof(float));
    float *g_dens = (float *)calloc((size_t)N * 2 + 1, sizeof(float));
    float *g_con = (float *)calloc((size_t)N * 3 + 1, sizeof(float));
    float *g_op = (float *)calloc((size_t)N + 1, sizeof(float));
    float *g_col = (float *)calloc((size_t)N * 3 + 1, sizeof(float));
    float *g_dep = (float *)calloc((size_t)N + 1, sizeof(float));
    if (!g_m2 || !g_dens || !g_con || !g_op || !g_col || !g_dep) {
        free(chunk_acc); free(g_m2); free(g_dens); free(g_con); free(g_op); free(g_col); free(g_dep);
        return -1;
    }
#pragma omp parallel for schedule(static)
    for (int i = 0; i < N; i++) {
        float r[NF] = {0};
        for (int ch = 0; ch < NCH; ch++) {
            const float *a = chunk_acc + ((size_t)ch * N + i) * NF;
            for (int k = 0; k < NF; k++) r[k] += a[k];
        }
        g_m2[2 * i] = r[0]; g_m2[2 * i + 1] = r[1];
        g_dens[2 * i] = r[2]; g_dens[2 * i + 1] = r[3];
        g_con[3 * i] = r[4]; g_con[3 * i + 1] = r[5]; g_con[3 * i + 2] = r[6];
        g_op[i] = r[7];
        g_col[3 * i] = r[8]; g_col[3 * i + 1] = r[9]; g_col[3 * i + 2] = r[10];
        g_dep[i] = r[11];
    }
    free(chunk_acc);
    const float fx = W / (2.f * s->tanfovx), fy = H / (2.f * s->tanfovy);
    memset(dL_dmeans3D, 0, sizeof(float) * 3 * N);
    if (dL_dshs) memset(dL_dshs, 0, sizeof(float) * 3 * M * N);
    if (dL_dscales) memset(dL_dscales, 0, sizeof(float) * 3 * N);
    if (dL_drots) memset(dL_drots, 0, sizeof(float) * 4 * N);
    if (dL_dcov3D) memset(dL_dcov3D, 0, sizeof(float) * 6 * N);
    for (int i = 0; i < N; i++) {
        dL_dmeans2D[3 * i] = g_m2[2 * i];
        dL_dmeans2D[3 * i + 1] = g_m2[2 * i + 1];
        dL_dmeans2D[3 * i + 2] = 0.f;
        dL_dmeans2D_densify[3 * i] = g_dens[2 * i];
        dL_dmeans2D_densify[3 * i + 1] = g_dens[2 * i + 1];
        dL_dmeans2D_densify[3 * i + 2] = 0.f;
        dL_dopac[i] = g_op[i];
        if (dL_dcolors) for (int c = 0; c < 3; c++) dL_dcolors[3 * i + c] = g_col[3 * i + c];
    }
#pragma omp parallel for schedule(static)
    for (int i = 0; i < N; i++) {
        if (st->radii[i] <= 0) continue;
        const float *pm = st->means3D + 3 * i;
        float dmean[3] = {0, 0, 0};
        /* (1) conic -> cov2D -> (cov3D, mean via J(t)) */
        float tv[3];
        xform43(s->viewmatrix, pm, tv);
        const float *cov3 = st->cov3D + 6 * i;
        float limx = 1.3f * s->tanfovx, limy = 1.3f * s->tanfovy;
        float txtz = tv[0] / tv[2], tytz = tv[1] / tv[2];
        float tx = fminf(limx, fmaxf(-limx, txtz)) * tv[2];
        float ty = fminf(limy, fmaxf(-limy, tytz)) * tv[2];
        float tz = tv[2];
        float xm = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
        float ym = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
        float J00 = fx / tz, J02 = -(fx * tx) / (tz * tz);
        float J11 = fy / tz, J12 = -(fy * ty) / (tz * tz);
        const float *vm = s->viewmatrix;
        float Wm[9] = {vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]};
        float Tm[6];
        for (int c = 0; c < 3; c++) {
            Tm[c] = J00 * Wm[c] + J02 * Wm[6 + c];
            Tm[3 + c] = J11 * Wm[3 + c] + J12 * Wm[6 + c];
        }
        float V[9] = {cov3[0], cov3[1], cov3[2], cov3[1], cov3[3], cov3[4], cov3[2], cov3[4], cov3[5]};
        float TV[6];
        for (int r = 0; r < 2; r++)
            for (int c = 0; c < 3; c++) {
                float a = 0.f;
                for (int k = 0; k < 3; k++) a += Tm[r * 3 + k] * V[k * 3 + c];
                TV[r * 3 + c] = a;
            }
        float a = 0.f, b = 0.f, c2 = 0.f;
        for (int k = 0; k < 3; k++) {
            a += TV[k] * Tm[k];
            b += TV[k] * Tm[3 + k];
            c2 += TV[3 + k] * Tm[3 + k];
        }
        a += 0.3f;
        c2 += 0.3f;
        float den = a * c2 - b * b;
        float d2i = 1.f / (den * den + 0.0000001f);
        const float *gc = g_con + 3 * i;
        float dLa = 0.f, dLb = 0.f, dLc = 0.f;
        if (d2i != 0.f) {
            /* gc[1] is half the gradient of the conic's off-diagonal entry (R6) */
            dLa = d2i * (-c2 * c2 * gc[0] + 2.f * b * c2 * gc[1] + (den - a * c2) * gc[2]);
            dLc = d2i * (-a * a * gc[2] + 2.f * a * b * gc[1] + (den - a * c2) * gc[0]);
            dLb = d2i * 2.f * (b * c2 * gc[0] - (den + 2.f * b * b) * gc[1] + a * b * gc[2]);
        }
        /* dL/dSigma (unique entries; off-diagonals appear twice in Sigma) */
        float dcov[6];
        dcov[0] = Tm[0] * Tm[0] * dLa + Tm[0] * Tm[3] * dLb + Tm[3] * Tm[3] * dLc;
        dcov[3] = Tm[1] * Tm[1] * dLa + Tm[1] * Tm[4] * dLb + Tm[4] * Tm[4] * dLc;
        dcov[5] = Tm[2] * Tm[2] * dLa + Tm[2] * Tm[5] * dLb + Tm[5] * Tm[5] * dLc;
        dcov[1] = 2.f * Tm[0] * Tm[1] * dLa + (Tm[0] * Tm[4] + Tm[1] * Tm[3]) * dLb + 2.f * Tm[3] * Tm[4] * dLc;
        dcov[2] = 2.f * Tm[0] * Tm[2] * dLa + (Tm[0] * Tm[5] + Tm[2] * Tm[3]) * dLb + 2.f * Tm[3] * Tm[5] * dLc;
        dcov[4] = 2.f * Tm[2] * Tm[1] * dLa + (Tm[1] * Tm[5] + Tm[2] * Tm[4]) * dLb + 2.f * Tm[4] * Tm[5] * dLc;
        /* dL/dT (2x3): row0 = 2 (V T0) dLa + (V T1) dLb ; row1 = 2 (V T1) dLc + (V T0) dLb */
        float dT[6];
        for (int k = 0; k < 3; k++) {
            float v0 = V[k * 3] * Tm[0] + V[k * 3 + 1] * Tm[1] + V[k * 3 + 2] * Tm[2];
            float v1 = V[k * 3] * Tm[3] + V[k * 3 + 1] * Tm[4] + V[k * 3 + 2] * Tm[5];
            dT[k] = 2.f * v0 * dLa + v1 * dLb;
            dT[3 + k] = 2.f * v1 * dLc + v0 * dLb;
        }
        /* T = J W  -> dJ = dT W^T */
        float dJ00 = Wm[0] * dT[0] + Wm[1] * dT[1] + Wm[2] * dT[2];
        float dJ02 = Wm[6] * dT[0] + Wm[7] * dT[1] + Wm[8] * dT[2];
        float dJ11 = Wm[3] * dT[3] + Wm[4] * dT[4] + Wm[5] * dT[5];
        float dJ12 = Wm[6] * dT[3] + Wm[7] * dT[4] + Wm[8] * dT[5];
        float tz2 = 1.f / (tz * tz), tz3 = tz2 / tz;
        float dtx = xm * -fx * tz2 * dJ02;
        float dty = ym * -fy * tz2 * dJ12;
        float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2.f * fx * tx) * tz3 * dJ02 +
                    (2.f * fy * ty) * tz3 * dJ12;
        /* t = W p + c -> dp = W^T dt */
        dmean[0] += Wm[0] * dtx + Wm[3] * dty + Wm[6] * dtz;
        dmean[1] += Wm[1] * dtx + Wm[4] * dty + Wm[7] * dtz;
        dmean[2] += Wm[2] * dtx + Wm[5] * dty + Wm[8] * dtz;
        /* (2) mean2D -> mean3D through the projection */
        {
            const float *pj = s->projmatrix;
            float ph[4];
            xform44(pj, pm, ph);
            float mw = 1.f / (ph[3] + 0.0000001f);
            float mul1 = ph[0] * mw * mw, mul2 = ph[1] * mw * mw;
            float gx = g_m2[2 * i], gy = g_m2[2 * i + 1];
            dmean[0] += (pj[0] * mw - pj[3] * mul1) * gx + (pj[1] * mw - pj[3] * mul2) * gy;
            dmean[1] += (pj[4] * mw - pj[7] * mul1) * gx + (pj[5] * mw - pj[7] * mul2) * gy;
            dmean[2] += (pj[8] * mw - pj[11] * mul1) * gx + (pj[9] * mw - pj[11] * mul2) * gy;
        }
        /* (3) SH -> (coefficients, mean via the view direction) */
        if (!st->colors_in) {
            float dv[3] = {pm[0] - s->campos[0], pm[1] - s->campos[1], pm[2] - s->campos[2]};
            float n = sqrtf(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
            float x = dv[0] / n, y = dv[1] / n, z = dv[2] / n;
            const float *sh = st->shs + (size_t)i * M * 3;
            float *dsh = dL_dshs + (size_t)i * M * 3;
            float dRGB[3];
            for (int c = 0; c < 3; c++) dRGB[c] = st->clamped[3 * i + c] ? 0.f : g_col[3 * i + c];
            float ddir[3] = {0, 0, 0};
            int deg = s->sh_degree;
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            for (int c = 0; c < 3; c++) {
                float g = dRGB[c];
#define SH(k) sh[(k) * 3 + c]
#define DSH(k, v) dsh[(k) * 3 + c] = (v) * g
                DSH(0, SH_C0);
                if (deg > 0) {
                    DSH(1, -SH_C1 * y);
                    DSH(2, SH_C1 * z);
                    DSH(3, -SH_C1 * x);
                    float gx = -SH_C1 * SH(3), gy = -SH_C1 * SH(1), gz = SH_C1 * SH(2);
                    if (deg > 1) {
                        DSH(4, SH_C2[0] * xy);
                        DSH(5, SH_C2[1] * yz);
                        DSH(6, SH_C2[2] * (2.f * zz - xx - yy));
                        DSH(7, SH_C2[3] * xz);
                        DSH(8, SH_C2[4] * (xx - yy));
                        gx += SH_C2[0] * y * SH(4) + SH_C2[2] * 2.f * -x * SH(6) + SH_C2[3] * z * SH(7) +
                              SH_C2[4] * 2.f * x * SH(8);
                        gy += SH_C2[0] * x * SH(4) + SH_C2[1] * z * SH(5) + SH_C2[2] * 2.f * -y * SH(6) +
                              SH_C2[4] * 2.f * -y * SH(8);
                        gz += SH_C2[1] * y * SH(5) + SH_C2[2] * 2.f * 2.f * z * SH(6) + SH_C2[3] * x * SH(7);
                        if (deg > 2) {
                            DSH(9, SH_C3[0] * y * (3.f * xx - yy));
                            DSH(10, SH_C3[1] * xy * z);
                            DSH(11, SH_C3[2] * y * (4.f * zz - xx - yy));
                            DSH(12, SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy));
                            DSH(13, SH_C3[4] * x * (4.f * zz - xx - yy));
                            DSH(14, SH_C3[5] * z * (xx - yy));
                            DSH(15, SH_C3[6] * x * (xx - 3.f * yy));
                            gx += SH_C3[0] * SH(9) * 3.f * 2.f * xy + SH_C3[1] * SH(10) * yz +
                                  SH_C3[2] * SH(11) * -2.f * xy + SH_C3[3] * SH(12) * -3.f * 2.f * xz +
                                  SH_C3[4] * SH(13) * (-3.f * xx + 4.f * zz - yy) +
                                  SH_C3[5] * SH(14) * 2.f * xz + SH_C3[6] * SH(15) * 3.f * (xx - yy);
                            gy += SH_C3[0] * SH(9) * 3.f * (xx - yy) + SH_C3[1] * SH(10) * xz +
                                  SH_C3[2] * SH(11) * (-3.f * yy + 4.f * zz - xx) +
                                  SH_C3[3] * SH(12) * -3.f * 2.f * yz + SH_C3[4] * SH(13) * -2.f * xy +
                                  SH_C3[5] * SH(14) * -2.f * yz + SH_C3[6] * SH(15) * -3.f * 2.f * xy;
                            gz += SH_C3[1] * SH(10) * xy + SH_C3[2] * SH(11) * 4.f * 2.f * yz +
                                  SH_C3[3] * SH(12) * 3.f * (2.f * zz - xx - yy) +
                                  SH_C3[4] * SH(13) * 4.f * 2.f * xz + SH_C3[5] * SH(14) * (xx - yy);
                        }
                    }
                    ddir[0] += gx * g;
                    ddir[1] += gy * g;
                    ddir[2] += gz * g;
                }
#undef SH
#undef DSH
            }
            /* d(v/|v|)/dv */
            float s2 = dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2];
            float inv32 = 1.f / sqrtf(s2 * s2 * s2);
            dmean[0] += ((s2 - dv[0] * dv[0]) * ddir[0] - dv[1] * dv[0] * ddir[1] - dv[2] * dv[0] * ddir[2]) * inv32;
            dmean[1] += (-dv[0] * dv[1] * ddir[0] + (s2 - dv[1] * dv[1]) * ddir[1] - dv[2] * dv[1] * ddir[2]) * inv32;
            dmean[2] += (-dv[0] * dv[2] * ddir[0] - dv[1] * dv[2] * ddir[1] + (s2 - dv[2] * dv[2]) * ddir[2]) * inv32;
        }
        /* depth output: depth_i = (W p + t).z -> dp += W[2][:] * dL/ddepth_i */
        dmean[0] += Wm[6] * g_dep[i];
        dmean[1] += Wm[7] * g_dep[i];
        dmean[2] += Wm[8] * g_dep[i];
        dL_dmeans3D[3 * i] = dmean[0];
        dL_dmeans3D[3 * i + 1] = dmean[1];
        dL_dmeans3D[3 * i + 2] = dmean[2];
        /* (4) cov3D -> (scale, rotation) */
        if (st->cov_in) {
            if (dL_dcov3D) memcpy(dL_dcov3D + 6 * i, dcov, 6 * sizeof(float));
        } else {
            const float *sc = st->scales + 3 * i;
            const float *q = st->rots + 4 * i;
            float mod = s->scale_modifier;
            float R[9];
            quat_to_R(q, R);
            float sp[3] = {mod * sc[0], mod * sc[1], mod * sc[2]};
            /* G = dL/dSigma as a symmetric matrix */
            float G[9] = {dcov[0], 0.5f * dcov[1], 0.5f * dcov[2], 0.5f * dcov[1], dcov[3],
                          0.5f * dcov[4], 0.5f * dcov[2], 0.5f * dcov[4], dcov[5]};
            /* Sigma = L L^T, L = R diag(sp): dL/dL = 2 G L */
            float L[9];
            for (int r = 0; r < 3; r++)
                for (int k = 0; k < 3; k++) L[r * 3 + k] = R[r * 3 + k] * sp[k];
            float dLm[9];
            for (int r = 0; r < 3; r++)
                for (int k = 0; k < 3; k++) {
                    float acc2 = 0.f;
                    for (int m = 0; m < 3; m++) acc2 += G[r * 3 + m] * L[m * 3 + k];
                    dLm[r * 3 + k] = 2.f * acc2;
                }
            float dRm[9];
            for (int k = 0; k < 3; k++) {
                float ds = 0.f;
                for (int r = 0; r < 3; r++) {
                    ds += dLm[r * 3 + k] * R[r * 3 + k];
                    dRm[r * 3 + k] = dLm[r * 3 + k] * sp[k];
                }
                /* upstream 3DGS computeCov3D backward returns the gradient w.r.t. the modified scale
                 * (mod * s): no factor mod here (libdgs_hip: dgs_raster_set_exact_scale_grad(0)) */
                dL_dscales[3 * i + k] = ds;
            }
            dR_dq(q, dRm, dL_drots + 4 * i);
        }
    }
    free(g_m2); free(g_dens); free(g_con); free(g_op); free(g_col); free(g_dep);
    return 0;
}

void or_free(void *p) {
    ORState *st = (ORState *)p;
    if (!st) return;
    free(st->means3D); free(st->shs); free(st->colors_in); free(st->opac); free(st->scales);
    free(st->rots); free(st->cov_in); free(st->depth); free(st->xy); free(st->conic_o);
    free(st->rgb); free(st->cov3D); free(st->radii); free(st->tiles); free(st->clamped); free(st->rgb_raw);
    free(st->keys); free(st->vals); free(st->range_lo); free(st->range_hi); free(st->final_T);
    free(st->n_contrib); free(st->radf); free(st->vz); free(st->pxy);
    free(st);
}

/* debug accessors for tests */
void or_geometry(void *p, float *xy, float *conic_o, float *rgb, float *depth, float *cov3D) {
    ORState *st = (ORState *)p;
    int N = st->N;
    if (xy) memcpy(xy, st->xy, sizeof(float) * 2 * N);
    if (conic_o) memcpy(conic_o, st->conic_o, sizeof(float) * 4 * N);
    if (rgb) memcpy(rgb, st->rgb, sizeof(float) * 3 * N);
    if (depth) memcpy(depth, st->depth, sizeof(float) * N);
    if (cov3D) memcpy(cov3D, st->cov3D, sizeof(float) * 6 * N);
}

void or_pixel_state(void *p, float *final_T, int *n_contrib) {
    ORState *st = (ORState *)p;
    size_t n = (size_t)st->s.image_height * st->s.image_width;
    if (final_T) memcpy(final_T, st->final_T, sizeof(float) * n);
    if (n_contrib) memcpy(n_contrib, st->n_contrib, sizeof(int) * n);
}

/* Per-Gaussian preprocess values behind the integer outputs (tests): radf = 3 sqrt(lambda_max)
   before the ceil (radius = ceil(radf)), vz = view-space z (culled at <= 0.2), pxy = pixel centre
   (also for Gaussians whose tile rectangle came out empty). 0 where the Gaussian was culled earlier. */
void or_preprocess_raw(void *p, float *radf, float *vz, float *pxy) {
    ORState *st = (ORState *)p;
    int N = st->N;
    if (radf) memcpy(radf, st->radf, sizeof(float) * N);
    if (vz) memcpy(vz, st->vz, sizeof(float) * N);
    if (pxy) memcpy(pxy, st->pxy, sizeof(float) * 2 * N);
}

/* Near-threshold decisions of the blend (tests). Replays every pixel's front-to-back loop and marks
   the discrete decisions whose input sits within a relative `eps` of its threshold, where two fp32
   implementations of the same math (another exp, fma contraction, exponent-form conic) may decide
   differently: the power > 0 skip (|power| <= eps), the alpha < 1/255 skip (|alpha - 1/255| <=
   eps/255), the alpha clamp at 0.99 (|o G - 0.99| <= 0.99 eps) and the T (1 - alpha) < 1e-4 stop
   (|T (1 - alpha) - 1e-4| <= 1e-4 eps). Such a decision changes the transmittance of everything
   behind it in that pixel (and whether the pixel stops there), so pflag[pixel] = 1 and every
   Gaussian listed in that pixel from the first such decision through one past the stop gets
   gflag = 1 (the Gaussians whose gradient from that pixel can differ by more than rounding).
   Returns the number of flagged pixels. */
int or_flip_flags(void *p, float eps, uint8_t *gflag, uint8_t *pflag) {
    ORState *st = (ORState *)p;
    const int H = st->s.image_height, W = st->s.image_width;
    const int T = st->grid_x * st->grid_y;
    memset(gflag, 0, (size_t)st->N);
    if (pflag) memset(pflag, 0, (size_t)H * W);
    int flagged = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : flagged)
    for (int t = 0; t < T; t++) {
        int tx = t % st->grid_x, ty = t / st->grid_x;
        const int lo = st->range_lo[t], hi = st->range_hi[t];
        for (int ly = 0; ly < BY; ly++)
            for (int lx = 0; lx < BX; lx++) {
                int px = tx * BX + lx, py = ty * BY + ly;
                if (px >= W || py >= H) continue;
                float pfx = (float)px, pfy = (float)py;
                float Tt = 1.f;
                int first = -1, stop = hi - 1;
                for (int j = lo; j < hi; j++) {
                    int g = st->vals[j];
                    float dx = st->xy[2 * g] - pfx, dy = st->xy[2 * g + 1] - pfy;
                    const float *co = st->conic_o + 4 * g;
                    float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    int near = fabsf(power) <= eps;
                    if (power > 0.f) {
                        if (near && first < 0) first = j;
                        continue;
                    }
                    float og = co[3] * expf(power);
                    float alpha = fminf(0.99f, og);
                    near |= fabsf(alpha - 1.f / 255.f) <= eps / 255.f;
                    near |= fabsf(og - 0.99f) <= 0.99f * eps;
                    if (alpha < 1.f / 255.f) {
                        if (near && first < 0) first = j;
                        continue;
                    }
                    float testT = Tt * (1.f - alpha);
                    near |= fabsf(testT - 0.0001f) <= 0.0001f * eps;
                    if (near && first < 0) first = j;
                    if (testT < 0.0001f) {
                        stop = j;
                        break;
                    }
                    Tt = testT;
                }
                if (first < 0) continue;
                flagged++;
                if (pflag) pflag[py * W + px] = 1;
                int end = stop + 1 < hi ? stop + 1 : hi - 1;
                for (int j = first; j <= end; j++) {
                    /* several threads may flag one Gaussian: an atomic store (all store 1) */
#pragma omp atomic write
                    gflag[st->vals[j]] = 1;
                }
            }
    }
    return flagged;
}

/* Near-threshold decisions of the preprocess that only switch a Gaussian's GRADIENT (its forward
   value is continuous across them), for the rendered Gaussians (tests): the frustum clamp of the EWA
   Jacobian (|t.x / t.z| within eps limx of limx = 1.3 tan(fovx / 2), or y: the x / y gradient of the
   view-space mean is zeroed past it) and the SH colour clamp at 0 (|SH colour + 0.5| <= eps: the
   colour's gradient is zeroed below it). gflag |= 1 for such Gaussians. Returns their number. */
int or_preprocess_flags(void *p, float eps, uint8_t *gflag) {
    ORState *st = (ORState *)p;
    const ORSettings *s = &st->s;
    const float limx = 1.3f * s->tanfovx, limy = 1.3f * s->tanfovy;
    int n = 0;
    for (int i = 0; i < st->N; i++) {
        if (st->radii[i] <= 0) continue;
        float tv[3];
        xform43(s->viewmatrix, st->means3D + 3 * i, tv);
        int near = fabsf(fabsf(tv[0] / tv[2]) - limx) <= eps * limx || fabsf(fabsf(tv[1] / tv[2]) - limy) <= eps * limy;
        if (!st->colors_in)
            for (int c = 0; c < 3; c++) near |= fabsf(st->rgb_raw[3 * i + c]) <= eps;
        if (near) {
            gflag[i] = 1;
            n++;
        }
    }
    return n;
}

/* Gaussians that contribute to the pixels in pmask (tests): every Gaussian listed in such a pixel's
   tile up to and including its stop that passes the power / alpha tests there. Used for pixels whose
   loss gradient itself sits at a decision (the L1 term's sign where the image equals the target within
   the image tolerance): the gradient of every Gaussian blended there can move by that pixel's share.
   gflag |= 1; returns the number of Gaussians newly flagged. */
int or_pixel_gaussians(void *p, const uint8_t *pmask, uint8_t *gflag) {
    ORState *st = (ORState *)p;
    const int H = st->s.image_height, W = st->s.image_width;
    int n = 0;
    for (int py = 0; py < H; py++)
        for (int px = 0; px < W; px++) {
            if (!pmask[py * W + px]) continue;
            const int t = (py / BY) * st->grid_x + px / BX;
            const float pfx = (float)px, pfy = (float)py;
            float Tt = 1.f;
            for (int j = st->range_lo[t]; j < st->range_hi[t]; j++) {
                int g = st->vals[j];
                float dx = st->xy[2 * g] - pfx, dy = st->xy[2 * g + 1] - pfy;
                const float *co = st->conic_o + 4 * g;
                float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                if (power > 0.f) continue;
                float alpha = fminf(0.99f, co[3] * expf(power));
                if (alpha < 1.f / 255.f) continue;
                if (!gflag[g]) n++;
                gflag[g] = 1;
                float testT = Tt * (1.f - alpha);
                if (testT < 0.0001f) break;
                Tt = testT;
            }
        }
    return n;
}
