// Differentiable tile rasterizer for MI355X (gfx950): forward + backward kernels and the C ABI
// entry points dgs_raster_forward / dgs_raster_backward / dgs_raster_ctx_free / dgs_mark_visible.
//
// Replaces diff_gaussian_rasterization._C (un-vendored submodule, .gitmodules:4-7) behind the call
// contract of gaussian_renderer/__init__.py:53-124.
//
// Pipeline (one HIP stream, all buffers in HBM, SoA per-Gaussian geometry):
//   k_preprocess   1 thread / Gaussian: cull, Sigma3D, EWA Sigma2D, conic, radius, tile rect, SH->RGB,
//                  depth key (float bits; culled -> all-ones)
//   depth sort     hipcub radix sort of the N Gaussians by depth (stable: ties in index order)
//   scan           inclusive sum of tiles_touched in depth order -> pair offsets; the pair count
//                  is copied to pinned host memory behind an event (speculative binning, below)
//   k_duplicate    emit (tile, id) pairs in depth order into the speculative capacity
//   radix sort     stable, on the tile bits only (16-bit keys): same final order as upstream's
//                  sort of (tile << 32 | depth_bits) keys over Gaussian-index-ordered pairs
//   k_ranges       [start,end) per tile (pair count read on the device)
//   k_blend_fwd    1 workgroup (4 waves) / 16x16 tile, LDS-staged 256-Gaussian batches, block-wide
//                  early exit; writes colour, depth, final T, last contributor
//   k_blend_bwd    back-to-front replay from the block's max contributor; the 12 per-Gaussian
//                  gradient sums reduce-scattered across the wave (permlane32/16 swaps + DPP) and
//                  added with 3 four-lane atomics per (wave, Gaussian)
//   k_preprocess_bwd 1 thread / Gaussian: conic->Sigma2D->(Sigma3D, mean), projection, SH, Sigma3D->(s,q)
#include <hip/hip_runtime.h>

#include <chrono>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <atomic>
#include <mutex>
#include <tuple>
#include <vector>

#include "radix.h"
#include "raster_kernels.h"

namespace dgs {

// ------------------------------------------------------------------------------------------------
// forward kernels
// ------------------------------------------------------------------------------------------------
// STAGE (M = 16, 16-byte aligned SH): the block's SH rows are read into LDS with coalesced
// 16-byte loads before any thread culls its Gaussian (see k_preprocess_bwd)
constexpr int SH_ROW = 48, SH_PAD = 49;  // odd LDS row stride: a thread-per-row access is conflict-free

// The block's nrow SH rows into LDS rows of SH_PAD floats: from one (P, 16, 3) tensor, or split
// (rest != nullptr) from features_dc (P, 1, 3) and features_rest (P, 15, 3) as the Gaussian model
// stores them (no concatenated copy). All loads are 16-byte units of contiguous row blocks, every
// load of a thread issued before its first LDS store (a rolled loop waited out one HBM round trip
// per 256 units: 12 in a row for the 256 rows of a block).
template <int MAXU>
__device__ __forceinline__ void sh_get(float *s_sh, const float *base, int rowlen, int off, int b0, int nrow) {
    const int n = nrow * rowlen;
    const float *src = base + (size_t)b0 * rowlen;
    const int nu = div_up(n, 4);
    auto put = [&](int u, const float *w) {
        int r = 4 * u / rowlen, c = 4 * u - r * rowlen;  // one division per unit, then carry
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (4 * u + j < n) s_sh[r * SH_PAD + off + c] = w[j];
            if (++c == rowlen) {
                c = 0;
                r++;
            }
        }
    };
    if (n % 4 == 0) {  // whole units (every block but possibly the tensor's last): loads first
        float4 v[MAXU];
#pragma unroll
        for (int k = 0; k < MAXU; k++) {
            const int u = threadIdx.x + 256 * k;
            if (u < nu) v[k] = reinterpret_cast<const float4 *>(src)[u];
        }
#pragma unroll
        for (int k = 0; k < MAXU; k++) {
            const int u = threadIdx.x + 256 * k;
            if (u < nu) {
                const float w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
                put(u, w);
            }
        }
        return;
    }
    for (int u = threadIdx.x; u < nu; u += 256) {
        float w[4];
        if (4 * u + 3 < n) {
            const float4 v = reinterpret_cast<const float4 *>(src)[u];
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else {  // the tensor's last partial unit: no read past its end
#pragma unroll
            for (int j = 0; j < 4; j++) w[j] = 4 * u + j < n ? src[4 * u + j] : 0.f;
        }
        put(u, w);
    }
}

__device__ __forceinline__ void sh_stage_in(float *s_sh, const float *shs, const float *rest, int b0, int nrow) {
    if (!rest) {
        sh_get<SH_ROW / 4>(s_sh, shs, SH_ROW, 0, b0, nrow);  // 256 rows x 12 units: 12 per thread
        return;
    }
    sh_get<1>(s_sh, shs, 3, 0, b0, nrow);                                  // 192 units
    sh_get<(256 * (SH_ROW - 3) / 4 + 255) / 256>(s_sh, rest, SH_ROW - 3, 3, b0, nrow);  // 2880 units
}

// LDS rows -> the (P, 16, 3) gradient, or split into the dc (P, 1, 3) / rest (P, 15, 3) gradients
__device__ __forceinline__ void sh_stage_out(const float *s_sh, float *dsh, float *drest, int b0, int nrow) {
    if (!drest) {
        float4 *dst = reinterpret_cast<float4 *>(dsh + (size_t)b0 * SH_ROW);
        for (int u = threadIdx.x; u < nrow * (SH_ROW / 4); u += 256) {
            const float *d = s_sh + (u / (SH_ROW / 4)) * SH_PAD + (u % (SH_ROW / 4)) * 4;
            dst[u] = make_float4(d[0], d[1], d[2], d[3]);
        }
        return;
    }
    auto put = [&](float *base, int rowlen, int off) {
        const int n = nrow * rowlen;
        float4 *dst = reinterpret_cast<float4 *>(base + (size_t)b0 * rowlen);
        for (int u = threadIdx.x; u < div_up(n, 4); u += 256) {
            float w[4];
            int r = 4 * u / rowlen, c = 4 * u - r * rowlen;  // one division per unit, then carry
#pragma unroll
            for (int j = 0; j < 4; j++) {
                w[j] = 4 * u + j < n ? s_sh[r * SH_PAD + off + c] : 0.f;
                if (++c == rowlen) {
                    c = 0;
                    r++;
                }
            }
            if (4 * u + 3 < n) {
                dst[u] = make_float4(w[0], w[1], w[2], w[3]);
            } else {
                for (int j = 0; 4 * u + j < n; j++) base[(size_t)b0 * rowlen + 4 * u + j] = w[j];
            }
        }
    };
    put(dsh, 3, 0);
    put(drest, SH_ROW - 3, 3);
}

template <bool STAGE>
__global__ __launch_bounds__(256) void k_preprocess(
    int P, int D, int M, const float *__restrict__ means3D, const float *__restrict__ scales, float mod,
    const float *__restrict__ rots, const float *__restrict__ cov_pre, const float *__restrict__ opac,
    const float *__restrict__ shs, const float *__restrict__ shs_rest, const float *__restrict__ colors_pre,
    const float *view, const float *proj, const float *campos, int W, int H, float tanx, float tany, float fx, float fy,
    int gx, int gy, int *__restrict__ radii, float2 *__restrict__ xy, float4 *__restrict__ conic_o,
    float4 *__restrict__ rgbd, uint32_t *__restrict__ tiles, uint8_t *__restrict__ clamped,
    uint32_t *__restrict__ dkey, uint32_t *__restrict__ gid, float4 *__restrict__ acc,
    uint8_t *__restrict__ visible) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < P;
    // every per-Gaussian input is in flight with the SH rows (one HBM round trip per block instead of
    // a chain of them: camera -> mean -> cull -> scale / rotation; the grid is ~1.5 blocks per CU)
    float3 p = make_float3(0.f, 0.f, 0.f), s = p;
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    float op = 0.f;
    if (live) {
        p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
        if (!cov_pre) {
            s = make_float3(scales[3 * i], scales[3 * i + 1], scales[3 * i + 2]);
            q = *reinterpret_cast<const float4 *>(rots + 4 * i);
        }
        op = opac[i];
    }
    Cam cam;
    load_cam(cam, view, proj, campos);
    [[maybe_unused]] const float *s_row = nullptr;
    if constexpr (STAGE) {
        __shared__ float s_sh[256 * SH_PAD];
        const int b0 = blockIdx.x * blockDim.x, nrow = min(256, P - b0);
        sh_stage_in(s_sh, shs, shs_rest, b0, nrow);
        __syncthreads();
        s_row = s_sh + threadIdx.x * SH_PAD;
    }
    if (!live) return;
    // zero this Gaussian's backward accumulator row (the blend backward adds into it): no memset
    // launch in the backward
    acc[3 * i] = acc[3 * i + 1] = acc[3 * i + 2] = make_float4(0.f, 0.f, 0.f, 0.f);
    radii[i] = 0;
    if (visible) visible[i] = 0;  // render()'s visibility_filter (radii > 0), when asked for
    tiles[i] = 0;
    dkey[i] = 0xffffffffu;  // culled: sorts last, emits no pairs
    gid[i] = (uint32_t)i;
    float3 pv = xform43(cam.v, p);
    if (pv.z <= 0.2f) return;
    float c3[6];
    if (cov_pre) {
#pragma unroll
        for (int k = 0; k < 6; k++) c3[k] = cov_pre[6 * i + k];
    } else {
        cov3d(s, mod, q, c3);
    }
    Ewa e;
    ewa_T(pv, fx, fy, tanx, tany, cam.v, e);
    float3 c2 = cov2d(e, c3);
    float det = c2.x * c2.z - c2.y * c2.y;
    if (det == 0.f) return;
    float di = 1.f / det;
    float3 con = make_float3(c2.z * di, -c2.y * di, c2.x * di);
    float mid = 0.5f * (c2.x + c2.z);
    float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    int rad = (int)ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    float4 ph = xform44(cam.p, p);
    float pw = 1.f / (ph.w + 0.0000001f);
    float px = ((ph.x * pw + 1.f) * W - 1.f) * 0.5f;
    float py = ((ph.y * pw + 1.f) * H - 1.f) * 0.5f;
    int x0, y0, x1, y1;
    tile_rect(px, py, rad, gx, gy, x0, y0, x1, y1);
    int area = (x1 - x0) * (y1 - y0);
    if (area == 0) return;
    float3 rgb;
    uint8_t cl = 0;
    if (colors_pre) {
        rgb = make_float3(colors_pre[3 * i], colors_pre[3 * i + 1], colors_pre[3 * i + 2]);
    } else {
        float dx = p.x - cam.c[0], dy = p.y - cam.c[1], dz = p.z - cam.c[2];
        float n = sqrtf(dx * dx + dy * dy + dz * dz);
        float x = dx / n, y = dy / n, z = dz / n;
        const float *sh = STAGE ? s_row : shs + (size_t)i * M * 3;
        float r[3];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            float v = SH_C0 * sh[c];
            if (D > 0) {
                v = v - SH_C1 * y * sh[3 + c] + SH_C1 * z * sh[6 + c] - SH_C1 * x * sh[9 + c];
                if (D > 1) {
                    float xx = x * x, yy = y * y, zz = z * z, xy_ = x * y, yz = y * z, xz = x * z;
                    v = v + SH_C2_0 * xy_ * sh[12 + c] + SH_C2_1 * yz * sh[15 + c] +
                        SH_C2_2 * (2.f * zz - xx - yy) * sh[18 + c] + SH_C2_3 * xz * sh[21 + c] +
                        SH_C2_4 * (xx - yy) * sh[24 + c];
                    if (D > 2) {
                        v = v + SH_C3_0 * y * (3.f * xx - yy) * sh[27 + c] + SH_C3_1 * xy_ * z * sh[30 + c] +
                            SH_C3_2 * y * (4.f * zz - xx - yy) * sh[33 + c] +
                            SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy) * sh[36 + c] +
                            SH_C3_4 * x * (4.f * zz - xx - yy) * sh[39 + c] +
                            SH_C3_5 * z * (xx - yy) * sh[42 + c] + SH_C3_6 * x * (xx - 3.f * yy) * sh[45 + c];
                    }
                }
            }
            v += 0.5f;
            cl |= (v < 0.f) << c;
            r[c] = v < 0.f ? 0.f : v;
        }
        rgb = make_float3(r[0], r[1], r[2]);
    }
    radii[i] = rad;
    if (visible) visible[i] = rad > 0;
    xy[i] = make_float2(px, py);
    conic_o[i] = make_float4(con.x, con.y, con.z, op);
    rgbd[i] = make_float4(rgb.x, rgb.y, rgb.z, pv.z);
    tiles[i] = (uint32_t)area;
    clamped[i] = cl;
    dkey[i] = __float_as_uint(pv.z);  // depth > 0.2: float bits order as the values
}

// Pairs are emitted in depth order (Gaussians pre-sorted by depth, stable on the index), so a
// stable sort on the tile id alone yields the reference's (tile, depth) key order, ties on the
// Gaussian index included: 2 radix passes over 16-bit keys instead of 6 over 64-bit ones.
__global__ __launch_bounds__(256) void k_gather_tiles(int P, const uint32_t *__restrict__ order,
                                                      const uint32_t *__restrict__ tiles,
                                                      uint32_t *__restrict__ tiles_sorted) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < P) tiles_sorted[j] = tiles[order[j]];
}

template <class KT>
__global__ __launch_bounds__(256) void k_duplicate(int P, const uint32_t *__restrict__ order,
                                                   const float2 *__restrict__ xy, const int *__restrict__ radii,
                                                   const uint32_t *__restrict__ offsets, int gx, int gy,
                                                   KT *__restrict__ keys, uint32_t *__restrict__ vals, uint32_t cap,
                                                   uint2 *__restrict__ ranges, int T) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    // folded fills (no separate memsets): empty tile ranges, and all-ones keys over the
    // speculative capacity past the pair count so the radix sort leaves the padding at the end
    const int nthreads = gridDim.x * blockDim.x;
    for (int t = j; t < T; t += nthreads) ranges[t] = make_uint2(0u, 0u);
    for (uint32_t k = offsets[P - 1] + (uint32_t)j; k < cap; k += (uint32_t)nthreads) keys[k] = (KT)~(KT)0;
    if (j >= P) return;
    const uint32_t g = order[j];
    const int r = radii[g];
    if (r <= 0) return;
    uint32_t off = (j == 0) ? 0u : offsets[j - 1];
    const float2 c = xy[g];
    int x0, y0, x1, y1;
    tile_rect(c.x, c.y, r, gx, gy, x0, y0, x1, y1);
    for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++) {
            if (off < cap) {  // speculative capacity: an overflowing launch is redone by the host
                keys[off] = (KT)(y * gx + x);
                vals[off] = g;
            }
            off++;
        }
}

// ------------------------------------------------------------------------------------------------
// Rect binning (the default for images up to RECT_MAX_TILES tiles): the (tile, Gaussian) pairs are
// placed directly at their position in the tile-sorted order instead of being emitted and radix-
// sorted. The Gaussians are already in depth order (stable on the index), and Gaussian j covers the
// tile rectangle of its 3-sigma radius, so the position of pair (j, t) in the stable tile sort is
//   tile_start[t] + #{j' < j : t in rect(j')}
// counted hierarchically over blocks of 256 depth-ordered Gaussians: k_rect_count (per block and
// tile), k_rect_colscan (exclusive down each tile's column of blocks, tile totals, pair count; its
// last workgroup scans the totals into the tile starts and ranges), k_rect_place (per wave and tile in
// LDS, then the lanes below in the wave). Same order as the sort, bit for bit; no keys.
// ------------------------------------------------------------------------------------------------
constexpr int RECT_MAX_TILES = 12288;     // LDS of the count/place kernels: 4 B per tile (<= 64 KiB)
constexpr long long RECT_MAX_CELLS = 1 << 24;  // blocks x tiles of the count matrix

__device__ inline bool gauss_rect(uint32_t g, const float2 *xy, const int *radii, int gx, int gy, int4 &rc) {
    const int r = radii[g];
    if (r <= 0) return false;
    const float2 c = xy[g];
    tile_rect(c.x, c.y, r, gx, gy, rc.x, rc.y, rc.z, rc.w);
    return rc.x < rc.z && rc.y < rc.w;
}

__global__ __launch_bounds__(256) void k_rect_count(int P, const uint32_t *__restrict__ order, const float2 *__restrict__ xy,
                                                    const int *__restrict__ radii, int gx, int gy,
                                                    uint32_t *__restrict__ cnt, uint32_t *__restrict__ total,
                                                    uint32_t *__restrict__ maxtodo) {
    extern __shared__ uint32_t h[];  // [T]  (total[0] = pair count, total[1] = column-scan ticket)
    const int T = gx * gy;
    for (int t = threadIdx.x; t < T; t += 256) h[t] = 0;
    if (blockIdx.x == 0 && threadIdx.x < 2) total[threadIdx.x] = 0;  // k_rect_colscan adds into them
    if (maxtodo && blockIdx.x == 0 && threadIdx.x == 0) *maxtodo = 0;  // k_blend_fwd maxes into it
    __syncthreads();
    const int j = blockIdx.x * 256 + threadIdx.x;
    int4 rc;
    if (j < P && gauss_rect(order ? order[j] : (uint32_t)j, xy, radii, gx, gy, rc))
        for (int y = rc.y; y < rc.w; y++)
            for (int x = rc.x; x < rc.z; x++) atomicAdd(&h[y * gx + x], 1u);
    __syncthreads();
    uint32_t *row = cnt + (size_t)blockIdx.x * T;
    for (int t = threadIdx.x; t < T; t += 256) row[t] = h[t];
}

// tile starts = exclusive scan of the tile totals, and the (unclipped) ranges; one workgroup of
// 1024 threads (the column scan's last workgroup). The totals come as agent-scope atomic words
// tagged with the launch generation (written by the other workgroups, no fences): spin on the tag.
__device__ inline uint32_t tagged_total(const unsigned long long *tot, int t, uint32_t gen) {
    unsigned long long v;
    do {
        v = __hip_atomic_load(tot + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } while ((uint32_t)(v >> 32) != gen);
    return (uint32_t)v;
}

__device__ void rect_starts(int T, const unsigned long long *__restrict__ tot, uint32_t gen, uint32_t *__restrict__ tile_start,
                            uint2 *__restrict__ ranges, uint32_t *wsum, uint32_t *host_total) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int MAXPER = 12;  // RECT_MAX_TILES / 1024
    const int per = div_up(T, 1024);
    const int t0 = tid * per;
    uint32_t c[MAXPER], local = 0;
#pragma unroll
    for (int k = 0; k < MAXPER; k++) {
        c[k] = (k < per && t0 + k < T) ? tagged_total(tot, t0 + k, gen) : 0u;
        local += c[k];
    }
    uint32_t x = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t run = x - local;
    for (int k = 0; k < w; k++) run += wsum[k];
#pragma unroll
    for (int k = 0; k < MAXPER; k++) {
        const int t = t0 + k;
        if (k < per && t < T) {
            tile_start[t] = run;
            ranges[t] = make_uint2(run, run + c[k]);
            run += c[k];
        }
    }
    // the pair count straight into the host's pinned word (no copy launch): the last thread's run
    if (host_total && tid == 1023) *host_total = run;
}

// the column of block counts of 64 tiles per workgroup -> exclusive offsets (in place), the tile
// totals, the pair count, then the tile starts and ranges (last workgroup): 16 waves take 32 rows each per 512-row chunk (loads all in flight),
// cross-wave prefix in LDS, carry between chunks
__global__ __launch_bounds__(1024) void k_rect_colscan(int nb, int T, uint32_t *__restrict__ cnt, unsigned long long *__restrict__ tot, uint32_t gen,
                                                       uint32_t *__restrict__ total, uint32_t *__restrict__ ticket,
                                                       uint32_t *__restrict__ tile_start, uint2 *__restrict__ ranges,
                                                       uint32_t *host_total) {
    __shared__ uint32_t part[16][64];
    __shared__ uint32_t carry[64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int t = blockIdx.x * 64 + lane;
    const bool ok = t < T;
    if (w == 0) carry[lane] = 0;
    for (int b0 = 0; b0 < nb; b0 += 512) {
        const int r0 = b0 + 32 * w;
        uint32_t v[32], sum = 0;
#pragma unroll
        for (int k = 0; k < 32; k++) {
            v[k] = (ok && r0 + k < nb) ? cnt[(size_t)(r0 + k) * T + t] : 0u;
            sum += v[k];
        }
        part[w][lane] = sum;
        __syncthreads();
        uint32_t run = carry[lane];
        for (int k = 0; k < w; k++) run += part[k][lane];
#pragma unroll
        for (int k = 0; k < 32; k++) {
            if (ok && r0 + k < nb) cnt[(size_t)(r0 + k) * T + t] = run;
            run += v[k];
        }
        __syncthreads();  // carry and part read by every wave
        if (w == 15) carry[lane] = run;
        __syncthreads();
    }
    if (w == 0) {
        const uint32_t c = carry[lane];
        if (ok) __hip_atomic_store(tot + t, ((unsigned long long)gen << 32) | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t s = c;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += (uint32_t)__shfl_xor((int)s, o);
        if (lane == 0) atomicAdd(total, s);
    }
    // the last workgroup to take a ticket scans the tile totals
    __shared__ uint32_t wsum[16];
    __shared__ bool last;
    if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    rect_starts(T, tot, gen, tile_start, ranges, wsum, host_total);
}

__host__ __device__ inline size_t rect_place_lds(int gx, int gy, bool stage) {
    return 4ull * ((gx * gy + 1) & ~1) * (stage ? 2 : 1) + 4ull * 8ull * (gx + gy);
}
// the block's output base per tile (tile start + the block's column offset) staged in LDS when it fits
__host__ __device__ inline bool rect_place_stage(int gx, int gy) { return rect_place_lds(gx, gy, true) <= 65536; }

// The pair positions of one block of depth-ordered Gaussians (one per thread): per wave and tile the
// lanes' counts packed one byte each, per wave the lanes whose rectangle spans each tile column / row; a
// pair's position is the tile start + the block's column offset + the waves below + its rank among the
// wave's lanes. f(g, t, pos) is called per covered tile t in row-major order (k_rect_place writes the
// list, k_rect_gather sums the deterministic blend backward's per-pair slots).
template <class F>
__device__ __forceinline__ void rect_walk(int P, const uint32_t *__restrict__ order, const float2 *__restrict__ xy,
                                          const int *__restrict__ radii, int gx, int gy,
                                          const uint32_t *__restrict__ cnt, const uint32_t *__restrict__ tile_start,
                                          int stage, uint32_t *lds, F &&f) {
    const int T = gx * gy, G = gx + gy;
    // per tile, the four waves' counts packed one byte each (a wave adds at most 64 per tile)
    const int Tp = (T + 1) & ~1;
    uint32_t *wc = lds;  // [T]
    // stage: the block's first output position per tile (tile start + this block's column offset),
    // read coalesced once instead of gathered per pair
    uint32_t *base = lds + Tp;  // [T] (stage)
    // per wave, the lanes whose rectangle spans tile column x ([x]) / tile row y ([gx + y])
    unsigned long long *span = reinterpret_cast<unsigned long long *>(lds + (stage ? 2 * Tp : Tp));  // [4][G]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t *crow = cnt + (size_t)blockIdx.x * T;
    for (int t = tid; t < T; t += 256) wc[t] = 0;
    if (stage)
        for (int t = tid; t < T; t += 256) base[t] = tile_start[t] + crow[t];
    for (int t = tid; t < 4 * G; t += 256) span[t] = 0ull;
    const int j = blockIdx.x * 256 + tid;
    // order == nullptr: index order (the per-tile sort orders each list by depth afterwards)
    const uint32_t g = j < P ? (order ? order[j] : (uint32_t)j) : 0u;
    int4 rc = make_int4(0, 0, 0, 0);
    if (j < P && !gauss_rect(g, xy, radii, gx, gy, rc)) rc = make_int4(0, 0, 0, 0);
    __syncthreads();
    unsigned long long *ws = span + w * G;
    const unsigned long long me = 1ull << lane;
    for (int x = rc.x; x < rc.z; x++) atomicOr(&ws[x], me);
    for (int y = rc.y; y < rc.w; y++) {
        atomicOr(&ws[gx + y], me);
        for (int x = rc.x; x < rc.z; x++) atomicAdd(&wc[y * gx + x], 1u << (8 * w));
    }
    __syncthreads();
    for (int y = rc.y; y < rc.w; y++) {
        const unsigned long long rows = ws[gx + y] & (me - 1ull);  // lanes below spanning row y
        for (int x = rc.x; x < rc.z; x++) {
            const int t = y * gx + x;
            const uint32_t rank = (uint32_t)__popcll(rows & ws[x]);
            // waves below: byte w-1 of the packed inclusive sums (partial sums <= 192, no carries)
            const uint32_t below = w ? ((wc[t] * 0x01010101u) >> (8 * (w - 1))) & 0xffu : 0u;
            f(g, t, (stage ? base[t] : tile_start[t] + crow[t]) + below + rank);
        }
    }
}

__global__ __launch_bounds__(256) void k_rect_place(int P, const uint32_t *__restrict__ order, const float2 *__restrict__ xy,
                                                    const int *__restrict__ radii, int gx, int gy,
                                                    const uint32_t *__restrict__ cnt, const uint32_t *__restrict__ tile_start,
                                                    uint32_t cap, uint32_t *__restrict__ vals, int stage) {
    extern __shared__ uint32_t lds[];
    // (writing each pair's depth key beside it here, for k_tile_sort to read coalesced, made this kernel
    // 15 us slower per step at the bench size, more than the gather it saved)
    rect_walk(P, order, xy, radii, gx, gy, cnt, tile_start, stage, lds, [&](uint32_t g, int, uint32_t pos) {
        if (pos < cap) vals[pos] = g;
    });
}

// Deterministic blend backward (dgs_raster_set_deterministic): k_blend_bwd2<DEPTH, true> leaves every
// pair of the replayed lists one 12-float slot (the pair's reduced sums in the accumulator row's field
// order, zeros for a pair the tile culled or both waves skipped) instead of adding them into acc with
// float atomics. This gather walks the same rectangles as k_rect_place (in its order: Gaussian index
// with the per-tile sort, whose position map takes each walked pair to its sorted list position; depth
// order without it), one thread per Gaussian, and sums its pairs' slots in tile row-major order: a fixed
// order, so acc (and every gradient after it) is bitwise reproducible. A pair past the launched
// capacity is skipped; one past its tile's replayed prefix holds zeros: neither adds anything, exactly
// as with the atomics. Every row of acc is written (zeros for a Gaussian without a rectangle).
__global__ __launch_bounds__(256) void k_rect_gather(int P, const uint32_t *__restrict__ order, const float2 *__restrict__ xy,
                                                     const int *__restrict__ radii, int gx, int gy,
                                                     const uint32_t *__restrict__ cnt, const uint32_t *__restrict__ tile_start,
                                                     uint32_t cap, const float4 *__restrict__ slot, float *__restrict__ acc,
                                                     int stage) {
    extern __shared__ uint32_t lds[];
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 s0 = z4, s1 = z4, s2 = z4;
    // one pair behind: a pair's slot loads are added at the next pair, so their latency overlaps the
    // walk to the next pair (same order of additions)
    float4 pa = z4, pb = z4, pc = z4;
    rect_walk(P, order, xy, radii, gx, gy, cnt, tile_start, stage, lds, [&](uint32_t, int, uint32_t pos) {
        float4 na = z4, nb = z4, nc = z4;
        if (pos < cap) {
            const float4 *q = slot + 3ull * pos;
            na = q[0];
            nb = q[1];
            nc = q[2];
        }
        s0 = s0 + pa;
        s1 = s1 + pb;
        s2 = s2 + pc;
        pa = na;
        pb = nb;
        pc = nc;
    });
    s0 = s0 + pa;
    s1 = s1 + pb;
    s2 = s2 + pc;
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= P) return;
    // (order == nullptr: the index-order walk of the per-tile sort's placement)
    float4 *dst = reinterpret_cast<float4 *>(acc + (size_t)(order ? order[j] : (uint32_t)j) * ACC_STRIDE);
    dst[0] = s0;
    dst[1] = s1;
    dst[2] = s2;
}

// Per-tile depth sort (rect binning, the default; DGS_TILE_SORT=0 restores the global depth sort): the
// count / place kernels run over the Gaussians in index order, so every tile's list comes out in index
// order, and each list is then sorted stably by its 32-bit depth key, i.e. by (depth, index): exactly
// the order the global stable depth sort produced. The lists, and everything computed from them, are
// bit-identical. k_tile_sort: one workgroup per tile, a stable LSD radix sort of up to TS_MAX entries
// in LDS — 8-bit digits, in-wave ranking by one ballot per digit bit (as radix.hip's passes), per-wave
// digit offsets from one block scan, scatter through LDS — skipping the passes whose digit is the same
// for every key of the tile (the depth exponent byte, typically). Per entry and pass that is ~15 VALU;
// a bitonic network in registers measured 37 us per step at the bench size (~55 exchange stages of
// 64-bit keys at E = 16 per lane), one in LDS 42 us, counting ranks from LDS 66 us (O(L^2)). A list
// longer than TS_MAX is sorted as TS_MAX-long runs into scratch as (depth << 32 | index) keys, then each
// entry's position = its index in its run + its lower bound in every other run (binary search, the run
// staged in LDS).
constexpr int TS_MAX = 1024;  // (2048: no faster at the bench size, whose longest list is 591)
constexpr int TS_THR = 256;
struct TileSortLds {
    union {
        struct {
            uint32_t key[TS_MAX], val[TS_MAX];
        } kv;
        unsigned long long run[TS_MAX];  // a long list's merge: one sorted run staged
    } u;
    uint32_t cnt[4][256];  // per-wave digit counts -> per-wave output offsets
    uint16_t opos[TS_MAX];  // POS: each sorted entry's position in the index-ordered list
    uint32_t misc[8];
};

// sorts the m <= TS_MAX entries ids[0, m) (index order) stably by dkey[id]; returns the number of passes
// run (0: the order is unchanged) with the sorted (key, id) pairs in L.u.kv
// POS (the deterministic backward): L.opos carries each entry's position in the input list along
template <int NI, bool POS>
__device__ __forceinline__ int ts_block_radix(TileSortLds &L, const uint32_t *ids, int m, const uint32_t *__restrict__ dkey,
                                              int tid) {
    const int lane = tid & 63, w = tid >> 6, base = w * 64 * NI;
    const uint64_t lanes_lt = (1ull << lane) - 1ull;
    uint32_t key[NI], val[NI];
    [[maybe_unused]] uint32_t opos[NI];
    if constexpr (POS) {
#pragma unroll
        for (int r = 0; r < NI; r++) opos[r] = (uint32_t)(base + 64 * r + lane);
    }
    uint32_t kor = 0u, kand = ~0u;
#pragma unroll
    for (int r = 0; r < NI; r++) {
        const int i = base + 64 * r + lane;
        val[r] = i < m ? ids[i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < NI; r++) {
        const int i = base + 64 * r + lane;
        key[r] = i < m ? dkey[val[r]] : 0u;
        if (i < m) {
            kor |= key[r];
            kand &= key[r];
        }
    }
    // the bits that differ between keys: a pass over a byte none of them has runs for nothing. Wave OR /
    // AND in DPP (row shifts, then the row broadcasts: lane 63 holds the wave's), combined across the
    // four waves in LDS (LDS atomics from every lane on one word cost 10 us per step at the bench size)
    {
        int o = (int)kor, n = (int)kand;
        o |= __builtin_amdgcn_update_dpp(0, o, 0x111, 0xf, 0xf, false);
        n &= __builtin_amdgcn_update_dpp(-1, n, 0x111, 0xf, 0xf, false);
        o |= __builtin_amdgcn_update_dpp(0, o, 0x112, 0xf, 0xf, false);
        n &= __builtin_amdgcn_update_dpp(-1, n, 0x112, 0xf, 0xf, false);
        o |= __builtin_amdgcn_update_dpp(0, o, 0x114, 0xf, 0xf, false);
        n &= __builtin_amdgcn_update_dpp(-1, n, 0x114, 0xf, 0xf, false);
        o |= __builtin_amdgcn_update_dpp(0, o, 0x118, 0xf, 0xf, false);
        n &= __builtin_amdgcn_update_dpp(-1, n, 0x118, 0xf, 0xf, false);
        o |= __builtin_amdgcn_update_dpp(0, o, 0x142, 0xa, 0xf, false);
        n &= __builtin_amdgcn_update_dpp(-1, n, 0x142, 0xa, 0xf, false);
        o |= __builtin_amdgcn_update_dpp(0, o, 0x143, 0xc, 0xf, false);
        n &= __builtin_amdgcn_update_dpp(-1, n, 0x143, 0xc, 0xf, false);
        if (lane == 63) {
            L.misc[2 * w] = (uint32_t)o;
            L.misc[2 * w + 1] = (uint32_t)n;
        }
    }
    __syncthreads();
    uint32_t kor4 = 0u, kand4 = ~0u;
#pragma unroll
    for (int ww = 0; ww < 4; ww++) {
        kor4 |= L.misc[2 * ww];
        kand4 &= L.misc[2 * ww + 1];
    }
    __syncthreads();  // misc is reused by the passes' scans
#ifdef TS_DIAG_PASSES  // diagnostic builds (tools/build_diag.sh): at most this many passes (wrong order)
    const uint32_t diff = TS_DIAG_PASSES == 0 ? 0u : (kor4 ^ kand4) & (0xffffffffu >> (32 - 8 * (TS_DIAG_PASSES + (TS_DIAG_PASSES == 0))));  // wrong order
#else
    const uint32_t diff = kor4 ^ kand4;
#endif
    int passes = 0;
    for (int shift = 0; shift < 32; shift += 8) {
        if (((diff >> shift) & 255u) == 0u) continue;  // workgroup-uniform
        passes++;
#pragma unroll
        for (int ww = 0; ww < 4; ww++) L.cnt[ww][tid] = 0;
        __syncthreads();
        uint32_t rank[NI];
#pragma unroll
        for (int r = 0; r < NI; r++) {
            const bool ok = base + 64 * r + lane < m;
            const uint32_t d = (key[r] >> shift) & 255u;
            // lanes holding the same digit: the ones where no digit bit differs from this lane's
            // (mismatch bits OR-ed per 32-lane half: one 3-input bit op per half and bit)
            const uint64_t okm = __ballot(ok);
            uint32_t xlo = ~(uint32_t)okm, xhi = ~(uint32_t)(okm >> 32);
#pragma unroll
            for (int bb = 0; bb < 8; bb++) {
                const uint64_t bal = __ballot((d >> bb) & 1u);
                const uint32_t t = (uint32_t)((int32_t)(d << (31 - bb)) >> 31);  // the bit, sign-extended
                xlo |= (uint32_t)bal ^ t;
                xhi |= (uint32_t)(bal >> 32) ^ t;
            }
            const uint64_t mk = ~(((uint64_t)xhi << 32) | xlo);
            const int leader = mk ? __ffsll((unsigned long long)mk) - 1 : 0;
            // every lane of a digit group reads the group's count before its leader advances it (the
            // wave's LDS operations complete in order): no broadcast from the leader needed
            const uint32_t b0 = ok ? L.cnt[w][d] : 0u;
            if (ok && lane == leader) L.cnt[w][d] = b0 + (uint32_t)__popcll(mk);
            rank[r] = b0 + (uint32_t)__popcll(mk & lanes_lt);
        }
        __syncthreads();
        {
            const int d = tid;  // one thread per digit: per-wave offsets, then the digit starts
            uint32_t c[4], tot = 0;
#pragma unroll
            for (int ww = 0; ww < 4; ww++) {
                c[ww] = L.cnt[ww][d];
                tot += c[ww];
            }
            // inclusive wave scan in DPP: row shifts 1/2/4/8, then the row broadcasts 15 / 31
            int x = (int)tot;
            x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
            x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
            x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
            x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
            x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
            x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
            if (lane == 63) L.misc[w] = (uint32_t)x;
            __syncthreads();
            uint32_t start = (uint32_t)x - tot;
            for (int ww = 0; ww < w; ww++) start += L.misc[ww];
#pragma unroll
            for (int ww = 0; ww < 4; ww++) {
                L.cnt[ww][d] = start;
                start += c[ww];
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < NI; r++) {
            if (base + 64 * r + lane < m) {
                const uint32_t dst = L.cnt[w][(key[r] >> shift) & 255u] + rank[r];
                L.u.kv.key[dst] = key[r];
                L.u.kv.val[dst] = val[r];
                if constexpr (POS) L.opos[dst] = (uint16_t)opos[r];
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < NI; r++) {
            const int i = base + 64 * r + lane;
            if (i < m) {
                key[r] = L.u.kv.key[i];
                val[r] = L.u.kv.val[i];
                if constexpr (POS) opos[r] = L.opos[i];
            }
        }
    }
    return passes;
}
template <bool POS = false>
__device__ __forceinline__ int ts_block_any(TileSortLds &L, const uint32_t *ids, int m, const uint32_t *__restrict__ dkey,
                                            int tid) {
    if (m <= 256) return ts_block_radix<1, POS>(L, ids, m, dkey, tid);
    if (m <= 512) return ts_block_radix<2, POS>(L, ids, m, dkey, tid);
    return ts_block_radix<4, POS>(L, ids, m, dkey, tid);
}

// pre (the deterministic backward, or nullptr): pre[a + p] = the position q, in the index-ordered list
// k_rect_place wrote, of the entry the sort put at position p (the backward leaves the pair's sums at
// a + q, where k_rect_gather's index-order walk finds them); vorig: scratch for the long-list path's
// copy of that list
template <bool PRE>
__global__ __launch_bounds__(TS_THR) void k_tile_sort(const uint2 *__restrict__ ranges, uint32_t cap,
                                                      const uint32_t *__restrict__ dkey, uint32_t *__restrict__ vals,
                                                      unsigned long long *__restrict__ scratch,
                                                      uint32_t *__restrict__ spos, uint32_t *__restrict__ pre,
                                                      uint32_t *__restrict__ vorig) {
    __shared__ TileSortLds L;
    const int tid = threadIdx.x;
    const uint2 rg = ranges[blockIdx.x];
    const uint32_t a = min(rg.x, cap), b = min(rg.y, cap);
    const int len = (int)(b - a);
    if (PRE && len == 1 && tid == 0) pre[a] = 0u;
    if (len <= 1) return;
    uint32_t *v = vals + a;
    if (len <= TS_MAX) {
        // every entry is read (into registers) before the first barrier; written back after the sort
        if (ts_block_any<PRE>(L, v, len, dkey, tid) == 0) {
            if constexpr (PRE)
                for (int i = tid; i < len; i += TS_THR) pre[a + i] = (uint32_t)i;
            return;
        }
        for (int i = tid; i < len; i += TS_THR) {
            v[i] = L.u.kv.val[i];
            if constexpr (PRE) pre[a + i] = L.opos[i];
        }
        return;
    }
    // a long list: TS_MAX-long runs sorted into scratch as (depth << 32 | index), then merged by rank
    unsigned long long *sc = scratch + a;
    uint32_t *ps = spos + a;
    if constexpr (PRE)  // the index-ordered list, kept for the positions (the list is overwritten below)
        for (int i = tid; i < len; i += TS_THR) vorig[a + i] = v[i];
    for (int c0 = 0; c0 < len; c0 += TS_MAX) {
        const int m = min(TS_MAX, len - c0);
        __syncthreads();  // L is reused
        if (ts_block_any(L, v + c0, m, dkey, tid) == 0) {  // all keys equal: the run is in index order
            for (int i = tid; i < m; i += TS_THR) {
                const uint32_t g = v[c0 + i];
                sc[c0 + i] = ((unsigned long long)dkey[g] << 32) | g;
            }
        } else {
            for (int i = tid; i < m; i += TS_THR) sc[c0 + i] = ((unsigned long long)L.u.kv.key[i] << 32) | L.u.kv.val[i];
        }
        for (int i = tid; i < m; i += TS_THR) ps[c0 + i] = (uint32_t)i;  // its rank in its own run
    }
    __threadfence();
    __syncthreads();
    // per run q staged in LDS: every entry of the other runs adds its lower bound in q
    for (int q0 = 0; q0 < len; q0 += TS_MAX) {
        const int mq = min(TS_MAX, len - q0);
        __syncthreads();  // the previous run's searches are done
        for (int i = tid; i < mq; i += TS_THR) L.u.run[i] = __hip_atomic_load(sc + q0 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        for (int i = tid; i < len; i += TS_THR) {
            if (i >= q0 && i < q0 + mq) continue;
            const unsigned long long k = __hip_atomic_load(sc + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int lo = 0, hi = mq;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (L.u.run[mid] < k) lo = mid + 1;
                else hi = mid;
            }
            ps[i] += (uint32_t)lo;  // this thread's own entry
        }
    }
    // every list entry was read in the run phase: the list is overwritten in place
    for (int i = tid; i < len; i += TS_THR) {
        const uint32_t g = (uint32_t)__hip_atomic_load(sc + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v[ps[i]] = g;
        if constexpr (PRE) {  // g's position in the index-ordered (ascending id) list
            int lo = 0, hi = len;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (__hip_atomic_load(vorig + a + mid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < g) lo = mid + 1;
                else hi = mid;
            }
            pre[a + ps[i]] = (uint32_t)lo;
        }
    }
}

// L (the pair count) is read on the device and clipped to the launched capacity: an overflowing
// speculative launch (count > cap) then covers exactly the cap sorted pairs it wrote, never the
// padding or stale slots past them, and every range stays inside [0, cap); the host redoes the
// whole binning at the exact size afterwards.
template <class KT>
__global__ __launch_bounds__(256) void k_ranges(const uint32_t *__restrict__ count, uint32_t cap,
                                                const KT *__restrict__ keys, uint2 *__restrict__ ranges) {
    int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int L = (int)min(*count, cap);
    if (idx >= L) return;
    uint32_t t = (uint32_t)keys[idx];
    if (idx == 0) {
        ranges[t].x = 0;
    } else {
        uint32_t prev = (uint32_t)keys[idx - 1];
        if (t != prev) {
            ranges[prev].y = idx;
            ranges[t].x = idx;
        }
    }
    if (idx == L - 1) ranges[t].y = L;
}

// Tile culling of a staged batch (blend fwd / bwd): a Gaussian of the tile's list whose
// alpha >= 1/255 ellipse misses every pixel centre of the tile is skipped by every pixel anyway
// (alpha < 1/255 -> `continue`), so the batch is compacted to the Gaussians that can reach the tile
// before the per-pixel loop. alpha = min(0.99, o exp(-Q/2)) with Q = c_x dx^2 + 2 c_y dx dy + c_z dy^2
// (the blend's power): a pixel can take part only if Q <= 2 ln(255 o). The minimum of the convex Q
// over the tile's pixel-centre rectangle is 0 when the centre is inside, else on an edge at the
// clamped 1-D stationary point. The bound is widened by 1 % + 1e-3 so the fp32 rounding of either
// side can never cull a contributor: images and gradients are unchanged (the list positions kept in
// n_contrib are those of the full list).
// min over the pixel-centre rectangle [x0, x1] x [y0, y1] of the conic's quadratic form <= thr
__device__ __forceinline__ bool rect_reach(float2 g, float4 co, float x0, float x1, float y0, float y1, float thr) {
    const float dxl = g.x - x1, dxh = g.x - x0;
    const float dyl = g.y - y1, dyh = g.y - y0;
    if (dxl <= 0.f && dxh >= 0.f && dyl <= 0.f && dyh >= 0.f) return true;
    auto Q = [&](float dx, float dy) { return co.x * dx * dx + 2.f * co.y * dx * dy + co.z * dy * dy; };
    float q = Q(dxl, fminf(fmaxf(-co.y * dxl / co.z, dyl), dyh));
    q = fminf(q, Q(dxh, fminf(fmaxf(-co.y * dxh / co.z, dyl), dyh)));
    q = fminf(q, Q(fminf(fmaxf(-co.y * dyl / co.x, dxl), dxh), dyl));
    q = fminf(q, Q(fminf(fmaxf(-co.y * dyh / co.x, dxl), dxh), dyh));
    return q <= thr;
}
__device__ __forceinline__ float reach_thr(float o) { return 2.f * __logf(255.f * o) * 1.01f + 1e-3f; }
__device__ __forceinline__ bool tile_reach(float2 g, float4 co, float x0, float y0) {
    if (!(co.w >= 1.f / 255.f)) return false;  // alpha <= o < 1/255 on every pixel
    return rect_reach(g, co, x0, x0 + (float)(TILE_X - 1), y0, y0 + (float)(TILE_Y - 1), reach_thr(co.w));
}
// The staged conic in exponent form: power * log2(e) = dx (q.x dx + q.y dy) + q.z dy^2 with
// q = (-0.5 a, -b, -0.5 c) log2(e) and q.w = opacity, so G = 2^p is one v_exp_f32 (no scaling
// multiply per pixel and Gaussian; 4 ops for the quadratic form). Every blend kernel evaluates
// alpha through q_power / q_alpha with the same fused operations, so the forward's and the
// backward's alphas agree bitwise (the backward's transmittance replay depends on it).
constexpr float BL_L2E = 1.4426950408889634f;
__device__ __forceinline__ float4 conic_q(float4 co) {
    return make_float4(-0.5f * BL_L2E * co.x, -BL_L2E * co.y, -0.5f * BL_L2E * co.z, co.w);
}
__device__ __forceinline__ float q_power(float4 q, float dx, float dy) {
    return fmaf(dx, fmaf(q.x, dx, q.y * dy), q.z * (dy * dy));
}

// Block-wide stable compaction slot of a kept item (tid order): (slot, kept count); two barriers
__device__ __forceinline__ int2 compact_slot(bool keep, int tid, uint32_t *s_wcnt) {
    const unsigned long long m = __ballot(keep);
    const int lane = tid & 63, wave = tid >> 6;
    const int below = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_wcnt[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < TILE_PIX / 64; w++) {
        const int c = (int)s_wcnt[w];
        base += w < wave ? c : 0;
        tot += c;
    }
    return make_int2(base + below, tot);
}

// Pixel of thread tid within its 16x16 tile: wave w takes the 8x8 quadrant (w & 1, w >> 1), not a
// 16x4 row strip, so a Gaussian covering part of the tile touches fewer waves (each (wave, Gaussian)
// pair costs the wave's whole gradient reduction in the backward): blend_bwd 0.336 -> 0.319 ms at
// P = 1.0 M pairs (3 A/B pairs, tools/variant_session.sh), forward unchanged. DGS_BLEND_STRIP: strips.
__device__ __forceinline__ int2 tile_pixel(int tid) {
    const int w = tid >> 6, l = tid & 63;
    return make_int2((w & 1) * 8 + (l & 7), (w >> 1) * 8 + (l >> 3));
}

// Segmented blend backward (k_blend_bwd2s): the forward leaves, every SEG list positions of a tile,
// each pixel's (T, C) before that position (a "checkpoint", state before the Gaussians from there on),
// and the tile's backward work (the largest last-contributor position + 1); the backward then runs
// every SEG-long segment of every tile as an independent work item (segment-major), starting from the
// checkpoint at the segment's end instead of replaying the whole list from the end.
constexpr int SEG = 128;
// checkpoint slot of list position gp (absolute, gp = tile start + a multiple of SEG, strictly inside the
// tile's list): gp / SEG is unique across tiles (the next tile's first boundary lies >= SEG past every
// boundary of this one)
__device__ __forceinline__ uint32_t ckpt_slot(uint32_t gp) { return gp / SEG; }

template <bool CK>  // CK: write the segmented backward's checkpoints, final state and per-tile work
__global__ __launch_bounds__(256) void k_blend_fwd(const uint2 *__restrict__ ranges, const uint32_t *__restrict__ vals,
                                                   uint32_t cap, int W, int H, int gx, const float2 *__restrict__ xy,
                                                   const float4 *__restrict__ conic_o, const float4 *__restrict__ rgbd,
                                                   const float *bg, float *__restrict__ final_T,
                                                   uint32_t *__restrict__ n_contrib, float *__restrict__ out_color,
                                                   float *__restrict__ out_depth, float4 *__restrict__ ckpt,
                                                   uint32_t *__restrict__ tile_todo, uint32_t *__restrict__ maxtodo,
                                                   float4 *__restrict__ cfin) {
    __shared__ float2 s_xy[TILE_PIX];
    __shared__ float4 s_co[TILE_PIX];
    __shared__ float4 s_cd[TILE_PIX];
    __shared__ int s_pos[TILE_PIX];
    __shared__ uint32_t s_wcnt[TILE_PIX / 64];
    const int tile = blockIdx.x;
    const int tid = threadIdx.x;
    const float tx0 = (float)((tile % gx) * TILE_X), ty0 = (float)((tile / gx) * TILE_Y);
    const int2 tp = tile_pixel(tid);
    const int px = (tile % gx) * TILE_X + tp.x;
    const int py = (tile / gx) * TILE_Y + tp.y;
    const bool inside = px < W && py < H;
    const float pfx = (float)px, pfy = (float)py;
    uint2 range = ranges[tile];
    range.x = min(range.x, cap);  // a speculative launch under capacity (redone at the exact size)
    range.y = min(range.y, cap);
    const int todo_total = (int)(range.y - range.x);
    const int rounds = div_up(todo_total, TILE_PIX);
    bool done = !inside;
    float T = 1.f, C0 = 0.f, C1 = 0.f, C2 = 0.f, Dd = 0.f;
    uint32_t last = 0;
    for (int r = 0; r < rounds; r++) {
        if (__syncthreads_count(done) == TILE_PIX) break;
        int prog = r * TILE_PIX + tid;
        bool keep = false;
        uint32_t id = 0;
        float2 gl;
        float4 cl;
        if ((int)range.x + prog < (int)range.y) {
            id = vals[range.x + prog];
            gl = xy[id];
            cl = conic_o[id];
            keep = tile_reach(gl, cl, tx0, ty0);
        }
        const int2 sl = compact_slot(keep, tid, s_wcnt);
        if (keep) {
            s_xy[sl.x] = gl;
            s_co[sl.x] = conic_q(cl);
            s_cd[sl.x] = rgbd[id];
            s_pos[sl.x] = prog;
        }
        // the batch is padded to a multiple of 4 with inert entries (zero conic and opacity: power 0,
        // alpha 0, never used), so the loop below tests for its early exit once per 4 Gaussians
        const int n = sl.y, n4 = (sl.y + 3) & ~3;
        if (tid >= n && tid < n4) {
            s_xy[tid] = make_float2(0.f, 0.f);
            s_co[tid] = make_float4(0.f, 0.f, 0.f, 0.f);
            s_cd[tid] = make_float4(0.f, 0.f, 0.f, 0.f);
            s_pos[tid] = 0;
        }
        __syncthreads();
        // checkpoints (segmented backward): the state before positions 256 r + 128 and 256 (r + 1); the
        // first half of the batch (threads 0..127 = waves 0, 1) staged jmid kept Gaussians
        const int jmid = CK ? (int)(s_wcnt[0] + s_wcnt[1]) : -1;
        const uint32_t pix = (uint32_t)(tp.y * TILE_X + tp.x);
        auto put_ckpt = [&](int p) {  // p: position in the tile's list (a multiple of SEG, > 0)
            if (CK && inside && p < todo_total)
                ckpt[(size_t)ckpt_slot(range.x + (uint32_t)p) * TILE_PIX + pix] = make_float4(T, C0, C1, C2);
        };
        bool mid_done = false;
        // branch-free per lane (a skipped Gaussian adds cd * 0): the skips and the stop of the
        // reference's loop become predicates, so the wave runs no exec-mask bookkeeping per
        // Gaussian; it leaves the batch once all of its lanes are done. Every staged word is a
        // broadcast read that still costs the wave's full LDS cycles (b64 2, b128 4), so the last
        // contributor is tracked as a batch index and mapped to its list position once per batch
        // (12 -> 10 LDS cycles per Gaussian and wave: blend_fwd -3.5 %)
        int lastj = 0;  // batch index + 1 of this batch's last contributor (0: none)
        for (int j0 = 0; j0 < n4; j0 += 4) {
            if (__ballot(!done) == 0ull) break;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = j0 + u;
                if constexpr (CK) {
                    if (j == jmid) {
                        put_ckpt(r * TILE_PIX + SEG);
                        mid_done = true;
                    }
                }
                const int pos1 = j + 1;
                const float2 g = s_xy[j];
                const float4 q = s_co[j];
                const float4 cd = s_cd[j];
                const float dx = g.x - pfx, dy = g.y - pfy;
                const float power = q_power(q, dx, dy);
                const float alpha = fminf(0.99f, q.w * __builtin_amdgcn_exp2f(power));
                const float testT = T * (1.f - alpha);
                bool use = !done && !(power > 0.f) && !(alpha < 1.f / 255.f);
                const bool stop = use && testT < 0.0001f;
                done = done || stop;
                use = use && !stop;
                const float w = use ? alpha * T : 0.f;
                C0 += cd.x * w;
                C1 += cd.y * w;
                C2 += cd.z * w;
                Dd += cd.w * w;
                T = use ? testT : T;
                lastj = use ? pos1 : lastj;
            }
        }
        if (lastj) last = (uint32_t)s_pos[lastj - 1] + 1u;  // list position + 1 (n_contrib of the full list)
        if constexpr (CK) {  // (a wave that left the batch early: its pixels are done, their state is final)
            if (!mid_done) put_ckpt(r * TILE_PIX + SEG);
            put_ckpt((r + 1) * TILE_PIX);
        }
    }
    if constexpr (CK) {  // the tile's backward work: the largest last-contributor position + 1
        __shared__ uint32_t s_todo;
        if (tid == 0) s_todo = 0;
        __syncthreads();
        if (inside) atomicMax(&s_todo, last);
        __syncthreads();
        if (tid == 0) {
            tile_todo[tile] = s_todo;
            atomicMax(maxtodo, s_todo);
        }
    }
    if (inside) {
        int pid = py * W + px;
        if constexpr (CK) cfin[pid] = make_float4(T, C0, C1, C2);  // the final state (segmented backward)
        final_T[pid] = T;
        n_contrib[pid] = last;
        int HW = H * W;
        out_color[pid] = C0 + T * bg[0];
        out_color[HW + pid] = C1 + T * bg[1];
        out_color[2 * HW + pid] = C2 + T * bg[2];
        out_depth[pid] = Dd;
    }
}

// ------------------------------------------------------------------------------------------------
// backward kernels
// ------------------------------------------------------------------------------------------------
// Reduce-scatter of the 12 per-Gaussian partial gradients over the 64 lanes (gfx950 lane swaps):
//   fold32(a, b): v_permlane32_swap pairs lane l with l+32 -> lanes 0-31 carry a, 32-63 carry b;
//   fold16(a, b): v_permlane16_swap pairs 16-lane rows 0<->1, 2<->3 -> each row carries one value;
//   row_sum15: DPP row_shr 1/2/4/8 -> the row total in the row's lane 15.
// 6 + 3 swaps and 3 x 4 DPP adds replace 12 independent 64-lane reductions (72 DPP adds + 12
// readlanes); the sums end in lanes 15/31/47/63 of three registers.
__device__ inline float fold32(float a, float b) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ inline float fold16(float a, float b) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ inline float row_sum15(float v) {
    int x = __float_as_int(v);
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true));
    x = __float_as_int(v);
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true));
    x = __float_as_int(v);
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true));
    x = __float_as_int(v);
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true));
    return v;
}

__global__ __launch_bounds__(256) void k_blend_bwd(const uint2 *__restrict__ ranges, const uint32_t *__restrict__ vals,
                                                   uint32_t cap, int W, int H, int gx, const float *bg,
                                                   const float2 *__restrict__ xy, const float4 *__restrict__ conic_o,
                                                   const float4 *__restrict__ rgbd, const float *__restrict__ final_T,
                                                   const uint32_t *__restrict__ n_contrib,
                                                   const float *__restrict__ dL_dpix, const float *__restrict__ dL_ddepth,
                                                   float *__restrict__ acc) {
    __shared__ float2 s_xy[TILE_PIX];
    __shared__ float4 s_co[TILE_PIX];
    __shared__ float4 s_q[TILE_PIX];
    __shared__ float4 s_cd[TILE_PIX];
    __shared__ uint32_t s_id[TILE_PIX];
    __shared__ int s_pos[TILE_PIX];
    __shared__ uint32_t s_wcnt[TILE_PIX / 64];
    __shared__ uint32_t s_maxlast;
    const int tile = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const float tx0 = (float)((tile % gx) * TILE_X), ty0 = (float)((tile / gx) * TILE_Y);
    const int2 tp = tile_pixel(tid);
    const int px = (tile % gx) * TILE_X + tp.x;
    const int py = (tile / gx) * TILE_Y + tp.y;
    const bool inside = px < W && py < H;
    const float pfx = (float)px, pfy = (float)py;
    uint2 range = ranges[tile];
    range.x = min(range.x, cap);  // a deferred count not resolved yet: the launched capacity bounds the list
    range.y = min(range.y, cap);
    const int pid = py * W + px;
    const int HW = H * W;
    float Tfinal = 1.f, dp0 = 0.f, dp1 = 0.f, dp2 = 0.f, ddep = 0.f;
    uint32_t last = 0;
    if (inside) {
        Tfinal = final_T[pid];
        last = n_contrib[pid];
        dp0 = dL_dpix[pid];
        dp1 = dL_dpix[HW + pid];
        dp2 = dL_dpix[2 * HW + pid];
        ddep = dL_ddepth ? dL_ddepth[pid] : 0.f;
    }
    if (tid == 0) s_maxlast = 0;
    __syncthreads();
    atomicMax(&s_maxlast, last);
    __syncthreads();
    const int todo_total = (int)s_maxlast;  // Gaussians past every pixel's last contributor are skipped
    const float b0 = bg[0], b1 = bg[1], b2 = bg[2];
    const float bgdot = b0 * dp0 + b1 * dp1 + b2 * dp2;
    const float hx = 0.5f * W, hy = 0.5f * H;
    float T = Tfinal;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, accd = 0.f;
    float lc0 = 0.f, lc1 = 0.f, lc2 = 0.f, lcd = 0.f, last_alpha = 0.f;
    int contributor = todo_total;
    const int rounds = div_up(todo_total, TILE_PIX);
    const int end = (int)range.x + todo_total;
    for (int r = 0; r < rounds; r++) {
        __syncthreads();
        int prog = r * TILE_PIX + tid;
        bool keep = false;
        uint32_t id = 0;
        float2 gl;
        float4 cl;
        if (prog < todo_total) {
            id = vals[end - prog - 1];
            gl = xy[id];
            cl = conic_o[id];
            keep = tile_reach(gl, cl, tx0, ty0);
        }
        const int2 sl = compact_slot(keep, tid, s_wcnt);
        if (keep) {
            s_id[sl.x] = id;
            s_xy[sl.x] = gl;
            s_co[sl.x] = cl;
            s_q[sl.x] = conic_q(cl);
            s_cd[sl.x] = rgbd[id];
            s_pos[sl.x] = prog;
        }
        __syncthreads();
        const int n = sl.y;
        for (int j = 0; j < n; j++) {
            contributor = todo_total - 1 - s_pos[j];  // position in the full list
            float2 g = s_xy[j];
            float4 co = s_co[j];
            float dx = g.x - pfx, dy = g.y - pfy;
            float power = q_power(s_q[j], dx, dy);
            float G = __builtin_amdgcn_exp2f(power);
            float alpha = fminf(0.99f, co.w * G);
            bool act = inside && (uint32_t)contributor < last && power <= 0.f && alpha >= 1.f / 255.f;
            if (__ballot(act) == 0ull) continue;  // wave-uniform
            float v_mx = 0.f, v_my = 0.f, v_cx = 0.f, v_cy = 0.f, v_cz = 0.f, v_op = 0.f;
            float v_r = 0.f, v_g = 0.f, v_b = 0.f, v_d = 0.f;
            if (act) {
                float4 cd = s_cd[j];
                // 1 / (1 - alpha): hardware reciprocal + one Newton step (<= 1 ulp, vs the ~10-op
                // IEEE division; the gradients' tolerance is 1e-3 relative)
                const float om = 1.f - alpha;
                float inv1ma = __builtin_amdgcn_rcpf(om);
                inv1ma = fmaf(inv1ma, fmaf(-om, inv1ma, 1.f), inv1ma);
                T = T * inv1ma;
                float w = alpha * T;
                acc0 = last_alpha * lc0 + (1.f - last_alpha) * acc0;
                acc1 = last_alpha * lc1 + (1.f - last_alpha) * acc1;
                acc2 = last_alpha * lc2 + (1.f - last_alpha) * acc2;
                accd = last_alpha * lcd + (1.f - last_alpha) * accd;
                lc0 = cd.x; lc1 = cd.y; lc2 = cd.z; lcd = cd.w;
                float dLda = (cd.x - acc0) * dp0 + (cd.y - acc1) * dp1 + (cd.z - acc2) * dp2 + (cd.w - accd) * ddep;
                v_r = w * dp0;
                v_g = w * dp1;
                v_b = w * dp2;
                v_d = w * ddep;
                dLda *= T;
                last_alpha = alpha;
                dLda += (-Tfinal * inv1ma) * bgdot;
                float dLdG = co.w * dLda;
                float gdx = G * dx, gdy = G * dy;
                float dGdx = -gdx * co.x - gdy * co.y;
                float dGdy = -gdy * co.z - gdx * co.y;
                v_mx = dLdG * dGdx * hx;
                v_my = dLdG * dGdy * hy;
                v_cx = -0.5f * gdx * dx * dLdG;
                v_cy = -0.5f * gdx * dy * dLdG;
                v_cz = -0.5f * gdy * dy * dLdG;
                v_op = G * dLda;
            }
            // pairs (a, b) fold to rows [a_lo, b_lo, a_hi, b_hi] of w: row r of w_k holds field
            // 4k + {0, 2, 1, 3}[r] (ACC_MX..ACC_DY order)
            const float w0 = row_sum15(fold16(fold32(v_mx, v_my), fold32(v_cx, v_cy)));
            const float w1 = row_sum15(fold16(fold32(v_cz, v_op), fold32(v_r, v_g)));
            const float w2 = row_sum15(fold16(fold32(v_b, v_d), fold32(fabsf(v_mx), fabsf(v_my))));
            if ((lane & 15) == 15) {
                const int row = lane >> 4;
                float *dst = acc + (size_t)s_id[j] * ACC_STRIDE + ((row & 1) << 1) + (row >> 1);
                atomicAdd(dst, w0);
                atomicAdd(dst + 4, w1);
                atomicAdd(dst + 8, w2);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Blend backward, two pixels per lane (the default): a 16x16 tile runs as ONE 128-thread workgroup of
// two waves; wave w covers the 16x8 half (rows 8w..8w+7), lane l the pixel pair (l & 7, row) and
// (8 + (l & 7), row): one dy, a packed dx, so the per-(pixel, Gaussian) arithmetic runs as packed fp32
// (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two pixels per instruction), and the per-(wave,
// Gaussian) gradient reduction covers 128 pixels instead of 64 (half as many reductions and atomics
// per Gaussian). Per-pixel activity that k_blend_bwd expresses with the exec mask becomes selects:
// an inactive pixel of a pair keeps its state and contributes zero. 128 Gaussians staged per round
// (6 KB of LDS: staging 256, two per thread, took 0.29 ms: 24 KB per workgroup capped the occupancy).
// blend_bwd 0.315-0.322 -> 0.283 ms at P = 1.0 M pairs (A/B against DGS_BLEND1=1).
// (The same packing in the forward was slower: 0.137 vs 0.127 ms; its per-Gaussian work is too small
// to pay for half the waves per tile.)
// ------------------------------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int B2 = 128;  // threads per tile (two waves), Gaussians staged per round

// Block-wide stable compaction slot of a kept item over NW waves: (slot, kept count)
template <int NW>
__device__ __forceinline__ int2 compact_slot_n(bool keep, int tid, uint32_t *s_wcnt) {
    const unsigned long long m = __ballot(keep);
    const int lane = tid & 63, wave = tid >> 6;
    const int below = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_wcnt[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const int c = (int)s_wcnt[w];
        base += w < wave ? c : 0;
        tot += c;
    }
    return make_int2(base + below, tot);
}

__device__ __forceinline__ f2 sel2(bool a, bool b, f2 x, f2 y) { return f2{a ? x.x : y.x, b ? x.y : y.y}; }

// Forward blend, two pixels per lane (DGS_BLEND_FWD2=1; the segmented backward's checkpoints stay on
// k_blend_fwd): k_blend_bwd2's layout — a 16x16 tile as two waves, lane l of wave w holding the pixel
// pair (l & 7, 8 w + l / 8) and (8 + l & 7, same row), 128-Gaussian batches — so every staged
// Gaussian's broadcast LDS reads serve two pixels and the per-pixel arithmetic runs on packed fp32
// pairs. Per pixel the operations, their order and the fused forms are k_blend_fwd's: the image,
// the transmittance and n_contrib are bitwise the same (GPU test).
__global__ __launch_bounds__(B2) void k_blend_fwd2(const uint2 *__restrict__ ranges, const uint32_t *__restrict__ vals,
                                                   uint32_t cap, int W, int H, int gx, const float2 *__restrict__ xy,
                                                   const float4 *__restrict__ conic_o, const float4 *__restrict__ rgbd,
                                                   const float *bg, float *__restrict__ final_T,
                                                   uint32_t *__restrict__ n_contrib, float *__restrict__ out_color,
                                                   float *__restrict__ out_depth) {
    __shared__ float2 s_xy[B2];
    __shared__ float4 s_co[B2];
    __shared__ float4 s_cd[B2];
    __shared__ int s_pos[B2];
    __shared__ uint32_t s_wcnt[B2 / 64];
    const int tile = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx0i = (tile % gx) * TILE_X, ty0i = (tile / gx) * TILE_Y;
    const float tx0 = (float)tx0i, ty0 = (float)ty0i;
    const int px0 = tx0i + (lane & 7), px1 = px0 + 8, py = ty0i + 8 * wv + (lane >> 3);
    const bool in0 = px0 < W && py < H, in1 = px1 < W && py < H;
    const f2 pfx = f2{(float)px0, (float)px1};
    const float pfy = (float)py;
    uint2 range = ranges[tile];
    range.x = min(range.x, cap);  // a speculative launch under capacity (redone at the exact size)
    range.y = min(range.y, cap);
    const int todo_total = (int)(range.y - range.x);
    const int rounds = div_up(todo_total, B2);
    bool done0 = !in0, done1 = !in1;
    const f2 zero = f2{0.f, 0.f};
    f2 T = f2{1.f, 1.f}, C0 = zero, C1 = zero, C2 = zero, Dd = zero;
    uint32_t last0 = 0, last1 = 0;
    for (int r = 0; r < rounds; r++) {
        if (__syncthreads_count(done0 && done1) == B2) break;
        const int prog = r * B2 + tid;
        bool keep = false;
        uint32_t id = 0;
        float2 gl;
        float4 cl;
        if ((int)range.x + prog < (int)range.y) {
            id = vals[range.x + prog];
            gl = xy[id];
            cl = conic_o[id];
            keep = tile_reach(gl, cl, tx0, ty0);
        }
        const int2 sl = compact_slot_n<B2 / 64>(keep, tid, s_wcnt);
        if (keep) {
            s_xy[sl.x] = gl;
            s_co[sl.x] = conic_q(cl);
            s_cd[sl.x] = rgbd[id];
            s_pos[sl.x] = prog;
        }
        const int n = sl.y, n4 = (sl.y + 3) & ~3;  // padded with inert entries, as k_blend_fwd
        if (tid >= n && tid < n4) {
            s_xy[tid] = make_float2(0.f, 0.f);
            s_co[tid] = make_float4(0.f, 0.f, 0.f, 0.f);
            s_cd[tid] = make_float4(0.f, 0.f, 0.f, 0.f);
            s_pos[tid] = 0;
        }
        __syncthreads();
        int lastj0 = 0, lastj1 = 0;
        for (int j0 = 0; j0 < n4; j0 += 4) {
            if (__ballot(!(done0 && done1)) == 0ull) break;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = j0 + u;
                const float2 g = s_xy[j];
                const float4 q = s_co[j];
                const float4 cd = s_cd[j];
                const f2 dx = g.x - pfx;
                const float dy = g.y - pfy;
                const f2 power = f2{q_power(q, dx.x, dy), q_power(q, dx.y, dy)};
                const f2 alpha = f2{fminf(0.99f, q.w * __builtin_amdgcn_exp2f(power.x)),
                                    fminf(0.99f, q.w * __builtin_amdgcn_exp2f(power.y))};
                const f2 testT = T * (1.f - alpha);
                bool use0 = !done0 && !(power.x > 0.f) && !(alpha.x < 1.f / 255.f);
                bool use1 = !done1 && !(power.y > 0.f) && !(alpha.y < 1.f / 255.f);
                const bool stop0 = use0 && testT.x < 0.0001f, stop1 = use1 && testT.y < 0.0001f;
                done0 = done0 || stop0;
                done1 = done1 || stop1;
                use0 = use0 && !stop0;
                use1 = use1 && !stop1;
                const f2 w = sel2(use0, use1, alpha * T, zero);
                C0 += cd.x * w;
                C1 += cd.y * w;
                C2 += cd.z * w;
                Dd += cd.w * w;
                T = sel2(use0, use1, testT, T);
                lastj0 = use0 ? j + 1 : lastj0;
                lastj1 = use1 ? j + 1 : lastj1;
            }
        }
        if (lastj0) last0 = (uint32_t)s_pos[lastj0 - 1] + 1u;  // list position + 1 (n_contrib of the full list)
        if (lastj1) last1 = (uint32_t)s_pos[lastj1 - 1] + 1u;
    }
    const int HW = H * W;
    if (in0) {
        const int pid = py * W + px0;
        final_T[pid] = T.x;
        n_contrib[pid] = last0;
        out_color[pid] = C0.x + T.x * bg[0];
        out_color[HW + pid] = C1.x + T.x * bg[1];
        out_color[2 * HW + pid] = C2.x + T.x * bg[2];
        out_depth[pid] = Dd.x;
    }
    if (in1) {
        const int pid = py * W + px1;
        final_T[pid] = T.y;
        n_contrib[pid] = last1;
        out_color[pid] = C0.y + T.y * bg[0];
        out_color[HW + pid] = C1.y + T.y * bg[1];
        out_color[2 * HW + pid] = C2.y + T.y * bg[2];
        out_depth[pid] = Dd.y;
    }
}

#define BWD2_OCC
// DEPTH: the depth output has a gradient (dL_ddepth != nullptr); without one (every training step: the
// loss reads only the image) the depth terms, the depth colour-behind state and its loads drop out.
// DET: the deterministic mode (k_rect_gather): the two waves' reduced sums for a staged Gaussian meet in
// an LDS row (each field gets at most one add per wave onto zero: a + b either way round), written out
// after the batch to the pair's slot (12 floats; the staging thread writes zeros for a culled entry), and
// the tile's replayed length to tile_todo, instead of adding into acc; the pairs past the replayed
// prefix get zeros. A pair's slot is its list position when the lists were placed in depth order, else
// (the per-tile sort) the position k_rect_place gave it in index order (tile start + pre[position]):
// where k_rect_gather's walk, in k_rect_place's order, finds it
template <bool DEPTH, bool DET>
__global__ __launch_bounds__(B2) BWD2_OCC void k_blend_bwd2(const uint2 *__restrict__ ranges, const uint32_t *__restrict__ vals,
                                                   uint32_t cap, int W, int H, int gx, const float *bg,
                                                   const float2 *__restrict__ xy, const float4 *__restrict__ conic_o,
                                                   const float4 *__restrict__ rgbd, const float *__restrict__ final_T,
                                                   const uint32_t *__restrict__ n_contrib,
                                                   const float *__restrict__ dL_dpix, const float *__restrict__ dL_ddepth,
                                                   float *__restrict__ acc, float *__restrict__ slot,
                                                   uint32_t *__restrict__ tile_todo, const uint32_t *__restrict__ pre) {
    __shared__ float4 s_q[B2];   // staged conic in exponent form + opacity
    __shared__ float4 s_xyc[B2]; // mean2D x, y, list position (bits), Gaussian id (bits)
    __shared__ float4 s_co[B2];
    __shared__ float4 s_cd[B2];
    __shared__ uint32_t s_wcnt[B2 / 64];
    __shared__ uint32_t s_maxlast;
    __shared__ float4 s_slot[DET ? 3 * B2 : 1];  // DET: per staged Gaussian, its 12 gradient sums
    const int tile = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx0 = (tile % gx) * TILE_X, ty0 = (tile / gx) * TILE_Y;
    const int px0 = tx0 + (lane & 7), px1 = px0 + 8, py = ty0 + 8 * wv + (lane >> 3);
    const bool in0 = px0 < W && py < H, in1 = px1 < W && py < H;
    const f2 pfx = f2{(float)px0, (float)px1};
    const float pfy = (float)py;
    uint2 range = ranges[tile];
    range.x = min(range.x, cap);  // a deferred count not resolved yet: the launched capacity bounds the list
    range.y = min(range.y, cap);
    const int HW = H * W;
    const int pid0 = py * W + px0, pid1 = py * W + px1;
    f2 Tfinal = f2{1.f, 1.f}, dp0 = f2{0.f, 0.f}, dp1 = dp0, dp2 = dp0, ddep = dp0;
    uint32_t last0 = 0, last1 = 0;
    if (in0) {
        Tfinal.x = final_T[pid0];
        last0 = n_contrib[pid0];
        dp0.x = dL_dpix[pid0];
        dp1.x = dL_dpix[HW + pid0];
        dp2.x = dL_dpix[2 * HW + pid0];
        if (DEPTH) ddep.x = dL_ddepth[pid0];
    }
    if (in1) {
        Tfinal.y = final_T[pid1];
        last1 = n_contrib[pid1];
        dp0.y = dL_dpix[pid1];
        dp1.y = dL_dpix[HW + pid1];
        dp2.y = dL_dpix[2 * HW + pid1];
        if (DEPTH) ddep.y = dL_ddepth[pid1];
    }
    if (tid == 0) s_maxlast = 0;
    __syncthreads();
    atomicMax(&s_maxlast, max(last0, last1));
    __syncthreads();
    const int todo_total = (int)s_maxlast;  // Gaussians past every pixel's last contributor are skipped
    if (DET && tid == 0) tile_todo[tile] = (uint32_t)todo_total;
    // DET: a pair's slot (pre: the per-tile sort's map back to the walk's index-order position)
    [[maybe_unused]] auto slot_of = [&](uint32_t lp) { return reinterpret_cast<float4 *>(slot + 12ull * (pre ? range.x + pre[lp] : lp)); };
    if constexpr (DET) {  // the pairs past the replayed prefix add nothing: zeros (the gather reads every pair)
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        for (uint32_t lp = range.x + (uint32_t)todo_total + tid; lp < range.y; lp += B2) {
            float4 *z = slot_of(lp);
            z[0] = z4;
            z[1] = z4;
            z[2] = z4;
        }
    }
    const float b0 = bg[0], b1 = bg[1], b2 = bg[2];
    const f2 kbg = -Tfinal * (b0 * dp0 + b1 * dp1 + b2 * dp2);  // dL/dalpha's background term / (1 - alpha)
    const float hx = 0.5f * W, hy = 0.5f * H;
    // the reduce-scatter leaves field 4k + {0, 2, 1, 3}[row] of register k in the row's lane 15: the
    // per-pixel terms are summed unscaled and each field's constant factor is applied once here
    const int frow = lane >> 4;
    const float sc0 = frow == 0 ? -hx : frow == 2 ? -hy : -0.5f;        // mean2D x, conic x, mean2D y, conic y
    const float sc1 = frow == 0 ? -0.5f : 1.f;                           // conic z, r, opacity, g
    const float sc2 = frow == 1 ? hx : frow == 3 ? hy : 1.f;             // b, |mean2D x|, depth, |mean2D y|
    f2 T = Tfinal;
    const f2 zero = f2{0.f, 0.f};
    f2 acc0 = zero, acc1 = zero, acc2 = zero, accd = zero;
    const int rounds = div_up(todo_total, B2);
    const int end = (int)range.x + todo_total;
    for (int r = 0; r < rounds; r++) {
        __syncthreads();
        const int prog = r * B2 + tid;
        bool keep = false;
        uint32_t id = 0;
        float2 gl;
        float4 cl;
        if (prog < todo_total) {
            id = vals[end - prog - 1];
            gl = xy[id];
            cl = conic_o[id];
            keep = tile_reach(gl, cl, (float)tx0, (float)ty0);
            if (DET && !keep) {
                float4 *z = slot_of((uint32_t)(end - prog - 1));
                const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
                z[0] = z4;
                z[1] = z4;
                z[2] = z4;
            }
        }
        if constexpr (DET) {  // this round's rows (the previous round's were written out before the barrier)
            const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
            s_slot[3 * tid] = z4;
            s_slot[3 * tid + 1] = z4;
            s_slot[3 * tid + 2] = z4;
        }
        const int2 sl = compact_slot_n<B2 / 64>(keep, tid, s_wcnt);
        if (keep) {
            // the position in the full list and the Gaussian's id, staged as bits beside the mean
            // (the atomic lanes used to read the id from a separate LDS array after the reduction,
            // a wait with the whole wave behind it)
            s_xyc[sl.x] = make_float4(gl.x, gl.y, __uint_as_float((uint32_t)(todo_total - 1 - prog)), __uint_as_float(id));
            s_co[sl.x] = cl;
            s_q[sl.x] = conic_q(cl);
            s_cd[sl.x] = rgbd[id];
        }
        __syncthreads();
        const int n = sl.y;
        // the next Gaussian's mean / position / id and conic are read while this one is processed:
        // the loop's first LDS reads otherwise waited out their latency at the top of every iteration
        // (blend_bwd -3.3 % at 86 VGPRs, occupancy 6 -> 5; also prefetching the colour and conic
        // read after the skip test was slower: profiles/r4zj_blend_bwd_prefetch_ab.txt, and again at
        // 96 VGPRs with the id staged here, occupancy 5 either way: profiles/r5g_blend_bwd_id_ab.txt)
        // two Gaussians per loop trip with alternating register sets: with one per trip the compiler
        // copied the prefetched mean / conic into the working registers every iteration (4 moves)
        auto gauss = [&](int j, const float4 &xc, const float4 &q) {
            const uint32_t contributor = __float_as_uint(xc.z);  // position in the full list
            const f2 dx = xc.x - pfx;
            const float dy = xc.y - pfy;
            const f2 power = f2{q_power(q, dx.x, dy), q_power(q, dx.y, dy)};
            const f2 G = f2{__builtin_amdgcn_exp2f(power.x), __builtin_amdgcn_exp2f(power.y)};
            const f2 alpha = f2{fminf(0.99f, q.w * G.x), fminf(0.99f, q.w * G.y)};
            // a pixel takes the Gaussian iff it lies within the pixel's contributors (last = 0 outside
            // the image), power <= 0 and alpha >= 1/255: the alpha gated by the first two decides, and
            // the wave's skip test is ONE compare on the larger of the pair (a ballot of a plain
            // compare is its lane mask; of a combined predicate the compiler materialises it first)
            const float ga0 = (contributor < last0 && power.x <= 0.f) ? alpha.x : 0.f;
            const float ga1 = (contributor < last1 && power.y <= 0.f) ? alpha.y : 0.f;
            if (__ballot(fmaxf(ga0, ga1) >= 1.f / 255.f) == 0ull) return;  // wave-uniform
            const bool act0 = ga0 >= 1.f / 255.f, act1 = ga1 >= 1.f / 255.f;
            const float4 cd = s_cd[j];
            const float4 co = s_co[j];
            // an inactive pixel of the pair runs with alpha = 0 and G = 0: T (1 / (1 - 0) = 1), its
            // pending colour and every gradient term stay unchanged / zero without per-state selects
            const f2 ae = sel2(act0, act1, alpha, zero);
            const f2 Ge = sel2(act0, act1, G, zero);
            // 1 / (1 - alpha): hardware reciprocal + one Newton step (<= 1 ulp; exactly 1 at alpha = 0)
            const f2 om = 1.f - ae;
            f2 inv = f2{__builtin_amdgcn_rcpf(om.x), __builtin_amdgcn_rcpf(om.y)};
            inv = inv * (1.f - om * inv) + inv;
            T = T * inv;
            const f2 w = ae * T;
            // colour behind this Gaussian (acc) is updated eagerly after its use: the reference's
            // deferred last_alpha * last_color + (1 - last_alpha) * acc at the next active Gaussian
            const f2 d0 = cd.x - acc0, d1 = cd.y - acc1, d2 = cd.z - acc2;
            f2 dLda = d0 * dp0 + d1 * dp1 + d2 * dp2;
            if constexpr (DEPTH) {
                const f2 d3 = cd.w - accd;
                dLda = dLda + d3 * ddep;
                accd = ae * d3 + accd;
            }
            acc0 = ae * d0 + acc0;
            acc1 = ae * d1 + acc1;
            acc2 = ae * d2 + acc2;
            dLda = dLda * T + kbg * inv;
            // dG/dmean2D = -G (conic . d), dG/dconic = -G d d^T / 2: with u = dL/dG G the per-pixel
            // terms are co (u d) and u d d^T, their factors (-hx, -hy, -0.5) applied after the sums
            const f2 vop = Ge * dLda;
            const f2 u = co.w * vop;
            const f2 udx = u * dx, udy = u * dy;
            const f2 mxp = co.x * udx + co.y * udy, myp = co.y * udx + co.z * udy;
            const f2 cxp = udx * dx, cyp = udx * dy, czp = udy * dy;
            const f2 vr = w * dp0, vg = w * dp1, vb = w * dp2, vd = DEPTH ? w * ddep : zero;
            const float w0 = row_sum15(fold16(fold32(mxp.x + mxp.y, myp.x + myp.y), fold32(cxp.x + cxp.y, cyp.x + cyp.y)));
            const float w1 = row_sum15(fold16(fold32(czp.x + czp.y, vop.x + vop.y), fold32(vr.x + vr.y, vg.x + vg.y)));
            const float w2 = row_sum15(fold16(fold32(vb.x + vb.y, vd.x + vd.y),
                                              fold32(fabsf(mxp.x) + fabsf(mxp.y), fabsf(myp.x) + fabsf(myp.y))));
            if ((lane & 15) == 15) {
                const int row = lane >> 4;
                const int fo = ((row & 1) << 1) + (row >> 1);
                if constexpr (DET) {
                    float *dst = reinterpret_cast<float *>(s_slot + 3 * j) + fo;
                    atomicAdd(dst, w0 * sc0);
                    atomicAdd(dst + 4, w1 * sc1);
                    atomicAdd(dst + 8, w2 * sc2);
                } else {
                    float *dst = acc + (size_t)__float_as_uint(xc.w) * ACC_STRIDE + fo;
                    atomicAdd(dst, w0 * sc0);
                    atomicAdd(dst + 4, w1 * sc1);
                    atomicAdd(dst + 8, w2 * sc2);
                }
            }
        };
        float4 xa = s_xyc[0], qa = s_q[0], xb, qb;
        int j = 0;
        for (; j + 1 < n; j += 2) {
            xb = s_xyc[j + 1];
            qb = s_q[j + 1];
            gauss(j, xa, qa);
            const int j2 = min(j + 2, B2 - 1);  // (the batch's last trip reads a spare slot)
            xa = s_xyc[j2];
            qa = s_q[j2];
            gauss(j + 1, xb, qb);
        }
        if (j < n) gauss(j, xa, qa);
        if constexpr (DET) {
            __syncthreads();  // both waves' adds are in
            if (tid < n) {
                float4 *dst = slot_of((uint32_t)range.x + __float_as_uint(s_xyc[tid].z));
                dst[0] = s_slot[3 * tid];
                dst[1] = s_slot[3 * tid + 1];
                dst[2] = s_slot[3 * tid + 2];
            }
        }
    }
}

// Segmented blend backward (no depth gradient: every training step). A persistent grid takes work items
// (segment s, tile) in segment-major order from a queue; item (s, tile) replays list positions
// [SEG s, min(SEG (s + 1), todo)) of the tile back to front, starting from the forward's checkpoint at
// the segment's end: T = the transmittance before that position, and the colour behind it (acc) =
// (C_final - C_before) / T. A long tile list thus runs as several concurrent work items instead of one
// serial replay, and the grid is filled with ~2x the waves of k_blend_bwd2. The per-(pixel, Gaussian)
// arithmetic and the reduction are k_blend_bwd2's. Numerics: acc's rounding error is ~1 ulp / T, but
// it enters dL/dalpha multiplied by the Gaussian's own transmittance (<= T), so the gradient error stays
// at the ulp level of dL/dpix.
constexpr int BWD_SEG_WGS_PER_CU = 12;
__global__ __launch_bounds__(B2) void k_blend_bwd2s(const uint2 *__restrict__ ranges, const uint32_t *__restrict__ vals,
                                                   uint32_t cap, int W, int H, int gx, int T_tiles, const float *bg,
                                                   const float2 *__restrict__ xy, const float4 *__restrict__ conic_o,
                                                   const float4 *__restrict__ rgbd, const float *__restrict__ final_T,
                                                   const uint32_t *__restrict__ n_contrib,
                                                   const float4 *__restrict__ cfin, const float4 *__restrict__ ckpt,
                                                   const uint32_t *__restrict__ tile_todo,
                                                   const uint32_t *__restrict__ maxtodo, uint32_t *__restrict__ queue,
                                                   const float *__restrict__ dL_dpix, float *__restrict__ acc) {
    __shared__ float2 s_xy[B2];
    __shared__ float4 s_co[B2];
    __shared__ float4 s_q[B2];
    __shared__ float4 s_cd[B2];
    __shared__ uint32_t s_id[B2];
    __shared__ int s_pos[B2];
    __shared__ uint32_t s_wcnt[B2 / 64];
    __shared__ int s_item;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int HW = H * W;
    const float b0 = bg[0], b1 = bg[1], b2 = bg[2];
    const float hx = 0.5f * W, hy = 0.5f * H;
    const int frow = lane >> 4;
    const float sc0 = frow == 0 ? -hx : frow == 2 ? -hy : -0.5f;
    const float sc1 = frow == 0 ? -0.5f : 1.f;
    const float sc2 = frow == 1 ? hx : frow == 3 ? hy : 1.f;
    const f2 zero = f2{0.f, 0.f};
    const int nitems = div_up((int)*maxtodo, SEG) * T_tiles;
    for (;;) {
        __syncthreads();  // the previous item's staged LDS and s_item are consumed
        if (tid == 0) s_item = (int)atomicAdd(queue, 1u);
        __syncthreads();
        const int item = s_item;
        if (item >= nitems) break;
        const int seg = item / T_tiles, tile = item - seg * T_tiles;
        const int todo = (int)tile_todo[tile];
        const int a = seg * SEG;
        if (a >= todo) continue;
        const int bnd = min(a + SEG, todo);  // the segment [a, bnd) of the tile's list
        const int tx0 = (tile % gx) * TILE_X, ty0 = (tile / gx) * TILE_Y;
        const int lx0 = lane & 7, ly = 8 * wv + (lane >> 3);
        const int px0 = tx0 + lx0, px1 = px0 + 8, py = ty0 + ly;
        const bool in0 = px0 < W && py < H, in1 = px1 < W && py < H;
        const f2 pfx = f2{(float)px0, (float)px1};
        const float pfy = (float)py;
        uint2 range = ranges[tile];
        range.x = min(range.x, cap);
        const int pid0 = py * W + px0, pid1 = py * W + px1;
        f2 Tfinal = f2{1.f, 1.f}, dp0 = zero, dp1 = zero, dp2 = zero;
        uint32_t last0 = 0, last1 = 0;
        f2 T = f2{1.f, 1.f}, acc0 = zero, acc1 = zero, acc2 = zero;
        const bool from_end = bnd == todo;
        const float4 *ck = from_end ? nullptr : ckpt + (size_t)ckpt_slot(range.x + (uint32_t)bnd) * TILE_PIX + ly * TILE_X + lx0;
        if (in0) {
            Tfinal.x = final_T[pid0];
            last0 = n_contrib[pid0];
            dp0.x = dL_dpix[pid0];
            dp1.x = dL_dpix[HW + pid0];
            dp2.x = dL_dpix[2 * HW + pid0];
            if (from_end) {
                T.x = Tfinal.x;
            } else {
                const float4 c = ck[0], f = cfin[pid0];
                const float it = 1.f / c.x;
                T.x = c.x;
                acc0.x = (f.y - c.y) * it;
                acc1.x = (f.z - c.z) * it;
                acc2.x = (f.w - c.w) * it;
            }
        }
        if (in1) {
            Tfinal.y = final_T[pid1];
            last1 = n_contrib[pid1];
            dp0.y = dL_dpix[pid1];
            dp1.y = dL_dpix[HW + pid1];
            dp2.y = dL_dpix[2 * HW + pid1];
            if (from_end) {
                T.y = Tfinal.y;
            } else {
                const float4 c = ck[8], f = cfin[pid1];
                const float it = 1.f / c.x;
                T.y = c.x;
                acc0.y = (f.y - c.y) * it;
                acc1.y = (f.z - c.z) * it;
                acc2.y = (f.w - c.w) * it;
            }
        }
        const f2 kbg = -Tfinal * (b0 * dp0 + b1 * dp1 + b2 * dp2);
        // stage the segment (<= SEG = B2 positions) back to front, tile-culled and compacted
        const int len = bnd - a;
        bool keep = false;
        uint32_t id = 0;
        float2 gl;
        float4 cl;
        if (tid < len) {
            id = vals[range.x + bnd - 1 - tid];
            gl = xy[id];
            cl = conic_o[id];
            keep = tile_reach(gl, cl, (float)tx0, (float)ty0);
        }
        const int2 sl = compact_slot_n<B2 / 64>(keep, tid, s_wcnt);
        if (keep) {
            s_id[sl.x] = id;
            s_xy[sl.x] = gl;
            s_co[sl.x] = cl;
            s_q[sl.x] = conic_q(cl);
            s_cd[sl.x] = rgbd[id];
            s_pos[sl.x] = tid;
        }
        __syncthreads();
        const int n = sl.y;
        for (int j = 0; j < n; j++) {
            const uint32_t contributor = (uint32_t)(bnd - 1 - s_pos[j]);  // position in the tile's list
            const float2 g = s_xy[j];
            const float4 q = s_q[j];
            const f2 dx = g.x - pfx;
            const float dy = g.y - pfy;
            const f2 power = f2{q_power(q, dx.x, dy), q_power(q, dx.y, dy)};
            const f2 G = f2{__builtin_amdgcn_exp2f(power.x), __builtin_amdgcn_exp2f(power.y)};
            const f2 alpha = f2{fminf(0.99f, q.w * G.x), fminf(0.99f, q.w * G.y)};
            const bool act0 = in0 && contributor < last0 && power.x <= 0.f && alpha.x >= 1.f / 255.f;
            const bool act1 = in1 && contributor < last1 && power.y <= 0.f && alpha.y >= 1.f / 255.f;
            if (__ballot(act0 || act1) == 0ull) continue;  // wave-uniform
            const float4 cd = s_cd[j];
            const float4 co = s_co[j];
            const f2 ae = sel2(act0, act1, alpha, zero);
            const f2 Ge = sel2(act0, act1, G, zero);
            const f2 om = 1.f - ae;
            f2 inv = f2{__builtin_amdgcn_rcpf(om.x), __builtin_amdgcn_rcpf(om.y)};
            inv = inv * (1.f - om * inv) + inv;
            T = T * inv;
            const f2 w = ae * T;
            const f2 d0 = cd.x - acc0, d1 = cd.y - acc1, d2 = cd.z - acc2;
            f2 dLda = d0 * dp0 + d1 * dp1 + d2 * dp2;
            acc0 = ae * d0 + acc0;
            acc1 = ae * d1 + acc1;
            acc2 = ae * d2 + acc2;
            dLda = dLda * T + kbg * inv;
            const f2 vop = Ge * dLda;
            const f2 u = co.w * vop;
            const f2 udx = u * dx, udy = u * dy;
            const f2 mxp = co.x * udx + co.y * udy, myp = co.y * udx + co.z * udy;
            const f2 cxp = udx * dx, cyp = udx * dy, czp = udy * dy;
            const f2 vr = w * dp0, vg = w * dp1, vb = w * dp2;
            const float w0 = row_sum15(fold16(fold32(mxp.x + mxp.y, myp.x + myp.y), fold32(cxp.x + cxp.y, cyp.x + cyp.y)));
            const float w1 = row_sum15(fold16(fold32(czp.x + czp.y, vop.x + vop.y), fold32(vr.x + vr.y, vg.x + vg.y)));
            const float w2 = row_sum15(fold16(fold32(vb.x + vb.y, 0.f),
                                              fold32(fabsf(mxp.x) + fabsf(mxp.y), fabsf(myp.x) + fabsf(myp.y))));
            if ((lane & 15) == 15) {
                const int row = lane >> 4;
                float *dst = acc + (size_t)s_id[j] * ACC_STRIDE + ((row & 1) << 1) + (row >> 1);
                atomicAdd(dst, w0 * sc0);
                atomicAdd(dst + 4, w1 * sc1);
                atomicAdd(dst + 8, w2 * sc2);
            }
        }
    }
    // the last workgroup to leave resets the queue for the next launch (every take has returned)
    if (tid == 0 && atomicAdd(queue + 1, 1u) == gridDim.x - 1) {
        atomicExch(queue, 0u);
        atomicExch(queue + 1, 0u);
    }
}

__device__ inline void dR_dq(float4 q, const float dR[9], float4 &dq) {
    float r = q.x, x = q.y, y = q.z, z = q.w;
    dq.x = 2.f * (-z * dR[1] + y * dR[2] + z * dR[3] - x * dR[5] - y * dR[6] + x * dR[7]);
    dq.y = 2.f * (y * dR[1] + z * dR[2] + y * dR[3] - r * dR[5] + z * dR[6] + r * dR[7]) - 4.f * x * (dR[4] + dR[8]);
    dq.z = 2.f * (x * dR[1] + r * dR[2] + x * dR[3] + z * dR[5] - r * dR[6] + z * dR[7]) - 4.f * y * (dR[0] + dR[8]);
    dq.w = 2.f * (-r * dR[1] + x * dR[2] + r * dR[3] + y * dR[5] + x * dR[6] + y * dR[7]) - 4.f * z * (dR[0] + dR[4]);
}

// one Gaussian's backward inputs, loaded before the block's SH staging so that they and the SH rows
// share one HBM round trip (the loads otherwise chained: accumulators -> radius -> scale / rotation)
struct PbIn {
    float4 a0, a1, a2;  // blend-backward accumulators (mx, my, cx, cy), (cz, op, r, g), (b, depth, dx, dy)
    float3 p, s;
    float4 q;
    int rad;
    uint8_t cl;
};

__device__ __forceinline__ void pb_load(PbIn &in, int i, const float *acc, const int *radii, const float *means3D,
                                        const float *scales, const float *rots, const float *cov_pre,
                                        const uint8_t *clamped) {
    const float *a = acc + (size_t)i * ACC_STRIDE;
    in.a0 = *reinterpret_cast<const float4 *>(a);
    in.a1 = *reinterpret_cast<const float4 *>(a + 4);
    in.a2 = *reinterpret_cast<const float4 *>(a + 8);
    in.rad = radii[i];
    in.p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
    in.s = make_float3(0.f, 0.f, 0.f);
    in.q = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!cov_pre) {
        in.s = make_float3(scales[3 * i], scales[3 * i + 1], scales[3 * i + 2]);
        in.q = *reinterpret_cast<const float4 *>(rots + 4 * i);
    }
    in.cl = clamped ? clamped[i] : (uint8_t)0;
}

// STAGE (degree-3 SH rows, M = 16, 16-byte aligned tensors): the block's SH rows (contiguous in
// HBM) are read into LDS with coalesced 16-byte loads, and its SH gradient rows are written back the
// same way (one thread per Gaussian would otherwise store 48 scattered words per row: 3x the HBM
// write traffic in partial lines).
template <bool STAGE>
__device__ __forceinline__ void preprocess_bwd_one(
    int i, int D, int M, const float *__restrict__ means3D, const float *__restrict__ scales, float mod,
    const float *__restrict__ rots, const float *__restrict__ cov_pre, const float *__restrict__ shs,
    const float *view, const float *proj, const float *campos, int W, int H, float tanx, float tany,
    float fx, float fy, const int *__restrict__ radii, const uint8_t *__restrict__ clamped,
    const float *__restrict__ acc, float *__restrict__ dL_dmeans3D, float *__restrict__ dL_dmeans2D,
    float *__restrict__ dL_ddens, float *__restrict__ dL_dcolors, float *__restrict__ dL_dopac,
    float *__restrict__ dL_dcov3D, float *__restrict__ dL_dshs, float *__restrict__ dL_dscales,
    float *__restrict__ dL_drots, float *s_row, float dsmul, const PbIn &in, const Cam &cam);

template <bool STAGE>
__global__ __launch_bounds__(256) void k_preprocess_bwd(
    int P, int D, int M, const float *__restrict__ means3D, const float *__restrict__ scales, float mod,
    const float *__restrict__ rots, const float *__restrict__ cov_pre, const float *__restrict__ shs,
    const float *view, const float *proj, const float *campos, int W, int H, float tanx, float tany,
    float fx, float fy, const int *__restrict__ radii, const uint8_t *__restrict__ clamped,
    const float *__restrict__ acc, float *__restrict__ dL_dmeans3D, float *__restrict__ dL_dmeans2D,
    float *__restrict__ dL_ddens, float *__restrict__ dL_dcolors, float *__restrict__ dL_dopac,
    float *__restrict__ dL_dcov3D, float *__restrict__ dL_dshs, float *__restrict__ dL_dscales,
    float *__restrict__ dL_drots, const float *__restrict__ shs_rest, float *__restrict__ dL_dshs_rest, float dsmul) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    [[maybe_unused]] const int b0 = blockIdx.x * blockDim.x, nrow = min(256, P - b0);
    [[maybe_unused]] float *s_row = nullptr;
    PbIn in;
    if (i < P) pb_load(in, i, acc, radii, means3D, scales, rots, cov_pre, clamped);
    Cam cam;
    load_cam(cam, view, proj, campos);
    if constexpr (STAGE) {
        __shared__ float s_sh[256 * SH_PAD];
        s_row = s_sh + threadIdx.x * SH_PAD;
        sh_stage_in(s_sh, shs, shs_rest, b0, nrow);
        __syncthreads();
        if (i < P) preprocess_bwd_one<STAGE>(i, D, M, means3D, scales, mod, rots, cov_pre, shs, view, proj, campos, W, H,
                                             tanx, tany, fx, fy, radii, clamped, acc, dL_dmeans3D, dL_dmeans2D, dL_ddens,
                                             dL_dcolors, dL_dopac, dL_dcov3D, dL_dshs, dL_dscales, dL_drots, s_row, dsmul,
                                             in, cam);
        __syncthreads();
        sh_stage_out(s_sh, dL_dshs, dL_dshs_rest, b0, nrow);
    } else {
        if (i < P) preprocess_bwd_one<STAGE>(i, D, M, means3D, scales, mod, rots, cov_pre, shs, view, proj, campos, W, H,
                                             tanx, tany, fx, fy, radii, clamped, acc, dL_dmeans3D, dL_dmeans2D, dL_ddens,
                                             dL_dcolors, dL_dopac, dL_dcov3D, dL_dshs, dL_dscales, dL_drots, nullptr, dsmul,
                                             in, cam);
    }
}

// one Gaussian of k_preprocess_bwd; STAGE: its SH row is s_row in LDS, overwritten by its gradient
template <bool STAGE>
__device__ __forceinline__ void preprocess_bwd_one(
    int i, int D, int M, const float *__restrict__ means3D, const float *__restrict__ scales, float mod,
    const float *__restrict__ rots, const float *__restrict__ cov_pre, const float *__restrict__ shs,
    const float *view, const float *proj, const float *campos, int W, int H, float tanx, float tany,
    float fx, float fy, const int *__restrict__ radii, const uint8_t *__restrict__ clamped,
    const float *__restrict__ acc, float *__restrict__ dL_dmeans3D, float *__restrict__ dL_dmeans2D,
    float *__restrict__ dL_ddens, float *__restrict__ dL_dcolors, float *__restrict__ dL_dopac,
    float *__restrict__ dL_dcov3D, float *__restrict__ dL_dshs, float *__restrict__ dL_dscales,
    float *__restrict__ dL_drots, float *s_row, float dsmul, const PbIn &in, const Cam &cam) {
    const float4 a0 = in.a0, a1 = in.a1, a2 = in.a2;
    // a0 = (mx, my, cx, cy), a1 = (cz, op, r, g), a2 = (b, depth, dx, dy)
    dL_dmeans2D[3 * i] = a0.x;
    dL_dmeans2D[3 * i + 1] = a0.y;
    dL_dmeans2D[3 * i + 2] = 0.f;
    dL_ddens[3 * i] = a2.z;
    dL_ddens[3 * i + 1] = a2.w;
    dL_ddens[3 * i + 2] = 0.f;
    dL_dopac[i] = a1.y;
    if (dL_dcolors) {
        dL_dcolors[3 * i] = a1.z;
        dL_dcolors[3 * i + 1] = a1.w;
        dL_dcolors[3 * i + 2] = a2.x;
    }
    const bool vis = in.rad > 0;
    const float3 p = in.p;
    float dm0 = 0.f, dm1 = 0.f, dm2 = 0.f;
    float dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float c3[6];
    const float3 s3 = in.s;
    const float4 q = in.q;
    if (vis) {
        if (cov_pre) {
#pragma unroll
            for (int k = 0; k < 6; k++) c3[k] = cov_pre[6 * i + k];
        } else {
            cov3d(s3, mod, q, c3);
        }
        float3 tv = xform43(cam.v, p);
        Ewa e;
        ewa_T(tv, fx, fy, tanx, tany, cam.v, e);
        const float *Tm = e.T;
        float3 c2 = cov2d(e, c3);
        float A = c2.x, B = c2.y, Cc = c2.z;
        float den = A * Cc - B * B;
        float d2i = 1.f / (den * den + 0.0000001f);
        float gcx = a0.z, gcy = a0.w, gcz = a1.x;
        float dLa = 0.f, dLb = 0.f, dLc = 0.f;
        if (d2i != 0.f) {
            dLa = d2i * (-Cc * Cc * gcx + 2.f * B * Cc * gcy + (den - A * Cc) * gcz);
            dLc = d2i * (-A * A * gcz + 2.f * A * B * gcy + (den - A * Cc) * gcx);
            dLb = d2i * 2.f * (B * Cc * gcx - (den + 2.f * B * B) * gcy + A * B * gcz);
        }
        dcov[0] = Tm[0] * Tm[0] * dLa + Tm[0] * Tm[3] * dLb + Tm[3] * Tm[3] * dLc;
        dcov[3] = Tm[1] * Tm[1] * dLa + Tm[1] * Tm[4] * dLb + Tm[4] * Tm[4] * dLc;
        dcov[5] = Tm[2] * Tm[2] * dLa + Tm[2] * Tm[5] * dLb + Tm[5] * Tm[5] * dLc;
        dcov[1] = 2.f * Tm[0] * Tm[1] * dLa + (Tm[0] * Tm[4] + Tm[1] * Tm[3]) * dLb + 2.f * Tm[3] * Tm[4] * dLc;
        dcov[2] = 2.f * Tm[0] * Tm[2] * dLa + (Tm[0] * Tm[5] + Tm[2] * Tm[3]) * dLb + 2.f * Tm[3] * Tm[5] * dLc;
        dcov[4] = 2.f * Tm[2] * Tm[1] * dLa + (Tm[1] * Tm[5] + Tm[2] * Tm[4]) * dLb + 2.f * Tm[4] * Tm[5] * dLc;
        float V[9] = {c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]};
        float dT[6];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            float v0 = V[k * 3] * Tm[0] + V[k * 3 + 1] * Tm[1] + V[k * 3 + 2] * Tm[2];
            float v1 = V[k * 3] * Tm[3] + V[k * 3 + 1] * Tm[4] + V[k * 3 + 2] * Tm[5];
            dT[k] = 2.f * v0 * dLa + v1 * dLb;
            dT[3 + k] = 2.f * v1 * dLc + v0 * dLb;
        }
        const float *vm = cam.v;
        // W rows: W0 = (vm0, vm4, vm8), W1 = (vm1, vm5, vm9), W2 = (vm2, vm6, vm10)
        float dJ00 = vm[0] * dT[0] + vm[4] * dT[1] + vm[8] * dT[2];
        float dJ02 = vm[2] * dT[0] + vm[6] * dT[1] + vm[10] * dT[2];
        float dJ11 = vm[1] * dT[3] + vm[5] * dT[4] + vm[9] * dT[5];
        float dJ12 = vm[2] * dT[3] + vm[6] * dT[4] + vm[10] * dT[5];
        float tz = e.tz;
        float tz2 = 1.f / (tz * tz), tz3 = tz2 / tz;
        float dtx = e.mx * -fx * tz2 * dJ02;
        float dty = e.my * -fy * tz2 * dJ12;
        float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2.f * fx * e.tx) * tz3 * dJ02 + (2.f * fy * e.ty) * tz3 * dJ12;
        dtz += a2.y;  // depth output: depth = t.z
        dm0 += vm[0] * dtx + vm[1] * dty + vm[2] * dtz;
        dm1 += vm[4] * dtx + vm[5] * dty + vm[6] * dtz;
        dm2 += vm[8] * dtx + vm[9] * dty + vm[10] * dtz;
        // projection: mean2D (NDC) -> mean3D
        const float *pj = cam.p;
        float4 ph = xform44(pj, p);
        float mw = 1.f / (ph.w + 0.0000001f);
        float mul1 = ph.x * mw * mw, mul2 = ph.y * mw * mw;
        float gx_ = a0.x, gy_ = a0.y;
        dm0 += (pj[0] * mw - pj[3] * mul1) * gx_ + (pj[1] * mw - pj[3] * mul2) * gy_;
        dm1 += (pj[4] * mw - pj[7] * mul1) * gx_ + (pj[5] * mw - pj[7] * mul2) * gy_;
        dm2 += (pj[8] * mw - pj[11] * mul1) * gx_ + (pj[9] * mw - pj[11] * mul2) * gy_;
    }
    // SH backward (also writes zeros for culled Gaussians)
    if (shs) {
        float *dsh = STAGE ? s_row : dL_dshs + (size_t)i * M * 3;
        if (!vis) {
            for (int k = 0; k < M * 3; k++) dsh[k] = 0.f;
        } else {
            float shr[STAGE ? SH_ROW : 1];  // STAGE: the row in registers (the LDS row is overwritten)
            const float *sh = shs + (size_t)i * M * 3;
            if constexpr (STAGE) {
#pragma unroll
                for (int k = 0; k < SH_ROW; k++) shr[k] = s_row[k];
                sh = shr;
            }
            float vx = p.x - cam.c[0], vy = p.y - cam.c[1], vz = p.z - cam.c[2];
            float n = sqrtf(vx * vx + vy * vy + vz * vz);
            float x = vx / n, y = vy / n, z = vz / n;
            const uint8_t cl = in.cl;
            float g3[3] = {(cl & 1) ? 0.f : a1.z, (cl & 2) ? 0.f : a1.w, (cl & 4) ? 0.f : a2.x};
            float ddx = 0.f, ddy = 0.f, ddz = 0.f;
            float xx = x * x, yy = y * y, zz = z * z, xy_ = x * y, yz = y * z, xz = x * z;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                float g = g3[c];
#define SHV(k) sh[(k) * 3 + c]
                dsh[c] = SH_C0 * g;
                float gxx = 0.f, gyy = 0.f, gzz = 0.f;
                if (D > 0) {
                    dsh[3 + c] = -SH_C1 * y * g;
                    dsh[6 + c] = SH_C1 * z * g;
                    dsh[9 + c] = -SH_C1 * x * g;
                    gxx = -SH_C1 * SHV(3);
                    gyy = -SH_C1 * SHV(1);
                    gzz = SH_C1 * SHV(2);
                    if (D > 1) {
                        dsh[12 + c] = SH_C2_0 * xy_ * g;
                        dsh[15 + c] = SH_C2_1 * yz * g;
                        dsh[18 + c] = SH_C2_2 * (2.f * zz - xx - yy) * g;
                        dsh[21 + c] = SH_C2_3 * xz * g;
                        dsh[24 + c] = SH_C2_4 * (xx - yy) * g;
                        gxx += SH_C2_0 * y * SHV(4) + SH_C2_2 * 2.f * -x * SHV(6) + SH_C2_3 * z * SHV(7) + SH_C2_4 * 2.f * x * SHV(8);
                        gyy += SH_C2_0 * x * SHV(4) + SH_C2_1 * z * SHV(5) + SH_C2_2 * 2.f * -y * SHV(6) + SH_C2_4 * 2.f * -y * SHV(8);
                        gzz += SH_C2_1 * y * SHV(5) + SH_C2_2 * 2.f * 2.f * z * SHV(6) + SH_C2_3 * x * SHV(7);
                        if (D > 2) {
                            dsh[27 + c] = SH_C3_0 * y * (3.f * xx - yy) * g;
                            dsh[30 + c] = SH_C3_1 * xy_ * z * g;
                            dsh[33 + c] = SH_C3_2 * y * (4.f * zz - xx - yy) * g;
                            dsh[36 + c] = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy) * g;
                            dsh[39 + c] = SH_C3_4 * x * (4.f * zz - xx - yy) * g;
                            dsh[42 + c] = SH_C3_5 * z * (xx - yy) * g;
                            dsh[45 + c] = SH_C3_6 * x * (xx - 3.f * yy) * g;
                            gxx += SH_C3_0 * SHV(9) * 3.f * 2.f * xy_ + SH_C3_1 * SHV(10) * yz + SH_C3_2 * SHV(11) * -2.f * xy_ +
                                   SH_C3_3 * SHV(12) * -3.f * 2.f * xz + SH_C3_4 * SHV(13) * (-3.f * xx + 4.f * zz - yy) +
                                   SH_C3_5 * SHV(14) * 2.f * xz + SH_C3_6 * SHV(15) * 3.f * (xx - yy);
                            gyy += SH_C3_0 * SHV(9) * 3.f * (xx - yy) + SH_C3_1 * SHV(10) * xz +
                                   SH_C3_2 * SHV(11) * (-3.f * yy + 4.f * zz - xx) + SH_C3_3 * SHV(12) * -3.f * 2.f * yz +
                                   SH_C3_4 * SHV(13) * -2.f * xy_ + SH_C3_5 * SHV(14) * -2.f * yz + SH_C3_6 * SHV(15) * -3.f * 2.f * xy_;
                            gzz += SH_C3_1 * SHV(10) * xy_ + SH_C3_2 * SHV(11) * 4.f * 2.f * yz +
                                   SH_C3_3 * SHV(12) * 3.f * (2.f * zz - xx - yy) + SH_C3_4 * SHV(13) * 4.f * 2.f * xz +
                                   SH_C3_5 * SHV(14) * (xx - yy);
                        }
                    }
                }
#undef SHV
                ddx += gxx * g;
                ddy += gyy * g;
                ddz += gzz * g;
            }
            int kmax = (D + 1) * (D + 1);
            for (int k = kmax; k < M; k++) {
                dsh[3 * k] = 0.f;
                dsh[3 * k + 1] = 0.f;
                dsh[3 * k + 2] = 0.f;
            }
            float s2 = vx * vx + vy * vy + vz * vz;
            float inv32 = 1.f / sqrtf(s2 * s2 * s2);
            dm0 += ((s2 - vx * vx) * ddx - vy * vx * ddy - vz * vx * ddz) * inv32;
            dm1 += (-vx * vy * ddx + (s2 - vy * vy) * ddy - vz * vy * ddz) * inv32;
            dm2 += (-vx * vz * ddx - vy * vz * ddy + (s2 - vz * vz) * ddz) * inv32;
        }
    }
    dL_dmeans3D[3 * i] = dm0;
    dL_dmeans3D[3 * i + 1] = dm1;
    dL_dmeans3D[3 * i + 2] = dm2;
    if (cov_pre) {
        if (dL_dcov3D)
            for (int k = 0; k < 6; k++) dL_dcov3D[6 * i + k] = dcov[k];
    } else {
        float ds0 = 0.f, ds1 = 0.f, ds2 = 0.f;
        float4 dq = make_float4(0.f, 0.f, 0.f, 0.f);
        if (vis) {
            float R[9];
            quat_to_R(q, R);
            float sp[3] = {mod * s3.x, mod * s3.y, mod * s3.z};
            float G[9] = {dcov[0], 0.5f * dcov[1], 0.5f * dcov[2], 0.5f * dcov[1], dcov[3], 0.5f * dcov[4],
                          0.5f * dcov[2], 0.5f * dcov[4], dcov[5]};
            float L[9];
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int k = 0; k < 3; k++) L[r * 3 + k] = R[r * 3 + k] * sp[k];
            float dRm[9];
            float ds[3];
#pragma unroll
            for (int k = 0; k < 3; k++) {
                float acc_s = 0.f;
#pragma unroll
                for (int r = 0; r < 3; r++) {
                    float dl = 2.f * (G[r * 3] * L[k] + G[r * 3 + 1] * L[3 + k] + G[r * 3 + 2] * L[6 + k]);
                    acc_s += dl * R[r * 3 + k];
                    dRm[r * 3 + k] = dl * sp[k];
                }
                ds[k] = acc_s * dsmul;  // upstream: dL/d(mod s) (dsmul = 1); exact: dL/ds (dsmul = mod)
            }
            ds0 = ds[0]; ds1 = ds[1]; ds2 = ds[2];
            dR_dq(q, dRm, dq);
        }
        dL_dscales[3 * i] = ds0;
        dL_dscales[3 * i + 1] = ds1;
        dL_dscales[3 * i + 2] = ds2;
        *reinterpret_cast<float4 *>(dL_drots + 4 * i) = dq;
    }
}

__global__ __launch_bounds__(256) void k_mark_visible(int P, const float *__restrict__ means3D, const float *view,
                                                      uint8_t *__restrict__ visible) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    float3 p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
    float3 pv = make_float3(0.f, 0.f, view[2] * p.x + view[6] * p.y + view[10] * p.z + view[14]);
    visible[i] = pv.z > 0.2f;
}

}  // namespace dgs

// ================================================================================================
// host side: context pool and C ABI
// ================================================================================================
using namespace dgs;

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) DGS_HIP_CHECK(hipFree(p));
        size_t nb = bytes + bytes / 4 + 4096;
        p = nullptr;
        DGS_HIP_CHECK(hipMalloc(&p, nb));
        cap = nb;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct dgs_raster_ctx {
    int device = 0;
    dgs_raster_settings s{};
    int P = 0, M = 0, H = 0, W = 0, gx = 0, gy = 0, num_rendered = 0;
    const float *means3D = nullptr, *shs = nullptr, *colors = nullptr, *opac = nullptr, *scales = nullptr,
                *rots = nullptr, *cov = nullptr;
    const float *shs_rest = nullptr;  // split SH rows (dgs_raster_forward_split_sh): shs = features_dc
    DevBuf geom, bin, img, acc, tmp, rect;
    // k_rect_colscan's generation-tagged tile totals: a buffer of their own, zeroed whenever it is
    // (re)allocated, so it only ever holds 0 or words a colscan launch wrote (never stale count-matrix
    // data whose upper half could equal the current generation)
    DevBuf rtot;
    // segmented blend backward (DGS_BLEND_SEG): the forward's per-pixel checkpoints every SEG list
    // positions, and [work queue (2) | maxtodo | - | tile_todo (T)] (zeroed when (re)allocated; the
    // queue resets itself at the end of every launch, maxtodo is zeroed by k_rect_count)
    DevBuf ckb, segq;
    // deterministic blend backward (dgs_raster_set_deterministic): [tile_todo (T, padded) | per-pair slots]
    DevBuf det;
    bool seg_ok = false;  // this forward wrote the checkpoints
    float4 *cfin = nullptr;  // the forward's final (T, C) per pixel (segmented backward)
    bool bwd_done = false;  // a backward already consumed the accumulators (a second one re-zeroes them)
    // carved views
    float2 *xy = nullptr;
    float4 *conic_o = nullptr, *rgbd = nullptr;
    uint32_t *tiles = nullptr, *offsets = nullptr;  // offsets: inclusive scan in depth order
    uint32_t *dkey = nullptr, *dkey_alt = nullptr, *gid = nullptr, *order = nullptr, *tiles_sorted = nullptr;
    uint8_t *clamped = nullptr;
    uint32_t *vals = nullptr;
    bool rect_mode = false;  // rect binning (k_rect_*) instead of duplicate + tile sort
    bool tsort = false;      // rect binning in index order + per-tile depth sort (k_tile_sort), no global depth sort
    bool det_fwd = false;    // deterministic mode at the forward: the det buffer holds the tile sort's position map
    int det_cap = 0;         // the pair capacity the det buffer was laid out for
    uint32_t *rect_cnt = nullptr, *rect_start = nullptr, *rect_total = nullptr;
    unsigned long long *rect_tot = nullptr;  // tile totals tagged with a launch generation (k_rect_colscan)
    uint2 *ranges = nullptr;
    float *final_T = nullptr;
    uint32_t *n_contrib = nullptr;
    int *radii = nullptr;
    hipEvent_t released = nullptr;
    hipStream_t last_stream = nullptr;
    bool pending_release = false;
    uint32_t *h_total = nullptr;  // pinned host word: the num_rendered read-back (no staging copy)
    uint32_t *d_total = nullptr;  // its device address (k_rect_colscan writes the count there)
    bool count_pending = false;   // deferred count: num_rendered not read yet (resolve_count)
    int spec_cap = 0;              // the speculative capacity the binning ran with
    hipEvent_t count_ev = nullptr;  // recorded after the read-back copy
};

namespace {
std::mutex g_pool_mu;
std::vector<dgs_raster_ctx *> g_pool;

size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// DGS_BLEND1=1: the one-pixel-per-lane blend backward (k_blend_bwd, 4 waves per tile) instead of the
// packed two-pixel one (k_blend_bwd2, the default)
bool blend_one_pixel() {
    static const bool v = [] {
        const char *e = getenv("DGS_BLEND1");
        return e && e[0] == '1';
    }();
    return v;
}

// DGS_BLEND_SEG=1: segmented blend backward (k_blend_bwd2s: SEG-long segments of every tile's list as
// independent work items, from checkpoints the forward leaves) instead of k_blend_bwd2's one serial
// replay per tile
std::atomic<int> g_blend_seg{-1};  // -1: not decided yet (DGS_BLEND_SEG), else dgs_debug_set_blend_seg
bool blend_segmented() {
    int v = g_blend_seg.load();
    if (v < 0) {
        const char *e = getenv("DGS_BLEND_SEG");
        int want = e && e[0] == '1' ? 1 : 0;
        g_blend_seg.compare_exchange_strong(v, want);
        v = g_blend_seg.load();
    }
    return v == 1;
}

// DGS_DETERMINISTIC=1 / dgs_raster_set_deterministic(1): the blend backward (rect binning) writes per-pair
// slots that k_rect_gather sums in a fixed order instead of float atomics into acc: bitwise reproducible
// gradients at the cost of the slot traffic (96 B per pair written and read)
std::atomic<int> g_det{-1};
bool blend_deterministic() {
    int v = g_det.load();
    if (v < 0) {
        const char *e = getenv("DGS_DETERMINISTIC");
        int want = e && e[0] == '1' ? 1 : 0;
        g_det.compare_exchange_strong(v, want);
        v = g_det.load();
    }
    return v == 1;
}

// DGS_BLEND_FWD2=1 / dgs_debug_set_blend_fwd2: the two-pixels-per-lane forward blend (k_blend_fwd2)
std::atomic<int> g_fwd2{-1};
bool blend_fwd2() {
    int v = g_fwd2.load();
    if (v < 0) {
        const char *e = getenv("DGS_BLEND_FWD2");
        int want = e && e[0] == '1' ? 1 : 0;
        g_fwd2.compare_exchange_strong(v, want);
        v = g_fwd2.load();
    }
    return v == 1;
}

// DGS_TILE_SORT=0: rect binning over the global depth sort's order (k_rect_* on depth-ordered Gaussians)
// instead of index order + the per-tile depth sort (k_tile_sort, the default); dgs_debug_set_tile_sort
std::atomic<int> g_tile_sort{-1};
bool tile_sort_enabled() {
    int v = g_tile_sort.load();
    if (v < 0) {
        const char *e = getenv("DGS_TILE_SORT");
        int want = e && e[0] == '0' ? 0 : 1;
        g_tile_sort.compare_exchange_strong(v, want);
        v = g_tile_sort.load();
    }
    return v == 1;
}

// DGS_HIPCUB_SORT=1: hipcub::DeviceRadixSort for the depth and tile sorts instead of radix.hip
bool hipcub_sort() {
    static const bool v = [] {
        const char *e = getenv("DGS_HIPCUB_SORT");
        return e && e[0] == '1';
    }();
    return v;
}

// Binning mode: 0 = rect binning up to RECT_MAX_TILES tiles and RECT_MAX_CELLS count-matrix cells
// (the default), 1 = duplicate + tile-key radix sort + ranges for every image. Initialized from
// DGS_BINNING=sort (or DGS_HIPCUB_SORT=1); dgs_debug_set_binning switches it at run time.
std::atomic<int> g_binning{-1};

int binning_mode() {
    int m = g_binning.load();
    if (m < 0) {
        const char *e = getenv("DGS_BINNING");
        m = ((e && strcmp(e, "sort") == 0) || hipcub_sort()) ? 1 : 0;
        g_binning.store(m);
    }
    return m;
}

// process-wide launch generations of k_rect_colscan: a tag never repeats across contexts whose
// buffers may be recycled
uint32_t next_rect_gen() {
    static std::atomic<uint32_t> g{0};
    uint32_t v = ++g;
    if (v == 0) v = ++g;
    return v;
}

bool rect_binning(int gx, int gy, int P) {
    const int T = gx * gy;
    return binning_mode() == 0 && T <= RECT_MAX_TILES && rect_place_lds(gx, gy, false) <= 65536 &&
           (long long)div_up(P, 256) * T <= RECT_MAX_CELLS;
}

// hipcub temp-storage sizes, cached per (device, size class): the size queries cost tens of us of
// host time each inside the num_rendered sync window. Sizes are queried for the class's upper end
// (temp storage grows monotonically with the item count).
std::mutex g_tmp_mu;
std::map<std::tuple<int, int, int, int>, size_t> g_tmp_sizes;  // (kind, device, class, end_bit)

int size_class(int n) {  // 1/16-octave classes
    if (n <= 4096) return 0;
    int hb = 31 - __builtin_clz((unsigned)n);
    int frac = (int)(((unsigned long long)n << 4 >> hb) & 15);
    return hb * 16 + frac + 1;
}
int class_upper(int cls) {
    if (cls == 0) return 4096;
    int hb = (cls - 1) / 16, frac = (cls - 1) % 16;
    unsigned long long v = ((16ull + frac + 1) << hb) >> 4;
    return v > 0x7fffffffull ? 0x7fffffff : (int)v;
}

// Speculative pair capacity per device: binning is launched for this many pairs before the host
// knows num_rendered, so the CPU does not drain the GPU queue at the read-back (it waits on an
// event recorded right after the scan while duplicate/sort/blend run). A count above the capacity
// re-runs binning with a grown capacity (results are always exact).
std::mutex g_cap_mu;
std::map<int, int> g_pair_cap;
long long g_redos = 0;  // overflowing speculative launches redone at the exact size (debug counter)

int grown_cap(long long nr) {
    long long c = nr + nr / 8 + 65536;
    return (int)std::min<long long>(c, 0x7fffffffLL);
}

int pair_cap_get(int device) {
    std::lock_guard<std::mutex> lk(g_cap_mu);
    auto it = g_pair_cap.find(device);
    return it == g_pair_cap.end() ? 0 : it->second;
}

void pair_cap_observe(int device, int nr) {
    std::lock_guard<std::mutex> lk(g_cap_mu);
    int &c = g_pair_cap[device];
    const int want = grown_cap(nr);
    if (want > c || (long long)nr * 2 < c) c = want;  // grow at once; shrink when far above
}

hipError_t scan_tmp_bytes(int device, int P, hipStream_t stream, size_t &bytes) {
    const int cls = size_class(P);
    std::lock_guard<std::mutex> lk(g_tmp_mu);
    auto key = std::make_tuple(0, device, cls, 0);
    auto it = g_tmp_sizes.find(key);
    if (it != g_tmp_sizes.end()) { bytes = it->second; return hipSuccess; }
    hipError_t e = hipcub::DeviceScan::InclusiveSum(nullptr, bytes, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                    class_upper(cls), stream);
    if (e == hipSuccess) g_tmp_sizes[key] = bytes;
    return e;
}

// radix-sort temp bytes for (KT keys, u32 values), cached per (key type, device, size class, bits)
template <class KT>
hipError_t sort_tmp_bytes(int device, int n, int end_bit, hipStream_t stream, size_t &bytes) {
    const int cls = size_class(n);
    std::lock_guard<std::mutex> lk(g_tmp_mu);
    auto key = std::make_tuple((int)sizeof(KT), device, cls, end_bit);
    auto it = g_tmp_sizes.find(key);
    if (it != g_tmp_sizes.end()) { bytes = it->second; return hipSuccess; }
    hipcub::DoubleBuffer<KT> kb(nullptr, nullptr);
    hipcub::DoubleBuffer<uint32_t> vb(nullptr, nullptr);
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, kb, vb, class_upper(cls), 0, end_bit, stream);
    if (e == hipSuccess) g_tmp_sizes[key] = bytes;
    return e;
}

int bits_for(uint32_t n) {
    int b = 0;
    while (n) {
        b++;
        n >>= 1;
    }
    return b;
}

dgs_raster_ctx *ctx_acquire(int device, hipStream_t stream) {
    dgs_raster_ctx *c = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t k = 0; k < g_pool.size(); k++) {
            if (g_pool[k]->device == device) {
                c = g_pool[k];
                g_pool.erase(g_pool.begin() + k);
                break;
            }
        }
    }
    if (!c) {
        c = new dgs_raster_ctx();
        c->device = device;
    }
    if (c->pending_release) {
        // the previous user's work on its stream precedes this one in stream order when the stream
        // is the same (the training loop): no marker at all (each costs ~6 us of GPU idle);
        // otherwise order this stream after everything queued on that stream so far
        if (c->last_stream != stream) {
            if (!c->released) (void)hipEventCreateWithFlags(&c->released, hipEventDisableTiming);
            (void)hipEventRecord(c->released, c->last_stream);
            (void)hipStreamWaitEvent(stream, c->released, 0);
        }
        c->pending_release = false;
    }
    return c;
}
}  // namespace

// The pair count of this frame on the host. Sort binning: the pinned word behind count_ev. Rect
// binning: k_rect_colscan stores the count into the coherent pinned word itself, so the host polls
// the word (no event record in the stream: one costs ~6 us of GPU idle). Only a wait longer than
// 20 ms queries the stream (then every 1024 polls), so a failed launch cannot spin forever: a query
// of a busy stream appends a completion marker at its tail, which cost ~6 us of GPU idle before the
// next launch (the optimizer's, when the native step waits for its own count at its end) on every step
// when the stream was queried every 1024 polls (profiles/r5ts_trace_summary.txt).
constexpr uint32_t COUNT_PENDING = 0xffffffffu;
std::atomic<long long> g_count_wait_ns{0}, g_count_waits{0};  // host time spent waiting for num_rendered

static int wait_count_impl(dgs_raster_ctx *c, hipStream_t stream, int &nr);
static int wait_count(dgs_raster_ctx *c, hipStream_t stream, int &nr) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = wait_count_impl(c, stream, nr);
    g_count_wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    g_count_waits++;
    return rc;
}

static int wait_count_impl(dgs_raster_ctx *c, hipStream_t stream, int &nr) {
    if (!c->rect_mode) {
        DGS_HIP_CHECK(hipEventSynchronize(c->count_ev));
        nr = (int)*c->h_total;
        return DGS_OK;
    }
    volatile uint32_t *w = c->h_total;
    const auto t0 = std::chrono::steady_clock::now();
    bool slow = false;
    for (uint32_t i = 1;; i++) {
        uint32_t v = *w;
        if (v == COUNT_PENDING && (i & 1023) == 0 && !slow)
            slow = std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20);
        if (v == COUNT_PENDING && (i & 1023) == 0 && slow) {
            const hipError_t e = hipStreamQuery(stream);
            if (e == hipSuccess) {
                v = *w;
                if (v == COUNT_PENDING) {
                    set_error("dgs_raster_forward: pair count not written by k_rect_colscan");
                    return DGS_ERR_HIP;
                }
            } else if (e != hipErrorNotReady) {
                DGS_HIP_CHECK(e);
            }
        }
        if (v != COUNT_PENDING) {
            std::atomic_thread_fence(std::memory_order_acquire);
            nr = (int)v;
            return DGS_OK;
        }
        __builtin_ia32_pause();
    }
}

// Binning for `cap` pairs (>= num_rendered, or the speculative capacity) + the blend: the key
// buffer is pre-filled with all-ones (past every tile id, so the unused tail sorts last and leaves
// the stable order of the real pairs untouched), bounded duplicate in depth order, stable radix sort
// of cap items on the tile bits, ranges from the device-side count, forward blend.
template <class KT>
static int bin_tiles(dgs_raster_ctx *c, int cap, int P, int device, hipStream_t stream, bool dbg) {
    const int T = c->gx * c->gy;
    const int end_bit = bits_for((uint32_t)T);
    const bool cub = hipcub_sort();
    size_t sort_tmp = 0;
    if (cub) DGS_HIP_CHECK(sort_tmp_bytes<KT>(device, cap, end_bit, stream, sort_tmp));
    size_t o_k0 = 0, o_k1 = align_up(sizeof(KT) * cap), o_v0 = align_up(o_k1 + sizeof(KT) * cap),
           o_v1 = align_up(o_v0 + 4ull * cap), o_t = align_up(o_v1 + 4ull * cap);
    if (int rc = c->bin.ensure(o_t + sort_tmp + 256)) return rc;
    char *b = (char *)c->bin.p;
    KT *k0 = (KT *)(b + o_k0), *k1 = (KT *)(b + o_k1);
    uint32_t *v0 = (uint32_t *)(b + o_v0), *v1 = (uint32_t *)(b + o_v1);
    {
        ScopedTimer tm("duplicate", stream);
        hipLaunchKernelGGL(k_duplicate<KT>, dim3(div_up(P, 256)), dim3(256), 0, stream, P, c->order, c->xy, c->radii,
                           c->offsets, c->gx, c->gy, k0, v0, (uint32_t)cap, c->ranges, c->gx * c->gy);
    }
    DGS_LAUNCH_CHECK("k_duplicate", dbg, stream);
    KT *ksorted = k0;
    {
        ScopedTimer tm("sort", stream);
        if (cub) {
            hipcub::DoubleBuffer<KT> kbuf(k0, k1);
            hipcub::DoubleBuffer<uint32_t> vbuf(v0, v1);
            DGS_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(b + o_t, sort_tmp, kbuf, vbuf, cap, 0, end_bit, stream));
            c->vals = vbuf.Current();
            ksorted = kbuf.Current();
        } else {
            int alt = 0;
            if (int rc = radix::sort_pairs<KT>(k0, k1, v0, v1, cap, end_bit, stream, &alt)) return rc;
            c->vals = alt ? v1 : v0;
            ksorted = alt ? k1 : k0;
        }
    }
    {
        ScopedTimer tm("ranges", stream);
        hipLaunchKernelGGL(k_ranges<KT>, dim3(div_up(cap, 256)), dim3(256), 0, stream, c->offsets + (P - 1),
                           (uint32_t)cap, ksorted, c->ranges);
    }
    DGS_LAUNCH_CHECK("k_ranges", dbg, stream);
    return DGS_OK;
}

// The deterministic mode's buffer for a pair capacity: [tile end (T, padded) | per-pair slots (12 floats)
// | the tile sort's position map (1 word per pair)], laid out for the capacity the forward binned with
static int det_layout(dgs_raster_ctx *c, int cap, uint32_t **tile_end, float **slot, uint32_t **pre) {
    const size_t T = (size_t)c->gx * c->gy, tpad = (T + 63) & ~(size_t)63, n = (size_t)std::max(cap, 1);
    if (int rc = c->det.ensure(4ull * tpad + 52ull * n)) return rc;
    c->det_cap = cap;
    uint32_t *te = (uint32_t *)c->det.p;
    float *sl = (float *)(te + tpad);
    if (tile_end) *tile_end = te;
    if (slot) *slot = sl;
    if (pre) *pre = (uint32_t *)(sl + 12 * n);
    return DGS_OK;
}

static int bin_and_blend(dgs_raster_ctx *c, int cap, int P, int device, hipStream_t stream, bool dbg, float *out_color,
                         float *out_depth) {
    const int T = c->gx * c->gy;
    if (c->rect_mode) {
        // tile sort: the lists, then 8 + 4 (+ 4: the deterministic mode's copy) bytes of scratch per pair for
    // lists longer than k_tile_sort's LDS
        const size_t vbytes = align_up(4ull * std::max(cap, 1) + 256);
        if (int rc = c->bin.ensure(vbytes + (c->tsort ? 16ull * std::max(cap, 1) + 256 : 0))) return rc;
        c->vals = (uint32_t *)c->bin.p;
        const int nb = div_up(P, 256);
        if (cap > 0) {
            ScopedTimer tm("place", stream);
            const bool stage = rect_place_stage(c->gx, c->gy);
            hipLaunchKernelGGL(k_rect_place, dim3(nb), dim3(256), rect_place_lds(c->gx, c->gy, stage), stream, P,
                               c->tsort ? nullptr : c->order, c->xy, c->radii, c->gx, c->gy, c->rect_cnt, c->rect_start,
                               (uint32_t)cap, c->vals, (int)stage);
        }
        DGS_LAUNCH_CHECK("k_rect_place", dbg, stream);
        if (cap > 0 && c->tsort) {
            ScopedTimer tm("tile_sort", stream);
            unsigned long long *scr = (unsigned long long *)((char *)c->bin.p + vbytes);
            uint32_t *spos = (uint32_t *)(scr + std::max(cap, 1)), *vorig = spos + std::max(cap, 1);
            if (c->det_fwd) {
                uint32_t *pre = nullptr;
                if (int rc = det_layout(c, cap, nullptr, nullptr, &pre)) return rc;
                hipLaunchKernelGGL(k_tile_sort<true>, dim3(T), dim3(TS_THR), 0, stream, c->ranges, (uint32_t)cap, c->dkey,
                                   c->vals, scr, spos, pre, vorig);
            } else {
                hipLaunchKernelGGL(k_tile_sort<false>, dim3(T), dim3(TS_THR), 0, stream, c->ranges, (uint32_t)cap, c->dkey,
                                   c->vals, scr, spos, nullptr, nullptr);
            }
            DGS_LAUNCH_CHECK("k_tile_sort", dbg, stream);
        }
    } else if (cap > 0) {  // k_duplicate clears c->ranges
        // 16-bit tile keys up to 65535 tiles (4080 x 4080 pixels), 32-bit beyond
        const int rc = T < 65535 ? bin_tiles<uint16_t>(c, cap, P, device, stream, dbg)
                                 : bin_tiles<uint32_t>(c, cap, P, device, stream, dbg);
        if (rc) return rc;
    } else {
        DGS_HIP_CHECK(hipMemsetAsync(c->ranges, 0, 8ull * T, stream));
        c->vals = nullptr;
    }
    float4 *ckpt = nullptr, *cfin = nullptr;
    uint32_t *todo = nullptr;
    if (c->seg_ok) {
        const size_t nck = (size_t)TILE_PIX * ((size_t)std::max(cap, 0) / SEG + 4);
        if (int rc = c->ckb.ensure(16ull * (nck + (size_t)c->H * c->W))) return rc;
        ckpt = (float4 *)c->ckb.p;
        cfin = ckpt + nck;
        c->cfin = cfin;
        todo = (uint32_t *)c->segq.p + 4;
    }
    if (!ckpt && blend_fwd2()) {
        ScopedTimer tm("blend_fwd", stream);
        hipLaunchKernelGGL(k_blend_fwd2, dim3(T), dim3(B2), 0, stream, c->ranges, c->vals, (uint32_t)cap, c->W, c->H, c->gx,
                           c->xy, c->conic_o, c->rgbd, c->s.bg, c->final_T, c->n_contrib, out_color, out_depth);
    } else {
        ScopedTimer tm("blend_fwd", stream);
        hipLaunchKernelGGL(ckpt ? k_blend_fwd<true> : k_blend_fwd<false>, dim3(T), dim3(TILE_PIX), 0, stream, c->ranges, c->vals, (uint32_t)cap, c->W, c->H, c->gx, c->xy,
                           c->conic_o, c->rgbd, c->s.bg, c->final_T, c->n_contrib, out_color, out_depth, ckpt, todo,
                           todo ? todo - 2 : nullptr, cfin);
    }
    DGS_LAUNCH_CHECK("k_blend_fwd", dbg, stream);
    return DGS_OK;
}

// Deferred pair count (dgs_raster_set_deferred_count): the forward returns without waiting for
// num_rendered; the count is read when the backward starts (the GPU is long past the scan by then)
// or when the context is freed. An overflow of the speculative capacity is then too late to redo the
// forward, so it is counted (dgs_raster_deferred_overflows) and the caller redoes the whole training
// step synchronously (deformgs/train_step.py); the backward runs on ranges clipped to the capacity
// so it stays in bounds.
std::atomic<int> g_deferred{0};
// dL/dscales: the upstream CUDA op returns the gradient w.r.t. the modified scale (scale_modifier * s),
// i.e. without the scale_modifier factor; dgs_raster_set_exact_scale_grad(1) applies the chain rule
// (identical whenever scale_modifier = 1, as in every training call)
std::atomic<int> g_exact_scale_grad{0};
std::atomic<long long> g_deferred_overflows{0};

__global__ void k_clip_ranges(int T, uint2 *ranges, uint32_t cap) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < T) {
        uint2 r = ranges[t];
        ranges[t] = make_uint2(min(r.x, cap), min(r.y, cap));
    }
}

static int resolve_count(dgs_raster_ctx *c, hipStream_t stream) {
    if (!c->count_pending) return DGS_OK;
    c->count_pending = false;
    int nr = 0;
    if (int rc = wait_count(c, stream, nr)) return rc;
    pair_cap_observe(c->device, nr);
    if (nr > c->spec_cap) {
        g_deferred_overflows++;
        const int T = c->gx * c->gy;
        hipLaunchKernelGGL(k_clip_ranges, dim3(div_up(T, 256)), dim3(256), 0, stream, T, c->ranges, (uint32_t)c->spec_cap);
        DGS_LAUNCH_CHECK("k_clip_ranges", false, stream);
        c->num_rendered = c->spec_cap;
    } else {
        c->num_rendered = nr;
    }
    return DGS_OK;
}

static int raster_forward(const dgs_raster_settings *s, int P, int M, const float *means3D, const float *shs,
                          const float *shs_rest, const float *colors_precomp, const float *opacities,
                          const float *scales, const float *rotations, const float *cov3D_precomp, float *out_color,
                          float *out_depth, int *out_radii, dgs_raster_ctx **ctx_out, int *num_rendered,
                          void *stream_, uint8_t *out_visible = nullptr) {
    hipStream_t stream = (hipStream_t)stream_;
    if (shs_rest && (M * 3 != SH_ROW || !shs || ((reinterpret_cast<uintptr_t>(shs) | reinterpret_cast<uintptr_t>(shs_rest)) & 15))) {
        set_error("dgs_raster_forward_split_sh: needs M = 16 and 16-byte aligned features_dc / features_rest");
        return DGS_ERR_ARGS;
    }
    if (!s || !ctx_out || P < 0 || !out_color || !out_depth || (P > 0 && (!means3D || !opacities || !out_radii))) {
        set_error("dgs_raster_forward: null argument");
        return DGS_ERR_ARGS;
    }
    // (an empty point set has null data pointers everywhere: nothing to validate)
    if (P > 0 && (shs == nullptr) == (colors_precomp == nullptr)) {
        set_error("Please provide exactly one of either SHs or precomputed colors!");
        return DGS_ERR_ARGS;
    }
    if (P > 0 && cov3D_precomp == nullptr && (scales == nullptr || rotations == nullptr)) {
        set_error("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
        return DGS_ERR_ARGS;
    }
    if (P > 0 && shs && (M < 1 || M < (s->sh_degree + 1) * (s->sh_degree + 1) || s->sh_degree > 3)) {
        set_error("dgs_raster_forward: SH degree/coefficient count unsupported (degree <= 3, M >= (D+1)^2)");
        return DGS_ERR_ARGS;
    }
    if (s->image_height <= 0 || s->image_width <= 0) {
        set_error("dgs_raster_forward: empty image");
        return DGS_ERR_ARGS;
    }
    int device = 0;
    DGS_HIP_CHECK(hipGetDevice(&device));
    dgs_raster_ctx *c = ctx_acquire(device, stream);
    c->s = *s;
    c->P = P;
    c->M = M;
    c->H = s->image_height;
    c->W = s->image_width;
    c->gx = div_up(c->W, TILE_X);
    c->gy = div_up(c->H, TILE_Y);
    c->means3D = means3D; c->shs = shs; c->shs_rest = shs_rest; c->colors = colors_precomp; c->opac = opacities;
    c->scales = scales; c->rots = rotations; c->cov = cov3D_precomp;
    c->radii = out_radii;
    c->last_stream = stream;
    c->bwd_done = false;
    const int T = c->gx * c->gy;
    const int HW = c->H * c->W;
    const bool dbg = s->debug != 0;
    // geometry
    size_t off_xy = 0, off_co = align_up(off_xy + 8ull * P), off_cd = align_up(off_co + 16ull * P),
           off_t = align_up(off_cd + 16ull * P), off_o = align_up(off_t + 4ull * P), off_cl = align_up(off_o + 4ull * P);
    size_t off_dk = align_up(off_cl + P), off_dk2 = align_up(off_dk + 4ull * P), off_gid = align_up(off_dk2 + 4ull * P),
           off_ord = align_up(off_gid + 4ull * P), off_ts = align_up(off_ord + 4ull * P);
    size_t scan_tmp = 0, dsort_tmp = 0;
    if (P > 0) {
        DGS_HIP_CHECK(scan_tmp_bytes(device, P, stream, scan_tmp));
        DGS_HIP_CHECK(sort_tmp_bytes<uint32_t>(device, P, 32, stream, dsort_tmp));
    }
    size_t off_st = align_up(off_ts + 4ull * P);
    if (int rc = c->geom.ensure(off_st + std::max(scan_tmp, dsort_tmp) + 256)) { ctx_out[0] = nullptr; delete c; return rc; }
    char *g = (char *)c->geom.p;
    c->xy = (float2 *)(g + off_xy);
    c->conic_o = (float4 *)(g + off_co);
    c->rgbd = (float4 *)(g + off_cd);
    c->tiles = (uint32_t *)(g + off_t);
    c->offsets = (uint32_t *)(g + off_o);
    c->clamped = (uint8_t *)(g + off_cl);
    c->dkey = (uint32_t *)(g + off_dk);
    c->dkey_alt = (uint32_t *)(g + off_dk2);
    c->gid = (uint32_t *)(g + off_gid);
    c->order = (uint32_t *)(g + off_ord);
    c->tiles_sorted = (uint32_t *)(g + off_ts);
    // image state
    size_t off_r = 0, off_T = align_up(off_r + 8ull * T), off_n = align_up(off_T + 4ull * HW);
    if (int rc = c->img.ensure(off_n + 4ull * HW)) { delete c; return rc; }
    char *im = (char *)c->img.p;
    c->ranges = (uint2 *)(im + off_r);
    c->final_T = (float *)(im + off_T);
    c->n_contrib = (uint32_t *)(im + off_n);
    c->rect_mode = P > 0 && rect_binning(c->gx, c->gy, P);
    if (c->rect_mode) {  // count matrix [blocks][tiles], tile totals, tile starts, pair count
        const size_t nb = div_up(P, 256);
        size_t o_cnt = 0, o_st = align_up(4ull * nb * T), o_n = align_up(o_st + 4ull * T);
        if (int rc = c->rect.ensure(o_n + 256)) return rc;
        char *r = (char *)c->rect.p;
        c->rect_cnt = (uint32_t *)(r + o_cnt);
        c->rect_start = (uint32_t *)(r + o_st);
        c->rect_total = (uint32_t *)(r + o_n);
        const size_t tot_cap = c->rtot.cap;
        if (int rc = c->rtot.ensure(8ull * T)) return rc;
        if (c->rtot.cap != tot_cap) DGS_HIP_CHECK(hipMemsetAsync(c->rtot.p, 0, c->rtot.cap, stream));
        c->rect_tot = (unsigned long long *)c->rtot.p;
    }
    c->tsort = c->rect_mode && tile_sort_enabled();
    c->det_fwd = c->rect_mode && blend_deterministic();
    c->seg_ok = c->rect_mode && blend_segmented();
    if (c->seg_ok) {
        const size_t cap0 = c->segq.cap;
        if (int rc = c->segq.ensure(4ull * (T + 4))) return rc;
        if (c->segq.cap != cap0) DGS_HIP_CHECK(hipMemsetAsync(c->segq.p, 0, c->segq.cap, stream));
    }

    const float fx = c->W / (2.f * s->tanfovx), fy = c->H / (2.f * s->tanfovy);
    int nr = 0;
    // backward accumulators [P][12] (zeroed by k_preprocess)
    if (P > 0)
        if (int rc = c->acc.ensure(4ull * ACC_STRIDE * P)) return rc;
    if (P > 0) {
        {
            ScopedTimer tm("preprocess_fwd", stream);
            const bool stage = shs && M * 3 == SH_ROW && (reinterpret_cast<uintptr_t>(shs) & 15) == 0;
            hipLaunchKernelGGL(stage ? k_preprocess<true> : k_preprocess<false>, dim3(div_up(P, 256)), dim3(256), 0, stream,
                               P, s->sh_degree, M, means3D, scales,
                               s->scale_modifier, rotations, cov3D_precomp, opacities, shs, shs_rest, colors_precomp, s->viewmatrix,
                               s->projmatrix, s->campos, c->W, c->H, s->tanfovx, s->tanfovy, fx, fy, c->gx, c->gy, out_radii,
                               c->xy, c->conic_o, c->rgbd, c->tiles, c->clamped, c->dkey, c->gid, (float4 *)c->acc.p,
                               out_visible);
        }
        DGS_LAUNCH_CHECK("k_preprocess", dbg, stream);
        if (!c->tsort) {
            // Gaussians by depth (stable on the index), then the pair offsets in that order
            ScopedTimer tm("depth_sort", stream);
            if (hipcub_sort()) {
                hipcub::DoubleBuffer<uint32_t> kb(c->dkey, c->dkey_alt), vb(c->gid, c->order);
                DGS_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(g + off_st, dsort_tmp, kb, vb, P, 0, 32, stream));
                c->order = vb.Current();  // either buffer, per the pass count
                hipLaunchKernelGGL(k_gather_tiles, dim3(div_up(P, 256)), dim3(256), 0, stream, P, c->order, c->tiles,
                                   c->tiles_sorted);
            } else {
                // the last pass also gathers tiles[order[j]] (the scan input) into tiles_sorted
                int alt = 0;
                uint32_t *gid = c->gid, *ord = c->order;
                if (int rc = radix::sort_pairs<uint32_t>(c->dkey, c->dkey_alt, gid, ord, P, 32, stream, &alt,
                                                         c->rect_mode ? nullptr : c->tiles,
                                                         c->rect_mode ? nullptr : c->tiles_sorted))
                    return rc;
                c->order = alt ? ord : gid;
            }
        }
        DGS_LAUNCH_CHECK("depth_sort", dbg, stream);
        if (!c->h_total) {  // coherent + mapped: k_rect_colscan stores the count into it directly
            DGS_HIP_CHECK(hipHostMalloc((void **)&c->h_total, sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped));
            DGS_HIP_CHECK(hipHostGetDevicePointer((void **)&c->d_total, c->h_total, 0));
        }
        if (!c->count_ev) DGS_HIP_CHECK(hipEventCreateWithFlags(&c->count_ev, hipEventDisableTiming));
        if (c->rect_mode) {
            const int nb = div_up(P, 256);
            *(volatile uint32_t *)c->h_total = COUNT_PENDING;  // k_rect_colscan overwrites it
            {
                ScopedTimer tm("count", stream);
                hipLaunchKernelGGL(k_rect_count, dim3(nb), dim3(256), 4ull * T, stream, P, c->tsort ? nullptr : c->order,
                                   c->xy, c->radii, c->gx,
                                   c->gy, c->rect_cnt, c->rect_total, c->seg_ok ? (uint32_t *)c->segq.p + 2 : nullptr);
            }
            DGS_LAUNCH_CHECK("k_rect_count", dbg, stream);
            {
                ScopedTimer tm("scan", stream);
                hipLaunchKernelGGL(k_rect_colscan, dim3(div_up(T, 64)), dim3(1024), 0, stream, nb, T, c->rect_cnt, c->rect_tot,
                                   next_rect_gen(), c->rect_total, c->rect_total + 1, c->rect_start, c->ranges,
                                   c->d_total);
            }
            DGS_LAUNCH_CHECK("k_rect_colscan", dbg, stream);
        } else {
            DGS_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(g + off_st, scan_tmp, c->tiles_sorted, c->offsets, P, stream));
            DGS_HIP_CHECK(hipMemcpyAsync(c->h_total, c->offsets + (P - 1), 4, hipMemcpyDeviceToHost, stream));
        }
        if (!c->rect_mode) DGS_HIP_CHECK(hipEventRecord(c->count_ev, stream));
        int cap = pair_cap_get(device);
        const bool speculative = cap > 0 && !dbg;
        if (!speculative) {
            if (int rc = wait_count(c, stream, nr)) return rc;
            cap = nr;
        }
        if (int rc = bin_and_blend(c, cap, P, device, stream, dbg, out_color, out_depth)) return rc;
        if (speculative && g_deferred.load()) {  // num_rendered read by the backward (resolve_count)
            c->count_pending = true;
            c->spec_cap = cap;
            c->num_rendered = cap;
            *ctx_out = c;
            if (num_rendered) *num_rendered = -1;
            return DGS_OK;
        }
        if (speculative) {
            if (int rc = wait_count(c, stream, nr)) return rc;
            if (nr > cap) {  // overflow: redo binning + blend at the exact size
                {
                    std::lock_guard<std::mutex> lk(g_cap_mu);
                    g_redos++;
                }
                if (int rc = bin_and_blend(c, nr, P, device, stream, dbg, out_color, out_depth)) return rc;
            }
        }
        pair_cap_observe(device, nr);
    } else {
        if (int rc = bin_and_blend(c, 0, P, device, stream, dbg, out_color, out_depth)) return rc;
    }
    c->num_rendered = nr;
    *ctx_out = c;
    if (num_rendered) *num_rendered = nr;
    return DGS_OK;
}

static int raster_backward(dgs_raster_ctx *c, const float *dL_dcolor, const float *dL_ddepth, float *dL_dmeans3D,
                           float *dL_dmeans2D, float *dL_dmeans2D_densify, float *dL_dcolors, float *dL_dopacity,
                           float *dL_dcov3D, float *dL_dshs, float *dL_dshs_rest, float *dL_dscales,
                           float *dL_drotations, void *stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    if (c && (c->shs_rest != nullptr) != (dL_dshs_rest != nullptr)) {
        set_error("dgs_raster_backward: split SH gradients go with a split SH forward");
        return DGS_ERR_ARGS;
    }
    if (c && dL_dshs_rest && ((reinterpret_cast<uintptr_t>(dL_dshs) | reinterpret_cast<uintptr_t>(dL_dshs_rest)) & 15)) {
        set_error("dgs_raster_backward_split_sh: SH gradients must be 16-byte aligned");
        return DGS_ERR_ARGS;
    }
    if (!c || !dL_dcolor) {
        set_error("dgs_raster_backward: null argument");
        return DGS_ERR_ARGS;
    }
    if (c->P == 0) return DGS_OK;
    if (!dL_dmeans3D || !dL_dmeans2D || !dL_dmeans2D_densify || !dL_dopacity) {
        set_error("dgs_raster_backward: null argument");
        return DGS_ERR_ARGS;
    }
    if ((c->shs && !dL_dshs) || (c->colors && !dL_dcolors) || (c->cov && !dL_dcov3D) ||
        (!c->cov && (!dL_dscales || !dL_drotations))) {
        set_error("dgs_raster_backward: missing gradient buffer for the forward's input combination");
        return DGS_ERR_ARGS;
    }
    const int P = c->P;
    c->last_stream = stream;
    if (P == 0) return DGS_OK;
    // A deferred pair count stays unresolved here (the host does not wait mid-step): the blend
    // backward clips the tile ranges to the speculative capacity the binning ran with, which is exact
    // unless it overflowed; dgs_raster_ctx_free resolves the count and counts an overflow (the
    // caller then redoes the step).
    const uint32_t cap = c->count_pending ? (uint32_t)c->spec_cap : (uint32_t)c->num_rendered;
    const bool dbg = c->s.debug != 0;
    const int T = c->gx * c->gy;
    float *acc = (float *)c->acc.p;  // [P][12], zeroed by the forward's k_preprocess
    // deterministic mode: k_rect_gather writes every row of acc (no zeroing needed)
    // deterministic: asked for at this forward too (the tile sort then left the position map)
    const bool det = blend_deterministic() && c->rect_mode && c->det_fwd && !blend_one_pixel();
    // a second backward through the same forward (retain_graph, or a context kept alive): the blend
    // backward adds into the accumulators, so they are cleared first instead of doubling the gradients
    if (c->bwd_done && !det) DGS_HIP_CHECK(hipMemsetAsync(acc, 0, 4ull * ACC_STRIDE * P, stream));
    c->bwd_done = true;
    if (cap > 0 && det) {
        uint32_t *todo = nullptr, *pre = nullptr;
        float *slot = nullptr;
        // with the tile sort, the forward laid the buffer out (its position map is in it)
        if (int rc = det_layout(c, c->tsort ? c->det_cap : (int)cap, &todo, &slot, &pre)) return rc;
        if (!c->tsort) pre = nullptr;  // lists placed in depth order: the slot index is the list position
        {
            ScopedTimer tm("blend_bwd", stream);
            hipLaunchKernelGGL((dL_ddepth ? k_blend_bwd2<true, true> : k_blend_bwd2<false, true>), dim3(T), dim3(B2), 0,
                               stream, c->ranges, c->vals, cap, c->W, c->H, c->gx, c->s.bg, c->xy, c->conic_o, c->rgbd,
                               c->final_T, c->n_contrib, dL_dcolor, dL_ddepth, acc, slot, todo, pre);
        }
        DGS_LAUNCH_CHECK("k_blend_bwd2<det>", dbg, stream);
        ScopedTimer tm("blend_gather", stream);
        const bool stage = rect_place_stage(c->gx, c->gy);
        hipLaunchKernelGGL(k_rect_gather, dim3(div_up(P, 256)), dim3(256), rect_place_lds(c->gx, c->gy, stage), stream, P,
                           c->tsort ? nullptr : c->order, c->xy, c->radii, c->gx, c->gy, c->rect_cnt, c->rect_start,
                           cap, (const float4 *)slot, acc, (int)stage);
    } else if (cap > 0) {
        ScopedTimer tm("blend_bwd", stream);
        if (blend_one_pixel())
            hipLaunchKernelGGL(k_blend_bwd, dim3(T), dim3(TILE_PIX), 0, stream, c->ranges, c->vals, cap, c->W, c->H, c->gx,
                               c->s.bg, c->xy, c->conic_o, c->rgbd, c->final_T, c->n_contrib, dL_dcolor, dL_ddepth, acc);
        else if (c->seg_ok && !dL_ddepth) {
            static int cus = 0;
            if (!cus) DGS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
            uint32_t *q = (uint32_t *)c->segq.p;
            hipLaunchKernelGGL(k_blend_bwd2s, dim3(cus * BWD_SEG_WGS_PER_CU), dim3(B2), 0, stream, c->ranges, c->vals, cap,
                               c->W, c->H, c->gx, T, c->s.bg, c->xy, c->conic_o, c->rgbd, c->final_T, c->n_contrib,
                               c->cfin, (const float4 *)c->ckb.p, q + 4, q + 2, q, dL_dcolor, acc);
        } else
            if (dL_ddepth)
                hipLaunchKernelGGL((k_blend_bwd2<true, false>), dim3(T), dim3(B2), 0, stream, c->ranges, c->vals, cap, c->W,
                                   c->H, c->gx, c->s.bg, c->xy, c->conic_o, c->rgbd, c->final_T, c->n_contrib, dL_dcolor,
                                   dL_ddepth, acc, nullptr, nullptr, nullptr);
            else
                hipLaunchKernelGGL((k_blend_bwd2<false, false>), dim3(T), dim3(B2), 0, stream, c->ranges, c->vals, cap, c->W,
                                   c->H, c->gx, c->s.bg, c->xy, c->conic_o, c->rgbd, c->final_T, c->n_contrib, dL_dcolor,
                                   nullptr, acc, nullptr, nullptr, nullptr);
    }
    DGS_LAUNCH_CHECK("k_blend_bwd", dbg, stream);
    const float fx = c->W / (2.f * c->s.tanfovx), fy = c->H / (2.f * c->s.tanfovy);
    {
        ScopedTimer tm("preprocess_bwd", stream);
        const bool stage = c->shs_rest || (c->shs && c->M * 3 == SH_ROW &&
                           ((reinterpret_cast<uintptr_t>(c->shs) | reinterpret_cast<uintptr_t>(dL_dshs)) & 15) == 0);
        hipLaunchKernelGGL(stage ? k_preprocess_bwd<true> : k_preprocess_bwd<false>, dim3(div_up(P, 256)), dim3(256), 0,
                           stream, P, c->s.sh_degree, c->M, c->means3D,
                           c->scales, c->s.scale_modifier, c->rots, c->cov, c->shs, c->s.viewmatrix, c->s.projmatrix,
                           c->s.campos, c->W, c->H, c->s.tanfovx, c->s.tanfovy, fx, fy, c->radii, c->clamped, acc,
                           dL_dmeans3D, dL_dmeans2D, dL_dmeans2D_densify, dL_dcolors, dL_dopacity, dL_dcov3D, dL_dshs,
                           dL_dscales, dL_drotations, c->shs_rest, dL_dshs_rest,
                           g_exact_scale_grad.load() ? c->s.scale_modifier : 1.f);
    }
    DGS_LAUNCH_CHECK("k_preprocess_bwd", dbg, stream);
    return DGS_OK;
}

extern "C" int dgs_raster_forward(const dgs_raster_settings *s, int P, int M, const float *means3D,
                                  const float *shs, const float *colors_precomp, const float *opacities,
                                  const float *scales, const float *rotations, const float *cov3D_precomp,
                                  float *out_color, float *out_depth, int *out_radii, dgs_raster_ctx **ctx_out,
                                  int *num_rendered, void *stream) {
    return raster_forward(s, P, M, means3D, shs, nullptr, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                          out_color, out_depth, out_radii, ctx_out, num_rendered, stream);
}

extern "C" int dgs_raster_forward_split_sh(const dgs_raster_settings *s, int P, const float *means3D,
                                           const float *features_dc, const float *features_rest,
                                           const float *opacities, const float *scales, const float *rotations,
                                           float *out_color, float *out_depth, int *out_radii,
                                           uint8_t *out_visible, dgs_raster_ctx **ctx_out, int *num_rendered,
                                           void *stream) {
    if (P > 0 && (!features_dc || !features_rest)) {
        set_error("dgs_raster_forward_split_sh: null SH argument");
        return DGS_ERR_ARGS;
    }
    return raster_forward(s, P, SH_ROW / 3, means3D, features_dc, P > 0 ? features_rest : nullptr, nullptr, opacities,
                          scales, rotations, nullptr, out_color, out_depth, out_radii, ctx_out, num_rendered, stream,
                          out_visible);
}

extern "C" int dgs_raster_backward(dgs_raster_ctx *c, const float *dL_dcolor, const float *dL_ddepth,
                                   float *dL_dmeans3D, float *dL_dmeans2D, float *dL_dmeans2D_densify,
                                   float *dL_dcolors, float *dL_dopacity, float *dL_dcov3D, float *dL_dshs,
                                   float *dL_dscales, float *dL_drotations, void *stream) {
    return raster_backward(c, dL_dcolor, dL_ddepth, dL_dmeans3D, dL_dmeans2D, dL_dmeans2D_densify, dL_dcolors,
                           dL_dopacity, dL_dcov3D, dL_dshs, nullptr, dL_dscales, dL_drotations, stream);
}

extern "C" int dgs_raster_backward_split_sh(dgs_raster_ctx *c, const float *dL_dcolor, const float *dL_ddepth,
                                            float *dL_dmeans3D, float *dL_dmeans2D, float *dL_dmeans2D_densify,
                                            float *dL_dopacity, float *dL_dfeatures_dc, float *dL_dfeatures_rest,
                                            float *dL_dscales, float *dL_drotations, void *stream) {
    if (c && c->P > 0 && (!dL_dfeatures_dc || !dL_dfeatures_rest)) {
        set_error("dgs_raster_backward_split_sh: null SH gradient");
        return DGS_ERR_ARGS;
    }
    return raster_backward(c, dL_dcolor, dL_ddepth, dL_dmeans3D, dL_dmeans2D, dL_dmeans2D_densify, nullptr,
                           dL_dopacity, nullptr, dL_dfeatures_dc, c && c->P > 0 ? dL_dfeatures_rest : nullptr,
                           dL_dscales, dL_drotations, stream);
}

extern "C" int dgs_raster_ctx_num_rendered(dgs_raster_ctx *c) {
    if (!c) return -1;
    if (resolve_count(c, c->last_stream)) return -1;
    return c->num_rendered;
}

extern "C" void dgs_raster_ctx_free(dgs_raster_ctx *c) {
    if (!c) return;
    (void)resolve_count(c, c->last_stream);  // a deferred count nobody read (forward without backward)
    // Buffers stay allocated for reuse by the next forward on this device; an acquirer on another
    // stream is ordered after the stream that last used them (ctx_acquire).
    c->pending_release = true;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (g_pool.size() < 64) {
        g_pool.push_back(c);
    } else {
        c->geom.release(); c->bin.release(); c->img.release(); c->acc.release(); c->tmp.release(); c->rect.release();
        c->rtot.release(); c->ckb.release(); c->segq.release(); c->det.release();
        if (c->h_total) (void)hipHostFree(c->h_total);
        delete c;
    }
}

extern "C" void dgs_raster_set_deferred_count(int on) { g_deferred.store(on ? 1 : 0); }

extern "C" void dgs_raster_set_exact_scale_grad(int on) { g_exact_scale_grad.store(on ? 1 : 0); }

extern "C" long long dgs_raster_deferred_overflows(void) { return g_deferred_overflows.load(); }

extern "C" void dgs_debug_set_pair_cap(int device, int cap) {
    std::lock_guard<std::mutex> lk(g_cap_mu);
    g_pair_cap[device] = cap < 0 ? 0 : cap;
}

extern "C" int dgs_debug_pair_cap(int device) { return pair_cap_get(device); }

extern "C" void dgs_debug_set_blend_seg(int on) { g_blend_seg.store(on ? 1 : 0); }
extern "C" void dgs_raster_set_deterministic(int on) { g_det.store(on ? 1 : 0); }
extern "C" void dgs_debug_set_tile_sort(int on) { g_tile_sort.store(on ? 1 : 0); }
extern "C" void dgs_debug_set_blend_fwd2(int on) { g_fwd2.store(on ? 1 : 0); }
extern "C" int dgs_debug_get_blend_fwd2(void) { return blend_fwd2() ? 1 : 0; }
extern "C" int dgs_debug_get_tile_sort(void) { return tile_sort_enabled() ? 1 : 0; }
extern "C" int dgs_raster_get_deterministic(void) { return blend_deterministic() ? 1 : 0; }
extern "C" int dgs_debug_get_blend_seg(void) { return blend_segmented() ? 1 : 0; }

extern "C" void dgs_debug_set_binning(int mode) { g_binning.store(mode == 1 ? 1 : 0); }

extern "C" long long dgs_debug_count_wait_ns(long long *waits) {
    if (waits) *waits = g_count_waits.load();
    return g_count_wait_ns.load();
}

extern "C" long long dgs_debug_binning_redos(void) {
    std::lock_guard<std::mutex> lk(g_cap_mu);
    return g_redos;
}

extern "C" int dgs_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                                uint8_t *visible, void *stream_) {
    (void)projmatrix;
    if (P <= 0) return DGS_OK;
    hipStream_t stream = (hipStream_t)stream_;
    hipLaunchKernelGGL(k_mark_visible, dim3(div_up(P, 256)), dim3(256), 0, stream, P, means3D, viewmatrix, visible);
    DGS_LAUNCH_CHECK("k_mark_visible", false, stream);
    return DGS_OK;
}
