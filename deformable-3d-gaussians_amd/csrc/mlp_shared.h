// Pieces shared by the two deformation-MLP paths: mlp.hip (fp32 MFMA, DGS_MLP_EXACT_FP32) and
// mlp_split.hip (the default: bf16 MFMA on an exact three-way operand split).
//
// Network shape (utils/time_utils.py:56-127, DeformNetwork :129-201): D=8, W=256, multires=10,
// skips=[4]; blender adds timenet Linear(13,256)+ReLU+Linear(256,30); heads d_xyz(3) | 6-DoF
// branch_w(3), branch_v(3), rotation(4), scaling(3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dgs_common.h"

namespace dgs {
namespace mlpc {

// padded feature offsets of the concatenated layer input (XE|TE|H)
constexpr int F_XE = 0, F_TE = 64, F_H = 96;

// saved-activation row offsets ([rows][Ns], feature-major); order keeps each layer input contiguous
constexpr int S_H0 = 0, S_XE = 1024, S_TE = 1088, S_H4 = 1120, S_TIN = 2144, S_TH = 2160;
__host__ __device__ constexpr int s_h(int i) { return i < 4 ? S_H0 + 256 * i : S_H4 + 256 * (i - 4); }
// timenet of a frame-uniform t (blender), evaluated once per launch by k_timenet into the tail of
// the saved buffer: [t0 | TIN (16) | TE (32) | TH (256) | C0 (256) | C5 (256)], C0 / C5 = the biases of
// linear.0 / linear.5 with the t_emb columns folded in (split path, uniform t)
constexpr int TC_T = 0, TC_TIN = 16, TC_TE = 32, TC_TH = 64, TC_C0 = 320, TC_C5 = 576, TC_FLOATS = 1024;
// relu' bit-mask rows: H0..H7 then TH (blender)
__host__ __device__ constexpr int m_h(int i) { return 256 * i; }
constexpr int M_TH = 2048;
// dZ scratch rows
constexpr int Z_L0 = 0, Z_G = 2048, Z_TE = 2080, Z_T1 = 2112;

struct Flags {
    bool blender, sixdof, norotscale;
    bool uniform_t;  // DGS_MLP_UNIFORM_T on a blender network: no per-point timenet backward
    int nout;     // head outputs: 10 or 13
    int tin;      // raw t PE channels: 13 (L=6) or 21 (L=10)
    int nsaved;   // saved rows
    int nmask;    // relu' bit-mask words per 32-point tile (16 bits per lane of a 32-row tile)
    int nz;       // dZ rows
};

__host__ __device__ inline Flags make_flags(int f) {
    Flags F;
    F.blender = f & DGS_MLP_BLENDER;
    F.sixdof = f & DGS_MLP_6DOF;
    F.norotscale = f & DGS_MLP_NO_ROTSCALE;
    F.uniform_t = F.blender && (f & DGS_MLP_UNIFORM_T);
    F.nout = F.sixdof ? 13 : 10;
    F.tin = F.blender ? 13 : 21;
    F.nsaved = F.blender ? 2416 : 2144;
    F.nmask = F.blender ? 2304 : 2048;
    F.nz = F.blender ? 2368 : 2080;
    return F;
}

struct Seg {  // padded index range [p0, p0+len) <- source index s0 + (p - p0)
    int p0, len, s0;
};
inline Seg seg(int p0, int len, int s0) { return Seg{p0, len, s0}; }

// source index of padded index p under segments (or -1 = zero padding)
__host__ __device__ inline int seg_lookup(const Seg *s, int ns, int p) {
    for (int q = 0; q < ns; q++)
        if (p >= s[q].p0 && p < s[q].p0 + s[q].len) return s[q].s0 + (p - s[q].p0);
    return -1;
}

// input-feature segments of the concatenated trunk inputs. With a frame-uniform t (F.uniform_t, the
// split path only) linear.0 / linear.5 see t_emb as a constant: its columns are folded into the bias
// (k_timenet: C0 = b0 + W0,te te, C5 likewise), so the forward GEMMs and dW cover x_emb (and h) only,
// and the t_emb columns' dW is gb (x) te (k_tgrad). fold = false: the full layout (the backward's
// transposed images, whose x_emb / t_emb rows are never read with a uniform t).
inline int layer_in_segs(const Flags &F, int layer, Seg *s, bool fold = true) {
    const int te = F.blender ? 30 : F.tin;
    if (fold && F.uniform_t && (layer == 0 || layer == 5)) {
        s[0] = seg(F_XE, 63, 0);
        if (layer == 0) return 1;
        s[1] = seg(64, 256, 63 + te);  // h right after x_emb
        return 2;
    }
    if (layer == 0) {
        s[0] = seg(F_XE, 63, 0);
        s[1] = seg(F_TE, te, 63);
        return 2;
    }
    if (layer == 5) {
        s[0] = seg(F_XE, 63, 0);
        s[1] = seg(F_TE, te, 63);
        s[2] = seg(F_H, 256, 63 + te);
        return 3;
    }
    s[0] = seg(0, 256, 0);
    return 1;
}

__host__ __device__ inline int layer_kpad(int layer) { return layer == 0 ? 96 : layer == 5 ? 352 : 256; }
// padded K of the forward GEMM / dW (t_emb folded with a uniform t)
__host__ __device__ inline int layer_kpad_f(const Flags &F, int layer) {
    return F.uniform_t && layer == 0 ? 64 : F.uniform_t && layer == 5 ? 320 : layer_kpad(layer);
}

// parameter indices in state_dict order (include/dgs.h)
struct Params {
    int pT0w = -1, pT0b = -1, pT2w = -1, pT2b = -1, pLw[8], pLb[8];
    int nheads;               // number of head linears (3 or 4)
    int pHw[4], pHb[4], hrows[4];
    int nparams;
};

inline Params make_params(const Flags &F) {
    Params P;
    int k = 0;
    if (F.blender) {
        P.pT0w = k++; P.pT0b = k++; P.pT2w = k++; P.pT2b = k++;
    }
    for (int i = 0; i < 8; i++) {
        P.pLw[i] = k++;
        P.pLb[i] = k++;
    }
    P.nheads = F.sixdof ? 4 : 3;
    const int hr6[4] = {3, 3, 4, 3}, hr3[3] = {3, 4, 3};
    for (int h = 0; h < P.nheads; h++) {
        P.pHw[h] = k++;
        P.pHb[h] = k++;
        P.hrows[h] = F.sixdof ? hr6[h] : hr3[h];
    }
    P.nparams = k;
    return P;
}

// (rows, cols) of parameter idx; cols = 0 for a bias
inline int param_shape(const Flags &F, const Params &P, int idx, int &rows, int &cols) {
    rows = cols = 0;
    if (F.blender) {
        if (idx == P.pT0w) { rows = 256; cols = F.tin; return 0; }
        if (idx == P.pT0b) { rows = 256; return 0; }
        if (idx == P.pT2w) { rows = 30; cols = 256; return 0; }
        if (idx == P.pT2b) { rows = 30; return 0; }
    }
    const int te = F.blender ? 30 : F.tin;
    for (int i = 0; i < 8; i++) {
        if (idx == P.pLw[i]) { rows = 256; cols = i == 0 ? 63 + te : i == 5 ? 256 + 63 + te : 256; return 0; }
        if (idx == P.pLb[i]) { rows = 256; return 0; }
    }
    for (int h = 0; h < P.nheads; h++) {
        if (idx == P.pHw[h]) { rows = P.hrows[h]; cols = 256; return 0; }
        if (idx == P.pHb[h]) { rows = P.hrows[h]; return 0; }
    }
    return -1;
}

// ------------------------------------------------------------------------------------------------
// dW = dZ X^T over all points: one <=256x256 tile per layer (L5: 256 + 96 input columns), split over
// the point axis (~one workgroup per CU finishing together), then a fixed-order slab reduction.
// ------------------------------------------------------------------------------------------------
constexpr int WT = 256;             // tile edge (rows of dZ, rows of X)
constexpr int SLAB = WT * WT + WT;  // tile + bias row sums
constexpr int MAXJ = 12;

struct WJob {
    int zrow, nrows;   // dZ rows [zrow, zrow + nrows) (padded layer outputs, <= 256)
    int xrow, krows;   // X rows [xrow, xrow + krows) in saved (<= 256)
    int nsplit;        // workgroups over the point axis
    int block0;        // first workgroup (= first slab) of this job
    int narrow;        // wave layout: 0 = 2 (rows) x 4 (cols) waves of 128 x 64; 1 = 8 x 1 waves of
                       // 32 x 128 (jobs with krows <= 128: every wave has work)
};
struct WJobs {
    WJob j[MAXJ];
    int n;
};

// dW job list for the flags (host): layers L0..L7 (L5 as two k-tiles), heads, T1, T2
struct WPlan {
    WJobs jobs;
    int layer_job[11][2];  // job index of k-tile 0/1 per layer (-1 if none)
    int layer_k1[11];      // padded feature where k-tile 1 starts (256; 64 for a folded linear.5)
    int nblocks;
};

// Splits: per-chunk cost = the busiest SIMD's MFMA tiles (waves w and w + 4 share SIMD w % 4) plus a
// per-chunk staging/barrier cost (`fixed`), floored at `floor_`; the smallest per-workgroup time whose
// ceil(cost * nch / T) fit `target` workgroups (whole jobs never straddle).
// shape_cost (optional, the split k_dws): measured per-chunk cost of the four job shapes instead of
// the MFMA-tile model, indexed by dw_shape().
inline int dw_shape(int nrows, int krows) {
    return krows == 256 ? (nrows == 256 ? 0 : 1) : (krows > 64 ? 2 : krows > 32 ? 4 : 3);
}
inline WPlan make_wplan(const Flags &F, int target, double fixed, double floor_, const double *shape_cost = nullptr) {
    WPlan W{};
    struct Raw {
        int zrow, nrows, xrow, krows, layer, kt;
    };
    Raw raw[MAXJ];
    int nr = 0;
    for (int l = 0; l < 11; l++) W.layer_k1[l] = WT;
    for (int i = 0; i < 8; i++) {
        if (F.uniform_t && (i == 0 || i == 5)) {  // folded t_emb: x_emb rows (+ h rows for linear.5)
            raw[nr++] = Raw{Z_L0 + 256 * i, 256, S_XE, 64, i, 0};
            if (i == 5) {
                raw[nr++] = Raw{Z_L0 + 256 * i, 256, S_H4, 256, i, 1};
                W.layer_k1[i] = 64;
            }
            continue;
        }
        int xrow = (i == 0 || i == 5) ? S_XE : s_h(i - 1);
        int kp = layer_kpad(i);
        for (int kt = 0; kt * WT < kp; kt++)
            raw[nr++] = Raw{Z_L0 + 256 * i, 256, xrow + kt * WT, kp - kt * WT < WT ? kp - kt * WT : WT, i, kt};
    }
    raw[nr++] = Raw{Z_G, 32, s_h(7), 256, 8, 0};
    if (F.blender && !F.uniform_t) {  // uniform t: timenet gradients from the bias gradients instead
        raw[nr++] = Raw{Z_T1, 256, S_TIN, 16, 9, 0};
        raw[nr++] = Raw{Z_TE, 32, S_TH, 256, 10, 0};
    }
    for (int l = 0; l < 11; l++) W.layer_job[l][0] = W.layer_job[l][1] = -1;
    double cost[MAXJ], total = 0;
    for (int q = 0; q < nr; q++) {
        const bool nar = raw[q].krows <= 128;
        int simd[4] = {0, 0, 0, 0};
        for (int w = 0; w < 8; w++) {
            int tr, tc;
            if (nar) {
                tr = 32 * w < raw[q].nrows ? 1 : 0;
                tc = div_up(raw[q].krows, 32);
                tc = tc < 4 ? tc : 4;
            } else {
                tr = div_up(raw[q].nrows - 128 * (w >> 2), 32);
                tr = tr < 0 ? 0 : tr > 4 ? 4 : tr;
                tc = div_up(raw[q].krows - 64 * (w & 3), 32);
                tc = tc < 0 ? 0 : tc > 2 ? 2 : tc;
            }
            simd[w & 3] += tr * tc;
        }
        int crit = simd[0];
        for (int s = 1; s < 4; s++) crit = simd[s] > crit ? simd[s] : crit;
        cost[q] = crit + fixed > floor_ ? crit + fixed : floor_;
        if (shape_cost) cost[q] = shape_cost[dw_shape(raw[q].nrows, raw[q].krows)];
        total += cost[q];
    }
    const int nch = 1 << 20;  // relative scale only (the chunk count cancels)
    double T = total * nch / target;
    int nsq[MAXJ];
    for (int it = 0; it < 400; it++, T *= 1.005) {
        int sum = 0;
        for (int q = 0; q < nr; q++) {
            nsq[q] = (int)ceil(cost[q] * nch / T - 1e-9);
            nsq[q] = nsq[q] < 1 ? 1 : nsq[q];
            sum += nsq[q];
        }
        if (sum <= target) break;
    }
    int b = 0;
    for (int q = 0; q < nr; q++) {
        const int ns = nsq[q];
        W.jobs.j[q] = WJob{raw[q].zrow, raw[q].nrows, raw[q].xrow, raw[q].krows, ns, b, raw[q].krows <= 128 ? 1 : 0};
        W.layer_job[raw[q].layer][raw[q].kt] = q;
        b += ns;
    }
    W.jobs.n = nr;
    W.nblocks = b;
    return W;
}

// Sums every parameter gradient out of the dW slabs in a fixed order (mlp.hip: k_dw_reduce), one
// launch for all parameters. grads: device pointers in state_dict order.
int launch_dw_reduce(const Flags &F, const WPlan &W, const float *slabs, float *const *grads, hipStream_t stream);

// relu' of a 32x32 accumulator tile (the MFMA C/D layout: lane (m = l & 31, h = l >> 5) holds rows
// 8(r >> 2) + 4h + (r & 3) of column m) as 16 bits per lane: bit r = [value > 0] (signed clamp of
// the float bits: -0.0 and +0.0 give 0). The backward GEMM over the same 32-row tile has the identical
// lane layout, so no transpose is needed either way.
template <class V>
__device__ inline void store_mask_bits(const V &c, __amdgpu_buffer_rsrc_t mrsrc, int soff_bytes, int lane) {
    uint32_t w = 0;
#pragma unroll
    for (int r = 0; r < 16; r++) w |= (uint32_t)min(max(__float_as_int(c[r]), 0), 1) << r;
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)w, mrsrc, lane * 2, soff_bytes, 0);
}

template <class V>
__device__ inline void mask_apply(V &acc, uint32_t bits) {
#pragma unroll
    for (int r = 0; r < 16; r++)  // bit r sign-extended to 0 / all-ones
        acc[r] = __int_as_float(__float_as_int(acc[r]) & __builtin_amdgcn_sbfe((int)bits, r, 1));
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS traffic (lgkmcnt 0) but not
// for its global stores (__syncthreads() also waits vmcnt(0), a release fence). No wave of the MLP
// kernels reads global memory another wave of the block wrote.
__device__ inline void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // gfx9 encoding: vmcnt 63, expcnt 7, lgkmcnt 0
    __builtin_amdgcn_s_barrier();
}

// A wave's 32-row tile of a feature-major [rows][Ns] array, addressed through a buffer descriptor
// whose base is the tile origin (wave-uniform: SGPRs): each access is one buffer instruction with
// the lane offset in a VGPR and the row offset in an SGPR, no per-access address arithmetic.
struct TileAddr {
    __amdgpu_buffer_rsrc_t rsrc;  // base = &dst[(row0 + n0) * Ns + p0]
    int voff;                     // (4h * Ns + m) * 4 bytes
    int ns4;                      // Ns * 4 bytes
    __device__ static constexpr int row(int r) { return 8 * (r >> 2) + (r & 3); }
    // column tile ct (32 points) at +128 B
    __device__ void st(int r, float v, int ct = 0) const {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc, voff + 128 * ct, row(r) * ns4, 0);
    }
};

__device__ inline TileAddr tile_addr(const float *dst, size_t Ns, int row0, int n0, int p0, int lane) {
    const float *base = dst + (size_t)(row0 + n0) * Ns + p0;
    // a 32-row tile spans 32 * Ns floats; the descriptor's record count only bounds-checks
    return TileAddr{__builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), 0, 0x7fffffff, 0x00020000),
                    (4 * (lane >> 5) * (int)Ns + (lane & 31)) * 4, (int)Ns * 4};
}

}  // namespace mlpc

// fp32-MFMA path (mlp.hip), selected by DGS_MLP_EXACT_FP32
namespace mlp {
size_t packed_floats(int flags);
size_t saved_floats(int flags, int N);
size_t scratch_floats(int flags, int N);
int pack(int flags, const float *const *params, float *packed, hipStream_t stream);
int forward(int flags, int N, const float *xyz, const float *t, const float *packed, float *out, float *saved,
            hipStream_t stream);
int backward(int flags, int N, const float *packed, const float *saved, const float *dout, float *scratch,
             float *const *grads, hipStream_t stream);
// dW (fp32-input MFMA) + reduction over [rows][Ns] dZ / saved arrays; slabs: dw_fp32_slab_floats
size_t dw_fp32_slab_floats(int flags);
int dw_fp32(const mlpc::Flags &F, size_t Ns, const float *dz, const float *saved, float *slabs, float *const *grads,
            hipStream_t stream);
}  // namespace mlp
}  // namespace dgs
