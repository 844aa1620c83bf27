// Fused deformation MLP (positional encoding + timenet + 8x256 trunk with skip + heads) on fp32
// MFMA (v_mfma_f32_32x32x2_f32: exact fp32 fma chains) for MI355X / gfx950.
//
// Replaces DeformNetworkBaseline.forward and its autograd backward (utils/time_utils.py:56-127;
// DeformNetwork :129-201 via DGS_MLP_NO_ROTSCALE; 6-DoF heads :114-121 emitted raw, exp_se3 stays
// in the host glue). Default and only supported shape: D=8, W=256, multires=10, skips=[4]
// (arguments/__init__.py:65-68 and every arguments/*.py config).
//
// Layout ("transposed" formulation, Y^T = W X^T): features on MFMA rows, points on MFMA columns.
// One workgroup = 64 points (two 32-point m-tiles) x 8 waves; wave w owns output n-tile w of a
// 256-wide layer for both m-tiles, so every weight fragment is read once per workgroup.
//  * Activations live in LDS as [feature/4][64 points][4] (16-byte groups): the B operand of a
//    k-step is one ds_read_b128 per lane, and the 32x32 accumulator rows (8j + 4h + 0..3) of a
//    layer are exactly one ds_write_b128 into the next layer's input image (no shuffles).
//    LDS regions (groups of 4 features): XE 0-15 | TE 16-23 | H 24-87 | TIN 88-91 | PART 92-123;
//    XE|TE|H contiguous makes cat(x_emb, t_emb) and cat(x_emb, t_emb, h) plain ranges.
//  * Weights are re-packed every call (they change every optimizer step) into MFMA A-fragment
//    order [n-tile][8-feature chunk][64 lanes][4] so each wave-load is 1 KiB contiguous.
//  * Narrow layers (timenet.2, heads, and the t_emb slices of the backward) split K over the 8
//    waves and sum their partials in a fixed order (deterministic, no LDS atomics).
//  * Forward saves every layer's input activations feature-major [F][Ns] (coalesced from the
//    accumulator layout); backward dX saves every dZ the same way; dW = dZ X^T is a separate
//    split-N MFMA GEMM + fixed-order slab reduction (deterministic).
#include <hip/hip_runtime.h>

#include <cmath>
#include <map>
#include <mutex>
#include <vector>

#include "dgs_common.h"
#include "mlp_shared.h"

namespace dgs {
namespace mlp {

using namespace mlpc;

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 32;          // points per workgroup
constexpr int NWAVE = 8;
constexpr int NTHR = NWAVE * 64;
// LDS group offsets (1 group = 32 points x 4 features = 512 B); PART = 8 K-part slots of 8 groups
constexpr int G_XE = 0, G_TE = 16, G_H = 24, G_TIN = 88, G_PART = 92, G_TOTAL = 156;
// ------------------------------------------------------------------------------------------------
// packing plan (host): which A-operand images exist and where
// ------------------------------------------------------------------------------------------------
struct PackJob {
    int src;            // parameter index (weight)
    int transpose;      // 0: A[n][f] = W[n][f]; 1: A[n][f] = W[f][n] (n over input features)
    int ntiles, nchunks;
    int nseg_n, nseg_f;
    Seg segn[3], segf[3];
    int off;            // float offset in packed buffer
};
struct BiasJob {
    int src;            // parameter index (bias)
    int npad;
    int nseg;
    Seg seg[3];
    int off;
};

struct Plan : Params {
    Flags F;
    std::vector<PackJob> jobs;
    std::vector<BiasJob> biases;
    // forward A images
    int fT1, fT2, fL[8], fHd;
    // forward biases (padded)
    int bT1, bT2, bL[8], bHd;
    // backward A images (transposed)
    int tHd, tL[8], tT2;
    int total;
};

Plan make_plan(int flags) {
    Plan P;
    P.F = make_flags(flags);
    const Flags &F = P.F;
    static_cast<Params &>(P) = make_params(F);
    int off = 0;
    auto add_job = [&](int src, int tr, int ntiles, int nchunks, int nsn, const Seg *sn, int nsf, const Seg *sf) {
        PackJob j{};
        j.src = src; j.transpose = tr; j.ntiles = ntiles; j.nchunks = nchunks;
        j.nseg_n = nsn; j.nseg_f = nsf;
        for (int q = 0; q < nsn; q++) j.segn[q] = sn[q];
        for (int q = 0; q < nsf; q++) j.segf[q] = sf[q];
        j.off = off;
        off += ntiles * nchunks * 256;
        P.jobs.push_back(j);
        return j.off;
    };
    auto add_bias = [&](int src, int npad, int ns, const Seg *s) {
        BiasJob b{};
        b.src = src; b.npad = npad; b.nseg = ns;
        for (int q = 0; q < ns; q++) b.seg[q] = s[q];
        b.off = off;
        off += npad;
        P.biases.push_back(b);
        return b.off;
    };
    Seg full256 = seg(0, 256, 0);
    if (F.blender) {
        Seg sf = seg(0, F.tin, 0);
        P.fT1 = add_job(P.pT0w, 0, 8, 2, 1, &full256, 1, &sf);
        Seg sn = seg(0, 30, 0);
        P.fT2 = add_job(P.pT2w, 0, 1, 32, 1, &sn, 1, &full256);
        P.bT1 = add_bias(P.pT0b, 256, 1, &full256);
        P.bT2 = add_bias(P.pT2b, 32, 1, &sn);
        // backward: A[n = TH feature][f = TE feature] = W_T2[f][n]
        P.tT2 = add_job(P.pT2w, 1, 8, 4, 1, &full256, 1, &sn);
    } else {
        P.fT1 = P.fT2 = P.bT1 = P.bT2 = P.tT2 = -1;
    }
    for (int i = 0; i < 8; i++) {
        Seg s[3];
        int ns = layer_in_segs(F, i, s);
        int kp = layer_kpad(i);
        P.fL[i] = add_job(P.pLw[i], 0, 8, kp / 8, 1, &full256, ns, s);
        P.bL[i] = add_bias(P.pLb[i], 256, 1, &full256);
        // backward image: rows = padded input features (kp), contraction over the 256 outputs
        P.tL[i] = add_job(P.pLw[i], 1, kp / 32, 32, ns, s, 1, &full256);
    }
    // heads: rows stacked in output order
    {
        // one job per head linear writing into row ranges of one 32-row tile: emulate by segments
        // on n with distinct sources is not expressible (different src params) -> pack per head.
        int base = off;
        off += 1 * 32 * 256;  // forward image, 1 n-tile x 32 chunks
        int tbase = off;
        off += 8 * 4 * 256;   // transposed image, 8 tiles x 4 chunks
        int bbase = off;
        off += 32;
        int r0 = 0;
        for (int h = 0; h < P.nheads; h++) {
            PackJob j{};
            j.src = P.pHw[h]; j.transpose = 0; j.ntiles = 1; j.nchunks = 32;
            j.nseg_n = 1; j.segn[0] = seg(r0, P.hrows[h], 0);
            j.nseg_f = 1; j.segf[0] = full256;
            j.off = base;
            P.jobs.push_back(j);
            PackJob t{};
            t.src = P.pHw[h]; t.transpose = 1; t.ntiles = 8; t.nchunks = 4;
            t.nseg_n = 1; t.segn[0] = full256;
            t.nseg_f = 1; t.segf[0] = seg(r0, P.hrows[h], 0);
            t.off = tbase;
            P.jobs.push_back(t);
            BiasJob b{};
            b.src = P.pHb[h]; b.npad = 32; b.nseg = 1; b.seg[0] = seg(r0, P.hrows[h], 0);
            b.off = bbase;
            P.biases.push_back(b);
            r0 += P.hrows[h];
        }
        P.fHd = base;
        P.tHd = tbase;
        P.bHd = bbase;
    }
    P.total = off;
    return P;
}

// Packing is one gather launch: map[i] = (parameter << 22) | element for packed float i, or -1 for
// zero padding. The map depends only on the flags (built once on the host, cached on the device).
constexpr int PACK_MAXP = 32;
constexpr int PACK_SHIFT = 22;
struct PackPtrs {
    const float *p[PACK_MAXP];
};

__global__ __launch_bounds__(256) void k_pack_map(const int *__restrict__ map, PackPtrs src, float *__restrict__ packed,
                                                  int total) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int c = map[i];
    packed[i] = c < 0 ? 0.f : src.p[c >> PACK_SHIFT][c & ((1 << PACK_SHIFT) - 1)];
}


// ------------------------------------------------------------------------------------------------
// device GEMM pieces
// ------------------------------------------------------------------------------------------------
__device__ inline f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; i++) z[i] = 0.f;
    return z;
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

#ifdef DGS_MLP_PROFILE  // diagnostic build only (tools/mlp_phase.cpp): per-phase s_memtime stamps
__device__ unsigned long long *dgs_mlp_prof;
#define DGS_STAMP(k)                                                                                \
    do {                                                                                            \
        if (threadIdx.x == 0) dgs_mlp_prof[blockIdx.x * 256 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define DGS_STAMP(k) \
    do {             \
    } while (0)
#endif

// The network inputs (positional encodings) leave LDS for the saved-activation array in the first
// trunk GEMM's prologue: XE and TE are adjacent both in LDS (groups 0..23) and in the saved rows
// (S_XE.. S_XE + 95), TIN (blender) is one more range. A unit = 4 features x 1 point: one
// ds_read_b128 + 4 coalesced stores; a fixed unit count keeps the GEMM straight-line.
struct InputStore {
    const float4 *lds;
    float *dst;
    size_t Ns;
    int p0, tid;
    bool blender;
    __device__ void put(int g, int m, int row) const {
        const float4 v = lds[g * BM + m];
        float *d = dst + (size_t)row * Ns + p0 + m;
        d[0] = v.x;
        d[Ns] = v.y;
        d[2 * Ns] = v.z;
        d[3 * Ns] = v.w;
    }
    __device__ void operator()() const {
        static_assert(G_TE == G_XE + 16 && S_TE == S_XE + 64, "XE|TE must be one range");
#pragma unroll
        for (int u = 0; u < 2; u++) {  // 24 groups x 32 points = 768 units over 512 threads
            const int e = min(tid + NTHR * u, 24 * BM - 1);  // past the end: rewrite the last unit
            put(G_XE + e / BM, e % BM, S_XE + 4 * (e / BM));
        }
        if (blender && tid < 4 * BM) put(G_TIN + tid / BM, tid % BM, S_TIN + 4 * (tid / BM));  // waves 0-1
    }
};

struct NoPre {
    __device__ void operator()() const {}
};

// The previous layer's output tile of this wave (rows n0 + 8(r>>2) + 4h + (r&3), point m), kept in
// registers and written to a feature-major [rows][Ns] array during the first two chunks of the
// next GEMM: 8 plain coalesced stores per chunk, issued after that GEMM's prologue loads so no
// A-fragment wait depends on them, with no LDS read and no index arithmetic.
struct NoStash {
    __device__ void store(int) const {}
};

struct Stash1 {
    f32x16 t;
    TileAddr d;
    __device__ void store(int k) const {
#pragma unroll
        for (int j = 0; j < 8; j++) d.st(8 * k + j, t[8 * k + j]);
    }
    __device__ void store_all() const {
        store(0);
        store(1);
    }
};

// acc += A . X over NCH chunks starting at chunk c0 of the A image and of the LDS image at group g0
// (chunk c = groups g0 + 2c + h). Fully unrolled straight-line schedule: per chunk the A fragment 4
// chunks ahead (4-deep ring) and the next chunk's B (double-buffered ds_read_b128) are issued
// before this chunk's 4 MFMAs (sched_barrier keeps that order; the scheduler otherwise sinks the
// loads next to their use; the dependent MFMA chain is covered by the SIMD's other 3 waves), and
// the stash stores in chunks 0-1. pre() runs after the A prologue (its loads are younger than the
// first fragments).
template <int NCH, class Pre = NoPre, class Stash = NoStash>
__device__ inline void gemm(const float4 *__restrict__ Apk, int c0, const float4 *lds, int g0, int lane, f32x16 &acc,
                            Pre pre = Pre(), const Stash stash = Stash()) {
    static_assert(NCH >= 1, "empty GEMM");
    const int h = lane >> 5, m = lane & 31;
    const float4 *Ap = Apk + c0 * 64 + lane;
    const float4 *Bp = lds + (g0 + 2 * c0 + h) * BM + m;
    float4 ring[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < NCH) ring[k] = Ap[k * 64];
    pre();
    float4 bx[2];
    bx[0] = Bp[0];
#pragma unroll
    for (int k = 0; k < NCH; k++) {
        const float4 a = ring[k & 3];
        if (k + 4 < NCH) ring[k & 3] = Ap[(k + 4) * 64];
        if (k + 1 < NCH) bx[(k + 1) & 1] = Bp[2 * (k + 1) * BM];
        __builtin_amdgcn_sched_barrier(0);
        const float4 b = bx[k & 1];
        acc = MFMA(a.x, b.x, acc);
        acc = MFMA(a.y, b.y, acc);
        acc = MFMA(a.z, b.z, acc);
        acc = MFMA(a.w, b.w, acc);
        if (k < 2) stash.store(k);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// timenet layer 0 (2 chunks) with its A fragments loaded by the caller (before the PE phase)
__device__ inline void gemm_t1(const float4 a0, const float4 a1, const float4 *lds, int g0, int lane, f32x16 &acc) {
    const int h = lane >> 5, m = lane & 31;
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const float4 a = c ? a1 : a0;
        const float4 b = lds[(g0 + 2 * c + h) * BM + m];
        acc = MFMA(a.x, b.x, acc);
        acc = MFMA(a.y, b.y, acc);
        acc = MFMA(a.z, b.z, acc);
        acc = MFMA(a.w, b.w, acc);
    }
}

// accumulator (n-tile base n0) -> LDS groups starting at gout
__device__ inline void acc_to_lds(const f32x16 &acc, float4 *lds, int gout, int n0, int lane) {
    const int h = lane >> 5, m = lane & 31;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int f = n0 + 8 * j + 4 * h;
        lds[(gout + f / 4) * BM + m] = make_float4(acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]);
    }
}

// bias of this lane's accumulator rows (n0 + 8j + 4h .. +3, j < 4), loaded ahead of the GEMM
struct Bias4 {
    float4 v[4];
};

__device__ inline Bias4 load_bias(const float *bias, int n0, int lane) {
    const int h = lane >> 5;
    Bias4 b;
#pragma unroll
    for (int j = 0; j < 4; j++) b.v[j] = *reinterpret_cast<const float4 *>(bias + n0 + 8 * j + 4 * h);
    return b;
}


// acc = relu(acc + bias) in place (the values kept for the deferred store)
__device__ inline void bias_relu(f32x16 &acc, const Bias4 &b) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        acc[4 * j] = fmaxf(acc[4 * j] + b.v[j].x, 0.f);
        acc[4 * j + 1] = fmaxf(acc[4 * j + 1] + b.v[j].y, 0.f);
        acc[4 * j + 2] = fmaxf(acc[4 * j + 2] + b.v[j].z, 0.f);
        acc[4 * j + 3] = fmaxf(acc[4 * j + 3] + b.v[j].w, 0.f);
    }
}

// LDS groups [g0, g0+ng) (features 4*ng) -> global rows [row0, row0 + 4ng) of a [rows][Ns] array
__device__ inline void lds_to_global(const float4 *lds, int g0, int ng, float *__restrict__ dst, int row0, size_t Ns,
                                     int p0, int tid) {
    // thread -> (feature, point): consecutive threads = consecutive points (coalesced)
    for (int e = tid; e < ng * 4 * BM; e += NTHR) {
        int m = e % BM;
        int f = e / BM;
        const float *src = reinterpret_cast<const float *>(lds + (g0 + f / 4) * BM + m);
        dst[(size_t)(row0 + f) * Ns + p0 + m] = src[f & 3];
    }
}

// 8 K-part partials (PART slots) -> sum in a fixed order (+bias) -> LDS groups gout..gout+7
__device__ inline void sum_parts(float4 *lds, int gout, const float *bias, int tid, bool accumulate) {
    for (int e = tid; e < 8 * BM; e += NTHR) {
        const int gi = e / BM, m = e % BM;
        float4 r = lds[(G_PART + gi) * BM + m];
#pragma unroll
        for (int q = 1; q < NWAVE; q++) {
            const float4 v = lds[(G_PART + 8 * q + gi) * BM + m];
            r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
        }
        if (bias) {
            const float4 b = *reinterpret_cast<const float4 *>(bias + 4 * gi);
            r.x += b.x; r.y += b.y; r.z += b.z; r.w += b.w;
        }
        float4 &d = lds[(gout + gi) * BM + m];
        if (accumulate) {
            d.x += r.x; d.y += r.y; d.z += r.z; d.w += r.w;
        } else {
            d = r;
        }
    }
}

// narrow layer (32 output rows): K (32 chunks) split over the 8 waves, 4 chunks each, partials
// summed in a fixed order (+bias) into LDS groups gout..gout+7
template <class Stash = NoStash>
__device__ inline void narrow_layer(const float4 *Apk, float4 *lds, int g0, int gout, const float *bias, int wave,
                                    int lane, int tid, const Stash stash = Stash()) {
    f32x16 acc = zero16();
    gemm<4>(Apk, wave * 4, lds, g0, lane, acc, NoPre(), stash);
    acc_to_lds(acc, lds, G_PART + 8 * wave, 0, lane);
    lds_barrier();
    sum_parts(lds, gout, bias, tid, false);
    lds_barrier();
}

// ------------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------------
struct FwdArgs {
    int N;
    size_t Ns;
    const float *xyz, *t;
    const float *packed;
    float *out;
    float *saved;
    uint32_t *mask;  // relu' bits, [block][nmask] words (after the saved rows)
    float *tc;       // timenet of t[0] (k_timenet), or nullptr
    int fT1, fT2, fL[8], fHd, bT1, bT2, bL[8], bHd;
    int flags;
};

// The reference feeds every Gaussian the same frame time (render(): fid.unsqueeze(0).expand(N, 1),
// train_baseline.py:107-108), so the timenet (time_utils.py:74-76, 13 -> 256 -> 30) has one value
// per launch. k_timenet evaluates it for t[0] (fp32, one workgroup); a k_mlp_fwd block whose points
// all carry that t broadcasts TE / TH instead of running T1, T2 and the t encodings per point.
__global__ __launch_bounds__(256) void k_timenet(FwdArgs a) {
    __shared__ float tin[16], th[256];
    const int j = threadIdx.x;
    const float t0 = a.t[0];
    const int tinF = 13;  // blender: t, sin / cos of 2^i t, i < 6
    if (j < 16) {
        float v = 0.f;
        if (j == 0) {
            v = t0;
        } else if (j < tinF) {
            float sv, cv;
            sincosf(t0 * (float)(1 << ((j - 1) >> 1)), &sv, &cv);
            v = (j & 1) ? sv : cv;
        }
        tin[j] = v;
        a.tc[TC_TIN + j] = v;
    }
    if (j == 0) a.tc[TC_T] = t0;
    __syncthreads();
    {  // TH[j]: A image element [tile j/32][chunk c][lane 32h + j%32] = W_T1[j][8c + 4h .. +3]
        const float4 *A = reinterpret_cast<const float4 *>(a.packed + a.fT1) + (j >> 5) * 2 * 64 + (j & 31);
        float acc = a.packed[a.bT1 + j];
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const float4 w = A[c * 64 + h * 32];
                const int f = 8 * c + 4 * h;
                acc += w.x * tin[f] + w.y * tin[f + 1] + w.z * tin[f + 2] + w.w * tin[f + 3];
            }
        acc = fmaxf(acc, 0.f);
        th[j] = acc;
        a.tc[TC_TH + j] = acc;
    }
    __syncthreads();
    {  // TE[k], k < 32 (rows 30, 31 are zero padding): 8 lanes per output, 32 features each
        const int k = j >> 3, q = j & 7;
        const float4 *A = reinterpret_cast<const float4 *>(a.packed + a.fT2);
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < 8; u++) {  // features 32q + 4u .. +3: chunk (32q + 4u) / 8, half u & 1
            const int f = 32 * q + 4 * u;
            const float4 w = A[(f >> 3) * 64 + ((f >> 2) & 1) * 32 + k];
            acc += w.x * th[f] + w.y * th[f + 1] + w.z * th[f + 2] + w.w * th[f + 3];
        }
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        acc += __shfl_xor(acc, 4);
        if (q == 0) a.tc[TC_TE + k] = acc + a.packed[a.bT2 + k];
    }
}

// Workgroup = 32 points x 8 waves (wave w owns output rows 32w..32w+31 of every 256-wide layer);
// 80 KB of LDS, so two workgroups share a CU (4 waves per SIMD): one block's barrier waits and
// epilogues run under the other's MFMAs, and a partial last round of blocks runs at full rate.
template <bool SAVE>
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_mlp_fwd(FwdArgs a) {
    __shared__ float4 lds[G_TOTAL * BM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (scalar branches)
    const int p0 = blockIdx.x * BM;
    const Flags F = make_flags(a.flags);
    const float4 *pk = reinterpret_cast<const float4 *>(a.packed);
    float *lf = reinterpret_cast<float *>(lds);
    const __amdgpu_buffer_rsrc_t mrsrc =
        __builtin_amdgcn_make_buffer_rsrc(a.mask + (SAVE ? (size_t)blockIdx.x * F.nmask : 0), 0, 0x7fffffff, 0x00020000);
    DGS_STAMP(0);
#ifdef DGS_MLP_PROFILE
    if (threadIdx.x == 0) {
        dgs_mlp_prof[blockIdx.x * 256 + 252] = __builtin_amdgcn_s_memrealtime();
        dgs_mlp_prof[blockIdx.x * 256 + 253] = __builtin_amdgcn_s_memtime();
    }
#endif
    // frame-uniform t: every valid point of the block carries k_timenet's t0 (wave-local check on the
    // same 32 values in every wave, so the branch is block-uniform without a barrier)
    float tv_own = 0.f, tc_t0 = 1.f;
    if (SAVE && F.blender && a.tc) {
        tc_t0 = a.tc[TC_T];
        tv_own = (lane < BM && p0 + lane < a.N) ? a.t[p0 + lane] : tc_t0;
    }
    // timenet layer 0 operands, in flight during the positional encodings
    float4 t1a0 = make_float4(0.f, 0.f, 0.f, 0.f), t1a1 = t1a0;
    Bias4 t1b{};
    if (F.blender) {
        const float4 *At1 = pk + a.fT1 / 4 + wave * 2 * 64 + lane;
        t1a0 = At1[0];
        t1a1 = At1[64];
        t1b = load_bias(a.packed + a.bT1, wave * 32, lane);
    }
    // ---- positional encodings (utils/time_utils.py:42-54): feature 3 band + d, band 0 = x,
    // band 1 + 2i = sin(2^i x), band 2 + 2i = cos(2^i x); one sincosf per (point, dim, frequency) ----
    bool uniform_t = false;
    auto put = [&](int g0, int f, int m, float v) { lf[((g0 + f / 4) * BM + m) * 4 + (f & 3)] = v; };
    {
        for (int e = tid; e < BM * 3 * 11; e += NTHR) {
            const int m = e % BM, r = e / BM, d = r % 3, i = r / 3;  // i = 10: identity band
            const int p = p0 + m;
            const float x = p < a.N ? a.xyz[3 * p + d] : 0.f;
            if (i == 10) {
                put(G_XE, d, m, p < a.N ? x : 0.f);
            } else {
                float sv, cv;
                sincosf(x * (float)(1 << i), &sv, &cv);
                put(G_XE, 3 * (1 + 2 * i) + d, m, p < a.N ? sv : 0.f);
                put(G_XE, 3 * (2 + 2 * i) + d, m, p < a.N ? cv : 0.f);
            }
        }
        for (int m = tid; m < BM; m += NTHR) put(G_XE, 63, m, 0.f);  // padding feature
        uniform_t = SAVE && F.blender && a.tc && __ballot(tv_own != tc_t0) == 0;
    }
    if (uniform_t) {  // TE and TIN images: k_timenet's values broadcast over the 32 points
        const float4 *tc4 = reinterpret_cast<const float4 *>(a.tc);
        for (int e = tid; e < 12 * BM; e += NTHR) {
            const int gi = e / BM, m = e % BM;
            if (gi < 8) lds[(G_TE + gi) * BM + m] = tc4[TC_TE / 4 + gi];
            else lds[(G_TIN + gi - 8) * BM + m] = tc4[TC_TIN / 4 + gi - 8];
        }
    } else {
        const int tg = F.blender ? G_TIN : G_TE;
        const int nfreq = (F.tin - 1) / 2, ng = F.blender ? 4 : 8;
        for (int e = tid; e < BM * 4 * ng; e += NTHR) {  // zero the whole t image (padding)
            const int m = e % BM, f = e / BM;
            if (f >= F.tin) put(tg, f, m, 0.f);
        }
        for (int e = tid; e < BM * (nfreq + 1); e += NTHR) {
            const int m = e % BM, i = e / BM;  // i = nfreq: identity
            const int p = p0 + m;
            const float x = p < a.N ? a.t[p] : 0.f;
            if (i == nfreq) {
                put(tg, 0, m, x);
            } else {
                float sv, cv;
                sincosf(x * (float)(1 << i), &sv, &cv);
                put(tg, 1 + 2 * i, m, p < a.N ? sv : 0.f);
                put(tg, 2 + 2 * i, m, p < a.N ? cv : 0.f);
            }
        }
    }
    lds_barrier();
    DGS_STAMP(1);
    // saved activations: the network inputs (XE|TE, TIN) leave LDS in the first trunk GEMM's
    // prologue (InputStore); every hidden layer's output is kept in registers and stored during the
    // next GEMM (Stash1)
    const float *bias = a.packed;
    f32x16 kt = zero16();  // previous layer's activations, awaiting their store
    // ---- timenet (blender): Linear(13,256) + ReLU -> H ; Linear(256,30) -> TE ----
    if (uniform_t) {  // TH tile of this wave from k_timenet: relu' bits and the saved rows
        const Bias4 th = load_bias(a.tc + TC_TH, wave * 32, lane);
        f32x16 c;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            c[4 * j] = th.v[j].x;
            c[4 * j + 1] = th.v[j].y;
            c[4 * j + 2] = th.v[j].z;
            c[4 * j + 3] = th.v[j].w;
        }
        store_mask_bits(c, mrsrc, (M_TH + wave * 32) * 4, lane);
        Stash1{c, tile_addr(a.saved, a.Ns, S_TH, wave * 32, p0, lane)}.store_all();
        DGS_STAMP(2);
    } else if (F.blender) {
        f32x16 c = zero16();
        gemm_t1(t1a0, t1a1, lds, G_TIN, lane, c);
        bias_relu(c, t1b);
        if (SAVE) store_mask_bits(c, mrsrc, (M_TH + wave * 32) * 4, lane);
        acc_to_lds(c, lds, G_H, wave * 32, lane);
        lds_barrier();
        DGS_STAMP(2);
        if (SAVE)
            narrow_layer(pk + a.fT2 / 4, lds, G_H, G_TE, bias + a.bT2, wave, lane, tid,
                         Stash1{c, tile_addr(a.saved, a.Ns, S_TH, wave * 32, p0, lane)});
        else
            narrow_layer(pk + a.fT2 / 4, lds, G_H, G_TE, bias + a.bT2, wave, lane, tid);
    }
    DGS_STAMP(3);
    // ---- trunk: 8 x (Linear + ReLU), skip cat after layer 4 (time_utils.py:107-112) ----
    for (int L = 0; L < 8; L++) {
        const int g0 = (L == 0 || L == 5) ? G_XE : G_H;
        const int nch = layer_kpad(L) / 8;
        f32x16 c = zero16();
        const float4 *Aw = pk + a.fL[L] / 4 + wave * nch * 64;
        const Bias4 bv = load_bias(bias + a.bL[L], wave * 32, lane);
        if (L == 0) {
            if (SAVE) gemm<12>(Aw, 0, lds, g0, lane, c, InputStore{lds, a.saved, a.Ns, p0, tid, F.blender});
            else gemm<12>(Aw, 0, lds, g0, lane, c);
        } else {
            const Stash1 st{kt, tile_addr(a.saved, a.Ns, s_h(L - 1), wave * 32, p0, lane)};
            if (L == 5) {
                if (SAVE) gemm<44>(Aw, 0, lds, g0, lane, c, NoPre(), st);
                else gemm<44>(Aw, 0, lds, g0, lane, c);
            } else {
                if (SAVE) gemm<32>(Aw, 0, lds, g0, lane, c, NoPre(), st);
                else gemm<32>(Aw, 0, lds, g0, lane, c);
            }
        }
        DGS_STAMP(4 + 3 * L);
        lds_barrier();  // all waves finished reading H before it is overwritten
        DGS_STAMP(5 + 3 * L);
        bias_relu(c, bv);
        if (SAVE) store_mask_bits(c, mrsrc, (m_h(L) + wave * 32) * 4, lane);
        acc_to_lds(c, lds, G_H, wave * 32, lane);
        lds_barrier();
        DGS_STAMP(6 + 3 * L);
        kt = c;
    }
    // ---- heads (no activation): [warp | branch_w, branch_v], rotation, scaling -> TE region ----
    if (SAVE)
        narrow_layer(pk + a.fHd / 4, lds, G_H, G_TE, bias + a.bHd, wave, lane, tid,
                     Stash1{kt, tile_addr(a.saved, a.Ns, s_h(7), wave * 32, p0, lane)});
    else
        narrow_layer(pk + a.fHd / 4, lds, G_H, G_TE, bias + a.bHd, wave, lane, tid);
    DGS_STAMP(28);
    for (int e = tid; e < F.nout * BM; e += NTHR) {
        int c = e % F.nout, m = e / F.nout;
        int p = p0 + m;
        if (p < a.N) a.out[(size_t)p * F.nout + c] = lf[((G_TE + c / 4) * BM + m) * 4 + (c & 3)];
    }
    DGS_STAMP(29);
#ifdef DGS_MLP_PROFILE
    if (threadIdx.x == 0) {  // shader-clock rate: s_memtime vs the 100 MHz s_memrealtime
        dgs_mlp_prof[blockIdx.x * 256 + 254] = __builtin_amdgcn_s_memrealtime();
        dgs_mlp_prof[blockIdx.x * 256 + 255] = __builtin_amdgcn_s_memtime();
    }
#endif
}

// ------------------------------------------------------------------------------------------------
// backward (dX chain): dZ_i for every layer -> scratch; deterministic
// ------------------------------------------------------------------------------------------------
struct BwdArgs {
    int N;
    size_t Ns;
    const float *packed;
    const float *saved;
    const uint32_t *mask;
    const float *dout;
    float *dz;
    int tHd, tL[8], tT2;
    int flags;
};

// relu' of the layer input for this wave's 32x32 tile: the forward's 16 bits per lane (same lane
// layout), one u16 load per lane ahead of the GEMM instead of 16 activation loads
struct MaskBits {
    uint32_t w;
};

struct MaskPre {
    MaskBits *mk;
    const uint32_t *words;  // &mask[block][mrow0 + n0]: 64 u16, one per lane
    int lane;
    __device__ void operator()() const {
        mk->w = reinterpret_cast<const unsigned short *>(words)[lane];
    }
};

__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_mlp_bwd(BwdArgs a) {
    __shared__ float4 lds[G_TOTAL * BM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (scalar branches)
    const int p0 = blockIdx.x * BM;
    const Flags F = make_flags(a.flags);
    const float4 *pk = reinterpret_cast<const float4 *>(a.packed);
    float *lf = reinterpret_cast<float *>(lds);
    const uint32_t *mwords = a.mask + (size_t)blockIdx.x * F.nmask + wave * 32;  // + mask row
    // dOut -> LDS TE region (the head-gradient image G) and dz rows Z_G
    for (int e = tid; e < 32 * BM; e += NTHR) {
        int m = e % BM, c = e / BM;
        int p = p0 + m;
        float v = (p < a.N && c < F.nout) ? a.dout[(size_t)p * F.nout + c] : 0.f;
        lf[((G_TE + c / 4) * BM + m) * 4 + (c & 3)] = v;
        a.dz[(size_t)(Z_G + c) * a.Ns + p] = v;
    }
    lds_barrier();
    // dZ_i of the trunk stays in registers and is stored during the next GEMM (Stash1)
    f32x16 kt;  // dZ of the layer whose GEMM runs next
    // heads^T: dH7 = W_h^T dOut (K = 32 from TE region) -> mask H7 -> dZ7
    {
        MaskBits mk;
        f32x16 c = zero16();
        gemm<4>(pk + a.tHd / 4 + wave * 4 * 64, 0, lds, G_TE, lane, c, MaskPre{&mk, mwords + m_h(7), lane});
        mask_apply(c, mk.w);
        lds_barrier();  // TE (dOut image) reads done before TE is reused for dTE
        acc_to_lds(c, lds, G_H, wave * 32, lane);
        kt = c;
    }
    // zero the dTE accumulator (TE region holds dL/dt_emb from layers 5 and 0)
    for (int e = tid; e < 8 * BM; e += NTHR) lds[G_TE * BM + e] = make_float4(0.f, 0.f, 0.f, 0.f);
    lds_barrier();
    for (int L = 7; L >= 1; L--) {
        // dX_L = W_L^T dZ_L ; H-part rows of the padded input live at tiles (F_H/32 + w) for L=5
        const int tile0 = (L == 5) ? F_H / 32 : 0;
        if (L == 5 && F.blender) {
            // t_emb slice (padded rows 64..95 = tile 2): K split over the 8 waves -> PART
            f32x16 ct = zero16();
            gemm<4>(pk + a.tL[5] / 4 + (F_TE / 32) * 32 * 64, wave * 4, lds, G_H, lane, ct);
            acc_to_lds(ct, lds, G_PART + 8 * wave, 0, lane);
        }
        MaskBits mk;  // relu' of H_{L-1}, in flight during the GEMM
        f32x16 c = zero16();
        gemm<32>(pk + a.tL[L] / 4 + (tile0 + wave) * 32 * 64, 0, lds, G_H, lane, c, MaskPre{&mk, mwords + m_h(L - 1), lane},
                 Stash1{kt, tile_addr(a.dz, a.Ns, Z_L0 + L * 256, wave * 32, p0, lane)});
        mask_apply(c, mk.w);
        lds_barrier();
        if (L == 5 && F.blender) sum_parts(lds, G_TE, nullptr, tid, true);
        acc_to_lds(c, lds, G_H, wave * 32, lane);
        lds_barrier();
        kt = c;
    }
    const Stash1 dz0{kt, tile_addr(a.dz, a.Ns, Z_L0, wave * 32, p0, lane)};
    if (!F.blender) {
        dz0.store_all();
        return;  // raw t PE has no parameters upstream of it
    }
    // layer 0: t_emb slice of W_0^T dZ_0 (K split over the waves); dZ_0 is stored under it
    {
        f32x16 ct = zero16();
        gemm<4>(pk + a.tL[0] / 4 + (F_TE / 32) * 32 * 64, wave * 4, lds, G_H, lane, ct, NoPre(), dz0);
        acc_to_lds(ct, lds, G_PART + 8 * wave, 0, lane);
        lds_barrier();
        sum_parts(lds, G_TE, nullptr, tid, true);
        lds_barrier();
    }
    // dTE (30 real rows) -> global (dW of timenet.2)
    lds_to_global(lds, G_TE, 8, a.dz, Z_TE, a.Ns, p0, tid);
    // timenet.2^T: dTH = W_T2^T dTE (K = 32) -> mask TH -> dZ_T1
    {
        MaskBits mk;
        f32x16 c = zero16();
        gemm<4>(pk + a.tT2 / 4 + wave * 4 * 64, 0, lds, G_TE, lane, c, MaskPre{&mk, mwords + M_TH, lane});
        mask_apply(c, mk.w);
        Stash1{c, tile_addr(a.dz, a.Ns, Z_T1, wave * 32, p0, lane)}.store_all();
    }
}

// ------------------------------------------------------------------------------------------------
// dW = dZ X^T over all points: one 256x256 tile per layer (L5: 256 + 96 input columns), split over
// the point axis in proportion to each tile's work so ~one workgroup per CU finishes together;
// fixed-order slab reduction (deterministic).
// ------------------------------------------------------------------------------------------------
constexpr int PC = 32;             // points per LDS chunk
constexpr int LDA = PC + 4;        // padded LDS row (floats)
constexpr int DW_THREADS = 512;    // 8 waves: 2 (n) x 4 (k), 128 x 64 per wave

// component-wise select (a select of the float4 struct itself can be lowered through scratch)
__device__ inline float4 zsel4(float4 v, bool ok) {
    return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}

template <bool NARROW>
__device__ __forceinline__ void dw_tile(const WJob &J, size_t Ns, const float *__restrict__ dz,
                                        const float *__restrict__ saved, float *__restrict__ slabs,
                                        float *ldsf) {
    const int split = blockIdx.x - J.block0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (scalar branches)
    const int wn = wave >> 2, wk = wave & 3;  // wide wave tile: rows [128 wn, +128), cols [64 wk, +64)
    const int h = lane >> 5, i = lane & 31;
    const int nch = (int)(Ns / PC);
    const int per = div_up(nch, J.nsplit);
    const int c0 = split * per;
    const int c1 = min(nch, c0 + per);
    // staging map: element e = tid + 512 j (j < 4): row = e / 8 (0..255), float4 column = e % 8
    const float *baseA = dz + (size_t)J.zrow * Ns;
    const float *baseB = saved + (size_t)J.xrow * Ns;
    const int ns = (int)Ns;  // 256 rows x Ns < 2^31
    const int srow = tid >> 3, scol = (tid & 7) * 4;
#define DW_OFF(lim, j) ((srow + 64 * (j)) < (lim) ? (srow + 64 * (j)) * ns + scol : -1)
    const int oA0 = DW_OFF(J.nrows, 0), oA1 = DW_OFF(J.nrows, 1), oA2 = DW_OFF(J.nrows, 2), oA3 = DW_OFF(J.nrows, 3);
    const int oB0 = DW_OFF(J.krows, 0), oB1 = DW_OFF(J.krows, 1), oB2 = DW_OFF(J.krows, 2), oB3 = DW_OFF(J.krows, 3);
#undef DW_OFF
    float4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
    // rows past the job's extent load row 0 (always valid) and are zeroed at the LDS store (after
    // the chunk's MFMAs, so the loads stay in flight across them): an
    // unconditional global_load keeps hipcc from turning `ok ? *p : 0` into a flat load of a
    // pointer select between global memory and a scratch-held zero
    // 32-bit byte offsets from a uniform base -> global_load with an SGPR base (saddr) and one
    // offset VGPR per load instead of a 64-bit address pair
#define DW_U(o) ((uint32_t)(((o) >= 0 ? (o) : scol) * 4))
    const uint32_t uA0 = DW_U(oA0), uA1 = DW_U(oA1), uA2 = DW_U(oA2), uA3 = DW_U(oA3);
    const uint32_t uB0 = DW_U(oB0), uB1 = DW_U(oB1), uB2 = DW_U(oB2), uB3 = DW_U(oB3);
#undef DW_U
#define DW_LD(base, u, po) (*reinterpret_cast<const float4 *>(reinterpret_cast<const char *>(base) + (uint32_t)((u) + (uint32_t)(po) * 4u)))
#define DW_Z(v, o) zsel4((v), (o) >= 0)
#define DW_GLOAD(c)                                                                                        \
    do {                                                                                                   \
        const int po_ = (c) * PC;                                                                          \
        ra0 = DW_LD(baseA, uA0, po_); ra1 = DW_LD(baseA, uA1, po_);                                        \
        ra2 = DW_LD(baseA, uA2, po_); ra3 = DW_LD(baseA, uA3, po_);                                        \
        rb0 = DW_LD(baseB, uB0, po_); rb1 = DW_LD(baseB, uB1, po_);                                        \
        rb2 = DW_LD(baseB, uB2, po_); rb3 = DW_LD(baseB, uB3, po_);                                        \
    } while (0)
#define DW_LSTORE(buf)                                                                                     \
    do {                                                                                                   \
        float *A_ = ldsf + (buf) * (2 * WT * LDA);                                                         \
        float *B_ = A_ + WT * LDA;                                                                         \
        const int row_ = tid >> 3, col_ = (tid & 7) * 4;                                                   \
        *reinterpret_cast<float4 *>(A_ + (row_ + 0) * LDA + col_) = DW_Z(ra0, oA0);                        \
        *reinterpret_cast<float4 *>(A_ + (row_ + 64) * LDA + col_) = DW_Z(ra1, oA1);                       \
        *reinterpret_cast<float4 *>(A_ + (row_ + 128) * LDA + col_) = DW_Z(ra2, oA2);                      \
        *reinterpret_cast<float4 *>(A_ + (row_ + 192) * LDA + col_) = DW_Z(ra3, oA3);                      \
        *reinterpret_cast<float4 *>(B_ + (row_ + 0) * LDA + col_) = DW_Z(rb0, oB0);                        \
        *reinterpret_cast<float4 *>(B_ + (row_ + 64) * LDA + col_) = DW_Z(rb1, oB1);                       \
        *reinterpret_cast<float4 *>(B_ + (row_ + 128) * LDA + col_) = DW_Z(rb2, oB2);                      \
        *reinterpret_cast<float4 *>(B_ + (row_ + 192) * LDA + col_) = DW_Z(rb3, oB3);                      \
    } while (0)
    // this wave's active sub-tiles (wave-uniform). wide: rows 128 wn + 32 t, cols 64 wk + 32 u
    // (acc[t][u]); narrow: rows 32 wave, cols 32 v (acc[v >> 1][v & 1], v < 4)
    constexpr bool narrow = NARROW;
    const int nact_r = narrow ? (32 * wave < J.nrows ? 1 : 0) : min(4, max(0, div_up(J.nrows - 128 * wn, 32)));
    const int nact_c = narrow ? min(4, div_up(J.krows, 32)) : min(2, max(0, div_up(J.krows - 64 * wk, 32)));
    const bool any = nact_r > 0 && nact_c > 0;
    f32x16 acc[4][2];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        acc[t][0] = zero16();
        acc[t][1] = zero16();
    }
    float bs0 = 0.f, bs1 = 0.f, bs2 = 0.f, bs3 = 0.f;
    if (c0 < c1) {
        DW_GLOAD(c0);
        DW_LSTORE(0);
    }
    __syncthreads();
    for (int c = c0; c < c1; c++) {
        const int buf = (c - c0) & 1;
        const bool more = c + 1 < c1;
        if (more) DW_GLOAD(c + 1);
        const float *A = ldsf + buf * (2 * WT * LDA);
        const float *B = A + WT * LDA;
        if (any && narrow) {
#pragma unroll
            for (int g = 0; g < PC / 8; g++) {
                const int o = 8 * g + 4 * h;
                const float4 a0 = *reinterpret_cast<const float4 *>(A + (32 * wave + i) * LDA + o);
                float4 bb[4];
#pragma unroll
                for (int v = 0; v < 4; v++) bb[v] = *reinterpret_cast<const float4 *>(B + (32 * v + i) * LDA + o);
                bs0 += (a0.x + a0.y) + (a0.z + a0.w);
#pragma unroll
                for (int v = 0; v < 4; v++) {
                    if (v >= nact_c) continue;
                    acc[v >> 1][v & 1] = MFMA(a0.x, bb[v].x, acc[v >> 1][v & 1]);
                    acc[v >> 1][v & 1] = MFMA(a0.y, bb[v].y, acc[v >> 1][v & 1]);
                    acc[v >> 1][v & 1] = MFMA(a0.z, bb[v].z, acc[v >> 1][v & 1]);
                    acc[v >> 1][v & 1] = MFMA(a0.w, bb[v].w, acc[v >> 1][v & 1]);
                }
            }
        } else if (any) {
#pragma unroll
            for (int g = 0; g < PC / 8; g++) {
                const int o = 8 * g + 4 * h;
                float4 a[4], bb[2];
#pragma unroll
                for (int t = 0; t < 4; t++) a[t] = *reinterpret_cast<const float4 *>(A + (128 * wn + 32 * t + i) * LDA + o);
#pragma unroll
                for (int u = 0; u < 2; u++) bb[u] = *reinterpret_cast<const float4 *>(B + (64 * wk + 32 * u + i) * LDA + o);
                if (wk == 0) {
                    bs0 += (a[0].x + a[0].y) + (a[0].z + a[0].w);
                    bs1 += (a[1].x + a[1].y) + (a[1].z + a[1].w);
                    bs2 += (a[2].x + a[2].y) + (a[2].z + a[2].w);
                    bs3 += (a[3].x + a[3].y) + (a[3].z + a[3].w);
                }
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    if (t >= nact_r) continue;
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        if (u >= nact_c) continue;
                        acc[t][u] = MFMA(a[t].x, bb[u].x, acc[t][u]);
                        acc[t][u] = MFMA(a[t].y, bb[u].y, acc[t][u]);
                        acc[t][u] = MFMA(a[t].z, bb[u].z, acc[t][u]);
                        acc[t][u] = MFMA(a[t].w, bb[u].w, acc[t][u]);
                    }
                }
            }
        }
#ifdef DGS_MLP_PROFILE
        if ((c - c0) >= 4 && (c - c0) < 8 && (tid & 63) == 0)
            dgs_mlp_prof[blockIdx.x * 256 + 64 + ((c - c0) - 4) * 16 + wave] = __builtin_amdgcn_s_memtime();
#endif
        if (more) DW_LSTORE(buf ^ 1);
        __syncthreads();
#ifdef DGS_MLP_PROFILE
        if ((c - c0) >= 3 && (c - c0) < 8 && tid == 0)
            dgs_mlp_prof[blockIdx.x * 256 + 160 + ((c - c0) - 3)] = __builtin_amdgcn_s_memtime();
#endif
    }
#undef DW_GLOAD
#undef DW_LSTORE
#undef DW_LD
#undef DW_Z
    float *slab = slabs + (size_t)blockIdx.x * SLAB;
    if (narrow) {
        // rows past nrows / cols past krows hold zeros or partial garbage that k_dw_reduce never reads
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int nb = 32 * wave, kb = 32 * v;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                int n = nb + 8 * (r >> 2) + 4 * h + (r & 3);
                slab[n * WT + kb + i] = acc[v >> 1][v & 1][r];
            }
        }
        float v0 = bs0 + __shfl_xor(bs0, 32);
        if (h == 0) slab[WT * WT + 32 * wave + i] = v0;
        return;
    }
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int nb = 128 * wn + 32 * t, kb = 64 * wk + 32 * u;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                int n = nb + 8 * (r >> 2) + 4 * h + (r & 3);
                slab[n * WT + kb + i] = acc[t][u][r];
            }
        }
    if (wk == 0) {
        // lanes l and l+32 hold the same row
        float v0 = bs0 + __shfl_xor(bs0, 32), v1 = bs1 + __shfl_xor(bs1, 32);
        float v2 = bs2 + __shfl_xor(bs2, 32), v3 = bs3 + __shfl_xor(bs3, 32);
        if (h == 0) {
            slab[WT * WT + 128 * wn + i] = v0;
            slab[WT * WT + 128 * wn + 32 + i] = v1;
            slab[WT * WT + 128 * wn + 64 + i] = v2;
            slab[WT * WT + 128 * wn + 96 + i] = v3;
        }
    }
}

__global__ __launch_bounds__(DW_THREADS) void k_dw(WJobs JT, size_t Ns, const float *__restrict__ dz,
                                                   const float *__restrict__ saved, float *__restrict__ slabs) {
    extern __shared__ float4 dw_lds[];
    // job of this workgroup: static-index selects over the kernel-argument table (no scratch copy)
    WJob J = JT.j[0];
#pragma unroll
    for (int q = 1; q < MAXJ; q++)
        if (q < JT.n && (int)blockIdx.x >= JT.j[q].block0) J = JT.j[q];
#ifdef DGS_MLP_PROFILE
    if (threadIdx.x == 0) dgs_mlp_prof[blockIdx.x * 256 + 200] = __builtin_amdgcn_s_memtime();
#endif
    // the two wave layouts are separate code regions (a runtime switch inside one loop makes the
    // register allocator spill the accumulators)
    if (J.narrow)
        dw_tile<true>(J, Ns, dz, saved, slabs, reinterpret_cast<float *>(dw_lds));
    else
        dw_tile<false>(J, Ns, dz, saved, slabs, reinterpret_cast<float *>(dw_lds));
#ifdef DGS_MLP_PROFILE
    __syncthreads();
    if (threadIdx.x == 0) {
        dgs_mlp_prof[blockIdx.x * 256 + 201] = __builtin_amdgcn_s_memtime();
        dgs_mlp_prof[blockIdx.x * 256 + 202] = (unsigned long long)(J.zrow * 10000 + J.xrow);
        dgs_mlp_prof[blockIdx.x * 256 + 203] = (unsigned long long)J.nsplit;
    }
#endif
}

struct RJob {
    float *dst;        // parameter gradient (rows x cols) or bias (rows)
    int rows, cols;    // cols == 0 -> bias
    int rowpad0;       // padded output row of source row 0 (head stacking)
    int nseg;
    Seg seg[3];        // source col <-> padded feature
    int block0[2];     // first slab of the layer's k-tile 0 / 1 (padded features [0,k1) / [k1,..))
    int nsplit[2];
    int k1;            // padded feature where k-tile 1 starts (WPlan::layer_k1)
};

constexpr int MAXR = 28;
struct RJobs {
    RJob j[MAXR];
    int begin[MAXR + 1];  // element prefix
    int n;
};

// one thread per gradient element of every parameter; sums the splits in a fixed order
// sum of one element over ns slabs in slab order (deterministic): RU loads issued before the adds
// that consume them (one HBM round trip per RU slabs; adding the predicated 0.f is exact)
#ifndef DGS_REDUCE_U
#define DGS_REDUCE_U 8
#endif
__device__ __forceinline__ float slab_sum(const float *sl, int ns) {
    constexpr int RU = DGS_REDUCE_U;
    float s = 0.f;
    for (int b = 0; b < ns; b += RU) {
        float v[RU];
#pragma unroll
        for (int k = 0; k < RU; k++) v[k] = b + k < ns ? sl[(size_t)(b + k) * SLAB] : 0.f;
#pragma unroll
        for (int k = 0; k < RU; k++) s += v[k];
    }
    return s;
}

__global__ __launch_bounds__(256) void k_dw_reduce(RJobs R, const float *__restrict__ slabs) {
    int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= R.begin[R.n]) return;
    int q = 0;
    while (idx >= R.begin[q + 1]) q++;
    const RJob &J = R.j[q];
    idx -= R.begin[q];
    int r = J.cols ? idx / J.cols : idx;
    int n = J.rowpad0 + r;
    float s = 0.f;
    if (J.cols) {
        int c = idx % J.cols;
        int f = -1;
        for (int k = 0; k < J.nseg; k++)
            if (c >= J.seg[k].s0 && c < J.seg[k].s0 + J.seg[k].len) f = J.seg[k].p0 + (c - J.seg[k].s0);
        if (f < 0) return;  // a folded t_emb column: written by k_tgrad
        const int kt = f >= J.k1 ? 1 : 0, kl = f - (kt ? J.k1 : 0);
        const float *sl = slabs + (size_t)J.block0[kt] * SLAB + n * WT + kl;
        s = slab_sum(sl, J.nsplit[kt]);
    } else {
        const float *sl = slabs + (size_t)J.block0[0] * SLAB + WT * WT + n;
        s = slab_sum(sl, J.nsplit[0]);
    }
    J.dst[idx] = s;
}

// fp32 dW split plan: per-chunk cost units calibrated with tools/dw_phase.cpp (full 256 x 256 tile
// 16 + 1.5 units ~ 18.9k cycles, narrow 6 + 1.5 ~ 8.3k, 32-row jobs ~ 4.2k); one 8-wave workgroup per
// CU (LDS 147 KiB)
static WPlan fp32_wplan(const Flags &F) { return make_wplan(F, 256, 1.5, 4.0); }

static size_t padded_points(int N) { return (size_t)div_up(N, BM) * BM; }

size_t packed_floats(int flags) { return (size_t)make_plan(flags).total; }
// saved activations [nsaved][Ns] floats, then the relu' bits [Ns / 32 blocks][nmask] u32 words, then
// the frame-uniform timenet values (TC_FLOATS)
size_t saved_floats(int flags, int N) {
    const Flags F = make_flags(flags);
    return (size_t)F.nsaved * padded_points(N) + (size_t)F.nmask * (padded_points(N) / BM) + TC_FLOATS;
}

size_t scratch_floats(int flags, int N) {
    Flags F = make_flags(flags);
    WPlan W = fp32_wplan(F);
    return (size_t)F.nz * padded_points(N) + (size_t)W.nblocks * SLAB;
}

// host emulation of the packed-image layout (forward A images, transposed backward images, biases)
static std::vector<int> build_pack_map(const Plan &P) {
    std::vector<int> map((size_t)P.total, -1);
    for (const PackJob &j : P.jobs) {
        int r, c;
        param_shape(P.F, P, j.src, r, c);
        const bool head = (j.off == P.fHd || j.off == P.tHd);  // head images are shared by several jobs
        const int total = j.ntiles * j.nchunks * 256;
        for (int idx = 0; idx < total; idx++) {
            int t = idx & 3, lane = (idx >> 2) & 63, rest = idx >> 8;
            int chunk = rest % j.nchunks, ntile = rest / j.nchunks;
            int n = ntile * 32 + (lane & 31);
            int f = chunk * 8 + 4 * (lane >> 5) + t;
            int sn = seg_lookup(j.segn, j.nseg_n, n);
            int sf = seg_lookup(j.segf, j.nseg_f, f);
            bool mine = j.transpose ? (sf >= 0) : (sn >= 0);
            int code = -1;
            if (sn >= 0 && sf >= 0) code = (j.src << PACK_SHIFT) | (j.transpose ? sf * c + sn : sn * c + sf);
            if (mine || !head) map[(size_t)j.off + idx] = code;
        }
    }
    for (const BiasJob &b : P.biases)
        for (int n = 0; n < b.npad; n++) {
            int sidx = seg_lookup(b.seg, b.nseg, n);
            if (sidx >= 0) map[(size_t)b.off + n] = (b.src << PACK_SHIFT) | sidx;
            else if (b.off != P.bHd) map[(size_t)b.off + n] = -1;
        }
    return map;
}

static std::mutex g_map_mu;
static std::map<std::pair<int, int>, int *> g_pack_maps;  // (device, flags) -> device map

static int *pack_map_for(const Plan &P, int flags) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_map_mu);
    auto it = g_pack_maps.find({dev, flags});
    if (it != g_pack_maps.end()) return it->second;
    std::vector<int> h = build_pack_map(P);
    int *d = nullptr;
    if (hipMalloc(&d, h.size() * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemcpy(d, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return nullptr;
    }
    g_pack_maps[{dev, flags}] = d;
    return d;
}

int pack(int flags, const float *const *params, float *packed, hipStream_t stream) {
    Plan P = make_plan(flags);
    if (P.nparams > PACK_MAXP) {
        set_error("dgs_deform_pack: too many parameters");
        return DGS_ERR_ARGS;
    }
    PackPtrs src{};
    for (int k = 0; k < P.nparams; k++) {
        if (!params[k]) {
            set_error("dgs_deform_pack: null parameter pointer");
            return DGS_ERR_ARGS;
        }
        src.p[k] = params[k];
    }
    const int *map = pack_map_for(P, flags);
    if (!map) {
        set_error("dgs_deform_pack: could not allocate the pack map");
        return DGS_ERR_HIP;
    }
    hipLaunchKernelGGL(k_pack_map, dim3(div_up(P.total, 256)), dim3(256), 0, stream, map, src, packed, P.total);
    DGS_LAUNCH_CHECK("k_pack_map", false, stream);
    return DGS_OK;
}

int forward(int flags, int N, const float *xyz, const float *t, const float *packed, float *out, float *saved,
            hipStream_t stream) {
    if (N < 0 || (N > 0 && (!xyz || !t || !packed || !out))) {
        set_error("dgs_deform_forward: null argument");
        return DGS_ERR_ARGS;
    }
    if (N == 0) return DGS_OK;
    Plan P = make_plan(flags);
    FwdArgs a{};
    a.N = N;
    a.Ns = padded_points(N);
    a.xyz = xyz; a.t = t; a.packed = packed; a.out = out; a.saved = saved;
    a.mask = saved ? reinterpret_cast<uint32_t *>(saved + (size_t)P.F.nsaved * a.Ns) : nullptr;
    a.fT1 = P.fT1; a.fT2 = P.fT2; a.fHd = P.fHd; a.bT1 = P.bT1; a.bT2 = P.bT2; a.bHd = P.bHd;
    for (int i = 0; i < 8; i++) { a.fL[i] = P.fL[i]; a.bL[i] = P.bL[i]; }
    a.flags = flags;
    {
        ScopedTimer tm("mlp_fwd", stream);
        if (saved && P.F.blender) {
            a.tc = saved + (size_t)P.F.nsaved * a.Ns + (size_t)P.F.nmask * (a.Ns / BM);
            hipLaunchKernelGGL(k_timenet, dim3(1), dim3(256), 0, stream, a);
        }
        if (saved)
            hipLaunchKernelGGL(k_mlp_fwd<true>, dim3(div_up(N, BM)), dim3(NTHR), 0, stream, a);
        else
            hipLaunchKernelGGL(k_mlp_fwd<false>, dim3(div_up(N, BM)), dim3(NTHR), 0, stream, a);
    }
    DGS_LAUNCH_CHECK("k_mlp_fwd", false, stream);
    return DGS_OK;
}

int backward(int flags, int N, const float *packed, const float *saved, const float *dout, float *scratch,
             float *const *grads, hipStream_t stream) {
    if (N < 0 || (N > 0 && (!packed || !saved || !dout || !scratch || !grads))) {
        set_error("dgs_deform_backward: null argument");
        return DGS_ERR_ARGS;
    }
    Plan P = make_plan(flags);
    const Flags &F = P.F;
    if (N == 0) {
        for (int k = 0; k < P.nparams; k++) {
            int r, c;
            param_shape(F, P, k, r, c);
            DGS_HIP_CHECK(hipMemsetAsync(grads[k], 0, sizeof(float) * r * (c ? c : 1), stream));
        }
        return DGS_OK;
    }
    const size_t Ns = padded_points(N);
    float *dz = scratch;
    float *slabs = scratch + (size_t)F.nz * Ns;
    BwdArgs b{};
    b.N = N; b.Ns = Ns; b.packed = packed; b.saved = saved; b.dout = dout; b.dz = dz;
    b.mask = reinterpret_cast<const uint32_t *>(saved + (size_t)F.nsaved * Ns);
    b.tHd = P.tHd; b.tT2 = P.tT2;
    for (int i = 0; i < 8; i++) b.tL[i] = P.tL[i];
    b.flags = flags;
    {
        ScopedTimer tm("mlp_bwd", stream);
        hipLaunchKernelGGL(k_mlp_bwd, dim3(div_up(N, BM)), dim3(NTHR), 0, stream, b);
    }
    DGS_LAUNCH_CHECK("k_mlp_bwd", false, stream);
    return dw_fp32(F, Ns, dz, saved, slabs, grads, stream);
}

// dW on fp32-input MFMA (k_dw) + the fixed-order slab reduction; shared with the split-bf16 path,
// whose dZ / saved-activation arrays have the same [rows][Ns] layout (Ns a multiple of 32)
size_t dw_fp32_slab_floats(int flags) { return (size_t)fp32_wplan(make_flags(flags)).nblocks * SLAB; }

int dw_fp32(const Flags &F, size_t Ns, const float *dz, const float *saved, float *slabs, float *const *grads,
            hipStream_t stream) {
    WPlan W = fp32_wplan(F);
    {
        const size_t lds_bytes = sizeof(float) * 2 * 2 * WT * LDA;
        // 147 KiB dynamic LDS: the attribute is per device, set once per (kernel, device)
        if (int rc = ensure_dynamic_lds((const void *)k_dw, (int)lds_bytes)) return rc;
        ScopedTimer tm("mlp_dw", stream);
        hipLaunchKernelGGL(k_dw, dim3(W.nblocks), dim3(DW_THREADS), lds_bytes, stream, W.jobs, Ns, dz, saved, slabs);
    }
    DGS_LAUNCH_CHECK("k_dw", false, stream);
    return launch_dw_reduce(F, W, slabs, grads, stream);
}

}  // namespace mlp

namespace mlpc {
int launch_dw_reduce(const Flags &F, const WPlan &W, const float *slabs, float *const *grads, hipStream_t stream) {
    const Params P = make_params(F);
    mlp::RJobs R{};
    int total = 0;
    auto add = [&](int pidx, int rowpad0, int ns, const Seg *sg, int layer, bool bias) {
        int r, c;
        param_shape(F, P, pidx, r, c);
        mlp::RJob &J = R.j[R.n];
        J.dst = grads[pidx]; J.rows = r; J.cols = bias ? 0 : c; J.rowpad0 = rowpad0; J.nseg = ns;
        for (int q = 0; q < ns; q++) J.seg[q] = sg[q];
        for (int kt = 0; kt < 2; kt++) {
            int jq = W.layer_job[layer][kt];
            J.block0[kt] = jq >= 0 ? W.jobs.j[jq].block0 : 0;
            J.nsplit[kt] = jq >= 0 ? W.jobs.j[jq].nsplit : 0;
        }
        J.k1 = W.layer_k1[layer];
        R.begin[R.n] = total;
        total += bias ? r : r * c;
        R.n++;
    };
    for (int i = 0; i < 8; i++) {
        Seg sg[3];
        int ns = layer_in_segs(F, i, sg);
        add(P.pLw[i], 0, ns, sg, i, false);
        add(P.pLb[i], 0, ns, sg, i, true);
    }
    {
        Seg full = seg(0, 256, 0);
        int r0 = 0;
        for (int hh = 0; hh < P.nheads; hh++) {
            add(P.pHw[hh], r0, 1, &full, 8, false);
            add(P.pHb[hh], r0, 1, &full, 8, true);
            r0 += P.hrows[hh];
        }
        if (F.blender && !F.uniform_t) {  // uniform t: written by the split path's k_tgrad
            Seg st = seg(0, F.tin, 0);
            add(P.pT0w, 0, 1, &st, 9, false);
            add(P.pT0b, 0, 1, &st, 9, true);
            add(P.pT2w, 0, 1, &full, 10, false);
            add(P.pT2b, 0, 1, &full, 10, true);
        }
    }
    R.begin[R.n] = total;
    {
        ScopedTimer tm("mlp_dw_reduce", stream);
        hipLaunchKernelGGL(mlp::k_dw_reduce, dim3(div_up(total, 256)), dim3(256), 0, stream, R, slabs);
    }
    DGS_LAUNCH_CHECK("k_dw_reduce", false, stream);
    return DGS_OK;
}
}  // namespace mlpc
}  // namespace dgs

#ifdef DGS_MLP_PROFILE
extern "C" void dgs_mlp_set_prof(unsigned long long *p) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(dgs::mlp::dgs_mlp_prof), &p, sizeof(p));
}
#endif
