// Fused deformation MLP (positional encoding + timenet + 8x256 trunk with skip + heads) on f16 MFMA
// with a scaled two-piece operand split: the default path of dgs_deform_* (the fp32-MFMA kernels of
// mlp.hip run instead under DGS_MLP_EXACT_FP32).
//
// Replaces DeformNetworkBaseline.forward and its autograd backward (utils/time_utils.py:56-127;
// DeformNetwork :129-201 via DGS_MLP_NO_ROTSCALE; 6-DoF heads :114-121 emitted raw, exp_se3 stays in
// the host glue).
//
// Numerics ("f16x3", round 6; rounds 1-5 ran a three-piece bf16 split with six products per fp32
// product). Every fp32 operand x is multiplied by a power of two S (exact) that puts its group's
// magnitude bound into [2^14, 2^15), then split into two f16 values
//   hi = f16(S x), lo = f16(S x - hi)                           (round to nearest)
// (S x - hi is exact in fp32; |S x - hi| <= 2^-11 |hi|, so lo carries the next 11 bits: S x = hi + lo
// to 2^-22 relative; below the f16 normal range the pieces keep 2^-25 absolute, i.e. 2^-39 of the
// group's bound). A product a*b is accumulated as the three f16 x f16 products hh + hl + lh, each
// exact in the fp32 accumulator of the MFMA (hl, lh <= 2^-11 |hh|; the dropped ll <= 2^-22 |ab|),
// hh in the running accumulator and hl + lh in their own (an MFMA aligns its terms and C to the
// largest within a limited window, tools/mfma_round_probe.hip), added once per GEMM. The scales are
// undone in fp32 (powers of two: exact) in the epilogue. F16 MFMA forms run at the bf16 rate
// (MI355X_MICROARCH: 'the F16 forms take the same cycles'), so the GEMMs issue half the MFMAs of the
// bf16x6 split (16/3 = 5.3x the fp32-MFMA rate), read two operand planes instead of three, and split
// in 5 VALU per two values instead of 11. Accuracy: tests/test_gpu_mlp.py holds every output and
// parameter gradient to 2x the exact-fp32 path's error against float64, including the bench step's
// own near-cancelling upstream gradient at 100k points (test_split_accuracy_bench_regime).
//   Scales. A (weights): one per (image, 16-row n-tile) over the whole K, from the tile's max |w|
// (k_pack, written into every k-slot of the tile). B (activations / dZ in LDS): one per layer, the
// same on every wave without any synchronisation: the writers of layer L's output all evaluate the
// bound  max_rows sum_k |W_L[row, k]| * max|input of L| + max|b_L|  (>= every output; the row abs
// sums are per-image statistics k_pack computes, the input maximum is the maximum of the ACTUAL
// maxima the previous layer's writers published in LDS before their hand-off signal, so the bound is
// loose by ~sqrt(K) at most, never compounding over layers). Inputs staged from memory (x_emb, t
// encodings, dOut) and the narrow per-point timenet outputs take their block's actual maximum behind
// the workgroup barrier their staging already has. A GEMM whose K spans two scale groups (x_emb |
// h of linear.5, x_emb | t_emb of linear.0) rescales its accumulators once at the boundary.
//
// Layout ("transposed" formulation, Y^T = W X^T: features on MFMA rows, points on MFMA columns),
// v_mfma_f32_16x16x32_f16:
//  * One workgroup = 64 points x 16 waves (4 per SIMD); wave r owns output rows 16r..16r+15 of every
//    256-wide layer for all four 16-point column tiles, so each 2 KiB weight fragment (16 rows x 32
//    features x 2 splits) fetched from L2 feeds 4 x 3 MFMAs. The training forward / dX chain run as
//    8 waves of two n-tiles (k_fwd8 / k_bwd8).
//  * Activations live in LDS split into hi/lo f16 images of 16-byte units (8 features x 1 point),
//    [8-feature group][split][64 points]: the B operand of a k-step (32 features) is one ds_read_b128
//    per split and column tile, and an accumulator's 4 rows are one 8-byte store per split into the
//    next layer's image. XE | TE | H groups are contiguous, so cat(x_emb, t_emb) and cat(x_emb, t_emb,
//    h) are plain group ranges.
//  * Narrow layers (timenet.2, heads, the t_emb rows of the backward) run as full-K 16x16 tiles on a
//    subset of the waves: no partial sums.
//  * Weights are packed every call (they change every optimizer step) by one gather + scale + split
//    launch into A-fragment images [n-tile][k-step][split][64 lanes][8 f16] (k-slot stride 3 KiB: hi,
//    lo, and the tile's inverse scale).
//  * Saved activations / dZ stay fp32 feature-major [rows][Ns] (mlp_shared.h row map; the dW GEMM
//    reads them), written in each layer's epilogue; relu' masks are one u16 per lane and 16-row
//    tile ([64-point block][row / 16][64 lanes]). Every reduction has a fixed order: bitwise
//    deterministic.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cassert>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

#include "dgs_common.h"
#include "mlp_shared.h"

namespace dgs {
namespace mlps {

using namespace mlpc;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));

constexpr int BM = 64;            // points per workgroup
constexpr int NQ = 4;             // 16-point column tiles per workgroup
constexpr int NWAVE = 16;         // one 16-row n-tile of a 256-wide layer per wave
constexpr int NTHR = NWAVE * 64;
constexpr int NSPLIT = 2;         // hi, lo
constexpr int PACK_MAXK = 11;     // k-slots of the widest A-image n-tile (linear.5's forward image: 352 / 32)
constexpr int UG = NSPLIT * BM;   // 16-B units per 8-feature group (all splits, all points)
constexpr int KSLOT = 3 * 64;     // units per (n-tile, k-step) of an A image: hi, lo, inverse scale
constexpr int KG = 4;             // 8-feature groups per k-step (32 features)
// forward LDS groups: XE (64 features) | TE (32) | H (256) | TIN (16 + 16 zero: one k-step)
constexpr int G_XE = 0, G_TE = 8, G_H = 12, G_TIN = 44, G_FWD = 48;
// backward LDS groups: H (dZ, 256) | G (dOut / dTE, 32)
constexpr int G_BH = 0, G_BG = 32, G_BWD = 36;
// fp32 staging rows (inside the H region): XE 0..63 | TE 64..95 | TIN 96..111
constexpr int ST_TE = 64, ST_TIN = 96;
// relu' masks per 64-point block (2 * nmask u32 words): the trunk's as [layer pair][row / 16][64 lanes]
// u32 (layer 2l in the low, 2l + 1 in the high 16 bits: one dword store per two layers), then the
// timenet TH tiles as [row / 16][64 lanes] u16 at tile MR_TH
constexpr int MR_TH = M_TH / 16;

static_assert(G_TE == G_XE + 8 && G_H == G_TE + 4, "XE|TE|H must be contiguous");
static_assert(G_FWD * UG * 16 + (8 * 256 + 16) * 4 + NTHR * 4 + 512 <= 160 * 1024 && G_BWD * UG * 16 <= 160 * 1024,
              "LDS (k_fwd: + trunk biases, pending relu' bits, hand-off counters, scales)");
static_assert(112 * BM * 4 <= 32 * UG * 16, "fp32 staging must fit the H region");

// ------------------------------------------------------------------------------------------------
// scaled two-piece f16 split
// ------------------------------------------------------------------------------------------------
// 2^e as a float (e in [-126, 127])
__device__ __forceinline__ float pow2f(int e) { return __uint_as_float((uint32_t)(e + 127) << 23); }
// the power-of-two scale S that brings a bound m >= max |x| into [2^14, 2^15), and 1 / S; exponents
// clamped to +-60 (a zero or tiny bound keeps S = 2^74, an infinite one 2^-46)
struct Scale {
    float s, inv;
};
__device__ __forceinline__ Scale scale_for(float m) {
    int e = (int)((__float_as_uint(m) >> 23) & 255u) - 127;
    e = min(max(e, -60), 60);
    return Scale{pow2f(14 - e), pow2f(e - 14)};
}

// hi = f16(a), lo = f16(a - hi) of two (already scaled) values, pairwise: v_cvt_pk_f16_f32, two
// f16 -> f32, a packed subtraction, v_cvt_pk_f16_f32 (5 VALU per two values)
__device__ __forceinline__ void hsplit2(float a, float b, uint32_t &h, uint32_t &l) {
    const h16x2 hv = __builtin_convertvector((f32x2){a, b}, h16x2);
    const f32x2 hf = __builtin_convertvector(hv, f32x2);
    const h16x2 lv = __builtin_convertvector((f32x2){a - hf[0], b - hf[1]}, h16x2);
    h = __builtin_bit_cast(uint32_t, hv);
    l = __builtin_bit_cast(uint32_t, lv);
}

struct Split4 {
    h16x4 h, l;
};

// four values times the scale S -> their hi / lo halves of a unit
__device__ inline Split4 split4(float a, float b, float c, float d, float S) {
    uint32_t h0, l0, h1, l1;
    hsplit2(a * S, b * S, h0, l0);
    hsplit2(c * S, d * S, h1, l1);
    return Split4{__builtin_bit_cast(h16x4, make_uint2(h0, h1)), __builtin_bit_cast(h16x4, make_uint2(l0, l1))};
}

// 8 consecutive features of one point -> the two 16-B units of group g (LDS image [g][split][BM])
__device__ inline void put_unit8(h16x8 *lds, int g, int m, const float (&v)[8], float S) {
    const Split4 a = split4(v[0], v[1], v[2], v[3], S);
    const Split4 b = split4(v[4], v[5], v[6], v[7], S);
    h16x8 *u = lds + g * UG + m;
    u[0] = __builtin_shufflevector(a.h, b.h, 0, 1, 2, 3, 4, 5, 6, 7);
    u[BM] = __builtin_shufflevector(a.l, b.l, 0, 1, 2, 3, 4, 5, 6, 7);
}

// max over the wave of non-negative floats (as u32: the same order), in every lane: DPP row shifts,
// the row broadcasts into lane 63, then readlane
__device__ __forceinline__ float wave_max(float v) {
    uint32_t x = __float_as_uint(v);
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
    return __uint_as_float(__builtin_amdgcn_readlane(x, 63));
}

// max |v| over this lane's tiles
template <int NQ_>
__device__ inline float tiles_absmax(const f32x4 (&v)[NQ_]) {
    float m = 0.f;
#pragma unroll
    for (int q = 0; q < NQ_; q++)
#pragma unroll
        for (int i = 0; i < 4; i++) m = fmaxf(m, fabsf(v[q][i]));
    return m;
}

// LDS max of non-negative floats (ds_max_u32 on the bits)
__device__ __forceinline__ void lds_fmax(uint32_t *p, float v) {
    __hip_atomic_fetch_max(p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Per-block scale state in LDS. Every B-operand scale is per 16-point column tile q (the MFMA's column
// block), so a point's arithmetic does not depend on which other points share its workgroup (the tail
// decomposition, block_split, stays bitwise equal to 64-point blocks):
//  ksc[k][q]: inverse scale of k-step k of the LDS image, column tile q (every writer of a k-step stores
//             the same value)
//  amax[par][w][q]: actual max |output| of writer wave w in the layer (chain step) of parity par
//  ain[i][q]: maxima of the staged inputs: [0] x_emb (forward) / dOut (backward), [1] t_emb
//  bsync[i][q]: block-wide maxima gathered behind a workgroup barrier (staging, narrow timenet tiles)
//  bmax[L]: max |bias| of trunk layer L (8: heads), from the launch-constant bias table
//  wstat[L]: max row abs sum of the layer's A image (k_pack's tile statistics; [8]: heads^T)
struct alignas(16) ScaleLDS {
    float ksc[12][4];
    float amax[2][16][4];
    float ain[2][4];
    uint32_t bsync[8][4];
    uint32_t bmax[10];
    uint32_t wstat[10];
};
// block-sync slots
constexpr int BS_XE = 0, BS_TE = 1, BS_TIN = 2, BS_TH = 3, BS_TET = 4, BS_G = 5, BS_GTE = 6;

// max over the nw writer waves of their published maxima, all four column tiles (one 16-B read per wave)
__device__ inline float4 amax_of4(const ScaleLDS *sc, int par, int nw) {
    float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int w = 0; w < nw; w++) {
        const float4 v = *reinterpret_cast<const float4 *>(sc->amax[par][w]);
        m = make_float4(fmaxf(m.x, v.x), fmaxf(m.y, v.y), fmaxf(m.z, v.z), fmaxf(m.w, v.w));
    }
    return m;
}
__device__ __forceinline__ float f4get(const float4 &v, int q) { return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w; }

// ------------------------------------------------------------------------------------------------
// GEMM pieces. 16x16x32 lane maps (cdna_hip_programming.md §3): lane l (kq = l >> 4, col = l & 15)
// holds A[row col][k = 8 kq + j] and B[k = 8 kq + j][col col]; C/D element i is row 4 kq + i, col col.
// ------------------------------------------------------------------------------------------------
#define MF16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_f16((a), (b), (c), 0, 0, 0)

struct AFrag {  // one operand fragment in its two split parts
    h16x8 h, l;
};

__device__ inline AFrag load_a(const h16x8 *p) { return AFrag{p[0], p[64]}; }

// B fragment of column tile q from the LDS image (p: this lane's unit of split 0, column tile 0)
__device__ inline AFrag load_b(const h16x8 *p, int q) { return AFrag{p[16 * q], p[BM + 16 * q]}; }

__device__ inline f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// The three split products of one k-step: hh into the running accumulator, the two corrections
// (|.| <= 2^-11 |hh|) into their own accumulator, added in fp32 once per GEMM
__device__ inline void mma3(const AFrag &a, const AFrag &b, f32x4 &acc, f32x4 &lo) {
    lo = MF16(a.l, b.h, lo);
    lo = MF16(a.h, b.l, lo);
    acc = MF16(a.h, b.h, acc);
}

// inverse scale of an A image's n-tile: the float after its first k-slot's two planes
__device__ __forceinline__ float a_inv(const h16x8 *tile_slot0) {
    return reinterpret_cast<const float *>(tile_slot0 + 128)[0];
}

#ifdef DGS_MLP_PROFILE  // diagnostic build only (tools/mlp_phase.py): per-phase s_memtime stamps
__device__ unsigned long long *dgs_mlps_prof;
// only the workgroup's first block (launched while every CU is busy) is stamped: p0 == blockIdx.x * BM
#define DGS_STAMP(k)                                                                                   \
    do {                                                                                               \
        if (threadIdx.x == 0 && p0 == (int)blockIdx.x * BM)                                            \
            dgs_mlps_prof[blockIdx.x * 64 + (k)] = __builtin_amdgcn_s_memtime();                       \
    } while (0)
#define DGS_WSTAMP(k, L)                                                                               \
    do {                                                                                               \
        if (L == 3 && (threadIdx.x & 63) == 0 && p0 == (int)blockIdx.x * BM)                           \
            dgs_mlps_prof[blockIdx.x * 64 + (k) + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime();  \
    } while (0)
// k_fwd8 (8 waves): layer DGS_PROF_LAYER of the workgroup's first block, stamp k + wave
#ifndef DGS_PROF_LAYER
#define DGS_PROF_LAYER 3
#endif
#define DGS_WSTAMP8(k, L)                                                                              \
    do {                                                                                               \
        if (L == DGS_PROF_LAYER && (threadIdx.x & 63) == 0 && p0 == (int)blockIdx.x * BM)              \
            dgs_mlps_prof[blockIdx.x * 64 + (k) + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime();  \
    } while (0)
#else
#define DGS_WSTAMP8(k, L) \
    do {                  \
    } while (0)
#define DGS_WSTAMP(k, L) \
    do {                 \
    } while (0)
#define DGS_STAMP(k) \
    do {             \
    } while (0)
#endif

struct NoPre {
    __device__ void operator()() const {}
};

// LDS hand-off between the waves of a workgroup without a workgroup barrier: monotonically growing
// per-k-step counters, a relaxed LDS load spun on (wave-uniform), a relaxed LDS add from one lane.
// A wave executes its LDS operations in issue order, so data written before a signal is visible to
// a wave that has seen the signal; the empty asm keeps the compiler from moving LDS accesses across.
// The spin is bounded so a wrong count can never hang the GPU; an expired bound is not silent: it
// counts into dgs_mlps_guard_expired (a global atomic from one lane), which the host reads with
// dgs_debug_guard_expiries() and every GPU test checks to be 0 (outputs after an expiry are invalid).
__device__ uint32_t dgs_mlps_guard_expired;

#ifdef DGS_CLOCK_STAMPS
// Diagnostic build only (tools/mlp_clock.py): per-workgroup in-kernel clock of k_fwd / k_bwd / k_dws
// (MI355X_MICROARCH 'DVFS give-back' item 6): shader-clock and 100 MHz real-time stamps of wave 0 at
// block start and end, into a buffer no kernel reads. The product build has no stamps.
constexpr int CLK_BLOCKS = 2048;
__device__ unsigned long long dgs_clk[3][CLK_BLOCKS][6];
struct ClkStamp {
    unsigned long long t, r;
    __device__ ClkStamp() : t(__builtin_amdgcn_s_memtime()), r(__builtin_amdgcn_s_memrealtime()) {}
    __device__ void end(int k) const {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0 && blockIdx.x < CLK_BLOCKS) {
            unsigned long long *p = dgs_clk[k][blockIdx.x];
            p[0] = t; p[1] = t1; p[2] = r; p[3] = r1;
            // HW_ID (CU / SH / SE fields) and XCC_ID: which CU ran the workgroup
            p[4] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                   ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
        }
    }
};
#define CLK_BEGIN() const ClkStamp clk_
#define CLK_END(k) clk_.end(k)
#else
#define CLK_BEGIN()
#define CLK_END(k)
#endif
#ifndef DGS_SPIN_SLEEP
#define DGS_SPIN_SLEEP 1  // s_sleep units (64 clocks) between polls of a hand-off counter
#endif
__device__ __forceinline__ uint32_t lds_peek(const uint32_t *f) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The first test of `seen` (peeked earlier, usually already satisfied) sits outside the spin loop:
// as the loop's header it merged with the loop's own fresh peek, so the compiler waited for EVERY
// outstanding LDS read there (lgkmcnt(0)) — the next tile's just-issued B fragment reads included —
// once per k-step of every GEMM; outside it, the wait covers the peek only.
__device__ __forceinline__ void lds_wait_ge(const uint32_t *f, uint32_t target, uint32_t seen) {
    if (__builtin_amdgcn_readfirstlane(seen) < target) {
        int guard = 0;
#pragma clang loop unroll(disable)
        do {
            __builtin_amdgcn_s_sleep(DGS_SPIN_SLEEP);
            seen = lds_peek(f);
        } while (__builtin_amdgcn_readfirstlane(seen) < target && ++guard < (1 << 20));
        if (guard == (1 << 20) && (threadIdx.x & 63) == 0)
            __hip_atomic_fetch_add(&dgs_mlps_guard_expired, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void lds_signal(uint32_t *f, int lane) {
    asm volatile("" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct NoGate {
    __device__ uint32_t peek(int) const { return 0; }
    __device__ void need(int, uint32_t) const {}
    __device__ void done(int) const {}
};

// Trunk gate: the H k-steps (GEMM k-steps k0..) may be read once both writer waves of the previous
// layer have signalled wr[j] (wr[j] >= wt), and each wave signals rd[j] once its reads of H k-step
// j are consumed (the next layer's writers wait for all 16)
struct HGate {
    uint32_t *wr, *rd;
    int k0;
    uint32_t wt;
    bool sig;
    int lane;
    __device__ uint32_t peek(int k) const { return k < k0 ? 0xffffffffu : lds_peek(wr + (k - k0)); }
    __device__ void need(int k, uint32_t seen) const {
        if (k >= k0) lds_wait_ge(wr + (k - k0), wt, seen);
    }
    __device__ void done(int k) const {
        if (sig && k >= k0) lds_signal(rd + (k - k0), lane);
    }
};

// acc[q] += A . X for the column tiles q0 .. q0 + NQ_ - 1 over NK k-steps of this wave's A image
// (Aw: unit pointer of its n-tile at k-step 0) and of the LDS image from group g0 (k-step c =
// groups g0 + 4c + kq). Fully unrolled; per k-step: each column tile's three MFMAs followed by its B
// fragment for the next k-step into the same registers, then the A fragment RING k-steps ahead
// (register ring: the A stream comes from L2). sched_barrier keeps that order per k-step; the other
// waves of the SIMD cover the B reload latency. pre() runs after the A prologue. SKIP: k-steps
// >= SKIP read the LDS image one k-step further on (linear.5 with t_emb folded: x_emb | h, past t_emb).
// Scales: ksc[g / 4][q] is the inverse scale of the image k-step at group g, column tile q (read once
// its writers have signalled). BND: bit k set = k-step k starts a new scale group (x_emb | t_emb | h);
// there the accumulators are brought to the new group's scale (one multiply by a power of two). ib[q]:
// the inverse scale of the last group: the result is acc[q] * (A's inverse scale) * ib[q].
template <int NK, int NQ_, class Pre = NoPre, class Gate = NoGate, int SKIP = (1 << 20), unsigned BND = 0u>
__device__ inline void gemm(const h16x8 *__restrict__ Aw, const h16x8 *lds, int g0, int q0, int lane,
                            f32x4 (&acc)[NQ_], float (&ib)[NQ_], const float (*ksc)[4], Pre pre = Pre(),
                            Gate gate = Gate()) {
    static_assert(NK >= 1, "empty GEMM");
    const int kq = lane >> 4, col = lane & 15;
    const h16x8 *Ap = Aw + lane;
    const int bunit = (g0 + kq) * UG + 16 * q0 + col;  // this lane's B unit at k-step 0
    constexpr int AK = KSLOT;
    constexpr int BK = KG * UG;
    auto bofs = [](int k) { return (k + (k >= SKIP ? 1 : 0)) * BK; };  // compile-time per unrolled k
    auto kidx = [&](int k) { return (g0 >> 2) + k + (k >= SKIP ? 1 : 0); };
    // the B fragments of k-step k from a base formed once per k-step (the unit index is opaque to the
    // compiler): the image spans > 64 KB, so a single base would need one address add per ds_read
    // (a DS immediate offset is 16 bits); from the k-step base every fragment is an immediate offset
    auto kbase = [&](int k) {
        int u = bunit + bofs(k);
        asm volatile("" : "+v"(u));
        return lds + u;
    };
    constexpr int RING = 2;
    AFrag ring[RING];
#pragma unroll
    for (int k = 0; k < RING; k++)
        if (k < NK) ring[k] = load_a(Ap + k * AK);
    pre();
    gate.need(0, gate.peek(0));
    float cur[NQ_], nxt[NQ_];
#pragma unroll
    for (int q = 0; q < NQ_; q++) nxt[q] = cur[q] = ksc[kidx(0)][q0 + q];
    const h16x8 *Bk = kbase(0);
    AFrag b = load_b(Bk, 0);
    f32x4 lo[NQ_];
#pragma unroll
    for (int q = 0; q < NQ_; q++) lo[q] = zero4();
#pragma unroll
    for (int k = 0; k < NK; k++) {
        __builtin_amdgcn_sched_barrier(0);
        if (k > 0) gate.done(k - 1);  // k-step k-1's B fragments were consumed by its MFMAs
        if (k > 0 && k < 32 && ((BND >> k) & 1u)) {  // a new scale group starts here
#pragma unroll
            for (int q = 0; q < NQ_; q++) {
                acc[q] = (acc[q] + lo[q]) * (cur[q] / nxt[q]);
                lo[q] = zero4();
                cur[q] = nxt[q];
            }
        }
        const uint32_t seen = k + 1 < NK ? gate.peek(k + 1) : 0u;
#pragma unroll
        for (int q = 0; q < NQ_; q++) {
            // the next tile's B fragment (or the next k-step's first) is in flight during this tile's MFMAs
            AFrag nb;
            if (q + 1 < NQ_) nb = load_b(Bk, q + 1);
            else if (k + 1 < NK) {
                gate.need(k + 1, seen);
                if (k + 1 < 32 && ((BND >> (k + 1)) & 1u))
#pragma unroll
                    for (int q2 = 0; q2 < NQ_; q2++) nxt[q2] = ksc[kidx(k + 1)][q0 + q2];
                Bk = kbase(k + 1);
                nb = load_b(Bk, 0);
            }
            // the reads stay ahead of ALL the MFMAs of this tile: without this barrier the scheduler,
            // short of registers, sank them below the tile's first MFMAs (reusing the current
            // fragment's registers), so the next tile's first MFMAs waited on them (k_fwd -1.4 %,
            // profiles/r5f_mlp_bread_pin_ab.txt)
            __builtin_amdgcn_sched_barrier(0);
            mma3(ring[k % RING], b, acc[q], lo[q]);
            if (q + 1 < NQ_ || k + 1 < NK) b = nb;
            // pin the order per column tile: the next fragment's reads stay ahead of this tile's
            // MFMAs (left to itself the scheduler pulls each read down to its first use and waits on
            // it: lgkmcnt(0) in front of most MFMAs)
            __builtin_amdgcn_sched_barrier(0);
        }
        if (k + RING < NK) ring[k % RING] = load_a(Ap + (k + RING) * AK);
        __builtin_amdgcn_sched_barrier(0);
    }
    gate.done(NK - 1);
#pragma unroll
    for (int q = 0; q < NQ_; q++) {
        acc[q] += lo[q];
        ib[q] = cur[q];
    }
}

// gemm() for TWO n-tiles per wave (the 8-wave k_fwd8 / k_bwd8): n-tile t's A image at Aw + t * astride
// units; every B fragment read from LDS feeds both n-tiles' MFMAs, so the activation image is read by 8
// waves per layer instead of 16. Each (n-tile, column tile) accumulator sees the same MFMA sequence as
// in gemm().
template <int NK, int NQ_, class Pre = NoPre, class Gate = NoGate, int SKIP = (1 << 20), unsigned BND = 0u>
__device__ inline void gemm2(const h16x8 *__restrict__ Aw, int astride, const h16x8 *lds, int g0, int q0, int lane,
                             f32x4 (&acc)[2][NQ_], float (&ib)[NQ_], const float (*ksc)[4], Pre pre = Pre(),
                             Gate gate = Gate()) {
    static_assert(NK >= 1, "empty GEMM");
    const int kq = lane >> 4, col = lane & 15;
    const h16x8 *Ap0 = Aw + lane, *Ap1 = Aw + astride + lane;
    const int bunit = (g0 + kq) * UG + 16 * q0 + col;
    constexpr int AK = KSLOT;
    constexpr int BK = KG * UG;
    auto bofs = [](int k) { return (k + (k >= SKIP ? 1 : 0)) * BK; };
    auto kidx = [&](int k) { return (g0 >> 2) + k + (k >= SKIP ? 1 : 0); };
    auto kbase = [&](int k) {
        int u = bunit + bofs(k);
        asm volatile("" : "+v"(u));
        return lds + u;
    };
    constexpr int RING = 2;
    AFrag ring[RING][2];
#pragma unroll
    for (int k = 0; k < RING; k++)
        if (k < NK) {
            ring[k][0] = load_a(Ap0 + k * AK);
            ring[k][1] = load_a(Ap1 + k * AK);
        }
    pre();
    gate.need(0, gate.peek(0));
    float cur[NQ_], nxt[NQ_];
#pragma unroll
    for (int q = 0; q < NQ_; q++) nxt[q] = cur[q] = ksc[kidx(0)][q0 + q];
    const h16x8 *Bk = kbase(0);
    AFrag b = load_b(Bk, 0);
    f32x4 lo[2][NQ_];
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
        for (int q = 0; q < NQ_; q++) lo[t][q] = zero4();
#pragma unroll
    for (int k = 0; k < NK; k++) {
        __builtin_amdgcn_sched_barrier(0);
        if (k > 0) gate.done(k - 1);
        if (k > 0 && k < 32 && ((BND >> k) & 1u)) {
#pragma unroll
            for (int q = 0; q < NQ_; q++) {
                const float r = cur[q] / nxt[q];
#pragma unroll
                for (int t = 0; t < 2; t++) {
                    acc[t][q] = (acc[t][q] + lo[t][q]) * r;
                    lo[t][q] = zero4();
                }
                cur[q] = nxt[q];
            }
        }
        const uint32_t seen = k + 1 < NK ? gate.peek(k + 1) : 0u;
#pragma unroll
        for (int q = 0; q < NQ_; q++) {
            AFrag nb;
            if (q + 1 < NQ_) nb = load_b(Bk, q + 1);
            else if (k + 1 < NK) {
                gate.need(k + 1, seen);
                if (k + 1 < 32 && ((BND >> (k + 1)) & 1u))
#pragma unroll
                    for (int q2 = 0; q2 < NQ_; q2++) nxt[q2] = ksc[kidx(k + 1)][q0 + q2];
                Bk = kbase(k + 1);
                nb = load_b(Bk, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            mma3(ring[k % RING][0], b, acc[0][q], lo[0][q]);
            mma3(ring[k % RING][1], b, acc[1][q], lo[1][q]);
            if (q + 1 < NQ_ || k + 1 < NK) b = nb;
            __builtin_amdgcn_sched_barrier(0);
        }
        if (k + RING < NK) {
            ring[k % RING][0] = load_a(Ap0 + (k + RING) * AK);
            ring[k % RING][1] = load_a(Ap1 + (k + RING) * AK);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    gate.done(NK - 1);
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
        for (int q = 0; q < NQ_; q++) acc[t][q] += lo[t][q];
#pragma unroll
    for (int q = 0; q < NQ_; q++) ib[q] = cur[q];
}

// accumulator tile q (rows 16r + 4kq + i of this wave, point 16q + col) -> its 8-byte half of the
// split units of group 2r + (kq >> 1) (LDS image from group gbase)
// (times the layer's scale S)
__device__ inline void acc_to_lds(const f32x4 &v, h16x8 *lds, int gbase, int r, int q, int lane, float S) {
    const int kq = lane >> 4, col = lane & 15;
    const Split4 s = split4(v[0], v[1], v[2], v[3], S);
    h16x4 *u = reinterpret_cast<h16x4 *>(lds + (gbase + 2 * r + (kq >> 1)) * UG + 16 * q + col) + (kq & 1);
    u[0] = s.h;
    u[2 * BM] = s.l;  // h16x4 units: one 16-B unit = 2 of them
}

// A wave's 16-row x 64-point tile of a feature-major [rows][Ns] array through a buffer descriptor
// whose base is the tile origin (wave-uniform: SGPRs): store (i, q) writes rows 4kq + i of column
// tile q, one buffer instruction each with the row offset in an SGPR.
struct Tile16 {
    __amdgpu_buffer_rsrc_t rsrc;  // base = &dst[row0 * Ns + p0]
    int voff;                     // (4kq * Ns + col) * 4 bytes
    int ns4;                      // Ns * 4 bytes
// Cache policy of these stores (the saved activations / dZ: ~0.95 GB per launch, read back only by
// the dW kernel after the whole launch): nt. A/B r5m against plain stores: k_fwd -1.7 %, k_bwd -3 %,
// k_dws (their reader) -4..-6 %, step +2.5 %; sc1 (write-through, line dropped from L2) was 3-7 %
// slower. (Without any of these stores k_fwd / k_bwd ran 7 / 15 % faster, r5j; 16-byte stores after a
// quad transpose were 5-6 % slower, r5k; the next layer's first A fragment issued ahead of the stores
// changed nothing, r5l.)
#ifndef DGS_TILE_STORE_AUX
#define DGS_TILE_STORE_AUX 2
#endif
    __device__ void st(int i, int q, float v) const {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc, voff + 64 * q, i * ns4, DGS_TILE_STORE_AUX);
    }
    template <int NQ_>
    __device__ void store(const f32x4 (&v)[NQ_], int q0 = 0) const {
#pragma unroll
        for (int q = 0; q < NQ_; q++)
#pragma unroll
            for (int i = 0; i < 4; i++) st(i, q0 + q, v[q][i]);
    }
};

__device__ inline Tile16 tile16(const float *dst, size_t Ns, int row0, int p0, int lane) {
    const float *base = dst + (size_t)row0 * Ns + p0;
    return Tile16{__builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), 0, 0x7fffffff, 0x00020000),
                  (4 * (lane >> 4) * (int)Ns + (lane & 15)) * 4, (int)Ns * 4};
}

// relu' bits of a wave's 16 x 64 tile: bit 4q + i of lane (kq, col) = [row 4kq + i of point 16q + col
// > 0] (signed clamp of the float bits: -0.0 and +0.0 give 0); the backward's tiles have the same map
template <int NQ_>
__device__ inline uint32_t relu_bits(const f32x4 (&v)[NQ_]) {
    uint32_t w = 0;
#pragma unroll
    for (int q = 0; q < NQ_; q++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            // v_med3_i32 + v_lshl_or_b32: 2 VALU per value (the compiler's own v_cmp + v_cndmask +
            // v_lshl + v_or3 take ~2.4)
            uint32_t m;
            asm("v_med3_i32 %0, %1, 0, 1" : "=v"(m) : "v"(__float_as_int(v[q][i])));
            if (q == 0 && i == 0) w = m;
            else asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(w) : "v"(m), "i"(4 * q + i), "v"(w));
        }
    return w;
}

template <int NQ_>
__device__ inline void mask_apply(f32x4 (&v)[NQ_], uint32_t bits) {
#pragma unroll
    for (int q = 0; q < NQ_; q++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            // v_bfe_i32 + v_and (2 VALU): left to itself the compiler turns the sign-extended bit into
            // v_and + v_cmp + v_cndmask (3 VALU per value)
            int m;
            asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(bits), "i"(4 * q + i));
            v[q][i] = __int_as_float(__float_as_int(v[q][i]) & m);
        }
}

// this lane's 4 rows (16r + 4kq .. +3) of a padded bias vector
__device__ inline float4 load_bias4(const float *bias, int r, int lane) {
    return *reinterpret_cast<const float4 *>(bias + 16 * r + 4 * (lane >> 4));
}

// v[q] * (ia * ib[q]) + b (ia: A's inverse scale, ib: the GEMM's B scales per column tile), then ReLU
template <int NQ_>
__device__ inline void bias_relu(f32x4 (&v)[NQ_], float ia, const float (&ib)[NQ_], float4 b, bool relu) {
#pragma unroll
    for (int q = 0; q < NQ_; q++) {
        v[q] = v[q] * (ia * ib[q]) + f32x4{b.x, b.y, b.z, b.w};
        if (relu)
#pragma unroll
            for (int i = 0; i < 4; i++) v[q][i] = fmaxf(v[q][i], 0.f);
    }
}

template <int NQ_>
__device__ inline void scale_tiles(f32x4 (&v)[NQ_], float ia, const float (&ib)[NQ_]) {
#pragma unroll
    for (int q = 0; q < NQ_; q++) v[q] *= ia * ib[q];
}

template <int NQ_>
__device__ inline void zero_tiles(f32x4 (&v)[NQ_]) {
#pragma unroll
    for (int q = 0; q < NQ_; q++) v[q] = zero4();
}

// ------------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------------
// Persistent launches (round 3): one workgroup per CU runs block after block, taking the next block
// index from a device counter, so faster XCDs take more blocks. The eight XCDs hold different clocks
// under this load (1.80-2.04 GHz measured, tools/mlp_clock.py) and the hardware hands workgroups to
// XCDs round-robin, so with one launch block per block the slowest XCD set the kernel time. Block b
// computes exactly what it computed before (same points, same mask slot): outputs are bitwise
// unchanged. The index of the next block is fetched at the start of the current one (latency hidden
// by the block); the last workgroup to finish zeroes the counter pair for the next launch.
__device__ __forceinline__ int queue_take(uint32_t *q) { return (int)gridDim.x + (int)atomicAdd(q, 1u); }
__device__ __forceinline__ void queue_release(uint32_t *q) {
    // every workgroup's final take has returned before its increment of q[1]
    if (threadIdx.x == 0 && atomicAdd(q + 1, 1u) == gridDim.x - 1) {
        atomicExch(q, 0u);
        atomicExch(q + 1, 0u);
    }
}

struct FwdArgs {
    int N;
    size_t Ns;
    const float *xyz, *t;
    const h16x8 *img;  // A images
    const float *fp;    // fp32 region: biases, timenet weights
    float *out;
    float *saved;
    uint32_t *mask;     // relu' bits, [64-point block][row / 16][64 lanes] u16 (after the saved rows)
    float *tc;          // timenet of t[0] (k_timenet), or nullptr
    int nfull;          // 64-point blocks; the rest of [0, Ns) runs in 16-point blocks (block_split)
    int fT1, fT2, fL[8], fHd;      // image k-slots
    int bT1, bT2, bL[8], bHd;      // fp32 offsets
    int wT1, wT2;                  // fp32 timenet weights [256][16], [32][256]
    int w0te, w5te;                // fp32 t_emb columns of linear.0 / linear.5 [256][32] (C0 / C5)
    int flags;
    uint32_t *queue;  // block queue (persistent launch, BlockQueue) or nullptr: one launch block per block
    int nblk;         // blocks (64-point + 16-point)
};

// k_pack's statistic of an image n-tile: max over its 16 rows of sum_k |A[row][k]| (the float after the
// tile's inverse scale)
__device__ __forceinline__ float tile_stat(const h16x8 *tile_slot0) {
    return reinterpret_cast<const float *>(tile_slot0 + 128)[1];
}

// The reference feeds every Gaussian the same frame time (train_baseline.py:107-110), so the
// timenet (time_utils.py:74-76, 13 -> 256 -> 30) has one value per launch: evaluated here once in
// fp32 (one workgroup); a k_fwd block whose points all carry that t broadcasts TE / TH.
// fpv(off): the value at offset `off` of the packed fp32 region k_pack wrote
template <class FPV>
__device__ __forceinline__ void timenet_body(const FwdArgs &a, FPV fpv) {
    __shared__ float tin[16], th[256], te[32];
    const int j = threadIdx.x;
    const float t0 = a.t[0];
    if (j < 16) {
        float v = 0.f;
        if (j == 0) {
            v = t0;
        } else if (j < 13) {  // blender: t, sin / cos of 2^i t, i < 6
            float sv, cv;
            sincosf(t0 * (float)(1 << ((j - 1) >> 1)), &sv, &cv);
            v = (j & 1) ? sv : cv;
        }
        tin[j] = v;
        a.tc[TC_TIN + j] = v;
    }
    if (j == 0) a.tc[TC_T] = t0;
    __syncthreads();
    {
        const int w = a.wT1 + j * 16;
        float acc = fpv(a.bT1 + j);
#pragma unroll
        for (int f = 0; f < 16; f++) acc = fmaf(fpv(w + f), tin[f], acc);
        acc = fmaxf(acc, 0.f);
        th[j] = acc;
        a.tc[TC_TH + j] = acc;
    }
    __syncthreads();
    {  // TE[k], k < 32 (rows 30, 31 are zero padding): 8 lanes per output, 32 features each
        const int k = j >> 3, q = j & 7;
        const int w = a.wT2 + k * 256 + 32 * q;
        float acc = 0.f;
#pragma unroll
        for (int f = 0; f < 32; f++) acc = fmaf(fpv(w + f), th[32 * q + f], acc);
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        acc += __shfl_xor(acc, 4);
        if (q == 0) {
            const float b = fpv(a.bT2 + k);
            a.tc[TC_TE + k] = acc + b;
            te[k] = k < 30 ? acc + b : 0.f;
        }
    }
    __syncthreads();
    {  // C0 / C5: the biases of linear.0 / linear.5 with the t_emb columns folded in (k_fwd, uniform t)
        const int w0 = a.w0te + j * 32, w5 = a.w5te + j * 32;
        float c0 = fpv(a.bL[0] + j), c5 = fpv(a.bL[5] + j);
#pragma unroll
        for (int k = 0; k < 30; k++) {
            c0 = fmaf(fpv(w0 + k), te[k], c0);
            c5 = fmaf(fpv(w5 + k), te[k], c5);
        }
        a.tc[TC_C0 + j] = c0;
        a.tc[TC_C5 + j] = c5;
    }
}

__global__ __launch_bounds__(256) void k_timenet(FwdArgs a) {
    const float *fp = a.fp;
    timenet_body(a, [fp](int o) { return fp[o]; });
}

// One block of NQB 16-point column tiles (NQB = 4: the 64-point blocks; NQB = 1: the 16-point tail
// blocks that spread the last, sparse round of blocks over the idle CUs). p0: first point; slot: the
// block's relu'-mask slot.

// per column tile q (16 points): max |v| over this wave's tiles of it (two n-tiles: both), in every lane
template <int NQ_>
__device__ inline void col_absmax(const f32x4 (&v)[NQ_], float (&m)[NQ_]) {
#pragma unroll
    for (int q = 0; q < NQ_; q++) {
        float x = 0.f;
#pragma unroll
        for (int i = 0; i < 4; i++) x = fmaxf(x, fabsf(v[q][i]));
        m[q] = fmaxf(m[q], x);
    }
}
template <int NQ_>
__device__ inline void col_wave_max(float (&m)[NQ_]) {
#pragma unroll
    for (int q = 0; q < NQ_; q++) m[q] = wave_max(m[q]);
}

// the stage value of point slot m (0 .. 63 of the image) goes to column tile m >> 4
__device__ __forceinline__ int qof(int m) { return m >> 4; }

template <bool SAVE, int NQB, bool FOLD>
__device__ __forceinline__ void fwd_block(const FwdArgs &a, h16x8 *lds, uint32_t *hwr, uint32_t *hrd, const float4 *sb,
                                          uint32_t *s_mpend, ScaleLDS *sc, int p0, int slot) {
    constexpr int BMB = 16 * NQB;  // points of this block (the LDS images keep the BM-point stride)
    float *lf = reinterpret_cast<float *>(lds);
    float *stage = lf + G_H * UG * 4;  // fp32 [112][BM] feature staging (H region, before the trunk)
    // re-derived per block (opaque to loop-invariant hoisting): in the persistent loop, lane
    // addresses hoisted out of it would stay live across the whole block and spill
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int r = __builtin_amdgcn_readfirstlane(tid >> 6);  // n-tile of this wave (provably uniform)
    const int kq = lane >> 4, col = lane & 15;
    const int pend = min(a.N, p0 + BMB);  // real points of the block: [p0, pend)
    const Flags F = make_flags(a.flags);
    const size_t Ns = a.Ns;
    const __amdgpu_buffer_rsrc_t mrsrc = __builtin_amdgcn_make_buffer_rsrc(
        a.mask + (SAVE ? (size_t)slot * 2 * F.nmask : 0), 0, 0x7fffffff, 0x00020000);
    auto store_mask = [&](uint32_t w, int mr) {  // u16 mask tile mr (= row / 16): the timenet's TH
        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)w, mrsrc, lane * 2, mr * 128, 0);
    };
    // the trunk's: layer L's bits wait in LDS (this thread's own word) until layer L + 1 (odd) stores
    // both as one dword: half the mask stores, and k_bwd loads one dword per two layers
    // (tools/mlp_time.py A/B: k_fwd -0.8 %, k_bwd -2 %, profiles/r4j_mlp_mask_pairs_ab.txt)
    auto trunk_mask = [&](uint32_t w, int L) {
        if ((L & 1) == 0) {
            s_mpend[64 * r + lane] = w;
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(s_mpend[64 * r + lane] | (w << 16), mrsrc, lane * 4,
                                                  (16 * (L >> 1) + r) * 256, 0);
        }
    };
    DGS_STAMP(0);
    // frame-uniform t: all points of the block carry k_timenet's t0 (every wave checks the same
    // values, so the branch is block-uniform without a barrier)
    bool uniform_t = FOLD || (F.uniform_t && a.tc);  // the caller's guarantee (DGS_MLP_UNIFORM_T), else checked
    if (!FOLD && F.blender && a.tc && !uniform_t) {
        const float t0 = a.tc[TC_T];
        const int p = p0 + lane;
        const float tv = (lane < BMB && p < a.N) ? a.t[p] : t0;
        uniform_t = __ballot(tv != t0) == 0;
    }
    // t_emb folded into the linear.0 / linear.5 biases (FOLD = DGS_MLP_UNIFORM_T; the host always
    // provides tc then): no t_emb / TIN staging, the trunk GEMMs read x_emb (| h) only
    constexpr bool fold = FOLD;
    if (tid < 8) {
        hwr[tid] = 0;
        hrd[tid] = 0;
    }
    if (tid < 32) (&sc->bsync[0][0])[tid] = 0;
    // ---- positional encodings (utils/time_utils.py:42-54) into fp32 staging: feature 3 band + d,
    // band 0 = x, band 1 + 2i = sin(2^i x), band 2 + 2i = cos(2^i x). The block's xyz rows are read
    // once (one coalesced load per thread, a single HBM round trip) into the identity band, then the
    // 10 sin/cos bands are evaluated from LDS in two rounds of the workgroup. x_emb's scale bound per
    // column tile: max(1, max |xyz|) (|sin|, |cos| <= 1) ----
    float xmax = 0.f;
    if (tid < 3 * BMB) {
        const int m = tid / 3, d = tid - 3 * m;
        const float v = p0 + m < pend ? a.xyz[3 * (size_t)p0 + tid] : 0.f;
        stage[d * BM + m] = v;
        xmax = fabsf(v);
    }
    if (tid < BMB) stage[63 * BM + tid] = 0.f;  // padding feature
    __syncthreads();
    if (tid < 3 * BMB) lds_fmax(&sc->bsync[BS_XE][qof(tid / 3)], xmax);
    for (int e = tid; e < BMB * 3 * 10; e += NTHR) {
        const int m = e % BMB, rr = e / BMB, d = rr % 3, i = rr / 3;
        const bool ok = p0 + m < pend;
        float sv, cv;
        sincosf(stage[d * BM + m] * (float)(1 << i), &sv, &cv);
        stage[(3 * (1 + 2 * i) + d) * BM + m] = ok ? sv : 0.f;
        stage[(3 * (2 + 2 * i) + d) * BM + m] = ok ? cv : 0.f;
    }
    if (fold) {
    } else if (uniform_t) {  // TE and TIN: k_timenet's values broadcast over the points
        for (int e = tid; e < 48 * BMB; e += NTHR) {
            const int f = e / BMB, m = e % BMB;
            const float v = f < 32 ? a.tc[TC_TE + f] : a.tc[TC_TIN + f - 32];
            stage[(ST_TE + f) * BM + m] = v;
            lds_fmax(&sc->bsync[f < 32 ? BS_TE : BS_TIN][qof(m)], fabsf(v));
        }
    } else {  // per-point t encodings: TIN (blender, 16 rows) or the raw t PE as TE (32 rows)
        const int row0 = F.blender ? ST_TIN : ST_TE, nrow = F.blender ? 16 : 32;
        for (int e = tid; e < nrow * BMB; e += NTHR) {
            const int f = e / BMB, m = e % BMB;
            const int p = p0 + m;
            const float x = p < pend ? a.t[p] : 0.f;
            float v = 0.f;
            if (p < pend && f < F.tin) {
                if (f == 0) {
                    v = x;
                } else {
                    float sv, cv;
                    sincosf(x * (float)(1 << ((f - 1) >> 1)), &sv, &cv);
                    v = (f & 1) ? sv : cv;
                }
            }
            stage[(row0 + f) * BM + m] = v;
            lds_fmax(&sc->bsync[F.blender ? BS_TIN : BS_TE][qof(m)], fabsf(v));
        }
    }
    __syncthreads();
    // column-tile scales of the staged inputs (every thread evaluates the same values)
    if (tid < 4) {
        const int q = tid;
        const float xe_b = fmaxf(1.f, __uint_as_float(sc->bsync[BS_XE][q]));
        sc->ksc[0][q] = sc->ksc[1][q] = scale_for(xe_b).inv;
        sc->ain[0][q] = xe_b;
        if (!fold) {
            sc->ksc[G_TE / 4][q] = scale_for(__uint_as_float(sc->bsync[BS_TE][q])).inv;
            sc->ksc[G_TIN / 4][q] = scale_for(__uint_as_float(sc->bsync[BS_TIN][q])).inv;
            sc->ain[1][q] = __uint_as_float(sc->bsync[BS_TE][q]);  // per-point blender: replaced by the TE tile's
        }
    }
    // saved network inputs (fp32, coalesced) and their split LDS images
    const bool te_ready = uniform_t || !F.blender;
    if (SAVE) {
        // XE | TE rows are adjacent in saved (S_TE = S_XE + 64); folded: dW reads x_emb only
        const int nrow = te_ready && !fold ? 96 : 64;
        for (int e = tid; e < nrow * BMB; e += NTHR) {
            const int f = e / BMB, m = e % BMB;
            a.saved[(size_t)(S_XE + f) * Ns + p0 + m] = stage[f * BM + m];
        }
        if (F.blender && !fold)
            for (int e = tid; e < 16 * BMB; e += NTHR) {
                const int f = e / BMB, m = e % BMB;
                a.saved[(size_t)(S_TIN + f) * Ns + p0 + m] = stage[(ST_TIN + f) * BM + m];
            }
    }
    {
        const int ngrp = fold ? 8 : F.blender ? 14 : 12;  // staging groups: XE 0-7 | TE 8-11 | TIN 12-13
        for (int u = tid; u < ngrp * BMB; u += NTHR) {
            const int g = u / BMB, m = u % BMB;
            if (g >= G_TE && g < G_H && !te_ready) continue;  // TE comes from the per-point timenet
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; j++) v[j] = stage[(8 * g + j) * BM + m];
            const int slot_b = g < G_TE ? BS_XE : g < 12 ? BS_TE : BS_TIN;
            const float bnd = __uint_as_float(sc->bsync[slot_b][qof(m)]);
            put_unit8(lds, g < 12 ? g : G_TIN + g - 12, m, v, scale_for(g < G_TE ? fmaxf(1.f, bnd) : bnd).s);
        }
        if (F.blender && !fold)  // TIN k-step padding (features 16..31): zero, not stale LDS
            for (int u = tid; u < 2 * UG; u += NTHR) lds[(G_TIN + 2) * UG + u] = h16x8{};
    }
    lds_barrier();
    DGS_STAMP(1);
    f32x4 c[NQB];
    float ib[NQB];
    if (SAVE && uniform_t && !F.uniform_t) {  // TH tile from k_timenet: relu' bits + saved rows (per-point backward)
        const float4 th = load_bias4(a.tc + TC_TH, r, lane);
#pragma unroll
        for (int q = 0; q < NQB; q++) c[q] = f32x4{th.x, th.y, th.z, th.w};
        store_mask(relu_bits(c), MR_TH + r);
        tile16(a.saved, Ns, S_TH + 16 * r, p0, lane).store(c);
    }
    // ---- per-point timenet (blender, t not frame-uniform): Linear(13,256)+ReLU -> H; Linear(256,30) -> TE.
    // Both outputs are narrow per-block tiles: their scales are the actual maxima per column tile,
    // gathered behind a workgroup barrier
    if (F.blender && !uniform_t) {
        zero_tiles(c);
        const h16x8 *A1 = a.img + (size_t)(a.fT1 + r) * KSLOT;
        gemm<1, NQB>(A1, lds, G_TIN, 0, lane, c, ib, sc->ksc);
        bias_relu(c, a_inv(A1), ib, load_bias4(a.fp + a.bT1, r, lane), true);
        if (SAVE) {
            store_mask(relu_bits(c), MR_TH + r);
            tile16(a.saved, Ns, S_TH + 16 * r, p0, lane).store(c);
        }
        float thm[NQB] = {};
        col_absmax(c, thm);
        col_wave_max(thm);
        if (lane == 0)
#pragma unroll
            for (int q = 0; q < NQB; q++) lds_fmax(&sc->bsync[BS_TH][q], thm[q]);
        lds_barrier();
#pragma unroll
        for (int q = 0; q < NQB; q++)
            acc_to_lds(c[q], lds, G_H, r, q, lane, scale_for(__uint_as_float(sc->bsync[BS_TH][q])).s);
        if (tid < 32) sc->ksc[G_H / 4 + (tid >> 2)][tid & 3] = scale_for(__uint_as_float(sc->bsync[BS_TH][tid & 3])).inv;
        lds_barrier();
        f32x4 c1[1] = {zero4()};
        if (r < 2 * NQB) {  // TE tile (n-tile r / NQB of 2, column tile r % NQB), full K on one wave
            const int nt = r / NQB, q = r % NQB;
            const h16x8 *A2 = a.img + (size_t)(a.fT2 + nt * 8) * KSLOT;
            float ib2[1];
            gemm<8, 1>(A2, lds, G_H, q, lane, c1, ib2, sc->ksc);
            const float4 b = load_bias4(a.fp + a.bT2, nt, lane);
            c1[0] = c1[0] * (a_inv(A2) * ib2[0]) + f32x4{b.x, b.y, b.z, b.w};
            if (SAVE) tile16(a.saved, Ns, S_TE + 16 * nt, p0, lane).store(c1, q);
            float tm[1] = {0.f};
            col_absmax(c1, tm);
            col_wave_max(tm);
            if (lane == 0) lds_fmax(&sc->bsync[BS_TET][q], tm[0]);
        }
        lds_barrier();
        if (r < 2 * NQB)  // TE groups: not read by the T2 GEMM
            acc_to_lds(c1[0], lds, G_TE, r / NQB, r % NQB, lane,
                       scale_for(__uint_as_float(sc->bsync[BS_TET][r % NQB])).s);
        if (tid < 4) {
            const float tet = __uint_as_float(sc->bsync[BS_TET][tid]);
            sc->ksc[G_TE / 4][tid] = scale_for(tet).inv;
            sc->ain[1][tid] = tet;
        }
        lds_barrier();
    }
    // ---- trunk: 8 x (Linear + ReLU), skip cat after layer 4 (time_utils.py:107-112) ----
    // No workgroup barriers: the four waves of a SIMD finish a GEMM thousands of cycles apart (the
    // oldest issues first), so each wave runs its epilogue as soon as every wave has read the H
    // k-step it overwrites (hrd), and the next layer reads an H k-step once its two writer waves
    // have stored it (hwr): early waves' epilogues overlap late waves' MFMAs. Every writer derives the
    // layer's output scales from the same bounds (header note), so none waits for another's maximum.
#pragma unroll 1
    for (int L = 0; L < 8; L++) {
        const int g0 = (L == 0 || L == 5) ? G_XE : G_H;
        const int nk = layer_kpad_f(F, L) / 32;
        zero_tiles(c);
        const h16x8 *Aw = a.img + (size_t)(a.fL[L] + r * nk) * KSLOT;
        const HGate hg{hwr, hrd, L == 5 ? (fold ? 2 : 3) : 0, 2u * L, true, lane};
        if (L == 0) {
            if constexpr (FOLD) gemm<2, NQB>(Aw, lds, g0, 0, lane, c, ib, sc->ksc);  // XE only
            else gemm<3, NQB, NoPre, NoGate, 1 << 20, 1u << 2>(Aw, lds, g0, 0, lane, c, ib, sc->ksc);  // XE | TE
        } else if (L == 5) {
            if constexpr (FOLD) gemm<10, NQB, NoPre, HGate, 2, 1u << 2>(Aw, lds, g0, 0, lane, c, ib, sc->ksc, NoPre(), hg);  // XE | H
            else gemm<11, NQB, NoPre, HGate, 1 << 20, (1u << 2) | (1u << 3)>(Aw, lds, g0, 0, lane, c, ib, sc->ksc, NoPre(), hg);  // XE | TE | H
        } else {
            gemm<8, NQB>(Aw, lds, g0, 0, lane, c, ib, sc->ksc, NoPre(), hg);
        }
        const float4 bv = sb[64 * L + 4 * r + kq];
        DGS_STAMP(4 + 2 * L);
        DGS_WSTAMP(22, L);  // per wave: GEMM end (layer 3)
        bias_relu(c, a_inv(Aw), ib, bv, true);
        if (SAVE) {
            trunk_mask(relu_bits(c), L);
#ifndef DGS_DIAG_NOSAVE  // diagnostic only (wrong backward): the trunk's saved-activation stores skipped
            tile16(a.saved, Ns, s_h(L) + 16 * r, p0, lane).store(c);
#endif
        }
        // the layer's output scales: max_rows sum |W_L| x max |input| + max |b_L| per column tile (the
        // same on every wave)
        float so[NQB], my[NQB] = {};
        const float ws = __uint_as_float(sc->wstat[L]), bm = __uint_as_float(sc->bmax[L]);
        const float4 am = L > 0 ? amax_of4(sc, (L - 1) & 1, NWAVE) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < NQB; q++) {
            float ain = fmaxf(L == 0 || L == 5 ? sc->ain[0][q] : 0.f, f4get(am, q));
            if (!fold && (L == 0 || L == 5)) ain = fmaxf(ain, sc->ain[1][q]);
            so[q] = fmaf(ws, ain, bm);
        }
        col_absmax(c, my);
        col_wave_max(my);
        if (L == 3 && r == 0) DGS_STAMP(54);
        // this wave's rows are H k-step r / 2: every wave must have read it (and its scales) in this layer
        if (L > 0) lds_wait_ge(hrd + (r >> 1), 16u * L, lds_peek(hrd + (r >> 1)));
        if (L == 3 && r == 0) DGS_STAMP(56);
#pragma unroll
        for (int q = 0; q < NQB; q++) {
            const Scale s = scale_for(so[q]);
            if (lane == 0) {
                sc->amax[L & 1][r][q] = my[q];
                sc->ksc[G_H / 4 + (r >> 1)][q] = s.inv;
            }
            acc_to_lds(c[q], lds, G_H, r, q, lane, s.s);
        }
        lds_signal(hwr + (r >> 1), lane);
        if (L == 3 && r == 0) DGS_STAMP(55);
        DGS_STAMP(5 + 2 * L);
    }
    DGS_STAMP(20);
    // ---- heads (no activation): [warp | branch_w, branch_v], rotation, scaling: 16 rows (nout <= 13),
    // one column tile per wave, once all 8 layers' writers have signalled ----
    // on the LAST wave of each SIMD (waves NWAVE - NQB ..): they finish layer 7 last (the MFMA pipe
    // serves the oldest wave of a SIMD first), so they start the heads without waiting on a signal,
    // while the earlier waves are already done
    const int hq = r - (NWAVE - NQB);
    if (hq >= 0) {
        f32x4 c1[1] = {zero4()};
        float ib1[1];
        const h16x8 *Ah = a.img + (size_t)a.fHd * KSLOT;
        gemm<8, 1>(Ah, lds, G_H, hq, lane, c1, ib1, sc->ksc, NoPre(), HGate{hwr, hrd, 0, 16u, false, lane});
        const float4 b = sb[8 * 64 + kq];
        c1[0] = c1[0] * (a_inv(Ah) * ib1[0]) + f32x4{b.x, b.y, b.z, b.w};
        const int p = p0 + 16 * hq + col;
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (p < pend && 4 * kq + i < F.nout) a.out[(size_t)p * F.nout + 4 * kq + i] = c1[0][i];
    }
    DGS_STAMP(21);
#ifdef DGS_MLP_PROFILE
    if (threadIdx.x == 0 && p0 == (int)blockIdx.x * BM) {
        dgs_mlps_prof[blockIdx.x * 64 + 60] = __builtin_amdgcn_s_memrealtime();
        dgs_mlps_prof[blockIdx.x * 64 + 61] = __builtin_amdgcn_s_memtime();
    }
#endif
}

// The launch-constant bias table of the forward kernels (one float4 per (layer, 4 rows), the heads' 16
// rows last; FOLD's linear.0 / linear.5 biases come from k_timenet), each layer's max |b| and the trunk
// images' row statistics (over their 16 n-tiles) for the output-scale bounds
template <bool FOLD>
__device__ inline void load_bias_table(const FwdArgs &a, float4 *s_bias, ScaleLDS *sc, int nthr) {
    if (threadIdx.x < 10) sc->bmax[threadIdx.x] = sc->wstat[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x < 8 * 16) {
        const int L = threadIdx.x >> 4, t = threadIdx.x & 15;
        const int nk = layer_kpad_f(make_flags(a.flags), L) / 32;
        lds_fmax(&sc->wstat[L], tile_stat(a.img + (size_t)(a.fL[L] + t * nk) * KSLOT));
    }
    for (int i = threadIdx.x; i < 8 * 64 + 4; i += nthr) {
        const int L = i >> 6;
        const float *bias = L == 8                ? a.fp + a.bHd
                            : FOLD && L == 0      ? a.tc + TC_C0
                            : FOLD && L == 5      ? a.tc + TC_C5
                                                  : a.fp + a.bL[L];
        const float4 v = reinterpret_cast<const float4 *>(bias)[i & 63];
        s_bias[i] = v;
        lds_fmax(&sc->bmax[L], fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
}

template <bool SAVE, bool FOLD>
__global__ __launch_bounds__(NTHR) void k_fwd(FwdArgs a) {
    __shared__ h16x8 lds[G_FWD * UG];
    __shared__ uint32_t hwr[8], hrd[8];  // trunk hand-off counters (HGate)
    __shared__ int s_next;
    __shared__ float4 s_bias[8 * 64 + 4];
    __shared__ uint32_t s_mpend[NTHR];  // relu' bits of an even trunk layer, per thread (fwd_block)
    __shared__ ScaleLDS sc;
    // the first block's staging barriers publish the bias table
    load_bias_table<FOLD>(a, s_bias, &sc, NTHR);
    CLK_BEGIN();
    for (int b = blockIdx.x;;) {
        int nx = 0;
        if (a.queue && threadIdx.x == 0) nx = queue_take(a.queue);
        if (b < a.nfull) fwd_block<SAVE, NQ, FOLD>(a, lds, hwr, hrd, s_bias, s_mpend, &sc, b * BM, b);
        else fwd_block<SAVE, 1, FOLD>(a, lds, hwr, hrd, s_bias, s_mpend, &sc, a.nfull * BM + (b - a.nfull) * 16, b);
        if (!a.queue) break;
        if (threadIdx.x == 0) s_next = nx;
        __syncthreads();  // also: the next block's staging overwrites LDS this one's heads read
        b = s_next;
        if (b >= a.nblk) break;
    }
    if (a.queue) queue_release(a.queue);
    CLK_END(0);
}


// The training forward (saved activations, frame-uniform t folded) as 8 waves of two n-tiles
// (k_fwd8, 512 threads, 2 waves per SIMD): wave w owns rows 32w .. 32w + 31 of every trunk layer = H
// k-step w, so each k-step has ONE writer (hand-off target L per layer) and 8 readers. Same LDS image,
// saved-activation / relu'-mask layouts, scales and arithmetic as fwd_block<true, NQB, true>.
constexpr int NW8 = 8, NTHR8 = NW8 * 64;
template <int NQB>
__device__ __forceinline__ void fwd_block8(const FwdArgs &a, h16x8 *lds, uint32_t *hwr, uint32_t *hrd, const float4 *sb,
                                           uint32_t *s_mpend, ScaleLDS *sc, int p0, int slot) {
    constexpr int BMB = 16 * NQB;
    float *lf = reinterpret_cast<float *>(lds);
    float *stage = lf + G_H * UG * 4;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // rows 32w .. 32w + 31: n-tiles 2w, 2w + 1
    const int kq = lane >> 4;
    const int pend = min(a.N, p0 + BMB);
    const Flags F = make_flags(a.flags);
    const size_t Ns = a.Ns;
    const __amdgpu_buffer_rsrc_t mrsrc =
        __builtin_amdgcn_make_buffer_rsrc(a.mask + (size_t)slot * 2 * F.nmask, 0, 0x7fffffff, 0x00020000);
    auto trunk_mask = [&](uint32_t m, int L, int nt) {  // as fwd_block's, per n-tile
        if ((L & 1) == 0) {
            s_mpend[64 * nt + lane] = m;
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(s_mpend[64 * nt + lane] | (m << 16), mrsrc, lane * 4,
                                                  (16 * (L >> 1) + nt) * 256, 0);
        }
    };
    DGS_STAMP(0);
    if (tid < 8) {
        hwr[tid] = 0;
        hrd[tid] = 0;
    }
    if (tid < 4) sc->bsync[BS_XE][tid] = 0;
    // positional encodings (utils/time_utils.py:42-54), as fwd_block
    float xmax = 0.f;
    if (tid < 3 * BMB) {
        const int m = tid / 3, d = tid - 3 * m;
        const float v = p0 + m < pend ? a.xyz[3 * (size_t)p0 + tid] : 0.f;
        stage[d * BM + m] = v;
        xmax = fabsf(v);
    }
    if (tid < BMB) stage[63 * BM + tid] = 0.f;
    __syncthreads();
    if (tid < 3 * BMB) lds_fmax(&sc->bsync[BS_XE][qof(tid / 3)], xmax);
    for (int e = tid; e < BMB * 3 * 10; e += NTHR8) {
        const int m = e % BMB, rr = e / BMB, d = rr % 3, i = rr / 3;
        const bool ok = p0 + m < pend;
        float sv, cv;
        sincosf(stage[d * BM + m] * (float)(1 << i), &sv, &cv);
        stage[(3 * (1 + 2 * i) + d) * BM + m] = ok ? sv : 0.f;
        stage[(3 * (2 + 2 * i) + d) * BM + m] = ok ? cv : 0.f;
    }
    __syncthreads();
    if (tid < 4) {
        const float xe_b = fmaxf(1.f, __uint_as_float(sc->bsync[BS_XE][tid]));
        sc->ksc[0][tid] = sc->ksc[1][tid] = scale_for(xe_b).inv;
        sc->ain[0][tid] = xe_b;
    }
    for (int e = tid; e < 64 * BMB; e += NTHR8) {  // saved x_emb rows (folded: dW reads x_emb only)
        const int f = e / BMB, m = e % BMB;
        a.saved[(size_t)(S_XE + f) * Ns + p0 + m] = stage[f * BM + m];
    }
    for (int u = tid; u < 8 * BMB; u += NTHR8) {
        const int g = u / BMB, m = u % BMB;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = stage[(8 * g + j) * BM + m];
        put_unit8(lds, g, m, v, scale_for(fmaxf(1.f, __uint_as_float(sc->bsync[BS_XE][qof(m)]))).s);
    }
    lds_barrier();
    DGS_STAMP(1);
    f32x4 c[2][NQB];
    float ib[NQB];
#pragma unroll 1
    for (int L = 0; L < 8; L++) {
        const int g0 = (L == 0 || L == 5) ? G_XE : G_H;
        const int nk = layer_kpad_f(F, L) / 32;
#pragma unroll
        for (int t = 0; t < 2; t++) zero_tiles(c[t]);
        const h16x8 *Aw = a.img + (size_t)(a.fL[L] + 2 * w * nk) * KSLOT;
        const int astride = nk * KSLOT;
        const HGate hg{hwr, hrd, L == 5 ? 2 : 0, 1u * L, true, lane};
        DGS_WSTAMP8(24, L);
        if (L == 0) gemm2<2, NQB>(Aw, astride, lds, g0, 0, lane, c, ib, sc->ksc);
        else if (L == 5) gemm2<10, NQB, NoPre, HGate, 2, 1u << 2>(Aw, astride, lds, g0, 0, lane, c, ib, sc->ksc, NoPre(), hg);
        else gemm2<8, NQB>(Aw, astride, lds, g0, 0, lane, c, ib, sc->ksc, NoPre(), hg);
        DGS_WSTAMP8(32, L);
        float my[NQB] = {};
#pragma unroll
        for (int t = 0; t < 2; t++) {
            const int nt = 2 * w + t;
            bias_relu(c[t], a_inv(Aw + t * astride), ib, sb[64 * L + 4 * nt + kq], true);
            trunk_mask(relu_bits(c[t]), L, nt);
#ifndef DGS_DIAG_NOSAVE  // diagnostic only (wrong backward): the trunk's saved-activation stores skipped
            tile16(a.saved, Ns, s_h(L) + 16 * nt, p0, lane).store(c[t]);
#endif
            col_absmax(c[t], my);
        }
        // the layer's output scales: max_rows sum |W_L| x max |input| + max |b_L| per column tile (the
        // same on every wave)
        float so[NQB];
        const float ws = __uint_as_float(sc->wstat[L]), bm = __uint_as_float(sc->bmax[L]);
        const float4 am = L > 0 ? amax_of4(sc, (L - 1) & 1, NW8) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < NQB; q++) so[q] = fmaf(ws, fmaxf(L == 0 || L == 5 ? sc->ain[0][q] : 0.f, f4get(am, q)), bm);
        col_wave_max(my);
        // this wave's rows are H k-step w: all 8 waves must have read it (and its scales) in this layer
        DGS_WSTAMP8(40, L);
        if (L > 0) lds_wait_ge(hrd + w, (uint32_t)NW8 * L, lds_peek(hrd + w));
        DGS_WSTAMP8(48, L);
#pragma unroll
        for (int q = 0; q < NQB; q++) {
            const Scale s = scale_for(so[q]);
            if (lane == 0) {
                sc->amax[L & 1][w][q] = my[q];
                sc->ksc[G_H / 4 + w][q] = s.inv;
            }
#pragma unroll
            for (int t = 0; t < 2; t++) acc_to_lds(c[t][q], lds, G_H, 2 * w + t, q, lane, s.s);
        }
        lds_signal(hwr + w, lane);
        DGS_WSTAMP8(56, L);
    }
    DGS_STAMP(20);
    // heads on the last NQB waves (one column tile each), once all 8 layers' writers have signalled
    const int hq = w - (NW8 - NQB);
    if (hq >= 0) {
        f32x4 c1[1] = {zero4()};
        float ib1[1];
        const h16x8 *Ah = a.img + (size_t)a.fHd * KSLOT;
        gemm<8, 1>(Ah, lds, G_H, hq, lane, c1, ib1, sc->ksc, NoPre(), HGate{hwr, hrd, 0, 8u, false, lane});
        const float4 b = sb[8 * 64 + kq];
        c1[0] = c1[0] * (a_inv(Ah) * ib1[0]) + f32x4{b.x, b.y, b.z, b.w};
        const int p = p0 + 16 * hq + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (p < pend && 4 * kq + i < F.nout) a.out[(size_t)p * F.nout + 4 * kq + i] = c1[0][i];
    }
}

__global__ __launch_bounds__(NTHR8) void k_fwd8(FwdArgs a) {
    __shared__ h16x8 lds[G_FWD * UG];
    __shared__ uint32_t hwr[8], hrd[8];
    __shared__ int s_next;
    __shared__ float4 s_bias[8 * 64 + 4];
    __shared__ uint32_t s_mpend[NTHR];  // [n-tile][64 lanes]
    __shared__ ScaleLDS sc;
    load_bias_table<true>(a, s_bias, &sc, NTHR8);
    for (int b = blockIdx.x;;) {
        int nx = 0;
        if (a.queue && threadIdx.x == 0) nx = queue_take(a.queue);
        if (b < a.nfull) fwd_block8<NQ>(a, lds, hwr, hrd, s_bias, s_mpend, &sc, b * BM, b);
        else fwd_block8<1>(a, lds, hwr, hrd, s_bias, s_mpend, &sc, a.nfull * BM + (b - a.nfull) * 16, b);
        if (!a.queue) break;
        if (threadIdx.x == 0) s_next = nx;
        __syncthreads();
        b = s_next;
        if (b >= a.nblk) break;
    }
    if (a.queue) queue_release(a.queue);
}

// ------------------------------------------------------------------------------------------------
// backward (dX chain): dZ_i for every layer -> scratch; deterministic
// ------------------------------------------------------------------------------------------------
struct BwdArgs {
    int N;
    size_t Ns;
    const h16x8 *img;
    const uint32_t *mask;
    const float *dout;
    float *dz;
    int nfull;            // as FwdArgs::nfull
    int tHd, tL[8], tT2;  // image k-slots
    int flags;
    uint32_t *queue;      // as FwdArgs
    int nblk;
};

// relu' bits of a trunk layer's output tile (the [layer pair][row / 16][64 lanes] u32 layout),
// loaded ahead of the GEMM
struct MaskPre32 {
    uint32_t *mk;
    const uint32_t *word;  // &mask[block][layer pair][row / 16][0]
    int shift, lane;
    __device__ void operator()() const { *mk = word[lane] >> shift; }
};

// relu' bits of the layer input for this wave's 16 x 64 tile (u16 tiles: TH), loaded ahead of the GEMM
struct MaskPre {
    uint32_t *mk;
    const unsigned short *tile;  // &mask[block][mr][0]
    int lane;
    __device__ void operator()() const { *mk = tile[lane]; }
};

// the dX chain's row statistics (launch constants): wstat[L] over tL[L]'s n-tiles (max column abs sum
// of W_L), wstat[8] over the heads' transposed image; published by the first block's staging barriers
__device__ inline void load_wstats_bwd(const BwdArgs &a, ScaleLDS *sc) {
    if (threadIdx.x < 10) sc->wstat[threadIdx.x] = 0;
    __syncthreads();
    const int i = threadIdx.x;
    if (i < 16) {
        lds_fmax(&sc->wstat[8], tile_stat(a.img + (size_t)(a.tHd + i) * KSLOT));
    } else if (i < 16 + 7 * 32) {
        const int L = 1 + (i - 16) / 32, t = (i - 16) % 32;
        if (t < layer_kpad(L) / 16) lds_fmax(&sc->wstat[L], tile_stat(a.img + (size_t)(a.tL[L] + t * 8) * KSLOT));
    }
}

// dOut -> dz rows Z_G (heads' dW) and the split G image, scaled by its max |dOut| per column tile
template <int NQB, int NT>
__device__ inline void stage_dout(const BwdArgs &a, h16x8 *lds, ScaleLDS *sc, float *stage, int p0, int tid) {
    constexpr int BMB = 16 * NQB;
    const Flags F = make_flags(a.flags);
    if (tid < 32) (&sc->bsync[0][0])[tid] = 0;
    for (int e = tid; e < 32 * BMB; e += NT) {
        const int c = e / BMB, m = e % BMB;
        const int p = p0 + m;
        const float v = (p < a.N && c < F.nout) ? a.dout[(size_t)p * F.nout + c] : 0.f;
        a.dz[(size_t)(Z_G + c) * a.Ns + p] = v;
        stage[c * BM + m] = v;
    }
    __syncthreads();
    for (int e = tid; e < 32 * BMB; e += NT) {
        const int c = e / BMB, m = e % BMB;
        lds_fmax(&sc->bsync[BS_G][qof(m)], fabsf(stage[c * BM + m]));
    }
    __syncthreads();
    if (tid < 4) {
        const float gmax = __uint_as_float(sc->bsync[BS_G][tid]);
        sc->ksc[G_BG / 4][tid] = scale_for(gmax).inv;
        sc->ain[0][tid] = gmax;
    }
    if (tid < 4 * BMB) {
        const int g = tid / BMB, m = tid % BMB;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = stage[(8 * g + j) * BM + m];
        put_unit8(lds, G_BG + g, m, v, scale_for(__uint_as_float(sc->bsync[BS_G][qof(m)])).s);
    }
    lds_barrier();
}

// The output scales of a dX-chain step per column tile: max_cols sum |W| x max |dZ in| (the relu' mask
// only zeroes), the same on every wave
template <int NQB>
__device__ inline void chain_scales(const ScaleLDS *sc, float ws, int par, int nw, float (&so)[NQB]) {
    const float4 am = par < 0 ? *reinterpret_cast<const float4 *>(sc->ain[0]) : amax_of4(sc, par, nw);
#pragma unroll
    for (int q = 0; q < NQB; q++) so[q] = ws * f4get(am, q);
}

// TE_ROWS: per-point dL/dt_emb (blender, t not frame-uniform); the other instantiation carries no
// t_emb registers or code (raw t PE has no parameters upstream; uniform t: k_tgrad)
template <bool TE_ROWS, int NQB>
__device__ __forceinline__ void bwd_block(const BwdArgs &a, h16x8 *lds, uint32_t *hwr, uint32_t *hrd, ScaleLDS *sc,
                                          int p0, int slot) {
    float *lf = reinterpret_cast<float *>(lds);
    float *stage = lf + G_BH * UG * 4;  // fp32 [32][BM] (H region, before the first dZ)
    // re-derived per block (opaque to loop-invariant hoisting): in the persistent loop, lane
    // addresses hoisted out of it would stay live across the whole block and spill
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int r = __builtin_amdgcn_readfirstlane(tid >> 6);
    const Flags F = make_flags(a.flags);
    const size_t Ns = a.Ns;
    const unsigned short *mtiles = reinterpret_cast<const unsigned short *>(a.mask + (size_t)slot * 2 * F.nmask);
    auto mask_tile = [&](int mr) { return mtiles + (size_t)mr * 64; };
    const uint32_t *mwords = a.mask + (size_t)slot * 2 * F.nmask;
    auto trunk_pre = [&](uint32_t *mk, int L) {  // layer L's output tile of this wave (MaskPre32)
        return MaskPre32{mk, mwords + (size_t)(16 * (L >> 1) + r) * 64, 16 * (L & 1), lane};
    };
    if (tid < 8) {
        hwr[tid] = 0;
        hrd[tid] = 0;
    }
    stage_dout<NQB, NTHR>(a, lds, sc, stage, p0, tid);
    f32x4 c[NQB];
    float ib[NQB];
    // The dZ chain runs without workgroup barriers (see k_fwd's trunk): step 0 (heads^T) and steps
    // i = 1..7 (layer L = 8 - i) each write dZ into H; step i reads H once both writers of each
    // k-step have signalled (hwr >= 2i) and overwrites its own k-step once all 16 waves have read
    // it (hrd >= 16i).
    // heads^T: dH7 = W_h^T dOut (K = 32 from G) -> mask H7 -> dZ7
    {
        uint32_t mk;
        zero_tiles(c);
        const h16x8 *Ah = a.img + (size_t)(a.tHd + r) * KSLOT;
        gemm<1, NQB>(Ah, lds, G_BG, 0, lane, c, ib, sc->ksc, trunk_pre(&mk, 7));
        scale_tiles(c, a_inv(Ah), ib);
        mask_apply(c, mk);
        tile16(a.dz, Ns, Z_L0 + 7 * 256 + 16 * r, p0, lane).store(c);
        float so[NQB], my[NQB] = {};
        chain_scales(sc, __uint_as_float(sc->wstat[8]), -1, 0, so);
        col_absmax(c, my);
        col_wave_max(my);
#pragma unroll
        for (int q = 0; q < NQB; q++) {
            const Scale s = scale_for(so[q]);
            if (lane == 0) {
                sc->amax[0][r][q] = my[q];
                sc->ksc[G_BH / 4 + (r >> 1)][q] = s.inv;
            }
            acc_to_lds(c[q], lds, G_BH, r, q, lane, s.s);
        }
        lds_signal(hwr + (r >> 1), lane);
    }
    f32x4 te5[1] = {zero4()};  // t_emb tile of layer 5's dX (waves 0-7, TE_ROWS), true units
#pragma unroll 1
    for (int L = 7; L >= 1; L--) {
        const uint32_t step = 8 - L;
        // dX_L = W_L^T dZ_L; the H-part rows of the padded L5 input are n-tiles F_H / 16 + r
        if (TE_ROWS && L == 5 && r < 2 * NQB) {  // t_emb rows (padded 64..95 = n-tiles 4, 5) x column tile r % NQB
            const h16x8 *At = a.img + (size_t)(a.tL[5] + (F_TE / 16 + r / NQB) * 8) * KSLOT;
            float ib1[1];
            gemm<8, 1>(At, lds, G_BH, r % NQB, lane, te5, ib1, sc->ksc, NoPre(), HGate{hwr, hrd, 0, 2u * step, false, lane});
            te5[0] *= a_inv(At) * ib1[0];
        }
        const int tile0 = (L == 5) ? F_H / 16 : 0;
        uint32_t mk;
        zero_tiles(c);
        const h16x8 *Aw = a.img + (size_t)(a.tL[L] + (tile0 + r) * 8) * KSLOT;
        gemm<8, NQB>(Aw, lds, G_BH, 0, lane, c, ib, sc->ksc, trunk_pre(&mk, L - 1), HGate{hwr, hrd, 0, 2u * step, true, lane});
        scale_tiles(c, a_inv(Aw), ib);
        mask_apply(c, mk);
#ifndef DGS_DIAG_NOSAVE  // diagnostic only (wrong dW): the dZ chain's stores skipped
        tile16(a.dz, Ns, Z_L0 + (L - 1) * 256 + 16 * r, p0, lane).store(c);
#endif
        float so[NQB], my[NQB] = {};
        chain_scales(sc, __uint_as_float(sc->wstat[L]), (step - 1) & 1, NWAVE, so);
        col_absmax(c, my);
        col_wave_max(my);
        lds_wait_ge(hrd + (r >> 1), 16u * step, lds_peek(hrd + (r >> 1)));
#pragma unroll
        for (int q = 0; q < NQB; q++) {
            const Scale s = scale_for(so[q]);
            if (lane == 0) {
                sc->amax[step & 1][r][q] = my[q];
                sc->ksc[G_BH / 4 + (r >> 1)][q] = s.inv;
            }
            acc_to_lds(c[q], lds, G_BH, r, q, lane, s.s);
        }
        lds_signal(hwr + (r >> 1), lane);
    }
    if (!TE_ROWS) return;
    // layer 0's t_emb rows added to layer 5's: dTE tile (n-tile r / NQB, column tile r % NQB) -> dz rows
    // Z_TE (timenet.2's dW) and the split G image (dOut's, no longer read), scaled by its column tile's max
    if (r < 2 * NQB) {
        const int nt = r / NQB, q = r % NQB;
        f32x4 t0[1] = {zero4()};
        float ib1[1];
        const h16x8 *At = a.img + (size_t)(a.tL[0] + (F_TE / 16 + nt) * 8) * KSLOT;
        gemm<8, 1>(At, lds, G_BH, q, lane, t0, ib1, sc->ksc, NoPre(), HGate{hwr, hrd, 0, 16u, false, lane});
        te5[0] += t0[0] * (a_inv(At) * ib1[0]);
        tile16(a.dz, Ns, Z_TE + 16 * nt, p0, lane).store(te5, q);
        float tm[1] = {0.f};
        col_absmax(te5, tm);
        col_wave_max(tm);
        if (lane == 0) lds_fmax(&sc->bsync[BS_GTE][q], tm[0]);
    }
    lds_barrier();
    if (r < 2 * NQB)
        acc_to_lds(te5[0], lds, G_BG, r / NQB, r % NQB, lane, scale_for(__uint_as_float(sc->bsync[BS_GTE][r % NQB])).s);
    if (tid < 4) sc->ksc[G_BG / 4][tid] = scale_for(__uint_as_float(sc->bsync[BS_GTE][tid])).inv;
    lds_barrier();
    // timenet.2^T: dTH = W_T2^T dTE (K = 32) -> mask TH -> dZ_T1
    {
        uint32_t mk;
        zero_tiles(c);
        const h16x8 *A2 = a.img + (size_t)(a.tT2 + r) * KSLOT;
        gemm<1, NQB>(A2, lds, G_BG, 0, lane, c, ib, sc->ksc, MaskPre{&mk, mask_tile(MR_TH + r), lane});
        scale_tiles(c, a_inv(A2), ib);
        mask_apply(c, mk);
        tile16(a.dz, Ns, Z_T1 + 16 * r, p0, lane).store(c);
    }
}

// The dX chain for a frame-uniform t (TE_ROWS = false: every training step) as 8 waves of two n-tiles
// (k_bwd8, as k_fwd8): wave w writes dZ rows 32w .. 32w + 31 = H k-step w (one writer per k-step and
// step, 8 readers). Same arithmetic, scales, layouts and outputs as bwd_block<false, NQB>.
struct MaskPre32x2 {
    uint32_t *mk;              // [2]
    const uint32_t *word;      // n-tile 2w's word row; 2w + 1's is 64 words on
    int shift, lane;
    __device__ void operator()() const {
        mk[0] = word[lane] >> shift;
        mk[1] = word[64 + lane] >> shift;
    }
};
template <int NQB>
__device__ __forceinline__ void bwd_block8(const BwdArgs &a, h16x8 *lds, uint32_t *hwr, uint32_t *hrd, ScaleLDS *sc,
                                           int p0, int slot) {
    float *lf = reinterpret_cast<float *>(lds);
    float *stage = lf + G_BH * UG * 4;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const Flags F = make_flags(a.flags);
    const size_t Ns = a.Ns;
    const uint32_t *mwords = a.mask + (size_t)slot * 2 * F.nmask;
    auto trunk_pre = [&](uint32_t *mk, int L) {  // layer L's output tiles 2w, 2w + 1
        return MaskPre32x2{mk, mwords + (size_t)(16 * (L >> 1) + 2 * w) * 64, 16 * (L & 1), lane};
    };
    if (tid < 8) {
        hwr[tid] = 0;
        hrd[tid] = 0;
    }
    stage_dout<NQB, NTHR8>(a, lds, sc, stage, p0, tid);
    f32x4 c[2][NQB];
    float ib[NQB];
    // one chain step's epilogue: scale, relu' mask, dz stores, output scales, hand-off
    auto epilogue = [&](const h16x8 *Aw, int astride, const uint32_t (&mk)[2], int zrow, float ws, int par_in,
                        uint32_t step) {
        float my[NQB] = {};
#pragma unroll
        for (int t = 0; t < 2; t++) {
            scale_tiles(c[t], a_inv(Aw + t * astride), ib);
            mask_apply(c[t], mk[t]);
#ifndef DGS_DIAG_NOSAVE  // diagnostic only (wrong dW): the dZ chain's stores skipped
            tile16(a.dz, Ns, zrow + 16 * (2 * w + t), p0, lane).store(c[t]);
#endif
            col_absmax(c[t], my);
        }
        float so[NQB];
        chain_scales(sc, ws, par_in, NW8, so);
        col_wave_max(my);
        if (step > 0) lds_wait_ge(hrd + w, (uint32_t)NW8 * step, lds_peek(hrd + w));
#pragma unroll
        for (int q = 0; q < NQB; q++) {
            const Scale s = scale_for(so[q]);
            if (lane == 0) {
                sc->amax[step & 1][w][q] = my[q];
                sc->ksc[G_BH / 4 + w][q] = s.inv;
            }
#pragma unroll
            for (int t = 0; t < 2; t++) acc_to_lds(c[t][q], lds, G_BH, 2 * w + t, q, lane, s.s);
        }
        lds_signal(hwr + w, lane);
    };
    {  // heads^T: dH7 = W_h^T dOut (K = 32 from G) -> mask H7 -> dZ7
        uint32_t mk[2];
#pragma unroll
        for (int t = 0; t < 2; t++) zero_tiles(c[t]);
        const h16x8 *Ah = a.img + (size_t)(a.tHd + 2 * w) * KSLOT;
        gemm2<1, NQB>(Ah, KSLOT, lds, G_BG, 0, lane, c, ib, sc->ksc, trunk_pre(mk, 7));
        epilogue(Ah, KSLOT, mk, Z_L0 + 7 * 256, __uint_as_float(sc->wstat[8]), -1, 0u);
    }
#pragma unroll 1
    for (int L = 7; L >= 1; L--) {
        const uint32_t step = 8 - L;
        const int tile0 = (L == 5) ? F_H / 16 : 0;
        uint32_t mk[2];
#pragma unroll
        for (int t = 0; t < 2; t++) zero_tiles(c[t]);
        const h16x8 *Aw = a.img + (size_t)(a.tL[L] + (tile0 + 2 * w) * 8) * KSLOT;
        gemm2<8, NQB>(Aw, 8 * KSLOT, lds, G_BH, 0, lane, c, ib, sc->ksc, trunk_pre(mk, L - 1),
                      HGate{hwr, hrd, 0, step, true, lane});
        epilogue(Aw, 8 * KSLOT, mk, Z_L0 + (L - 1) * 256, __uint_as_float(sc->wstat[L]), (int)((step - 1) & 1), step);
    }
}

__global__ __launch_bounds__(NTHR8) void k_bwd8(BwdArgs a) {
    __shared__ h16x8 lds[G_BWD * UG];
    __shared__ uint32_t hwr[8], hrd[8];
    __shared__ int s_next;
    __shared__ ScaleLDS sc;
    load_wstats_bwd(a, &sc);
    for (int b = blockIdx.x;;) {
        int nx = 0;
        if (a.queue && threadIdx.x == 0) nx = queue_take(a.queue);
        if (b < a.nfull) bwd_block8<NQ>(a, lds, hwr, hrd, &sc, b * BM, b);
        else bwd_block8<1>(a, lds, hwr, hrd, &sc, a.nfull * BM + (b - a.nfull) * 16, b);
        if (!a.queue) break;
        if (threadIdx.x == 0) s_next = nx;
        __syncthreads();
        b = s_next;
        if (b >= a.nblk) break;
    }
    if (a.queue) queue_release(a.queue);
}

template <bool TE_ROWS>
__global__ __launch_bounds__(NTHR) void k_bwd(BwdArgs a) {
    __shared__ h16x8 lds[G_BWD * UG];
    __shared__ uint32_t hwr[8], hrd[8];  // dZ hand-off counters (HGate), as in k_fwd's trunk
    __shared__ int s_next;
    __shared__ ScaleLDS sc;
    load_wstats_bwd(a, &sc);
    CLK_BEGIN();
    for (int b = blockIdx.x;;) {  // persistent: as k_fwd
        int nx = 0;
        if (a.queue && threadIdx.x == 0) nx = queue_take(a.queue);
        if (b < a.nfull) bwd_block<TE_ROWS, NQ>(a, lds, hwr, hrd, &sc, b * BM, b);
        else bwd_block<TE_ROWS, 1>(a, lds, hwr, hrd, &sc, a.nfull * BM + (b - a.nfull) * 16, b);
        if (!a.queue) break;
        if (threadIdx.x == 0) s_next = nx;
        __syncthreads();
        b = s_next;
        if (b >= a.nblk) break;
    }
    if (a.queue) queue_release(a.queue);
    CLK_END(1);
}

// Timenet gradients for a frame-uniform t (DGS_MLP_UNIFORM_T). With one TIN / TH for every point,
// dL/dt_emb summed over points is S = W0[:, TE]^T gb0 + W5[:, TE]^T gb5 (gb = the layer-0 / 5 bias
// gradients = sums of dZ over points), and then
//   timenet.2: dW = S TH^T, db = S;   dZ_T1 = relu'(TH) (W_T2^T S);   timenet.0: dW = dZ_T1 TIN^T, db = dZ_T1
// — the per-point sums of the general path (time_utils.py:74-76 autograd) regrouped. TG_WG
// workgroups: each evaluates S (same order in every one: identical values) and writes the outputs
// of its TG_N rows n (the single-workgroup version was a 17 us latency chain); bitwise deterministic.
constexpr int TG_WG = 8, TG_N = 256 / TG_WG;
struct TGradArgs {
    const float *fp;
    int w0te, w5te, wT2;  // fp32 [256][32] t_emb columns of linear.0 / linear.5, [32][256] timenet.2
    const float *tc;      // k_timenet's TIN / TH
    const float *gb0, *gb5;
    float *gT0w, *gT0b, *gT2w, *gT2b;
    float *gW0, *gW5;     // linear.0 / linear.5 weight gradients: their folded t_emb columns
    int tin;
};

__global__ __launch_bounds__(1024) void k_tgrad(TGradArgs a) {
    __shared__ float S[32], th[TG_N], dz1[TG_N], Sp[32][33];
    const int j = threadIdx.x;
    const int n0 = blockIdx.x * TG_N;
    if (j < TG_N) th[j] = a.tc[TC_TH + n0 + j];
    {  // S[k]: thread (part, k) sums 16 of the 512 (n, layer) terms (a wave reads two 128-B rows of
       // the [n][32] weight images per step: coalesced), then 32 threads add the parts in order
        const int k = j & 31, part = j >> 5;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int n = part * 16 + i;  // n < 256: linear.0, else linear.5
            const float w = n < 256 ? a.fp[a.w0te + n * 32 + k] : a.fp[a.w5te + (n - 256) * 32 + k];
            const float gb = n < 256 ? a.gb0[n] : a.gb5[n - 256];
            s = fmaf(w, gb, s);
        }
        Sp[part][k] = s;
        __syncthreads();
        if (j < 32) {
            float t = 0.f;
#pragma unroll
            for (int q = 0; q < 32; q++) t += Sp[q][j];
            S[j] = t;
        }
    }
    // the folded t_emb columns 63..92 of linear.0 / linear.5: dW = gb (x) te (the dW kernel covers
    // x_emb and h only)
    for (int e = j; e < TG_N * 30; e += 1024) {
        const int n = n0 + e / 30, k = e % 30;
        const float te = a.tc[TC_TE + k];
        a.gW0[n * 93 + 63 + k] = a.gb0[n] * te;
        a.gW5[n * 349 + 63 + k] = a.gb5[n] * te;
    }
    __syncthreads();
    for (int e = j; e < 30 * TG_N; e += 1024) {
        const int k = e / TG_N, n = e % TG_N;
        a.gT2w[k * 256 + n0 + n] = S[k] * th[n];
    }
    if (blockIdx.x == 0 && j < 30) a.gT2b[j] = S[j];
    if (j < 4 * TG_N) {  // dZ_T1[n]: 4 lanes per n over 8 of the 30 (+2 zero) k terms each, then a fixed xor tree
        const int n = j >> 2, q = j & 3;
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int k = q * 8 + i;
            if (k < 30) d = fmaf(a.fp[a.wT2 + k * 256 + n0 + n], S[k], d);
        }
        d += __shfl_xor(d, 1);
        d += __shfl_xor(d, 2);
        d = th[n] > 0.f ? d : 0.f;
        if (q == 0) {
            dz1[n] = d;
            a.gT0b[n0 + n] = d;
        }
    }
    __syncthreads();
    for (int e = j; e < TG_N * a.tin; e += 1024) {  // coalesced [256][tin] outer product (this block's rows)
        const int n = e / a.tin, f = e - n * a.tin;
        a.gT0w[(n0 + n) * a.tin + f] = dz1[n] * a.tc[TC_TIN + f];
    }
}

// ------------------------------------------------------------------------------------------------
// dW = dZ X^T on split f16 (k_dws, the default dW). Per job tile (<= 256 dZ rows x 256 X rows) and
// 32-point chunk, each wave owns 32 rows of ONE operand ("private": loaded, scaled, split and kept as
// MFMA fragments in its own registers) against all rows of the other ("shared": staged by the whole
// workgroup, scaled and split once, through LDS):
//   COL (krows = 256 jobs): private = X rows 32 w..+31, shared = dZ rows (NS tiles)
//   ROW (krows <= 96 jobs): private = dZ rows 32 w..+31, shared = X rows (NS tiles)
// so every fp32 value is split exactly once per workgroup and only the shared operand makes the LDS
// round trip. The private fragments are always the A operand and the shared ones B (the 32x32x16 A and
// B lane maps are the same): a tile's MFMA output is [private row][shared row], lane i holding shared
// row i. Per chunk: split the private registers -> fragments | MFMAs on LDS buffer c & 1 with the next
// chunk's shared split (2 ds_write_b64 per float4) and loads interleaved | ONE barrier.
//   Scales (power of two, as the forward): the private operand one per (wave, chunk) from the wave's
// max over its 32 rows x 32 points; the shared operand one per (row, chunk) from the 8 lanes that stage
// the row (3 DPP steps), kept in LDS beside the planes. Lane i of a tile's output then carries ONE
// inverse scale (private x shared row i), applied when the chunk's fresh accumulator T joins the
// running sum: acc = T * s + acc (one fma per element, where the bf16x6 split had one add).
//   LDS: split planes in fragment order, unit (16 B) [split][k-step][32-row block][lane = 32 h + i]
//   (row i, points 8h..8h+7): a fragment is one conflict-free ds_read_b128 per split; 2 x 32 KiB.
//   Numerics: each tile's six products of a chunk (per k-step the two corrections, then hh) go into a
// fresh accumulator T, added to the running sum in fp32 (tools/mfma_accum_probe.hip: a long running
// MFMA C loses the low bits of small terms with a bias; within one chunk's T that loss stays below
// fp32's own rounding of T).
//   Output: ROW jobs' tiles are [dZ row][X row] (the slab's own layout, stored as before); COL jobs'
// are [X row][dZ row] and go through a per-wave LDS transpose so the slab stores stay coalesced.
// Same job plan, slab layout and k_dw_reduce as the fp32 k_dw.
// ------------------------------------------------------------------------------------------------
constexpr int DW_THREADS = 512;
constexpr int S_UNITS = NSPLIT * 2 * 8 * 64;  // 16-B units per chunk buffer
constexpr int S_NBUF = 2;
constexpr int S_RSC = WT;                     // shared-row inverse scales per buffer (floats)
constexpr int S_LDS = S_NBUF * S_UNITS * 16 + S_NBUF * S_RSC * 4;  // bytes (66 KiB)
constexpr int S_TRP = 32 * 33;                // per-wave transpose scratch (floats), after the loop
static_assert(S_LDS <= 160 * 1024 && 8 * S_TRP * 4 <= S_LDS, "dWs LDS");

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_f16((a), (b), (c), 0, 0, 0)
#ifdef DGS_DIAG_DWS_L2  // diagnostic (wrong results): every chunk re-reads the split's first chunk (L2-resident)
#define DWS_DIAG_C(c) (c0)
#else
#define DWS_DIAG_C(c) (c)
#endif

// unit of (split p, k-step ks, row block rb, point half hh, row i): each 32-unit half is rotated
// by 4 ks + 2 hh, so the row-major staging stores (8 lanes per row: all (ks, hh, 8-byte half)
// combinations of 2 rows per 16-lane group) hit 32 distinct banks; a fragment read stays one
// conflict-free 1 KiB ds_read_b128
__device__ __forceinline__ constexpr int s_unit(int p, int ks, int rb, int hh, int i) {
    return ((p * 2 + ks) * 8 + rb) * 64 + 32 * hh + ((i + 4 * ks + 2 * hh) & 31);
}

__device__ __forceinline__ AFrag s_frag(const h16x8 *L, int ks, int rb, int lane) {
    const int hh = lane >> 5, i = lane & 31;
    return AFrag{L[s_unit(0, ks, rb, hh, i)], L[s_unit(1, ks, rb, hh, i)]};
}

// 8 fp32 (one row, points 8h .. 8h + 7) times S -> the hi / lo f16 fragments
__device__ __forceinline__ AFrag split8(const float4 &a, const float4 &b, float S) {
    uint32_t h[4], l[4];
    hsplit2(a.x * S, a.y * S, h[0], l[0]);
    hsplit2(a.z * S, a.w * S, h[1], l[1]);
    hsplit2(b.x * S, b.y * S, h[2], l[2]);
    hsplit2(b.z * S, b.w * S, h[3], l[3]);
    return AFrag{__builtin_bit_cast(h16x8, make_uint4(h[0], h[1], h[2], h[3])),
                 __builtin_bit_cast(h16x8, make_uint4(l[0], l[1], l[2], l[3]))};
}

__device__ __forceinline__ float sum8(const float4 &a, const float4 &b) {
    return ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
}

__device__ __forceinline__ float absmax4(const float4 &v) {
    return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}

// one k-step's three products into t (the two corrections first)
__device__ __forceinline__ f32x16 mma3_into(const AFrag &a, const AFrag &b, f32x16 t) {
    t = MFMA32(a.l, b.h, t);
    t = MFMA32(a.h, b.l, t);
    return MFMA32(a.h, b.h, t);
}

// max over the 8 consecutive lanes (aligned groups) of non-negative floats, in every lane of the group:
// quad_perm [1,0,3,2], [2,3,0,1], then row_half_mirror
__device__ __forceinline__ float max8(float v) {
    uint32_t x = __float_as_uint(v);
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xb1, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4e, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xf, 0xf, false));
    return __uint_as_float(x);
}

template <bool COL, int NS>
__device__ __forceinline__ void dws_run(const WJob &J, size_t Ns, const float *__restrict__ dz,
                                        const float *__restrict__ saved, float *__restrict__ slabs, h16x8 *lds) {
    constexpr int SROWS = 32 * NS;                   // shared rows staged per chunk
    constexpr int NSF = (SROWS * 8 + 511) / 512;     // staged float4 per thread per chunk
    const int split = blockIdx.x - J.block0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5, i = lane & 31;
    const int nch = (int)(Ns / 32);
    const int per = div_up(nch, J.nsplit);
    const int c0 = split * per;
    const int c1 = min(nch, c0 + per);
    // operands through buffer descriptors whose record count ends at the job's extent: rows past
    // it read as zero (32-bit offsets: the host keeps 256 rows x Ns x 4 B below 2^31)
    const float *zb = dz + (size_t)J.zrow * Ns, *xb = saved + (size_t)J.xrow * Ns;
    const __amdgpu_buffer_rsrc_t rsS = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(COL ? zb : xb), 0, (int)((COL ? J.nrows : J.krows) * Ns * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsP = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(COL ? xb : zb), 0, (int)((COL ? J.krows : J.nrows) * Ns * 4), 0x00020000);
    const bool pact = 32 * wave < (COL ? J.krows : J.nrows);  // this wave has private rows (uniform)
    // private: lane (i, h) holds row 32 w + i, points 8 h .. + 7 of each k-step (fragment layout)
#ifdef DGS_DIAG_DWS_TILED  // diagnostic (wrong results): chunk-major addressing [chunk][row][32 points]
    const int pvoff = ((32 * wave + i) * 32 + 8 * h) * 4;
    const int pcst = (COL ? J.krows : J.nrows) * 128, scst = (COL ? J.nrows : J.krows) * 128;
#else
    const int pvoff = ((32 * wave + i) * (int)Ns + 8 * h) * 4;
    constexpr int pcst = 128, scst = 128;
#endif
    float4 pr[4];  // [k-step][half]
    auto pload = [&](int c) {
#pragma unroll
        for (int q = 0; q < 4; q++)
            pr[q] = __builtin_bit_cast(float4,
                                       __builtin_amdgcn_raw_buffer_load_b128(rsP, pvoff, DWS_DIAG_C(c) * pcst + (q >> 1) * 64 + (q & 1) * 16, 0));
    };
    // shared staging: slot g = tid + 512 f -> row g >> 3, points 4 (g & 7) .. + 3 of the chunk (8
    // lanes read a row's 128 B)
    float4 st[NSF];
    auto sslot = [&](int f, int &row, int &q) {
        const int g = tid + 512 * f;
        row = g >> 3;
        q = g & 7;
        return SROWS * 8 % 512 == 0 || g < SROWS * 8;
    };
    auto sload = [&](int c) {
#pragma unroll
        for (int f = 0; f < NSF; f++) {
            int row, q;
            if (sslot(f, row, q))
                st[f] = __builtin_bit_cast(
#ifdef DGS_DIAG_DWS_TILED
                    float4, __builtin_amdgcn_raw_buffer_load_b128(rsS, (row * 32 + 4 * q) * 4, DWS_DIAG_C(c) * scst, 0));
#else
                    float4, __builtin_amdgcn_raw_buffer_load_b128(rsS, (row * (int)Ns + 4 * q) * 4, DWS_DIAG_C(c) * scst, 0));
#endif
        }
    };
    float bsum[NSF] = {};  // COL: bias row sums of the staged dZ rows; ROW: bsum[0] of the private row
    char *lb = reinterpret_cast<char *>(lds);
    float *rsc = reinterpret_cast<float *>(lb + S_NBUF * S_UNITS * 16);  // [buffer][row]
    // `live`: the staged chunk is a real one (the last chunk re-splits a stale copy into the buffer
    // nobody reads again; it must not count in the bias sums)
    auto sput = [&](int f, int buf, bool live) {
        int row, q;
        const bool ok = sslot(f, row, q);
        const float4 v = st[f];
        // the row's scale: max over its 8 staging lanes (a partial last slot group lies in one wave, past
        // the valid rows: its lanes see zeros, never a valid row's)
#ifdef DGS_DIAG_DWS_NOSCALE  // diagnostic (wrong results): constant scales, no per-chunk maxima
        const Scale s = Scale{1024.f, 1.f / 1024.f};
#else
        const Scale s = scale_for(max8(ok ? absmax4(v) : 0.f));
#endif
        if (!ok) return;
        if (COL) bsum[f] += live ? (v.x + v.y) + (v.z + v.w) : 0.f;
        const Split4 sp = split4(v.x, v.y, v.z, v.w, s.s);
        char *p = lb + buf * (S_UNITS * 16) +
                  s_unit(0, q >> 2, row >> 5, (q >> 1) & 1, row & 31) * 16 + 8 * (q & 1);
        *reinterpret_cast<h16x4 *>(p) = sp.h;
        *reinterpret_cast<h16x4 *>(p + 2 * 8 * 64 * 16) = sp.l;
        // the row's 8 lanes store the same value (a `q == 0` branch here split the block and cost 72
        // VGPRs of spills)
        rsc[buf * S_RSC + row] = s.inv;
    };
    f32x16 acc[NS];
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
        for (int r = 0; r < 16; r++) acc[s][r] = 0.f;
    if (c0 < c1) {
        sload(c0);
        pload(c0);
#pragma unroll
        for (int f = 0; f < NSF; f++) sput(f, 0, true);
        sload(min(c0 + 1, c1 - 1));
    }
    lds_barrier();
    // shared float4 f of the next chunk is split after tile put_at(f) of this one (within the first
    // half of the tiles), then the loads of the chunk after are issued
    constexpr int NH = (NS + 1) / 2;
    auto put_at = [](int f) { return (f * NH) / NSF; };
    auto chunk = [&](int c, auto BUFC) {
        constexpr int buf = decltype(BUFC)::value;
        const h16x8 *L = lds + buf * S_UNITS;
        const bool more = c + 1 < c1;
        if (pact) {
            // private fragments of this chunk (scaled by the wave's max), then the private loads of
            // the next (in flight for the whole chunk)
#ifdef DGS_DIAG_DWS_NOSCALE
            const Scale sp = Scale{1024.f, 1.f / 1024.f};
#else
            const float pm = wave_max(fmaxf(fmaxf(absmax4(pr[0]), absmax4(pr[1])), fmaxf(absmax4(pr[2]), absmax4(pr[3]))));
            const Scale sp = scale_for(pm);
#endif
            AFrag pf0 = split8(pr[0], pr[1], sp.s), pf1 = split8(pr[2], pr[3], sp.s);
            if (!COL) bsum[0] += sum8(pr[0], pr[1]) + sum8(pr[2], pr[3]);
            pload(min(c + 1, c1 - 1));
#pragma unroll
            for (int s = 0; s < NS; s++) {
                // the tile's two k-steps into a fresh accumulator, one shared fragment live at a time
                const float si = sp.inv * rsc[buf * S_RSC + 32 * s + i];
                const AFrag s0 = s_frag(L, 0, s, lane);
#ifdef DGS_DIAG_DWS_NOFOLD  // diagnostic (wrong results): the MFMAs accumulate into acc directly
                acc[s] = mma3_into(pf0, s0, acc[s]);
                const AFrag s1 = s_frag(L, 1, s, lane);
                acc[s] = mma3_into(pf1, s1, acc[s]);
                (void)si;
#else
                f32x16 T = mma3_into(pf0, s0, (f32x16)(0.f));
                const AFrag s1 = s_frag(L, 1, s, lane);
                T = mma3_into(pf1, s1, T);
#pragma unroll
                for (int r = 0; r < 16; r++) acc[s][r] = fmaf(T[r], si, acc[s][r]);
#endif
#pragma unroll
                for (int f = 0; f < NSF; f++)
                    if (put_at(f) == s) sput(f, buf ^ 1, more);
                if (s == put_at(NSF - 1)) sload(min(c + 2, c1 - 1));
            }
        } else {
            pload(min(c + 1, c1 - 1));  // (keeps the waves' vmcnt streams alike; reads row 0 + OOB zeros)
#pragma unroll
            for (int f = 0; f < NSF; f++) sput(f, buf ^ 1, more);
            sload(min(c + 2, c1 - 1));
        }
        lds_barrier();
    };
    for (int c = c0; c < c1; c += 2) {
        chunk(c, std::integral_constant<int, 0>{});
        if (c + 1 < c1) chunk(c + 1, std::integral_constant<int, 1>{});
    }
    float *slab = slabs + (size_t)blockIdx.x * SLAB;
    if (COL) {
        // bias row sums: the 8 lanes staging a row hold its partial sums (fixed xor-tree order)
#pragma unroll
        for (int f = 0; f < NSF; f++) {
            float v = bsum[f];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            int row, q;
            if (sslot(f, row, q) && q == 0) slab[WT * WT + row] = v;
        }
    } else if (pact) {
        const float v = bsum[0] + __shfl_xor(bsum[0], 32);
        if (h == 0) slab[WT * WT + 32 * wave + i] = v;
    }
    if (!pact) return;
    // rows past nrows / cols past krows hold zeros that k_dw_reduce never reads
    if (!COL) {
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int nb = 32 * wave, kb = 32 * s;
#pragma unroll
            for (int r = 0; r < 16; r++) slab[(nb + TileAddr::row(r) + 4 * h) * WT + kb + i] = acc[s][r];
        }
        return;
    }
    // COL: tile s is [X row 32 w + row(r) + 4 h][dZ row 32 s + i]; through this wave's LDS scratch so
    // that 32 lanes store 32 consecutive X rows of one dZ row (the last chunk's barrier ended every
    // wave's reads of the planes)
    float *tp = reinterpret_cast<float *>(lds) + wave * S_TRP;
#pragma unroll
    for (int s = 0; s < NS; s++) {
#pragma unroll
        for (int r = 0; r < 16; r++) tp[i * 33 + TileAddr::row(r) + 4 * h] = acc[s][r];
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes before its reads
#pragma unroll
        for (int rr = 0; rr < 16; rr++) {
            const int m = 2 * rr + h;  // dZ row 32 s + m, X rows 32 w + i
            slab[(32 * s + m) * WT + 32 * wave + i] = tp[m * 33 + i];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // the reads done before the next tile's writes
    }
}

__global__ __launch_bounds__(DW_THREADS) void k_dws(WJobs JT, size_t Ns, const float *__restrict__ dz,
                                                    const float *__restrict__ saved, float *__restrict__ slabs) {
    extern __shared__ h16x8 dws_lds[];
    WJob J = JT.j[0];
#pragma unroll
    for (int q = 1; q < MAXJ; q++)
        if (q < JT.n && (int)blockIdx.x >= JT.j[q].block0) J = JT.j[q];
    // job shapes (host-checked in dw_split_once): krows = 256 with nrows 256 or 32 -> COL; nrows =
    // 256 with krows 96, 64 (folded t_emb) or 16 -> ROW
    CLK_BEGIN();
    if (J.krows == 256) {
        if (J.nrows == 256)
            dws_run<true, 8>(J, Ns, dz, saved, slabs, dws_lds);
        else
            dws_run<true, 1>(J, Ns, dz, saved, slabs, dws_lds);
    } else if (J.krows > 64) {
        dws_run<false, 3>(J, Ns, dz, saved, slabs, dws_lds);
    } else if (J.krows > 32) {
        dws_run<false, 2>(J, Ns, dz, saved, slabs, dws_lds);
    } else {
        dws_run<false, 1>(J, Ns, dz, saved, slabs, dws_lds);
    }
    CLK_END(2);
}

// ------------------------------------------------------------------------------------------------
// packing plan (host)
// ------------------------------------------------------------------------------------------------
struct Img {           // one A-operand image: ntiles x nk k-slots
    int src;           // parameter index (weight)
    int transpose;     // 0: A[n][f] = W[n][f]; 1: A[n][f] = W[f][n]
    int ntiles, nk;
    int nseg_n, nseg_f;
    Seg segn[3], segf[3];
    int slot;          // first k-slot
};
struct F32Job {        // fp32 region entry: dst[r * cpad + c] = W[sr][sc] (bias: cpad = 1)
    int src;
    int rpad, cpad;
    int nseg_r, nseg_c;
    Seg segr[3], segc[3];
    int off;
};

struct Plan : Params {
    Flags F;
    std::vector<Img> imgs;
    std::vector<F32Job> f32;
    int fT1 = -1, fT2 = -1, fL[8], fHd, tHd, tL[8], tT2 = -1;  // k-slots
    int bT1 = -1, bT2 = -1, bL[8], bHd, wT1 = -1, wT2 = -1;     // fp32 offsets
    int w0te = -1, w5te = -1;                                    // fp32 t_emb columns of linear.0 / .5
    int nslots = 0, nf32 = 0;
    std::vector<int> units;  // k_pack's workgroups: (first k-slot, k-slots) of every 16-row n-tile
    size_t img_floats() const { return (size_t)nslots * KSLOT * 4; }  // 16-B unit = 4 floats
    size_t total() const { return img_floats() + nf32; }
};

Plan make_plan(int flags) {
    Plan P;
    P.F = make_flags(flags);
    const Flags &F = P.F;
    static_cast<Params &>(P) = make_params(F);
    auto img = [&](int src, int tr, int ntiles, int nk, int nsn, const Seg *sn, int nsf, const Seg *sf, int slot) {
        Img j{};
        j.src = src; j.transpose = tr; j.ntiles = ntiles; j.nk = nk; j.nseg_n = nsn; j.nseg_f = nsf;
        for (int q = 0; q < nsn; q++) j.segn[q] = sn[q];
        for (int q = 0; q < nsf; q++) j.segf[q] = sf[q];
        j.slot = slot;
        P.imgs.push_back(j);
    };
    auto new_img = [&](int src, int tr, int ntiles, int nk, int nsn, const Seg *sn, int nsf, const Seg *sf) {
        const int slot = P.nslots;
        img(src, tr, ntiles, nk, nsn, sn, nsf, sf, slot);
        P.nslots += ntiles * nk;
        return slot;
    };
    auto f32 = [&](int src, int rpad, int cpad, int nsr, const Seg *sr, int nsc, const Seg *sc, int off) {
        F32Job j{};
        j.src = src; j.rpad = rpad; j.cpad = cpad; j.nseg_r = nsr; j.nseg_c = nsc;
        for (int q = 0; q < nsr; q++) j.segr[q] = sr[q];
        for (int q = 0; q < nsc; q++) j.segc[q] = sc[q];
        j.off = off;
        P.f32.push_back(j);
    };
    auto new_f32 = [&](int src, int rpad, int cpad, int nsr, const Seg *sr, int nsc, const Seg *sc) {
        const int off = P.nf32;
        f32(src, rpad, cpad, nsr, sr, nsc, sc, off);
        P.nf32 += rpad * cpad;
        return off;
    };
    const Seg full = seg(0, 256, 0), one = seg(0, 1, 0);
    if (F.blender) {
        const Seg st = seg(0, F.tin, 0), s30 = seg(0, 30, 0);
        P.fT1 = new_img(P.pT0w, 0, 16, 1, 1, &full, 1, &st);   // K = TIN (13) padded to one k-step
        P.fT2 = new_img(P.pT2w, 0, 2, 8, 1, &s30, 1, &full);
        P.tT2 = new_img(P.pT2w, 1, 16, 1, 1, &full, 1, &s30);  // A[n = TH feature][f = TE feature]
        P.bT1 = new_f32(P.pT0b, 256, 1, 1, &full, 1, &one);
        P.bT2 = new_f32(P.pT2b, 32, 1, 1, &s30, 1, &one);
        P.wT1 = new_f32(P.pT0w, 256, 16, 1, &full, 1, &st);
        P.wT2 = new_f32(P.pT2w, 32, 256, 1, &s30, 1, &full);
        const Seg te0 = seg(0, 30, 63);  // linear.0 / linear.5 columns 63..92 = t_emb (layer_in_segs)
        P.w0te = new_f32(P.pLw[0], 256, 32, 1, &full, 1, &te0);
        P.w5te = new_f32(P.pLw[5], 256, 32, 1, &full, 1, &te0);
    }
    for (int i = 0; i < 8; i++) {
        Seg s[3], sf[3];
        const int ns = layer_in_segs(F, i, s);             // forward: t_emb folded with a uniform t
        const int nsf = layer_in_segs(F, i, sf, false);    // backward: the full padded input
        P.fL[i] = new_img(P.pLw[i], 0, 16, layer_kpad_f(F, i) / 32, 1, &full, ns, s);
        P.tL[i] = new_img(P.pLw[i], 1, layer_kpad(i) / 16, 8, nsf, sf, 1, &full);  // rows = padded input features
        P.bL[i] = new_f32(P.pLb[i], 256, 1, 1, &full, 1, &one);
    }
    // heads: rows stacked in output order (nout <= 13) in one 16-row image each way
    P.fHd = P.nslots;
    P.nslots += 8;   // 1 n-tile x 8 k-steps
    P.tHd = P.nslots;
    P.nslots += 16;  // 16 n-tiles x 1 k-step (K = head rows padded to 32)
    P.bHd = P.nf32;
    P.nf32 += 32;
    int r0 = 0;
    for (int h = 0; h < P.nheads; h++) {
        const Seg sr = seg(r0, P.hrows[h], 0);
        img(P.pHw[h], 0, 1, 8, 1, &sr, 1, &full, P.fHd);
        img(P.pHw[h], 1, 16, 1, 1, &full, 1, &sr, P.tHd);
        f32(P.pHb[h], 32, 1, 1, &sr, 1, &one, P.bHd);
        r0 += P.hrows[h];
    }
    P.nf32 = (P.nf32 + 3) & ~3;
    // one pack workgroup per n-tile of every image region (its scale and row statistics span the tile's
    // whole K): the region list is fixed by the flags
    auto region = [&](int slot0, int ntiles, int nk) {
        assert(nk <= PACK_MAXK);
        for (int t = 0; t < ntiles; t++) {
            P.units.push_back(slot0 + t * nk);
            P.units.push_back(nk);
        }
    };
    if (F.blender) {
        region(P.fT1, 16, 1);
        region(P.fT2, 2, 8);
        region(P.tT2, 16, 1);
    }
    for (int i = 0; i < 8; i++) {
        region(P.fL[i], 16, layer_kpad_f(F, i) / 32);
        region(P.tL[i], layer_kpad(i) / 16, 8);
    }
    region(P.fHd, 1, 8);
    region(P.tHd, 16, 1);
    return P;
}

// Packing is one gather + scale + split launch over map[i] = (parameter << 22) | element, or -1 for
// zero padding: i < nslots * 512 are the A-image elements in [k-slot][lane][8] order, the rest the
// fp32 region. The map depends only on the flags (built once on the host, cached on the device).
// Workgroup b < nunits packs one 16-row n-tile (its k-slots slot0 .. slot0 + nk - 1): the tile's max
// |w| sets its power-of-two scale S (scale_for), each element x is stored as hi = f16(S x) and lo =
// f16(S x - hi) in the slot's first two planes, and the third plane of the tile's first slot holds
// [1 / S, max over the tile's 16 rows of sum_k |w|] (the output-scale bounds of the forward / dX
// kernels); the other workgroups copy the fp32 region.
constexpr int PACK_MAXP = 32;
constexpr int PACK_SHIFT = 22;
struct PackPtrs {
    const float *p[PACK_MAXP];
};

__global__ __launch_bounds__(512) void k_pack(const int *__restrict__ map, PackPtrs src, const int2 *__restrict__ units,
                                              int nunits, _Float16 *__restrict__ img, float *__restrict__ fp, int nimg,
                                              int nf32) {
    __shared__ float s_rs[4][16];
    __shared__ uint32_t s_max;
    const int b = blockIdx.x, tid = threadIdx.x;
    auto gather = [&](int i) {
        const int c = map[i];
        return c < 0 ? 0.f : src.p[c >> PACK_SHIFT][c & ((1 << PACK_SHIFT) - 1)];
    };
    if (b >= nunits) {
        const int j = (b - nunits) * 512 + tid;
        if (j < nf32) fp[j] = gather(nimg + j);
        return;
    }
    const int2 u = units[b];  // (first k-slot, k-slots <= PACK_MAXK)
    if (tid == 0) s_max = 0;
    // element tid of a slot: lane l = tid >> 3 holds row l & 15 of the tile (v_mfma_f32_16x16x32_f16 A map);
    // the tile's values stay in registers between the statistics and the split: one gather each, all
    // in flight at once (the rolled loops made 2 x k-slots dependent map -> parameter round trips)
    float v[PACK_MAXK];
    float am = 0.f, rs = 0.f;
#pragma unroll
    for (int k = 0; k < PACK_MAXK; k++) {
        v[k] = k < u.y ? gather((u.x + k) * 512 + tid) : 0.f;
        am = fmaxf(am, fabsf(v[k]));
        rs += fabsf(v[k]);
    }
    rs += __shfl_xor(rs, 1);  // the 8 elements of a lane (tid bits 0-2): same row
    rs += __shfl_xor(rs, 2);
    rs += __shfl_xor(rs, 4);
    __syncthreads();
    am = wave_max(am);
    if ((tid & 63) == 0) lds_fmax(&s_max, am);
    if ((tid & 7) == 0) s_rs[tid >> 7][(tid >> 3) & 15] = rs;  // tid bits 7-8: the four k quarters
    __syncthreads();
    const Scale S = scale_for(__uint_as_float(s_max));
#pragma unroll
    for (int k = 0; k < PACK_MAXK; k++) {
        if (k >= u.y) break;
        const float x = v[k] * S.s;
        const _Float16 hi = (_Float16)x;
        const _Float16 lo = (_Float16)(x - (float)hi);
        _Float16 *d = img + (size_t)(u.x + k) * 1536 + tid;  // k-slot: hi, lo, scale plane of 512 f16
        d[0] = hi;
        d[512] = lo;
    }
    if (tid == 0) {
        float m = 0.f;
        for (int r = 0; r < 16; r++) m = fmaxf(m, (s_rs[0][r] + s_rs[1][r]) + (s_rs[2][r] + s_rs[3][r]));
        float *t = reinterpret_cast<float *>(img + (size_t)u.x * 1536 + 1024);
        t[0] = S.inv;
        t[1] = m;
    }
}

static std::vector<int> build_pack_map(const Plan &P) {
    const size_t nimg = (size_t)P.nslots * 512;
    std::vector<int> map(nimg + P.nf32, -1);
    for (const Img &j : P.imgs) {
        int r, c;
        param_shape(P.F, P, j.src, r, c);
        for (int idx = 0; idx < j.ntiles * j.nk * 512; idx++) {
            const int e = idx & 7, lane = (idx >> 3) & 63, slot = idx >> 9;
            const int k = slot % j.nk, ntile = slot / j.nk;
            const int n = ntile * 16 + (lane & 15);  // v_mfma_f32_16x16x32_bf16 A map
            const int f = 32 * k + 8 * (lane >> 4) + e;
            const int sn = seg_lookup(j.segn, j.nseg_n, n);
            const int sf = seg_lookup(j.segf, j.nseg_f, f);
            if (sn >= 0 && sf >= 0)
                map[(size_t)j.slot * 512 + idx] = (j.src << PACK_SHIFT) | (j.transpose ? sf * c + sn : sn * c + sf);
        }
    }
    for (const F32Job &j : P.f32) {
        int r, c;
        param_shape(P.F, P, j.src, r, c);
        for (int rr = 0; rr < j.rpad; rr++)
            for (int cc = 0; cc < j.cpad; cc++) {
                const int sr = seg_lookup(j.segr, j.nseg_r, rr), sc = seg_lookup(j.segc, j.nseg_c, cc);
                if (sr >= 0 && sc >= 0) map[nimg + j.off + rr * j.cpad + cc] = (j.src << PACK_SHIFT) | (c ? sr * c + sc : sr);
            }
    }
    return map;
}

static std::mutex g_map_mu;
static std::map<std::pair<int, int>, int *> g_pack_maps;  // (device, flags) -> device map
static std::map<std::pair<int, int>, int2 *> g_pack_units;  // (device, flags) -> n-tile table

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

static const int2 *pack_units_for(const Plan &P, int flags) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_map_mu);
    auto it = g_pack_units.find({dev, flags});
    if (it != g_pack_units.end()) return it->second;
    int2 *d = nullptr;
    const size_t bytes = P.units.size() * sizeof(int);
    if (hipMalloc(&d, bytes) != hipSuccess) return nullptr;
    if (hipMemcpy(d, P.units.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return nullptr;
    }
    g_pack_units[{dev, flags}] = d;
    return d;
}

// dW split plan: one 8-wave workgroup per CU (LDS 144 KiB); per-chunk cost in MFMA tiles + staging
// k_dws per-chunk cost by job shape (dw_shape: COL 256x256, COL 32-row head, ROW 96-col, ROW 16-col,
// ROW 64-col),
// relative to the full tile, from the per-workgroup durations of tools/mlp_clock.py at 100k points
// (profiles/r3p_mlp_clock_before.json: a full-tile chunk 4.5 us, a 96-col chunk 2.6 us, a head chunk
// 1.5 us; the MFMA-tile model gave the narrow jobs too few workgroups, which then finished 25 % after
// the rest. With these costs every job's workgroups end within 4 %: profiles/r3p_mlp_clock.json)
// (the folded t_emb's 64-column ROW shape: 1.89 us per chunk vs 4.64 for a full tile, the head 1.59:
// profiles/r3s_mlp_clock_fold.json)
static const double kDwsShapeCost[5] = {1.0, 0.34, 0.58, 0.30, 0.41};
// target: workgroups of the plan (256, one per CU; the slab scratch is sized for it; fewer with
// reserved CUs)
static WPlan split_wplan(const Flags &F, int target = 256) {
    static const bool model = [] {  // A/B only: the MFMA-tile cost model
        const char *e = getenv("DGS_DWS_TILE_MODEL");
        return e && *e == '1';
    }();
    return make_wplan(F, target, 1.5, 4.0, model ? nullptr : kDwsShapeCost);
}


static size_t padded_points(int N) { return (size_t)div_up(N, BM) * BM; }

// Block decomposition of the fused forward / dX kernels (one 147 KB workgroup per CU): when the last
// round of 64-point blocks would occupy at most a quarter of the CUs, those blocks run as four times
// as many 16-point blocks instead (fwd_block / bwd_block NQB = 1), so the sparse last round ends in
// roughly a third of a full block's time (the A stream, not the MFMAs, bounds a 16-point block).
// DGS_MLP_NO_TAIL=1 keeps 64-point blocks throughout. Mask slots: one per block (<= nb + 3 min(nb, 128)).
constexpr int TAIL_MAX_LAST = 128;
struct Blocks {
    int nfull, ntail;
};
static int cu_count() {
    static std::mutex mu;
    static std::map<int, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cache[dev] = v;
    return v;
}
// CUs the MLP kernels leave free for concurrent work (the data-parallel step's gradient all-reduce runs
// on its own stream under the network backward): the persistent k_fwd / k_bwd grids
// launch cu_count() - reserve workgroups (one per CU) and k_dws's plan spans 256 - reserve workgroups.
// dgs_mlp_set_reserved_cus / DGS_MLP_RESERVE_CUS; default 0.
static std::atomic<int> g_reserve_cus{-1};
static int reserved_cus() {
    int v = g_reserve_cus.load();
    if (v < 0) {
        const char *e = getenv("DGS_MLP_RESERVE_CUS");
        int want = e ? atoi(e) : 0;
        want = want < 0 ? 0 : want > 64 ? 64 : want;
        g_reserve_cus.compare_exchange_strong(v, want);
        v = g_reserve_cus.load();
    }
    return v;
}
static int mlp_cus() { return std::max(1, cu_count() - reserved_cus()); }
static Blocks block_split(int N) {
    const int nb = div_up(N, BM);
    static const bool off = [] {
        const char *e = getenv("DGS_MLP_NO_TAIL");
        return e && e[0] == '1';
    }();
    if (off || nb == 0) return {nb, 0};
    const int ncu = mlp_cus();
    const int rounds = div_up(nb, ncu), last = nb - ncu * (rounds - 1);
    if (rounds < 2 || last > TAIL_MAX_LAST || 4 * last > ncu) return {nb, 0};
    return {nb - last, 4 * last};
}
// Block-queue counters of the persistent k_fwd / k_bwd, one zeroed pair per (device, stream, kernel)
// (two launches in flight on two streams must not share one). DGS_MLP_STATIC=1: one launch block per
// block, no queue (A/B).
static uint32_t *block_queue(hipStream_t stream, int kernel) {
    static const bool off = [] {
        const char *e = getenv("DGS_MLP_STATIC");
        return e && e[0] == '1';
    }();
    if (off) return nullptr;
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, uint32_t *> words;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    uint32_t *&w = words[{dev, stream}];
    if (!w) {
        if (hipMalloc(&w, 4 * sizeof(uint32_t)) != hipSuccess) {
            w = nullptr;
            return nullptr;
        }
        if (hipMemset(w, 0, 4 * sizeof(uint32_t)) != hipSuccess) return nullptr;
    }
    return w + 2 * kernel;
}
// k_timenet's output for a forward without saved activations (inference with a uniform t), one
// TC_FLOATS buffer per (device, stream)
static float *timenet_scratch(hipStream_t stream) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, float *> bufs;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    float *&b = bufs[{dev, stream}];
    if (!b && hipMalloc(&b, TC_FLOATS * sizeof(float)) != hipSuccess) b = nullptr;
    return b;
}
static int persistent_grid(int nblk, const uint32_t *queue) { return queue ? std::min(nblk, mlp_cus()) : nblk; }

static size_t mask_words(const Flags &F, size_t Ns) {
    const size_t nb = Ns / BM;
    return (size_t)F.nmask * 2 * (nb + 3 * std::min<size_t>(nb, TAIL_MAX_LAST));
}

size_t saved_floats(int flags, int N) {
    const Flags F = make_flags(flags);
    const size_t Ns = padded_points(N);
    return (size_t)F.nsaved * Ns + mask_words(F, Ns) + TC_FLOATS;
}

// dW arithmetic (DGS_MLP_SPLIT_DW): 3 (default) = the split-f16 k_dws (private / shared operands, every
// value split once), 0 = the fp32-input MFMA k_dw of mlp.hip, both on the same [rows][Ns] arrays (the
// bf16 k_dw / k_dwg variants, modes 1 and 2, were removed with the bf16x6 arithmetic in round 6)
static int dw_mode() {
    static const int m = [] {
        const char *e = getenv("DGS_MLP_SPLIT_DW");
        return (e && e[0] == '0') ? 0 : 3;
    }();
    return m;
}
static int dw_split_once(const Flags &F, size_t Ns, const float *dz, const float *saved, float *slabs,
                         float *const *grads, hipStream_t stream);

size_t scratch_floats(int flags, int N) {
    const Flags F = make_flags(flags);
    const size_t slabs = std::max((size_t)split_wplan(F).nblocks * SLAB, mlp::dw_fp32_slab_floats(flags));
    return (size_t)F.nz * padded_points(N) + slabs;
}

int pack(int flags, const float *const *params, float *packed, hipStream_t stream) {
    const Plan P = make_plan(flags);
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
    const int2 *units = pack_units_for(P, flags);
    if (!map || !units) {
        set_error("dgs_deform_pack: could not allocate the pack map");
        return DGS_ERR_HIP;
    }
    const int nimg = P.nslots * 512, nunits = (int)P.units.size() / 2;
    hipLaunchKernelGGL(k_pack, dim3(nunits + div_up(P.nf32, 512)), dim3(512), 0, stream, map, src, units, nunits,
                       reinterpret_cast<_Float16 *>(packed), packed + P.img_floats(), nimg, P.nf32);
    DGS_LAUNCH_CHECK("k_pack", false, stream);
    return DGS_OK;
}

static void fwd_args(const Plan &P, int flags, int N, const float *xyz, const float *t, const float *packed, float *out,
                     float *saved, FwdArgs &a, hipStream_t stream);

int forward(int flags, int N, const float *xyz, const float *t, const float *packed, float *out, float *saved,
            hipStream_t stream) {
    const Plan P = make_plan(flags);
    FwdArgs a{};
    fwd_args(P, flags, N, xyz, t, packed, out, saved, a, stream);
    const int grid = persistent_grid(a.nblk, a.queue);
    if (P.F.blender && (saved || P.F.uniform_t)) {
        // the folded biases (uniform t) are needed without saved activations too (inference)
        if (!a.tc) {
            set_error("dgs_deform_forward: could not allocate the timenet scratch");
            return DGS_ERR_HIP;
        }
        hipLaunchKernelGGL(k_timenet, dim3(1), dim3(256), 0, stream, a);
    }
    {
        ScopedTimer tm("mlp_fwd", stream);  // k_fwd only: the class's FLOP count is the trunk's + heads'
        const bool fold = P.F.uniform_t;  // t_emb folded into the biases (a.tc is set above)
        static const bool fwd8 = [] {  // DGS_MLP_FWD8=0: the 16-wave k_fwd (A/B)
            const char *e = getenv("DGS_MLP_FWD8");
            return !(e && e[0] == '0');
        }();
        if (saved && fold && fwd8)
            hipLaunchKernelGGL(k_fwd8, dim3(grid), dim3(NTHR8), 0, stream, a);
        else if (saved && fold)
            hipLaunchKernelGGL((k_fwd<true, true>), dim3(grid), dim3(NTHR), 0, stream, a);
        else if (saved)
            hipLaunchKernelGGL((k_fwd<true, false>), dim3(grid), dim3(NTHR), 0, stream, a);
        else if (fold)
            hipLaunchKernelGGL((k_fwd<false, true>), dim3(grid), dim3(NTHR), 0, stream, a);
        else
            hipLaunchKernelGGL((k_fwd<false, false>), dim3(grid), dim3(NTHR), 0, stream, a);
    }
    DGS_LAUNCH_CHECK("k_fwd", false, stream);
    return DGS_OK;
}

// The training step's pack + forward: pack() then forward() (k_pack, k_timenet, k_fwd). Round 5 tried
// the timenet inside the pack launch (one extra workgroup gathering its weights through the pack map):
// 59 us for that launch against 9 + 7 us for the two (rocprofv3, profiles/r5b_pack_tn_regression.txt;
// the map double-indirection serialised the timenet's loads and its registers lowered the pack's
// occupancy), so the two launches stay.
int pack_forward(int flags, const float *const *params, int N, const float *xyz, const float *t, float *packed,
                 float *out, float *saved, hipStream_t stream) {
    if (int rc = pack(flags, params, packed, stream)) return rc;
    return forward(flags, N, xyz, t, packed, out, saved, stream);
}

static void fwd_args(const Plan &P, int flags, int N, const float *xyz, const float *t, const float *packed, float *out,
                     float *saved, FwdArgs &a, hipStream_t stream) {
    a.N = N;
    a.Ns = padded_points(N);
    a.xyz = xyz; a.t = t; a.out = out; a.saved = saved;
    a.img = reinterpret_cast<const h16x8 *>(packed);
    a.fp = packed + P.img_floats();
    a.mask = saved ? reinterpret_cast<uint32_t *>(saved + (size_t)P.F.nsaved * a.Ns) : nullptr;
    a.fT1 = P.fT1; a.fT2 = P.fT2; a.fHd = P.fHd;
    a.bT1 = P.bT1; a.bT2 = P.bT2; a.bHd = P.bHd; a.wT1 = P.wT1; a.wT2 = P.wT2;
    a.w0te = P.w0te; a.w5te = P.w5te;
    for (int i = 0; i < 8; i++) { a.fL[i] = P.fL[i]; a.bL[i] = P.bL[i]; }
    a.flags = flags;
    const Blocks bs = block_split(N);
    a.nfull = bs.nfull;
    const int nblk = bs.nfull + bs.ntail;
    a.nblk = nblk;
    a.queue = nblk > 0 ? block_queue(stream, 0) : nullptr;
    a.tc = nullptr;
    if (P.F.blender && (saved || P.F.uniform_t))
        a.tc = saved ? saved + (size_t)P.F.nsaved * a.Ns + mask_words(P.F, a.Ns) : timenet_scratch(stream);
}

int backward(int flags, int N, const float *packed, const float *saved, const float *dout, float *scratch,
             float *const *grads, hipStream_t stream) {
    const Plan P = make_plan(flags);
    const Flags &F = P.F;
    const size_t Ns = padded_points(N);
    float *dz = scratch;
    float *slabs = scratch + (size_t)F.nz * Ns;
    BwdArgs b{};
    b.N = N; b.Ns = Ns; b.dout = dout; b.dz = dz;
    b.img = reinterpret_cast<const h16x8 *>(packed);
    b.mask = reinterpret_cast<const uint32_t *>(saved + (size_t)F.nsaved * Ns);
    b.tHd = P.tHd; b.tT2 = P.tT2;
    for (int i = 0; i < 8; i++) b.tL[i] = P.tL[i];
    b.flags = flags;
    const Blocks bs = block_split(N);
    b.nfull = bs.nfull;
    const int nblk = bs.nfull + bs.ntail;
    b.nblk = nblk;
    b.queue = nblk > 0 ? block_queue(stream, 1) : nullptr;
    const int grid = persistent_grid(nblk, b.queue);
    {
        ScopedTimer tm("mlp_bwd", stream);
        if (F.blender && !F.uniform_t)
            hipLaunchKernelGGL(k_bwd<true>, dim3(grid), dim3(NTHR), 0, stream, b);
        else
        {
            // the 8-wave k_bwd8 (bitwise equal to the 16-wave kernel): neutral on the bf16x6 split (r5u),
            // +0.5 % steps/s on the f16 split (mlp_bwd 0.333 -> 0.325 ms, profiles/r6f_mlp_variants_ab.txt);
            // DGS_MLP_BWD8=0 keeps the 16-wave k_bwd
            static const bool bwd8 = [] {
                const char *e = getenv("DGS_MLP_BWD8");
                return !(e && e[0] == '0');
            }();
            if (bwd8)
                hipLaunchKernelGGL(k_bwd8, dim3(grid), dim3(NTHR8), 0, stream, b);
            else
                hipLaunchKernelGGL(k_bwd<false>, dim3(grid), dim3(NTHR), 0, stream, b);
        }
    }
    DGS_LAUNCH_CHECK("k_bwd", false, stream);
    int rc;
    if (dw_mode() == 0)
        rc = mlp::dw_fp32(F, Ns, dz, saved, slabs, grads, stream);
    else
        rc = dw_split_once(F, Ns, dz, saved, slabs, grads, stream);
    if (rc != DGS_OK || !F.uniform_t) return rc;
    TGradArgs g{};
    g.fp = packed + P.img_floats();
    g.w0te = P.w0te; g.w5te = P.w5te; g.wT2 = P.wT2;
    g.tc = saved + (size_t)F.nsaved * Ns + mask_words(F, Ns);
    g.gb0 = grads[P.pLb[0]]; g.gb5 = grads[P.pLb[5]];
    g.gT0w = grads[P.pT0w]; g.gT0b = grads[P.pT0b]; g.gT2w = grads[P.pT2w]; g.gT2b = grads[P.pT2b];
    g.gW0 = grads[P.pLw[0]]; g.gW5 = grads[P.pLw[5]];
    g.tin = F.tin;
    {
        ScopedTimer tm("mlp_tgrad", stream);
        hipLaunchKernelGGL(k_tgrad, dim3(TG_WG), dim3(1024), 0, stream, g);
    }
    DGS_LAUNCH_CHECK("k_tgrad", false, stream);
    return DGS_OK;
}

// dW launches handed to the fp32 k_dw because a 256-row operand exceeds k_dws's 32-bit byte offsets
// (N > ~2.1 M points; dgs_debug_dw_fallbacks)
static std::atomic<long long> g_dw_fallbacks{0};
static int dw_split_once(const Flags &F, size_t Ns, const float *dz, const float *saved, float *slabs,
                         float *const *grads, hipStream_t stream) {
    if ((size_t)WT * Ns * 4 >= 0x7fffffffull) {  // 32-bit byte offsets of a 256-row operand
        g_dw_fallbacks.fetch_add(1);
        return mlp::dw_fp32(F, Ns, dz, saved, slabs, grads, stream);
    }
    const WPlan W = split_wplan(F, std::max(32, 256 - reserved_cus()));
    for (int q = 0; q < W.jobs.n; q++) {  // the shapes k_dws instantiates
        const WJob &j = W.jobs.j[q];
        const bool ok = (j.krows == 256 && (j.nrows == 256 || j.nrows == 32)) ||
                        (j.nrows == 256 && (j.krows == 96 || j.krows == 64 || j.krows == 16));
        if (!ok) {
            set_error("dgs_deform_backward: dW job shape outside k_dws's instantiations");
            return DGS_ERR_ARGS;
        }
    }
    {
        if (int rc = ensure_dynamic_lds((const void *)k_dws, S_LDS)) return rc;
        ScopedTimer tm("mlp_dw", stream);
        hipLaunchKernelGGL(k_dws, dim3(W.nblocks), dim3(DW_THREADS), S_LDS, stream, W.jobs, Ns, dz, saved, slabs);
    }
    DGS_LAUNCH_CHECK("k_dws", false, stream);
    return launch_dw_reduce(F, W, slabs, grads, stream);
}

}  // namespace mlps
}  // namespace dgs

#ifdef DGS_MLP_PROFILE
extern "C" void dgs_mlps_set_prof(unsigned long long *p) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(dgs::mlps::dgs_mlps_prof), &p, sizeof(p));
}
#endif

// ------------------------------------------------------------------------------------------------
// C ABI (include/dgs.h): the split-bf16 path unless DGS_MLP_EXACT_FP32 is set in the flags
// ------------------------------------------------------------------------------------------------
using namespace dgs;

static bool exact_fp32(int flags) { return (flags & DGS_MLP_EXACT_FP32) != 0; }
static int net_flags(int flags) {
    return exact_fp32(flags) ? flags & (DGS_MLP_BLENDER | DGS_MLP_6DOF | DGS_MLP_NO_ROTSCALE)
                             : flags & (DGS_MLP_BLENDER | DGS_MLP_6DOF | DGS_MLP_NO_ROTSCALE | DGS_MLP_UNIFORM_T);
}

#ifdef DGS_CLOCK_STAMPS
// kernel k (0 k_fwd, 1 k_bwd, 2 k_dws): the last launch's per-workgroup stamps, out[6 b ..] =
// (shader clock start, end, 100 MHz real time start, end, HW_ID | XCC_ID << 32, 0) for b < n
// (diagnostic builds only)
extern "C" int dgs_debug_clock(int k, int n, unsigned long long *out) {
    static unsigned long long h[mlps::CLK_BLOCKS][6];
    if (k < 0 || k > 2 || n > mlps::CLK_BLOCKS) return -1;
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(dgs::mlps::dgs_clk), sizeof(h), sizeof(h) * k) != hipSuccess) return -1;
    for (int b = 0; b < n; b++)
        for (int q = 0; q < 6; q++) out[6 * b + q] = h[b][q];
    return 0;
}
#endif

extern "C" void dgs_mlp_set_reserved_cus(int k) { mlps::g_reserve_cus.store(k < 0 ? 0 : k > 64 ? 64 : k); }
extern "C" int dgs_mlp_reserved_cus(void) { return mlps::reserved_cus(); }

extern "C" long long dgs_debug_dw_fallbacks(void) { return mlps::g_dw_fallbacks.load(); }

extern "C" long long dgs_debug_guard_expiries(void) {
    uint32_t v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(dgs::mlps::dgs_mlps_guard_expired), sizeof(v)) != hipSuccess) return -1;
    return (long long)v;
}

extern "C" int dgs_deform_outputs(int flags) { return mlpc::make_flags(flags).nout; }
extern "C" int dgs_deform_num_params(int flags) { return mlpc::make_params(mlpc::make_flags(flags)).nparams; }

extern "C" size_t dgs_deform_packed_floats(int flags) {
    return exact_fp32(flags) ? mlp::packed_floats(net_flags(flags)) : mlps::make_plan(net_flags(flags)).total();
}

extern "C" size_t dgs_deform_saved_floats(int flags, int N) {
    return exact_fp32(flags) ? mlp::saved_floats(net_flags(flags), N) : mlps::saved_floats(net_flags(flags), N);
}

extern "C" size_t dgs_deform_scratch_floats(int flags, int N) {
    return exact_fp32(flags) ? mlp::scratch_floats(net_flags(flags), N) : mlps::scratch_floats(net_flags(flags), N);
}

extern "C" int dgs_deform_pack(int flags, const float *const *params, float *packed, void *stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    if (!params || !packed) {
        set_error("dgs_deform_pack: null argument");
        return DGS_ERR_ARGS;
    }
    return exact_fp32(flags) ? mlp::pack(net_flags(flags), params, packed, stream)
                             : mlps::pack(net_flags(flags), params, packed, stream);
}

extern "C" int dgs_deform_forward(int flags, int N, const float *xyz, const float *t, const float *packed, float *out,
                                  float *saved, void *stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    if (N < 0 || (N > 0 && (!xyz || !t || !packed || !out))) {
        set_error("dgs_deform_forward: null argument");
        return DGS_ERR_ARGS;
    }
    if (N == 0) return DGS_OK;
    return exact_fp32(flags) ? mlp::forward(net_flags(flags), N, xyz, t, packed, out, saved, stream)
                             : mlps::forward(net_flags(flags), N, xyz, t, packed, out, saved, stream);
}

extern "C" int dgs_deform_pack_forward(int flags, const float *const *params, int N, const float *xyz, const float *t,
                                       float *packed, float *out, float *saved, void *stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    if (!params || !packed || N < 0 || (N > 0 && (!xyz || !t || !out))) {
        set_error("dgs_deform_pack_forward: null argument");
        return DGS_ERR_ARGS;
    }
    if (exact_fp32(flags) || N == 0) {
        if (int rc = dgs_deform_pack(flags, params, packed, stream_)) return rc;
        return dgs_deform_forward(flags, N, xyz, t, packed, out, saved, stream_);
    }
    return mlps::pack_forward(net_flags(flags), params, N, xyz, t, packed, out, saved, stream);
}

extern "C" int dgs_deform_backward(int flags, int N, const float *packed, const float *saved, const float *dout,
                                   float *scratch, float *const *grads, void *stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    if (N < 0 || (N > 0 && (!packed || !saved || !dout || !scratch || !grads))) {
        set_error("dgs_deform_backward: null argument");
        return DGS_ERR_ARGS;
    }
    const mlpc::Flags F = mlpc::make_flags(flags);
    const mlpc::Params P = mlpc::make_params(F);
    if (N == 0) {
        for (int k = 0; k < P.nparams; k++) {
            int r, c;
            mlpc::param_shape(F, P, k, r, c);
            DGS_HIP_CHECK(hipMemsetAsync(grads[k], 0, sizeof(float) * r * (c ? c : 1), stream));
        }
        return DGS_OK;
    }
    return exact_fp32(flags) ? mlp::backward(net_flags(flags), N, packed, saved, dout, scratch, grads, stream)
                             : mlps::backward(net_flags(flags), N, packed, saved, dout, scratch, grads, stream);
}
