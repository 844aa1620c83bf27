// Fused deformation MLP (positional encoding + timenet + 8x256 trunk with skip + heads) on bf16 MFMA
// with an exact three-way operand split: the default path of dgs_deform_* (the fp32-MFMA kernels of
// mlp.hip run instead under DGS_MLP_EXACT_FP32).
//
// Replaces DeformNetworkBaseline.forward and its autograd backward (utils/time_utils.py:56-127;
// DeformNetwork :129-201 via DGS_MLP_NO_ROTSCALE; 6-DoF heads :114-121 emitted raw, exp_se3 stays in
// the host glue).
//
// Numerics ("bf16x6"). Every fp32 operand x is split EXACTLY into three bf16 values
//   hi = bf16(x), mid = bf16(x - hi), lo = x - hi - mid        (round to nearest)
// (x - hi is exact in fp32 and has at most 16 significant bits, so lo has at most 8: x = hi+mid+lo,
// |mid| <= 2^-8 |x|, |lo| <= 2^-16 |x|). A product a*b is accumulated as the six bf16 x bf16 products
// hh + hm + mh + hl + lh + mm, each exact in the fp32 accumulator of the MFMA; the dropped ml + lm +
// ll are below 2^-23 |ab| (fp32's own rounding of a product is up to 2^-24 |ab|). An MFMA aligns its
// products and C to the largest term within a limited window (tools/mfma_round_probe.hip), so the
// five corrections of each k-step go into a fresh accumulator that is added to the running sum in
// fp32 (tools/mfma_accum_probe.hip: as accurate as the fp32 fma chain). The GEMMs keep fp32 accuracy
// (tests/test_gpu_mlp.py holds them to the exact-fp32 path's error) at 16/6 = 2.67x the fp32-MFMA
// rate (MI355X: bf16 MFMA = 16x f32 MFMA per clock). Biases, ReLU, PE and reductions stay fp32.
//
// Layout ("transposed" formulation, Y^T = W X^T: features on MFMA rows, points on MFMA columns),
// v_mfma_f32_16x16x32_bf16:
//  * One workgroup = 64 points x 16 waves (4 per SIMD); wave r owns output rows 16r..16r+15 of every
//    256-wide layer for all four 16-point column tiles, so each 3 KiB weight fragment (16 rows x 32
//    features x 3 splits) fetched from L2 feeds 4 x 6 MFMAs.
//  * Activations live in LDS split into hi/mid/lo bf16 images of 16-byte units (8 features x 1
//    point), [8-feature group][split][64 points]: the B operand of a k-step (32 features) is one
//    ds_read_b128 per split and column tile, and an accumulator's 4 rows are one 8-byte store per
//    split into the next layer's image. XE | TE | H groups are contiguous, so cat(x_emb, t_emb) and
//    cat(x_emb, t_emb, h) are plain group ranges (147 KB of LDS: one block per CU).
//  * Narrow layers (timenet.2, heads, the t_emb rows of the backward) run as full-K 16x16 tiles on a
//    subset of the waves: no partial sums.
//  * Weights are packed every call (they change every optimizer step) by one gather + split launch
//    into A-fragment images [n-tile][k-step][split][64 lanes][8 bf16].
//  * Saved activations / dZ stay fp32 feature-major [rows][Ns] (mlp_shared.h row map; the dW GEMM
//    reads them), written in each layer's epilogue; relu' masks are one u16 per lane and 16-row
//    tile ([64-point block][row / 16][64 lanes]). Every reduction has a fixed order: bitwise
//    deterministic.
#include <hip/hip_runtime.h>

#include <atomic>

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
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 64;            // points per workgroup
constexpr int NQ = 4;             // 16-point column tiles per workgroup
constexpr int NWAVE = 16;         // one 16-row n-tile of a 256-wide layer per wave
constexpr int NTHR = NWAVE * 64;
constexpr int NSPLIT = 3;         // hi, mid, lo
constexpr int UG = NSPLIT * BM;   // 16-B units per 8-feature group (all splits, all points)
constexpr int KSLOT = 3 * 64;     // units per (n-tile, k-step) of an A image: 3 splits x 64 lanes
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
static_assert(G_FWD * UG * 16 + (8 * 256 + 16) * 4 + NTHR * 4 + 128 <= 160 * 1024 && G_BWD * UG * 16 <= 160 * 1024,
              "LDS (k_fwd: + trunk biases, pending relu' bits, hand-off counters)");
static_assert(112 * BM * 4 <= 32 * UG * 16, "fp32 staging must fit the H region");

// ------------------------------------------------------------------------------------------------
// exact three-way split
// ------------------------------------------------------------------------------------------------
struct Split4 {
    bf16x4 h, m, l;
};

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// RNE of two floats into one packed bf16 pair (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t cvt2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

// the exact split of two values, pairwise: 3 v_cvt_pk_bf16_f32 + 4 unpacks (the bf16 -> f32 of
// a packed pair is a shift / mask) + 4 subtractions
__device__ __forceinline__ void split2(float a, float b, uint32_t &h, uint32_t &m, uint32_t &l) {
    h = cvt2(a, b);
    const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xffff0000u);
    m = cvt2(ra, rb);
    l = cvt2(ra - __uint_as_float(m << 16), rb - __uint_as_float(m & 0xffff0000u));
}

__device__ inline Split4 split4(float a, float b, float c, float d) {
    uint32_t h0, m0, l0, h1, m1, l1;
    split2(a, b, h0, m0, l0);
    split2(c, d, h1, m1, l1);
    Split4 s;
    s.h = __builtin_bit_cast(bf16x4, make_uint2(h0, h1));
    s.m = __builtin_bit_cast(bf16x4, make_uint2(m0, m1));
    s.l = __builtin_bit_cast(bf16x4, make_uint2(l0, l1));
    return s;
}

// 8 consecutive features of one point -> the three 16-B units of group g (LDS image [g][split][BM])
__device__ inline void put_unit8(bf16x8 *lds, int g, int m, const float (&v)[8]) {
    const Split4 a = split4(v[0], v[1], v[2], v[3]);
    const Split4 b = split4(v[4], v[5], v[6], v[7]);
    bf16x8 *u = lds + g * UG + m;
    u[0] = __builtin_shufflevector(a.h, b.h, 0, 1, 2, 3, 4, 5, 6, 7);
    u[BM] = __builtin_shufflevector(a.m, b.m, 0, 1, 2, 3, 4, 5, 6, 7);
    u[2 * BM] = __builtin_shufflevector(a.l, b.l, 0, 1, 2, 3, 4, 5, 6, 7);
}

// ------------------------------------------------------------------------------------------------
// GEMM pieces. 16x16x32 lane maps (cdna_hip_programming.md §3): lane l (kq = l >> 4, col = l & 15)
// holds A[row col][k = 8 kq + j] and B[k = 8 kq + j][col col]; C/D element i is row 4 kq + i, col col.
// ------------------------------------------------------------------------------------------------
#define MF16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

struct AFrag {  // one operand fragment in its three split parts
    bf16x8 h, m, l;
};

__device__ inline AFrag load_a(const bf16x8 *p) { return AFrag{p[0], p[64], p[128]}; }

// B fragment of column tile q from the LDS image (p: this lane's unit of split 0, column tile 0)
__device__ inline AFrag load_b(const bf16x8 *p, int q) { return AFrag{p[16 * q], p[BM + 16 * q], p[2 * BM + 16 * q]}; }

__device__ inline f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// The six split products of one k-step: hh into the running accumulator, the five corrections
// (|.| <= 2^-8 |hh|) into their own accumulator, added in fp32 once per GEMM (see the numerics note:
// at 2^-8 of the sum's magnitude the corrections lose nothing in their own C)
__device__ inline void mma6(const AFrag &a, const AFrag &b, f32x4 &acc, f32x4 &lo) {
    lo = MF16(a.m, b.m, lo);
    lo = MF16(a.h, b.l, lo);
    lo = MF16(a.l, b.h, lo);
    lo = MF16(a.h, b.m, lo);
    lo = MF16(a.m, b.h, lo);
    acc = MF16(a.h, b.h, acc);
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
#else
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
// groups g0 + 4c + kq). Fully unrolled; per k-step: each column tile's six MFMAs followed by its B
// fragment for the next k-step into the same registers, then the A fragment RING k-steps ahead
// (register ring: the A stream comes from L2). sched_barrier keeps that order per k-step; the other
// three waves of the SIMD cover the B reload latency. pre() runs after the A prologue. SKIP: k-steps
// >= SKIP read the LDS image one k-step further on (linear.5 with t_emb folded: x_emb | h, past t_emb).
template <int NK, int NQ_, class Pre = NoPre, class Gate = NoGate, int SKIP = (1 << 20)>
__device__ inline void gemm(const bf16x8 *__restrict__ Aw, const bf16x8 *lds, int g0, int q0, int lane,
                            f32x4 (&acc)[NQ_], Pre pre = Pre(), Gate gate = Gate()) {
    static_assert(NK >= 1, "empty GEMM");
    const int kq = lane >> 4, col = lane & 15;
    const bf16x8 *Ap = Aw + lane;
    const int bunit = (g0 + kq) * UG + 16 * q0 + col;  // this lane's B unit at k-step 0
    constexpr int AK = KSLOT;
    constexpr int BK = KG * UG;
    auto bofs = [](int k) { return (k + (k >= SKIP ? 1 : 0)) * BK; };  // compile-time per unrolled k
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
    const bf16x8 *Bk = kbase(0);
    AFrag b = load_b(Bk, 0);
    f32x4 lo[NQ_];
#pragma unroll
    for (int q = 0; q < NQ_; q++) lo[q] = zero4();
#pragma unroll
    for (int k = 0; k < NK; k++) {
        __builtin_amdgcn_sched_barrier(0);
        if (k > 0) gate.done(k - 1);  // k-step k-1's B fragments were consumed by its MFMAs
        const uint32_t seen = k + 1 < NK ? gate.peek(k + 1) : 0u;
#pragma unroll
        for (int q = 0; q < NQ_; q++) {
            // the next tile's B fragment (or the next k-step's first) is in flight during this tile's MFMAs
            AFrag nb;
#ifdef DGS_DIAG_BHALF  // diagnostic only (wrong results): every other tile reuses the previous B fragment
            if (q + 1 < NQ_) nb = ((q + 1) & 1) ? b : load_b(Bk, q + 1);
#else
            if (q + 1 < NQ_) nb = load_b(Bk, q + 1);
#endif
            else if (k + 1 < NK) {
                gate.need(k + 1, seen);
                Bk = kbase(k + 1);
                nb = load_b(Bk, 0);
            }
            // the reads stay ahead of ALL six MFMAs of this tile: without this barrier the scheduler,
            // short of registers, sank them below the tile's first four MFMAs (reusing the current
            // fragment's registers), so the next tile's first MFMAs waited on them (k_fwd -1.4 %,
            // profiles/r5f_mlp_bread_pin_ab.txt)
            __builtin_amdgcn_sched_barrier(0);
            mma6(ring[k % RING], b, acc[q], lo[q]);
            if (q + 1 < NQ_ || k + 1 < NK) b = nb;
            // pin the order per column tile: the next fragment's reads stay ahead of this tile's six
            // MFMAs (left to itself the scheduler, at the 128-VGPR cap, pulls each read down to its
            // first use and waits on it: lgkmcnt(0) in front of most MFMAs)
            __builtin_amdgcn_sched_barrier(0);
        }
        if (k + RING < NK) ring[k % RING] = load_a(Ap + (k + RING) * AK);
        __builtin_amdgcn_sched_barrier(0);
    }
    gate.done(NK - 1);
#pragma unroll
    for (int q = 0; q < NQ_; q++) acc[q] += lo[q];
}

// gemm() for TWO n-tiles per wave (the 8-wave k_fwd8): n-tile t's A image at Aw + t * astride units;
// every B fragment read from LDS feeds both n-tiles' six MFMAs, so the activation image is read by 8
// waves per layer instead of 16. Each (n-tile, column tile) accumulator sees the same MFMA sequence
// as in gemm(): outputs bitwise equal to the 16-wave kernel.
template <int NK, int NQ_, class Pre = NoPre, class Gate = NoGate, int SKIP = (1 << 20)>
__device__ inline void gemm2(const bf16x8 *__restrict__ Aw, int astride, const bf16x8 *lds, int g0, int q0, int lane,
                             f32x4 (&acc)[2][NQ_], Pre pre = Pre(), Gate gate = Gate()) {
    static_assert(NK >= 1, "empty GEMM");
    const int kq = lane >> 4, col = lane & 15;
    const bf16x8 *Ap0 = Aw + lane, *Ap1 = Aw + astride + lane;
    const int bunit = (g0 + kq) * UG + 16 * q0 + col;
    constexpr int AK = KSLOT;
    constexpr int BK = KG * UG;
    auto bofs = [](int k) { return (k + (k >= SKIP ? 1 : 0)) * BK; };
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
    const bf16x8 *Bk = kbase(0);
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
        const uint32_t seen = k + 1 < NK ? gate.peek(k + 1) : 0u;
#pragma unroll
        for (int q = 0; q < NQ_; q++) {
            AFrag nb;
            if (q + 1 < NQ_) nb = load_b(Bk, q + 1);
            else if (k + 1 < NK) {
                gate.need(k + 1, seen);
                Bk = kbase(k + 1);
                nb = load_b(Bk, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            mma6(ring[k % RING][0], b, acc[0][q], lo[0][q]);
            mma6(ring[k % RING][1], b, acc[1][q], lo[1][q]);
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
}

// accumulator tile q (rows 16r + 4kq + i of this wave, point 16q + col) -> its 8-byte half of the
// split units of group 2r + (kq >> 1) (LDS image from group gbase)
__device__ inline void acc_to_lds(const f32x4 &v, bf16x8 *lds, int gbase, int r, int q, int lane) {
    const int kq = lane >> 4, col = lane & 15;
    const Split4 s = split4(v[0], v[1], v[2], v[3]);
    bf16x4 *u = reinterpret_cast<bf16x4 *>(lds + (gbase + 2 * r + (kq >> 1)) * UG + 16 * q + col) + (kq & 1);
    u[0] = s.h;
    u[2 * BM] = s.m;  // bf16x4 units: one 16-B unit = 2 of them
    u[4 * BM] = s.l;
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

template <int NQ_>
__device__ inline void bias_relu(f32x4 (&v)[NQ_], float4 b, bool relu) {
#pragma unroll
    for (int q = 0; q < NQ_; q++) {
        v[q] += f32x4{b.x, b.y, b.z, b.w};  // two v_pk_add_f32
        if (relu)
#pragma unroll
            for (int i = 0; i < 4; i++) v[q][i] = fmaxf(v[q][i], 0.f);
    }
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
    const bf16x8 *img;  // A images
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
template <bool SAVE, int NQB, bool FOLD>
__device__ __forceinline__ void fwd_block(const FwdArgs &a, bf16x8 *lds, uint32_t *hwr, uint32_t *hrd, const float4 *sb,
                                          uint32_t *s_mpend, int p0, int slot) {
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
    // ---- positional encodings (utils/time_utils.py:42-54) into fp32 staging: feature 3 band + d,
    // band 0 = x, band 1 + 2i = sin(2^i x), band 2 + 2i = cos(2^i x). The block's xyz rows are read
    // once (one coalesced load per thread, a single HBM round trip) into the identity band, then the
    // 10 sin/cos bands are evaluated from LDS in two rounds of the workgroup ----
    if (tid < 3 * BMB) {
        const int m = tid / 3, d = tid - 3 * m;
        stage[d * BM + m] = p0 + m < pend ? a.xyz[3 * (size_t)p0 + tid] : 0.f;
    }
    if (tid < BMB) stage[63 * BM + tid] = 0.f;  // padding feature
    __syncthreads();
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
            stage[(ST_TE + f) * BM + m] = f < 32 ? a.tc[TC_TE + f] : a.tc[TC_TIN + f - 32];
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
        }
    }
    __syncthreads();
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
            put_unit8(lds, g < 12 ? g : G_TIN + g - 12, m, v);
        }
        if (F.blender && !fold)  // TIN k-step padding (features 16..31): zero, not stale LDS
            for (int u = tid; u < 2 * UG; u += NTHR) lds[(G_TIN + 2) * UG + u] = bf16x8{};
    }
    lds_barrier();
    DGS_STAMP(1);
    f32x4 c[NQB];
    if (SAVE && uniform_t && !F.uniform_t) {  // TH tile from k_timenet: relu' bits + saved rows (per-point backward)
        const float4 th = load_bias4(a.tc + TC_TH, r, lane);
#pragma unroll
        for (int q = 0; q < NQB; q++) c[q] = f32x4{th.x, th.y, th.z, th.w};
        store_mask(relu_bits(c), MR_TH + r);
        tile16(a.saved, Ns, S_TH + 16 * r, p0, lane).store(c);
    }
    // ---- per-point timenet (blender, t not frame-uniform): Linear(13,256)+ReLU -> H; Linear(256,30) -> TE
    if (F.blender && !uniform_t) {
        zero_tiles(c);
        gemm<1, NQB>(a.img + (size_t)(a.fT1 + r) * KSLOT, lds, G_TIN, 0, lane, c);
        bias_relu(c, load_bias4(a.fp + a.bT1, r, lane), true);
        if (SAVE) {
            store_mask(relu_bits(c), MR_TH + r);
            tile16(a.saved, Ns, S_TH + 16 * r, p0, lane).store(c);
        }
#pragma unroll
        for (int q = 0; q < NQB; q++) acc_to_lds(c[q], lds, G_H, r, q, lane);
        lds_barrier();
        if (r < 2 * NQB) {  // TE tile (n-tile r / NQB of 2, column tile r % NQB), full K on one wave
            const int nt = r / NQB, q = r % NQB;
            f32x4 c1[1] = {zero4()};
            gemm<8, 1>(a.img + (size_t)(a.fT2 + nt * 8) * KSLOT, lds, G_H, q, lane, c1);
            const float4 b = load_bias4(a.fp + a.bT2, nt, lane);
            c1[0] += f32x4{b.x, b.y, b.z, b.w};
            if (SAVE) tile16(a.saved, Ns, S_TE + 16 * nt, p0, lane).store(c1, q);
            acc_to_lds(c1[0], lds, G_TE, nt, q, lane);  // TE groups: not read by the T2 GEMM
        }
        lds_barrier();
    }
    // ---- trunk: 8 x (Linear + ReLU), skip cat after layer 4 (time_utils.py:107-112) ----
    // No workgroup barriers: the four waves of a SIMD finish a GEMM thousands of cycles apart (the
    // oldest issues first), so each wave runs its epilogue as soon as every wave has read the H
    // k-step it overwrites (hrd), and the next layer reads an H k-step once its two writer waves
    // have stored it (hwr): early waves' epilogues overlap late waves' MFMAs.
#pragma unroll 1
    for (int L = 0; L < 8; L++) {
        const int g0 = (L == 0 || L == 5) ? G_XE : G_H;
        const int nk = layer_kpad_f(F, L) / 32;
        zero_tiles(c);
        const bf16x8 *Aw = a.img + (size_t)(a.fL[L] + r * nk) * KSLOT;
        float4 bv;
        // the bias comes from the workgroup's LDS copy after the GEMM (sb): a register preload
        // across the GEMM was spilled at 128 VGPRs and its scratch reload sat in every epilogue
        using PreT = NoPre;
        const PreT bp{};
        const HGate hg{hwr, hrd, L == 5 ? (fold ? 2 : 3) : 0, 2u * L, true, lane};
        if (L == 0) {
            if constexpr (FOLD) gemm<2, NQB>(Aw, lds, g0, 0, lane, c, bp);  // XE only
            else gemm<3, NQB>(Aw, lds, g0, 0, lane, c, bp);                 // XE | TE
        } else if (L == 5) {
            if constexpr (FOLD) gemm<10, NQB, PreT, HGate, 2>(Aw, lds, g0, 0, lane, c, bp, hg);  // XE | H
            else gemm<11, NQB>(Aw, lds, g0, 0, lane, c, bp, hg);                                    // XE | TE | H
        } else {
            gemm<8, NQB>(Aw, lds, g0, 0, lane, c, bp, hg);
        }
        bv = sb[64 * L + 4 * r + kq];
        DGS_STAMP(4 + 2 * L);
        DGS_WSTAMP(22, L);  // per wave: GEMM end (layer 3)
        bias_relu(c, bv, true);
        if (SAVE) {
            trunk_mask(relu_bits(c), L);
#ifndef DGS_DIAG_NOSAVE  // diagnostic only (wrong backward): the trunk's saved-activation stores skipped
            tile16(a.saved, Ns, s_h(L) + 16 * r, p0, lane).store(c);
#endif
        }
        if (L == 3 && r == 0) DGS_STAMP(54);
        // this wave's rows are H k-step r / 2: every wave must have read it in this layer
        if (L > 0) lds_wait_ge(hrd + (r >> 1), 16u * L, lds_peek(hrd + (r >> 1)));
        if (L == 3 && r == 0) DGS_STAMP(56);
#pragma unroll
        for (int q = 0; q < NQB; q++) acc_to_lds(c[q], lds, G_H, r, q, lane);
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
        gemm<8, 1>(a.img + (size_t)a.fHd * KSLOT, lds, G_H, hq, lane, c1, NoPre(), HGate{hwr, hrd, 0, 16u, false, lane});
        const float4 b = sb[8 * 64 + kq];
        c1[0] += f32x4{b.x, b.y, b.z, b.w};
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

template <bool SAVE, bool FOLD>
__global__ __launch_bounds__(NTHR) void k_fwd(FwdArgs a) {
    __shared__ bf16x8 lds[G_FWD * UG];
    __shared__ uint32_t hwr[8], hrd[8];  // trunk hand-off counters (HGate)
    __shared__ int s_next;
    // trunk and head biases (launch constants: FOLD's linear.0 / linear.5 biases come from
    // k_timenet), one float4 per (layer, 4 rows), the heads' 16 rows last; the first block's staging
    // barriers publish them
    __shared__ float4 s_bias[8 * 64 + 4];
    __shared__ uint32_t s_mpend[NTHR];  // relu' bits of an even trunk layer, per thread (fwd_block)
    for (int i = threadIdx.x; i < 8 * 64 + 4; i += NTHR) {
        const int L = i >> 6;
        const float *bias = L == 8                ? a.fp + a.bHd
                            : FOLD && L == 0      ? a.tc + TC_C0
                            : FOLD && L == 5      ? a.tc + TC_C5
                                                  : a.fp + a.bL[L];
        s_bias[i] = reinterpret_cast<const float4 *>(bias)[i & 63];
    }
    CLK_BEGIN();
    for (int b = blockIdx.x;;) {
        int nx = 0;
        if (a.queue && threadIdx.x == 0) nx = queue_take(a.queue);
        if (b < a.nfull) fwd_block<SAVE, NQ, FOLD>(a, lds, hwr, hrd, s_bias, s_mpend, b * BM, b);
        else fwd_block<SAVE, 1, FOLD>(a, lds, hwr, hrd, s_bias, s_mpend, a.nfull * BM + (b - a.nfull) * 16, b);
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
// (k_fwd8, 512 threads, 2 waves per SIMD, 256 VGPRs): wave w owns rows 32w .. 32w + 31 of every trunk
// layer = H k-step w, so each k-step has ONE writer (hand-off target L per layer) and 8 readers.
// Same LDS image, saved-activation / relu'-mask layouts and arithmetic as fwd_block<true, NQB, true>.
constexpr int NW8 = 8, NTHR8 = NW8 * 64;
template <int NQB>
__device__ __forceinline__ void fwd_block8(const FwdArgs &a, bf16x8 *lds, uint32_t *hwr, uint32_t *hrd, const float4 *sb,
                                           uint32_t *s_mpend, int p0, int slot) {
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
    if (tid < 8) {
        hwr[tid] = 0;
        hrd[tid] = 0;
    }
    // positional encodings (utils/time_utils.py:42-54), as fwd_block
    if (tid < 3 * BMB) {
        const int m = tid / 3, d = tid - 3 * m;
        stage[d * BM + m] = p0 + m < pend ? a.xyz[3 * (size_t)p0 + tid] : 0.f;
    }
    if (tid < BMB) stage[63 * BM + tid] = 0.f;
    __syncthreads();
    for (int e = tid; e < BMB * 3 * 10; e += NTHR8) {
        const int m = e % BMB, rr = e / BMB, d = rr % 3, i = rr / 3;
        const bool ok = p0 + m < pend;
        float sv, cv;
        sincosf(stage[d * BM + m] * (float)(1 << i), &sv, &cv);
        stage[(3 * (1 + 2 * i) + d) * BM + m] = ok ? sv : 0.f;
        stage[(3 * (2 + 2 * i) + d) * BM + m] = ok ? cv : 0.f;
    }
    __syncthreads();
    for (int e = tid; e < 64 * BMB; e += NTHR8) {  // saved x_emb rows (folded: dW reads x_emb only)
        const int f = e / BMB, m = e % BMB;
        a.saved[(size_t)(S_XE + f) * Ns + p0 + m] = stage[f * BM + m];
    }
    for (int u = tid; u < 8 * BMB; u += NTHR8) {
        const int g = u / BMB, m = u % BMB;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = stage[(8 * g + j) * BM + m];
        put_unit8(lds, g, m, v);
    }
    lds_barrier();
    f32x4 c[2][NQB];
#pragma unroll 1
    for (int L = 0; L < 8; L++) {
        const int g0 = (L == 0 || L == 5) ? G_XE : G_H;
        const int nk = layer_kpad_f(F, L) / 32;
#pragma unroll
        for (int t = 0; t < 2; t++) zero_tiles(c[t]);
        const bf16x8 *Aw = a.img + (size_t)(a.fL[L] + 2 * w * nk) * KSLOT;
        const int astride = nk * KSLOT;
        const HGate hg{hwr, hrd, L == 5 ? 2 : 0, 1u * L, true, lane};
        if (L == 0) gemm2<2, NQB>(Aw, astride, lds, g0, 0, lane, c);
        else if (L == 5) gemm2<10, NQB, NoPre, HGate, 2>(Aw, astride, lds, g0, 0, lane, c, NoPre(), hg);
        else gemm2<8, NQB>(Aw, astride, lds, g0, 0, lane, c, NoPre(), hg);
#pragma unroll
        for (int t = 0; t < 2; t++) {
            const int nt = 2 * w + t;
            bias_relu(c[t], sb[64 * L + 4 * nt + kq], true);
            trunk_mask(relu_bits(c[t]), L, nt);
            tile16(a.saved, Ns, s_h(L) + 16 * nt, p0, lane).store(c[t]);
        }
        // this wave's rows are H k-step w: all 8 waves must have read it in this layer
        if (L > 0) lds_wait_ge(hrd + w, (uint32_t)NW8 * L, lds_peek(hrd + w));
#pragma unroll
        for (int t = 0; t < 2; t++)
#pragma unroll
            for (int q = 0; q < NQB; q++) acc_to_lds(c[t][q], lds, G_H, 2 * w + t, q, lane);
        lds_signal(hwr + w, lane);
    }
    // heads on the last NQB waves (one column tile each), once all 8 layers' writers have signalled
    const int hq = w - (NW8 - NQB);
    if (hq >= 0) {
        f32x4 c1[1] = {zero4()};
        gemm<8, 1>(a.img + (size_t)a.fHd * KSLOT, lds, G_H, hq, lane, c1, NoPre(), HGate{hwr, hrd, 0, 8u, false, lane});
        const float4 b = sb[8 * 64 + kq];
        c1[0] += f32x4{b.x, b.y, b.z, b.w};
        const int p = p0 + 16 * hq + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (p < pend && 4 * kq + i < F.nout) a.out[(size_t)p * F.nout + 4 * kq + i] = c1[0][i];
    }
}

__global__ __launch_bounds__(NTHR8) void k_fwd8(FwdArgs a) {
    __shared__ bf16x8 lds[G_FWD * UG];
    __shared__ uint32_t hwr[8], hrd[8];
    __shared__ int s_next;
    __shared__ float4 s_bias[8 * 64 + 4];
    __shared__ uint32_t s_mpend[NTHR];  // [n-tile][64 lanes]
    for (int i = threadIdx.x; i < 8 * 64 + 4; i += NTHR8) {
        const int L = i >> 6;
        const float *bias = L == 8 ? a.fp + a.bHd : L == 0 ? a.tc + TC_C0 : L == 5 ? a.tc + TC_C5 : a.fp + a.bL[L];
        s_bias[i] = reinterpret_cast<const float4 *>(bias)[i & 63];
    }
    for (int b = blockIdx.x;;) {
        int nx = 0;
        if (a.queue && threadIdx.x == 0) nx = queue_take(a.queue);
        if (b < a.nfull) fwd_block8<NQ>(a, lds, hwr, hrd, s_bias, s_mpend, b * BM, b);
        else fwd_block8<1>(a, lds, hwr, hrd, s_bias, s_mpend, a.nfull * BM + (b - a.nfull) * 16, b);
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
    const bf16x8 *img;
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

// TE_ROWS: per-point dL/dt_emb (blender, t not frame-uniform); the other instantiation carries no
// t_emb registers or code (raw t PE has no parameters upstream; uniform t: k_tgrad)
template <bool TE_ROWS, int NQB>
__device__ __forceinline__ void bwd_block(const BwdArgs &a, bf16x8 *lds, uint32_t *hwr, uint32_t *hrd, int p0, int slot) {
    constexpr int BMB = 16 * NQB;  // points of this block (fwd_block)
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
    // dOut -> dz rows Z_G (heads' dW) and the split G image
    for (int e = tid; e < 32 * BMB; e += NTHR) {
        const int c = e / BMB, m = e % BMB;
        const int p = p0 + m;
        const float v = (p < a.N && c < F.nout) ? a.dout[(size_t)p * F.nout + c] : 0.f;
        a.dz[(size_t)(Z_G + c) * Ns + p] = v;
        stage[c * BM + m] = v;
    }
    __syncthreads();
    if (tid < 4 * BMB) {
        const int g = tid / BMB, m = tid % BMB;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = stage[(8 * g + j) * BM + m];
        put_unit8(lds, G_BG + g, m, v);
    }
    lds_barrier();
    f32x4 c[NQB];
    // The dZ chain runs without workgroup barriers (see k_fwd's trunk): step 0 (heads^T) and steps
    // i = 1..7 (layer L = 8 - i) each write dZ into H; step i reads H once both writers of each
    // k-step have signalled (hwr >= 2i) and overwrites its own k-step once all 16 waves have read
    // it (hrd >= 16i).
    // heads^T: dH7 = W_h^T dOut (K = 32 from G) -> mask H7 -> dZ7
    {
        uint32_t mk;
        zero_tiles(c);
        gemm<1, NQB>(a.img + (size_t)(a.tHd + r) * KSLOT, lds, G_BG, 0, lane, c, trunk_pre(&mk, 7));
        mask_apply(c, mk);
        tile16(a.dz, Ns, Z_L0 + 7 * 256 + 16 * r, p0, lane).store(c);
#pragma unroll
        for (int q = 0; q < NQB; q++) acc_to_lds(c[q], lds, G_BH, r, q, lane);
        lds_signal(hwr + (r >> 1), lane);
    }
    f32x4 te5[1] = {zero4()};  // t_emb tile of layer 5's dX (waves 0-7, TE_ROWS)
#pragma unroll 1
    for (int L = 7; L >= 1; L--) {
        const uint32_t step = 8 - L;
        // dX_L = W_L^T dZ_L; the H-part rows of the padded L5 input are n-tiles F_H / 16 + r
        if (TE_ROWS && L == 5 && r < 2 * NQB)  // t_emb rows (padded 64..95 = n-tiles 4, 5) x column tile r % NQB
            gemm<8, 1>(a.img + (size_t)(a.tL[5] + (F_TE / 16 + r / NQB) * 8) * KSLOT, lds, G_BH, r % NQB, lane, te5,
                       NoPre(), HGate{hwr, hrd, 0, 2u * step, false, lane});
        const int tile0 = (L == 5) ? F_H / 16 : 0;
        uint32_t mk;
        zero_tiles(c);
        gemm<8, NQB>(a.img + (size_t)(a.tL[L] + (tile0 + r) * 8) * KSLOT, lds, G_BH, 0, lane, c,
                    trunk_pre(&mk, L - 1), HGate{hwr, hrd, 0, 2u * step, true, lane});
        mask_apply(c, mk);
#ifndef DGS_DIAG_NOSAVE  // diagnostic only (wrong dW): the dZ chain's stores skipped
        tile16(a.dz, Ns, Z_L0 + (L - 1) * 256 + 16 * r, p0, lane).store(c);
#endif
        lds_wait_ge(hrd + (r >> 1), 16u * step, lds_peek(hrd + (r >> 1)));
#pragma unroll
        for (int q = 0; q < NQB; q++) acc_to_lds(c[q], lds, G_BH, r, q, lane);
        lds_signal(hwr + (r >> 1), lane);
    }
    if (!TE_ROWS) return;
    // layer 0's t_emb rows added to layer 5's: dTE tile (n-tile r / NQB, column tile r % NQB) -> dz rows
    // Z_TE (timenet.2's dW) and the split G image (dOut's, no longer read)
    if (r < 2 * NQB) {
        const int nt = r / NQB, q = r % NQB;
        gemm<8, 1>(a.img + (size_t)(a.tL[0] + (F_TE / 16 + nt) * 8) * KSLOT, lds, G_BH, q, lane, te5, NoPre(),
                   HGate{hwr, hrd, 0, 16u, false, lane});
        tile16(a.dz, Ns, Z_TE + 16 * nt, p0, lane).store(te5, q);
        acc_to_lds(te5[0], lds, G_BG, nt, q, lane);
    }
    lds_barrier();
    // timenet.2^T: dTH = W_T2^T dTE (K = 32) -> mask TH -> dZ_T1
    {
        uint32_t mk;
        zero_tiles(c);
        gemm<1, NQB>(a.img + (size_t)(a.tT2 + r) * KSLOT, lds, G_BG, 0, lane, c, MaskPre{&mk, mask_tile(MR_TH + r), lane});
        mask_apply(c, mk);
        tile16(a.dz, Ns, Z_T1 + 16 * r, p0, lane).store(c);
    }
}

// The dX chain for a frame-uniform t (TE_ROWS = false: every training step) as 8 waves of two n-tiles
// (k_bwd8, as k_fwd8): wave w writes dZ rows 32w .. 32w + 31 = H k-step w (one writer per k-step and
// step, 8 readers). Same arithmetic, layouts and outputs as bwd_block<false, NQB>.
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
__device__ __forceinline__ void bwd_block8(const BwdArgs &a, bf16x8 *lds, uint32_t *hwr, uint32_t *hrd, int p0, int slot) {
    constexpr int BMB = 16 * NQB;
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
    for (int e = tid; e < 32 * BMB; e += NTHR8) {  // dOut -> dz rows Z_G and the split G image
        const int c = e / BMB, m = e % BMB;
        const int p = p0 + m;
        const float v = (p < a.N && c < F.nout) ? a.dout[(size_t)p * F.nout + c] : 0.f;
        a.dz[(size_t)(Z_G + c) * Ns + p] = v;
        stage[c * BM + m] = v;
    }
    __syncthreads();
    if (tid < 4 * BMB) {
        const int g = tid / BMB, m = tid % BMB;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = stage[(8 * g + j) * BM + m];
        put_unit8(lds, G_BG + g, m, v);
    }
    lds_barrier();
    f32x4 c[2][NQB];
    {  // heads^T: dH7 = W_h^T dOut (K = 32 from G) -> mask H7 -> dZ7
        uint32_t mk[2];
#pragma unroll
        for (int t = 0; t < 2; t++) zero_tiles(c[t]);
        gemm2<1, NQB>(a.img + (size_t)(a.tHd + 2 * w) * KSLOT, KSLOT, lds, G_BG, 0, lane, c, trunk_pre(mk, 7));
#pragma unroll
        for (int t = 0; t < 2; t++) {
            mask_apply(c[t], mk[t]);
            tile16(a.dz, Ns, Z_L0 + 7 * 256 + 16 * (2 * w + t), p0, lane).store(c[t]);
        }
#pragma unroll
        for (int t = 0; t < 2; t++)
#pragma unroll
            for (int q = 0; q < NQB; q++) acc_to_lds(c[t][q], lds, G_BH, 2 * w + t, q, lane);
        lds_signal(hwr + w, lane);
    }
#pragma unroll 1
    for (int L = 7; L >= 1; L--) {
        const uint32_t step = 8 - L;
        const int tile0 = (L == 5) ? F_H / 16 : 0;
        uint32_t mk[2];
#pragma unroll
        for (int t = 0; t < 2; t++) zero_tiles(c[t]);
        gemm2<8, NQB>(a.img + (size_t)(a.tL[L] + (tile0 + 2 * w) * 8) * KSLOT, 8 * KSLOT, lds, G_BH, 0, lane, c,
                      trunk_pre(mk, L - 1), HGate{hwr, hrd, 0, step, true, lane});
#pragma unroll
        for (int t = 0; t < 2; t++) {
            mask_apply(c[t], mk[t]);
            tile16(a.dz, Ns, Z_L0 + (L - 1) * 256 + 16 * (2 * w + t), p0, lane).store(c[t]);
        }
        lds_wait_ge(hrd + w, (uint32_t)NW8 * step, lds_peek(hrd + w));
#pragma unroll
        for (int t = 0; t < 2; t++)
#pragma unroll
            for (int q = 0; q < NQB; q++) acc_to_lds(c[t][q], lds, G_BH, 2 * w + t, q, lane);
        lds_signal(hwr + w, lane);
    }
}

__global__ __launch_bounds__(NTHR8) void k_bwd8(BwdArgs a) {
    __shared__ bf16x8 lds[G_BWD * UG];
    __shared__ uint32_t hwr[8], hrd[8];
    __shared__ int s_next;
    for (int b = blockIdx.x;;) {
        int nx = 0;
        if (a.queue && threadIdx.x == 0) nx = queue_take(a.queue);
        if (b < a.nfull) bwd_block8<NQ>(a, lds, hwr, hrd, b * BM, b);
        else bwd_block8<1>(a, lds, hwr, hrd, a.nfull * BM + (b - a.nfull) * 16, b);
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
    __shared__ bf16x8 lds[G_BWD * UG];
    __shared__ uint32_t hwr[8], hrd[8];  // dZ hand-off counters (HGate), as in k_fwd's trunk
    __shared__ int s_next;
    CLK_BEGIN();
    for (int b = blockIdx.x;;) {  // persistent: as k_fwd
        int nx = 0;
        if (a.queue && threadIdx.x == 0) nx = queue_take(a.queue);
        if (b < a.nfull) bwd_block<TE_ROWS, NQ>(a, lds, hwr, hrd, b * BM, b);
        else bwd_block<TE_ROWS, 1>(a, lds, hwr, hrd, a.nfull * BM + (b - a.nfull) * 16, b);
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
// dW = dZ X^T over all points (split-N): operands staged fp32 -> split bf16 planes in LDS, 16 points
// (one bf16 k-step) per chunk, double-buffered; per-workgroup slabs reduced by k_dw_reduce (mlp.hip)
// ------------------------------------------------------------------------------------------------
constexpr int PC = 16;                 // points per chunk = one k-step
constexpr int PITCH = 24;              // bf16 per LDS row: 16 + 8 pad (48 B: conflict-free b128 reads)
constexpr int PLANE = WT * PITCH;      // bf16 per split plane
constexpr int OPND = NSPLIT * PLANE;   // bf16 per operand
constexpr int DW_LDS = 2 * 2 * OPND * 2;  // bytes: 2 buffers x (A, B)
constexpr int DW_THREADS = 512;
static_assert(DW_LDS <= 160 * 1024, "dW LDS");

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

// the six split products into one 32x32 accumulator, smallest first
__device__ inline void mma6_1(const AFrag &a, const AFrag &b, f32x16 &c) {
    c = MFMA32(a.m, b.m, c);
    c = MFMA32(a.h, b.l, c);
    c = MFMA32(a.l, b.h, c);
    c = MFMA32(a.h, b.m, c);
    c = MFMA32(a.m, b.h, c);
    c = MFMA32(a.h, b.h, c);
}

__device__ inline AFrag load_plane_frag(const __bf16 *op, int row, int h) {
    const __bf16 *p = op + row * PITCH + 8 * h;
    return AFrag{*reinterpret_cast<const bf16x8 *>(p), *reinterpret_cast<const bf16x8 *>(p + PLANE),
                 *reinterpret_cast<const bf16x8 *>(p + 2 * PLANE)};
}

// one float4 (row, 4 points) -> the three planes
__device__ inline void stage_split(__bf16 *op, int row, int col4, float4 v) {
    const Split4 s = split4(v.x, v.y, v.z, v.w);
    bf16x4 *p = reinterpret_cast<bf16x4 *>(op + row * PITCH + 4 * col4);
    p[0] = s.h;
    p[PLANE / 4] = s.m;
    p[2 * PLANE / 4] = s.l;
}

__device__ inline float4 zsel4(float4 v, bool ok) {
    return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}

template <bool NARROW>
__device__ __forceinline__ void dw_tile(const WJob &J, size_t Ns, const float *__restrict__ dz,
                                        const float *__restrict__ saved, float *__restrict__ slabs, __bf16 *lds) {
    const int split = blockIdx.x - J.block0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave >> 2, wk = wave & 3;  // wide wave tile: rows [128 wn, +128), cols [64 wk, +64)
    const int h = lane >> 5, i = lane & 31;
    const int nch = (int)(Ns / PC);
    const int per = div_up(nch, J.nsplit);
    const int c0 = split * per;
    const int c1 = min(nch, c0 + per);
    // staging: float4 q = tid + 512 j (j < 2): row = q / 4 (0..255), points 4 (q % 4) .. +3
    const int srow = tid >> 2, scol = tid & 3;
    const float *baseA = dz + (size_t)J.zrow * Ns;
    const float *baseB = saved + (size_t)J.xrow * Ns;
    const bool okA0 = srow < J.nrows, okA1 = srow + 128 < J.nrows;
    const bool okB0 = srow < J.krows, okB1 = srow + 128 < J.krows;
    // 32-bit byte offsets from a uniform base; rows past the extent load row 0 (always valid) and are
    // zeroed at the LDS store, so the loads stay in flight across the chunk's MFMAs
    const uint32_t ns = (uint32_t)Ns;
    const uint32_t uA0 = ((okA0 ? srow : 0) * ns + 4 * scol) * 4, uA1 = ((okA1 ? srow + 128 : 0) * ns + 4 * scol) * 4;
    const uint32_t uB0 = ((okB0 ? srow : 0) * ns + 4 * scol) * 4, uB1 = ((okB1 ? srow + 128 : 0) * ns + 4 * scol) * 4;
#define DW_LD(base, u, c) \
    (*reinterpret_cast<const float4 *>(reinterpret_cast<const char *>(base) + (uint32_t)((u) + (uint32_t)(c) * (PC * 4u))))
    struct Stage {
        float4 a0, a1, b0, b1;
    };
    float bs0 = 0.f, bs1 = 0.f;  // bias row sums of the staged dZ rows
    auto gload = [&](Stage &r, int c) {
        r.a0 = DW_LD(baseA, uA0, c);
        r.a1 = DW_LD(baseA, uA1, c);
        r.b0 = DW_LD(baseB, uB0, c);
        r.b1 = DW_LD(baseB, uB1, c);
    };
    auto lstore = [&](const Stage &r, int buf) {
        __bf16 *A = lds + buf * 2 * OPND;
        __bf16 *B = A + OPND;
        const float4 a0 = zsel4(r.a0, okA0), a1 = zsel4(r.a1, okA1);
        bs0 += (a0.x + a0.y) + (a0.z + a0.w);
        bs1 += (a1.x + a1.y) + (a1.z + a1.w);
        stage_split(A, srow, scol, a0);
        stage_split(A, srow + 128, scol, a1);
        stage_split(B, srow, scol, zsel4(r.b0, okB0));
        stage_split(B, srow + 128, scol, zsel4(r.b1, okB1));
    };
#undef DW_LD
    // this wave's active sub-tiles (wave-uniform). wide: rows 128 wn + 32 t, cols 64 wk + 32 u
    // (acc[t][u]); narrow: rows 32 wave, cols 32 v (acc[v >> 1][v & 1], v < 4)
    const int nact_r = NARROW ? (32 * wave < J.nrows ? 1 : 0) : min(4, max(0, div_up(J.nrows - 128 * wn, 32)));
    const int nact_c = NARROW ? min(4, div_up(J.krows, 32)) : min(2, max(0, div_up(J.krows - 64 * wk, 32)));
    const bool any = nact_r > 0 && nact_c > 0;
    f32x16 acc[4][2];
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[t][u][r] = 0.f;
    auto compute = [&](int buf) {
        const __bf16 *A = lds + buf * 2 * OPND;
        const __bf16 *B = A + OPND;
        if (any && NARROW) {
            const AFrag a0 = load_plane_frag(A, 32 * wave + i, h);
#pragma unroll
            for (int v = 0; v < 4; v++) {
                if (v >= nact_c) continue;
                const AFrag b = load_plane_frag(B, 32 * v + i, h);
                mma6_1(a0, b, acc[v >> 1][v & 1]);
            }
        } else if (any) {
            AFrag bb[2];
#pragma unroll
            for (int u = 0; u < 2; u++) bb[u] = load_plane_frag(B, 64 * wk + 32 * u + i, h);
#pragma unroll
            for (int t = 0; t < 4; t++) {
                if (t >= nact_r) continue;
                const AFrag at = load_plane_frag(A, 128 * wn + 32 * t + i, h);
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    if (u >= nact_c) continue;
                    mma6_1(at, bb[u], acc[t][u]);
                }
            }
        }
    };
    // Pipeline: LDS buffers alternate per chunk; two register stages keep the global loads two chunks
    // ahead. Barriers wait for LDS only (lds_barrier): a __syncthreads() would also drain the
    // prefetched global loads (vmcnt 0) every 48 MFMAs.
    Stage R0, R1;
    if (c0 < c1) gload(R0, c0);
    if (c0 + 1 < c1) gload(R1, c0 + 1);
    if (c0 < c1) lstore(R0, 0);
    if (c0 + 2 < c1) gload(R0, c0 + 2);
    lds_barrier();
    for (int c = c0; c < c1; c += 2) {
        // buffer 0 holds chunk c, R1 chunk c + 1, R0 chunk c + 2 (in flight)
        compute(0);
        if (c + 1 < c1) lstore(R1, 1);
        if (c + 3 < c1) gload(R1, c + 3);
        lds_barrier();
        if (c + 1 >= c1) break;
        compute(1);
        if (c + 2 < c1) lstore(R0, 0);
        if (c + 4 < c1) gload(R0, c + 4);
        lds_barrier();
    }
    float *slab = slabs + (size_t)blockIdx.x * SLAB;
    // bias row sums: the 4 lanes staging a row hold its partial sums (fixed xor-tree order)
    bs0 += __shfl_xor(bs0, 1);
    bs0 += __shfl_xor(bs0, 2);
    bs1 += __shfl_xor(bs1, 1);
    bs1 += __shfl_xor(bs1, 2);
    if (scol == 0) {
        slab[WT * WT + srow] = bs0;
        slab[WT * WT + srow + 128] = bs1;
    }
    // rows past nrows / cols past krows hold zeros or partial garbage that k_dw_reduce never reads
    if (NARROW) {
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int nb = 32 * wave, kb = 32 * v;
#pragma unroll
            for (int r = 0; r < 16; r++) slab[(nb + TileAddr::row(r) + 4 * h) * WT + kb + i] = acc[v >> 1][v & 1][r];
        }
        return;
    }
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int nb = 128 * wn + 32 * t, kb = 64 * wk + 32 * u;
#pragma unroll
            for (int r = 0; r < 16; r++) slab[(nb + TileAddr::row(r) + 4 * h) * WT + kb + i] = acc[t][u][r];
        }
}

__global__ __launch_bounds__(DW_THREADS) void k_dw(WJobs JT, size_t Ns, const float *__restrict__ dz,
                                                   const float *__restrict__ saved, float *__restrict__ slabs) {
    extern __shared__ bf16x8 dw_lds[];
    // job of this workgroup: static-index selects over the kernel-argument table (no scratch copy)
    WJob J = JT.j[0];
#pragma unroll
    for (int q = 1; q < MAXJ; q++)
        if (q < JT.n && (int)blockIdx.x >= JT.j[q].block0) J = JT.j[q];
    // the two wave layouts are separate code regions (one loop with a runtime switch spills)
    if (J.narrow)
        dw_tile<true>(J, Ns, dz, saved, slabs, reinterpret_cast<__bf16 *>(dw_lds));
    else
        dw_tile<false>(J, Ns, dz, saved, slabs, reinterpret_cast<__bf16 *>(dw_lds));
}

// ------------------------------------------------------------------------------------------------
// dW = dZ X^T on split bf16 with LDS-DMA staging (k_dwg). The fp32 dZ / X rows stream global ->
// LDS through global_load_lds_dwordx4 (no VGPR staging, no staging VALU, no lock-step store
// phase): 32 points (two 16-point k-steps) per chunk, two buffers, ONE barrier per chunk, the next
// chunk's DMA in flight during this chunk's MFMAs. Each wave splits its fp32 fragments in registers
// right before its MFMAs. Same job plan, slab layout and k_dw_reduce as the fp32 k_dw.
//   Numerics: each k-step's six split products go into a fresh accumulator T (C = 0) added to the
// running sum in fp32 (RNE): tools/mfma_accum_probe.hip measured this as more accurate than the fp32
// fma chain at K = 4096 (one running C loses the low bits of the small terms with a bias).
//   LDS image per operand and buffer: 16-B units (4 points of one row) [s][rb][q][i]: k-step s (2),
//   32-row block rb (8), point quad q (4), row i (32). One DMA wave-instruction fills the 1 KiB of
//   (s, rb, q pair) lane-linearly (lane l -> q = 2 qp + (l >> 5), i = l & 31); a 32x32x16 fragment
//   (lane (i, h): row i, points 8h..8h+7) is two conflict-free ds_read_b128 (units q = 2h, 2h + 1).
// ------------------------------------------------------------------------------------------------
constexpr int GPC = 32;                 // points per chunk
constexpr int G_OPND = 2 * 8 * 4 * 32;  // 16-B units per operand and buffer
constexpr int G_BUF = 2 * G_OPND;       // units per buffer (dZ, X)
constexpr int G_LDS = 2 * G_BUF * 16;   // bytes (128 KiB)
static_assert(G_LDS <= 160 * 1024, "dWg LDS");

__device__ __forceinline__ constexpr int g_unit(int s, int rb, int q, int i) { return ((s * 8 + rb) * 4 + q) * 32 + i; }

// 8 fp32 (one row, points 8h .. 8h + 7) -> the hi / mid / lo bf16 fragments
__device__ __forceinline__ AFrag split8(const float4 &a, const float4 &b) {
    uint32_t h[4], m[4], l[4];
    split2(a.x, a.y, h[0], m[0], l[0]);
    split2(a.z, a.w, h[1], m[1], l[1]);
    split2(b.x, b.y, h[2], m[2], l[2]);
    split2(b.z, b.w, h[3], m[3], l[3]);
    return AFrag{__builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3])),
                 __builtin_bit_cast(bf16x8, make_uint4(m[0], m[1], m[2], m[3])),
                 __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]))};
}

__device__ __forceinline__ float sum8(const float4 &a, const float4 &b) {
    return ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
}

// one k-step's six split products into a fresh T, then acc += T in fp32
__device__ __forceinline__ void mma6_fresh(const AFrag &a, const AFrag &b, f32x16 &acc) {
    f32x16 t = MFMA32(a.m, b.m, (f32x16)(0.f));
    t = MFMA32(a.h, b.l, t);
    t = MFMA32(a.l, b.h, t);
    t = MFMA32(a.h, b.m, t);
    t = MFMA32(a.m, b.h, t);
    t = MFMA32(a.h, b.h, t);
    acc += t;
}

typedef __attribute__((address_space(1))) void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;

template <bool NARROW>
__device__ __forceinline__ void dwg_tile(const WJob &J, size_t Ns, const float *__restrict__ dz,
                                         const float *__restrict__ saved, float *__restrict__ slabs, float4 *lds) {
    const int split = blockIdx.x - J.block0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave >> 2, wk = wave & 3;
    const int h = lane >> 5, i = lane & 31;
    const int nch = (int)(Ns / GPC);
    const int per = div_up(nch, J.nsplit);
    const int c0 = split * per;
    const int c1 = min(nch, c0 + per);
    // this wave's 8 DMA instructions per chunk: d = 8 wave + j -> operand d >> 5 (waves 0-3 dZ,
    // 4-7 X), k-step, row block and quad pair of the 1 KiB they fill (all wave-uniform but the lane
    // offset). Row blocks past the job's extent are not loaded; the rows of a partial block past it
    // are in bounds (every job's rows rounded up to 32 lie inside saved / dZ, mlp_shared.h row maps)
    // and only feed outputs k_dw_reduce never reads.
    const int op = wave >> 2;
    const float *obase = op ? saved + (size_t)J.xrow * Ns : dz + (size_t)J.zrow * Ns;
    const int ext = op ? J.krows : J.nrows;
    // buffer form: lane offset in one VGPR, row-block offset in an SGPR, chunk base in the
    // descriptor (the host keeps 256 rows x Ns x 4 B below 2^31)
    const uint32_t lane_off = (uint32_t)((i * Ns + 4 * h) * 4);
    auto issue = [&](int c, int buf) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(obase + (size_t)c * GPC), 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int e = (8 * wave + j) & 31;
            const int s = e >> 4, rb = (e >> 1) & 7, qp = e & 1;
            if (rb * 32 < ext)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (lptr_t)(lds + buf * G_BUF + op * G_OPND + g_unit(s, rb, 2 * qp, 0)), 16, lane_off,
                    (uint32_t)((rb * 32 * Ns + s * 16 + 8 * qp) * 4), 0, 0);
        }
    };
    const int nact_r = NARROW ? (32 * wave < J.nrows ? 1 : 0) : min(4, max(0, div_up(J.nrows - 128 * wn, 32)));
    const int nact_c = NARROW ? min(4, div_up(J.krows, 32)) : min(2, max(0, div_up(J.krows - 64 * wk, 32)));
    const bool any = nact_r > 0 && nact_c > 0;
    f32x16 acc[4][2];
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[t][u][r] = 0.f;
    float bs[4] = {0.f, 0.f, 0.f, 0.f};  // bias row sums of this lane's dZ rows (fixed order)
    const bool bias_wave = NARROW || wk == 0;
    if (c0 < c1) issue(c0, 0);
    for (int c = c0; c < c1; c++) {
        const int buf = (c - c0) & 1;
        // this wave's DMAs of chunk c have landed; after the barrier everyone's have, and every wave
        // is done reading the other buffer (chunk c - 1), which the next DMAs overwrite
        __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) expcnt(7) lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        if (c + 1 < c1) issue(c + 1, buf ^ 1);
        if (!any) continue;
        const float4 *A = lds + buf * G_BUF;
        const float4 *B = A + G_OPND;
#pragma unroll
        for (int s = 0; s < 2; s++) {
            if (NARROW) {
                const float4 a0 = A[g_unit(s, wave, 2 * h, i)], a1 = A[g_unit(s, wave, 2 * h + 1, i)];
                bs[0] += sum8(a0, a1);
                const AFrag at = split8(a0, a1);
#pragma unroll
                for (int v = 0; v < 4; v++) {
                    if (v >= nact_c) continue;
                    const AFrag b = split8(B[g_unit(s, v, 2 * h, i)], B[g_unit(s, v, 2 * h + 1, i)]);
                    mma6_fresh(at, b, acc[v >> 1][v & 1]);
                }
            } else {
                AFrag bb[2];
#pragma unroll
                for (int u = 0; u < 2; u++)
                    if (u < nact_c) bb[u] = split8(B[g_unit(s, 2 * wk + u, 2 * h, i)], B[g_unit(s, 2 * wk + u, 2 * h + 1, i)]);
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    if (t >= nact_r) continue;
                    const float4 a0 = A[g_unit(s, 4 * wn + t, 2 * h, i)], a1 = A[g_unit(s, 4 * wn + t, 2 * h + 1, i)];
                    if (bias_wave) bs[t] += sum8(a0, a1);
                    const AFrag at = split8(a0, a1);
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        if (u >= nact_c) continue;
                        mma6_fresh(at, bb[u], acc[t][u]);
                    }
                }
            }
        }
    }
    float *slab = slabs + (size_t)blockIdx.x * SLAB;
    // rows past nrows / cols past krows hold garbage that k_dw_reduce never reads
    if (NARROW) {
        const float v0 = bs[0] + __shfl_xor(bs[0], 32);
        if (h == 0) slab[WT * WT + 32 * wave + i] = v0;
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int nb = 32 * wave, kb = 32 * v;
#pragma unroll
            for (int r = 0; r < 16; r++) slab[(nb + TileAddr::row(r) + 4 * h) * WT + kb + i] = acc[v >> 1][v & 1][r];
        }
        return;
    }
    if (bias_wave) {
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const float v = bs[t] + __shfl_xor(bs[t], 32);
            if (h == 0) slab[WT * WT + 128 * wn + 32 * t + i] = v;
        }
    }
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int nb = 128 * wn + 32 * t, kb = 64 * wk + 32 * u;
#pragma unroll
            for (int r = 0; r < 16; r++) slab[(nb + TileAddr::row(r) + 4 * h) * WT + kb + i] = acc[t][u][r];
        }
}

__global__ __launch_bounds__(DW_THREADS) void k_dwg(WJobs JT, size_t Ns, const float *__restrict__ dz,
                                                    const float *__restrict__ saved, float *__restrict__ slabs) {
    extern __shared__ float4 dwg_lds[];
    WJob J = JT.j[0];
#pragma unroll
    for (int q = 1; q < MAXJ; q++)
        if (q < JT.n && (int)blockIdx.x >= JT.j[q].block0) J = JT.j[q];
    if (J.narrow)
        dwg_tile<true>(J, Ns, dz, saved, slabs, dwg_lds);
    else
        dwg_tile<false>(J, Ns, dz, saved, slabs, dwg_lds);
}

// ------------------------------------------------------------------------------------------------
// dW = dZ X^T on split bf16 (k_dws, the default dW). Per job tile (<= 256 dZ rows x 256 X rows) and
// 32-point chunk, each wave owns 32 rows of ONE operand ("private": loaded, split and kept as MFMA
// fragments in its own registers) against all rows of the other ("shared": staged by the whole
// workgroup, split once, through LDS):
//   COL (krows = 256 jobs): private = X rows 32 w..+31 (B fragments), shared = dZ rows (A, NS tiles)
//   ROW (krows <= 96 jobs): private = dZ rows 32 w..+31 (A fragments), shared = X rows (B, NS tiles)
// so every fp32 value is split exactly once per workgroup and only the shared operand makes the LDS
// round trip (k_dwg split each fragment in every wave reading it; k_dw split once but through LDS
// for both operands). Per chunk: split the private registers -> fragments | MFMAs on LDS buffer c & 1
// with the next chunk's shared split (3 ds_write_b64 per float4) and loads interleaved | ONE barrier.
//   LDS: split planes in fragment order, unit (16 B) [split][k-step][32-row block][lane = 32 h + i]
//   (row i, points 8h..8h+7): a fragment is one conflict-free ds_read_b128 per split; 2 x 48 KiB.
//   Numerics: each tile's twelve products of a chunk (per k-step the five corrections, then hh) go
//   into a fresh accumulator T, added to the running sum in fp32 (tools/mfma_accum_probe.hip: a
//   long running MFMA C loses the low bits of small terms with a bias; within one chunk's T that
//   loss stays below fp32's own rounding of T).
// Same job plan, slab layout and k_dw_reduce as the fp32 k_dw.
// ------------------------------------------------------------------------------------------------
constexpr int S_UNITS = NSPLIT * 2 * 8 * 64;  // 16-B units per chunk buffer
constexpr int S_NBUF = 2;
constexpr int S_LDS = S_NBUF * S_UNITS * 16;  // bytes (96 / 144 KiB)
static_assert(S_LDS <= 160 * 1024, "dWs LDS");

// unit of (split p, k-step ks, row block rb, point half hh, row i): each 32-unit half is rotated
// by 4 ks + 2 hh, so the row-major staging stores (8 lanes per row: all (ks, hh, 8-byte half)
// combinations of 2 rows per 16-lane group) hit 32 distinct banks; a fragment read stays one
// conflict-free 1 KiB ds_read_b128
__device__ __forceinline__ constexpr int s_unit(int p, int ks, int rb, int hh, int i) {
    return ((p * 2 + ks) * 8 + rb) * 64 + 32 * hh + ((i + 4 * ks + 2 * hh) & 31);
}

__device__ __forceinline__ AFrag s_frag(const bf16x8 *L, int ks, int rb, int lane) {
    const int hh = lane >> 5, i = lane & 31;
    return AFrag{L[s_unit(0, ks, rb, hh, i)], L[s_unit(1, ks, rb, hh, i)], L[s_unit(2, ks, rb, hh, i)]};
}

// one k-step's six products into t (the five corrections first)
__device__ __forceinline__ f32x16 mma6_into(const AFrag &a, const AFrag &b, f32x16 t) {
    t = MFMA32(a.m, b.m, t);
    t = MFMA32(a.h, b.l, t);
    t = MFMA32(a.l, b.h, t);
    t = MFMA32(a.h, b.m, t);
    t = MFMA32(a.m, b.h, t);
    return MFMA32(a.h, b.h, t);
}

// acc += t (v_pk_add_f32 or v_add_f32: measured alike here)
__device__ __forceinline__ void add16(f32x16 &acc, const f32x16 &t) { acc += t; }

template <bool COL, int NS>
__device__ __forceinline__ void dws_run(const WJob &J, size_t Ns, const float *__restrict__ dz,
                                        const float *__restrict__ saved, float *__restrict__ slabs, bf16x8 *lds) {
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
    const int pvoff = ((32 * wave + i) * (int)Ns + 8 * h) * 4;
    float4 pr[4];  // [k-step][half]
#define DWS_C(c) (c)
    auto pload = [&](int c) {
#pragma unroll
        for (int q = 0; q < 4; q++)
            pr[q] = __builtin_bit_cast(float4,
                                       __builtin_amdgcn_raw_buffer_load_b128(rsP, pvoff, DWS_C(c) * 128 + (q >> 1) * 64 + (q & 1) * 16, 0));
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
                    float4, __builtin_amdgcn_raw_buffer_load_b128(rsS, (row * (int)Ns + 4 * q) * 4, DWS_C(c) * 128, 0));
        }
    };
    float bsum[NSF] = {};  // COL: bias row sums of the staged dZ rows; ROW: bsum[0] of the private row
    char *lb = reinterpret_cast<char *>(lds);
    // `live`: the staged chunk is a real one (the last chunk re-splits a stale copy into the buffer
    // nobody reads again; it must not count in the bias sums)
    auto sput = [&](int f, int buf, bool live) {
        int row, q;
        if (!sslot(f, row, q)) return;
        const float4 v = st[f];
        if (COL) bsum[f] += live ? (v.x + v.y) + (v.z + v.w) : 0.f;
        const Split4 s = split4(v.x, v.y, v.z, v.w);
        char *p = lb + buf * (S_UNITS * 16) +
                  s_unit(0, q >> 2, row >> 5, (q >> 1) & 1, row & 31) * 16 + 8 * (q & 1);
        *reinterpret_cast<bf16x4 *>(p) = s.h;
        *reinterpret_cast<bf16x4 *>(p + 2 * 8 * 64 * 16) = s.m;
        *reinterpret_cast<bf16x4 *>(p + 2 * 2 * 8 * 64 * 16) = s.l;
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
        const bf16x8 *L = lds + buf * S_UNITS;
        const bool more = c + 1 < c1;
        if (pact) {
            // private fragments of this chunk, then the private loads of the next (in flight for
            // the whole chunk)
            AFrag pf0 = split8(pr[0], pr[1]), pf1 = split8(pr[2], pr[3]);
            if (!COL) bsum[0] += sum8(pr[0], pr[1]) + sum8(pr[2], pr[3]);
            pload(min(c + 1, c1 - 1));
#pragma unroll
            for (int s = 0; s < NS; s++) {
                // the tile's two k-steps into a fresh accumulator, one shared fragment live at a time
                const AFrag s0 = s_frag(L, 0, s, lane);
                f32x16 T = COL ? mma6_into(s0, pf0, (f32x16)(0.f)) : mma6_into(pf0, s0, (f32x16)(0.f));
                const AFrag s1 = s_frag(L, 1, s, lane);
                add16(acc[s], COL ? mma6_into(s1, pf1, T) : mma6_into(pf1, s1, T));
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
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const int nb = COL ? 32 * s : 32 * wave, kb = COL ? 32 * wave : 32 * s;
#pragma unroll
        for (int r = 0; r < 16; r++) slab[(nb + TileAddr::row(r) + 4 * h) * WT + kb + i] = acc[s][r];
    }
}

__global__ __launch_bounds__(DW_THREADS) void k_dws(WJobs JT, size_t Ns, const float *__restrict__ dz,
                                                    const float *__restrict__ saved, float *__restrict__ slabs) {
    extern __shared__ bf16x8 dws_lds[];
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
    return P;
}

// Packing is one gather + split launch over map[i] = (parameter << 22) | element, or -1 for zero
// padding: i < nslots * 512 are the A-image elements in [k-slot][lane][8] order (each split into
// three bf16 planes of its k-slot), the rest the fp32 region. The map depends only on the flags
// (built once on the host, cached on the device).
constexpr int PACK_MAXP = 32;
constexpr int PACK_SHIFT = 22;
struct PackPtrs {
    const float *p[PACK_MAXP];
};

__global__ __launch_bounds__(256) void k_pack(const int *__restrict__ map, PackPtrs src, __bf16 *__restrict__ img,
                                              float *__restrict__ fp, int nimg, int total) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int c = map[i];
    const float v = c < 0 ? 0.f : src.p[c >> PACK_SHIFT][c & ((1 << PACK_SHIFT) - 1)];
    if (i < nimg) {
        const __bf16 hb = (__bf16)v;
        const float r = v - (float)hb;
        const __bf16 mb = (__bf16)r;
        __bf16 *d = img + (size_t)(i >> 9) * 1536 + (i & 511);  // k-slot: 3 planes of 512 bf16
        d[0] = hb;
        d[512] = mb;
        d[1024] = (__bf16)(r - (float)mb);
    } else {
        fp[i - nimg] = v;
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
static int dw_split(const Flags &F, size_t Ns, const float *dz, const float *saved, float *slabs, float *const *grads,
                    hipStream_t stream);

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

// dW arithmetic (DGS_MLP_SPLIT_DW): 3 (default) = the split-bf16 k_dws (private / shared operands,
// every value split once), 2 = the split-bf16 k_dwg (LDS-DMA staged, per-wave splits), 1 = the
// split-bf16 k_dw (VGPR staged, split phase), 0 = the fp32-input MFMA k_dw of mlp.hip, all on the
// same [rows][Ns] arrays
static int dw_mode() {
    static const int m = [] {
        const char *e = getenv("DGS_MLP_SPLIT_DW");
        return (e && e[0] >= '0' && e[0] <= '3') ? e[0] - '0' : 3;
    }();
    return m;
}
static int dw_glds(const Flags &F, size_t Ns, const float *dz, const float *saved, float *slabs, float *const *grads,
                   hipStream_t stream);
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
    if (!map) {
        set_error("dgs_deform_pack: could not allocate the pack map");
        return DGS_ERR_HIP;
    }
    const int nimg = P.nslots * 512, total = nimg + P.nf32;
    hipLaunchKernelGGL(k_pack, dim3(div_up(total, 256)), dim3(256), 0, stream, map, src,
                       reinterpret_cast<__bf16 *>(packed), packed + P.img_floats(), nimg, total);
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
    a.img = reinterpret_cast<const bf16x8 *>(packed);
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
    b.img = reinterpret_cast<const bf16x8 *>(packed);
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
            // DGS_MLP_BWD8=1: the 8-wave k_bwd8 (bitwise equal; A/B r5u: neutral, so the 16-wave kernel
            // stays the default)
            static const bool bwd8 = [] {
                const char *e = getenv("DGS_MLP_BWD8");
                return e && e[0] == '1';
            }();
            if (bwd8)
                hipLaunchKernelGGL(k_bwd8, dim3(grid), dim3(NTHR8), 0, stream, b);
            else
                hipLaunchKernelGGL(k_bwd<false>, dim3(grid), dim3(NTHR), 0, stream, b);
        }
    }
    DGS_LAUNCH_CHECK("k_bwd", false, stream);
    int rc;
    if (F.uniform_t && (dw_mode() == 1 || dw_mode() == 2)) {  // A/B variants predate the folded t_emb jobs
        set_error("dgs_deform_backward: DGS_MLP_SPLIT_DW=1/2 do not support a uniform t (folded t_emb)");
        return DGS_ERR_ARGS;
    }
    if (dw_mode() == 0)
        rc = mlp::dw_fp32(F, Ns, dz, saved, slabs, grads, stream);
    else if (dw_mode() == 1)
        rc = dw_split(F, Ns, dz, saved, slabs, grads, stream);
    else if (dw_mode() == 2)
        rc = dw_glds(F, Ns, dz, saved, slabs, grads, stream);
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

static int dw_split(const Flags &F, size_t Ns, const float *dz, const float *saved, float *slabs, float *const *grads,
                    hipStream_t stream) {
    const WPlan W = split_wplan(F);
    {
        // 144 KiB dynamic LDS: the attribute is per device, set once per (kernel, device)
        if (int rc = ensure_dynamic_lds((const void *)k_dw, DW_LDS)) return rc;
        ScopedTimer tm("mlp_dw", stream);
        hipLaunchKernelGGL(k_dw, dim3(W.nblocks), dim3(DW_THREADS), DW_LDS, stream, W.jobs, Ns, dz, saved, slabs);
    }
    DGS_LAUNCH_CHECK("k_dw", false, stream);
    return launch_dw_reduce(F, W, slabs, grads, stream);
}

static int dw_split_once(const Flags &F, size_t Ns, const float *dz, const float *saved, float *slabs,
                         float *const *grads, hipStream_t stream) {
    if ((size_t)WT * Ns * 4 >= 0x7fffffffull)  // 32-bit byte offsets of a 256-row operand
        return mlp::dw_fp32(F, Ns, dz, saved, slabs, grads, stream);
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

static int dw_glds(const Flags &F, size_t Ns, const float *dz, const float *saved, float *slabs, float *const *grads,
                   hipStream_t stream) {
    if ((size_t)WT * Ns * 4 >= 0x7fffffffull)  // buffer offsets of a 256-row tile must fit 31 bits
        return mlp::dw_fp32(F, Ns, dz, saved, slabs, grads, stream);
    const WPlan W = split_wplan(F);
    {
        // 128 KiB dynamic LDS: the attribute is per device, set once per (kernel, device)
        if (int rc = ensure_dynamic_lds((const void *)k_dwg, G_LDS)) return rc;
        ScopedTimer tm("mlp_dw", stream);
        hipLaunchKernelGGL(k_dwg, dim3(W.nblocks), dim3(DW_THREADS), G_LDS, stream, W.jobs, Ns, dz, saved, slabs);
    }
    DGS_LAUNCH_CHECK("k_dwg", false, stream);
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
