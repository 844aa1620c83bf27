// Stable LSD radix sort of (key, u32 value) pairs on MI355X (gfx950) for the rasterizer's binning:
// the depth sort of the Gaussians (32-bit float-bit keys, 4 passes) and the stable tile sort of the
// (tile, Gaussian) pairs (16-bit keys, 12 bits: 2 passes). The reference's upstream rasterizer sorts
// with cub::DeviceRadixSort (SURVEY.md §2 kernel inventory, R2/R3); this is the build's own.
//
// Launches per sort: k_hist (the digit histograms of every pass in one sweep) + one k_scatter per
// 8-bit pass. k_scatter is a "onesweep" pass: a workgroup takes its 4096-item tile by ticket (so a
// workgroup only ever waits on tiles whose workgroups are already running), ranks the digits of the
// tile stably in registers, publishes its per-digit counts, adds up its predecessors' counts by
// decoupled look-back and scatters the tile, reordered through LDS into digit runs, to
// histogram-prefix + look-back-prefix + local rank. No memsets: the look-back words carry a
// (call, pass) tag, the histogram is double-buffered across calls (each k_hist zeroes the next
// call's), the last workgroup of a pass resets the ticket.
//   In-tile order is the input order (wave w owns items [1024 w, +1024), round r the 64 items
//   [64 r, +64) of that), so equal digits keep their order: stable.
//   Look-back words are single 8-byte agent-scope atomics, [tag 30 | flag 2 | count 32]: the handed
//   off value IS the atomic word (MI355X_MICROARCH.md, inter-workgroup visibility: 8-B agent atomics
//   both sides).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include "dgs_common.h"
#include "radix.h"

namespace dgs {
namespace radix {

constexpr int RB = 256;             // threads per workgroup
constexpr int DIG = 256;            // bins per pass
constexpr int MAXPASS = 4;
constexpr uint32_t FLAG_A = 1, FLAG_P = 2;  // look-back word: aggregate / inclusive prefix
static_assert(RB == DIG, "one thread per digit in the look-back");

__device__ inline uint64_t lb_word(uint32_t tag, uint32_t flag, uint32_t count) {
    return ((uint64_t)tag << 34) | ((uint64_t)flag << 32) | count;
}

// digit histograms of all passes; block 0 also zeroes the next call's histogram buffer
template <class KT>
__global__ __launch_bounds__(RB) void k_hist(const KT *__restrict__ keys, int n, int npass, int end_bit,
                                             uint32_t *__restrict__ hist, uint32_t *__restrict__ hist_next) {
    __shared__ uint32_t h[MAXPASS * DIG];
    for (int i = threadIdx.x; i < MAXPASS * DIG; i += RB) h[i] = 0;
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < MAXPASS * DIG; i += RB) hist_next[i] = 0;
    __syncthreads();
    // the last pass's digit is masked to the bits below end_bit, as in k_scatter
    const uint32_t lmask = end_bit - 8 * (npass - 1) >= 8 ? 255u : (1u << (end_bit - 8 * (npass - 1))) - 1u;
    for (int i = blockIdx.x * RB + threadIdx.x; i < n; i += gridDim.x * RB) {
        const uint32_t k = (uint32_t)keys[i];
        for (int p = 0; p < npass; p++)
            atomicAdd(&h[p * DIG + ((k >> (8 * p)) & (p == npass - 1 ? lmask : 255u))], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < npass * DIG; i += RB) {
        const uint32_t v = h[i];
        if (v) atomicAdd(&hist[i], v);
    }
}

// inclusive wave scan (64 lanes)
__device__ inline uint32_t wave_incl_scan(uint32_t x, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x;
}

template <class KT, int ITEMS>
__global__ __launch_bounds__(RB) void k_scatter(const KT *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                KT *__restrict__ kout, uint32_t *__restrict__ vout, int n, int shift,
                                                int bits, const uint32_t *__restrict__ hist, uint64_t *lb,
                                                uint32_t *ticket, uint32_t tag, int nblocks,
                                                const uint32_t *__restrict__ aux_src, uint32_t *__restrict__ aux_out) {
    __shared__ uint32_t s_bid;
    __shared__ uint32_t cnt[4][DIG];   // per-wave digit counts -> per-wave exclusive offsets
    __shared__ uint32_t s_bstart[DIG];  // tile-local start of each digit run
    __shared__ uint32_t s_gbase[DIG];   // global output position of each digit run of this tile
    __shared__ uint32_t s_w1[4], s_w2[4];
    constexpr int TILE = RB * ITEMS;  // items per workgroup
    __shared__ uint32_t s_key[TILE];
    __shared__ uint32_t s_val[TILE];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) {
        const uint32_t b = atomicAdd(ticket, 1u);
        if (b == (uint32_t)nblocks - 1) atomicExch(ticket, 0u);  // every other ticket is taken: reset
        s_bid = b;
    }
    for (int i = tid; i < 4 * DIG; i += RB) (&cnt[0][0])[i] = 0;
    __syncthreads();
    const int bid = (int)s_bid;
    const int base = bid * TILE + w * (TILE / 4);
    const uint32_t mask = (1u << bits) - 1u;
    const uint64_t lanes_lt = (1ull << lane) - 1ull;
    uint32_t key[ITEMS], val[ITEMS], rank[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const int pos = base + 64 * r + lane;
        key[r] = pos < n ? (uint32_t)kin[pos] : 0u;
        val[r] = pos < n ? vin[pos] : 0u;
    }
    // stable in-wave ranking: lanes holding the same digit found by one ballot per digit bit; the
    // lowest such lane advances the wave's counter for the digit
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const bool ok = base + 64 * r + lane < n;
        const uint32_t d = (key[r] >> shift) & mask;
        uint64_t m = __ballot(ok);
        for (int b = 0; b < bits; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
        const int leader = m ? __ffsll((unsigned long long)m) - 1 : 0;
        uint32_t b0 = 0;
        if (ok && lane == leader) {
            b0 = cnt[w][d];
            cnt[w][d] = b0 + (uint32_t)__popcll(m);
        }
        b0 = (uint32_t)__shfl((int)b0, leader);
        rank[r] = b0 + (uint32_t)__popcll(m & lanes_lt);
    }
    __syncthreads();
    {
        const int d = tid;  // one thread per digit
        uint32_t total = 0;
#pragma unroll
        for (int ww = 0; ww < 4; ww++) {
            const uint32_t c = cnt[ww][d];
            cnt[ww][d] = total;
            total += c;
        }
        const uint32_t hv = hist[d];
        const uint32_t xs = wave_incl_scan(total, lane), hs = wave_incl_scan(hv, lane);
        if (lane == 63) {
            s_w1[w] = xs;
            s_w2[w] = hs;
        }
        // publish this tile's count for the digit before waiting on anything
        __hip_atomic_store(&lb[(size_t)bid * DIG + d], lb_word(tag, FLAG_A, total), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        uint32_t o1 = 0, o2 = 0;
        for (int ww = 0; ww < w; ww++) {
            o1 += s_w1[ww];
            o2 += s_w2[ww];
        }
        s_bstart[d] = o1 + xs - total;
        // decoupled look-back: predecessors' counts until an inclusive prefix, 8 words in flight per
        // round (consumed nearest first; a not-yet-published word ends the round and is re-read)
        constexpr int LBW = 8;
        uint32_t prefix = 0;
        for (int b = bid - 1; b >= 0;) {
            uint64_t v[LBW];
#pragma unroll
            for (int k = 0; k < LBW; k++)
                v[k] = b - k >= 0 ? __hip_atomic_load(&lb[(size_t)(b - k) * DIG + d], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT)
                                  : 0ull;
            bool stop = false, wait = false;
#pragma unroll
            for (int k = 0; k < LBW; k++) {
                if (stop || wait || b < 0) continue;
                const uint32_t f = (uint32_t)(v[k] >> 32) & 3u;
                if ((uint32_t)(v[k] >> 34) != tag || f == 0u) {
                    wait = true;
                    continue;
                }
                prefix += (uint32_t)v[k];
                if (f == FLAG_P) stop = true;
                else b--;
            }
            if (stop) break;
            if (wait) __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(&lb[(size_t)bid * DIG + d], lb_word(tag, FLAG_P, prefix + total), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        s_gbase[d] = (o2 + hs - hv) + prefix;
    }
    __syncthreads();
    // reorder the tile into digit runs (LDS), then write each run contiguously
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        if (base + 64 * r + lane >= n) continue;
        const uint32_t d = (key[r] >> shift) & mask;
        const uint32_t li = s_bstart[d] + cnt[w][d] + rank[r];
        s_key[li] = key[r];
        s_val[li] = val[r];
    }
    __syncthreads();
    const int nvalid = min(TILE, n - bid * TILE);
    for (int i = tid; i < nvalid; i += RB) {
        const uint32_t k = s_key[i], v = s_val[i];
        const uint32_t d = (k >> shift) & mask;
        const uint32_t o = s_gbase[d] + ((uint32_t)i - s_bstart[d]);
        kout[o] = (KT)k;
        vout[o] = v;
        if (aux_out) aux_out[o] = aux_src[v];
    }
}

// ------------------------------------------------------------------------------------------------
// host: scratch (histograms, tickets, look-back words) per (device, stream) and the launch sequence.
// Calls that share a scratch run in stream order, so a k_scatter's tickets, look-back tags and
// histogram buffers are never touched by another launch while it runs; sorts on two streams at once
// (two rasterizer contexts on different streams) use two scratches.
// ------------------------------------------------------------------------------------------------
struct State {
    uint32_t *hist = nullptr;    // [2][MAXPASS][DIG]
    uint32_t *ticket = nullptr;  // [MAXPASS]
    uint64_t *lb = nullptr;      // [blocks][DIG]
    int lb_blocks = 0;
    uint32_t gen = 0;
};
static std::mutex g_mu;
static std::map<std::pair<int, hipStream_t>, State> g_state;

// items per thread of k_scatter (a workgroup's tile = 256 x items): small tiles for small sorts so
// a pass has enough workgroups; DGS_RADIX_ITEMS (4 / 8 / 16) overrides (tuning)
static int radix_items(int n) {
    static const int forced = [] {
        const char *e = getenv("DGS_RADIX_ITEMS");
        const int v = e ? atoi(e) : 0;
        return (v == 4 || v == 8 || v == 16) ? v : 0;
    }();
    if (forced) return forced;
    return n <= (1 << 19) ? 4 : 8;
}

template <class KT>
int sort_pairs(KT *k0, KT *k1, uint32_t *v0, uint32_t *v1, int n, int end_bit, hipStream_t stream, int *alt,
               const uint32_t *aux_src, uint32_t *aux_out) {
    *alt = 0;
    if (n <= 0 || end_bit <= 0) return DGS_OK;
    const int npass = std::min(MAXPASS, div_up(end_bit, 8));
    const int nblocks = div_up(n, RB * radix_items(n));
    int device = 0;
    DGS_HIP_CHECK(hipGetDevice(&device));
    std::lock_guard<std::mutex> lk(g_mu);
    State &S = g_state[{device, stream}];
    if (!S.hist) {
        DGS_HIP_CHECK(hipMalloc(&S.hist, sizeof(uint32_t) * 2 * MAXPASS * DIG));
        DGS_HIP_CHECK(hipMalloc(&S.ticket, sizeof(uint32_t) * MAXPASS));
        DGS_HIP_CHECK(hipMemsetAsync(S.hist, 0, sizeof(uint32_t) * 2 * MAXPASS * DIG, stream));
        DGS_HIP_CHECK(hipMemsetAsync(S.ticket, 0, sizeof(uint32_t) * MAXPASS, stream));
    }
    if (S.lb_blocks < nblocks) {
        if (S.lb) {
            DGS_HIP_CHECK(hipStreamSynchronize(stream));  // growth only: no launch may still use the old words
            DGS_HIP_CHECK(hipFree(S.lb));
        }
        const int nb = nblocks + nblocks / 4 + 16;
        DGS_HIP_CHECK(hipMalloc(&S.lb, sizeof(uint64_t) * (size_t)nb * DIG));
        DGS_HIP_CHECK(hipMemsetAsync(S.lb, 0, sizeof(uint64_t) * (size_t)nb * DIG, stream));  // tag 0: never used
        S.lb_blocks = nb;
    }
    const int items = radix_items(n);
    S.gen = (S.gen + 1) & 0x0fffffffu;
    if (S.gen == 0) S.gen = 1;
    uint32_t *hcur = S.hist + (S.gen & 1) * MAXPASS * DIG, *hnext = S.hist + ((S.gen + 1) & 1) * MAXPASS * DIG;
    hipLaunchKernelGGL(k_hist<KT>, dim3(std::min(256, div_up(n, RB * 8))), dim3(RB), 0, stream, k0, n, npass, end_bit,
                       hcur, hnext);
    DGS_LAUNCH_CHECK("radix::k_hist", false, stream);
    KT *ki = k0, *ko = k1;
    uint32_t *vi = v0, *vo = v1;
    for (int p = 0; p < npass; p++) {
        const bool last = p == npass - 1;
        const int bits = std::min(8, end_bit - 8 * p);
        const uint32_t tag = (S.gen * 4u + (uint32_t)p) & 0x3fffffffu;
        const uint32_t *as = last ? aux_src : nullptr;
        uint32_t *ao = last ? aux_out : nullptr;
        if (items == 16)
            hipLaunchKernelGGL((k_scatter<KT, 16>), dim3(nblocks), dim3(RB), 0, stream, ki, vi, ko, vo, n, 8 * p, bits,
                               hcur + p * DIG, S.lb, S.ticket + p, tag, nblocks, as, ao);
        else if (items == 8)
            hipLaunchKernelGGL((k_scatter<KT, 8>), dim3(nblocks), dim3(RB), 0, stream, ki, vi, ko, vo, n, 8 * p, bits,
                               hcur + p * DIG, S.lb, S.ticket + p, tag, nblocks, as, ao);
        else
            hipLaunchKernelGGL((k_scatter<KT, 4>), dim3(nblocks), dim3(RB), 0, stream, ki, vi, ko, vo, n, 8 * p, bits,
                               hcur + p * DIG, S.lb, S.ticket + p, tag, nblocks, as, ao);
        DGS_LAUNCH_CHECK("radix::k_scatter", false, stream);
        std::swap(ki, ko);
        std::swap(vi, vo);
    }
    *alt = npass & 1;
    return DGS_OK;
}

template int sort_pairs<uint32_t>(uint32_t *, uint32_t *, uint32_t *, uint32_t *, int, int, hipStream_t, int *,
                                  const uint32_t *, uint32_t *);
template int sort_pairs<uint16_t>(uint16_t *, uint16_t *, uint32_t *, uint32_t *, int, int, hipStream_t, int *,
                                  const uint32_t *, uint32_t *);

}  // namespace radix
}  // namespace dgs

// include/dgs.h test hook: the sort with its result copied back into (k0, v0)
extern "C" int dgs_debug_sort_pairs(void *k0, void *k1, uint32_t *v0, uint32_t *v1, int n, int key_bytes, int end_bit,
                                    void *stream_) {
    using namespace dgs;
    hipStream_t stream = (hipStream_t)stream_;
    if (n < 0 || !k0 || !k1 || !v0 || !v1 || (key_bytes != 2 && key_bytes != 4) || end_bit < 0 ||
        end_bit > 8 * key_bytes) {
        set_error("dgs_debug_sort_pairs: bad argument");
        return DGS_ERR_ARGS;
    }
    int alt = 0, rc;
    if (key_bytes == 4)
        rc = radix::sort_pairs<uint32_t>((uint32_t *)k0, (uint32_t *)k1, v0, v1, n, end_bit, stream, &alt);
    else
        rc = radix::sort_pairs<uint16_t>((uint16_t *)k0, (uint16_t *)k1, v0, v1, n, end_bit, stream, &alt);
    if (rc != DGS_OK || !alt) return rc;
    DGS_HIP_CHECK(hipMemcpyAsync(k0, k1, (size_t)n * key_bytes, hipMemcpyDeviceToDevice, stream));
    DGS_HIP_CHECK(hipMemcpyAsync(v0, v1, (size_t)n * 4, hipMemcpyDeviceToDevice, stream));
    return DGS_OK;
}
