// Stable LSD radix sort of (key, u32 value) pairs for the rasterizer's binning (radix.hip): one
// histogram launch for all passes + one scatter launch per 8-bit digit pass (onesweep: decoupled
// look-back between workgroups), no memsets. Replaces hipcub::DeviceRadixSort::SortPairs for the
// depth sort (32-bit float keys) and the tile sort (16-bit tile keys); results are identical (both
// are stable sorts by the same key bits).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dgs {
namespace radix {

// Sorts n pairs (k0, v0) by key bits [0, end_bit), using (k1, v1) as the ping-pong buffers. On return
// *alt = 0 if the result is in (k0, v0), 1 if in (k1, v1). If aux_src is given, the last pass also
// writes aux_out[i] = aux_src[sorted value i]. Stream-ordered; per-device scratch is kept inside.
template <class KT>
int sort_pairs(KT *k0, KT *k1, uint32_t *v0, uint32_t *v1, int n, int end_bit, hipStream_t stream, int *alt,
               const uint32_t *aux_src = nullptr, uint32_t *aux_out = nullptr);

}  // namespace radix
}  // namespace dgs
