// Shared helpers for libdgs_hip.so (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/dgs.h"

namespace dgs {

void set_error(const std::string &msg);

#define DGS_HIP_CHECK(expr)                                                                  \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) {                                                              \
            ::dgs::set_error(std::string(#expr) + " failed: " + hipGetErrorString(_e) +      \
                             " (" __FILE__ ":" + std::to_string(__LINE__) + ")");            \
            return DGS_ERR_HIP;                                                              \
        }                                                                                    \
    } while (0)

#define DGS_LAUNCH_CHECK(name, debug, stream)                                                \
    do {                                                                                     \
        hipError_t _e = hipGetLastError();                                                   \
        if (_e == hipSuccess && (debug)) _e = hipStreamSynchronize(stream);                  \
        if (_e != hipSuccess) {                                                              \
            ::dgs::set_error(std::string("kernel ") + name + ": " + hipGetErrorString(_e));  \
            return DGS_ERR_HIP;                                                              \
        }                                                                                    \
    } while (0)

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) applies to the current device: set it once per
// (kernel, device) under a lock, so a process driving several GPUs, or several host threads, never
// launches a kernel on a device where the attribute is missing.
int ensure_dynamic_lds(const void *kernel, int bytes);

// Kernel timing (bench.py roofline): events recorded around selected launches on their stream.
struct ScopedTimer {
    const char *name;
    hipStream_t stream;
    void *ev0;
    ScopedTimer(const char *n, hipStream_t s);
    ~ScopedTimer();
};

constexpr int WAVE = 64;
constexpr int TILE_X = 16;
constexpr int TILE_Y = 16;
constexpr int TILE_PIX = TILE_X * TILE_Y;

__host__ __device__ inline int div_up(int a, int b) { return (a + b - 1) / b; }

}  // namespace dgs
