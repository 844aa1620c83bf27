// Error reporting, version and the kernel-timing hooks of libdgs_hip.so.
#include <hip/hip_runtime.h>

#include <map>
#include <set>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "dgs_common.h"

namespace dgs {
namespace {
thread_local std::string g_err;
std::mutex g_tmu;
bool g_timing = false;
std::set<std::string> g_timing_sel;  // empty = every class
struct Pending {
    std::string name;
    hipEvent_t a, b;
};
std::vector<Pending> g_pending;
std::vector<hipEvent_t> g_free_events;
std::map<std::string, std::pair<double, int>> g_acc;
int g_period = 1;                      // time every g_period-th launch of a class (dgs_timing_sample)
std::map<std::string, long long> g_seen;  // launches of each selected class since the last reset

hipEvent_t take_event() {
    if (!g_free_events.empty()) {
        hipEvent_t e = g_free_events.back();
        g_free_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

void drain_locked() {
    for (auto &p : g_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            auto &a = g_acc[p.name];
            a.first += ms;
            a.second += 1;
        }
        g_free_events.push_back(p.a);
        g_free_events.push_back(p.b);
    }
    g_pending.clear();
}
}  // namespace

void set_error(const std::string &msg) { g_err = msg; }

int ensure_dynamic_lds(const void *kernel, int bytes) {
    static std::mutex mu;
    static std::set<std::tuple<const void *, int, int>> done;  // (kernel, device, bytes)
    int device = 0;
    DGS_HIP_CHECK(hipGetDevice(&device));
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(kernel, device, bytes);
    if (done.count(key)) return DGS_OK;
    DGS_HIP_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    done.insert(key);
    return DGS_OK;
}

ScopedTimer::ScopedTimer(const char *n, hipStream_t s) : name(n), stream(s), ev0(nullptr) {
    if (!g_timing) return;
    std::lock_guard<std::mutex> lk(g_tmu);
    if (!g_timing_sel.empty() && !g_timing_sel.count(n)) return;
    // each event record is a stream marker (~6 us of GPU idle): sampled launches only
    if ((g_seen[n]++ % g_period) != 0) return;
    hipEvent_t e = take_event();
    (void)hipEventRecord(e, stream);
    ev0 = (void *)e;
}

ScopedTimer::~ScopedTimer() {
    if (!ev0) return;
    std::lock_guard<std::mutex> lk(g_tmu);
    hipEvent_t e = take_event();
    (void)hipEventRecord(e, stream);
    g_pending.push_back({name, (hipEvent_t)ev0, e});
    if (g_pending.size() > 4096) drain_locked();
}

}  // namespace dgs

extern "C" const char *dgs_last_error(void) { return dgs::g_err.c_str(); }
extern "C" const char *dgs_version(void) { return "libdgs_hip 0.1 (gfx950)"; }

extern "C" void dgs_timing_enable(int on) {
    std::lock_guard<std::mutex> lk(dgs::g_tmu);
    dgs::g_timing = on != 0;
}

extern "C" void dgs_timing_select(const char *csv) {
    std::lock_guard<std::mutex> lk(dgs::g_tmu);
    dgs::g_timing_sel.clear();
    if (!csv) return;
    std::string cur;
    for (const char *p = csv;; p++) {
        if (*p == ',' || *p == 0) {
            if (!cur.empty()) dgs::g_timing_sel.insert(cur);
            cur.clear();
            if (*p == 0) break;
        } else {
            cur += *p;
        }
    }
}

extern "C" double dgs_timing_query(const char *name, int *launches) {
    std::lock_guard<std::mutex> lk(dgs::g_tmu);
    dgs::drain_locked();
    auto it = dgs::g_acc.find(name);
    if (it == dgs::g_acc.end()) {
        if (launches) *launches = 0;
        return 0.0;
    }
    if (launches) *launches = it->second.second;
    return it->second.first;
}

extern "C" long long dgs_timing_launches(const char *name) {
    std::lock_guard<std::mutex> lk(dgs::g_tmu);
    auto it = dgs::g_seen.find(name);
    return it == dgs::g_seen.end() ? 0 : it->second;
}

extern "C" void dgs_timing_reset(void) {
    std::lock_guard<std::mutex> lk(dgs::g_tmu);
    dgs::drain_locked();
    dgs::g_acc.clear();
    dgs::g_seen.clear();
}

extern "C" void dgs_timing_sample(int period) {
    std::lock_guard<std::mutex> lk(dgs::g_tmu);
    dgs::g_period = period < 1 ? 1 : period;
}

// ------------------------------------------------------------------------------------------------
// Stand-in for the data-parallel step's gradient all-reduce (tools/overlap_probe.py):
// the one-GPU box cannot run RCCL with two ranks, so the question "does a collective get compute
// units while the persistent MLP grid runs phase 2" is asked with a kernel shaped like an RCCL ring
// all-reduce: `nwg` workgroups of 256 threads (RCCL's channel count) streaming `passes` read-modify-
// write sweeps over the gradient buffer (a ring all-reduce reads and writes each element about twice:
// reduce-scatter, all-gather). Values: x <- 0.5 x + 0.5 x = x per sweep (the buffer is left unchanged
// up to rounding, so a probe can run it on live gradients).
// ------------------------------------------------------------------------------------------------
namespace dgs {
namespace {
__global__ __launch_bounds__(256) void k_collective_standin(float4 *__restrict__ buf, long long n4, int passes) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (int p = 0; p < passes; p++)
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
            float4 v = buf[i];
            v.x = 0.5f * v.x + 0.5f * v.x;
            v.y = 0.5f * v.y + 0.5f * v.y;
            v.z = 0.5f * v.z + 0.5f * v.z;
            v.w = 0.5f * v.w + 0.5f * v.w;
            buf[i] = v;
        }
}
}  // namespace
}  // namespace dgs

extern "C" int dgs_debug_collective_standin(float *buf, long long n, int nwg, int passes, void *stream_) {
    if (!buf || n < 0 || nwg <= 0 || nwg > 4096 || passes <= 0 || (reinterpret_cast<uintptr_t>(buf) & 15)) {
        dgs::set_error("dgs_debug_collective_standin: bad argument (16-byte aligned buffer, 0 < nwg <= 4096)");
        return DGS_ERR_ARGS;
    }
    hipStream_t stream = (hipStream_t)stream_;
    const long long n4 = n / 4;
    if (n4 == 0) return DGS_OK;
    hipLaunchKernelGGL(dgs::k_collective_standin, dim3(nwg), dim3(256), 0, stream,
                       reinterpret_cast<float4 *>(buf), n4, passes);
    DGS_LAUNCH_CHECK("k_collective_standin", false, stream);
    return DGS_OK;
}
