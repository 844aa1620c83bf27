// Row selection over many tensors in one launch: the stream compaction of densification
// (scene/gaussian_model.py:206-246 upstream layout). prune_points keeps the rows of
// ~mask of every Gaussian tensor, its two Adam moments and the densification statistics (21 tensors),
// densify_and_clone / _split gather the selected rows of the six parameters; torch does each with a
// nonzero (host sync) + index_select per tensor. Here: one exclusive scan of the mask (positions)
// and one gather launch over a table of (src, dst, row width) jobs, blocks of 256 rows x job.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <map>
#include <mutex>

#include "dgs_common.h"

namespace dgs {
namespace compact {

constexpr int MAXJ = 32;
constexpr int ROWS = 256;  // rows per block (per job)

struct Job {
    const float *src;
    float *dst;
    int width;  // floats per row
};
struct Jobs {
    Job j[MAXJ];
    int n;
};

// block (x = row block, y = job): the block's rows in order, `width` consecutive floats each, so
// reads and writes are contiguous runs of the selected rows
__global__ __launch_bounds__(256) void k_select(int nrows, const uint8_t *__restrict__ mask, const int *__restrict__ pos,
                                                Jobs J) {
    const Job jb = J.j[blockIdx.y];
    const int r0 = blockIdx.x * ROWS;
    const int nr = min(ROWS, nrows - r0);
    const long long ne = (long long)nr * jb.width;
    for (long long e = threadIdx.x; e < ne; e += blockDim.x) {
        const int r = r0 + (int)(e / jb.width), c = (int)(e % jb.width);
        if (mask[r]) jb.dst[(long long)pos[r] * jb.width + c] = jb.src[(long long)r * jb.width + c];
    }
}

struct ToInt {  // the scan accumulates in int, not in the mask's byte type
    __host__ __device__ int operator()(uint8_t v) const { return v ? 1 : 0; }
};

std::mutex g_mu;
// per (device, stream): scan temp storage + positions (launches sharing one run in stream order)
std::map<std::pair<int, hipStream_t>, std::pair<void *, size_t>> g_tmp;

}  // namespace compact
}  // namespace dgs

using namespace dgs;

extern "C" int dgs_select_rows(int nrows, const uint8_t *mask, int njobs, const dgs_row_job *jobs, void *stream_) {
    if (nrows < 0 || njobs < 0 || (njobs > 0 && !jobs) || (nrows > 0 && !mask)) {
        set_error("dgs_select_rows: bad arguments");
        return DGS_ERR_ARGS;
    }
    for (int k = 0; k < njobs; k++)
        if (jobs[k].width <= 0 || (nrows > 0 && (!jobs[k].src || !jobs[k].dst))) {
            set_error("dgs_select_rows: bad job (width <= 0 or null pointer)");
            return DGS_ERR_ARGS;
        }
    if (nrows == 0 || njobs == 0) return DGS_OK;
    hipStream_t stream = (hipStream_t)stream_;
    int device = 0;
    DGS_HIP_CHECK(hipGetDevice(&device));
    size_t tmp = 0;
    hipcub::TransformInputIterator<int, compact::ToInt, const uint8_t *> flags(mask, compact::ToInt());
    DGS_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, flags, (int *)nullptr, nrows, stream));
    const size_t need = tmp + 256 + 4ull * nrows;
    void *buf = nullptr;
    {
        std::lock_guard<std::mutex> lk(compact::g_mu);
        auto &e = compact::g_tmp[{device, stream}];
        if (e.second < need) {
            // the previous buffer may still be read by queued launches on this stream
            if (e.first) DGS_HIP_CHECK(hipStreamSynchronize(stream));
            if (e.first) DGS_HIP_CHECK(hipFree(e.first));
            e.first = nullptr;
            e.second = 0;
            DGS_HIP_CHECK(hipMalloc(&e.first, need + need / 4));
            e.second = need + need / 4;
        }
        buf = e.first;
    }
    int *pos = (int *)((char *)buf + ((tmp + 255) / 256) * 256);
    DGS_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(buf, tmp, flags, pos, nrows, stream));
    const int nb = (nrows + compact::ROWS - 1) / compact::ROWS;
    for (int k0 = 0; k0 < njobs; k0 += compact::MAXJ) {
        compact::Jobs J{};
        J.n = std::min(compact::MAXJ, njobs - k0);
        for (int k = 0; k < J.n; k++) J.j[k] = compact::Job{jobs[k0 + k].src, jobs[k0 + k].dst, jobs[k0 + k].width};
        hipLaunchKernelGGL(compact::k_select, dim3(nb, J.n), dim3(256), 0, stream, nrows, mask, pos, J);
        DGS_LAUNCH_CHECK("k_select", false, stream);
    }
    return DGS_OK;
}
