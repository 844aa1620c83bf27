// Fused photometric loss for MI355X: L = (1-l) * mean|I-G| + l * (1 - mean SSIM(I,G)) and dL/dI.
// Replaces utils/loss_utils.py:18-73 (l1_loss + ssim: 11x11 Gaussian window sigma 1.5, zero-padded
// 'same' depthwise conv2d, C1 = 0.01^2, C2 = 0.03^2) inside the training step
// (train_baseline.py:126-128), which PyTorch runs as 5+3 MIOpen convolutions per direction.
//
// The 2-D window is the outer product of the 1-D one, so every filtered map is a separable
// 11-tap row pass + 11-tap column pass through LDS (32x32 output tile, 42x42 halo tile; each thread
// keeps a register window per pass: 18 inputs for 8 row outputs, 14 for 4 column outputs).
// Forward: 5 maps (mu1, mu2, E[I^2], E[G^2], E[IG]) -> per pixel SSIM and the three coefficient
// maps A, B, C of dSSIM/d(mu1, E[I^2], E[IG]) -> HBM; per-block partial sums (deterministic).
// Backward: dSSIM_sum/dI = w*A + 2 I (w*B) + G (w*C) (window symmetric), plus the L1 sign term.
#include <hip/hip_runtime.h>

#include <cstring>

#include "dgs_common.h"

namespace dgs {
namespace ssim {

constexpr int T = 32;            // output tile (32 x 32 pixels per 256-thread workgroup)
constexpr int R = 5;             // window radius
constexpr int S = T + 2 * R;     // 42: input tile with halo
constexpr int SP = S + 1;        // padded LDS row of the input tile
constexpr int HP = T + 1;        // padded LDS row of the row-filtered maps
constexpr int HX = 8;            // row pass: outputs per thread (one row, 8 columns: 168 items)
constexpr int VY = 4;            // column pass: outputs per thread (one column, 4 rows: 256 items)
constexpr float C1 = 0.01f * 0.01f;
constexpr float C2 = 0.03f * 0.03f;

struct Win {
    float w[11];
};

__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// NM maps of the halo tile (zero outside the image) from `src` planes (plane stride `plane`) into
// LDS, 42 x 42 each. Every load of the thread is issued before the first LDS store (unrolled: a
// rolled loop waited out one HBM round trip per 256 elements, 7 in a row)
template <int NM>
__device__ __forceinline__ void load_tile(float (*sm)[S][SP], const float *const src[NM], int H, int W, int x0,
                                          int y0) {
    constexpr int NIT = (S * S + 255) / 256;
    float v[NIT][NM];
#pragma unroll
    for (int it = 0; it < NIT; it++) {
        const int e = threadIdx.x + 256 * it;
        const int ly = e / S, lx = e - ly * S;
        const int gy = y0 + ly - R, gx = x0 + lx - R;
        const bool in = e < S * S && gy >= 0 && gy < H && gx >= 0 && gx < W;
        const size_t p = in ? (size_t)gy * W + gx : 0;
#pragma unroll
        for (int q = 0; q < NM; q++) v[it][q] = in ? src[q][p] : 0.f;
    }
#pragma unroll
    for (int it = 0; it < NIT; it++) {
        const int e = threadIdx.x + 256 * it;
        const int ly = e / S, lx = e - ly * S;
        if (e < S * S)
#pragma unroll
            for (int q = 0; q < NM; q++) sm[q][ly][lx] = v[it][q];
    }
}

// forward: 5 maps (mu1, mu2, E[I^2], E[G^2], E[IG]); the products are formed on the fly from the two
// input tiles. Row pass: each item = one tile row x 8 columns from 18 inputs held in registers;
// column pass: each thread slides 14 row-filtered values down one column for 4 outputs.
// block (tile) partial sums: [blocks][2] = (sum |I-G|, sum ssim)
__global__ __launch_bounds__(256) void k_ssim_fwd(int H, int W, const float *__restrict__ I, const float *__restrict__ G,
                                                  Win win, float *__restrict__ maps, float *__restrict__ partial) {
    __shared__ float sx[2][S][SP];
    __shared__ float hq[5][S][HP];
    __shared__ float red[2][4];
    const int c = blockIdx.z;
    const int x0 = blockIdx.x * T, y0 = blockIdx.y * T;
    const int tid = threadIdx.x;
    const size_t plane = (size_t)H * W;
    const float *src[2] = {I + c * plane, G + c * plane};
    load_tile<2>(sx, src, H, W, x0, y0);
    __syncthreads();
    if (tid < S * (T / HX)) {
        const int ly = tid / (T / HX), lx0 = (tid % (T / HX)) * HX;
        float a[HX + 10], b[HX + 10];
#pragma unroll
        for (int k = 0; k < HX + 10; k++) {
            a[k] = sx[0][ly][lx0 + k];
            b[k] = sx[1][ly][lx0 + k];
        }
#pragma unroll
        for (int j = 0; j < HX; j++) {
            float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f, m4 = 0.f;
#pragma unroll
            for (int k = 0; k < 11; k++) {
                const float i = a[j + k], g = b[j + k], w = win.w[k];
                m0 += w * i;
                m1 += w * g;
                m2 += w * (i * i);
                m3 += w * (g * g);
                m4 += w * (i * g);
            }
            hq[0][ly][lx0 + j] = m0; hq[1][ly][lx0 + j] = m1; hq[2][ly][lx0 + j] = m2;
            hq[3][ly][lx0 + j] = m3; hq[4][ly][lx0 + j] = m4;
        }
    }
    __syncthreads();
    const int lx = tid % T, ly0 = (tid / T) * VY;
    const int x = x0 + lx;
    float mu[5][VY];
#pragma unroll
    for (int m = 0; m < 5; m++) {
        float v[VY + 10];
#pragma unroll
        for (int k = 0; k < VY + 10; k++) v[k] = hq[m][ly0 + k][lx];
#pragma unroll
        for (int j = 0; j < VY; j++) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < 11; k++) acc += win.w[k] * v[j + k];
            mu[m][j] = acc;
        }
    }
    float l1 = 0.f, s = 0.f;
#pragma unroll
    for (int j = 0; j < VY; j++) {
        const int y = y0 + ly0 + j;
        if (x < W && y < H) {
            const float mu1 = mu[0][j], mu2 = mu[1][j];
            const float mu1s = mu1 * mu1, mu2s = mu2 * mu2, mu12 = mu1 * mu2;
            const float s11 = mu[2][j] - mu1s, s22 = mu[3][j] - mu2s, s12 = mu[4][j] - mu12;
            const float n1 = 2.f * mu12 + C1, n2 = 2.f * s12 + C2;
            const float d1 = mu1s + mu2s + C1, d2 = s11 + s22 + C2;
            const float inv = 1.f / (d1 * d2);
            const float sv = n1 * n2 * inv;
            const float A = 2.f * mu2 * n2 * inv - 2.f * mu1 * sv / d1 + 2.f * mu1 * sv / d2 - mu2 * 2.f * n1 * inv;
            const float B = -sv / d2;
            const float Cc = 2.f * n1 * inv;
            const size_t p = (size_t)y * W + x;
            maps[(3 * c + 0) * plane + p] = A;
            maps[(3 * c + 1) * plane + p] = B;
            maps[(3 * c + 2) * plane + p] = Cc;
            l1 += fabsf(sx[0][ly0 + j + R][lx + R] - sx[1][ly0 + j + R][lx + R]);
            s += sv;
        }
    }
    l1 = wave_sum(l1);
    s = wave_sum(s);
    const int wv = tid >> 6;
    if ((tid & 63) == 0) {
        red[0][wv] = l1;
        red[1][wv] = s;
    }
    __syncthreads();
    if (tid == 0) {
        size_t b = ((size_t)c * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        partial[2 * b] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
        partial[2 * b + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    }
}

// (Round 5 tried this reduction in k_ssim_fwd's last workgroup — ticket, sc1 partials — to save the
// launch: fwd + final 0.0378 vs 0.0335 ms per step, bench kernel timers; the single workgroup's tail
// costs more than the launch boundary. Not kept.)
// out[0] = loss, out[1] = mean L1, out[2] = mean SSIM; one workgroup of 1024 (16 waves: the partial
// sums are a latency chain of double adds per thread), fixed order (deterministic)
__global__ __launch_bounds__(1024) void k_ssim_final(int nblocks, float n, float lambda, const float *__restrict__ partial,
                                                     float *__restrict__ out) {
    __shared__ double red[2][16];
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < nblocks; i += 1024) {
        a += (double)partial[2 * i];
        b += (double)partial[2 * i + 1];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = a;
        red[1][threadIdx.x >> 6] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double sa = 0.0, sb = 0.0;
        for (int w = 0; w < 16; w++) {
            sa += red[0][w];
            sb += red[1][w];
        }
        float l1 = (float)(sa / n), ss = (float)(sb / n);
        out[0] = (1.f - lambda) * l1 + lambda * (1.f - ss);
        out[1] = l1;
        out[2] = ss;
    }
}

// grad = dloss * [ (1-l)/n sign(I-G) - l/n (w*A + 2 I w*B + G w*C) ]  (same row / column passes)
__global__ __launch_bounds__(256) void k_ssim_bwd(int H, int W, const float *__restrict__ I, const float *__restrict__ G,
                                                  const float *__restrict__ maps, Win win, float wl1, float wss,
                                                  const float *__restrict__ dloss, float *__restrict__ grad) {
    __shared__ float sm[3][S][SP];
    __shared__ float hq[3][S][HP];
    const int c = blockIdx.z;
    const int x0 = blockIdx.x * T, y0 = blockIdx.y * T;
    const int tid = threadIdx.x;
    const size_t plane = (size_t)H * W;
    const float *src[3] = {maps + (3 * c) * plane, maps + (3 * c + 1) * plane, maps + (3 * c + 2) * plane};
    load_tile<3>(sm, src, H, W, x0, y0);
    __syncthreads();
    if (tid < S * (T / HX)) {
        const int ly = tid / (T / HX), lx0 = (tid % (T / HX)) * HX;
#pragma unroll
        for (int m = 0; m < 3; m++) {
            float v[HX + 10];
#pragma unroll
            for (int k = 0; k < HX + 10; k++) v[k] = sm[m][ly][lx0 + k];
#pragma unroll
            for (int j = 0; j < HX; j++) {
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < 11; k++) acc += win.w[k] * v[j + k];
                hq[m][ly][lx0 + j] = acc;
            }
        }
    }
    __syncthreads();
    const int lx = tid % T, ly0 = (tid / T) * VY;
    const int x = x0 + lx;
    float f[3][VY];
#pragma unroll
    for (int m = 0; m < 3; m++) {
        float v[VY + 10];
#pragma unroll
        for (int k = 0; k < VY + 10; k++) v[k] = hq[m][ly0 + k][lx];
#pragma unroll
        for (int j = 0; j < VY; j++) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < 11; k++) acc += win.w[k] * v[j + k];
            f[m][j] = acc;
        }
    }
    const float dl = dloss ? dloss[0] : 1.f;
#pragma unroll
    for (int j = 0; j < VY; j++) {
        const int y = y0 + ly0 + j;
        if (x >= W || y >= H) continue;
        const size_t p = c * plane + (size_t)y * W + x;
        const float i = I[p], g = G[p];
        const float d = i - g;
        const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        grad[p] = dl * (wl1 * sg - wss * (f[0][j] + 2.f * i * f[1][j] + g * f[2][j]));
    }
}

Win make_window() {
    // utils/loss_utils.py:30-39 builds the 11-tap Gaussian (sigma 1.5) in fp32 and filters with the
    // fp32-ROUNDED outer product as a 2-D window; this kernel filters separably, i.e. with the exact
    // outer product of its 1-D weights, whose total differs from the reference window's: the fp32
    // 1-D weights sum to 1 + 4e-8, the reference's 121 rounded products to 1 - 6.9e-8. Against a target
    // close to the render the SSIM variances cancel against C2 and that normalisation reached the loss at
    // 4.2e-5 relative (the bench step vs the float64 reference, r5h; reproduced by a numpy emulation).
    // The weights below are the reference's 1-D weights (torch fp32: gaussian(11, 1.5)) with taps 0/10
    // +1 ulp and 1/9 -4 ulps, chosen so that (sum w)^2 equals the reference window's sum to 6e-11: the
    // emulated fp32 loss then sits 7e-8 from the float64 reference (the reference's own fp32: 6e-8).
    // tests/test_host_mirrors.py re-derives both sums from the reference formula.
    static const uint32_t bits[11] = {0x3a86cab7u, 0x3bf8fefdu, 0x3d13758cu, 0x3ddff87fu, 0x3e5a1e1fu, 0x3e8832b0u,
                                      0x3e5a1e1fu, 0x3ddff87fu, 0x3d13758cu, 0x3bf8fefdu, 0x3a86cab7u};
    Win w;
    for (int k = 0; k < 11; k++) {
        uint32_t u = bits[k];
        std::memcpy(&w.w[k], &u, 4);
    }
    return w;
}

}  // namespace ssim
}  // namespace dgs

using namespace dgs;

extern "C" size_t dgs_l1_ssim_scratch_floats(int C, int H, int W) {
    size_t nb = (size_t)C * div_up(H, ssim::T) * div_up(W, ssim::T);
    return 3ull * C * H * W + 2 * nb;
}

extern "C" int dgs_l1_ssim_forward(int C, int H, int W, const float *img, const float *gt, float lambda, float *out3,
                                   float *scratch, void *stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    if (C <= 0 || H <= 0 || W <= 0 || !img || !gt || !out3 || !scratch) {
        set_error("dgs_l1_ssim_forward: bad argument");
        return DGS_ERR_ARGS;
    }
    dim3 grid(div_up(W, ssim::T), div_up(H, ssim::T), C);
    const int nb = grid.x * grid.y * grid.z;
    float *maps = scratch;
    float *partial = scratch + 3ull * C * H * W;
    {
        ScopedTimer tm("ssim_fwd", stream);
        hipLaunchKernelGGL(ssim::k_ssim_fwd, grid, dim3(256), 0, stream, H, W, img, gt, ssim::make_window(), maps, partial);
        hipLaunchKernelGGL(ssim::k_ssim_final, dim3(1), dim3(1024), 0, stream, nb, (float)C * H * W, lambda, partial, out3);
    }
    DGS_LAUNCH_CHECK("k_ssim_fwd", false, stream);
    return DGS_OK;
}

extern "C" int dgs_l1_ssim_backward(int C, int H, int W, const float *img, const float *gt, float lambda,
                                    const float *scratch, const float *dloss, float *grad, void *stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    if (C <= 0 || H <= 0 || W <= 0 || !img || !gt || !scratch || !grad) {
        set_error("dgs_l1_ssim_backward: bad argument");
        return DGS_ERR_ARGS;
    }
    dim3 grid(div_up(W, ssim::T), div_up(H, ssim::T), C);
    const float n = (float)C * H * W;
    {
        ScopedTimer tm("ssim_bwd", stream);
        hipLaunchKernelGGL(ssim::k_ssim_bwd, grid, dim3(256), 0, stream, H, W, img, gt, scratch, ssim::make_window(),
                           (1.f - lambda) / n, lambda / n, dloss, grad);
    }
    DGS_LAUNCH_CHECK("k_ssim_bwd", false, stream);
    return DGS_OK;
}

// the fused loss's 11 separable window taps (host-side constant, no GPU needed; tests)
extern "C" void dgs_l1_ssim_window(float *out11) {
    const ssim::Win w = ssim::make_window();
    for (int k = 0; k < 11; k++) out11[k] = w.w[k];
}
