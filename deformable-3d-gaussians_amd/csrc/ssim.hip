// Fused photometric loss for MI355X: L = (1-l) * mean|I-G| + l * (1 - mean SSIM(I,G)) and dL/dI.
// Replaces utils/loss_utils.py:18-73 (l1_loss + ssim: 11x11 Gaussian window sigma 1.5, zero-padded
// 'same' depthwise conv2d, C1 = 0.01^2, C2 = 0.03^2) inside the training step
// (train_baseline.py:126-128), which PyTorch runs as 5+3 MIOpen convolutions per direction.
//
// The 2-D window is the outer product of the 1-D one, so every filtered map is a separable
// 11-tap row pass + 11-tap column pass through LDS (16x16 output tile, 26x26 halo tile).
// Forward: 5 maps (mu1, mu2, E[I^2], E[G^2], E[IG]) -> per pixel SSIM and the three coefficient
// maps A, B, C of dSSIM/d(mu1, E[I^2], E[IG]) -> HBM; per-block partial sums (deterministic).
// Backward: dSSIM_sum/dI = w*A + 2 I (w*B) + G (w*C) (window symmetric), plus the L1 sign term.
#include <hip/hip_runtime.h>

#include "dgs_common.h"

namespace dgs {
namespace ssim {

constexpr int T = 16;            // output tile
constexpr int R = 5;             // window radius
constexpr int S = T + 2 * R;     // 26: input tile with halo
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

// block (tile) partial sums: [blocks][2] = (sum |I-G|, sum ssim)
__global__ __launch_bounds__(256) void k_ssim_fwd(int H, int W, const float *__restrict__ I, const float *__restrict__ G,
                                                  Win win, float *__restrict__ maps, float *__restrict__ partial) {
    __shared__ float sI[S][S + 1], sG[S][S + 1];
    __shared__ float hq[5][S][T + 1];
    __shared__ float red[2][4];
    const int c = blockIdx.z;
    const int x0 = blockIdx.x * T, y0 = blockIdx.y * T;
    const int tid = threadIdx.x;
    const size_t plane = (size_t)H * W;
    const float *Ic = I + c * plane, *Gc = G + c * plane;
    for (int e = tid; e < S * S; e += 256) {
        int ly = e / S, lx = e % S;
        int gy = y0 + ly - R, gx = x0 + lx - R;
        bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        sI[ly][lx] = in ? Ic[(size_t)gy * W + gx] : 0.f;
        sG[ly][lx] = in ? Gc[(size_t)gy * W + gx] : 0.f;
    }
    __syncthreads();
    for (int e = tid; e < S * T; e += 256) {
        int ly = e / T, lx = e % T;
        float a = 0.f, b = 0.f, aa = 0.f, bb = 0.f, ab = 0.f;
#pragma unroll
        for (int k = 0; k < 11; k++) {
            float i = sI[ly][lx + k], g = sG[ly][lx + k], w = win.w[k];
            a += w * i;
            b += w * g;
            aa += w * (i * i);
            bb += w * (g * g);
            ab += w * (i * g);
        }
        hq[0][ly][lx] = a; hq[1][ly][lx] = b; hq[2][ly][lx] = aa; hq[3][ly][lx] = bb; hq[4][ly][lx] = ab;
    }
    __syncthreads();
    const int lx = tid % T, ly = tid / T;
    const int x = x0 + lx, y = y0 + ly;
    float mu1 = 0.f, mu2 = 0.f, m11 = 0.f, m22 = 0.f, m12 = 0.f;
#pragma unroll
    for (int k = 0; k < 11; k++) {
        float w = win.w[k];
        mu1 += w * hq[0][ly + k][lx];
        mu2 += w * hq[1][ly + k][lx];
        m11 += w * hq[2][ly + k][lx];
        m22 += w * hq[3][ly + k][lx];
        m12 += w * hq[4][ly + k][lx];
    }
    float l1 = 0.f, s = 0.f;
    if (x < W && y < H) {
        float mu1s = mu1 * mu1, mu2s = mu2 * mu2, mu12 = mu1 * mu2;
        float s11 = m11 - mu1s, s22 = m22 - mu2s, s12 = m12 - mu12;
        float n1 = 2.f * mu12 + C1, n2 = 2.f * s12 + C2;
        float d1 = mu1s + mu2s + C1, d2 = s11 + s22 + C2;
        float inv = 1.f / (d1 * d2);
        s = n1 * n2 * inv;
        float A = 2.f * mu2 * n2 * inv - 2.f * mu1 * s / d1 + 2.f * mu1 * s / d2 - mu2 * 2.f * n1 * inv;
        float B = -s / d2;
        float Cc = 2.f * n1 * inv;
        size_t p = (size_t)y * W + x;
        maps[(3 * c + 0) * plane + p] = A;
        maps[(3 * c + 1) * plane + p] = B;
        maps[(3 * c + 2) * plane + p] = Cc;
        l1 = fabsf(sI[ly + R][lx + R] - sG[ly + R][lx + R]);
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

// grad = dloss * [ (1-l)/n sign(I-G) - l/n (w*A + 2 I w*B + G w*C) ]
__global__ __launch_bounds__(256) void k_ssim_bwd(int H, int W, const float *__restrict__ I, const float *__restrict__ G,
                                                  const float *__restrict__ maps, Win win, float wl1, float wss,
                                                  const float *__restrict__ dloss, float *__restrict__ grad) {
    __shared__ float sm[3][S][S + 1];
    __shared__ float hq[3][S][T + 1];
    const int c = blockIdx.z;
    const int x0 = blockIdx.x * T, y0 = blockIdx.y * T;
    const int tid = threadIdx.x;
    const size_t plane = (size_t)H * W;
    for (int e = tid; e < S * S; e += 256) {
        int ly = e / S, lx = e % S;
        int gy = y0 + ly - R, gx = x0 + lx - R;
        bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        size_t p = (size_t)gy * W + gx;
#pragma unroll
        for (int q = 0; q < 3; q++) sm[q][ly][lx] = in ? maps[(3 * c + q) * plane + p] : 0.f;
    }
    __syncthreads();
    for (int e = tid; e < S * T; e += 256) {
        int ly = e / T, lx = e % T;
        float a = 0.f, b = 0.f, cc = 0.f;
#pragma unroll
        for (int k = 0; k < 11; k++) {
            float w = win.w[k];
            a += w * sm[0][ly][lx + k];
            b += w * sm[1][ly][lx + k];
            cc += w * sm[2][ly][lx + k];
        }
        hq[0][ly][lx] = a; hq[1][ly][lx] = b; hq[2][ly][lx] = cc;
    }
    __syncthreads();
    const int lx = tid % T, ly = tid / T;
    const int x = x0 + lx, y = y0 + ly;
    if (x >= W || y >= H) return;
    float fa = 0.f, fb = 0.f, fc = 0.f;
#pragma unroll
    for (int k = 0; k < 11; k++) {
        float w = win.w[k];
        fa += w * hq[0][ly + k][lx];
        fb += w * hq[1][ly + k][lx];
        fc += w * hq[2][ly + k][lx];
    }
    size_t p = c * plane + (size_t)y * W + x;
    float i = I[p], g = G[p];
    float d = i - g;
    float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    float dl = dloss ? dloss[0] : 1.f;
    grad[p] = dl * (wl1 * sg - wss * (fa + 2.f * i * fb + g * fc));
}

Win make_window() {
    // utils/loss_utils.py:30-39: gauss = exp(-(x-5)^2 / (2*1.5^2)), normalised in fp32
    Win w;
    float s = 0.f;
    for (int k = 0; k < 11; k++) {
        float v = (float)std::exp(-(double)((k - 5) * (k - 5)) / (2.0 * 1.5 * 1.5));
        w.w[k] = v;
        s += v;
    }
    for (int k = 0; k < 11; k++) w.w[k] /= s;
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
