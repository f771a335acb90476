// ssim.hip -- fused SSIM map forward/backward for gfx950: the drop-in for the reference's
// optional `fused_ssim` (submodule fused-ssim, un-vendored; call site train.py:31-35,121-124)
// and for the `fusedssim` / `fusedssim_backward` ops utils/loss_utils.py:17-38 imports from
// diff_gaussian_rasterization._C.  Semantics are those of the reference's own PyTorch SSIM
// (utils/loss_utils.py:56-86): an 11x11 Gaussian window (sigma 1.5, normalised in float32),
// zero padding ("same"), per channel, C1 = 0.01^2, C2 = 0.03^2:
//   mu = w * x, sigma_xx = w * x^2 - mu_x^2, sigma_xy = w * (x y) - mu_x mu_y,
//   map = (2 mu_x mu_y + C1)(2 sigma_xy + C2) / ((mu_x^2 + mu_y^2 + C1)(sigma_xx + sigma_yy + C2)).
//
// One 256-thread workgroup per 32x32 output tile of one (batch, channel) plane: the 42x42
// halo of both images is staged in LDS, the window is applied separably (horizontal pass for
// the five moments over the 42 halo rows, then vertical), so each pixel costs 2 x 5 x 11 FMAs
// and the kernel streams HBM once (2 images in; map + 3 partial-derivative planes out).
// The backward applies the window to the three partial planes times dL/dmap and finishes
//   dL/dx(p) = (w * (g A))(p) + 2 x(p) (w * (g B))(p) + y(p) (w * (g C))(p)
// with A = dmap/dmu_x (through mu_x in sigma_xx and sigma_xy included), B = dmap/dsigma_xx,
// C = dmap/dsigma_xy.  No atomics: results are bitwise reproducible.
#include "gsr_common.h"
#include "gsr_kernels.h"

#include <cmath>

namespace gsr {

constexpr int SS_T = 32;              // output tile edge
constexpr int SS_R = 5;               // window radius (11 taps)
constexpr int SS_H = SS_T + 2 * SS_R;  // halo edge, 42

struct SsimWeights {
    float w[11];
};

// Stage a 42x42 halo of `plane` (zero outside the image) into s[42][43].
__device__ __forceinline__ void ss_stage(const float* plane, int H, int W, int y0, int x0, float (*s)[SS_H + 1])
{
    for (int i = threadIdx.x; i < SS_H * SS_H; i += 256) {
        const int r = i / SS_H, c = i - r * SS_H;
        const int y = y0 - SS_R + r, x = x0 - SS_R + c;
        s[r][c] = (y >= 0 && y < H && x >= 0 && x < W) ? plane[(size_t)y * W + x] : 0.f;
    }
}

template <bool TRAIN>
__global__ void __launch_bounds__(256) ssim_fwd_kernel(int H, int W, float C1, float C2, SsimWeights wt,
                                                       const float* img1, const float* img2, float* map, float* dA,
                                                       float* dB, float* dC)
{
    __shared__ float s1[SS_H][SS_H + 1], s2[SS_H][SS_H + 1];
    __shared__ float hs[5][SS_H][SS_T + 1];  // horizontal pass: x, y, xx, yy, xy
    const size_t plane = (size_t)blockIdx.z * H * W;
    const int x0 = blockIdx.x * SS_T, y0 = blockIdx.y * SS_T;
    ss_stage(img1 + plane, H, W, y0, x0, s1);
    ss_stage(img2 + plane, H, W, y0, x0, s2);
    __syncthreads();
    for (int i = threadIdx.x; i < SS_H * SS_T; i += 256) {
        const int r = i / SS_T, c = i - r * SS_T;
        float mx = 0.f, my = 0.f, mxx = 0.f, myy = 0.f, mxy = 0.f;
#pragma unroll
        for (int t = 0; t < 11; t++) {
            const float a = s1[r][c + t], b = s2[r][c + t], w = wt.w[t];
            mx = __builtin_fmaf(w, a, mx);
            my = __builtin_fmaf(w, b, my);
            mxx = __builtin_fmaf(w, a * a, mxx);
            myy = __builtin_fmaf(w, b * b, myy);
            mxy = __builtin_fmaf(w, a * b, mxy);
        }
        hs[0][r][c] = mx; hs[1][r][c] = my; hs[2][r][c] = mxx; hs[3][r][c] = myy; hs[4][r][c] = mxy;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < SS_T * SS_T; i += 256) {
        const int r = i / SS_T, c = i - r * SS_T;
        const int y = y0 + r, x = x0 + c;
        if (y >= H || x >= W) continue;
        float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 11; t++) {
#pragma unroll
            for (int k = 0; k < 5; k++) m[k] = __builtin_fmaf(wt.w[t], hs[k][r + t][c], m[k]);
        }
        const float mu1 = m[0], mu2 = m[1];
        const float s11 = m[2] - mu1 * mu1, s22 = m[3] - mu2 * mu2, s12 = m[4] - mu1 * mu2;
        const float A = 2.f * mu1 * mu2 + C1, B = 2.f * s12 + C2;
        const float Cc = mu1 * mu1 + mu2 * mu2 + C1, D = s11 + s22 + C2;
        const float val = (A * B) / (Cc * D);
        const size_t o = plane + (size_t)y * W + x;
        map[o] = val;
        if constexpr (TRAIN) {
            const float f_mu1 = (2.f * mu2 * B) / (Cc * D) - (2.f * mu1 * val) / Cc;
            const float f_s11 = -val / D;
            const float f_s12 = (2.f * A) / (Cc * D);
            dA[o] = f_mu1 - 2.f * mu1 * f_s11 - mu2 * f_s12;
            dB[o] = f_s11;
            dC[o] = f_s12;
        }
    }
}

// dL/dimg1 from dL/dmap and the forward's partial-derivative planes.
__global__ void __launch_bounds__(256) ssim_bwd_kernel(int H, int W, SsimWeights wt, const float* img1,
                                                       const float* img2, const float* dmap, const float* dA,
                                                       const float* dB, const float* dC, float* dimg1)
{
    __shared__ float g[3][SS_H][SS_H + 1];   // g*A, g*B, g*C over the halo (zero outside)
    __shared__ float hs[3][SS_H][SS_T + 1];
    const size_t plane = (size_t)blockIdx.z * H * W;
    const int x0 = blockIdx.x * SS_T, y0 = blockIdx.y * SS_T;
    for (int i = threadIdx.x; i < SS_H * SS_H; i += 256) {
        const int r = i / SS_H, c = i - r * SS_H;
        const int y = y0 - SS_R + r, x = x0 - SS_R + c;
        float a = 0.f, b = 0.f, cc = 0.f;
        if (y >= 0 && y < H && x >= 0 && x < W) {
            const size_t o = plane + (size_t)y * W + x;
            const float gm = dmap[o];
            a = gm * dA[o];
            b = gm * dB[o];
            cc = gm * dC[o];
        }
        g[0][r][c] = a; g[1][r][c] = b; g[2][r][c] = cc;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < SS_H * SS_T; i += 256) {
        const int r = i / SS_T, c = i - r * SS_T;
        float s[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 11; t++) {
#pragma unroll
            for (int k = 0; k < 3; k++) s[k] = __builtin_fmaf(wt.w[t], g[k][r][c + t], s[k]);
        }
        hs[0][r][c] = s[0]; hs[1][r][c] = s[1]; hs[2][r][c] = s[2];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < SS_T * SS_T; i += 256) {
        const int r = i / SS_T, c = i - r * SS_T;
        const int y = y0 + r, x = x0 + c;
        if (y >= H || x >= W) continue;
        float s[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 11; t++) {
#pragma unroll
            for (int k = 0; k < 3; k++) s[k] = __builtin_fmaf(wt.w[t], hs[k][r + t][c], s[k]);
        }
        const size_t o = plane + (size_t)y * W + x;
        dimg1[o] = s[0] + 2.f * img1[o] * s[1] + img2[o] * s[2];
    }
}

// The reference's window (utils/loss_utils.py:46-53): exp in double, stored as float32,
// normalised in float32 (gauss / gauss.sum()).
static SsimWeights ssim_weights()
{
    SsimWeights w;
    float g[11], sum = 0.f;
    for (int x = 0; x < 11; x++) {
        g[x] = (float)std::exp(-((double)(x - 5) * (double)(x - 5)) / (2.0 * 1.5 * 1.5));
    }
    for (int x = 0; x < 11; x++) sum += g[x];  // torch's float32 sum of 11 terms
    for (int x = 0; x < 11; x++) w.w[x] = g[x] / sum;
    return w;
}

hipError_t launch_ssim_fwd(int planes, int H, int W, float C1, float C2, const float* img1, const float* img2,
                           float* map, float* dA, float* dB, float* dC, hipStream_t s)
{
    if (planes <= 0 || H <= 0 || W <= 0) return hipSuccess;
    const dim3 grid((W + SS_T - 1) / SS_T, (H + SS_T - 1) / SS_T, planes);
    const SsimWeights w = ssim_weights();
    if (dA && dB && dC)
        hipLaunchKernelGGL(ssim_fwd_kernel<true>, grid, dim3(256), 0, s, H, W, C1, C2, w, img1, img2, map, dA, dB,
                           dC);
    else
        hipLaunchKernelGGL(ssim_fwd_kernel<false>, grid, dim3(256), 0, s, H, W, C1, C2, w, img1, img2, map, dA, dB,
                           dC);
    return hipGetLastError();
}

hipError_t launch_ssim_bwd(int planes, int H, int W, const float* img1, const float* img2, const float* dmap,
                           const float* dA, const float* dB, const float* dC, float* dimg1, hipStream_t s)
{
    if (planes <= 0 || H <= 0 || W <= 0) return hipSuccess;
    const dim3 grid((W + SS_T - 1) / SS_T, (H + SS_T - 1) / SS_T, planes);
    hipLaunchKernelGGL(ssim_bwd_kernel, grid, dim3(256), 0, s, H, W, ssim_weights(), img1, img2, dmap, dA, dB, dC,
                       dimg1);
    return hipGetLastError();
}

}  // namespace gsr
