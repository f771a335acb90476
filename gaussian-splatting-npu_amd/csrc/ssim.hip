// ssim.hip -- fused SSIM map forward/backward for gfx950: the drop-in for the reference's
// optional `fused_ssim` (submodule fused-ssim, un-vendored; call site train.py:31-35,121-124)
// and for the `fusedssim` / `fusedssim_backward` ops utils/loss_utils.py:17-38 imports from
// diff_gaussian_rasterization._C.  Semantics are those of the reference's own PyTorch SSIM
// (utils/loss_utils.py:56-86): an 11x11 Gaussian window (sigma 1.5, normalised in float32),
// zero padding ("same"), per channel, C1 = 0.01^2, C2 = 0.03^2:
//   mu = w * x, sigma_xx = w * x^2 - mu_x^2, sigma_xy = w * (x y) - mu_x mu_y,
//   map = (2 mu_x mu_y + C1)(2 sigma_xy + C2) / ((mu_x^2 + mu_y^2 + C1)(sigma_xx + sigma_yy + C2)).
//
// Output tiles of 64x32 pixels of one (batch, channel) plane.  A persistent grid (2 workgroups
// of 256 threads per CU) walks the tiles; each tile's 74x42 halo of both images goes through
// LDS, and the NEXT tile's halo loads are issued into registers before the current tile is
// computed, so HBM latency hides behind the arithmetic.  The window is applied separably
// (horizontal pass for the five moments over the 42 halo rows, then a vertical pass with a
// rolling 4-row window in registers), two columns per thread as packed-f32 pairs: each pixel
// costs 2 x 5 x 11 / 2 packed FMAs and the kernel streams HBM once (2 images in; map + 3
// partial-derivative planes out).
// The backward applies the window to the three partial planes times dL/dmap and finishes
//   dL/dx(p) = (w * (g A))(p) + 2 x(p) (w * (g B))(p) + y(p) (w * (g C))(p)
// with A = dmap/dmu_x (through mu_x in sigma_xx and sigma_xy included), B = dmap/dsigma_xx,
// C = dmap/dsigma_xy.  No atomics: results are bitwise reproducible.
#include "gsr_common.h"
#include "gsr_kernels.h"

#include <cmath>

namespace gsr {

// Thread (p = tid & 31, q = tid >> 5) owns the column PAIR (p, p + 32) of a tile, so every tap of
// both passes is one packed v_pk_fma_f32 on (col p, col p + 32) with the tap weight broadcast;
// ds_read2_b32 brings the two columns' inputs into adjacent registers.  Horizontal-pass rows are
// dealt to the 8 thread rows q, q + 8, ...; in the vertical pass thread row q owns output rows
// 4q .. 4q + 3.
constexpr int SS_TW = 64;                 // output tile width
constexpr int SS_TH = 32;                 // output tile height
constexpr int SS_R = 5;                   // window radius (11 taps)
constexpr int SS_HH = SS_TH + 2 * SS_R;   // halo rows, 42
constexpr int SS_HW = SS_TW + 2 * SS_R;   // halo columns, 74
constexpr int SS_LS = 76;                 // LDS row stride of the staged planes (floats)
constexpr int SS_STAGE = SS_HH * SS_LS;            // staged floats per plane
constexpr int SS_STAGE_IT = (SS_STAGE + 255) / 256;  // per thread, 13
constexpr int SS_BLOCKS_PER_CU = 2;       // LDS-limited (79 KB forward, 70 KB backward)

typedef float f2 __attribute__((ext_vector_type(2)));

struct SsimWeights {
    float w[11];
};

struct SsGrid {
    int H, W, tx, ty, ntiles;
};

struct SsTile {
    size_t plane;  // offset of the tile's plane
    int x0, y0;
};

__device__ __forceinline__ SsTile ss_tile(const SsGrid& g, int t)
{
    const int x = t % g.tx, r = t / g.tx, y = r % g.ty, z = r / g.ty;
    return {(size_t)z * g.H * g.W, x * SS_TW, y * SS_TH};
}

__device__ __forceinline__ f2 pk_fma(float w, f2 a, f2 c) { return __builtin_elementwise_fma(f2{w, w}, a, c); }

// This thread's NP-plane share of one tile's halo, held in registers between the load (issued one
// tile ahead) and the LDS store.  Elements outside the image / the 74 columns load from the plane
// origin (a valid address) and are zeroed at the store.
template <int NP>
struct SsHalo {
    float v[NP][SS_STAGE_IT];
    uint32_t outside;  // bit j: element j lies outside

    __device__ __forceinline__ void load(const float* const (&src)[NP], const SsGrid& g, const SsTile& t)
    {
        outside = 0;
#pragma unroll
        for (int j = 0; j < SS_STAGE_IT; j++) {
            const int i = threadIdx.x + j * 256;
            const int r = i / SS_LS, c = i - r * SS_LS;
            const int y = t.y0 - SS_R + r, x = t.x0 - SS_R + c;
            const bool in = i < SS_STAGE && c < SS_HW && y >= 0 && y < g.H && x >= 0 && x < g.W;
            const size_t o = t.plane + (in ? (size_t)y * g.W + x : 0);
            outside |= (in ? 0u : 1u) << j;
#pragma unroll
            for (int k = 0; k < NP; k++) v[k][j] = src[k][o];
        }
    }
    __device__ __forceinline__ float get(int k, int j) const { return (outside >> j) & 1 ? 0.f : v[k][j]; }
};

template <bool TRAIN>
__global__ void __launch_bounds__(256) ssim_fwd_kernel(SsGrid g, float C1, float C2, SsimWeights wt,
                                                       const float* img1, const float* img2, float* map, float* dA,
                                                       float* dB, float* dC)
{
    __shared__ float s1[SS_STAGE], s2[SS_STAGE];
    __shared__ f2 hs[5][SS_HH][32];  // horizontal pass per column pair: x, y, xx, yy, xy
    const int p = threadIdx.x & 31, q = threadIdx.x >> 5;
    const float* const src[2] = {img1, img2};
    int t = blockIdx.x;
    if (t >= g.ntiles) return;  // uniform over the workgroup
    SsHalo<2> halo;
    halo.load(src, g, ss_tile(g, t));
    for (; t < g.ntiles; t += gridDim.x) {
        const SsTile cur = ss_tile(g, t);
        __syncthreads();  // the previous tile is done with s1, s2 and hs
#pragma unroll
        for (int j = 0; j < SS_STAGE_IT; j++) {
            const int i = threadIdx.x + j * 256;
            if (j == SS_STAGE_IT - 1 && i >= SS_STAGE) break;
            s1[i] = halo.get(0, j);
            s2[i] = halo.get(1, j);
        }
        if (t + (int)gridDim.x < g.ntiles) halo.load(src, g, ss_tile(g, t + gridDim.x));
        __syncthreads();
        for (int r = q; r < SS_HH; r += 8) {
            f2 mx = {0.f, 0.f}, my = mx, mxx = mx, myy = mx, mxy = mx;
            const float* r1 = s1 + r * SS_LS + p;
            const float* r2 = s2 + r * SS_LS + p;
#pragma unroll
            for (int k = 0; k < 11; k++) {
                const f2 a = {r1[k], r1[k + 32]}, b = {r2[k], r2[k + 32]};
                const float w = wt.w[k];
                mx = pk_fma(w, a, mx);
                my = pk_fma(w, b, my);
                mxx = pk_fma(w, a * a, mxx);
                myy = pk_fma(w, b * b, myy);
                mxy = pk_fma(w, a * b, mxy);
            }
            hs[0][r][p] = mx; hs[1][r][p] = my; hs[2][r][p] = mxx; hs[3][r][p] = myy; hs[4][r][p] = mxy;
        }
        __syncthreads();
        // vertical pass: each of the 14 halo rows thread row q needs is read once and folded
        // into all four of its outputs
        f2 m4[4][5];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int k = 0; k < 5; k++) m4[i][k] = f2{0.f, 0.f};
#pragma unroll
        for (int rr = 0; rr < 14; rr++) {
            f2 v[5];
#pragma unroll
            for (int k = 0; k < 5; k++) v[k] = hs[k][4 * q + rr][p];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int tap = rr - i;
                if (tap < 0 || tap > 10) continue;
#pragma unroll
                for (int k = 0; k < 5; k++) m4[i][k] = pk_fma(wt.w[tap], v[k], m4[i][k]);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int y = cur.y0 + 4 * q + i;
            if (y >= g.H) break;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int x = cur.x0 + p + 32 * h;
                if (x >= g.W) continue;
                const float mu1 = m4[i][0][h], mu2 = m4[i][1][h];
                const float s11 = m4[i][2][h] - mu1 * mu1, s22 = m4[i][3][h] - mu2 * mu2;
                const float s12 = m4[i][4][h] - mu1 * mu2;
                const float A = 2.f * mu1 * mu2 + C1, B = 2.f * s12 + C2;
                const float Cc = mu1 * mu1 + mu2 * mu2 + C1, D = s11 + s22 + C2;
                const float inv = 1.f / (Cc * D);
                const float val = A * B * inv;
                const size_t o = cur.plane + (size_t)y * g.W + x;
                map[o] = val;
                if constexpr (TRAIN) {
                    // d map / d mu1 = 2 mu2 B / (C D) - 2 mu1 val / C, with 1/C = D inv, 1/D = C inv
                    const float f_mu1 = 2.f * inv * (mu2 * B - mu1 * val * D);
                    const float f_s11 = -val * Cc * inv;
                    const float f_s12 = 2.f * A * inv;
                    dA[o] = f_mu1 - 2.f * mu1 * f_s11 - mu2 * f_s12;
                    dB[o] = f_s11;
                    dC[o] = f_s12;
                }
            }
        }
    }
}

// dL/dimg1 from dL/dmap and the forward's partial-derivative planes.
__global__ void __launch_bounds__(256) ssim_bwd_kernel(SsGrid g, SsimWeights wt, const float* img1,
                                                       const float* img2, const float* dmap, const float* dA,
                                                       const float* dB, const float* dC, float* dimg1)
{
    __shared__ float gs[3][SS_STAGE];  // g*A, g*B, g*C over the halo (zero outside)
    __shared__ f2 hs[3][SS_HH][32];
    const int p = threadIdx.x & 31, q = threadIdx.x >> 5;
    const float* const src[4] = {dmap, dA, dB, dC};
    int t = blockIdx.x;
    if (t >= g.ntiles) return;
    SsHalo<4> halo;
    halo.load(src, g, ss_tile(g, t));
    for (; t < g.ntiles; t += gridDim.x) {
        const SsTile cur = ss_tile(g, t);
        // this thread's output pixels' img1 / img2 values
        float i1[4][2], i2[4][2];
#pragma unroll
        for (int j = 0; j < 4; j++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int y = cur.y0 + 4 * q + j, x = cur.x0 + p + 32 * h;
                const size_t o = cur.plane + ((y < g.H && x < g.W) ? (size_t)y * g.W + x : 0);
                i1[j][h] = img1[o];
                i2[j][h] = img2[o];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < SS_STAGE_IT; j++) {
            const int i = threadIdx.x + j * 256;
            if (j == SS_STAGE_IT - 1 && i >= SS_STAGE) break;
            const float gm = halo.get(0, j);
            gs[0][i] = gm * halo.v[1][j];
            gs[1][i] = gm * halo.v[2][j];
            gs[2][i] = gm * halo.v[3][j];
        }
        if (t + (int)gridDim.x < g.ntiles) halo.load(src, g, ss_tile(g, t + gridDim.x));
        __syncthreads();
        for (int r = q; r < SS_HH; r += 8) {
            f2 s[3] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
            for (int k = 0; k < 11; k++) {
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const float* row = gs[c] + r * SS_LS + p;
                    s[c] = pk_fma(wt.w[k], f2{row[k], row[k + 32]}, s[c]);
                }
            }
            hs[0][r][p] = s[0]; hs[1][r][p] = s[1]; hs[2][r][p] = s[2];
        }
        __syncthreads();
        f2 s4[4][3];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int c = 0; c < 3; c++) s4[i][c] = f2{0.f, 0.f};
#pragma unroll
        for (int rr = 0; rr < 14; rr++) {
            f2 v[3];
#pragma unroll
            for (int c = 0; c < 3; c++) v[c] = hs[c][4 * q + rr][p];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int tap = rr - i;
                if (tap < 0 || tap > 10) continue;
#pragma unroll
                for (int c = 0; c < 3; c++) s4[i][c] = pk_fma(wt.w[tap], v[c], s4[i][c]);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int y = cur.y0 + 4 * q + j;
            if (y >= g.H) break;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int x = cur.x0 + p + 32 * h;
                if (x >= g.W) continue;
                const size_t o = cur.plane + (size_t)y * g.W + x;
                dimg1[o] = s4[j][0][h] + 2.f * i1[j][h] * s4[j][1][h] + i2[j][h] * s4[j][2][h];
            }
        }
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

static hipError_t ssim_grid(int planes, int H, int W, SsGrid* g, int* blocks)
{
    g->H = H;
    g->W = W;
    g->tx = (W + SS_TW - 1) / SS_TW;
    g->ty = (H + SS_TH - 1) / SS_TH;
    const long n = (long)g->tx * g->ty * planes;
    if (n > 0x7FFFFFFF) return hipErrorInvalidValue;
    g->ntiles = (int)n;
    int dev = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    const long b = (long)(cus > 0 ? cus : 1) * SS_BLOCKS_PER_CU;
    *blocks = (int)(b < n ? b : n);
    return hipSuccess;
}

hipError_t launch_ssim_fwd(int planes, int H, int W, float C1, float C2, const float* img1, const float* img2,
                           float* map, float* dA, float* dB, float* dC, hipStream_t s)
{
    if (planes <= 0 || H <= 0 || W <= 0) return hipSuccess;
    SsGrid g;
    int blocks;
    hipError_t e = ssim_grid(planes, H, W, &g, &blocks);
    if (e != hipSuccess) return e;
    const SsimWeights w = ssim_weights();
    if (dA && dB && dC)
        hipLaunchKernelGGL(ssim_fwd_kernel<true>, dim3(blocks), dim3(256), 0, s, g, C1, C2, w, img1, img2, map, dA,
                           dB, dC);
    else
        hipLaunchKernelGGL(ssim_fwd_kernel<false>, dim3(blocks), dim3(256), 0, s, g, C1, C2, w, img1, img2, map,
                           dA, dB, dC);
    return hipGetLastError();
}

hipError_t launch_ssim_bwd(int planes, int H, int W, const float* img1, const float* img2, const float* dmap,
                           const float* dA, const float* dB, const float* dC, float* dimg1, hipStream_t s)
{
    if (planes <= 0 || H <= 0 || W <= 0) return hipSuccess;
    SsGrid g;
    int blocks;
    hipError_t e = ssim_grid(planes, H, W, &g, &blocks);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ssim_bwd_kernel, dim3(blocks), dim3(256), 0, s, g, ssim_weights(), img1, img2, dmap, dA, dB,
                       dC, dimg1);
    return hipGetLastError();
}

}  // namespace gsr
