// render.hip -- per-tile alpha blending, forward (FORWARD::render / renderCUDA,
// forward.cu:277-430) and backward (BACKWARD::render / renderCUDA,
// backward.cu:452-638, launch :714-753), for gfx950.
//
// CDNA4 mapping: one 256-thread workgroup (4 wave64s) per 16x16 tile; wave w
// owns pixel rows 4w..4w+3.  The tile's Gaussian list is streamed through LDS
// in batches of 256 records (id, xy, conic+opacity, rgb, 1/depth): every lane of
// a wave then reads the same LDS address (broadcast, conflict-free).  A wave
// whose 64 pixels are all saturated stops evaluating (ballot), and the block
// stops fetching once all four waves are done (the reference's
// __syncthreads_count early-out, forward.cu:329-331).
//
// Backward: the traversal is back-to-front from each pixel's n_contrib; batches
// behind the tile's largest n_contrib are skipped without loading.  The ten
// per-(pixel, Gaussian) gradient terms are summed across the wave with a
// butterfly before a single lane issues the global float atomics (the
// reference issues up to ten atomics per contributing pixel).
#include "gsr_common.h"
#include "gsr_kernels.h"

namespace gsr {

constexpr int BATCH = 256;

__global__ void __launch_bounds__(256) render_fwd_kernel(RenderFwdArgs a)
{
    const uint32_t tile = blockIdx.x;
    const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int tid = threadIdx.x;
    const uint32_t px = tx * GSR_BLOCK_X + (tid & 15), py = ty * GSR_BLOCK_Y + (tid >> 4);
    const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint2 range = a.ranges[tile];
    const int todo = (int)(range.y - range.x);

    __shared__ float4 s_co[BATCH];   // conic.x conic.y conic.z opacity
    __shared__ float4 s_xyr[BATCH];  // x y r g
    __shared__ float2 s_bd[BATCH];   // b invdepth

    bool done = !inside;
    float T = 1.0f;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f, ID = 0.f;
    uint32_t last_contributor = 0;

    for (int base = 0; base < todo; base += BATCH) {
        if (__syncthreads_and(done)) break;
        const int k = base + tid;
        if (k < todo) {
            const uint32_t id = a.point_list[range.x + k];
            const float2 xy = a.means2D[id];
            s_co[tid] = a.conic_opacity[id];
            const float* f = a.features + 3 * (size_t)id;
            s_xyr[tid] = make_float4(xy.x, xy.y, f[0], f[1]);
            s_bd[tid] = make_float2(f[2], 1.0f / a.depths[id]);
        }
        __syncthreads();
        const int n = min(BATCH, todo - base);
        for (int j = 0; j < n; j++) {
            if (__all(done)) break;
            const float4 co = s_co[j];
            const float4 xyr = s_xyr[j];
            const float dx = xyr.x - pfx, dy = xyr.y - pfy;
            const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
            const float alpha = fminf(0.99f, co.w * __expf(power));
            bool contrib = !done && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
            const float test_T = T * (1 - alpha);
            if (contrib && test_T < 0.0001f) {
                done = true;
                contrib = false;
            }
            if (contrib) {
                const float2 bd = s_bd[j];
                C0 += xyr.z * alpha * T;
                C1 += xyr.w * alpha * T;
                C2 += bd.x * alpha * T;
                ID += bd.y * alpha * T;
                T = test_T;
                last_contributor = (uint32_t)(base + j + 1);
            }
        }
    }

    if (inside) {
        const uint32_t pix_id = (uint32_t)a.W * py + px;
        const size_t HW = (size_t)a.H * a.W;
        a.final_T[pix_id] = T;
        a.n_contrib[pix_id] = last_contributor;
        a.out_color[0 * HW + pix_id] = C0 + T * a.bg[0];
        a.out_color[1 * HW + pix_id] = C1 + T * a.bg[1];
        a.out_color[2 * HW + pix_id] = C2 + T * a.bg[2];
        if (a.invdepth) a.invdepth[pix_id] = ID;
    }
}

__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d, 64));
    return v;
}

__global__ void __launch_bounds__(256) render_bwd_kernel(RenderBwdArgs a)
{
    const uint32_t tile = blockIdx.x;
    const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const uint32_t px = tx * GSR_BLOCK_X + (tid & 15), py = ty * GSR_BLOCK_Y + (tid >> 4);
    const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint2 range = a.ranges[tile];
    const int todo = (int)(range.y - range.x);
    const uint32_t pix_id = (uint32_t)a.W * py + px;
    const size_t HW = (size_t)a.H * a.W;

    __shared__ float4 s_co[BATCH];
    __shared__ float2 s_xy[BATCH];
    __shared__ float4 s_col[BATCH];  // r g b invdepth
    __shared__ uint32_t s_id[BATCH];
    __shared__ uint32_t s_wmax[4];

    const float T_final = inside ? a.final_Ts[pix_id] : 0.f;
    float T = T_final;
    const uint32_t last_contributor = inside ? a.n_contrib[pix_id] : 0;
    float dpix0 = 0.f, dpix1 = 0.f, dpix2 = 0.f, dinv = 0.f;
    if (inside) {
        dpix0 = a.dL_dpixels[0 * HW + pix_id];
        dpix1 = a.dL_dpixels[1 * HW + pix_id];
        dpix2 = a.dL_dpixels[2 * HW + pix_id];
        if (a.dL_invdepths) dinv = a.dL_invdepths[pix_id];
    }
    const bool has_inv = a.dL_dinvdepths != nullptr;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc_inv = 0.f;
    float last_alpha = 0.f, last_c0 = 0.f, last_c1 = 0.f, last_c2 = 0.f, last_inv = 0.f;
    const float ddelx_dx = 0.5 * a.W;
    const float ddely_dy = 0.5 * a.H;
    const float bg_dot_dpixel = a.bg[0] * dpix0 + a.bg[1] * dpix1 + a.bg[2] * dpix2;

    // Largest n_contrib in this wave / tile: list entries at or behind it contribute nothing.
    const uint32_t wmax = wave_max_u32(last_contributor);
    if (lane == 0) s_wmax[wid] = wmax;
    __syncthreads();
    const uint32_t tmax = max(max(s_wmax[0], s_wmax[1]), max(s_wmax[2], s_wmax[3]));
    // entries with list position >= tmax are skipped: start traversal at position tmax-1
    const int skip = todo - (int)tmax;  // number of trailing entries to skip

    for (int base = skip; base < todo; base += BATCH) {
        __syncthreads();
        const int k = base + tid;
        if (k < todo) {
            const uint32_t id = a.point_list[range.y - k - 1];
            s_id[tid] = id;
            s_xy[tid] = a.means2D[id];
            s_co[tid] = a.conic_opacity[id];
            const float* c = a.colors + 3 * (size_t)id;
            s_col[tid] = make_float4(c[0], c[1], c[2], has_inv ? 1.f / a.depths[id] : 0.f);
        }
        __syncthreads();
        const int n = min(BATCH, todo - base);
        for (int j = 0; j < n; j++) {
            const uint32_t pos = (uint32_t)(todo - 1 - (base + j));
            if (pos >= wmax) continue;  // wave-uniform
            const float4 co = s_co[j];
            const float2 xy = s_xy[j];
            const float dx = xy.x - pfx, dy = xy.y - pfy;
            const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
            const float G = __expf(power);
            const float alpha = fminf(0.99f, co.w * G);
            const bool contrib = inside && pos < last_contributor && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
            float g_c0 = 0.f, g_c1 = 0.f, g_c2 = 0.f, g_inv = 0.f, g_mx = 0.f, g_my = 0.f, g_ca = 0.f,
                  g_cb = 0.f, g_cc = 0.f, g_op = 0.f;
            if (contrib) {
                const float4 col = s_col[j];
                T = T / (1.f - alpha);
                const float dchannel_dcolor = alpha * T;
                float dL_dalpha = 0.0f;
                acc0 = last_alpha * last_c0 + (1.f - last_alpha) * acc0;
                acc1 = last_alpha * last_c1 + (1.f - last_alpha) * acc1;
                acc2 = last_alpha * last_c2 + (1.f - last_alpha) * acc2;
                last_c0 = col.x; last_c1 = col.y; last_c2 = col.z;
                dL_dalpha += (col.x - acc0) * dpix0;
                dL_dalpha += (col.y - acc1) * dpix1;
                dL_dalpha += (col.z - acc2) * dpix2;
                g_c0 = dchannel_dcolor * dpix0;
                g_c1 = dchannel_dcolor * dpix1;
                g_c2 = dchannel_dcolor * dpix2;
                if (has_inv) {
                    const float invd = col.w;
                    acc_inv = last_alpha * last_inv + (1.f - last_alpha) * acc_inv;
                    last_inv = invd;
                    dL_dalpha += (invd - acc_inv) * dinv;
                    g_inv = dchannel_dcolor * dinv;
                }
                dL_dalpha *= T;
                last_alpha = alpha;
                dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot_dpixel;
                const float dL_dG = co.w * dL_dalpha;
                const float gdx = G * dx;
                const float gdy = G * dy;
                const float dG_ddelx = -gdx * co.x - gdy * co.y;
                const float dG_ddely = -gdy * co.z - gdx * co.y;
                g_mx = dL_dG * dG_ddelx * ddelx_dx;
                g_my = dL_dG * dG_ddely * ddely_dy;
                g_ca = -0.5f * gdx * dx * dL_dG;
                g_cb = -0.5f * gdx * dy * dL_dG;
                g_cc = -0.5f * gdy * dy * dL_dG;
                g_op = G * dL_dalpha;
            }
            if (__any(contrib)) {
                g_c0 = wave_sum(g_c0);
                g_c1 = wave_sum(g_c1);
                g_c2 = wave_sum(g_c2);
                g_mx = wave_sum(g_mx);
                g_my = wave_sum(g_my);
                g_ca = wave_sum(g_ca);
                g_cb = wave_sum(g_cb);
                g_cc = wave_sum(g_cc);
                g_op = wave_sum(g_op);
                if (has_inv) g_inv = wave_sum(g_inv);
                if (lane == 0) {
                    const uint32_t gid = s_id[j];
                    atomicAdd(&a.dL_dcolors[3 * (size_t)gid + 0], g_c0);
                    atomicAdd(&a.dL_dcolors[3 * (size_t)gid + 1], g_c1);
                    atomicAdd(&a.dL_dcolors[3 * (size_t)gid + 2], g_c2);
                    atomicAdd(&a.dL_dmean2D[3 * (size_t)gid + 0], g_mx);
                    atomicAdd(&a.dL_dmean2D[3 * (size_t)gid + 1], g_my);
                    atomicAdd(&a.dL_dconic2D[4 * (size_t)gid + 0], g_ca);
                    atomicAdd(&a.dL_dconic2D[4 * (size_t)gid + 1], g_cb);
                    atomicAdd(&a.dL_dconic2D[4 * (size_t)gid + 3], g_cc);
                    atomicAdd(&a.dL_dopacity[gid], g_op);
                    if (has_inv) atomicAdd(&a.dL_dinvdepths[gid], g_inv);
                }
            }
        }
    }
}

hipError_t launch_render_fwd(const RenderFwdArgs& a, int T, hipStream_t s)
{
    if (T <= 0) return hipSuccess;
    hipLaunchKernelGGL(render_fwd_kernel, dim3(T), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_render_bwd(const RenderBwdArgs& a, int T, hipStream_t s)
{
    if (T <= 0) return hipSuccess;
    hipLaunchKernelGGL(render_bwd_kernel, dim3(T), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace gsr
