// render.hip -- per-tile alpha blending, forward (FORWARD::render / renderCUDA,
// forward.cu:277-430) and backward (BACKWARD::render / renderCUDA,
// backward.cu:452-638, launch :714-753), for gfx950.
//
// CDNA4 mapping: one 256-thread workgroup (4 wave64s) per 16x16 tile; wave w owns
// the 8x8 pixel quadrant (w&1, w>>1).  The tile's Gaussian list is streamed through
// LDS in batches of 256 packed 48 B records (xy + cull extent, conic + opacity,
// rgb + 1/depth); every lane of a wave reads the same LDS address (broadcast).
//
// Per-wave culling: each record carries the half-extents of the box outside which
// alpha < 1/255 for every pixel (computed in preprocess with a safety margin).  At
// each batch, every wave compacts (ballot + popcount) the list of records whose box
// meets its 8x8 quadrant and evaluates only those -- a pair skipped this way is one
// the reference evaluates and rejects at `alpha < 1/255` (forward.cu:364,
// backward.cu:570), so outputs are unchanged while ~half the pair work disappears.
// n_contrib keeps the reference's meaning (list position + 1 of the last blended
// entry), so the backward replay is unchanged.
//
// Forward early-out: a wave whose 64 pixels are saturated stops (ballot); the block
// stops fetching once all four are (the reference's __syncthreads_count,
// forward.cu:329-331).
//
// Backward: traversal is back-to-front from each pixel's n_contrib; entries behind a
// wave's largest n_contrib are culled for that wave, batches behind the tile's largest
// are not loaded.  The ten per-(pixel, Gaussian) gradient terms are reduced over the
// tile's 256 pixels on chip (transposed cross-lane reduction, then LDS in a fixed order)
// and stored once per (tile, Gaussian) entry -- no global atomics, bitwise-reproducible
// sums (the reference issues up to ten float atomics per contributing pixel,
// backward.cu:593-635).
#include "gsr_common.h"
#include "gsr_kernels.h"

namespace gsr {

constexpr int BATCH = 256;

// Pixel of thread `tid` in tile (tx, ty): wave w covers the 8x8 quadrant (w & 1, w >> 1).
__device__ __forceinline__ void quad_pixel(uint32_t tx, uint32_t ty, int tid, uint32_t& px, uint32_t& py)
{
    const int w = tid >> 6, lane = tid & 63;
    px = tx * GSR_BLOCK_X + (w & 1) * 8 + (lane & 7);
    py = ty * GSR_BLOCK_Y + (w >> 1) * 8 + (lane >> 3);
}

// Minimum of q(d) = a dx^2 + 2 b dx dy + c dy^2 over the axis-aligned box of offsets
// [dx0, dx1] x [dy0, dy1] (a, c > 0, ac > b^2): 0 if the box holds the origin, else the
// smallest of the four edge minima (each a clamped 1-D parabola).
__device__ __forceinline__ float box_min_quadform(float a, float b, float c, float dx0, float dx1, float dy0,
                                                  float dy1)
{
    if (dx0 <= 0.f && dx1 >= 0.f && dy0 <= 0.f && dy1 >= 0.f) return 0.f;
    const float ia = 1.0f / a, ic = 1.0f / c;
    float m = 3.0e38f;
    {  // vertical edges dx = dx0, dx1
        float dy = fminf(fmaxf(-b * dx0 * ic, dy0), dy1);
        m = fminf(m, a * dx0 * dx0 + 2.f * b * dx0 * dy + c * dy * dy);
        dy = fminf(fmaxf(-b * dx1 * ic, dy0), dy1);
        m = fminf(m, a * dx1 * dx1 + 2.f * b * dx1 * dy + c * dy * dy);
    }
    {  // horizontal edges dy = dy0, dy1
        float dx = fminf(fmaxf(-b * dy0 * ia, dx0), dx1);
        m = fminf(m, a * dx * dx + 2.f * b * dx * dy0 + c * dy0 * dy0);
        dx = fminf(fmaxf(-b * dy1 * ia, dx0), dx1);
        m = fminf(m, a * dx * dx + 2.f * b * dx * dy1 + c * dy1 * dy1);
    }
    return m;
}

// 4-bit mask: bit w set <=> some pixel centre of wave w's 8x8 quadrant lies inside the
// record's cull ellipse (d^T conic d <= cullK, see preprocess.hip), i.e. can reach
// alpha >= 1/255.  Evaluated once per loaded record by one lane (lane-parallel).
__device__ __forceinline__ uint32_t quad_mask(const float4 r0, const float4 co, uint32_t tx, uint32_t ty)
{
    const float K = r0.z;
    if (K > 1.0e37f) return 0xFu;  // degenerate conic: never cull
    if (K < 0.f) return 0u;
    const float dx0 = (float)(tx * GSR_BLOCK_X) - r0.x, dy0 = (float)(ty * GSR_BLOCK_Y) - r0.y;
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const float ox = dx0 + (float)((q & 1) * 8), oy = dy0 + (float)((q >> 1) * 8);
        if (box_min_quadform(co.x, co.y, co.z, ox, ox + 7.f, oy, oy + 7.f) <= K) m |= 1u << q;
    }
    return m;
}

// Wave-level stream compaction of the batch entries whose mask bit `w` is set, in order.
// Returns the count; indices land in list[0..count).
__device__ __forceinline__ int compact_batch(const uint8_t* s_mask, int n, int w, int lane, uint8_t* list)
{
    int cnt = 0;
#pragma unroll
    for (int r = 0; r < BATCH / 64; r++) {
        const int j = r * 64 + lane;
        const bool keep = j < n && ((s_mask[j] >> w) & 1);
        const uint64_t b = __ballot(keep);
        const int before = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0));
        if (keep) list[cnt + before] = (uint8_t)j;
        cnt += __popcll(b);
    }
    return cnt;
}

__global__ void __launch_bounds__(256) render_fwd_kernel(RenderFwdArgs a)
{
#pragma clang fp contract(fast)
    const uint32_t tile = blockIdx.x;
    const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    uint32_t px, py;
    quad_pixel(tx, ty, tid, px, py);
    const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint2 range = a.ranges[tile];
    const int todo = (int)(range.y - range.x);

    __shared__ float4 s_rec[BATCH * 3];
    __shared__ uint8_t s_mask[BATCH];
    __shared__ uint8_t s_list[4][BATCH];

    bool done = !inside;
    float T = 1.0f;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f, ID = 0.f;
    uint32_t last_contributor = 0;

    for (int base = 0; base < todo; base += BATCH) {
        if (__syncthreads_and(done)) break;
        const int k = base + tid;
        uint32_t m = 0;
        if (k < todo) {
            const uint32_t id = a.point_list[range.x + k];
            const float4* r = a.splat + 3 * (size_t)id;
            const float4 r0 = r[0];
            s_rec[tid] = r0;
            const float4 r1 = r[1];
            s_rec[BATCH + tid] = r1;
            s_rec[2 * BATCH + tid] = r[2];
            m = quad_mask(r0, r1, tx, ty);
        }
        s_mask[tid] = (uint8_t)m;
        __syncthreads();
        const int n = min(BATCH, todo - base);
        const int cnt = compact_batch(s_mask, n, wid, lane, s_list[wid]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int c = 0; c < cnt; c++) {
            if (__all(done)) break;
            const int j = s_list[wid][c];
            const float4 xy = s_rec[j];
            const float4 co = s_rec[BATCH + j];
            const float dx = xy.x - pfx, dy = xy.y - pfy;
            const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
            const float alpha = fminf(0.99f, co.w * __expf(power));
            bool contrib = !done && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
            const float test_T = T * (1 - alpha);
            if (contrib && test_T < 0.0001f) {
                done = true;
                contrib = false;
            }
            if (contrib) {
                const float4 col = s_rec[2 * BATCH + j];
                C0 += col.x * alpha * T;
                C1 += col.y * alpha * T;
                C2 += col.z * alpha * T;
                ID += col.w * alpha * T;
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

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d, 64));
    return v;
}

// ---- transposed wave reduction (CDNA4 cross-lane ops, no LDS) ------------------------------
__device__ __forceinline__ void xswap32(float& a, float& b)
{
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void xswap16(float& a, float& b)
{
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
template <int CTRL>
__device__ __forceinline__ float dpp(float x)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141, DPP_QUAD_2301 = 0x4E, DPP_QUAD_1032 = 0xB1;

// Sums 64 per-lane values over the 64 lanes of the wave and returns, in lane l, the wave
// total of v[l].  Recursive halving: each exchange step hands half of the live values to the
// partner lane (v_permlane32_swap, v_permlane16_swap, then DPP row_mirror / row_half_mirror /
// quad_perm fused into v_add_f32_dpp), so 64 totals cost ~141 VALU ops instead of the
// 64 x 6 shuffle+add pairs of per-value butterflies.
__device__ __forceinline__ float wave_transpose_reduce64(float (&v)[64], int lane)
{
#pragma unroll
    for (int i = 0; i < 32; i++) { xswap32(v[i], v[i + 32]); v[i] = v[i] + v[i + 32]; }
#pragma unroll
    for (int i = 0; i < 16; i++) { xswap16(v[i], v[i + 16]); v[i] = v[i] + v[i + 16]; }
    const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const float keep = b3 ? v[i + 8] : v[i], send = b3 ? v[i] : v[i + 8];
        v[i] = keep + dpp<DPP_ROW_MIRROR>(send);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const float keep = b2 ? v[i + 4] : v[i], send = b2 ? v[i] : v[i + 4];
        v[i] = keep + dpp<DPP_ROW_HALF_MIRROR>(send);
    }
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const float keep = b1 ? v[i + 2] : v[i], send = b1 ? v[i] : v[i + 2];
        v[i] = keep + dpp<DPP_QUAD_2301>(send);
    }
    const float keep = b0 ? v[1] : v[0], send = b0 ? v[0] : v[1];
    return keep + dpp<DPP_QUAD_1032>(send);
}

constexpr int GROUP = 6;  // Gaussians per transposed reduction (6 x 10 gradient terms <= 64 lanes)

__global__ void __launch_bounds__(256, 2) render_bwd_kernel(RenderBwdArgs a)
{
#pragma clang fp contract(fast)
    const uint32_t tile = blockIdx.x;
    const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    uint32_t px, py;
    quad_pixel(tx, ty, tid, px, py);
    const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint2 range = a.ranges[tile];
    const int todo = (int)(range.y - range.x);
    const uint32_t pix_id = (uint32_t)a.W * py + px;
    const size_t HW = (size_t)a.H * a.W;

    __shared__ float4 s_rec[BATCH * 3];
    __shared__ uint8_t s_mask[BATCH];
    __shared__ uint8_t s_list[4][BATCH];
    __shared__ float s_part[4][BATCH * GF_NUM];
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
    const bool has_inv = a.dL_invdepths != nullptr;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc_inv = 0.f;
    float last_alpha = 0.f, last_c0 = 0.f, last_c1 = 0.f, last_c2 = 0.f, last_inv = 0.f;
    const float ddelx_dx = 0.5 * a.W;
    const float ddely_dy = 0.5 * a.H;
    const float bg_dot_dpixel = a.bg[0] * dpix0 + a.bg[1] * dpix1 + a.bg[2] * dpix2;

    // Entries at or behind the largest n_contrib of a wave (tile) contribute nothing to it.
    const uint32_t wmax = wave_max_u32(last_contributor);
    if (lane == 0) s_wmax[wid] = wmax;
    __syncthreads();
    const uint32_t tmax = max(max(s_wmax[0], s_wmax[1]), max(s_wmax[2], s_wmax[3]));
    const uint32_t wm0 = s_wmax[0], wm1 = s_wmax[1], wm2 = s_wmax[2], wm3 = s_wmax[3];
    const int skip = todo - (int)tmax;
    // zero records for the skipped tail (list positions tmax..todo-1)
    {
        float4* z = reinterpret_cast<float4*>(a.grad_inst + (size_t)(range.x + tmax) * GRAD_REC);
        for (int k = tid; k < skip * (GRAD_REC / 4); k += 256) z[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }

    for (int base = skip; base < todo; base += BATCH) {
        __syncthreads();
        const int k = base + tid;
        uint32_t m = 0;
        if (k < todo) {
            const uint32_t id = a.point_list[range.y - k - 1];
            const float4* r = a.splat + 3 * (size_t)id;
            const float4 r0 = r[0];
            s_rec[tid] = r0;
            const float4 r1 = r[1];
            s_rec[BATCH + tid] = r1;
            s_rec[2 * BATCH + tid] = r[2];
            m = quad_mask(r0, r1, tx, ty);
            const uint32_t pos = (uint32_t)(todo - 1 - k);
            m &= (uint32_t)(pos < wm0) | ((uint32_t)(pos < wm1) << 1) | ((uint32_t)(pos < wm2) << 2) |
                 ((uint32_t)(pos < wm3) << 3);
        }
        s_mask[tid] = (uint8_t)m;
        {
            float4* zp = reinterpret_cast<float4*>(s_part[wid]);
            for (int q = lane; q < BATCH * GF_NUM / 4; q += 64) zp[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        __syncthreads();
        const int n = min(BATCH, todo - base);
        const int cnt = compact_batch(s_mask, n, wid, lane, s_list[wid]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int g0 = 0; g0 < cnt; g0 += GROUP) {
            float v[64];
            bool anyc = false;
#pragma unroll
            for (int jj = 0; jj < GROUP; jj++) {
                float* o = v + jj * GF_NUM;
#pragma unroll
                for (int q = 0; q < GF_NUM; q++) o[q] = 0.f;
                if (g0 + jj < cnt) {  // wave-uniform
                    const int j = s_list[wid][g0 + jj];
                    const uint32_t pos = (uint32_t)(todo - 1 - (base + j));
                    const float4 xy = s_rec[j];
                    const float4 co = s_rec[BATCH + j];
                    const float dx = xy.x - pfx, dy = xy.y - pfy;
                    const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                    const float G = __expf(power);
                    const float alpha = fminf(0.99f, co.w * G);
                    const bool contrib =
                        inside && pos < last_contributor && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
                    if (contrib) {
                        anyc = true;
                        const float4 col = s_rec[2 * BATCH + j];
                        const float one_m = 1.f - alpha;
                        // v_rcp_f32 (1 ulp) in place of the IEEE divisions of backward.cu:573,615
                        const float r_om = __builtin_amdgcn_rcpf(one_m);
                        T = T * r_om;
                        const float dchannel_dcolor = alpha * T;
                        float dL_dalpha = 0.0f;
                        acc0 = last_alpha * last_c0 + (1.f - last_alpha) * acc0;
                        acc1 = last_alpha * last_c1 + (1.f - last_alpha) * acc1;
                        acc2 = last_alpha * last_c2 + (1.f - last_alpha) * acc2;
                        last_c0 = col.x; last_c1 = col.y; last_c2 = col.z;
                        dL_dalpha += (col.x - acc0) * dpix0;
                        dL_dalpha += (col.y - acc1) * dpix1;
                        dL_dalpha += (col.z - acc2) * dpix2;
                        o[GF_COLOR_R] = dchannel_dcolor * dpix0;
                        o[GF_COLOR_G] = dchannel_dcolor * dpix1;
                        o[GF_COLOR_B] = dchannel_dcolor * dpix2;
                        if (has_inv) {
                            const float invd = col.w;
                            acc_inv = last_alpha * last_inv + (1.f - last_alpha) * acc_inv;
                            last_inv = invd;
                            dL_dalpha += (invd - acc_inv) * dinv;
                            o[GF_INVDEPTH] = dchannel_dcolor * dinv;
                        }
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        dL_dalpha += (-T_final * r_om) * bg_dot_dpixel;
                        const float dL_dG = co.w * dL_dalpha;
                        const float gdx = G * dx;
                        const float gdy = G * dy;
                        const float dG_ddelx = -gdx * co.x - gdy * co.y;
                        const float dG_ddely = -gdy * co.z - gdx * co.y;
                        o[GF_MEAN2D_X] = dL_dG * dG_ddelx * ddelx_dx;
                        o[GF_MEAN2D_Y] = dL_dG * dG_ddely * ddely_dy;
                        o[GF_CONIC_A] = -0.5f * gdx * dx * dL_dG;
                        o[GF_CONIC_B] = -0.5f * gdx * dy * dL_dG;
                        o[GF_CONIC_C] = -0.5f * gdy * dy * dL_dG;
                        o[GF_OPACITY] = G * dL_dalpha;
                    }
                }
            }
#pragma unroll
            for (int q = GROUP * GF_NUM; q < 64; q++) v[q] = 0.f;
            if (__any(anyc)) {
                const float r = wave_transpose_reduce64(v, lane);
                const int jj = lane / GF_NUM;
                if (lane < GROUP * GF_NUM && g0 + jj < cnt)
                    s_part[wid][s_list[wid][g0 + jj] * GF_NUM + (lane - jj * GF_NUM)] = r;
            }
        }
        __syncthreads();
        if (tid < n) {
            float rec[GRAD_REC];
#pragma unroll
            for (int q = 0; q < GF_NUM; q++)
                rec[q] = ((s_part[0][tid * GF_NUM + q] + s_part[1][tid * GF_NUM + q]) + s_part[2][tid * GF_NUM + q]) +
                         s_part[3][tid * GF_NUM + q];
            rec[10] = 0.f;
            rec[11] = 0.f;
            float4* dst = reinterpret_cast<float4*>(a.grad_inst + (size_t)(range.y - (base + tid) - 1) * GRAD_REC);
            dst[0] = make_float4(rec[0], rec[1], rec[2], rec[3]);
            dst[1] = make_float4(rec[4], rec[5], rec[6], rec[7]);
            dst[2] = make_float4(rec[8], rec[9], rec[10], rec[11]);
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
