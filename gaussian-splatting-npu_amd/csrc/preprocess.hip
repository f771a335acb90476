// preprocess.hip -- FORWARD::preprocess (forward.cu:154-272, launch :459-486),
// markVisible/checkFrustum (rasterizer_impl.cu:54-66, 141-153) and the
// inclusive scan of tiles_touched (cub::DeviceScan::InclusiveSum,
// rasterizer_impl.cu:280) for gfx950.
//
// Compiled with -ffp-contract=off: every value on the key-producing path is
// bit-identical to oracle/gsr_oracle.c (depth bits, radii, rect, tile counts).
// One thread per Gaussian, 256-thread blocks (4 wave64s).  HBM-bound: the
// per-Gaussian input is 236 B at SH degree 3 (means 12, scales 12, rot 16,
// opacity 4, SH 192); output record 44 B.
#include "gsr_common.h"
#include "gsr_kernels.h"

namespace gsr {


// forward.cu:74-109
__device__ __forceinline__ f3 computeCov2D(const f3 mean, float focal_x, float focal_y, float tan_fovx,
                                           float tan_fovy, const float* cov3D, const float* v)
{
    f3 t = transformPoint4x3(mean, v);
    const float limx = 1.3f * tan_fovx;
    const float limy = 1.3f * tan_fovy;
    const float txtz = t.x / t.z;
    const float tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    mat3 J = mat3_cols(focal_x / t.z, 0.0f, -(focal_x * t.x) / (t.z * t.z),
                       0.0f, focal_y / t.z, -(focal_y * t.y) / (t.z * t.z),
                       0, 0, 0);
    mat3 W = mat3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    mat3 T = mat3_mul(W, J);
    mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4],
                         cov3D[5]);
    mat3 cov = mat3_mul(mat3_mul(mat3_T(T), mat3_T(Vrk)), T);
    return {cov.m[0][0], cov.m[0][1], cov.m[1][1]};
}

// forward.cu:20-71
// `sh0` holds coefficient 0 and sh[3k..3k+2] coefficient k >= 1 (sh0 == sh for one (P,M,3) row;
// with a separate dc row, sh = rest row - 3, never dereferenced below index 3).
__device__ __forceinline__ f3 computeColorFromSH(const f3 pos, int deg, const float* sh0, const float* sh,
                                                 const float* campos, uint8_t& clamped)
{
    f3 dir = {pos.x - campos[0], pos.y - campos[1], pos.z - campos[2]};
    const float len = sqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
    dir.x = dir.x / len; dir.y = dir.y / len; dir.z = dir.z / len;
    float res[3];
#pragma unroll
    for (int c = 0; c < 3; c++) res[c] = SH_C0 * sh0[c];
    if (deg > 0) {
        const float x = dir.x, y = dir.y, z = dir.z;
#pragma unroll
        for (int c = 0; c < 3; c++)
            res[c] = res[c] - SH_C1 * y * sh[1 * 3 + c] + SH_C1 * z * sh[2 * 3 + c] - SH_C1 * x * sh[3 * 3 + c];
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
#pragma unroll
            for (int c = 0; c < 3; c++)
                res[c] = res[c] + SH_C2_0 * xy * sh[4 * 3 + c] + SH_C2_1 * yz * sh[5 * 3 + c] +
                         SH_C2_2 * (2.0f * zz - xx - yy) * sh[6 * 3 + c] + SH_C2_3 * xz * sh[7 * 3 + c] +
                         SH_C2_4 * (xx - yy) * sh[8 * 3 + c];
            if (deg > 2) {
#pragma unroll
                for (int c = 0; c < 3; c++)
                    res[c] = res[c] + SH_C3_0 * y * (3.0f * xx - yy) * sh[9 * 3 + c] +
                             SH_C3_1 * xy * z * sh[10 * 3 + c] +
                             SH_C3_2 * y * (4.0f * zz - xx - yy) * sh[11 * 3 + c] +
                             SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[12 * 3 + c] +
                             SH_C3_4 * x * (4.0f * zz - xx - yy) * sh[13 * 3 + c] +
                             SH_C3_5 * z * (xx - yy) * sh[14 * 3 + c] +
                             SH_C3_6 * x * (xx - 3.0f * yy) * sh[15 * 3 + c];
            }
        }
    }
    uint8_t cl = 0;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        res[c] += 0.5f;
        if (res[c] < 0) cl |= (uint8_t)(1u << c);
        res[c] = res[c] < 0.0f ? 0.0f : res[c];
    }
    clamped = cl;
    return {res[0], res[1], res[2]};
}

// A Gaussian's own inputs (the same in every view), loaded before the block's SH staging barrier
// so their round trip overlaps the staging.
struct GaussIn {
    f3 p;
    float4 rot;
    float scl[3];
    float opacity;
    float cov3D[6];  // cov3D_precomp only
};

__device__ __forceinline__ GaussIn load_gauss(const PreprocessArgs& a, int idx)
{
    GaussIn g;
    g.p = {a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]};
    g.rot = make_float4(0.f, 0.f, 0.f, 0.f);
    g.scl[0] = g.scl[1] = g.scl[2] = 0.f;
#pragma unroll
    for (int k = 0; k < 6; k++) g.cov3D[k] = 0.f;
    if (!a.cov3D_precomp) {
        const float* rp = a.rotations + 4 * (size_t)idx;
        g.rot = make_float4(rp[0], rp[1], rp[2], rp[3]);
        const float* sp = a.scales + 3 * (size_t)idx;
        g.scl[0] = sp[0]; g.scl[1] = sp[1]; g.scl[2] = sp[2];
    } else {
        const float* c = a.cov3D_precomp + (size_t)idx * 6;
#pragma unroll
        for (int k = 0; k < 6; k++) g.cov3D[k] = c[k];
    }
    g.opacity = a.opacities[idx];
    return g;
}

// One Gaussian; `sh` points at its SH coefficients (global memory or its LDS staging row).
__device__ __forceinline__ void preprocess_one(const PreprocessArgs& a, int idx, const GaussIn& gi, const float* sh0,
                                               const float* sh)
{

    // culled: these four are written here and only here (a visible Gaussian writes them once, below)
    auto cull = [&]() {
        a.radii[idx] = 0;
        a.tiles_touched[idx] = 0;
        if (a.rect4) a.rect4[idx] = 0u;
        else a.rect[idx] = make_uint2(0u, 0u);
        a.dkey[idx] = 0xFFFFFFFFu;  // culled Gaussians sort behind every visible one
    };

    const f3 p_orig = gi.p;
    const float opacity_in = gi.opacity;
    // in_frustum (auxiliary.h:151-176)
    const f3 p_view = transformPoint4x3(p_orig, a.view);
    if (p_view.z <= 0.2f) {
        if (a.prefiltered) __hip_atomic_store(a.host_flags, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        cull();
        return;
    }
    const float4 p_hom = transformPoint4x4(p_orig, a.proj);
    const float p_w = 1.0f / (p_hom.w + 0.0000001f);
    const float ppx = p_hom.x * p_w, ppy = p_hom.y * p_w;

    // One local array filled either way: a pointer choosing between global memory and a local
    // array forced the local copy into scratch (32 B/lane; 0.099 -> 0.094 ms without it).
    float cov3D[6];
    if (a.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; k++) cov3D[k] = gi.cov3D[k];
    } else {
        computeCov3D(gi.scl, a.scale_modifier, gi.rot, cov3D);  // recomputed by preprocess_bwd, not stored
    }

    f3 cov = computeCov2D(p_orig, a.focal_x, a.focal_y, a.tan_fovx, a.tan_fovy, cov3D, a.view);
    const float h_var = 0.3f;
    const float det_cov = cov.x * cov.z - cov.y * cov.y;
    cov.x += h_var;
    cov.z += h_var;
    const float det_cov_plus_h_cov = cov.x * cov.z - cov.y * cov.y;
    float h_convolution_scaling = 1.0f;
    if (a.antialiasing) h_convolution_scaling = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus_h_cov));

    const float det = det_cov_plus_h_cov;
    if (det == 0.0f) { cull(); return; }
    const float det_inv = 1.f / det;
    const float conic_x = cov.z * det_inv, conic_y = -cov.y * det_inv, conic_z = cov.x * det_inv;

    const float mid = 0.5f * (cov.x + cov.z);
    const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
    const float pix_x = ndc2Pix(ppx, a.W), pix_y = ndc2Pix(ppy, a.H);
    uint32_t rminx, rminy, rmaxx, rmaxy;
    getRect(pix_x, pix_y, (int)my_radius, a.grid_x, a.grid_y, rminx, rminy, rmaxx, rmaxy);
    if ((rmaxx - rminx) * (rmaxy - rminy) == 0) { cull(); return; }

    f3 rgb;
    if (!a.colors_precomp) {
        uint8_t cl;
        rgb = computeColorFromSH(p_orig, a.D, sh0, sh, a.campos, cl);
        if (a.rgb) {
            a.rgb[3 * (size_t)idx + 0] = rgb.x;
            a.rgb[3 * (size_t)idx + 1] = rgb.y;
            a.rgb[3 * (size_t)idx + 2] = rgb.z;
        }
        a.clamped[idx] = cl;
    } else {
        const float* c = a.colors_precomp + 3 * (size_t)idx;
        rgb = {c[0], c[1], c[2]};
    }
    if (a.depths) a.depths[idx] = p_view.z;
    a.dkey[idx] = __float_as_uint(p_view.z);  // z > 0.2: float bits are monotone in z
    a.radii[idx] = (int)my_radius;
    if (a.means2D) reinterpret_cast<float2*>(a.means2D)[idx] = make_float2(pix_x, pix_y);
    const float opacity = opacity_in * h_convolution_scaling;
    if (a.conic_opacity)  // (the batched forward stores none: preprocess_bwd recomputes it)
        reinterpret_cast<float4*>(a.conic_opacity)[idx] = make_float4(conic_x, conic_y, conic_z, opacity);
    a.tiles_touched[idx] = (rmaxy - rminy) * (rmaxx - rminx);
    if (a.rect4) a.rect4[idx] = rect_pack(rminx, rminy, rmaxx, rmaxy);
    else a.rect[idx] = make_uint2(rminx | (rminy << 16), rmaxx | (rmaxy << 16));

    // Render record.  cullK bounds the ellipse d^T Q d <= K = 2 ln(255 opacity) outside which
    // alpha = opacity * exp(power) < 1/255 (Q = the fp32 conic the render kernels evaluate),
    // widened by a margin far above the fp32 rounding of `power`.  The render kernels use it
    // only to skip (Gaussian, 8x8-quadrant) pairs in which no pixel can pass the reference's
    // alpha >= 1/255 test (forward.cu:364, backward.cu:570), so results are unchanged.
    // Opacity below 1/255 can never pass: cullK < 0 culls everywhere.
    float cullK = -1.0f;
    if (opacity >= 1.0f / 255.0f) cullK = (float)(2.0 * log(255.0 * (double)opacity) * 1.002 + 0.02);
    if (!(conic_x > 0.f && conic_z > 0.f && conic_x * conic_z - conic_y * conic_y > 0.f)) cullK = 3.0e38f;
    // The record carries the conic pre-scaled into the log2-domain falloff the render kernels
    // evaluate (render.hip Falloff: p2 = ka dx^2 + kb dx dy + kc dy^2 = log2(e) * power), and
    // cullK in the same scale (q' = -(ka dx^2 + kb dx dy + kc dy^2) <= log2(e)/2 * K).
    [[maybe_unused]] constexpr float LOG2E = 1.4426950408889634f;
#if !GSR_REF_ALPHA
    if (cullK >= 0.f && cullK < 1.0e37f) cullK = cullK * (0.5f * LOG2E);
#endif
    float4* sp = a.splat + 3 * (size_t)idx;
    // (word 3: the packed tile rect, from which render_bwd derives an instance's record slot)
    sp[0] = make_float4(pix_x, pix_y, cullK, a.rect4 ? __uint_as_float(rect_pack(rminx, rminy, rmaxx, rmaxy)) : 0.0f);
#if GSR_REF_ALPHA  // (test build: the plain conic, cullK in units of d^T conic d)
    sp[1] = make_float4(conic_x, conic_y, conic_z, opacity);
#else
    sp[1] = make_float4((-0.5f * LOG2E) * conic_x, (-LOG2E) * conic_y, (-0.5f * LOG2E) * conic_z, opacity);
#endif
    sp[2] = make_float4(rgb.x, rgb.y, rgb.z, 1.0f / p_view.z);
}

// SH coefficients are 192 of the 236 bytes read per Gaussian at degree 3.  STAGED: the block's
// 256 x 3M floats arrive through LDS with coalesced 16-byte loads (rows padded to an odd number
// of dwords, so the per-thread row walks are bank-conflict-free) instead of every lane striding
// 3M floats through global memory.  NV > 1: the block's Gaussians for up to NV views of the same
// Gaussians (a batch of views, gsr_forward_views): their parameters and SH rows are read from HBM
// once, each view's outputs go to its own buffers (A.a[v]).
// Threads (Gaussians) per preprocess workgroup.  64 lets the next view's preprocess slip into
// single-wave holes beside a running render_bwd, but once render_bwd frees 4-wave holes
// (BWD_TPW) 256 measures as fast (same-box A/B 2,302 vs 2,325 Mpix/s).
constexpr int PF_TPB = 256;

template <int NV>
struct PreprocessBatch {
    PreprocessArgs a[NV];
    int V;
};

template <bool STAGED, int NV>
__global__ void __launch_bounds__(PF_TPB) preprocess_fwd_kernel(const PreprocessBatch<NV> A, int lds_stride)
{
    extern __shared__ __attribute__((aligned(16))) float s_sh[];
    const PreprocessArgs& a = A.a[0];  // the Gaussian inputs (the same in every view)
    const int base = blockIdx.x * PF_TPB;
    const int idx = base + (int)threadIdx.x;
    const int V = NV == 1 ? 1 : A.V;
    for (int v = 0; v < V; v++)
        if (idx < A.a[v].scan_status_words) A.a[v].scan_status[idx] = 0;  // the scans run after this kernel
    if (idx < a.P)  // render_bwd ORs the records it writes into it
        for (int v = 0; v < V; v++) A.a[v].rec_mask[idx] = 0u;
    for (int v = 0; v < V; v++)  // tile_hist adds into it after this kernel (grid-stride: P may be small)
        if (A.a[v].tile_diff)
            for (int c = idx; c < A.a[v].tile_diff_words; c += (int)gridDim.x * PF_TPB) A.a[v].tile_diff[c] = 0;
    for (int v = 0; v < V; v++)  // the depth sort's count kernels add into them after this kernel
        if (A.a[v].dsort_gsum)
            for (int c = idx; c < A.a[v].dsort_gsum_words; c += (int)gridDim.x * PF_TPB) A.a[v].dsort_gsum[c] = 0u;
    // the Gaussian's own inputs first: their loads are in flight during the SH staging
    GaussIn gi;
    if (idx < a.P) gi = load_gauss(a, idx);
    auto views = [&](const float* sh0, const float* sh) {
        if (idx >= a.P) return;
        for (int v = 0; v < V; v++) preprocess_one(A.a[v], idx, gi, sh0, sh);
    };
    if (!STAGED) {
        const float* row = a.shs ? a.shs + (size_t)idx * a.M * 3 : nullptr;
        views(row, row);
        return;
    }
    if (a.dc && a.M <= 16) {  // separate dc, verbatim: dc rows at 0, rest rows (stride 3(M-1)) after them
        const int n = min(PF_TPB, a.P - base), wr = (a.M - 1) * 3;
        float* s_rest = s_sh + 3 * PF_TPB;
        lds_copy_in(s_sh, a.dc + (size_t)base * 3, n * 3);
        if (wr > 0) lds_copy_in(s_rest, a.shs + (size_t)base * wr, n * wr);
        __syncthreads();
        views(s_sh + 3 * threadIdx.x, s_rest + wr * threadIdx.x - 3);
        return;
    }
    if (a.dc) {  // separate dc, wide rest rows: coefficient 0 into columns 0-2, the rest after it (16 used)
        const int n = min(PF_TPB, a.P - base), ncols = min(a.M, 16) * 3;
        lds_rows_in(s_sh, lds_stride, 0, ncols, a.dc + (size_t)base * 3, 3, n);
        if (a.shs && a.M > 1) lds_rows_in(s_sh, lds_stride, 3, ncols, a.shs + (size_t)base * (a.M - 1) * 3,
                                          (a.M - 1) * 3, n);
        __syncthreads();
        const float* row = s_sh + threadIdx.x * lds_stride;
        views(row, row);
        return;
    }
    const int W3 = a.M * 3;  // multiple of 4 on this path
    const int nv4 = min(PF_TPB, a.P - base) * (W3 / 4);
    const float4* src = reinterpret_cast<const float4*>(a.shs + (size_t)base * W3);
    auto put = [&](int f, const float4 v) {
        const int g = (f * 4) / W3, w = (f * 4) - g * W3;
        float* d = &s_sh[g * lds_stride + w];
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    };
    // 12 loads in flight per thread (a whole block at degree 3) before the first LDS store: one
    // loop iteration per load would wait out 12 round trips
    constexpr int U = 12;
    int f = threadIdx.x;
    for (; f + (U - 1) * PF_TPB < nv4; f += U * PF_TPB) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = src[f + u * PF_TPB];
#pragma unroll
        for (int u = 0; u < U; u++) put(f + u * PF_TPB, v[u]);
    }
    for (; f < nv4; f += PF_TPB) put(f, src[f]);
    __syncthreads();
    const float* row = s_sh + threadIdx.x * lds_stride;
    views(row, row);
}

__global__ void __launch_bounds__(256) mark_visible_kernel(int P, const float* means3D, const float* view,
                                                           bool* present)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const f3 p = {means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]};
    present[idx] = !(transformPoint4x3(p, view).z <= 0.2f);
}

// ---------------------------------------------------------------------------
// Inclusive scan of u32 counts in one launch (cub::DeviceScan::InclusiveSum,
// rasterizer_impl.cu:166,280): chunks of SCAN_ITEMS take a ticket (so every chunk's
// predecessors were scheduled before it), reduce locally, publish their aggregate, then
// resolve their exclusive prefix by decoupled look-back: one wave reads the status words of
// the 64 preceding chunks at once and sums back to the nearest inclusive one.  A status word
// is {flag (2 bits), value (32 bits)} in one 64-bit agent-scope atomic, so the value travels
// with its flag.
// ---------------------------------------------------------------------------
constexpr uint64_t SCAN_AGG = 1ull << 62, SCAN_INC = 2ull << 62, SCAN_FLAGS = 3ull << 62;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t n = __shfl_up(v, d, 64);
        if (lane >= d) v += n;
    }
    return v;
}

// block-wide exclusive scan of one value per thread (256 threads); returns exclusive prefix, total in *tot
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* lds4, uint32_t& total)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(v);
    if (lane == 63) lds4[wid] = inc;
    __syncthreads();
    uint32_t wprefix = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        uint32_t s = lds4[w];
        if (w < wid) wprefix += s;
        total += s;
    }
    __syncthreads();
    return wprefix + inc - v;
}

// Exclusive prefix of chunk c from the status words of chunks < c (run by one whole wave).
__device__ __forceinline__ uint32_t scan_lookback(uint64_t* status, int c, int lane)
{
    uint32_t excl = 0;
    int j = c - 1;  // newest predecessor not yet summed
    while (j >= 0) {
        const int k = j - lane;
        uint64_t st = k >= 0 ? __hip_atomic_load(status + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : SCAN_INC;
        const uint64_t inc = __ballot((st & SCAN_FLAGS) == SCAN_INC);
        const int stop = inc ? (int)__builtin_ctzll(inc) : 63;  // lanes [0, stop] are needed
        const uint64_t missing = __ballot((st & SCAN_FLAGS) == 0 && lane <= stop);
        if (missing) continue;  // a needed predecessor has not published yet: re-read
        uint32_t v = lane <= stop && k >= 0 ? (uint32_t)st : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v += (uint32_t)__shfl_xor((int)v, d, 64);
        excl += v;
        if (inc) break;
        j -= 64;
    }
    return excl;
}

// Inclusive (or, with `exclusive`, exclusive) scan of in[gather[i]] into out; the total goes to
// total_out (may be null).
struct ScanKArgs {
    const uint32_t* in;
    const uint32_t* gather;
    int n, nchunks;
    uint64_t* status;
    uint32_t* out;
    uint32_t* total_out;
};
__global__ void __launch_bounds__(256) scan_lookback_kernel(const ViewBatch<ScanKArgs> B, bool exclusive)
{
    const ScanKArgs& J = B.v[blockIdx.y];
    const int nchunks = J.nchunks;
    if ((int)blockIdx.x >= nchunks) return;  // past this view's chunks (uniform, before taking a ticket)
    const uint32_t* in = J.in;
    const uint32_t* gather = J.gather;
    const int n = J.n;
    uint64_t* status = J.status;
    uint32_t* out = J.out;
    uint32_t* total_out = J.total_out;
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t s_chunk, s_excl;
    uint32_t* ticket = reinterpret_cast<uint32_t*>(status + nchunks);
    if (threadIdx.x == 0) s_chunk = atomicAdd(ticket, 1u);
    __syncthreads();
    const int c = (int)s_chunk;
    // each thread owns 16 consecutive items; every load issued before the first use
    const size_t base = (size_t)c * SCAN_ITEMS + (size_t)threadIdx.x * 16;
    uint32_t v[16];
    if (!gather && base + 16 <= (size_t)n && ((uintptr_t)in & 15) == 0) {  // 4 x 16-byte loads
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 q = reinterpret_cast<const uint4*>(in + base)[k];
            v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const size_t i = base + k;
            v[k] = i < (size_t)n ? (gather ? gather[i] : (uint32_t)i) : 0u;
        }
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = base + k < (size_t)n ? in[v[k]] : 0u;
    }
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) s += v[k];
    uint32_t total;
    uint32_t ex = block_excl_scan256(s, lds4, total);
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        if (lane == 0)
            __hip_atomic_store(status + c, (c == 0 ? SCAN_INC : SCAN_AGG) | total, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t excl = c == 0 ? 0u : scan_lookback(status, c, lane);
        if (lane == 0) {
            if (c > 0)
                __hip_atomic_store(status + c, SCAN_INC | (uint64_t)(excl + total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            if (c == nchunks - 1 && total_out)
                __hip_atomic_store(total_out, excl + total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            s_excl = excl;
        }
    }
    __syncthreads();
    ex += s_excl;
    const bool incl = !exclusive;
    if (base + 16 <= (size_t)n && ((uintptr_t)out & 15) == 0) {  // 4 x 16-byte stores
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t o[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const uint32_t nx = ex + v[4 * k + e];
                o[e] = incl ? nx : ex;
                ex = nx;
            }
            reinterpret_cast<uint4*>(out + base)[k] = make_uint4(o[0], o[1], o[2], o[3]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t nx = ex + v[k];
            const size_t i = base + k;
            if (i < (size_t)n) out[i] = incl ? nx : ex;
            ex = nx;
        }
    }
}

template <int NV>
static hipError_t launch_preprocess_batch(const PreprocessBatch<NV>& A, hipStream_t s)
{
    const PreprocessArgs& a = A.a[0];
    if (a.P <= 0) return hipSuccess;
    const int W3 = a.M * 3;
    const bool staged = a.shs && !a.colors_precomp && W3 > 0 && W3 % 4 == 0 && W3 <= 64 &&
                        ((uintptr_t)a.shs % 16) == 0;
    const dim3 grid((a.P + PF_TPB - 1) / PF_TPB), block(PF_TPB);
    if (a.dc && !a.colors_precomp) {  // separate dc: always staged (any M, any alignment)
        const int stride = (min(a.M, 16) * 3) | 1;
        const size_t lds = a.M <= 16 ? ((size_t)PF_TPB * 3 + PF_TPB * (size_t)(a.M - 1) * 3) * sizeof(float)
                                     : PF_TPB * stride * sizeof(float);
        hipLaunchKernelGGL((preprocess_fwd_kernel<true, NV>), grid, block, lds, s, A, stride);
    } else if (staged) {
        const int stride = W3 | 1;
        hipLaunchKernelGGL((preprocess_fwd_kernel<true, NV>), grid, block, PF_TPB * stride * sizeof(float), s, A,
                           stride);
    } else {
        hipLaunchKernelGGL((preprocess_fwd_kernel<false, NV>), grid, block, 0, s, A, 0);
    }
    return hipGetLastError();
}

hipError_t launch_preprocess(const PreprocessArgs& a, hipStream_t s)
{
    PreprocessBatch<1> A;
    A.a[0] = a;
    A.V = 1;
    return launch_preprocess_batch(A, s);
}

hipError_t launch_preprocess_views(const PreprocessArgs* a, int V, hipStream_t s)
{
    for (int v0 = 0; v0 < V; v0 += PREPROCESS_BATCH) {
        PreprocessBatch<PREPROCESS_BATCH> A;
        A.V = min(PREPROCESS_BATCH, V - v0);
        for (int v = 0; v < A.V; v++) A.a[v] = a[v0 + v];
        const hipError_t e = launch_preprocess_batch(A, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_mark_visible(int P, const float* means3D, const float* view, bool* present, hipStream_t s)
{
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, view, present);
    return hipGetLastError();
}

int scan_status_words(int n) { return (n + SCAN_ITEMS - 1) / SCAN_ITEMS + 1; }  // + the ticket

hipError_t launch_inclusive_scan(const uint32_t* in, const uint32_t* gather, uint32_t* out, int n, uint64_t* status,
                                 uint32_t* total_out, hipStream_t s, bool exclusive)
{
    if (n <= 0) return hipSuccess;
    const int nb = (n + SCAN_ITEMS - 1) / SCAN_ITEMS;
    ViewBatch<ScanKArgs> B;
    B.n = 1;
    B.v[0] = {in, gather, n, nb, status, out, total_out};
    hipLaunchKernelGGL(scan_lookback_kernel, dim3(nb), dim3(256), 0, s, B, exclusive);
    return hipGetLastError();
}

hipError_t launch_scan_batch(const ScanJob* jobs, int V, bool exclusive, hipStream_t s)
{
    for (int v0 = 0; v0 < V; v0 += VIEW_BATCH) {
        const int nv = min(VIEW_BATCH, V - v0);
        ViewBatch<ScanKArgs> B;
        B.n = nv;
        int maxc = 0;
        for (int v = 0; v < nv; v++) {
            const ScanJob& j = jobs[v0 + v];
            const int nb = j.n > 0 ? (j.n + SCAN_ITEMS - 1) / SCAN_ITEMS : 0;
            B.v[v] = {j.in, nullptr, j.n, nb, j.status, j.out, j.total_out};
            maxc = max(maxc, nb);
        }
        if (maxc == 0) continue;
        hipLaunchKernelGGL(scan_lookback_kernel, dim3((unsigned)maxc, (unsigned)nv), dim3(256), 0, s, B, exclusive);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace gsr
