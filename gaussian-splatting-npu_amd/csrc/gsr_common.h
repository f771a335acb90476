// gsr_common.h -- shared device helpers and state-buffer layouts for the
// gfx950 rasterizer.  Device math restates the reference helpers in
// cuda_rasterizer/auxiliary.h and the GLM 0.9.9.9 mat3 products the
// reference kernels use (forward.cu, backward.cu); the floating-point
// expression order is kept so that, with -ffp-contract=off (this library's
// default), preprocess outputs are bit-identical to oracle/gsr_oracle.c.
#pragma once
#include <algorithm>

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#define GSR_BLOCK_X 16
#define GSR_BLOCK_Y 16
#define GSR_TILE_PIX (GSR_BLOCK_X * GSR_BLOCK_Y)

namespace gsr {

// auxiliary.h:21-38
__device__ constexpr float SH_C0 = 0.28209479177387814f;
__device__ constexpr float SH_C1 = 0.4886025119029199f;
__device__ constexpr float SH_C2_0 = 1.0925484305920792f;
__device__ constexpr float SH_C2_1 = -1.0925484305920792f;
__device__ constexpr float SH_C2_2 = 0.31539156525252005f;
__device__ constexpr float SH_C2_3 = -1.0925484305920792f;
__device__ constexpr float SH_C2_4 = 0.5462742152960396f;
__device__ constexpr float SH_C3_0 = -0.5900435899266435f;
__device__ constexpr float SH_C3_1 = 2.890611442640554f;
__device__ constexpr float SH_C3_2 = -0.4570457994644658f;
__device__ constexpr float SH_C3_3 = 0.3731763325901154f;
__device__ constexpr float SH_C3_4 = -0.4570457994644658f;
__device__ constexpr float SH_C3_5 = 1.445305721320277f;
__device__ constexpr float SH_C3_6 = -0.5900435899266435f;

struct f3 { float x, y, z; };

// glm::mat3 storage m[col][row]
struct mat3 { float m[3][3]; };

__device__ __forceinline__ mat3 mat3_cols(float a, float b, float c, float d, float e, float f, float g,
                                          float h, float i)
{
    mat3 r;
    r.m[0][0] = a; r.m[0][1] = b; r.m[0][2] = c;
    r.m[1][0] = d; r.m[1][1] = e; r.m[1][2] = f;
    r.m[2][0] = g; r.m[2][1] = h; r.m[2][2] = i;
    return r;
}

// glm type_mat3x3.inl operator*(mat3, mat3)
__device__ __forceinline__ mat3 mat3_mul(const mat3& a, const mat3& b)
{
    mat3 r;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int w = 0; w < 3; w++)
            r.m[c][w] = a.m[0][w] * b.m[c][0] + a.m[1][w] * b.m[c][1] + a.m[2][w] * b.m[c][2];
    return r;
}

__device__ __forceinline__ mat3 mat3_T(const mat3& a)
{
    mat3 r;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int w = 0; w < 3; w++) r.m[c][w] = a.m[w][c];
    return r;
}

// auxiliary.h:70-78
__device__ __forceinline__ f3 transformPoint4x3(const f3 p, const float* m)
{
    return {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
            m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
}

// auxiliary.h:80-89
__device__ __forceinline__ float4 transformPoint4x4(const f3 p, const float* m)
{
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                       m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14],
                       m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}

// auxiliary.h:101-109
__device__ __forceinline__ f3 transformVec4x3Transpose(const f3 p, const float* m)
{
    return {m[0] * p.x + m[1] * p.y + m[2] * p.z,
            m[4] * p.x + m[5] * p.y + m[6] * p.z,
            m[8] * p.x + m[9] * p.y + m[10] * p.z};
}

// auxiliary.h:119-129
__device__ __forceinline__ f3 dnormvdv(const f3 v, const f3 dv)
{
    float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    f3 r;
    r.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}

// auxiliary.h:40-43 (double arithmetic, as the reference's 1.0 literals imply)
__device__ __forceinline__ float ndc2Pix(float v, int S)
{
    return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

// auxiliary.h:45-55
__device__ __forceinline__ void getRect(float px, float py, int max_radius, uint32_t gx, uint32_t gy,
                                        uint32_t& rminx, uint32_t& rminy, uint32_t& rmaxx, uint32_t& rmaxy)
{
    int a;
    a = (int)((px - (float)max_radius) / (float)GSR_BLOCK_X); a = a > 0 ? a : 0;
    rminx = (uint32_t)a < gx ? (uint32_t)a : gx;
    a = (int)((py - (float)max_radius) / (float)GSR_BLOCK_Y); a = a > 0 ? a : 0;
    rminy = (uint32_t)a < gy ? (uint32_t)a : gy;
    a = (int)((px + (float)max_radius + (float)GSR_BLOCK_X - 1.0f) / (float)GSR_BLOCK_X); a = a > 0 ? a : 0;
    rmaxx = (uint32_t)a < gx ? (uint32_t)a : gx;
    a = (int)((py + (float)max_radius + (float)GSR_BLOCK_Y - 1.0f) / (float)GSR_BLOCK_Y); a = a > 0 ? a : 0;
    rmaxy = (uint32_t)a < gy ? (uint32_t)a : gy;
}

// forward.cu:114-151 (also the backward's recomputation: bit-identical under -ffp-contract=off)
__device__ __forceinline__ void computeCov3D(const float* scale, float mod, const float4 rot, float* cov3D)
{
    mat3 S = mat3_cols(1.0f, 0.0f, 0.0f, 0.0f, 1.0f, 0.0f, 0.0f, 0.0f, 1.0f);
    S.m[0][0] = mod * scale[0];
    S.m[1][1] = mod * scale[1];
    S.m[2][2] = mod * scale[2];
    const float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
    mat3 R = mat3_cols(
        1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
        2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
        2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    mat3 M = mat3_mul(S, R);
    mat3 Sigma = mat3_mul(mat3_T(M), M);
    cov3D[0] = Sigma.m[0][0];
    cov3D[1] = Sigma.m[0][1];
    cov3D[2] = Sigma.m[0][2];
    cov3D[3] = Sigma.m[1][1];
    cov3D[4] = Sigma.m[1][2];
    cov3D[5] = Sigma.m[2][2];
}

// ----------------------------------------------------------------------------
// State-buffer layouts (the reference's GeometryState / ImageState /
// BinningState, rasterizer_impl.h:29-65, re-laid out for this implementation).
// Every array starts on a 256-byte boundary.
// ----------------------------------------------------------------------------
__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) & ~(a - 1); }

enum GeomArray {
    GEOM_DEPTH = 0,       // f32[P] view-space z
    GEOM_RADII,           // i32[P] internal radii (used when caller passes radii=NULL)
    GEOM_CLAMPED,         // u8[P]  bit c <=> rgb channel c was clamped (forward.cu:67-69)
    GEOM_MEANS2D,         // f32x2[P]
    GEOM_CONIC_OPACITY,   // f32x4[P]
    GEOM_RGB,             // f32[3P]
    GEOM_TILES_TOUCHED,   // u32[P]
    GEOM_POINT_OFFSETS,   // u32[P] inclusive scan of tiles_touched in depth order
    GEOM_SPLAT,           // f32x12[P] render record: {x, y, cullK, packed rect bits (0 on grids of more than
                          // 255 tiles per axis)} {ka, kb, kc, opacity} {r, g, b, 1/depth}
                          // (ka, kb, kc) = -log2(e) * (a/2, b, c/2) of the conic; cullK scaled by log2(e)/2
    GEOM_DKEY,            // u32[P] depth-sort key: depth bits, 0xFFFFFFFF if culled
    GEOM_SORTED_IDS,      // u32[P] Gaussian ids in (depth bits, index) order
    GEOM_EMIT_START,      // u32[P] first gradient-record slot of each Gaussian (index-order exclusive scan
                          // of tiles_touched)
    GEOM_RECT,            // u16x4[P] tile rect {x0, y0, x1, y1} (getRect), zero if culled; on grids of
                          // <= 255 x 255 tiles the first 4P bytes hold it packed instead (u8x4, rect_pack)
    GEOM_SORTED_RECT,     // u16x4[P] the rects in depth order (last depth-sort pass)
    GEOM_DSORT_TMP,       // depth-sort ping-pong: u32[P] k0, u32x2[P] v0, u32[P] k1, u32x2[P] v1 (payload:
                          // id, packed rect); then the count matrix of the
                          // fused emission + first tile-sort pass (gsr_forward_views)
    GEOM_RADIX_SCRATCH,   // count matrix + digit totals of the depth sort
    GEOM_SCAN_SCRATCH,    // 2 x u64[scan chunks + 1] look-back status words + chunk ticket of the two
                          // scans (depth order, index order; zeroed by preprocess)
    GEOM_REC_MASK,        // u32[P] bit k: Gaussian i's record at slot emit_start[i] + k was written (render_bwd,
                          // k < 32; zeroed by preprocess) -- its records without the valid-word round trip
    GEOM_COUNT
};

enum ImageArray {
    IMG_RANGES = 0,       // u32x2[T]
    IMG_FINAL_T,          // f32[N]
    IMG_N_CONTRIB,        // u32[N]
    IMG_TILE_ORDER,       // u32[T] render launch order: tiles by decreasing work (longest first)
    IMG_TILE_WORK,        // u32[T] largest n_contrib of each tile (written by render_fwd, orders render_bwd)
    IMG_TILE_DIFF,        // i32[(grid_x + 1) (grid_y + 1)] 2-D difference array of the tile rects (tile_hist;
                          // zeroed by preprocess): its 2-D prefix sums are the per-tile instance counts
    IMG_COUNT
};

enum BinArray {
    BIN_POINT_LIST = 0,   // u32[L] Gaussian id of sorted position
    BIN_SORTED_TILES,     // u32[L] tile id of sorted position
    BIN_SLOT,             // u32[L] gradient-record slot of sorted position (GSR_SLOT_LOCAL: minus the
                          // Gaussian's emit_start, i.e. the instance's index in its rect)
    BIN_GRAD_INST,        // f32x12[L] per-(tile, Gaussian) gradient records (backward); during the forward
                          // it hosts the tile sort's ping-pong buffers (24 B/instance)
    BIN_RADIX_SCRATCH,    // count matrix + digit totals of the tile sort
    BIN_VALID,            // u32[ceil(L/32)] bit per record slot: its gradient record was written (backward)
    BIN_HIT,              // u8[L] per sorted position: quadrants (bit w = 8x8 quadrant w) with a pixel the
                          // entry contributed to in the forward (render_fwd), read by render_bwd
    BIN_COUNT
};

constexpr int SCAN_ITEMS = 4096;  // items per scan block (256 threads x 16)
constexpr int DEPTH_BITS = 32;  // depth keys are full float bit patterns

// A tile rect packed into one word (x0, y0, x1, y1: one byte each), for grids of at most 255 x 255
// tiles (4080 x 4080 pixels): the depth sort carries it as payload beside the Gaussian id, so its
// last pass writes the depth-ordered rects without gathering them by id.
__host__ __device__ inline bool rect_packable(uint32_t grid_x, uint32_t grid_y) { return grid_x <= 255u && grid_y <= 255u; }
__host__ __device__ inline uint32_t rect_pack(uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1)
{
    return x0 | (y0 << 8) | (x1 << 16) | (y1 << 24);
}
// the unpacked u16x4 form {x0 | y0 << 16, x1 | y1 << 16}
__host__ __device__ inline uint2 rect_unpack(uint32_t r)
{
    return make_uint2((r & 0xFFu) | (((r >> 8) & 0xFFu) << 16), ((r >> 16) & 0xFFu) | ((r >> 24) << 16));
}

// Tile ranges from the rects' 2-D difference array (tile_hist + tile_order) instead of a pass over
// the sorted tile ids (tile_ranges): grids whose packed rects exist (<= 255 x 255 tiles), whose
// difference array fits a workgroup's LDS and whose tiles one tile-order pass covers (<= 8,192:
// 1080p and below).
constexpr int TILE_DIFF_MAX_CELLS = 8704;
#ifndef GSR_TILE_DIFF
#define GSR_TILE_DIFF 1
#endif
// records found through each Gaussian's record mask (GEOM_REC_MASK, set by render_bwd) instead of
// the valid words
#ifndef GSR_REC_MASK
#define GSR_REC_MASK 1
#endif
// the tile sort's second digit carried in the id word (radix.hip tile_sort_fused_batch)
#ifndef GSR_TILE_PACK
#define GSR_TILE_PACK 1
#endif
// BIN_SLOT holds each instance's index inside its Gaussian's tile rect (its record slot minus the
// Gaussian's emit_start) instead of the absolute record slot
// floats per per-instance gradient record (GRAD_INST): 10 used; 10 = 40 B packed (8-B accesses), 12 =
// 48 B (16-B accesses).  The tile sort's ping-pong buffers (<= 32 B per instance) live in the region.
#ifndef GSR_GRAD_REC
#define GSR_GRAD_REC 10
#endif
static_assert(GSR_GRAD_REC == 10 || GSR_GRAD_REC == 12, "gradient record: 10 or 12 floats");
#ifndef GSR_SLOT_LOCAL
#define GSR_SLOT_LOCAL 1
#endif
// TEST-ONLY build (make refalpha -> refalpha/libgsr_hip_refalpha.so, never loaded by the package):
// the render record carries the plain conic and the render kernels compute power and alpha in the
// reference's operation order with the shared exp of gsr_ref_exp.h (forward.cu:353-363,
// backward.cu:556-571), so that tests/test_ref_alpha_exact.py can hold the blend bit-exact against
// the oracle.  The production build (0) evaluates exp2 of the log2(e)-prescaled falloff instead.
#ifndef GSR_REF_ALPHA
#define GSR_REF_ALPHA 0
#endif
// on grids of packed rects (rect_packable): no record slots at all -- render_bwd derives an instance's
// index in its Gaussian's rect from the packed rect preprocess stores in the render record's free word
// (SPLAT word 3) and the tile, and the tile sort moves 4 B per instance instead of 8
#ifndef GSR_SLOT_RECT
#define GSR_SLOT_RECT 1
#endif
__host__ __device__ inline bool slots_from_rect(uint32_t grid_x, uint32_t grid_y)
{
    return GSR_SLOT_LOCAL && GSR_SLOT_RECT && rect_packable(grid_x, grid_y);
}
// the instance of tile (tx, ty) in the packed rect r: its index in the rect's y-major order
// (duplicateWithKeys, rasterizer_impl.cu:98-109)
__host__ __device__ inline uint32_t rect_local(uint32_t r, uint32_t tx, uint32_t ty)
{
    const uint32_t x0 = r & 0xFFu, y0 = (r >> 8) & 0xFFu, x1 = (r >> 16) & 0xFFu;
    return (ty - y0) * (x1 - x0) + (tx - x0);
}
__host__ __device__ inline bool use_tile_diff(uint32_t grid_x, uint32_t grid_y)
{
    return GSR_TILE_DIFF && rect_packable(grid_x, grid_y) && (grid_x + 1) * (grid_y + 1) <= (uint32_t)TILE_DIFF_MAX_CELLS &&
           grid_x * grid_y <= 8192u;
}

struct GeomLayout { size_t off[GEOM_COUNT + 1]; };
struct ImageLayout { size_t off[IMG_COUNT + 1]; };
struct BinLayout { size_t off[BIN_COUNT + 1]; };

size_t radix_status_bytes(int n, int npass);
size_t fused_pass1_scratch_bytes(int P);  // radix.hip: the fused emission pass's count matrix

inline GeomLayout geom_layout(int P)
{
    size_t p = (size_t)(P > 0 ? P : 0);
    size_t sizes[GEOM_COUNT] = {4 * p, 4 * p, p, 8 * p, 16 * p, 12 * p, 4 * p, 4 * p, 48 * p,
                                4 * p, 4 * p, 4 * p, 8 * p, 8 * p,
                                // (after the depth sort, the fused tile-sort pass's count matrix)
                                std::max(24 * p + 2048, fused_pass1_scratch_bytes(P)), radix_status_bytes(P, 4),
                                16 * ((p + SCAN_ITEMS - 1) / SCAN_ITEMS + 1), 4 * p};
    GeomLayout l;
    size_t o = 0;
    for (int i = 0; i < GEOM_COUNT; i++) { l.off[i] = o; o = align_up(o + sizes[i], 256); }
    l.off[GEOM_COUNT] = o;
    return l;
}

inline ImageLayout image_layout(int W, int H)
{
    size_t n = (size_t)W * H;
    const size_t gx = (size_t)((W + GSR_BLOCK_X - 1) / GSR_BLOCK_X), gy = (size_t)((H + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y);
    size_t t = gx * gy;
    size_t sizes[IMG_COUNT] = {8 * t, 4 * n, 4 * n, 4 * t, 4 * t, 4 * (gx + 1) * (gy + 1)};
    ImageLayout l;
    size_t o = 0;
    for (int i = 0; i < IMG_COUNT; i++) { l.off[i] = o; o = align_up(o + sizes[i], 256); }
    l.off[IMG_COUNT] = o;
    return l;
}

inline BinLayout bin_layout(int L)
{
    size_t n = (size_t)(L > 0 ? L : 0);
    size_t sizes[BIN_COUNT] = {4 * n, 4 * n, 4 * n, 4 * (size_t)GSR_GRAD_REC * n + 4096, radix_status_bytes(L, 4),
                               4 * ((n + 31) / 32), n};
    BinLayout l;
    size_t o = 0;
    for (int i = 0; i < BIN_COUNT; i++) { l.off[i] = o; o = align_up(o + sizes[i], 256); }
    l.off[BIN_COUNT] = o;
    return l;
}

// ---------------------------------------------------------------------------
// Separate-DC SH layout (the `dc=` input of the accelerated upstream rasterizer that
// train.py selects with SparseGaussianAdam, train.py:37-41, gaussian_renderer/__init__.py:82-100):
// coefficient 0 lives in dc (P,1,3), coefficients 1.. in a (P,M-1,3) "rest" array.  Both
// preprocess kernels stage a workgroup's 256 SH rows through LDS; these helpers move a block
// of rows of `w` floats between a global array and LDS columns [col0, col0 + w) of rows of
// `stride` dwords, coalesced (16-byte accesses when the array is 16-byte aligned -- a block
// of 256 rows starts at a multiple of 1 KB, so alignment of the array is alignment of the
// block), dropping (in) / zero-filling (out) columns at or beyond `ncols`.
// ---------------------------------------------------------------------------
constexpr int LDS_IN_BATCH = 6;
__device__ __forceinline__ void lds_rows_in(float* lds, int stride, int col0, int ncols, const float* src, int w,
                                            int n)
{
    const int total = n * w;
    int e0 = 0;
    if (((uintptr_t)src & 15) == 0) {
        const int nv4 = total >> 2;
        const float4* s4 = reinterpret_cast<const float4*>(src);
        auto put = [&](int f, const float4 v) {
            const float vv[4] = {v.x, v.y, v.z, v.w};
            int g = (4 * f) / w, j = 4 * f - g * w;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (col0 + j < ncols) lds[g * stride + col0 + j] = vv[q];
                if (++j == w) { j = 0; g++; }
            }
        };
        // LDS_IN_BATCH loads in flight per thread before their stores (not one round trip each)
        const int bd = (int)blockDim.x;
        int f = threadIdx.x;
        for (; f + (LDS_IN_BATCH - 1) * bd < nv4; f += LDS_IN_BATCH * bd) {
            float4 v[LDS_IN_BATCH];
#pragma unroll
            for (int u = 0; u < LDS_IN_BATCH; u++) v[u] = s4[f + u * bd];
#pragma unroll
            for (int u = 0; u < LDS_IN_BATCH; u++) put(f + u * bd, v[u]);
        }
        for (; f < nv4; f += bd) put(f, s4[f]);
        e0 = nv4 << 2;
    }
    for (int e = e0 + threadIdx.x; e < total; e += blockDim.x) {
        const int g = e / w, j = e - g * w;
        if (col0 + j < ncols) lds[g * stride + col0 + j] = src[e];
    }
}

// Stores d4[f] = val(f) for f in [0, nv4) over the block's threads; with acc, d4[f] += val(f)
// (in-place gradient accumulation).  Accumulating, each thread first issues the loads of up to
// ACC_BATCH of its old values at once and only then adds and stores, so a block pays one memory
// latency per ACC_BATCH elements instead of one per element.
constexpr int ACC_BATCH = 6;
template <typename F>
__device__ __forceinline__ void store_f4(float4* d4, int nv4, bool acc, F val)
{
    if (!acc) {
        for (int f = threadIdx.x; f < nv4; f += blockDim.x) d4[f] = val(f);
        return;
    }
    for (int f0 = 0; f0 < nv4; f0 += ACC_BATCH * (int)blockDim.x) {
        float4 old[ACC_BATCH];
#pragma unroll
        for (int i = 0; i < ACC_BATCH; i++) {
            const int f = f0 + i * (int)blockDim.x + (int)threadIdx.x;
            if (f < nv4) old[i] = d4[f];
        }
#pragma unroll
        for (int i = 0; i < ACC_BATCH; i++) {
            const int f = f0 + i * (int)blockDim.x + (int)threadIdx.x;
            if (f < nv4) {
                const float4 v = val(f);
                d4[f] = make_float4(old[i].x + v.x, old[i].y + v.y, old[i].z + v.z, old[i].w + v.w);
            }
        }
    }
}

__device__ __forceinline__ void lds_rows_out(float* dst, int w, int n, const float* lds, int stride, int col0,
                                             int ncols, bool acc = false)
{
    const int total = n * w;
    int e0 = 0;
    if (((uintptr_t)dst & 15) == 0) {
        const int nv4 = total >> 2;
        store_f4(reinterpret_cast<float4*>(dst), nv4, acc, [&](int f) {
            float vv[4];
            int g = (4 * f) / w, j = 4 * f - g * w;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                vv[q] = col0 + j < ncols ? lds[g * stride + col0 + j] : 0.f;
                if (++j == w) { j = 0; g++; }
            }
            return make_float4(vv[0], vv[1], vv[2], vv[3]);
        });
        e0 = nv4 << 2;
    }
    for (int e = e0 + threadIdx.x; e < total; e += blockDim.x) {
        const int g = e / w, j = e - g * w;
        const float v = col0 + j < ncols ? lds[g * stride + col0 + j] : 0.f;
        dst[e] = acc ? dst[e] + v : v;
    }
}

// Verbatim block copies between a global array and LDS (the separate-DC staging with rows of
// <= 16 coefficients keeps the global row layout in LDS: the dc rows have a stride of 3 dwords and
// degree-3 rest rows 45, both odd, so per-thread row walks are bank-conflict-free without
// padding, and the copy needs no index arithmetic).  16-byte accesses when both sides allow it.
__device__ __forceinline__ void lds_copy_in(float* lds, const float* src, int total)
{
    int e0 = 0;
    if (((uintptr_t)src & 15) == 0 && ((uintptr_t)lds & 15) == 0) {
        const int nv4 = total >> 2, bd = (int)blockDim.x;
        const float4* s4 = reinterpret_cast<const float4*>(src);
        float4* l4 = reinterpret_cast<float4*>(lds);
        int f = threadIdx.x;
        for (; f + (LDS_IN_BATCH - 1) * bd < nv4; f += LDS_IN_BATCH * bd) {
            float4 v[LDS_IN_BATCH];
#pragma unroll
            for (int u = 0; u < LDS_IN_BATCH; u++) v[u] = s4[f + u * bd];
#pragma unroll
            for (int u = 0; u < LDS_IN_BATCH; u++) l4[f + u * bd] = v[u];
        }
        for (; f < nv4; f += bd) l4[f] = s4[f];
        e0 = nv4 << 2;
    }
    for (int e = e0 + threadIdx.x; e < total; e += blockDim.x) lds[e] = src[e];
}

__device__ __forceinline__ void lds_copy_out(float* dst, const float* lds, int total, bool acc = false)
{
    int e0 = 0;
    if (((uintptr_t)dst & 15) == 0 && ((uintptr_t)lds & 15) == 0) {
        const int nv4 = total >> 2;
        store_f4(reinterpret_cast<float4*>(dst), nv4, acc,
                 [&](int f) { return reinterpret_cast<const float4*>(lds)[f]; });
        e0 = nv4 << 2;
    }
    for (int e = e0 + threadIdx.x; e < total; e += blockDim.x) dst[e] = acc ? dst[e] + lds[e] : lds[e];
}

// Reference getHigherMsb (rasterizer_impl.cu:35-50)
inline uint32_t higher_msb(uint32_t n)
{
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

}  // namespace gsr
