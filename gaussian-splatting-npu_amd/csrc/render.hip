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
// Backward: one wave64 per tile, split into four 16-lane groups, one per quadrant, each lane
// owning 4 pixels of its group's quadrant; each group walks only the entries that contributed
// in its quadrant in the forward, back to front (as the reference).  The ten per-(pixel, Gaussian) gradient terms
// are reduced on chip (in-lane over the 4 pixels, a transposed cross-lane reduction over the
// group, the <= 4 quadrant partials added in LDS in a fixed order) and stored once per
// (tile, Gaussian) entry -- no global atomics, bitwise-reproducible sums
// (the reference issues up to ten float atomics per contributing pixel,
// backward.cu:593-635).
#include "gsr_common.h"
#include "gsr_kernels.h"
#if GSR_REF_ALPHA
#define GSR_REF_EXP_QUAL static __device__ __forceinline__
#include "gsr_ref_exp.h"
#endif

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
    // v_rcp_f32 (1 ulp): the test is conservative by the cullK margin, far above that
    const float ia = __builtin_amdgcn_rcpf(a), ic = __builtin_amdgcn_rcpf(c);
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
// alpha >= 1/255.  The record holds the conic and cullK both scaled by log2(e)/2 (the falloff
// form (ka, kb, kc) = -log2(e) (a/2, b, c/2)).  Evaluated once per loaded record by one lane.
__device__ __forceinline__ uint32_t quad_mask(const float4 r0, const float4 k, uint32_t tx, uint32_t ty)
{
    const float K = r0.z;
    if (K > 1.0e37f) return 0xFu;  // degenerate conic: never cull
    if (K < 0.f) return 0u;
    const float dx0 = (float)(tx * GSR_BLOCK_X) - r0.x, dy0 = (float)(ty * GSR_BLOCK_Y) - r0.y;
#if GSR_REF_ALPHA  // (test build: the record holds the plain conic and K)
    const float qa = k.x, qb = k.y, qc = k.z;
#else
    const float qa = -k.x, qb = -0.5f * k.y, qc = -k.z;
#endif
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const float ox = dx0 + (float)((q & 1) * 8), oy = dy0 + (float)((q >> 1) * 8);
        if (box_min_quadform(qa, qb, qc, ox, ox + 7.f, oy, oy + 7.f) <= K) m |= 1u << q;
    }
    return m;
}

// ---- packed-f32 pixel pairs -----------------------------------------------------------------
// gfx950 issues v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 at the cost of one scalar f32 op, so
// the backward evaluates its pixels two at a time: each lane owns two pairs of pixels (x, x + 4)
// in one row of one 8x8 quadrant.
typedef float v2f __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2f fma2(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }

// Gaussian falloff exponent in the log2 domain, shared by forward and backward so that both
// make identical alpha decisions: with (ka, kb, kc) = -log2(e) * (a/2, b, c/2) of the conic,
// p2 = (ka dx + kb dy) dx + kc dy^2 = log2(e) * power (forward.cu:353-354), G = 2^p2.
// preprocess stores (ka, kb, kc) in the render record (.xyz of its second float4).
struct Falloff {
    float ka, kb, kc;
};
__device__ __forceinline__ Falloff falloff(const float4 co) { return {co.x, co.y, co.z}; }
__device__ __forceinline__ float falloff_p2(const Falloff f, float dx, float dy)
{
    const float bq = f.kb * dy;
    const float cq = (f.kc * dy) * dy;
    return __builtin_fmaf(__builtin_fmaf(f.ka, dx, bq), dx, cq);
}
__device__ __forceinline__ v2f falloff_p2(const Falloff f, v2f dx, float dy)
{
    const float bq = f.kb * dy;
    const float cq = (f.kc * dy) * dy;
    return fma2(fma2((v2f)(f.ka), dx, (v2f)(bq)), dx, (v2f)(cq));
}

#if GSR_REF_ALPHA
// TEST BUILD ONLY (GSR_REF_ALPHA): the reference's falloff, forward.cu:353-354 / backward.cu:556-557,
// in its operation order without contraction, on the record's plain conic (co.xyz), and its alpha
// with the shared exp (gsr_ref_exp.h) -- what oracle/gsr_oracle.c computes with shared_exp set.
__device__ __forceinline__ float ref_power(const float4 co, float dx, float dy)
{
#pragma clang fp contract(off)
    return -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
}
#endif

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d, 64));
    return v;
}

// ---- longest-first tile order ---------------------------------------------------------------
// One 1024-thread workgroup sorts the T tiles into 64 work classes, heaviest first, and writes
// the launch order.  Workgroups start roughly in blockIdx order,
// so the long tiles are dispatched first and the tail of the launch is made of short ones
// (list scheduling, LPT; 64 classes schedule within 1 % of an exact sort on the 1080p scene).
// Ranking is atomic-free: each wave matches its 64 lanes' classes with 6 ballots, like the
// radix scatter, so the order is deterministic.  Tiles are independent, so the launch order
// changes timing only, never a result.
constexpr int ORDER_BITS = 6;         // 64 work classes; tiles without work join the last one
constexpr int ORDER_PER_THREAD = 8;   // tiles per thread and pass: 8,192 per pass (one pass at 1080p)

// what a tile's work is: its largest n_contrib (the backward), its range length (the forward), or
// its instance count from the rects' 2-D difference array (the forward; the ranges are written here)
enum OrderMode { ORD_WORK = 0, ORD_RANGES = 1, ORD_DIFF = 2 };

// Inclusive prefix sums along one line of a row-major LDS grid (n cells, `stride` apart), by one wave.
__device__ __forceinline__ void wave_line_scan(int* line, int n, int stride, int lane)
{
    int carry = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        int v = i < n ? line[i * stride] : 0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(v, d, 64);
            if (lane >= d) v += y;
        }
        v += carry;
        if (i < n) line[i * stride] = v;
        carry = __shfl(v, 63, 64);
    }
}

template <int MODE>
__global__ void __launch_bounds__(1024) tile_order_kernel(const ViewBatch<OrderJob> B, int T)
{
    const OrderJob& J = B.v[blockIdx.x];  // one workgroup per view
    const uint2* ranges = J.ranges;
    const uint32_t* work = J.work;
    uint32_t* order = J.order;
    __shared__ uint32_t s_cnt[16][1 << ORDER_BITS];  // per-wave class counts, then per-wave starts
    __shared__ uint32_t s_order[1024 * ORDER_PER_THREAD];  // the pass's order, stored out coalesced
    __shared__ uint32_t s_max;
    // ORD_DIFF: the difference array, turned into per-tile counts in place
    __shared__ int s_d[MODE == ORD_DIFF ? TILE_DIFF_MAX_CELLS : 1];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t gx = J.grid_x, sx = J.grid_x + 1;
    if constexpr (MODE == ORD_DIFF) {
        // counts: 2-D inclusive prefix sums of the difference array (rows, then columns; the last
        // row and column only hold the -1s of rects ending at the grid's edge), then the ranges:
        // the exclusive scan of the counts in tile order, (0, 0) for an empty tile
        // (identifyTileRanges' result, rasterizer_impl.cu:116-138 + the memset at :313)
        const int gy = (int)J.grid_y, cells = (int)(sx * (J.grid_y + 1));
        for (int c = tid; c < cells; c += 1024) s_d[c] = J.diff[c];
        __syncthreads();
        for (int r = wid; r < gy; r += 16) wave_line_scan(s_d + r * sx, (int)gx, 1, lane);
        __syncthreads();
        for (int x = wid; x < (int)gx; x += 16) wave_line_scan(s_d + x, gy, (int)sx, lane);
        __syncthreads();
        uint32_t c8[ORDER_PER_THREAD], sum = 0;
#pragma unroll
        for (int i = 0; i < ORDER_PER_THREAD; i++) {
            const int t = tid * ORDER_PER_THREAD + i;
            c8[i] = t < T ? (uint32_t)s_d[(uint32_t)t / gx * sx + (uint32_t)t % gx] : 0u;
            sum += c8[i];
        }
        uint32_t inc = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= d) inc += y;
        }
        if (lane == 63) s_cnt[0][wid] = inc;
        __syncthreads();
        uint32_t start = inc - sum;
        for (int q = 0; q < wid; q++) start += s_cnt[0][q];
#pragma unroll
        for (int i = 0; i < ORDER_PER_THREAD; i++) {
            const int t = tid * ORDER_PER_THREAD + i;
            if (t < T) J.ranges_out[t] = c8[i] ? make_uint2(start, start + c8[i]) : make_uint2(0u, 0u);
            start += c8[i];
        }
        __syncthreads();  // s_cnt is reused below
    }
    // unconditional (clamped) loads, so that a pass has all of them in flight at once
    auto load_work = [&](int t) -> uint32_t {
        const int tc = min(t, T - 1);
        uint32_t v;
        if constexpr (MODE == ORD_RANGES) {
            const uint2 r = ranges[tc];
            v = r.y - r.x;
        } else if constexpr (MODE == ORD_DIFF) {
            v = (uint32_t)s_d[(uint32_t)tc / gx * sx + (uint32_t)tc % gx];
        } else {
            v = work[tc];
        }
        return t < T ? v : 0u;
    };
    if (tid == 0) s_max = 0;
    // Above 8,192 tiles the passes order each 8K block separately (longest-first inside it).
    for (int t0 = 0; t0 < T; t0 += 1024 * ORDER_PER_THREAD) {
        uint32_t w[ORDER_PER_THREAD];  // wave wid, item i: the 64 consecutive tiles t0 + (i * 16 + wid) * 64 + lane
#pragma unroll
        for (int i = 0; i < ORDER_PER_THREAD; i++) w[i] = load_work(t0 + (i * 16 + wid) * 64 + lane);
        for (int q = tid; q < 16 * (1 << ORDER_BITS); q += 1024) (&s_cnt[0][0])[q] = 0;
        if (t0 == 0) {  // classes are relative to the largest work of ALL tiles
            uint32_t mx = 0;
            for (int t = 1024 * ORDER_PER_THREAD + tid; t < T; t += 1024) mx = max(mx, load_work(t));
#pragma unroll
            for (int i = 0; i < ORDER_PER_THREAD; i++) mx = max(mx, w[i]);
            mx = wave_max_u32(mx);
            __syncthreads();
            if (lane == 0) atomicMax(&s_max, mx);
        }
        __syncthreads();
        const float scale = 63.0f / (float)max(s_max, 1u);
        uint32_t cls[ORDER_PER_THREAD], rank[ORDER_PER_THREAD];
#pragma unroll
        for (int i = 0; i < ORDER_PER_THREAD; i++) {
            const int t = t0 + (i * 16 + wid) * 64 + lane;
            cls[i] = 0u;
            rank[i] = 0u;
            if (t0 + (i * 16 + wid) * 64 >= T) continue;  // the wave's 64 tiles are all past T (uniform)
            const uint32_t c = 63u - min((uint32_t)((float)w[i] * scale), 63u);
            cls[i] = c;
            uint64_t peers = __ballot(t < T);
#pragma unroll
            for (int bit = 0; bit < ORDER_BITS; bit++) {
                const uint64_t bal = __ballot((c >> bit) & 1u);
                peers &= ((c >> bit) & 1u) ? bal : ~bal;
            }
            const uint32_t before = s_cnt[wid][c];  // the wave's running count of class c
            rank[i] = before + (uint32_t)__popcll(peers & lt);
            if (t < T && (peers & lt) == 0ull) s_cnt[wid][c] = before + (uint32_t)__popcll(peers);
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
        // thread (wave q, class c = lane): start of wave q's class-c tiles = class start + the
        // class-c counts of waves < q; class starts = exclusive scan of the class totals
        {
            uint32_t tot = 0, mine = 0;
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const uint32_t n = s_cnt[q][lane];
                mine += q < wid ? n : 0u;
                tot += n;
            }
            uint32_t inc = tot;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)inc, d, 64);
                if (lane >= d) inc += y;
            }
            __syncthreads();
            s_cnt[wid][lane] = inc - tot + mine;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < ORDER_PER_THREAD; i++) {
            const int t = t0 + (i * 16 + wid) * 64 + lane;
            if (t < T) s_order[s_cnt[wid][cls[i]] + rank[i]] = (uint32_t)t;
        }
        __syncthreads();
        const int n = min(T - t0, 1024 * ORDER_PER_THREAD);
        for (int q = tid; q < n; q += 1024) order[t0 + q] = s_order[q];
        __syncthreads();
    }
}

// quadrant bits of batch entry e from the per-wave round masks
__device__ __forceinline__ uint32_t hit_bits(const uint64_t (*s_hitw)[BATCH / 64], int e)
{
    uint32_t h = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) h |= (uint32_t)((s_hitw[w][e >> 6] >> (e & 63)) & 1ull) << w;
    return h;
}

// One launch renders a batch of views (grid.y = view): the views' tiles are dispatched one view
// after the other, so a view's long tiles start while the previous view's short tail still runs --
// one launch tail per batch instead of one per view.
#ifndef GSR_FWD_WAVES
#define GSR_FWD_WAVES 8  // waves per SIMD (VGPR budget)
#endif
#ifndef GSR_FWD_STATS
#define GSR_FWD_STATS 0  // diagnostic build: per (tile, batch, wave) entries walked, view 0 only
#endif
#if GSR_FWD_STATS
__device__ uint32_t* g_fwd_stats;  // [tile][32 batches][4 waves]
extern "C" int gsr_debug_fwd_stats(void* p)
{
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_fwd_stats), &p, sizeof(p));
}
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSR_FWD_WAVES)))
render_fwd_kernel(const ViewBatch<RenderFwdArgs> B)
{
#if GSR_REF_ALPHA  // (test build: every blend operation in the reference's order, forward.cu:353-380)
#pragma clang fp contract(off)
#else
#pragma clang fp contract(fast)
#endif
    const RenderFwdArgs& a = B.v[blockIdx.y];
    const uint32_t tile = a.tile_order[blockIdx.x];
    const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    uint32_t px, py;
    quad_pixel(tx, ty, tid, px, py);
    const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint2 range = a.ranges[tile];
    const int todo = (int)(range.y - range.x);

    // one record of padding in front: the walk's look-ahead past a round's last entry reads
    // s_rec[r * 64 - 1] (unused), which for r = 0 is that pad
    __shared__ float4 s_recp[1 + BATCH * 3];
    float4* const s_rec = s_recp + 1;
    __shared__ uint8_t s_mask[BATCH];
    // per wave and 64-entry round of a batch: bit i = entry (round, i) contributed to some pixel of
    // the wave's quadrant (kept in scalar registers during the round, stored once per round)
    __shared__ uint64_t s_hitw[4][BATCH / 64];

    float live = inside ? 1.0f : 0.0f;  // 0 once the pixel is finished (or outside the image)
    float T = 1.0f;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f, ID = 0.f;
    uint32_t last_contributor = 0;

    // list ids are fetched one batch ahead, so a batch waits for its record gather only
    uint32_t next_id = todo > 0 ? a.point_list[range.x + min(tid, todo - 1)] : 0u;
    int flushed = 0;  // entries [0, flushed) have their contribution bits in a.hit
    for (int base = 0; base < todo; base += BATCH) {
        if (__syncthreads_and(live == 0.0f)) break;
        if (base > 0) {  // the previous batch's contribution bits (every wave has finished it)
            a.hit[range.x + base - BATCH + tid] = (uint8_t)hit_bits(s_hitw, tid);
            flushed = base;
        }
        const int k = base + tid;
        const uint32_t id = next_id;
        next_id = a.point_list[range.x + min(k + BATCH, todo - 1)];
        // unconditional (clamped) record loads: no branch between issue and use
        const float4* r = a.splat + 3 * (size_t)id;
        const float4 r0 = r[0], r1 = r[1], r2 = r[2];
        s_rec[tid] = r0;
        s_rec[BATCH + tid] = r1;
        s_rec[2 * BATCH + tid] = r2;
        const uint32_t m = k < todo ? quad_mask(r0, r1, tx, ty) : 0u;
        s_mask[tid] = (uint8_t)m;
        __syncthreads();
        // each wave clears its own round words after the barrier: every wave has flushed the
        // previous batch's bits (above, before the barrier), and the wave's own stores below
        // follow in program order
        if (lane < BATCH / 64) s_hitw[wid][lane] = 0ull;
        const int n = min(BATCH, todo - base);
#if GSR_FWD_STATS
        uint32_t walked = 0;
#endif
        // Walk the entries whose mask has this wave's quadrant bit, in list order: one ballot
        // per 64 entries, then a scalar bit scan; each record is read one entry ahead of use.
        for (int r = 0; r < BATCH / 64; r++) {
            if (__all(live == 0.0f)) break;
            const int jr = r * 64 + lane;
            uint64_t rem = __ballot(jr < n && ((s_mask[jr] >> wid) & 1));
            if (rem == 0) continue;
            uint64_t hitbits = 0;  // wave-uniform
            // two entries per iteration with ping-pong record registers (no rotation copies).  take():
            // the lowest set bit (s_ff1, -1 once none is left) and its clear (one s_bitset0; with
            // none left it clears bit 63 of a zero mask), as the batch position r * 64 + bit
            auto take = [&]() -> int {
                int jl;
                asm("s_ff1_i32_b64 %0, %1\n\ts_bitset0_b64 %1, %0" : "=&s"(jl), "+s"(rem));
                return r * 64 + jl;  // r * 64 - 1 once none is left (clamped by the caller)
            };
            // Branch-free blend: every test is a compare feeding a select (no exec-mask branch, no
            // scalar mask algebra -- the scalar unit, shared by the CU's four SIMDs, is the busier
            // issue port in this loop).  a = 0 for a finished pixel (live = 0) or power > 0; an
            // entry that would take T below 1e-4 finishes the pixel without blending
            // (forward.cu:356-376); ae = the alpha actually blended (0 or a).
            auto blend = [&](int j, const float4 xy, const float4 co, const float4 col) {
#if GSR_REF_ALPHA
                const float p2 = ref_power(co, xy.x - pfx, xy.y - pfy);  // power (test build)
                const float alpha = fminf(0.99f, co.w * gsr_ref_expf(p2));
#else
                const float p2 = falloff_p2(falloff(co), xy.x - pfx, xy.y - pfy);
                const float alpha = fminf(0.99f, __builtin_amdgcn_exp2f(p2) * co.w);
#endif
                const float a = (p2 > 0.0f ? 0.0f : alpha) * live;
                const bool contrib = a >= 1.0f / 255.0f;
                const float test_T = T * (1 - a);
                const bool stop = (contrib ? test_T : 1.0f) < 0.0001f;
                live = stop ? 0.0f : live;
                const float ae = stop ? 0.0f : (contrib ? a : 0.0f);
                const bool blended = ae > 0.0f;
                {  // hitbits |= (any lane blended) ? bit j : 0 -- as one 64-bit scalar select (the
                   // compiler splits it into two 32-bit ones: one scalar instruction more per entry)
                    uint64_t t;
                    asm("s_cmp_lg_u64 %1, 0\n\ts_cselect_b64 %0, %2, 0"
                        : "=s"(t)
                        : "s"(__ballot(blended)), "s"(1ull << (j & 63))
                        : "scc");
                    hitbits |= t;
                }
#if GSR_REF_ALPHA  // features * alpha * T, left to right (forward.cu:373-375)
                C0 += col.x * ae * T;
                C1 += col.y * ae * T;
                C2 += col.z * ae * T;
                ID += col.w * ae * T;
#else
                const float aT = ae * T;  // 0 leaves the sums unchanged
                C0 += col.x * aT;
                C1 += col.y * aT;
                C2 += col.z * aT;
                ID += col.w * aT;
#endif
                T = blended ? test_T : T;
                last_contributor = blended ? (uint32_t)(base + j + 1) : last_contributor;
            };
            // cnt entries to walk (rem != 0): a counted loop, so take() needs no end test; the
            // look-ahead take() past the last entry returns r * 64 - 1 (a record it never uses).
            // The all-finished exit is tested every second entry (blending into finished pixels
            // is a no-op), at the end of each two-entry turn.
            int left = __popcll(rem);
#if GSR_FWD_STATS
            const int left0 = left;
#endif
            int j = take();
            float4 axy = s_rec[j], aco = s_rec[BATCH + j], acol = s_rec[2 * BATCH + j];
            while (true) {
                const int jb = take();
                const float4 bxy = s_rec[jb], bco = s_rec[BATCH + jb], bcol = s_rec[2 * BATCH + jb];
                blend(j, axy, aco, acol);
                if (--left == 0) break;
                j = take();
                axy = s_rec[j];
                aco = s_rec[BATCH + j];
                acol = s_rec[2 * BATCH + j];
                blend(jb, bxy, bco, bcol);
                if (--left == 0 || __all(live == 0.0f)) break;
            }
            if (lane == 0 && hitbits) s_hitw[wid][r] = hitbits;
#if GSR_FWD_STATS
            walked += (uint32_t)(left0 - left);
#endif
        }
#if GSR_FWD_STATS
        if (blockIdx.y == 0 && lane == 0 && base / BATCH < 32) g_fwd_stats[(tile * 32 + base / BATCH) * 4 + wid] = walked + 1;
#endif
    }

    __shared__ uint32_t s_lc[4];
    const uint32_t wl = wave_max_u32(last_contributor);
    if (lane == 0) s_lc[wid] = wl;
    __syncthreads();
    // the last processed batch's contribution bits (entries past it are never read: the
    // backward stops at the tile's largest n_contrib, all of whose entries were processed)
    if (flushed + tid < todo && tid < BATCH) a.hit[range.x + flushed + tid] = (uint8_t)hit_bits(s_hitw, tid);
    if (tid == 0) a.tile_work[tile] = max(max(s_lc[0], s_lc[1]), max(s_lc[2], s_lc[3]));

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

// ---- transposed wave reduction (CDNA4 cross-lane ops, no LDS) ------------------------------
// The swaps (GSR_SWAP8 below) exchange the two registers in place (both operands are read and
// written).  Through the builtin the compiler copies one operand to a scratch register before each
// swap (a v_mov per exchanged pair); as inline asm on "+v" operands it swaps the values where they
// live.  The s_nop 1 is the gfx950 hazard a VALU write -> v_permlane*_swap read requires (two wait
// states), which the compiler cannot see inside the asm.

// Sums 32 per-lane values over each of four 16-lane groups and returns in r0 / r1 of lane l the
// group totals of v[2 (l >> 2)] / v[2 (l >> 2) + 1].  Recursive halving: each exchange step hands
// half of the live values to the partner lane -- l ^ 32 (v_permlane32_swap), l ^ 16
// (v_permlane16_swap), then DPP row_mirror (l ^ 15) and row_half_mirror (l ^ 7) fused into
// v_add_f32_dpp.  A group, quad_group(l), is the set of lanes those four partners connect: the
// coset of l & 15 under {0, 7, 8, 15}, across the four rows.  66 instructions for 4 x 32 totals,
// against 32 x 4 shuffle+add pairs of per-value butterflies.
__device__ __forceinline__ int quad_group(int lane) { return (lane & 4) ? 3 - (lane & 3) : (lane & 3); }
// Eight swaps back to back behind ONE s_nop 1: every swapped register was written before the block,
// so the two wait states cover them all (one per swap otherwise).
#define GSR_SWAP8(OP, a, b)                                                                              \
    asm("s_nop 1\n\t" OP " %0, %8\n\t" OP " %1, %9\n\t" OP " %2, %10\n\t" OP " %3, %11\n\t" OP           \
        " %4, %12\n\t" OP " %5, %13\n\t" OP " %6, %14\n\t" OP " %7, %15"                                  \
        : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]),      \
          "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]))
__device__ __forceinline__ void group_transpose_reduce32(float (&v)[32], int lane, float& r0, float& r1)
{
    GSR_SWAP8("v_permlane32_swap_b32_e32", (&v[0]), (&v[16]));
    GSR_SWAP8("v_permlane32_swap_b32_e32", (&v[8]), (&v[24]));
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = v[i] + v[i + 16];
    GSR_SWAP8("v_permlane16_swap_b32_e32", (&v[0]), (&v[8]));
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = v[i] + v[i + 8];
    // The last two stages pair lane l with its row mirror (l ^ 15: bit 3 flips) and then its half-row
    // mirror (l ^ 7: bit 2 flips).  Lanes on either side keep different halves, so each output is
    // two v_add_f32_dpp restricted by bank_mask to one side (a 4-lane bank = lane bits 3:2) instead
    // of two selects and an add: lanes with bit 3 clear take v[i] + mirror(v[i]), the others
    // v[i + 4] + mirror(v[i + 4]) (the partner of a clear lane holds its v[i] at the other side).
    // The leading s_nop 1 gives the DPP reads of the registers the adds above wrote their two
    // wait states.
    (void)lane;
    asm("s_nop 1\n\t"
        "v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0x3\n\t"
        "v_add_f32_dpp %0, %4, %4 row_mirror row_mask:0xf bank_mask:0xc\n\t"
        "v_add_f32_dpp %1, %1, %1 row_mirror row_mask:0xf bank_mask:0x3\n\t"
        "v_add_f32_dpp %1, %5, %5 row_mirror row_mask:0xf bank_mask:0xc\n\t"
        "v_add_f32_dpp %2, %2, %2 row_mirror row_mask:0xf bank_mask:0x3\n\t"
        "v_add_f32_dpp %2, %6, %6 row_mirror row_mask:0xf bank_mask:0xc\n\t"
        "v_add_f32_dpp %3, %3, %3 row_mirror row_mask:0xf bank_mask:0x3\n\t"
        "v_add_f32_dpp %3, %7, %7 row_mirror row_mask:0xf bank_mask:0xc"
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])
        : "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]));
    asm("s_nop 1\n\t"
        "v_add_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0x5\n\t"
        "v_add_f32_dpp %0, %2, %2 row_half_mirror row_mask:0xf bank_mask:0xa\n\t"
        "v_add_f32_dpp %1, %1, %1 row_half_mirror row_mask:0xf bank_mask:0x5\n\t"
        "v_add_f32_dpp %1, %3, %3 row_half_mirror row_mask:0xf bank_mask:0xa"
        : "+v"(v[0]), "+v"(v[1])
        : "v"(v[2]), "v"(v[3]));
    r0 = v[0];
    r1 = v[1];
}

// State of two pixels of the backward pass (backward.cu:498-528).  Pixels outside the image carry
// last_contributor = 0, so no list entry contributes to them.
//
// Each pixel's list is replayed back to front, as the reference does: T is rebuilt from final_T
// by the reciprocal of (1 - alpha) (backward.cu:581), and the colour behind entry j enters as ONE
// normalised scalar, Bn_j = accum_rec_j . dL/dpixel (+ the inverse-depth channel), since dL/dpixel
// is constant along the walk: Bn_{j-1} = Bn_j + alpha_j (cd_j - Bn_j), cd_j = c_j . dL/dpixel, a
// convex recurrence (backward.cu:586-600), and
//     dL/dalpha_j = T_j (cd_j - Bn_j) - T_final / (1 - alpha_j) (bg . dL/dpixel)   (:601-612).
// The background term folds into Bn: with Bn' = Bn + T_final (bg . dL) / T_{j+1} (the background
// as the colour behind the last entry, normalised the same way), Bn' obeys the same recurrence
// from Bn' = bg . dL/dpixel behind the last entry, and dL/dalpha_j = T_j (cd_j - Bn'_j) --
// since T_j / T_{j+1} = 1 / (1 - alpha_j) -- one multiply and one register less per pixel.
// Rounds 1-3 walked front to back with B_j = R - sum_{k <= j} alpha_k T_k cd_k (R = the forward's
// out_color . dL): as cheap per entry, but B is a difference of O(1) terms that ends small, so its
// absolute rounding error (~eps |R| per entry) grew to ~5x the reference's relative error on the
// chair fixture (tools/dbg/bwd_accuracy.py: p99.9 record error 2-8e-3 vs 0.7-1.3e-3 for the
// reference's order against float64; this walk: 0.4-1.2e-3).  The walk needs no accumulated
// colour from the forward either (16 B per pixel neither written nor read).
struct BwdPair {
    v2f T, Bn, dp0, dp1, dp2, dinv;  // Bn: the colour behind, the background's included
    uint32_t lc0, lc1;               // last_contributor
};

// A lane's sums over its two pixel pairs for one Gaussian: the colour and invdepth terms per
// pixel, and u = G * dL/dalpha with its dx, dx^2 moments.  The lane's four pixels share one row, so
// the dy-moments need no per-pixel sums: sum u dy = dy sum u, sum u dx dy = dy sum u dx and
// sum u dy^2 = dy^2 sum u (bwd_lane_terms).
struct BwdAcc {
    v2f col0, col1, col2, inv, u, udx, udx2;
};

// Two pixels x one Gaussian, branch-free: a pixel the Gaussian does not contribute to gets
// alpha = G = 0, which leaves its state bitwise unchanged (T * (1 - 0) = T, B - 0 * cd = B)
// and adds exact zeros.  Per-Gaussian constant factors are left to preprocess_bwd (see
// GradField): the record holds sum u (opacity), sum u*dx and sum u*dy (mean2D: (a Sx + b Sy,
// b Sx + c Sy) times -opacity * W/2 resp. H/2) and sum u*dx*dx, u*dx*dy, u*dy*dy (conic, times
// -opacity/2).  FIRST: the sums are assigned, not accumulated (no zero-initialisation).
template <bool HAS_INV, bool FIRST>
__device__ __forceinline__ void bwd_pair(BwdPair& s, v2f pfx, uint32_t pos, const float4 xy, float dy, float bq, float cq,
                                         const Falloff f, const float4 co, const float4 col, BwdAcc& o)
{
    const v2f dx = (v2f)(xy.x) - pfx;
#if GSR_REF_ALPHA  // (test build: power and G = exp(power) as backward.cu:556-568; bq, cq unused)
    (void)bq;
    (void)cq;
    const v2f p2 = {ref_power(co, dx.x, dy), ref_power(co, dx.y, dy)};
    const v2f G = {gsr_ref_expf(p2.x), gsr_ref_expf(p2.y)};
#else
    (void)dy;
    const v2f p2 = fma2(fma2((v2f)(f.ka), dx, (v2f)(bq)), dx, (v2f)(cq));
    const v2f G = {__builtin_amdgcn_exp2f(p2.x), __builtin_amdgcn_exp2f(p2.y)};
#endif
    const v2f al = G * co.w;
    const bool c0 = pos < s.lc0 && !(p2.x > 0.0f) && !(al.x < 1.0f / 255.0f);
    const bool c1 = pos < s.lc1 && !(p2.y > 0.0f) && !(al.y < 1.0f / 255.0f);
    const v2f Gc = {c0 ? G.x : 0.f, c1 ? G.y : 0.f};
    const v2f a = Gc * co.w;  // alpha before the 0.99 clamp (0 where the pixel is not reached)
    const v2f alpha = {fminf(0.99f, a.x), fminf(0.99f, a.y)};
    const v2f one_m = 1.f - alpha;
    // v_rcp_f32 (1 ulp) in place of the IEEE divisions of backward.cu:581,612 (exact for
    // alpha = 0: T stays bitwise unchanged for entries that do not reach the pixel)
    const v2f r_om = {__builtin_amdgcn_rcpf(one_m.x), __builtin_amdgcn_rcpf(one_m.y)};
    s.T = s.T * r_om;  // T in front of this entry
    v2f cd = fma2((v2f)(col.z), s.dp2, fma2((v2f)(col.y), s.dp1, (v2f)(col.x) * s.dp0));
    if constexpr (HAS_INV) cd = fma2((v2f)(col.w), s.dinv, cd);
    const v2f diff = cd - s.Bn;  // (c - accum_rec) . dL/dpixel
    const v2f aT = alpha * s.T;  // dL/dcolour / dL/dpixel (backward.cu:586-590)
    const v2f dL = s.T * diff;
    s.Bn = fma2(alpha, diff, s.Bn);  // the colour behind the entry in front
    const v2f u = Gc * dL;
    const v2f ux = u * dx;
    if constexpr (FIRST) {
        o.col0 = aT * s.dp0;
        o.col1 = aT * s.dp1;
        o.col2 = aT * s.dp2;
        o.inv = HAS_INV ? aT * s.dinv : (v2f)(0.f);
        o.u = u;
        o.udx = ux;
        o.udx2 = ux * dx;
    } else {
        o.col0 = fma2(aT, s.dp0, o.col0);
        o.col1 = fma2(aT, s.dp1, o.col1);
        o.col2 = fma2(aT, s.dp2, o.col2);
        if constexpr (HAS_INV) o.inv = fma2(aT, s.dinv, o.inv);
        o.u += u;
        o.udx += ux;
        o.udx2 = fma2(ux, dx, o.udx2);
    }
}

// x + y of a packed pair as ONE v_add_f32: left to itself the compiler emits v_pk_add_f32 with
// op_sel (both halves computed, two issue slots for one useful sum)
__device__ __forceinline__ float hsum(v2f a)
{
    float r;
    asm("v_add_f32_e32 %0, %1, %2" : "=v"(r) : "v"(a.x), "v"(a.y));
    return r;
}

// The ten per-Gaussian values of one lane (its four pixels) for the transposed reduction.
__device__ __forceinline__ void bwd_lane_terms(const BwdAcc& o, float dy, float* v)
{
    const float su = hsum(o.u), sudx = hsum(o.udx);
    v[GF_OPACITY] = su;
    v[GF_MEAN2D_X] = sudx;
    v[GF_MEAN2D_Y] = dy * su;
    v[GF_CONIC_A] = hsum(o.udx2);
    v[GF_CONIC_B] = dy * sudx;
    v[GF_CONIC_C] = (dy * dy) * su;
    v[GF_COLOR_R] = hsum(o.col0);
    v[GF_COLOR_G] = hsum(o.col1);
    v[GF_COLOR_B] = hsum(o.col2);
    v[GF_INVDEPTH] = hsum(o.inv);
}

// Backward: ONE wave per 16x16 tile, so there are no workgroup barriers in the main loop and no
// cross-wave combine.  Lane group quad_group(lane) owns quadrant (g & 1, g >> 1); lane
// l >> 2 of it the pixels (x, x + 4) and (x + 2, x + 6) of one quadrant row as two packed pairs.
// The list below the tile's largest n_contrib is walked back to front in batches of 64 entries:
// each lane stages the record of its entry if that entry contributed anywhere in the forward, and
// each quadrant's contributing entries are listed in LDS (ballot + mbcnt, list order).  Iteration
// i then evaluates the i-th last entry of every quadrant at once (pixels of different quadrants share no
// state; a group past its list evaluates a staged record at position "never", which adds zeros),
// three iterations per transposed reduction, whose group totals go to a per-wave LDS row of
// partials with one 8-B store per lane; at the end of the batch every contributing entry's lane
// adds its <= 4 quadrant partials (it knows each one's iteration from its place in the quadrant
// lists) and stores its record (10 floats) at its record slot and flags it valid.  (Until round 5
// the groups added their totals into per-entry LDS sums by read-add-write, two phases per
// reduction: 0.79 bank-conflict cycles per LDS instruction at random entries; -1 %.)  Against one
// 64-lane pass per entry over the half-tiles it reaches, this skips the pixel pairs of quadrants
// an entry does not reach (25 % of them) and reduces over 16 lanes: render_bwd -11 %.
// Tiles (independent waves) per workgroup.  Round 2 chose 4: a retiring 4-wave workgroup frees one
// wave slot on each SIMD of its CU -- the footprint of a 256-thread binning-prefix workgroup of the
// next view, which then ran beside this launch when views alternated over two streams (1 -> 2 -> 4
// -> 8 tiles: 2,258 / 2,285 / 2,340 / 2,323 Mpix/s then).  Since the views are batched, the prefix
// runs before the renders and nothing needs that hole: one tile per workgroup (the finest dispatch
// granularity) measured render_bwd 1,910-1,915 -> 1,873-1,883 us per 8 views (round 5, 3 rounds).
#ifndef GSR_BWD_TPW
#define GSR_BWD_TPW 1
#endif
constexpr int BWD_TPW = GSR_BWD_TPW;
// reduction blocks of partial rows per wave: 11 blocks = 33 iterations per pass (5.5 KB per wave)
#ifndef GSR_BWD_PART_BLOCKS
#define GSR_BWD_PART_BLOCKS 11
#endif
constexpr int BWD_PART_BLOCKS = GSR_BWD_PART_BLOCKS;
#ifndef GSR_BWD_PART_STRIDE
#define GSR_BWD_PART_STRIDE 132
#endif
constexpr int BWD_PART_STRIDE = GSR_BWD_PART_STRIDE;  // floats per block of partial rows (>= 4 x 32, even)
static_assert(BWD_PART_STRIDE >= 128 && BWD_PART_STRIDE % 2 == 0, "partial rows: 4 groups x 32 values, 8-B aligned");
#ifndef GSR_BWD_WAVES
#define GSR_BWD_WAVES 4  // waves per SIMD (VGPR budget)
#endif
// (Measured and dropped, DESIGN §10: a reduction group's three entries as ONE basic block, 2 %
// slower; entry jj + 1's staged record read from LDS while entry jj computes, 2 % slower.)

template <bool HAS_INV>
__global__ void __launch_bounds__(64 * BWD_TPW) __attribute__((amdgpu_waves_per_eu(GSR_BWD_WAVES))) render_bwd_kernel(const ViewBatch<RenderBwdArgs> B)
{
#pragma clang fp contract(fast)
    const RenderBwdArgs& a = B.v[blockIdx.y];  // a batch of views: one launch tail per batch
    constexpr int G = 3;  // entries per group and transposed reduction (3 x 10 gradient terms <= 32 values)
    // a pass evaluates <= 32 entries per quadrant (the two-pass split below): they must fit the rows
    static_assert(G * BWD_PART_BLOCKS >= 32, "partial rows: a half batch's 32 entries per quadrant");
    const int wv = BWD_TPW == 1 ? 0 : (int)(threadIdx.x >> 6);
    const int ti = (int)blockIdx.x * BWD_TPW + wv;
    if (ti >= a.T) return;  // waves are independent: no workgroup barrier below
    const uint32_t tile = a.tile_order[ti];
    const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int lane = (int)(threadIdx.x & 63);
    // quadrant group (quadrant (grp & 1, grp >> 1)) and index in it (see group_transpose_reduce32)
    const int grp = quad_group(lane), li = lane >> 2;
    const uint2 range = a.ranges[tile];
    const size_t HW = (size_t)a.H * a.W;
    // pixels p = 0..3 of this lane: row qy, columns qx0 + 2 (p >> 1) + 4 (p & 1); pair h = p >> 1
    const uint32_t qx0 = tx * GSR_BLOCK_X + 8 * (grp & 1) + (li & 1);
    const uint32_t qy = ty * GSR_BLOCK_Y + 8 * (grp >> 1) + (li >> 1);
    const float fx0 = (float)qx0, pfy = (float)qy;
    const v2f pfx0 = {fx0, fx0 + 4.f}, pfx1 = {fx0 + 2.f, fx0 + 6.f};

    // Pixel state: every load issued before the first use (clamped addresses, masked after), so
    // the prologue costs one memory round trip instead of one per pixel.
    float Tf[4], dp0[4], dp1[4], dp2[4], dinv[4];
    uint32_t lc[4];
    bool inside[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const uint32_t px = qx0 + 2 * (p >> 1) + 4 * (p & 1);
        inside[p] = px < (uint32_t)a.W && qy < (uint32_t)a.H;
        const uint32_t pix_id = inside[p] ? (uint32_t)a.W * qy + px : 0u;
        Tf[p] = a.final_Ts[pix_id];
        lc[p] = a.n_contrib[pix_id];
        dp0[p] = a.dL_dpixels[0 * HW + pix_id];
        dp1[p] = a.dL_dpixels[1 * HW + pix_id];
        dp2[p] = a.dL_dpixels[2 * HW + pix_id];
        dinv[p] = HAS_INV ? a.dL_invdepths[pix_id] : 0.f;
    }
    const float bg0 = a.bg[0], bg1 = a.bg[1], bg2 = a.bg[2];
    BwdPair st[2];
    float bgd[4];  // bg . dL/dpixel: the colour behind the last entry (the background, backward.cu:610-612)
#pragma unroll
    for (int p = 0; p < 4; p++) {
        if (!inside[p]) {
            Tf[p] = 0.f;
            lc[p] = 0u;
            dp0[p] = dp1[p] = dp2[p] = dinv[p] = 0.f;
        }
        bgd[p] = bg0 * dp0[p] + bg1 * dp1[p] + bg2 * dp2[p];
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
        BwdPair& s = st[h];
        s.T = {Tf[2 * h], Tf[2 * h + 1]};
        s.Bn = {bgd[2 * h], bgd[2 * h + 1]};
        s.dp0 = {dp0[2 * h], dp0[2 * h + 1]};
        s.dp1 = {dp1[2 * h], dp1[2 * h + 1]};
        s.dp2 = {dp2[2 * h], dp2[2 * h + 1]};
        s.dinv = {dinv[2 * h], dinv[2 * h + 1]};
        s.lc0 = lc[2 * h];
        s.lc1 = lc[2 * h + 1];
    }
    // the tile's largest n_contrib, as render_fwd stored it (the max of lc over the tile's pixels): a
    // scalar load beside the range's, so the first batch's list loads do not wait for the pixel state
    const uint32_t tmax = a.tile_work[tile];

    __shared__ float4 s_recw[BWD_TPW][3][64];
    __shared__ uint8_t s_lqw[BWD_TPW][4][64];
    // The groups' partial totals, one 32-float row per (reduction block, group): block b holds the
    // group's iterations 3b .. 3b + 2 (value jj * GF_NUM + f = term f of iteration 3b + jj).  Every
    // reduction writes its block with ONE conflict-free 8-B store per lane (the 64 lanes cover 512
    // contiguous bytes); each entry's lane sums its <= 4 quadrant partials when the pass ends.
    // (blocks BWD_PART_STRIDE = 132 floats apart, not 128: an entry's lane reads its partial from
    // block b at a lane-dependent b, and with a 128-float stride (0 mod the 64 banks) the up to 33
    // lanes reading one quadrant's partials fell into 3 banks -- 11-way conflicts; 132 spreads them
    // to 2 LDS cycles, the minimum for 64 lanes x 8 B)
    __shared__ __attribute__((aligned(16))) float s_partw[BWD_TPW][BWD_PART_BLOCKS * BWD_PART_STRIDE];
    float4 (&s_rec)[3][64] = s_recw[wv];
    uint8_t (&s_lq)[4][64] = s_lqw[wv];  // per quadrant: the batch entries it evaluates, in list order
    float* s_part = s_partw[wv];  // block b, group g, value k at b * BWD_PART_STRIDE + 32 g + k

    // Only the quadrants in which an entry contributed to some pixel in the forward (render_fwd's
    // a.hit bits: alpha >= 1/255 and the pixel not yet saturated, the tests this loop repeats per
    // pixel) are evaluated; entries that contributed nowhere (and list positions >= tmax) get no
    // record: valid[slot] stays 0 and preprocess_bwd skips them.

    // The list is walked back to front in batches of 64 (the last batch first); list ids, slots
    // and contribution bits are fetched one batch ahead (the batch in front); the records of the
    // batch's contributing entries are all in flight before the first is used
    const int last = (int)tmax - 1;
    const int pfirst = tmax > 0 ? (last & ~63) : -64;
    uint32_t next_id = 0, next_slot = 0, next_hit = 0;
    if (tmax > 0) {
        next_id = a.point_list[range.x + min(pfirst + lane, last)];
        if (a.slot) next_slot = a.slot[range.x + min(pfirst + lane, last)];
        next_hit = a.hit[range.x + min(pfirst + lane, last)];
    }
    for (int p0 = pfirst; p0 >= 0; p0 -= 64) {
        const int pos_l = p0 + lane;  // this lane's entry; lane order = list order
        const uint32_t id = next_id, hit = next_hit;
        uint32_t myslot = next_slot;  // (without a.slot: from the record's packed rect, below)
        const int pn = max(p0 - 64, 0) + lane;  // (the first batch re-reads itself: never used)
        next_id = a.point_list[range.x + pn];
        if (a.slot) next_slot = a.slot[range.x + pn];
        next_hit = a.hit[range.x + pn];
        const uint32_t m = pos_l < (int)tmax ? hit : 0u;
        // only entries that contributed somewhere in the forward are read (43 % of the entries
        // below tmax contributed nowhere: their 48-B record gathers are skipped)
        uint32_t es = 0;  // the Gaussian's first record slot (its record mask bit, the slot at the store)
        if (m != 0) {
            const float4* r = a.splat + 3 * (size_t)id;
            const float4 r0 = r[0], r1 = r[1], r2 = r[2];
            if (GSR_REC_MASK || GSR_SLOT_LOCAL) es = a.emit_start[id];
            if (!a.slot) myslot = rect_local(__float_as_uint(r0.w), tx, ty);
            s_rec[0][lane] = r0;
            s_rec[1][lane] = r1;
            s_rec[2][lane] = r2;
        }
        if (__ballot(m != 0) == 0) continue;  // nothing staged, nothing to store
        // A batch whose busiest quadrant has more entries than the partial rows hold runs as two
        // passes, its back half (lanes 32..63: the later entries) first; each half has <= 32
        // entries per quadrant.  An entry is evaluated and stored in one pass.
        int big = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) big |= __popcll(__ballot((m >> q) & 1u)) > G * BWD_PART_BLOCKS;
        for (int hp = big ? 1 : 0; hp >= 0; hp--) {
            const uint32_t mm = (big && (lane >> 5) != hp) ? 0u : m;
            const uint64_t any = __ballot(mm != 0);
            if (any == 0) continue;
            int cq[4];
            uint32_t bef = 0;  // this entry's index in each quadrant's list (a byte per quadrant)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const bool in = (mm >> q) & 1u;
                const uint64_t bq = __ballot(in);
                const int before =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(bq >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bq, 0));
                if (in) s_lq[q][before] = (uint8_t)lane;
                bef |= (uint32_t)before << (8 * q);
                cq[q] = __popcll(bq);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

            // Each quadrant group walks its own entries back to front (pixels of different quadrants
            // share no state), iteration i of all four groups at once; a group past its count
            // evaluates a staged record at position "never" (alpha = 0: state unchanged, zero terms).
            const int fv = (int)__builtin_ctzll(any);
            const int mycnt = grp == 0 ? cq[0] : grp == 1 ? cq[1] : grp == 2 ? cq[2] : cq[3];
            const int niter = max(max(cq[0], cq[1]), max(cq[2], cq[3]));
            for (int i0 = 0, blk = 0; i0 < niter; i0 += G, blk++) {
                int ej[G];
                bool act[G];
#pragma unroll
                for (int jj = 0; jj < G; jj++) {
                    act[jj] = i0 + jj < mycnt;
                    ej[jj] = act[jj] ? (int)s_lq[grp][mycnt - 1 - (i0 + jj)] : fv;
                }
                float v[32];
#pragma unroll
                for (int jj = 0; jj < G; jj++) {
                    // a wave-uniform branch per entry (a block per entry): the iterations past niter
                    // evaluate nothing
                    if (i0 + jj < niter) {
                        const float4 xy = s_rec[0][ej[jj]], co = s_rec[1][ej[jj]], col = s_rec[2][ej[jj]];
                        const uint32_t pos = act[jj] ? (uint32_t)(p0 + ej[jj]) : 0xFFFFFFFFu;
                        const Falloff f = falloff(co);
                        // the falloff's dy terms, shared by the lane's two pairs (one row)
                        const float dy = xy.y - pfy;
                        const float bq = f.kb * dy, cq = (f.kc * dy) * dy;
                        BwdAcc o;
                        bwd_pair<HAS_INV, true>(st[0], pfx0, pos, xy, dy, bq, cq, f, co, col, o);
                        bwd_pair<HAS_INV, false>(st[1], pfx1, pos, xy, dy, bq, cq, f, co, col, o);
                        bwd_lane_terms(o, dy, &v[jj * GF_NUM]);
                    } else {
#pragma unroll
                        for (int q = 0; q < GF_NUM; q++) v[jj * GF_NUM + q] = 0.f;
                    }
                }
#pragma unroll
                for (int q = G * GF_NUM; q < 32; q++) v[q] = 0.f;
                float r0, r1;
                group_transpose_reduce32(v, lane, r0, r1);
                // lane li of a group holds the group totals of values 2 li and 2 li + 1
                *reinterpret_cast<float2*>(&s_part[blk * BWD_PART_STRIDE + 32 * grp + 2 * li]) = make_float2(r0, r1);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // one gradient record per contributing entry, stored by its own lane: its quadrant partials
            // summed as (q0 + q2) + (q1 + q3), a fixed order (bitwise reproducible)
            if (mm != 0) {
                float t0[GF_NUM], t1[GF_NUM];
#pragma unroll
                for (int f = 0; f < GF_NUM; f++) t0[f] = t1[f] = 0.f;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if ((mm >> q) & 1u) {
                        const int i = cq[q] - 1 - (int)((bef >> (8 * q)) & 0xFFu);  // its iteration
                        const int b = i / G, jj = i - G * b;
                        const float2* src =
                            reinterpret_cast<const float2*>(&s_part[b * BWD_PART_STRIDE + 32 * q + jj * GF_NUM]);
#pragma unroll
                        for (int h = 0; h < GF_NUM / 2; h++) {
                            const float2 pv = src[h];
                            if (q & 1) {
                                t1[2 * h] += pv.x;
                                t1[2 * h + 1] += pv.y;
                            } else {
                                t0[2 * h] += pv.x;
                                t0[2 * h + 1] += pv.y;
                            }
                        }
                    }
                }
                const uint32_t slot = GSR_SLOT_LOCAL ? es + myslot : myslot;  // (BIN_SLOT: the index in the rect)
                float* rec = a.grad_inst + (size_t)slot * GRAD_REC;
                float t[GF_NUM];
#pragma unroll
                for (int f = 0; f < GF_NUM; f++) t[f] = t0[f] + t1[f];
                if constexpr (GRAD_REC % 4 == 0) {  // 16-B aligned records
                    reinterpret_cast<float4*>(rec)[0] = make_float4(t[0], t[1], t[2], t[3]);
                    reinterpret_cast<float4*>(rec)[1] = make_float4(t[4], t[5], t[6], t[7]);
                    reinterpret_cast<float2*>(rec)[4] = make_float2(t[8], t[9]);
                } else {  // packed 40-B records: 8-B aligned
#pragma unroll
                    for (int h = 0; h < GF_NUM / 2; h++) reinterpret_cast<float2*>(rec)[h] = make_float2(t[2 * h], t[2 * h + 1]);
                }
                // flagged in the Gaussian's own mask when it is one of its first 32 slots (preprocess_bwd
                // then finds the records without a dependent load of the valid words), else in the valid
                // words: one atomic per record either way
                const uint32_t local = slot - es;
                if (GSR_REC_MASK && local < 32u) atomicOr(&a.rec_mask[id], 1u << local);
                else atomicOr(&a.valid[slot >> 5], 1u << (slot & 31u));
            }
            __builtin_amdgcn_wave_barrier();  // s_rec / s_lq / s_part reuse in the next pass
        }
    }
}

hipError_t launch_tile_order_batch(const OrderJob* jobs, int V, int T, hipStream_t s)
{
    if (T <= 0) return hipSuccess;
    for (int v0 = 0; v0 < V; v0 += VIEW_BATCH) {
        const int nv = min(VIEW_BATCH, V - v0);
        ViewBatch<OrderJob> B;
        B.n = nv;
        for (int v = 0; v < nv; v++) B.v[v] = jobs[v0 + v];
        if (B.v[0].diff) {
            for (int v = 0; v < nv; v++)
                if (!B.v[v].diff || !use_tile_diff(B.v[v].grid_x, B.v[v].grid_y) || B.v[v].grid_x * B.v[v].grid_y != (uint32_t)T)
                    return hipErrorInvalidValue;
            hipLaunchKernelGGL(tile_order_kernel<ORD_DIFF>, dim3((unsigned)nv), dim3(1024), 0, s, B, T);
        } else if (B.v[0].ranges) {
            hipLaunchKernelGGL(tile_order_kernel<ORD_RANGES>, dim3((unsigned)nv), dim3(1024), 0, s, B, T);
        } else {
            hipLaunchKernelGGL(tile_order_kernel<ORD_WORK>, dim3((unsigned)nv), dim3(1024), 0, s, B, T);
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_tile_order(const uint2* ranges, const uint32_t* work, int T, uint32_t* order, hipStream_t s)
{
    const OrderJob j = {ranges, work, order};
    return launch_tile_order_batch(&j, 1, T, s);
}

hipError_t launch_render_fwd_batch(const RenderFwdArgs* a, int V, int T, hipStream_t s)
{
    if (T <= 0) return hipSuccess;
    for (int v0 = 0; v0 < V; v0 += VIEW_BATCH) {
        ViewBatch<RenderFwdArgs> B;
        B.n = min(VIEW_BATCH, V - v0);
        for (int v = 0; v < B.n; v++) B.v[v] = a[v0 + v];
        hipLaunchKernelGGL(render_fwd_kernel, dim3((unsigned)T, (unsigned)B.n), dim3(256), 0, s, B);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_render_fwd(const RenderFwdArgs& a, int T, hipStream_t s) { return launch_render_fwd_batch(&a, 1, T, s); }

hipError_t launch_render_bwd_batch(const RenderBwdArgs* a, int V, int T, hipStream_t s)
{
    if (T <= 0) return hipSuccess;
    for (int v0 = 0; v0 < V; v0 += VIEW_BATCH) {
        ViewBatch<RenderBwdArgs> B;
        B.n = min(VIEW_BATCH, V - v0);
        bool inv = false;
        for (int v = 0; v < B.n; v++) {
            B.v[v] = a[v0 + v];
            if (B.v[v].T != T) return hipErrorInvalidValue;
            inv = inv || B.v[v].dL_invdepths != nullptr;
        }
        for (int v = 0; v < B.n; v++)  // one kernel variant per launch: all views with or without invdepth
            if ((B.v[v].dL_invdepths != nullptr) != inv) return hipErrorInvalidValue;
        const dim3 grid((unsigned)((T + BWD_TPW - 1) / BWD_TPW), (unsigned)B.n), block(64 * BWD_TPW);
        if (inv) hipLaunchKernelGGL(render_bwd_kernel<true>, grid, block, 0, s, B);
        else hipLaunchKernelGGL(render_bwd_kernel<false>, grid, block, 0, s, B);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_render_bwd(const RenderBwdArgs& a, int T, hipStream_t s) { return launch_render_bwd_batch(&a, 1, T, s); }

}  // namespace gsr
