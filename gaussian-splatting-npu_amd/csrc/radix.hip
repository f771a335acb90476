// radix.hip -- stable LSD radix sort for gfx950 (replaces the reference's
// cub::DeviceRadixSort::SortPairs, rasterizer_impl.cu:303-311), and the depth-first
// binning built on it.
//
// Binning scheme (same result as the reference's 64-bit tile|depth key sort):
//   1. sort the P Gaussians by depth bits (4 x 8-bit passes; ties keep index order;
//      culled Gaussians carry key 0xFFFFFFFF and land last);
//   2. the (tile, Gaussian) instances in that depth order (y-major, then x, inside each
//      Gaussian's rect, exactly like duplicateWithKeys, rasterizer_impl.cu:98-109) are
//      stably sorted by tile id alone: ceil(bit/8) passes over bit = msb(T) bits (2 at 1080p)
//      instead of the reference's ceil((32+bit)/8) passes over 12-byte pairs; the first pass
//      generates the instances itself from the depth-ordered rects (no emission array).
// Because both sorts are stable, every tile's list comes out ordered by (depth bits,
// Gaussian index) -- the reference's order -- and the sorted key array
// (tile << 32 | depth bits) is bit-identical to the reference's.
//
// One pass = three kernels, no inter-workgroup waiting: (1) every 2048-element chunk counts
// its digits (digit-major count matrix); (2) one workgroup per digit scans that digit's row
// over the chunks; (3) every chunk ranks its elements stably per digit (wave-level ballot
// match + per-wave running counters in LDS), adds the digit's offset (exclusive scan of the
// 2^bits digit totals, redone in LDS by each chunk) and its row prefix, and scatters through
// LDS so that global writes are contiguous runs per digit.  Digit widths are balanced over
// the passes (the tile sort at 1080p: 13 bits = 7 + 6).  The payload is one u32 (the
// element's input index in pass 1).
#include "gsr_common.h"
#include "gsr_kernels.h"

#include <type_traits>

namespace gsr {

constexpr int RS_THREADS = 256;
constexpr int RS_THREADS_WIDE = 512;            // 9-bit passes: 4,096-key chunks
constexpr int RS_ITEMS = 8;                     // elements per thread, long sorts (the tile sort; 16: -20 % slower)
constexpr int RS_ITEMS_SHORT = 8;               // short sorts (the depth sort; 4 measures the same)
constexpr int RS_SHORT_MAX = 1 << 21;           // n up to which a sort counts as short
constexpr int RS_MAXBINS = 256;
constexpr int RS_SCRATCH_BINS = 512;            // count-matrix rows reserved per sort (9-bit depth digits)
// GSR_DEPTH_GSUM: the three-pass depth sort launches no column scan.  Each count workgroup also adds
// its digit counts into its chunk group's row (GS_CHUNKS chunks per group, atomic adds of integers:
// exact in any order), and each scatter workgroup derives its own digit offsets from the group rows
// and the chunk rows of its group in its prologue (<= 31 loads per digit at P = 1M) -- 3 launches per
// depth sort fewer (the single view's train.py path runs its depth sort alone on the GPU: each launch
// is latency, ~7 us).  The pass-3 key range is reduced by workgroup 0 of the pass-2 count kernel.
#ifndef GSR_DEPTH_GSUM
#define GSR_DEPTH_GSUM 1
#endif
constexpr int GS_CHUNKS = 16;

// Kernel-name tags: which sort a radix pass belongs to (the depth sort, the tile sort's later
// passes, distCUDA2's cell sort) -- the kernels are identical, the names let a profile (rocprofv3
// --pmc, tools/pmc_summary.py) attribute every dispatch to its sort.
struct DepthSort;
struct TileSort;
struct CellSort;

__device__ __forceinline__ uint32_t digit_of(uint32_t k, int shift, uint32_t mask) { return (k >> shift) & mask; }

// The count matrix of a pass: chunk-major, counts[c * nb + d] (cmaj: each chunk's counts are one
// contiguous write of the count kernel and one contiguous read of the scatter kernel, and the scan
// over the chunks reads 16 digits = 64 B per chunk row -- for passes of at most CS_CHUNKS chunks, which
// one LDS block of radix_colscan_kernel scans: the depth sort), or digit-major counts[d * nchunks + c]
// (one row-scan workgroup per digit: the tile sort's thousands of chunks).
#ifndef GSR_COLSCAN
#define GSR_COLSCAN 1
#endif
__device__ __forceinline__ size_t cm_index(uint32_t d, uint32_t c, uint32_t nb, uint32_t nchunks, bool cmaj)
{
    return cmaj ? (size_t)c * nb + d : (size_t)d * nchunks + c;
}

// XCD-aware chunk order of the scatter kernels: workgroups are dealt round-robin over the 8 XCDs
// (blocks b and b + 8 share one, MI355X_MICROARCH.md §Workgroup dispatch), so with grid.x a multiple
// of 8 (scatter_grid) the chunks [x q, (x + 1) q) of block class x = b % 8 run on one XCD, in order.
// A digit's output runs from consecutive chunks are adjacent in memory: their partial cache lines
// then meet in one L2 instead of being written back from several.  A bijection on [0, grid.x).
#ifndef GSR_XCD_CHUNKS
#define GSR_XCD_CHUNKS 1
#endif
__device__ __forceinline__ uint32_t xcd_chunk(uint32_t b, uint32_t gx)
{
    if (!GSR_XCD_CHUNKS || (gx & 7u)) return b;
    return (b & 7u) * (gx >> 3) + (b >> 3);
}
static inline unsigned scatter_grid(int maxc) { return GSR_XCD_CHUNKS ? (unsigned)((maxc + 7) & ~7) : (unsigned)maxc; }

// The depth sort in three 9-bit passes: passes 1 and 2 take key bits [0, 9) and [9, 18); pass 3
// takes bits [18, 32) RELATIVE to the smallest key that is not 0xFFFFFFFF (culled):
// digit = (k >> 18) - (min >> 18), and 511 for 0xFFFFFFFF.  That is monotone in k, so the three passes
// sort exactly whenever the keys other than 0xFFFFFFFF span at most 511 values of k >> 18 (visible
// depths within a factor of ~2^16: 0.2 ... 13,000).  Pass 1 gathers the range (per-chunk min / max,
// reduced by an extra workgroup of its scan into RangeWord).  A wider range is reported to the host
// (SortJob::host_wide, a pinned word it reads with num_rendered): that call's depth sort then runs
// again in four 8-bit passes (radix_sort_batch four_pass; capi.hip depth_sort_rerun_wide) -- per call,
// no state is kept.
// mode: DIG_RAW (k >> shift) & mask; DIG_REL (the relative digit above when the range fits, else raw).
enum DigitMode { DIG_RAW = 0, DIG_REL = 1 };
struct RangeWord { uint32_t base, fits; };  // min >> rel_shift of the keys other than 0xFFFFFFFF; range fits
struct Digit {
    int shift;
    uint32_t mask;
    bool rel;
    uint32_t base;
    __device__ __forceinline__ uint32_t operator()(uint32_t k) const
    {
        return rel ? (k == 0xFFFFFFFFu ? mask : (k >> shift) - base) : (k >> shift) & mask;
    }
};
// (mode, range) -> the digit function of a pass
__device__ __forceinline__ Digit make_digit(int shift, int nbits, int mode, const RangeWord* range)
{
    Digit d{shift, (1u << nbits) - 1u, false, 0u};
    if (mode == DIG_REL && __builtin_amdgcn_readfirstlane(range->fits)) {
        d.rel = true;
        d.base = __builtin_amdgcn_readfirstlane(range->base);
    }
    return d;
}

// (1) counts[cm_index(d, c)] = number of elements of chunk c with digit d (view blockIdx.y).
struct CountJob {
    const uint32_t* keys;
    int n, nchunks;
    uint32_t* counts;
    // keys == null: the key is pairs_hi[i].y >> hi_shift (the tile sort's second digit carried in
    // the top bits of the id word, see TileSortJob)
    const uint2* pairs_hi;
    int hi_shift;
    const uint32_t* hi_words;  // (instead of pairs_hi) the 4-B words holding the key in their high bits
    int mode;                  // DigitMode
    const RangeWord* range;    // (DIG_REL)
    uint32_t* cmin;            // non-null: per-chunk min / max of the keys other than 0xFFFFFFFF
    uint32_t* cmax;
    bool cmaj;                 // chunk-major count matrix (cm_index)
    // GSR_DEPTH_GSUM: non-null: each chunk's digit counts are also added into
    // gsum[(chunk / GS_CHUNKS) * nb + d] (zero on entry)
    uint32_t* gsum = nullptr;
    // non-null: workgroup 0 reduces the per-chunk key min / max of an earlier pass (rcmin / rcmax,
    // rnchunks chunks) into *range_out (the relative pass's RangeWord; reduce_range)
    RangeWord* range_out = nullptr;
    const uint32_t* rcmin = nullptr;
    const uint32_t* rcmax = nullptr;
    int rnchunks = 0, rel_shift = 0, rel_bits = 0;
    uint32_t* host_wide = nullptr;
};
// The keys' range from per-chunk min / max (nchunks of them) -> *out (base, fits) for a relative pass
// on bits [rel_shift, rel_shift + rel_bits); a range that does not fit is flagged in *host_wide.  Every
// thread of the workgroup (NT threads) calls it.
template <int NT>
__device__ void reduce_range_nt(const uint32_t* cmin, const uint32_t* cmax, int nchunks, RangeWord* out, int rel_shift,
                                int rel_bits, uint32_t* host_wide)
{
    constexpr int NW = NT / 64;
    __shared__ uint32_t s_rr[2][NW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
    for (int c = tid; c < nchunks; c += NT) {
        mn = min(mn, cmin[c]);
        mx = max(mx, cmax[c]);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, off, 64));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
    }
    if (lane == 0) {
        s_rr[0][w] = mn;
        s_rr[1][w] = mx;
    }
    __syncthreads();
    if (tid == 0) {
        for (int q = 1; q < NW; q++) {
            mn = min(mn, s_rr[0][q]);
            mx = max(mx, s_rr[1][q]);
        }
        RangeWord r;
        if (mn > mx) {  // nothing but 0xFFFFFFFF
            r.base = 0u;
            r.fits = 1u;
        } else {
            r.base = mn >> rel_shift;
            // the largest relative digit stays below 2^rel_bits - 1, the digit of 0xFFFFFFFF
            r.fits = ((mx >> rel_shift) - r.base) <= (1u << rel_bits) - 2u ? 1u : 0u;
        }
        *out = r;
        if (!r.fits && host_wide) __hip_atomic_store(host_wide, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
template <int ITEMS, typename KIND, int MAXB, int NT = RS_THREADS>
__global__ void __launch_bounds__(NT) radix_count_kernel(const ViewBatch<CountJob> B, int shift, int nbits)
{
    const CountJob& J = B.v[blockIdx.y];
    if ((int)blockIdx.x >= J.nchunks) return;  // past this view's chunks (uniform)
    const Digit dig = make_digit(shift, nbits, J.mode, J.range);
    const uint32_t* keys = J.keys;
    const int n = J.n;
    constexpr int NW = NT / 64;
    __shared__ uint32_t h[NW][MAXB];
    __shared__ uint32_t s_mm[2][NW];
    const int tid = threadIdx.x, w = tid >> 6;
    const uint32_t nb = 1u << nbits;
    {
    const uint32_t chunk = blockIdx.x;
    for (int q = 0; q < NW; q++)
        for (int d = tid; d < MAXB; d += NT) h[q][d] = 0;
    __syncthreads();
    const size_t base = (size_t)chunk * (NT * ITEMS);
    uint32_t k[ITEMS];
    // the range of the keys other than 0xFFFFFFFF (the depth sort's first pass; `full`: every k[i]
    // is a key of this chunk, else the ones at an index < n)
    auto chunk_range = [&](bool full) {
        if (!J.cmin) return;
        uint32_t mn = 0xFFFFFFFFu, mx = 0u;
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const bool in = full || base + (size_t)i * NT + tid < (size_t)n;
            if (in && k[i] != 0xFFFFFFFFu) {
                mn = min(mn, k[i]);
                mx = max(mx, k[i]);
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            mn = min(mn, (uint32_t)__shfl_xor((int)mn, off, 64));
            mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
        }
        if ((tid & 63) == 0) {
            s_mm[0][w] = mn;
            s_mm[1][w] = mx;
        }
    };
    if (!keys) {  // keys in the pairs' high bits (8-B loads; the slot word rides along unused)
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const size_t e = min(base + (size_t)i * NT + tid, (size_t)n - 1);
            k[i] = (J.hi_words ? J.hi_words[e] : J.pairs_hi[e].y) >> J.hi_shift;
        }
#pragma unroll
        for (int i = 0; i < ITEMS; i++)
            if (base + (size_t)i * NT + tid < (size_t)n) atomicAdd(&h[w][dig(k[i])], 1u);
    } else if (base + NT * ITEMS <= (size_t)n && ((uintptr_t)keys & 15) == 0 && ITEMS % 4 == 0) {
        // full chunk: 16-byte loads (a histogram does not care which thread counts which key)
        const uint4* k4 = reinterpret_cast<const uint4*>(keys + base);
#pragma unroll
        for (int j = 0; j < ITEMS / 4; j++) {
            const uint4 q = k4[j * NT + tid];
            k[4 * j] = q.x; k[4 * j + 1] = q.y; k[4 * j + 2] = q.z; k[4 * j + 3] = q.w;
        }
        chunk_range(true);
        // a wave whose 64 keys share one digit (the depth keys' top byte, mostly) adds once: 64
        // same-address LDS atomics would serialise
        const int lane = tid & 63;
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t d = dig(k[i]);
            const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
            if (__all(d == d0)) {
                if (lane == 0) atomicAdd(&h[w][d0], 64u);
            } else {
                atomicAdd(&h[w][d], 1u);
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < ITEMS; i++) k[i] = keys[min(base + (size_t)i * NT + tid, (size_t)n - 1)];
        chunk_range(false);
#pragma unroll
        for (int i = 0; i < ITEMS; i++)
            if (base + (size_t)i * NT + tid < (size_t)n) atomicAdd(&h[w][dig(k[i])], 1u);
    }
    __syncthreads();
    for (uint32_t d = tid; d < nb; d += NT) {
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < NW; q++) c += h[q][d];
        J.counts[cm_index(d, chunk, nb, J.nchunks, J.cmaj)] = c;
        if (J.gsum && c) atomicAdd(&J.gsum[(size_t)(chunk / GS_CHUNKS) * nb + d], c);
    }
    if (J.range_out && chunk == 0) reduce_range_nt<NT>(J.rcmin, J.rcmax, J.rnchunks, J.range_out, J.rel_shift, J.rel_bits,
                                                       J.host_wide);
    if (J.cmin && tid == 0) {
        uint32_t mn = s_mm[0][0], mx = s_mm[1][0];
        for (int q = 1; q < NW; q++) {
            mn = min(mn, s_mm[0][q]);
            mx = max(mx, s_mm[1][q]);
        }
        J.cmin[chunk] = mn;
        J.cmax[chunk] = mx;
    }
    }
}

// (2) one workgroup per digit: exclusive scan of counts[d, 0..nchunks) in place; the row total
// goes to totals[d].
struct RowJob {
    uint32_t* counts;
    int nchunks;
    uint32_t* totals;
    uint32_t* host_wide;       // (range_out) pinned host word: set to 1 when the range does not fit
    // non-null (the depth sort's first pass): workgroup `nbins` (one past the digit rows) reduces the
    // per-chunk min / max into *range_out for a relative pass on bits [rel_shift, rel_shift + rel_bits)
    const uint32_t* cmin;
    const uint32_t* cmax;
    RangeWord* range_out;
    int nbins, rel_shift, rel_bits;
};
// the extra workgroup of a row scan: the keys' range from the per-chunk min / max (RowJob)
__device__ void reduce_range(const RowJob& J)
{
    __shared__ uint32_t s_mm[2][4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
    for (int c = tid; c < J.nchunks; c += RS_THREADS) {
        mn = min(mn, J.cmin[c]);
        mx = max(mx, J.cmax[c]);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, off, 64));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
    }
    if (lane == 0) {
        s_mm[0][w] = mn;
        s_mm[1][w] = mx;
    }
    __syncthreads();
    if (tid == 0) {
        mn = min(min(s_mm[0][0], s_mm[0][1]), min(s_mm[0][2], s_mm[0][3]));
        mx = max(max(s_mm[1][0], s_mm[1][1]), max(s_mm[1][2], s_mm[1][3]));
        RangeWord r;
        if (mn > mx) {  // nothing but 0xFFFFFFFF
            r.base = 0u;
            r.fits = 1u;
        } else {
            r.base = mn >> J.rel_shift;
            // the largest relative digit stays below 2^rel_bits - 1, the digit of 0xFFFFFFFF
            r.fits = ((mx >> J.rel_shift) - r.base) <= (1u << J.rel_bits) - 2u ? 1u : 0u;
        }
        *J.range_out = r;
        if (!r.fits && J.host_wide) __hip_atomic_store(J.host_wide, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
template <typename KIND>
__global__ void __launch_bounds__(RS_THREADS) radix_rowscan_kernel(const ViewBatch<RowJob> B)
{
    const RowJob& J = B.v[blockIdx.y];
    if (J.cmin && (int)blockIdx.x == J.nbins) {
        reduce_range(J);
        return;
    }
    uint32_t* counts = J.counts;
    const int nchunks = J.nchunks;
    uint32_t* totals = J.totals;
    __shared__ uint32_t s_wave[4];
    __shared__ uint32_t s_carry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t* row = counts + (size_t)blockIdx.x * nchunks;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (int c0 = 0; c0 < nchunks; c0 += RS_THREADS) {
        const int c = c0 + tid;
        const uint32_t v = c < nchunks ? row[c] : 0u;
        uint32_t x = v;  // inclusive wave scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) s_wave[w] = x;
        __syncthreads();
        uint32_t wpre = s_carry;
        for (int q = 0; q < w; q++) wpre += s_wave[q];
        if (c < nchunks) row[c] = wpre + x - v;
        __syncthreads();
        if (tid == RS_THREADS - 1) s_carry = wpre + x;
        __syncthreads();
    }
    if (tid == 0) totals[blockIdx.x] = s_carry;
}

// (2') the same for rows of up to RS_ROW_LDS chunks (every sort at <= 4K resolution): the row is
// staged in LDS with all its loads in flight at once, each thread scans a contiguous segment
// serially, and one block-wide scan of the segment sums joins them -- one global round trip and
// two barriers instead of three barriers per 256 chunks.
constexpr int RS_ROW_LDS = 12288;
template <typename KIND>
__global__ void __launch_bounds__(RS_THREADS) radix_rowscan_lds_kernel(const ViewBatch<RowJob> RB)
{
    const RowJob& J = RB.v[blockIdx.y];
    if (J.cmin && (int)blockIdx.x == J.nbins) {
        reduce_range(J);
        return;
    }
    uint32_t* counts = J.counts;
    const int nchunks = J.nchunks;
    uint32_t* totals = J.totals;
    __shared__ uint32_t s_row[RS_ROW_LDS];
    __shared__ uint32_t s_wave[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t* row = counts + (size_t)blockIdx.x * nchunks;
    constexpr int B = 8;
    for (int c0 = 0; c0 < nchunks; c0 += RS_THREADS * B) {
        uint32_t v[B];
#pragma unroll
        for (int i = 0; i < B; i++) {
            const int c = c0 + i * RS_THREADS + tid;
            v[i] = c < nchunks ? row[c] : 0u;
        }
#pragma unroll
        for (int i = 0; i < B; i++) {
            const int c = c0 + i * RS_THREADS + tid;
            if (c < nchunks) s_row[c] = v[i];
        }
    }
    __syncthreads();
    const int seg = (nchunks + RS_THREADS - 1) / RS_THREADS;
    const int j0 = min(tid * seg, nchunks), j1 = min(j0 + seg, nchunks);
    uint32_t sum = 0;
    for (int j = j0; j < j1; j++) sum += s_row[j];
    uint32_t x = sum;  // inclusive wave scan of the segment sums
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) s_wave[w] = x;
    __syncthreads();
    uint32_t run = x - sum;
    for (int q = 0; q < w; q++) run += s_wave[q];
    if (tid == RS_THREADS - 1) totals[blockIdx.x] = run + sum;
    for (int j = j0; j < j1; j++) {
        const uint32_t c = s_row[j];
        s_row[j] = run;
        run += c;
    }
    __syncthreads();
    for (int c = tid; c < nchunks; c += RS_THREADS) row[c] = s_row[c];
}

// (2') GSR_COLSCAN: the exclusive scan over the chunks of each digit's counts, on the chunk-major
// matrix: workgroup g takes digits [16 g, 16 g + 16); thread (dl = tid >> 4, sg = tid & 15) scans a
// contiguous segment of chunks of digit 16 g + dl; blocks of CS_CHUNKS chunks are staged in LDS with
// every load in flight (16 digits = 64 contiguous bytes per chunk row), each digit's running total
// carried from block to block.  Workgroup ceil(nbins / 16) (the depth sort's first pass) reduces the
// keys' range instead.
constexpr int CS_DIG = 16;
constexpr int CS_CHUNKS = 960;  // chunks per LDS block (960 x 17 words = 64 KB)
template <typename KIND>
__global__ void __launch_bounds__(RS_THREADS) radix_colscan_kernel(const ViewBatch<RowJob> B)
{
    const RowJob& J = B.v[blockIdx.y];
    const int ngroups = (J.nbins + CS_DIG - 1) / CS_DIG;
    if (J.cmin && (int)blockIdx.x == ngroups) {
        reduce_range(J);
        return;
    }
    if ((int)blockIdx.x >= ngroups) return;
    __shared__ uint32_t s_col[CS_CHUNKS * (CS_DIG + 1)];  // [chunk][digit], rows padded to 17 words
    const int tid = threadIdx.x, dl = tid >> 4, sg = tid & 15;
    const uint32_t nb = (uint32_t)J.nbins, nchunks = (uint32_t)J.nchunks;
    const uint32_t d0 = blockIdx.x * CS_DIG;
    const uint32_t nd = min((uint32_t)CS_DIG, nb - d0);
    uint32_t* counts = J.counts;
    uint32_t carry = 0;  // this thread's digit (sg == 15 keeps the column total)
    for (uint32_t c0 = 0; c0 < nchunks; c0 += CS_CHUNKS) {
        const uint32_t nc = min((uint32_t)CS_CHUNKS, nchunks - c0);
        constexpr int U = 8;
        for (uint32_t i0 = tid; i0 < nc * CS_DIG; i0 += U * RS_THREADS) {
            uint32_t v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t i = i0 + u * RS_THREADS, c = i >> 4, dd = i & 15;
                v[u] = (i < nc * CS_DIG && dd < nd) ? counts[(size_t)(c0 + c) * nb + d0 + dd] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t i = i0 + u * RS_THREADS;
                if (i < nc * CS_DIG) s_col[(i >> 4) * (CS_DIG + 1) + (i & 15)] = v[u];
            }
        }
        __syncthreads();
        // segment scan: 16 segments of ceil(nc / 16) chunks per digit
        const uint32_t seg = (nc + 15) / 16;
        const uint32_t j0 = min(sg * seg, nc), j1 = min(j0 + seg, nc);
        uint32_t sum = 0;
        for (uint32_t j = j0; j < j1; j++) sum += s_col[j * (CS_DIG + 1) + dl];
        uint32_t x = sum;  // inclusive scan over the 16 segments of this digit (lanes 16 dl' .. 16 dl' + 15)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 16);
            if (sg >= o) x += y;
        }
        const uint32_t block_total = (uint32_t)__shfl((int)x, 15, 16);
        uint32_t run = carry + x - sum;
        for (uint32_t j = j0; j < j1; j++) {
            const uint32_t c = s_col[j * (CS_DIG + 1) + dl];
            s_col[j * (CS_DIG + 1) + dl] = run;
            run += c;
        }
        carry += block_total;
        __syncthreads();
        for (uint32_t i = tid; i < nc * CS_DIG; i += RS_THREADS) {
            const uint32_t c = i >> 4, dd = i & 15;
            if (dd < nd) counts[(size_t)(c0 + c) * nb + d0 + dd] = s_col[c * (CS_DIG + 1) + dd];
        }
        __syncthreads();  // s_col reuse
    }
    if (sg == 0 && (uint32_t)dl < nd) J.totals[d0 + dl] = carry;
}

struct SortPassArgs {
    int n, shift, nbits, nchunks;
    const uint32_t* keys_in;
    const uint32_t* vals_in;   // payload in; null (unpaired sorts' first pass): the input index
    uint32_t* keys_out;        // intermediate pass: keys_out[dst], vals_out[dst] (u32 or u32x2)
    uint32_t* vals_out;
    // final pass (keys_out == null): out_x[dst] = v.x, out_y[dst] = v.y, sorted_keys[dst] = key
    uint32_t* out_x;
    uint32_t* out_y;
    uint32_t* sorted_keys;
    // final pass, single payload (the depth sort): sorted_rects[dst] = rects[v] and
    // sorted_counts[dst] = its tile count (may be null)
    const uint2* rects;
    uint2* sorted_rects;
    uint32_t* sorted_counts;
    const uint32_t* row_prefix;  // (nbins, nchunks) exclusive row scans
    const uint32_t* totals;      // (nbins) digit totals
    // PAIR, first pass: the payload is (input index, rects4_in[index]) -- the packed rect carried
    // beside the id (the depth sort); the last pass then unpacks v.y into sorted_rects / sorted_counts
    const uint32_t* rects4_in;
    // PAIR, > 0: there is no key array; the key is vals_in[i].y >> key_hi_shift and out_y receives
    // v.y with those bits cleared (the tile sort's second pass, see TileSortJob)
    int key_hi_shift;
    const uint32_t* vals_in_y;  // non-null: the pairs as two arrays, x = vals_in[i], y = vals_in_y[i]
    int mode;                // DigitMode
    const RangeWord* range;
    bool cmaj;               // chunk-major count matrix (cm_index)
    // GSR_DEPTH_GSUM: non-null: row_prefix holds the raw chunk-major counts (no column scan ran) and
    // gsum their per-group sums; the digit offsets are derived from both here
    const uint32_t* gsum = nullptr;
};

// Exclusive scan of one value per thread over the 256-thread block: wave scans by shuffles, then
// one barrier to add the preceding waves' totals (s4: 4 words, not reused before a later barrier).
template <int WAVES>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sw)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) sw[w] = x;
    __syncthreads();
    uint32_t pre = x - v;
    for (int q = 0; q < w; q++) pre += sw[q];
    return pre;
}
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* s4) { return block_excl_scan<4>(v, s4); }

// (3) stable rank + scatter of one chunk.  PAIR: the payload is two u32 words.  NBITS <= 9: up to
// 512 digits (two per thread in the digit-indexed steps).
template <int ITEMS, bool PAIR, typename KIND, int NBITS, int NT = RS_THREADS>
__global__ void __launch_bounds__(NT) radix_scatter_kernel(const ViewBatch<SortPassArgs> B)
{
    const SortPassArgs& a = B.v[blockIdx.y];
    const uint32_t chunk = xcd_chunk(blockIdx.x, gridDim.x);
    if ((int)chunk >= a.nchunks) return;  // past this view's chunks (uniform)
    const Digit dig = make_digit(a.shift, NBITS, a.mode, a.range);
    const bool is_last = a.keys_out == nullptr;
    constexpr int TILE = NT * ITEMS;
    constexpr int NB = 1 << NBITS;
    constexpr int NBA = NB < NT ? NT : NB;  // digit-indexed arrays: at least one per thread
    constexpr int DPT = NBA / NT;                     // digits per thread (1 or 2)
    static_assert(NB <= 2 * NT, "at most 9-bit digits");
    using Val = typename std::conditional<PAIR, uint2, uint32_t>::type;
    constexpr int NW = NT / 64;
    __shared__ uint32_t s_cnt[NW][NBA];  // per-wave running digit counts, then per-wave prefixes
    __shared__ uint32_t s_blk[NBA];     // block-local start of each digit
    __shared__ uint32_t s_base[NBA];    // global start of each digit for this chunk
    __shared__ uint32_t s_keys[TILE];
    __shared__ Val s_vals[TILE];
    __shared__ uint32_t s_w0[NW], s_w1[NW];    // wave totals of the two block scans

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    {
#pragma unroll
    for (int i = 0; i < DPT; i++)
        for (int q = 0; q < NW; q++) s_cnt[q][tid * DPT + i] = 0;
    // digit offsets: exclusive scan of the totals, plus this chunk's row prefix (thread t owns digits
    // [t DPT, t DPT + DPT))
    uint32_t tot[DPT], rowp[DPT], tsum = 0;
    if (a.gsum) {  // digit d: its total = the sum of the group rows; this chunk's offset = the groups
                   // before its own + the chunks of its group before it (chunk-major raw counts)
        const uint32_t ng = ((uint32_t)a.nchunks + GS_CHUNKS - 1) / GS_CHUNKS, cg = chunk / GS_CHUNKS;
#pragma unroll
        for (int i = 0; i < DPT; i++) {
            const uint32_t d = (uint32_t)(tid * DPT + i);
            uint32_t t = 0, pre = 0;
            if (d < (uint32_t)NB) {  // every load of a block issued before the first add (clamped)
                for (uint32_t g0 = 0; g0 < ng; g0 += GS_CHUNKS) {
                    uint32_t x[GS_CHUNKS];
#pragma unroll
                    for (int u = 0; u < GS_CHUNKS; u++) x[u] = a.gsum[(size_t)min(g0 + u, ng - 1) * NB + d];
#pragma unroll
                    for (int u = 0; u < GS_CHUNKS; u++) {
                        const uint32_t g = g0 + u, v = g < ng ? x[u] : 0u;
                        t += v;
                        pre += g < cg ? v : 0u;
                    }
                }
                const uint32_t c0 = cg * GS_CHUNKS, nprev = chunk - c0;  // < GS_CHUNKS
                uint32_t y[GS_CHUNKS - 1];
#pragma unroll
                for (int u = 0; u < GS_CHUNKS - 1; u++) y[u] = a.row_prefix[(size_t)(c0 + min((uint32_t)u, chunk - c0)) * NB + d];
#pragma unroll
                for (int u = 0; u < GS_CHUNKS - 1; u++) pre += (uint32_t)u < nprev ? y[u] : 0u;
            }
            tot[i] = t;
            rowp[i] = pre;
            tsum += t;
        }
    } else {
#pragma unroll
        for (int i = 0; i < DPT; i++) {
            const uint32_t d = (uint32_t)(tid * DPT + i);
            tot[i] = d < (uint32_t)NB ? a.totals[d] : 0u;
            rowp[i] = d < (uint32_t)NB ? a.row_prefix[cm_index(d, chunk, NB, a.nchunks, a.cmaj)] : 0u;
            tsum += tot[i];
        }
    }
    uint32_t gbase[DPT];
    {
        uint32_t run = block_excl_scan<NW>(tsum, s_w0);  // its barrier also publishes s_cnt = 0
#pragma unroll
        for (int i = 0; i < DPT; i++) {
            gbase[i] = run + rowp[i];
            run += tot[i];
        }
    }

    const size_t base = (size_t)chunk * TILE;
    const int nvalid = (int)min((size_t)TILE, (size_t)a.n - base);
    uint32_t key[ITEMS], rank[ITEMS];
    Val val[ITEMS];
    const uint64_t lt = (1ull << lane) - 1ull;
    // issue every load of the chunk before the first ballot (unconditional, clamped addresses)
    auto gidx = [&](int i) { return base + (size_t)min(w * (ITEMS * 64) + i * 64 + lane, nvalid - 1); };
    if (!PAIR && a.key_hi_shift) {  // one-word payload whose high bits hold the key
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            if constexpr (!PAIR) {
                val[i] = a.vals_in[gidx(i)];
                key[i] = val[i] >> a.key_hi_shift;
            }
        }
    } else if (PAIR && a.key_hi_shift) {  // the key rides in the payload's high bits
        if (a.vals_in_y) {
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                if constexpr (PAIR) val[i] = make_uint2(a.vals_in[gidx(i)], a.vals_in_y[gidx(i)]);
            }
        } else {
#pragma unroll
            for (int i = 0; i < ITEMS; i++) val[i] = reinterpret_cast<const Val*>(a.vals_in)[gidx(i)];
        }
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            if constexpr (PAIR) key[i] = val[i].y >> a.key_hi_shift;
        }
    } else {
#pragma unroll
        for (int i = 0; i < ITEMS; i++) key[i] = a.keys_in[gidx(i)];
    }
    if (a.key_hi_shift) {
    } else if (PAIR && a.rects4_in) {  // first pass of a rect-carrying sort: (index, packed rect)
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            if constexpr (PAIR) val[i] = make_uint2((uint32_t)gidx(i), a.rects4_in[gidx(i)]);
        }
    } else if (PAIR || a.vals_in) {  // PAIR: the caller's pairs in the first pass
#pragma unroll
        for (int i = 0; i < ITEMS; i++) val[i] = reinterpret_cast<const Val*>(a.vals_in)[gidx(i)];
    } else {
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            if constexpr (!PAIR) val[i] = (uint32_t)gidx(i);
        }
    }
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const int li = w * (ITEMS * 64) + i * 64 + lane;
        const bool valid = li < nvalid;
        const uint32_t d = dig(key[i]);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < NBITS; b++) {
            const uint64_t bal = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? bal : ~bal;
        }
        const uint32_t before = s_cnt[w][d];
        rank[i] = before + (uint32_t)__popcll(peers & lt);
        const bool leader = valid && (peers & lt) == 0ull;
        if (leader) s_cnt[w][d] = before + (uint32_t)__popcll(peers);
        if (!valid) rank[i] = 0xFFFFFFFFu;
    }
    __syncthreads();

    // per-digit block totals, per-wave exclusive prefixes, block-local digit starts
    uint32_t dtot[DPT], bsum = 0;
#pragma unroll
    for (int i = 0; i < DPT; i++) {
        const int d = tid * DPT + i;
        uint32_t run = 0;
#pragma unroll
        for (int q = 0; q < NW; q++) {  // per-wave exclusive prefixes of the digit
            const uint32_t c = s_cnt[q][d];
            s_cnt[q][d] = run;
            run += c;
        }
        dtot[i] = run;
        bsum += run;
    }
    {
        uint32_t run = block_excl_scan<NW>(bsum, s_w1);
#pragma unroll
        for (int i = 0; i < DPT; i++) {
            s_blk[tid * DPT + i] = run;
            s_base[tid * DPT + i] = gbase[i];
            run += dtot[i];
        }
    }
    __syncthreads();

    // scatter into LDS in block-local sorted (stable) order
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        if (rank[i] != 0xFFFFFFFFu) {
            const uint32_t d = dig(key[i]);
            const uint32_t lpos = s_blk[d] + s_cnt[w][d] + rank[i];
            s_keys[lpos] = key[i];
            s_vals[lpos] = val[i];
        }
    }
    __syncthreads();
    // contiguous write-out: runs of one digit map to consecutive global addresses
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const int lpos = i * NT + tid;
        if (lpos < nvalid) {
            const uint32_t k = s_keys[lpos];
            const uint32_t d = dig(k);
            const uint32_t dst = s_base[d] + ((uint32_t)lpos - s_blk[d]);
            const Val v = s_vals[lpos];
            if (!is_last) {
                a.keys_out[dst] = k;
                reinterpret_cast<Val*>(a.vals_out)[dst] = v;
            } else {
                if constexpr (PAIR) {
                    if (a.out_x) a.out_x[dst] = v.x;
                    if (a.out_y) a.out_y[dst] = a.key_hi_shift ? v.y & ((1u << a.key_hi_shift) - 1u) : v.y;
                    if (a.sorted_rects) {  // the carried packed rect (no gather by id)
                        const uint2 rc = rect_unpack(v.y);
                        a.sorted_rects[dst] = rc;
                        a.sorted_counts[dst] = ((rc.y & 0xFFFFu) - (rc.x & 0xFFFFu)) * ((rc.y >> 16) - (rc.x >> 16));
                    }
                } else {
                    if (a.out_x) a.out_x[dst] = a.key_hi_shift ? v & ((1u << a.key_hi_shift) - 1u) : v;
                    if (a.rects) {
                        const uint2 rc = a.rects[v];
                        a.sorted_rects[dst] = rc;
                        a.sorted_counts[dst] = ((rc.y & 0xFFFFu) - (rc.x & 0xFFFFu)) * ((rc.y >> 16) - (rc.x >> 16));
                    }
                }
                if (a.sorted_keys) a.sorted_keys[dst] = k;
            }
        }
    }
    }
}

// ---------------------------------------------------------------------------
// Emission fused into the first tile-sort pass.  Chunk c of a view = the instances of its depth
// ranks [c * FE_RANKS, (c + 1) * FE_RANKS) in emission order (depth rank, then y-major inside the
// rect: duplicateWithKeys, rasterizer_impl.cu:98-109).  Both kernels stage the chunk's ranks
// (instance start, rect, and for the scatter the Gaussian id and record start) in LDS and derive
// every instance -- owner by binary search over the starts, tile from the owner's rect -- instead of
// reading emitted (tile, slot, id) arrays: the 12 B per instance that emission wrote and the pass
// read back (twice: count and scatter) never touch HBM.  The scatter ranks a chunk in rounds of
// RS_THREADS * ITEMS instances (one round on average: ~6 instances per rank), carrying each digit's
// running output position from round to round, so a chunk of any size stays stable.
// ---------------------------------------------------------------------------
constexpr int FE_RANKS = 256;
#ifndef GSR_TILE_SOA
#define GSR_TILE_SOA 1
#endif

struct FusedPassArgs {
    int P, L, nchunks;
    const uint32_t* sorted_ids;
    const uint32_t* offsets;
    const uint2* sorted_rects;
    const uint32_t* rec_start;
    uint32_t* counts;  // (bins, nchunks)
    uint32_t* totals;  // (bins)
    // outputs: keys_out / vals_out (u32x2) -- or, if this is the only pass, the final arrays
    uint32_t* keys_out;
    uint2* vals_out;
    uint32_t* out_slot;
    uint32_t* out_ids;
    uint32_t* out_tiles;
    uint32_t* valid;
    uint2* ranges;
    // > 0 (two passes, no tile ids wanted): no key array; the pass writes (slot, id | (tile >> w1)
    // << pack_shift) and the second pass takes its key from those bits -- as two arrays (soa_x: slot,
    // soa_y: the id word), so that the second pass's count kernel reads 4 B per instance, not 8
    int pack_shift, pack_w1;
    uint32_t* soa_x;
    uint32_t* soa_y;
};

// GSR_FE_AOS: a rank's fields as one 16-B {start, x0 | y0 << 16, w, 1/w} and one 8-B {record start,
// id} LDS entry (one ds_read_b128 + one ds_read_b64 per derived instance at the write-out, whose
// owners are random across the lanes), instead of seven separate arrays (seven reads)
#ifndef GSR_FE_AOS
#define GSR_FE_AOS 1
#endif
struct FeRanks {
    uint32_t start[FE_RANKS];  // (also in geo: the owner search reads this array)
#if GSR_FE_AOS
    uint4 geo[FE_RANKS];
    uint2 idr[FE_RANKS];
#else
    uint32_t x0[FE_RANKS], y0[FE_RANKS], w[FE_RANKS], g[FE_RANKS], rec[FE_RANKS];
    float rw[FE_RANKS];  // 1 / w
#endif
};

// Stages chunk c's ranks; [wbeg, wend) is its instance range.  Ends with a barrier.
template <bool IDS>
__device__ __forceinline__ void fe_stage(const FusedPassArgs& J, int c, FeRanks& s, uint32_t& wbeg, uint32_t& wend)
{
    const int tid = threadIdx.x;
    const int k0 = c * FE_RANKS, k = k0 + tid;
    uint32_t start = 0xFFFFFFFFu, x0 = 0, y0 = 0, wd = 1, g = 0, rec = 0;
    if (k < J.P) {
        start = k == 0 ? 0u : J.offsets[k - 1];
        const uint2 rc = J.sorted_rects[k];
        x0 = rc.x & 0xFFFFu;
        y0 = rc.x >> 16;
        wd = max((rc.y & 0xFFFFu) - x0, 1u);
        if (IDS) {
            g = J.sorted_ids[k];
            // GSR_SLOT_LOCAL: the instance's index inside its Gaussian's rect is stored instead of the
            // absolute record slot (render_bwd adds emit_start[id], which it loads anyway): no
            // dependent gather of the record start behind the id here
            rec = GSR_SLOT_LOCAL ? 0u : J.rec_start[g];
        }
    }
    s.start[tid] = start;
#if GSR_FE_AOS
    s.geo[tid] = make_uint4(start, x0 | (y0 << 16), wd, __float_as_uint(1.0f / (float)wd));
    if (IDS) s.idr[tid] = make_uint2(rec, g);
#else
    s.x0[tid] = x0;
    s.y0[tid] = y0;
    s.w[tid] = wd;
    s.rw[tid] = 1.0f / (float)wd;
    if (IDS) {
        s.g[tid] = g;
        s.rec[tid] = rec;
    }
#endif
    wbeg = k0 == 0 ? 0u : J.offsets[k0 - 1];
    wend = J.offsets[min(k0 + FE_RANKS, J.P) - 1];
    __syncthreads();
}

// The owner of instance sl (the largest staged rank whose start is <= sl: ranks without instances
// share their successor's start) and its local index inside the owner's rect.
__device__ __forceinline__ int fe_owner(const FeRanks& s, uint32_t sl)
{
    int j = 0;
#pragma unroll
    for (int step = FE_RANKS / 2; step >= 1; step >>= 1)
        if (s.start[j + step] <= sl) j += step;
    return j;
}

__device__ __forceinline__ uint32_t fe_tile(const FeRanks& s, int j, uint32_t sl, uint32_t gx, uint32_t& local)
{
#if GSR_FE_AOS
    const uint4 q = s.geo[j];
    const uint32_t st = q.x, x0 = q.y & 0xFFFFu, y0 = q.y >> 16, wj = q.z;
    const float rw = __uint_as_float(q.w);
#else
    const uint32_t st = s.start[j], x0 = s.x0[j], y0 = s.y0[j], wj = s.w[j];
    const float rw = s.rw[j];
#endif
    local = sl - st;
    // local / wj by a reciprocal estimate (off by at most one for local < 2^24) and one correction
    // each way, instead of the ~40-instruction integer division
    uint32_t yy = (uint32_t)((float)local * rw);
    yy -= yy * wj > local ? 1u : 0u;
    yy += (yy + 1u) * wj <= local ? 1u : 0u;
    const uint32_t xx = local - yy * wj;
    return (y0 + yy) * gx + (x0 + xx);
}

__global__ void __launch_bounds__(RS_THREADS) fused_pass1_count_kernel(const ViewBatch<FusedPassArgs> B, uint32_t gx,
                                                                      int T, int nbits)
{
    const FusedPassArgs& J = B.v[blockIdx.y];
    const int c = (int)blockIdx.x;
    if (c >= J.nchunks) return;  // past this view's chunks (uniform)
    __shared__ uint32_t h[4][RS_MAXBINS];
    const int tid = threadIdx.x, w = tid >> 6;
    // ranges must be zero for tile_ranges (empty tiles keep (0, 0)): cleared here, not by a memset
    if (J.ranges)  // (null: the tile order writes every range from the rects' difference array)
        for (int t = c * RS_THREADS + tid; t < T; t += J.nchunks * RS_THREADS) J.ranges[t] = make_uint2(0u, 0u);
    for (int q = 0; q < 4; q++) h[q][tid] = 0;
    __syncthreads();
    // a histogram needs no instance order: each thread walks its own rank's rect (no owner search)
    const uint32_t nb = 1u << nbits, mask = nb - 1u;
    const int k = c * FE_RANKS + tid;
    if (k < J.P) {
        const uint32_t start = k == 0 ? 0u : J.offsets[k - 1], end = J.offsets[k];
        if (end > start) {
            const uint2 rc = J.sorted_rects[k];
            const uint32_t x0 = rc.x & 0xFFFFu, y0 = rc.x >> 16, x1 = rc.y & 0xFFFFu, y1 = rc.y >> 16;
            for (uint32_t y = y0; y < y1; y++)
                for (uint32_t x = x0; x < x1; x++) atomicAdd(&h[w][(y * gx + x) & mask], 1u);
        }
    }
    __syncthreads();
    if ((uint32_t)tid < nb) J.counts[cm_index(tid, c, nb, J.nchunks, false)] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

template <int ITEMS, int NBITS>
__global__ void __launch_bounds__(RS_THREADS) fused_pass1_scatter_kernel(const ViewBatch<FusedPassArgs> B, uint32_t gx)
{
    constexpr int nbits = NBITS;  // the digit width, a compile-time constant (unrolled ballot ranking)
    constexpr int TILE = RS_THREADS * ITEMS;
    const FusedPassArgs& J = B.v[blockIdx.y];
    // (no xcd_chunk here: a chunk's instance count falls with the depth of its ranks, and contiguous
    // depth ranges per XCD unbalance the XCDs -- measured +16 %)
    const int c = (int)blockIdx.x;
    if (c >= J.nchunks) return;  // past this view's chunks (uniform)
    __shared__ FeRanks s;
    __shared__ uint32_t s_cnt[4][RS_MAXBINS];  // per-wave running digit counts, then per-wave prefixes
    __shared__ uint32_t s_blk[RS_MAXBINS];     // round-local start of each digit
    __shared__ uint32_t s_base[RS_MAXBINS];    // global position of each digit's next element
    __shared__ uint16_t s_idx[TILE];  // round position of the element at each sorted slot
    __shared__ __attribute__((aligned(8))) uint8_t s_own[TILE];  // owner (staged rank) of each round position
    __shared__ uint32_t s_w0[4], s_w1[4], s_w2[4];
    static_assert(TILE == 8 * RS_THREADS && FE_RANKS <= 256, "owner scan: 8 positions per thread, u8 ranks");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t nb = 1u << nbits, mask = nb - 1u;
    for (int q = 0; q < 4; q++) s_cnt[q][tid] = 0;
    const uint32_t tot = (uint32_t)tid < nb ? J.totals[tid] : 0u;
    const uint32_t rowp = (uint32_t)tid < nb ? J.counts[cm_index(tid, c, nb, J.nchunks, false)] : 0u;
    const uint32_t gbase = block_excl_scan256(tot, s_w0) + rowp;
    s_base[tid] = gbase;
    reinterpret_cast<uint64_t*>(s_own)[tid] = 0ull;  // the first round's owner marks start from zero
    uint32_t wbeg, wend;
    fe_stage<true>(J, c, s, wbeg, wend);  // its barrier also publishes s_cnt = 0, s_base and s_own
    const uint64_t lt = (1ull << lane) - 1ull;
    const bool last = J.keys_out == nullptr && !J.pack_shift;
    // this thread's staged rank: start and end of its instances
    const uint32_t my_start = s.start[tid];
    const uint32_t my_end = min(tid + 1 < FE_RANKS ? s.start[tid + 1] : wend, wend);
    // the backward flags the records it writes: clear the bit words starting in this rank's
    // instances (here, not in the count kernel, which runs before L and the binning buffer exist)
    if (my_end > my_start)
        for (uint32_t sl = (my_start + 31u) & ~31u; sl < my_end; sl += 32u) J.valid[sl >> 5] = 0u;
    for (uint32_t r0 = wbeg; r0 < wend; r0 += TILE) {
        const int nvalid = (int)min((uint32_t)TILE, wend - r0);
        // owners of the round's positions without a search per instance: every rank starting inside
        // the round marks its first position (s_own is zero here), and an inclusive max-scan (ranks
        // increase with the position) seeded with the owner of r0 fills the rest
        if (my_end > my_start && my_start >= r0 && my_start < r0 + (uint32_t)nvalid)
            s_own[my_start - r0] = (uint8_t)tid;
        __syncthreads();
        {
            const uint32_t j0 = (uint32_t)fe_owner(s, r0);
            const uint64_t q = reinterpret_cast<const uint64_t*>(s_own)[tid];
            uint32_t b[8], mt = 0;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                b[e] = (uint32_t)(q >> (8 * e)) & 0xFFu;
                mt = max(mt, b[e]);
            }
            uint32_t inc = mt;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)inc, d, 64);
                if (lane >= d) inc = max(inc, y);
            }
            if (lane == 63) s_w2[w] = inc;
            __syncthreads();
            uint32_t run = j0;
            for (int qq = 0; qq < w; qq++) run = max(run, s_w2[qq]);
            const uint32_t ex = (uint32_t)__shfl_up((int)inc, 1, 64);
            if (lane > 0) run = max(run, ex);
            uint64_t o = 0;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                run = max(run, b[e]);
                o |= (uint64_t)run << (8 * e);
            }
            reinterpret_cast<uint64_t*>(s_own)[tid] = o;
        }
        __syncthreads();
        // only the digit is kept per element (the sorted slots stage round positions, and the
        // write-out derives tile, slot and id again): 2 B of LDS per element instead of 12, and
        // no payload registers
        // a partial round (most rounds: a chunk holds ~1,500 instances of its 2,048 slots) leaves
        // whole 64-element items of the last waves empty: they skip the digit derivation and the
        // ballots (wave-uniform test)
        uint32_t key[ITEMS], rank[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const int li = w * (ITEMS * 64) + i * 64 + lane;
            key[i] = 0u;
            if (w * (ITEMS * 64) + i * 64 >= nvalid) continue;
            const uint32_t sl = r0 + (uint32_t)min(li, nvalid - 1);
            const int j = s_own[min(li, nvalid - 1)];
            uint32_t local;
            key[i] = fe_tile(s, j, sl, gx, local) & mask;
        }
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const int li = w * (ITEMS * 64) + i * 64 + lane;
            rank[i] = 0xFFFFFFFFu;
            if (w * (ITEMS * 64) + i * 64 >= nvalid) continue;
            const bool valid = li < nvalid;
            const uint32_t d = key[i];
            uint64_t peers = __ballot(valid);
#pragma unroll
            for (int b = 0; b < NBITS; b++) {
                const uint64_t bal = __ballot((d >> b) & 1u);
                peers &= ((d >> b) & 1u) ? bal : ~bal;
            }
            const uint32_t before = s_cnt[w][d];
            rank[i] = before + (uint32_t)__popcll(peers & lt);
            const bool leader = valid && (peers & lt) == 0ull;
            if (leader) s_cnt[w][d] = before + (uint32_t)__popcll(peers);
            if (!valid) rank[i] = 0xFFFFFFFFu;
        }
        __syncthreads();
        const uint32_t c0 = s_cnt[0][tid], c1 = s_cnt[1][tid], c2 = s_cnt[2][tid], c3 = s_cnt[3][tid];
        const uint32_t total = c0 + c1 + c2 + c3;
        s_cnt[0][tid] = 0;
        s_cnt[1][tid] = c0;
        s_cnt[2][tid] = c0 + c1;
        s_cnt[3][tid] = c0 + c1 + c2;
        s_blk[tid] = block_excl_scan256(total, s_w1);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            if (rank[i] != 0xFFFFFFFFu) {
                const uint32_t d = key[i];
                const uint32_t lpos = s_blk[d] + s_cnt[w][d] + rank[i];
                s_idx[lpos] = (uint16_t)(w * (ITEMS * 64) + i * 64 + lane);
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {  // contiguous write-out: runs of one digit
            const int lpos = i * RS_THREADS + tid;
            if (lpos < nvalid) {
                const uint32_t li = s_idx[lpos];
                const int j = s_own[li];
                uint32_t local;
                const uint32_t k = fe_tile(s, j, r0 + li, gx, local);
                const uint32_t d = k & mask;
                const uint32_t dst = s_base[d] + ((uint32_t)lpos - s_blk[d]);
#if GSR_FE_AOS
                const uint2 ig = s.idr[j];
                const uint2 v = make_uint2(ig.x + local, ig.y);
#else
                const uint2 v = make_uint2(s.rec[j] + local, s.g[j]);
#endif
                if (J.pack_shift) {
                    if (J.soa_y) {
                        if (J.soa_x) J.soa_x[dst] = v.x;  // (no slot array: slots_from_rect)
                        J.soa_y[dst] = v.y | ((k >> J.pack_w1) << J.pack_shift);
                    } else {
                        J.vals_out[dst] = make_uint2(v.x, v.y | ((k >> J.pack_w1) << J.pack_shift));
                    }
                } else if (!last) {
                    J.keys_out[dst] = k;
                    J.vals_out[dst] = v;
                } else {
                    if (J.out_slot) J.out_slot[dst] = v.x;
                    J.out_ids[dst] = v.y;
                    if (J.out_tiles) J.out_tiles[dst] = k;
                }
            }
        }
        // most chunks take one round: they skip the next round's set-up and its two barriers
        if (r0 + (uint32_t)TILE >= wend) break;
        __syncthreads();
        s_base[tid] += total;  // the next round's elements follow this round's in every digit
        s_cnt[0][tid] = s_cnt[1][tid] = s_cnt[2][tid] = s_cnt[3][tid] = 0;
        reinterpret_cast<uint64_t*>(s_own)[tid] = 0ull;
        __syncthreads();
    }
}

// identifyTileRanges (rasterizer_impl.cu:116-138): four consecutive instances per thread (one
// 16-byte load); each element's predecessor comes from the same load or, for the first, from the
// neighbouring lane (the wave's first lane loads it).
__global__ void __launch_bounds__(256) tile_ranges_kernel(const ViewBatch<RangesJob> B)
{
    const int L = B.v[blockIdx.y].L;
    const uint32_t* sorted_tiles = B.v[blockIdx.y].sorted_tiles;
    uint2* ranges = B.v[blockIdx.y].ranges;
    if ((int)blockIdx.x * 256 * 4 >= L) return;  // past this view's instances (uniform)
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const int i0 = 4 * t;
    uint32_t v[4];
    if (i0 + 4 <= L) {
        const uint4 q = reinterpret_cast<const uint4*>(sorted_tiles)[t];
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = i0 + k < L ? sorted_tiles[i0 + k] : 0u;
    }
    uint32_t prev = (uint32_t)__shfl_up((int)v[3], 1, 64);  // every lane, before any exit
    if (lane == 0 && i0 > 0 && i0 - 1 < L) prev = sorted_tiles[i0 - 1];
    if (i0 >= L) return;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = i0 + k;
        if (i >= L) break;
        const uint32_t cur = v[k];
        const uint32_t p = k == 0 ? prev : v[k - 1];
        if (i == 0) ranges[cur].x = 0;
        else if (cur != p) {
            ranges[p].y = (uint32_t)i;
            ranges[cur].x = (uint32_t)i;
        }
        if (i == L - 1) ranges[cur].y = (uint32_t)L;
    }
}

// The rects' 2-D difference array (TileHistJob): every workgroup of a view takes a strided share of
// the P packed rects (culled Gaussians have an empty rect), adds +1 / -1 at the four corners into an
// LDS copy of the array, and adds its non-zero cells into the view's array in HBM (zeroed by
// preprocess) with integer atomics: 16 x 33 KB of contiguous atomic traffic per 1080p view instead
// of a pass over the L sorted tile ids (tile_ranges) and their L x 4 B written by the tile sort.
constexpr int TILE_HIST_WGS = 16;
__global__ void __launch_bounds__(1024) tile_hist_kernel(const ViewBatch<TileHistJob> B, uint32_t gx, uint32_t gy)
{
    const TileHistJob& J = B.v[blockIdx.y];
    extern __shared__ int s_h[];
    const uint32_t sx = gx + 1;
    const int cells = (int)(sx * (gy + 1));
    const int tid = threadIdx.x;
    for (int c = tid; c < cells; c += 1024) s_h[c] = 0;
    __syncthreads();
    auto add = [&](uint32_t r) {
        const uint32_t x0 = r & 0xFFu, y0 = (r >> 8) & 0xFFu, x1 = (r >> 16) & 0xFFu, y1 = r >> 24;
        if (x1 > x0 && y1 > y0) {
            atomicAdd(&s_h[y0 * sx + x0], 1);
            atomicAdd(&s_h[y0 * sx + x1], -1);
            atomicAdd(&s_h[y1 * sx + x0], -1);
            atomicAdd(&s_h[y1 * sx + x1], 1);
        }
    };
    // four rects per 16-B load, eight loads in flight per thread before the first LDS atomic (the
    // loop is latency-bound otherwise: one dependent round trip per rect)
    constexpr int U = 8, STRIDE = TILE_HIST_WGS * 1024;
    const int n4 = J.P >> 2;
    const uint4* r4 = reinterpret_cast<const uint4*>(J.rect4);
    for (int i0 = (int)blockIdx.x * 1024 + tid; i0 < n4; i0 += U * STRIDE) {
        uint4 q[U];
#pragma unroll
        for (int u = 0; u < U; u++) q[u] = i0 + u * STRIDE < n4 ? r4[i0 + u * STRIDE] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int u = 0; u < U; u++) {
            add(q[u].x);
            add(q[u].y);
            add(q[u].z);
            add(q[u].w);
        }
    }
    if (blockIdx.x == 0 && tid < (J.P & 3)) add(J.rect4[4 * n4 + tid]);  // the last P mod 4 rects
    __syncthreads();
    for (int c = tid; c < cells; c += 1024) {
        const int v = s_h[c];
        if (v) atomicAdd(&J.diff[c], v);
    }
}

// the reference's 64-bit keys (tile << 32 | depth bits, rasterizer_impl.cu:98-106) of the sorted
// instances, from the depth-sort keys (the depth bits of every listed Gaussian: preprocess writes
// them in single-view and batched forwards alike)
__global__ void __launch_bounds__(256) debug_keys_kernel(int L, const uint32_t* sorted_tiles, const uint32_t* point_list,
                                                         const uint32_t* dkeys, uint64_t* keys)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= L) return;
    keys[idx] = ((uint64_t)sorted_tiles[idx] << 32) | dkeys[point_list[idx]];
}

static inline int rs_items(int n) { return n <= RS_SHORT_MAX ? RS_ITEMS_SHORT : RS_ITEMS; }
static inline size_t rs_chunks_tile(int n, int tile) { return ((size_t)(n > 0 ? n : 0) + tile - 1) / tile; }
static inline size_t rs_chunks(int n)
{
    const size_t tile = (size_t)RS_THREADS * rs_items(n);
    return ((size_t)(n > 0 ? n : 0) + tile - 1) / tile;
}

// Scratch of one sort: the (bins x chunks) count matrix and the bin totals (reused by every pass),
// then the per-chunk key min / max and the RangeWord of a three-pass depth sort.
static inline size_t rs_count_bytes(int n) { return align_up(rs_chunks(n) * RS_SCRATCH_BINS * 4 + 256, 256); }
static inline size_t rs_totals_bytes() { return align_up(RS_SCRATCH_BINS * 4, 256); }
// ... then the chunk-group digit counts of the three passes of a depth sort (GSR_DEPTH_GSUM)
static inline size_t rs_gsum_stride(int n)
{
    return align_up((rs_chunks(n) + GS_CHUNKS - 1) / GS_CHUNKS * RS_SCRATCH_BINS * 4, 256);
}
size_t radix_gsum_offset(int n) { return rs_count_bytes(n) + rs_totals_bytes() + align_up(2 * rs_chunks(n) * 4 + 64, 256); }
size_t radix_gsum_bytes(int n) { return 3 * rs_gsum_stride(n); }  // (DEPTH3_PASSES)
size_t radix_status_bytes(int n, int npass)
{
    (void)npass;
    return radix_gsum_offset(n) + radix_gsum_bytes(n);
}
static_assert(RS_THREADS * RS_ITEMS == 2048 && RS_THREADS * RS_ITEMS_SHORT == 2048 && RS_MAXBINS == 256,
              "2,048-key chunks");

// Full LSD sort of n u32 keys over bits [0, nbits), stable.  Payload: the input index i, or with
// `pairs` the u32x2 pairs[i].  Ping-pongs between (k0,v0) and (k1,v1) (v: u32, or u32x2 with
// pairs); the last pass writes out_x[dst] = i (pairs[i].x), out_y[dst] = pairs[i].y and
// sorted_keys[dst] = key (any of them may be null); without pairs it can also lay out rects[i]
// and their tile counts in sorted order.  All writes are contiguous runs: no scattered stores.
// radix_sort_batch: V such sorts (one per view, same bit width and pairing), each pass's three
// kernels launched once for all of them (grid.y = view).
template <typename F>
static hipError_t for_groups(int V, F f)
{
    for (int v0 = 0; v0 < V; v0 += VIEW_BATCH) {
        const hipError_t e = f(v0, min(VIEW_BATCH, V - v0));
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

static inline uint32_t* sort_counts(const SortJob& j) { return reinterpret_cast<uint32_t*>(j.scratch); }
static inline uint32_t* sort_totals(const SortJob& j)
{
    return reinterpret_cast<uint32_t*>(j.scratch + rs_count_bytes(j.n));
}
// per-chunk min (nchunks words), max (nchunks words), then the RangeWord (8-B aligned)
static inline uint32_t* sort_minmax(const SortJob& j)
{
    return reinterpret_cast<uint32_t*>(j.scratch + rs_count_bytes(j.n) + rs_totals_bytes());
}
static inline RangeWord* sort_range(const SortJob& j)
{
    return reinterpret_cast<RangeWord*>(sort_minmax(j) + 2 * ((rs_chunks(j.n) + 1) & ~(size_t)1));
}
static inline uint32_t* sort_gsum(const SortJob& j, int pass)
{
    return reinterpret_cast<uint32_t*>(j.scratch + radix_gsum_offset(j.n) + (size_t)pass * rs_gsum_stride(j.n));
}

// (2) for a pass of nbins digits over (up to) maxc chunks: the per-digit exclusive scans over the
// chunks and the digit totals (+ the range workgroup)
static inline bool chunk_major(int maxc) { return GSR_COLSCAN && maxc <= CS_CHUNKS; }
template <typename KIND>
static void launch_scan_rows(const ViewBatch<RowJob>& rb, int nv, int nbins, int maxc, bool range, hipStream_t s)
{
    const dim3 b(RS_THREADS);
    if (chunk_major(maxc)) {
        const dim3 g((unsigned)((nbins + CS_DIG - 1) / CS_DIG + (range ? 1 : 0)), (unsigned)nv);
        hipLaunchKernelGGL(radix_colscan_kernel<KIND>, g, b, 0, s, rb);
        return;
    }
    const dim3 g((unsigned)(nbins + (range ? 1 : 0)), (unsigned)nv);
    if (maxc <= RS_ROW_LDS)
        hipLaunchKernelGGL(radix_rowscan_lds_kernel<KIND>, g, b, 0, s, rb);
    else
        hipLaunchKernelGGL(radix_rowscan_kernel<KIND>, g, b, 0, s, rb);
}

size_t radix_range_offset(int n)
{
    return rs_count_bytes(n) + rs_totals_bytes() + 4 * 2 * ((rs_chunks(n) + 1) & ~(size_t)1);
}

// One radix pass of a sort: digit width, key shift, DigitMode.
struct PassSpec { int w, shift, mode; };
// The full 32-bit key sorts (the depth sort) in three 9-bit passes, the third relative to the keys'
// minimum (DigitMode); after a range that did not fit (four_pass), four 8-bit passes.
constexpr int DEPTH3_PASSES = 3;  // (radix_gsum_bytes: one group matrix per pass)
constexpr PassSpec DEPTH3[DEPTH3_PASSES] = {{9, 0, DIG_RAW}, {9, 9, DIG_RAW}, {9, 18, DIG_REL}};
#ifndef GSR_DEPTH3
#define GSR_DEPTH3 1
#endif
// test hook (gsr_debug_set_depth_wide): this host thread's depth sorts run four passes
static thread_local bool t_force_wide = false;
void set_depth_force_wide(bool on) { t_force_wide = on; }
bool depth_force_wide() { return t_force_wide || !GSR_DEPTH3; }

template <typename KIND>
static hipError_t radix_sort_batch_k(const SortJob* jobs, int V, int nbits, hipStream_t s, int shift0, bool four_pass)
{
    if (nbits < 1) nbits = 1;
    const bool depth3 = !four_pass && !depth_force_wide() && nbits == 32 && shift0 == 0 &&
                        std::is_same<KIND, DepthSort>::value;
    const int npass = depth3 ? DEPTH3_PASSES : (nbits + 7) / 8;
    const bool gsum = depth3 && GSR_DEPTH_GSUM;  // no column-scan launches (see GS_CHUNKS)
    return for_groups(V, [&](int v0, int nv) -> hipError_t {
        if (gsum)
            for (int v = 0; v < nv; v++) {
                const SortJob& j = jobs[v0 + v];
                if (!j.gsum_zeroed && j.n > 0) {
                    const hipError_t e = hipMemsetAsync(sort_gsum(j, 0), 0, radix_gsum_bytes(j.n), s);
                    if (e != hipSuccess) return e;
                }
            }
        int maxc = 0;
        bool pair = false;
        for (int v = 0; v < nv; v++) {
            maxc = max(maxc, (int)rs_chunks(jobs[v0 + v].n));
            pair = jobs[v0 + v].pairs != nullptr || jobs[v0 + v].rects4 != nullptr || jobs[v0 + v].soa_x != nullptr;
        }
        for (int v = 0; v < nv; v++)  // one payload width per launch
            if ((jobs[v0 + v].pairs != nullptr || jobs[v0 + v].rects4 != nullptr || jobs[v0 + v].soa_x != nullptr) != pair)
                return hipErrorInvalidValue;
        if (maxc == 0) return hipSuccess;
        const uint32_t* kin[VIEW_BATCH];
        const uint32_t* vin[VIEW_BATCH];
        for (int v = 0; v < nv; v++) {
            kin[v] = jobs[v0 + v].keys_in;
            vin[v] = reinterpret_cast<const uint32_t*>(jobs[v0 + v].pairs);
            // keys carried in the pairs' high bits: one pass only (the bits hold one digit)
            if (jobs[v0 + v].key_hi_shift && (npass != 1 || !(jobs[v0 + v].pairs || jobs[v0 + v].soa_y)))
                return hipErrorInvalidValue;
            if (jobs[v0 + v].soa_x) vin[v] = jobs[v0 + v].soa_x;
            else if (jobs[v0 + v].soa_y) vin[v] = jobs[v0 + v].soa_y;  // one-word payload
        }
        int shift = shift0;
        for (int p = 0; p < npass; p++) {
            const int w = depth3 ? DEPTH3[p].w : nbits / npass + (p < nbits % npass ? 1 : 0);  // balanced widths
            if (depth3) shift = DEPTH3[p].shift;
            const int mode = depth3 ? DEPTH3[p].mode : DIG_RAW;
            // 9-bit passes rank 4,096-key chunks with 512 threads, so that each digit's run in a chunk
            // stays as long as an 8-bit pass's over 2,048 keys (coalesced write-out)
            const bool wide = w > 8;
            const int nt = wide ? RS_THREADS_WIDE : RS_THREADS;
            int maxc_p = 0;
            for (int v = 0; v < nv; v++) maxc_p = max(maxc_p, (int)rs_chunks_tile(jobs[v0 + v].n, nt * RS_ITEMS));
            const bool last = p == npass - 1;
            const bool final_out = last;
            ViewBatch<CountJob> cb;
            ViewBatch<RowJob> rb;
            ViewBatch<SortPassArgs> sb;
            cb.n = rb.n = sb.n = nv;
            for (int v = 0; v < nv; v++) {
                const SortJob& j = jobs[v0 + v];
                const int nchunks = (int)rs_chunks_tile(j.n, nt * RS_ITEMS);
                cb.v[v] = {kin[v], j.n, nchunks, sort_counts(j), j.key_hi_shift ? j.pairs : nullptr, j.key_hi_shift};
                if (j.key_hi_shift) cb.v[v].keys = nullptr;
                cb.v[v].hi_words = j.key_hi_shift ? j.soa_y : nullptr;
                cb.v[v].mode = mode;
                cb.v[v].range = sort_range(j);
                cb.v[v].cmaj = gsum || chunk_major(maxc_p);
                if (gsum) {
                    cb.v[v].gsum = sort_gsum(j, p);
                    if (p == 1) {  // the pass-3 key range, from pass 1's per-chunk min / max
                        cb.v[v].range_out = sort_range(j);
                        cb.v[v].rcmin = sort_minmax(j);
                        cb.v[v].rcmax = sort_minmax(j) + nchunks;
                        cb.v[v].rnchunks = nchunks;  // (every pass of a depth sort: the same 4,096-key chunks)
                        cb.v[v].rel_shift = DEPTH3[2].shift;
                        cb.v[v].rel_bits = DEPTH3[2].w;
                        cb.v[v].host_wide = j.host_wide;
                    }
                }
                rb.v[v] = {sort_counts(j), nchunks, sort_totals(j)};
                if (depth3 && p == 0) {  // the keys' range, for the relative pass
                    cb.v[v].cmin = sort_minmax(j);
                    cb.v[v].cmax = sort_minmax(j) + nchunks;
                    rb.v[v].cmin = cb.v[v].cmin;
                    rb.v[v].cmax = cb.v[v].cmax;
                    rb.v[v].range_out = sort_range(j);
                    rb.v[v].nbins = 1 << w;
                    rb.v[v].rel_shift = DEPTH3[2].shift;
                    rb.v[v].rel_bits = DEPTH3[2].w;
                    rb.v[v].host_wide = j.host_wide;
                }
                SortPassArgs& a = sb.v[v];
                a.n = j.n;
                a.shift = shift;
                a.nbits = w;
                a.nchunks = nchunks;
                a.keys_in = kin[v];
                a.vals_in = vin[v];
                a.keys_out = last ? nullptr : ((p & 1) ? j.k1 : j.k0);
                a.vals_out = last ? nullptr : ((p & 1) ? j.v1 : j.v0);
                a.out_x = j.out_x;
                a.out_y = j.out_y;
                a.sorted_keys = j.sorted_keys;
                a.rects = (final_out && !pair) ? j.rects : nullptr;
                a.rects4_in = p == 0 ? j.rects4 : nullptr;
                a.sorted_rects = (final_out && (!pair || j.rects4)) ? j.sorted_rects : nullptr;
                a.sorted_counts = j.sorted_counts;
                a.row_prefix = sort_counts(j);
                a.totals = sort_totals(j);
                a.key_hi_shift = j.key_hi_shift;
                a.vals_in_y = (p == 0 && j.soa_x) ? j.soa_y : nullptr;
                a.mode = mode;
                a.range = sort_range(j);
                a.cmaj = gsum || chunk_major(maxc_p);
                a.gsum = gsum ? sort_gsum(j, p) : nullptr;
                kin[v] = a.keys_out;
                vin[v] = a.vals_out;
            }
            const dim3 g((unsigned)maxc_p, (unsigned)nv), b(RS_THREADS), bw(RS_THREADS_WIDE);
            const dim3 gs(scatter_grid(maxc_p), (unsigned)nv);  // (xcd_chunk)
            if (wide)
                hipLaunchKernelGGL((radix_count_kernel<RS_ITEMS, KIND, 512, RS_THREADS_WIDE>), g, bw, 0, s, cb, shift, w);
            else
                hipLaunchKernelGGL((radix_count_kernel<RS_ITEMS, KIND, RS_MAXBINS>), g, b, 0, s, cb, shift, w);
            for (int v = 0; v < nv; v++) rb.v[v].nbins = 1 << w;
            if (!gsum) launch_scan_rows<KIND>(rb, nv, 1 << w, maxc_p, depth3 && p == 0, s);
            if (wide) {
                if (pair)
                    hipLaunchKernelGGL((radix_scatter_kernel<RS_ITEMS, true, KIND, 9, RS_THREADS_WIDE>), gs, bw, 0, s, sb);
                else
                    hipLaunchKernelGGL((radix_scatter_kernel<RS_ITEMS, false, KIND, 9, RS_THREADS_WIDE>), gs, bw, 0, s, sb);
                shift += w;
                continue;
            }
            switch (w * 2 + (pair ? 1 : 0)) {
#define GSR_SCATTER_W(W_)                                                                                    \
    case 2 * W_: hipLaunchKernelGGL((radix_scatter_kernel<RS_ITEMS, false, KIND, W_>), gs, b, 0, s, sb); break; \
    case 2 * W_ + 1: hipLaunchKernelGGL((radix_scatter_kernel<RS_ITEMS, true, KIND, W_>), gs, b, 0, s, sb); break;
                GSR_SCATTER_W(1) GSR_SCATTER_W(2) GSR_SCATTER_W(3) GSR_SCATTER_W(4)
                GSR_SCATTER_W(5) GSR_SCATTER_W(6) GSR_SCATTER_W(7) GSR_SCATTER_W(8)
#undef GSR_SCATTER_W
            default: return hipErrorInvalidValue;
            }
            shift += w;
        }
        return hipGetLastError();
    });
}

hipError_t radix_sort_batch(const SortJob* jobs, int V, int nbits, hipStream_t s, int shift0, SortKind kind,
                            bool four_pass)
{
    switch (kind) {
    case SORT_TILE: return radix_sort_batch_k<TileSort>(jobs, V, nbits, s, shift0, four_pass);
    case SORT_CELLS: return radix_sort_batch_k<CellSort>(jobs, V, nbits, s, shift0, four_pass);
    default: return radix_sort_batch_k<DepthSort>(jobs, V, nbits, s, shift0, four_pass);
    }
}

#ifndef GSR_TILE_W1_DELTA
#define GSR_TILE_W1_DELTA -1
#endif

size_t fused_pass1_scratch_bytes(int P)
{
    const size_t chunks = ((size_t)(P > 0 ? P : 0) + FE_RANKS - 1) / FE_RANKS;
    return align_up(chunks * RS_MAXBINS * 4 + 256, 256) + align_up(RS_MAXBINS * 4, 256);
}

hipError_t tile_sort_fused_batch(const TileSortJob* jobs, int V, uint32_t gx, int T, hipStream_t s, int phases)
{
    const int nbits = max((int)higher_msb((uint32_t)T), 1);
    const int npass = (nbits + 7) / 8;
    // the first (fused) pass's digit width: one bit narrower than balanced when there are two passes
    // (the fused pass costs more per digit bit than the plain second one: 6 + 7 bits at 1080p measured
    // 480-487 us per 8-view tile sort against 490-493 for 7 + 6, and 8 + 5 567-579)
    int w1 = nbits / npass + (nbits % npass ? 1 : 0);
    if (npass == 2) w1 = min(max(w1 + GSR_TILE_W1_DELTA, nbits - 8), 8);
    return for_groups(V, [&](int v0, int nv) -> hipError_t {
        ViewBatch<FusedPassArgs> fb;
        ViewBatch<RowJob> rb;
        SortJob rest[VIEW_BATCH];
        bool packed = false;
        fb.n = rb.n = nv;
        int maxc = 0;
        for (int v = 0; v < nv; v++) {
            const TileSortJob& j = jobs[v0 + v];
            FusedPassArgs& a = fb.v[v];
            a.P = j.P;
            a.L = j.L;
            a.nchunks = (j.P + FE_RANKS - 1) / FE_RANKS;
            a.sorted_ids = j.sorted_ids;
            a.offsets = j.offsets;
            a.sorted_rects = j.sorted_rects;
            a.rec_start = j.rec_start;
            a.counts = reinterpret_cast<uint32_t*>(j.pass1_scratch);
            a.totals = reinterpret_cast<uint32_t*>(j.pass1_scratch +
                                                   align_up((size_t)a.nchunks * RS_MAXBINS * 4 + 256, 256));
            // the fused pass writes (k1, v1), so that the later passes ping-pong k0 <- k1 <- k0 ...
            a.keys_out = npass > 1 ? j.k1 : nullptr;
            a.vals_out = npass > 1 ? reinterpret_cast<uint2*>(j.v1) : nullptr;
            // two passes and no tile ids wanted (the ranges come from the rects' difference array):
            // the second digit goes into the id word's free high bits, so the first pass writes 8
            // bytes per instance instead of 12 and the second reads 8 instead of 12
            a.pack_shift = 0;
            a.pack_w1 = w1;
            a.soa_x = a.soa_y = nullptr;
            if (GSR_TILE_PACK && npass == 2 && !j.out_tiles && (uint64_t)j.P <= (1ull << (32 - (nbits - w1)))) {
                a.pack_shift = 32 - (nbits - w1);
                a.keys_out = nullptr;
                if (GSR_TILE_SOA) {  // the v1 ping-pong region (8 B per instance) as two 4-B arrays
                    a.soa_x = j.slotless ? nullptr : j.v1;
                    a.soa_y = j.v1 + align_up(4 * (size_t)(j.L > 0 ? j.L : 0), 256) / 4;
                }
            }
            a.out_slot = j.slotless ? nullptr : j.out_slot;
            a.out_ids = j.out_ids;
            a.out_tiles = j.out_tiles;
            a.valid = j.valid;
            a.ranges = j.ranges;
            rb.v[v] = {a.counts, a.nchunks, a.totals};
            maxc = max(maxc, a.nchunks);
            rest[v] = {j.L, a.pack_shift ? nullptr : j.k1, reinterpret_cast<const uint2*>(j.v1), j.k0, j.v0, j.k1, j.v1,
                       j.out_slot, j.out_ids, j.out_tiles, j.scratch, nullptr, nullptr, nullptr};
            rest[v].key_hi_shift = a.pack_shift;
            if (a.soa_y) {  // (slotless: the id words alone, a one-word payload)
                rest[v].pairs = nullptr;
                rest[v].soa_x = a.soa_x;
                rest[v].soa_y = a.soa_y;
                if (!a.soa_x) rest[v].out_x = j.out_ids, rest[v].out_y = nullptr;
            }
            packed = a.pack_shift != 0;
        }
        if (maxc == 0) return hipSuccess;
        const dim3 g((unsigned)maxc, (unsigned)nv), b(RS_THREADS);
        if (phases & FUSED_COUNT) {
            hipLaunchKernelGGL(fused_pass1_count_kernel, g, b, 0, s, fb, gx, T, w1);
            for (int v = 0; v < nv; v++) rb.v[v].nbins = 1 << w1;
            // (the fused pass's count matrix is digit-major: thousands of 256-rank chunks)
            launch_scan_rows<TileSort>(rb, nv, 1 << w1, max(maxc, CS_CHUNKS + 1), false, s);
        }
        if (!(phases & FUSED_SCATTER)) return hipGetLastError();
        const dim3 gs((unsigned)maxc, (unsigned)nv);
        switch (w1) {  // the first pass's digit width: ceil(msb(T) / passes) -- 7 at 1080p
#define GSR_FUSED_W(W_) case W_: hipLaunchKernelGGL((fused_pass1_scatter_kernel<RS_ITEMS, W_>), gs, b, 0, s, fb, gx); break;
            GSR_FUSED_W(1) GSR_FUSED_W(2) GSR_FUSED_W(3) GSR_FUSED_W(4)
            GSR_FUSED_W(5) GSR_FUSED_W(6) GSR_FUSED_W(7) GSR_FUSED_W(8)
#undef GSR_FUSED_W
        default: return hipErrorInvalidValue;
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess || npass == 1) return e;
        // the later passes: key bits [w1, nbits), ping-pong k1/v1 -> k0/v0 -> ...
        // (packed: the second digit, already shifted down, in the id word's high bits)
        return radix_sort_batch(rest, nv, nbits - w1, s, packed ? 0 : w1, SORT_TILE);
    });
}

hipError_t radix_sort(int n, int nbits, const uint32_t* keys_in, const uint2* pairs, uint32_t* k0, uint32_t* v0,
                      uint32_t* k1, uint32_t* v1, uint32_t* out_x, uint32_t* out_y, uint32_t* sorted_keys,
                      char* scratch, hipStream_t s, const uint2* rects, uint2* sorted_rects, uint32_t* sorted_counts,
                      SortKind kind)
{
    if (n <= 0) return hipSuccess;
    const SortJob j = {n, keys_in, pairs, k0, v0, k1, v1, out_x, out_y, sorted_keys, scratch, rects, sorted_rects,
                       sorted_counts};
    return radix_sort_batch(&j, 1, nbits, s, 0, kind);
}

hipError_t launch_tile_ranges_batch(const RangesJob* jobs, int V, int T, hipStream_t s)
{
    for (int v = 0; v < V; v++) {
        if (jobs[v].L <= 0) {  // no tile sort ran to clear them
            const hipError_t e = hipMemsetAsync(jobs[v].ranges, 0, sizeof(uint2) * (size_t)T, s);
            if (e != hipSuccess) return e;
        } else if ((uintptr_t)jobs[v].sorted_tiles & 15) {
            return hipErrorInvalidValue;  // binning arrays are 256-B aligned
        }
    }
    return for_groups(V, [&](int v0, int nv) -> hipError_t {
        ViewBatch<RangesJob> B;
        B.n = nv;
        int maxl = 0;
        for (int v = 0; v < nv; v++) {
            B.v[v] = jobs[v0 + v];
            maxl = max(maxl, B.v[v].L);
        }
        if (maxl <= 0) return hipSuccess;
        const int quads = (maxl + 3) / 4;
        hipLaunchKernelGGL(tile_ranges_kernel, dim3((unsigned)((quads + 255) / 256), (unsigned)nv), dim3(256), 0, s, B);
        return hipGetLastError();
    });
}

hipError_t launch_tile_hist_batch(const TileHistJob* jobs, int V, uint32_t gx, uint32_t gy, hipStream_t s)
{
    if (!use_tile_diff(gx, gy)) return hipErrorInvalidValue;
    const size_t lds = 4 * (size_t)(gx + 1) * (gy + 1);
    return for_groups(V, [&](int v0, int nv) -> hipError_t {
        ViewBatch<TileHistJob> B;
        B.n = nv;
        int maxp = 0;
        for (int v = 0; v < nv; v++) {
            B.v[v] = jobs[v0 + v];
            maxp = max(maxp, B.v[v].P);
        }
        if (maxp <= 0) return hipSuccess;
        hipLaunchKernelGGL(tile_hist_kernel, dim3(TILE_HIST_WGS, (unsigned)nv), dim3(1024), lds, s, B, gx, gy);
        return hipGetLastError();
    });
}

// the sorted keys of a forward whose tile sort wrote no tile ids (use_tile_diff): each tile's range
// [x, y) of the sorted instances gets the tile's id
__global__ void __launch_bounds__(256) debug_keys_from_ranges_kernel(int T, const uint2* ranges, const uint32_t* point_list,
                                                                     const uint32_t* dkeys, uint64_t* keys)
{
    const int t = blockIdx.x;
    if (t >= T) return;
    const uint2 r = ranges[t];
    for (uint32_t i = r.x + threadIdx.x; i < r.y; i += 256) keys[i] = ((uint64_t)t << 32) | dkeys[point_list[i]];
}

hipError_t launch_debug_keys_from_ranges(int T, const uint2* ranges, const uint32_t* point_list, const uint32_t* dkeys,
                                         uint64_t* keys, hipStream_t s)
{
    if (T <= 0) return hipSuccess;
    hipLaunchKernelGGL(debug_keys_from_ranges_kernel, dim3((unsigned)T), dim3(256), 0, s, T, ranges, point_list, dkeys,
                       keys);
    return hipGetLastError();
}

hipError_t launch_tile_ranges(int L, const uint32_t* sorted_tiles, uint2* ranges, int T, hipStream_t s)
{
    const RangesJob j = {L, sorted_tiles, ranges};
    return launch_tile_ranges_batch(&j, 1, T, s);
}

hipError_t launch_debug_keys(int L, const uint32_t* sorted_tiles, const uint32_t* point_list, const uint32_t* dkeys,
                             uint64_t* keys, hipStream_t s)
{
    if (L <= 0) return hipSuccess;
    hipLaunchKernelGGL(debug_keys_kernel, dim3((L + 255) / 256), dim3(256), 0, s, L, sorted_tiles, point_list, dkeys,
                       keys);
    return hipGetLastError();
}

}  // namespace gsr
