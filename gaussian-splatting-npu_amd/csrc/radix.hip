// radix.hip -- stable LSD onesweep radix sort for gfx950 (replaces the reference's
// cub::DeviceRadixSort::SortPairs, rasterizer_impl.cu:303-311), and the depth-first
// binning built on it.
//
// Binning scheme (same result as the reference's 64-bit tile|depth key sort):
//   1. sort the P Gaussians by depth bits (4 x 8-bit passes; ties keep index order;
//      culled Gaussians carry key 0xFFFFFFFF and land last);
//   2. emit (tile, Gaussian) instances in that depth order (y-major, then x, inside each
//      Gaussian's rect, exactly like duplicateWithKeys, rasterizer_impl.cu:98-109);
//   3. stable-sort the instances by tile id alone: ceil(bit/8) passes of 8 bits (2 at 1080p)
//      instead of the reference's ceil((32+bit)/8) passes over 12-byte pairs.
// Because both sorts are stable, every tile's list comes out ordered by (depth bits,
// Gaussian index) -- the reference's order -- and the sorted key array
// (tile << 32 | depth bits) is bit-identical to the reference's.
//
// One pass = one kernel: each 256-thread workgroup takes the next 4096-element chunk
// (atomic ticket, so chunk c-1 is always already running), ranks its elements stably per
// 8-bit digit (wave-level ballot match + per-wave running counters in LDS), publishes its
// per-digit counts and resolves its global offsets by decoupled look-back over the
// previous chunks' status words (64-bit {flag, count} granules, relaxed agent-scope
// atomics: the data is the flag), then scatters through LDS so that global writes are
// contiguous runs per digit.
#include "gsr_common.h"
#include "gsr_kernels.h"

namespace gsr {

constexpr int RS_THREADS = 256;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;  // 4096 elements per chunk
constexpr int RS_BINS = 256;
constexpr uint64_t ST_AGG = 1ull << 62, ST_INC = 2ull << 62, ST_MASK = 3ull << 62;
constexpr uint32_t SPIN_LIMIT = 1u << 22;

__device__ __forceinline__ uint64_t ld_status(const uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Histograms of every 8-bit digit pass at once: hist[p * 256 + d].
__global__ void __launch_bounds__(RS_THREADS) radix_histogram_kernel(const uint32_t* keys, int n, int npass,
                                                                    uint32_t* hist)
{
    __shared__ uint32_t h[4][RS_BINS];
    for (int p = 0; p < 4; p++) h[p][threadIdx.x] = 0;
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * RS_THREADS + threadIdx.x; i < (size_t)n; i += (size_t)gridDim.x * RS_THREADS) {
        const uint32_t k = keys[i];
        for (int p = 0; p < npass; p++) atomicAdd(&h[p][(k >> (8 * p)) & 255u], 1u);
    }
    __syncthreads();
    for (int p = 0; p < npass; p++) {
        const uint32_t c = h[p][threadIdx.x];
        if (c) atomicAdd(&hist[p * RS_BINS + threadIdx.x], c);
    }
}

// In-place exclusive scan of each pass's 256-bin histogram (one block, thread = bin).
__global__ void __launch_bounds__(RS_THREADS) radix_digit_scan_kernel(uint32_t* hist, int npass)
{
    __shared__ uint32_t s[RS_BINS];
    for (int p = 0; p < npass; p++) {
        const uint32_t v = hist[p * RS_BINS + threadIdx.x];
        s[threadIdx.x] = v;
        __syncthreads();
        for (int d = 1; d < RS_BINS; d <<= 1) {
            const uint32_t a = threadIdx.x >= (unsigned)d ? s[threadIdx.x - d] : 0u;
            __syncthreads();
            s[threadIdx.x] += a;
            __syncthreads();
        }
        hist[p * RS_BINS + threadIdx.x] = s[threadIdx.x] - v;
        __syncthreads();
    }
}

struct OnesweepArgs {
    int n;
    int shift;
    const uint32_t* keys_in;
    const uint2* vals_in;       // payload in (null: synthesise {vals32_in[i] or i, i})
    const uint32_t* vals32_in;  // optional first-pass payload .x
    uint32_t* keys_out;
    uint2* vals_out;
    // final tile-sort mode (vals_out == null): point_list[dst] = v.x, inv[v.y] = dst, tiles[dst] = key
    uint32_t* point_list;
    uint32_t* inv;
    uint32_t* sorted_keys;
    const uint32_t* digit_offsets;  // exclusive digit offsets of this pass (256)
    uint64_t* status;               // nchunks * 256 zeroed granules
    uint32_t* ticket;               // zeroed chunk counter
    uint32_t* error;                // set to 1 if a look-back spin gives up
};

__global__ void __launch_bounds__(RS_THREADS) onesweep_kernel(OnesweepArgs a)
{
    __shared__ uint32_t s_cnt[4][RS_BINS];  // per-wave running digit counts, then per-wave prefixes
    __shared__ uint32_t s_blk[RS_BINS];     // block-local start of each digit
    __shared__ uint32_t s_base[RS_BINS];    // global start of each digit for this chunk
    __shared__ uint32_t s_keys[RS_TILE];
    __shared__ uint2 s_vals[RS_TILE];
    __shared__ uint32_t s_chunk;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_chunk = atomicAdd(a.ticket, 1u);
    for (int q = 0; q < 4; q++) s_cnt[q][tid] = 0;
    __syncthreads();
    const uint32_t chunk = s_chunk;
    const size_t base = (size_t)chunk * RS_TILE;
    const int nvalid = (int)min((size_t)RS_TILE, (size_t)a.n - base);

    uint32_t key[RS_ITEMS];
    uint2 val[RS_ITEMS];
    uint32_t rank[RS_ITEMS];
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int i = 0; i < RS_ITEMS; i++) {
        const int li = w * (RS_ITEMS * 64) + i * 64 + lane;  // chunk-local index; order = (wave, item, lane)
        const bool valid = li < nvalid;
        const size_t gi = base + li;
        key[i] = valid ? a.keys_in[gi] : 0u;
        if (a.vals_in) val[i] = valid ? a.vals_in[gi] : make_uint2(0u, 0u);
        else val[i] = make_uint2(valid ? (a.vals32_in ? a.vals32_in[gi] : (uint32_t)gi) : 0u, (uint32_t)gi);
        const uint32_t d = (key[i] >> a.shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
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
    const uint32_t c0 = s_cnt[0][tid], c1 = s_cnt[1][tid], c2 = s_cnt[2][tid], c3 = s_cnt[3][tid];
    const uint32_t total = c0 + c1 + c2 + c3;
    s_cnt[0][tid] = 0;
    s_cnt[1][tid] = c0;
    s_cnt[2][tid] = c0 + c1;
    s_cnt[3][tid] = c0 + c1 + c2;
    // publish this chunk's aggregate for digit tid as early as possible
    uint64_t* st = a.status + (size_t)chunk * RS_BINS + tid;
    if (chunk == 0) st_status(st, ST_INC | total);
    else st_status(st, ST_AGG | total);
    // block-local exclusive scan of totals over digits
    s_blk[tid] = total;
    __syncthreads();
    for (int d = 1; d < RS_BINS; d <<= 1) {
        const uint32_t v = tid >= d ? s_blk[tid - d] : 0u;
        __syncthreads();
        s_blk[tid] += v;
        __syncthreads();
    }
    const uint32_t blk_start = s_blk[tid] - total;
    // decoupled look-back for digit tid
    uint32_t prefix = 0;
    if (chunk > 0) {
        int j = (int)chunk - 1;
        while (j >= 0) {
            const uint64_t* sp = a.status + (size_t)j * RS_BINS + tid;
            uint64_t s = ld_status(sp);
            uint32_t spins = 0;
            while ((s & ST_MASK) == 0ull && ++spins < SPIN_LIMIT) {
                __builtin_amdgcn_s_sleep(1);
                s = ld_status(sp);
            }
            if ((s & ST_MASK) == 0ull) {
                atomicOr(a.error, 1u);
                break;
            }
            prefix += (uint32_t)s;
            if ((s & ST_MASK) == ST_INC) break;
            j--;
        }
        st_status(st, ST_INC | (prefix + total));
    }
    __syncthreads();
    s_blk[tid] = blk_start;
    s_base[tid] = a.digit_offsets[tid] + prefix;
    __syncthreads();

    // scatter into LDS in block-local sorted (stable) order
#pragma unroll
    for (int i = 0; i < RS_ITEMS; i++) {
        if (rank[i] != 0xFFFFFFFFu) {
            const uint32_t d = (key[i] >> a.shift) & 255u;
            const uint32_t lpos = s_blk[d] + s_cnt[w][d] + rank[i];
            s_keys[lpos] = key[i];
            s_vals[lpos] = val[i];
        }
    }
    __syncthreads();
    // contiguous write-out: runs of one digit map to consecutive global addresses
#pragma unroll
    for (int i = 0; i < RS_ITEMS; i++) {
        const int lpos = i * RS_THREADS + tid;
        if (lpos < nvalid) {
            const uint32_t k = s_keys[lpos];
            const uint32_t d = (k >> a.shift) & 255u;
            const uint32_t dst = s_base[d] + ((uint32_t)lpos - s_blk[d]);
            const uint2 v = s_vals[lpos];
            if (a.vals_out) {
                a.keys_out[dst] = k;
                a.vals_out[dst] = v;
            } else {
                if (a.point_list) a.point_list[dst] = v.x;
                if (a.inv) a.inv[v.y] = dst;
                if (a.sorted_keys) a.sorted_keys[dst] = k;
            }
        }
    }
}

// Emission in depth order: instance slots [off(k-1), off(k)) of depth rank k belong to
// Gaussian g = sorted_ids[k]; tiles y-major then x inside its rect (rasterizer_impl.cu:98-109).
__global__ void __launch_bounds__(256) emit_instances_kernel(int P, const uint32_t* sorted_ids,
                                                             const uint32_t* offsets_d, const float2* means2D,
                                                             const int* radii, uint32_t gx, uint32_t gy,
                                                             uint32_t* tile_keys, uint32_t* gids,
                                                             uint32_t* emit_start)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P) return;
    const uint32_t g = sorted_ids[k];
    const int r = radii[g];
    uint32_t off = k == 0 ? 0u : offsets_d[k - 1];
    emit_start[g] = off;
    if (r <= 0) return;
    const float2 xy = means2D[g];
    uint32_t rminx, rminy, rmaxx, rmaxy;
    getRect(xy.x, xy.y, r, gx, gy, rminx, rminy, rmaxx, rmaxy);
    for (uint32_t y = rminy; y < rmaxy; y++)
        for (uint32_t x = rminx; x < rmaxx; x++) {
            tile_keys[off] = y * gx + x;
            gids[off] = g;
            off++;
        }
}

__global__ void __launch_bounds__(256) tile_ranges_kernel(int L, const uint32_t* sorted_tiles, uint2* ranges)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= L) return;
    const uint32_t cur = sorted_tiles[idx];
    if (idx == 0) ranges[cur].x = 0;
    else {
        const uint32_t prev = sorted_tiles[idx - 1];
        if (cur != prev) {
            ranges[prev].y = idx;
            ranges[cur].x = idx;
        }
    }
    if (idx == L - 1) ranges[cur].y = L;
}

__global__ void __launch_bounds__(256) debug_keys_kernel(int L, const uint32_t* sorted_tiles, const uint32_t* point_list,
                                                         const float* depths, uint64_t* keys)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= L) return;
    keys[idx] = ((uint64_t)sorted_tiles[idx] << 32) | __float_as_uint(depths[point_list[idx]]);
}

size_t radix_status_bytes(int n, int npass)
{
    const size_t chunks = ((size_t)(n > 0 ? n : 0) + RS_TILE - 1) / RS_TILE;
    return align_up((size_t)npass * (chunks * RS_BINS * 8 + 256) + (size_t)npass * RS_BINS * 4 + 256, 256);
}

// Full LSD sort of n (key, payload) pairs over `npass` 8-bit digits starting at bit 0.
// scratch: radix_status_bytes(n, npass) bytes.  Ping-pongs between (k0,v0) and (k1,v1);
// the last pass either writes (keys_final, vals_final) or the final tile outputs.
hipError_t radix_sort(int n, int npass, const uint32_t* keys_in, const uint32_t* vals32_in, uint32_t* k0, uint2* v0,
                      uint32_t* k1, uint2* v1, uint32_t* keys_final, uint2* vals_final, uint32_t* point_list,
                      uint32_t* inv, uint32_t* sorted_keys, char* scratch, uint32_t* error, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    const size_t chunks = ((size_t)n + RS_TILE - 1) / RS_TILE;
    const size_t per_pass = chunks * RS_BINS * 8 + 256;
    uint32_t* hist = reinterpret_cast<uint32_t*>(scratch + (size_t)npass * per_pass);
    hipError_t e = hipMemsetAsync(scratch, 0, radix_status_bytes(n, npass), s);
    if (e != hipSuccess) return e;
    const int hgrid = (int)min((size_t)1024, (size_t)(n + RS_THREADS - 1) / RS_THREADS);
    hipLaunchKernelGGL(radix_histogram_kernel, dim3(hgrid), dim3(RS_THREADS), 0, s, keys_in, n, npass, hist);
    hipLaunchKernelGGL(radix_digit_scan_kernel, dim3(1), dim3(RS_THREADS), 0, s, hist, npass);
    const uint32_t* kin = keys_in;
    const uint2* vin = nullptr;
    for (int p = 0; p < npass; p++) {
        const bool last = p == npass - 1;
        OnesweepArgs a;
        a.n = n;
        a.shift = 8 * p;
        a.keys_in = kin;
        a.vals_in = vin;
        a.vals32_in = p == 0 ? vals32_in : nullptr;
        uint32_t* ko = (p & 1) ? k1 : k0;
        uint2* vo = (p & 1) ? v1 : v0;
        if (last) {
            ko = keys_final;
            vo = vals_final;
        }
        a.keys_out = ko;
        a.vals_out = vo;
        a.point_list = point_list;
        a.inv = inv;
        a.sorted_keys = sorted_keys;
        a.digit_offsets = hist + p * RS_BINS;
        char* pass_base = scratch + (size_t)p * per_pass;
        a.status = reinterpret_cast<uint64_t*>(pass_base + 256);
        a.ticket = reinterpret_cast<uint32_t*>(pass_base);
        a.error = error;
        hipLaunchKernelGGL(onesweep_kernel, dim3((unsigned)chunks), dim3(RS_THREADS), 0, s, a);
        kin = ko;
        vin = vo;
    }
    return hipGetLastError();
}

hipError_t launch_emit_instances(int P, const uint32_t* sorted_ids, const uint32_t* offsets_d, const float2* means2D,
                                 const int* radii, uint32_t gx, uint32_t gy, uint32_t* tile_keys, uint32_t* gids,
                                 uint32_t* emit_start, hipStream_t s)
{
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(emit_instances_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, sorted_ids, offsets_d,
                       means2D, radii, gx, gy, tile_keys, gids, emit_start);
    return hipGetLastError();
}

hipError_t launch_tile_ranges(int L, const uint32_t* sorted_tiles, uint2* ranges, int T, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(ranges, 0, sizeof(uint2) * (size_t)T, s);
    if (e != hipSuccess || L <= 0) return e;
    hipLaunchKernelGGL(tile_ranges_kernel, dim3((L + 255) / 256), dim3(256), 0, s, L, sorted_tiles, ranges);
    return hipGetLastError();
}

hipError_t launch_debug_keys(int L, const uint32_t* sorted_tiles, const uint32_t* point_list, const float* depths,
                             uint64_t* keys, hipStream_t s)
{
    if (L <= 0) return hipSuccess;
    hipLaunchKernelGGL(debug_keys_kernel, dim3((L + 255) / 256), dim3(256), 0, s, L, sorted_tiles, point_list, depths,
                       keys);
    return hipGetLastError();
}

}  // namespace gsr
