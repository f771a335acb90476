// binning.hip -- tile|depth key emission (duplicateWithKeys,
// rasterizer_impl.cu:70-111), stable key/value sort on bits [0, 32+bit)
// (cub::DeviceRadixSort::SortPairs, rasterizer_impl.cu:303-311) and tile range
// identification (identifyTileRanges, rasterizer_impl.cu:116-138) for gfx950.
#include <hipcub/hipcub.hpp>

#include "gsr_common.h"
#include "gsr_kernels.h"

namespace gsr {

// One thread per Gaussian; keys y-major then x within the rect, exactly the
// reference emission order (rasterizer_impl.cu:98-109).
__global__ void __launch_bounds__(256) duplicate_with_keys_kernel(int P, const float2* means2D, const float* depths,
                                                                  const uint32_t* offsets, const int* radii,
                                                                  uint32_t gx, uint32_t gy, uint64_t* keys,
                                                                  uint32_t* emit_gid, uint32_t* emit_e)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const int r = radii[idx];
    if (r <= 0) return;
    uint32_t off = idx == 0 ? 0 : offsets[idx - 1];
    const float2 xy = means2D[idx];
    uint32_t rminx, rminy, rmaxx, rmaxy;
    getRect(xy.x, xy.y, r, gx, gy, rminx, rminy, rmaxx, rmaxy);
    const uint32_t dbits = __float_as_uint(depths[idx]);
    for (uint32_t y = rminy; y < rmaxy; y++)
        for (uint32_t x = rminx; x < rmaxx; x++) {
            keys[off] = ((uint64_t)(y * gx + x) << 32) | dbits;
            emit_gid[off] = (uint32_t)idx;
            emit_e[off] = off;
            off++;
        }
}

// After the sort: point_list[pos] = Gaussian of the sorted entry, inv[e] = pos (the
// emission-slot -> sorted-position map the deterministic backward gathers through),
// and the tile ranges of identifyTileRanges (rasterizer_impl.cu:116-138).
__global__ void __launch_bounds__(256) finalize_kernel(int L, const uint64_t* keys, const uint32_t* sorted_e,
                                                       const uint32_t* emit_gid, uint32_t* point_list, uint32_t* inv,
                                                       uint2* ranges)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= L) return;
    const uint32_t e = sorted_e[idx];
    point_list[idx] = emit_gid[e];
    inv[e] = (uint32_t)idx;
    const uint32_t currtile = (uint32_t)(keys[idx] >> 32);
    if (idx == 0) ranges[currtile].x = 0;
    else {
        const uint32_t prevtile = (uint32_t)(keys[idx - 1] >> 32);
        if (currtile != prevtile) {
            ranges[prevtile].y = idx;
            ranges[currtile].x = idx;
        }
    }
    if (idx == L - 1) ranges[currtile].y = L;
}

size_t sort_scratch_bytes(int L)
{
    size_t bytes = 0;
    if (L <= 0) return 256;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, L, 0, 64, (hipStream_t)0);
    return bytes + 256;
}

hipError_t launch_duplicate_with_keys(int P, const float2* means2D, const float* depths, const uint32_t* offsets,
                                      const int* radii, uint32_t gx, uint32_t gy, uint64_t* keys, uint32_t* emit_gid,
                                      uint32_t* emit_e, hipStream_t s)
{
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(duplicate_with_keys_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, means2D, depths,
                       offsets, radii, gx, gy, keys, emit_gid, emit_e);
    return hipGetLastError();
}

hipError_t launch_sort_pairs(void* scratch, size_t scratch_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                             const uint32_t* vals_in, uint32_t* vals_out, int n, int end_bit, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    size_t bytes = scratch_bytes;
    return hipcub::DeviceRadixSort::SortPairs(scratch, bytes, keys_in, keys_out, vals_in, vals_out, n, 0, end_bit,
                                              s);
}

hipError_t launch_finalize(int L, const uint64_t* keys, const uint32_t* sorted_e, const uint32_t* emit_gid,
                           uint32_t* point_list, uint32_t* inv, uint2* ranges, int T, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(ranges, 0, sizeof(uint2) * (size_t)T, s);
    if (e != hipSuccess || L <= 0) return e;
    hipLaunchKernelGGL(finalize_kernel, dim3((L + 255) / 256), dim3(256), 0, s, L, keys, sorted_e, emit_gid,
                       point_list, inv, ranges);
    return hipGetLastError();
}

}  // namespace gsr
