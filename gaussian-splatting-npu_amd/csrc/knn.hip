// knn.hip -- distCUDA2 (simple-knn, the reference's un-vendored submodule; call site
// scene/gaussian_model.py:159-160) for gfx950: per point, the mean squared distance to its
// 3 nearest other points.  Exact 3-NN over a uniform grid instead of simple-knn's Morton
// boxes of 1024 points scanned by every query:
//   1. bounds (per-workgroup partials folded by one workgroup into mapped host words), read on
//      the host to size the grid (~2 points/cell);
//   2. cell id per point; stable radix sort of (cell, index) with the rasterizer's own sort;
//   3. points gathered into cell order (16-B rows), cell ranges;
//   4. one thread per point (in cell order, so a wave's queries share cells in L1/L2) visits
//      cells in Chebyshev shells of growing radius r and stops once its third-best squared
//      distance is below the squared lower bound r*h of every unvisited cell.
// The squared distance is d.x*d.x + d.y*d.y + d.z*d.z contracted as nvcc contracts the
// reference's updateKBest (fma(dz, dz, fma(dy, dy, dx*dx))); the three best are kept in
// ascending order and combined as (b0 + b1 + b2) / 3 with FLT_MAX for missing neighbours,
// as the reference does.  oracle/knn_oracle.c restates the same definition (brute force).
#include "gsr_common.h"
#include "gsr_kernels.h"

#include <float.h>
#include <string.h>

#include <cmath>

namespace gsr {

__device__ __forceinline__ uint32_t f2ord(float f)
{
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

constexpr int KNN_BOUNDS_BLOCKS = 256;

// Per-workgroup min/max of the three coordinates (no atomics: 24k same-address atomics from every
// wave cost ~0.28 ms at P = 1M), then one workgroup folds the partials and stores the six
// ordered words straight into the caller's mapped host page (no memset, no D2H copy).
__global__ void __launch_bounds__(256) knn_bounds_kernel(int P, const float* pts, float* partial)
{
    __shared__ float red[6][4];
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = blockIdx.x * 256 + (int)threadIdx.x; i < P; i += gridDim.x * 256) {
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const float v = pts[3 * (size_t)i + a];
            mn[a] = fminf(mn[a], v);
            mx[a] = fmaxf(mx[a], v);
        }
    }
#pragma unroll
    for (int a = 0; a < 3; a++) {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], d, 64));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], d, 64));
        }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int a = 0; a < 3; a++) {
            red[a][w] = mn[a];
            red[3 + a][w] = mx[a];
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        float v = red[k][0];
        for (int j = 1; j < 4; j++) v = k < 3 ? fminf(v, red[k][j]) : fmaxf(v, red[k][j]);
        partial[blockIdx.x * 8 + k] = v;
    }
}

__global__ void __launch_bounds__(64) knn_bounds_final_kernel(int nblocks, const float* partial, uint32_t* host_out)
{
    const int k = threadIdx.x & 7;
    if (k >= 6) return;
    float v = k < 3 ? FLT_MAX : -FLT_MAX;
    for (int b = threadIdx.x >> 3; b < nblocks; b += 8) {
        const float x = partial[b * 8 + k];
        v = k < 3 ? fminf(v, x) : fmaxf(v, x);
    }
#pragma unroll
    for (int d = 8; d <= 32; d <<= 1) {
        const float o = __shfl_xor(v, d, 64);
        v = k < 3 ? fminf(v, o) : fmaxf(v, o);
    }
    if (threadIdx.x < 6)
        __hip_atomic_store(host_out + k, f2ord(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct KnnGrid {
    float ox, oy, oz, inv_h, h;
    float tol;  // absolute slack for rounding of cell coordinates (a few ulps of the coordinates)
    int nx, ny, nz;
};

__device__ __forceinline__ int cell_coord(float v, float o, float inv_h, int n)
{
    const int c = (int)floorf((v - o) * inv_h);
    return min(max(c, 0), n - 1);
}

__global__ void __launch_bounds__(256) knn_cell_kernel(int P, const float* pts, KnnGrid g, uint32_t* cells)
{
    const int i = blockIdx.x * 256 + (int)threadIdx.x;
    if (i >= P) return;
    const float x = pts[3 * (size_t)i], y = pts[3 * (size_t)i + 1], z = pts[3 * (size_t)i + 2];
    const int cx = cell_coord(x, g.ox, g.inv_h, g.nx), cy = cell_coord(y, g.oy, g.inv_h, g.ny),
              cz = cell_coord(z, g.oz, g.inv_h, g.nz);
    cells[i] = ((uint32_t)cz * (uint32_t)g.ny + (uint32_t)cy) * (uint32_t)g.nx + (uint32_t)cx;
}

__global__ void __launch_bounds__(256) knn_gather_kernel(int P, const float* pts, const uint32_t* sorted_idx,
                                                         const uint32_t* sorted_cells, float4* spts, uint2* cell_range)
{
    const int k = blockIdx.x * 256 + (int)threadIdx.x;
    if (k >= P) return;
    const uint32_t i = sorted_idx[k];
    spts[k] = make_float4(pts[3 * (size_t)i], pts[3 * (size_t)i + 1], pts[3 * (size_t)i + 2], 0.f);
    const uint32_t c = sorted_cells[k];
    if (k == 0 || sorted_cells[k - 1] != c) cell_range[c].x = (uint32_t)k;
    if (k == P - 1 || sorted_cells[k + 1] != c) cell_range[c].y = (uint32_t)k + 1;
}

// updateKBest<3> of simple-knn: insertion into the ascending best list.
__device__ __forceinline__ void update3(float (&b)[3], float d)
{
#pragma unroll
    for (int j = 0; j < 3; j++) {
        if (b[j] > d) {
            const float t = b[j];
            b[j] = d;
            d = t;
        }
    }
}

__global__ void __launch_bounds__(256) knn_query_kernel(int P, const float4* spts, const uint32_t* sorted_idx,
                                                        const uint32_t* sorted_cells, const uint2* cell_range,
                                                        KnnGrid g, float* dist2)
{
    const int k = blockIdx.x * 256 + (int)threadIdx.x;
    if (k >= P) return;
    const float4 q = spts[k];
    const uint32_t c = sorted_cells[k];
    const int cx = (int)(c % (uint32_t)g.nx), cy = (int)((c / (uint32_t)g.nx) % (uint32_t)g.ny),
              cz = (int)(c / ((uint32_t)g.nx * (uint32_t)g.ny));
    float b[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    // q's offsets inside its own cell, for the squared distance from q to another cell's box
    const float fx = q.x - (g.ox + (float)cx * g.h), fy = q.y - (g.oy + (float)cy * g.h),
                fz = q.z - (g.oz + (float)cz * g.h);
    auto axis_gap = [&](int d, float f) {  // distance along one axis to a cell d cells away
        return d > 0 ? fmaxf(0.f, (float)d * g.h - f - g.tol)
                     : (d < 0 ? fmaxf(0.f, f - (float)(d + 1) * g.h - g.tol) : 0.f);
    };
    auto scan_cell = [&](int x, int y, int z) {
        // Skip a cell whose box lies farther than the current third-best.  The gaps are shrunk by
        // tol (rounding of q's offset and of the box corners); clamped boundary cells only ever
        // make a box nearer than it is.
        const float gx = axis_gap(x - cx, fx), gy = axis_gap(y - cy, fy), gz = axis_gap(z - cz, fz);
        if ((gx * gx + gy * gy + gz * gz) * (1.0f - 1e-5f) > b[2]) return;
        const uint2 r = cell_range[((uint32_t)z * (uint32_t)g.ny + (uint32_t)y) * (uint32_t)g.nx + (uint32_t)x];
        for (uint32_t j = r.x; j < r.y; j++) {
            if ((int)j == k) continue;
            const float4 p = spts[j];
            const float dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;
            update3(b, __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx)));
        }
    };
    const int rmax = max(max(g.nx, g.ny), g.nz);
    for (int r = 0; r <= rmax; r++) {
        const int z0 = max(cz - r, 0), z1 = min(cz + r, g.nz - 1);
        const int y0 = max(cy - r, 0), y1 = min(cy + r, g.ny - 1);
        const int x0 = max(cx - r, 0), x1 = min(cx + r, g.nx - 1);
        for (int z = z0; z <= z1; z++) {
            const bool zface = z == cz - r || z == cz + r;
            for (int y = y0; y <= y1; y++) {
                if (zface || y == cy - r || y == cy + r) {
                    for (int x = x0; x <= x1; x++) scan_cell(x, y, z);
                } else {  // interior row of the shell: only its two end cells
                    if (cx - r >= 0) scan_cell(cx - r, y, z);
                    if (r > 0 && cx + r < g.nx) scan_cell(cx + r, y, z);
                }
            }
        }
        // Every unvisited point lies in a cell at Chebyshev distance > r, hence farther than
        // r * h from q (q lies in its own cell; a small margin covers rounding and clamping).
        const float lb = fmaxf(0.f, (float)r * g.h - g.tol);
        if (b[2] <= lb * lb * (1.0f - 1e-5f)) break;
    }
    dist2[sorted_idx[k]] = (b[0] + b[1] + b[2]) / 3.0f;
}

namespace {
struct KnnLayout {
    size_t off[10];
};
// cells, k0, v0, k1, v1, sorted_idx, sorted_cells, spts (float4), cell_range (uint2), radix scratch + bounds
KnnLayout knn_layout(int P)
{
    const size_t p = (size_t)(P > 0 ? P : 0);
    const size_t maxcells = 2 * p + 64;
    const size_t sizes[9] = {4 * p, 4 * p, 4 * p, 4 * p, 4 * p, 4 * p, 4 * p, 16 * p, 8 * maxcells};
    KnnLayout l;
    size_t o = 0;
    for (int i = 0; i < 9; i++) {
        l.off[i] = o;
        o = align_up(o + sizes[i], 256);
    }
    l.off[9] = o;  // radix scratch, then 64 B of bounds
    return l;
}
}  // namespace

size_t knn_workspace_bytes(int P)
{
    const KnnLayout l = knn_layout(P);
    return l.off[9] + align_up(radix_status_bytes(P, 4), 256) + 32 * KNN_BOUNDS_BLOCKS;
}

// Host: bounds -> grid of ~P/2 cells (at most 2P + 64), then sort, gather, query.
hipError_t knn_dist2(int P, const float* pts, float* dist2, char* ws, uint32_t* host_bounds, hipStream_t s)
{
    if (P <= 0) return hipSuccess;
    const KnnLayout l = knn_layout(P);
    auto at32 = [&](int i) { return reinterpret_cast<uint32_t*>(ws + l.off[i]); };
    float* partial = reinterpret_cast<float*>(ws + l.off[9] + align_up(radix_status_bytes(P, 4), 256));
    uint32_t* bounds_dev = nullptr;
    hipError_t e;
    if ((e = hipHostGetDevicePointer((void**)&bounds_dev, host_bounds, 0)) != hipSuccess) return e;
    const int nb = min((P + 255) / 256, KNN_BOUNDS_BLOCKS);
    hipLaunchKernelGGL(knn_bounds_kernel, dim3(nb), dim3(256), 0, s, P, pts, partial);
    hipLaunchKernelGGL(knn_bounds_final_kernel, dim3(1), dim3(64), 0, s, nb, partial, bounds_dev);
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    float lo[3], hi[3];
    for (int a = 0; a < 3; a++) {
        uint32_t m = host_bounds[a], M = host_bounds[3 + a];
        m = (m & 0x80000000u) ? (m & 0x7FFFFFFFu) : ~m;
        M = (M & 0x80000000u) ? (M & 0x7FFFFFFFu) : ~M;
        memcpy(&lo[a], &m, 4);
        memcpy(&hi[a], &M, 4);
    }
    double ext[3], emax = 0.0;
    for (int a = 0; a < 3; a++) {
        ext[a] = (double)hi[a] - (double)lo[a];
        emax = ext[a] > emax ? ext[a] : emax;
    }
    KnnGrid g;
    const double target = P / 2.0 > 1.0 ? P / 2.0 : 1.0;
    double h;
    if (!(emax > 0.0) || !std::isfinite(emax)) {
        h = 1.0;  // all points coincide (or non-finite input): one cell
    } else {
        const double floor_ext = emax * 1e-3;  // flat clouds: thin axes count as 1/1000 of the widest
        double vol = 1.0;
        for (int a = 0; a < 3; a++) vol *= ext[a] > floor_ext ? ext[a] : floor_ext;
        h = cbrt(vol / target);
    }
    int n[3];
    for (;;) {  // at most 2P + 64 cells
        size_t cells = 1;
        for (int a = 0; a < 3; a++) {
            const double c = std::isfinite(ext[a] / h) ? ceil(ext[a] / h) : 1.0;
            n[a] = (int)(c < 1.0 ? 1.0 : (c > 1024.0 ? 1024.0 : c));
            cells *= (size_t)n[a];
        }
        if (cells <= 2 * (size_t)P + 64) break;
        h *= 1.25;
    }
    g.ox = lo[0]; g.oy = lo[1]; g.oz = lo[2];
    g.h = (float)h;
    g.inv_h = (float)(1.0 / h);
    double amax = 0.0;
    for (int a = 0; a < 3; a++) amax = fmax(amax, fmax(fabs((double)lo[a]), fabs((double)hi[a])));
    g.tol = (float)(16.0 * FLT_EPSILON * (amax + h));
    g.nx = n[0]; g.ny = n[1]; g.nz = n[2];
    const uint32_t ncells = (uint32_t)n[0] * (uint32_t)n[1] * (uint32_t)n[2];

    const dim3 grid((P + 255) / 256), blk(256);
    hipLaunchKernelGGL(knn_cell_kernel, grid, blk, 0, s, P, pts, g, at32(0));
    const int nbits = (int)higher_msb(ncells);  // as the reference sizes its tile sort
    if ((e = radix_sort(P, nbits, at32(0), nullptr, at32(1), at32(2), at32(3), at32(4), at32(5), nullptr, at32(6),
                        ws + l.off[9], s, nullptr, nullptr, nullptr, SORT_CELLS)) != hipSuccess)
        return e;
    uint2* cell_range = reinterpret_cast<uint2*>(ws + l.off[8]);
    if ((e = hipMemsetAsync(cell_range, 0, 8 * (size_t)ncells, s)) != hipSuccess) return e;
    float4* spts = reinterpret_cast<float4*>(ws + l.off[7]);
    hipLaunchKernelGGL(knn_gather_kernel, grid, blk, 0, s, P, pts, at32(5), at32(6), spts, cell_range);
    hipLaunchKernelGGL(knn_query_kernel, grid, blk, 0, s, P, spts, at32(5), at32(6), cell_range, g, dist2);
    return hipGetLastError();
}

}  // namespace gsr
