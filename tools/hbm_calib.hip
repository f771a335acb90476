// HBM-counter calibration: kernels with known access patterns and byte
// counts, so that rocprofv3's FETCH_SIZE / WRITE_SIZE (and the TCC_EA0 request counters behind
// them) can be read as bytes for the access shapes the rasterizer actually has:
//   stream_read    16 B/lane coalesced reads of a 2 GiB buffer (MI355X_MICROARCH.md: FETCH_SIZE = 1/2)
//   stream_write   16 B/lane coalesced stores
//   gather48       one random 48-B record per lane (three 16-B loads) from a 1.5 GiB table
//                  (render_bwd / preprocess_bwd records, render_fwd's SPLAT records)
//   gather4        one random 4-B word per lane from a 1 GiB table (ids, record starts)
//   scatter12      one 12-B element per lane to a random slot (the radix scatter at worst)
//   scatter12_runs 12-B elements in runs of 8 consecutive slots, the runs at random places (the
//                  radix scatter's digit runs through LDS)
//   gather48_lds   as gather48 but the 48-B records land in LDS by one 16-B DMA per lane-quarter
// Every table is far larger than the 256 MiB Infinity Cache.  The host prints, per kernel, the
// algorithmic bytes and the distinct 32 / 64 / 128-B units the access touches (exact, from the same
// index function), one JSON object per line.  Run under rocprofv3 --pmc (tools/hbm_calib.sh).
//
// Test infrastructure, not product code.  Build: hipcc --offload-arch=gfx950 -O3 -o hbm_calib hbm_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));             \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

// a bijection on [0, 2^k): odd multiplier, xor-shift, masked (the mask keeps it on [0, 2^k))
__host__ __device__ inline uint32_t perm(uint32_t i, uint32_t mask) {
    uint32_t x = (i * 2654435761u) & mask;
    x ^= (x >> 7) & mask;  // xor with a right shift of itself: invertible on k bits
    return (x * 0x9E3779B1u) & mask;
}

__global__ void stream_read(const float4* __restrict__ a, size_t n4, float* __restrict__ out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 123.456f) out[0] = s;  // never true on the zero-filled buffer: keeps the loads alive
}

__global__ void stream_write(float4* __restrict__ a, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

__global__ void gather48(const float4* __restrict__ table, uint32_t mask, uint32_t n, float* __restrict__ out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t r = perm(i, mask);
    const float4* p = table + 3 * (size_t)r;
    float4 a = p[0], b = p[1], c = p[2];
    float s = a.x + b.y + c.z + a.w + b.w + c.w;
    if (s == 123.456f) out[i] = s;
}

__global__ void gather4(const uint32_t* __restrict__ table, uint32_t mask, uint32_t n, uint32_t* __restrict__ out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t v = table[perm(i, mask)];
    if (v == 0xDEADBEEFu) out[i] = v;
}

__global__ void scatter12(uint32_t* __restrict__ out, uint32_t mask, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t* p = out + 3 * (size_t)perm(i, mask);
    p[0] = i;
    p[1] = i ^ 1u;
    p[2] = i ^ 2u;
}

__global__ void scatter12_runs(uint32_t* __restrict__ out, uint32_t run_mask, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    size_t slot = (size_t)perm(i >> 3, run_mask) * 8 + (i & 7u);
    uint32_t* p = out + 3 * slot;
    p[0] = i;
    p[1] = i ^ 1u;
    p[2] = i ^ 2u;
}

// random 48-B records into LDS: lanes 4j..4j+2 of a wave each DMA one 16-B quarter of record j
// (the fourth lane of each group idles); 16 records per wave-instruction
__global__ void __launch_bounds__(256) gather48_lds(const float4* __restrict__ table, uint32_t mask, uint32_t n,
                                                    float* __restrict__ out) {
    __shared__ float4 lds[256];
    uint32_t rec = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    uint32_t q = threadIdx.x & 3u;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rec < n && q < 3u) v = table[3 * (size_t)perm(rec, mask) + q];
    lds[threadIdx.x] = v;
    __syncthreads();
    float4 w = lds[threadIdx.x ^ 1u];
    if (w.x + w.y == 123.456f) out[rec] = w.z;
}

// distinct `unit`-byte units touched by n accesses of `len` bytes at byte offsets off(i)
template <typename F>
static uint64_t units(uint64_t n, uint64_t len, uint64_t span, uint64_t unit, F off) {
    std::vector<bool> seen(span / unit + 2, false);
    uint64_t c = 0;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t a = off(i), b = a + len - 1;
        for (uint64_t u = a / unit; u <= b / unit; ++u)
            if (!seen[u]) {
                seen[u] = true;
                ++c;
            }
    }
    return c;
}

template <typename F>
static void report(const char* name, const char* dir, uint64_t n, uint64_t len, uint64_t span, F off) {
    printf("{\"kernel\": \"%s\", \"dir\": \"%s\", \"accesses\": %llu, \"bytes_per_access\": %llu, "
           "\"algorithmic_bytes\": %llu, \"touched_32B\": %llu, \"touched_64B\": %llu, \"touched_128B\": %llu}\n",
           name, dir, (unsigned long long)n, (unsigned long long)len, (unsigned long long)(n * len),
           (unsigned long long)(units(n, len, span, 32, off) * 32), (unsigned long long)(units(n, len, span, 64, off) * 64),
           (unsigned long long)(units(n, len, span, 128, off) * 128));
    fflush(stdout);
}

int main() {
    const size_t stream_bytes = 2ull << 30;                 // 2 GiB
    const uint32_t rec_bits = 25, rec_mask = (1u << rec_bits) - 1;  // 32M records x 48 B = 1.5 GiB
    const uint32_t n_gather = 1u << 23;                    // 8M records gathered (384 MB)
    const uint32_t w_bits = 28, w_mask = (1u << w_bits) - 1;  // 256M words = 1 GiB
    const uint32_t n_gather4 = 1u << 24;                   // 16M words
    const uint32_t s_bits = 26, s_mask = (1u << s_bits) - 1;  // 64M slots x 12 B = 768 MB
    const uint32_t n_scatter = 1u << 24;                   // 16M elements (192 MB)
    const uint32_t run_bits = s_bits - 3, run_mask = (1u << run_bits) - 1;

    void *buf, *out;
    size_t big = stream_bytes;
    CHECK(hipMalloc(&buf, big));
    CHECK(hipMalloc(&out, 64ull << 20));
    CHECK(hipMemset(buf, 0, big));
    CHECK(hipMemset(out, 0, 64ull << 20));
    CHECK(hipDeviceSynchronize());
    const int T = 256;

    stream_read<<<256 * 16, T>>>((const float4*)buf, stream_bytes / 16, (float*)out);
    CHECK(hipDeviceSynchronize());
    report("stream_read", "read", stream_bytes / 16, 16, stream_bytes, [](uint64_t i) { return 16 * i; });
    stream_write<<<256 * 16, T>>>((float4*)buf, stream_bytes / 16);
    CHECK(hipDeviceSynchronize());
    report("stream_write", "write", stream_bytes / 16, 16, stream_bytes, [](uint64_t i) { return 16 * i; });

    gather48<<<n_gather / T, T>>>((const float4*)buf, rec_mask, n_gather, (float*)out);
    CHECK(hipDeviceSynchronize());
    report("gather48", "read", n_gather, 48, 48ull << rec_bits,
           [&](uint64_t i) { return 48ull * perm((uint32_t)i, rec_mask); });

    gather48_lds<<<n_gather * 4 / T, T>>>((const float4*)buf, rec_mask, n_gather, (float*)out);
    CHECK(hipDeviceSynchronize());
    report("gather48_lds", "read", n_gather, 48, 48ull << rec_bits,
           [&](uint64_t i) { return 48ull * perm((uint32_t)i, rec_mask); });

    gather4<<<n_gather4 / T, T>>>((const uint32_t*)buf, w_mask, n_gather4, (uint32_t*)out);
    CHECK(hipDeviceSynchronize());
    report("gather4", "read", n_gather4, 4, 4ull << w_bits, [&](uint64_t i) { return 4ull * perm((uint32_t)i, w_mask); });

    scatter12<<<n_scatter / T, T>>>((uint32_t*)buf, s_mask, n_scatter);
    CHECK(hipDeviceSynchronize());
    report("scatter12", "write", n_scatter, 12, 12ull << s_bits,
           [&](uint64_t i) { return 12ull * perm((uint32_t)i, s_mask); });

    scatter12_runs<<<n_scatter / T, T>>>((uint32_t*)buf, run_mask, n_scatter);
    CHECK(hipDeviceSynchronize());
    report("scatter12_runs", "write", n_scatter, 12, 12ull << s_bits,
           [&](uint64_t i) { return 12ull * ((uint64_t)perm((uint32_t)(i >> 3), run_mask) * 8 + (i & 7)); });

    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
