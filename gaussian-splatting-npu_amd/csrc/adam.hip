// adam.hip -- visibility-masked ("sparse") Adam step for the Gaussian parameters (SURVEY.md §8f
// row 4).  The caller is train.py:180-183 (`gaussians.optimizer.step(radii > 0, N)`) through
// SparseGaussianAdam (scene/gaussian_model.py:194-196).  That class and its `_C.adamUpdate` op live
// in the accelerated upstream diff-gaussian-rasterization, which the reference does not vendor (its
// rasterizer package does not export it), so this restates the published update:
// for every element of a Gaussian whose visibility flag is set
//     m <- b1 m + (1 - b1) g;   v <- b2 v + (1 - b2) g^2;   p <- p - lr m / (sqrt(v) + eps)
// (no bias correction, the step count is not used); rows of invisible Gaussians are not touched.
//
// HBM-bound, 28 B per visible element (read p, g, m, v; write p, m, v) + 1 B per Gaussian.  All
// groups of a step go in one launch; each thread owns 4 consecutive elements (16-byte loads/stores when the five arrays are 16-byte aligned
// and the element count is a multiple of 4; scalar otherwise) and reads the flags of the Gaussians
// those elements belong to; a fully invisible quad issues no parameter traffic at all.
#include "gsr_kernels.h"

namespace gsr {

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float lr, float b1, float b2,
                                         float eps)
{
    m = b1 * m + (1.0f - b1) * g;
    v = b2 * v + (1.0f - b2) * g * g;
    p += -lr * m / (sqrtf(v) + eps);
}

// One quad (4 consecutive elements, q-th of the group) of one parameter group.
template <bool VEC>
__device__ __forceinline__ void adam_quad(const AdamArgs& a, uint32_t q)
{
    const uint32_t n = (uint32_t)a.N * (uint32_t)a.M;  // host checks n < 2^32
    const uint32_t e0 = 4 * q;
    uint32_t g = e0 / (uint32_t)a.M, r = e0 - g * (uint32_t)a.M;
    bool vis[4];
    bool any = false;
#pragma unroll
    for (int k = 0; k < 4; k++) {  // flag of the Gaussian owning element e0 + k
        vis[k] = e0 + k < n && a.visible[g] != 0;
        any |= vis[k];
        if (++r == (uint32_t)a.M) { r = 0; g++; }
    }
    if (!any) return;
    if (VEC) {  // n % 4 == 0 and every array 16-byte aligned
        float4 p = reinterpret_cast<float4*>(a.param)[q];
        const float4 gr = reinterpret_cast<const float4*>(a.grad)[q];
        float4 m = reinterpret_cast<float4*>(a.exp_avg)[q];
        float4 v = reinterpret_cast<float4*>(a.exp_avg_sq)[q];
        float pp[4] = {p.x, p.y, p.z, p.w}, mm[4] = {m.x, m.y, m.z, m.w}, vv[4] = {v.x, v.y, v.z, v.w};
        const float gg[4] = {gr.x, gr.y, gr.z, gr.w};
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (vis[k]) adam_one(pp[k], gg[k], mm[k], vv[k], a.lr, a.b1, a.b2, a.eps);
        reinterpret_cast<float4*>(a.param)[q] = make_float4(pp[0], pp[1], pp[2], pp[3]);
        reinterpret_cast<float4*>(a.exp_avg)[q] = make_float4(mm[0], mm[1], mm[2], mm[3]);
        reinterpret_cast<float4*>(a.exp_avg_sq)[q] = make_float4(vv[0], vv[1], vv[2], vv[3]);
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t e = e0 + k;
            if (!vis[k]) continue;
            float p = a.param[e], m = a.exp_avg[e], v = a.exp_avg_sq[e];
            adam_one(p, a.grad[e], m, v, a.lr, a.b1, a.b2, a.eps);
            a.param[e] = p;
            a.exp_avg[e] = m;
            a.exp_avg_sq[e] = v;
        }
    }
}

__device__ __forceinline__ bool adam_vec_ok(const AdamArgs& a)
{
    return ((size_t)a.N * a.M) % 4 == 0 &&
           (((uintptr_t)a.param | (uintptr_t)a.grad | (uintptr_t)a.exp_avg | (uintptr_t)a.exp_avg_sq) & 15) == 0;
}

// Every parameter group of a step in ONE launch (SparseGaussianAdam.step steps six groups, five of
// them only 1-4 floats per Gaussian: as separate launches they are latency-bound).  Workgroup b
// belongs to the group whose [block_start, block_start of the next) range holds b; one quad per
// thread.  The vector/scalar choice is uniform per group.
__global__ void __launch_bounds__(256) adam_update_multi_kernel(AdamMultiArgs a)
{
    int gi = 0;
#pragma unroll
    for (int k = 1; k < ADAM_MAX_GROUPS; k++)
        if (k < a.n_groups && blockIdx.x >= a.block_start[k]) gi = k;
    const AdamArgs& g = a.g[gi];
    const uint32_t q = (blockIdx.x - a.block_start[gi]) * 256 + threadIdx.x;
    if (q >= ((uint32_t)g.N * (uint32_t)g.M + 3) / 4) return;
    if (adam_vec_ok(g)) adam_quad<true>(g, q);
    else adam_quad<false>(g, q);
}

hipError_t launch_adam_update_multi(const AdamArgs* groups, int n_groups, hipStream_t s)
{
    AdamMultiArgs a;
    a.n_groups = 0;
    uint32_t blocks = 0;
    for (int i = 0; i < n_groups; i++) {
        const size_t n = (size_t)groups[i].N * groups[i].M;
        if (n == 0) continue;
        if (n >= 0xFFFFFFF0ull) return hipErrorInvalidValue;  // 32-bit element indices
        if (a.n_groups == ADAM_MAX_GROUPS) {  // flush a full launch
            hipLaunchKernelGGL(adam_update_multi_kernel, dim3(blocks), dim3(256), 0, s, a);
            a.n_groups = 0;
            blocks = 0;
        }
        a.g[a.n_groups] = groups[i];
        a.block_start[a.n_groups] = blocks;
        blocks += (uint32_t)(((n + 3) / 4 + 255) / 256);
        a.n_groups++;
    }
    if (a.n_groups) hipLaunchKernelGGL(adam_update_multi_kernel, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_adam_update(const AdamArgs& a, hipStream_t s) { return launch_adam_update_multi(&a, 1, s); }

}  // namespace gsr
