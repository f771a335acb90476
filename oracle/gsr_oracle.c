/*
 * gsr_oracle.c -- CPU restatement of the reference differentiable Gaussian
 * rasterizer (aki-k-no/gaussian-splatting-npu, vendored dr_aa rasterizer under
 * diff-gaussian-rasterization-npu/cuda_rasterizer/).
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline).  The product path (the HIP library under
 * gaussian-splatting-npu_amd/) never links, loads or falls back to it.
 *
 * Every function below restates one reference function and cites it.  The
 * floating-point operation order follows the reference source expression by
 * expression (left-associative C evaluation, GLM 0.9.9.9 column-major mat3
 * products, glm::dot = (x*x + y*y) + z*z).  The library is compiled with
 * -ffp-contract=off; the HIP preprocess kernel is compiled the same way, so
 * every value on the key-producing path (depth bits, radii, rects, tile
 * counts, conic, rgb) is bit-identical between the two.
 *
 * Pinning (see DESIGN.md "Oracle"): the reference ships no tests or golden
 * vectors for this path and cannot be built here (no nvcc/CUB).  The oracle is
 * pinned by (i) the reference's own importable Python pieces
 * (utils/sh_utils.py eval_sh, utils/graphics_utils.py camera matrices,
 * utils/general_utils.py build_rotation/build_scaling_rotation) through
 * tests/golden/make_golden.py, and (ii) torch.autograd + finite differences on
 * a dense differentiable restatement of the same forward (tests/test_oracle.py).
 * Key/value sort order is the definition of a stable LSD radix sort, which is
 * what cub::DeviceRadixSort::SortPairs computes (rasterizer_impl.cu:306).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BLOCK_X 16
#define BLOCK_Y 16
#define NUM_CHANNELS 3

/* auxiliary.h:21-38 */
static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;
/* glm::mat3 storage: m[col][row] */
typedef struct { float m[3][3]; } mat3;

static inline float fminf_(float a, float b) { return fminf(a, b); }

/* exp() of the blend (forward.cu:363, backward.cu:568): the host libm's expf by default; with
 * gsr_oracle_set_shared_exp(1) the test-only gsr_ref_expf that the GSR_REF_ALPHA build of the HIP
 * render kernels evaluates too (gsr_ref_exp.h), so that the two compare bit for bit. */
#include "../gaussian-splatting-npu_amd/csrc/gsr_ref_exp.h"
static int g_shared_exp = 0;
void gsr_oracle_set_shared_exp(int on) { g_shared_exp = on; }
float gsr_oracle_ref_expf(float x) { return gsr_ref_expf(x); } /* (for tests/test_oracle.py) */
static inline float blend_expf(float x) { return g_shared_exp ? gsr_ref_expf(x) : expf(x); }
static inline float fmaxf_(float a, float b) { return fmaxf(a, b); }

/* glm type_mat3x3.inl operator*(mat3, mat3) */
static mat3 mat3_mul(const mat3 a, const mat3 b)
{
    mat3 r;
    for (int c = 0; c < 3; c++)
        for (int w = 0; w < 3; w++)
            r.m[c][w] = a.m[0][w] * b.m[c][0] + a.m[1][w] * b.m[c][1] + a.m[2][w] * b.m[c][2];
    return r;
}

/* glm func_matrix.inl compute_transpose<3,3> */
static mat3 mat3_T(const mat3 a)
{
    mat3 r;
    for (int c = 0; c < 3; c++)
        for (int w = 0; w < 3; w++)
            r.m[c][w] = a.m[w][c];
    return r;
}

/* glm::mat3(a..i): fills columns */
static mat3 mat3_cols(float a, float b, float c, float d, float e, float f, float g, float h, float i)
{
    mat3 r;
    r.m[0][0] = a; r.m[0][1] = b; r.m[0][2] = c;
    r.m[1][0] = d; r.m[1][1] = e; r.m[1][2] = f;
    r.m[2][0] = g; r.m[2][1] = h; r.m[2][2] = i;
    return r;
}

/* auxiliary.h:70-78 */
static inline f3 transformPoint4x3(const f3 p, const float* m)
{
    f3 t = {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
            m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
    return t;
}

/* auxiliary.h:80-89 */
static inline f4 transformPoint4x4(const f3 p, const float* m)
{
    f4 t = {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
            m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14],
            m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]};
    return t;
}

/* auxiliary.h:101-109 */
static inline f3 transformVec4x3Transpose(const f3 p, const float* m)
{
    f3 t = {m[0] * p.x + m[1] * p.y + m[2] * p.z,
            m[4] * p.x + m[5] * p.y + m[6] * p.z,
            m[8] * p.x + m[9] * p.y + m[10] * p.z};
    return t;
}

/* auxiliary.h:119-129 */
static inline f3 dnormvdv(const f3 v, const f3 dv)
{
    float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    f3 r;
    r.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}

/* auxiliary.h:40-43 -- computed in double (1.0 literals), rounded to float */
static inline float ndc2Pix(float v, int S)
{
    return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

/* auxiliary.h:45-55 */
static inline void getRect(float px, float py, int max_radius, uint32_t gx, uint32_t gy,
                           uint32_t* rmin_x, uint32_t* rmin_y, uint32_t* rmax_x, uint32_t* rmax_y)
{
    int a;
    a = (int)((px - (float)max_radius) / (float)BLOCK_X); a = a > 0 ? a : 0;
    *rmin_x = (uint32_t)a < gx ? (uint32_t)a : gx;
    a = (int)((py - (float)max_radius) / (float)BLOCK_Y); a = a > 0 ? a : 0;
    *rmin_y = (uint32_t)a < gy ? (uint32_t)a : gy;
    a = (int)((px + (float)max_radius + (float)BLOCK_X - 1.0f) / (float)BLOCK_X); a = a > 0 ? a : 0;
    *rmax_x = (uint32_t)a < gx ? (uint32_t)a : gx;
    a = (int)((py + (float)max_radius + (float)BLOCK_Y - 1.0f) / (float)BLOCK_Y); a = a > 0 ? a : 0;
    *rmax_y = (uint32_t)a < gy ? (uint32_t)a : gy;
}

/* forward.cu:114-151 (quaternion NOT normalised, forward.cu:123) */
static void computeCov3D(const float* scale, float mod, const float* rot, float* cov3D)
{
    mat3 S = mat3_cols(1.0f, 0.0f, 0.0f, 0.0f, 1.0f, 0.0f, 0.0f, 0.0f, 1.0f);
    S.m[0][0] = mod * scale[0];
    S.m[1][1] = mod * scale[1];
    S.m[2][2] = mod * scale[2];
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
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

/* forward.cu:74-109 */
static f3 computeCov2D(const f3 mean, float focal_x, float focal_y, float tan_fovx, float tan_fovy,
                       const float* cov3D, const float* viewmatrix)
{
    f3 t = transformPoint4x3(mean, viewmatrix);
    const float limx = 1.3f * tan_fovx;
    const float limy = 1.3f * tan_fovy;
    const float txtz = t.x / t.z;
    const float tytz = t.y / t.z;
    t.x = fminf_(limx, fmaxf_(-limx, txtz)) * t.z;
    t.y = fminf_(limy, fmaxf_(-limy, tytz)) * t.z;

    mat3 J = mat3_cols(focal_x / t.z, 0.0f, -(focal_x * t.x) / (t.z * t.z),
                       0.0f, focal_y / t.z, -(focal_y * t.y) / (t.z * t.z),
                       0, 0, 0);
    const float* v = viewmatrix;
    mat3 W = mat3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    mat3 T = mat3_mul(W, J);
    mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    mat3 cov = mat3_mul(mat3_mul(mat3_T(T), mat3_T(Vrk)), T);
    f3 r = {cov.m[0][0], cov.m[0][1], cov.m[1][1]};
    return r;
}

/* forward.cu:20-71 */
static void computeColorFromSH(int idx, int deg, int max_coeffs, const float* means, const float* campos,
                               const float* shs, uint8_t* clamped, float* out)
{
    f3 pos = {means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]};
    f3 dir = {pos.x - campos[0], pos.y - campos[1], pos.z - campos[2]};
    float len = sqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
    dir.x = dir.x / len; dir.y = dir.y / len; dir.z = dir.z / len;

    const float* sh = shs + (size_t)idx * max_coeffs * 3;
    float res[3];
    for (int c = 0; c < 3; c++) res[c] = SH_C0 * sh[0 * 3 + c];
    if (deg > 0) {
        float x = dir.x, y = dir.y, z = dir.z;
        for (int c = 0; c < 3; c++)
            res[c] = res[c] - SH_C1 * y * sh[1 * 3 + c] + SH_C1 * z * sh[2 * 3 + c] - SH_C1 * x * sh[3 * 3 + c];
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            for (int c = 0; c < 3; c++)
                res[c] = res[c] +
                         SH_C2[0] * xy * sh[4 * 3 + c] +
                         SH_C2[1] * yz * sh[5 * 3 + c] +
                         SH_C2[2] * (2.0f * zz - xx - yy) * sh[6 * 3 + c] +
                         SH_C2[3] * xz * sh[7 * 3 + c] +
                         SH_C2[4] * (xx - yy) * sh[8 * 3 + c];
            if (deg > 2) {
                for (int c = 0; c < 3; c++)
                    res[c] = res[c] +
                             SH_C3[0] * y * (3.0f * xx - yy) * sh[9 * 3 + c] +
                             SH_C3[1] * xy * z * sh[10 * 3 + c] +
                             SH_C3[2] * y * (4.0f * zz - xx - yy) * sh[11 * 3 + c] +
                             SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[12 * 3 + c] +
                             SH_C3[4] * x * (4.0f * zz - xx - yy) * sh[13 * 3 + c] +
                             SH_C3[5] * z * (xx - yy) * sh[14 * 3 + c] +
                             SH_C3[6] * x * (xx - 3.0f * yy) * sh[15 * 3 + c];
            }
        }
    }
    uint8_t cl = 0;
    for (int c = 0; c < 3; c++) {
        res[c] += 0.5f;
        if (res[c] < 0) cl |= (uint8_t)(1u << c);
        out[c] = res[c] < 0.0f ? 0.0f : res[c];
    }
    clamped[idx] = cl;
}

/* ------------------------------------------------------------------------ */
typedef struct {
    int P, D, M, W, H, L;
    uint32_t gx, gy;
    int antialiasing;
    float* depths;
    uint8_t* clamped;   /* bit c set <=> channel c clamped (geomState.clamped[3*idx+c]) */
    int* radii;
    float* means2D;     /* P x 2 */
    float* cov3D;       /* P x 6 */
    float* conic_opacity; /* P x 4 */
    float* rgb;         /* P x 3 */
    uint32_t* tiles_touched;
    uint32_t* point_offsets;
    uint64_t* keys_unsorted;
    uint32_t* vals_unsorted;
    uint64_t* keys;
    uint32_t* vals;
    uint32_t* ranges;   /* T x 2 */
    float* final_T;
    uint32_t* n_contrib;
    int colors_precomp;
} oracle_state;

enum {
    OR_DEPTHS = 0, OR_CLAMPED, OR_RADII, OR_MEANS2D, OR_COV3D, OR_CONIC, OR_RGB, OR_TILES_TOUCHED,
    OR_POINT_OFFSETS, OR_KEYS_UNSORTED, OR_VALS_UNSORTED, OR_KEYS, OR_VALS, OR_RANGES, OR_FINAL_T, OR_N_CONTRIB
};

/* rasterizer_impl.cu:35-50 */
uint32_t gsr_oracle_higher_msb(uint32_t n)
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

/* Stable LSD radix sort of (key,val) on bits [0, end_bit): the definition of
 * cub::DeviceRadixSort::SortPairs(..., 0, 32 + bit) (rasterizer_impl.cu:306-311). */
static void radix_sort_pairs(uint64_t* keys, uint32_t* vals, uint64_t* ktmp, uint32_t* vtmp, int n, int end_bit)
{
    uint64_t* ks = keys; uint32_t* vs = vals; uint64_t* kd = ktmp; uint32_t* vd = vtmp;
    size_t count[256];
    for (int shift = 0; shift < end_bit; shift += 8) {
        int bits = end_bit - shift < 8 ? end_bit - shift : 8;
        uint64_t mask = (1ull << bits) - 1;
        memset(count, 0, sizeof(count));
        for (int i = 0; i < n; i++) count[(ks[i] >> shift) & mask]++;
        size_t s = 0;
        for (int d = 0; d < 256; d++) { size_t c = count[d]; count[d] = s; s += c; }
        for (int i = 0; i < n; i++) {
            size_t d = count[(ks[i] >> shift) & mask]++;
            kd[d] = ks[i]; vd[d] = vs[i];
        }
        uint64_t* t1 = ks; ks = kd; kd = t1;
        uint32_t* t2 = vs; vs = vd; vd = t2;
    }
    if (ks != keys) { memcpy(keys, ks, sizeof(uint64_t) * n); memcpy(vals, vs, sizeof(uint32_t) * n); }
}

static int g_nthreads = 1;
static void set_threads(int n)
{
    g_nthreads = n > 0 ? n : 1;
#ifdef _OPENMP
    omp_set_num_threads(g_nthreads);
#endif
}

/* rasterizer_impl.cu:54-66 + auxiliary.h:151-176 */
void gsr_oracle_mark_visible(int P, const float* means3D, const float* view, const float* proj, uint8_t* present)
{
    (void)proj;
    for (int i = 0; i < P; i++) {
        f3 p = {means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]};
        f3 pv = transformPoint4x3(p, view);
        present[i] = pv.z <= 0.2f ? 0 : 1;
    }
}

/* forward.cu:154-272 (preprocessCUDA) for one Gaussian; returns 0 ok, 1 if prefiltered violated */
static int preprocess_one(int idx, oracle_state* st, const float* orig_points, const float* scales, float scale_modifier,
                          const float* rotations, const float* opacities, const float* shs,
                          const float* cov3D_precomp, const float* colors_precomp,
                          const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                          float tan_fovx, float tan_fovy, float focal_x, float focal_y, int prefiltered,
                          int antialiasing)
{
    st->radii[idx] = 0;
    st->tiles_touched[idx] = 0;

    f3 p_orig = {orig_points[3 * idx], orig_points[3 * idx + 1], orig_points[3 * idx + 2]};
    /* in_frustum (auxiliary.h:151-176) */
    f3 p_view = transformPoint4x3(p_orig, viewmatrix);
    if (p_view.z <= 0.2f) return prefiltered ? 1 : 0;

    f4 p_hom = transformPoint4x4(p_orig, projmatrix);
    float p_w = 1.0f / (p_hom.w + 0.0000001f);
    f3 p_proj = {p_hom.x * p_w, p_hom.y * p_w, p_hom.z * p_w};

    const float* cov3D;
    if (cov3D_precomp) cov3D = cov3D_precomp + (size_t)idx * 6;
    else {
        computeCov3D(scales + 3 * (size_t)idx, scale_modifier, rotations + 4 * (size_t)idx, st->cov3D + (size_t)idx * 6);
        cov3D = st->cov3D + (size_t)idx * 6;
    }

    f3 cov = computeCov2D(p_orig, focal_x, focal_y, tan_fovx, tan_fovy, cov3D, viewmatrix);
    const float h_var = 0.3f;
    const float det_cov = cov.x * cov.z - cov.y * cov.y;
    cov.x += h_var;
    cov.z += h_var;
    const float det_cov_plus_h_cov = cov.x * cov.z - cov.y * cov.y;
    float h_convolution_scaling = 1.0f;
    if (antialiasing) h_convolution_scaling = sqrtf(fmaxf_(0.000025f, det_cov / det_cov_plus_h_cov));

    const float det = det_cov_plus_h_cov;
    if (det == 0.0f) return 0;
    float det_inv = 1.f / det;
    f3 conic = {cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv};

    float mid = 0.5f * (cov.x + cov.z);
    float lambda1 = mid + sqrtf(fmaxf_(0.1f, mid * mid - det));
    float lambda2 = mid - sqrtf(fmaxf_(0.1f, mid * mid - det));
    float my_radius = ceilf(3.f * sqrtf(fmaxf_(lambda1, lambda2)));
    float px = ndc2Pix(p_proj.x, st->W), py = ndc2Pix(p_proj.y, st->H);
    uint32_t rminx, rminy, rmaxx, rmaxy;
    getRect(px, py, (int)my_radius, st->gx, st->gy, &rminx, &rminy, &rmaxx, &rmaxy);
    if ((rmaxx - rminx) * (rmaxy - rminy) == 0) return 0;

    if (!colors_precomp)
        computeColorFromSH(idx, st->D, st->M, orig_points, cam_pos, shs, st->clamped, st->rgb + 3 * (size_t)idx);

    st->depths[idx] = p_view.z;
    st->radii[idx] = (int)my_radius;
    st->means2D[2 * idx] = px;
    st->means2D[2 * idx + 1] = py;
    float opacity = opacities[idx];
    st->conic_opacity[4 * idx + 0] = conic.x;
    st->conic_opacity[4 * idx + 1] = conic.y;
    st->conic_opacity[4 * idx + 2] = conic.z;
    st->conic_opacity[4 * idx + 3] = opacity * h_convolution_scaling;
    st->tiles_touched[idx] = (rmaxy - rminy) * (rmaxx - rminx);
    return 0;
}

/* forward.cu:277-400 (renderCUDA) for one tile */
static void render_tile(const oracle_state* st, uint32_t tx, uint32_t ty, const float* features, const float* bg,
                        float* out_color, float* invdepth)
{
    const int W = st->W, H = st->H;
    const uint32_t* range = st->ranges + 2 * (ty * st->gx + tx);
    for (uint32_t ly = 0; ly < BLOCK_Y; ly++)
        for (uint32_t lx = 0; lx < BLOCK_X; lx++) {
            uint32_t pxi = tx * BLOCK_X + lx, pyi = ty * BLOCK_Y + ly;
            if (!(pxi < (uint32_t)W && pyi < (uint32_t)H)) continue;
            uint32_t pix_id = (uint32_t)W * pyi + pxi;
            float pfx = (float)pxi, pfy = (float)pyi;
            float T = 1.0f;
            uint32_t contributor = 0, last_contributor = 0;
            float C[3] = {0, 0, 0};
            float expected_invdepth = 0.0f;
            for (uint32_t k = range[0]; k < range[1]; k++) {
                contributor++;
                uint32_t id = st->vals[k];
                float dx = st->means2D[2 * id] - pfx, dy = st->means2D[2 * id + 1] - pfy;
                const float* co = st->conic_opacity + 4 * (size_t)id;
                float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                if (power > 0.0f) continue;
                float alpha = fminf_(0.99f, co[3] * blend_expf(power));
                if (alpha < 1.0f / 255.0f) continue;
                float test_T = T * (1 - alpha);
                if (test_T < 0.0001f) break; /* done = true */
                for (int ch = 0; ch < 3; ch++) C[ch] += features[id * 3 + ch] * alpha * T;
                expected_invdepth += (1 / st->depths[id]) * alpha * T;
                T = test_T;
                last_contributor = contributor;
            }
            st->final_T[pix_id] = T;
            st->n_contrib[pix_id] = last_contributor;
            for (int ch = 0; ch < 3; ch++) out_color[ch * H * W + pix_id] = C[ch] + T * bg[ch];
            if (invdepth) invdepth[pix_id] = expected_invdepth;
        }
}

/* Pixels whose blend takes a decision within `rel` of its threshold (test infrastructure, not a
 * restatement): power within rel of its terms' magnitude of 0 (forward.cu:355), alpha within
 * rel * (1/255) of 1/255
 * (:364) or test_T within rel * 1e-4 of 1e-4 (:369), over the entries the pixel's walk
 * evaluates.  A float32 evaluation in another order (v_exp_f32 of a log2-scaled falloff on the
 * GPU) may take such a decision the other way without moving the pixel's colour past the
 * parity tests' IMG_ATOL; tests/common.check_rel_truth leaves the Gaussians of these pixels' walks
 * out with those of the flipped pixels.  out[N]: 1 = near a threshold; out_gauss[P] (may be NULL):
 * 1 = the Gaussian whose decision it is (the one whose term appears or vanishes). */
int gsr_oracle_near_threshold(void* p, float rel, uint8_t* out, uint8_t* out_gauss)
{
    const oracle_state* st = (const oracle_state*)p;
    const int W = st->W, H = st->H;
    memset(out, 0, (size_t)W * H);
    if (out_gauss) memset(out_gauss, 0, (size_t)st->P);
    const int T = (int)(st->gx * st->gy);
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < T; t++) {
        const uint32_t tx = (uint32_t)t % st->gx, ty = (uint32_t)t / st->gx;
        const uint32_t* range = st->ranges + 2 * (size_t)t;
        for (uint32_t ly = 0; ly < BLOCK_Y; ly++)
            for (uint32_t lx = 0; lx < BLOCK_X; lx++) {
                uint32_t pxi = tx * BLOCK_X + lx, pyi = ty * BLOCK_Y + ly;
                if (!(pxi < (uint32_t)W && pyi < (uint32_t)H)) continue;
                const uint32_t pix_id = (uint32_t)W * pyi + pxi;
                const float pfx = (float)pxi, pfy = (float)pyi;
                float Tr = 1.0f;
                int near = 0;
                for (uint32_t k = range[0]; k < range[1] && !near; k++) {
                    const uint32_t id = st->vals[k];
                    const float dx = st->means2D[2 * id] - pfx, dy = st->means2D[2 * id + 1] - pfy;
                    const float* co = st->conic_opacity + 4 * (size_t)id;
                    const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    /* power's sign can flip by rounding only where its terms nearly cancel */
                    const float terms = 0.5f * (fabsf(co[0]) * dx * dx + fabsf(co[2]) * dy * dy) + fabsf(co[1] * dx * dy);
                    if (fabsf(power) <= rel * terms) near = 1;
                    if (power <= 0.0f) {
                        const float alpha = fminf_(0.99f, co[3] * blend_expf(power));
                        if (fabsf(alpha - 1.0f / 255.0f) <= rel * (1.0f / 255.0f)) near = 1;
                        if (alpha >= 1.0f / 255.0f) {
                            const float test_T = Tr * (1 - alpha);
                            if (fabsf(test_T - 0.0001f) <= rel * 0.0001f) near = 1;
                            if (test_T < 0.0001f && !near) break;
                            Tr = test_T;
                        }
                    }
                    if (near && out_gauss) out_gauss[id] = 1;  /* (benign race: every writer stores 1) */
                }
                out[pix_id] = (uint8_t)near;
            }
    }
    return 0;
}

void gsr_oracle_free(void* p)
{
    oracle_state* st = (oracle_state*)p;
    if (!st) return;
    free(st->depths); free(st->clamped); free(st->radii); free(st->means2D); free(st->cov3D);
    free(st->conic_opacity); free(st->rgb); free(st->tiles_touched); free(st->point_offsets);
    free(st->keys_unsorted); free(st->vals_unsorted); free(st->keys); free(st->vals); free(st->ranges);
    free(st->final_T); free(st->n_contrib);
    free(st);
}

static char g_err[256];
const char* gsr_oracle_last_error(void) { return g_err; }

/* rasterizer_impl.cu:198-341 (Rasterizer::forward) */
void* gsr_oracle_forward(int P, int D, int M, const float* bg, int W, int H,
                         const float* means3D, const float* shs, const float* colors_precomp,
                         const float* opacities, const float* scales, float scale_modifier,
                         const float* rotations, const float* cov3D_precomp,
                         const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                         float tan_fovx, float tan_fovy, int prefiltered, int antialiasing,
                         float* out_color, float* out_invdepth, int* radii_out, int nthreads, int* num_rendered)
{
    set_threads(nthreads);
    oracle_state* st = (oracle_state*)calloc(1, sizeof(oracle_state));
    st->P = P; st->D = D; st->M = M; st->W = W; st->H = H; st->antialiasing = antialiasing;
    st->colors_precomp = colors_precomp != NULL;
    st->gx = (uint32_t)((W + BLOCK_X - 1) / BLOCK_X);
    st->gy = (uint32_t)((H + BLOCK_Y - 1) / BLOCK_Y);
    size_t Pn = P > 0 ? (size_t)P : 1;
    st->depths = (float*)calloc(Pn, 4);
    st->clamped = (uint8_t*)calloc(Pn, 1);
    st->radii = (int*)calloc(Pn, 4);
    st->means2D = (float*)calloc(Pn * 2, 4);
    st->cov3D = (float*)calloc(Pn * 6, 4);
    st->conic_opacity = (float*)calloc(Pn * 4, 4);
    st->rgb = (float*)calloc(Pn * 3, 4);
    st->tiles_touched = (uint32_t*)calloc(Pn, 4);
    st->point_offsets = (uint32_t*)calloc(Pn, 4);
    size_t T = (size_t)st->gx * st->gy;
    st->ranges = (uint32_t*)calloc(T * 2 + 2, 4);
    size_t N = (size_t)W * H;
    st->final_T = (float*)calloc(N + 1, 4);
    st->n_contrib = (uint32_t*)calloc(N + 1, 4);

    /* rasterize_points.cu:69-76: outputs start at zero */
    memset(out_color, 0, sizeof(float) * 3 * N);
    if (out_invdepth) memset(out_invdepth, 0, sizeof(float) * N);
    *num_rendered = 0;
    if (P == 0) return st;

    const float focal_y = H / (2.0f * tan_fovy);
    const float focal_x = W / (2.0f * tan_fovx);

    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int i = 0; i < P; i++)
        bad |= preprocess_one(i, st, means3D, scales, scale_modifier, rotations, opacities, shs, cov3D_precomp,
                              colors_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, focal_x,
                              focal_y, prefiltered, antialiasing);
    if (bad) {
        snprintf(g_err, sizeof(g_err), "Point is filtered although prefiltered is set.");
        gsr_oracle_free(st);
        return NULL;
    }
    memcpy(radii_out, st->radii, sizeof(int) * P);

    /* cub::DeviceScan::InclusiveSum (rasterizer_impl.cu:280) */
    uint64_t acc = 0;
    for (int i = 0; i < P; i++) { acc += st->tiles_touched[i]; st->point_offsets[i] = (uint32_t)acc; }
    int L = (int)st->point_offsets[P - 1];
    st->L = L;
    *num_rendered = L;
    size_t Ln = L > 0 ? (size_t)L : 1;
    st->keys_unsorted = (uint64_t*)malloc(Ln * 8);
    st->vals_unsorted = (uint32_t*)malloc(Ln * 4);
    st->keys = (uint64_t*)malloc(Ln * 8);
    st->vals = (uint32_t*)malloc(Ln * 4);

    /* duplicateWithKeys (rasterizer_impl.cu:70-111) */
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        if (st->radii[idx] > 0) {
            uint32_t off = idx == 0 ? 0 : st->point_offsets[idx - 1];
            uint32_t rminx, rminy, rmaxx, rmaxy;
            getRect(st->means2D[2 * idx], st->means2D[2 * idx + 1], st->radii[idx], st->gx, st->gy,
                    &rminx, &rminy, &rmaxx, &rmaxy);
            uint32_t dbits;
            memcpy(&dbits, &st->depths[idx], 4);
            for (uint32_t y = rminy; y < rmaxy; y++)
                for (uint32_t x = rminx; x < rmaxx; x++) {
                    uint64_t key = (uint64_t)(y * st->gx + x);
                    key <<= 32;
                    key |= dbits;
                    st->keys_unsorted[off] = key;
                    st->vals_unsorted[off] = (uint32_t)idx;
                    off++;
                }
        }
    }

    /* SortPairs on bits [0, 32+bit) (rasterizer_impl.cu:303-311) */
    int bit = (int)gsr_oracle_higher_msb(st->gx * st->gy);
    memcpy(st->keys, st->keys_unsorted, Ln * 8);
    memcpy(st->vals, st->vals_unsorted, Ln * 4);
    if (L > 0) {
        uint64_t* kt = (uint64_t*)malloc(Ln * 8);
        uint32_t* vt = (uint32_t*)malloc(Ln * 4);
        radix_sort_pairs(st->keys, st->vals, kt, vt, L, 32 + bit);
        free(kt); free(vt);
    }

    /* memset + identifyTileRanges (rasterizer_impl.cu:313-320, 116-138) */
    memset(st->ranges, 0, sizeof(uint32_t) * 2 * T);
    for (int idx = 0; idx < L; idx++) {
        uint32_t currtile = (uint32_t)(st->keys[idx] >> 32);
        if (idx == 0) st->ranges[2 * currtile] = 0;
        else {
            uint32_t prevtile = (uint32_t)(st->keys[idx - 1] >> 32);
            if (currtile != prevtile) { st->ranges[2 * prevtile + 1] = idx; st->ranges[2 * currtile] = idx; }
        }
        if (idx == L - 1) st->ranges[2 * currtile + 1] = L;
    }

    /* FORWARD::render (rasterizer_impl.cu:324-338) */
    const float* features = colors_precomp ? colors_precomp : st->rgb;
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < (int)T; t++)
        render_tile(st, (uint32_t)t % st->gx, (uint32_t)t / st->gx, features, bg, out_color, out_invdepth);
    return st;
}

int gsr_oracle_get(void* p, int which, void* dst)
{
    oracle_state* st = (oracle_state*)p;
    size_t P = (size_t)st->P, L = (size_t)st->L, N = (size_t)st->W * st->H, T = (size_t)st->gx * st->gy;
    switch (which) {
    case OR_DEPTHS: memcpy(dst, st->depths, P * 4); break;
    case OR_CLAMPED: memcpy(dst, st->clamped, P); break;
    case OR_RADII: memcpy(dst, st->radii, P * 4); break;
    case OR_MEANS2D: memcpy(dst, st->means2D, P * 8); break;
    case OR_COV3D: memcpy(dst, st->cov3D, P * 24); break;
    case OR_CONIC: memcpy(dst, st->conic_opacity, P * 16); break;
    case OR_RGB: memcpy(dst, st->rgb, P * 12); break;
    case OR_TILES_TOUCHED: memcpy(dst, st->tiles_touched, P * 4); break;
    case OR_POINT_OFFSETS: memcpy(dst, st->point_offsets, P * 4); break;
    case OR_KEYS_UNSORTED: if (L) memcpy(dst, st->keys_unsorted, L * 8); break;
    case OR_VALS_UNSORTED: if (L) memcpy(dst, st->vals_unsorted, L * 4); break;
    case OR_KEYS: if (L) memcpy(dst, st->keys, L * 8); break;
    case OR_VALS: if (L) memcpy(dst, st->vals, L * 4); break;
    case OR_RANGES: memcpy(dst, st->ranges, T * 8); break;
    case OR_FINAL_T: memcpy(dst, st->final_T, N * 4); break;
    case OR_N_CONTRIB: memcpy(dst, st->n_contrib, N * 4); break;
    default: return -1;
    }
    return 0;
}

/* ----------------------------- backward ---------------------------------- */

static inline void atomic_addf(float* p, float v)
{
#pragma omp atomic
    *p += v;
}

/* backward.cu:452-638 (renderCUDA) for one tile.  The reference adds every pixel's terms into the
 * per-Gaussian sums with float atomics, in no fixed order.  With `ts` (tile sums, gsr_oracle_set_bwd_
 * tile_sums) the same per-pixel terms are first added into per-list-entry sums of this tile (pixel
 * order), which are then added into the per-Gaussian sums: the same terms in another summation
 * order, without 10 atomics per contribution (the training tests' oracle loops). */
enum { TS_M2X, TS_M2Y, TS_C0, TS_C1, TS_C3, TS_OP, TS_R, TS_G, TS_B, TS_INVD, TS_N };
static void render_bwd_tile(const oracle_state* st, uint32_t tx, uint32_t ty, const float* bg, const float* colors,
                            const float* dL_dpixels, const float* dL_invdepths, float* dL_dmean2D, float* dL_dconic2D,
                            float* dL_dopacity, float* dL_dcolors, float* dL_dinvdepths, float* ts)
{
    const int W = st->W, H = st->H;
    const uint32_t* range = st->ranges + 2 * (ty * st->gx + tx);
    if (ts) memset(ts, 0, sizeof(float) * TS_N * (size_t)(range[1] - range[0]));
#define TS_ADD(field, ptr, v) \
    do { if (ts) ts[(size_t)(k - range[0]) * TS_N + (field)] += (v); else atomic_addf((ptr), (v)); } while (0)
    const float ddelx_dx = 0.5 * W;
    const float ddely_dy = 0.5 * H;
    for (uint32_t ly = 0; ly < BLOCK_Y; ly++)
        for (uint32_t lx = 0; lx < BLOCK_X; lx++) {
            uint32_t pxi = tx * BLOCK_X + lx, pyi = ty * BLOCK_Y + ly;
            if (!(pxi < (uint32_t)W && pyi < (uint32_t)H)) continue;
            uint32_t pix_id = (uint32_t)W * pyi + pxi;
            float pfx = (float)pxi, pfy = (float)pyi;
            const float T_final = st->final_T[pix_id];
            float T = T_final;
            uint32_t contributor = range[1] - range[0];
            const uint32_t last_contributor = st->n_contrib[pix_id];
            float accum_rec[3] = {0, 0, 0};
            float dL_dpixel[3];
            float dL_invdepth = 0;
            float accum_invdepth_rec = 0;
            for (int i = 0; i < 3; i++) dL_dpixel[i] = dL_dpixels[i * H * W + pix_id];
            if (dL_invdepths) dL_invdepth = dL_invdepths[pix_id];
            float last_alpha = 0;
            float last_color[3] = {0, 0, 0};
            float last_invdepth = 0;
            for (int64_t k = (int64_t)range[1] - 1; k >= (int64_t)range[0]; k--) {
                contributor--;
                if (contributor >= last_contributor) continue;
                uint32_t gid = st->vals[k];
                float dx = st->means2D[2 * gid] - pfx, dy = st->means2D[2 * gid + 1] - pfy;
                const float* co = st->conic_opacity + 4 * (size_t)gid;
                const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                if (power > 0.0f) continue;
                const float G = blend_expf(power);
                const float alpha = fminf_(0.99f, co[3] * G);
                if (alpha < 1.0f / 255.0f) continue;
                T = T / (1.f - alpha);
                const float dchannel_dcolor = alpha * T;
                float dL_dalpha = 0.0f;
                for (int ch = 0; ch < 3; ch++) {
                    const float c = colors[gid * 3 + ch];
                    accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
                    last_color[ch] = c;
                    const float dL_dchannel = dL_dpixel[ch];
                    dL_dalpha += (c - accum_rec[ch]) * dL_dchannel;
                    TS_ADD(TS_R + ch, &dL_dcolors[gid * 3 + ch], dchannel_dcolor * dL_dchannel);
                }
                if (dL_dinvdepths) {
                    const float invd = 1.f / st->depths[gid];
                    accum_invdepth_rec = last_alpha * last_invdepth + (1.f - last_alpha) * accum_invdepth_rec;
                    last_invdepth = invd;
                    dL_dalpha += (invd - accum_invdepth_rec) * dL_invdepth;
                    TS_ADD(TS_INVD, &dL_dinvdepths[gid], dchannel_dcolor * dL_invdepth);
                }
                dL_dalpha *= T;
                last_alpha = alpha;
                float bg_dot_dpixel = 0;
                for (int i = 0; i < 3; i++) bg_dot_dpixel += bg[i] * dL_dpixel[i];
                dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot_dpixel;
                const float dL_dG = co[3] * dL_dalpha;
                const float gdx = G * dx;
                const float gdy = G * dy;
                const float dG_ddelx = -gdx * co[0] - gdy * co[1];
                const float dG_ddely = -gdy * co[2] - gdx * co[1];
                TS_ADD(TS_M2X, &dL_dmean2D[3 * gid + 0], dL_dG * dG_ddelx * ddelx_dx);
                TS_ADD(TS_M2Y, &dL_dmean2D[3 * gid + 1], dL_dG * dG_ddely * ddely_dy);
                TS_ADD(TS_C0, &dL_dconic2D[4 * gid + 0], -0.5f * gdx * dx * dL_dG);
                TS_ADD(TS_C1, &dL_dconic2D[4 * gid + 1], -0.5f * gdx * dy * dL_dG);
                TS_ADD(TS_C3, &dL_dconic2D[4 * gid + 3], -0.5f * gdy * dy * dL_dG);
                TS_ADD(TS_OP, &dL_dopacity[gid], G * dL_dalpha);
            }
        }
#undef TS_ADD
    if (!ts) return;
    for (uint32_t k = range[0]; k < range[1]; k++) {
        const float* e = ts + (size_t)(k - range[0]) * TS_N;
        const uint32_t gid = st->vals[k];
        if (e[TS_M2X] != 0.0f) atomic_addf(&dL_dmean2D[3 * gid + 0], e[TS_M2X]);
        if (e[TS_M2Y] != 0.0f) atomic_addf(&dL_dmean2D[3 * gid + 1], e[TS_M2Y]);
        if (e[TS_C0] != 0.0f) atomic_addf(&dL_dconic2D[4 * gid + 0], e[TS_C0]);
        if (e[TS_C1] != 0.0f) atomic_addf(&dL_dconic2D[4 * gid + 1], e[TS_C1]);
        if (e[TS_C3] != 0.0f) atomic_addf(&dL_dconic2D[4 * gid + 3], e[TS_C3]);
        if (e[TS_OP] != 0.0f) atomic_addf(&dL_dopacity[gid], e[TS_OP]);
        for (int ch = 0; ch < 3; ch++)
            if (e[TS_R + ch] != 0.0f) atomic_addf(&dL_dcolors[gid * 3 + ch], e[TS_R + ch]);
        if (dL_dinvdepths && e[TS_INVD] != 0.0f) atomic_addf(&dL_dinvdepths[gid], e[TS_INVD]);
    }
}

/* The same per-pixel walk with the gradient arithmetic in float64 -- the accuracy yardstick of the
 * parity tests (tests/common.py check_rel_truth), not a restatement: the contribution DECISIONS
 * (power > 0, alpha < 1/255, the last contributor) are the float32 ones above, so both walks sum
 * the same terms; G, alpha, the transmittances (a front-to-back float64 product, not the
 * reference's division chain), the colour behind each entry and every accumulation are float64. */
static inline void atomic_addd(double* p, double v)
{
#pragma omp atomic
    *p += v;
}
static void render_bwd_tile_f64(const oracle_state* st, uint32_t tx, uint32_t ty, const float* bg, const float* colors,
                                const float* dL_dpixels, const float* dL_invdepths, double* g_mean2D, double* g_conic,
                                double* g_opacity, double* g_colors, double* g_invdepths, double* scratch)
{
    const int W = st->W, H = st->H;
    const uint32_t* range = st->ranges + 2 * (ty * st->gx + tx);
    const double ddelx_dx = 0.5 * W, ddely_dy = 0.5 * H;
    /* scratch: per contributing entry (k, G, alpha, T in front) of one pixel */
    for (uint32_t ly = 0; ly < BLOCK_Y; ly++)
        for (uint32_t lx = 0; lx < BLOCK_X; lx++) {
            uint32_t pxi = tx * BLOCK_X + lx, pyi = ty * BLOCK_Y + ly;
            if (!(pxi < (uint32_t)W && pyi < (uint32_t)H)) continue;
            uint32_t pix_id = (uint32_t)W * pyi + pxi;
            const float pfx = (float)pxi, pfy = (float)pyi;
            const uint32_t last_contributor = st->n_contrib[pix_id];
            double dpx[3];
            for (int i = 0; i < 3; i++) dpx[i] = dL_dpixels[i * H * W + pix_id];
            const double dinv = dL_invdepths ? dL_invdepths[pix_id] : 0.0;
            /* front to back: the contributing entries, float32 decisions, float64 values */
            int n = 0;
            double T = 1.0;
            for (uint32_t j = 0; j < last_contributor && range[0] + j < range[1]; j++) {
                uint32_t gid = st->vals[range[0] + j];
                const float* co = st->conic_opacity + 4 * (size_t)gid;
                const float dxf = st->means2D[2 * gid] - pfx, dyf = st->means2D[2 * gid + 1] - pfy;
                const float power = -0.5f * (co[0] * dxf * dxf + co[2] * dyf * dyf) - co[1] * dxf * dyf;
                if (power > 0.0f) continue;
                const float alpha_f = fminf_(0.99f, co[3] * blend_expf(power));
                if (alpha_f < 1.0f / 255.0f) continue;
                const double dx = dxf, dy = dyf;
                const double pw = -0.5 * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                const double G = exp(pw);
                const double alpha = fmin(0.99, co[3] * G);
                double* e = scratch + 4 * (size_t)n++;
                e[0] = (double)gid;
                e[1] = G;
                e[2] = alpha;
                e[3] = T;
                T *= 1.0 - alpha;
            }
            const double T_final = T;
            double bg_dot = 0.0;
            for (int i = 0; i < 3; i++) bg_dot += (double)bg[i] * dpx[i];
            /* back to front: behind = colour (and inverse depth) . dL behind the entry, absolute */
            double behind = T_final * bg_dot;
            for (int q = n - 1; q >= 0; q--) {
                const double* e = scratch + 4 * (size_t)q;
                const uint32_t gid = (uint32_t)e[0];
                const double G = e[1], alpha = e[2], Tj = e[3];
                const float* co = st->conic_opacity + 4 * (size_t)gid;
                const double dx = (double)(st->means2D[2 * gid] - pfx), dy = (double)(st->means2D[2 * gid + 1] - pfy);
                double cd = 0.0;
                for (int ch = 0; ch < 3; ch++) {
                    cd += (double)colors[gid * 3 + ch] * dpx[ch];
                    atomic_addd(&g_colors[gid * 3 + ch], alpha * Tj * dpx[ch]);
                }
                if (dL_invdepths) {
                    const double invd = 1.0 / (double)st->depths[gid];
                    cd += invd * dinv;
                    atomic_addd(&g_invdepths[gid], alpha * Tj * dinv);
                }
                /* dL/dalpha = T_j (c_j . dL) - (light behind j) / (1 - alpha_j) */
                const double dL_dalpha = Tj * cd - behind / (1.0 - alpha);
                behind += alpha * Tj * cd;
                const double dL_dG = co[3] * dL_dalpha;
                const double gdx = G * dx, gdy = G * dy;
                const double dG_ddelx = -gdx * co[0] - gdy * co[1];
                const double dG_ddely = -gdy * co[2] - gdx * co[1];
                atomic_addd(&g_mean2D[3 * gid + 0], dL_dG * dG_ddelx * ddelx_dx);
                atomic_addd(&g_mean2D[3 * gid + 1], dL_dG * dG_ddely * ddely_dy);
                atomic_addd(&g_conic[4 * gid + 0], -0.5 * gdx * dx * dL_dG);
                atomic_addd(&g_conic[4 * gid + 1], -0.5 * gdx * dy * dL_dG);
                atomic_addd(&g_conic[4 * gid + 3], -0.5 * gdy * dy * dL_dG);
                atomic_addd(&g_opacity[gid], G * dL_dalpha);
            }
        }
}

static int g_bwd_f64 = 0;
static int g_bwd_tile_sums = 0;
void gsr_oracle_set_bwd_tile_sums(int on) { g_bwd_tile_sums = on; }
/* 1: gsr_oracle_backward runs the render backward in float64 (render_bwd_tile_f64) and rounds its
 * per-Gaussian sums to float32 once, before the (float32) preprocess backward. */
void gsr_oracle_set_bwd_f64(int on) { g_bwd_f64 = on; }

static inline float sq(float x) { return x * x; }

/* backward.cu:147-326 (computeCov2DCUDA) for one Gaussian */
static void cov2d_bwd_one(int idx, const float* means, const float* cov3Ds, float h_x, float h_y, float tan_fovx,
                          float tan_fovy, const float* view_matrix, const float* opacities, const float* dL_dconics,
                          float* dL_dopacity, const float* dL_dinvdepth, float* dL_dmeans, float* dL_dcov,
                          int antialiasing)
{
    const float* cov3D = cov3Ds + 6 * (size_t)idx;
    f3 mean = {means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]};
    f3 dL_dconic = {dL_dconics[4 * idx], dL_dconics[4 * idx + 1], dL_dconics[4 * idx + 3]};
    f3 t = transformPoint4x3(mean, view_matrix);
    const float limx = 1.3f * tan_fovx;
    const float limy = 1.3f * tan_fovy;
    const float txtz = t.x / t.z;
    const float tytz = t.y / t.z;
    t.x = fminf_(limx, fmaxf_(-limx, txtz)) * t.z;
    t.y = fminf_(limy, fmaxf_(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;

    mat3 J = mat3_cols(h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z),
                       0.0f, h_y / t.z, -(h_y * t.y) / (t.z * t.z), 0, 0, 0);
    const float* v = view_matrix;
    mat3 Wm = mat3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    mat3 T = mat3_mul(Wm, J);
    mat3 cov2D = mat3_mul(mat3_mul(mat3_T(T), mat3_T(Vrk)), T);

    float c_xx = cov2D.m[0][0];
    float c_xy = cov2D.m[0][1];
    float c_yy = cov2D.m[1][1];
    const float h_var = 0.3f;
    float d_inside_root = 0.f;
    if (antialiasing) {
        const float det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const float det_cov_plus_h_cov = c_xx * c_yy - c_xy * c_xy;
        const float h_convolution_scaling = sqrtf(fmaxf_(0.000025f, det_cov / det_cov_plus_h_cov));
        const float dL_dopacity_v = dL_dopacity[idx];
        const float d_h_convolution_scaling = dL_dopacity_v * opacities[idx];
        dL_dopacity[idx] = dL_dopacity_v * h_convolution_scaling;
        d_inside_root = (det_cov / det_cov_plus_h_cov) <= 0.000025f ? 0.f : d_h_convolution_scaling / (2 * h_convolution_scaling);
    } else {
        c_xx += h_var;
        c_yy += h_var;
    }
    float dL_dc_xx = 0, dL_dc_xy = 0, dL_dc_yy = 0;
    if (antialiasing) {
        const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
        const float denom_f = d_inside_root / sq(w * w + w * (x + y) + x * y - z * z);
        const float dL_dx = w * (w * y + y * y + z * z) * denom_f;
        const float dL_dy = w * (w * x + x * x + z * z) * denom_f;
        const float dL_dz = -2.f * w * z * (w + x + y) * denom_f;
        dL_dc_xx = dL_dx;
        dL_dc_yy = dL_dy;
        dL_dc_xy = dL_dz;
    }
    float denom = c_xx * c_yy - c_xy * c_xy;
    float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    float* dc = dL_dcov + 6 * (size_t)idx;
    if (denom2inv != 0) {
        dL_dc_xx += denom2inv * (-c_yy * c_yy * dL_dconic.x + 2 * c_xy * c_yy * dL_dconic.y + (denom - c_xx * c_yy) * dL_dconic.z);
        dL_dc_yy += denom2inv * (-c_xx * c_xx * dL_dconic.z + 2 * c_xx * c_xy * dL_dconic.y + (denom - c_xx * c_yy) * dL_dconic.x);
        dL_dc_xy += denom2inv * 2 * (c_xy * c_yy * dL_dconic.x - (denom + 2 * c_xy * c_xy) * dL_dconic.y + c_xx * c_xy * dL_dconic.z);
        const float (*Tm)[3] = T.m;
        dc[0] = (Tm[0][0] * Tm[0][0] * dL_dc_xx + Tm[0][0] * Tm[1][0] * dL_dc_xy + Tm[1][0] * Tm[1][0] * dL_dc_yy);
        dc[3] = (Tm[0][1] * Tm[0][1] * dL_dc_xx + Tm[0][1] * Tm[1][1] * dL_dc_xy + Tm[1][1] * Tm[1][1] * dL_dc_yy);
        dc[5] = (Tm[0][2] * Tm[0][2] * dL_dc_xx + Tm[0][2] * Tm[1][2] * dL_dc_xy + Tm[1][2] * Tm[1][2] * dL_dc_yy);
        dc[1] = 2 * Tm[0][0] * Tm[0][1] * dL_dc_xx + (Tm[0][0] * Tm[1][1] + Tm[0][1] * Tm[1][0]) * dL_dc_xy + 2 * Tm[1][0] * Tm[1][1] * dL_dc_yy;
        dc[2] = 2 * Tm[0][0] * Tm[0][2] * dL_dc_xx + (Tm[0][0] * Tm[1][2] + Tm[0][2] * Tm[1][0]) * dL_dc_xy + 2 * Tm[1][0] * Tm[1][2] * dL_dc_yy;
        dc[4] = 2 * Tm[0][2] * Tm[0][1] * dL_dc_xx + (Tm[0][1] * Tm[1][2] + Tm[0][2] * Tm[1][1]) * dL_dc_xy + 2 * Tm[1][1] * Tm[1][2] * dL_dc_yy;
    } else {
        for (int i = 0; i < 6; i++) dc[i] = 0;
    }
    const float (*Tm)[3] = T.m;
    const float (*V)[3] = Vrk.m;
    float dL_dT00 = 2 * (Tm[0][0] * V[0][0] + Tm[0][1] * V[0][1] + Tm[0][2] * V[0][2]) * dL_dc_xx +
                    (Tm[1][0] * V[0][0] + Tm[1][1] * V[0][1] + Tm[1][2] * V[0][2]) * dL_dc_xy;
    float dL_dT01 = 2 * (Tm[0][0] * V[1][0] + Tm[0][1] * V[1][1] + Tm[0][2] * V[1][2]) * dL_dc_xx +
                    (Tm[1][0] * V[1][0] + Tm[1][1] * V[1][1] + Tm[1][2] * V[1][2]) * dL_dc_xy;
    float dL_dT02 = 2 * (Tm[0][0] * V[2][0] + Tm[0][1] * V[2][1] + Tm[0][2] * V[2][2]) * dL_dc_xx +
                    (Tm[1][0] * V[2][0] + Tm[1][1] * V[2][1] + Tm[1][2] * V[2][2]) * dL_dc_xy;
    float dL_dT10 = 2 * (Tm[1][0] * V[0][0] + Tm[1][1] * V[0][1] + Tm[1][2] * V[0][2]) * dL_dc_yy +
                    (Tm[0][0] * V[0][0] + Tm[0][1] * V[0][1] + Tm[0][2] * V[0][2]) * dL_dc_xy;
    float dL_dT11 = 2 * (Tm[1][0] * V[1][0] + Tm[1][1] * V[1][1] + Tm[1][2] * V[1][2]) * dL_dc_yy +
                    (Tm[0][0] * V[1][0] + Tm[0][1] * V[1][1] + Tm[0][2] * V[1][2]) * dL_dc_xy;
    float dL_dT12 = 2 * (Tm[1][0] * V[2][0] + Tm[1][1] * V[2][1] + Tm[1][2] * V[2][2]) * dL_dc_yy +
                    (Tm[0][0] * V[2][0] + Tm[0][1] * V[2][1] + Tm[0][2] * V[2][2]) * dL_dc_xy;
    const float (*Wq)[3] = Wm.m;
    float dL_dJ00 = Wq[0][0] * dL_dT00 + Wq[0][1] * dL_dT01 + Wq[0][2] * dL_dT02;
    float dL_dJ02 = Wq[2][0] * dL_dT00 + Wq[2][1] * dL_dT01 + Wq[2][2] * dL_dT02;
    float dL_dJ11 = Wq[1][0] * dL_dT10 + Wq[1][1] * dL_dT11 + Wq[1][2] * dL_dT12;
    float dL_dJ12 = Wq[2][0] * dL_dT10 + Wq[2][1] * dL_dT11 + Wq[2][2] * dL_dT12;
    float tz = 1.f / t.z;
    float tz2 = tz * tz;
    float tz3 = tz2 * tz;
    float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
    float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
    float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t.x) * tz3 * dL_dJ02 + (2 * h_y * t.y) * tz3 * dL_dJ12;
    if (dL_dinvdepth) dL_dtz -= dL_dinvdepth[idx] / (t.z * t.z);
    f3 dt = {dL_dtx, dL_dty, dL_dtz};
    f3 dL_dmean = transformVec4x3Transpose(dt, view_matrix);
    dL_dmeans[3 * idx + 0] = dL_dmean.x;
    dL_dmeans[3 * idx + 1] = dL_dmean.y;
    dL_dmeans[3 * idx + 2] = dL_dmean.z;
}

/* backward.cu:23-142 (computeColorFromSH backward) */
static void sh_bwd_one(int idx, int deg, int max_coeffs, const float* means, const float* campos, const float* shs,
                       const uint8_t* clamped, const float* dL_dcolor, float* dL_dmeans, float* dL_dshs)
{
    f3 pos = {means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]};
    f3 dir_orig = {pos.x - campos[0], pos.y - campos[1], pos.z - campos[2]};
    float len = sqrtf(dir_orig.x * dir_orig.x + dir_orig.y * dir_orig.y + dir_orig.z * dir_orig.z);
    f3 dir = {dir_orig.x / len, dir_orig.y / len, dir_orig.z / len};
    const float* sh = shs + (size_t)idx * max_coeffs * 3;
    float dRGB[3];
    for (int c = 0; c < 3; c++) {
        dRGB[c] = dL_dcolor[3 * idx + c];
        dRGB[c] *= (clamped[idx] >> c) & 1 ? 0 : 1;
    }
    float dx_[3] = {0, 0, 0}, dy_[3] = {0, 0, 0}, dz_[3] = {0, 0, 0};
    float x = dir.x, y = dir.y, z = dir.z;
    float* dsh = dL_dshs + (size_t)idx * max_coeffs * 3;
#define SETSH(k, coef) for (int c = 0; c < 3; c++) dsh[(k) * 3 + c] = (coef) * dRGB[c]
    float dRGBdsh0 = SH_C0;
    SETSH(0, dRGBdsh0);
    if (deg > 0) {
        float dRGBdsh1 = -SH_C1 * y;
        float dRGBdsh2 = SH_C1 * z;
        float dRGBdsh3 = -SH_C1 * x;
        SETSH(1, dRGBdsh1); SETSH(2, dRGBdsh2); SETSH(3, dRGBdsh3);
        for (int c = 0; c < 3; c++) {
            dx_[c] = -SH_C1 * sh[3 * 3 + c];
            dy_[c] = -SH_C1 * sh[1 * 3 + c];
            dz_[c] = SH_C1 * sh[2 * 3 + c];
        }
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            float dRGBdsh4 = SH_C2[0] * xy;
            float dRGBdsh5 = SH_C2[1] * yz;
            float dRGBdsh6 = SH_C2[2] * (2.f * zz - xx - yy);
            float dRGBdsh7 = SH_C2[3] * xz;
            float dRGBdsh8 = SH_C2[4] * (xx - yy);
            SETSH(4, dRGBdsh4); SETSH(5, dRGBdsh5); SETSH(6, dRGBdsh6); SETSH(7, dRGBdsh7); SETSH(8, dRGBdsh8);
            for (int c = 0; c < 3; c++) {
                const float* s = sh + c;
                dx_[c] += SH_C2[0] * y * s[4 * 3] + SH_C2[2] * 2.f * -x * s[6 * 3] + SH_C2[3] * z * s[7 * 3] + SH_C2[4] * 2.f * x * s[8 * 3];
                dy_[c] += SH_C2[0] * x * s[4 * 3] + SH_C2[1] * z * s[5 * 3] + SH_C2[2] * 2.f * -y * s[6 * 3] + SH_C2[4] * 2.f * -y * s[8 * 3];
                dz_[c] += SH_C2[1] * y * s[5 * 3] + SH_C2[2] * 2.f * 2.f * z * s[6 * 3] + SH_C2[3] * x * s[7 * 3];
            }
            if (deg > 2) {
                float dRGBdsh9 = SH_C3[0] * y * (3.f * xx - yy);
                float dRGBdsh10 = SH_C3[1] * xy * z;
                float dRGBdsh11 = SH_C3[2] * y * (4.f * zz - xx - yy);
                float dRGBdsh12 = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
                float dRGBdsh13 = SH_C3[4] * x * (4.f * zz - xx - yy);
                float dRGBdsh14 = SH_C3[5] * z * (xx - yy);
                float dRGBdsh15 = SH_C3[6] * x * (xx - 3.f * yy);
                SETSH(9, dRGBdsh9); SETSH(10, dRGBdsh10); SETSH(11, dRGBdsh11); SETSH(12, dRGBdsh12);
                SETSH(13, dRGBdsh13); SETSH(14, dRGBdsh14); SETSH(15, dRGBdsh15);
                for (int c = 0; c < 3; c++) {
                    const float* s = sh + c;
                    dx_[c] += (SH_C3[0] * s[9 * 3] * 3.f * 2.f * xy +
                               SH_C3[1] * s[10 * 3] * yz +
                               SH_C3[2] * s[11 * 3] * -2.f * xy +
                               SH_C3[3] * s[12 * 3] * -3.f * 2.f * xz +
                               SH_C3[4] * s[13 * 3] * (-3.f * xx + 4.f * zz - yy) +
                               SH_C3[5] * s[14 * 3] * 2.f * xz +
                               SH_C3[6] * s[15 * 3] * 3.f * (xx - yy));
                    dy_[c] += (SH_C3[0] * s[9 * 3] * 3.f * (xx - yy) +
                               SH_C3[1] * s[10 * 3] * xz +
                               SH_C3[2] * s[11 * 3] * (-3.f * yy + 4.f * zz - xx) +
                               SH_C3[3] * s[12 * 3] * -3.f * 2.f * yz +
                               SH_C3[4] * s[13 * 3] * -2.f * xy +
                               SH_C3[5] * s[14 * 3] * -2.f * yz +
                               SH_C3[6] * s[15 * 3] * -3.f * 2.f * xy);
                    dz_[c] += (SH_C3[1] * s[10 * 3] * xy +
                               SH_C3[2] * s[11 * 3] * 4.f * 2.f * yz +
                               SH_C3[3] * s[12 * 3] * 3.f * (2.f * zz - xx - yy) +
                               SH_C3[4] * s[13 * 3] * 4.f * 2.f * xz +
                               SH_C3[5] * s[14 * 3] * (xx - yy));
                }
            }
        }
    }
#undef SETSH
    /* glm::dot(a,b) = (a.x*b.x + a.y*b.y) + a.z*b.z */
    f3 dL_ddir = {dx_[0] * dRGB[0] + dx_[1] * dRGB[1] + dx_[2] * dRGB[2],
                  dy_[0] * dRGB[0] + dy_[1] * dRGB[1] + dy_[2] * dRGB[2],
                  dz_[0] * dRGB[0] + dz_[1] * dRGB[1] + dz_[2] * dRGB[2]};
    f3 dL_dmean = dnormvdv(dir_orig, dL_ddir);
    dL_dmeans[3 * idx + 0] += dL_dmean.x;
    dL_dmeans[3 * idx + 1] += dL_dmean.y;
    dL_dmeans[3 * idx + 2] += dL_dmean.z;
}

/* backward.cu:330-393 (computeCov3D backward) */
static void cov3d_bwd_one(int idx, const float* scale, float mod, const float* rot, const float* dL_dcov3Ds,
                          float* dL_dscales, float* dL_drots)
{
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    mat3 R = mat3_cols(
        1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
        2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
        2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    mat3 S = mat3_cols(1.0f, 0.0f, 0.0f, 0.0f, 1.0f, 0.0f, 0.0f, 0.0f, 1.0f);
    f3 s = {mod * scale[0], mod * scale[1], mod * scale[2]};
    S.m[0][0] = s.x; S.m[1][1] = s.y; S.m[2][2] = s.z;
    mat3 M = mat3_mul(S, R);
    const float* d = dL_dcov3Ds + 6 * (size_t)idx;
    mat3 dL_dSigma = mat3_cols(d[0], 0.5f * d[1], 0.5f * d[2],
                               0.5f * d[1], d[3], 0.5f * d[4],
                               0.5f * d[2], 0.5f * d[4], d[5]);
    /* glm: 2.0f * M (scalar * mat) then * dL_dSigma */
    mat3 M2;
    for (int c = 0; c < 3; c++) for (int w = 0; w < 3; w++) M2.m[c][w] = 2.0f * M.m[c][w];
    mat3 dL_dM = mat3_mul(M2, dL_dSigma);
    mat3 Rt = mat3_T(R);
    mat3 dL_dMt = mat3_T(dL_dM);
    float* ds = dL_dscales + 3 * (size_t)idx;
    ds[0] = Rt.m[0][0] * dL_dMt.m[0][0] + Rt.m[0][1] * dL_dMt.m[0][1] + Rt.m[0][2] * dL_dMt.m[0][2];
    ds[1] = Rt.m[1][0] * dL_dMt.m[1][0] + Rt.m[1][1] * dL_dMt.m[1][1] + Rt.m[1][2] * dL_dMt.m[1][2];
    ds[2] = Rt.m[2][0] * dL_dMt.m[2][0] + Rt.m[2][1] * dL_dMt.m[2][1] + Rt.m[2][2] * dL_dMt.m[2][2];
    for (int w = 0; w < 3; w++) { dL_dMt.m[0][w] *= s.x; dL_dMt.m[1][w] *= s.y; dL_dMt.m[2][w] *= s.z; }
    const float (*G)[3] = dL_dMt.m;
    float* dq = dL_drots + 4 * (size_t)idx;
    dq[0] = 2 * z * (G[0][1] - G[1][0]) + 2 * y * (G[2][0] - G[0][2]) + 2 * x * (G[1][2] - G[2][1]);
    dq[1] = 2 * y * (G[1][0] + G[0][1]) + 2 * z * (G[2][0] + G[0][2]) + 2 * r * (G[1][2] - G[2][1]) - 4 * x * (G[2][2] + G[1][1]);
    dq[2] = 2 * x * (G[1][0] + G[0][1]) + 2 * r * (G[2][0] - G[0][2]) + 2 * z * (G[1][2] + G[2][1]) - 4 * y * (G[2][2] + G[0][0]);
    dq[3] = 2 * r * (G[0][1] - G[1][0]) + 2 * x * (G[2][0] + G[0][2]) + 2 * y * (G[1][2] + G[2][1]) - 4 * z * (G[1][1] + G[0][0]);
}

/* rasterizer_impl.cu:345-450 (Rasterizer::backward) + rasterize_points.cu:163-182 (zero-init).
 * All outputs are fully written here (zeros for culled Gaussians). dL_dinvdepth may be NULL
 * (rasterize_points.cu:176-182). */
int gsr_oracle_backward(void* p, const float* bg, const float* means3D, const float* shs,
                        const float* colors_precomp, const float* opacities, const float* scales,
                        float scale_modifier, const float* rotations, const float* cov3D_precomp,
                        const float* viewmatrix, const float* projmatrix, const float* campos,
                        float tan_fovx, float tan_fovy, const float* dL_dpix, const float* dL_dinvdepth_pix,
                        float* dL_dmean2D, float* dL_dconic, float* dL_dopacity, float* dL_dcolor,
                        float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale, float* dL_drot,
                        int nthreads)
{
    oracle_state* st = (oracle_state*)p;
    set_threads(nthreads);
    const int P = st->P, W = st->W, H = st->H, D = st->D, M = st->M;
    size_t Pn = (size_t)P;
    memset(dL_dmean2D, 0, Pn * 12);
    memset(dL_dconic, 0, Pn * 16);
    memset(dL_dopacity, 0, Pn * 4);
    memset(dL_dcolor, 0, Pn * 12);
    memset(dL_dmean3D, 0, Pn * 12);
    memset(dL_dcov3D, 0, Pn * 24);
    if (M > 0) memset(dL_dsh, 0, Pn * M * 12);
    memset(dL_dscale, 0, Pn * 12);
    memset(dL_drot, 0, Pn * 16);
    if (P == 0) return 0;
    float* dL_dinvdepths = dL_dinvdepth_pix ? (float*)calloc(Pn, 4) : NULL;

    const float focal_y = H / (2.0f * tan_fovy);
    const float focal_x = W / (2.0f * tan_fovx);
    const float* color_ptr = colors_precomp ? colors_precomp : st->rgb;
    size_t T = (size_t)st->gx * st->gy;
    if (g_bwd_f64) {
        double* acc = (double*)calloc(Pn * 12, sizeof(double));  /* mean2D 3 | conic 4 | opacity 1 | colour 3 | invdepth 1 */
        uint32_t maxlen = 0;
        for (size_t t = 0; t < T; t++) maxlen = maxlen > st->ranges[2 * t + 1] - st->ranges[2 * t] ? maxlen : st->ranges[2 * t + 1] - st->ranges[2 * t];
        if (!acc) return -1;
        int fail = 0;
#pragma omp parallel
        {
            double* scratch = (double*)malloc(((size_t)maxlen + 1) * 4 * sizeof(double));
            if (!scratch) {
#pragma omp atomic write
                fail = 1;
            } else {
#pragma omp for schedule(dynamic, 4)
                for (int t = 0; t < (int)T; t++)
                    render_bwd_tile_f64(st, (uint32_t)t % st->gx, (uint32_t)t / st->gx, bg, color_ptr, dL_dpix,
                                        dL_dinvdepth_pix, acc, acc + 3 * Pn, acc + 7 * Pn, acc + 8 * Pn, acc + 11 * Pn,
                                        scratch);
                free(scratch);
            }
        }
        if (fail) {
            free(acc);
            return -1;
        }
        for (size_t i = 0; i < 3 * Pn; i++) dL_dmean2D[i] = (float)acc[i];
        for (size_t i = 0; i < 4 * Pn; i++) dL_dconic[i] = (float)acc[3 * Pn + i];
        for (size_t i = 0; i < Pn; i++) dL_dopacity[i] = (float)acc[7 * Pn + i];
        for (size_t i = 0; i < 3 * Pn; i++) dL_dcolor[i] = (float)acc[8 * Pn + i];
        if (dL_dinvdepths)
            for (size_t i = 0; i < Pn; i++) dL_dinvdepths[i] = (float)acc[11 * Pn + i];
        free(acc);
    } else if (g_bwd_tile_sums) {
        uint32_t maxlen = 0;
        for (size_t t = 0; t < T; t++) maxlen = maxlen > st->ranges[2 * t + 1] - st->ranges[2 * t] ? maxlen : st->ranges[2 * t + 1] - st->ranges[2 * t];
        int fail = 0;
#pragma omp parallel
        {
            float* ts = (float*)malloc(((size_t)maxlen + 1) * TS_N * sizeof(float));
            if (!ts) {
#pragma omp atomic write
                fail = 1;
            } else {
#pragma omp for schedule(dynamic, 4)
                for (int t = 0; t < (int)T; t++)
                    render_bwd_tile(st, (uint32_t)t % st->gx, (uint32_t)t / st->gx, bg, color_ptr, dL_dpix,
                                    dL_dinvdepth_pix, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor, dL_dinvdepths, ts);
                free(ts);
            }
        }
        if (fail) return -1;
    } else {
#pragma omp parallel for schedule(dynamic, 4)
        for (int t = 0; t < (int)T; t++)
            render_bwd_tile(st, (uint32_t)t % st->gx, (uint32_t)t / st->gx, bg, color_ptr, dL_dpix, dL_dinvdepth_pix,
                            dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor, dL_dinvdepths, NULL);
    }

    const float* cov3D_ptr = cov3D_precomp ? cov3D_precomp : st->cov3D;
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        if (!(st->radii[idx] > 0)) continue;
        cov2d_bwd_one(idx, means3D, cov3D_ptr, focal_x, focal_y, tan_fovx, tan_fovy, viewmatrix, opacities,
                      dL_dconic, dL_dopacity, dL_dinvdepths, dL_dmean3D, dL_dcov3D, st->antialiasing);
    }
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        if (!(st->radii[idx] > 0)) continue;
        /* backward.cu:423-440 */
        f3 m = {means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]};
        const float* proj = projmatrix;
        f4 m_hom = transformPoint4x4(m, proj);
        float m_w = 1.0f / (m_hom.w + 0.0000001f);
        float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        const float* g2 = dL_dmean2D + 3 * (size_t)idx;
        float dmx = (proj[0] * m_w - proj[3] * mul1) * g2[0] + (proj[1] * m_w - proj[3] * mul2) * g2[1];
        float dmy = (proj[4] * m_w - proj[7] * mul1) * g2[0] + (proj[5] * m_w - proj[7] * mul2) * g2[1];
        float dmz = (proj[8] * m_w - proj[11] * mul1) * g2[0] + (proj[9] * m_w - proj[11] * mul2) * g2[1];
        dL_dmean3D[3 * idx + 0] += dmx;
        dL_dmean3D[3 * idx + 1] += dmy;
        dL_dmean3D[3 * idx + 2] += dmz;
        if (shs) sh_bwd_one(idx, D, M, means3D, campos, shs, st->clamped, dL_dcolor, dL_dmean3D, dL_dsh);
        if (scales) cov3d_bwd_one(idx, scales + 3 * (size_t)idx, scale_modifier, rotations + 4 * (size_t)idx,
                                  dL_dcov3D, dL_dscale, dL_drot);
    }
    free(dL_dinvdepths);
    return 0;
}

int gsr_oracle_num_tiles(void* p) { oracle_state* st = (oracle_state*)p; return (int)(st->gx * st->gy); }
