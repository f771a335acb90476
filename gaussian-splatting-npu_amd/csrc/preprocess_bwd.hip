// preprocess_bwd.hip -- BACKWARD::preprocess (backward.cu:640-712): the
// reference's two per-Gaussian kernels computeCov2DCUDA (backward.cu:147-326)
// and preprocessCUDA (backward.cu:398-449, with computeColorFromSH :23-142 and
// computeCov3D :330-393) fused into one gfx950 kernel for one view or a batch
// of views: LPG lanes per Gaussian, one per view (one lane for a single view,
// gsr_backward).  Every output row is written (zeros for culled Gaussians), so the
// caller does not have to pre-zero dL_dmean3D / dL_dcov3D / dL_dsh /
// dL_dscale / dL_drot.  HBM-bound: reads ~236 B/G of parameters + the 44 B/G
// gradient record, writes ~232 B/G.
#include "gsr_common.h"
#include "gsr_kernels.h"

namespace gsr {

__device__ __forceinline__ float sq(float x) { return x * x; }


// One output element: written, or added to when the caller accumulates into it (AccBits).
__device__ __forceinline__ void put(float* p, float v, bool acc) { *p = acc ? *p + v : v; }
// the same with the old value already loaded (bwd_gather prefetches them)
__device__ __forceinline__ void put(float* p, float v, bool acc, float old) { *p = acc ? old + v : v; }

// Per-Gaussian inputs, loaded before the workgroup's SH staging so that their memory round trips
// overlap it (and each other): every load is issued unconditionally (clamped indices, values
// masked after), so no branch sits between a load and the next one.
struct BwdIn {
    float cov[6];
    f3 mean;
    float4 rot;
    f3 scale;
    float opacity;
    // accumulating (AccBits): the outputs' current values, loaded here with everything else
    float old_mean[3], old_opacity, old_scale[3], old_rot[4];
};

// records in flight per lane (the V lanes of a Gaussian already gather side by side; twice as many
// at one lane per Gaussian)
#ifndef GSR_VIEW_REC_BATCH
#define GSR_VIEW_REC_BATCH 4
#endif
constexpr int REC_BATCH = GSR_VIEW_REC_BATCH;

// B records (slots sl[k], v[k]: present) loaded side by side, then added to g in slot order.
template <int B>
__device__ __forceinline__ void rec_batch(const bool (&v)[B], const uint32_t (&sl)[B], const float* grad_inst,
                                          float (&g)[GF_NUM])
{
    float r[B][GF_NUM];
#pragma unroll
    for (int k = 0; k < B; k++) {
        if (v[k]) {
            if constexpr (GRAD_REC % 4 == 0) {  // 16-B aligned records
                const float4* rec = reinterpret_cast<const float4*>(grad_inst + (size_t)sl[k] * GRAD_REC);
                const float4 a0 = rec[0], a1 = rec[1], a2 = rec[2];
                r[k][0] = a0.x; r[k][1] = a0.y; r[k][2] = a0.z; r[k][3] = a0.w;
                r[k][4] = a1.x; r[k][5] = a1.y; r[k][6] = a1.z; r[k][7] = a1.w;
                r[k][8] = a2.x; r[k][9] = a2.y;
            } else {  // packed 40-B records
                const float2* rec = reinterpret_cast<const float2*>(grad_inst + (size_t)sl[k] * GRAD_REC);
#pragma unroll
                for (int h = 0; h < GF_NUM / 2; h++) {
                    const float2 x = rec[h];
                    r[k][2 * h] = x.x;
                    r[k][2 * h + 1] = x.y;
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < B; k++) {
        if (v[k]) {
#pragma unroll
            for (int q = 0; q < GF_NUM; q++) g[q] += r[k][q];
        }
    }
}

// Sum of one Gaussian's per-tile gradient records of one view.  Its records are contiguous
// (slots [emit_start, + tiles_touched)); entries that contributed to no pixel were never written (their bit in the valid
// mask is 0) and are not read (most slots: records are sparse).  The mask has one bit per slot
// (L/8 bytes: it stays in L2), so a Gaussian's flags are one or two words; its flagged records are
// then read B at a time in slot order (bitwise reproducible sums).
template <int B = REC_BATCH, bool INIT = true>
__device__ __forceinline__ void gather_range(uint32_t e0, uint32_t e1, const uint32_t* valid, const float* grad_inst,
                                             float (&g)[GF_NUM])
{
    if (INIT) {
#pragma unroll
        for (int q = 0; q < GF_NUM; q++) g[q] = 0.f;
    }
    for (uint32_t w0 = e0 & ~31u; w0 < e1; w0 += 32) {
        uint32_t bits = valid[w0 >> 5];
        if (w0 < e0) bits &= ~0u << (e0 - w0);
        if (e1 - w0 < 32u) bits &= (1u << (e1 - w0)) - 1u;
        while (bits) {
            bool v[B];
            uint32_t sl[B];
#pragma unroll
            for (int k = 0; k < B; k++) {
                v[k] = bits != 0u;
                sl[k] = w0 + (v[k] ? (uint32_t)__builtin_ctz(bits) : 0u);
                bits &= bits - 1u;
            }
            rec_batch<B>(v, sl, grad_inst, g);
        }
    }
}

// The records of a Gaussian with at most 32 slots from its own record mask (bit k: slot e0 + k holds
// a record, render_bwd), loaded beside e0 and n: no dependent load of the valid words.  Same slot
// order as gather_range: the same sums bit for bit.
template <int B = REC_BATCH>
__device__ __forceinline__ void gather_mask(uint32_t e0, uint32_t bits, const float* grad_inst, float (&g)[GF_NUM])
{
#pragma unroll
    for (int q = 0; q < GF_NUM; q++) g[q] = 0.f;
    while (bits) {
        bool v[B];
        uint32_t sl[B];
#pragma unroll
        for (int k = 0; k < B; k++) {
            v[k] = bits != 0u;
            sl[k] = e0 + (v[k] ? (uint32_t)__builtin_ctz(bits) : 0u);
            bits &= bits - 1u;
        }
        rec_batch<B>(v, sl, grad_inst, g);
    }
}

// One Gaussian's records of one view: its first 32 slots by its record mask, the rest (Gaussians
// of more than 32 tiles only) through the valid words -- render_bwd flags each record in exactly one
// of the two.  Slot order throughout: the sums are those of one walk over the valid words, bit for bit.
template <int B = REC_BATCH>
__device__ __forceinline__ void gather_any(uint32_t e0, uint32_t n, uint32_t mask, const uint32_t* valid,
                                           const float* grad_inst, float (&g)[GF_NUM])
{
    if (!GSR_REC_MASK) {
        gather_range<B>(e0, e0 + n, valid, grad_inst, g);
        return;
    }
    gather_mask<B>(e0, mask, grad_inst, g);
    if (n > 32u) gather_range<B, false>(e0 + 32u, e0 + n, valid, grad_inst, g);
}

// The per-Gaussian parameters (and, accumulating, the outputs' old values).
__device__ __forceinline__ void bwd_gather(const PreprocessBwdArgs& a, int idx, BwdIn& in)
{
    const size_t i = (size_t)idx;
    if (a.cov3D_precomp) {  // uniform over the launch
#pragma unroll
        for (int k = 0; k < 6; k++) in.cov[k] = a.cov3D_precomp[6 * i + k];
    }
    in.mean = {a.means3D[3 * i], a.means3D[3 * i + 1], a.means3D[3 * i + 2]};
    in.opacity = a.opacities[idx];
    if (a.scales) {  // uniform over the launch
        const float* rp = a.rotations + 4 * i;
        in.rot = make_float4(rp[0], rp[1], rp[2], rp[3]);
        in.scale = {a.scales[3 * i], a.scales[3 * i + 1], a.scales[3 * i + 2]};
    }
    if (a.acc & ACC_MEANS3D) {
        in.old_mean[0] = a.dL_dmean3D[3 * i]; in.old_mean[1] = a.dL_dmean3D[3 * i + 1];
        in.old_mean[2] = a.dL_dmean3D[3 * i + 2];
    }
    if (a.acc & ACC_OPACITY) in.old_opacity = a.dL_dopacity[i];
    if (a.acc & ACC_SCALES) {
        in.old_scale[0] = a.dL_dscale[3 * i]; in.old_scale[1] = a.dL_dscale[3 * i + 1];
        in.old_scale[2] = a.dL_dscale[3 * i + 2];
    }
    if (a.acc & ACC_ROTATIONS) {  // the destination is the caller's .grad: no alignment assumed
        const float* r = a.dL_drot + 4 * i;
        in.old_rot[0] = r[0]; in.old_rot[1] = r[1]; in.old_rot[2] = r[2]; in.old_rot[3] = r[3];
    }
}

// Coefficient k's factor dRGB/dsh_k (backward.cu:51-100, same expressions: dL/dsh is
// bit-identical) and its derivatives along the normalised view direction (the per-coefficient
// terms of dRGBdx / dRGBdy / dRGBdz, backward.cu:60-127).  k is a compile-time constant after
// unrolling, so the switch folds away.
__device__ __forceinline__ void sh_term(int k, float x, float y, float z, float& b, float& gx, float& gy, float& gz)
{
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    gx = gy = gz = 0.f;
    switch (k) {
    case 0: b = SH_C0; break;
    case 1: b = -SH_C1 * y; gy = -SH_C1; break;
    case 2: b = SH_C1 * z; gz = SH_C1; break;
    case 3: b = -SH_C1 * x; gx = -SH_C1; break;
    case 4: b = SH_C2_0 * xy; gx = SH_C2_0 * y; gy = SH_C2_0 * x; break;
    case 5: b = SH_C2_1 * yz; gy = SH_C2_1 * z; gz = SH_C2_1 * y; break;
    case 6:
        b = SH_C2_2 * (2.f * zz - xx - yy);
        gx = SH_C2_2 * 2.f * -x; gy = SH_C2_2 * 2.f * -y; gz = SH_C2_2 * 2.f * 2.f * z;
        break;
    case 7: b = SH_C2_3 * xz; gx = SH_C2_3 * z; gz = SH_C2_3 * x; break;
    case 8: b = SH_C2_4 * (xx - yy); gx = SH_C2_4 * 2.f * x; gy = SH_C2_4 * 2.f * -y; break;
    case 9: b = SH_C3_0 * y * (3.f * xx - yy); gx = SH_C3_0 * 3.f * 2.f * xy; gy = SH_C3_0 * 3.f * (xx - yy); break;
    case 10: b = SH_C3_1 * xy * z; gx = SH_C3_1 * yz; gy = SH_C3_1 * xz; gz = SH_C3_1 * xy; break;
    case 11:
        b = SH_C3_2 * y * (4.f * zz - xx - yy);
        gx = SH_C3_2 * -2.f * xy; gy = SH_C3_2 * (-3.f * yy + 4.f * zz - xx); gz = SH_C3_2 * 4.f * 2.f * yz;
        break;
    case 12:
        b = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
        gx = SH_C3_3 * -3.f * 2.f * xz; gy = SH_C3_3 * -3.f * 2.f * yz; gz = SH_C3_3 * 3.f * (2.f * zz - xx - yy);
        break;
    case 13:
        b = SH_C3_4 * x * (4.f * zz - xx - yy);
        gx = SH_C3_4 * (-3.f * xx + 4.f * zz - yy); gy = SH_C3_4 * -2.f * xy; gz = SH_C3_4 * 4.f * 2.f * xz;
        break;
    case 14: b = SH_C3_5 * z * (xx - yy); gx = SH_C3_5 * 2.f * xz; gy = SH_C3_5 * -2.f * yz; gz = SH_C3_5 * (xx - yy); break;
    default: b = SH_C3_6 * x * (xx - 3.f * yy); gx = SH_C3_6 * 3.f * (xx - yy); gy = SH_C3_6 * -3.f * 2.f * xy; break;
    }
}

// One camera of the backward: the launch's own (single view) or an entry of the multi-view table.
struct ViewCam {
    const float* view;
    const float* proj;
    const float* campos;
    float focal_x, focal_y, tan_fovx, tan_fovy;
};

// One view's contribution to one visible Gaussian's gradients (no memory access).
struct ViewGrad {
    float g[GF_NUM];      // record sums with the per-Gaussian factors applied (dL/dmean2D, dL/dconic)
    float dopacity;       // dL/dopacity (rescaled by the AA factor with antialiasing)
    float dcov[6];        // dL/dcov3D
    float dmx, dmy, dmz;  // dL/dmean3D without the view-direction (SH) term
    f3 dir_orig;          // SH set-up: mean - campos, its normalisation and the unclamped dL/dcolor
    float x, y, z;
    float dRGB[3];
};

// The 3D covariance of a Gaussian: precomputed, or recomputed from scale and rotation
// (forward.cu:114-151; bit-identical to the forward's).  Always into the local array: a pointer
// choosing between two arrays would force both into scratch memory.
__device__ __forceinline__ void cov3d_of(const PreprocessBwdArgs& a, const BwdIn& in, float (&cov)[6])
{
    if (a.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; k++) cov[k] = in.cov[k];
        return;
    }
    const float scl[3] = {in.scale.x, in.scale.y, in.scale.z};
    computeCov3D(scl, a.scale_modifier, in.rot, cov);
}

// computeCov2DCUDA (backward.cu:147-326), the projection part of preprocessCUDA
// (backward.cu:423-440) and the set-up of computeColorFromSH's backward (backward.cu:28-49) for
// one view: `gin` are the view's record sums, `co` its conic + rendered opacity.
// The view's conic and (AA-scaled) opacity -- GeometryState's conic_opacity, which the batched
// forward does not store -- are recomputed here from the 2D covariance this function recomputes
// anyway, with the forward's own operations (preprocess.hip preprocess_one, -ffp-contract=off):
// bit-identical to the stored values.
__device__ __forceinline__ void view_grad(const PreprocessBwdArgs& a, const ViewCam& vc, const float (&gin)[GF_NUM],
                                          uint8_t clamped, const f3 mean, float opacity, const float (&cov3D)[6],
                                          ViewGrad& o)
{
    float* g = o.g;
#pragma unroll
    for (int q = 0; q < GF_NUM; q++) g[q] = gin[q];

    // ---------------- computeCov2DCUDA (backward.cu:147-326) ----------------
    const float* view = vc.view;
    f3 t = transformPoint4x3(mean, view);
    const float limx = 1.3f * vc.tan_fovx;
    const float limy = 1.3f * vc.tan_fovy;
    const float txtz = t.x / t.z;
    const float tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
    const float h_x = vc.focal_x, h_y = vc.focal_y;
    const mat3 J = mat3_cols(h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z),
                             0.0f, h_y / t.z, -(h_y * t.y) / (t.z * t.z), 0, 0, 0);
    const mat3 Wm = mat3_cols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    const mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4],
                               cov3D[5]);
    const mat3 T = mat3_mul(Wm, J);
    const mat3 cov2D = mat3_mul(mat3_mul(mat3_T(T), mat3_T(Vrk)), T);
    float c_xx = cov2D.m[0][0];
    float c_xy = cov2D.m[0][1];
    float c_yy = cov2D.m[1][1];
    const float h_var = 0.3f;
    float d_inside_root = 0.f;
    float op = opacity;  // the opacity the render blended (forward.cu:262-266)
    if (a.antialiasing) {
        const float det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const float det_cov_plus_h_cov = c_xx * c_yy - c_xy * c_xy;
        const float h_convolution_scaling = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus_h_cov));
        op = opacity * h_convolution_scaling;
        const float dL_dopacity_v = g[GF_OPACITY];
        const float d_h_convolution_scaling = dL_dopacity_v * opacity;
        o.dopacity = dL_dopacity_v * h_convolution_scaling;
        d_inside_root = (det_cov / det_cov_plus_h_cov) <= 0.000025f ? 0.f
                                                                    : d_h_convolution_scaling / (2 * h_convolution_scaling);
    } else {
        c_xx += h_var;
        c_yy += h_var;
        o.dopacity = g[GF_OPACITY];
    }
    const float denom = c_xx * c_yy - c_xy * c_xy;
    {
        // the conic (forward.cu:218-222 as preprocess_one computes it), then the per-Gaussian
        // factors of the record sums (see GradField; backward.cu:619-636)
        const float det_inv = 1.f / denom;
        const float cx = c_yy * det_inv, cy = -c_xy * det_inv, cz = c_xx * det_inv;
        const float sx = g[GF_MEAN2D_X], sy = g[GF_MEAN2D_Y];
        g[GF_MEAN2D_X] = (cx * sx + cy * sy) * (-op * (0.5f * a.W));
        g[GF_MEAN2D_Y] = (cy * sx + cz * sy) * (-op * (0.5f * a.H));
        g[GF_CONIC_A] *= -0.5f * op;
        g[GF_CONIC_B] *= -0.5f * op;
        g[GF_CONIC_C] *= -0.5f * op;
    }
    const f3 dL_dconic = {g[GF_CONIC_A], g[GF_CONIC_B], g[GF_CONIC_C]};
    float dL_dc_xx = 0, dL_dc_xy = 0, dL_dc_yy = 0;
    if (a.antialiasing) {
        const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
        const float denom_f = d_inside_root / sq(w * w + w * (x + y) + x * y - z * z);
        dL_dc_xx = w * (w * y + y * y + z * z) * denom_f;
        dL_dc_yy = w * (w * x + x * x + z * z) * denom_f;
        dL_dc_xy = -2.f * w * z * (w + x + y) * denom_f;
    }
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    const float(*Tm)[3] = T.m;
    float* dcov = o.dcov;
    // denom2inv == 0 (backward.cu:230-283): no conic terms and dL/dcov3D = 0 -- as selects, not a
    // branch (a divergent branch here made the compiler spill dcov to scratch)
    const bool nz = denom2inv != 0;
    dL_dc_xx += nz ? denom2inv * (-c_yy * c_yy * dL_dconic.x + 2 * c_xy * c_yy * dL_dconic.y +
                                  (denom - c_xx * c_yy) * dL_dconic.z)
                   : 0.f;
    dL_dc_yy += nz ? denom2inv * (-c_xx * c_xx * dL_dconic.z + 2 * c_xx * c_xy * dL_dconic.y +
                                  (denom - c_xx * c_yy) * dL_dconic.x)
                   : 0.f;
    dL_dc_xy += nz ? denom2inv * 2 *
                         (c_xy * c_yy * dL_dconic.x - (denom + 2 * c_xy * c_xy) * dL_dconic.y + c_xx * c_xy * dL_dconic.z)
                   : 0.f;
    dcov[0] = (Tm[0][0] * Tm[0][0] * dL_dc_xx + Tm[0][0] * Tm[1][0] * dL_dc_xy + Tm[1][0] * Tm[1][0] * dL_dc_yy);
    dcov[3] = (Tm[0][1] * Tm[0][1] * dL_dc_xx + Tm[0][1] * Tm[1][1] * dL_dc_xy + Tm[1][1] * Tm[1][1] * dL_dc_yy);
    dcov[5] = (Tm[0][2] * Tm[0][2] * dL_dc_xx + Tm[0][2] * Tm[1][2] * dL_dc_xy + Tm[1][2] * Tm[1][2] * dL_dc_yy);
    dcov[1] = 2 * Tm[0][0] * Tm[0][1] * dL_dc_xx + (Tm[0][0] * Tm[1][1] + Tm[0][1] * Tm[1][0]) * dL_dc_xy +
              2 * Tm[1][0] * Tm[1][1] * dL_dc_yy;
    dcov[2] = 2 * Tm[0][0] * Tm[0][2] * dL_dc_xx + (Tm[0][0] * Tm[1][2] + Tm[0][2] * Tm[1][0]) * dL_dc_xy +
              2 * Tm[1][0] * Tm[1][2] * dL_dc_yy;
    dcov[4] = 2 * Tm[0][2] * Tm[0][1] * dL_dc_xx + (Tm[0][1] * Tm[1][2] + Tm[0][2] * Tm[1][1]) * dL_dc_xy +
              2 * Tm[1][1] * Tm[1][2] * dL_dc_yy;
#pragma unroll
    for (int k = 0; k < 6; k++) dcov[k] = nz ? dcov[k] : 0.f;
    const float(*V)[3] = Vrk.m;
    const float dL_dT00 = 2 * (Tm[0][0] * V[0][0] + Tm[0][1] * V[0][1] + Tm[0][2] * V[0][2]) * dL_dc_xx +
                          (Tm[1][0] * V[0][0] + Tm[1][1] * V[0][1] + Tm[1][2] * V[0][2]) * dL_dc_xy;
    const float dL_dT01 = 2 * (Tm[0][0] * V[1][0] + Tm[0][1] * V[1][1] + Tm[0][2] * V[1][2]) * dL_dc_xx +
                          (Tm[1][0] * V[1][0] + Tm[1][1] * V[1][1] + Tm[1][2] * V[1][2]) * dL_dc_xy;
    const float dL_dT02 = 2 * (Tm[0][0] * V[2][0] + Tm[0][1] * V[2][1] + Tm[0][2] * V[2][2]) * dL_dc_xx +
                          (Tm[1][0] * V[2][0] + Tm[1][1] * V[2][1] + Tm[1][2] * V[2][2]) * dL_dc_xy;
    const float dL_dT10 = 2 * (Tm[1][0] * V[0][0] + Tm[1][1] * V[0][1] + Tm[1][2] * V[0][2]) * dL_dc_yy +
                          (Tm[0][0] * V[0][0] + Tm[0][1] * V[0][1] + Tm[0][2] * V[0][2]) * dL_dc_xy;
    const float dL_dT11 = 2 * (Tm[1][0] * V[1][0] + Tm[1][1] * V[1][1] + Tm[1][2] * V[1][2]) * dL_dc_yy +
                          (Tm[0][0] * V[1][0] + Tm[0][1] * V[1][1] + Tm[0][2] * V[1][2]) * dL_dc_xy;
    const float dL_dT12 = 2 * (Tm[1][0] * V[2][0] + Tm[1][1] * V[2][1] + Tm[1][2] * V[2][2]) * dL_dc_yy +
                          (Tm[0][0] * V[2][0] + Tm[0][1] * V[2][1] + Tm[0][2] * V[2][2]) * dL_dc_xy;
    const float(*Wq)[3] = Wm.m;
    const float dL_dJ00 = Wq[0][0] * dL_dT00 + Wq[0][1] * dL_dT01 + Wq[0][2] * dL_dT02;
    const float dL_dJ02 = Wq[2][0] * dL_dT00 + Wq[2][1] * dL_dT01 + Wq[2][2] * dL_dT02;
    const float dL_dJ11 = Wq[1][0] * dL_dT10 + Wq[1][1] * dL_dT11 + Wq[1][2] * dL_dT12;
    const float dL_dJ12 = Wq[2][0] * dL_dT10 + Wq[2][1] * dL_dT11 + Wq[2][2] * dL_dT12;
    const float tz = 1.f / t.z;
    const float tz2 = tz * tz;
    const float tz3 = tz2 * tz;
    const float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
    const float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
    float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t.x) * tz3 * dL_dJ02 +
                   (2 * h_y * t.y) * tz3 * dL_dJ12;
    if (a.has_invdepth) dL_dtz -= g[GF_INVDEPTH] / (t.z * t.z);
    const f3 dm_cov = transformVec4x3Transpose({dL_dtx, dL_dty, dL_dtz}, view);
    float dmx = dm_cov.x, dmy = dm_cov.y, dmz = dm_cov.z;

    // ---------------- preprocessCUDA (backward.cu:423-440) ----------------
    {
        const float* proj = vc.proj;
        const f3 m = mean;
        const float4 m_hom = transformPoint4x4(m, proj);
        const float m_w = 1.0f / (m_hom.w + 0.0000001f);
        const float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        const float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        const float g2x = g[GF_MEAN2D_X], g2y = g[GF_MEAN2D_Y];
        dmx += (proj[0] * m_w - proj[3] * mul1) * g2x + (proj[1] * m_w - proj[3] * mul2) * g2y;
        dmy += (proj[4] * m_w - proj[7] * mul1) * g2x + (proj[5] * m_w - proj[7] * mul2) * g2y;
        dmz += (proj[8] * m_w - proj[11] * mul1) * g2x + (proj[9] * m_w - proj[11] * mul2) * g2y;
    }
    o.dmx = dmx;
    o.dmy = dmy;
    o.dmz = dmz;

    // ---------------- computeColorFromSH backward: set-up (backward.cu:28-49) ----------------
    if (a.shs || a.dc) {
        o.dir_orig = {mean.x - vc.campos[0], mean.y - vc.campos[1], mean.z - vc.campos[2]};
        const f3 d = o.dir_orig;
        const float len = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
        o.x = d.x / len;
        o.y = d.y / len;
        o.z = d.z / len;
#pragma unroll
        for (int c = 0; c < 3; c++) o.dRGB[c] = g[GF_COLOR_R + c] * ((clamped >> c) & 1 ? 0 : 1);
    }
}

// SH coefficients in use: (D + 1)^2, at most M and 16 (0: colors_precomp)
__device__ __forceinline__ int sh_ncoef(const PreprocessBwdArgs& a)
{
    if (!a.shs && !a.dc) return 0;
    int nc = (a.D + 1) * (a.D + 1);
    nc = nc < a.M ? nc : a.M;
    return nc < 16 ? nc : 16;
}

// computeCov3D backward (backward.cu:330-393): dL/dscale and dL/drot (w.r.t. the given, assumed
// unit quaternion) from dL/dcov3D.
__device__ __forceinline__ void cov3d_bwd(const PreprocessBwdArgs& a, const BwdIn& in, const float* d, float (&ds)[3],
                                          float4& dq)
{
    const float r = in.rot.x, x = in.rot.y, y = in.rot.z, z = in.rot.w;
    const mat3 R = mat3_cols(
        1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
        2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
        2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    mat3 S = mat3_cols(1.0f, 0.0f, 0.0f, 0.0f, 1.0f, 0.0f, 0.0f, 0.0f, 1.0f);
    const float mod = a.scale_modifier;
    const f3 s = {mod * in.scale.x, mod * in.scale.y, mod * in.scale.z};
    S.m[0][0] = s.x; S.m[1][1] = s.y; S.m[2][2] = s.z;
    const mat3 M = mat3_mul(S, R);
    const mat3 dL_dSigma = mat3_cols(d[0], 0.5f * d[1], 0.5f * d[2], 0.5f * d[1], d[3], 0.5f * d[4],
                                     0.5f * d[2], 0.5f * d[4], d[5]);
    mat3 M2;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int w = 0; w < 3; w++) M2.m[c][w] = 2.0f * M.m[c][w];
    const mat3 dL_dM = mat3_mul(M2, dL_dSigma);
    const mat3 Rt = mat3_T(R);
    mat3 G = mat3_T(dL_dM);
    ds[0] = Rt.m[0][0] * G.m[0][0] + Rt.m[0][1] * G.m[0][1] + Rt.m[0][2] * G.m[0][2];
    ds[1] = Rt.m[1][0] * G.m[1][0] + Rt.m[1][1] * G.m[1][1] + Rt.m[1][2] * G.m[1][2];
    ds[2] = Rt.m[2][0] * G.m[2][0] + Rt.m[2][1] * G.m[2][1] + Rt.m[2][2] * G.m[2][2];
#pragma unroll
    for (int w = 0; w < 3; w++) { G.m[0][w] *= s.x; G.m[1][w] *= s.y; G.m[2][w] *= s.z; }
    const float(*gm)[3] = G.m;
    dq.x = 2 * z * (gm[0][1] - gm[1][0]) + 2 * y * (gm[2][0] - gm[0][2]) + 2 * x * (gm[1][2] - gm[2][1]);
    dq.y = 2 * y * (gm[1][0] + gm[0][1]) + 2 * z * (gm[2][0] + gm[0][2]) + 2 * r * (gm[1][2] - gm[2][1]) -
           4 * x * (gm[2][2] + gm[1][1]);
    dq.z = 2 * x * (gm[1][0] + gm[0][1]) + 2 * r * (gm[2][0] - gm[0][2]) + 2 * z * (gm[1][2] + gm[2][1]) -
           4 * y * (gm[2][2] + gm[0][0]);
    dq.w = 2 * r * (gm[0][1] - gm[1][0]) + 2 * x * (gm[2][0] + gm[0][2]) + 2 * y * (gm[1][2] + gm[2][1]) -
           4 * z * (gm[1][1] + gm[0][0]);
}

// The scale / rotation outputs from dL/dcov3D (zeros without scales), written or accumulated.
__device__ __forceinline__ void put_scale_rot(const PreprocessBwdArgs& a, int idx, const BwdIn& in, const float* dcov)
{
    const size_t i = (size_t)idx;
    if (a.scales) {
        float ds[3];
        float4 dq;
        cov3d_bwd(a, in, dcov, ds, dq);
        float* dsp = a.dL_dscale + 3 * i;
        const bool acc_s = a.acc & ACC_SCALES;
        put(dsp, ds[0], acc_s, in.old_scale[0]);
        put(dsp + 1, ds[1], acc_s, in.old_scale[1]);
        put(dsp + 2, ds[2], acc_s, in.old_scale[2]);
        float* dr = a.dL_drot + 4 * i;
        const bool acc_r = a.acc & ACC_ROTATIONS;
        put(dr, dq.x, acc_r, in.old_rot[0]); put(dr + 1, dq.y, acc_r, in.old_rot[1]);
        put(dr + 2, dq.z, acc_r, in.old_rot[2]); put(dr + 3, dq.w, acc_r, in.old_rot[3]);
    } else {
        if (a.dL_dscale && !(a.acc & ACC_SCALES)) {
            a.dL_dscale[3 * i] = 0.f; a.dL_dscale[3 * i + 1] = 0.f; a.dL_dscale[3 * i + 2] = 0.f;
        }
        if (a.dL_drot && !(a.acc & ACC_ROTATIONS)) {
            float* dr = a.dL_drot + 4 * i; dr[0] = 0.f; dr[1] = 0.f; dr[2] = 0.f; dr[3] = 0.f;
        }
    }
}

// SH coefficients (48 floats per Gaussian at degree 3) are the bulk of this kernel's traffic.
// STAGED (M = 16): the workgroup's 256 rows are read with coalesced 16-byte loads into LDS rows
// padded to 49 dwords (an odd stride: the 64 lanes walking their own rows hit 64 different
// banks), each thread works on its row in place, and the SH gradients leave the same way.
// (Staging in two 24-float halves halves the LDS and raises occupancy, but measured 3 % slower:
// most 128-B lines of a row are then fetched in both halves.)
constexpr int SH_STRIDE = 49;  // LDS dwords per row (odd)

// ---- multi-view batch (gsr_backward_views) ------------------------------------------------
// LPG lanes per Gaussian (the next power of two >= V), lane v of a group working on view v: its
// records, the 2D chain rule (view_grad), that view's screen-space gradient and the SH terms of
// that view's direction.  The per-view contributions to dL/dcov3D, dL/dmean3D, dL/dopacity,
// dL/dcolor and dL/dsh are summed over the group's lanes with DPP butterflies (a fixed tree: the
// sums are identical in every lane and reproducible), and scale / rotation are differentiated once
// from the summed dL/dcov3D (linear in it).  The parameters (236 B per Gaussian at degree 3) are
// read and their gradients written once per batch instead of once per view, and the V views'
// dependent gathers (records) are in flight side by side instead of one after another.
// x from another lane of its DPP row (CTRL: a dpp_ctrl code)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}

// x summed over the LPG consecutive lanes of this lane's group (LPG <= 16: within one DPP row).
// Every lane of the group must be active.
template <int LPG>
__device__ __forceinline__ float group_sum(float x)
{
    if constexpr (LPG >= 2) x += dpp_mov<0xB1>(x);   // quad_perm [1,0,3,2]: lane ^ 1
    if constexpr (LPG >= 4) x += dpp_mov<0x4E>(x);   // quad_perm [2,3,0,1]: lane ^ 2
    if constexpr (LPG >= 8) x += dpp_mov<0x141>(x);  // row_half_mirror: the other quad of 8 lanes
    if constexpr (LPG >= 16) x += dpp_mov<0x140>(x); // row_mirror: the other half of the row
    return x;
}

// A lane's view inputs, loaded in the kernel's prologue (unconditionally, clamped), so that their
// round trip overlaps the SH staging and the record gather is the only dependent one after it.
struct ViewIn {
    uint8_t cl;
    uint32_t e0, n;  // record slots [e0, e0 + n)
    uint32_t mask;   // which of the first 32 hold a record
    bool drawn;      // the single-view launch (a.radii set): radius > 0 (backward.cu:420)
};

__device__ __forceinline__ void view_load(const PreprocessBwdViewsArgs& A, int idx, int v, ViewIn& vi)
{
    const BwdView& bv = A.v[v < A.V ? v : 0];
    vi.cl = bv.clamped[idx];
    vi.e0 = bv.emit_start[idx];
    vi.n = bv.tiles_touched[idx];
    vi.mask = bv.rec_mask[idx];
    vi.drawn = A.a.radii ? A.a.radii[idx] > 0 : true;
}

// The batch's cameras in LDS (view 16, proj 16, campos 3, focal_x, focal_y, tan_fovx, tan_fovy),
// read by the lanes of each view instead of through two dependent global loads per lane.  The rows
// are GSR_CAM_STRIDE floats apart: an odd stride puts the 8 views' copies of one camera field in 8
// different banks (a 40-float stride put views v and v + 4 in one bank: every camera read of a
// wave, which holds lanes of all 8 views, took two LDS cycles).
#ifndef GSR_CAM_STRIDE
#define GSR_CAM_STRIDE 41
#endif
constexpr int CAM_FLOATS = GSR_CAM_STRIDE;
__device__ __forceinline__ void cams_to_lds(const PreprocessBwdViewsArgs& A, float (*s_cam)[CAM_FLOATS])
{
    for (int t = threadIdx.x; t < A.V * CAM_FLOATS; t += blockDim.x) {
        const int v = t / CAM_FLOATS, j = t - v * CAM_FLOATS;
        const BwdView& bv = A.v[v];
        float x = 0.f;
        if (j < 16) x = bv.view[j];
        else if (j < 32) x = bv.proj[j - 16];
        else if (j < 35) x = bv.campos[j - 32];
        else if (j == 35) x = bv.focal_x;
        else if (j == 36) x = bv.focal_y;
        else if (j == 37) x = bv.tan_fovx;
        else if (j == 38) x = bv.tan_fovy;
        s_cam[v][j] = x;
    }
}

__device__ __forceinline__ ViewCam cam_of_lds(const float* c)
{
    return {c, c + 16, c + 32, c[35], c[36], c[37], c[38]};
}

// visible <=> radius > 0 (backward.cu:163,420) <=> a tile count > 0: preprocess culls a Gaussian whose
// rect is empty and writes radius 0 and no tiles for every culled one (4 B per view less to read)
// (the single-view launch keeps the reference's test on the caller's radii)
__device__ __forceinline__ bool view_visible_in(const PreprocessBwdViewsArgs& A, bool live, int v, const ViewIn& vi)
{
    return live && v < A.V && (A.a.radii ? vi.drawn : vi.n > 0);
}

template <int LPG>
__device__ __forceinline__ void bwd_views_group_gs(const PreprocessBwdViewsArgs& A, int idx, bool live, int v,
                                                   const BwdIn& in, const ViewIn& vi, const float (&gs)[GF_NUM],
                                                   const float* cam, const float* c0, const float* cr, float* d0,
                                                   float* dr, int kw, bool acc_dc, bool acc_sh);

// One lane's share of a Gaussian of the batch.  c0: SH coefficient 0 (3 floats), cr: coefficient
// k >= 1 at cr[3 (k - 1)]; d0 / dr the same for dL/dsh (may alias c0 / cr: every lane of the group
// reads coefficient k before its sum is written), kw the number of coefficients to write (zeros from
// the first unused one); acc: add to d0 / dr.  `live`: the lane's Gaussian exists (lanes past P
// run the same code on a clamped index, write nothing, and keep every lane in the reductions).
template <int LPG>
__device__ __forceinline__ void bwd_views_group(const PreprocessBwdViewsArgs& A, int idx, bool live, int v,
                                                const BwdIn& in, const ViewIn& vi, const float* cam,
                                                const float* c0, const float* cr, float* d0, float* dr, int kw,
                                                bool acc_dc, bool acc_sh)
{
    const BwdView& bv = A.v[v < A.V ? v : 0];
    float gs[GF_NUM];
    if (view_visible_in(A, live, v, vi)) {
        // one lane per Gaussian: 8 records in flight (145 VGPRs; the SH staging caps it at 3 waves/SIMD
        // anyway): 145 -> 141 us per 1080p view
        gather_any<LPG == 1 ? 2 * REC_BATCH : REC_BATCH>(vi.e0, vi.n, vi.mask, bv.valid, bv.grad_inst, gs);
    } else {
#pragma unroll
        for (int q = 0; q < GF_NUM; q++) gs[q] = 0.f;
    }
    bwd_views_group_gs<LPG>(A, idx, live, v, in, vi, gs, cam, c0, cr, d0, dr, kw, acc_dc, acc_sh);
}

// gs: the lane's view records, summed (zeros for an invisible view)
template <int LPG>
__device__ __forceinline__ void bwd_views_group_gs(const PreprocessBwdViewsArgs& A, int idx, bool live, int v,
                                                   const BwdIn& in, const ViewIn& vi, const float (&gs)[GF_NUM],
                                                   const float* cam, const float* c0, const float* cr, float* d0,
                                                   float* dr, int kw, bool acc_dc, bool acc_sh)
{
    const PreprocessBwdArgs& a = A.a;
    const size_t i = (size_t)idx;
    const bool has_view = live && v < A.V;
    const BwdView& bv = A.v[v < A.V ? v : 0];
    const bool vis = view_visible_in(A, live, v, vi);
    float cov3D[6];
    cov3d_of(a, in, cov3D);
    ViewGrad o;
    if (vis) {
        view_grad(a, cam_of_lds(cam), gs, vi.cl, in.mean, in.opacity, cov3D, o);
    } else {
#pragma unroll
        for (int q = 0; q < GF_NUM; q++) o.g[q] = 0.f;
        o.dopacity = 0.f;
#pragma unroll
        for (int k = 0; k < 6; k++) o.dcov[k] = 0.f;
        o.dmx = o.dmy = o.dmz = 0.f;
        o.dir_orig = {1.f, 0.f, 0.f};
        o.x = o.y = o.z = 0.f;
        o.dRGB[0] = o.dRGB[1] = o.dRGB[2] = 0.f;
    }
    if (has_view) {
        float* m2 = bv.dL_dmean2D + 3 * i;
        m2[0] = o.g[GF_MEAN2D_X]; m2[1] = o.g[GF_MEAN2D_Y]; m2[2] = 0.f;
        if (a.dL_dconic) {  // the single-view launch's other render-pass gradients (rasterize_points.cu:164-172)
            float* dc4 = a.dL_dconic + 4 * i;
            dc4[0] = o.g[GF_CONIC_A]; dc4[1] = o.g[GF_CONIC_B]; dc4[2] = 0.f; dc4[3] = o.g[GF_CONIC_C];
        }
        if (a.dL_dinvdepth) a.dL_dinvdepth[i] = o.g[GF_INVDEPTH];
    }
    const bool writer = live && v == 0;
    {
        const float dop = group_sum<LPG>(o.dopacity);
        if (writer) put(a.dL_dopacity + i, dop, a.acc & ACC_OPACITY, in.old_opacity);
    }
    {
        float dcol[3];
#pragma unroll
        for (int c = 0; c < 3; c++) dcol[c] = group_sum<LPG>(o.g[GF_COLOR_R + c]);
        if (writer && a.dL_dcolor) {
            const bool acc = a.acc & ACC_COLORS;
#pragma unroll
            for (int c = 0; c < 3; c++) put(a.dL_dcolor + 3 * i + c, dcol[c], acc);
        }
    }
    {
        float dcov[6];
#pragma unroll
        for (int k = 0; k < 6; k++) dcov[k] = group_sum<LPG>(o.dcov[k]);
        if (writer) {
#pragma unroll
            for (int k = 0; k < 6; k++) put(a.dL_dcov3D + 6 * i + k, dcov[k], a.acc & ACC_COV3D);
            put_scale_rot(a, idx, in, dcov);
        }
    }
    float dm[3] = {o.dmx, o.dmy, o.dmz};
    const int nc = sh_ncoef(a);
    if (nc > 0) {  // computeColorFromSH backward (backward.cu:51-141) for this lane's view direction
        float ddir[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const bool mine = live && (k % LPG) == v;  // the lane that writes coefficient k
            if (k < nc) {
                float b, gx, gy, gz;
                sh_term(k, o.x, o.y, o.z, b, gx, gy, gz);
                const float* shk = k == 0 ? c0 : cr + 3 * (k - 1);
                float* dk = k == 0 ? d0 : (dr ? dr + 3 * (k - 1) : nullptr);
                const bool acc = k == 0 ? acc_dc : acc_sh;
                float sum[3];
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const float t = shk[c] * o.dRGB[c];
                    sum[c] = group_sum<LPG>(b * o.dRGB[c]);
                    ddir[0] += t * gx;
                    ddir[1] += t * gy;
                    ddir[2] += t * gz;
                }
                if (mine && dk) {
#pragma unroll
                    for (int c = 0; c < 3; c++) put(dk + c, sum[c], acc);
                }
            } else if (k < kw && mine && k > 0 && dr && !acc_sh) {
#pragma unroll
                for (int c = 0; c < 3; c++) dr[3 * (k - 1) + c] = 0.f;
            }
        }
        if (vis && nc > 1) {  // degree 0 has no direction dependence
            const f3 dn = dnormvdv(o.dir_orig, {ddir[0], ddir[1], ddir[2]});
            dm[0] += dn.x;
            dm[1] += dn.y;
            dm[2] += dn.z;
        }
    }
#pragma unroll
    for (int c = 0; c < 3; c++) dm[c] = group_sum<LPG>(dm[c]);
    if (writer) {
        const bool acc_m = a.acc & ACC_MEANS3D;
        float* dmean = a.dL_dmean3D + 3 * i;
        put(dmean, dm[0], acc_m, in.old_mean[0]);
        put(dmean + 1, dm[1], acc_m, in.old_mean[1]);
        put(dmean + 2, dm[2], acc_m, in.old_mean[2]);
    }
}

// The SH rows of a workgroup's n Gaussians (from `base`, at most ROWS) staged through LDS: read
// with coalesced 16-byte loads, work(c0, cr, kw) runs on row r in place, and the rows leave the
// same way (see SH_STRIDE).  Every thread of the workgroup must call this.
template <int ROWS, class Work>
__device__ __forceinline__ void staged_sh(const PreprocessBwdArgs& a, float* s_sh, int base, int n, int r, Work work)
{
    if (a.dc && a.M <= 16) {  // separate dc (train.py's sparse-Adam layout), verbatim rows (see preprocess.hip)
        const int wr = (a.M - 1) * 3;
        float* s_rest = s_sh + 3 * ROWS;
        lds_copy_in(s_sh, a.dc + (size_t)base * 3, n * 3);
        if (wr > 0) lds_copy_in(s_rest, a.shs + (size_t)base * wr, n * wr);
        __syncthreads();
        work(s_sh + 3 * r, s_rest + wr * r, a.M);
        __syncthreads();
        lds_copy_out(a.dL_ddc + (size_t)base * 3, s_sh, n * 3, a.acc & ACC_DC);
        if (wr > 0) lds_copy_out(a.dL_dsh + (size_t)base * wr, s_rest, n * wr, a.acc & ACC_SH);
        return;
    }
    if (a.dc) {  // separate dc, wide rest rows: dc -> columns 0-2, rest -> 3..47
        const int wr = (a.M - 1) * 3;
        lds_rows_in(s_sh, SH_STRIDE, 0, 48, a.dc + (size_t)base * 3, 3, n);
        if (a.shs && wr > 0) lds_rows_in(s_sh, SH_STRIDE, 3, 48, a.shs + (size_t)base * wr, wr, n);
        __syncthreads();
        float* row = s_sh + r * SH_STRIDE;
        work(row, row + 3, 16);
        __syncthreads();
        lds_rows_out(a.dL_ddc + (size_t)base * 3, 3, n, s_sh, SH_STRIDE, 0, 48, a.acc & ACC_DC);
        if (a.dL_dsh && wr > 0)
            lds_rows_out(a.dL_dsh + (size_t)base * wr, wr, n, s_sh, SH_STRIDE, 3, 48, a.acc & ACC_SH);
        return;
    }
    const float4* src = reinterpret_cast<const float4*>(a.shs + (size_t)base * 48);
    auto put = [&](int f, const float4 v) {
        const int g = f / 12, j = f - g * 12;
        float* d = &s_sh[g * SH_STRIDE + 4 * j];
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    };
    // LDS_IN_BATCH loads in flight per thread before their stores (not one round trip each)
    const int bd = (int)blockDim.x;
    int f = threadIdx.x;
    for (; f + (LDS_IN_BATCH - 1) * bd < n * 12; f += LDS_IN_BATCH * bd) {
        float4 v[LDS_IN_BATCH];
#pragma unroll
        for (int u = 0; u < LDS_IN_BATCH; u++) v[u] = src[f + u * bd];
#pragma unroll
        for (int u = 0; u < LDS_IN_BATCH; u++) put(f + u * bd, v[u]);
    }
    for (; f < n * 12; f += bd) put(f, src[f]);
    __syncthreads();
    float* row = s_sh + r * SH_STRIDE;
    work(row, row + 3, 16);
    __syncthreads();
    store_f4(reinterpret_cast<float4*>(a.dL_dsh + (size_t)base * 48), n * 12, a.acc & ACC_SH, [&](int f) {
        const int g = f / 12, j = f - g * 12;
        const float* q = &s_sh[g * SH_STRIDE + 4 * j];
        return make_float4(q[0], q[1], q[2], q[3]);
    });
}

// Shared-memory bytes of staged_sh for ROWS rows (either layout).
constexpr int staged_lds_bytes(int rows) { return rows * SH_STRIDE * 4; }

// The multi-view batch: 256 / LPG Gaussians per workgroup, LPG lanes each (bwd_views_group).
template <int LPG, bool STAGED>
__global__ void __launch_bounds__(256) preprocess_bwd_views_kernel(const PreprocessBwdViewsArgs A)
{
    constexpr int G = 256 / LPG;
    extern __shared__ __attribute__((aligned(16))) float s_sh[];
    const PreprocessBwdArgs& a = A.a;
    const int gl = (int)threadIdx.x / LPG, v = (int)threadIdx.x % LPG;
    // the launch covers Gaussians [g_begin, g_end) (a chunk of the batch: gradient reduction
    // overlapped with the later chunks)
    const int base = A.g_begin + (int)blockIdx.x * G;
    const bool live = base + gl < A.g_end;
    const int idx = live ? base + gl : A.g_end - 1;  // clamped: all lanes take part in the reductions
    __shared__ float s_cam[MAX_VIEWS][CAM_FLOATS];
    BwdIn in;
    bwd_gather(a, idx, in);
    ViewIn vi;
    view_load(A, idx, v, vi);  // in flight during the camera and SH staging
    cams_to_lds(A, s_cam);
    const float* cam = s_cam[v < A.V ? v : 0];
    if (!STAGED) {
        __syncthreads();
        const size_t w3 = (size_t)a.M * 3;
        const float* row = a.shs ? a.shs + idx * w3 : nullptr;
        float* drow = (a.shs && a.dL_dsh) ? a.dL_dsh + idx * w3 : nullptr;
        bwd_views_group<LPG>(A, idx, live, v, in, vi, cam, row, row ? row + 3 : nullptr, drow,
                             drow ? drow + 3 : nullptr, a.M, a.acc & ACC_SH, a.acc & ACC_SH);
        if (live && a.dL_dsh && !(a.acc & ACC_SH))  // columns past the SH coefficients (M > 16 or no SH)
            for (int k = (a.shs ? 48 : 0) + v; k < a.M * 3; k += LPG) a.dL_dsh[idx * w3 + k] = 0.f;
        return;
    }
    staged_sh<G>(a, s_sh, base, min(G, A.g_end - base), gl, [&](float* c0, float* cr, int kw) {
        bwd_views_group<LPG>(A, idx, live, v, in, vi, cam, c0, cr, c0, cr, kw, false, false);
    });
}

// The same work as preprocess_bwd_views_kernel<LPG, true> for the interleaved SH layout, with
// GSR_PBWD_PIPE chunks of G Gaussians per workgroup in straight-line code: every chunk's view
// inputs (record range and mask) are loaded up front, so a later chunk's record gathers are issued
// together with its parameter and SH loads -- one memory round trip before its compute instead of two.
// (As a loop over chunks the compiler keeps ~60 more VGPRs live: 2 waves/SIMD instead of 4.)
#ifndef GSR_PBWD_PIPE
#define GSR_PBWD_PIPE 2  // chunks per workgroup, lane groups (the batch launches; 0: one chunk, the plain kernel)
#endif
#ifndef GSR_PBWD_PIPE1
#define GSR_PBWD_PIPE1 0  // the same for the single view's one lane per Gaussian
#endif
#ifndef GSR_PBWD_PIPE2
#define GSR_PBWD_PIPE2 0  // the same for two lanes per Gaussian (batches of 1-2 views)
#endif
template <int LPG>
__device__ __forceinline__ void pbwd_chunk(const PreprocessBwdViewsArgs& A, float* s_sh, const float* cam, int chunk,
                                           const ViewIn& vi)
{
    constexpr int G = 256 / LPG;
    constexpr int PER = (G * 12 + 255) / 256;  // SH float4 loads per thread and chunk
    const PreprocessBwdArgs& a = A.a;
    const int gl = (int)threadIdx.x / LPG, v = (int)threadIdx.x % LPG;
    const int base = A.g_begin + chunk * G;
    const bool live = base + gl < A.g_end;
    const int idx = min(base + gl, A.g_end - 1);  // clamped: all lanes take part in the reductions
    const int n = min(G, A.g_end - base);
    BwdIn in;
    bwd_gather(a, idx, in);
    const float4* src = reinterpret_cast<const float4*>(a.shs + (size_t)base * 48);
    float4 sv[PER];
#pragma unroll
    for (int u = 0; u < PER; u++) {
        const int f = (int)threadIdx.x + u * 256;
        if (f < n * 12) sv[u] = src[f];
    }
    float gs[GF_NUM];
    if (view_visible_in(A, live, v, vi)) {
        const BwdView& bv = A.v[v < A.V ? v : 0];
        gather_any<REC_BATCH>(vi.e0, vi.n, vi.mask, bv.valid, bv.grad_inst, gs);
    } else {
#pragma unroll
        for (int q = 0; q < GF_NUM; q++) gs[q] = 0.f;
    }
#pragma unroll
    for (int u = 0; u < PER; u++) {
        const int f = (int)threadIdx.x + u * 256;
        if (f < n * 12) {
            const int g = f / 12, j = f - g * 12;
            float* d = &s_sh[g * SH_STRIDE + 4 * j];
            d[0] = sv[u].x; d[1] = sv[u].y; d[2] = sv[u].z; d[3] = sv[u].w;
        }
    }
    __syncthreads();
    float* row = s_sh + gl * SH_STRIDE;
    bwd_views_group_gs<LPG>(A, idx, live, v, in, vi, gs, cam, row, row + 3, row, row + 3, 16, false, false);
    __syncthreads();
    store_f4(reinterpret_cast<float4*>(a.dL_dsh + (size_t)base * 48), n * 12, a.acc & ACC_SH, [&](int f) {
        const int g = f / 12, j = f - g * 12;
        const float* q = &s_sh[g * SH_STRIDE + 4 * j];
        return make_float4(q[0], q[1], q[2], q[3]);
    });
}

template <int LPG, int NCH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LPG == 1 ? 3 : 1)))
preprocess_bwd_views_pipe_kernel(const PreprocessBwdViewsArgs A, int nchunks)
{
    constexpr int G = 256 / LPG;
    extern __shared__ __attribute__((aligned(16))) float s_sh[];
    const int gl = (int)threadIdx.x / LPG, v = (int)threadIdx.x % LPG;
    __shared__ float s_cam[MAX_VIEWS][CAM_FLOATS];
    const int c0 = (int)blockIdx.x * NCH;
    ViewIn vi[NCH];
#pragma unroll
    for (int k = 0; k < NCH; k++) view_load(A, min(A.g_begin + min(c0 + k, nchunks - 1) * G + gl, A.g_end - 1), v, vi[k]);
    cams_to_lds(A, s_cam);  // (read after the first chunk's barrier)
    const float* cam = s_cam[v < A.V ? v : 0];
#pragma unroll
    for (int k = 0; k < NCH; k++) {
        if (c0 + k >= nchunks) break;  // (uniform)
        if (k > 0) __syncthreads();  // the rows are restaged
        pbwd_chunk<LPG>(A, s_sh, cam, c0 + k, vi[k]);
    }
}

static bool staged_layout(const PreprocessBwdArgs& a)
{
    const bool interleaved = a.shs && a.dL_dsh && a.M == 16 && ((uintptr_t)a.shs % 16) == 0 &&
                             ((uintptr_t)a.dL_dsh % 16) == 0;
    return interleaved || (a.dc && a.dL_ddc);
}

template <int LPG>
static hipError_t launch_views(const PreprocessBwdViewsArgs& A, hipStream_t s)
{
    constexpr int G = 256 / LPG;
    const dim3 grid((A.g_end - A.g_begin + G - 1) / G), block(256);
    constexpr int NCH = LPG >= 4 ? GSR_PBWD_PIPE : LPG == 2 ? GSR_PBWD_PIPE2 : GSR_PBWD_PIPE1;
    if constexpr (NCH > 0) {
        if (staged_layout(A.a) && !A.a.dc) {
            const int nchunks = (int)grid.x, blocks = (nchunks + NCH - 1) / NCH;
            hipLaunchKernelGGL((preprocess_bwd_views_pipe_kernel<LPG, NCH>), dim3(blocks), block, staged_lds_bytes(G), s,
                               A, nchunks);
            return hipGetLastError();
        }
    }
    if (staged_layout(A.a))
        hipLaunchKernelGGL((preprocess_bwd_views_kernel<LPG, true>), grid, block, staged_lds_bytes(G), s, A);
    else
        hipLaunchKernelGGL((preprocess_bwd_views_kernel<LPG, false>), grid, block, 0, s, A);
    return hipGetLastError();
}

hipError_t launch_preprocess_bwd_single(const PreprocessBwdViewsArgs& A, hipStream_t s)
{
    if (A.V != 1 || !A.a.radii || A.g_begin != 0 || A.g_end != A.a.P) return hipErrorInvalidValue;
    if (A.a.P <= 0) return hipSuccess;
    return launch_views<1>(A, s);
}

hipError_t launch_preprocess_bwd_views(const PreprocessBwdViewsArgs& A, hipStream_t s)
{
    if (A.V < 1 || A.V > MAX_VIEWS) return hipErrorInvalidValue;
    if (A.g_begin < 0 || A.g_end > A.a.P || A.g_begin > A.g_end) return hipErrorInvalidValue;
    if (A.a.P <= 0 || A.g_end == A.g_begin) return hipSuccess;
    if (A.V <= 2) return launch_views<2>(A, s);
    if (A.V <= 4) return launch_views<4>(A, s);
    if (A.V <= 8) return launch_views<8>(A, s);
    return launch_views<16>(A, s);
}

}  // namespace gsr
