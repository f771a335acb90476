// preprocess_bwd.hip -- BACKWARD::preprocess (backward.cu:640-712): the
// reference's two per-Gaussian kernels computeCov2DCUDA (backward.cu:147-326)
// and preprocessCUDA (backward.cu:398-449, with computeColorFromSH :23-142 and
// computeCov3D :330-393) fused into one gfx950 kernel, one thread per
// Gaussian.  Every output row is written (zeros for culled Gaussians), so the
// caller does not have to pre-zero dL_dmean3D / dL_dcov3D / dL_dsh /
// dL_dscale / dL_drot.  HBM-bound: reads ~236 B/G of parameters + the 44 B/G
// gradient record, writes ~232 B/G.
#include "gsr_common.h"
#include "gsr_kernels.h"

namespace gsr {

__device__ __forceinline__ float sq(float x) { return x * x; }

// Per-Gaussian inputs, loaded before the workgroup's SH staging so that their memory round trips
// overlap it (and each other): every load is issued unconditionally (clamped indices, values
// masked after), so no branch sits between a load and the next one.
struct BwdIn {
    bool visible;
    float g[GF_NUM];  // sums of this Gaussian's per-tile gradient records
    float4 co;        // conic + (rendered) opacity
    float cov[6];
    f3 mean;
    float4 rot;
    f3 scale;
    float opacity;
    uint8_t clamped;
};

__device__ __forceinline__ void bwd_gather(const PreprocessBwdArgs& a, int idx, BwdIn& in)
{
    const size_t i = (size_t)idx;
    in.visible = a.radii[idx] > 0;
    in.co = a.conic_opacity[idx];
    if (a.cov3D_precomp) {  // uniform over the launch
#pragma unroll
        for (int k = 0; k < 6; k++) in.cov[k] = a.cov3D_precomp[6 * i + k];
    }
    in.mean = {a.means3D[3 * i], a.means3D[3 * i + 1], a.means3D[3 * i + 2]};
    in.opacity = a.opacities[idx];
    in.clamped = a.clamped[idx];
    if (a.scales) {  // uniform over the launch
        const float* rp = a.rotations + 4 * i;
        in.rot = make_float4(rp[0], rp[1], rp[2], rp[3]);
        in.scale = {a.scales[3 * i], a.scales[3 * i + 1], a.scales[3 * i + 2]};
    }
#pragma unroll
    for (int q = 0; q < GF_NUM; q++) in.g[q] = 0.f;
    // This Gaussian's records are contiguous (emission order); entries that contributed to no
    // pixel were never written (valid = 0) and are not read (most slots: records are sparse).
    // Eight flags per step in flight together, then the flagged records; the sum order stays
    // the slot order (bitwise reproducible).
    const uint32_t e0 = a.emit_start[idx];
    const uint32_t e1 = e0 + a.tiles_touched[idx];  // 0 tiles for culled Gaussians
    for (uint32_t e = e0; e < e1; e += 8) {
        bool v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = a.valid[min(e + k, e1 - 1)] != 0 && e + k < e1;
        float4 r[8][3];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (v[k]) {
                const float4* rec = reinterpret_cast<const float4*>(a.grad_inst + (size_t)(e + k) * GRAD_REC);
                r[k][0] = rec[0];
                r[k][1] = rec[1];
                r[k][2] = rec[2];
            }
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (v[k]) {
                float* g = in.g;
                g[0] += r[k][0].x; g[1] += r[k][0].y; g[2] += r[k][0].z; g[3] += r[k][0].w;
                g[4] += r[k][1].x; g[5] += r[k][1].y; g[6] += r[k][1].z; g[7] += r[k][1].w;
                g[8] += r[k][2].x; g[9] += r[k][2].y;
            }
        }
    }
}

// One Gaussian.  `sh` / `dsh` point at this Gaussian's SH coefficients and SH gradient,
// either in global memory or in the workgroup's LDS staging slot (the same slot for both).
__device__ __forceinline__ void preprocess_bwd_one(const PreprocessBwdArgs& a, int idx, const BwdIn& in,
                                                   const float* sh, float* dsh)
{
    const size_t i = (size_t)idx;
    float* dmean = a.dL_dmean3D + 3 * i;
    float* dcov = a.dL_dcov3D + 6 * i;

    if (!in.visible) {
        a.dL_dmean2D[3 * i] = 0.f; a.dL_dmean2D[3 * i + 1] = 0.f; a.dL_dmean2D[3 * i + 2] = 0.f;
        a.dL_dconic[4 * i] = 0.f; a.dL_dconic[4 * i + 1] = 0.f; a.dL_dconic[4 * i + 2] = 0.f;
        a.dL_dconic[4 * i + 3] = 0.f;
        a.dL_dopacity[i] = 0.f;
        a.dL_dcolor[3 * i] = 0.f; a.dL_dcolor[3 * i + 1] = 0.f; a.dL_dcolor[3 * i + 2] = 0.f;
        if (a.dL_dinvdepth) a.dL_dinvdepth[i] = 0.f;
        dmean[0] = 0.f; dmean[1] = 0.f; dmean[2] = 0.f;
#pragma unroll
        for (int k = 0; k < 6; k++) dcov[k] = 0.f;
        if (dsh)
            for (int k = 0; k < a.M * 3; k++) dsh[k] = 0.f;
        if (a.dL_dscale) { a.dL_dscale[3 * i] = 0.f; a.dL_dscale[3 * i + 1] = 0.f; a.dL_dscale[3 * i + 2] = 0.f; }
        if (a.dL_drot) { float* dr = a.dL_drot + 4 * i; dr[0] = 0.f; dr[1] = 0.f; dr[2] = 0.f; dr[3] = 0.f; }
        return;
    }

    float g[GF_NUM];
#pragma unroll
    for (int q = 0; q < GF_NUM; q++) g[q] = in.g[q];
    {
        // per-Gaussian factors of the record sums (see GradField; backward.cu:619-636)
        const float4 co = in.co;
        const float op = co.w;
        const float sx = g[GF_MEAN2D_X], sy = g[GF_MEAN2D_Y];
        g[GF_MEAN2D_X] = (co.x * sx + co.y * sy) * (-op * (0.5f * a.W));
        g[GF_MEAN2D_Y] = (co.y * sx + co.z * sy) * (-op * (0.5f * a.H));
        g[GF_CONIC_A] *= -0.5f * op;
        g[GF_CONIC_B] *= -0.5f * op;
        g[GF_CONIC_C] *= -0.5f * op;
    }
    // render-pass gradients of the reference glue (rasterize_points.cu:164-172), fully written
    a.dL_dmean2D[3 * i] = g[GF_MEAN2D_X]; a.dL_dmean2D[3 * i + 1] = g[GF_MEAN2D_Y]; a.dL_dmean2D[3 * i + 2] = 0.f;
    a.dL_dconic[4 * i] = g[GF_CONIC_A]; a.dL_dconic[4 * i + 1] = g[GF_CONIC_B]; a.dL_dconic[4 * i + 2] = 0.f;
    a.dL_dconic[4 * i + 3] = g[GF_CONIC_C];
    a.dL_dcolor[3 * i] = g[GF_COLOR_R]; a.dL_dcolor[3 * i + 1] = g[GF_COLOR_G]; a.dL_dcolor[3 * i + 2] = g[GF_COLOR_B];
    if (a.dL_dinvdepth) a.dL_dinvdepth[i] = g[GF_INVDEPTH];

    // ---------------- computeCov2DCUDA (backward.cu:147-326) ----------------
    float cov_local[6];
    const float* cov3D = in.cov;
    if (!a.cov3D_precomp) {  // forward.cu:114-151 recomputed (bit-identical to the forward's)
        const float scl[3] = {in.scale.x, in.scale.y, in.scale.z};
        computeCov3D(scl, a.scale_modifier, in.rot, cov_local);
        cov3D = cov_local;
    }
    const f3 mean = in.mean;
    const f3 dL_dconic = {g[GF_CONIC_A], g[GF_CONIC_B], g[GF_CONIC_C]};
    const float* view = a.view;
    f3 t = transformPoint4x3(mean, view);
    const float limx = 1.3f * a.tan_fovx;
    const float limy = 1.3f * a.tan_fovy;
    const float txtz = t.x / t.z;
    const float tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
    const float h_x = a.focal_x, h_y = a.focal_y;
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
    if (a.antialiasing) {
        const float det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const float det_cov_plus_h_cov = c_xx * c_yy - c_xy * c_xy;
        const float h_convolution_scaling = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus_h_cov));
        const float dL_dopacity_v = g[GF_OPACITY];
        const float d_h_convolution_scaling = dL_dopacity_v * in.opacity;
        a.dL_dopacity[idx] = dL_dopacity_v * h_convolution_scaling;
        d_inside_root = (det_cov / det_cov_plus_h_cov) <= 0.000025f ? 0.f
                                                                    : d_h_convolution_scaling / (2 * h_convolution_scaling);
    } else {
        c_xx += h_var;
        c_yy += h_var;
        a.dL_dopacity[idx] = g[GF_OPACITY];
    }
    float dL_dc_xx = 0, dL_dc_xy = 0, dL_dc_yy = 0;
    if (a.antialiasing) {
        const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
        const float denom_f = d_inside_root / sq(w * w + w * (x + y) + x * y - z * z);
        dL_dc_xx = w * (w * y + y * y + z * z) * denom_f;
        dL_dc_yy = w * (w * x + x * x + z * z) * denom_f;
        dL_dc_xy = -2.f * w * z * (w + x + y) * denom_f;
    }
    const float denom = c_xx * c_yy - c_xy * c_xy;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    const float(*Tm)[3] = T.m;
    if (denom2inv != 0) {
        dL_dc_xx += denom2inv * (-c_yy * c_yy * dL_dconic.x + 2 * c_xy * c_yy * dL_dconic.y +
                                 (denom - c_xx * c_yy) * dL_dconic.z);
        dL_dc_yy += denom2inv * (-c_xx * c_xx * dL_dconic.z + 2 * c_xx * c_xy * dL_dconic.y +
                                 (denom - c_xx * c_yy) * dL_dconic.x);
        dL_dc_xy += denom2inv * 2 *
                    (c_xy * c_yy * dL_dconic.x - (denom + 2 * c_xy * c_xy) * dL_dconic.y + c_xx * c_xy * dL_dconic.z);
        dcov[0] = (Tm[0][0] * Tm[0][0] * dL_dc_xx + Tm[0][0] * Tm[1][0] * dL_dc_xy + Tm[1][0] * Tm[1][0] * dL_dc_yy);
        dcov[3] = (Tm[0][1] * Tm[0][1] * dL_dc_xx + Tm[0][1] * Tm[1][1] * dL_dc_xy + Tm[1][1] * Tm[1][1] * dL_dc_yy);
        dcov[5] = (Tm[0][2] * Tm[0][2] * dL_dc_xx + Tm[0][2] * Tm[1][2] * dL_dc_xy + Tm[1][2] * Tm[1][2] * dL_dc_yy);
        dcov[1] = 2 * Tm[0][0] * Tm[0][1] * dL_dc_xx + (Tm[0][0] * Tm[1][1] + Tm[0][1] * Tm[1][0]) * dL_dc_xy +
                  2 * Tm[1][0] * Tm[1][1] * dL_dc_yy;
        dcov[2] = 2 * Tm[0][0] * Tm[0][2] * dL_dc_xx + (Tm[0][0] * Tm[1][2] + Tm[0][2] * Tm[1][0]) * dL_dc_xy +
                  2 * Tm[1][0] * Tm[1][2] * dL_dc_yy;
        dcov[4] = 2 * Tm[0][2] * Tm[0][1] * dL_dc_xx + (Tm[0][1] * Tm[1][2] + Tm[0][2] * Tm[1][1]) * dL_dc_xy +
                  2 * Tm[1][1] * Tm[1][2] * dL_dc_yy;
    } else {
#pragma unroll
        for (int k = 0; k < 6; k++) dcov[k] = 0;
    }
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
        const float* proj = a.proj;
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

    // ---------------- computeColorFromSH backward (backward.cu:23-142) ----------------
    if (a.shs) {
        const int deg = a.D;
        const f3 dir_orig = {mean.x - a.campos[0], mean.y - a.campos[1], mean.z - a.campos[2]};
        const float len = sqrtf(dir_orig.x * dir_orig.x + dir_orig.y * dir_orig.y + dir_orig.z * dir_orig.z);
        const float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
        const uint8_t cl = in.clamped;
        float dRGB[3];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            dRGB[c] = g[GF_COLOR_R + c];
            dRGB[c] *= (cl >> c) & 1 ? 0 : 1;
        }
        float ddx[3] = {0, 0, 0}, ddy[3] = {0, 0, 0}, ddz[3] = {0, 0, 0};
        // dRGB/dsh_k coefficients; dL_dsh is written after every read of sh (sh and dsh may
        // share an LDS slot), coefficient k * dRGB exactly as backward.cu:51-100.
        float coef[16];
        int ncoef = 0;
#define SETSH(k, cf)      \
    do {                  \
        coef[k] = (cf);   \
        ncoef = (k) + 1;  \
    } while (0)
        const float dRGBdsh0 = SH_C0;
        SETSH(0, dRGBdsh0);
        if (deg > 0) {
            const float dRGBdsh1 = -SH_C1 * y;
            const float dRGBdsh2 = SH_C1 * z;
            const float dRGBdsh3 = -SH_C1 * x;
            SETSH(1, dRGBdsh1);
            SETSH(2, dRGBdsh2);
            SETSH(3, dRGBdsh3);
#pragma unroll
            for (int c = 0; c < 3; c++) {
                ddx[c] = -SH_C1 * sh[3 * 3 + c];
                ddy[c] = -SH_C1 * sh[1 * 3 + c];
                ddz[c] = SH_C1 * sh[2 * 3 + c];
            }
            if (deg > 1) {
                const float xx = x * x, yy = y * y, zz = z * z;
                const float xy = x * y, yz = y * z, xz = x * z;
                SETSH(4, SH_C2_0 * xy);
                SETSH(5, SH_C2_1 * yz);
                SETSH(6, SH_C2_2 * (2.f * zz - xx - yy));
                SETSH(7, SH_C2_3 * xz);
                SETSH(8, SH_C2_4 * (xx - yy));
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const float* s = sh + c;
                    ddx[c] += SH_C2_0 * y * s[4 * 3] + SH_C2_2 * 2.f * -x * s[6 * 3] + SH_C2_3 * z * s[7 * 3] +
                              SH_C2_4 * 2.f * x * s[8 * 3];
                    ddy[c] += SH_C2_0 * x * s[4 * 3] + SH_C2_1 * z * s[5 * 3] + SH_C2_2 * 2.f * -y * s[6 * 3] +
                              SH_C2_4 * 2.f * -y * s[8 * 3];
                    ddz[c] += SH_C2_1 * y * s[5 * 3] + SH_C2_2 * 2.f * 2.f * z * s[6 * 3] + SH_C2_3 * x * s[7 * 3];
                }
                if (deg > 2) {
                    SETSH(9, SH_C3_0 * y * (3.f * xx - yy));
                    SETSH(10, SH_C3_1 * xy * z);
                    SETSH(11, SH_C3_2 * y * (4.f * zz - xx - yy));
                    SETSH(12, SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy));
                    SETSH(13, SH_C3_4 * x * (4.f * zz - xx - yy));
                    SETSH(14, SH_C3_5 * z * (xx - yy));
                    SETSH(15, SH_C3_6 * x * (xx - 3.f * yy));
#pragma unroll
                    for (int c = 0; c < 3; c++) {
                        const float* s = sh + c;
                        ddx[c] += (SH_C3_0 * s[9 * 3] * 3.f * 2.f * xy + SH_C3_1 * s[10 * 3] * yz +
                                   SH_C3_2 * s[11 * 3] * -2.f * xy + SH_C3_3 * s[12 * 3] * -3.f * 2.f * xz +
                                   SH_C3_4 * s[13 * 3] * (-3.f * xx + 4.f * zz - yy) +
                                   SH_C3_5 * s[14 * 3] * 2.f * xz + SH_C3_6 * s[15 * 3] * 3.f * (xx - yy));
                        ddy[c] += (SH_C3_0 * s[9 * 3] * 3.f * (xx - yy) + SH_C3_1 * s[10 * 3] * xz +
                                   SH_C3_2 * s[11 * 3] * (-3.f * yy + 4.f * zz - xx) +
                                   SH_C3_3 * s[12 * 3] * -3.f * 2.f * yz + SH_C3_4 * s[13 * 3] * -2.f * xy +
                                   SH_C3_5 * s[14 * 3] * -2.f * yz + SH_C3_6 * s[15 * 3] * -3.f * 2.f * xy);
                        ddz[c] += (SH_C3_1 * s[10 * 3] * xy + SH_C3_2 * s[11 * 3] * 4.f * 2.f * yz +
                                   SH_C3_3 * s[12 * 3] * 3.f * (2.f * zz - xx - yy) +
                                   SH_C3_4 * s[13 * 3] * 4.f * 2.f * xz + SH_C3_5 * s[14 * 3] * (xx - yy));
                    }
                }
            }
        }
#undef SETSH
        {
            const int kmax = a.M < 16 ? a.M : 16;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                if (k < kmax) {
#pragma unroll
                    for (int c = 0; c < 3; c++) dsh[k * 3 + c] = k < ncoef ? coef[k] * dRGB[c] : 0.f;
                }
            }
            for (int k = 48; k < a.M * 3; k++) dsh[k] = 0.f;
        }
        const f3 dL_ddir = {ddx[0] * dRGB[0] + ddx[1] * dRGB[1] + ddx[2] * dRGB[2],
                            ddy[0] * dRGB[0] + ddy[1] * dRGB[1] + ddy[2] * dRGB[2],
                            ddz[0] * dRGB[0] + ddz[1] * dRGB[1] + ddz[2] * dRGB[2]};
        const f3 dn = dnormvdv(dir_orig, dL_ddir);
        dmx += dn.x;
        dmy += dn.y;
        dmz += dn.z;
    }
    dmean[0] = dmx;
    dmean[1] = dmy;
    dmean[2] = dmz;

    // ---------------- computeCov3D backward (backward.cu:330-393) ----------------
    if (a.scales) {
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
        const float* d = dcov;
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
        float* ds = a.dL_dscale + 3 * i;
        ds[0] = Rt.m[0][0] * G.m[0][0] + Rt.m[0][1] * G.m[0][1] + Rt.m[0][2] * G.m[0][2];
        ds[1] = Rt.m[1][0] * G.m[1][0] + Rt.m[1][1] * G.m[1][1] + Rt.m[1][2] * G.m[1][2];
        ds[2] = Rt.m[2][0] * G.m[2][0] + Rt.m[2][1] * G.m[2][1] + Rt.m[2][2] * G.m[2][2];
#pragma unroll
        for (int w = 0; w < 3; w++) { G.m[0][w] *= s.x; G.m[1][w] *= s.y; G.m[2][w] *= s.z; }
        const float(*gm)[3] = G.m;
        float4 dq;
        dq.x = 2 * z * (gm[0][1] - gm[1][0]) + 2 * y * (gm[2][0] - gm[0][2]) + 2 * x * (gm[1][2] - gm[2][1]);
        dq.y = 2 * y * (gm[1][0] + gm[0][1]) + 2 * z * (gm[2][0] + gm[0][2]) + 2 * r * (gm[1][2] - gm[2][1]) -
               4 * x * (gm[2][2] + gm[1][1]);
        dq.z = 2 * x * (gm[1][0] + gm[0][1]) + 2 * r * (gm[2][0] - gm[0][2]) + 2 * z * (gm[1][2] + gm[2][1]) -
               4 * y * (gm[2][2] + gm[0][0]);
        dq.w = 2 * r * (gm[0][1] - gm[1][0]) + 2 * x * (gm[2][0] + gm[0][2]) + 2 * y * (gm[1][2] + gm[2][1]) -
               4 * z * (gm[1][1] + gm[0][0]);
        float* dr = a.dL_drot + 4 * i;
        dr[0] = dq.x; dr[1] = dq.y; dr[2] = dq.z; dr[3] = dq.w;
    } else {
        if (a.dL_dscale) { a.dL_dscale[3 * i] = 0.f; a.dL_dscale[3 * i + 1] = 0.f; a.dL_dscale[3 * i + 2] = 0.f; }
        if (a.dL_drot) { float* dr = a.dL_drot + 4 * i; dr[0] = 0.f; dr[1] = 0.f; dr[2] = 0.f; dr[3] = 0.f; }
    }
}

// SH coefficients (48 floats per Gaussian at degree 3) are the bulk of this kernel's
// traffic.  STAGED: the workgroup's 256 x 3M floats are read with coalesced 16-byte loads
// into LDS (row stride padded to an odd number of dwords, so the 64 lanes walking their own
// rows hit 64 different banks), each thread works on its row in place, and the SH gradients leave the same way -- instead
// of every lane striding 192 B through global memory.
template <bool STAGED>
__global__ void __launch_bounds__(256) preprocess_bwd_kernel(PreprocessBwdArgs a, int lds_stride)
{
    extern __shared__ __attribute__((aligned(16))) float s_sh[];
    const int base = blockIdx.x * 256;
    const int idx = base + (int)threadIdx.x;
    BwdIn in;
    if (idx < a.P) bwd_gather(a, idx, in);  // in flight during the SH staging below
    if (!STAGED) {
        if (idx < a.P) {
            const size_t w3 = (size_t)a.M * 3;
            preprocess_bwd_one(a, idx, in, a.shs ? a.shs + idx * w3 : nullptr,
                               a.dL_dsh ? a.dL_dsh + idx * w3 : nullptr);
        }
        return;
    }
    const int W3 = a.M * 3;  // multiple of 4 on this path
    const int n = min(256, a.P - base);
    const int nv4 = n * (W3 / 4);
    const float4* src = reinterpret_cast<const float4*>(a.shs + (size_t)base * W3);
    for (int f = threadIdx.x; f < nv4; f += 256) {
        const int g = (f * 4) / W3, w = (f * 4) - g * W3;
        const float4 v = src[f];
        float* d = &s_sh[g * lds_stride + w];
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
    __syncthreads();
    if (idx < a.P) {
        float* row = s_sh + threadIdx.x * lds_stride;
        preprocess_bwd_one(a, idx, in, row, row);
    }
    __syncthreads();
    float4* dst = reinterpret_cast<float4*>(a.dL_dsh + (size_t)base * W3);
    for (int f = threadIdx.x; f < nv4; f += 256) {
        const int g = (f * 4) / W3, w = (f * 4) - g * W3;
        const float* q = &s_sh[g * lds_stride + w];
        dst[f] = make_float4(q[0], q[1], q[2], q[3]);
    }
}

hipError_t launch_preprocess_bwd(const PreprocessBwdArgs& a, hipStream_t s)
{
    if (a.P <= 0) return hipSuccess;
    const int W3 = a.M * 3;
    const bool staged = a.shs && a.dL_dsh && W3 > 0 && W3 % 4 == 0 && W3 <= 64 &&
                        ((uintptr_t)a.shs % 16) == 0 && ((uintptr_t)a.dL_dsh % 16) == 0;
    if (staged) {
        const int stride = W3 | 1;  // odd number of dwords per row: the per-thread row walks are conflict-free
        hipLaunchKernelGGL(preprocess_bwd_kernel<true>, dim3((a.P + 255) / 256), dim3(256),
                           256 * stride * sizeof(float), s, a, stride);
    } else {
        hipLaunchKernelGGL(preprocess_bwd_kernel<false>, dim3((a.P + 255) / 256), dim3(256), 0, s, a, 0);
    }
    return hipGetLastError();
}

}  // namespace gsr
