/* gsr_ref_exp.h -- TEST-ONLY float exp(), written once and compiled into two places:
 *
 *   - the GSR_REF_ALPHA=1 test build of render.hip (refalpha/libgsr_hip_refalpha.so, never loaded by
 *     the package), whose render_fwd / render_bwd then compute power and alpha in the reference's
 *     operation order (forward.cu:353-363, backward.cu:556-571) instead of the production kernels'
 *     exp2 of a log2(e)-prescaled falloff;
 *   - oracle/gsr_oracle.c, when a test selects it (gsr_oracle_set_shared_exp(1)) in place of the host
 *     libm's expf.
 *
 * The reference calls CUDA's expf (accurate to 2 ulp, implementation-defined below that), so no
 * particular rounding of exp() is the reference's; what makes the two builds comparable bit for bit
 * is that both evaluate the SAME function.  It uses only IEEE-754 single-precision +, -, * and
 * integer bit operations, with contraction off (both includers compile this body with
 * -ffp-contract=off; clang is also told so here), so gcc on x86-64 and clang on gfx950 round every
 * step identically.  Cody-Waite reduction x = n ln2 + r (|r| <= ln2/2, n ln2_hi exact for |n| < 2^9),
 * a degree-7 Taylor polynomial of e^r (truncation < 0.1 ulp), and 2^n applied as two exact
 * power-of-two factors.  Accuracy about 1 ulp on [-103, 88]; 0 below (where the rasterizer rejects
 * alpha < 1/255 anyway); arguments above 88 are clamped to 88 (the rasterizer discards power > 0).
 *
 * The includer defines GSR_REF_EXP_QUAL (e.g. `static __device__ __forceinline__`); default
 * `static inline`.
 */
#ifndef GSR_REF_EXP_H
#define GSR_REF_EXP_H

#include <stdint.h>

#ifndef GSR_REF_EXP_QUAL
#define GSR_REF_EXP_QUAL static inline
#endif

GSR_REF_EXP_QUAL float gsr_ref_pow2i(int k)
{
    /* 2^k for k in [-126, 127]: the exponent field alone */
    union { uint32_t u; float f; } v;
    v.u = (uint32_t)(k + 127) << 23;
    return v.f;
}

GSR_REF_EXP_QUAL float gsr_ref_expf(float x)
{
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    if (!(x > -103.0f)) return 0.0f; /* (NaN too) */
    if (x > 88.0f) x = 88.0f;
    const float shifter = 12582912.0f;              /* 1.5 * 2^23: t - shifter = rint(x log2(e)) */
    const float t = x * 1.44269502162933349609375f + shifter;
    const float n = t - shifter;
    const float ln2_hi = 0.693145751953125f;         /* 15 significant bits: n * ln2_hi exact */
    const float ln2_lo = 1.428606765330187045e-06f;
    float r = x - n * ln2_hi;
    r = r - n * ln2_lo;
    float p = 1.0f / 5040.0f;
    p = p * r + 1.0f / 720.0f;
    p = p * r + 1.0f / 120.0f;
    p = p * r + 1.0f / 24.0f;
    p = p * r + 1.0f / 6.0f;
    p = p * r + 0.5f;
    p = p * r + 1.0f;
    p = p * r + 1.0f;
    const int ni = (int)n;                           /* [-149, 127] */
    const int n1 = ni / 2, n2 = ni - n1;             /* each in [-75, 64] */
    return (p * gsr_ref_pow2i(n1)) * gsr_ref_pow2i(n2);
}

#endif
