/*
 * gsr_cpu_abi.c -- the C oracle (gsr_oracle.c) behind the product's own C ABI.
 *
 * TEST INFRASTRUCTURE ONLY (see gsr_oracle.c): built into oracle/libgsr_cpu.so, loaded only by
 * tests/ and the cpu_baseline leg of bench.py.  It exports gsr_forward / gsr_backward /
 * gsr_last_error with exactly the signatures of include/gsr.h, so the CPU baseline runs the same
 * host-side calling sequence as the HIP library ("the build's C++ CPU
 * restatement (same C ABI)"): resize callbacks for the three state buffers, then the backward on
 * those buffers.  Pointers are HOST pointers here and `stream` is ignored.
 *
 * State: the oracle keeps its forward state (depths, radii, conics, keys, ranges, final_T,
 * n_contrib: the reference's GeometryState / BinningState / ImageState, rasterizer_impl.h:21-73)
 * in one heap object; the geometry buffer the caller's callback provides holds the pointer to it
 * (8 bytes), the binning and image buffers hold nothing.  gsr_cpu_release(geometry_buffer) frees
 * it.  gsr_cpu_set_threads(n) sets the OpenMP thread count of the following calls.
 */
#include <stdio.h>
#include <string.h>

#include "../include/gsr.h"

void* gsr_oracle_forward(int P, int D, int M, const float* bg, int W, int H, const float* means3D, const float* shs,
                         const float* colors_precomp, const float* opacities, const float* scales,
                         float scale_modifier, const float* rotations, const float* cov3D_precomp,
                         const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                         float tan_fovy, int prefiltered, int antialiasing, float* out_color, float* out_invdepth,
                         int* radii_out, int nthreads, int* num_rendered);
int gsr_oracle_backward(void* p, const float* bg, const float* means3D, const float* shs, const float* colors_precomp,
                        const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                        const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                        const float* campos, float tan_fovx, float tan_fovy, const float* dL_dpix,
                        const float* dL_dinvdepth_pix, float* dL_dmean2D, float* dL_dconic, float* dL_dopacity,
                        float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale,
                        float* dL_drot, int nthreads);
void gsr_oracle_free(void* p);
const char* gsr_oracle_last_error(void);

static int g_threads = 1;
static char g_cpu_err[256];

static int cpu_fail(int code, const char* msg)
{
    snprintf(g_cpu_err, sizeof(g_cpu_err), "%s", msg);
    return code;
}

const char* gsr_last_error(void) { return g_cpu_err; }
void gsr_cpu_set_threads(int n) { g_threads = n > 0 ? n : 1; }

void gsr_cpu_release(char* geometry_buffer)
{
    void* st = NULL;
    if (!geometry_buffer) return;
    memcpy(&st, geometry_buffer, sizeof(st));
    gsr_oracle_free(st);
    memset(geometry_buffer, 0, sizeof(st));
}

/* Rasterizer::forward (rasterizer.h:31-55; rasterizer_impl.cu:198-341): the oracle's forward, its
 * state handle stored in the geometry buffer. */
int gsr_forward(gsr_resize_fn geometryBuffer, void* geometry_ctx, gsr_resize_fn binningBuffer, void* binning_ctx,
                gsr_resize_fn imageBuffer, void* image_ctx, int P, int D, int M, const float* background, int width,
                int height, const float* means3D, const float* shs, const float* colors_precomp,
                const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                float tan_fovx, float tan_fovy, bool prefiltered, float* out_color, float* depth, bool antialiasing,
                int* radii, bool debug, gsr_stream_t stream, int* num_rendered)
{
    (void)debug;
    (void)stream;
    if (!num_rendered) return cpu_fail(GSR_ERR_INVALID, "num_rendered is NULL");
    *num_rendered = 0;
    if (P < 0) return cpu_fail(GSR_ERR_INVALID, "P must be >= 0");
    char* gb = geometryBuffer(geometry_ctx, sizeof(void*));
    char* ib = imageBuffer(image_ctx, 1);
    if (!gb || !ib) return cpu_fail(GSR_ERR_ALLOC, "a resize callback returned NULL");
    int L = 0;
    void* st = gsr_oracle_forward(P, D, M, background, width, height, means3D, shs, colors_precomp, opacities,
                                  scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos,
                                  tan_fovx, tan_fovy, prefiltered, antialiasing, out_color, depth, radii, g_threads,
                                  &L);
    if (!st) return cpu_fail(GSR_ERR_PREFILTERED, gsr_oracle_last_error());
    memcpy(gb, &st, sizeof(st));
    if (!binningBuffer(binning_ctx, 1)) return cpu_fail(GSR_ERR_ALLOC, "a resize callback returned NULL");
    *num_rendered = L;
    return GSR_OK;
}

/* Rasterizer::backward (rasterizer.h:57-90; rasterizer_impl.cu:345-450) on the forward's state. */
int gsr_backward(int P, int D, int M, int R, const float* background, int width, int height, const float* means3D,
                 const float* shs, const float* colors_precomp, const float* opacities, const float* scales,
                 float scale_modifier, const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                 const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                 char* geom_buffer, char* binning_buffer, char* image_buffer, const float* dL_dpix,
                 const float* dL_invdepths, float* dL_dmean2D, float* dL_dconic, float* dL_dopacity,
                 float* dL_dcolor, float* dL_dinvdepth, float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh,
                 float* dL_dscale, float* dL_drot, bool antialiasing, bool debug, gsr_stream_t stream)
{
    (void)D; (void)M; (void)R; (void)width; (void)height; (void)radii; (void)binning_buffer; (void)image_buffer;
    (void)antialiasing; (void)debug; (void)stream;
    if (P <= 0) return GSR_OK;
    /* the per-Gaussian invdepth gradient is folded into dL_dmean3D inside the oracle (backward.cu:
     * 314-315) and not kept on its own: written as zeros */
    if (dL_dinvdepth) memset(dL_dinvdepth, 0, 4 * (size_t)P);
    void* st = NULL;
    if (!geom_buffer) return cpu_fail(GSR_ERR_ALLOC, "null state buffer");
    memcpy(&st, geom_buffer, sizeof(st));
    if (!st) return cpu_fail(GSR_ERR_INVALID, "geometry buffer holds no forward state");
    const int rc = gsr_oracle_backward(st, background, means3D, shs, colors_precomp, opacities, scales, scale_modifier,
                                       rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy,
                                       dL_dpix, dL_invdepths, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor,
                                       dL_dmean3D, dL_dcov3D, dL_dsh, dL_dscale, dL_drot, g_threads);
    return rc ? cpu_fail(GSR_ERR_INVALID, "oracle backward failed") : GSR_OK;
}
