/*
 * gsr.h -- C ABI of the MI355X-native differentiable Gaussian-splatting
 * rasterizer (libgsr_hip.so, built for gfx950).
 *
 * This is the drop-in boundary for the reference's native rasterizer
 * `CudaRasterizer::Rasterizer` (diff-gaussian-rasterization-npu/
 * cuda_rasterizer/rasterizer.h:20-91).  Argument order and meaning follow the
 * reference one-for-one; the differences are C-ABI plumbing only:
 *   - std::function<char*(size_t)> resize lambdas (rasterize_points.cu:27-33)
 *     become a C function pointer + context (gsr_resize_fn);
 *   - every entry point takes the HIP stream it must run on (hipStream_t as
 *     void*; NULL = legacy default stream, as in the reference);
 *   - errors are returned as an int status (0 = ok) with a thread-local
 *     message from gsr_last_error(); nothing throws across the ABI.
 * All data pointers are DEVICE pointers owned by the caller.  Absent optional
 * inputs are NULL, exactly like `.data<float>()` of the empty tensors the
 * reference passes (shs / colors_precomp / scales+rotations / cov3D_precomp,
 * rasterize_points.cu:104-110).  No torch types cross this boundary.
 */
#ifndef GSR_H_INCLUDED
#define GSR_H_INCLUDED

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* gsr_stream_t; /* hipStream_t */

/* Resize callback: must return a device pointer to at least `bytes` bytes
 * (rasterize_points.cu:27-33 resizeFunctional). */
typedef char* (*gsr_resize_fn)(void* ctx, size_t bytes);

enum {
    GSR_OK = 0,
    GSR_ERR_INVALID = 1,     /* bad argument / shape                          */
    GSR_ERR_HIP = 2,         /* HIP runtime error (launch, memcpy, sync)      */
    GSR_ERR_ALLOC = 3,       /* a resize callback returned NULL               */
    GSR_ERR_PREFILTERED = 4  /* prefiltered=true but a point was near-culled  */
                             /* (reference: printf + __trap, auxiliary.h:168-172) */
};

/* Thread-local description of the last error returned on this thread. */
const char* gsr_last_error(void);
/* Build identification string ("gsr-hip <version> gfx950"). */
const char* gsr_version(void);

/* Scratch sizes (bytes) of the three opaque state buffers.  They replace
 * required<GeometryState/ImageState/BinningState> (rasterizer_impl.h:67-73). */
size_t gsr_geometry_buffer_size(int P);
size_t gsr_image_buffer_size(int width, int height);
size_t gsr_binning_buffer_size(int num_rendered);

/* Replaces Rasterizer::markVisible (rasterizer.h:24-29; kernel
 * rasterizer_impl.cu:54-66): present[i] = view-space z of point i > 0.2. */
int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     bool* present, gsr_stream_t stream);

/* Replaces Rasterizer::forward (rasterizer.h:31-55; rasterizer_impl.cu:198-341).
 * Writes out_color (3,H,W), depth = inverse depth (1,H,W) (may be NULL),
 * radii (P) (may be NULL: an internal array is used), and *num_rendered. */
int gsr_forward(gsr_resize_fn geometryBuffer, void* geometry_ctx,
                gsr_resize_fn binningBuffer, void* binning_ctx,
                gsr_resize_fn imageBuffer, void* image_ctx,
                int P, int D, int M,
                const float* background,
                int width, int height,
                const float* means3D,
                const float* shs,
                const float* colors_precomp,
                const float* opacities,
                const float* scales,
                float scale_modifier,
                const float* rotations,
                const float* cov3D_precomp,
                const float* viewmatrix,
                const float* projmatrix,
                const float* cam_pos,
                float tan_fovx, float tan_fovy,
                bool prefiltered,
                float* out_color,
                float* depth,
                bool antialiasing,
                int* radii,
                bool debug,
                gsr_stream_t stream,
                int* num_rendered);

/* Two-phase form of gsr_forward for hosts that own allocation (the Python
 * package): phase 1 = preprocess + tile-count scan + the one D2H of
 * num_rendered (rasterizer_impl.cu:250-284) into caller buffers of
 * gsr_geometry_buffer_size(P) / gsr_image_buffer_size(W,H) bytes; phase 2 =
 * key emission, tile|depth sort, tile ranges and render
 * (rasterizer_impl.cu:286-338) with a binning buffer of
 * gsr_binning_buffer_size(num_rendered) bytes. */
int gsr_forward_geometry(char* geometry_buffer, char* image_buffer,
                         int P, int D, int M, int width, int height,
                         const float* means3D, const float* shs, const float* colors_precomp,
                         const float* opacities, const float* scales, float scale_modifier,
                         const float* rotations, const float* cov3D_precomp,
                         const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                         float tan_fovx, float tan_fovy, bool prefiltered, bool antialiasing,
                         int* radii, bool debug, gsr_stream_t stream, int* num_rendered);

int gsr_forward_render(char* geometry_buffer, char* binning_buffer, char* image_buffer,
                       int P, int num_rendered, const float* background, int width, int height,
                       const float* colors_precomp, float* out_color, float* depth, int* radii,
                       bool debug, gsr_stream_t stream);

/* Both phases in one call when the caller's binning buffer is already big enough:
 * gsr_forward_geometry, then, if gsr_binning_buffer_size(*num_rendered) <=
 * binning_capacity, gsr_forward_render into binning_buffer and *rendered = 1;
 * otherwise *rendered = 0 and the caller allocates the exact size and calls
 * gsr_forward_render itself.  Replaces the allocator round trip between the
 * reference's two halves (binningBuffer resize lambda, rasterizer_impl.cu:286-288)
 * when the host can guess the size, so the GPU does not idle while the host
 * allocates. */
int gsr_forward_prealloc(char* geometry_buffer, char* image_buffer, char* binning_buffer,
                         size_t binning_capacity, int P, int D, int M, const float* background,
                         int width, int height, const float* means3D, const float* shs,
                         const float* colors_precomp, const float* opacities, const float* scales,
                         float scale_modifier, const float* rotations, const float* cov3D_precomp,
                         const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                         float tan_fovx, float tan_fovy, bool prefiltered, bool antialiasing,
                         float* out_color, float* depth, int* radii, bool debug,
                         gsr_stream_t stream, int* num_rendered, int* rendered);

/* Replaces Rasterizer::backward (rasterizer.h:57-90; rasterizer_impl.cu:345-450).
 * dL_dinvdepths / dL_dinvdepth may both be NULL (rasterize_points.cu:174-182).
 * Every output is fully written (zeros for culled Gaussians), so unlike the
 * reference glue (rasterize_points.cu:163-182) the caller need not zero them.
 * The render-pass gradients (dL_dmean2D (P,3), dL_dconic (P,2,2),
 * dL_dopacity (P), dL_dcolor (P,3), dL_dinvdepth (P)) are reduced on chip and
 * gathered per Gaussian in a fixed order: results are bitwise reproducible
 * run to run (the reference sums with float atomics).
 * radii (may be NULL: the forward's own, in geom_buffer) gate each Gaussian as
 * backward.cu:163,420 do; a Gaussian with radius 0 gets zeros in EVERY output,
 * including the render-pass ones the reference would still report from its
 * render backward -- the two agree for radii produced by the forward (radius 0
 * <=> no tile <=> no record). */
int gsr_backward(int P, int D, int M, int R,
                 const float* background,
                 int width, int height,
                 const float* means3D,
                 const float* shs,
                 const float* colors_precomp,
                 const float* opacities,
                 const float* scales,
                 float scale_modifier,
                 const float* rotations,
                 const float* cov3D_precomp,
                 const float* viewmatrix,
                 const float* projmatrix,
                 const float* campos,
                 float tan_fovx, float tan_fovy,
                 const int* radii,
                 char* geom_buffer,
                 char* binning_buffer,
                 char* image_buffer,
                 const float* dL_dpix,
                 const float* dL_invdepths,
                 float* dL_dmean2D,
                 float* dL_dconic,
                 float* dL_dopacity,
                 float* dL_dcolor,
                 float* dL_dinvdepth,
                 float* dL_dmean3D,
                 float* dL_dcov3D,
                 float* dL_dsh,
                 float* dL_dscale,
                 float* dL_drot,
                 bool antialiasing,
                 bool debug,
                 gsr_stream_t stream);

/* Separate-DC ("dc=") forms of the four entry points above: the accelerated
 * upstream rasterizer's Rasterizer::forward/backward, which take `dc` (P,1,3,
 * SH coefficient 0) and `shs` (P,M,3, coefficients 1..M) as two arrays and
 * return dL_ddc / dL_dsh separately.  train.py picks that surface whenever the
 * package exports SparseGaussianAdam (train.py:37-41 -> gaussian_renderer/
 * __init__.py:82-100, rasterizer(dc=features_dc, shs=features_rest)), which
 * saves the caller's torch.cat of the two parameter tensors (192 B/Gaussian
 * written and read again) and the split of its gradient.  Here M counts the
 * rest coefficients only (sh.size(1) of features_rest; 15 at degree 3) and may
 * be 0 with shs NULL; dc NULL makes each call identical to its non-dc form. */
int gsr_forward_dc(gsr_resize_fn geometryBuffer, void* geometry_ctx,
                   gsr_resize_fn binningBuffer, void* binning_ctx,
                   gsr_resize_fn imageBuffer, void* image_ctx,
                   int P, int D, int M, const float* background, int width, int height,
                   const float* means3D, const float* dc, const float* shs,
                   const float* colors_precomp, const float* opacities, const float* scales,
                   float scale_modifier, const float* rotations, const float* cov3D_precomp,
                   const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                   float tan_fovx, float tan_fovy, bool prefiltered, float* out_color, float* depth,
                   bool antialiasing, int* radii, bool debug, gsr_stream_t stream, int* num_rendered);

int gsr_forward_geometry_dc(char* geometry_buffer, char* image_buffer,
                            int P, int D, int M, int width, int height,
                            const float* means3D, const float* dc, const float* shs,
                            const float* colors_precomp, const float* opacities, const float* scales,
                            float scale_modifier, const float* rotations, const float* cov3D_precomp,
                            const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                            float tan_fovx, float tan_fovy, bool prefiltered, bool antialiasing,
                            int* radii, bool debug, gsr_stream_t stream, int* num_rendered);

int gsr_forward_prealloc_dc(char* geometry_buffer, char* image_buffer, char* binning_buffer,
                            size_t binning_capacity, int P, int D, int M, const float* background,
                            int width, int height, const float* means3D, const float* dc,
                            const float* shs, const float* colors_precomp, const float* opacities,
                            const float* scales, float scale_modifier, const float* rotations,
                            const float* cov3D_precomp, const float* viewmatrix,
                            const float* projmatrix, const float* cam_pos, float tan_fovx,
                            float tan_fovy, bool prefiltered, bool antialiasing, float* out_color,
                            float* depth, int* radii, bool debug, gsr_stream_t stream,
                            int* num_rendered, int* rendered);

int gsr_backward_dc(int P, int D, int M, int R, const float* background, int width, int height,
                    const float* means3D, const float* dc, const float* shs,
                    const float* colors_precomp, const float* opacities, const float* scales,
                    float scale_modifier, const float* rotations, const float* cov3D_precomp,
                    const float* viewmatrix, const float* projmatrix, const float* campos,
                    float tan_fovx, float tan_fovy, const int* radii, char* geom_buffer,
                    char* binning_buffer, char* image_buffer, const float* dL_dpix,
                    const float* dL_invdepths, float* dL_dmean2D, float* dL_dconic,
                    float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth, float* dL_dmean3D,
                    float* dL_dcov3D, float* dL_ddc, float* dL_dsh, float* dL_dscale, float* dL_drot,
                    bool antialiasing, bool debug, gsr_stream_t stream);

/* gsr_backward_dc with in-place gradient accumulation: for every GSR_ACC_* bit set
 * in `accumulate`, the matching parameter-gradient array is ADDED to (out += this
 * call's gradient, one fp32 add per element, as autograd's AccumulateGrad does
 * `grad += new`) instead of overwritten.  A multi-view step (several views'
 * backward passes into one gradient buffer) then costs no separate
 * accumulation pass over the 236 B/Gaussian of gradients.  The render-pass outputs
 * (dL_dmean2D, dL_dconic, dL_dinvdepth) are always written. */
enum {
    GSR_ACC_MEANS3D = 1, GSR_ACC_DC = 2, GSR_ACC_SH = 4, GSR_ACC_OPACITY = 8, GSR_ACC_SCALES = 16,
    GSR_ACC_ROTATIONS = 32, GSR_ACC_COV3D = 64, GSR_ACC_COLORS = 128, GSR_ACC_ALL = 255
};
int gsr_backward_dc_acc(int P, int D, int M, int R, const float* background, int width, int height,
                        const float* means3D, const float* dc, const float* shs,
                        const float* colors_precomp, const float* opacities, const float* scales,
                        float scale_modifier, const float* rotations, const float* cov3D_precomp,
                        const float* viewmatrix, const float* projmatrix, const float* campos,
                        float tan_fovx, float tan_fovy, const int* radii, char* geom_buffer,
                        char* binning_buffer, char* image_buffer, const float* dL_dpix,
                        const float* dL_invdepths, float* dL_dmean2D, float* dL_dconic,
                        float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth, float* dL_dmean3D,
                        float* dL_dcov3D, float* dL_ddc, float* dL_dsh, float* dL_dscale, float* dL_drot,
                        bool antialiasing, bool debug, unsigned accumulate, gsr_stream_t stream);

/* Backward of a batch of V <= 16 camera views rendered from the same Gaussians (each with its
 * own gsr_forward* call and state buffers): per view BACKWARD::render (rasterizer_impl.cu:399-418),
 * then ONE pass of BACKWARD::preprocess over the Gaussians that reads each Gaussian's parameters
 * once, walks the V views' records and writes the parameter gradients summed over the views
 * (the views' loss terms add up) -- instead of V passes that each read the 236 B/Gaussian of
 * parameters and write (or accumulate) the 236 B/Gaussian of gradients.  Per-view arrays hold
 * one device pointer per view (viewmatrices, projmatrices, campos, radii (may be NULL: the
 * forward's internal copy), state buffers, dL_dpix, dL_invdepths (NULL: no invdepth term in
 * any view), dL_dmean2D: each view's (P,3) screen-space gradient); R, tan_fovx and tan_fovy are
 * host arrays.  dL_dcolor (may be NULL) and the parameter gradients are the sums over the views;
 * `accumulate` as in gsr_backward_dc_acc.  Results equal the sum of V gsr_backward_dc calls up to
 * fp32 summation order.
 * radii: accepted for the reference's argument list but NOT read -- the batched preprocess
 * backward (and gsr_backward_preprocess_views / _range below) takes a Gaussian's visibility in a
 * view from that view's forward state (its tiles_touched, i.e. radius > 0 as the forward computed
 * it), where the reference gates on the radii passed in (backward.cu:163,420).  The two agree for
 * radii produced by the forward; a caller that edits radii between forward and backward has that
 * edit ignored here (the single-view gsr_backward* entry points do read radii). */
int gsr_backward_views(int V, int P, int D, int M, const int* R, const float* background, int width, int height,
                       const float* means3D, const float* dc, const float* shs, const float* colors_precomp,
                       const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                       const float* cov3D_precomp, const float* const* viewmatrices,
                       const float* const* projmatrices, const float* const* campos, const float* tan_fovx,
                       const float* tan_fovy, const int* const* radii, char* const* geom_buffers,
                       char* const* binning_buffers, char* const* image_buffers, const float* const* dL_dpix,
                       const float* const* dL_invdepths, float* const* dL_dmean2D, float* dL_dcolor,
                       float* dL_dopacity, float* dL_dmean3D, float* dL_dcov3D, float* dL_ddc, float* dL_dsh,
                       float* dL_dscale, float* dL_drot, bool antialiasing, bool debug, unsigned accumulate,
                       gsr_stream_t stream);

/* The two halves of gsr_backward_views, for callers that run each view's backward as soon as its
 * image gradient exists and the parameter gradients once per batch (diff_gaussian_rasterization.
 * deferred_backward: view v's render backward beside view v+1's forward on another stream).
 * gsr_backward_render: BACKWARD::render of one view (rasterizer_impl.cu:399-418) -- its
 * per-(tile, Gaussian) gradient records into its binning buffer, nothing else.
 * gsr_backward_preprocess_views: BACKWARD::preprocess (rasterizer_impl.cu:423-449) of V <= 16
 * such views in one pass over the Gaussians, arguments as gsr_backward_views; has_invdepth: some
 * view's render backward had an inverse-depth gradient.  Running the first for every view and then
 * the second equals gsr_backward_views bit for bit. */
int gsr_backward_render(int P, int R, const float* background, int width, int height, char* geom_buffer,
                        char* binning_buffer, char* image_buffer, const float* dL_dpix, const float* dL_invdepths,
                        bool debug, gsr_stream_t stream);
int gsr_backward_preprocess_views(int V, int P, int D, int M, const int* R, int width, int height,
                                  const float* means3D, const float* dc, const float* shs,
                                  const float* colors_precomp, const float* opacities, const float* scales,
                                  float scale_modifier, const float* rotations, const float* cov3D_precomp,
                                  const float* const* viewmatrices, const float* const* projmatrices,
                                  const float* const* campos, const float* tan_fovx, const float* tan_fovy,
                                  const int* const* radii, char* const* geom_buffers, char* const* binning_buffers,
                                  bool has_invdepth, float* const* dL_dmean2D, float* dL_dcolor, float* dL_dopacity,
                                  float* dL_dmean3D, float* dL_dcov3D, float* dL_ddc, float* dL_dsh,
                                  float* dL_dscale, float* dL_drot, bool antialiasing, bool debug,
                                  unsigned accumulate, gsr_stream_t stream);
/* gsr_backward_render_views: the BACKWARD::render half of gsr_backward_views for all V views (one
 * tile-order launch and one render launch per batch).  gsr_backward_preprocess_views_range: the
 * BACKWARD::preprocess half restricted to the Gaussians [g_begin, g_end) -- only their rows of the
 * parameter gradients (and of each view's dL_dmean2D) are written, so a caller can hand finished
 * row ranges to a gradient all-reduce while the next range computes (the collective
 * overlapped with the backward).  Chunks covering [0, P) equal one full call bit for bit. */
int gsr_backward_render_views(int V, int P, const int* R, const float* background, int width, int height,
                              char* const* geom_buffers, char* const* binning_buffers, char* const* image_buffers,
                              const float* const* dL_dpix, const float* const* dL_invdepths, bool debug,
                              gsr_stream_t stream);
int gsr_backward_preprocess_views_range(int V, int P, int D, int M, const int* R, int width, int height,
                                        const float* means3D, const float* dc, const float* shs,
                                        const float* colors_precomp, const float* opacities, const float* scales,
                                        float scale_modifier, const float* rotations, const float* cov3D_precomp,
                                        const float* const* viewmatrices, const float* const* projmatrices,
                                        const float* const* campos, const float* tan_fovx, const float* tan_fovy,
                                        const int* const* radii, char* const* geom_buffers,
                                        char* const* binning_buffers, bool has_invdepth, float* const* dL_dmean2D,
                                        float* dL_dcolor, float* dL_dopacity, float* dL_dmean3D, float* dL_dcov3D,
                                        float* dL_ddc, float* dL_dsh, float* dL_dscale, float* dL_drot,
                                        bool antialiasing, bool debug, unsigned accumulate, int g_begin, int g_end,
                                        gsr_stream_t stream);

/* Forward of a batch of V <= 16 camera views of the same Gaussians (the forward half of
 * gsr_backward_views; each view the result of gsr_forward_prealloc_dc with its own state buffers).
 * Every stage is ONE launch over up to 8 views (grid.y = view), on an internal high-priority
 * stream: preprocess (the Gaussians' parameters read once for the batch; GeometryState's means2D,
 * depths and rgb, read by nothing downstream, are not written), the record-slot scans (beside the
 * depth sorts, on an auxiliary stream), the depth sorts, the tile-count scans; then every view's
 * num_rendered is read back (the one host hand-off, rasterizer_impl.cu:283-284); then the tile
 * sorts with the instance emission fused into their first pass, tile ranges, tile orders, and on
 * the caller's stream one render launch for the views (one launch tail per batch).  Per-view arrays hold one pointer per view
 * (viewmatrices, projmatrices, campos, the three state buffers, out_colors (3,H,W), out_invdepths
 * (1,H,W), radii (P) -- radii may be NULL); tan_fovx, tan_fovy, binning_capacity, num_rendered and
 * rendered are host arrays.  rendered[v] = 0: view v's binning buffer was NULL or smaller than
 * gsr_binning_buffer_size(num_rendered[v]) -- the caller allocates that and finishes the view with
 * gsr_forward_render.  Every result is bit-identical to the single-view call's. */
int gsr_forward_views(int V, int P, int D, int M, const float* background, int width, int height,
                      const float* means3D, const float* dc, const float* shs, const float* colors_precomp,
                      const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                      const float* cov3D_precomp, const float* const* viewmatrices, const float* const* projmatrices,
                      const float* const* campos, const float* tan_fovx, const float* tan_fovy, bool prefiltered,
                      bool antialiasing, char* const* geometry_buffers, char* const* image_buffers,
                      char* const* binning_buffers, const size_t* binning_capacity, float* const* out_colors,
                      float* const* out_invdepths, int* const* radii, bool debug, gsr_stream_t stream,
                      int* num_rendered, int* rendered);

/* Visibility-masked Adam step (the accelerated upstream's `_C.adamUpdate`, called
 * by SparseGaussianAdam.step(visibility, N) from train.py:180-183): for each of the
 * N Gaussians with visible[i] set, its M consecutive elements of param are updated
 *   m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;  param -= lr m / (sqrt(v) + eps)
 * (no bias correction); other rows are left untouched.  N*M < 2^32. */
int gsr_adam_update(float* param, const float* param_grad, float* exp_avg, float* exp_avg_sq,
                    const bool* visible, float lr, float b1, float b2, float eps, int N, int M,
                    gsr_stream_t stream);

/* The same step for n_groups parameter tensors sharing one visibility mask (one
 * SparseGaussianAdam.step over its per-attribute groups, scene/gaussian_model.py:
 * 181-196) in a single launch: group i has Ms[i] elements per Gaussian, learning
 * rate lrs[i] and epsilon epss[i].  Per group identical to gsr_adam_update. */
int gsr_adam_update_multi(int n_groups, float* const* params, const float* const* param_grads,
                          float* const* exp_avgs, float* const* exp_avg_sqs, const int* Ms,
                          const float* lrs, const float* epss, const bool* visible, float b1,
                          float b2, int N, gsr_stream_t stream);

/* Where the forward's binning prefix (preprocess .. tile order) runs.  on = 1: on an internal
 * stream of the highest priority, forked from and joined back into the caller's stream, its side
 * work (record-slot scan, tile histogram, forward tile order) on a second internal stream;
 * on = 2: on the caller's stream, the side work on the internal one (no join before render_fwd);
 * on = 0: every launch on the caller's stream.  Other values: GSR_ERR_INVALID.  Per host
 * thread; the default is the library's build-time GSR_PREFIX_MODE_DEFAULT. */
int gsr_set_prefix_stream(int on);

/* Debug / parity helper: writes the sorted 64-bit tile|depth keys
 * (rasterizer_impl.cu:102-104 layout, after the sort of :306-311) and the
 * sorted Gaussian ids of the last forward held in these buffers. */
int gsr_debug_sorted_keys(const char* geometry_buffer, const char* binning_buffer, const char* image_buffer,
                          int P, int num_rendered, int width, int height,
                          uint64_t* keys_out, uint32_t* vals_out, uint32_t* ranges_out,
                          gsr_stream_t stream);

/* Debug / parity helper: the forward's depth sort alone (the first half of the
 * rasterizer_impl.cu:306-311 key sort): out_ids = the stable order of n u32 keys
 * (the forward's depth keys: float bit patterns, 0xFFFFFFFF = culled, sorted
 * last).
 * workspace: gsr_debug_depth_sort_workspace_size(n) device bytes. */
size_t gsr_debug_depth_sort_workspace_size(int n);
int gsr_debug_depth_sort(const uint32_t* keys, int n, uint32_t* out_ids, char* workspace, gsr_stream_t stream);

/* The depth sort runs three 9-bit passes, the third relative to the smallest visible key; in a forward
 * whose visible depth keys span too wide a range for that (depths beyond a factor of ~2^16) that
 * view's depth sort and tile-count scan run again in four 8-bit passes -- for that call only, no
 * state is kept (the reference's sort is stateless, rasterizer_impl.cu:306-311).
 * Test hooks: gsr_debug_set_depth_wide(1) forces four passes for every depth sort of the calling host
 * thread (0 releases it; gsr_debug_depth_wide reads it); gsr_debug_last_depth_passes(v) = the passes
 * the final depth sort of view v of this thread's last forward ran (3, or 4 after a re-run or when
 * forced; 0 before any forward). */
int gsr_debug_depth_wide(void);
int gsr_debug_set_depth_wide(int on);
int gsr_debug_last_depth_passes(int view);

/* Floats per per-instance gradient record in the binning buffer's GRAD_INST region (the build's
 * GSR_GRAD_REC: 10 = 40 B), for diagnostics that decode the records. */
int gsr_debug_grad_record_floats(void);

/* Byte offsets of the arrays inside each opaque state buffer (n entries
 * written, count of arrays returned; entry [count] is the total size).  For
 * parity tests and debugging only; the layout is private to this library. */
int gsr_geometry_layout(int P, size_t* offsets, int n);
int gsr_image_layout(int width, int height, size_t* offsets, int n);
int gsr_binning_layout(int num_rendered, size_t* offsets, int n);

/* Per-kernel timing with HIP events recorded on the launch stream (used by
 * bench.py's roofline measurement).  gsr_profile_enable(1) starts recording
 * (and resets); gsr_profile_read waits for the recorded events and returns,
 * per kernel id, the summed milliseconds and launch counts since the last
 * enable/read.  Both return the number of kernel ids. */
int gsr_profile_enable(int on);
int gsr_profile_read(double* total_ms, int* counts, int n);
const char* gsr_profile_kernel_name(int kernel_id);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H_INCLUDED */
