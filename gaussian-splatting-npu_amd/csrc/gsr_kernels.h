// gsr_kernels.h -- kernel argument blocks and host launchers (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsr {

struct PreprocessArgs {
    int P, D, M, W, H;
    const float* means3D;
    const float* scales;
    float scale_modifier;
    const float* rotations;
    const float* opacities;
    const float* shs;  // (P,M,3); with dc: the (P,M-1,3) rest coefficients (M counts the dc one)
    const float* dc;   // separate coefficient 0 (P,1,3), or null
    const float* cov3D_precomp;
    const float* colors_precomp;
    const float* view;
    const float* proj;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    uint32_t grid_x, grid_y;
    int prefiltered, antialiasing;
    // outputs (means2D, depths, rgb: GeometryState fields nothing downstream reads -- kept for the
    // single-view forward's parity with the reference, null in the batched forward)
    int* radii;
    float* means2D;
    float* depths;
    float* rgb;
    float* conic_opacity;
    uint8_t* clamped;
    uint32_t* tiles_touched;
    uint32_t* host_flags;     // pinned host word: set to 1 on a prefiltered violation (no device memset)
    uint64_t* scan_status;    // look-back status words of the tiles_touched scan, zeroed here
    int scan_status_words;
    float4* splat;  // 3 x float4 per Gaussian (GEOM_SPLAT)
    uint32_t* dkey; // depth-sort key per Gaussian
    uint2* rect;    // {x0 | y0 << 16, x1 | y1 << 16} per Gaussian (zero if culled); null with rect4
    uint32_t* rect4;  // the rect packed (rect_pack) instead, on grids of <= 255 x 255 tiles
    int* tile_diff;   // IMG_TILE_DIFF, zeroed here (tile_hist adds into it), or null
    int tile_diff_words;
    uint32_t* rec_mask;  // GEOM_REC_MASK, zeroed here (render_bwd sets it)
    uint32_t* dsort_gsum;  // the depth sort's chunk-group digit counts (radix_gsum_*), zeroed here, or null
    int dsort_gsum_words;
};

struct RenderFwdArgs {
    const uint2* ranges;
    const uint32_t* tile_order;  // IMG_TILE_ORDER: block b renders tile tile_order[b]
    uint32_t* tile_work;         // IMG_TILE_WORK: largest n_contrib of the tile (out)
    const uint32_t* point_list;
    int W, H;
    uint32_t grid_x;
    const float4* splat;  // GEOM_SPLAT records (xy+extent, conic+opacity, rgb+1/depth)
    const float* bg;
    float* final_T;
    uint32_t* n_contrib;
    float* out_color;
    float* invdepth;
    uint8_t* hit;   // BIN_HIT: contributing quadrants of every processed list entry (out)
};

struct RenderBwdArgs {
    const uint2* ranges;
    const uint32_t* tile_order;  // IMG_TILE_ORDER (re-ordered from IMG_TILE_WORK for the backward)
    const uint32_t* tile_work;   // IMG_TILE_WORK (render_fwd): the tile's largest n_contrib
    const uint32_t* point_list;
    int W, H;
    uint32_t grid_x;
    int T;  // tiles
    const float* bg;
    const float4* splat;
    const float* final_Ts;
    const uint32_t* n_contrib;
    const float* dL_dpixels;
    const float* dL_invdepths;  // (1,H,W) or null
    const uint32_t* slot;       // gradient-record slot of each sorted position
    uint32_t* valid;            // bit (slot & 31) of valid[slot >> 5] set for every record written (cleared by emit)
    float* grad_inst;           // f32x12[L]: one gradient record per (tile, Gaussian) entry, at its record slot
    const uint8_t* hit;         // BIN_HIT (render_fwd): the quadrants each entry contributed to
    const uint32_t* emit_start; // GEOM_EMIT_START: first record slot of each Gaussian
    uint32_t* rec_mask;         // GEOM_REC_MASK: bit (slot - emit_start[id]) set for records at local index < 32
};

// Layout of one per-instance gradient record (GRAD_REC floats: 40 B, or 48 B padded).  With u = G dL/dalpha
// per pixel, the mean2D fields hold Sx = sum u dx, Sy = sum u dy and the conic fields
// sum u dx^2, u dx dy, u dy^2 -- WITHOUT the per-Gaussian factors (backward.cu:619-636):
// preprocess_bwd forms dL/dmean2D = (a Sx + b Sy, b Sx + c Sy) * (-opacity W/2, -opacity H/2)
// from the conic (a, b, c) and scales the conic sums by -opacity/2, once per Gaussian.
enum GradField {
    GF_MEAN2D_X = 0, GF_MEAN2D_Y, GF_CONIC_A, GF_CONIC_B, GF_CONIC_C, GF_OPACITY, GF_COLOR_R, GF_COLOR_G,
    GF_COLOR_B, GF_INVDEPTH, GF_NUM
};
#ifndef GSR_GRAD_REC
#define GSR_GRAD_REC 10  // (the same default as gsr_common.h, which sizes BIN_GRAD_INST with it)
#endif
constexpr int GRAD_REC = GSR_GRAD_REC;

// In-place gradient accumulation (gsr_backward_dc_acc): bit set = that output array is added to.
enum AccBits : uint32_t {
    ACC_MEANS3D = 1u, ACC_DC = 2u, ACC_SH = 4u, ACC_OPACITY = 8u, ACC_SCALES = 16u, ACC_ROTATIONS = 32u,
    ACC_COV3D = 64u, ACC_COLORS = 128u
};

struct PreprocessBwdArgs {
    int P, D, M;
    const float* means3D;
    const int* radii;  // the single-view launch: visibility radius > 0 (backward.cu:420); null for batches
    const float* shs;  // as PreprocessArgs: with dc, the rest coefficients and M counts dc
    const float* dc;
    const float* opacities;
    const float* scales;
    const float* rotations;
    float scale_modifier;
    const float* cov3D_precomp;  // null: cov3D is recomputed from scales/rotations
    int antialiasing;
    int has_invdepth;
    int W, H;
    // the single-view launch's other render-pass gradients (outputs of the reference glue; null for batches)
    float* dL_dconic;    // (P,4)
    float* dL_dinvdepth; // (P) or null
    float* dL_dopacity;  // (P)
    float* dL_dcolor;    // (P,3)
    float* dL_dmean3D;
    float* dL_dcov3D;
    float* dL_dsh;
    float* dL_ddc;  // (P,1,3) when dc is given
    float* dL_dscale;
    float* dL_drot;
    uint32_t acc;  // GSR_ACC_* bits (include/gsr.h): outputs added to instead of overwritten
};

// Multi-view backward (gsr_backward_views): one entry per camera view of the batch.  The
// per-Gaussian parameters and their gradients are shared (PreprocessBwdArgs), everything
// view-dependent comes from here; each view's screen-space gradient is written separately.
constexpr int MAX_VIEWS = 16;
struct BwdView {
    const float* view;
    const float* proj;
    const float* campos;
    float focal_x, focal_y, tan_fovx, tan_fovy;
    const int* radii;
    const float4* conic_opacity;
    const uint8_t* clamped;
    const uint32_t* emit_start;
    const uint32_t* tiles_touched;
    const float* grad_inst;
    const uint32_t* valid;
    const uint32_t* rec_mask;
    float* dL_dmean2D;  // (P,3)
};
struct PreprocessBwdViewsArgs {
    PreprocessBwdArgs a;
    int V;  // 0: the single view of `a`
    int g_begin, g_end;  // the Gaussians [g_begin, g_end) of this launch (a chunk of [0, P))
    BwdView v[MAX_VIEWS];
};

struct AdamArgs {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    const uint8_t* visible;  // one flag per Gaussian (bool)
    float lr, b1, b2, eps;
    int N, M;  // N Gaussians of M elements each
};
constexpr int ADAM_MAX_GROUPS = 8;
struct AdamMultiArgs {
    AdamArgs g[ADAM_MAX_GROUPS];
    uint32_t block_start[ADAM_MAX_GROUPS];  // first workgroup of each group
    int n_groups;
};
hipError_t launch_adam_update(const AdamArgs& a, hipStream_t s);
hipError_t launch_adam_update_multi(const AdamArgs* groups, int n_groups, hipStream_t s);

hipError_t launch_preprocess(const PreprocessArgs& a, hipStream_t s);
// V views of the same Gaussians (a[v] differ in camera and output buffers only), PREPROCESS_BATCH
// views per launch: each launch reads the Gaussians' parameters once.
constexpr int PREPROCESS_BATCH = 8;
hipError_t launch_preprocess_views(const PreprocessArgs* a, int V, hipStream_t s);
hipError_t launch_mark_visible(int P, const float* means3D, const float* view, bool* present, hipStream_t s);
// Inclusive scan of in[gather[i]] (gather may be null): one launch, chained chunks with decoupled
// look-back over `status` (scan_status_words(n) u64 words, zero on entry: preprocess clears them).
// The total goes to *total_out (pinned host memory is fine).
int scan_status_words(int n);
// exclusive: exclusive sums instead; total_out may be null.
hipError_t launch_inclusive_scan(const uint32_t* in, const uint32_t* gather, uint32_t* out, int n, uint64_t* status,
                                 uint32_t* total_out, hipStream_t s, bool exclusive = false);

// Batched prefix launches (gsr_forward_views): up to VIEW_BATCH views per launch, view =
// blockIdx.y, each with its own arrays and sizes (workgroups past a view's size exit at once).
// One launch per step over all views replaces V launches of a few hundred workgroups each: the
// latency-bound prefix kernels of one 1M-Gaussian view fill a fraction of the chip.
constexpr int VIEW_BATCH = 8;
template <typename A>
struct ViewBatch {
    A v[VIEW_BATCH];
    int n;
};

struct ScanJob {  // launch_inclusive_scan's arguments for one view
    const uint32_t* in;
    uint32_t* out;
    int n;
    uint64_t* status;
    uint32_t* total_out;
};
hipError_t launch_scan_batch(const ScanJob* jobs, int V, bool exclusive, hipStream_t s);

struct SortJob {  // radix_sort's arguments for one view
    int n;
    const uint32_t* keys_in;
    const uint2* pairs;
    uint32_t *k0, *v0, *k1, *v1;
    uint32_t *out_x, *out_y, *sorted_keys;
    char* scratch;
    const uint2* rects;
    uint2* sorted_rects;
    uint32_t* sorted_counts;
    // packed rects (rect_pack) in key order: carried as payload beside the id (v0 / v1 then hold
    // u32x2), the last pass unpacks them into sorted_rects -- no gather by id
    const uint32_t* rects4 = nullptr;
    // > 0 (one pass, pairs given, keys_in null): the key is pairs[i].y >> key_hi_shift, and out_y
    // gets pairs[i].y with those bits cleared
    int key_hi_shift = 0;
    // (with key_hi_shift, instead of pairs) the pairs as two arrays: x[i], y[i] -- the count kernel then
    // reads the 4-B y words only
    const uint32_t* soa_x = nullptr;
    const uint32_t* soa_y = nullptr;
    // the three-pass depth sort: a pinned host word set to 1 when the keys' range was too wide for it
    uint32_t* host_wide = nullptr;
    // the three-pass depth sort's chunk-group counts (radix_gsum_offset/bytes inside `scratch`) are
    // already zero (preprocess clears them); otherwise the sort clears them itself
    bool gsum_zeroed = false;
};
// The chunk-group digit counts of the three-pass depth sort inside its scratch: byte offset and size
// (zero-initialised by the caller, see SortJob::gsum_zeroed).
size_t radix_gsum_offset(int n);
size_t radix_gsum_bytes(int n);
// After a depth sort reported a range too wide for three 9-bit passes (SortJob::host_wide), the
// forward re-runs that sort with four_pass (radix_sort_batch), for that call only.  Test hook: force
// four passes for every depth sort of the calling host thread.
void set_depth_force_wide(bool on);
bool depth_force_wide();
// byte offset, inside a sort's scratch (radix_status_bytes(n)), of its {base, fits} range word
size_t radix_range_offset(int n);
// which sort a radix pass serves (selects the kernels' name tag only: profiles attribute dispatches)
enum SortKind { SORT_DEPTH = 0, SORT_TILE = 1, SORT_CELLS = 2 };
// V independent stable sorts over the same bit width (key bits [shift0, shift0 + nbits)), pass by
// pass in shared launches.
// four_pass: the depth sort (32-bit keys, shift0 0) in four 8-bit passes instead of three 9-bit ones
// (keys whose range is too wide for the relative third pass).
hipError_t radix_sort_batch(const SortJob* jobs, int V, int nbits, hipStream_t s, int shift0 = 0,
                            SortKind kind = SORT_DEPTH, bool four_pass = false);

// Emission fused into the tile sort (gsr_forward_views): the instances are generated from the
// depth-ordered rects inside the first radix pass's count and scatter kernels instead of being
// written out by an emission kernel and read back by that pass.
struct TileSortJob {
    int P, L;
    const uint32_t* sorted_ids;
    const uint32_t* offsets;      // inclusive scan of the tile counts in depth order
    const uint2* sorted_rects;
    const uint32_t* rec_start;    // first gradient-record slot per Gaussian
    char* pass1_scratch;          // fused_pass1_scratch_bytes(P): the first pass's count matrix
    uint32_t *k0, *v0, *k1, *v1;  // ping-pong (v: u32x2)
    char* scratch;                // radix_status_bytes(L) for the later passes
    uint32_t* out_slot;           // BIN_SLOT
    uint32_t* out_ids;            // BIN_POINT_LIST
    uint32_t* out_tiles;          // BIN_SORTED_TILES
    uint32_t* valid;              // BIN_VALID, cleared
    uint2* ranges;                // IMG_RANGES, cleared
    bool slotless;                // slots_from_rect: no record slots written (render_bwd derives them)
};
size_t fused_pass1_scratch_bytes(int P);
// phases: FUSED_COUNT = the first pass's histogram and row scan (needs neither L nor the binning
// buffer: the batched forward runs it while the host reads L back), FUSED_SCATTER = the rest
enum FusedPhase { FUSED_COUNT = 1, FUSED_SCATTER = 2, FUSED_ALL = 3 };
hipError_t tile_sort_fused_batch(const TileSortJob* jobs, int V, uint32_t gx, int T, hipStream_t s,
                                 int phases = FUSED_ALL);

struct RangesJob {
    int L;
    const uint32_t* sorted_tiles;
    uint2* ranges;
};
// views with L == 0 get their ranges zeroed (no emission cleared them)
hipError_t launch_tile_ranges_batch(const RangesJob* jobs, int V, int T, hipStream_t s);

struct OrderJob {
    const uint2* ranges;
    const uint32_t* work;
    uint32_t* order;
    // the forward's order from the rects' difference array (use_tile_diff): the kernel derives the
    // per-tile counts, WRITES the ranges (ranges_out) and orders by count; ranges and work unused
    const int* diff;
    uint2* ranges_out;
    uint32_t grid_x, grid_y;
};
// every job with ranges (the forward's order), every job with diff (the forward's, ranges written),
// or every job with work (the backward's)
hipError_t launch_tile_order_batch(const OrderJob* jobs, int V, int T, hipStream_t s);

// The rects' 2-D difference array (+1 at (x0, y0) and (x1, y1), -1 at (x1, y0) and (x0, y1) of every
// packed rect, rect_pack) added into diff (zeroed by preprocess): TILE_HIST_WGS workgroups per view
// accumulate in LDS and add their arrays into diff with integer atomics (order-independent).
struct TileHistJob {
    const uint32_t* rect4;
    int P;
    int* diff;
};
hipError_t launch_tile_hist_batch(const TileHistJob* jobs, int V, uint32_t grid_x, uint32_t grid_y, hipStream_t s);

hipError_t radix_sort(int n, int nbits, const uint32_t* keys_in, const uint2* pairs, uint32_t* k0, uint32_t* v0,
                      uint32_t* k1, uint32_t* v1, uint32_t* out_x, uint32_t* out_y, uint32_t* sorted_keys,
                      char* scratch, hipStream_t s, const uint2* rects = nullptr, uint2* sorted_rects = nullptr,
                      uint32_t* sorted_counts = nullptr, SortKind kind = SORT_DEPTH);
// ranges must be zero on entry unless L == 0 (the fused tile sort's first pass clears them)
hipError_t launch_tile_ranges(int L, const uint32_t* sorted_tiles, uint2* ranges, int T, hipStream_t s);
hipError_t launch_debug_keys(int L, const uint32_t* sorted_tiles, const uint32_t* point_list, const uint32_t* dkeys,
                             uint64_t* keys, hipStream_t s);
hipError_t launch_debug_keys_from_ranges(int T, const uint2* ranges, const uint32_t* point_list, const uint32_t* dkeys,
                                         uint64_t* keys, hipStream_t s);

// Longest-first launch order of the T tiles: order[] = tiles by decreasing work, work = range length
// (ranges != null, the forward) or work[] (the backward's per-tile largest n_contrib).
hipError_t launch_tile_order(const uint2* ranges, const uint32_t* work, int T, uint32_t* order, hipStream_t s);
hipError_t launch_render_fwd(const RenderFwdArgs& a, int T, hipStream_t s);
hipError_t launch_render_bwd(const RenderBwdArgs& a, int T, hipStream_t s);
// V views of one image size in one launch per VIEW_BATCH views (grid.y = view); render_bwd: every
// view with dL_invdepths, or none
hipError_t launch_render_fwd_batch(const RenderFwdArgs* a, int V, int T, hipStream_t s);
hipError_t launch_render_bwd_batch(const RenderBwdArgs* a, int V, int T, hipStream_t s);
hipError_t launch_preprocess_bwd_views(const PreprocessBwdViewsArgs& a, hipStream_t s);
// one view through the batched kernel at one lane per Gaussian (a.radii set: the view's visibility)
hipError_t launch_preprocess_bwd_single(const PreprocessBwdViewsArgs& a, hipStream_t s);

// fused SSIM (ssim.hip); dA/dB/dC null: map only
hipError_t launch_ssim_fwd(int planes, int H, int W, float C1, float C2, const float* img1, const float* img2,
                           float* map, float* dA, float* dB, float* dC, hipStream_t s);
hipError_t launch_ssim_bwd(int planes, int H, int W, const float* img1, const float* img2, const float* dmap,
                           const float* dA, const float* dB, const float* dC, float* dimg1, hipStream_t s);

// distCUDA2 (knn.hip); host_bounds: 6 words of pinned host memory
size_t knn_workspace_bytes(int P);
hipError_t knn_dist2(int P, const float* pts, float* dist2, char* workspace, uint32_t* host_bounds, hipStream_t s);

}  // namespace gsr
