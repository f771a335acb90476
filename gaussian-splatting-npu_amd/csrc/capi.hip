// capi.hip -- C-ABI entry points (include/gsr.h).  Host-side orchestration that
// replaces CudaRasterizer::Rasterizer::{markVisible, forward, backward}
// (rasterizer_impl.cu:141-450): state-buffer carving, launch order, the one
// stream-ordered D2H of num_rendered, and error reporting.  No exceptions
// cross the ABI; every launch goes to the caller's stream.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "gsr.h"
#include "simple_knn.h"
#include "fused_ssim.h"
#include "gsr_common.h"
#include "gsr_kernels.h"

using namespace gsr;

static_assert(GSR_ACC_MEANS3D == ACC_MEANS3D && GSR_ACC_DC == ACC_DC && GSR_ACC_SH == ACC_SH &&
                  GSR_ACC_OPACITY == ACC_OPACITY && GSR_ACC_SCALES == ACC_SCALES &&
                  GSR_ACC_ROTATIONS == ACC_ROTATIONS && GSR_ACC_COV3D == ACC_COV3D && GSR_ACC_COLORS == ACC_COLORS,
              "include/gsr.h accumulate bits match the kernel's");

namespace {

thread_local std::string g_err;
thread_local uint32_t* g_pinned = nullptr;
constexpr uint32_t L_PENDING = 0xFFFFFFFFu;  // h[2] before the scan stores num_rendered (< 2^31)
// forward_geometry_wait: the depth keys' range was too wide for the three-pass depth sort (h[1]); that
// call's depth sort and tile-count scan are re-run with four passes (depth_sort_rerun_wide) --
// internal, never returned to a caller
constexpr int GSR_RERUN_WIDE = -100;
// depth-sort passes of this thread's last forward (per view: 3, or 4 after a re-run of its depth
// sort; gsr_debug_last_depth_passes)
thread_local int t_last_depth_passes[16] = {};

int fail(int code, const char* msg)
{
    g_err = msg;
    return code;
}

int fail_hip(hipError_t e, int line)
{
    char buf[256];
    snprintf(buf, sizeof(buf), "HIP error: %s (capi.hip:%d)", hipGetErrorString(e), line);
    g_err = buf;
    return GSR_ERR_HIP;
}

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail_hip(e_, __LINE__);                                   \
    } while (0)

#define DEBUG_SYNC(stream)                                                                    \
    do {                                                                                      \
        if (debug) {                                                                          \
            HIP_TRY(hipStreamSynchronize(stream));                                            \
            HIP_TRY(hipGetLastError());                                                       \
        }                                                                                     \
    } while (0)

// Pinned, device-mapped host words of this host thread, one 16-word slot per view of a
// multi-view forward (slot 0 for a single view).  The forward's kernels store the
// prefiltered-violation flag and num_rendered straight into them (system-scope stores), so the
// forward needs neither a device memset nor a D2H copy before its one stream synchronisation.
constexpr int PINNED_SLOT_WORDS = 16;
int pinned(int slot, uint32_t** out)
{
    if (!g_pinned) {
        hipError_t e = hipHostMalloc((void**)&g_pinned, 4 * PINNED_SLOT_WORDS * MAX_VIEWS,
                                     hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) return fail_hip(e, __LINE__);
    }
    *out = g_pinned + PINNED_SLOT_WORDS * slot;
    return GSR_OK;
}

// ---------------------------------------------------------------------------
// The forward's binning prefix (preprocess, depth sort, scans, tile sort, tile ranges,
// tile order: small, latency-bound launches) runs on an internal stream of the highest priority,
// forked from the caller's stream and joined back into it before render_fwd.  When the caller
// overlaps views on several streams (the forward of view v+1 beside the backward of view v,
// bench.py), the dispatcher then places the prefix's workgroups ahead of the queued workgroups of
// the other view's long kernels instead of behind them.  Buffers stay stream-ordered for the caller:
// everything the prefix writes is joined into its stream before the entry point returns.
// ---------------------------------------------------------------------------
// the fork / join events order streams of one device only: no system-scope fence (the host never
// inspects them; what the host reads -- num_rendered -- the scan stores with system-scope atomics)
#ifndef GSR_EVENT_FLAGS
#define GSR_EVENT_FLAGS (hipEventDisableTiming | hipEventDisableSystemFence)
#endif
constexpr int PREFIX_STREAMS = 4;  // views whose binning prefixes run side by side (gsr_forward_views)
struct PrefixStream {
    hipStream_t s[PREFIX_STREAMS] = {};
    hipEvent_t fork = nullptr, join = nullptr;
    // side work of a prefix (the index-order scan) beside its critical path
    hipStream_t aux = nullptr;
    hipEvent_t aux_in = nullptr, aux_out = nullptr;
};
constexpr int MAX_DEVICES = 64;
thread_local PrefixStream g_prefix[MAX_DEVICES];
// gsr_set_prefix_stream: 0 = everything on the caller's stream; 1 = the prefix on its own
// high-priority stream (forked from the caller's, joined before render_fwd) and its side work on
// the auxiliary stream; 2 = the prefix on the caller's stream, its side work on the auxiliary stream
#ifndef GSR_PREFIX_MODE_DEFAULT
#define GSR_PREFIX_MODE_DEFAULT 1
#endif
thread_local int g_prefix_mode = GSR_PREFIX_MODE_DEFAULT;

// n (<= PREFIX_STREAMS) prefix streams of the current device, each forked from `caller`; all of
// them the caller's own stream when the prefix streams are off (or the device is out of range).
int prefix_fork(hipStream_t caller, int n, hipStream_t* out)
{
    for (int k = 0; k < n; k++) out[k] = caller;
    if (g_prefix_mode != 1) return GSR_OK;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fail_hip(e, __LINE__);
    if (dev < 0 || dev >= MAX_DEVICES) return GSR_OK;
    PrefixStream& ps = g_prefix[dev];
    if (!ps.fork) {
        if ((e = hipEventCreateWithFlags(&ps.fork, GSR_EVENT_FLAGS)) != hipSuccess) return fail_hip(e, __LINE__);
        if ((e = hipEventCreateWithFlags(&ps.join, GSR_EVENT_FLAGS)) != hipSuccess) return fail_hip(e, __LINE__);
    }
    if ((e = hipEventRecord(ps.fork, caller)) != hipSuccess) return fail_hip(e, __LINE__);
    for (int k = 0; k < n; k++) {
        if (!ps.s[k]) {
            int least = 0, greatest = 0;
            if ((e = hipDeviceGetStreamPriorityRange(&least, &greatest)) != hipSuccess) return fail_hip(e, __LINE__);
            if ((e = hipStreamCreateWithPriority(&ps.s[k], hipStreamNonBlocking, greatest)) != hipSuccess)
                return fail_hip(e, __LINE__);
        }
        if ((e = hipStreamWaitEvent(ps.s[k], ps.fork, 0)) != hipSuccess) return fail_hip(e, __LINE__);
        out[k] = ps.s[k];
    }
    return GSR_OK;
}

int prefix_begin(hipStream_t caller, hipStream_t* out) { return prefix_fork(caller, 1, out); }

int current_device()
{
    int dev = 0;
    return hipGetDevice(&dev) == hipSuccess ? dev : 0;
}

// The auxiliary stream of the current device, forked from `s` (s itself when the prefix streams
// are off); aux_join makes `s` wait for everything enqueued on it so far.
int aux_fork(hipStream_t s, hipStream_t* out)
{
    *out = s;
    if (g_prefix_mode == 0) return GSR_OK;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fail_hip(e, __LINE__);
    if (dev < 0 || dev >= MAX_DEVICES) return GSR_OK;
    PrefixStream& ps = g_prefix[dev];
    if (!ps.aux) {
        int least = 0, greatest = 0;
        if ((e = hipDeviceGetStreamPriorityRange(&least, &greatest)) != hipSuccess) return fail_hip(e, __LINE__);
        if ((e = hipStreamCreateWithPriority(&ps.aux, hipStreamNonBlocking, greatest)) != hipSuccess)
            return fail_hip(e, __LINE__);
        if ((e = hipEventCreateWithFlags(&ps.aux_in, GSR_EVENT_FLAGS)) != hipSuccess) return fail_hip(e, __LINE__);
        if ((e = hipEventCreateWithFlags(&ps.aux_out, GSR_EVENT_FLAGS)) != hipSuccess)
            return fail_hip(e, __LINE__);
    }
    if ((e = hipEventRecord(ps.aux_in, s)) != hipSuccess) return fail_hip(e, __LINE__);
    if ((e = hipStreamWaitEvent(ps.aux, ps.aux_in, 0)) != hipSuccess) return fail_hip(e, __LINE__);
    *out = ps.aux;
    return GSR_OK;
}

int aux_join(hipStream_t s, hipStream_t aux)
{
    if (aux == s) return GSR_OK;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fail_hip(e, __LINE__);
    PrefixStream& ps = g_prefix[dev];
    if ((e = hipEventRecord(ps.aux_out, aux)) != hipSuccess) return fail_hip(e, __LINE__);
    if ((e = hipStreamWaitEvent(s, ps.aux_out, 0)) != hipSuccess) return fail_hip(e, __LINE__);
    return GSR_OK;
}

// the caller's stream waits for everything enqueued on the prefix stream so far
int prefix_end(hipStream_t caller, hipStream_t prefix)
{
    if (prefix == caller) return GSR_OK;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fail_hip(e, __LINE__);
    PrefixStream& ps = g_prefix[dev];
    if ((e = hipEventRecord(ps.join, prefix)) != hipSuccess) return fail_hip(e, __LINE__);
    if ((e = hipStreamWaitEvent(caller, ps.join, 0)) != hipSuccess) return fail_hip(e, __LINE__);
    return GSR_OK;
}

// ---------------------------------------------------------------------------
// Optional per-kernel timing with HIP events recorded on the launch stream
// (bench.py's roofline leg).  Off by default; costs two event records per
// launch when on.
// ---------------------------------------------------------------------------
enum ProfKernel {
    PK_PREPROCESS = 0, PK_DEPTH_SORT, PK_SCAN, PK_EMIT, PK_TILE_SORT, PK_RANGES, PK_RENDER_FWD, PK_RENDER_BWD,
    PK_PREPROCESS_BWD, PK_TILE_ORDER,
    PK_COUNT
};
const char* kProfNames[PK_COUNT] = {"preprocess_fwd", "depth_sort", "scan", "emit_instances", "tile_sort",
                                    "tile_ranges", "render_fwd", "render_bwd", "preprocess_bwd", "tile_order"};
struct Prof {
    bool on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool[PK_COUNT];
    size_t used[PK_COUNT] = {};
    size_t parts[PK_COUNT] = {};  // scopes that continue the kernel's previous one (not a new launch)
};
Prof g_prof;

hipEvent_t prof_begin(int k, hipStream_t s)
{
    if (!g_prof.on) return nullptr;
    auto& pool = g_prof.pool[k];
    if (g_prof.used[k] == pool.size()) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return nullptr;
        pool.push_back({a, b});
    }
    hipEvent_t e = pool[g_prof.used[k]].first;
    (void)hipEventRecord(e, s);
    return e;
}

void prof_end(int k, hipStream_t s, hipEvent_t begun, bool part)
{
    if (!g_prof.on || !begun) return;
    (void)hipEventRecord(g_prof.pool[k][g_prof.used[k]].second, s);
    g_prof.used[k]++;
    if (part) g_prof.parts[k]++;
}

// part: the scope times the rest of a kernel stage whose first part had a scope of its own (its time
// adds to the stage's total, not to its launch count)
struct ProfScope {
    int k; hipStream_t s; hipEvent_t e; bool part;
    ProfScope(int k_, hipStream_t s_, bool part_ = false) : k(k_), s(s_), e(prof_begin(k_, s_)), part(part_) {}
    ~ProfScope() { prof_end(k, s, e, part); }
};

template <typename T>
T* at(char* base, size_t off) { return reinterpret_cast<T*>(base + off); }
template <typename T>
const T* at(const char* base, size_t off) { return reinterpret_cast<const T*>(base + off); }

}  // namespace

extern "C" {

const char* gsr_last_error(void) { return g_err.c_str(); }

const char* gsr_version(void) { return GSR_REF_ALPHA ? "gsr-hip 0.1 gfx950 ref-alpha (TEST BUILD)" : "gsr-hip 0.1 gfx950"; }

int gsr_set_prefix_stream(int on)
{
    if (on < 0 || on > 2) return fail(GSR_ERR_INVALID, "prefix stream mode must be 0, 1 or 2");
    g_prefix_mode = on;
    return GSR_OK;
}

int gsr_profile_enable(int on)
{
    g_prof.on = on != 0;
    for (int k = 0; k < PK_COUNT; k++) g_prof.used[k] = 0;
    return PK_COUNT;
}

const char* gsr_profile_kernel_name(int k) { return (k >= 0 && k < PK_COUNT) ? kProfNames[k] : ""; }

// Waits for every recorded event, returns per-kernel summed milliseconds and launch counts
// since the last enable/read, and resets the counters.
int gsr_profile_read(double* total_ms, int* counts, int n)
{
    for (int k = 0; k < PK_COUNT && k < n; k++) {
        double acc = 0.0;
        for (size_t j = 0; j < g_prof.used[k]; j++) {
            auto& ev = g_prof.pool[k][j];
            HIP_TRY(hipEventSynchronize(ev.second));
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, ev.first, ev.second));
            acc += ms;
        }
        total_ms[k] = acc;
        counts[k] = (int)(g_prof.used[k] - g_prof.parts[k]);
        g_prof.used[k] = 0;
        g_prof.parts[k] = 0;
    }
    return PK_COUNT;
}

size_t gsr_geometry_buffer_size(int P) { return geom_layout(P).off[GEOM_COUNT] + 256; }
size_t gsr_image_buffer_size(int width, int height) { return image_layout(width, height).off[IMG_COUNT] + 256; }
size_t gsr_binning_buffer_size(int num_rendered) { return bin_layout(num_rendered).off[BIN_COUNT] + 256; }

// Byte offsets of the arrays inside each state buffer (test/debug introspection).
int gsr_geometry_layout(int P, size_t* offsets, int n)
{
    GeomLayout l = geom_layout(P);
    for (int i = 0; i < n && i <= GEOM_COUNT; i++) offsets[i] = l.off[i];
    return GEOM_COUNT;
}
int gsr_image_layout(int W, int H, size_t* offsets, int n)
{
    ImageLayout l = image_layout(W, H);
    for (int i = 0; i < n && i <= IMG_COUNT; i++) offsets[i] = l.off[i];
    return IMG_COUNT;
}
int gsr_binning_layout(int L, size_t* offsets, int n)
{
    BinLayout l = bin_layout(L);
    for (int i = 0; i < n && i <= BIN_COUNT; i++) offsets[i] = l.off[i];
    return BIN_COUNT;
}

int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix, bool* present,
                     gsr_stream_t stream)
{
    (void)projmatrix;
    if (P < 0) return fail(GSR_ERR_INVALID, "P must be >= 0");
    if (P == 0) return GSR_OK;
    if (!means3D || !viewmatrix || !present) return fail(GSR_ERR_INVALID, "null pointer");
    HIP_TRY(launch_mark_visible(P, means3D, viewmatrix, present, (hipStream_t)stream));
    return GSR_OK;
}


// The arguments of one view's preprocess (argument checks; the view's pinned read-back slot is
// reset: *h_out its host words, *hdev_out their device address).
static int forward_geometry_args(char* geometry_buffer, char* image_buffer, int P, int D, int M, int width,
                                 int height, const float* means3D, const float* dc, const float* shs,
                                 const float* colors_precomp, const float* opacities, const float* scales,
                                 float scale_modifier, const float* rotations, const float* cov3D_precomp,
                                 const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                                 float tan_fovx, float tan_fovy, bool prefiltered, bool antialiasing, int* radii,
                                 int slot, PreprocessArgs* out, uint32_t** h_out, uint32_t** hdev_out)
{
    if (width <= 0 || height <= 0) return fail(GSR_ERR_INVALID, "image size must be positive");
    if (!colors_precomp && !dc && (!shs || M <= 0))
        return fail(GSR_ERR_INVALID, "Please provide exactly one of either SHs or precomputed colors!");
    if (dc && M < 0) return fail(GSR_ERR_INVALID, "M (rest SH coefficients) must be >= 0");
    if (dc && colors_precomp)
        return fail(GSR_ERR_INVALID, "Please provide exactly one of either SHs or precomputed colors!");
    if (dc && M > 0 && !shs) return fail(GSR_ERR_INVALID, "dc given with M > 0 rest coefficients but shs is NULL");
    if (!cov3D_precomp && (!scales || !rotations))
        return fail(GSR_ERR_INVALID,
                    "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    if (!geometry_buffer || !image_buffer) return fail(GSR_ERR_ALLOC, "null state buffer");

    const GeomLayout g = geom_layout(P);
    char* gb = geometry_buffer;
    // h[0]: prefiltered violation (written by preprocess), h[2]: num_rendered (written by the scan).
    // This thread's previous forward has read its num_rendered back, so no kernel still writes them.
    uint32_t* h;
    int rc = pinned(slot, &h);
    if (rc) return rc;
    h[0] = 0;
    h[1] = 0;  // the depth sort's "range too wide" flag
    __atomic_store_n(&h[2], L_PENDING, __ATOMIC_RELEASE);
    uint32_t* h_dev = nullptr;
    HIP_TRY(hipHostGetDevicePointer((void**)&h_dev, h, 0));

    PreprocessArgs& a = *out;
    a.P = P; a.D = D; a.M = dc ? M + 1 : M; a.W = width; a.H = height;  // kernels count the dc coefficient
    a.dc = dc;
    a.means3D = means3D; a.scales = scales; a.scale_modifier = scale_modifier; a.rotations = rotations;
    a.opacities = opacities; a.shs = shs; a.cov3D_precomp = cov3D_precomp; a.colors_precomp = colors_precomp;
    a.view = viewmatrix; a.proj = projmatrix; a.campos = cam_pos;
    a.tan_fovx = tan_fovx; a.tan_fovy = tan_fovy;
    a.focal_y = height / (2.0f * tan_fovy);
    a.focal_x = width / (2.0f * tan_fovx);
    a.grid_x = (uint32_t)((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X);
    a.grid_y = (uint32_t)((height + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y);
    a.prefiltered = prefiltered; a.antialiasing = antialiasing;
    a.radii = radii ? radii : at<int>(gb, g.off[GEOM_RADII]);
    a.means2D = at<float>(gb, g.off[GEOM_MEANS2D]);
    a.depths = at<float>(gb, g.off[GEOM_DEPTH]);
    a.rgb = at<float>(gb, g.off[GEOM_RGB]);
    a.conic_opacity = at<float>(gb, g.off[GEOM_CONIC_OPACITY]);
    a.clamped = at<uint8_t>(gb, g.off[GEOM_CLAMPED]);
    a.tiles_touched = at<uint32_t>(gb, g.off[GEOM_TILES_TOUCHED]);
    a.host_flags = h_dev;
    a.scan_status = at<uint64_t>(gb, g.off[GEOM_SCAN_SCRATCH]);
    a.scan_status_words = 2 * scan_status_words(P);  // the depth-order and the index-order scan
    a.splat = at<float4>(gb, g.off[GEOM_SPLAT]);
    a.dkey = at<uint32_t>(gb, g.off[GEOM_DKEY]);
    a.rect = at<uint2>(gb, g.off[GEOM_RECT]);
    a.rect4 = nullptr;
    if (rect_packable(a.grid_x, a.grid_y)) {  // the depth sort carries the packed rect as payload
        a.rect4 = at<uint32_t>(gb, g.off[GEOM_RECT]);
        a.rect = nullptr;
    }
    a.rec_mask = at<uint32_t>(gb, g.off[GEOM_REC_MASK]);
    // the depth sort's chunk-group counts, zeroed by preprocess (SortJob::gsum_zeroed)
    a.dsort_gsum = at<uint32_t>(gb, g.off[GEOM_RADIX_SCRATCH] + radix_gsum_offset(P));
    a.dsort_gsum_words = (int)(radix_gsum_bytes(P) / 4);
    a.tile_diff = nullptr;
    a.tile_diff_words = 0;
    if (use_tile_diff(a.grid_x, a.grid_y)) {  // the tile ranges from the rects' difference array
        a.tile_diff = at<int>(image_buffer, image_layout(width, height).off[IMG_TILE_DIFF]);
        a.tile_diff_words = (int)((a.grid_x + 1) * (a.grid_y + 1));
    }
    *h_out = h;
    *hdev_out = h_dev;
    return GSR_OK;
}

// The forward tile order of a view whose tile ranges come from the rects' difference array
// (tile_hist): it needs nothing from the tile sort, so it runs on the auxiliary stream right after
// tile_hist, beside the depth and tile sorts, instead of between the tile sort and render_fwd.
static OrderJob diff_order_job(char* ib, int width, int height, uint32_t gx, uint32_t gy)
{
    const ImageLayout im = image_layout(width, height);
    OrderJob oj = {};
    oj.order = at<uint32_t>(ib, im.off[IMG_TILE_ORDER]);
    oj.diff = at<int>(ib, im.off[IMG_TILE_DIFF]);
    oj.ranges_out = at<uint2>(ib, im.off[IMG_RANGES]);
    oj.grid_x = gx;
    oj.grid_y = gy;
    return oj;
}

// After preprocess: the record-slot scan, the depth sort and the tile-count scan of one view.
static int forward_geometry_sort(const PreprocessArgs& a, char* gb, char* ib, int width, int height, int P,
                                 uint32_t* h_dev, hipStream_t s, bool debug, bool use_aux, SortJob* dsort_out,
                                 ScanJob* off_out)
{
    const GeomLayout g = geom_layout(P);
    // 1b. each Gaussian's first gradient-record slot: index-order exclusive scan of the tile counts
    //     (records in Gaussian order: preprocess_bwd's per-Gaussian gathers are contiguous), on the
    //     auxiliary stream beside the depth sort; the tile sort's first pass (which reads it) waits for it
    hipStream_t aux = s;
    {
        // (one auxiliary stream per device: views whose prefixes run side by side on several
        // prefix streams scan inline instead of coupling their streams through it)
        int rc = use_aux ? aux_fork(s, &aux) : GSR_OK;
        if (rc) return rc;
    }
    // every exit after the fork joins the auxiliary stream back first (the caller's stream stays
    // ordered after the scan queued there, which writes into the caller's geometry buffer)
    hipError_t e = launch_inclusive_scan(a.tiles_touched, nullptr, at<uint32_t>(gb, g.off[GEOM_EMIT_START]), P,
                                         a.scan_status + scan_status_words(P), nullptr, aux, true);
    if (e == hipSuccess && a.tile_diff) {  // the rects' difference array, beside the depth sort as well
        ProfScope ps_(PK_RANGES, aux);
        const TileHistJob hj = {a.rect4, P, a.tile_diff};
        e = launch_tile_hist_batch(&hj, 1, a.grid_x, a.grid_y, aux);
    }
    if (e == hipSuccess && a.tile_diff) {  // ... and from it the tile ranges and the forward's tile order
        ProfScope ps_(PK_TILE_ORDER, aux);
        const OrderJob oj = diff_order_job(ib, width, height, a.grid_x, a.grid_y);
        e = launch_tile_order_batch(&oj, 1, (int)(a.grid_x * a.grid_y), aux);
    }

    // 2. stable depth sort of the Gaussians (first half of the reference's tile|depth key sort)
    uint32_t* sorted_ids = at<uint32_t>(gb, g.off[GEOM_SORTED_IDS]);
    if (e == hipSuccess) {
        char* tmp = gb + g.off[GEOM_DSORT_TMP];
        const size_t q = align_up(4 * (size_t)P, 256);
        // keys u32, payload u32x2 (id, packed rect): k0 | v0 v0 | k1 | v1 v1
        uint32_t* k0 = reinterpret_cast<uint32_t*>(tmp);
        uint32_t* v0 = reinterpret_cast<uint32_t*>(tmp + q);
        uint32_t* k1 = reinterpret_cast<uint32_t*>(tmp + 3 * q);
        uint32_t* v1 = reinterpret_cast<uint32_t*>(tmp + 4 * q);
        ProfScope ps_(PK_DEPTH_SORT, s);
        // the last pass also lays the tile rects and tile counts out in depth order (the counts
        // into point_offsets, which the scan then turns into offsets in place)
        SortJob j = {P, a.dkey, nullptr, k0, v0, k1, v1, sorted_ids, nullptr, nullptr, gb + g.off[GEOM_RADIX_SCRATCH],
                     a.rect, at<uint2>(gb, g.off[GEOM_SORTED_RECT]), at<uint32_t>(gb, g.off[GEOM_POINT_OFFSETS]),
                     a.rect4};
        j.host_wide = h_dev + 1;
        j.gsum_zeroed = true;  // (preprocess)
        *dsort_out = j;
        e = radix_sort_batch(&j, 1, DEPTH_BITS, s);
    }
    if (debug && e == hipSuccess) e = hipStreamSynchronize(s);

    // 3. instance offsets in depth order (cub::DeviceScan::InclusiveSum, rasterizer_impl.cu:280)
    uint32_t* offsets = at<uint32_t>(gb, g.off[GEOM_POINT_OFFSETS]);
    *off_out = {offsets, offsets, P, a.scan_status, h_dev + 2};
    if (e == hipSuccess) {
        ProfScope ps_(PK_SCAN, s);
        e = launch_inclusive_scan(offsets, nullptr, offsets, P, a.scan_status, h_dev + 2, s);
    }
    {
        const int rc = aux_join(s, aux);
        if (e != hipSuccess) return fail_hip(e, __LINE__);
        if (rc) return rc;
    }
    DEBUG_SYNC(s);
    return GSR_OK;
}

// Forward, first half: preprocess, depth sort and the tile-count scan are enqueued; *h_out is the
// pinned word block the scan publishes num_rendered into (forward_geometry_wait reads it).
static int forward_geometry_launch(char* geometry_buffer, char* image_buffer, int P, int D, int M, int width,
                                   int height, const float* means3D, const float* dc, const float* shs,
                                   const float* colors_precomp, const float* opacities, const float* scales,
                                   float scale_modifier, const float* rotations, const float* cov3D_precomp,
                                   const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                                   float tan_fovx, float tan_fovy, bool prefiltered, bool antialiasing, int* radii,
                                   bool debug, gsr_stream_t stream, uint32_t** h_out, SortJob* dsort_out,
                                   ScanJob* off_out, int slot = 0, bool use_aux = true)
{
    hipStream_t s = (hipStream_t)stream;
    PreprocessArgs a;
    uint32_t* h_dev = nullptr;
    int rc = forward_geometry_args(geometry_buffer, image_buffer, P, D, M, width, height, means3D, dc, shs,
                                   colors_precomp, opacities, scales, scale_modifier, rotations, cov3D_precomp,
                                   viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered, antialiasing,
                                   radii, slot, &a, h_out, &h_dev);
    if (rc) return rc;
    // 1. preprocess (forward.cu:154-272)
    {
        ProfScope ps_(PK_PREPROCESS, s);
        HIP_TRY(launch_preprocess(a, s));
    }
    DEBUG_SYNC(s);
    return forward_geometry_sort(a, geometry_buffer, image_buffer, width, height, P, h_dev, s, debug, use_aux,
                                 dsort_out, off_out);
}

static int forward_geometry_wait(uint32_t* h, gsr_stream_t stream, int* num_rendered)
{
    hipStream_t s = (hipStream_t)stream;
    // 4. the one device->host hand-off of the forward: num_rendered (rasterizer_impl.cu:283-284),
    //    stored by the scan into pinned memory, plus the error flag.  The host polls the word
    //    itself (no driver wake-up on the critical path); hipStreamQuery now and then notices a
    //    stream that failed, or finished without storing it.
    for (uint32_t spin = 1;; spin++) {
        if (__atomic_load_n(&h[2], __ATOMIC_ACQUIRE) != L_PENDING) break;
        if ((spin & 1023u) == 0u) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) return fail_hip(q, __LINE__);
        }
    }
    if (__atomic_load_n(&h[2], __ATOMIC_ACQUIRE) == L_PENDING) return fail(GSR_ERR_HIP, "scan did not publish num_rendered");
    if (h[0] & 1u)
        return fail(GSR_ERR_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
    if (__atomic_load_n(&h[1], __ATOMIC_ACQUIRE)) return GSR_RERUN_WIDE;  // (stored before the scan ran: visible with L)
    if (h[2] > 0x7fffffffu) return fail(GSR_ERR_INVALID, "num_rendered overflows int");
    *num_rendered = (int)h[2];
    return GSR_OK;
}

// A view whose visible depth keys spanned too wide a range for the three-pass depth sort
// (forward_geometry_wait returned GSR_RERUN_WIDE): its depth sort runs again in four 8-bit passes and
// the tile-count scan re-publishes num_rendered (its status words cleared first), for THIS call only
// -- the next forward starts with three passes again (the reference's sort keeps no state,
// rasterizer_impl.cu:306-311).  Preprocess, the record-slot scan, the rects' difference array and the
// forward tile order do not depend on the depth order and stand.  (What follows the scan -- the tile
// sort's first-pass histograms -- is the caller's to enqueue again.)  h: the views' pinned words, whose
// scans have published (no kernel still writes them).
static int depth_sort_rerun_wide(SortJob* dsort, const ScanJob* off, uint32_t* const* h, int V, hipStream_t s)
{
    for (int v = 0; v < V; v++) {
        h[v][1] = 0;
        __atomic_store_n(&h[v][2], L_PENDING, __ATOMIC_RELEASE);
        dsort[v].host_wide = nullptr;  // (four passes: no range to report)
        HIP_TRY(hipMemsetAsync(off[v].status, 0, sizeof(uint64_t) * (size_t)scan_status_words(off[v].n), s));
    }
    {
        ProfScope ps_(PK_DEPTH_SORT, s);
        HIP_TRY(radix_sort_batch(dsort, V, DEPTH_BITS, s, 0, SORT_DEPTH, /*four_pass=*/true));
    }
    ProfScope ps_(PK_SCAN, s);
    HIP_TRY(launch_scan_batch(off, V, false, s));
    return GSR_OK;
}

int gsr_debug_last_depth_passes(int view) { return view >= 0 && view < 16 ? t_last_depth_passes[view] : 0; }

int gsr_debug_grad_record_floats(void) { return GRAD_REC; }

int gsr_forward_geometry_dc(char* geometry_buffer, char* image_buffer, int P, int D, int M, int width, int height,
                         const float* means3D, const float* dc, const float* shs, const float* colors_precomp,
                         const float* opacities, const float* scales, float scale_modifier,
                         const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                         const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                         bool prefiltered, bool antialiasing, int* radii, bool debug, gsr_stream_t stream,
                         int* num_rendered)
{
    *num_rendered = 0;
    if (P <= 0) return P < 0 ? fail(GSR_ERR_INVALID, "P must be >= 0") : GSR_OK;
    uint32_t* h = nullptr;
    hipStream_t ps = nullptr;
    int rc = prefix_begin((hipStream_t)stream, &ps);
    if (rc) return rc;
    SortJob dsort;
    ScanJob off;
    rc = forward_geometry_launch(geometry_buffer, image_buffer, P, D, M, width, height, means3D, dc, shs,
                                 colors_precomp, opacities, scales, scale_modifier, rotations, cov3D_precomp,
                                 viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered, antialiasing,
                                 radii, debug, ps, &h, &dsort, &off);
    if (rc) return rc;
    rc = forward_geometry_wait(h, ps, num_rendered);
    t_last_depth_passes[0] = depth_force_wide() ? 4 : 3;
    if (rc == GSR_RERUN_WIDE) {  // this call only: the depth sort in four passes
        rc = depth_sort_rerun_wide(&dsort, &off, &h, 1, ps);
        if (!rc) rc = forward_geometry_wait(h, ps, num_rendered);
        t_last_depth_passes[0] = 4;
    }
    const int rj = prefix_end((hipStream_t)stream, ps);
    return rc ? rc : rj;
}

static int forward_render_impl(char* geometry_buffer, char* binning_buffer, char* image_buffer, int P,
                               int num_rendered, const float* background, int width, int height, float* out_color,
                               float* depth, bool debug, gsr_stream_t stream, hipStream_t prefix,
                               bool counted = false);

// The tile sort of one view (L > 0 instances) with the instance emission fused into its first
// pass: the instances are generated from the depth-ordered rects; the sort's ping-pong buffers live
// in the (not yet used) gradient-record region of the binning buffer, the first pass's count
// matrix in the depth sort's ping-pong buffer (free by then).
static TileSortJob fused_tile_sort_job(char* gb, char* bb, char* ib, int P, int L, int width, int height)
{
    const GeomLayout g = geom_layout(P);
    const ImageLayout im = image_layout(width, height);
    const BinLayout b = bin_layout(L);
    const size_t q = align_up(4 * (size_t)L, 256);
    TileSortJob j = {};
    j.P = P;
    j.L = L;
    j.sorted_ids = at<uint32_t>(gb, g.off[GEOM_SORTED_IDS]);
    j.offsets = at<uint32_t>(gb, g.off[GEOM_POINT_OFFSETS]);
    j.sorted_rects = at<uint2>(gb, g.off[GEOM_SORTED_RECT]);
    j.rec_start = at<uint32_t>(gb, g.off[GEOM_EMIT_START]);
    j.pass1_scratch = gb + g.off[GEOM_DSORT_TMP];
    const bool diff = use_tile_diff((uint32_t)((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X),
                                    (uint32_t)((height + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y));
    // with the difference array the tile order writes every range and nothing reads the sorted
    // tile ids: no clearing of the ranges, no tile id written per instance
    j.ranges = diff ? nullptr : at<uint2>(ib, im.off[IMG_RANGES]);
    if (!bb) return j;  // the histogram phase only (FUSED_COUNT): no binning buffer yet
    char* w = bb + b.off[BIN_GRAD_INST];
    j.k0 = reinterpret_cast<uint32_t*>(w + 2 * q);
    j.k1 = reinterpret_cast<uint32_t*>(w + 3 * q);
    j.v0 = reinterpret_cast<uint32_t*>(w + 4 * q);  // u32x2 payloads
    j.v1 = reinterpret_cast<uint32_t*>(w + 6 * q);
    j.scratch = bb + b.off[BIN_RADIX_SCRATCH];
    j.slotless = slots_from_rect((uint32_t)((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X),
                                 (uint32_t)((height + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y));
    j.out_slot = j.slotless ? nullptr : at<uint32_t>(bb, b.off[BIN_SLOT]);
    j.out_ids = at<uint32_t>(bb, b.off[BIN_POINT_LIST]);
    j.out_tiles = diff ? nullptr : at<uint32_t>(bb, b.off[BIN_SORTED_TILES]);
    j.valid = at<uint32_t>(bb, b.off[BIN_VALID]);
    return j;
}

int gsr_forward_render(char* geometry_buffer, char* binning_buffer, char* image_buffer, int P, int num_rendered,
                       const float* background, int width, int height, const float* colors_precomp,
                       float* out_color, float* depth, int* radii, bool debug, gsr_stream_t stream)
{
    (void)radii;
    (void)colors_precomp;
    hipStream_t ps = nullptr;
    const int rc = prefix_begin((hipStream_t)stream, &ps);
    if (rc) return rc;
    return forward_render_impl(geometry_buffer, binning_buffer, image_buffer, P, num_rendered, background, width,
                               height, out_color, depth, debug, stream, ps);
}

// render_fwd's arguments for a view whose binning is complete
static RenderFwdArgs render_fwd_args(char* gb, char* bb, char* ib, int P, int L, const float* background, int width,
                                     int height, float* out_color, float* depth)
{
    const GeomLayout g = geom_layout(P);
    const ImageLayout im = image_layout(width, height);
    const BinLayout b = bin_layout(L);
    RenderFwdArgs r;
    r.ranges = at<uint2>(ib, im.off[IMG_RANGES]);
    r.tile_order = at<uint32_t>(ib, im.off[IMG_TILE_ORDER]);
    r.tile_work = at<uint32_t>(ib, im.off[IMG_TILE_WORK]);
    r.point_list = L > 0 ? at<uint32_t>(bb, b.off[BIN_POINT_LIST]) : nullptr;
    r.W = width; r.H = height;
    r.grid_x = (uint32_t)((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X);
    r.splat = at<float4>(gb, g.off[GEOM_SPLAT]);
    r.bg = background;
    r.final_T = at<float>(ib, im.off[IMG_FINAL_T]);
    r.n_contrib = at<uint32_t>(ib, im.off[IMG_N_CONTRIB]);
    r.out_color = out_color;
    r.invdepth = depth;
    r.hit = L > 0 ? at<uint8_t>(bb, b.off[BIN_HIT]) : nullptr;
    return r;
}

// Forward, second half: the tile sort (emission fused in), tile ranges and tile order on the
// prefix stream, render_fwd on the caller's.
// counted: the tile sort's first-pass histograms already ran (enqueued before the L read-back)
static int forward_render_impl(char* geometry_buffer, char* binning_buffer, char* image_buffer, int P,
                               int num_rendered, const float* background, int width, int height, float* out_color,
                               float* depth, bool debug, gsr_stream_t stream, hipStream_t prefix, bool counted)
{
    // (colors_precomp was folded into the render record by preprocess)
    hipStream_t s = prefix;
    hipStream_t caller = (hipStream_t)stream;
    if (P <= 0) return prefix_end(caller, prefix);
    const int L = num_rendered;
    const ImageLayout im = image_layout(width, height);
    const BinLayout b = bin_layout(L);
    char* gb = geometry_buffer;
    char* ib = image_buffer;
    char* bb = binning_buffer;
    if (L > 0 && !bb) return fail(GSR_ERR_ALLOC, "null binning buffer");
    const uint32_t gx = (uint32_t)((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X);
    const uint32_t gy = (uint32_t)((height + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y);
    const int T = (int)(gx * gy);
    uint32_t* sorted_tiles = L > 0 ? at<uint32_t>(bb, b.off[BIN_SORTED_TILES]) : nullptr;
    if (L > 0) {
        // stable sort by tile id over bits [0, msb(T)) of the depth-ordered instances
        // (rasterizer_impl.cu:303-311 sorts [0, 32 + msb(T)) of the tile|depth keys)
        const TileSortJob j = fused_tile_sort_job(gb, bb, ib, P, L, width, height);
        ProfScope ps_(PK_TILE_SORT, s, counted);
        HIP_TRY(tile_sort_fused_batch(&j, 1, gx, T, s, counted ? FUSED_SCATTER : FUSED_ALL));
    }
    DEBUG_SYNC(s);
    uint2* ranges = at<uint2>(ib, im.off[IMG_RANGES]);
    uint32_t* tile_order = at<uint32_t>(ib, im.off[IMG_TILE_ORDER]);
    if (use_tile_diff(gx, gy)) {
        // ranges and order: written from the rects' difference array by the geometry half (the
        // auxiliary stream, joined before the tile-count scan)
    } else {
        {
            ProfScope ps_(PK_RANGES, s);
            HIP_TRY(launch_tile_ranges(L, sorted_tiles, ranges, T, s));
        }
        DEBUG_SYNC(s);
        ProfScope ps_(PK_TILE_ORDER, s);
        HIP_TRY(launch_tile_order(ranges, nullptr, T, tile_order, s));
    }
    {
        const int rc = prefix_end(caller, prefix);
        if (rc) return rc;
    }
    s = caller;
    const RenderFwdArgs r = render_fwd_args(gb, bb, ib, P, L, background, width, height, out_color, depth);
    {
        ProfScope ps_(PK_RENDER_FWD, s);
        HIP_TRY(launch_render_fwd(r, T, s));
    }
    DEBUG_SYNC(s);
    return GSR_OK;
}

int gsr_forward_dc(gsr_resize_fn geometryBuffer, void* geometry_ctx, gsr_resize_fn binningBuffer, void* binning_ctx,
                gsr_resize_fn imageBuffer, void* image_ctx, int P, int D, int M, const float* background, int width,
                int height, const float* means3D, const float* dc, const float* shs, const float* colors_precomp,
                const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                float tan_fovx, float tan_fovy, bool prefiltered, float* out_color, float* depth, bool antialiasing,
                int* radii, bool debug, gsr_stream_t stream, int* num_rendered)
{
    *num_rendered = 0;
    if (P == 0) return GSR_OK;  // rasterize_points.cu:88 -- outputs stay as allocated
    char* gb = geometryBuffer(geometry_ctx, gsr_geometry_buffer_size(P));
    char* ib = imageBuffer(image_ctx, gsr_image_buffer_size(width, height));
    if (!gb || !ib) return fail(GSR_ERR_ALLOC, "resize callback returned NULL");
    int L = 0;
    int rc = gsr_forward_geometry_dc(gb, ib, P, D, M, width, height, means3D, dc, shs, colors_precomp, opacities, scales,
                                  scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx,
                                  tan_fovy, prefiltered, antialiasing, radii, debug, stream, &L);
    if (rc) return rc;
    char* bb = binningBuffer(binning_ctx, gsr_binning_buffer_size(L));
    if (!bb) return fail(GSR_ERR_ALLOC, "resize callback returned NULL");
    rc = gsr_forward_render(gb, bb, ib, P, L, background, width, height, colors_precomp, out_color, depth, radii,
                            debug, stream);
    if (rc) return rc;
    *num_rendered = L;
    return GSR_OK;
}

int gsr_forward_prealloc_dc(char* geometry_buffer, char* image_buffer, char* binning_buffer, size_t binning_capacity,
                         int P, int D, int M, const float* background, int width, int height, const float* means3D,
                         const float* dc, const float* shs, const float* colors_precomp, const float* opacities,
                         const float* scales, float scale_modifier, const float* rotations,
                         const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                         const float* cam_pos, float tan_fovx, float tan_fovy, bool prefiltered, bool antialiasing,
                         float* out_color, float* depth, int* radii, bool debug, gsr_stream_t stream,
                         int* num_rendered, int* rendered)
{
    (void)colors_precomp;
    *rendered = 0;
    *num_rendered = 0;
    if (P <= 0) return P < 0 ? fail(GSR_ERR_INVALID, "P must be >= 0") : GSR_OK;
    uint32_t* h = nullptr;
    hipStream_t ps = nullptr;
    int rc = prefix_begin((hipStream_t)stream, &ps);
    if (rc) return rc;
    SortJob dsort;
    ScanJob off;
    rc = forward_geometry_launch(geometry_buffer, image_buffer, P, D, M, width, height, means3D, dc, shs,
                                 colors_precomp, opacities, scales, scale_modifier, rotations, cov3D_precomp,
                                 viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered, antialiasing,
                                 radii, debug, ps, &h, &dsort, &off);
    if (rc) return rc;
    // the tile sort's first-pass histograms need only the depth-ordered rects and offsets (not L or
    // the binning buffer): enqueued before the read-back, they run while the host waits
    auto count_pass = [&]() -> int {
        const uint32_t gx = (uint32_t)((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X);
        const int T = (int)(gx * (uint32_t)((height + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y));
        const TileSortJob cj = fused_tile_sort_job(geometry_buffer, nullptr, image_buffer, P, 0, width, height);
        ProfScope ps_(PK_TILE_SORT, ps);
        const hipError_t e = tile_sort_fused_batch(&cj, 1, gx, T, ps, FUSED_COUNT);
        return e == hipSuccess ? GSR_OK : fail_hip(e, __LINE__);
    };
    rc = count_pass();
    if (rc) {
        prefix_end((hipStream_t)stream, ps);
        return rc;
    }
    int L = 0;
    rc = forward_geometry_wait(h, ps, &L);
    t_last_depth_passes[0] = depth_force_wide() ? 4 : 3;
    if (rc == GSR_RERUN_WIDE) {  // this call only: the depth sort in four passes, then its histograms again
        rc = depth_sort_rerun_wide(&dsort, &off, &h, 1, ps);
        if (!rc) rc = count_pass();
        if (!rc) rc = forward_geometry_wait(h, ps, &L);
        t_last_depth_passes[0] = 4;
    }
    *num_rendered = L;
    if (rc) {
        prefix_end((hipStream_t)stream, ps);
        return rc;
    }
    if (!binning_buffer || gsr_binning_buffer_size(L) > binning_capacity)  // caller allocates
        return prefix_end((hipStream_t)stream, ps);
    rc = forward_render_impl(geometry_buffer, binning_buffer, image_buffer, P, L, background, width, height,
                             out_color, depth, debug, stream, ps, true);
    if (rc) return rc;
    *rendered = 1;
    return GSR_OK;
}

int gsr_forward_views(int V, int P, int D, int M, const float* background, int width, int height,
                      const float* means3D, const float* dc, const float* shs, const float* colors_precomp,
                      const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                      const float* cov3D_precomp, const float* const* viewmatrices, const float* const* projmatrices,
                      const float* const* campos, const float* tan_fovx, const float* tan_fovy, bool prefiltered,
                      bool antialiasing, char* const* geometry_buffers, char* const* image_buffers,
                      char* const* binning_buffers, const size_t* binning_capacity, float* const* out_colors,
                      float* const* out_invdepths, int* const* radii, bool debug, gsr_stream_t stream,
                      int* num_rendered, int* rendered)
{
    if (V < 1 || V > MAX_VIEWS) return fail(GSR_ERR_INVALID, "V must be in [1, 16]");
    if (!viewmatrices || !projmatrices || !campos || !tan_fovx || !tan_fovy || !geometry_buffers || !image_buffers ||
        !binning_buffers || !binning_capacity || !out_colors || !out_invdepths || !num_rendered || !rendered)
        return fail(GSR_ERR_INVALID, "null per-view array");
    for (int v = 0; v < V; v++) {
        num_rendered[v] = 0;
        rendered[v] = 0;
    }
    if (P <= 0) return P < 0 ? fail(GSR_ERR_INVALID, "P must be >= 0") : GSR_OK;
    hipStream_t caller = (hipStream_t)stream;
    const uint32_t gx = (uint32_t)((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X);
    const uint32_t gy = (uint32_t)((height + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y);
    const int T = (int)(gx * gy);
    const GeomLayout g = geom_layout(P);
    const ImageLayout im = image_layout(width, height);

    uint32_t* h[MAX_VIEWS];
    PreprocessArgs pa[MAX_VIEWS];
    uint32_t* hdev[MAX_VIEWS];
    for (int v = 0; v < V; v++) {
        if (!geometry_buffers[v] || !image_buffers[v]) return fail(GSR_ERR_ALLOC, "null state buffer");
        if (!out_colors[v] || !out_invdepths[v]) return fail(GSR_ERR_INVALID, "null per-view output");
        const int rc = forward_geometry_args(geometry_buffers[v], image_buffers[v], P, D, M, width, height, means3D, dc,
                                             shs, colors_precomp, opacities, scales, scale_modifier, rotations,
                                             cov3D_precomp, viewmatrices[v], projmatrices[v], campos[v], tan_fovx[v],
                                             tan_fovy[v], prefiltered, antialiasing, radii ? radii[v] : nullptr, v,
                                             &pa[v], &h[v], &hdev[v]);
        if (rc) return rc;
        // GeometryState's means2D, depths, rgb and conic_opacity are read by nothing after the forward: the
        // batched forward does not write them (40 B per visible Gaussian and view)
        pa[v].means2D = nullptr;
        pa[v].depths = nullptr;
        pa[v].rgb = nullptr;
        pa[v].conic_opacity = nullptr;  // (preprocess_bwd recomputes it: 16 B per visible Gaussian and view)
    }
    // The binning prefix of all V views, batched: every stage is one launch over all views
    // (grid.y = view), on the caller's stream like the renders that follow (a separate prefix
    // stream would overlap nothing here -- it would fork from the caller's previous work and the
    // render would join it -- and each hop between the queues costs ~10 us of idle GPU).
    hipStream_t ps = caller;
    int rc = GSR_OK;
    {
        ProfScope ps_(PK_PREPROCESS, ps);
        HIP_TRY(launch_preprocess_views(pa, V, ps));  // the parameters and SH rows read once per 8 views
    }
    DEBUG_SYNC(ps);
    ScanJob rec[MAX_VIEWS], off[MAX_VIEWS];
    SortJob dsort[MAX_VIEWS];
    for (int v = 0; v < V; v++) {
        char* gb = geometry_buffers[v];
        const PreprocessArgs& a = pa[v];
        // each Gaussian's first gradient-record slot (index-order exclusive scan of the tile counts)
        rec[v] = {a.tiles_touched, at<uint32_t>(gb, g.off[GEOM_EMIT_START]), P, a.scan_status + scan_status_words(P),
                  nullptr};
        char* tmp = gb + g.off[GEOM_DSORT_TMP];
        const size_t q = align_up(4 * (size_t)P, 256);
        // keys u32, payload u32x2 (id, packed rect): k0 | v0 v0 | k1 | v1 v1
        dsort[v] = {P, a.dkey, nullptr, reinterpret_cast<uint32_t*>(tmp), reinterpret_cast<uint32_t*>(tmp + q),
                    reinterpret_cast<uint32_t*>(tmp + 3 * q), reinterpret_cast<uint32_t*>(tmp + 4 * q),
                    at<uint32_t>(gb, g.off[GEOM_SORTED_IDS]), nullptr, nullptr, gb + g.off[GEOM_RADIX_SCRATCH], a.rect,
                    at<uint2>(gb, g.off[GEOM_SORTED_RECT]), at<uint32_t>(gb, g.off[GEOM_POINT_OFFSETS]), a.rect4};
        uint32_t* offsets = at<uint32_t>(gb, g.off[GEOM_POINT_OFFSETS]);
        off[v] = {offsets, offsets, P, a.scan_status, hdev[v] + 2};  // L -> the view's pinned word
        dsort[v].host_wide = hdev[v] + 1;
        dsort[v].gsum_zeroed = true;  // (preprocess)
    }
    // the record-slot scans (read only by the fused tile sort) on the auxiliary stream, beside the
    // depth sorts
    hipStream_t aux = ps;
    rc = aux_fork(ps, &aux);
    if (rc) return rc;
    {
        // every exit after the fork joins the auxiliary stream back first: the caller's stream
        // must stay ordered after what is already queued there (it writes the caller's buffers)
        hipError_t e = launch_scan_batch(rec, V, true, aux);
        if (e == hipSuccess && use_tile_diff(gx, gy)) {  // the rects' difference arrays, beside the depth sorts
            TileHistJob hj[MAX_VIEWS];
            for (int v = 0; v < V; v++) hj[v] = {pa[v].rect4, P, pa[v].tile_diff};
            {
                ProfScope ps_(PK_RANGES, aux);
                e = launch_tile_hist_batch(hj, V, gx, gy, aux);
            }
            if (e == hipSuccess) {  // the views' tile ranges and forward tile orders, beside the sorts
                OrderJob dj[MAX_VIEWS];
                for (int v = 0; v < V; v++) dj[v] = diff_order_job(image_buffers[v], width, height, gx, gy);
                ProfScope ps_(PK_TILE_ORDER, aux);
                e = launch_tile_order_batch(dj, V, T, aux);
            }
        }
        if (e == hipSuccess) {
            ProfScope ps_(PK_DEPTH_SORT, ps);
            e = radix_sort_batch(dsort, V, DEPTH_BITS, ps);
        }
        rc = aux_join(ps, aux);
        if (e != hipSuccess) return fail_hip(e, __LINE__);
    }
    if (rc) return rc;
    {
        ProfScope ps_(PK_SCAN, ps);
        HIP_TRY(launch_scan_batch(off, V, false, ps));
    }
    // the first tile-sort pass's histograms need only the depth-ordered rects and offsets: the GPU
    // computes them while the host waits for L below
    auto count_pass = [&](const int* which, int n) -> hipError_t {
        TileSortJob cj[MAX_VIEWS];
        for (int i = 0; i < n; i++)
            cj[i] = fused_tile_sort_job(geometry_buffers[which[i]], nullptr, image_buffers[which[i]], P, 0, width, height);
        ProfScope ps_(PK_TILE_SORT, ps);
        return tile_sort_fused_batch(cj, n, gx, T, ps, FUSED_COUNT);
    };
    {
        int all[MAX_VIEWS];
        for (int v = 0; v < V; v++) all[v] = v;
        HIP_TRY(count_pass(all, V));
    }
    DEBUG_SYNC(ps);
    // the one host hand-off: every view's num_rendered (rasterizer_impl.cu:283-284); a view whose depth
    // range was too wide for three passes re-runs its depth sort in four (this call only)
    int L[MAX_VIEWS];
    int wide[MAX_VIEWS], nw = 0;
    for (int v = 0; v < V && !rc; v++) {
        rc = forward_geometry_wait(h[v], ps, &L[v]);
        t_last_depth_passes[v] = depth_force_wide() ? 4 : 3;
        if (rc == GSR_RERUN_WIDE) {
            wide[nw++] = v;
            rc = GSR_OK;
        }
    }
    if (!rc && nw) {
        SortJob wj[MAX_VIEWS];
        ScanJob wo[MAX_VIEWS];
        uint32_t* wh[MAX_VIEWS];
        for (int i = 0; i < nw; i++) {
            wj[i] = dsort[wide[i]];
            wo[i] = off[wide[i]];
            wh[i] = h[wide[i]];
            t_last_depth_passes[wide[i]] = 4;
        }
        rc = depth_sort_rerun_wide(wj, wo, wh, nw, ps);
        if (!rc) {
            const hipError_t e = count_pass(wide, nw);
            if (e != hipSuccess) rc = fail_hip(e, __LINE__);
        }
        for (int i = 0; i < nw && !rc; i++) rc = forward_geometry_wait(h[wide[i]], ps, &L[wide[i]]);
    }
    for (int v = 0; v < V; v++) num_rendered[v] = rc ? 0 : L[v];
    if (rc) {
        prefix_end(caller, ps);
        return rc;
    }
    // views whose binning buffer holds them: emission fused into the tile sort, tile ranges and
    // tile order, batched (the others are left to the caller: allocate
    // gsr_binning_buffer_size(num_rendered[v]), then gsr_forward_render)
    int fit[MAX_VIEWS], nf = 0;
    TileSortJob tsort[MAX_VIEWS];
    RangesJob rj[MAX_VIEWS];
    OrderJob oj[MAX_VIEWS];
    int ns = 0;
    for (int v = 0; v < V; v++) {
        if (!binning_buffers[v] || binning_capacity[v] == 0 || gsr_binning_buffer_size(L[v]) > binning_capacity[v])
            continue;
        char* bb = binning_buffers[v];
        char* ib = image_buffers[v];
        char* gb = geometry_buffers[v];
        const BinLayout b = bin_layout(L[v]);
        if (L[v] > 0) tsort[ns++] = fused_tile_sort_job(gb, bb, ib, P, L[v], width, height);
        rj[nf] = {L[v], L[v] > 0 ? at<uint32_t>(bb, b.off[BIN_SORTED_TILES]) : nullptr, at<uint2>(ib, im.off[IMG_RANGES])};
        oj[nf] = {at<uint2>(ib, im.off[IMG_RANGES]), nullptr, at<uint32_t>(ib, im.off[IMG_TILE_ORDER])};
        fit[nf++] = v;
    }
    if (ns) {
        ProfScope ps_(PK_TILE_SORT, ps, true);
        HIP_TRY(tile_sort_fused_batch(tsort, ns, gx, T, ps, FUSED_SCATTER));
    }
    if (nf && !use_tile_diff(gx, gy)) {  // (with the difference array: ranges and orders are done)
        {
            ProfScope ps_(PK_RANGES, ps);
            HIP_TRY(launch_tile_ranges_batch(rj, nf, T, ps));
        }
        ProfScope ps_(PK_TILE_ORDER, ps);
        HIP_TRY(launch_tile_order_batch(oj, nf, T, ps));
    }
    DEBUG_SYNC(ps);
    rc = prefix_end(caller, ps);
    if (rc) return rc;
    RenderFwdArgs ra[MAX_VIEWS];
    for (int k = 0; k < nf; k++) {
        const int v = fit[k];
        ra[k] = render_fwd_args(geometry_buffers[v], binning_buffers[v], image_buffers[v], P, L[v], background, width,
                                height, out_colors[v], out_invdepths[v]);
        rendered[v] = 1;
    }
    if (nf) {  // every view's render in one launch (one launch tail per batch)
        ProfScope ps_(PK_RENDER_FWD, caller);
        HIP_TRY(launch_render_fwd_batch(ra, nf, T, caller));
    }
    DEBUG_SYNC(caller);
    return GSR_OK;
}

int gsr_backward_dc_acc(int P, int D, int M, int R, const float* background, int width, int height,
                        const float* means3D, const float* dc, const float* shs, const float* colors_precomp,
                        const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                        const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                        const float* campos, float tan_fovx, float tan_fovy, const int* radii, char* geom_buffer,
                        char* binning_buffer, char* image_buffer, const float* dL_dpix, const float* dL_invdepths,
                        float* dL_dmean2D, float* dL_dconic, float* dL_dopacity, float* dL_dcolor,
                        float* dL_dinvdepth, float* dL_dmean3D, float* dL_dcov3D, float* dL_ddc, float* dL_dsh,
                        float* dL_dscale, float* dL_drot, bool antialiasing, bool debug, unsigned accumulate,
                        gsr_stream_t stream)
{
    if (accumulate & ~(unsigned)GSR_ACC_ALL) return fail(GSR_ERR_INVALID, "unknown accumulate bits");
    if (dc && !dL_ddc) return fail(GSR_ERR_INVALID, "dc given without dL_ddc");
    if (dc && colors_precomp)
        return fail(GSR_ERR_INVALID, "Please provide exactly one of either SHs or precomputed colors!");
    if (dc && M > 0 && (!shs || !dL_dsh)) return fail(GSR_ERR_INVALID, "dc given with M > 0 but shs/dL_dsh NULL");
    (void)colors_precomp;
    hipStream_t s = (hipStream_t)stream;
    if (P <= 0) return GSR_OK;
    const GeomLayout g = geom_layout(P);
    const ImageLayout im = image_layout(width, height);
    const BinLayout b = bin_layout(R);
    char* gb = geom_buffer;
    char* ib = image_buffer;
    char* bb = binning_buffer;
    if (R > 0 && !bb) return fail(GSR_ERR_ALLOC, "null binning buffer");
    const uint32_t gx = (uint32_t)((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X);
    const uint32_t gy = (uint32_t)((height + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y);
    const int T = (int)(gx * gy);
    const int* rad = radii ? radii : at<int>(gb, g.off[GEOM_RADII]);
    if ((dL_invdepths == nullptr) != (dL_dinvdepth == nullptr) && dL_dinvdepth == nullptr)
        return fail(GSR_ERR_INVALID, "dL_dinvdepth must be given with dL_invdepths");

    // BACKWARD::render (rasterizer_impl.cu:399-418): per-(tile, Gaussian) gradient records
    RenderBwdArgs r;
    r.ranges = at<uint2>(ib, im.off[IMG_RANGES]);
    r.tile_order = at<uint32_t>(ib, im.off[IMG_TILE_ORDER]);
    r.tile_work = at<uint32_t>(ib, im.off[IMG_TILE_WORK]);
    r.point_list = R > 0 ? at<uint32_t>(bb, b.off[BIN_POINT_LIST]) : nullptr;
    r.W = width; r.H = height; r.grid_x = gx;
    r.T = (int)(gx * gy);
    r.bg = background;
    r.splat = at<float4>(gb, g.off[GEOM_SPLAT]);
    r.final_Ts = at<float>(ib, im.off[IMG_FINAL_T]);
    r.n_contrib = at<uint32_t>(ib, im.off[IMG_N_CONTRIB]);
    r.dL_dpixels = dL_dpix;
    r.dL_invdepths = dL_invdepths;
    r.grad_inst = R > 0 ? at<float>(bb, b.off[BIN_GRAD_INST]) : nullptr;
    r.slot = R > 0 && !slots_from_rect(gx, gy) ? at<uint32_t>(bb, b.off[BIN_SLOT]) : nullptr;
    r.valid = R > 0 ? at<uint32_t>(bb, b.off[BIN_VALID]) : nullptr;
    r.hit = R > 0 ? at<uint8_t>(bb, b.off[BIN_HIT]) : nullptr;
    r.emit_start = at<uint32_t>(gb, g.off[GEOM_EMIT_START]);
    r.rec_mask = at<uint32_t>(gb, g.off[GEOM_REC_MASK]);
    if (R > 0) {
        {
            ProfScope ps_(PK_TILE_ORDER, s);
            HIP_TRY(launch_tile_order(nullptr, at<uint32_t>(ib, im.off[IMG_TILE_WORK]), T,
                                      at<uint32_t>(ib, im.off[IMG_TILE_ORDER]), s));
        }
        {
            ProfScope ps_(PK_RENDER_BWD, s);  // valid[] was cleared by the forward's tile sort
            HIP_TRY(launch_render_bwd(r, T, s));
        }
        DEBUG_SYNC(s);
    }

    // BACKWARD::preprocess (rasterizer_impl.cu:423-449), with the per-Gaussian gather of the records:
    // the batched kernel at one lane per Gaussian (launch_preprocess_bwd_single)
    PreprocessBwdViewsArgs A;
    PreprocessBwdArgs& p = A.a;
    p.P = P; p.D = D; p.M = dc ? M + 1 : M;
    p.means3D = means3D; p.radii = rad; p.shs = shs; p.dc = dc; p.dL_ddc = dc ? dL_ddc : nullptr;
    p.opacities = opacities; p.scales = scales; p.rotations = rotations; p.scale_modifier = scale_modifier;
    p.cov3D_precomp = cov3D_precomp;
    p.antialiasing = antialiasing;
    p.has_invdepth = dL_invdepths != nullptr;
    p.W = width; p.H = height;
    p.dL_dconic = dL_dconic; p.dL_dinvdepth = dL_dinvdepth;
    p.dL_dopacity = dL_dopacity; p.dL_dcolor = dL_dcolor;
    p.dL_dmean3D = dL_dmean3D; p.dL_dcov3D = dL_dcov3D; p.dL_dsh = (shs && M > 0) ? dL_dsh : nullptr;
    p.dL_dscale = dL_dscale; p.dL_drot = dL_drot;
    p.acc = accumulate;
    A.V = 1;
    A.g_begin = 0;
    A.g_end = P;
    BwdView& bv = A.v[0];
    bv.view = viewmatrix; bv.proj = projmatrix; bv.campos = campos;
    bv.focal_y = height / (2.0f * tan_fovy);
    bv.focal_x = width / (2.0f * tan_fovx);
    bv.tan_fovx = tan_fovx; bv.tan_fovy = tan_fovy;
    bv.radii = rad;
    bv.conic_opacity = at<float4>(gb, g.off[GEOM_CONIC_OPACITY]);
    bv.clamped = at<uint8_t>(gb, g.off[GEOM_CLAMPED]);
    bv.emit_start = at<uint32_t>(gb, g.off[GEOM_EMIT_START]);
    bv.tiles_touched = at<uint32_t>(gb, g.off[GEOM_TILES_TOUCHED]);
    bv.grad_inst = R > 0 ? at<float>(bb, b.off[BIN_GRAD_INST]) : nullptr;
    bv.valid = R > 0 ? at<uint32_t>(bb, b.off[BIN_VALID]) : nullptr;
    bv.rec_mask = at<uint32_t>(gb, g.off[GEOM_REC_MASK]);
    bv.dL_dmean2D = dL_dmean2D;
    {
        ProfScope ps_(PK_PREPROCESS_BWD, s);
        HIP_TRY(launch_preprocess_bwd_single(A, s));
    }
    DEBUG_SYNC(s);
    return GSR_OK;
}

int gsr_backward_dc(int P, int D, int M, int R, const float* background, int width, int height, const float* means3D,
                    const float* dc, const float* shs, const float* colors_precomp, const float* opacities,
                    const float* scales, float scale_modifier, const float* rotations, const float* cov3D_precomp,
                    const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                    float tan_fovy, const int* radii, char* geom_buffer, char* binning_buffer, char* image_buffer,
                    const float* dL_dpix, const float* dL_invdepths, float* dL_dmean2D, float* dL_dconic,
                    float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth, float* dL_dmean3D, float* dL_dcov3D,
                    float* dL_ddc, float* dL_dsh, float* dL_dscale, float* dL_drot, bool antialiasing, bool debug,
                    gsr_stream_t stream)
{
    return gsr_backward_dc_acc(P, D, M, R, background, width, height, means3D, dc, shs, colors_precomp, opacities,
                               scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos,
                               tan_fovx, tan_fovy, radii, geom_buffer, binning_buffer, image_buffer, dL_dpix,
                               dL_invdepths, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor, dL_dinvdepth, dL_dmean3D,
                               dL_dcov3D, dL_ddc, dL_dsh, dL_dscale, dL_drot, antialiasing, debug, 0u, stream);
}

// render_bwd's arguments for one view (P, R > 0)
static RenderBwdArgs render_bwd_args(int P, int R, const float* background, int width, int height, char* gb,
                                     char* bb, char* ib, const float* dL_dpix, const float* dL_invdepths)
{
    const GeomLayout g = geom_layout(P);
    const ImageLayout im = image_layout(width, height);
    const BinLayout b = bin_layout(R);
    const uint32_t gx = (uint32_t)((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X);
    const uint32_t gy = (uint32_t)((height + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y);
    RenderBwdArgs r;
    r.ranges = at<uint2>(ib, im.off[IMG_RANGES]);
    r.tile_order = at<uint32_t>(ib, im.off[IMG_TILE_ORDER]);
    r.tile_work = at<uint32_t>(ib, im.off[IMG_TILE_WORK]);
    r.point_list = at<uint32_t>(bb, b.off[BIN_POINT_LIST]);
    r.W = width; r.H = height; r.grid_x = gx;
    r.T = (int)(gx * gy);
    r.bg = background;
    r.splat = at<float4>(gb, g.off[GEOM_SPLAT]);
    r.final_Ts = at<float>(ib, im.off[IMG_FINAL_T]);
    r.n_contrib = at<uint32_t>(ib, im.off[IMG_N_CONTRIB]);
    r.dL_dpixels = dL_dpix;
    r.dL_invdepths = dL_invdepths;
    r.grad_inst = at<float>(bb, b.off[BIN_GRAD_INST]);
    r.slot = slots_from_rect(gx, gy) ? nullptr : at<uint32_t>(bb, b.off[BIN_SLOT]);  // (render_bwd derives them)
    r.valid = at<uint32_t>(bb, b.off[BIN_VALID]);
    r.hit = at<uint8_t>(bb, b.off[BIN_HIT]);
    r.emit_start = at<uint32_t>(gb, g.off[GEOM_EMIT_START]);
    r.rec_mask = at<uint32_t>(gb, g.off[GEOM_REC_MASK]);
    return r;
}

int gsr_backward_render(int P, int R, const float* background, int width, int height, char* geom_buffer,
                        char* binning_buffer, char* image_buffer, const float* dL_dpix, const float* dL_invdepths,
                        bool debug, gsr_stream_t stream)
{
    hipStream_t s = (hipStream_t)stream;
    if (P < 0 || R < 0) return fail(GSR_ERR_INVALID, "P and R must be >= 0");
    if (P == 0 || R == 0) return GSR_OK;
    if (!geom_buffer || !image_buffer || !binning_buffer) return fail(GSR_ERR_ALLOC, "null state buffer");
    if (!dL_dpix) return fail(GSR_ERR_INVALID, "null dL_dpix");
    const ImageLayout im = image_layout(width, height);
    const RenderBwdArgs r = render_bwd_args(P, R, background, width, height, geom_buffer, binning_buffer, image_buffer,
                                            dL_dpix, dL_invdepths);
    {
        ProfScope ps_(PK_TILE_ORDER, s);
        HIP_TRY(launch_tile_order(nullptr, at<uint32_t>(image_buffer, im.off[IMG_TILE_WORK]), r.T,
                                  at<uint32_t>(image_buffer, im.off[IMG_TILE_ORDER]), s));
    }
    {
        ProfScope ps_(PK_RENDER_BWD, s);  // valid[] was cleared by the forward's tile sort
        HIP_TRY(launch_render_bwd(r, r.T, s));
    }
    DEBUG_SYNC(s);
    return GSR_OK;
}

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
                                  unsigned accumulate, gsr_stream_t stream)
{
    return gsr_backward_preprocess_views_range(V, P, D, M, R, width, height, means3D, dc, shs, colors_precomp,
                                               opacities, scales, scale_modifier, rotations, cov3D_precomp,
                                               viewmatrices, projmatrices, campos, tan_fovx, tan_fovy, radii,
                                               geom_buffers, binning_buffers, has_invdepth, dL_dmean2D, dL_dcolor,
                                               dL_dopacity, dL_dmean3D, dL_dcov3D, dL_ddc, dL_dsh, dL_dscale, dL_drot,
                                               antialiasing, debug, accumulate, 0, P, stream);
}

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
                                        gsr_stream_t stream)
{
    if (V < 1 || V > MAX_VIEWS) return fail(GSR_ERR_INVALID, "V must be in [1, 16]");
    if (g_begin < 0 || g_end > P || g_begin > g_end) return fail(GSR_ERR_INVALID, "range outside [0, P)");
    if (accumulate & ~(unsigned)GSR_ACC_ALL) return fail(GSR_ERR_INVALID, "unknown accumulate bits");
    if (dc && !dL_ddc) return fail(GSR_ERR_INVALID, "dc given without dL_ddc");
    if (dc && colors_precomp)
        return fail(GSR_ERR_INVALID, "Please provide exactly one of either SHs or precomputed colors!");
    if (dc && M > 0 && (!shs || !dL_dsh)) return fail(GSR_ERR_INVALID, "dc given with M > 0 but shs/dL_dsh NULL");
    if (!R || !viewmatrices || !projmatrices || !campos || !tan_fovx || !tan_fovy || !geom_buffers ||
        !binning_buffers || !dL_dmean2D)
        return fail(GSR_ERR_INVALID, "null per-view array");
    hipStream_t s = (hipStream_t)stream;
    if (P <= 0) return GSR_OK;
    const GeomLayout g = geom_layout(P);

    PreprocessBwdViewsArgs A;
    PreprocessBwdArgs& p = A.a;
    p.P = P; p.D = D; p.M = dc ? M + 1 : M;
    p.means3D = means3D; p.radii = nullptr; p.shs = shs; p.dc = dc; p.dL_ddc = dc ? dL_ddc : nullptr;
    p.opacities = opacities; p.scales = scales; p.rotations = rotations; p.scale_modifier = scale_modifier;
    p.cov3D_precomp = cov3D_precomp;
    p.antialiasing = antialiasing;
    // a view rendered without an inverse-depth gradient has zero invdepth fields in its records:
    // subtracting their (zero) term leaves its gradients bit-identical
    p.has_invdepth = has_invdepth;
    p.W = width; p.H = height;
    p.dL_dconic = nullptr; p.dL_dinvdepth = nullptr;
    p.dL_dopacity = dL_dopacity; p.dL_dcolor = dL_dcolor;
    p.dL_dmean3D = dL_dmean3D; p.dL_dcov3D = dL_dcov3D; p.dL_dsh = (shs && M > 0) ? dL_dsh : nullptr;
    p.dL_dscale = dL_dscale; p.dL_drot = dL_drot;
    p.acc = accumulate;
    A.V = V;
    A.g_begin = g_begin;
    A.g_end = g_end;
    for (int v = 0; v < V; v++) {
        char* gb = geom_buffers[v];
        char* bb = binning_buffers[v];
        const int L = R[v];
        if (!gb || (L > 0 && !bb)) return fail(GSR_ERR_ALLOC, "null state buffer");
        if (!dL_dmean2D[v]) return fail(GSR_ERR_INVALID, "null per-view gradient");
        const BinLayout b = bin_layout(L);
        BwdView& bv = A.v[v];
        bv.view = viewmatrices[v];
        bv.proj = projmatrices[v];
        bv.campos = campos[v];
        bv.tan_fovx = tan_fovx[v];
        bv.tan_fovy = tan_fovy[v];
        bv.focal_y = height / (2.0f * tan_fovy[v]);
        bv.focal_x = width / (2.0f * tan_fovx[v]);
        bv.radii = (radii && radii[v]) ? radii[v] : at<int>(gb, g.off[GEOM_RADII]);
        bv.conic_opacity = at<float4>(gb, g.off[GEOM_CONIC_OPACITY]);
        bv.clamped = at<uint8_t>(gb, g.off[GEOM_CLAMPED]);
        bv.emit_start = at<uint32_t>(gb, g.off[GEOM_EMIT_START]);
        bv.tiles_touched = at<uint32_t>(gb, g.off[GEOM_TILES_TOUCHED]);
        bv.grad_inst = L > 0 ? at<float>(bb, b.off[BIN_GRAD_INST]) : nullptr;
        bv.valid = L > 0 ? at<uint32_t>(bb, b.off[BIN_VALID]) : nullptr;
        bv.rec_mask = at<uint32_t>(gb, g.off[GEOM_REC_MASK]);
        bv.dL_dmean2D = dL_dmean2D[v];
    }
    // BACKWARD::preprocess (rasterizer_impl.cu:423-449) of the whole batch: one pass over the Gaussians
    {
        ProfScope ps_(PK_PREPROCESS_BWD, s);
        HIP_TRY(launch_preprocess_bwd_views(A, s));
    }
    DEBUG_SYNC(s);
    return GSR_OK;
}

int gsr_backward_render_views(int V, int P, const int* R, const float* background, int width, int height,
                              char* const* geom_buffers, char* const* binning_buffers, char* const* image_buffers,
                              const float* const* dL_dpix, const float* const* dL_invdepths, bool debug,
                              gsr_stream_t stream)
{
    if (V < 1 || V > MAX_VIEWS) return fail(GSR_ERR_INVALID, "V must be in [1, 16]");
    if (!R || !geom_buffers || !binning_buffers || !image_buffers || !dL_dpix)
        return fail(GSR_ERR_INVALID, "null per-view array");
    const bool has_inv = dL_invdepths != nullptr;
    if (P <= 0) return GSR_OK;
    // every view's backward tile order (longest n_contrib first) in one launch
    OrderJob oj[MAX_VIEWS];
    int no = 0;
    const ImageLayout im = image_layout(width, height);
    const int T = (int)(((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X) * ((height + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y));
    for (int v = 0; v < V; v++) {
        if (!image_buffers[v]) return fail(GSR_ERR_ALLOC, "null state buffer");
        if (R[v] > 0)
            oj[no++] = {nullptr, at<uint32_t>(image_buffers[v], im.off[IMG_TILE_WORK]),
                        at<uint32_t>(image_buffers[v], im.off[IMG_TILE_ORDER])};
    }
    // BACKWARD::render of every view (its per-(tile, Gaussian) records), one launch per batch
    RenderBwdArgs ra[MAX_VIEWS];
    int nr = 0;
    for (int v = 0; v < V; v++) {
        if (!dL_dpix[v] || (has_inv && !dL_invdepths[v])) return fail(GSR_ERR_INVALID, "null per-view gradient");
        if (R[v] < 0) return fail(GSR_ERR_INVALID, "R must be >= 0");
        if (R[v] == 0) continue;
        if (!geom_buffers[v] || !binning_buffers[v]) return fail(GSR_ERR_ALLOC, "null state buffer");
        ra[nr++] = render_bwd_args(P, R[v], background, width, height, geom_buffers[v], binning_buffers[v],
                                   image_buffers[v], dL_dpix[v], has_inv ? dL_invdepths[v] : nullptr);
    }
    if (no) {
        ProfScope ps_(PK_TILE_ORDER, (hipStream_t)stream);
        HIP_TRY(launch_tile_order_batch(oj, no, T, (hipStream_t)stream));
    }
    if (nr) {
        ProfScope ps_(PK_RENDER_BWD, (hipStream_t)stream);  // valid[] was cleared by the forward
        HIP_TRY(launch_render_bwd_batch(ra, nr, T, (hipStream_t)stream));
    }
    DEBUG_SYNC((hipStream_t)stream);
    return GSR_OK;
}

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
                       gsr_stream_t stream)
{
    const int rc = gsr_backward_render_views(V, P, R, background, width, height, geom_buffers, binning_buffers,
                                             image_buffers, dL_dpix, dL_invdepths, debug, stream);
    if (rc || P <= 0) return rc;
    return gsr_backward_preprocess_views(V, P, D, M, R, width, height, means3D, dc, shs, colors_precomp, opacities,
                                         scales, scale_modifier, rotations, cov3D_precomp, viewmatrices,
                                         projmatrices, campos, tan_fovx, tan_fovy, radii, geom_buffers,
                                         binning_buffers, dL_invdepths != nullptr, dL_dmean2D, dL_dcolor,
                                         dL_dopacity, dL_dmean3D, dL_dcov3D, dL_ddc, dL_dsh, dL_dscale, dL_drot,
                                         antialiasing, debug, accumulate, stream);
}

// ---- the non-dc entry points: the reference's Rasterizer API (rasterizer.h:31-90) ----
int gsr_forward_geometry(char* geometry_buffer, char* image_buffer, int P, int D, int M, int width, int height,
                         const float* means3D, const float* shs, const float* colors_precomp,
                         const float* opacities, const float* scales, float scale_modifier,
                         const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                         const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                         bool prefiltered, bool antialiasing, int* radii, bool debug, gsr_stream_t stream,
                         int* num_rendered)
{
    return gsr_forward_geometry_dc(geometry_buffer, image_buffer, P, D, M, width, height, means3D, nullptr, shs,
                                   colors_precomp, opacities, scales, scale_modifier, rotations, cov3D_precomp,
                                   viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered, antialiasing,
                                   radii, debug, stream, num_rendered);
}

int gsr_forward(gsr_resize_fn geometryBuffer, void* geometry_ctx, gsr_resize_fn binningBuffer, void* binning_ctx,
                gsr_resize_fn imageBuffer, void* image_ctx, int P, int D, int M, const float* background, int width,
                int height, const float* means3D, const float* shs, const float* colors_precomp,
                const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                float tan_fovx, float tan_fovy, bool prefiltered, float* out_color, float* depth, bool antialiasing,
                int* radii, bool debug, gsr_stream_t stream, int* num_rendered)
{
    return gsr_forward_dc(geometryBuffer, geometry_ctx, binningBuffer, binning_ctx, imageBuffer, image_ctx, P, D, M,
                          background, width, height, means3D, nullptr, shs, colors_precomp, opacities, scales,
                          scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx,
                          tan_fovy, prefiltered, out_color, depth, antialiasing, radii, debug, stream, num_rendered);
}

int gsr_forward_prealloc(char* geometry_buffer, char* image_buffer, char* binning_buffer, size_t binning_capacity,
                         int P, int D, int M, const float* background, int width, int height, const float* means3D,
                         const float* shs, const float* colors_precomp, const float* opacities, const float* scales,
                         float scale_modifier, const float* rotations, const float* cov3D_precomp,
                         const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                         float tan_fovy, bool prefiltered, bool antialiasing, float* out_color, float* depth,
                         int* radii, bool debug, gsr_stream_t stream, int* num_rendered, int* rendered)
{
    return gsr_forward_prealloc_dc(geometry_buffer, image_buffer, binning_buffer, binning_capacity, P, D, M,
                                   background, width, height, means3D, nullptr, shs, colors_precomp, opacities,
                                   scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos,
                                   tan_fovx, tan_fovy, prefiltered, antialiasing, out_color, depth, radii, debug,
                                   stream, num_rendered, rendered);
}

int gsr_backward(int P, int D, int M, int R, const float* background, int width, int height, const float* means3D,
                 const float* shs, const float* colors_precomp, const float* opacities, const float* scales,
                 float scale_modifier, const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                 const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                 char* geom_buffer, char* binning_buffer, char* image_buffer, const float* dL_dpix,
                 const float* dL_invdepths, float* dL_dmean2D, float* dL_dconic, float* dL_dopacity, float* dL_dcolor,
                 float* dL_dinvdepth, float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale,
                 float* dL_drot, bool antialiasing, bool debug, gsr_stream_t stream)
{
    return gsr_backward_dc(P, D, M, R, background, width, height, means3D, nullptr, shs, colors_precomp, opacities,
                           scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx,
                           tan_fovy, radii, geom_buffer, binning_buffer, image_buffer, dL_dpix, dL_invdepths,
                           dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor, dL_dinvdepth, dL_dmean3D, dL_dcov3D, nullptr,
                           dL_dsh, dL_dscale, dL_drot, antialiasing, debug, stream);
}

// ---- sparse Adam (adam.hip) ----
int gsr_adam_update(float* param, const float* param_grad, float* exp_avg, float* exp_avg_sq, const bool* visible,
                    float lr, float b1, float b2, float eps, int N, int M, gsr_stream_t stream)
{
    if (N < 0 || M < 0) return fail(GSR_ERR_INVALID, "N and M must be >= 0");
    if ((size_t)N * M == 0) return GSR_OK;
    if ((size_t)N * M >= 0xFFFFFFF0ull) return fail(GSR_ERR_INVALID, "N*M must be < 2^32");
    if (!param || !param_grad || !exp_avg || !exp_avg_sq || !visible) return fail(GSR_ERR_INVALID, "null pointer");
    AdamArgs a;
    a.param = param; a.grad = param_grad; a.exp_avg = exp_avg; a.exp_avg_sq = exp_avg_sq;
    a.visible = reinterpret_cast<const uint8_t*>(visible);
    a.lr = lr; a.b1 = b1; a.b2 = b2; a.eps = eps; a.N = N; a.M = M;
    HIP_TRY(launch_adam_update(a, (hipStream_t)stream));
    return GSR_OK;
}

int gsr_adam_update_multi(int n_groups, float* const* params, const float* const* param_grads,
                          float* const* exp_avgs, float* const* exp_avg_sqs, const int* Ms, const float* lrs,
                          const float* epss, const bool* visible, float b1, float b2, int N, gsr_stream_t stream)
{
    if (n_groups < 0 || N < 0) return fail(GSR_ERR_INVALID, "n_groups and N must be >= 0");
    if (n_groups == 0 || N == 0) return GSR_OK;
    if (!params || !param_grads || !exp_avgs || !exp_avg_sqs || !Ms || !lrs || !epss || !visible)
        return fail(GSR_ERR_INVALID, "null pointer");
    std::vector<AdamArgs> g((size_t)n_groups);
    for (int i = 0; i < n_groups; i++) {
        if (Ms[i] < 0) return fail(GSR_ERR_INVALID, "M must be >= 0");
        if ((size_t)N * Ms[i] >= 0xFFFFFFF0ull) return fail(GSR_ERR_INVALID, "N*M must be < 2^32");
        if (Ms[i] > 0 && (!params[i] || !param_grads[i] || !exp_avgs[i] || !exp_avg_sqs[i]))
            return fail(GSR_ERR_INVALID, "null group pointer");
        AdamArgs& a = g[i];
        a.param = params[i]; a.grad = param_grads[i]; a.exp_avg = exp_avgs[i]; a.exp_avg_sq = exp_avg_sqs[i];
        a.visible = reinterpret_cast<const uint8_t*>(visible);
        a.lr = lrs[i]; a.b1 = b1; a.b2 = b2; a.eps = epss[i]; a.N = N; a.M = Ms[i];
    }
    HIP_TRY(launch_adam_update_multi(g.data(), n_groups, (hipStream_t)stream));
    return GSR_OK;
}

// ---- fused_ssim.h ----
int gsr_ssim_forward(int planes, int H, int W, float C1, float C2, const float* img1, const float* img2,
                     float* ssim_map, float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12, void* stream)
{
    if (planes < 0 || H < 0 || W < 0) return fail(GSR_ERR_INVALID, "negative image size");
    if ((size_t)planes * H * W == 0) return GSR_OK;
    if (!img1 || !img2 || !ssim_map) return fail(GSR_ERR_INVALID, "null pointer");
    const bool train = dm_dmu1 && dm_dsigma1_sq && dm_dsigma12;
    HIP_TRY(launch_ssim_fwd(planes, H, W, C1, C2, img1, img2, ssim_map, train ? dm_dmu1 : nullptr,
                            train ? dm_dsigma1_sq : nullptr, train ? dm_dsigma12 : nullptr, (hipStream_t)stream));
    return GSR_OK;
}

int gsr_ssim_backward(int planes, int H, int W, float C1, float C2, const float* img1, const float* img2,
                      const float* dL_dmap, const float* dm_dmu1, const float* dm_dsigma1_sq,
                      const float* dm_dsigma12, float* dL_dimg1, void* stream)
{
    (void)C1;
    (void)C2;  // folded into the forward's partial derivatives
    if (planes < 0 || H < 0 || W < 0) return fail(GSR_ERR_INVALID, "negative image size");
    if ((size_t)planes * H * W == 0) return GSR_OK;
    if (!img1 || !img2 || !dL_dmap || !dm_dmu1 || !dm_dsigma1_sq || !dm_dsigma12 || !dL_dimg1)
        return fail(GSR_ERR_INVALID, "null pointer");
    HIP_TRY(launch_ssim_bwd(planes, H, W, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12, dL_dimg1,
                            (hipStream_t)stream));
    return GSR_OK;
}

// ---- simple_knn.h ----
size_t gsr_knn_workspace_size(int P) { return knn_workspace_bytes(P); }

int gsr_knn_dist2(int P, const float* points, float* dist2_out, void* workspace, void* stream)
{
    if (P < 0) return fail(GSR_ERR_INVALID, "P must be >= 0");
    if (P == 0) return GSR_OK;
    if (!points || !dist2_out || !workspace) return fail(GSR_ERR_INVALID, "null pointer");
    uint32_t* h;
    int rc = pinned(0, &h);
    if (rc) return rc;
    HIP_TRY(knn_dist2(P, points, dist2_out, static_cast<char*>(workspace), h + 8, (hipStream_t)stream));
    return GSR_OK;
}

int gsr_debug_sorted_keys(const char* geometry_buffer, const char* binning_buffer, const char* image_buffer, int P,
                          int num_rendered, int width, int height, uint64_t* keys_out, uint32_t* vals_out,
                          uint32_t* ranges_out, gsr_stream_t stream)
{
    hipStream_t s = (hipStream_t)stream;
    const GeomLayout g = geom_layout(P);
    const BinLayout b = bin_layout(num_rendered);
    const ImageLayout im = image_layout(width, height);
    const uint32_t gx = (uint32_t)((width + GSR_BLOCK_X - 1) / GSR_BLOCK_X);
    const uint32_t gy = (uint32_t)((height + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y);
    if (num_rendered > 0) {
        const uint32_t* point_list = at<uint32_t>(binning_buffer, b.off[BIN_POINT_LIST]);
        if (keys_out && use_tile_diff(gx, gy))  // no tile ids were written: each tile's range carries its id
            HIP_TRY(launch_debug_keys_from_ranges((int)(gx * gy), at<uint2>(image_buffer, im.off[IMG_RANGES]),
                                                  point_list, at<uint32_t>(geometry_buffer, g.off[GEOM_DKEY]),
                                                  keys_out, s));
        else if (keys_out)
            HIP_TRY(launch_debug_keys(num_rendered, at<uint32_t>(binning_buffer, b.off[BIN_SORTED_TILES]), point_list,
                                      at<uint32_t>(geometry_buffer, g.off[GEOM_DKEY]), keys_out, s));
        if (vals_out)
            HIP_TRY(hipMemcpyAsync(vals_out, point_list, 4 * (size_t)num_rendered, hipMemcpyDeviceToDevice, s));
    }
    if (ranges_out)
        HIP_TRY(hipMemcpyAsync(ranges_out, image_buffer + im.off[IMG_RANGES], 8 * (size_t)gx * gy,
                               hipMemcpyDeviceToDevice, s));
    return GSR_OK;
}

int gsr_debug_depth_wide(void) { return depth_force_wide() ? 1 : 0; }

int gsr_debug_set_depth_wide(int on)
{
    set_depth_force_wide(on != 0);
    return GSR_OK;
}

size_t gsr_debug_depth_sort_workspace_size(int n)
{
    const size_t q = align_up(4 * (size_t)(n > 0 ? n : 0), 256);
    return 4 * q + align_up(radix_status_bytes(n, 4), 256);
}

int gsr_debug_depth_sort(const uint32_t* keys, int n, uint32_t* out_ids, char* workspace, gsr_stream_t stream)
{
    if (n < 0 || (n > 0 && (!keys || !out_ids || !workspace))) return fail(GSR_ERR_INVALID, "bad depth-sort arguments");
    if (n == 0) return GSR_OK;
    hipStream_t s = (hipStream_t)stream;
    const size_t q = align_up(4 * (size_t)n, 256);
    uint32_t* k0 = reinterpret_cast<uint32_t*>(workspace);
    uint32_t* v0 = reinterpret_cast<uint32_t*>(workspace + q);
    uint32_t* k1 = reinterpret_cast<uint32_t*>(workspace + 2 * q);
    uint32_t* v1 = reinterpret_cast<uint32_t*>(workspace + 3 * q);
    // the forward's call (forward_geometry_sort) without the rect gather
    HIP_TRY(radix_sort(n, DEPTH_BITS, keys, nullptr, k0, v0, k1, v1, out_ids, nullptr, nullptr, workspace + 4 * q, s));
    if (!depth_force_wide()) {  // three passes: the range word says whether they sufficed (else four, as the forward)
        uint32_t rw[2] = {0u, 1u};
        HIP_TRY(hipMemcpyAsync(rw, workspace + 4 * q + radix_range_offset(n), 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (!rw[1]) {
            const SortJob j = {n, keys, nullptr, k0, v0, k1, v1, out_ids, nullptr, nullptr, workspace + 4 * q};
            HIP_TRY(radix_sort_batch(&j, 1, DEPTH_BITS, s, 0, SORT_DEPTH, /*four_pass=*/true));
        }
    }
    return GSR_OK;
}

}  // extern "C"
