/*
 * simple_knn.h -- C ABI of the MI355X-native replacement for the reference's
 * `simple_knn._C.distCUDA2` (submodule simple-knn, gitlab.inria.fr/bkerbl/simple-knn,
 * un-vendored in the reference: submodules/simple-knn is empty; its one call site is
 * scene/gaussian_model.py:21,159-160, which initialises every Gaussian's scale from
 *   dist2 = clamp_min(distCUDA2(points), 1e-7); scales = log(sqrt(dist2)) (x3)).
 *
 * distCUDA2(points[P,3]) -> dist2[P]: for each point, the mean of the squared Euclidean
 * distances to its 3 nearest OTHER points (positions in the point list; a duplicate
 * position at another index counts, at distance 0).  simple-knn's published algorithm
 * (Morton-sorted boxes of 1024 points + box pruning) is an exact 3-NN search, so the
 * result is fixed by the definition; the reference's combination
 * (best0 + best1 + best2) / 3 with best* ascending and FLT_MAX for missing neighbours
 * (P < 4) is kept.
 *
 * Same conventions as gsr.h: device pointers, explicit stream, int status +
 * gsr_last_error(), nothing throws.  Lives in libgsr_hip.so.
 */
#ifndef SIMPLE_KNN_H_INCLUDED
#define SIMPLE_KNN_H_INCLUDED

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Device scratch (bytes) gsr_knn_dist2 needs for P points. */
size_t gsr_knn_workspace_size(int P);

/* dist2_out[i] = mean squared distance of points[i] to its 3 nearest other points.
 * points: float32 [P,3] device, dist2_out: float32 [P] device, workspace: at least
 * gsr_knn_workspace_size(P) bytes of device memory.  Synchronises the stream once
 * (the grid is sized from the point bounds on the host). */
int gsr_knn_dist2(int P, const float* points, float* dist2_out, void* workspace, void* stream);

#ifdef __cplusplus
}
#endif

#endif
