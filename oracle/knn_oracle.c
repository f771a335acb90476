/*
 * knn_oracle.c -- CPU restatement of simple-knn's distCUDA2 (TEST INFRASTRUCTURE ONLY:
 * loaded by tests/ and bench_knn.py's cpu_baseline leg, never by the product).
 *
 * simple-knn (gitlab.inria.fr/bkerbl/simple-knn) is an un-vendored submodule of the
 * reference (submodules/simple-knn is empty; .gitmodules pins no commit), so this restates
 * its published definition, anchored on its only call site, scene/gaussian_model.py:159-160:
 * for each point i, best[0..2] = the three smallest squared distances to points j != i
 * (updateKBest<3>: ascending insertion, initial FLT_MAX), d = dx*dx + dy*dy + dz*dz as nvcc
 * contracts it (fma(dz, dz, fma(dy, dy, dx*dx))), dist2[i] = (best[0] + best[1] + best[2]) / 3.
 * simple-knn's Morton boxes only prune the search; an exact brute force gives the same three
 * distances.  O(P^2) with OpenMP: for test sizes (P <= ~50k).  Parity of the HIP grid search
 * against this restatement is bit-exact; against simple-knn itself it is unpinned (no golden
 * vectors exist in the reference).
 */
#include <float.h>
#include <math.h>

static inline void update3(float* b, float d)
{
    for (int j = 0; j < 3; j++) {
        if (b[j] > d) {
            const float t = b[j];
            b[j] = d;
            d = t;
        }
    }
}

void gsr_oracle_knn_dist2(int P, const float* pts, float* dist2, int nthreads)
{
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads > 0 ? nthreads : 1)
    for (int i = 0; i < P; i++) {
        const float qx = pts[3 * i], qy = pts[3 * i + 1], qz = pts[3 * i + 2];
        float b[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
        for (int j = 0; j < P; j++) {
            if (j == i) continue;
            const float dx = pts[3 * j] - qx, dy = pts[3 * j + 1] - qy, dz = pts[3 * j + 2] - qz;
            update3(b, fmaf(dz, dz, fmaf(dy, dy, dx * dx)));
        }
        dist2[i] = (b[0] + b[1] + b[2]) / 3.0f;
    }
}
