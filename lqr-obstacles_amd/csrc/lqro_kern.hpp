// lqro_kern.hpp — launch functions of the kernels compiled in their own
// objects (lqro_kern_hull.hip, lqro_kern_synth.hip, lqro_kern_dyn.hip), so
// that liblqro.so's large kernels compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/lqro.h"

namespace lqro {
struct HullArgs;
// k_hull: grid x 8 waves, topology in LDS
void launch_hull(dim3 grid, hipStream_t s, const HullArgs& A);
// k_hull_big: one inserting wave, topology in global memory
void launch_hull_big(dim3 grid, hipStream_t s, const HullArgs& A);
// k_lhull: grid x 4 waves, one inside-hull pair at a time from a local hull
// around vrel; the pairs it cannot decide go to A.lqueue (for k_hull)
void launch_lhull(dim3 grid, hipStream_t s, const HullArgs& A);
// k_qhull (LQRO_FLAG_QHULL_ORDER): grid x 1 wave, one inside-hull pair per
// wave (one wave per CU: its LDS) with Qhull's build order (lqro_qhull3.hpp); A.qscratch holds
// A.block_base + grid workers of qhull_worker_bytes(H*NP) bytes.  Pairs beyond
// its per-insertion caps go to A.rqueue for k_qhull_big (lqro_qhull.hpp),
// which with A.big_main takes the main queue instead.
void launch_qhull(dim3 grid, hipStream_t s, const HullArgs& A);
void launch_qhull_big(dim3 grid, hipStream_t s, const HullArgs& A);
size_t qhull_lds_doubles();   // k_qhull's LDS block (k_qside sweeps rows in it)
size_t qhull_worker_bytes(int hnp);
// k_stale: the facet-0 pairs' loop-carried normals, then the carry out
void launch_stale(hipStream_t s, float* planes, const double* qnrm, const int* list, const int* count, int cap,
                  const double* x, int X, int npr, int row_begin, int row_stride, double* carry,
                  lqro_pair_record* recs, long nslots);
void launch_rowlast(hipStream_t s, const float* planes, const double* qnrm, int npr, int nrows, int row_begin,
                    int row_stride, double* rowtab);
void launch_stale_rows(hipStream_t s, float* planes, const double* qnrm, const int* list, const int* count, int cap,
                       const double* x, int X, int npr, int row_begin, int row_stride, const double* rowtab, int N,
                       double* carry, lqro_pair_record* recs, long nslots);
// controlMatrices for n models into out (stride X*X + 12X + 25 doubles):
// k_synthw (one wave per agent) or, lane = true, k_synth (one agent per lane)
void launch_synth(int x_dim, bool lane, const lqro_model* d_models, int n, double* d_out);
// the agent loop LQRO:1437-1446: k_dynw or, lane = true, k_dyn
void launch_dyn(bool lane, const lqro_model* models, int n_models, int n, int per_agent, const lqro_agents& A,
                hipStream_t s);
}  // namespace lqro
