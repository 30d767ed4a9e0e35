// lqro_kern_hull.hip — the hull kernels (k_hull, k_hull_big; lqro_hull.hpp; k_lhull;
// lqro_lhull.hpp; k_qhull: lqro_qhull3.hpp; k_qhull_big, k_stale: lqro_qhull.hpp)
// and their launch functions (lqro_kern.hpp).
#define LQRO_HULL_TU 1
#include <hip/hip_runtime.h>

#include "lqro_hull.hpp"
#include "lqro_lhull.hpp"
#include "lqro_qhull.hpp"
#include "lqro_qhull3.hpp"
#include "lqro_kern.hpp"

namespace lqro {

void launch_hull(dim3 grid, hipStream_t s, const HullArgs& A) {
  hipLaunchKernelGGL(k_hull, grid, dim3(HULL_CTHREADS), 0, s, A);
}

void launch_hull_big(dim3 grid, hipStream_t s, const HullArgs& A) {
  hipLaunchKernelGGL(k_hull_big, grid, dim3(HULL_THREADS), 0, s, A);
}

void launch_lhull(dim3 grid, hipStream_t s, const HullArgs& A) {
  hipLaunchKernelGGL(k_lhull, grid, dim3(LH_THREADS), 0, s, A);
}

// (the LDS block is k_qhull's or, for a build past its caps rebuilt in place,
// k_qhull_big's: q3_big_inline)
union Q3U {
  Q3L q3;
  QhL qh;
};
static_assert(sizeof(Q3U) == sizeof(Q3L), "k_qhull_big's LDS fits in k_qhull's");

// BIG: a build past the caps is rebuilt in place (q3_big_inline).  A kernel of
// its own: the rebuild's code in the same kernel costs the common path its
// registers (C3 step 19.7 -> 20.1 ms), so it runs only where builds reach the
// caps (the runtime's choice, HullArgs::big_inline)
template <bool BIG>
__global__ void __launch_bounds__(64 * Q3_WAVES) k_qhull(HullArgs A) {
  __shared__ Q3U U;
  q3_body(A, U.q3, BIG ? &U.qh : nullptr);
}

// the pairs k_qhull's caps turned away (the retry queue), or with
// A.big_main every pair of the main queue
__global__ void __launch_bounds__(64) k_qhull_big(HullArgs A) {
  __shared__ QhL L;
  qh_body(A, L, !A.big_main);
}

void launch_qhull(dim3 grid, hipStream_t s, const HullArgs& A) {
  // wave 0 builds, wave 1 speculates the next insertion, wave 2 prefetches its
  // partition sequence, waves 1-3 locate a long sequence's chunks
  if (A.big_inline) hipLaunchKernelGGL(k_qhull<true>, grid, dim3(64 * Q3_WAVES), 0, s, A);
  else hipLaunchKernelGGL(k_qhull<false>, grid, dim3(64 * Q3_WAVES), 0, s, A);
}

void launch_qhull_big(dim3 grid, hipStream_t s, const HullArgs& A) {
  hipLaunchKernelGGL(k_qhull_big, grid, dim3(64), 0, s, A);
}

size_t qhull_lds_doubles() { return sizeof(Q3L) / 8; }

size_t qhull_worker_bytes(int hnp) {
  const size_t a = qh_worker_bytes(hnp), b = q3_worker_bytes(hnp);
  return (a > b ? a : b) + QW_TAG_BYTES;   // (+ the owner tag, qw_owner)
}

void launch_stale(hipStream_t s, float* planes, const double* qnrm, const int* list, const int* count, int cap,
                  const double* x, int X, int npr, int row_begin, int row_stride, double* carry,
                  lqro_pair_record* recs, long nslots) {
  hipLaunchKernelGGL(k_stale, dim3(16), dim3(64), 0, s, planes, qnrm, list, count, cap, x, X, npr, row_begin,
                     row_stride, carry, recs, nslots);
}

void launch_rowlast(hipStream_t s, const float* planes, const double* qnrm, int npr, int nrows, int row_begin,
                    int row_stride, double* rowtab) {
  hipLaunchKernelGGL(k_rowlast, dim3((unsigned)std::min(std::max(nrows, 1), 4096)), dim3(64), 0, s, planes, qnrm, npr,
                     nrows, row_begin, row_stride, rowtab);
}

void launch_stale_rows(hipStream_t s, float* planes, const double* qnrm, const int* list, const int* count, int cap,
                       const double* x, int X, int npr, int row_begin, int row_stride, const double* rowtab, int N,
                       double* carry, lqro_pair_record* recs, long nslots) {
  (void)nslots;
  hipLaunchKernelGGL(k_stale_rows, dim3(16), dim3(64), 0, s, planes, qnrm, list, count, cap, x, X, npr, row_begin,
                     row_stride, rowtab, N, carry, recs);
}

}  // namespace lqro
