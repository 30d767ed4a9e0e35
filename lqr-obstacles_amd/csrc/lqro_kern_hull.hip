// lqro_kern_hull.hip — the hull kernels (k_hull, k_hull_big; lqro_hull.hpp; k_lhull;
// lqro_lhull.hpp)
// and their launch functions (lqro_kern.hpp).
#define LQRO_HULL_TU 1
#include <hip/hip_runtime.h>

#include "lqro_hull.hpp"
#include "lqro_lhull.hpp"
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

}  // namespace lqro
