// lqro_pair_inst.hip — one instantiation set of the pair kernels, compiled
// once per (state width, record mode): -DLQRO_INST_X=16|12 -DLQRO_INST_RECS=0|1.
// Each object holds k_pair (row, hot-shared, hot-per-agent launches) and
// k_side for that combination; lqro_runtime.hip calls them through the
// launch functions below.  Splitting the instantiations over four objects
// lets them compile in parallel (the hull and pair bodies are large).
#ifndef LQRO_INST_X
#error "compile with -DLQRO_INST_X=16|12 -DLQRO_INST_RECS=0|1"
#endif
#define LQRO_PAIR_TU 1   // the shared non-template kernels live in lqro_runtime.hip
#include <hip/hip_runtime.h>

#include "lqro_pair_launch.hpp"
#include "lqro_hull.hpp"
#include "lqro_qhull3.hpp"

namespace lqro {

// k_side: the side stream's hull workers (the hot pairs' hulls, topology in
// LDS as k_hull), which turn into k_pair row workers once the hull queue is
// drained, so the side CUs never idle while the sweep goes on.  The pair
// tables and per-wave regions reuse the hull's LDS (host checks the fit).
template <int X, bool RECS>
__global__ void __launch_bounds__(HULL_CTHREADS) k_side(HullArgs A, PairArgs P) {
  __shared__ HullLdsC<HULL_CWAVES> L;
  __shared__ HullMemC M;
  hull_body_mw<HULL_CWAVES>(A, M, L);
  __syncthreads();
  if (P.nrows > 0) pair_block<X, RECS, kRowLaunch>(P, reinterpret_cast<double*>(&M));
}

// k_qside: the side stream's k_qhull workers (the hot pairs' builds in
// Qhull's order, 3 waves a CU), which turn into k_pair row workers once the
// hull queue is drained: a CU whose build is done sweeps rows (finer row
// units keep the 3-wave workers' last unit short) instead of idling until
// the slowest build ends.  The pair tables and per-wave regions reuse the
// build's LDS (the host checks the fit and sets P.max_waves).
template <int X, bool RECS>
__global__ void __launch_bounds__(192) k_qside(HullArgs A, PairArgs P) {
  __shared__ Q3L L;
  q3_body(A, L);
  __syncthreads();
  if (P.nrows > 0) pair_block<X, RECS, kRowLaunch>(P, reinterpret_cast<double*>(&L));
}

template <int X, bool R>
void launch_qside_t(dim3 grid, hipStream_t s, const HullArgs& H, const PairArgs& P) {
  hipLaunchKernelGGL((k_qside<X, R>), grid, dim3(192), 0, s, H, P);
}

template <int X, bool R>
void launch_pair_t(dim3 grid, dim3 block, size_t lds, hipStream_t s, const PairArgs& P) {
  const int h = P.hot_only == 0 ? kRowLaunch : (P.per_agent ? kHotPerAgent : kHotShared);
  if (h == kRowLaunch) hipLaunchKernelGGL((k_pair<X, R, kRowLaunch>), grid, block, lds, s, P);
  else if (h == kHotShared) hipLaunchKernelGGL((k_pair<X, R, kHotShared>), grid, block, lds, s, P);
  else hipLaunchKernelGGL((k_pair<X, R, kHotPerAgent>), grid, block, lds, s, P);
}

template <int X, bool R>
void launch_side_t(dim3 grid, dim3 block, hipStream_t s, const HullArgs& H, const PairArgs& P) {
  hipLaunchKernelGGL((k_side<X, R>), grid, block, 0, s, H, P);
}

template <int X, bool R>
bool pair_set_lds_t(int bytes) {
  const void* ks[3] = {(const void*)k_pair<X, R, kRowLaunch>, (const void*)k_pair<X, R, kHotShared>,
                       (const void*)k_pair<X, R, kHotPerAgent>};
  for (const void* k : ks)
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) return false;
  return true;
}

template void launch_pair_t<LQRO_INST_X, (bool)LQRO_INST_RECS>(dim3, dim3, size_t, hipStream_t, const PairArgs&);
template void launch_side_t<LQRO_INST_X, (bool)LQRO_INST_RECS>(dim3, dim3, hipStream_t, const HullArgs&,
                                                               const PairArgs&);
template bool pair_set_lds_t<LQRO_INST_X, (bool)LQRO_INST_RECS>(int);
template void launch_qside_t<LQRO_INST_X, (bool)LQRO_INST_RECS>(dim3, hipStream_t, const HullArgs&, const PairArgs&);

}  // namespace lqro
