// lqro_pair_launch.hpp — the pair kernels' launch functions, instantiated in
// lqro_pair_inst.hip (one object per state width and record mode) and called
// by lqro_runtime.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "lqro_pair.hpp"

namespace lqro {

struct HullArgs;

// k_pair for P's launch kind (row / hot-shared / hot-per-agent)
template <int X, bool R>
void launch_pair_t(dim3 grid, dim3 block, size_t lds, hipStream_t s, const PairArgs& P);
// k_side: hot hulls, then rows
template <int X, bool R>
void launch_side_t(dim3 grid, dim3 block, hipStream_t s, const HullArgs& H, const PairArgs& P);
// k_qside: hot builds in Qhull's order, then rows
template <int X, bool R>
void launch_qside_t(dim3 grid, hipStream_t s, const HullArgs& H, const PairArgs& P);
// dynamic LDS limit of the three k_pair launch kinds
template <int X, bool R>
bool pair_set_lds_t(int bytes);

extern template void launch_pair_t<16, false>(dim3, dim3, size_t, hipStream_t, const PairArgs&);
extern template void launch_pair_t<16, true>(dim3, dim3, size_t, hipStream_t, const PairArgs&);
extern template void launch_pair_t<12, false>(dim3, dim3, size_t, hipStream_t, const PairArgs&);
extern template void launch_pair_t<12, true>(dim3, dim3, size_t, hipStream_t, const PairArgs&);
extern template void launch_side_t<16, false>(dim3, dim3, hipStream_t, const HullArgs&, const PairArgs&);
extern template void launch_side_t<16, true>(dim3, dim3, hipStream_t, const HullArgs&, const PairArgs&);
extern template void launch_side_t<12, false>(dim3, dim3, hipStream_t, const HullArgs&, const PairArgs&);
extern template void launch_side_t<12, true>(dim3, dim3, hipStream_t, const HullArgs&, const PairArgs&);
extern template void launch_qside_t<16, false>(dim3, hipStream_t, const HullArgs&, const PairArgs&);
extern template void launch_qside_t<16, true>(dim3, hipStream_t, const HullArgs&, const PairArgs&);
extern template void launch_qside_t<12, false>(dim3, hipStream_t, const HullArgs&, const PairArgs&);
extern template void launch_qside_t<12, true>(dim3, hipStream_t, const HullArgs&, const PairArgs&);
extern template bool pair_set_lds_t<16, false>(int);
extern template bool pair_set_lds_t<16, true>(int);
extern template bool pair_set_lds_t<12, false>(int);
extern template bool pair_set_lds_t<12, true>(int);

}  // namespace lqro
