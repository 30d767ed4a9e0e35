// lqro_kern_synth.hip — the batched gain-synthesis kernels (controlMatrices,
// LQRObstacles.cpp:520-582) and their launch function (lqro_kern.hpp).
#include <hip/hip_runtime.h>

#include "lqro_kern.hpp"
#include "lqro_synth.hpp"
#include "lqro_synthw.hpp"

namespace lqro {

template <int X>
__global__ void __launch_bounds__(64) k_synth(const lqro_model* models, int n, double* out) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= n) return;
  constexpr int S = X * X + 12 * X + 25;
  double* o = out + (size_t)a * S;
  double* p[8];
  p[0] = o;
  p[1] = p[0] + X * X; p[2] = p[1] + X * 4; p[3] = p[2] + X; p[4] = p[3] + 4 * X; p[5] = p[4] + 12;
  p[6] = p[5] + 4; p[7] = p[6] + 3 * X;
  synth::gains_x<X>(models + a, p[0], p[1], p[2], p[3], p[4], p[6], p[7], p[5]);
}

// The same synthesis with one wave per agent (lqro_synthw.hpp): the agent's
// matrices in LDS, products and sums over the lanes in the reference's order.
// The default; LQRO_SYNTH_LANE=1 selects k_synth.
template <int X>
__global__ void __launch_bounds__(64) k_synthw(const lqro_model* models, int n, double* out) {
  extern __shared__ double sw[];
  const int a = blockIdx.x;
  if (a >= n) return;
  constexpr int S = X * X + 12 * X + 25;
  double* o = out + (size_t)a * S;
  double* p[8];
  p[0] = o;
  p[1] = p[0] + X * X; p[2] = p[1] + X * 4; p[3] = p[2] + X; p[4] = p[3] + 4 * X; p[5] = p[4] + 12;
  p[6] = p[5] + 4; p[7] = p[6] + 3 * X;
  synthw::gains<X>(models + a, p[0], p[1], p[2], p[3], p[4], p[6], p[7], p[5], sw, threadIdx.x);
}

void launch_synth(int x_dim, bool lane, const lqro_model* d_m, int n, double* d_out) {
  if (lane && x_dim == 16)
    hipLaunchKernelGGL(k_synth<16>, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, 0, d_m, n, d_out);
  else if (lane)
    hipLaunchKernelGGL(k_synth<12>, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, 0, d_m, n, d_out);
  else if (x_dim == 16)
    hipLaunchKernelGGL(k_synthw<16>, dim3((unsigned)n), dim3(64), sizeof(double) * synthw::Lay<16>::Total, 0, d_m,
                       n, d_out);
  else
    hipLaunchKernelGGL(k_synthw<12>, dim3((unsigned)n), dim3(64), sizeof(double) * synthw::Lay<12>::Total, 0, d_m,
                       n, d_out);
}

}  // namespace lqro
