// lqro_kern_dyn.hip — the per-agent dynamics / estimation kernels (the agent
// loop LQRObstacles.cpp:1437-1446) and their launch function (lqro_kern.hpp).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "lqro_dyn.hpp"
#include "lqro_dynw.hpp"
#include "lqro_kern.hpp"

namespace lqro {

// ---- the per-agent step after the pair loop (LQRO:1437-1446) -------------
// One agent per lane: the step is a chain of 16x16 products, exponentials and
// a Jacobi sweep with data-dependent control flow (lqro_dyn.hpp), fp64,
// ~10 MFLOP per agent, latency bound on per-lane scratch.
__global__ void __launch_bounds__(64) k_dyn(const lqro_model* models, int n_models, int n, int per_agent,
                                            lqro_agents A) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= n) return;
  const size_t g = per_agent ? (size_t)a : 0;
  dyn::AgentParams p;
  p.model = models + (n_models > 1 ? a : 0);
  p.L = A.L + g * dyn::kU * dyn::kX;
  p.E = A.E + g * dyn::kU * dyn::kV;
  p.l = A.l + g * dyn::kU;
  p.Lh = A.Lh + g * dyn::kV * dyn::kX;
  p.Eh = A.Eh + g * dyn::kV * dyn::kV;
  p.u_goal = A.u_goal + (size_t)a * dyn::kU;
  p.p_goal = A.p_goal + (size_t)a * 3;
  p.M = A.M;
  p.Nz = A.N;
  p.normals = A.normals + (size_t)a * dyn::kNormals;
  p.keyframe = A.keyframes ? A.keyframes + (size_t)a * 8 : nullptr;
  p.time = A.time;
  dyn::agent_step(p, A.x + (size_t)a * dyn::kX, A.rot + (size_t)a * 9, A.x_true + (size_t)a * dyn::kX,
                  A.rot_true + (size_t)a * 9, A.P + (size_t)a * dyn::kX * dyn::kX, A.vgoal + (size_t)a * 3,
                  A.u ? A.u + (size_t)a * dyn::kU : nullptr);
}

// The same step with one wave per agent (lqro_dynw.hpp): the agent's 16x16
// matrices in LDS, the products, exponentials, solves and Jacobi sweep over
// the lanes.  The default; LQRO_DYN_LANE=1 selects k_dyn.
__global__ void __launch_bounds__(64) k_dynw(const lqro_model* models, int n_models, int n, int per_agent,
                                             lqro_agents A, unsigned long long* prof) {
  __shared__ double w[dynw::kWaveDoubles];
  const int a = blockIdx.x;
  if (a >= n) return;
  const int lane = threadIdx.x;
  const size_t g = per_agent ? (size_t)a : 0;
  dyn::AgentParams p;
  p.model = models + (n_models > 1 ? a : 0);
  p.L = A.L + g * dyn::kU * dyn::kX;
  p.E = A.E + g * dyn::kU * dyn::kV;
  p.l = A.l + g * dyn::kU;
  p.Lh = A.Lh + g * dyn::kV * dyn::kX;
  p.Eh = A.Eh + g * dyn::kV * dyn::kV;
  p.u_goal = A.u_goal + (size_t)a * dyn::kU;
  p.p_goal = A.p_goal + (size_t)a * 3;
  p.M = A.M;
  p.Nz = A.N;
  p.normals = A.normals + (size_t)a * dyn::kNormals;
  p.keyframe = A.keyframes ? A.keyframes + (size_t)a * 8 : nullptr;
  p.time = A.time;
  dynw::agent_step(p, A.x + (size_t)a * dyn::kX, A.rot + (size_t)a * 9, A.x_true + (size_t)a * dyn::kX,
                   A.rot_true + (size_t)a * 9, A.P + (size_t)a * dyn::kX * dyn::kX, A.vgoal + (size_t)a * 3,
                   A.u ? A.u + (size_t)a * dyn::kU : nullptr, w, lane, prof);
}

// LQRO_DYN_PROFILE=1: k_dynw's phases (lqro_dynw.hpp DynProf) into a device
// buffer per device (the current one at each launch), read by
// lqro_debug_dyn_profile for the current device (not in lqro.h;
// scripts/dyn_prof.py)
constexpr int kDynProfDevices = 64;
static unsigned long long* g_dprof[kDynProfDevices] = {nullptr};

static unsigned long long** dyn_prof_slot() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kDynProfDevices) return nullptr;
  return &g_dprof[dev];
}

extern "C" int lqro_debug_dyn_profile(unsigned long long* out32, int reset) {
  if (!out32) return -1;
  unsigned long long** slot = dyn_prof_slot();
  if (!slot || !*slot) { for (int k = 0; k < 32; ++k) out32[k] = 0; return 0; }
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  if (hipMemcpy(out32, *slot, sizeof(unsigned long long) * 32, hipMemcpyDeviceToHost) != hipSuccess) return -2;
  if (reset && hipMemset(*slot, 0, sizeof(unsigned long long) * 32) != hipSuccess) return -2;
  return 0;
}

void launch_dyn(bool lane, const lqro_model* models, int n_models, int n, int per_agent, const lqro_agents& A,
                hipStream_t s) {
  if (lane)
    hipLaunchKernelGGL(k_dyn, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, models, n_models, n, per_agent, A);
  else {
    static const int prof_on = getenv("LQRO_DYN_PROFILE") ? atoi(getenv("LQRO_DYN_PROFILE")) : 0;
    unsigned long long* prof = nullptr;
    if (prof_on) {   // (the launching device's own buffer)
      unsigned long long** slot = dyn_prof_slot();
      if (slot && !*slot && hipMalloc(slot, sizeof(unsigned long long) * 32) == hipSuccess)
        (void)hipMemset(*slot, 0, sizeof(unsigned long long) * 32);
      if (slot) prof = *slot;
    }
    hipLaunchKernelGGL(k_dynw, dim3((unsigned)n), dim3(64), 0, s, models, n_models, n, per_agent, A, prof);
  }
}

}  // namespace lqro
