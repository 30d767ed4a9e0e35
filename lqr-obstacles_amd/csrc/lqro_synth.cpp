// lqro_synth.cpp — setup-time host helpers of liblqro.so: the model defaults
// (setup(), LQRObstacles.cpp:169-189, 1275-1286, 559-561) and createSpheres
// (:735-750), and the reference's noise stream (normal(), :334-350).  The gain synthesis itself (controlMatrices) is shared by the
// host and the device: lqro_synth.hpp, entry points in lqro_runtime.hip.
#include <cmath>

#include "../../include/lqro.h"

extern "C" void lqro_model_default(lqro_model* m) {
  m->dt = 1.0 / 30.0;
  m->gravity = 9.80665;
  m->mass = 0.500;
  m->inertia = 0.1;
  m->moment_const = 1.5e-9 / 6.11e-8;
  m->thrust_latency = 40.0;
  m->length = 0.3429 / 2;
  m->j_step = 0.0009765625;
  m->qv = 100;
  m->qp = 0.1;
  m->r = 5;
  m->pos_weight = 0.05;
}

extern "C" int lqro_sphere(int32_t np, double xy_radius, double z_radius, double* out) {
  if (np <= 0 || !out) return LQRO_E_ARG;
  double dlong = M_PI * (3.0 - std::sqrt(5.0));
  double dz = 2.0 / np;
  double lon = 0;
  double z = 1.0 - dz / 2.0;
  for (int i = 0; i < np; i++) {
    out[3 * i + 0] = 2 * xy_radius * std::cos(lon) * std::sqrt(1 - z * z);
    out[3 * i + 1] = 2 * xy_radius * std::sin(lon) * std::sqrt(1 - z * z);
    out[3 * i + 2] = 2 * z_radius * z;
    z -= dz;
    lon += dlong;
  }
  return LQRO_OK;
}

// MSVC rand(): seed = seed*214013 + 2531011, (seed >> 16) & 0x7fff (RAND_MAX 32767)
static int msvc_rand(uint32_t* seed) {
  *seed = *seed * 214013u + 2531011u;
  return (int)((*seed >> 16) & 0x7fff);
}

// random() (LQRO:334-337); the two rand() calls are taken left to right
static double ref_uniform(uint32_t* seed) {
  const int a = msvc_rand(seed);
  const int b = msvc_rand(seed);
  return (double)(a * (32767 + 1) + b) / (32767 * (32767 + 2));
}

extern "C" int lqro_normals(uint32_t* seed, int64_t count, double* out) {
  if (!seed || count < 0 || (count > 0 && !out)) return LQRO_E_ARG;
  for (int64_t k = 0; k < count; ++k) {   // normal() (LQRO:340-350)
    double u = 0, v = 0, s = 0;
    while (s == 0 || s > 1) {
      u = 2 * ref_uniform(seed) - 1;
      v = 2 * ref_uniform(seed) - 1;
      s = u * u + v * v;
    }
    out[k] = u * std::sqrt(-2 * std::log(s) / s);
  }
  return LQRO_OK;
}
