// lqro_device.hpp — device-side fixed-size math shared by the lqro kernels.
//
// Exactness contract: liblqro.so is compiled with -ffp-contract=off, so each
// +, -, *, / below rounds once, exactly like the reference's x86-64 build.
// fp64 division and sqrt are IEEE correctly rounded on gfx950 (the default
// HIP lowering); fp32 division/sqrt use -fhip-fp32-correctly-rounded-divide-sqrt
// (hipcc's default).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lqro {

constexpr int kWave = 64;

// A row's LP may run as soon as every one of its planes is final.  rowpend
// (zeroed per step) adds LQRO_ROW_BIG for each finished row unit of the
// sweep, +1 for each hot pair (k_prio) and each inside-hull pair the sweep
// queues, -1 for each hot pair done without a hull and each hull job done:
// it equals row_split * LQRO_ROW_BIG exactly when the row has nothing open.
#define LQRO_ROW_BIG (1 << 20)
// The step's work, for the next steps' schedule (the side's width): the
// sweep's workgroup time summed over k_pair's workgroups (one a CU), the
// Qhull-order builds' time summed and their maximum, on the 100 MHz clock
// (s_memrealtime); words of the context's stats array (lqro_hull.hpp)
#define LQRO_ST_SWORK 144
#define LQRO_ST_BWORK 145
#define LQRO_ST_BMAX 146

// Workgroup-scope fence pair: orders this wave's LDS writes before other
// lanes' later reads (LDS executes a wave's instructions in order; this keeps
// the compiler from reordering and waits for lgkmcnt).
// x, opaque to the optimiser: values derived from it are recomputed after
// this point instead of being hoisted out of loops (each hoisted lane
// constant holds a VGPR for the whole kernel)
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// DPP lane moves (VALU, a few cycles) instead of ds_bpermute shuffles (LDS
// crossbar round trips) for wave reductions and scans.
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_i(int old, int x) {
  return __builtin_amdgcn_update_dpp(old, x, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_d(double old, double x) {
  const long long o = __double_as_longlong(old), v = __double_as_longlong(x);
  const int lo = dpp_i<CTRL, ROWS>((int)o, (int)v);
  const int hi = dpp_i<CTRL, ROWS>((int)(o >> 32), (int)(v >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// inclusive prefix sum over the 64 lanes (all lanes active): row_shr steps
// inside each 16-lane row, then row_bcast:15 / row_bcast:31 across rows
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += dpp_i<0x111, 0xF>(0, x);
  x += dpp_i<0x112, 0xF>(0, x);
  x += dpp_i<0x114, 0xF>(0, x);
  x += dpp_i<0x118, 0xF>(0, x);
  x += dpp_i<0x142, 0xA>(0, x);
  x += dpp_i<0x143, 0xC>(0, x);
  return x;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// operator! of include/matrix.h:603-671 for a 3x3: full pivoting, first
// strict maximum in (row, col) scan order, then back substitution and the
// column reshuffle.  Fully unrolled so the permutation stays in registers.
__device__ inline void inverse3(const double* q, double* out) {
  double m[9], inv[9];
  int rp[3] = {0, 1, 2}, cp[3] = {0, 1, 2};
#pragma unroll
  for (int i = 0; i < 9; ++i) { m[i] = q[i]; inv[i] = (i % 4 == 0) ? 1.0 : 0.0; }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    double best = 0.0; int br = k, bc = k;
#pragma unroll
    for (int i = k; i < 3; ++i)
#pragma unroll
      for (int j = k; j < 3; ++j) {
        double a = fabs(m[rp[i] * 3 + cp[j]]);
        if (a > best) { best = a; br = i; bc = j; }
      }
    int t = rp[k]; rp[k] = rp[br]; rp[br] = t;
    t = cp[k]; cp[k] = cp[bc]; cp[bc] = t;
#pragma unroll
    for (int i = k + 1; i < 3; ++i) {
      double f = m[rp[i] * 3 + cp[k]] / m[rp[k] * 3 + cp[k]];
#pragma unroll
      for (int j = k + 1; j < 3; ++j) m[rp[i] * 3 + cp[j]] -= f * m[rp[k] * 3 + cp[j]];
#pragma unroll
      for (int j = 0; j < k; ++j) inv[rp[i] * 3 + rp[j]] -= f * inv[rp[k] * 3 + rp[j]];
      inv[rp[i] * 3 + rp[k]] = -f;
    }
  }
#pragma unroll
  for (int k = 2; k >= 0; --k) {
    double qk = m[rp[k] * 3 + cp[k]];
#pragma unroll
    for (int j = 0; j < 3; ++j) inv[rp[k] * 3 + j] /= qk;
#pragma unroll
    for (int i = 0; i < k; ++i) {
      double f = m[rp[i] * 3 + cp[k]];
#pragma unroll
      for (int j = 0; j < 3; ++j) inv[rp[i] * 3 + j] -= f * inv[rp[k] * 3 + j];
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) out[cp[i] * 3 + j] = inv[rp[i] * 3 + j];
}

// Exact emulation of what qconvex reads back from pointList.txt: the value
// printed by ostream's default format (%g, 6 significant digits, round half
// to even on the exact binary value, LQRObstacles.cpp:871-873) and parsed
// back with correct rounding.  Exact for 1e-15 <= |v| < 1e21 (two-product /
// exact-remainder arithmetic decides the rounding); outside that range
// *out_of_range is set.
__device__ inline double round6(double v, int* out_of_range) {
  if (v == 0.0 || !isfinite(v)) return v;
  const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                          1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  double a = fabs(v);
  if (!(a >= 1e-15 && a < 1e21)) { *out_of_range = 1; return v; }
  int e = (int)floor(log10(a));
  double m = 0.0;
  for (int iter = 0; iter < 3; ++iter) {
    int k = 5 - e;                 // scale a by 10^k into [1e5, 1e6)
    double y, lo;                  // exact value = y + lo (lo tiny)
    int dir;                       // sign of the exact residual: -1, 0, +1
    if (k >= 0) {
      double s = p10[k];
      y = a * s;
      lo = fma(a, s, -y);
      dir = (lo > 0) - (lo < 0);
    } else {
      double d = p10[-k];
      y = a / d;
      double r = fma(-y, d, a);    // a - y*d exactly
      lo = r;
      dir = (r > 0) - (r < 0);
    }
    (void)lo;
    // make sure 1e5 <= exact < 1e6
    if (y < 1e5 || (y == 1e5 && dir < 0)) { e -= 1; continue; }
    if (y > 1e6 || (y == 1e6 && dir >= 0)) { e += 1; continue; }
    double m0 = rint(y);           // half-even on y
    double t = y - m0;             // exact
    if (t == 0.5) {                // y = m0 + 0.5, m0 even
      if (dir > 0) m0 += 1.0;
    } else if (t == -0.5) {        // y = m0 - 0.5, m0 even
      if (dir < 0) m0 -= 1.0;
    }
    m = m0;
    break;
  }
  double r;
  int k = e - 5;
  if (k >= 0) r = m * p10[k];
  else r = m / p10[-k];
  return v < 0 ? -r : r;
}

}  // namespace lqro
