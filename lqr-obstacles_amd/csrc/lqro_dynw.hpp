// lqro_dynw.hpp — the per-agent step of lqro_dyn.hpp (LQRObstacles.cpp:
// 1437-1446) with one WAVE per agent: the 16x16 work (the two Jacobians of f,
// the four matrix exponentials with their full-pivot solves, the noise
// covariance products, the covariance updates, the Jacobi sweep) is spread
// over the 64 lanes with the agent's matrices in LDS; the 3-vector and 3x3
// work (controllers, rotation resets, the 6x6 observation draw and inverse)
// runs redundantly in every lane on lqro_dyn.hpp's scalar code.
//
// Each output element is computed by one lane in the reference's operation
// order (dot products accumulate from 0.0 in k order, element-wise chains
// left to right), and the pivot searches pick the reference's pivot (first
// strict maximum in scan order), so the wave version computes exactly what
// the one-lane version does: tests/test_gpu_dyn.py checks both against the
// oracle and against each other.
#pragma once
#include "lqro_device.hpp"
#include "lqro_dyn.hpp"

namespace lqro {
namespace dynw {

using dyn::kNormals;
using dyn::kU;
using dyn::kV;
using dyn::kX;
using dyn::kZ;
using synth::Mat;
using synth::Quad;
using synth::Vec3;

constexpr int kMM = kX * kX;   // 256
// per-wave LDS block, doubles
enum : int {
  oF = 0, oA = 1 * kMM, oA2 = 2 * kMM, oMM = 3 * kMM, oP = 4 * kMM, oM = 5 * kMM, oT1 = 6 * kMM,
  oT2 = 7 * kMM, oE0 = 8 * kMM, oE1 = 9 * kMM, oE2 = 10 * kMM, oE3 = 11 * kMM, oE4 = 12 * kMM,
  oE5 = 13 * kMM, oInt = 14 * kMM, kWaveDoubles = 14 * kMM + 32
};

__device__ __forceinline__ void sync() { wave_lds_sync(); }

// LQRO_DYN_PROFILE (launch_dyn): cycles per phase summed over the agents
// (s_memtime; prof null: off, the stamps compile to a branch)
struct DynProf {
  unsigned long long* prof;
  unsigned long long t;
  int lane;
  __device__ __forceinline__ void stamp(int k) {
    if (!prof) return;
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    if (lane == 0) atomicAdd(&prof[k], n - t);
    t = n;
  }
};

// C = A B (16x16x16), C distinct from A and B.  Lane L computes the
// elements (L/16 + 4t, L%16), t < 4: its column of B is read once into
// registers (the stores to C cannot alias it), every sum in k order from 0.0
__device__ __forceinline__ void mm(const double* __restrict__ A, const double* __restrict__ B, double* __restrict__ C,
                                   int lane) {
  const int i0 = lane >> 4, j = lane & 15;
  double b[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) b[k] = B[k * 16 + j];
  double acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    acc[t] = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[t] += A[(i0 + 4 * t) * 16 + k] * b[k];
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) C[(i0 + 4 * t) * 16 + j] = acc[t];
  sync();
}
// C = A B^T
__device__ __forceinline__ void mm_nt(const double* __restrict__ A, const double* __restrict__ B,
                                      double* __restrict__ C, int lane) {
  const int i0 = lane >> 4, j = lane & 15;
  double b[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) b[k] = B[j * 16 + k];
  double acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    acc[t] = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[t] += A[(i0 + 4 * t) * 16 + k] * b[k];
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) C[(i0 + 4 * t) * 16 + j] = acc[t];
  sync();
}

// wave arg-max of (v, q), the lowest q among the lanes holding the maximum
// (the first strict maximum of a scan in q order), in every lane: DPP row
// shifts and row broadcasts, no LDS crossbar round trips
__device__ __forceinline__ void argmax64(double& v, int& q) {
  double m = v;
  m = fmax(m, dpp_d<0x111, 0xF>(-INFINITY, m));   // row_shr:1
  m = fmax(m, dpp_d<0x112, 0xF>(-INFINITY, m));   // row_shr:2
  m = fmax(m, dpp_d<0x114, 0xF>(-INFINITY, m));   // row_shr:4
  m = fmax(m, dpp_d<0x118, 0xF>(-INFINITY, m));   // row_shr:8
  m = fmax(m, dpp_d<0x142, 0xA>(-INFINITY, m));   // row_bcast:15
  m = fmax(m, dpp_d<0x143, 0xC>(-INFINITY, m));   // row_bcast:31
  const long long b = __double_as_longlong(m);
  const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  m = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  int t = v == m ? q : INT_MAX;
  t = min(t, dpp_i<0x111, 0xF>(INT_MAX, t));
  t = min(t, dpp_i<0x112, 0xF>(INT_MAX, t));
  t = min(t, dpp_i<0x114, 0xF>(INT_MAX, t));
  t = min(t, dpp_i<0x118, 0xF>(INT_MAX, t));
  t = min(t, dpp_i<0x142, 0xA>(INT_MAX, t));
  t = min(t, dpp_i<0x143, 0xC>(INT_MAX, t));
  q = __builtin_amdgcn_readlane(t, 63);
  v = m;
}
// y = A v (16x16 by a wave-uniform 16-vector), broadcast through `scratch`
__device__ __forceinline__ Mat<kX, 1> mv(const double* A, const Mat<kX, 1>& v, double* scratch, int lane) {
  if (lane < 16) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += A[lane * 16 + k] * v.e[k];
    scratch[lane] = acc;
  }
  sync();
  Mat<kX, 1> y;
#pragma unroll
  for (int k = 0; k < 16; ++k) y.e[k] = scratch[k];
  sync();
  return y;
}
__device__ __forceinline__ void copy(const double* S, double* D, int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t) D[lane + 64 * t] = S[lane + 64 * t];
  sync();
}

// first strict maximum of |m| in (row, col) scan order over the trailing
// (N-k)^2 block of the permuted matrix, as operator! picks it
template <int N = 16>
__device__ __forceinline__ void pivot(const double* m, const int* rp, const int* cp, int k, int lane,
                                      int& br, int& bc) {
  const int w = N - k;
  constexpr int kU = (N * N + 63) / 64;
  // the lane's elements idx = lane + 64 u, loaded at once (independent reads)
  double a[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int idx = lane + 64 * u;
    a[u] = 0.0;
    if (idx < w * w) {
      const int i = k + idx / w, j = k + idx % w;
      a[u] = fabs(m[rp[i] * N + cp[j]]);
    }
  }
  double best = 0.0;
  int bi = INT_MAX;
#pragma unroll
  for (int u = 0; u < kU; ++u)
    if (a[u] > best) { best = a[u]; bi = lane + 64 * u; }
  argmax64(best, bi);
  if (bi == INT_MAX) { br = k; bc = k; }
  else { br = k + bi / w; bc = k + bi % w; }
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  return __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(b >> 32), l) << 32) |
                              (unsigned)__builtin_amdgcn_readlane((int)b, l));
}
__device__ __forceinline__ void lds_order() { __asm__ __volatile__("" ::: "memory"); }
// bank swizzle of a 16 x 16 work matrix: (i, j) at 16 i + (j ^ i).  A
// column read (16 rows, one column; ds_read_b64 banks (a/4) mod 64) and a
// column write (16 lanes, ds_write_b64 banks (a/4) mod 32) then touch
// distinct banks; rows stay rows (permuted within)
template <int N = 16>
__device__ __forceinline__ int swz(int i, int j) { return N == 16 ? i * 16 + (j ^ i) : i * N + j; }

// X = P^-1 Q by full pivoting with the reference's final reshuffle
// (operator%, MAT:370-442, = synth::solve_ix): m (P) and x (Q) in LDS, both
// overwritten; the solution is left in x.
//
// The reference permutes through index vectors (m(rp i, cp j)); here the
// rows and columns are swapped in place, so M[i][j] = m(rp i, cp j) and
// X[i][j] = x(rp i, j) are read directly, and rp / cp live in lanes 0-15 of
// a register (readlane / writelane).  Every element sees the reference's
// operations in its order; only the storage differs, and the reshuffle's
// net row permutation (the same swaps, tracked on row labels) is applied
// once at the end.  One wave, so LDS operations execute in program order:
// between the passes only a compiler barrier (lds_order).
//  - pivot: lane (row k + g + 4u, column lane%16), g = lane/16; the first
//    strict maximum of |M| in (row, column) order, key 16 row + column;
//  - swap + elimination in one pass: lane row i = lane%16, columns
//    c = g + 4u of [M | X]; it reads the swapped matrix's element, its
//    row's multiplier source and the pivot row, divides once per row.
//  NS systems at once (expm's two exponentials): the same passes, each
//  system's operations interleaved with the other's (independent chains:
//  one's LDS latency is the other's issue slots).
template <int NS>
__device__ __forceinline__ void solveN(double* const* m, double* const* x, int lane,
                                       unsigned long long* prof = nullptr) {
  DynProf sp{prof, prof ? __builtin_amdgcn_s_memtime() : 0ull, lane};
  int rpv[NS], cpv[NS];
  const int g = lane >> 4, l16 = lane & 15;
#pragma unroll
  for (int y = 0; y < NS; ++y) rpv[y] = cpv[y] = l16;
  // every read and write below is unconditional (addresses in range, the
  // unused values selected away; a row or column that does not change is
  // written back as read): no exec-mask branches around LDS operations
  for (int k = 0; k < 16; ++k) {
    double a[NS][4];
#pragma unroll
    for (int y = 0; y < NS; ++y)
#pragma unroll
      for (int u = 0; u < 4; ++u) a[y][u] = fabs(m[y][swz(min(k + g + 4 * u, 15), l16)]);
    int br[NS], bc[NS];
#pragma unroll
    for (int y = 0; y < NS; ++y) {
      double best = 0.0;
      int bi = INT_MAX;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = l16 >= k && k + g + 4 * u < 16;
        if (ok && a[y][u] > best) { best = a[y][u]; bi = (k + g + 4 * u) * 16 + l16; }
      }
      argmax64(best, bi);
      br[y] = bi == INT_MAX ? k : bi >> 4;
      bc[y] = bi == INT_MAX ? k : bi & 15;
      const int r0 = __builtin_amdgcn_readlane(rpv[y], k), r1 = __builtin_amdgcn_readlane(rpv[y], br[y]);
      rpv[y] = lane == k ? r1 : rpv[y];
      rpv[y] = lane == br[y] ? r0 : rpv[y];
      const int c0 = __builtin_amdgcn_readlane(cpv[y], k), c1 = __builtin_amdgcn_readlane(cpv[y], bc[y]);
      cpv[y] = lane == k ? c1 : cpv[y];
      cpv[y] = lane == bc[y] ? c0 : cpv[y];
    }
    lds_order();
    // swapped matrix: M'[i][c] = M[sw(i)][tw(c)], X'[i][c] = X[sw(i)][c];
    // u < 4: M columns g + 4u, u >= 4: X columns g + 4(u - 4)
    const int i = l16;
    const bool elim = i > k;
    double v[NS][8], pr[NS][8], fs[NS], pv[NS];
#pragma unroll
    for (int y = 0; y < NS; ++y) {
      const int si = i == k ? br[y] : (i == br[y] ? k : i);
      fs[y] = m[y][swz(si, bc[y])];
      pv[y] = m[y][swz(br[y], bc[y])];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u < 4) {
          const int c = g + 4 * u;
          const int tc = c == k ? bc[y] : (c == bc[y] ? k : c);
          v[y][u] = m[y][swz(si, tc)];
          pr[y][u] = m[y][swz(br[y], tc)];
        } else {
          const int c = g + 4 * (u - 4);
          v[y][u] = x[y][swz(si, c)];
          pr[y][u] = x[y][swz(br[y], c)];
        }
      }
    }
#pragma unroll
    for (int y = 0; y < NS; ++y) {
      const double f = fs[y] / pv[y];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool e = elim && (u >= 4 || g + 4 * u > k);
        const double nv = v[y][u] - f * pr[y][u];
        v[y][u] = e ? nv : v[y][u];
      }
    }
#pragma unroll
    for (int y = 0; y < NS; ++y)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u < 4) m[y][swz(i, g + 4 * u)] = v[y][u];
        else x[y][swz(i, g + 4 * (u - 4))] = v[y][u];
      }
    lds_order();
  }
  sp.stamp(24);
  // back substitution: lane column j = lane%16, rows g + 4u
  for (int k = 15; k >= 0; --k) {
    double qk[NS], xr[NS], f[NS][4], xv[NS][4];
#pragma unroll
    for (int y = 0; y < NS; ++y) {
      qk[y] = m[y][swz(k, k)];
      xr[y] = x[y][swz(k, l16)];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        f[y][u] = m[y][swz(g + 4 * u, k)];
        xv[y][u] = x[y][swz(g + 4 * u, l16)];
      }
    }
#pragma unroll
    for (int y = 0; y < NS; ++y) {
      const double xk = xr[y] / qk[y];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = g + 4 * u;
        const double nv = xv[y][u] - f[y][u] * xk;
        x[y][swz(i, l16)] = i < k ? nv : (i == k ? xk : xv[y][u]);
      }
    }
    lds_order();
  }
  sp.stamp(25);
  // the reshuffle (MAT:428-441): x(rp i) holds X[i]; the reference swaps
  // x's rows cp i / rp i in turn and updates rp / irp; the swaps are
  // tracked on row labels (lab[s]: the row of x(rp .) now at s), the data
  // moved once: out[s] = X[irp0[lab[s]]]
  double o[NS][4];
#pragma unroll
  for (int y = 0; y < NS; ++y) {
    const int irp0 = __builtin_amdgcn_ds_permute((lane < 16 ? rpv[y] : lane) * 4, l16);
    int irpv = irp0, labv = l16, rp = rpv[y];
    for (int q = 0; q < 16; ++q) {
      const int ri = __builtin_amdgcn_readlane(rp, q), ci = __builtin_amdgcn_readlane(cpv[y], q);
      const int l1 = __builtin_amdgcn_readlane(labv, ci), l2 = __builtin_amdgcn_readlane(labv, ri);
      labv = lane == ci ? l2 : labv;
      labv = lane == ri ? l1 : labv;
      const int a = __builtin_amdgcn_readlane(irpv, ci);
      rp = lane == a ? ri : rp;
      irpv = lane == ri ? a : irpv;
    }
    const int src = __builtin_amdgcn_ds_bpermute(labv * 4, irp0);   // lanes 0-15: irp0[lab[s]]
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int srow = __builtin_amdgcn_ds_bpermute((g + 4 * u) * 4, src);
      o[y][u] = x[y][swz(srow, l16)];
    }
  }
  lds_order();
#pragma unroll
  for (int y = 0; y < NS; ++y)
#pragma unroll
    for (int u = 0; u < 4; ++u) x[y][(g + 4 * u) * 16 + l16] = o[y][u];
  sync();
  sp.stamp(26);
}

// C_y = A_y B_y for NS products at once (C distinct from A and B): lane L
// computes the elements (L/16 + 4t, L%16); with VU, the products are
// A6 = A2 A4 and, instead of storing them, V = A6 b6 + A4 b4 + A2 b2 + I b0
// and U' = A6 b7 + A4 b5 + A2 b3 + I b1 go to C_y and D_y (expm, MAT:776-781)
template <int NS, bool VU = false>
__device__ __forceinline__ void mmN(const double* const* A, const double* const* B, double* const* C, int lane,
                                    double* const* D = nullptr) {
  const int i0 = lane >> 4, j = lane & 15;
  double acc[NS][4];
#pragma unroll
  for (int y = 0; y < NS; ++y) {
    double b[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) b[k] = B[y][k * 16 + j];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[y][t] = 0.0;
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[y][t] += A[y][(i0 + 4 * t) * 16 + k] * b[k];
    }
  }
  if constexpr (VU) {
    const double b0 = 1729728e1, b1 = 864864e1, b2 = 199584e1, b3 = 2772e2, b4 = 252e2, b5 = 1512e0,
                 b6 = 56e0, b7 = 1e0;
#pragma unroll
    for (int y = 0; y < NS; ++y)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int e = (i0 + 4 * t) * 16 + j;
        const double I = (i0 + 4 * t) == j ? 1.0 : 0.0;
        const double a2 = A[y][e], a4 = B[y][e], a6 = acc[y][t];
        C[y][e] = a6 * b6 + a4 * b4 + a2 * b2 + I * b0;
        D[y][e] = a6 * b7 + a4 * b5 + a2 * b3 + I * b1;
      }
  } else {
#pragma unroll
    for (int y = 0; y < NS; ++y)
#pragma unroll
      for (int t = 0; t < 4; ++t) C[y][(i0 + 4 * t) * 16 + j] = acc[y][t];
  }
  sync();
}

// out_y = exp(q_y) for NS matrices at once (MAT:763-790, = synth::expm<16>,
// degree-7 Pade with scaling and squaring), interleaved as solveN.  q_y is
// scaled in place (it becomes A); four work matrices a system, wk[4y..4y+3]
// (X2, X4, V, U), none aliasing q or out.  A6 is never stored: the product
// A2 A4 goes straight into V and U' (mmN<VU>).
template <int NS>
__device__ __forceinline__ void expmN(double* const* q, double* const* out, double* const* wk, int lane,
                                      unsigned long long* prof = nullptr) {
  DynProf ep{prof, prof ? __builtin_amdgcn_s_memtime() : 0ull, lane};
  const double lim = 9.504178996162932e-1;
  int sq[NS];
#pragma unroll
  for (int y = 0; y < NS; ++y) {
    // 1-norm: column sums in i order, the max of them (order-free)
    double cs = 0.0;
    if (lane < 16)
      for (int i = 0; i < 16; ++i) cs += fabs(q[y][i * 16 + lane]);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) cs = fmax(cs, __shfl_xor(cs, off));
    const double c = ceil(log(cs / lim) * M_LOG2E);
    sq[y] = (int)(0.0 < c ? c : 0.0);
    const double p2 = pow(2.0, sq[y]);
#pragma unroll
    for (int t = 0; t < 4; ++t) q[y][lane + 64 * t] = q[y][lane + 64 * t] / p2;
  }
  sync();
  const double* cA[NS];
  double *X2[NS], *X4[NS], *V[NS], *U[NS];
  const double *cX2[NS], *cX4[NS], *cU[NS];
#pragma unroll
  for (int y = 0; y < NS; ++y) {
    cA[y] = q[y];
    X2[y] = wk[4 * y]; X4[y] = wk[4 * y + 1]; V[y] = wk[4 * y + 2]; U[y] = wk[4 * y + 3];
    cX2[y] = X2[y]; cX4[y] = X4[y]; cU[y] = U[y];
  }
  mmN<NS>(cA, cA, X2, lane);
  mmN<NS>(cX2, cX2, X4, lane);
  mmN<NS, true>(cX2, cX4, V, lane, U);
  ep.stamp(19);
  mmN<NS>(cA, cU, X2, lane);   // X2 <- U = A U'
#pragma unroll
  for (int y = 0; y < NS; ++y)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int e = lane + 64 * t;
      const double vv = V[y][e], uu = X2[y][e];
      X4[y][swz(e >> 4, e & 15)] = vv - uu;   // P = V - U (swizzled for solveN)
      U[y][swz(e >> 4, e & 15)] = vv + uu;    // Q = V + U
    }
  sync();
  ep.stamp(20);
  solveN<NS>(X4, U, lane, prof);
  ep.stamp(21);
#pragma unroll
  for (int y = 0; y < NS; ++y) {
    double* cur = U[y];
    double* nxt = X2[y];
    for (int i = 0; i < sq[y]; ++i) {
      const double* a1[1] = {cur};
      double* c1[1] = {nxt};
      mmN<1>(a1, a1, c1, lane);
      double* t = cur; cur = nxt; nxt = t;
    }
    copy(cur, out[y], lane);
  }
  ep.stamp(22);
  if (prof && lane == 0) atomicAdd(&prof[23], (unsigned long long)(sq[0] + (NS > 1 ? sq[NS - 1] : 0)));
}

// jacobi (MAT:674-759, = dyn::jacobi<N>) of m: V, D in LDS (row stride N).
// One wave, so its LDS operations execute in program order: inside the loop
// only a compiler barrier separates a write from a later read (no wait for
// the write to land).  Per iteration:
//  - the pivot scan over the lanes, its N-1 entries one a lane, the
//    reference's first strict maximum as a DPP arg-max;
//  - D(p,q) from the scanning lane's register, D(p,p), D(q,q) from the
//    diagonal, which lives in registers (lane i: D(i,i); no rotation lane
//    touches it) and goes back to D at the end;
//  - one pass over lanes [0, 2N): the rotation of D's entries (r,p), (r,q)
//    (lanes r != p, q) and of V's (lanes N + r), both entries read, both
//    written; lanes p and q write D(p,q) = 0 and update their diagonal.
template <int N>
__device__ __forceinline__ void jacobi(const double* m, double* V, double* D, int lane,
                                       unsigned long long* prof = nullptr) {
  int iters = 0, rots = 0;
  for (int e = lane; e < N * N; e += 64) {
    D[swz<N>(e / N, e % N)] = m[e];
    V[swz<N>(e / N, e % N)] = (e / N == e % N) ? 1.0 : 0.0;
  }
  double dg = lane < N ? m[lane * N + lane] : 0.0;
  // the reference's loop ends after N scans without a rotation when no entry
  // above the diagonal exceeds DBL_EPSILON (a diagonal matrix: the
  // observation covariance): one scan then, D = diag and V = I either way
  bool any = false;
  for (int e = lane; e < N * N; e += 64) any |= e / N < e % N && fabs(m[e]) > DBL_EPSILON;
  const bool diag = __ballot(any) == 0ull;
  sync();
  int pivot = 0, zeros = diag ? N - 1 : 0;
  if (diag) iters = N - 1;
  // phase cycles summed in registers, added once (per-iteration atomics
  // from every wave serialise on the counters)
  const bool jprof = N == 16 && prof;
  unsigned long long jt = jprof ? __builtin_amdgcn_s_memtime() : 0ull, jacc[3] = {0, 0, 0};
  auto jstamp = [&](int k) {
    if (!jprof) return;
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    jacc[k] += n - jt;
    jt = n;
  };
  for (;;) {
    ++iters;
    // scan position l: (l, pivot) above the diagonal for l < pivot, then
    // (pivot, l + 1) right of it.  Lane l reads position l; the first strict
    // maximum above 0 in scan order is the largest value at the lowest
    // position (DPP within the first 16 lanes, lane 15 holds it)
    double sv = 0.0;
    if (lane < N - 1) {
      const int a = lane < pivot ? lane : pivot, b = lane < pivot ? pivot : lane + 1;
      sv = D[swz<N>(a, b)];
    }
    const double av = fabs(sv);
    double mx = av;
    mx = fmax(mx, dpp_d<0x111, 0xF>(-INFINITY, mx));   // row_shr:1
    mx = fmax(mx, dpp_d<0x112, 0xF>(-INFINITY, mx));   // row_shr:2
    mx = fmax(mx, dpp_d<0x114, 0xF>(-INFINITY, mx));   // row_shr:4
    mx = fmax(mx, dpp_d<0x118, 0xF>(-INFINITY, mx));   // row_shr:8
    const double maximum = readlane_d(mx, 15);
    int pos = (lane < N - 1 && av == maximum) ? lane : INT_MAX;
    pos = min(pos, dpp_i<0x111, 0xF>(INT_MAX, pos));
    pos = min(pos, dpp_i<0x112, 0xF>(INT_MAX, pos));
    pos = min(pos, dpp_i<0x114, 0xF>(INT_MAX, pos));
    pos = min(pos, dpp_i<0x118, 0xF>(INT_MAX, pos));
    pos = __builtin_amdgcn_readlane(pos, 15);
    const int pv = pivot;
    pivot = (pivot + 1) % N;
    jstamp(0);
    if (maximum <= DBL_EPSILON) {
      if (++zeros == N) break;
      continue;
    }
    const int p = pos < pv ? pos : pv, q = pos < pv ? pv : pos + 1;
    zeros = 0;
    ++rots;
    const double dpq = readlane_d(sv, pos);
    const double theta = 0.5 * (readlane_d(dg, q) - readlane_d(dg, p)) / dpq;
    double t = 1 / (fabs(theta) + hypot(theta, 1.0));
    if (theta < 0) t = -t;
    const double c = 1 / hypot(t, 1.0);
    const double s = c * t;
    const double tau = s / (1 + c);
    jstamp(1);
    lds_order();   // the scan's reads before the rotation's writes
    if (lane < 2 * N) {
      const bool dl = lane < N;
      const int r = dl ? lane : lane - N;
      double* W = dl ? D : V;
      const bool pq = dl && (r == p || r == q);
      // the two entries row/col r of the rotation touches: D's {r,p}, {r,q}
      // in the upper triangle (V's (r,p), (r,q)); lanes p, q zero D(p,q)
      const int ra = pq ? p : (dl ? min(r, p) : r), ca = pq ? q : (dl ? max(r, p) : p);
      const int rb = pq ? p : (dl ? min(r, q) : r), cb = pq ? q : (dl ? max(r, q) : q);
      const int ia = swz<N>(ra, ca), ib = swz<N>(rb, cb);
      const double a = W[ia], b = W[ib];
      const double na = pq ? 0.0 : a - s * (b + tau * a);
      const double nb = pq ? 0.0 : b + s * (a - tau * b);
      W[ia] = na;
      W[ib] = nb;
      if (lane == p) dg -= t * dpq;
      if (lane == q) dg += t * dpq;
    }
    lds_order();
    jstamp(2);
  }
  sync();
  // back to the plain layout: D = diag(dg), V's rows un-permuted (every
  // lane's reads before its writes)
  {
    constexpr int kT = (N * N + 63) / 64;
    double vv[kT];
#pragma unroll
    for (int t = 0; t < kT; ++t) {
      const int e = lane + 64 * t;
      vv[t] = e < N * N ? V[swz<N>(e / N, e % N)] : 0.0;
    }
    lds_order();
#pragma unroll
    for (int t = 0; t < kT; ++t) {
      const int e = lane + 64 * t;
      if (e < N * N) {
        V[e] = vv[t];
        D[e] = 0;
      }
    }
    if (lane < N) D[lane * N + lane] = dg;
  }
  sync();
  if (jprof && lane == 0)
    for (int k = 0; k < 3; ++k) atomicAdd(&prof[16 + k], jacc[k]);
  if (prof && lane == 0) { atomicAdd(&prof[11 + (N == 16 ? 0 : 2)], (unsigned long long)iters);
                           atomicAdd(&prof[12 + (N == 16 ? 0 : 2)], (unsigned long long)rots); }
}

// operator! (MAT:603-671, = synth::inverse_ix<N>) of m in LDS, over the
// lanes: full-pivot Gauss-Jordan, the same pivots and per-element operation
// order; m is overwritten with the inverse, inv is work space
template <int N>
__device__ __forceinline__ void inverse(double* m, double* inv, int* ip, int lane) {
  int* rp = ip;
  int* cp = ip + N;
  for (int e = lane; e < N * N; e += 64) inv[e] = (e / N == e % N) ? 1.0 : 0.0;
  if (lane < N) { rp[lane] = lane; cp[lane] = lane; }
  sync();
  for (int k = 0; k < N; ++k) {
    int br, bc;
    pivot<N>(m, rp, cp, k, lane, br, bc);
    const int rk = rp[br], ck = cp[bc], rb = rp[k], cb = cp[k];
    sync();
    if (lane == 0) { rp[k] = rk; rp[br] = rb; cp[k] = ck; cp[bc] = cb; }
    sync();
    // rows i > k against row k: m's columns after k, inv's columns rp[j < k], inv(rp i, rp k) = -f
    const double piv = m[rp[k] * N + cp[k]];
    for (int idx = lane; idx < (N - 1 - k) * N; idx += 64) {
      const int i = k + 1 + idx / N, c = idx % N;
      const double f = m[rp[i] * N + cp[k]] / piv;
      if (c > k) m[rp[i] * N + cp[c]] -= f * m[rp[k] * N + cp[c]];
      else if (c < k) inv[rp[i] * N + rp[c]] -= f * inv[rp[k] * N + rp[c]];
      else inv[rp[i] * N + rp[k]] = -f;
    }
    sync();
  }
  for (int k = N - 1; k >= 0; --k) {
    const double qk = m[rp[k] * N + cp[k]];
    if (lane < N) inv[rp[k] * N + lane] /= qk;
    sync();
    for (int idx = lane; idx < k * N; idx += 64) {
      const int i = idx / N, j = idx % N;
      const double f = m[rp[i] * N + cp[k]];
      inv[rp[i] * N + j] -= f * inv[rp[k] * N + j];
    }
    sync();
  }
  for (int idx = lane; idx < N * N; idx += 64) {
    const int i = idx / N, j = idx % N;
    m[cp[i] * N + j] = inv[rp[i] * N + j];
  }
  sync();
}

// A = exp(dt F), A2 = exp(dt/2 F), MM, dx as dyn::discretize; F from 32
// lanes' f evaluations
__device__ __forceinline__ void discretize(const Quad& q, const Mat<kX, 1>& x, const Mat<3, 3>& R,
                                          const Mat<kU, 1>& u, double* w, int lane, Mat<kX, 1>& dx, DynProf& pf) {
  double* fr = w + oE0;   // rows 0..15 f(x + h e_i), 16..31 f(x - h e_i), 32 f(x)
  {
    Mat<kX, 1> xp;
    const int i = lane & 15;
    const bool minus = (lane >> 4) == 1;
    const bool centre = lane >= 32;
#pragma unroll
    for (int c = 0; c < kX; ++c)
      xp.e[c] = (centre || c != i) ? x.e[c] : (minus ? x.e[c] - q.h : x.e[c] + q.h);
    const Mat<kX, 1> f = synth::dynamics(q, xp, R, u);
    if (lane <= 32)
#pragma unroll
      for (int k = 0; k < kX; ++k) fr[lane * 16 + k] = f.e[k];
  }
  sync();
  double* F = w + oF;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int e = lane + 64 * t, k = e >> 4, i = e & 15;
    F[e] = (fr[i * 16 + k] - fr[(16 + i) * 16 + k]) / (2 * q.h);
  }
  Mat<kX, 1> xdot;
#pragma unroll
  for (int k = 0; k < kX; ++k) xdot.e[k] = fr[32 * 16 + k];
  sync();
  pf.stamp(8);   // the Jacobians (f at 33 points)
  double* A = w + oA;
  double* A2 = w + oA2;
  double* T1 = w + oT1;
  double* T2 = w + oT2;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    T1[lane + 64 * t] = q.dt * F[lane + 64 * t];
    T2[lane + 64 * t] = (q.dt * 0.5) * F[lane + 64 * t];
  }
  sync();
  {
    // both exponentials at once; F and MM are free until after them
    double* const qs[2] = {T1, T2};
    double* const outs[2] = {A, A2};
    double* const wk[8] = {w + oE0, w + oE1, w + oE2, w + oE3, w + oE4, w + oE5, F, w + oMM};
    expmN<2>(qs, outs, wk, lane, pf.prof);
  }
  pf.stamp(9);   // the two exponentials
  // MM = (dt/6) (M + 4 A2 M A2^T + A M A^T)
  const double* M = w + oM;
  double* MM = w + oMM;
#pragma unroll
  for (int t = 0; t < 4; ++t) T2[lane + 64 * t] = 4 * A2[lane + 64 * t];
  sync();
  mm(T2, M, T1, lane);
  mm_nt(T1, A2, T2, lane);        // 4 A2 M A2^T
  mm(A, M, T1, lane);
  mm_nt(T1, A, F, lane);          // A M A^T (F is free now)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int e = lane + 64 * t;
    MM[e] = (q.dt / 6) * (M[e] + T2[e] + F[e]);
  }
  sync();
  // dx = (dt/6) (xdot + 4 (A2 xdot) + A xdot)
  const Mat<kX, 1> a2x = mv(A2, xdot, T1, lane);
  const Mat<kX, 1> ax = mv(A, xdot, T1, lane);
  dx = (q.dt / 6) * (xdot + 4 * a2x + ax);
  pf.stamp(10);   // MM and dx
}

// sampleGaussian(0, MM, nrm) (simulator2.h:21-32) on the LDS matrix MM
__device__ __forceinline__ Mat<kX, 1> noise(double* w, const double* nrm, int lane, unsigned long long* prof) {
  double* V = w + oT1;
  double* D = w + oT2;
  jacobi<16>(w + oMM, V, D, lane, prof);
  if (lane < 16) D[lane * 17] = sqrt(D[lane * 17]);
  sync();
  mm(V, D, w + oE0, lane);
  Mat<kX, 1> smp;
#pragma unroll
  for (int k = 0; k < kX; ++k) smp.e[k] = nrm[k];
  return mv(w + oE0, smp, w + oE1, lane) + Mat<kX, 1>::zero();
}

// kalmanFilter2 (LQRO:507-518) with P in LDS (inlined: no call frame)
__device__ __forceinline__ void kalman_update(const Quad& q, Mat<kX, 1>& x, Mat<3, 3>& R, const Mat<kZ, 1>& z,
                              const double* Nz, double* w, int lane) {
  double* P = w + oP;
  double* H = w + oE0;          // 6x16
  double* PHt = w + oE0 + 96;   // 16x6
  double* HP = w + oE0 + 192;   // 6x16
  double* S = w + oE1 + 64;     // 6x6
  double* K = w + oE1 + 128;    // 16x6
  double* KH = w + oE2;         // 16x16
  double* T1 = w + oT1;
  // x through LDS: the lanes index it by their element (no private array)
  double* xs = w + oE2 + 240;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < kX; ++k) xs[k] = x.e[k];
  sync();
  // Jacobian_hx (LQRO:443-452): row k observes x[9 + k] (k < 3) or x[k - 3]
  for (int e = lane; e < 96; e += 64) {
    const int k = e >> 4, i = e & 15;
    const int ok = k < 3 ? 9 + k : k - 3;
    const double xv = xs[i];
    const bool hit = ok == i;
    const double hr = hit ? xv + q.h : xs[ok];
    const double hl = hit ? xv - q.h : xs[ok];
    H[e] = (hr - hl) / (2 * q.h);
  }
  sync();
  for (int e = lane; e < 96; e += 64) {
    {   // P H^T (16x6)
      const int i = e / 6, j = e % 6;
      double acc = 0.0;
      for (int k = 0; k < 16; ++k) acc += P[i * 16 + k] * H[j * 16 + k];
      PHt[e] = acc;
    }
    {   // H P (6x16)
      const int i = e >> 4, j = e & 15;
      double acc = 0.0;
      for (int k = 0; k < 16; ++k) acc += H[i * 16 + k] * P[k * 16 + j];
      HP[e] = acc;
    }
  }
  sync();
  if (lane < 36) {   // H P H^T + N
    const int i = lane / 6, j = lane % 6;
    double acc = 0.0;
    for (int k = 0; k < 16; ++k) acc += HP[i * 16 + k] * H[j * 16 + k];
    S[lane] = acc + Nz[lane];
  }
  sync();
  // S^-1 (synth::inverse) over the lanes, in place
  inverse<kZ>(S, w + oE1 + 224, reinterpret_cast<int*>(w + oInt), lane);
  for (int e = lane; e < 96; e += 64) {   // K = P H^T S^-1
    const int i = e / 6, j = e % 6;
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) acc += PHt[i * 6 + k] * S[k * 6 + j];
    K[e] = acc;
  }
  sync();
  const Mat<kZ, 1> innov = z - dyn::observe(x);
  if (lane < 16) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) acc += K[lane * 6 + k] * innov.e[k];
    T1[lane] = acc;
  }
  sync();
  Mat<kX, 1> kz;
#pragma unroll
  for (int k = 0; k < kX; ++k) kz.e[k] = T1[k];
  x = x + kz;
#pragma unroll
  for (int t = 0; t < 4; ++t) {   // I - K H
    const int e = lane + 64 * t, i = e >> 4, j = e & 15;
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) acc += K[i * 6 + k] * H[k * 16 + j];
    KH[e] = (i == j ? 1.0 : 0.0) - acc;
  }
  sync();
  mm(KH, P, T1, lane);
  copy(T1, P, lane);
  dyn::reset_rot(x, R);
}

// One agent through LQRO:1438-1445 (= dyn::agent_step), one wave
__device__ __forceinline__ void agent_step(const dyn::AgentParams& a, double* x_, double* rot_, double* xt_, double* rott_,
                           double* P_, double* vgoal_, double* u_out, double* w, int lane,
                           unsigned long long* prof = nullptr) {
  using dyn::get;
  DynProf pf{prof, prof ? __builtin_amdgcn_s_memtime() : 0ull, lane};
  const Quad q = dyn::quad(a.model);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    w[oP + lane + 64 * t] = P_[lane + 64 * t];
    w[oM + lane + 64 * t] = a.M[lane + 64 * t];
  }
  sync();
  Mat<kX, 1> x = get<kX, 1>(x_), xtrue = get<kX, 1>(xt_);
  Mat<3, 3> R = get<3, 3>(rot_), Rtrue = get<3, 3>(rott_);
  const Mat<kU, 1> ug = get<kU, 1>(a.u_goal);
  const Mat<kU, 1> u = dyn::control_velocity(x, R, get<3, 1>(vgoal_), ug, get<kU, kX>(a.L),
                                             get<kU, kV>(a.E), get<kU, 1>(a.l));        // findU
  pf.stamp(0);
  {                                                                                   // propagateU
    Mat<kX, 1> dx;
    discretize(q, xtrue, Rtrue, u, w, lane, dx, pf);
    pf.stamp(1);
    const Mat<kX, 1> g = noise(w, a.normals, lane, prof);
    pf.stamp(2);
    xtrue = xtrue + dx + g;
    dyn::reset_rot(xtrue, Rtrue);
  }
  {                                                                                   // kalmanFilter1
    Mat<kX, 1> dx;
    discretize(q, x, R, u, w, lane, dx, pf);
    pf.stamp(3);
    x = x + dx;
    double* P = w + oP;
    mm(w + oA, P, w + oT1, lane);
    mm_nt(w + oT1, w + oA, w + oT2, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t) P[lane + 64 * t] = w[oT2 + lane + 64 * t] + w[oMM + lane + 64 * t];
    sync();
    dyn::reset_rot(x, R);
  }
  pf.stamp(4);
  // the observation draw: sampleGaussian(h(xTrue), N) (simulator2.h:21-32,
  // = dyn::sample_gaussian<6>) over the lanes
  Mat<kZ, 1> z;
  {
    double* Nm = w + oT1;          // 6x6
    double* V = w + oT1 + 64;
    double* D = w + oT1 + 128;
    double* VD = w + oT1 + 192;
    double* zb = w + oT2;
    const Mat<kZ, 1> mean = dyn::observe(xtrue);
    if (lane < kZ * kZ) Nm[lane] = a.Nz[lane];
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < kZ; ++k) zb[8 + k] = mean.e[k];
    sync();
    jacobi<kZ>(Nm, V, D, lane, prof);
    if (lane < kZ) D[lane * (kZ + 1)] = sqrt(D[lane * (kZ + 1)]);
    sync();
    if (lane < kZ * kZ) {   // V D
      const int i = lane / kZ, j = lane % kZ;
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < kZ; ++k) acc += V[i * kZ + k] * D[k * kZ + j];
      VD[lane] = acc;
    }
    sync();
    if (lane < kZ) {        // (V D) smp + mean
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < kZ; ++k) acc += VD[lane * kZ + k] * a.normals[kX + k];
      zb[lane] = acc + zb[8 + lane];
    }
    sync();
#pragma unroll
    for (int k = 0; k < kZ; ++k) z.e[k] = zb[k];
    sync();
  }
  pf.stamp(5);
  kalman_update(q, x, R, z, a.Nz, w, lane);                                           // kalmanFilter2
  pf.stamp(6);
  const Vec3 vn = dyn::control_position(x, R, get<3, 1>(a.p_goal), ug, get<kV, kX>(a.Lh),
                                        get<kV, kV>(a.Eh));                           // findVGoal
#pragma unroll
  for (int t = 0; t < 4; ++t) P_[lane + 64 * t] = w[oP + lane + 64 * t];
  if (lane == 0) {
    synth::put(x_, x); synth::put(rot_, R);
    synth::put(xt_, xtrue); synth::put(rott_, Rtrue);
    synth::put(vgoal_, vn);
    synth::put(u_out, u);
    dyn::keyframe(a.keyframe, a.time, xtrue, Rtrue);                                  // visualize
  }
  pf.stamp(7);
  if (prof && lane == 0) atomicAdd(&prof[15], 1ull);
}

}  // namespace dynw
}  // namespace lqro
