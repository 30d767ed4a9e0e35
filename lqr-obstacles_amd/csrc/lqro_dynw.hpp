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

// C = A B (16x16x16), C distinct from A and B
__device__ __forceinline__ void mm(const double* A, const double* B, double* C, int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int e = lane + 64 * t, i = e >> 4, j = e & 15;
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += A[i * 16 + k] * B[k * 16 + j];
    C[e] = acc;
  }
  sync();
}
// C = A B^T
__device__ __forceinline__ void mm_nt(const double* A, const double* B, double* C, int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int e = lane + 64 * t, i = e >> 4, j = e & 15;
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += A[i * 16 + k] * B[j * 16 + k];
    C[e] = acc;
  }
  sync();
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
// (16-k)^2 block of the permuted matrix, as operator% / operator! pick it
template <int N = 16>
__device__ __forceinline__ void pivot(const double* m, const int* rp, const int* cp, int k, int lane,
                                      int& br, int& bc) {
  const int w = N - k;
  double best = 0.0;
  int bi = INT_MAX;
  for (int idx = lane; idx < w * w; idx += 64) {
    const int i = k + idx / w, j = k + idx % w;
    const double a = fabs(m[rp[i] * N + cp[j]]);
    if (a > best) { best = a; bi = idx; }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ob = __shfl_xor(best, off);
    const int oi = __shfl_xor(bi, off);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (bi == INT_MAX) { br = k; bc = k; }
  else { br = k + bi / w; bc = k + bi % w; }
}

// X = P^-1 Q by full pivoting with the reference's final reshuffle
// (operator%, MAT:370-442, = synth::solve): m (P) and x (Q) in LDS, both
// overwritten; the solution is left in x.
__device__ __forceinline__ void solve(double* m, double* x, int* ip, int lane) {
  int* rp = ip;
  int* cp = ip + 16;
  int* irp = ip + 32;
  if (lane < 16) { rp[lane] = lane; cp[lane] = lane; }
  sync();
  for (int k = 0; k < 16; ++k) {
    int br, bc;
    pivot(m, rp, cp, k, lane, br, bc);
    const int rk = rp[br], ck = cp[bc], rb = rp[k], cb = cp[k];
    sync();
    if (lane == 0) { rp[k] = rk; rp[br] = rb; cp[k] = ck; cp[bc] = cb; }
    sync();
    // rows i > k: m[rp i][cp j] (j > k) and x[rp i][*] against row k
    const int w = 15 - k;
    const double piv = m[rp[k] * 16 + cp[k]];
    for (int idx = lane; idx < w * (w + 16); idx += 64) {
      const int i = k + 1 + idx / (w + 16), c = idx % (w + 16);
      const double f = m[rp[i] * 16 + cp[k]] / piv;
      if (c < w) {
        const int j = k + 1 + c;
        m[rp[i] * 16 + cp[j]] -= f * m[rp[k] * 16 + cp[j]];
      } else {
        const int j = c - w;
        x[rp[i] * 16 + j] -= f * x[rp[k] * 16 + j];
      }
    }
    sync();
  }
  for (int k = 15; k >= 0; --k) {
    const double qk = m[rp[k] * 16 + cp[k]];
    if (lane < 16) x[rp[k] * 16 + lane] /= qk;
    sync();
    for (int idx = lane; idx < k * 16; idx += 64) {
      const int i = idx >> 4, j = idx & 15;
      const double f = m[rp[i] * 16 + cp[k]];
      x[rp[i] * 16 + j] -= f * x[rp[k] * 16 + j];
    }
    sync();
  }
  if (lane < 16) irp[rp[lane]] = lane;
  sync();
  for (int i = 0; i < 16; ++i) {
    const int ci = cp[i], ri = rp[i];
    if (lane < 16) {
      const double t = x[ci * 16 + lane];
      x[ci * 16 + lane] = x[ri * 16 + lane];
      x[ri * 16 + lane] = t;
    }
    sync();
    if (lane == 0) {
      const int a = irp[ci];
      rp[a] = ri;
      irp[ri] = a;
    }
    sync();
  }
}

// out = exp(q) (MAT:763-790, = synth::expm<16>); q and out may not alias the
// six work matrices E0..E5
__device__ __forceinline__ void expm(const double* q, double* out, double* w, int lane) {
  const double b0 = 1729728e1, b1 = 864864e1, b2 = 199584e1, b3 = 2772e2, b4 = 252e2, b5 = 1512e0,
               b6 = 56e0, b7 = 1e0, lim = 9.504178996162932e-1;
  double* A = w + oE0;
  double* A2 = w + oE1;
  double* A4 = w + oE2;
  double* A6 = w + oE3;
  double* U = w + oE4;
  double* V = w + oE5;
  int* ip = reinterpret_cast<int*>(w + oInt);
  // 1-norm: column sums in i order, the max of them (order-free)
  double cs = 0.0;
  if (lane < 16)
    for (int i = 0; i < 16; ++i) cs += fabs(q[i * 16 + lane]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) cs = fmax(cs, __shfl_xor(cs, off));
  const double c = ceil(log(cs / lim) * M_LOG2E);
  const int s = (int)(0.0 < c ? c : 0.0);
  const double p2 = pow(2.0, s);
#pragma unroll
  for (int t = 0; t < 4; ++t) A[lane + 64 * t] = q[lane + 64 * t] / p2;
  sync();
  mm(A, A, A2, lane);
  mm(A2, A2, A4, lane);
  mm(A2, A4, A6, lane);
  // V = A6 b6 + A4 b4 + A2 b2 + I b0 ; U <- A6 b7 + A4 b5 + A2 b3 + I b1 (then A U)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int e = lane + 64 * t;
    const double I = ((e >> 4) == (e & 15)) ? 1.0 : 0.0;
    V[e] = A6[e] * b6 + A4[e] * b4 + A2[e] * b2 + I * b0;
    U[e] = A6[e] * b7 + A4[e] * b5 + A2[e] * b3 + I * b1;
  }
  sync();
  mm(A, U, A2, lane);   // A2 <- U = A (..)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int e = lane + 64 * t;
    A4[e] = V[e] - A2[e];   // P = V - U
    A6[e] = V[e] + A2[e];   // Q = V + U
  }
  sync();
  solve(A4, A6, ip, lane);
  double* cur = A6;
  double* nxt = U;
  for (int i = 0; i < s; ++i) {
    mm(cur, cur, nxt, lane);
    double* t = cur; cur = nxt; nxt = t;
  }
  copy(cur, out, lane);
}

// jacobi (MAT:674-759, = dyn::jacobi<N>) of m: V, D in LDS (row stride N);
// the pivot scan in every lane, the rotation over lanes [0, N) (D) and
// [N, 2N) (V)
template <int N>
__device__ __forceinline__ void jacobi(const double* m, double* V, double* D, int lane) {
  for (int e = lane; e < N * N; e += 64) {
    D[e] = m[e];
    V[e] = (e / N == e % N) ? 1.0 : 0.0;
  }
  sync();
  int pivot = 0, zeros = 0;
  for (;;) {
    double maximum = 0;
    int p = 0, q = 0;
    for (int i = 0; i < pivot; ++i)
      if (fabs(D[i * N + pivot]) > maximum) { maximum = fabs(D[i * N + pivot]); p = i; q = pivot; }
    for (int j = pivot + 1; j < N; ++j)
      if (fabs(D[pivot * N + j]) > maximum) { maximum = fabs(D[pivot * N + j]); p = pivot; q = j; }
    pivot = (pivot + 1) % N;
    if (maximum <= DBL_EPSILON) {
      if (++zeros == N) break;
      continue;
    }
    zeros = 0;
    const double theta = 0.5 * (D[q * N + q] - D[p * N + p]) / D[p * N + q];
    double t = 1 / (fabs(theta) + hypot(theta, 1.0));
    if (theta < 0) t = -t;
    const double c = 1 / hypot(t, 1.0);
    const double s = c * t;
    const double tau = s / (1 + c);
    sync();   // every lane has read D for the scan
    if (lane < N && lane != p && lane != q) {
      const int r = lane;
      int ia, ib;   // the two entries row/col r of the rotation touches
      if (r < p) { ia = r * N + p; ib = r * N + q; }
      else if (r < q) { ia = p * N + r; ib = r * N + q; }
      else { ia = p * N + r; ib = q * N + r; }
      const double a = D[ia], b = D[ib];
      D[ia] -= s * (b + tau * a);
      D[ib] += s * (a - tau * b);
    }
    if (lane >= N && lane < 2 * N) {
      const int r = lane - N;
      const double a = V[r * N + p], b = V[r * N + q];
      V[r * N + p] -= s * (b + tau * a);
      V[r * N + q] += s * (a - tau * b);
    }
    sync();
    if (lane == 0) {
      D[p * N + p] -= t * D[p * N + q];
      D[q * N + q] += t * D[p * N + q];
      D[p * N + q] = 0;
    }
    sync();
  }
  for (int e = lane; e < N * N; e += 64)
    if (e / N != e % N) D[e] = 0;
  sync();
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
                                          const Mat<kU, 1>& u, double* w, int lane, Mat<kX, 1>& dx) {
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
  double* A = w + oA;
  double* A2 = w + oA2;
  double* T1 = w + oT1;
  double* T2 = w + oT2;
#pragma unroll
  for (int t = 0; t < 4; ++t) T1[lane + 64 * t] = q.dt * F[lane + 64 * t];
  sync();
  expm(T1, A, w, lane);
#pragma unroll
  for (int t = 0; t < 4; ++t) T1[lane + 64 * t] = (q.dt * 0.5) * F[lane + 64 * t];
  sync();
  expm(T1, A2, w, lane);
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
}

// sampleGaussian(0, MM, nrm) (simulator2.h:21-32) on the LDS matrix MM
__device__ __forceinline__ Mat<kX, 1> noise(double* w, const double* nrm, int lane) {
  double* V = w + oT1;
  double* D = w + oT2;
  jacobi<16>(w + oMM, V, D, lane);
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
                           double* P_, double* vgoal_, double* u_out, double* w, int lane) {
  using dyn::get;
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
  {                                                                                   // propagateU
    Mat<kX, 1> dx;
    discretize(q, xtrue, Rtrue, u, w, lane, dx);
    const Mat<kX, 1> g = noise(w, a.normals, lane);
    xtrue = xtrue + dx + g;
    dyn::reset_rot(xtrue, Rtrue);
  }
  {                                                                                   // kalmanFilter1
    Mat<kX, 1> dx;
    discretize(q, x, R, u, w, lane, dx);
    x = x + dx;
    double* P = w + oP;
    mm(w + oA, P, w + oT1, lane);
    mm_nt(w + oT1, w + oA, w + oT2, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t) P[lane + 64 * t] = w[oT2 + lane + 64 * t] + w[oMM + lane + 64 * t];
    sync();
    dyn::reset_rot(x, R);
  }
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
    jacobi<kZ>(Nm, V, D, lane);
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
  kalman_update(q, x, R, z, a.Nz, w, lane);                                           // kalmanFilter2
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
}

}  // namespace dynw
}  // namespace lqro
