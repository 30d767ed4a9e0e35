// lqro_synth.hpp — controlMatrices (LQRObstacles.cpp:520-582) with
// linearizeDiscretize (:456-471), f (:368-397), Jacobian_fx/fu (:421-441) and
// the matrix semantics they rely on (include/matrix.h: operator* :218-231,
// operator! :603-671, operator% :370-442, exp :763-790), written once for the
// host (lqro_synthesize_gains: one agent type) and for the device (k_synth in
// lqro_runtime.hip: one agent per lane, lqro_synthesize_gains_batch for swarms
// of heterogeneous agents).
//
// Every rounding happens where the reference's does: the library is compiled
// with -ffp-contract=off, products accumulate from 0.0 in k order, expression
// chains associate left to right.  The transcendental calls cannot move a
// result bit: log in exp's scaling exponent only selects an integer, and tan in
// f is reached at a rotation error of j_step where it multiplies a zero body
// rate.  So host and device agree bit for bit (tests/test_gpu_synth.py).
#pragma once
#include <cfloat>
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/lqro.h"

#define LQRO_HD __host__ __device__ inline

namespace lqro {
namespace synth {

template <int R, int C>
struct Mat {
  double e[R * C];
  LQRO_HD double& operator()(int r, int c) { return e[r * C + c]; }
  LQRO_HD double operator()(int r, int c) const { return e[r * C + c]; }
  static LQRO_HD Mat zero() {
    Mat m;
    for (int i = 0; i < R * C; ++i) m.e[i] = 0.0;
    return m;
  }
};
template <int N>
LQRO_HD Mat<N, N> eye() {
  Mat<N, N> m;
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) m(i, j) = (i == j ? 1.0 : 0.0);
  return m;
}
template <int R, int K, int C>
LQRO_HD Mat<R, C> operator*(const Mat<R, K>& a, const Mat<K, C>& b) {
  Mat<R, C> m;
  for (int i = 0; i < R; ++i)
    for (int j = 0; j < C; ++j) {
      double acc = 0.0;
      for (int k = 0; k < K; ++k) acc += a(i, k) * b(k, j);
      m(i, j) = acc;
    }
  return m;
}
template <int R, int C>
LQRO_HD Mat<R, C> operator+(const Mat<R, C>& a, const Mat<R, C>& b) {
  Mat<R, C> m;
  for (int i = 0; i < R * C; ++i) m.e[i] = a.e[i] + b.e[i];
  return m;
}
template <int R, int C>
LQRO_HD Mat<R, C> operator-(const Mat<R, C>& a, const Mat<R, C>& b) {
  Mat<R, C> m;
  for (int i = 0; i < R * C; ++i) m.e[i] = a.e[i] - b.e[i];
  return m;
}
template <int R, int C>
LQRO_HD Mat<R, C> operator-(const Mat<R, C>& a) {
  Mat<R, C> m;
  for (int i = 0; i < R * C; ++i) m.e[i] = -a.e[i];
  return m;
}
// matrix*scalar and scalar*matrix both evaluate elem*s in the reference
template <int R, int C>
LQRO_HD Mat<R, C> operator*(const Mat<R, C>& a, double s) {
  Mat<R, C> m;
  for (int i = 0; i < R * C; ++i) m.e[i] = a.e[i] * s;
  return m;
}
template <int R, int C>
LQRO_HD Mat<R, C> operator*(double s, const Mat<R, C>& a) { return a * s; }
template <int R, int C>
LQRO_HD Mat<R, C> operator/(const Mat<R, C>& a, double s) {
  Mat<R, C> m;
  for (int i = 0; i < R * C; ++i) m.e[i] = a.e[i] / s;
  return m;
}
template <int R, int C>
LQRO_HD Mat<C, R> tr(const Mat<R, C>& a) {
  Mat<C, R> m;
  for (int i = 0; i < C; ++i)
    for (int j = 0; j < R; ++j) m(i, j) = a(j, i);
  return m;
}

// ---- the pivoted small matrices without indexed storage (N <= 4) ----
// The reference's full-pivot routines reach rows and columns through the
// pivot permutations rp, cp (m(rp[i], cp[j])).  On the device a run-time
// index into a per-lane array is private (scratch) memory: the 3x3
// exponentials of f, the rotation resets and controllers and the 3x3 / 4x4
// inverses ran through it in every lane of k_dynw.  For N <= 4 the routines
// below keep the matrix in its pivoted order instead (M[i][j] = m(rp[i],
// cp[j])) and move rows and columns with selects; every arithmetic operation
// takes the operands the indexed version gives it, in the same order, so the
// results are bit-identical (tests/test_host_abi.py::test_small_pivot_routines
// checks them against the indexed versions, kept as inverse_ix / solve_ix).
// The permutations themselves are packed 4 bits an entry into one integer:
// the compiler turned select chains over a 3-int array back into an indexed
// load, which put the array in scratch again (k_dynw's resets).
template <int N>
struct SmIx {
  static_assert(N <= 8, "4 bits an entry");
  unsigned v = 0u;
  LQRO_HD int operator[](int i) const { return (int)((v >> (4 * i)) & 15u); }
  LQRO_HD void set(int i, int x) { v = (v & ~(15u << (4 * i))) | ((unsigned)x << (4 * i)); }
};
template <int N>
LQRO_HD int sm_get(const SmIx<N>& a, int k) {
  return a[k];
}
// the first strict maximum of |M[i][j]|, i, j >= k, in (row, col) order
template <int N>
LQRO_HD void sm_pivot(const double (&M)[N][N], int k, int& br, int& bc) {
  double best = 0.0;
  br = k;
  bc = k;
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (i >= k && j >= k) {
        const double a = fabs(M[i][j]);
        if (a > best) { best = a; br = i; bc = j; }
      }
}
// swap rows k and r (r >= k run-time) of an N x C array
template <int N, int C>
LQRO_HD void sm_swap_rows(double (&M)[N][C], int k, int r) {
#pragma unroll
  for (int t = 0; t < N; ++t)
    if (t > k) {
      const bool s = r == t;
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const double a = M[k][j], b = M[t][j];
        M[k][j] = s ? b : a;
        M[t][j] = s ? a : b;
      }
    }
}
template <int N, int C>
LQRO_HD void sm_swap_cols(double (&M)[N][C], int k, int c) {
#pragma unroll
  for (int t = 0; t < C; ++t)
    if (t > k) {
      const bool s = c == t;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const double a = M[i][k], b = M[i][t];
        M[i][k] = s ? b : a;
        M[i][t] = s ? a : b;
      }
    }
}
template <int N>
LQRO_HD void sm_swap_ix(SmIx<N>& a, int k, int r) {
  const int ak = a[k], ar = a[r];
  a.set(r, ak);
  a.set(k, ar);
}

// P X = Q (operator%, MAT:370-442) for N <= 4; = solve_ix below
template <int N, int C>
LQRO_HD Mat<N, C> solve_sm(const Mat<N, N>& p, const Mat<N, C>& q) {
  double M[N][N], X[N][C];   // M[i][j] = m(rp[i], cp[j]), X[i][j] = x(rp[i], j)
  SmIx<N> rp, cp;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    rp.set(i, i);
    cp.set(i, i);
#pragma unroll
    for (int j = 0; j < N; ++j) M[i][j] = p(i, j);
#pragma unroll
    for (int j = 0; j < C; ++j) X[i][j] = q(i, j);
  }
#pragma unroll
  for (int k = 0; k < N; ++k) {
    int br, bc;
    sm_pivot<N>(M, k, br, bc);
    sm_swap_rows<N, N>(M, k, br);
    sm_swap_rows<N, C>(X, k, br);
    sm_swap_ix<N>(rp, k, br);
    sm_swap_cols<N, N>(M, k, bc);
    sm_swap_ix<N>(cp, k, bc);
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      const double f = M[i][k] / M[k][k];
#pragma unroll
      for (int j = k + 1; j < N; ++j) M[i][j] -= f * M[k][j];
#pragma unroll
      for (int j = 0; j < C; ++j) X[i][j] -= f * X[k][j];
    }
  }
#pragma unroll
  for (int k = N - 1; k >= 0; --k) {
    const double qk = M[k][k];
#pragma unroll
    for (int j = 0; j < C; ++j) X[k][j] /= qk;
#pragma unroll
    for (int i = 0; i < k; ++i) {
      const double f = M[i][k];
#pragma unroll
      for (int j = 0; j < C; ++j) X[i][j] -= f * X[k][j];
    }
  }
  // the reference's final reshuffle on the physical rows x(r) = X[l], rp[l] = r
  double Y[N][C];
  SmIx<N> irp;
#pragma unroll
  for (int r = 0; r < N; ++r) {
#pragma unroll
    for (int j = 0; j < C; ++j) Y[r][j] = 0.0;
  }
#pragma unroll
  for (int l = 0; l < N; ++l)
#pragma unroll
    for (int r = 0; r < N; ++r) {   // (selects, not branches: the arrays stay in registers)
      const bool hit = rp[l] == r;
      if (hit) irp.set(r, l);
#pragma unroll
      for (int j = 0; j < C; ++j) Y[r][j] = hit ? X[l][j] : Y[r][j];
    }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int a = cp[i], b = rp[i];
#pragma unroll
    for (int j = 0; j < C; ++j) {
      double ya = Y[0][j], yb = Y[0][j];
#pragma unroll
      for (int r = 1; r < N; ++r) { ya = a == r ? Y[r][j] : ya; yb = b == r ? Y[r][j] : yb; }
      // x(a) = x(b), then x(b) = the old x(a) (a == b: unchanged)
#pragma unroll
      for (int r = 0; r < N; ++r) Y[r][j] = r == b ? ya : (r == a ? yb : Y[r][j]);
    }
    const int ia = sm_get(irp, a);
    // rp[irp[cp[i]]] = rp[i]; irp[rp[i]] = irp[cp[i]]
    rp.set(ia, b);
    irp.set(b, ia);
  }
  Mat<N, C> out;
#pragma unroll
  for (int r = 0; r < N; ++r)
#pragma unroll
    for (int j = 0; j < C; ++j) out(r, j) = Y[r][j];
  return out;
}

// operator! (MAT:603-671) for N <= 4; = inverse_ix below.  inv(rp[i], rp[j])
// is held as I[i][j] while the rows are eliminated (a row swap of rp swaps
// its rows and columns), inv(rp[i], j) as J[i][j] during back substitution.
template <int N>
LQRO_HD Mat<N, N> inverse_sm(const Mat<N, N>& q) {
  double M[N][N], I[N][N];
  SmIx<N> rp, cp;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    rp.set(i, i);
    cp.set(i, i);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      M[i][j] = q(i, j);
      I[i][j] = i == j ? 1.0 : 0.0;
    }
  }
#pragma unroll
  for (int k = 0; k < N; ++k) {
    int br, bc;
    sm_pivot<N>(M, k, br, bc);
    sm_swap_rows<N, N>(M, k, br);
    sm_swap_rows<N, N>(I, k, br);
    sm_swap_cols<N, N>(I, k, br);
    sm_swap_ix<N>(rp, k, br);
    sm_swap_cols<N, N>(M, k, bc);
    sm_swap_ix<N>(cp, k, bc);
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      const double f = M[i][k] / M[k][k];
#pragma unroll
      for (int j = k + 1; j < N; ++j) M[i][j] -= f * M[k][j];
#pragma unroll
      for (int j = 0; j < k; ++j) I[i][j] -= f * I[k][j];
      I[i][k] = -f;
    }
  }
  // J[i][c] = inv(rp[i], c) = I[i][l] with rp[l] = c
  double J[N][N];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int c = 0; c < N; ++c) {
      double v = I[i][0];
#pragma unroll
      for (int l = 1; l < N; ++l) v = rp[l] == c ? I[i][l] : v;
      J[i][c] = v;
    }
#pragma unroll
  for (int k = N - 1; k >= 0; --k) {
    const double qk = M[k][k];
#pragma unroll
    for (int j = 0; j < N; ++j) J[k][j] /= qk;
#pragma unroll
    for (int i = 0; i < k; ++i) {
      const double f = M[i][k];
#pragma unroll
      for (int j = 0; j < N; ++j) J[i][j] -= f * J[k][j];
    }
  }
  // m(cp[i], j) = inv(rp[i], j)
  Mat<N, N> out;
#pragma unroll
  for (int r = 0; r < N; ++r)
#pragma unroll
    for (int j = 0; j < N; ++j) {
      double v = J[0][j];
#pragma unroll
      for (int i = 1; i < N; ++i) v = cp[i] == r ? J[i][j] : v;
      out(r, j) = v;
    }
  return out;
}

// full-pivot Gauss-Jordan, pivot = first strict maximum in (row, col) scan order
template <int N>
LQRO_HD Mat<N, N> inverse_ix(const Mat<N, N>& q) {
  Mat<N, N> m = q, inv = eye<N>();
  int rp[N], cp[N];
  for (int i = 0; i < N; ++i) rp[i] = cp[i] = i;
  for (int k = 0; k < N; ++k) {
    double best = 0.0;
    int br = k, bc = k;
    for (int i = k; i < N; ++i)
      for (int j = k; j < N; ++j) {
        double a = fabs(m(rp[i], cp[j]));
        if (a > best) { best = a; br = i; bc = j; }
      }
    int t = rp[k]; rp[k] = rp[br]; rp[br] = t;
    t = cp[k]; cp[k] = cp[bc]; cp[bc] = t;
    for (int i = k + 1; i < N; ++i) {
      double f = m(rp[i], cp[k]) / m(rp[k], cp[k]);
      for (int j = k + 1; j < N; ++j) m(rp[i], cp[j]) -= f * m(rp[k], cp[j]);
      for (int j = 0; j < k; ++j) inv(rp[i], rp[j]) -= f * inv(rp[k], rp[j]);
      inv(rp[i], rp[k]) = -f;
    }
  }
  for (int k = N - 1; k >= 0; --k) {
    double qk = m(rp[k], cp[k]);
    for (int j = 0; j < N; ++j) inv(rp[k], j) /= qk;
    for (int i = 0; i < k; ++i) {
      double f = m(rp[i], cp[k]);
      for (int j = 0; j < N; ++j) inv(rp[i], j) -= f * inv(rp[k], j);
    }
  }
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) m(cp[i], j) = inv(rp[i], j);
  return m;
}

// P X = Q by full-pivot elimination with the reference's final reshuffle
template <int N, int C>
LQRO_HD Mat<N, C> solve_ix(const Mat<N, N>& p, const Mat<N, C>& q) {
  Mat<N, N> m = p;
  Mat<N, C> x = q;
  int rp[N], cp[N], irp[N];
  for (int i = 0; i < N; ++i) rp[i] = cp[i] = i;
  for (int k = 0; k < N; ++k) {
    double best = 0.0;
    int br = k, bc = k;
    for (int i = k; i < N; ++i)
      for (int j = k; j < N; ++j) {
        double a = fabs(m(rp[i], cp[j]));
        if (a > best) { best = a; br = i; bc = j; }
      }
    int t = rp[k]; rp[k] = rp[br]; rp[br] = t;
    t = cp[k]; cp[k] = cp[bc]; cp[bc] = t;
    for (int i = k + 1; i < N; ++i) {
      double f = m(rp[i], cp[k]) / m(rp[k], cp[k]);
      for (int j = k + 1; j < N; ++j) m(rp[i], cp[j]) -= f * m(rp[k], cp[j]);
      for (int j = 0; j < C; ++j) x(rp[i], j) -= f * x(rp[k], j);
    }
  }
  for (int k = N - 1; k >= 0; --k) {
    double qk = m(rp[k], cp[k]);
    for (int j = 0; j < C; ++j) x(rp[k], j) /= qk;
    for (int i = 0; i < k; ++i) {
      double f = m(rp[i], cp[k]);
      for (int j = 0; j < C; ++j) x(rp[i], j) -= f * x(rp[k], j);
    }
  }
  for (int i = 0; i < N; ++i) irp[rp[i]] = i;
  for (int i = 0; i < N; ++i) {
    for (int j = 0; j < C; ++j) {
      double t = x(cp[i], j);
      x(cp[i], j) = x(rp[i], j);
      x(rp[i], j) = t;
    }
    rp[irp[cp[i]]] = rp[i];
    irp[rp[i]] = irp[cp[i]];
  }
  return x;
}

template <int N>
LQRO_HD Mat<N, N> inverse(const Mat<N, N>& q) {
  if constexpr (N <= 4) return inverse_sm<N>(q);
  else return inverse_ix<N>(q);
}
template <int N, int C>
LQRO_HD Mat<N, C> solve(const Mat<N, N>& p, const Mat<N, C>& q) {
  if constexpr (N <= 4) return solve_sm<N, C>(p, q);
  else return solve_ix<N, C>(p, q);
}

template <int N>
LQRO_HD double norm1(const Mat<N, N>& q) {
  double best = 0.0;
  for (int j = 0; j < N; ++j) {
    double s = 0.0;
    for (int i = 0; i < N; ++i) s += fabs(q(i, j));
    if (s > best) best = s;
  }
  return best;
}

// degree-7 Pade with scaling and squaring (MAT:763-790)
template <int N>
LQRO_HD Mat<N, N> expm(const Mat<N, N>& q) {
  const double b0 = 1729728e1, b1 = 864864e1, b2 = 199584e1, b3 = 2772e2, b4 = 252e2,
               b5 = 1512e0, b6 = 56e0, b7 = 1e0, lim = 9.504178996162932e-1;
  Mat<N, N> A = q;
  double c = ceil(log(norm1(A) / lim) * M_LOG2E);
  int s = (int)(0.0 < c ? c : 0.0);
  double p2 = pow(2.0, s);
  for (int i = 0; i < N * N; ++i) A.e[i] /= p2;
  Mat<N, N> A2 = A * A, A4 = A2 * A2, A6 = A2 * A4, I = eye<N>();
  Mat<N, N> U = A * (A6 * b7 + A4 * b5 + A2 * b3 + I * b1);
  Mat<N, N> V = A6 * b6 + A4 * b4 + A2 * b2 + I * b0;
  Mat<N, N> R = solve(V - U, V + U);
  for (int i = 0; i < s; ++i) R = R * R;
  return R;
}

// jacobi2 (MAT:887-1037): Householder tridiagonalisation + QL iteration, the
// reference's eigen-decomposition of a symmetric matrix (Numerical Recipes;
// no eigenvalue sort).  z = eigenvectors (columns), D = diag(eigenvalues).
template <int N>
LQRO_HD void jacobi2(const Mat<N, N>& q, Mat<N, N>& z, Mat<N, N>& D) {
  z = q;
  double d[N], e[N];
  for (int i = 0; i < N; ++i) d[i] = e[i] = 0.0;
  int l, k, j, i, m, iter;
  double scale, hh, h, g, f, s, r, p, dd, c, b, absf, absg, pfg;
  for (i = N - 1; i > 0; i--) {
    l = i - 1;
    h = scale = 0.0;
    if (l > 0) {
      for (k = 0; k < i; k++) scale += fabs(z(i, k));
      if (scale == 0.0)
        e[i] = z(i, l);
      else {
        for (k = 0; k < i; k++) {
          z(i, k) /= scale;
          h += z(i, k) * z(i, k);
        }
        f = z(i, l);
        g = (f >= 0.0 ? -sqrt(h) : sqrt(h));
        e[i] = scale * g;
        h -= f * g;
        z(i, l) = f - g;
        f = 0.0;
        for (j = 0; j < i; j++) {
          z(j, i) = z(i, j) / h;
          g = 0.0;
          for (k = 0; k < j + 1; k++) g += z(j, k) * z(i, k);
          for (k = j + 1; k < i; k++) g += z(k, j) * z(i, k);
          e[j] = g / h;
          f += e[j] * z(i, j);
        }
        hh = f / (h + h);
        for (j = 0; j < i; j++) {
          f = z(i, j);
          e[j] = g = e[j] - hh * f;
          for (k = 0; k < j + 1; k++) z(j, k) -= (f * e[k] + g * z(i, k));
        }
      }
    } else {
      e[i] = z(i, l);
    }
    d[i] = h;
  }
  d[0] = 0.0;
  e[0] = 0.0;
  for (i = 0; i < N; i++) {
    if (d[i] != 0.0) {
      for (j = 0; j < i; j++) {
        g = 0.0;
        for (k = 0; k < i; k++) g += z(i, k) * z(k, j);
        for (k = 0; k < i; k++) z(k, j) -= g * z(k, i);
      }
    }
    d[i] = z(i, i);
    z(i, i) = 1.0;
    for (j = 0; j < i; j++) z(j, i) = z(i, j) = 0.0;
  }
  for (i = 1; i < N; i++) e[i - 1] = e[i];
  e[N - 1] = 0.0;
  for (l = 0; l < N; l++) {
    iter = 0;
    do {
      for (m = l; m < N - 1; m++) {
        dd = fabs(d[m]) + fabs(d[m + 1]);
        if (fabs(e[m]) <= DBL_EPSILON * dd) break;
      }
      if (m != l) {
        if (iter++ == 30) break;   // the reference prints "Too many iterations" and exits
        g = (d[l + 1] - d[l]) / (2.0 * e[l]);
        absg = fabs(g);
        r = ((absg > 1.0) ? absg * sqrt(1.0 + (1.0 / absg) * (1.0 / absg)) : sqrt(1.0 + absg * absg));
        g = d[m] - d[l] + e[l] / (g + ((g >= 0.0) ? fabs(r) : -fabs(r)));
        s = c = 1.0;
        p = 0.0;
        for (i = m - 1; i >= l; i--) {
          f = s * e[i];
          b = c * e[i];
          absf = fabs(f);
          absg = fabs(g);
          pfg = (absf > absg ? absf * sqrt(1.0 + (absg / absf) * (absg / absf))
                             : (absg == 0.0 ? 0.0 : absg * sqrt(1.0 + (absf / absg) * (absf / absg))));
          e[i + 1] = (r = pfg);
          if (r == 0.0) {
            d[i + 1] -= p;
            e[m] = 0.0;
            break;
          }
          s = f / r;
          c = g / r;
          g = d[i + 1] - p;
          r = (d[i] - g) * s + 2.0 * c * b;
          d[i + 1] = g + (p = s * r);
          g = c * r - b;
          for (k = 0; k < N; k++) {
            f = z(k, i + 1);
            z(k, i + 1) = s * z(k, i) + c * f;
            z(k, i) = c * z(k, i) - s * f;
          }
        }
        if (r == 0.0 && i >= l) continue;
        d[l] -= p;
        e[l] = g;
        e[m] = 0.0;
      }
    } while (m != l);
  }
  D = Mat<N, N>::zero();
  for (i = 0; i < N; ++i) D(i, i) = d[i];
}

// pseudoInverse (MAT:450-477) of a square matrix (the _numColumns <=
// _numRows branch): (Vec Val^+ Vec^T) q^T with jacobi2(q^T q)
template <int N>
LQRO_HD Mat<N, N> pseudo_inverse(const Mat<N, N>& q) {
  Mat<N, N> Vec, Val;
  jacobi2<N>(tr(q) * q, Vec, Val);
  for (int i = 0; i < N; ++i) {
    if (fabs(Val(i, i)) <= sqrt(DBL_EPSILON)) Val(i, i) = 0.0;
    else Val(i, i) = 1.0 / Val(i, i);
  }
  return (Vec * Val * tr(Vec)) * tr(q);
}

typedef Mat<3, 1> Vec3;
LQRO_HD Mat<3, 3> skew(const Vec3& v) {
  Mat<3, 3> m = Mat<3, 3>::zero();
  m(0, 1) = -v.e[2]; m(0, 2) = v.e[1];
  m(1, 0) = v.e[2];  m(1, 2) = -v.e[0];
  m(2, 0) = -v.e[1]; m(2, 1) = v.e[0];
  return m;
}
LQRO_HD double hypot3(const Vec3& v) {
  double X = fabs(v.e[0]), Y = fabs(v.e[1]), Z = fabs(v.e[2]);
  if (X > Y && X > Z) return X * sqrt(1.0 + (Y / X) * (Y / X) + (Z / X) * (Z / X));
  if (Y > Z) return Y * sqrt(1.0 + (X / Y) * (X / Y) + (Z / Y) * (Z / Y));
  return Z * sqrt(1.0 + (X / Z) * (X / Z) + (Y / Z) * (Y / Z));
}

struct Quad {
  double dt, g, mass, kM, lat, arm, h;
  Mat<3, 3> J, Jinv;
};

// hover dynamics x' = f(x, R, u) (LQRO:368-397).  X = 16: the reference's
// quadrotor (position, velocity, rotation error, body rates, rotor forces
// with first-order lag (u - F) * thrust_latency).  X = 12: the reduced model
// of BASELINE config 5 — the 4 rotor-force states dropped, the
// rotors follow their command at once (F = u); every other term as X = 16.
template <int X>
LQRO_HD Mat<X, 1> dynamics(const Quad& q, const Mat<X, 1>& x, const Mat<3, 3>& R, const Mat<4, 1>& u) {
  static_assert(X == 16 || X == 12, "x_dim is 16 or 12");
  Vec3 eX = Vec3::zero(), eY = Vec3::zero(), eZ = Vec3::zero();
  eX.e[0] = 1; eY.e[1] = 1; eZ.e[2] = 1;
  Vec3 v, r, w;
  double F[4];
  for (int k = 0; k < 3; ++k) { v.e[k] = x.e[3 + k]; r.e[k] = x.e[6 + k]; w.e[k] = x.e[9 + k]; }
  for (int k = 0; k < 4; ++k) F[k] = X == 16 ? x.e[(12 + k) % X] : u.e[k];
  Mat<X, 1> xd;
  for (int k = 0; k < 3; ++k) xd.e[k] = v.e[k];
  Vec3 acc = -q.g * eZ + R * expm(skew(r)) * ((F[0] + F[1] + F[2] + F[3]) / q.mass) * eZ;
  for (int k = 0; k < 3; ++k) xd.e[3 + k] = acc.e[k];
  double l = hypot3(r);
  Vec3 rd;
  if (0.5 * l > 0.0)
    rd = w + 0.5 * skew(r) * w + (1.0 - 0.5 * l / tan(0.5 * l)) * skew(r / l) * (skew(r / l) * w);
  else
    rd = w + 0.5 * skew(r) * w;
  for (int k = 0; k < 3; ++k) xd.e[6 + k] = rd.e[k];
  Vec3 wd = q.Jinv * (q.arm * (F[1] - F[3]) * eX + q.arm * (F[2] - F[0]) * eY +
                      (F[0] - F[1] + F[2] - F[3]) * q.kM * eZ - skew(w) * q.J * w);
  for (int k = 0; k < 3; ++k) xd.e[9 + k] = wd.e[k];
  if (X == 16)
    for (int k = 0; k < 4; ++k) xd.e[(12 + k) % X] = (u.e[k] - F[k]) * q.lat;
  return xd;
}

template <int R, int C>
LQRO_HD void put(double* out, const Mat<R, C>& m) {
  if (out)
#pragma unroll
    for (int i = 0; i < R * C; ++i) out[i] = m.e[i];
}

// l of controlMatrices (LQRO:552, 557), with S the converged velocity-LQR
// Riccati matrix and xstar = xGoal (hover; Qx = 0 makes Qx*xstar zero):
//   a = pseudoInverse(~A - ~A*S*B*!(R+~B*S*B)*~B - I)
//         * (Qx*xstar - ~A*S*c + ~A*S*B*!(R+~B*S*B)*~B*S*c)
//   l = -!(R+~B*S*B) * (~B*S*c + ~B*a)
// (exactly 0 for the reference's model, whose hover point has c = 0)
template <int X>
LQRO_HD Mat<4, 1> ell(const Mat<X, X>& A, const Mat<X, 4>& B, const Mat<X, 1>& c, const Mat<X, X>& S,
                      const Mat<4, 4>& Rw, const Mat<X, 1>& xstar) {
  const Mat<X, X> At = tr(A), Qx = Mat<X, X>::zero();
  const Mat<4, X> Bt = tr(B);
  const Mat<X, X> M1 = At - At * S * B * inverse(Rw + Bt * S * B) * Bt - eye<X>();
  const Mat<X, 1> v1 = Qx * xstar - At * S * c + At * S * B * inverse(Rw + Bt * S * B) * Bt * S * c;
  const Mat<X, 1> a = pseudo_inverse<X>(M1) * v1;
  return -inverse(Rw + Bt * S * B) * (Bt * S * c + Bt * a);
}

// controlMatrices for one agent's model: A (X*X), B (X*U), c (X), L (U*X),
// E (U*3), Lh (3*X), Eh (3*3); any output may be null.  X = 12: the reduced
// model above, linearised at the same hover point.
template <int X>
LQRO_HD void gains_x(const lqro_model* md, double* Ao, double* Bo, double* co, double* Lo, double* Eo,
                     double* Lho, double* Eho, double* lo = nullptr) {
  Quad q;
  q.dt = md->dt; q.g = md->gravity; q.mass = md->mass; q.kM = md->moment_const;
  q.lat = md->thrust_latency; q.arm = md->length; q.h = md->j_step;
  q.J = md->inertia * eye<3>();
  q.Jinv = inverse(q.J);
  const double hover = q.g * q.mass / 4;
  Mat<4, 1> u0;
  for (int k = 0; k < 4; ++k) u0.e[k] = hover;
  Mat<X, 1> x0 = Mat<X, 1>::zero();
  for (int k = 12; k < X; ++k) x0.e[k] = hover;
  Mat<3, 3> R0 = eye<3>();

  // central-difference Jacobians, then A = e^{F dt}, B/c by Simpson's rule
  Mat<X, X> F;
  Mat<X, 4> G;
  {
    Mat<X, 1> xr = x0, xl = x0;
    for (int i = 0; i < X; ++i) {
      xr.e[i] += q.h; xl.e[i] -= q.h;
      Mat<X, 1> col = (dynamics<X>(q, xr, R0, u0) - dynamics<X>(q, xl, R0, u0)) / (2 * q.h);
      for (int k = 0; k < X; ++k) F(k, i) = col.e[k];
      xr.e[i] = xl.e[i] = x0.e[i];
    }
    Mat<4, 1> ur = u0, ul = u0;
    for (int i = 0; i < 4; ++i) {
      ur.e[i] += q.h; ul.e[i] -= q.h;
      Mat<X, 1> col = (dynamics<X>(q, x0, R0, ur) - dynamics<X>(q, x0, R0, ul)) / (2 * q.h);
      for (int k = 0; k < X; ++k) G(k, i) = col.e[k];
      ur.e[i] = ul.e[i] = u0.e[i];
    }
  }
  Mat<X, 1> xdot = dynamics<X>(q, x0, R0, u0);
  Mat<X, X> A = expm(q.dt * F);
  Mat<X, X> Int = (q.dt / 6.0) * (eye<X>() + 4.0 * expm(0.5 * q.dt * F) + A);
  Mat<X, 4> B = Int * G;
  Mat<X, 1> c = Int * xdot;

  // velocity LQR: 300 Riccati sweeps with a velocity-tracking term
  Mat<3, X> Vs = Mat<3, X>::zero(), Ps = Mat<3, X>::zero();
  Vs(0, 3) = Vs(1, 4) = Vs(2, 5) = 1;
  Ps(0, 0) = Ps(1, 1) = Ps(2, 2) = 1;
  Mat<3, 3> Qv = md->qv * eye<3>(), Qp = md->qp * eye<3>();
  Mat<4, 4> Rw = md->r * eye<4>();
  Mat<X, X> Qx = Mat<X, X>::zero();
  Mat<X, X> At = tr(A);
  Mat<4, X> Bt = tr(B);
  Mat<X, 3> Vt = tr(Vs);
  Mat<X, X> S = Vt * Qv * Vs;
  Mat<X, 3> T = -Vt * Qv;
  for (int it = 0; it < 300; ++it) {
    Mat<X, 4> K = At * S * B * inverse(Rw + Bt * S * B);
    Mat<X, 3> Tn = -Vt * Qv + At * T - K * Bt * T;
    Mat<X, X> Sn = Vt * Qv * Vs + Qx + At * S * A - K * (Bt * S * A);
    T = Tn;
    S = Sn;
  }
  Mat<4, 4> Ri = inverse(Rw + Bt * S * B);
  Mat<4, X> L = -Ri * Bt * S * A;
  Mat<4, 3> E = -Ri * Bt * T;
  if (lo) put(lo, ell<X>(A, B, c, S, Rw, x0));

  // position LQR on the closed velocity loop, with the cross term
  const double wgt = md->pos_weight;
  Mat<X, X> Qpt = tr(Ps) * Qp * Ps + wgt * tr(L) * Rw * L;
  Mat<3, 3> Rt = wgt * tr(E) * Rw * E;
  Mat<3, X> Pt = wgt * tr(E) * Rw * L;
  Mat<X, X> Acl = A + B * L;
  Mat<X, 3> Bcl = B * E;
  Mat<X, X> Aclt = tr(Acl);
  Mat<3, X> Bclt = tr(Bcl);
  Mat<X, 3> Ptt = tr(Pt);
  Mat<X, X> St = Qpt;
  Mat<X, 3> Tt = -tr(Ps) * Qp;
  for (int it = 0; it < 300; ++it) {
    Mat<X, 3> K = (Ptt + Aclt * St * Bcl) * inverse(Rt + Bclt * St * Bcl);
    Mat<X, 3> Ttn = -tr(Ps) * Qp + Aclt * Tt - K * Bclt * Tt;
    Mat<X, X> Stn = Qpt + Aclt * St * Acl - K * (Pt + Bclt * St * Acl);
    Tt = Ttn;
    St = Stn;
  }
  Mat<3, 3> RRi = inverse(Rt + Bclt * St * Bcl);
  Mat<3, X> Lh = -RRi * (Pt + Bclt * St * Acl);
  Mat<3, 3> Eh = -RRi * (Bclt * Tt);

  put(Ao, A); put(Bo, B); put(co, c); put(Lo, L); put(Eo, E); put(Lho, Lh); put(Eho, Eh);
}

LQRO_HD void gains(const lqro_model* md, double* Ao, double* Bo, double* co, double* Lo, double* Eo,
                   double* Lho, double* Eho) {
  gains_x<16>(md, Ao, Bo, co, Lo, Eo, Lho, Eho);
}

}  // namespace synth
}  // namespace lqro
