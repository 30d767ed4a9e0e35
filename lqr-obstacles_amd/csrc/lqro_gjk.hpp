// lqro_gjk.hpp — gjk_distance (gjk.cpp:296-501, Cameron's Oxford GJK v2.4)
// specialised to the call the path makes (run_gjk, LQRObstacles.cpp:814-853):
// object 1 is the single point vrel (hill climbing on a one-vertex ring
// returns it), object 2 is the reachable point set with a brute-force
// support function (support_simple, gjk.cpp:770-794).
//
// The simplex bookkeeping runs redundantly in every lane (all values are
// wave-uniform); the support query is supplied by the caller and must return
// the lowest-index maximiser, which is what support_simple's strict '>' scan
// returns.  Johnson's sub-algorithm (compute_subterms, default_distance,
// backup_distance, reset_simplex: gjk.cpp:527-736) and the constant subset
// tables (gjk.cpp:86-160) are restated one-for-one.
#pragma once
#include <hip/hip_runtime.h>

namespace lqro {

__constant__ int g_card[16] = {0, 1, 1, 2, 1, 2, 2, 3, 1, 2, 2, 3, 2, 3, 3, 4};
__constant__ int g_maxe[16] = {-1, 0, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3};
__constant__ int g_elts[16][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {1, 0, 0, 0}, {0, 1, 0, 0},
                                  {2, 0, 0, 0}, {0, 2, 0, 0}, {1, 2, 0, 0}, {0, 1, 2, 0},
                                  {3, 0, 0, 0}, {0, 3, 0, 0}, {1, 3, 0, 0}, {0, 1, 3, 0},
                                  {2, 3, 0, 0}, {0, 2, 3, 0}, {1, 2, 3, 0}, {0, 1, 2, 3}};
__constant__ int g_nonelts[16][4] = {{0, 1, 2, 3}, {1, 2, 3, 0}, {0, 2, 3, 0}, {2, 3, 0, 0},
                                     {0, 1, 3, 0}, {1, 3, 0, 0}, {0, 3, 0, 0}, {3, 0, 0, 0},
                                     {0, 1, 2, 0}, {1, 2, 0, 0}, {0, 2, 0, 0}, {2, 0, 0, 0},
                                     {0, 1, 0, 0}, {1, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
__constant__ int g_pred[16][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {2, 1, 0, 0},
                                  {0, 0, 0, 0}, {4, 1, 0, 0}, {4, 2, 0, 0}, {6, 5, 3, 0},
                                  {0, 0, 0, 0}, {8, 1, 0, 0}, {8, 2, 0, 0}, {10, 9, 3, 0},
                                  {8, 4, 0, 0}, {12, 9, 5, 0}, {12, 10, 6, 0}, {14, 13, 11, 7}};
__constant__ int g_succ[16][4] = {{1, 2, 4, 8}, {3, 5, 9, 0}, {3, 6, 10, 0}, {7, 11, 0, 0},
                                  {5, 6, 12, 0}, {7, 13, 0, 0}, {7, 14, 0, 0}, {15, 0, 0, 0},
                                  {9, 10, 12, 0}, {11, 13, 0, 0}, {11, 14, 0, 0}, {15, 0, 0, 0},
                                  {13, 14, 0, 0}, {15, 0, 0, 0}, {15, 0, 0, 0}, {0, 0, 0, 0}};

struct GjkState {
  int npts;
  int s2[4];          // point ids (q = k*NP + p) of the hull-side simplex vertices
  double lambdas[4];
  double c1[4][3], c2[4][3];
  double dv[16][4];   // delta_values (gjk.cpp:163)
  double dp[4][4];    // dot_products (gjk.cpp:164)
  double dsum[16];    // delta (gjk.cpp:522)
};

struct GjkOut {
  double sqrd, w1[3], w2[3];
  int iters, backup;
};

__device__ inline void gjk_subterms(GjkState& g) {
  const int size = g.npts;
  double csp[4][3];
  for (int i = 0; i < size; i++)
    for (int j = 0; j < 3; j++) csp[i][j] = g.c1[i][j] - g.c2[i][j];
  for (int i = 0; i < size; i++)
    for (int j = i; j < size; j++)
      g.dp[i][j] = g.dp[j][i] = csp[i][0] * csp[j][0] + csp[i][1] * csp[j][1] + csp[i][2] * csp[j][2];
  for (int s = 1; s < 16 && g_maxe[s] < size; s++) {
    if (g_card[s] <= 1) { g.dv[s][g_elts[s][0]] = 1.0; continue; }
    if (g_card[s] == 2) {
      int e0 = g_elts[s][0], e1 = g_elts[s][1];
      g.dv[s][e0] = g.dp[e1][e1] - g.dp[e1][e0];
      g.dv[s][e1] = g.dp[e0][e0] - g.dp[e0][e1];
      continue;
    }
    for (int j = 0; j < g_card[s]; j++) {
      int jelt = g_elts[s][j], jsub = g_pred[s][j];
      double sum = 0;
      for (int i = 0; i < g_card[jsub]; i++) {
        int ielt = g_elts[jsub][i];
        sum += g.dv[jsub][ielt] * (g.dp[ielt][g_elts[jsub][0]] - g.dp[ielt][jelt]);
      }
      g.dv[s][jelt] = sum;
    }
  }
}

__device__ inline void gjk_reset(GjkState& g, int subset) {
  for (int j = 0; j < g_card[subset]; j++) {
    int oldpos = g_elts[subset][j];
    if (oldpos != j) {
      g.s2[j] = g.s2[oldpos];
      for (int i = 0; i < 3; i++) { g.c1[j][i] = g.c1[oldpos][i]; g.c2[j][i] = g.c2[oldpos][i]; }
    }
    g.lambdas[j] = g.dv[subset][g_elts[subset][j]] / g.dsum[subset];
  }
  g.npts = g_card[subset];
}

__device__ inline int gjk_default(GjkState& g) {
  int s, ok = 0, size = g.npts;
  for (s = 1; s < 16 && g_maxe[s] < size; s++) {
    g.dsum[s] = 0.0; ok = 1;
    for (int j = 0; ok && j < g_card[s]; j++) {
      if (g.dv[s][g_elts[s][j]] > 0.0) g.dsum[s] += g.dv[s][g_elts[s][j]];
      else ok = 0;
    }
    for (int k = 0; ok && k < size - g_card[s]; k++)
      if (g.dv[g_succ[s][k]][g_nonelts[s][k]] > 0) ok = 0;
    if (ok && g.dsum[s] >= 1.0e-20) break;
  }
  if (ok) { gjk_reset(g, s); return 1; }
  return 0;
}

__device__ inline void gjk_backup(GjkState& g) {
  int size = g.npts, bests = 0;
  double num[16], den[16];
  for (int s = 1; s < 16 && g_maxe[s] < size; s++) {
    if (g.dsum[s] <= 0.0) continue;
    int i;
    for (i = 0; i < g_card[s]; i++)
      if (g.dv[s][g_elts[s][i]] <= 0.0) break;
    if (i < g_card[s]) continue;
    num[s] = 0.0;
    for (int j = 0; j < g_card[s]; j++)
      for (int k = 0; k < g_card[s]; k++)
        num[s] += (g.dv[s][g_elts[s][j]] * g.dv[s][g_elts[s][k]]) * g.dp[g_elts[s][j]][g_elts[s][k]];
    den[s] = g.dsum[s] * g.dsum[s];
    if ((bests < 1) || (num[s] * den[bests] < num[bests] * den[s])) bests = s;
  }
  gjk_reset(g, bests);
}

__device__ __forceinline__ void gjk_point(double* pt, int len, const double (*v)[3], const double* lam) {
  for (int d = 0; d < 3; d++) {
    pt[d] = 0;
    for (int i = 0; i < len; i++) pt[d] += v[i][d] * lam[i];
  }
}

// Sup must provide:
//   void support(double d0, double d1, double d2, double& value, int& q)
//   void point(int q, double* pt)
template <class Sup>
__device__ void gjk_run(Sup& sup, int qfirst, int n, const double* vrel, GjkState& g, GjkOut& o) {
  for (int s = 0; s < 16; ++s) {
    g.dsum[s] = 0.0;
    for (int k = 0; k < 4; ++k) g.dv[s][k] = 0.0;
  }
  int use_default = 1, first_iteration = 1, max_iterations = n;
  double oldsqrd = 0.0, sqrd = 0.0;
  double disp[3], rdisp[3];
  o.iters = 0; o.backup = 0;
  g.npts = 1; g.s2[0] = qfirst; g.lambdas[0] = 1.0;
  {
    double f[3];
    sup.point(qfirst, f);
    for (int d = 0; d < 3; d++) { g.c1[0][d] = vrel[d]; g.c2[0][d] = f[d]; }
  }
  while (max_iterations-- > 0) {
    if (g.npts == 1) g.lambdas[0] = 1.0;
    else {
      gjk_subterms(g);
      if (use_default) use_default = gjk_default(g);
      if (!use_default) { gjk_backup(g); o.backup = 1; }
    }
    gjk_point(o.w1, g.npts, g.c1, g.lambdas);
    gjk_point(o.w2, g.npts, g.c2, g.lambdas);
    for (int d = 0; d < 3; d++) { disp[d] = o.w2[d] - o.w1[d]; rdisp[d] = -disp[d]; }
    sqrd = disp[0] * disp[0] + disp[1] * disp[1] + disp[2] * disp[2];
    if (sqrd < 1.0e-8) { o.sqrd = sqrd; return; }
    const double maxv = vrel[0] * disp[0] + vrel[1] * disp[1] + vrel[2] * disp[2];
    double minus_minv;
    int minq;
    sup.support(rdisp[0], rdisp[1], rdisp[2], minus_minv, minq);
    o.iters++;
    double g_val = sqrd + maxv + minus_minv;
    if (g_val < 0.0) g_val = 0;
    if (g_val < 1.0e-8) { o.sqrd = sqrd; return; }
    if ((first_iteration || (sqrd < oldsqrd)) && (g.npts <= 3)) {
      double f[3];
      sup.point(minq, f);
      const int np_ = g.npts;
      g.s2[np_] = minq;
      g.lambdas[np_] = 0.0;
      for (int d = 0; d < 3; d++) { g.c1[np_][d] = vrel[d]; g.c2[np_][d] = f[d]; }
      g.npts++;
      oldsqrd = sqrd;
      first_iteration = 0;
      use_default = 1;
      continue;
    }
    if (use_default) use_default = 0;
    else { o.sqrd = sqrd; return; }
  }
  o.sqrd = 0.0;
}

}  // namespace lqro
