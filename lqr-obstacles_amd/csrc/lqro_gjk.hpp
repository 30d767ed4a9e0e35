// lqro_gjk.hpp — gjk_distance (gjk.cpp:296-501, Cameron's Oxford GJK v2.4)
// specialised to the call the path makes (run_gjk, LQRObstacles.cpp:814-853):
// object 1 is the single point vrel (hill climbing on its one-vertex ring
// returns it), object 2 is the reachable point set with a brute-force support
// function (support_simple, gjk.cpp:770-794), no transforms, no seed.
//
// The simplex bookkeeping runs redundantly in every lane (all values are
// wave-uniform).  Johnson's sub-algorithm — compute_subterms, default_distance,
// backup_distance, reset_simplex (gjk.cpp:527-736) over the constant subset
// tables (gjk.cpp:86-160) — is restated with every loop fully unrolled over
// the 15 subsets, so all table lookups and state indices are compile-time and
// the state stays in registers; the arithmetic and its order are unchanged.
// Object 1's simplex coordinates are all vrel, so coords1[i] is not stored.
#pragma once
#include <hip/hip_runtime.h>

#include "lqro_device.hpp"

namespace lqro {

struct GjkTab {
  static constexpr int card[16] = {0, 1, 1, 2, 1, 2, 2, 3, 1, 2, 2, 3, 2, 3, 3, 4};
  static constexpr int maxe[16] = {-1, 0, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3};
  static constexpr int elts[16][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {1, 0, 0, 0}, {0, 1, 0, 0},
                                      {2, 0, 0, 0}, {0, 2, 0, 0}, {1, 2, 0, 0}, {0, 1, 2, 0},
                                      {3, 0, 0, 0}, {0, 3, 0, 0}, {1, 3, 0, 0}, {0, 1, 3, 0},
                                      {2, 3, 0, 0}, {0, 2, 3, 0}, {1, 2, 3, 0}, {0, 1, 2, 3}};
  static constexpr int nonelts[16][4] = {{0, 1, 2, 3}, {1, 2, 3, 0}, {0, 2, 3, 0}, {2, 3, 0, 0},
                                         {0, 1, 3, 0}, {1, 3, 0, 0}, {0, 3, 0, 0}, {3, 0, 0, 0},
                                         {0, 1, 2, 0}, {1, 2, 0, 0}, {0, 2, 0, 0}, {2, 0, 0, 0},
                                         {0, 1, 0, 0}, {1, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  static constexpr int pred[16][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {2, 1, 0, 0},
                                      {0, 0, 0, 0}, {4, 1, 0, 0}, {4, 2, 0, 0}, {6, 5, 3, 0},
                                      {0, 0, 0, 0}, {8, 1, 0, 0}, {8, 2, 0, 0}, {10, 9, 3, 0},
                                      {8, 4, 0, 0}, {12, 9, 5, 0}, {12, 10, 6, 0}, {14, 13, 11, 7}};
  static constexpr int succ[16][4] = {{1, 2, 4, 8}, {3, 5, 9, 0}, {3, 6, 10, 0}, {7, 11, 0, 0},
                                      {5, 6, 12, 0}, {7, 13, 0, 0}, {7, 14, 0, 0}, {15, 0, 0, 0},
                                      {9, 10, 12, 0}, {11, 13, 0, 0}, {11, 14, 0, 0}, {15, 0, 0, 0},
                                      {13, 14, 0, 0}, {15, 0, 0, 0}, {15, 0, 0, 0}, {0, 0, 0, 0}};
};

struct GjkState {
  int npts;
  int s2[4];          // point ids (q = k*NP + p) of the hull-side simplex vertices
  double lam[4];
  double c2[4][3];    // coords2 (coords1 are all vrel)
  double dv[16][4];   // delta_values (gjk.cpp:163)
  double dp[4][4];    // dot_products (gjk.cpp:164)
  double dsum[16];    // delta (gjk.cpp:522)
};

struct GjkOut {
  double sqrd, w1[3], w2[3];
  int iters, backup;
};

// compute_subterms (gjk.cpp:527-581)
__device__ __forceinline__ void gjk_subterms(GjkState& g, const double* vrel) {
  using T = GjkTab;
  const int size = g.npts;
  double csp[4][3];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) csp[i][j] = vrel[j] - g.c2[i][j];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = i; j < 4; j++)
      if (j < size)
        g.dp[i][j] = g.dp[j][i] = csp[i][0] * csp[j][0] + csp[i][1] * csp[j][1] + csp[i][2] * csp[j][2];
#pragma unroll
  for (int s = 1; s < 16; s++) {
    if (T::maxe[s] < size) {
      if (T::card[s] <= 1) {
        g.dv[s][T::elts[s][0]] = 1.0;
      } else if (T::card[s] == 2) {
        constexpr int dummy = 0; (void)dummy;
        const int e0 = T::elts[s][0], e1 = T::elts[s][1];
        g.dv[s][e0] = g.dp[e1][e1] - g.dp[e1][e0];
        g.dv[s][e1] = g.dp[e0][e0] - g.dp[e0][e1];
      } else {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if (j < T::card[s]) {
            const int jelt = T::elts[s][j], jsub = T::pred[s][j];
            double sum = 0;
#pragma unroll
            for (int i = 0; i < 4; i++)
              if (i < T::card[jsub]) {
                const int ielt = T::elts[jsub][i];
                sum += g.dv[jsub][ielt] * (g.dp[ielt][T::elts[jsub][0]] - g.dp[ielt][jelt]);
              }
            g.dv[s][jelt] = sum;
          }
        }
      }
    }
  }
}

// reset_simplex (gjk.cpp:708-736) for a subset chosen at run time
__device__ __forceinline__ void gjk_reset(GjkState& g, int subset) {
  using T = GjkTab;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    if (t == subset) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if (j < T::card[t]) {
          const int oldpos = T::elts[t][j];
          if (oldpos != j) {
            g.s2[j] = g.s2[oldpos];
#pragma unroll
            for (int i = 0; i < 3; i++) g.c2[j][i] = g.c2[oldpos][i];
          }
          g.lam[j] = g.dv[t][T::elts[t][j]] / g.dsum[t];
        }
      }
      g.npts = T::card[t];
    }
  }
}

// default_distance (gjk.cpp:593-657)
__device__ __forceinline__ int gjk_default(GjkState& g) {
  using T = GjkTab;
  const int size = g.npts;
  int ok = 0, found = 0, sel = 0, s_end = 16;
#pragma unroll
  for (int s = 1; s < 16; s++) {
    if (!found && T::maxe[s] < size) {
      g.dsum[s] = 0.0;
      ok = 1;
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (j < T::card[s] && ok) {
          const double v = g.dv[s][T::elts[s][j]];
          if (v > 0.0) g.dsum[s] += v;
          else ok = 0;
        }
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (k < 4 - T::card[s] && k < size - T::card[s] && ok)
          if (g.dv[T::succ[s][k]][T::nonelts[s][k]] > 0) ok = 0;
      if (ok && g.dsum[s] >= 1.0e-20) { found = 1; sel = s; }
    } else if (!found && s_end == 16) {
      s_end = s;
    }
  }
  if (!found) {
    // loop ran out: the reference then calls reset_simplex(s) with the
    // terminating s if the last subset tested was ok (tiny delta sum)
    if (ok && s_end < 16) sel = s_end;
    else return 0;
  }
  gjk_reset(g, sel);
  return 1;
}

// backup_distance (gjk.cpp:663-706)
__device__ __forceinline__ void gjk_backup(GjkState& g) {
  using T = GjkTab;
  const int size = g.npts;
  int bests = 0;
  double bnum = 0.0, bden = 0.0;
#pragma unroll
  for (int s = 1; s < 16; s++) {
    if (T::maxe[s] < size && g.dsum[s] > 0.0) {
      bool viable = true;
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (i < T::card[s] && g.dv[s][T::elts[s][i]] <= 0.0) viable = false;
      if (viable) {
        double num = 0.0;
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (j < T::card[s] && k < T::card[s])
              num += (g.dv[s][T::elts[s][j]] * g.dv[s][T::elts[s][k]]) *
                     g.dp[T::elts[s][j]][T::elts[s][k]];
        const double den = g.dsum[s] * g.dsum[s];
        if ((bests < 1) || (num * bden < bnum * den)) { bests = s; bnum = num; bden = den; }
      }
    }
  }
  gjk_reset(g, bests);
}

// compute_point (gjk.cpp:851-862): sum_i vertices[i][d] * lambdas[i] from 0
__device__ __forceinline__ void gjk_witnesses(const GjkState& g, const double* vrel, double* w1,
                                              double* w2) {
#pragma unroll
  for (int d = 0; d < 3; d++) {
    double a = 0, b = 0;
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (i < g.npts) { a += vrel[d] * g.lam[i]; b += g.c2[i][d] * g.lam[i]; }
    w1[d] = a;
    w2[d] = b;
  }
}

// Sup must provide:
//   void support(double d0, double d1, double d2, double& value, int& q[, double* pt])
//   void point(int q, double* pt)
template <class Sup>
__device__ void gjk_run(Sup& sup, int qfirst, int n, const double* vrel, GjkState& g, GjkOut& o) {
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    g.dsum[s] = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) g.dv[s][k] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    g.s2[i] = -1;
    g.lam[i] = 0.0;
#pragma unroll
    for (int d = 0; d < 3; ++d) g.c2[i][d] = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) g.dp[i][j] = 0.0;
  }
  int use_default = 1, first_iteration = 1, max_iterations = n;
  double oldsqrd = 0.0, sqrd = 0.0;
  double disp[3], rdisp[3];
  o.iters = 0; o.backup = 0;
  g.npts = 1; g.s2[0] = qfirst; g.lam[0] = 1.0;
  sup.point(qfirst, g.c2[0]);
  while (max_iterations-- > 0) {
    if (g.npts == 1) g.lam[0] = 1.0;
    else {
      gjk_subterms(g, vrel);
      if (use_default) use_default = gjk_default(g);
      if (!use_default) { gjk_backup(g); o.backup = 1; }
    }
    gjk_witnesses(g, vrel, o.w1, o.w2);
#pragma unroll
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
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k == g.npts) {
          g.s2[k] = minq;
          g.lam[k] = 0.0;
#pragma unroll
          for (int d = 0; d < 3; d++) g.c2[k][d] = f[d];
        }
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


// ---------------------------------------------------------------------------
// Wave-parallel Johnson sub-algorithm (what k_pair runs).
//
// The same arithmetic as gjk_subterms/gjk_default/gjk_backup/gjk_reset above,
// element by element and in the same order, but spread over the wave instead
// of repeated in every lane: lane L = 4 s + j holds delta_values[s][elts[s][j]]
// (subset s, its j-th element) and delta[s]; the subsets of one cardinality
// are computed together (cardinality 2, then 3 reading 2, then 4 reading 3),
// the first acceptable subset is found with a ballot.  The simplex (coords2,
// lambdas, point ids) lives in a 20-word per-wave LDS block, so the
// per-lane register state is two doubles.
//
// Subset s is the bit set of its elements: elts[s] are its set bits in
// increasing order, pred[s][j] = s without elts[s][j], maxe[s] its highest
// bit, succ[s][k] = s with its k-th missing element added (gjk.cpp:86-160).

struct GjkWave {
  double* c2;   // [4][3] coords2 of the simplex (LDS)
  double* lam;  // [4] lambdas (LDS)
  int* s2;      // [4] point ids (LDS)
};

// position of the n-th set bit of the 4-bit mask m (0 when m has fewer), as
// a 2-bit entry of a 128-bit constant table indexed by 4 m + n: branch-free
// (a per-lane loop here became exec-mask branching in the wave-parallel code)
constexpr int gjk_nth_bit_ref(int m, int n) {
  for (int b = 0; b < 4; ++b)
    if ((m >> b) & 1) {
      if (n == 0) return b;
      --n;
    }
  return 0;
}
constexpr unsigned long long gjk_nth_tab(int half) {
  unsigned long long t = 0;
  for (int idx = 0; idx < 32; ++idx) {
    const int g = 32 * half + idx;
    t |= (unsigned long long)gjk_nth_bit_ref(g >> 2, g & 3) << (2 * idx);
  }
  return t;
}
__device__ __forceinline__ int gjk_nth_bit(int m, int n) {
  constexpr unsigned long long lo = gjk_nth_tab(0), hi = gjk_nth_tab(1);
  const int idx = ((m & 15) << 2) | (n & 3);
  const unsigned long long t = idx < 32 ? lo : hi;
  return (int)((t >> (2 * (idx & 31))) & 3ull);
}

// v of lane src (0..63, per lane): ds_bpermute on both halves, no width
// arithmetic on the lane id
__device__ __forceinline__ double gjk_shfl(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)b);
  const int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// v of a wave-uniform lane: two v_readlane (no LDS round trip)
__device__ __forceinline__ double gjk_rdl(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, src);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// dv of lane 4 (lane / 4) + J: a quad_perm DPP broadcast inside each group of
// four lanes (VALU) instead of a ds_bpermute round trip
template <int J>
__device__ __forceinline__ double gjk_quad(double v) {
  return dpp_d<J * 0x55, 0xF>(0.0, v);
}

// dot_products[a][b] (gjk.cpp:541-548): csp_a . csp_b, csp = coords1 - coords2;
// symmetric exactly (each product commutes, same summation order)
__device__ __forceinline__ double gjk_dp(const GjkWave& G, const double* vrel, int a, int b) {
  const double* ca = G.c2 + 3 * a;
  const double* cb = G.c2 + 3 * b;
  const double a0 = vrel[0] - ca[0], a1 = vrel[1] - ca[1], a2 = vrel[2] - ca[2];
  const double b0 = vrel[0] - cb[0], b1 = vrel[1] - cb[1], b2 = vrel[2] - cb[2];
  return a0 * b0 + a1 * b1 + a2 * b2;
}

// compute_subterms (gjk.cpp:527-581) into this lane's dv
__device__ __forceinline__ void gjkw_subterms(const GjkWave& G, const double* vrel, int size,
                                              int lane, double& dv) {
  lane = opaque(lane);
  const int s = lane >> 2, j = lane & 3;
  const int card = __popc(s);
  const bool live = s >= 1 && j < card && (s >> size) == 0;   // maxe[s] < size
  const int e = gjk_nth_bit(s, j);
  if (live && card == 1) dv = 1.0;
  if (live && card == 2) {
    // j = 0: dp[e1][e1] - dp[e1][e0];  j = 1: dp[e0][e0] - dp[e0][e1]
    const int e0 = gjk_nth_bit(s, 0), e1 = gjk_nth_bit(s, 1);
    const int a = j == 0 ? e1 : e0, b = j == 0 ? e0 : e1;
    dv = gjk_dp(G, vrel, a, a) - gjk_dp(G, vrel, a, b);
  }
#pragma unroll
  for (int c = 3; c <= 4; ++c) {
    if (size < c) break;
    const int jsub = s & ~(1 << e);
    const int f0 = gjk_nth_bit(jsub, 0);
    double sum = 0;
#pragma unroll
    for (int i = 0; i < c - 1; ++i) {
      const int ielt = gjk_nth_bit(jsub, i);
      const double dsub = gjk_shfl(dv, 4 * jsub + i);   // delta_values[jsub][ielt]
      sum += dsub * (gjk_dp(G, vrel, ielt, f0) - gjk_dp(G, vrel, ielt, e));
    }
    if (live && card == c) dv = sum;
  }
}

// reset_simplex (gjk.cpp:708-736) for a wave-uniform subset; returns the new size
__device__ __forceinline__ int gjkw_reset(const GjkWave& G, int subset, double dv, double dsum,
                                          int lane) {
  lane = opaque(lane);
  const int card = __popc(subset);
  const double ds = gjk_rdl(dsum, 4 * subset);
  const double lv = gjk_shfl(dv, 4 * subset + (lane & 3));
  // lanes 0..11 move coords2, lanes 0..3 the ids and lambdas
  double cv = 0.0;
  int sv = 0;
  const int jj = lane / 3, d = lane - 3 * jj;
  if (lane < 3 * card) cv = G.c2[3 * gjk_nth_bit(subset, jj) + d];
  if (lane < card) sv = G.s2[gjk_nth_bit(subset, lane)];
  wave_lds_sync();
  if (lane < 3 * card) G.c2[lane] = cv;
  if (lane < card) {
    G.s2[lane] = sv;
    G.lam[lane] = lv / ds;
  }
  wave_lds_sync();
  return card;
}

// default_distance (gjk.cpp:593-657): 1 and the new size through *size, or 0
__device__ __forceinline__ int gjkw_default(const GjkWave& G, int& size, double dv, double& dsum,
                                            int lane) {
  lane = opaque(lane);
  const int s = lane >> 2;
  const int card = __popc(s);
  const bool valid = s >= 1 && (s >> size) == 0;
  int ok = 1;
  double ds = 0.0;
  const double q[4] = {gjk_quad<0>(dv), gjk_quad<1>(dv), gjk_quad<2>(dv), gjk_quad<3>(dv)};
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const double v = q[jj];   // delta_values[s][elts[s][jj]]
    if (jj < card && ok) {
      if (v > 0.0) ds += v;
      else ok = 0;
    }
  }
  int nk = 0;   // k-th element missing from s, below size
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const bool cand = ((s >> b) & 1) == 0 && b < size;
    const int sc = s | (1 << b);
    const int pos = __popc(sc & ((1 << b) - 1));
    const double v = gjk_shfl(dv, 4 * (sc & 15) + pos);   // delta_values[succ][nonelt]
    if (cand) {
      if (ok && v > 0) ok = 0;
      ++nk;
    }
  }
  const bool found = valid && ok && ds >= 1.0e-20;
  const unsigned long long bal = __ballot(found && (lane & 3) == 0);
  int sel;
  if (bal) {
    sel = (__ffsll((long long)bal) - 1) >> 2;
    if (valid && s <= sel) dsum = ds;
  } else {
    if (valid) dsum = ds;
    // the loop ran out: reset_simplex(s) with the terminating s when the
    // last subset tested was ok (it had a tiny delta sum)
    const int last = (1 << size) - 1;
    const int okl = __builtin_amdgcn_readlane(ok, 4 * last);
    if (!(okl && size < 4)) return 0;
    sel = 1 << size;
  }
  size = gjkw_reset(G, sel, dv, dsum, lane);
  return 1;
}

// backup_distance (gjk.cpp:663-706)
__device__ __forceinline__ int gjkw_backup(const GjkWave& G, const double* vrel, int size, double dv,
                                           double dsum, int lane) {
  lane = opaque(lane);
  const int s = lane >> 2;
  const int card = __popc(s);
  const bool valid = s >= 1 && (s >> size) == 0;
  const double v[4] = {gjk_quad<0>(dv), gjk_quad<1>(dv), gjk_quad<2>(dv), gjk_quad<3>(dv)};
  bool viable = valid && dsum > 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (i < card && v[i] <= 0.0) viable = false;
  double num = 0.0;
  if (viable) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        if (jj < card && kk < card)
          num += (v[jj] * v[kk]) *
                 gjk_dp(G, vrel, gjk_nth_bit(s, jj), gjk_nth_bit(s, kk));
  }
  const double den = dsum * dsum;
  const unsigned long long vb = __ballot(viable && (lane & 3) == 0);
  int bests = 0;
  double bnum = 0.0, bden = 0.0;
  for (int t = 1; t < 16; ++t) {
    if (!((vb >> (4 * t)) & 1ull)) continue;
    const double tn = gjk_rdl(num, 4 * t), td = gjk_rdl(den, 4 * t);
    if ((bests < 1) || (tn * bden < bnum * td)) { bests = t; bnum = tn; bden = td; }
  }
  return gjkw_reset(G, bests, dv, dsum, lane);
}

// gjk_run with the wave-parallel sub-algorithm.  Sup as for gjk_run.
template <class Sup>
__device__ void gjkw_run(Sup& sup, const GjkWave& G, int lane, int qfirst, int n,
                         const double* vrel, int& npts, GjkOut& o) {
  double dv = 0.0, dsum = 0.0;            // delta_values / delta (zeroed per call)
  int use_default = 1, first_iteration = 1, max_iterations = n;
  double oldsqrd = 0.0, sqrd = 0.0;
  o.iters = 0; o.backup = 0;
  {
    double f[3];
    sup.point(qfirst, f);
    if (lane < 3) G.c2[lane] = f[lane == 0 ? 0 : (lane == 1 ? 1 : 2)];
    if (lane == 0) { G.s2[0] = qfirst; G.lam[0] = 1.0; }
    wave_lds_sync();
  }
  npts = 1;
#ifdef LQRO_PAIR_PROFILE
  unsigned long long t_ = __builtin_amdgcn_s_memtime();
#define GJK_STAMP(k)                                          \
  do {                                                        \
    const unsigned long long u_ = __builtin_amdgcn_s_memtime(); \
    sup.pc[k] += u_ - t_;                                     \
    t_ = u_;                                                  \
  } while (0)
#else
#define GJK_STAMP(k) do {} while (0)
#endif
  while (max_iterations-- > 0) {
    if (npts == 1) {
      if (lane == 0) G.lam[0] = 1.0;
      wave_lds_sync();
    } else {
      gjkw_subterms(G, vrel, npts, lane, dv);
      if (use_default) use_default = gjkw_default(G, npts, dv, dsum, lane);
      if (!use_default) { npts = gjkw_backup(G, vrel, npts, dv, dsum, lane); o.backup = 1; }
    }
    GJK_STAMP(3);
    // compute_point (gjk.cpp:851-862)
#pragma unroll
    for (int d = 0; d < 3; d++) {
      double a = 0, b = 0;
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (i < npts) { a += vrel[d] * G.lam[i]; b += G.c2[3 * i + d] * G.lam[i]; }
      o.w1[d] = a;
      o.w2[d] = b;
    }
    double disp[3], rdisp[3];
#pragma unroll
    for (int d = 0; d < 3; d++) { disp[d] = o.w2[d] - o.w1[d]; rdisp[d] = -disp[d]; }
    sqrd = disp[0] * disp[0] + disp[1] * disp[1] + disp[2] * disp[2];
    GJK_STAMP(4);
    if (sqrd < 1.0e-8) { o.sqrd = sqrd; return; }
    const double maxv = vrel[0] * disp[0] + vrel[1] * disp[1] + vrel[2] * disp[2];
    double minus_minv;
    int minq;
    double f[3];   // the support point (== sup.point(minq))
    sup.support(rdisp[0], rdisp[1], rdisp[2], minus_minv, minq, f);
#ifdef LQRO_PAIR_PROFILE
    t_ = __builtin_amdgcn_s_memtime();
#endif
    o.iters++;
    double g_val = sqrd + maxv + minus_minv;
    if (g_val < 0.0) g_val = 0;
    if (g_val < 1.0e-8) { o.sqrd = sqrd; return; }
    if ((first_iteration || (sqrd < oldsqrd)) && (npts <= 3)) {
      wave_lds_sync();   // every lane has read the old simplex
      if (lane < 3) G.c2[3 * npts + lane] = f[lane == 0 ? 0 : (lane == 1 ? 1 : 2)];
      if (lane == 0) { G.s2[npts] = minq; G.lam[npts] = 0.0; }
      wave_lds_sync();
      GJK_STAMP(5);
      npts++;
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
#undef GJK_STAMP

}  // namespace lqro
