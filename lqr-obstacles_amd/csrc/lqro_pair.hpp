// lqro_pair.hpp — the pair kernel: one wavefront per ordered pair (i, j),
// one workgroup per row agent i (its horizon tables staged in LDS).
//
// Reference (LQRObstacles.cpp, "LQRO"):
//   createObstacle      :770-783  point(k,p) = T_k (s_p + Translate_k),
//                                 Translate_k = (-C F_k)(x_i - x_j)
//   findReachableObstacle :786-812 |point - vrel|^2/30^2 < 1, kept in k*NP+p order
//   pointInHull / run_gjk :814-864 GJK point-to-hull distance (lqro_gjk.hpp)
//   createHalfPlanes    :1208-1221
//
// Work-efficient but exact.  A horizon step k ("slice") holds NP points that
// lie on the ellipsoid c_k + T_k diag(2r_xy, 2r_xy, 2r_z) S^2, c_k = T_k tr_k.
// From that ellipsoid the kernel derives, per pair:
//   * a slice class: every point certainly reachable (IN), certainly not
//     (OUT), or MIXED — only MIXED slices run the per-point test;
//   * for a GJK support direction d, an upper bound d.c_k + |S T_k^T d| on
//     every point value in the slice: slices are evaluated in decreasing bound
//     order and skipped once their bound is below the best value found.
// Bounds carry a 1e-9 relative margin (far above fp64 rounding), and every
// value that is compared or returned is computed exactly as the reference
// computes it, so n_reach, the reachable list, the support points and hence
// the GJK result are bit-identical to evaluating every point.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lqro.h"
#include "lqro_device.hpp"
#include "lqro_gjk.hpp"

namespace lqro {

enum : int { kSliceOut = 0, kSliceIn = 1, kSliceMixed = 2 };
// k_pair launch kinds: the row launch (rows off a queue, row tables staged in
// LDS), the hot launch with shared tables (staged once), the hot launch with
// per-agent tables (read from global memory, pairs of any row)
enum : int { kRowLaunch = 0, kHotShared = 1, kHotPerAgent = 2 };
constexpr int kMaxPW = 4;
constexpr int kMaxKS = 4;   // H <= 64 kMaxKS = 256 (per-lane slice slots)
#ifndef LQRO_PAIR_LB
#define LQRO_PAIR_LB 1024
#endif  // 16 waves (4 per SIMD: <= 128 VGPRs); NP <= 256 (one 64-bit reachable mask per 64 points)

struct PairArgs {
  int N, H, NP, PW, min_reach;
  int row_begin, nrows, npr;          // npr = pairs per row = N-1
  int row_stride;                     // local row r is agent row_begin + r * row_stride
  int waves;
  int max_waves;                      // waves of a workgroup that take pairs (k_side's LDS fits fewer)
  int* row_counter;                   // persistent row queue (zeroed per step)
  int row_split;                      // pair ranges per row
  int per_agent;
  double vmax, r2, r2_lo, r2_hi;      // reachable radius, its square, fast-test bounds
  double rad0, rad1, rad2, umax;      // sphere semi-axes (2 r_xy, 2 r_xy, 2 r_z); max |u_p|
  const double* T;                    // per agent H x 9
  const double* NCF;                  // per agent H x 3 x X
  const double* R;                    // per agent H: bound on |T_k s_p|
  const double* TF;                   // per agent H: ||T_k||_F
  const double* S;                    // NP x 3
  const unsigned long long* shash;    // H: sum_p mix64(k*NP+p)
  const double* x;                    // N x X
  float* planes;                      // nrows*npr x 8
  lqro_pair_record* recs;             // nullable
  int* hull_queue;
  int* hull_count;
  int hull_cap;
  unsigned long long* stats;          // 8 counters
  unsigned long long* prof;           // LQRO_PAIR_PROFILE: per-phase cycles (16 words)
  // hot phase (k_prio's list of likely inside-hull pairs; null: none)
  const int* hot_list;
  const unsigned char* hot_mark;      // per slot: 1 = in the hot list
  const int* hot_count;
  int* hot_next;
  int hot_cap;
  int hot_only;                       // 1: this launch computes the hot list only
  int* hot_done;                      // hot launch: +1 per finished workgroup (k_qhull workers wait on it), null: none
  // Qhull order, speculative builds: per slot 2 = the last step's inside-hull
  // pair, already queued for k_qhull at the step's start; this hot launch
  // evaluates it and sets 3 (inside: the build may commit) or 4 (not: the
  // build is discarded), after its plane and record, with a release.  null: off
  unsigned char* spec_mark;
  const int* nbr_list;                // culling on: per row npr (= K) neighbour jj, ascending, -1 = none
  double* qnrm;                       // LQRO_FLAG_QHULL_ORDER: per slot normal, dist (k_stale reads them)
  int* rowpend;                       // early LP: per row open work (LQRO_ROW_BIG), null: off
  // LDS layout, in doubles
  int XP, lds_T, lds_N, lds_S, lds_R, lds_TF, lds_H, lds_wave, wave_doubles;
};

struct BlockTabs {
  const double* T;
  const double* N;    // H x 3 rows of pitch `pitch` (X + 1 in LDS, X in global memory)
  int pitch;
  const double* S;    // SoA: x[NP], y[NP], z[NP]
  const double* R;
  const double* TF;
  const unsigned long long* shash;
};

struct WaveTabs {
  double* tr;                // H x 3
  double* sc;                // H: magnitude scale for the margins
  int* cls;                  // H
  int* cnt;                  // H: reachable points in the slice
  int* mixed;                // H: list of MIXED slices
  unsigned long long* mask;  // H x PW
  GjkWave gjk;               // the GJK simplex (18 doubles)
  unsigned long long* st;    // 5 counters (reach, iters, planes, inside, backup), lane 0 adds
};

// a wave-private LDS counter: ds_add_u64 with no return, so nothing waits on it
__device__ __forceinline__ void lds_count(unsigned long long* c, unsigned long long v) {
  __hip_atomic_fetch_add(c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Transform*(points[p] + Translate) (LQRO:776); Matrix::operator* accumulates
// from 0.0 (include/matrix.h:223-227)
__device__ __forceinline__ void exact_point(const BlockTabs& B, const WaveTabs& W, int NP, int k,
                                            int p, double* x) {
  const double* Tk = B.T + 9 * k;
  const double* tk = W.tr + 3 * k;
  const double u0 = B.S[p] + tk[0];
  const double u1 = B.S[NP + p] + tk[1];
  const double u2 = B.S[2 * NP + p] + tk[2];
  x[0] = ((0.0 + Tk[0] * u0) + Tk[1] * u1) + Tk[2] * u2;
  x[1] = ((0.0 + Tk[3] * u0) + Tk[4] * u1) + Tk[5] * u2;
  x[2] = ((0.0 + Tk[6] * u0) + Tk[7] * u1) + Tk[8] * u2;
}

// findReachableObstacle's test (LQRO:799), pow(x,2) = x*x; decided by a
// 1e-12-margin pre-test except near the sphere, where the reference's
// divisions run literally.
__device__ __forceinline__ bool reach_exact(double a, double b, double c, const PairArgs& P) {
  const double t = a * a + b * b + c * c;
  if (t < P.r2_lo) return true;
  if (t > P.r2_hi) return false;
  return (a * a) / P.r2 + (b * b) / P.r2 + (c * c) / P.r2 < 1.0;
}

__device__ __forceinline__ bool better(double v, int q, double bv, int bq) {
  return v > bv || (v == bv && q < bq);
}

template <int CTRL, int ROWS>
__device__ __forceinline__ void argmax_step(double& v, int& q) {
  const double ov = dpp_d<CTRL, ROWS>(-INFINITY, v);
  const int oq = dpp_i<CTRL, ROWS>(INT_MAX, q);
  if (better(ov, oq, v, q)) { v = ov; q = oq; }
}

template <int CTRL, int ROWS>
__device__ __forceinline__ void max_step(double& v) {
  v = fmax(v, dpp_d<CTRL, ROWS>(-INFINITY, v));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ void max_step_f(float& v) {
  v = fmaxf(v, __int_as_float(dpp_i<CTRL, ROWS>(__float_as_int(-INFINITY), __float_as_int(v))));
}
// v of a wave-uniform lane (two v_readlane)
__device__ __forceinline__ double rdl_d(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, src);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

#ifndef LQRO_ARGMAX_PAIRS
template <int CTRL, int ROWS>
__device__ __forceinline__ void min_step(int& q) {
  q = min(q, dpp_i<CTRL, ROWS>(INT_MAX, q));
}
// wave arg-max of (v, q), lowest q on ties, result in every lane: the wave
// maximum of v (row_shr prefix maxima in each 16-lane row, row_bcast across
// rows: lane 63 holds it), then the wave minimum of q over the lanes holding
// that value, and v read from that lane (so a -0.0 / +0.0 tie returns the
// winner's own zero, as the sequential scan would)
__device__ __forceinline__ void wave_argmax(double& v, int& q) {
  double m = v;
  max_step<0x111, 0xF>(m);   // row_shr:1
  max_step<0x112, 0xF>(m);   // row_shr:2
  max_step<0x114, 0xF>(m);   // row_shr:4
  max_step<0x118, 0xF>(m);   // row_shr:8
  max_step<0x142, 0xA>(m);   // row_bcast:15
  max_step<0x143, 0xC>(m);   // row_bcast:31
  const long long b = __double_as_longlong(m);
  const int lo = __builtin_amdgcn_readlane((int)b, 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  m = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  int t = v == m ? q : INT_MAX;
  min_step<0x111, 0xF>(t);
  min_step<0x112, 0xF>(t);
  min_step<0x114, 0xF>(t);
  min_step<0x118, 0xF>(t);
  min_step<0x142, 0xA>(t);
  min_step<0x143, 0xC>(t);
  const int qw = __builtin_amdgcn_readlane(t, 63);
  const unsigned long long w = __ballot(v == m && q == qw);
  if (w) {
    const int wl = __ffsll((long long)w) - 1;
    const long long vb = __double_as_longlong(v);
    const int vlo = __builtin_amdgcn_readlane((int)vb, wl);
    const int vhi = __builtin_amdgcn_readlane((int)(vb >> 32), wl);
    v = __longlong_as_double(((long long)vhi << 32) | (unsigned)vlo);
  } else {
    v = m;
  }
  q = qw;
}
#else
// wave arg-max of (v, q), lowest q on ties, result in every lane: row_shr
// prefix maxima within each 16-lane row, row_bcast to combine the rows
// (lane 63 then holds the result), readlane to broadcast
__device__ __forceinline__ void wave_argmax(double& v, int& q) {
  argmax_step<0x111, 0xF>(v, q);   // row_shr:1
  argmax_step<0x112, 0xF>(v, q);   // row_shr:2
  argmax_step<0x114, 0xF>(v, q);   // row_shr:4
  argmax_step<0x118, 0xF>(v, q);   // row_shr:8
  argmax_step<0x142, 0xA>(v, q);   // row_bcast:15
  argmax_step<0x143, 0xC>(v, q);   // row_bcast:31
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  v = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  q = __builtin_amdgcn_readlane(q, 63);
}
#endif

struct SliceSupport {
  const PairArgs& P;
  const BlockTabs& B;
  const WaveTabs& W;
  int lane;
#ifdef LQRO_PAIR_PROFILE
  unsigned long long* pc;   // [0] support cycles, [1] calls, [2] candidate slices, [3] Johnson, [4] witness, [5] point
#endif

  __device__ void point(int q, double* x) const {
    const int k = q / P.NP;
    exact_point(B, W, P.NP, k, q - k * P.NP, x);
  }

  // the winner of a wave arg-max: every lane gets the point coordinates the
  // winning lane computed (lanes' q are distinct; none won: unchanged)
  __device__ __forceinline__ static void take_point(int myq, int qw, const double* mx, double* bx) {
    const unsigned long long w = __ballot(myq == qw && qw != INT_MAX);
    if (!w) return;
    const int wl = __ffsll((long long)w) - 1;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const long long b = __double_as_longlong(mx[c]);
      const int lo = __builtin_amdgcn_readlane((int)b, wl);
      const int hi = __builtin_amdgcn_readlane((int)(b >> 32), wl);
      bx[c] = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
    }
  }

  // best (value, q, point) over the reachable points of slice k, merged into
  // (bv, bq, bx).  Lane L holds points p = L + 64 pw, in increasing p, so a
  // strict > keeps each lane's first maximiser; the slice's first maximiser
  // is then the lowest lane of the lowest pw group among the lanes holding
  // the wave maximum (ballots, no index reduction).
  __device__ void eval_slice(int k, double d0, double d1, double d2, double& bv, int& bq, double* bx) const {
    const double* Tk = B.T + 9 * k;
    const double* tk = W.tr + 3 * k;
    double T[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) T[e] = Tk[e];
    const double t0 = tk[0], t1 = tk[1], t2 = tk[2];
    double lv = -INFINITY;
    int lp = INT_MAX;
    double lx[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int pw = 0; pw < kMaxPW; ++pw) {
      if (pw >= P.PW) break;
      const int p = pw * 64 + lane;
      const unsigned long long bits = W.mask[k * P.PW + pw];
      if (p < P.NP && ((bits >> lane) & 1ull)) {
        // exact_point (LQRO:776, matrix.h:223-227)
        const double u0 = B.S[p] + t0;
        const double u1 = B.S[P.NP + p] + t1;
        const double u2 = B.S[2 * P.NP + p] + t2;
        const double x0 = ((0.0 + T[0] * u0) + T[1] * u1) + T[2] * u2;
        const double x1 = ((0.0 + T[3] * u0) + T[4] * u1) + T[5] * u2;
        const double x2 = ((0.0 + T[6] * u0) + T[7] * u1) + T[8] * u2;
        const double v = x0 * d0 + x1 * d1 + x2 * d2;   // SUPPORT_DOT_PRODUCT
        if (v > lv) { lv = v; lp = p; lx[0] = x0; lx[1] = x1; lx[2] = x2; }
      }
    }
    double m = lv;
    max_step<0x111, 0xF>(m);   // row_shr:1
    max_step<0x112, 0xF>(m);   // row_shr:2
    max_step<0x114, 0xF>(m);   // row_shr:4
    max_step<0x118, 0xF>(m);   // row_shr:8
    max_step<0x142, 0xA>(m);   // row_bcast:15
    max_step<0x143, 0xC>(m);   // row_bcast:31
    m = rdl_d(m, 63);
    unsigned long long w = 0;
#pragma unroll
    for (int pw = 0; pw < kMaxPW; ++pw) {
      if (pw >= P.PW) break;
      w = __ballot(lv == m && (lp >> 6) == pw);
      if (w) break;
    }
    if (!w) return;
    const int wl = __ffsll((long long)w) - 1;
    const double v = rdl_d(lv, wl);
    const int q = k * P.NP + __builtin_amdgcn_readlane(lp, wl);
    if (better(v, q, bv, bq)) {
      bv = v;
      bq = q;
#pragma unroll
      for (int c = 0; c < 3; ++c) bx[c] = rdl_d(lx[c], wl);
    }
  }

  // support_simple semantics: lowest-index maximiser of p.d over the reachable set.
  // 1. an upper bound ub_k on every point value of each live slice;
  // 2. the slice with the largest bound is evaluated exactly: its best value
  //    bv is a lower bound on the answer;
  // 3. every other slice with ub_k >= bv (the only ones that can hold a value
  //    >= bv, ties included) is evaluated in one flattened pass, lanes over
  //    (candidate, point), and one arg-max merges the lanes.
  // bx: the support point itself (the coordinates the winning lane computed,
  // exactly what point(bq) recomputes)
  __device__ void support(double d0, double d1, double d2, double& bv, int& bq, double* bx) const {
#ifdef LQRO_PAIR_PROFILE
    const unsigned long long t0_ = __builtin_amdgcn_s_memtime();
    pc[1] += 1;
    support_(d0, d1, d2, bv, bq, bx);
    pc[0] += __builtin_amdgcn_s_memtime() - t0_;
  }
  __device__ void support_(double d0, double d1, double d2, double& bv, int& bq, double* bx) const {
#endif
    // magnitudes below only scale the 1e-9 margins: the hardware square root
    // (a few ulp) is ample there
#ifdef LQRO_PAIR_PROFILE
    const unsigned long long t0s_ = __builtin_amdgcn_s_memtime();
#endif
    const double dn = __builtin_amdgcn_sqrt(d0 * d0 + d1 * d1 + d2 * d2);
    double cu = -INFINITY;
    int ck = INT_MAX;
    // the bounds stay in registers: lane owns slices lane + 64 s (H <= 64 kMaxKS)
    double ubr[kMaxKS];
#pragma unroll
    for (int s = 0; s < kMaxKS; ++s) {
      const int k = lane + 64 * s;
      double ub = -INFINITY;
      if (k < P.H && W.cls[k] != kSliceOut) {
        const double* Tk = B.T + 9 * k;
        const double w0 = Tk[0] * d0 + Tk[3] * d1 + Tk[6] * d2;
        const double w1 = Tk[1] * d0 + Tk[4] * d1 + Tk[7] * d2;
        const double w2 = Tk[2] * d0 + Tk[5] * d1 + Tk[8] * d2;
        const double a0 = P.rad0 * w0, a1 = P.rad1 * w1, a2 = P.rad2 * w2;
        // c_k.d = (T_k tr_k).d = tr_k.(T_k^T d); the reassociation error is
        // ~1e-16 |tr| ||T|| |d|, far inside the 1e-9 dn sc margin
        const double* tk = W.tr + 3 * k;
        ub = tk[0] * w0 + tk[1] * w1 + tk[2] * w2 +
             __builtin_amdgcn_sqrt(a0 * a0 + a1 * a1 + a2 * a2) * P.umax + 1e-9 * dn * W.sc[k];
        if (ub > cu) { cu = ub; ck = k; }
      }
      ubr[s] = ub;
    }
    // the slice evaluated first only needs a (near-)largest bound — any
    // choice gives the same result, the candidate pass covers the rest — so
    // the maximum is taken in fp32 and its lowest lane wins
    {
      float mf = (float)cu;
      const float cf = mf;
      max_step_f<0x111, 0xF>(mf);
      max_step_f<0x112, 0xF>(mf);
      max_step_f<0x114, 0xF>(mf);
      max_step_f<0x118, 0xF>(mf);
      max_step_f<0x142, 0xA>(mf);
      max_step_f<0x143, 0xC>(mf);
      mf = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mf), 63));
      const unsigned long long w = __ballot(ck != INT_MAX && cf == mf);
      ck = w ? __builtin_amdgcn_readlane(ck, __ffsll((long long)w) - 1) : INT_MAX;
    }
#ifdef LQRO_PAIR_PROFILE
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime();
    pc[6] += t1_ - t0s_;
#endif
    bv = -INFINITY;
    bq = INT_MAX;
    if (ck == INT_MAX) return;
    eval_slice(ck, d0, d1, d2, bv, bq, bx);
#ifdef LQRO_PAIR_PROFILE
    pc[7] += __builtin_amdgcn_s_memtime() - t1_;
#endif
    // candidates: the other slices whose bound reaches bv (usually none)
    unsigned long long cb[kMaxKS];
    unsigned long long any = 0;
#pragma unroll
    for (int s = 0; s < kMaxKS; ++s) {
      const int k = lane + 64 * s;
      cb[s] = __ballot(k < P.H && k != ck && ubr[s] > -INFINITY && ubr[s] >= bv);
      any |= cb[s];
    }
    if (!any) return;
    wave_lds_sync();   // the previous query's readers of W.mixed are done
    int ncand = 0;
#pragma unroll
    for (int s = 0; s < kMaxKS; ++s) {
      if ((cb[s] >> lane) & 1ull) W.mixed[ncand + __popcll(cb[s] & ((1ull << lane) - 1ull))] = lane + 64 * s;
      ncand += __popcll(cb[s]);
    }
#ifdef LQRO_PAIR_PROFILE
    pc[2] += ncand;
#endif
    wave_lds_sync();
    double lv = -INFINITY;
    int lq = INT_MAX;
    double lx[3] = {0.0, 0.0, 0.0};
    // lane walks (c, p) = divmod(idx, NP) for idx = lane, lane+64, ...
    int c = 0, p = lane;
    while (p >= P.NP) { p -= P.NP; ++c; }
    while (c < ncand) {
      const int k = W.mixed[c];
      const unsigned long long bits = W.mask[k * P.PW + (p >> 6)];
      if ((bits >> (p & 63)) & 1ull) {
        double x[3];
        exact_point(B, W, P.NP, k, p, x);
        const double v = x[0] * d0 + x[1] * d1 + x[2] * d2;   // SUPPORT_DOT_PRODUCT
        const int q = k * P.NP + p;
        if (better(v, q, lv, lq)) { lv = v; lq = q; lx[0] = x[0]; lx[1] = x[1]; lx[2] = x[2]; }
      }
      p += 64;
      while (p >= P.NP) { p -= P.NP; ++c; }
    }
    const int myq = lq;
    wave_argmax(lv, lq);
    if (better(lv, lq, bv, bq)) { bv = lv; bq = lq; take_point(myq, lq, lx, bx); }
  }
};

// rank of point q in the reachable list (the reachablePoints index)
__device__ inline int reach_rank(const PairArgs& P, const WaveTabs& W, int lane, int q) {
  const int kq = q / P.NP, pq = q - kq * P.NP;
  int cnt = 0;
  for (int k = lane; k < kq; k += 64) cnt += W.cnt[k];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
  for (int pw = 0; pw < P.PW; ++pw) {
    const unsigned long long bits = W.mask[kq * P.PW + pw];
    const int lo = pw * 64;
    if (lo + 64 <= pq) cnt += __popcll(bits);
    else if (lo < pq) cnt += __popcll(bits & ((1ull << (pq - lo)) - 1ull));
  }
  return cnt;
}

#ifdef LQRO_PAIR_PROFILE
#define PSTAMP(k)                                                   \
  do {                                                              \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();     \
    pp[k] += t_ - p_last;                                           \
    p_last = t_;                                                    \
  } while (0)
#else
#define PSTAMP(k) do {} while (0)
#endif

// One workgroup's share of a k_pair launch (LDS at `lds`, laid out per
// PairArgs; waves = blockDim.x / 64 <= P.waves).  Also the tail of k_side.
template <int X, bool RECS, int HOT>
__device__ __forceinline__ void pair_block(const PairArgs& P, double* lds) {
#ifdef LQRO_PAIR_PROFILE
  unsigned long long pp[16] = {0};
  unsigned long long p_last = __builtin_amdgcn_s_memtime();
#endif
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: SGPR
  const int H = P.H, NP = P.NP, XP = P.XP;
  __shared__ int s_row, s_next;
  const unsigned long long t_wg = __builtin_amdgcn_s_memrealtime();   // (LQRO_ST_SWORK)

  double* sT = lds + P.lds_T;
  double* sN = lds + P.lds_N;
  double* sS = lds + P.lds_S;
  double* sR = lds + P.lds_R;
  double* sTF = lds + P.lds_TF;
  unsigned long long* sH = reinterpret_cast<unsigned long long*>(lds + P.lds_H);
  BlockTabs B;
  B.T = sT; B.N = sN; B.S = sS; B.R = sR; B.TF = sTF; B.shash = sH; B.pitch = XP;
  WaveTabs W;
  {
    double* w = lds + P.lds_wave + (size_t)wave * P.wave_doubles;
    W.tr = w;            w += 3 * H;
    W.sc = w;            w += H;
    W.mask = reinterpret_cast<unsigned long long*>(w);  w += H * P.PW;
    int* wi = reinterpret_cast<int*>(w);
    W.cls = wi;          wi += H;
    W.cnt = wi;          wi += H;
    W.mixed = wi;        wi += H + (H & 1);
    W.gjk.c2 = reinterpret_cast<double*>(wi);
    W.gjk.lam = W.gjk.c2 + 12;
    W.gjk.s2 = reinterpret_cast<int*>(W.gjk.c2 + 16);
    W.st = reinterpret_cast<unsigned long long*>(W.gjk.c2 + 18);
  }
  // per-wave statistics live in the wave's LDS region (registers held across
  // the persistent loop were spilled to scratch and reloaded every pair)
  const bool has_region = wave < P.max_waves;
  if (has_region && lane < 5) W.st[lane] = 0;
#ifdef LQRO_PAIR_PROFILE
  unsigned long long pc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  SliceSupport sup{P, B, W, lane, pc};
#else
  SliceSupport sup{P, B, W, lane};
#endif

  // one ordered pair (i, j = jj-th other agent) of local row lrow
  auto do_pair = [&](const int i, const int lrow, const int jj) {
    // the lane id, opaque per pair: lane-derived constants are rebuilt here
    // rather than hoisted into registers held across the persistent loop
    const int ln = opaque(lane);
#ifdef LQRO_PAIR_PROFILE
    SliceSupport sp{P, B, W, ln, pc};
#else
    SliceSupport sp{P, B, W, ln};
#endif
    const double* xi = P.x + (size_t)i * X;
    // culling on (lqro_set_neighbors): slot q of the row holds its q-th neighbour
    const int jq = P.nbr_list != nullptr ? P.nbr_list[(size_t)lrow * P.npr + jj] : jj;
    if (jq < 0) {   // fewer neighbours than slots
      if (ln == 0) {
        const size_t cs = (size_t)lrow * P.npr + jj;
        float4* dst = reinterpret_cast<float4*>(P.planes + cs * 8);
        dst[0] = make_float4(0.f, 0.f, 0.f, 0.f);
        dst[1] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (RECS) {
          lqro_pair_record rec;
          memset(&rec, 0, sizeof rec);
          rec.i = i; rec.j = -1; rec.n_reach = -1;
          P.recs[cs] = rec;
        }
      }
      return;
    }
    const int j = jq < i ? jq : jq + 1;
    const double* xj = P.x + (size_t)j * X;
    double d[X];
#pragma unroll
    for (int c = 0; c < X; ++c) d[c] = xi[c] - xj[c];                       // (xInit1-xInit2)
    const double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};    // :794-796
    unsigned long long hsh = 0;
    constexpr bool want_hash = RECS;
    const double vabs = fabs(vrel[0]) + fabs(vrel[1]) + fabs(vrel[2]);
    PSTAMP(7);

    // 1. per slice: Translate (exact), centre, class       (lanes <-> k)
    for (int k = ln; k < H; k += 64) {
      const int np = HOT == kHotPerAgent ? B.pitch : XP;
      const double* nc = B.N + (size_t)k * 3 * np;
      double t0 = 0.0, t1 = 0.0, t2 = 0.0;
#pragma unroll
      for (int c = 0; c < X; ++c) t0 += nc[c] * d[c];
#pragma unroll
      for (int c = 0; c < X; ++c) t1 += nc[np + c] * d[c];
#pragma unroll
      for (int c = 0; c < X; ++c) t2 += nc[2 * np + c] * d[c];
      W.tr[3 * k] = t0; W.tr[3 * k + 1] = t1; W.tr[3 * k + 2] = t2;
      const double* Tk = B.T + 9 * k;
      const double c0 = Tk[0] * t0 + Tk[1] * t1 + Tk[2] * t2;
      const double c1 = Tk[3] * t0 + Tk[4] * t1 + Tk[5] * t2;
      const double c2 = Tk[6] * t0 + Tk[7] * t1 + Tk[8] * t2;
      const double Rk = B.R[k];
      // magnitudes for the 1e-9 relative margins: the hardware square root
      // (error a few ulp) suffices; |vrel| covers dc's own rounding
      const double sc = __builtin_amdgcn_sqrt(c0 * c0 + c1 * c1 + c2 * c2) + Rk +
                        B.TF[k] * __builtin_amdgcn_sqrt(t0 * t0 + t1 * t1 + t2 * t2) + 1.0;
      W.sc[k] = sc;
      const double e0 = c0 - vrel[0], e1 = c1 - vrel[1], e2 = c2 - vrel[2];
      const double dc = __builtin_amdgcn_sqrt(e0 * e0 + e1 * e1 + e2 * e2);
      const double slack = 1e-9 * (sc + vabs);
      int cls = kSliceMixed;
      if (dc + Rk < P.vmax - slack) cls = kSliceIn;
      else if (dc - Rk > P.vmax + slack) cls = kSliceOut;
      W.cls[k] = cls;
      // masks are read for live slices only (MIXED ones are written by the
      // per-point test); counts only by the records' simplex ranks
      if (cls == kSliceIn)
        for (int pw = 0; pw < P.PW; ++pw) {
          const int left = NP - pw * 64;
          W.mask[k * P.PW + pw] = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
        }
      if (RECS) W.cnt[k] = cls == kSliceIn ? NP : 0;
      if (cls == kSliceIn) hsh += B.shash[k];
    }
    wave_lds_sync();
    PSTAMP(1);

    // 2. MIXED slices: per-point exact test                 (lanes <-> p)
    // n_reach and the first reachable point come out of the same ballots,
    // wave-uniform: IN slices count NP each, MIXED ones their ballot bits.
    // The MIXED slices are walked as the set bits of their class ballots
    // (increasing k), each slice's T_k / Translate_k read once for its pw
    // groups.
    int nmixed = 0, n = 0, qfirst = INT_MAX;
    unsigned long long mmask[kMaxKS];
#pragma unroll
    for (int s = 0; s < kMaxKS; ++s) {
      const int k = 64 * s + ln;
      const int c = k < H ? W.cls[k] : kSliceOut;
      const unsigned long long bal = __ballot(c == kSliceMixed);
      const unsigned long long bin = __ballot(c == kSliceIn);
      mmask[s] = bal;
      nmixed += __popcll(bal);
      n += NP * __popcll(bin);
      if (bin && qfirst == INT_MAX) qfirst = (64 * s + __ffsll((long long)bin) - 1) * NP;
    }
#pragma unroll
    for (int s = 0; s < kMaxKS; ++s) {
      unsigned long long mm = mmask[s];
      while (mm) {
        const int k = 64 * s + __ffsll((long long)mm) - 1;
        mm &= mm - 1ull;
        const double* Tk = B.T + 9 * k;
        const double* tk = W.tr + 3 * k;
        double T[9];
#pragma unroll
        for (int e = 0; e < 9; ++e) T[e] = Tk[e];
        const double t0 = tk[0], t1 = tk[1], t2 = tk[2];
        bool ok[kMaxPW];
#pragma unroll
        for (int pw = 0; pw < kMaxPW; ++pw) {
          const int p = pw * 64 + ln;
          ok[pw] = false;
          if (pw < P.PW && p < NP) {
            // exact_point (LQRO:776, matrix.h:223-227)
            const double u0 = B.S[p] + t0;
            const double u1 = B.S[NP + p] + t1;
            const double u2 = B.S[2 * NP + p] + t2;
            const double x0 = ((0.0 + T[0] * u0) + T[1] * u1) + T[2] * u2;
            const double x1 = ((0.0 + T[3] * u0) + T[4] * u1) + T[5] * u2;
            const double x2 = ((0.0 + T[6] * u0) + T[7] * u1) + T[8] * u2;
            ok[pw] = reach_exact(x0 - vrel[0], x1 - vrel[1], x2 - vrel[2], P);
          }
        }
        int cnt = 0;
#pragma unroll
        for (int pw = 0; pw < kMaxPW; ++pw) {
          if (pw >= P.PW) break;
          const unsigned long long bal = __ballot(ok[pw]);
          if (ok[pw] && want_hash) hsh += mix64((uint64_t)(k * NP + pw * 64 + ln));   // records only
          if (ln == 0) W.mask[k * P.PW + pw] = bal;
          // mixed slices come in increasing k: the first set bit seen is the
          // first reachable point of the MIXED slices
          if (bal && cnt == 0 && k * NP < qfirst) qfirst = k * NP + pw * 64 + __ffsll((long long)bal) - 1;
          cnt += __popcll(bal);
        }
        n += cnt;
        if (ln == 0) {
          if (RECS) W.cnt[k] = cnt;
          if (cnt == 0) W.cls[k] = kSliceOut;
        }
      }
    }
    wave_lds_sync();
    PSTAMP(2);
#ifdef LQRO_PAIR_PROFILE
    pp[10] += nmixed;
#endif
    if (want_hash) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) hsh += __shfl_xor(hsh, off);
    }
    PSTAMP(2);

    // 3. GJK and the half-plane
    int flags = 0;
    float pl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double dist = 0.0, nrm[3] = {0, 0, 0};
    GjkOut go;
    go.iters = 0; go.backup = 0; go.sqrd = 0;
    for (int q = 0; q < 3; ++q) { go.w1[q] = 0; go.w2[q] = 0; }
    int npts = 0;
    bool inside = false;
    if (n > P.min_reach) {                                    // :1409
      gjkw_run(sp, W.gjk, ln, qfirst, n, vrel, npts, go);
      double distance = sqrt(go.sqrd);                          // :843
      nrm[0] = (go.w1[0] - go.w2[0]) / distance;                // :850-852
      nrm[1] = (go.w1[1] - go.w2[1]) / distance;
      nrm[2] = (go.w1[2] - go.w2[2]) / distance;
      inside = (distance < 0.0001 && distance > -1 * 0.0001);  // :860
      flags = LQRO_REC_PLANE | (inside ? LQRO_REC_INSIDE : 0) | (go.backup ? LQRO_REC_BACKUP : 0);
      dist = distance;
      if (!inside) {
        distance *= 0.5;                                        // :1416
        const double mult = -1.0;                               // :1215
        pl[0] = (float)(xi[3] + mult * distance * nrm[0]);      // :1217
        pl[1] = (float)(xi[4] + mult * distance * nrm[1]);
        pl[2] = (float)(xi[5] + mult * distance * nrm[2]);
        pl[3] = (float)nrm[0]; pl[4] = (float)nrm[1]; pl[5] = (float)nrm[2];
        pl[6] = __int_as_float(1);
      } else {
        pl[6] = __int_as_float(2);                              // completed by k_hull
      }
    }
    PSTAMP(4);
    const size_t slot = (size_t)lrow * P.npr + jj;
    int sranks[4] = {-1, -1, -1, -1};
    if (RECS && npts > 0)
      for (int s = 0; s < 4; ++s)
        if (s < npts) sranks[s] = reach_rank(P, W, ln, W.gjk.s2[s]);
    if (ln == 0) {
      float4* dst = reinterpret_cast<float4*>(P.planes + slot * 8);
      dst[0] = make_float4(pl[0], pl[1], pl[2], pl[3]);
      dst[1] = make_float4(pl[4], pl[5], pl[6], pl[7]);
      if (P.qnrm && flags && !inside) {   // normalVector as run_gjk left it (LQRO:850-852)
        double4* qd = reinterpret_cast<double4*>(P.qnrm + slot * 4);
        *qd = make_double4(nrm[0], nrm[1], nrm[2], dist);
      }
      lds_count(&W.st[0], (unsigned long long)n);
      if (flags) {
        lds_count(&W.st[1], (unsigned long long)go.iters);
        lds_count(&W.st[inside ? 3 : 2], 1ull);
        if (go.backup) lds_count(&W.st[4], 1ull);
      }
      if constexpr (HOT != kRowLaunch) {
        // a hot pair (counted by k_prio) is done unless its hull is open
        if (P.rowpend && !inside) {
          __threadfence();
          atomicSub(&P.rowpend[lrow], 1);
        }
      } else {
        if (P.rowpend && inside) atomicAdd(&P.rowpend[lrow], 1);   // before its job is visible
      }
      // (a speculative pair is in the queue already: its build only waits
      // for the verdict, stored below after the record)
      const bool spec = HOT != kRowLaunch && P.spec_mark != nullptr && P.spec_mark[slot] == 2;
      if (inside && !spec) {
        // published with release: k_hull workers may already be polling
        const int qi = atomicAdd(P.hull_count, 1);
        if (qi < P.hull_cap)
          __hip_atomic_store(P.hull_queue + qi, (int)slot, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (RECS) {
        lqro_pair_record rec;
        rec.i = i; rec.j = j; rec.n_reach = n; rec.flags = flags;
        rec.gjk_iters = go.iters; rec.simplex_n = npts;
        for (int s = 0; s < 4; ++s) rec.simplex[s] = sranks[s];
        rec.facet[0] = rec.facet[1] = rec.facet[2] = -1;
        rec.n_facets = 0;
        rec.reach_hash = hsh;
        rec.dist = dist;
        for (int q = 0; q < 3; ++q) {
          rec.normal[q] = nrm[q];
          rec.wpt_vrel[q] = go.w1[q];
          rec.wpt_hull[q] = go.w2[q];
          rec.plane_point[q] = pl[q];
          rec.plane_normal[q] = pl[3 + q];
        }
        P.recs[slot] = rec;
      }
      if (spec) {   // the verdict for the speculative build, after the plane and record
        __threadfence();
        __hip_atomic_store(P.spec_mark + slot, (unsigned char)(inside ? 3 : 4), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    wave_lds_sync();
    PSTAMP(5);
#ifdef LQRO_PAIR_PROFILE
    pp[11] += 1;
    pp[12] = pc[0]; pp[13] = pc[1]; pp[14] = pc[2];
    pp[6] = pc[3]; pp[8] = pc[4]; pp[9] = pc[5]; pp[15] = pc[6]; pp[3] = pc[7];
#endif
    };
  // Hot launch (shared gains only): the pairs k_prio marked as likely
  // inside-hull, one per wave, so that their hulls can run on side-stream
  // k_hull workers while the row launch sweeps the rest.  Scheduling only:
  // every pair is computed by the same code.
  if constexpr (HOT != kRowLaunch) {
    if constexpr (HOT == kHotShared) {
      for (int q = threadIdx.x; q < H * 9; q += blockDim.x) sT[q] = P.T[q];
      for (int q = threadIdx.x; q < H * 3 * X; q += blockDim.x) sN[(q / X) * XP + (q % X)] = P.NCF[q];
      for (int q = threadIdx.x; q < H; q += blockDim.x) {
        sR[q] = P.R[q];
        sTF[q] = P.TF[q];
      }
    }
    for (int q = threadIdx.x; q < NP * 3; q += blockDim.x) sS[(q % 3) * NP + q / 3] = P.S[q];
    for (int q = threadIdx.x; q < H; q += blockDim.x) sH[q] = P.shash[q];
    __syncthreads();
    const int nhot = min(*P.hot_count, P.hot_cap);
    for (;;) {
      int h = 0;
      if (lane == 0) h = atomicAdd(P.hot_next, 1);
      h = __shfl(h, 0);
      if (h >= nhot) break;
      const int slot = P.hot_list[h];
      const int lrow = slot / P.npr;
      if constexpr (HOT == kHotPerAgent) {
        // per-agent gains: the row agent's tables straight from global memory
        // (the workgroup's waves work on pairs of different rows)
        const size_t i = (size_t)P.row_begin + (size_t)lrow * P.row_stride;
        B.T = P.T + i * H * 9;
        B.N = P.NCF + i * H * 3 * X;
        B.pitch = X;
        B.R = P.R + i * H;
        B.TF = P.TF + i * H;
      }
#ifdef LQRO_HOT_STAMPS
      // diagnostic: each hot pair's start / end on the 100 MHz clock, bit 63
      // of the end = inside-hull (scripts/hot_stamps.py)
      const unsigned long long hs0 = __builtin_amdgcn_s_memrealtime();
#endif
      do_pair(P.row_begin + lrow * P.row_stride, lrow, slot - lrow * P.npr);
#ifdef LQRO_HOT_STAMPS
      if (lane == 0 && P.prof && h < 8192) {
        const unsigned long long hs1 = __builtin_amdgcn_s_memrealtime();
        const int fl = __float_as_int(P.planes[(size_t)slot * 8 + 6]);
        P.prof[48 + 2 * h] = hs0;
        P.prof[49 + 2 * h] = hs1 | ((unsigned long long)(fl == 2) << 63);
      }
#endif
    }
  } else {
  // Persistent: the workgroup takes whole rows (agent i) off a queue; its
  // waves take the row's pairs one at a time (LDS counter), so uneven pair
  // costs balance inside the row.  Agent i's horizon tables are staged into
  // LDS only when they change (once per workgroup with shared gains).
  long staged = -1;
  for (;;) {
    // work unit = (row, part): a row is split into row_split pair ranges
    // when there are fewer rows than workgroups (many GPUs / small N)
    if (threadIdx.x == 0) {
      const int u = atomicAdd(P.row_counter, 1);
      s_row = u;
      s_next = (int)((long)(u % P.row_split) * P.npr / P.row_split);
    }
    __syncthreads();
    const int unit = s_row;
    if (unit >= P.nrows * P.row_split) break;
    const int lrow = unit / P.row_split;
    const int jj_end = (int)((long)(unit % P.row_split + 1) * P.npr / P.row_split);
    const int i = P.row_begin + lrow * P.row_stride;
    const long ag = P.per_agent ? (long)i : 0;
    if (ag != staged) {
      const double* Ti = P.T + ag * H * 9;
      const double* Ni = P.NCF + ag * H * 3 * X;
      const double* Ri = P.R + ag * H;
      const double* TFi = P.TF + ag * H;
      for (int q = threadIdx.x; q < H * 9; q += blockDim.x) sT[q] = Ti[q];
      for (int q = threadIdx.x; q < H * 3 * X; q += blockDim.x) sN[(q / X) * XP + (q % X)] = Ni[q];
      for (int q = threadIdx.x; q < NP * 3; q += blockDim.x) sS[(q % 3) * NP + q / 3] = P.S[q];
      for (int q = threadIdx.x; q < H; q += blockDim.x) {
        sR[q] = Ri[q];
        sTF[q] = TFi[q];
        sH[q] = P.shash[q];
      }
      staged = ag;
      __syncthreads();
    }
    PSTAMP(0);
  for (;;) {
    if (wave >= P.max_waves) break;    // k_side: no LDS region for this wave
    int jj = 0;
    if (lane == 0) jj = atomicAdd(&s_next, 1);
    jj = __builtin_amdgcn_readlane(jj, 0);
    if (jj >= jj_end) break;
    if (P.hot_mark != nullptr && P.hot_mark[(size_t)lrow * P.npr + jj]) continue;   // done in the hot phase
    do_pair(i, lrow, jj);
  }
    if (P.rowpend) {
      // the unit's planes are written: release them, then count the unit
      __threadfence();
      __syncthreads();
      if (threadIdx.x == 0) atomicAdd(&P.rowpend[lrow], LQRO_ROW_BIG);
    }
    __syncthreads();   // the row is done before s_row / the tables change
  }
  }   // row launch
#ifdef LQRO_PAIR_PROFILE
  if (lane == 0 && P.prof)
    for (int k = 0; k < 16; ++k) atomicAdd(&P.prof[k], pp[k]);
#endif
  // the waves' counters summed in LDS, then one atomic per counter and
  // workgroup, none for a zero: 5 same-address atomics from every wave
  // serialised at the L2 — 0.19 ms for an empty 192-workgroup launch, the
  // side stream's row launch after k_qhull, on the step's critical path
  __syncthreads();
  if (threadIdx.x < 5) {
    const int nw = min((int)(blockDim.x >> 6), P.max_waves);
    const size_t st_off = (size_t)(reinterpret_cast<double*>(W.st) - (lds + P.lds_wave + (size_t)wave * P.wave_doubles));
    unsigned long long sum = 0;
    for (int w = 0; w < nw; ++w)
      sum += reinterpret_cast<const unsigned long long*>(lds + P.lds_wave + (size_t)w * P.wave_doubles + st_off)[threadIdx.x];
    const int dst = threadIdx.x == 0 ? 6 : threadIdx.x == 1 ? 7 : threadIdx.x == 2 ? 1 : threadIdx.x == 3 ? 2 : 5;
    if (sum) atomicAdd(&P.stats[dst], sum);
  }
  if (threadIdx.x == 64) atomicAdd(&P.stats[LQRO_ST_SWORK], __builtin_amdgcn_s_memrealtime() - t_wg);
  if constexpr (HOT != kRowLaunch) {
    // every wave's pairs are done (the barrier above) and their hull jobs
    // published: count the workgroup for the k_qhull workers waiting on it
    if (P.hot_done && threadIdx.x == 0) {
      __threadfence();
      atomicAdd(P.hot_done, 1);
    }
  }
}

// RECS: per-pair records on (LQRO_FLAG_RECORDS); the bench path compiles
// without the record code and its registers.  HOT: the hot launch (P.hot_only)
// and the row launch are separate instantiations, so neither carries the
// other's loop around do_pair.
template <int X, bool RECS, int HOT>
__global__ void __launch_bounds__(LQRO_PAIR_LB) k_pair(PairArgs P) {
  extern __shared__ double lds[];
  pair_block<X, RECS, HOT>(P, lds);
}

#ifndef LQRO_PAIR_TU   // the non-template kernels: defined once, in lqro_runtime.hip
// k_nbr: opt-in neighbour culling (RVO2 computeNeighbors /
// insertAgentNeighbor, AGT:74-81,153-174).  One wave per row: agent i keeps
// the k agents j != i with the smallest (d2, j), d2 = |p_i - p_j|^2 < r2 —
// the set RVO2's sorted insertion keeps when agents are visited in j order.
// Found by k rounds of a wave arg-min above the previous key; writes the
// row's list of K = min(k, npr) slots (neighbour jj ascending, -1 padded)
// and counts the kept pairs into stats[0].
__global__ void __launch_bounds__(64) k_nbr(const double* x, int X, int N, int row_begin, int row_stride, int npr,
                                            double r2,
                                            int k, int K, int* list, unsigned long long* stats) {
  constexpr int kCap = 1024;   // candidates within r held in LDS
  __shared__ double cd[kCap];
  __shared__ int cj[kCap];
  const int lrow = blockIdx.x, lane = threadIdx.x, i = row_begin + lrow * row_stride;
  const double* xi = x + (size_t)i * X;
  // one scan: the agents within r (ascending j), usually a few dozen
  int ncand = 0;
  for (int base = 0; base < N; base += 64) {
    const int j = base + lane;
    double d2 = INFINITY;
    if (j < N && j != i) {
      const double* xj = x + (size_t)j * X;
      const double dx = xi[0] - xj[0], dy = xi[1] - xj[1], dz = xi[2] - xj[2];
      d2 = dx * dx + dy * dy + dz * dz;
    }
    const bool c = d2 < r2;
    const unsigned long long bal = __ballot(c);
    const int pos = ncand + __popcll(bal & ((1ull << lane) - 1ull));
    if (c && pos < kCap) { cd[pos] = d2; cj[pos] = j; }
    ncand += __popcll(bal);
  }
  wave_lds_sync();
  const bool in_lds = ncand <= kCap;
  double ld = -1.0;   // last selected key (d2, j); d2 >= 0
  int lj = -1, taken = 0;
  for (int it = 0; it < k; ++it) {
    double bd = INFINITY;
    int bj = INT_MAX;
    if (in_lds) {
      for (int q = lane; q < ncand; q += 64) {
        const double d2 = cd[q];
        const int j = cj[q];
        if (d2 < ld || (d2 == ld && j <= lj)) continue;   // already taken
        if (d2 < bd || (d2 == bd && j < bj)) { bd = d2; bj = j; }
      }
    } else {
      for (int j = lane; j < N; j += 64) {
        if (j == i) continue;
        const double* xj = x + (size_t)j * X;
        const double dx = xi[0] - xj[0], dy = xi[1] - xj[1], dz = xi[2] - xj[2];
        const double d2 = dx * dx + dy * dy + dz * dz;
        if (!(d2 < r2)) continue;
        if (d2 < ld || (d2 == ld && j <= lj)) continue;
        if (d2 < bd || (d2 == bd && j < bj)) { bd = d2; bj = j; }
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double od = __shfl_xor(bd, off);
      const int oj = __shfl_xor(bj, off);
      if (od < bd || (od == bd && oj < bj)) { bd = od; bj = oj; }
    }
    if (bj == INT_MAX) break;
    ld = bd; lj = bj; ++taken;
  }
  int* row = list + (size_t)lrow * K;
  int cnt = 0;
  if (in_lds) {   // candidates are in ascending j: keep those at or below the last key
    for (int base = 0; base < ncand; base += 64) {
      const int q = base + lane;
      bool sel = false;
      int jj = 0;
      if (q < ncand && taken > 0) {
        const double d2 = cd[q];
        const int j = cj[q];
        jj = j < i ? j : j - 1;
        sel = d2 < ld || (d2 == ld && j <= lj);
      }
      const unsigned long long bal = __ballot(sel);
      if (sel) row[cnt + __popcll(bal & ((1ull << lane) - 1ull))] = jj;
      cnt += __popcll(bal);
    }
  } else
  for (int base = 0; base < npr; base += 64) {
    const int jj = base + lane;
    bool sel = false;
    if (jj < npr && taken > 0) {
      const int j = jj < i ? jj : jj + 1;
      const double* xj = x + (size_t)j * X;
      const double dx = xi[0] - xj[0], dy = xi[1] - xj[1], dz = xi[2] - xj[2];
      const double d2 = dx * dx + dy * dy + dz * dz;
      sel = d2 < r2 && (d2 < ld || (d2 == ld && j <= lj));
    }
    const unsigned long long bal = __ballot(sel);
    if (sel) row[cnt + __popcll(bal & ((1ull << lane) - 1ull))] = jj;
    cnt += __popcll(bal);
  }
  for (int q = cnt + lane; q < K; q += 64) row[q] = -1;
  if (lane == 0) atomicAdd(&stats[0], (unsigned long long)taken);
}

// k_prio: which pairs go first.  A pair whose relative motion brings the two
// agents within hot_r of each other in the next t_hot seconds (closest
// approach of p_i - p_j + t (v_i - v_j), t in [0, t_hot]) is likely to put
// vrel inside its LQR-obstacle hull; those pairs are listed (and marked) so
// that k_pair computes them first and their hulls overlap the rest of the
// sweep.  A heuristic for ORDER only: a missed or extra pair changes no
// result, only when its hull starts.
struct PrioArgs {
  int npr, nrows, row_begin, row_stride, X;
  const double* x;
  double t_hot, r2_hot;
  int* list;
  unsigned char* mark;
  int* count;
  int cap;
  int* rowpend;   // early LP: +1 per listed pair (null: off)
  // Qhull order, split hot launch: the last step's inside-hull pairs head the
  // list (k_prio_prev, marked 2 for k_prio) and form the side stream's first
  // hot launch; k_prio's own pairs follow (the main stream's hot launch).
  // null: one hot list
  const int* prev;
  const int* prevn;
  int* hot1n;     // the first launch's pair count
  int* hot2next;  // the second launch's first list position
  // speculative builds: the last step's inside-hull pairs also go straight
  // into the hull queue (hq, hcount); the main hot launch then evaluates the
  // whole list (null: off)
  int* hq;
  int* hcount;
  int hq_cap;
  int* spec_n;   // (the speculative entries' count, for hull_take_job)
};

// the last step's inside-hull pairs at the head of the hot list (one block)
__global__ void __launch_bounds__(256) k_prio_prev(PrioArgs A) {
  const long total = (long)A.nrows * A.npr;
  const int m = min(min(*A.prevn, A.cap), A.hq ? A.hq_cap : A.cap);
  for (int q = threadIdx.x; q < m; q += blockDim.x) {
    const int slot = A.prev[q];
    A.list[q] = slot;
    if (A.hq) A.hq[q] = slot;
    if (slot >= 0 && slot < total) {
      A.mark[slot] = 2;
      if (A.rowpend) atomicAdd(&A.rowpend[slot / A.npr], 1);
    }
  }
  if (threadIdx.x == 0) {
    *A.count = m;
    *A.hot1n = m;
    *A.hot2next = A.hq ? 0 : m;
    if (A.hq) {
      A.hcount[0] = m;   // the queue's count
      A.hcount[1] = m;   // its head, past the entries handed out by spec_next
      *A.spec_n = m;
    }
  }
}

// the step's inside-hull pairs (its hull queue) for the next step's
// k_prio_prev (one block; the order is schedule only): longest build first
// when this step's build records (hbuild: slot | kernel << 40, start, end)
// are given, so that with fewer side workers than builds the short ones
// wait (longest-processing-time-first)
constexpr int kSaveSort = 1024;
__global__ void __launch_bounds__(256) k_prio_save(const int* hq, const int* hcount, int cap_hq, int* prev,
                                                   int* prevn, int cap, const unsigned char* mark,
                                                   const unsigned long long* hbuild,
                                                   const unsigned long long* nbuild, int hbuild_cap,
                                                   const int* hot_list, const int* hot1n, unsigned char* clear,
                                                   long nslots) {
  // (mark: speculative builds on — a queued pair marked 4 was not inside)
  // (clear: the split hot launch's marks — k_prio_prev's 2s are reset here,
  // at the end of their step, so that k_prio never takes a stale 2 of a
  // pair that was inside two steps back but not last step for "listed")
  __shared__ int n;
  __shared__ unsigned long long key[kSaveSort];   // duration << 32 | slot
  __shared__ unsigned long long rec[kSaveSort];   // the builds: duration << 32 | slot
  if (threadIdx.x == 0) n = 0;
  __syncthreads();
  const int c = min(*hcount, cap_hq);
  for (int q = threadIdx.x; q < c; q += blockDim.x) {
    const int slot = hq[q];
    if (slot < 0) continue;
    if (mark && mark[slot] == 4) continue;
    const int at = atomicAdd(&n, 1);
    if (at < cap) prev[at] = slot;
    if (at < kSaveSort) key[at] = (unsigned)slot;
  }
  __syncthreads();
  const int m = min(n, cap);
  const int nb = hbuild ? (int)min(*nbuild, (unsigned long long)hbuild_cap) : 0;
  if (hbuild && m > 1 && m <= kSaveSort && nb <= kSaveSort) {
    for (int k = threadIdx.x; k < nb; k += blockDim.x) {
      const unsigned long long* r = hbuild + 4 * k;
      const unsigned long long d = min(r[2] - r[1], 0x7fffffffull);
      rec[k] = (d << 32) | (unsigned)r[0];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < m; q += blockDim.x) {
      const unsigned slot = (unsigned)key[q];
      unsigned long long d = 0;
      for (int k = 0; k < nb; ++k)
        if ((unsigned)rec[k] == slot) d = max(d, rec[k] >> 32);
      key[q] = (d << 32) | slot;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < m; q += blockDim.x) {
      const unsigned long long kq = key[q];
      int r = 0;
      for (int p = 0; p < m; ++p) r += key[p] > kq;
      prev[r] = (int)(unsigned)kq;
    }
  }
  if (clear) {
    __syncthreads();   // (every mark read above before any is reset)
    const int h = *hot1n;
    for (int q = threadIdx.x; q < h; q += blockDim.x) {
      const int slot = hot_list[q];
      if (slot >= 0 && slot < nslots && clear[slot] == 2) clear[slot] = 0;
    }
  }
  if (threadIdx.x == 0) *prevn = m;
}

__global__ void __launch_bounds__(256) k_prio(PrioArgs A) {
  const long total = (long)A.nrows * A.npr;
  const int lane = threadIdx.x & 63;
  for (long base = (long)blockIdx.x * 256 + (threadIdx.x & ~63); base < total; base += (long)gridDim.x * 256) {
    const long slot = base + lane;
    bool hot = false, pre = false;
    if (slot < total && A.prev) pre = A.mark[slot] == 2;   // listed by k_prio_prev
    if (slot < total && !pre) {
      const int lrow = (int)(slot / A.npr), jj = (int)(slot - (long)lrow * A.npr);
      const int i = A.row_begin + lrow * A.row_stride, j = jj < i ? jj : jj + 1;
      const double* xi = A.x + (size_t)i * A.X;
      const double* xj = A.x + (size_t)j * A.X;
      const double p0 = xi[0] - xj[0], p1 = xi[1] - xj[1], p2 = xi[2] - xj[2];
      const double v0 = xi[3] - xj[3], v1 = xi[4] - xj[4], v2 = xi[5] - xj[5];
      const double vv = v0 * v0 + v1 * v1 + v2 * v2;
      double t = vv > 0.0 ? -(p0 * v0 + p1 * v1 + p2 * v2) / vv : 0.0;
      t = fmin(fmax(t, 0.0), A.t_hot);
      const double e0 = p0 + t * v0, e1 = p1 + t * v1, e2 = p2 + t * v2;
      hot = e0 * e0 + e1 * e1 + e2 * e2 <= A.r2_hot;
    }
    const unsigned long long b = __ballot(hot);
    int pos = 0;
    if (lane == 0 && b) pos = atomicAdd(A.count, __popcll(b));
    pos = __shfl(pos, 0) + __popcll(b & ((1ull << lane) - 1ull));
    if (hot && pos >= A.cap) hot = false;
    if (hot) {
      A.list[pos] = (int)slot;
      if (A.rowpend) atomicAdd(&A.rowpend[slot / A.npr], 1);
    }
    if (slot < total) A.mark[slot] = pre ? 2 : (hot ? 1 : 0);
  }
}
#endif  // LQRO_PAIR_TU

}  // namespace lqro
