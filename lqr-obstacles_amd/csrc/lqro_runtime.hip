// lqro_runtime.hip — liblqro.so: HIP kernels for gfx950 and the C-ABI of
// include/lqro.h.
//
// One control step = the pair loop of LQRObstacles.cpp:1393-1436:
//   k_pair  — one wavefront per ordered pair (i, j): sweep of the H x NP
//             LQR-obstacle point cloud (createObstacle :770-783), reachable
//             filter (:786-812), GJK point-in-hull / distance (:814-864,
//             gjk.cpp:296-501), half-plane (:1208-1221).  Workgroup = one row
//             agent i; its horizon tables live in LDS.
//   k_hull  — inside-hull pairs (queue): in-kernel convex hull of the
//             %g-rounded reachable points, replacing qconvex.exe + files
//             (:867-969).
//   k_lp    — per agent, the fp32 RVO2-3D linear program (:1001-1234).
// k_tables builds the per-agent horizon tables once per set of gains
// (findFG :723-732 and the two factors of createObstacle :771-773).
//
// Exactness: see lqro_device.hpp.  Everything on the pair path is fp64 in the
// reference's operation order, so reachable sets, GJK results and half-planes
// are bit-identical to the reference's CPU path (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/lqro.h"
#include "lqro_device.hpp"
#include "lqro_lp.hpp"
#include "lqro_pair_launch.hpp"
#include "lqro_hull.hpp"
#include "lqro_synth.hpp"
#include "lqro_dyn.hpp"
#include "lqro_kern.hpp"

// hull: 32 counters + 2 words per job; pair: 16; hull wave phases: 16; local hull hand-overs: 16;
// local-hull per-job words 4 x 4096
#define LQRO_PROF_WORDS (32 + 2 * 4096 + 16 + 16 + 16 + 4 * 4096 + 64 + 24 * 1024)   // + 64: k_qhull's wave 1 (Q3_PROF_W1); + 24 x 1024: LQRO_QHULL_LONGPROF
#define LQRO_PROF_HULL_WORDS (32 + 2 * 4096 + 32)   // what lqro_debug_hull_profile returns

using namespace lqro;

// k_pair / k_side for the context's state width and record mode (the
// instantiations live in lqro_pair_inst.hip, one object per combination)
static void launch_pair(int x_dim, dim3 grid, dim3 block, size_t lds, hipStream_t s, const PairArgs& P) {
  const bool r = P.recs != nullptr;
  if (x_dim == 16) {
    if (r) launch_pair_t<16, true>(grid, block, lds, s, P);
    else launch_pair_t<16, false>(grid, block, lds, s, P);
  } else {
    if (r) launch_pair_t<12, true>(grid, block, lds, s, P);
    else launch_pair_t<12, false>(grid, block, lds, s, P);
  }
}
static void launch_side(int x_dim, dim3 grid, dim3 block, hipStream_t s, const HullArgs& H, const PairArgs& P) {
  const bool r = P.recs != nullptr;
  if (x_dim == 16) {
    if (r) launch_side_t<16, true>(grid, block, s, H, P);
    else launch_side_t<16, false>(grid, block, s, H, P);
  } else {
    if (r) launch_side_t<12, true>(grid, block, s, H, P);
    else launch_side_t<12, false>(grid, block, s, H, P);
  }
}

static void launch_qside(int x_dim, dim3 grid, hipStream_t s, const HullArgs& H, const PairArgs& P) {
  const bool r = P.recs != nullptr;
  if (x_dim == 16) {
    if (r) launch_qside_t<16, true>(grid, s, H, P);
    else launch_qside_t<16, false>(grid, s, H, P);
  } else {
    if (r) launch_qside_t<12, true>(grid, s, H, P);
    else launch_qside_t<12, false>(grid, s, H, P);
  }
}

#define LQRO_MAXX 16
constexpr size_t kHullLdsMaxHNP = (size_t)(1 << 19) / HULL_SBMULT;   // 21,845 (C5: H*NP = 20,000)

// ---------------------------------------------------------------------------
// Horizon tables (per agent): T_k = !(C*G_k) (3x3), NCF_k = (-C)*F_k (3xX),
// with F_k, G_k from findFG iterated from F=I, G=0.  One workgroup per agent;
// thread (r, c) owns entry (r, c) of the X x X recursion.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_tables(int X, int U, int H, const double* __restrict__ A,
                                                const double* __restrict__ B,
                                                const double* __restrict__ L,
                                                const double* __restrict__ E, int per_agent,
                                                double* __restrict__ Tout,
                                                double* __restrict__ Nout,
                                                double* __restrict__ Rout,
                                                double* __restrict__ TFout, double rad0,
                                                double rad1, double rad2, double umax,
                                                int* __restrict__ err) {
  __shared__ double sAt[LQRO_MAXX * LQRO_MAXX], sBt[LQRO_MAXX * 3];
  __shared__ double sF[LQRO_MAXX * LQRO_MAXX], sG[LQRO_MAXX * 3];
  __shared__ double sFn[LQRO_MAXX * LQRO_MAXX], sGn[LQRO_MAXX * 3];
  __shared__ double sA[LQRO_MAXX * LQRO_MAXX], sB[LQRO_MAXX * 4], sL[4 * LQRO_MAXX], sE[4 * 3];
  const int agent = blockIdx.x;
  const double* Li = L + (per_agent ? (size_t)agent * U * X : 0);
  const double* Ei = E + (per_agent ? (size_t)agent * U * 3 : 0);
  const int t = threadIdx.x;
  for (int q = t; q < X * X; q += blockDim.x) sA[q] = A[q];
  for (int q = t; q < X * U; q += blockDim.x) sB[q] = B[q];
  for (int q = t; q < U * X; q += blockDim.x) sL[q] = Li[q];
  for (int q = t; q < U * 3; q += blockDim.x) sE[q] = Ei[q];
  __syncthreads();
  const int r = t / X, c = t % X;
  const bool act = t < X * X;
  if (act) {
    // Atilde = A + (B*L), Btilde = B*E   (LQRObstacles.cpp:725-728)
    double bl = 0.0;
    for (int k = 0; k < U; ++k) bl += sB[r * U + k] * sL[k * X + c];
    sAt[r * X + c] = sA[r * X + c] + bl;
    if (c < 3) {
      double be = 0.0;
      for (int k = 0; k < U; ++k) be += sB[r * U + k] * sE[k * 3 + c];
      sBt[r * 3 + c] = be;
    }
    sF[r * X + c] = (r == c) ? 1.0 : 0.0;   // Ft = identity (:1401)
    if (c < 3) sG[r * 3 + c] = 0.0;          // Gt = zeros   (:1402)
  }
  __syncthreads();
  double* Ta = Tout + (size_t)agent * H * 9;
  double* Na = Nout + (size_t)agent * H * 3 * X;
  for (int k = 0; k < H; ++k) {
    if (act) {
      double f = 0.0;
      for (int m = 0; m < X; ++m) f += sAt[r * X + m] * sF[m * X + c];
      sFn[r * X + c] = f;
      if (c < 3) {
        double g = 0.0;
        for (int m = 0; m < X; ++m) g += sAt[r * X + m] * sG[m * 3 + c];
        sGn[r * 3 + c] = g + sBt[r * 3 + c];
      }
    }
    __syncthreads();
    if (act) {
      sF[r * X + c] = sFn[r * X + c];
      if (c < 3) sG[r * 3 + c] = sGn[r * 3 + c];
    }
    __syncthreads();
    // NCF_k = (-C)*F_k, entries of -C are -1.0 / -0.0 (:773)
    if (t < 3 * X) {
      const int rr = t / X, cc = t % X;
      double s = 0.0;
      for (int m = 0; m < X; ++m) {
        double nc = (m == rr) ? -1.0 : -0.0;
        s += nc * sF[m * X + cc];
      }
      Na[(size_t)k * 3 * X + rr * X + cc] = s;
    }
    if (t == 0) {
      // T_k = !(C*G_k)  (:771)
      double cg[9], inv[9];
      for (int rr = 0; rr < 3; ++rr)
        for (int cc = 0; cc < 3; ++cc) {
          double s = 0.0;
          for (int m = 0; m < X; ++m) s += ((m == rr) ? 1.0 : 0.0) * sG[m * 3 + cc];
          cg[rr * 3 + cc] = s;
        }
      inverse3(cg, inv);
      for (int q = 0; q < 9; ++q) {
        Ta[(size_t)k * 9 + q] = inv[q];
        if (!isfinite(inv[q])) atomicOr(err, 1);
      }
      // slice bounds for k_pair: |T_k s_p| <= ||T_k diag(rad)||_F * max|u_p|
      const double rad[3] = {rad0, rad1, rad2};
      double fr = 0.0, ff = 0.0;
      for (int rr = 0; rr < 3; ++rr)
        for (int cc = 0; cc < 3; ++cc) {
          const double tv = inv[rr * 3 + cc];
          fr += (tv * rad[cc]) * (tv * rad[cc]);
          ff += tv * tv;
        }
      Rout[(size_t)agent * H + k] = sqrt(fr) * umax * (1.0 + 1e-12);
      TFout[(size_t)agent * H + k] = sqrt(ff);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// LP kernel: one wavefront per row agent (lqro_lp.hpp), fp32 as the reference
// ---------------------------------------------------------------------------
struct LpArgs {
  int npr, nrows, row_begin, row_stride;
  double vmax;
  const float* slots;   // per row npr x 8 (flag in [6]: 1 = plane)
  float* compact;       // per row npr x 8: emitted planes in j order
  float* proj;          // per row npr x 8: linearProgram4's projected planes
  const double* vgoal;
  double* newv;
  unsigned long long* prof;   // LQRO_LP_PROFILE: cycles per row
  // rows whose linearProgram3 fails go to k_lp4 (null: linearProgram4 inline)
  int* lp4_list;              // 6 ints per row: lrow, fail, m, nv.xyz (float bits)
  int* lp4_count;
  int* lp4_next;
  // early LP (lqro_hull.hpp hull_row_done): mode 1 runs the rows whose
  // count reached row_target and that it claims; mode 2 (the tail) skips the
  // rows claimed earlier.  rowclaim null: every row.
  const int* rowpend;
  int* rowclaim;
  int row_target;
  int mode;
};

// one row's LP; `planes` holds its compacted plane list (stride PS floats:
// 6 in LDS, 8 in global memory)
template <int PS>
__device__ __forceinline__ void lp_row(const LpArgs& A, int lrow, float* planes, int lane) {
  const int i = A.row_begin + lrow * A.row_stride;
  const int m = lp_compact<PS>(A.slots + (size_t)lrow * A.npr * 8, A.npr, planes, lane);
  const v3 pref = V3((float)A.vgoal[3 * i], (float)A.vgoal[3 * i + 1], (float)A.vgoal[3 * i + 2]);
  v3 nv = V3(0.0f, 0.0f, 0.0f);
  const int fail = w_lp3<PS>(planes, m, A.vmax, pref, false, nv, lane);          // :1228
#ifdef LQRO_LP_PROFILE
  int lp4_iters = 0;
  if (fail < m)
    w_lp4<PS>(planes, m, fail, (float)A.vmax, nv, A.proj + (size_t)lrow * A.npr * PS, lane, lp4_iters);
  if (lane == 0 && A.prof && lrow < 4096) A.prof[32 + 4096 + lrow] = ((unsigned long long)m << 40) |
                                               ((unsigned long long)fail << 20) | (unsigned)lp4_iters;
#else
  if (fail < m && A.lp4_list != nullptr) {
    // linearProgram4 (:1230) in k_lp4, with its projected planes in LDS too:
    // hand over the compacted planes (stride PS) and linearProgram3's result
    float* dst = A.compact + (size_t)lrow * A.npr * 8;
    if (dst != planes)
      for (int q = lane; q < PS * m; q += 64) dst[q] = planes[q];
    if (lane == 0) {
      const int k = atomicAdd(A.lp4_count, 1);
      int* e = A.lp4_list + 6 * (size_t)k;
      e[0] = lrow; e[1] = fail; e[2] = m;
      e[3] = __float_as_int(nv.x); e[4] = __float_as_int(nv.y); e[5] = __float_as_int(nv.z);
    }
    return;
  }
  if (fail < m)
    w_lp4<PS>(planes, m, fail, (float)A.vmax, nv, A.proj + (size_t)lrow * A.npr * PS, lane);  // :1230
#endif
  if (lane == 0) {
    A.newv[3 * i] = nv.x;
    A.newv[3 * i + 1] = nv.y;
    A.newv[3 * i + 2] = nv.z;
  }
}

// plane list in global scratch (rows with more planes than LDS holds)
__global__ void __launch_bounds__(256) k_lp(LpArgs A) {
  const int lane = threadIdx.x & 63;
  const int lrow = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (lrow >= A.nrows) return;
  lp_row<8>(A, lrow, A.compact + (size_t)lrow * A.npr * 8, lane);
}

// one wave per workgroup, the row's plane list in LDS (the LP rescans it for
// every violated plane: LDS round trips instead of L2 ones), 32 B a plane
// (16-B aligned loads) up to 2,048 planes, 24 B beyond (C4: 4,095)
template <int PS>
__global__ void __launch_bounds__(64) k_lp_lds(LpArgs A) {
  extern __shared__ float lp_planes[];
  const int lrow = blockIdx.x;
  if (lrow >= A.nrows) return;
  if (A.rowclaim) {
    int go;
    if (A.mode == 1) {
      go = 0;
      if (threadIdx.x == 0)
        go = __hip_atomic_load(A.rowpend + lrow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == A.row_target &&
             atomicCAS(A.rowclaim + lrow, 0, 1) == 0;
      go = __builtin_amdgcn_readfirstlane(go);
      __threadfence();   // the row's planes (acquire)
    } else {
      go = A.rowclaim[lrow] != 1;
    }
    if (!go) return;
  }
#ifdef LQRO_LP_PROFILE
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
  lp_row<PS>(A, lrow, lp_planes, threadIdx.x);
#ifdef LQRO_LP_PROFILE
  if (threadIdx.x == 0 && lrow < 8192) A.prof[32 + lrow] = __builtin_amdgcn_s_memtime() - t0;
#endif
}

// linearProgram4 for the rows k_lp_lds listed (one wave per row): the planes
// in LDS, and their projections too when both fit (else the projections in
// global memory), so the O(m^2) rescans of linearProgram4's inner
// linearProgram3 stay out of L2
template <int PS>
__global__ void __launch_bounds__(64) k_lp4(LpArgs A, int proj_in_lds) {
  extern __shared__ float lp4_sm[];
  float* planes = lp4_sm;
  const int lane = threadIdx.x;
  {
    // one workgroup per listed row (a persistent loop over the list around
    // these ballot-driven loops hung on gfx950; the extra workgroups exit at once)
    const int job = blockIdx.x;
    if (job >= *A.lp4_count) return;
    const int* e = A.lp4_list + 6 * (size_t)job;
    const int lrow = e[0], fail = e[1], m = e[2];
    float* proj = proj_in_lds ? lp4_sm + (size_t)A.npr * PS : A.proj + (size_t)lrow * A.npr * PS;
    v3 nv = V3(__int_as_float(e[3]), __int_as_float(e[4]), __int_as_float(e[5]));
    const float* src = A.compact + (size_t)lrow * A.npr * 8;
    for (int q = lane; q < PS * m; q += 64) planes[q] = src[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#ifdef LQRO_LP_PROFILE
    int lp4_iters = 0;
    w_lp4<PS>(planes, m, fail, (float)A.vmax, nv, proj, lane, lp4_iters);  // :1230
#else
    w_lp4<PS>(planes, m, fail, (float)A.vmax, nv, proj, lane);              // :1230
#endif
    if (lane == 0) {
      const int i = A.row_begin + lrow * A.row_stride;
      A.newv[3 * i] = nv.x;
      A.newv[3 * i + 1] = nv.y;
      A.newv[3 * i + 2] = nv.z;
    }
  }
}

constexpr size_t kLpLdsMax = 160 * 1024;   // one CU's LDS

// lqro_step_device_end after an early LP in _begin: the rows it ran (claimed
// 1) have their newV in the context's buffer; the tail wrote the others
__global__ void __launch_bounds__(256) k_copy_claimed(const int* rowclaim, int nrows, int rb, int rs,
                                                      const double* src, double* dst) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows || rowclaim[r] != 1) return;
  const size_t i = (size_t)rb + (size_t)r * rs;
  dst[3 * i] = src[3 * i];
  dst[3 * i + 1] = src[3 * i + 1];
  dst[3 * i + 2] = src[3 * i + 2];
}

template <int PS>
static hipError_t launch_lp_lds(LpArgs La, hipStream_t s) {
  const size_t lds = (size_t)La.npr * 4 * PS;
  hipError_t e = hipFuncSetAttribute((const void*)k_lp_lds<PS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)kLpLdsMax);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_lp_lds<PS>, dim3((unsigned)La.nrows), dim3(64), lds, s, La);
  e = hipGetLastError();
  if (e != hipSuccess || La.lp4_list == nullptr) return e;
  e = hipFuncSetAttribute((const void*)k_lp4<PS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLpLdsMax);
  if (e != hipSuccess) return e;
  const int proj_in_lds = 2 * lds <= kLpLdsMax;
  hipLaunchKernelGGL(k_lp4<PS>, dim3((unsigned)La.nrows), dim3(64), proj_in_lds ? 2 * lds : lds, s, La,
                     proj_in_lds);
  return hipGetLastError();
}

// La.lp4_count / lp4_next must be zero (or lp4_list null)
static hipError_t launch_lp(LpArgs La, hipStream_t s) {
  if ((size_t)La.npr * 32 <= 64 * 1024) return launch_lp_lds<8>(La, s);
  if ((size_t)La.npr * 24 <= kLpLdsMax) return launch_lp_lds<6>(La, s);
  La.lp4_list = nullptr;
  hipLaunchKernelGGL(k_lp, dim3((unsigned)((La.nrows + 3) / 4)), dim3(256), 0, s, La);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Host side: context + C-ABI
// ---------------------------------------------------------------------------
struct lqro_ctx {
  lqro_config cfg;
  double *d_R, *d_TF, umax;
  unsigned long long* d_shash;
  int rb, re, rs, nrows, npr;   // rows rb, rb + rs, ... < re
  int have_gains, per_agent;
  hipStream_t stream;
  hipEvent_t ev[5];
  hipStream_t side;          // k_hull workers running beside k_pair
  hipEvent_t xev[2];         // cross-stream ordering (no timing)
  double *d_T, *d_NCF, *d_S, *d_x, *d_vgoal, *d_newv;
  double *d_A, *d_B, *d_L, *d_E;
  float *d_planes, *d_lpscratch, *d_lpcompact;
  lqro_pair_record* d_recs;
  int *d_hq, *d_hcount, *d_hnext, *d_err, *d_rq;
  void* d_hbig;
  HullWide* d_hwide;
  int* d_hbag;
  int* d_lp4;                // k_lp_lds -> k_lp4 row list (6 ints per row)
  int* d_hotlist;            // k_prio: likely inside-hull pairs (slots), computed first
  int* d_prevq;              // Qhull order: the last step's inside-hull pairs (k_prio_save), hot_cap
  int* d_hot2;               // [0] their count, [1] first hot launch's count, [2] its next, [3] the
                             // second's next, [4] its finished workgroups
  int hot_split;             // LQRO_HOT_SPLIT (default 1): the split hot launch in Qhull order
  int qside_pct;             // LQRO_QHULL_SIDE_PCT: side CUs per 100 of the last step's inside-hull pairs (default 100)
  int qhull_inline;          // LQRO_QHULL_INLINE_BIG: k_qhull rebuilds a capped build in place (default 1)
  int qhull_flags;           // LQRO_QHULL_FLAGS: k_qhull's helper waves (1), emit lane state (2), queue pre-scan (4),
                             // a long emit over the waves (16); default 23
  int qbalance;              // LQRO_QHULL_BALANCE: the side's width from the measured work (default 1)
  int qspare;                // LQRO_QHULL_SPARE: side CUs beyond the last step's inside-hull count (default 4; -1: count/16 + 4)
  int hot_spec;              // LQRO_HOT_SPEC (default 1): with the split, the last step's inside pairs are built speculatively from the step's start
  unsigned char* d_hotmark;  // per slot: in the hot list
  int* d_nbrlist;            // culling on: per row K neighbour slots (lqro_set_neighbors)
  double nbr_r2;
  int nbr_k, nbr_cap;         // k; rows x nbr_cap ints allocated
  int hot_cap;
  int hot_on;                // LQRO_HOT (default 1)
  int hull_big_only;         // LQRO_HULL_BIG: skip the LDS hull (A/B)
  int local_hull;            // LQRO_LOCAL_HULL (default 1): k_lhull first, k_hull for what it hands over
  int* d_lq;                 // k_lhull -> k_hull queue
  int lside_cus;             // side CUs with the local hull (LQRO_LOCAL_SIDE_CUS, default 3/16 of the CUs)
  double hot_t, hot_r;       // k_prio horizon (s) and radius (m): LQRO_HOT_T, LQRO_HOT_R
  // inside-hull pairs of an earlier step (pinned, copied at the end of each
  // step; ~0 = none yet) size the side stream: beyond 2 per side CU it widens
  // by a third (at most half the CUs), beyond 4 per (widened) side CU the
  // side CUs cannot keep up with the hulls and the plain schedule (every CU
  // on the hulls after the sweep) is faster (scripts/crowded.py)
  unsigned long long* h_inside;   // 2 pinned slots of 8 words: step t writes slot t & 1: inside-hull
                                  //   pairs, then LQRO_ST_SWORK, _BWORK, _BMAX (100 MHz ticks),
                                  //   then LQRO_ST_RETRY (builds past k_qhull's caps)
  hipEvent_t iev[2];              // recorded after the copy into slot k
  long long nstep;                // steps enqueued
  long hot_max_inside;       // LQRO_HOT_MAX_INSIDE (-1: 4 x the side CUs)
  int hull_big_blocks;
  int n_cu;
  int side_cus;              // CUs running k_hull beside k_pair (LQRO_SIDE_HULL_CUS)
  double* d_hscratch;
  int* d_hiscratch;
  float* d_hfscratch;
  unsigned long long* d_hfbest;
  int *d_hvpid, *d_hstack;
  void* d_hfaces;
  int hull_blocks, hull_cap;
  unsigned long long* d_stats;
  unsigned long long* d_prof;
  int lds_bytes;
  int stepped;               // a step was enqueued (ev[3] recorded)
  int pending;               // lqro_step_device_begin ran, _end not yet
  const double* pend_x;
  const double* pend_vgoal;
  hipStream_t pend_stream;
  int lhull_prof;            // LQRO_LHULL_PROFILE: k_lhull writes its per-job words
  // LQRO_FLAG_QHULL_ORDER: k_qhull workers, per-slot normals, facet-0 slots,
  // the loop-carried normal in [0..2], out [3..5]
  int qhull_order;
  int qhull_big;            // LQRO_QHULL_BIG=1: every pair in k_qhull_big (A/B runs)
  int qworkers;
  size_t qstride;
  char* d_qscratch;
  double* d_qnrm;
  int* d_qstale;
  unsigned long long* d_hbuild;   // LQRO_HBUILD_CAP x 4 words: the builds' timing records
  double* d_carry;
  // early LP (LQRO_EARLY_LP, default 1): per row open work and LP claim
  // (lqro_hull.hpp hull_row_done)
  int early_lp;
  int early_step;            // the step being enqueued runs the early LP
  int early_internal;        // ... into d_newv (lqro_step_device_begin: the caller's buffer comes with _end)
  int qside;                 // LQRO_QSIDE=1: k_qhull side workers sweep rows after their builds (default off)
  int* d_rowpend;
  int* d_rowclaim;
  PairArgs pa;
};

// the last step's final event was recorded on whichever stream it was
// enqueued on (the caller's for lqro_step_device): wait on that, not on
// c->stream; a context that never stepped has nothing to wait for
static hipError_t wait_last_step(lqro_ctx* c) {
  if (!c->stepped) return hipStreamSynchronize(c->stream);
  return hipEventSynchronize(c->ev[3]);
}

#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "liblqro: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, \
              __LINE__);                                                                 \
      return LQRO_E_HIP;                                                                 \
    }                                                                                    \
  } while (0)

extern "C" {

int lqro_version(void) { return 1; }

const char* lqro_status_string(int s) {
  switch (s) {
    case LQRO_OK: return "ok";
    case LQRO_E_ARG: return "bad argument";
    case LQRO_E_HIP: return "HIP runtime error";
    case LQRO_E_NOMEM: return "out of memory";
    case LQRO_E_STATE: return "call order violated";
    case LQRO_E_SINGULAR: return "singular C*G_k";
    case LQRO_E_NODEVICE: return "no gfx950 device";
    case LQRO_E_OVERFLOW: return "work queue overflow";
    case LQRO_E_HULL: return "an inside-hull pair's hull could not be built (degenerate input or capacity; lqro_get_hull_failures)";
    case LQRO_E_QHMERGE:
      return "an inside-hull pair's winning facet may be one qconvex's pre-merge joins: its half-plane is not pinned "
             "to the reference (LQRO_REC_QHMERGE_WIN; lqro_get_qhmerge_pairs)";
  }
  return "unknown";
}

void lqro_config_default(lqro_config* c, int32_t n, int32_t h, int32_t np) {
  c->n_agents = n;
  c->x_dim = 16;
  c->u_dim = 4;
  c->horizon = h;
  c->n_points = np;
  c->min_reach = 4;
  c->xy_radius = 0.26;
  c->z_radius = 0.75;
  c->vmax_reach = 30.0;
  c->vmax_lp = 100.0;
  c->row_begin = 0;
  c->row_end = 0;
  c->row_stride = 0;
  c->device = 0;
  c->flags = LQRO_FLAG_QHULL_ORDER;   // the reference's own inside-hull rule (drop-in default)
}

void lqro_destroy(lqro_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->cfg.device);
  void* ps[] = {c->d_R, c->d_TF, c->d_shash, c->d_T, c->d_NCF, c->d_S, c->d_x, c->d_vgoal, c->d_newv, c->d_A, c->d_B,
                c->d_L, c->d_E, c->d_planes, c->d_lpscratch, c->d_lpcompact, c->d_recs, c->d_hq, c->d_hcount,
                c->d_err, c->d_hfaces, /* d_hnext points into d_hcount */ c->d_hscratch, c->d_hiscratch, c->d_hfscratch, c->d_stats, c->d_prof, c->d_rq, c->d_hbig, c->d_hwide, c->d_hbag, c->d_lp4, c->d_hotlist, c->d_hotmark, c->d_nbrlist, c->d_hfbest, c->d_hvpid, c->d_hstack, c->d_lq,
                c->d_qscratch, c->d_qnrm, c->d_qstale, c->d_hbuild, c->d_carry, c->d_rowpend /* d_rowclaim inside */,
                c->d_prevq, c->d_hot2};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  for (int k = 0; k < 5; ++k)
    if (c->ev[k]) (void)hipEventDestroy(c->ev[k]);
  for (int k = 0; k < 2; ++k) {
    if (c->xev[k]) (void)hipEventDestroy(c->xev[k]);
    if (c->iev[k]) (void)hipEventDestroy(c->iev[k]);
  }
  if (c->h_inside) (void)hipHostFree(c->h_inside);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

static int ctx_alloc(lqro_ctx* c) {
  const lqro_config& g = c->cfg;
  const size_t N = g.n_agents, X = g.x_dim, H = g.horizon, NP = g.n_points;
  const size_t slots = (size_t)c->nrows * c->npr;
  HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  for (int k = 0; k < 5; ++k) HIPCHK(hipEventCreate(&c->ev[k]));
  HIPCHK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
  for (int k = 0; k < 2; ++k) HIPCHK(hipEventCreateWithFlags(&c->xev[k], hipEventDisableTiming));
  HIPCHK(hipMalloc(&c->d_S, sizeof(double) * NP * 3));
  HIPCHK(hipMalloc(&c->d_x, sizeof(double) * N * X));
  HIPCHK(hipMalloc(&c->d_vgoal, sizeof(double) * N * 3));
  HIPCHK(hipMalloc(&c->d_newv, sizeof(double) * N * 3));
  HIPCHK(hipMalloc(&c->d_A, sizeof(double) * X * X));
  HIPCHK(hipMalloc(&c->d_B, sizeof(double) * X * g.u_dim));
  HIPCHK(hipMalloc(&c->d_L, sizeof(double) * N * g.u_dim * X));
  HIPCHK(hipMalloc(&c->d_E, sizeof(double) * N * g.u_dim * 3));
  HIPCHK(hipMalloc(&c->d_T, sizeof(double) * N * H * 9));
  HIPCHK(hipMalloc(&c->d_NCF, sizeof(double) * N * H * 3 * X));
  HIPCHK(hipMalloc(&c->d_R, sizeof(double) * N * H));
  HIPCHK(hipMalloc(&c->d_TF, sizeof(double) * N * H));
  HIPCHK(hipMalloc(&c->d_shash, sizeof(unsigned long long) * H));
  HIPCHK(hipMalloc(&c->d_planes, sizeof(float) * 8 * (slots ? slots : 1)));
  HIPCHK(hipMalloc(&c->d_lpscratch, sizeof(float) * 8 * (slots ? slots : 1)));
  HIPCHK(hipMalloc(&c->d_lpcompact, sizeof(float) * 8 * (slots ? slots : 1)));
  if (g.flags & LQRO_FLAG_RECORDS)
    HIPCHK(hipMalloc(&c->d_recs, sizeof(lqro_pair_record) * (slots ? slots : 1)));
  // one entry per slot: a pair enqueues at most one hull job per step, so the
  // queue cannot overflow (C5's 2048 x 16383-slot shard: 134 MB, of 288 GB)
  c->hull_cap = (int)(slots > 0 ? slots : 1);
  HIPCHK(hipMalloc(&c->d_hq, sizeof(int) * c->hull_cap));
  // hull count, next, retry count, retry next, pair rows, -, hot count, hot next, -, lp4 count, lp4 next,
  // local-hull hand-over count, its next, local-hull decided
  HIPCHK(hipMalloc(&c->d_hcount, sizeof(int) * 16));
  c->d_hnext = c->d_hcount + 1;
  HIPCHK(hipMalloc(&c->d_rq, sizeof(int) * c->hull_cap));
  HIPCHK(hipMalloc(&c->d_lq, sizeof(int) * c->hull_cap));
  HIPCHK(hipMalloc(&c->d_err, sizeof(int)));
  HIPCHK(hipMalloc(&c->d_stats, sizeof(unsigned long long) * LQRO_ST_WORDS));
  HIPCHK(hipHostMalloc((void**)&c->h_inside, 16 * sizeof(unsigned long long), hipHostMallocDefault));
  for (int k = 0; k < 16; ++k) c->h_inside[k] = k % 8 ? 0ull : ~0ull;
  for (int k = 0; k < 2; ++k) HIPCHK(hipEventCreateWithFlags(&c->iev[k], hipEventDisableTiming));
  HIPCHK(hipMalloc(&c->d_prof, sizeof(unsigned long long) * LQRO_PROF_WORDS));
  HIPCHK(hipMemset(c->d_prof, 0, sizeof(unsigned long long) * LQRO_PROF_WORDS));
  c->hull_blocks = 256;   // one 138 KB-LDS workgroup per CU, persistent over the queue
  HIPCHK(hipMalloc(&c->d_hscratch, sizeof(double) * 6 * H * NP * c->hull_blocks));
  HIPCHK(hipMalloc(&c->d_hiscratch, sizeof(int) * 2 * H * NP * HULL_SCR_WAVES * c->hull_blocks));
  HIPCHK(hipMalloc(&c->d_hfscratch, sizeof(float) * H * NP * HULL_WAVES * c->hull_blocks));
  HIPCHK(hipMalloc(&c->d_hfbest, sizeof(unsigned long long) * HULL_FB_STRIDE * (size_t)c->hull_blocks));
  HIPCHK(hipMalloc(&c->d_hvpid, sizeof(int) * HULL_VG_STRIDE * (size_t)c->hull_blocks));
  HIPCHK(hipMalloc(&c->d_hstack, sizeof(int) * HULL_STKMULT * H * NP * (size_t)c->hull_blocks));
  HIPCHK(hipMalloc(&c->d_hfaces, sizeof(HullPt) * HULL_SBMULT * H * NP * (size_t)c->hull_blocks));
  c->hull_big_blocks = c->n_cu;   // one 1-inserting-wave hull per CU (topology in global memory)
  HIPCHK(hipMalloc(&c->d_hbig, sizeof(HullMemBig) * (size_t)c->hull_big_blocks));
  HIPCHK(hipMalloc(&c->d_hwide, sizeof(HullWide) * HULL_CWAVES * (size_t)c->hull_blocks));
  HIPCHK(hipMalloc(&c->d_hbag, sizeof(int) * HULL_BAGCAP * (size_t)c->hull_blocks));
  HIPCHK(hipMemset(c->d_hbag, 0xFF, sizeof(int) * HULL_BAGCAP * (size_t)c->hull_blocks));
  c->hot_cap = (int)std::max<size_t>(16384, slots / 32);
  HIPCHK(hipMalloc(&c->d_hotlist, sizeof(int) * c->hot_cap));
  HIPCHK(hipMalloc(&c->d_hotmark, slots ? slots : 1));
  // (k_prio keeps a mark of 2 it finds — k_prio_prev's "listed" — so the marks
  // start at 0: the first split step after the plain ones would otherwise
  // take recycled device memory's bytes for marks and skip those pairs)
  HIPCHK(hipMemset(c->d_hotmark, 0, slots ? slots : 1));
  HIPCHK(hipMalloc(&c->d_lp4, sizeof(int) * 6 * (size_t)std::max(1, c->nrows)));
  HIPCHK(hipMalloc(&c->d_carry, sizeof(double) * 6));
  HIPCHK(hipMalloc(&c->d_rowpend, sizeof(int) * 2 * (size_t)std::max(1, c->nrows)));
  c->d_rowclaim = c->d_rowpend + std::max(1, c->nrows);
  HIPCHK(hipMemset(c->d_carry, 0, sizeof(double) * 6));
  HIPCHK(hipMemset(c->d_lp4, 0, sizeof(int) * 6 * (size_t)std::max(1, c->nrows)));
  HIPCHK(hipMemset(c->d_rowpend, 0, sizeof(int) * 2 * (size_t)std::max(1, c->nrows)));
  if (c->qhull_order) {
    // k_qhull: one one-wave worker per CU (the build's facets fill the CU's
    // LDS), each with its own build scratch
    c->qworkers = c->n_cu;
    c->qstride = (qhull_worker_bytes((int)(H * NP)) + 255) & ~(size_t)255;
    HIPCHK(hipMalloc(&c->d_qscratch, c->qstride * (size_t)c->qworkers));
    HIPCHK(hipMemset(c->d_qscratch, 0, c->qstride * (size_t)c->qworkers));   // k_qhull_big's visit stamps
    HIPCHK(hipMalloc(&c->d_qnrm, sizeof(double) * 4 * (slots ? slots : 1)));
    HIPCHK(hipMalloc(&c->d_qstale, sizeof(int) * (slots ? slots : 1)));
    HIPCHK(hipMalloc(&c->d_hbuild, sizeof(unsigned long long) * 4 * LQRO_HBUILD_CAP));
    HIPCHK(hipMalloc(&c->d_prevq, sizeof(int) * (size_t)c->hot_cap));
    HIPCHK(hipMalloc(&c->d_hot2, sizeof(int) * 8));
    HIPCHK(hipMemset(c->d_hot2, 0, sizeof(int) * 8));
    HIPCHK(hipMemset(c->d_prevq, 0xFF, sizeof(int) * (size_t)c->hot_cap));
    HIPCHK(hipMemset(c->d_qstale, 0xFF, sizeof(int) * (slots ? slots : 1)));
    HIPCHK(hipMemset(c->d_hbuild, 0, sizeof(unsigned long long) * 4 * LQRO_HBUILD_CAP));
  }
  return LQRO_OK;
}

int lqro_create(const lqro_config* cfg, lqro_ctx** out) {
  if (!cfg || !out) return LQRO_E_ARG;
  *out = nullptr;
  const lqro_config& g = *cfg;
  if (g.n_agents < 2 || (g.x_dim != 16 && g.x_dim != 12) || g.u_dim != 4 || g.horizon < 1 ||
      g.n_points < 1 || g.vmax_reach <= 0 || g.n_points > 64 * kMaxPW || g.horizon > 64 * kMaxKS)
    return LQRO_E_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= g.device) return LQRO_E_NODEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, g.device) != hipSuccess) return LQRO_E_NODEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    fprintf(stderr, "liblqro: device %d is %s, built for gfx950\n", g.device, prop.gcnArchName);
    return LQRO_E_NODEVICE;
  }
  if (hipSetDevice(g.device) != hipSuccess) return LQRO_E_HIP;
  lqro_ctx* c = new (std::nothrow) lqro_ctx;
  if (!c) return LQRO_E_NOMEM;
  memset(c, 0, sizeof *c);
  c->cfg = g;
  c->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  c->qhull_order = (g.flags & LQRO_FLAG_QHULL_ORDER) ? 1 : 0;
  {
    const char* qb = getenv("LQRO_QHULL_BIG");
    c->qhull_big = qb ? atoi(qb) != 0 : 0;
  }
  {
    // CUs running k_hull workers beside k_pair (the hot-pair hulls); default 3/8
    const char* e = getenv("LQRO_SIDE_HULL_CUS");
    c->side_cus = e ? atoi(e) : (3 * c->n_cu) / 8;
    if (c->side_cus < 0) c->side_cus = 0;
    if (c->side_cus > c->n_cu / 2) c->side_cus = c->n_cu / 2;
    const char* hb = getenv("LQRO_HULL_BIG");   // every hull job in k_hull_big (A/B runs)
    c->hull_big_only = hb ? atoi(hb) != 0 : 0;
    const char* lh = getenv("LQRO_LOCAL_HULL");
    c->local_hull = lh ? atoi(lh) != 0 : 1;
    const char* ls = getenv("LQRO_LOCAL_SIDE_CUS");
    c->lside_cus = ls ? atoi(ls) : (3 * c->n_cu) / 16;
    if (c->lside_cus < 0) c->lside_cus = 0;
    if (c->lside_cus > c->n_cu / 2) c->lside_cus = c->n_cu / 2;
    const char* h = getenv("LQRO_HOT");
    c->hot_on = h ? atoi(h) != 0 : 1;
    const char* ht = getenv("LQRO_HOT_T");
    const char* hr = getenv("LQRO_HOT_R");
    c->hot_t = ht ? atof(ht) : 3.0;
    c->hot_r = hr ? atof(hr) : 3.0;
    const char* lp = getenv("LQRO_LHULL_PROFILE");
    c->lhull_prof = lp ? atoi(lp) != 0 : 0;
    const char* hm = getenv("LQRO_HOT_MAX_INSIDE");
    c->hot_max_inside = hm ? atol(hm) : -1L;
    const char* el = getenv("LQRO_EARLY_LP");
    c->early_lp = el ? atoi(el) != 0 : 1;
    // Qhull order: the last step's inside-hull pairs in a hot launch of their
    // own on the side stream, so the builds start when they are found rather
    // than behind the other hot pairs' stragglers (which go to the main stream)
    const char* hs = getenv("LQRO_HOT_SPLIT");
    c->hot_split = hs ? atoi(hs) != 0 : 1;
    const char* hp = getenv("LQRO_HOT_SPEC");
    c->hot_spec = hp ? atoi(hp) != 0 : 1;
    const char* qsp = getenv("LQRO_QHULL_SPARE");
    c->qspare = qsp ? atoi(qsp) : 4;
    const char* qpc = getenv("LQRO_QHULL_SIDE_PCT");
    c->qside_pct = qpc ? std::max(1, std::min(100, atoi(qpc))) : 100;
    // off by default: with 3 waves a CU the side workers sweep rows at ~1/5 of a
    // 16-wave workgroup's rate, so where the sweep outlasts the builds (C4:
    // 227 vs 114 ms per step) it loses; at C3 it ties (22.0 ms either way)
    const char* qs = getenv("LQRO_QSIDE");
    c->qside = qs ? atoi(qs) != 0 : 0;
    // a build past k_qhull's caps rebuilt at once on its CU (q3_big_inline)
    // instead of in the k_qhull_big launch after the sweep
    const char* qi = getenv("LQRO_QHULL_INLINE_BIG");
    c->qhull_inline = qi ? atoi(qi) != 0 : 1;
    const char* qf = getenv("LQRO_QHULL_FLAGS");
    c->qhull_flags = qf ? atoi(qf) : 23;
    // the side's width from the measured work of the step two before (the
    // sweep's CU time, the builds' total and longest): no wider than leaves
    // the sweep no longer than the builds (LQRO_QHULL_BALANCE=0: one CU per
    // expected build, round 5's rule)
    const char* qbal = getenv("LQRO_QHULL_BALANCE");
    c->qbalance = qbal ? atoi(qbal) != 0 : 1;
  }
  c->rb = g.row_begin;
  c->re = (g.row_end > g.row_begin) ? g.row_end : g.n_agents;
  if (g.row_end == 0 && g.row_begin == 0) { c->rb = 0; c->re = g.n_agents; }
  c->rs = g.row_stride > 1 ? g.row_stride : 1;
  if (c->rb < 0 || c->re > g.n_agents || c->rb >= c->re || g.row_stride < 0) { delete c; return LQRO_E_ARG; }
  c->nrows = (c->re - c->rb + c->rs - 1) / c->rs;
  c->npr = g.n_agents - 1;
  // LDS layout of k_pair (in doubles): block tables, then one region per wave
  const int H = g.horizon, NP = g.n_points, X = g.x_dim, XP = X + 1;
  if (NP > 64 * kMaxPW || H > 64 * kMaxKS) { delete c; return LQRO_E_ARG; }
  int off = 0;
  PairArgs& P = c->pa;
  P.XP = XP;
  P.PW = (NP + 63) / 64;
  P.lds_T = off; off += H * 9;
  P.lds_N = off; off += H * 3 * XP;
  P.lds_S = off; off += 3 * NP;
  P.lds_R = off; off += H;
  P.lds_TF = off; off += H;
  P.lds_H = off; off += H;
  P.lds_wave = off;
  // tr 3H, sc H, mask H*PW (u64), cls/cnt/mixed 3H ints (mixed padded to
  // even), GJK simplex 18, statistics 5
  P.wave_doubles = 4 * H + H * P.PW + H + (H + (H & 1)) / 2 + 18 + 5;
  const int budget = 160 * 1024 / 8;
  int waves = (budget - off) / P.wave_doubles;
  if (waves > LQRO_PAIR_LB / 64) waves = LQRO_PAIR_LB / 64;
  if (waves < 1) {
    fprintf(stderr, "liblqro: horizon %d x %d points does not fit in LDS\n", H, NP);
    delete c;
    return LQRO_E_ARG;
  }
  P.waves = waves;
  P.max_waves = waves;
  off += waves * P.wave_doubles;
  c->lds_bytes = off * 8;
  int rc = ctx_alloc(c);
  if (rc) { lqro_destroy(c); return rc; }
  std::vector<double> S(3 * (size_t)NP);
  lqro_sphere(NP, g.xy_radius, g.z_radius, S.data());
  // max |u_p| with s_p = diag(2r_xy, 2r_xy, 2r_z) u_p (createSpheres, :743-745)
  {
    const double rad[3] = {2 * g.xy_radius, 2 * g.xy_radius, 2 * g.z_radius};
    double um = 0.0;
    for (int p = 0; p < NP; ++p) {
      double u2 = 0.0;
      for (int d = 0; d < 3; ++d) { const double u = S[3 * p + d] / rad[d]; u2 += u * u; }
      um = std::max(um, std::sqrt(u2));
    }
    c->umax = um * (1.0 + 1e-12);
    P.rad0 = rad[0]; P.rad1 = rad[1]; P.rad2 = rad[2]; P.umax = c->umax;
  }
  {
    std::vector<unsigned long long> sh(H, 0ull);
    for (int k = 0; k < H; ++k)
      for (int p = 0; p < NP; ++p) {
        unsigned long long z = (unsigned long long)(k * NP + p) + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        sh[k] += z ^ (z >> 31);
      }
    if (hipMemcpy(c->d_shash, sh.data(), sizeof(unsigned long long) * H, hipMemcpyHostToDevice) != hipSuccess) {
      lqro_destroy(c);
      return LQRO_E_HIP;
    }
  }
  if (hipMemcpy(c->d_S, S.data(), sizeof(double) * S.size(), hipMemcpyHostToDevice) != hipSuccess) {
    lqro_destroy(c);
    return LQRO_E_HIP;
  }
  const bool attr_ok = pair_set_lds_t<16, false>(c->lds_bytes) && pair_set_lds_t<16, true>(c->lds_bytes) &&
                       pair_set_lds_t<12, false>(c->lds_bytes) && pair_set_lds_t<12, true>(c->lds_bytes);
  if (!attr_ok) {
    lqro_destroy(c);
    return LQRO_E_HIP;
  }
  *out = c;
  return LQRO_OK;
}

int lqro_set_neighbors(lqro_ctx* c, double neighbor_dist, int32_t max_neighbors) {
  if (!c) return LQRO_E_ARG;
  if (c->pending) return LQRO_E_STATE;   // lqro_step_device_begin's half-step still reads them
  if (max_neighbors <= 0) { c->nbr_k = 0; return LQRO_OK; }
  if (!(neighbor_dist > 0)) return LQRO_E_ARG;
  HIPCHK(hipSetDevice(c->cfg.device));
  const int K = std::min<int>(max_neighbors, c->npr);
  if (K > c->nbr_cap) {
    if (c->d_nbrlist) (void)hipFree(c->d_nbrlist);
    c->d_nbrlist = nullptr;
    c->nbr_cap = 0;
    if (hipMalloc(&c->d_nbrlist, sizeof(int) * (size_t)c->nrows * K + 4) != hipSuccess) return LQRO_E_NOMEM;
    c->nbr_cap = K;
  }
  c->nbr_r2 = neighbor_dist * neighbor_dist;
  c->nbr_k = max_neighbors;
  return LQRO_OK;
}

int lqro_set_gains(lqro_ctx* c, const double* A, const double* B, const double* L,
                   const double* E, int32_t per_agent) {
  if (!c || !A || !B || !L || !E) return LQRO_E_ARG;
  if (c->pending) return LQRO_E_STATE;   // the pending half-step reads d_T / d_NCF on the caller's stream
  const lqro_config& g = c->cfg;
  HIPCHK(hipSetDevice(g.device));
  const size_t X = g.x_dim, U = g.u_dim, N = g.n_agents;
  const size_t na = per_agent ? N : 1;
  HIPCHK(wait_last_step(c));   // a step in flight still reads d_T / d_NCF
  HIPCHK(hipMemcpyAsync(c->d_A, A, sizeof(double) * X * X, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_B, B, sizeof(double) * X * U, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_L, L, sizeof(double) * na * U * X, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_E, E, sizeof(double) * na * U * 3, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemsetAsync(c->d_err, 0, sizeof(int), c->stream));
  hipLaunchKernelGGL(k_tables, dim3((unsigned)na), dim3(256), 0, c->stream, (int)X, (int)U,
                     g.horizon, c->d_A, c->d_B, c->d_L, c->d_E, per_agent ? 1 : 0, c->d_T,
                     c->d_NCF, c->d_R, c->d_TF, c->pa.rad0, c->pa.rad1, c->pa.rad2, c->umax,
                     c->d_err);
  HIPCHK(hipGetLastError());
  int err = 0;
  HIPCHK(hipMemcpyAsync(&err, c->d_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (err) return LQRO_E_SINGULAR;
  c->per_agent = per_agent ? 1 : 0;
  c->have_gains = 1;
  return LQRO_OK;
}

static int enqueue_tail(lqro_ctx* c, const double* d_x, const double* d_vgoal, double* d_newv, hipStream_t s,
                        const double* d_rowtab);
static int qhull_side_balance(int n, double w_sweep, double w_build, double b_max);

// the LP launch's arguments for this context's rows (every row, the tail's
// k_lp4 list)
static LpArgs lp_args(const lqro_ctx* c, int npr, const double* d_vgoal, double* d_newv) {
  LpArgs La{};
  La.npr = npr; La.nrows = c->nrows; La.row_begin = c->rb; La.row_stride = c->rs; La.vmax = c->cfg.vmax_lp;
  La.slots = c->d_planes; La.compact = c->d_lpcompact; La.proj = c->d_lpscratch;
  La.vgoal = d_vgoal; La.newv = d_newv; La.prof = c->d_prof;
  La.lp4_list = c->d_lp4; La.lp4_count = c->d_hcount + 9; La.lp4_next = c->d_hcount + 10;
  return La;
}

// phase 0: the whole step.  Row shards in Qhull order split it around the
// exchange of the loop-carried normal (lqro_step_device_begin / _end):
// phase 1 runs the sweep and the hulls and writes each own row's last
// normal into d_rowtab; phase 2 (enqueue_tail) resolves the facet-0 pairs
// against every rank's rows and runs the LP.
static int enqueue_step(lqro_ctx* c, const double* d_x, const double* d_vgoal, double* d_newv,
                        hipStream_t s, int phase = 0, double* d_rowtab = nullptr) {
  const lqro_config& g = c->cfg;
  PairArgs P = c->pa;
  P.N = g.n_agents; P.H = g.horizon; P.NP = g.n_points; P.min_reach = g.min_reach;
  // culling on: each row's slots are its K neighbours (k_nbr), not its N-1 pairs
  const int npr = c->nbr_k > 0 ? std::min(c->nbr_k, c->npr) : c->npr;
  P.row_begin = c->rb; P.row_stride = c->rs; P.nrows = c->nrows; P.npr = npr;
  P.per_agent = c->per_agent;
  P.vmax = g.vmax_reach;
  P.r2 = g.vmax_reach * g.vmax_reach;
  P.r2_lo = P.r2 * (1.0 - 1e-12);
  P.r2_hi = P.r2 * (1.0 + 1e-12);
  P.T = c->d_T; P.NCF = c->d_NCF; P.R = c->d_R; P.TF = c->d_TF; P.S = c->d_S;
  P.shash = c->d_shash; P.x = d_x;
  P.planes = c->d_planes; P.recs = c->d_recs;
  P.hull_queue = c->d_hq; P.hull_count = c->d_hcount; P.hull_cap = c->hull_cap;
  P.stats = c->d_stats;
  P.prof = c->d_prof + 32 + 2 * 4096;
  // persistent: one workgroup per CU (LDS-bound), rows off a queue.
  //   main:  k_prio -> k_pair(rows, n_cu - side blocks) -> [side done] -> k_hull -> k_hull_big -> k_lp
  //   side:  [k_prio done] -> k_pair(hot, side blocks) -> k_side(hot hulls, then rows)
  // The hot launch computes the pairs k_prio predicts to be inside-hull, so
  // their hulls run on the side CUs while the row launch sweeps the rest on
  // the others; each side workgroup joins the sweep as soon as the hull
  // queue is drained.  No kernel waits on another running kernel (streams
  // sharing a hardware queue just serialise), and the two concurrent grids
  // add up to one workgroup per CU.  Hull jobs the prediction missed are
  // taken by the k_hull after the sweep.
  P.row_counter = c->d_hcount + 4;
  P.qnrm = c->qhull_order ? c->d_qnrm : nullptr;
  // the context's scratch (queues, counters, plane slots, tables) is reused by
  // every step: a step enqueued on another stream than the last one, or a
  // set_gains on c->stream, must not overlap the step still in flight
  if (c->stepped) HIPCHK(hipStreamWaitEvent(s, c->ev[3], 0));
  HIPCHK(hipEventRecord(c->ev[0], s));
  HIPCHK(hipMemsetAsync(c->d_hcount, 0, sizeof(int) * 16, s));
  HIPCHK(hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * LQRO_ST_WORDS, s));
  HIPCHK(hipMemsetAsync(c->d_hq, 0xFF, sizeof(int) * (size_t)c->hull_cap, s));
  // Qhull order: the normal the last step's last eligible pair left enters this step
  if (c->qhull_order)
    HIPCHK(hipMemcpyAsync(c->d_carry, c->d_carry + 3, sizeof(double) * 3, hipMemcpyDeviceToDevice, s));
  P.nbr_list = nullptr;
  if (c->nbr_k > 0) {
    hipLaunchKernelGGL(k_nbr, dim3((unsigned)c->nrows), dim3(64), 0, s, d_x, g.x_dim, g.n_agents, c->rb, c->rs,
                       c->npr,
                       c->nbr_r2, c->nbr_k, npr, c->d_nbrlist, c->d_stats);
    HIPCHK(hipGetLastError());
    P.nbr_list = c->d_nbrlist;
  }
  // the LDS hull variant packs outside-set extents in 32 bits (lqro_hull.hpp
  // seg_put: 15-bit count, 17-bit offset / 4 into HULL_SBMULT * H*NP entries)
  const bool lds_ok = (size_t)g.horizon * g.n_points <= kHullLdsMaxHNP && !c->hull_big_only;
  const long slots = (long)c->nrows * npr;
  // k_side sweeps rows in the hull's LDS (HullMemC) after its hulls: as many
  // of its waves take pairs as per-wave regions fit beside the row tables
  const long side_room = (long)(sizeof(HullMemC) / 8) - P.lds_wave;
  const int side_waves = side_room > 0 ? (int)std::min<long>(std::min(HULL_CWAVES, P.waves),
                                                              side_room / P.wave_doubles) : 0;
  // the overlap pays where the hot pairs' hulls fit k_side's LDS topology
  // (C3: 177 hulls of <= 1,700 vertices); at H*NP > 16,383 (C5: 40 % of the
  // hulls outgrow its 2,048 vertices and retry in k_hull_big) the plain
  // schedule is faster (516 vs 1,150 ms per C5 shard step, scripts/c5_once.py)
  // crowded swarms (many inside-hull pairs in an earlier step: the value is
  // read without waiting for the copy, it only picks the schedule, and every
  // schedule gives bit-identical results) take the plain schedule
  // The inside-hull count that picks the schedule is step t-2's, read after
  // that step's copy completed (the host runs at most one step ahead of the
  // GPU here), so the schedule does not depend on host/GPU timing.
  const int slot = (int)(c->nstep & 1);
  unsigned long long inside_prev = ~0ull;
  double w_sweep = 0.0, w_build = 0.0, b_max = 0.0;   // CU-ms, ms (the step two before)
  unsigned long long retried_prev = 0;
  if (c->nstep >= 2) {
    HIPCHK(hipEventSynchronize(c->iev[slot]));
    inside_prev = c->h_inside[8 * slot];
    w_sweep = 1e-5 * (double)c->h_inside[8 * slot + 1];
    w_build = 1e-5 * (double)c->h_inside[8 * slot + 2];
    b_max = 1e-5 * (double)c->h_inside[8 * slot + 3];
    retried_prev = c->h_inside[8 * slot + 4];
  }
  const bool known = inside_prev != ~0ull;
  const bool lhull = c->local_hull || c->qhull_order;   // k_lhull or k_qhull on the side
  int side = lhull ? c->lside_cus : c->side_cus;
  const unsigned long long qspare =
      !known ? 0ull : c->qspare >= 0 ? (unsigned long long)c->qspare : inside_prev / 16 + 4;
  // the side's builds (workers): the last step's inside-hull count, or a
  // share of it (LQRO_QHULL_SIDE_PCT: the longest builds first, k_prio_save)
  unsigned long long qwant =
      known ? (inside_prev * (unsigned long long)c->qside_pct + 99ull) / 100ull + qspare : 0ull;
  if (c->qhull_order && c->qbalance && known && w_sweep > 0.0 && b_max > 0.0)
    qwant = std::min(qwant, (unsigned long long)qhull_side_balance(c->n_cu, w_sweep, w_build, b_max));
  if (c->qhull_order) {
    // Qhull's build is one long dependent chain per pair (one wave per CU):
    // the side takes one CU per expected hull, so every hot hull starts at
    // once, plus a few for pairs new this step (LQRO_QHULL_SPARE, default 4:
    // a pair beyond them waits for the first build to end), leaving at least
    // an eighth of the CUs to the sweep (unknown count: half the CUs).  With
    // speculative builds the main stream's sweep is as long as the slowest
    // build: each CU given back to it shortens the step (C3: 192 -> 181 side
    // CUs, 19.85 -> 19.35 ms, profiles/r5ak_ab_qhull_spare.txt)
    const unsigned long long want = known ? qwant : (unsigned long long)(c->n_cu / 2);
    side = (int)std::min<unsigned long long>((unsigned long long)(c->n_cu - c->n_cu / 8),
                                             std::max<unsigned long long>((unsigned long long)side, want));
  } else if (lhull) {
    // local hulls: at most ~3.7 inside-hull pairs per side CU (C3: 177 on
    // 48 CUs), widening up to half the CUs as the swarm gets denser
    if (known)
      side = (int)std::max<unsigned long long>(
          (unsigned long long)side,
          std::min<unsigned long long>(c->n_cu / 2, (inside_prev * 10ull + 36ull) / 37ull));
  } else if (known && inside_prev > 2ull * (unsigned long long)side) {
    side = std::min(c->n_cu / 2, (4 * side) / 3);
  }
  // local hulls: the overlap pays up to ~16 inside-hull pairs per CU of the
  // widest side (1,067 at 22 m: 15.5 vs 18.0 ms plain; 2,496 at 16 m: a tie)
  // (Qhull's order: the overlap always pays, the hulls outlast the sweep)
  const long max_inside = c->hot_max_inside >= 0 ? c->hot_max_inside
                          : c->qhull_order   ? LONG_MAX
                          : (lhull ? 16L * std::max(side, c->n_cu / 2) : 4L * side);
  const bool crowded = known && inside_prev > (unsigned long long)max_inside;
  // with the local hull the side stream is k_pair(hot) -> k_lhull -> k_pair
  // (rows, the same row queue): no LDS-topology condition
  // (Qhull order: until the work of a step is known — a context's first two
  // steps — the plain schedule: every CU sweeps, then the builds.  A side
  // guessed at half the CUs starved the sweep where it outweighs the builds:
  // C5's whole swarm took 11.7 s per unknown step against 3.4 s plain)
  const bool hot = c->hot_on && c->n_cu >= 64 && slots >= 65536 && c->nbr_k <= 0 && !crowded && side >= 1 &&
                   (known || !c->qhull_order) &&
                   (lhull || (lds_ok && (size_t)g.horizon * g.n_points <= 16383 && side_waves >= 1));
  const int nwait = hot ? side : 0;
  P.row_split = std::max(1, std::min(16, (2 * c->n_cu + c->nrows - 1) / c->nrows));
  // Qhull order: the side's k_qhull workers sweep rows in their build's LDS
  // once the hot builds are taken (k_qside, 3 waves a CU): rows in units of
  // ~128 pairs, so a 3-wave worker's last unit ends soon after the 16-wave
  // workgroups' (shared gains: the tables are staged once per workgroup)
  const long qside_room = (long)qhull_lds_doubles() - P.lds_wave;
  const int qside_waves = qside_room > 0 ? (int)std::min<long>(3, qside_room / P.wave_doubles) : 0;
  const bool qside = hot && c->qside && c->qhull_order && !c->qhull_big && qside_waves >= 1;
  if (qside && !c->per_agent) P.row_split = std::max(P.row_split, std::min(16, std::max(1, npr / 128)));
  // early LP (Qhull order, beside the hulls): a row whose planes are all
  // final runs its LP at once — in a k_lp_lds after the main sweep, or in the
  // k_qhull job that completes it (lqro_hull.hpp hull_row_done; rows of at
  // most LQRO_EARLY_LP_MAX_NPR pairs, longer ones go to the tail) — and the
  // tail only runs the rest (rows waiting on k_stale, rows closed late)
  // (the split step, lqro_step_device_begin / _end: the early rows' newV go
  // to the context's own buffer, copied into the caller's by _end; rows with
  // a facet-0 pair wait for the row-normal exchange in the tail as before)
  double* d_lpnv = d_newv != nullptr ? d_newv : (phase == 1 ? c->d_newv : nullptr);
  const bool early = hot && c->early_lp && c->qhull_order && !c->qhull_big && phase != 2 && c->nbr_k <= 0 &&
                     (size_t)npr * 32 <= kLpLdsMax && d_lpnv != nullptr;
  c->early_step = early ? 1 : 0;
  c->early_internal = early && d_lpnv != d_newv ? 1 : 0;
  P.rowpend = early ? c->d_rowpend : nullptr;
  if (early) HIPCHK(hipMemsetAsync(c->d_rowpend, 0, sizeof(int) * 2 * (size_t)c->nrows, s));
  const int units = c->nrows * P.row_split;
  const unsigned nblk = (unsigned)std::min(units, c->n_cu - nwait);
  const unsigned nside = (unsigned)std::max(0, std::min(units - (int)nblk, nwait));
  P.hot_list = nullptr; P.hot_mark = nullptr; P.hot_count = nullptr;
  P.hot_next = nullptr; P.hot_cap = 0; P.hot_only = 0; P.hot_done = nullptr;
  // Qhull order, split hot launch (every pair of the last step's list gets a
  // side CU of its own): side: the last step's inside-hull pairs, then
  // k_qhull; main: k_prio's other hot pairs, then the rows.  k_qhull's workers
  // wait for the main hot launch before leaving an empty queue.
  const bool split = hot && c->qhull_order && c->hot_split && !qside && !c->qhull_big && known &&
                     qwant <= (unsigned long long)nwait;
  // speculative builds (with the split): the last step's inside-hull pairs go
  // straight into the hull queue, so the side's k_qhull workers start building
  // them at once instead of after their evaluation (~0.5 ms at C3); the main
  // stream's hot launch evaluates them first, and each build commits only if
  // its pair is inside (PairArgs::spec_mark)
  const bool spec = split && c->hot_spec;
  if (hot) {
    PrioArgs Q{};
    Q.npr = c->npr; Q.nrows = c->nrows; Q.row_begin = c->rb; Q.row_stride = c->rs; Q.X = g.x_dim; Q.x = d_x;
    Q.t_hot = c->hot_t; Q.r2_hot = c->hot_r * c->hot_r;   // seconds, metres (scheduling heuristic)
    Q.list = c->d_hotlist; Q.mark = c->d_hotmark; Q.count = c->d_hcount + 6; Q.cap = c->hot_cap;
    Q.rowpend = P.rowpend;
    if (split) {
      HIPCHK(hipMemsetAsync(c->d_hot2 + 1, 0, sizeof(int) * 6, s));
      Q.prev = c->d_prevq; Q.prevn = c->d_hot2; Q.hot1n = c->d_hot2 + 1; Q.hot2next = c->d_hot2 + 3;
      if (spec) { Q.hq = c->d_hq; Q.hcount = c->d_hcount; Q.hq_cap = c->hull_cap; Q.spec_n = c->d_hot2 + 5; }
      hipLaunchKernelGGL(k_prio_prev, dim3(1), dim3(256), 0, s, Q);
      HIPCHK(hipGetLastError());
    }
    const long nb = std::min<long>((slots + 255) / 256, 8L * c->n_cu);
    hipLaunchKernelGGL(k_prio, dim3((unsigned)nb), dim3(256), 0, s, Q);
    HIPCHK(hipGetLastError());
    P.hot_list = c->d_hotlist; P.hot_mark = c->d_hotmark; P.hot_count = c->d_hcount + 6;
    P.hot_next = c->d_hcount + 7; P.hot_cap = c->hot_cap;
  }
  HullArgs Hh{};
  Hh.N = g.n_agents; Hh.X = g.x_dim; Hh.H = g.horizon; Hh.NP = g.n_points;
  Hh.row_begin = c->rb; Hh.row_stride = c->rs; Hh.npr = npr; Hh.per_agent = c->per_agent;
  Hh.nbr_list = P.nbr_list;
  Hh.r2 = P.r2; Hh.r2_lo = P.r2_lo; Hh.r2_hi = P.r2_hi;
  Hh.T = c->d_T; Hh.NCF = c->d_NCF; Hh.S = c->d_S; Hh.x = d_x;
  Hh.planes = c->d_planes; Hh.recs = c->d_recs;
  Hh.queue = c->d_hq; Hh.count = c->d_hcount; Hh.cap = c->hull_cap; Hh.next = c->d_hnext;
  Hh.scratch = c->d_hscratch; Hh.iscratch = c->d_hiscratch; Hh.fscratch = c->d_hfscratch;
  Hh.sb = reinterpret_cast<HullPt*>(c->d_hfaces);
  Hh.fbest = c->d_hfbest;
  Hh.vpid = c->d_hvpid; Hh.stack = c->d_hstack;
  Hh.rqueue = c->d_rq; Hh.rcount = c->d_hcount + 2; Hh.rnext = c->d_hcount + 3;
  Hh.bigmem = c->d_hbig;
  Hh.wide = c->d_hwide;
  Hh.bag = c->d_hbag;
  Hh.stats = c->d_stats;
  Hh.prof = c->d_prof;
  Hh.block_base = 0;
  Hh.big_main = 0;
  Hh.lqueue = c->d_lq; Hh.lcount = c->d_hcount + 11; Hh.ldone = c->d_hcount + 13;
  Hh.lfail = c->d_prof + 32 + 2 * 4096 + 32;
  Hh.ext_pts = nullptr; Hh.ext_n = 0; Hh.ext_max = 0; Hh.ext_facets = nullptr; Hh.ext_nf = nullptr;
  Hh.ext_full = 0;
  // per-job stamps only when asked for (LQRO_LHULL_PROFILE=1, scripts/lhull_jobs.py);
  // lfail counts hand-over reasons since the context was created
  Hh.ljobs = c->lhull_prof ? c->d_prof + 32 + 2 * 4096 + 48 : nullptr;
  Hh.qscratch = c->d_qscratch; Hh.qstride = c->qstride; Hh.qnrm = c->d_qnrm;
  Hh.qstale = c->d_qstale; Hh.qstale_count = c->d_hcount + 15; Hh.qstale_cap = c->hull_cap;
  Hh.rowpend = P.rowpend; Hh.rowclaim = early ? c->d_rowclaim : nullptr;
  Hh.row_lp = npr <= LQRO_EARLY_LP_MAX_NPR ? 1 : 0;
  Hh.row_target = P.row_split * LQRO_ROW_BIG;
  Hh.lp_vgoal = d_vgoal; Hh.lp_newv = d_lpnv; Hh.lp_vmax = g.vmax_lp;
  Hh.hbuild = c->d_hbuild; Hh.hbuild_cap = LQRO_HBUILD_CAP;
  // (k_qhull's in-place rebuild of capped builds where they happen: hulls of
  // more than 10,000 points (C5's ~19,000), or builds capped two steps before)
  Hh.big_inline =
      c->qhull_inline && !c->qhull_big && ((size_t)g.horizon * g.n_points > 10000 || retried_prev > 0) ? 1 : 0;
  Hh.qflags = c->qhull_flags;
  if (g.x_dim != 16 && g.x_dim != 12) return LQRO_E_ARG;
  // the row launch is submitted before the side stream's work: should the two
  // streams land on one hardware queue (a second context in the process), the
  // main grid still runs first on its CUs instead of k_side's row tail
  // sweeping every row on the side CUs alone
  if (nwait > 0) HIPCHK(hipEventRecord(c->xev[0], s));
  if (split) {   // the main stream's hot launch: k_prio's pairs after the last step's
    PairArgs P2 = P;
    P2.hot_only = 1;
    P2.hot_next = c->d_hot2 + 3;
    P2.hot_done = c->d_hot2 + 4;
    if (spec) P2.spec_mark = c->d_hotmark;   // (its list from position 0: the speculative pairs first)
    launch_pair(g.x_dim, dim3(nblk), dim3(P.waves * 64), c->lds_bytes, s, P2);
    HIPCHK(hipGetLastError());
  }
  launch_pair(g.x_dim, dim3(nblk), dim3(P.waves * 64), c->lds_bytes, s, P);
  HIPCHK(hipGetLastError());
  if (early) {
    // the rows the main sweep closed (no open hull): their LP on its CUs
    // while the side stream's hulls run
    LpArgs Le = lp_args(c, npr, d_vgoal, d_lpnv);
    Le.lp4_list = nullptr;
    Le.rowpend = c->d_rowpend; Le.rowclaim = c->d_rowclaim; Le.row_target = Hh.row_target; Le.mode = 1;
    HIPCHK(hipFuncSetAttribute((const void*)k_lp_lds<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLpLdsMax));
    hipLaunchKernelGGL(k_lp_lds<8>, dim3((unsigned)c->nrows), dim3(64), (size_t)npr * 32, s, Le);
    HIPCHK(hipGetLastError());
  }
  if (nwait > 0) {
    HIPCHK(hipStreamWaitEvent(c->side, c->xev[0], 0));
    PairArgs Ph = P;
    Ph.hot_only = 1;
    if (split) { Ph.hot_count = c->d_hot2 + 1; Ph.hot_next = c->d_hot2 + 2; }
    if (!spec) {   // (speculative builds: the side goes straight to k_qhull)
      launch_pair(g.x_dim, dim3(nwait), dim3(P.waves * 64), c->lds_bytes, c->side, Ph);
      HIPCHK(hipGetLastError());
    }
    if (c->qhull_order) {
      // the hot pairs' hulls in Qhull's order (k_qhull leaves when the queue
      // is empty), then the row sweep
      if (qside) {
        PairArgs Pq = P;
        Pq.max_waves = qside_waves;
        if (nside == 0) Pq.nrows = 0;
        launch_qside(g.x_dim, dim3(std::min(nwait, c->qworkers)), c->side, Hh, Pq);
        HIPCHK(hipGetLastError());
      } else {
        if (!c->qhull_big) {
          HullArgs Hs = Hh;
          if (split) { Hs.prod_done = c->d_hot2 + 4; Hs.prod_total = (int)nblk; }
          if (spec) { Hs.spec_mark = c->d_hotmark; Hs.spec_n = c->d_hot2 + 5; Hs.spec_next = c->d_hot2 + 6; }
          launch_qhull(dim3(std::min(nwait, c->qworkers)), c->side, Hs);
          HIPCHK(hipGetLastError());
        }
        if (nside > 0) {
          launch_pair(g.x_dim, dim3(nwait), dim3(P.waves * 64), c->lds_bytes, c->side, P);
          HIPCHK(hipGetLastError());
        }
      }
    } else if (c->local_hull) {
      // the hot pairs' local hulls (k_lhull leaves when the queue is empty:
      // later jobs go to the k_lhull after the sweep), then the row sweep
      launch_lhull(dim3(nwait), c->side, Hh);
      HIPCHK(hipGetLastError());
      if (lds_ok) {
        // the pairs it handed over (rare: near-coplanar input) in the full
        // hull right away, still beside the sweep (scratch blocks 0..nwait-1;
        // the k_hull after the sweep uses nwait.. and starts after the side)
        HullArgs Hf = Hh;
        Hf.queue = c->d_lq; Hf.count = c->d_hcount + 11; Hf.next = c->d_hcount + 12;
        launch_hull(dim3(nwait), c->side, Hf);
        HIPCHK(hipGetLastError());
      }
      if (nside > 0) {
        launch_pair(g.x_dim, dim3(nwait), dim3(P.waves * 64), c->lds_bytes, c->side, P);
        HIPCHK(hipGetLastError());
      }
    } else {
      PairArgs Pt = P;
      Pt.max_waves = side_waves;
      if (nside == 0) Pt.nrows = 0;
      launch_side(g.x_dim, dim3(nwait), dim3(HULL_CTHREADS), c->side, Hh, Pt);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(c->xev[1], c->side));
    HIPCHK(hipStreamWaitEvent(s, c->xev[1], 0));
  }
  HIPCHK(hipEventRecord(c->ev[1], s));
  if (c->qhull_order) {
    // every hull job left, the ones beyond k_qhull's caps, then the facet-0
    // pairs' loop-carried normals
    if (spec) {   // (a speculative job not taken on the side)
      Hh.spec_mark = c->d_hotmark; Hh.spec_n = c->d_hot2 + 5; Hh.spec_next = c->d_hot2 + 6;
    }
    if (!c->qhull_big) {
      launch_qhull(dim3(c->qworkers), s, Hh);
      HIPCHK(hipGetLastError());
    }
    Hh.big_main = c->qhull_big;
    launch_qhull_big(dim3(c->qworkers), s, Hh);
    HIPCHK(hipGetLastError());
    Hh.big_main = 0;
    // this step's inside-hull pairs head the next step's hot list
    hipLaunchKernelGGL(k_prio_save, dim3(1), dim3(256), 0, s, c->d_hq, c->d_hcount, c->hull_cap, c->d_prevq,
                       c->d_hot2, c->hot_cap, spec ? (const unsigned char*)c->d_hotmark : nullptr,
                       (const unsigned long long*)c->d_hbuild, (const unsigned long long*)(c->d_stats + LQRO_ST_NBUILD),
                       (int)LQRO_HBUILD_CAP, c->d_hotlist, c->d_hot2 + 1, split ? c->d_hotmark : nullptr, slots);
    HIPCHK(hipGetLastError());
    if (phase == 0) {
      launch_stale(s, c->d_planes, c->d_qnrm, c->d_qstale, c->d_hcount + 15, c->hull_cap, d_x, g.x_dim, npr, c->rb,
                   c->rs, c->d_carry, c->d_recs, slots);
      HIPCHK(hipGetLastError());
    }
  } else if (c->local_hull) {
    // k_lhull takes the queue k_pair filled; k_hull / k_hull_big then take
    // the pairs it handed over (scratch: hull_blocks blocks of 6 H*NP doubles)
    launch_lhull(dim3(c->hull_blocks), s, Hh);
    HIPCHK(hipGetLastError());
    Hh.queue = c->d_lq; Hh.count = c->d_hcount + 11; Hh.next = c->d_hcount + 12;
  }
  if (!c->qhull_order) {
    Hh.block_base = nwait;
    Hh.big_main = lds_ok ? 0 : 1;
    if (lds_ok) {
      launch_hull(dim3(c->hull_blocks - nwait), s, Hh);
      HIPCHK(hipGetLastError());
    }
    Hh.block_base = 0;
    launch_hull_big(dim3(c->hull_big_blocks), s, Hh);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(c->ev[2], s));
  if (phase == 1) {
    // each own row's last normal (none without Qhull order)
    launch_rowlast(s, c->qhull_order ? c->d_planes : nullptr, c->d_qnrm, npr, c->nrows, c->rb, c->rs, d_rowtab);
    HIPCHK(hipGetLastError());
    c->pend_x = d_x;
    c->pend_vgoal = d_vgoal;
    c->pend_stream = s;
    c->pending = 1;
    return LQRO_OK;
  }
  return enqueue_tail(c, d_x, d_vgoal, d_newv, s, nullptr);
}

// The side's width in Qhull order from the work measured two steps before:
// with k side CUs the builds end no sooner than max(b_max, 1.15 w_build / k)
// (LPT packing of chains, 15 % margin) and the sweep's rows no sooner than
// w_sweep / (n - k).  The widest k within 2 % of the best such bound: where
// the builds bound the step (C3: the slowest build) every build keeps a CU
// of its own as long as the sweep stays shorter; where the sweep does (C5: its
// 2048-row shard is ~86 CU-s of sweep against ~21 CU-s of builds) the side
// shrinks to what the builds need (224 -> ~60 CUs: 4.7 s -> ~0.6 s a step).
static int qhull_side_balance(int n, double w_sweep, double w_build, double b_max) {
  const int kmax = n - n / 8;
  double best = 1e300;
  std::vector<double> t((size_t)kmax + 1, 0.0);
  for (int k = 1; k <= kmax; ++k) {
    t[k] = std::max(std::max(b_max, 1.15 * w_build / k), w_sweep / (double)(n - k));
    best = std::min(best, t[k]);
  }
  for (int k = kmax; k >= 1; --k)
    if (t[k] <= 1.02 * best) return k;
  return kmax;
}

static int enqueue_tail(lqro_ctx* c, const double* d_x, const double* d_vgoal, double* d_newv, hipStream_t s,
                        const double* d_rowtab) {
  const lqro_config& g = c->cfg;
  const int npr = c->nbr_k > 0 ? std::min(c->nbr_k, c->npr) : c->npr;
  const long slots = (long)c->nrows * npr;
  const int slot = (int)(c->nstep & 1);
  if (d_rowtab && c->qhull_order) {
    launch_stale_rows(s, c->d_planes, c->d_qnrm, c->d_qstale, c->d_hcount + 15, c->hull_cap, d_x, g.x_dim, npr,
                      c->rb, c->rs, d_rowtab, g.n_agents, c->d_carry, c->d_recs, slots);
    HIPCHK(hipGetLastError());
  }
  c->pending = 0;
  LpArgs La = lp_args(c, npr, d_vgoal, d_newv);
  if (c->early_step) {   // the rows the early LP ran are done
    La.rowclaim = c->d_rowclaim;
    La.mode = 2;
  }
  HIPCHK(launch_lp(La, s));
  if (c->early_step && c->early_internal && d_newv != c->d_newv) {   // the rows the early LP ran, into the caller's newV
    hipLaunchKernelGGL(k_copy_claimed, dim3((unsigned)((c->nrows + 255) / 256)), dim3(256), 0, s, c->d_rowclaim,
                       c->nrows, c->rb, c->rs, (const double*)c->d_newv, d_newv);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipMemcpyAsync(c->h_inside + 8 * slot, c->d_stats + 2, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(c->h_inside + 8 * slot + 1, c->d_stats + LQRO_ST_SWORK, 3 * sizeof(unsigned long long),
                        hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(c->h_inside + 8 * slot + 4, c->d_stats + LQRO_ST_RETRY, sizeof(unsigned long long),
                        hipMemcpyDeviceToHost, s));
  HIPCHK(hipEventRecord(c->iev[slot], s));
  HIPCHK(hipEventRecord(c->ev[3], s));
  c->stepped = 1;
  c->nstep++;
  return LQRO_OK;
}

// `stream` is the caller's HIP stream; NULL is the default (null) stream, as
// in lqro_dynamics_step_device, so the step is ordered with the work the
// caller (e.g. torch's default stream, RCCL's waits on it) has on it.
int lqro_step_device(lqro_ctx* c, const double* d_x, const double* d_vgoal, double* d_newv,
                     void* stream) {
  if (!c || !d_x || !d_vgoal || !d_newv) return LQRO_E_ARG;
  if (!c->have_gains || c->pending) return LQRO_E_STATE;
  HIPCHK(hipSetDevice(c->cfg.device));
  return enqueue_step(c, d_x, d_vgoal, d_newv, (hipStream_t)stream);
}

int lqro_step_device_begin(lqro_ctx* c, const double* d_x, const double* d_vgoal, double* d_rowtab, void* stream) {
  if (!c || !d_x || !d_vgoal || !d_rowtab) return LQRO_E_ARG;
  if (!c->have_gains) return LQRO_E_STATE;
  if (c->pending) return LQRO_E_STATE;
  HIPCHK(hipSetDevice(c->cfg.device));
  return enqueue_step(c, d_x, d_vgoal, nullptr, (hipStream_t)stream, 1, d_rowtab);
}

int lqro_step_device_end(lqro_ctx* c, const double* d_rowtab, double* d_newv, void* stream) {
  if (!c || !d_rowtab || !d_newv) return LQRO_E_ARG;
  if (!c->pending) return LQRO_E_STATE;
  HIPCHK(hipSetDevice(c->cfg.device));
  hipStream_t s = (hipStream_t)stream;
  if (s != c->pend_stream) {   // the begin's work first
    HIPCHK(hipEventRecord(c->xev[0], c->pend_stream));
    HIPCHK(hipStreamWaitEvent(s, c->xev[0], 0));
  }
  return enqueue_tail(c, c->pend_x, c->pend_vgoal, d_newv, s, d_rowtab);
}

int lqro_step(lqro_ctx* c, const double* x, const double* vgoal, double* newv) {
  if (!c || !x || !vgoal || !newv) return LQRO_E_ARG;
  if (!c->have_gains || c->pending) return LQRO_E_STATE;
  const lqro_config& g = c->cfg;
  HIPCHK(hipSetDevice(g.device));
  const size_t N = g.n_agents, X = g.x_dim;
  HIPCHK(hipMemcpyAsync(c->d_x, x, sizeof(double) * N * X, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_vgoal, vgoal, sizeof(double) * N * 3, hipMemcpyHostToDevice, c->stream));
  int rc = enqueue_step(c, c->d_x, c->d_vgoal, c->d_newv, c->stream);
  if (rc) return rc;
  if (c->rs == 1) {
    HIPCHK(hipMemcpyAsync(newv + (size_t)c->rb * 3, c->d_newv + (size_t)c->rb * 3,
                          sizeof(double) * 3 * c->nrows, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  } else {   // cyclic rows: the whole array, then this context's rows
    std::vector<double> all(N * 3);
    HIPCHK(hipMemcpyAsync(all.data(), c->d_newv, sizeof(double) * 3 * N, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int r = 0; r < c->nrows; ++r) {
      const size_t i = (size_t)c->rb + (size_t)r * c->rs;
      for (int q = 0; q < 3; ++q) newv[3 * i + q] = all[3 * i + q];
    }
  }
  int hc = 0;
  HIPCHK(hipMemcpy(&hc, c->d_hcount, sizeof(int), hipMemcpyDeviceToHost));
  if (hc > c->hull_cap) return LQRO_E_OVERFLOW;
  // a pair whose hull the kernels could not build has no half-plane: the
  // step says so (the reference always gets a hull from qconvex, LQRO:879-880)
  unsigned long long st[LQRO_ST_FAILS];
  HIPCHK(hipMemcpy(st, c->d_stats, sizeof st, hipMemcpyDeviceToHost));
  if (st[4]) return LQRO_E_HULL;
  // a pair whose winner qconvex may have merged (Qhull's pre-merge is not
  // restated): never a silent difference from the reference (LQRO:925-967)
  if (st[LQRO_ST_MWIN]) return LQRO_E_QHMERGE;
  return LQRO_OK;
}

// ---------------------------------------------------------------------------
// Gain synthesis (controlMatrices, LQRO:520-582): host for one agent type,
// device for heterogeneous swarms (one agent per lane; lqro_synth.hpp)
// ---------------------------------------------------------------------------
int lqro_synthesize_gains(const lqro_model* md, double* Ao, double* Bo, double* co, double* Lo,
                          double* Eo, double* Lho, double* Eho) {
  if (!md) return LQRO_E_ARG;
  synth::gains(md, Ao, Bo, co, Lo, Eo, Lho, Eho);
  return LQRO_OK;
}

int lqro_synthesize_gains_x(const lqro_model* md, int32_t x_dim, double* Ao, double* Bo, double* co,
                            double* Lo, double* Eo, double* lo, double* Lho, double* Eho) {
  if (!md) return LQRO_E_ARG;
  if (x_dim == 16) synth::gains_x<16>(md, Ao, Bo, co, Lo, Eo, Lho, Eho, lo);
  else if (x_dim == 12) synth::gains_x<12>(md, Ao, Bo, co, Lo, Eo, Lho, Eho, lo);
  else return LQRO_E_ARG;
  return LQRO_OK;
}

// per-agent output block, in doubles: A X*X, B X*4, c X, L 4*X, E 12, l 4, Lh 3*X, Eh 9
static void synth_sizes(int X, int* sz) {
  sz[0] = X * X; sz[1] = X * 4; sz[2] = X; sz[3] = 4 * X; sz[4] = 12; sz[5] = 4; sz[6] = 3 * X; sz[7] = 9;
}
static int synth_stride(int X) { return X * X + 12 * X + 25; }

int lqro_synthesize_gains_batch_x(const lqro_model* models, int32_t n, int32_t x_dim, double* A, double* B,
                                  double* c, double* L, double* E, double* l, double* Lh, double* Eh,
                                  int32_t device) {
  if (!models || n <= 0 || (x_dim != 16 && x_dim != 12)) return LQRO_E_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return LQRO_E_NODEVICE;
  if (hipSetDevice(device) != hipSuccess) return LQRO_E_HIP;
  const int stride = synth_stride(x_dim);
  int sz[8];
  synth_sizes(x_dim, sz);
  lqro_model* d_m = nullptr;
  double* d_out = nullptr;
  int rc = LQRO_OK;
  if (hipMalloc(&d_m, sizeof(lqro_model) * (size_t)n) != hipSuccess ||
      hipMalloc(&d_out, sizeof(double) * stride * (size_t)n) != hipSuccess) {
    rc = LQRO_E_NOMEM;
  } else if (hipMemcpy(d_m, models, sizeof(lqro_model) * (size_t)n, hipMemcpyHostToDevice) != hipSuccess) {
    rc = LQRO_E_HIP;
  } else {
    const char* lane_env = getenv("LQRO_SYNTH_LANE");
    launch_synth(x_dim, lane_env && atoi(lane_env) == 1, d_m, (int)n, d_out);
    std::vector<double> h((size_t)stride * n);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(h.data(), d_out, sizeof(double) * h.size(), hipMemcpyDeviceToHost) != hipSuccess) {
      rc = LQRO_E_HIP;
    } else {
      double* outs[8] = {A, B, c, L, E, l, Lh, Eh};
      int off = 0;
      for (int k = 0; k < 8; ++k) {
        if (outs[k])
          for (int a = 0; a < n; ++a)
            memcpy(outs[k] + (size_t)a * sz[k], h.data() + (size_t)a * stride + off, sizeof(double) * sz[k]);
        off += sz[k];
      }
    }
  }
  if (d_m) (void)hipFree(d_m);
  if (d_out) (void)hipFree(d_out);
  return rc;
}

int lqro_synthesize_gains_batch(const lqro_model* models, int32_t n, double* A, double* B, double* c,
                                double* L, double* E, double* Lh, double* Eh, int32_t device) {
  return lqro_synthesize_gains_batch_x(models, n, 16, A, B, c, L, E, nullptr, Lh, Eh, device);
}

static bool agents_complete(const lqro_agents* a) {
  return a && a->x && a->rot && a->x_true && a->rot_true && a->P && a->vgoal && a->u_goal && a->p_goal &&
         a->L && a->E && a->l && a->Lh && a->Eh && a->M && a->N && a->normals;
}

int lqro_dynamics_step_device(const lqro_model* models, int32_t n_models, int32_t n, int32_t per_agent_gains,
                              const lqro_agents* agents, void* stream) {
  if (!models || n <= 0 || (n_models != 1 && n_models != n) || !agents_complete(agents)) return LQRO_E_ARG;
  const char* lane = getenv("LQRO_DYN_LANE");
  launch_dyn(lane && atoi(lane) == 1, models, (int)n_models, (int)n, (int)(per_agent_gains != 0), *agents,
             (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? LQRO_OK : LQRO_E_HIP;
}

int lqro_dynamics_step(const lqro_model* models, int32_t n_models, int32_t n, int32_t per_agent_gains,
                       const lqro_agents* agents, int32_t device) {
  if (!models || n <= 0 || (n_models != 1 && n_models != n) || !agents_complete(agents)) return LQRO_E_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return LQRO_E_NODEVICE;
  if (hipSetDevice(device) != hipSuccess) return LQRO_E_HIP;
  const size_t G = per_agent_gains ? (size_t)n : 1, N = (size_t)n;
  using namespace dyn;
  // (host source, element count, written back)
  struct Buf { const double* h; double* out; size_t cnt; double* d; };
  Buf b[17] = {
      {agents->x, agents->x, N * kX, nullptr},            {agents->rot, agents->rot, N * 9, nullptr},
      {agents->x_true, agents->x_true, N * kX, nullptr},  {agents->rot_true, agents->rot_true, N * 9, nullptr},
      {agents->P, agents->P, N * kX * kX, nullptr},       {agents->vgoal, agents->vgoal, N * 3, nullptr},
      {nullptr, agents->u, agents->u ? N * kU : 0, nullptr},
      {agents->u_goal, nullptr, N * kU, nullptr},         {agents->p_goal, nullptr, N * 3, nullptr},
      {agents->L, nullptr, G * kU * kX, nullptr},         {agents->E, nullptr, G * kU * kV, nullptr},
      {agents->l, nullptr, G * kU, nullptr},              {agents->Lh, nullptr, G * kV * kX, nullptr},
      {agents->Eh, nullptr, G * kV * kV, nullptr},        {agents->M, nullptr, (size_t)kX * kX, nullptr},
      {agents->N, nullptr, (size_t)kZ * kZ, nullptr},     {agents->normals, nullptr, N * kNormals, nullptr}};
  lqro_model* d_m = nullptr;
  float* d_kf = nullptr;
  int rc = LQRO_OK;
  if (hipMalloc(&d_m, sizeof(lqro_model) * (size_t)n_models) != hipSuccess) rc = LQRO_E_NOMEM;
  if (rc == LQRO_OK && agents->keyframes && hipMalloc(&d_kf, sizeof(float) * 8 * N) != hipSuccess)
    rc = LQRO_E_NOMEM;
  for (auto& q : b)
    if (rc == LQRO_OK && q.cnt && hipMalloc(&q.d, sizeof(double) * q.cnt) != hipSuccess) rc = LQRO_E_NOMEM;
  if (rc == LQRO_OK &&
      hipMemcpy(d_m, models, sizeof(lqro_model) * (size_t)n_models, hipMemcpyHostToDevice) != hipSuccess)
    rc = LQRO_E_HIP;
  for (auto& q : b)
    if (rc == LQRO_OK && q.h && hipMemcpy(q.d, q.h, sizeof(double) * q.cnt, hipMemcpyHostToDevice) != hipSuccess)
      rc = LQRO_E_HIP;
  if (rc == LQRO_OK) {
    lqro_agents d;
    d.x = b[0].d; d.rot = b[1].d; d.x_true = b[2].d; d.rot_true = b[3].d; d.P = b[4].d; d.vgoal = b[5].d;
    d.u = b[6].d; d.u_goal = b[7].d; d.p_goal = b[8].d; d.L = b[9].d; d.E = b[10].d; d.l = b[11].d;
    d.Lh = b[12].d; d.Eh = b[13].d; d.M = b[14].d; d.N = b[15].d; d.normals = b[16].d;
    d.keyframes = d_kf; d.time = agents->time;
    rc = lqro_dynamics_step_device(d_m, n_models, n, per_agent_gains, &d, nullptr);
    if (rc == LQRO_OK && hipDeviceSynchronize() != hipSuccess) rc = LQRO_E_HIP;
  }
  for (auto& q : b)
    if (rc == LQRO_OK && q.out && hipMemcpy(q.out, q.d, sizeof(double) * q.cnt, hipMemcpyDeviceToHost) != hipSuccess)
      rc = LQRO_E_HIP;
  if (rc == LQRO_OK && d_kf &&
      hipMemcpy(agents->keyframes, d_kf, sizeof(float) * 8 * N, hipMemcpyDeviceToHost) != hipSuccess)
    rc = LQRO_E_HIP;
  if (d_m) (void)hipFree(d_m);
  if (d_kf) (void)hipFree(d_kf);
  for (auto& q : b)
    if (q.d) (void)hipFree(q.d);
  return rc;
}

int lqro_calculate_new_v(const float* planes, const int64_t* offsets, int32_t n_agents,
                         const double* vgoal, double vmax_lp, double* newv, int32_t device) {
  if (!planes || !offsets || !vgoal || !newv || n_agents <= 0) return LQRO_E_ARG;
  HIPCHK(hipSetDevice(device));
  int64_t mmax = 1;
  for (int r = 0; r < n_agents; ++r) {
    const int64_t m = offsets[r + 1] - offsets[r];
    if (m < 0) return LQRO_E_ARG;
    if (m > mmax) mmax = m;
  }
  const size_t slots = (size_t)n_agents * (size_t)mmax;
  std::vector<float> h(slots * 8, 0.0f);
  for (int r = 0; r < n_agents; ++r)
    for (int64_t k = offsets[r]; k < offsets[r + 1]; ++k) {
      float* d = &h[((size_t)r * mmax + (size_t)(k - offsets[r])) * 8];
      for (int q = 0; q < 6; ++q) d[q] = planes[6 * k + q];
      int one = 1;
      memcpy(&d[6], &one, 4);
    }
  float *d_slots = nullptr, *d_compact = nullptr, *d_proj = nullptr;
  double *d_vg = nullptr, *d_nv = nullptr;
  int *d_l4 = nullptr, *d_l4c = nullptr;
  int rc = LQRO_OK;
  if (hipMalloc(&d_slots, sizeof(float) * 8 * slots) != hipSuccess ||
      hipMalloc(&d_compact, sizeof(float) * 8 * slots) != hipSuccess ||
      hipMalloc(&d_proj, sizeof(float) * 8 * slots) != hipSuccess ||
      hipMalloc(&d_vg, sizeof(double) * 3 * n_agents) != hipSuccess ||
      hipMalloc(&d_nv, sizeof(double) * 3 * n_agents) != hipSuccess ||
      hipMalloc(&d_l4, sizeof(int) * 6 * n_agents) != hipSuccess ||
      hipMalloc(&d_l4c, sizeof(int) * 2) != hipSuccess || hipMemset(d_l4c, 0, sizeof(int) * 2) != hipSuccess) {
    rc = LQRO_E_NOMEM;
  } else if (hipMemcpy(d_slots, h.data(), sizeof(float) * 8 * slots, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(d_vg, vgoal, sizeof(double) * 3 * n_agents, hipMemcpyHostToDevice) != hipSuccess) {
    rc = LQRO_E_HIP;
  } else {
    LpArgs La{};
    La.npr = (int)mmax; La.nrows = n_agents; La.row_begin = 0; La.row_stride = 1; La.vmax = vmax_lp;
    La.slots = d_slots; La.compact = d_compact; La.proj = d_proj; La.vgoal = d_vg; La.newv = d_nv; La.prof = nullptr;
    La.lp4_list = d_l4; La.lp4_count = d_l4c; La.lp4_next = d_l4c + 1;
    if (launch_lp(La, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(newv, d_nv, sizeof(double) * 3 * n_agents, hipMemcpyDeviceToHost) != hipSuccess)
      rc = LQRO_E_HIP;
  }
  void* ps[] = {d_slots, d_compact, d_proj, d_vg, d_nv, d_l4, d_l4c};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  return rc;
}

int lqro_set_carry_normal(lqro_ctx* c, const double* n3) {
  if (!c || !n3) return LQRO_E_ARG;
  if (c->pending) return LQRO_E_STATE;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(wait_last_step(c));
  const double v[6] = {n3[0], n3[1], n3[2], n3[0], n3[1], n3[2]};
  HIPCHK(hipMemcpy(c->d_carry, v, sizeof v, hipMemcpyHostToDevice));
  return LQRO_OK;
}

int lqro_get_carry_normal(lqro_ctx* c, double* n3) {
  if (!c || !n3) return LQRO_E_ARG;
  if (c->pending) return LQRO_E_STATE;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(wait_last_step(c));
  HIPCHK(hipMemcpy(n3, c->d_carry + 3, sizeof(double) * 3, hipMemcpyDeviceToHost));
  return LQRO_OK;
}

int lqro_get_records(lqro_ctx* c, lqro_pair_record* out, int64_t cap, int64_t* n_out) {
  if (!c || !out) return LQRO_E_ARG;
  if (!c->d_recs || c->pending) return LQRO_E_STATE;
  const int64_t n = (int64_t)c->nrows * (c->nbr_k > 0 ? std::min(c->nbr_k, c->npr) : c->npr);
  if (cap < n) return LQRO_E_ARG;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(wait_last_step(c));
  HIPCHK(hipMemcpy(out, c->d_recs, sizeof(lqro_pair_record) * (size_t)n, hipMemcpyDeviceToHost));
  if (n_out) *n_out = n;
  return LQRO_OK;
}

int lqro_get_stats_ex(lqro_ctx* c, int64_t* st, int32_t n) {
  if (!c || !st || n < 1) return LQRO_E_ARG;
  if (c->pending) return LQRO_E_STATE;   // the half-step's counters are not final
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(wait_last_step(c));
  unsigned long long h[LQRO_ST_FAILS];
  HIPCHK(hipMemcpy(h, c->d_stats, sizeof h, hipMemcpyDeviceToHost));
  if (c->nbr_k <= 0) h[0] = (unsigned long long)c->nrows * c->npr;   // else k_nbr counted the kept pairs
  // [0..10] the device words; [11] LQRO_REC_QHMERGE_WIN pairs (device word
  // LQRO_ST_MWIN; word 11 counts the failures lqro_get_hull_failures names)
  for (int k = 0; k < n; ++k)
    st[k] = k < LQRO_ST_NFAIL ? (int64_t)h[k] : k == 11 ? (int64_t)h[LQRO_ST_MWIN] : 0;
  return LQRO_OK;
}

int lqro_get_hull_builds(lqro_ctx* c, lqro_hull_build* out, int64_t cap, int64_t* n_out) {
  if (!c || !n_out || (cap > 0 && !out)) return LQRO_E_ARG;
  if (c->pending) return LQRO_E_STATE;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(wait_last_step(c));
  *n_out = 0;
  if (!c->d_hbuild) return LQRO_OK;   // not in Qhull order: no builds
  unsigned long long h[LQRO_ST_FAILS];
  HIPCHK(hipMemcpy(h, c->d_stats, sizeof h, hipMemcpyDeviceToHost));
  const int64_t n = (int64_t)h[LQRO_ST_NBUILD];
  *n_out = n;
  const int64_t m = std::min<int64_t>(std::min<int64_t>(n, LQRO_HBUILD_CAP), cap);
  if (m <= 0) return LQRO_OK;
  std::vector<unsigned long long> r(4 * (size_t)m);
  HIPCHK(hipMemcpy(r.data(), c->d_hbuild, sizeof(unsigned long long) * r.size(), hipMemcpyDeviceToHost));
  const int npr = c->nbr_k > 0 ? std::min(c->nbr_k, c->npr) : c->npr;
  std::vector<int> nbr;
  if (c->nbr_k > 0) {   // culled rows: slot -> neighbour index
    nbr.resize((size_t)c->nrows * npr);
    HIPCHK(hipMemcpy(nbr.data(), c->d_nbrlist, sizeof(int) * nbr.size(), hipMemcpyDeviceToHost));
  }
  for (int64_t k = 0; k < m; ++k) {
    const unsigned long long* w = &r[4 * (size_t)k];
    const long slot = (long)(w[0] & 0xFFFFFFFFFFull);
    const int lrow = (int)(slot / npr), jj = nbr.empty() ? (int)(slot % npr) : nbr[slot];
    lqro_hull_build& b = out[k];
    b.i = c->rb + lrow * c->rs;
    b.j = jj < b.i ? jj : jj + 1;
    b.kernel = (int32_t)(w[0] >> 40);
    b.t_start = w[1];
    b.t_end = w[2];
    b.n_points = (int32_t)(w[3] & 0xFFFFF);
    b.insertions = (int32_t)((w[3] >> 20) & 0xFFFFF);
    b.facet_slots = (int32_t)((w[3] >> 40) & 0xFFFFF);
  }
  return LQRO_OK;
}

int lqro_get_stats(lqro_ctx* c, int64_t* st) { return lqro_get_stats_ex(c, st, 8); }

// the pairs named in the step's counters: count word `wn`, slots from word `w0`
static int named_pairs(lqro_ctx* c, int wn, int w0, int64_t* pairs, int64_t cap, int64_t* n_out) {
  if (!c || !n_out || (cap > 0 && !pairs)) return LQRO_E_ARG;
  if (c->pending) return LQRO_E_STATE;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(wait_last_step(c));
  unsigned long long h[LQRO_ST_WORDS];
  HIPCHK(hipMemcpy(h, c->d_stats, sizeof h, hipMemcpyDeviceToHost));
  const int64_t n = (int64_t)h[wn];
  *n_out = n;
  const int npr = c->nbr_k > 0 ? std::min(c->nbr_k, c->npr) : c->npr;
  std::vector<int> nbr;
  const int64_t m = std::min<int64_t>(std::min<int64_t>(n, LQRO_ST_FAILMAX), cap);
  if (m > 0 && c->nbr_k > 0) {   // culled rows: slot -> neighbour index
    nbr.resize((size_t)c->nrows * npr);
    HIPCHK(hipMemcpy(nbr.data(), c->d_nbrlist, sizeof(int) * nbr.size(), hipMemcpyDeviceToHost));
  }
  for (int64_t k = 0; k < m; ++k) {
    const long slot = (long)h[w0 + k];
    const int lrow = (int)(slot / npr), jj = nbr.empty() ? (int)(slot % npr) : nbr[slot];
    const int i = c->rb + lrow * c->rs;
    pairs[2 * k] = i;
    pairs[2 * k + 1] = jj < i ? jj : jj + 1;
  }
  return LQRO_OK;
}

int lqro_get_hull_failures(lqro_ctx* c, int64_t* pairs, int64_t cap, int64_t* n_out) {
  return named_pairs(c, LQRO_ST_NFAIL, LQRO_ST_FAILS, pairs, cap, n_out);
}

int lqro_get_qhmerge_pairs(lqro_ctx* c, int64_t* pairs, int64_t cap, int64_t* n_out) {
  return named_pairs(c, LQRO_ST_MWIN, LQRO_ST_MWINS, pairs, cap, n_out);
}

/* diagnostic (not in lqro.h): inside-hull pairs of the last step decided by
 * the local hull (out[0]) and handed to the full hull (out[1]); out[2..17]:
 * hand-over reasons since the context was created (k_lhull's fail code - 20;
 * 0: the point set / initial tetrahedron) */
int lqro_debug_local_hull(lqro_ctx* c, long long* out) {
  if (!c || !out) return LQRO_E_ARG;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(wait_last_step(c));
  int h[16];
  HIPCHK(hipMemcpy(h, c->d_hcount, sizeof h, hipMemcpyDeviceToHost));
  unsigned long long r[16];
  HIPCHK(hipMemcpy(r, c->d_prof + 32 + 2 * 4096 + 32, sizeof r, hipMemcpyDeviceToHost));
  out[0] = h[13];
  out[1] = h[11];
  for (int k = 0; k < 16; ++k) out[2 + k] = (long long)r[k];
  return LQRO_OK;
}

/* test hook (not in lqro.h): the inside-hull branch on n given points
 * (already %g-rounded, as qconvex reads them; n <= H * NP of the context)
 * with relative velocity vrel.  local = 0: k_hull, its facets (point ids)
 * into facets (max_facets x 3) and their count into *n_facets; local = 1:
 * k_lhull (no facet list; *n_facets = -1 when it handed the points over);
 * local = 2: k_qhull, Qhull's build order and the reference's selection;
 * pts then holds the n rounded points followed by the n full-precision ones
 * (*n_facets = the build's status bits, 0: Qhull's build reproduced).
 * rec receives the selected facet, distance and normal. */
int lqro_debug_hull_points(lqro_ctx* c, const double* pts, int32_t n, const double* vrel, int32_t local,
                           int32_t* facets, int32_t max_facets, int32_t* n_facets, lqro_pair_record* rec) {
  if (!c || !pts || !vrel || !n_facets || !rec || n < 4 || (size_t)n > (size_t)c->cfg.horizon * c->cfg.n_points ||
      (!local && (!facets || max_facets < 1)) || local < 0 || local > 2)
    return LQRO_E_ARG;
  const lqro_config& g = c->cfg;
  HIPCHK(hipSetDevice(g.device));
  HIPCHK(wait_last_step(c));
  const int X = g.x_dim;
  std::vector<double> xh(2 * (size_t)X, 0.0);
  for (int q = 0; q < 3; ++q) xh[3 + q] = vrel[q];       // x_i - x_j = vrel, at rest otherwise
  double *d_pts = nullptr, *d_x = nullptr;
  int *d_q = nullptr, *d_f = nullptr;
  lqro_pair_record* d_rec = nullptr;
  float* d_pl = nullptr;
  unsigned long long* d_st = nullptr;
  char* d_qw = nullptr;
  double* d_qn = nullptr;
  int rc = LQRO_OK;
  const int fmax = (local == 1 || !facets) ? 1 : max_facets;
  const size_t qstride = (qhull_worker_bytes(g.horizon * g.n_points) + 255) & ~(size_t)255;
  if (local == 2 && (hipMalloc(&d_qw, qstride) != hipSuccess || hipMemset(d_qw, 0, qstride) != hipSuccess ||
                     hipMalloc(&d_qn, sizeof(double) * 8) != hipSuccess))
    rc = LQRO_E_NOMEM;
  if (rc != LQRO_OK) {
  } else if (hipMalloc(&d_st, sizeof(unsigned long long) * LQRO_ST_WORDS) != hipSuccess ||
      hipMemset(d_st, 0, sizeof(unsigned long long) * LQRO_ST_WORDS) != hipSuccess ||
      hipMalloc(&d_pts, sizeof(double) * (local == 2 ? 6 : 3) * n) != hipSuccess || hipMalloc(&d_x, sizeof(double) * 2 * X) != hipSuccess ||
      hipMalloc(&d_q, sizeof(int) * 16) != hipSuccess || hipMalloc(&d_f, sizeof(int) * 3 * fmax) != hipSuccess ||
      hipMalloc(&d_rec, sizeof(lqro_pair_record)) != hipSuccess || hipMalloc(&d_pl, sizeof(float) * 8) != hipSuccess) {
    rc = LQRO_E_NOMEM;
  } else {
    // queue = {slot 0}; count 1; next, local hand-over count / next, done, facet count 0
    const int q0[16] = {0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    lqro_pair_record r0;
    memset(&r0, 0, sizeof r0);
    r0.flags = LQRO_REC_INSIDE;
    if (hipMemcpy(d_pts, pts, sizeof(double) * (local == 2 ? 6 : 3) * n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_x, xh.data(), sizeof(double) * 2 * X, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_q, q0, sizeof q0, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_rec, &r0, sizeof r0, hipMemcpyHostToDevice) != hipSuccess) {
      rc = LQRO_E_HIP;
    } else {
      HullArgs Hh{};
      memset(&Hh, 0, sizeof Hh);
      Hh.N = 2; Hh.X = X; Hh.H = g.horizon; Hh.NP = g.n_points;
      Hh.row_begin = 0; Hh.row_stride = 1; Hh.npr = 1; Hh.per_agent = 0;
      Hh.r2 = g.vmax_reach * g.vmax_reach; Hh.r2_lo = Hh.r2; Hh.r2_hi = Hh.r2;
      Hh.T = c->d_T; Hh.NCF = c->d_NCF; Hh.S = c->d_S; Hh.x = d_x;
      Hh.planes = d_pl; Hh.recs = d_rec;
      Hh.queue = d_q + 8; Hh.count = d_q + 1; Hh.cap = 1; Hh.next = d_q + 2;   // d_q[8] = 0: slot 0
      Hh.scratch = c->d_hscratch; Hh.iscratch = c->d_hiscratch; Hh.fscratch = c->d_hfscratch;
      Hh.sb = reinterpret_cast<HullPt*>(c->d_hfaces);
      Hh.fbest = c->d_hfbest; Hh.vpid = c->d_hvpid; Hh.stack = c->d_hstack;
      Hh.rqueue = d_q + 12; Hh.rcount = d_q + 3; Hh.rnext = d_q + 4;
      Hh.bigmem = c->d_hbig; Hh.wide = c->d_hwide; Hh.bag = c->d_hbag;
      Hh.stats = d_st; Hh.prof = nullptr;   // the hook never alters the step's statistics
      Hh.lqueue = d_q + 13; Hh.lcount = d_q + 5; Hh.ldone = d_q + 6;
      Hh.ext_pts = d_pts; Hh.ext_n = n; Hh.ext_max = fmax;
      Hh.ext_facets = (local == 1 || !facets) ? nullptr : d_f; Hh.ext_nf = d_q + 7;
      Hh.ext_full = local == 2;   // k_qhull: rounded points, then the full-precision ones
      Hh.qscratch = d_qw; Hh.qstride = qstride; Hh.qnrm = d_qn; Hh.qflags = c->qhull_flags;
      Hh.qstale = d_q + 14; Hh.qstale_count = d_q + 9; Hh.qstale_cap = 1;
      if (local == 2) {
        Hh.big_main = c->qhull_big;
        if (!c->qhull_big) launch_qhull(dim3(1), c->stream, Hh);
        launch_qhull_big(dim3(1), c->stream, Hh);
      }
      else if (local) launch_lhull(dim3(1), c->stream, Hh);
      else launch_hull(dim3(1), c->stream, Hh);
      if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) {
        rc = LQRO_E_HIP;
      } else {
        int qh[16];
        if (hipMemcpy(qh, d_q, sizeof qh, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(rec, d_rec, sizeof *rec, hipMemcpyDeviceToHost) != hipSuccess) {
          rc = LQRO_E_HIP;
        } else if (local == 2) {
          *n_facets = qh[7];                 // k_qhull's build status
          if (facets && hipMemcpy(facets, d_f, sizeof(int) * 3 * fmax, hipMemcpyDeviceToHost) != hipSuccess)
            rc = LQRO_E_HIP;
          // lqro_step's rule: a merge-suspect winner is reported (LQRO_E_QHMERGE)
          unsigned long long mw = 0;
          if (rc == LQRO_OK && hipMemcpy(&mw, d_st + LQRO_ST_MWIN, sizeof mw, hipMemcpyDeviceToHost) != hipSuccess)
            rc = LQRO_E_HIP;
          if (rc == LQRO_OK && mw) rc = LQRO_E_QHMERGE;
        } else if (local) {
          *n_facets = qh[5] > 0 ? -1 : 0;   // handed over: the full hull would decide
        } else {
          *n_facets = qh[7];
          if (qh[3] > 0) *n_facets = -2;     // k_hull's capacity: k_hull_big would decide
          const int k = std::min(qh[7], max_facets);
          if (k > 0 && hipMemcpy(facets, d_f, sizeof(int) * 3 * k, hipMemcpyDeviceToHost) != hipSuccess) rc = LQRO_E_HIP;
        }
      }
    }
  }
  for (void* p : {(void*)d_pts, (void*)d_x, (void*)d_q, (void*)d_f, (void*)d_rec, (void*)d_pl, (void*)d_st,
                  (void*)d_qw, (void*)d_qn})
    if (p) (void)hipFree(p);
  return rc;
}

/* diagnostic (not in lqro.h): n profile words from offset (k_qhull's wave 1
 * and per-class phases of a -DLQRO_QHULL_PROFILE build: offset Q3_PROF_W1) */
int lqro_debug_prof_words(lqro_ctx* c, int64_t offset, int64_t n, unsigned long long* out) {
  if (!c || !out || offset < 0 || n < 0 || offset + n > LQRO_PROF_WORDS) return LQRO_E_ARG;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(wait_last_step(c));
  HIPCHK(hipMemcpy(out, c->d_prof + offset, sizeof(unsigned long long) * (size_t)n, hipMemcpyDeviceToHost));
  return LQRO_OK;
}

/* diagnostic (not in lqro.h): k_lhull's per-job words of the last step
 * (4 x 4096: point ticks, loop ticks at 100 MHz, iterations | nv << 16 |
 * live points << 32, n | fail << 32 | faces << 40) */
int lqro_debug_local_hull_jobs(lqro_ctx* c, unsigned long long* out) {
  if (!c || !out) return LQRO_E_ARG;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(wait_last_step(c));
  HIPCHK(hipMemcpy(out, c->d_prof + 32 + 2 * 4096 + 48, sizeof(unsigned long long) * 4 * 4096, hipMemcpyDeviceToHost));
  return LQRO_OK;
}

/* diagnostic (not in lqro.h): accumulated k_hull phase cycles of a
 * -DLQRO_HULL_PROFILE build */
int lqro_debug_hull_profile(lqro_ctx* c, unsigned long long* out16) {
  if (!c || !out16) return LQRO_E_ARG;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(wait_last_step(c));
  // the documented prefix only (32 hull counters, 2 x 4096 job words, 32
  // pair / wave-phase words): callers size their buffer to it
  HIPCHK(hipMemcpy(out16, c->d_prof, sizeof(unsigned long long) * LQRO_PROF_HULL_WORDS, hipMemcpyDeviceToHost));
  return LQRO_OK;
}

int lqro_get_timings(lqro_ctx* c, float* ms) {
  if (!c || !ms) return LQRO_E_ARG;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(hipEventSynchronize(c->ev[3]));
  HIPCHK(hipEventElapsedTime(&ms[0], c->ev[0], c->ev[1]));
  HIPCHK(hipEventElapsedTime(&ms[1], c->ev[1], c->ev[2]));
  HIPCHK(hipEventElapsedTime(&ms[2], c->ev[2], c->ev[3]));
  HIPCHK(hipEventElapsedTime(&ms[3], c->ev[0], c->ev[3]));
  return LQRO_OK;
}

}  // extern "C"
