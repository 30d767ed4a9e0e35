// lqro_hull.hpp — the inside-hull branch, in-kernel.
//
// Replaces convexHull (LQRObstacles.cpp:867-969), which writes the reachable
// points to pointList.txt at iostream's default 6 significant digits
// (:869-874), runs qconvex.exe twice (:879-880) and takes
//     min_f | n_f . (vrel - P[first vertex of f]) |   (:955-968)
// over the hull facets, n_f from the hull of the ROUNDED points, P at full
// precision.  One single-wave workgroup per inside-hull pair (persistent over
// the queue k_pair fills):
//   1. recomputes the pair's reachable points in reference order (exact, as
//      k_pair does) and their %g round trip (lqro_device.hpp: round6);
//   2. builds the hull of the rounded points by quickhull: a LIFO stack of
//      faces with outside points; each step inserts the furthest point of
//      the popped face, grows its visible region over the face adjacency,
//      links a cone over the horizon and re-distributes the region's outside
//      points over the cone.  Topology (vertex slots, adjacency, stamps) and
//      vertex coordinates live in LDS; outside sets, their extents and the
//      furthest-point keys in per-block global scratch.  With one wave every
//      step is a handful of dependent LDS round trips;
//   3. evaluates the reference's facet formula on every facet (canonical
//      facet order, lowest-index vertex) and writes the
//      half-plane (createHalfPlanes, :1208-1221, inside => mult = +1).
// A point is beyond a face iff n.(p - a) > eps |n|, n = (b-a) x (c-a),
// eps = 1e-13 (max|coord| + 1) — the rule of the oracle's hull, so the facet
// set (unique for points in general position) is the oracle's.  Jobs whose
// hull outgrows the LDS capacities are re-run by k_hull_big with the same
// code and the topology in global memory.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lqro.h"
#include "lqro_device.hpp"

namespace lqro {

#define HULL_WAVES 4             // the points / initial hull / facet phases use 4 waves,
#define HULL_THREADS (64 * HULL_WAVES)   // the insertions one

#define HULL_SBMULT 16           // outside-set segment buffer: HULL_SBMULT * H*NP entries
#define HULL_STKMULT 4           // work stack: HULL_STKMULT * H*NP faces
#define HULL_FB_STRIDE 16384     // per-block face records in global scratch (= big faces)
#define HULL_VG_STRIDE 8192      // per-block vertex records in global scratch (= big vertices)

// an outside-set entry: the point and its (rounded) coordinates, so that
// re-distributing it needs one load
struct HullPt {
  double x, y, z;
  int q, pad;
};

struct HullArgs {
  int N, X, H, NP;
  int row_begin, npr, per_agent;
  double r2, r2_lo, r2_hi;
  const double* T;
  const double* NCF;
  const double* S;
  const double* x;
  float* planes;
  lqro_pair_record* recs;
  const int* queue;
  const int* count;
  int cap;
  int* next;
  double* scratch;                  // per block: H*NP*6 doubles (rounded, full)
  int* iscratch;                    // per block: 2*H*NP ints (moved point, target face)
  float* fscratch;                  // per block: H*NP floats (distance beyond the target)
  HullPt* sb;                       // per block: HULL_SBMULT*H*NP entries (outside-set segments)
  unsigned long long* fbest;        // per block: HULL_FB_STRIDE furthest-point keys
  int* vpid;                        // per block: HULL_VG_STRIDE vertex -> point ids
  int* stack;                       // per block: HULL_STKMULT*H*NP faces
  int* rqueue;                      // pairs that overflowed the LDS variant
  int* rcount;
  int* rnext;
  void* bigmem;                     // per block of k_hull_big: one HullMemBig
  int block_base;                   // scratch index of this launch's block 0
  int big_main;                     // k_hull_big takes the main queue (H*NP too large for LDS)
  int wait_pairs;                   // poll the queue until k_pair has finished
  int pair_blocks;                  //   (its workgroup count)
  const int* pair_done;
  unsigned long long* stats;
  unsigned long long* prof;          // LQRO_HULL_PROFILE: per-phase cycles
};

// Hull topology and vertex coordinates: LDS for the common case, global
// scratch (larger capacities) for the jobs that overflow it.
template <int FMAX, int VTX, class SEG>
struct HullMem {
  static constexpr int kFaces = FMAX, kVerts = VTX;
  SEG seg[FMAX];                     // outside set of face f: sb[off .. off+cnt)
  unsigned short fv[FMAX][3];        // vertex slots, outward counter-clockwise
  unsigned short fa[FMAX][3];        // fa[f][e]: face across edge (fv[e], fv[e+1])
  unsigned short vst[FMAX];          // visible-region stamp (insertion number)
  unsigned short freel[FMAX];        // retired face slots
  unsigned char alive[FMAX];
  double vx[VTX][3];                 // hull vertex coordinates (rounded points)
  unsigned short vmap[VTX];          // horizon: vertex slot -> edge leaving it
};
// LDS variant: extent packed as off << 14 | cnt (H*NP <= 16383, see runtime)
typedef HullMem<4160, 2048, unsigned int> HullMemSmall;   // ~141 KB: LDS
typedef HullMem<16384, 8192, unsigned long long> HullMemBig;   // ~610 KB: global scratch

// per-step work lists (always LDS)
template <int RG, int HZ>
struct HullLdsT {
  static constexpr int kRegion = RG, kHorizon = HZ;
  unsigned short region[RG];                 // visible region of the apex
  int roff[RG], rcnt[RG], rpre[RG + 1];      //   their outside sets
  unsigned short h_a[HZ], h_b[HZ], h_out[HZ], h_new[HZ];   // horizon edges, cone faces
  int hcnt[HZ], hoff[HZ];
  double cn[HZ][8];                          // cone planes: n, a, |n|, eps |n|
  double tr[3 * 128];
  double rk[HULL_THREADS / 64];
  int ri[HULL_THREADS / 64];
  int scan[HULL_THREADS / 64];
  int nf, nfree, nvtx, fail, n, job, slot, init[4], sbtop, sp, qh, it;
  double eps;
};
typedef HullLdsT<512, 128> HullLdsSmall;
typedef HullLdsT<2048, 1024> HullLdsBig;


// Ordering point between the lanes of one wave.  A wave
// executes its LDS and its global memory operations in issue order, so only
// the compiler has to be kept from moving memory operations across this
// point; no s_waitcnt / s_barrier is needed (a workgroup fence would stall on
// every outstanding global store).
__device__ __forceinline__ void hl_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// outside-set extent of face f
__device__ __forceinline__ void seg_get(unsigned int s, int& off, int& cnt) {
  off = (int)(s >> 14); cnt = (int)(s & 0x3FFFu);
}
__device__ __forceinline__ void seg_get(unsigned long long s, int& off, int& cnt) {
  off = (int)(s >> 32); cnt = (int)(s & 0xFFFFFFFFu);
}
__device__ __forceinline__ void seg_put(unsigned int& s, int off, int cnt) {
  s = ((unsigned int)off << 14) | (unsigned int)cnt;
}
__device__ __forceinline__ void seg_put(unsigned long long& s, int off, int cnt) {
  s = ((unsigned long long)(unsigned)off << 32) | (unsigned)cnt;
}

// Barrier across the workgroup's waves.
__device__ __forceinline__ void hl_bar() { __syncthreads(); }

// n = (b-a) x (c-a) of face f
template <class Mem>
__device__ __forceinline__ void hl_normal(const Mem& L, int f, double* n) {
  const double* a = L.vx[L.fv[f][0]];
  const double* b = L.vx[L.fv[f][1]];
  const double* c = L.vx[L.fv[f][2]];
  const double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  const double e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  n[0] = e1[1] * e2[2] - e1[2] * e2[1];
  n[1] = e1[2] * e2[0] - e1[0] * e2[2];
  n[2] = e1[0] * e2[1] - e1[1] * e2[0];
}
// is p beyond face f: d > eps |n| with d = n.(p - a), tested squared (no
// sqrt on the hot path): d > 0 and d^2 > eps^2 (n.n).  *dist = d / |n|.
template <class Mem>
__device__ __forceinline__ bool hl_beyond(const Mem& L, int f, const double* p, double eps2,
                                          double* dist) {
  double n[3];
  hl_normal(L, f, n);
  const double* a = L.vx[L.fv[f][0]];
  const double d = n[0] * (p[0] - a[0]) + n[1] * (p[1] - a[1]) + n[2] * (p[2] - a[2]);
  const double nn = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
  if (dist) *dist = d / sqrt(nn);
  return d > 0.0 && d * d > eps2 * nn;
}


// block-wide argmax of (key, idx), lowest idx on ties; result in every thread
template <class LT>
__device__ __forceinline__ void hl_argmax(LT& L, double& key, int& idx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ok = __shfl_xor(key, off);
    const int oi = __shfl_xor(idx, off);
    if (ok > key || (ok == key && oi < idx)) { key = ok; idx = oi; }
  }
  if (lane == 0) { L.rk[wave] = key; L.ri[wave] = idx; }
  hl_bar();
  key = L.rk[0]; idx = L.ri[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
    if (L.rk[w] > key || (L.rk[w] == key && L.ri[w] < idx)) { key = L.rk[w]; idx = L.ri[w]; }
  hl_bar();
}

// exclusive block scan of v (0/1); total in *tot
template <class LT>
__device__ __forceinline__ int hl_scan(LT& L, int v, int* tot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long b = __ballot(v != 0);
  const int in_wave = __popcll(b & ((1ull << lane) - 1ull));
  if (lane == 0) L.scan[wave] = __popcll(b);
  hl_bar();
  int base = 0, t = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
    if (w < wave) base += L.scan[w];
    t += L.scan[w];
  }
  *tot = t;
  hl_bar();
  return base + in_wave;
}

// exclusive block scan of v (any int); total in *tot
template <class LT>
__device__ __forceinline__ int hl_scan_val(LT& L, int v, int* tot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) L.scan[wave] = x;
  hl_bar();
  int base = 0, t = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
    if (w < wave) base += L.scan[w];
    t += L.scan[w];
  }
  *tot = t;
  hl_bar();
  return base + x - v;
}

#ifdef LQRO_HULL_PROFILE
#define HSUB(k)                                                     \
  do {                                                              \
    if (tid == 0) {                                                 \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
      prof_sub[k] += t_ - prof_last;                                \
      prof_last = t_;                                               \
    }                                                               \
  } while (0)
#define HSTAMP(k)                                                   \
  do {                                                              \
    if (tid == 0) {                                                 \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
      prof_acc[k] += t_ - prof_last;                                \
      prof_last = t_;                                               \
    }                                                               \
  } while (0)
#else
#define HSTAMP(k) do {} while (0)
#define HSUB(k) do {} while (0)
#endif

template <class Mem, class LT>
__device__ __forceinline__ void hull_body(const HullArgs& A, Mem& M, LT& L, bool big) {
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
#ifdef LQRO_HULL_PROFILE
  unsigned long long prof_acc[16] = {0};
  unsigned long long prof_sub[6] = {0};
  unsigned long long prof_last = __builtin_amdgcn_s_memtime();
#endif
  const int HNP = A.H * A.NP;
  const int hb = A.block_base + blockIdx.x;                   // scratch slot
  double* Pr = A.scratch + (size_t)hb * HNP * 6;    // rounded points
  double* Pf = Pr + (size_t)HNP * 3;                         // full-precision points
  int* tq = A.iscratch + (size_t)hb * HNP * 2;      // moved point ids
  int* th = tq + HNP;                                        // their target cone face
  float* td = A.fscratch + (size_t)hb * HNP;         // distance beyond it
  HullPt* sb = A.sb + (size_t)hb * HNP * HULL_SBMULT;
  const int sbcap = HNP * HULL_SBMULT;
  // per face: furthest outside point (dist bits << 32) | ~q, outside-set extent
  unsigned long long* fbest = A.fbest + (size_t)hb * HULL_FB_STRIDE;
  int* vpid = A.vpid + (size_t)hb * HULL_VG_STRIDE;
  int* stk = A.stack + (size_t)hb * HNP * HULL_STKMULT;
  const int stkcap = HNP * HULL_STKMULT;

  const bool retryq = big && !A.big_main;
  const int* queue = retryq ? A.rqueue : A.queue;
  const int* qcount = retryq ? A.rcount : A.count;
  int* qnext = retryq ? A.rnext : A.next;
  for (;;) {
    // Take the next job.  Workers launched beside k_pair (wait_pairs) poll:
    // an entry is valid once k_pair's release-store made it non-negative,
    // and the queue is closed when every k_pair workgroup has finished.
    if (tid == 0) {
      const int job = atomicAdd(qnext, 1);
      int slot = -1;
      for (long spins = 0;; ++spins) {
        const int cnt = __hip_atomic_load(qcount, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (job < min(cnt, A.cap)) {
          int v = __hip_atomic_load(queue + job, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
          for (long w = 0; v < 0 && w < (1l << 26); ++w) {
            __builtin_amdgcn_s_sleep(2);
            v = __hip_atomic_load(queue + job, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
          }
          slot = v;
          break;
        }
        if (retryq || !A.wait_pairs) break;
        if (__hip_atomic_load(A.pair_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= A.pair_blocks) {
          if (job < min(__hip_atomic_load(qcount, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT), A.cap))
            continue;
          break;
        }
        if (spins > (1l << 26)) { atomicAdd(&A.stats[4], 1ull); break; }   // bounded wait
        __builtin_amdgcn_s_sleep(8);
      }
      L.job = job;
      L.slot = slot;
    }
    hl_bar();
    const int job = L.job;
    const int slot = L.slot;
    if (slot < 0) break;
    const int lrow = slot / A.npr, jj = slot % A.npr;
    const int i = A.row_begin + lrow;
    const int j = jj < i ? jj : jj + 1;
    const double* xi = A.x + (size_t)i * A.X;
    const double* xj = A.x + (size_t)j * A.X;
    const double* Ti = A.T + (A.per_agent ? (size_t)i * A.H * 9 : 0);
    const double* Ni = A.NCF + (A.per_agent ? (size_t)i * A.H * 3 * A.X : 0);
    const double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};
#ifdef LQRO_HULL_PROFILE
    const unsigned long long job_t0 = __builtin_amdgcn_s_memtime();
#endif

    HSTAMP(15);
    // 1. reachable points in reference order, full + %g-rounded
    if (tid == 0) { L.n = 0; L.fail = 0; }
    hl_bar();
    for (int k0 = 0; k0 < A.H; k0 += 128) {
      for (int it = tid; it < 3 * 128; it += blockDim.x) {
        const int k = k0 + it / 3, r = it % 3;
        if (k < A.H) {
          double d = 0.0;
          for (int c = 0; c < A.X; ++c) d += Ni[((size_t)k * 3 + r) * A.X + c] * (xi[c] - xj[c]);
          L.tr[it] = d;
        }
      }
      hl_bar();
      const int kend = min(A.H, k0 + 128);
      for (int q0 = k0 * A.NP; q0 < kend * A.NP; q0 += blockDim.x) {
        const int q = q0 + tid;
        bool ok = false;
        double p0 = 0, p1 = 0, p2 = 0;
        if (q < kend * A.NP) {
          const int k = q / A.NP, p = q % A.NP;
          const double* Tk = Ti + (size_t)k * 9;
          const double* tk = L.tr + (k - k0) * 3;
          const double u0 = A.S[3 * p] + tk[0], u1 = A.S[3 * p + 1] + tk[1], u2 = A.S[3 * p + 2] + tk[2];
          p0 = ((0.0 + Tk[0] * u0) + Tk[1] * u1) + Tk[2] * u2;
          p1 = ((0.0 + Tk[3] * u0) + Tk[4] * u1) + Tk[5] * u2;
          p2 = ((0.0 + Tk[6] * u0) + Tk[7] * u1) + Tk[8] * u2;
          const double a = p0 - vrel[0], b = p1 - vrel[1], c = p2 - vrel[2];
          const double t = a * a + b * b + c * c;
          if (t < A.r2_lo) ok = true;
          else if (t > A.r2_hi) ok = false;
          else ok = (a * a) / A.r2 + (b * b) / A.r2 + (c * c) / A.r2 < 1.0;
        }
        int tot;
        const int pos = L.n + hl_scan(L, ok ? 1 : 0, &tot);
        if (ok) {
          int oor = 0;
          Pf[3 * pos] = p0; Pf[3 * pos + 1] = p1; Pf[3 * pos + 2] = p2;
          Pr[3 * pos] = round6(p0, &oor);
          Pr[3 * pos + 1] = round6(p1, &oor);
          Pr[3 * pos + 2] = round6(p2, &oor);
          if (oor) L.fail = 7;
        }
        hl_bar();
        if (tid == 0) L.n += tot;
        hl_bar();
      }
    }
    const int n = L.n;

    // 2. tolerance, as the oracle's hull: 1e-13 (max|coord| + 1)
    {
      double mx = 0.0;
      int dummy = 0;
      for (int q = tid; q < 3 * n; q += blockDim.x) mx = fmax(mx, fabs(Pr[q]));
      hl_argmax(L, mx, dummy);
      if (tid == 0) {
        L.eps = 1e-13 * (mx + 1.0);
        if (n < 4) L.fail = 8;
      }
      hl_bar();
    }
    const double eps = L.eps;
    const double eps2 = eps * eps;

    HSTAMP(0);
    // 3. initial tetrahedron from extreme points
    if (!L.fail) {
      double key; int idx;
      key = -INFINITY; idx = INT_MAX;
      for (int q = tid; q < n; q += blockDim.x) {
        const double v = -Pr[3 * q];
        if (v > key || (v == key && q < idx)) { key = v; idx = q; }
      }
      hl_argmax(L, key, idx);
      const int i0 = idx;
      const double* P0 = Pr + 3 * i0;
      key = -INFINITY; idx = INT_MAX;
      for (int q = tid; q < n; q += blockDim.x) {
        const double dx = Pr[3 * q] - P0[0], dy = Pr[3 * q + 1] - P0[1], dz = Pr[3 * q + 2] - P0[2];
        const double v = dx * dx + dy * dy + dz * dz;
        if (v > key || (v == key && q < idx)) { key = v; idx = q; }
      }
      hl_argmax(L, key, idx);
      const int i1 = idx;
      const double* P1 = Pr + 3 * i1;
      key = -INFINITY; idx = INT_MAX;
      for (int q = tid; q < n; q += blockDim.x) {
        const double e1[3] = {P1[0] - P0[0], P1[1] - P0[1], P1[2] - P0[2]};
        const double e2[3] = {Pr[3 * q] - P0[0], Pr[3 * q + 1] - P0[1], Pr[3 * q + 2] - P0[2]};
        const double cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2], cz = e1[0] * e2[1] - e1[1] * e2[0];
        const double v = cx * cx + cy * cy + cz * cz;
        if (v > key || (v == key && q < idx)) { key = v; idx = q; }
      }
      hl_argmax(L, key, idx);
      const int i2 = idx;
      if (tid == 0) {
        for (int d = 0; d < 3; ++d) {
          M.vx[0][d] = Pr[3 * i0 + d]; M.vx[1][d] = Pr[3 * i1 + d]; M.vx[2][d] = Pr[3 * i2 + d];
        }
        M.fv[0][0] = 0; M.fv[0][1] = 1; M.fv[0][2] = 2;
      }
      hl_bar();
      key = -INFINITY; idx = INT_MAX;
      for (int q = tid; q < n; q += blockDim.x) {
        double dd;
        hl_beyond(M, 0, Pr + 3 * q, eps2, &dd);
        const double v = fabs(dd);
        if (v > key || (v == key && q < idx)) { key = v; idx = q; }
      }
      hl_argmax(L, key, idx);
      const int i3 = idx;
      if (tid == 0) {
        if (!(key > eps) || i0 == i1 || i1 == i2 || i2 == i3) L.fail = 8;
        L.init[0] = i0; L.init[1] = i1; L.init[2] = i2; L.init[3] = i3;
        if (!L.fail) {
          for (int v = 0; v < 4; ++v) {
            vpid[v] = L.init[v];
            for (int d = 0; d < 3; ++d) M.vx[v][d] = Pr[3 * L.init[v] + d];
          }
          L.nvtx = 4;
          const int fvv[4][3] = {{0, 1, 2}, {0, 3, 1}, {1, 3, 2}, {0, 2, 3}};
          for (int f = 0; f < 4; ++f) {
            for (int e = 0; e < 3; ++e) M.fv[f][e] = (unsigned short)fvv[f][e];
            const int other = 6 - fvv[f][0] - fvv[f][1] - fvv[f][2];
            double dd;
            hl_beyond(M, f, M.vx[other], 0.0, &dd);
            if (dd > 0) { const unsigned short t = M.fv[f][1]; M.fv[f][1] = M.fv[f][2]; M.fv[f][2] = t; }
            M.alive[f] = 1;
          }
          for (int f = 0; f < 4; ++f)
            for (int e = 0; e < 3; ++e) {
              const int a = M.fv[f][e], b = M.fv[f][(e + 1) % 3];
              for (int g = 0; g < 4; ++g)
                for (int e2 = 0; e2 < 3; ++e2)
                  if (M.fv[g][e2] == b && M.fv[g][(e2 + 1) % 3] == a) M.fa[f][e] = (unsigned short)g;
            }
          L.nf = 4;
          L.nfree = 0;
        }
      }
      hl_bar();
    }

    if (!L.fail) {
      // 4. outside sets of the tetrahedron's faces
      if (tid < 4) { fbest[tid] = 0ull; L.hcnt[tid] = 0; }
      if (tid == 0) { L.sbtop = 0; L.sp = 0; L.qh = 0; L.it = 0; }
      hl_bar();
      for (int q = tid; q < n; q += blockDim.x) {
        int c = -1;
        double dd = 0.0;
        if (q != L.init[0] && q != L.init[1] && q != L.init[2] && q != L.init[3]) {
          const double p[3] = {Pr[3 * q], Pr[3 * q + 1], Pr[3 * q + 2]};
          for (int f = 0; f < 4; ++f)
            if (hl_beyond(M, f, p, eps2, &dd)) { c = f; break; }
        }
        th[q] = c;
        td[q] = (float)dd;
        if (c >= 0) atomicAdd(&L.hcnt[c], 1);
      }
      hl_bar();
      if (tid == 0) {
        int o = 0;
        for (int f = 0; f < 4; ++f) {
          seg_put(M.seg[f], o, L.hcnt[f]);
          L.hoff[f] = o;
          o += L.hcnt[f];
          M.vst[f] = 0;
        }
        for (int f = 0; f < 4; ++f)
          if (L.hcnt[f] > 0) stk[L.sp++] = f;
        L.sbtop = o;
      }
      hl_bar();
      for (int q = tid; q < n; q += blockDim.x) {
        const int c = th[q];
        if (c < 0) continue;
        HullPt e;
        e.x = Pr[3 * q]; e.y = Pr[3 * q + 1]; e.z = Pr[3 * q + 2]; e.q = q; e.pad = 0;
        sb[atomicAdd(&L.hoff[c], 1)] = e;
        const unsigned long long key =
            ((unsigned long long)__float_as_uint(td[q]) << 32) | (unsigned long long)(~(unsigned)q);
        atomicMax(&fbest[c], key);
      }
      hl_bar();

      HSTAMP(1);
      // Insertions run on wave 0 alone (the other waves helped with the
      // points and the initial hull and wait for the facet selection).
      if (wave == 0) {
      // 5. quickhull: take the oldest live face with outside points (FIFO
      //    work queue: the hull grows evenly, which wastes fewer insertions
      //    on points that later fall inside than depth-first order), insert
      //    its furthest point.  One wave, and every insertion is a chain of
      //    dependent LDS round trips, so the loop keeps its control state in
      //    (wave-uniform) registers, passes lists between lanes with ballots,
      //    readlane and DPP scans, and touches LDS only for the topology.
      // The next queue entry's face, key and apex coordinates are fetched
      // during the current insertion (three dependent global loads off the
      // critical path).  They stay valid unless that face is retired (it is
      // in the current region) or was dead when checked (its slot may be
      // reused by a cone face of this insertion).
      int qh = 0, sp = L.sp, nvtx = L.nvtx, it = 0, nf = L.nf, nfree = L.nfree, sbtop = L.sbtop;
      int fail = 0;
      const unsigned long long lt = (1ull << tid) - 1ull;
      int pf_idx = -1, pf_face = 0;
      bool pf_ok = false;
      unsigned long long pf_key = 0ull;
      double pf_p[3] = {0.0, 0.0, 0.0};
      for (;;) {
        if (qh == sp) break;
        const bool use_pf = pf_ok && pf_idx == qh;
        const int f = use_pf ? pf_face : stk[qh];
        ++qh;
        // stale entries: the face was retired (its slot maybe reused by a
        // face without outside points) after it was pushed
        const unsigned long long key = use_pf ? pf_key : fbest[f];
        pf_ok = false;
        if (!M.alive[f] || key == 0ull) continue;
        const int apex = (int)(~(unsigned)(key & 0xFFFFFFFFull));
        if (apex < 0 || apex >= n || it >= 4 * Mem::kVerts) { fail = 9; break; }
        if (nvtx >= Mem::kVerts) { fail = 1; break; }
        const int av = nvtx++;
        const unsigned short stamp = (unsigned short)(++it);
        double p[3];
        if (use_pf) { p[0] = pf_p[0]; p[1] = pf_p[1]; p[2] = pf_p[2]; }
        else { p[0] = Pr[3 * apex]; p[1] = Pr[3 * apex + 1]; p[2] = Pr[3 * apex + 2]; }
        pf_idx = qh < sp ? qh : -1;
        if (pf_idx >= 0) pf_face = stk[pf_idx];
        if (tid == 0) {
          M.vx[av][0] = p[0]; M.vx[av][1] = p[1]; M.vx[av][2] = p[2];
          vpid[av] = apex;
          M.vst[f] = stamp;
        }
        hl_sync();
        HSTAMP(2);
        // (a) visible region: grown over adjacency from f; lanes 0..2 test
        //     the three neighbours of one region face at a time.  Lane r
        //     holds region face r (LDS copy for r >= 64 and for later phases).
        int rg = tid == 0 ? f : -1;
        if (tid == 0) L.region[0] = (unsigned short)f;
        int R = 1;
        for (int r = 0; r < R; ++r) {
          const int g = r < 64 ? __builtin_amdgcn_readlane(rg, r) : (int)L.region[r];
          int nb = -1, vis = 0;
          if (tid < 3) {
            nb = M.fa[g][tid];
            vis = (M.vst[nb] != stamp) && hl_beyond(M, nb, p, eps2, nullptr);
          }
          const unsigned long long b = __ballot(vis);
          if (vis) {
            const int pos = R + __popcll(b & lt);
            if (pos < LT::kRegion) { L.region[pos] = (unsigned short)nb; M.vst[nb] = stamp; }
          }
          // hand the new entries to lanes R, R+1, ...
          const int n0 = __builtin_amdgcn_readlane(nb, 0), n1 = __builtin_amdgcn_readlane(nb, 1),
                    n2 = __builtin_amdgcn_readlane(nb, 2);
          int k = R;
          if (b & 1ull) { if (tid == k) rg = n0; ++k; }
          if (b & 2ull) { if (tid == k) rg = n1; ++k; }
          if (b & 4ull) { if (tid == k) rg = n2; ++k; }
          R = k;
          if (R > LT::kRegion) break;
          hl_sync();
        }
        if (R > LT::kRegion) { fail = 2; break; }
        if (pf_idx >= 0) {
          pf_ok = M.alive[pf_face] && M.vst[pf_face] != stamp;
          if (pf_ok) pf_key = fbest[pf_face];
        }
        HSTAMP(3);
        // (b) horizon: region edges whose neighbour is not in the region,
        //     in (region order, edge) order
        int nh = 0;
        for (int b0 = 0; b0 < 3 * R; b0 += 64) {
          const int t = b0 + tid;
          int ha = 0, hb = 0, ho = 0, is = 0;
          if (t < 3 * R) {
            const int g = L.region[t / 3], e = t % 3;
            ho = M.fa[g][e];
            if (M.vst[ho] != stamp) { is = 1; ha = M.fv[g][e]; hb = M.fv[g][(e + 1) % 3]; }
          }
          const unsigned long long b = __ballot(is);
          const int pos = nh + __popcll(b & lt);
          if (is && pos < LT::kHorizon) {
            L.h_a[pos] = (unsigned short)ha; L.h_b[pos] = (unsigned short)hb; L.h_out[pos] = (unsigned short)ho;
          }
          nh += __popcll(b);
        }
        if (nh > LT::kHorizon || nh < 3) { fail = 3; break; }
        const int nf0 = nf, nfree0 = nfree;
        if (nf0 + max(0, nh - nfree0) > Mem::kFaces) { fail = 4; break; }
        // (c) cone face slots (retired slots first) and the vertex -> edge map
        for (int h = tid; h < nh; h += 64) {
          const int sf = h < nfree0 ? M.freel[nfree0 - 1 - h] : nf0 + (h - nfree0);
          L.h_new[h] = (unsigned short)sf;
          M.vmap[L.h_a[h]] = (unsigned short)h;
          L.hcnt[h] = 0;
        }
        hl_sync();
        HSTAMP(4);
        // (d) cone faces (a, b, apex): adjacency, outer neighbours, planes
        int bad = 0;
        for (int h = tid; h < nh; h += 64) {
          const int sf = L.h_new[h];
          const int ha = L.h_a[h], hb = L.h_b[h], on = L.h_out[h];
          const int k = M.vmap[hb];                    // edge leaving b
          M.fv[sf][0] = (unsigned short)ha;
          M.fv[sf][1] = (unsigned short)hb;
          M.fv[sf][2] = (unsigned short)av;
          M.fa[sf][0] = (unsigned short)on;
          M.fa[sf][1] = L.h_new[k];                    // across (b, apex)
          M.fa[L.h_new[k]][2] = (unsigned short)sf;    // k's (apex, a_k = b)
          M.vst[sf] = 0;
          for (int e = 0; e < 3; ++e)
            if (M.fv[on][e] == hb && M.fv[on][(e + 1) % 3] == ha) M.fa[on][e] = (unsigned short)sf;
          if (L.h_a[k] != hb) bad = 1;
          // plane of the new face, as hl_normal / hl_beyond compute it
          const double* a = M.vx[ha];
          const double* bb = M.vx[hb];
          const double e1[3] = {bb[0] - a[0], bb[1] - a[1], bb[2] - a[2]};
          const double e2[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
          const double nx = e1[1] * e2[2] - e1[2] * e2[1];
          const double ny = e1[2] * e2[0] - e1[0] * e2[2];
          const double nz = e1[0] * e2[1] - e1[1] * e2[0];
          double* cp = L.cn[h];
          cp[0] = nx; cp[1] = ny; cp[2] = nz;
          cp[3] = a[0]; cp[4] = a[1]; cp[5] = a[2];
          const double nn = nx * nx + ny * ny + nz * nz;
          cp[6] = 1.0 / sqrt(nn);                      // for the distance key only
          cp[7] = eps2 * nn;
          fbest[sf] = 0ull;
        }
        if (__ballot(bad)) { fail = 5; break; }
        // retired faces' outside-set extents: lane r holds region face r's
        // (r < 64; longer regions take the scratch path below)
        int roff = 0, rcnt = 0;
        if (tid < R) {
          const int g = R <= 64 ? rg : (int)L.region[tid];
          seg_get(M.seg[g], roff, rcnt);
        }
        const int rinc = wave_incl_scan(rcnt);          // prefix over region faces
        const int total = R <= 64 ? __builtin_amdgcn_readlane(rinc, 63) : -1;
        HSTAMP(5);
        if (pf_ok) {
          const int pa = (int)(~(unsigned)(pf_key & 0xFFFFFFFFull));
          if (pa >= 0 && pa < n) { pf_p[0] = Pr[3 * pa]; pf_p[1] = Pr[3 * pa + 1]; pf_p[2] = Pr[3 * pa + 2]; }
        }
        HSUB(0);
        // (e) the retired faces' outside points: first cone face they are beyond
        if (total >= 0 && total <= 4 * 64) {
          // up to four points per lane; each point's rank within its target
          // cone face from an LDS atomic; no scratch round trip
          int tg[4], rk[4];
          HullPt pt[4];
          float dv[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            tg[c] = -1; rk[c] = 0; dv[c] = 0.0f; pt[c].q = -1;
            const int t = c * 64 + tid;
            if (c * 64 < total) {
              // region face holding item t: the first r with rinc[r] > t
              int lo = 0, base = 0, off0 = __builtin_amdgcn_readlane(roff, 0);
              for (int r = 0; r < R - 1; ++r) {
                const int inc = __builtin_amdgcn_readlane(rinc, r);
                if (t >= inc) { lo = r + 1; base = inc; }
              }
              for (int r = 1; r < R; ++r) {
                const int o = __builtin_amdgcn_readlane(roff, r);
                if (r == lo) off0 = o;
              }
              if (t < total) pt[c] = sb[off0 + (t - base)];
            }
          }
          HSUB(1);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int q = pt[c].q;
            if (q >= 0 && q != apex) {
              const double x0 = pt[c].x, x1 = pt[c].y, x2 = pt[c].z;
              for (int h = 0; h < nh; ++h) {
                const double* cp = L.cn[h];
                const double d = cp[0] * (x0 - cp[3]) + cp[1] * (x1 - cp[4]) + cp[2] * (x2 - cp[5]);
                if (d > 0.0 && d * d > cp[7]) { tg[c] = h; dv[c] = (float)(d * cp[6]); break; }
              }
              if (tg[c] >= 0) rk[c] = atomicAdd(&L.hcnt[tg[c]], 1);
            }
          }
          hl_sync();
          HSUB(2);
          int run = sbtop;
          for (int h0 = 0; h0 < nh; h0 += 64) {
            const int h = h0 + tid;
            const int v = h < nh ? L.hcnt[h] : 0;
            const int x = wave_incl_scan(v);
            if (h < nh) {
              L.hoff[h] = run + x - v;
              seg_put(M.seg[L.h_new[h]], run + x - v, v);
            }
            run += __builtin_amdgcn_readlane(x, 63);
          }
          if (run > sbcap) { fail = 6; break; }
          hl_sync();
          HSUB(3);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (tg[c] >= 0) {
              sb[L.hoff[tg[c]] + rk[c]] = pt[c];
              const unsigned long long k2 =
                  ((unsigned long long)__float_as_uint(dv[c]) << 32) | (unsigned long long)(~(unsigned)pt[c].q);
              atomicMax(&fbest[L.h_new[tg[c]]], k2);
            }
          }
          HSUB(4);
          sbtop = run;
          HSUB(5);
        } else {
          // long regions / many points: through LDS + scratch
          for (int r = tid; r < R; r += 64) {
            int so, sc;
            seg_get(M.seg[L.region[r]], so, sc);
            L.roff[r] = so;
            L.rcnt[r] = sc;
          }
          hl_sync();
          int run0 = 0;
          for (int r0 = 0; r0 < R; r0 += 64) {
            const int r = r0 + tid;
            const int v = r < R ? L.rcnt[r] : 0;
            const int x = wave_incl_scan(v);
            if (r < R) L.rpre[r] = run0 + x - v;
            run0 += __builtin_amdgcn_readlane(x, 63);
          }
          if (tid == 0) L.rpre[R] = run0;
          hl_sync();
          const int tot2 = run0;
          for (int t = tid; t < tot2; t += 64) {
            int lo = 0, hi = R - 1;
            while (lo < hi) {
              const int mid = (lo + hi + 1) >> 1;
              if (L.rpre[mid] <= t) lo = mid; else hi = mid - 1;
            }
            const HullPt e = sb[L.roff[lo] + (t - L.rpre[lo])];
            const int q = e.q;
            int tgt = -1;
            float dd = 0.0f;
            if (q != apex) {
              const double x0 = e.x, x1 = e.y, x2 = e.z;
              for (int h = 0; h < nh; ++h) {
                const double* cp = L.cn[h];
                const double d = cp[0] * (x0 - cp[3]) + cp[1] * (x1 - cp[4]) + cp[2] * (x2 - cp[5]);
                if (d > 0.0 && d * d > cp[7]) { tgt = h; dd = (float)(d * cp[6]); break; }
              }
            }
            tq[t] = q;
            th[t] = tgt;
            td[t] = dd;
            if (tgt >= 0) atomicAdd(&L.hcnt[tgt], 1);
          }
          hl_sync();
          int run = sbtop;
          for (int h0 = 0; h0 < nh; h0 += 64) {
            const int h = h0 + tid;
            const int v = h < nh ? L.hcnt[h] : 0;
            const int x = wave_incl_scan(v);
            if (h < nh) {
              seg_put(M.seg[L.h_new[h]], run + x - v, v);
              L.hoff[h] = run + x - v;
            }
            run += __builtin_amdgcn_readlane(x, 63);
          }
          if (run > sbcap) { fail = 6; break; }
          sbtop = run;
          hl_sync();
          for (int t = tid; t < tot2; t += 64) {
            const int h = th[t];
            if (h < 0) continue;
            const int q = tq[t];
            HullPt e;
            e.x = Pr[3 * q]; e.y = Pr[3 * q + 1]; e.z = Pr[3 * q + 2]; e.q = q; e.pad = 0;
            sb[atomicAdd(&L.hoff[h], 1)] = e;
            const unsigned long long k2 =
                ((unsigned long long)__float_as_uint(td[t]) << 32) | (unsigned long long)(~(unsigned)q);
            atomicMax(&fbest[L.h_new[h]], k2);
          }
        }
        HSTAMP(6);
        // (f) retire the region, commit the cone, push the cone faces that
        //     have outside points (in horizon order)
        const int used = min(nh, nfree0);
        for (int r = tid; r < R; r += 64) {
          const int g = R <= 64 ? rg : (int)L.region[r];
          M.alive[g] = 0;
          M.freel[nfree0 - used + r] = (unsigned short)g;
        }
        int npush = 0;
        for (int h0 = 0; h0 < nh; h0 += 64) {
          const int h = h0 + tid;
          int is = 0;
          if (h < nh) {
            M.alive[L.h_new[h]] = 1;
            is = L.hcnt[h] > 0;
          }
          const unsigned long long b = __ballot(is);
          const int pos = sp + npush + __popcll(b & lt);
          if (is && pos < stkcap) stk[pos] = L.h_new[h];
          npush += __popcll(b);
        }
        if (sp + npush > stkcap) { fail = 6; break; }
        nfree = nfree0 - used + R;
        nf = nf0 + (nh - used);
        sp += npush;
        hl_sync();
        HSTAMP(7);
#ifdef LQRO_HULL_PROFILE
        if (tid == 0) { prof_acc[14] += 1; prof_acc[10] += (unsigned long long)R; prof_acc[11] += (unsigned long long)nh; prof_acc[12] += (unsigned long long)(total > 0 ? total : 0); }
#endif
      }
      if (tid == 0) {
        L.nf = nf; L.nfree = nfree; L.nvtx = nvtx; L.sbtop = sbtop; L.sp = sp;
        if (fail) L.fail = fail;
      }
      }
      hl_bar();
    }
    hl_bar();

    HSTAMP(8);
    // 6. the reference's facet selection over all facets (canonical order)
    double best = INFINITY;
    int bt0 = INT_MAX, bt1 = INT_MAX, bt2 = INT_MAX, nfac = 0;
    double bn[3] = {0, 0, 0};
    if (!L.fail) {
      for (int f = tid; f < L.nf; f += blockDim.x) {
        if (!M.alive[f]) continue;
        nfac++;
        int t0 = vpid[M.fv[f][0]], t1 = vpid[M.fv[f][1]], t2 = vpid[M.fv[f][2]];
        while (!(t0 < t1 && t0 < t2)) { const int a = t0; t0 = t1; t1 = t2; t2 = a; }
        const double *a = Pr + 3 * t0, *b = Pr + 3 * t1, *c = Pr + 3 * t2;
        const double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
        const double e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
        double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        const double len = sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
        nv[0] /= len; nv[1] /= len; nv[2] /= len;
        const double* p0 = Pf + 3 * t0;
        const double dd = fabs(nv[0] * (vrel[0] - p0[0]) + nv[1] * (vrel[1] - p0[1]) + nv[2] * (vrel[2] - p0[2]));
        const int s1 = min(t1, t2), s2 = max(t1, t2);
        const bool bt = dd < best || (dd == best && (t0 < bt0 || (t0 == bt0 && (s1 < bt1 || (s1 == bt1 && s2 < bt2)))));
        if (bt) { best = dd; bt0 = t0; bt1 = s1; bt2 = s2; bn[0] = nv[0]; bn[1] = nv[1]; bn[2] = nv[2]; }
      }
    }
    // block arg-min by (distance, triple): wave shuffles, then across waves
    {
      const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const double ob = __shfl_xor(best, off);
        const int o0 = __shfl_xor(bt0, off), o1 = __shfl_xor(bt1, off), o2 = __shfl_xor(bt2, off);
        const double on0 = __shfl_xor(bn[0], off), on1 = __shfl_xor(bn[1], off), on2 = __shfl_xor(bn[2], off);
        nfac += __shfl_xor(nfac, off);
        const bool bt = ob < best || (ob == best && (o0 < bt0 || (o0 == bt0 && (o1 < bt1 || (o1 == bt1 && o2 < bt2)))));
        if (bt) { best = ob; bt0 = o0; bt1 = o1; bt2 = o2; bn[0] = on0; bn[1] = on1; bn[2] = on2; }
      }
      __shared__ double s_best[HULL_THREADS / 64], s_n[HULL_THREADS / 64][3];
      __shared__ int s_t[HULL_THREADS / 64][3], s_cnt[HULL_THREADS / 64];
      if (lane == 0) {
        s_best[wave] = best; s_t[wave][0] = bt0; s_t[wave][1] = bt1; s_t[wave][2] = bt2;
        s_n[wave][0] = bn[0]; s_n[wave][1] = bn[1]; s_n[wave][2] = bn[2]; s_cnt[wave] = nfac;
      }
      hl_bar();
      if (tid == 0) {
        int fo = 0, total = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
          total += s_cnt[w];
          const bool bt = s_best[w] < s_best[fo] ||
                          (s_best[w] == s_best[fo] &&
                           (s_t[w][0] < s_t[fo][0] || (s_t[w][0] == s_t[fo][0] &&
                            (s_t[w][1] < s_t[fo][1] || (s_t[w][1] == s_t[fo][1] && s_t[w][2] < s_t[fo][2])))));
          if (bt) fo = w;
        }
        const bool ok = !L.fail && total > 0 && s_t[fo][0] != INT_MAX;
        // capacity overflow in the LDS variant: hand the pair to k_hull_big
        const bool retry = !big && L.fail >= 1 && L.fail <= 4;
#ifdef LQRO_HULL_PROFILE
        if (A.prof) atomicAdd(&A.prof[16 + (L.fail & 15)], 1ull);
#endif
        if (retry) {
          const int r = atomicAdd(A.rcount, 1);
          if (r < A.cap) A.rqueue[r] = slot;
        }
        float* pl = A.planes + (size_t)slot * 8;
        const double distance = s_best[fo];
        const double nrm[3] = {s_n[fo][0], s_n[fo][1], s_n[fo][2]};
        if (retry) {
          // written by k_hull_big
        } else if (ok) {
          const double dh = distance * 0.5;                  // :1416
          const double mult = 1.0;                           // :1213
          pl[0] = (float)(xi[3] + mult * dh * nrm[0]);
          pl[1] = (float)(xi[4] + mult * dh * nrm[1]);
          pl[2] = (float)(xi[5] + mult * dh * nrm[2]);
          pl[3] = (float)nrm[0]; pl[4] = (float)nrm[1]; pl[5] = (float)nrm[2];
          pl[6] = __int_as_float(1);
          atomicAdd(&A.stats[3], 1ull);
        } else {
          pl[6] = __int_as_float(0);                         // no usable plane
          atomicAdd(&A.stats[4], 1ull);
        }
        if (A.recs && !retry) {
          lqro_pair_record& rec = A.recs[slot];
          rec.flags |= ok ? LQRO_REC_HULL : LQRO_REC_HULLFAIL;
          rec.n_facets = ok ? total : -1;
          if (ok) {
            rec.facet[0] = s_t[fo][0]; rec.facet[1] = s_t[fo][1]; rec.facet[2] = s_t[fo][2];
            rec.dist = distance;
            for (int q = 0; q < 3; ++q) {
              rec.normal[q] = nrm[q];
              rec.plane_point[q] = pl[q];
              rec.plane_normal[q] = pl[3 + q];
            }
          }
        }
      }
      hl_bar();
    }
    HSTAMP(9);
#ifdef LQRO_HULL_PROFILE
    if (tid == 0 && A.prof && job < 2048) {
      const int pj = 32 + 2 * (big ? 2048 + job : job);
      A.prof[pj] = __builtin_amdgcn_s_memtime() - job_t0;
      A.prof[pj + 1] = (unsigned long long)L.nvtx | ((unsigned long long)n << 20) |
                       ((unsigned long long)L.fail << 40) | ((unsigned long long)slot << 44);
    }
#endif
  }
#ifdef LQRO_HULL_PROFILE
  if (tid == 0 && A.prof)
    for (int k = 0; k < 16; ++k) atomicAdd(&A.prof[k], prof_acc[k]);
  if (tid == 0 && A.prof)
    for (int k = 0; k < 6; ++k) atomicAdd(&A.prof[26 + k], prof_sub[k]);
#endif
}

__global__ void __launch_bounds__(HULL_THREADS) k_hull(HullArgs A) {
  __shared__ HullLdsSmall L;
  __shared__ HullMemSmall M;
  hull_body(A, M, L, false);
}

__global__ void __launch_bounds__(HULL_THREADS) k_hull_big(HullArgs A) {
  __shared__ HullLdsBig L;
  HullMemBig& M = reinterpret_cast<HullMemBig*>(A.bigmem)[blockIdx.x];
  hull_body(A, M, L, true);
}

}  // namespace lqro
