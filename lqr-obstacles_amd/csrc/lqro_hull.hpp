// lqro_hull.hpp — the inside-hull branch, in-kernel.
//
// Replaces convexHull (LQRObstacles.cpp:867-969), which writes the reachable
// points to pointList.txt at iostream's default 6 significant digits
// (:869-874), runs qconvex.exe twice (:879-880) and takes
//     min_f | n_f . (vrel - P[first vertex of f]) |   (:955-968)
// over the hull facets, n_f from the hull of the ROUNDED points, P at full
// precision.  Here one workgroup per inside-hull pair (persistent over the
// queue k_pair fills):
//   1. recomputes the pair's reachable points in reference order (exact, as
//      k_pair does) and their %g round trip (lqro_device.hpp: round6);
//   2. builds the hull of the rounded points by quickhull.  The hull's
//      vertices (coordinates) and faces (vertex slots + adjacency) live in
//      LDS; every insertion step — visible faces, horizon, cone, reassignment
//      of outside points — runs across the workgroup.  Each point keeps the
//      face it is outside of ("conflict") in global scratch, and an active
//      list shrinks as points fall inside;
//   3. evaluates the reference's facet formula on every facet (canonical
//      facet order, lowest-index vertex) and writes the
//      half-plane (createHalfPlanes, :1208-1221, inside => mult = +1).
// A point is beyond a face iff n.(p - a) > eps |n|, n = (b-a) x (c-a),
// eps = 1e-13 (max|coord| + 1) — the rule of the oracle's hull, so the facet
// set (unique for points in general position) is the oracle's.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lqro.h"
#include "lqro_device.hpp"

namespace lqro {

#define HULL_THREADS 256
#define HULL_FMAX 3072     // face slots per workgroup
#define HULL_VTX 1400      // hull vertex slots per workgroup
#define HULL_SBMULT 24     // outside-set segment buffer: HULL_SBMULT * H*NP entries
#define HULL_HMAX 512      // horizon edges per insertion
#define HULL_VMAX 1024     // visible faces per insertion

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
  int* sb;                          // per block: HULL_SBMULT*H*NP ints (outside-set segments)
  int* rqueue;                      // pairs that overflowed the LDS variant
  int* rcount;
  int* rnext;
  void* bigmem;                     // per block of k_hull_big: one HullMemBig
  unsigned long long* stats;
  unsigned long long* prof;          // LQRO_HULL_PROFILE: per-phase cycles
};

// Hull topology and outside sets: in LDS for the common case, in global
// scratch (larger capacities) for the jobs that overflow it.
template <int FMAX, int VTX>
struct HullMem {
  static constexpr int kFaces = FMAX, kVerts = VTX;
  unsigned short fv[FMAX][3];        // vertex slots, outward counter-clockwise
  unsigned short fa[FMAX][3];        // fa[f][e]: face across edge (fv[e], fv[e+1])
  unsigned char alive[FMAX];
  unsigned char vis[FMAX];
  unsigned short freel[FMAX];
  int soff[FMAX], scnt[FMAX];        // outside set of face f: sb[soff .. soff+scnt)
  unsigned long long fbest[FMAX];    // furthest outside point: (dist bits << 32) | ~q
  double vx[VTX][3];                 // hull vertex coordinates (rounded points)
  int vpid[VTX];                     // vertex slot -> reachable-point index
};
typedef HullMem<3072, 1400> HullMemSmall;   // ~135 KB: LDS
typedef HullMem<16384, 8192> HullMemBig;    // ~750 KB: global scratch

// per-workgroup control state (always LDS)
struct HullLds {
  int hcnt[HULL_HMAX], hoff[HULL_HMAX];
  int vpre[HULL_VMAX + 1];
  unsigned short vlist[HULL_VMAX];
  unsigned short h_a[HULL_HMAX], h_b[HULL_HMAX], h_out[HULL_HMAX], h_new[HULL_HMAX];
  double tr[3 * 128];
  double rk[HULL_THREADS / 64];
  int ri[HULL_THREADS / 64];
  int scan[HULL_THREADS];
  int nf, nfree, nvtx, nvis, nh, fail, n, job, init[4], sbtop, fstar;
  unsigned long long kstar;
  double eps;
};

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
// is p beyond face f?  *dist = signed distance
template <class Mem>
__device__ __forceinline__ bool hl_beyond(const Mem& L, int f, const double* p, double eps,
                                          double* dist) {
  double n[3];
  hl_normal(L, f, n);
  const double* a = L.vx[L.fv[f][0]];
  const double d = n[0] * (p[0] - a[0]) + n[1] * (p[1] - a[1]) + n[2] * (p[2] - a[2]);
  const double nl = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  if (dist) *dist = d / nl;
  return d > eps * nl;
}

// block-wide argmax of (key, idx), lowest idx on ties; result in every thread
__device__ __forceinline__ void hl_argmax(HullLds& L, double& key, int& idx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ok = __shfl_xor(key, off);
    const int oi = __shfl_xor(idx, off);
    if (ok > key || (ok == key && oi < idx)) { key = ok; idx = oi; }
  }
  if (lane == 0) { L.rk[wave] = key; L.ri[wave] = idx; }
  __syncthreads();
  key = L.rk[0]; idx = L.ri[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
    if (L.rk[w] > key || (L.rk[w] == key && L.ri[w] < idx)) { key = L.rk[w]; idx = L.ri[w]; }
  __syncthreads();
}

// exclusive block scan of v (0/1); total in *tot
__device__ __forceinline__ int hl_scan(HullLds& L, int v, int* tot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long b = __ballot(v != 0);
  const int in_wave = __popcll(b & ((1ull << lane) - 1ull));
  if (lane == 0) L.scan[wave] = __popcll(b);
  __syncthreads();
  int base = 0, t = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
    if (w < wave) base += L.scan[w];
    t += L.scan[w];
  }
  *tot = t;
  __syncthreads();
  return base + in_wave;
}

#ifdef LQRO_HULL_PROFILE
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
#endif

template <class Mem>
__device__ __forceinline__ void hull_body(const HullArgs& A, Mem& M, HullLds& L, bool big) {
  const int tid = threadIdx.x;
#ifdef LQRO_HULL_PROFILE
  unsigned long long prof_acc[16] = {0};
  unsigned long long prof_last = __builtin_amdgcn_s_memtime();
#endif
  const int HNP = A.H * A.NP;
  double* Pr = A.scratch + (size_t)blockIdx.x * HNP * 6;    // rounded points
  double* Pf = Pr + (size_t)HNP * 3;                         // full-precision points
  int* tq = A.iscratch + (size_t)blockIdx.x * HNP * 2;      // moved point ids
  int* th = tq + HNP;                                        // their target cone face
  float* td = A.fscratch + (size_t)blockIdx.x * HNP;         // distance beyond it
  int* sb = A.sb + (size_t)blockIdx.x * HNP * HULL_SBMULT;
  const int sbcap = HNP * HULL_SBMULT;

  const int* queue = big ? A.rqueue : A.queue;
  const int* qcount = big ? A.rcount : A.count;
  int* qnext = big ? A.rnext : A.next;
  for (;;) {
    if (tid == 0) L.job = atomicAdd(qnext, 1);
    __syncthreads();
    const int job = L.job;
    if (job >= min(*qcount, A.cap)) break;
    const int slot = queue[job];
    const int lrow = slot / A.npr, jj = slot % A.npr;
    const int i = A.row_begin + lrow;
    const int j = jj < i ? jj : jj + 1;
    const double* xi = A.x + (size_t)i * A.X;
    const double* xj = A.x + (size_t)j * A.X;
    const double* Ti = A.T + (A.per_agent ? (size_t)i * A.H * 9 : 0);
    const double* Ni = A.NCF + (A.per_agent ? (size_t)i * A.H * 3 * A.X : 0);
    const double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};

    HSTAMP(15);
    // 1. reachable points in reference order, full + %g-rounded
    if (tid == 0) { L.n = 0; L.fail = 0; }
    __syncthreads();
    for (int k0 = 0; k0 < A.H; k0 += 128) {
      for (int it = tid; it < 3 * 128; it += blockDim.x) {
        const int k = k0 + it / 3, r = it % 3;
        if (k < A.H) {
          double d = 0.0;
          for (int c = 0; c < A.X; ++c) d += Ni[((size_t)k * 3 + r) * A.X + c] * (xi[c] - xj[c]);
          L.tr[it] = d;
        }
      }
      __syncthreads();
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
        __syncthreads();
        if (tid == 0) L.n += tot;
        __syncthreads();
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
      __syncthreads();
    }
    const double eps = L.eps;

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
      __syncthreads();
      key = -INFINITY; idx = INT_MAX;
      for (int q = tid; q < n; q += blockDim.x) {
        double dd;
        hl_beyond(M, 0, Pr + 3 * q, eps, &dd);
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
            M.vpid[v] = L.init[v];
            for (int d = 0; d < 3; ++d) M.vx[v][d] = Pr[3 * L.init[v] + d];
          }
          L.nvtx = 4;
          const int fvv[4][3] = {{0, 1, 2}, {0, 3, 1}, {1, 3, 2}, {0, 2, 3}};
          for (int f = 0; f < 4; ++f) {
            for (int e = 0; e < 3; ++e) M.fv[f][e] = (unsigned short)fvv[f][e];
            const int other = 6 - fvv[f][0] - fvv[f][1] - fvv[f][2];
            double dd;
            hl_beyond(M, f, M.vx[other], -INFINITY, &dd);
            if (dd > 0) { const unsigned short t = M.fv[f][1]; M.fv[f][1] = M.fv[f][2]; M.fv[f][2] = t; }
            M.alive[f] = 1;
            M.vis[f] = 0;
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
      __syncthreads();
    }

    if (!L.fail) {
      // 4. outside sets of the tetrahedron's faces
      if (tid < 4) { M.scnt[tid] = 0; M.fbest[tid] = 0ull; }
      if (tid == 0) L.sbtop = 0;
      __syncthreads();
      for (int q = tid; q < n; q += blockDim.x) {
        int c = -1;
        double dd = 0.0;
        if (q != L.init[0] && q != L.init[1] && q != L.init[2] && q != L.init[3]) {
          const double p[3] = {Pr[3 * q], Pr[3 * q + 1], Pr[3 * q + 2]};
          for (int f = 0; f < 4; ++f)
            if (hl_beyond(M, f, p, eps, &dd)) { c = f; break; }
        }
        th[q] = c;
        td[q] = (float)dd;
        if (c >= 0) atomicAdd(&M.scnt[c], 1);
      }
      __syncthreads();
      if (tid == 0) {
        int o = 0;
        for (int f = 0; f < 4; ++f) { M.soff[f] = o; L.hcnt[f] = 0; o += M.scnt[f]; }
        L.sbtop = o;
      }
      __syncthreads();
      for (int q = tid; q < n; q += blockDim.x) {
        const int c = th[q];
        if (c < 0) continue;
        sb[M.soff[c] + atomicAdd(&L.hcnt[c], 1)] = q;
        const unsigned long long key =
            ((unsigned long long)__float_as_uint(td[q]) << 32) | (unsigned long long)(~(unsigned)q);
        atomicMax(&M.fbest[c], key);
      }
      __syncthreads();

      HSTAMP(1);
      // 5. quickhull insertions
      for (;;) {
        // (0) the face whose outside set holds the furthest point, and that point
        if (tid == 0) { L.kstar = 0ull; L.fstar = -1; }
        __syncthreads();
        {
          unsigned long long kb = 0ull;
          for (int f = tid; f < L.nf; f += blockDim.x)
            if (M.alive[f] && M.scnt[f] > 0 && M.fbest[f] > kb) kb = M.fbest[f];
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) {
            const unsigned long long o = __shfl_xor(kb, off);
            kb = o > kb ? o : kb;
          }
          if ((tid & 63) == 0 && kb) atomicMax(&L.kstar, kb);
        }
        __syncthreads();
        if (L.kstar == 0ull) break;
        const int apex = (int)(~(unsigned)(L.kstar & 0xFFFFFFFFull));
        if (tid == 0) {
          if (L.nvtx < Mem::kVerts) {
            const int v = L.nvtx++;
            M.vpid[v] = apex;
            M.vx[v][0] = Pr[3 * apex]; M.vx[v][1] = Pr[3 * apex + 1]; M.vx[v][2] = Pr[3 * apex + 2];
          } else {
            L.fail = 1;
          }
          L.nvis = 0;
          L.nh = 0;
        }
        __syncthreads();
        if (L.fail) break;
        const int av = L.nvtx - 1;                   // the apex's vertex slot
        HSTAMP(2);
        // (a) visible faces: every live face the apex is beyond
        for (int f = tid; f < L.nf; f += blockDim.x) {
          if (!M.alive[f]) continue;
          if (hl_beyond(M, f, M.vx[av], eps, nullptr)) {
            M.vis[f] = 1;
            const int t = atomicAdd(&L.nvis, 1);
            if (t < HULL_VMAX) L.vlist[t] = (unsigned short)f;
            else L.fail = 2;
          }
        }
        __syncthreads();
        if (L.fail || L.nvis == 0) { if (tid == 0 && !L.fail) L.fail = 9; break; }
        const int nvis = L.nvis;
        HSTAMP(3);
        // (b) horizon: edges of visible faces whose neighbour is not visible
        for (int t = tid; t < nvis; t += blockDim.x) {
          const int fh = L.vlist[t];
          for (int e = 0; e < 3; ++e) {
            const int nb = M.fa[fh][e];
            if (!M.vis[nb]) {
              const int h = atomicAdd(&L.nh, 1);
              if (h < HULL_HMAX) {
                L.h_a[h] = M.fv[fh][e];
                L.h_b[h] = M.fv[fh][(e + 1) % 3];
                L.h_out[h] = (unsigned short)nb;
              } else {
                L.fail = 3;
              }
            }
          }
        }
        __syncthreads();
        if (L.fail) break;
        const int nh = L.nh;
        // (c) slots for the cone (faces retired in earlier rounds first);
        //     prefix of the retired faces' outside-set sizes
        for (int h = tid; h < nh; h += blockDim.x) {
          int sf;
          if (h < L.nfree) sf = M.freel[L.nfree - 1 - h];
          else sf = L.nf + (h - L.nfree);
          if (sf >= Mem::kFaces) { L.fail = 4; sf = 0; }
          L.h_new[h] = (unsigned short)sf;
          L.hcnt[h] = 0;
        }
        if (tid == 0) {
          int o = 0;
          for (int t = 0; t < nvis; ++t) { L.vpre[t] = o; o += M.scnt[L.vlist[t]]; }
          L.vpre[nvis] = o;
        }
        __syncthreads();
        if (L.fail) break;
        HSTAMP(4);
        // (d) cone faces (a, b, apex); patch the outer neighbours
        for (int h = tid; h < nh; h += blockDim.x) {
          const int sf = L.h_new[h];
          M.fv[sf][0] = L.h_a[h];
          M.fv[sf][1] = L.h_b[h];
          M.fv[sf][2] = (unsigned short)av;
          M.fa[sf][0] = L.h_out[h];
          int n1 = -1, n2 = -1;
          for (int g = 0; g < nh; ++g) {
            if (L.h_a[g] == L.h_b[h]) n1 = L.h_new[g];   // edge (b, apex)
            if (L.h_b[g] == L.h_a[h]) n2 = L.h_new[g];   // edge (apex, a)
          }
          if (n1 < 0 || n2 < 0) L.fail = 5;
          M.fa[sf][1] = (unsigned short)(n1 < 0 ? 0 : n1);
          M.fa[sf][2] = (unsigned short)(n2 < 0 ? 0 : n2);
          M.vis[sf] = 0;
          M.scnt[sf] = 0;
          M.fbest[sf] = 0ull;
          const int on = L.h_out[h];
          for (int e = 0; e < 3; ++e)
            if (M.fv[on][e] == L.h_b[h] && M.fv[on][(e + 1) % 3] == L.h_a[h]) M.fa[on][e] = (unsigned short)sf;
        }
        __syncthreads();
        if (L.fail) break;
        HSTAMP(5);
        // (e) the retired faces' outside points: which cone face (if any) now
        const int total = L.vpre[nvis];
        for (int t = tid; t < total; t += blockDim.x) {
          int lo = 0, hi = nvis - 1;                 // face owning item t
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (L.vpre[mid] <= t) lo = mid; else hi = mid - 1;
          }
          const int fo = L.vlist[lo];
          const int q = sb[M.soff[fo] + (t - L.vpre[lo])];
          int tgt = -1;
          double dd = 0.0;
          if (q != apex) {
            const double p[3] = {Pr[3 * q], Pr[3 * q + 1], Pr[3 * q + 2]};
            for (int h = 0; h < nh; ++h)
              if (hl_beyond(M, L.h_new[h], p, eps, &dd)) { tgt = h; break; }
          }
          tq[t] = q;
          th[t] = tgt;
          td[t] = (float)dd;
          if (tgt >= 0) atomicAdd(&L.hcnt[tgt], 1);
        }
        __syncthreads();
        if (tid == 0) {
          int o = L.sbtop;
          for (int h = 0; h < nh; ++h) {
            L.hoff[h] = o;
            M.soff[L.h_new[h]] = o;
            M.scnt[L.h_new[h]] = L.hcnt[h];
            o += L.hcnt[h];
            L.hcnt[h] = 0;
          }
          if (o > sbcap) L.fail = 6;
          L.sbtop = o;
        }
        __syncthreads();
        if (L.fail) break;
        for (int t = tid; t < total; t += blockDim.x) {
          const int h = th[t];
          if (h < 0) continue;
          const int q = tq[t];
          sb[L.hoff[h] + atomicAdd(&L.hcnt[h], 1)] = q;
          const unsigned long long key =
              ((unsigned long long)__float_as_uint(td[t]) << 32) | (unsigned long long)(~(unsigned)q);
          atomicMax(&M.fbest[L.h_new[h]], key);
        }
        HSTAMP(6);
        // (f) retire the visible faces, commit the cone
        for (int t = tid; t < nvis; t += blockDim.x) {
          const int f = L.vlist[t];
          M.alive[f] = 0;
          M.vis[f] = 0;
          M.freel[L.nfree + t] = (unsigned short)f;
        }
        __syncthreads();
        for (int h = tid; h < nh; h += blockDim.x) M.alive[L.h_new[h]] = 1;
        if (tid == 0) {
          // cone slots came off the top of the free list: move the retired
          // faces (just pushed above it) down over them
          const int used_free = min(nh, L.nfree);
          if (used_free > 0)
            for (int t = 0; t < nvis; ++t) M.freel[L.nfree - used_free + t] = M.freel[L.nfree + t];
          L.nfree += nvis - used_free;
          if (nh > used_free) L.nf += nh - used_free;
        }
        __syncthreads();
        HSTAMP(7);
#ifdef LQRO_HULL_PROFILE
        if (tid == 0) prof_acc[14] += 1;
#endif
      }
    }
    __syncthreads();

    HSTAMP(8);
    // 6. the reference's facet selection over all facets (canonical order)
    double best = INFINITY;
    int bt0 = INT_MAX, bt1 = INT_MAX, bt2 = INT_MAX, nfac = 0;
    double bn[3] = {0, 0, 0};
    if (!L.fail) {
      for (int f = tid; f < L.nf; f += blockDim.x) {
        if (!M.alive[f]) continue;
        nfac++;
        int t0 = M.vpid[M.fv[f][0]], t1 = M.vpid[M.fv[f][1]], t2 = M.vpid[M.fv[f][2]];
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
      __syncthreads();
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
      __syncthreads();
    }
    HSTAMP(9);
  }
#ifdef LQRO_HULL_PROFILE
  if (tid == 0 && A.prof)
    for (int k = 0; k < 16; ++k) atomicAdd(&A.prof[k], prof_acc[k]);
#endif
}

__global__ void __launch_bounds__(HULL_THREADS) k_hull(HullArgs A) {
  __shared__ HullLds L;
  __shared__ HullMemSmall M;
  hull_body(A, M, L, false);
}

__global__ void __launch_bounds__(HULL_THREADS) k_hull_big(HullArgs A) {
  __shared__ HullLds L;
  HullMemBig& M = reinterpret_cast<HullMemBig*>(A.bigmem)[blockIdx.x];
  hull_body(A, M, L, true);
}

}  // namespace lqro
