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
#include "lqro_pair.hpp"

using namespace lqro;

#define LQRO_MAXX 16
#define HULL_THREADS 256
#define HULL_FMAX 8192               // face slots per hull workgroup (global scratch)
#define HULL_VMAX 2048               // visible faces per insertion
#define HULL_HMAX 256                // horizon edges per insertion

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
// Hull kernel: one workgroup per inside-hull pair (persistent over the queue)
// ---------------------------------------------------------------------------
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
  int* iscratch;                    // per block: H*NP ints (conflict face)
  float* fscratch;                  // per block: H*NP floats (conflict distance)
  void* faces;                      // per block: HULL_FMAX HFace + HULL_FMAX free-list ints
  unsigned long long* stats;
};

struct HFace {
  int v[3];
  int adj[3];    // adj[e] = face across edge (v[e], v[e+1])
  double n[3];
  int alive;
};

__device__ __forceinline__ double hface_dist(const HFace& f, const double* P, int p) {
  const double* a = P + 3 * f.v[0];
  const double* q = P + 3 * p;
  return f.n[0] * (q[0] - a[0]) + f.n[1] * (q[1] - a[1]) + f.n[2] * (q[2] - a[2]);
}
__device__ __forceinline__ void hface_plane(HFace& f, const double* P) {
  const double *a = P + 3 * f.v[0], *b = P + 3 * f.v[1], *c = P + 3 * f.v[2];
  double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  double e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  f.n[0] = e1[1] * e2[2] - e1[2] * e2[1];
  f.n[1] = e1[2] * e2[0] - e1[0] * e2[2];
  f.n[2] = e1[0] * e2[1] - e1[1] * e2[0];
}

// block-wide argmax of (key, idx) with lowest idx on ties
__device__ void block_argmax(double& key, int& idx, double* sk, int* si) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    double ok = __shfl_xor(key, off);
    int oi = __shfl_xor(idx, off);
    if (ok > key || (ok == key && oi < idx)) { key = ok; idx = oi; }
  }
  if (lane == 0) { sk[wave] = key; si[wave] = idx; }
  __syncthreads();
  key = sk[0]; idx = si[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
    if (sk[w] > key || (sk[w] == key && si[w] < idx)) { key = sk[w]; idx = si[w]; }
  __syncthreads();
}

__global__ void __launch_bounds__(HULL_THREADS) k_hull(HullArgs A) {
  __shared__ unsigned char vis[HULL_FMAX];
  __shared__ int s_job, s_n, s_nf, s_fail, s_apex, s_nvis, s_nh, s_nnew;
  __shared__ int s_nfree;
  __shared__ int s_vis[HULL_VMAX];
  __shared__ int h_a[HULL_HMAX], h_b[HULL_HMAX], h_out[HULL_HMAX], h_new[HULL_HMAX];
  __shared__ double sk[HULL_THREADS / 64];
  __shared__ int si[HULL_THREADS / 64];
  __shared__ int s_scan[HULL_THREADS];
  __shared__ double s_tr[3 * 256];
  __shared__ int s_init[4];
  __shared__ double s_eps;

  const int tid = threadIdx.x;
  const int HNP = A.H * A.NP;
  double* Pr = A.scratch + (size_t)blockIdx.x * HNP * 6;    // rounded points
  double* Pf = Pr + (size_t)HNP * 3;                         // full-precision points
  int* conf = A.iscratch + (size_t)blockIdx.x * HNP;
  float* cd = A.fscratch + (size_t)blockIdx.x * HNP;
  HFace* F = reinterpret_cast<HFace*>(A.faces) + (size_t)blockIdx.x * HULL_FMAX;
  int* s_free = reinterpret_cast<int*>(reinterpret_cast<HFace*>(A.faces) + (size_t)gridDim.x * HULL_FMAX) +
               (size_t)blockIdx.x * HULL_FMAX;

  for (;;) {
    if (tid == 0) s_job = atomicAdd(A.next, 1);
    __syncthreads();
    const int job = s_job;
    __syncthreads();
    if (job >= min(*A.count, A.cap)) break;
    const int slot = A.queue[job];
    const int lrow = slot / A.npr, jj = slot % A.npr;
    const int i = A.row_begin + lrow;
    const int j = jj < i ? jj : jj + 1;
    const double* xi = A.x + (size_t)i * A.X;
    const double* xj = A.x + (size_t)j * A.X;
    const double* Ti = A.T + (A.per_agent ? (size_t)i * A.H * 9 : 0);
    const double* Ni = A.NCF + (A.per_agent ? (size_t)i * A.H * 3 * A.X : 0);
    const double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};

    // 1. reachable points in reference order (compacted), full + %g-rounded
    if (tid == 0) { s_n = 0; s_fail = 0; }
    __syncthreads();
    for (int k0 = 0; k0 < A.H; k0 += 256) {
      for (int it = tid; it < 3 * 256; it += blockDim.x) {
        int k = k0 + it / 3, r = it % 3;
        if (k < A.H) {
          double d = 0.0;
          for (int c = 0; c < A.X; ++c) d += Ni[((size_t)k * 3 + r) * A.X + c] * (xi[c] - xj[c]);
          s_tr[it] = d;
        }
      }
      __syncthreads();
      const int kend = min(A.H, k0 + 256);
      for (int q0 = k0 * A.NP; q0 < kend * A.NP; q0 += blockDim.x) {
        const int q = q0 + tid;
        bool ok = false;
        double p0 = 0, p1 = 0, p2 = 0;
        if (q < kend * A.NP) {
          const int k = q / A.NP, p = q % A.NP;
          const double* Tk = Ti + (size_t)k * 9;
          const double* tk = s_tr + (k - k0) * 3;
          double u0 = A.S[3 * p] + tk[0], u1 = A.S[3 * p + 1] + tk[1], u2 = A.S[3 * p + 2] + tk[2];
          p0 = ((0.0 + Tk[0] * u0) + Tk[1] * u1) + Tk[2] * u2;
          p1 = ((0.0 + Tk[3] * u0) + Tk[4] * u1) + Tk[5] * u2;
          p2 = ((0.0 + Tk[6] * u0) + Tk[7] * u1) + Tk[8] * u2;
          double a = p0 - vrel[0], b = p1 - vrel[1], c = p2 - vrel[2];
          double t = a * a + b * b + c * c;
          if (t < A.r2_lo) ok = true;
          else if (t > A.r2_hi) ok = false;
          else ok = (a * a) / A.r2 + (b * b) / A.r2 + (c * c) / A.r2 < 1.0;
        }
        // block exclusive scan of ok
        s_scan[tid] = ok ? 1 : 0;
        __syncthreads();
        for (int off = 1; off < (int)blockDim.x; off <<= 1) {
          int v = tid >= off ? s_scan[tid - off] : 0;
          __syncthreads();
          s_scan[tid] += v;
          __syncthreads();
        }
        const int base = s_n;
        const int pos = base + s_scan[tid] - (ok ? 1 : 0);
        if (ok) {
          int oor = 0;
          Pf[3 * pos] = p0; Pf[3 * pos + 1] = p1; Pf[3 * pos + 2] = p2;
          Pr[3 * pos] = round6(p0, &oor);
          Pr[3 * pos + 1] = round6(p1, &oor);
          Pr[3 * pos + 2] = round6(p2, &oor);
          if (oor) s_fail = 1;
        }
        __syncthreads();
        if (tid == blockDim.x - 1) s_n = base + s_scan[tid];
        __syncthreads();
      }
    }
    const int n = s_n;

    // 2. scale-aware coplanarity tolerance (as the oracle's hull)
    {
      double mx = 0.0;
      for (int q = tid; q < 3 * n; q += blockDim.x) mx = fmax(mx, fabs(Pr[q]));
      int dummy = tid;
      block_argmax(mx, dummy, sk, si);
      if (tid == 0) s_eps = 1e-13 * (mx + 1.0);
      __syncthreads();
    }
    const double eps = s_eps;

    // 3. initial tetrahedron (extreme points)
    if (n < 4) { if (tid == 0) s_fail = 1; }
    __syncthreads();
    if (!s_fail) {
      double key; int idx;
      // i0: min x
      key = -INFINITY; idx = INT_MAX;
      for (int q = tid; q < n; q += blockDim.x) {
        double v = -Pr[3 * q];
        if (v > key || (v == key && q < idx)) { key = v; idx = q; }
      }
      block_argmax(key, idx, sk, si);
      const int i0 = idx;
      key = -INFINITY; idx = INT_MAX;
      for (int q = tid; q < n; q += blockDim.x) {
        double dx = Pr[3 * q] - Pr[3 * i0], dy = Pr[3 * q + 1] - Pr[3 * i0 + 1], dz = Pr[3 * q + 2] - Pr[3 * i0 + 2];
        double v = dx * dx + dy * dy + dz * dz;
        if (v > key || (v == key && q < idx)) { key = v; idx = q; }
      }
      block_argmax(key, idx, sk, si);
      const int i1 = idx;
      key = -INFINITY; idx = INT_MAX;
      for (int q = tid; q < n; q += blockDim.x) {
        double e1[3] = {Pr[3 * i1] - Pr[3 * i0], Pr[3 * i1 + 1] - Pr[3 * i0 + 1], Pr[3 * i1 + 2] - Pr[3 * i0 + 2]};
        double e2[3] = {Pr[3 * q] - Pr[3 * i0], Pr[3 * q + 1] - Pr[3 * i0 + 1], Pr[3 * q + 2] - Pr[3 * i0 + 2]};
        double cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2], cz = e1[0] * e2[1] - e1[1] * e2[0];
        double v = cx * cx + cy * cy + cz * cz;
        if (v > key || (v == key && q < idx)) { key = v; idx = q; }
      }
      block_argmax(key, idx, sk, si);
      const int i2 = idx;
      HFace tf;
      tf.v[0] = i0; tf.v[1] = i1; tf.v[2] = i2;
      hface_plane(tf, Pr);
      const double nn = sqrt(tf.n[0] * tf.n[0] + tf.n[1] * tf.n[1] + tf.n[2] * tf.n[2]);
      key = -INFINITY; idx = INT_MAX;
      for (int q = tid; q < n; q += blockDim.x) {
        double v = fabs(hface_dist(tf, Pr, q)) / nn;
        if (v > key || (v == key && q < idx)) { key = v; idx = q; }
      }
      block_argmax(key, idx, sk, si);
      const int i3 = idx;
      if (tid == 0) {
        if (!(key > eps) || i0 == i1 || i1 == i2 || i2 == i3) s_fail = 1;
        s_init[0] = i0; s_init[1] = i1; s_init[2] = i2; s_init[3] = i3;
      }
      __syncthreads();
    }
    if (!s_fail && tid == 0) {
      const int tet[4] = {s_init[0], s_init[1], s_init[2], s_init[3]};
      const int fv[4][3] = {{0, 1, 2}, {0, 3, 1}, {1, 3, 2}, {0, 2, 3}};
      for (int f = 0; f < 4; ++f) {
        HFace h;
        h.v[0] = tet[fv[f][0]]; h.v[1] = tet[fv[f][1]]; h.v[2] = tet[fv[f][2]];
        hface_plane(h, Pr);
        const int other = tet[6 - fv[f][0] - fv[f][1] - fv[f][2]];
        if (hface_dist(h, Pr, other) > 0) {
          int t = h.v[1]; h.v[1] = h.v[2]; h.v[2] = t;
          hface_plane(h, Pr);
        }
        h.alive = 1;
        F[f] = h;
      }
      // adjacency by matching reversed edges
      for (int f = 0; f < 4; ++f)
        for (int e = 0; e < 3; ++e) {
          int a = F[f].v[e], b = F[f].v[(e + 1) % 3];
          F[f].adj[e] = -1;
          for (int g = 0; g < 4; ++g)
            for (int e2 = 0; e2 < 3; ++e2)
              if (F[g].v[e2] == b && F[g].v[(e2 + 1) % 3] == a) F[f].adj[e] = g;
        }
      s_nf = 4;
      s_nfree = 0;
    }
    __syncthreads();
    if (!s_fail) {
      // 4. initial conflict assignment
      for (int q = tid; q < n; q += blockDim.x) {
        int c = -1; double dd = 0.0;
        if (q != s_init[0] && q != s_init[1] && q != s_init[2] && q != s_init[3]) {
          for (int f = 0; f < 4; ++f) {
            const double nl = sqrt(F[f].n[0] * F[f].n[0] + F[f].n[1] * F[f].n[1] + F[f].n[2] * F[f].n[2]);
            const double dist = hface_dist(F[f], Pr, q);
            if (dist > eps * nl) { c = f; dd = dist / nl; break; }
          }
        }
        conf[q] = c;
        cd[q] = (float)dd;
      }
      __syncthreads();
      // 5. quickhull iterations
      for (int iter = 0; iter < 100000; ++iter) {
        double key = -INFINITY; int idx = INT_MAX;
        for (int q = tid; q < n; q += blockDim.x) {
          if (conf[q] >= 0) {
            double v = (double)cd[q];
            if (v > key || (v == key && q < idx)) { key = v; idx = q; }
          }
        }
        block_argmax(key, idx, sk, si);
        if (idx == INT_MAX) break;
        const int apex = idx;
        // visible region: BFS from the apex's conflict face (thread 0)
        for (int f = tid; f < s_nf; f += blockDim.x) vis[f] = 0;
        __syncthreads();
        if (tid == 0) {
          s_apex = apex;
          int nv = 0, nh = 0;
          const int f0 = conf[apex];
          vis[f0] = 1; s_vis[nv++] = f0;
          for (int h = 0; h < nv; ++h) {
            const HFace& fh = F[s_vis[h]];
            for (int e = 0; e < 3; ++e) {
              const int nb = fh.adj[e];
              if (nb < 0) { s_fail = 1; continue; }
              if (vis[nb]) continue;
              const double nl = sqrt(F[nb].n[0] * F[nb].n[0] + F[nb].n[1] * F[nb].n[1] + F[nb].n[2] * F[nb].n[2]);
              if (hface_dist(F[nb], Pr, apex) > eps * nl) {
                vis[nb] = 1;
                if (nv < HULL_VMAX) s_vis[nv++] = nb; else s_fail = 1;
              }
            }
          }
          // horizon
          for (int h = 0; h < nv; ++h) {
            const HFace& fh = F[s_vis[h]];
            for (int e = 0; e < 3; ++e) {
              const int nb = fh.adj[e];
              if (nb >= 0 && !vis[nb]) {
                if (nh < HULL_HMAX) { h_a[nh] = fh.v[e]; h_b[nh] = fh.v[(e + 1) % 3]; h_out[nh] = nb; nh++; }
                else s_fail = 1;
              }
            }
          }
          // retire the visible faces, make the cone (a slot retired in this
          // round is reused only from the next round on, after the
          // reassignment below has seen it dead)
          for (int h = 0; h < nv; ++h) F[s_vis[h]].alive = 0;
          for (int h = 0; h < nh && !s_fail; ++h) {
            int slotf;
            if (s_nfree > 0) slotf = s_free[--s_nfree];
            else if (s_nf < HULL_FMAX) slotf = s_nf++;
            else { s_fail = 1; break; }
            h_new[h] = slotf;
            HFace nf;
            nf.v[0] = h_a[h]; nf.v[1] = h_b[h]; nf.v[2] = apex;
            nf.alive = 1;
            nf.adj[0] = h_out[h];
            nf.adj[1] = -1; nf.adj[2] = -1;
            hface_plane(nf, Pr);
            F[slotf] = nf;
            vis[slotf] = 0;
            // outer neighbour: its edge (b, a) now faces the new face
            HFace& on = F[h_out[h]];
            for (int e = 0; e < 3; ++e)
              if (on.v[e] == h_b[h] && on.v[(e + 1) % 3] == h_a[h]) on.adj[e] = slotf;
          }
          if (!s_fail)
            for (int h = 0; h < nh; ++h) {
              // edge (b, apex) <-> face whose horizon edge starts at b
              // edge (apex, a) <-> face whose horizon edge ends at a
              for (int g = 0; g < nh; ++g) {
                if (h_a[g] == h_b[h]) F[h_new[h]].adj[1] = h_new[g];
                if (h_b[g] == h_a[h]) F[h_new[h]].adj[2] = h_new[g];
              }
              if (F[h_new[h]].adj[1] < 0 || F[h_new[h]].adj[2] < 0) s_fail = 1;
            }
          for (int h = 0; h < nv; ++h) s_free[s_nfree++] = s_vis[h];
          s_nvis = nv;
          s_nh = nh;
        }
        __syncthreads();
        if (s_fail) break;
        // reassign the conflict points of the visible faces
        const int nh = s_nh;
        for (int q = tid; q < n; q += blockDim.x) {
          const int c = conf[q];
          if (c < 0) continue;
          if (q == apex) { conf[q] = -1; continue; }
          if (F[c].alive) continue;          // c was visible (freed) this round
          int nc = -1; double dd = 0.0;
          for (int h = 0; h < nh; ++h) {
            const HFace& f = F[h_new[h]];
            const double nl = sqrt(f.n[0] * f.n[0] + f.n[1] * f.n[1] + f.n[2] * f.n[2]);
            const double dist = hface_dist(f, Pr, q);
            if (dist > eps * nl) { nc = h_new[h]; dd = dist / nl; break; }
          }
          conf[q] = nc;
          cd[q] = (float)dd;
        }
        __syncthreads();
      }
    }
    __syncthreads();

    // 6. arg-min facet (LQRObstacles.cpp:955-968) in canonical facet order:
    //    normal from the rounded vertices (lowest index first), distance from
    //    the full-precision lowest-index vertex.
    double best = INFINITY;
    int bt0 = INT_MAX, bt1 = INT_MAX, bt2 = INT_MAX;
    double bn[3] = {0, 0, 0};
    int nfac = 0;
    if (!s_fail) {
      for (int f = tid; f < s_nf; f += blockDim.x) {
        if (!F[f].alive) continue;
        nfac++;
        int t0 = F[f].v[0], t1 = F[f].v[1], t2 = F[f].v[2];
        while (!(t0 < t1 && t0 < t2)) { int a = t0; t0 = t1; t1 = t2; t2 = a; }
        const double *a = Pr + 3 * t0, *b = Pr + 3 * t1, *c = Pr + 3 * t2;
        double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
        double e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
        double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        double len = sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
        nv[0] /= len; nv[1] /= len; nv[2] /= len;
        const double* p0 = Pf + 3 * t0;
        double dd = fabs(nv[0] * (vrel[0] - p0[0]) + nv[1] * (vrel[1] - p0[1]) + nv[2] * (vrel[2] - p0[2]));
        // canonical triple order key = sorted (t0, min(t1,t2), max(t1,t2))
        int s1 = min(t1, t2), s2 = max(t1, t2);
        bool better = dd < best || (dd == best && (t0 < bt0 || (t0 == bt0 && (s1 < bt1 || (s1 == bt1 && s2 < bt2)))));
        if (better) {
          best = dd; bt0 = t0; bt1 = s1; bt2 = s2;
          bn[0] = nv[0]; bn[1] = nv[1]; bn[2] = nv[2];
        }
      }
    }
    // block reduction of (best, triple)
    __shared__ double r_best[HULL_THREADS];
    __shared__ int r_t[HULL_THREADS][3];
    __shared__ double r_n[HULL_THREADS][3];
    __shared__ int r_cnt[HULL_THREADS];
    r_best[tid] = best; r_t[tid][0] = bt0; r_t[tid][1] = bt1; r_t[tid][2] = bt2;
    r_n[tid][0] = bn[0]; r_n[tid][1] = bn[1]; r_n[tid][2] = bn[2];
    r_cnt[tid] = nfac;
    __syncthreads();
    if (tid == 0) {
      int fo = 0, total = 0;
      for (int t = 0; t < (int)blockDim.x; ++t) {
        total += r_cnt[t];
        bool better = r_best[t] < r_best[fo] ||
                      (r_best[t] == r_best[fo] &&
                       (r_t[t][0] < r_t[fo][0] || (r_t[t][0] == r_t[fo][0] &&
                        (r_t[t][1] < r_t[fo][1] || (r_t[t][1] == r_t[fo][1] && r_t[t][2] < r_t[fo][2])))));
        if (better) fo = t;
      }
      const bool ok = !s_fail && total > 0 && r_t[fo][0] != INT_MAX;
      float* pl = A.planes + (size_t)slot * 8;
      double distance = r_best[fo];
      double nrm[3] = {r_n[fo][0], r_n[fo][1], r_n[fo][2]};
      if (ok) {
        double dh = distance * 0.5;                       // :1416
        const double mult = 1.0;                          // :1213
        pl[0] = (float)(xi[3] + mult * dh * nrm[0]);
        pl[1] = (float)(xi[4] + mult * dh * nrm[1]);
        pl[2] = (float)(xi[5] + mult * dh * nrm[2]);
        pl[3] = (float)nrm[0]; pl[4] = (float)nrm[1]; pl[5] = (float)nrm[2];
        pl[6] = __int_as_float(1);
        atomicAdd(&A.stats[3], 1ull);
      } else {
        pl[6] = __int_as_float(0);                        // no usable plane
        atomicAdd(&A.stats[4], 1ull);
      }
      if (A.recs) {
        lqro_pair_record& rec = A.recs[slot];
        rec.flags |= ok ? LQRO_REC_HULL : LQRO_REC_HULLFAIL;
        rec.n_facets = ok ? total : -1;
        if (ok) {
          rec.facet[0] = r_t[fo][0]; rec.facet[1] = r_t[fo][1]; rec.facet[2] = r_t[fo][2];
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
}

// ---------------------------------------------------------------------------
// LP kernel: one wavefront per row agent (lqro_lp.hpp), fp32 as the reference
// ---------------------------------------------------------------------------
struct LpArgs {
  int npr, nrows, row_begin;
  double vmax;
  const float* slots;   // per row npr x 8 (flag in [6]: 1 = plane)
  float* compact;       // per row npr x 8: emitted planes in j order
  float* proj;          // per row npr x 8: linearProgram4's projected planes
  const double* vgoal;
  double* newv;
};

__global__ void __launch_bounds__(256) k_lp(LpArgs A) {
  const int lane = threadIdx.x & 63;
  const int lrow = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (lrow >= A.nrows) return;
  const int i = A.row_begin + lrow;
  const float* src = A.slots + (size_t)lrow * A.npr * 8;
  float* planes = A.compact + (size_t)lrow * A.npr * 8;
  // orcaPlanes_ in push order (j order, LQRObstacles.cpp:1220)
  int m = 0;
  for (int base = 0; base < A.npr; base += 64) {
    const int sidx = base + lane;
    float4 a = make_float4(0, 0, 0, 0), b = make_float4(0, 0, 0, 0);
    bool f = false;
    if (sidx < A.npr) {
      const float4* p = reinterpret_cast<const float4*>(src + 8 * (size_t)sidx);
      a = p[0];
      b = p[1];
      f = __float_as_int(b.z) == 1;
    }
    const unsigned long long bal = __ballot(f);
    if (f) {
      float4* d = reinterpret_cast<float4*>(planes + 8 * (size_t)(m + __popcll(bal & ((1ull << lane) - 1ull))));
      d[0] = a;
      d[1] = b;
    }
    m += __popcll(bal);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const v3 pref = V3((float)A.vgoal[3 * i], (float)A.vgoal[3 * i + 1], (float)A.vgoal[3 * i + 2]);
  v3 nv = V3(0.0f, 0.0f, 0.0f);
  const int fail = w_lp3(planes, m, A.vmax, pref, false, nv, lane);          // :1228
  if (fail < m)
    w_lp4(planes, m, fail, (float)A.vmax, nv, A.proj + (size_t)lrow * A.npr * 8, lane);  // :1230
  if (lane == 0) {
    A.newv[3 * i] = nv.x;
    A.newv[3 * i + 1] = nv.y;
    A.newv[3 * i + 2] = nv.z;
  }
}

// ---------------------------------------------------------------------------
// Host side: context + C-ABI
// ---------------------------------------------------------------------------
struct lqro_ctx {
  lqro_config cfg;
  double *d_R, *d_TF, umax;
  unsigned long long* d_shash;
  int rb, re, nrows, npr;
  int have_gains, per_agent;
  hipStream_t stream;
  hipEvent_t ev[5];
  double *d_T, *d_NCF, *d_S, *d_x, *d_vgoal, *d_newv;
  double *d_A, *d_B, *d_L, *d_E;
  float *d_planes, *d_lpscratch, *d_lpcompact;
  lqro_pair_record* d_recs;
  int *d_hq, *d_hcount, *d_hnext, *d_err;
  double* d_hscratch;
  int* d_hiscratch;
  float* d_hfscratch;
  void* d_hfaces;
  int hull_blocks, hull_cap;
  unsigned long long* d_stats;
  int lds_bytes;
  PairArgs pa;
};

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
  c->device = 0;
  c->flags = 0;
}

void lqro_destroy(lqro_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->cfg.device);
  void* ps[] = {c->d_R, c->d_TF, c->d_shash, c->d_T, c->d_NCF, c->d_S, c->d_x, c->d_vgoal, c->d_newv, c->d_A, c->d_B,
                c->d_L, c->d_E, c->d_planes, c->d_lpscratch, c->d_lpcompact, c->d_recs, c->d_hq, c->d_hcount,
                c->d_err, c->d_hfaces, /* d_hnext points into d_hcount */ c->d_hscratch, c->d_hiscratch, c->d_hfscratch, c->d_stats};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  for (int k = 0; k < 5; ++k)
    if (c->ev[k]) (void)hipEventDestroy(c->ev[k]);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

static int ctx_alloc(lqro_ctx* c) {
  const lqro_config& g = c->cfg;
  const size_t N = g.n_agents, X = g.x_dim, H = g.horizon, NP = g.n_points;
  const size_t slots = (size_t)c->nrows * c->npr;
  HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  for (int k = 0; k < 5; ++k) HIPCHK(hipEventCreate(&c->ev[k]));
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
  c->hull_cap = (int)(slots < (1u << 22) ? slots : (1u << 22));
  if (c->hull_cap < 1) c->hull_cap = 1;
  HIPCHK(hipMalloc(&c->d_hq, sizeof(int) * c->hull_cap));
  HIPCHK(hipMalloc(&c->d_hcount, sizeof(int) * 2));
  c->d_hnext = c->d_hcount + 1;
  HIPCHK(hipMalloc(&c->d_err, sizeof(int)));
  HIPCHK(hipMalloc(&c->d_stats, sizeof(unsigned long long) * 8));
  c->hull_blocks = 512;
  HIPCHK(hipMalloc(&c->d_hscratch, sizeof(double) * 6 * H * NP * c->hull_blocks));
  HIPCHK(hipMalloc(&c->d_hiscratch, sizeof(int) * H * NP * c->hull_blocks));
  HIPCHK(hipMalloc(&c->d_hfscratch, sizeof(float) * H * NP * c->hull_blocks));
  HIPCHK(hipMalloc(&c->d_hfaces, (sizeof(HFace) + sizeof(int)) * HULL_FMAX * (size_t)c->hull_blocks));
  return LQRO_OK;
}

int lqro_create(const lqro_config* cfg, lqro_ctx** out) {
  if (!cfg || !out) return LQRO_E_ARG;
  *out = nullptr;
  const lqro_config& g = *cfg;
  if (g.n_agents < 2 || (g.x_dim != 16 && g.x_dim != 12) || g.u_dim != 4 || g.horizon < 1 ||
      g.n_points < 1 || g.vmax_reach <= 0)
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
  c->rb = g.row_begin;
  c->re = (g.row_end > g.row_begin) ? g.row_end : g.n_agents;
  if (g.row_end == 0 && g.row_begin == 0) { c->rb = 0; c->re = g.n_agents; }
  if (c->rb < 0 || c->re > g.n_agents || c->rb >= c->re) { delete c; return LQRO_E_ARG; }
  c->nrows = c->re - c->rb;
  c->npr = g.n_agents - 1;
  // LDS layout of k_pair (in doubles): block tables, then one region per wave
  const int H = g.horizon, NP = g.n_points, X = g.x_dim, XP = X + 1;
  if (NP > 64 * kMaxPW) { delete c; return LQRO_E_ARG; }
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
  // tr 3H, c 3H, sc H, ub H, mask H*PW (u64), cls/cnt/mixed 3H ints
  P.wave_doubles = 8 * H + H * P.PW + (3 * H + 1) / 2;
  const int budget = 160 * 1024 / 8;
  int waves = (budget - off) / P.wave_doubles;
  if (waves > 16) waves = 16;
  if (waves < 1) {
    fprintf(stderr, "liblqro: horizon %d x %d points does not fit in LDS\n", H, NP);
    delete c;
    return LQRO_E_ARG;
  }
  P.waves = waves;
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
  if (hipFuncSetAttribute((const void*)k_pair<16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          c->lds_bytes) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_pair<12>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          c->lds_bytes) != hipSuccess) {
    lqro_destroy(c);
    return LQRO_E_HIP;
  }
  *out = c;
  return LQRO_OK;
}

int lqro_set_gains(lqro_ctx* c, const double* A, const double* B, const double* L,
                   const double* E, int32_t per_agent) {
  if (!c || !A || !B || !L || !E) return LQRO_E_ARG;
  const lqro_config& g = c->cfg;
  HIPCHK(hipSetDevice(g.device));
  const size_t X = g.x_dim, U = g.u_dim, N = g.n_agents;
  const size_t na = per_agent ? N : 1;
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

static int enqueue_step(lqro_ctx* c, const double* d_x, const double* d_vgoal, double* d_newv,
                        hipStream_t s) {
  const lqro_config& g = c->cfg;
  PairArgs P = c->pa;
  P.N = g.n_agents; P.H = g.horizon; P.NP = g.n_points; P.min_reach = g.min_reach;
  P.row_begin = c->rb; P.nrows = c->nrows; P.npr = c->npr;
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
  // one workgroup = P.waves wavefronts on one row; each wave takes several pairs
  P.pairs_per_block = P.waves * 4;
  P.blocks_per_row = (c->npr + P.pairs_per_block - 1) / P.pairs_per_block;
  HIPCHK(hipMemsetAsync(c->d_hcount, 0, sizeof(int) * 2, s));
  HIPCHK(hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * 8, s));
  HIPCHK(hipEventRecord(c->ev[0], s));
  const unsigned nblk = (unsigned)P.blocks_per_row * (unsigned)c->nrows;
  if (g.x_dim == 16)
    hipLaunchKernelGGL(k_pair<16>, dim3(nblk), dim3(P.waves * 64), c->lds_bytes, s, P);
  else if (g.x_dim == 12)
    hipLaunchKernelGGL(k_pair<12>, dim3(nblk), dim3(P.waves * 64), c->lds_bytes, s, P);
  else
    return LQRO_E_ARG;
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev[1], s));
  HullArgs Hh;
  Hh.N = g.n_agents; Hh.X = g.x_dim; Hh.H = g.horizon; Hh.NP = g.n_points;
  Hh.row_begin = c->rb; Hh.npr = c->npr; Hh.per_agent = c->per_agent;
  Hh.r2 = P.r2; Hh.r2_lo = P.r2_lo; Hh.r2_hi = P.r2_hi;
  Hh.T = c->d_T; Hh.NCF = c->d_NCF; Hh.S = c->d_S; Hh.x = d_x;
  Hh.planes = c->d_planes; Hh.recs = c->d_recs;
  Hh.queue = c->d_hq; Hh.count = c->d_hcount; Hh.cap = c->hull_cap; Hh.next = c->d_hnext;
  Hh.scratch = c->d_hscratch; Hh.iscratch = c->d_hiscratch; Hh.fscratch = c->d_hfscratch;
  Hh.faces = c->d_hfaces;
  Hh.stats = c->d_stats;
  hipLaunchKernelGGL(k_hull, dim3(c->hull_blocks), dim3(HULL_THREADS), 0, s, Hh);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev[2], s));
  LpArgs La;
  La.npr = c->npr; La.nrows = c->nrows; La.row_begin = c->rb; La.vmax = g.vmax_lp;
  La.slots = c->d_planes; La.compact = c->d_lpcompact; La.proj = c->d_lpscratch;
  La.vgoal = d_vgoal; La.newv = d_newv;
  hipLaunchKernelGGL(k_lp, dim3((unsigned)((c->nrows + 3) / 4)), dim3(256), 0, s, La);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev[3], s));
  return LQRO_OK;
}

int lqro_step_device(lqro_ctx* c, const double* d_x, const double* d_vgoal, double* d_newv,
                     void* stream) {
  if (!c || !d_x || !d_vgoal || !d_newv) return LQRO_E_ARG;
  if (!c->have_gains) return LQRO_E_STATE;
  HIPCHK(hipSetDevice(c->cfg.device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  return enqueue_step(c, d_x, d_vgoal, d_newv, s);
}

int lqro_step(lqro_ctx* c, const double* x, const double* vgoal, double* newv) {
  if (!c || !x || !vgoal || !newv) return LQRO_E_ARG;
  if (!c->have_gains) return LQRO_E_STATE;
  const lqro_config& g = c->cfg;
  HIPCHK(hipSetDevice(g.device));
  const size_t N = g.n_agents, X = g.x_dim;
  HIPCHK(hipMemcpyAsync(c->d_x, x, sizeof(double) * N * X, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_vgoal, vgoal, sizeof(double) * N * 3, hipMemcpyHostToDevice, c->stream));
  int rc = enqueue_step(c, c->d_x, c->d_vgoal, c->d_newv, c->stream);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(newv + (size_t)c->rb * 3, c->d_newv + (size_t)c->rb * 3,
                        sizeof(double) * 3 * c->nrows, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  int hc = 0;
  HIPCHK(hipMemcpy(&hc, c->d_hcount, sizeof(int), hipMemcpyDeviceToHost));
  if (hc > c->hull_cap) return LQRO_E_OVERFLOW;
  return LQRO_OK;
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
  int rc = LQRO_OK;
  if (hipMalloc(&d_slots, sizeof(float) * 8 * slots) != hipSuccess ||
      hipMalloc(&d_compact, sizeof(float) * 8 * slots) != hipSuccess ||
      hipMalloc(&d_proj, sizeof(float) * 8 * slots) != hipSuccess ||
      hipMalloc(&d_vg, sizeof(double) * 3 * n_agents) != hipSuccess ||
      hipMalloc(&d_nv, sizeof(double) * 3 * n_agents) != hipSuccess) {
    rc = LQRO_E_NOMEM;
  } else if (hipMemcpy(d_slots, h.data(), sizeof(float) * 8 * slots, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(d_vg, vgoal, sizeof(double) * 3 * n_agents, hipMemcpyHostToDevice) != hipSuccess) {
    rc = LQRO_E_HIP;
  } else {
    LpArgs La;
    La.npr = (int)mmax; La.nrows = n_agents; La.row_begin = 0; La.vmax = vmax_lp;
    La.slots = d_slots; La.compact = d_compact; La.proj = d_proj; La.vgoal = d_vg; La.newv = d_nv;
    hipLaunchKernelGGL(k_lp, dim3((unsigned)((n_agents + 3) / 4)), dim3(256), 0, 0, La);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(newv, d_nv, sizeof(double) * 3 * n_agents, hipMemcpyDeviceToHost) != hipSuccess)
      rc = LQRO_E_HIP;
  }
  void* ps[] = {d_slots, d_compact, d_proj, d_vg, d_nv};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  return rc;
}

int lqro_get_records(lqro_ctx* c, lqro_pair_record* out, int64_t cap, int64_t* n_out) {
  if (!c || !out) return LQRO_E_ARG;
  if (!c->d_recs) return LQRO_E_STATE;
  const int64_t n = (int64_t)c->nrows * c->npr;
  if (cap < n) return LQRO_E_ARG;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out, c->d_recs, sizeof(lqro_pair_record) * (size_t)n, hipMemcpyDeviceToHost));
  if (n_out) *n_out = n;
  return LQRO_OK;
}

int lqro_get_stats(lqro_ctx* c, int64_t* st) {
  if (!c || !st) return LQRO_E_ARG;
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(hipStreamSynchronize(c->stream));
  unsigned long long h[8];
  HIPCHK(hipMemcpy(h, c->d_stats, sizeof h, hipMemcpyDeviceToHost));
  for (int k = 0; k < 8; ++k) st[k] = (int64_t)h[k];
  st[0] = (int64_t)c->nrows * c->npr;
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
