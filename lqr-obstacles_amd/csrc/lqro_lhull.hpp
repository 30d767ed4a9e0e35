// lqro_lhull.hpp — the inside-hull branch from a LOCAL hull around vrel.
//
// convexHull (LQRObstacles.cpp:867-969) needs only the hull facets near
// vrel: the rule takes the facet minimising
//     | n_f . (vrel - P[t0(f)]) |
// n_f from the rounded points, P at full precision.  k_lhull (one 8-wave
// workgroup per inside-hull pair, persistent over the queue k_pair fills)
// grows a small hull Q of the pair's rounded points EPA-style instead of the
// whole hull (~800 vertices at C3):
//   1. the pair's points (hull_points) and the initial tetrahedron
//      (hull_tetra), as k_hull does;
//   2. until vrel is strictly inside Q, the facet vrel is on or beyond takes
//      its furthest point;
//   3. every Q-facet whose plane distance from vrel is within W = V* + delta
//      is CERTIFIED (a scan over all points finds none beyond it by the
//      hull's eps rule: it is a facet of the full hull) or takes its furthest
//      point; V* = the smallest rule value of a certified facet, delta
//      bounds | P - P_rounded | (rule value vs plane distance);
//   4. so is every Q-facet sharing a vertex with such a window facet.
// Why the window is then complete: D(u) = h(u) - u.vrel is
// positive and concave along great-circle arcs inside a vertex's normal cone,
// so any direction with D_Q(u) <= W lies in the normal cone of a vertex of a
// window facet; those vertices have only certified facets around them, so Q
// and the full hull share their normal cones there, and every full-hull facet
// with plane distance <= W — the only ones whose rule value can reach V* — is
// a certified facet of Q.  The selection (hull_select over the certified
// facets) is then the full hull's, bit for bit.
// The full hull (k_hull) decides instead whenever the argument's premises are
// not met by a margin: vrel on or outside a facet of the full hull (GJK's
// inside test has a tolerance), a point within 64 eps of a facet's plane or
// of a new vertex's horizon (64 eps: near-coplanar input, where the facet set
// depends on the hull's tie rules), capacity (LH_VMAX vertices, LH_FMAX
// faces), a degenerate point set.  Those pairs go to k_hull's queue.
#pragma once
#include "lqro_hull.hpp"

namespace lqro {

#define LH_THREADS 512
#define LH_DIRS 32                // initial support directions (Fibonacci sphere)
#define LH_VMAX 256
#define LH_FMAX 512
#define LH_EMAX 1536
#define LH_ITERS 2048
#define LH_BATCH 8                // faces scanned together
#define LH_LCAP 2560              // live points kept in LDS once compaction gets them this few

struct LHullL {
  // hull_points / hull_tetra / hl_argmax / hl_scan / hull_take_job
  double tr[3 * 128];
  double rk[LH_THREADS / 64];
  int ri[LH_THREADS / 64];
  int scan[LH_THREADS / 64];
  int n, fail, job, slot, init[4];
  double eps;
  // the local hull Q
  double vx[LH_VMAX][3];             // vertex coordinates (rounded points)
  int vpid[LH_VMAX];                 // vertex -> point id
  unsigned short fv[LH_FMAX][3];     // outward counter-clockwise
  unsigned short fa[LH_FMAX][3];     // written by hull_tetra, unused
  double fn[LH_FMAX][4];             // n = (b-a) x (c-a), n.n
  double sd[LH_FMAX];                // n.(vrel - a) / |n|  (< 0: vrel inside)
  unsigned char alive[LH_FMAX], cert[LH_FMAX];
  unsigned short freel[LH_FMAX];     // retired face slots (a stack)
  unsigned short ea[LH_EMAX], eb[LH_EMAX];   // edges of the visible region
  unsigned int vmark[LH_VMAX / 32];
  int nf, nfree, nv, ne, nh, task, tface, nb;
  int bf[LH_BATCH];                  // this iteration's faces
  double bkey[LH_BATCH];             // their furthest point: n.(p - a), id
  int bidx[LH_BATCH];
  unsigned short bt[LH_BATCH][3];    // their vertices (a slot may be reused by an insertion)
  double sk[LH_BATCH * (LH_THREADS / 64)];
  int si[LH_BATCH * (LH_THREADS / 64)];
  int nc, cb, ncompact, inlds, npk;       // live points, their global buffer, next compaction at nv, in lp
  double4 lp[LH_LCAP];               // the live points when nc <= LH_LCAP
  double4 pk[LH_FMAX];               // compaction: alive faces {n, n.a - band |n| / 2}
  double dir[LH_DIRS][3];
  int sup[LH_DIRS];
  double best, delta;
};

// face f's plane and vrel's signed distance from it (one thread)
__device__ __forceinline__ void lh_face(LHullL& L, int f, const double* vrel) {
  double n[3];
  hl_normal(L, f, n);
  const double* a = L.vx[L.fv[f][0]];
  const double nn = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
  L.fn[f][0] = n[0]; L.fn[f][1] = n[1]; L.fn[f][2] = n[2]; L.fn[f][3] = nn;
  L.sd[f] = (n[0] * (vrel[0] - a[0]) + n[1] * (vrel[1] - a[1]) + n[2] * (vrel[2] - a[2])) / sqrt(nn);
  L.alive[f] = 1;
  L.cert[f] = 0;
}

// the rule value of face f (hull_select's arithmetic: canonical rotation,
// normal from the rounded points, distance from the full-precision vertex)
__device__ __forceinline__ double lh_rule(const LHullL& L, int f, const double* Pr, const double* Pf,
                                          const double* vrel) {
  int t0 = L.vpid[L.fv[f][0]], t1 = L.vpid[L.fv[f][1]], t2 = L.vpid[L.fv[f][2]];
  while (!(t0 < t1 && t0 < t2)) { const int a = t0; t0 = t1; t1 = t2; t2 = a; }
  const double *a = Pr + 3 * t0, *b = Pr + 3 * t1, *c = Pr + 3 * t2;
  const double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  const double e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
  const double len = sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
  nv[0] /= len; nv[1] /= len; nv[2] /= len;
  const double* p0 = Pf + 3 * t0;
  return fabs(nv[0] * (vrel[0] - p0[0]) + nv[1] * (vrel[1] - p0[1]) + nv[2] * (vrel[2] - p0[2]));
}

__device__ __forceinline__ int lh_wmin(int v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = min(v, __shfl_xor(v, off));
  return v;
}

// wave 0: this iteration's faces (L.bf, L.nb).  task 1: vrel on or beyond
// them (within margin); 2: the LH_BATCH nearest uncertified window faces;
// 3: uncertified faces sharing a vertex with a window face; 0: done.
__device__ __forceinline__ void lh_choose(LHullL& L, int lane, double margin) {
  const int nf = L.nf;
  int nb = 0;
  for (int f0 = 0; f0 < nf && nb < LH_BATCH; f0 += 64) {
    const int f = f0 + lane;
    unsigned long long m = __ballot(f < nf && L.alive[f] && L.sd[f] >= -margin);
    while (m && nb < LH_BATCH) {
      if (lane == 0) L.bf[nb] = f0 + __builtin_ctzll(m);
      m &= m - 1;
      nb++;
    }
  }
  if (nb) {
    if (lane == 0) { L.task = 1; L.nb = nb; }
    return;
  }
  const double W = L.best + L.delta;
  unsigned taken = 0u;                     // bit k: face lane + 64 k chosen
  for (int r = 0; r < LH_BATCH; ++r) {
    double kb = INFINITY;
    int fb = INT_MAX;
    for (int k = 0; lane + 64 * k < nf; ++k) {
      const int f = lane + 64 * k;
      const double v = -L.sd[f];
      if (!((taken >> k) & 1u) && L.alive[f] && !L.cert[f] && v <= W && (v < kb || (v == kb && f < fb))) {
        kb = v; fb = f;
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double ok = __shfl_xor(kb, off);
      const int of = __shfl_xor(fb, off);
      if (ok < kb || (ok == kb && of < fb)) { kb = ok; fb = of; }
    }
    if (fb == INT_MAX) break;
    if ((fb & 63) == lane) taken |= 1u << (fb >> 6);
    if (lane == 0) L.bf[nb] = fb;
    nb++;
  }
  if (nb) {
    if (lane == 0) { L.task = 2; L.nb = nb; }
    return;
  }
  for (int w = lane; w < LH_VMAX / 32; w += 64) L.vmark[w] = 0u;
  hl_sync();
  for (int f = lane; f < nf; f += 64)
    if (L.alive[f] && -L.sd[f] <= W)
      for (int k = 0; k < 3; ++k) atomicOr(&L.vmark[L.fv[f][k] >> 5], 1u << (L.fv[f][k] & 31));
  hl_sync();
  for (int f0 = 0; f0 < nf && nb < LH_BATCH; f0 += 64) {
    const int f = f0 + lane;
    bool touch = false;
    if (f < nf && L.alive[f] && !L.cert[f])
      for (int k = 0; k < 3; ++k) touch |= ((L.vmark[L.fv[f][k] >> 5] >> (L.fv[f][k] & 31)) & 1u) != 0;
    unsigned long long m = __ballot(touch);
    while (m && nb < LH_BATCH) {
      if (lane == 0) L.bf[nb] = f0 + __builtin_ctzll(m);
      m &= m - 1;
      nb++;
    }
  }
  if (lane == 0) { L.task = nb ? 3 : 0; L.nb = nb; }
}

// insert point q into Q: the faces it is beyond go, a cone joins the
// horizon to the new vertex (nothing visible: q is inside Q, no change).
// Workgroup-wide; slots are assigned by workgroup scans in face / edge order,
// so Q's evolution (and which pairs are handed over) is deterministic.
__device__ __forceinline__ void lh_insert(LHullL& L, const double* Pr, int q, double eps2, double band2,
                                          const double* vrel) {
  const int tid = threadIdx.x, bd = blockDim.x;
  const double p0 = Pr[3 * q], p1 = Pr[3 * q + 1], p2 = Pr[3 * q + 2];
  if (tid == 0) {
    if (L.nv >= LH_VMAX) L.fail = 24;
    else {
      L.vx[L.nv][0] = p0; L.vx[L.nv][1] = p1; L.vx[L.nv][2] = p2;
      L.vpid[L.nv] = q;
    }
  }
  hl_bar();
  if (L.fail) return;
  const int v = L.nv, nf = L.nf, nfree0 = L.nfree;
  int nvis = 0;
  for (int f0 = 0; f0 < nf; f0 += bd) {
    const int f = f0 + tid;
    bool vis = false;
    if (f < nf && L.alive[f]) {
      const double* a = L.vx[L.fv[f][0]];
      const double d = L.fn[f][0] * (p0 - a[0]) + L.fn[f][1] * (p1 - a[1]) + L.fn[f][2] * (p2 - a[2]);
      const double nn = L.fn[f][3];
      if (d > 0.0 && d * d > eps2 * nn) {
        vis = true;
        if (L.cert[f]) L.fail = 25;                  // cannot happen: nothing is beyond a certified face
      } else if (d > 0.0 || d * d <= band2 * nn) {
        L.fail = 27;                                 // near-coplanar with the new vertex
      }
    }
    int tot;
    const int pos = nvis + hl_scan(L, vis ? 1 : 0, &tot);
    if (vis) {
      if (3 * pos + 3 > LH_EMAX) L.fail = 26;
      else {
        for (int k = 0; k < 3; ++k) { L.ea[3 * pos + k] = L.fv[f][k]; L.eb[3 * pos + k] = L.fv[f][(k + 1) % 3]; }
        L.freel[nfree0 + pos] = (unsigned short)f;
      }
    }
    nvis += tot;
  }
  hl_bar();
  if (L.fail || nvis == 0) return;   // nothing visible: q is inside Q
  for (int f0 = 0; f0 < nf; f0 += bd) {
    const int f = f0 + tid;
    if (f < nf && L.alive[f]) {
      const double* a = L.vx[L.fv[f][0]];
      const double d = L.fn[f][0] * (p0 - a[0]) + L.fn[f][1] * (p1 - a[1]) + L.fn[f][2] * (p2 - a[2]);
      if (d > 0.0 && d * d > eps2 * L.fn[f][3]) L.alive[f] = 0;
    }
  }
  const int ne = 3 * nvis, nfree = nfree0 + nvis;
  int nh = 0;
  for (int e0 = 0; e0 < ne; e0 += bd) {
    const int e = e0 + tid;
    bool hz = false;
    int a = 0, b = 0;
    if (e < ne) {
      a = L.ea[e]; b = L.eb[e];
      hz = true;
      for (int e2 = 0; e2 < ne; ++e2)
        if (L.ea[e2] == b && L.eb[e2] == a) { hz = false; break; }
    }
    int tot;
    const int k = nh + hl_scan(L, hz ? 1 : 0, &tot);
    if (hz) {
      const int f = k < nfree ? L.freel[nfree - 1 - k] : nf + (k - nfree);
      if (f >= LH_FMAX) L.fail = 28;
      else {
        L.fv[f][0] = (unsigned short)a; L.fv[f][1] = (unsigned short)b; L.fv[f][2] = (unsigned short)v;
        lh_face(L, f, vrel);
      }
    }
    nh += tot;
  }
  hl_bar();
  if (tid == 0 && !L.fail) {
    if (nh < 3) L.fail = 29;
    if (nh <= nfree) L.nfree = nfree - nh;
    else { L.nf = nf + (nh - nfree); L.nfree = 0; }
    L.nv = v + 1;
  }
  hl_bar();
}

// the support points of directions D0 .. D0+ND-1 (lowest id on ties) -> L.sup
template <int D0, int ND>
__device__ __forceinline__ void lh_support(LHullL& L, const double* Pr, int n) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  double bk[ND];
  int bi[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) { bk[d] = -INFINITY; bi[d] = INT_MAX; }
  for (int q = tid; q < n; q += blockDim.x) {
    const double x = Pr[3 * q], y = Pr[3 * q + 1], z = Pr[3 * q + 2];
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      const double v = L.dir[D0 + d][0] * x + L.dir[D0 + d][1] * y + L.dir[D0 + d][2] * z;
      if (v > bk[d]) { bk[d] = v; bi[d] = q; }   // q ascends per thread: first max = lowest id
    }
  }
  double* sk = reinterpret_cast<double*>(L.lp);                 // scratch: lp is not in use yet
  int* si = reinterpret_cast<int*>(sk + ND * (LH_THREADS / 64));
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    double k = bk[d];
    int i = bi[d];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double ok = __shfl_xor(k, off);
      const int oi = __shfl_xor(i, off);
      if (ok > k || (ok == k && oi < i)) { k = ok; i = oi; }
    }
    if (lane == 0) { sk[d * nw + wave] = k; si[d * nw + wave] = i; }
  }
  hl_bar();
  if (tid < ND) {
    double k = sk[tid * nw];
    int i = si[tid * nw];
    for (int w = 1; w < nw; ++w) {
      const double ok = sk[tid * nw + w];
      const int oi = si[tid * nw + w];
      if (ok > k || (ok == k && oi < i)) { k = ok; i = oi; }
    }
    L.sup[D0 + tid] = i;
  }
  hl_bar();
}

// Drop the live points that are inside Q by more than band / 2 from every
// face plane: Q only grows, so such a point is never beyond a later face nor
// within a few eps of one (the test n.p < n.a - band |n| / 2 differs from
// n.(p - a) by rounding far below band).  Workgroup-wide; the survivors go to
// the other buffer, and into LDS when they fit.
__device__ __forceinline__ void lh_compact(LHullL& L, double4* C0, double4* C1, double band) {
  const int tid = threadIdx.x;
  if (tid == 0) L.npk = 0;
  hl_bar();
  for (int f = tid; f < L.nf; f += blockDim.x) {
    if (!L.alive[f]) continue;
    const double* a = L.vx[L.fv[f][0]];
    const double n0 = L.fn[f][0], n1 = L.fn[f][1], n2 = L.fn[f][2];
    L.pk[atomicAdd(&L.npk, 1)] = make_double4(n0, n1, n2, n0 * a[0] + n1 * a[1] + n2 * a[2] - 0.5 * band * sqrt(L.fn[f][3]));
  }
  hl_bar();
  const double4* src = L.inlds ? L.lp : (L.cb ? C1 : C0);
  double4* dst = L.cb ? C0 : C1;
  const int nc = L.nc, npk = L.npk;
  int base = 0;
  for (int k0 = 0; k0 < nc; k0 += blockDim.x) {
    const int k = k0 + tid;
    bool keep = false;
    double4 c;
    if (k < nc) {
      c = src[k];
      for (int g = 0; g < npk && !keep; g += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const double4 P = L.pk[min(g + u, npk - 1)];
          keep |= P.x * c.x + P.y * c.y + P.z * c.z >= P.w;
        }
      }
    }
    int tot;
    const int pos = hl_scan(L, keep ? 1 : 0, &tot);
    if (keep) dst[base + pos] = c;
    base += tot;
  }
  const bool lds = base <= LH_LCAP;
  if (lds) {
    hl_bar();   // every lp read above is done; dst's stores are this block's own
    for (int k = tid; k < base; k += blockDim.x) L.lp[k] = dst[k];
  }
  hl_bar();
  if (tid == 0) { L.nc = base; L.cb ^= 1; L.ncompact = 2 * L.nv; L.inlds = lds ? 1 : 0; }
  hl_bar();
}

// for each of the nb batch faces, the arg-max of n.(c - a) over the live
// points (the face's own vertices excluded), lowest id on ties -> L.bkey /
// L.bidx.  Workgroup-wide.
template <int U, class P>
__device__ __forceinline__ void lh_scan_batch(LHullL& L, const P* C, int nc, int nb) {
  const int tid = threadIdx.x, bd = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = bd >> 6;
  double n0[LH_BATCH], n1[LH_BATCH], n2[LH_BATCH], a0[LH_BATCH], a1[LH_BATCH], a2[LH_BATCH], key[LH_BATCH];
  int x0[LH_BATCH], x1[LH_BATCH], x2[LH_BATCH], idx[LH_BATCH];
#pragma unroll
  for (int b = 0; b < LH_BATCH; ++b) {
    const int f = L.bf[b < nb ? b : 0];
    n0[b] = L.fn[f][0]; n1[b] = L.fn[f][1]; n2[b] = L.fn[f][2];
    const double* av = L.vx[L.fv[f][0]];
    a0[b] = av[0]; a1[b] = av[1]; a2[b] = av[2];
    x0[b] = L.vpid[L.fv[f][0]]; x1[b] = L.vpid[L.fv[f][1]]; x2[b] = L.vpid[L.fv[f][2]];
    key[b] = -INFINITY; idx[b] = INT_MAX;
  }
  for (int k0 = tid; k0 < nc; k0 += U * bd) {
    double4 c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * bd;
      c[u] = k < nc ? C[k] : make_double4(0.0, 0.0, 0.0, -1.0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = (int)c[u].w;
      if (q < 0) continue;
#pragma unroll
      for (int b = 0; b < LH_BATCH; ++b) {
        if (b >= nb) break;
        const double d = n0[b] * (c[u].x - a0[b]) + n1[b] * (c[u].y - a1[b]) + n2[b] * (c[u].z - a2[b]);
        if (q != x0[b] && q != x1[b] && q != x2[b] && (d > key[b] || (d == key[b] && q < idx[b]))) {
          key[b] = d; idx[b] = q;
        }
      }
    }
  }
#pragma unroll
  for (int b = 0; b < LH_BATCH; ++b) {
    if (b >= nb) break;
    double k = key[b];
    int i = idx[b];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double ok = __shfl_xor(k, off);
      const int oi = __shfl_xor(i, off);
      if (ok > k || (ok == k && oi < i)) { k = ok; i = oi; }
    }
    if (lane == 0) { L.sk[b * nw + wave] = k; L.si[b * nw + wave] = i; }
  }
  hl_bar();
  if (tid < nb) {
    double k = L.sk[tid * nw];
    int i = L.si[tid * nw];
    for (int w = 1; w < nw; ++w) {
      const double ok = L.sk[tid * nw + w];
      const int oi = L.si[tid * nw + w];
      if (ok > k || (ok == k && oi < i)) { k = ok; i = oi; }
    }
    L.bkey[tid] = k;
    L.bidx[tid] = i;
    for (int e = 0; e < 3; ++e) L.bt[tid][e] = L.fv[L.bf[tid]][e];
  }
  hl_bar();
}

// hull_points for k_lhull: the same points, in the same order and
// arithmetic, with the row's T_k, the sphere and the pair's translations
// staged in LDS (the lp region, free until the first compaction), one
// workgroup scan per round, and eps, delta and the live-point list produced
// in the same pass.  Sets L.n, L.fail, L.eps, L.delta.
static_assert(LH_LCAP * 4 >= 12 * 256 + 3 * 256, "lp stages T_k, translations (H <= 256) and the sphere (NP <= 256)");
__device__ __forceinline__ int lh_points(const HullArgs& A, LHullL& L, const double* Ti, const double* Ni,
                                         const double* xi, const double* xj, const double* vrel, double* Pr,
                                         double* Pf, double4* C0) {
  const int tid = threadIdx.x, bd = blockDim.x;
  const int H = A.H, NP = A.NP;
  double* sT = reinterpret_cast<double*>(L.lp);
  double* str = sT + H * 9;
  double* sS = str + H * 3;
  for (int q = tid; q < H * 9; q += bd) sT[q] = Ti[q];
  for (int q = tid; q < NP * 3; q += bd) sS[q] = A.S[q];
  for (int it = tid; it < 3 * H; it += bd) {
    const int k = it / 3, r = it % 3;
    double d = 0.0;
    for (int c = 0; c < A.X; ++c) d += Ni[((size_t)k * 3 + r) * A.X + c] * (xi[c] - xj[c]);
    str[it] = d;
  }
  if (tid == 0) L.fail = 0;
  hl_bar();
  int base = 0, oor = 0;
  double mx = 0.0, md = 0.0;
  const int ncand = A.ext_pts ? A.ext_n : H * NP;
  for (int q0 = 0; q0 < ncand; q0 += bd) {
    const int q = q0 + tid;
    bool ok = false;
    double p0 = 0, p1 = 0, p2 = 0;
    if (q < ncand && A.ext_pts) {
      ok = true;   // lqro_debug_hull_points: the points as given (rounded already)
      p0 = A.ext_pts[3 * q]; p1 = A.ext_pts[3 * q + 1]; p2 = A.ext_pts[3 * q + 2];
    } else if (q < ncand) {
      const int k = q / NP, p = q % NP;
      const double* Tk = sT + k * 9;
      const double* tk = str + k * 3;
      const double u0 = sS[3 * p] + tk[0], u1 = sS[3 * p + 1] + tk[1], u2 = sS[3 * p + 2] + tk[2];
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
    const int pos = base + hl_scan(L, ok ? 1 : 0, &tot);
    if (ok) {
      const bool given = A.ext_pts != nullptr;   // given points are rounded already (k_hull: P = P_rounded)
      const double r0 = given ? p0 : round6(p0, &oor), r1 = given ? p1 : round6(p1, &oor),
                   r2 = given ? p2 : round6(p2, &oor);
      Pf[3 * pos] = p0; Pf[3 * pos + 1] = p1; Pf[3 * pos + 2] = p2;
      Pr[3 * pos] = r0; Pr[3 * pos + 1] = r1; Pr[3 * pos + 2] = r2;
      C0[pos] = make_double4(r0, r1, r2, (double)pos);
      mx = fmax(mx, fmax(fabs(r0), fmax(fabs(r1), fabs(r2))));
      const double dx = p0 - r0, dy = p1 - r1, dz = p2 - r2;
      md = fmax(md, dx * dx + dy * dy + dz * dz);
    }
    base += tot;
  }
  if (oor) L.fail = 7;
  int dmy = 0;
  hl_argmax(L, mx, dmy);
  dmy = 0;
  hl_argmax(L, md, dmy);
  if (tid == 0) {
    L.n = base;
    L.eps = 1e-13 * (mx + 1.0);
    // delta = max |P - P_rounded|, with room for the rule's rounding
    L.delta = sqrt(md) * (1.0 + 1e-6) + 64.0 * L.eps;
    if (base < 4) L.fail = 8;
  }
  hl_bar();
  return base;
}

__device__ __forceinline__ void lhull_body(const HullArgs& A, LHullL& L) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int HNP = A.H * A.NP;
  double* Pr = A.scratch + (size_t)blockIdx.x * HNP * 6;   // rounded points
  double* Pf = Pr + (size_t)HNP * 3;                        // full-precision points
  // live points {x, y, z, id} (rounded), two buffers of H*NP
  double4* C0 = reinterpret_cast<double4*>(A.iscratch + (size_t)blockIdx.x * HNP * 2 * HULL_SCR_WAVES);
  double4* C1 = C0 + HNP;
  for (;;) {
    const int slot = hull_take_job(A, L, false);
    if (slot < 0) break;
    const int lrow = slot / A.npr, jj = A.nbr_list ? A.nbr_list[slot] : slot % A.npr;
    const int i = A.row_begin + lrow * A.row_stride;
    const int j = jj < i ? jj : jj + 1;
    const double* xi = A.x + (size_t)i * A.X;
    const double* xj = A.x + (size_t)j * A.X;
    const double* Ti = A.T + (A.per_agent ? (size_t)i * A.H * 9 : 0);
    const double* Ni = A.NCF + (A.per_agent ? (size_t)i * A.H * 3 * A.X : 0);
    const double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int n = lh_points(A, L, Ti, Ni, xi, xj, vrel, Pr, Pf, C0);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    int iters = 0, ncomp = 0;
    unsigned long long tcomp = 0, tset = 0;
    const double eps = L.eps, eps2 = eps * eps;
    const double band = 64.0 * eps, band2 = band * band;
    if (!L.fail) {
      hull_tetra(L, L, Pr, n, eps, eps2, L.vpid);
      hl_bar();
    }
    if (!L.fail) {
      if (tid < 4) lh_face(L, tid, vrel);
      if (tid == 0) { L.nf = 4; L.nv = 4; L.nfree = 0; L.best = INFINITY; L.nc = n; L.cb = 0; L.inlds = 0; }
      hl_bar();
      // a first Q from the support points of LH_DIRS directions (no scans
      // per insertion), then the first compaction
      lh_support<0, 8>(L, Pr, n);
      lh_support<8, 8>(L, Pr, n);
      lh_support<16, 8>(L, Pr, n);
      lh_support<24, 8>(L, Pr, n);
      for (int d = 0; d < LH_DIRS && !L.fail; ++d) {
        const int q = L.sup[d];
        bool dup = false;
        for (int v = 0; v < L.nv; ++v) dup |= L.vpid[v] == q;
        if (!dup) lh_insert(L, Pr, q, eps2, band2, vrel);
      }
      if (tid == 0) L.ncompact = L.nv;
      hl_bar();
      tset = __builtin_amdgcn_s_memrealtime() - t1;
      for (int it = 0;; ++it) {
        if (L.nv >= L.ncompact) {
          const unsigned long long tc = __builtin_amdgcn_s_memrealtime();
          lh_compact(L, C0, C1, band);
          tcomp += __builtin_amdgcn_s_memrealtime() - tc;
          ncomp++;
        }
        if (wave == 0) lh_choose(L, lane, band);
        hl_bar();
        const int task = L.task, nb = L.nb;
        iters = it;
        if (task == 0) break;
        if (it >= LH_ITERS) {
          if (tid == 0) L.fail = 21;
          break;
        }
        // the batch faces' furthest points, one pass over the live points
        if (L.inlds) lh_scan_batch<1>(L, L.lp, L.nc, nb);
        else lh_scan_batch<2>(L, L.cb ? C1 : C0, L.nc, nb);
        // in batch order: a face with a point beyond it takes that point (an
        // earlier insertion may have removed it), one without is certified
        for (int b = 0; b < nb && !L.fail; ++b) {
          const int f = L.bf[b];
          // gone, or its slot now holds a face of an earlier insertion
          if (!L.alive[f] || L.fv[f][0] != L.bt[b][0] || L.fv[f][1] != L.bt[b][1] || L.fv[f][2] != L.bt[b][2])
            continue;
          const double key = L.bkey[b], nn = L.fn[f][3];
          if (key > 0.0 && key * key > eps2 * nn) {
            lh_insert(L, Pr, L.bidx[b], eps2, band2, vrel);
          } else if (key > 0.0 || key * key <= band2 * nn) {
            if (tid == 0) L.fail = 22;                   // a point near the facet's plane
            hl_bar();
          } else if (task == 1) {
            if (tid == 0) L.fail = 23;                   // vrel on or beyond a full-hull facet
            hl_bar();
          } else {
            if (tid == 0) {
              L.cert[f] = 1;
              L.best = fmin(L.best, lh_rule(L, f, Pr, Pf, vrel));
            }
            hl_bar();
          }
        }
        if (L.fail) break;
      }
    }
    hl_bar();
    const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && A.ljobs && L.job < 4096) {
      unsigned long long* J = A.ljobs + 4 * (size_t)L.job;
      J[0] = (t1 - t0) | (tset << 32);
      J[1] = (t2 - t1) | (tcomp << 32);
      J[2] = (unsigned long long)iters | ((unsigned long long)L.nv << 16) | ((unsigned long long)(L.nc & 0xFFFF) << 32) |
             ((unsigned long long)gridDim.x << 48);
      J[3] = (unsigned long long)(n & 0xFFFF) | ((unsigned long long)blockIdx.x << 16) |
             ((unsigned long long)L.fail << 32) | ((unsigned long long)L.nf << 40) |
             ((unsigned long long)min(ncomp, 255) << 56);
    }
    if (!L.fail) {
      hull_select(A, L, L, Pr, Pf, L.vpid, L.nf, [&](int g) { return L.alive[g] && L.cert[g]; }, xi, vrel, slot,
                  true);
      if (tid == 0) {
        if (A.recs) A.recs[slot].flags |= LQRO_REC_LOCAL;
        atomicAdd(A.ldone, 1);
      }
    } else if (tid == 0) {
      A.lqueue[atomicAdd(A.lcount, 1)] = slot;             // the full hull decides
      if (A.lfail) atomicAdd(&A.lfail[L.fail >= 21 && L.fail <= 35 ? L.fail - 20 : 0], 1ull);
    }
    hl_bar();
  }
}

__global__ void __launch_bounds__(LH_THREADS) k_lhull(HullArgs A) {
  __shared__ LHullL L;
  if (threadIdx.x < LH_DIRS) {
    const int d = threadIdx.x;
    const double z = 1.0 - (2.0 * d + 1.0) / LH_DIRS, r = sqrt(1.0 - z * z), ph = 2.399963229728653 * d;
    L.dir[d][0] = r * cos(ph); L.dir[d][1] = r * sin(ph); L.dir[d][2] = z;
  }
  lhull_body(A, L);
}

}  // namespace lqro
