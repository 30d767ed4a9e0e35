// lqro_qhull.hpp — k_qhull: the inside-hull branch with the reference's OWN
// rule (LQRObstacles.cpp:867-969, LQRO_FLAG_QHULL_ORDER).
//
// convexHull writes the reachable points at 6 digits, runs qconvex n / Fv and
// takes min_f |n_f . (vrel - P[Fv_f[0]])| over the facets IN QHULL'S ORDER,
// measured from each facet's FIRST Fv vertex at full precision, strict '<';
// facet 0 never writes `normal` (LQRO:925-968).  Both the order and the first
// vertex (a simplicial facet lists its vertices newest first) are artefacts
// of Qhull's incremental build, so this kernel re-runs that build: Qhull
// 2019.1's 3-d algorithm with qconvex's defaults, restated in
// oracle/lqro_qhull.c (pinned to Qhull itself, facet for facet, bit for bit:
// tests/test_qhull_order.py) and here step for step: qh_maxmin,
// qh_maxsimplex, qh_initialhull, qh_partitionall, qh_furthestnext, then per
// point qh_nextfurthest, qh_findhorizon, qh_makenew_simplicial,
// qh_matchnewfacets, qh_makenewplanes (qh_sethyperplane_det / _gauss),
// qh_checkzero, qh_partitionvisible (qh_findbest, qh_findbestnew,
// qh_findbesthorizon, qh_partitionpoint), qh_deletevisible.
//
// One wave per inside-hull pair (a persistent grid over the hull queue; many
// waves per CU: the build is a chain of dependent steps, latency-bound).
// The facet list, planes, neighbours and outside sets live in the wave's
// global scratch (QhW); the chain runs uniformly on every lane; the per-point
// work — partitioning a visible region's outside points, the planes of the
// new facets, the convexity test, the selection — is spread over the lanes.
// Partitioning keeps Qhull's sequential semantics exactly: outside sets keep
// Qhull's order (the furthest point last; a displaced furthest point stays
// where it was), and the few order-dependent state changes inside one
// partition (the findbest -> findbestnew switch after the first interior
// point, an old facet that receives a point and moves behind the new ones, a
// coplanar point raising max_outside) are applied at their point, the rest of
// the sequence re-evaluated after them.
//
// Hulls that Qhull resolves by merging facets (coplanar horizon, a new facet
// not clearly convex, flipped, nearly singular) are built on merge-free, as
// the oracle does, and flagged LQRO_REC_QHMERGE.
#pragma once
#include <float.h>

#include "lqro_hull.hpp"
#include "lqro_dec16.hpp"

namespace lqro {

#ifndef QH_NEWCAP
#define QH_NEWCAP 1024    // new facets of one insertion (C5: > 256 seen)
#endif
#ifndef QH_VISCAP
#define QH_VISCAP 2048    // visible facets of one insertion (C5: > 256 seen)
#endif
#define QH_HZCAP 64       // facets one point's horizon walk visits (per lane)
#define QH_COPCAP 16      // qh.coplanarfacetset of one walk (per lane)
#define QH_MOVCAP 32      // old facets moved behind the new ones in one partition
#define QH_SBMULT 32      // outside-set entries: QH_SBMULT * H*NP per worker

#define QF_TOP 1
#define QF_VISIBLE 2
#define QF_NEW 4
#define QF_FLIPPED 8
#define QF_LIVE 16

// status bits (= oracle/lqro_qhull.h QHO_*)
#define QHS_INPUT 1
#define QHS_COPLANAR 2
#define QHS_NONCONVEX 4
#define QHS_FLIPPED 8
#define QHS_NARROW 16
#define QHS_SINGULAR 32
#define QHS_TOPOLOGY 64
#define QHS_CAPACITY 128   // a cap of this kernel (not Qhull's): the pair's record is a hull failure
// which cap (k_qhull_big; in the record's status with QHS_CAPACITY)
#define QHS_CAP_HZ 0x100
#define QHS_CAP_COP 0x200
#define QHS_CAP_MOV 0x400
#define QHS_CAP_SB 0x800
#define QHS_CAP_VIS 0x1000
#define QHS_CAP_NEW 0x2000
#define QHS_CAP_FACETS 0x4000
#define QHS_TIMEOUT 0x8000  // k_qhull: a wave handshake timed out (with QHS_CAPACITY: k_qhull_big rebuilds the pair)

struct QhW {
  double* Pr;      // 3 HNP rounded points (qconvex's input)
  double* Pf;      // 3 HNP full precision
  double* pl;      // 4 FC: facet normal, offset
  double* fdist;   // FC: furthestdist
  double* pdd;     // HNP: partition distance per sequence position
  int* fv;         // 3 FC: vertex ids (decreasing)
  int* fnb;        // 3 FC: neighbour opposite fv[k]
  int* flink;      // 2 FC: prev, next (facet list)
  int* frep;       // FC: f.replace
  int* fflag;      // FC: QF_*
  int* fseg;       // 2 FC: outside set: offset, count (last = furthest)
  int* fnew;       // FC: index in L.newf while the facet is new
  int* vpt;        // HNP + 8: vertex id -> point id
  int* sb;         // SB: outside-set entries
  int* pq;         // HNP: partition sequence: point ids
  int* pst;        // HNP: its start facet
  int* pdst;       // HNP: destination facet (-1: not outside) | event bits
  int* fstack;     // FC: free facet slots
  int* fvis;       // FC: qh_findhorizon visit stamp
  unsigned* vstamp;  // (QH_NEWCAP - 256) x 64: qh_findbest's visit marks of new facets >= 256, per lane
  unsigned* vctr;    // 64: each lane's last stamp (zeroed with the scratch, never reset)
  int FC, SB, HNP;
};

// A worker's scratch block is shared by k_qhull (Q3W) and k_qhull_big (QhW)
// of the same block index, and each keeps state across its jobs there (wave
// 1's epochs W.mark2 / W.ctr; the per-lane visit stamps W.vstamp / W.vctr).
// The block's last word names the kernel whose state it holds: a kernel that
// finds the other's tag resets its own cross-job state before its job (the
// wave that uses the state does it, so no other wave has to see the stores).
#define QW_TAG_BYTES 256
#define QW_OWNER_Q3 0x51335133u
#define QW_OWNER_QH 0x51485148u
__device__ __forceinline__ unsigned* qw_owner(char* block, size_t stride) {
  return reinterpret_cast<unsigned*>(block + stride - 4);
}

__host__ __device__ inline size_t qh_worker_bytes(int HNP) {
  const size_t FC = 2 * (size_t)HNP + QH_NEWCAP + 16, SB = (size_t)QH_SBMULT * HNP;
  return 8 * (7 * (size_t)HNP + 5 * FC) + 4 * (15 * FC + 4 * (size_t)HNP + 8 + SB) + 256 +
         4 * ((size_t)(QH_NEWCAP - 256) * 64 + 64);
}

__device__ inline QhW qh_worker(char* base, int HNP) {
  QhW W;
  W.HNP = HNP;
  W.FC = 2 * HNP + QH_NEWCAP + 16;
  W.SB = QH_SBMULT * HNP;
  double* d = reinterpret_cast<double*>(base);
  W.Pr = d; d += 3 * (size_t)HNP;
  W.Pf = d; d += 3 * (size_t)HNP;
  W.pl = d; d += 4 * (size_t)W.FC;
  W.fdist = d; d += W.FC;
  W.pdd = d; d += HNP;
  int* p = reinterpret_cast<int*>(d);
  W.fv = p; p += 3 * (size_t)W.FC;
  W.fnb = p; p += 3 * (size_t)W.FC;
  W.flink = p; p += 2 * (size_t)W.FC;
  W.frep = p; p += W.FC;
  W.fflag = p; p += W.FC;
  W.fseg = p; p += 2 * (size_t)W.FC;
  W.fnew = p; p += W.FC;
  W.fstack = p; p += W.FC;
  W.fvis = p; p += W.FC;
  W.vstamp = reinterpret_cast<unsigned*>(p); p += (size_t)(QH_NEWCAP - 256) * 64;
  W.vctr = reinterpret_cast<unsigned*>(p); p += 64;
  W.vpt = p; p += HNP + 8;
  W.pq = p; p += HNP;
  W.pst = p; p += HNP;
  W.pdst = p; p += HNP;
  W.sb = p;
  return W;
}

// the wave's LDS: hull_points / hull_take_job interface, then the build state
struct QhL {
  int n, fail, job, slot;
  double eps;
  double tr[3 * 128];
  double rk[4];            // (four: q3_big_inline runs hull_points on all of k_qhull's waves)
  int ri[4];
  int scan[4];
  int newf[QH_NEWCAP];     // new facets, creation (= list) order
  int visf[QH_VISCAP];     // visible facets, qh_findhorizon order
  int movf[QH_MOVCAP];     // old facets moved behind the new ones this partition (scan order)
  int oldf[QH_MOVCAP];     // old facets receiving points this partition (destinations)
  int dfac[QH_NEWCAP + QH_MOVCAP];   // destination -> facet
  int dcnt[QH_NEWCAP + QH_MOVCAP];   // running set size
  int doff[QH_NEWCAP + QH_MOVCAP];   // its new segment
  int dchamp[QH_NEWCAP + QH_MOVCAP]; // running furthest point
  double dmax[QH_NEWCAP + QH_MOVCAP];
  int pcnt[QH_NEWCAP + QH_MOVCAP];   // points added this partition
};

// Qhull's scalar state of one build (registers, uniform over the wave)
struct QhS {
  int facet_list, facet_tail, facet_next, newfacet_list, visible_list;
  int nins;                     // insertions (qh_addpoint calls), for the build's timing record
  int nalloc, nfree, nv, sbtop, status;
  int nnew, nvis, nmov, nold, epoch;
  int findbestnew, notsharp;
  double MAXabs_coord, MAXsumcoord, MAXwidth, NEARzero[3];
  double DISTround, MINvisible, MAXcoplanar, MINoutside, MINdenom, MINdenom_2, max_outside;
  double interior[3];
  unsigned long long tph[12];   // LQRO_QHULL_PROFILE: cycles per phase
};
#ifdef LQRO_QHULL_PROFILE
#define QHT(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); S.tph[k] += t_ - tq_; tq_ = t_; } while (0)
#else
#define QHT(k) do {} while (0)
#endif

// ---- the facet list (poly_r.c: qh_appendfacet, qh_removefacet, qh_prependfacet) ----
__device__ __forceinline__ int qh_prev(const QhW& W, int f) { return W.flink[2 * f]; }
__device__ __forceinline__ int qh_next(const QhW& W, int f) { return W.flink[2 * f + 1]; }

__device__ __forceinline__ void qh_appendfacet(const QhW& W, QhS& S, int f) {
  const int tail = S.facet_tail;
  if (tail == S.newfacet_list) {
    S.newfacet_list = f;
    if (tail == S.visible_list) S.visible_list = f;
  }
  if (tail == S.facet_next) S.facet_next = f;
  const int tp = qh_prev(W, tail);
  W.flink[2 * f] = tp;
  W.flink[2 * f + 1] = tail;
  if (tp >= 0) W.flink[2 * tp + 1] = f;
  else S.facet_list = f;
  W.flink[2 * tail] = f;
}

__device__ __forceinline__ void qh_removefacet(const QhW& W, QhS& S, int f) {
  const int nx = qh_next(W, f), pv = qh_prev(W, f);
  if (f == S.newfacet_list) S.newfacet_list = nx;
  if (f == S.facet_next) S.facet_next = nx;
  if (f == S.visible_list) S.visible_list = nx;
  if (pv >= 0) {
    W.flink[2 * pv + 1] = nx;
    W.flink[2 * nx] = pv;
  } else {
    S.facet_list = nx;
    W.flink[2 * nx] = -1;
  }
}

__device__ __forceinline__ int qh_newfacet(const QhW& W, QhS& S) {
  int f;
  if (S.nfree > 0) f = W.fstack[--S.nfree];
  else if (S.nalloc < W.FC) f = S.nalloc++;
  else { S.status |= QHS_CAPACITY | QHS_CAP_FACETS; f = 0; }
  W.fv[3 * f] = W.fv[3 * f + 1] = W.fv[3 * f + 2] = 0;
  W.fnb[3 * f] = W.fnb[3 * f + 1] = W.fnb[3 * f + 2] = -1;
  W.flink[2 * f] = W.flink[2 * f + 1] = -1;
  W.frep[f] = -1;
  W.fvis[f] = 0;
  W.fflag[f] = QF_NEW;
  W.fseg[2 * f] = 0;
  W.fseg[2 * f + 1] = 0;
  W.fdist[f] = 0.0;
  return f;
}

// ---- geometry (geom_r.c, geom2_r.c) ----
__device__ __forceinline__ double qh_dist(const QhW& W, const double* p, int f) {   // qh_distplane
  const double* q = W.pl + 4 * (size_t)f;
  return q[3] + p[0] * q[0] + p[1] * q[1] + p[2] * q[2];
}

#define QH_DET2(a1, a2, b1, b2) ((a1) * (b2) - (a2) * (b1))

// qh_sethyperplane_gauss (dim 3): qh_gausselim + qh_backnormal + qh_normalize2
__device__ inline void qh_plane_gauss(const QhS& S, int& status, const double* r0, const double* r1,
                                      const double* r2, int toporient, double* nrm, double* offset) {
  double ra[3] = {r1[0] - r0[0], r1[1] - r0[1], r1[2] - r0[2]};
  double rb[3] = {r2[0] - r0[0], r2[1] - r0[1], r2[2] - r0[2]};
  double* rows[2] = {ra, rb};
  int sign = toporient;
  for (int k = 0; k < 2; k++) {
    double pivot_abs = fabs(rows[k][k]);
    int pivoti = k;
    for (int i = k + 1; i < 2; i++) {
      const double temp = fabs(rows[i][k]);
      if (temp > pivot_abs) { pivot_abs = temp; pivoti = i; }
    }
    if (pivoti != k) {
      double* t = rows[pivoti];
      rows[pivoti] = rows[k];
      rows[k] = t;
      sign ^= 1;
    }
    if (pivot_abs <= S.NEARzero[k]) {
      status |= QHS_SINGULAR;
      if (pivot_abs == 0.0) continue;
    }
    const double pivot = rows[k][k];
    for (int i = k + 1; i < 2; i++) {
      const double nn = rows[i][k] / pivot;
      for (int j = k + 1; j < 3; j++) rows[i][j] -= nn * rows[k][j];
    }
  }
  for (int k = 2; k--;)
    if (rows[k][k] < 0) sign ^= 1;
  nrm[2] = sign ? -1.0 : 1.0;
  for (int i = 2; i--;) {
    double acc = 0.0;
    for (int j = i + 1; j < 3; j++) acc -= rows[i][j] * nrm[j];
    const double diagonal = rows[i][i];
    if (fabs(diagonal) > S.MINdenom_2) acc /= diagonal;
    else status |= QHS_SINGULAR;
    nrm[i] = acc;
  }
  const double norm = sqrt(nrm[0] * nrm[0] + nrm[1] * nrm[1] + nrm[2] * nrm[2]);
  if (norm > S.MINdenom) {
    nrm[0] /= norm;
    nrm[1] /= norm;
    nrm[2] /= norm;
  } else {
    status |= QHS_SINGULAR;
  }
  double off = -(r0[0] * nrm[0]);
  off -= r0[1] * nrm[1];
  off -= r0[2] * nrm[2];
  *offset = off;
}

// qh_setfacetplane (qh_sethyperplane_det, nearzero -> _gauss) + the flipped
// test of qh_checkflipped(qh_ALL); returns the plane in pl, sets QF_FLIPPED
__device__ inline void qh_setfacetplane(const QhW& W, const QhS& S, int& status, int f) {
  const double* r0 = W.Pr + 3 * (size_t)W.vpt[W.fv[3 * f]];
  const double* r1 = W.Pr + 3 * (size_t)W.vpt[W.fv[3 * f + 1]];
  const double* r2 = W.Pr + 3 * (size_t)W.vpt[W.fv[3 * f + 2]];
  const int top = W.fflag[f] & QF_TOP;
  const double dX10 = r1[0] - r0[0], dY10 = r1[1] - r0[1], dZ10 = r1[2] - r0[2];
  const double dX20 = r2[0] - r0[0], dY20 = r2[1] - r0[1], dZ20 = r2[2] - r0[2];
  double n[3];
  n[0] = QH_DET2(dY20, dZ20, dY10, dZ10);
  n[1] = QH_DET2(dX10, dZ10, dX20, dZ20);
  n[2] = QH_DET2(dX20, dY20, dX10, dY10);
  double norm = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  if (norm > S.MINdenom) {
    if (!top) norm = -norm;
    n[0] /= norm;
    n[1] /= norm;
    n[2] /= norm;
  } else {
    status |= QHS_SINGULAR;
  }
  double off = -(r0[0] * n[0] + r0[1] * n[1] + r0[2] * n[2]);
  const double d2 = off + (r2[0] * n[0] + r2[1] * n[1] + r2[2] * n[2]);
  const double d1 = off + (r1[0] * n[0] + r1[1] * n[1] + r1[2] * n[2]);
  if (d2 > S.DISTround || d2 < -S.DISTround || d1 > S.DISTround || d1 < -S.DISTround)
    qh_plane_gauss(S, status, r0, r1, r2, top, n, &off);
  double* q = W.pl + 4 * (size_t)f;
  q[0] = n[0]; q[1] = n[1]; q[2] = n[2]; q[3] = off;
  const double di = off + S.interior[0] * n[0] + S.interior[1] * n[1] + S.interior[2] * n[2];
  if (di >= -S.DISTround) W.fflag[f] |= QF_FLIPPED;
  else W.fflag[f] &= ~QF_FLIPPED;
}

// ---- point location, per lane (geom_r.c) ----
// qh_findbesthorizon; the walk's visited facets in a per-lane list
__device__ inline int qh_findbesthorizon(const QhW& W, const QhS& S, const double* p, int startfacet,
                                         double* bestdist, int& lstatus) {
  int bestfacet = startfacet;
  const double searchdist = S.max_outside + 2 * S.DISTround + fmax(S.MINvisible, S.MAXcoplanar);
  double minsearch = *bestdist - searchdist;
  int vis[QH_HZCAP];
  int nvis = 0;
  int cop[QH_COPCAP];
  int ncop = 0;
  int nextfacet = -1;
  vis[nvis++] = startfacet;
  int facet = startfacet;
  for (;;) {
    for (int k = 0; k < 3; k++) {
      const int nb = W.fnb[3 * facet + k];
      bool seen = false;
      for (int t = 0; t < nvis; t++) seen |= vis[t] == nb;
      if (seen) continue;
      if (nvis == QH_HZCAP) { lstatus |= QHS_CAPACITY | QHS_CAP_HZ; return bestfacet; }
      vis[nvis++] = nb;
      if (!(W.fflag[nb] & QF_FLIPPED)) {
        const double dist = qh_dist(W, p, nb);
        if (dist > *bestdist) {
          minsearch = dist - searchdist;
          if (dist > *bestdist + searchdist) ncop = 0;
          bestfacet = nb;
          *bestdist = dist;
        } else if (dist < minsearch) {
          continue;
        }
      }
      if (nextfacet >= 0) {
        if (ncop == QH_COPCAP) { lstatus |= QHS_CAPACITY | QHS_CAP_COP; return bestfacet; }
        cop[ncop++] = nextfacet;
      }
      nextfacet = nb;
    }
    facet = nextfacet;
    if (facet >= 0) nextfacet = -1;
    else if (!ncop) break;
    else if (ncop == 1) { facet = cop[0]; ncop = 0; }
    else facet = cop[--ncop];
  }
  return bestfacet;
}

// qh_findbestnew over the scan list (the new facets from startfacet on, the
// moved old facets, then the new facets before startfacet: the facet list
// from startfacet to its end, then from qh.newfacet_list)
__device__ inline int qh_findbestnew(const QhW& W, const QhS& S, const QhL& L, const double* p, int startfacet,
                                     double* dist, int bestoutside, int* isoutside, int& lstatus) {
  double bestdist = -DBL_MAX / 2;
  int bestfacet = -1;
  const double distoutside = fmax(2 * S.MINoutside, S.max_outside);    // qh_DISToutside
  *isoutside = 1;
  const int s0 = W.fnew[startfacet];
  const int total = S.nnew + S.nmov;
  for (int t = 0; t < total; t++) {
    int f;
    if (t < S.nnew - s0) f = L.newf[s0 + t];
    else if (t < S.nnew - s0 + S.nmov) f = L.movf[t - (S.nnew - s0)];
    else f = L.newf[t - (S.nnew - s0) - S.nmov];
    if (W.fflag[f] & QF_FLIPPED) continue;
    const double d = qh_dist(W, p, f);
    if (d > bestdist) {
      bestfacet = f;
      if (!bestoutside && d >= distoutside) { *dist = d; return bestfacet; }
      bestdist = d;
    }
  }
  bestfacet = qh_findbesthorizon(W, S, p, bestfacet >= 0 ? bestfacet : startfacet, &bestdist, lstatus);
  *dist = bestdist;
  if (bestdist < S.MINoutside) *isoutside = 0;
  return bestfacet;
}

// qh_sharpnewfacets
__device__ inline int qh_sharpnewfacets(const QhW& W, const QhS& S, const QhL& L) {
  int quadrant[3];
  for (int t = 0; t < S.nnew; t++) {
    const double* n = W.pl + 4 * (size_t)L.newf[t];
    if (t == 0) {
      for (int k = 3; k--;) quadrant[k] = n[k] > 0;
    } else {
      for (int k = 3; k--;)
        if (quadrant[k] != (n[k] > 0)) return 1;
    }
  }
  return 0;
}

// One partitioned point under the state (S.findbestnew, S.notsharp): its
// facet and distance, and whether it changes the state ("trigger": the
// first point whose directed search ends inside; Qhull then tests the new
// facets' sharpness).  qh_partitionpoint -> qh_findbest(isnewfacets) /
// qh_findbestnew.
__device__ inline int qh_locate(const QhW& W, const QhS& S, const QhL& L, const double* p, int startfacet,
                                int sharp, double* bestdist_out, int* isoutside, int* trigger, int& lstatus) {
  *trigger = 0;
  if (S.findbestnew) return qh_findbestnew(W, S, L, p, startfacet, bestdist_out, 0, isoutside, lstatus);
  // qh_findbest(point, startfacet, bestoutside 0, isnewfacets 1, noupper 0)
  double bestdist = -DBL_MAX / 2;
  int bestfacet = -1;
  *isoutside = 1;
  // new facets visited: a bit per new-facet index below 256; beyond (an
  // insertion with more than 256 new facets, C5), a per-lane stamp in the
  // worker's scratch, fresh for this call
  unsigned long long s0 = 0ull, s1 = 0ull, s2 = 0ull, s3 = 0ull;
  const int ln = threadIdx.x & 63;
  unsigned stamp = 0u;
  auto mark = [&](int f) {
    const int t = W.fnew[f];
    if (t >= 256) {
      if (!stamp) { stamp = W.vctr[ln] + 1u; if (!stamp) stamp = 1u; W.vctr[ln] = stamp; }
      W.vstamp[(size_t)(t - 256) * 64 + ln] = stamp;
      return;
    }
    const unsigned long long b = 1ull << (t & 63);
    if (t < 64) s0 |= b;
    else if (t < 128) s1 |= b;
    else if (t < 192) s2 |= b;
    else s3 |= b;
  };
  auto was = [&](int f) -> bool {
    const int t = W.fnew[f];
    if (t >= 256) return stamp && W.vstamp[(size_t)(t - 256) * 64 + ln] == stamp;
    const unsigned long long w = t < 64 ? s0 : t < 128 ? s1 : t < 192 ? s2 : s3;
    return (w >> (t & 63)) & 1ull;
  };
  if (!(W.fflag[startfacet] & QF_FLIPPED)) {
    const double d = qh_dist(W, p, startfacet);
    if (d >= S.MINoutside) { *bestdist_out = d; return startfacet; }
    bestdist = d;
    bestfacet = startfacet;
  }
  mark(startfacet);
  int facet = startfacet;
  while (facet >= 0) {
    int nxt = -1;
    for (int k = 0; k < 3; k++) {
      const int nb = W.fnb[3 * facet + k];
      if (!(W.fflag[nb] & QF_NEW)) continue;
      if (was(nb)) continue;
      mark(nb);
      if (!(W.fflag[nb] & QF_FLIPPED)) {
        const double d = qh_dist(W, p, nb);
        if (d > bestdist) {
          if (d >= S.MINoutside) { *bestdist_out = d; return nb; }
          bestfacet = nb;
          bestdist = d;
          nxt = nb;
          break;
        }
      }
    }
    facet = nxt;
  }
  if (bestfacet < 0) {
    return qh_findbestnew(W, S, L, p, L.newf[0], bestdist_out, 0, isoutside, lstatus);
  }
  if (!S.notsharp && bestdist < -S.DISTround) {
    *trigger = 1;
    if (sharp) return qh_findbestnew(W, S, L, p, bestfacet, bestdist_out, 0, isoutside, lstatus);
  }
  bestfacet = qh_findbesthorizon(W, S, p, bestfacet, &bestdist, lstatus);
  *bestdist_out = bestdist;
  if (bestdist < S.MINoutside) *isoutside = 0;
  return bestfacet;
}

// ---- partitioning in Qhull's order ----
// wave-wide OR of a lane flag
// (no lane flagged — the common case — costs one ballot; otherwise a DPP
// reduction to lane 63, no LDS round trip)
__device__ __forceinline__ int qh_wave_or(int v) {
  if (!__ballot(v != 0)) return 0;
  v |= __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v |= __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v |= __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v |= __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
  v |= __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
  v |= __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
  return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ bool qh_in_movf(const QhS& S, const QhL& L, int f) {
  for (int t = 0; t < S.nmov; t++)
    if (L.movf[t] == f) return true;
  return false;
}

// Locate the points of the sequence W.pq[0..np) (start facets W.pst),
// qh_partitionpoint's search for each in order; W.pdst = facet or -1, W.pdd =
// distance.  Three results change the state for the points after them: the
// first interior point of the directed search (Qhull tests the new facets'
// sharpness: findbestnew from then on, or findbest without the test), a
// coplanar point above max_outside, and a first point for an old facet with
// an empty outside set (qh_partitionpoint moves it behind the new facets,
// where later findbestnew scans reach it).  The lanes locate a chunk at a
// time; at the first such point the state changes and the rest of the
// sequence is located again.  all_phase: qh_partitionall's remainder (every
// point starts at the head of the facet list; a moved facet changes it).
__device__ inline void qh_locate_seq(const QhW& W, QhS& S, QhL& L, int np, int sharp, bool all_phase,
                                     int lane) {
  int from = 0;
  while (from < np) {
    int ev_pos = np, ev_kind = 0;
    for (int c = from; c < np; c += 64) {
      const int pos = c + lane;
      int kind = 0, ls = 0;
      if (pos < np) {
        const int pid = W.pq[pos];
        double d;
        int isout, trig;
        const int f = qh_locate(W, S, L, W.Pr + 3 * (size_t)pid, W.pst[pos], sharp, &d, &isout, &trig, ls);
        int dst = -1;
        if (isout) {
          dst = f;
          if (!(W.fflag[f] & QF_NEW) && W.fseg[2 * f + 1] == 0 && !qh_in_movf(S, L, f)) kind |= 4;
        } else if (d >= -S.MAXcoplanar && d > S.max_outside) {
          kind |= 2;
        }
        if (trig) kind |= 1;
        W.pdst[pos] = dst;
        W.pdd[pos] = d;
      }
      ls = qh_wave_or(ls);
      S.status |= ls;
      const unsigned long long b = __ballot(kind != 0);
      hl_sync();
      if (b) {
        const int l = __ffsll((long long)b) - 1;
        ev_pos = c + l;
        ev_kind = __builtin_amdgcn_readlane(kind, l);
        break;
      }
    }
    if (ev_pos < np) {
      if (ev_kind & 1) {
        if (sharp) S.findbestnew = 1;
        else S.notsharp = 1;
      }
      if (ev_kind & 2) S.max_outside = W.pdd[ev_pos];
      if (ev_kind & 4) {
        const int f = W.pdst[ev_pos];
        if (S.nmov == QH_MOVCAP) S.status |= QHS_CAPACITY | QHS_CAP_MOV;
        else {
          qh_removefacet(W, S, f);        // "make sure it's after qh.facet_next"
          qh_appendfacet(W, S, f);
          if (all_phase) {
            // the remainder's scan list is the facet list itself: move f to its end
            int t0 = W.fnew[f];
            for (int t = t0; t + 1 < S.nnew; t++) {
              L.newf[t] = L.newf[t + 1];
              W.fnew[L.newf[t]] = t;
            }
            L.newf[S.nnew - 1] = f;
            W.fnew[f] = S.nnew - 1;
            L.movf[S.nmov++] = f;   // counts as moved (no second move), not scanned twice
            for (int q = ev_pos + 1 + lane; q < np; q += 64) W.pst[q] = S.facet_list;
          } else {
            L.movf[S.nmov++] = f;
          }
        }
      }
      hl_sync();
    }
    from = ev_pos + 1;
  }
}

// The located points into their facets' outside sets, in sequence order,
// with Qhull's placement (qh_partitionpoint: append when further than the
// furthest point, else insert before it).  For the points one facet receives
// in order, point 0 is the furthest so far and is held aside; point k > 0
// lands at position (count before) + k - 1 and is itself, or — when it is
// further than the furthest — the displaced furthest point; the last furthest
// point ends the set.  A facet with points already (an old facet) continues
// its set in a fresh segment.
__device__ inline void qh_emit_seq(const QhW& W, QhS& S, QhL& L, int np, int lane) {
  // destinations: new facets d = fnew (0..nnew-1); old facets QH_NEWCAP + k
  for (int t = lane; t < S.nnew; t += 64) { L.pcnt[t] = 0; L.dfac[t] = L.newf[t]; }
  S.nold = 0;
  hl_sync();
  for (int c = 0; c < np; c += 64) {
    const int pos = c + lane;
    int dst = pos < np ? W.pdst[pos] : -1;
    const bool isnew = dst >= 0 && (W.fflag[dst] & QF_NEW);
    if (isnew) atomicAdd(&L.pcnt[W.fnew[dst]], 1);
    unsigned long long old = __ballot(dst >= 0 && !isnew);
    while (old) {   // old facets: registered in sequence order (rare)
      const int l = __ffsll((long long)old) - 1;
      old &= old - 1;
      const int f = __builtin_amdgcn_readlane(dst, l);
      int k = -1;
      for (int t = 0; t < S.nold; t++)
        if (L.oldf[t] == f) k = t;
      if (k < 0) {
        if (S.nold == QH_MOVCAP) { S.status |= QHS_CAPACITY | QHS_CAP_MOV; continue; }
        k = S.nold++;
        if (lane == 0) { L.oldf[k] = f; L.pcnt[QH_NEWCAP + k] = 0; L.dfac[QH_NEWCAP + k] = f; }
        hl_sync();
      }
      if (lane == 0) L.pcnt[QH_NEWCAP + k]++;
      hl_sync();
    }
    hl_sync();
  }
  hl_sync();
  if (S.status & QHS_CAPACITY) return;
  // segments: each destination's set continues (old) or starts (new)
  for (int g0 = 0; g0 < S.nnew + S.nold; g0++) {
    const int g = g0 < S.nnew ? g0 : QH_NEWCAP + (g0 - S.nnew);
    const int add = L.pcnt[g];
    if (!add) continue;
    const int f = L.dfac[g];
    const int cnt0 = W.fseg[2 * f + 1], off0 = W.fseg[2 * f];
    const int size = cnt0 + add;
    if (S.sbtop + size > W.SB) { S.status |= QHS_CAPACITY | QHS_CAP_SB; return; }
    const int off = S.sbtop;
    S.sbtop += size;
    for (int t = lane; t < cnt0 - 1; t += 64) W.sb[off + t] = W.sb[off0 + t];
    if (lane == 0) {
      L.doff[g] = off;
      L.dcnt[g] = cnt0;
      L.dmax[g] = W.fdist[f];
      L.dchamp[g] = cnt0 ? W.sb[off0 + cnt0 - 1] : -1;
    }
    if (g >= QH_NEWCAP) { if (lane == 0) W.fnew[f] = g; }   // old facet -> its destination
    hl_sync();
  }
  hl_sync();
  // the sequence in order: a chunk's lanes, grouped by destination
  for (int c = 0; c < np; c += 64) {
    const int pos = c + lane;
    const bool act = pos < np;
    const int dst = act ? W.pdst[pos] : -1;
    const int g = dst >= 0 ? W.fnew[dst] : -1;
    const int pid = act ? W.pq[pos] : -1;
    const double dd = act ? W.pdd[pos] : 0.0;
    unsigned long long todo = __ballot(g >= 0);
    while (todo) {
      const int lead = __ffsll((long long)todo) - 1;
      const int gg = __builtin_amdgcn_readlane(g, lead);
      const unsigned long long grp = __ballot(g == gg);
      todo &= ~grp;
      int cnt = L.dcnt[gg];
      double mx = L.dmax[gg];
      int champ = L.dchamp[gg];
      const int off = L.doff[gg];
      unsigned long long m = grp;
      while (m) {
        const int l = __ffsll((long long)m) - 1;
        m &= m - 1;
        const int q = __builtin_amdgcn_readlane(pid, l);
        const double dq = hl_rl(dd, l);
        if (cnt == 0) {
          champ = q;
          mx = dq;
        } else if (mx < dq) {
          if (lane == 0) W.sb[off + cnt - 1] = champ;
          champ = q;
          mx = dq;
        } else {
          if (lane == 0) W.sb[off + cnt - 1] = q;
        }
        cnt++;
      }
      if (lane == 0) { L.dcnt[gg] = cnt; L.dmax[gg] = mx; L.dchamp[gg] = champ; }
      hl_sync();
    }
  }
  hl_sync();
  for (int g0 = lane; g0 < S.nnew + S.nold; g0 += 64) {
    const int g = g0 < S.nnew ? g0 : QH_NEWCAP + (g0 - S.nnew);
    if (!L.pcnt[g]) continue;
    const int f = L.dfac[g];
    W.sb[L.doff[g] + L.dcnt[g] - 1] = L.dchamp[g];
    W.fseg[2 * f] = L.doff[g];
    W.fseg[2 * f + 1] = L.dcnt[g];
    W.fdist[f] = L.dmax[g];
    if (g >= QH_NEWCAP) W.fnew[f] = 0x7fffffff;
  }
  hl_sync();
}

// ---- the build ----
__device__ inline void qh_set_top(const QhW& W, int f, int top) {
  W.fflag[f] = top ? (W.fflag[f] | QF_TOP) : (W.fflag[f] & ~QF_TOP);
}

// first (lowest index) extreme per coordinate, qh_maxmin
__device__ inline void qh_extreme(const double* Pr, int n, int k, bool want_max, int lane, int* idx_out) {
  double key = -DBL_MAX;
  int idx = 0x7fffffff;
  for (int q = lane; q < n; q += 64) {
    const double v = want_max ? Pr[3 * q + k] : -Pr[3 * q + k];
    if (v > key || (v == key && q < idx)) { key = v; idx = q; }
  }
  for (int off = 32; off >= 1; off >>= 1) {
    const double ok = __shfl_xor(key, off);
    const int oi = __shfl_xor(idx, off);
    if (ok > key || (ok == key && oi < idx)) { key = ok; idx = oi; }
  }
  *idx_out = idx;
}

__device__ inline double qh_detsimplex(const QhS& S, const double* Pr, const int* simplex, int dim, int apex,
                                       int* nearzero) {
  double rows[3][3];
  const double* a = Pr + 3 * (size_t)apex;
  for (int i = 0; i < dim; i++)
    for (int k = 0; k < dim; k++) rows[i][k] = Pr[3 * (size_t)simplex[i] + k] - a[k];
  double det;
  if (dim == 2) {
    det = QH_DET2(rows[0][0], rows[0][1], rows[1][0], rows[1][1]);
    *nearzero = fabs(det) < 10 * S.NEARzero[1];
  } else {
    det = rows[0][0] * QH_DET2(rows[1][1], rows[1][2], rows[2][1], rows[2][2]) -
          rows[1][0] * QH_DET2(rows[0][1], rows[0][2], rows[2][1], rows[2][2]) +
          rows[2][0] * QH_DET2(rows[0][1], rows[0][2], rows[1][1], rows[1][2]);
    *nearzero = fabs(det) < 10 * S.NEARzero[2];
  }
  return det;
}

// qh_qhull on W.Pr[0..n): S holds the final facet list
__device__ inline void qh_build(const QhW& W, QhS& S, QhL& L, int n, int lane) {
#ifdef LQRO_QHULL_PROFILE
  unsigned long long tq_ = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < 12; k++) S.tph[k] = 0;
#endif
  S.status = 0;
  S.nalloc = 1;   // slot 0: the tail sentinel
  S.nfree = 0;
  S.sbtop = 0;
  S.nnew = S.nvis = S.nmov = S.nold = 0;
  S.epoch = 0;
  S.findbestnew = S.notsharp = 0;
  S.facet_tail = 0;
  W.flink[0] = -1;
  W.flink[1] = -1;
  W.fflag[0] = 0;
  W.fnew[0] = 0x7fffffff;
  S.facet_list = S.facet_next = S.newfacet_list = S.visible_list = 0;
  S.nv = 1;
  // qh_maxmin
  int maxpoints[6];
  S.max_outside = 0.0;
  S.MAXabs_coord = 0.0;
  S.MAXwidth = -DBL_MAX;
  S.MAXsumcoord = 0.0;
  for (int k = 0; k < 3; k++) {
    int mn, mx;
    qh_extreme(W.Pr, n, k, false, lane, &mn);
    qh_extreme(W.Pr, n, k, true, lane, &mx);
    const double maxk = W.Pr[3 * (size_t)mx + k], mink = W.Pr[3 * (size_t)mn + k];
    const double maxcoord = fmax(maxk, -mink);
    const double temp = maxk - mink;
    if (temp > S.MAXwidth) S.MAXwidth = temp;
    if (maxcoord > S.MAXabs_coord) S.MAXabs_coord = maxcoord;
    S.MAXsumcoord += maxcoord;
    maxpoints[2 * k] = mn;
    maxpoints[2 * k + 1] = mx;
    S.NEARzero[k] = 80 * S.MAXsumcoord * DBL_EPSILON;
  }
  // qh_detroundoff (C-0)
  {
    double maxdistsum = sqrt(3.0) * S.MAXabs_coord;
    if (S.MAXsumcoord < maxdistsum) maxdistsum = S.MAXsumcoord;
    S.DISTround = DBL_EPSILON * (3 * maxdistsum * 1.01 + S.MAXabs_coord);
    const double MINdenom_1 = fmax(1.0 / DBL_MAX, DBL_MIN);
    S.MINdenom = MINdenom_1 * S.MAXabs_coord;
    S.MINdenom_2 = sqrt(MINdenom_1 * 3) * S.MAXabs_coord;
    S.MINvisible = 0.0 + 2 * S.DISTround;
    S.MAXcoplanar = S.MINvisible;
    S.MINoutside = 2 * S.MINvisible;
  }
  // qh_maxsimplex
  int simplex[4];
  {
    double maxcoord = -DBL_MAX, mincoord = DBL_MAX;
    int minx = -1, maxx = -1;
    for (int i = 0; i < 6; i++) {
      const double c = W.Pr[3 * (size_t)maxpoints[i]];
      if (maxcoord < c) { maxcoord = c; maxx = maxpoints[i]; }
      if (mincoord > c) { mincoord = c; minx = maxpoints[i]; }
    }
    double maxdet = maxcoord - mincoord;
    int ns = 0;
    simplex[ns++] = minx;
    if (maxx != minx) simplex[ns++] = maxx;
    if (ns < 2) { S.status |= QHS_INPUT; return; }
    for (int i = 2; i < 4; i++) {
      const double prevdet = maxdet;
      int maxpoint = -1, maxnearzero = 0, nearzero;
      maxdet = -1.0;
      for (int m = 0; m < 6; m++) {
        const int p = maxpoints[m];
        bool ins = false;
        for (int t = 0; t < i; t++) ins |= simplex[t] == p;
        if (!ins && p != maxpoint) {
          double det = fabs(qh_detsimplex(S, W.Pr, simplex, i, p, &nearzero));
          if (det > maxdet) { maxdet = det; maxpoint = p; maxnearzero = nearzero; }
        }
      }
      const double targetdet = prevdet * S.MAXwidth;
      const bool falsenarrow = maxdet > 0.0 && maxdet / targetdet < 1.0e-3;
      if (maxpoint < 0 || maxnearzero || falsenarrow) {
        double key = -1.0;
        int idx = 0x7fffffff;
        for (int q = lane; q < n; q += 64) {
          bool skip = false;
          for (int t = 0; t < 6; t++) skip |= maxpoints[t] == q;
          for (int t = 0; t < i; t++) skip |= simplex[t] == q;
          if (skip) continue;
          const double det = fabs(qh_detsimplex(S, W.Pr, simplex, i, q, &nearzero));
          if (det > key || (det == key && q < idx)) { key = det; idx = q; }
        }
        for (int off = 32; off >= 1; off >>= 1) {
          const double ok = __shfl_xor(key, off);
          const int oi = __shfl_xor(idx, off);
          if (ok > key || (ok == key && oi < idx)) { key = ok; idx = oi; }
        }
        if (idx != 0x7fffffff && key > maxdet) { maxdet = key; maxpoint = idx; }
      }
      if (maxpoint < 0) { S.status |= QHS_INPUT; return; }
      simplex[i] = maxpoint;
    }
  }
  // qh_initialvertices (v1..v4 = simplex[0..3]; the set is [v4 v3 v2 v1]), qh_createsimplex
  int vset[4];
  for (int i = 0; i < 4; i++) {
    W.vpt[S.nv] = simplex[i];
    vset[3 - i] = S.nv++;
  }
  int fs[4];
  {
    int top = 1;
    for (int i = 0; i < 4; i++) {
      const int f = qh_newfacet(W, S);
      int m = 0;
      for (int t = 0; t < 4; t++)
        if (t != i) W.fv[3 * f + m++] = vset[t];
      W.fflag[f] = QF_LIVE | (top ? QF_TOP : 0);
      qh_appendfacet(W, S, f);
      fs[i] = f;
      top ^= 1;
    }
    for (int i = 0; i < 4; i++) {
      int m = 0;
      for (int t = 0; t < 4; t++)
        if (t != i) W.fnb[3 * fs[i] + m++] = fs[t];
    }
    S.newfacet_list = S.visible_list = -1;
    S.facet_next = S.facet_list;
    for (int k = 0; k < 3; k++) {
      double c = 0.0;
      for (int t = 0; t < 4; t++) c += W.Pr[3 * (size_t)W.vpt[vset[t]] + k];
      S.interior[k] = c / 4;
    }
    hl_sync();
    // qh_initialhull: orientation from the first facet
    qh_setfacetplane(W, S, S.status, fs[0]);
    hl_sync();
    if (qh_dist(W, S.interior, fs[0]) > S.DISTround)
      for (int i = 0; i < 4; i++) qh_set_top(W, fs[i], !(W.fflag[fs[i]] & QF_TOP));
    hl_sync();
    for (int i = 0; i < 4; i++) qh_setfacetplane(W, S, S.status, fs[i]);
    hl_sync();
    for (int i = 0; i < 4; i++)
      if (W.fflag[fs[i]] & QF_FLIPPED) S.status |= QHS_FLIPPED;
    double minangle = DBL_MAX;
    for (int i = 0; i < 4; i++)
      for (int t = 0; t < 3; t++) {
        const double* a = W.pl + 4 * (size_t)fs[i];
        const double* b = W.pl + 4 * (size_t)W.fnb[3 * fs[i] + t];
        double angle = 0.0;
        for (int k = 0; k < 3; k++) angle += a[k] * b[k];
        if (angle < minangle) minangle = angle;
      }
    if (minangle < -0.99999999) S.status |= QHS_NARROW;
  }
  // qh_partitionall: every point but the simplex, in index order; each facet
  // in list order takes the ones at or beyond distoutside
  int np = 0;
  for (int c = 0; c < n; c += 64) {
    const int q = c + lane;
    const bool ok = q < n && q != simplex[0] && q != simplex[1] && q != simplex[2] && q != simplex[3];
    const unsigned long long b = __ballot(ok);
    if (ok) W.pq[np + __popcll(b & ((1ull << lane) - 1ull))] = q;
    np += __popcll(b);
  }
  hl_sync();
  {
    const double distoutside = fmax(2 * S.MINoutside, S.max_outside);
    for (int f = S.facet_list; f != S.facet_tail; f = qh_next(W, f)) {
      // count first, then emit with the champion rule into a fresh segment
      int cnt = 0;
      const int off = S.sbtop;
      double mx = 0.0;
      int champ = -1, w = 0;
      for (int c = 0; c < np; c += 64) {
        const int pos = c + lane;
        int pid = -1;
        double d = -DBL_MAX;
        if (pos < np) {
          pid = W.pq[pos];
          d = qh_dist(W, W.Pr + 3 * (size_t)pid, f);
        }
        const bool out = pos < np && d >= distoutside;
        const bool keep = pos < np && !out;
        const unsigned long long bk = __ballot(keep);
        hl_sync();
        if (keep) W.pq[w + __popcll(bk & ((1ull << lane) - 1ull))] = pid;
        w += __popcll(bk);
        unsigned long long bo = __ballot(out);
        while (bo) {
          const int l = __ffsll((long long)bo) - 1;
          bo &= bo - 1;
          const int q = __builtin_amdgcn_readlane(pid, l);
          const double dq = hl_rl(d, l);
          if (cnt == 0) {
            champ = q; mx = dq;
          } else if (dq > mx) {
            if (off + cnt - 1 < W.SB && lane == 0) W.sb[off + cnt - 1] = champ;
            champ = q; mx = dq;
          } else {
            if (off + cnt - 1 < W.SB && lane == 0) W.sb[off + cnt - 1] = q;
          }
          cnt++;
        }
        hl_sync();
      }
      if (cnt) {
        if (off + cnt > W.SB) { S.status |= QHS_CAPACITY | QHS_CAP_SB; return; }
        if (lane == 0) W.sb[off + cnt - 1] = champ;
        W.fseg[2 * f] = off;
        W.fseg[2 * f + 1] = cnt;
        W.fdist[f] = mx;
        S.sbtop += cnt;
      }
      np = w;
      hl_sync();
    }
    // the remainder through qh_partitionpoint with findbestnew from the head
    // of the facet list (MERGING): the scan list is the facet list
    if (np > 0) {
      int t = 0;
      for (int f = S.facet_list; f != S.facet_tail; f = qh_next(W, f)) {
        L.newf[t] = f;
        W.fnew[f] = t;
        t++;
      }
      S.nnew = t;
      S.nmov = 0;
      S.findbestnew = 1;
      for (int q = lane; q < np; q += 64) W.pst[q] = S.facet_list;
      hl_sync();
      qh_locate_seq(W, S, L, np, 0, true, lane);
      qh_emit_seq(W, S, L, np, lane);
      for (int f = S.facet_list; f != S.facet_tail; f = qh_next(W, f)) W.fnew[f] = 0x7fffffff;
      S.findbestnew = 0;
      S.nnew = 0;
      S.nmov = 0;
      hl_sync();
    }
  }
  QHT(0);
  if (S.status & (QHS_INPUT | QHS_TOPOLOGY | QHS_CAPACITY)) return;
  // qh_furthestnext
  {
    int best = -1;
    double bd = -DBL_MAX;
    for (int f = S.facet_list; f != S.facet_tail; f = qh_next(W, f))
      if (W.fseg[2 * f + 1] && W.fdist[f] > bd) { best = f; bd = W.fdist[f]; }
    if (best >= 0) {
      qh_removefacet(W, S, best);
      // qh_prependfacet(best, &qh.facet_next)
      const int list = S.facet_next;
      const int pv = qh_prev(W, list);
      W.flink[2 * best] = pv;
      if (pv >= 0) W.flink[2 * pv + 1] = best;
      W.flink[2 * list] = best;
      W.flink[2 * best + 1] = list;
      if (S.facet_list == list) S.facet_list = best;
      if (S.facet_next == list) S.facet_next = best;
    }
  }
  hl_sync();
  // qh_buildhull
  S.facet_next = S.facet_list;
  for (;;) {
    // qh_nextfurthest
    int facet = -1, furthest = -1;
    while ((facet = S.facet_next) != S.facet_tail) {
      const int cnt = W.fseg[2 * facet + 1];
      if (!cnt) {
        S.facet_next = qh_next(W, facet);
        continue;
      }
      furthest = W.sb[W.fseg[2 * facet] + cnt - 1];
      hl_sync();
      W.fseg[2 * facet + 1] = cnt - 1;
      break;
    }
    QHT(1);
    if (furthest < 0) break;
    S.nins++;
    const double* apexp = W.Pr + 3 * (size_t)furthest;
    // qh_findhorizon
    S.epoch++;
    qh_removefacet(W, S, facet);
    qh_appendfacet(W, S, facet);
    W.fflag[facet] |= QF_VISIBLE;
    W.frep[facet] = -1;
    S.visible_list = facet;
    W.fvis[facet] = S.epoch;
    S.nvis = 0;
    L.visf[S.nvis++] = facet;
    hl_sync();
    for (int vi = 0; vi < S.nvis; vi++) {
      const int vis = L.visf[vi];
      for (int k = 0; k < 3; k++) {
        const int nb = W.fnb[3 * vis + k];
        if (W.fvis[nb] == S.epoch) continue;
        W.fvis[nb] = S.epoch;
        const double dist = qh_dist(W, apexp, nb);
        if (dist >= S.MINvisible) {
          qh_removefacet(W, S, nb);
          qh_appendfacet(W, S, nb);
          W.fflag[nb] |= QF_VISIBLE;
          W.frep[nb] = -1;
          if (S.nvis == QH_VISCAP) { S.status |= QHS_CAPACITY | QHS_CAP_VIS; return; }
          if (lane == 0) L.visf[S.nvis] = nb;
          S.nvis++;
        } else if (dist >= -S.MAXcoplanar) {
          S.status |= QHS_COPLANAR;   // Qhull merges a coplanar horizon facet: built on merge-free
        }
        hl_sync();
      }
    }
    QHT(2);
    // qh_makenewfacets -> qh_makenew_simplicial
    S.newfacet_list = S.facet_tail;
    const int apex = S.nv++;
    W.vpt[apex] = furthest;
    S.nnew = 0;
    for (int vi = 0; vi < S.nvis; vi++) {
      const int vis = L.visf[vi];
      int newfacet = -1;
      for (int k = 0; k < 3; k++) {
        const int nb = W.fnb[3 * vis + k];
        if (W.fflag[nb] & QF_VISIBLE) continue;
        int hskip = -1;
        for (int t = 0; t < 3; t++)
          if (W.fnb[3 * nb + t] == vis) hskip = t;
        if (hskip < 0) { S.status |= QHS_TOPOLOGY; return; }
        const int top = (W.fflag[nb] & QF_TOP) ? (hskip & 1) : ((hskip & 1) ^ 1);
        int vs[2], m = 0;
        for (int t = 0; t < 3; t++)
          if (t != hskip) vs[m++] = W.fv[3 * nb + t];
        if (S.nnew == QH_NEWCAP) { S.status |= QHS_CAPACITY | QHS_CAP_NEW; return; }
        const int nf = qh_newfacet(W, S);
        if (S.status & QHS_CAPACITY) return;
        W.fv[3 * nf] = apex;
        W.fv[3 * nf + 1] = vs[0];
        W.fv[3 * nf + 2] = vs[1];
        W.fflag[nf] = QF_NEW | QF_LIVE | (top ? QF_TOP : 0);
        W.fnb[3 * nf] = nb;
        qh_appendfacet(W, S, nf);
        W.fnb[3 * nb + hskip] = nf;
        W.fnew[nf] = S.nnew;
        if (lane == 0) L.newf[S.nnew] = nf;
        S.nnew++;
        newfacet = nf;
        hl_sync();
      }
      W.frep[vis] = newfacet;
    }
    hl_sync();
    QHT(3);
    // qh_matchnewfacets (nb[1] shares {apex, v2}, nb[2] shares {apex, v1}),
    // qh_makenewplanes, qh_checkzero: one new facet per lane
    int ls = 0;
    for (int t = lane; t < S.nnew; t += 64) {
      const int f = L.newf[t];
      for (int k = 1; k < 3; k++) {
        const int w = W.fv[3 * f + 3 - k];
        int found = -1, cnt = 0;
        for (int u = 0; u < S.nnew; u++) {
          const int g = L.newf[u];
          if (g != f && (W.fv[3 * g + 1] == w || W.fv[3 * g + 2] == w)) { found = g; cnt++; }
        }
        if (cnt != 1) ls |= QHS_TOPOLOGY;
        W.fnb[3 * f + k] = found;
      }
      qh_setfacetplane(W, S, ls, f);
      if (W.fflag[f] & QF_FLIPPED) ls |= QHS_FLIPPED;
    }
    hl_sync();
    if (!(qh_wave_or(ls) & QHS_FLIPPED)) {
      for (int t = lane; t < S.nnew; t += 64) {
        const int f = L.newf[t];
        for (int k = 1; k < 3; k++) {
          const int nb = W.fnb[3 * f + k];
          if (nb < 0) continue;
          const double d = qh_dist(W, W.Pr + 3 * (size_t)W.vpt[W.fv[3 * f + k]], nb);
          if (d >= -2 * S.DISTround) ls |= QHS_NONCONVEX;
        }
        const int hz = W.fnb[3 * f];
        for (int k = 0; k < 3; k++) {
          const int v = W.fv[3 * hz + k];
          if (v != W.fv[3 * f] && v != W.fv[3 * f + 1] && v != W.fv[3 * f + 2]) {
            const double d = qh_dist(W, W.Pr + 3 * (size_t)W.vpt[v], f);
            if (d >= -2 * S.DISTround) ls |= QHS_NONCONVEX;
            break;
          }
        }
      }
    }
    S.status |= qh_wave_or(ls);
    QHT(4);
    if (S.status & (QHS_TOPOLOGY | QHS_CAPACITY)) return;
    // qh_partitionvisible: the visible facets' outside sets, in order
    {
      int np2 = 0;
      for (int vi = 0; vi < S.nvis; vi++) {
        const int vis = L.visf[vi];
        const int cnt = W.fseg[2 * vis + 1];
        if (!cnt) continue;
        int start = W.frep[vis];
        while (start >= 0 && (W.fflag[start] & QF_VISIBLE)) start = W.frep[start];
        if (start < 0) start = L.newf[0];
        const int off = W.fseg[2 * vis];
        for (int t = lane; t < cnt; t += 64) {
          W.pq[np2 + t] = W.sb[off + t];
          W.pst[np2 + t] = start;
        }
        np2 += cnt;
      }
      hl_sync();
      S.findbestnew = 0;
      S.notsharp = 0;
      S.nmov = 0;
      const int sharp = qh_sharpnewfacets(W, S, L);
      QHT(5);
      if (np2) {
        qh_locate_seq(W, S, L, np2, sharp, false, lane);
        QHT(6);
        qh_emit_seq(W, S, L, np2, lane);
        QHT(7);
      }
    }
    // deleted vertices (a visible facet's vertex on no new facet) close to a
    // new facet: Qhull's qh_partitioncoplanar would act (not restated)
    {
      int lsd = 0;
      for (int t = lane; t < 3 * S.nvis; t += 64) {
        const int v = W.fv[3 * L.visf[t / 3] + t % 3];
        bool onnew = false;
        for (int u = 0; u < S.nnew && !onnew; u++) {
          const int g = L.newf[u];
          onnew = W.fv[3 * g + 1] == v || W.fv[3 * g + 2] == v;
        }
        if (!onnew) {
          double d;
          int iso;
          qh_findbestnew(W, S, L, W.Pr + 3 * (size_t)W.vpt[v], L.newf[0], &d, 1, &iso, lsd);
          if (d >= -S.MAXcoplanar) lsd |= QHS_COPLANAR;
        }
      }
      S.status |= qh_wave_or(lsd);
    }
    QHT(8);
    if (S.status & QHS_CAPACITY) return;
    S.findbestnew = 0;
    S.notsharp = 0;
    // qh_deletevisible, qh_resetlists
    for (int vi = 0; vi < S.nvis; vi++) {
      const int vis = L.visf[vi];
      qh_removefacet(W, S, vis);
      W.fflag[vis] = 0;
      if (lane == 0) W.fstack[S.nfree] = vis;
      S.nfree++;
    }
    for (int t = lane; t < S.nnew; t += 64) {
      const int f = L.newf[t];
      W.fflag[f] &= ~QF_NEW;
      W.fnew[f] = 0x7fffffff;
    }
    S.newfacet_list = -1;
    S.visible_list = -1;
    S.nnew = 0;
    S.nmov = 0;
    hl_sync();
    QHT(9);
  }
}

// ---- the reference's selection (LQRO:925-968) over the finished hull ----
// convexHull measures facet f as |n_f . (vrel - P_f)| with n_f the plane as
// qconvex prints it and operator>> reads it back (16 significant digits,
// LQRO:889-899; lqro_dec16.hpp) and P_f the first Fv vertex at full
// precision (LQRO:925-939).  qsel_dist: that distance with Qhull's own
// plane, and a bound b on its change under the read-back (the decimal
// rounding <= 6.2e-16 |n_k| per coefficient, both evaluations' rounding
// <= 3.4e-16 of sum |n_k| |vrel_k - P_k| each; b is 3x their sum);
// qsel_dist16: the distance with the read-back plane, exactly the reference's
// expression.
__device__ __forceinline__ double qsel_dist(const double* q, const double* P, const double* vrel, double* b) {
  const double a0 = vrel[0] - P[0], a1 = vrel[1] - P[1], a2 = vrel[2] - P[2];
  *b = 4e-15 * (fabs(q[0] * a0) + fabs(q[1] * a1) + fabs(q[2] * a2)) + 1e-300;
  return fabs(q[0] * a0 + q[1] * a1 + q[2] * a2);
}
__device__ inline double qsel_dist16(const double* q, const double* P, const double* vrel, double* n16) {
  bool e0, e1, e2;
  n16[0] = dec16(q[0], &e0);
  n16[1] = dec16(q[1], &e1);
  n16[2] = dec16(q[2], &e2);
  return fabs(n16[0] * (vrel[0] - P[0]) + n16[1] * (vrel[1] - P[1]) + n16[2] * (vrel[2] - P[2]));
}

// LQRO_REC_QHMERGE_WIN, as q3_merge_suspect (lqro_qhull3.hpp): a facet
// within 1e-6 of the winning distance with another hull vertex within
// 1e-9 (|coord|max + 1) of its plane; wave-uniform
__device__ inline bool qh_merge_suspect(const QhW& W, const QhS& S, int lane, const double* vrel, double best) {
  const double T = -LQRO_QHMERGE_K * S.DISTround;   // (lqro_qhull3.hpp q3_merge_suspect)
  bool sus = false;
  for (int f0 = 1; f0 < S.nalloc; f0 += 64) {
    const int f = f0 + lane;
    bool con = false;
    if (f < S.nalloc && (W.fflag[f] & QF_LIVE)) {
      const double* q = W.pl + 4 * (size_t)f;
      const double* P = W.Pf + 3 * (size_t)W.vpt[W.fv[3 * f]];
      con = fabs(q[0] * (vrel[0] - P[0]) + q[1] * (vrel[1] - P[1]) + q[2] * (vrel[2] - P[2])) <= best + 1e-6 ||
            f == S.facet_list;
    }
    unsigned long long m = __ballot(con);
    while (m) {
      const int src = __ffsll((long long)m) - 1;
      m &= m - 1;
      const int fc = __shfl(f, src);
      const double* qc = W.pl + 4 * (size_t)fc;
      const int a = W.vpt[W.fv[3 * fc]], b = W.vpt[W.fv[3 * fc + 1]], c = W.vpt[W.fv[3 * fc + 2]];
      for (int g = 1 + lane; g < S.nalloc; g += 64) {
        if (!(W.fflag[g] & QF_LIVE)) continue;
        for (int t = 0; t < 3; t++) {
          const int id = W.vpt[W.fv[3 * g + t]];
          if (id == a || id == b || id == c) continue;
          const double* p = W.Pr + 3 * (size_t)id;
          if (qc[3] + p[0] * qc[0] + p[1] * qc[1] + p[2] * qc[2] >= T) sus = true;
        }
      }
    }
  }
  return __ballot(sus) != 0;
}

// Facets in Qhull's order, each measured from its first Fv vertex (its
// newest) with the read-back plane, strict '<': the minimum, the earliest
// facet in list order on a tie (a walk of the list, only then).  Facet 0 (the
// list head) winning leaves `normal` to the loop-carried value: the plane
// waits for k_stale.  Two passes: every facet at full precision for the
// bound on the minimum, then the read-back planes of the facets within it.
__device__ inline void qh_select(const HullArgs& A, const QhW& W, const QhS& S, int lane, const double* xi,
                                 const double* vrel, int slot) {
  const bool fail = (S.status & (QHS_INPUT | QHS_TOPOLOGY | QHS_CAPACITY)) != 0;
  double ub = INFINITY;
  int nfac = 0;
  if (!fail) {
    for (int f = 1 + lane; f < S.nalloc; f += 64) {
      if (!(W.fflag[f] & QF_LIVE)) continue;
      nfac++;
      const double* q = W.pl + 4 * (size_t)f;
      const double* P = W.Pf + 3 * (size_t)W.vpt[W.fv[3 * f]];
      double b;
      const double d = qsel_dist(q, P, vrel, &b);
      ub = fmin(ub, d + b);
    }
  }
  for (int off = 32; off >= 1; off >>= 1) {
    nfac += __shfl_xor(nfac, off);
    ub = fmin(ub, __shfl_xor(ub, off));
  }
  double best = INFINITY, bn[3] = {0.0, 0.0, 0.0};
  int bf = 0x7fffffff;
  if (!fail) {
    for (int f = 1 + lane; f < S.nalloc; f += 64) {
      if (!(W.fflag[f] & QF_LIVE)) continue;
      const double* q = W.pl + 4 * (size_t)f;
      const double* P = W.Pf + 3 * (size_t)W.vpt[W.fv[3 * f]];
      double b, n16[3];
      if (qsel_dist(q, P, vrel, &b) - b > ub) continue;
      const double d = qsel_dist16(q, P, vrel, n16);
      if (d < best || (d == best && f < bf)) { best = d; bf = f; bn[0] = n16[0]; bn[1] = n16[1]; bn[2] = n16[2]; }
    }
  }
  int ties = 0;
  for (int off = 32; off >= 1; off >>= 1) {
    const double ob = __shfl_xor(best, off);
    const int of = __shfl_xor(bf, off);
    const double o0 = __shfl_xor(bn[0], off), o1 = __shfl_xor(bn[1], off), o2 = __shfl_xor(bn[2], off);
    if (ob < best || (ob == best && of < bf)) { best = ob; bf = of; bn[0] = o0; bn[1] = o1; bn[2] = o2; }
  }
  if (!fail) {
    for (int f = 1 + lane; f < S.nalloc; f += 64) {
      if (!(W.fflag[f] & QF_LIVE)) continue;
      const double* q = W.pl + 4 * (size_t)f;
      const double* P = W.Pf + 3 * (size_t)W.vpt[W.fv[3 * f]];
      double b, n16[3];
      if (qsel_dist(q, P, vrel, &b) - b > ub) continue;
      ties += qsel_dist16(q, P, vrel, n16) == best;
    }
    for (int off = 32; off >= 1; off >>= 1) ties += __shfl_xor(ties, off);
    if (ties > 1)   // the first in Qhull's order
      for (int f = S.facet_list; f != S.facet_tail; f = qh_next(W, f)) {
        const double* q = W.pl + 4 * (size_t)f;
        const double* P = W.Pf + 3 * (size_t)W.vpt[W.fv[3 * f]];
        double b, n16[3];
        if (qsel_dist(q, P, vrel, &b) - b > ub) continue;
        if (qsel_dist16(q, P, vrel, n16) == best) { bf = f; bn[0] = n16[0]; bn[1] = n16[1]; bn[2] = n16[2]; break; }
      }
  }
  const bool ok = !fail && nfac > 0 && bf != 0x7fffffff;
  const bool stale = ok && bf == S.facet_list;
  const bool merged = (S.status & (QHS_COPLANAR | QHS_NONCONVEX | QHS_FLIPPED | QHS_NARROW | QHS_SINGULAR)) != 0;
  const bool mwin = ok && merged && qh_merge_suspect(W, S, lane, vrel, best);
  if (lane == 0) {
    float* pl = A.planes + (size_t)slot * 8;
    double* qn = A.qnrm + (size_t)slot * 4;
    double nrm[3] = {0.0, 0.0, 0.0};
    if (ok && !stale) {
      nrm[0] = bn[0]; nrm[1] = bn[1]; nrm[2] = bn[2];
      const double dh = best * 0.5;                      // :1416
      const double mult = 1.0;                           // :1213
      pl[0] = (float)(xi[3] + mult * dh * nrm[0]);
      pl[1] = (float)(xi[4] + mult * dh * nrm[1]);
      pl[2] = (float)(xi[5] + mult * dh * nrm[2]);
      pl[3] = (float)nrm[0]; pl[4] = (float)nrm[1]; pl[5] = (float)nrm[2];
      pl[6] = __int_as_float(1);
      qn[0] = nrm[0]; qn[1] = nrm[1]; qn[2] = nrm[2]; qn[3] = best;
      atomicAdd(&A.stats[3], 1ull);
    } else if (stale) {
      pl[6] = __int_as_float(3);                         // pending: the loop-carried normal (k_stale)
      qn[0] = qn[1] = qn[2] = 0.0; qn[3] = best;
      const int k = atomicAdd(A.qstale_count, 1);
      if (k < A.qstale_cap) A.qstale[k] = slot;
      atomicAdd(&A.stats[3], 1ull);
    } else {
      pl[6] = __int_as_float(0);
      hull_fail_note(A.stats, slot);
    }
    if (ok && merged) atomicAdd(&A.stats[LQRO_ST_MERGED], 1ull);
    if (mwin) qhmerge_note(A.stats, slot);
    if (A.recs) {
      lqro_pair_record& rec = A.recs[slot];
      rec.flags |= ok ? LQRO_REC_HULL : LQRO_REC_HULLFAIL;
      if (stale) rec.flags |= LQRO_REC_STALE;
      if (merged) rec.flags |= LQRO_REC_QHMERGE;
      if (mwin) rec.flags |= LQRO_REC_QHMERGE_WIN;
      rec.n_facets = ok ? nfac : -(S.status & 0xffff) - 1;   // a failure: -(build status bits) - 1
      if (ok) {
        for (int k = 0; k < 3; k++) rec.facet[k] = W.vpt[W.fv[3 * bf + k]];
        rec.dist = best;
        for (int q = 0; q < 3; ++q) {
          rec.normal[q] = nrm[q];
          rec.plane_point[q] = stale ? 0.0f : pl[q];
          rec.plane_normal[q] = stale ? 0.0f : pl[3 + q];
        }
      }
    }
    hull_row_done(A, slot, stale, false);   // k_qhull_big leaves the LP to the tail
  }
  hl_sync();
}

// the wave that builds (lane = its lane): the scratch's visit stamps are
// this kernel's, or reset (zero stamps and counters = a fresh scratch)
__device__ inline void qh_claim_scratch(const QhW& W, unsigned* owner, int lane) {
  if (*owner == QW_OWNER_QH) return;
  for (int q = lane; q < (QH_NEWCAP - 256) * 64; q += 64) W.vstamp[q] = 0u;
  W.vctr[lane] = 0u;
  if (lane == 0) *owner = QW_OWNER_QH;
}

// one inside-hull pair per wave, persistent over the hull queue (k_qhull_big:
// the retry queue k_qhull's caps fill, or the main queue under LQRO_QHULL_BIG)
__device__ inline void qh_body(const HullArgs& A, QhL& L, bool retryq) {
  const int lane = threadIdx.x & 63;
  const int HNP = A.H * A.NP;
  const QhW W = qh_worker(A.qscratch + (size_t)(A.block_base + blockIdx.x) * A.qstride, HNP);
  for (;;) {
    const int slot = hull_take_job(A, L, retryq);
    if (slot < 0) break;
    const unsigned long long tjob = __builtin_amdgcn_s_memrealtime();   // (lqro_get_hull_builds)
    const int lrow = slot / A.npr, jj = A.nbr_list ? A.nbr_list[slot] : slot % A.npr;
    const int i = A.row_begin + lrow * A.row_stride;
    const int j = jj < i ? jj : jj + 1;
    const double* xi = A.x + (size_t)i * A.X;
    const double* xj = A.x + (size_t)j * A.X;
    const double* Ti = A.T + (A.per_agent ? (size_t)i * A.H * 9 : 0);
    const double* Ni = A.NCF + (A.per_agent ? (size_t)i * A.H * 3 * A.X : 0);
    const double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};
    const int n = hull_points(A, L, Ti, Ni, xi, xj, vrel, W.Pr, W.Pf);
    qh_claim_scratch(W, qw_owner(A.qscratch + (size_t)(A.block_base + blockIdx.x) * A.qstride, A.qstride), lane);
    QhS S;
#ifdef LQRO_QHULL_PROFILE
    for (int k = 0; k < 12; k++) S.tph[k] = 0;
#endif
    S.status = 0;
    S.nalloc = 1;
    S.nins = 0;
    S.facet_list = S.facet_tail = 0;
    if (L.fail || n < 4) S.status = QHS_INPUT;
    else qh_build(W, S, L, n, lane);
    hl_sync();
#ifdef LQRO_QHULL_PROFILE
    unsigned long long tq_ = __builtin_amdgcn_s_memtime();
#endif
    qh_select(A, W, S, lane, xi, vrel, slot);
    if (lane == 0) hull_build_note(A, slot, 1, tjob, n, S.nins, S.nalloc - 1);
#ifdef LQRO_QHULL_PROFILE
    S.tph[10] = __builtin_amdgcn_s_memtime() - tq_;
    S.tph[11] = 1;
    if (A.prof && lane == 0)
      for (int k = 0; k < 12; k++) atomicAdd(&A.prof[k], S.tph[k]);
#endif
    if (A.ext_nf && lane == 0) *A.ext_nf = S.status;   // test hook: the build's status bits
    if (A.ext_facets && lane == 0) {                     // test hook: the facet list, Fv order
      int k = 0;
      for (int f = S.facet_list; f != S.facet_tail && k < A.ext_max; f = qh_next(W, f), k++)
        for (int t = 0; t < 3; t++) A.ext_facets[3 * k + t] = W.vpt[W.fv[3 * f + t]];
      if (k < A.ext_max) A.ext_facets[3 * k] = -1;
    }
  }
}

// k_stale: a pair whose facet 0 won keeps normalVector from the last pair
// before it (in (i, j) order) with more than min_reach points: walking back
// over the slots — no plane: skipped; another facet-0 pair (its normal slot
// is 0, 0, 0 — a unit normal never is): passed — to the first normal
// written, or, before the context's first slot, the carry entering the step
// (carry[0..2]).  The entry after the list leaves carry[3..5] for the next
// step: the normal the context's last eligible pair leaves.
__device__ __forceinline__ bool qh_slot_normal(const float* planes, const double* qnrm, long s) {
  const int fl = __float_as_int(planes[(size_t)s * 8 + 6]);
  if (fl != 1 && fl != 3) return false;
  const double* q = qnrm + (size_t)s * 4;
  return !(q[0] == 0.0 && q[1] == 0.0 && q[2] == 0.0);
}

#ifdef LQRO_HULL_TU   // the kernels: defined once, in lqro_kern_hull.hip
__global__ void __launch_bounds__(64) k_stale(float* planes, const double* qnrm, const int* list, const int* count,
                                              int cap, const double* x, int X, int npr, int row_begin,
                                              int row_stride, double* carry, lqro_pair_record* recs, long nslots) {
  const int lane = threadIdx.x & 63;
  const int n = min(*count, cap);
  for (int e = blockIdx.x; e <= n; e += gridDim.x) {
    const bool is_carry = e == n;
    const long s0 = is_carry ? nslots : (long)list[e];
    long found = -1;
    for (long b = s0 - 1; b >= 0 && found < 0; b -= 64) {
      const long s = b - lane;
      const bool hit = s >= 0 && qh_slot_normal(planes, qnrm, s);
      const unsigned long long m = __ballot(hit);
      if (m) found = b - (__ffsll((long long)m) - 1);
    }
    double nrm[3];
    for (int k = 0; k < 3; k++) nrm[k] = found >= 0 ? qnrm[(size_t)found * 4 + k] : carry[k];
    if (lane != 0) continue;
    if (is_carry) {
      for (int k = 0; k < 3; k++) carry[3 + k] = nrm[k];
      continue;
    }
    const long slot = s0;
    const int lrow = (int)(slot / npr);
    const int i = row_begin + lrow * row_stride;
    const double* xi = x + (size_t)i * X;
    const double dh = qnrm[(size_t)slot * 4 + 3] * 0.5;   // :1416
    const double mult = 1.0;                              // :1213
    float* pl = planes + (size_t)slot * 8;
    pl[0] = (float)(xi[3] + mult * dh * nrm[0]);
    pl[1] = (float)(xi[4] + mult * dh * nrm[1]);
    pl[2] = (float)(xi[5] + mult * dh * nrm[2]);
    pl[3] = (float)nrm[0]; pl[4] = (float)nrm[1]; pl[5] = (float)nrm[2];
    pl[7] = 0.0f;
    __hip_atomic_store(reinterpret_cast<int*>(pl + 6), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (recs) {
      lqro_pair_record& rec = recs[slot];
      for (int q = 0; q < 3; ++q) {
        rec.normal[q] = nrm[q];
        rec.plane_point[q] = pl[q];
        rec.plane_normal[q] = pl[3 + q];
      }
    }
  }
}

// Row shards (lqro_step_device_begin / _end): the loop-carried normal
// crosses the shard boundaries.  k_rowlast leaves, per own row, the normal of
// its last pair with one (rowtab[4 i + 0..2], rowtab[4 i + 3] = 1; 0 0 0 0
// for none, or without Qhull order: planes == nullptr); the caller gathers
// every rank's rows.  k_stale_rows then resolves a facet-0 pair from its own
// row's earlier slots, else the last row before it (any rank) with a normal,
// else the carry entering the step — the reference's (t, i, j) order over
// the whole swarm — and leaves the swarm's last normal in carry[3..5].
__global__ void __launch_bounds__(64) k_rowlast(const float* planes, const double* qnrm, int npr, int nrows,
                                                int row_begin, int row_stride, double* rowtab) {
  const int lane = threadIdx.x & 63;
  for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
    const long s_lo = (long)r * npr;
    long found = -1;
    if (planes)
      for (long b = s_lo + npr - 1; b >= s_lo && found < 0; b -= 64) {
        const long sl = b - lane;
        const bool hit = sl >= s_lo && qh_slot_normal(planes, qnrm, sl);
        const unsigned long long m = __ballot(hit);
        if (m) found = b - (__ffsll((long long)m) - 1);
      }
    if (lane == 0) {
      double* o = rowtab + 4 * ((size_t)row_begin + (size_t)r * row_stride);
      for (int k = 0; k < 3; k++) o[k] = found >= 0 ? qnrm[(size_t)found * 4 + k] : 0.0;
      o[3] = found >= 0 ? 1.0 : 0.0;
    }
  }
}

// the last row before `i` (agent order) with a normal: its index, or -1
__device__ __forceinline__ int qh_row_before(const double* rowtab, int i) {
  const int lane = threadIdx.x & 63;
  for (int b = i - 1; b >= 0; b -= 64) {
    const int r = b - lane;
    const bool hit = r >= 0 && rowtab[4 * (size_t)r + 3] != 0.0;
    const unsigned long long m = __ballot(hit);
    if (m) return b - (__ffsll((long long)m) - 1);
  }
  return -1;
}

__global__ void __launch_bounds__(64) k_stale_rows(float* planes, const double* qnrm, const int* list,
                                                   const int* count, int cap, const double* x, int X, int npr,
                                                   int row_begin, int row_stride, const double* rowtab, int N,
                                                   double* carry, lqro_pair_record* recs) {
  const int lane = threadIdx.x & 63;
  const int n = min(*count, cap);
  for (int e = blockIdx.x; e <= n; e += gridDim.x) {
    double nrm[3];
    if (e == n) {   // the normal the swarm's last eligible pair leaves
      const int r = qh_row_before(rowtab, N);
      for (int k = 0; k < 3; k++) nrm[k] = r >= 0 ? rowtab[4 * (size_t)r + k] : carry[k];
      if (lane == 0)
        for (int k = 0; k < 3; k++) carry[3 + k] = nrm[k];
      continue;
    }
    const long s0 = (long)list[e];
    const int lrow = (int)(s0 / npr);
    const long s_lo = (long)lrow * npr;
    const int i = row_begin + lrow * row_stride;
    long found = -1;
    for (long b = s0 - 1; b >= s_lo && found < 0; b -= 64) {
      const long sl = b - lane;
      const bool hit = sl >= s_lo && qh_slot_normal(planes, qnrm, sl);
      const unsigned long long m = __ballot(hit);
      if (m) found = b - (__ffsll((long long)m) - 1);
    }
    if (found >= 0) {
      for (int k = 0; k < 3; k++) nrm[k] = qnrm[(size_t)found * 4 + k];
    } else {
      const int r = qh_row_before(rowtab, i);
      for (int k = 0; k < 3; k++) nrm[k] = r >= 0 ? rowtab[4 * (size_t)r + k] : carry[k];
    }
    if (lane != 0) continue;
    const double* xi = x + (size_t)i * X;
    const double dh = qnrm[(size_t)s0 * 4 + 3] * 0.5;   // :1416
    const double mult = 1.0;                            // :1213
    float* pl = planes + (size_t)s0 * 8;
    pl[0] = (float)(xi[3] + mult * dh * nrm[0]);
    pl[1] = (float)(xi[4] + mult * dh * nrm[1]);
    pl[2] = (float)(xi[5] + mult * dh * nrm[2]);
    pl[3] = (float)nrm[0]; pl[4] = (float)nrm[1]; pl[5] = (float)nrm[2];
    pl[7] = 0.0f;
    __hip_atomic_store(reinterpret_cast<int*>(pl + 6), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (recs) {
      lqro_pair_record& rec = recs[s0];
      for (int q = 0; q < 3; ++q) {
        rec.normal[q] = nrm[q];
        rec.plane_point[q] = pl[q];
        rec.plane_normal[q] = pl[3 + q];
      }
    }
  }
}

#endif  // LQRO_HULL_TU

}  // namespace lqro
