// lqro_qhull2.hpp — k_qhull's fast build: the same restatement of Qhull
// 2019.1's build as lqro_qhull.hpp (which stays as k_qhull_big, the
// fallback for hulls beyond this variant's per-insertion caps), laid out for
// the GPU's memory latency instead of as a transcription:
//
//  * a facet is one 64-byte record (plane, neighbours, flags, vertices), so
//    visiting it costs one round trip instead of one per field;
//  * no linked facet list: Qhull's list order is the order facets were
//    appended (qh_appendfacet), so each facet carries a key — its position in
//    that order (0 for the facet qh_furthestnext prepends, a fresh key when
//    qh_partitionpoint moves an old facet behind the new ones) — and
//    qh_nextfurthest's cursor becomes a queue of the facets that received
//    outside points, in key order;
//  * qh_findhorizon's breadth-first search runs a level at a time over the
//    lanes (the same visiting order: a facet is taken by the first visible
//    facet in queue order that reaches it);
//  * qh_makenew_simplicial runs one horizon ridge per lane (creation order =
//    the ridges in visible-list order), new facets reuse the visible facets'
//    slots, and the new facets' planes and neighbours are cached in LDS for
//    the partition that follows.
#pragma once
#include "lqro_qhull.hpp"

namespace lqro {

#define Q2_NEWCAP 128     // new facets of one insertion (more: the pair goes to k_qhull_big)
#define Q2_VISCAP 128     // visible facets of one insertion
#define Q2_MOVCAP 16
#define Q2_HZCAP 24       // facets one point's horizon walk visits
#define Q2_COPCAP 8

struct QFr {              // a facet, 64 B
  double n[3], off;
  int nb[3];
  int flags;
  int v[3];
  int aux;                // while new: its index among the new facets
};

struct Q2W {
  double* Pr;
  double* Pf;
  QFr* F;                 // FC records
  int* seg;               // 2 FC: outside set offset, count
  double* fdist;          // FC
  unsigned* key;          // FC: position in Qhull's facet list
  int* vpt;               // HNP + 8
  int* sb;                // SB outside-set entries
  int* pq; int* pst; int* pdst; double* pdd;   // partition sequence (HNP)
  int* fq; unsigned* fqk; // queue of facets with outside points (QC)
  int* fstack;            // FC free slots
  int FC, SB, HNP, QC;
};

__host__ __device__ inline size_t q2_worker_bytes(int HNP) {
  const size_t FC = 2 * (size_t)HNP + Q2_NEWCAP + 16, SB = (size_t)QH_SBMULT * HNP, QC = 4 * (size_t)HNP + 64;
  return 8 * (7 * (size_t)HNP + FC) + 64 * FC + 4 * (2 * FC + FC + FC + (size_t)HNP + 8 + SB + 3 * (size_t)HNP) +
         8 * QC + 512;
}

__device__ inline Q2W q2_worker(char* base, int HNP) {
  Q2W W;
  W.HNP = HNP;
  W.FC = 2 * HNP + Q2_NEWCAP + 16;
  W.SB = QH_SBMULT * HNP;
  W.QC = 4 * HNP + 64;
  char* p = base;
  auto take = [&](size_t bytes) { char* r = p; p += (bytes + 63) & ~(size_t)63; return r; };
  W.F = reinterpret_cast<QFr*>(take(64 * (size_t)W.FC));
  W.Pr = reinterpret_cast<double*>(take(24 * (size_t)HNP));
  W.Pf = reinterpret_cast<double*>(take(24 * (size_t)HNP));
  W.pdd = reinterpret_cast<double*>(take(8 * (size_t)HNP));
  W.fdist = reinterpret_cast<double*>(take(8 * (size_t)W.FC));
  W.seg = reinterpret_cast<int*>(take(8 * (size_t)W.FC));
  W.key = reinterpret_cast<unsigned*>(take(4 * (size_t)W.FC));
  W.fstack = reinterpret_cast<int*>(take(4 * (size_t)W.FC));
  W.vpt = reinterpret_cast<int*>(take(4 * ((size_t)HNP + 8)));
  W.pq = reinterpret_cast<int*>(take(4 * (size_t)HNP));
  W.pst = reinterpret_cast<int*>(take(4 * (size_t)HNP));
  W.pdst = reinterpret_cast<int*>(take(4 * (size_t)HNP));
  W.fq = reinterpret_cast<int*>(take(4 * (size_t)W.QC));
  W.fqk = reinterpret_cast<unsigned*>(take(4 * (size_t)W.QC));
  W.sb = reinterpret_cast<int*>(take(4 * (size_t)W.SB));
  return W;
}

struct Q2L {
  // hull_points / hull_take_job interface
  int n, fail, job, slot;
  double eps;
  double tr[3 * 128];
  double rk[1];
  int ri[1];
  int scan[1];
  // the insertion: visible facets (qh_findhorizon order) with what the cone
  // and the partition still need once their slots are reused
  int visf[Q2_VISCAP];
  int vsoff[Q2_VISCAP], vscnt[Q2_VISCAP], vinc[Q2_VISCAP];
  int vvert[3 * Q2_VISCAP];
  int repl[Q2_VISCAP];            // qh_getreplacement: new-facet index
  // the new facets, creation order: slot, vertices, neighbours (nb0 = the
  // horizon facet's slot; nb1/nb2 as new-facet indices), plane, flags
  int nslot[Q2_NEWCAP];
  int nv[3 * Q2_NEWCAP];
  int nhz[Q2_NEWCAP], nhskip[Q2_NEWCAP], nopp[Q2_NEWCAP];   // horizon slot, its ridge index, its other vertex
  int nn1[Q2_NEWCAP], nn2[Q2_NEWCAP];
  double npl[4 * Q2_NEWCAP];
  int nflag[Q2_NEWCAP];
  int movf[Q2_MOVCAP];            // old facets moved behind the new ones (scan order)
  // partition destinations (new facets, then old facets receiving points)
  int dfac[Q2_NEWCAP + Q2_MOVCAP], dcnt[Q2_NEWCAP + Q2_MOVCAP], doff[Q2_NEWCAP + Q2_MOVCAP];
  int dchamp[Q2_NEWCAP + Q2_MOVCAP], pcnt[Q2_NEWCAP + Q2_MOVCAP];
  double dmax[Q2_NEWCAP + Q2_MOVCAP];
  int oldf[Q2_MOVCAP];
  int cop[Q2_COPCAP * 64];        // the horizon walks' coplanar facet sets, per lane
};

struct Q2S {
  int nalloc, nfree, nv, sbtop, status, qhead, qtail;
  unsigned keyc;
  int nnew, nvis, nmov, nold;
  int findbestnew, notsharp;
  double MAXabs_coord, MAXsumcoord, MAXwidth, NEARzero[3];
  double DISTround, MINvisible, MAXcoplanar, MINoutside, MINdenom, MINdenom_2, max_outside;
  double interior[3];
  unsigned long long tph[12];
};

#ifdef LQRO_QHULL_PROFILE
#define Q2T(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); S.tph[k] += t_ - tq_; tq_ = t_; } while (0)
#else
#define Q2T(k) do {} while (0)
#endif

// the adapter that lets the verified plane code (qh_plane_gauss) read Q2S
__device__ __forceinline__ QhS q2_as_qhs(const Q2S& S) {
  QhS T;
  T.DISTround = S.DISTround;
  T.MINdenom = S.MINdenom;
  T.MINdenom_2 = S.MINdenom_2;
  for (int k = 0; k < 3; k++) T.NEARzero[k] = S.NEARzero[k];
  return T;
}

// qh_setfacetplane for a facet with vertex points r0, r1, r2 (its vertex order)
__device__ inline void q2_plane(const Q2S& S, int& status, const double* r0, const double* r1, const double* r2,
                                int top, double* q, bool* flipped) {
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
  if (d2 > S.DISTround || d2 < -S.DISTround || d1 > S.DISTround || d1 < -S.DISTround) {
    const QhS T = q2_as_qhs(S);
    qh_plane_gauss(T, status, r0, r1, r2, top, n, &off);
  }
  q[0] = n[0]; q[1] = n[1]; q[2] = n[2]; q[3] = off;
  const double di = off + S.interior[0] * n[0] + S.interior[1] * n[1] + S.interior[2] * n[2];
  *flipped = di >= -S.DISTround;
}

__device__ __forceinline__ double q2_distq(const double* q, const double* p) {   // qh_distplane
  return q[3] + p[0] * q[0] + p[1] * q[1] + p[2] * q[2];
}

// a facet's plane, flags and neighbours: one record
__device__ __forceinline__ void q2_getpl(const Q2W& W, int f, double* q, int* flags, int* nb) {
  const QFr& r = W.F[f];
  q[0] = r.n[0]; q[1] = r.n[1]; q[2] = r.n[2]; q[3] = r.off;
  *flags = r.flags;
  nb[0] = r.nb[0]; nb[1] = r.nb[1]; nb[2] = r.nb[2];
}

// ---- point location, per lane ----
__device__ inline int q2_findbesthorizon(const Q2W& W, const Q2S& S, const Q2L& L, const double* p, int startfacet,
                                         double* bestdist, int& lstatus) {
  int bestfacet = startfacet;
  const double searchdist = S.max_outside + 2 * S.DISTround + fmax(S.MINvisible, S.MAXcoplanar);
  double minsearch = *bestdist - searchdist;
  int vis[Q2_HZCAP];
  int nvis = 0;
  int* cop = const_cast<int*>(L.cop) + (threadIdx.x & 63);   // qh.coplanarfacetset, [k][lane] in LDS
  int ncop = 0;
  int nextfacet = -1, nextnb[3] = {-1, -1, -1};
  vis[nvis++] = startfacet;
  int facet = startfacet;
  int cur[3];
  {
    const QFr& fr = W.F[facet];
    cur[0] = fr.nb[0]; cur[1] = fr.nb[1]; cur[2] = fr.nb[2];
  }
  for (;;) {
    // the three neighbours' records in one round trip; the one the walk
    // moves to brings its own neighbours along
    double q[3][4];
    int fl[3], nn[3][3];
    for (int k = 0; k < 3; k++) q2_getpl(W, cur[k], q[k], &fl[k], nn[k]);
    for (int k = 0; k < 3; k++) {
      const int nb = cur[k];
      bool seen = false;
      for (int t = 0; t < nvis; t++) seen |= vis[t] == nb;
      if (seen) continue;
      if (nvis == Q2_HZCAP) { lstatus |= QHS_CAPACITY; return bestfacet; }
      vis[nvis++] = nb;
      if (!(fl[k] & QF_FLIPPED)) {
        const double dist = q2_distq(q[k], p);
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
        if (ncop == Q2_COPCAP) { lstatus |= QHS_CAPACITY; return bestfacet; }
        cop[64 * ncop++] = nextfacet;
      }
      nextfacet = nb;
      nextnb[0] = nn[k][0]; nextnb[1] = nn[k][1]; nextnb[2] = nn[k][2];
    }
    facet = nextfacet;
    if (facet >= 0) {
      nextfacet = -1;
      cur[0] = nextnb[0]; cur[1] = nextnb[1]; cur[2] = nextnb[2];
      continue;
    }
    if (!ncop) break;
    if (ncop == 1) { facet = cop[0]; ncop = 0; }
    else facet = cop[64 * --ncop];
    const QFr& fr = W.F[facet];
    cur[0] = fr.nb[0]; cur[1] = fr.nb[1]; cur[2] = fr.nb[2];
  }
  return bestfacet;
}

// qh_findbestnew over the scan list (new facets from startfacet's index,
// the moved old facets, the new facets before it)
__device__ inline int q2_findbestnew(const Q2W& W, const Q2S& S, const Q2L& L, const double* p, int s0,
                                     double* dist, int bestoutside, int* isoutside, int& lstatus) {
  double bestdist = -DBL_MAX / 2;
  int bestfacet = -1;
  const double distoutside = fmax(2 * S.MINoutside, S.max_outside);
  *isoutside = 1;
  const int total = S.nnew + S.nmov;
  for (int t = 0; t < total; t++) {
    int f;
    double q[4];
    int fl;
    if (t < S.nnew - s0) {
      const int u = s0 + t;
      f = L.nslot[u];
      for (int k = 0; k < 4; k++) q[k] = L.npl[4 * u + k];
      fl = L.nflag[u];
    } else if (t < S.nnew - s0 + S.nmov) {
      f = L.movf[t - (S.nnew - s0)];
      const QFr& r = W.F[f];
      q[0] = r.n[0]; q[1] = r.n[1]; q[2] = r.n[2]; q[3] = r.off;
      fl = r.flags;
    } else {
      const int u = t - (S.nnew - s0) - S.nmov;
      f = L.nslot[u];
      for (int k = 0; k < 4; k++) q[k] = L.npl[4 * u + k];
      fl = L.nflag[u];
    }
    if (fl & QF_FLIPPED) continue;
    const double d = q2_distq(q, p);
    if (d > bestdist) {
      bestfacet = f;
      if (!bestoutside && d >= distoutside) { *dist = d; return bestfacet; }
      bestdist = d;
    }
  }
  bestfacet = q2_findbesthorizon(W, S, L, p, bestfacet >= 0 ? bestfacet : L.nslot[s0], &bestdist, lstatus);
  *dist = bestdist;
  if (bestdist < S.MINoutside) *isoutside = 0;
  return bestfacet;
}

__device__ inline int q2_sharpnewfacets(const Q2S& S, const Q2L& L) {
  int quadrant[3];
  for (int t = 0; t < S.nnew; t++) {
    const double* n = L.npl + 4 * t;
    if (t == 0) {
      for (int k = 3; k--;) quadrant[k] = n[k] > 0;
    } else {
      for (int k = 3; k--;)
        if (quadrant[k] != (n[k] > 0)) return 1;
    }
  }
  return 0;
}

// qh_partitionpoint's search (s0: the start facet's new-facet index);
// sharp = 2: qh_findbestnew(bestoutside) for a deleted vertex
__device__ inline int q2_locate(const Q2W& W, const Q2S& S, const Q2L& L, const double* p,
                                                   int s0, int sharp, double* bestdist_out, int* isoutside,
                                                   int* trigger, int& lstatus) {
  *trigger = 0;
  if (sharp == 2) return q2_findbestnew(W, S, L, p, s0, bestdist_out, 1, isoutside, lstatus);
  if (S.findbestnew) return q2_findbestnew(W, S, L, p, s0, bestdist_out, 0, isoutside, lstatus);
  double bestdist = -DBL_MAX / 2;
  int bestu = -1;
  *isoutside = 1;
  unsigned long long m0 = 0ull, m1 = 0ull;   // new facets visited (index < Q2_NEWCAP = 128)
  if (!(L.nflag[s0] & QF_FLIPPED)) {
    const double d = q2_distq(L.npl + 4 * s0, p);
    if (d >= S.MINoutside) { *bestdist_out = d; return L.nslot[s0]; }
    bestdist = d;
    bestu = s0;
  }
  if (s0 < 64) m0 |= 1ull << s0; else m1 |= 1ull << (s0 - 64);
  int u = s0;
  while (u >= 0) {
    int nxt = -1;
    // neighbours: nb0 the horizon facet (old: skipped, isnewfacets), nb1, nb2 new
    const int cand[2] = {L.nn1[u], L.nn2[u]};
    for (int k = 0; k < 2; k++) {
      const int c = cand[k];
      const bool was = c < 64 ? (m0 >> c) & 1ull : (m1 >> (c - 64)) & 1ull;
      if (was) continue;
      if (c < 64) m0 |= 1ull << c; else m1 |= 1ull << (c - 64);
      if (!(L.nflag[c] & QF_FLIPPED)) {
        const double d = q2_distq(L.npl + 4 * c, p);
        if (d > bestdist) {
          if (d >= S.MINoutside) { *bestdist_out = d; return L.nslot[c]; }
          bestu = c;
          bestdist = d;
          nxt = c;
          break;
        }
      }
    }
    u = nxt;
  }
  if (bestu < 0) return q2_findbestnew(W, S, L, p, 0, bestdist_out, 0, isoutside, lstatus);
  if (!S.notsharp && bestdist < -S.DISTround) {
    *trigger = 1;
    if (sharp) return q2_findbestnew(W, S, L, p, bestu, bestdist_out, 0, isoutside, lstatus);
  }
  const int bf = q2_findbesthorizon(W, S, L, p, L.nslot[bestu], &bestdist, lstatus);
  *bestdist_out = bestdist;
  if (bestdist < S.MINoutside) *isoutside = 0;
  return bf;
}

__device__ __forceinline__ bool q2_in_movf(const Q2S& S, const Q2L& L, int f) {
  for (int t = 0; t < S.nmov; t++)
    if (L.movf[t] == f) return true;
  return false;
}

// the partition sequence W.pq[0..np), start facets (new-facet indices) W.pst
__device__ inline void q2_locate_seq(const Q2W& W, Q2S& S, Q2L& L, int np, int sharp, int lane) {
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
        const int f = q2_locate(W, S, L, W.Pr + 3 * (size_t)pid, W.pst[pos], sharp, &d, &isout, &trig, ls);
        int dst = -1;
        if (isout) {
          dst = f;
          const int fl = W.F[f].flags;
          if (!(fl & QF_NEW) && W.seg[2 * f + 1] == 0 && !q2_in_movf(S, L, f)) kind |= 4;
        } else if (d >= -S.MAXcoplanar && d > S.max_outside) {
          kind |= 2;
        }
        if (trig) kind |= 1;
        W.pdst[pos] = dst;
        W.pdd[pos] = d;
      }
      S.status |= qh_wave_or(ls);
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
        // qh_partitionpoint moves the old facet behind the new ones: a fresh key
        const int f = W.pdst[ev_pos];
        if (S.nmov == Q2_MOVCAP) S.status |= QHS_CAPACITY;
        else {
          if (lane == 0) { L.movf[S.nmov] = f; W.key[f] = S.keyc; }
          S.keyc++;
          S.nmov++;
        }
      }
      hl_sync();
    }
    from = ev_pos + 1;
  }
}

// outside sets in Qhull's order (see lqro_qhull.hpp qh_emit_seq); the
// facets that receive their first points join the queue in key order
__device__ inline void q2_emit_seq(const Q2W& W, Q2S& S, Q2L& L, int np, int lane) {
  for (int t = lane; t < S.nnew; t += 64) { L.pcnt[t] = 0; L.dfac[t] = L.nslot[t]; }
  S.nold = 0;
  hl_sync();
  for (int c = 0; c < np; c += 64) {
    const int pos = c + lane;
    const int dst = pos < np ? W.pdst[pos] : -1;
    const int fl = dst >= 0 ? W.F[dst].flags : 0;
    const bool isnew = dst >= 0 && (fl & QF_NEW);
    if (isnew) atomicAdd(&L.pcnt[W.F[dst].aux], 1);
    unsigned long long old = __ballot(dst >= 0 && !isnew);
    while (old) {
      const int l = __ffsll((long long)old) - 1;
      old &= old - 1;
      const int f = __builtin_amdgcn_readlane(dst, l);
      int k = -1;
      for (int t = 0; t < S.nold; t++)
        if (L.oldf[t] == f) k = t;
      if (k < 0) {
        if (S.nold == Q2_MOVCAP) { S.status |= QHS_CAPACITY; continue; }
        k = S.nold++;
        if (lane == 0) { L.oldf[k] = f; L.pcnt[Q2_NEWCAP + k] = 0; L.dfac[Q2_NEWCAP + k] = f; }
        hl_sync();
      }
      if (lane == 0) L.pcnt[Q2_NEWCAP + k]++;
      hl_sync();
    }
    hl_sync();
  }
  hl_sync();
  if (S.status & QHS_CAPACITY) return;
  // segments (new facets: fresh; old: continued)
  for (int g0 = 0; g0 < S.nnew + S.nold; g0++) {
    const int g = g0 < S.nnew ? g0 : Q2_NEWCAP + (g0 - S.nnew);
    const int add = L.pcnt[g];
    if (!add) continue;
    const int f = L.dfac[g];
    const int cnt0 = g < Q2_NEWCAP ? 0 : W.seg[2 * f + 1];
    const int off0 = g < Q2_NEWCAP ? 0 : W.seg[2 * f];
    const int size = cnt0 + add;
    if (S.sbtop + size > W.SB) { S.status |= QHS_CAPACITY; return; }
    const int off = S.sbtop;
    S.sbtop += size;
    for (int t = lane; t < cnt0 - 1; t += 64) W.sb[off + t] = W.sb[off0 + t];
    if (lane == 0) {
      L.doff[g] = off;
      L.dcnt[g] = cnt0;
      L.dmax[g] = g < Q2_NEWCAP ? 0.0 : W.fdist[f];
      L.dchamp[g] = cnt0 ? W.sb[off0 + cnt0 - 1] : -1;
      if (g >= Q2_NEWCAP) W.F[f].aux = g;      // an old facet's destination index (cleared below)
    }
    hl_sync();
  }
  hl_sync();
  for (int c = 0; c < np; c += 64) {
    const int pos = c + lane;
    const bool act = pos < np;
    const int dst = act ? W.pdst[pos] : -1;
    const int g = dst >= 0 ? W.F[dst].aux : -1;
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
    const int g = g0 < S.nnew ? g0 : Q2_NEWCAP + (g0 - S.nnew);
    if (!L.pcnt[g]) continue;
    const int f = L.dfac[g];
    W.sb[L.doff[g] + L.dcnt[g] - 1] = L.dchamp[g];
    W.seg[2 * f] = L.doff[g];
    W.seg[2 * f + 1] = L.dcnt[g];
    W.fdist[f] = L.dmax[g];
    if (g >= Q2_NEWCAP) W.F[f].aux = -1;
  }
  hl_sync();
  // the queue (qh.facet_next's walk): new facets with points in key order,
  // then the moved old facets in move order
  {
    int qt = S.qtail;
    for (int c = 0; c < S.nnew; c += 64) {
      const int t = c + lane;
      const bool has = t < S.nnew && L.pcnt[t] > 0;
      const unsigned long long b = __ballot(has);
      if (has) {
        const int at = qt + __popcll(b & ((1ull << lane) - 1ull));
        if (at < W.QC) { W.fq[at] = L.nslot[t]; W.fqk[at] = W.key[L.nslot[t]]; }
      }
      qt += __popcll(b);
    }
    for (int t = 0; t < S.nmov; t++) {
      if (lane == 0 && qt < W.QC) { W.fq[qt] = L.movf[t]; W.fqk[qt] = W.key[L.movf[t]]; }
      qt++;
    }
    if (qt > W.QC) S.status |= QHS_CAPACITY;
    S.qtail = qt;
  }
  hl_sync();
}

// a new facet index for the facets created in this insertion
__device__ __forceinline__ int q2_alloc(const Q2W& W, Q2S& S, const Q2L& L, int t) {
  if (t < S.nvis) return L.visf[t];         // the cone reuses the visible facets' slots
  const int e = t - S.nvis;                 // beyond: free slots, then fresh ones
  if (e < S.nfree) return W.fstack[S.nfree - 1 - e];
  return S.nalloc + (e - S.nfree);
}

// qh_qhull on W.Pr[0..n)
__device__ inline void q2_build(const Q2W& W, Q2S& S, Q2L& L, int n, int lane) {
#ifdef LQRO_QHULL_PROFILE
  unsigned long long tq_ = __builtin_amdgcn_s_memtime();
#endif
  S.status = 0;
  S.nalloc = 1;
  S.nfree = 0;
  S.sbtop = 0;
  S.nnew = S.nvis = S.nmov = S.nold = 0;
  S.findbestnew = S.notsharp = 0;
  S.keyc = 1;
  S.qhead = S.qtail = 0;
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
    QhS T = q2_as_qhs(S);
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
          double det = fabs(qh_detsimplex(T, W.Pr, simplex, i, p, &nearzero));
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
          const double det = fabs(qh_detsimplex(T, W.Pr, simplex, i, q, &nearzero));
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
  // qh_initialvertices, qh_createsimplex (facet slots 1..4, keys 1..4)
  int vset[4];
  for (int i = 0; i < 4; i++) {
    if (lane == 0) W.vpt[S.nv] = simplex[i];
    vset[3 - i] = S.nv++;
  }
  {
    int fs[4], top = 1;
    for (int i = 0; i < 4; i++) {
      const int f = S.nalloc++;
      fs[i] = f;
      if (lane == 0) {
        QFr& r = W.F[f];
        int m = 0;
        for (int t = 0; t < 4; t++)
          if (t != i) r.v[m++] = vset[t];
        m = 0;
        r.flags = QF_LIVE | (top ? QF_TOP : 0);
        r.aux = -1;
        W.seg[2 * f] = 0;
        W.seg[2 * f + 1] = 0;
        W.fdist[f] = 0.0;
        W.key[f] = S.keyc;
      }
      S.keyc++;
      top ^= 1;
    }
    hl_sync();
    if (lane == 0)
      for (int i = 0; i < 4; i++) {
        int m = 0;
        for (int t = 0; t < 4; t++)
          if (t != i) W.F[fs[i]].nb[m++] = fs[t];
      }
    for (int k = 0; k < 3; k++) {
      double c = 0.0;
      for (int t = 0; t < 4; t++) c += W.Pr[3 * (size_t)W.vpt[vset[t]] + k];
      S.interior[k] = c / 4;
    }
    hl_sync();
    // qh_initialhull: the first facet's orientation decides
    int ls = 0;
    auto plane_of = [&](int f, bool* flipped) {
      const QFr& r = W.F[f];
      double q[4];
      q2_plane(S, ls, W.Pr + 3 * (size_t)W.vpt[r.v[0]], W.Pr + 3 * (size_t)W.vpt[r.v[1]],
               W.Pr + 3 * (size_t)W.vpt[r.v[2]], r.flags & QF_TOP, q, flipped);
      hl_sync();
      if (lane == 0) {
        QFr& w = W.F[f];
        w.n[0] = q[0]; w.n[1] = q[1]; w.n[2] = q[2]; w.off = q[3];
        w.flags = *flipped ? (w.flags | QF_FLIPPED) : (w.flags & ~QF_FLIPPED);
      }
      hl_sync();
    };
    bool fl0;
    plane_of(fs[0], &fl0);
    {
      const QFr& r = W.F[fs[0]];
      const double q[4] = {r.n[0], r.n[1], r.n[2], r.off};
      const bool flip = q2_distq(q, S.interior) > S.DISTround;
      hl_sync();
      if (flip && lane == 0)
        for (int i = 0; i < 4; i++) W.F[fs[i]].flags ^= QF_TOP;
      hl_sync();
    }
    bool anyflip = false;
    for (int i = 0; i < 4; i++) {
      bool fl;
      plane_of(fs[i], &fl);
      anyflip |= fl;
    }
    if (anyflip) ls |= QHS_FLIPPED;
    double minangle = DBL_MAX;
    for (int i = 0; i < 4; i++)
      for (int t = 0; t < 3; t++) {
        const QFr& a = W.F[fs[i]];
        const QFr& b = W.F[a.nb[t]];
        double angle = 0.0;
        for (int k = 0; k < 3; k++) angle += a.n[k] * b.n[k];
        if (angle < minangle) minangle = angle;
      }
    if (minangle < -0.99999999) ls |= QHS_NARROW;
    S.status |= ls;
    // qh_partitionall
    int np = 0;
    for (int c = 0; c < n; c += 64) {
      const int q = c + lane;
      const bool ok = q < n && q != simplex[0] && q != simplex[1] && q != simplex[2] && q != simplex[3];
      const unsigned long long b = __ballot(ok);
      if (ok) W.pq[np + __popcll(b & ((1ull << lane) - 1ull))] = q;
      np += __popcll(b);
    }
    hl_sync();
    const double distoutside = fmax(2 * S.MINoutside, S.max_outside);
    for (int i = 0; i < 4; i++) {
      const int f = fs[i];
      const QFr& r = W.F[f];
      const double q[4] = {r.n[0], r.n[1], r.n[2], r.off};
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
          d = q2_distq(q, W.Pr + 3 * (size_t)pid);
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
          const int qq = __builtin_amdgcn_readlane(pid, l);
          const double dq = hl_rl(d, l);
          if (cnt == 0) {
            champ = qq; mx = dq;
          } else if (dq > mx) {
            if (off + cnt - 1 < W.SB && lane == 0) W.sb[off + cnt - 1] = champ;
            champ = qq; mx = dq;
          } else {
            if (off + cnt - 1 < W.SB && lane == 0) W.sb[off + cnt - 1] = qq;
          }
          cnt++;
        }
        hl_sync();
      }
      if (cnt) {
        if (off + cnt > W.SB) { S.status |= QHS_CAPACITY; return; }
        if (lane == 0) {
          W.sb[off + cnt - 1] = champ;
          W.seg[2 * f] = off;
          W.seg[2 * f + 1] = cnt;
          W.fdist[f] = mx;
        }
        S.sbtop += cnt;
      }
      np = w;
      hl_sync();
    }
    // the remainder: qh_partitionpoint with findbestnew over the facet list
    // (the four facets in list order act as the scan list; moved facets go
    // to its end)
    if (np > 0) {
      S.nnew = 4;
      for (int i = 0; i < 4; i++) {
        if (lane == 0) {
          L.nslot[i] = fs[i];
          const QFr& r = W.F[fs[i]];
          L.npl[4 * i] = r.n[0]; L.npl[4 * i + 1] = r.n[1]; L.npl[4 * i + 2] = r.n[2]; L.npl[4 * i + 3] = r.off;
          L.nflag[i] = r.flags;
          L.nn1[i] = L.nn2[i] = -1;
        }
      }
      S.nmov = 0;
      S.findbestnew = 1;
      for (int q = lane; q < np; q += 64) W.pst[q] = 0;
      hl_sync();
      // sequential semantics: a moved facet changes the list head for later
      // points; handled by q2_locate_seq's event (fresh key) and, here, a
      // rotation of the scan list
      int from = 0;
      while (from < np) {
        int ev_pos = np, ev_kind = 0;
        for (int c = from; c < np; c += 64) {
          const int pos = c + lane;
          int kind = 0, ls2 = 0;
          if (pos < np) {
            double d;
            int isout;
            int trig;
            const int f = q2_locate(W, S, L, W.Pr + 3 * (size_t)W.pq[pos], 0, 0, &d, &isout, &trig, ls2);
            int dst = -1;
            if (isout) {
              dst = f;
              if (W.seg[2 * f + 1] == 0 && !q2_in_movf(S, L, f)) kind |= 4;
            } else if (d >= -S.MAXcoplanar && d > S.max_outside) {
              kind |= 2;
            }
            W.pdst[pos] = dst;
            W.pdd[pos] = d;
          }
          S.status |= qh_wave_or(ls2);
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
          if (ev_kind & 2) S.max_outside = W.pdd[ev_pos];
          if (ev_kind & 4) {
            const int f = W.pdst[ev_pos];
            if (S.nmov == Q2_MOVCAP) S.status |= QHS_CAPACITY;
            if (lane == 0) {
              int t0 = 0;
              for (int t = 0; t < 4; t++)
                if (L.nslot[t] == f) t0 = t;
              for (int t = t0; t + 1 < 4; t++) {
                L.nslot[t] = L.nslot[t + 1];
                for (int k = 0; k < 4; k++) L.npl[4 * t + k] = L.npl[4 * (t + 1) + k];
                L.nflag[t] = L.nflag[t + 1];
              }
              L.nslot[3] = f;
              const QFr& r = W.F[f];
              L.npl[12] = r.n[0]; L.npl[13] = r.n[1]; L.npl[14] = r.n[2]; L.npl[15] = r.off;
              L.nflag[3] = r.flags;
              L.movf[S.nmov < Q2_MOVCAP ? S.nmov : 0] = f;
              W.key[f] = S.keyc;
            }
            S.keyc++;
            S.nmov++;
          }
          hl_sync();
        }
        from = ev_pos + 1;
      }
      // the remainder's outside points: continue the four sets (moved facets
      // are old facets with an empty set)
      S.nnew = 0;
      S.nmov = 0;
      if (!(S.status & QHS_CAPACITY)) q2_emit_seq(W, S, L, np, lane);
      S.qtail = 0;    // the queue is built below, after qh_furthestnext
      S.findbestnew = 0;
      hl_sync();
    }
    if (S.status & (QHS_INPUT | QHS_TOPOLOGY | QHS_CAPACITY)) return;
    // qh_furthestnext: the first facet in list order with the furthest
    // outside point moves to the front (key 0)
    {
      int order[4] = {fs[0], fs[1], fs[2], fs[3]};
      unsigned kk[4];
      for (int i = 0; i < 4; i++) kk[i] = W.key[order[i]];
      for (int a = 0; a < 4; a++)
        for (int b = a + 1; b < 4; b++)
          if (kk[b] < kk[a]) {
            const unsigned tk = kk[a]; kk[a] = kk[b]; kk[b] = tk;
            const int to = order[a]; order[a] = order[b]; order[b] = to;
          }
      int best = -1;
      double bd = -DBL_MAX;
      for (int i = 0; i < 4; i++) {
        const int f = order[i];
        if (W.seg[2 * f + 1] && W.fdist[f] > bd) { best = f; bd = W.fdist[f]; }
      }
      hl_sync();
      if (best >= 0) {
        if (lane == 0) W.key[best] = 0;
        for (int i = 0; i < 4; i++)
          if (order[i] == best) {
            for (int t = i; t > 0; t--) { order[t] = order[t - 1]; kk[t] = kk[t - 1]; }
            order[0] = best;
            kk[0] = 0;
            break;
          }
      }
      // the queue: facets with points in list order
      int qt = 0;
      for (int i = 0; i < 4; i++)
        if (W.seg[2 * order[i] + 1]) {
          if (lane == 0) { W.fq[qt] = order[i]; W.fqk[qt] = kk[i]; }
          qt++;
        }
      S.qhead = 0;
      S.qtail = qt;
      hl_sync();
    }
  }
  Q2T(0);
  const unsigned long long ltmask = (1ull << (threadIdx.x & 63)) - 1ull;
  // qh_buildhull
  for (;;) {
    // qh_nextfurthest: the first queued facet still alive with points
    int facet = -1, furthest = -1;
    while (S.qhead < S.qtail) {
      const int f = W.fq[S.qhead];
      const unsigned k = W.fqk[S.qhead];
      const int fl = W.F[f].flags;
      const int cnt = W.seg[2 * f + 1];
      const unsigned fk = W.key[f];
      if ((fl & QF_LIVE) && fk == k && cnt > 0) {
        facet = f;
        furthest = W.sb[W.seg[2 * f] + cnt - 1];
        hl_sync();
        if (lane == 0) W.seg[2 * f + 1] = cnt - 1;
        hl_sync();
        break;
      }
      S.qhead++;
    }
    Q2T(1);
    if (furthest < 0) break;
    const double* apexp = W.Pr + 3 * (size_t)furthest;
    // qh_findhorizon, a level of the breadth-first search at a time: the
    // candidates of a level in (visible facet, neighbour) order, a facet
    // taken at its first occurrence
    if (lane == 0) { L.visf[0] = facet; W.F[facet].flags |= QF_VISIBLE; }
    hl_sync();
    int ls = 0, nvis = 1;
    for (int lo = 0; lo < nvis;) {
      const int hi = nvis;
      const int ncand = 3 * (hi - lo);
      for (int c0 = 0; c0 < ncand; c0 += 64) {
        const int c = c0 + lane;
        int nb = -1, fl = QF_VISIBLE;
        double q[4] = {0.0, 0.0, 0.0, 0.0};
        if (c < ncand) {
          nb = W.F[L.visf[lo + c / 3]].nb[c % 3];
          const QFr& r = W.F[nb];
          fl = r.flags;
          q[0] = r.n[0]; q[1] = r.n[1]; q[2] = r.n[2]; q[3] = r.off;
        }
        bool cand = !(fl & QF_VISIBLE);
        bool dup = false;
        for (unsigned long long mm = __ballot(cand); mm;) {
          const int l = __ffsll((long long)mm) - 1;
          mm &= mm - 1;
          dup |= (l < lane) && __builtin_amdgcn_readlane(nb, l) == nb;
        }
        cand = cand && !dup;
        const double dist = cand ? q2_distq(q, apexp) : 0.0;
        const bool vis = cand && dist >= S.MINvisible;
        if (cand && !vis && dist >= -S.MAXcoplanar) ls |= QHS_COPLANAR;   // Qhull merges it: built on merge-free
        const unsigned long long bv = __ballot(vis);
        if (vis) {
          const int at = nvis + __popcll(bv & ltmask);
          if (at < Q2_VISCAP) L.visf[at] = nb;
          W.F[nb].flags = fl | QF_VISIBLE;
        }
        nvis += __popcll(bv);
        hl_sync();
      }
      lo = hi;
      if (nvis > Q2_VISCAP) { S.status |= QHS_CAPACITY; return; }
    }
    S.status |= qh_wave_or(ls);
    S.nvis = nvis;
    Q2T(2);
    // qh_makenew_simplicial: one new facet per horizon ridge, created in
    // (visible facet, neighbour) order; first what the visible facets' slots
    // still hold
    const int apex = S.nv++;
    if (lane == 0) W.vpt[apex] = furthest;
    for (int vi = lane; vi < nvis; vi += 64) {
      const int f = L.visf[vi];
      const QFr& r = W.F[f];
      L.vvert[3 * vi] = r.v[0]; L.vvert[3 * vi + 1] = r.v[1]; L.vvert[3 * vi + 2] = r.v[2];
      L.vsoff[vi] = W.seg[2 * f];
      L.vscnt[vi] = W.seg[2 * f + 1];
      L.repl[vi] = -1;
    }
    hl_sync();
    int nnew = 0, ts = 0;
    for (int c0 = 0; c0 < 3 * nvis; c0 += 64) {
      const int c = c0 + lane;
      int vis = -1, nb = -1, hf = QF_VISIBLE;
      int hn0 = -1, hn1 = -1, hn2 = -1, hv0 = 0, hv1 = 0, hv2 = 0;
      if (c < 3 * nvis) {
        vis = L.visf[c / 3];
        nb = W.F[vis].nb[c % 3];
        const QFr& h = W.F[nb];
        hf = h.flags;
        hn0 = h.nb[0]; hn1 = h.nb[1]; hn2 = h.nb[2];
        hv0 = h.v[0]; hv1 = h.v[1]; hv2 = h.v[2];
      }
      const bool ridge = !(hf & QF_VISIBLE);
      const unsigned long long b = __ballot(ridge);
      if (ridge) {
        const int t = nnew + __popcll(b & ltmask);
        const int hskip = hn0 == vis ? 0 : hn1 == vis ? 1 : hn2 == vis ? 2 : -1;
        if (hskip < 0) {
          ts |= QHS_TOPOLOGY;
        } else if (t < Q2_NEWCAP) {
          const int top = (hf & QF_TOP) ? (hskip & 1) : ((hskip & 1) ^ 1);
          L.nv[3 * t] = apex;
          L.nv[3 * t + 1] = hskip == 0 ? hv1 : hv0;
          L.nv[3 * t + 2] = hskip == 2 ? hv1 : hv2;
          L.nhz[t] = nb;
          L.nhskip[t] = hskip;
          L.nopp[t] = hskip == 0 ? hv0 : hskip == 1 ? hv1 : hv2;
          L.nflag[t] = QF_NEW | QF_LIVE | (top ? QF_TOP : 0);
          atomicMax(&L.repl[c / 3], t);     // qh_getreplacement: the last new facet of the visible one
        }
      }
      nnew += __popcll(b);
    }
    S.status |= qh_wave_or(ts);
    if (nnew > Q2_NEWCAP) S.status |= QHS_CAPACITY;
    if (S.status & (QHS_TOPOLOGY | QHS_CAPACITY)) return;
    S.nnew = nnew;
    {
      // slots: the visible facets', then free ones, then fresh ones
      const int extra = nnew > nvis ? nnew - nvis : 0;
      const int take = extra < S.nfree ? extra : S.nfree;
      if (S.nalloc + extra - take > W.FC) { S.status |= QHS_CAPACITY; return; }
      hl_sync();
      for (int t = lane; t < nnew; t += 64) L.nslot[t] = q2_alloc(W, S, L, t);
      S.nfree -= take;
      S.nalloc += extra - take;
      hl_sync();
    }
    Q2T(3);
    // qh_matchnewfacets (nb[1] shares {apex, v2}, nb[2] shares {apex, v1}),
    // qh_makenewplanes; the new facets' records; the horizon facets' links
    int lm = 0;
    const unsigned key0 = S.keyc;
    for (int t = lane; t < nnew; t += 64) {
      int nbu[2];
      for (int k = 1; k < 3; k++) {
        const int w = L.nv[3 * t + 3 - k];
        int found = -1, cnt = 0;
        for (int u = 0; u < nnew; u++)
          if (u != t && (L.nv[3 * u + 1] == w || L.nv[3 * u + 2] == w)) { found = u; cnt++; }
        if (cnt != 1) lm |= QHS_TOPOLOGY;
        nbu[k - 1] = found;
      }
      L.nn1[t] = nbu[0] >= 0 ? nbu[0] : 0;
      L.nn2[t] = nbu[1] >= 0 ? nbu[1] : 0;
      double q[4];
      bool flipped;
      const int v1 = L.nv[3 * t + 1], v2 = L.nv[3 * t + 2];
      int fl = L.nflag[t];
      q2_plane(S, lm, apexp, W.Pr + 3 * (size_t)W.vpt[v1], W.Pr + 3 * (size_t)W.vpt[v2], fl & QF_TOP, q, &flipped);
      if (flipped) { fl |= QF_FLIPPED; lm |= QHS_FLIPPED; }
      L.nflag[t] = fl;
      L.npl[4 * t] = q[0]; L.npl[4 * t + 1] = q[1]; L.npl[4 * t + 2] = q[2]; L.npl[4 * t + 3] = q[3];
      const int s = L.nslot[t];
      double4* rd = reinterpret_cast<double4*>(W.F + s);
      int4* ri = reinterpret_cast<int4*>(W.F + s);
      rd[0] = make_double4(q[0], q[1], q[2], q[3]);
      ri[2] = make_int4(L.nhz[t], nbu[0] >= 0 ? L.nslot[nbu[0]] : -1, nbu[1] >= 0 ? L.nslot[nbu[1]] : -1, fl);
      ri[3] = make_int4(apex, v1, v2, t);
      W.F[L.nhz[t]].nb[L.nhskip[t]] = s;
      W.seg[2 * s] = 0;
      W.seg[2 * s + 1] = 0;
      W.fdist[s] = 0.0;
      W.key[s] = key0 + (unsigned)t;
    }
    S.keyc += (unsigned)nnew;
    hl_sync();
    // qh_checkzero: each new facet clearly convex to its neighbours
    if (!(qh_wave_or(lm) & QHS_FLIPPED)) {
      for (int t = lane; t < nnew; t += 64) {
        const double* pt = L.npl + 4 * t;
        const double d1 = q2_distq(L.npl + 4 * L.nn1[t], W.Pr + 3 * (size_t)W.vpt[L.nv[3 * t + 1]]);
        const double d2 = q2_distq(L.npl + 4 * L.nn2[t], W.Pr + 3 * (size_t)W.vpt[L.nv[3 * t + 2]]);
        const double d3 = q2_distq(pt, W.Pr + 3 * (size_t)W.vpt[L.nopp[t]]);
        if (d1 >= -2 * S.DISTround || d2 >= -2 * S.DISTround || d3 >= -2 * S.DISTround) lm |= QHS_NONCONVEX;
      }
    }
    S.status |= qh_wave_or(lm);
    Q2T(4);
    if (S.status & (QHS_TOPOLOGY | QHS_CAPACITY)) return;
    // qh_partitionvisible: the visible facets' outside sets in visible order,
    // each from its replacement (or the first new facet)
    int np2 = 0;
    for (int c0 = 0; c0 < nvis; c0 += 64) {
      const int vi = c0 + lane;
      const int cnt = vi < nvis ? L.vscnt[vi] : 0;
      int inc = cnt;
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(inc, off);
        if (lane >= off) inc += o;
      }
      if (vi < nvis) L.vinc[vi] = np2 + inc;
      np2 += __shfl(inc, 63);
    }
    hl_sync();
    for (int pos = lane; pos < np2; pos += 64) {
      int a = 0, b = nvis - 1;
      while (a < b) {
        const int mid = (a + b) >> 1;
        if (L.vinc[mid] > pos) b = mid;
        else a = mid + 1;
      }
      const int within = pos - (L.vinc[a] - L.vscnt[a]);
      W.pq[pos] = W.sb[L.vsoff[a] + within];
      W.pst[pos] = L.repl[a] >= 0 ? L.repl[a] : 0;
    }
    hl_sync();
    S.findbestnew = 0;
    S.notsharp = 0;
    S.nmov = 0;
    const int sharp = q2_sharpnewfacets(S, L);
    Q2T(5);
    if (np2) {
      q2_locate_seq(W, S, L, np2, sharp, lane);
      Q2T(6);
      q2_emit_seq(W, S, L, np2, lane);
      Q2T(7);
    }
    // deleted vertices (a visible facet's vertex on no new facet) close to a
    // new facet: Qhull's qh_partitioncoplanar would act (not restated)
    {
      int lsd = 0;
      for (int t = lane; t < 3 * nvis; t += 64) {
        const int v = L.vvert[t];
        bool skip = false;
        for (int u = 0; u < nnew && !skip; u++) skip = L.nv[3 * u + 1] == v || L.nv[3 * u + 2] == v;
        for (int e = 0; e < t && !skip; e++) skip = L.vvert[e] == v;
        if (skip) continue;
        double d;
        int iso;
        int trig;
        q2_locate(W, S, L, W.Pr + 3 * (size_t)W.vpt[v], 0, 2, &d, &iso, &trig, lsd);
        if (d >= -S.MAXcoplanar) lsd |= QHS_COPLANAR;
      }
      S.status |= qh_wave_or(lsd);
    }
    Q2T(8);
    if (S.status & QHS_CAPACITY) return;
    // qh_deletevisible: the visible slots no new facet took are freed; the
    // new facets become old
    for (int t = nnew + lane; t < nvis; t += 64) {
      const int f = L.visf[t];
      W.F[f].flags = 0;
      W.fstack[S.nfree + (t - nnew)] = f;
    }
    if (nvis > nnew) S.nfree += nvis - nnew;
    for (int t = lane; t < nnew; t += 64) {
      const int s = L.nslot[t];
      W.F[s].flags = L.nflag[t] & ~QF_NEW;
      W.F[s].aux = -1;
    }
    S.nnew = 0;
    S.nmov = 0;
    S.findbestnew = 0;
    S.notsharp = 0;
    hl_sync();
    Q2T(9);
  }
}

// the reference's selection (LQRO:925-968; see lqro_qhull.hpp qh_select):
// Qhull's facet order is key order, so the first facet on a tie is the one
// with the smaller key, and facet 0 is the smallest key alive
__device__ inline void q2_select(const HullArgs& A, const Q2W& W, const Q2S& S, int lane, const double* xi,
                                 const double* vrel, int slot) {
  const bool fail = (S.status & (QHS_INPUT | QHS_TOPOLOGY | QHS_CAPACITY)) != 0;
  double best = INFINITY;
  unsigned bkey = 0xffffffffu, minkey = 0xffffffffu;
  int bf = -1, nfac = 0;
  if (!fail) {
    for (int f = 1 + lane; f < S.nalloc; f += 64) {
      const QFr& r = W.F[f];
      if (!(r.flags & QF_LIVE)) continue;
      nfac++;
      const unsigned k = W.key[f];
      minkey = k < minkey ? k : minkey;
      const double* P = W.Pf + 3 * (size_t)W.vpt[r.v[0]];
      const double d = fabs(r.n[0] * (vrel[0] - P[0]) + r.n[1] * (vrel[1] - P[1]) + r.n[2] * (vrel[2] - P[2]));
      if (d < best || (d == best && k < bkey)) { best = d; bkey = k; bf = f; }
    }
  }
  for (int off = 32; off >= 1; off >>= 1) {
    const double ob = __shfl_xor(best, off);
    const unsigned ok = (unsigned)__shfl_xor((int)bkey, off);
    const int of = __shfl_xor(bf, off);
    const unsigned om = (unsigned)__shfl_xor((int)minkey, off);
    nfac += __shfl_xor(nfac, off);
    minkey = om < minkey ? om : minkey;
    if (ob < best || (ob == best && ok < bkey)) { best = ob; bkey = ok; bf = of; }
  }
  const bool ok = !fail && nfac > 0 && bf >= 0;
  const bool stale = ok && bkey == minkey;
  const bool merged = (S.status & (QHS_COPLANAR | QHS_NONCONVEX | QHS_FLIPPED | QHS_NARROW | QHS_SINGULAR)) != 0;
  if (lane == 0) {
    float* pl = A.planes + (size_t)slot * 8;
    double* qn = A.qnrm + (size_t)slot * 4;
    double nrm[3] = {0.0, 0.0, 0.0};
    if (ok && !stale) {
      const QFr& r = W.F[bf];
      nrm[0] = r.n[0]; nrm[1] = r.n[1]; nrm[2] = r.n[2];
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
      atomicAdd(&A.stats[4], 1ull);
    }
    if (A.recs) {
      lqro_pair_record& rec = A.recs[slot];
      rec.flags |= ok ? LQRO_REC_HULL : LQRO_REC_HULLFAIL;
      if (stale) rec.flags |= LQRO_REC_STALE;
      if (merged) rec.flags |= LQRO_REC_QHMERGE;
      rec.n_facets = ok ? nfac : -(S.status & 0xffff) - 1;
      if (ok) {
        const QFr& r = W.F[bf];
        rec.facet[0] = W.vpt[r.v[0]]; rec.facet[1] = W.vpt[r.v[1]]; rec.facet[2] = W.vpt[r.v[2]];
        rec.dist = best;
        for (int q = 0; q < 3; ++q) {
          rec.normal[q] = nrm[q];
          rec.plane_point[q] = stale ? 0.0f : pl[q];
          rec.plane_normal[q] = stale ? 0.0f : pl[3 + q];
        }
      }
    }
  }
  hl_sync();
}

// one inside-hull pair per wave, persistent over the hull queue; a build
// beyond this variant's caps goes to the retry queue (k_qhull_big)
__device__ inline void q2_body(const HullArgs& A, Q2L& L) {
  const int lane = threadIdx.x & 63;
  const int HNP = A.H * A.NP;
  const Q2W W = q2_worker(A.qscratch + (size_t)(A.block_base + blockIdx.x) * A.qstride, HNP);
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
    const int n = hull_points(A, L, Ti, Ni, xi, xj, vrel, W.Pr, W.Pf);
    Q2S S;
#ifdef LQRO_QHULL_PROFILE
    for (int k = 0; k < 12; k++) S.tph[k] = 0;
#endif
    S.status = 0;
    S.nalloc = 1;
    if (L.fail || n < 4) S.status = QHS_INPUT;
    else q2_build(W, S, L, n, lane);
    hl_sync();
    if (S.status & QHS_CAPACITY) {
      if (lane == 0) {
        const int r = atomicAdd(A.rcount, 1);
        if (r < A.cap) A.rqueue[r] = slot;
      }
      hl_sync();
      continue;
    }
#ifdef LQRO_QHULL_PROFILE
    unsigned long long tq_ = __builtin_amdgcn_s_memtime();
#endif
    q2_select(A, W, S, lane, xi, vrel, slot);
#ifdef LQRO_QHULL_PROFILE
    S.tph[10] = __builtin_amdgcn_s_memtime() - tq_;
    S.tph[11] = 1;
    if (A.prof && lane == 0)
      for (int k = 0; k < 12; k++) atomicAdd(&A.prof[k], S.tph[k]);
#endif
    if (A.ext_nf && lane == 0) *A.ext_nf = S.status;   // test hook: the build's status bits
    if (A.ext_facets) {                                  // test hook: the facet list in key order
      for (int f = 1 + lane; f < S.nalloc; f += 64) {
        if (!(W.F[f].flags & QF_LIVE)) continue;
        const unsigned k = W.key[f];
        int rank = 0, nl = 0;
        for (int g = 1; g < S.nalloc; g++)
          if (W.F[g].flags & QF_LIVE) { nl++; rank += W.key[g] < k; }
        if (rank < A.ext_max)
          for (int t = 0; t < 3; t++) A.ext_facets[3 * rank + t] = W.vpt[W.F[f].v[t]];
        if (rank == 0 && nl < A.ext_max) A.ext_facets[3 * nl] = -1;
      }
      hl_sync();
    }
  }
}

}  // namespace lqro
