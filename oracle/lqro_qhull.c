/*
 * lqro_qhull.c — TEST INFRASTRUCTURE ONLY (linked into oracle/liboracle.so).
 *
 * What the reference's convexHull (LQRObstacles.cpp:867-969) reads back from
 *     qconvex n  TO "Planes.txt"        < pointList.txt      (LQRO:879)
 *     qconvex Fv TO "facetVertices.txt" < pointList.txt      (LQRO:880)
 * is decided by Qhull's incremental build: the facet order of both files is
 * Qhull's facet list, and the first Fv vertex of a simplicial facet is its
 * NEWEST vertex (vertex sets are kept in decreasing vertex id).  The
 * reference takes min_f |n_f . (vrel - P[Fv_f[0]])| over that order with a
 * strict '<' and leaves `normal` untouched when facet 0 wins (LQRO:955-968).
 *
 * qconvex.exe (Qhull 2012.1, Win32) is not run here.  SURVEY.md §8c names
 * scipy's bundled qhull_r 7.3.2 (2019.1.r 2019/06/21) as its stand-in: it
 * reproduces the reference's own fixture (tests/golden/qhull) facet for
 * facet, first vertices included.  This file restates the 2019.1 algorithm
 * for 3-d input with qconvex's default options ("C-0" pre-merge, zero
 * centrum; no 'Qt') — the functions below carry Qhull's names (libqhull_r:
 * geom_r.c, geom2_r.c, poly_r.c, poly2_r.c, libqhull_r.c, merge_r.c) — and
 * is pinned against that library, called like qconvex (tests/golden/
 * qhull_lib.py), by tests/test_qhull_order.py: facet order, every facet's
 * vertex list in Fv order, and the facet planes bit for bit.
 *
 * Scope: the general-position build.  Everything Qhull would resolve by
 * merging facets (a coplanar horizon facet, a new facet not clearly convex
 * against a neighbour (qh_checkzero), a flipped facet, a narrow initial
 * simplex, a nearly singular hyperplane, a duplicate ridge) is DETECTED and
 * reported as a status bit instead of restated: the caller treats such a
 * hull as "not reproduced" (counted; the GPU path does the same).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lqro_qhull.h"

#define REALepsilon DBL_EPSILON
#define REALmax DBL_MAX
#define REALmin DBL_MIN
#define qh_RATIOmaxsimplex 1.0e-3
#define qh_MAXnarrow -0.99999999

typedef struct {
  int prev, next;       /* facet list (ids); the tail sentinel is facet 0 */
  int v[3];             /* vertex ids, decreasing (Qhull's sorted vertex set) */
  int nb[3];            /* nb[k] is the neighbour opposite v[k] */
  double n[3], off;
  double furthestdist;
  int* os;              /* outside set (point ids), last = furthest */
  int os_n, os_cap;
  int replace;          /* f.replace */
  unsigned visitid;
  unsigned char top, visible, isnew, flipped, deleted;
} QF;

typedef struct {
  const double* P;      /* points, n x 3 */
  int n;
  QF* F;
  int nf, fcap;
  int* vpt;             /* vertex id -> point id */
  int nv, vcap;
  int facet_list, facet_tail, facet_next, newfacet_list, visible_list;
  unsigned visit_id;
  double MAXabs_coord, MAXsumcoord, MAXwidth, NEARzero[3];
  double DISTround, MINvisible, MAXcoplanar, MINoutside, MINdenom, MINdenom_2;
  double max_outside;
  double interior[3];
  int findbestnew, findbest_notsharp;
  int status;
  int keep_going;       /* diagnostics: build on past a merge condition */
  /* scratch */
  int* horizon_buf;
  int hcap;
  orc_qhull_out* st;    /* statistics */
} QH;

/* ---- sets / lists (poly_r.c: qh_appendfacet, qh_removefacet, qh_prependfacet) ---- */
static void os_append(QF* f, int p) {
  if (f->os_n == f->os_cap) {
    f->os_cap = f->os_cap ? 2 * f->os_cap : 8;
    f->os = (int*)realloc(f->os, sizeof(int) * (size_t)f->os_cap);
  }
  f->os[f->os_n++] = p;
}
static void os_append2ndlast(QF* f, int p) {   /* qh_setappend2ndlast */
  os_append(f, p);
  if (f->os_n >= 2) {
    const int t = f->os[f->os_n - 1];
    f->os[f->os_n - 1] = f->os[f->os_n - 2];
    f->os[f->os_n - 2] = t;
  }
}

static int new_facet(QH* q) {                   /* qh_newfacet */
  if (q->nf == q->fcap) {
    q->fcap *= 2;
    q->F = (QF*)realloc(q->F, sizeof(QF) * (size_t)q->fcap);
  }
  QF* f = &q->F[q->nf];
  memset(f, 0, sizeof *f);
  f->prev = f->next = -1;
  f->replace = -1;
  f->nb[0] = f->nb[1] = f->nb[2] = -1;
  f->isnew = 1;
  return q->nf++;
}

static int new_vertex(QH* q, int point) {      /* qh_newvertex */
  if (q->nv == q->vcap) {
    q->vcap *= 2;
    q->vpt = (int*)realloc(q->vpt, sizeof(int) * (size_t)q->vcap);
  }
  q->vpt[q->nv] = point;
  return q->nv++;
}

static void appendfacet(QH* q, int f) {
  const int tail = q->facet_tail;
  QF* F = q->F;
  if (tail == q->newfacet_list) {
    q->newfacet_list = f;
    if (tail == q->visible_list) q->visible_list = f;
  }
  if (tail == q->facet_next) q->facet_next = f;
  F[f].prev = F[tail].prev;
  F[f].next = tail;
  if (F[tail].prev >= 0) F[F[tail].prev].next = f;
  else q->facet_list = f;
  F[tail].prev = f;
}

static void removefacet(QH* q, int f) {
  QF* F = q->F;
  const int next = F[f].next, prev = F[f].prev;
  if (f == q->newfacet_list) q->newfacet_list = next;
  if (f == q->facet_next) q->facet_next = next;
  if (f == q->visible_list) q->visible_list = next;
  if (prev >= 0) {
    F[prev].next = next;
    F[next].prev = prev;
  } else {
    q->facet_list = next;
    F[next].prev = -1;
  }
}

static void prependfacet_next(QH* q, int f) {   /* qh_prependfacet(facet, &qh->facet_next) */
  QF* F = q->F;
  const int list = q->facet_next;
  const int prevfacet = F[list].prev;
  F[f].prev = prevfacet;
  if (prevfacet >= 0) F[prevfacet].next = f;
  F[list].prev = f;
  F[f].next = list;
  if (q->facet_list == list) q->facet_list = f;
  if (q->facet_next == list) q->facet_next = f;
}

/* ---- geometry (geom_r.c, geom2_r.c) ---- */
static inline double distplane(const QH* q, const double* p, int f) {   /* qh_distplane, dim 3 */
  const QF* F = &q->F[f];
  return F->off + p[0] * F->n[0] + p[1] * F->n[1] + p[2] * F->n[2];
}

#define det2_(a1, a2, b1, b2) ((a1) * (b2) - (a2) * (b1))
#define det3_(a1, a2, a3, b1, b2, b3, c1, c2, c3) \
  ((a1) * det2_(b2, b3, c2, c3) - (b1) * det2_(a2, a3, c2, c3) + (c1) * det2_(a2, a3, b2, b3))

/* qh_gausselim + qh_backnormal + qh_normalize2 for the 2 x 3 system of
 * qh_sethyperplane_gauss (dim 3): rows = {P1 - P0, P2 - P0} */
static void sethyperplane_gauss(QH* q, const double* r0, const double* r1, const double* r2, int toporient,
                                double* normal, double* offset) {
  double ra[3] = {r1[0] - r0[0], r1[1] - r0[1], r1[2] - r0[2]};
  double rb[3] = {r2[0] - r0[0], r2[1] - r0[1], r2[2] - r0[2]};
  double* rows[2] = {ra, rb};
  int sign = toporient;
  /* qh_gausselim(rows, 2, 3, &sign, &nearzero) */
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
    if (pivot_abs <= q->NEARzero[k]) {
      q->status |= QHO_SINGULAR;   /* nearly singular: Qhull re-orients (not restated) */
      if (pivot_abs == 0.0) continue;
    }
    const double* pivotrow = rows[k] + k;
    const double pivot = *pivotrow++;
    for (int i = k + 1; i < 2; i++) {
      double* ai = rows[i] + k;
      const double* ak = pivotrow;
      const double nn = (*ai++) / pivot;
      for (int j = 3 - (k + 1); j--;) *ai++ -= nn * *ak++;
    }
  }
  for (int k = 2; k--;)      /* for (k=dim-1; k--; ): the diagonals k = 1, 0 */
    if (rows[k][k] < 0) sign ^= 1;
  /* qh_backnormal(rows, 2, 3, sign, normal) */
  normal[2] = sign ? -1.0 : 1.0;
  for (int i = 2; i--;) {
    double acc = 0.0;
    const double* ai = rows[i] + i + 1;
    const double* ak = normal + i + 1;
    for (int j = i + 1; j < 3; j++) acc -= *ai++ * *ak++;
    const double diagonal = rows[i][i];
    if (fabs(diagonal) > q->MINdenom_2) acc /= diagonal;
    else q->status |= QHO_SINGULAR;
    normal[i] = acc;
  }
  /* qh_normalize2(normal, 3, True) */
  const double norm = sqrt(normal[0] * normal[0] + normal[1] * normal[1] + normal[2] * normal[2]);
  if (norm > q->MINdenom) {
    normal[0] /= norm;
    normal[1] /= norm;
    normal[2] /= norm;
  } else {
    q->status |= QHO_SINGULAR;
  }
  double off = -(r0[0] * normal[0]);
  off -= r0[1] * normal[1];
  off -= r0[2] * normal[2];
  *offset = off;
}

/* qh_setfacetplane -> qh_sethyperplane_det (dim 3) -> qh_normalize2, the
 * Gaussian-elimination retry when a vertex is off the determinant plane by
 * more than DISTround, then the flipped test of qh_checkflipped(qh_ALL) */
static void setfacetplane(QH* q, int f) {
  QF* F = &q->F[f];
  const double* r0 = q->P + 3 * (size_t)q->vpt[F->v[0]];
  const double* r1 = q->P + 3 * (size_t)q->vpt[F->v[1]];
  const double* r2 = q->P + 3 * (size_t)q->vpt[F->v[2]];
  const double dX10 = r1[0] - r0[0], dY10 = r1[1] - r0[1], dZ10 = r1[2] - r0[2];
  const double dX20 = r2[0] - r0[0], dY20 = r2[1] - r0[1], dZ20 = r2[2] - r0[2];
  double n0 = det2_(dY20, dZ20, dY10, dZ10);
  double n1 = det2_(dX10, dZ10, dX20, dZ20);
  double n2 = det2_(dX20, dY20, dX10, dY10);
  double norm = sqrt(n0 * n0 + n1 * n1 + n2 * n2);
  if (norm > q->MINdenom) {
    if (!F->top) norm = -norm;
    n0 /= norm;
    n1 /= norm;
    n2 /= norm;
  } else {
    q->status |= QHO_SINGULAR;
  }
  F->n[0] = n0; F->n[1] = n1; F->n[2] = n2;
  F->off = -(r0[0] * n0 + r0[1] * n1 + r0[2] * n2);
  /* nearzero: rows scanned i = 2, 1 (point0 skipped) */
  int nearzero = 0;
  const double* rr[2] = {r2, r1};
  for (int i = 0; i < 2 && !nearzero; i++) {
    const double d = F->off + (rr[i][0] * n0 + rr[i][1] * n1 + rr[i][2] * n2);
    if (d > q->DISTround || d < -q->DISTround) nearzero = 1;
  }
  if (nearzero) sethyperplane_gauss(q, r0, r1, r2, F->top, F->n, &F->off);
  const double di = distplane(q, q->interior, f);
  F->flipped = di >= -q->DISTround;
}

/* qh_detsimplex + qh_determinant for dim 2, 3 */
static double detsimplex(const QH* q, const double* apex, const int* simplex, int dim, int* nearzero) {
  double rows[3][3];
  for (int i = 0; i < dim; i++)
    for (int k = 0; k < dim; k++) rows[i][k] = q->P[3 * (size_t)simplex[i] + k] - apex[k];
  double det;
  if (dim == 2) {
    det = det2_(rows[0][0], rows[0][1], rows[1][0], rows[1][1]);
    *nearzero = fabs(det) < 10 * q->NEARzero[1];
  } else {
    det = det3_(rows[0][0], rows[0][1], rows[0][2], rows[1][0], rows[1][1], rows[1][2], rows[2][0], rows[2][1],
                rows[2][2]);
    *nearzero = fabs(det) < 10 * q->NEARzero[2];
  }
  return det;
}

/* qh_maxmin: maxpoints = [min0, max0, min1, max1, min2, max2]; the extents
 * that set the roundoff constants */
static void maxmin(QH* q, int* maxpoints) {
  q->max_outside = 0.0;
  q->MAXabs_coord = 0.0;
  q->MAXwidth = -REALmax;
  q->MAXsumcoord = 0.0;
  for (int k = 0; k < 3; k++) {
    int mn = 0, mx = 0;
    for (int p = 0; p < q->n; p++) {
      const double c = q->P[3 * (size_t)p + k];
      if (q->P[3 * (size_t)mx + k] < c) mx = p;
      else if (q->P[3 * (size_t)mn + k] > c) mn = p;
    }
    const double maxk = q->P[3 * (size_t)mx + k], mink = q->P[3 * (size_t)mn + k];
    const double maxcoord = fmax(maxk, -mink);
    const double temp = maxk - mink;
    if (temp > q->MAXwidth) q->MAXwidth = temp;
    if (maxcoord > q->MAXabs_coord) q->MAXabs_coord = maxcoord;
    q->MAXsumcoord += maxcoord;
    maxpoints[2 * k] = mn;
    maxpoints[2 * k + 1] = mx;
    q->NEARzero[k] = 80 * q->MAXsumcoord * REALepsilon;
  }
}

/* qh_detroundoff for the default options (C-0: premerge_centrum 0) */
static void detroundoff(QH* q) {
  double maxdistsum = sqrt(3.0) * q->MAXabs_coord;
  if (q->MAXsumcoord < maxdistsum) maxdistsum = q->MAXsumcoord;
  q->DISTround = REALepsilon * (3 * maxdistsum * 1.01 + q->MAXabs_coord);   /* qh_distround */
  const double MINdenom_1 = fmax(1.0 / REALmax, REALmin);
  q->MINdenom = MINdenom_1 * q->MAXabs_coord;
  q->MINdenom_2 = sqrt(MINdenom_1 * 3) * q->MAXabs_coord;
  const double premerge_centrum = 0.0 + 2 * q->DISTround;
  q->MINvisible = premerge_centrum;          /* hull_dim <= 3 */
  q->MAXcoplanar = q->MINvisible;
  q->MINoutside = 2 * q->MINvisible;
}

static int in_set(const int* s, int n, int p) {
  for (int i = 0; i < n; i++)
    if (s[i] == p) return 1;
  return 0;
}

/* qh_maxsimplex (2019.1) for dim 3 */
static int maxsimplex(QH* q, const int* maxpoints, int* simplex) {
  int ns = 0;
  double maxcoord = -REALmax, mincoord = REALmax;
  int minx = -1, maxx = -1;
  for (int i = 0; i < 6; i++) {
    const int p = maxpoints[i];
    const double c = q->P[3 * (size_t)p];
    if (maxcoord < c) { maxcoord = c; maxx = p; }
    if (mincoord > c) { mincoord = c; minx = p; }
  }
  double maxdet = maxcoord - mincoord;
  simplex[ns++] = minx;                      /* qh_setunique */
  if (maxx != minx) simplex[ns++] = maxx;
  if (ns < 2) return -1;
  for (int i = ns; i < 4; i++) {
    const double prevdet = maxdet;
    int maxpoint = -1, maxnearzero = 0, nearzero;
    maxdet = -1.0;
    for (int m = 0; m < 6; m++) {
      const int p = maxpoints[m];
      if (!in_set(simplex, i, p) && p != maxpoint) {
        double det = detsimplex(q, q->P + 3 * (size_t)p, simplex, i, &nearzero);
        if ((det = fabs(det)) > maxdet) { maxdet = det; maxpoint = p; maxnearzero = nearzero; }
      }
    }
    int maybe_falsenarrow = 0;
    const double targetdet = prevdet * q->MAXwidth;
    if (maxdet > 0.0 && maxdet / targetdet < qh_RATIOmaxsimplex) maybe_falsenarrow = 1;
    if (maxpoint < 0 || maxnearzero || maybe_falsenarrow) {
      for (int p = 0; p < q->n; p++) {
        if (!in_set(maxpoints, 6, p) && !in_set(simplex, i, p)) {
          double det = detsimplex(q, q->P + 3 * (size_t)p, simplex, i, &nearzero);
          if ((det = fabs(det)) > maxdet) { maxdet = det; maxpoint = p; maxnearzero = nearzero; }
        }
      }
    }
    if (maxpoint < 0) return -1;
    simplex[i] = maxpoint;
  }
  return 0;
}

/* ---- point location (geom_r.c: qh_findbest, qh_findbestnew, qh_findbesthorizon) ---- */
static int findbesthorizon(QH* q, const double* point, int startfacet, double* bestdist) {
  QF* F = q->F;
  int bestfacet = startfacet;
  const double searchdist = q->max_outside + 2 * q->DISTround + fmax(q->MINvisible, q->MAXcoplanar);
  double minsearch = *bestdist - searchdist;
  const unsigned visitid = ++q->visit_id;
  int* cop = q->horizon_buf;               /* qh.coplanarfacetset */
  int ncop = 0;
  int nextfacet = -1, nvisit = 0;
  F[startfacet].visitid = visitid;
  int facet = startfacet;
  for (;;) {
    for (int k = 0; k < 3; k++) {
      const int nb = F[facet].nb[k];
      if (F[nb].visitid == visitid) continue;
      F[nb].visitid = visitid;
      nvisit++;
      if (!F[nb].flipped) {
        const double dist = distplane(q, point, nb);
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
        if (ncop == q->hcap) {
          q->hcap *= 2;
          q->horizon_buf = cop = (int*)realloc(cop, sizeof(int) * (size_t)q->hcap);
        }
        cop[ncop++] = nextfacet;
      }
      nextfacet = nb;
    }
    if (ncop > q->st->st_cop_max) q->st->st_cop_max = ncop;
    facet = nextfacet;
    if (facet >= 0) nextfacet = -1;
    else if (!ncop) break;
    else if (ncop == 1) { facet = cop[0]; ncop = 0; }
    else facet = cop[--ncop];
  }
  if (nvisit > q->st->st_horizon_max) q->st->st_horizon_max = nvisit;
  q->st->st_horizon_sum += nvisit;
  return bestfacet;
}

static int findbestnew(QH* q, const double* point, int startfacet, double* dist, int bestoutside,
                       int* isoutside) {
  QF* F = q->F;
  double bestdist = -REALmax / 2;
  int bestfacet = -1;
  const unsigned visitid = ++q->visit_id;
  const int isdistoutside = !bestoutside;
  const double distoutside = fmax(2 * q->MINoutside, q->max_outside);   /* qh_DISToutside */
  *isoutside = 1;
  for (int i = 0, facet = startfacet; i < 2; i++, facet = q->newfacet_list) {
    for (int f = facet; f >= 0 && F[f].next >= 0; f = F[f].next) {
      if (f == startfacet && i) break;
      F[f].visitid = visitid;
      if (!F[f].flipped) {
        *dist = distplane(q, point, f);
        if (*dist > bestdist) {
          bestfacet = f;
          if (isdistoutside && *dist >= distoutside) return bestfacet;
          bestdist = *dist;
        }
      }
    }
  }
  bestfacet = findbesthorizon(q, point, bestfacet >= 0 ? bestfacet : startfacet, &bestdist);
  *dist = bestdist;
  if (*dist < q->MINoutside) *isoutside = 0;
  return bestfacet;
}

static int sharpnewfacets(QH* q) {
  QF* F = q->F;
  int quadrant[3];
  for (int f = q->newfacet_list; f >= 0 && F[f].next >= 0; f = F[f].next) {
    if (f == q->newfacet_list) {
      for (int k = 3; k--;) quadrant[k] = F[f].n[k] > 0;
    } else {
      for (int k = 3; k--;)
        if (quadrant[k] != (F[f].n[k] > 0)) return 1;
    }
  }
  return 0;
}

/* qh_findbest(point, startfacet, bestoutside=False, isnewfacets=True, noupper=False) */
static int findbest_new(QH* q, const double* point, int startfacet, double* dist, int* isoutside) {
  QF* F = q->F;
  double bestdist = -REALmax / 2;
  int bestfacet = -1;
  const unsigned visitid = ++q->visit_id;
  *isoutside = 1;
  if (!F[startfacet].flipped) {
    *dist = distplane(q, point, startfacet);
    if (*dist >= q->MINoutside) return startfacet;
    bestdist = *dist;
    bestfacet = startfacet;
  }
  F[startfacet].visitid = visitid;
  int facet = startfacet;
  while (facet >= 0) {
    int nb = -1;
    for (int k = 0; k < 3; k++) {
      nb = F[facet].nb[k];
      if (!F[nb].isnew) { nb = -1; continue; }
      if (F[nb].visitid == visitid) { nb = -1; continue; }
      F[nb].visitid = visitid;
      if (!F[nb].flipped) {
        *dist = distplane(q, point, nb);
        if (*dist > bestdist) {
          if (*dist >= q->MINoutside) return nb;
          bestfacet = nb;
          bestdist = *dist;
          break;
        }
      }
      nb = -1;
    }
    facet = nb;
  }
  if (bestfacet < 0) {
    bestdist = -REALmax / 2;
    bestfacet = findbestnew(q, point, q->newfacet_list, &bestdist, 0, isoutside);
    *dist = bestdist;
    return bestfacet;
  }
  if (!q->findbest_notsharp && bestdist < -q->DISTround) {
    if (sharpnewfacets(q)) {
      bestfacet = findbestnew(q, point, bestfacet, &bestdist, 0, isoutside);
      q->findbestnew = 1;
      *dist = bestdist;
      return bestfacet;
    }
    q->findbest_notsharp = 1;
  }
  bestfacet = findbesthorizon(q, point, bestfacet, &bestdist);
  *dist = bestdist;
  if (bestdist < q->MINoutside) *isoutside = 0;
  return bestfacet;
}

/* qh_partitioncoplanar without KEEPcoplanar: only qh.max_outside moves */
static void partitioncoplanar(QH* q, const double* point, int facet, double* distp) {
  double bestdist;
  if (!distp) {
    int isout;
    findbestnew(q, point, facet, &bestdist, 1, &isout);
    if (bestdist < -q->MAXcoplanar) return;
    q->status |= QHO_COPLANAR;   /* a deleted vertex near a new facet: not restated */
    return;
  }
  bestdist = *distp;
  if (bestdist > q->max_outside) q->max_outside = bestdist;
}

/* qh_partitionpoint */
static void partitionpoint(QH* q, int pid, int facet) {
  const double* point = q->P + 3 * (size_t)pid;
  double bestdist;
  int isoutside;
  int bestfacet = q->findbestnew ? findbestnew(q, point, facet, &bestdist, 0, &isoutside)
                                 : findbest_new(q, point, facet, &bestdist, &isoutside);
  QF* B = &q->F[bestfacet];
  q->st->st_partition++;
  if (isoutside) {
    if (!B->os_n) {
      os_append(B, pid);
      if (!B->isnew) {            /* make sure it's after qh.facet_next */
        q->st->st_old_append++;
        removefacet(q, bestfacet);
        appendfacet(q, bestfacet);
      }
      B->furthestdist = bestdist;
    } else if (B->furthestdist < bestdist) {
      os_append(B, pid);
      B->furthestdist = bestdist;
    } else {
      os_append2ndlast(B, pid);
    }
  } else if (bestdist >= -q->MAXcoplanar) {
    if (bestdist > q->max_outside) partitioncoplanar(q, point, bestfacet, &bestdist);
  }
}

/* ---- the build (libqhull_r.c: qh_qhull, qh_buildhull, qh_addpoint; poly*_r.c) ---- */
static void findhorizon(QH* q, const double* point, int facet) {
  QF* F = q->F;
  removefacet(q, facet);
  appendfacet(q, facet);
  F[facet].visible = 1;
  F[facet].replace = -1;
  q->visible_list = facet;
  const unsigned vid = ++q->visit_id;
  F[facet].visitid = vid;
  for (int vis = q->visible_list; vis >= 0 && F[vis].visible; vis = F[vis].next) {
    F[vis].visitid = vid;
    for (int k = 0; k < 3; k++) {
      const int nb = F[vis].nb[k];
      if (F[nb].visitid == vid) continue;
      F[nb].visitid = vid;
      const double dist = distplane(q, point, nb);
      if (dist >= q->MINvisible) {
        removefacet(q, nb);
        appendfacet(q, nb);
        F[nb].visible = 1;
        F[nb].replace = -1;
      } else if (dist >= -q->MAXcoplanar) {
        q->status |= QHO_COPLANAR;   /* coplanar horizon: Qhull merges */
      }
    }
  }
}

/* qh_checkzero(!qh_ALL) on the new facets: "clearly convex" or a pre-merge */
static void checkzero_new(QH* q) {
  QF* F = q->F;
  for (int f = q->newfacet_list; f >= 0 && F[f].next >= 0; f = F[f].next)
    if (F[f].flipped) { q->status |= QHO_FLIPPED; return; }
  for (int f = q->newfacet_list; f >= 0 && F[f].next >= 0; f = F[f].next) {
    for (int k = 1; k < 3; k++) {
      const int nb = F[f].nb[k];
      const double d = distplane(q, q->P + 3 * (size_t)q->vpt[F[f].v[k]], nb);
      if (d >= -2 * q->DISTround) { q->status |= QHO_NONCONVEX; return; }
    }
    const int hz = F[f].nb[0];
    for (int k = 0; k < 3; k++) {
      const int v = F[hz].v[k];
      if (v != F[f].v[0] && v != F[f].v[1] && v != F[f].v[2]) {
        const double d = distplane(q, q->P + 3 * (size_t)q->vpt[v], f);
        if (d >= -2 * q->DISTround) { q->status |= QHO_NONCONVEX; return; }
        break;
      }
    }
  }
}

static void addpoint(QH* q, int furthest, int facet) {
  QF* F;
  q->st->st_addpoints++;
  const double* point = q->P + 3 * (size_t)furthest;
  findhorizon(q, point, facet);
  /* qh_makenewfacets -> qh_makenew_simplicial */
  q->newfacet_list = q->facet_tail;
  const int apex = new_vertex(q, furthest);
  for (int vis = q->visible_list; vis >= 0 && q->F[vis].visible; vis = q->F[vis].next) {
    int newfacet = -1;
    for (int k = 0; k < 3; k++) {
      F = q->F;
      const int nb = F[vis].nb[k];
      if (F[nb].visible) continue;
      /* qh_facetintersect(neighbor, visible): skips */
      int hskip = -1;
      for (int s = 0; s < 3; s++)
        if (F[nb].nb[s] == vis) { hskip = s; break; }
      if (hskip < 0) { q->status |= QHO_TOPOLOGY; return; }
      const int top = F[nb].top ? (hskip & 1) : ((hskip & 1) ^ 1);
      int vs[2], m = 0;
      for (int s = 0; s < 3; s++)
        if (s != hskip) vs[m++] = F[nb].v[s];
      const int nf = new_facet(q);
      F = q->F;
      F[nf].v[0] = apex; F[nf].v[1] = vs[0]; F[nf].v[2] = vs[1];
      F[nf].top = (unsigned char)top;
      F[nf].nb[0] = nb;
      appendfacet(q, nf);
      F[nb].nb[hskip] = nf;
      newfacet = nf;
    }
    q->F[vis].replace = newfacet;
  }
  F = q->F;
  /* qh_matchnewfacets: nb[1] shares {apex, v2}, nb[2] shares {apex, v1} */
  {
    int cnt = 0, nvis = 0;
    for (int f = q->newfacet_list; f >= 0 && F[f].next >= 0; f = F[f].next) cnt++;
    for (int f = q->visible_list; f >= 0 && F[f].visible; f = F[f].next) nvis++;
    if (cnt > q->st->st_new_max) q->st->st_new_max = cnt;
    if (nvis > q->st->st_visible_max) q->st->st_visible_max = nvis;
    for (int f = q->newfacet_list; f >= 0 && F[f].next >= 0; f = F[f].next) {
      for (int k = 1; k < 3; k++) {
        const int w = F[f].v[3 - k];       /* the vertex shared with nb[k] besides the apex */
        int found = -1, dup = 0;
        for (int g = q->newfacet_list; g >= 0 && F[g].next >= 0; g = F[g].next) {
          if (g == f) continue;
          if (F[g].v[1] == w || F[g].v[2] == w) {
            if (found >= 0) dup = 1;
            found = g;
          }
        }
        if (found < 0 || dup) { q->status |= QHO_TOPOLOGY; return; }
        F[f].nb[k] = found;
      }
    }
    (void)cnt;
  }
  /* qh_makenewplanes */
  for (int f = q->newfacet_list; f >= 0 && F[f].next >= 0; f = F[f].next) setfacetplane(q, f);
  /* qh_premerge: qh_checkzero fast path */
  checkzero_new(q);
  if (q->status && !q->keep_going) return;
  /* qh_partitionvisible */
  q->findbestnew = 0;
  for (int vis = q->visible_list; vis >= 0 && q->F[vis].visible; vis = q->F[vis].next) {
    QF* V = &q->F[vis];
    if (!V->os_n) continue;
    int newfacet = V->replace;
    while (newfacet >= 0 && q->F[newfacet].visible) newfacet = q->F[newfacet].replace;
    if (newfacet < 0) newfacet = q->newfacet_list;
    int* pts = V->os;
    const int np = V->os_n;
    if (np > q->st->st_partition_max) q->st->st_partition_max = np;
    V->os = NULL; V->os_n = V->os_cap = 0;
    for (int i = 0; i < np; i++) partitionpoint(q, pts[i], newfacet);
    free(pts);
  }
  /* deleted vertices: qh_partitioncoplanar(point, newfacet_list, NULL, qh_ALL) */
  {
    F = q->F;
    for (int vis = q->visible_list; vis >= 0 && F[vis].visible; vis = F[vis].next) {
      for (int k = 0; k < 3; k++) {
        const int v = F[vis].v[k];
        int onnew = 0;
        for (int f = q->newfacet_list; f >= 0 && F[f].next >= 0 && !onnew; f = F[f].next)
          onnew = F[f].v[1] == v || F[f].v[2] == v;
        if (!onnew) partitioncoplanar(q, q->P + 3 * (size_t)q->vpt[v], q->newfacet_list, NULL);
        F = q->F;
      }
    }
  }
  q->findbestnew = 0;
  q->findbest_notsharp = 0;
  /* qh_deletevisible */
  F = q->F;
  for (int vis = q->visible_list, nx; vis >= 0 && F[vis].visible; vis = nx) {
    nx = F[vis].next;
    removefacet(q, vis);
    F[vis].deleted = 1;
    free(F[vis].os);
    F[vis].os = NULL;
    F[vis].os_n = 0;
  }
  /* qh_resetlists */
  for (int f = q->newfacet_list; f >= 0 && F[f].next >= 0; f = F[f].next) F[f].isnew = 0;
  q->newfacet_list = -1;
  q->visible_list = -1;
}

int orc_qhull(const double* pts, int n, orc_qhull_out* out) { return orc_qhull_ex(pts, n, out, 0); }

int orc_qhull_ex(const double* pts, int n, orc_qhull_out* out, int keep_going) {
  memset(out, 0, sizeof *out);
  out->status = 0;
  if (n < 4) { out->status = QHO_INPUT; return -1; }
  QH qs;
  QH* q = &qs;
  memset(q, 0, sizeof *q);
  q->P = pts;
  q->n = n;
  q->keep_going = keep_going;
  q->st = out;
  q->fcap = 64;
  q->F = (QF*)malloc(sizeof(QF) * (size_t)q->fcap);
  q->vcap = 64;
  q->vpt = (int*)malloc(sizeof(int) * (size_t)q->vcap);
  q->hcap = 64;
  q->horizon_buf = (int*)malloc(sizeof(int) * (size_t)q->hcap);
  /* qh_initbuild: sentinels f0 (facet_tail), v0 (vertex_tail) */
  q->facet_tail = new_facet(q);
  q->F[q->facet_tail].isnew = 0;
  q->facet_list = q->facet_next = q->facet_tail;
  q->newfacet_list = q->visible_list = q->facet_tail;
  new_vertex(q, -1);
  int maxpoints[6], simplex[4];
  maxmin(q, maxpoints);
  detroundoff(q);
  if (maxsimplex(q, maxpoints, simplex)) { out->status = QHO_INPUT; goto done; }
  /* qh_initialvertices: vertices v1..v4 for simplex[0..3], set [v4, v3, v2, v1] */
  int vset[4];
  for (int i = 0; i < 4; i++) vset[3 - i] = new_vertex(q, simplex[i]);
  /* qh_createsimplex */
  {
    int fs[4];
    int top = 1;
    for (int i = 0; i < 4; i++) {
      const int f = new_facet(q);
      int m = 0;
      for (int s = 0; s < 4; s++)
        if (s != i) q->F[f].v[m++] = vset[s];
      q->F[f].top = (unsigned char)top;
      appendfacet(q, f);
      fs[i] = f;
      top ^= 1;
    }
    for (int i = 0; i < 4; i++) {
      int m = 0;
      for (int s = 0; s < 4; s++)
        if (s != i) q->F[fs[i]].nb[m++] = fs[s];
    }
    /* qh_resetlists */
    for (int i = 0; i < 4; i++) q->F[fs[i]].isnew = 0;
    q->newfacet_list = q->visible_list = -1;
    q->facet_next = q->facet_list;
    /* qh_getcenter over [v4, v3, v2, v1] */
    for (int k = 0; k < 3; k++) {
      double c = 0.0;
      for (int s = 0; s < 4; s++) c += q->P[3 * (size_t)q->vpt[vset[s]] + k];
      q->interior[k] = c / 4;
    }
    /* qh_initialhull: orientation from the first facet */
    setfacetplane(q, fs[0]);
    q->F[fs[0]].flipped = 0;
    if (distplane(q, q->interior, fs[0]) > q->DISTround)
      for (int i = 0; i < 4; i++) q->F[fs[i]].top ^= 1;
    for (int i = 0; i < 4; i++) setfacetplane(q, fs[i]);
    for (int i = 0; i < 4; i++)
      if (q->F[fs[i]].flipped) q->status |= QHO_FLIPPED;
    double minangle = REALmax;
    for (int i = 0; i < 4; i++)
      for (int s = 0; s < 3; s++) {
        const QF *a = &q->F[fs[i]], *b = &q->F[a->nb[s]];
        double angle = 0.0;
        for (int k = 0; k < 3; k++) angle += a->n[k] * b->n[k];
        if (angle < minangle) minangle = angle;
      }
    if (minangle < qh_MAXnarrow) q->status |= QHO_NARROW;
    if (q->status && !q->keep_going) goto done;
    /* qh_partitionall */
    int* pset = (int*)malloc(sizeof(int) * (size_t)n);
    int np = 0;
    for (int p = 0; p < n; p++)
      if (!in_set(simplex, 4, p)) pset[np++] = p;
    const double distoutside = fmax(2 * q->MINoutside, q->max_outside);
    for (int f = q->facet_list; f >= 0 && q->F[f].next >= 0; f = q->F[f].next) {
      QF* Fa = &q->F[f];
      int bestpoint = -1, point_end = 0;
      double bestdist = -REALmax;
      for (int i = 0; i < np; i++) {
        const int p = pset[i];
        const double dist = distplane(q, q->P + 3 * (size_t)p, f);
        if (dist < distoutside) {
          pset[point_end++] = p;
        } else if (bestpoint < 0) {
          bestpoint = p;
          bestdist = dist;
        } else if (dist > bestdist) {
          os_append(Fa, bestpoint);
          bestpoint = p;
          bestdist = dist;
        } else {
          os_append(Fa, p);
        }
      }
      if (bestpoint >= 0) {
        os_append(Fa, bestpoint);
        Fa->furthestdist = bestdist;
      }
      np = point_end;
    }
    /* MERGING: the rest through qh_partitionpoint with findbestnew */
    q->findbestnew = 1;
    q->newfacet_list = q->facet_tail;   /* no new facets: the scan covers the facet list */
    for (int i = 0; i < np; i++) partitionpoint(q, pset[i], q->facet_list);
    q->findbestnew = 0;
    q->newfacet_list = -1;
    free(pset);
  }
  /* qh_furthestnext */
  {
    int best = -1;
    double bd = -REALmax;
    for (int f = q->facet_list; f >= 0 && q->F[f].next >= 0; f = q->F[f].next)
      if (q->F[f].os_n && q->F[f].furthestdist > bd) { best = f; bd = q->F[f].furthestdist; }
    if (best >= 0) {
      removefacet(q, best);
      prependfacet_next(q, best);
    }
  }
  /* qh_buildhull */
  q->facet_next = q->facet_list;
  for (;;) {
    /* qh_nextfurthest */
    int facet, furthest = -1;
    while ((facet = q->facet_next) != q->facet_tail) {
      if (!q->F[facet].os_n) {
        q->facet_next = q->F[facet].next;
        continue;
      }
      furthest = q->F[facet].os[--q->F[facet].os_n];
      break;
    }
    if (furthest < 0) break;
    addpoint(q, furthest, facet);
    if (q->status & (q->keep_going ? QHO_TOPOLOGY : ~0)) goto done;
  }
  /* output: the facet list in order (qh_printfacets) */
  if (!q->status || keep_going) {
    int cnt = 0;
    for (int f = q->facet_list; f >= 0 && q->F[f].next >= 0; f = q->F[f].next) cnt++;
    out->nfacets = cnt;
    out->fv = (int*)malloc(sizeof(int) * 3 * (size_t)(cnt ? cnt : 1));
    out->plane = (double*)malloc(sizeof(double) * 4 * (size_t)(cnt ? cnt : 1));
    out->facet_id = (int*)malloc(sizeof(int) * (size_t)(cnt ? cnt : 1));
    int i = 0;
    for (int f = q->facet_list; f >= 0 && q->F[f].next >= 0; f = q->F[f].next, i++) {
      for (int k = 0; k < 3; k++) out->fv[3 * i + k] = q->vpt[q->F[f].v[k]];
      for (int k = 0; k < 3; k++) out->plane[4 * i + k] = q->F[f].n[k];
      out->plane[4 * i + 3] = q->F[f].off;
      out->facet_id[i] = f;
    }
    out->nvertices = q->nv - 1;
  }
done:
  out->status |= q->status;
  out->distround = q->DISTround;
  out->st_facets_created = q->nf - 1;
  for (int f = 0; f < q->nf; f++) free(q->F[f].os);
  free(q->F);
  free(q->vpt);
  free(q->horizon_buf);
  if (keep_going && out->nfacets > 0 && !(out->status & QHO_TOPOLOGY)) return out->nfacets;
  return out->status ? -1 : out->nfacets;
}

void orc_qhull_free(orc_qhull_out* out) {
  free(out->fv);
  free(out->plane);
  free(out->facet_id);
  memset(out, 0, sizeof *out);
}
