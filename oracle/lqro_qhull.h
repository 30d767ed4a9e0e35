/* lqro_qhull.h — TEST INFRASTRUCTURE ONLY: Qhull's build order restated
 * (lqro_qhull.c).  Used by the oracle's reference-rule hull branch. */
#ifndef LQRO_QHULL_H
#define LQRO_QHULL_H

#ifdef __cplusplus
extern "C" {
#endif

/* status bits: why a hull is not reproduced (Qhull would merge facets) */
#define QHO_INPUT     1    /* < 4 points or no initial simplex */
#define QHO_COPLANAR  2    /* coplanar horizon facet / point near a new facet */
#define QHO_NONCONVEX 4    /* qh_checkzero: a new facet not clearly convex */
#define QHO_FLIPPED   8    /* a facet's plane faces the interior point */
#define QHO_NARROW    16   /* narrow initial simplex */
#define QHO_SINGULAR  32   /* nearly singular hyperplane (Gaussian elimination) */
#define QHO_TOPOLOGY  64   /* duplicate ridge / broken horizon */

typedef struct {
  int nfacets;       /* facets in Qhull's output order */
  int nvertices;
  int* fv;           /* nfacets x 3 point ids, Fv order (fv[3f] = newest vertex) */
  double* plane;     /* nfacets x 4: normal, offset (Qhull's doubles, unprinted) */
  int* facet_id;     /* Qhull's facet ids (creation order), for diagnostics */
  int status;        /* QHO_* bits; 0 = reproduced */
  /* build statistics (sizing the GPU restatement) */
  int st_addpoints, st_partition, st_horizon_max, st_horizon_sum, st_cop_max, st_old_append;
  int st_visible_max, st_new_max, st_partition_max, st_facets_created;
  double distround;  /* qh DISTround of the build (qh_detroundoff) */
} orc_qhull_out;

/* Qhull 2019.1 on n 3-d points (qconvex defaults).  Returns nfacets, or -1
 * with out->status set.  Free with orc_qhull_free. */
int  orc_qhull(const double* pts, int n, orc_qhull_out* out);
void orc_qhull_free(orc_qhull_out* out);
/* keep_going = 1: build on as if Qhull had not merged (diagnostics: how far
 * a merge-free build stays from Qhull's output); status still reports it */
int  orc_qhull_ex(const double* pts, int n, orc_qhull_out* out, int keep_going);

#ifdef __cplusplus
}
#endif
#endif
