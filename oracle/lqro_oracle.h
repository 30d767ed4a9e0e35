/*
 * lqro_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded CPU restatement of the reference's per-timestep
 * LQR-Obstacle path (hihixuyang/LQR-Obstacles, QuadrotorHoverController/
 * LQRObstacles.cpp = "LQRO", gjk.cpp = "GJK", include/matrix.h = "MAT",
 * Vector3.h = "V3").  Every function cites the reference lines it restates.
 *
 * Who may use it: tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg — as the checker / the timed CPU baseline only.  The
 * product (liblqro.so) never links, loads or calls anything here.
 *
 * Pinning: tests/test_oracle_vs_ref.py compares it bit-for-bit against the
 * reference's own functions compiled from /root/reference (oracle/_ref, see
 * oracle/Makefile) and against the hull fixture the reference ships
 * (pointList.txt / Planes.txt / facetVertices.txt); tests/golden/ holds the
 * vectors generated from oracle/_ref for use where /root/reference is absent.
 */
#ifndef LQRO_ORACLE_H
#define LQRO_ORACLE_H

#include <stdint.h>
#include "../include/lqro.h"   /* record / config / model layouts only */

#ifdef __cplusplus
extern "C" {
#endif

int  orc_version(void);

/* LQRO:169-189 + 1275-1286 + 559-561 (same numbers as lqro_model_default). */
void orc_model_default(lqro_model* m);

/* controlMatrices (LQRO:520-582) incl. linearizeDiscretize (LQRO:456-471),
 * f (LQRO:368-397), Jacobian_fx/fu (LQRO:421-441), exp (MAT:773-790).
 * X = 16, U = 4, V = 3.  `l` (LQRO:552,557) is not produced: it needs
 * pseudoInverse and is not read by the pair path. */
int  orc_synthesize(const lqro_model* m, double* A, double* B, double* c,
                    double* L, double* E, double* Lh, double* Eh);
/* the same for x_dim 16 or 12 (BASELINE config 5's reduced model: no
 * rotor-force states, F = u); not in the reference (SURVEY §7 hazard 7) */
/* pseudoInverse (MAT:450-477) of a square n x n matrix, n <= 16 */
void orc_pinv(int n, const double* q, double* out);
int  orc_synthesize_x(const lqro_model* m, int x_dim, double* A, double* B, double* c,
                      double* L, double* E, double* l, double* Lh, double* Eh);

/* createSpheres (LQRO:735-750). */
void orc_sphere(int np, double xy_radius, double z_radius, double* s);

/* The per-agent horizon tables: findFG (LQRO:723-732) iterated H times from
 * F=I, G=0 (LQRO:1401-1404), and for every step k the two factors of
 * createObstacle (LQRO:771-773): T_k = !(C*G_k) (3x3) and NCF_k = (-C)*F_k
 * (3xX).  Depends on agent i only, never on j — computing it once per agent
 * is bit-identical to the reference's per-pair recomputation. */
int  orc_tables(int X, int U, int H, const double* A, const double* B,
                const double* L, const double* E, double* T /* H*9 */,
                double* NCF /* H*3*X */);

/* One ordered pair (i,j): LQRO:1401-1417 with the reference's operation
 * order.  Writes the record; if reach_idx != NULL it receives the reachable
 * point indices (k*NP+p order), if reach_pts != NULL their coordinates.
 * Returns 0, or LQRO_E_OVERFLOW/LQRO_E_ARG. */
int  orc_pair(int X, int H, int NP, int min_reach, double vmax_reach,
              const double* T, const double* NCF, const double* S,
              const double* xi, const double* xj, int i, int j,
              lqro_pair_record* rec, int32_t* reach_idx, double* reach_pts);

/* calculateNewV (LQRO:1223-1234) with linearProgram1-4 (LQRO:1001-1206),
 * fp32 Vector3 arithmetic (V3).  planes: m x {point[3], normal[3]} floats. */
long long orc_lp_chain(int m, const float* planes, const double* vgoal, double vmax_lp);
void orc_newv(int m, const float* planes, const double* vgoal, double vmax_lp,
              double* newv);

/* Whole step (LQRO:1393-1436): rows [r0,r1), all j.  Tables are per agent
 * (per_agent=1: T is N*H*9, NCF is N*H*3*X) or shared (per_agent=0).
 * recs: (r1-r0)*(N-1) records or NULL.  newv: N*3 (rows r0..r1 written). */
int  orc_step(int N, int X, int H, int NP, int min_reach, double vmax_reach,
              double vmax_lp, int per_agent, const double* T, const double* NCF,
              const double* S, const double* x, const double* vgoal,
              int r0, int r1, double* newv, lqro_pair_record* recs);

/* Opt-in neighbour culling for orc_step / orc_step_mt (RVO2 computeNeighbors,
 * AGT:74-81,153-174): max_nbr <= 0 restores all pairs.  Culled pairs get a
 * record with n_reach = -1 and no plane.  orc_neighbors: agent i's selection
 * (sel[j] = 1), RVO2's sorted insertion with a shrinking range. */
void orc_set_neighbors(double nbr_dist, int max_nbr);
void orc_neighbors(int N, int X, const double* x, int i, double r2, int k, unsigned char* sel);

/* Same as orc_step, rows split over `threads` POSIX threads (private
 * scratch per thread; the reference itself is single-threaded). */
int  orc_step_mt(int N, int X, int H, int NP, int min_reach, double vmax_reach,
                 double vmax_lp, int per_agent, const double* T, const double* NCF,
                 const double* S, const double* x, const double* vgoal,
                 int r0, int r1, double* newv, lqro_pair_record* recs, int threads);
/* orc_step_mt with the reference's per-pair cost structure: F, G, Transform
 * and -C*F recomputed per pair from A, B, L, E (LQRO:1401-1406, 723-732,
 * 770-773) and GJK run twice for an outside pair (LQRO:1410, 1414).  Results
 * are bit-identical to orc_step_mt; bench.py times it as the CPU baseline. */
int  orc_step_faithful_mt(int N, int X, int H, int NP, int min_reach, double vmax_reach,
                          double vmax_lp, int per_agent, const double* A, const double* B,
                          const double* L, const double* E, const double* S, const double* x,
                          const double* vgoal, int r0, int r1, double* newv,
                          lqro_pair_record* recs, int threads);

/* GJK restatement (GJK:296-501) for the path's call run_gjk (LQRO:814-853):
 * object 1 = the single point vrel, object 2 = pts[n][3].  Returns dist^2;
 * wpt1/wpt2 = witnesses; iters/simplex as in lqro_pair_record. */
double orc_gjk(const double vrel[3], int n, const double* pts, double wpt1[3],
               double wpt2[3], int* iters, int* simplex_n, int simplex[4],
               int* backup);

/* Hull branch (LQRO:867-969 + qconvex): hull of the %g-rounded points
 * (LQRO:871-873), then min_f |n_f . (vrel - P[v_f])| over facets.  Qhull's
 * facet order and per-facet first vertex are history-dependent artefacts of
 * qconvex; this restatement uses the canonical facet order (sorted vertex
 * triples) and the lowest-index vertex of each facet.
 * Returns number of facets (<=0 on failure). */
int  orc_hull_branch(int n, const double* pts_full, const double vrel[3],
                     double* dist, double normal[3], int facet[3]);

/* The reference's own rule over Qhull's output (lqro_qhull.c): facets in
 * Qhull's order, first Fv vertex, strict '<' (LQRO:925-968).  *stale = 1 when
 * facet 0 wins (normal untouched, LQRO:956-958); *qstatus = QHO_* bits of a
 * hull Qhull would merge (built merge-free).  Returns the facet count. */
int  orc_hull_branch_ref(int n, const double* pts_full, const double vrel[3], double* dist,
                         double normal[3], int facet[3], int* stale, int* qstatus);
/* rule 0: the canonical rule above (default); 1: the reference's rule for
 * orc_pair / orc_step*, with the loop-carried normalVector resolved in row
 * order from the carry (set/get: the value entering / leaving a step's
 * rows).  round16: planes read back as qconvex prints them (%.16g). */
void orc_set_hull_rule(int rule, int round16);
/* thread-time spent in the hull branch and inside-hull pairs (all threads)
 * since the last reset */
void orc_hull_time(double* seconds, long long* count, int reset);
void orc_set_carry_normal(const double* n);
void orc_get_carry_normal(double* n);

/* Full hull of n points (no rounding applied here): writes up to cap facets
 * as outward-oriented index triples; returns the facet count or <0. */
int  orc_hull(int n, const double* pts, int32_t* facets, int cap);

/* %g (6 significant digits) round trip of one double: what qconvex reads
 * back from pointList.txt (LQRO:871-873). */
/* operator! (MAT:603-671) on 3x3 / 4x4 row-major matrices. */
void orc_inverse3(const double* in, double* out);
void orc_inverse4(const double* in, double* out);

double orc_round6(double v);

/* quatFromRot (stdafx.h:24-33); Quadrotor::visualize's keyframe (LQRO:128-133):
 * out[8] = (float) t, (float) xTrue[0..2], (float) quatFromRot(RotTrue). */
void orc_quat_from_rot(const double* R, double* q);
void orc_keyframe(double t, const double* xTrue, const double* RTrue, float* out);

/* ---- the per-agent step after the pair loop (LQRO:1437-1446) ----------- */
/* jacobi (MAT:674-759) on an n x n symmetric matrix (n <= 16). */
void orc_jacobi(int n, const double* m, double* V, double* D);
/* riccatiControllerSteady (LQRO:594-617) -> u (4). */
void orc_control_velocity(const double* x, const double* R0, const double* vGoal,
                          const double* uGoal, const double* L, const double* E,
                          const double* l, double* u);
/* riccatiControllerSteadyPosition (LQRO:619-645) -> v (3). */
void orc_control_position(const double* x, const double* R0, const double* pGoal,
                          const double* uGoal, const double* Lh, const double* Eh, double* v);
/* propagate (LQRO:473-486); nrm = the 16 normal() draws of its sampleGaussian. */
void orc_propagate(const lqro_model* m, double* x, double* R, const double* u, const double* M,
                   const double* nrm);
/* kalmanFilter1 (LQRO:488-505), kalmanFilter2 (LQRO:507-518). */
void orc_kalman1(const lqro_model* m, double* x, double* R, const double* u, const double* M,
                 double* P);
void orc_kalman2(const lqro_model* m, double* x, double* R, const double* z, const double* N,
                 double* P);
/* One agent through LQRO:1438-1445: findU, propagateU, kalmanFilter1, the
 * observation draw (LQRO:1442), kalmanFilter2, findVGoal.  nrm: 22 draws
 * (16 propagate, 6 observation).  vgoal: in newV, out the new vGoal. */
void orc_agent_step(const lqro_model* m, const double* L, const double* E, const double* l,
                    const double* Lh, const double* Eh, const double* uGoal, const double* pGoal,
                    const double* M, const double* N, const double* nrm, double* x, double* R,
                    double* xTrue, double* RTrue, double* P, double* vgoal, double* u_out);

#ifdef __cplusplus
}
#endif
#endif
