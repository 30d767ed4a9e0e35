/*
 * ref_harness.cpp — TEST INFRASTRUCTURE ONLY.
 *
 * Compiles the reference's OWN per-pair path functions (extracted verbatim
 * from /root/reference by extract_ref.sh into oracle/_ref/, never committed)
 * together with the reference's headers (include/matrix.h, gjk.h, Vector3.h)
 * and gjk.cpp, and exposes them through a small C API for the tests.  The
 * drivers below re-enact the body of the reference's pair loop
 * (LQRO:1401-1417, 1435) by calling the reference functions in the same order;
 * they contain no arithmetic of their own.
 *
 * Not reproducible here: convexHull (LQRO:867-969) shells out to qconvex.exe,
 * a Win32 binary; ref_pair reports inside-hull pairs and stops there.
 */
#include <math.h>     /* first: ::abs(double) as MSVC's <math.h> provides it */
#include <stdlib.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "matrix.h"
#include "gjk.h"
#include "Vector3.h"

/* what simulator2.h:4-14 provide (that header also pulls in <tchar.h> and
 * Callisto via stdafx.h, so it is not included) */
#define X_DIM 16
#define V_DIM 3
#define U_DIM 4
#define Z_DIM 6
typedef Matrix<X_DIM> State;
typedef Matrix<U_DIM> Input;
typedef Matrix<Z_DIM> Observation;
typedef Matrix<3, 3> Rotation;
typedef Matrix<3, 1> Velocity;
typedef Matrix<3, 1> Position;

/* LQRO:9-14 are compile-time macros; the harness makes NUM_POINTS and
 * OBSTACLE_STEPS runtime so one build serves every configuration. */
static int g_np = 100;
static int g_h = 45;
#define NUM_POINTS g_np
#define OBSTACLE_STEPS g_h
#define XYRADIUS 0.26
#define ZRADIUS 0.75

#include "ref_stdafx_helpers.inc"
#include "ref_globals.inc"
#include "ref_model.inc"
#include "ref_path.inc"

static void ref_setup_consts() {
#include "ref_setup_body.inc"
}
static void ref_set_weights() {
#include "ref_weights_body.inc"
}

template <size_t R, size_t C>
static void load(Matrix<R, C>& m, const double* p) {
  for (size_t i = 0; i < R * C; ++i) m[i] = p[i];
}
template <size_t R, size_t C>
static void store(const Matrix<R, C>& m, double* p) {
  if (p)
    for (size_t i = 0; i < R * C; ++i) p[i] = m[i];
}

extern "C" {

int ref_version(void) { return 1; }

/* setup() constants + _tmain weights + Quadrotor::findMatrices (LQRO:1370-1372) */
int ref_synthesize(double* A_, double* B_, double* c_, double* L_, double* E_, double* Lh_,
                   double* Eh_) {
  ref_setup_consts();
  ref_set_weights();
  Input uGoal;
  uGoal[0] = uGoal[1] = uGoal[2] = uGoal[3] = nominalInput;          /* LQRO:1272-1273 */
  State xGoal = zeros<X_DIM>();
  xGoal[12] = xGoal[13] = xGoal[14] = xGoal[15] = nominalInput;       /* LQRO:1299-1300 */
  Matrix<X_DIM, X_DIM> A;
  Matrix<X_DIM, U_DIM> B;
  Matrix<X_DIM, 1> c;
  Matrix<U_DIM, X_DIM> L;
  Matrix<U_DIM, V_DIM> E;
  Matrix<U_DIM, 1> l;
  Matrix<V_DIM, X_DIM> Lh;
  Matrix<V_DIM, V_DIM> Eh;
  controlMatrices(uGoal, xGoal, A, B, c, L, E, l, Lh, Eh);
  store(A, A_); store(B, B_); store(c, c_); store(L, L_); store(E, E_); store(Lh, Lh_);
  store(Eh, Eh_);
  return 0;
}

void ref_sphere(int np, double* out) {
  g_np = np;
  std::vector<Matrix<3, 1> > pts;
  createSpheres(pts);
  for (int i = 0; i < np; ++i)
    for (int k = 0; k < 3; ++k) out[3 * i + k] = pts[i][k];
}

/* matrix.h operator! on 3x3 / 4x4 (the pivoting the kernels must follow) */
void ref_inverse3(const double* in, double* out) {
  Matrix<3, 3> m; load(m, in); store(!m, out);
}
void ref_inverse4(const double* in, double* out) {
  Matrix<4, 4> m; load(m, in); store(!m, out);
}
void ref_expm16(const double* in, double* out) {
  Matrix<16, 16> m; load(m, in); store(exp(m), out);
}

/* GJK as run_gjk sets it up (LQRO:814-843), also returning the witnesses */
double ref_gjk(int n, const double* pts, const double* vrel, double* wpt_vrel,
               double* wpt_hull) {
  struct Object_structure VrelPoint;
  VrelPoint.numpoints = 1;
  REAL points1[1][3] = {{vrel[0], vrel[1], vrel[2]}};
  VrelPoint.vertices = points1;
  int ring1[3] = {1, 0, -1};
  VrelPoint.rings = ring1;
  struct Object_structure ConvexHull;
  ConvexHull.numpoints = n;
  std::vector<REAL> buf(3 * (size_t)n);
  memcpy(buf.data(), pts, sizeof(double) * 3 * (size_t)n);
  ConvexHull.vertices = (REAL(*)[3])buf.data();
  ConvexHull.rings = NULL;
  wpt_vrel[0] = wpt_vrel[1] = wpt_vrel[2] = wpt_hull[0] = wpt_hull[1] = wpt_hull[2] = 0;
  return gjk_distance(&VrelPoint, NULL, &ConvexHull, NULL, wpt_vrel, wpt_hull, NULL, 0);
}

/* One ordered pair: the body of LQRO:1397-1418 with the reference functions.
 * Returns 0 ok, 1 = inside hull (stops before convexHull), 2 = gated out. */
int ref_pair(int np, int H, int min_reach, double vmax_reach, const double* A_,
             const double* B_, const double* L_, const double* E_, const double* xi_,
             const double* xj_, int* n_reach, int32_t* reach_idx, double* reach_pts,
             double* dist, double* normal, double* wpt_vrel, double* wpt_hull,
             float* plane6) {
  g_np = np;
  g_h = H;
  Matrix<X_DIM, X_DIM> A; load(A, A_);
  Matrix<X_DIM, U_DIM> B; load(B, B_);
  Matrix<U_DIM, X_DIM> L; load(L, L_);
  Matrix<U_DIM, V_DIM> E; load(E, E_);
  State xi, xj; load(xi, xi_); load(xj, xj_);
  std::vector<Matrix<3, 1> > points;
  createSpheres(points);                                        /* LQRO:1376 */
  Matrix<3, X_DIM> C = zeros<3, X_DIM>();                        /* LQRO:1359-1360 */
  C(0, 0) = C(1, 1) = C(2, 2) = 1;
  std::vector<Matrix<3, 1> > ellipsoids, reachable;
  Matrix<3, 3> Transform;
  Matrix<3, 1> Translate;
  Matrix<X_DIM, X_DIM> Ft = identity<X_DIM>();                   /* LQRO:1401-1402 */
  Matrix<X_DIM, V_DIM> Gt = zeros<X_DIM, V_DIM>();
  for (size_t k = 0; k < (size_t)H; ++k) {                       /* LQRO:1403-1406 */
    findFG(A, B, L, E, Ft, Gt);
    createObstacle(ellipsoids, points, Transform, Translate, 0, Ft, Gt, C, xi, xj, 1);
  }
  findReachableObstacle(ellipsoids, reachable, xi, xj, vmax_reach); /* LQRO:1407 */
  int n = (int)reachable.size();
  *n_reach = n;
  {
    size_t e = 0;
    for (int r = 0; r < n; ++r) {
      while (!(ellipsoids[e] == reachable[r])) ++e;
      if (reach_idx) reach_idx[r] = (int32_t)e;
      if (reach_pts)
        for (int d = 0; d < 3; ++d) reach_pts[3 * r + d] = reachable[r][d];
      ++e;
    }
  }
  if (!(n > min_reach)) return 2;                                /* LQRO:1409 */
  bool insideHull = false;
  pointInHull(reachable, insideHull, xi, xj);                    /* LQRO:1410 */
  double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};
  if (reach_pts && wpt_vrel && wpt_hull) ref_gjk(n, reach_pts, vrel, wpt_vrel, wpt_hull);
  if (insideHull) return 1;
  double distance;
  Matrix<3, 1> normalVector;
  run_gjk(xi, xj, reachable, distance, normalVector);            /* LQRO:1414 */
  *dist = distance;
  store(normalVector, normal);
  distance *= 0.5;                                               /* LQRO:1416 */
  std::vector<Plane> planes;
  createHalfPlanes(xi, distance, normalVector, insideHull, planes); /* LQRO:1417 */
  plane6[0] = planes[0].point[0]; plane6[1] = planes[0].point[1]; plane6[2] = planes[0].point[2];
  plane6[3] = planes[0].normal[0]; plane6[4] = planes[0].normal[1]; plane6[5] = planes[0].normal[2];
  return 0;
}

/* calculateNewV (LQRO:1223-1234) */
void ref_newv(int m, const float* pl, const double* vgoal, double* newv) {
  std::vector<Plane> planes;
  for (int k = 0; k < m; ++k) {
    Plane p;
    p.point = Vector3(pl[6 * k], pl[6 * k + 1], pl[6 * k + 2]);
    p.normal = Vector3(pl[6 * k + 3], pl[6 * k + 4], pl[6 * k + 5]);
    planes.push_back(p);
  }
  Matrix<3, 1> g, nv;
  g[0] = vgoal[0]; g[1] = vgoal[1]; g[2] = vgoal[2];
  calculateNewV(planes, g, nv);
  newv[0] = nv[0]; newv[1] = nv[1]; newv[2] = nv[2];
}

/* The whole pair loop of one step (LQRO:1393-1436) for rows [r0,r1), all
 * agents sharing A,B,L,E (LQRO:1370-1371).  Returns the number of
 * inside-hull pairs met (their rows' newv are not produced: newv_ok[i]=0). */
int ref_step(int N, int np, int H, int min_reach, double vmax_reach, const double* A_,
             const double* B_, const double* L_, const double* E_, const double* x_,
             const double* vgoal_, int r0, int r1, double* newv, int32_t* newv_ok) {
  g_np = np;
  g_h = H;
  Matrix<X_DIM, X_DIM> A; load(A, A_);
  Matrix<X_DIM, U_DIM> B; load(B, B_);
  Matrix<U_DIM, X_DIM> L; load(L, L_);
  Matrix<U_DIM, V_DIM> E; load(E, E_);
  std::vector<State> x(N);
  for (int i = 0; i < N; ++i) load(x[i], x_ + (size_t)i * X_DIM);
  std::vector<Matrix<3, 1> > points;
  createSpheres(points);
  Matrix<3, X_DIM> C = zeros<3, X_DIM>();
  C(0, 0) = C(1, 1) = C(2, 2) = 1;
  Matrix<X_DIM, X_DIM> Ft;
  Matrix<X_DIM, V_DIM> Gt;
  bool insideHull = false;
  double distance = 0;
  Matrix<3, 1> normalVector = zeros<3, 1>();
  std::vector<Plane> orcaPlanes_;
  std::vector<Matrix<3, 1> > ellipsoids, reachable;
  Matrix<3, 3> Transform;
  Matrix<3, 1> Translate;
  int n_inside = 0;
  for (int i = r0; i < r1; ++i) {
    int inside_row = 0;
    for (int j = 0; j < N; ++j) {
      ellipsoids.clear();
      reachable.clear();
      if (i == j) continue;
      Ft = identity<X_DIM>();
      Gt = zeros<X_DIM, V_DIM>();
      for (size_t k = 0; k < (size_t)H; ++k) {
        findFG(A, B, L, E, Ft, Gt);
        createObstacle(ellipsoids, points, Transform, Translate, 0, Ft, Gt, C, x[i], x[j], 1);
      }
      findReachableObstacle(ellipsoids, reachable, x[i], x[j], vmax_reach);
      int numObstacle = (int)reachable.size();
      if (numObstacle > min_reach) {
        pointInHull(reachable, insideHull, x[i], x[j]);
        if (insideHull) { inside_row = 1; n_inside++; continue; }
        run_gjk(x[i], x[j], reachable, distance, normalVector);
        distance *= 0.5;
        createHalfPlanes(x[i], distance, normalVector, insideHull, orcaPlanes_);
      }
    }
    Matrix<3, 1> g, nv;
    g[0] = vgoal_[3 * i]; g[1] = vgoal_[3 * i + 1]; g[2] = vgoal_[3 * i + 2];
    calculateNewV(orcaPlanes_, g, nv);
    newv[3 * i] = nv[0]; newv[3 * i + 1] = nv[1]; newv[3 * i + 2] = nv[2];
    newv_ok[i] = !inside_row;
  }
  return n_inside;
}

/* ---- the per-agent step after the pair loop (LQRO:1437-1446) ---------
 * The reference's own controllers and filters.  propagate (LQRO:473-486) and
 * the observation draw (LQRO:1442) call sampleGaussian (simulator2.h:21-32),
 * whose jacobi (MAT:674-759) calls MSVC's _hypot, which this image lacks:
 * they are not built here (the oracle's jacobi is pinned by its properties,
 * tests/test_oracle_dyn.py).  Weights M, N are the reference's (LQRO:1285-1286). */

/* pseudoInverse (MAT:450-477, over jacobi2 MAT:887-1037) of a 16 x 16 matrix,
 * the form controlMatrices applies it in (LQRO:552) */
void ref_pinv16(const double* in, double* out) {
  Matrix<16, 16> q;
  load(q, in);
  store(pseudoInverse(q), out);
}

/* l of controlMatrices (LQRO:552,557), which the pair path does not read */
void ref_gain_l(double* l_) {
  ref_setup_consts();
  ref_set_weights();
  Input uGoal;
  uGoal[0] = uGoal[1] = uGoal[2] = uGoal[3] = nominalInput;
  State xGoal = zeros<X_DIM>();
  xGoal[12] = xGoal[13] = xGoal[14] = xGoal[15] = nominalInput;
  Matrix<X_DIM, X_DIM> A; Matrix<X_DIM, U_DIM> B; Matrix<X_DIM, 1> c;
  Matrix<U_DIM, X_DIM> L; Matrix<U_DIM, V_DIM> E; Matrix<U_DIM, 1> l;
  Matrix<V_DIM, X_DIM> Lh; Matrix<V_DIM, V_DIM> Eh;
  controlMatrices(uGoal, xGoal, A, B, c, L, E, l, Lh, Eh);
  store(l, l_);
}

void ref_control_velocity(const double* x_, const double* R_, const double* vg_,
                          const double* ug_, const double* L_, const double* E_,
                          const double* l_, double* u_) {
  State x; Rotation R0, RG = identity<3>(); Velocity vg; Input ug;
  Matrix<U_DIM, X_DIM> L; Matrix<U_DIM, V_DIM> E; Matrix<U_DIM, 1> l;
  load(x, x_); load(R0, R_); load(vg, vg_); load(ug, ug_); load(L, L_); load(E, E_); load(l, l_);
  store(riccatiControllerSteady(x, R0, vg, RG, ug, L, E, l), u_);
}

void ref_control_position(const double* x_, const double* R_, const double* pg_,
                          const double* ug_, const double* Lh_, const double* Eh_, double* v_) {
  State x; Rotation R0, RG = identity<3>(); Position pg; Input ug;
  Matrix<V_DIM, X_DIM> Lh; Matrix<V_DIM, V_DIM> Eh;
  load(x, x_); load(R0, R_); load(pg, pg_); load(ug, ug_); load(Lh, Lh_); load(Eh, Eh_);
  store(riccatiControllerSteadyPosition(x, R0, pg, RG, ug, Lh, Eh), v_);
}

void ref_kalman1(double* x_, double* R_, const double* u_, double* P_) {
  ref_setup_consts();
  ref_set_weights();
  State x; Rotation R0; Input u; Matrix<X_DIM, X_DIM> P;
  load(x, x_); load(R0, R_); load(u, u_); load(P, P_);
  kalmanFilter1(x, R0, u, M, P);
  store(x, x_); store(R0, R_); store(P, P_);
}

void ref_kalman2(double* x_, double* R_, const double* z_, double* P_) {
  ref_setup_consts();
  ref_set_weights();
  State x; Rotation R0; Observation z; Matrix<X_DIM, X_DIM> P;
  load(x, x_); load(R0, R_); load(z, z_); load(P, P_);
  kalmanFilter2(x, R0, z, N, P);
  store(x, x_); store(R0, R_); store(P, P_);
}

/* quatFromRot (stdafx.h:24-33), which Quadrotor::visualize keys Callisto with */
void ref_quat_from_rot(const double* R_, double* q_) {
  Rotation R; load(R, R_);
  store(quatFromRot(R), q_);
}

} /* extern "C" */
