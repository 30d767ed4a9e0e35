/*
 * lqro.h — C-ABI of the MI355X-native LQR-Obstacle step (liblqro.so).
 *
 * This is the drop-in boundary for the per-timestep pair loop of the
 * reference simulator (hihixuyang/LQR-Obstacles,
 * QuadrotorHoverController/LQRObstacles.cpp, "LQRO" below).  The reference
 * has no plugin/FFI API: the path is a set of free functions driven by the
 * loop at LQRO:1391-1436.  Each entry point below names the reference code it
 * replaces.  Conventions:
 *   - every function returns an int status: 0 = LQRO_OK, negative = error;
 *     no C++ exception crosses the ABI;
 *   - the caller owns every host array; the context owns device buffers and
 *     its HIP stream;
 *   - one context per host thread; contexts are independent of each other;
 *   - matrices are row-major fp64, exactly the element order of the
 *     reference's Matrix<R,C> (include/matrix.h:16,48).
 */
#ifndef LQRO_H
#define LQRO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
enum {
  LQRO_OK = 0,
  LQRO_E_ARG = -1,       /* bad argument / config                          */
  LQRO_E_HIP = -2,       /* a HIP runtime call failed                      */
  LQRO_E_NOMEM = -3,     /* device or host allocation failed               */
  LQRO_E_STATE = -4,     /* call order violated (e.g. step before gains)   */
  LQRO_E_SINGULAR = -5,  /* singular 3x3 C*G_k (reference asserts, MAT:632) */
  LQRO_E_NODEVICE = -6,  /* no usable gfx950 device                        */
  LQRO_E_OVERFLOW = -7,  /* an internal work queue overflowed              */
  LQRO_E_HULL = -8,      /* an inside-hull pair's hull could not be built    */
                         /*   (degenerate / too few points, or every hull    */
                         /*   kernel's capacity exceeded): its half-plane is */
                         /*   missing (lqro_get_hull_failures names pairs)   */
  LQRO_E_QHMERGE = -9    /* the step completed (newv written), but an inside- */
                         /*   hull pair's winning facet may be one qconvex's  */
                         /*   default pre-merge joins (LQRO_REC_QHMERGE_WIN): */
                         /*   this build restates Qhull merge-free, so that   */
                         /*   pair's facet, distance and half-plane are not   */
                         /*   pinned to the reference (LQRO:925-939, 956-967; */
                         /*   lqro_get_qhmerge_pairs names the pairs).        */
                         /*   LQRO_E_HULL takes precedence when both apply.   */
};

/* ---- flags ------------------------------------------------------------- */
#define LQRO_FLAG_RECORDS     0x1  /* keep per-pair records for lqro_get_records */
#define LQRO_FLAG_QHULL_ORDER 0x2  /* inside-hull branch with the reference's own rule   */
                                   /*   (LQRO:925-968): Qhull's facet order and each    */
                                   /*   facet's first Fv vertex, strict '<', and the    */
                                   /*   loop-carried normalVector when facet 0 wins     */
                                   /*   (LQRO:956-968, 1385); built in-kernel by k_qhull */

/* per-pair record flags (lqro_pair_record.flags) */
#define LQRO_REC_PLANE    0x01  /* n_reach > min_reach: a half-plane was emitted (LQRO:1409) */
#define LQRO_REC_INSIDE   0x02  /* GJK put vrel inside the hull (LQRO:855-864)          */
#define LQRO_REC_BACKUP   0x04  /* GJK took its backup procedure (GJK:663-706)          */
#define LQRO_REC_HULL     0x08  /* the in-kernel hull produced the plane (LQRO:867-969) */
#define LQRO_REC_HULLFAIL 0x10  /* hull degenerate / capacity exceeded                  */
#define LQRO_REC_LOCAL    0x20  /* the plane came from the local hull (k_lhull)          */
#define LQRO_REC_STALE    0x40  /* Qhull order: facet 0 won, normal = the loop-carried    */
                                /*   normalVector of the previous pair (LQRO:956-968)    */
#define LQRO_REC_QHMERGE  0x80  /* Qhull order: Qhull would merge facets in this hull;   */
                                /*   built merge-free                       */
#define LQRO_REC_QHMERGE_WIN 0x100 /* with LQRO_REC_QHMERGE: a facet within 1e-6 of the  */
                                /*   winning distance has another hull vertex within    */
                                /*   1e-9 (|coord|max + 1) of its plane, so qconvex's     */
                                /*   pre-merge may have joined the winner into a merged */
                                /*   facet: the pair's facet, distance and normal are    */
                                /*   then not pinned to the reference;    */
                                /*   lqro_get_stats_ex [11] counts these pairs           */

/* Static configuration.  The names follow the reference's compile-time
 * macros (LQRO:9-14) and the constants of its driver (LQRO:1387, 1224). */
typedef struct lqro_config {
  int32_t n_agents;      /* NUM_QUADS                                             */
  int32_t x_dim;         /* X_DIM (simulator2.h:4) — 16                           */
  int32_t u_dim;         /* U_DIM — 4                                             */
  int32_t horizon;       /* OBSTACLE_STEPS (LQRO:11)                              */
  int32_t n_points;      /* NUM_POINTS (LQRO:12) points per sampled ellipsoid     */
  int32_t min_reach;     /* pairs with n_reach <= min_reach emit no plane (4, LQRO:1409) */
  double  xy_radius;     /* XYRADIUS (LQRO:13); the sphere uses 2*XYRADIUS        */
  double  z_radius;      /* ZRADIUS  (LQRO:14)                                    */
  double  vmax_reach;    /* reachable-velocity radius, 30 (LQRO:1387)             */
  double  vmax_lp;       /* LP speed bound, 100 (LQRO:1224)                        */
  int32_t row_begin;     /* agents [row_begin,row_end) are this context's rows    */
  int32_t row_end;       /*   (multi-GPU sharding; 0,0 = all rows)                 */
  int32_t device;        /* HIP device ordinal                                    */
  int32_t flags;         /* LQRO_FLAG_*                                           */
  int32_t row_stride;    /* 0/1: rows row_begin..row_end-1; s > 1: rows row_begin,  */
                         /*   row_begin+s, ... < row_end (cyclic sharding: rank,  */
                         /*   world); records, newv rows and the LP follow it      */
} lqro_config;

/* Physical model + cost weights: the globals set by setup() and _tmain
 * (LQRO:169-189, 1275-1286, 559-561). */
typedef struct lqro_model {
  double dt, gravity, mass, inertia, moment_const, thrust_latency, length;
  double j_step;          /* central-difference step (LQRO:189)   */
  double qv, qp, r;       /* Qv = qv*I3, Qp = qp*I3, R = r*I4     */
  double pos_weight;      /* 0.05 in LQRO:559-561 (0.25 in PCW)   */
} lqro_model;

/* One record per ordered pair (i, j), j != i, kept when LQRO_FLAG_RECORDS
 * is set.  Field-for-field what the reference computes in LQRO:1401-1417. */
typedef struct lqro_pair_record {
  int32_t i, j;
  int32_t n_reach;        /* reachablePoints.size() (LQRO:1408)              */
  int32_t flags;          /* LQRO_REC_*                                      */
  int32_t gjk_iters;      /* G-tests performed by gjk_distance               */
  int32_t simplex_n;      /* final GJK simplex size                          */
  int32_t simplex[4];     /* final GJK simplex: indices into reachablePoints */
  int32_t facet[3];       /* hull branch: arg-min facet (reachable indices); */
                          /*   Qhull order: in Fv order, facet[0] = the vertex */
                          /*   the distance is measured from (LQRO:934-937)  */
  int32_t n_facets;       /* hull branch: number of hull facets (LQRO_REC_LOCAL: */
                          /*   the certified facets of the local hull)       */
  uint64_t reach_hash;    /* sum of splitmix64(q) over reachable point ids q */
  double dist;            /* distance before the *0.5 of LQRO:1416           */
  double normal[3];       /* normalVector fed to createHalfPlanes            */
  double wpt_vrel[3];     /* GJK witness on the vrel point                   */
  double wpt_hull[3];     /* GJK witness on the hull                         */
  float  plane_point[3];  /* Plane.point  (fp32, LQRO:1217-1219)             */
  float  plane_normal[3]; /* Plane.normal (fp32, LQRO:1210)                  */
} lqro_pair_record;

typedef struct lqro_ctx lqro_ctx;

/* Defaults: LQRO's constants (N given by the caller); flags =
 * LQRO_FLAG_QHULL_ORDER, the reference's own inside-hull rule.  Clearing it
 * selects the faster canonical facet rule, a measured deviation from the
 * reference. */
void lqro_config_default(lqro_config* cfg, int32_t n_agents, int32_t horizon, int32_t n_points);
void lqro_model_default(lqro_model* m);

/* Replaces controlMatrices (LQRO:520-582) and linearizeDiscretize (LQRO:456-471):
 * the velocity LQR (A,B,c,L,E) and the position LQR (Lh,Eh) at hover.
 * Host C++ (setup time, once per agent type).  Any out pointer may be NULL. */
int lqro_synthesize_gains(const lqro_model* m,
                          double* A  /* X*X */, double* B  /* X*U */, double* c /* X */,
                          double* L  /* U*X */, double* E  /* U*3 */,
                          double* Lh /* 3*X */, double* Eh /* 3*3 */);

/* The same synthesis for a swarm of heterogeneous agents, on the GPU (one
 * agent per lane): models[n]; outputs are n consecutive blocks of the shapes
 * above (A n*X*X, B n*X*U, c n*X, L n*U*X, E n*U*3, Lh n*3*X, Eh n*3*3), host
 * arrays, any may be NULL.  Bit-identical to lqro_synthesize_gains per model.
 * Feeds lqro_set_gains(..., per_agent = 1).  Synchronous. */
int lqro_synthesize_gains_batch(const lqro_model* models, int32_t n,
                                double* A, double* B, double* c, double* L, double* E,
                                double* Lh, double* Eh, int32_t device);

/* The same two syntheses for a state width x_dim: 16 (the reference's
 * quadrotor, identical to the two calls above) or 12, the reduced model of
 * BASELINE config 5: the 4 rotor-force states of X_DIM = 16
 * (simulator2.h:4) dropped, rotor forces = the command (no thrust lag), every
 * other term of f (LQRO:368-397) unchanged, linearised at the same hover
 * point.  Shapes as above with X = x_dim.  Both also return l (U), the
 * feedforward of controlMatrices (LQRO:552-557: pseudoInverse over jacobi2,
 * MAT:450-477, 887-1037), 0 at the reference's hover point (c = 0). */
int lqro_synthesize_gains_x(const lqro_model* m, int32_t x_dim,
                            double* A, double* B, double* c, double* L, double* E,
                            double* l /* U: the feedforward term, LQRO:552-557 */,
                            double* Lh, double* Eh);
int lqro_synthesize_gains_batch_x(const lqro_model* models, int32_t n, int32_t x_dim,
                                  double* A, double* B, double* c, double* L, double* E,
                                  double* l /* n*U */, double* Lh, double* Eh, int32_t device);

/* Replaces createSpheres (LQRO:735-750): NP Fibonacci-sphere points. */
int lqro_sphere(int32_t n_points, double xy_radius, double z_radius, double* out /* NP*3 */);

int  lqro_create(const lqro_config* cfg, lqro_ctx** out);
void lqro_destroy(lqro_ctx* ctx);

/* Gains read by the pair loop: A, B shared (LQRO:1265-1266, 1371); L_i, E_i
 * per agent (Quadrotor::L,E, LQRO:90-91).  per_agent = 0: one L,E for all
 * agents (the reference's case: every agent gets the same gains, LQRO:1371);
 * per_agent = 1: L is n_agents*U*X, E is n_agents*U*3.  Builds the per-agent
 * horizon tables on the device (findFG + createObstacle's Transform, LQRO:723-732,
 * 770-773). */
int lqro_set_gains(lqro_ctx* ctx, const double* A, const double* B,
                   const double* L, const double* E, int32_t per_agent);

/* Opt-in neighbour culling, in place of the all-pairs
 * loop (LQRO:1396): agent i then computes only the pairs with the
 * max_neighbors agents j != i of smallest |p_i - p_j|^2 < neighbor_dist^2
 * (ties to the lower j), RVO2-3D's computeNeighbors / insertAgentNeighbor
 * (Agent.cpp:74-81, 153-174) with agents visited in j order; its LP sees those
 * planes in j order.  A row then has K = min(max_neighbors, n_agents-1) slots
 * instead of n_agents-1: lqro_get_records returns rows x K records, the q-th
 * the row's q-th neighbour in ascending j; unused slots have j = -1 and
 * n_reach = -1.  lqro_get_stats()[0] counts the kept pairs.  This CHANGES
 * results against the reference.  max_neighbors <= 0 restores all pairs. */
int lqro_set_neighbors(lqro_ctx* ctx, double neighbor_dist, int32_t max_neighbors);

/* One control step: the pair loop LQRO:1393-1436 for the context's rows.
 * x: n_agents*X agent states (Quadrotor::x), vgoal: n_agents*3,
 * newv: n_agents*3 (only rows [row_begin,row_end) are written).  Host
 * pointers; blocks until newv is ready.  Returns LQRO_E_HULL (newv still
 * written) when an inside-hull pair got no half-plane, else LQRO_E_QHMERGE
 * (newv written) when an inside-hull pair's winner may be a facet qconvex
 * merges (LQRO_REC_QHMERGE_WIN). */
int lqro_step(lqro_ctx* ctx, const double* x, const double* vgoal, double* newv);

/* Same, device-resident: d_x, d_vgoal, d_newv are device pointers on the
 * context's device; the work is enqueued on `stream` (hipStream_t; NULL = the
 * default null stream, as in lqro_dynamics_step_device) behind whatever the
 * caller queued there before, and the call returns without synchronising.
 * lqro_get_stats / lqro_get_records / lqro_get_timings wait for the last
 * enqueued step on the stream it was enqueued on.  The hull queue holds one
 * entry per pair slot, so a step cannot overflow it. */
int lqro_step_device(lqro_ctx* ctx, const double* d_x, const double* d_vgoal,
                     double* d_newv, void* stream);
/* (The device-resident calls cannot report a hull failure when they return:
 * lqro_get_stats()[4] / lqro_get_hull_failures after the step do, and
 * lqro_get_stats_ex()[11] / lqro_get_qhmerge_pairs the merge suspects.  While a
 * lqro_step_device_begin is pending, every call but lqro_step_device_end
 * returns LQRO_E_STATE.) */

/* lqro_step_device in two halves around the exchange a row-sharded caller
 * needs in Qhull order (LQRO_FLAG_QHULL_ORDER): the loop-carried
 * normalVector (LQRO:1385) runs through every pair of the swarm in (i, j)
 * order, across the shards.  _begin enqueues the sweep and the hulls and
 * writes, for each of the context's own rows i, the normal of its last pair
 * with one: d_rowtab[4 i + 0..2], d_rowtab[4 i + 3] = 1 (0 0 0 0 for none, or
 * without the flag).  The caller then fills the other ranks' rows of the
 * n_agents x 4 table (an all-gather) and calls _end, which resolves the
 * facet-0 pairs from the whole table (their own row's earlier pairs, else
 * the last row before theirs with a normal, else the normal entering the
 * step), runs the LP and writes d_newv.  Every rank then carries the same
 * normal into the next step.  For a context that owns every row the two
 * halves equal lqro_step_device.  lqro_step / lqro_step_device on a shard
 * other than the first resolve facet-0 pairs from the context's own rows
 * only. */
int lqro_step_device_begin(lqro_ctx* ctx, const double* d_x, const double* d_vgoal,
                           double* d_rowtab, void* stream);
int lqro_step_device_end(lqro_ctx* ctx, const double* d_rowtab, double* d_newv, void* stream);

/* calculateNewV (LQRO:1223-1234) for a batch of independent agents on the
 * GPU: agent r's planes are planes[offsets[r] .. offsets[r+1]) (6 floats
 * each: point xyz, normal xyz, in orcaPlanes_ push order), its preferred
 * velocity vgoal[3r..3r+2]; writes newv[3r..3r+2].  Synchronous. */
int lqro_calculate_new_v(const float* planes, const int64_t* offsets, int32_t n_agents,
                         const double* vgoal, double vmax_lp, double* newv, int32_t device);

/* LQRO_FLAG_QHULL_ORDER: the loop-carried normalVector (LQRO:1385) entering
 * the context's first row (set; 0,0,0 at creation) and leaving its last
 * eligible pair after the last step (get).  A single context carries it
 * from step to step itself; row-sharded callers chain ranks with these. */
int lqro_set_carry_normal(lqro_ctx* ctx, const double* n3);
int lqro_get_carry_normal(lqro_ctx* ctx, double* n3);

/* Per-pair records of the last step (LQRO_FLAG_RECORDS): rows
 * [row_begin,row_end) x (n_agents-1) neighbours in j order. */
int lqro_get_records(lqro_ctx* ctx, lqro_pair_record* out, int64_t capacity, int64_t* n_out);

/* Counters of the last step: [0]=pairs, [1]=planes, [2]=inside, [3]=hull ok,
 * [4]=hull fail, [5]=gjk backups, [6]=sum n_reach, [7]=sum G-tests. */
int lqro_get_stats(lqro_ctx* ctx, int64_t* stats8);
/* The same counters and n - 8 more (n <= 12; words past 11 read 0):
 * [8] LQRO_FLAG_QHULL_ORDER hulls in which Qhull would merge facets
 *     (LQRO_REC_QHMERGE: built merge-free);
 * [9] builds k_qhull's per-insertion caps handed to k_qhull_big;
 * [10] of those, the ones a wave handshake timeout stopped;
 * [11] pairs whose winning facet qconvex's pre-merge may have merged
 *     (LQRO_REC_QHMERGE_WIN). */
int lqro_get_stats_ex(lqro_ctx* ctx, int64_t* stats, int32_t n);

/* The inside-hull pairs of the last step flagged LQRO_REC_QHMERGE_WIN (stats
 * [11]; lqro_step then returns LQRO_E_QHMERGE): *n_out = their number;
 * pairs[2k], pairs[2k+1] = (i, j) of the first min(*n_out, 64, capacity).
 * Replaces nothing in the reference: it names the pairs whose half-plane
 * may differ from convexHull's over a merged qconvex facet (LQRO:925-967). */
int lqro_get_qhmerge_pairs(lqro_ctx* ctx, int64_t* pairs, int64_t capacity, int64_t* n_out);

/* One Qhull-order hull build of the last step (LQRO_FLAG_QHULL_ORDER): the
 * in-kernel replacement of convexHull's qconvex run (LQRO:867-969) for the
 * pair (i, j), timed on the GPU's constant 100 MHz clock (s_memrealtime,
 * shared by every CU): from taking the job (the pair's points are computed
 * first) to its half-plane.  kernel: 0 k_qhull, 1 k_qhull_big (the build
 * beyond k_qhull's caps), 2 a k_qhull build handed to k_qhull_big (its
 * record ends where the hand-over happened). */
typedef struct lqro_hull_build {
  int32_t i, j;
  int32_t n_points;       /* reachablePoints.size(), qconvex's input             */
  int32_t insertions;     /* points Qhull added (qh_addpoint calls)              */
  int32_t facet_slots;    /* facets created (slots used)                         */
  int32_t kernel;
  uint64_t t_start, t_end;  /* 100 MHz ticks                                     */
} lqro_hull_build;
/* *n_out = the builds of the last step (at most the first `capacity` and
 * 16384 are written, in completion order). */
int lqro_get_hull_builds(lqro_ctx* ctx, lqro_hull_build* out, int64_t capacity, int64_t* n_out);

/* The pairs of the last step left without a half-plane because their hull
 * could not be built — degenerate input or every hull kernel's capacity
 * exceeded (stats [4]; lqro_step then returns
 * LQRO_E_HULL, the reference's qconvex always returns a hull, LQRO:879-880):
 * *n_out = their number; pairs[2k], pairs[2k+1] = (i, j) of the first
 * min(*n_out, 64, capacity). */
int lqro_get_hull_failures(lqro_ctx* ctx, int64_t* pairs, int64_t capacity, int64_t* n_out);

/* Device time of the kernels of the last step, ms, measured with HIP events on
 * the context's stream: [0]=pair sweep+GJK, [1]=hull, [2]=LP, [3]=whole step. */
int lqro_get_timings(lqro_ctx* ctx, float* ms4);

/* ---- the per-agent step after the pair loop ------
 * Replaces the agent loop LQRO:1437-1446: vGoal = newV; u = findU()
 * (riccatiControllerSteady, LQRO:594-617); propagateU (propagate,
 * LQRO:473-486) of the true state; kalmanFilter1 (LQRO:488-505); the
 * observation z = sampleGaussian(h(xTrue, RotTrue), N) (LQRO:1442);
 * kalmanFilter2 (LQRO:507-518); vGoal = findVGoal()
 * (riccatiControllerSteadyPosition, LQRO:619-645).  Quadrotor::visualize
 * (LQRO:1444) becomes a keyframe record instead of Callisto calls
 * (SURVEY §8f next #4).  X = 16, U = 4, Z = 6.
 * The reference draws its noise from rand() in agent order (normal(),
 * LQRO:334-350): the caller supplies the draws, LQRO_NORMALS_PER_AGENT per
 * agent (16 for propagate, then 6 for the observation); lqro_normals
 * reproduces the stream. */
#define LQRO_NORMALS_PER_AGENT 22

typedef struct lqro_agents {
  double* x;             /* n*16  Quadrotor::x: the estimate lqro_step reads     */
  double* rot;           /* n*9   Quadrotor::Rot                                 */
  double* x_true;        /* n*16  Quadrotor::xTrue                               */
  double* rot_true;      /* n*9   Quadrotor::RotTrue                             */
  double* P;             /* n*256 Quadrotor::P, state covariance                 */
  double* vgoal;         /* n*3   in: newV (lqro_step); out: findVGoal()         */
  double* u;             /* n*4   out: findU(); may be NULL                      */
  const double* u_goal;  /* n*4   Quadrotor::uGoal                               */
  const double* p_goal;  /* n*3   Quadrotor::pGoal                               */
  const double* L;       /* U*X   gains (Quadrotor::L,E,l,Lh,Eh): one block, or  */
  const double* E;       /* U*3     n blocks with per_agent_gains = 1            */
  const double* l;       /* U                                                    */
  const double* Lh;      /* 3*X                                                  */
  const double* Eh;      /* 3*3                                                  */
  const double* M;       /* X*X   motion noise variance (LQRO:1285)              */
  const double* N;       /* 6*6   observation noise variance (LQRO:1286)         */
  const double* normals; /* n*LQRO_NORMALS_PER_AGENT                             */
  float* keyframes;      /* n*8 out, may be NULL: Quadrotor::visualize's keyframe */
                         /*   (LQRO:128-133): time, (float) xTrue[0..2],          */
                         /*   (float) quatFromRot(RotTrue) (stdafx.h:24-33)       */
  double time;           /* t*dt, the keyframe time (LQRO:1444)                   */
} lqro_agents;

/* Host arrays; synchronous.  models: n_models = 1 (shared) or n. */
int lqro_dynamics_step(const lqro_model* models, int32_t n_models, int32_t n,
                       int32_t per_agent_gains, const lqro_agents* agents, int32_t device);
/* Device-resident: every pointer in *agents and `models` is a device pointer on
 * the current device; enqueued on `stream` (hipStream_t, NULL = default),
 * returns without synchronising.  d_x then feeds lqro_step_device directly. */
int lqro_dynamics_step_device(const lqro_model* models, int32_t n_models, int32_t n,
                              int32_t per_agent_gains, const lqro_agents* agents, void* stream);
/* normal() (LQRO:340-350) over random() (LQRO:334-337) on the MSVC rand()
 * stream (seed' = seed*214013 + 2531011, rand = (seed' >> 16) & 0x7fff; srand(s)
 * sets seed = s).  Writes `count` draws, advances *seed. */
int lqro_normals(uint32_t* seed, int64_t count, double* out);

const char* lqro_status_string(int status);
int lqro_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LQRO_H */
