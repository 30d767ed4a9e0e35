// lqro_dyn.hpp — the per-agent step that follows the pair loop
// (LQRObstacles.cpp:1437-1446): findU
// (riccatiControllerSteady, :594-617), propagateU (propagate, :473-486),
// kalmanFilter1 (:488-505), the observation draw (h :399-419, sampleGaussian
// simulator2.h:21-32), kalmanFilter2 (:507-518) and findVGoal
// (riccatiControllerSteadyPosition, :619-645), with jacobi (matrix.h:674-759),
// errFromRot (stdafx.h:35-48) and Jacobian_hx (:443-452).
//
// Written once for host and device on top of lqro_synth.hpp's matrix code, in
// the reference's operation order (-ffp-contract=off).  Unlike the gain
// synthesis, this step calls libm on live values (tan in f, asin in the
// controllers, atan2 in errFromRot, hypot in jacobi), where the device's and
// glibc's results may differ in the last bit: parity is within a relative
// tolerance (tests/test_gpu_dyn.py), not bit-exact.
//
// The reference draws its Gaussian noise from a global rand() stream
// (normal(), :334-350) in agent order.  The caller supplies the normals
// (lqro_normals reproduces that stream on the host): 16 for propagate, then 6
// for the observation, per agent.
#pragma once
#include <float.h>

#include "lqro_synth.hpp"

namespace lqro {
namespace dyn {

using synth::Mat;
using synth::Vec3;
using synth::Quad;
using synth::eye;
using synth::expm;
using synth::inverse;
using synth::skew;
using synth::tr;

constexpr int kX = 16, kU = 4, kV = 3, kZ = 6;
constexpr int kNormals = kX + kZ;   // per agent per step

LQRO_HD Quad quad(const lqro_model* md) {
  Quad q;
  q.dt = md->dt; q.g = md->gravity; q.mass = md->mass; q.kM = md->moment_const;
  q.lat = md->thrust_latency; q.arm = md->length; q.h = md->j_step;
  q.J = md->inertia * eye<3>();
  q.Jinv = inverse(q.J);
  return q;
}

// jacobi (MAT:674-759): cyclic-by-row Jacobi rotations on the upper triangle
template <int N>
LQRO_HD void jacobi(const Mat<N, N>& m, Mat<N, N>& V, Mat<N, N>& D) {
  D = m;
  V = eye<N>();
  if (N <= 1) return;
  int pivot = 0, zeros = 0;
  for (;;) {
    double maximum = 0;
    int p = 0, q = 0;
    for (int i = 0; i < pivot; ++i)
      if (fabs(D(i, pivot)) > maximum) { maximum = fabs(D(i, pivot)); p = i; q = pivot; }
    for (int j = pivot + 1; j < N; ++j)
      if (fabs(D(pivot, j)) > maximum) { maximum = fabs(D(pivot, j)); p = pivot; q = j; }
    pivot = (pivot + 1) % N;
    if (maximum <= DBL_EPSILON) {
      if (++zeros == N) break;
      continue;
    }
    zeros = 0;
    const double theta = 0.5 * (D(q, q) - D(p, p)) / D(p, q);
    double t = 1 / (fabs(theta) + hypot(theta, 1.0));
    if (theta < 0) t = -t;
    const double c = 1 / hypot(t, 1.0);
    const double s = c * t;
    const double tau = s / (1 + c);
    for (int r = 0; r < p; ++r) {
      const double a = D(r, p), b = D(r, q);
      D(r, p) -= s * (b + tau * a);
      D(r, q) += s * (a - tau * b);
    }
    for (int r = p + 1; r < q; ++r) {
      const double a = D(p, r), b = D(r, q);
      D(p, r) -= s * (b + tau * a);
      D(r, q) += s * (a - tau * b);
    }
    for (int r = q + 1; r < N; ++r) {
      const double a = D(p, r), b = D(q, r);
      D(p, r) -= s * (b + tau * a);
      D(q, r) += s * (a - tau * b);
    }
    D(p, p) -= t * D(p, q);
    D(q, q) += t * D(p, q);
    D(p, q) = 0;
    for (int r = 0; r < N; ++r) {
      const double a = V(r, p), b = V(r, q);
      V(r, p) -= s * (b + tau * a);
      V(r, q) += s * (a - tau * b);
    }
  }
  for (int i = 0; i < N - 1; ++i)
    for (int j = i + 1; j < N; ++j) D(j, i) = D(i, j) = 0;
}

// sampleGaussian (simulator2.h:21-32) with the draws supplied
template <int N>
LQRO_HD Mat<N, 1> sample_gaussian(const Mat<N, 1>& mean, const Mat<N, N>& var, const double* nrm) {
  Mat<N, 1> smp;
  for (int j = 0; j < N; ++j) smp.e[j] = nrm[j];
  Mat<N, N> V, D;
  jacobi(var, V, D);
  for (int i = 0; i < N; ++i) D(i, i) = sqrt(D(i, i));
  return V * D * smp + mean;
}

// h (LQRO:399-419): rate gyros, then position
LQRO_HD Mat<kZ, 1> observe(const Mat<kX, 1>& x) {
  Mat<kZ, 1> z;
  for (int k = 0; k < 3; ++k) { z.e[k] = x.e[9 + k]; z.e[3 + k] = x.e[k]; }
  return z;
}

// Jacobian_fx (LQRO:421-430)
LQRO_HD Mat<kX, kX> jac_fx(const Quad& q, const Mat<kX, 1>& x, const Mat<3, 3>& R, const Mat<kU, 1>& u) {
  Mat<kX, kX> F;
  Mat<kX, 1> xr = x, xl = x;
  for (int i = 0; i < kX; ++i) {
    xr.e[i] += q.h; xl.e[i] -= q.h;
    const Mat<kX, 1> col = (synth::dynamics(q, xr, R, u) - synth::dynamics(q, xl, R, u)) / (2 * q.h);
    for (int k = 0; k < kX; ++k) F(k, i) = col.e[k];
    xr.e[i] = xl.e[i] = x.e[i];
  }
  return F;
}

// Jacobian_hx (LQRO:443-452)
LQRO_HD Mat<kZ, kX> jac_hx(const Quad& q, const Mat<kX, 1>& x) {
  Mat<kZ, kX> H;
  Mat<kX, 1> xr = x, xl = x;
  for (int i = 0; i < kX; ++i) {
    xr.e[i] += q.h; xl.e[i] -= q.h;
    const Mat<kZ, 1> col = (observe(xr) - observe(xl)) / (2 * q.h);
    for (int k = 0; k < kZ; ++k) H(k, i) = col.e[k];
    xr.e[i] = xl.e[i] = x.e[i];
  }
  return H;
}

// R = R*exp([x_6:9]); x_6:9 = 0 (the rotation-error reset, LQRO:483-485)
// (always inlined: as a call, k_dynw kept its live registers in scratch
// around each of the three resets)
__host__ __device__ __forceinline__ void reset_rot(Mat<kX, 1>& x, Mat<3, 3>& R) {
  Vec3 r;
  for (int k = 0; k < 3; ++k) r.e[k] = x.e[6 + k];
  R = R * expm(skew(r));
  x.e[6] = 0; x.e[7] = 0; x.e[8] = 0;
}

// A = exp(dt F), A2 = exp(dt/2 F), MM = dt/6 (M + 4 A2 M A2^T + A M A^T) and
// the Simpson increment dt/6 (xdot + 4 A2 xdot + A xdot): the common head of
// propagate and kalmanFilter1
LQRO_HD void discretize(const Quad& q, const Mat<kX, 1>& x, const Mat<3, 3>& R, const Mat<kU, 1>& u,
                        const Mat<kX, kX>& M, Mat<kX, kX>& A, Mat<kX, kX>& MM, Mat<kX, 1>& dx) {
  const Mat<kX, kX> F = jac_fx(q, x, R, u);
  const Mat<kX, 1> xdot = synth::dynamics(q, x, R, u);
  A = expm(q.dt * F);
  const Mat<kX, kX> A2 = expm((q.dt * 0.5) * F);
  MM = (q.dt / 6) * (M + 4 * A2 * M * tr(A2) + A * M * tr(A));
  dx = (q.dt / 6) * (xdot + 4 * (A2 * xdot) + A * xdot);
}

// propagate (LQRO:473-486)
LQRO_HD void propagate(const Quad& q, Mat<kX, 1>& x, Mat<3, 3>& R, const Mat<kU, 1>& u,
                       const Mat<kX, kX>& M, const double* nrm) {
  Mat<kX, kX> A, MM;
  Mat<kX, 1> dx;
  discretize(q, x, R, u, M, A, MM, dx);
  x = x + dx + sample_gaussian(Mat<kX, 1>::zero(), MM, nrm);
  reset_rot(x, R);
}

// kalmanFilter1 (LQRO:488-505)
LQRO_HD void kalman_predict(const Quad& q, Mat<kX, 1>& x, Mat<3, 3>& R, const Mat<kU, 1>& u,
                            const Mat<kX, kX>& M, Mat<kX, kX>& P) {
  Mat<kX, kX> A, MM;
  Mat<kX, 1> dx;
  discretize(q, x, R, u, M, A, MM, dx);
  x = x + dx;
  P = A * P * tr(A) + MM;
  reset_rot(x, R);
}

// kalmanFilter2 (LQRO:507-518)
LQRO_HD void kalman_update(const Quad& q, Mat<kX, 1>& x, Mat<3, 3>& R, const Mat<kZ, 1>& z,
                           const Mat<kZ, kZ>& Nz, Mat<kX, kX>& P) {
  const Mat<kZ, kX> H = jac_hx(q, x);
  const Mat<kX, kZ> K = P * tr(H) * inverse(H * P * tr(H) + Nz);
  x = x + K * (z - observe(x));
  P = (eye<kX>() - K * H) * P;
  reset_rot(x, R);
}

// errFromRot (stdafx.h:35-48)
LQRO_HD Vec3 err_from_rot(const Mat<3, 3>& R) {
  Vec3 q;
  q.e[0] = R(2, 1) - R(1, 2);
  q.e[1] = R(0, 2) - R(2, 0);
  q.e[2] = R(1, 0) - R(0, 1);
  const double r = sqrt(q.e[0] * q.e[0] + q.e[1] * q.e[1] + q.e[2] * q.e[2]);
  const double t = R(0, 0) + R(1, 1) + R(2, 2) - 1;
  if (r == 0) return Vec3::zero();
  return q * (atan2(r, t) / r);
}

// the yaw-only frame and xTilde shared by both controllers (LQRO:597-616)
LQRO_HD Mat<3, 3> local_frame(const Mat<kX, 1>& x, const Mat<3, 3>& R0, const Mat<kU, 1>& u_goal,
                              Mat<kX, 1>& xt) {
  Vec3 z0, ez = Vec3::zero();
  z0.e[0] = R0(0, 2); z0.e[1] = R0(1, 2); z0.e[2] = R0(2, 2);
  ez.e[2] = 1;
  Vec3 axis = skew(z0) * ez;
  const double sinangle = sqrt(axis.e[0] * axis.e[0] + axis.e[1] * axis.e[1] + axis.e[2] * axis.e[2]);
  const double angle = asin(sinangle);
  if (sinangle != 0) axis = axis * (angle / sinangle);
  const Mat<3, 3> RL = expm(skew(axis)) * R0;
  const Mat<3, 3> RLt = tr(RL);
  Vec3 p, v, w;
  for (int k = 0; k < 3; ++k) { p.e[k] = x.e[k]; v.e[k] = x.e[3 + k]; w.e[k] = x.e[9 + k]; }
  const Vec3 pl = RLt * p, vl = RLt * v, el = err_from_rot(RLt * R0);
  for (int k = 0; k < 3; ++k) {
    xt.e[k] = pl.e[k]; xt.e[3 + k] = vl.e[k]; xt.e[6 + k] = el.e[k]; xt.e[9 + k] = w.e[k];
  }
  for (int k = 0; k < 4; ++k) xt.e[12 + k] = x.e[12 + k] - u_goal.e[k];
  return RL;
}

// riccatiControllerSteady (LQRO:594-617): u = uGoal + L xTilde + E vTildeGoal + l
LQRO_HD Mat<kU, 1> control_velocity(const Mat<kX, 1>& x, const Mat<3, 3>& R0, const Vec3& vgoal,
                                    const Mat<kU, 1>& u_goal, const Mat<kU, kX>& L,
                                    const Mat<kU, kV>& E, const Mat<kU, 1>& l) {
  Mat<kX, 1> xt;
  const Mat<3, 3> RL = local_frame(x, R0, u_goal, xt);
  const Vec3 vt = tr(RL) * vgoal;
  return u_goal + L * xt + E * vt + l;
}

// riccatiControllerSteadyPosition (LQRO:619-645): RLocal (Lh xTilde + Eh pTildeGoal)
LQRO_HD Vec3 control_position(const Mat<kX, 1>& x, const Mat<3, 3>& R0, const Vec3& pgoal,
                              const Mat<kU, 1>& u_goal, const Mat<kV, kX>& Lh,
                              const Mat<kV, kV>& Eh) {
  Mat<kX, 1> xt;
  const Mat<3, 3> RL = local_frame(x, R0, u_goal, xt);
  const Vec3 pt = tr(RL) * pgoal;
  return RL * (Lh * xt + Eh * pt);
}

// std::max(a, 0.0)
LQRO_HD double max0(double a) { return (a < 0.0) ? 0.0 : a; }

// quatFromRot (stdafx.h:24-33)
LQRO_HD Mat<4, 1> quat_from_rot(const Mat<3, 3>& R) {
  Mat<4, 1> q;
  q.e[0] = 0.5 * sqrt(max0(1 + R(0, 0) - R(1, 1) - R(2, 2))) * (R(2, 1) - R(1, 2) >= 0 ? 1 : -1);
  q.e[1] = 0.5 * sqrt(max0(1 - R(0, 0) + R(1, 1) - R(2, 2))) * (R(0, 2) - R(2, 0) >= 0 ? 1 : -1);
  q.e[2] = 0.5 * sqrt(max0(1 - R(0, 0) - R(1, 1) + R(2, 2))) * (R(1, 0) - R(0, 1) >= 0 ? 1 : -1);
  q.e[3] = 0.5 * sqrt(max0(1 + R(0, 0) + R(1, 1) + R(2, 2)));
  return q;
}

// Quadrotor::visualize's keyframe (LQRO:128-133): (float) time, position of
// xTrue, quatFromRot(RotTrue), as handed to CAL_AddGroupKeyState
LQRO_HD void keyframe(float* out, double time, const Mat<kX, 1>& xtrue, const Mat<3, 3>& Rtrue) {
  if (!out) return;
  const Mat<4, 1> q = quat_from_rot(Rtrue);
  out[0] = (float)time;
  for (int k = 0; k < 3; ++k) out[1 + k] = (float)xtrue.e[k];
  for (int k = 0; k < 4; ++k) out[4 + k] = (float)q.e[k];
}

template <int R, int C>
LQRO_HD Mat<R, C> get(const double* p) {
  Mat<R, C> m;
#pragma unroll
  for (int i = 0; i < R * C; ++i) m.e[i] = p[i];
  return m;
}

// Gains and noise weights of one agent.
struct AgentParams {
  const lqro_model* model;
  const double *L, *E, *l, *Lh, *Eh;   // U*X, U*V, U, V*X, V*V
  const double *u_goal, *p_goal;       // U, V
  const double *M, *Nz;                // X*X, Z*Z
  const double* normals;               // kNormals
  float* keyframe;                     // 8 floats or null
  double time;
};

// One agent through LQRO:1438-1445.  vgoal: in newV, out findVGoal(); u_out
// (may be null) receives findU().
LQRO_HD void agent_step(const AgentParams& a, double* x_, double* rot_, double* xt_, double* rott_,
                        double* P_, double* vgoal_, double* u_out) {
  const Quad q = quad(a.model);
  Mat<kX, 1> x = get<kX, 1>(x_), xtrue = get<kX, 1>(xt_);
  Mat<3, 3> R = get<3, 3>(rot_), Rtrue = get<3, 3>(rott_);
  Mat<kX, kX> P = get<kX, kX>(P_);
  const Mat<kX, kX> M = get<kX, kX>(a.M);
  const Mat<kZ, kZ> Nz = get<kZ, kZ>(a.Nz);
  const Mat<kU, 1> ug = get<kU, 1>(a.u_goal);
  const Vec3 vg = get<3, 1>(vgoal_);                                     // vGoal = newV
  const Mat<kU, 1> u = control_velocity(x, R, vg, ug, get<kU, kX>(a.L), get<kU, kV>(a.E),
                                        get<kU, 1>(a.l));                // findU
  propagate(q, xtrue, Rtrue, u, M, a.normals);                           // propagateU
  kalman_predict(q, x, R, u, M, P);                                      // kalmanFilter1
  const Mat<kZ, 1> z = sample_gaussian(observe(xtrue), Nz, a.normals + kX);
  kalman_update(q, x, R, z, Nz, P);                                      // kalmanFilter2
  const Vec3 vn = control_position(x, R, get<3, 1>(a.p_goal), ug, get<kV, kX>(a.Lh),
                                   get<kV, kV>(a.Eh));                   // findVGoal
  synth::put(x_, x); synth::put(rot_, R);
  synth::put(xt_, xtrue); synth::put(rott_, Rtrue);
  synth::put(P_, P); synth::put(vgoal_, vn);
  synth::put(u_out, u);
  keyframe(a.keyframe, a.time, xtrue, Rtrue);                            // visualize
}

}  // namespace dyn
}  // namespace lqro
