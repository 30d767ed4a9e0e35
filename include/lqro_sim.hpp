// lqro_sim.hpp — header-only C++ host side of liblqro.so, shaped like the
// reference simulator's agent loop so that it drops into it.
//
// Reference (hihixuyang/LQR-Obstacles, QuadrotorHoverController/):
//   class Quadrotor            LQRObstacles.cpp:73-165 (the fields the loop uses)
//   findMatrices / setup       LQRObstacles.cpp:1370-1373 (controlMatrices per agent)
//   the pair loop              LQRObstacles.cpp:1391-1436  -> Simulator::step()
//   the agent loop             LQRObstacles.cpp:1437-1446  -> Simulator::update()
//   simulator2.h:34-45         the prototypes of f, h, the filters and controllers
//                              these two calls replace on the GPU
//
// Everything numeric runs in liblqro.so through the C-ABI of lqro.h; this
// header only gathers the agents' fields into the flat arrays the ABI takes
// and scatters the results back.  Matrices are row-major double arrays, the
// element order of the reference's Matrix<R,C> (include/matrix.h:16,48).
// A non-zero status from the library is thrown as lqro::Error (the C-ABI
// itself never throws).
#ifndef LQRO_SIM_HPP
#define LQRO_SIM_HPP

#include <algorithm>
#include <array>
#include <cstdint>
#include <utility>
#include <stdexcept>
#include <string>
#include <vector>

#include "lqro.h"

namespace lqro {

constexpr int kX = 16, kU = 4, kV = 3;

struct Error : std::runtime_error {
  int status;
  Error(const std::string& what, int s) : std::runtime_error(what + ": " + lqro_status_string(s)), status(s) {}
};

inline void check(int s, const char* what) {
  if (s != LQRO_OK) throw Error(what, s);
}

// The Quadrotor fields of LQRO:73-165 that the pair loop and the agent loop
// read and write.
struct Quadrotor {
  std::array<double, kX> x{};                 // estimate (State x)
  std::array<double, 9> Rot{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
  std::array<double, kX> xTrue{};
  std::array<double, 9> RotTrue{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
  std::array<double, kX * kX> P{};
  std::array<double, kV> vGoal{}, newV{}, pGoal{};
  std::array<double, kU> uGoal{};
  std::array<double, kU * kX> L{};
  std::array<double, kU * kV> E{};
  std::array<double, kU> l{};
  std::array<double, kV * kX> Lh{};
  std::array<double, kV * kV> Eh{};

  // setupQuadrotors (LQRO:107-122) without its initial noise draw: xTrue = x,
  // RotTrue = Rot, P = p0 I, uGoal = hover
  void setup(const std::array<double, kX>& x0, const std::array<double, kV>& p_goal, double hover,
             double p0 = 1e-9) {
    x = x0;
    xTrue = x0;
    pGoal = p_goal;
    for (int k = 0; k < kU; ++k) uGoal[k] = hover;
    for (int k = 0; k < kX * kX; ++k) P[k] = (k % (kX + 1) == 0) ? p0 : 0.0;
  }
};

class Simulator {
 public:
  // qlist is held by reference, as the reference's qlist of Quadrotor*.
  Simulator(std::vector<Quadrotor>& qlist, int horizon, int n_points = 100, int device = 0)
      : q_(qlist), device_(device) {
    lqro_model_default(&model_);
    lqro_config cfg;
    lqro_config_default(&cfg, (int32_t)q_.size(), horizon, n_points);
    cfg.device = device;
    check(lqro_create(&cfg, &ctx_), "lqro_create");
    const size_t n = q_.size();
    xs_.resize(n * kX);
    vg_.resize(n * kV);
    nv_.resize(n * kV);
  }
  ~Simulator() { lqro_destroy(ctx_); }
  Simulator(const Simulator&) = delete;
  Simulator& operator=(const Simulator&) = delete;

  const lqro_model& model() const { return model_; }

  // controlMatrices at hover for every agent (LQRO:1370-1373): one synthesis,
  // the same L, E, Lh, Eh for all agents as in the reference; A, B feed the
  // pair loop's findFG (LQRO:1265-1266).
  void findMatrices() {
    std::vector<double> c(kX);
    check(lqro_synthesize_gains_x(&model_, kX, A_.data(), B_.data(), c.data(), q_[0].L.data(), q_[0].E.data(),
                                  q_[0].l.data(), q_[0].Lh.data(), q_[0].Eh.data()),
          "lqro_synthesize_gains_x");
    for (auto& q : q_) {
      q.L = q_[0].L; q.E = q_[0].E; q.l = q_[0].l; q.Lh = q_[0].Lh; q.Eh = q_[0].Eh;
    }
    check(lqro_set_gains(ctx_, A_.data(), B_.data(), q_[0].L.data(), q_[0].E.data(), 0), "lqro_set_gains");
  }

  // The pair loop LQRO:1393-1436 on the GPU: every Quadrotor::newV.
  // LQRO_E_HULL (a pair without its half-plane) and LQRO_E_QHMERGE (a pair
  // whose winning facet qconvex's pre-merge may join: its half-plane is not
  // pinned to the reference) still write newV: it is stored, then thrown
  // as lqro::Error (status(), hull_failures(), qhmerge_pairs() say which).
  void step() {
    for (size_t i = 0; i < q_.size(); ++i)
      for (int c = 0; c < kX; ++c) xs_[i * kX + c] = q_[i].x[c];
    for (size_t i = 0; i < q_.size(); ++i)
      for (int c = 0; c < kV; ++c) vg_[i * kV + c] = q_[i].vGoal[c];
    const int s = lqro_step(ctx_, xs_.data(), vg_.data(), nv_.data());
    if (s == LQRO_OK || s == LQRO_E_HULL || s == LQRO_E_QHMERGE)
      for (size_t i = 0; i < q_.size(); ++i)
        for (int c = 0; c < kV; ++c) q_[i].newV[c] = nv_[i * kV + c];
    check(s, "lqro_step");
  }

  // (i, j) of the last step's pairs lqro_get_hull_failures /
  // lqro_get_qhmerge_pairs name (at most 64 each)
  std::vector<std::pair<int, int>> hull_failures() const { return named(lqro_get_hull_failures); }
  std::vector<std::pair<int, int>> qhmerge_pairs() const { return named(lqro_get_qhmerge_pairs); }

  // The agent loop LQRO:1437-1446 on the GPU: vGoal = newV, findU,
  // propagate, kalmanFilter1, the observation draw, kalmanFilter2,
  // vGoal = findVGoal.  Noise from the reference's rand() stream at `seed`
  // (srand); returns the next seed.
  uint32_t update(uint32_t seed) {
    const size_t n = q_.size();
    std::vector<double> x(n * kX), rot(n * 9), xt(n * kX), rott(n * 9), P(n * kX * kX), vg(n * kV), ug(n * kU),
        pg(n * kV), L(n * kU * kX), E(n * kU * kV), l(n * kU), Lh(n * kV * kX), Eh(n * kV * kV),
        nrm(n * LQRO_NORMALS_PER_AGENT), M(kX * kX, 0.0), Nz(36, 0.0);
    for (int k = 0; k < kX; ++k) M[k * (kX + 1)] = 1e-9;   // LQRO:1285
    for (int k = 0; k < 6; ++k) Nz[k * 7] = 1e-9;          // LQRO:1286
    auto put = [](std::vector<double>& dst, size_t i, const double* src, size_t len) {
      for (size_t k = 0; k < len; ++k) dst[i * len + k] = src[k];
    };
    for (size_t i = 0; i < n; ++i) {
      const Quadrotor& q = q_[i];
      put(x, i, q.x.data(), kX); put(rot, i, q.Rot.data(), 9); put(xt, i, q.xTrue.data(), kX);
      put(rott, i, q.RotTrue.data(), 9); put(P, i, q.P.data(), kX * kX);
      put(vg, i, q.newV.data(), kV);   // vGoal = newV (LQRO:1438)
      put(ug, i, q.uGoal.data(), kU); put(pg, i, q.pGoal.data(), kV);
      put(L, i, q.L.data(), kU * kX); put(E, i, q.E.data(), kU * kV); put(l, i, q.l.data(), kU);
      put(Lh, i, q.Lh.data(), kV * kX); put(Eh, i, q.Eh.data(), kV * kV);
    }
    check(lqro_normals(&seed, (int64_t)nrm.size(), nrm.data()), "lqro_normals");
    lqro_agents a;
    a.x = x.data(); a.rot = rot.data(); a.x_true = xt.data(); a.rot_true = rott.data(); a.P = P.data();
    a.vgoal = vg.data(); a.u = nullptr; a.u_goal = ug.data(); a.p_goal = pg.data();
    a.L = L.data(); a.E = E.data(); a.l = l.data(); a.Lh = Lh.data(); a.Eh = Eh.data();
    a.M = M.data(); a.N = Nz.data(); a.normals = nrm.data(); a.keyframes = nullptr;
    a.time = t_ * model_.dt;
    check(lqro_dynamics_step(&model_, 1, (int32_t)n, 1, &a, device_), "lqro_dynamics_step");
    auto get = [](std::vector<double>& src, size_t i, double* dst, size_t len) {
      for (size_t k = 0; k < len; ++k) dst[k] = src[i * len + k];
    };
    for (size_t i = 0; i < n; ++i) {
      Quadrotor& q = q_[i];
      get(x, i, q.x.data(), kX); get(rot, i, q.Rot.data(), 9); get(xt, i, q.xTrue.data(), kX);
      get(rott, i, q.RotTrue.data(), 9); get(P, i, q.P.data(), kX * kX); get(vg, i, q.vGoal.data(), kV);
    }
    ++t_;
    return seed;
  }

 private:
  std::vector<std::pair<int, int>> named(int (*get)(lqro_ctx*, int64_t*, int64_t, int64_t*)) const {
    int64_t p[128], n = 0;
    check(get(ctx_, p, 64, &n), "lqro_get_*_pairs");
    std::vector<std::pair<int, int>> out;
    for (int64_t k = 0; k < std::min<int64_t>(n, 64); ++k) out.emplace_back((int)p[2 * k], (int)p[2 * k + 1]);
    return out;
  }

  std::vector<Quadrotor>& q_;
  int device_;
  lqro_model model_;
  lqro_ctx* ctx_ = nullptr;
  std::array<double, kX * kX> A_{};
  std::array<double, kX * kU> B_{};
  std::vector<double> xs_, vg_, nv_;
  int t_ = 0;
};

}  // namespace lqro
#endif  // LQRO_SIM_HPP
