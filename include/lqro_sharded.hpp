// lqro_sharded.hpp — the multi-GPU host in C++: one process per GPU, each
// rank the reference's agent loop (LQRObstacles.cpp:1391-1446) for its block
// of agents, one RCCL all-gather of the agents' state per iteration.
//
// The reference runs the loop on one CPU; its pair loop (LQRO:1393-1436) is
// independent per row i, and the agent loop (LQRO:1437-1446) per agent, so
// rows shard with no exchange inside a step.  What a rank needs from the
// others is only the next iteration's x_j of every agent (the pair loop reads
// all of them): one ncclAllGather of the X doubles per agent, enqueued on the
// same stream as the kernels that produce them, so nothing synchronises
// inside an iteration.
//
//   per iteration, on `stream`:
//     lqro_step_device_begin      the pair loop's sweep and hulls for rows [row_begin, row_end)
//     ncclAllGather               each row's last normal (the reference's loop-carried
//                                 normalVector, LQRO:1385, runs through every row)
//     lqro_step_device_end        the facet-0 pairs' normals, the LP: newV of the own rows
//     hipMemcpyAsync              vGoal = newV (LQRO:1438), own rows
//     lqro_dynamics_step_device   findU, propagate, kalmanFilter1/2, findVGoal (LQRO:1439-1445), own rows
//     ncclAllGather               x of every agent, in place
//     (host)                      the iteration's hull failures and merge suspects,
//                                 exchanged so every rank throws lqro::Error
//                                 (LQRO_E_HULL, else LQRO_E_QHMERGE) together
//
// The noise draws follow the reference's single rand() stream in agent order
// (normal(), LQRO:334-350): every rank draws the whole iteration's stream
// (lqro_normals) and uploads its own rows' slice, so any world size replays
// the same trajectory as lqro::Simulator (lqro_sim.hpp) on one GPU.
//
// Build: hipcc -std=c++17 -Iinclude app.cpp -Llqr-obstacles_amd -llqro -lrccl
// (tests/cpp/lqro_sharded_main.cpp, __graft_entry__.build_cpp_sharded).
#ifndef LQRO_SHARDED_HPP
#define LQRO_SHARDED_HPP

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <functional>
#include <vector>

#include "lqro_sim.hpp"

namespace lqro {

inline void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(std::string(what) + " (" + hipGetErrorString(e) + ")", LQRO_E_HIP);
}
inline void check_nccl(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw Error(std::string(what) + " (" + ncclGetErrorString(r) + ")", LQRO_E_HIP);
}

class ShardedSimulator {
 public:
  // The row exchange: d is a row-major n x w device table of which every
  // rank r holds rows [block_begin(n, r, world), block_begin(n, r+1, world));
  // afterwards every rank holds all of it (an allgatherv), ordered on
  // `stream`.  The default is RCCL (allgather_rows below); a caller running
  // several ranks in one process passes its own (tests/cpp/lqro_sharded_main.cpp).
  using Exchange = std::function<void(double* d, int w, hipStream_t stream)>;

  // qlist: every agent (each rank holds the whole list, as the reference's
  // qlist); rank r owns rows [r*n/world, (r+1)*n/world) — lqro.shard_rows'
  // balanced blocks, so the C++ and Python hosts lay shards out alike; a
  // rank may own no row (n < world) and still takes part in the exchanges.
  // id: ncclGetUniqueId on rank 0, handed to the others by the caller (a
  // file, MPI, torch.distributed ...).
  ShardedSimulator(std::vector<Quadrotor>& qlist, int horizon, int n_points, int rank, int world,
                   const ncclUniqueId& id, int device = 0)
      : q_(qlist), rank_(rank), world_(world), device_(device) {
    init(horizon, n_points);
    check_nccl(ncclCommInitRank(&comm_, world_, id, rank_), "ncclCommInitRank");
    ex_ = [this](double* d, int w, hipStream_t s) { allgather_rows(d, w, s); };
  }
  ShardedSimulator(std::vector<Quadrotor>& qlist, int horizon, int n_points, int rank, int world, Exchange ex,
                   int device = 0)
      : q_(qlist), rank_(rank), world_(world), device_(device), ex_(std::move(ex)) {
    init(horizon, n_points);
  }

 private:
  void init(int horizon, int n_points) {
    n_ = (int)q_.size();
    rb_ = block_begin(n_, rank_, world_);
    re_ = block_begin(n_, rank_ + 1, world_);
    rows_ = re_ - rb_;
    lqro_model_default(&model_);
    lqro_config cfg;
    lqro_config_default(&cfg, n_, horizon, n_points);
    cfg.device = device_;
    cfg.row_begin = rb_;
    cfg.row_end = re_;
    // (a rank without rows needs no context; a zero-row context is invalid)
    if (rows_ > 0) check(lqro_create(&cfg, &ctx_), "lqro_create");   // fails loudly without a gfx950 device
    else check_device();
    check_hip(hipSetDevice(device_), "hipSetDevice");
    check_hip(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    const size_t na = (size_t)n_, r = (size_t)std::max(rows_, 1);
    alloc(&d_x_, na * kX);
    alloc(&d_vg_, na * kV);
    alloc(&d_newv_, na * kV);
    alloc(&d_rowtab_, na * 4);
    alloc(&d_fail_, na * 2);
    alloc(&d_rot_, r * 9);
    alloc(&d_xt_, r * kX);
    alloc(&d_rott_, r * 9);
    alloc(&d_P_, r * kX * kX);
    alloc(&d_ug_, r * kU);
    alloc(&d_pg_, r * kV);
    alloc(&d_nrm_, r * LQRO_NORMALS_PER_AGENT);
    alloc(&d_L_, kU * kX);
    alloc(&d_E_, kU * kV);
    alloc(&d_l_, kU);
    alloc(&d_Lh_, kV * kX);
    alloc(&d_Eh_, kV * kV);
    alloc(&d_M_, kX * kX);
    alloc(&d_N_, 36);
    check_hip(hipMalloc(&d_model_, sizeof(lqro_model)), "hipMalloc");
    upload();
  }

 public:
  ~ShardedSimulator() {
    if (comm_) ncclCommDestroy(comm_);
    for (double* p : {d_x_, d_vg_, d_newv_, d_rowtab_, d_fail_, d_rot_, d_xt_, d_rott_, d_P_, d_ug_, d_pg_, d_nrm_, d_L_, d_E_, d_l_,
                      d_Lh_, d_Eh_, d_M_, d_N_})
      if (p) (void)hipFree(p);
    if (d_model_) (void)hipFree(d_model_);
    if (stream_) (void)hipStreamDestroy(stream_);
    if (ctx_) lqro_destroy(ctx_);
  }
  ShardedSimulator(const ShardedSimulator&) = delete;
  ShardedSimulator& operator=(const ShardedSimulator&) = delete;

  int row_begin() const { return rb_; }
  lqro_ctx* context() const { return ctx_; }   // null on a rank without rows
  int row_end() const { return re_; }
  // rank r's first row: floor(r n / world) (lqro.shard_rows' block mode)
  static int block_begin(int n, int r, int world) { return (int)(((long long)r * n) / world); }

  // controlMatrices at hover (LQRO:1370-1373), the same synthesis as
  // Simulator::findMatrices, on every rank
  void findMatrices() {
    std::vector<double> c(kX);
    check(lqro_synthesize_gains_x(&model_, kX, A_.data(), B_.data(), c.data(), q_[0].L.data(), q_[0].E.data(),
                                  q_[0].l.data(), q_[0].Lh.data(), q_[0].Eh.data()),
          "lqro_synthesize_gains_x");
    for (auto& q : q_) {
      q.L = q_[0].L; q.E = q_[0].E; q.l = q_[0].l; q.Lh = q_[0].Lh; q.Eh = q_[0].Eh;
    }
    if (ctx_) check(lqro_set_gains(ctx_, A_.data(), B_.data(), q_[0].L.data(), q_[0].E.data(), 0), "lqro_set_gains");
    put(d_L_, q_[0].L.data(), kU * kX);
    put(d_E_, q_[0].E.data(), kU * kV);
    put(d_l_, q_[0].l.data(), kU);
    put(d_Lh_, q_[0].Lh.data(), kV * kX);
    put(d_Eh_, q_[0].Eh.data(), kV * kV);
    check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
  }

  // One iteration of LQRO:1393-1446 for this rank's rows, then the state
  // exchange; returns the next seed of the rand() stream.  Enqueued only:
  // download() waits for it.
  uint32_t iterate(uint32_t seed) {
    nrm_.resize((size_t)n_ * LQRO_NORMALS_PER_AGENT);
    check(lqro_normals(&seed, (int64_t)nrm_.size(), nrm_.data()), "lqro_normals");
    if (world_ > 1) {
      // Qhull order (lqro_config_default): the normal entering each shard is
      // the last one of the rows before it, on whichever rank
      if (ctx_) check(lqro_step_device_begin(ctx_, d_x_, d_vg_, d_rowtab_, stream_), "lqro_step_device_begin");
      ex_(d_rowtab_, 4, stream_);
      if (ctx_) check(lqro_step_device_end(ctx_, d_rowtab_, d_newv_, stream_), "lqro_step_device_end");
    } else {
      check(lqro_step_device(ctx_, d_x_, d_vg_, d_newv_, stream_), "lqro_step_device");
    }
    if (rows_ > 0) {
      check_hip(hipMemcpyAsync(d_vg_ + (size_t)rb_ * kV, d_newv_ + (size_t)rb_ * kV, sizeof(double) * rows_ * kV,
                               hipMemcpyDeviceToDevice, stream_),
                "hipMemcpyAsync");   // vGoal = newV (LQRO:1438)
      check_hip(hipMemcpyAsync(d_nrm_, nrm_.data() + (size_t)rb_ * LQRO_NORMALS_PER_AGENT,
                               sizeof(double) * rows_ * LQRO_NORMALS_PER_AGENT, hipMemcpyHostToDevice, stream_),
                "hipMemcpyAsync");
      lqro_agents a;
      a.x = d_x_ + (size_t)rb_ * kX; a.rot = d_rot_; a.x_true = d_xt_; a.rot_true = d_rott_; a.P = d_P_;
      a.vgoal = d_vg_ + (size_t)rb_ * kV; a.u = nullptr; a.u_goal = d_ug_; a.p_goal = d_pg_;
      a.L = d_L_; a.E = d_E_; a.l = d_l_; a.Lh = d_Lh_; a.Eh = d_Eh_; a.M = d_M_; a.N = d_N_;
      a.normals = d_nrm_; a.keyframes = nullptr;
      a.time = t_ * model_.dt;
      check(lqro_dynamics_step_device(d_model_, 1, rows_, 0, &a, stream_), "lqro_dynamics_step_device");
    }
    // x of every agent for the next pair loop (in place: rank r's rows are its send buffer)
    ex_(d_x_, kX, stream_);
    // the host copy waits for the iteration (the normals' staging buffer is reused)
    check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    ++t_;
    // A hull this rank could not build left a pair without its half-plane
    // (the reference's qconvex always returns one, LQRO:879-880), and a pair
    // whose winner qconvex's pre-merge may join has a half-plane not pinned
    // to the reference (LQRO:925-967): never silently.  Every rank learns the
    // swarm's totals (one n x 2 exchange: each rank's two counts in its first
    // row), so all of them throw together and none is left waiting in the
    // next iteration's collectives.
    int64_t st[12] = {0};
    if (ctx_) check(lqro_get_stats_ex(ctx_, st, 12), "lqro_get_stats_ex");
    rank_hull_fail_ = st[4];
    rank_qhmerge_ = st[11];
    std::vector<double> f((size_t)n_ * 2, 0.0);
    if (rows_ > 0) {
      f[2 * (size_t)rb_] = (double)st[4];
      f[2 * (size_t)rb_ + 1] = (double)st[11];
      put(d_fail_ + 2 * (size_t)rb_, f.data() + 2 * (size_t)rb_, 2 * (size_t)rows_);
    }
    ex_(d_fail_, 2, stream_);
    get(f.data(), d_fail_, 2 * (size_t)n_);   // (ordered after the exchange on stream_)
    double tot = 0.0, totm = 0.0;
    for (int i = 0; i < n_; ++i) { tot += f[2 * (size_t)i]; totm += f[2 * (size_t)i + 1]; }
    hull_fail_ = (int64_t)tot;
    qhmerge_ = (int64_t)totm;
    if (hull_fail_ > 0)
      throw Error("lqro::ShardedSimulator: " + std::to_string(hull_fail_) +
                      " inside-hull pair(s) left without a half-plane (rank " + std::to_string(rank_) + ": " +
                      std::to_string(rank_hull_fail_) + "; lqro_get_hull_failures)",
                  LQRO_E_HULL);
    if (qhmerge_ > 0)
      throw Error("lqro::ShardedSimulator: " + std::to_string(qhmerge_) +
                      " inside-hull pair(s) whose winning facet qconvex may merge (rank " + std::to_string(rank_) +
                      ": " + std::to_string(rank_qhmerge_) + "; lqro_get_qhmerge_pairs)",
                  LQRO_E_QHMERGE);
    return seed;
  }

  // hull failures of the last iteration: the whole swarm's (every rank sees
  // the same number) and this rank's own rows'
  int64_t hull_failures() const { return hull_fail_; }
  int64_t rank_hull_failures() const { return rank_hull_fail_; }
  // merge-suspect pairs (LQRO_REC_QHMERGE_WIN) of the last iteration: the
  // swarm's and this rank's
  int64_t qhmerge_pairs() const { return qhmerge_; }
  int64_t rank_qhmerge_pairs() const { return rank_qhmerge_; }

  // The device state back into qlist: every agent's x, this rank's rows'
  // full state and newV.
  void download() {
    check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    std::vector<double> x((size_t)n_ * kX), nv((size_t)std::max(rows_, 1) * kV), vg(nv.size()),
        rot((size_t)std::max(rows_, 1) * 9), xt((size_t)std::max(rows_, 1) * kX), rott(rot.size()),
        P((size_t)std::max(rows_, 1) * kX * kX);
    get(x.data(), d_x_, x.size());
    for (int i = 0; i < n_; ++i)
      for (int c = 0; c < kX; ++c) q_[i].x[c] = x[(size_t)i * kX + c];
    if (rows_ == 0) return;
    get(nv.data(), d_newv_ + (size_t)rb_ * kV, (size_t)rows_ * kV);
    get(vg.data(), d_vg_ + (size_t)rb_ * kV, (size_t)rows_ * kV);
    get(rot.data(), d_rot_, (size_t)rows_ * 9);
    get(xt.data(), d_xt_, (size_t)rows_ * kX);
    get(rott.data(), d_rott_, (size_t)rows_ * 9);
    get(P.data(), d_P_, (size_t)rows_ * kX * kX);
    for (int r = 0; r < rows_; ++r) {
      Quadrotor& q = q_[rb_ + r];
      for (int c = 0; c < kV; ++c) { q.newV[c] = nv[(size_t)r * kV + c]; q.vGoal[c] = vg[(size_t)r * kV + c]; }
      for (int c = 0; c < 9; ++c) { q.Rot[c] = rot[(size_t)r * 9 + c]; q.RotTrue[c] = rott[(size_t)r * 9 + c]; }
      for (int c = 0; c < kX; ++c) q.xTrue[c] = xt[(size_t)r * kX + c];
      for (int c = 0; c < kX * kX; ++c) q.P[c] = P[(size_t)r * kX * kX + c];
    }
  }

 private:
  // The all-gather of a row-major n x w table whose rows [rb_r, re_r) rank r
  // holds.  Equal blocks (n a multiple of world: C4, C5 at 8 GPUs): one
  // in-place ncclAllGather (rank r's send buffer is its own rows of d).
  // Unequal blocks: one broadcast per rank, from its rows in place, in one
  // group (an allgatherv).
  void allgather_rows(double* d, int w, hipStream_t stream) {
    if (n_ % world_ == 0) {
      const size_t cnt = (size_t)(n_ / world_) * w;
      check_nccl(ncclAllGather(d + (size_t)rb_ * w, d, cnt, ncclDouble, comm_, stream), "ncclAllGather");
      return;
    }
    check_nccl(ncclGroupStart(), "ncclGroupStart");
    for (int r = 0; r < world_; ++r) {
      const int b = block_begin(n_, r, world_), e = block_begin(n_, r + 1, world_);
      if (e > b)
        check_nccl(ncclBroadcast(d + (size_t)b * w, d + (size_t)b * w, (size_t)(e - b) * w, ncclDouble, r, comm_,
                                 stream),
                   "ncclBroadcast");
    }
    check_nccl(ncclGroupEnd(), "ncclGroupEnd");
  }
  // what lqro_create checks, for a rank that owns no row
  void check_device() {
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device_ >= nd) throw Error("no gfx950 device", LQRO_E_NODEVICE);
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, device_) != hipSuccess || std::string(pr.gcnArchName).rfind("gfx950", 0) != 0)
      throw Error("no gfx950 device", LQRO_E_NODEVICE);
  }
  void alloc(double** p, size_t n) {
    check_hip(hipMalloc(p, sizeof(double) * std::max<size_t>(n, 1)), "hipMalloc");
    check_hip(hipMemsetAsync(*p, 0, sizeof(double) * std::max<size_t>(n, 1), stream_), "hipMemsetAsync");
  }
  void put(double* d, const double* h, size_t n) {
    check_hip(hipMemcpyAsync(d, h, sizeof(double) * n, hipMemcpyHostToDevice, stream_), "hipMemcpyAsync");
  }
  // stream-ordered: stream_ is non-blocking, so a plain hipMemcpy on the
  // null stream would not wait for the exchange enqueued on it
  void get(double* h, const double* d, size_t n) {
    check_hip(hipMemcpyAsync(h, d, sizeof(double) * n, hipMemcpyDeviceToHost, stream_), "hipMemcpyAsync");
    check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
  }
  // qlist -> device: every agent's x and vGoal, the own rows' state; the
  // noise variances M, N (LQRO:1285-1286)
  void upload() {
    std::vector<double> x((size_t)n_ * kX), vg((size_t)n_ * kV);
    for (int i = 0; i < n_; ++i) {
      for (int c = 0; c < kX; ++c) x[(size_t)i * kX + c] = q_[i].x[c];
      for (int c = 0; c < kV; ++c) vg[(size_t)i * kV + c] = q_[i].vGoal[c];
    }
    put(d_x_, x.data(), x.size());
    put(d_vg_, vg.data(), vg.size());
    std::vector<double> rot((size_t)std::max(rows_, 1) * 9), xt((size_t)std::max(rows_, 1) * kX), rott(rot.size()),
        P((size_t)std::max(rows_, 1) * kX * kX), ug((size_t)std::max(rows_, 1) * kU),
        pg((size_t)std::max(rows_, 1) * kV);
    for (int r = 0; r < rows_; ++r) {
      const Quadrotor& q = q_[rb_ + r];
      for (int c = 0; c < 9; ++c) { rot[(size_t)r * 9 + c] = q.Rot[c]; rott[(size_t)r * 9 + c] = q.RotTrue[c]; }
      for (int c = 0; c < kX; ++c) xt[(size_t)r * kX + c] = q.xTrue[c];
      for (int c = 0; c < kX * kX; ++c) P[(size_t)r * kX * kX + c] = q.P[c];
      for (int c = 0; c < kU; ++c) ug[(size_t)r * kU + c] = q.uGoal[c];
      for (int c = 0; c < kV; ++c) pg[(size_t)r * kV + c] = q.pGoal[c];
    }
    if (rows_ > 0) {
      put(d_rot_, rot.data(), (size_t)rows_ * 9);
      put(d_xt_, xt.data(), (size_t)rows_ * kX);
      put(d_rott_, rott.data(), (size_t)rows_ * 9);
      put(d_P_, P.data(), (size_t)rows_ * kX * kX);
      put(d_ug_, ug.data(), (size_t)rows_ * kU);
      put(d_pg_, pg.data(), (size_t)rows_ * kV);
    }
    std::vector<double> M(kX * kX, 0.0), Nz(36, 0.0);
    for (int k = 0; k < kX; ++k) M[k * (kX + 1)] = 1e-9;   // LQRO:1285
    for (int k = 0; k < 6; ++k) Nz[k * 7] = 1e-9;          // LQRO:1286
    put(d_M_, M.data(), M.size());
    put(d_N_, Nz.data(), Nz.size());
    check_hip(hipMemcpyAsync(d_model_, &model_, sizeof model_, hipMemcpyHostToDevice, stream_), "hipMemcpyAsync");
    check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
  }

  std::vector<Quadrotor>& q_;
  int n_ = 0, rank_ = 0, world_ = 1, device_ = 0, rb_ = 0, re_ = 0, rows_ = 0, t_ = 0;
  int64_t hull_fail_ = 0, rank_hull_fail_ = 0, qhmerge_ = 0, rank_qhmerge_ = 0;
  lqro_model model_;
  lqro_ctx* ctx_ = nullptr;
  hipStream_t stream_ = nullptr;
  ncclComm_t comm_ = nullptr;
  Exchange ex_;
  std::array<double, kX * kX> A_{};
  std::array<double, kX * kU> B_{};
  std::vector<double> nrm_;
  double *d_x_ = nullptr, *d_vg_ = nullptr, *d_newv_ = nullptr, *d_rowtab_ = nullptr, *d_fail_ = nullptr, *d_rot_ = nullptr, *d_xt_ = nullptr,
         *d_rott_ = nullptr, *d_P_ = nullptr, *d_ug_ = nullptr, *d_pg_ = nullptr, *d_nrm_ = nullptr, *d_L_ = nullptr,
         *d_E_ = nullptr, *d_l_ = nullptr, *d_Lh_ = nullptr, *d_Eh_ = nullptr, *d_M_ = nullptr, *d_N_ = nullptr;
  lqro_model* d_model_ = nullptr;
};

}  // namespace lqro
#endif  // LQRO_SHARDED_HPP
