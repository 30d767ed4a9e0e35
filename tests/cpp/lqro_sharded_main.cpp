// The C++ multi-rank host (include/lqro_sharded.hpp) against the one-GPU
// host (include/lqro_sim.hpp): the reference's agent loop
// (LQRObstacles.cpp:1391-1446) run by both from the same swarm and rand()
// seed.
// usage: lqro_sharded_main IN OUT [G]
//   no G: world size 1, an RCCL communicator of one rank;
//   G >= 2: G ranks in G threads on device 0 (RCCL takes one rank per GPU),
//     the ShardedSimulator's world > 1 path — lqro_step_device_begin, the
//     exchange of the row-normal table, lqro_step_device_end, the dynamics,
//     the exchange of x — with the exchange done in-process (every rank's
//     rows copied device to device between two barriers) instead of RCCL
//   IN : int32 N, H, NP, steps; uint32 seed; N*16 x; N*3 vGoal; N*3 pGoal (doubles)
//   OUT: per step: Simulator newV (N*3), x (N*16); ShardedSimulator newV (N*3), x (N*16)
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

#include "lqro_sharded.hpp"

static std::vector<lqro::Quadrotor> swarm(int N, const std::vector<double>& x, const std::vector<double>& vg,
                                          const std::vector<double>& pg) {
  std::vector<lqro::Quadrotor> qlist(N);
  lqro_model m;
  lqro_model_default(&m);
  const double hover = m.gravity * m.mass / 4;   // nominalInput (LQRO:188)
  for (int i = 0; i < N; ++i) {
    std::array<double, 16> xi;
    std::array<double, 3> pgi;
    for (int c = 0; c < 16; ++c) xi[c] = x[i * 16 + c];
    for (int c = 0; c < 3; ++c) pgi[c] = pg[i * 3 + c];
    qlist[i].setup(xi, pgi, hover);
    for (int c = 0; c < 3; ++c) qlist[i].vGoal[c] = vg[i * 3 + c];
  }
  return qlist;
}

// G ranks in one process: a barrier and every rank's buffer of the table
// being exchanged
struct Bus {
  int world;
  std::vector<double*> buf;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long gen = 0;
  explicit Bus(int g) : world(g), buf(g, nullptr) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const long my = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != my; });
    }
  }
};

// the threaded run: per step, the merged newV (each row from its owner) and
// x (every rank holds all of it: rank 0's)
static int run_threads(int G, int N, int H, int NP, int steps, uint32_t seed, const std::vector<double>& x,
                       const std::vector<double>& vg, const std::vector<double>& pg, std::vector<double>& nv_out,
                       std::vector<double>& x_out) {
  Bus bus(G);
  nv_out.assign((size_t)steps * N * 3, 0.0);
  x_out.assign((size_t)steps * N * 16, 0.0);
  std::vector<int> rc(G, 0);
  std::vector<std::string> err(G);
  std::vector<std::thread> th;
  for (int r = 0; r < G; ++r)
    th.emplace_back([&, r] {
      try {
        std::vector<lqro::Quadrotor> q = swarm(N, x, vg, pg);
        auto ex = [&, r](double* d, int w, hipStream_t s) {
          lqro::check_hip(hipStreamSynchronize(s), "hipStreamSynchronize");
          bus.buf[r] = d;
          bus.barrier();
          for (int o = 0; o < G; ++o) {
            const int b = lqro::ShardedSimulator::block_begin(N, o, G), e = lqro::ShardedSimulator::block_begin(N, o + 1, G);
            if (o != r && e > b)
              lqro::check_hip(hipMemcpy(d + (size_t)b * w, bus.buf[o] + (size_t)b * w, sizeof(double) * (e - b) * w,
                                        hipMemcpyDeviceToDevice),
                              "hipMemcpy");
          }
          bus.barrier();   // no rank overwrites its table before every rank copied it
        };
        lqro::ShardedSimulator sh(q, H, NP, r, G, ex);
        sh.findMatrices();
        uint32_t sd = seed;
        for (int t = 0; t < steps; ++t) {
          sd = sh.iterate(sd);
          sh.download();
          for (int i = sh.row_begin(); i < sh.row_end(); ++i)
            for (int c = 0; c < 3; ++c) nv_out[((size_t)t * N + i) * 3 + c] = q[i].newV[c];
          if (r == 0)
            for (int i = 0; i < N; ++i)
              for (int c = 0; c < 16; ++c) x_out[((size_t)t * N + i) * 16 + c] = q[i].x[c];
        }
      } catch (const lqro::Error& e) {
        rc[r] = 1;
        err[r] = e.what();
      }
    });
  for (auto& t : th) t.join();
  for (int r = 0; r < G; ++r)
    if (rc[r]) {
      std::fprintf(stderr, "lqro_sharded_main: rank %d: %s\n", r, err[r].c_str());
      return 1;
    }
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 3 && argc != 4) {
    std::fprintf(stderr, "usage: %s IN OUT [G]\n", argv[0]);
    return 2;
  }
  const int G = argc == 4 ? std::atoi(argv[3]) : 1;
  FILE* in = std::fopen(argv[1], "rb");
  if (!in) return 2;
  int32_t hdr[4];
  uint32_t seed = 0;
  if (std::fread(hdr, sizeof hdr, 1, in) != 1 || std::fread(&seed, sizeof seed, 1, in) != 1) return 2;
  const int N = hdr[0], H = hdr[1], NP = hdr[2], steps = hdr[3];
  std::vector<double> x(N * 16), vg(N * 3), pg(N * 3);
  if (std::fread(x.data(), sizeof(double), x.size(), in) != x.size() ||
      std::fread(vg.data(), sizeof(double), vg.size(), in) != vg.size() ||
      std::fread(pg.data(), sizeof(double), pg.size(), in) != pg.size())
    return 2;
  std::fclose(in);
  FILE* out = std::fopen(argv[2], "wb");
  if (!out) return 2;
  try {
    std::vector<lqro::Quadrotor> qa = swarm(N, x, vg, pg), qb = swarm(N, x, vg, pg);
    lqro::Simulator sim(qa, H, NP);
    sim.findMatrices();
    // the context first: without a gfx950 device this throws before RCCL is touched
    lqro_config probe;
    lqro_config_default(&probe, N, H, NP);
    lqro_ctx* c = nullptr;
    lqro::check(lqro_create(&probe, &c), "lqro_create");
    lqro_destroy(c);
    if (G >= 2) {
      std::vector<double> nvb, xb;
      if (run_threads(G, N, H, NP, steps, seed, x, vg, pg, nvb, xb)) {
        std::fclose(out);
        return 1;
      }
      uint32_t sa = seed;
      for (int t = 0; t < steps; ++t) {
        sim.step();
        sa = sim.update(sa);
        for (const auto& q : qa) std::fwrite(q.newV.data(), sizeof(double), 3, out);
        for (const auto& q : qa) std::fwrite(q.x.data(), sizeof(double), 16, out);
        std::fwrite(nvb.data() + (size_t)t * N * 3, sizeof(double), (size_t)N * 3, out);
        std::fwrite(xb.data() + (size_t)t * N * 16, sizeof(double), (size_t)N * 16, out);
      }
      std::fclose(out);
      return 0;
    }
    ncclUniqueId id;
    lqro::check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
    lqro::ShardedSimulator sh(qb, H, NP, 0, 1, id);
    sh.findMatrices();
    uint32_t sa = seed, sb = seed;
    for (int t = 0; t < steps; ++t) {
      sim.step();
      sa = sim.update(sa);
      sb = sh.iterate(sb);
      sh.download();
      for (const auto& q : qa) std::fwrite(q.newV.data(), sizeof(double), 3, out);
      for (const auto& q : qa) std::fwrite(q.x.data(), sizeof(double), 16, out);
      for (const auto& q : qb) std::fwrite(q.newV.data(), sizeof(double), 3, out);
      for (const auto& q : qb) std::fwrite(q.x.data(), sizeof(double), 16, out);
    }
    if (sa != sb) {
      std::fprintf(stderr, "lqro_sharded_main: rand() streams diverged\n");
      std::fclose(out);
      return 1;
    }
  } catch (const lqro::Error& e) {
    std::fprintf(stderr, "lqro_sharded_main: %s\n", e.what());
    std::fclose(out);
    return 1;
  }
  std::fclose(out);
  return 0;
}
