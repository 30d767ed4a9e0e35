// The C++ multi-rank host (include/lqro_sharded.hpp) against the one-GPU
// host (include/lqro_sim.hpp): the reference's agent loop
// (LQRObstacles.cpp:1391-1446) run by both from the same swarm and rand()
// seed, world size 1 (an RCCL communicator of one rank; the 2-rank exchange
// is the gloo tests' subject).
// usage: lqro_sharded_main IN OUT
//   IN : int32 N, H, NP, steps; uint32 seed; N*16 x; N*3 vGoal; N*3 pGoal (doubles)
//   OUT: per step: Simulator newV (N*3), x (N*16); ShardedSimulator newV (N*3), x (N*16)
#include <cstdio>
#include <cstdlib>
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

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s IN OUT\n", argv[0]);
    return 2;
  }
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
