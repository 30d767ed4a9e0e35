// bench.py --host cpp: one rank of the C++ multi-GPU host
// (include/lqro_sharded.hpp, lqro::ShardedSimulator) timed over K iterations
// of the reference's agent loop (LQRObstacles.cpp:1391-1446) — the pair loop
// (begin, row-normal all-gather, end when world > 1), the dynamics and the
// all-gather of x over RCCL — one process per GPU.
// usage: lqro_bench_main IN UID_FILE RANK WORLD DEVICE WARMUP STEPS
//   IN: int32 N, H, NP, steps; uint32 seed; N*16 x; N*3 vGoal; N*3 pGoal (doubles)
//       (tests/cpp/lqro_sharded_main.cpp's format)
//   UID_FILE: rank 0 writes two ncclUniqueIds there (the simulator's and the
//       timing communicator's; written to UID_FILE.tmp, then renamed); the
//       other ranks wait up to 120 s for it
// Prints on rank 0 one line "lqro_bench_main key=value ...": elapsed_s is the
// max over ranks of the timed iterations' wall time, between two barriers
// (an all-reduce, then a stream synchronize).
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
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

static bool uids(const char* path, int rank, ncclUniqueId id[2]) {
  if (rank == 0) {
    for (int k = 0; k < 2; ++k) lqro::check_nccl(ncclGetUniqueId(&id[k]), "ncclGetUniqueId");
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f || std::fwrite(id, sizeof(ncclUniqueId), 2, f) != 2 || std::fclose(f) != 0) return false;
    return std::rename(tmp.c_str(), path) == 0;
  }
  for (int t = 0; t < 12000; ++t) {
    FILE* f = std::fopen(path, "rb");
    if (f) {
      const bool ok = std::fread(id, sizeof(ncclUniqueId), 2, f) == 2;
      std::fclose(f);
      if (ok) return true;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  return false;
}

int main(int argc, char** argv) {
  if (argc != 8) {
    std::fprintf(stderr, "usage: %s IN UID_FILE RANK WORLD DEVICE WARMUP STEPS\n", argv[0]);
    return 2;
  }
  const int rank = std::atoi(argv[3]), world = std::atoi(argv[4]), device = std::atoi(argv[5]);
  const int warmup = std::atoi(argv[6]), steps = std::atoi(argv[7]);
  FILE* in = std::fopen(argv[1], "rb");
  if (!in) return 2;
  int32_t hdr[4];
  uint32_t seed = 0;
  if (std::fread(hdr, sizeof hdr, 1, in) != 1 || std::fread(&seed, sizeof seed, 1, in) != 1) return 2;
  const int N = hdr[0], H = hdr[1], NP = hdr[2];
  std::vector<double> x((size_t)N * 16), vg((size_t)N * 3), pg((size_t)N * 3);
  if (std::fread(x.data(), sizeof(double), x.size(), in) != x.size() ||
      std::fread(vg.data(), sizeof(double), vg.size(), in) != vg.size() ||
      std::fread(pg.data(), sizeof(double), pg.size(), in) != pg.size())
    return 2;
  std::fclose(in);
  try {
    lqro::check_hip(hipSetDevice(device), "hipSetDevice");
    ncclUniqueId id[2];
    if (!uids(argv[2], rank, id)) {
      std::fprintf(stderr, "lqro_bench_main: rank %d: no communicator id in %s\n", rank, argv[2]);
      return 1;
    }
    std::vector<lqro::Quadrotor> q = swarm(N, x, vg, pg);
    lqro::ShardedSimulator sh(q, H, NP, rank, world, id[0], device);
    ncclComm_t tc = nullptr;
    lqro::check_nccl(ncclCommInitRank(&tc, world, id[1], rank), "ncclCommInitRank");
    hipStream_t ts = nullptr;
    lqro::check_hip(hipStreamCreateWithFlags(&ts, hipStreamNonBlocking), "hipStreamCreate");
    double* d_t = nullptr;
    lqro::check_hip(hipMalloc(&d_t, sizeof(double)), "hipMalloc");
    auto allmax = [&](double v) {
      lqro::check_hip(hipMemcpyAsync(d_t, &v, sizeof v, hipMemcpyHostToDevice, ts), "hipMemcpyAsync");
      lqro::check_nccl(ncclAllReduce(d_t, d_t, 1, ncclDouble, ncclMax, tc, ts), "ncclAllReduce");
      lqro::check_hip(hipMemcpyAsync(&v, d_t, sizeof v, hipMemcpyDeviceToHost, ts), "hipMemcpyAsync");
      lqro::check_hip(hipStreamSynchronize(ts), "hipStreamSynchronize");
      return v;
    };
    sh.findMatrices();
    for (int k = 0; k < warmup; ++k) seed = sh.iterate(seed);
    lqro::check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
    allmax(0.0);   // barrier
    lqro::check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < steps; ++k) seed = sh.iterate(seed);   // (each iteration ends synchronised)
    lqro::check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
    allmax(0.0);   // barrier
    lqro::check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double elmax = allmax(el);
    int64_t st[11] = {0};
    if (sh.context()) lqro::check(lqro_get_stats_ex(sh.context(), st, 11), "lqro_get_stats_ex");
    const double inside = allmax((double)st[2]);   // (the last iteration's, max over ranks)
    const double fails = allmax((double)st[4]);
    if (rank == 0)
      std::printf("lqro_bench_main N=%d H=%d NP=%d world=%d steps=%d warmup=%d elapsed_s=%.9f ms_per_step=%.6f "
                  "max_rank_inside=%.0f max_rank_hull_fail=%.0f\n",
                  N, H, NP, world, steps, warmup, elmax, 1e3 * elmax / std::max(1, steps), inside, fails);
    std::fflush(stdout);
    ncclCommDestroy(tc);
    (void)hipFree(d_t);
    (void)hipStreamDestroy(ts);
  } catch (const lqro::Error& e) {
    std::fprintf(stderr, "lqro_bench_main: rank %d: %s\n", rank, e.what());
    return 1;
  }
  return 0;
}
