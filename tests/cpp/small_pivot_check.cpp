// The register-held pivoted routines of lqro_synth.hpp (solve_sm,
// inverse_sm, used for N <= 4) against the indexed ones (solve_ix,
// inverse_ix, the reference's operator% / operator! transcribed with pivot
// permutations), on the host: random matrices, integer matrices with many
// equal magnitudes (pivot ties) and singular ones.  Every result must be
// bit-identical.  Prints "ok <cases>" or the first mismatch.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../lqr-obstacles_amd/csrc/lqro_synth.hpp"

using namespace lqro::synth;

template <int R, int C>
static bool same(const Mat<R, C>& a, const Mat<R, C>& b) {
  return std::memcmp(a.e, b.e, sizeof a.e) == 0;
}

template <int N>
static int run(std::mt19937_64& g, int reps) {
  std::uniform_real_distribution<double> u(-2.0, 2.0);
  std::uniform_int_distribution<int> ui(-3, 3);
  for (int t = 0; t < reps; ++t) {
    Mat<N, N> p;
    Mat<N, 3> q;
    const int kind = t % 3;
    for (int i = 0; i < N * N; ++i) p.e[i] = kind == 0 ? u(g) : (double)ui(g);
    if (kind == 2) for (int j = 0; j < N; ++j) p(N - 1, j) = p(0, j);   // singular
    for (int i = 0; i < N * 3; ++i) q.e[i] = u(g);
    if (!same(solve_sm<N, 3>(p, q), solve_ix<N, 3>(p, q))) { std::printf("solve N=%d case %d\n", N, t); return 1; }
    if (!same(solve_sm<N, N>(p, p), solve_ix<N, N>(p, p))) { std::printf("solveNN N=%d case %d\n", N, t); return 1; }
    if (!same(inverse_sm<N>(p), inverse_ix<N>(p))) { std::printf("inverse N=%d case %d\n", N, t); return 1; }
    if (!same(expm<N>(p * 0.1), [&] {   // exp through the indexed solve
          Mat<N, N> A = p * 0.1;
          const double b0 = 1729728e1, b1 = 864864e1, b2 = 199584e1, b3 = 2772e2, b4 = 252e2, b5 = 1512e0,
                       b6 = 56e0, b7 = 1e0, lim = 9.504178996162932e-1;
          double c = ceil(log(norm1(A) / lim) * M_LOG2E);
          int s = (int)(0.0 < c ? c : 0.0);
          double p2 = pow(2.0, s);
          for (int i = 0; i < N * N; ++i) A.e[i] /= p2;
          Mat<N, N> A2 = A * A, A4 = A2 * A2, A6 = A2 * A4, I = eye<N>();
          Mat<N, N> U = A * (A6 * b7 + A4 * b5 + A2 * b3 + I * b1);
          Mat<N, N> V = A6 * b6 + A4 * b4 + A2 * b2 + I * b0;
          Mat<N, N> Rr = solve_ix(V - U, V + U);
          for (int i = 0; i < s; ++i) Rr = Rr * Rr;
          return Rr;
        }())) { std::printf("expm N=%d case %d\n", N, t); return 1; }
  }
  return 0;
}

int main() {
  std::mt19937_64 g(0x4C51524F);
  const int reps = 20000;
  if (run<2>(g, reps) || run<3>(g, reps) || run<4>(g, reps)) return 1;
  std::printf("ok %d\n", 3 * reps);
  return 0;
}
