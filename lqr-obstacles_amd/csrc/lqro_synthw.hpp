// lqro_synthw.hpp — controlMatrices (LQRObstacles.cpp:520-582, with
// linearizeDiscretize :456-471) with one WAVE per agent, for the batched
// heterogeneous synthesis (lqro_synthesize_gains_batch_x).
//
// The agent's matrices live in a per-wave LDS block; every matrix product,
// sum and scaling is spread over the 64 lanes, one output element per lane
// and pass, computed in the reference's operation order (dot products from
// 0.0 in k order, element-wise chains left to right, exactly the expression
// trees of synth::gains_x).  The small inverses (4x4, 3x3, full-pivot
// Gauss-Jordan) run redundantly in every lane on synth::inverse; the Padé
// exponentials' full-pivot solves run over the lanes with the reference's
// pivot rule (first strict maximum in scan order).  So the wave kernel is
// bit-identical to the one-lane synth::gains_x (tests/test_gpu_synth.py).
//
// X = 16 (the reference's quadrotor) or 12 (config 5's reduced model).
#pragma once
#include "lqro_device.hpp"
#include "lqro_synth.hpp"

namespace lqro {
namespace synthw {

using synth::Mat;
using synth::Quad;

__device__ __forceinline__ void sync() { wave_lds_sync(); }

// C (R x Cc) = A (R x K) * B (K x Cc); C distinct from A, B.  Each element
// is one dot product from 0.0 in k order; large products give each lane a
// 2 x 2 block (every loaded A and B value feeds two products).
template <int R, int K, int Cc>
__device__ __forceinline__ void mm(const double* A, const double* B, double* C, int lane) {
  if constexpr (R % 2 == 0 && Cc % 2 == 0 && R * Cc >= 128) {
    constexpr int BC = Cc / 2;
    for (int e = lane; e < (R / 2) * BC; e += 64) {
      const int i = 2 * (e / BC), j = 2 * (e - (e / BC) * BC);
      double c00 = 0.0, c01 = 0.0, c10 = 0.0, c11 = 0.0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const double a0 = A[i * K + k], a1 = A[(i + 1) * K + k];
        const double b0 = B[k * Cc + j], b1 = B[k * Cc + j + 1];
        c00 += a0 * b0; c01 += a0 * b1; c10 += a1 * b0; c11 += a1 * b1;
      }
      C[i * Cc + j] = c00; C[i * Cc + j + 1] = c01; C[(i + 1) * Cc + j] = c10; C[(i + 1) * Cc + j + 1] = c11;
    }
  } else {
    for (int e = lane; e < R * Cc; e += 64) {
      const int i = e / Cc, j = e - i * Cc;
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < K; ++k) acc += A[i * K + k] * B[k * Cc + j];
      C[e] = acc;
    }
  }
  sync();
}
// D (C x R) = A^T (A is R x C)
template <int R, int C>
__device__ __forceinline__ void tr(const double* A, double* D, int lane) {
  for (int e = lane; e < R * C; e += 64) {
    const int i = e / R, j = e - i * R;   // D(i, j) = A(j, i)
    D[e] = A[j * C + i];
  }
  sync();
}
// first strict maximum of |m| in (row, col) scan order over the trailing
// (N-k)^2 block of the permuted matrix (synth::solve's pivot)
template <int N>
__device__ __forceinline__ void pivot(const double* m, const int* rp, const int* cp, int k, int lane, int& br,
                                      int& bc) {
  const int w = N - k;
  double best = 0.0;
  int bi = INT_MAX;
  for (int idx = lane; idx < w * w; idx += 64) {
    const int i = k + idx / w, j = k + idx % w;
    const double a = fabs(m[rp[i] * N + cp[j]]);
    if (a > best) { best = a; bi = idx; }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ob = __shfl_xor(best, off);
    const int oi = __shfl_xor(bi, off);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (bi == INT_MAX) { br = k; bc = k; }
  else { br = k + bi / w; bc = k + bi % w; }
}

// X = P^-1 Q (N x N each) by full pivoting with the reference's final
// reshuffle (synth::solve); m (P) and x (Q) in LDS, overwritten; result in x
template <int N>
__device__ void solve(double* m, double* x, int* ip, int lane) {
  int* rp = ip;
  int* cp = ip + 16;
  int* irp = ip + 32;
  if (lane < N) { rp[lane] = lane; cp[lane] = lane; }
  sync();
  for (int k = 0; k < N; ++k) {
    int br, bc;
    pivot<N>(m, rp, cp, k, lane, br, bc);
    const int rk = rp[br], ck = cp[bc], rb = rp[k], cb = cp[k];
    sync();
    if (lane == 0) { rp[k] = rk; rp[br] = rb; cp[k] = ck; cp[bc] = cb; }
    sync();
    const int w = N - 1 - k;
    const double piv = m[rp[k] * N + cp[k]];
    for (int idx = lane; idx < w * (w + N); idx += 64) {
      const int i = k + 1 + idx / (w + N), c = idx % (w + N);
      const double f = m[rp[i] * N + cp[k]] / piv;
      if (c < w) {
        const int j = k + 1 + c;
        m[rp[i] * N + cp[j]] -= f * m[rp[k] * N + cp[j]];
      } else {
        const int j = c - w;
        x[rp[i] * N + j] -= f * x[rp[k] * N + j];
      }
    }
    sync();
  }
  for (int k = N - 1; k >= 0; --k) {
    const double qk = m[rp[k] * N + cp[k]];
    if (lane < N) x[rp[k] * N + lane] /= qk;
    sync();
    for (int idx = lane; idx < k * N; idx += 64) {
      const int i = idx / N, j = idx % N;
      const double f = m[rp[i] * N + cp[k]];
      x[rp[i] * N + j] -= f * x[rp[k] * N + j];
    }
    sync();
  }
  if (lane < N) irp[rp[lane]] = lane;
  sync();
  for (int i = 0; i < N; ++i) {
    const int ci = cp[i], ri = rp[i];
    if (lane < N) {
      const double t = x[ci * N + lane];
      x[ci * N + lane] = x[ri * N + lane];
      x[ri * N + lane] = t;
    }
    sync();
    if (lane == 0) {
      const int a = irp[ci];
      rp[a] = ri;
      irp[ri] = a;
    }
    sync();
  }
}

// D = !M (N x N, N <= 4) as solve(M, I): the same operations on the same
// values as synth::inverse's in-place Gauss-Jordan (the identity's columns
// beyond the pivot step are still zero when it skips them), over the lanes
// instead of redundantly in every lane (whose dynamic pivot indexing spills
// to scratch).  wm, wx: 16 doubles each; D may alias M.
template <int N>
__device__ __forceinline__ void inv_small(const double* M, double* D, double* wm, double* wx, int* ip, int lane) {
  if (lane < N * N) {
    wm[lane] = M[lane];
    wx[lane] = (lane / N == lane % N) ? 1.0 : 0.0;
  }
  sync();
  solve<N>(wm, wx, ip, lane);
  if (lane < N * N) D[lane] = wx[lane];
  sync();
}

// out = exp(q) (N x N, Padé 7 with scaling and squaring, = synth::expm);
// w: 6 N x N work matrices, ip: 48 ints
template <int N>
__device__ void expm(const double* q, double* out, double* w, int* ip, int lane) {
  constexpr int NN = N * N;
  const double b0 = 1729728e1, b1 = 864864e1, b2 = 199584e1, b3 = 2772e2, b4 = 252e2, b5 = 1512e0,
               b6 = 56e0, b7 = 1e0, lim = 9.504178996162932e-1;
  double* A = w;
  double* A2 = w + NN;
  double* A4 = w + 2 * NN;
  double* A6 = w + 3 * NN;
  double* U = w + 4 * NN;
  double* V = w + 5 * NN;
  double cs = 0.0;   // 1-norm: column sums in i order, then their maximum (order-free)
  if (lane < N)
    for (int i = 0; i < N; ++i) cs += fabs(q[i * N + lane]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) cs = fmax(cs, __shfl_xor(cs, off));
  const double c = ceil(log(cs / lim) * M_LOG2E);
  const int s = (int)(0.0 < c ? c : 0.0);
  const double p2 = pow(2.0, s);
  for (int e = lane; e < NN; e += 64) A[e] = q[e] / p2;
  sync();
  mm<N, N, N>(A, A, A2, lane);
  mm<N, N, N>(A2, A2, A4, lane);
  mm<N, N, N>(A2, A4, A6, lane);
  for (int e = lane; e < NN; e += 64) {
    const double I = (e / N == e % N) ? 1.0 : 0.0;
    V[e] = A6[e] * b6 + A4[e] * b4 + A2[e] * b2 + I * b0;
    U[e] = A6[e] * b7 + A4[e] * b5 + A2[e] * b3 + I * b1;
  }
  sync();
  mm<N, N, N>(A, U, A2, lane);   // U = A (..)
  for (int e = lane; e < NN; e += 64) {
    A4[e] = V[e] - A2[e];   // V - U
    A6[e] = V[e] + A2[e];   // V + U
  }
  sync();
  solve<N>(A4, A6, ip, lane);
  double* cur = A6;
  double* nxt = U;
  for (int i = 0; i < s; ++i) {
    mm<N, N, N>(cur, cur, nxt, lane);
    double* t = cur; cur = nxt; nxt = t;
  }
  for (int e = lane; e < NN; e += 64) out[e] = cur[e];
  sync();
}

// per-wave LDS block (doubles), X <= 16: A, B, L, E (and the solve's pivot
// ints) live throughout; the linearisation's, the velocity LQR's and the
// position LQR's work matrices overlay one region, each phase's set laid out
// on its own (a phase starts after the previous one's last sync)
template <int X>
struct Lay {
  static constexpr int XX = X * X, X3 = X * 3, X4 = X * 4;
  enum : int {
    A = 0, B = A + XX, L = B + X4, E = L + X4, Cp = E + 12, Ip = Cp + X, Wm = Ip + 24, Wx = Wm + 16,
    V0 = Wx + 16,
    // linearisation
    Fr = V0, F = Fr + (2 * X + 9) * X, G = F + XX, Int = G + X4, Cv = Int + XX, E2 = Cv + X, Ex = E2 + XX,
    LinEnd = Ex + 6 * XX,
    // velocity LQR
    At = V0, Bt = At + XX, S = Bt + X4, T = S + XX, AtS = T + X3, AtSB = AtS + XX, BtS = AtSB + X4,
    BtSB = BtS + X4, Ri = BtSB + 16, K = Ri + 16, AtT = K + X4, KBt = AtT + X3, KBtT = KBt + XX,
    AtSA = KBtT + X3, BtSA = AtSA + XX, KBtSA = BtSA + X4, C1 = KBtSA + XX, C2 = C1 + X3, VelEnd = C2 + XX,
    // position LQR
    Qpt = V0, Acl = Qpt + XX, Aclt = Acl + XX, St = Aclt + XX, AS = St + XX, K2Bt = AS + XX, ASA = K2Bt + XX,
    Stn = ASA + XX, TXX = Stn + XX, Bcl = TXX + XX, Tt = Bcl + X3, CPs = Tt + X3, Ptt = CPs + X3,
    K1 = Ptt + X3, K2 = K1 + X3, C3 = K2 + X3, AT = C3 + X3, Ttn = AT + X3, Bclt = Ttn + X3, Pt = Bclt + X3,
    BS = Pt + X3, BSA = BS + X3, PB = BSA + X3, WLt = PB + X3, WLtR = WLt + X4, Rt = WLtR + X4, RR = Rt + 9,
    BSB = RR + 9, WEtR = BSB + 18, PosEnd = WEtR + 12,
    Total = (LinEnd > VelEnd ? (LinEnd > PosEnd ? LinEnd : PosEnd) : (VelEnd > PosEnd ? VelEnd : PosEnd))
  };
};
constexpr int kSynthWaveDoubles = Lay<16>::Total;

// controlMatrices for agent model md, outputs as synth::gains_x (any null)
template <int X>
__device__ void gains(const lqro_model* md, double* Ao, double* Bo, double* co, double* Lo, double* Eo,
                      double* Lho, double* Eho, double* lo, double* w, int lane) {
  using Y = Lay<X>;
  constexpr int XX = X * X;
  Quad q;
  q.dt = md->dt; q.g = md->gravity; q.mass = md->mass; q.kM = md->moment_const;
  q.lat = md->thrust_latency; q.arm = md->length; q.h = md->j_step;
  q.J = md->inertia * synth::eye<3>();
  q.Jinv = synth::inverse(q.J);
  const double hover = q.g * q.mass / 4;
  int* ip = reinterpret_cast<int*>(w + Y::Ip);

  // linearizeDiscretize (LQRO:456-471): lanes 0..X-1 f(x0 + h e_i), X..2X-1
  // f(x0 - h e_i), 2X f(x0), 2X+1..2X+4 f(u0 + h e_i), 2X+5..2X+8 f(u0 - h e_i)
  {
    Mat<X, 1> x0 = Mat<X, 1>::zero();
    for (int k = 12; k < X; ++k) x0.e[k] = hover;
    Mat<4, 1> u0;
    for (int k = 0; k < 4; ++k) u0.e[k] = hover;
    if (lane <= 2 * X + 8) {
      Mat<X, 1> xp = x0;
      Mat<4, 1> up = u0;
      if (lane < 2 * X) {
        const int i = lane % X;
        xp.e[i] = lane < X ? x0.e[i] + q.h : x0.e[i] - q.h;
      } else if (lane > 2 * X) {
        const int m = lane - 2 * X - 1, i = m & 3;
        up.e[i] = m < 4 ? u0.e[i] + q.h : u0.e[i] - q.h;
      }
      const Mat<X, 1> f = synth::dynamics<X>(q, xp, synth::eye<3>(), up);
      for (int k = 0; k < X; ++k) w[Y::Fr + lane * X + k] = f.e[k];
    }
    sync();
    for (int e = lane; e < XX; e += 64) {
      const int k = e / X, i = e % X;   // F(k, i)
      w[Y::F + e] = (w[Y::Fr + i * X + k] - w[Y::Fr + (X + i) * X + k]) / (2 * q.h);
    }
    for (int e = lane; e < X * 4; e += 64) {
      const int k = e / 4, i = e % 4;   // G(k, i)
      w[Y::G + e] = (w[Y::Fr + (2 * X + 1 + i) * X + k] - w[Y::Fr + (2 * X + 5 + i) * X + k]) / (2 * q.h);
    }
    sync();
    double* tmp = w + Y::Int;   // dt F, then (dt/2) F
    for (int e = lane; e < XX; e += 64) tmp[e] = q.dt * w[Y::F + e];
    sync();
    expm<X>(tmp, w + Y::A, w + Y::Ex, ip, lane);
    for (int e = lane; e < XX; e += 64) tmp[e] = 0.5 * q.dt * w[Y::F + e];
    sync();
    double* E2 = w + Y::E2;   // exp((dt/2) F)
    expm<X>(tmp, E2, w + Y::Ex, ip, lane);
    // Int = (dt/6) (I + 4 exp(dt F / 2) + A)
    for (int e = lane; e < XX; e += 64) {
      const double I = (e / X == e % X) ? 1.0 : 0.0;
      w[Y::Int + e] = (q.dt / 6.0) * ((I + 4.0 * E2[e]) + w[Y::A + e]);
    }
    sync();
    mm<X, X, 4>(w + Y::Int, w + Y::G, w + Y::B, lane);                 // B = Int G
    mm<X, X, 1>(w + Y::Int, w + Y::Fr + 2 * X * X, w + Y::Cv, lane);  // c = Int xdot
    for (int e = lane; e < X; e += 64) {
      w[Y::Cp + e] = w[Y::Cv + e];   // kept for l
      if (co) co[e] = w[Y::Cv + e];
    }
  }

  // velocity LQR (LQRO:541-557): Vs selects x[3..5]; Qx = 0
  const double qv = md->qv, r = md->r;
  tr<X, X>(w + Y::A, w + Y::At, lane);
  tr<X, 4>(w + Y::B, w + Y::Bt, lane);
  // C1 = (-Vt) Qv, C2 = ((Vt Qv) Vs) + Qx: entries of the selection products,
  // each a 3-term dot from 0.0 in k order (Vt has one 1 per column)
  for (int e = lane; e < X * 3; e += 64) {
    const int i = e / 3, j = e % 3;
    double a = 0.0;
    for (int k = 0; k < 3; ++k) {
      const double vt = (i == 3 + k) ? 1.0 : 0.0;
      const double qk = (k == j) ? qv : 0.0;
      a += (-vt) * qk;
    }
    w[Y::C1 + e] = a;
  }
  for (int e = lane; e < XX; e += 64) {
    const int i = e / X, j = e % X;
    double acc = 0.0;   // ((Vt Qv) Vs)(i, j) = sum_k (Vt Qv)(i, k) Vs(k, j)
    for (int k = 0; k < 3; ++k) {
      double vq = 0.0;
      for (int m = 0; m < 3; ++m) vq += ((i == 3 + m) ? 1.0 : 0.0) * ((m == k) ? qv : 0.0);
      acc += vq * ((j == 3 + k) ? 1.0 : 0.0);
    }
    w[Y::C2 + e] = acc + 0.0;   // + Qx
    w[Y::S + e] = acc;          // S = Vt Qv Vs
  }
  for (int e = lane; e < X * 3; e += 64) w[Y::T + e] = w[Y::C1 + e];   // T = -Vt Qv
  sync();
  for (int it = 0; it < 300; ++it) {
    mm<X, X, X>(w + Y::At, w + Y::S, w + Y::AtS, lane);
    mm<X, X, 4>(w + Y::AtS, w + Y::B, w + Y::AtSB, lane);
    mm<4, X, X>(w + Y::Bt, w + Y::S, w + Y::BtS, lane);
    mm<4, X, 4>(w + Y::BtS, w + Y::B, w + Y::BtSB, lane);
    for (int e = lane; e < 16; e += 64) w[Y::BtSB + e] = ((e >> 2) == (e & 3) ? r : 0.0) + w[Y::BtSB + e];
    sync();
    inv_small<4>(w + Y::BtSB, w + Y::Ri, w + Y::Wm, w + Y::Wx, ip, lane);
    mm<X, 4, 4>(w + Y::AtSB, w + Y::Ri, w + Y::K, lane);          // K = At S B !(R + Bt S B)
    mm<X, X, 3>(w + Y::At, w + Y::T, w + Y::AtT, lane);
    mm<X, 4, X>(w + Y::K, w + Y::Bt, w + Y::KBt, lane);
    mm<X, X, 3>(w + Y::KBt, w + Y::T, w + Y::KBtT, lane);
    mm<X, X, X>(w + Y::AtS, w + Y::A, w + Y::AtSA, lane);
    mm<4, X, X>(w + Y::BtS, w + Y::A, w + Y::BtSA, lane);
    mm<X, 4, X>(w + Y::K, w + Y::BtSA, w + Y::KBtSA, lane);
    for (int e = lane; e < X * 3; e += 64)
      w[Y::T + e] = (w[Y::C1 + e] + w[Y::AtT + e]) - w[Y::KBtT + e];
    for (int e = lane; e < XX; e += 64)
      w[Y::S + e] = (w[Y::C2 + e] + w[Y::AtSA + e]) - w[Y::KBtSA + e];
    sync();
  }
  // Ri = !(R + Bt S B); L = ((-Ri) Bt) S A; E = ((-Ri) Bt) T
  mm<4, X, X>(w + Y::Bt, w + Y::S, w + Y::BtS, lane);
  mm<4, X, 4>(w + Y::BtS, w + Y::B, w + Y::BtSB, lane);
  for (int e = lane; e < 16; e += 64) w[Y::BtSB + e] = ((e >> 2) == (e & 3) ? r : 0.0) + w[Y::BtSB + e];
  sync();
  inv_small<4>(w + Y::BtSB, w + Y::Ri, w + Y::Wm, w + Y::Wx, ip, lane);
  for (int e = lane; e < 16; e += 64) w[Y::Ri + e] = -w[Y::Ri + e];
  sync();
  mm<4, 4, X>(w + Y::Ri, w + Y::Bt, w + Y::BtS, lane);        // (-Ri) Bt
  mm<4, X, X>(w + Y::BtS, w + Y::S, w + Y::BtSA, lane);       // ((-Ri) Bt) S
  mm<4, X, X>(w + Y::BtSA, w + Y::A, w + Y::L, lane);         // L
  mm<4, X, 3>(w + Y::BtS, w + Y::T, w + Y::E, lane);          // E
  if (lo && lane == 0) {
    // l (LQRO:552, 557): once per agent, one lane, on synth::ell
    Mat<X, X> Am, Sm;
    Mat<X, 4> Bm;
    Mat<X, 1> cm, xs = Mat<X, 1>::zero();
    for (int e = 0; e < XX; ++e) { Am.e[e] = w[Y::A + e]; Sm.e[e] = w[Y::S + e]; }
    for (int e = 0; e < X * 4; ++e) Bm.e[e] = w[Y::B + e];
    for (int e = 0; e < X; ++e) cm.e[e] = w[Y::Cp + e];
    for (int k = 12; k < X; ++k) xs.e[k] = hover;
    const Mat<4, 1> lv = synth::ell<X>(Am, Bm, cm, Sm, r * synth::eye<4>(), xs);
    for (int k = 0; k < 4; ++k) lo[k] = lv.e[k];
  }
  sync();

  // position LQR with the cross term (LQRO:559-581); the velocity phase's
  // buffers are reused (A, B, L, E stay)
  const double wgt = md->pos_weight, qp = md->qp;
  double* Qpt = w + Y::Qpt;
  double* Acl = w + Y::Acl;
  double* Aclt = w + Y::Aclt;
  double* St = w + Y::St;
  double* AS = w + Y::AS;
  double* K2Bt = w + Y::K2Bt;
  double* ASA = w + Y::ASA;
  double* Stn = w + Y::Stn;
  double* tXX = w + Y::TXX;
  double* Bcl = w + Y::Bcl;
  double* Tt = w + Y::Tt;
  double* cPs = w + Y::CPs;
  double* Ptt = w + Y::Ptt;
  double* K1 = w + Y::K1;
  double* K2 = w + Y::K2;
  double* c3 = w + Y::C3;
  double* AT = w + Y::AT;
  double* Ttn = w + Y::Ttn;
  double* Bclt = w + Y::Bclt;
  double* Pt = w + Y::Pt;
  double* BS = w + Y::BS;
  double* BSA = w + Y::BSA;
  double* PB = w + Y::PB;
  double* Rt = w + Y::Rt;
  double* RR = w + Y::RR;
  double* BSB = w + Y::BSB;
  double* wEtR = w + Y::WEtR;
  double* wLt = w + Y::WLt;
  double* wLtR = w + Y::WLtR;
  // Qpt = ((Ps^T Qp) Ps) + (((wgt L^T) Rw) L)
  tr<4, X>(w + Y::L, wLt, lane);
  for (int e = lane; e < X * 4; e += 64) wLt[e] = wgt * wLt[e];
  sync();
  for (int e = lane; e < X * 4; e += 64) {
    const int i = e / 4, j = e % 4;
    double acc = 0.0;
    for (int k = 0; k < 4; ++k) acc += wLt[i * 4 + k] * ((k == j) ? r : 0.0);
    wLtR[e] = acc;
  }
  sync();
  mm<X, 4, X>(wLtR, w + Y::L, tXX, lane);
  for (int e = lane; e < XX; e += 64) {
    const int i = e / X, j = e % X;
    double acc = 0.0;
    for (int k = 0; k < 3; ++k) {
      double pq = 0.0;
      for (int m = 0; m < 3; ++m) pq += ((i == m) ? 1.0 : 0.0) * ((m == k) ? qp : 0.0);
      acc += pq * ((j == k) ? 1.0 : 0.0);
    }
    Qpt[e] = acc + tXX[e];
  }
  // Rt = ((wgt E^T) Rw) E, Pt = ((wgt E^T) Rw) L
  for (int e = lane; e < 12; e += 64) {
    const int i = e / 4, j = e % 4;
    double acc = 0.0;
    for (int k = 0; k < 4; ++k) acc += (wgt * w[Y::E + k * 3 + i]) * ((k == j) ? r : 0.0);
    wEtR[e] = acc;
  }
  sync();
  mm<3, 4, 3>(wEtR, w + Y::E, Rt, lane);
  mm<3, 4, X>(wEtR, w + Y::L, Pt, lane);
  mm<X, 4, X>(w + Y::B, w + Y::L, tXX, lane);
  for (int e = lane; e < XX; e += 64) Acl[e] = w[Y::A + e] + tXX[e];   // A + B L
  sync();
  mm<X, 4, 3>(w + Y::B, w + Y::E, Bcl, lane);                          // B E
  tr<X, X>(Acl, Aclt, lane);
  tr<X, 3>(Bcl, Bclt, lane);
  tr<3, X>(Pt, Ptt, lane);
  for (int e = lane; e < XX; e += 64) St[e] = Qpt[e];
  for (int e = lane; e < X * 3; e += 64) {   // (-Ps^T) Qp
    const int i = e / 3, j = e % 3;
    double acc = 0.0;
    for (int k = 0; k < 3; ++k) acc += (-((i == k) ? 1.0 : 0.0)) * ((k == j) ? qp : 0.0);
    cPs[e] = acc;
    Tt[e] = acc;
  }
  sync();
  for (int it = 0; it < 300; ++it) {
    mm<X, X, X>(Aclt, St, AS, lane);
    mm<X, X, 3>(AS, Bcl, K1, lane);
    for (int e = lane; e < X * 3; e += 64) K1[e] = Ptt[e] + K1[e];       // Ptt + Aclt St Bcl
    mm<3, X, X>(Bclt, St, BS, lane);
    mm<3, X, 3>(BS, Bcl, BSB, lane);
    for (int e = lane; e < 9; e += 64) RR[e] = Rt[e] + BSB[e];
    sync();
    inv_small<3>(RR, RR, w + Y::Wm, w + Y::Wx, ip, lane);
    mm<X, 3, 3>(K1, RR, K2, lane);                                          // K
    mm<X, 3, X>(K2, Bclt, K2Bt, lane);
    mm<X, X, 3>(K2Bt, Tt, c3, lane);
    mm<X, X, 3>(Aclt, Tt, AT, lane);
    for (int e = lane; e < X * 3; e += 64) Ttn[e] = (cPs[e] + AT[e]) - c3[e];
    mm<3, X, X>(BS, Acl, BSA, lane);
    for (int e = lane; e < 3 * X; e += 64) PB[e] = Pt[e] + BSA[e];
    sync();
    mm<X, 3, X>(K2, PB, tXX, lane);                                         // c4
    mm<X, X, X>(AS, Acl, ASA, lane);
    for (int e = lane; e < XX; e += 64) Stn[e] = (Qpt[e] + ASA[e]) - tXX[e];
    sync();
    for (int e = lane; e < X * 3; e += 64) Tt[e] = Ttn[e];
    for (int e = lane; e < XX; e += 64) St[e] = Stn[e];
    sync();
  }
  // RRi = !(Rt + Bclt St Bcl); Lh = (-RRi)(Pt + Bclt St Acl); Eh = (-RRi)(Bclt Tt)
  mm<3, X, X>(Bclt, St, BS, lane);
  mm<3, X, 3>(BS, Bcl, BSB, lane);
  for (int e = lane; e < 9; e += 64) RR[e] = Rt[e] + BSB[e];
  sync();
  inv_small<3>(RR, RR, w + Y::Wm, w + Y::Wx, ip, lane);
  for (int e = lane; e < 9; e += 64) RR[e] = -RR[e];
  sync();
  mm<3, X, X>(BS, Acl, BSA, lane);
  for (int e = lane; e < 3 * X; e += 64) PB[e] = Pt[e] + BSA[e];
  sync();
  mm<3, 3, X>(RR, PB, BSA, lane);           // Lh
  mm<3, X, 3>(Bclt, Tt, BSB, lane);
  mm<3, 3, 3>(RR, BSB, BSB + 9, lane);      // Eh

  if (Ao) for (int e = lane; e < XX; e += 64) Ao[e] = w[Y::A + e];
  if (Bo) for (int e = lane; e < X * 4; e += 64) Bo[e] = w[Y::B + e];
  if (Lo) for (int e = lane; e < 4 * X; e += 64) Lo[e] = w[Y::L + e];
  if (Eo) for (int e = lane; e < 12; e += 64) Eo[e] = w[Y::E + e];
  if (Lho) for (int e = lane; e < 3 * X; e += 64) Lho[e] = BSA[e];
  if (Eho) for (int e = lane; e < 9; e += 64) Eho[e] = BSB[9 + e];
}

}  // namespace synthw
}  // namespace lqro
