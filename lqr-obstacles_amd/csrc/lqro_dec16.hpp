// lqro_dec16.hpp — a plane coefficient as convexHull reads it back.
//
// qconvex prints each facet's hyperplane with 16 significant digits (Qhull's
// "%6.16g " for option 'n'; tests/golden/qhull/Planes.txt) and convexHull
// reads them with operator>> (LQRObstacles.cpp:889-899), so the normal the
// reference measures with (LQRO:955-967) and hands to createHalfPlanes is
// strtod(sprintf("%.16g", n_k)) — not Qhull's double.  Sixteen digits do not
// round-trip a double (17 do), so the two differ in the last bits for about
// half the coefficients.
//
// dec16() computes that round trip exactly, in integers: the 16-digit decimal
// D * 10^-K nearest to |v| (ties to even, printf's rounding), then the double
// nearest to D * 10^-K (ties to even, strtod's).  Plane normals are unit
// vectors: |v| <= 1, so K >= 15; big integers of DEC16_W 64-bit words carry
// the products for |v| >= 1e-115 (K <= DEC16_KMAX).  Outside that range (and
// for subnormals) v is returned unchanged with *exact = false (never seen: a
// component below 1e-115 of a unit normal).  Per-lane, loop-only code: it
// runs for the few facets whose distance is within rounding of the minimum.
#pragma once
#include <math.h>

#ifndef __HIPCC__
#define __host__
#define __device__
#endif

namespace lqro {

__host__ __device__ inline unsigned long long dec16_bits(double v) { return __builtin_bit_cast(unsigned long long, v); }
__host__ __device__ inline double dec16_double(unsigned long long b) { return __builtin_bit_cast(double, b); }

#define DEC16_W 8
#define DEC16_KMAX 130

struct Dec16Big {
  unsigned long long w[DEC16_W];   // little-endian 64-bit words
};

__host__ __device__ inline unsigned long long dec16_mulhi(unsigned long long a, unsigned long long b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (unsigned long long)(((unsigned __int128)a * b) >> 64);
#endif
}

__host__ __device__ inline void dec16_set(Dec16Big& b, unsigned long long v) {
#pragma unroll
  for (int k = 0; k < DEC16_W; ++k) b.w[k] = 0;
  b.w[0] = v;
}

// b *= m
__host__ __device__ inline void dec16_mul(Dec16Big& b, unsigned long long m) {
  unsigned long long carry = 0;
#pragma unroll
  for (int k = 0; k < DEC16_W; ++k) {
    const unsigned long long lo = b.w[k] * m, hi = dec16_mulhi(b.w[k], m);
    const unsigned long long s = lo + carry;
    carry = hi + (s < lo ? 1ull : 0ull);
    b.w[k] = s;
  }
}

// b <<= s (s < 64 * DEC16_W): whole words first (constant indices), then bits
__host__ __device__ inline void dec16_shl(Dec16Big& b, int s) {
  for (; s >= 64; s -= 64) {
#pragma unroll
    for (int k = DEC16_W - 1; k > 0; --k) b.w[k] = b.w[k - 1];
    b.w[0] = 0;
  }
  if (s > 0) {
#pragma unroll
    for (int k = DEC16_W - 1; k > 0; --k) b.w[k] = (b.w[k] << s) | (b.w[k - 1] >> (64 - s));
    b.w[0] <<= s;
  }
}

// b >>= s; *half: bit s-1 of b before the shift; *sticky: any bit below it
__host__ __device__ inline void dec16_shr(Dec16Big& b, int s, bool* half, bool* sticky) {
  bool h = false, st = false;
  for (; s > 64; s -= 64) {        // (keep one last partial step of 1..64 bits)
    st = st || h || b.w[0] != 0;
    h = false;
#pragma unroll
    for (int k = 0; k < DEC16_W - 1; ++k) b.w[k] = b.w[k + 1];
    b.w[DEC16_W - 1] = 0;
  }
  if (s > 0) {
    const unsigned long long low = s == 64 ? b.w[0] : (b.w[0] & ((1ull << s) - 1));
    const unsigned long long hb = 1ull << (s - 1);
    h = (low & hb) != 0;
    st = st || (low & (hb - 1)) != 0;
    if (s == 64) {
#pragma unroll
      for (int k = 0; k < DEC16_W - 1; ++k) b.w[k] = b.w[k + 1];
      b.w[DEC16_W - 1] = 0;
    } else {
#pragma unroll
      for (int k = 0; k < DEC16_W - 1; ++k) b.w[k] = (b.w[k] >> s) | (b.w[k + 1] << (64 - s));
      b.w[DEC16_W - 1] >>= s;
    }
  }
  *half = h;
  *sticky = st;
}

// -1, 0, 1 as a <, ==, > b
__host__ __device__ inline int dec16_cmp(const Dec16Big& a, const Dec16Big& b) {
  int r = 0;
#pragma unroll
  for (int k = DEC16_W - 1; k >= 0; --k)
    if (r == 0 && a.w[k] != b.w[k]) r = a.w[k] < b.w[k] ? -1 : 1;
  return r;
}

// 10^K
__host__ __device__ inline void dec16_pow10(Dec16Big& b, int K) {
  dec16_set(b, 1);
  for (; K >= 19; K -= 19) dec16_mul(b, 10000000000000000000ull);
  unsigned long long m = 1;
  for (; K > 0; --K) m *= 10;
  dec16_mul(b, m);
}

// the sign of V - num * 2^e, V = D * 10^-K (e < 0): of D * 2^-e - num * 10^K
__host__ __device__ inline int dec16_cmpv(unsigned long long D, const Dec16Big& p10K, unsigned long long num, int e) {
  Dec16Big l, r = p10K;
  dec16_set(l, D);
  dec16_shl(l, -e);
  dec16_mul(r, num);
  return dec16_cmp(l, r);
}

__host__ __device__ inline double dec16(double v, bool* exact) {
  *exact = true;
  const unsigned long long bits = dec16_bits(v);
  const unsigned long long sign = bits & 0x8000000000000000ull;
  const int expo = (int)((bits >> 52) & 0x7ff);
  if (expo == 0 || expo == 0x7ff) {   // zero (exact), subnormal, inf, nan
    *exact = expo == 0 && (bits << 1) == 0;
    return v;
  }
  unsigned long long M = (bits & 0xFFFFFFFFFFFFFull) | 0x10000000000000ull;
  int E = expo - 1075;                // |v| = M 2^E
  const double a = dec16_double(bits & ~0x8000000000000000ull);
  int K = 15 - (int)floor(log10(a));  // 10^15 <= |v| 10^K < 10^16, corrected below
  if (K < 15 || K > DEC16_KMAX) { *exact = false; return v; }
  Dec16Big P;
  unsigned long long D = 0;
  bool half = false, sticky = false;
  for (int tries = 0; tries < 3; ++tries) {
    dec16_pow10(P, K);
    dec16_mul(P, M);
    dec16_shr(P, -E, &half, &sticky);          // floor(|v| 10^K), the discarded bits
    bool big = false;
#pragma unroll
    for (int k = 1; k < DEC16_W; ++k) big = big || P.w[k] != 0;
    D = P.w[0];
    if (!big && D >= 1000000000000000ull && D < 10000000000000000ull) break;
    K += (!big && D < 1000000000000000ull) ? 1 : -1;
    if (tries == 2 || K < 15 || K > DEC16_KMAX) { *exact = false; return v; }
  }
  if (half && (sticky || (D & 1))) ++D;        // printf: nearest, ties to even
  if (D == 10000000000000000ull) { D = 1000000000000000ull; --K; }
  if (K < 15) { *exact = false; return v; }
  // strtod: the double nearest to V = D 10^-K, searched from |v| (within ~5 ulps)
  Dec16Big p10K;
  dec16_pow10(p10K, K);
  for (int it = 0; it < 16; ++it) {            // up: V beyond the midpoint to the next double
    const int c = dec16_cmpv(D, p10K, 2 * M + 1, E - 1);
    if (c < 0 || (c == 0 && !(M & 1))) break;
    if (++M == 0x20000000000000ull) { M = 0x10000000000000ull; ++E; }
  }
  for (int it = 0; it < 16; ++it) {            // down: V below the midpoint to the previous one
    // (the previous double is (M-1) 2^E, or (2^53-1) 2^(E-1) at the binade's bottom)
    const int c = dec16_cmpv(D, p10K, M == 0x10000000000000ull ? 4 * M - 1 : 4 * M - 2, E - 2);
    if (c > 0 || (c == 0 && !(M & 1))) break;
    if (--M < 0x10000000000000ull) { M = 0x1FFFFFFFFFFFFFull; --E; }
  }
  const unsigned long long ob = sign | ((unsigned long long)(E + 1075) << 52) | (M & 0xFFFFFFFFFFFFFull);
  return dec16_double(ob);
}

}  // namespace lqro
