// lqro_lp.hpp — the new-velocity linear program (calculateNewV,
// LQRObstacles.cpp:1223-1234, with linearProgram1-4 :1001-1206, RVO2-3D) as
// one wavefront per agent.
//
// The reference runs the LP in fp32 (Vector3 stores float, Vector3.h:340).
// Every per-plane expression here is evaluated exactly as there; only the
// plane loops are spread over the 64 lanes:
//   * "first plane i >= i0 that the current result violates" (the sequential
//     scans of linearProgram2/3/4) = a 64-plane ballot + find-first-set;
//   * linearProgram1's loop is a max/min reduction (exact, order-free) plus an
//     "any parallel plane rejects" test — returning false at the first
//     failing plane or after the loop gives the same answer because tLeft
//     only grows and tRight only shrinks.
// So the result is bit-identical to the sequential fp32 LP.
//
// The LP is one long dependent chain (C3's hardest rows: ~1,500 violated
// planes and linearProgram1 calls in sequence, almost all over fewer than
// 64 planes), so the code is written for latency, not throughput:
//   * each scan keeps its current 64-plane chunk in registers (one plane a
//     lane, the next chunk's loads already issued); a violated plane is
//     broadcast with readlane, and linearProgram1 over planes of that chunk
//     reads the same registers — no LDS round trip per violation;
//   * linearProgram2's line for plane i (direction, point: they depend on
//     planes i and planeNo only, not on the current result) is computed for
//     the whole chunk at its first violation, once per chunk, and each
//     later violation in the chunk reads its lane's line;
//   * linearProgram1's max/min reductions are DPP lane moves and four
//     readlanes (uniform result), not ds_bpermute shuffles.
#pragma once
#include <hip/hip_runtime.h>

namespace lqro {

struct v3 { float x, y, z; };
__device__ __forceinline__ v3 V3(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 vmul(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }   // Vector3*float
__device__ __forceinline__ v3 smul(float s, v3 a) { return V3(s * a.x, s * a.y, s * a.z); }   // float*Vector3
__device__ __forceinline__ v3 vcross(v3 a, v3 b) {
  return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ v3 vnormalize(v3 a) {     // vector / abs(vector)
  float l = sqrtf(vdot(a, a));
  const float inv = 1.0f / l;
  return V3(a.x * inv, a.y * inv, a.z * inv);
}
__device__ __forceinline__ float sqrf(float s) { return s * s; }
__device__ __forceinline__ float stdmax(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float stdmin(float a, float b) { return (b < a) ? b : a; }
constexpr float kRvoEps = 0.00001f;

// A plane list holds {point.xyz, normal.xyz} per plane with a stride of PS
// floats: PS = 8 is the 32-B slot k_pair writes ({.., flag, pad}, 16-B
// aligned loads, global memory); PS = 6 packs the LDS copies (24 B a plane,
// so a 4,095-plane row of C4 fits one CU's LDS).
struct LPPlane { v3 point, normal; };
template <int PS>
__device__ __forceinline__ LPPlane ld_plane(const float* base, int i) {
  LPPlane r;
  if constexpr (PS == 8) {
    const float4* p = reinterpret_cast<const float4*>(base + 8 * (size_t)i);
    float4 a = p[0], b = p[1];
    r.point = V3(a.x, a.y, a.z);
    r.normal = V3(a.w, b.x, b.y);
  } else {
    const float2* p = reinterpret_cast<const float2*>(base + 6 * (size_t)i);
    float2 a = p[0], b = p[1], c = p[2];
    r.point = V3(a.x, a.y, b.x);
    r.normal = V3(b.y, c.x, c.y);
  }
  return r;
}
template <int PS>
__device__ __forceinline__ void st_plane(float* base, int i, v3 pt, v3 nm) {
  if constexpr (PS == 8) {
    float4* d = reinterpret_cast<float4*>(base + 8 * (size_t)i);
    d[0] = make_float4(pt.x, pt.y, pt.z, nm.x);
    d[1] = make_float4(nm.y, nm.z, 0.0f, 0.0f);
  } else {
    float2* d = reinterpret_cast<float2*>(base + 6 * (size_t)i);
    d[0] = make_float2(pt.x, pt.y);
    d[1] = make_float2(pt.z, nm.x);
    d[2] = make_float2(nm.y, nm.z);
  }
}

// orcaPlanes_ in push order (j order, LQRObstacles.cpp:1220): a row's plane
// slots (k_pair's 32-B records, [6] = 1 for a plane) compacted into `planes`
// (stride PS); returns their count
template <int PS>
__device__ __forceinline__ int lp_compact(const float* src, int npr, float* planes, int lane) {
  int m = 0;
  for (int base = 0; base < npr; base += 64) {
    const int sidx = base + lane;
    float4 a = make_float4(0, 0, 0, 0), b = make_float4(0, 0, 0, 0);
    bool f = false;
    if (sidx < npr) {
      const float4* p = reinterpret_cast<const float4*>(src + 8 * (size_t)sidx);
      a = p[0];
      b = p[1];
      f = __float_as_int(b.z) == 1;
    }
    const unsigned long long bal = __ballot(f);
    if (f)
      st_plane<PS>(planes, m + __popcll(bal & ((1ull << lane) - 1ull)), V3(a.x, a.y, a.z), V3(a.w, b.x, b.y));
    m += __popcll(bal);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return m;
}

// lane k's value of x (k uniform): the result is wave-uniform
__device__ __forceinline__ float lp_rl(float x, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), k));
}
__device__ __forceinline__ v3 lp_rl3(v3 a, int k) { return V3(lp_rl(a.x, k), lp_rl(a.y, k), lp_rl(a.z, k)); }
template <int CTRL>
__device__ __forceinline__ float lp_dpp(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), CTRL, 0xF, 0xF, false));
}
// max / min over the 64 lanes with stdmax / stdmin (all lanes active): xor 1,
// xor 2 (quad_perm), half-row and row mirrors, then the four rows' values
__device__ __forceinline__ float lp_wave_max(float v) {
  v = stdmax(v, lp_dpp<0xB1>(v));
  v = stdmax(v, lp_dpp<0x4E>(v));
  v = stdmax(v, lp_dpp<0x141>(v));
  v = stdmax(v, lp_dpp<0x140>(v));
  return stdmax(stdmax(lp_rl(v, 0), lp_rl(v, 16)), stdmax(lp_rl(v, 32), lp_rl(v, 48)));
}
__device__ __forceinline__ float lp_wave_min(float v) {
  v = stdmin(v, lp_dpp<0xB1>(v));
  v = stdmin(v, lp_dpp<0x4E>(v));
  v = stdmin(v, lp_dpp<0x141>(v));
  v = stdmin(v, lp_dpp<0x140>(v));
  return stdmin(stdmin(lp_rl(v, 0), lp_rl(v, 16)), stdmin(lp_rl(v, 32), lp_rl(v, 48)));
}
template <int PS>
__device__ __forceinline__ LPPlane ld_plane_if(const float* base, int i, int n) {
  if (i < n) return ld_plane<PS>(base, i);
  LPPlane z;
  z.point = V3(0, 0, 0);
  z.normal = V3(0, 0, 0);
  return z;
}
// normal.(point - r) > thresh: plane violated by r (LQRO:1083, 1138, 1170)
__device__ __forceinline__ bool lp_violates(const LPPlane& p, v3 r, float thresh) {
  return vdot(p.normal, vsub(p.point, r)) > thresh;
}

// linearProgram1 (LQRO:1001-1046) on planes [0, planeNo) and the line (lpt,
// ldir); the planes of chunk cb (64-aligned, planeNo <= cb + 64) are the
// lanes' registers pc
template <int PS>
__device__ __forceinline__ bool w_lp1(const float* planes, int planeNo, int cb, const LPPlane& pc, v3 lpt,
                                      v3 ldir, float radius, v3 opt, bool dirOpt, v3& result, int lane) {
  const float dotProduct = vdot(lpt, ldir);
  const float disc = sqrf(dotProduct) + sqrf(radius) - vdot(lpt, lpt);
  if (disc < 0.0f) return false;
  const float sq = sqrtf(disc);
  float tLeft = -dotProduct - sq;
  float tRight = -dotProduct + sq;
  float lmax = -INFINITY, lmin = INFINITY;
  bool reject = false;
  for (int base = 0; base < planeNo; base += 64) {
    const int i = base + lane;
    const LPPlane pi = base == cb ? pc : ld_plane_if<PS>(planes, i, planeNo);
    if (i < planeNo) {
      const float numerator = vdot(vsub(pi.point, lpt), pi.normal);
      const float denominator = vdot(ldir, pi.normal);
      if (sqrf(denominator) <= kRvoEps) {
        if (numerator > 0.0f) reject = true;
      } else {
        const float t = numerator / denominator;
        if (denominator >= 0.0f) lmax = stdmax(lmax, t);
        else lmin = stdmin(lmin, t);
      }
    }
  }
  if (__ballot(reject)) return false;
  tLeft = stdmax(tLeft, lp_wave_max(lmax));
  tRight = stdmin(tRight, lp_wave_min(lmin));
  if (tLeft > tRight) return false;
  if (dirOpt) {
    if (vdot(opt, ldir) > 0.0f) result = vadd(lpt, smul(tRight, ldir));
    else result = vadd(lpt, smul(tLeft, ldir));
  } else {
    const float t = vdot(ldir, vsub(opt, lpt));
    if (t < tLeft) result = vadd(lpt, smul(tLeft, ldir));
    else if (t > tRight) result = vadd(lpt, smul(tRight, ldir));
    else result = vadd(lpt, smul(t, ldir));
  }
  return true;
}

// linearProgram2 (LQRO:1048-1104) for plane planeNo = pn; the planes of chunk
// ob (64-aligned) are the caller's registers po
template <int PS>
__device__ __forceinline__ bool w_lp2(const float* planes, int planeNo, const LPPlane& pn, int ob,
                                      const LPPlane& po, float radius, v3 opt, bool dirOpt, v3& result, int lane) {
  const float planeDist = vdot(pn.point, pn.normal);
  const float planeDistSq = sqrf(planeDist);
  const float radiusSq = sqrf(radius);
  if (planeDistSq > radiusSq) return false;
  const float planeRadiusSq = radiusSq - planeDistSq;
  const v3 planeCenter = smul(planeDist, pn.normal);
  if (dirOpt) {
    const v3 pov = vsub(opt, smul(vdot(opt, pn.normal), pn.normal));
    const float povSq = vdot(pov, pov);
    if (povSq <= kRvoEps) result = planeCenter;
    else result = vadd(planeCenter, smul(sqrtf(planeRadiusSq / povSq), pov));
  } else {
    result = vadd(opt, smul(vdot(vsub(pn.point, opt), pn.normal), pn.normal));
    if (vdot(result, result) > radiusSq) {
      const v3 pr = vsub(result, planeCenter);
      const float prSq = vdot(pr, pr);
      result = vadd(planeCenter, smul(sqrtf(planeRadiusSq / prSq), pr));
    }
  }
  LPPlane nx = planeNo > 0 ? (ob == 0 ? po : ld_plane_if<PS>(planes, lane, planeNo)) : po;
  for (int base = 0; base < planeNo; base += 64) {
    const LPPlane pj = nx;
    if (base + 64 < planeNo) nx = base + 64 == ob ? po : ld_plane_if<PS>(planes, base + 64 + lane, planeNo);
    const bool inr = base + lane < planeNo;
    unsigned long long b = __ballot(inr && lp_violates(pj, result, 0.0f));
    if (!b) continue;
    // the chunk's lines (LQRO:1086-1097), once, at its first violated plane
    const v3 cp = vcross(pj.normal, pn.normal);
    const unsigned long long parb = __ballot(vdot(cp, cp) <= kRvoEps);
    const v3 ldir = vnormalize(cp);
    const v3 lineNormal = vcross(ldir, pn.normal);
    const v3 lpt = vadd(pn.point, smul(vdot(vsub(pj.point, pn.point), pj.normal) / vdot(lineNormal, pj.normal),
                                       lineNormal));
    for (;;) {
      const int k = __ffsll((long long)b) - 1;
      if ((parb >> k) & 1ull) return false;
      if (!w_lp1<PS>(planes, base + k, base, pj, lp_rl3(lpt, k), lp_rl3(ldir, k), radius, opt, dirOpt, result,
                     lane))
        return false;
      b = __ballot(inr && lane > k && lp_violates(pj, result, 0.0f));
      if (!b) break;
    }
  }
  return true;
}

// linearProgram3 (LQRO:1106-1129): the index of the plane it fails on, or m
template <int PS>
__device__ __forceinline__ int w_lp3(const float* planes, int m, double radius, v3 opt, bool dirOpt, v3& result,
                                     int lane) {
  const float rf = (float)radius;
  if (dirOpt) result = vmul(opt, rf);
  else if (vdot(opt, opt) > sqrf(rf)) result = vmul(vnormalize(opt), rf);
  else result = opt;
  LPPlane nx = ld_plane_if<PS>(planes, lane, m);
  for (int base = 0; base < m; base += 64) {
    const LPPlane pj = nx;
    if (base + 64 < m) nx = ld_plane_if<PS>(planes, base + 64 + lane, m);
    const bool inr = base + lane < m;
    unsigned long long b = __ballot(inr && lp_violates(pj, result, 0.0f));
    while (b) {
      const int k = __ffsll((long long)b) - 1;
      LPPlane pn;
      pn.point = lp_rl3(pj.point, k);
      pn.normal = lp_rl3(pj.normal, k);
      const v3 tmp = result;
      if (!w_lp2<PS>(planes, base + k, pn, base, pj, rf, opt, dirOpt, result, lane)) {
        result = tmp;
        return base + k;
      }
      b = __ballot(inr && lane > k && lp_violates(pj, result, 0.0f));
    }
  }
  return m;
}

// linearProgram4 (LQRO:1131-1206): the projected planes of plane i are built
// in parallel and compacted in j order (skipped same-direction parallels keep
// their order)
template <int PS>
__device__ __forceinline__ void w_lp4(const float* planes, int m, int beginPlane, float radius, v3& result,
                      float* proj, int lane
#ifdef LQRO_LP_PROFILE
                      , int& lp4_iters
#endif
                      ) {
  float distance = 0.0f;
  for (int base = beginPlane; base < m; base += 64) {
    const LPPlane pc = ld_plane_if<PS>(planes, base + lane, m);
    const bool inr = base + lane < m;
    unsigned long long b = __ballot(inr && lp_violates(pc, result, distance));
    while (b) {
      const int k = __ffsll((long long)b) - 1;
      const int i = base + k;
      LPPlane pi;
      pi.point = lp_rl3(pc.point, k);
      pi.normal = lp_rl3(pc.normal, k);
      int np = 0;
      for (int jb = 0; jb < i; jb += 64) {
        const int j = jb + lane;
        bool keep = false;
        v3 ppt = V3(0, 0, 0), pnm = V3(0, 0, 0);
        if (j < i) {
          const LPPlane pj = ld_plane<PS>(planes, j);
          const v3 cp = vcross(pj.normal, pi.normal);
          keep = true;
          if (vdot(cp, cp) <= kRvoEps) {
            if (vdot(pi.normal, pj.normal) > 0.0f) keep = false;
            else ppt = smul(0.5f, vadd(pi.point, pj.point));
          } else {
            const v3 lineNormal = vcross(cp, pi.normal);
            ppt = vadd(pi.point, smul(vdot(vsub(pj.point, pi.point), pj.normal) /
                                          vdot(lineNormal, pj.normal),
                                      lineNormal));
          }
          if (keep) pnm = vnormalize(vsub(pj.normal, pi.normal));
        }
        const unsigned long long kb = __ballot(keep);
        if (keep) st_plane<PS>(proj, np + __popcll(kb & ((1ull << lane) - 1ull)), ppt, pnm);
        np += __popcll(kb);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const v3 tmp = result;
      if (w_lp3<PS>(proj, np, radius, pi.normal, true, result, lane) < np) result = tmp;
      distance = vdot(pi.normal, vsub(pi.point, result));
#ifdef LQRO_LP_PROFILE
      ++lp4_iters;
#endif
      b = __ballot(inr && lane > k && lp_violates(pc, result, distance));
    }
  }
}

}  // namespace lqro
