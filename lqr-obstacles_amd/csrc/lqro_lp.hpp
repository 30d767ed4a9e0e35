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

// first plane index in [i0, n) with normal.(point - r) > thresh, or n
template <int PS>
__device__ __forceinline__ int first_violated(const float* planes, int i0, int n, v3 r, float thresh,
                                              int lane) {
  for (int base = i0; base < n; base += 64) {
    const int i = base + lane;
    bool v = false;
    if (i < n) {
      LPPlane p = ld_plane<PS>(planes, i);
      v = vdot(p.normal, vsub(p.point, r)) > thresh;
    }
    unsigned long long b = __ballot(v);
    if (b) return base + __ffsll((long long)b) - 1;
  }
  return n;
}

template <int PS>
__device__ __forceinline__ bool w_lp1(const float* planes, int planeNo, v3 lpt, v3 ldir, float radius, v3 opt,
                      bool dirOpt, v3& result, int lane) {
  const float dotProduct = vdot(lpt, ldir);
  const float disc = sqrf(dotProduct) + sqrf(radius) - vdot(lpt, lpt);
  if (disc < 0.0f) return false;
  const float sq = sqrtf(disc);
  float tLeft = -dotProduct - sq;
  float tRight = -dotProduct + sq;
  float lmax = -INFINITY, lmin = INFINITY;
  bool reject = false;
  for (int i = lane; i < planeNo; i += 64) {
    LPPlane pi = ld_plane<PS>(planes, i);
    const float numerator = vdot(vsub(pi.point, lpt), pi.normal);
    const float denominator = vdot(ldir, pi.normal);
    if (sqrf(denominator) <= kRvoEps) {
      if (numerator > 0.0f) reject = true;
      continue;
    }
    const float t = numerator / denominator;
    if (denominator >= 0.0f) lmax = stdmax(lmax, t);
    else lmin = stdmin(lmin, t);
  }
  if (__ballot(reject)) return false;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    lmax = stdmax(lmax, __shfl_xor(lmax, off));
    lmin = stdmin(lmin, __shfl_xor(lmin, off));
  }
  tLeft = stdmax(tLeft, lmax);
  tRight = stdmin(tRight, lmin);
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

template <int PS>
__device__ __forceinline__ bool w_lp2(const float* planes, int planeNo, float radius, v3 opt, bool dirOpt,
                      v3& result, int lane) {
  const LPPlane pn = ld_plane<PS>(planes, planeNo);
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
  for (int i = first_violated<PS>(planes, 0, planeNo, result, 0.0f, lane); i < planeNo;
       i = first_violated<PS>(planes, i + 1, planeNo, result, 0.0f, lane)) {
    const LPPlane pi = ld_plane<PS>(planes, i);
    v3 cp = vcross(pi.normal, pn.normal);
    if (vdot(cp, cp) <= kRvoEps) return false;
    const v3 ldir = vnormalize(cp);
    const v3 lineNormal = vcross(ldir, pn.normal);
    const v3 lpt = vadd(pn.point, smul(vdot(vsub(pi.point, pn.point), pi.normal) /
                                           vdot(lineNormal, pi.normal),
                                       lineNormal));
    if (!w_lp1<PS>(planes, i, lpt, ldir, radius, opt, dirOpt, result, lane)) return false;
  }
  return true;
}

template <int PS>
__device__ __forceinline__ int w_lp3(const float* planes, int m, double radius, v3 opt, bool dirOpt, v3& result,
                     int lane) {
  const float rf = (float)radius;
  if (dirOpt) result = vmul(opt, rf);
  else if (vdot(opt, opt) > sqrf(rf)) result = vmul(vnormalize(opt), rf);
  else result = opt;
  for (int i = first_violated<PS>(planes, 0, m, result, 0.0f, lane); i < m;
       i = first_violated<PS>(planes, i + 1, m, result, 0.0f, lane)) {
    const v3 tmp = result;
    if (!w_lp2<PS>(planes, i, rf, opt, dirOpt, result, lane)) { result = tmp; return i; }
  }
  return m;
}

// linearProgram4: the projected planes of plane i are built in parallel and
// compacted in j order (skipped same-direction parallels keep their order).
template <int PS>
__device__ __forceinline__ void w_lp4(const float* planes, int m, int beginPlane, float radius, v3& result,
                      float* proj, int lane
#ifdef LQRO_LP_PROFILE
                      , int& lp4_iters
#endif
                      ) {
  float distance = 0.0f;
  for (int i = first_violated<PS>(planes, beginPlane, m, result, distance, lane); i < m;
       i = first_violated<PS>(planes, i + 1, m, result, distance, lane)) {
    const LPPlane pi = ld_plane<PS>(planes, i);
    int np = 0;
    for (int base = 0; base < i; base += 64) {
      const int j = base + lane;
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
      const unsigned long long b = __ballot(keep);
      if (keep) st_plane<PS>(proj, np + __popcll(b & ((1ull << lane) - 1ull)), ppt, pnm);
      np += __popcll(b);
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
  }
}

}  // namespace lqro
