// lqro_hull.hpp — the inside-hull branch, in-kernel.
//
// Replaces convexHull (LQRObstacles.cpp:867-969), which writes the reachable
// points to pointList.txt at iostream's default 6 significant digits
// (:869-874), runs qconvex.exe twice (:879-880) and takes
//     min_f | n_f . (vrel - P[first vertex of f]) |   (:955-968)
// over the hull facets, n_f from the hull of the ROUNDED points, P at full
// precision.  One workgroup per inside-hull pair (persistent over the queue
// k_pair fills):
//   1. recomputes the pair's reachable points in reference order (exact, as
//      k_pair does) and their %g round trip (lqro_device.hpp: round6);
//   2. builds the hull of the rounded points by quickhull: faces with outside
//      points wait in work queues; an insertion takes a face, adds its
//      furthest outside point as a vertex, grows the point's visible region
//      over the face adjacency, links a cone over the horizon and
//      re-distributes the region's outside points over the cone;
//   3. evaluates the reference's facet formula on every facet (canonical
//      facet order, lowest-index vertex) and writes the
//      half-plane (createHalfPlanes, :1208-1221, inside => mult = +1).
// A point is beyond a face iff n.(p - a) > eps |n|, n = (b-a) x (c-a),
// eps = 1e-13 (max|coord| + 1) — the rule of the oracle's hull, so the facet
// set (unique for points in general position) is the oracle's, whatever the
// insertion order.
//
// k_hull (topology in LDS) runs the insertions on all HULL_CWAVES waves at
// once: each wave inserts on its own, and two insertions proceed together
// when their visible regions and the faces bordering them are disjoint.
// Every face carries a lock word; an insertion locks its region and border
// faces as it grows the region, and backs off (re-queueing its face) when it
// meets a face another wave holds.  Holding every face it reads or writes
// until it is done makes the insertions serialisable, so the result is that
// of some sequential insertion order.  Jobs whose hull outgrows the LDS
// capacities are re-run by k_hull_big: one inserting wave, topology in
// global memory.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lqro.h"
#include "lqro_device.hpp"

namespace lqro {

#define HULL_WAVES 4             // k_hull_big: the points / initial hull / facet phases use 4 waves,
#define HULL_THREADS (64 * HULL_WAVES)   // the insertions one
#ifndef HULL_CWAVES
#define HULL_CWAVES 8            // k_hull: waves, all of them inserting
#endif
#define HULL_CTHREADS (64 * HULL_CWAVES)
#define HULL_SCR_WAVES 8         // per-block integer scratch: 2*H*NP ints per wave

#define HULL_SBMULT 24           // outside-set segment buffer: HULL_SBMULT * H*NP entries
#define HULL_STKMULT 4           // work stack: HULL_STKMULT * H*NP faces
#define HULL_FB_STRIDE 16384     // per-block face records in global scratch (= big faces)
#define HULL_VG_STRIDE 8192      // per-block vertex records in global scratch (= big vertices)

#define HULL_QCAP 512            // k_hull: per-wave face queue (LDS ring)
#define HULL_FLCAP 256           // k_hull: per-wave list of retired face slots
#define HULL_BAGCAP 16384        // k_hull: per-block overflow bag in global memory

// an outside-set entry: the point and its (rounded) coordinates, so that
// re-distributing it needs one load
struct HullPt {
  double x, y, z;
  int q, pad;
};

struct HullWide;

struct HullArgs {
  int N, X, H, NP;
  int row_begin, npr, per_agent;
  int row_stride;                   // local row r is agent row_begin + r * row_stride
  const int* nbr_list;   // culling on: slot -> neighbour jj (see PairArgs), else null
  double r2, r2_lo, r2_hi;
  const double* T;
  const double* NCF;
  const double* S;
  const double* x;
  float* planes;
  lqro_pair_record* recs;
  const int* queue;
  const int* count;
  int cap;
  int* next;
  double* scratch;                  // per block: H*NP*6 doubles (rounded, full)
  int* iscratch;                    // per block: 2*H*NP*HULL_SCR_WAVES ints
  float* fscratch;                  // per block: H*NP floats (distance beyond the target)
  HullPt* sb;                       // per block: HULL_SBMULT*H*NP entries (outside-set segments)
  unsigned long long* fbest;        // per block: HULL_FB_STRIDE furthest-point keys
  int* vpid;                        // per block: HULL_VG_STRIDE vertex -> point ids
  int* stack;                       // per block: HULL_STKMULT*H*NP faces
  int* rqueue;                      // pairs that overflowed the LDS variant
  int* rcount;
  int* rnext;
  void* bigmem;                     // per block of k_hull_big: one HullMemBig
  HullWide* wide;                   // per block of k_hull: HULL_CWAVES wide-insertion lists
  int* bag;                         // per block of k_hull: HULL_BAGCAP overflow face ids (-1: empty)
  int block_base;                   // scratch index of this launch's block 0
  int big_main;                     // k_hull_big takes the main queue (H*NP too large for LDS)
  int big_inline;                   // k_qhull rebuilds a build past its caps in place (q3_big_inline)
  int qflags;                       // k_qhull: 1 helper waves locate long sequences, 2 the emit's lane state,
                                    // 4 wave 1 pre-scans the next speculation's queue entry, 16 a long
                                    // emit split over the waves
  int* lqueue;                      // k_lhull: pairs the local hull hands to the full hull
  int* lcount;
  int* ldone;                       // k_lhull: pairs it decided
  unsigned long long* lfail;        // k_lhull: hand-over reasons (16 counters, cumulative)
  unsigned long long* ljobs;        // k_lhull: per job (< 4096) 4 words: point / loop ticks (100 MHz), counts
  // lqro_debug_hull_points (test hook): the job's points given (already
  // rounded: P = P_rounded), k_hull's facets written out
  const double* ext_pts;
  int ext_n, ext_max;
  int ext_full;                     // ext_pts also holds the full-precision points (k_qhull hook)
  int* ext_facets;                  // ext_max x 3 point ids
  int* ext_nf;
  unsigned long long* stats;
  unsigned long long* prof;          // LQRO_HULL_PROFILE: per-phase cycles
  // k_qhull (LQRO_FLAG_QHULL_ORDER): per-worker scratch, per-slot normal and
  // distance, the slots whose facet 0 won (resolved by k_stale)
  char* qscratch;
  size_t qstride;
  double* qnrm;
  int* qstale;
  int* qstale_count;
  int qstale_cap;
  // early LP (lqro_runtime.hip, LQRO_ROW_BIG): rowpend counts each row's
  // open work down, rowclaim says who runs its LP (0 free, 1 claimed, 2 late:
  // a facet-0 pair waits for k_stale); the k_qhull job that completes a row
  // runs calculateNewV for it (lp_vgoal -> lp_newv).  Null: off.
  int* rowpend;
  int* rowclaim;
  int row_target;
  const double* lp_vgoal;
  double* lp_newv;
  double lp_vmax;
  // Qhull order: one timing record per build (hull_build_note), null: off
  unsigned long long* hbuild;
  int hbuild_cap;
  // jobs still being produced by a concurrent hot launch: a worker that finds
  // the queue empty waits until *prod_done reaches prod_total (its workgroups
  // finished) before it leaves; null: leave at once
  const int* prod_done;
  int prod_total;
  // Qhull order, speculative builds (PairArgs::spec_mark): a job whose slot
  // is marked >= 2 was queued before its pair was evaluated; the build
  // commits only once the mark is 3.  null: off
  const unsigned char* spec_mark;
  // ... and their queue entries 0 .. *spec_n - 1 are handed out by a plain
  // counter (*spec_next, one atomicAdd a worker: at the step's start every
  // side worker asks at once, and the head's compare-and-swap would hand
  // them out one round trip at a time); the queue's own head starts at
  // *spec_n.  null: off
  const int* spec_n;
  int* spec_next;
  // early LP: 1 when a k_qhull job that closes a row may run its LP in its
  // own LDS (rows of at most LQRO_EARLY_LP_MAX_NPR pairs); 0: such rows are
  // left to the tail
  int row_lp;
};

// (LQRO_ROW_BIG, lqro_device.hpp: the row counter's protocol; the early LP
// runs in k_qhull's facet-plane LDS: rows of at most LQRO_EARLY_LP_MAX_NPR
// pairs, planes and projections 32 B each)
#define LQRO_EARLY_LP_MAX_NPR 1024
// lane 0, after the job's plane (or its pending / failed flag) is written:
// count the row down; true when this job closed the row and claimed its LP
// (can_run: the caller will run it)
__device__ inline bool hull_row_done(const HullArgs& A, int slot, bool stale, bool can_run) {
  if (!A.rowpend) return false;
  const int lrow = slot / A.npr;
  if (stale) atomicExch(&A.rowclaim[lrow], 2);
  __threadfence();
  const int old = atomicSub(&A.rowpend[lrow], 1);
  const bool go = can_run && old - 1 == A.row_target && atomicCAS(&A.rowclaim[lrow], 0, 1) == 0;
  __threadfence();
  return go;
}

// Hull topology and vertex coordinates for k_hull_big (global scratch).
template <int FMAX, int VTX, class SEG>
struct HullMem {
  static constexpr int kFaces = FMAX, kVerts = VTX;
  SEG seg[FMAX];                     // outside set of face f: sb[off .. off+cnt)
  unsigned short fv[FMAX][3];        // vertex slots, outward counter-clockwise
  unsigned short fa[FMAX][3];        // fa[f][e]: face across edge (fv[e], fv[e+1])
  unsigned short vst[FMAX];          // visible-region stamp (insertion number)
  unsigned short freel[FMAX];        // retired face slots
  unsigned char alive[FMAX];
  double vx[VTX][3];                 // hull vertex coordinates (rounded points)
  unsigned short vmap[VTX];          // horizon: vertex slot -> edge leaving it
};
typedef HullMem<16384, 8192, unsigned long long> HullMemBig;   // ~610 KB: global scratch

// k_hull_big's per-step work lists (LDS)
template <int RG, int HZ, int NW>
struct HullLdsT {
  static constexpr int kRegion = RG, kHorizon = HZ;
  unsigned short region[RG];                 // visible region of the apex
  int roff[RG], rcnt[RG], rpre[RG + 1];      //   their outside sets
  unsigned short h_a[HZ], h_b[HZ], h_out[HZ], h_new[HZ];   // horizon edges, cone faces
  int hcnt[HZ], hoff[HZ];
  double cn[HZ][8];                          // cone planes: n, a, |n|, eps |n|
  double tr[3 * 128];
  double rk[NW];
  int ri[NW];
  int scan[NW];
  int nf, nfree, nvtx, fail, n, job, slot, init[4], sbtop, sp, qh, it;
  double eps;
};
typedef HullLdsT<2048, 1024, HULL_WAVES> HullLdsBig;

// k_hull's topology (LDS, ~129 KB).  own[f], the face's lock word:
//   bits  0-15  its furthest outside point (HULL_NOPT: none)
//   bits 16-23  lock, one bit per wave
//   bits 24-31  visible-region mark, one bit per wave; all set: retired slot
// Extents are packed as (off / 4) << 15 | cnt: k_hull's segments start at
// multiples of 4 entries (seg_round), so H*NP <= kHullLdsMaxHNP (see runtime).
#define HULL_NOPT 0xFFFFu
#define HULL_DEAD 0xFF00FFFFu
struct HullMemC {
  static constexpr int kFaces = 4160, kVerts = 2048;
  unsigned int seg[kFaces];
  unsigned int own[kFaces];
  unsigned short fv[kFaces][3];
  unsigned short fa[kFaces][3];
  double vx[kVerts][3];
};

// one inserting wave's lists for an insertion whose visible region or
// horizon exceeds 64 faces (rare; global scratch)
#define HULL_WIDE 1024
struct HullWide {
  int reg[HULL_WIDE];                       // region faces 64..R-1
  int ha[HULL_WIDE], hb[HULL_WIDE], on[HULL_WIDE], sf[HULL_WIDE];   // horizon edges, cone faces
  int cnt[HULL_WIDE], off[HULL_WIDE];
  unsigned long long kmax[HULL_WIDE];
  double cn[HULL_WIDE][8];                  // cone planes: n, a, 1/|n|, eps^2 |n|^2
  int vnext[2048], vprev[2048];             // horizon vertex -> edge leaving / entering it
};

// one inserting wave's LDS: its face queue (a ring; the owner appends, any
// wave takes from the head), retired slots, horizon staging, per-cone-face
// counters
struct HullWaveL {
  unsigned long long kmax[64];
  int hcnt[64];
  unsigned short q[HULL_QCAP];
  unsigned short freel[HULL_FLCAP];
  unsigned short h_a[64], h_b[64], h_out[64];
  unsigned short ovf[64];                   // staging: queue overflow -> local batch
  int head, tail;
};

template <int NW>
struct HullLdsC {
  double tr[3 * 128];
  double rk[NW];
  int ri[NW];
  int scan[NW];
  unsigned long long kmax4[4];
  int n, fail, job, slot, init[4], hcnt[4], hoff[4];
  int nf, nvtx, sbtop, work;
  int gb_head, gb_tail;              // overflow bag (global memory) of this job
  double eps;
  HullWaveL wl[NW];
};

// Ordering point between the lanes of one wave.  A wave
// executes its LDS and its global memory operations in issue order, so only
// the compiler has to be kept from moving memory operations across this
// point; no s_waitcnt / s_barrier is needed (a workgroup fence would stall on
// every outstanding global store).
// The step's counters (lqro_get_stats_ex): [0..7] lqro_get_stats' words;
// [8] Qhull-order hulls Qhull would merge facets in (LQRO_REC_QHMERGE);
// [9] builds k_qhull's caps handed to k_qhull_big; [10] k_qhull wave-handshake
// timeouts (the build went to k_qhull_big); [11] pairs left without their
// half-plane, the first LQRO_ST_FAILMAX of their slots in [16 ..]
#define LQRO_ST_MERGED 8
#define LQRO_ST_RETRY 9
#define LQRO_ST_TIMEOUT 10
#define LQRO_ST_NFAIL 11
#define LQRO_ST_MWIN 12     // pairs flagged LQRO_REC_QHMERGE_WIN (lqro_get_stats_ex [11])
#define LQRO_QHMERGE_K 1024.0   // the merge-suspect test's reach, x qh DISTround (q3_merge_suspect)
#define LQRO_ST_NBUILD 13   // Qhull-order build records written (A.hbuild)
#define LQRO_HBUILD_CAP 16384
#define LQRO_ST_FAILS 16
#define LQRO_ST_FAILMAX 64
#define LQRO_ST_MWINS (LQRO_ST_FAILS + LQRO_ST_FAILMAX)   // the first LQRO_ST_FAILMAX MWIN slots
#define LQRO_ST_WORDS (LQRO_ST_MWINS + LQRO_ST_FAILMAX + 4)   // + LQRO_ST_SWORK, _BWORK, _BMAX (lqro_device.hpp)
static_assert(LQRO_ST_SWORK == LQRO_ST_MWINS + LQRO_ST_FAILMAX, "the work words follow the named pairs");

// an inside-hull pair left without its half-plane (a hull capacity): counted
// in stats[4] and named, so the step reports it (LQRO_E_HULL) instead of
// dropping the constraint silently
__device__ __forceinline__ void hull_fail_note(unsigned long long* stats, int slot) {
  atomicAdd(&stats[4], 1ull);
  const unsigned long long k = atomicAdd(&stats[LQRO_ST_NFAIL], 1ull);
  if (k < LQRO_ST_FAILMAX) stats[LQRO_ST_FAILS + k] = (unsigned long long)slot;
}

// a pair flagged LQRO_REC_QHMERGE_WIN: counted and named, so that lqro_step
// returns LQRO_E_QHMERGE instead of a silent difference from qconvex's merged
// facet (LQRO:925-967)
__device__ __forceinline__ void qhmerge_note(unsigned long long* stats, int slot) {
  const unsigned long long k = atomicAdd(&stats[LQRO_ST_MWIN], 1ull);
  if (k < LQRO_ST_FAILMAX) stats[LQRO_ST_MWINS + k] = (unsigned long long)slot;
}

// lane 0: a Qhull-order build's timing record (lqro_get_hull_builds):
// slot | kernel << 40, start, end (s_memrealtime, 100 MHz), points |
// insertions << 20 | facet slots << 40
__device__ __forceinline__ int hull_build_note(const HullArgs& A, int slot, int kernel, unsigned long long t0,
                                                int n, int nins, int nfac) {
  if (!A.hbuild) return -1;
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  atomicAdd(&A.stats[LQRO_ST_BWORK], t1 - t0);   // (the next steps' side width)
  atomicMax(&A.stats[LQRO_ST_BMAX], t1 - t0);
  const unsigned long long k = atomicAdd(&A.stats[LQRO_ST_NBUILD], 1ull);
  if (k >= (unsigned long long)A.hbuild_cap) return -1;
  unsigned long long* r = A.hbuild + 4 * k;
  r[0] = (unsigned long long)(unsigned)slot | ((unsigned long long)kernel << 40);
  r[1] = t0;
  r[2] = t1;
  r[3] = (unsigned long long)(n & 0xFFFFF) | ((unsigned long long)(nins & 0xFFFFF) << 20) |
         ((unsigned long long)(nfac & 0xFFFFF) << 40);
  return (int)k;
}

__device__ __forceinline__ void hl_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// compiler-only ordering of memory operations (LDS executes a wave's
// operations in issue order)
__device__ __forceinline__ void hl_cfence() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ int hl_ld(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void hl_st(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ double hl_rl(double v, int k) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, k);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), k);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// outside-set extent of face f
__device__ __forceinline__ void seg_get(unsigned int s, int& off, int& cnt) {
  off = (int)((s >> 15) << 2); cnt = (int)(s & 0x7FFFu);
}
__device__ __forceinline__ void seg_get(unsigned long long s, int& off, int& cnt) {
  off = (int)(s >> 32); cnt = (int)(s & 0xFFFFFFFFu);
}
__device__ __forceinline__ void seg_put(unsigned int& s, int off, int cnt) {
  s = (((unsigned int)off >> 2) << 15) | (unsigned int)cnt;
}
// room a segment of cnt entries takes in k_hull's buffer (starts stay 4-aligned)
__device__ __forceinline__ int seg_round(int cnt) { return (cnt + 3) & ~3; }
__device__ __forceinline__ void seg_put(unsigned long long& s, int off, int cnt) {
  s = ((unsigned long long)(unsigned)off << 32) | (unsigned)cnt;
}

// Barrier across the workgroup's waves.
__device__ __forceinline__ void hl_bar() { __syncthreads(); }

// n = (b-a) x (c-a) of face f
template <class Mem>
__device__ __forceinline__ void hl_normal(const Mem& L, int f, double* n) {
  const double* a = L.vx[L.fv[f][0]];
  const double* b = L.vx[L.fv[f][1]];
  const double* c = L.vx[L.fv[f][2]];
  const double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  const double e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  n[0] = e1[1] * e2[2] - e1[2] * e2[1];
  n[1] = e1[2] * e2[0] - e1[0] * e2[2];
  n[2] = e1[0] * e2[1] - e1[1] * e2[0];
}
// is p beyond face f: d > eps |n| with d = n.(p - a), tested squared (no
// sqrt on the hot path): d > 0 and d^2 > eps^2 (n.n).  *dist = d / |n|.
template <class Mem>
__device__ __forceinline__ bool hl_beyond(const Mem& L, int f, const double* p, double eps2,
                                          double* dist) {
  double n[3];
  hl_normal(L, f, n);
  const double* a = L.vx[L.fv[f][0]];
  const double d = n[0] * (p[0] - a[0]) + n[1] * (p[1] - a[1]) + n[2] * (p[2] - a[2]);
  const double nn = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
  if (dist) *dist = d / sqrt(nn);
  return d > 0.0 && d * d > eps2 * nn;
}


// block-wide argmax of (key, idx), lowest idx on ties; result in every thread
template <class LT>
__device__ __forceinline__ void hl_argmax(LT& L, double& key, int& idx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ok = __shfl_xor(key, off);
    const int oi = __shfl_xor(idx, off);
    if (ok > key || (ok == key && oi < idx)) { key = ok; idx = oi; }
  }
  if (lane == 0) { L.rk[wave] = key; L.ri[wave] = idx; }
  hl_bar();
  key = L.rk[0]; idx = L.ri[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
    if (L.rk[w] > key || (L.rk[w] == key && L.ri[w] < idx)) { key = L.rk[w]; idx = L.ri[w]; }
  hl_bar();
}

// exclusive block scan of v (0/1); total in *tot
template <class LT>
__device__ __forceinline__ int hl_scan(LT& L, int v, int* tot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long b = __ballot(v != 0);
  const int in_wave = __popcll(b & ((1ull << lane) - 1ull));
  if (lane == 0) L.scan[wave] = __popcll(b);
  hl_bar();
  int base = 0, t = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
    if (w < wave) base += L.scan[w];
    t += L.scan[w];
  }
  *tot = t;
  hl_bar();
  return base + in_wave;
}

#ifdef LQRO_HULL_PROFILE
#define HSUB(k)                                                     \
  do {                                                              \
    if (tid == 0) {                                                 \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
      prof_sub[k] += t_ - prof_last;                                \
      prof_last = t_;                                               \
    }                                                               \
  } while (0)
#define HSTAMP(k)                                                   \
  do {                                                              \
    if (tid == 0) {                                                 \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
      prof_acc[k] += t_ - prof_last;                                \
      prof_last = t_;                                               \
    }                                                               \
  } while (0)
#define WSTAMP(k)                                                   \
  do {                                                              \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();     \
    wacc[k] += t_ - wlast;                                          \
    wlast = t_;                                                     \
  } while (0)
#else
#define HSTAMP(k) do {} while (0)
#define HSUB(k) do {} while (0)
#define WSTAMP(k) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// Phases shared by both kernels
// ---------------------------------------------------------------------------

// Take the next job (pair slot), or -1 when the queue holds no untaken entry.
template <class LT>
__device__ __forceinline__ int hull_take_job(const HullArgs& A, LT& L, bool retryq) {
  const int* queue = retryq ? A.rqueue : A.queue;
  const int* qcount = retryq ? A.rcount : A.count;
  int* qnext = retryq ? A.rnext : A.next;
  if (threadIdx.x == 0) {
    // take an entry only if it is there (CAS on the head): a workgroup that
    // finds the queue empty consumes no index, so entries a concurrent k_pair
    // launch appends later are still taken (by the k_hull after the sweep)
    int job = -1, slot = -1;
    long waited = 0;
    if (A.spec_next && !retryq) {
      const int m = __hip_atomic_load(A.spec_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int j = m > 0 ? atomicAdd(A.spec_next, 1) : m;
      if (j < m) {   // (written by k_prio_prev, a kernel before this one)
        job = j;
        slot = queue[j];
      }
    }
    for (; job < 0;) {
      // (the producers' count first: once it is complete, every job they
      // appended is in qcount)
      const int pd = (A.prod_done && !retryq) ? __hip_atomic_load(A.prod_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                                              : A.prod_total;
      const int nx = __hip_atomic_load(qnext, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      const int cnt = min(__hip_atomic_load(qcount, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT), A.cap);
      if (nx >= cnt) {
        // bounded: a worker that gives up leaves later jobs to the k_qhull
        // after the sweep (results do not depend on who builds)
        if (pd < A.prod_total && ++waited < (1l << 22)) {
          __builtin_amdgcn_s_sleep(4);
          continue;
        }
        break;
      }
      if (atomicCAS(qnext, nx, nx + 1) != nx) continue;
      job = nx;
      // counted before published: wait for k_pair's release store
      int v = __hip_atomic_load(queue + job, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      for (long w = 0; v < 0 && w < (1l << 26); ++w) {
        __builtin_amdgcn_s_sleep(2);
        v = __hip_atomic_load(queue + job, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      }
      slot = v;
      break;
    }
    L.job = job;
    L.slot = slot;
  }
  hl_bar();
  return L.slot;
}

// 1. The pair's reachable points in reference order, full precision (Pf)
// and %g-rounded (Pr); returns their number.  2. The tolerance eps, as the
// oracle's hull: 1e-13 (max|coord| + 1), in L.eps.
template <class LT>
__device__ __forceinline__ int hull_points(const HullArgs& A, LT& L, const double* Ti, const double* Ni,
                                           const double* xi, const double* xj, const double* vrel,
                                           double* Pr, double* Pf) {
  const int tid = threadIdx.x;
  if (tid == 0) { L.n = A.ext_pts ? A.ext_n : 0; L.fail = 0; }
  hl_bar();
  if (A.ext_pts)
    for (int q = tid; q < 3 * A.ext_n; q += blockDim.x) {
      Pr[q] = A.ext_pts[q];
      Pf[q] = A.ext_full ? A.ext_pts[3 * A.ext_n + q] : A.ext_pts[q];
    }
  for (int k0 = 0; k0 < (A.ext_pts ? 0 : A.H); k0 += 128) {
    for (int it = tid; it < 3 * 128; it += blockDim.x) {
      const int k = k0 + it / 3, r = it % 3;
      if (k < A.H) {
        double d = 0.0;
        for (int c = 0; c < A.X; ++c) d += Ni[((size_t)k * 3 + r) * A.X + c] * (xi[c] - xj[c]);
        L.tr[it] = d;
      }
    }
    hl_bar();
    const int kend = min(A.H, k0 + 128);
    for (int q0 = k0 * A.NP; q0 < kend * A.NP; q0 += blockDim.x) {
      const int q = q0 + tid;
      bool ok = false;
      double p0 = 0, p1 = 0, p2 = 0;
      if (q < kend * A.NP) {
        const int k = q / A.NP, p = q % A.NP;
        const double* Tk = Ti + (size_t)k * 9;
        const double* tk = L.tr + (k - k0) * 3;
        const double u0 = A.S[3 * p] + tk[0], u1 = A.S[3 * p + 1] + tk[1], u2 = A.S[3 * p + 2] + tk[2];
        p0 = ((0.0 + Tk[0] * u0) + Tk[1] * u1) + Tk[2] * u2;
        p1 = ((0.0 + Tk[3] * u0) + Tk[4] * u1) + Tk[5] * u2;
        p2 = ((0.0 + Tk[6] * u0) + Tk[7] * u1) + Tk[8] * u2;
        const double a = p0 - vrel[0], b = p1 - vrel[1], c = p2 - vrel[2];
        const double t = a * a + b * b + c * c;
        if (t < A.r2_lo) ok = true;
        else if (t > A.r2_hi) ok = false;
        else ok = (a * a) / A.r2 + (b * b) / A.r2 + (c * c) / A.r2 < 1.0;
      }
      int tot;
      const int pos = L.n + hl_scan(L, ok ? 1 : 0, &tot);
      if (ok) {
        int oor = 0;
        Pf[3 * pos] = p0; Pf[3 * pos + 1] = p1; Pf[3 * pos + 2] = p2;
        Pr[3 * pos] = round6(p0, &oor);
        Pr[3 * pos + 1] = round6(p1, &oor);
        Pr[3 * pos + 2] = round6(p2, &oor);
        if (oor) L.fail = 7;
      }
      hl_bar();
      if (tid == 0) L.n += tot;
      hl_bar();
    }
  }
  const int n = L.n;
  double mx = 0.0;
  int dummy = 0;
  for (int q = tid; q < 3 * n; q += blockDim.x) mx = fmax(mx, fabs(Pr[q]));
  hl_argmax(L, mx, dummy);
  if (tid == 0) {
    L.eps = 1e-13 * (mx + 1.0);
    if (n < 4) L.fail = 8;
  }
  hl_bar();
  return n;
}

// 3. Initial tetrahedron from extreme points: vertex slots 0..3, faces 0..3
// (outward, adjacency linked), L.init = their point ids.  Sets L.fail = 8
// for a degenerate point set.  Thread 0 writes; callers barrier after.
template <class Mem, class LT>
__device__ __forceinline__ void hull_tetra(Mem& M, LT& L, const double* Pr, int n, double eps,
                                           double eps2, int* vpid) {
  const int tid = threadIdx.x;
  double key; int idx;
  key = -INFINITY; idx = INT_MAX;
  for (int q = tid; q < n; q += blockDim.x) {
    const double v = -Pr[3 * q];
    if (v > key || (v == key && q < idx)) { key = v; idx = q; }
  }
  hl_argmax(L, key, idx);
  const int i0 = idx;
  const double* P0 = Pr + 3 * i0;
  key = -INFINITY; idx = INT_MAX;
  for (int q = tid; q < n; q += blockDim.x) {
    const double dx = Pr[3 * q] - P0[0], dy = Pr[3 * q + 1] - P0[1], dz = Pr[3 * q + 2] - P0[2];
    const double v = dx * dx + dy * dy + dz * dz;
    if (v > key || (v == key && q < idx)) { key = v; idx = q; }
  }
  hl_argmax(L, key, idx);
  const int i1 = idx;
  const double* P1 = Pr + 3 * i1;
  key = -INFINITY; idx = INT_MAX;
  for (int q = tid; q < n; q += blockDim.x) {
    const double e1[3] = {P1[0] - P0[0], P1[1] - P0[1], P1[2] - P0[2]};
    const double e2[3] = {Pr[3 * q] - P0[0], Pr[3 * q + 1] - P0[1], Pr[3 * q + 2] - P0[2]};
    const double cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2], cz = e1[0] * e2[1] - e1[1] * e2[0];
    const double v = cx * cx + cy * cy + cz * cz;
    if (v > key || (v == key && q < idx)) { key = v; idx = q; }
  }
  hl_argmax(L, key, idx);
  const int i2 = idx;
  if (tid == 0) {
    for (int d = 0; d < 3; ++d) {
      M.vx[0][d] = Pr[3 * i0 + d]; M.vx[1][d] = Pr[3 * i1 + d]; M.vx[2][d] = Pr[3 * i2 + d];
    }
    M.fv[0][0] = 0; M.fv[0][1] = 1; M.fv[0][2] = 2;
  }
  hl_bar();
  key = -INFINITY; idx = INT_MAX;
  for (int q = tid; q < n; q += blockDim.x) {
    double dd;
    hl_beyond(M, 0, Pr + 3 * q, eps2, &dd);
    const double v = fabs(dd);
    if (v > key || (v == key && q < idx)) { key = v; idx = q; }
  }
  hl_argmax(L, key, idx);
  const int i3 = idx;
  if (tid == 0) {
    if (!(key > eps) || i0 == i1 || i1 == i2 || i2 == i3) L.fail = 8;
    L.init[0] = i0; L.init[1] = i1; L.init[2] = i2; L.init[3] = i3;
    if (!L.fail) {
      for (int v = 0; v < 4; ++v) {
        vpid[v] = L.init[v];
        for (int d = 0; d < 3; ++d) M.vx[v][d] = Pr[3 * L.init[v] + d];
      }
      const int fvv[4][3] = {{0, 1, 2}, {0, 3, 1}, {1, 3, 2}, {0, 2, 3}};
      for (int f = 0; f < 4; ++f) {
        for (int e = 0; e < 3; ++e) M.fv[f][e] = (unsigned short)fvv[f][e];
        const int other = 6 - fvv[f][0] - fvv[f][1] - fvv[f][2];
        double dd;
        hl_beyond(M, f, M.vx[other], 0.0, &dd);
        if (dd > 0) { const unsigned short t = M.fv[f][1]; M.fv[f][1] = M.fv[f][2]; M.fv[f][2] = t; }
      }
      for (int f = 0; f < 4; ++f)
        for (int e = 0; e < 3; ++e) {
          const int a = M.fv[f][e], b = M.fv[f][(e + 1) % 3];
          for (int g = 0; g < 4; ++g)
            for (int e2 = 0; e2 < 3; ++e2)
              if (M.fv[g][e2] == b && M.fv[g][(e2 + 1) % 3] == a) M.fa[f][e] = (unsigned short)g;
        }
    }
  }
}

// 6. The reference's facet selection over all live faces f < nf (canonical
// order, see the file comment), then the half-plane, the record, the stats.
// A capacity failure of k_hull (fail 1-4, 11) hands the pair to k_hull_big.
template <class Mem, class LT, class Alive>
__device__ __forceinline__ void hull_select(const HullArgs& A, const Mem& M, LT& L, const double* Pr,
                                            const double* Pf, const int* vpid, int nf, Alive alive,
                                            const double* xi, const double* vrel, int slot, bool big) {
  const int tid = threadIdx.x;
  double best = INFINITY;
  int bt0 = INT_MAX, bt1 = INT_MAX, bt2 = INT_MAX, nfac = 0;
  double bn[3] = {0, 0, 0};
  if (!L.fail) {
    for (int f = tid; f < nf; f += blockDim.x) {
      if (!alive(f)) continue;
      nfac++;
      int t0 = vpid[M.fv[f][0]], t1 = vpid[M.fv[f][1]], t2 = vpid[M.fv[f][2]];
      while (!(t0 < t1 && t0 < t2)) { const int a = t0; t0 = t1; t1 = t2; t2 = a; }
      const double *a = Pr + 3 * t0, *b = Pr + 3 * t1, *c = Pr + 3 * t2;
      const double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
      const double e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
      double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
      const double len = sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
      nv[0] /= len; nv[1] /= len; nv[2] /= len;
      const double* p0 = Pf + 3 * t0;
      const double dd = fabs(nv[0] * (vrel[0] - p0[0]) + nv[1] * (vrel[1] - p0[1]) + nv[2] * (vrel[2] - p0[2]));
      const int s1 = min(t1, t2), s2 = max(t1, t2);
      const bool bt = dd < best || (dd == best && (t0 < bt0 || (t0 == bt0 && (s1 < bt1 || (s1 == bt1 && s2 < bt2)))));
      if (bt) { best = dd; bt0 = t0; bt1 = s1; bt2 = s2; bn[0] = nv[0]; bn[1] = nv[1]; bn[2] = nv[2]; }
    }
  }
  // block arg-min by (distance, triple): wave shuffles, then across waves
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ob = __shfl_xor(best, off);
    const int o0 = __shfl_xor(bt0, off), o1 = __shfl_xor(bt1, off), o2 = __shfl_xor(bt2, off);
    const double on0 = __shfl_xor(bn[0], off), on1 = __shfl_xor(bn[1], off), on2 = __shfl_xor(bn[2], off);
    nfac += __shfl_xor(nfac, off);
    const bool bt = ob < best || (ob == best && (o0 < bt0 || (o0 == bt0 && (o1 < bt1 || (o1 == bt1 && o2 < bt2)))));
    if (bt) { best = ob; bt0 = o0; bt1 = o1; bt2 = o2; bn[0] = on0; bn[1] = on1; bn[2] = on2; }
  }
  __shared__ double s_best[8], s_n[8][3];
  __shared__ int s_t[8][3], s_cnt[8];
  if (lane == 0) {
    s_best[wave] = best; s_t[wave][0] = bt0; s_t[wave][1] = bt1; s_t[wave][2] = bt2;
    s_n[wave][0] = bn[0]; s_n[wave][1] = bn[1]; s_n[wave][2] = bn[2]; s_cnt[wave] = nfac;
  }
  hl_bar();
  if (tid == 0) {
    int fo = 0, total = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      total += s_cnt[w];
      const bool bt = s_best[w] < s_best[fo] ||
                      (s_best[w] == s_best[fo] &&
                       (s_t[w][0] < s_t[fo][0] || (s_t[w][0] == s_t[fo][0] &&
                        (s_t[w][1] < s_t[fo][1] || (s_t[w][1] == s_t[fo][1] && s_t[w][2] < s_t[fo][2])))));
      if (bt) fo = w;
    }
    const bool ok = !L.fail && total > 0 && s_t[fo][0] != INT_MAX;
    // capacity overflow in the LDS variant: hand the pair to k_hull_big
    const bool retry = !big && ((L.fail >= 1 && L.fail <= 4) || L.fail == 6 || L.fail == 11);
    if (A.prof) atomicAdd(&A.prof[16 + (L.fail & 15)], 1ull);   // outcome histogram
    if (retry) {
      const int r = atomicAdd(A.rcount, 1);
      if (r < A.cap) A.rqueue[r] = slot;
    }
    float* pl = A.planes + (size_t)slot * 8;
    const double distance = s_best[fo];
    const double nrm[3] = {s_n[fo][0], s_n[fo][1], s_n[fo][2]};
    if (retry) {
      // written by k_hull_big
    } else if (ok) {
      const double dh = distance * 0.5;                  // :1416
      const double mult = 1.0;                           // :1213
      pl[0] = (float)(xi[3] + mult * dh * nrm[0]);
      pl[1] = (float)(xi[4] + mult * dh * nrm[1]);
      pl[2] = (float)(xi[5] + mult * dh * nrm[2]);
      pl[3] = (float)nrm[0]; pl[4] = (float)nrm[1]; pl[5] = (float)nrm[2];
      pl[6] = __int_as_float(1);
      atomicAdd(&A.stats[3], 1ull);
    } else {
      pl[6] = __int_as_float(0);                         // no usable plane
      hull_fail_note(A.stats, slot);
    }
    if (A.recs && !retry) {
      lqro_pair_record& rec = A.recs[slot];
      rec.flags |= ok ? LQRO_REC_HULL : LQRO_REC_HULLFAIL;
      rec.n_facets = ok ? total : -1;
      if (ok) {
        rec.facet[0] = s_t[fo][0]; rec.facet[1] = s_t[fo][1]; rec.facet[2] = s_t[fo][2];
        rec.dist = distance;
        for (int q = 0; q < 3; ++q) {
          rec.normal[q] = nrm[q];
          rec.plane_point[q] = pl[q];
          rec.plane_normal[q] = pl[3 + q];
        }
      }
    }
  }
  hl_bar();
}

// ---------------------------------------------------------------------------
// k_hull: concurrent insertions, topology in LDS
// ---------------------------------------------------------------------------

// take the oldest entry of wave queue Q (-1: empty); lane 0
__device__ __forceinline__ int hq_pop(HullWaveL& Q) {
  for (int tries = 0; tries < 16; ++tries) {
    const int h = hl_ld(&Q.head);
    hl_cfence();
    const int t = hl_ld(&Q.tail);
    hl_cfence();
    if (h >= t) return -1;
    const int e = __hip_atomic_load(&Q.q[h % HULL_QCAP], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    hl_cfence();
    if (atomicCAS(&Q.head, h, h + 1) == h) return e;
  }
  return -1;
}

// Stage the faces of the lanes with `is` (ballot order) behind the own
// queue's unpublished tail (mytail + qn).  What does not fit in the ring goes
// to the wave's local batch (lanes lbn.., taken next by this wave), so a full
// queue costs order, not a retry.  Returns 0, or 11 when both are full.
// The overflow bag: faces that fit neither the ring nor the local batch
// (global memory, filled by any wave, taken when the queues run dry).  Slots
// hold -1 until written; the job's used prefix is cleared when it ends.
struct HullBag {
  int* slot;
  int* head;   // LDS
  int* tail;   // LDS
};

__device__ __forceinline__ int hq_stage(HullWaveL& W, int mytail, int& qn, int& lb, int& lbn, bool is,
                                        int face, const HullBag& BG) {
  const int lane = threadIdx.x & 63;
  const unsigned long long b = __ballot(is);
  const int np = __popcll(b);
  if (np == 0) return 0;
  const int room = max(HULL_QCAP - (mytail + qn - hl_ld(&W.head)), 0);
  const int nq = min(np, room);
  const int rank = __popcll(b & ((1ull << lane) - 1ull));
  if (is && rank < nq) W.q[(mytail + qn + rank) % HULL_QCAP] = (unsigned short)face;
  qn += nq;
  const int nx = np - nq;
  if (nx == 0) return 0;
  if (lbn + nx > 64) {
    int pos = 0;
    if (lane == 0) pos = atomicAdd(BG.tail, nx);
    pos = __builtin_amdgcn_readlane(pos, 0);
    if (pos + nx > HULL_BAGCAP) return 11;
    if (is && rank >= nq)
      __hip_atomic_store(BG.slot + pos + rank - nq, face, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (is && rank >= nq) W.ovf[rank - nq] = (unsigned short)face;
  hl_sync();
  if (lane >= lbn && lane < lbn + nx) lb = W.ovf[lane - lbn];
  hl_sync();
  lbn += nx;
  return 0;
}

// take one face from the bag (lane 0; -1: empty)
__device__ __forceinline__ int hq_bag_take(const HullBag& BG) {
  for (int tries = 0; tries < 16; ++tries) {
    const int h = hl_ld(BG.head);
    hl_cfence();
    const int t = hl_ld(BG.tail);
    if (h >= t || h >= HULL_BAGCAP) return -1;
    if (atomicCAS(BG.head, h, h + 1) == h) {
      int e;
      for (int spin = 0;; ++spin) {   // the writer has reserved the slot; its store is in flight
        e = __hip_atomic_load(BG.slot + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (e >= 0 || spin > (1 << 20)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      return e;
    }
  }
  return -1;
}

// One insertion whose region (R) or horizon exceeds 64 faces: the steps of
// hull_insert_mw, chunked over 64 lanes with the lists in per-wave global
// scratch (WG).  The wave holds the region and the faces around it.
// Returns 0 or a failure code; updates the free-list length and queue tail.
template <int NW>
__device__ __noinline__ int hull_insert_wide(HullMemC& M, HullLdsC<NW>& L, HullWaveL& W, HullWide& WG,
                                             const double* Pr, int* vpid, HullPt* sb, int sbcap, int* sq,
                                             int HNP, int apex, const double* p, double eps2, int R, int rg,
                                             int& nfree, int& mytail, int& lb, int& lbn, const HullBag& BG,
                                             unsigned LK, unsigned RB) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = (1ull << lane) - 1ull;
  constexpr int kF = HullMemC::kFaces, kV = HullMemC::kVerts;
  auto region = [&](int r0, int r) { return r0 == 0 ? rg : WG.reg[r]; };
  // horizon, in (region order, edge) order
  int nh = 0;
  for (int b0 = 0; b0 < 3 * R; b0 += 64) {
    const int t = b0 + lane;
    const int rr = t / 3;
    int g = __shfl(rg, min(rr, 63));
    int ha = 0, hb = 0, ho = 0, is = 0;
    if (t < 3 * R) {
      if (rr >= 64) g = WG.reg[rr];
      const int e = t % 3;
      ho = M.fa[g][e];
      if (!(M.own[ho] & RB)) { is = 1; ha = M.fv[g][e]; hb = M.fv[g][e == 2 ? 0 : e + 1]; }
    }
    const unsigned long long b = __ballot(is);
    const int pos = nh + __popcll(b & lt);
    if (is && pos < HULL_WIDE) { WG.ha[pos] = ha; WG.hb[pos] = hb; WG.on[pos] = ho; }
    nh += __popcll(b);
  }
  if (nh > HULL_WIDE || nh < 3) return 3;
  // cone face slots, apex vertex, horizon vertex maps
  const int used = min(nh, nfree);
  int sfb = 0, av = 0;
  if (lane == 0) { sfb = atomicAdd(&L.nf, nh - used); av = atomicAdd(&L.nvtx, 1); }
  sfb = __builtin_amdgcn_readlane(sfb, 0);
  av = __builtin_amdgcn_readlane(av, 0);
  if (sfb + (nh - used) > kF) return 4;
  if (av >= kV) return 1;
  if (lane == 0) {
    M.vx[av][0] = p[0]; M.vx[av][1] = p[1]; M.vx[av][2] = p[2];
    vpid[av] = apex;
  }
  for (int h0 = 0; h0 < nh; h0 += 64) {
    const int h = h0 + lane;
    if (h < nh) {
      WG.sf[h] = h < used ? (int)W.freel[nfree - 1 - h] : sfb + (h - used);
      WG.vnext[WG.ha[h]] = h;
      WG.vprev[WG.hb[h]] = h;
    }
  }
  hl_sync();
  int bad = 0;
  for (int h0 = 0; h0 < nh; h0 += 64) {
    const int h = h0 + lane;
    if (h >= nh) continue;
    const int ha = WG.ha[h], hb = WG.hb[h], on = WG.on[h], sf = WG.sf[h];
    const int kn = WG.vnext[hb], kp = WG.vprev[ha];        // edge leaving b, edge entering a
    if (kn < 0 || kn >= nh || kp < 0 || kp >= nh || WG.ha[kn] != hb || WG.hb[kp] != ha) { bad = 1; continue; }
    M.own[sf] = LK | HULL_NOPT;
    M.fv[sf][0] = (unsigned short)ha;
    M.fv[sf][1] = (unsigned short)hb;
    M.fv[sf][2] = (unsigned short)av;
    M.fa[sf][0] = (unsigned short)on;
    M.fa[sf][1] = (unsigned short)WG.sf[kn];
    M.fa[sf][2] = (unsigned short)WG.sf[kp];
    for (int e = 0; e < 3; ++e)
      if (M.fv[on][e] == hb && M.fv[on][e == 2 ? 0 : e + 1] == ha) M.fa[on][e] = (unsigned short)sf;
    const double* a = M.vx[ha];
    const double* bb = M.vx[hb];
    const double e1[3] = {bb[0] - a[0], bb[1] - a[1], bb[2] - a[2]};
    const double e2[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
    const double cx = e1[1] * e2[2] - e1[2] * e2[1];
    const double cy = e1[2] * e2[0] - e1[0] * e2[2];
    const double cz = e1[0] * e2[1] - e1[1] * e2[0];
    const double nn = cx * cx + cy * cy + cz * cz;
    double* cp = WG.cn[h];
    cp[0] = cx; cp[1] = cy; cp[2] = cz; cp[3] = a[0]; cp[4] = a[1]; cp[5] = a[2];
    cp[6] = 1.0 / sqrt(nn);
    cp[7] = eps2 * nn;
    WG.cnt[h] = 0;
    WG.kmax[h] = 0ull;
  }
  if (__ballot(bad)) return 5;
  hl_sync();
  // release the faces around the region, retire the region (see the fast path)
  for (int h0 = 0; h0 < nh; h0 += 64) {
    const int h = h0 + lane;
    if (h < nh) atomicAnd(&M.own[WG.on[h]], ~LK);
  }
  for (int r0 = 0; r0 < R; r0 += 64) {
    const int r = r0 + lane;
    if (r < R) M.own[region(r0, r)] = HULL_DEAD;
  }
  // the retired faces' outside points, one region face at a time:
  // first cone face beyond, rank and key by global atomics, to scratch
  int items = 0;
  for (int r = 0; r < R; ++r) {
    const int g = r < 64 ? __builtin_amdgcn_readlane(rg, r) : WG.reg[r];
    int so, sc;
    seg_get(M.seg[g], so, sc);
    for (int c0 = 0; c0 < sc; c0 += 64) {
      const int t = c0 + lane;
      HullPt e;
      e.q = -1;
      if (t < sc) e = sb[so + t];
      int tg = -1;
      float dv = 0.0f;
      bool pend = t < sc && e.q != apex;
      for (int h = 0; h < nh; ++h) {
        if (!__ballot(pend)) break;
        if (pend) {
          const double* cp = WG.cn[h];
          const double d = cp[0] * (e.x - cp[3]) + cp[1] * (e.y - cp[4]) + cp[2] * (e.z - cp[5]);
          if (d > 0.0 && d * d > cp[7]) { tg = h; dv = (float)(d * cp[6]); pend = false; }
        }
      }
      int code = 0;
      if (tg >= 0) {
        const int rk = atomicAdd(&WG.cnt[tg], 1);
        atomicMax(&WG.kmax[tg], ((unsigned long long)__float_as_uint(dv) << 32) |
                                    (unsigned long long)(~(unsigned)e.q));
        code = (rk << 11) | (tg + 1);
      }
      if (t < sc) { sq[items + t] = e.q; sq[HNP + items + t] = code; }
    }
    items += sc;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // the rank atomics have returned
  int run = 0;
  for (int h0 = 0; h0 < nh; h0 += 64) {
    const int h = h0 + lane;
    const int cnt = h < nh ? WG.cnt[h] : 0;
    const int x = wave_incl_scan(seg_round(cnt));
    if (h < nh) WG.off[h] = run + x - seg_round(cnt);
    run += __builtin_amdgcn_readlane(x, 63);
  }
  int base = 0;
  if (lane == 0) base = atomicAdd(&L.sbtop, run);
  base = __builtin_amdgcn_readlane(base, 0);
  if (base + run > sbcap) return 6;
  for (int h0 = 0; h0 < nh; h0 += 64) {
    const int h = h0 + lane;
    if (h < nh) {
      const int cnt = WG.cnt[h], sf = WG.sf[h];
      const unsigned long long km = WG.kmax[h];
      const int off = base + WG.off[h];
      WG.off[h] = off;
      seg_put(M.seg[sf], off, cnt);
      M.own[sf] = LK | (cnt ? ((~(unsigned)km) & 0xFFFFu) : HULL_NOPT);
    }
  }
  hl_sync();
  for (int t0 = 0; t0 < items; t0 += 64) {
    const int t = t0 + lane;
    if (t < items) {
      const int q = sq[t], code = sq[HNP + t];
      if (code) {
        HullPt e;
        e.x = Pr[3 * q]; e.y = Pr[3 * q + 1]; e.z = Pr[3 * q + 2]; e.q = q; e.pad = 0;
        sb[WG.off[(code & 2047) - 1] + (code >> 11)] = e;
      }
    }
  }
  // retire the region, release, queue the cone faces with outside points
  const int keep = nfree - used;
  for (int r0 = 0; r0 < R; r0 += 64) {
    const int r = r0 + lane;
    if (r < R && keep + r < HULL_FLCAP) W.freel[keep + r] = (unsigned short)region(r0, r);
  }
  nfree = min(keep + R, HULL_FLCAP);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int np = 0, qn = 0;
  for (int h0 = 0; h0 < nh; h0 += 64) {
    const int h = h0 + lane;
    int is = 0, sf = 0;
    if (h < nh) {
      sf = WG.sf[h];
      atomicAnd(&M.own[sf], ~LK);
      is = WG.cnt[h] > 0;
    }
    np += __popcll(__ballot(is));
    const int rc = hq_stage(W, mytail, qn, lb, lbn, is, sf, BG);
    if (rc) return rc;
  }
  mytail += qn;
  hl_sync();
  if (lane == 0) {
    atomicAdd(&L.work, np - 1);
    hl_cfence();
    hl_st(&W.tail, mytail);
  }
  return 0;
}

// The insertion loop of one wave.  L.work counts the queued faces plus the
// insertions in progress; the loop returns when it reaches 0, or on a
// failure (L.fail).  Conflicts are resolved wait-die: a wave that meets a
// face held by a higher-numbered wave waits for it, one that meets a face
// held by a lower-numbered wave backs off (releases everything, re-queues
// its face).  Waits only go from lower to higher wave numbers, so they end.
template <int NW>
__device__ __forceinline__ void hull_insert_mw(HullMemC& M, HullLdsC<NW>& L, const double* Pr, int n,
                                               double eps2, int* vpid, HullPt* sb, int sbcap,
                                               int* sq, int HNP, HullWide& WG, const HullBag& BG,
                                               unsigned long long* pstat) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned LK = 1u << (16 + w), RB = 1u << (24 + w);
  const unsigned OLDER = ((1u << w) - 1u) << 16;        // lock bits of lower-numbered waves
  HullWaveL& W = L.wl[w];
  const unsigned long long lt = (1ull << lane) - 1ull;
  int nfree = 0, mytail = hl_ld(&W.tail), attempts = 0, idle = 0;
  unsigned long long n_ins = 0, n_conf = 0, n_stale = 0, n_big = 0;
  constexpr int kF = HullMemC::kFaces, kV = HullMemC::kVerts;
  // a batch of entries taken from the own queue at once (lanes 0..lbn-1)
  int lb = -1, lbn = 0;
  // re-queue face f (wave-uniform; the entry keeps its unit of L.work)
  auto requeue = [&](int f) {
    int qn = 0;
    if (hq_stage(W, mytail, qn, lb, lbn, lane == 0, f, BG)) {
      if (lane == 0) atomicMax(&L.fail, 11);
      return;
    }
    if (qn) {
      mytail += qn;
      hl_sync();
      if (lane == 0) hl_st(&W.tail, mytail);
    }
  };
#ifdef LQRO_HULL_PROFILE
  unsigned long long wacc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long wlast = __builtin_amdgcn_s_memtime();
#endif
  unsigned maxr = 0;
  unsigned long long n_held = 0;
  for (;;) {
    if (hl_ld(&L.fail)) break;
    // (a) a face: from the local batch; refill it from the own queue (up to
    //     8 entries, one CAS), else take one entry of another wave's queue
    if (lbn == 0) {
      for (int tries = 0; tries < 16; ++tries) {
        int h = 0, t = 0;
        if (lane == 0) {
          h = hl_ld(&W.head);
          hl_cfence();
          t = hl_ld(&W.tail);
        }
        h = __builtin_amdgcn_readlane(h, 0);
        t = __builtin_amdgcn_readlane(t, 0);
        const int m = min(t - h, 8);
        if (m <= 0) break;
        int e = -1;
        if (lane < m) e = __hip_atomic_load(&W.q[(h + lane) % HULL_QCAP], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        hl_cfence();
        int ok = 0;
        if (lane == 0) ok = atomicCAS(&W.head, h, h + m) == h;
        if (__builtin_amdgcn_readlane(ok, 0)) { lb = e; lbn = m; break; }
      }
      if (lbn == 0) {
        int e = -1;
        if (lane == 0) {
          for (int k = 1; k < NW && e < 0; ++k) e = hq_pop(L.wl[(w + k) % NW]);
          if (e < 0) e = hq_bag_take(BG);
        }
        e = __builtin_amdgcn_readlane(e, 0);
        if (e >= 0) { lb = lane == 0 ? e : -1; lbn = 1; }
      }
      if (lbn > 0) {
        // drop retired faces and faces without outside points (a hint: the
        // lock below decides)
        int live = 0;
        if (lane < lbn) {
          if (lb >= hl_ld(&L.nf)) { atomicMax(&L.fail, 9); }
          else {
            const unsigned o = M.own[lb];
            live = (o >> 24) != 0xFFu && (o & 0xFFFFu) != HULL_NOPT;
          }
        }
        const unsigned long long b = __ballot(live);
        const int nl = __popcll(b);
        if (nl < lbn && lane == 0) atomicSub(&L.work, lbn - nl);
        int nlb = -1, k = 0;
        for (int j = 0; j < lbn; ++j)
          if (b & (1ull << j)) {
            const int v = __builtin_amdgcn_readlane(lb, j);
            if (lane == k) nlb = v;
            ++k;
          }
        lb = nlb;
        lbn = nl;
      }
    }
    WSTAMP(8);
    int f = -1;
    if (lbn > 0) {
      f = __builtin_amdgcn_readlane(lb, 0);
      lb = __shfl(lb, min(lane + 1, 63));
      --lbn;
    }
    if (f < 0) {
      int done = 0;
      if (lane == 0) done = hl_ld(&L.work) <= 0;
      if (__builtin_amdgcn_readlane(done, 0)) break;
      if (++idle > (1 << 24)) { if (lane == 0) atomicMax(&L.fail, 9); break; }   // bounded wait
      __builtin_amdgcn_s_sleep(2);
      WSTAMP(5);
      continue;
    }
    idle = 0;
    // (b) lock it.  Skip retired slots and faces without outside points.
    //     A face in another wave's visible region is dropped (retired, or
    //     re-queued by that wave if it backs off); one held around another
    //     wave's region is re-queued.
    unsigned old = 0;
    if (lane == 0) old = atomicOr(&M.own[f], LK);
    old = (unsigned)__builtin_amdgcn_readlane((int)old, 0);
    if ((old & 0x00FF0000u) || (old >> 24) == 0xFFu || (old & 0xFFFFu) == HULL_NOPT) {
      if (lane == 0) atomicAnd(&M.own[f], ~LK);
      if ((old & 0x00FF0000u) && (old >> 24) == 0u) {
        ++n_held;
        requeue(f);
        if (++n_stale > (1u << 22)) { if (lane == 0) atomicMax(&L.fail, 9); break; }
        __builtin_amdgcn_s_sleep(1);
      } else if (lane == 0) {
        atomicSub(&L.work, 1);
      }
      WSTAMP(9);
      continue;
    }
    if (++attempts > 16 * kV) { if (lane == 0) atomicMax(&L.fail, 9); break; }
    const int apex = (int)(old & 0xFFFFu);
    if (apex >= n) { if (lane == 0) atomicMax(&L.fail, 9); break; }
    const double p[3] = {Pr[3 * apex], Pr[3 * apex + 1], Pr[3 * apex + 2]};
    if (lane == 0) atomicOr(&M.own[f], RB);
    WSTAMP(0);
    if (p[0] + p[1] + p[2] == 1e300) atomicAdd(&L.fail, 0);   // profiling: wait for the apex load
    WSTAMP(10);
    // (c) visible region, grown over adjacency from f; lanes 0..2 lock and
    //     test the three neighbours of one region face at a time.  Lane r
    //     holds region face r.
    int rg = lane == 0 ? f : -1;
    int R = 1, conflict = 0;
    for (int r = 0; r < R; ++r) {
      const int g = r < 64 ? __builtin_amdgcn_readlane(rg, r) : WG.reg[r];
      int nb = -1, vis = 0, cf = 0;
      bool need = lane < 3;
      if (need) nb = M.fa[g][lane];
      for (int spin = 0;; ++spin) {
        if (need) {
          const unsigned o = atomicOr(&M.own[nb], LK);
          if (o & LK) {
            need = false;                                  // in the region or around it already
          } else if (!(o & 0x00FF0000u)) {
            need = false;
            vis = hl_beyond(M, nb, p, eps2, nullptr);
            if (vis) atomicOr(&M.own[nb], RB);
          } else {
            atomicAnd(&M.own[nb], ~LK);
            if (o & OLDER) { cf = 1; need = false; }       // held by a lower-numbered wave: back off
          }
        }
        if (__ballot(cf) || !__ballot(need)) break;
        if (spin > (1 << 20) || hl_ld(&L.fail)) { cf = 1; break; }
        __builtin_amdgcn_s_sleep(1);                       // wait for a higher-numbered wave
      }
      if (__ballot(cf)) { conflict = 1; break; }
      const unsigned long long b = __ballot(vis);
      const int n0 = __builtin_amdgcn_readlane(nb, 0), n1 = __builtin_amdgcn_readlane(nb, 1),
                n2 = __builtin_amdgcn_readlane(nb, 2);
      int k = R;
      const int nn3[3] = {n0, n1, n2};
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (b & (1ull << c)) {
          if (k < 64) { if (lane == k) rg = nn3[c]; }
          else if (lane == 0) WG.reg[k] = nn3[c];
          ++k;
        }
      R = k;
      if (R > HULL_WIDE - 3) break;
    }
    maxr = max(maxr, (unsigned)R);
    n_big += R > 32;
    if (R > HULL_WIDE - 3) { if (lane == 0) atomicMax(&L.fail, 2); break; }
    if (conflict) {
      // release the region and the faces around it; re-queue the region's
      // faces that have outside points (f with its unit of L.work, the
      // others with a new one: a popper may have dropped their entries)
      int nq = 0, qn = 0, full = 0;
      for (int r0 = 0; r0 < R; r0 += 64) {
        const int r = r0 + lane;
        int g = -1, is = 0;
        if (r < R) {
          g = r0 == 0 ? rg : WG.reg[r];
          for (int e = 0; e < 3; ++e) atomicAnd(&M.own[M.fa[g][e]], ~(LK | RB));
          const unsigned o = atomicAnd(&M.own[g], ~(LK | RB));
          is = (o & 0xFFFFu) != HULL_NOPT;
        }
        nq += __popcll(__ballot(is));
        if (hq_stage(W, mytail, qn, lb, lbn, is, g, BG)) { full = 1; break; }
      }
      if (full) { if (lane == 0) atomicMax(&L.fail, 11); break; }
      mytail += qn;
      hl_sync();
      if (lane == 0) {
        atomicAdd(&L.work, nq - 1);
        hl_cfence();
        hl_st(&W.tail, mytail);
      }
      ++n_conf;
      __builtin_amdgcn_s_sleep(4);
      WSTAMP(2);
      continue;
    }
    WSTAMP(1);
    // (d) horizon: region edges whose neighbour is not in the region, in
    //     (region order, edge) order, staged through LDS into lanes
    int nh = 0;
    if (R <= 64) {
      for (int b0 = 0; b0 < 3 * R; b0 += 64) {
        const int t = b0 + lane;
        const int g = __shfl(rg, min(t / 3, 63));
        int ha = 0, hb = 0, ho = 0, is = 0;
        if (t < 3 * R) {
          const int e = t % 3;
          ho = M.fa[g][e];
          if (!(M.own[ho] & RB)) { is = 1; ha = M.fv[g][e]; hb = M.fv[g][e == 2 ? 0 : e + 1]; }
        }
        const unsigned long long b = __ballot(is);
        const int pos = nh + __popcll(b & lt);
        if (is && pos < 64) {
          W.h_a[pos] = (unsigned short)ha; W.h_b[pos] = (unsigned short)hb; W.h_out[pos] = (unsigned short)ho;
        }
        nh += __popcll(b);
      }
    }
    if (R > 64 || nh > 64) {
      // ---- wide insertion: region / horizon lists in global scratch ----
      const int rc = hull_insert_wide(M, L, W, WG, Pr, vpid, sb, sbcap, sq, HNP, apex, p, eps2, R, rg,
                                      nfree, mytail, lb, lbn, BG, LK, RB);
      if (rc) { if (lane == 0) atomicMax(&L.fail, rc); break; }
      ++n_ins;
      WSTAMP(7);
      continue;
    }
    if (nh < 3) { if (lane == 0) atomicMax(&L.fail, 3); break; }
    hl_sync();
    const bool hl = lane < nh;
    int ha = 0, hb = 0, on = 0;
    if (hl) { ha = W.h_a[lane]; hb = W.h_b[lane]; on = W.h_out[lane]; }
    // (e) cone face slots (own retired slots first), the apex vertex
    const int used = min(nh, nfree);
    int sfb = 0, av = 0;
    if (lane == 0) { sfb = atomicAdd(&L.nf, nh - used); av = atomicAdd(&L.nvtx, 1); }
    sfb = __builtin_amdgcn_readlane(sfb, 0);
    av = __builtin_amdgcn_readlane(av, 0);
    if (sfb + (nh - used) > kF) { if (lane == 0) atomicMax(&L.fail, 4); break; }
    if (av >= kV) { if (lane == 0) atomicMax(&L.fail, 1); break; }
    int sf = 0;
    if (hl) sf = lane < used ? (int)W.freel[nfree - 1 - lane] : sfb + (lane - used);
    if (lane == 0) {
      M.vx[av][0] = p[0]; M.vx[av][1] = p[1]; M.vx[av][2] = p[2];
      vpid[av] = apex;
    }
    // cone neighbours: the edge leaving b (next) and the edge entering a (prev)
    int nx = -1, pv = -1;
    for (int k = 0; k < nh; ++k) {
      const int ak = __builtin_amdgcn_readlane(ha, k), bk = __builtin_amdgcn_readlane(hb, k);
      if (ak == hb) nx = k;
      if (bk == ha) pv = k;
    }
    if (__ballot(hl && (nx < 0 || pv < 0))) { if (lane == 0) atomicMax(&L.fail, 5); break; }
    const int sfn = __shfl(sf, max(nx, 0)), sfp = __shfl(sf, max(pv, 0));
    double cx = 0, cy = 0, cz = 0, ax = 0, ay = 0, az = 0, ci = 0, ce = 0;
    if (hl) {
      M.own[sf] = LK | HULL_NOPT;
      M.fv[sf][0] = (unsigned short)ha;
      M.fv[sf][1] = (unsigned short)hb;
      M.fv[sf][2] = (unsigned short)av;
      M.fa[sf][0] = (unsigned short)on;
      M.fa[sf][1] = (unsigned short)sfn;
      M.fa[sf][2] = (unsigned short)sfp;
      for (int e = 0; e < 3; ++e)
        if (M.fv[on][e] == hb && M.fv[on][e == 2 ? 0 : e + 1] == ha) M.fa[on][e] = (unsigned short)sf;
      // plane of the new face, as hl_normal / hl_beyond compute it
      const double* a = M.vx[ha];
      const double* bb = M.vx[hb];
      const double e1[3] = {bb[0] - a[0], bb[1] - a[1], bb[2] - a[2]};
      const double e2[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
      cx = e1[1] * e2[2] - e1[2] * e2[1];
      cy = e1[2] * e2[0] - e1[0] * e2[2];
      cz = e1[0] * e2[1] - e1[1] * e2[0];
      ax = a[0]; ay = a[1]; az = a[2];
      const double nn = cx * cx + cy * cy + cz * cz;
      ci = 1.0 / sqrt(nn);                            // for the distance key only
      ce = eps2 * nn;
      W.hcnt[lane] = 0;
      W.kmax[lane] = 0ull;
    }
    // the cone is linked: release the faces around the region and retire
    // the region now (its outside sets stay readable: retired slots are
    // reused only by this wave); the cone stays locked until its outside
    // sets are written
    hl_cfence();
    if (hl) atomicAnd(&M.own[on], ~LK);
    if (lane < R) M.own[rg] = HULL_DEAD;
    WSTAMP(3);
    // (f) the retired faces' outside points: first cone face they are beyond
    int roff = 0, rcnt = 0;
    if (lane < R) seg_get(M.seg[rg], roff, rcnt);
    const int rinc = wave_incl_scan(rcnt);
    const int total = __builtin_amdgcn_readlane(rinc, 63);
    hl_sync();
    // item t -> its region face's extent
    auto locate = [&](int t, int& src) {
      int base = 0, off0 = __builtin_amdgcn_readlane(roff, 0);
      for (int r = 0; r < R - 1; ++r) {
        const int inc = __builtin_amdgcn_readlane(rinc, r);
        const int o = __builtin_amdgcn_readlane(roff, r + 1);
        if (t >= inc) { base = inc; off0 = o; }
      }
      src = off0 + (t - base);
    };
    // first cone face (in horizon order) p is beyond; its key in *kd
    auto target = [&](const HullPt& e, bool act, int& tg, float& dv) {
      tg = -1;
      dv = 0.0f;
      bool pend = act && e.q != apex;
      for (int h = 0; h < nh; ++h) {
        if (!__ballot(pend)) break;
        const double c0 = hl_rl(cx, h), c1 = hl_rl(cy, h), c2 = hl_rl(cz, h);
        const double a0 = hl_rl(ax, h), a1 = hl_rl(ay, h), a2 = hl_rl(az, h), cc = hl_rl(ce, h);
        if (pend) {
          const double d = c0 * (e.x - a0) + c1 * (e.y - a1) + c2 * (e.z - a2);
          if (d > 0.0 && d * d > cc) { tg = h; dv = (float)(d * hl_rl(ci, h)); pend = false; }
        }
      }
    };
    int base = 0;
    if (total <= 4 * 64) {
      int tg[4], rk[4];
      HullPt pt[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        tg[c] = -1; rk[c] = 0; pt[c].q = -1;
        const int t = c * 64 + lane;
        if (c * 64 < total) {
          int src;
          locate(t, src);
          if (t < total) pt[c] = sb[src];
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c * 64 < total) {
          float dv;
          target(pt[c], c * 64 + lane < total, tg[c], dv);
          if (tg[c] >= 0) {
            rk[c] = atomicAdd(&W.hcnt[tg[c]], 1);
            atomicMax(&W.kmax[tg[c]], ((unsigned long long)__float_as_uint(dv) << 32) |
                                          (unsigned long long)(~(unsigned)pt[c].q));
          }
        }
      }
      hl_sync();
      const int cnt = hl ? W.hcnt[lane] : 0;
      const unsigned long long km = hl ? W.kmax[lane] : 0ull;
      const int cinc = wave_incl_scan(seg_round(cnt));
      const int tot = __builtin_amdgcn_readlane(cinc, 63);
      if (lane == 0) base = atomicAdd(&L.sbtop, tot);
      base = __builtin_amdgcn_readlane(base, 0);
      if (base + tot > sbcap) { if (lane == 0) atomicMax(&L.fail, 6); break; }
      const int off = base + cinc - seg_round(cnt);
      if (hl) {
        seg_put(M.seg[sf], off, cnt);
        M.own[sf] = LK | (cnt ? ((~(unsigned)km) & 0xFFFFu) : HULL_NOPT);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int o = __shfl(off, max(tg[c], 0));
        if (tg[c] >= 0) sb[o + rk[c]] = pt[c];
      }
    } else {
      // many points (early insertions): two passes through per-wave scratch
      for (int t0 = 0; t0 < total; t0 += 64) {
        const int t = t0 + lane;
        int src;
        locate(t, src);
        HullPt e;
        e.q = -1;
        if (t < total) e = sb[src];
        int tg;
        float dv;
        target(e, t < total, tg, dv);
        int code = 0;
        if (tg >= 0) {
          const int rk = atomicAdd(&W.hcnt[tg], 1);
          atomicMax(&W.kmax[tg], ((unsigned long long)__float_as_uint(dv) << 32) |
                                     (unsigned long long)(~(unsigned)e.q));
          code = (rk << 7) | (tg + 1);
        }
        if (t < total) { sq[t] = e.q; sq[HNP + t] = code; }
      }
      hl_sync();
      const int cnt = hl ? W.hcnt[lane] : 0;
      const unsigned long long km = hl ? W.kmax[lane] : 0ull;
      const int cinc = wave_incl_scan(seg_round(cnt));
      const int tot = __builtin_amdgcn_readlane(cinc, 63);
      if (lane == 0) base = atomicAdd(&L.sbtop, tot);
      base = __builtin_amdgcn_readlane(base, 0);
      if (base + tot > sbcap) { if (lane == 0) atomicMax(&L.fail, 6); break; }
      const int off = base + cinc - seg_round(cnt);
      if (hl) {
        seg_put(M.seg[sf], off, cnt);
        M.own[sf] = LK | (cnt ? ((~(unsigned)km) & 0xFFFFu) : HULL_NOPT);
      }
      for (int t0 = 0; t0 < total; t0 += 64) {
        const int t = t0 + lane;
        int code = 0, q = 0;
        if (t < total) { q = sq[t]; code = sq[HNP + t]; }
        const int tg = (code & 127) - 1;
        const int o = __shfl(off, max(tg, 0));
        if (code) {
          HullPt e;
          e.x = Pr[3 * q]; e.y = Pr[3 * q + 1]; e.z = Pr[3 * q + 2]; e.q = q; e.pad = 0;
          sb[o + (code >> 7)] = e;
        }
      }
    }
    WSTAMP(4);
    const int cnt_mine = hl ? W.hcnt[lane] : 0;
    // (g) retire the region (slots to this wave's list), then, once this
    //     wave's global stores are done, release the cone and the faces
    //     around it and queue the cone faces that have outside points
    {
      const int keep = nfree - used;
      if (lane < R && keep + lane < HULL_FLCAP) W.freel[keep + lane] = (unsigned short)rg;
      nfree = min(keep + R, HULL_FLCAP);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (hl) atomicAnd(&M.own[sf], ~LK);
    {
      const int is = hl && cnt_mine > 0;
      const int np = __popcll(__ballot(is));
      int qn = 0;
      if (hq_stage(W, mytail, qn, lb, lbn, is, sf, BG)) { if (lane == 0) atomicMax(&L.fail, 11); break; }
      mytail += qn;
      hl_sync();
      if (lane == 0) {
        atomicAdd(&L.work, np - 1);                        // before the entries are visible
        hl_cfence();
        hl_st(&W.tail, mytail);
      }
    }
    ++n_ins;
    WSTAMP(6);
  }
#ifdef LQRO_HULL_PROFILE
  if (lane == 0 && pstat)
    for (int k = 0; k < 12; ++k) atomicAdd(&pstat[32 + 2 * 4096 + 16 - 10 + k], wacc[k]);
  if (lane == 0 && pstat) {
    atomicAdd(&pstat[0], n_ins);
    atomicAdd(&pstat[1], n_conf);
    atomicAdd(&pstat[2], n_stale);
    atomicMax(&pstat[3], (unsigned long long)maxr);
    atomicAdd(&pstat[4], n_big);
    atomicAdd(&pstat[32 + 2 * 4096 + 16 - 10 + 15], n_held);
  }
#else
  (void)n_ins; (void)n_conf; (void)n_stale; (void)pstat; (void)maxr; (void)n_big; (void)n_held;
#endif
}

template <int NW>
__device__ __forceinline__ void hull_body_mw(const HullArgs& A, HullMemC& M, HullLdsC<NW>& L) {
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
#ifdef LQRO_HULL_PROFILE
  unsigned long long prof_acc[16] = {0};
  unsigned long long prof_last = __builtin_amdgcn_s_memtime();
#endif
  const int HNP = A.H * A.NP;
  const int hb = A.block_base + blockIdx.x;                   // scratch slot
  double* Pr = A.scratch + (size_t)hb * HNP * 6;              // rounded points
  double* Pf = Pr + (size_t)HNP * 3;                          // full-precision points
  int* isc = A.iscratch + (size_t)hb * HNP * 2 * HULL_SCR_WAVES;
  float* td = A.fscratch + (size_t)hb * HNP;
  HullPt* sb = A.sb + (size_t)hb * HNP * HULL_SBMULT;
  const int sbcap = HNP * HULL_SBMULT;
  int* vpid = A.vpid + (size_t)hb * HULL_VG_STRIDE;
  const HullBag BG{A.bag + (size_t)hb * HULL_BAGCAP, &L.gb_head, &L.gb_tail};
  if (tid == 0) L.gb_tail = 0;
  for (;;) {
    const int slot = hull_take_job(A, L, false);
    if (slot < 0) break;
    const int lrow = slot / A.npr, jj = A.nbr_list ? A.nbr_list[slot] : slot % A.npr;
    const int i = A.row_begin + lrow * A.row_stride;
    const int j = jj < i ? jj : jj + 1;
    const double* xi = A.x + (size_t)i * A.X;
    const double* xj = A.x + (size_t)j * A.X;
    const double* Ti = A.T + (A.per_agent ? (size_t)i * A.H * 9 : 0);
    const double* Ni = A.NCF + (A.per_agent ? (size_t)i * A.H * 3 * A.X : 0);
    const double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};
#ifdef LQRO_HULL_PROFILE
    const unsigned long long job_t0 = __builtin_amdgcn_s_memtime();
#endif
    HSTAMP(15);
    const int n = hull_points(A, L, Ti, Ni, xi, xj, vrel, Pr, Pf);
    const double eps2 = L.eps * L.eps;
    HSTAMP(0);
    if (!L.fail) {
      hull_tetra(M, L, Pr, n, L.eps, eps2, vpid);
      hl_bar();
    }
    if (!L.fail) {
      // 4. outside sets of the tetrahedron's faces; the faces go to the
      //    wave queues round-robin
      int* th = isc;
      if (tid < 4) { L.hcnt[tid] = 0; L.kmax4[tid] = 0ull; }
      if (tid < NW) { L.wl[tid].head = 0; L.wl[tid].tail = 0; }
      if (tid == 0) { L.gb_head = 0; L.gb_tail = 0; }
      hl_bar();
      for (int q = tid; q < n; q += blockDim.x) {
        int c = -1;
        double dd = 0.0;
        if (q != L.init[0] && q != L.init[1] && q != L.init[2] && q != L.init[3]) {
          const double p[3] = {Pr[3 * q], Pr[3 * q + 1], Pr[3 * q + 2]};
          for (int f = 0; f < 4; ++f)
            if (hl_beyond(M, f, p, eps2, &dd)) { c = f; break; }
        }
        th[q] = c;
        td[q] = (float)dd;
        if (c >= 0) atomicAdd(&L.hcnt[c], 1);
      }
      hl_bar();
      if (tid == 0) {
        int o = 0;
        for (int f = 0; f < 4; ++f) {
          seg_put(M.seg[f], o, L.hcnt[f]);
          L.hoff[f] = o;
          o += seg_round(L.hcnt[f]);
        }
        L.sbtop = o;
        L.nf = 4;
        L.nvtx = 4;
        L.work = 0;
      }
      hl_bar();
      for (int q = tid; q < n; q += blockDim.x) {
        const int c = th[q];
        if (c < 0) continue;
        HullPt e;
        e.x = Pr[3 * q]; e.y = Pr[3 * q + 1]; e.z = Pr[3 * q + 2]; e.q = q; e.pad = 0;
        sb[atomicAdd(&L.hoff[c], 1)] = e;
        const unsigned long long key =
            ((unsigned long long)__float_as_uint(td[q]) << 32) | (unsigned long long)(~(unsigned)q);
        atomicMax(&L.kmax4[c], key);
      }
      hl_bar();
      if (tid == 0) {
        for (int f = 0; f < 4; ++f) {
          M.own[f] = L.hcnt[f] ? ((~(unsigned)L.kmax4[f]) & 0xFFFFu) : HULL_NOPT;
          if (L.hcnt[f]) {
            HullWaveL& Q = L.wl[f % NW];
            Q.q[Q.tail++] = (unsigned short)f;
            L.work++;
          }
        }
      }
      hl_bar();
      HSTAMP(1);
      // 5. quickhull, every wave inserting
      hull_insert_mw<NW>(M, L, Pr, n, eps2, vpid, sb, sbcap, isc + (size_t)wave * 2 * HNP, HNP,
                         A.wide[(size_t)hb * NW + wave], BG,
#ifdef LQRO_HULL_PROFILE
                         A.prof ? A.prof + 10 : nullptr
#else
                         nullptr
#endif
      );
      hl_bar();
      HSTAMP(6);
    }
    hl_bar();
    // the bag's used prefix back to empty (-1) for the next job
    for (int q = tid; q < min(L.gb_tail, HULL_BAGCAP); q += blockDim.x) BG.slot[q] = -1;
    if (tid == 0) L.gb_tail = 0;
    HSTAMP(8);
    // 6. facet selection
    const int nf = L.nf;
    if (A.ext_facets && !L.fail)
      for (int f = tid; f < nf; f += blockDim.x)
        if ((M.own[f] >> 24) != 0xFFu) {
          const int k = atomicAdd(A.ext_nf, 1);
          if (k < A.ext_max)
            for (int e = 0; e < 3; ++e) A.ext_facets[3 * k + e] = vpid[M.fv[f][e]];
        }
    hull_select(A, M, L, Pr, Pf, vpid, nf, [&](int f) { return (M.own[f] >> 24) != 0xFFu; }, xi, vrel,
                slot, false);
    HSTAMP(9);
#ifdef LQRO_HULL_PROFILE
    if (tid == 0 && A.prof && L.job < 2048) {
      const int pj = 32 + 2 * L.job;
      A.prof[pj] = __builtin_amdgcn_s_memtime() - job_t0;
      A.prof[pj + 1] = (unsigned long long)L.nvtx | ((unsigned long long)n << 20) |
                       ((unsigned long long)L.fail << 40) | ((unsigned long long)slot << 44);
    }
#endif
  }
#ifdef LQRO_HULL_PROFILE
  if (tid == 0 && A.prof)
    for (int k = 0; k < 10; ++k) atomicAdd(&A.prof[k], prof_acc[k]);
  if (tid == 0 && A.prof) atomicAdd(&A.prof[15], prof_acc[15]);
#endif
}

// ---------------------------------------------------------------------------
// k_hull_big: one inserting wave, topology in global memory
// ---------------------------------------------------------------------------
template <class Mem, class LT>
__device__ __forceinline__ void hull_body(const HullArgs& A, Mem& M, LT& L, bool big) {
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
#ifdef LQRO_HULL_PROFILE
  unsigned long long prof_acc[16] = {0};
  unsigned long long prof_last = __builtin_amdgcn_s_memtime();
#endif
  const int HNP = A.H * A.NP;
  const int hb = A.block_base + blockIdx.x;                   // scratch slot
  double* Pr = A.scratch + (size_t)hb * HNP * 6;    // rounded points
  double* Pf = Pr + (size_t)HNP * 3;                         // full-precision points
  int* tq = A.iscratch + (size_t)hb * HNP * 2 * HULL_SCR_WAVES;   // moved point ids
  int* th = tq + HNP;                                        // their target cone face
  float* td = A.fscratch + (size_t)hb * HNP;         // distance beyond it
  HullPt* sb = A.sb + (size_t)hb * HNP * HULL_SBMULT;
  const int sbcap = HNP * HULL_SBMULT;
  // per face: furthest outside point (dist bits << 32) | ~q, outside-set extent
  unsigned long long* fbest = A.fbest + (size_t)hb * HULL_FB_STRIDE;
  int* vpid = A.vpid + (size_t)hb * HULL_VG_STRIDE;
  int* stk = A.stack + (size_t)hb * HNP * HULL_STKMULT;
  const int stkcap = HNP * HULL_STKMULT;

  const bool retryq = big && !A.big_main;
  for (;;) {
    const int slot = hull_take_job(A, L, retryq);
    if (slot < 0) break;
    const int lrow = slot / A.npr, jj = A.nbr_list ? A.nbr_list[slot] : slot % A.npr;
    const int i = A.row_begin + lrow * A.row_stride;
    const int j = jj < i ? jj : jj + 1;
    const double* xi = A.x + (size_t)i * A.X;
    const double* xj = A.x + (size_t)j * A.X;
    const double* Ti = A.T + (A.per_agent ? (size_t)i * A.H * 9 : 0);
    const double* Ni = A.NCF + (A.per_agent ? (size_t)i * A.H * 3 * A.X : 0);
    const double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};
#ifdef LQRO_HULL_PROFILE
    const unsigned long long job_t0 = __builtin_amdgcn_s_memtime();
#endif

    HSTAMP(15);
    const int n = hull_points(A, L, Ti, Ni, xi, xj, vrel, Pr, Pf);
    const double eps = L.eps;
    const double eps2 = eps * eps;

    HSTAMP(0);
    if (!L.fail) {
      hull_tetra(M, L, Pr, n, L.eps, eps2, vpid);
      if (tid == 0 && !L.fail) {
        for (int f = 0; f < 4; ++f) M.alive[f] = 1;
        L.nvtx = 4;
        L.nf = 4;
        L.nfree = 0;
      }
      hl_bar();
    }

    if (!L.fail) {
      // 4. outside sets of the tetrahedron's faces
      if (tid < 4) { fbest[tid] = 0ull; L.hcnt[tid] = 0; }
      if (tid == 0) { L.sbtop = 0; L.sp = 0; L.qh = 0; L.it = 0; }
      hl_bar();
      for (int q = tid; q < n; q += blockDim.x) {
        int c = -1;
        double dd = 0.0;
        if (q != L.init[0] && q != L.init[1] && q != L.init[2] && q != L.init[3]) {
          const double p[3] = {Pr[3 * q], Pr[3 * q + 1], Pr[3 * q + 2]};
          for (int f = 0; f < 4; ++f)
            if (hl_beyond(M, f, p, eps2, &dd)) { c = f; break; }
        }
        th[q] = c;
        td[q] = (float)dd;
        if (c >= 0) atomicAdd(&L.hcnt[c], 1);
      }
      hl_bar();
      if (tid == 0) {
        int o = 0;
        for (int f = 0; f < 4; ++f) {
          seg_put(M.seg[f], o, L.hcnt[f]);
          L.hoff[f] = o;
          o += L.hcnt[f];
          M.vst[f] = 0;
        }
        for (int f = 0; f < 4; ++f)
          if (L.hcnt[f] > 0) stk[L.sp++] = f;
        L.sbtop = o;
      }
      hl_bar();
      for (int q = tid; q < n; q += blockDim.x) {
        const int c = th[q];
        if (c < 0) continue;
        HullPt e;
        e.x = Pr[3 * q]; e.y = Pr[3 * q + 1]; e.z = Pr[3 * q + 2]; e.q = q; e.pad = 0;
        sb[atomicAdd(&L.hoff[c], 1)] = e;
        const unsigned long long key =
            ((unsigned long long)__float_as_uint(td[q]) << 32) | (unsigned long long)(~(unsigned)q);
        atomicMax(&fbest[c], key);
      }
      hl_bar();

      HSTAMP(1);
      // Insertions run on wave 0 alone (the other waves helped with the
      // points and the initial hull and wait for the facet selection).
      if (wave == 0) {
      // 5. quickhull: take the oldest live face with outside points (FIFO
      //    work queue), insert its furthest point.  The loop keeps its
      //    control state in (wave-uniform) registers, passes lists between
      //    lanes with ballots, readlane and DPP scans.
      int qh = 0, sp = L.sp, nvtx = L.nvtx, it = 0, nf = L.nf, nfree = L.nfree, sbtop = L.sbtop;
      int fail = 0;
      const unsigned long long lt = (1ull << tid) - 1ull;
      for (;;) {
        if (qh == sp) break;
        const int f = stk[qh];
        ++qh;
        // stale entries: the face was retired (its slot maybe reused by a
        // face without outside points) after it was pushed
        const unsigned long long key = fbest[f];
        if (!M.alive[f] || key == 0ull) continue;
        const int apex = (int)(~(unsigned)(key & 0xFFFFFFFFull));
        if (apex < 0 || apex >= n || it >= 4 * Mem::kVerts) { fail = 9; break; }
        if (nvtx >= Mem::kVerts) { fail = 1; break; }
        const int av = nvtx++;
        const unsigned short stamp = (unsigned short)(++it);
        const double p[3] = {Pr[3 * apex], Pr[3 * apex + 1], Pr[3 * apex + 2]};
        if (tid == 0) {
          M.vx[av][0] = p[0]; M.vx[av][1] = p[1]; M.vx[av][2] = p[2];
          vpid[av] = apex;
          M.vst[f] = stamp;
        }
        hl_sync();
        // (a) visible region over adjacency from f
        int rg = tid == 0 ? f : -1;
        if (tid == 0) L.region[0] = (unsigned short)f;
        int R = 1;
        for (int r = 0; r < R; ++r) {
          const int g = r < 64 ? __builtin_amdgcn_readlane(rg, r) : (int)L.region[r];
          int nb = -1, vis = 0;
          if (tid < 3) {
            nb = M.fa[g][tid];
            vis = (M.vst[nb] != stamp) && hl_beyond(M, nb, p, eps2, nullptr);
          }
          const unsigned long long b = __ballot(vis);
          if (vis) {
            const int pos = R + __popcll(b & lt);
            if (pos < LT::kRegion) { L.region[pos] = (unsigned short)nb; M.vst[nb] = stamp; }
          }
          const int n0 = __builtin_amdgcn_readlane(nb, 0), n1 = __builtin_amdgcn_readlane(nb, 1),
                    n2 = __builtin_amdgcn_readlane(nb, 2);
          int k = R;
          if (b & 1ull) { if (tid == k) rg = n0; ++k; }
          if (b & 2ull) { if (tid == k) rg = n1; ++k; }
          if (b & 4ull) { if (tid == k) rg = n2; ++k; }
          R = k;
          if (R > LT::kRegion) break;
          hl_sync();
        }
        if (R > LT::kRegion) { fail = 2; break; }
        // (b) horizon
        int nh = 0;
        for (int b0 = 0; b0 < 3 * R; b0 += 64) {
          const int t = b0 + tid;
          int ha = 0, hb2 = 0, ho = 0, is = 0;
          if (t < 3 * R) {
            const int g = L.region[t / 3], e = t % 3;
            ho = M.fa[g][e];
            if (M.vst[ho] != stamp) { is = 1; ha = M.fv[g][e]; hb2 = M.fv[g][(e + 1) % 3]; }
          }
          const unsigned long long b = __ballot(is);
          const int pos = nh + __popcll(b & lt);
          if (is && pos < LT::kHorizon) {
            L.h_a[pos] = (unsigned short)ha; L.h_b[pos] = (unsigned short)hb2; L.h_out[pos] = (unsigned short)ho;
          }
          nh += __popcll(b);
        }
        if (nh > LT::kHorizon || nh < 3) { fail = 3; break; }
        const int nf0 = nf, nfree0 = nfree;
        if (nf0 + max(0, nh - nfree0) > Mem::kFaces) { fail = 4; break; }
        // (c) cone face slots (retired slots first) and the vertex -> edge map
        for (int h = tid; h < nh; h += 64) {
          const int sf = h < nfree0 ? M.freel[nfree0 - 1 - h] : nf0 + (h - nfree0);
          L.h_new[h] = (unsigned short)sf;
          M.vmap[L.h_a[h]] = (unsigned short)h;
          L.hcnt[h] = 0;
        }
        hl_sync();
        // (d) cone faces (a, b, apex): adjacency, outer neighbours, planes
        int bad = 0;
        for (int h = tid; h < nh; h += 64) {
          const int sf = L.h_new[h];
          const int ha = L.h_a[h], hb2 = L.h_b[h], on = L.h_out[h];
          const int k = M.vmap[hb2];                   // edge leaving b
          M.fv[sf][0] = (unsigned short)ha;
          M.fv[sf][1] = (unsigned short)hb2;
          M.fv[sf][2] = (unsigned short)av;
          M.fa[sf][0] = (unsigned short)on;
          M.fa[sf][1] = L.h_new[k];                    // across (b, apex)
          M.fa[L.h_new[k]][2] = (unsigned short)sf;    // k's (apex, a_k = b)
          M.vst[sf] = 0;
          for (int e = 0; e < 3; ++e)
            if (M.fv[on][e] == hb2 && M.fv[on][(e + 1) % 3] == ha) M.fa[on][e] = (unsigned short)sf;
          if (L.h_a[k] != hb2) bad = 1;
          const double* a = M.vx[ha];
          const double* bb = M.vx[hb2];
          const double e1[3] = {bb[0] - a[0], bb[1] - a[1], bb[2] - a[2]};
          const double e2[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
          const double nx = e1[1] * e2[2] - e1[2] * e2[1];
          const double ny = e1[2] * e2[0] - e1[0] * e2[2];
          const double nz = e1[0] * e2[1] - e1[1] * e2[0];
          double* cp = L.cn[h];
          cp[0] = nx; cp[1] = ny; cp[2] = nz;
          cp[3] = a[0]; cp[4] = a[1]; cp[5] = a[2];
          const double nn = nx * nx + ny * ny + nz * nz;
          cp[6] = 1.0 / sqrt(nn);                      // for the distance key only
          cp[7] = eps2 * nn;
          fbest[sf] = 0ull;
        }
        if (__ballot(bad)) { fail = 5; break; }
        // (e) the retired faces' outside points, through LDS + scratch
        for (int r = tid; r < R; r += 64) {
          int so, sc;
          seg_get(M.seg[L.region[r]], so, sc);
          L.roff[r] = so;
          L.rcnt[r] = sc;
        }
        hl_sync();
        int run0 = 0;
        for (int r0 = 0; r0 < R; r0 += 64) {
          const int r = r0 + tid;
          const int v = r < R ? L.rcnt[r] : 0;
          const int x = wave_incl_scan(v);
          if (r < R) L.rpre[r] = run0 + x - v;
          run0 += __builtin_amdgcn_readlane(x, 63);
        }
        if (tid == 0) L.rpre[R] = run0;
        hl_sync();
        const int tot2 = run0;
        for (int t = tid; t < tot2; t += 64) {
          int lo = 0, hi = R - 1;
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (L.rpre[mid] <= t) lo = mid; else hi = mid - 1;
          }
          const HullPt e = sb[L.roff[lo] + (t - L.rpre[lo])];
          const int q = e.q;
          int tgt = -1;
          float dd = 0.0f;
          if (q != apex) {
            const double x0 = e.x, x1 = e.y, x2 = e.z;
            for (int h = 0; h < nh; ++h) {
              const double* cp = L.cn[h];
              const double d = cp[0] * (x0 - cp[3]) + cp[1] * (x1 - cp[4]) + cp[2] * (x2 - cp[5]);
              if (d > 0.0 && d * d > cp[7]) { tgt = h; dd = (float)(d * cp[6]); break; }
            }
          }
          tq[t] = q;
          th[t] = tgt;
          td[t] = dd;
          if (tgt >= 0) atomicAdd(&L.hcnt[tgt], 1);
        }
        hl_sync();
        int run = sbtop;
        for (int h0 = 0; h0 < nh; h0 += 64) {
          const int h = h0 + tid;
          const int v = h < nh ? L.hcnt[h] : 0;
          const int x = wave_incl_scan(v);
          if (h < nh) {
            seg_put(M.seg[L.h_new[h]], run + x - v, v);
            L.hoff[h] = run + x - v;
          }
          run += __builtin_amdgcn_readlane(x, 63);
        }
        if (run > sbcap) { fail = 6; break; }
        sbtop = run;
        hl_sync();
        for (int t = tid; t < tot2; t += 64) {
          const int h = th[t];
          if (h < 0) continue;
          const int q = tq[t];
          HullPt e;
          e.x = Pr[3 * q]; e.y = Pr[3 * q + 1]; e.z = Pr[3 * q + 2]; e.q = q; e.pad = 0;
          sb[atomicAdd(&L.hoff[h], 1)] = e;
          const unsigned long long k2 =
              ((unsigned long long)__float_as_uint(td[t]) << 32) | (unsigned long long)(~(unsigned)q);
          atomicMax(&fbest[L.h_new[h]], k2);
        }
        // (f) retire the region, commit the cone, push the cone faces that
        //     have outside points (in horizon order)
        const int used = min(nh, nfree0);
        for (int r = tid; r < R; r += 64) {
          const int g = L.region[r];
          M.alive[g] = 0;
          M.freel[nfree0 - used + r] = (unsigned short)g;
        }
        int npush = 0;
        for (int h0 = 0; h0 < nh; h0 += 64) {
          const int h = h0 + tid;
          int is = 0;
          if (h < nh) {
            M.alive[L.h_new[h]] = 1;
            is = L.hcnt[h] > 0;
          }
          const unsigned long long b = __ballot(is);
          const int pos = sp + npush + __popcll(b & lt);
          if (is && pos < stkcap) stk[pos] = L.h_new[h];
          npush += __popcll(b);
        }
        if (sp + npush > stkcap) { fail = 6; break; }
        nfree = nfree0 - used + R;
        nf = nf0 + (nh - used);
        sp += npush;
        hl_sync();
      }
      if (tid == 0) {
        L.nf = nf; L.nfree = nfree; L.nvtx = nvtx; L.sbtop = sbtop; L.sp = sp;
        if (fail) L.fail = fail;
      }
      }
      hl_bar();
    }
    hl_bar();
    HSTAMP(8);
    hull_select(A, M, L, Pr, Pf, vpid, L.nf, [&](int f) { return M.alive[f] != 0; }, xi, vrel, slot, big);
    HSTAMP(9);
#ifdef LQRO_HULL_PROFILE
    if (tid == 0 && A.prof && L.job < 2048) {
      const int pj = 32 + 2 * (2048 + L.job);
      A.prof[pj] = __builtin_amdgcn_s_memtime() - job_t0;
      A.prof[pj + 1] = (unsigned long long)L.nvtx | ((unsigned long long)n << 20) |
                       ((unsigned long long)L.fail << 40) | ((unsigned long long)slot << 44);
    }
#endif
  }
#ifdef LQRO_HULL_PROFILE
  if (tid == 0 && A.prof)
    for (int k = 0; k < 10; ++k) atomicAdd(&A.prof[k], prof_acc[k]);
#endif
  (void)wave;
}

#ifdef LQRO_HULL_TU   // defined once, in lqro_kern_hull.hip
__global__ void __launch_bounds__(HULL_CTHREADS) k_hull(HullArgs A) {
  __shared__ HullLdsC<HULL_CWAVES> L;
  __shared__ HullMemC M;
  hull_body_mw<HULL_CWAVES>(A, M, L);
}

__global__ void __launch_bounds__(HULL_THREADS) k_hull_big(HullArgs A) {
  __shared__ HullLdsBig L;
  HullMemBig& M = reinterpret_cast<HullMemBig*>(A.bigmem)[blockIdx.x];
  hull_body(A, M, L, true);
}
#endif

}  // namespace lqro
