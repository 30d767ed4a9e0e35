// lqro_qhull3.hpp — k_qhull: Qhull 2019.1's build (the restatement in
// lqro_qhull.hpp, which stays as k_qhull_big, the fallback for builds beyond
// this kernel's caps), laid out for the CU instead of transcribed.  The build
// is one long chain of dependent steps per pair, so its speed is the latency
// of each step; this layout keeps that chain in LDS:
//
//  * the facets' hot fields — plane, neighbours, flags, list key, outside-set
//    count and furthest point — live in LDS for the first Q3_FL facet slots
//    (a whole CU's LDS, one wave per CU); slots beyond spill to a 64-byte
//    global record.  Vertices (as point ids), outside-set offsets and
//    furthest distances, touched once per insertion in parallel, stay in
//    global memory;
//  * no linked facet list: Qhull's list order is the order facets were
//    appended (qh_appendfacet), so each facet carries a key — its position in
//    that order (0 for the facet qh_furthestnext prepends, a fresh key when
//    qh_partitionpoint moves an old facet behind the new ones) — and
//    qh_nextfurthest's cursor is a queue of the facets that received outside
//    points, in key order, validated 64 entries at a time;
//  * qh_findhorizon's breadth-first search runs a level at a time over the
//    lanes (same visiting order: a facet is taken by the first visible facet
//    in queue order that reaches it); qh_makenew_simplicial runs one horizon
//    ridge per lane (creation order = the ridges in visible-list order); new
//    facets reuse the visible facets' slots;
//  * outside-set entries are point ids (4 B: the sets' footprint stays in
//    L2), their coordinates read from Pr when a set is re-partitioned (wave
//    2's prefetch does both loads for the usual one-chunk sequence), and the
//    partition sequence is read straight from the visible facets' sets;
//  * the point search keeps Qhull's sequential semantics as lqro_qhull.hpp
//    does (order-dependent state changes applied at their point, the rest of
//    the sequence re-evaluated), and counts each point into its destination
//    as soon as its result is final.
#pragma once
#include "lqro_qhull.hpp"
#include "lqro_lp.hpp"

namespace lqro {

#ifndef Q3_NEWCAP
#define Q3_NEWCAP 128     // new facets of one insertion (more: the pair goes to k_qhull_big)
#endif
#ifndef Q3_VISCAP
#define Q3_VISCAP 192     // visible facets of one insertion (the crowded 30 m swarm's widest: 166)
#endif
#define Q3_MOVCAP 16      // old facets moved / receiving points in one partition
#define Q3_HZCAP 24       // facets one point's horizon walk visits
#define Q3_COPCAP 8       // its coplanar facet set
#define Q3_FSTK 512       // free facet slots kept for reuse (more are left unused)
#define Q3_ND (Q3_NEWCAP + Q3_MOVCAP)
#define Q3_WAVES 4        // wave 0 builds, 1 speculates, 2 prefetches; 1-3 locate a long sequence's chunks
#define Q3_HR 4           // chunk results held for wave 0 (chunk k in buffer k % Q3_HR)
// poll intervals (s_sleep units of 64 clocks): wave 0 waiting on wave 1, and
// the idle loops of waves 1 and 2
#ifndef Q3_W0_SLEEP
#define Q3_W0_SLEEP 1
#endif
#ifndef Q3_W1_SLEEP
#define Q3_W1_SLEEP 1
#endif
#ifndef Q3_W2_SLEEP
#define Q3_W2_SLEEP 1
#endif
#ifndef Q3_FL
#define Q3_FL 2240        // facet slots with their hot fields in LDS (the rest of 160 KB)
#endif
#define Q3_PROF_RETRY (32 + 2 * 4096 + 16)   // profile words: builds handed to k_qhull_big (16)
#ifdef LQRO_QHULL_PROFILE
#define Q3_CAPBIT(b) (b)   // which cap sent a build to k_qhull_big (scripts/qhull_prof.py)
#else
#define Q3_CAPBIT(b) 0
#endif

struct Q3G {              // a facet slot >= Q3_FL, 64 B
  double pl[4];
  int nb[3];
  int fa;                 // QF_* | new-facet index << 8
  unsigned key;
  unsigned cc;            // outside set: count | furthest point << 16
  int pad[2];
};

struct Q3V {              // a facet's vertices: rounded points and point ids, Fv order (newest first)
  double p[9];
  double pad;
  int id[4];
};

struct Q3W {
  double* Pr;             // 3 HNP rounded points (qconvex's input)
  double* Pf;             // 3 HNP full precision
  Q3G* G;                 // FC - Q3_FL spilled slots
  Q3V* vv;                // FC: vertices
  double* ncoord;         // 9 Q3_NEWCAP: the new facets' ridge and opposite points (a cone too wide for registers)
  int* soff;              // FC: outside set offset in sb
  double* fdist;          // FC: furthest outside distance
  int* sb;                // SB outside-set entries: point ids (coordinates from Pr)
  int* pq;                // HNP: qh_partitionall's remainder
  int* pdst;              // HNP: partition sequence -> destination index
  double* pdd;            // HNP: its distance
  double* ncoord2;        // 9 Q3_NEWCAP: the speculated cone's ridge and opposite points (wave 1)
  unsigned* mark2;        // FC: wave 1's visit epochs of slots >= Q3_FL
  unsigned* ctr;          // wave 1's last epoch (across jobs; zeroed with the scratch)
  unsigned short* hvis;   // (Q3_WAVES - 1) x Q3_HZCAP x 64: the helper waves' visited-facet columns (Q3Col)
  int* hcop;              // (Q3_WAVES - 1) x Q3_COPCAP x 64: their coplanar-set columns
  int* fq;                // QC: facets that received points, key order
  unsigned* fqk;          // QC: their key then
  HullPt* fqc;            // QC: their furthest point then (q = -1: not recorded)
  int FC, SB, HNP, QC;
};

__host__ __device__ inline size_t q3_align(size_t b) { return (b + 255) & ~(size_t)255; }

__host__ __device__ inline size_t q3_worker_bytes(int HNP) {
  const size_t FC = 2 * (size_t)HNP + Q3_NEWCAP + 16, SB = (size_t)QH_SBMULT * HNP, QC = 4 * (size_t)HNP + 64;
  const size_t NG = FC > Q3_FL ? FC - Q3_FL : 1;
  return q3_align(24 * (size_t)HNP) * 2 + q3_align(64 * NG) + q3_align(96 * FC) + q3_align(72 * Q3_NEWCAP) +
         q3_align(4 * FC) +
         q3_align(8 * FC) + q3_align(4 * SB) + q3_align(4 * (size_t)HNP) * 2 + q3_align(8 * (size_t)HNP) +
         q3_align(4 * QC) * 2 + q3_align(32 * QC) + q3_align(72 * Q3_NEWCAP) + q3_align(4 * FC) + 256 +
         q3_align(2 * (Q3_WAVES - 1) * Q3_HZCAP * 64) + q3_align(4 * (Q3_WAVES - 1) * Q3_COPCAP * 64);
}

__device__ inline Q3W q3_worker(char* base, int HNP) {
  Q3W W;
  W.HNP = HNP;
  W.FC = 2 * HNP + Q3_NEWCAP + 16;
  W.SB = QH_SBMULT * HNP;
  W.QC = 4 * HNP + 64;
  const size_t NG = W.FC > Q3_FL ? W.FC - Q3_FL : 1;
  char* p = base;
  auto take = [&](size_t bytes) { char* r = p; p += q3_align(bytes); return r; };
  W.Pr = reinterpret_cast<double*>(take(24 * (size_t)HNP));
  W.Pf = reinterpret_cast<double*>(take(24 * (size_t)HNP));
  W.G = reinterpret_cast<Q3G*>(take(64 * NG));
  W.vv = reinterpret_cast<Q3V*>(take(96 * (size_t)W.FC));
  W.ncoord = reinterpret_cast<double*>(take(72 * (size_t)Q3_NEWCAP));
  W.soff = reinterpret_cast<int*>(take(4 * (size_t)W.FC));
  W.fdist = reinterpret_cast<double*>(take(8 * (size_t)W.FC));
  W.sb = reinterpret_cast<int*>(take(4 * (size_t)W.SB));
  W.pq = reinterpret_cast<int*>(take(4 * (size_t)HNP));
  W.pdst = reinterpret_cast<int*>(take(4 * (size_t)HNP));
  W.pdd = reinterpret_cast<double*>(take(8 * (size_t)HNP));
  W.fq = reinterpret_cast<int*>(take(4 * (size_t)W.QC));
  W.fqk = reinterpret_cast<unsigned*>(take(4 * (size_t)W.QC));
  W.fqc = reinterpret_cast<HullPt*>(take(32 * (size_t)W.QC));
  W.ncoord2 = reinterpret_cast<double*>(take(72 * (size_t)Q3_NEWCAP));
  W.mark2 = reinterpret_cast<unsigned*>(take(4 * (size_t)W.FC));
  W.ctr = reinterpret_cast<unsigned*>(take(256));
  W.hvis = reinterpret_cast<unsigned short*>(take(2 * (Q3_WAVES - 1) * Q3_HZCAP * 64));
  W.hcop = reinterpret_cast<int*>(take(4 * (Q3_WAVES - 1) * Q3_COPCAP * 64));
  return W;
}

// the wave's LDS (one wave per CU)
struct Q3L {
  // hull_points / hull_take_job interface
  int n, fail, job, slot;
  double eps;
  double tr[3 * 128];
  double rk[4];                      // (up to four waves: hull_points' block scans)
  int ri[4];
  int scan[4];
  // facet slots < Q3_FL
  double4 pl[Q3_FL];
  ushort4 tp[Q3_FL];                 // neighbours, QF_* | new-facet index << 8
  unsigned key[Q3_FL];
  unsigned cc[Q3_FL];
  unsigned short fstk[Q3_FSTK];
  // the insertion: visible facets (qh_findhorizon order) and what their
  // slots held (the cone reuses them)
  int visf[Q3_VISCAP];
  int vsoff[Q3_VISCAP], vscnt[Q3_VISCAP], vinc[Q3_VISCAP];
  int vvert[3 * Q3_VISCAP];
  int repl[Q3_VISCAP];               // qh_getreplacement: new-facet index
  // the new facets, creation order: slot, vertices (point ids), horizon
  // facet and its ridge index, neighbours nb1/nb2 (new
  // indices), plane, flags
  int nslot[Q3_NEWCAP];
  int nv[3 * Q3_NEWCAP];
  int nhz[Q3_NEWCAP], nhskip[Q3_NEWCAP];
  int nn1[Q3_NEWCAP], nn2[Q3_NEWCAP];
  alignas(32) double npl[4 * Q3_NEWCAP];
  int nflag[Q3_NEWCAP];
  int movf[Q3_MOVCAP];               // old facets moved behind the new ones (scan order)
  int oldf[Q3_MOVCAP];               // old facets receiving points (destinations Q3_NEWCAP + k)
  // partition destinations: new facets 0.., old facets Q3_NEWCAP + k
  int dfac[Q3_ND], dcnt[Q3_ND], doff[Q3_ND], dchamp[Q3_ND], pcnt[Q3_ND];
  double dmax[Q3_ND];
  double dchp[3 * Q3_ND];            // the furthest point's coordinates
  int cop[Q3_COPCAP * 64];           // the horizon walks' coplanar facet sets, [k][lane]
  unsigned short hvis[Q3_HZCAP * 64];  // the horizon walks' visited facets, [k][lane]
  // Two-wave build: while wave 0 partitions insertion k, wave 1 speculates
  // insertion k+1's horizon and cone (q3_spec) into these; wave 0 adopts them
  // when the facet is still the queue's next with the same furthest point.
  int sp_visf[Q3_VISCAP];
  int sp_repl[Q3_VISCAP];
  int sp_v1[Q3_NEWCAP], sp_v2[Q3_NEWCAP], sp_nhz[Q3_NEWCAP], sp_nhskip[Q3_NEWCAP], sp_nflag[Q3_NEWCAP];
  int sp_nn1[Q3_NEWCAP], sp_nn2[Q3_NEWCAP];   // qh_matchnewfacets' neighbours (new-facet indices)
  int sp_vvert[3 * Q3_VISCAP];                 // the visible facets' vertices
  alignas(32) double sp_npl[4 * Q3_NEWCAP];
  unsigned short mark[Q3_FL];        // wave 1's visit epochs (slots < Q3_FL)
  // wave 1's horizon: the neighbours of the k-th visible facet, sp_cand[3 k ..],
  // stored when it is found (its neighbour list is in hand then): a level's
  // candidates and the cone's ridges are then one LDS read each
  unsigned short sp_cand[3 * Q3_VISCAP];
  // Wave 2 prefetches the next partition sequence's head while wave 1 builds
  // the cone: once wave 1 publishes its horizon (sp_hz = phase, sp_hnvis), the
  // visible facets' outside-set offsets and sizes and the sequence's first 64
  // points (pf_pre, and the visible facet each came from, pf_prea) are read
  // from global memory into LDS (pf_done = phase, pf_np the sequence length).
  // Wave 0 takes them when no visible facet was a destination of the
  // partition that ran meanwhile (their outside sets are then unchanged).
  int sp_hz, sp_hnvis, pf_done, pf_np;
  int pf_vsoff[Q3_VISCAP], pf_vscnt[Q3_VISCAP];
  HullPt pf_pre[64];
  unsigned char pf_prea[64];
  double sp_apex[3];
  double c_dist[8];                  // MINvisible, MAXcoplanar, DISTround, MINdenom, MINdenom_2, NEARzero[3]
  double c_interior[3];
  int ph, sp_done, sp_ok, sp_facet, sp_furthest, sp_pos, sp_nvis, sp_nnew, sp_status, sp_sharp;
  // sp_done releases the speculation's LDS results only; sp_gdone, stored
  // right after with a full release, its global stores too (the vertex
  // records): wave 0 waits for it only where it reads them (its own cone,
  // the selection)
  int sp_gdone;
  unsigned sp_key;
  int pub_qhead, pub_qtail;
  int pub_adopt, pub_nnew;           // the published cone was wave 1's: it writes the vertex records
  // Waves 1-3 locate a partition sequence's chunks beside wave 0 (q3_help):
  // the sequence and wave 0's state (hq_*) posted with hctl = generation << 16
  // | the next chunk to claim (0: none); a wave claims a chunk with a CAS on
  // hctl, holding hbusy meanwhile, once its buffer is free (chunk < hcons +
  // Q3_HR), and releases its results with hr_st = chunk + 1.  Wave 0 stops
  // the claims (hctl = 0) and waits for hbusy = 0 before its state changes.
  double hr_d[Q3_HR * 64];
  unsigned short hr_f[Q3_HR * 64];   // the destination facet (0xffff: none)
  unsigned short hr_k[Q3_HR * 64];   // the event kind | an old destination << 3 | (new-facet index + 1) << 8
  int hr_ls[Q3_HR], hr_st[Q3_HR];
  unsigned hctl;
  int hbusy, hcons;
  // a long sequence's emit split over the waves (q3_emit_bucket): bucket b is
  // the destinations i with i % 4 == b (each destination's points are placed
  // in sequence order by one wave); ectl = generation << 8 | the next bucket
  // to claim (0: none), edone the buckets finished
  unsigned ectl;
  int edone, ej_np, ej_nd, ej_ndnew, ej_init, ej_nvis;
  int hq_end, hq_from, hq_np, hq_sharp, hq_init;
  int hq_findbestnew, hq_notsharp, hq_nnew, hq_nmov, hq_nvis;
  double hq_max_outside;
#ifdef LQRO_QHULL_LONGPROF
  unsigned long long hprof[12];      // helper chunks, their ticks locating, claim to release; wave 1:
                                     // speculations, publication -> seen, seen -> done; wave 0: done -> seen;
                                     // wave 1: queue-window reloads, ticks in the queue scan, in the horizon
  unsigned long long lp_pubr, lp_doner;   // the last publication's / speculation end's real time
#endif
  int big_slot;                      // a build past the caps, rebuilt in place by qh_build (q3_body)
  int qflags;                        // HullArgs::qflags
#ifdef LQRO_QHULL_PROFILE
  unsigned long long pub_t, done_t, done_t2;   // the last publication / speculation end, after its store
  unsigned long long pub_r, start_r, done_r;    // the same on the 100 MHz real-time clock (one clock for all waves)
#endif
};
static_assert(sizeof(Q3L) <= 160 * 1024, "k_qhull's LDS exceeds a CU");

struct Q3S {
  int nalloc, nfs, sbtop, status, qhead, qtail;
  int nins;               // insertions (qh_addpoint calls), for the build's timing record
  unsigned keyc;
  unsigned key0_last;   // the first key of the last insertion's new facets
  int nnew, nvis, nmov, nold;
  int findbestnew, notsharp;
  int hgen;               // q3_locate_seq's posts to the helper waves (hctl's generation)
  int egen;               // q3_emit_seq's posts (ectl's generation)
  double MAXabs_coord, MAXsumcoord, MAXwidth, NEARzero[3];
  double DISTround, MINvisible, MAXcoplanar, MINoutside, MINdenom, MINdenom_2, max_outside;
  double interior[3];
  unsigned long long tph[32];   // LQRO_QHULL_PROFILE: phase cycles 0..20, counters 21..28
  unsigned long long tq;         // LQRO_QHULL_PROFILE: the last stamp
  unsigned long long tw, nw;     // LQRO_QHULL_PROFILE: waiting for wave 1's speculation
  unsigned long long tdl;        // LQRO_QHULL_PROFILE: its end until wave 0 sees it
  unsigned long long tw1, nw1;   // LQRO_QHULL_PROFILE: the waits after one-chunk insertions
  unsigned long long tse, tsn;   // LQRO_QHULL_PROFILE: publication -> speculation end, -> wave 0 past the wait
  unsigned long long tfr, nsp;   // LQRO_QHULL_PROFILE: the wait's first read, its spins
  unsigned long long tfr2, trel;
  unsigned long long r_start, r_done, r_seen, r_gseen;
  unsigned long long tseen, tpre, npre, tstart;
  int prev1;
  unsigned long long tps[24], nps;   // LQRO_QHULL_PROFILE: phases of the one-chunk insertions
  unsigned long long lp_n, lp_pts, lp_t, lp_all, lp_tloc, lp_wait, lp_adopt, lp_tail, lp_tw;   // LQRO_QHULL_LONGPROF
  unsigned long long lp_own, lp_got, lp_hwait, lp_stop, lp_ev, lp_posts;
};

#if defined(LQRO_QHULL_PROFILE) && defined(LQRO_QHULL_PROF_LIGHT)
// (light: no drain — a phase is charged the waits the build itself makes
// there, so the phases add up to the undisturbed critical path)
#define Q3T(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); S.tph[k] += t_ - S.tq; S.tq = t_; } while (0)
#elif defined(LQRO_QHULL_PROFILE)
// (every outstanding load and store drained first: a phase is charged its own memory waits)
#define Q3T(k) do { __builtin_amdgcn_s_waitcnt(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); S.tph[k] += t_ - S.tq; S.tq = t_; } while (0)
#else
#define Q3T(k) do {} while (0)
#endif
// LQRO_QHULL_PROFILE counters: 21 insertions, 22 partitioned points, 23 located
// chunks, 24 sequence events, 25 emitted destination groups, 31 adopted speculations
// Wave 1's own phases and wave 0's wait for it (LQRO_QHULL_PROFILE): prof words
// Q3_PROF_W1 + k: 0 speculation total, 1 the adopted cone's vertex records,
// 2 queue scan, 3 horizon, 4 cone, 5 match / checkzero / sharp, 6 serving
// chunks, 7 speculations, 8 chunks served, 9 wave 0 waiting for a speculation,
// 10 waits; 16 + k: wave 0's phase k (Q3T) over the insertions whose partition
// sequence fits one chunk (np <= 64), 40 their number; cycles summed over the
// step's hulls (lqro_debug_prof_words)
#define Q3_PROF_W1 (32 + 2 * 4096 + 48 + 4 * 4096)
// LQRO_QHULL_LONGPROF (a diagnostic build, scripts/build_variant.sh): per
// build record k (lqro_get_hull_builds order, k < 1024), prof words
// Q3_PROF_LONG + 24 k: insertions whose partition sequence is longer than one
// chunk, their points, their ticks (100 MHz, from the publication to the end
// of the emit), the ticks of all the build's partitions, the long ones' ticks
// to the end of their locate; wave 0's ticks waiting for the speculation,
// from the wait to the publication, from the emit's end to the next wait;
// chunks of helped sequences wave 0 located, chunks the helpers did, ticks
// waiting for them, ticks stopping them, events, posts; helper chunks and
// their ticks; wave 1's speculations, publication -> seen and seen -> done
// ticks; wave 0's waits and their speculation-end -> seen ticks
#define Q3_PROF_LONG (Q3_PROF_W1 + 64)
struct Q3P {
  unsigned long long tq2 = 0;   // LQRO_QHULL_PROFILE: the last speculation's end (this wave's clock)
  unsigned long long t[16];
  unsigned long long tq;
};
#if defined(LQRO_QHULL_PROFILE) && defined(LQRO_QHULL_PROF_LIGHT)
#define W1T(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); P.t[k] += t_ - P.tq; P.tq = t_; } while (0)
#elif defined(LQRO_QHULL_PROFILE)
#define W1T(k) do { __builtin_amdgcn_s_waitcnt(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); P.t[k] += t_ - P.tq; P.tq = t_; } while (0)
#else
#define W1T(k) do {} while (0)
#endif
#ifdef LQRO_QHULL_PROFILE
#define Q3C(k, v) do { S.tph[k] += (unsigned long long)(v); } while (0)
#else
#define Q3C(k, v) do {} while (0)
#endif

// ---- facet fields: LDS below Q3_FL, the global record beyond ----
// Every access names its address space: with two generic pointers the
// compiler merges the LDS and the global load of an accessor into one flat
// load behind a pointer select, and a flat load waits for every outstanding
// global access (s_waitcnt vmcnt(0) lgkmcnt(0)).
#define Q3_AS3 __attribute__((address_space(3)))
#define Q3_AS1 __attribute__((address_space(1)))
template <class T> __device__ __forceinline__ T q3_lds(const T& r) { return *(const Q3_AS3 T*)(&r); }
template <class T> __device__ __forceinline__ void q3_lds_st(T& r, const T& v) { *(Q3_AS3 T*)(&r) = v; }
template <class T> __device__ __forceinline__ T q3_glb(const T& r) { return *(const Q3_AS1 T*)(&r); }
template <class T> __device__ __forceinline__ void q3_glb_st(T& r, const T& v) { *(Q3_AS1 T*)(&r) = v; }
typedef double q3_v4d __attribute__((ext_vector_type(4)));
typedef int q3_v4i __attribute__((ext_vector_type(4)));
typedef unsigned q3_v2u __attribute__((ext_vector_type(2)));
// the vector records (HIP's vector classes have no address-space copies)
__device__ __forceinline__ double4 q3_lds(const double4& r) {
  const q3_v4d v = *(const Q3_AS3 q3_v4d*)(&r);
  return make_double4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void q3_lds_st(double4& r, const double4& v) {
  q3_v4d t; t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
  *(Q3_AS3 q3_v4d*)(&r) = t;
}
__device__ __forceinline__ ushort4 q3_lds(const ushort4& r) {
  const q3_v2u v = *(const Q3_AS3 q3_v2u*)(&r);
  return make_ushort4((unsigned short)(v.x & 0xffffu), (unsigned short)(v.x >> 16), (unsigned short)(v.y & 0xffffu),
                      (unsigned short)(v.y >> 16));
}
__device__ __forceinline__ void q3_lds_st(ushort4& r, const ushort4& v) {
  q3_v2u t;
  t.x = (unsigned)v.x | ((unsigned)v.y << 16);
  t.y = (unsigned)v.z | ((unsigned)v.w << 16);
  *(Q3_AS3 q3_v2u*)(&r) = t;
}
__device__ __forceinline__ double4 q3_glb(const double4& r) {
  const q3_v4d v = *(const Q3_AS1 q3_v4d*)(&r);
  return make_double4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void q3_glb_st(double4& r, const double4& v) {
  q3_v4d t; t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
  *(Q3_AS1 q3_v4d*)(&r) = t;
}
__device__ __forceinline__ int4 q3_glb(const int4& r) {
  const q3_v4i v = *(const Q3_AS1 q3_v4i*)(&r);
  return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void q3_glb_st(int4& r, const int4& v) {
  q3_v4i t; t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
  *(Q3_AS1 q3_v4i*)(&r) = t;
}

// A lane's columns for qh_findbesthorizon's visited facets and coplanar set
// ([k][lane], stride 64): wave 0's in LDS (L.hvis, L.cop), each helper
// wave's in its worker scratch (W.hvis, W.hcop) — one column per lane of
// every wave that locates points at the same time
struct Q3Col {
  unsigned short* vis;
  int* cop;
};
template <bool G, class T> __device__ __forceinline__ T q3_col(const T& r) {
  if constexpr (G) return q3_glb(r);
  else return q3_lds(r);
}
template <bool G, class T> __device__ __forceinline__ void q3_col_st(T& r, const T& v) {
  if constexpr (G) q3_glb_st(r, v);
  else q3_lds_st(r, v);
}
__device__ __forceinline__ Q3Col q3_col0(const Q3L& L, int lane) {
  Q3Col C;
  C.vis = const_cast<unsigned short*>(L.hvis) + lane;
  C.cop = const_cast<int*>(L.cop) + lane;
  return C;
}
__device__ __forceinline__ Q3Col q3_colh(const Q3W& W, int wave, int lane) {   // helper waves 1..Q3_WAVES-1
  Q3Col C;
  C.vis = W.hvis + (size_t)(wave - 1) * Q3_HZCAP * 64 + lane;
  C.cop = W.hcop + (size_t)(wave - 1) * Q3_COPCAP * 64 + lane;
  return C;
}

__device__ __forceinline__ void q3_get(const Q3W& W, const Q3L& L, int f, double* q, int* nb, int* fa) {
  if (f < Q3_FL) {
    const double4 p = q3_lds(L.pl[f]);
    const ushort4 t = q3_lds(L.tp[f]);
    q[0] = p.x; q[1] = p.y; q[2] = p.z; q[3] = p.w;
    nb[0] = t.x; nb[1] = t.y; nb[2] = t.z; *fa = t.w;
  } else {
    const Q3G& g = W.G[f - Q3_FL];
    const double4 p = q3_glb(*reinterpret_cast<const double4*>(g.pl));
    const int4 t = q3_glb(*reinterpret_cast<const int4*>(g.nb));
    q[0] = p.x; q[1] = p.y; q[2] = p.z; q[3] = p.w;
    nb[0] = t.x; nb[1] = t.y; nb[2] = t.z; *fa = t.w;
  }
}
__device__ __forceinline__ void q3_pl(const Q3W& W, const Q3L& L, int f, double* q) {
  const double4 p = f < Q3_FL ? q3_lds(L.pl[f]) : q3_glb(*reinterpret_cast<const double4*>(W.G[f - Q3_FL].pl));
  q[0] = p.x; q[1] = p.y; q[2] = p.z; q[3] = p.w;
}
__device__ __forceinline__ int q3_nb(const Q3W& W, const Q3L& L, int f, int k) {
  if (f < Q3_FL) return q3_lds(reinterpret_cast<const unsigned short*>(&L.tp[f])[k]);
  return q3_glb(W.G[f - Q3_FL].nb[k]);
}
__device__ __forceinline__ void q3_tp(const Q3W& W, const Q3L& L, int f, int* nb, int* fa) {
  if (f < Q3_FL) {
    const ushort4 t = q3_lds(L.tp[f]);
    nb[0] = t.x; nb[1] = t.y; nb[2] = t.z; *fa = t.w;
  } else {
    const int4 t = q3_glb(*reinterpret_cast<const int4*>(W.G[f - Q3_FL].nb));
    nb[0] = t.x; nb[1] = t.y; nb[2] = t.z; *fa = t.w;
  }
}
__device__ __forceinline__ int q3_fa(const Q3W& W, const Q3L& L, int f) {
  return f < Q3_FL ? (int)q3_lds(L.tp[f].w) : q3_glb(W.G[f - Q3_FL].fa);
}
__device__ __forceinline__ unsigned q3_key(const Q3W& W, const Q3L& L, int f) {
  return f < Q3_FL ? q3_lds(L.key[f]) : q3_glb(W.G[f - Q3_FL].key);
}
__device__ __forceinline__ unsigned q3_cc(const Q3W& W, const Q3L& L, int f) {
  return f < Q3_FL ? q3_lds(L.cc[f]) : q3_glb(W.G[f - Q3_FL].cc);
}
__device__ __forceinline__ void q3_set_fa(const Q3W& W, Q3L& L, int f, int fa) {
  if (f < Q3_FL) q3_lds_st(L.tp[f].w, (unsigned short)fa);
  else q3_glb_st(W.G[f - Q3_FL].fa, fa);
}
__device__ __forceinline__ void q3_set_nb(const Q3W& W, Q3L& L, int f, int k, int v) {
  if (f < Q3_FL) q3_lds_st(reinterpret_cast<unsigned short*>(&L.tp[f])[k], (unsigned short)v);
  else q3_glb_st(W.G[f - Q3_FL].nb[k], v);
}
__device__ __forceinline__ void q3_set_key(const Q3W& W, Q3L& L, int f, unsigned k) {
  if (f < Q3_FL) q3_lds_st(L.key[f], k);
  else q3_glb_st(W.G[f - Q3_FL].key, k);
}
__device__ __forceinline__ void q3_set_cc(const Q3W& W, Q3L& L, int f, unsigned c) {
  if (f < Q3_FL) q3_lds_st(L.cc[f], c);
  else q3_glb_st(W.G[f - Q3_FL].cc, c);
}
__device__ __forceinline__ void q3_set_facet(const Q3W& W, Q3L& L, int f, const double* q, int nb0, int nb1, int nb2,
                                             int fa) {
  if (f < Q3_FL) {
    q3_lds_st(L.pl[f], make_double4(q[0], q[1], q[2], q[3]));
    q3_lds_st(L.tp[f], make_ushort4((unsigned short)nb0, (unsigned short)nb1, (unsigned short)nb2, (unsigned short)fa));
  } else {
    Q3G& g = W.G[f - Q3_FL];
    q3_glb_st(*reinterpret_cast<double4*>(g.pl), make_double4(q[0], q[1], q[2], q[3]));
    q3_glb_st(*reinterpret_cast<int4*>(g.nb), make_int4(nb0, nb1, nb2, fa));
  }
}

// the adapter that lets the verified plane code (qh_plane_gauss, qh_detsimplex) read Q3S
__device__ __forceinline__ QhS q3_as_qhs(const Q3S& S) {
  QhS T;
  T.DISTround = S.DISTround;
  T.MINdenom = S.MINdenom;
  T.MINdenom_2 = S.MINdenom_2;
  for (int k = 0; k < 3; k++) T.NEARzero[k] = S.NEARzero[k];
  return T;
}

// qh_setfacetplane (qh_sethyperplane_det, nearly singular -> _gauss) for a
// facet with vertex points r0, r1, r2 in its vertex order; qh_checkflipped
__device__ inline void q3_plane(const Q3S& S, int& status, const double* r0, const double* r1, const double* r2,
                                int top, double* q, bool* flipped) {
  const double dX10 = r1[0] - r0[0], dY10 = r1[1] - r0[1], dZ10 = r1[2] - r0[2];
  const double dX20 = r2[0] - r0[0], dY20 = r2[1] - r0[1], dZ20 = r2[2] - r0[2];
  double n[3];
  n[0] = QH_DET2(dY20, dZ20, dY10, dZ10);
  n[1] = QH_DET2(dX10, dZ10, dX20, dZ20);
  n[2] = QH_DET2(dX20, dY20, dX10, dY10);
  double norm = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  if (norm > S.MINdenom) {
    if (!top) norm = -norm;
    n[0] /= norm;
    n[1] /= norm;
    n[2] /= norm;
  } else {
    status |= QHS_SINGULAR;
  }
  double off = -(r0[0] * n[0] + r0[1] * n[1] + r0[2] * n[2]);
  const double d2 = off + (r2[0] * n[0] + r2[1] * n[1] + r2[2] * n[2]);
  const double d1 = off + (r1[0] * n[0] + r1[1] * n[1] + r1[2] * n[2]);
  if (d2 > S.DISTround || d2 < -S.DISTround || d1 > S.DISTround || d1 < -S.DISTround) {
    const QhS T = q3_as_qhs(S);
    qh_plane_gauss(T, status, r0, r1, r2, top, n, &off);
  }
  q[0] = n[0]; q[1] = n[1]; q[2] = n[2]; q[3] = off;
  const double di = off + S.interior[0] * n[0] + S.interior[1] * n[1] + S.interior[2] * n[2];
  *flipped = di >= -S.DISTround;
}

__device__ __forceinline__ double q3_distq(const double* q, const double* p) {   // qh_distplane
  return q[3] + p[0] * q[0] + p[1] * q[1] + p[2] * q[2];
}

// inclusive wave scan (sum) with DPP row shifts and row broadcasts
__device__ __forceinline__ int q3_scan_add(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
  return v;
}

// inclusive wave scan (max) of a double, -DBL_MAX where a lane has no
// predecessor (DPP on the two halves)
#define Q3_MAXSTEP(V, CTRL, RM)                                                                    \
  do {                                                                                           \
    const long long u_ = __double_as_longlong(V);                                                \
    const int lo_ = __builtin_amdgcn_update_dpp(-1, (int)u_, CTRL, RM, 0xf, false);              \
    const int hi_ = __builtin_amdgcn_update_dpp((int)0xFFEFFFFF, (int)(u_ >> 32), CTRL, RM, 0xf, false); \
    V = fmax(V, __longlong_as_double(((long long)hi_ << 32) | (long long)(unsigned)lo_));        \
  } while (0)
__device__ __forceinline__ double q3_scan_max(double v) {
  Q3_MAXSTEP(v, 0x111, 0xf);   // row_shr:1
  Q3_MAXSTEP(v, 0x112, 0xf);   // row_shr:2
  Q3_MAXSTEP(v, 0x114, 0xf);   // row_shr:4
  Q3_MAXSTEP(v, 0x118, 0xf);   // row_shr:8
  Q3_MAXSTEP(v, 0x142, 0xa);   // row_bcast:15 -> rows 1, 3
  Q3_MAXSTEP(v, 0x143, 0xc);   // row_bcast:31 -> rows 2, 3
  return v;
}

// Qhull's outside-set placement (qh_partitionpoint: a point further than the
// set's furthest point is appended and becomes the furthest; any other is
// put second-to-last, before the furthest) for the lanes of grp in lane
// order, all at once.  A point's slot is fixed when it arrives (the count
// before it, less one) unless it is a new furthest point: that one stays
// last until the next new furthest point arrives, and is then fixed just
// before it.  The furthest point itself is held aside (cx, cy, cz, champ)
// and written by the caller at the end.  Entries at or beyond lim are not
// written (the caller reports the capacity).  The lane's entry is returned
// (wpos >= 0, wr), not stored: a chunk's lanes are in one group each, so the
// caller stores once per chunk after all its groups — a fixed number of
// stores between the next chunk's loads and their use (vmcnt is in order:
// a data-dependent store count made every chunk wait for all its stores)
__device__ __forceinline__ void q3_place(unsigned long long grp, int lane, unsigned long long ltmask,
                                         double dd, const HullPt& pt, int off, int lim, int& cnt, double& mx,
                                         int& champ, double& cx, double& cy, double& cz, int& wpos, int& wr) {
  const bool mem = (grp >> lane) & 1ull;
  const int cb = cnt + __popcll(grp & ltmask);   // points before this one in the set
  double run = -DBL_MAX;                         // the largest distance among them
  if (grp & (grp - 1ull)) {
    const double inc = q3_scan_max(mem ? dd : -DBL_MAX);
    // the running maximum before this lane: wave_shr:1 (lane 0 gets -DBL_MAX)
    const long long u_ = __double_as_longlong(inc);
    const int lo_ = __builtin_amdgcn_update_dpp(-1, (int)u_, 0x138, 0xf, 0xf, false);
    const int hi_ = __builtin_amdgcn_update_dpp((int)0xFFEFFFFF, (int)(u_ >> 32), 0x138, 0xf, 0xf, false);
    run = __longlong_as_double(((long long)hi_ << 32) | (long long)(unsigned)lo_);
  }
  if (cnt > 0) run = fmax(run, mx);
  const bool rec = mem && (cb == 0 || run < dd);
  const unsigned long long recm = __ballot(rec);
  const unsigned long long prevm = recm & ltmask;
  int pq = 0;
  if (recm & (recm - 1ull)) {   // a new furthest point displacing another one of this pass
    const int pl = prevm ? 63 - __clzll((long long)prevm) : lane;
    pq = __shfl(pt.q, pl);
  }
  if (mem && cb > 0 && off + cb - 1 < lim) {
    // the furthest point it displaces: the previous new furthest here, or the held one
    wpos = off + cb - 1;
    wr = rec ? (prevm ? pq : champ) : pt.q;
  }
  if (recm) {
    const int l = 63 - __clzll((long long)recm);
    champ = __builtin_amdgcn_readlane(pt.q, l);
    cx = hl_rl(pt.x, l); cy = hl_rl(pt.y, l); cz = hl_rl(pt.z, l);
    mx = hl_rl(dd, l);
  }
  cnt += __popcll(grp);
}

// ---- point location, per lane (geom_r.c) ----
// qh_findbesthorizon; a step reads the three neighbours together, and the
// one the walk moves to brings its own neighbours along
template <bool G>
__device__ inline int q3_findbesthorizon(const Q3W& W, const Q3S& S, const Q3L& L, const double* p, int startfacet,
                                         double* bestdist, int& lstatus, const Q3Col& C) {
  int bestfacet = startfacet;
  const double searchdist = S.max_outside + 2 * S.DISTround + fmax(S.MINvisible, S.MAXcoplanar);
  double minsearch = *bestdist - searchdist;
  // the facets visited (qh.visit_id), in the lane's column (a register array
  // with a run-time length compiles to a select per slot and check), and
  // qh.coplanarfacetset
  unsigned short* vis = C.vis;
  int nvis = 0;
  int* cop = C.cop;
  int ncop = 0;
  int nextfacet = -1, nextnb[3] = {-1, -1, -1};
  q3_col_st<G>(vis[0], (unsigned short)startfacet);
  nvis = 1;
  int cur[3] = {q3_nb(W, L, startfacet, 0), q3_nb(W, L, startfacet, 1), q3_nb(W, L, startfacet, 2)};
  for (;;) {
    double q[3][4];
    int fl[3], nn[3][3];
    for (int k = 0; k < 3; k++) q3_get(W, L, cur[k], q[k], nn[k], &fl[k]);
    bool seen3[3] = {false, false, false};
    for (int t = 0; t < nvis; t++) {
      const int v = q3_col<G>(vis[64 * t]);
      seen3[0] |= v == cur[0]; seen3[1] |= v == cur[1]; seen3[2] |= v == cur[2];
    }
    for (int k = 0; k < 3; k++) {
      const int nb = cur[k];
      // (a neighbour listed twice: the first takes it)
      const bool seen = seen3[k] || (k >= 1 && nb == cur[0]) || (k == 2 && nb == cur[1]);
      if (seen) continue;
      if (nvis == Q3_HZCAP) { lstatus |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_HZ); return bestfacet; }
      q3_col_st<G>(vis[64 * nvis], (unsigned short)nb);
      nvis++;
      if (!(fl[k] & QF_FLIPPED)) {
        const double dist = q3_distq(q[k], p);
        if (dist > *bestdist) {
          minsearch = dist - searchdist;
          if (dist > *bestdist + searchdist) ncop = 0;
          bestfacet = nb;
          *bestdist = dist;
        } else if (dist < minsearch) {
          continue;
        }
      }
      if (nextfacet >= 0) {
        if (ncop == Q3_COPCAP) { lstatus |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_COP); return bestfacet; }
        q3_col_st<G>(cop[64 * ncop++], nextfacet);
      }
      nextfacet = nb;
      nextnb[0] = nn[k][0]; nextnb[1] = nn[k][1]; nextnb[2] = nn[k][2];
    }
    if (nextfacet >= 0) {
      nextfacet = -1;
      cur[0] = nextnb[0]; cur[1] = nextnb[1]; cur[2] = nextnb[2];
      continue;
    }
    if (!ncop) break;
    int facet;
    if (ncop == 1) { facet = q3_col<G>(cop[0]); ncop = 0; }
    else facet = q3_col<G>(cop[64 * --ncop]);
    cur[0] = q3_nb(W, L, facet, 0); cur[1] = q3_nb(W, L, facet, 1); cur[2] = q3_nb(W, L, facet, 2);
  }
  return bestfacet;
}

// qh_findbestnew over the scan list: the new facets from index s0, the moved
// old facets, the new facets before s0 (the facet list from startfacet to
// its end, then from qh.newfacet_list)
template <bool G>
__device__ inline int q3_findbestnew(const Q3W& W, const Q3S& S, const Q3L& L, const double* p, int s0,
                                     double* dist, int bestoutside, int* isoutside, int& lstatus, const Q3Col& C) {
  double bestdist = -DBL_MAX / 2;
  int bestfacet = -1;
  const double distoutside = fmax(2 * S.MINoutside, S.max_outside);    // qh_DISToutside
  *isoutside = 1;
  const int total = S.nnew + S.nmov;
  // the scan list, four facets' planes fetched at a time (in order; the
  // first one at or beyond distoutside ends the scan)
  auto fetch = [&](int t, int& f, int& fl, double* q) {
    if (t < S.nnew - s0 || t >= S.nnew - s0 + S.nmov) {
      const int u = t < S.nnew - s0 ? s0 + t : t - (S.nnew - s0) - S.nmov;
      f = L.nslot[u];
      const double4 v = q3_lds(*reinterpret_cast<const double4*>(L.npl + 4 * u));
      q[0] = v.x; q[1] = v.y; q[2] = v.z; q[3] = v.w;
      fl = L.nflag[u];
    } else {
      f = L.movf[t - (S.nnew - s0)];
      q3_pl(W, L, f, q);
      fl = q3_fa(W, L, f);
    }
  };
  for (int t0 = 0; t0 < total; t0 += 4) {
    int f[4], fl[4];
    double q[4][4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      f[k] = -1; fl[k] = QF_FLIPPED;
      if (t0 + k < total) fetch(t0 + k, f[k], fl[k], q[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (fl[k] & QF_FLIPPED) continue;
      const double d = q3_distq(q[k], p);
      if (d > bestdist) {
        bestfacet = f[k];
        if (!bestoutside && d >= distoutside) { *dist = d; return bestfacet; }
        bestdist = d;
      }
    }
  }
  bestfacet = q3_findbesthorizon<G>(W, S, L, p, bestfacet >= 0 ? bestfacet : L.nslot[s0], &bestdist, lstatus, C);
  *dist = bestdist;
  if (bestdist < S.MINoutside) *isoutside = 0;
  return bestfacet;
}

// qh_sharpnewfacets: a new facet's normal in another quadrant than the first's
__device__ inline int q3_sharpnewfacets(const Q3S& S, const Q3L& L, int lane) {
  if (S.nnew == 0) return 0;
  const bool q0 = L.npl[0] > 0, q1 = L.npl[1] > 0, q2 = L.npl[2] > 0;
  bool diff = false;
  for (int t = lane; t < S.nnew; t += 64) {
    const double* n = L.npl + 4 * t;
    diff |= (n[0] > 0) != q0 || (n[1] > 0) != q1 || (n[2] > 0) != q2;
  }
  return __ballot(diff) != 0ull;
}

// One partitioned point under the state (S.findbestnew, S.notsharp): its
// facet and distance, and whether it changes the state (lqro_qhull.hpp
// qh_locate).  s0: the start facet's new-facet index; sharp = 2:
// qh_findbestnew(bestoutside) for a deleted vertex.
template <bool G>
__device__ inline int q3_locate(const Q3W& W, const Q3S& S, const Q3L& L, const double* p, int s0, int sharp,
                                double* bestdist_out, int* isoutside, int* trigger, int& lstatus, const Q3Col& C) {
  *trigger = 0;
  if (sharp == 2) return q3_findbestnew<G>(W, S, L, p, s0, bestdist_out, 1, isoutside, lstatus, C);
  if (S.findbestnew) return q3_findbestnew<G>(W, S, L, p, s0, bestdist_out, 0, isoutside, lstatus, C);
  // qh_findbest(point, startfacet, bestoutside 0, isnewfacets 1, noupper 0):
  // the new facets only, their neighbours nb1 / nb2 (nb0 is the horizon facet)
  double bestdist = -DBL_MAX / 2;
  int bestu = -1;
  *isoutside = 1;
  unsigned long long m0 = 0ull, m1 = 0ull;   // new facets visited (index < Q3_NEWCAP = 128)
  if (!(L.nflag[s0] & QF_FLIPPED)) {
    const double d = q3_distq(L.npl + 4 * s0, p);
    if (d >= S.MINoutside) { *bestdist_out = d; return L.nslot[s0]; }
    bestdist = d;
    bestu = s0;
  }
  if (s0 < 64) m0 |= 1ull << s0; else m1 |= 1ull << (s0 - 64);
  int u = s0;
  while (u >= 0) {
    int nxt = -1;
    const int cand[2] = {L.nn1[u], L.nn2[u]};
    // both neighbours' flags and planes in one round trip
    const int cfl[2] = {L.nflag[cand[0]], L.nflag[cand[1]]};
    double cq[2][4];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const double4 v = q3_lds(*reinterpret_cast<const double4*>(L.npl + 4 * cand[k]));
      cq[k][0] = v.x; cq[k][1] = v.y; cq[k][2] = v.z; cq[k][3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int c = cand[k];
      const bool was = c < 64 ? (m0 >> c) & 1ull : (m1 >> (c - 64)) & 1ull;
      if (was) continue;
      if (c < 64) m0 |= 1ull << c; else m1 |= 1ull << (c - 64);
      if (!(cfl[k] & QF_FLIPPED)) {
        const double d = q3_distq(cq[k], p);
        if (d > bestdist) {
          if (d >= S.MINoutside) { *bestdist_out = d; return L.nslot[c]; }
          bestu = c;
          bestdist = d;
          nxt = c;
          break;
        }
      }
    }
    u = nxt;
  }
  if (bestu < 0) return q3_findbestnew<G>(W, S, L, p, 0, bestdist_out, 0, isoutside, lstatus, C);
  if (!S.notsharp && bestdist < -S.DISTround) {
    *trigger = 1;
    if (sharp) return q3_findbestnew<G>(W, S, L, p, bestu, bestdist_out, 0, isoutside, lstatus, C);
  }
  const int bf = q3_findbesthorizon<G>(W, S, L, p, L.nslot[bestu], &bestdist, lstatus, C);
  *bestdist_out = bestdist;
  if (bestdist < S.MINoutside) *isoutside = 0;
  return bf;
}

__device__ __forceinline__ bool q3_in_movf(const Q3S& S, const Q3L& L, int f) {
  for (int t = 0; t < S.nmov; t++)
    if (L.movf[t] == f) return true;
  return false;
}

// the partition sequence's point at pos and its start facet (new-facet
// index): qh_partitionall's remainder (W.pq), or the visible facets' outside
// sets in visible order (qh_partitionvisible)
__device__ __forceinline__ HullPt q3_seqpt(const Q3W& W, const Q3L& L, int nvis, bool init, int pos, int* start) {
  HullPt r;
  if (init) {
    const int q = W.pq[pos];
    r.x = W.Pr[3 * (size_t)q]; r.y = W.Pr[3 * (size_t)q + 1]; r.z = W.Pr[3 * (size_t)q + 2];
    r.q = q;
    r.pad = 0;
    *start = 0;
    return r;
  }
  int a = 0, b = nvis - 1;
  while (a < b) {
    const int mid = (a + b) >> 1;
    if (L.vinc[mid] > pos) b = mid;
    else a = mid + 1;
  }
  *start = L.repl[a] >= 0 ? L.repl[a] : 0;
  const int q = W.sb[L.vsoff[a] + pos - (L.vinc[a] - L.vscnt[a])];
  r.x = W.Pr[3 * (size_t)q]; r.y = W.Pr[3 * (size_t)q + 1]; r.z = W.Pr[3 * (size_t)q + 2];
  r.q = q;
  r.pad = 0;
  return r;
}

__device__ __forceinline__ int q3_ld_acq(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void q3_st_rel(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// a release of this wave's LDS writes only: no wait for its global stores
// (a workgroup-scope release waits until every one of them is acknowledged)
__device__ __forceinline__ void q3_st_rel_lds(int* p, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wait (bounded) until *p != v (ne) or == v (!ne); the last value read
__device__ __forceinline__ int q3_wait(const int* p, int v, bool ne) {
  int x = q3_ld_acq(p);
  for (long w = 0; (ne ? x == v : x != v) && w < (1l << 24); ++w) {
    __builtin_amdgcn_s_sleep(Q3_W0_SLEEP);
    x = q3_ld_acq(p);
  }
  return x;
}

// One chunk of the partition sequence located under the state S: the point
// at position c + lane (when from <= pos < np), its facet, distance and
// flags (qh_locate).  Wave 0 runs it for the chunks it claims, waves 1-3 for
// theirs under a copy of wave 0's state (q3_help).
template <bool G>
__device__ __forceinline__ void q3_chunk_locate(const Q3W& W, const Q3S& S, const Q3L& L, int c, int from, int np,
                                                int sharp, bool init, int lane, const HullPt& pre, int prestart,
                                                int prec, HullPt& pt, int& f, double& d, int& isout, int& trig,
                                                int& ls, const Q3Col& C) {
  const int pos = c + lane;
  pt = pre;
  f = -1; d = 0.0; isout = 0; trig = 0;
  if (pos >= from && pos < np) {
    int start = prestart;
    if (c != prec) pt = q3_seqpt(W, L, S.nvis, init, pos, &start);   // (prec: the chunk pre holds)
    const double p[3] = {pt.x, pt.y, pt.z};
    f = q3_locate<G>(W, S, L, p, start, sharp, &d, &isout, &trig, ls, C);
  }
}

// Waves 1-3: claim and locate the posted sequence's next chunk, if any is
// free (the state wave 0 had when it posted); true when one was located
__device__ inline bool q3_help(const Q3W& W, Q3L& L, int lane, const Q3Col& C) {
  const unsigned v = (unsigned)q3_ld_acq(reinterpret_cast<const int*>(&L.hctl));
  if (v == 0u) return false;
  const int k = (int)(v & 0xffffu);
  if (k >= L.hq_end || k >= hl_ld(&L.hcons) + Q3_HR) return false;
  int got = 0;
  if (lane == 0) {
    __hip_atomic_fetch_add(&L.hbusy, 1, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP);
    unsigned e = v;
    got = __hip_atomic_compare_exchange_strong(&L.hctl, &e, v + 1u, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
    if (!got) __hip_atomic_fetch_add(&L.hbusy, -1, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (!__builtin_amdgcn_readfirstlane(got)) return false;
#ifdef LQRO_QHULL_LONGPROF
  const unsigned long long th0 = __builtin_amdgcn_s_memrealtime();
#endif
  Q3S S;
  S.MINvisible = L.c_dist[0]; S.MAXcoplanar = L.c_dist[1]; S.DISTround = L.c_dist[2];
  S.MINoutside = 2 * S.MINvisible;
  S.findbestnew = L.hq_findbestnew; S.notsharp = L.hq_notsharp;
  S.nnew = L.hq_nnew; S.nmov = L.hq_nmov; S.nvis = L.hq_nvis;
  S.max_outside = L.hq_max_outside;
  HullPt pt, pre;
  pre.x = pre.y = pre.z = 0.0; pre.q = -1; pre.pad = 0;
  int f, isout, trig, ls = 0;
  double d;
  const int from = L.hq_from, np = L.hq_np, pos = 64 * k + lane;
  q3_chunk_locate<true>(W, S, L, 64 * k, from, np, L.hq_sharp, L.hq_init != 0, lane, pre, 0, -1, pt, f, d, isout,
                        trig, ls, C);
#ifdef LQRO_QHULL_LONGPROF
  const unsigned long long th1 = __builtin_amdgcn_s_memrealtime();
#endif
  // what wave 0 does with each result (q3_locate_seq), under the same state:
  // the event kind and the destination (a new facet's index; an old facet's
  // is wave 0's to give)
  int kind = 0, dst = -1, dfa = 0;
  if (pos >= from && pos < np) {
    if (isout) {
      dst = f;
      dfa = q3_fa(W, L, f);
      if (!(dfa & QF_NEW) && (q3_cc(W, L, f) & 0xffffu) == 0 && !q3_in_movf(S, L, f)) kind |= 4;
    } else if (d >= -S.MAXcoplanar && d > S.max_outside) {
      kind |= 2;
    }
    if (trig) kind |= 1;
  }
  const bool old = dst >= 0 && !(dfa & QF_NEW);
  const int b = k % Q3_HR;
  L.hr_d[64 * b + lane] = d;
  L.hr_f[64 * b + lane] = (unsigned short)dst;
  L.hr_k[64 * b + lane] = (unsigned short)(kind | (old ? 8 : 0) | ((dst >= 0 && !old ? (dfa >> 8) + 1 : 0) << 8));
  const int st = qh_wave_or(ls);
  if (lane == 0) {
    L.hr_ls[b] = st;
    q3_st_rel_lds(&L.hr_st[b], k + 1);   // (the results are in LDS)
    __hip_atomic_fetch_add(&L.hbusy, -1, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef LQRO_QHULL_LONGPROF
    const unsigned long long th2 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(&L.hprof[0], 1ull);
    atomicAdd(&L.hprof[1], th1 - th0);
    atomicAdd(&L.hprof[2], th2 - th0);
#endif
  }
  return true;
}

// Locate the partition sequence in order (lqro_qhull.hpp qh_locate_seq) and
// count each point into its destination (a new facet's index, or Q3_NEWCAP
// + k for the k-th old facet to receive points) once its result is final.
// Chunks stay aligned to the lanes (position 64 k + lane), so a sequence of
// at most 64 points leaves each lane's final destination, distance and point
// in rg, rd, rpt; a longer one goes through W.pdst, W.pdd.  pre /
// prestart: position `lane`'s point, fetched by the caller (havepre).
// init: qh_partitionall's remainder (the scan list is the facet list; a
// moved facet goes to its end).
__device__ inline void q3_locate_seq(const Q3W& W, Q3S& S, Q3L& L, int np, int sharp, bool init, int lane,
                                     const HullPt& pre, int prestart, bool havepre, int& rg, double& rd,
                                     HullPt& rpt) {
  for (int t = lane; t < Q3_NEWCAP; t += 64) L.pcnt[t] = 0;
  S.nold = 0;
  rg = -1;
  rd = 0.0;
  rpt = pre;
  hl_sync();
  // a sequence of more than one chunk: waves 1-3 locate chunks ahead of wave
  // 0 under its current state, posted from `from` on; an event (a state
  // change) stops them and posts the rest again under the new state
  const bool help = np > 64 && (L.qflags & 1);
  const Q3Col C0 = q3_col0(L, lane);
  auto post = [&](int from2) {   // (no helper holds a claim: hctl = 0, hbusy = 0)
    S.hgen = S.hgen % 32767 + 1;
    if (lane == 0) {
      L.hq_end = (np + 63) >> 6; L.hq_from = from2; L.hq_np = np; L.hq_sharp = sharp; L.hq_init = init ? 1 : 0;
      L.hq_findbestnew = S.findbestnew; L.hq_notsharp = S.notsharp; L.hq_nnew = S.nnew; L.hq_nmov = S.nmov;
      L.hq_nvis = S.nvis; L.hq_max_outside = S.max_outside;
      L.hcons = from2 >> 6;
      for (int b = 0; b < Q3_HR; b++) L.hr_st[b] = 0;
      // (a full release: the new facets' spilled records are global); the
      // first chunk is wave 0's own (it would wait for it anyway, and it
      // locates it with its LDS columns)
      q3_st_rel(reinterpret_cast<int*>(&L.hctl), (int)(((unsigned)S.hgen << 16) | (unsigned)((from2 >> 6) + 1)));
    }
  };
  auto stop = [&]() {   // no further claims; the held ones answered
    if (lane == 0) __hip_atomic_exchange(&L.hctl, 0u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP);
    int b = __hip_atomic_load(&L.hbusy, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (long w = 0; b != 0 && w < (1l << 24); ++w) {
      __builtin_amdgcn_s_sleep(Q3_W0_SLEEP);
      b = __hip_atomic_load(&L.hbusy, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // a helper that never answered may still write: the build stops here and
    // is rebuilt (k_qhull_big)
    if (b != 0) S.status |= QHS_CAPACITY | QHS_TIMEOUT;
  };
  int from = 0;
  while (from < np && !(S.status & QHS_CAPACITY)) {
    int ev_pos = np, ev_kind = 0, ev_dst = -1;
    double ev_d = 0.0;
    if (help) post(from);
    bool first = help;   // (the posted sequence's first chunk: claimed by the post)
    for (int c = from & ~63; c < np; c += 64) {
      Q3C(23, 1);
      const int pos = c + lane;
      const bool act = pos >= from && pos < np;
      int kind = 0, ls = 0, dst = -1, dfa = 0;
      double d = 0.0;
      HullPt pt = pre;
      int f = -1, isout = 0, trig = 0;
      bool mine = !help || first;
      if (help && !first) {
        // this chunk's results from a helper, or claimed and located here
        const int k = c >> 6, b = k % Q3_HR;
        int st = q3_ld_acq(&L.hr_st[b]);
        if (st != k + 1) {
          int m = 0;
          if (lane == 0) {
            unsigned e = __hip_atomic_load(&L.hctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if ((e & 0xffffu) == (unsigned)k)
              m = __hip_atomic_compare_exchange_strong(&L.hctl, &e, e + 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          mine = __builtin_amdgcn_readfirstlane(m) != 0;
#ifdef LQRO_QHULL_LONGPROF
          const unsigned long long tw0 = __builtin_amdgcn_s_memrealtime();
#endif
          if (!mine) st = q3_wait(&L.hr_st[b], k + 1, false);
#ifdef LQRO_QHULL_LONGPROF
          if (!mine) S.lp_hwait += __builtin_amdgcn_s_memrealtime() - tw0;
#endif
        }
#ifdef LQRO_QHULL_LONGPROF
        if (mine) S.lp_own++; else S.lp_got++;
#endif
        int kv = 0;
        if (!mine) {
          if (st != k + 1) { S.status |= QHS_CAPACITY | QHS_TIMEOUT; break; }
          const int fv = L.hr_f[64 * b + lane];
          kv = L.hr_k[64 * b + lane];
          ls = L.hr_ls[b];
          dst = fv == 0xffff ? -1 : fv;
          kind = act ? kv & 7 : 0;
          // (a new destination's index: dfa's bits; an old one's: QF_NEW clear)
          dfa = (kv & 8) ? 0 : (((kv >> 8) - 1) << 8) | QF_NEW;
          d = L.hr_d[64 * b + lane];
        }
      }
      first = false;
      Q3T(12);
      if (mine) q3_chunk_locate<false>(W, S, L, c, from, np, sharp, init, lane, pre, prestart, havepre ? 0 : -1, pt, f,
                                       d, isout, trig, ls, C0);
      Q3T(13);
      if (mine && act) {
        if (isout) {
          dst = f;
          dfa = q3_fa(W, L, f);
          if (!(dfa & QF_NEW) && (q3_cc(W, L, f) & 0xffffu) == 0 && !q3_in_movf(S, L, f)) kind |= 4;
        } else if (d >= -S.MAXcoplanar && d > S.max_outside) {
          kind |= 2;
        }
        if (trig) kind |= 1;
      }
      S.status |= qh_wave_or(ls);
      if (help && lane == 0) q3_st_rel_lds(&L.hcons, (c >> 6) + 1);   // (its buffer is read)
      const unsigned long long b = __ballot(kind != 0);
      const int last = b ? __ffsll((long long)b) - 1 : 63;   // positions up to c+last are final
      const bool fin = act && lane <= last;
      int g = -1;
      if (fin && dst >= 0 && (dfa & QF_NEW)) {
        g = dfa >> 8;
        atomicAdd(&L.pcnt[g], 1);
      }
      unsigned long long old = __ballot(fin && dst >= 0 && !(dfa & QF_NEW));
      while (old) {   // old facets: registered in sequence order (rare)
        const int l = __ffsll((long long)old) - 1;
        old &= old - 1;
        const int f = __builtin_amdgcn_readlane(dst, l);
        int k = -1;
        for (int t = 0; t < S.nold; t++)
          if (L.oldf[t] == f) k = t;
        if (k < 0) {
          if (S.nold == Q3_MOVCAP) { S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_MOV); continue; }
          k = S.nold++;
          if (lane == 0) { L.oldf[k] = f; L.pcnt[Q3_NEWCAP + k] = 0; L.dfac[Q3_NEWCAP + k] = f; }
          hl_sync();
        }
        if (lane == 0) L.pcnt[Q3_NEWCAP + k]++;
        if (lane == l) g = Q3_NEWCAP + k;
        hl_sync();
      }
      if (fin) {
        rg = g;
        rd = d;
        rpt = pt;
        if (np > 64) {   // (the point itself is read again from the sequence)
          W.pdst[pos] = g;
          W.pdd[pos] = d;
        }
      }
      hl_sync();
      Q3T(14);
      if (b) {
        ev_pos = c + last;
        ev_kind = __builtin_amdgcn_readlane(kind, last);
        ev_dst = __builtin_amdgcn_readlane(dst, last);
        ev_d = hl_rl(d, last);
        break;
      }
    }
#ifdef LQRO_QHULL_LONGPROF
    const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();
#endif
    if (help) stop();   // (the rest, if any, is posted again under the new state)
#ifdef LQRO_QHULL_LONGPROF
    if (help) { S.lp_stop += __builtin_amdgcn_s_memrealtime() - ts0; S.lp_posts++; if (ev_pos < np) S.lp_ev++; }
#endif
    if (S.status & QHS_CAPACITY) return;
    if (ev_pos < np) {
      Q3C(24, 1);
      if (ev_kind & 1) {
        if (sharp) S.findbestnew = 1;
        else S.notsharp = 1;
      }
      if (ev_kind & 2) S.max_outside = ev_d;
      if (ev_kind & 4) {
        // qh_partitionpoint: "make sure it's after qh.facet_next" — the old
        // facet moves behind the new ones (a fresh key)
        const int f = ev_dst;
        if (S.nmov == Q3_MOVCAP) {
          S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_MOV);
          return;
        }
        if (lane == 0) {
          L.movf[S.nmov] = f;
          if (init) {
            // the remainder's scan list is the facet list itself: f to its end
            int t0 = 0;
            for (int t = 0; t < S.nnew; t++)
              if (L.nslot[t] == f) t0 = t;
            for (int t = t0; t + 1 < S.nnew; t++) {
              L.nslot[t] = L.nslot[t + 1];
              for (int k = 0; k < 4; k++) L.npl[4 * t + k] = L.npl[4 * (t + 1) + k];
              L.nflag[t] = L.nflag[t + 1];
            }
            double q[4];
            q3_pl(W, L, f, q);
            L.nslot[S.nnew - 1] = f;
            for (int k = 0; k < 4; k++) L.npl[4 * (S.nnew - 1) + k] = q[k];
            L.nflag[S.nnew - 1] = q3_fa(W, L, f);
          }
        }
        q3_set_key(W, L, f, S.keyc);   // (every lane writes the same value)
        S.keyc++;
        S.nmov++;
      }
      hl_sync();
    }
    from = ev_pos + 1;
  }
}

// One bucket of a long sequence's emit (q3_emit_seq): the destinations i
// with i % 4 == b, their state in their lanes (destination i in lane i),
// every chunk of the sequence read, this bucket's destination groups placed
// in sequence order — the same placement as the single-wave loop, each
// destination's points by one wave
__device__ inline void q3_emit_bucket(const Q3W& W, Q3L& L, int lane, int b) {
  const int np = L.ej_np, nd = L.ej_nd, ndnew = L.ej_ndnew, nvis = L.ej_nvis;
  const bool init = L.ej_init != 0;
  const int gl = lane < ndnew ? lane : Q3_NEWCAP + (lane - ndnew);
  const bool has = lane < nd && (lane & 3) == b && L.pcnt[gl];
  int Rc = 0, Rch = -1, Ro = 0;
  double Rm = 0.0, Rx = 0.0, Ry = 0.0, Rz = 0.0;
  if (has) {
    Rc = L.dcnt[gl]; Rm = L.dmax[gl]; Rch = L.dchamp[gl]; Ro = L.doff[gl];
    Rx = L.dchp[3 * gl]; Ry = L.dchp[3 * gl + 1]; Rz = L.dchp[3 * gl + 2];
  }
  const unsigned long long ltmask = (1ull << lane) - 1ull;
  int ng = -1;
  double ndd = 0.0;
  HullPt npt;
  npt.x = npt.y = npt.z = 0.0; npt.q = -1; npt.pad = 0;
  auto ldc = [&](int c) {
    const int pos = c + lane;
    ng = -1;
    ndd = 0.0;
    if (pos < np) {
      ng = W.pdst[pos];
      ndd = W.pdd[pos];
      int st;
      npt = q3_seqpt(W, L, nvis, init, pos, &st);
    }
  };
  ldc(0);
  for (int c = 0; c < np; c += 64) {
    const int g = ng;
    const double dd = ndd;
    const HullPt pt = npt;
    if (c + 64 < np) ldc(c + 64);
    const int i = g < 0 ? -1 : (g < Q3_NEWCAP ? g : ndnew + (g - Q3_NEWCAP));
    const bool mine = i >= 0 && (i & 3) == b;
    unsigned long long todo = __ballot(mine);
    int wpos = -1, wr = 0;
    while (todo) {
      const int lead = __ffsll((long long)todo) - 1;
      const int gg = __builtin_amdgcn_readlane(g, lead);
      const unsigned long long grp = __ballot(mine && g == gg);
      todo &= ~grp;
      const int l = __builtin_amdgcn_readlane(i, lead);
      int cnt = __builtin_amdgcn_readlane(Rc, l), champ = __builtin_amdgcn_readlane(Rch, l);
      double mx = hl_rl(Rm, l), cx = hl_rl(Rx, l), cy = hl_rl(Ry, l), cz = hl_rl(Rz, l);
      q3_place(grp, lane, ltmask, dd, pt, __builtin_amdgcn_readlane(Ro, l), W.SB, cnt, mx, champ, cx, cy, cz, wpos,
               wr);
      if (lane == l) { Rc = cnt; Rm = mx; Rch = champ; Rx = cx; Ry = cy; Rz = cz; }
    }
    if (wpos >= 0) W.sb[wpos] = wr;
  }
  if (has) {
    L.dcnt[gl] = Rc; L.dmax[gl] = Rm; L.dchamp[gl] = Rch;
    L.dchp[3 * gl] = Rx; L.dchp[3 * gl + 1] = Ry; L.dchp[3 * gl + 2] = Rz;
  }
}

// claim the posted emit's next bucket (-1: none left)
__device__ __forceinline__ int q3_emit_claim(Q3L& L, int lane) {
  int k = -1;
  if (lane == 0) {
    for (;;) {
      unsigned v = (unsigned)q3_ld_acq(reinterpret_cast<const int*>(&L.ectl));
      if (v == 0u || (v & 0xffu) >= 4u) break;
      unsigned e = v;
      if (__hip_atomic_compare_exchange_strong(&L.ectl, &e, v + 1u, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP)) {
        k = (int)(v & 0xffu);
        break;
      }
    }
  }
  return __builtin_amdgcn_readfirstlane(k);
}

// waves 1-3: a bucket of a posted emit, if one is left
__device__ inline bool q3_emit_help(const Q3W& W, Q3L& L, int lane) {
  const unsigned v = (unsigned)q3_ld_acq(reinterpret_cast<const int*>(&L.ectl));
  if (v == 0u || (v & 0xffu) >= 4u) return false;
  const int k = q3_emit_claim(L, lane);
  if (k < 0) return false;
  q3_emit_bucket(W, L, lane, k);
  if (lane == 0) {
    // (its set entries before the count: wave 0 reads the count, then the
    // next partition and the other waves read the sets)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __hip_atomic_fetch_add(&L.edone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  return true;
}

// The located points into their destinations' outside sets, in sequence
// order, with Qhull's placement (lqro_qhull.hpp qh_emit_seq: the furthest
// point so far held aside, a displaced one stays where it was).  Old
// facets continue their set in a fresh segment.  ndnew: new-facet
// destinations (0 in qh_partitionall).  The new facets that received
// points, then the moved old facets, join the queue in key order.
__device__ inline void q3_emit_seq(const Q3W& W, Q3S& S, Q3L& L, int np, int ndnew, bool init, int lane, int rg,
                                   double rd, const HullPt& rpt) {
  if (S.status & QHS_CAPACITY) return;
  // One chunk with new-facet destinations only (the usual insertion): each
  // destination is one group of the chunk and starts from an empty set, so
  // its state lives in lane g from the segment scan to the queue, with no
  // LDS round trip per group.  The same placement and stores as below.
  if (!init && np <= 64 && S.nold == 0 && ndnew <= 64) {
    const int g = lane;
    int pc = 0, f = 0;
    if (g < ndnew) { f = L.nslot[g]; pc = L.pcnt[g]; }
    const int inc = q3_scan_add(pc);
    const int top = S.sbtop + __builtin_amdgcn_readlane(inc, 63);
    if (top > W.SB) {
      S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_SB);
      return;
    }
    const int doff = S.sbtop + inc - pc;
    S.sbtop = top;
    Q3T(15);
    int dcnt = 0, dchamp = -1;
    double dmax = 0.0, dx = 0.0, dy = 0.0, dz = 0.0;
    const unsigned long long ltmask = (1ull << lane) - 1ull;
    const int rgl = lane < np ? rg : -1;
    unsigned long long todo = __ballot(rgl >= 0);
    int wpos = -1, wr = 0;
    Q3T(16);
    while (todo) {
      const int lead = __ffsll((long long)todo) - 1;
      const int gg = __builtin_amdgcn_readlane(rgl, lead);
      const unsigned long long grp = __ballot(rgl == gg);
      todo &= ~grp;
      int cnt = 0, champ = -1;
      double mx = 0.0, cx = 0.0, cy = 0.0, cz = 0.0;
      q3_place(grp, lane, ltmask, rd, rpt, __builtin_amdgcn_readlane(doff, gg), W.SB, cnt, mx, champ, cx, cy, cz,
               wpos, wr);
      Q3C(25, 1);
      if (lane == gg) { dcnt = cnt; dmax = mx; dchamp = champ; dx = cx; dy = cy; dz = cz; }
    }
    if (wpos >= 0) W.sb[wpos] = wr;
    Q3T(17);
    // the furthest point ends each set
    if (g < ndnew && pc) {
      W.sb[doff + dcnt - 1] = dchamp;
      W.soff[f] = doff;
      W.fdist[f] = dmax;
      q3_set_cc(W, L, f, (unsigned)dcnt | ((unsigned)dchamp << 16));
    }
    // the queue: new facets with points in key order (a new facet's key is
    // this insertion's first key + its index, from the adoption)
    const bool has = g < ndnew && pc > 0;
    const unsigned long long b = __ballot(has);
    int qt = S.qtail;
    if (has) {
      const int at = qt + __popcll(b & ltmask);
      if (at < W.QC) {
        W.fq[at] = f;
        W.fqk[at] = S.key0_last + (unsigned)g;
        HullPt r;
        r.x = dx; r.y = dy; r.z = dz; r.q = dchamp; r.pad = 0;
        W.fqc[at] = r;
      }
    }
    qt += __popcll(b);
    if (qt > W.QC) S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_FACETS);
    S.qtail = qt;
    hl_sync();
    Q3T(18);
    return;
  }
  // segments: an exclusive scan of the destinations' sizes
  const int nd = ndnew + S.nold;
  int base = S.sbtop;
  for (int c0 = 0; c0 < nd; c0 += 64) {
    const int i = c0 + lane;
    int size = 0, g = -1, cnt0 = 0;
    if (i < nd) {
      g = i < ndnew ? i : Q3_NEWCAP + (i - ndnew);
      if (g < Q3_NEWCAP) L.dfac[g] = L.nslot[g];
      if (L.pcnt[g]) {
        cnt0 = g < Q3_NEWCAP ? 0 : (int)(q3_cc(W, L, L.dfac[g]) & 0xffffu);
        size = cnt0 + L.pcnt[g];
      }
    }
    const int inc = q3_scan_add(size);   // (DPP: no LDS round trips)
    if (size) {
      L.doff[g] = base + inc - size;
      L.dcnt[g] = cnt0;
      L.dmax[g] = 0.0;
      L.dchamp[g] = -1;
    }
    base += __builtin_amdgcn_readlane(inc, 63);
  }
  if (base > W.SB) {
    S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_SB);
    return;
  }
  S.sbtop = base;
  hl_sync();
  // old destinations (rare): their set so far, furthest point held aside
  for (int k = 0; k < S.nold; k++) {
    const int g = Q3_NEWCAP + k;
    const int f = L.dfac[g];
    const int cnt0 = L.dcnt[g];
    if (!L.pcnt[g] || !cnt0) continue;
    const int off0 = W.soff[f];
    const int off = L.doff[g];
    for (int t = lane; t < cnt0 - 1; t += 64) W.sb[off + t] = W.sb[off0 + t];
    const int chq = W.sb[off0 + cnt0 - 1];
    const double fd = W.fdist[f];
    if (lane == 0) {
      L.dchamp[g] = chq;
      L.dchp[3 * g] = W.Pr[3 * (size_t)chq]; L.dchp[3 * g + 1] = W.Pr[3 * (size_t)chq + 1];
      L.dchp[3 * g + 2] = W.Pr[3 * (size_t)chq + 2];
      L.dmax[g] = fd;
    }
    hl_sync();
  }
  hl_sync();
  Q3T(15);
  // a long sequence with at most 64 destinations: the destinations in four
  // buckets, placed by wave 0 and whichever helper waves are free
  if (np > 64 && nd <= 64 && (L.qflags & 16)) {
    S.egen = S.egen % 0xffffff + 1;
    if (lane == 0) {
      L.ej_np = np; L.ej_nd = nd; L.ej_ndnew = ndnew; L.ej_init = init ? 1 : 0; L.ej_nvis = S.nvis;
      L.edone = 0;
      // (a full release: pdst / pdd are global stores of this wave)
      q3_st_rel(reinterpret_cast<int*>(&L.ectl), (int)((unsigned)S.egen << 8));
    }
    int mine = 0;
    for (int k = q3_emit_claim(L, lane); k >= 0; k = q3_emit_claim(L, lane)) {
      q3_emit_bucket(W, L, lane, k);
      ++mine;
    }
    hl_sync();
    int dn = q3_ld_acq(&L.edone);
    for (long w = 0; dn != 4 - mine && w < (1l << 24); ++w) {
      __builtin_amdgcn_s_sleep(Q3_W0_SLEEP);
      dn = q3_ld_acq(&L.edone);
    }
    if (lane == 0) __hip_atomic_store(&L.ectl, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // a helper that never finished may still write: the build stops
    // (k_qhull_big rebuilds the pair)
    if (dn != 4 - mine) { S.status |= QHS_CAPACITY | QHS_TIMEOUT; return; }
  } else {
  // at most 64 destinations (the usual long sequence): destination i's state
  // in lane i (new facet i, then the old ones) from here to the end of the
  // sequence, read by the group with lane reads — no LDS round trip and no
  // wave barrier per destination group
  const bool inl = nd <= 64 && (L.qflags & 2);
  int Rc = 0, Rch = -1, Ro = 0;
  double Rm = 0.0, Rx = 0.0, Ry = 0.0, Rz = 0.0;
  if (inl && lane < nd) {
    const int g = lane < ndnew ? lane : Q3_NEWCAP + (lane - ndnew);
    if (L.pcnt[g]) {
      Rc = L.dcnt[g]; Rm = L.dmax[g]; Rch = L.dchamp[g]; Ro = L.doff[g];
      Rx = L.dchp[3 * g]; Ry = L.dchp[3 * g + 1]; Rz = L.dchp[3 * g + 2];
    }
  }
  // the sequence in order: a chunk's lanes, grouped by destination (a long
  // sequence's next chunk loaded while this one is placed)
  int ng = -1;
  double ndd = 0.0;
  HullPt npt = rpt;
  // (the three loads are independent: the point is read whatever its
  // destination, not behind a branch on the loaded one)
  auto ldc = [&](int c) {
    const int pos = c + lane;
    ng = -1;
    ndd = 0.0;
    if (pos < np) {
      ng = W.pdst[pos];
      ndd = W.pdd[pos];
      int st;
      npt = q3_seqpt(W, L, S.nvis, init, pos, &st);
    }
  };
  if (np > 64) ldc(0);
  for (int c = 0; c < np; c += 64) {
    const int pos = c + lane;
    const bool act = pos < np;
    int g = rg;
    double dd = rd;
    HullPt pt = rpt;
    if (np > 64) {   // (at most 64: the lanes' own results)
      g = ng;
      dd = ndd;
      pt = npt;
      if (c + 64 < np) ldc(c + 64);
    } else if (!act) {
      g = -1;
    }
    Q3T(16);
    unsigned long long todo = __ballot(g >= 0);
    const unsigned long long ltmask = (1ull << lane) - 1ull;
    int wpos = -1, wr = 0;
    while (todo) {
      const int lead = __ffsll((long long)todo) - 1;
      const int gg = __builtin_amdgcn_readlane(g, lead);
      const unsigned long long grp = __ballot(g == gg);
      todo &= ~grp;
      if (inl) {
        const int l = gg < Q3_NEWCAP ? gg : ndnew + (gg - Q3_NEWCAP);
        int cnt = __builtin_amdgcn_readlane(Rc, l), champ = __builtin_amdgcn_readlane(Rch, l);
        double mx = hl_rl(Rm, l), cx = hl_rl(Rx, l), cy = hl_rl(Ry, l), cz = hl_rl(Rz, l);
        q3_place(grp, lane, ltmask, dd, pt, __builtin_amdgcn_readlane(Ro, l), W.SB, cnt, mx, champ, cx, cy, cz, wpos,
                 wr);
        if (lane == l) { Rc = cnt; Rm = mx; Rch = champ; Rx = cx; Ry = cy; Rz = cz; }
      } else {
        int cnt = L.dcnt[gg];
        double mx = L.dmax[gg];
        int champ = L.dchamp[gg];
        double cx = L.dchp[3 * gg], cy = L.dchp[3 * gg + 1], cz = L.dchp[3 * gg + 2];
        const int off = L.doff[gg];
        q3_place(grp, lane, ltmask, dd, pt, off, W.SB, cnt, mx, champ, cx, cy, cz, wpos, wr);
        if (lane == 0) {
          L.dcnt[gg] = cnt; L.dmax[gg] = mx; L.dchamp[gg] = champ;
          L.dchp[3 * gg] = cx; L.dchp[3 * gg + 1] = cy; L.dchp[3 * gg + 2] = cz;
        }
        hl_sync();
      }
      Q3C(25, 1);
    }
    if (wpos >= 0) W.sb[wpos] = wr;
  }
  if (inl && lane < nd) {   // (the lanes' state back for the sets' ends and the queue)
    const int g = lane < ndnew ? lane : Q3_NEWCAP + (lane - ndnew);
    if (L.pcnt[g]) {
      L.dcnt[g] = Rc; L.dmax[g] = Rm; L.dchamp[g] = Rch;
      L.dchp[3 * g] = Rx; L.dchp[3 * g + 1] = Ry; L.dchp[3 * g + 2] = Rz;
    }
  }
  }   // (the single-wave emit)
  hl_sync();
  Q3T(17);
  // the furthest point ends each set
  for (int i = lane; i < nd; i += 64) {
    const int g = i < ndnew ? i : Q3_NEWCAP + (i - ndnew);
    if (!L.pcnt[g]) continue;
    const int f = L.dfac[g];
    W.sb[L.doff[g] + L.dcnt[g] - 1] = L.dchamp[g];
    W.soff[f] = L.doff[g];
    W.fdist[f] = L.dmax[g];
    q3_set_cc(W, L, f, (unsigned)L.dcnt[g] | ((unsigned)L.dchamp[g] << 16));
  }
  hl_sync();
  if (init) return;   // qh_partitionall: the queue is built after qh_furthestnext
  // the queue (qh.facet_next's walk): new facets with points in key order,
  // then the moved old facets in move order
  int qt = S.qtail;
  for (int c = 0; c < ndnew; c += 64) {
    const int t = c + lane;
    const bool has = t < ndnew && L.pcnt[t] > 0;
    const unsigned long long b = __ballot(has);
    if (has) {
      const int at = qt + __popcll(b & ((1ull << lane) - 1ull));
      if (at < W.QC) {
        W.fq[at] = L.nslot[t];
        W.fqk[at] = q3_key(W, L, L.nslot[t]);
        HullPt r;
        r.x = L.dchp[3 * t]; r.y = L.dchp[3 * t + 1]; r.z = L.dchp[3 * t + 2]; r.q = L.dchamp[t]; r.pad = 0;
        W.fqc[at] = r;
      }
    }
    qt += __popcll(b);
  }
  for (int t = lane; t < S.nmov; t += 64)
    if (qt + t < W.QC) {
      W.fq[qt + t] = L.movf[t];
      W.fqk[qt + t] = q3_key(W, L, L.movf[t]);
      HullPt r;
      r.x = r.y = r.z = 0.0; r.q = -1; r.pad = 0;   // (rare: the apex is read from the points)
      W.fqc[qt + t] = r;
    }
  qt += S.nmov;
  if (qt > W.QC) S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_FACETS);
  S.qtail = qt;
  hl_sync();
  Q3T(18);
}

// the slot of the t-th new facet: the visible facets' slots, then free
// ones, then fresh ones
__device__ __forceinline__ int q3_alloc(const Q3S& S, const Q3L& L, int t) {
  if (t < S.nvis) return L.visf[t];
  const int e = t - S.nvis;
  if (e < S.nfs) return L.fstk[S.nfs - 1 - e];
  return S.nalloc + (e - S.nfs);
}

// ---- wave 1: the next insertion, speculated (two-wave build) ----
// Handshake (LDS, workgroup scope): wave 0 publishes L.ph = k after insertion
// k's cone is built (the queue head and tail, the topology fixed until its
// partition ends); wave 1 speculates insertion k+1 — the queue's next live
// facet with points, its furthest point, qh_findhorizon, the cone's ridges
// and planes — and answers L.sp_done = k.  Insertion k's partition changes
// no neighbour link, plane or FLIPPED / TOP flag, so the speculated horizon
// and cone are exactly the sequential ones as long as the facet is still the
// queue's next with the same key and furthest point when wave 0 checks it.
// Wave 1 marks visited facets with its own epochs (no facet flag written).
// Wave 1's queue window: entries qcb .. qcb + qcn - 1 in its lanes (entries
// never change once written), across the speculations of one build.
struct Q3QC {
  int qcb, qcn, qf, qp;
  unsigned qk;
  double qx, qy, qz;
  // the last speculated cone when it took one ridge per lane: this lane's new
  // facet (rt, -1: none) and its ridge points, for its vertex record once
  // wave 0 adopts the cone (no reload of ncoord2 from global memory)
  int one, rt;
  double r[6];
  // the next speculation's queue entry, scanned after this one (q3_prescan):
  // from position pc_from (this speculation's facet), the first entry valid
  // then (pc_pos, facet pc_f, key pc_k, recorded furthest point pc_p at pc_x
  // .. pc_z), or none before pc_end (pc_pos = -1); pc_from = -1: no scan
  int pc_from, pc_pos, pc_end, pc_f, pc_p;
  unsigned pc_k;
  double pc_x, pc_y, pc_z;
};

__device__ inline void q3_spec(const Q3W& W, Q3L& L, int lane, unsigned short ep, unsigned ep2, Q3QC& Q, Q3P& P,
                               int phase) {
  const unsigned long long ltmask = (1ull << lane) - 1ull;
  Q3S C;   // the constants q3_plane reads
  C.MINvisible = L.c_dist[0]; C.MAXcoplanar = L.c_dist[1]; C.DISTround = L.c_dist[2];
  C.MINdenom = L.c_dist[3]; C.MINdenom_2 = L.c_dist[4];
  for (int k = 0; k < 3; k++) { C.NEARzero[k] = L.c_dist[5 + k]; C.interior[k] = L.c_interior[k]; }
  auto marked = [&](int f) -> bool {
    return f < Q3_FL ? q3_lds(L.mark[f]) == ep : q3_glb(W.mark2[f]) == ep2;
  };
  auto mark = [&](int f) {
    if (f < Q3_FL) q3_lds_st(L.mark[f], ep);
    else q3_glb_st(W.mark2[f], ep2);
  };
  // 0. the cone wave 0 adopted from the last speculation: its vertex records
  // (slots allocated by wave 0, points in this wave's ncoord2, apex in
  // sp_apex), before any of them is read
  if (L.pub_adopt) {
    const int nn = L.pub_nnew;
    if (Q.one) {
      if (Q.rt >= 0) {
        const int t = Q.rt;
        Q3V& v = W.vv[L.nslot[t]];
        *reinterpret_cast<double4*>(v.p) = make_double4(L.sp_apex[0], L.sp_apex[1], L.sp_apex[2], Q.r[0]);
        *reinterpret_cast<double4*>(v.p + 4) = make_double4(Q.r[1], Q.r[2], Q.r[3], Q.r[4]);
        *reinterpret_cast<double2*>(v.p + 8) = make_double2(Q.r[5], 0.0);
        *reinterpret_cast<int4*>(v.id) = make_int4(L.nv[3 * t], L.nv[3 * t + 1], L.nv[3 * t + 2], 0);
      }
    } else {
      for (int t = lane; t < nn; t += 64) {
        Q3V& v = W.vv[L.nslot[t]];
        const double* nc = W.ncoord2 + 9 * t;
        *reinterpret_cast<double4*>(v.p) = make_double4(L.sp_apex[0], L.sp_apex[1], L.sp_apex[2], nc[0]);
        *reinterpret_cast<double4*>(v.p + 4) = make_double4(nc[1], nc[2], nc[3], nc[4]);
        *reinterpret_cast<double2*>(v.p + 8) = make_double2(nc[5], 0.0);
        *reinterpret_cast<int4*>(v.id) = make_int4(L.nv[3 * t], L.nv[3 * t + 1], L.nv[3 * t + 2], 0);
      }
    }
    // (no wait for the stores here: the horizon reads no record; the fence
    // before the cone orders them)
  }
  Q.one = 0;
  Q.rt = -1;
  W1T(1);
#ifdef LQRO_QHULL_LONGPROF
  const unsigned long long tq0_ = __builtin_amdgcn_s_memrealtime();
  int reloads_ = 0;
#endif
  int ok = 0;
  // 1. the queue's next live facet with points (not one insertion k made visible)
  const int qt = L.pub_qtail;
  int facet = -1, furthest = -1, fpos = -1;
  unsigned fkey = 0;
  double apex[3] = {0.0, 0.0, 0.0};
  int qh0 = L.pub_qhead;
  if (Q.pc_from >= 0 && Q.pc_from == qh0 && L.pub_adopt) {
    // the entries q3_prescan found invalid stay invalid (a dead facet stays
    // dead, a key only changes to a fresh one — an old facet's first point
    // included —, and cc > 0 only ever comes with a fresh key), so its
    // candidate, checked now, is the scan's answer; else the scan resumes
    // after it
    if (Q.pc_pos >= 0) {
      const int fa = q3_fa(W, L, Q.pc_f);
      const unsigned c = q3_cc(W, L, Q.pc_f);
      if ((fa & QF_LIVE) && !(fa & QF_VISIBLE) && q3_key(W, L, Q.pc_f) == Q.pc_k && (c & 0xffffu) > 0) {
        fpos = Q.pc_pos;
        facet = Q.pc_f;
        fkey = Q.pc_k;
        furthest = (int)(c >> 16);
        if (Q.pc_p == furthest) {
          apex[0] = Q.pc_x; apex[1] = Q.pc_y; apex[2] = Q.pc_z;
        } else {
          apex[0] = W.Pr[3 * (size_t)furthest];
          apex[1] = W.Pr[3 * (size_t)furthest + 1];
          apex[2] = W.Pr[3 * (size_t)furthest + 2];
        }
      } else {
        qh0 = Q.pc_pos + 1;
      }
    } else {
      qh0 = max(qh0, Q.pc_end);
    }
  }
  Q.pc_from = -1;
  for (int qh = qh0; facet < 0 && qh < qt;) {
    if (qh >= Q.qcb + Q.qcn || qh < Q.qcb) {
#ifdef LQRO_QHULL_LONGPROF
      ++reloads_;
#endif
      Q.qcb = qh;
      Q.qcn = min(64, qt - qh);
      if (lane < Q.qcn) {
        Q.qf = W.fq[qh + lane];
        Q.qk = W.fqk[qh + lane];
        const HullPt e = W.fqc[qh + lane];
        Q.qx = e.x; Q.qy = e.y; Q.qz = e.z; Q.qp = e.q;
      }
    }
    bool good = false;
    unsigned c = 0;
    if (lane < Q.qcn && Q.qcb + lane >= qh && Q.qcb + lane < qt) {
      const int fa = q3_fa(W, L, Q.qf);
      c = q3_cc(W, L, Q.qf);
      good = (fa & QF_LIVE) && !(fa & QF_VISIBLE) && q3_key(W, L, Q.qf) == Q.qk && (c & 0xffffu) > 0;
    }
    const unsigned long long b = __ballot(good);
    if (b) {
      const int l = __ffsll((long long)b) - 1;
      fpos = Q.qcb + l;
      facet = __builtin_amdgcn_readlane(Q.qf, l);
      fkey = (unsigned)__builtin_amdgcn_readlane((int)Q.qk, l);
      furthest = (int)((unsigned)__builtin_amdgcn_readlane((int)c, l) >> 16);
      if (__builtin_amdgcn_readlane(Q.qp, l) == furthest) {
        apex[0] = hl_rl(Q.qx, l); apex[1] = hl_rl(Q.qy, l); apex[2] = hl_rl(Q.qz, l);
      } else {
        apex[0] = W.Pr[3 * (size_t)furthest];
        apex[1] = W.Pr[3 * (size_t)furthest + 1];
        apex[2] = W.Pr[3 * (size_t)furthest + 2];
      }
      break;
    }
    qh = Q.qcb + Q.qcn;
  }
  int ls = 0, nvis = 0, nnew = 0, ts = 0, lm = 0;
  W1T(2);
#ifdef LQRO_QHULL_LONGPROF
  const unsigned long long tq1_ = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) { L.hprof[8] += (unsigned long long)reloads_; L.hprof[9] += tq1_ - tq0_; }
#endif
  if (facet >= 0) {
    // 2. qh_findhorizon, as wave 0's (level order, first occurrence), visits as epochs
    if (lane == 0) L.sp_visf[0] = facet;
    if (lane < 3) L.sp_cand[lane] = (unsigned short)q3_nb(W, L, facet, lane);
    mark(facet);
    hl_sync();
    nvis = 1;
    bool cap = false;
    for (int lo = 0; lo < nvis && !cap;) {
      const int hi = nvis;
      const int ncand = 3 * (hi - lo);
      for (int c0 = 0; c0 < ncand; c0 += 64) {
        const int c = c0 + lane;
        int nb = -1;
        bool cand = false;
        double q[4] = {0.0, 0.0, 0.0, 0.0};
        int nn[3] = {0, 0, 0};
        if (c < ncand) {
          nb = L.sp_cand[3 * lo + c];
          int fa;
          q3_get(W, L, nb, q, nn, &fa);
          cand = !marked(nb);
        }
        const double dist = cand ? q3_distq(q, apex) : 0.0;
        bool vis = cand && dist >= C.MINvisible;
        if (cand && !vis && dist >= -C.MAXcoplanar) ls |= QHS_COPLANAR;
        bool dup = false;
        for (unsigned long long mm = __ballot(vis); mm;) {
          const int l = __ffsll((long long)mm) - 1;
          mm &= mm - 1;
          dup |= (l < lane) && __builtin_amdgcn_readlane(nb, l) == nb;
        }
        vis = vis && !dup;
        const unsigned long long bv = __ballot(vis);
        if (vis) {
          const int at = nvis + __popcll(bv & ltmask);
          if (at < Q3_VISCAP) {
            L.sp_visf[at] = nb;
            L.sp_cand[3 * at] = (unsigned short)nn[0];
            L.sp_cand[3 * at + 1] = (unsigned short)nn[1];
            L.sp_cand[3 * at + 2] = (unsigned short)nn[2];
          }
          mark(nb);
        }
        nvis += __popcll(bv);
        hl_sync();
      }
      lo = hi;
      if (nvis > Q3_VISCAP) cap = true;
#ifdef LQRO_QHULL_PROFILE
      P.t[11] += 1;
#endif
    }
#ifdef LQRO_QHULL_LONGPROF
    if (lane == 0) L.hprof[10] += __builtin_amdgcn_s_memrealtime() - tq1_;
#endif
    // the horizon to wave 2, which fetches the partition sequence's head
    if (!cap && lane == 0) {
      L.sp_hnvis = nvis;
      q3_st_rel_lds(&L.sp_hz, phase);   // (LDS only: wave 2 reads no global store of this wave)
    }
    W1T(3);
    // 3. the cone: one new facet per horizon ridge, as wave 0's
    const bool one = 3 * nvis <= 64;   // one ridge per lane: its points stay in registers
    int my_t = -1, rv1 = -1, rv2 = -1, mn1 = 0, mn2 = 0;
    double P1[3] = {0.0, 0.0, 0.0}, P2[3] = {0.0, 0.0, 0.0}, PO[3] = {0.0, 0.0, 0.0};
    double Q4[4] = {0.0, 0.0, 0.0, 0.0};   // (one pass) this lane's new facet's plane
    unsigned long long rb = 0ull;   // (one pass) the ridge lanes, in new-facet order
    if (!cap) {
      for (int vi = lane; vi < nvis; vi += 64) L.sp_repl[vi] = -1;
      hl_sync();
      for (int c0 = 0; c0 < 3 * nvis; c0 += 64) {
        const int c = c0 + lane;
        int vis = -1, nb = -1, hfa = 0;
        bool ridge = false;
        int hn[3] = {-1, -1, -1};
        if (c < 3 * nvis) {
          const int vi = c / 3;
          vis = L.sp_visf[vi];
          nb = L.sp_cand[c];
          q3_tp(W, L, nb, hn, &hfa);
          ridge = !marked(nb);
          if (c == 3 * vi) {
            const Q3V& vw = W.vv[vis];
            L.sp_vvert[3 * vi] = vw.id[0]; L.sp_vvert[3 * vi + 1] = vw.id[1]; L.sp_vvert[3 * vi + 2] = vw.id[2];
          }
        }
        const unsigned long long b = __ballot(ridge);
        if (one) rb = b;
        if (ridge) {
          const int t = nnew + __popcll(b & ltmask);
          const int hskip = hn[0] == vis ? 0 : hn[1] == vis ? 1 : hn[2] == vis ? 2 : -1;
          if (hskip < 0) {
            ts |= QHS_TOPOLOGY;
          } else if (t < Q3_NEWCAP) {
            const Q3V& h = W.vv[nb];
            const int top = (hfa & QF_TOP) ? (hskip & 1) : ((hskip & 1) ^ 1);
            const int i1 = hskip == 0 ? 1 : 0, i2 = hskip == 2 ? 1 : 2;
            double p1[3], p2[3], po[3];
            for (int k = 0; k < 3; k++) {
              p1[k] = h.p[3 * i1 + k];
              p2[k] = h.p[3 * i2 + k];
              po[k] = h.p[3 * hskip + k];
            }
            L.sp_v1[t] = h.id[i1];
            L.sp_v2[t] = h.id[i2];
            L.sp_nhz[t] = nb;
            L.sp_nhskip[t] = hskip;
            atomicMax(&L.sp_repl[c / 3], t);
            double q[4];
            bool flipped;
            int fl = QF_NEW | QF_LIVE | (top ? QF_TOP : 0);
            q3_plane(C, lm, apex, p1, p2, top, q, &flipped);
            if (flipped) { fl |= QF_FLIPPED; lm |= QHS_FLIPPED; }
            L.sp_nflag[t] = fl;
            L.sp_npl[4 * t] = q[0]; L.sp_npl[4 * t + 1] = q[1]; L.sp_npl[4 * t + 2] = q[2]; L.sp_npl[4 * t + 3] = q[3];
            if (one) {   // the ridge's points stay in this lane (no ncoord2)
              my_t = t;
              rv1 = h.id[i1];
              rv2 = h.id[i2];
              for (int k = 0; k < 4; k++) Q4[k] = q[k];
              for (int k = 0; k < 3; k++) { P1[k] = p1[k]; P2[k] = p2[k]; PO[k] = po[k]; }
            } else {
              for (int k = 0; k < 3; k++) {
                W.ncoord2[9 * t + k] = p1[k]; W.ncoord2[9 * t + 3 + k] = p2[k]; W.ncoord2[9 * t + 6 + k] = po[k];
              }
            }
          }
        }
        nnew += __popcll(b);
      }
      ok = nnew <= Q3_NEWCAP;
      if (one) {
        Q.one = 1;
        Q.rt = my_t;
        for (int k = 0; k < 3; k++) { Q.r[k] = P1[k]; Q.r[3 + k] = P2[k]; }
      }
      W1T(4);
      if (ok) {
        hl_sync();
        // qh_matchnewfacets (nb1: the other new facet with v2, nb2: with v1) and
        // qh_checkzero, as wave 0's
        if (one) {
          // the ridges are in the lanes in new-facet order: each lane walks
          // the others' vertex pairs with lane reads (no LDS round trips)
          int nbu[2] = {-1, -1}, cnt[2] = {0, 0};
          int u = 0;
          for (unsigned long long bb = rb; bb; bb &= bb - 1ull, ++u) {
            const int l = __ffsll((long long)bb) - 1;
            const int a = __builtin_amdgcn_readlane(rv1, l), c2 = __builtin_amdgcn_readlane(rv2, l);
            const bool o = u != my_t;
            if (o && (a == rv2 || c2 == rv2)) { nbu[0] = u; cnt[0]++; }
            if (o && (a == rv1 || c2 == rv1)) { nbu[1] = u; cnt[1]++; }
          }
          if (my_t >= 0) {
            if (cnt[0] != 1 || cnt[1] != 1) lm |= QHS_TOPOLOGY;
            mn1 = nbu[0] >= 0 ? nbu[0] : 0;
            mn2 = nbu[1] >= 0 ? nbu[1] : 0;
            L.sp_nn1[my_t] = mn1;
            L.sp_nn2[my_t] = mn2;
          }
        } else {
          for (int t = lane; t < nnew; t += 64) {
            int nbu[2] = {-1, -1}, cnt[2] = {0, 0};
            const int w0 = L.sp_v2[t], w1 = L.sp_v1[t];
#pragma unroll 4
            for (int u = 0; u < nnew; u++) {
              const int a = L.sp_v1[u], bb = L.sp_v2[u];
              const bool o = u != t;
              if (o && (a == w0 || bb == w0)) { nbu[0] = u; cnt[0]++; }
              if (o && (a == w1 || bb == w1)) { nbu[1] = u; cnt[1]++; }
            }
            if (cnt[0] != 1 || cnt[1] != 1) lm |= QHS_TOPOLOGY;
            L.sp_nn1[t] = nbu[0] >= 0 ? nbu[0] : 0;
            L.sp_nn2[t] = nbu[1] >= 0 ? nbu[1] : 0;
          }
        }
        hl_sync();
        W1T(12);
        if (!(qh_wave_or(lm) & QHS_FLIPPED)) {
          auto zero = [&](int t, const double* p1, const double* p2, const double* po) {
            const double d1 = q3_distq(L.sp_npl + 4 * L.sp_nn1[t], p1);
            const double d2 = q3_distq(L.sp_npl + 4 * L.sp_nn2[t], p2);
            const double d3 = q3_distq(L.sp_npl + 4 * t, po);
            if (d1 >= -2 * C.DISTround || d2 >= -2 * C.DISTround || d3 >= -2 * C.DISTround) lm |= QHS_NONCONVEX;
          };
          if (one) {   // (the lane's own plane and neighbours from registers)
            if (my_t >= 0) {
              const double4 a = q3_lds(*reinterpret_cast<const double4*>(L.sp_npl + 4 * mn1));
              const double4 b = q3_lds(*reinterpret_cast<const double4*>(L.sp_npl + 4 * mn2));
              const double qa[4] = {a.x, a.y, a.z, a.w}, qb[4] = {b.x, b.y, b.z, b.w};
              const double d1 = q3_distq(qa, P1), d2 = q3_distq(qb, P2), d3 = q3_distq(Q4, PO);
              if (d1 >= -2 * C.DISTround || d2 >= -2 * C.DISTround || d3 >= -2 * C.DISTround) lm |= QHS_NONCONVEX;
            }
          } else {
            for (int t = lane; t < nnew; t += 64) {
              double p1[3], p2[3], po[3];
              for (int k = 0; k < 3; k++) {
                p1[k] = W.ncoord2[9 * t + k]; p2[k] = W.ncoord2[9 * t + 3 + k]; po[k] = W.ncoord2[9 * t + 6 + k];
              }
              zero(t, p1, p2, po);
            }
          }
        }
        W1T(13);
        // qh_sharpnewfacets
        bool diff = false;
        if (one && rb) {   // the planes are in the ridge lanes; new facet 0's is the first's
          const int l0 = __ffsll((long long)rb) - 1;
          const bool q0 = hl_rl(Q4[0], l0) > 0, q1 = hl_rl(Q4[1], l0) > 0, q2 = hl_rl(Q4[2], l0) > 0;
          if (my_t >= 0) diff = (Q4[0] > 0) != q0 || (Q4[1] > 0) != q1 || (Q4[2] > 0) != q2;
        } else if (nnew > 0) {
          const bool q0 = L.sp_npl[0] > 0, q1 = L.sp_npl[1] > 0, q2 = L.sp_npl[2] > 0;
          for (int t = lane; t < nnew; t += 64) {
            const double* nn = L.sp_npl + 4 * t;
            diff |= (nn[0] > 0) != q0 || (nn[1] > 0) != q1 || (nn[2] > 0) != q2;
          }
        }
        const bool sh = __ballot(diff) != 0ull;
        if (lane == 0) L.sp_sharp = sh;
      }
    }
  }
  const int st = qh_wave_or(ls | ts | lm);
  W1T(5);
  hl_sync();
  Q.pc_end = qt;   // (q3_prescan's range: the entries this publication released)
  if (lane == 0) {
    L.sp_ok = ok;
    L.sp_facet = facet;
    L.sp_key = fkey;
    L.sp_furthest = furthest;
    L.sp_pos = fpos;
    L.sp_nvis = nvis;
    L.sp_nnew = nnew;
    L.sp_status = st;
    L.sp_apex[0] = apex[0]; L.sp_apex[1] = apex[1]; L.sp_apex[2] = apex[2];
  }
}

// Wave 1, after releasing speculation k+1 (while wave 0 partitions k and
// adopts k+1): the queue scan of speculation k+2, from k+1's facet, facets
// k+1 makes visible (this speculation's marks) counted as dead.  The facet
// fields are read while wave 0 changes them; q3_spec checks the candidate
// after the next publication (an entry found invalid here stays invalid).
__device__ inline void q3_prescan(const Q3W& W, Q3L& L, int lane, unsigned short ep, unsigned ep2, Q3QC& Q) {
  Q.pc_from = -1;
  const int from = L.sp_pos, qt = Q.pc_end;
  if (!L.sp_ok || L.sp_facet < 0 || from < 0) return;
  auto marked = [&](int f) -> bool {
    return f < Q3_FL ? q3_lds(L.mark[f]) == ep : q3_glb(W.mark2[f]) == ep2;
  };
  Q.pc_pos = -1;
  for (int qh = from; qh < qt;) {
    if (qh >= Q.qcb + Q.qcn || qh < Q.qcb) {
      Q.qcb = qh;
      Q.qcn = min(64, qt - qh);
      if (lane < Q.qcn) {
        Q.qf = W.fq[qh + lane];
        Q.qk = W.fqk[qh + lane];
        const HullPt e = W.fqc[qh + lane];
        Q.qx = e.x; Q.qy = e.y; Q.qz = e.z; Q.qp = e.q;
      }
    }
    bool good = false;
    if (lane < Q.qcn && Q.qcb + lane >= qh && Q.qcb + lane < qt) {
      const int fa = q3_fa(W, L, Q.qf);
      const unsigned c = q3_cc(W, L, Q.qf);
      good = (fa & QF_LIVE) && !marked(Q.qf) && q3_key(W, L, Q.qf) == Q.qk && (c & 0xffffu) > 0;
    }
    const unsigned long long b = __ballot(good);
    if (b) {
      const int l = __ffsll((long long)b) - 1;
      Q.pc_pos = Q.qcb + l;
      Q.pc_f = __builtin_amdgcn_readlane(Q.qf, l);
      Q.pc_k = (unsigned)__builtin_amdgcn_readlane((int)Q.qk, l);
      Q.pc_p = __builtin_amdgcn_readlane(Q.qp, l);
      Q.pc_x = hl_rl(Q.qx, l); Q.pc_y = hl_rl(Q.qy, l); Q.pc_z = hl_rl(Q.qz, l);
      break;
    }
    qh = Q.qcb + Q.qcn;
  }
  Q.pc_from = from;
}

// wave 2: the head of the next partition sequence (qh_partitionvisible: the
// visible facets' outside sets in visible order) for the horizon wave 1
// published, into LDS; the apex facet (visible facet 0) loses its furthest
// point when wave 0 adopts the insertion, so its set counts one less
__device__ inline void q3_prefetch(const Q3W& W, Q3L& L, int lane, int p) {
  const int nvis = L.sp_hnvis;
  int np = 0;
  for (int c0 = 0; c0 < nvis; c0 += 64) {
    const int vi = c0 + lane;
    int cnt = 0;
    if (vi < nvis) {
      const int f = L.sp_visf[vi];
      cnt = (int)(q3_cc(W, L, f) & 0xffffu) - (vi == 0 ? 1 : 0);
      L.pf_vsoff[vi] = W.soff[f];
      L.pf_vscnt[vi] = cnt;
    }
    np += __builtin_amdgcn_readlane(q3_scan_add(cnt), 63);
  }
  hl_sync();
  if (lane < np) {
    // the visible facet holding sequence position `lane`
    int a = 0, base = 0;
    for (;;) {
      const int k = L.pf_vscnt[a];
      if (lane < base + k || a == nvis - 1) break;
      base += k;
      ++a;
    }
    const int q = W.sb[L.pf_vsoff[a] + lane - base];
    HullPt r;
    r.x = W.Pr[3 * (size_t)q]; r.y = W.Pr[3 * (size_t)q + 1]; r.z = W.Pr[3 * (size_t)q + 2];
    r.q = q;
    r.pad = 0;
    L.pf_pre[lane] = r;
    L.pf_prea[lane] = (unsigned char)a;
  }
  hl_sync();
  if (lane == 0) {
    L.pf_np = np;
    q3_st_rel(&L.pf_done, p);
  }
}

// qh_qhull on W.Pr[0..n) (qconvex's defaults; lqro_qhull.hpp qh_build step
// for step)
__device__ inline void q3_build(const Q3W& W, Q3S& S, Q3L& L, int n, int lane) {
#ifdef LQRO_QHULL_PROFILE
  S.tq = __builtin_amdgcn_s_memtime();
#endif
  const unsigned long long ltmask = (1ull << lane) - 1ull;
  S.status = 0;
  S.nalloc = 1;
  S.nfs = 0;
  S.sbtop = 0;
  S.nnew = S.nvis = S.nmov = S.nold = 0;
  S.findbestnew = S.notsharp = 0;
  S.hgen = 0;
  S.egen = 0;
  S.keyc = 1;
  S.key0_last = 0;
  S.qhead = S.qtail = 0;
  if (W.FC > 65535) {   // 16-bit facet and point ids
    S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_FACETS);
    return;
  }
  // qh_maxmin
  int maxpoints[6];
  S.max_outside = 0.0;
  S.MAXabs_coord = 0.0;
  S.MAXwidth = -DBL_MAX;
  S.MAXsumcoord = 0.0;
  for (int k = 0; k < 3; k++) {
    int mn, mx;
    qh_extreme(W.Pr, n, k, false, lane, &mn);
    qh_extreme(W.Pr, n, k, true, lane, &mx);
    const double maxk = W.Pr[3 * (size_t)mx + k], mink = W.Pr[3 * (size_t)mn + k];
    const double maxcoord = fmax(maxk, -mink);
    const double temp = maxk - mink;
    if (temp > S.MAXwidth) S.MAXwidth = temp;
    if (maxcoord > S.MAXabs_coord) S.MAXabs_coord = maxcoord;
    S.MAXsumcoord += maxcoord;
    maxpoints[2 * k] = mn;
    maxpoints[2 * k + 1] = mx;
    S.NEARzero[k] = 80 * S.MAXsumcoord * DBL_EPSILON;
  }
  // qh_detroundoff (C-0)
  {
    double maxdistsum = sqrt(3.0) * S.MAXabs_coord;
    if (S.MAXsumcoord < maxdistsum) maxdistsum = S.MAXsumcoord;
    S.DISTround = DBL_EPSILON * (3 * maxdistsum * 1.01 + S.MAXabs_coord);
    const double MINdenom_1 = fmax(1.0 / DBL_MAX, DBL_MIN);
    S.MINdenom = MINdenom_1 * S.MAXabs_coord;
    S.MINdenom_2 = sqrt(MINdenom_1 * 3) * S.MAXabs_coord;
    S.MINvisible = 0.0 + 2 * S.DISTround;
    S.MAXcoplanar = S.MINvisible;
    S.MINoutside = 2 * S.MINvisible;
  }
  // qh_maxsimplex
  int simplex[4];
  {
    const QhS T = q3_as_qhs(S);
    double maxcoord = -DBL_MAX, mincoord = DBL_MAX;
    int minx = -1, maxx = -1;
    for (int i = 0; i < 6; i++) {
      const double c = W.Pr[3 * (size_t)maxpoints[i]];
      if (maxcoord < c) { maxcoord = c; maxx = maxpoints[i]; }
      if (mincoord > c) { mincoord = c; minx = maxpoints[i]; }
    }
    double maxdet = maxcoord - mincoord;
    int ns = 0;
    simplex[ns++] = minx;
    if (maxx != minx) simplex[ns++] = maxx;
    if (ns < 2) { S.status |= QHS_INPUT; return; }
    for (int i = 2; i < 4; i++) {
      const double prevdet = maxdet;
      int maxpoint = -1, maxnearzero = 0, nearzero;
      maxdet = -1.0;
      for (int m = 0; m < 6; m++) {
        const int p = maxpoints[m];
        bool ins = false;
        for (int t = 0; t < i; t++) ins |= simplex[t] == p;
        if (!ins && p != maxpoint) {
          const double det = fabs(qh_detsimplex(T, W.Pr, simplex, i, p, &nearzero));
          if (det > maxdet) { maxdet = det; maxpoint = p; maxnearzero = nearzero; }
        }
      }
      const double targetdet = prevdet * S.MAXwidth;
      const bool falsenarrow = maxdet > 0.0 && maxdet / targetdet < 1.0e-3;
      if (maxpoint < 0 || maxnearzero || falsenarrow) {
        double key = -1.0;
        int idx = 0x7fffffff;
        for (int q = lane; q < n; q += 64) {
          bool skip = false;
          for (int t = 0; t < 6; t++) skip |= maxpoints[t] == q;
          for (int t = 0; t < i; t++) skip |= simplex[t] == q;
          if (skip) continue;
          const double det = fabs(qh_detsimplex(T, W.Pr, simplex, i, q, &nearzero));
          if (det > key || (det == key && q < idx)) { key = det; idx = q; }
        }
        for (int off = 32; off >= 1; off >>= 1) {
          const double ok = __shfl_xor(key, off);
          const int oi = __shfl_xor(idx, off);
          if (ok > key || (ok == key && oi < idx)) { key = ok; idx = oi; }
        }
        if (idx != 0x7fffffff && key > maxdet) { maxdet = key; maxpoint = idx; }
      }
      if (maxpoint < 0) { S.status |= QHS_INPUT; return; }
      simplex[i] = maxpoint;
    }
  }
  // qh_initialvertices (the vertex set is [v4 v3 v2 v1], v_k = simplex[k-1]),
  // qh_createsimplex: facet slots 1..4, keys 1..4, facet i without vertex i
  const int pset[4] = {simplex[3], simplex[2], simplex[1], simplex[0]};
  int fs[4];
  {
    int top = 1, tops[4];
    for (int i = 0; i < 4; i++) {
      fs[i] = S.nalloc++;
      tops[i] = top;
      top ^= 1;
    }
    for (int k = 0; k < 3; k++) {
      double c = 0.0;
      for (int t = 0; t < 4; t++) c += W.Pr[3 * (size_t)pset[t] + k];
      S.interior[k] = c / 4;
    }
    int fv[4][3];
    for (int i = 0; i < 4; i++) {
      int m = 0;
      for (int t = 0; t < 4; t++)
        if (t != i) fv[i][m++] = pset[t];
    }
    // qh_initialhull: the first facet's orientation decides
    int ls = 0;
    double q[4][4];
    bool fl[4];
    q3_plane(S, ls, W.Pr + 3 * (size_t)fv[0][0], W.Pr + 3 * (size_t)fv[0][1], W.Pr + 3 * (size_t)fv[0][2], tops[0],
             q[0], &fl[0]);
    if (q3_distq(q[0], S.interior) > S.DISTround)
      for (int i = 0; i < 4; i++) tops[i] ^= 1;
    bool anyflip = false;
    for (int i = 0; i < 4; i++) {
      q3_plane(S, ls, W.Pr + 3 * (size_t)fv[i][0], W.Pr + 3 * (size_t)fv[i][1], W.Pr + 3 * (size_t)fv[i][2],
               tops[i], q[i], &fl[i]);
      anyflip |= fl[i];
    }
    if (anyflip) ls |= QHS_FLIPPED;
    int nbs[4][3];
    for (int i = 0; i < 4; i++) {
      int m = 0;
      for (int t = 0; t < 4; t++)
        if (t != i) nbs[i][m++] = fs[t];
    }
    double minangle = DBL_MAX;
    for (int i = 0; i < 4; i++)
      for (int t = 0; t < 3; t++) {
        int j = 0;
        for (int u = 0; u < 4; u++)
          if (fs[u] == nbs[i][t]) j = u;
        double angle = 0.0;
        for (int k = 0; k < 3; k++) angle += q[i][k] * q[j][k];
        if (angle < minangle) minangle = angle;
      }
    if (minangle < -0.99999999) ls |= QHS_NARROW;
    S.status |= ls;
    hl_sync();
    if (lane == 0)
      for (int i = 0; i < 4; i++) {
        const int f = fs[i];
        q3_set_facet(W, L, f, q[i], nbs[i][0], nbs[i][1], nbs[i][2],
                     QF_LIVE | (tops[i] ? QF_TOP : 0) | (fl[i] ? QF_FLIPPED : 0));
        q3_set_key(W, L, f, S.keyc + i);
        q3_set_cc(W, L, f, 0u);
        Q3V& v = W.vv[f];
        for (int t = 0; t < 3; t++) {
          for (int k = 0; k < 3; k++) v.p[3 * t + k] = W.Pr[3 * (size_t)fv[i][t] + k];
          v.id[t] = fv[i][t];
        }
      }
    S.keyc += 4;
    hl_sync();
    // qh_partitionall: every point but the simplex, in index order; each
    // facet in list order takes the ones at or beyond distoutside
    int np = 0;
    for (int c = 0; c < n; c += 64) {
      const int qi = c + lane;
      const bool ok = qi < n && qi != simplex[0] && qi != simplex[1] && qi != simplex[2] && qi != simplex[3];
      const unsigned long long b = __ballot(ok);
      if (ok) W.pq[np + __popcll(b & ltmask)] = qi;
      np += __popcll(b);
    }
    hl_sync();
    const double distoutside = fmax(2 * S.MINoutside, S.max_outside);
    for (int i = 0; i < 4; i++) {
      const int f = fs[i];
      int cnt = 0;
      const int off = S.sbtop;
      double mx = 0.0, cx = 0.0, cy = 0.0, cz = 0.0;
      int champ = -1, w = 0;
      for (int c = 0; c < np; c += 64) {
        const int pos = c + lane;
        HullPt pt;
        pt.x = pt.y = pt.z = 0.0;
        pt.q = -1;
        pt.pad = 0;
        double d = -DBL_MAX;
        if (pos < np) {
          pt.q = W.pq[pos];
          pt.x = W.Pr[3 * (size_t)pt.q]; pt.y = W.Pr[3 * (size_t)pt.q + 1]; pt.z = W.Pr[3 * (size_t)pt.q + 2];
          const double p[3] = {pt.x, pt.y, pt.z};
          d = q3_distq(q[i], p);
        }
        const bool out = pos < np && d >= distoutside;
        const bool keep = pos < np && !out;
        const unsigned long long bk = __ballot(keep);
        hl_sync();
        if (keep) W.pq[w + __popcll(bk & ltmask)] = pt.q;
        w += __popcll(bk);
        const unsigned long long bo = __ballot(out);
        if (bo) {
          int wpos = -1, wr = 0;
          q3_place(bo, lane, ltmask, d, pt, off, W.SB, cnt, mx, champ, cx, cy, cz, wpos, wr);
          if (wpos >= 0) W.sb[wpos] = wr;
        }
        hl_sync();
      }
      if (cnt) {
        if (off + cnt > W.SB) { S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_SB); return; }
        if (lane == 0) {
          W.sb[off + cnt - 1] = champ;
          W.soff[f] = off;
          W.fdist[f] = mx;
          q3_set_cc(W, L, f, (unsigned)cnt | ((unsigned)champ << 16));
        }
        S.sbtop += cnt;
      }
      np = w;
      hl_sync();
    }
    // the remainder: qh_partitionpoint with findbestnew from the head of the
    // facet list (MERGING): the scan list is the facet list
    if (np > 0) {
      S.nnew = 4;
      if (lane == 0)
        for (int i = 0; i < 4; i++) {
          L.nslot[i] = fs[i];
          for (int k = 0; k < 4; k++) L.npl[4 * i + k] = q[i][k];
          L.nflag[i] = q3_fa(W, L, fs[i]);
          L.nn1[i] = L.nn2[i] = 0;
        }
      S.nmov = 0;
      S.findbestnew = 1;
      hl_sync();
      int rg;
      double rd;
      HullPt rpt, pre;
      pre.x = pre.y = pre.z = 0.0;
      pre.q = -1;
      pre.pad = 0;
      q3_locate_seq(W, S, L, np, 0, true, lane, pre, 0, false, rg, rd, rpt);
      q3_emit_seq(W, S, L, np, 0, true, lane, rg, rd, rpt);
      S.findbestnew = 0;
      S.nnew = 0;
      S.nmov = 0;
      hl_sync();
    }
    if (S.status & (QHS_INPUT | QHS_TOPOLOGY | QHS_CAPACITY)) return;
    // qh_furthestnext: the first facet in list order with the furthest
    // outside point moves to the front (key 0); the queue: the facets with
    // points in list order
    {
      int order[4] = {fs[0], fs[1], fs[2], fs[3]};
      unsigned kk[4];
      for (int i = 0; i < 4; i++) kk[i] = q3_key(W, L, order[i]);
      for (int a = 0; a < 4; a++)
        for (int b = a + 1; b < 4; b++)
          if (kk[b] < kk[a]) {
            const unsigned tk = kk[a]; kk[a] = kk[b]; kk[b] = tk;
            const int to = order[a]; order[a] = order[b]; order[b] = to;
          }
      int best = -1;
      double bd = -DBL_MAX;
      for (int i = 0; i < 4; i++) {
        const int f = order[i];
        if ((q3_cc(W, L, f) & 0xffffu) && W.fdist[f] > bd) { best = f; bd = W.fdist[f]; }
      }
      hl_sync();
      if (best >= 0) {
        q3_set_key(W, L, best, 0u);
        for (int i = 0; i < 4; i++)
          if (order[i] == best) {
            for (int t = i; t > 0; t--) { order[t] = order[t - 1]; kk[t] = kk[t - 1]; }
            order[0] = best;
            kk[0] = 0;
            break;
          }
      }
      int qt = 0;
      for (int i = 0; i < 4; i++)
        if (q3_cc(W, L, order[i]) & 0xffffu) {
          if (lane == 0) {
            W.fq[qt] = order[i];
            W.fqk[qt] = kk[i];
            HullPt r;
            r.x = r.y = r.z = 0.0; r.q = -1; r.pad = 0;
            W.fqc[qt] = r;
          }
          qt++;
        }
      S.qhead = 0;
      S.qtail = qt;
      hl_sync();
    }
  }
  Q3T(0);
  // the constants wave 1's speculation needs (published with the first phase)
  if (lane == 0) {
    L.c_dist[0] = S.MINvisible; L.c_dist[1] = S.MAXcoplanar; L.c_dist[2] = S.DISTround;
    L.c_dist[3] = S.MINdenom; L.c_dist[4] = S.MINdenom_2;
    for (int k = 0; k < 3; k++) { L.c_dist[5 + k] = S.NEARzero[k]; L.c_interior[k] = S.interior[k]; }
  }
  int phase = 0;
  // qh_buildhull
  // the queue's next 64 entries stay in the lanes (lane k: entry qcb + k;
  // entries never change once written, appends go to the tail), with the
  // furthest point each facet had when it was queued
  int qcb = 0, qcn = 0;
  int qf = 0, qp = -1;
  unsigned qk = 0;
  double qx = 0.0, qy = 0.0, qz = 0.0;
  for (;;) {
#ifdef LQRO_QHULL_PROFILE
    unsigned long long snap_[21];
    for (int k = 0; k < 21; k++) snap_[k] = S.tph[k];
#endif
    // qh_nextfurthest: the first queued facet still alive (same key) with
    // points
    int facet = -1, furthest = -1;
    double apexp[3] = {0.0, 0.0, 0.0};
    // wave 1's speculation of this insertion: adopted when its facet is still
    // the queue's next live one with points and the same furthest point
    bool adopt = false;
    bool pfv = false;   // wave 2's prefetch of this insertion's partition sequence is used
    bool fast = false;  // adopted in one pass (below): the cone, slots and new facets are in place
    int nvis = 0, nnew = 0, lm = 0;
    const double* ncb = W.ncoord;
    HullPt pre;
    pre.x = pre.y = pre.z = 0.0;
    pre.q = -1;
    pre.pad = 0;
    int pfa = 0, pfnp = -1;
#ifdef LQRO_QHULL_LONGPROF
    const unsigned long long lp_ta = __builtin_amdgcn_s_memrealtime();
    S.lp_tail += S.lp_tw ? lp_ta - S.lp_tw : 0ull;
#endif
    if (phase > 0) {
#ifdef LQRO_QHULL_PROFILE
      const unsigned long long tw_ = __builtin_amdgcn_s_memtime();
#endif
#ifdef LQRO_QHULL_PROFILE
      int spins_ = 0;
      int dn = q3_ld_acq(&L.sp_done);
      const unsigned long long tf_ = __builtin_amdgcn_s_memtime();   // the first read back
      for (long w = 0; dn != phase && w < (1l << 24); ++w) {
        __builtin_amdgcn_s_sleep(Q3_W0_SLEEP);
        dn = q3_ld_acq(&L.sp_done);
        ++spins_;
      }
      if (S.prev1) { S.tfr += tf_ - tw_; S.nsp += (unsigned long long)spins_; }
#else
      const int dn = q3_wait(&L.sp_done, phase, false);
#endif
#ifdef LQRO_QHULL_LONGPROF
      {   // (wave 0 waited: the speculation's end -> seen here)
        const unsigned long long tn = __builtin_amdgcn_s_memrealtime();
        const unsigned long long de = q3_lds(L.lp_doner);
        if (tn - lp_ta > 20 && tn > de && lane == 0) { L.hprof[6] += tn - de; L.hprof[7] += 1; }
      }
#endif
#ifdef LQRO_QHULL_PROFILE
      {
        const unsigned long long tn_ = __builtin_amdgcn_s_memtime();
        S.tw += tn_ - tw_;
        S.nw += 1;
        if (tn_ - tw_ > 200) S.tdl += tn_ - L.done_t;   // (waited) speculation end -> seen here
        S.tseen = tn_;
        if (S.prev1) {   // after a one-chunk insertion: its wait, publication -> speculation end / -> seen
          S.tw1 += tn_ - tw_; S.nw1 += 1;
          S.tse += L.done_t - L.pub_t; S.tsn += tn_ - L.pub_t;
          S.tfr2 += L.done_t2 - L.pub_t;
          const unsigned long long nr_ = __builtin_amdgcn_s_memrealtime();
          S.r_start += L.start_r - L.pub_r; S.r_done += L.done_r - L.pub_r; S.r_seen += nr_ - L.pub_r;
        }
      }
#endif
#ifdef LQRO_QHULL_LONGPROF
      S.lp_wait += __builtin_amdgcn_s_memrealtime() - lp_ta;
#endif
      if (dn != phase) {   // wave 1 still speculating (it writes vertex records from L.nslot): stop
        S.status |= QHS_CAPACITY | QHS_TIMEOUT;
        return;
      }
      // The usual case, both lists within one pass of the lanes: the check
      // and the whole adoption — the speculated lists, the slots, the new
      // facets' fields — as one round of loads, one of dependent loads and
      // one of stores (the general path below goes a list at a time, a round
      // trip each).  The same values and the same store order as that path.
      {
        const int sok = L.sp_ok, F = L.sp_facet, sfur = L.sp_furthest, spos = L.sp_pos;
        const int snv = L.sp_nvis, snn = L.sp_nnew, sst = L.sp_status;
        const unsigned skey = L.sp_key;
        const double sax = L.sp_apex[0], say = L.sp_apex[1], saz = L.sp_apex[2];
        const int vf = L.sp_visf[lane], vr = L.sp_repl[lane];
        const int vv0 = L.sp_vvert[3 * lane], vv1 = L.sp_vvert[3 * lane + 1], vv2 = L.sp_vvert[3 * lane + 2];
        const int t1 = L.sp_v1[lane], t2 = L.sp_v2[lane], thz = L.sp_nhz[lane], thk = L.sp_nhskip[lane];
        const int tfl = L.sp_nflag[lane], tn1 = L.sp_nn1[lane], tn2 = L.sp_nn2[lane];
        const double4 tpl = q3_lds(*reinterpret_cast<const double4*>(L.sp_npl + 4 * lane));
        const int oldv = lane < Q3_MOVCAP ? L.oldf[lane] : -1;
        // wave 2's prefetch: its flag, then (in LDS issue order, which the
        // compiler keeps here) what it released with it
        const int pfd = hl_ld(&L.pf_done);
        hl_cfence();
        const int pso = L.pf_vsoff[lane], psc = L.pf_vscnt[lane], ppnp = L.pf_np, ppfa = L.pf_prea[lane];
        const HullPt ppre = L.pf_pre[lane];
        if (sok && F >= 0 && snv >= 1 && snv <= 64 && snn >= 1 && snn <= 64) {
          const unsigned c = q3_cc(W, L, F), k0 = q3_key(W, L, F);
          const int fa0 = q3_fa(W, L, F);
          int vfa = 0;
          unsigned vkey = 0u;
          if (lane < snv) { vfa = q3_fa(W, L, vf); vkey = q3_key(W, L, vf); }
          const int e = lane - snv;
          int fsl = 0;
          if (e >= 0 && e < S.nfs) fsl = L.fstk[S.nfs - 1 - e];
          adopt = (fa0 & QF_LIVE) && k0 == skey && (c & 0xffffu) > 0 && (int)(c >> 16) == sfur;
          if (adopt) {
            facet = F;
            furthest = sfur;
            apexp[0] = sax; apexp[1] = say; apexp[2] = saz;
            S.qhead = spos;
            q3_set_cc(W, L, F, (c & 0xffffu) - 1u);   // qh_setdellast
            nvis = snv;
            nnew = snn;
            bool bad = false;
            if (lane < nvis) {
              bad = vkey >= S.key0_last;
              for (int t = 0; t < S.nold; t++) bad |= __builtin_amdgcn_readlane(oldv, t) == vf;
            }
            pfv = pfd == phase && __ballot(bad) == 0ull;
            if (lane < nvis) {
              int so = pso, sc = psc;
              if (!pfv) {   // (F's count as just decremented)
                so = W.soff[vf];
                sc = vf == F ? (int)((c & 0xffffu) - 1u) : (int)(q3_cc(W, L, vf) & 0xffffu);
              }
              L.visf[lane] = vf;
              L.repl[lane] = vr;
              q3_set_fa(W, L, vf, vfa | QF_VISIBLE);
              L.vvert[3 * lane] = vv0; L.vvert[3 * lane + 1] = vv1; L.vvert[3 * lane + 2] = vv2;
              L.vsoff[lane] = so;
              L.vscnt[lane] = sc;
            }
            if (lane < nnew) {
              L.nv[3 * lane] = furthest; L.nv[3 * lane + 1] = t1; L.nv[3 * lane + 2] = t2;
              L.nhz[lane] = thz;
              L.nhskip[lane] = thk;
              L.nflag[lane] = tfl;
              L.nn1[lane] = tn1;
              L.nn2[lane] = tn2;
              q3_lds_st(*reinterpret_cast<double4*>(L.npl + 4 * lane), tpl);
            }
            S.status |= sst;
            S.nvis = nvis;
            lm = sst & QHS_FLIPPED;
            ncb = W.ncoord2;
            fast = true;
            if (!(S.status & (QHS_TOPOLOGY | QHS_CAPACITY))) {
              S.nnew = nnew;
              if (pfv) { pfnp = ppnp; pre = ppre; pfa = ppfa; }
              // slots: the visible facets', then free ones, then fresh ones (q3_alloc)
              const int extra = nnew > nvis ? nnew - nvis : 0;
              const int take = extra < S.nfs ? extra : S.nfs;
              if (S.nalloc + extra - take > W.FC) {
                S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_FACETS);
              } else {
                const int slot = lane < nvis ? vf : (e < S.nfs ? fsl : S.nalloc + (e - S.nfs));
                if (lane < nnew) L.nslot[lane] = slot;
                S.nfs -= take;
                S.nalloc += extra - take;
                // the new facets' fields (matched by wave 1), the horizon facets' links
                const unsigned key0 = S.keyc;
                const int s1 = __builtin_amdgcn_ds_bpermute(tn1 << 2, slot);
                const int s2 = __builtin_amdgcn_ds_bpermute(tn2 << 2, slot);
                if (lane < nnew) {
                  const double q[4] = {tpl.x, tpl.y, tpl.z, tpl.w};
                  q3_set_facet(W, L, slot, q, thz, s1, s2, tfl | (lane << 8));
                  q3_set_key(W, L, slot, key0 + (unsigned)lane);
                  q3_set_cc(W, L, slot, 0u);
                  q3_set_nb(W, L, thz, thk, slot);
                }
                S.keyc += (unsigned)nnew;
                S.key0_last = key0;
              }
            }
            hl_sync();
          }
        }
      }
      if (!fast && L.sp_ok) {
        const int F = L.sp_facet;
        const unsigned c = q3_cc(W, L, F);
        adopt = (q3_fa(W, L, F) & QF_LIVE) && q3_key(W, L, F) == L.sp_key && (c & 0xffffu) > 0 &&
                (int)(c >> 16) == L.sp_furthest;
        if (adopt) {
          facet = F;
          furthest = L.sp_furthest;
          apexp[0] = L.sp_apex[0]; apexp[1] = L.sp_apex[1]; apexp[2] = L.sp_apex[2];
          S.qhead = L.sp_pos;
          hl_sync();
          q3_set_cc(W, L, facet, (c & 0xffffu) - 1u);   // qh_setdellast
          hl_sync();
        }
      }
    }
    while (!adopt && S.qhead < S.qtail) {
      if (S.qhead >= qcb + qcn) {
        qcb = S.qhead;
        qcn = min(64, S.qtail - S.qhead);
        if (lane < qcn) {
          qf = W.fq[qcb + lane];
          qk = W.fqk[qcb + lane];
          const HullPt e = W.fqc[qcb + lane];
          qx = e.x; qy = e.y; qz = e.z; qp = e.q;
        }
      }
      bool ok = false;
      unsigned c = 0;
      if (lane < qcn && qcb + lane >= S.qhead) {
        const int fa = q3_fa(W, L, qf);
        c = q3_cc(W, L, qf);
        ok = (fa & QF_LIVE) && q3_key(W, L, qf) == qk && (c & 0xffffu) > 0;
      }
      const unsigned long long b = __ballot(ok);
      if (b) {
        const int l = __ffsll((long long)b) - 1;
        S.qhead = qcb + l;
        facet = __builtin_amdgcn_readlane(qf, l);
        const unsigned cf = (unsigned)__builtin_amdgcn_readlane((int)c, l);
        furthest = (int)(cf >> 16);
        if (__builtin_amdgcn_readlane(qp, l) == furthest) {
          apexp[0] = hl_rl(qx, l); apexp[1] = hl_rl(qy, l); apexp[2] = hl_rl(qz, l);
        } else {   // a further point arrived since (or none was recorded)
          apexp[0] = W.Pr[3 * (size_t)furthest];
          apexp[1] = W.Pr[3 * (size_t)furthest + 1];
          apexp[2] = W.Pr[3 * (size_t)furthest + 2];
        }
        hl_sync();
        q3_set_cc(W, L, facet, (cf & 0xffffu) - 1u);   // qh_setdellast (the facet is visible: no new furthest)
        hl_sync();
        break;
      }
      S.qhead = qcb + qcn;
    }
    Q3T(1);
#ifdef LQRO_QHULL_PROFILE
    const unsigned long long tins_ = S.tq;   // this insertion's start (for the long-sequence split)
#endif
    if (furthest < 0) {
      // the build is done: the selection reads vertex records wave 1 wrote
      if (phase > 0 && q3_wait(&L.sp_gdone, phase, false) != phase) S.status |= QHS_CAPACITY | QHS_TIMEOUT;
      break;
    }
    int ts = 0, my_t = -1;
    bool one = false;
    double P1[3] = {0.0, 0.0, 0.0}, P2[3] = {0.0, 0.0, 0.0}, PO[3] = {0.0, 0.0, 0.0};
    if (fast) {
      // (adopted above)
    } else if (adopt) {
      // the speculated visible set (flagged now) and cone
      nvis = L.sp_nvis;
      nnew = L.sp_nnew;
      // wave 2's copy of the visible facets' outside sets holds unless one of
      // them received points in the partition since (a destination then: a
      // new or moved facet of the last insertion, key >= key0_last, or an
      // old one listed in oldf)
      // (every LDS read of a lane is issued before its writes: the compiler
      // cannot tell the speculation's arrays from these and would otherwise
      // wait on each read in turn)
      const bool pfr = q3_ld_acq(&L.pf_done) == phase;
      if (nvis <= 64) {
        int f = 0, rp = 0, v0 = 0, v1 = 0, v2 = 0, pso = 0, psc = 0, fa = 0;
        unsigned key = 0u;
        bool bad = false;
        if (lane < nvis) {
          f = L.sp_visf[lane];
          rp = L.sp_repl[lane];
          v0 = L.sp_vvert[3 * lane]; v1 = L.sp_vvert[3 * lane + 1]; v2 = L.sp_vvert[3 * lane + 2];
          pso = L.pf_vsoff[lane];
          psc = L.pf_vscnt[lane];
          fa = q3_fa(W, L, f);
          key = q3_key(W, L, f);
          bad = key >= S.key0_last;
          for (int t = 0; t < S.nold; t++) bad |= L.oldf[t] == f;
        }
        pfv = pfr && __ballot(bad) == 0ull;
        if (lane < nvis) {
          int so = pso, sc = psc;
          if (!pfv) {
            so = W.soff[f];
            sc = (int)(q3_cc(W, L, f) & 0xffffu);
          }
          L.visf[lane] = f;
          L.repl[lane] = rp;
          q3_set_fa(W, L, f, fa | QF_VISIBLE);
          L.vvert[3 * lane] = v0; L.vvert[3 * lane + 1] = v1; L.vvert[3 * lane + 2] = v2;
          L.vsoff[lane] = so;
          L.vscnt[lane] = sc;
        }
      } else {
        for (int vi = lane; vi < nvis; vi += 64) {
          const int f = L.sp_visf[vi];
          L.visf[vi] = f;
          L.repl[vi] = L.sp_repl[vi];
          q3_set_fa(W, L, f, q3_fa(W, L, f) | QF_VISIBLE);
          L.vvert[3 * vi] = L.sp_vvert[3 * vi]; L.vvert[3 * vi + 1] = L.sp_vvert[3 * vi + 1];
          L.vvert[3 * vi + 2] = L.sp_vvert[3 * vi + 2];
          L.vsoff[vi] = W.soff[f];
          L.vscnt[vi] = (int)(q3_cc(W, L, f) & 0xffffu);
        }
      }
      for (int t = lane; t < nnew; t += 64) {
        const int a1 = L.sp_v1[t], a2 = L.sp_v2[t], hz = L.sp_nhz[t], hk = L.sp_nhskip[t], fl = L.sp_nflag[t];
        const int m1 = L.sp_nn1[t], m2 = L.sp_nn2[t];
        const double4 pl = q3_lds(*reinterpret_cast<const double4*>(L.sp_npl + 4 * t));
        L.nv[3 * t] = furthest; L.nv[3 * t + 1] = a1; L.nv[3 * t + 2] = a2;
        L.nhz[t] = hz;
        L.nhskip[t] = hk;
        L.nflag[t] = fl;
        L.nn1[t] = m1;
        L.nn2[t] = m2;
        q3_lds_st(*reinterpret_cast<double4*>(L.npl + 4 * t), pl);
      }
      S.status |= L.sp_status;
      S.nvis = nvis;
      lm = L.sp_status & QHS_FLIPPED;   // (qh_checkzero skips a cone with a flipped facet)
      ncb = W.ncoord2;
      hl_sync();
      Q3T(2);   // (profile: the adopted cone's copy)
    } else {
    // this cone reads vertex records, some of which wave 1 wrote
    if (phase > 0 && q3_wait(&L.sp_gdone, phase, false) != phase) {
      S.status |= QHS_CAPACITY | QHS_TIMEOUT;
      return;
    }
    // qh_findhorizon, a level of the breadth-first search at a time: the
    // candidates of a level in (visible facet, neighbour) order, a facet
    // taken at its first occurrence
    {
      const int fa0 = q3_fa(W, L, facet);
      hl_sync();
      if (lane == 0) L.visf[0] = facet;
      q3_set_fa(W, L, facet, fa0 | QF_VISIBLE);
      hl_sync();
    }
    int ls = 0;
    nvis = 1;
    for (int lo = 0; lo < nvis;) {
      const int hi = nvis;
      const int ncand = 3 * (hi - lo);
      for (int c0 = 0; c0 < ncand; c0 += 64) {
        const int c = c0 + lane;
        int nb = -1, fa = QF_VISIBLE;
        double q[4] = {0.0, 0.0, 0.0, 0.0};
        if (c < ncand) {
          nb = q3_nb(W, L, L.visf[lo + c / 3], c % 3);
          int nn[3];
          q3_get(W, L, nb, q, nn, &fa);
        }
        const bool cand = !(fa & QF_VISIBLE);
        const double dist = cand ? q3_distq(q, apexp) : 0.0;
        bool vis = cand && dist >= S.MINvisible;
        if (cand && !vis && dist >= -S.MAXcoplanar) ls |= QHS_COPLANAR;   // Qhull merges it: built on merge-free
        // a facet reached twice in this pass is taken at its first occurrence
        // (its copies compute the same distance: only visible ones matter)
        bool dup = false;
        for (unsigned long long mm = __ballot(vis); mm;) {
          const int l = __ffsll((long long)mm) - 1;
          mm &= mm - 1;
          dup |= (l < lane) && __builtin_amdgcn_readlane(nb, l) == nb;
        }
        vis = vis && !dup;
        const unsigned long long bv = __ballot(vis);
        if (vis) {
          const int at = nvis + __popcll(bv & ltmask);
          if (at < Q3_VISCAP) L.visf[at] = nb;
          q3_set_fa(W, L, nb, fa | QF_VISIBLE);
        }
        nvis += __popcll(bv);
        hl_sync();
      }
      lo = hi;
      if (nvis > Q3_VISCAP) { S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_VIS); return; }
    }
    S.status |= qh_wave_or(ls);
    S.nvis = nvis;
    Q3T(2);
    // qh_makenew_simplicial: one new facet per horizon ridge, created in
    // (visible facet, neighbour) order, its plane (qh_makenewplanes) made by
    // the ridge's lane from the horizon facet's vertex record; with it what
    // the visible facets' slots still hold.  When every ridge fits one pass
    // (3 nvis <= 64) the lane keeps its facet's points for qh_checkzero.
    for (int vi = lane; vi < nvis; vi += 64) L.repl[vi] = -1;
    hl_sync();
    one = 3 * nvis <= 64;
    for (int c0 = 0; c0 < 3 * nvis; c0 += 64) {
      const int c = c0 + lane;
      int vis = -1, nb = -1, hfa = QF_VISIBLE;
      int hn[3] = {-1, -1, -1};
      if (c < 3 * nvis) {
        const int vi = c / 3;
        vis = L.visf[vi];
        nb = q3_nb(W, L, vis, c - 3 * vi);
        q3_tp(W, L, nb, hn, &hfa);
        if (c == 3 * vi) {
          const Q3V& vw = W.vv[vis];
          L.vvert[3 * vi] = vw.id[0]; L.vvert[3 * vi + 1] = vw.id[1]; L.vvert[3 * vi + 2] = vw.id[2];
          L.vsoff[vi] = W.soff[vis];
          L.vscnt[vi] = (int)(q3_cc(W, L, vis) & 0xffffu);
        }
      }
      const bool ridge = !(hfa & QF_VISIBLE);
      const unsigned long long b = __ballot(ridge);
      if (ridge) {
        const int t = nnew + __popcll(b & ltmask);
        const int hskip = hn[0] == vis ? 0 : hn[1] == vis ? 1 : hn[2] == vis ? 2 : -1;
        if (hskip < 0) {
          ts |= QHS_TOPOLOGY;
        } else if (t < Q3_NEWCAP) {
          const Q3V& h = W.vv[nb];
          const int top = (hfa & QF_TOP) ? (hskip & 1) : ((hskip & 1) ^ 1);
          // the ridge: the horizon facet's vertices but the one opposite the visible facet
          const int i1 = hskip == 0 ? 1 : 0, i2 = hskip == 2 ? 1 : 2;
          double p1[3], p2[3], po[3];
          for (int k = 0; k < 3; k++) {
            p1[k] = h.p[3 * i1 + k];
            p2[k] = h.p[3 * i2 + k];
            po[k] = h.p[3 * hskip + k];
          }
          L.nv[3 * t] = furthest;
          L.nv[3 * t + 1] = h.id[i1];
          L.nv[3 * t + 2] = h.id[i2];
          L.nhz[t] = nb;
          L.nhskip[t] = hskip;
          atomicMax(&L.repl[c / 3], t);     // qh_getreplacement: the visible facet's last new facet
          double q[4];
          bool flipped;
          int fl = QF_NEW | QF_LIVE | (top ? QF_TOP : 0);
          q3_plane(S, lm, apexp, p1, p2, top, q, &flipped);
          if (flipped) { fl |= QF_FLIPPED; lm |= QHS_FLIPPED; }
          L.nflag[t] = fl;
          L.npl[4 * t] = q[0]; L.npl[4 * t + 1] = q[1]; L.npl[4 * t + 2] = q[2]; L.npl[4 * t + 3] = q[3];
          if (one) {
            my_t = t;
            for (int k = 0; k < 3; k++) { P1[k] = p1[k]; P2[k] = p2[k]; PO[k] = po[k]; }
          } else {
            for (int k = 0; k < 3; k++) {
              W.ncoord[9 * t + k] = p1[k]; W.ncoord[9 * t + 3 + k] = p2[k]; W.ncoord[9 * t + 6 + k] = po[k];
            }
          }
        }
      }
      nnew += __popcll(b);
    }
    Q3T(19);
    }   // (speculation adopted / computed here)
    S.status |= qh_wave_or(ts);
    if (nnew > Q3_NEWCAP) S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_NEW);
    if (S.status & (QHS_TOPOLOGY | QHS_CAPACITY)) return;
    S.nnew = nnew;
    hl_sync();
    // wave 2's head of the partition sequence, read before wave 1 may start
    // the next speculation (whose horizon restarts wave 2's prefetch)
    if (pfv && !fast) {
      pfnp = L.pf_np;
      pre = L.pf_pre[lane];
      pfa = L.pf_prea[lane];
    }
    if (!fast) {
      // slots: the visible facets', then free ones, then fresh ones
      const int extra = nnew > nvis ? nnew - nvis : 0;
      const int take = extra < S.nfs ? extra : S.nfs;
      if (S.nalloc + extra - take > W.FC) { S.status |= QHS_CAPACITY | Q3_CAPBIT(QHS_CAP_FACETS); return; }
      for (int t = lane; t < nnew; t += 64) L.nslot[t] = q3_alloc(S, L, t);
      S.nfs -= take;
      S.nalloc += extra - take;
      hl_sync();
    }
    Q3T(3);
    // qh_matchnewfacets (nb[1] shares {apex, v2}, nb[2] shares {apex, v1});
    // the new facets' fields and vertex records; the horizon facets' links
    const unsigned key0 = S.keyc;
    auto finish = [&](int t, const double* p1, const double* p2) {
      // nb1: the other new facet with v2, nb2: the other one with v1 (one pass)
      int nbu[2] = {-1, -1};
      if (adopt) {   // matched by wave 1 (a topology failure is in its status)
        nbu[0] = L.nn1[t];
        nbu[1] = L.nn2[t];
      } else {
        int cnt[2] = {0, 0};
        const int w0 = L.nv[3 * t + 2], w1 = L.nv[3 * t + 1];
#pragma unroll 4
        for (int u = 0; u < nnew; u++) {
          const int a = L.nv[3 * u + 1], b = L.nv[3 * u + 2];
          const bool o = u != t;
          if (o && (a == w0 || b == w0)) { nbu[0] = u; cnt[0]++; }
          if (o && (a == w1 || b == w1)) { nbu[1] = u; cnt[1]++; }
        }
        if (cnt[0] != 1 || cnt[1] != 1) lm |= QHS_TOPOLOGY;
        L.nn1[t] = nbu[0] >= 0 ? nbu[0] : 0;
        L.nn2[t] = nbu[1] >= 0 ? nbu[1] : 0;
      }
      // (every read before the first write: see the adoption above)
      const int s = L.nslot[t];
      const double4 q4 = q3_lds(*reinterpret_cast<const double4*>(L.npl + 4 * t));
      const int hz = L.nhz[t], hk = L.nhskip[t], fl = L.nflag[t], id1 = L.nv[3 * t + 1], id2 = L.nv[3 * t + 2];
      const int s1 = nbu[0] >= 0 ? L.nslot[nbu[0]] : 0, s2 = nbu[1] >= 0 ? L.nslot[nbu[1]] : 0;
      const double q[4] = {q4.x, q4.y, q4.z, q4.w};
      q3_set_facet(W, L, s, q, hz, s1, s2, fl | (t << 8));
      q3_set_key(W, L, s, key0 + (unsigned)t);
      q3_set_cc(W, L, s, 0u);
      if (!adopt) {   // (an adopted cone's records: wave 1 writes them from its copy)
        Q3V& v = W.vv[s];
        *reinterpret_cast<double4*>(v.p) = make_double4(apexp[0], apexp[1], apexp[2], p1[0]);
        *reinterpret_cast<double4*>(v.p + 4) = make_double4(p1[1], p1[2], p2[0], p2[1]);
        *reinterpret_cast<double2*>(v.p + 8) = make_double2(p2[2], 0.0);
        *reinterpret_cast<int4*>(v.id) = make_int4(furthest, id1, id2, 0);
      }
      q3_set_nb(W, L, hz, hk, s);
    };
    if (fast) {
      // (the new facets' fields written above)
    } else if (one) {
      if (my_t >= 0) finish(my_t, P1, P2);
    } else {
      for (int t = lane; t < nnew; t += 64) {
        double p1[3] = {0.0, 0.0, 0.0}, p2[3] = {0.0, 0.0, 0.0};
        if (!adopt)
          for (int k = 0; k < 3; k++) { p1[k] = ncb[9 * t + k]; p2[k] = ncb[9 * t + 3 + k]; }
        finish(t, p1, p2);
      }
    }
    if (!fast) {
      S.keyc += (unsigned)nnew;
      S.key0_last = key0;
    }
    hl_sync();
    // qh_checkzero: each new facet clearly convex to its neighbours (an
    // adopted cone's: wave 1's, in its status)
    if (!adopt && !(qh_wave_or(lm) & QHS_FLIPPED)) {
      auto zero = [&](int t, const double* p1, const double* p2, const double* po) {
        const double d1 = q3_distq(L.npl + 4 * L.nn1[t], p1);
        const double d2 = q3_distq(L.npl + 4 * L.nn2[t], p2);
        const double d3 = q3_distq(L.npl + 4 * t, po);
        if (d1 >= -2 * S.DISTround || d2 >= -2 * S.DISTround || d3 >= -2 * S.DISTround) lm |= QHS_NONCONVEX;
      };
      if (one) {
        if (my_t >= 0) zero(my_t, P1, P2, PO);
      } else {
        for (int t = lane; t < nnew; t += 64) {
          double p1[3], p2[3], po[3];
          for (int k = 0; k < 3; k++) {
            p1[k] = ncb[9 * t + k]; p2[k] = ncb[9 * t + 3 + k]; po[k] = ncb[9 * t + 6 + k];
          }
          zero(t, p1, p2, po);
        }
      }
    }
    S.status |= qh_wave_or(lm);
    Q3T(4);
    if (S.status & (QHS_TOPOLOGY | QHS_CAPACITY)) return;
    // the cone is built: wave 1 may speculate the next insertion meanwhile
    hl_sync();
    if (lane == 0) {
      L.pub_qhead = S.qhead;
      L.pub_qtail = S.qtail;
      L.pub_adopt = adopt ? 1 : 0;
      L.pub_nnew = nnew;
    }
    ++phase;
#ifdef LQRO_QHULL_PROFILE
    if (lane == 0) { L.pub_t = __builtin_amdgcn_s_memtime(); L.pub_r = __builtin_amdgcn_s_memrealtime(); }
    if (S.tseen) { S.tpre += __builtin_amdgcn_s_memtime() - S.tseen; S.npre += 1; }   // (this wave's clock) seen -> publication
#endif
#ifdef LQRO_QHULL_LONGPROF
    const unsigned long long lp_t0 = __builtin_amdgcn_s_memrealtime();
    S.lp_adopt += lp_t0 - lp_ta;   // (less the wait, in lp_wait)
    if (lane == 0) L.lp_pubr = lp_t0;
#endif
    if (lane == 0) q3_st_rel(&L.ph, phase);
#ifdef LQRO_QHULL_PROFILE
    if (lane == 0) S.trel += __builtin_amdgcn_s_memtime() - L.pub_t;   // the release's own cost
#endif
    S.findbestnew = 0;
    S.notsharp = 0;
    S.nmov = 0;
    // qh_partitionvisible's sequence: the visible facets' outside sets in
    // visible order (its extent and first 64 points: after the publication,
    // beside the next speculation)
    int np2 = 0;
    for (int c0 = 0; c0 < nvis; c0 += 64) {
      const int vi = c0 + lane;
      const int cnt = vi < nvis ? L.vscnt[vi] : 0;
      const int inc = q3_scan_add(cnt);
      if (vi < nvis) L.vinc[vi] = np2 + inc;
      np2 += __builtin_amdgcn_readlane(inc, 63);
    }
    hl_sync();
    int prestart = 0;
    if (pfv && np2 == pfnp) {   // wave 2's head of the sequence
      if (lane < np2) prestart = L.repl[pfa] >= 0 ? L.repl[pfa] : 0;
    } else if (lane < np2) {
      pre = q3_seqpt(W, L, nvis, false, lane, &prestart);
    }
    Q3T(5);
    const int sharp = adopt ? L.sp_sharp : q3_sharpnewfacets(S, L, lane);
    Q3T(20);
    Q3C(21, 1);
    S.nins++;
    Q3C(31, adopt ? 1 : 0);   // insertions whose horizon and cone wave 1 speculated
    Q3C(22, np2);
    if (np2) {
      int rg;
      double rd;
      HullPt rpt;
      q3_locate_seq(W, S, L, np2, sharp, false, lane, pre, prestart, true, rg, rd, rpt);
#ifdef LQRO_QHULL_LONGPROF
      if (np2 > 64) S.lp_tloc += __builtin_amdgcn_s_memrealtime() - lp_t0;
#endif
      Q3T(6);
      q3_emit_seq(W, S, L, np2, nnew, false, lane, rg, rd, rpt);
      Q3T(7);
    }
#ifdef LQRO_QHULL_LONGPROF
    {
      const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - lp_t0;
      S.lp_all += dt;
      if (np2 > 64) { S.lp_n += 1; S.lp_pts += (unsigned long long)np2; S.lp_t += dt; }
      S.lp_tw = lp_t0 + dt;
    }
#endif
    if (S.status & QHS_CAPACITY) return;
    // deleted vertices (a visible facet's vertex on no new facet) close to a
    // new facet: Qhull's qh_partitioncoplanar would act (not restated).  The
    // visible facets are a region of the triangulated sphere (genus 0) whose
    // boundary is the horizon, one edge per new facet, and qh_matchnewfacets
    // passed, so every boundary vertex is on exactly two horizon edges.  Euler:
    // its interior vertices number 2 - b + (nvis - nnew) / 2 with b boundary
    // cycles, so nnew == nvis + 2 forces b = 1 and none: no deleted vertex is
    // possible then (97 % of the C3 insertions) and the search is skipped
    if (nnew != nvis + 2) {
      int lsd = 0;
      for (int t = lane; t < 3 * nvis; t += 64) {
        const int v = L.vvert[t];
        bool skip = false;
        for (int u = 0; u < nnew && !skip; u++) skip = L.nv[3 * u + 1] == v || L.nv[3 * u + 2] == v;
        for (int e = 0; e < t && !skip; e++) skip = L.vvert[e] == v;
        if (skip) continue;
        const double p[3] = {W.Pr[3 * (size_t)v], W.Pr[3 * (size_t)v + 1], W.Pr[3 * (size_t)v + 2]};
        double d;
        int iso, trig;
        q3_locate<false>(W, S, L, p, 0, 2, &d, &iso, &trig, lsd, q3_col0(L, lane));
        if (d >= -S.MAXcoplanar) lsd |= QHS_COPLANAR;
      }
      S.status |= qh_wave_or(lsd);
    }
    Q3T(8);
    if (S.status & QHS_CAPACITY) return;
    // qh_deletevisible: the visible slots no new facet took are freed; the
    // new facets become old
    for (int t = nnew + lane; t < nvis; t += 64) {
      const int f = L.visf[t];
      q3_set_fa(W, L, f, 0);
      const int at = S.nfs + (t - nnew);
      if (at < Q3_FSTK) L.fstk[at] = (unsigned short)f;
    }
    if (nvis > nnew) S.nfs = min(Q3_FSTK, S.nfs + (nvis - nnew));
    for (int t = lane; t < nnew; t += 64) q3_set_fa(W, L, L.nslot[t], L.nflag[t] & ~QF_NEW);
    S.nnew = 0;
    S.nmov = 0;
    S.findbestnew = 0;
    S.notsharp = 0;
    hl_sync();
    Q3T(9);
#ifdef LQRO_QHULL_PROFILE
    // insertions whose partition sequence is longer than one chunk: 29 cycles, 30 count
    S.prev1 = np2 <= 64;
    if (np2 > 64) { S.tph[29] += S.tq - tins_; S.tph[30] += 1; }
    else {
      for (int k = 0; k < 21; k++) S.tps[k] += S.tph[k] - snap_[k];
      S.nps += 1;
    }
#endif
  }
}

// LQRO_REC_QHMERGE_WIN (a build where Qhull's merge tests fired): does a
// facet that can decide the rule — one within 1e-6 of the winning distance,
// or facet 0 (the list head: its merge would change which facet keeps the
// loop-carried normal) — have a hull vertex other than its own within
// LQRO_QHMERGE_K x qh DISTround of its plane: a facet qconvex's pre-merge
// (centrum radius, coplanar horizon and qh_checkzero all at 2 DISTround for
// C-0) may have joined with a neighbour, so that the reference's winner may
// be a merged facet?  The same test as the oracle's (lqro_oracle.c
// orc_hull_branch_ref); wave-uniform.  (Round 5 reached 1e-9 (|coord|max +
// 1), ~1e6 DISTround: C5 flagged 216 of 4,867 sampled inside pairs, none of
// 48 checked against live Qhull merged at the winner; this reach flags 1.)
__device__ inline bool q3_merge_suspect(const Q3W& W, const Q3L& L, const Q3S& S, int lane, const double* vrel,
                                        double best, int head) {
  const double T = -LQRO_QHMERGE_K * S.DISTround;
  bool sus = false;
  for (int f0 = 1; f0 < S.nalloc; f0 += 64) {
    const int f = f0 + lane;
    double q[4] = {0.0, 0.0, 0.0, 0.0};
    bool con = false;
    if (f < S.nalloc && (q3_fa(W, L, f) & QF_LIVE)) {
      q3_pl(W, L, f, q);
      const double* P = W.Pf + 3 * (size_t)W.vv[f].id[0];
      con = fabs(q[0] * (vrel[0] - P[0]) + q[1] * (vrel[1] - P[1]) + q[2] * (vrel[2] - P[2])) <= best + 1e-6 ||
            f == head;
    }
    unsigned long long m = __ballot(con);
    while (m) {
      const int src = __ffsll((long long)m) - 1;
      m &= m - 1;
      const int fc = __shfl(f, src);
      double qc[4];
      for (int k = 0; k < 4; k++) qc[k] = __shfl(q[k], src);
      const int a = W.vv[fc].id[0], b = W.vv[fc].id[1], c = W.vv[fc].id[2];
      for (int g = 1 + lane; g < S.nalloc; g += 64) {
        if (!(q3_fa(W, L, g) & QF_LIVE)) continue;
        for (int t = 0; t < 3; t++) {
          const int id = W.vv[g].id[t];
          if (id == a || id == b || id == c) continue;
          if (q3_distq(qc, W.Pr + 3 * (size_t)id) >= T) sus = true;
        }
      }
    }
  }
  return __ballot(sus) != 0;
}

// the reference's selection (LQRO:925-968; lqro_qhull.hpp qh_select) over
// the finished hull: Qhull's facet order is key order, so a tie goes to the
// smaller key and facet 0 is the smallest key alive.  The planes are the ones
// convexHull reads back (16 significant digits, lqro_dec16.hpp): a first pass
// at full precision bounds every facet's distance within rounding (qsel_bound),
// a second one evaluates the facets that can still be the minimum with the
// read-back planes
// returns (wave-uniform) whether this job closed its row and claimed the
// row's LP (hull_row_done)
__device__ inline bool q3_select(const HullArgs& A, const Q3W& W, const Q3L& L, const Q3S& S, int lane,
                                 const double* xi, const double* vrel, int slot) {
  const bool fail = (S.status & (QHS_INPUT | QHS_TOPOLOGY | QHS_CAPACITY)) != 0;
  double ub = INFINITY;
  unsigned minkey = 0xffffffffu;
  int nfac = 0, head = -1;   // (head: the live facet of the smallest key, Qhull's facet 0)
  if (!fail) {
    for (int f0 = 1; f0 < S.nalloc; f0 += 256) {
      // four slots a lane: their first vertices' points in one round trip
      int fs[4], fa[4], v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        fs[u] = f0 + 64 * u + lane;
        fa[u] = fs[u] < S.nalloc ? q3_fa(W, L, fs[u]) : 0;
        v[u] = (fa[u] & QF_LIVE) ? W.vv[fs[u]].id[0] : 0;
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (!(fa[u] & QF_LIVE)) continue;
        const int f = fs[u];
        nfac++;
        const unsigned k = q3_key(W, L, f);
        if (k < minkey) { minkey = k; head = f; }
        double q[4];
        q3_pl(W, L, f, q);
        const double* P = W.Pf + 3 * (size_t)v[u];
        double b;
        const double d = qsel_dist(q, P, vrel, &b);
        ub = fmin(ub, d + b);
      }
    }
  }
  for (int off = 32; off >= 1; off >>= 1) {
    const unsigned om = (unsigned)__shfl_xor((int)minkey, off);
    const int oh = __shfl_xor(head, off);
    nfac += __shfl_xor(nfac, off);
    if (om < minkey) { minkey = om; head = oh; }
    ub = fmin(ub, __shfl_xor(ub, off));
  }
  // the facets within rounding of the minimum, with the read-back planes
  double best = INFINITY, bn[3] = {0.0, 0.0, 0.0};
  unsigned bkey = 0xffffffffu;
  int bf = -1;
  if (!fail) {
    for (int f = 1 + lane; f < S.nalloc; f += 64) {
      if (!(q3_fa(W, L, f) & QF_LIVE)) continue;
      double q[4];
      q3_pl(W, L, f, q);
      const double* P = W.Pf + 3 * (size_t)W.vv[f].id[0];
      double b;
      const double d0 = qsel_dist(q, P, vrel, &b);
      if (d0 - b > ub) continue;
      double n16[3];
      const double d = qsel_dist16(q, P, vrel, n16);
      const unsigned k = q3_key(W, L, f);
      if (d < best || (d == best && k < bkey)) {
        best = d; bkey = k; bf = f;
        bn[0] = n16[0]; bn[1] = n16[1]; bn[2] = n16[2];
      }
    }
  }
  for (int off = 32; off >= 1; off >>= 1) {
    const double ob = __shfl_xor(best, off);
    const unsigned ok = (unsigned)__shfl_xor((int)bkey, off);
    const int of = __shfl_xor(bf, off);
    const double o0 = __shfl_xor(bn[0], off), o1 = __shfl_xor(bn[1], off), o2 = __shfl_xor(bn[2], off);
    if (ob < best || (ob == best && ok < bkey)) { best = ob; bkey = ok; bf = of; bn[0] = o0; bn[1] = o1; bn[2] = o2; }
  }
  const bool ok = !fail && nfac > 0 && bf >= 0;
  const bool stale = ok && bkey == minkey;
  const bool merged = (S.status & (QHS_COPLANAR | QHS_NONCONVEX | QHS_FLIPPED | QHS_NARROW | QHS_SINGULAR)) != 0;
  const bool mwin = ok && merged && q3_merge_suspect(W, L, S, lane, vrel, best, head);
  int bv[3] = {0, 0, 0};
  if (ok)
    for (int t = 0; t < 3; t++) bv[t] = W.vv[bf].id[t];
  int go = 0;
  if (lane == 0) {
    float* pl = A.planes + (size_t)slot * 8;
    double* qn = A.qnrm + (size_t)slot * 4;
    double nrm[3] = {0.0, 0.0, 0.0};
    if (ok && !stale) {
      nrm[0] = bn[0]; nrm[1] = bn[1]; nrm[2] = bn[2];
      const double dh = best * 0.5;                      // :1416
      const double mult = 1.0;                           // :1213
      pl[0] = (float)(xi[3] + mult * dh * nrm[0]);
      pl[1] = (float)(xi[4] + mult * dh * nrm[1]);
      pl[2] = (float)(xi[5] + mult * dh * nrm[2]);
      pl[3] = (float)nrm[0]; pl[4] = (float)nrm[1]; pl[5] = (float)nrm[2];
      pl[6] = __int_as_float(1);
      qn[0] = nrm[0]; qn[1] = nrm[1]; qn[2] = nrm[2]; qn[3] = best;
      atomicAdd(&A.stats[3], 1ull);
    } else if (stale) {
      pl[6] = __int_as_float(3);                         // pending: the loop-carried normal (k_stale)
      qn[0] = qn[1] = qn[2] = 0.0; qn[3] = best;
      const int k = atomicAdd(A.qstale_count, 1);
      if (k < A.qstale_cap) A.qstale[k] = slot;
      atomicAdd(&A.stats[3], 1ull);
    } else {
      pl[6] = __int_as_float(0);
      hull_fail_note(A.stats, slot);
    }
    if (ok && merged) atomicAdd(&A.stats[LQRO_ST_MERGED], 1ull);
    if (mwin) qhmerge_note(A.stats, slot);
    if (A.recs) {
      lqro_pair_record& rec = A.recs[slot];
      rec.flags |= ok ? LQRO_REC_HULL : LQRO_REC_HULLFAIL;
      if (stale) rec.flags |= LQRO_REC_STALE;
      if (merged) rec.flags |= LQRO_REC_QHMERGE;
      if (mwin) rec.flags |= LQRO_REC_QHMERGE_WIN;
      rec.n_facets = ok ? nfac : -(S.status & 0xffff) - 1;
      if (ok) {
        rec.facet[0] = bv[0]; rec.facet[1] = bv[1]; rec.facet[2] = bv[2];
        rec.dist = best;
        for (int q = 0; q < 3; ++q) {
          rec.normal[q] = nrm[q];
          rec.plane_point[q] = stale ? 0.0f : pl[q];
          rec.plane_normal[q] = stale ? 0.0f : pl[3 + q];
        }
      }
    }
    go = hull_row_done(A, slot, stale, A.row_lp != 0);
  }
  hl_sync();
  return __builtin_amdgcn_readfirstlane(go) != 0;
}

// calculateNewV (LQRO:1223-1234) for the row a job closed (hull_row_done),
// wave 0, in the LDS of the facet planes (the build is over): the row's
// planes and linearProgram4's projections, 32 B each (the runtime enables
// the early LP only where 2 * npr * 32 B fit)
__device__ inline void q3_row_lp(const HullArgs& A, Q3L& L, int slot, int lane) {
  static_assert(sizeof(L.pl) >= 2 * LQRO_EARLY_LP_MAX_NPR * 32, "q3_row_lp: the planes must fit");
  const int lrow = slot / A.npr;
  const int i = A.row_begin + lrow * A.row_stride;
  float* planes = reinterpret_cast<float*>(L.pl);
  float* proj = planes + (size_t)A.npr * 8;
  __threadfence();   // the row's planes other workgroups wrote (acquire)
  const int m = lp_compact<8>(A.planes + (size_t)lrow * A.npr * 8, A.npr, planes, lane);
  const v3 pref = V3((float)A.lp_vgoal[3 * i], (float)A.lp_vgoal[3 * i + 1], (float)A.lp_vgoal[3 * i + 2]);
  v3 nv = V3(0.0f, 0.0f, 0.0f);
  const int fail = w_lp3<8>(planes, m, A.lp_vmax, pref, false, nv, lane);       // :1228
  if (fail < m) w_lp4<8>(planes, m, fail, (float)A.lp_vmax, nv, proj, lane);    // :1230
  if (lane == 0) {
    A.lp_newv[3 * i] = nv.x;
    A.lp_newv[3 * i + 1] = nv.y;
    A.lp_newv[3 * i + 2] = nv.z;
  }
  hl_sync();
}

// A build past k_qhull's caps, rebuilt at once on the same CU by k_qhull_big's
// code (qh_build: topology in global memory, caps 2,048 visible / 1,024 new
// facets) in the LDS the k_qhull build used (LB aliases L), instead of
// waiting in the retry queue for the k_qhull_big launch after the sweep —
// C5's largest hulls (~19,000 points) hit k_qhull's caps within ~25 ms and
// then waited ~4.5 s for that launch (profiles/r6c_c5_shard_timeline.txt).
// Every wave takes part in hull_points (workgroup barriers), wave 0 builds
// and selects; the record names kernel 1 and starts at the job's start.
#ifdef LQRO_QBIG_NOINLINE
__device__ __attribute__((noinline)) void q3_big_inline(const HullArgs& A, QhL& LB, int slot, unsigned long long tjob,
                                                        int wave) {
#else
__device__ inline void q3_big_inline(const HullArgs& A, QhL& LB, int slot, unsigned long long tjob, int wave) {
#endif
  const int lane = threadIdx.x & 63;
  const int HNP = A.H * A.NP;
  const QhW W = qh_worker(A.qscratch + (size_t)(A.block_base + blockIdx.x) * A.qstride, HNP);
  const int lrow = slot / A.npr, jj = A.nbr_list ? A.nbr_list[slot] : slot % A.npr;
  const int i = A.row_begin + lrow * A.row_stride;
  const int j = jj < i ? jj : jj + 1;
  const double* xi = A.x + (size_t)i * A.X;
  const double* xj = A.x + (size_t)j * A.X;
  const double* Ti = A.T + (A.per_agent ? (size_t)i * A.H * 9 : 0);
  const double* Ni = A.NCF + (A.per_agent ? (size_t)i * A.H * 3 * A.X : 0);
  const double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};
  const int n = hull_points(A, LB, Ti, Ni, xi, xj, vrel, W.Pr, W.Pf);
  unsigned* owner = qw_owner(A.qscratch + (size_t)(A.block_base + blockIdx.x) * A.qstride, A.qstride);
  if (wave == 0) {
    qh_claim_scratch(W, owner, lane);
    QhS S;
#ifdef LQRO_QHULL_PROFILE
    for (int k = 0; k < 12; k++) S.tph[k] = 0;
#endif
    S.status = 0;
    S.nalloc = 1;
    S.nins = 0;
    S.facet_list = S.facet_tail = 0;
    if (LB.fail || n < 4) S.status = QHS_INPUT;
    else qh_build(W, S, LB, n, lane);
    hl_sync();
    qh_select(A, W, S, lane, xi, vrel, slot);
    if (lane == 0) hull_build_note(A, slot, 1, tjob, n, S.nins, S.nalloc - 1);
  }
}

// one inside-hull pair per wave (one wave per CU), persistent over the hull
// queue; a build beyond this kernel's caps is rebuilt in place by
// q3_big_inline when the kernel passes its LDS as LB (k_qhull), else it goes
// to the retry queue (k_qhull_big after the sweep)
__device__ __forceinline__ void q3_body(const HullArgs& A, Q3L& L, QhL* LB = nullptr) {   // (inlined into each kernel)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // 0: the build, 1: its speculation
  const int HNP = A.H * A.NP;
  const Q3W W = q3_worker(A.qscratch + (size_t)(A.block_base + blockIdx.x) * A.qstride, HNP);
  for (;;) {
    const int slot = hull_take_job(A, L, false);
    if (slot < 0) break;
    const unsigned long long tjob = __builtin_amdgcn_s_memrealtime();   // (lqro_get_hull_builds)
    // a speculative job (the last step's inside-hull pair, queued before
    // its evaluation): built now, committed only if the pair is inside
    const bool spec = A.spec_mark != nullptr && A.spec_mark[slot] >= 2;
    // a fresh handshake and wave 1's epochs for this job (ordered by
    // hull_points' barriers)
    if (threadIdx.x == 0) {
      L.ph = 0; L.sp_done = 0; L.sp_gdone = 0; L.hctl = 0u; L.hbusy = 0; L.sp_hz = 0; L.pf_done = 0;
      L.ectl = 0u; L.edone = 0;
      L.qflags = A.qflags;
#ifdef LQRO_QHULL_LONGPROF
      for (int k = 0; k < 12; k++) L.hprof[k] = 0ull;
      L.lp_pubr = L.lp_doner = 0ull;
#endif
      L.big_slot = -1;
    }
    for (int q = threadIdx.x; q < Q3_FL / 2; q += blockDim.x) reinterpret_cast<unsigned*>(L.mark)[q] = 0u;
    const int lrow = slot / A.npr, jj = A.nbr_list ? A.nbr_list[slot] : slot % A.npr;
    const int i = A.row_begin + lrow * A.row_stride;
    const int j = jj < i ? jj : jj + 1;
    const double* xi = A.x + (size_t)i * A.X;
    const double* xj = A.x + (size_t)j * A.X;
    const double* Ti = A.T + (A.per_agent ? (size_t)i * A.H * 9 : 0);
    const double* Ni = A.NCF + (A.per_agent ? (size_t)i * A.H * 3 * A.X : 0);
    const double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]};
    const int n = hull_points(A, L, Ti, Ni, xi, xj, vrel, W.Pr, W.Pf);
    bool lp_go = false;
    if (wave >= 2) {
      // wave 2: prefetch each horizon wave 1 publishes; waves 2 and 3: locate
      // posted chunks; until the build ends
      const Q3Col CH = q3_colh(W, wave, lane);
      int last = 0;
      long idle = 0;
      for (;;) {
        if (wave == 2) {
          const int hz = q3_ld_acq(&L.sp_hz);
          if (hz != last && hz > 0) {
            last = hz;
            q3_prefetch(W, L, lane, hz);
            idle = 0;
            continue;
          }
        }
        if (q3_help(W, L, lane, CH)) { idle = 0; continue; }
        if (q3_emit_help(W, L, lane)) { idle = 0; continue; }
        if (q3_ld_acq(&L.ph) < 0) break;
        if (++idle > (1l << 24)) break;
        __builtin_amdgcn_s_sleep(Q3_W2_SLEEP);
      }
    } else if (wave == 1) {
      // speculate each published phase until the build ends (ph = -1)
      // (wave 1's epochs: reset when k_qhull_big's code used the scratch)
      unsigned* owner = qw_owner(A.qscratch + (size_t)(A.block_base + blockIdx.x) * A.qstride, A.qstride);
      if (*owner != QW_OWNER_Q3) {
        for (int q = lane; q < W.FC; q += 64) W.mark2[q] = 0u;
        if (lane == 0) { W.ctr[0] = 0u; *owner = QW_OWNER_Q3; }
      }
      unsigned ep2 = W.ctr[0];
      unsigned short ep = 0;
      const Q3Col CH = q3_colh(W, 1, lane);
      int last = 0;
      Q3QC Q;
      Q.qcb = 0; Q.qcn = 0; Q.qf = 0; Q.qp = -1; Q.qk = 0u; Q.qx = Q.qy = Q.qz = 0.0;
      Q.pc_from = -1; Q.pc_pos = -1; Q.pc_end = 0; Q.pc_f = 0; Q.pc_p = -1; Q.pc_k = 0u;
      Q.pc_x = Q.pc_y = Q.pc_z = 0.0;
      Q.one = 0; Q.rt = -1;
      for (int k = 0; k < 6; k++) Q.r[k] = 0.0;
      long idle = 0;
      Q3P P;
      for (int k = 0; k < 16; k++) P.t[k] = 0;
      for (;;) {
        const int p = q3_ld_acq(&L.ph);
        if (p != last) {
          if (p < 0) break;
          last = p;
          ++ep;
          ++ep2;
#ifdef LQRO_QHULL_PROFILE
          const unsigned long long t0_ = __builtin_amdgcn_s_memtime();
          P.tq = t0_;
          P.t[14] += t0_ - L.pub_t;   // publication -> speculation start
          if (P.tq2) P.t[15] += t0_ - P.tq2;   // (this wave's clock) its last speculation's end -> this start
          if (lane == 0) L.start_r = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef LQRO_QHULL_LONGPROF
          const unsigned long long ts_ = __builtin_amdgcn_s_memrealtime();
#endif
          q3_spec(W, L, lane, ep, ep2, Q, P, p);
          hl_sync();
#ifdef LQRO_QHULL_LONGPROF
          if (lane == 0) {
            const unsigned long long te_ = __builtin_amdgcn_s_memrealtime();
            L.hprof[3] += 1; L.hprof[4] += ts_ - q3_lds(L.lp_pubr); L.hprof[5] += te_ - ts_;
            L.lp_doner = te_;
          }
#endif
#ifdef LQRO_QHULL_PROFILE
          if (lane == 0) L.done_t = __builtin_amdgcn_s_memtime();
#endif
          if (lane == 0) q3_st_rel_lds(&L.sp_done, p);
          if (lane == 0) q3_st_rel(&L.sp_gdone, p);
          if (L.qflags & 4) q3_prescan(W, L, lane, ep, ep2, Q);
#ifdef LQRO_QHULL_PROFILE
          if (lane == 0) { L.done_t2 = __builtin_amdgcn_s_memtime(); L.done_r = __builtin_amdgcn_s_memrealtime(); }
          P.tq2 = __builtin_amdgcn_s_memtime();
          P.t[0] += __builtin_amdgcn_s_memtime() - t0_;
          P.t[7] += 1;
#endif
          idle = 0;
          continue;
        }
        {
#ifdef LQRO_QHULL_PROFILE
          const unsigned long long t0_ = __builtin_amdgcn_s_memtime();
#endif
          if (q3_help(W, L, lane, CH)) {   // a posted chunk
#ifdef LQRO_QHULL_PROFILE
            P.t[6] += __builtin_amdgcn_s_memtime() - t0_;
            P.t[8] += 1;
#endif
            idle = 0;
            continue;
          }
        }
        if (q3_emit_help(W, L, lane)) { idle = 0; continue; }   // a posted emit's bucket
        if (++idle > (1l << 24)) break;
        __builtin_amdgcn_s_sleep(Q3_W1_SLEEP);
      }
#ifdef LQRO_QHULL_PROFILE
      if (A.prof && lane == 0)
        for (int k = 0; k < 16; k++) atomicAdd(&A.prof[Q3_PROF_W1 + k], P.t[k]);
#endif
      if (lane == 0) W.ctr[0] = ep2;
    } else {
    Q3S S;
#ifdef LQRO_QHULL_PROFILE
    for (int k = 0; k < 32; k++) S.tph[k] = 0;
    S.tw = S.nw = 0;
    S.tdl = 0;
    S.tw1 = S.nw1 = 0;
    S.tse = S.tsn = 0;
    S.tfr = S.nsp = 0;
    S.tfr2 = 0;
    S.trel = 0;
    S.r_start = S.r_done = S.r_seen = S.r_gseen = 0;
    S.tseen = S.tpre = S.npre = S.tstart = 0;
    S.prev1 = 0;
    for (int k = 0; k < 24; k++) S.tps[k] = 0;
    S.nps = 0;
    const unsigned long long tjob_ = __builtin_amdgcn_s_memtime();
#endif
    S.status = 0;
    S.nalloc = 1;
    S.nins = 0;
    S.lp_n = S.lp_pts = S.lp_t = S.lp_all = S.lp_tloc = S.lp_wait = S.lp_adopt = S.lp_tail = S.lp_tw = 0;
    S.lp_own = S.lp_got = S.lp_hwait = S.lp_stop = S.lp_ev = S.lp_posts = 0;
    if (L.fail || n < 4) S.status = QHS_INPUT;
    else q3_build(W, S, L, n, lane);
    hl_sync();
    if (lane == 0) q3_st_rel(&L.ph, -1);   // the build is over: wave 1 stops
    bool keep = true;
    if (spec) {
      // the pair's verdict from the hot launch (3 inside, 4 not; it is
      // normally in long before the build ends); bounded wait
      int m = 0;
      if (lane == 0) {
        m = __hip_atomic_load(A.spec_mark + slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        for (long w = 0; m == 2 && w < (1l << 26); ++w) {
          __builtin_amdgcn_s_sleep(8);
          m = __hip_atomic_load(A.spec_mark + slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (m == 2) {   // never evaluated (not expected): reported, nothing committed
          atomicAdd(&A.stats[LQRO_ST_TIMEOUT], 1ull);
          hull_fail_note(A.stats, slot);
        }
      }
      keep = __builtin_amdgcn_readfirstlane(m) == 3;
    }
    if (!keep) {
      // not inside this step: k_pair wrote its plane; the build is dropped
    } else if (S.status & QHS_CAPACITY) {
      if (lane == 0) {
        atomicAdd(&A.stats[LQRO_ST_RETRY], 1ull);
        if (S.status & QHS_TIMEOUT) atomicAdd(&A.stats[LQRO_ST_TIMEOUT], 1ull);
        if (LB) {
          L.big_slot = slot;   // rebuilt below, on this CU
        } else {
          const int r = atomicAdd(A.rcount, 1);
          if (r < A.cap) A.rqueue[r] = slot;
        }
        hull_build_note(A, slot, 2, tjob, n, S.nins, S.nalloc - 1);
#ifdef LQRO_QHULL_PROFILE
        // the builds handed to k_qhull_big: count, the caps they hit, slots
        if (A.prof) {
          const unsigned long long k = atomicAdd(&A.prof[Q3_PROF_RETRY], 1ull);
          atomicOr(&A.prof[Q3_PROF_RETRY + 1], (unsigned long long)S.status);
          if (k < 14) A.prof[Q3_PROF_RETRY + 2 + k] = (unsigned long long)slot | ((unsigned long long)S.status << 32);
        }
#endif
      }
      hl_sync();
    } else {
#ifdef LQRO_QHULL_PROFILE
    unsigned long long tq_ = __builtin_amdgcn_s_memtime();
#endif
    lp_go = q3_select(A, W, L, S, lane, xi, vrel, slot);
    if (lane == 0) {
      const int k = hull_build_note(A, slot, 0, tjob, n, S.nins, S.nalloc - 1);
#ifdef LQRO_QHULL_LONGPROF
      if (A.prof && k >= 0 && k < 1024) {
        unsigned long long* r = A.prof + Q3_PROF_LONG + 24 * k;
        r[0] = S.lp_n; r[1] = S.lp_pts; r[2] = S.lp_t; r[3] = S.lp_all;
        r[4] = S.lp_tloc; r[5] = S.lp_wait; r[6] = S.lp_adopt - S.lp_wait; r[7] = S.lp_tail;
        r[8] = S.lp_own; r[9] = S.lp_got; r[10] = S.lp_hwait; r[11] = S.lp_stop; r[12] = S.lp_ev; r[13] = S.lp_posts;
        r[14] = L.hprof[0]; r[15] = L.hprof[1] | (L.hprof[2] << 32);
        for (int q = 3; q < 11; q++) r[13 + q] = L.hprof[q];   // r[16..23]
      }
#else
      (void)k;
#endif
    }
#ifdef LQRO_QHULL_PROFILE
    S.tph[10] = __builtin_amdgcn_s_memtime() - tq_;
    S.tph[27] = __builtin_amdgcn_s_memtime() - tjob_;   // the whole job (26: its max over jobs)
    S.tph[28] = (unsigned long long)n;
    if (A.prof && lane == 0) {
      for (int k = 0; k < 32; k++)
        if (k != 26 && k != 11) atomicAdd(&A.prof[k], S.tph[k]);
      atomicAdd(&A.prof[Q3_PROF_W1 + 9], S.tw);
      atomicAdd(&A.prof[Q3_PROF_W1 + 10], S.nw);
      for (int k = 0; k < 24; k++) atomicAdd(&A.prof[Q3_PROF_W1 + 16 + k], S.tps[k]);
      atomicAdd(&A.prof[Q3_PROF_W1 + 40], S.nps);
      atomicAdd(&A.prof[Q3_PROF_W1 + 41], S.tdl);
      atomicAdd(&A.prof[Q3_PROF_W1 + 42], S.tw1);
      atomicAdd(&A.prof[Q3_PROF_W1 + 43], S.nw1);
      atomicAdd(&A.prof[Q3_PROF_W1 + 44], S.tse);
      atomicAdd(&A.prof[Q3_PROF_W1 + 45], S.tsn);
      atomicAdd(&A.prof[Q3_PROF_W1 + 46], S.tfr);
      atomicAdd(&A.prof[Q3_PROF_W1 + 47], S.nsp);
      atomicAdd(&A.prof[Q3_PROF_W1 + 48], S.tfr2);
      atomicAdd(&A.prof[Q3_PROF_W1 + 49], S.trel);
      atomicAdd(&A.prof[Q3_PROF_W1 + 50], S.r_start);
      atomicAdd(&A.prof[Q3_PROF_W1 + 51], S.r_done);
      atomicAdd(&A.prof[Q3_PROF_W1 + 52], S.r_seen);
      atomicAdd(&A.prof[Q3_PROF_W1 + 53], S.r_gseen);
      atomicAdd(&A.prof[Q3_PROF_W1 + 54], S.tpre);
      atomicAdd(&A.prof[Q3_PROF_W1 + 55], S.npre);
      atomicAdd(&A.prof[Q3_PROF_W1 + 56], S.tstart);
      atomicMax(&A.prof[26], S.tph[27]);
      // per job (words 32 + 2j): cycles; insertions | points << 20 | facet slots << 40
      const unsigned long long j = atomicAdd(&A.prof[11], 1ull);
      if (j < 4096) {
        A.prof[32 + 2 * j] = S.tph[27];
        A.prof[33 + 2 * j] = S.tph[21] | ((unsigned long long)n << 20) | ((unsigned long long)S.nalloc << 40);
      }
    }
#endif
    if (A.ext_nf && lane == 0) *A.ext_nf = S.status;   // test hook: the build's status bits
    if (A.ext_facets) {                                  // test hook: the facet list in key order
      for (int f = 1 + lane; f < S.nalloc; f += 64) {
        if (!(q3_fa(W, L, f) & QF_LIVE)) continue;
        const unsigned k = q3_key(W, L, f);
        int rank = 0, nl = 0;
        for (int g = 1; g < S.nalloc; g++)
          if (q3_fa(W, L, g) & QF_LIVE) { nl++; rank += q3_key(W, L, g) < k; }
        if (rank < A.ext_max)
          for (int t = 0; t < 3; t++) A.ext_facets[3 * rank + t] = W.vv[f].id[t];
        if (rank == 0 && nl < A.ext_max) A.ext_facets[3 * nl] = -1;
      }
      hl_sync();
    }
    }   // the build was not handed over
    }   // wave 0
#ifndef LQRO_QHULL_NO_INLINE_BIG
    if (LB) {
      __syncthreads();   // waves 1 and 2 are done with the build's LDS; big_slot is set
      const int bs = L.big_slot;
      __syncthreads();   // (read by every wave before LB, which aliases L, is written)
      if (bs >= 0) {
        q3_big_inline(A, *LB, bs, tjob, wave);
        __syncthreads();
      }
    }
#endif
    if (A.rowpend) {
      // this job closed its row: wave 0 runs the row's LP in the facet
      // planes' LDS once waves 1 and 2 (which read them while speculating)
      // are done with the build (the next hull_take_job waits for it)
      __syncthreads();
      if (wave == 0 && lp_go) q3_row_lp(A, L, slot, lane);
    }
  }
}

}  // namespace lqro
