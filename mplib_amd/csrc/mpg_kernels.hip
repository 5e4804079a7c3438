// mpg_kernels.hip -- MI355X (gfx950) kernels and the C ABI of include/mpgpu.h.
//
// Hot path: one batched launch evaluates, per joint configuration,
//   setQposAll(q) -> FK -> getLinkPose quaternion round trip -> collision
//   object transforms (src/articulated_model.cpp:101-127,
//   src/fcl_model.cpp:139-148), then every pair of the world's pair table
//   with fcl::collide semantics for CollisionRequest() (GST_LIBCCD ->
//   ccdMPRIntersect, FCL 0.7.0 / libccd 2.1), then the ACM filter
//   (src/planning_world.cpp:265-274).
//
// Two phases per chunk of configurations (DESIGN.md "Kernels"):
//   A  cull_kernel      lane per configuration: fp32 FK + conservative broad
//                       phase (mpg_broadphase.h) -> survivor bits [word][cfg]
//      (cull also writes the per-tile survivor counts)
//      pair_scan / chunk_scan / scatter: bucket the survivors
//                       into per-pair candidate lists (deterministic, no
//                       global atomics)
//   B  narrow_kernel    wave per 64 candidates of ONE pair: exact fp64 FK of
//                       the two objects' chains + libccd MPR; hull reads are
//                       wave-uniform scalar loads.
// A pair culled in A is separated by more than kBpMargin, so MPR would say
// "no intersection": the output bits equal evaluating every pair.
//
// Everything that decides an output bit (phase B) is fp64 with
// -ffp-contract=off, bit-identical to the reference's operation order.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mpgpu.h"
#include "mpg_math.h"
#include "mpg_fk.h"
#include "mpg_hostpipe.h"

using namespace mpg;

namespace {


thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                 \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess)                                                             \
      return set_error(MPG_E_HIP, std::string(#expr " failed: ") + hipGetErrorString(_e)); \
  } while (0)

// ---------------------------------------------------------------------------
// device snapshot
// ---------------------------------------------------------------------------



// ---------------------------------------------------------------------------
// FCL GJK objects + libccd MPR
// ---------------------------------------------------------------------------
struct GObj {
  CQ4 rot, rot_inv;  // libccd ccd_quat_t (ccd_real)
  CV3 pos;
  int geom;
  int type;
};

// vertex i of hull `geom` (AoSoA-4 groups: x0..3, y0..3, z0..3)
__device__ __forceinline__ V3 hull_vertex(const DevWorld& w, cptr<double> HV, int geom, int i) {
  const cptr<double> G = HV + 12 * (size_t)(w.geom_gstart[geom] + (i >> 2)) + (i & 3);
  return v3(G[0], G[4], G[8]);
}

// Dot product in Eigen's Vector3d::dot order, as Convex::findExtremeVertex
// evaluates v_C.dot(vertex): (x0*p0 + x1*p1) + x2*p2.
__device__ __forceinline__ double edot(const V3& d, const V3& p) { return (d.x * p.x + d.y * p.y) + d.z * p.z; }

// Convex::findExtremeVertex, linear branch (hulls of <= 32 vertices, or whose
// faces failed FCL's ValidateTopology): argmax dir . vertex (fp64), first
// maximum wins.  The AoSoA groups are padded with copies of the hull's first
// vertex, which can never win the strict '>', so the result equals the
// unpadded scan.  Only for directions without a cell.
__device__ __forceinline__ V3 convex_full_scan(const DevWorld& w, cptr<double> HV, int geom, const V3& dir) {
  const int g0 = w.geom_gstart[geom], ng = w.geom_ng[geom];
  const cptr<double> P = HV + 12 * (size_t)g0;
  double best = -DBL_MAX;
  int bi = 0;
  for (int g = 0; g < ng; ++g) {
    const cptr<double> G = P + 12 * g;
    double dd[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) dd[k] = (dir.x * G[k] + dir.y * G[4 + k]) + dir.z * G[8 + k];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (dd[k] > best) {
        best = dd[k];
        bi = 4 * g + k;
      }
  }
  const cptr<double> B = P + 12 * (bi >> 2) + (bi & 3);
  return v3(B[0], B[4], B[8]);
}

// Convex::findExtremeVertex, neighbour-walk branch [ext FCL 0.7.0
// geometry/shape/convex-inl.h] (hulls of > 32 vertices whose faces passed
// ValidateTopology, oracle/collide_oracle.c support_convex): start at vertex
// 0, scan the current vertex's neighbour list (FindVertexNeighbors: sorted,
// from the faces), step to every unvisited neighbour whose value is >= the
// best so far, until a pass moves nowhere.
//
// Most supports never walk: the direction's cell record settles them
// (walk_cell_fast).  The few that must walk -- a lane or two per wave every
// few MPR steps -- are resolved by the whole wave together, one pending lane
// at a time (wave_walk): per step of the climb the active lanes load the
// current vertex's neighbours and their dot products in parallel and the
// pass's sequential '>=' scan replays from LDS, so a climb costs one memory
// round trip per step instead of one per neighbour, and the per-lane rare path
// no longer holds the other 63 lanes for the length of a serial walk.
constexpr int kWalkWords = kMaxWalkVerts / 64;
struct WalkScratch {  // one per wave (blocks of <= 512 threads)
  uint64_t vis[kWalkWords];
  double dd[64];
  int vi[64];
};

__device__ __forceinline__ WalkScratch& walk_scratch() {
  __shared__ WalkScratch s_walk[8];  // one per wave: 256-thread blocks, the 512-thread latency server
  return s_walk[(threadIdx.x >> 6) & 7];
}

// LDS written by some lanes of this wave, read by others: keep the compiler
// from moving the accesses across (the LDS unit serves one wave in order)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ double lane_bcast(double v, int L) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, L);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), L);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// The climb for one (wave-uniform) direction d, by the wave's active lanes
// (rank among nact), from vertex 0 or resumed from a prefix record (pre:
// mpg_hullcells.h WalkPrefix, the state where the host's replay stopped).
// Returns the final vertex index (uniform).
// A hull above kMaxWalkVerts vertices keeps its visited set in one slot of the
// world's global pool (big_vis, zero while free): the wave's first active lane
// claims a free slot (big_busy 0 -> 1), the wave clears the slot's words after
// the climb and releases it.  Holders never wait, so a wave that finds every
// slot taken only spins until one of them finishes.
__device__ __forceinline__ int big_vis_acquire(const DevWorld& w, int rank) {
  int slot = 0;
  if (rank == 0) {
    const int n = w.big_slots;
    int k = (int)((blockIdx.x * 8u + (threadIdx.x >> 6)) % (unsigned)n);
    while (atomicCAS(&w.big_busy[k], 0, 1) != 0) k = k + 1 == n ? 0 : k + 1;
    slot = k;
  }
  // rank 0 is the first active lane
  return __builtin_amdgcn_readfirstlane(slot);
}

__device__ __forceinline__ int wave_walk(const DevWorld& w, cptr<double> HV, int geom, const V3& d, int rank,
                                         int nact, cptr<int> pre) {
  WalkScratch& S = walk_scratch();
  const cptr<int> hd = w.hull_nbr + 2 * w.geom_nbr[geom];
  const int nwords = (w.geom_nvert[geom] + 63) >> 6;
  const bool big = nwords > kWalkWords;  // no cell tables either: pre == nullptr
  const int slot = big ? big_vis_acquire(w, rank) : -1;
  // the visited set: the wave's LDS bitset or the pool slot, one flat pointer
  unsigned long long* vis = big ? w.big_vis + (size_t)slot * w.big_words : (unsigned long long*)S.vis;
  if (big) {
    if (rank == 0) atomicOr(&vis[0], 1ull);  // vertex 0: the start (the slot is zero)
    __threadfence();
  } else {
    for (int j = rank; j < nwords; j += nact)
      S.vis[j] = pre ? (uint64_t)(uint32_t)pre[4 + 2 * j] | ((uint64_t)(uint32_t)pre[5 + 2 * j] << 32) : (j == 0 ? 1ull : 0ull);
  }
  wave_lds_sync();
  int bi = pre ? pre[0] : 0, pv = pre ? pre[1] : 0, k0 = pre ? pre[2] : 0;
  bool keep = pre ? pre[3] != 0 : false, first = true;
  double best = edot(d, hull_vertex(w, HV, geom, bi));
  do {
    const int v = first ? pv : bi;  // the pass scans v's list (v fixed for the pass)
    const int skip = first ? k0 : 0;
    bool moved = first && keep;
    first = false;
    const int start = hd[2 * v] + skip, cnt = hd[2 * v + 1] - skip;
    for (int c0 = 0; c0 < cnt; c0 += nact) {
      const int m = min(cnt - c0, nact);
      if (rank < m) {
        const cptr<double> e = w.nbr_ent + 4 * (size_t)(start + c0 + rank);
        const int vi = (int)e[3];
        const uint64_t bit = 1ull << (vi & 63);
        // test-and-set (a neighbour list has no repeats)
        const bool seen = (atomicOr(&vis[vi >> 6], (unsigned long long)bit) & bit) != 0ull;
        S.vi[rank] = seen ? -1 : vi;
        S.dd[rank] = seen ? 0.0 : (d.x * e[0] + d.y * e[1]) + d.z * e[2];
      }
      wave_lds_sync();
      for (int k = 0; k < m; ++k) {  // the pass's scan, in list order
        const int vi = S.vi[k];
        const double dd = S.dd[k];
        if (vi >= 0 && dd >= best) {
          moved = true;
          bi = vi;
          best = dd;
        }
      }
      wave_lds_sync();
    }
    bi = __builtin_amdgcn_readfirstlane(bi);
    keep = moved;
  } while (keep);
  if (big) {  // leave the slot zero, then free it
    for (int j = rank; j < nwords; j += nact) atomicExch(&vis[j], 0ull);
    __threadfence();
    wave_lds_sync();
    if (rank == 0) atomicExch(&w.big_busy[slot], 0);
  }
  return bi;
}

// true if some neighbour of vertex vi has a dot product strictly above dd: then
// the walk cannot end at vi (every vertex it evaluates is compared with the
// running maximum, which only grows)
__device__ __forceinline__ bool neighbour_beats(const DevWorld& w, cptr<double> HV, int geom, int vi, double dd,
                                                const V3& d) {
  const cptr<int> hd = w.hull_nbr + 2 * (w.geom_nbr[geom] + vi);
  const cptr<double> e = w.nbr_ent + 4 * (size_t)hd[0];
  const int cnt = hd[1];
  for (int k = 0; k < cnt; ++k)
    if ((d.x * e[4 * k] + d.y * e[4 * k + 1]) + d.z * e[4 * k + 2] > dd) return true;
  return false;
}

// Walk-hull support through its cell record (mpg_hullcells.h
// build_walk_cells).  In a trap-free subcell the walk ends at the unique
// global maximum, the maximum of the record's linear list: returned, pend =
// false.  In a trapped subcell whose fine cell has a certified endpoint (one
// climb path for the whole fine cone) that vertex is returned.  Otherwise (a
// tie at the maximum, or an uncertified fine cell) pend = true with the
// linear list's first maximum in hand, for walk_resolve_wave.
__device__ __forceinline__ V3 walk_cell_fast(const DevWorld& w, cptr<double> HV, int geom, cptr<double> R, int sub,
                                             int fine, int fine2, const V3& d, bool& pend, int& pre,
                                             unsigned long long t_cell = 0) {
#ifdef MPG_STATS  // phase stamps (s_memtime after the value each phase produces)
  unsigned long long t_rec = 0, t_ovf = 0;
#endif
  const long long no = (long long)R[9];
  const int n = (int)(no & ((1 << kCellCountBits) - 1));
  const cptr<double> ovf = w.wcell_ovf + 4 * (size_t)(no >> kCellCountBits);
  // first maximum (strict '>', as the reference's scan) ...
  double best = -DBL_MAX;
  int g = 0;
  double di[kCellInline];
#pragma unroll
  for (int k = 0; k < kCellInline; ++k) {
    di[k] = (d.x * R[3 * k] + d.y * R[3 * k + 1]) + d.z * R[3 * k + 2];
    if (k < n && di[k] > best) {
      best = di[k];
      g = k;
    }
  }
#ifdef MPG_STATS
  asm volatile("" ::"v"(best));
  t_rec = __builtin_amdgcn_s_memtime();
#endif
  int nmax = 0;  // ... and how many entries reach it (a tie when > 1)
  // the overflow entries kOvfBatch at a time: their loads issued together
  // (one memory round per batch, not per entry), then compared in list order
  for (int k0 = kCellInline; k0 < n; k0 += kOvfBatch) {
    double ex[kOvfBatch], ey[kOvfBatch], ez[kOvfBatch];
#pragma unroll
    for (int j = 0; j < kOvfBatch; ++j) {
      const cptr<double> e = ovf + 4 * (min(k0 + j, n - 1) - kCellInline);
      ex[j] = e[0];
      ey[j] = e[1];
      ez[j] = e[2];
    }
#pragma unroll
    for (int j = 0; j < kOvfBatch; ++j) {
      if (k0 + j >= n) break;
      const double dd = (d.x * ex[j] + d.y * ey[j]) + d.z * ez[j];
      if (dd > best) {  // a new maximum: the inline entries are all below it
        best = dd;
        g = k0 + j;
        nmax = 1;
      } else if (dd == best) {
        ++nmax;
      }
    }
  }
#ifdef MPG_STATS
  asm volatile("" ::"v"(best));
  t_ovf = __builtin_amdgcn_s_memtime();
#endif
  // the inline entries, compared with the final maximum (short lists repeat
  // their first entry: count only k < n)
#pragma unroll
  for (int k = 0; k < kCellInline; ++k) nmax += (k < n && di[k] == best) ? 1 : 0;
  bool tie = nmax > 1;
  const uint64_t free_mask = (uint64_t)__double_as_longlong(R[11]);
  const bool sub_free = (free_mask >> sub) & 1ull;
  pend = !(sub_free && !tie);
  int endp = -1;
  if (__builtin_expect(!sub_free, 0)) {  // trapped subcell: its fine cell's certified endpoint, if any
    const cptr<double> A = w.wcell_aux + kWalkAux * (size_t)(R[10] - 1.0);
    const int t = (int)A[0] + __popcll(~free_mask & ((1ull << sub) - 1ull));
    endp = w.wcell_end[(size_t)t * (kSub2K * kSub2K) + fine];
    if (endp <= -2) endp = w.wcell_end2[(size_t)(-2 - endp) * (kSub3K * kSub3K) + fine2];
    pend = endp < 0;
    pre = endp <= -2 ? -2 - endp : -1;
  }
#ifdef MPG_STATS
  if (w.stats && t_cell) {  // support phases, first active lane: cell lookup -> record + inline dots ->
    asm volatile("" ::"v"(pend));  // overflow entries -> tie / trap checks
    const unsigned long long t_end = __builtin_amdgcn_s_memtime();
    if ((uint32_t)__lane_id() == (uint32_t)__builtin_ctzll(__ballot(true))) {
      atomicAdd(&w.stats[49], t_rec - t_cell);
      atomicAdd(&w.stats[50], t_ovf - t_rec);
      atomicAdd(&w.stats[51], t_end - t_ovf);
      atomicAdd(&w.stats[52], 1ull);
    }
  }
  if (w.stats) {
    atomicAdd(&w.stats[10], 1ull);
    if (!pend) atomicAdd(&w.stats[11], 1ull);
    if (endp >= 0) atomicAdd(&w.stats[14], 1ull);
    if (pend) atomicAdd(&w.stats[sub_free ? 16 : 17], 1ull);  // pending: tie / uncertified fine cell
  }
#endif
  if (endp >= 0) return hull_vertex(w, HV, geom, endp);
  const cptr<double> e = g < kCellInline ? R + 3 * g : ovf + 4 * (g - kCellInline);
  return v3(e[0], e[1], e[2]);
}

// The pending lanes of a wave, one at a time by every active lane.  For lane
// L's trapped cell: the walk ends at the first maximum g of the walk list when
// every other listed vertex has a strictly greater neighbour (g itself when
// adjacent, else usually its witness, else a neighbour scan); the entries are
// checked in parallel.  g is the global first maximum, already in lane L's p.
// If that fails (a local maximum of the non-convex triangulation, a tie, or no
// cell) the climb is run (wave_walk).
__device__ __forceinline__ V3 walk_resolve_wave(const DevWorld& w, cptr<double> HV, int geom, const V3& d, int c,
                                                bool pend, int pre, V3 p) {
  unsigned long long pm = __ballot(pend);
  if (__builtin_expect(pm == 0ull, 1)) return p;
  const unsigned long long act = __ballot(true);
  const int nact = __popcll(act);
  const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
  const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  while (pm) {
    const int L = __builtin_ctzll(pm);
    pm &= pm - 1ull;
    // lane L's hull (the same on every lane when the wave's pair is uniform)
    const int geomL = __builtin_amdgcn_readlane(geom, L);
    const int cb = w.geom_cbase[geomL];
    const V3 dL = v3(lane_bcast(d.x, L), lane_bcast(d.y, L), lane_bcast(d.z, L));
    const int cL = __builtin_amdgcn_readlane(c, L);
    const int preL = __builtin_amdgcn_readlane(pre, L);
    if (preL >= 0) {  // undecided finer cell: resume the climb where the host's replay stopped
      const int bi = wave_walk(w, HV, geomL, dL, rank, nact, w.wcell_pre + kWalkPre * (size_t)preL);
      if (lane == L) p = hull_vertex(w, HV, geomL, bi);
#ifdef MPG_STATS
      if (w.stats && rank == 0) atomicAdd(&w.stats[18], 1ull);
#endif
      continue;
    }
    bool ok = false;
#ifdef MPG_STATS
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
    if (cL >= 0) {
      const double info = w.wcell_rec[kCellRec * (size_t)(cb + cL) + 10];
#ifdef MPG_WALK_NOVERIFY  // timing ablation: every pending lane climbs
      ok = false;
#else
      ok = info > 0.0;  // trap-free cell but tied: straight to the walk
#endif
      if (ok) {
        const cptr<double> A = w.wcell_aux + kWalkAux * (size_t)(info - 1.0);
        const int nw = (int)A[1];
        const cptr<double> E = A + kWalkAux;  // walk-list entries
        double bL = -DBL_MAX;
        int gL = 0;
        for (int k = 0; k < nw; ++k) {  // its first maximum (uniform)
          const cptr<double> e = E + kWalkAux * k;
          const double dd = (dL.x * e[5] + dL.y * e[6]) + dL.z * e[7];
          if (dd > bL) {
            bL = dd;
            gL = k;
          }
        }
        bool fail = false;
        for (int k = rank; k < nw; k += nact) {
          if (k == gL) continue;
          const cptr<double> a = E + kWalkAux * k;
          const double dd = (dL.x * a[5] + dL.y * a[6]) + dL.z * a[7];
          // the maximum g is a neighbour of this entry and strictly above it
          if (gL < 32 && ((((uint32_t)a[4]) >> gL) & 1u) && bL > dd) continue;
          const double dw = (dL.x * a[1] + dL.y * a[2]) + dL.z * a[3];
          if (dw > dd) continue;
          if (!neighbour_beats(w, HV, geomL, (int)a[0], dd, dL)) fail = true;
        }
        ok = __ballot(fail) == 0ull;
      }
    }
#ifdef MPG_STATS
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (w.stats && rank == 0) {
      atomicAdd(&w.stats[ok ? 12 : 13], 1ull);
      atomicAdd(&w.stats[9], t1 - t0);
    }
#endif
    if (!ok) {
      const int bi = wave_walk(w, HV, geomL, dL, rank, nact, nullptr);
      if (lane == L) p = hull_vertex(w, HV, geomL, bi);
#ifdef MPG_STATS
      if (w.stats && rank == 0) atomicAdd(&w.stats[15], __builtin_amdgcn_s_memtime() - t1);
#endif
    }
  }
  return p;
}

// Convex support in the hull frame (FCL 0.7.0 supportConvex: the ccd
// direction converted to Vector3<double>, findExtremeVertex in fp64).  Called
// by all active lanes of the wave together (geom is wave-uniform).
__device__ __forceinline__ V3 convex_support_fast(const DevWorld& w, cptr<double> HV, int geom, const V3& d, bool& pend,
                                                  int& cell, int& pre) {
  const int cb = w.geom_cbase[geom];
  pend = false;
  cell = -1;
  pre = -1;
  if (w.geom_nbr[geom] >= 0) {  // neighbour-walk hull (wave-uniform branch)
    int sub = 0, fine = 0, fine2 = 0;
    pend = true;
#ifdef MPG_STATS
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
    cell = cb >= 0 ? hull_cell_sub(d.x, d.y, d.z, w.walk_subk, &sub, &fine, &fine2) : -1;
    unsigned long long t_cell = 0;
#ifdef MPG_STATS
    asm volatile("" ::"v"(cell), "v"(sub), "v"(fine));
    t_cell = __builtin_amdgcn_s_memtime();
    if (w.stats && (uint32_t)__lane_id() == (uint32_t)__builtin_ctzll(__ballot(true))) atomicAdd(&w.stats[48], t_cell - t0);
#endif
    V3 p = v3(0.0, 0.0, 0.0);
    if (cell >= 0)
      p = walk_cell_fast(w, HV, geom, w.wcell_rec + kCellRec * (size_t)(cb + cell), sub, fine, fine2, d, pend, pre,
                         t_cell);
    return p;
  }
  const int c = cb >= 0 ? hull_cell(d.x, d.y, d.z) : -1;
  if (c < 0) return convex_full_scan(w, HV, geom, d);
  double p[3];
  cell_record_support(w.cell_rec + kCellRec * (size_t)(cb + c), w.cell_ovf, d.x, d.y, d.z, p);
  return v3(p[0], p[1], p[2]);
}

__device__ __forceinline__ V3 convex_support_local(const DevWorld& w, cptr<double> HV, int geom, const V3& d) {
  bool pend;
  int cell, pre;
  const V3 p = convex_support_fast(w, HV, geom, d, pend, cell, pre);
  if (w.geom_nbr[geom] < 0) return p;
  return walk_resolve_wave(w, HV, geom, d, cell, pend, pre, p);
}

// support mapping of one shape in its own frame (FCL shapeToGJK supports:
// supportConvex, supportBox, supportSphere, supportCap, supportCyl), in the
// libccd scalar: the shape parameters are the ccd_real values FCL's
// *ToGJK functions store (box: dim = side / 2; capsule / cylinder: height =
// lz / 2).
__device__ __forceinline__ CV3 support_local(const DevWorld& w, cptr<double> HV, int geom, int type, const CV3& dir) {
  const cptr<double> rec = w.geom_rec + G_STRIDE * geom;
  CV3 v;
  if (type == MPG_GEOM_CONVEX) {
    const V3 p = convex_support_local(w, HV, geom, to_v3(dir));
    v = cv3(p.x, p.y, p.z);
  } else if (type == MPG_GEOM_BOX) {
    const ccd_real hx = (ccd_real)(rec[G_PARAM + 0] / 2.0), hy = (ccd_real)(rec[G_PARAM + 1] / 2.0),
                   hz = (ccd_real)(rec[G_PARAM + 2] / 2.0);
    v = CV3{(dir.x >= 0 ? ccd_real(1) : ccd_real(-1)) * hx, (dir.y >= 0 ? ccd_real(1) : ccd_real(-1)) * hy,
            (dir.z >= 0 ? ccd_real(1) : ccd_real(-1)) * hz};
  } else if (type == MPG_GEOM_SPHERE) {
    const ccd_real r = (ccd_real)rec[G_PARAM];
    v = vscale(vscale(dir, r), ccd_real(1) / std::sqrt(vdot(dir, dir)));
  } else if (type == MPG_GEOM_CAPSULE) {
    const ccd_real r = (ccd_real)rec[G_PARAM], h = (ccd_real)(rec[G_PARAM + 1] / 2.0);
    const CV3 n = vscale(vnormalize(dir), r);
    CV3 p1 = CV3{0, 0, h}, p2 = CV3{0, 0, -h};
    p1 = vadd(p1, n);
    p2 = vadd(p2, n);
    v = dir.z > 0 ? p1 : p2;
  } else if (type == MPG_GEOM_CONE) {  // supportCone (coneToGJK: height = lz / 2)
    const ccd_real r = (ccd_real)rec[G_PARAM], h = (ccd_real)(rec[G_PARAM + 1] / 2.0);
    ccd_real zdist = dir.x * dir.x + dir.y * dir.y;
    ccd_real len = zdist + dir.z * dir.z;
    zdist = std::sqrt(zdist);
    len = std::sqrt(len);
    const ccd_real sin_a = r / std::sqrt(r * r + 4 * h * h);
    if (dir.z > len * sin_a) {
      v = CV3{0, 0, h};
    } else if (zdist > 0) {
      const ccd_real rad = r / zdist;
      v = CV3{rad * dir.x, rad * dir.y, -h};
    } else {
      v = CV3{0, 0, -h};
    }
  } else if (type == MPG_GEOM_TRIANGLE) {  // supportTriangle: first maximum of dir . (p - c), ccd_real
    const cptr<double> G = HV + 12 * (size_t)w.geom_gstart[geom];
    const CV3 c = cv3(rec[G_INTERIOR], rec[G_INTERIOR + 1], rec[G_INTERIOR + 2]);
    ccd_real maxdot = -FLT_MAX;
    v = cv3(G[0], G[4], G[8]);
    for (int i = 0; i < 3; ++i) {
      const CV3 p = cv3(G[i], G[4 + i], G[8 + i]);
      const ccd_real dot = vdot(dir, vsub(p, c));
      if (dot > maxdot) {
        v = p;
        maxdot = dot;
      }
    }
  } else if (type == MPG_GEOM_ELLIPSOID) {  // supportEllipsoid
    const ccd_real a = (ccd_real)rec[G_PARAM], b = (ccd_real)rec[G_PARAM + 1], c = (ccd_real)rec[G_PARAM + 2];
    const CV3 p = CV3{(a * a) * dir.x, (b * b) * dir.y, (c * c) * dir.z};
    v = vscale(p, ccd_real(1) / std::sqrt(vdot(p, dir)));
  } else {  // cylinder
    const ccd_real r = (ccd_real)rec[G_PARAM], h = (ccd_real)(rec[G_PARAM + 1] / 2.0);
    ccd_real zdist = dir.x * dir.x + dir.y * dir.y;
    zdist = std::sqrt(zdist);
    if (std::fabs(zdist) < kCcdEps) {
      v = CV3{0, 0, (dir.z > 0 ? ccd_real(1) : ccd_real(-1)) * h};
    } else {
      const ccd_real rad = r / zdist;
      v = CV3{rad * dir.x, rad * dir.y, (dir.z > 0 ? ccd_real(1) : ccd_real(-1)) * h};
    }
  }
  return v;
}

#include "mpg_gjk_indep.h"

// True extreme point of a shape along dir in its own frame, fp64 (every
// vertex for hulls, whatever FCL's walk would return): conservative range
// tests only, never an output bit.
__device__ __forceinline__ V3 support_local_exact(const DevWorld& w, cptr<double> HV, int geom, int type, const V3& dir) {
  const cptr<double> rec = w.geom_rec + G_STRIDE * geom;
  if (type == MPG_GEOM_CONVEX || type == MPG_GEOM_TRIANGLE) return convex_full_scan(w, HV, geom, dir);
  if (type == MPG_GEOM_BOX)
    return v3((dir.x >= 0 ? 1.0 : -1.0) * rec[G_PARAM] / 2.0, (dir.y >= 0 ? 1.0 : -1.0) * rec[G_PARAM + 1] / 2.0,
              (dir.z >= 0 ? 1.0 : -1.0) * rec[G_PARAM + 2] / 2.0);
  if (type == MPG_GEOM_SPHERE) return vscale(vscale(dir, rec[G_PARAM]), 1.0 / std::sqrt(vdot(dir, dir)));
  if (type == MPG_GEOM_ELLIPSOID) {
    const V3 p = v3(rec[G_PARAM] * rec[G_PARAM] * dir.x, rec[G_PARAM + 1] * rec[G_PARAM + 1] * dir.y,
                    rec[G_PARAM + 2] * rec[G_PARAM + 2] * dir.z);
    return vscale(p, 1.0 / std::sqrt(vdot(p, dir)));
  }
  const double r = rec[G_PARAM], h = rec[G_PARAM + 1] / 2.0;
  if (type == MPG_GEOM_CAPSULE) return vadd(v3(0.0, 0.0, dir.z > 0 ? h : -h), vscale(vnormalize(dir), r));
  if (type == MPG_GEOM_CONE) {  // the better of the apex and the base rim point along dir
    const double zd = std::sqrt(dir.x * dir.x + dir.y * dir.y);
    const double rad = zd > 0.0 ? r / zd : 0.0;
    const V3 rim = v3(rad * dir.x, rad * dir.y, -h);
    return dir.z * h > vdot(dir, rim) ? v3(0.0, 0.0, h) : rim;
  }
  const double zd = std::sqrt(dir.x * dir.x + dir.y * dir.y);  // cylinder
  const double rad = zd > 0.0 ? r / zd : 0.0;
  return v3(rad * dir.x, rad * dir.y, (dir.z > 0 ? 1.0 : -1.0) * h);
}

// libccd support of one GJK object: direction into the object frame
// (ccdQuatRotVec with rot_inv), local support, back to the world frame.  The
// geometry is the same on every lane of the wave (one pair per wave): say so,
// so parameter reads stay scalar loads.
__device__ __forceinline__ CV3 support(const DevWorld& w, cptr<double> HV, const GObj& o, const CV3& dir_world) {
  const CV3 dir = quat_rot(dir_world, o.rot_inv);
  const int geom = __builtin_amdgcn_readfirstlane(o.geom), type = __builtin_amdgcn_readfirstlane(o.type);
  return vadd(quat_rot(support_local(w, HV, geom, type, dir), o.rot), o.pos);
}

// centerConvex (interior point ccdVec3Set, rotated, translated) / centerShape
template <bool UNI = true>
__device__ __forceinline__ CV3 center(const DevWorld& w, const GObj& o) {
  const int t = UNI ? __builtin_amdgcn_readfirstlane(o.type) : o.type;
  if (t == MPG_GEOM_CONVEX || t == MPG_GEOM_TRIANGLE) {  // centerConvex / centerTriangle
    const cptr<double> rec = w.geom_rec + G_STRIDE * (UNI ? __builtin_amdgcn_readfirstlane(o.geom) : o.geom);
    return vadd(quat_rot(cv3(rec[G_INTERIOR], rec[G_INTERIOR + 1], rec[G_INTERIOR + 2]), o.rot), o.pos);
  }
  return o.pos;
}

__device__ __forceinline__ bool is_zero(ccd_real v) { return std::fabs(v) < kCcdEps; }

__device__ __forceinline__ bool ccd_eq(ccd_real _a, ccd_real _b) {
  const ccd_real ab = std::fabs(_a - _b);
  if (std::fabs(ab) < kCcdEps) return true;
  const ccd_real a = std::fabs(_a), b = std::fabs(_b);
  if (b > a) return ab < kCcdEps * b;
  return ab < kCcdEps * a;
}

__device__ __forceinline__ bool vec_is_origin(const CV3& v) {
  return ccd_eq(v.x, ccd_real(0)) && ccd_eq(v.y, ccd_real(0)) && ccd_eq(v.z, ccd_real(0));
}

// libccd __ccdSupport: v = support1(dir) - support2(-dir)
// UNI: the geometries are the same on every lane (one pair per wave): their
// parameters come through scalar loads; otherwise every lane has its own pair
template <bool UNI = true>
__device__ __forceinline__ CV3 msupport(const DevWorld& w, cptr<double> HV, const GObj& a,
                                        const GObj& b, const CV3& dir) {
  const CV3 da = quat_rot(dir, a.rot_inv), db = quat_rot(vscale(dir, ccd_real(-1)), b.rot_inv);
  const int ga = UNI ? __builtin_amdgcn_readfirstlane(a.geom) : a.geom, ta = UNI ? __builtin_amdgcn_readfirstlane(a.type) : a.type;
  const int gb = UNI ? __builtin_amdgcn_readfirstlane(b.geom) : b.geom, tb = UNI ? __builtin_amdgcn_readfirstlane(b.type) : b.type;
  // walk hulls: both fast paths first, then one resolve site for the lanes
  // either left pending (one inlined copy of the rare path instead of two)
  bool pa = false, pb = false;
  int ca = -1, cb = -1, qa = -1, qb = -1;
  CV3 la, lb;
  if (ta == MPG_GEOM_CONVEX) {
    const V3 p = convex_support_fast(w, HV, ga, to_v3(da), pa, ca, qa);
    la = cv3(p.x, p.y, p.z);
  } else {
    la = support_local(w, HV, ga, ta, da);
  }
  if (tb == MPG_GEOM_CONVEX) {
    const V3 p = convex_support_fast(w, HV, gb, to_v3(db), pb, cb, qb);
    lb = cv3(p.x, p.y, p.z);
  } else {
    lb = support_local(w, HV, gb, tb, db);
  }
  if (__builtin_expect(__ballot(pa || pb) != 0ull, 0)) {  // rare: laid out off the hot path
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {
      const int g = s ? gb : ga;
      const CV3 l = s ? lb : la;
      const V3 p = walk_resolve_wave(w, HV, g, to_v3(s ? db : da), s ? cb : ca, s ? pb : pa, s ? qb : qa,
                                     v3(l.x, l.y, l.z));
      if (s) lb = cv3(p.x, p.y, p.z);
      else la = cv3(p.x, p.y, p.z);
    }
  }
  return vsub(vadd(quat_rot(la, a.rot), a.pos), vadd(quat_rot(lb, b.rot), b.pos));
}

// msupport on two half-waves: every lane of one half carries the same MPR
// state as its partner lane ^ 32 of the other; lanes of side 0 evaluate a's
// support, side 1 b's (at once, instead of one after the other on one lane),
// then the halves swap their world points.  The arithmetic of each support is
// msupport's, so the result is the same bits.  Geometry per lane (the halves
// hold different shapes).
__device__ __forceinline__ CV3 msupport_split(const DevWorld& w, cptr<double> HV, const GObj& a, const GObj& b,
                                              const CV3& dir, bool side) {
  const GObj o = side ? b : a;
  const CV3 dl = quat_rot(side ? vscale(dir, ccd_real(-1)) : dir, o.rot_inv);
  bool pend = false;
  int cell = -1, pre = -1;
  CV3 l;
  if (o.type == MPG_GEOM_CONVEX) {
    const V3 p = convex_support_fast(w, HV, o.geom, to_v3(dl), pend, cell, pre);
    l = cv3(p.x, p.y, p.z);
  } else {
    l = support_local(w, HV, o.geom, o.type, dl);
  }
  if (__builtin_expect(__ballot(pend) != 0ull, 0)) {
    const V3 p = walk_resolve_wave(w, HV, o.geom, to_v3(dl), cell, pend, pre, v3(l.x, l.y, l.z));
    l = cv3(p.x, p.y, p.z);
  }
  const CV3 mine = vadd(quat_rot(l, o.rot), o.pos);
  const CV3 other = CV3{__shfl_xor(mine.x, 32), __shfl_xor(mine.y, 32), __shfl_xor(mine.z, 32)};
  return side ? vsub(other, mine) : vsub(mine, other);
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// Link Isometry from a (p, wxyz) pose vector (FCLModel::updateCollisionObjects,
// src/fcl_model.cpp:151-167 / ArticulatedModel::setQpos re-matrix).
__device__ __forceinline__ SE3 link_from_pose7(const double* p7) {
  SE3 T;
  quat_to_mat(p7[3], p7[4], p7[5], p7[6], T.R);
  T.p[0] = p7[0];
  T.p[1] = p7[1];
  T.p[2] = p7[2];
  return T;
}

// Moving object -> FCL GJK object (shapeToGJK on link pose * offset).
// world transform of moving object `id` (link pose * collision origin) -- the
// Isometry FCLModel::updateCollisionObjects hands to setTransform
// USE_SC: joint (sin, cos) precomputed in `sc` (phase A), else computed inline
// sc_row: the configuration's [dof][2] (sin, cos), or nullptr (computed inline)
template <bool FROM_POSES>
__device__ __forceinline__ SE3 moving_tf_row(const DevWorld& w, const double* __restrict__ in,
                                             const double* sc_row, long long cfg, int id) {
  const int l = w.moving_link[id];
  const SE3 L = FROM_POSES ? link_from_pose7(in + (cfg * w.n_links + l) * 7)
                           : link_from_oMi(w, chain_oMi(w, in + cfg * w.dof, l, sc_row), l, nullptr);
  return se3_mul(L, load_se3(w.moving_offset + 12 * id));
}
template <bool FROM_POSES, bool USE_SC = true>
__device__ __forceinline__ SE3 moving_tf(const DevWorld& w, const double* __restrict__ in,
                                         const double* __restrict__ sc, long long cfg, int id) {
  return moving_tf_row<FROM_POSES>(w, in, USE_SC ? sc + cfg * w.dof * 2 : nullptr, cfg, id);
}

// Moving object -> FCL GJK object (shapeToGJK on link pose * offset).
template <bool FROM_POSES>
__device__ __forceinline__ GObj moving_obj(const DevWorld& w, const double* __restrict__ in,
                                           const double* __restrict__ sc, long long cfg, int id) {
  const SE3 T = moving_tf<FROM_POSES>(w, in, sc, cfg, id);
  GObj o;
  o.rot = gjk_rot_from_matrix(T.R);
  o.rot_inv = quat_invert2(o.rot);
  o.pos = cv3(T.p[0], T.p[1], T.p[2]);
  o.geom = w.moving_geom[id];
  o.type = w.geom_type[o.geom];
  return o;
}

// ---------------------------------------------------------------------------
// FCL 0.7.0 closed-form shape pairs (GJKSolver_libccd::shapeIntersect
// specialisations, both argument orders), boolean part; same operation order
// as the oracle (oracle/collide_oracle.c box_box_intersect & co.)
// ---------------------------------------------------------------------------
enum : int {
  CF_NONE = 0, CF_BOX_BOX = 1, CF_SPHERE_SPHERE = 2, CF_SPHERE_BOX = 3, CF_BOX_SPHERE = 4, CF_OCTREE = 5,
  CF_SPHERE_CAPSULE = 6, CF_CAPSULE_SPHERE = 7, CF_SPHERE_CYLINDER = 8, CF_CYLINDER_SPHERE = 9, CF_MESH = 10,
  CF_GJK = 11  // GST_INDEP worlds: FCL's own GJK (mpg_gjk_indep.h) in place of libccd MPR
};
// narrow-phase classes of the candidate lists: each its own kernel instance
enum : int { CLS_CLOSED = 0, CLS_OCTREE = 1, CLS_MESH = 2, CLS_GJK = 3 };
__host__ __device__ __forceinline__ int cf_class(int cf) {
  return cf == CF_OCTREE ? CLS_OCTREE : cf == CF_MESH ? CLS_MESH : cf == CF_GJK ? CLS_GJK : CLS_CLOSED;
}

// detail::boxBox2 (box_box-inl.h, from ODE dBoxBox): return_code != 0
__device__ __forceinline__ bool box_box_intersect(const double* side1, const SE3& T1, const double* side2,
                                                  const SE3& T2) {
  const double p[3] = {T2.p[0] - T1.p[0], T2.p[1] - T1.p[1], T2.p[2] - T1.p[2]};
  double pp[3], A[3], B[3], R[3][3], Q[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i) pp[i] = (T1.R[i] * p[0] + T1.R[3 + i] * p[1]) + T1.R[6 + i] * p[2];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    A[i] = side1[i] * 0.5;
    B[i] = side2[i] * 0.5;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      R[i][j] = (T1.R[i] * T2.R[j] + T1.R[3 + i] * T2.R[3 + j]) + T1.R[6 + i] * T2.R[6 + j];
      Q[i][j] = std::fabs(R[i][j]);
    }
  double s = -DBL_MAX, s2, tmp;
  int code = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {  // axes u1, u2, u3
    tmp = pp[i];
    s2 = std::fabs(tmp) - (((Q[i][0] * B[0] + Q[i][1] * B[1]) + Q[i][2] * B[2]) + A[i]);
    if (s2 > 0) return false;
    if (s2 > s) {
      s = s2;
      code = 1 + i;
    }
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {  // axes v1, v2, v3
    tmp = (T2.R[j] * p[0] + T2.R[3 + j] * p[1]) + T2.R[6 + j] * p[2];
    s2 = std::fabs(tmp) - (((Q[0][j] * A[0] + Q[1][j] * A[1]) + Q[2][j] * A[2]) + B[j]);
    if (s2 > 0) return false;
    if (s2 > s) {
      s = s2;
      code = 4 + j;
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) Q[i][j] += 1.0e-6;  // ODE's edge-axis tolerance
  const double eps = DBL_EPSILON, fudge = 1.05;
  auto edge = [&](double t, double rad, double n0, double n1, double n2, int c) -> bool {
    const double e2 = std::fabs(t) - rad;
    if (e2 > eps) return true;
    const double l = std::sqrt((n0 * n0 + n1 * n1) + n2 * n2);
    if (l > eps) {
      const double e3 = e2 / l;
      if (e3 * fudge > s) {
        s = e3;
        code = c;
      }
    }
    return false;
  };
  // u1 x (v1, v2, v3)
  if (edge(pp[2] * R[1][0] - pp[1] * R[2][0], ((A[1] * Q[2][0] + A[2] * Q[1][0]) + B[1] * Q[0][2]) + B[2] * Q[0][1], 0,
           -R[2][0], R[1][0], 7)) return false;
  if (edge(pp[2] * R[1][1] - pp[1] * R[2][1], ((A[1] * Q[2][1] + A[2] * Q[1][1]) + B[0] * Q[0][2]) + B[2] * Q[0][0], 0,
           -R[2][1], R[1][1], 8)) return false;
  if (edge(pp[2] * R[1][2] - pp[1] * R[2][2], ((A[1] * Q[2][2] + A[2] * Q[1][2]) + B[0] * Q[0][1]) + B[1] * Q[0][0], 0,
           -R[2][2], R[1][2], 9)) return false;
  // u2 x (v1, v2, v3)
  if (edge(pp[0] * R[2][0] - pp[2] * R[0][0], ((A[0] * Q[2][0] + A[2] * Q[0][0]) + B[1] * Q[1][2]) + B[2] * Q[1][1],
           R[2][0], 0, -R[0][0], 10)) return false;
  if (edge(pp[0] * R[2][1] - pp[2] * R[0][1], ((A[0] * Q[2][1] + A[2] * Q[0][1]) + B[0] * Q[1][2]) + B[2] * Q[1][0],
           R[2][1], 0, -R[0][1], 11)) return false;
  if (edge(pp[0] * R[2][2] - pp[2] * R[0][2], ((A[0] * Q[2][2] + A[2] * Q[0][2]) + B[0] * Q[1][1]) + B[1] * Q[1][0],
           R[2][2], 0, -R[0][2], 12)) return false;
  // u3 x (v1, v2, v3)
  if (edge(pp[1] * R[0][0] - pp[0] * R[1][0], ((A[0] * Q[1][0] + A[1] * Q[0][0]) + B[1] * Q[2][2]) + B[2] * Q[2][1],
           -R[1][0], R[0][0], 0, 13)) return false;
  if (edge(pp[1] * R[0][1] - pp[0] * R[1][1], ((A[0] * Q[1][1] + A[1] * Q[0][1]) + B[0] * Q[2][2]) + B[2] * Q[2][0],
           -R[1][1], R[0][1], 0, 14)) return false;
  if (edge(pp[1] * R[0][2] - pp[0] * R[1][2], ((A[0] * Q[1][2] + A[1] * Q[0][2]) + B[0] * Q[2][1]) + B[1] * Q[2][0],
           -R[1][2], R[0][2], 0, 15)) return false;
  return code != 0;
}

// detail::sphereSphereIntersect
__device__ __forceinline__ bool sphere_sphere_intersect(double r1, const SE3& T1, double r2, const SE3& T2) {
  const double d0 = T2.p[0] - T1.p[0], d1 = T2.p[1] - T1.p[1], d2 = T2.p[2] - T1.p[2];
  const double len = std::sqrt((d0 * d0 + d1 * d1) + d2 * d2);
  return !(len > r1 + r2);
}

// detail::sphereBoxIntersect: X_BS = X_FB.inverse() * X_FS, nearestPointInBox
__device__ __forceinline__ bool sphere_box_intersect(double r, const SE3& TS, const double* side, const SE3& TB) {
  double c[3];
  bool clamped = false;
  double dd = 0.0;
  double d[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double inv_t = -((TB.R[i] * TB.p[0] + TB.R[3 + i] * TB.p[1]) + TB.R[6 + i] * TB.p[2]);
    c[i] = ((TB.R[i] * TS.p[0] + TB.R[3 + i] * TS.p[1]) + TB.R[6 + i] * TS.p[2]) + inv_t;
    const double h = side[i] / 2;
    double nq = c[i];
    if (c[i] < -h) {
      clamped = true;
      nq = -h;
    }
    if (c[i] > h) {
      clamped = true;
      nq = h;
    }
    d[i] = c[i] - nq;
  }
  dd = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
  return !(clamped && dd > r * r);
}

// the sphere centre in the other shape's frame: X_FO.inverse() * X_FS
// translation, R^T p_S + (-(R^T p_O)) with Eigen's evaluation order
__device__ __forceinline__ void centre_in_frame(const SE3& TS, const SE3& TO, double* c) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double inv_t = -((TO.R[i] * TO.p[0] + TO.R[3 + i] * TO.p[1]) + TO.R[6 + i] * TO.p[2]);
    c[i] = ((TO.R[i] * TS.p[0] + TO.R[3 + i] * TS.p[1]) + TO.R[6 + i] * TS.p[2]) + inv_t;
  }
}

// detail::sphereCapsuleIntersect (sphere_capsule-inl.h): the closest point of
// the capsule's axis segment (0,0,+lz/2)-(0,0,-lz/2) to the sphere centre
// (lineSegmentPointClosestToPoint), then |diff| - r1 - r2 > 0 -> separated
__device__ __forceinline__ bool sphere_capsule_intersect(double r1, const SE3& TS, double r2, double lz,
                                                         const SE3& TC) {
  double c[3];
  centre_in_frame(TS, TC, c);
  const double s1z = 0.5 * lz, s2z = -s1z;
  const double vz = s2z - s1z;
  const double w2 = c[2] - s1z;
  const double c1 = (c[0] * 0.0 + c[1] * 0.0) + w2 * vz;
  const double c2 = (0.0 * 0.0 + 0.0 * 0.0) + vz * vz;
  double spz;
  if (c1 <= 0) spz = s1z;
  else if (c2 <= c1) spz = s2z;
  else spz = s1z + vz * (c1 / c2);
  const double d0 = c[0], d1 = c[1], d2 = c[2] - spz;
  const double dist = std::sqrt((d0 * d0 + d1 * d1) + d2 * d2) - r1 - r2;
  return !(dist > 0);
}

// detail::sphereCylinderIntersect (sphere_cylinder-inl.h): nearestPointInCylinder
// (clamp z to +-lz/2, the radial part to the radius), inside -> intersect,
// else squared distance against r^2
__device__ __forceinline__ bool sphere_cylinder_intersect(double r, const SE3& TS, double rc, double lz,
                                                          const SE3& TC) {
  double c[3], n[3];
  centre_in_frame(TS, TC, c);
  const double h = lz / 2;
  bool clamped = false;
  n[0] = c[0];
  n[1] = c[1];
  n[2] = c[2];
  if (c[2] > h) {
    n[2] = h;
    clamped = true;
  } else if (c[2] < -h) {
    n[2] = -h;
    clamped = true;
  }
  const double rd2 = c[0] * c[0] + c[1] * c[1];
  if (rd2 > rc * rc) {
    const double scale = rc / std::sqrt(rd2);
    n[0] = c[0] * scale;
    n[1] = c[1] * scale;
    clamped = true;
  }
  if (!clamped) return true;
  const double d0 = n[0] - c[0], d1 = n[1] - c[1], d2 = n[2] - c[2];
  return !(((d0 * d0 + d1 * d1) + d2 * d2) > r * r);
}

__device__ __forceinline__ bool closed_form(int kind, const DevWorld& w, int ga, const SE3& TA, int gb,
                                            const SE3& TB) {
  const cptr<double> pa = w.geom_rec + G_STRIDE * ga + G_PARAM, pb = w.geom_rec + G_STRIDE * gb + G_PARAM;
  const double sa[3] = {pa[0], pa[1], pa[2]}, sb[3] = {pb[0], pb[1], pb[2]};
  switch (kind) {
    case CF_BOX_BOX: return box_box_intersect(sa, TA, sb, TB);
    case CF_SPHERE_SPHERE: return sphere_sphere_intersect(sa[0], TA, sb[0], TB);
    case CF_SPHERE_BOX: return sphere_box_intersect(sa[0], TA, sb, TB);
    case CF_SPHERE_CAPSULE: return sphere_capsule_intersect(sa[0], TA, sb[0], sb[1], TB);
    case CF_CAPSULE_SPHERE: return sphere_capsule_intersect(sb[0], TB, sa[0], sa[1], TA);
    case CF_SPHERE_CYLINDER: return sphere_cylinder_intersect(sa[0], TA, sb[0], sb[1], TB);
    case CF_CYLINDER_SPHERE: return sphere_cylinder_intersect(sb[0], TB, sa[0], sa[1], TA);
    default: return sphere_box_intersect(sb[0], TB, sa, TA);  // CF_BOX_SPHERE
  }
}

// fcl::OBB::overlap -> obbDisjoint (fcl/math/bv/OBB-inl.h [ext FCL 0.7.0]):
// B = R1^T R2 (row-major), T = R1^T (c2 - c1), a / b the half extents; the
// |B| entries are widened by 1e-6 before the 15 separating-axis tests.
__device__ __forceinline__ bool obb_disjoint(const double* B, const double* T, const double* a, const double* b) {
  const double reps = 1e-6;
  double Bf[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Bf[i] = std::fabs(B[i]) + reps;
  if (std::fabs(T[0]) > a[0] + ((Bf[0] * b[0] + Bf[1] * b[1]) + Bf[2] * b[2])) return true;
  if (std::fabs((B[0] * T[0] + B[3] * T[1]) + B[6] * T[2]) > b[0] + ((Bf[0] * a[0] + Bf[3] * a[1]) + Bf[6] * a[2]))
    return true;
  if (std::fabs(T[1]) > a[1] + ((Bf[3] * b[0] + Bf[4] * b[1]) + Bf[5] * b[2])) return true;
  if (std::fabs(T[2]) > a[2] + ((Bf[6] * b[0] + Bf[7] * b[1]) + Bf[8] * b[2])) return true;
  if (std::fabs((B[1] * T[0] + B[4] * T[1]) + B[7] * T[2]) > b[1] + ((Bf[1] * a[0] + Bf[4] * a[1]) + Bf[7] * a[2]))
    return true;
  if (std::fabs((B[2] * T[0] + B[5] * T[1]) + B[8] * T[2]) > b[2] + ((Bf[2] * a[0] + Bf[5] * a[1]) + Bf[8] * a[2]))
    return true;
#define MPG_B(i, j) B[3 * (i) + (j)]
#define MPG_BF(i, j) Bf[3 * (i) + (j)]
#pragma unroll
  for (int j = 0; j < 3; ++j) {  // A0 x Bj
    const int j1 = j == 0 ? 1 : 0, j2 = j == 2 ? 1 : 2;
    const double sv = T[2] * MPG_B(1, j) - T[1] * MPG_B(2, j);
    if (std::fabs(sv) > a[1] * MPG_BF(2, j) + a[2] * MPG_BF(1, j) + b[j1] * MPG_BF(0, j2) + b[j2] * MPG_BF(0, j1))
      return true;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {  // A1 x Bj
    const int j1 = j == 0 ? 1 : 0, j2 = j == 2 ? 1 : 2;
    const double sv = T[0] * MPG_B(2, j) - T[2] * MPG_B(0, j);
    if (std::fabs(sv) > a[0] * MPG_BF(2, j) + a[2] * MPG_BF(0, j) + b[j1] * MPG_BF(1, j2) + b[j2] * MPG_BF(1, j1))
      return true;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {  // A2 x Bj
    const int j1 = j == 0 ? 1 : 0, j2 = j == 2 ? 1 : 2;
    const double sv = T[1] * MPG_B(0, j) - T[0] * MPG_B(1, j);
    if (std::fabs(sv) > a[0] * MPG_BF(1, j) + a[1] * MPG_BF(0, j) + b[j1] * MPG_BF(2, j2) + b[j2] * MPG_BF(2, j1))
      return true;
  }
#undef MPG_B
#undef MPG_BF
  return false;
}

__device__ __forceinline__ GObj static_obj(const DevWorld& w, int sid) {
  const cptr<double> r = w.static_rec + S_STRIDE * sid;
  GObj o;
  // static_record stores the ccd_real values (exactly representable in fp64)
  o.rot = CQ4{(ccd_real)r[S_ROT], (ccd_real)r[S_ROT + 1], (ccd_real)r[S_ROT + 2], (ccd_real)r[S_ROT + 3]};
  o.rot_inv = CQ4{(ccd_real)r[S_ROTINV], (ccd_real)r[S_ROTINV + 1], (ccd_real)r[S_ROTINV + 2], (ccd_real)r[S_ROTINV + 3]};
  o.pos = cv3(r[S_POS], r[S_POS + 1], r[S_POS + 2]);
  o.geom = w.static_geom[sid];
  o.type = w.geom_type[o.geom];
  return o;
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// ---------------------------------------------------------------------------
// Phase A: one lane per configuration (mpg_broadphase.h).
//   1. fp32 FK over the tree -> per moving object its world OBB centre in LDS
//      ([object][3][lane]) and its rotation quaternion in the workspace
//      (rq[object][4][cfg]: its rotation as a quaternion, read back only by
//      the SAT stage);
//   2. pairs are walked grouped by their moving object (host-built schedule,
//      ACM-allowed pairs dropped): the object's centre is loaded once, then
//      a cheap bounding test per partner (sphere-OBB against static objects,
//      sphere-sphere against moving ones);
//   3. pairs that pass are queued per wave in LDS as (pair, lane) entries and
//      the 15-axis OBB SAT runs 64 queued entries at a time with every lane
//      busy -- one lane's survivor no longer makes the whole wave pay;
//   4. SAT survivors set the configuration's bit in an LDS survivor word,
//      written to surv[word][cfg] at the end (no global atomics).
// Also zeroes this configuration's outputs for phase B.
// ---------------------------------------------------------------------------
#ifndef MPG_TASK
#define MPG_TASK 128
#endif
#ifndef MPG_REFILL
#define MPG_REFILL 32
#endif
constexpr int kQueue = 128;  // entries per wave: < 64 pending + <= 64 pushed
constexpr uint32_t kTask = MPG_TASK;  // narrow phase: candidates of one pair per wave task

// inclusive scan of one value per lane across the wave
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = __shfl_up(v, off);
    if (lane >= (uint32_t)off) v += u;
  }
  return v;
}

template <int BLOCK>
__device__ __forceinline__ FObb bp_obb(const DevWorld& w, const float* __restrict__ cen, const float* __restrict__ rq,
                                       long long cap, int id, int t, long long cfg) {
  FObb o;
  if (id < w.n_moving) {
    const float* q = rq + (size_t)id * 4 * cap + cfg;
    f_quat_to_mat(q[3 * cap], q[0], q[cap], q[2 * cap], o.R);
    const float* c = cen + (size_t)id * 3 * BLOCK + t;
    o.c[0] = c[0];
    o.c[1] = c[BLOCK];
    o.c[2] = c[2 * BLOCK];
    const cptr<float> g = w.bp.mobj + BM_STRIDE * id;
    o.e[0] = g[BM_E];
    o.e[1] = g[BM_E + 1];
    o.e[2] = g[BM_E + 2];
  } else {
    const cptr<float> g = w.bp.sobj + BS_STRIDE * (id - w.n_moving);
#pragma unroll
    for (int k = 0; k < 3; ++k) o.c[k] = g[BS_C + k];
#pragma unroll
    for (int k = 0; k < 9; ++k) o.R[k] = g[BS_R + k];
#pragma unroll
    for (int k = 0; k < 3; ++k) o.e[k] = g[BS_E + k];
  }
  return o;
}

template <int BLOCK>
__device__ __forceinline__ void sat_drain(const DevWorld& w, const float* __restrict__ cen, const float* __restrict__ rq,
                                          long long cap, long long cfg0, uint32_t* survw, const uint32_t* queue,
                                          uint32_t head, uint32_t cnt, int wbase, uint32_t lane) {
  __builtin_amdgcn_wave_barrier();
  if (lane < cnt) {
    const uint32_t e = queue[(head + lane) & (kQueue - 1)];  // (schedule entry, lane)
    const int p = w.sched_pair[(int)(e >> 6)], t = wbase + (int)(e & 63u);
    const FObb A = bp_obb<BLOCK>(w, cen, rq, cap, w.pair_a[p], t, cfg0 + t);
    const FObb B = bp_obb<BLOCK>(w, cen, rq, cap, w.pair_b[p], t, cfg0 + t);
    if (!fobb_separated(A, B, w.bp_margin)) atomicOr(&survw[(p >> 5) * BLOCK + t], 1u << (p & 31));
  }
  __builtin_amdgcn_wave_barrier();
}

template <int BLOCK, bool FROM_POSES>
__global__ __launch_bounds__(BLOCK) void cull_kernel(DevWorld w, const double* __restrict__ in, long long n,
                                                    uint8_t* __restrict__ flags, uint32_t* __restrict__ masks,
                                                    uint32_t* __restrict__ surv, float* __restrict__ rq,
                                                    double* __restrict__ sc, long long cap,
                                                    uint32_t* __restrict__ cnt, int n_tiles) {
  extern __shared__ __attribute__((aligned(16))) float lds_f[];
  float* cen = lds_f;                                                    // [n_moving][3][BLOCK]
  float* save = cen + (size_t)w.n_moving * 3 * BLOCK;  // [n_saves - kRegSaves][12][BLOCK]
  uint32_t* survw = reinterpret_cast<uint32_t*>(save + (size_t)max(w.bp.n_saves - kRegSaves, 0) * 12 * BLOCK);  // [W][BLOCK]
  const int tid = threadIdx.x;
  uint32_t* queue = survw + (size_t)w.W * BLOCK + (tid >> 6) * kQueue;  // [BLOCK/64][kQueue]
  const uint32_t lane = lane_id();
  const int wbase = tid & ~63;
  const long long cfg0 = (long long)blockIdx.x * BLOCK;
  const long long cfg = cfg0 + tid;
  const bool live = cfg < n;
  const long long c = live ? cfg : n - 1;  // dead lanes shadow a valid row and never queue
  if (live) {
    flags[cfg] = 0;
    if (masks)
      for (int k = 0; k < w.W; ++k) masks[cfg * w.W + k] = 0u;
  }
  for (int k = 0; k < w.W; ++k) survw[k * BLOCK + tid] = 0u;
  if (w.dbg(14)) return;  // diagnostics: the launch and the output zeroing alone

  // object m's rotation (quaternion q) to rq, its OBB centre to cen
  auto store_obj = [&](int m, const float* q, const float* c) {
    if (live && !w.dbg(13)) {  // 13: diagnostics, FK without the rq stores
      float* r = rq + (size_t)m * 4 * cap + cfg;
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k * cap] = q[k];
    }
    float* r = cen + (size_t)m * 3 * BLOCK + tid;
#pragma unroll
    for (int i = 0; i < 3; ++i) r[i * BLOCK] = c[i];
  };
  // link-pose input: the object's world transform
  auto put = [&](int m, const F34& T) {
    float q[4], c[3];
    f_mat_to_quat(T.R, q);
    const cptr<float> g = w.bp.mobj + BM_STRIDE * m;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      c[i] = T.R[3 * i] * g[BM_C] + T.R[3 * i + 1] * g[BM_C + 1] + T.R[3 * i + 2] * g[BM_C + 2] + T.p[i];
    store_obj(m, q, c);
  };
  // joint-value input: the object's joint frame J (and its quaternion jq)
  auto put_j = [&](int m, const F34& J, const float* jq) {
    MPG_FP32_CONTRACT
    float q[4], c[3];
    const cptr<float> oq = w.bp.oquat + 4 * m, oc = w.bp.ocen + 3 * m;
    const float o[4] = {oq[0], oq[1], oq[2], oq[3]};
    f_quat_mul(jq, o, q);
#pragma unroll
    for (int i = 0; i < 3; ++i) c[i] = J.R[3 * i] * oc[0] + J.R[3 * i + 1] * oc[1] + J.R[3 * i + 2] * oc[2] + J.p[i];
    store_obj(m, q, c);
  };
  // a configuration outside the bounds the cull's margins assume (a prismatic
  // value beyond its travel bound, or a given link pose beyond the chain's
  // reach) is evaluated with every pair
  bool forced = false;
  if (FROM_POSES) {
    for (int m = 0; m < w.n_moving; ++m) put(m, bp_from_pose7(w.bp, in + (c * w.n_links + w.moving_link[m]) * 7, m));
    for (int l = 0; l < w.n_links; ++l) {
      const double* pl = in + (c * w.n_links + l) * 7;
      forced |= !(std::fabs(pl[0]) <= w.pose_bound && std::fabs(pl[1]) <= w.pose_bound && std::fabs(pl[2]) <= w.pose_bound);
    }
  } else {
    bp_fk(w.bp, in + c * w.dof, save + tid, BLOCK, put_j);
    if (w.n_prism)
      for (int j = 0; j < w.nj; ++j)
        if (w.prism_bound[j] >= 0.0) forced |= !(std::fabs(in[c * w.dof + w.joint_q_source[j]]) <= w.prism_bound[j]);
  }
  if (w.dbg(1) || w.dbg(13)) {
    if (live && cen[tid] == 12345.f) flags[cfg] = 2;  // keep the records alive
    return;
  }

  uint32_t head = 0, tail = 0;  // wave-uniform queue cursors
  uint32_t dbg_keep = 0u;       // diagnostics (11): the bounding tests' bits, kept alive
  // queue the entries [eb, eb + 32) some lane kept (kb: this lane's bits);
  // drain 64 queued (pair, lane) entries through the SAT at a time
  auto push = [&](int eb, uint32_t kb) {
    if (!live) kb = 0u;
    if (w.dbg(11)) {
      dbg_keep += kb;
      return;
    }
    if (w.dbg(2)) {
      for (int i = 0; i < 32; ++i) {
        if (!((kb >> i) & 1u)) continue;
        const int p = w.sched_pair[eb + i];
        survw[(p >> 5) * BLOCK + tid] |= 1u << (p & 31);
      }
      return;
    }
    // one wave scan of the kept counts: each lane writes its own entries
    // (schedule index, lane) at its offset, no per-entry wave-level loop
    {
    const uint32_t c = (uint32_t)__popc(kb);
    // the prefix sum by bit planes of the counts (<= 32: six ballots), no LDS
    uint32_t ex = 0u, total = 0u;
#pragma unroll
    for (int bit = 0; bit < 6; ++bit) {
      const unsigned long long m = __ballot((c >> bit) & 1u);
      ex += __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << bit;
      total += (uint32_t)__popcll(m) << bit;
    }
    const uint32_t incl = ex + c;
    if (total == 0u) return;
    if (tail - head + total <= (uint32_t)kQueue) {
      uint32_t pos = tail + incl - c;
      while (kb) {
        const int i = __builtin_ctz(kb);
        kb &= kb - 1u;
        queue[pos++ & (kQueue - 1)] = ((uint32_t)(eb + i) << 6) | lane;
      }
      tail += total;
      while (tail - head >= 64) {
        sat_drain<BLOCK>(w, cen, rq, cap, cfg0, survw, queue, head, 64, wbase, lane);
        head += 64;
      }
      return;
    }
    }
    // more than the queue holds: entry by entry, draining as it fills
    uint32_t any_kb = kb;  // entries some lane of the wave kept
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) any_kb |= (uint32_t)__shfl_xor((int)any_kb, sh);
    any_kb = __builtin_amdgcn_readfirstlane(any_kb);
    while (any_kb) {
      const int i = __builtin_ctz(any_kb);
      any_kb &= any_kb - 1u;
      const bool keep = (kb >> i) & 1u;
      const unsigned long long bal = __ballot(keep);
      if (keep) {
        const uint32_t rank =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        queue[(tail + rank) & (kQueue - 1)] = ((uint32_t)(eb + i) << 6) | lane;
      }
      tail += (uint32_t)__popcll(bal);
      if (tail - head >= 64) {
        sat_drain<BLOCK>(w, cen, rq, cap, cfg0, survw, queue, head, 64, wbase, lane);
        head += 64;
      }
    }
  };
  // moving-static pairs, static-major: the static's OBB record is loaded
  // once (scalar registers) for all its entries, each entry a moving object's
  // bounding sphere (centre from LDS); group 1 (objects whose reach ball
  // never comes near the static) only for link-pose input, which does not
  // assume the kinematics
  const int ns = w.n_static;
  for (int g = 0; g < (FROM_POSES ? 2 : 1) && !w.dbg(12); ++g) {  // 12: diagnostics, without these tests
    const int E0 = w.st_start[g * (ns + 1)], E1 = w.st_start[g * (ns + 1) + ns];
    if (E0 == E1) continue;
    int eb = E0;
    uint32_t kb = 0u;
    for (int sid = 0; sid < ns; ++sid) {
      const int e0 = w.st_start[g * (ns + 1) + sid], e1 = w.st_start[g * (ns + 1) + sid + 1];
      if (e0 == e1) continue;
      const cptr<float> rec = w.bp.sobj + BS_STRIDE * sid;
      float sr[BS_STRIDE];
#pragma unroll
      for (int k = 0; k < BS_STRIDE; ++k) sr[k] = rec[k];
#pragma unroll 2
      for (int e = e0; e < e1; ++e) {
        if (e - eb == 32) {
          push(eb, kb);
          eb = e;
          kb = 0u;
        }
        const float* rm = cen + (size_t)w.st_m[e] * 3 * BLOCK + tid;
        const float cm[3] = {rm[0], rm[BLOCK], rm[2 * BLOCK]};
        kb |= (uint32_t)!fsphere_obb_separated(cm, w.st_r[e], sr, w.bp_margin) << (e - eb);
      }
    }
    push(eb, kb);
  }
  // moving-moving pairs: bounding spheres (both centres from LDS)
  for (int m = 0; m < w.n_moving; ++m) {
    const int e0 = w.sched_start[m], e1 = w.sched_start[m + 1];
    if (e0 == e1) continue;
    const float* rm = cen + (size_t)m * 3 * BLOCK + tid;
    const float cm[3] = {rm[0], rm[BLOCK], rm[2 * BLOCK]};
    const float r_m = w.bp.mobj[BM_STRIDE * m + BM_R];
    for (int eb = e0; eb < e1; eb += 32) {
      const int ee = min(e1, eb + 32);
      uint32_t kb = 0u;
#pragma unroll 4
      for (int e = eb; e < ee; ++e) {
        const int o = w.sched_other[e];
        const float* ro = cen + (size_t)o * 3 * BLOCK + tid;
        const float dx = ro[0] - cm[0], dy = ro[BLOCK] - cm[1], dz = ro[2 * BLOCK] - cm[2];
        const float rr = r_m + w.bp.mobj[BM_STRIDE * o + BM_R] + w.bp_margin;
        kb |= (uint32_t)(dx * dx + dy * dy + dz * dz <= rr * rr) << (e - eb);
      }
      push(eb, kb);
    }
  }
  if (tail != head) sat_drain<BLOCK>(w, cen, rq, cap, cfg0, survw, queue, head, tail - head, wbase, lane);
  if (forced)
    for (int k = 0; k < w.W; ++k) survw[k * BLOCK + tid] = (uint32_t)w.all_mask[k];
  if (w.dbg(8) || w.dbg(11)) {  // ablation: bounding tests + SAT only (11: without the queue and SAT)
    if (live && (survw[tid] == 12345u || dbg_keep == 12345u)) flags[cfg] = 2;
    return;
  }
  // survivor words -> surv, and this wave's candidate count per pair ->
  // cnt[pair][tile] (the bucketing's tile counts; cnt is zeroed before the
  // launch, pairs without a survivor in the tile are skipped).  The counts
  // are a per-wave histogram in the idle queue area: 8-bit counters (<= 64
  // each), four per word, every lane adding its own survivors, then each lane
  // writes the counts of pairs lane, lane + 64, ...  Worlds with more pairs
  // than the area holds (W > kQueue / 8) take one ballot per distinct pair.
  bool any = false;
  const long long tile = (cfg0 >> 6) + (tid >> 6);
  if (w.W * 8 <= kQueue) {
    uint32_t* hist = queue;
    for (int i = (int)lane; i < w.W * 8; i += 64) hist[i] = 0u;
    wave_lds_sync();
    for (int k = 0; k < w.W; ++k) {
      uint32_t x = live ? survw[k * BLOCK + tid] : 0u;
      if (live) surv[(long long)k * cap + cfg] = x;
      any |= x != 0u;
      while (x) {
        const int p = k * 32 + __builtin_ctz(x);
        x &= x - 1u;
        atomicAdd(&hist[p >> 2], 1u << (8 * (p & 3)));
      }
    }
    wave_lds_sync();
    for (int p = (int)lane; p < w.W * 32; p += 64) {
      const uint32_t c = (hist[p >> 2] >> (8 * (p & 3))) & 0xffu;
      if (c) cnt[(long long)p * n_tiles + tile] = c;
    }
  } else {
    for (int k = 0; k < w.W; ++k) {
      uint32_t x = live ? survw[k * BLOCK + tid] : 0u;
      if (live) surv[(long long)k * cap + cfg] = x;
      any |= x != 0u;
      for (;;) {
        const unsigned long long m = __ballot(x != 0u);
        if (m == 0) break;
        const uint32_t xl = __builtin_amdgcn_readlane(x, __builtin_ctzll(m));
        const int b = __builtin_ctz(xl);
        const unsigned long long bb = __ballot((x >> b) & 1u);
        x &= ~(1u << b);
        if (lane == 0) cnt[(long long)(k * 32 + b) * n_tiles + tile] = (uint32_t)__popcll(bb);
      }
    }
  }
  if (FROM_POSES || w.dbg(9)) return;  // 9: ablation without the sincos pass
  // Exact fp64 sin/cos of every revolute move-group joint for the narrow
  // phase's chain FK (the glibc sincos restatement), only for configurations
  // with a candidate pair (about a quarter of them): compacted across the
  // block through LDS (the SAT queues are free now) so every lane works.
  uint32_t* list = survw + (size_t)w.W * BLOCK;  // [BLOCK] + per-wave counts [BLOCK / 64]
  uint32_t* wcnt = list + BLOCK;
  __syncthreads();
  const unsigned long long bal = __ballot(any);
  if (lane == 0) wcnt[tid >> 6] = (uint32_t)__popcll(bal);
  __syncthreads();
  uint32_t off = 0, total = 0;
  for (int k = 0; k < BLOCK / 64; ++k) {
    off += k < (tid >> 6) ? wcnt[k] : 0u;
    total += wcnt[k];
  }
  if (any)
    list[off + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = tid;
  __syncthreads();
  if ((uint32_t)tid < total) {
    const long long r = cfg0 + list[tid];
    for (int j = 0; j < w.nj; ++j) {
      const int src = w.joint_q_source[j];
      if (src < 0 || !joint_is_revolute(w.joint_type[j])) continue;
      double sv, cv;
      mpg_sincos(in[r * w.dof + src], &sv, &cv);
      sc[(r * w.dof + src) * 2] = sv;
      sc[(r * w.dof + src) * 2 + 1] = cv;
    }
  }
}

// ---------------------------------------------------------------------------
// Deterministic bucketing of the survivor bits into per-pair candidate lists
// (no global atomics): count per (pair, 64-config tile) -> per-pair scan ->
// scatter.  Candidates of a pair end up contiguous and sorted by config.
// ---------------------------------------------------------------------------
// one block per pair: exclusive scan of its tile counts (in place) + total.
// Each thread holds up to 16 consecutive counts in registers (loads issued
// together), one wave scan + one LDS exchange of the 16 wave totals.
__global__ __launch_bounds__(1024) void pair_scan_kernel(uint32_t* __restrict__ cnt, int n_tiles,
                                                        uint32_t* __restrict__ seg_len) {
  __shared__ uint32_t part[16];
  uint32_t* c = cnt + (long long)blockIdx.x * n_tiles;
  const int per = (n_tiles + 1023) / 1024;
  const int lo = threadIdx.x * per, hi = min(n_tiles, lo + per);
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint32_t v[16];
  uint32_t sum = 0;
  if (per <= 16) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      v[k] = lo + k < hi ? c[lo + k] : 0u;
      sum += v[k];
    }
  } else {
    for (int i = lo; i < hi; ++i) sum += c[i];
  }
  const uint32_t incl = wave_inclusive_scan(sum, lane);
  if (lane == 63u) part[wv] = incl;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    const uint32_t x = part[k];
    pre += k < wv ? x : 0u;
    tot += x;
  }
  uint32_t run = pre + incl - sum;
  if (per <= 16) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (lo + k < hi) c[lo + k] = run;
      run += v[k];
    }
  } else {
    for (int i = lo; i < hi; ++i) {
      const uint32_t x = c[i];
      c[i] = run;
      run += x;
    }
  }
  if (threadIdx.x == 0) seg_len[blockIdx.x] = tot;
}

// segment starts + prefix of narrow-phase tasks (ts candidates of one pair
// each): one block, 256 pairs per round.  The task size adapts to the batch:
// ts = total candidates / target tasks (the narrow grid's resident waves),
// clamped to [kTaskMin, kTask] and rounded up to a multiple of 8 -- small
// batches (cfg2's 2^16 self pairs: ~27k candidates) spread over the whole
// chip instead of a few hundred full waves.  prefix[n_pairs] = task count,
// prefix[n_pairs + 1] = the narrow phase's task counter, prefix[n_pairs + 2]
// = ts, prefix[n_pairs + 3] = the candidate count.
#ifndef MPG_TASK_MIN
#define MPG_TASK_MIN 8
#endif
constexpr uint32_t kTaskMin = MPG_TASK_MIN;

__device__ __forceinline__ uint32_t block_sum256(uint32_t v, uint32_t* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if ((threadIdx.x & 63u) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void chunk_scan_kernel(const uint32_t* __restrict__ seg_len, int n_pairs,
                                                        uint32_t* __restrict__ seg_start,
                                                        uint32_t* __restrict__ prefix, unsigned long long* units,
                                                        uint32_t target_tasks) {
  __shared__ uint32_t wl[4], wt[4], red[4];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint32_t part = 0;
  for (int p = (int)threadIdx.x; p < n_pairs; p += 256) part += seg_len[p];
  const uint32_t all = block_sum256(part, red);
  uint32_t ts = target_tasks ? (all + target_tasks - 1) / target_tasks : kTask;
  ts = ts < kTaskMin ? kTaskMin : (ts > kTask ? kTask : ts);
  ts = (ts + 7u) & ~7u;
  uint32_t cl = 0, ct = 0;  // carries over rounds
  for (int p0 = 0; p0 < n_pairs; p0 += 256) {
    const int p = p0 + (int)threadIdx.x;
    const uint32_t len = p < n_pairs ? seg_len[p] : 0u;
    const uint32_t tasks = (len + ts - 1) / ts;
    const uint32_t il = wave_inclusive_scan(len, lane), it = wave_inclusive_scan(tasks, lane);
    if (lane == 63) {
      wl[wv] = il;
      wt[wv] = it;
    }
    __syncthreads();
    uint32_t bl = cl, bt = ct;
    for (uint32_t k = 0; k < wv; ++k) {
      bl += wl[k];
      bt += wt[k];
    }
    if (p < n_pairs) {
      seg_start[p] = bl + il - len;
      prefix[p] = bt + it - tasks;
    }
    for (uint32_t k = 0; k < 4; ++k) {
      cl += wl[k];
      ct += wt[k];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    prefix[n_pairs] = ct;
    prefix[n_pairs + 1] = 0;  // narrow-phase task counter
    prefix[n_pairs + 2] = ts;
    prefix[n_pairs + 3] = cl;  // candidates in all (diagnostics)
    if (units) atomicAdd(units, (unsigned long long)cl);  // profiling: narrow-phase candidates
  }
}

// one wave per (survivor word, 64-config tile): the slot bases of the
// word's surviving pairs come in one parallel load (lane b: pair 32 wd + b),
// then each surviving pair's configurations are written at base + rank
__global__ __launch_bounds__(256) void scatter_kernel(const uint32_t* __restrict__ surv, long long n, long long cap,
                                                     int n_pairs, int W, int n_tiles,
                                                     const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ seg_start,
                                                     uint32_t* __restrict__ cand) {
  const uint32_t lane = lane_id();
  const long long wid = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (wid >= (long long)n_tiles * W) return;
  const int wd = (int)(wid / n_tiles), t = (int)(wid % n_tiles);
  const long long cfg = (long long)t * 64 + lane;
  const uint32_t x = cfg < n ? surv[(long long)wd * cap + cfg] : 0u;
  uint32_t o = x;
#pragma unroll
  for (int sh = 1; sh < 64; sh <<= 1) o |= (uint32_t)__shfl_xor((int)o, sh);
  o = __builtin_amdgcn_readfirstlane(o);
  if (o == 0u) return;
  uint32_t base = 0u;
  if (lane < 32u && ((o >> lane) & 1u)) {
    const int p = wd * 32 + (int)lane;
    base = seg_start[p] + off[(long long)p * n_tiles + t];
  }
  for (uint32_t m = o; m; m &= m - 1u) {
    const int b = __builtin_ctz(m);
    const uint32_t bit = (x >> b) & 1u;
    const unsigned long long bal = __ballot(bit);
    const uint32_t bs = __builtin_amdgcn_readlane(base, b);
    if (bit)
      cand[bs + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] =
          (uint32_t)cfg;
  }
}

// binary search of the pair whose task range holds task tk: prefix[p] <= tk < prefix[p + 1]
__device__ __forceinline__ int task_pair(const uint32_t* __restrict__ prefix, int n_pairs, uint32_t tk) {
  int lo = 0, hi = n_pairs;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (prefix[mid] <= tk) lo = mid;
    else hi = mid;
  }
  return lo;
}

// ---------------------------------------------------------------------------
// Phase B: exact narrow phase.  Each wave takes 64 candidates of ONE pair, so
// every lane scans the same hull (wave-uniform scalar loads of the vertices)
// and only the MPR iteration count diverges.  Poses are rebuilt in fp64 from
// the joint values (chain FK), bit-identical to phase A / the reference.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Phase B: exact narrow phase (fp64, bit-identical to the reference).
//
// A wave takes a task of up to kTask candidates of ONE pair, so every lane
// scans the same hull (wave-uniform scalar loads).  libccd's MPR is run as a
// per-lane state machine whose every step is exactly one Minkowski support
// call: all lanes step together through the (uniform) support scan and only
// the cheap portal update diverges.  A lane that finishes takes the next
// candidate of the task; refills are batched (>= 32 idle lanes, or none
// active) so the fp64 chain FK of the refilled lanes runs at high lane
// occupancy too.  Results: atomicOr into the pair mask, flag = 1.
//
// States follow ccdMPRIntersect (libccd 2.1 mpr.c): discoverPortal's v1, v2
// and v3 support points (1, 2, 3), then refinePortal's v4 (4).
// ---------------------------------------------------------------------------
enum : int { MPR_DONE = 0, MPR_V1 = 1, MPR_V2 = 2, MPR_V3 = 3, MPR_V4 = 4 };

__device__ __forceinline__ bool octree_wave(const DevWorld& w, cptr<double> HV, int go, const SE3& TO, int gs,
                                           const SE3& TS);

template <int CLS>
__device__ __forceinline__ unsigned long long walk_wave_eval(const DevWorld& w, cptr<double> HV, int ga, const SE3& TA,
                                                            int gb, const SE3& TB, bool active);

// one pair evaluation of class CLS: closed form, octree walk or BVH mesh
// walk; each class lives in its own kernel instance so the walks' registers
// never lower the other kernels' occupancy
template <int CLS>
__device__ __forceinline__ bool pair_closed_form(int cf, const DevWorld& w, int ga, const SE3& TA, int gb,
                                                 const SE3& TB) {
  if constexpr (CLS == CLS_CLOSED) return closed_form(cf, w, ga, TA, gb, TB);
  if constexpr (CLS == CLS_GJK) return gjk_indep_intersect(w, ga, TA, gb, TB);
  return false;  // octree / mesh pairs: evaluated wave-wide (walk_wave_eval)
}

// FCL closed-form pairs (box-box, sphere-sphere, sphere-box) and octree
// pairs of the candidate lists: one test per candidate.  A kernel of its own so the closed forms'
// registers do not lower the MPR kernel's occupancy.
template <bool FROM_POSES, int CLS>
__global__ __launch_bounds__(256, CLS == CLS_OCTREE ? 2 : 1) void closed_form_kernel(DevWorld w, const double* __restrict__ in,
                                                         const uint32_t* __restrict__ seg_len,
                                                         const uint32_t* __restrict__ seg_start,
                                                         const uint32_t* __restrict__ prefix,
                                                         const uint32_t* __restrict__ cand,
                                                         uint8_t* __restrict__ flags, uint32_t* __restrict__ masks,
                                                         const double* __restrict__ sc) {
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t total = prefix[w.n_pairs];
  for (uint32_t tk = wave; tk < total; tk += n_waves) {
    int lo = 0, hi = w.n_pairs;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (prefix[mid] <= tk) lo = mid;
      else hi = mid;
    }
    const int p = lo;
    const int cf = w.pair_cf[p];
    if (cf == CF_NONE || cf_class(cf) != CLS) continue;
    const uint32_t ts = prefix[w.n_pairs + 2];
    const uint32_t t0 = (tk - prefix[p]) * ts, t1 = min(seg_len[p], t0 + ts);
    const int a = w.pair_a[p], b = w.pair_b[p];
    const bool am = a < w.n_moving, bm = b < w.n_moving;
    const int ga = am ? w.moving_geom[a] : w.static_geom[a - w.n_moving];
    const int gb = bm ? w.moving_geom[b] : w.static_geom[b - w.n_moving];
    const uint32_t* __restrict__ cl = cand + seg_start[p];
    for (uint32_t base = t0; base < t1; base += 64) {
      const uint32_t idx = base + lane;
      if constexpr (CLS == CLS_OCTREE || CLS == CLS_MESH) {  // the wave walks each candidate together
        const bool active = idx < t1;
        const long long c = active ? cl[idx] : 0;
        SE3 TA = {}, TB = {};
        if (active) {
          TA = am ? moving_tf<FROM_POSES>(w, in, sc, c, a) : load_se3(w.static_T + 12 * (a - w.n_moving));
          TB = bm ? moving_tf<FROM_POSES>(w, in, sc, c, b) : load_se3(w.static_T + 12 * (b - w.n_moving));
        }
        const unsigned long long hits = walk_wave_eval<CLS>(w, w.hull, ga, TA, gb, TB, active);
        if ((hits >> lane) & 1ull) {
          if (masks) atomicOr(&masks[c * w.W + (p >> 5)], 1u << (p & 31));
          flags[c] = 1;
        }
        continue;
      }
      if (idx >= t1) continue;
      const long long c = cl[idx];
      const SE3 TA = am ? moving_tf<FROM_POSES>(w, in, sc, c, a) : load_se3(w.static_T + 12 * (a - w.n_moving));
      const SE3 TB = bm ? moving_tf<FROM_POSES>(w, in, sc, c, b) : load_se3(w.static_T + 12 * (b - w.n_moving));
      if (pair_closed_form<CLS>(cf, w, ga, TA, gb, TB)) {
        if (masks) atomicOr(&masks[c * w.W + (p >> 5)], 1u << (p & 31));
        flags[c] = 1;
      }
    }
  }
}

// One libccd MPR step (ccdMPRIntersect = discoverPortal + refinePortal) for
// a lane whose new Minkowski support point in direction `dir` is `s`.
// States: MPR_V1..V3 discoverPortal (finding v1, v2, v3), MPR_V4 refinePortal.
// Returns 1 = intersect, -1 = separated, 0 = continue with the updated dir.
// The state is copied into locals and written back unconditionally: stores
// under branches through the reference parameters get merged into stores
// through a selected pointer, which keeps the caller's registers on the stack.
__device__ __forceinline__ int mpr_advance(ccd_real mpr_tol, const CV3& s, int& st_io, CV3& v0_io, CV3& v1_io, CV3& v2_io,
                                           CV3& v3_io, CV3& dir_io) {
  int st = st_io;
  CV3 v0 = v0_io, v1 = v1_io, v2 = v2_io, v3 = v3_io, dir = dir_io;
  int res = 0;  // 1 = intersect, -1 = separated
  // Every state ends in one new search direction dir = normalize(a x b);
  // the states only pick (a, b), so the costly normalize (sqrt + divide)
  // runs once per step for all lanes instead of once per state branch.
  const ccd_real dsd = vdot(s, dir);
  CV3 ca, cb;
  bool post_swap = false, post_encl = false;
  if (st == MPR_V4) {  // refinePortal: expand the portal (v1, v2, v3) towards v4 = s
    if (!(is_zero(dsd) || dsd > 0)) {
      res = -1;
    } else {
      const ccd_real dv1 = vdot(v1, dir), dv2 = vdot(v2, dir), dv3 = vdot(v3, dir);
      ccd_real d1 = dsd - dv1;
      const ccd_real dd2 = dsd - dv2, dd3 = dsd - dv3;
      d1 = (d1 < dd2) ? d1 : dd2;  // CCD_FMIN
      d1 = (d1 < dd3) ? d1 : dd3;
      if (ccd_eq(d1, mpr_tol) || d1 < mpr_tol) {
        res = -1;
      } else {
        const CV3 v4v0 = vcross(s, v0);
        if (vdot(v1, v4v0) > 0) {
          if (vdot(v2, v4v0) > 0) v1 = s;
          else v3 = s;
        } else {
          if (vdot(v3, v4v0) > 0) v2 = s;
          else v1 = s;
        }
        ca = vsub(v2, v1);
        cb = vsub(v3, v1);
        post_encl = true;
      }
    }
  } else if (is_zero(dsd) || dsd < 0) {  // discoverPortal: support not past the origin
    res = -1;
  } else if (st == MPR_V1) {
    v1 = s;
    ca = v0;
    cb = v1;
  } else if (st == MPR_V2) {
    v2 = s;
    ca = vsub(v1, v0);
    cb = vsub(v2, v0);
    post_swap = true;
  } else {  // MPR_V3
    v3 = s;
    bool cont = false;
    ccd_real d2 = vdot(vcross(v1, v3), v0);
    if (d2 < 0 && !is_zero(d2)) {
      v2 = v3;
      cont = true;
    }
    if (!cont) {
      d2 = vdot(vcross(v3, v2), v0);
      if (d2 < 0 && !is_zero(d2)) {
        v1 = v3;
        cont = true;
      }
    }
    if (cont) {
      ca = vsub(v1, v0);
      cb = vsub(v2, v0);
    } else {  // portal found: refinePortal starts with (v1, v2, v3)
      ca = vsub(v2, v1);
      cb = vsub(v3, v1);
      post_encl = true;
      st = MPR_V4;
    }
  }
  if (res == 0) {
    const CV3 cr = vcross(ca, cb);
    if (st == MPR_V1 && is_zero(vdot(cr, cr))) {
      res = 1;  // origin on v1 or on segment v0-v1
    } else {
      dir = vnormalize(cr);
      if (st == MPR_V1) {
        st = MPR_V2;
      } else if (post_swap) {
        if (vdot(dir, v0) > 0) {
          const CV3 t = v1;
          v1 = v2;
          v2 = t;
          dir = vscale(dir, ccd_real(-1));
        }
        st = MPR_V3;
      } else if (post_encl) {  // portalEncapsulesOrigin
        const ccd_real d = vdot(dir, v1);
        if (is_zero(d) || d > 0) res = 1;
      }
    }
  }
  st_io = st;
  v0_io = v0;
  v1_io = v1;
  v2_io = v2;
  v3_io = v3;
  dir_io = dir;
  return res;
}

// ccdMPRIntersect's start: findOrigin (v0 = centre difference, nudged off the
// origin) and discoverPortal's first direction
__device__ __forceinline__ void mpr_begin(const CV3& ca, const CV3& cb, int& st, CV3& v0, CV3& dir) {
  v0 = vsub(ca, cb);
  if (vec_is_origin(v0)) v0 = vadd(v0, cv3(kCcdEps * ccd_real(10), 0.0, 0.0));
  dir = vnormalize(vscale(v0, ccd_real(-1)));
  st = MPR_V1;
}

// libccd support of (box with per-lane half sizes h) - (uniform shape b)
__device__ __forceinline__ CV3 msupport_box(const GObj& a, const ccd_real* h, const DevWorld& w, cptr<double> HV,
                                           const GObj& b, const CV3& dir) {
  const CV3 da = quat_rot(dir, a.rot_inv), db = quat_rot(vscale(dir, ccd_real(-1)), b.rot_inv);
  const CV3 la = CV3{(da.x >= 0 ? ccd_real(1) : ccd_real(-1)) * h[0], (da.y >= 0 ? ccd_real(1) : ccd_real(-1)) * h[1],
                     (da.z >= 0 ? ccd_real(1) : ccd_real(-1)) * h[2]};
  const int gb = __builtin_amdgcn_readfirstlane(b.geom), tb = __builtin_amdgcn_readfirstlane(b.type);
  const CV3 lb = support_local(w, HV, gb, tb, db);
  return vsub(vadd(quat_rot(la, a.rot), a.pos), vadd(quat_rot(lb, b.rot), b.pos));
}

// The occupied leaves of octree `go` listed in the grid cells under the box
// [blo, bhi] (octree frame), handed out one per lane: the cells of the range
// 64 at a time (one per lane, loads in parallel), then a wave prefix sum of
// their leaf counts gives the leaves 64 at a time.  leaf_hit(leaf) -> bool;
// true as soon as some lane's leaf hits.  Wave-uniform inputs.  (A leaf in
// several cells may be tested more than once: the answer is an OR.)
template <typename F>
__device__ __forceinline__ bool octree_range_any(const DevWorld& w, int go, const double* blo, const double* bhi,
                                                 F leaf_hit) {
  const cptr<double> og = w.oct_grid + OG_STRIDE * go;
  const double inv = og[OG_INV];
  int c0[3], c1[3], dims[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    dims[i] = (int)og[OG_DIMS + i];
    const double f0 = std::floor((blo[i] - og[OG_ORIGIN + i]) * inv);
    const double f1 = std::floor((bhi[i] - og[OG_ORIGIN + i]) * inv);
    if (f1 < 0.0 || f0 >= (double)dims[i]) return false;
    c0[i] = f0 < 0.0 ? 0 : (int)f0;
    c1[i] = f1 >= (double)dims[i] ? dims[i] - 1 : (int)f1;
  }
  __shared__ int s_k0[4][64], s_end[4][64];  // per wave of the 256-thread block
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const int cell0 = (int)og[OG_CELL0];
  const int nx = c1[0] - c0[0] + 1, ny = c1[1] - c0[1] + 1, nz = c1[2] - c0[2] + 1;
  const int ncell = nx * ny * nz;
  for (int cb = 0; cb < ncell; cb += 64) {
    const int ci = cb + (int)lane;
    int k0 = 0, cnt = 0;
    if (ci < ncell) {
      const int z = ci % nz, y = (ci / nz) % ny, x = ci / (nz * ny);
      const int cell = cell0 + ((c0[0] + x) * dims[1] + (c0[1] + y)) * dims[2] + (c0[2] + z);
      k0 = w.oct_cells[cell];
      cnt = w.oct_cells[cell + 1] - k0;
    }
    const uint32_t incl = wave_inclusive_scan((uint32_t)cnt, lane);
    const int total = (int)__builtin_amdgcn_readlane(incl, 63);
    s_k0[wv][lane] = k0;
    s_end[wv][lane] = (int)incl;
    __builtin_amdgcn_wave_barrier();
    for (int ib = 0; ib < total; ib += 64) {
      const int j = ib + (int)lane;
      bool hit = false;
      if (j < total) {
        int lo = 0, hi = 63;  // first cell slot whose inclusive end exceeds j
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (s_end[wv][mid] > j) hi = mid;
          else lo = mid + 1;
        }
        const int start = lo > 0 ? s_end[wv][lo - 1] : 0;
        hit = leaf_hit(w.oct_list[s_k0[wv][lo] + (j - start)]);
      }
      if (__ballot(hit) != 0) return true;
    }
    __builtin_amdgcn_wave_barrier();
  }
  return false;
}

// One lane's (shape, octree) pair: fcl OcTreeSolver::OcTreeShapeIntersectRecurse
// [ext FCL 0.7.0] reduced to its result -- some occupied leaf whose OBB
// overlaps the shape's OBB (computeBV(shape, I) -> convertBV(., tf), then
// obbDisjoint) and whose box intersects the shape: shapeIntersect(box,
// box_tf, shape, tf) with the leaf box first (box-box / box-sphere closed
// forms, otherwise libccd MPR).  An ancestor's OBB contains its leaves', so
// the recursion's pruning never hides a leaf this test would accept.  Leaves
// come from the octree's grid cells under the shape's box in the octree frame
// widened exactly as obbDisjoint's first three axes (|R| + 1e-6): a leaf
// outside it fails those axes.  Inputs are wave-uniform: the whole wave
// walks one candidate.
__device__ __forceinline__ bool octree_wave(const DevWorld& w, cptr<double> HV, int go, const SE3& TO, int gs,
                                           const SE3& TS) {
  const cptr<double> grs = w.geom_rec + G_STRIDE * gs;
  const int ts = w.geom_type[gs];
  double sc[3], se[3], Rl[9], cl[3], hq[3];
#pragma unroll
  // FCL's exact computeBV extents: with float libccd behind the gate, a leaf
  // the gate passes only by a widening could become an MPR hit
  for (int i = 0; i < 3; ++i) se[i] = grs[G_AABB_E + i];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    sc[i] = ((TS.R[3 * i] * grs[G_OBB_C] + TS.R[3 * i + 1] * grs[G_OBB_C + 1]) + TS.R[3 * i + 2] * grs[G_OBB_C + 2]) +
            TS.p[i];
  const double dsc[3] = {sc[0] - TO.p[0], sc[1] - TO.p[1], sc[2] - TO.p[2]};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    cl[i] = (TO.R[i] * dsc[0] + TO.R[3 + i] * dsc[1]) + TO.R[6 + i] * dsc[2];
#pragma unroll
    for (int j = 0; j < 3; ++j) Rl[3 * i + j] = (TO.R[i] * TS.R[j] + TO.R[3 + i] * TS.R[3 + j]) + TO.R[6 + i] * TS.R[6 + j];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
    hq[i] = ((std::fabs(Rl[3 * i]) + 1e-6) * se[0] + (std::fabs(Rl[3 * i + 1]) + 1e-6) * se[1] +
             (std::fabs(Rl[3 * i + 2]) + 1e-6) * se[2]) * (1.0 + 1e-12) + 1e-12;
  // tighter: the shape's own extent along the octree axes (its support in
  // +-axis), padded; a leaf beyond it on an octree axis is separated from
  // the shape, so every leaf test on it fails
  double blo[3], bhi[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double ax[3] = {TO.R[i], TO.R[3 + i], TO.R[6 + i]};
    const V3 dl = v3((TS.R[0] * ax[0] + TS.R[3] * ax[1]) + TS.R[6] * ax[2],
                     (TS.R[1] * ax[0] + TS.R[4] * ax[1]) + TS.R[7] * ax[2],
                     (TS.R[2] * ax[0] + TS.R[5] * ax[1]) + TS.R[8] * ax[2]);
    const V3 sp = support_local_exact(w, HV, gs, ts, dl), sn = support_local_exact(w, HV, gs, ts, vscale(dl, -1.0));
    double ep = 0.0, en = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double lp = (k == 0 ? sp.x : k == 1 ? sp.y : sp.z), ln = (k == 0 ? sn.x : k == 1 ? sn.y : sn.z);
      ep += ax[0] * TS.R[k] * lp + ax[1] * TS.R[3 + k] * lp + ax[2] * TS.R[6 + k] * lp;
      en += ax[0] * TS.R[k] * ln + ax[1] * TS.R[3 + k] * ln + ax[2] * TS.R[6 + k] * ln;
    }
    const double base = (ax[0] * (TS.p[0] - TO.p[0]) + ax[1] * (TS.p[1] - TO.p[1])) + ax[2] * (TS.p[2] - TO.p[2]);
    // libccd MPR can report a leaf within kCcdFalseHitReach of the shape as
    // touching (mpg_math.h): keep every such leaf
    const double pad = kCcdFalseHitReach * (1.0 + 1e-3) + 1e-5 + 1e-5 * (std::fabs(base) + std::fabs(ep) + std::fabs(en));
    blo[i] = fmax(cl[i] - hq[i], base + en - pad);
    bhi[i] = fmin(cl[i] + hq[i], base + ep + pad);
    if (blo[i] > bhi[i]) return false;
  }
  GObj A, B;  // A: the leaf box (rotation of the octree, per-leaf centre), B: the shape
  A.rot = gjk_rot_from_matrix(TO.R);
  A.rot_inv = quat_invert2(A.rot);
  A.geom = go;
  A.type = MPG_GEOM_BOX;
  B.rot = gjk_rot_from_matrix(TS.R);
  B.rot_inv = quat_invert2(B.rot);
  B.pos = cv3(TS.p[0], TS.p[1], TS.p[2]);
  B.geom = gs;
  B.type = ts;
  // one candidate per wave: the leaves listed in the cells under the box
  // are queued 64 at a time (one per lane) and tested side by side
  auto leaf_hit = [&](int leaf) -> bool {
    const cptr<double> L = w.oct_leaf + 6 * (size_t)leaf;
    bool out = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) out |= L[i] > bhi[i] || L[3 + i] < blo[i];
    if (out) return false;
    // leaf OBB: axes TO.R, centre TO * c, extent (max - min) * 0.5
    double c[3], cw[3], a[3], side[3], T[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      c[i] = (L[i] + L[3 + i]) * 0.5;
      side[i] = L[3 + i] - L[i];
      a[i] = side[i] * 0.5;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) cw[i] = ((TO.R[3 * i] * c[0] + TO.R[3 * i + 1] * c[1]) + TO.R[3 * i + 2] * c[2]) + TO.p[i];
    const double t[3] = {sc[0] - cw[0], sc[1] - cw[1], sc[2] - cw[2]};
#pragma unroll
    for (int i = 0; i < 3; ++i) T[i] = (TO.R[i] * t[0] + TO.R[3 + i] * t[1]) + TO.R[6 + i] * t[2];
    if (obb_disjoint(Rl, T, a, se)) return false;
    SE3 TL;  // box_tf = tf * Translation(centre)
#pragma unroll
    for (int i = 0; i < 9; ++i) TL.R[i] = TO.R[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) TL.p[i] = cw[i];
    if (ts == MPG_GEOM_BOX) {
      const double sb[3] = {grs[G_PARAM], grs[G_PARAM + 1], grs[G_PARAM + 2]};
      return box_box_intersect(side, TL, sb, TS);
    }
    if (ts == MPG_GEOM_SPHERE) return sphere_box_intersect(grs[G_PARAM], TS, side, TL);
    GObj A1 = A;
    A1.pos = cv3(cw[0], cw[1], cw[2]);
    const ccd_real h[3] = {(ccd_real)(side[0] / 2.0), (ccd_real)(side[1] / 2.0), (ccd_real)(side[2] / 2.0)};  // boxToGJK
    int st;
    CV3 v0, v1, v2, v3_, dir;
    mpr_begin(A1.pos, center(w, B), st, v0, dir);
    int res = 0;
    while (res == 0) {
      const CV3 sp = msupport_box(A1, h, w, HV, B, dir);
      res = mpr_advance(w.mpr_tol, sp, st, v0, v1, v2, v3_, dir);
    }
    return res > 0;
  };
  return octree_range_any(w, go, blo, bhi, leaf_hit);
}

// fcl OcTreeSolver::OcTreeIntersectRecurse [ext FCL 0.7.0] without contacts
// or costs, reduced to its result: some occupied leaf of tree 1 (the pair's
// o1) whose OBB overlaps some occupied leaf's OBB of tree 2 -- no box test
// (oracle octree_octree_intersect).  The wave takes tree 1's leaves 64 at a
// time, one per lane; a lane lists tree 2's leaves in the grid cells under
// the box obbDisjoint's tree-2 axis tests leave open (centre R2^T (c1 - p2),
// half extents sum_i (|R_ik| + 1e-6) a_i, padded far above rounding) and
// runs obbDisjoint(R1^T R2, R1^T (c2 - c1), a1, a2) on each.  Wave-uniform
// inputs.
__device__ bool octree_octree_wave(const DevWorld& w, int g1, const SE3& T1, int g2, const SE3& T2) {
  const cptr<double> r1 = w.geom_rec + G_STRIDE * g1;
  const long long l0 = (long long)r1[G_PARAM], l1 = l0 + (long long)r1[G_PARAM + 1];
  double R[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) R[3 * i + j] = (T1.R[i] * T2.R[j] + T1.R[3 + i] * T2.R[3 + j]) + T1.R[6 + i] * T2.R[6 + j];
  const cptr<double> og = w.oct_grid + OG_STRIDE * g2;
  const double inv = og[OG_INV];
  const int dims[3] = {(int)og[OG_DIMS], (int)og[OG_DIMS + 1], (int)og[OG_DIMS + 2]};
  const int cell0 = (int)og[OG_CELL0];
  for (long long base = l0; base < l1; base += 64) {
    const long long la = base + (long long)lane_id();
    bool hit = false;
    if (la < l1) {
      const cptr<double> L = w.oct_leaf + 6 * (size_t)la;
      double a[3], cw[3];
      {
        double c[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          c[k] = (L[k] + L[3 + k]) * 0.5;
          a[k] = (L[3 + k] - L[k]) * 0.5;
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) cw[i] = ((T1.R[3 * i] * c[0] + T1.R[3 * i + 1] * c[1]) + T1.R[3 * i + 2] * c[2]) + T1.p[i];
      }
      const double dq[3] = {cw[0] - T2.p[0], cw[1] - T2.p[1], cw[2] - T2.p[2]};
      double blo[3], bhi[3];
      int c0[3], c1[3];
      bool empty = false;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double q = (T2.R[k] * dq[0] + T2.R[3 + k] * dq[1]) + T2.R[6 + k] * dq[2];
        const double h = ((std::fabs(R[k]) + 1e-6) * a[0] + (std::fabs(R[3 + k]) + 1e-6) * a[1] +
                          (std::fabs(R[6 + k]) + 1e-6) * a[2]) * (1.0 + 1e-9) + 1e-9 * (1.0 + std::fabs(q));
        blo[k] = q - h;
        bhi[k] = q + h;
        const double f0 = std::floor((blo[k] - og[OG_ORIGIN + k]) * inv);
        const double f1 = std::floor((bhi[k] - og[OG_ORIGIN + k]) * inv);
        empty |= f1 < 0.0 || f0 >= (double)dims[k];
        c0[k] = f0 < 0.0 ? 0 : (int)fmin(f0, (double)(dims[k] - 1));
        c1[k] = f1 >= (double)dims[k] ? dims[k] - 1 : (f1 < 0.0 ? 0 : (int)f1);
      }
      for (int x = c0[0]; !empty && !hit && x <= c1[0]; ++x)
        for (int y = c0[1]; !hit && y <= c1[1]; ++y)
          for (int z = c0[2]; !hit && z <= c1[2]; ++z) {
            const int cell = cell0 + (x * dims[1] + y) * dims[2] + z;
            for (int k = w.oct_cells[cell], ke = w.oct_cells[cell + 1]; k < ke && !hit; ++k) {
              const cptr<double> K = w.oct_leaf + 6 * (size_t)w.oct_list[k];
              bool out = false;
#pragma unroll
              for (int i = 0; i < 3; ++i) out |= K[i] > bhi[i] || K[3 + i] < blo[i];
              if (out) continue;
              double b[3], d[3], t[3], T[3];
#pragma unroll
              for (int i = 0; i < 3; ++i) {
                d[i] = (K[i] + K[3 + i]) * 0.5;
                b[i] = (K[3 + i] - K[i]) * 0.5;
              }
#pragma unroll
              for (int i = 0; i < 3; ++i)
                t[i] = (((T2.R[3 * i] * d[0] + T2.R[3 * i + 1] * d[1]) + T2.R[3 * i + 2] * d[2]) + T2.p[i]) - cw[i];
#pragma unroll
              for (int i = 0; i < 3; ++i) T[i] = (T1.R[i] * t[0] + T1.R[3 + i] * t[1]) + T1.R[6 + i] * t[2];
              hit = !obb_disjoint(R, T, a, b);
            }
          }
    }
    if (__ballot(hit) != 0) return true;
  }
  return false;
}

// ---------------------------------------------------------------------------
// BVH meshes (fcl::BVHModel<OBBRSS>, load_mesh_as_BVH src/urdf_utils.cpp:
// 136-155).  fcl::collide's BVH traversal only prunes triangle (pairs) whose
// bounding volumes are disjoint, so the boolean answer is "some leaf test
// succeeds"; the wave walks one candidate's triangles at a time (64 lanes
// side by side) behind a conservative AABB test in the mesh frame (widened
// by 1e-9, far above rounding: a pruned triangle is genuinely separated).  Leaf tests as FCL 0.7.0 runs them:
//   mesh-mesh   Intersect::intersect_Triangle(p, q, R, T), R = R1^T R2,
//               T = R1^T (t2 - t1), q' = R q + T
//   shape-mesh  shapeTriangleIntersect(shape, tf, P1, P2, P3, tf_mesh): shape
//               first; sphereTriangleIntersect for spheres, else libccd MPR
//               on the triangle GJK object (triCreateGJKObject)
// Same operation order as the oracle (oracle/collide_oracle.c).
// ---------------------------------------------------------------------------
constexpr double kMeshPad = 1e-9;
// shape-triangle pairs run libccd MPR: a triangle it can report as touching
// lies within kCcdFalseHitReach of the shape (mpg_math.h)
constexpr double kMeshShapePad = kCcdFalseHitReach * (1.0 + 1e-3) + 1e-5;

__device__ __forceinline__ double d3(const double* a, const double* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
__device__ __forceinline__ void c3(double* o, const double* a, const double* b) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// Intersect::project6
__device__ __forceinline__ bool project6(const double* ax, const double* p2, const double* p3, const double* q1,
                                         const double* q2, const double* q3) {
  const double P1 = (ax[0] * 0.0 + ax[1] * 0.0) + ax[2] * 0.0;  // p1 = 0
  const double P2 = d3(ax, p2), P3 = d3(ax, p3), Q1 = d3(ax, q1), Q2 = d3(ax, q2), Q3 = d3(ax, q3);
  const double mx1 = fmax(P1, fmax(P2, P3)), mn1 = fmin(P1, fmin(P2, P3));
  const double mx2 = fmax(Q1, fmax(Q2, Q3)), mn2 = fmin(Q1, fmin(Q2, Q3));
  return !(mn1 > mx2) && !(mn2 > mx1);
}

// Intersect::intersect_Triangle without contact output: n1, m1, the nine
// edge cross products, g1..g3, h1..h3
__device__ __forceinline__ bool tri_tri_intersect(const double* P, const double* Q) {
  double p2[3], p3[3], q1[3], q2[3], q3[3], e[3][3], f[3][3], n1[3], m1[3], ax[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    p2[k] = P[3 + k] - P[k];
    p3[k] = P[6 + k] - P[k];
    q1[k] = Q[k] - P[k];
    q2[k] = Q[3 + k] - P[k];
    q3[k] = Q[6 + k] - P[k];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    e[0][k] = p2[k] - 0.0;
    e[1][k] = p3[k] - p2[k];
    e[2][k] = 0.0 - p3[k];
    f[0][k] = q2[k] - q1[k];
    f[1][k] = q3[k] - q2[k];
    f[2][k] = q1[k] - q3[k];
  }
  c3(n1, e[0], e[1]);
  c3(m1, f[0], f[1]);
  if (!project6(n1, p2, p3, q1, q2, q3)) return false;
  if (!project6(m1, p2, p3, q1, q2, q3)) return false;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      c3(ax, e[i], f[j]);
      if (!project6(ax, p2, p3, q1, q2, q3)) return false;
    }
  for (int i = 0; i < 3; ++i) {
    c3(ax, e[i], n1);
    if (!project6(ax, p2, p3, q1, q2, q3)) return false;
  }
  for (int i = 0; i < 3; ++i) {
    c3(ax, f[i], m1);
    if (!project6(ax, p2, p3, q1, q2, q3)) return false;
  }
  return true;
}

// segmentSqrDistance (sphere_triangle-inl.h)
__device__ __forceinline__ double segment_sqr_distance(const double* from, const double* to, const double* p) {
  double diff[3], v[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    diff[k] = p[k] - from[k];
    v[k] = to[k] - from[k];
  }
  double t = d3(v, diff);
  if (t > 0) {
    const double vv = d3(v, v);
    if (t < vv) {
      t /= vv;
#pragma unroll
      for (int k = 0; k < 3; ++k) diff[k] -= v[k] * t;
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) diff[k] -= v[k];
    }
  }
  return d3(diff, diff);
}

// sphereTriangleIntersect (sphere_triangle-inl.h), boolean part; W = world
// triangle (tf_mesh * P), c = sphere centre
__device__ __forceinline__ bool sphere_triangle_intersect(double radius, const double* c, const double* W) {
  double a[3], b[3], n[3], pc[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    a[k] = W[3 + k] - W[k];
    b[k] = W[6 + k] - W[k];
  }
  c3(n, a, b);
  const double z = d3(n, n);
  if (z > 0) {
    const double s = std::sqrt(z);
    n[0] /= s;
    n[1] /= s;
    n[2] /= s;
  }
  const double rt = radius + DBL_EPSILON;
#pragma unroll
  for (int k = 0; k < 3; ++k) pc[k] = c[k] - W[k];
  double dist = d3(pc, n);
  if (dist < 0) {
    dist *= -1;
    n[0] *= -1;
    n[1] *= -1;
    n[2] *= -1;
  }
  if (!(dist < rt)) return false;
  {  // projectInTriangle
    double e1[3], e2[3], e3[3], u[3], v[3], x[3], en[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      e1[k] = W[3 + k] - W[k];
      e2[k] = W[6 + k] - W[3 + k];
      e3[k] = W[k] - W[6 + k];
      u[k] = c[k] - W[k];
      v[k] = c[k] - W[3 + k];
      x[k] = c[k] - W[6 + k];
    }
    c3(en, e1, n);
    const double r1 = d3(en, u);
    c3(en, e2, n);
    const double r2 = d3(en, v);
    c3(en, e3, n);
    const double r3 = d3(en, x);
    if ((r1 > 0 && r2 > 0 && r3 > 0) || (r1 <= 0 && r2 <= 0 && r3 <= 0)) return true;
  }
  const double r2 = rt * rt;
  if (segment_sqr_distance(W, W + 3, c) < r2) return true;
  if (segment_sqr_distance(W + 3, W + 6, c) < r2) return true;
  if (segment_sqr_distance(W + 6, W, c) < r2) return true;
  return false;
}

// libccd support of (uniform shape a) - (per-lane triangle b: vertices P in
// the mesh frame, centroid tc): supportTriangle picks argmax dir . (p - c)
__device__ __forceinline__ CV3 msupport_tri(const DevWorld& w, cptr<double> HV, const GObj& a, const GObj& b,
                                            const CV3* P, const CV3& tc, const CV3& dir) {
  const CV3 da = quat_rot(dir, a.rot_inv), db = quat_rot(vscale(dir, ccd_real(-1)), b.rot_inv);
  const int ga = __builtin_amdgcn_readfirstlane(a.geom), ta = __builtin_amdgcn_readfirstlane(a.type);
  const CV3 la = support_local(w, HV, ga, ta, da);
  ccd_real maxdot = -FLT_MAX;
  CV3 lb = P[0];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const CV3 pc = vsub(P[i], tc);
    const ccd_real dot = vdot(db, pc);
    if (dot > maxdot) {
      lb = P[i];
      maxdot = dot;
    }
  }
  return vsub(vadd(quat_rot(la, a.rot), a.pos), vadd(quat_rot(lb, b.rot), b.pos));
}

// One (config, pair) at a time per wave, the 64 lanes split the triangle
// loops.  Inputs are wave-uniform (broadcast from the lane that owns the
// candidate).
__device__ __forceinline__ double bcast(double v, int k) {
  const unsigned long long u = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, k), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), k);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ SE3 bcast_se3(const SE3& T, int k) {
  SE3 o;
#pragma unroll
  for (int i = 0; i < 9; ++i) o.R[i] = bcast(T.R[i], k);
#pragma unroll
  for (int i = 0; i < 3; ++i) o.p[i] = bcast(T.p[i], k);
  return o;
}

// ---------------------------------------------------------------------------
// FCL's BVH traversal gates.  fcl::collide on a BVHModel<OBBRSS> runs a leaf
// test only when every bounding-volume test on its way down the tree passed
// (collisionRecurse; BVTesting = !overlap(R0, T0, bv1, bv2), OBB-inl.h).  The
// device finds the intersecting triangles (pairs) with its own pruning (which
// only drops triangles that cannot hit); fcl_gate_* then replays the OBB tests
// of FCL's path to that leaf (pair), so a hit counts only where FCL would have
// reached it.  Oracle: the traversal itself (oracle/collide_oracle.c
// bvh_shape_walk / bvh_mesh_walk).
// ---------------------------------------------------------------------------
// overlap(R0, T0, a, b): R = a.axis^T (R0 b.axis), T = (R0 b.To + T0 - a.To)^T a.axis
__device__ __forceinline__ bool fcl_overlap(const double* R0, const double* T0, const double* aA, const double* aT,
                                            const double* aE, cptr<double> b) {
  double R0b[9], R[9], Tt[3], T[3], bE[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      R0b[3 * i + j] = (R0[3 * i] * b[FB_AXIS + j] + R0[3 * i + 1] * b[FB_AXIS + 3 + j]) + R0[3 * i + 2] * b[FB_AXIS + 6 + j];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) R[3 * i + j] = (aA[i] * R0b[j] + aA[3 + i] * R0b[3 + j]) + aA[6 + i] * R0b[6 + j];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    Tt[i] = (((R0[3 * i] * b[FB_TO] + R0[3 * i + 1] * b[FB_TO + 1]) + R0[3 * i + 2] * b[FB_TO + 2]) + T0[i]) - aT[i];
#pragma unroll
  for (int j = 0; j < 3; ++j) T[j] = (Tt[0] * aA[j] + Tt[1] * aA[3 + j]) + Tt[2] * aA[6 + j];
#pragma unroll
  for (int k = 0; k < 3; ++k) bE[k] = b[FB_EXT + k];
  return !obb_disjoint(R, T, aE, bE);
}

// the shape's OBB in the world (computeBV<OBB>(shape, tf): convex / box /
// capsule / cylinder axis = R axis_local, sphere axis I; To = R To_local + T)
__device__ __forceinline__ void fcl_shape_obb_world(const DevWorld& w, int gs, int ts, const SE3& TS, double* A,
                                                    double* To, double* E) {
  const cptr<double> o = w.sobb + FB_STRIDE * gs;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      A[3 * i + j] = ts == MPG_GEOM_SPHERE ? o[FB_AXIS + 3 * i + j]
                                           : (TS.R[3 * i] * o[FB_AXIS + j] + TS.R[3 * i + 1] * o[FB_AXIS + 3 + j]) +
                                                 TS.R[3 * i + 2] * o[FB_AXIS + 6 + j];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    To[i] = ((TS.R[3 * i] * o[FB_TO] + TS.R[3 * i + 1] * o[FB_TO + 1]) + TS.R[3 * i + 2] * o[FB_TO + 2]) + TS.p[i];
#pragma unroll
  for (int k = 0; k < 3; ++k) E[k] = o[FB_EXT + k];
}

// MeshShape: the path from the root to triangle t's leaf (t: index in the
// mesh), every node's OBB against the shape's (world) under (TM.R, TM.p).
// mpg_world_create refuses trees deeper than kFclMaxDepth, so every descent
// reaches its leaf inside the loop; the trailing `return true` (the hit
// stands) is only there so that no bound can turn a hit into a miss.
constexpr int kFclMaxDepth = 255;
__device__ __forceinline__ bool fcl_gate_shape(const DevWorld& w, int gm, const SE3& TM, const double* sA,
                                               const double* sT, const double* sE, int t) {
  const int pos = w.tri_pos[(int)w.geom_rec[G_STRIDE * gm + G_PARAM] + t];
  int node = w.fb_root[gm];
  for (int depth = 0; depth <= kFclMaxDepth; ++depth) {
    if (!fcl_overlap(TM.R, TM.p, sA, sT, sE, w.fb_box + FB_STRIDE * node)) return false;
    const int c = w.fb_link[3 * node];
    if (c < 0) return true;
    node = pos < w.fb_link[3 * c + 1] + w.fb_link[3 * c + 2] ? c : c + 1;
  }
  return true;
}

__device__ __forceinline__ double fcl_obb_size(cptr<double> b) {
  return (b[FB_EXT] * b[FB_EXT] + b[FB_EXT + 1] * b[FB_EXT + 1]) + b[FB_EXT + 2] * b[FB_EXT + 2];
}

// MeshMesh: FCL's descent to the leaf pair (ta in A, tb in B) -- the first
// tree is descended when the second node is a leaf or the first is not and
// is larger (firstOverSecond); key (optional) collects the left / right
// choices, whose lexicographic order is FCL's visit order of leaf pairs
__device__ __forceinline__ bool fcl_gate_mesh(const DevWorld& w, int ga, int gb, const double* R, const double* T,
                                              int ta, int tb, uint64_t* key = nullptr) {
  const int pa = w.tri_pos[(int)w.geom_rec[G_STRIDE * ga + G_PARAM] + ta];
  const int pb = w.tri_pos[(int)w.geom_rec[G_STRIDE * gb + G_PARAM] + tb];
  int a = w.fb_root[ga], b = w.fb_root[gb], nk = 0;
  for (int depth = 0; depth <= 2 * kFclMaxDepth; ++depth) {
    const cptr<double> ba = w.fb_box + FB_STRIDE * a;
    double aA[9], aT[3], aE[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) aA[k] = ba[FB_AXIS + k];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      aT[k] = ba[FB_TO + k];
      aE[k] = ba[FB_EXT + k];
    }
    const cptr<double> bb = w.fb_box + FB_STRIDE * b;
    if (!fcl_overlap(R, T, aA, aT, aE, bb)) return false;
    const int ca = w.fb_link[3 * a], cb = w.fb_link[3 * b];
    if (ca < 0 && cb < 0) return true;
    bool right;
    if (cb < 0 || (ca >= 0 && fcl_obb_size(ba) > fcl_obb_size(bb))) {
      right = !(pa < w.fb_link[3 * ca + 1] + w.fb_link[3 * ca + 2]);
      a = right ? ca + 1 : ca;
    } else {
      right = !(pb < w.fb_link[3 * cb + 1] + w.fb_link[3 * cb + 2]);
      b = right ? cb + 1 : cb;
    }
    if (key && nk < 128) {
      if (right) key[nk >> 6] |= 1ull << (63 - (nk & 63));
      ++nk;
    }
  }
  return true;
}

// MeshOcTree: OcTreeMeshIntersectRecurse's descent to the (occupied leaf l,
// triangle t) pair [ext FCL 0.7.0; oracle octmesh_rec].  Every node pair is
// tested as two world OBBs: the octree node's AABB under TO (To = TO centre,
// axis = R, half sizes) against the mesh node's OBBRSS under TM (To = TM To,
// axis = R axis).  The octree node is split (its child on l's path, oct_path)
// when the mesh node is a leaf or the octree node is not and its AABB size
// (full width squared) exceeds the OBB's (half extents squared); else the mesh
// node (left / right by t's position).  key (optional) collects the octree
// child indices (3 bits) and the mesh choices (1 bit); at the first point two
// descents differ they take the same kind of step, so the lexicographic order
// of keys is the traversal's visit order (children 0..7, left before right).
__device__ __forceinline__ bool fcl_overlap_world(const SE3& TO, const double* lo, const double* hi, const SE3& TM,
                                                  cptr<double> b) {
  double ctr[3], E1[3], To1[3], To2[3], ax2[9], t[3], T[3], R[9], E2[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    ctr[k] = (lo[k] + hi[k]) * 0.5;
    E1[k] = (hi[k] - lo[k]) * 0.5;
    E2[k] = b[FB_EXT + k];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    To1[i] = ((TO.R[3 * i] * ctr[0] + TO.R[3 * i + 1] * ctr[1]) + TO.R[3 * i + 2] * ctr[2]) + TO.p[i];
    To2[i] = ((TM.R[3 * i] * b[FB_TO] + TM.R[3 * i + 1] * b[FB_TO + 1]) + TM.R[3 * i + 2] * b[FB_TO + 2]) + TM.p[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      ax2[3 * i + j] = (TM.R[3 * i] * b[FB_AXIS + j] + TM.R[3 * i + 1] * b[FB_AXIS + 3 + j]) + TM.R[3 * i + 2] * b[FB_AXIS + 6 + j];
#pragma unroll
  for (int k = 0; k < 3; ++k) t[k] = To2[k] - To1[k];
#pragma unroll
  for (int i = 0; i < 3; ++i) T[i] = (TO.R[i] * t[0] + TO.R[3 + i] * t[1]) + TO.R[6 + i] * t[2];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) R[3 * i + j] = (TO.R[i] * ax2[j] + TO.R[3 + i] * ax2[3 + j]) + TO.R[6 + i] * ax2[6 + j];
  return !obb_disjoint(R, T, E1, E2);
}

constexpr int kOctKeyWords = 5;  // 16 octree levels x 3 bits + 2 x kFclMaxDepth mesh bits
__device__ __forceinline__ bool fcl_gate_octree_mesh(const DevWorld& w, int go, const SE3& TO, int gm, const SE3& TM,
                                                     int l, int t, uint64_t* key = nullptr) {
  const double delta = (double)(1 << 16) * w.geom_rec[G_STRIDE * go + G_PARAM + 2] / 2;
  double lo[3] = {-delta, -delta, -delta}, hi[3] = {delta, delta, delta};
  const uint64_t path = w.oct_path[l];
  const int od = w.oct_depth[l];
  const int pos = w.tri_pos[(int)w.geom_rec[G_STRIDE * gm + G_PARAM] + t];
  int lev = 0, node = w.fb_root[gm], nk = 0;
  auto put = [&](unsigned v, int bits) {
    if (!key) return;
    for (int b = bits - 1; b >= 0; --b, ++nk)
      if (((v >> b) & 1u) && nk < 64 * kOctKeyWords) key[nk >> 6] |= 1ull << (63 - (nk & 63));
  };
  for (int step = 0; step <= 16 + kFclMaxDepth; ++step) {
    const cptr<double> bb = w.fb_box + FB_STRIDE * node;
    if (!fcl_overlap_world(TO, lo, hi, TM, bb)) return false;
    const bool oleaf = lev == od;
    const int c = w.fb_link[3 * node];
    if (oleaf && c < 0) return true;
    const double d0 = hi[0] - lo[0], d1 = hi[1] - lo[1], d2 = hi[2] - lo[2];
    if (c < 0 || (!oleaf && ((d0 * d0 + d1 * d1) + d2 * d2) > fcl_obb_size(bb))) {
      const unsigned ci = (unsigned)(path >> (3 * (od - 1 - lev))) & 7u;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double mid = (lo[k] + hi[k]) * 0.5;
        if ((ci >> k) & 1u) lo[k] = mid;
        else hi[k] = mid;
      }
      ++lev;
      put(ci, 3);
    } else {
      const bool right = !(pos < w.fb_link[3 * c + 1] + w.fb_link[3 * c + 2]);
      node = right ? c + 1 : c;
      put(right ? 1u : 0u, 1);
    }
  }
  return true;
}

__device__ __forceinline__ bool mesh_mesh_wave(const DevWorld& w, int ga, const SE3& TA, int gb, const SE3& TB) {
  // lanes take 64 of B's triangles into A's frame; each one that meets A's
  // box is then broadcast, A's cluster boxes are tested one per lane, and
  // the triangles of up to 8 overlapping clusters are tested at once (8
  // lanes per cluster)
  const uint32_t lane = lane_id();
  const cptr<double> gra = w.geom_rec + G_STRIDE * ga, grb = w.geom_rec + G_STRIDE * gb;
  const int b0 = (int)grb[G_PARAM], b1 = b0 + (int)grb[G_PARAM + 1];
  const int c0 = w.mesh_tree[2 * ga], c1 = c0 + w.mesh_tree[2 * ga + 1];
  double R[9], T[3], alo[3], ahi[3];
  const double dt[3] = {TB.p[0] - TA.p[0], TB.p[1] - TA.p[1], TB.p[2] - TA.p[2]};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) R[3 * i + j] = (TA.R[i] * TB.R[j] + TA.R[3 + i] * TB.R[3 + j]) + TA.R[6 + i] * TB.R[6 + j];
    T[i] = (TA.R[i] * dt[0] + TA.R[3 + i] * dt[1]) + TA.R[6 + i] * dt[2];
    alo[i] = gra[G_OBB_C + i] - gra[G_OBB_E + i];
    ahi[i] = gra[G_OBB_C + i] + gra[G_OBB_E + i];
  }
  for (int j0 = b0; j0 < b1; j0 += 64) {
    const int j = j0 + (int)lane;
    bool keep = j < b1;
    const cptr<double> rq = w.mesh_tri + TR_STRIDE * (size_t)(keep ? j : b0);
    double Q[9], qlo[3], qhi[3];
#pragma unroll
    for (int v = 0; v < 3; ++v)
#pragma unroll
      for (int i = 0; i < 3; ++i)
        Q[3 * v + i] = ((R[3 * i] * rq[3 * v] + R[3 * i + 1] * rq[3 * v + 1]) + R[3 * i + 2] * rq[3 * v + 2]) + T[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      qlo[i] = fmin(Q[i], fmin(Q[3 + i], Q[6 + i])) - kMeshPad;
      qhi[i] = fmax(Q[i], fmax(Q[3 + i], Q[6 + i])) + kMeshPad;
      keep &= !(qlo[i] > ahi[i] || qhi[i] < alo[i]);
    }
    unsigned long long todo = __ballot(keep);
    while (todo) {
      const int k = __builtin_ctzll(todo);
      todo &= todo - 1;
      double Qk[9], lk[3], hk[3];
#pragma unroll
      for (int i = 0; i < 9; ++i) Qk[i] = bcast(Q[i], k);
      const int tbk = (int)bcast(rq[TR_ID], k);  // B's triangle (read while every lane is active)
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        lk[i] = bcast(qlo[i], k);
        hk[i] = bcast(qhi[i], k);
      }
      for (int cb = c0; cb < c1; cb += 64) {
        const int c = cb + (int)lane;
        bool ov = c < c1;
        if (ov) {
          const cptr<double> bx = w.mesh_node + 6 * (size_t)c;
#pragma unroll
          for (int i = 0; i < 3; ++i) ov &= !(bx[i] > hk[i] || bx[3 + i] < lk[i]);
        }
        unsigned long long m = __ballot(ov);
        while (m) {
          int myc = -1;  // cluster of this lane's group of 8
          for (int g = 0; g < 8 && m; ++g) {
            const int cc = __builtin_ctzll(m);
            m &= m - 1;
            if (g == (int)(lane >> 3)) myc = cb + cc;
          }
          bool hit = false;
          if (myc >= 0) {
            const int t1 = w.mesh_link[2 * myc] + w.mesh_link[2 * myc + 1];
            for (int t = w.mesh_link[2 * myc] + (int)(lane & 7); t < t1 && !hit; t += 8) {
              const cptr<double> rp = w.mesh_tri + TR_STRIDE * (size_t)t;
              bool o2 = false;
#pragma unroll
              for (int i = 0; i < 3; ++i) o2 |= rp[TR_LO + i] > hk[i] || rp[TR_HI + i] < lk[i];
              if (o2) continue;
              double P[9];
#pragma unroll
              for (int q = 0; q < 9; ++q) P[q] = rp[TR_P + q];
              hit = tri_tri_intersect(P, Qk) && fcl_gate_mesh(w, ga, gb, R, T, (int)rp[TR_ID], tbk);
            }
          }
          if (__ballot(hit) != 0) return true;
        }
      }
    }
  }
  return false;
}

__device__ __forceinline__ bool mesh_shape_wave(const DevWorld& w, cptr<double> HV, int gm, const SE3& TM, int gs,
                                             const SE3& TS) {
  const uint32_t lane = lane_id();
  const cptr<double> grm = w.geom_rec + G_STRIDE * gm, grs = w.geom_rec + G_STRIDE * gs;
  const int ts = w.geom_type[gs];
  const int t0 = (int)grm[G_PARAM], t1 = t0 + (int)grm[G_PARAM + 1];
  double sc[3], cl[3], Rl[9], hq[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    sc[i] = ((TS.R[3 * i] * grs[G_OBB_C] + TS.R[3 * i + 1] * grs[G_OBB_C + 1]) + TS.R[3 * i + 2] * grs[G_OBB_C + 2]) + TS.p[i];
  const double dsc[3] = {sc[0] - TM.p[0], sc[1] - TM.p[1], sc[2] - TM.p[2]};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    cl[i] = (TM.R[i] * dsc[0] + TM.R[3 + i] * dsc[1]) + TM.R[6 + i] * dsc[2];
#pragma unroll
    for (int j = 0; j < 3; ++j) Rl[3 * i + j] = (TM.R[i] * TS.R[j] + TM.R[3 + i] * TS.R[3 + j]) + TM.R[6 + i] * TS.R[6 + j];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
    hq[i] = ((std::fabs(Rl[3 * i]) * grs[G_OBB_E] + std::fabs(Rl[3 * i + 1]) * grs[G_OBB_E + 1]) +
             std::fabs(Rl[3 * i + 2]) * grs[G_OBB_E + 2]) * (1.0 + 1e-9) +
            kMeshShapePad * (1.0 + std::fabs(TS.p[0]) + std::fabs(TS.p[1]) + std::fabs(TS.p[2]) + std::fabs(TM.p[0]) +
                             std::fabs(TM.p[1]) + std::fabs(TM.p[2]));
  GObj A, B;
  A.rot = gjk_rot_from_matrix(TS.R);
  A.rot_inv = quat_invert2(A.rot);
  A.pos = cv3(TS.p[0], TS.p[1], TS.p[2]);
  A.geom = gs;
  A.type = ts;
  B.rot = gjk_rot_from_matrix(TM.R);
  B.rot_inv = quat_invert2(B.rot);
  B.pos = cv3(TM.p[0], TM.p[1], TM.p[2]);
  B.geom = gm;
  B.type = MPG_GEOM_MESH;
  const CV3 ca = center(w, A);
  double sA[9], sT[3], sE[3];  // FCL's OBB of the shape (the traversal's BV tests)
  fcl_shape_obb_world(w, gs, ts, TS, sA, sT, sE);
  for (int b = t0; b < t1; b += 64) {
    const int t = b + (int)lane;
    bool cand = t < t1;
    const cptr<double> rec = w.mesh_tri + TR_STRIDE * (size_t)(cand ? t : t0);
#pragma unroll
    for (int i = 0; i < 3; ++i) cand &= !(rec[TR_LO + i] > cl[i] + hq[i] || rec[TR_HI + i] < cl[i] - hq[i]);
    if (__ballot(cand) == 0) continue;
    bool hit = false;
    if (cand) {
      double P[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) P[k] = rec[TR_P + k];
      if (ts == MPG_GEOM_SPHERE) {
        double W[9];
#pragma unroll
        for (int v = 0; v < 3; ++v)
#pragma unroll
          for (int i = 0; i < 3; ++i)
            W[3 * v + i] = ((TM.R[3 * i] * P[3 * v] + TM.R[3 * i + 1] * P[3 * v + 1]) + TM.R[3 * i + 2] * P[3 * v + 2]) + TM.p[i];
        hit = sphere_triangle_intersect(grs[G_PARAM], TS.p, W);
      } else {
        // triCreateGJKObject: centre in fp64, then vertices and centre as ccd_real
        const CV3 tc = cv3((P[0] + P[3] + P[6]) / 3, (P[1] + P[4] + P[7]) / 3, (P[2] + P[5] + P[8]) / 3);
        const CV3 TP[3] = {cv3(P[0], P[1], P[2]), cv3(P[3], P[4], P[5]), cv3(P[6], P[7], P[8])};
        int st;
        CV3 v0, v1, v2, v3_, dir;
        mpr_begin(ca, vadd(quat_rot(tc, B.rot), B.pos), st, v0, dir);
        int res = 0;
        while (res == 0) {
          const CV3 sp = msupport_tri(w, HV, A, B, TP, tc, dir);
          res = mpr_advance(w.mpr_tol, sp, st, v0, v1, v2, v3_, dir);
        }
        hit = res > 0;
      }
      hit = hit && fcl_gate_shape(w, gm, TM, sA, sT, sE, (int)rec[TR_ID]);
    }
    if (__ballot(hit) != 0) return true;
  }
  return false;
}

// libccd support of (box, per-lane half sizes h) - (triangle, per-lane: its
// vertices P and centroid tc in the mesh frame, rotation/position of b)
__device__ __forceinline__ CV3 msupport_box_tri(const GObj& a, const ccd_real* h, const GObj& b, const CV3* P,
                                                const CV3& tc, const CV3& dir) {
  const CV3 da = quat_rot(dir, a.rot_inv), db = quat_rot(vscale(dir, ccd_real(-1)), b.rot_inv);
  const CV3 la = CV3{(da.x >= 0 ? ccd_real(1) : ccd_real(-1)) * h[0], (da.y >= 0 ? ccd_real(1) : ccd_real(-1)) * h[1],
                     (da.z >= 0 ? ccd_real(1) : ccd_real(-1)) * h[2]};
  ccd_real maxdot = -FLT_MAX;
  CV3 lb = P[0];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const ccd_real dot = vdot(db, vsub(P[i], tc));
    if (dot > maxdot) {
      lb = P[i];
      maxdot = dot;
    }
  }
  return vsub(vadd(quat_rot(la, a.rot), a.pos), vadd(quat_rot(lb, b.rot), b.pos));
}

// fcl::collide(mesh, OcTree) in either order [ext FCL 0.7.0 OcTreeSolver::
// OcTreeMeshIntersectRecurse; MeshOcTreeIntersect passes the tree first]:
// some (occupied leaf, triangle) whose shapeTriangleIntersect(Box(leaf),
// box_tf, P1, P2, P3, tf_mesh) -- libccd MPR, leaf box first, triangle GJK
// object second -- reports a hit (oracle mesh_octree_intersect).  The
// traversal's BV tests only prune genuinely separated pairs, so every pair
// within libccd's false-hit reach is run.  Leaves: the octree grid cells under
// the mesh's box (octree frame, padded), one leaf per lane; each lane walks
// the mesh's cluster boxes and triangle boxes against its leaf's box in the
// mesh frame (padded) and runs MPR on the survivors.  Wave-uniform inputs.
__device__ __forceinline__ bool mesh_octree_wave(const DevWorld& w, int gm, const SE3& TM, int go, const SE3& TO) {
  const cptr<double> grm = w.geom_rec + G_STRIDE * gm;
  const double pad = kMeshShapePad * (1.0 + std::fabs(TO.p[0]) + std::fabs(TO.p[1]) + std::fabs(TO.p[2]) +
                                      std::fabs(TM.p[0]) + std::fabs(TM.p[1]) + std::fabs(TM.p[2]));
  double Rm[9], Ro[9];  // Rm = TO.R^T TM.R (mesh axes in the octree frame), Ro = Rm^T
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      Rm[3 * i + j] = (TO.R[i] * TM.R[j] + TO.R[3 + i] * TM.R[3 + j]) + TO.R[6 + i] * TM.R[6 + j];
      Ro[3 * j + i] = Rm[3 * i + j];
    }
  // the mesh's local box (G_OBB) in the octree frame, padded
  double mcw[3], blo[3], bhi[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    mcw[i] = ((TM.R[3 * i] * grm[G_OBB_C] + TM.R[3 * i + 1] * grm[G_OBB_C + 1]) + TM.R[3 * i + 2] * grm[G_OBB_C + 2]) +
             TM.p[i];
  const double dmo[3] = {mcw[0] - TO.p[0], mcw[1] - TO.p[1], mcw[2] - TO.p[2]};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double c = (TO.R[i] * dmo[0] + TO.R[3 + i] * dmo[1]) + TO.R[6 + i] * dmo[2];
    const double e = ((std::fabs(Rm[3 * i]) * grm[G_OBB_E] + std::fabs(Rm[3 * i + 1]) * grm[G_OBB_E + 1]) +
                      std::fabs(Rm[3 * i + 2]) * grm[G_OBB_E + 2]) * (1.0 + 1e-9) + 1e-9 + pad;
    blo[i] = c - e;
    bhi[i] = c + e;
  }
  GObj A, B;  // A: the leaf box (octree rotation, per-leaf centre), B: the mesh frame of the triangles
  A.rot = gjk_rot_from_matrix(TO.R);
  A.rot_inv = quat_invert2(A.rot);
  A.geom = go;
  A.type = MPG_GEOM_BOX;
  B.rot = gjk_rot_from_matrix(TM.R);
  B.rot_inv = quat_invert2(B.rot);
  B.pos = cv3(TM.p[0], TM.p[1], TM.p[2]);
  B.geom = gm;
  B.type = MPG_GEOM_MESH;
  const int c0 = w.mesh_tree[2 * gm], c1 = c0 + w.mesh_tree[2 * gm + 1];
  auto leaf_hit = [&](int leaf) -> bool {
    const cptr<double> L = w.oct_leaf + 6 * (size_t)leaf;
    bool out = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) out |= L[i] > bhi[i] || L[3 + i] < blo[i];
    if (out) return false;
    double c[3], side[3], cw[3], cm[3], hm[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      c[i] = (L[i] + L[3 + i]) * 0.5;
      side[i] = L[3 + i] - L[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) cw[i] = ((TO.R[3 * i] * c[0] + TO.R[3 * i + 1] * c[1]) + TO.R[3 * i + 2] * c[2]) + TO.p[i];
    const double dm[3] = {cw[0] - TM.p[0], cw[1] - TM.p[1], cw[2] - TM.p[2]};
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // the leaf box in the mesh frame: centre, padded half extents
      cm[i] = (TM.R[i] * dm[0] + TM.R[3 + i] * dm[1]) + TM.R[6 + i] * dm[2];
      hm[i] = ((std::fabs(Ro[3 * i]) * side[0] + std::fabs(Ro[3 * i + 1]) * side[1]) + std::fabs(Ro[3 * i + 2]) * side[2]) *
                  0.5 * (1.0 + 1e-9) + 1e-9 + pad;
    }
    GObj A1 = A;
    A1.pos = cv3(cw[0], cw[1], cw[2]);
    const ccd_real h[3] = {(ccd_real)(side[0] / 2.0), (ccd_real)(side[1] / 2.0), (ccd_real)(side[2] / 2.0)};  // boxToGJK
    for (int cl = c0; cl < c1; ++cl) {
      const cptr<double> bx = w.mesh_node + 6 * (size_t)cl;
      bool away = false;
#pragma unroll
      for (int i = 0; i < 3; ++i) away |= bx[i] > cm[i] + hm[i] || bx[3 + i] < cm[i] - hm[i];
      if (away) continue;
      const int t1 = w.mesh_link[2 * cl] + w.mesh_link[2 * cl + 1];
      for (int t = w.mesh_link[2 * cl]; t < t1; ++t) {
        const cptr<double> rec = w.mesh_tri + TR_STRIDE * (size_t)t;
        bool o2 = false;
#pragma unroll
        for (int i = 0; i < 3; ++i) o2 |= rec[TR_LO + i] > cm[i] + hm[i] || rec[TR_HI + i] < cm[i] - hm[i];
        if (o2) continue;
        double P[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) P[k] = rec[TR_P + k];
        // triCreateGJKObject: centre in fp64, then vertices and centre as ccd_real
        const CV3 tc = cv3((P[0] + P[3] + P[6]) / 3, (P[1] + P[4] + P[7]) / 3, (P[2] + P[5] + P[8]) / 3);
        const CV3 TP[3] = {cv3(P[0], P[1], P[2]), cv3(P[3], P[4], P[5]), cv3(P[6], P[7], P[8])};
        int st;
        CV3 v0, v1, v2, v3_, dir;
        mpr_begin(A1.pos, vadd(quat_rot(tc, B.rot), B.pos), st, v0, dir);
        int res = 0;
        while (res == 0) {
          const CV3 sp = msupport_box_tri(A1, h, B, TP, tc, dir);
          res = mpr_advance(w.mpr_tol, sp, st, v0, v1, v2, v3_, dir);
        }
        if (res > 0 && fcl_gate_octree_mesh(w, go, TO, gm, TM, leaf, (int)rec[TR_ID])) return true;
      }
    }
    return false;
  };
  return octree_range_any(w, go, blo, bhi, leaf_hit);
}

// every active lane's (TA, TB) candidate of the (wave-uniform) mesh or
// octree pair (ga, gb), one after the other with the whole wave; bit k =
// lane k's hit
template <int CLS>
__device__ __forceinline__ unsigned long long walk_wave_eval(const DevWorld& w, cptr<double> HV, int ga, const SE3& TA,
                                                            int gb, const SE3& TB, bool active) {
  const int tga = w.geom_type[ga], tgb = w.geom_type[gb];
  if constexpr (CLS == CLS_OCTREE) {
    unsigned long long todo = __ballot(active), hits = 0;
    while (todo) {
      const int k = __builtin_ctzll(todo);
      todo &= todo - 1;
      const SE3 A = bcast_se3(TA, k), B = bcast_se3(TB, k);
      const bool h = tga == MPG_GEOM_OCTREE && tgb == MPG_GEOM_OCTREE ? octree_octree_wave(w, ga, A, gb, B)
                     : tga == MPG_GEOM_OCTREE                         ? octree_wave(w, HV, ga, A, gb, B)
                                                                      : octree_wave(w, HV, gb, B, ga, A);
      if (h) hits |= 1ull << k;
    }
    return hits;
  } else {
    const bool am = tga == MPG_GEOM_MESH, bm = tgb == MPG_GEOM_MESH;
    unsigned long long todo = __ballot(active), hits = 0;
    while (todo) {
      const int k = __builtin_ctzll(todo);
      todo &= todo - 1;
      const SE3 A = bcast_se3(TA, k), B = bcast_se3(TB, k);
      if (w.dbg(am && bm ? 5 : 6)) continue;
      bool h;
      if (am && bm) h = mesh_mesh_wave(w, ga, A, gb, B);
      else if (tgb == MPG_GEOM_OCTREE) h = mesh_octree_wave(w, ga, A, gb, B);
      else if (tga == MPG_GEOM_OCTREE) h = mesh_octree_wave(w, gb, B, ga, A);
      else if (am) h = mesh_shape_wave(w, HV, ga, A, gb, B);
      else h = mesh_shape_wave(w, HV, gb, B, ga, A);
      if (h) hits |= 1ull << k;
    }
    return hits;
  }
}



// Refill idle lanes once at least this many are idle.  A refill hands out
// candidates whose GJK objects and MPR start were staged in LDS beforehand
// (all 64 lanes compute the chain FK of the next 64 candidates at once), so
// it costs a few LDS reads and can run every few steps.
#ifndef MPG_REFILL_MIN
#define MPG_REFILL_MIN 8
#endif
// take the next task early once the current one is handed out and this many
// lanes are idle: a task of the same pair continues without a drain
#ifndef MPG_STEAL_MIN
#define MPG_STEAL_MIN 64
#endif

// staged candidate of the narrow phase: per moving object its GJK rotation,
// inverse rotation and position (11 floats), then the MPR start v0 and dir
enum { STG_A = 0, STG_B = 11, STG_V0 = 22, STG_DIR = 25, STG_N = 28 };

__device__ __forceinline__ void stage_obj(float (*stg)[64], int c0, uint32_t slot, const GObj& o) {
  stg[c0 + 0][slot] = o.rot.x;
  stg[c0 + 1][slot] = o.rot.y;
  stg[c0 + 2][slot] = o.rot.z;
  stg[c0 + 3][slot] = o.rot.w;
  stg[c0 + 4][slot] = o.rot_inv.x;
  stg[c0 + 5][slot] = o.rot_inv.y;
  stg[c0 + 6][slot] = o.rot_inv.z;
  stg[c0 + 7][slot] = o.rot_inv.w;
  stg[c0 + 8][slot] = o.pos.x;
  stg[c0 + 9][slot] = o.pos.y;
  stg[c0 + 10][slot] = o.pos.z;
}

__device__ __forceinline__ void unstage_obj(float (*stg)[64], int c0, uint32_t slot, GObj& o) {
  o.rot = CQ4{stg[c0 + 0][slot], stg[c0 + 1][slot], stg[c0 + 2][slot], stg[c0 + 3][slot]};
  o.rot_inv = CQ4{stg[c0 + 4][slot], stg[c0 + 5][slot], stg[c0 + 6][slot], stg[c0 + 7][slot]};
  o.pos = CV3{stg[c0 + 8][slot], stg[c0 + 9][slot], stg[c0 + 10][slot]};
}

template <bool FROM_POSES>
// 3 waves per SIMD: the kernel sits at the 168-VGPR edge of that occupancy
// (a few registers more, e.g. an inlined rare path, would drop it to 2 and
// cost ~40 % of its throughput)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void narrow_kernel(DevWorld w, const double* __restrict__ in,
                                                    const uint32_t* __restrict__ seg_len,
                                                    const uint32_t* __restrict__ seg_start,
                                                    const uint32_t* __restrict__ prefix,
                                                    const uint32_t* __restrict__ cand,
                                                    uint8_t* __restrict__ flags, uint32_t* __restrict__ masks,
                                                    uint32_t* __restrict__ task_ctr, const double* __restrict__ sc) {
  // hull reads are wave-uniform: scalar loads through the constant cache
  // (staging the hulls in LDS measured slower: +60 VGPRs, occupancy 4 -> 3)
  const cptr<double> HV = w.hull;
  const uint32_t lane = lane_id();
  const uint32_t total = prefix[w.n_pairs], ts = prefix[w.n_pairs + 2];
  __shared__ float s_stage[4][STG_N][64];
  __shared__ uint32_t s_cfg[4][64];
  float (*stg)[64] = s_stage[threadIdx.x >> 6];
  uint32_t* scfg = s_cfg[threadIdx.x >> 6];
  // dynamic task queue: waves that drew cheap tasks take more.
  // The first task of every wave is its wave index (the counter starts past
  // them): half the atomics on the one counter, which a small batch's waves
  // otherwise all hit at once.  (A relaxed load to skip the atomic once the
  // queue is drained measured 2x slower on cfg3: keep atomics out of the loop.)
  const uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
  auto fetch = [&]() {
    uint32_t t = 0;
    if (lane == 0) t = n_waves + atomicAdd(task_ctr, 1u);
    return (uint32_t)__builtin_amdgcn_readfirstlane(t);
  };
  uint32_t tk = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  while (tk < total) {
    const int p = task_pair(prefix, w.n_pairs, tk);
    if (w.pair_cf[p] != CF_NONE) {  // closed-form pairs: closed_form_kernel
      tk = fetch();
      continue;
    }
    uint32_t next = (tk - prefix[p]) * ts;  // wave-uniform cursor into the pair's candidates
    uint32_t t1 = min(seg_len[p], next + ts);
    uint32_t pend = 0xffffffffu;  // a task of another pair, taken early: runs after this one
    bool more = true;             // the queue may still hold tasks
    const uint32_t* __restrict__ cl = cand + seg_start[p];
    const int a = w.pair_a[p], b = w.pair_b[p];
    const bool am = a < w.n_moving, bm = b < w.n_moving;
    const uint32_t bit = 1u << (p & 31);
    int st = MPR_DONE;
    long long cfg = 0;
    GObj A, B;
    if (!am) A = static_obj(w, a - w.n_moving);
    if (!bm) B = static_obj(w, b - w.n_moving);
    if (am) {
      A.geom = w.moving_geom[a];
      A.type = w.geom_type[A.geom];
    }
    if (bm) {
      B.geom = w.moving_geom[b];
      B.type = w.geom_type[B.geom];
    }
    CV3 v0, v1, v2, v3, dir;
    uint32_t sh = 0, sn = 0;  // staged candidates: [sh, sn) not yet handed out
#ifdef MPG_STATS
    int nsteps = 0;
#endif
    for (;;) {
      const unsigned long long idle = __ballot(st == MPR_DONE);
      const uint32_t n_idle = (uint32_t)__popcll(idle);
      if (next >= t1 && sh == sn && pend == 0xffffffffu && more && n_idle >= MPG_STEAL_MIN) {
        const uint32_t t2 = fetch();
        if (t2 >= total) {
          more = false;
        } else if (task_pair(prefix, w.n_pairs, t2) == p) {  // same pair: continue without draining
          next = (t2 - prefix[p]) * ts;
          t1 = min(seg_len[p], next + ts);
        } else {
          pend = t2;
        }
      }
#ifdef MPG_STATS
      const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#endif
      if ((sh < sn || next < t1) && (n_idle >= MPG_REFILL_MIN || n_idle == 64)) {
        if (sh == sn) {  // stage the next <= 64 candidates: chain FK and MPR start with every lane
          const uint32_t cnt = min(64u, t1 - next);
          if (lane < cnt) {
            const long long c = cl[next + lane];
            GObj sa = A, sb = B;
            if (am) sa = moving_obj<FROM_POSES>(w, in, sc, c, a);
            if (bm) sb = moving_obj<FROM_POSES>(w, in, sc, c, b);
            int s0;
            CV3 w0, d0;
            mpr_begin(center(w, sa), center(w, sb), s0, w0, d0);
            scfg[lane] = (uint32_t)c;
            if (am) stage_obj(stg, STG_A, lane, sa);
            if (bm) stage_obj(stg, STG_B, lane, sb);
            stg[STG_V0][lane] = w0.x;
            stg[STG_V0 + 1][lane] = w0.y;
            stg[STG_V0 + 2][lane] = w0.z;
            stg[STG_DIR][lane] = d0.x;
            stg[STG_DIR + 1][lane] = d0.y;
            stg[STG_DIR + 2][lane] = d0.z;
          }
          wave_lds_sync();
          sh = 0;
          sn = cnt;
          next += cnt;
        }
        if (st == MPR_DONE) {  // hand the staged candidates to the idle lanes
          const uint32_t rank =
              __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
          if (rank < sn - sh) {
            const uint32_t k = sh + rank;
            cfg = scfg[k];
            if (am) unstage_obj(stg, STG_A, k, A);
            if (bm) unstage_obj(stg, STG_B, k, B);
            v0 = CV3{stg[STG_V0][k], stg[STG_V0 + 1][k], stg[STG_V0 + 2][k]};
            dir = CV3{stg[STG_DIR][k], stg[STG_DIR + 1][k], stg[STG_DIR + 2][k]};
            st = MPR_V1;
#ifdef MPG_STATS
            nsteps = 0;
#endif
          }
        }
        sh = min(sn, sh + n_idle);
        wave_lds_sync();  // every read done before the next staging overwrites
      }
#ifdef MPG_STATS
      const unsigned long long c1 = __builtin_amdgcn_s_memtime();
      const unsigned long long n_act = (unsigned long long)__popcll(__ballot(st != MPR_DONE));
      if (w.stats && lane_id() == 0) {
        atomicAdd(&w.stats[3], c1 - c0);
        atomicAdd(&w.stats[6], n_act);
        atomicAdd(&w.stats[7], 1ull);
      }
#endif
      if (__ballot(st != MPR_DONE) == 0) {
        if (next >= t1 && sh == sn && (pend != 0xffffffffu || !more)) break;
        continue;
      }
#ifdef MPG_STATS
      unsigned long long c2 = 0;
#endif
      if (st != MPR_DONE) {
        const CV3 s = msupport(w, HV, A, B, dir);
#ifdef MPG_STATS
        ++nsteps;
        c2 = __builtin_amdgcn_s_memtime();
#endif
        const int res = mpr_advance(w.mpr_tol, s, st, v0, v1, v2, v3, dir);
        if (res != 0) {
          if (res > 0) {
            if (masks) atomicOr(&masks[cfg * w.W + (p >> 5)], bit);
            flags[cfg] = 1;
          }
          st = MPR_DONE;
#ifdef MPG_STATS
          if (w.stats) {
            atomicAdd(&w.stats[res > 0 ? 0 : 1], (unsigned long long)nsteps);
            atomicAdd(&w.stats[res > 0 ? 2 : 8], 1ull);
          }
#endif
        }
      }
#ifdef MPG_STATS
      {
        const unsigned long long c3 = __builtin_amdgcn_s_memtime();
        unsigned long long c2m = c2 ? c2 : ~0ull;  // earliest support end over the active lanes
        for (int off = 32; off > 0; off >>= 1) {
          const unsigned long long o = ((unsigned long long)__shfl_xor((unsigned)(c2m >> 32), off) << 32) |
                                       (unsigned)__shfl_xor((unsigned)c2m, off);
          c2m = o < c2m ? o : c2m;
        }
        if (w.stats && lane_id() == 0 && c2m != ~0ull) {
          atomicAdd(&w.stats[4], c2m - c1);
          atomicAdd(&w.stats[5], c3 - c2m);
        }
      }
#endif
    }
    tk = pend != 0xffffffffu ? pend : (more ? fetch() : total);
  }
}

// ---------------------------------------------------------------------------
// Latency path for small batches (the planner's regime: a few to a few
// thousand states per call, one round trip each).  The two-phase pipeline
// costs six dependent launches and a lane-serial cull whose critical path
// alone is ~60 us; here ONE launch covers the batch with parallelism over
// (pair x configuration): one wave per (pair, 64-configuration tile), the
// pair wave-uniform as the MPR support scans need.  Per lane: exact fp64 FK of
// the pair's two objects (sincos inline), a bounding-sphere separation test
// (margin kSmallMargin >> MPR tolerance + fp64 FK error, so a skipped pair
// cannot intersect), then the FCL closed form or libccd MPR -- the same
// mpr_advance / support code as narrow_kernel, so every bit matches it.
// Output: hit bytes [n_pairs][n], each written exactly once (no
// initialisation, safe in host-mapped memory); the host folds them into
// flags and pair masks.
// ---------------------------------------------------------------------------
constexpr double kSmallMargin = 1e-4;

// the latency path's joint sin/cos: one lane per (configuration, move-group
// dof), shared by every pair's wave of the following small_kernel
__global__ __launch_bounds__(256) void small_sincos_kernel(DevWorld w, const double* __restrict__ in, long long n,
                                                          double* __restrict__ sc) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * w.dof) return;
  const long long r = i / w.dof;
  const int src = (int)(i - r * w.dof);
  for (int j = 0; j < w.nj; ++j) {
    if (w.joint_q_source[j] != src || !joint_is_revolute(w.joint_type[j])) continue;
    double sv, cv;
    mpg_sincos(in[r * w.dof + src], &sv, &cv);
    sc[(r * w.dof + src) * 2] = sv;
    sc[(r * w.dof + src) * 2 + 1] = cv;
    return;
  }
}

// INLINE_SC: each lane computes its configuration's exact joint sin/cos itself
// (one launch per validity batch -- the planner's round trip) into its own LDS
// row, kLatScGroup independent evaluations at a time so that their table loads
// overlap (evaluated inside the chain walk they serialise: two objects' chains
// of up to nine joints, each waiting on its table reads); otherwise they come
// from small_sincos_kernel (larger batches, where the P-fold recomputation
// costs more than the extra launch)
constexpr int kLatScDof = 16;   // move-group dof the inline path holds (host: more -> small_sincos_kernel)
constexpr int kLatScGroup = 4;

// The latency kernel's joint table, staged per wave in LDS by one round of
// parallel loads (lane j: joint j; lanes 0..31 / 32..63: the two objects'
// chains): the chain walk then reads LDS instead of waiting, joint after
// joint, on dependent scalar loads of the chain list and the joint records.
struct LatJoints {
  double place[kMaxJoints][12];
  double axis[kMaxJoints][3];
  double qc[kMaxJoints];
  int type[kMaxJoints], src[kMaxJoints];
  int chain[2][kMaxJoints];
};

__device__ __forceinline__ void stage_lat_joints(const DevWorld& w, LatJoints& J, uint32_t lane, int la, int lb) {
  if ((int)lane < w.nj) {
    const int j = (int)lane;
#pragma unroll
    for (int i = 0; i < 12; ++i) J.place[j][i] = w.joint_place[12 * j + i];
#pragma unroll
    for (int i = 0; i < 3; ++i) J.axis[j][i] = w.joint_axis[3 * j + i];
    J.qc[j] = w.joint_q_const[j];
    J.type[j] = w.joint_type[j];
    J.src[j] = w.joint_q_source[j];
  }
  const int s = lane >> 5, k = (int)(lane & 31u), l = s ? lb : la;
  if (l >= 0 && k < w.link_chain_len[l]) J.chain[s][k] = w.chain_joints[w.link_chain_start[l] + k];
  wave_lds_sync();
}

// chain_oMi on the staged table: the same products in the same order
__device__ __forceinline__ SE3 chain_oMi_lat(const DevWorld& w, const LatJoints& J, int s, int l,
                                             const double* __restrict__ qrow, const double* screw) {
  const int cl = w.link_chain_len[l];
  SE3 T;
  se3_identity(T);
  for (int k = 0; k < cl; ++k) {
    const int j = J.chain[s][k];
    const int src = J.src[j - 1];
    const int type = J.type[j - 1];
    const bool pre = src >= 0 && joint_is_revolute(type);
    const double v = pre ? 0.0 : src >= 0 ? qrow[src] : J.qc[j - 1];
    const SE3 M = joint_motion(type, J.axis[j - 1], v, pre ? screw + 2 * src : nullptr);
    SE3 P;
#pragma unroll
    for (int i = 0; i < 9; ++i) P.R[i] = J.place[j - 1][i];
    P.p[0] = J.place[j - 1][9];
    P.p[1] = J.place[j - 1][10];
    P.p[2] = J.place[j - 1][11];
    const SE3 li = se3_mul(P, M);
    T = k == 0 ? li : se3_mul(T, li);
  }
  return T;
}
// World transform of one side of a latency record (LS_* layout: chain of
// joints, link placement, moving offset; a static side holds its world
// transform at LS_OFF): chain_oMi + link_from_oMi + the moving offset, the
// same products in the same order
__device__ __forceinline__ SE3 rec_side_tf(const double* S, bool moving, const double* qrow, const double* sc_row) {
  if (!moving) return load_se3(S + LS_OFF);
  const int cl = (int)S[LS_CL];
  SE3 T;
  se3_identity(T);
  for (int k = 0; k < cl; ++k) {
    const double* J = S + LS_J + LJ_STRIDE * k;
    const int type = (int)J[0], srcq = (int)J[1];
    const bool pre = srcq >= 0 && joint_is_revolute(type);
    const double qv = pre ? 0.0 : srcq >= 0 ? qrow[srcq] : J[2];
    const SE3 M = joint_motion(type, J + 3, qv, pre ? sc_row + 2 * srcq : nullptr);
    const SE3 li = se3_mul(load_se3(J + 6), M);
    T = k == 0 ? li : se3_mul(T, li);
  }
  const SE3 L = se3_mul(T, load_se3(S + LS_LINKPL));
  double qw, qxyz[3];
  mat_to_quat(L.R, &qw, qxyz);
  SE3 Lr;
  quat_to_mat(qw, qxyz[0], qxyz[1], qxyz[2], Lr.R);
  Lr.p[0] = L.p[0];
  Lr.p[1] = L.p[1];
  Lr.p[2] = L.p[2];
  return se3_mul(Lr, load_se3(S + LS_OFF));
}

// The latency paths' second bounding test (after the spheres): the two
// objects' oriented boxes (local AABBs, world rotation) in fp64, every bound
// widened by `margin` (the latency margin: at least libccd's false-hit reach,
// as the cull's fp32 test), so a separated pair cannot be an MPR hit.  R:
// row-major world rotation (column j = box axis j), c: world centre, e: half
// extents.
__device__ __forceinline__ bool dobb_separated(const double* RA, const double* ca, const double* ea, const double* RB,
                                               const double* cb, const double* eb, double margin) {
  const double d[3] = {cb[0] - ca[0], cb[1] - ca[1], cb[2] - ca[2]};
  double Rm[3][3], Ab[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      Rm[i][j] = RA[i] * RB[j] + RA[3 + i] * RB[3 + j] + RA[6 + i] * RB[6 + j];
      Ab[i][j] = std::fabs(Rm[i][j]) + 1e-12;
    }
  double t[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = d[0] * RA[i] + d[1] * RA[3 + i] + d[2] * RA[6 + i];
  bool sep = false;
#pragma unroll
  for (int i = 0; i < 3; ++i) sep |= std::fabs(t[i]) > ea[i] + (eb[0] * Ab[i][0] + eb[1] * Ab[i][1] + eb[2] * Ab[i][2]) + margin;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double ra = ea[0] * Ab[0][j] + ea[1] * Ab[1][j] + ea[2] * Ab[2][j];
    sep |= std::fabs(t[0] * Rm[0][j] + t[1] * Rm[1][j] + t[2] * Rm[2][j]) > ra + eb[j] + margin;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      const double ra = ea[i1] * Ab[i2][j] + ea[i2] * Ab[i1][j];
      const double rb = eb[j1] * Ab[i][j2] + eb[j2] * Ab[i][j1];
      sep |= std::fabs(t[i2] * Rm[i1][j] - t[i1] * Rm[i2][j]) > ra + rb + margin;
    }
  }
  return sep;
}

// The smallest batches' rows by value in the kernel arguments (which the
// launch writes to device memory anyway): row c = q[dof], then sin/cos
// [2 dof] (revolute sources only), no read of host memory from the kernel
constexpr int kLatIn = 256;  // 12 states of a 7-dof group
struct LatIn {
  double d[kLatIn];
};
static_assert(sizeof(DevWorld) + sizeof(LatIn) + 64 <= 4096, "small_kernel arguments exceed the kernarg limit");

__device__ __forceinline__ double dbl_xor32(double v) {  // lane ^ 32's value
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)u, 32), hi = (unsigned)__shfl_xor((int)(unsigned)(u >> 32), 32);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// SCM (joint sin/cos source): 0 = sc buffer (device), chain FK from the
// snapshot; 1 = computed inline per lane, joints staged in LDS; 2 = sc rows
// in host-mapped memory (computed on the host), copied to LDS in one round of
// loads, FK on the pair's record; 3 = as 2 with the rows in the kernel
// arguments (LatIn)
template <bool FROM_POSES, int CLS, int SCM = 0>
__global__ __launch_bounds__(256) void small_kernel(DevWorld w, const double* __restrict__ in, long long n, int n_tiles,
                                                   uint8_t* __restrict__ hits, const double* __restrict__ sc, LatIn args) {
  constexpr bool INLINE_SC = SCM == 1, STAGED = SCM >= 1, REC = SCM >= 2 && !FROM_POSES;
  if (w.dbg(10)) return;  // diagnostics: the launch alone
  // MPG_STATS: per-wave phase times (s_memrealtime, 100 MHz) into stats[24..31]
  const uint64_t ts0 = w.stats ? __builtin_amdgcn_s_memrealtime() : 0;
  uint64_t tm[6] = {ts0, ts0, ts0, ts0, ts0, ts0};  // phase ends (pre, record, fk, spheres, narrow, store)
  auto tmark = [&](int k, uint64_t&) {
    if (w.stats) tm[k] = __builtin_amdgcn_s_memrealtime();
  };
  uint64_t tlast = ts0;
  const cptr<double> HV = w.hull;
  const uint32_t lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  const int p = wave / n_tiles;
  if (p >= w.n_pairs) return;
  if (cf_class(w.pair_cf[p]) != CLS) return;  // octree / mesh pairs: their own instances
  const long long cfg = (long long)(wave - p * n_tiles) * 64 + lane;
  const bool live = cfg < n;
  const long long c = live ? cfg : n - 1;
  uint8_t hit = 0;
  const int a = w.pair_a[p], b = w.pair_b[p];
  const bool am = a < w.n_moving, bm = b < w.n_moving;
  const int cf = w.pair_cf[p];
  if (!w.pair_allowed[p]) {  // ACM-allowed pairs are never reported (filterCollisions)
    const double* sc_row = FROM_POSES ? nullptr : sc + c * w.dof * 2;
    if constexpr (INLINE_SC && !FROM_POSES) {
      __shared__ double lat_sc[4][64][2 * kLatScDof];
      double* mine = lat_sc[threadIdx.x >> 6][lane];
      const double* qrow = in + c * w.dof;
      if ((am || bm) && w.dof > 0) {  // dof 0: no row (q may be null), every joint is a constant
        // the row first, in one round of loads (it may sit in host memory)
        double qv[kLatScDof];
#pragma unroll
        for (int k = 0; k < kLatScDof; ++k) qv[k] = qrow[min(k, w.dof - 1)];
#pragma unroll
        for (int k = 0; k < kLatScDof; ++k)
          if (k < w.dof) mine[2 * k] = qv[k];
        for (int k0 = 0; k0 < w.dof; k0 += kLatScGroup) {
          double sv[kLatScGroup], cv[kLatScGroup];
#pragma unroll
          for (int i = 0; i < kLatScGroup; ++i) mpg_sincos(mine[2 * min(k0 + i, w.dof - 1)], &sv[i], &cv[i]);
#pragma unroll
          for (int i = 0; i < kLatScGroup; ++i)
            if (k0 + i < w.dof) {
              mine[2 * (k0 + i)] = sv[i];
              mine[2 * (k0 + i) + 1] = cv[i];
            }
        }
      }
      sc_row = mine;
    }
    double* sc2_wave = nullptr;
    if constexpr (SCM == 2 && !FROM_POSES) {
      __shared__ double lat_sc2[4][64][2 * kLatScDof];
      sc2_wave = lat_sc2[threadIdx.x >> 6][0];
      double* mine = lat_sc2[threadIdx.x >> 6][lane];
      if ((am || bm) && w.dof > 0) {
        double v[2 * kLatScDof];
#pragma unroll
        for (int k = 0; k < 2 * kLatScDof; ++k) v[k] = sc_row[min(k, 2 * w.dof - 1)];
#pragma unroll
        for (int k = 0; k < 2 * kLatScDof; ++k)
          if (k < 2 * w.dof) mine[k] = v[k];
      }
      sc_row = mine;
    }
    SE3 TA, TB;
    const double* LRec = nullptr;  // SCM 2/3: the pair's record in LDS
    if constexpr (REC) {
      // the pair's record in LDS: one round of loads (every lane a slice)
      __shared__ double lat_r[4][LR_STRIDE];
      double* R = lat_r[threadIdx.x >> 6];
      LRec = R;
      tmark(0, tlast);  // kernel entry -> before the record loads
      const cptr<double> src = w.lat_rec + (size_t)LR_STRIDE * p;
      constexpr int kPer = (LR_STRIDE + 63) / 64;
      double v[kPer];
#pragma unroll
      for (int i = 0; i < kPer; ++i) v[i] = (int)lane + 64 * i < LR_STRIDE ? src[lane + 64 * i] : 0.0;
      const double* qrow = in + c * w.dof;
      // half waves: with at most 32 states, lanes 0-31 run side A's chain and
      // lanes 32-63 side B's for state lane & 31, then swap (the products are
      // the same, each computed once)
      const bool split = n <= 32;
      const int cs = split ? (int)min((long long)(lane & 31), n - 1) : (int)c;
      if constexpr (SCM == 3) {
        __shared__ double lat_in[4][kLatIn];
        double* I = lat_in[threadIdx.x >> 6];
        const int nin = (int)n * 3 * w.dof;
        for (int i = (int)lane; i < nin; i += 64) I[i] = args.d[i];
        sc_row = I + (size_t)cs * 3 * w.dof + w.dof;
        qrow = I + (size_t)cs * 3 * w.dof;
      } else if (split) {  // state cs's rows: lane cs's LDS copy
        sc_row = sc2_wave + (size_t)cs * 2 * kLatScDof;
        qrow = in + (size_t)cs * w.dof;
      }
#pragma unroll
      for (int i = 0; i < kPer; ++i)
        if ((int)lane + 64 * i < LR_STRIDE) R[lane + 64 * i] = v[i];
      wave_lds_sync();
      auto tf = [&](int sd) {
        return rec_side_tf(R + LR_SIDE + LS_STRIDE * sd, R[sd ? LR_BM : LR_AM] != 0.0, qrow, sc_row);
      };
      tmark(1, tlast);  // the record in LDS
      if (split) {
        const int sd = (int)(lane >> 5);
        const SE3 T = tf(sd);
        SE3 O;
#pragma unroll
        for (int i = 0; i < 9; ++i) O.R[i] = dbl_xor32(T.R[i]);
#pragma unroll
        for (int i = 0; i < 3; ++i) O.p[i] = dbl_xor32(T.p[i]);
        TA = sd ? O : T;
        TB = sd ? T : O;
      } else {
        TA = tf(0);
        TB = tf(1);
      }
      tmark(2, tlast);  // FK of both objects
    } else if constexpr (STAGED && !FROM_POSES) {
      __shared__ LatJoints lat_j[4];
      LatJoints& J = lat_j[threadIdx.x >> 6];
      const int la = am ? w.moving_link[a] : -1, lb = bm ? w.moving_link[b] : -1;
      stage_lat_joints(w, J, lane, la, lb);
      const double* qrow = in + c * w.dof;
      auto tf = [&](int id, int s, int l) {
        const SE3 L = link_from_oMi(w, chain_oMi_lat(w, J, s, l, qrow, sc_row), l, nullptr);
        return se3_mul(L, load_se3(w.moving_offset + 12 * id));
      };
      TA = am ? tf(a, 0, la) : load_se3(w.static_T + 12 * (a - w.n_moving));
      TB = bm ? tf(b, 1, lb) : load_se3(w.static_T + 12 * (b - w.n_moving));
    } else {
      TA = am ? moving_tf_row<FROM_POSES>(w, in, sc_row, c, a) : load_se3(w.static_T + 12 * (a - w.n_moving));
      TB = bm ? moving_tf_row<FROM_POSES>(w, in, sc_row, c, b) : load_se3(w.static_T + 12 * (b - w.n_moving));
    }
    int ga, gb;
    double oa[3], ob[3], rsum;
    if (REC) {
      ga = __builtin_amdgcn_readfirstlane((int)LRec[LR_GA]);
      gb = __builtin_amdgcn_readfirstlane((int)LRec[LR_GB]);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        oa[i] = LRec[LR_SIDE + LS_OBBC + i];
        ob[i] = LRec[LR_SIDE + LS_STRIDE + LS_OBBC + i];
      }
      rsum = LRec[LR_RA] + LRec[LR_RB];
    } else {
      ga = am ? w.moving_geom[a] : w.static_geom[a - w.n_moving];
      gb = bm ? w.moving_geom[b] : w.static_geom[b - w.n_moving];
      const cptr<double> ra = w.geom_rec + G_STRIDE * ga, rb = w.geom_rec + G_STRIDE * gb;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        oa[i] = ra[G_OBB_C + i];
        ob[i] = rb[G_OBB_C + i];
      }
      rsum = ra[G_RADIUS] + rb[G_RADIUS];
    }
    double d2 = 0.0, wc[2][3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double ci = ((TA.R[3 * i] * oa[0] + TA.R[3 * i + 1] * oa[1]) + TA.R[3 * i + 2] * oa[2]) + TA.p[i];
      const double cj = ((TB.R[3 * i] * ob[0] + TB.R[3 * i + 1] * ob[1]) + TB.R[3 * i + 2] * ob[2]) + TB.p[i];
      wc[0][i] = ci;
      wc[1][i] = cj;
      d2 += (ci - cj) * (ci - cj);
    }
    const double rr = rsum + w.small_margin;
    bool near = live && d2 <= rr * rr && !w.dbg(3) && !(w.dbg(7) && d2 >= 0.0);
    if ((CLS == CLS_CLOSED || CLS == CLS_GJK) && __ballot(near) != 0ull) {  // the boxes next (MPR / closed forms)
      const cptr<double> ra = w.geom_rec + G_STRIDE * ga, rb = w.geom_rec + G_STRIDE * gb;
      const double ea[3] = {ra[G_OBB_E], ra[G_OBB_E + 1], ra[G_OBB_E + 2]};
      const double eb[3] = {rb[G_OBB_E], rb[G_OBB_E + 1], rb[G_OBB_E + 2]};
      if (near && dobb_separated(TA.R, wc[0], ea, TB.R, wc[1], eb, w.small_margin)) near = false;
    }
    tmark(3, tlast);  // bounding spheres
    if constexpr (CLS == CLS_OCTREE || CLS == CLS_MESH) {
      hit = (walk_wave_eval<CLS>(w, HV, ga, TA, gb, TB, near) >> lane) & 1ull;
    } else if (cf != CF_NONE) {
      if (near && pair_closed_form<CLS>(cf, w, ga, TA, gb, TB)) hit = 1;
    } else if (__ballot(near) != 0) {
      GObj A, B;
      A.rot = gjk_rot_from_matrix(TA.R);
      A.rot_inv = quat_invert2(A.rot);
      A.pos = cv3(TA.p[0], TA.p[1], TA.p[2]);
      A.geom = ga;
      A.type = w.geom_type[ga];
      B.rot = gjk_rot_from_matrix(TB.R);
      B.rot_inv = quat_invert2(B.rot);
      B.pos = cv3(TB.p[0], TB.p[1], TB.p[2]);
      B.geom = gb;
      B.type = w.geom_type[gb];
      int st = MPR_DONE;
      CV3 v0, v1, v2, v3, dir;
      if (near) mpr_begin(center(w, A), center(w, B), st, v0, dir);
      while (__ballot(st != MPR_DONE) != 0) {
        if (st != MPR_DONE) {
          const CV3 s = msupport(w, HV, A, B, dir);
          const int res = mpr_advance(w.mpr_tol, s, st, v0, v1, v2, v3, dir);
          if (res != 0) {
            hit = res > 0 ? 1 : 0;
            st = MPR_DONE;
          }
        }
      }
    }
    tmark(4, tlast);  // narrow test
  }
  if (live) hits[(size_t)p * n + cfg] = hit;
  if (w.stats) {
    tmark(5, tlast);  // hit store issued
    // phases that did not run (other kernel paths) took no time
    for (int k = 1; k < 6; ++k) tm[k] = tm[k] < tm[k - 1] ? tm[k - 1] : tm[k];
    if (lane_id() == 0) {
      uint64_t prev = ts0;
      for (int k = 0; k < 6; ++k) {
        atomicAdd(&w.stats[24 + k], tm[k] - prev);
        atomicMax(&w.stats[32 + k], tm[k] - prev);
        prev = tm[k];
      }
      atomicAdd(&w.stats[30], tm[5] - ts0);
      atomicMax(&w.stats[38], tm[5] - ts0);
      atomicMax(&w.stats[31], ((tm[4] - tm[3]) << 12) | (uint64_t)p);  // the slowest narrow test's pair
    }
  }
}

// ---------------------------------------------------------------------------
// Latency server: one resident workgroup that serves the smallest host
// batches without a kernel launch each.  The host writes the rows (q, then
// the joint sin/cos it computed) into host-mapped memory and bumps `seq`;
// thread 0 polls it (system-scope loads, s_sleep between polls) and the
// workgroup then runs one batch: FK per (state, moving object) from the
// objects' records in LDS, the bounding-sphere test per (pair, state), the
// near pairs' closed forms / MPR one pair per wave with lanes = states (the
// code small_kernel runs), pair-mask words written with system-scope stores,
// one barrier, ONE system-scope release store of `done` = seq.  It returns
// after idle_ticks (s_memrealtime, 100 MHz) without a request, or when the
// host sets `quit`: every path through the poll loop ends.
// ---------------------------------------------------------------------------
constexpr int kSrvN = 32;        // states per served batch (at most)
constexpr int kSrvMaxG = 8;      // workgroups (pair p belongs to workgroup p % G)
constexpr int kSrvMaxW = 16;     // pair-mask words per state (512 pairs)
constexpr int kSrvThreads = 512;
constexpr int kSrvPT = 24;       // pair-table doubles per pair
struct SrvCtl {
  unsigned long long seq, quit, pad[6];
  unsigned long long done[kSrvMaxG];   // per workgroup: the last batch it published
  unsigned long long gone[kSrvMaxG];   // per workgroup: 1 once it has left (idle or quit)
  unsigned long long phase[8];         // workgroup 0's s_memrealtime at the batch's phase ends (diagnostics)
  double rows[kSrvN * 3 * kLatScDof];  // per state: q[dof], then (sin, cos)[dof]
  uint32_t out[kSrvMaxG][kSrvN * kSrvMaxW];  // per workgroup, per state: its pairs' mask words
};

__device__ __forceinline__ unsigned long long sys_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kSrvJT = 20;   // joint table: type, source, constant, parent, axis[3], pad, placement[12]
constexpr int kSrvOB = 25;   // object table: link placement[12], moving offset[12], the link's parent joint
// one element of se3_mul(A, B) (lane e: row e / 4, column e % 4 of the 3x4
// [R | p]), by se3_mul's formula; se3_slot: where it lives in the 12 doubles
__device__ __forceinline__ int se3_slot(int e) { return (e & 3) < 3 ? 3 * (e >> 2) + (e & 3) : 9 + (e >> 2); }
__device__ __forceinline__ double se3_elem(const double* A, const double* B, int e) {
  const int i = e >> 2, j = e & 3;
  const double* a = A + 3 * i;
  if (j < 3) return (a[0] * B[j] + a[1] * B[3 + j]) + a[2] * B[6 + j];
  return ((a[0] * B[9] + a[1] * B[10]) + a[2] * B[11]) + A[9 + i];
}
// LDS carve-up (doubles, then 32-bit words): joint table, object table,
// static rotations, pair table, rows, joint frames per state, object
// transforms per state, near masks, near-pair list, hit masks
__host__ __device__ inline size_t srv_lds_bytes(int M, int P, int dof, int W, int nj, int ns) {
  const size_t dbl = (size_t)nj * kSrvJT + (size_t)M * kSrvOB + (size_t)ns * 9 + (size_t)P * kSrvPT +
                     (size_t)kSrvN * 3 * dof + (size_t)2 * kSrvN * nj * 12 + (size_t)kSrvN * M * 12;
  return dbl * 8 + ((size_t)2 * P + (size_t)kSrvN * W) * 4;
}

__global__ __launch_bounds__(kSrvThreads) void lat_server_kernel(DevWorld w, SrvCtl* ctl, unsigned long long idle_ticks,
                                                                 int phases) {
  extern __shared__ double srv_lds[];
  const int M = w.n_moving, P = w.n_pairs, dof = w.dof, W = w.W, nj = w.nj, NS = w.n_static;
  double* JT = srv_lds;
  double* OBJ = JT + (size_t)nj * kSrvJT;
  double* SROT = OBJ + (size_t)M * kSrvOB;
  double* PT = SROT + (size_t)NS * 9;
  double* ROWS = PT + (size_t)P * kSrvPT;
  double* OMI = ROWS + (size_t)kSrvN * 3 * dof;
  double* LI = OMI + (size_t)kSrvN * nj * 12;
  double* TT = LI + (size_t)kSrvN * nj * 12;
  uint32_t* NEAR = reinterpret_cast<uint32_t*>(TT + (size_t)kSrvN * M * 12);
  int* NLIST = reinterpret_cast<int*>(NEAR + P);
  uint32_t* HM = reinterpret_cast<uint32_t*>(NLIST + P);
  __shared__ unsigned long long s_cmd;
  __shared__ int s_nl;
  const int t = (int)threadIdx.x, g = (int)blockIdx.x, G = (int)gridDim.x;
  const int PG = P > g ? (P - g + G - 1) / G : 0;  // this workgroup's pairs: g, g + G, ...
  const cptr<double> HV = w.hull;
  unsigned long long last = sys_load(&ctl->done[g]);  // batches up to it are published
  unsigned long long ph[6];  // thread 0's phase stamps
  auto stamp = [&](int k) {
    if (t == 0) ph[k] = __builtin_amdgcn_s_memrealtime();
  };
  // once per residency: joint, object, static-rotation and pair tables
  for (int j = t; j < nj; j += kSrvThreads) {
    double* J = JT + (size_t)kSrvJT * j;
    J[0] = w.joint_type[j];
    J[1] = w.joint_q_source[j];
    J[2] = w.joint_q_const[j];
    J[3] = w.joint_parent[j];
    for (int i = 0; i < 3; ++i) J[4 + i] = w.joint_axis[3 * j + i];
    for (int i = 0; i < 12; ++i) J[8 + i] = w.joint_place[12 * j + i];
  }
  for (int m = t; m < M; m += kSrvThreads) {
    double* O = OBJ + (size_t)kSrvOB * m;
    const int l = w.moving_link[m];
    for (int i = 0; i < 12; ++i) O[i] = w.link_place[12 * l + i];
    for (int i = 0; i < 12; ++i) O[12 + i] = w.moving_offset[12 * m + i];
    O[24] = w.link_parent[l];
  }
  for (int i = t; i < NS * 9; i += kSrvThreads) SROT[i] = w.static_T[12 * (i / 9) + i % 9];
  int probe_cb = -1;  // MPG_STATS probe: the first walk hull's cell records
  if (w.stats && g == 0 && t == 0)
    for (int gg = 0; gg < w.n_geoms && probe_cb < 0; ++gg)
      if (w.geom_nbr[gg] >= 0 && w.geom_cbase[gg] >= 0) probe_cb = w.geom_cbase[gg];
  if (probe_cb >= 0) {
    // shader clocks of 16 dependent loads through one hull's walk cell
    // records, first pass and again (the same addresses)
    const int nrec = kCellsPerHull;
    for (int pass = 0; pass < 2; ++pass) {
      int idx = 7;
      const unsigned long long c0 = __builtin_amdgcn_s_memtime();
      for (int k = 0; k < 16; ++k) {
        const double v = w.wcell_rec[kCellRec * (size_t)(probe_cb + (idx * 97 + k * 131) % nrec) + 9];
        idx = (int)v & 1023;  // the next address depends on this load
      }
      asm volatile("" ::"v"(idx));  // the chain has completed before the clock is read
      const unsigned long long c1 = __builtin_amdgcn_s_memtime();
      atomicAdd(&w.stats[40 + pass], (c1 - c0) + (idx == -1 ? 1ull : 0ull));
      atomicAdd(&w.stats[42 + pass], 16ull);
    }
  }
  for (int p = t; p < P; p += kSrvThreads) {
    const cptr<double> R = w.lat_rec + (size_t)LR_STRIDE * p;
    double* E = PT + (size_t)kSrvPT * p;
    E[0] = R[LR_ALLOWED];
    E[1] = R[LR_CF];
    E[2] = R[LR_GA];
    E[3] = R[LR_GB];
    E[4] = w.pair_a[p];
    E[5] = w.pair_b[p];
    E[6] = R[LR_RA] + R[LR_RB];
    for (int i = 0; i < 3; ++i) {  // half extents of the boxes
      E[13 + i] = w.geom_rec[G_STRIDE * (int)R[LR_GA] + G_OBB_E + i];
      E[16 + i] = w.geom_rec[G_STRIDE * (int)R[LR_GB] + G_OBB_E + i];
    }
    for (int sd = 0; sd < 2; ++sd) {
      const cptr<double> S = R + LR_SIDE + LS_STRIDE * sd;
      const double o0 = S[LS_OBBC], o1 = S[LS_OBBC + 1], o2 = S[LS_OBBC + 2];
      if (R[sd ? LR_BM : LR_AM] != 0.0) {  // moving: the centre in its own frame
        E[7 + 3 * sd] = o0;
        E[8 + 3 * sd] = o1;
        E[9 + 3 * sd] = o2;
      } else {  // static: its world centre, as small_kernel computes it
        const SE3 T = load_se3(S + LS_OFF);
        for (int i = 0; i < 3; ++i)
          E[7 + 3 * sd + i] = ((T.R[3 * i] * o0 + T.R[3 * i + 1] * o1) + T.R[3 * i + 2] * o2) + T.p[i];
      }
    }
  }
  __syncthreads();
  for (;;) {
    if (t == 0) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      unsigned long long cmd = 0;
      for (;;) {
        const unsigned long long sq = sys_load(&ctl->seq);
        if (sq != last) {
          // The host stores the rows, then seq with release (x86: in order).
          // The rows are read below with system-coherent loads (sys_load: sc0
          // sc1, past L1 and L2), issued only after this value returned (the
          // branch waits on it), so they see the host's row stores.  The
          // compiler fence keeps them after this load in the program; a
          // system-scope acquire would add an L2 invalidate per batch, which
          // measured +1.8 us on the one-state round trip
          // (profiles/r05a/server_acquire.txt) and protects nothing here.
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
          cmd = sq;
          break;
        }
        if (sys_load(&ctl->quit) != 0ull) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
        __builtin_amdgcn_s_sleep(2);
      }
      s_cmd = cmd;  // the batch size rides in the low byte of seq
      s_nl = 0;
    }
    __syncthreads();
    const unsigned long long cmd = s_cmd;
    if (cmd == 0ull) {  // idle or quit: the whole workgroup leaves together
      if (t == 0) __hip_atomic_store(&ctl->gone[g], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    last = cmd;
    stamp(0);
    const int n = (int)min(cmd & 255ull, (unsigned long long)kSrvN);
    for (int i = t; i < n * 3 * dof; i += kSrvThreads)
      ROWS[i] = __longlong_as_double((long long)sys_load(reinterpret_cast<const unsigned long long*>(&ctl->rows[i])));
    for (int i = t; i < P; i += kSrvThreads) NEAR[i] = 0u;
    for (int i = t; i < n * W; i += kSrvThreads) HM[i] = 0u;
    __syncthreads();
    stamp(1);
    // FK, first the joint frames (forward_kinematics: oMi[j] = oMi[parent] *
    // (placement * M(q)), the products chain_oMi forms for every link), one
    // SE3 element per lane (se3_elem: se3_mul's formula for that element):
    // every joint's placement * M(q) at once ...
    for (int k = t; k < n * nj * 12; k += kSrvThreads) {
      const int e = k % 12, cj = k / 12, c = cj / nj, j = cj - c * nj;
      const double* row = ROWS + (size_t)c * 3 * dof;
      const double* J = JT + (size_t)kSrvJT * j;
      const int type = (int)J[0], srcq = (int)J[1];
      const bool pre = srcq >= 0 && joint_is_revolute(type);
      const double qv = pre ? 0.0 : srcq >= 0 ? row[srcq] : J[2];
      const SE3 Mq = joint_motion(type, J + 4, qv, pre ? row + dof + 2 * srcq : nullptr);
      const int jc = e & 3;  // the column of M(q) this element reads
      const double b0 = jc == 0 ? Mq.R[0] : jc == 1 ? Mq.R[1] : jc == 2 ? Mq.R[2] : Mq.p[0];
      const double b1 = jc == 0 ? Mq.R[3] : jc == 1 ? Mq.R[4] : jc == 2 ? Mq.R[5] : Mq.p[1];
      const double b2 = jc == 0 ? Mq.R[6] : jc == 1 ? Mq.R[7] : jc == 2 ? Mq.R[8] : Mq.p[2];
      const double* a = J + 8 + 3 * (e >> 2);
      const double v = jc < 3 ? (a[0] * b0 + a[1] * b1) + a[2] * b2 : ((a[0] * b0 + a[1] * b1) + a[2] * b2) + J[8 + 9 + (e >> 2)];
      LI[(size_t)cj * 12 + se3_slot(e)] = v;
    }
    __syncthreads();
    // ... then the chain, joint after joint, twelve lanes per state (five
    // states per wave, the group never straddles a wave)
    {
      const int g = lane_id() / 12, e = (int)lane_id() - 12 * g;
      const int c = (t >> 6) * 5 + g;
      if (g < 5 && c < n) {
        double* om = OMI + (size_t)c * nj * 12;
        const double* lic = LI + (size_t)c * nj * 12;
        for (int j = 0; j < nj; ++j) {
          const int par = (int)JT[(size_t)kSrvJT * j + 3];
          const double v = par > 0 ? se3_elem(om + 12 * (par - 1), lic + 12 * j, e) : lic[12 * j + se3_slot(e)];
          om[12 * j + se3_slot(e)] = v;
          wave_lds_sync();
        }
      }
    }
    __syncthreads();
    // ... then one (state, moving object) per thread: link_from_oMi and the
    // moving offset, as rec_side_tf
    for (int k = t; k < n * M; k += kSrvThreads) {
      const int c = k / M, m = k - c * M;
      const double* O = OBJ + (size_t)kSrvOB * m;
      const int jl = (int)O[24];
      SE3 P0;
      if (jl > 0) P0 = load_se3(OMI + ((size_t)c * nj + jl - 1) * 12);
      else se3_identity(P0);
      const SE3 L = se3_mul(P0, load_se3(O));
      double qw, qxyz[3];
      mat_to_quat(L.R, &qw, qxyz);
      SE3 Lr;
      quat_to_mat(qw, qxyz[0], qxyz[1], qxyz[2], Lr.R);
      Lr.p[0] = L.p[0];
      Lr.p[1] = L.p[1];
      Lr.p[2] = L.p[2];
      const SE3 T = se3_mul(Lr, load_se3(O + 12));
      double* o = TT + ((size_t)c * M + m) * 12;
#pragma unroll
      for (int i = 0; i < 9; ++i) o[i] = T.R[i];
      o[9] = T.p[0];
      o[10] = T.p[1];
      o[11] = T.p[2];
    }
    __syncthreads();
    stamp(2);
    // bounding spheres: one (pair, state) per thread
    for (int k = t; k < PG * n; k += kSrvThreads) {
      const int p = g + G * (k / n), c = k % n;
      const double* E = PT + (size_t)kSrvPT * p;
      if (E[0] != 0.0) continue;  // ACM-allowed
      double ce[2][3];
      const double* Rs[2];
      for (int sd = 0; sd < 2; ++sd) {
        const int id = (int)E[4 + sd];
        const double* oc = E + 7 + 3 * sd;
        if (id < M) {
          const double* T = TT + ((size_t)c * M + id) * 12;
          Rs[sd] = T;
#pragma unroll
          for (int i = 0; i < 3; ++i) ce[sd][i] = ((T[3 * i] * oc[0] + T[3 * i + 1] * oc[1]) + T[3 * i + 2] * oc[2]) + T[9 + i];
        } else {
          Rs[sd] = nullptr;
#pragma unroll
          for (int i = 0; i < 3; ++i) ce[sd][i] = oc[i];
        }
      }
      double d2 = 0.0;
#pragma unroll
      for (int i = 0; i < 3; ++i) d2 += (ce[0][i] - ce[1][i]) * (ce[0][i] - ce[1][i]);
      const double rr = E[6] + w.small_margin;
      if (!(d2 <= rr * rr)) continue;
      for (int sd = 0; sd < 2; ++sd)  // static sides: their world rotation
        if (!Rs[sd]) Rs[sd] = SROT + 9 * ((int)E[4 + sd] - M);
      if (!dobb_separated(Rs[0], ce[0], E + 13, Rs[1], ce[1], E + 16, w.small_margin)) atomicOr(&NEAR[p], 1u << c);
    }
    __syncthreads();
    for (int p = g + G * t; p < P; p += G * kSrvThreads)
      if (NEAR[p]) NLIST[atomicAdd(&s_nl, 1)] = p;
    __syncthreads();
    stamp(3);
    // narrow: one near pair per wave at a time, lanes = states.  With at most
    // 32 states both half-waves run every state's MPR (lane and lane ^ 32
    // carry the same state) and split each support: one half a's, the other
    // b's (msupport_split), which halves the support's dependent chain
    const int wv = t >> 6, lane = t & 63, nl = s_nl;
    const bool split = n <= 32;
    const int sl = split ? (lane & 31) : lane;  // the state this lane carries
    for (int k = wv; k < nl; k += kSrvThreads / 64) {
      const int p = __builtin_amdgcn_readfirstlane(NLIST[k]);
      const double* E = PT + (size_t)kSrvPT * p;
      const int cf = __builtin_amdgcn_readfirstlane((int)E[1]);
      const int ga = __builtin_amdgcn_readfirstlane((int)E[2]), gb = __builtin_amdgcn_readfirstlane((int)E[3]);
      const int a = __builtin_amdgcn_readfirstlane((int)E[4]), b = __builtin_amdgcn_readfirstlane((int)E[5]);
      const bool near = sl < n && ((NEAR[p] >> sl) & 1u);
      const int c = sl < n ? sl : 0;
      const SE3 TA = a < M ? load_se3(TT + ((size_t)c * M + a) * 12) : load_se3(w.static_T + 12 * (a - M));
      const SE3 TB = b < M ? load_se3(TT + ((size_t)c * M + b) * 12) : load_se3(w.static_T + 12 * (b - M));
      bool hit = false;
      if (cf != CF_NONE) {
        if (near && pair_closed_form<CLS_CLOSED>(cf, w, ga, TA, gb, TB)) hit = true;
      } else {
        GObj A, B;
        A.rot = gjk_rot_from_matrix(TA.R);
        A.rot_inv = quat_invert2(A.rot);
        A.pos = cv3(TA.p[0], TA.p[1], TA.p[2]);
        A.geom = ga;
        A.type = w.geom_type[ga];
        B.rot = gjk_rot_from_matrix(TB.R);
        B.rot_inv = quat_invert2(B.rot);
        B.pos = cv3(TB.p[0], TB.p[1], TB.p[2]);
        B.geom = gb;
        B.type = w.geom_type[gb];
        int st = MPR_DONE;
        CV3 v0, v1, v2, v3, dir;
        if (near) mpr_begin(center(w, A), center(w, B), st, v0, dir);
        unsigned long long t_sup = 0, t_adv = 0, n_it = 0;  // MPG_STATS: MPR step costs (shader clocks)
        while (__ballot(st != MPR_DONE) != 0) {
          const unsigned long long c0 = w.stats ? __builtin_amdgcn_s_memtime() : 0ull;
          if (st != MPR_DONE) {
            const CV3 sp = split ? msupport_split(w, HV, A, B, dir, lane >= 32) : msupport(w, HV, A, B, dir);
            const unsigned long long c1 = w.stats ? __builtin_amdgcn_s_memtime() : 0ull;
            const int res = mpr_advance(w.mpr_tol, sp, st, v0, v1, v2, v3, dir);
            if (res != 0) {
              hit = res > 0;
              st = MPR_DONE;
            }
            if (w.stats) {
              t_sup += c1 - c0;
              t_adv += __builtin_amdgcn_s_memtime() - c1;
            }
          }
          ++n_it;
        }
        if (w.stats && lane == 0 && n_it > 0) {
          atomicAdd(&w.stats[20], n_it);
          atomicAdd(&w.stats[21], t_sup);
          atomicAdd(&w.stats[22], t_adv);
          atomicMax(&w.stats[23], n_it);
        }
      }
      if (hit && (!split || lane < 32)) atomicOr(&HM[c * W + (p >> 5)], 1u << (p & 31));
    }
    __syncthreads();
    stamp(4);
    // publish: wave 0 writes every pair-mask word, then its lane 0 releases
    // `done` at system scope (the release waits for the whole wave's stores)
    if (t < 64) {
      for (int i = t; i < n * W; i += 64) __hip_atomic_store(&ctl->out[g][i], HM[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (t == 0 && g == 0 && phases) {  // MPG_STATS only: six more stores for the release to wait on
        ph[5] = __builtin_amdgcn_s_memrealtime();
        for (int k = 0; k < 6; ++k) __hip_atomic_store(&ctl->phase[k], ph[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __builtin_amdgcn_s_waitcnt(0);
      if (t == 0) __hip_atomic_store(&ctl->done[g], cmd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------------------
// Diagnostics: fcl::collide of two posed geometries of the world, n pose
// pairs at a time (one lane each; the geometries are the same for the whole
// launch, as the narrow phase's wave-uniform support scans need): the exact
// dispatch collide() uses -- FCL closed form, octree or BVH-mesh walk, or
// libccd MPR.  Lets tests compare the narrow phase with the oracle directly,
// without forward kinematics (mpg_debug_collide_pairs).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void debug_pairs_kernel(DevWorld w, int ga, int gb, int cf, long long n,
                                                         const double* __restrict__ Ta, const double* __restrict__ Tb,
                                                         uint8_t* __restrict__ hit) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = i < n;
  const long long c = live ? i : n - 1;
  const SE3 TA = load_se3(Ta + 12 * c), TB = load_se3(Tb + 12 * c);
  bool h = false;
  if (cf == CF_OCTREE) {
    h = (walk_wave_eval<CLS_OCTREE>(w, w.hull, ga, TA, gb, TB, live) >> lane_id()) & 1ull;
  } else if (cf == CF_MESH) {
    h = (walk_wave_eval<CLS_MESH>(w, w.hull, ga, TA, gb, TB, live) >> lane_id()) & 1ull;
  } else if (cf != CF_NONE) {
    h = live && closed_form(cf, w, ga, TA, gb, TB);
  } else {
    GObj A, B;
    A.rot = gjk_rot_from_matrix(TA.R);
    A.rot_inv = quat_invert2(A.rot);
    A.pos = cv3(TA.p[0], TA.p[1], TA.p[2]);
    A.geom = ga;
    A.type = w.geom_type[ga];
    B.rot = gjk_rot_from_matrix(TB.R);
    B.rot_inv = quat_invert2(B.rot);
    B.pos = cv3(TB.p[0], TB.p[1], TB.p[2]);
    B.geom = gb;
    B.type = w.geom_type[gb];
    int st = MPR_DONE;
    CV3 v0, v1, v2, v3, dir;
    if (live) mpr_begin(center(w, A), center(w, B), st, v0, dir);
    while (__ballot(st != MPR_DONE) != 0) {
      if (st != MPR_DONE) {
        const CV3 s = msupport(w, w.hull, A, B, dir);
        const int res = mpr_advance(w.mpr_tol, s, st, v0, v1, v2, v3, dir);
        if (res != 0) {
          h = res > 0;
          st = MPR_DONE;
        }
      }
    }
  }
  if (live) hit[i] = h ? 1 : 0;
}

// ---------------------------------------------------------------------------
// Batched distance (PlanningWorld::distanceSelf / distanceOthers,
// src/planning_world.cpp:493-720): exact fp64 object poses once per
// configuration (pose_kernel), then per configuration every non-allowed pair
// in order with a bounding-sphere lower bound against the running minimum,
// GJK distance on the FCL support mappings (-1 for penetrating pairs, as
// fcl::distance with DistanceRequest() reports), strict '<' keeps the first
// minimum.  Same algorithm as the oracle (oracle/collide_oracle.c
// gjk_distance); the north star's bar vs FCL's GJK is 1e-5.
// ---------------------------------------------------------------------------
constexpr int kPoseStride = 20;  // rot xyzw, pos xyz, world OBB centre xyz, fp64 rotation (mesh pairs), pad

template <bool FROM_POSES>
__global__ __launch_bounds__(128) void pose_kernel(DevWorld w, const double* __restrict__ in, long long n,
                                                   double* __restrict__ poses, double* __restrict__ save64) {
  const long long cfg = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (cfg >= n) return;
  auto store = [&](int m, const SE3& T) {
    const CQ4 r = gjk_rot_from_matrix(T.R);
    double* g = poses + ((size_t)m * kPoseStride) * n + cfg;  // [m][field][cfg]
    g[0 * n] = r.x;
    g[1 * n] = r.y;
    g[2 * n] = r.z;
    g[3 * n] = r.w;
    g[4 * n] = T.p[0];
    g[5 * n] = T.p[1];
    g[6 * n] = T.p[2];
    const cptr<double> gr = w.geom_rec + G_STRIDE * w.moving_geom[m];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      g[(7 + i) * n] = ((T.R[3 * i] * gr[G_OBB_C] + T.R[3 * i + 1] * gr[G_OBB_C + 1]) + T.R[3 * i + 2] * gr[G_OBB_C + 2]) +
                       T.p[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) g[(10 + i) * n] = T.R[i];
  };
  if (FROM_POSES) {
    for (int m = 0; m < w.n_moving; ++m)
      store(m, se3_mul(link_from_pose7(in + (cfg * w.n_links + w.moving_link[m]) * 7), load_se3(w.moving_offset + 12 * m)));
    return;
  }
  // oMi[j] = oMi[parent] * (jointPlacement_j * M_j(q)); branch frames spilled
  const double* qrow = in + cfg * w.dof;
  SE3 cur;
  se3_identity(cur);
  for (int j = 0; j <= w.nj; ++j) {
    if (j > 0) {
      const int jj = j - 1;
      const int src = w.joint_q_source[jj];
      const double v = src >= 0 ? qrow[src] : w.joint_q_const[jj];
      const SE3 li = se3_mul(load_se3(w.joint_place + 12 * jj), joint_motion(w.joint_type[jj], w.joint_axis + 3 * jj, v));
      const int sidx = w.bp.jsrc[jj];
      if (sidx < 0) {
        cur = li;
      } else if (sidx > 0) {
        SE3 P;
        const double* sp = save64 + (size_t)(sidx - 1) * 12 * n + cfg;
        for (int i = 0; i < 9; ++i) P.R[i] = sp[i * n];
        for (int i = 0; i < 3; ++i) P.p[i] = sp[(9 + i) * n];
        cur = se3_mul(P, li);
      } else {
        cur = se3_mul(cur, li);
      }
      const int sv = w.bp.jsave[jj];
      if (sv >= 0) {
        double* sp = save64 + (size_t)sv * 12 * n + cfg;
        for (int i = 0; i < 9; ++i) sp[i * n] = cur.R[i];
        for (int i = 0; i < 3; ++i) sp[(9 + i) * n] = cur.p[i];
      }
    }
    for (int k = w.bp.link_start[j]; k < w.bp.link_start[j + 1]; ++k) {
      const int l = w.bp.link_order[k];
      const int o0 = w.bp.obj_start[l], o1 = w.bp.obj_start[l + 1];
      if (o0 == o1) continue;
      SE3 root;
      se3_identity(root);
      const SE3 L = link_from_oMi(w, j == 0 ? root : cur, l, nullptr);
      for (int o = o0; o < o1; ++o) {
        const int m = w.bp.obj_order[o];
        store(m, se3_mul(L, load_se3(w.moving_offset + 12 * m)));
      }
    }
  }
}

__device__ __forceinline__ double d3dot(const V3& a, const V3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// ---------------------------------------------------------------------------
// FCL 0.7.0 shape distance: GJKDistance / GJKSignedDistance on float libccd
// (mpg_ccd_dist.h, the twin of oracle/fcl_gjk_dist.h), the closed forms of
// GJKSolver_libccd::shapeDistance, and the support mappings they run on.
// ---------------------------------------------------------------------------
#include "mpg_ccd_dist.h"

// __ccdSupport of (uniform shape a) - (uniform shape b), both points kept
__device__ __forceinline__ ccdx::Sup csup(const DevWorld& w, cptr<double> HV, const GObj& a, const GObj& b,
                                         const CV3& dir) {
  const CV3 da = quat_rot(dir, a.rot_inv), db = quat_rot(vscale(dir, ccd_real(-1)), b.rot_inv);
  const int ga = __builtin_amdgcn_readfirstlane(a.geom), ta = __builtin_amdgcn_readfirstlane(a.type);
  const int gb = __builtin_amdgcn_readfirstlane(b.geom), tb = __builtin_amdgcn_readfirstlane(b.type);
  const CV3 la = support_local(w, HV, ga, ta, da), lb = support_local(w, HV, gb, tb, db);
  ccdx::Sup s;
  s.v1 = vadd(quat_rot(la, a.rot), a.pos);
  s.v2 = vadd(quat_rot(lb, b.rot), b.pos);
  s.v = vsub(s.v1, s.v2);
  return s;
}

// boxToGJK support with per-lane half sizes h (an octree leaf box)
__device__ __forceinline__ CV3 box_support_world(const GObj& a, const ccd_real* h, const CV3& dir) {
  const CV3 da = quat_rot(dir, a.rot_inv);
  const CV3 la = CV3{(da.x >= 0 ? ccd_real(1) : ccd_real(-1)) * h[0], (da.y >= 0 ? ccd_real(1) : ccd_real(-1)) * h[1],
                     (da.z >= 0 ? ccd_real(1) : ccd_real(-1)) * h[2]};
  return vadd(quat_rot(la, a.rot), a.pos);
}

// (leaf box a) - (uniform shape b)
__device__ __forceinline__ ccdx::Sup csup_box(const GObj& a, const ccd_real* h, const DevWorld& w, cptr<double> HV,
                                              const GObj& b, const CV3& dir) {
  ccdx::Sup s;
  s.v1 = box_support_world(a, h, dir);
  const CV3 db = quat_rot(vscale(dir, ccd_real(-1)), b.rot_inv);
  const int gb = __builtin_amdgcn_readfirstlane(b.geom), tb = __builtin_amdgcn_readfirstlane(b.type);
  s.v2 = vadd(quat_rot(support_local(w, HV, gb, tb, db), b.rot), b.pos);
  s.v = vsub(s.v1, s.v2);
  return s;
}

__device__ __forceinline__ CV3 tri_support(const GObj& b, const CV3* P, const CV3& tc, const CV3& dir);

// (uniform shape a) - (triangle b: vertices P and centroid tc in the mesh frame)
__device__ __forceinline__ ccdx::Sup csup_tri(const DevWorld& w, cptr<double> HV, const GObj& a, const GObj& b,
                                              const CV3* P, const CV3& tc, const CV3& dir) {
  ccdx::Sup s;
  const CV3 da = quat_rot(dir, a.rot_inv);
  const int ga = __builtin_amdgcn_readfirstlane(a.geom), ta = __builtin_amdgcn_readfirstlane(a.type);
  s.v1 = vadd(quat_rot(support_local(w, HV, ga, ta, da), a.rot), a.pos);
  s.v2 = tri_support(b, P, tc, vscale(dir, ccd_real(-1)));
  s.v = vsub(s.v1, s.v2);
  return s;
}

// (leaf box a) - (triangle b)
__device__ __forceinline__ ccdx::Sup csup_box_tri(const GObj& a, const ccd_real* h, const GObj& b, const CV3* P,
                                                  const CV3& tc, const CV3& dir) {
  ccdx::Sup s;
  s.v1 = box_support_world(a, h, dir);
  s.v2 = tri_support(b, P, tc, vscale(dir, ccd_real(-1)));
  s.v = vsub(s.v1, s.v2);
  return s;
}

// ccdx status -> the pair-index sentinel the distance outputs carry
constexpr int kDistThrow = MPG_DISTANCE_FCL_THROWS, kDistOverflow = MPG_DISTANCE_EPA_CAPACITY;

// ---- closed-form shape distances (GJKSolver_libccd::shapeDistance's
// specialisations [ext FCL 0.7.0]; oracle/fcl_gjk_dist.h cf_*, same order)
__device__ __forceinline__ void cf_tf_point(const SE3& T, const double* p, double* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = ((T.R[3 * i] * p[0] + T.R[3 * i + 1] * p[1]) + T.R[3 * i + 2] * p[2]) + T.p[i];
}
__device__ __forceinline__ double cf_norm(const double* v) { return std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]); }
// X_FO.inverse() * X_FS: the sphere centre in the other shape's frame
__device__ __forceinline__ void cf_centre_in_frame(const SE3& TS, const SE3& TO, double* c) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double inv_t = -((TO.R[i] * TO.p[0] + TO.R[3 + i] * TO.p[1]) + TO.R[6 + i] * TO.p[2]);
    c[i] = ((TO.R[i] * TS.p[0] + TO.R[3 + i] * TS.p[1]) + TO.R[6 + i] * TS.p[2]) + inv_t;
  }
}

__device__ double cf_sphere_sphere(double r1, const SE3& T1, double r2, const SE3& T2, double* p1, double* p2) {
  const double diff[3] = {T1.p[0] - T2.p[0], T1.p[1] - T2.p[1], T1.p[2] - T2.p[2]};
  const double len = cf_norm(diff);
  if (len > r1 + r2) {
    for (int i = 0; i < 3; ++i) {
      p1[i] = T1.p[i] - diff[i] * (r1 / len);
      p2[i] = T2.p[i] + diff[i] * (r2 / len);
    }
    return len - (r1 + r2);
  }
  return -1.0;
}

__device__ double cf_sphere_capsule(double r1, const SE3& TS, double r2, double lz, const SE3& TC, double* p1,
                                    double* p2) {
  const double a[3] = {0.0, 0.0, 0.5 * lz}, b[3] = {0.0, 0.0, -0.5 * lz};
  double pos1[3], pos2[3], sp[3];
  cf_tf_point(TC, a, pos1);
  cf_tf_point(TC, b, pos2);
  const double* sc = TS.p;
  const double v[3] = {pos2[0] - pos1[0], pos2[1] - pos1[1], pos2[2] - pos1[2]};
  const double wv[3] = {sc[0] - pos1[0], sc[1] - pos1[1], sc[2] - pos1[2]};
  const double c1 = (wv[0] * v[0] + wv[1] * v[1]) + wv[2] * v[2];
  const double c2 = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
  if (c1 <= 0) {
    for (int i = 0; i < 3; ++i) sp[i] = pos1[i];
  } else if (c2 <= c1) {
    for (int i = 0; i < 3; ++i) sp[i] = pos2[i];
  } else {
    const double bb = c1 / c2;
    for (int i = 0; i < 3; ++i) sp[i] = pos1[i] + v[i] * bb;
  }
  double diff[3] = {sc[0] - sp[0], sc[1] - sp[1], sc[2] - sp[2]};
  const double distance = cf_norm(diff) - r1 - r2;
  if (distance <= 0) return -1.0;
  const double n = cf_norm(diff);
  for (int i = 0; i < 3; ++i) diff[i] /= n;
  for (int i = 0; i < 3; ++i) {
    p1[i] = sc[i] - diff[i] * r1;
    p2[i] = sp[i] + diff[i] * r2;
  }
  return distance;
}

__device__ double cf_sphere_box(double r, const SE3& TS, const double* side, const SE3& TB, double* pS, double* pB) {
  double c[3], nq[3];
  cf_centre_in_frame(TS, TB, c);
  bool clamped = false;
  for (int i = 0; i < 3; ++i) {
    const double h = side[i] / 2;
    nq[i] = c[i];
    if (c[i] < -h) {
      clamped = true;
      nq[i] = -h;
    }
    if (c[i] > h) {
      clamped = true;
      nq[i] = h;
    }
  }
  if (clamped) {
    const double nc[3] = {c[0] - nq[0], c[1] - nq[1], c[2] - nq[2]};
    const double sq = (nc[0] * nc[0] + nc[1] * nc[1]) + nc[2] * nc[2];
    if (sq > r * r) {
      const double d = std::sqrt(sq);
      double pSb[3];
      for (int i = 0; i < 3; ++i) pSb[i] = (nc[i] / d) * (d - r) + nq[i];
      cf_tf_point(TB, nq, pB);
      cf_tf_point(TB, pSb, pS);
      return d - r;
    }
  }
  return -1.0;
}

__device__ double cf_sphere_cylinder(double r, const SE3& TS, double rc, double lz, const SE3& TC, double* pS,
                                     double* pC) {
  double c[3], n[3];
  cf_centre_in_frame(TS, TC, c);
  const double h = lz / 2;
  bool clamped = false;
  n[0] = c[0];
  n[1] = c[1];
  n[2] = c[2];
  if (c[2] > h) {
    n[2] = h;
    clamped = true;
  } else if (c[2] < -h) {
    n[2] = -h;
    clamped = true;
  }
  const double rd2 = c[0] * c[0] + c[1] * c[1];
  if (rd2 > rc * rc) {
    const double scale = rc / std::sqrt(rd2);
    n[0] = c[0] * scale;
    n[1] = c[1] * scale;
    clamped = true;
  }
  if (clamped) {
    const double nc[3] = {c[0] - n[0], c[1] - n[1], c[2] - n[2]};
    const double sq = (nc[0] * nc[0] + nc[1] * nc[1]) + nc[2] * nc[2];
    if (sq > r * r) {
      const double d = std::sqrt(sq);
      double pSc[3];
      for (int i = 0; i < 3; ++i) pSc[i] = (nc[i] / d) * (d - r) + n[i];
      cf_tf_point(TC, n, pC);
      cf_tf_point(TC, pSc, pS);
      return d - r;
    }
  }
  return -1.0;
}

__device__ __forceinline__ double cf_clamp01(double v) { return v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v); }

__device__ double cf_capsule_capsule(double r1, double lz1, const SE3& T1, double r2, double lz2, const SE3& T2,
                                     double* p1, double* p2) {
  const double eps = 0x1.6a09e667f3bcdp-46, eps2 = eps * eps;  // constants<double>::eps_78() = pow(DBL_EPSILON, 7/8)
  double P1[3], Q1[3], P2[3], Q2[3];
  for (int i = 0; i < 3; ++i) {
    const double h1 = (lz1 / 2) * T1.R[3 * i + 2], h2 = (lz2 / 2) * T2.R[3 * i + 2];
    P1[i] = T1.p[i] + h1;
    Q1[i] = T1.p[i] - h1;
    P2[i] = T2.p[i] + h2;
    Q2[i] = T2.p[i] - h2;
  }
  double d1[3], d2[3], rr[3];
  for (int i = 0; i < 3; ++i) {
    d1[i] = Q1[i] - P1[i];
    d2[i] = Q2[i] - P2[i];
    rr[i] = P1[i] - P2[i];
  }
  const double a = (d1[0] * d1[0] + d1[1] * d1[1]) + d1[2] * d1[2];
  const double e = (d2[0] * d2[0] + d2[1] * d2[1]) + d2[2] * d2[2];
  const double f = (d2[0] * rr[0] + d2[1] * rr[1]) + d2[2] * rr[2];
  double s, t;
  if (a <= eps2 && e <= eps2) {
    s = t = 0.0;
  } else if (a <= eps2) {
    s = 0.0;
    t = cf_clamp01(f / e);
  } else {
    const double c = (d1[0] * rr[0] + d1[1] * rr[1]) + d1[2] * rr[2];
    if (e <= eps2) {
      t = 0.0;
      s = cf_clamp01(-c / a);
    } else {
      const double b = (d1[0] * d2[0] + d1[1] * d2[1]) + d1[2] * d2[2];
      const double den0 = a * e - b * b, denom = den0 > 0.0 ? den0 : 0.0;
      s = denom > eps2 ? cf_clamp01((b * f - c * e) / denom) : 0.0;
      t = (b * s + f) / e;
      if (t < 0.0) {
        t = 0.0;
        s = cf_clamp01(-c / a);
      } else if (t > 1.0) {
        t = 1.0;
        s = cf_clamp01((b - c) / a);
      }
    }
  }
  double N1[3], N2[3], v[3];
  for (int i = 0; i < 3; ++i) {
    N1[i] = P1[i] + d1[i] * s;
    N2[i] = P2[i] + d2[i] * t;
    v[i] = N2[i] - N1[i];
  }
  const double seg = std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
  double vh[3];
  if (seg > eps) {
    for (int i = 0; i < 3; ++i) vh[i] = v[i] / seg;
  } else {
    double n[3] = {d1[1] * d2[2] - d1[2] * d2[1], d1[2] * d2[0] - d1[0] * d2[2], d1[0] * d2[1] - d1[1] * d2[0]};
    double nl = cf_norm(n);
    if (!(nl > eps)) {
      const double ax[3] = {std::fabs(d1[0]) < std::fabs(d1[1]) ? 1.0 : 0.0,
                            std::fabs(d1[0]) < std::fabs(d1[1]) ? 0.0 : 1.0, 0.0};
      n[0] = d1[1] * ax[2] - d1[2] * ax[1];
      n[1] = d1[2] * ax[0] - d1[0] * ax[2];
      n[2] = d1[0] * ax[1] - d1[1] * ax[0];
      nl = cf_norm(n);
    }
    for (int i = 0; i < 3; ++i) vh[i] = nl > 0.0 ? n[i] / nl : (i == 2 ? 1.0 : 0.0);
  }
  for (int i = 0; i < 3; ++i) {
    p1[i] = N1[i] + vh[i] * r1;
    p2[i] = N2[i] - vh[i] * r2;
  }
  return seg - r1 - r2;
}

// 1 if (ta, tb) has a closed form; d and the points (zeros for -1)
__device__ bool cf_shape_distance(const DevWorld& w, int ga, int ta, const SE3& Ta, int gb, int tb, const SE3& Tb,
                                  double& d, V3& q1, V3& q2) {
  const cptr<double> pa = w.geom_rec + G_STRIDE * ga + G_PARAM, pb = w.geom_rec + G_STRIDE * gb + G_PARAM;
  double p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
  if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_SPHERE) {
    d = cf_sphere_sphere(pa[0], Ta, pb[0], Tb, p1, p2);
  } else if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_CAPSULE) {
    d = cf_sphere_capsule(pa[0], Ta, pb[0], pb[1], Tb, p1, p2);
  } else if (ta == MPG_GEOM_CAPSULE && tb == MPG_GEOM_SPHERE) {
    d = cf_sphere_capsule(pb[0], Tb, pa[0], pa[1], Ta, p2, p1);
  } else if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_BOX) {
    const double side[3] = {pb[0], pb[1], pb[2]};
    d = cf_sphere_box(pa[0], Ta, side, Tb, p1, p2);
  } else if (ta == MPG_GEOM_BOX && tb == MPG_GEOM_SPHERE) {
    const double side[3] = {pa[0], pa[1], pa[2]};
    d = cf_sphere_box(pb[0], Tb, side, Ta, p2, p1);
  } else if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_CYLINDER) {
    d = cf_sphere_cylinder(pa[0], Ta, pb[0], pb[1], Tb, p1, p2);
  } else if (ta == MPG_GEOM_CYLINDER && tb == MPG_GEOM_SPHERE) {
    d = cf_sphere_cylinder(pb[0], Tb, pa[0], pa[1], Ta, p2, p1);
  } else if (ta == MPG_GEOM_CAPSULE && tb == MPG_GEOM_CAPSULE) {
    d = cf_capsule_capsule(pa[0], pa[1], Ta, pb[0], pb[1], Tb, p1, p2);
  } else {
    return false;
  }
  if (d == -1.0) p1[0] = p1[1] = p1[2] = p2[0] = p2[1] = p2[2] = 0.0;
  q1 = V3{p1[0], p1[1], p1[2]};
  q2 = V3{p2[0], p2[1], p2[2]};
  return true;
}

// Project<S>::projectLine / projectTriangle and sphereTriangleDistance with
// points (oracle cf_project_line / cf_project_triangle / cf_sphere_triangle)
struct CfProj {
  double param[4], sqr_distance;
};
__device__ CfProj cf_project_line(const double* a, const double* b, const double* p) {
  CfProj r = {{0, 0, 0, 0}, -1.0};
  const double d[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  const double l = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
  if (l > 0) {
    const double pa[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
    const double t = (pa[0] * d[0] + pa[1] * d[1]) + pa[2] * d[2];
    r.param[1] = (t >= l) ? 1 : ((t <= 0) ? 0 : (t / l));
    r.param[0] = 1 - r.param[1];
    double v[3];
    if (t >= l) {
      for (int i = 0; i < 3; ++i) v[i] = p[i] - b[i];
    } else if (t <= 0) {
      for (int i = 0; i < 3; ++i) v[i] = p[i] - a[i];
    } else {
      for (int i = 0; i < 3; ++i) v[i] = (a[i] + d[i] * r.param[1]) - p[i];
    }
    r.sqr_distance = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
  }
  return r;
}
__device__ __forceinline__ void cf_cross(double* o, const double* a, const double* b) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ CfProj cf_project_triangle(const double* a, const double* b, const double* c, const double* p) {
  CfProj r = {{0, 0, 0, 0}, -1.0};
  const double* vt[3] = {a, b, c};
  double dl[3][3], n[3];
  for (int i = 0; i < 3; ++i) {
    dl[0][i] = a[i] - b[i];
    dl[1][i] = b[i] - c[i];
    dl[2][i] = c[i] - a[i];
  }
  cf_cross(n, dl[0], dl[1]);
  const double l = (n[0] * n[0] + n[1] * n[1]) + n[2] * n[2];
  if (l > 0) {
    double mindist = -1;
    for (int i = 0; i < 3; ++i) {
      double vp[3], dn[3];
      for (int k = 0; k < 3; ++k) vp[k] = vt[i][k] - p[k];
      cf_cross(dn, dl[i], n);
      if ((vp[0] * dn[0] + vp[1] * dn[1]) + vp[2] * dn[2] > 0) {
        const int j = i == 2 ? 0 : i + 1;
        const CfProj rl = cf_project_line(vt[i], vt[j], p);
        if (mindist < 0 || rl.sqr_distance < mindist) {
          mindist = rl.sqr_distance;
          r.param[i] = rl.param[0];
          r.param[j] = rl.param[1];
          r.param[j == 2 ? 0 : j + 1] = 0;
        }
      }
    }
    if (mindist < 0) {
      const double ap[3] = {a[0] - p[0], a[1] - p[1], a[2] - p[2]};
      const double d = (ap[0] * n[0] + ap[1] * n[1]) + ap[2] * n[2];
      const double s = std::sqrt(l);
      double pp[3], t1[3], t2[3], x[3];
      for (int k = 0; k < 3; ++k) pp[k] = n[k] * (d / l);
      mindist = (pp[0] * pp[0] + pp[1] * pp[1]) + pp[2] * pp[2];
      for (int k = 0; k < 3; ++k) t1[k] = (b[k] - p[k]) - pp[k];
      cf_cross(x, dl[1], t1);
      r.param[0] = cf_norm(x) / s;
      for (int k = 0; k < 3; ++k) t2[k] = (c[k] - p[k]) - pp[k];
      cf_cross(x, dl[2], t2);
      r.param[1] = cf_norm(x) / s;
      r.param[2] = 1 - r.param[0] - r.param[1];
    }
    r.sqr_distance = mindist;
  }
  return r;
}
// W: the triangle's world vertices [3][3]
__device__ double cf_sphere_triangle(double radius, const double* o, const double* W, double* pS, double* pT) {
  const CfProj r = cf_project_triangle(W, W + 3, W + 6, o);
  if (r.sqr_distance > radius * radius) {
    double pp[3], dir[3];
    for (int k = 0; k < 3; ++k) pp[k] = (W[k] * r.param[0] + W[3 + k] * r.param[1]) + W[6 + k] * r.param[2];
    for (int k = 0; k < 3; ++k) dir[k] = o[k] - pp[k];
    const double n = cf_norm(dir);
    for (int k = 0; k < 3; ++k) dir[k] /= n;
    for (int k = 0; k < 3; ++k) {
      pS[k] = o[k] - dir[k] * radius;
      pT[k] = pp[k];
    }
    return std::sqrt(r.sqr_distance) - radius;
  }
  return -1.0;
}

// lower-bound pruning slack (oracle mesh_dist_slack): a pair / leaf / triangle
// is skipped only when its bounding-volume lower bound is above the running
// minimum by more than the float support rounding of libccd's GJK objects
__device__ __forceinline__ double dist_slack(const double* pa, const double* pb) {
  return 1e-5 * (1.0 + std::fabs(pa[0]) + std::fabs(pa[1]) + std::fabs(pa[2]) + std::fabs(pb[0]) + std::fabs(pb[1]) +
                 std::fabs(pb[2]));
}

// fcl::distance(shape, OcTree) [ext FCL 0.7.0 OcTreeShapeDistanceRecurse]:
// shapeDistance(leaf box, box_tf, shape, tf) per occupied leaf in FCL's DFS
// order (Box-Sphere closed form, else GJKDistance), strict '<' -> the first
// minimum; points (leaf box, shape).  Leaves whose bounding sphere cannot be
// below `bound` (the group's running minimum) by the slack are skipped.
// Returns the pair's minimum (DBL_MAX if every leaf was skipped) or a
// kDist* sentinel status in st.
__device__ double octree_distance(const DevWorld& w, cptr<double> HV, int go, const SE3& TO, const GObj& S,
                                  const SE3& TS, const V3& cs, double rs, double bound, ccd_real tol, V3& pb, V3& ps,
                                  int& st) {
  const cptr<double> go_rec = w.geom_rec + G_STRIDE * go;
  const int l0 = (int)go_rec[G_PARAM], ln = (int)go_rec[G_PARAM + 1];
  const bool sphere = S.type == MPG_GEOM_SPHERE;
  const double rsph = w.geom_rec[G_STRIDE * S.geom + G_PARAM];
  const double slack = dist_slack(TO.p, TS.p);
  GObj A;
  A.rot = gjk_rot_from_matrix(TO.R);
  A.rot_inv = quat_invert2(A.rot);
  A.geom = go;
  A.type = MPG_GEOM_BOX;
  double best = DBL_MAX;
  pb = ps = V3{0, 0, 0};
  for (int l = l0; l < l0 + ln && best != -1.0; ++l) {
    const cptr<double> L = w.oct_leaf + 6 * (size_t)l;
    double c[3], side[3], cw[3];
    for (int i = 0; i < 3; ++i) {
      c[i] = (L[i] + L[3 + i]) * 0.5;
      side[i] = L[3 + i] - L[i];
    }
    for (int i = 0; i < 3; ++i) cw[i] = ((TO.R[3 * i] * c[0] + TO.R[3 * i + 1] * c[1]) + TO.R[3 * i + 2] * c[2]) + TO.p[i];
    const double dx = cw[0] - cs.x, dy = cw[1] - cs.y, dz = cw[2] - cs.z;
    const double rl = 0.5 * std::sqrt((side[0] * side[0] + side[1] * side[1]) + side[2] * side[2]) * (1.0 + 1e-9) + 1e-9;
    if (std::sqrt(dx * dx + dy * dy + dz * dz) - rs - rl > fmin(best, bound) + slack) continue;
    double d;
    V3 qb{0, 0, 0}, qs{0, 0, 0};
    if (sphere) {
      SE3 TL;
      for (int k = 0; k < 9; ++k) TL.R[k] = TO.R[k];
      for (int k = 0; k < 3; ++k) TL.p[k] = cw[k];
      double a1[3], a2[3];
      d = cf_sphere_box(rsph, TS, side, TL, a2, a1);
      if (d != -1.0) {
        qb = V3{a1[0], a1[1], a1[2]};
        qs = V3{a2[0], a2[1], a2[2]};
      }
    } else {
      GObj A1 = A;
      A1.pos = cv3(cw[0], cw[1], cw[2]);
      const ccd_real h[3] = {(ccd_real)(side[0] / 2.0), (ccd_real)(side[1] / 2.0), (ccd_real)(side[2] / 2.0)};
      auto sup = [&](const CV3& dir) { return csup_box(A1, h, w, HV, S, dir); };
      ccd_real df;
      CV3 c1, c2;
      const int r = ccdx::gjk_distance<false>(sup, tol, (ccdx::Polytope*)nullptr, df, c1, c2);
      if (r != ccdx::kOk) {
        st = r == ccdx::kThrow ? kDistThrow : kDistOverflow;
        return DBL_MAX;
      }
      d = df;
      qb = to_v3(c1);
      qs = to_v3(c2);
    }
    if (d < best) {
      best = d;
      pb = qb;
      ps = qs;
    }
  }
  return best;
}

__device__ __forceinline__ GObj pose_obj(const DevWorld& w, const double* __restrict__ poses, long long n, long long cfg,
                                         int id, V3& c) {
  if (id < w.n_moving) {
    const double* g = poses + ((size_t)id * kPoseStride) * n + cfg;
    GObj o;
    o.rot = CQ4{(ccd_real)g[0], (ccd_real)g[n], (ccd_real)g[2 * n], (ccd_real)g[3 * n]};
    o.rot_inv = quat_invert2(o.rot);
    o.pos = cv3(g[4 * n], g[5 * n], g[6 * n]);
    o.geom = w.moving_geom[id];
    o.type = w.geom_type[o.geom];
    c = v3(g[7 * n], g[8 * n], g[9 * n]);
    return o;
  }
  const int sid = id - w.n_moving;
  const cptr<double> r = w.static_rec + S_STRIDE * sid;
  c = v3(r[S_OBBC], r[S_OBBC + 1], r[S_OBBC + 2]);
  return static_obj(w, sid);
}

// fp64 transform of object `id` for configuration cfg (pose_kernel fields)
__device__ __forceinline__ SE3 pose_se3(const DevWorld& w, const double* __restrict__ poses, long long n, long long cfg,
                                        int id) {
  if (id >= w.n_moving) return load_se3(w.static_T + 12 * (id - w.n_moving));
  const double* g = poses + ((size_t)id * kPoseStride) * n + cfg;
  SE3 T;
#pragma unroll
  for (int i = 0; i < 9; ++i) T.R[i] = g[(10 + i) * n];
#pragma unroll
  for (int i = 0; i < 3; ++i) T.p[i] = g[(4 + i) * n];
  return T;
}

// ---------------------------------------------------------------------------
// Distance with BVH meshes (fcl::distance on BVHModel<OBBRSS>, FCL 0.7.0):
//   mesh-shape   MeshShapeDistanceTraversalNodeOBBRSS: min over triangles of
//                shapeTriangleDistance(shape, tf, P1, P2, P3, tf_mesh) (GJK,
//                shape first; -1 once one intersects)
//   mesh-mesh    MeshDistanceTraversalNodeOBBRSS: min of triDistance over the
//                triangle pairs, B's triangles in A's frame (0 if one pair
//                intersects)
//   mesh-OcTree  OcTreeMeshDistanceRecurse: min over (leaf box, triangle) of
//                shapeTriangleDistance(box, box_tf, ...), box first
// The traversal only skips what cannot lower the running minimum; here the
// cluster and triangle boxes are skipped when their lower bound exceeds the
// running minimum by more than the float support rounding (dist_slack).  One
// lane per configuration, as distance_kernel.
// ---------------------------------------------------------------------------

// distance from point c to the box [lo, hi]
__device__ __forceinline__ double point_box_distance(const double* c, const double* lo, const double* hi) {
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double e = fmax(fmax(lo[i] - c[i], c[i] - hi[i]), 0.0);
    s += e * e;
  }
  return std::sqrt(s);
}

// PQP TriDist as FCL's TriangleDistance::segPoints / triDistance (oracle
// seg_points / tri_face_case / tri_distance, same operation order)
__device__ void seg_points(const double* P, const double* A, const double* Q, const double* B, double* VEC, double* X,
                           double* Y) {
  double T[3], TMP[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) T[k] = Q[k] - P[k];
  const double AA = d3(A, A), BB = d3(B, B), AB = d3(A, B), AT = d3(A, T), BT = d3(B, T);
  const double denom = AA * BB - AB * AB;
  double t = (AT * BB - BT * AB) / denom;
  if (t < 0 || std::isnan(t)) t = 0;
  else if (t > 1) t = 1;
  const double u = (t * AB - BT) / BB;
  if (u <= 0 || std::isnan(u)) {
    for (int k = 0; k < 3; ++k) Y[k] = Q[k];
    t = AT / AA;
    if (t <= 0 || std::isnan(t)) {
      for (int k = 0; k < 3; ++k) {
        X[k] = P[k];
        VEC[k] = Q[k] - P[k];
      }
    } else if (t >= 1) {
      for (int k = 0; k < 3; ++k) {
        X[k] = P[k] + A[k];
        VEC[k] = Q[k] - X[k];
      }
    } else {
      for (int k = 0; k < 3; ++k) X[k] = P[k] + A[k] * t;
      c3(TMP, T, A);
      c3(VEC, A, TMP);
    }
  } else if (u >= 1) {
    for (int k = 0; k < 3; ++k) Y[k] = Q[k] + B[k];
    t = (AB + AT) / AA;
    if (t <= 0 || std::isnan(t)) {
      for (int k = 0; k < 3; ++k) {
        X[k] = P[k];
        VEC[k] = Y[k] - P[k];
      }
    } else if (t >= 1) {
      for (int k = 0; k < 3; ++k) {
        X[k] = P[k] + A[k];
        VEC[k] = Y[k] - X[k];
      }
    } else {
      for (int k = 0; k < 3; ++k) {
        X[k] = P[k] + A[k] * t;
        T[k] = Y[k] - P[k];
      }
      c3(TMP, T, A);
      c3(VEC, A, TMP);
    }
  } else {
    for (int k = 0; k < 3; ++k) Y[k] = Q[k] + B[k] * u;
    if (t <= 0 || std::isnan(t)) {
      for (int k = 0; k < 3; ++k) X[k] = P[k];
      c3(TMP, T, B);
      c3(VEC, B, TMP);
    } else if (t >= 1) {
      for (int k = 0; k < 3; ++k) {
        X[k] = P[k] + A[k];
        T[k] = Q[k] - X[k];
      }
      c3(TMP, T, B);
      c3(VEC, B, TMP);
    } else {
      for (int k = 0; k < 3; ++k) X[k] = P[k] + A[k] * t;
      c3(VEC, A, B);
      if (d3(VEC, T) < 0)
        for (int k = 0; k < 3; ++k) VEC[k] = -VEC[k];
    }
  }
}

// Pf: the projection of T's closest vertex on S's face, Qf: that vertex
__device__ bool tri_face_case(const double* S, const double* Sv, const double* T, bool& disjoint, double& dist,
                              double* Pf, double* Qf) {
  double Sn[3], V[3], Z[3], Tp[3];
  c3(Sn, Sv, Sv + 3);
  const double Snl = d3(Sn, Sn);
  if (!(Snl > 1e-15)) return false;
  for (int i = 0; i < 3; ++i) {
    for (int k = 0; k < 3; ++k) V[k] = S[k] - T[3 * i + k];
    Tp[i] = d3(V, Sn);
  }
  int point = -1;
  if (Tp[0] > 0 && Tp[1] > 0 && Tp[2] > 0) {
    point = Tp[0] < Tp[1] ? 0 : 1;
    if (Tp[2] < Tp[point]) point = 2;
  } else if (Tp[0] < 0 && Tp[1] < 0 && Tp[2] < 0) {
    point = Tp[0] > Tp[1] ? 0 : 1;
    if (Tp[2] > Tp[point]) point = 2;
  }
  if (point < 0) return false;
  disjoint = true;
  for (int e = 0; e < 3; ++e) {
    for (int k = 0; k < 3; ++k) V[k] = T[3 * point + k] - S[3 * e + k];
    c3(Z, Sn, Sv + 3 * e);
    if (!(d3(V, Z) > 0)) return false;
  }
  double D[3];
  const double s = Tp[point] / Snl;
  for (int k = 0; k < 3; ++k) {
    Pf[k] = T[3 * point + k] + Sn[k] * s;
    Qf[k] = T[3 * point + k];
    D[k] = Pf[k] - Qf[k];
  }
  dist = std::sqrt(d3(D, D));
  return true;
}

// TriangleDistance::triDistance(S, T, P, Q) (oracle tri_distance_pq); S, T:
// 3 vertices each, row-major [3][3]; P, Q zero when they intersect
__device__ double tri_distance_pq(const double* S, const double* T, double* P, double* Q) {
  double Sv[9], Tv[9], VEC[3], Pc[3], Qc[3], V[3], Z[3], minP[3] = {0, 0, 0}, minQ[3] = {0, 0, 0};
  for (int k = 0; k < 3; ++k) {
    Sv[k] = S[3 + k] - S[k];
    Sv[3 + k] = S[6 + k] - S[3 + k];
    Sv[6 + k] = S[k] - S[6 + k];
    Tv[k] = T[3 + k] - T[k];
    Tv[3 + k] = T[6 + k] - T[3 + k];
    Tv[6 + k] = T[k] - T[6 + k];
    P[k] = 0.0;
    Q[k] = 0.0;
  }
  bool shown_disjoint = false;
  for (int k = 0; k < 3; ++k) V[k] = S[k] - T[k];
  double mindd = d3(V, V) + 1;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      seg_points(S + 3 * i, Sv + 3 * i, T + 3 * j, Tv + 3 * j, VEC, Pc, Qc);
      for (int k = 0; k < 3; ++k) V[k] = Qc[k] - Pc[k];
      const double dd = d3(V, V);
      if (dd <= mindd) {
        for (int k = 0; k < 3; ++k) {
          minP[k] = Pc[k];
          minQ[k] = Qc[k];
        }
        mindd = dd;
        const int i2 = (i + 2) % 3, j2 = (j + 2) % 3;
        for (int k = 0; k < 3; ++k) Z[k] = S[3 * i2 + k] - Pc[k];
        double a = d3(Z, VEC);
        for (int k = 0; k < 3; ++k) Z[k] = T[3 * j2 + k] - Qc[k];
        double b = d3(Z, VEC);
        if (a <= 0 && b >= 0) {
          for (int k = 0; k < 3; ++k) {
            P[k] = Pc[k];
            Q[k] = Qc[k];
          }
          return std::sqrt(dd);
        }
        const double p = d3(V, VEC);
        if (a < 0) a = 0;
        if (b > 0) b = 0;
        if (p - a + b > 0) shown_disjoint = true;
      }
    }
  double d;
  if (tri_face_case(S, Sv, T, shown_disjoint, d, P, Q)) return d;
  if (tri_face_case(T, Tv, S, shown_disjoint, d, Q, P)) return d;
  if (shown_disjoint) {
    for (int k = 0; k < 3; ++k) {
      P[k] = minP[k];
      Q[k] = minQ[k];
    }
    return std::sqrt(mindd);
  }
  return 0.0;
}

__device__ __forceinline__ GObj mesh_frame_obj(int gm, const SE3& TM) {
  GObj B;
  B.rot = gjk_rot_from_matrix(TM.R);
  B.rot_inv = quat_invert2(B.rot);
  B.pos = cv3(TM.p[0], TM.p[1], TM.p[2]);
  B.geom = gm;
  B.type = MPG_GEOM_MESH;
  return B;
}

// point p (world) in the frame T
__device__ __forceinline__ void to_frame(const SE3& T, const double* p, double* o) {
  const double d[3] = {p[0] - T.p[0], p[1] - T.p[1], p[2] - T.p[2]};
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = (T.R[i] * d[0] + T.R[3 + i] * d[1]) + T.R[6 + i] * d[2];
}

// mesh-shape (MeshShapeDistanceTraversalNodeOBBRSS leaf): the minimum over
// the triangles of shapeTriangleDistance(shape, tf, P1, P2, P3, tf_mesh)
// (sphereTriangleDistance for spheres, else GJKDistance with the shape first),
// points (mesh, shape).  Triangles are met in cluster order; ties go to the
// lower triangle index, as the oracle's index-order scan with strict '<'.
// Clusters / triangles whose lower bound is above min(own minimum, bound) by
// the slack are skipped.  DBL_MAX when everything was skipped.
__device__ double mesh_shape_distance_lane(const DevWorld& w, cptr<double> HV, int gm, const SE3& TM, const GObj& S,
                                           const SE3& TS, double bound, ccd_real tol, V3& pm, V3& ps, int& st) {
  const cptr<double> grs = w.geom_rec + G_STRIDE * S.geom;
  double cs[3], csm[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    cs[i] = ((TS.R[3 * i] * grs[G_OBB_C] + TS.R[3 * i + 1] * grs[G_OBB_C + 1]) + TS.R[3 * i + 2] * grs[G_OBB_C + 2]) + TS.p[i];
  to_frame(TM, cs, csm);
  const double rs = grs[G_RADIUS], slack = dist_slack(TM.p, TS.p);
  const bool sphere = S.type == MPG_GEOM_SPHERE;
  const GObj B = mesh_frame_obj(gm, TM);
  const int c0 = w.mesh_tree[2 * gm], c1 = c0 + w.mesh_tree[2 * gm + 1];
  double best = DBL_MAX;
  int best_id = INT_MAX;
  pm = ps = V3{0, 0, 0};
  for (int cl = c0; cl < c1 && best != -1.0; ++cl) {
    const cptr<double> bx = w.mesh_node + 6 * (size_t)cl;
    const double lo[3] = {bx[0], bx[1], bx[2]}, hi[3] = {bx[3], bx[4], bx[5]};
    if (point_box_distance(csm, lo, hi) - rs > fmin(best, bound) + slack) continue;
    const int t1 = w.mesh_link[2 * cl] + w.mesh_link[2 * cl + 1];
    for (int t = w.mesh_link[2 * cl]; t < t1 && best != -1.0; ++t) {
      const cptr<double> rec = w.mesh_tri + TR_STRIDE * (size_t)t;
      const double tlo[3] = {rec[TR_LO], rec[TR_LO + 1], rec[TR_LO + 2]}, thi[3] = {rec[TR_HI], rec[TR_HI + 1], rec[TR_HI + 2]};
      if (point_box_distance(csm, tlo, thi) - rs > fmin(best, bound) + slack) continue;
      const int id = (int)rec[TR_ID];
      double P[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) P[k] = rec[TR_P + k];
      double d;
      V3 qm{0, 0, 0}, qs{0, 0, 0};
      if (sphere) {
        double W[9], a1[3], a2[3];
        for (int v = 0; v < 3; ++v)
          for (int i = 0; i < 3; ++i)
            W[3 * v + i] = ((TM.R[3 * i] * P[3 * v] + TM.R[3 * i + 1] * P[3 * v + 1]) + TM.R[3 * i + 2] * P[3 * v + 2]) + TM.p[i];
        d = cf_sphere_triangle(grs[G_PARAM], TS.p, W, a1, a2);
        if (d != -1.0) {
          qs = V3{a1[0], a1[1], a1[2]};
          qm = V3{a2[0], a2[1], a2[2]};
        }
      } else {
        const CV3 tc = cv3((P[0] + P[3] + P[6]) / 3, (P[1] + P[4] + P[7]) / 3, (P[2] + P[5] + P[8]) / 3);
        const CV3 TP[3] = {cv3(P[0], P[1], P[2]), cv3(P[3], P[4], P[5]), cv3(P[6], P[7], P[8])};
        auto sup = [&](const CV3& dir) { return csup_tri(w, HV, S, B, TP, tc, dir); };
        ccd_real df;
        CV3 c1, c2;
        const int r = ccdx::gjk_distance<false>(sup, tol, (ccdx::Polytope*)nullptr, df, c1, c2);
        if (r != ccdx::kOk) {
          st = r == ccdx::kThrow ? kDistThrow : kDistOverflow;
          return DBL_MAX;
        }
        d = df;
        qs = to_v3(c1);
        qm = to_v3(c2);
      }
      if (d < best || (d == best && id < best_id)) {
        best = d;
        best_id = id;
        pm = qm;
        ps = qs;
      }
    }
  }
  return best;
}

// mesh-mesh (MeshDistanceTraversalNodeOBBRSS): the minimum of triDistance
// over the triangle pairs, B's triangles in A's frame; 0 once a pair
// intersects (zero points); points (A, B) in A's frame -> world.  Ties go to
// the lexicographically lower (A index, B index), the oracle's scan order.
__device__ double mesh_mesh_distance_lane(const DevWorld& w, int ga, const SE3& TA, int gb, const SE3& TB, double bound,
                                          V3& pa, V3& pb) {
  double R[9], T[3];
  const double dt[3] = {TB.p[0] - TA.p[0], TB.p[1] - TA.p[1], TB.p[2] - TA.p[2]};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) R[3 * i + j] = (TA.R[i] * TB.R[j] + TA.R[3 + i] * TB.R[3 + j]) + TA.R[6 + i] * TB.R[6 + j];
    T[i] = (TA.R[i] * dt[0] + TA.R[3 + i] * dt[1]) + TA.R[6 + i] * dt[2];
  }
  const double slack = dist_slack(TA.p, TB.p);
  const int a0 = w.mesh_tree[2 * ga], a1 = a0 + w.mesh_tree[2 * ga + 1];
  const int b0 = w.mesh_tree[2 * gb], b1 = b0 + w.mesh_tree[2 * gb + 1];
  double best = DBL_MAX, bP[3] = {0, 0, 0}, bQ[3] = {0, 0, 0};
  long long best_key = LLONG_MAX;
  for (int cb = b0; cb < b1 && best != 0.0; ++cb) {
    const cptr<double> bb = w.mesh_node + 6 * (size_t)cb;
    double cc[3], cca[3], e2 = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      cc[k] = (bb[k] + bb[3 + k]) * 0.5;
      e2 += (bb[3 + k] - bb[k]) * (bb[3 + k] - bb[k]);
    }
    const double rb = 0.5 * std::sqrt(e2) * (1.0 + 1e-9) + 1e-9;
#pragma unroll
    for (int i = 0; i < 3; ++i) cca[i] = ((R[3 * i] * cc[0] + R[3 * i + 1] * cc[1]) + R[3 * i + 2] * cc[2]) + T[i];
    for (int ca = a0; ca < a1 && best != 0.0; ++ca) {
      const cptr<double> ba = w.mesh_node + 6 * (size_t)ca;
      const double lo[3] = {ba[0], ba[1], ba[2]}, hi[3] = {ba[3], ba[4], ba[5]};
      if (point_box_distance(cca, lo, hi) - rb > fmin(best, bound) + slack) continue;
      const int tb1 = w.mesh_link[2 * cb] + w.mesh_link[2 * cb + 1];
      for (int tb = w.mesh_link[2 * cb]; tb < tb1 && best != 0.0; ++tb) {
        const cptr<double> rq = w.mesh_tri + TR_STRIDE * (size_t)tb;
        double Q[9], qc[3], qr = 0.0;
#pragma unroll
        for (int v = 0; v < 3; ++v)
#pragma unroll
          for (int i = 0; i < 3; ++i)
            Q[3 * v + i] = ((R[3 * i] * rq[3 * v] + R[3 * i + 1] * rq[3 * v + 1]) + R[3 * i + 2] * rq[3 * v + 2]) + T[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) qc[i] = (Q[i] + Q[3 + i] + Q[6 + i]) / 3.0;
#pragma unroll
        for (int v = 0; v < 3; ++v) {
          const double dx = Q[3 * v] - qc[0], dy = Q[3 * v + 1] - qc[1], dz = Q[3 * v + 2] - qc[2];
          qr = fmax(qr, dx * dx + dy * dy + dz * dz);
        }
        qr = std::sqrt(qr) * (1.0 + 1e-9) + 1e-9;
        if (point_box_distance(qc, lo, hi) - qr > fmin(best, bound) + slack) continue;
        const long long idb = (long long)rq[TR_ID];
        const int ta1 = w.mesh_link[2 * ca] + w.mesh_link[2 * ca + 1];
        for (int ta = w.mesh_link[2 * ca]; ta < ta1; ++ta) {
          const cptr<double> rp = w.mesh_tri + TR_STRIDE * (size_t)ta;
          const double tlo[3] = {rp[TR_LO], rp[TR_LO + 1], rp[TR_LO + 2]}, thi[3] = {rp[TR_HI], rp[TR_HI + 1], rp[TR_HI + 2]};
          if (point_box_distance(qc, tlo, thi) - qr > fmin(best, bound) + slack) continue;
          double P[9], Pp[3], Qq[3];
#pragma unroll
          for (int k = 0; k < 9; ++k) P[k] = rp[TR_P + k];
          const double d = tri_distance_pq(P, Q, Pp, Qq);
          const long long key = ((long long)rp[TR_ID] << 32) | idb;
          if (d < best || (d == best && key < best_key)) {
            best = d;
            best_key = key;
            for (int k = 0; k < 3; ++k) {
              bP[k] = Pp[k];
              bQ[k] = Qq[k];
            }
          }
          if (best == 0.0) break;
        }
      }
    }
  }
  double wa[3], wb[3];
  cf_tf_point(TA, bP, wa);
  cf_tf_point(TA, bQ, wb);
  pa = V3{wa[0], wa[1], wa[2]};
  pb = V3{wb[0], wb[1], wb[2]};
  return best;
}

// mesh-OcTree (OcTreeMeshDistanceRecurse): the minimum over (occupied leaf,
// triangle) of shapeTriangleDistance(Box(leaf), box_tf, triangle) (GJK, leaf
// box first); points (box, triangle); ties to the earlier leaf, then the
// lower triangle index, as the oracle's leaf-major scan
__device__ double mesh_octree_distance_lane(const DevWorld& w, int gm, const SE3& TM, int go, const SE3& TO, double bound,
                                            ccd_real tol, V3& pbox, V3& ptri, int& st) {
  const cptr<double> grm = w.geom_rec + G_STRIDE * gm, go_rec = w.geom_rec + G_STRIDE * go;
  const int l0 = (int)go_rec[G_PARAM], ln = (int)go_rec[G_PARAM + 1];
  double mcw[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    mcw[i] = ((TM.R[3 * i] * grm[G_OBB_C] + TM.R[3 * i + 1] * grm[G_OBB_C + 1]) + TM.R[3 * i + 2] * grm[G_OBB_C + 2]) + TM.p[i];
  const double rm = grm[G_RADIUS], slack = dist_slack(TM.p, TO.p);
  const GObj B = mesh_frame_obj(gm, TM);
  GObj A;
  A.rot = gjk_rot_from_matrix(TO.R);
  A.rot_inv = quat_invert2(A.rot);
  A.geom = go;
  A.type = MPG_GEOM_BOX;
  const int c0 = w.mesh_tree[2 * gm], c1 = c0 + w.mesh_tree[2 * gm + 1];
  double best = DBL_MAX;
  int best_id = INT_MAX;
  pbox = ptri = V3{0, 0, 0};
  for (int l = l0; l < l0 + ln && best != -1.0; ++l) {
    const cptr<double> L = w.oct_leaf + 6 * (size_t)l;
    double c[3], side[3], cw[3], cm[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      c[i] = (L[i] + L[3 + i]) * 0.5;
      side[i] = L[3 + i] - L[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) cw[i] = ((TO.R[3 * i] * c[0] + TO.R[3 * i + 1] * c[1]) + TO.R[3 * i + 2] * c[2]) + TO.p[i];
    const double rl = 0.5 * std::sqrt((side[0] * side[0] + side[1] * side[1]) + side[2] * side[2]) * (1.0 + 1e-9) + 1e-9;
    const double dx = cw[0] - mcw[0], dy = cw[1] - mcw[1], dz = cw[2] - mcw[2];
    if (std::sqrt(dx * dx + dy * dy + dz * dz) - rl - rm > fmin(best, bound) + slack) continue;
    to_frame(TM, cw, cm);
    GObj A1 = A;
    A1.pos = cv3(cw[0], cw[1], cw[2]);
    const ccd_real h[3] = {(ccd_real)(side[0] / 2.0), (ccd_real)(side[1] / 2.0), (ccd_real)(side[2] / 2.0)};
    const double leaf_best = best;  // a later leaf wins only when strictly below the earlier leaves
    for (int cl = c0; cl < c1 && best != -1.0; ++cl) {
      const cptr<double> bx = w.mesh_node + 6 * (size_t)cl;
      const double lo[3] = {bx[0], bx[1], bx[2]}, hi[3] = {bx[3], bx[4], bx[5]};
      if (point_box_distance(cm, lo, hi) - rl > fmin(best, bound) + slack) continue;
      const int t1 = w.mesh_link[2 * cl] + w.mesh_link[2 * cl + 1];
      for (int t = w.mesh_link[2 * cl]; t < t1 && best != -1.0; ++t) {
        const cptr<double> rec = w.mesh_tri + TR_STRIDE * (size_t)t;
        const double tlo[3] = {rec[TR_LO], rec[TR_LO + 1], rec[TR_LO + 2]}, thi[3] = {rec[TR_HI], rec[TR_HI + 1], rec[TR_HI + 2]};
        if (point_box_distance(cm, tlo, thi) - rl > fmin(best, bound) + slack) continue;
        const int id = (int)rec[TR_ID];
        double P[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) P[k] = rec[TR_P + k];
        const CV3 tc = cv3((P[0] + P[3] + P[6]) / 3, (P[1] + P[4] + P[7]) / 3, (P[2] + P[5] + P[8]) / 3);
        const CV3 TP[3] = {cv3(P[0], P[1], P[2]), cv3(P[3], P[4], P[5]), cv3(P[6], P[7], P[8])};
        auto sup = [&](const CV3& dir) { return csup_box_tri(A1, h, B, TP, tc, dir); };
        ccd_real df;
        CV3 q1, q2;
        const int r = ccdx::gjk_distance<false>(sup, tol, (ccdx::Polytope*)nullptr, df, q1, q2);
        if (r != ccdx::kOk) {
          st = r == ccdx::kThrow ? kDistThrow : kDistOverflow;
          return DBL_MAX;
        }
        const double d = df;
        // within this leaf: the lower triangle index among equals; against
        // earlier leaves: strictly below
        if (d < leaf_best && (d < best || (d == best && id < best_id))) {
          best = d;
          best_id = id;
          pbox = to_v3(q1);
          ptri = to_v3(q2);
        }
      }
    }
  }
  return best;
}

// (MODE bit) PTS: write the nearest points; SIGNED: enable_signed_distance;
// NP: enable_nearest_points (mesh-mesh points, the (shape, mesh) swap)
// INDEP: DistanceRequest(gjk_solver_type=GST_INDEP), unsigned shape pairs only
constexpr int MPG_DIST_POINTS = 1, MPG_DIST_SIGNED = 2, MPG_DIST_NP = 4, MPG_DIST_INDEP = 8;
constexpr int kBigPool = 16;  // big EPA polytopes per world (distance_redo_kernel)

// Per configuration, every non-allowed pair in order with the group's strict
// '<' (planning_world.cpp:513): fcl::distance with DistanceRequest's options
// (oracle/collide_oracle.c pair_distance: which algorithm each pair kind runs
// and which point is which).  Shape pairs whose bounding spheres are apart
// by more than the running minimum plus the slack are skipped (their GJK
// value cannot be below it).  A configuration on which FCL throws
// (p = kDistThrow) or whose EPA outgrows the polytope arrays (p =
// kDistOverflow) gets NaN distances in both groups.
// PT: the signed instances' EPA polytope type; ptp its storage (private in
// distance_kernel, a global pool slot in distance_redo_kernel).
template <int MODE, class PT>
__device__ __forceinline__ void distance_config(const DevWorld& w, const double* __restrict__ poses, long long n,
                                                long long cfg, bool live, int n_self, ccd_real tol, double dtol,
                                                PT* ptp, double* __restrict__ d_self, int32_t* __restrict__ p_self,
                                                double* __restrict__ d_others, int32_t* __restrict__ p_others,
                                                double* __restrict__ pts_self, double* __restrict__ pts_others) {
  constexpr bool SIGNED = (MODE & MPG_DIST_SIGNED) != 0;
  constexpr bool PTS = (MODE & MPG_DIST_POINTS) != 0;
  constexpr bool NP = (MODE & MPG_DIST_NP) != 0;
  constexpr bool INDEP = (MODE & MPG_DIST_INDEP) != 0;
  static_assert(!(INDEP && SIGNED), "GST_INDEP signed distance (FCL's EPA) is not restated");
  const cptr<double> HV = w.hull;
  double best[2] = {DBL_MAX, DBL_MAX};
  int bp[2] = {-1, -1};
  V3 bpt[2][2] = {{{0, 0, 0}, {0, 0, 0}}, {{0, 0, 0}, {0, 0, 0}}};
  int st = 0;
  for (int p = 0; p < w.n_pairs && !st; ++p) {
    if (w.pair_allowed[p]) continue;  // ACM before distance (planning_world.cpp:509-510)
    const int g = p < n_self ? 0 : 1;
    const int a = w.pair_a[p], b = w.pair_b[p];
    V3 ca, cb;
    const GObj A = pose_obj(w, poses, n, cfg, a, ca);
    const GObj B = pose_obj(w, poses, n, cfg, b, cb);
    const double ra = w.geom_rec[G_STRIDE * A.geom + G_RADIUS], rb = w.geom_rec[G_STRIDE * B.geom + G_RADIUS];
    double d = DBL_MAX;
    V3 q1{0, 0, 0}, q2{0, 0, 0};
    if (w.pair_cf[p] == CF_MESH) {  // mesh pairs report unsigned values, never below -1
      if (!live || best[g] <= -1.0) continue;
      const SE3 TA = pose_se3(w, poses, n, cfg, a), TB = pose_se3(w, poses, n, cfg, b);
      if (A.type == MPG_GEOM_MESH && B.type == MPG_GEOM_MESH) {
        d = mesh_mesh_distance_lane(w, A.geom, TA, B.geom, TB, best[g], q1, q2);
        if (!NP) q1 = q2 = V3{0, 0, 0};
      } else if (A.type == MPG_GEOM_OCTREE) {
        d = mesh_octree_distance_lane(w, B.geom, TB, A.geom, TA, best[g], tol, q1, q2, st);
      } else if (B.type == MPG_GEOM_OCTREE) {
        d = mesh_octree_distance_lane(w, A.geom, TA, B.geom, TB, best[g], tol, q1, q2, st);
      } else if (A.type == MPG_GEOM_MESH) {
        d = mesh_shape_distance_lane(w, HV, A.geom, TA, B, TB, best[g], tol, q1, q2, st);
      } else {
        V3 pm, ps;
        d = mesh_shape_distance_lane(w, HV, B.geom, TB, A, TA, best[g], tol, pm, ps, st);
        q1 = NP ? ps : pm;  // distance() swaps the points back with enable_nearest_points
        q2 = NP ? pm : ps;
      }
    } else if (w.pair_cf[p] == CF_OCTREE) {  // leaf box first whatever the order; unsigned
      if (!live || best[g] <= -1.0) continue;
      const bool oa = A.type == MPG_GEOM_OCTREE;
      const SE3 TO = pose_se3(w, poses, n, cfg, oa ? a : b);  // static, or riding on a link / attached body
      const SE3 TS = pose_se3(w, poses, n, cfg, oa ? b : a);
      d = oa ? octree_distance(w, HV, A.geom, TO, B, TS, cb, rb, best[g], tol, q1, q2, st)
             : octree_distance(w, HV, B.geom, TO, A, TS, ca, ra, best[g], tol, q1, q2, st);
    } else {
      if (!live) continue;
      const V3 dc = vsub(cb, ca);
      const double lb = std::sqrt(d3dot(dc, dc)) - ra - rb - 1e-9;
      const double slack = dist_slack(&ca.x, &cb.x);
      // with signed distances a pair is skipped only when its shapes are
      // apart: an intersecting pair reaches EPA, which can throw
      // (FCL_THROW_FAILED_AT_THIS_CONFIGURATION) however deep the running
      // minimum already is, and FCL runs every pair (planning_world.cpp:509-537)
      if (lb > best[g] + slack && (!SIGNED || lb > slack)) continue;
      bool done = false;
      if constexpr (!SIGNED) {
        const SE3 TA = pose_se3(w, poses, n, cfg, a), TB = pose_se3(w, poses, n, cfg, b);
        done = cf_shape_distance(w, A.geom, A.type, TA, B.geom, B.type, TB, d, q1, q2);
        if constexpr (INDEP) {  // FCL's own GJK in double (the same closed forms first)
          if (!done) d = gjk_indep_distance(w, HV, A.geom, TA, B.geom, TB, dtol, q1, q2);
          done = true;
        }
      }
      if (!done) {
        auto sup = [&](const CV3& dir) { return csup(w, HV, A, B, dir); };
        ccd_real df;
        CV3 c1, c2;
        const int r = ccdx::gjk_distance<SIGNED>(sup, tol, ptp, df, c1, c2);
        if (r != ccdx::kOk) st = r == ccdx::kThrow ? kDistThrow : kDistOverflow;
        d = df;
        q1 = to_v3(c1);
        q2 = to_v3(c2);
      }
    }
    if (st) break;
    if (d < best[g]) {
      best[g] = d;
      bp[g] = p;
      if constexpr (PTS) {
        bpt[g][0] = q1;
        bpt[g][1] = q2;
      }
    }
  }
  if (!live) return;
  if (st) {
    best[0] = best[1] = __longlong_as_double(0x7ff8000000000000ll);
    bp[0] = bp[1] = st;
  }
  d_self[cfg] = best[0];
  p_self[cfg] = bp[0];
  d_others[cfg] = best[1];
  p_others[cfg] = bp[1];
  if constexpr (PTS) {
    for (int g = 0; g < 2; ++g) {
      double* o = (g ? pts_others : pts_self) + 6 * cfg;
      o[0] = bpt[g][0].x;
      o[1] = bpt[g][0].y;
      o[2] = bpt[g][0].z;
      o[3] = bpt[g][1].x;
      o[4] = bpt[g][1].y;
      o[5] = bpt[g][1].z;
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(128) void distance_kernel(DevWorld w, const double* __restrict__ poses, long long n,
                                                       int n_self, ccd_real tol, double dtol,
                                                       double* __restrict__ d_self, int32_t* __restrict__ p_self,
                                                       double* __restrict__ d_others, int32_t* __restrict__ p_others,
                                                       double* __restrict__ pts_self, double* __restrict__ pts_others) {
  constexpr bool SIGNED = (MODE & MPG_DIST_SIGNED) != 0;
  const long long cfg0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = cfg0 < n;
  const long long cfg = live ? cfg0 : n - 1;
  struct NoPolytope {};
  std::conditional_t<SIGNED, ccdx::Polytope, NoPolytope> polytope;
  ccdx::Polytope* ptp = nullptr;
  if constexpr (SIGNED) ptp = &polytope;
  distance_config<MODE>(w, poses, n, cfg, live, n_self, tol, dtol, ptp, d_self, p_self, d_others, p_others, pts_self,
                        pts_others);
}

// Signed instances only: the configurations distance_kernel left at
// kDistOverflow (an EPA past kPtV vertices; rare -- 29 at most on the parity
// batches, 124 for a sphere deep in a sphere) are listed (overflow_list_kernel:
// list[0] = count, ids after it; the count zeroed by the host), then evaluated
// again from the start by kBigPool lanes, lane k with the k-th kBigPtV-vertex
// polytope of `pool`, taking every kBigPool-th listed configuration.
__global__ __launch_bounds__(256) void overflow_list_kernel(const int32_t* __restrict__ p_self, long long n,
                                                            unsigned* __restrict__ list) {
  const long long cfg = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (cfg < n && p_self[cfg] == kDistOverflow) list[1 + atomicAdd(&list[0], 1u)] = (unsigned)cfg;
}

template <int MODE>
__global__ __launch_bounds__(64) void distance_redo_kernel(DevWorld w, const double* __restrict__ poses, long long n,
                                                           int n_self, ccd_real tol, double dtol,
                                                           double* __restrict__ d_self,
                                                           int32_t* __restrict__ p_self, double* __restrict__ d_others,
                                                           int32_t* __restrict__ p_others,
                                                           double* __restrict__ pts_self,
                                                           double* __restrict__ pts_others,
                                                           ccdx::BigPolytope* __restrict__ pool,
                                                           const unsigned* __restrict__ list) {
  const unsigned k = threadIdx.x, count = list[0];
  for (unsigned i = k; i < count; i += kBigPool)
    distance_config<MODE>(w, poses, n, (long long)list[1 + i], true, n_self, tol, dtol, pool + k, d_self, p_self,
                          d_others, p_others, pts_self, pts_others);
}

// ---------------------------------------------------------------------------
// Contacts: CollisionRequest(enable_contact=True) -> FCL GJKCollide ->
// libccd 2.1 ccdMPRPenetration (discoverPortal, refinePortal, findPenetr /
// findPenetrTouch / findPenetrSegment, findPos; max_iterations 500), the same
// restatement as oracle/collide_oracle.c mpr_penetration.  Runs after the
// collide pipeline on the pairs it reported, one lane per candidate; the
// portal keeps each vertex's per-object support points (v1, v2) for findPos.
// ---------------------------------------------------------------------------
struct SupP {
  CV3 v, v1, v2;
};

__device__ __forceinline__ SupP msupport3(const DevWorld& w, cptr<double> HV, const GObj& a, const GObj& b,
                                          const CV3& dir) {
  SupP s;
  s.v1 = support(w, HV, a, dir);
  s.v2 = support(w, HV, b, vscale(dir, ccd_real(-1)));
  s.v = vsub(s.v1, s.v2);
  return s;
}

__device__ __forceinline__ CV3 portal_dir3(const SupP P[4]) {
  return vnormalize(vcross(vsub(P[2].v, P[1].v), vsub(P[3].v, P[1].v)));
}

__device__ __forceinline__ bool reach_tol(const SupP P[4], const CV3& v4, const CV3& dir, ccd_real tol) {
  const ccd_real dv1 = vdot(P[1].v, dir), dv2 = vdot(P[2].v, dir), dv3 = vdot(P[3].v, dir), dv4 = vdot(v4, dir);
  ccd_real d1 = dv4 - dv1;
  const ccd_real d2 = dv4 - dv2, d3 = dv4 - dv3;
  d1 = (d1 < d2) ? d1 : d2;
  d1 = (d1 < d3) ? d1 : d3;
  return ccd_eq(d1, tol) || d1 < tol;
}

__device__ __forceinline__ void expand3(SupP P[4], const SupP& v4) {
  const CV3 v4v0 = vcross(v4.v, P[0].v);
  if (vdot(P[1].v, v4v0) > 0.0) {
    if (vdot(P[2].v, v4v0) > 0.0) P[1] = v4;
    else P[3] = v4;
  } else {
    if (vdot(P[3].v, v4v0) > 0.0) P[2] = v4;
    else P[1] = v4;
  }
}

__device__ __forceinline__ ccd_real seg_dist2(const CV3& x0, const CV3& b, CV3& wit) {
  const CV3 d = vsub(b, x0), a = x0;  // P = origin
  ccd_real t = -1.0 * vdot(a, d);
  t /= vdot(d, d);
  if (t < 0.0 || is_zero(t)) {
    wit = x0;
  } else if (t > 1.0 || ccd_eq(t, 1.0)) {
    wit = b;
  } else {
    wit = vadd(vscale(d, t), x0);
  }
  return vdot(wit, wit);
}

// ccdVec3PointTriDist2(origin, x0, B, C, witness)
__device__ __forceinline__ ccd_real tri_dist2(const CV3& x0, const CV3& B, const CV3& C, CV3& wit) {
  const CV3 d1 = vsub(B, x0), d2 = vsub(C, x0), a = x0;
  const ccd_real v = vdot(d1, d1), w_ = vdot(d2, d2), p = vdot(a, d1), q = vdot(a, d2), r = vdot(d1, d2);
  const ccd_real d = w_ * v - r * r;
  ccd_real s, t;
  if (is_zero(d)) {
    s = t = -1.0;
  } else {
    s = (q * r - w_ * p) / d;
    t = (-s * r - q) / w_;
  }
  if ((is_zero(s) || s > 0.0) && (ccd_eq(s, 1.0) || s < 1.0) && (is_zero(t) || t > 0.0) && (ccd_eq(t, 1.0) || t < 1.0) &&
      (ccd_eq(t + s, 1.0) || t + s < 1.0)) {
    wit = vadd(vadd(x0, vscale(d1, s)), vscale(d2, t));
    return vdot(wit, wit);
  }
  CV3 w2;
  ccd_real dist = seg_dist2(x0, B, wit);
  ccd_real dist2 = seg_dist2(x0, C, w2);
  if (dist2 < dist) {
    dist = dist2;
    wit = w2;
  }
  dist2 = seg_dist2(B, C, w2);
  if (dist2 < dist) {
    dist = dist2;
    wit = w2;
  }
  return dist;
}

__device__ __forceinline__ CV3 find_pos3(const SupP P[4]) {
  const CV3 dir = portal_dir3(P);
  ccd_real b[4];
  b[0] = vdot(vcross(P[1].v, P[2].v), P[3].v);
  b[1] = vdot(vcross(P[3].v, P[2].v), P[0].v);
  b[2] = vdot(vcross(P[0].v, P[1].v), P[3].v);
  b[3] = vdot(vcross(P[2].v, P[1].v), P[0].v);
  ccd_real sum = b[0] + b[1] + b[2] + b[3];
  if (is_zero(sum) || sum < 0.0) {
    b[0] = 0.0;
    b[1] = vdot(vcross(P[2].v, P[3].v), dir);
    b[2] = vdot(vcross(P[3].v, P[1].v), dir);
    b[3] = vdot(vcross(P[1].v, P[2].v), dir);
    sum = b[1] + b[2] + b[3];
  }
  const ccd_real inv = ccd_real(1) / sum;
  CV3 p1{0, 0, 0}, p2{0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    p1 = vadd(p1, vscale(P[i].v1, b[i]));
    p2 = vadd(p2, vscale(P[i].v2, b[i]));
  }
  p1 = vscale(p1, inv);
  p2 = vscale(p2, inv);
  return vscale(vadd(p1, p2), ccd_real(0.5));
}

// ccdMPRPenetration: true if penetrating (depth, dir, pos set); sup(dir)
// gives the Minkowski support with both objects' points, c1 / c2 the centres
template <typename Sup3>
__device__ bool mpr_penetration_core(ccd_real tol, const CV3& c1, const CV3& c2, Sup3 msup, ccd_real& depth,
                                     CV3& dir_out, CV3& pos_out) {
  SupP P[4];
  P[0].v1 = c1;
  P[0].v2 = c2;
  P[0].v = vsub(P[0].v1, P[0].v2);
  if (vec_is_origin(P[0].v)) P[0].v = vadd(P[0].v, cv3(kCcdEps * ccd_real(10), 0.0, 0.0));
  CV3 dir = vnormalize(vscale(P[0].v, ccd_real(-1)));
  P[1] = msup(dir);
  ccd_real dot = vdot(P[1].v, dir);
  if (is_zero(dot) || dot < 0.0) return false;
  dir = vcross(P[0].v, P[1].v);
  if (is_zero(vdot(dir, dir))) {
    pos_out = vscale(vadd(P[1].v1, P[1].v2), ccd_real(0.5));
    if (vec_is_origin(P[1].v)) {  // findPenetrTouch
      depth = 0.0;
      dir_out = cv3(0.0, 0.0, 0.0);
    } else {  // findPenetrSegment
      dir_out = P[1].v;
      depth = std::sqrt(vdot(dir_out, dir_out));
      dir_out = vnormalize(dir_out);
    }
    return true;
  }
  dir = vnormalize(dir);
  P[2] = msup(dir);
  dot = vdot(P[2].v, dir);
  if (is_zero(dot) || dot < 0.0) return false;
  dir = vnormalize(vcross(vsub(P[1].v, P[0].v), vsub(P[2].v, P[0].v)));
  if (vdot(dir, P[0].v) > 0.0) {
    const SupP t = P[1];
    P[1] = P[2];
    P[2] = t;
    dir = vscale(dir, ccd_real(-1));
  }
  for (;;) {
    P[3] = msup(dir);
    dot = vdot(P[3].v, dir);
    if (is_zero(dot) || dot < 0.0) return false;
    bool cont = false;
    ccd_real d2 = vdot(vcross(P[1].v, P[3].v), P[0].v);
    if (d2 < 0.0 && !is_zero(d2)) {
      P[2] = P[3];
      cont = true;
    }
    if (!cont) {
      d2 = vdot(vcross(P[3].v, P[2].v), P[0].v);
      if (d2 < 0.0 && !is_zero(d2)) {
        P[1] = P[3];
        cont = true;
      }
    }
    if (!cont) break;
    dir = vnormalize(vcross(vsub(P[1].v, P[0].v), vsub(P[2].v, P[0].v)));
  }
  // refinePortal
  for (;;) {
    dir = portal_dir3(P);
    const ccd_real d = vdot(dir, P[1].v);
    if (is_zero(d) || d > 0.0) break;
    const SupP v4 = msup(dir);
    const ccd_real dv4 = vdot(v4.v, dir);
    if (!(is_zero(dv4) || dv4 > 0.0) || reach_tol(P, v4.v, dir, tol)) return false;
    expand3(P, v4);
  }
  // findPenetr
  for (unsigned long it = 0;; ++it) {
    dir = portal_dir3(P);
    const SupP v4 = msup(dir);
    if (reach_tol(P, v4.v, dir, tol) || it > 500UL) {
      CV3 wit;
      depth = std::sqrt(tri_dist2(P[1].v, P[2].v, P[3].v, wit));
      dir_out = is_zero(depth) ? cv3(0.0, 0.0, 0.0) : vnormalize(wit);
      pos_out = find_pos3(P);
      return true;
    }
    expand3(P, v4);
  }
}

__device__ bool mpr_penetration_ccd(const DevWorld& w, cptr<double> HV, const GObj& A, const GObj& B, ccd_real& depth,
                                    CV3& dir_out, CV3& pos_out) {
  return mpr_penetration_core(w.mpr_tol, center(w, A), center(w, B),
                              [&](const CV3& d) { return msupport3(w, HV, A, B, d); }, depth, dir_out, pos_out);
}

// FCL reads the contact back into fp64 (Contact<double>)
__device__ bool mpr_penetration(const DevWorld& w, cptr<double> HV, const GObj& A, const GObj& B, double& depth,
                                V3& dir_out, V3& pos_out) {
  ccd_real d = 0;
  CV3 n{0, 0, 0}, ps{0, 0, 0};
  const bool hit = mpr_penetration_ccd(w, HV, A, B, d, n, ps);
  if (hit) {
    depth = d;
    dir_out = to_v3(n);
    pos_out = to_v3(ps);
  }
  return hit;
}

// ---------------------------------------------------------------------------
// FCL closed-form contacts (CollisionRequest(enable_contact=True) on box-box,
// sphere-sphere, sphere-box, sphere-capsule, sphere-cylinder pairs, both orders): the contacts FCL 0.7.0's
// GJKSolver_libccd::shapeIntersect specialisations emit, reduced to the one
// ShapeShapeCollide keeps for num_max_contacts = 1 (partial_sort by
// descending penetration_depth, first of equals).  Same operation order as
// oracle/collide_oracle.c box_box_contact & co (parity unpinned: FCL's
// contact code is not under /root/reference).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cf_keep(int& n, double pd, const double* nrm, const double* p, double& depth, V3& nd,
                                        V3& ps) {
  if (n == 0 || pd > depth) {
    depth = pd;
    nd = v3(nrm[0], nrm[1], nrm[2]);
    ps = v3(p[0], p[1], p[2]);
  }
  ++n;
}

// ODE intersectRectQuad (box_box-inl.h intersectRectQuad2)
__device__ int cf_rect_quad(const double h[2], double p[8], double ret[16]) {
  int nq = 4, nr = 0;
  double buffer[16];
  double* q = p;
  double* r = ret;
  for (int dir = 0; dir <= 1; ++dir) {
    for (int sign = -1; sign <= 1; sign += 2) {
      double* pq = q;
      double* pr = r;
      nr = 0;
      for (int i = nq; i > 0; --i) {
        if (sign * pq[dir] < h[dir]) {
          pr[0] = pq[0];
          pr[1] = pq[1];
          pr += 2;
          nr++;
          if (nr & 8) {
            q = r;
            goto done;
          }
        }
        double* nextq = (i > 1) ? pq + 2 : q;
        if ((sign * pq[dir] < h[dir]) ^ (sign * nextq[dir] < h[dir])) {
          pr[1 - dir] = pq[1 - dir] + (nextq[1 - dir] - pq[1 - dir]) / (nextq[dir] - pq[dir]) * (sign * h[dir] - pq[dir]);
          pr[dir] = sign * h[dir];
          pr += 2;
          nr++;
          if (nr & 8) {
            q = r;
            goto done;
          }
        }
        pq += 2;
      }
      q = r;
      r = (q == ret) ? buffer : ret;
      nq = nr;
    }
  }
done:
  if (q != ret)
    for (int i = 0; i < 2 * nr; ++i) ret[i] = q[i];
  return nr;
}

// ODE cullPoints (box_box-inl.h cullPoints2)
__device__ void cf_cull_points(int n, const double* p, int m, int i0, int* iret) {
  double a, cx, cy, q;
  if (n == 1) {
    cx = p[0];
    cy = p[1];
  } else if (n == 2) {
    cx = 0.5 * (p[0] + p[2]);
    cy = 0.5 * (p[1] + p[3]);
  } else {
    a = 0;
    cx = 0;
    cy = 0;
    for (int i = 0; i < n - 1; ++i) {
      q = p[i * 2] * p[i * 2 + 3] - p[i * 2 + 2] * p[i * 2 + 1];
      a += q;
      cx += q * (p[i * 2] + p[i * 2 + 2]);
      cy += q * (p[i * 2 + 1] + p[i * 2 + 3]);
    }
    q = p[n * 2 - 2] * p[1] - p[0] * p[n * 2 - 1];
    if (std::fabs(a + q) > DBL_EPSILON) a = 1 / (3 * (a + q));
    else a = (double)1e18f;
    cx = a * (cx + q * (p[n * 2 - 2] + p[0]));
    cy = a * (cy + q * (p[n * 2 - 1] + p[1]));
  }
  double A[8];
  int avail[8];
  for (int i = 0; i < n; ++i) {
    A[i] = std::atan2(p[i * 2 + 1] - cy, p[i * 2] - cx);
    avail[i] = 1;
  }
  avail[i0] = 0;
  iret[0] = i0;
  const double pi = 3.14159265358979323846;
  for (int j = 1; j < m; ++j) {
    a = j * (2 * pi / m) + A[i0];
    if (a > pi) a -= 2 * pi;
    double maxdiff = 1e9, diff;
    iret[j] = i0;
    for (int i = 0; i < n; ++i) {
      if (avail[i]) {
        diff = std::fabs(A[i] - a);
        if (diff > pi) diff = 2 * pi - diff;
        if (diff < maxdiff) {
          maxdiff = diff;
          iret[j] = i;
        }
      }
    }
    avail[iret[j]] = 0;
  }
}

// detail::boxBox2 with contacts (maxc 4) -> the kept contact
__device__ bool box_box_contact(const double* side1, const SE3& T1, const double* side2, const SE3& T2, double& dout,
                                V3& nout, V3& pout) {
#define R1_(i, j) T1.R[3 * (i) + (j)]
#define R2_(i, j) T2.R[3 * (i) + (j)]
  int nc = 0;
  const double p[3] = {T2.p[0] - T1.p[0], T2.p[1] - T1.p[1], T2.p[2] - T1.p[2]};
  double pp[3], A[3], B[3], R[3][3], Q[3][3];
  for (int i = 0; i < 3; ++i) pp[i] = (R1_(0, i) * p[0] + R1_(1, i) * p[1]) + R1_(2, i) * p[2];
  for (int i = 0; i < 3; ++i) {
    A[i] = side1[i] * 0.5;
    B[i] = side2[i] * 0.5;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      R[i][j] = (R1_(0, i) * R2_(0, j) + R1_(1, i) * R2_(1, j)) + R1_(2, i) * R2_(2, j);
      Q[i][j] = std::fabs(R[i][j]);
    }
  double s = -DBL_MAX, s2, tmp, normalC[3] = {0, 0, 0};
  int code = 0, best_col = -1, normal_r2 = 0, invert = 0;
  for (int i = 0; i < 3; ++i) {
    tmp = pp[i];
    s2 = std::fabs(tmp) - (((Q[i][0] * B[0] + Q[i][1] * B[1]) + Q[i][2] * B[2]) + A[i]);
    if (s2 > 0) return false;
    if (s2 > s) {
      s = s2;
      best_col = i;
      normal_r2 = 0;
      invert = tmp < 0;
      code = 1 + i;
    }
  }
  for (int j = 0; j < 3; ++j) {
    tmp = (R2_(0, j) * p[0] + R2_(1, j) * p[1]) + R2_(2, j) * p[2];
    s2 = std::fabs(tmp) - (((Q[0][j] * A[0] + Q[1][j] * A[1]) + Q[2][j] * A[2]) + B[j]);
    if (s2 > 0) return false;
    if (s2 > s) {
      s = s2;
      best_col = j;
      normal_r2 = 1;
      invert = tmp < 0;
      code = 4 + j;
    }
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Q[i][j] += 1.0e-6;
  const double eps = DBL_EPSILON, fudge = 1.05;
  auto edge = [&](double t, double rad, double n0, double n1, double n2, int c) -> bool {
    tmp = t;
    s2 = std::fabs(tmp) - rad;
    if (s2 > eps) return true;
    const double l = std::sqrt((n0 * n0 + n1 * n1) + n2 * n2);
    if (l > eps) {
      s2 /= l;
      if (s2 * fudge > s) {
        s = s2;
        best_col = -1;
        invert = tmp < 0;
        code = c;
        normalC[0] = n0 / l;
        normalC[1] = n1 / l;
        normalC[2] = n2 / l;
      }
    }
    return false;
  };
  if (edge(pp[2] * R[1][0] - pp[1] * R[2][0], ((A[1] * Q[2][0] + A[2] * Q[1][0]) + B[1] * Q[0][2]) + B[2] * Q[0][1], 0,
           -R[2][0], R[1][0], 7)) return false;
  if (edge(pp[2] * R[1][1] - pp[1] * R[2][1], ((A[1] * Q[2][1] + A[2] * Q[1][1]) + B[0] * Q[0][2]) + B[2] * Q[0][0], 0,
           -R[2][1], R[1][1], 8)) return false;
  if (edge(pp[2] * R[1][2] - pp[1] * R[2][2], ((A[1] * Q[2][2] + A[2] * Q[1][2]) + B[0] * Q[0][1]) + B[1] * Q[0][0], 0,
           -R[2][2], R[1][2], 9)) return false;
  if (edge(pp[0] * R[2][0] - pp[2] * R[0][0], ((A[0] * Q[2][0] + A[2] * Q[0][0]) + B[1] * Q[1][2]) + B[2] * Q[1][1],
           R[2][0], 0, -R[0][0], 10)) return false;
  if (edge(pp[0] * R[2][1] - pp[2] * R[0][1], ((A[0] * Q[2][1] + A[2] * Q[0][1]) + B[0] * Q[1][2]) + B[2] * Q[1][0],
           R[2][1], 0, -R[0][1], 11)) return false;
  if (edge(pp[0] * R[2][2] - pp[2] * R[0][2], ((A[0] * Q[2][2] + A[2] * Q[0][2]) + B[0] * Q[1][1]) + B[1] * Q[1][0],
           R[2][2], 0, -R[0][2], 12)) return false;
  if (edge(pp[1] * R[0][0] - pp[0] * R[1][0], ((A[0] * Q[1][0] + A[1] * Q[0][0]) + B[1] * Q[2][2]) + B[2] * Q[2][1],
           -R[1][0], R[0][0], 0, 13)) return false;
  if (edge(pp[1] * R[0][1] - pp[0] * R[1][1], ((A[0] * Q[1][1] + A[1] * Q[0][1]) + B[0] * Q[2][2]) + B[2] * Q[2][0],
           -R[1][1], R[0][1], 0, 14)) return false;
  if (edge(pp[1] * R[0][2] - pp[0] * R[1][2], ((A[0] * Q[1][2] + A[1] * Q[0][2]) + B[0] * Q[2][1]) + B[1] * Q[2][0],
           -R[1][2], R[0][2], 0, 15)) return false;
  if (!code) return false;
  double normal[3];
  if (best_col != -1) {
    const double* Rm = normal_r2 ? T2.R : T1.R;
    for (int i = 0; i < 3; ++i) normal[i] = Rm[3 * i + best_col];
  } else {
    for (int i = 0; i < 3; ++i) normal[i] = (R1_(i, 0) * normalC[0] + R1_(i, 1) * normalC[1]) + R1_(i, 2) * normalC[2];
  }
  if (invert)
    for (int i = 0; i < 3; ++i) normal[i] = -normal[i];
  const double depth = -s;
  if (code > 6) {  // edge-edge: the closest point of box 2's edge
    double pa[3] = {T1.p[0], T1.p[1], T1.p[2]}, pb[3] = {T2.p[0], T2.p[1], T2.p[2]}, sign;
    for (int j = 0; j < 3; ++j) {
      sign = (((R1_(0, j) * normal[0] + R1_(1, j) * normal[1]) + R1_(2, j) * normal[2]) > 0) ? 1 : -1;
      for (int i = 0; i < 3; ++i) pa[i] += R1_(i, j) * (A[j] * sign);
    }
    for (int j = 0; j < 3; ++j) {
      sign = (((R2_(0, j) * normal[0] + R2_(1, j) * normal[1]) + R2_(2, j) * normal[2]) > 0) ? -1 : 1;
      for (int i = 0; i < 3; ++i) pb[i] += R2_(i, j) * (B[j] * sign);
    }
    const int ca = (code - 7) / 3, cb = (code - 7) % 3;
    const double ua[3] = {R1_(0, ca), R1_(1, ca), R1_(2, ca)}, ub[3] = {R2_(0, cb), R2_(1, cb), R2_(2, cb)};
    // lineClosestApproach (ODE dLineClosestApproach); only beta is used
    const double d0 = pb[0] - pa[0], d1 = pb[1] - pa[1], d2 = pb[2] - pa[2];
    const double uaub = (ua[0] * ub[0] + ua[1] * ub[1]) + ua[2] * ub[2];
    const double q1 = (ua[0] * d0 + ua[1] * d1) + ua[2] * d2;
    const double q2 = -((ub[0] * d0 + ub[1] * d1) + ub[2] * d2);
    double dd = 1 - uaub * uaub, beta = 0;
    if (!(dd <= (double)0.0001f)) {
      dd = 1 / dd;
      beta = (uaub * q1 + q2) * dd;
    }
    for (int i = 0; i < 3; ++i) pb[i] += ub[i] * beta;
    cf_keep(nc, -depth, normal, pb, dout, nout, pout);
    return true;
  }
  // face-something: reference face on box a, incident box b
  const double* Ra = code <= 3 ? T1.R : T2.R;
  const double* Rb = code <= 3 ? T2.R : T1.R;
  const double* pa = code <= 3 ? T1.p : T2.p;
  const double* pb = code <= 3 ? T2.p : T1.p;
  const double* Sa = code <= 3 ? A : B;
  const double* Sb = code <= 3 ? B : A;
#define RA(i, j) Ra[3 * (i) + (j)]
#define RB(i, j) Rb[3 * (i) + (j)]
  double normal2[3], nr[3], anr[3];
  for (int i = 0; i < 3; ++i) normal2[i] = code <= 3 ? normal[i] : -normal[i];
  for (int j = 0; j < 3; ++j) {
    nr[j] = (RB(0, j) * normal2[0] + RB(1, j) * normal2[1]) + RB(2, j) * normal2[2];
    anr[j] = std::fabs(nr[j]);
  }
  int lanr, a1, a2;
  if (anr[1] > anr[0]) {
    if (anr[1] > anr[2]) { a1 = 0; lanr = 1; a2 = 2; }
    else { a1 = 0; a2 = 1; lanr = 2; }
  } else {
    if (anr[0] > anr[2]) { lanr = 0; a1 = 1; a2 = 2; }
    else { a1 = 0; a2 = 1; lanr = 2; }
  }
  double center[3];
  for (int i = 0; i < 3; ++i)
    center[i] = nr[lanr] < 0 ? (pb[i] - pa[i]) + RB(i, lanr) * Sb[lanr] : (pb[i] - pa[i]) - RB(i, lanr) * Sb[lanr];
  const int codeN = code <= 3 ? code - 1 : code - 4;
  const int code1 = codeN == 0 ? 1 : 0, code2 = codeN == 2 ? 1 : 2;
  const double c1 = (RA(0, code1) * center[0] + RA(1, code1) * center[1]) + RA(2, code1) * center[2];
  const double c2 = (RA(0, code2) * center[0] + RA(1, code2) * center[1]) + RA(2, code2) * center[2];
  double m11 = (RB(0, a1) * RA(0, code1) + RB(1, a1) * RA(1, code1)) + RB(2, a1) * RA(2, code1);
  double m12 = (RB(0, a2) * RA(0, code1) + RB(1, a2) * RA(1, code1)) + RB(2, a2) * RA(2, code1);
  double m21 = (RB(0, a1) * RA(0, code2) + RB(1, a1) * RA(1, code2)) + RB(2, a1) * RA(2, code2);
  double m22 = (RB(0, a2) * RA(0, code2) + RB(1, a2) * RA(1, code2)) + RB(2, a2) * RA(2, code2);
  double quad[8];
  {
    const double k1 = m11 * Sb[a1], k2 = m21 * Sb[a1], k3 = m12 * Sb[a2], k4 = m22 * Sb[a2];
    quad[0] = c1 - k1 - k3;
    quad[1] = c2 - k2 - k4;
    quad[2] = c1 - k1 + k3;
    quad[3] = c2 - k2 + k4;
    quad[4] = c1 + k1 + k3;
    quad[5] = c2 + k2 + k4;
    quad[6] = c1 + k1 - k3;
    quad[7] = c2 + k2 - k4;
  }
  const double rect[2] = {Sa[code1], Sa[code2]};
  double ret[16];
  const int n_intersect = cf_rect_quad(rect, quad, ret);
  if (n_intersect < 1) return true;  // collision without a contact point
  double points[8][3], dep[8];
  const double det1 = 1.f / (m11 * m22 - m12 * m21);
  m11 *= det1;
  m12 *= det1;
  m21 *= det1;
  m22 *= det1;
  int cnum = 0;
  for (int j = 0; j < n_intersect; ++j) {
    const double k1 = m22 * (ret[j * 2] - c1) - m12 * (ret[j * 2 + 1] - c2);
    const double k2 = -m21 * (ret[j * 2] - c1) + m11 * (ret[j * 2 + 1] - c2);
    for (int i = 0; i < 3; ++i) points[cnum][i] = (center[i] + RB(i, a1) * k1) + RB(i, a2) * k2;
    dep[cnum] = Sa[codeN] - ((normal2[0] * points[cnum][0] + normal2[1] * points[cnum][1]) + normal2[2] * points[cnum][2]);
    if (dep[cnum] >= 0) {
      ret[cnum * 2] = ret[j * 2];
      ret[cnum * 2 + 1] = ret[j * 2 + 1];
      cnum++;
    }
  }
  if (cnum < 1) return true;
  int iret[8];
  if (cnum <= 4) {
    for (int j = 0; j < cnum; ++j) iret[j] = j;
  } else {
    int i1 = 0;
    double maxdepth = dep[0];
    for (int i = 1; i < cnum; ++i)
      if (dep[i] > maxdepth) {
        maxdepth = dep[i];
        i1 = i;
      }
    cf_cull_points(cnum, ret, 4, i1, iret);
    cnum = 4;
  }
  for (int j = 0; j < cnum; ++j) {
    const int k = iret[j];
    double wpt[3];
    for (int i = 0; i < 3; ++i) wpt[i] = code < 4 ? points[k][i] + pa[i] : (points[k][i] + pa[i]) - normal[i] * dep[k];
    cf_keep(nc, -dep[k], normal, wpt, dout, nout, pout);
  }
#undef RA
#undef RB
#undef R1_
#undef R2_
  return true;
}

// detail::sphereSphereIntersect with its contact
__device__ bool sphere_sphere_contact(double r1, const SE3& T1, double r2, const SE3& T2, double& depth, V3& nd,
                                      V3& ps) {
  const double d0 = T2.p[0] - T1.p[0], d1 = T2.p[1] - T1.p[1], d2 = T2.p[2] - T1.p[2];
  const double len = std::sqrt((d0 * d0 + d1 * d1) + d2 * d2);
  if (len > r1 + r2) return false;
  nd = len > 0 ? v3(d0 / len, d1 / len, d2 / len) : v3(d0, d1, d2);
  ps = v3(T1.p[0] + d0 * r1 / (r1 + r2), T1.p[1] + d1 * r1 / (r1 + r2), T1.p[2] + d2 * r1 / (r1 + r2));
  depth = r1 + r2 - len;
  return true;
}

// detail::sphereBoxIntersect with its contact (normal from the sphere into the box)
__device__ bool sphere_box_contact(double r, const SE3& TS, const double* side, const SE3& TB, double& depth, V3& nd,
                                   V3& ps) {
  double c[3], d[3];
  bool clamped = false;
  for (int i = 0; i < 3; ++i) {
    const double inv_t = -((TB.R[i] * TB.p[0] + TB.R[3 + i] * TB.p[1]) + TB.R[6 + i] * TB.p[2]);
    c[i] = ((TB.R[i] * TS.p[0] + TB.R[3 + i] * TS.p[1]) + TB.R[6 + i] * TS.p[2]) + inv_t;
    const double h = side[i] / 2;
    double nq = c[i];
    if (c[i] < -h) {
      clamped = true;
      nq = -h;
    }
    if (c[i] > h) {
      clamped = true;
      nq = h;
    }
    d[i] = c[i] - nq;
  }
  const double dd = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
  if (clamped && dd > r * r) return false;
  double n[3] = {0, 0, 0}, dep;
  if (clamped) {
    const double dist = std::sqrt(dd);
    for (int i = 0; i < 3; ++i) n[i] = -d[i] / dist;
    dep = r - dist;
  } else {
    double min_d = INFINITY;
    int ax = 0;
    for (int i = 0; i < 3; ++i) {
      const double di = side[i] / 2 - std::fabs(c[i]);
      if (di < min_d) {
        min_d = di;
        ax = i;
      }
    }
    n[ax] = c[ax] >= 0 ? -1 : 1;
    dep = min_d + r;
  }
  double pc[3], nw[3], pw[3];
  for (int i = 0; i < 3; ++i) pc[i] = c[i] + n[i] * (r - dep / 2);
  for (int i = 0; i < 3; ++i) {
    nw[i] = (TB.R[3 * i] * n[0] + TB.R[3 * i + 1] * n[1]) + TB.R[3 * i + 2] * n[2];
    pw[i] = ((TB.R[3 * i] * pc[0] + TB.R[3 * i + 1] * pc[1]) + TB.R[3 * i + 2] * pc[2]) + TB.p[i];
  }
  nd = v3(nw[0], nw[1], nw[2]);
  ps = v3(pw[0], pw[1], pw[2]);
  depth = dep;
  return true;
}

// detail::sphereCapsuleIntersect with its contact (oracle sphere_capsule_contact)
__device__ bool sphere_capsule_contact(double r1, const SE3& TS, double r2, double lz, const SE3& TC, double& depth,
                                       V3& nd, V3& ps) {
  double c[3];
  centre_in_frame(TS, TC, c);
  const double s1z = 0.5 * lz, s2z = -s1z;
  const double vz = s2z - s1z;
  const double w2 = c[2] - s1z;
  const double c1 = (c[0] * 0.0 + c[1] * 0.0) + w2 * vz;
  const double c2 = (0.0 * 0.0 + 0.0 * 0.0) + vz * vz;
  double spz;
  if (c1 <= 0) spz = s1z;
  else if (c2 <= c1) spz = s2z;
  else spz = s1z + vz * (c1 / c2);
  const double d[3] = {c[0], c[1], c[2] - spz};
  const double sq = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
  const double dist = std::sqrt(sq) - r1 - r2;
  if (dist > 0) return false;
  const double nn = std::sqrt(sq);
  double ln[3], lp[3], nw[3], pw[3];
  for (int i = 0; i < 3; ++i) ln[i] = sq > 0 ? -(d[i] / nn) : -d[i];
  lp[0] = 0.0 + ln[0] * dist;
  lp[1] = 0.0 + ln[1] * dist;
  lp[2] = spz + ln[2] * dist;
  for (int i = 0; i < 3; ++i) {
    nw[i] = (TC.R[3 * i] * ln[0] + TC.R[3 * i + 1] * ln[1]) + TC.R[3 * i + 2] * ln[2];
    pw[i] = ((TC.R[3 * i] * lp[0] + TC.R[3 * i + 1] * lp[1]) + TC.R[3 * i + 2] * lp[2]) + TC.p[i];
  }
  nd = v3(nw[0], nw[1], nw[2]);
  ps = v3(pw[0], pw[1], pw[2]);
  depth = -dist;
  return true;
}

// detail::sphereCylinderIntersect with its contact (oracle sphere_cylinder_contact)
__device__ bool sphere_cylinder_contact(double r, const SE3& TS, double rc, double lz, const SE3& TC, double& depth,
                                        V3& nd, V3& ps) {
  double c[3], q[3];
  centre_in_frame(TS, TC, c);
  const double h = lz / 2;
  bool clamped = false;
  q[0] = c[0];
  q[1] = c[1];
  q[2] = c[2];
  if (c[2] > h) {
    q[2] = h;
    clamped = true;
  } else if (c[2] < -h) {
    q[2] = -h;
    clamped = true;
  }
  const double rd2 = c[0] * c[0] + c[1] * c[1];
  if (rd2 > rc * rc) {
    const double scale = rc / std::sqrt(rd2);
    q[0] = c[0] * scale;
    q[1] = c[1] * scale;
    clamped = true;
  }
  const double d[3] = {q[0] - c[0], q[1] - c[1], q[2] - c[2]};
  const double dd = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
  if (clamped && dd > r * r) return false;
  double n[3] = {0, 0, 0}, dep;
  if (clamped) {
    const double dist = std::sqrt(dd);
    for (int i = 0; i < 3; ++i) n[i] = d[i] / dist;
    dep = r - dist;
  } else {
    const double face = h - std::fabs(c[2]);
    const double rad = std::sqrt(rd2);
    const double barrel = rc - rad;
    if (face <= barrel) {
      n[2] = c[2] >= 0 ? -1 : 1;
      dep = face + r;
    } else {
      if (rad > 0) {
        n[0] = -(c[0] / rad);
        n[1] = -(c[1] / rad);
      } else {
        n[0] = -1;
      }
      dep = barrel + r;
    }
  }
  double pc[3], nw[3], pw[3];
  for (int i = 0; i < 3; ++i) pc[i] = c[i] + n[i] * (r - dep / 2);
  for (int i = 0; i < 3; ++i) {
    nw[i] = (TC.R[3 * i] * n[0] + TC.R[3 * i + 1] * n[1]) + TC.R[3 * i + 2] * n[2];
    pw[i] = ((TC.R[3 * i] * pc[0] + TC.R[3 * i + 1] * pc[1]) + TC.R[3 * i + 2] * pc[2]) + TC.p[i];
  }
  nd = v3(nw[0], nw[1], nw[2]);
  ps = v3(pw[0], pw[1], pw[2]);
  depth = dep;
  return true;
}

// CollisionRequest(enable_contact=True) on a (shape, OcTree) pair
// [ext FCL 0.7.0 OcTreeShapeIntersectRecurse with contacts]: the first
// occupied leaf in traversal order (the leaf list's order) whose OBB
// overlaps the shape's and whose box intersects it; its contact from
// shapeIntersect(leaf box, shape): the tree is the contact's o1, the normal
// points from the leaf into the shape (oracle octree_contact).  One lane
// walks the whole leaf list: contacts are a scalar-API path.
__device__ bool octree_first_contact(const DevWorld& w, cptr<double> HV, int go, const SE3& TO, int gs, const SE3& TS,
                                     double& depth, V3& nd, V3& ps) {
  const cptr<double> grs = w.geom_rec + G_STRIDE * gs;
  const int ts = w.geom_type[gs];
  double sc[3], se[3], Rl[9];
  for (int i = 0; i < 3; ++i) se[i] = grs[G_AABB_E + i];
  for (int i = 0; i < 3; ++i)
    sc[i] = ((TS.R[3 * i] * grs[G_OBB_C] + TS.R[3 * i + 1] * grs[G_OBB_C + 1]) + TS.R[3 * i + 2] * grs[G_OBB_C + 2]) +
            TS.p[i];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Rl[3 * i + j] = (TO.R[i] * TS.R[j] + TO.R[3 + i] * TS.R[3 + j]) + TO.R[6 + i] * TS.R[6 + j];
  GObj B;
  B.rot = gjk_rot_from_matrix(TS.R);
  B.rot_inv = quat_invert2(B.rot);
  B.pos = cv3(TS.p[0], TS.p[1], TS.p[2]);
  B.geom = gs;
  B.type = ts;
  GObj A;
  A.rot = gjk_rot_from_matrix(TO.R);
  A.rot_inv = quat_invert2(A.rot);
  A.geom = go;
  A.type = MPG_GEOM_BOX;
  const double sb[3] = {grs[G_PARAM], grs[G_PARAM + 1], grs[G_PARAM + 2]};
  const cptr<double> gor = w.geom_rec + G_STRIDE * go;
  const int l0 = (int)gor[G_PARAM], ln = (int)gor[G_PARAM + 1];
  for (int l = l0; l < l0 + ln; ++l) {
    const cptr<double> L = w.oct_leaf + 6 * (size_t)l;
    double c[3], cw[3], a[3], side[3], t[3], T[3];
    for (int i = 0; i < 3; ++i) {
      c[i] = (L[i] + L[3 + i]) * 0.5;
      side[i] = L[3 + i] - L[i];
      a[i] = side[i] * 0.5;
    }
    for (int i = 0; i < 3; ++i) cw[i] = ((TO.R[3 * i] * c[0] + TO.R[3 * i + 1] * c[1]) + TO.R[3 * i + 2] * c[2]) + TO.p[i];
    for (int i = 0; i < 3; ++i) t[i] = sc[i] - cw[i];
    for (int i = 0; i < 3; ++i) T[i] = (TO.R[i] * t[0] + TO.R[3 + i] * t[1]) + TO.R[6 + i] * t[2];
    if (obb_disjoint(Rl, T, a, se)) continue;
    SE3 TL;
    for (int i = 0; i < 9; ++i) TL.R[i] = TO.R[i];
    for (int i = 0; i < 3; ++i) TL.p[i] = cw[i];
    depth = 0.0;
    nd = v3(0, 0, 0);
    ps = v3(0, 0, 0);
    bool hit;
    if (ts == MPG_GEOM_BOX) {
      hit = box_box_contact(side, TL, sb, TS, depth, nd, ps);
    } else if (ts == MPG_GEOM_SPHERE) {
      hit = sphere_box_contact(sb[0], TS, side, TL, depth, nd, ps);
      nd = v3(-nd.x, -nd.y, -nd.z);  // flipNormal
    } else {
      GObj A1 = A;
      A1.pos = cv3(cw[0], cw[1], cw[2]);
      const ccd_real h[3] = {(ccd_real)(side[0] / 2.0), (ccd_real)(side[1] / 2.0), (ccd_real)(side[2] / 2.0)};
      ccd_real dc = 0;
      CV3 n{0, 0, 0}, pc{0, 0, 0};
      hit = mpr_penetration_core(
          w.mpr_tol, A1.pos, center(w, B),
          [&](const CV3& d) {
            SupP sp;
            const CV3 da = quat_rot(d, A1.rot_inv);
            const CV3 la = CV3{(da.x >= 0 ? ccd_real(1) : ccd_real(-1)) * h[0], (da.y >= 0 ? ccd_real(1) : ccd_real(-1)) * h[1],
                               (da.z >= 0 ? ccd_real(1) : ccd_real(-1)) * h[2]};
            sp.v1 = vadd(quat_rot(la, A1.rot), A1.pos);
            sp.v2 = support(w, HV, B, vscale(d, ccd_real(-1)));
            sp.v = vsub(sp.v1, sp.v2);
            return sp;
          },
          dc, n, pc);
      if (hit) {
        depth = dc;
        nd = to_v3(n);
        ps = to_v3(pc);
      }
    }
    if (hit) return true;
  }
  depth = 0.0;
  nd = v3(0, 0, 0);
  ps = v3(0, 0, 0);
  return false;
}

__host__ __device__ __forceinline__ bool cf_has_contact(int cf) {
  return cf != CF_NONE && cf != CF_OCTREE && cf != CF_MESH;
}

__device__ bool closed_form_contact(int cf, const DevWorld& w, int ga, const SE3& TA, int gb, const SE3& TB,
                                    double& depth, V3& nd, V3& ps) {
  const cptr<double> pa = w.geom_rec + G_STRIDE * ga + G_PARAM, pb = w.geom_rec + G_STRIDE * gb + G_PARAM;
  const double sa[3] = {pa[0], pa[1], pa[2]}, sb[3] = {pb[0], pb[1], pb[2]};
  switch (cf) {
    case CF_BOX_BOX: return box_box_contact(sa, TA, sb, TB, depth, nd, ps);
    case CF_SPHERE_SPHERE: return sphere_sphere_contact(sa[0], TA, sb[0], TB, depth, nd, ps);
    case CF_SPHERE_BOX: return sphere_box_contact(sa[0], TA, sb, TB, depth, nd, ps);
    case CF_SPHERE_CAPSULE: return sphere_capsule_contact(sa[0], TA, sb[0], sb[1], TB, depth, nd, ps);
    case CF_SPHERE_CYLINDER: return sphere_cylinder_contact(sa[0], TA, sb[0], sb[1], TB, depth, nd, ps);
    default: break;
  }
  // the shape-sphere orders: the sphere first, then flipNormal
  bool h;
  if (cf == CF_CAPSULE_SPHERE) h = sphere_capsule_contact(sb[0], TB, sa[0], sa[1], TA, depth, nd, ps);
  else if (cf == CF_CYLINDER_SPHERE) h = sphere_cylinder_contact(sb[0], TB, sa[0], sa[1], TA, depth, nd, ps);
  else h = sphere_box_contact(sb[0], TB, sa, TA, depth, nd, ps);  // CF_BOX_SPHERE
  nd = v3(-nd.x, -nd.y, -nd.z);
  return h;
}

// ---------------------------------------------------------------------------
// Contacts on BVH-mesh pairs (CollisionRequest(enable_contact=True)), one lane
// per reported (configuration, pair), the lane alone -- the same restatement
// as oracle/collide_oracle.c mesh_contact [ext FCL 0.7.0, parity unpinned]:
// the first hit in FCL's traversal order (the reachable hit whose descent key
// -- fcl_gate_shape's leaf position, fcl_gate_mesh's left / right choices,
// fcl_gate_octree_mesh's octree children and mesh choices -- is smallest),
// then
//   mesh-mesh    intersect_Triangle's contact branch (computeDeepestPoints
//                of each triangle against the other's plane), o1's frame ->
//                world;
//   shape-mesh   sphereTriangleIntersect's contact for spheres, libccd MPR
//                penetration of (shape, triangle GJK object) otherwise; the
//                mesh-first order negates the normal;
//   mesh-OcTree  MPR penetration of (leaf box, triangle) of the first hit in
//                OcTreeMeshIntersectRecurse's visit order.
// The AABB prefilters only skip separated triangles and the gates replay
// FCL's descent, so the first hit is the one the oracle's recursion finds.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void tri_plane(const double* v1, const double* v2, const double* v3, double* n, double& t) {
  double a[3], b[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    a[k] = v2[k] - v1[k];
    b[k] = v3[k] - v1[k];
  }
  c3(n, a, b);
  const double z = d3(n, n);
  if (!(z > 0)) {
    n[0] = n[1] = n[2] = 0.0;
    t = 0.0;
    return;
  }
  const double r = std::sqrt(z);
#pragma unroll
  for (int k = 0; k < 3; ++k) n[k] /= r;
  t = d3(n, v1);
}

// Intersect::computeDeepestPoints: depth and the first deepest vertex
__device__ __forceinline__ int deepest_points(const double* T, const double* n, double t, double& pen, double* first) {
  double max_depth = -DBL_MAX;
  int num = 0, num_neg = 0, num_pos = 0, num_zero = 0;
  for (int i = 0; i < 3; ++i) {
    const double dist = -(d3(n, T + 3 * i) - t);
    if (dist > 1e-5) num_pos++;
    else if (dist < -1e-5) num_neg++;
    else num_zero++;
    if (dist > max_depth) {
      max_depth = dist;
      num = 1;
      first[0] = T[3 * i];
      first[1] = T[3 * i + 1];
      first[2] = T[3 * i + 2];
    } else if (dist + 1e-6 >= max_depth) {
      num++;
    }
  }
  if (max_depth < -1e-5) num = 0;
  if (num_zero == 0 && (num_neg == 0 || num_pos == 0)) num = 0;
  pen = max_depth;
  return num;
}

__device__ int tri_tri_contact(const double* P, const double* Q, double* point, double* normal, double& depth) {
  double n1[3], n2[3], t1, t2, d1[3] = {0, 0, 0}, d2[3] = {0, 0, 0}, pen1, pen2;
  tri_plane(P, P + 3, P + 6, n1, t1);
  tri_plane(Q, Q + 3, Q + 6, n2, t2);
  const int k2 = deepest_points(Q, n1, t1, pen2, d2);
  const int k1 = deepest_points(P, n2, t2, pen1, d1);
  if (pen1 > pen2) {
    for (int k = 0; k < 3; ++k) {
      point[k] = d2[k];
      normal[k] = -n1[k];
    }
    depth = pen2;
    return min(k2, 2);
  }
  for (int k = 0; k < 3; ++k) {
    point[k] = d1[k];
    normal[k] = n2[k];
  }
  depth = pen1;
  return min(k1, 2);
}

__device__ __forceinline__ double seg_sqr_dist_nearest(const double* from, const double* to, const double* p,
                                                       double* nearest) {
  double diff[3], v[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    diff[k] = p[k] - from[k];
    v[k] = to[k] - from[k];
  }
  double t = d3(v, diff);
  if (t > 0) {
    const double vv = d3(v, v);
    if (t < vv) {
      t /= vv;
#pragma unroll
      for (int k = 0; k < 3; ++k) diff[k] -= v[k] * t;
    } else {
      t = 1;
#pragma unroll
      for (int k = 0; k < 3; ++k) diff[k] -= v[k];
    }
  } else {
    t = 0;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) nearest[k] = from[k] + v[k] * t;
  return d3(diff, diff);
}

// sphereTriangleIntersect with its contact (W = world triangle)
__device__ bool sphere_triangle_contact(double radius, const double* c, const double* W, double& depth, V3& nd,
                                        V3& ps) {
  double a[3], b[3], n[3], pc[3], cp[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    a[k] = W[3 + k] - W[k];
    b[k] = W[6 + k] - W[k];
  }
  c3(n, a, b);
  const double z = d3(n, n);
  if (z > 0) {
    const double s = std::sqrt(z);
    n[0] /= s;
    n[1] /= s;
    n[2] /= s;
  }
  const double rt = radius + DBL_EPSILON;
#pragma unroll
  for (int k = 0; k < 3; ++k) pc[k] = c[k] - W[k];
  double dist = d3(pc, n);
  if (dist < 0) {
    dist *= -1;
    n[0] *= -1;
    n[1] *= -1;
    n[2] *= -1;
  }
  bool has = false;
  if (dist < rt) {
    double e1[3], e2[3], e3[3], u[3], v[3], x[3], en[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      e1[k] = W[3 + k] - W[k];
      e2[k] = W[6 + k] - W[3 + k];
      e3[k] = W[k] - W[6 + k];
      u[k] = c[k] - W[k];
      v[k] = c[k] - W[3 + k];
      x[k] = c[k] - W[6 + k];
    }
    c3(en, e1, n);
    const double r1 = d3(en, u);
    c3(en, e2, n);
    const double r2 = d3(en, v);
    c3(en, e3, n);
    const double r3 = d3(en, x);
    if ((r1 > 0 && r2 > 0 && r3 > 0) || (r1 <= 0 && r2 <= 0 && r3 <= 0)) {
      has = true;
#pragma unroll
      for (int k = 0; k < 3; ++k) cp[k] = c[k] - n[k] * dist;
    } else {
      const double rr = rt * rt;
      double ne[3];
      if (seg_sqr_dist_nearest(W, W + 3, c, ne) < rr) {
        has = true;
        cp[0] = ne[0]; cp[1] = ne[1]; cp[2] = ne[2];
      }
      if (seg_sqr_dist_nearest(W + 3, W + 6, c, ne) < rr) {
        has = true;
        cp[0] = ne[0]; cp[1] = ne[1]; cp[2] = ne[2];
      }
      if (seg_sqr_dist_nearest(W + 6, W, c, ne) < rr) {
        has = true;
        cp[0] = ne[0]; cp[1] = ne[1]; cp[2] = ne[2];
      }
    }
  }
  if (!has) return false;
  const double cc[3] = {cp[0] - c[0], cp[1] - c[1], cp[2] - c[2]};
  const double d2 = d3(cc, cc);
  if (!(d2 < rt * rt)) return false;
  if (d2 > 0) {
    const double d = std::sqrt(d2);
    nd = v3(cc[0] / d, cc[1] / d, cc[2] / d);
    depth = -(radius - d);
  } else {
    nd = v3(-n[0], -n[1], -n[2]);
    depth = -radius;
  }
  ps = v3(cp[0], cp[1], cp[2]);
  return true;
}

// triangle GJK object support (supportTriangle) in world coordinates
__device__ __forceinline__ CV3 tri_support(const GObj& b, const CV3* P, const CV3& tc, const CV3& dir) {
  const CV3 db = quat_rot(dir, b.rot_inv);
  ccd_real maxdot = -FLT_MAX;
  CV3 lb = P[0];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const ccd_real dot = vdot(db, vsub(P[i], tc));
    if (dot > maxdot) {
      lb = P[i];
      maxdot = dot;
    }
  }
  return vadd(quat_rot(lb, b.rot), b.pos);
}

// MPR penetration of (object a, triangle of record rec in b's frame); a is a
// shape (h == nullptr) or a box with half sizes h
__device__ bool tri_mpr_penetration(const DevWorld& w, cptr<double> HV, const GObj& a, const ccd_real* h,
                                    const GObj& b, cptr<double> rec, double& depth, V3& nd, V3& ps) {
  double P[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) P[k] = rec[TR_P + k];
  const CV3 tc = cv3((P[0] + P[3] + P[6]) / 3, (P[1] + P[4] + P[7]) / 3, (P[2] + P[5] + P[8]) / 3);
  const CV3 TP[3] = {cv3(P[0], P[1], P[2]), cv3(P[3], P[4], P[5]), cv3(P[6], P[7], P[8])};
  ccd_real dc = 0;
  CV3 n{0, 0, 0}, pc{0, 0, 0};
  const CV3 ca = h ? a.pos : center(w, a);
  const bool hit = mpr_penetration_core(
      w.mpr_tol, ca, vadd(quat_rot(tc, b.rot), b.pos),
      [&](const CV3& d) {
        SupP sp;
        if (h) {
          const CV3 da = quat_rot(d, a.rot_inv);
          const CV3 la = CV3{(da.x >= 0 ? ccd_real(1) : ccd_real(-1)) * h[0], (da.y >= 0 ? ccd_real(1) : ccd_real(-1)) * h[1],
                             (da.z >= 0 ? ccd_real(1) : ccd_real(-1)) * h[2]};
          sp.v1 = vadd(quat_rot(la, a.rot), a.pos);
        } else {
          sp.v1 = support(w, HV, a, d);
        }
        sp.v2 = tri_support(b, TP, tc, vscale(d, ccd_real(-1)));
        sp.v = vsub(sp.v1, sp.v2);
        return sp;
      },
      dc, n, pc);
  if (hit) {
    depth = dc;
    nd = to_v3(n);
    ps = to_v3(pc);
  }
  return hit;
}

__device__ __forceinline__ GObj posed_obj(const SE3& T, int g, int type) {
  GObj o;
  o.rot = gjk_rot_from_matrix(T.R);
  o.rot_inv = quat_invert2(o.rot);
  o.pos = cv3(T.p[0], T.p[1], T.p[2]);
  o.geom = g;
  o.type = type;
  return o;
}

__device__ bool mesh_shape_first_contact(const DevWorld& w, cptr<double> HV, int gm, const SE3& TM, int gs,
                                         const SE3& TS, bool mesh_first, double& depth, V3& nd, V3& ps) {
  const cptr<double> grm = w.geom_rec + G_STRIDE * gm, grs = w.geom_rec + G_STRIDE * gs;
  const int ts = w.geom_type[gs];
  const int t0 = (int)grm[G_PARAM], t1 = t0 + (int)grm[G_PARAM + 1];
  double sc[3], cl[3], Rl[9], hq[3];  // the shape's box in the mesh frame, as mesh_shape_wave
  for (int i = 0; i < 3; ++i)
    sc[i] = ((TS.R[3 * i] * grs[G_OBB_C] + TS.R[3 * i + 1] * grs[G_OBB_C + 1]) + TS.R[3 * i + 2] * grs[G_OBB_C + 2]) + TS.p[i];
  const double dsc[3] = {sc[0] - TM.p[0], sc[1] - TM.p[1], sc[2] - TM.p[2]};
  for (int i = 0; i < 3; ++i) {
    cl[i] = (TM.R[i] * dsc[0] + TM.R[3 + i] * dsc[1]) + TM.R[6 + i] * dsc[2];
    for (int j = 0; j < 3; ++j) Rl[3 * i + j] = (TM.R[i] * TS.R[j] + TM.R[3 + i] * TS.R[3 + j]) + TM.R[6 + i] * TS.R[6 + j];
  }
  for (int i = 0; i < 3; ++i)
    hq[i] = ((std::fabs(Rl[3 * i]) * grs[G_OBB_E] + std::fabs(Rl[3 * i + 1]) * grs[G_OBB_E + 1]) +
             std::fabs(Rl[3 * i + 2]) * grs[G_OBB_E + 2]) * (1.0 + 1e-9) +
            kMeshShapePad * (1.0 + std::fabs(TS.p[0]) + std::fabs(TS.p[1]) + std::fabs(TS.p[2]) + std::fabs(TM.p[0]) +
                             std::fabs(TM.p[1]) + std::fabs(TM.p[2]));
  const GObj A = posed_obj(TS, gs, ts), B = posed_obj(TM, gm, MPG_GEOM_MESH);
  double sA[9], sT[3], sE[3];
  fcl_shape_obb_world(w, gs, ts, TS, sA, sT, sE);
  // FCL's traversal visits the leaves left to right: the first hit is the
  // reachable (gated) hit of smallest leaf position
  int best = INT_MAX;
  double bd = 0.0;
  V3 bn{0, 0, 0}, bp{0, 0, 0};
  for (int t = t0; t < t1; ++t) {
    const cptr<double> rec = w.mesh_tri + TR_STRIDE * (size_t)t;
    const int id = w.tri_pos[t0 + (int)rec[TR_ID]];  // leaf position
    if (id >= best) continue;
    bool out = false;
    for (int i = 0; i < 3; ++i) out |= rec[TR_LO + i] > cl[i] + hq[i] || rec[TR_HI + i] < cl[i] - hq[i];
    if (out) continue;
    double dp = 0.0;
    V3 n{0, 0, 0}, p{0, 0, 0};
    bool hit;
    if (ts == MPG_GEOM_SPHERE) {
      double W[9];
      for (int v = 0; v < 3; ++v)
        for (int i = 0; i < 3; ++i)
          W[3 * v + i] = ((TM.R[3 * i] * rec[3 * v] + TM.R[3 * i + 1] * rec[3 * v + 1]) + TM.R[3 * i + 2] * rec[3 * v + 2]) +
                         TM.p[i];
      hit = sphere_triangle_contact(grs[G_PARAM], TS.p, W, dp, n, p);
    } else {
      hit = tri_mpr_penetration(w, HV, A, nullptr, B, rec, dp, n, p);
    }
    if (hit && fcl_gate_shape(w, gm, TM, sA, sT, sE, (int)rec[TR_ID])) {
      best = id;
      bd = dp;
      bn = n;
      bp = p;
    }
  }
  depth = bd;
  nd = mesh_first ? v3(-bn.x, -bn.y, -bn.z) : bn;
  ps = bp;
  return best != INT_MAX;
}

__device__ bool mesh_mesh_first_contact(const DevWorld& w, int ga, const SE3& TA, int gb, const SE3& TB, double& depth,
                                        V3& nd, V3& ps) {
  const cptr<double> gra = w.geom_rec + G_STRIDE * ga, grb = w.geom_rec + G_STRIDE * gb;
  const int b0 = (int)grb[G_PARAM], b1 = b0 + (int)grb[G_PARAM + 1];
  const int c0 = w.mesh_tree[2 * ga], c1 = c0 + w.mesh_tree[2 * ga + 1];
  double R[9], T[3], alo[3], ahi[3];
  const double dt[3] = {TB.p[0] - TA.p[0], TB.p[1] - TA.p[1], TB.p[2] - TA.p[2]};
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) R[3 * i + j] = (TA.R[i] * TB.R[j] + TA.R[3 + i] * TB.R[3 + j]) + TA.R[6 + i] * TB.R[6 + j];
    T[i] = (TA.R[i] * dt[0] + TA.R[3 + i] * dt[1]) + TA.R[6 + i] * dt[2];
    alo[i] = gra[G_OBB_C + i] - gra[G_OBB_E + i];
    ahi[i] = gra[G_OBB_C + i] + gra[G_OBB_E + i];
  }
  // the first hit in FCL's visit order: the reachable intersecting pair whose
  // descent (fcl_gate_mesh's left / right choices) is lexicographically smallest
  uint64_t best[2] = {~0ull, ~0ull};
  int best_a = -1, best_b = -1;
  for (int j = b0; j < b1; ++j) {
    const cptr<double> rq = w.mesh_tri + TR_STRIDE * (size_t)j;
    const long long idb = (long long)rq[TR_ID];
    double Q[9], qlo[3], qhi[3];
    for (int v = 0; v < 3; ++v)
      for (int i = 0; i < 3; ++i)
        Q[3 * v + i] = ((R[3 * i] * rq[3 * v] + R[3 * i + 1] * rq[3 * v + 1]) + R[3 * i + 2] * rq[3 * v + 2]) + T[i];
    bool keep = true;
    for (int i = 0; i < 3; ++i) {
      qlo[i] = fmin(Q[i], fmin(Q[3 + i], Q[6 + i])) - kMeshPad;
      qhi[i] = fmax(Q[i], fmax(Q[3 + i], Q[6 + i])) + kMeshPad;
      keep &= !(qlo[i] > ahi[i] || qhi[i] < alo[i]);
    }
    if (!keep) continue;
    for (int c = c0; c < c1; ++c) {
      const cptr<double> bx = w.mesh_node + 6 * (size_t)c;
      bool ov = true;
      for (int i = 0; i < 3; ++i) ov &= !(bx[i] > qhi[i] || bx[3 + i] < qlo[i]);
      if (!ov) continue;
      const int t1 = w.mesh_link[2 * c] + w.mesh_link[2 * c + 1];
      for (int t = w.mesh_link[2 * c]; t < t1; ++t) {
        const cptr<double> rp = w.mesh_tri + TR_STRIDE * (size_t)t;
        bool o2 = false;
        for (int i = 0; i < 3; ++i) o2 |= rp[TR_LO + i] > qhi[i] || rp[TR_HI + i] < qlo[i];
        if (o2) continue;
        double P[9];
        for (int q = 0; q < 9; ++q) P[q] = rp[TR_P + q];
        if (!tri_tri_intersect(P, Q)) continue;
        uint64_t key[2] = {0ull, 0ull};
        if (!fcl_gate_mesh(w, ga, gb, R, T, (int)rp[TR_ID], (int)idb, key)) continue;
        if (key[0] < best[0] || (key[0] == best[0] && key[1] < best[1])) {
          best[0] = key[0];
          best[1] = key[1];
          best_a = t;
          best_b = j;
        }
      }
    }
  }
  depth = 0.0;
  nd = v3(0, 0, 0);
  ps = v3(0, 0, 0);
  if (best_a < 0) return false;
  double P[9], Q[9], pt[3], nl[3], pen;
  const cptr<double> rp = w.mesh_tri + TR_STRIDE * (size_t)best_a, rq = w.mesh_tri + TR_STRIDE * (size_t)best_b;
  for (int q = 0; q < 9; ++q) P[q] = rp[TR_P + q];
  for (int v = 0; v < 3; ++v)
    for (int i = 0; i < 3; ++i)
      Q[3 * v + i] = ((R[3 * i] * rq[3 * v] + R[3 * i + 1] * rq[3 * v + 1]) + R[3 * i + 2] * rq[3 * v + 2]) + T[i];
  if (tri_tri_contact(P, Q, pt, nl, pen) > 0) {
    double wp[3], wn[3];
    for (int i = 0; i < 3; ++i) {
      wp[i] = ((TA.R[3 * i] * pt[0] + TA.R[3 * i + 1] * pt[1]) + TA.R[3 * i + 2] * pt[2]) + TA.p[i];
      wn[i] = (TA.R[3 * i] * nl[0] + TA.R[3 * i + 1] * nl[1]) + TA.R[3 * i + 2] * nl[2];
    }
    depth = pen;
    nd = v3(wn[0], wn[1], wn[2]);
    ps = v3(wp[0], wp[1], wp[2]);
  }
  return true;
}

__device__ bool mesh_octree_first_contact(const DevWorld& w, int gm, const SE3& TM, int go, const SE3& TO,
                                          double& depth, V3& nd, V3& ps) {
  const cptr<double> grm = w.geom_rec + G_STRIDE * gm;
  const double pad = kMeshShapePad * (1.0 + std::fabs(TO.p[0]) + std::fabs(TO.p[1]) + std::fabs(TO.p[2]) +
                                      std::fabs(TM.p[0]) + std::fabs(TM.p[1]) + std::fabs(TM.p[2]));
  double Rm[9], Ro[9], mcw[3], blo[3], bhi[3];  // as mesh_octree_wave
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      Rm[3 * i + j] = (TO.R[i] * TM.R[j] + TO.R[3 + i] * TM.R[3 + j]) + TO.R[6 + i] * TM.R[6 + j];
      Ro[3 * j + i] = Rm[3 * i + j];
    }
  for (int i = 0; i < 3; ++i)
    mcw[i] = ((TM.R[3 * i] * grm[G_OBB_C] + TM.R[3 * i + 1] * grm[G_OBB_C + 1]) + TM.R[3 * i + 2] * grm[G_OBB_C + 2]) +
             TM.p[i];
  const double dmo[3] = {mcw[0] - TO.p[0], mcw[1] - TO.p[1], mcw[2] - TO.p[2]};
  for (int i = 0; i < 3; ++i) {
    const double c = (TO.R[i] * dmo[0] + TO.R[3 + i] * dmo[1]) + TO.R[6 + i] * dmo[2];
    const double e = ((std::fabs(Rm[3 * i]) * grm[G_OBB_E] + std::fabs(Rm[3 * i + 1]) * grm[G_OBB_E + 1]) +
                      std::fabs(Rm[3 * i + 2]) * grm[G_OBB_E + 2]) * (1.0 + 1e-9) + 1e-9 + pad;
    blo[i] = c - e;
    bhi[i] = c + e;
  }
  GObj A = posed_obj(TO, go, MPG_GEOM_BOX);
  const GObj B = posed_obj(TM, gm, MPG_GEOM_MESH);
  const int c0 = w.mesh_tree[2 * gm], c1 = c0 + w.mesh_tree[2 * gm + 1];
  const cptr<double> gor = w.geom_rec + G_STRIDE * go;
  const int l0 = (int)gor[G_PARAM], ln = (int)gor[G_PARAM + 1];
  // the first hit in OcTreeMeshIntersectRecurse's visit order: the reachable
  // (leaf, triangle) hit whose descent key (fcl_gate_octree_mesh) is smallest
  uint64_t best[kOctKeyWords];
  for (int k = 0; k < kOctKeyWords; ++k) best[k] = ~0ull;
  bool found = false;
  double bd = 0.0;
  V3 bn{0, 0, 0}, bp{0, 0, 0};
  for (int l = l0; l < l0 + ln; ++l) {
    const cptr<double> L = w.oct_leaf + 6 * (size_t)l;
    bool out = false;
    for (int i = 0; i < 3; ++i) out |= L[i] > bhi[i] || L[3 + i] < blo[i];
    if (out) continue;
    double c[3], side[3], cw[3], cm[3], hm[3];
    for (int i = 0; i < 3; ++i) {
      c[i] = (L[i] + L[3 + i]) * 0.5;
      side[i] = L[3 + i] - L[i];
    }
    for (int i = 0; i < 3; ++i) cw[i] = ((TO.R[3 * i] * c[0] + TO.R[3 * i + 1] * c[1]) + TO.R[3 * i + 2] * c[2]) + TO.p[i];
    const double dm[3] = {cw[0] - TM.p[0], cw[1] - TM.p[1], cw[2] - TM.p[2]};
    for (int i = 0; i < 3; ++i) {
      cm[i] = (TM.R[i] * dm[0] + TM.R[3 + i] * dm[1]) + TM.R[6 + i] * dm[2];
      hm[i] = ((std::fabs(Ro[3 * i]) * side[0] + std::fabs(Ro[3 * i + 1]) * side[1]) + std::fabs(Ro[3 * i + 2]) * side[2]) *
                  0.5 * (1.0 + 1e-9) + 1e-9 + pad;
    }
    A.pos = cv3(cw[0], cw[1], cw[2]);
    const ccd_real h[3] = {(ccd_real)(side[0] / 2.0), (ccd_real)(side[1] / 2.0), (ccd_real)(side[2] / 2.0)};
    for (int cl = c0; cl < c1; ++cl) {
      const cptr<double> bx = w.mesh_node + 6 * (size_t)cl;
      bool away = false;
      for (int i = 0; i < 3; ++i) away |= bx[i] > cm[i] + hm[i] || bx[3 + i] < cm[i] - hm[i];
      if (away) continue;
      const int t1 = w.mesh_link[2 * cl] + w.mesh_link[2 * cl + 1];
      for (int t = w.mesh_link[2 * cl]; t < t1; ++t) {
        const cptr<double> rec = w.mesh_tri + TR_STRIDE * (size_t)t;
        const int id = (int)rec[TR_ID];
        bool o2 = false;
        for (int i = 0; i < 3; ++i) o2 |= rec[TR_LO + i] > cm[i] + hm[i] || rec[TR_HI + i] < cm[i] - hm[i];
        if (o2) continue;
        double dp = 0.0;
        V3 n{0, 0, 0}, p{0, 0, 0};
        if (!tri_mpr_penetration(w, w.hull, A, h, B, rec, dp, n, p)) continue;
        uint64_t key[kOctKeyWords] = {0ull, 0ull, 0ull, 0ull, 0ull};
        if (!fcl_gate_octree_mesh(w, go, TO, gm, TM, l, id, key)) continue;
        bool less = false;
        for (int k = 0; k < kOctKeyWords; ++k)
          if (key[k] != best[k]) {
            less = key[k] < best[k];
            break;
          }
        if (!found || less) {
          for (int k = 0; k < kOctKeyWords; ++k) best[k] = key[k];
          found = true;
          bd = dp;
          bn = n;
          bp = p;
        }
      }
    }
  }
  depth = found ? bd : 0.0;
  nd = found ? bn : v3(0, 0, 0);
  ps = found ? bp : v3(0, 0, 0);
  return found;
}

__device__ bool mesh_first_contact(const DevWorld& w, cptr<double> HV, int ga, const SE3& TA, int gb, const SE3& TB,
                                   double& depth, V3& nd, V3& ps) {
  const int ta = w.geom_type[ga], tb = w.geom_type[gb];
  if (ta == MPG_GEOM_MESH && tb == MPG_GEOM_MESH) return mesh_mesh_first_contact(w, ga, TA, gb, TB, depth, nd, ps);
  if (tb == MPG_GEOM_OCTREE) return mesh_octree_first_contact(w, ga, TA, gb, TB, depth, nd, ps);
  if (ta == MPG_GEOM_OCTREE) return mesh_octree_first_contact(w, gb, TB, ga, TA, depth, nd, ps);
  if (ta == MPG_GEOM_MESH) return mesh_shape_first_contact(w, HV, ga, TA, gb, TB, true, depth, nd, ps);
  return mesh_shape_first_contact(w, HV, gb, TB, ga, TA, false, depth, nd, ps);
}

template <bool FROM_POSES>
__global__ __launch_bounds__(256) void contact_kernel(DevWorld w, const double* __restrict__ in,
                                                     const uint32_t* __restrict__ seg_len,
                                                     const uint32_t* __restrict__ seg_start,
                                                     const uint32_t* __restrict__ prefix,
                                                     const uint32_t* __restrict__ cand,
                                                     const uint32_t* __restrict__ masks, const double* __restrict__ sc,
                                                     double* __restrict__ depth, double* __restrict__ normal,
                                                     double* __restrict__ pos) {
  const cptr<double> HV = w.hull;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t total = prefix[w.n_pairs];
  for (uint32_t tk = wave; tk < total; tk += n_waves) {
    int lo = 0, hi = w.n_pairs;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (prefix[mid] <= tk) lo = mid;
      else hi = mid;
    }
    const int p = lo;
    const uint32_t ts = prefix[w.n_pairs + 2];
    const uint32_t t0 = (tk - prefix[p]) * ts, t1 = min(seg_len[p], t0 + ts);
    const int a = w.pair_a[p], b = w.pair_b[p];
    for (uint32_t base = t0; base < t1; base += 64) {
      const uint32_t idx = base + lane;
      if (idx >= t1) continue;
      const long long c = cand[seg_start[p] + idx];
      if (!((masks[c * w.W + (p >> 5)] >> (p & 31)) & 1u)) continue;
      double dp = 0.0;
      V3 nd{0, 0, 0}, ps{0, 0, 0};
      if (w.pair_cf[p] == CF_OCTREE) {  // the octree is side b (octree-first pairs are refused on the host)
        const SE3 TA = a < w.n_moving ? moving_tf<FROM_POSES>(w, in, sc, c, a) : load_se3(w.static_T + 12 * (a - w.n_moving));
        const SE3 TB = b < w.n_moving ? moving_tf<FROM_POSES>(w, in, sc, c, b) : load_se3(w.static_T + 12 * (b - w.n_moving));
        const int ga = a < w.n_moving ? w.moving_geom[a] : w.static_geom[a - w.n_moving];
        const int gb = b < w.n_moving ? w.moving_geom[b] : w.static_geom[b - w.n_moving];
        octree_first_contact(w, HV, gb, TB, ga, TA, dp, nd, ps);
      } else if (w.pair_cf[p] == CF_MESH) {
        const SE3 TA = a < w.n_moving ? moving_tf<FROM_POSES>(w, in, sc, c, a) : load_se3(w.static_T + 12 * (a - w.n_moving));
        const SE3 TB = b < w.n_moving ? moving_tf<FROM_POSES>(w, in, sc, c, b) : load_se3(w.static_T + 12 * (b - w.n_moving));
        const int ga = a < w.n_moving ? w.moving_geom[a] : w.static_geom[a - w.n_moving];
        const int gb = b < w.n_moving ? w.moving_geom[b] : w.static_geom[b - w.n_moving];
        mesh_first_contact(w, HV, ga, TA, gb, TB, dp, nd, ps);
      } else if (cf_has_contact(w.pair_cf[p])) {
        const SE3 TA = a < w.n_moving ? moving_tf<FROM_POSES>(w, in, sc, c, a) : load_se3(w.static_T + 12 * (a - w.n_moving));
        const SE3 TB = b < w.n_moving ? moving_tf<FROM_POSES>(w, in, sc, c, b) : load_se3(w.static_T + 12 * (b - w.n_moving));
        const int ga = a < w.n_moving ? w.moving_geom[a] : w.static_geom[a - w.n_moving];
        const int gb = b < w.n_moving ? w.moving_geom[b] : w.static_geom[b - w.n_moving];
        closed_form_contact(w.pair_cf[p], w, ga, TA, gb, TB, dp, nd, ps);
      } else {
        const GObj A = a < w.n_moving ? moving_obj<FROM_POSES>(w, in, sc, c, a) : static_obj(w, a - w.n_moving);
        const GObj B = b < w.n_moving ? moving_obj<FROM_POSES>(w, in, sc, c, b) : static_obj(w, b - w.n_moving);
        mpr_penetration(w, HV, A, B, dp, nd, ps);
      }
      const size_t k = (size_t)c * w.n_pairs + p;
      depth[k] = dp;
      normal[3 * k] = nd.x;
      normal[3 * k + 1] = nd.y;
      normal[3 * k + 2] = nd.z;
      pos[3 * k] = ps.x;
      pos[3 * k + 1] = ps.y;
      pos[3 * k + 2] = ps.z;
    }
  }
}

__global__ void fk_kernel(DevWorld w, const double* __restrict__ q, long long n, double* __restrict__ out) {
  const long long cfg = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (cfg >= n) return;
  FkState st;
  forward_kinematics(w, q + cfg * w.dof, st);
  for (int l = 0; l < w.n_links; ++l) link_transform(w, st, l, out + (cfg * w.n_links + l) * 7);
}

// ---------------------------------------------------------------------------
// Batched motion validation (OMPL DiscreteMotionValidator over the MPlib
// compound state space, src/ompl_planner.cpp:248-293): per edge the segment
// count, the interpolated states, then the per-edge reduction of their flags.
// ---------------------------------------------------------------------------
// ompl::base::SO2StateSpace::distance / RealVectorStateSpace(1)::distance,
// summed with weight 1.0 by CompoundStateSpace::distance
__device__ __forceinline__ double motion_distance(const double* a, const double* b, int dof, uint32_t so2) {
  double d = 0.0;
  for (int i = 0; i < dof; ++i) {
    double di;
    if ((so2 >> i) & 1u) {
      di = std::fabs(a[i] - b[i]);
      di = (di > M_PI) ? 2.0 * M_PI - di : di;
    } else {
      const double diff = a[i] - b[i];
      di = std::sqrt(diff * diff);
    }
    d += 1.0 * di;
  }
  return d;
}

__global__ void motion_count_kernel(const double* __restrict__ from, const double* __restrict__ to, long long n,
                                    int dof, uint32_t so2, double lvs, int32_t* __restrict__ segs) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  // StateSpace::validSegmentCount: factor 1 * (unsigned)ceil(distance / longestValidSegment)
  const unsigned nd = (unsigned)std::ceil(motion_distance(from + e * dof, to + e * dof, dof, so2) / lvs);
  segs[e] = (int32_t)(nd > 1u ? nd : 1u);  // states j/nd, j = 1..nd (s1 is assumed valid)
}

__global__ void motion_states_kernel(const double* __restrict__ from, const double* __restrict__ to, long long n,
                                     int dof, uint32_t so2, const int32_t* __restrict__ segs,
                                     const long long* __restrict__ offs, double* __restrict__ states) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const double* a = from + e * dof;
  const double* b = to + e * dof;
  const int m = segs[e];
  double* out = states + offs[e] * dof;
  for (int j = 1; j <= m; ++j, out += dof) {
    if (j == m) {  // checkMotion tests s2 itself
      for (int i = 0; i < dof; ++i) out[i] = b[i];
      continue;
    }
    const double t = (double)j / (double)m;
    for (int i = 0; i < dof; ++i) {
      if ((so2 >> i) & 1u) {  // SO2StateSpace::interpolate
        double diff = b[i] - a[i];
        double v;
        if (std::fabs(diff) <= M_PI) {
          v = a[i] + diff * t;
        } else {
          diff = diff > 0.0 ? 2.0 * M_PI - diff : -2.0 * M_PI - diff;
          v = a[i] - diff * t;
          if (v > M_PI) v -= 2.0 * M_PI;
          else if (v < -M_PI) v += 2.0 * M_PI;
        }
        out[i] = v;
      } else {  // RealVectorStateSpace::interpolate
        out[i] = a[i] + (b[i] - a[i]) * t;
      }
    }
  }
}

__global__ void motion_reduce_kernel(const uint8_t* __restrict__ flags, long long n, const int32_t* __restrict__ segs,
                                     const long long* __restrict__ offs, uint8_t* __restrict__ valid,
                                     int32_t* __restrict__ first_invalid) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint8_t* f = flags + offs[e];
  int bad = -1;
  for (int j = 0; j < segs[e]; ++j)
    if (f[j]) {
      bad = j + 1;
      break;
    }
  valid[e] = bad < 0 ? 1 : 0;
  if (first_invalid) first_invalid[e] = bad;
}

__global__ void sincos_kernel(const double* __restrict__ x, long long n, double* s, double* c) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  mpg_sincos(x[i], s + i, c + i);
}

// ---------------------------------------------------------------------------
// generate_collision_pair (mplib/planner.py:118-163), batched: random full
// configurations drawn on the device, the pairs collide_full() reports
// counted per pair.
// Sampler: value i (row-major, rows counted from the call's first sample) is
// lo + (hi - lo) * u, u = (splitmix64(seed + (i + 1) * golden) >> 11) * 2^-53
// (mplib_amd/planner.py sample_uniform restates it on the host).
// ---------------------------------------------------------------------------
constexpr int kSampleMaxDof = 64;
struct SampleRange {
  double lo[kSampleMaxDof], hi[kSampleMaxDof];
};

__device__ __forceinline__ double splitmix_u01(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1ull) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

__global__ __launch_bounds__(256) void sample_uniform_kernel(SampleRange r, int dof, long long n, uint64_t seed,
                                                            long long row0, double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * dof) return;
  const int k = (int)(i % dof);
  const double u = splitmix_u01(seed, (uint64_t)(row0 * dof + i));
  out[i] = r.lo[k] + (r.hi[k] - r.lo[k]) * u;
}

// per pair, the configurations whose pair mask has its bit: LDS counters per
// block (atomics on the block's own copy), then one global add per pair
__global__ __launch_bounds__(256) void pair_count_kernel(const uint32_t* __restrict__ masks, long long n, int W,
                                                        int P, unsigned long long* __restrict__ counts) {
  extern __shared__ uint32_t c_lds[];
  for (int p = threadIdx.x; p < P; p += blockDim.x) c_lds[p] = 0u;
  __syncthreads();
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    for (int k = 0; k < W; ++k) {
      uint32_t x = masks[i * W + k];
      while (x) {
        atomicAdd(&c_lds[32 * k + __builtin_ctz(x)], 1u);
        x &= x - 1u;
      }
    }
  __syncthreads();
  for (int p = threadIdx.x; p < P; p += blockDim.x)
    if (c_lds[p]) atomicAdd(&counts[p], (unsigned long long)c_lds[p]);
}

// ---------------------------------------------------------------------------
// Host-buffer pipeline (collide_host_pipelined): the pair-mask rows of the
// colliding configurations only, packed in configuration order and written
// straight into pinned host memory.  flags[i] != 0 exactly when row i has a
// bit (collide() == !collideFull().empty(), planning_world.h:248-250), so the
// host rebuilds the full [m, W] mask from the flags and the packed rows.
// Block b covers configurations [b * kPackCfg, (b + 1) * kPackCfg).
// ---------------------------------------------------------------------------
constexpr int kPackCfg = 4096;

__device__ __forceinline__ int block_sum256(int v, int* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const int s = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(256) void flag_count_kernel(const uint8_t* __restrict__ fl, long long m,
                                                         uint32_t* __restrict__ bcnt, uint32_t* __restrict__ bcnt_host) {
  __shared__ int red[4];
  const long long base = (long long)blockIdx.x * kPackCfg;
  int c = 0;
  for (int r = 0; r < kPackCfg / 256; ++r) {
    const long long i = base + r * 256 + threadIdx.x;
    c += (i < m && fl[i]) ? 1 : 0;
  }
  c = block_sum256(c, red);
  if (threadIdx.x == 0) {
    bcnt[blockIdx.x] = (uint32_t)c;
    bcnt_host[blockIdx.x] = (uint32_t)c;
  }
}

// STAGED: the block's packed rows go through LDS (256 * W words), so each
// store instruction writes consecutive words of host memory; otherwise each
// colliding lane writes its own row (wide masks only)
// The flags go to host memory too (fl_out); W = 0: flags only.
template <bool STAGED>
__global__ __launch_bounds__(256) void mask_pack_kernel(const uint8_t* __restrict__ fl, const uint32_t* __restrict__ mk,
                                                        long long m, int W, const uint32_t* __restrict__ bcnt,
                                                        uint32_t* __restrict__ out, uint8_t* __restrict__ fl_out) {
  extern __shared__ uint32_t pk_lds[];
  __shared__ int red[4];
  __shared__ int wcnt[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int off = 0;
  for (int b = tid; b < (int)blockIdx.x; b += 256) off += (int)bcnt[b];
  long long run = block_sum256(off, red);
  const long long base = (long long)blockIdx.x * kPackCfg;
  for (int r = 0; r < kPackCfg / 256; ++r) {
    const long long i = base + r * 256 + tid;
    if (base + r * 256 >= m) break;  // block-uniform
    const bool f = i < m && fl[i];
    if (i < m) fl_out[i] = f ? 1 : 0;
    if (W == 0) continue;  // block-uniform
    const unsigned long long bal = __ballot(f);
    const int lpos = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wcnt[wv] = __popcll(bal);
    __syncthreads();
    int woff = 0;
    for (int k = 0; k < wv; ++k) woff += wcnt[k];
    const int total = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    if constexpr (STAGED) {
      if (f)
        for (int k = 0; k < W; ++k) pk_lds[(woff + lpos) * W + k] = mk[i * W + k];
      __syncthreads();
      uint32_t* o = out + run * W;
      for (int d = tid; d < total * W; d += 256) o[d] = pk_lds[d];
    } else {
      if (f)
        for (int k = 0; k < W; ++k) out[(run + woff + lpos) * W + k] = mk[i * W + k];
    }
    run += total;
    __syncthreads();
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// host side: snapshot build + C ABI
// ---------------------------------------------------------------------------
struct mpg_world {
  int device = 0;
  DevWorld dw{};
  int n_geoms = 0;
  std::vector<int> geom_type_h;  // host copy of the geometry kinds (diagnostics)
  void* blob = nullptr;
  size_t blob_bytes = 0;
  uint64_t snapshot_hash = 0;  // FNV-1a of the snapshot blob (mpg_collide_batch_multi's same-scene check)
  hipEvent_t gather_ev = nullptr;  // mpg_collide_batch_multi_device: this shard's gather copies are queued
  int block = 128;
  size_t lds_bytes = 0;
  // staging for MPG_MEM_HOST
  std::mutex host_mu;
  double* d_q = nullptr;
  uint8_t* d_flags = nullptr;
  uint32_t* d_masks = nullptr;
  double* d_out = nullptr;
  size_t cap_cfg = 0;
  size_t cap_out = 0;
  // phase A/B workspace, one per stream so concurrent streams never share it
  struct Workspace {
    uint32_t* surv = nullptr;       // [W * cap] survivor bits, word-major
    uint32_t* cnt = nullptr;        // [n_pairs * n_tiles] tile counts -> offsets
    uint32_t* seg_len = nullptr;    // [n_pairs]
    uint32_t* seg_start = nullptr;  // [n_pairs]
    uint32_t* prefix = nullptr;     // [n_pairs + 2] task prefix + task counter
    uint32_t* cand = nullptr;       // [n_pairs * cap] worst case
    float* rq = nullptr;            // [n_moving * 4 * cap] phase-A rotations (quaternions) for the SAT stage
    double* sc = nullptr;           // [cap * dof * 2] exact joint (sin, cos) for phase B
    long long cap = 0;
    uint64_t last = 0;              // LRU tick (get_workspace)
  };
  std::mutex ws_mu;
  std::map<hipStream_t, Workspace> ws;
  // optional per-stage timing (mpg_profile_enable)
  struct Mark {
    int stage;
    hipEvent_t a, b;
  };
  // batched motion validation buffers (grow-only)
  struct Motion {
    double* edges = nullptr;
    size_t edges_cap = 0;
    int32_t* segs = nullptr;
    size_t segs_cap = 0;
    long long* offs = nullptr;
    size_t offs_cap = 0;
    int32_t* out = nullptr;  // staging: first_invalid[n] then valid[n] bytes
    size_t out_cap = 0;
    double* states = nullptr;
    size_t states_cap = 0;
    uint8_t* flags = nullptr;
    size_t flags_cap = 0;
    hipEvent_t last = nullptr;  // the previous call's work (scratch order across streams)
  } motion;
  std::mutex motion_mu;
  bool has_closed_form = false;  // a non-allowed pair uses an FCL closed form
  bool has_octree = false;       // a non-allowed pair involves an octree
  bool octree_first = false;     // a non-allowed pair has its octree as o1 (C ABI only; pymp puts it second)
  bool any_closed_form = false;  // some pair (allowed or not) does, octrees aside
  bool any_octree = false;       // some pair involves an octree
  bool has_mesh = false;         // a non-allowed pair involves a BVH mesh
  bool any_mesh = false;         // some pair involves a BVH mesh
  bool any_gjk = false;          // GST_INDEP world: some pair runs FCL's own GJK (CF_GJK)
  bool has_octree2 = false;      // a non-allowed pair of two OcTrees
  // batched distance buffers (grow-only)
  struct Dist {
    double* poses = nullptr;
    size_t poses_cap = 0;
    double* save64 = nullptr;
    size_t save_cap = 0;
    double* q = nullptr;
    size_t q_cap = 0;
    char* out = nullptr;
    size_t out_cap = 0;
    double* pts = nullptr;  // device-buffer calls: points nobody asked for
    size_t pts_cap = 0;
    hipEvent_t last = nullptr;  // the previous call's work (scratch order across streams)
    ccdx::BigPolytope* big = nullptr;  // kBigPool EPA polytopes (distance_redo_kernel)
    size_t big_cap = 0;
    unsigned* list = nullptr;  // overflowed configurations: [count, ids...]
    size_t list_cap = 0;
  } dist;
  // host-buffer contact calls: grow-only device staging (guarded by host_mu)
  struct ContactStage {
    double *in = nullptr, *out = nullptr;
    uint8_t* fl = nullptr;
    uint32_t* mk = nullptr;
    size_t in_cap = 0, out_cap = 0, fl_cap = 0, mk_cap = 0;
  } contact;
  std::mutex dist_mu;
  std::mutex prof_mu;
  bool prof = false;
  std::vector<Mark> marks;
  std::vector<hipEvent_t> ev_pool;
  double prof_ms[MPG_NUM_STAGES] = {0, 0, 0};
  int64_t prof_n[MPG_NUM_STAGES] = {0, 0, 0};
  int64_t prof_cfg = 0;                       // configurations launched while profiling
  unsigned long long* prof_units = nullptr;   // device counter: narrow candidates
  long long max_chunk = 1 << 20;
  int narrow_blocks = 1024;
  // large batches: two halves, the second on an internal stream, so one
  // half's latency-bound bucketing overlaps the other's compute
  long long overlap_min = 1 << 18;  // 0 disables (env MPG_OVERLAP_MIN)
  int overlap_parts = 2;             // env MPG_OVERLAP_PARTS
  // large batches: half of the parts on a side stream (per caller stream)
  struct Side {
    hipStream_t side;
    hipEvent_t fork, join;
    uint64_t last;
  };
  std::map<hipStream_t, Side> sides;  // guarded by ws_mu
  // per-stream state (workspaces, side streams) is kept for at most
  // kMaxStreamState caller streams, least recently used evicted first;
  // mpg_release_stream drops one explicitly
  static constexpr size_t kMaxStreamState = 32;
  uint64_t ws_tick = 0;
  // caller streams with a call in progress (StreamPin): never evicted, so no
  // thread frees a workspace or side stream another thread is using
  std::map<hipStream_t, int> busy;  // guarded by ws_mu
  // small-batch latency path (host buffers, n <= small_max): pinned input
  // staging + host-mapped hit bytes written by small_kernel
  long long small_max = 1024;
  double* h_q = nullptr;       // pinned, [small cap * row]
  uint8_t* h_hits = nullptr;   // pinned coherent host-mapped, [n_pairs * small cap]
  uint8_t* d_hits = nullptr;   // device alias of h_hits
  double* d_qs = nullptr;      // device input of the latency path
  double* d_qmap = nullptr;    // h_q as the device sees it (zero-copy input)
  double* d_ssc = nullptr;     // latency path joint (sin, cos) [small cap * dof * 2]
  double* h_ssc = nullptr;     // pinned host-mapped twin: sin/cos computed on the host (small batches)
  double* d_sscmap = nullptr;  // h_ssc as the device sees it
  int64_t small_host_sc = 64;  // latency batches up to this size: sin/cos on the host (MPG_SMALL_HOST_SC)
  bool small_args = true;      // the fewest states' rows in the kernel arguments (MPG_SMALL_ARGS=0: off)
  std::vector<int> h_rev_src;  // move-group slots of revolute joints (host copy of the snapshot's rule)
  // host-buffer calls without a stream run on this non-blocking stream (not
  // the legacy default stream, whose synchronisation covers every blocking
  // stream of the device); MPG_OWN_STREAM=0 keeps the caller's NULL stream
  hipStream_t own_stream = nullptr;
  bool small_zero_copy = true; // MPG_SMALL_ZEROCOPY=0: stage through d_qs
  int64_t small_inline_sc = 256;  // latency batches up to this size: sin/cos inline (MPG_SMALL_INLINE_SC)
  // latency server (lat_server_kernel): control block in host-mapped memory,
  // its own stream; started on demand, leaves after srv_idle_us idle
  SrvCtl* srv_h = nullptr;
  SrvCtl* srv_d = nullptr;
  hipStream_t srv_stream = nullptr;
  unsigned long long srv_seq = 0;
  bool srv_running = false;
  bool srv_ok = false;      // the world fits the server (closed-form / MPR pairs only, records, LDS)
  bool srv_broken = false;  // it failed to answer: launches until srv_retry_at
  std::chrono::steady_clock::time_point srv_retry_at{};
  bool srv_quitting = false;  // quit was set after a missed answer; the stream may still run
  int64_t srv_served = 0, srv_starts = 0, srv_fallbacks = 0;  // mpg_latency_server_stats
  int srv_mode = 1;         // MPG_SMALL_SERVER=0: off
  long long srv_idle_us = 1000;
  int srv_g = 8;            // workgroups (MPG_SMALL_SERVER_WG)
  int srv_max_n = kSrvN;    // batches up to this size go to the server (MPG_SMALL_SERVER_MAX)
  size_t srv_lds = 0;
  bool srv_stats = false;
  double srv_stat[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  size_t small_cap = 0;   // configurations (hit bytes per pair)
  size_t small_qcap = 0;  // input doubles (h_q, d_qs)
  // host-buffer batches above small_max (collide_host_pipelined): chunks
  // through a ring of slots -- the input of one chunk crosses PCIe while the
  // previous one computes and the one before is unpacked on the host.
  // Grow-only, guarded by host_mu.
  static constexpr int kRing = 3;
  struct Ring {
    double* d_in[kRing] = {};
    uint8_t* d_fl[kRing] = {};
    uint32_t* d_mk[kRing] = {};
    uint32_t* d_bcnt[kRing] = {};  // colliding configurations per kPackCfg block
    uint8_t* h_fl[kRing] = {};     // pinned, host-mapped: the chunk's flags (mask_pack_kernel)
    uint32_t* h_mk[kRing] = {};    // pinned, host-mapped: packed mask rows (mask_pack_kernel)
    uint32_t* h_mk_d[kRing] = {};  // h_mk as the device sees it
    uint32_t* h_bcnt[kRing] = {};  // pinned, host-mapped copy of d_bcnt (where each block's packed rows start)
    uint8_t* h_fl_d[kRing] = {};   // device aliases of h_fl, h_bcnt
    uint32_t* h_bcnt_d[kRing] = {};
    hipEvent_t e_in[kRing] = {}, e_done[kRing] = {};
    hipStream_t h2d = nullptr;     // input copies
    hipStream_t side = nullptr;    // odd chunks compute here (one chunk's narrow tail overlaps the next's cull)
    size_t cap = 0;                // configurations per slot
    size_t in_cap = 0;             // input doubles per slot
  } ring;
  // chunk sizes: profiles/r06a/host_ab*.txt (2^18 / 2^19 chunks, head and
  // tail sizes within +-3 % of each other on cfg3 2^20; this is the best seen)
  long long ring_chunk = 1 << 19;  // largest chunk (env MPG_HOST_CHUNK)
  int ring_streams = 2;            // compute streams of the pipeline (env MPG_HOST_STREAMS: 1 or 2)
  int host_threads = 8;            // threads unpacking a finished chunk (env MPG_HOST_THREADS)
  long long ring_head = 1 << 17, ring_tail = 1 << 16;  // smaller first / last chunk (env MPG_HOST_HEAD / _TAIL)
  std::unique_ptr<mpg_hostpipe::Pool> pool;
  // MPG_STATS: host pipeline phase sums (us): calls, input copy, issue,
  // result wait, unpack, whole call
  double hp_stat[6] = {0, 0, 0, 0, 0, 0};
};

namespace {

// Spatial clusters of one mesh's triangle records: the leaves of a median
// split (centroids, longest axis) with at most `leaf` triangles each, in
// order; triangle k of the clusters' ranges is rec[order[k]].
void mesh_build_clusters(const std::vector<double>& rec, std::vector<int>& order, int lo, int hi, int leaf, int rec0,
                         std::vector<double>& box, std::vector<int>& link) {
  auto cen = [&](int t, int k) {
    const double* r = rec.data() + (size_t)TR_STRIDE * t;
    return r[TR_LO + k] + r[TR_HI + k];
  };
  if (hi - lo <= leaf) {
    double blo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, bhi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    for (int i = lo; i < hi; ++i) {
      const double* r = rec.data() + (size_t)TR_STRIDE * order[i];
      for (int k = 0; k < 3; ++k) {
        blo[k] = std::min(blo[k], r[TR_LO + k]);
        bhi[k] = std::max(bhi[k], r[TR_HI + k]);
      }
    }
    box.insert(box.end(), {blo[0], blo[1], blo[2], bhi[0], bhi[1], bhi[2]});
    link.insert(link.end(), {rec0 + lo, hi - lo});
    return;
  }
  double clo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, chi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
  for (int i = lo; i < hi; ++i)
    for (int k = 0; k < 3; ++k) {
      clo[k] = std::min(clo[k], cen(order[i], k));
      chi[k] = std::max(chi[k], cen(order[i], k));
    }
  int ax = 0;
  for (int k = 1; k < 3; ++k)
    if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
  const int mid = (lo + hi) / 2;
  std::nth_element(order.begin() + lo, order.begin() + mid, order.begin() + hi,
                   [&](int a, int b) { return cen(a, ax) < cen(b, ax) || (cen(a, ax) == cen(b, ax) && a < b); });
  mesh_build_clusters(rec, order, lo, mid, leaf, rec0, box, link);
  mesh_build_clusters(rec, order, mid, hi, leaf, rec0, box, link);
}

struct BlobBuilder {
  std::vector<char> bytes;
  template <class T>
  size_t add(const T* data, size_t count) {
    size_t off = (bytes.size() + 15) & ~size_t(15);
    bytes.resize(off + sizeof(T) * std::max<size_t>(count, 1), 0);
    if (count) std::memcpy(bytes.data() + off, data, sizeof(T) * count);
    return off;
  }
};

bool finite_all(const double* p, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (!std::isfinite(p[i])) return false;
  return true;
}

int obj_geom_type(const mpg_world_desc* d, int id) {
  return d->geom_type[id < d->n_moving ? d->moving_geom[id] : d->static_geom[id - d->n_moving]];
}

// FCL closed-form pair for (o1, o2) in fcl::collide argument order
int closed_form_kind(const mpg_world_desc* d, int a, int b) {
  const int ta = obj_geom_type(d, a), tb = obj_geom_type(d, b);
  if (ta == MPG_GEOM_MESH || tb == MPG_GEOM_MESH) return CF_MESH;
  if (ta == MPG_GEOM_OCTREE || tb == MPG_GEOM_OCTREE) return CF_OCTREE;
  if (ta == MPG_GEOM_BOX && tb == MPG_GEOM_BOX) return CF_BOX_BOX;
  if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_SPHERE) return CF_SPHERE_SPHERE;
  if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_BOX) return CF_SPHERE_BOX;
  if (ta == MPG_GEOM_BOX && tb == MPG_GEOM_SPHERE) return CF_BOX_SPHERE;
  if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_CAPSULE) return CF_SPHERE_CAPSULE;
  if (ta == MPG_GEOM_CAPSULE && tb == MPG_GEOM_SPHERE) return CF_CAPSULE_SPHERE;
  if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_CYLINDER) return CF_SPHERE_CYLINDER;
  if (ta == MPG_GEOM_CYLINDER && tb == MPG_GEOM_SPHERE) return CF_CYLINDER_SPHERE;
  return CF_NONE;
}

int validate(const mpg_world_desc* d) {
  if (!d) return set_error(MPG_E_INVALID, "desc is NULL");
  if (d->gjk_solver != MPG_GJK_LIBCCD && d->gjk_solver != MPG_GJK_INDEP)
    return set_error(MPG_E_INVALID, "gjk_solver must be MPG_GJK_LIBCCD or MPG_GJK_INDEP");
  if (d->n_joints < 0 || d->n_joints > kMaxJoints) return set_error(MPG_E_INVALID, "n_joints out of range [0, 32]");
  if (d->dof < 0) return set_error(MPG_E_INVALID, "dof < 0");
  if (d->n_links < 0 || d->n_geoms < 0 || d->n_moving < 0 || d->n_static < 0 || d->n_pairs < 0)
    return set_error(MPG_E_INVALID, "negative count");
  for (int j = 0; j < d->n_joints; ++j) {
    if (d->joint_type[j] < 0 || d->joint_type[j] > MPG_JOINT_RUB_UNALIGNED)
      return set_error(MPG_E_INVALID, "bad joint type");
    if (d->joint_parent[j] < 0 || d->joint_parent[j] > j)
      return set_error(MPG_E_INVALID, "joint_parent must reference an earlier joint (0 = universe)");
    if (d->joint_q_source[j] >= d->dof) return set_error(MPG_E_INVALID, "joint_q_source >= dof");
  }
  for (int l = 0; l < d->n_links; ++l)
    if (d->link_parent[l] < 0 || d->link_parent[l] > d->n_joints) return set_error(MPG_E_INVALID, "bad link_parent");
  for (int g = 0; g < d->n_geoms; ++g) {
    const int t = d->geom_type[g];
    if (t < MPG_GEOM_CONVEX || t > MPG_GEOM_TRIANGLE) return set_error(MPG_E_UNSUPPORTED, "unsupported geometry type");
    if (t == MPG_GEOM_TRIANGLE && (d->geom_vertex_count[g] != 3 || d->geom_vertex_start[g] < 0 ||
                                   (int64_t)d->geom_vertex_start[g] + 3 > d->n_vertices))
      return set_error(MPG_E_INVALID, "a TriangleP needs 3 vertices inside the vertex array");
    if (t == MPG_GEOM_ELLIPSOID || t == MPG_GEOM_CONE) {
      const double* p = d->geom_param + 4 * g;
      const int np = t == MPG_GEOM_ELLIPSOID ? 3 : 2;
      for (int k = 0; k < np; ++k)
        if (!(p[k] > 0.0 && std::isfinite(p[k])))
          return set_error(MPG_E_INVALID, "ellipsoid radii / cone radius and lz must be positive and finite");
    }
    if (t == MPG_GEOM_CONVEX || t == MPG_GEOM_MESH) {
      if (d->geom_vertex_count[g] <= 0 || d->geom_vertex_start[g] < 0 ||
          (int64_t)d->geom_vertex_start[g] + d->geom_vertex_count[g] > d->n_vertices)
        return set_error(MPG_E_INVALID, "convex vertex range out of bounds");
    }
    if (t == MPG_GEOM_CONVEX) {  // faces (FCL layout) inside convex_face, indices inside the hull
      const double f0 = d->geom_param[4 * g], fn = d->geom_param[4 * g + 1];
      if (!(f0 >= 0 && fn >= 0 && f0 == std::floor(f0) && fn == std::floor(fn)))
        return set_error(MPG_E_INVALID, "convex face range out of bounds");
      if (fn > 0) {
        if (!d->convex_face) return set_error(MPG_E_INVALID, "bad convex face array");
        int64_t i = (int64_t)f0;
        for (int64_t f = 0; f < (int64_t)fn; ++f) {
          if (i >= d->n_convex_face_ints) return set_error(MPG_E_INVALID, "convex face range out of bounds");
          const int cnt = d->convex_face[i];
          if (cnt < 1 || i + cnt >= d->n_convex_face_ints) return set_error(MPG_E_INVALID, "convex face range out of bounds");
          for (int k = 1; k <= cnt; ++k)
            if (d->convex_face[i + k] < 0 || d->convex_face[i + k] >= d->geom_vertex_count[g])
              return set_error(MPG_E_INVALID, "convex face vertex index out of range");
          i += cnt + 1;
        }
      }
    }
    if (t == MPG_GEOM_MESH) {
      const double t0 = d->geom_param[4 * g], tn = d->geom_param[4 * g + 1];
      if (!(t0 >= 0 && tn >= 0 && t0 == std::floor(t0) && tn == std::floor(tn) && t0 + tn <= (double)d->n_mesh_triangles))
        return set_error(MPG_E_INVALID, "mesh triangle range out of bounds");
      if (tn > 0 && !d->mesh_triangle) return set_error(MPG_E_INVALID, "bad mesh triangle array");
      for (int64_t i = (int64_t)t0; i < (int64_t)(t0 + tn); ++i)
        for (int k = 0; k < 3; ++k)
          if (d->mesh_triangle[3 * i + k] < 0 || d->mesh_triangle[3 * i + k] >= d->geom_vertex_count[g])
            return set_error(MPG_E_INVALID, "mesh triangle vertex index out of range");
    }
  }
  for (int m = 0; m < d->n_moving; ++m) {
    if (d->moving_link[m] < 0 || d->moving_link[m] >= d->n_links) return set_error(MPG_E_INVALID, "bad moving_link");
    if (d->moving_geom[m] < 0 || d->moving_geom[m] >= d->n_geoms) return set_error(MPG_E_INVALID, "bad moving_geom");
  }
  if (d->n_mesh_triangles < 0 || (d->n_mesh_triangles > 0 && !d->mesh_triangle))
    return set_error(MPG_E_INVALID, "bad mesh triangle array");
  if (d->n_octree_leaves < 0 || (d->n_octree_leaves > 0 && !d->octree_leaf))
    return set_error(MPG_E_INVALID, "bad octree leaf array");
  for (int g = 0; g < d->n_geoms; ++g) {
    if (d->geom_type[g] != MPG_GEOM_OCTREE) continue;
    const double l0 = d->geom_param[4 * g], ln = d->geom_param[4 * g + 1];
    if (!(l0 >= 0 && ln >= 0 && l0 == std::floor(l0) && ln == std::floor(ln) && l0 + ln <= (double)d->n_octree_leaves))
      return set_error(MPG_E_INVALID, "octree leaf range out of bounds");
  }
  if (!finite_all(d->octree_leaf, 6 * (size_t)d->n_octree_leaves))
    return set_error(MPG_E_INVALID, "non-finite octree leaf");
  for (int s = 0; s < d->n_static; ++s)
    if (d->static_geom[s] < 0 || d->static_geom[s] >= d->n_geoms) return set_error(MPG_E_INVALID, "bad static_geom");
  const int nobj = d->n_moving + d->n_static;
  for (int p = 0; p < d->n_pairs; ++p) {
    const int a = d->pair_a[p], b = d->pair_b[p];
    if (a < 0 || a >= nobj || b < 0 || b >= nobj) return set_error(MPG_E_INVALID, "pair object id out of range");
    if (a >= d->n_moving && b >= d->n_moving) return set_error(MPG_E_INVALID, "static-static pair");
    // an OcTree may ride on a link or an attached body (attachObject takes any
    // FCL geometry, planning_world.cpp:174-191), and meet another OcTree
    // (octree_octree_wave; its contacts and distance are refused per call)
    // FCL 0.7.0 GJKSolver_libccd: box-box, sphere-sphere, sphere-box,
    // sphere-capsule and sphere-cylinder have closed forms (all on the
    // device, closed_form_kind); every other shape pair is MPR
    if (!(d->pair_allowed && d->pair_allowed[p])) {
      const int ta = obj_geom_type(d, a), tb = obj_geom_type(d, b);
      const bool tri = ta == MPG_GEOM_TRIANGLE || tb == MPG_GEOM_TRIANGLE;
      if (tri && (ta == MPG_GEOM_MESH || tb == MPG_GEOM_MESH || ta == MPG_GEOM_OCTREE || tb == MPG_GEOM_OCTREE))
        return set_error(MPG_E_UNSUPPORTED, "a TriangleP paired with an OcTree or BVH mesh is not implemented");
    }
    if (d->gjk_solver == MPG_GJK_INDEP && !(d->pair_allowed && d->pair_allowed[p])) {
      const int ta = obj_geom_type(d, a), tb = obj_geom_type(d, b);
      if (ta == MPG_GEOM_MESH || tb == MPG_GEOM_MESH || ta == MPG_GEOM_OCTREE || tb == MPG_GEOM_OCTREE)
        return set_error(MPG_E_UNSUPPORTED,
                         "gjk_solver MPG_GJK_INDEP with an OcTree or BVH mesh in a pair is not implemented");
    }
  }
  if (!finite_all(d->joint_placement, 12 * (size_t)d->n_joints) || !finite_all(d->link_placement, 12 * (size_t)d->n_links) ||
      !finite_all(d->vertices, 3 * (size_t)d->n_vertices))
    return set_error(MPG_E_INVALID, "non-finite value in descriptor");
  if (!(d->gjk_tolerance > 0)) return set_error(MPG_E_INVALID, "gjk_tolerance must be > 0");
  return MPG_OK;
}

void geom_record(const mpg_world_desc* d, int g, double* rec) {
  for (int k = 0; k < G_STRIDE; ++k) rec[k] = 0.0;
  for (int k = 0; k < 4; ++k) rec[G_PARAM + k] = d->geom_param[4 * g + k];
  const int t = d->geom_type[g];
  double lo[3], hi[3];
  if (t == MPG_GEOM_CONVEX || t == MPG_GEOM_MESH) {
    const double* V = d->vertices + 3 * (size_t)d->geom_vertex_start[g];
    const int nv = d->geom_vertex_count[g];
    // FCL 0.7.0 Convex: interior point = (sum of vertices) * (1.0 / n)
    double s[3] = {0.0, 0.0, 0.0};
    for (int i = 0; i < nv; ++i) {
      s[0] += V[3 * i];
      s[1] += V[3 * i + 1];
      s[2] += V[3 * i + 2];
    }
    const double inv = 1.0 / (double)nv;
    for (int k = 0; k < 3; ++k) rec[G_INTERIOR + k] = s[k] * inv;
    for (int k = 0; k < 3; ++k) lo[k] = hi[k] = V[k];
    for (int i = 1; i < nv; ++i)
      for (int k = 0; k < 3; ++k) {
        lo[k] = std::min(lo[k], V[3 * i + k]);
        hi[k] = std::max(hi[k], V[3 * i + k]);
      }
  } else if (t == MPG_GEOM_BOX) {
    for (int k = 0; k < 3; ++k) {
      hi[k] = d->geom_param[4 * g + k] / 2.0;
      lo[k] = -hi[k];
    }
  } else if (t == MPG_GEOM_SPHERE) {
    for (int k = 0; k < 3; ++k) {
      hi[k] = d->geom_param[4 * g];
      lo[k] = -hi[k];
    }
  } else if (t == MPG_GEOM_TRIANGLE) {  // triCreateGJKObject: centre ((a + b) + c) / 3
    const double* V = d->vertices + 3 * (size_t)d->geom_vertex_start[g];
    for (int k = 0; k < 3; ++k) {
      rec[G_INTERIOR + k] = (V[k] + V[3 + k] + V[6 + k]) / 3;
      lo[k] = std::min(V[k], std::min(V[3 + k], V[6 + k]));
      hi[k] = std::max(V[k], std::max(V[3 + k], V[6 + k]));
    }
  } else if (t == MPG_GEOM_ELLIPSOID) {
    for (int k = 0; k < 3; ++k) {
      hi[k] = d->geom_param[4 * g + k];
      lo[k] = -hi[k];
    }
  } else if (t == MPG_GEOM_OCTREE) {  // union of the occupied leaf boxes (octree frame)
    const int64_t l0 = (int64_t)d->geom_param[4 * g], ln = (int64_t)d->geom_param[4 * g + 1];
    for (int k = 0; k < 3; ++k) {
      lo[k] = ln > 0 ? DBL_MAX : 0.0;
      hi[k] = ln > 0 ? -DBL_MAX : 0.0;
    }
    for (int64_t i = l0; i < l0 + ln; ++i)
      for (int k = 0; k < 3; ++k) {
        lo[k] = std::min(lo[k], d->octree_leaf[6 * i + k]);
        hi[k] = std::max(hi[k], d->octree_leaf[6 * i + 3 + k]);
      }
  } else {  // capsule / cylinder / cone along z
    const double r = d->geom_param[4 * g], hz = d->geom_param[4 * g + 1] / 2.0 + (t == MPG_GEOM_CAPSULE ? r : 0.0);
    lo[0] = lo[1] = -r;
    hi[0] = hi[1] = r;
    lo[2] = -hz;
    hi[2] = hz;
  }
  // local box, widened by a relative epsilon so rounding never shrinks it
  double r2 = 0.0;
  for (int k = 0; k < 3; ++k) {
    const double c = 0.5 * (lo[k] + hi[k]);
    const double e = 0.5 * (hi[k] - lo[k]);
    rec[G_OBB_C + k] = c;
    rec[G_OBB_E + k] = e * (1.0 + 1e-12) + 1e-12;
    rec[G_AABB_E + k] = (hi[k] - lo[k]) * 0.5;
    r2 += rec[G_OBB_E + k] * rec[G_OBB_E + k];
  }
  if (t == MPG_GEOM_CONVEX || t == MPG_GEOM_MESH || t == MPG_GEOM_TRIANGLE) {  // bounding sphere about the box centre: farthest vertex
    const double* V = d->vertices + 3 * (size_t)d->geom_vertex_start[g];
    r2 = 0.0;
    for (int i = 0; i < d->geom_vertex_count[g]; ++i) {
      double s2 = 0.0;
      for (int k = 0; k < 3; ++k) {
        const double dv = V[3 * i + k] - rec[G_OBB_C + k];
        s2 += dv * dv;
      }
      r2 = std::max(r2, s2);
    }
  }
  rec[G_RADIUS] = std::sqrt(r2) * (1.0 + 1e-12) + 1e-12;
  double vmax = 0.0;
  if (t == MPG_GEOM_CONVEX) {
    const double* V = d->vertices + 3 * (size_t)d->geom_vertex_start[g];
    for (int i = 0; i < 3 * d->geom_vertex_count[g]; ++i) vmax = std::max(vmax, std::fabs(V[i]));
  }
  rec[G_VMAX] = vmax;
}

// ---------------------------------------------------------------------------
// FCL 0.7.0 BVHModel<OBBRSS>::endModel -> buildTree for the meshes
// (load_mesh_as_BVH, src/urdf_utils.cpp:136-155) [ext FCL BVH_model-inl.h,
// BV_fitter-inl.h, BV_splitter-inl.h, math/geometry-inl.h; restated, FCL is
// not under /root/reference]: BVFitter<OBBRSS>::fit (covariance of the
// node's triangle vertices, Jacobi eigen_old, axisFromEigen, extent and
// centre of the projections; only the OBB half decides collisions), the
// SPLIT_METHOD_MEAN rule along the first axis (centroid . axis > mean goes
// right, the rest are swapped to the front; an empty side -> n / 2), child
// pairs allocated at num_bvs before recursing.  The oracle builds the same
// tree from its own code (oracle/collide_oracle.c orc_bvh_build).
// ---------------------------------------------------------------------------
struct FclBvh {
  std::vector<double> box;  // [n][FB_STRIDE]
  std::vector<int> link;    // [n][3]
  int max_depth = 0;        // deepest leaf (root = 0), bounds the device gates' descent
};

// eigen_old: Jacobi rotations; vout(r, c) = v[c][r], dout = eigenvalues
void fcl_eigen_old(const double m[9], double dout[3], double vout[9]) {
  double R[3][3] = {{m[0], m[1], m[2]}, {m[3], m[4], m[5]}, {m[6], m[7], m[8]}};
  double b[3], z[3], v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}, d[3];
  for (int ip = 0; ip < 3; ++ip) {
    b[ip] = d[ip] = R[ip][ip];
    z[ip] = 0;
  }
  for (int i = 0; i < 50; ++i) {
    double sm = 0;
    for (int ip = 0; ip < 3; ++ip)
      for (int iq = ip + 1; iq < 3; ++iq) sm += std::fabs(R[ip][iq]);
    if (sm == 0.0) {
      for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) vout[3 * r + c] = v[c][r];
      for (int k = 0; k < 3; ++k) dout[k] = d[k];
      return;
    }
    const double tresh = i < 3 ? 0.2 * sm / (3 * 3) : 0.0;
    for (int ip = 0; ip < 3; ++ip)
      for (int iq = ip + 1; iq < 3; ++iq) {
        double g = 100.0 * std::fabs(R[ip][iq]);
        if (i > 3 && std::fabs(d[ip]) + g == std::fabs(d[ip]) && std::fabs(d[iq]) + g == std::fabs(d[iq])) {
          R[ip][iq] = 0.0;
        } else if (std::fabs(R[ip][iq]) > tresh) {
          double h = d[iq] - d[ip], t;
          if (std::fabs(h) + g == std::fabs(h)) {
            t = R[ip][iq] / h;
          } else {
            const double theta = 0.5 * h / R[ip][iq];
            t = 1.0 / (std::fabs(theta) + std::sqrt(1.0 + theta * theta));
            if (theta < 0.0) t = -t;
          }
          const double c = 1.0 / std::sqrt(1 + t * t), s = t * c, tau = s / (1.0 + c);
          h = t * R[ip][iq];
          z[ip] -= h;
          z[iq] += h;
          d[ip] -= h;
          d[iq] += h;
          R[ip][iq] = 0.0;
          auto rot = [&](double& x, double& y) {
            const double gg = x, hh = y;
            x = gg - s * (hh + gg * tau);
            y = hh + s * (gg - hh * tau);
          };
          for (int j = 0; j < ip; ++j) rot(R[j][ip], R[j][iq]);
          for (int j = ip + 1; j < iq; ++j) rot(R[ip][j], R[j][iq]);
          for (int j = iq + 1; j < 3; ++j) rot(R[ip][j], R[iq][j]);
          for (int j = 0; j < 3; ++j) rot(v[j][ip], v[j][iq]);
        }
      }
    for (int ip = 0; ip < 3; ++ip) {
      b[ip] += z[ip];
      d[ip] = b[ip];
      z[ip] = 0.0;
    }
  }
}

// covariance sums -> M -> eigen -> axisFromEigen -> extent / centre of pts
void fcl_fit_obb(const double S1[3], const double S2[6], double n_points, const std::vector<const double*>& pts,
                 double* box) {
  double M[9], E[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, ev[3] = {0, 0, 0};
  M[0] = S2[0] - S1[0] * S1[0] / n_points;
  M[4] = S2[1] - S1[1] * S1[1] / n_points;
  M[8] = S2[2] - S1[2] * S1[2] / n_points;
  M[1] = M[3] = S2[3] - S1[0] * S1[1] / n_points;
  M[5] = M[7] = S2[5] - S1[1] * S1[2] / n_points;
  M[2] = M[6] = S2[4] - S1[0] * S1[2] / n_points;
  fcl_eigen_old(M, ev, E);
  int mn, mid, mx;
  if (ev[0] > ev[1]) {
    mx = 0;
    mn = 1;
  } else {
    mn = 0;
    mx = 1;
  }
  if (ev[2] < ev[mn]) {
    mid = mn;
    mn = 2;
  } else if (ev[2] > ev[mx]) {
    mid = mx;
    mx = 2;
  } else {
    mid = 2;
  }
  double* ax = box + FB_AXIS;
  for (int r = 0; r < 3; ++r) {
    ax[3 * r] = E[3 * mx + r];
    ax[3 * r + 1] = E[3 * mid + r];
  }
  ax[2] = ax[3] * ax[7] - ax[6] * ax[4];
  ax[5] = ax[6] * ax[1] - ax[0] * ax[7];
  ax[8] = ax[0] * ax[4] - ax[3] * ax[1];
  double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
  for (const double* p : pts)
    for (int k = 0; k < 3; ++k) {
      const double pr = (ax[k] * p[0] + ax[3 + k] * p[1]) + ax[6 + k] * p[2];
      if (pr > hi[k]) hi[k] = pr;
      if (pr < lo[k]) lo[k] = pr;
    }
  double o[3];
  for (int k = 0; k < 3; ++k) o[k] = (hi[k] + lo[k]) / 2;
  for (int i = 0; i < 3; ++i) box[FB_TO + i] = (ax[3 * i] * o[0] + ax[3 * i + 1] * o[1]) + ax[3 * i + 2] * o[2];
  for (int k = 0; k < 3; ++k) box[FB_EXT + k] = (hi[k] - lo[k]) * 0.5;
}

void fcl_bvh_node(FclBvh& B, const double* V, const int32_t* tri, std::vector<int>& prim, int id, int first, int n,
                  int base, int depth = 0) {
  if (depth > B.max_depth) B.max_depth = depth;
  int* cur = prim.data() + first;
  double S1[3] = {0, 0, 0}, S2[6] = {0, 0, 0, 0, 0, 0};
  std::vector<const double*> pts;
  pts.reserve(3 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    const int32_t* t = tri + 3 * cur[i];
    const double *p1 = V + 3 * t[0], *p2 = V + 3 * t[1], *p3 = V + 3 * t[2];
    for (int k = 0; k < 3; ++k) S1[k] += (p1[k] + p2[k]) + p3[k];
    S2[0] += (p1[0] * p1[0] + p2[0] * p2[0]) + p3[0] * p3[0];
    S2[1] += (p1[1] * p1[1] + p2[1] * p2[1]) + p3[1] * p3[1];
    S2[2] += (p1[2] * p1[2] + p2[2] * p2[2]) + p3[2] * p3[2];
    S2[3] += (p1[0] * p1[1] + p2[0] * p2[1]) + p3[0] * p3[1];
    S2[4] += (p1[0] * p1[2] + p2[0] * p2[2]) + p3[0] * p3[2];
    S2[5] += (p1[1] * p1[2] + p2[1] * p2[2]) + p3[1] * p3[2];
    pts.push_back(p1);
    pts.push_back(p2);
    pts.push_back(p3);
  }
  double* box = B.box.data() + (size_t)FB_STRIDE * (base + id);
  fcl_fit_obb(S1, S2, 3.0 * n, pts, box);
  int* lk = B.link.data() + 3 * (size_t)(base + id);
  lk[1] = first;
  lk[2] = n;
  if (n == 1) {
    lk[0] = -(cur[0] + 1);
    return;
  }
  const double sv[3] = {box[FB_AXIS], box[FB_AXIS + 3], box[FB_AXIS + 6]};
  double c[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i) {
    const int32_t* t = tri + 3 * cur[i];
    for (int k = 0; k < 3; ++k) c[k] += (V[3 * t[0] + k] + V[3 * t[1] + k]) + V[3 * t[2] + k];
  }
  const double split = ((c[0] * sv[0] + c[1] * sv[1]) + c[2] * sv[2]) / (3 * n);
  const int child = (int)(B.link.size() / 3) - base;  // num_bvs
  lk[0] = base + child;
  B.box.resize(B.box.size() + 2 * FB_STRIDE);
  B.link.resize(B.link.size() + 6);
  int c1 = 0;
  for (int i = 0; i < n; ++i) {
    const int32_t* t = tri + 3 * cur[i];
    double p[3];
    for (int k = 0; k < 3; ++k) p[k] = ((V[3 * t[0] + k] + V[3 * t[1] + k]) + V[3 * t[2] + k]) / 3.0;
    if (!(((sv[0] * p[0] + sv[1] * p[1]) + sv[2] * p[2]) > split)) std::swap(cur[i], cur[c1++]);
  }
  if (c1 == 0 || c1 == n) c1 = n / 2;
  fcl_bvh_node(B, V, tri, prim, child, first, c1, base, depth + 1);
  fcl_bvh_node(B, V, tri, prim, child + 1, first + c1, n - c1, base, depth + 1);
}

// computeBV<OBB>(shape, identity): box I / side/2; sphere I / r; capsule
// I / (r, r, lz/2 + r); cylinder and cone I / (r, r, lz/2); ellipsoid I /
// radii; convex: fitn over the
// vertices (covariance of the points)
void fcl_shape_obb(const mpg_world_desc* d, int g, double* o) {
  std::fill(o, o + FB_STRIDE, 0.0);
  o[FB_AXIS] = o[FB_AXIS + 4] = o[FB_AXIS + 8] = 1.0;
  const double* p = d->geom_param + 4 * g;
  switch (d->geom_type[g]) {
    case MPG_GEOM_BOX:
      for (int k = 0; k < 3; ++k) o[FB_EXT + k] = p[k] * 0.5;
      break;
    case MPG_GEOM_SPHERE:
      o[FB_EXT] = o[FB_EXT + 1] = o[FB_EXT + 2] = p[0];
      break;
    case MPG_GEOM_CAPSULE:
      o[FB_EXT] = o[FB_EXT + 1] = p[0];
      o[FB_EXT + 2] = p[1] / 2 + p[0];
      break;
    case MPG_GEOM_CYLINDER:
    case MPG_GEOM_CONE:
      o[FB_EXT] = o[FB_EXT + 1] = p[0];
      o[FB_EXT + 2] = p[1] / 2;
      break;
    case MPG_GEOM_ELLIPSOID:
      for (int k = 0; k < 3; ++k) o[FB_EXT + k] = p[k];
      break;
    case MPG_GEOM_CONVEX: {
      const double* V = d->vertices + 3 * (size_t)d->geom_vertex_start[g];
      const int nv = d->geom_vertex_count[g];
      double S1[3] = {0, 0, 0}, S2[6] = {0, 0, 0, 0, 0, 0};
      std::vector<const double*> pts;
      for (int i = 0; i < nv; ++i) {
        const double* q = V + 3 * i;
        for (int k = 0; k < 3; ++k) S1[k] += q[k];
        S2[0] += q[0] * q[0];
        S2[1] += q[1] * q[1];
        S2[2] += q[2] * q[2];
        S2[3] += q[0] * q[1];
        S2[4] += q[0] * q[2];
        S2[5] += q[1] * q[2];
        pts.push_back(q);
      }
      if (nv > 0) fcl_fit_obb(S1, S2, (double)nv, pts, o);
      break;
    }
    default:
      break;
  }
}

void static_record(const mpg_world_desc* d, int s, const double* geom_rec_all, double* rec) {
  const double* T = d->static_transform + 12 * s;
  const CQ4 r = gjk_rot_from_matrix(T);  // the ccd_real rotation MPR uses
  const CQ4 ri = quat_invert2(r);
  rec[S_ROT] = r.x; rec[S_ROT + 1] = r.y; rec[S_ROT + 2] = r.z; rec[S_ROT + 3] = r.w;
  rec[S_ROTINV] = ri.x; rec[S_ROTINV + 1] = ri.y; rec[S_ROTINV + 2] = ri.z; rec[S_ROTINV + 3] = ri.w;
  rec[S_POS] = T[9]; rec[S_POS + 1] = T[10]; rec[S_POS + 2] = T[11];
  // broad-phase OBB from the same rotation MPR uses
  double R[9];
  quat_to_mat(r.w, r.x, r.y, r.z, R);
  const double* g = geom_rec_all + G_STRIDE * d->static_geom[s];
  for (int i = 0; i < 3; ++i)
    rec[S_OBBC + i] = ((R[3 * i] * g[G_OBB_C] + R[3 * i + 1] * g[G_OBB_C + 1]) + R[3 * i + 2] * g[G_OBB_C + 2]) + T[9 + i];
  for (int k = 0; k < 9; ++k) rec[S_R + k] = R[k];
}

// phase A LDS bytes per thread: records + FK save slots + survivor words + queue share
size_t cull_lds_per_thread(int n_moving, int n_saves, int W) {
  return (size_t)std::max(n_moving, 1) * 3 * sizeof(float) + (size_t)std::max(n_saves - kRegSaves, 0) * 12 * sizeof(float) +
         (size_t)W * sizeof(uint32_t) + (kQueue / 64) * sizeof(uint32_t);
}

// block size that keeps the most waves resident per CU (160 KiB of LDS),
// ties to the larger block; -1 if even one wave does not fit
int choose_block(size_t per_thread, size_t* lds) {
  int best = -1, best_waves = 0;
  for (int b : {256, 128, 64}) {
    const size_t bytes = per_thread * b;
    if (bytes > 160 * 1024) continue;
    const int waves = std::min(32, (int)(160 * 1024 / bytes) * (b / 64));
    if (waves > best_waves) {
      best_waves = waves;
      best = b;
    }
  }
  if (best > 0) *lds = per_thread * best;
  return best;
}

void free_workspace(mpg_world::Workspace& ws) {
  for (uint32_t* p : {ws.surv, ws.cnt, ws.seg_len, ws.seg_start, ws.prefix, ws.cand})
    if (p) hipFree(p);
  if (ws.rq) hipFree(ws.rq);
  if (ws.sc) hipFree(ws.sc);
  ws = mpg_world::Workspace{};
}

// drops the state kept for caller stream s (its workspace, its side stream
// and the side stream's workspace); the device is synchronised first, so no
// queued kernel still uses the buffers.  Caller holds ws_mu.
void release_stream_locked(mpg_world* w, hipStream_t s) {
  const auto wi = w->ws.find(s);
  const auto si = w->sides.find(s);
  if (wi == w->ws.end() && si == w->sides.end()) return;
  hipDeviceSynchronize();
  if (wi != w->ws.end()) {
    free_workspace(wi->second);
    w->ws.erase(wi);
  }
  if (si != w->sides.end()) {
    const auto sw = w->ws.find(si->second.side);
    if (sw != w->ws.end()) {
      free_workspace(sw->second);
      w->ws.erase(sw);
    }
    hipStreamDestroy(si->second.side);
    hipEventDestroy(si->second.fork);
    hipEventDestroy(si->second.join);
    w->sides.erase(si);
  }
}

// evicts the least recently used caller stream's state when a new stream
// would exceed kMaxStreamState (side-stream workspaces are owned by their
// caller stream's entry).  Caller holds ws_mu.
void evict_streams_locked(mpg_world* w) {
  std::map<hipStream_t, uint64_t> callers;
  for (auto& kv : w->ws) callers[kv.first] = kv.second.last;
  for (auto& kv : w->sides) {
    callers.erase(kv.second.side);
    uint64_t& t = callers[kv.first];
    t = std::max(t, kv.second.last);
  }
  for (auto& kv : w->busy)
    if (kv.second > 0) callers.erase(kv.first);  // in use by a call: not evictable
  size_t pinned = 0;
  for (auto& kv : w->busy) pinned += kv.second > 0;
  while (!callers.empty() && callers.size() + pinned >= mpg_world::kMaxStreamState) {
    auto lru = callers.begin();
    for (auto it = callers.begin(); it != callers.end(); ++it)
      if (it->second < lru->second) lru = it;
    release_stream_locked(w, lru->first);
    callers.erase(lru);
  }
}

// keeps a caller stream's state (workspace, side stream) from eviction for
// the duration of one call
struct StreamPin {
  mpg_world* w;
  hipStream_t s;
  StreamPin(mpg_world* w_, hipStream_t s_) : w(w_), s(s_) {
    std::lock_guard<std::mutex> lk(w->ws_mu);
    ++w->busy[s];
  }
  ~StreamPin() {
    std::lock_guard<std::mutex> lk(w->ws_mu);
    if (--w->busy[s] <= 0) w->busy.erase(s);
  }
};

bool is_side_stream_locked(const mpg_world* w, hipStream_t s) {
  for (auto& kv : w->sides)
    if (kv.second.side == s) return true;
  return false;
}

int get_workspace(mpg_world* w, hipStream_t s, long long want, mpg_world::Workspace** out) {
  std::lock_guard<std::mutex> lk(w->ws_mu);
  if (w->ws.find(s) == w->ws.end() && !is_side_stream_locked(w, s) && w->sides.find(s) == w->sides.end())
    evict_streams_locked(w);
  auto& ws = w->ws[s];
  ws.last = ++w->ws_tick;
  const long long np = std::max(w->dw.n_pairs, 1);
  if (ws.cap < want) {
    free_workspace(ws);
    ws.last = w->ws_tick;
    const long long tiles = (want + 63) / 64;
    HIP_TRY(hipMalloc(&ws.surv, sizeof(uint32_t) * w->dw.W * want));
    HIP_TRY(hipMalloc(&ws.cnt, sizeof(uint32_t) * np * tiles));
    HIP_TRY(hipMalloc(&ws.seg_len, sizeof(uint32_t) * np));
    HIP_TRY(hipMalloc(&ws.seg_start, sizeof(uint32_t) * np));
    HIP_TRY(hipMalloc(&ws.prefix, sizeof(uint32_t) * (np + 4)));
    HIP_TRY(hipMalloc(&ws.cand, sizeof(uint32_t) * np * want));
    HIP_TRY(hipMalloc(&ws.rq, sizeof(float) * 4 * std::max(w->dw.n_moving, 1) * want));
    HIP_TRY(hipMalloc(&ws.sc, sizeof(double) * 2 * std::max(w->dw.dof, 1) * want));
    ws.cap = want;
  }
  *out = &ws;
  return MPG_OK;
}

hipEvent_t prof_event(mpg_world* w) {
  if (!w->ev_pool.empty()) {
    hipEvent_t e = w->ev_pool.back();
    w->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// records the start of a stage on `stream` when profiling is on
struct StageTimer {
  mpg_world* w;
  hipStream_t s;
  int stage;
  hipEvent_t a = nullptr;
  StageTimer(mpg_world* w_, hipStream_t s_, int st) : w(w_), s(s_), stage(st) {
    if (!w->prof) return;
    std::lock_guard<std::mutex> lk(w->prof_mu);
    a = prof_event(w);
    if (a) hipEventRecord(a, s);
  }
  void stop() {
    if (!a) return;
    std::lock_guard<std::mutex> lk(w->prof_mu);
    hipEvent_t b = prof_event(w);
    if (!b) return;
    hipEventRecord(b, s);
    w->marks.push_back({stage, a, b});
    a = nullptr;
  }
  ~StageTimer() { stop(); }
};

struct ContactOut {
  double *depth, *normal, *pos;  // [n*P], [n*P*3], [n*P*3]
};

template <bool FROM_POSES>
int launch_collide(mpg_world* w, const double* in, long long n, uint8_t* flags, uint32_t* masks, hipStream_t stream,
                   const ContactOut* co = nullptr) {
  if (n == 0) return MPG_OK;
  StreamPin pin(w, stream);
  const long long chunk = std::min<long long>(n, w->max_chunk);
  mpg_world::Workspace* ws = nullptr;
  int rc = get_workspace(w, stream, chunk, &ws);
  if (rc) return rc;
  const size_t row = FROM_POSES ? (size_t)w->dw.n_links * 7 : (size_t)w->dw.dof;
  for (long long off = 0; off < n; off += chunk) {
    const long long m = std::min(chunk, n - off);
    const double* qin = in + off * row;
    uint8_t* fl = flags + off;
    uint32_t* mk = masks ? masks + off * w->dw.W : nullptr;
    const unsigned grid = (unsigned)((m + w->block - 1) / w->block);
    const int n_tiles = (int)((m + 63) / 64);
    StageTimer t_cull(w, stream, MPG_STAGE_CULL);
    if (w->prof) w->prof_cfg += m;
    HIP_TRY(hipMemsetAsync(ws->cnt, 0, sizeof(uint32_t) * std::max(w->dw.n_pairs, 1) * (size_t)n_tiles, stream));
    switch (w->block) {
      case 256:
        hipLaunchKernelGGL((cull_kernel<256, FROM_POSES>), dim3(grid), dim3(256), w->lds_bytes, stream, w->dw, qin,
                           m, fl, mk, ws->surv, ws->rq, ws->sc, ws->cap, ws->cnt, n_tiles);
        break;
      case 128:
        hipLaunchKernelGGL((cull_kernel<128, FROM_POSES>), dim3(grid), dim3(128), w->lds_bytes, stream, w->dw, qin,
                           m, fl, mk, ws->surv, ws->rq, ws->sc, ws->cap, ws->cnt, n_tiles);
        break;
      default:
        hipLaunchKernelGGL((cull_kernel<64, FROM_POSES>), dim3(grid), dim3(64), w->lds_bytes, stream, w->dw, qin, m,
                           fl, mk, ws->surv, ws->rq, ws->sc, ws->cap, ws->cnt, n_tiles);
        break;
    }
    HIP_TRY(hipGetLastError());
    t_cull.stop();
    StageTimer t_bucket(w, stream, MPG_STAGE_BUCKET);
    const long long tw = (long long)n_tiles * w->dw.W;  // one wave per (word, tile)
    const unsigned gb = (unsigned)((tw + 3) / 4);
    if (w->dw.n_pairs > 0) {
      hipLaunchKernelGGL(pair_scan_kernel, dim3(w->dw.n_pairs), dim3(1024), 0, stream, ws->cnt, n_tiles, ws->seg_len);
      HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(chunk_scan_kernel, dim3(1), dim3(256), 0, stream, ws->seg_len, w->dw.n_pairs, ws->seg_start,
                       ws->prefix, w->prof ? w->prof_units : nullptr, (uint32_t)(4 * w->narrow_blocks));
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(scatter_kernel, dim3(gb), dim3(256), 0, stream, ws->surv, m, ws->cap, w->dw.n_pairs, w->dw.W,
                       n_tiles, ws->cnt, ws->seg_start, ws->cand);
    HIP_TRY(hipGetLastError());
    t_bucket.stop();
    StageTimer t_narrow(w, stream, MPG_STAGE_NARROW);
    // persistent narrow phase: enough waves to fill the chip, fewer for tiny batches
    const long long want_waves = (m * std::max(w->dw.n_pairs, 1) + kTaskMin - 1) / kTaskMin;
    const unsigned nb = (unsigned)std::max<long long>(1, std::min<long long>(w->narrow_blocks, (want_waves + 3) / 4));
    hipLaunchKernelGGL((narrow_kernel<FROM_POSES>), dim3(nb), dim3(256), 0, stream, w->dw, qin, ws->seg_len,
                       ws->seg_start, ws->prefix, ws->cand, fl, mk, ws->prefix + w->dw.n_pairs + 1, ws->sc);
    HIP_TRY(hipGetLastError());
    if (w->any_closed_form) {
      hipLaunchKernelGGL((closed_form_kernel<FROM_POSES, CLS_CLOSED>), dim3(w->narrow_blocks), dim3(256), 0, stream,
                         w->dw, qin, ws->seg_len, ws->seg_start, ws->prefix, ws->cand, fl, mk, ws->sc);
      HIP_TRY(hipGetLastError());
    }
    if (w->any_octree) {
      hipLaunchKernelGGL((closed_form_kernel<FROM_POSES, CLS_OCTREE>), dim3(w->narrow_blocks), dim3(256), 0, stream,
                         w->dw, qin, ws->seg_len, ws->seg_start, ws->prefix, ws->cand, fl, mk, ws->sc);
      HIP_TRY(hipGetLastError());
    }
    if (w->any_mesh) {
      hipLaunchKernelGGL((closed_form_kernel<FROM_POSES, CLS_MESH>), dim3(w->narrow_blocks), dim3(256), 0, stream,
                         w->dw, qin, ws->seg_len, ws->seg_start, ws->prefix, ws->cand, fl, mk, ws->sc);
      HIP_TRY(hipGetLastError());
    }
    if (w->any_gjk) {
      hipLaunchKernelGGL((closed_form_kernel<FROM_POSES, CLS_GJK>), dim3(w->narrow_blocks), dim3(256), 0, stream,
                         w->dw, qin, ws->seg_len, ws->seg_start, ws->prefix, ws->cand, fl, mk, ws->sc);
      HIP_TRY(hipGetLastError());
    }
    if (co) {  // penetration info of the reported pairs (enable_contact)
      const size_t P = (size_t)w->dw.n_pairs;
      HIP_TRY(hipMemsetAsync(co->depth + off * P, 0, sizeof(double) * m * P, stream));
      HIP_TRY(hipMemsetAsync(co->normal + off * P * 3, 0, sizeof(double) * m * P * 3, stream));
      HIP_TRY(hipMemsetAsync(co->pos + off * P * 3, 0, sizeof(double) * m * P * 3, stream));
      hipLaunchKernelGGL((contact_kernel<FROM_POSES>), dim3(nb), dim3(256), 0, stream, w->dw, qin, ws->seg_len,
                         ws->seg_start, ws->prefix, ws->cand, mk, ws->sc, co->depth + off * P, co->normal + off * P * 3,
                         co->pos + off * P * 3);
      HIP_TRY(hipGetLastError());
    }
  }
  return MPG_OK;
}

int ensure_staging(mpg_world* w, size_t ncfg, size_t nout) {
  if (ncfg > w->cap_cfg) {
    hipFree(w->d_q);
    hipFree(w->d_flags);
    hipFree(w->d_masks);
    w->d_q = nullptr;
    w->d_flags = nullptr;
    w->d_masks = nullptr;
    HIP_TRY(hipMalloc(&w->d_q, sizeof(double) * std::max<size_t>(1, ncfg * std::max(w->dw.dof, 1))));
    HIP_TRY(hipMalloc(&w->d_flags, std::max<size_t>(1, ncfg)));
    HIP_TRY(hipMalloc(&w->d_masks, sizeof(uint32_t) * std::max<size_t>(1, ncfg * w->dw.W)));
    w->cap_cfg = ncfg;
  }
  if (nout > w->cap_out) {
    hipFree(w->d_out);
    w->d_out = nullptr;
    HIP_TRY(hipMalloc(&w->d_out, sizeof(double) * nout));
    w->cap_out = nout;
  }
  return MPG_OK;
}

// the host pipeline's slot buffers (not its stream and events)
void free_ring(mpg_world* w) {
  auto& R = w->ring;
  for (int j = 0; j < mpg_world::kRing; ++j) {
    if (R.d_in[j]) hipFree(R.d_in[j]);
    if (R.d_fl[j]) hipFree(R.d_fl[j]);
    if (R.d_mk[j]) hipFree(R.d_mk[j]);
    if (R.d_bcnt[j]) hipFree(R.d_bcnt[j]);
    if (R.h_fl[j]) hipHostFree(R.h_fl[j]);
    if (R.h_mk[j]) hipHostFree(R.h_mk[j]);
    if (R.h_bcnt[j]) hipHostFree(R.h_bcnt[j]);
    R.h_bcnt[j] = nullptr;
    R.h_fl_d[j] = nullptr;
    R.h_bcnt_d[j] = nullptr;
    R.d_in[j] = nullptr;
    R.d_fl[j] = nullptr;
    R.d_mk[j] = nullptr;
    R.d_bcnt[j] = nullptr;
    R.h_fl[j] = nullptr;
    R.h_mk[j] = nullptr;
    R.h_mk_d[j] = nullptr;
  }
  R.cap = 0;
  R.in_cap = 0;
}

// World-owned scratch (distance, motion validation) used by calls on any
// stream: a call's work waits for the previous call's (`last`, whatever its
// stream), and a buffer is freed to grow only after that work has finished,
// so two host threads on two streams never run over the same buffers at once
// (calls on one world are serialised on the device; their enqueueing already
// is, by the world's mutex).  Caller holds the scratch's mutex.
int scratch_begin(hipEvent_t& last, hipStream_t s) {
  if (!last) HIP_TRY(hipEventCreateWithFlags(&last, hipEventDisableTiming));
  else HIP_TRY(hipStreamWaitEvent(s, last, 0));
  return MPG_OK;
}
int scratch_grow(hipEvent_t last, void** p, size_t& cap, size_t want) {
  if (cap >= want) return MPG_OK;
  if (*p) {
    if (last) HIP_TRY(hipEventSynchronize(last));
    HIP_TRY(hipFree(*p));
  }
  *p = nullptr;
  cap = 0;
  HIP_TRY(hipMalloc(p, want));
  cap = want;
  return MPG_OK;
}

// slots of `cap` configurations with `row` input doubles each (grow-only)
int ensure_ring(mpg_world* w, size_t cap, size_t row) {
  auto& R = w->ring;
  if (!R.h2d) {
    HIP_TRY(hipStreamCreateWithFlags(&R.h2d, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&R.side, hipStreamNonBlocking));
    for (int j = 0; j < mpg_world::kRing; ++j) {
      HIP_TRY(hipEventCreateWithFlags(&R.e_in[j], hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&R.e_done[j], hipEventDisableTiming));
    }
  }
  const size_t in = cap * std::max<size_t>(row, 1);
  if (cap <= R.cap && in <= R.in_cap) return MPG_OK;
  cap = std::max(cap, R.cap);
  const size_t in_cap = std::max(in, R.in_cap);
  free_ring(w);
  const size_t W = (size_t)std::max(w->dw.W, 1);
  for (int j = 0; j < mpg_world::kRing; ++j) {
    HIP_TRY(hipMalloc(&R.d_in[j], sizeof(double) * in_cap));
    HIP_TRY(hipMalloc(&R.d_fl[j], cap));
    HIP_TRY(hipMalloc(&R.d_mk[j], sizeof(uint32_t) * W * cap));
    HIP_TRY(hipMalloc(&R.d_bcnt[j], sizeof(uint32_t) * ((cap + kPackCfg - 1) / kPackCfg)));
    HIP_TRY(hipHostMalloc((void**)&R.h_fl[j], cap, hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void**)&R.h_fl_d[j], R.h_fl[j], 0));
    HIP_TRY(hipHostMalloc((void**)&R.h_mk[j], sizeof(uint32_t) * W * cap, hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void**)&R.h_mk_d[j], R.h_mk[j], 0));
    HIP_TRY(hipHostMalloc((void**)&R.h_bcnt[j], sizeof(uint32_t) * ((cap + kPackCfg - 1) / kPackCfg),
                          hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void**)&R.h_bcnt_d[j], R.h_bcnt[j], 0));
  }
  R.cap = cap;
  R.in_cap = in_cap;
  return MPG_OK;
}

}  // namespace

extern "C" {

const char* mpg_last_error(void) { return g_last_error.c_str(); }

int mpg_fcl_bvh_build(const double* vertices, int32_t n_vertices, const int32_t* triangles, int32_t n_triangles,
                      double* boxes, int32_t* links, int32_t* leaf_order) {
  if (n_triangles <= 0 || !vertices || !triangles || !boxes || !links || !leaf_order)
    return set_error(MPG_E_INVALID, "mpg_fcl_bvh_build: empty mesh or NULL buffer");
  for (int64_t i = 0; i < 3 * (int64_t)n_triangles; ++i)
    if (triangles[i] < 0 || triangles[i] >= n_vertices) return set_error(MPG_E_INVALID, "triangle vertex out of range");
  FclBvh B;
  B.box.resize(FB_STRIDE);
  B.link.resize(3);
  std::vector<int> prim((size_t)n_triangles);
  for (int t = 0; t < n_triangles; ++t) prim[t] = t;
  fcl_bvh_node(B, vertices, triangles, prim, 0, 0, n_triangles, 0);
  std::copy(B.box.begin(), B.box.end(), boxes);
  std::copy(B.link.begin(), B.link.end(), links);
  std::copy(prim.begin(), prim.end(), leaf_order);
  return (int)(B.link.size() / 3);
}

int mpg_last_error_copy(char* buf, size_t size) {
  const size_t len = g_last_error.size();
  if (buf && size > 0) {
    const size_t k = std::min(len, size - 1);
    std::memcpy(buf, g_last_error.data(), k);
    buf[k] = '\0';
  }
  return (int)std::min<size_t>(len, 0x7fffffff);
}

const char* mpg_version(void) { return "mpgpu 0.1 (gfx950, fp64, libccd-MPR)"; }

int mpg_device_count(int* count) {
  if (!count) return set_error(MPG_E_INVALID, "count is NULL");
  HIP_TRY(hipGetDeviceCount(count));
  return MPG_OK;
}

int mpg_profile_enable(mpg_world* w, int enable) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  HIP_TRY(hipSetDevice(w->device));
  std::lock_guard<std::mutex> lk(w->prof_mu);
  if (enable && !w->prof_units) {
    HIP_TRY(hipMalloc(&w->prof_units, sizeof(unsigned long long)));
    HIP_TRY(hipMemset(w->prof_units, 0, sizeof(unsigned long long)));
  }
  w->prof = enable != 0;
  return MPG_OK;
}

int mpg_profile_read(mpg_world* w, double* ms, int64_t* launches, int64_t* units, int n_stages) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  HIP_TRY(hipSetDevice(w->device));
  std::lock_guard<std::mutex> lk(w->prof_mu);
  unsigned long long cand = 0;
  if (w->prof_units) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(&cand, w->prof_units, sizeof(cand), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(w->prof_units, 0, sizeof(cand)));
  }
  const int64_t u[MPG_NUM_STAGES] = {w->prof_cfg, w->prof_cfg, (int64_t)cand};
  w->prof_cfg = 0;
  for (auto& mk : w->marks) {
    HIP_TRY(hipEventSynchronize(mk.b));
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, mk.a, mk.b));
    w->prof_ms[mk.stage] += t;
    w->prof_n[mk.stage] += 1;
    w->ev_pool.push_back(mk.a);
    w->ev_pool.push_back(mk.b);
  }
  w->marks.clear();
  for (int k = 0; k < MPG_NUM_STAGES; ++k) {
    if (k < n_stages) {
      if (ms) ms[k] = w->prof_ms[k];
      if (launches) launches[k] = w->prof_n[k];
      if (units) units[k] = u[k];
    }
    w->prof_ms[k] = 0.0;
    w->prof_n[k] = 0;
  }
  return MPG_OK;
}

int mpg_latency_server_stats(mpg_world* w, int64_t* served, int64_t* starts, int64_t* fallbacks, int32_t* state) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  if (served) *served = w->srv_served;
  if (starts) *starts = w->srv_starts;
  if (fallbacks) *fallbacks = w->srv_fallbacks;
  if (state) *state = !(w->srv_mode && w->srv_ok) ? 0 : w->srv_broken ? 2 : 1;
  return MPG_OK;
}

int mpg_synchronize(int device) {
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipDeviceSynchronize());
  return MPG_OK;
}

int mpg_world_create(const mpg_world_desc* d, int device, mpg_world** out) {
  if (!out) return set_error(MPG_E_INVALID, "out is NULL");
  *out = nullptr;
  int rc = validate(d);
  if (rc) return rc;
  std::vector<double> geom_rec((size_t)G_STRIDE * std::max(d->n_geoms, 1), 0.0);
  for (int g = 0; g < d->n_geoms; ++g) geom_record(d, g, geom_rec.data() + (size_t)G_STRIDE * g);
  std::vector<double> obb((size_t)7 * std::max(d->n_geoms, 1), 0.0);
  for (int g = 0; g < d->n_geoms; ++g) {
    const double* r = geom_rec.data() + (size_t)G_STRIDE * g;
    for (int k = 0; k < 3; ++k) obb[7 * g + k] = r[G_OBB_C + k];
    for (int k = 0; k < 3; ++k) obb[7 * g + 3 + k] = r[G_OBB_E + k];
    obb[7 * g + 6] = r[G_RADIUS];
  }
  BpProgram bpp;
  bp_build(d, obb, bpp);
  size_t lds = 0;
  const int W = std::max(1, (d->n_pairs + 31) / 32);
  const int block = choose_block(cull_lds_per_thread(d->n_moving, bpp.n_saves, W), &lds);
  if (block < 0) return set_error(MPG_E_UNSUPPORTED, "world too large for the phase-A LDS budget");
  HIP_TRY(hipSetDevice(device));

  std::vector<double> static_rec((size_t)S_STRIDE * std::max(d->n_static, 1), 0.0);
  for (int s = 0; s < d->n_static; ++s) static_record(d, s, geom_rec.data(), static_rec.data() + (size_t)S_STRIDE * s);
  // hulls in AoSoA-4 groups, padded with copies of the hull's first vertex
  std::vector<int> gstart(std::max(d->n_geoms, 1), 0), ngroups(std::max(d->n_geoms, 1), 0);
  std::vector<double> hull;
  std::vector<int> cbase(std::max(d->n_geoms, 1), -1), geom_nbr(std::max(d->n_geoms, 1), -1), hull_nbr, wcell_end, wcell_end2, wcell_pre;
  std::vector<double> cell_rec, cell_ovf, wcell_rec, wcell_ovf, wcell_aux, nbr_ent;
  const int walk_subk =
      std::getenv("MPG_WALK_SUBK") ? std::max(1, std::min(8, std::atoi(std::getenv("MPG_WALK_SUBK")))) : kSubK;
  int big_words = 0;  // walk hulls above kMaxWalkVerts: the widest visited set
  for (int g = 0; g < d->n_geoms; ++g) {
    if (d->geom_type[g] != MPG_GEOM_CONVEX) continue;
    const double* Vg = d->vertices + 3 * (size_t)d->geom_vertex_start[g];
    const int nvg = d->geom_vertex_count[g];
    // FCL 0.7.0 Convex: neighbour walk for > 32 vertices with valid faces
    std::vector<int> enc;
    const int nf = (int)d->geom_param[4 * g + 1];
    bool walk = nf > 0 && fcl_convex_neighbors(nvg, d->convex_face + (int64_t)d->geom_param[4 * g], nf, enc);
#ifdef MPG_DIAG  // ablation builds only (changes results)
    if (std::getenv("MPG_DEBUG_NO_WALK")) walk = false;
#endif
    if (walk) {
      geom_nbr[g] = (int)(hull_nbr.size() / 2);
      if (nvg > kMaxWalkVerts) big_words = std::max(big_words, (nvg + 63) / 64);  // pooled visited set
      for (int i = 0; i < nvg; ++i) {
        const int st = enc[i], cnt = enc[st];
        hull_nbr.push_back((int)(nbr_ent.size() / 4));
        hull_nbr.push_back(cnt);
        for (int k = 1; k <= cnt; ++k) {
          const int vi = enc[st + k];
          nbr_ent.insert(nbr_ent.end(), {Vg[3 * vi], Vg[3 * vi + 1], Vg[3 * vi + 2], (double)vi});
        }
      }
      const size_t r0 = wcell_rec.size();
      if (build_walk_cells(Vg, nvg, enc.data(), walk_subk, wcell_rec, wcell_ovf, wcell_aux, wcell_end, wcell_end2, wcell_pre))
        cbase[g] = (int)(r0 / kCellRec);
    } else {
      std::vector<uint32_t> cstart;
      std::vector<double> cpts;
      if (build_hull_cells(Vg, nvg, cstart, cpts)) {
        cbase[g] = (int)(cell_rec.size() / kCellRec);
        pack_cell_records(cstart.data(), cpts.data(), cell_rec, cell_ovf);
      }
    }
    const double* V = d->vertices + 3 * (size_t)d->geom_vertex_start[g];
    const int nv = d->geom_vertex_count[g], ng = (nv + 3) / 4;
    gstart[g] = (int)(hull.size() / 12);
    ngroups[g] = ng;
    for (int q = 0; q < ng; ++q)
      for (int k = 0; k < 3; ++k)
        for (int l = 0; l < 4; ++l) {
          const int i = 4 * q + l < nv ? 4 * q + l : 0;
          hull.push_back(V[3 * i + k]);
        }
  }
  for (int g = 0; g < d->n_geoms; ++g) {  // TriangleP: its three vertices as one group (supportTriangle reads them)
    if (d->geom_type[g] != MPG_GEOM_TRIANGLE) continue;
    const double* V = d->vertices + 3 * (size_t)d->geom_vertex_start[g];
    gstart[g] = (int)(hull.size() / 12);
    ngroups[g] = 1;
    for (int k = 0; k < 3; ++k)
      for (int l = 0; l < 4; ++l) hull.push_back(V[3 * (l < 3 ? l : 0) + k]);
  }
  if (hull.empty()) hull.assign(12, 0.0);
  if (cell_rec.empty()) cell_rec.assign(kCellRec, 0.0);
  if (cell_ovf.empty()) cell_ovf.assign(4, 0.0);
  if (hull_nbr.empty()) hull_nbr.assign(2, 0);
  if (nbr_ent.empty()) nbr_ent.assign(4, 0.0);
  if (wcell_rec.empty()) wcell_rec.assign(kCellRec, 0.0);
  if (wcell_ovf.empty()) wcell_ovf.assign(4, 0.0);
  if (wcell_aux.empty()) wcell_aux.assign(kWalkAux, 0.0);
  if (wcell_end.empty()) wcell_end.assign(1, -1);
  if (wcell_end2.empty()) wcell_end2.assign(1, -1);
  if (wcell_pre.empty()) wcell_pre.assign(kWalkPre, 0);
  // octrees: leaf boxes + a uniform grid per octree geometry (cells of at
  // least the largest leaf, <= 64 per axis); a leaf is listed in every cell
  // its box overlaps
  // BVH meshes: per triangle its vertices (mesh frame) and AABB (TR_*), in
  // cluster order
  std::vector<double> mesh_tri((size_t)TR_STRIDE * std::max<int64_t>(d->n_mesh_triangles, 1), 0.0);
  std::vector<double> mesh_node;
  std::vector<int> mesh_link, mesh_tree(2 * (size_t)std::max(d->n_geoms, 1), 0);
  for (int g = 0; g < d->n_geoms; ++g) {
    if (d->geom_type[g] != MPG_GEOM_MESH) continue;
    const double* V = d->vertices + 3 * (size_t)d->geom_vertex_start[g];
    const int64_t t0 = (int64_t)d->geom_param[4 * g], tn = (int64_t)d->geom_param[4 * g + 1];
    std::vector<double> rec((size_t)TR_STRIDE * std::max<int64_t>(tn, 1), 0.0);
    for (int64_t t = 0; t < tn; ++t) {
      double* r = rec.data() + (size_t)TR_STRIDE * t;
      for (int v = 0; v < 3; ++v)
        for (int k = 0; k < 3; ++k) r[TR_P + 3 * v + k] = V[3 * (size_t)d->mesh_triangle[3 * (t0 + t) + v] + k];
      for (int k = 0; k < 3; ++k) {
        r[TR_LO + k] = std::min(r[TR_P + k], std::min(r[TR_P + 3 + k], r[TR_P + 6 + k]));
        r[TR_HI + k] = std::max(r[TR_P + k], std::max(r[TR_P + 3 + k], r[TR_P + 6 + k]));
      }
      r[TR_ID] = (double)t;  // the triangle's index in the mesh (its leaf position: tri_pos)
    }
    std::vector<int> order((size_t)tn);
    for (int64_t t = 0; t < tn; ++t) order[t] = (int)t;
    // clusters of <= max(8, T / 64) triangles: ~64 cluster boxes per mesh
    mesh_tree[2 * g] = (int)(mesh_link.size() / 2);
    mesh_build_clusters(rec, order, 0, (int)tn, std::max<int>(8, (int)((tn + 63) / 64)), (int)t0, mesh_node, mesh_link);
    mesh_tree[2 * g + 1] = (int)(mesh_link.size() / 2) - mesh_tree[2 * g];
    for (int64_t k = 0; k < tn; ++k)
      std::copy(rec.begin() + (size_t)TR_STRIDE * order[k], rec.begin() + (size_t)TR_STRIDE * (order[k] + 1),
                mesh_tri.begin() + (size_t)TR_STRIDE * (t0 + k));
  }
  if (mesh_node.empty()) mesh_node.assign(6, 0.0);
  if (mesh_link.empty()) mesh_link.assign(2, 0);
  // FCL's BVHModel<OBBRSS> trees (the traversal gates of mesh pairs) and the
  // shapes' computeBV OBBs
  FclBvh fbvh;
  std::vector<int> fb_root(std::max(d->n_geoms, 1), -1), tri_pos(std::max<int64_t>(d->n_mesh_triangles, 1), 0);
  std::vector<double> sobb((size_t)FB_STRIDE * std::max(d->n_geoms, 1), 0.0);
  for (int g = 0; g < d->n_geoms; ++g) {
    fcl_shape_obb(d, g, sobb.data() + (size_t)FB_STRIDE * g);
    if (d->geom_type[g] != MPG_GEOM_MESH) continue;
    const int64_t t0 = (int64_t)d->geom_param[4 * g], tn = (int64_t)d->geom_param[4 * g + 1];
    if (tn <= 0) continue;
    const int base = (int)(fbvh.link.size() / 3);
    fb_root[g] = base;
    fbvh.box.resize(fbvh.box.size() + FB_STRIDE);
    fbvh.link.resize(fbvh.link.size() + 3);
    std::vector<int> prim((size_t)tn);
    for (int64_t t = 0; t < tn; ++t) prim[t] = (int)t;
    fbvh.max_depth = 0;
    fcl_bvh_node(fbvh, d->vertices + 3 * (size_t)d->geom_vertex_start[g], d->mesh_triangle + 3 * t0, prim, 0, 0,
                 (int)tn, base);
    if (fbvh.max_depth > kFclMaxDepth)
      return set_error(MPG_E_UNSUPPORTED, "BVH mesh geometry " + std::to_string(g) + ": FCL's mean-split tree is " +
                                              std::to_string(fbvh.max_depth) + " levels deep (the device gates descend at most " +
                                              std::to_string(kFclMaxDepth) + ")");
    for (int64_t k = 0; k < tn; ++k) tri_pos[t0 + prim[k]] = (int)k;
  }
  if (fbvh.box.empty()) {
    fbvh.box.assign(FB_STRIDE, 0.0);
    fbvh.link.assign(3, 0);
  }
  std::vector<double> oct_leaf(6 * (size_t)std::max<int64_t>(d->n_octree_leaves, 1), 0.0);
  if (d->n_octree_leaves > 0) std::copy(d->octree_leaf, d->octree_leaf + 6 * d->n_octree_leaves, oct_leaf.begin());
  // each leaf's path down FCL's octree: getRootBV (delta = 2^16 resolution /
  // 2) halved by computeChildBV until the leaf box (the leaves were cut that
  // way: host octree.cpp collect, octomap's 16 levels)
  std::vector<uint64_t> oct_path(std::max<int64_t>(d->n_octree_leaves, 1), 0);
  std::vector<int> oct_depth(std::max<int64_t>(d->n_octree_leaves, 1), 0);
  for (int g = 0; g < d->n_geoms; ++g) {
    if (d->geom_type[g] != MPG_GEOM_OCTREE) continue;
    const int64_t l0 = (int64_t)d->geom_param[4 * g], ln = (int64_t)d->geom_param[4 * g + 1];
    const double delta = (double)(1 << 16) * d->geom_param[4 * g + 2] / 2;
    for (int64_t l = l0; l < l0 + ln; ++l) {
      const double* L = d->octree_leaf + 6 * l;
      double lo[3] = {-delta, -delta, -delta}, hi[3] = {delta, delta, delta};
      uint64_t code = 0;
      int depth = 0;
      while (!(lo[0] == L[0] && lo[1] == L[1] && lo[2] == L[2] && hi[0] == L[3] && hi[1] == L[4] && hi[2] == L[5])) {
        if (++depth > 16)
          return set_error(MPG_E_INVALID, "octree geometry " + std::to_string(g) + ": leaf " + std::to_string(l - l0) +
                                              " is not a box of FCL's root-BV halving (getRootBV / computeChildBV)");
        int ci = 0;
        for (int k = 0; k < 3; ++k) {
          const double mid = (lo[k] + hi[k]) * 0.5;
          if (L[k] >= mid) {
            ci |= 1 << k;
            lo[k] = mid;
          } else {
            hi[k] = mid;
          }
        }
        code = (code << 3) | (uint64_t)ci;
      }
      oct_path[l] = code;
      oct_depth[l] = depth;
    }
  }
  std::vector<double> oct_grid((size_t)OG_STRIDE * std::max(d->n_geoms, 1), 0.0);
  std::vector<int> oct_cells, oct_list;
  for (int g = 0; g < d->n_geoms; ++g) {
    if (d->geom_type[g] != MPG_GEOM_OCTREE) continue;
    const int64_t l0 = (int64_t)d->geom_param[4 * g], ln = (int64_t)d->geom_param[4 * g + 1];
    double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0}, big = 0.0;
    for (int64_t i = l0; i < l0 + ln; ++i)
      for (int k = 0; k < 3; ++k) {
        const double a = d->octree_leaf[6 * i + k], b = d->octree_leaf[6 * i + 3 + k];
        lo[k] = i == l0 ? a : std::min(lo[k], a);
        hi[k] = i == l0 ? b : std::max(hi[k], b);
        big = std::max(big, b - a);
      }
    double ext = 0.0;
    for (int k = 0; k < 3; ++k) ext = std::max(ext, hi[k] - lo[k]);
    const double cell = std::max({big, ext / 64.0, 1e-9});
    int dims[3];
    for (int k = 0; k < 3; ++k) dims[k] = std::max(1, std::min(66, (int)std::ceil((hi[k] - lo[k]) / cell) + 1));
    double* og = oct_grid.data() + (size_t)OG_STRIDE * g;
    for (int k = 0; k < 3; ++k) og[OG_ORIGIN + k] = lo[k];
    og[OG_INV] = 1.0 / cell;
    for (int k = 0; k < 3; ++k) og[OG_DIMS + k] = dims[k];
    og[OG_CELL0] = (double)oct_cells.size();
    const size_t nc = (size_t)dims[0] * dims[1] * dims[2];
    std::vector<std::vector<int>> lists(nc);
    // the same cell arithmetic as the device query, so a leaf is found from
    // every cell a query box overlapping it can touch
    auto cidx = [&](double v, int k) {
      const double f = std::floor((v - lo[k]) * og[OG_INV]);
      return f < 0.0 ? 0 : (f >= dims[k] ? dims[k] - 1 : (int)f);
    };
    for (int64_t i = l0; i < l0 + ln; ++i) {
      const double* L = d->octree_leaf + 6 * i;
      for (int x = cidx(L[0], 0); x <= cidx(L[3], 0); ++x)
        for (int y = cidx(L[1], 1); y <= cidx(L[4], 1); ++y)
          for (int z = cidx(L[2], 2); z <= cidx(L[5], 2); ++z)
            lists[((size_t)x * dims[1] + y) * dims[2] + z].push_back((int)i);
    }
    for (size_t c = 0; c < nc; ++c) {
      oct_cells.push_back((int)oct_list.size());
      oct_list.insert(oct_list.end(), lists[c].begin(), lists[c].end());
    }
  }
  oct_cells.push_back((int)oct_list.size());
  if (oct_list.empty()) oct_list.push_back(0);
  // per link: joints from the root to link_parent (chain FK in phase B)
  std::vector<int> chain_start, chain_len, chain_joints;
  for (int l = 0; l < d->n_links; ++l) {
    std::vector<int> c;
    for (int j = d->link_parent[l]; j > 0; j = d->joint_parent[j - 1]) c.push_back(j);
    std::reverse(c.begin(), c.end());
    chain_start.push_back((int)chain_joints.size());
    chain_len.push_back((int)c.size());
    chain_joints.insert(chain_joints.end(), c.begin(), c.end());
  }
  std::vector<int> allowed(std::max(d->n_pairs, 1), 0);
  for (int p = 0; p < d->n_pairs; ++p) allowed[p] = d->pair_allowed ? (d->pair_allowed[p] != 0) : 0;
  std::vector<int> pair_cf(std::max(d->n_pairs, 1), 0);
  for (int p = 0; p < d->n_pairs; ++p) {
    pair_cf[p] = closed_form_kind(d, d->pair_a[p], d->pair_b[p]);
    // GST_INDEP: the shape pairs without a closed form run FCL's own GJK
    // (GJKSolver_indep keeps the same closed forms as GJKSolver_libccd)
    if (d->gjk_solver == MPG_GJK_INDEP && pair_cf[p] == CF_NONE) pair_cf[p] = CF_GJK;
  }
  // latency pair records (LR_*): one round of loads per wave instead of a
  // chain of dependent snapshot lookups (pair -> object -> link -> chain ->
  // joints -> geometry)
  std::vector<double> lat_rec((size_t)LR_STRIDE * std::max(d->n_pairs, 1), 0.0);
  bool lat_rec_ok = true;
  for (int p = 0; p < d->n_pairs; ++p) {
    double* R = lat_rec.data() + (size_t)LR_STRIDE * p;
    const int ids[2] = {d->pair_a[p], d->pair_b[p]};
    R[LR_ALLOWED] = allowed[p];
    R[LR_CF] = pair_cf[p];
    for (int s2 = 0; s2 < 2; ++s2) {
      const int id = ids[s2];
      const bool mv = id < d->n_moving;
      const int g = mv ? d->moving_geom[id] : d->static_geom[id - d->n_moving];
      R[s2 ? LR_GB : LR_GA] = g;
      R[s2 ? LR_BM : LR_AM] = mv ? 1.0 : 0.0;
      R[s2 ? LR_RB : LR_RA] = geom_rec[G_STRIDE * (size_t)g + G_RADIUS];
      double* S = R + LR_SIDE + LS_STRIDE * s2;
      for (int k = 0; k < 3; ++k) S[LS_OBBC + k] = geom_rec[G_STRIDE * (size_t)g + G_OBB_C + k];
      if (!mv) {
        std::copy(d->static_transform + 12 * (size_t)(id - d->n_moving),
                  d->static_transform + 12 * (size_t)(id - d->n_moving) + 12, S + LS_OFF);
        continue;
      }
      const int l = d->moving_link[id];
      const int cl = chain_len[l];
      if (cl > kLatChain) {
        lat_rec_ok = false;
        continue;
      }
      S[LS_CL] = cl;
      std::copy(d->link_placement + 12 * (size_t)l, d->link_placement + 12 * (size_t)l + 12, S + LS_LINKPL);
      std::copy(d->moving_offset + 12 * (size_t)id, d->moving_offset + 12 * (size_t)id + 12, S + LS_OFF);
      for (int k = 0; k < cl; ++k) {
        const int j = chain_joints[chain_start[l] + k] - 1;
        double* J = S + LS_J + LJ_STRIDE * k;
        J[0] = d->joint_type[j];
        J[1] = d->joint_q_source[j];
        J[2] = d->joint_q_const[j];
        for (int i = 0; i < 3; ++i) J[3 + i] = d->joint_axis[3 * (size_t)j + i];
        for (int i = 0; i < 12; ++i) J[6 + i] = d->joint_placement[12 * (size_t)j + i];
      }
    }
  }
  // phase-A schedule: non-allowed pairs grouped by their lower moving object
  // ---- culling margins: pairs that can reach libccd MPR (directly, on octree
  // leaves or on mesh triangles) keep everything within its false-hit reach
  bool may_mpr = false;
  for (int p = 0; p < d->n_pairs; ++p) {
    if (allowed[p]) continue;
    const int ta = obj_geom_type(d, d->pair_a[p]), tb = obj_geom_type(d, d->pair_b[p]);
    const bool closed = pair_cf[p] != CF_NONE && cf_class(pair_cf[p]) == CLS_CLOSED;
    const bool mesh_mesh = ta == MPG_GEOM_MESH && tb == MPG_GEOM_MESH;
    may_mpr |= !closed && !mesh_mesh;
  }
  const double reach = kCcdFalseHitReach * (1.0 + 1e-3) + 1e-5;
  float bp_margin = may_mpr ? (float)std::max((double)kBpMargin, reach) : kBpMargin;
  // The travel of each prismatic joint: a move-group joint's value bound from
  // its limits (kDefaultTravel when unbounded), a fixed joint's own value.
  // A configuration whose prismatic value exceeds its bound is evaluated with
  // every pair (the cull's coordinate bound below would not hold for it).
  auto sq3 = [](const double* v) { return v[0] * v[0] + v[1] * v[1] + v[2] * v[2]; };
  // prism_bound < 0: not a move-group prismatic joint (a [0, 0] limit is a real bound of 0)
  std::vector<double> travel(std::max(d->n_joints, 1), 0.0), prism_bound(std::max(d->n_joints, 1), -1.0);
  int n_prism = 0;
  for (int j = 0; j < d->n_joints; ++j) {
    const int t = d->joint_type[j];
    if (t < MPG_JOINT_PX || t > MPG_JOINT_PRISMATIC_UNALIGNED) continue;
    const double an = t == MPG_JOINT_PRISMATIC_UNALIGNED ? std::sqrt(sq3(d->joint_axis + 3 * j)) : 1.0;
    if (d->joint_q_source[j] >= 0) {
      double qb = kDefaultTravel;
      if (d->joint_lower && d->joint_upper && std::isfinite(d->joint_lower[j]) && std::isfinite(d->joint_upper[j]))
        qb = std::max(std::fabs(d->joint_lower[j]), std::fabs(d->joint_upper[j]));
      prism_bound[j] = qb;
      ++n_prism;
      travel[j] = qb * an;
    } else {
      travel[j] = std::fabs(d->joint_q_const[j]) * an;
    }
  }
  // the fp32 broad phase's rounding grows with coordinate magnitude: bound
  // every world coordinate the cull computes (the chain's reach -- sum of the
  // placement translations and prismatic travels, revolute joints cannot
  // lengthen it --, moving offsets, static poses, geometry radii) and keep the
  // margin above kFp32CullRel of it (kBpMargin covers a ~2 m world near the
  // origin)
  double reach_x = 0.0, geo_r = 0.0, stat_x = 0.0;
  for (int j = 0; j < d->n_joints; ++j) reach_x += std::sqrt(sq3(d->joint_placement + 12 * j + 9)) + travel[j];
  for (int l = 0; l < d->n_links; ++l) reach_x += std::sqrt(sq3(d->link_placement + 12 * l + 9));
  double off = 0.0;
  for (int m = 0; m < d->n_moving; ++m) off = std::max(off, std::sqrt(sq3(d->moving_offset + 12 * m + 9)));
  for (int g = 0; g < d->n_geoms; ++g) geo_r = std::max(geo_r, geom_rec[G_STRIDE * g + G_RADIUS] +
                                                                   std::sqrt(sq3(&geom_rec[G_STRIDE * g + G_OBB_C])));
  for (int s2 = 0; s2 < d->n_static; ++s2) stat_x = std::max(stat_x, std::sqrt(sq3(d->static_transform + 12 * s2 + 9)));
  const double X = std::max(reach_x + off, stat_x) + geo_r;
  bp_margin = std::max(bp_margin, (float)(kFp32CullRel * X));
  const double small_margin = may_mpr ? std::max(kSmallMargin, reach) : kSmallMargin;
  // link poses given directly (mpg_collide_link_poses): a pose beyond the
  // chain's reach falls outside the coordinate bound -> every pair
  const double pose_bound = reach_x;
  // Reach ball of each moving object: its centre stays within radius R of
  // the origin of the first joint of its chain (every later joint origin is
  // a fixed distance from its parent's, plus a prismatic travel; revolute
  // angles cannot lengthen the chain), or is fixed when the chain is empty.
  // A static partner farther than R + the object's radius + the culling
  // margin from that ball can never be a candidate: its schedule entry is
  // kept only for the link-pose input, whose poses are not kinematic.
  std::vector<std::array<double, 4>> ball(std::max(d->n_moving, 1));  // centre, radius (object radius included)
  for (int m = 0; m < d->n_moving; ++m) {
    const int l = d->moving_link[m];
    const double* g = geom_rec.data() + G_STRIDE * d->moving_geom[m];
    const double* mo = d->moving_offset + 12 * m;
    const double* lp = d->link_placement + 12 * l;
    double a[3], bpt[3];
    for (int i = 0; i < 3; ++i)
      a[i] = mo[3 * i] * g[G_OBB_C] + mo[3 * i + 1] * g[G_OBB_C + 1] + mo[3 * i + 2] * g[G_OBB_C + 2] + mo[9 + i];
    for (int i = 0; i < 3; ++i) bpt[i] = lp[3 * i] * a[0] + lp[3 * i + 1] * a[1] + lp[3 * i + 2] * a[2] + lp[9 + i];
    const int cs = chain_start[l], cn = chain_len[l];
    double R = g[G_RADIUS];
    if (cn == 0) {
      ball[m] = {bpt[0], bpt[1], bpt[2], R};
      continue;
    }
    const int j1 = chain_joints[cs] - 1;
    const double* p1 = d->joint_placement + 12 * j1 + 9;
    R += travel[j1] + std::sqrt(sq3(bpt));
    for (int k = 1; k < cn; ++k) {
      const int j = chain_joints[cs + k] - 1;
      R += std::sqrt(sq3(d->joint_placement + 12 * j + 9)) + travel[j];
    }
    ball[m] = {p1[0], p1[1], p1[2], R * (1.0 + 1e-9) + 1e-9};
  }
  auto never_near = [&](int m, int sid) {  // exact fp64 distance, reach ball vs the static OBB
    const double* sr = static_rec.data() + (size_t)S_STRIDE * sid;
    const double* gs = geom_rec.data() + G_STRIDE * d->static_geom[sid];
    double e2 = 0.0;
    for (int k = 0; k < 3; ++k) {  // box axis k = column k of S_R
      double t = 0.0;
      for (int i = 0; i < 3; ++i) t += (ball[m][i] - sr[S_OBBC + i]) * sr[S_R + 3 * i + k];
      const double ex = std::max(std::fabs(t) - gs[G_OBB_E + k], 0.0);
      e2 += ex * ex;
    }
    const double slack = 1e-6 * (1.0 + X);
    return std::sqrt(e2) - ball[m][3] > (double)bp_margin + slack;
  };
  // bits of every non-allowed pair (a configuration evaluated with all pairs)
  std::vector<int> all_mask(std::max(W, 1), 0);
  for (int p = 0; p < d->n_pairs; ++p)
    if (!allowed[p]) all_mask[p >> 5] |= (int)(1u << (p & 31));
  // moving-moving pairs by their lower moving object, then the moving-static
  // pairs static-major (one static record serves all its entries), those the
  // object's reach ball can bring near (group 0) before the rest (group 1)
  const int ns = d->n_static;
  std::vector<int> sched_start(d->n_moving + 1, 0), sched_pair, sched_other, st_start(2 * (ns + 1), 0), st_m;
  std::vector<float> st_r;
  for (int m = 0; m < d->n_moving; ++m) {
    sched_start[m] = (int)sched_pair.size();
    for (int p = 0; p < d->n_pairs; ++p) {
      if (allowed[p]) continue;
      const int a = d->pair_a[p], b = d->pair_b[p];
      const int lo = std::min(a, b), hi = std::max(a, b);  // static ids are >= n_moving
      if (lo != m || hi >= d->n_moving) continue;
      sched_pair.push_back(p);
      sched_other.push_back(hi);
      st_m.push_back(0);
      st_r.push_back(0.f);
    }
  }
  sched_start[d->n_moving] = (int)sched_pair.size();
  for (int g = 0; g < 2; ++g) {
    for (int sid = 0; sid < ns; ++sid) {
      st_start[g * (ns + 1) + sid] = (int)sched_pair.size();
      for (int m = 0; m < d->n_moving; ++m)
        for (int p = 0; p < d->n_pairs; ++p) {
          if (allowed[p]) continue;
          const int a = d->pair_a[p], b = d->pair_b[p];
          if (std::min(a, b) != m || std::max(a, b) != d->n_moving + sid) continue;
          if (never_near(m, sid) != (g == 1)) continue;
          sched_pair.push_back(p);
          sched_other.push_back(d->n_moving + sid);
          st_m.push_back(m);
          st_r.push_back(bpp.mobj[BM_STRIDE * m + BM_R]);
        }
    }
    st_start[g * (ns + 1) + ns] = (int)sched_pair.size();
  }
  if (sched_pair.empty()) {
    sched_pair.push_back(0);
    sched_other.push_back(0);
    st_m.push_back(0);
    st_r.push_back(0.f);
  }

  BlobBuilder bb;
  const size_t o_jt = bb.add(d->joint_type, d->n_joints);
  const size_t o_jp = bb.add(d->joint_parent, d->n_joints);
  const size_t o_jqs = bb.add(d->joint_q_source, d->n_joints);
  const size_t o_jqc = bb.add(d->joint_q_const, d->n_joints);
  const size_t o_ja = bb.add(d->joint_axis, 3 * (size_t)d->n_joints);
  const size_t o_jpl = bb.add(d->joint_placement, 12 * (size_t)d->n_joints);
  const size_t o_lp = bb.add(d->link_parent, d->n_links);
  const size_t o_lpl = bb.add(d->link_placement, 12 * (size_t)d->n_links);
  const size_t o_gt = bb.add(d->geom_type, d->n_geoms);
  const size_t o_gvs = bb.add(gstart.data(), gstart.size());
  const size_t o_gnv = bb.add(ngroups.data(), ngroups.size());
  std::vector<int> nvert(std::max(d->n_geoms, 1), 0);
  for (int g = 0; g < d->n_geoms; ++g) nvert[g] = d->geom_type[g] == MPG_GEOM_CONVEX ? d->geom_vertex_count[g] : 0;
  const size_t o_gnvt = bb.add(nvert.data(), nvert.size());
  const size_t o_grec = bb.add(geom_rec.data(), geom_rec.size());
  const size_t o_v = bb.add(hull.data(), hull.size());
  const size_t o_cb = bb.add(cbase.data(), cbase.size());
  const size_t o_crec = bb.add(cell_rec.data(), cell_rec.size());
  const size_t o_covf = bb.add(cell_ovf.data(), cell_ovf.size());
  const size_t o_gnb = bb.add(geom_nbr.data(), geom_nbr.size());
  const size_t o_hnb = bb.add(hull_nbr.data(), hull_nbr.size());
  const size_t o_nent = bb.add(nbr_ent.data(), nbr_ent.size());
  const size_t o_wrec = bb.add(wcell_rec.data(), wcell_rec.size());
  const size_t o_wovf = bb.add(wcell_ovf.data(), wcell_ovf.size());
  const size_t o_waux = bb.add(wcell_aux.data(), wcell_aux.size());
  const size_t o_wend = bb.add(wcell_end.data(), wcell_end.size());
  const size_t o_wend2 = bb.add(wcell_end2.data(), wcell_end2.size());
  const size_t o_wpre = bb.add(wcell_pre.data(), wcell_pre.size());
  const size_t o_ml = bb.add(d->moving_link, d->n_moving);
  const size_t o_mg = bb.add(d->moving_geom, d->n_moving);
  const size_t o_mo = bb.add(d->moving_offset, 12 * (size_t)d->n_moving);
  const size_t o_sg = bb.add(d->static_geom, d->n_static);
  const size_t o_srec = bb.add(static_rec.data(), static_rec.size());
  const size_t o_pa = bb.add(d->pair_a, d->n_pairs);
  const size_t o_pb = bb.add(d->pair_b, d->n_pairs);
  const size_t o_al = bb.add(allowed.data(), allowed.size());
  const size_t o_cf = bb.add(pair_cf.data(), pair_cf.size());
  const size_t o_sT = bb.add(d->static_transform, 12 * (size_t)d->n_static);
  const size_t o_cs = bb.add(chain_start.data(), chain_start.size());
  const size_t o_cl = bb.add(chain_len.data(), chain_len.size());
  const size_t o_cj = bb.add(chain_joints.data(), chain_joints.size());
  const size_t o_ss = bb.add(sched_start.data(), sched_start.size());
  const size_t o_sp = bb.add(sched_pair.data(), sched_pair.size());
  const size_t o_so = bb.add(sched_other.data(), sched_other.size());
  const size_t o_sts = bb.add(st_start.data(), st_start.size());
  const size_t o_stm = bb.add(st_m.data(), st_m.size());
  const size_t o_str = bb.add(st_r.data(), st_r.size());
  const size_t o_pbd = bb.add(prism_bound.data(), prism_bound.size());
  const size_t o_amk = bb.add(all_mask.data(), all_mask.size());
  const size_t o_bjs = bb.add(bpp.jsrc.data(), bpp.jsrc.size());
  const size_t o_bjv = bb.add(bpp.jsave.data(), bpp.jsave.size());
  const size_t o_bja = bb.add(bpp.jaxis.data(), bpp.jaxis.size());
  const size_t o_bjp = bb.add(bpp.jplace.data(), bpp.jplace.size());
  const size_t o_bls = bb.add(bpp.link_start.data(), bpp.link_start.size());
  const size_t o_blo = bb.add(bpp.link_order.data(), bpp.link_order.size());
  const size_t o_blp = bb.add(bpp.lplace.data(), bpp.lplace.size());
  const size_t o_bos = bb.add(bpp.obj_start.data(), bpp.obj_start.size());
  const size_t o_boo = bb.add(bpp.obj_order.data(), bpp.obj_order.size());
  const size_t o_bmo = bb.add(bpp.moff.data(), bpp.moff.size());
  const size_t o_bmb = bb.add(bpp.mobj.data(), bpp.mobj.size());
  const size_t o_bsb = bb.add(bpp.sobj.data(), bpp.sobj.size());
  if (bpp.jobj_order.empty()) bpp.jobj_order.push_back(0);
  const size_t o_bjk = bb.add(bpp.jkind.data(), bpp.jkind.size());
  const size_t o_bjo = bb.add(bpp.jobj_start.data(), bpp.jobj_start.size());
  const size_t o_bjr = bb.add(bpp.jobj_order.data(), bpp.jobj_order.size());
  const size_t o_bop = bb.add(bpp.oplace.data(), bpp.oplace.size());
  const size_t o_boq = bb.add(bpp.oquat.data(), bpp.oquat.size());
  const size_t o_boc = bb.add(bpp.ocen.data(), bpp.ocen.size());
  const size_t o_olf = bb.add(oct_leaf.data(), oct_leaf.size());
  const size_t o_mtr = bb.add(mesh_tri.data(), mesh_tri.size());
  const size_t o_mnd = bb.add(mesh_node.data(), mesh_node.size());
  const size_t o_mln = bb.add(mesh_link.data(), mesh_link.size());
  const size_t o_mtt = bb.add(mesh_tree.data(), mesh_tree.size());
  const size_t o_lrec = bb.add(lat_rec.data(), lat_rec.size());
  const size_t o_fbb = bb.add(fbvh.box.data(), fbvh.box.size());
  const size_t o_fbl = bb.add(fbvh.link.data(), fbvh.link.size());
  const size_t o_fbr = bb.add(fb_root.data(), fb_root.size());
  const size_t o_tps = bb.add(tri_pos.data(), tri_pos.size());
  const size_t o_sob = bb.add(sobb.data(), sobb.size());
  const size_t o_ogr = bb.add(oct_grid.data(), oct_grid.size());
  const size_t o_oce = bb.add(oct_cells.data(), oct_cells.size());
  const size_t o_oli = bb.add(oct_list.data(), oct_list.size());
  const size_t o_opa = bb.add(oct_path.data(), oct_path.size());
  const size_t o_ode = bb.add(oct_depth.data(), oct_depth.size());

  mpg_world* w = new mpg_world();
  w->device = device;
  w->n_geoms = d->n_geoms;
  w->geom_type_h.assign(d->geom_type, d->geom_type + d->n_geoms);
  w->block = block;
  w->lds_bytes = lds;
  w->blob_bytes = bb.bytes.size();
  {  // FNV-1a over the snapshot: worlds built from the same descriptor agree
    uint64_t h = 1469598103934665603ull;
    for (const char c : bb.bytes) h = (h ^ (uint8_t)c) * 1099511628211ull;
    w->snapshot_hash = h;
  }
  hipError_t e = hipMalloc(&w->blob, w->blob_bytes);
  if (e != hipSuccess) {
    delete w;
    return set_error(MPG_E_HIP, std::string("hipMalloc(snapshot): ") + hipGetErrorString(e));
  }
  e = hipMemcpy(w->blob, bb.bytes.data(), w->blob_bytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    hipFree(w->blob);
    delete w;
    return set_error(MPG_E_HIP, std::string("hipMemcpy(snapshot): ") + hipGetErrorString(e));
  }
  char* base = static_cast<char*>(w->blob);
  DevWorld& dw = w->dw;
  dw.nj = d->n_joints;
  dw.dof = d->dof;
  dw.n_links = d->n_links;
  dw.n_geoms = d->n_geoms;
  dw.n_moving = d->n_moving;
  dw.n_static = d->n_static;
  dw.n_pairs = d->n_pairs;
  dw.W = W;
  dw.mpr_tol = d->gjk_tolerance;
  dw.bp_margin = bp_margin;
  dw.small_margin = small_margin;
  dw.n_prism = n_prism;
  dw.prism_bound = to_cptr<double>(base + o_pbd);
  dw.pose_bound = pose_bound;
  dw.all_mask = to_cptr<int>(base + o_amk);
#ifdef MPG_DIAG  // ablation builds only (changes results)
  if (const char* m = std::getenv("MPG_DEBUG_MARGIN")) {
    dw.bp_margin = (float)std::atof(m);
    dw.small_margin = std::atof(m);
  }
#endif
  dw.debug_mode = 0;
#ifdef MPG_DIAG  // ablation builds only (changes results)
  if (const char* e = std::getenv("MPG_DEBUG_CULL")) dw.debug_mode = std::atoi(e);
#endif
  dw.big_vis = nullptr;
  dw.big_busy = nullptr;
  dw.big_slots = 0;
  dw.big_words = big_words;
  if (big_words > 0) {  // one visited set per resident wave at most (256 CUs x 32 waves)
    dw.big_slots = 8192;
    HIP_TRY(hipMalloc(&dw.big_vis, sizeof(unsigned long long) * (size_t)dw.big_slots * big_words));
    HIP_TRY(hipMemset(dw.big_vis, 0, sizeof(unsigned long long) * (size_t)dw.big_slots * big_words));
    HIP_TRY(hipMalloc(&dw.big_busy, sizeof(int) * (size_t)dw.big_slots));
    HIP_TRY(hipMemset(dw.big_busy, 0, sizeof(int) * (size_t)dw.big_slots));
  }
  dw.stats = nullptr;
  if (std::getenv("MPG_STATS") && std::atoi(std::getenv("MPG_STATS")) > 0) {
    HIP_TRY(hipMalloc(&dw.stats, 64 * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(dw.stats, 0, 64 * sizeof(unsigned long long)));
  }
  dw.joint_type = to_cptr<int>(base + o_jt);
  dw.joint_parent = to_cptr<int>(base + o_jp);
  dw.joint_q_source = to_cptr<int>(base + o_jqs);
  dw.joint_q_const = to_cptr<double>(base + o_jqc);
  dw.joint_axis = to_cptr<double>(base + o_ja);
  dw.joint_place = to_cptr<double>(base + o_jpl);
  dw.link_parent = to_cptr<int>(base + o_lp);
  dw.link_place = to_cptr<double>(base + o_lpl);
  dw.geom_type = to_cptr<int>(base + o_gt);
  dw.geom_gstart = to_cptr<int>(base + o_gvs);
  dw.geom_ng = to_cptr<int>(base + o_gnv);
  dw.geom_nvert = to_cptr<int>(base + o_gnvt);
  dw.geom_rec = to_cptr<double>(base + o_grec);
  dw.hull = to_cptr<double>(base + o_v);
  dw.hull_doubles = (int)hull.size();
  dw.geom_cbase = to_cptr<int>(base + o_cb);
  dw.cell_rec = to_cptr<double>(base + o_crec);
  dw.cell_ovf = to_cptr<double>(base + o_covf);
  dw.geom_nbr = to_cptr<int>(base + o_gnb);
  dw.hull_nbr = to_cptr<int>(base + o_hnb);
  dw.nbr_ent = to_cptr<double>(base + o_nent);
  dw.wcell_rec = to_cptr<double>(base + o_wrec);
  dw.wcell_ovf = to_cptr<double>(base + o_wovf);
  dw.wcell_aux = to_cptr<double>(base + o_waux);
  dw.wcell_end = to_cptr<int>(base + o_wend);
  dw.wcell_end2 = to_cptr<int>(base + o_wend2);
  dw.wcell_pre = to_cptr<int>(base + o_wpre);
  dw.walk_subk = walk_subk;
  dw.moving_link = to_cptr<int>(base + o_ml);
  dw.moving_geom = to_cptr<int>(base + o_mg);
  dw.moving_offset = to_cptr<double>(base + o_mo);
  dw.static_geom = to_cptr<int>(base + o_sg);
  dw.static_rec = to_cptr<double>(base + o_srec);
  dw.pair_a = to_cptr<int>(base + o_pa);
  dw.pair_b = to_cptr<int>(base + o_pb);
  dw.pair_allowed = to_cptr<int>(base + o_al);
  dw.pair_cf = to_cptr<int>(base + o_cf);
  for (int p = 0; p < d->n_pairs; ++p) {
    w->has_closed_form |= pair_cf[p] != CF_NONE && !allowed[p];
    w->has_octree |= pair_cf[p] == CF_OCTREE && !allowed[p];
    w->octree_first |= pair_cf[p] == CF_OCTREE && !allowed[p] && obj_geom_type(d, d->pair_a[p]) == MPG_GEOM_OCTREE;
    w->any_closed_form |= pair_cf[p] != CF_NONE && cf_class(pair_cf[p]) == CLS_CLOSED;
    w->any_octree |= pair_cf[p] == CF_OCTREE;
    w->has_mesh |= pair_cf[p] == CF_MESH && !allowed[p];
    w->any_mesh |= pair_cf[p] == CF_MESH;
    w->any_gjk |= pair_cf[p] == CF_GJK;
    w->has_octree2 |= !allowed[p] && obj_geom_type(d, d->pair_a[p]) == MPG_GEOM_OCTREE &&
                      obj_geom_type(d, d->pair_b[p]) == MPG_GEOM_OCTREE;
  }
  dw.static_T = to_cptr<double>(base + o_sT);
  dw.link_chain_start = to_cptr<int>(base + o_cs);
  dw.link_chain_len = to_cptr<int>(base + o_cl);
  dw.chain_joints = to_cptr<int>(base + o_cj);
  auto I = [&](size_t o) { return to_cptr<int>(base + o); };
  dw.sched_start = I(o_ss);
  dw.sched_pair = I(o_sp);
  dw.sched_other = I(o_so);
  dw.st_start = I(o_sts);
  dw.st_m = I(o_stm);
  dw.st_r = to_cptr<float>(base + o_str);
  auto F = [&](size_t o) { return to_cptr<float>(base + o); };
  BpView& bp = dw.bp;
  bp.nj = d->n_joints;
  bp.n_links = d->n_links;
  bp.n_moving = d->n_moving;
  bp.n_static = d->n_static;
  bp.n_saves = bpp.n_saves;
  bp.joint_type = dw.joint_type;
  bp.joint_q_source = dw.joint_q_source;
  bp.joint_q_const = dw.joint_q_const;
  bp.jsrc = I(o_bjs);
  bp.jsave = I(o_bjv);
  bp.jaxis = F(o_bja);
  bp.jplace = F(o_bjp);
  bp.link_start = I(o_bls);
  bp.link_order = I(o_blo);
  bp.lplace = F(o_blp);
  bp.obj_start = I(o_bos);
  bp.obj_order = I(o_boo);
  bp.moving_link = dw.moving_link;
  bp.moff = F(o_bmo);
  bp.mobj = F(o_bmb);
  bp.sobj = F(o_bsb);
  bp.jkind = I(o_bjk);
  bp.jobj_start = I(o_bjo);
  bp.jobj_order = I(o_bjr);
  bp.oplace = F(o_bop);
  bp.oquat = F(o_boq);
  bp.ocen = F(o_boc);
  dw.oct_leaf = to_cptr<double>(base + o_olf);
  dw.oct_path = to_cptr<uint64_t>(base + o_opa);
  dw.oct_depth = to_cptr<int>(base + o_ode);
  dw.mesh_tri = to_cptr<double>(base + o_mtr);
  dw.mesh_node = to_cptr<double>(base + o_mnd);
  dw.mesh_link = to_cptr<int>(base + o_mln);
  dw.mesh_tree = to_cptr<int>(base + o_mtt);
  dw.fb_box = to_cptr<double>(base + o_fbb);
  dw.fb_link = to_cptr<int>(base + o_fbl);
  dw.fb_root = to_cptr<int>(base + o_fbr);
  dw.tri_pos = to_cptr<int>(base + o_tps);
  dw.sobb = to_cptr<double>(base + o_sob);
  dw.lat_rec = to_cptr<double>(base + o_lrec);
  dw.lat_rec_ok = lat_rec_ok ? 1 : 0;
  dw.oct_grid = to_cptr<double>(base + o_ogr);
  dw.oct_cells = I(o_oce);
  dw.oct_list = I(o_oli);
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  // persistent narrow grid: exactly the resident workgroups
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, narrow_kernel<false>, 256, 0) != hipSuccess || per_cu <= 0)
    per_cu = 2;
  w->narrow_blocks = cus * per_cu;
  // bound the candidate lists to 1 GiB: cap * n_pairs * 4 B
  w->max_chunk = std::max<long long>(4096, std::min<long long>(1 << 20, (1ll << 28) / std::max(d->n_pairs, 1)));
  if (const char* e = std::getenv("MPG_SMALL_BATCH_MAX")) w->small_max = std::atoll(e);
  if (const char* e = std::getenv("MPG_SMALL_ZEROCOPY")) w->small_zero_copy = std::atoi(e) != 0;
  if (const char* e = std::getenv("MPG_OVERLAP_MIN")) w->overlap_min = std::atoll(e);
  if (const char* e = std::getenv("MPG_HOST_STREAMS")) w->ring_streams = std::atoi(e) > 1 ? 2 : 1;
  if (const char* e = std::getenv("MPG_HOST_THREADS")) w->host_threads = std::max(1, std::min(64, std::atoi(e)));
  if (const char* e = std::getenv("MPG_HOST_HEAD")) w->ring_head = std::max(0ll, std::atoll(e));
  if (const char* e = std::getenv("MPG_HOST_TAIL")) w->ring_tail = std::max(0ll, std::atoll(e));
  if (const char* e = std::getenv("MPG_HOST_CHUNK"))
    w->ring_chunk = std::max(64ll, std::min((long long)w->max_chunk, (std::atoll(e) + 63) / 64 * 64));
  if (const char* e = std::getenv("MPG_SMALL_INLINE_SC")) w->small_inline_sc = std::atoll(e);
  if (const char* e = std::getenv("MPG_OVERLAP_PARTS")) w->overlap_parts = std::atoi(e);
  if (const char* e = std::getenv("MPG_SMALL_HOST_SC")) w->small_host_sc = std::atoll(e);
  if (const char* e = std::getenv("MPG_SMALL_ARGS")) w->small_args = std::atoi(e) != 0;
  for (int j = 0; j < d->n_joints; ++j)
    if (d->joint_q_source[j] >= 0 && joint_is_revolute(d->joint_type[j]) &&
        std::find(w->h_rev_src.begin(), w->h_rev_src.end(), d->joint_q_source[j]) == w->h_rev_src.end())
      w->h_rev_src.push_back(d->joint_q_source[j]);
  if (const char* e = std::getenv("MPG_SMALL_SERVER")) w->srv_mode = std::atoi(e);
  w->srv_stats = std::getenv("MPG_STATS") != nullptr;
  if (const char* e = std::getenv("MPG_SMALL_SERVER_IDLE_US")) w->srv_idle_us = std::max(10ll, std::atoll(e));
  if (const char* e = std::getenv("MPG_SMALL_SERVER_WG")) w->srv_g = std::min(kSrvMaxG, std::max(1, std::atoi(e)));
  if (const char* e = std::getenv("MPG_SMALL_SERVER_MAX")) w->srv_max_n = std::min(kSrvN, std::max(1, std::atoi(e)));
  w->srv_lds = srv_lds_bytes(d->n_moving, d->n_pairs, d->dof, w->dw.W, d->n_joints, d->n_static);
  w->srv_ok = lat_rec_ok && !w->any_octree && !w->any_mesh && !w->any_gjk && d->dof > 0 && d->dof <= kLatScDof &&
              d->n_pairs > 0 && w->dw.W <= kSrvMaxW && w->srv_lds <= 144 * 1024;  // + ~11 KB static LDS
  const char* own = std::getenv("MPG_OWN_STREAM");
  if (!own || std::atoi(own) != 0) HIP_TRY(hipStreamCreateWithFlags(&w->own_stream, hipStreamNonBlocking));
  *out = w;
  return MPG_OK;
}

int mpg_world_destroy(mpg_world* w) {
  if (!w) return MPG_OK;
  hipSetDevice(w->device);
  if (w->dw.big_vis) hipFree(w->dw.big_vis);
  if (w->dw.big_busy) hipFree(w->dw.big_busy);
  if (w->dw.stats) {
    unsigned long long st[64];
    hipDeviceSynchronize();
    hipMemcpy(st, w->dw.stats, sizeof(st), hipMemcpyDeviceToHost);
    std::fprintf(stderr,
                 "[mpg stats] small_kernel phases (sum over waves / max per wave, us): pre %.1f/%.2f, record %.1f/%.2f, "
                 "fk %.1f/%.2f, spheres %.1f/%.2f, narrow %.1f/%.2f, store %.1f/%.2f, wave %.1f/%.2f\n",
                 st[24] / 100.0, st[32] / 100.0, st[25] / 100.0, st[33] / 100.0, st[26] / 100.0, st[34] / 100.0,
                 st[27] / 100.0, st[35] / 100.0, st[28] / 100.0, st[36] / 100.0, st[29] / 100.0, st[37] / 100.0,
                 st[30] / 100.0, st[38] / 100.0);
    if (st[42])
      std::fprintf(stderr, "[mpg stats] latency server probe: dependent cell-record loads, shader clocks each: "
                   "first pass %.0f, again %.0f\n", (double)st[40] / st[42], (double)st[41] / st[43]);
    if (st[20])
      std::fprintf(stderr, "[mpg stats] latency server MPR steps: %llu (max %llu per pair), shader clocks per step: "
                   "support %.0f, advance %.0f\n", st[20], st[23], (double)st[21] / st[20], (double)st[22] / st[20]);
    if (st[52])
      std::fprintf(stderr, "[mpg stats] walk-hull support phases, shader clocks per hull support (%llu): cell lookup "
                   "%.0f, record load + inline dots %.0f, overflow entries %.0f, tie / trap checks %.0f\n",
                   st[52], (double)st[48] / st[52], (double)st[49] / st[52], (double)st[50] / st[52],
                   (double)st[51] / st[52]);
    std::fprintf(stderr, "[mpg stats] small_kernel slowest narrow test: pair %llu, %.2f us\n",
                 (unsigned long long)(st[31] & 4095), (st[31] >> 12) / 100.0);
    std::fprintf(stderr, "[mpg stats] walk hulls: supports %llu, trap-free fast %llu, verified %llu, full walks %llu, "
                 "certified endpoints %llu; pending: tie %llu, uncertified %llu, resumed %llu; resolve ticks: verify %llu, walk %llu\n",
                 st[10], st[11], st[12], st[13], st[14], st[16], st[17], st[18], st[9], st[15]);
    std::fprintf(stderr,
                 "[mpg stats] narrow: refill %llu, support %llu, update %llu (memtime ticks, summed over waves); "
                 "steps %llu, mean active lanes/step %.1f; hits %llu (%.2f supports each), misses %llu (%.2f)\n",
                 st[3], st[4], st[5], st[7], st[7] ? (double)st[6] / st[7] : 0.0, st[2],
                 st[2] ? (double)st[0] / st[2] : 0.0, st[8], st[8] ? (double)st[1] / st[8] : 0.0);
    hipFree(w->dw.stats);
  }
  if (w->srv_stats && w->srv_stat[5] > 0)
    std::fprintf(stderr, "[mpg stats] latency server, mean us over %.0f batches: rows %.2f, fk %.2f, spheres %.2f, "
                 "narrow %.2f, publish %.2f; host post->done %.2f\n", w->srv_stat[5], w->srv_stat[0] / w->srv_stat[5],
                 w->srv_stat[1] / w->srv_stat[5], w->srv_stat[2] / w->srv_stat[5], w->srv_stat[3] / w->srv_stat[5],
                 w->srv_stat[4] / w->srv_stat[5], w->srv_stat[6] / w->srv_stat[5]);
  if (w->srv_stats && w->hp_stat[0] > 0)
    std::fprintf(stderr, "[mpg stats] host pipeline, mean us over %.0f calls: input copies %.1f, issue %.1f, "
                 "result wait %.1f, unpack %.1f; whole call %.1f\n", w->hp_stat[0], w->hp_stat[1] / w->hp_stat[0],
                 w->hp_stat[2] / w->hp_stat[0], w->hp_stat[3] / w->hp_stat[0], w->hp_stat[4] / w->hp_stat[0],
                 w->hp_stat[5] / w->hp_stat[0]);
  if (w->srv_h) {  // the server leaves at its next poll
    __atomic_store_n(&w->srv_h->quit, 1ull, __ATOMIC_RELEASE);
    hipStreamSynchronize(w->srv_stream);
    hipStreamDestroy(w->srv_stream);
    hipHostFree(w->srv_h);
  }
  hipFree(w->blob);
  if (w->h_q) hipHostFree(w->h_q);
  if (w->h_hits) hipHostFree(w->h_hits);
  hipFree(w->d_qs);
  if (w->d_ssc) hipFree(w->d_ssc);
  if (w->h_ssc) hipHostFree(w->h_ssc);
  if (w->own_stream) hipStreamDestroy(w->own_stream);
  for (auto& kv : w->sides) {
    hipStreamDestroy(kv.second.side);
    hipEventDestroy(kv.second.fork);
    hipEventDestroy(kv.second.join);
  }
  hipFree(w->d_q);
  hipFree(w->d_flags);
  hipFree(w->d_masks);
  hipFree(w->d_out);
  free_ring(w);
  w->pool.reset();
  if (w->ring.h2d) {
    hipStreamDestroy(w->ring.h2d);
    hipStreamDestroy(w->ring.side);
    for (int j = 0; j < mpg_world::kRing; ++j) {
      hipEventDestroy(w->ring.e_in[j]);
      hipEventDestroy(w->ring.e_done[j]);
    }
  }
  for (auto& mk : w->marks) {
    hipEventDestroy(mk.a);
    hipEventDestroy(mk.b);
  }
  for (hipEvent_t e : w->ev_pool) hipEventDestroy(e);
  hipFree(w->dist.poses);
  hipFree(w->dist.save64);
  hipFree(w->dist.q);
  hipFree(w->dist.out);
  hipFree(w->dist.pts);
  if (w->dist.last) hipEventDestroy(w->dist.last);
  hipFree(w->dist.big);
  hipFree(w->dist.list);
  if (w->gather_ev) hipEventDestroy(w->gather_ev);
  if (w->motion.last) hipEventDestroy(w->motion.last);
  hipFree(w->contact.in);
  hipFree(w->contact.out);
  hipFree(w->contact.fl);
  hipFree(w->contact.mk);
  hipFree(w->motion.edges);
  hipFree(w->motion.segs);
  hipFree(w->motion.offs);
  hipFree(w->motion.out);
  hipFree(w->motion.states);
  hipFree(w->motion.flags);
  hipFree(w->prof_units);
  for (auto& kv : w->ws)
  {
    for (uint32_t* p : {kv.second.surv, kv.second.cnt, kv.second.seg_len, kv.second.seg_start, kv.second.prefix,
                        kv.second.cand})
      hipFree(p);
    hipFree(kv.second.rq);
    hipFree(kv.second.sc);
  }
  delete w;
  return MPG_OK;
}

int mpg_world_get_info(const mpg_world* w, mpg_world_info* info) {
  if (!w || !info) return set_error(MPG_E_INVALID, "NULL argument");
  info->n_pairs = w->dw.n_pairs;
  info->mask_words = w->dw.W;
  info->dof = w->dw.dof;
  info->n_links = w->dw.n_links;
  info->device = w->device;
  info->block_size = w->block;
  info->snapshot_bytes = (int64_t)w->blob_bytes;
  return MPG_OK;
}

}  // extern "C"

namespace {
// pinned input rows (ncfg * row doubles: q rows or link poses), hit bytes
// (n_pairs * ncfg) and joint sincos: the input capacity is tracked in doubles,
// since the same buffers serve q rows (dof) and link-pose rows (n_links * 7)
int ensure_small(mpg_world* w, size_t ncfg, size_t row) {
  const size_t want_q = ncfg * std::max<size_t>(row, 1);
  if (ncfg <= w->small_cap && want_q <= w->small_qcap) return MPG_OK;
  ncfg = std::max(ncfg, w->small_cap);
  const size_t qcap = std::max(want_q, w->small_qcap);
  if (w->h_q) hipHostFree(w->h_q);
  if (w->h_hits) hipHostFree(w->h_hits);
  if (w->d_qs) hipFree(w->d_qs);
  if (w->d_ssc) hipFree(w->d_ssc);
  if (w->h_ssc) hipHostFree(w->h_ssc);
  w->d_ssc = nullptr;
  w->h_ssc = nullptr;
  w->h_q = nullptr;
  w->h_hits = nullptr;
  w->d_qs = nullptr;
  w->small_cap = 0;
  w->small_qcap = 0;
  const size_t P = (size_t)std::max(w->dw.n_pairs, 1);
  HIP_TRY(hipHostMalloc((void**)&w->h_q, sizeof(double) * qcap, hipHostMallocMapped | hipHostMallocCoherent));
  HIP_TRY(hipHostGetDevicePointer((void**)&w->d_qmap, w->h_q, 0));
  HIP_TRY(hipHostMalloc((void**)&w->h_hits, P * ncfg, hipHostMallocMapped | hipHostMallocCoherent));
  HIP_TRY(hipHostGetDevicePointer((void**)&w->d_hits, w->h_hits, 0));
  HIP_TRY(hipMalloc(&w->d_qs, sizeof(double) * qcap));
  HIP_TRY(hipMalloc(&w->d_ssc, sizeof(double) * 2 * ncfg * std::max<int>(w->dw.dof, 1)));
  HIP_TRY(hipHostMalloc((void**)&w->h_ssc, sizeof(double) * 2 * ncfg * std::max<int>(w->dw.dof, 1),
                        hipHostMallocMapped | hipHostMallocCoherent));
  HIP_TRY(hipHostGetDevicePointer((void**)&w->d_sscmap, w->h_ssc, 0));
  w->small_cap = ncfg;
  w->small_qcap = qcap;
  return MPG_OK;
}

// (re)start the latency server; it takes `done` as the last batch served
int srv_start(mpg_world* w) {
  if (!w->srv_h) {
    HIP_TRY(hipHostMalloc((void**)&w->srv_h, sizeof(SrvCtl), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(w->srv_h, 0, sizeof(SrvCtl));
    HIP_TRY(hipHostGetDevicePointer((void**)&w->srv_d, w->srv_h, 0));
    HIP_TRY(hipStreamCreateWithFlags(&w->srv_stream, hipStreamNonBlocking));
    HIP_TRY(hipFuncSetAttribute((const void*)lat_server_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)w->srv_lds));
  }
  for (int k = 0; k < kSrvMaxG; ++k) __atomic_store_n(&w->srv_h->gone[k], 0ull, __ATOMIC_RELAXED);
  __atomic_store_n(&w->srv_h->quit, 0ull, __ATOMIC_RELEASE);
  ++w->srv_starts;
  hipLaunchKernelGGL(lat_server_kernel, dim3(w->srv_g), dim3(kSrvThreads), w->srv_lds, w->srv_stream, w->dw, w->srv_d,
                     (unsigned long long)w->srv_idle_us * 100ull, w->srv_stats ? 1 : 0);
  HIP_TRY(hipGetLastError());
  w->srv_running = true;
  return MPG_OK;
}

// one batch through the resident server: rows (q, host sin/cos) into the
// control block, seq bumped, the host spins on `done`.  The server may have
// left (idle) before it saw the request: every 50 us the host looks for
// workgroups that have left (`gone`) without answering -- all of them (stream
// complete): start it again; some of them: stop the rest and start all again.
// Workgroups that are only slow (another stream sharing the GPU) are waited
// for.  No answer within 2 s: the server is stopped, MPG_E_HIP (the caller
// launches instead for a while, then tries the server again).
int collide_served(mpg_world* w, const double* q, int64_t n, uint8_t* flags, uint32_t* pair_mask) {
  if (w->srv_running && w->srv_quitting) {  // told to quit after a missed answer
    if (hipStreamQuery(w->srv_stream) != hipSuccess) return set_error(MPG_E_HIP, "latency server has not left yet");
    w->srv_running = false;
    w->srv_quitting = false;
  }
  if (!w->srv_running) {
    const int rc = srv_start(w);
    if (rc) return rc;
  }
  SrvCtl* C = w->srv_h;
  const int dof = w->dw.dof, W = w->dw.W;
  for (int64_t c = 0; c < n; ++c) {
    double* r = C->rows + c * 3 * dof;
    std::memcpy(r, q + c * dof, sizeof(double) * (size_t)dof);
    for (const int src : w->h_rev_src) mpg_sincos(q[c * dof + src], &r[dof + 2 * src], &r[dof + 2 * src + 1]);
  }
  const unsigned long long seq = (++w->srv_seq << 8) | (unsigned long long)n;
  __atomic_store_n(&C->seq, seq, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  long long next_us = 50;
  bool forced = false;
  auto all_done = [&] {
    for (int k = 0; k < w->srv_g; ++k)
      if (__atomic_load_n(&C->done[k], __ATOMIC_ACQUIRE) != seq) return false;
    return true;
  };
  while (!all_done()) {
    __builtin_ia32_pause();
    const long long us =
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    if (us < next_us) continue;
    next_us = us + 50;
    hipError_t e = hipStreamQuery(w->srv_stream);
    bool partial = false;  // a workgroup left before this request, others are still resident
    for (int k = 0; k < w->srv_g && e == hipErrorNotReady; ++k)
      partial |= __atomic_load_n(&C->gone[k], __ATOMIC_ACQUIRE) != 0ull &&
                 __atomic_load_n(&C->done[k], __ATOMIC_ACQUIRE) != seq;
    if (partial && !forced) {
      // stop the ones still polling and start all again (once per request);
      // they see quit within one poll, so this wait is short
      __atomic_store_n(&C->quit, 1ull, __ATOMIC_RELEASE);
      e = hipStreamSynchronize(w->srv_stream);
      forced = true;
    }
    if (e == hipSuccess) {  // it left before this request: start it again
      w->srv_running = false;
      const int rc = srv_start(w);
      if (rc) return rc;
    } else if (e != hipErrorNotReady || us > 2000000) {
      __atomic_store_n(&C->quit, 1ull, __ATOMIC_RELEASE);
      w->srv_quitting = true;  // not waited for here: the next try checks that it has left
      return set_error(MPG_E_HIP, "latency server did not answer");
    }
  }
  ++w->srv_served;
  if (w->prof) {  // a served batch counts as one narrow-stage "launch" of its post -> done time
    std::lock_guard<std::mutex> lk(w->prof_mu);
    w->prof_ms[MPG_STAGE_NARROW] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    w->prof_n[MPG_STAGE_NARROW] += 1;
    w->prof_cfg += n;
  }
  if (w->srv_stats) {  // MPG_STATS: phase sums (rows, fk, spheres, narrow, publish), us
    w->srv_stat[5] += 1.0;
    for (int k = 0; k < 5; ++k) w->srv_stat[k] += (double)(C->phase[k + 1] - C->phase[k]) / 100.0;
    w->srv_stat[6] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  }
  for (int64_t c = 0; c < n; ++c) {
    uint32_t any = 0;
    for (int k = 0; k < W; ++k) {
      uint32_t v = 0;
      for (int gg = 0; gg < w->srv_g; ++gg) v |= __atomic_load_n(&C->out[gg][c * W + k], __ATOMIC_RELAXED);
      any |= v;
      if (pair_mask) pair_mask[c * W + k] = v;
    }
    flags[c] = any ? 1 : 0;
  }
  return MPG_OK;
}

// one round trip: input to the device, one small_kernel launch writing hit
// bytes straight into host memory, one synchronisation; the host folds the
// hits into flags / pair masks
template <bool FROM_POSES>
int collide_small(mpg_world* w, const double* q, int64_t n, uint8_t* flags, uint32_t* pair_mask, hipStream_t s) {
  if (!FROM_POSES && w->srv_mode && w->srv_ok && n <= w->srv_max_n && !w->dw.dbg(3) && !w->dw.dbg(7) &&
      (!w->srv_broken || std::chrono::steady_clock::now() >= w->srv_retry_at)) {
    if (collide_served(w, q, n, flags, pair_mask) == MPG_OK) {
      w->srv_broken = false;
      return MPG_OK;
    }
    // the server could not be started or did not answer: launches for the
    // next second, then the server is tried again
    std::fprintf(stderr, "mplib_amd: latency server unavailable (%s); one launch per batch for 1 s\n",
                 g_last_error.c_str());
    w->srv_broken = true;
    ++w->srv_fallbacks;
    w->srv_retry_at = std::chrono::steady_clock::now() + std::chrono::seconds(1);
    (void)hipGetLastError();
  }
  const size_t row = FROM_POSES ? (size_t)w->dw.n_links * 7 : (size_t)w->dw.dof;
  const size_t cap = std::max<size_t>((size_t)n, std::min<size_t>((size_t)w->small_max, 256));
  int rc = ensure_small(w, cap, row);
  if (rc) return rc;
  const int P = w->dw.n_pairs, W = w->dw.W;
  std::memset(flags, 0, (size_t)n);
  if (pair_mask) std::memset(pair_mask, 0, sizeof(uint32_t) * (size_t)n * W);
  if (P == 0) return MPG_OK;
  const double* qin = w->small_zero_copy ? w->d_qmap : w->d_qs;
  if (row) {  // zero-copy: the kernel reads the pinned rows directly, no copy launch
    std::memcpy(w->h_q, q, sizeof(double) * (size_t)n * row);
    if (!w->small_zero_copy)
      HIP_TRY(hipMemcpyAsync(w->d_qs, w->h_q, sizeof(double) * (size_t)n * row, hipMemcpyHostToDevice, s));
  }
  const int n_tiles = (int)((n + 63) / 64);
  const long long waves = (long long)P * n_tiles;
  StageTimer t_small(w, s, MPG_STAGE_NARROW);
  if (w->prof) w->prof_cfg += n;
  // the smallest batches: joint sin/cos on the host (mpg_sincos, the device's
  // own restatement of glibc's, bit for bit) into pinned mapped memory, one
  // launch without the sin/cos work; up to small_inline_sc states: one launch
  // with sin/cos inline; larger: a sin/cos launch first
  const bool host_sc = !FROM_POSES && w->dw.dof > 0 && n <= w->small_host_sc;
  const bool inline_sc = !host_sc && (FROM_POSES || (n <= w->small_inline_sc && w->dw.dof <= kLatScDof));
  double* sc_src = w->d_ssc;
  if (host_sc) {
    const int dof = w->dw.dof;
    for (int64_t c = 0; c < n; ++c)
      for (const int src : w->h_rev_src) {
        double sv, cv;
        mpg_sincos(q[c * dof + src], &sv, &cv);
        w->h_ssc[(c * dof + src) * 2] = sv;
        w->h_ssc[(c * dof + src) * 2 + 1] = cv;
      }
    sc_src = w->d_sscmap;
  }
  if (!inline_sc && !host_sc && w->dw.dof > 0) {
    const long long nt = n * w->dw.dof;
    hipLaunchKernelGGL(small_sincos_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, w->dw, qin,
                       (long long)n, w->d_ssc);
    HIP_TRY(hipGetLastError());
  }
  const dim3 grid((unsigned)((waves + 3) / 4));
  const bool host_staged = host_sc && w->dw.dof <= kLatScDof && w->dw.lat_rec_ok;
  // the fewest states: their rows travel in the kernel arguments
  const bool by_args = host_staged && n * 3 * (int64_t)w->dw.dof <= kLatIn && w->small_args;
  LatIn args{};
  if (by_args) {
    const int dof = w->dw.dof;
    for (int64_t c = 0; c < n; ++c) {
      double* r = args.d + c * 3 * dof;
      std::memcpy(r, q + c * dof, sizeof(double) * (size_t)dof);
      std::memcpy(r + dof, w->h_ssc + c * 2 * dof, sizeof(double) * 2 * (size_t)dof);
    }
  }
  auto launch = [&](auto kern) {  // every class instance reads the same sin/cos source
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, w->dw, qin, (long long)n, n_tiles, w->d_hits, sc_src, args);
    return hipGetLastError();
  };
  auto pick = [&](auto k0, auto k1, auto k2, auto k3) {
    return inline_sc ? launch(k1) : by_args ? launch(k3) : host_staged ? launch(k2) : launch(k0);
  };
  HIP_TRY(pick(small_kernel<FROM_POSES, CLS_CLOSED, 0>, small_kernel<FROM_POSES, CLS_CLOSED, 1>,
               small_kernel<FROM_POSES, CLS_CLOSED, 2>, small_kernel<FROM_POSES, CLS_CLOSED, 3>));
  if (w->any_octree)
    HIP_TRY(pick(small_kernel<FROM_POSES, CLS_OCTREE, 0>, small_kernel<FROM_POSES, CLS_OCTREE, 1>,
                 small_kernel<FROM_POSES, CLS_OCTREE, 2>, small_kernel<FROM_POSES, CLS_OCTREE, 3>));
  if (w->any_mesh)
    HIP_TRY(pick(small_kernel<FROM_POSES, CLS_MESH, 0>, small_kernel<FROM_POSES, CLS_MESH, 1>,
                 small_kernel<FROM_POSES, CLS_MESH, 2>, small_kernel<FROM_POSES, CLS_MESH, 3>));
  if (w->any_gjk)
    HIP_TRY(pick(small_kernel<FROM_POSES, CLS_GJK, 0>, small_kernel<FROM_POSES, CLS_GJK, 1>,
                 small_kernel<FROM_POSES, CLS_GJK, 2>, small_kernel<FROM_POSES, CLS_GJK, 3>));
  t_small.stop();
  HIP_TRY(hipStreamSynchronize(s));
  const uint8_t* h = w->h_hits;
  for (int p = 0; p < P; ++p) {
    const uint8_t* hp = h + (size_t)p * n;
    const uint32_t bit = 1u << (p & 31);
    for (int64_t c = 0; c < n; ++c)
      if (hp[c]) {
        flags[c] = 1;
        if (pair_mask) pair_mask[(size_t)c * W + (p >> 5)] |= bit;
      }
  }
  return MPG_OK;
}

// stream-ordered for the caller: the side stream waits for everything queued
// on `s` before the call, and `s` waits for the side stream's half
template <bool FROM_POSES>
int launch_collide_overlapped(mpg_world* w, const double* in, long long n, uint8_t* flags, uint32_t* masks,
                              hipStream_t s) {
  StreamPin pin(w, s);
  // one chunk or less runs on the caller's stream alone: its two halves'
  // cull and narrow kernels each fill the chip and are latency-bound, so on a
  // second stream they only time-share the CUs (cfg3, 2^20: single stream
  // +0.7-1.3 %; cfg4, 4 chunks: overlapped +16 %, profiles/r05a/overlap_ab.txt)
  if (w->overlap_min <= 0 || n < w->overlap_min || n <= w->max_chunk)
    return launch_collide<FROM_POSES>(w, in, n, flags, masks, s);
  // one side stream and fork/join event pair per caller stream: callers on
  // different streams (one host thread each, include/mpgpu.h) never record
  // into or wait on each other's events, and each side stream has its own
  // workspace (get_workspace keys by stream)
  mpg_world::Side sd;
  {
    std::lock_guard<std::mutex> lk(w->ws_mu);
    auto it = w->sides.find(s);
    if (it == w->sides.end()) {
      if (w->ws.find(s) == w->ws.end()) evict_streams_locked(w);
      mpg_world::Side n{};
      HIP_TRY(hipStreamCreateWithFlags(&n.side, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&n.fork, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&n.join, hipEventDisableTiming));
      it = w->sides.emplace(s, n).first;
    }
    it->second.last = ++w->ws_tick;
    sd = it->second;
  }
  const size_t row = FROM_POSES ? (size_t)w->dw.n_links * 7 : (size_t)w->dw.dof;
  // parts alternate between the caller's stream and the side stream
  const int parts = std::max(2, w->overlap_parts);
  const long long step = ((n + parts - 1) / parts + 63) / 64 * 64;
  HIP_TRY(hipEventRecord(sd.fork, s));
  HIP_TRY(hipStreamWaitEvent(sd.side, sd.fork, 0));
  int k = 0;
  for (long long off = 0; off < n; off += step, ++k) {
    const long long m = std::min(step, n - off);
    const int rc = launch_collide<FROM_POSES>(w, in + (size_t)off * row, m, flags + off,
                                              masks ? masks + (size_t)off * w->dw.W : nullptr, (k & 1) ? sd.side : s);
    if (rc) return rc;
  }
  HIP_TRY(hipEventRecord(sd.join, sd.side));
  HIP_TRY(hipStreamWaitEvent(s, sd.join, 0));
  return MPG_OK;
}

// Host buffers above the latency path's sizes (mpg_hostpipe.h): per chunk,
// the rows are copied from the caller's (pageable) buffer on the ring's copy
// stream by the feeder thread; the compute stream waits for them, runs the
// collide pipeline into the slot's device outputs, packs the colliding
// configurations' mask rows straight into pinned host memory and copies the
// flags back; the issuing thread unpacks a finished chunk into the caller's
// buffers while the next chunks are in flight.  PCIe carries the rows in
// (8 * row B per configuration) and 1 + 4W B per colliding configuration
// back instead of 1 + 4W B per configuration.  Caller holds host_mu.
template <bool FROM_POSES>
struct HostPipeOps {
  mpg_world* w;
  const double* q;
  uint8_t* flags;
  uint32_t* pair_mask;
  hipStream_t s;
  size_t row;
  // the first error text of the feeder / issuer threads (g_last_error is per
  // thread); finish() runs on the caller's thread and sets g_last_error itself
  std::mutex err_mu;
  std::string thread_err;
  bool fin_failed = false;

  int thread_fail(int rc, const std::string& msg) {
    std::lock_guard<std::mutex> lk(err_mu);
    if (thread_err.empty()) thread_err = msg;
    return rc;
  }
  int bind_thread() {
    if (hipSetDevice(w->device) != hipSuccess) return thread_fail(MPG_E_HIP, "hipSetDevice failed in a pipeline thread");
    return MPG_OK;
  }
  double t_in = 0, t_issue = 0, t_wait = 0, t_unpack = 0;
  static double us_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  }
  int h2d(int64_t, int j, int64_t start, int64_t m) {
    auto& R = w->ring;
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = hipSuccess;
    if (row) e = hipMemcpyAsync(R.d_in[j], q + (size_t)start * row, sizeof(double) * (size_t)m * row,
                                hipMemcpyHostToDevice, R.h2d);
    if (e == hipSuccess) e = hipEventRecord(R.e_in[j], R.h2d);
    t_in += us_since(t0);
    if (e != hipSuccess) return thread_fail(MPG_E_HIP, std::string("host pipeline input copy failed: ") + hipGetErrorString(e));
    return MPG_OK;
  }
  int issue(int64_t k, int j, int64_t start, int64_t m) {
    const int rc = issue_chunk(k, j, start, m);
    return rc ? thread_fail(rc, g_last_error) : MPG_OK;  // g_last_error of this (issuer) thread
  }
  int issue_chunk(int64_t k, int j, int64_t, int64_t m) {
    auto& R = w->ring;
    const auto t0 = std::chrono::steady_clock::now();
    const hipStream_t cs = (w->ring_streams > 1 && (k & 1)) ? R.side : s;
    HIP_TRY(hipStreamWaitEvent(cs, R.e_in[j], 0));
    const int rc = launch_collide<FROM_POSES>(w, R.d_in[j], m, R.d_fl[j], R.d_mk[j], cs);
    if (rc) return rc;
    // results straight into pinned host memory: the flags, and with masks the
    // block counts and the packed rows (no copy launches)
    const int Wp = pair_mask ? w->dw.W : 0;
    const unsigned nb = (unsigned)((m + kPackCfg - 1) / kPackCfg);
    if (Wp > 0) {
      hipLaunchKernelGGL(flag_count_kernel, dim3(nb), dim3(256), 0, cs, R.d_fl[j], (long long)m, R.d_bcnt[j],
                         R.h_bcnt_d[j]);
      HIP_TRY(hipGetLastError());
    }
    const size_t lds = sizeof(uint32_t) * 256 * (size_t)Wp;
    if (lds <= 64 * 1024)
      hipLaunchKernelGGL(mask_pack_kernel<true>, dim3(nb), dim3(256), lds, cs, R.d_fl[j], R.d_mk[j], (long long)m, Wp,
                         R.d_bcnt[j], R.h_mk_d[j], R.h_fl_d[j]);
    else
      hipLaunchKernelGGL(mask_pack_kernel<false>, dim3(nb), dim3(256), 0, cs, R.d_fl[j], R.d_mk[j], (long long)m, Wp,
                         R.d_bcnt[j], R.h_mk_d[j], R.h_fl_d[j]);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(R.e_done[j], cs));
    t_issue += us_since(t0);
    return MPG_OK;
  }
  int finish(int64_t, int j, int64_t start, int64_t m) {
    auto& R = w->ring;
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = hipEventSynchronize(R.e_done[j]);
    if (e != hipSuccess) {
      fin_failed = true;
      return set_error(MPG_E_HIP, std::string("host pipeline: ") + hipGetErrorString(e));
    }
    const auto t1 = std::chrono::steady_clock::now();
    t_wait += std::chrono::duration<double, std::micro>(t1 - t0).count();
    mpg_hostpipe::unpack_chunk(w->pool.get(), R.h_fl[j], R.h_mk[j], R.h_bcnt[j], kPackCfg, m, w->dw.W, flags + start,
                               pair_mask && w->dw.W > 0 ? pair_mask + (size_t)start * w->dw.W : nullptr);
    t_unpack += us_since(t1);
    return MPG_OK;
  }
  void drain() {
    hipStreamSynchronize(w->ring.h2d);
    hipStreamSynchronize(w->ring.side);
    hipStreamSynchronize(s);
  }
};

template <bool FROM_POSES>
int collide_host_pipelined(mpg_world* w, const double* q, int64_t n, uint8_t* flags, uint32_t* pair_mask,
                           hipStream_t s) {
  const mpg_hostpipe::Plan p =
      mpg_hostpipe::plan(n, w->ring_chunk, 1 << 15, mpg_world::kRing, w->ring_head, w->ring_tail);
  const size_t row = FROM_POSES ? (size_t)w->dw.n_links * 7 : (size_t)w->dw.dof;
  int rc = ensure_ring(w, (size_t)p.chunk, row);
  if (rc) return rc;
  if (!w->pool && w->host_threads > 1 && p.chunk >= 2 * kPackCfg)
    w->pool.reset(new mpg_hostpipe::Pool(w->host_threads - 1));
  HostPipeOps<FROM_POSES> ops{w, q, flags, pair_mask, s, row};
  const auto t0 = std::chrono::steady_clock::now();
  rc = mpg_hostpipe::run(p, n, ops);
  if (w->srv_stats) {
    const double v[6] = {1.0, ops.t_in, ops.t_issue, ops.t_wait, ops.t_unpack, HostPipeOps<FROM_POSES>::us_since(t0)};
    for (int k = 0; k < 6; ++k) w->hp_stat[k] += v[k];
  }
  if (rc && !ops.fin_failed) return set_error(rc, ops.thread_err);
  return rc;
}

template <bool FROM_POSES>
int collide_common(mpg_world* w, const double* q, int64_t n, uint8_t* flags, uint32_t* pair_mask, int mem,
                   void* stream) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  if (n < 0) return set_error(MPG_E_INVALID, "n < 0");
  const size_t row = FROM_POSES ? (size_t)w->dw.n_links * 7 : (size_t)w->dw.dof;
  // a world without inputs (dof 0) may pass q = NULL
  if (n > 0 && ((!q && row > 0) || !flags)) return set_error(MPG_E_INVALID, "input/flags is NULL");
  HIP_TRY(hipSetDevice(w->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (mem == MPG_MEM_DEVICE) return launch_collide_overlapped<FROM_POSES>(w, q, n, flags, pair_mask, s);
  if (mem != MPG_MEM_HOST) return set_error(MPG_E_INVALID, "bad mem kind");
  std::lock_guard<std::mutex> lk(w->host_mu);
  if (!s && w->own_stream) s = w->own_stream;
  if (n == 0) return MPG_OK;
  if (n <= w->small_max) return collide_small<FROM_POSES>(w, q, n, flags, pair_mask, s);
  return collide_host_pipelined<FROM_POSES>(w, q, n, flags, pair_mask, s);
}
}  // namespace

extern "C" {

int mpg_release_stream(mpg_world* w, void* stream) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  HIP_TRY(hipSetDevice(w->device));
  std::lock_guard<std::mutex> lk(w->ws_mu);
  const auto b = w->busy.find(static_cast<hipStream_t>(stream));
  if (b != w->busy.end() && b->second > 0) return set_error(MPG_E_INVALID, "stream has a call in progress");
  release_stream_locked(w, static_cast<hipStream_t>(stream));
  return MPG_OK;
}

int mpg_set_small_batch_max(mpg_world* w, int64_t n) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  if (n < 0) return set_error(MPG_E_INVALID, "n < 0");
  std::lock_guard<std::mutex> lk(w->host_mu);
  w->small_max = n;
  return MPG_OK;
}

int mpg_collide_batch(mpg_world* w, const double* q, int64_t n, uint8_t* flags, uint32_t* pair_mask, int mem,
                      void* stream) {
  return collide_common<false>(w, q, n, flags, pair_mask, mem, stream);
}

int mpg_collide_batch_multi(mpg_world* const* worlds, int32_t n_worlds, const double* q, int64_t n, uint8_t* flags,
                            uint32_t* pair_mask) {
  if (n_worlds <= 0 || !worlds) return set_error(MPG_E_INVALID, "no worlds");
  if (n < 0) return set_error(MPG_E_INVALID, "n < 0");
  if (n > 0 && (!q || !flags)) return set_error(MPG_E_INVALID, "q / flags is NULL");
  mpg_world_info i0{};
  for (int k = 0; k < n_worlds; ++k) {
    mpg_world_info ik{};
    if (!worlds[k]) return set_error(MPG_E_INVALID, "world " + std::to_string(k) + " is NULL");
    mpg_world_get_info(worlds[k], &ik);
    if (k == 0) {
      i0 = ik;
    } else if (ik.dof != i0.dof || ik.n_pairs != i0.n_pairs || ik.mask_words != i0.mask_words ||
               ik.n_links != i0.n_links || ik.snapshot_bytes != i0.snapshot_bytes ||
               worlds[k]->snapshot_hash != worlds[0]->snapshot_hash) {
      return set_error(MPG_E_INVALID, "world " + std::to_string(k) + " was not built from world 0's descriptor");
    }
    for (int j = 0; j < k; ++j)
      if (worlds[j] == worlds[k]) return set_error(MPG_E_INVALID, "a world is listed twice");
  }
  std::vector<int> rc(n_worlds, MPG_OK);
  std::vector<std::string> err(n_worlds);
  auto run = [&](int k) {
    int64_t start = 0, count = 0;
    mpg_shard_range(n, k, n_worlds, &start, &count);
    if (count == 0) return;
    rc[k] = mpg_collide_batch(worlds[k], q + (size_t)start * i0.dof, count, flags + start,
                              pair_mask ? pair_mask + (size_t)start * i0.mask_words : nullptr, MPG_MEM_HOST, nullptr);
    if (rc[k]) err[k] = g_last_error;  // the worker thread's error text
  };
  std::vector<std::thread> th;
  for (int k = 1; k < n_worlds; ++k) th.emplace_back(run, k);
  run(0);
  for (auto& t : th) t.join();
  for (int k = 0; k < n_worlds; ++k)
    if (rc[k]) return set_error(rc[k], "world " + std::to_string(k) + ": " + err[k]);
  return MPG_OK;
}

int mpg_shard_range(int64_t n, int32_t k, int32_t n_parts, int64_t* start, int64_t* count) {
  if (n < 0 || n_parts <= 0 || k < 0 || k >= n_parts || !start || !count)
    return set_error(MPG_E_INVALID, "mpg_shard_range: bad arguments");
  // contiguous shards, the first n % n_parts one row longer (mplib_amd.dist.shard_range)
  const int64_t base = n / n_parts, rem = n % n_parts;
  *start = k * base + std::min<int64_t>(k, rem);
  *count = base + (k < rem ? 1 : 0);
  return MPG_OK;
}

int mpg_collide_batch_multi_device(mpg_world* const* worlds, int32_t n_worlds, const double* const* q,
                                   const int64_t* counts, uint8_t* const* flags, uint32_t* const* pair_mask,
                                   void* const* streams, uint8_t* gather_flags, uint32_t* gather_masks) {
  if (n_worlds <= 0 || !worlds) return set_error(MPG_E_INVALID, "no worlds");
  if (!counts || !q || !flags) return set_error(MPG_E_INVALID, "counts / q / flags array is NULL");
  if (gather_masks && !pair_mask) return set_error(MPG_E_INVALID, "gather_masks needs pair_mask");
  for (int k = 0; k < n_worlds; ++k) {
    if (!worlds[k]) return set_error(MPG_E_INVALID, "world " + std::to_string(k) + " is NULL");
    if (counts[k] < 0) return set_error(MPG_E_INVALID, "counts[" + std::to_string(k) + "] < 0");
    for (int j = 0; j < k; ++j)
      if (worlds[j] == worlds[k]) return set_error(MPG_E_INVALID, "a world is listed twice");
  }
  const mpg_world* w0 = worlds[0];
  for (int k = 0; k < n_worlds; ++k) {
    const mpg_world* wk = worlds[k];
    if (wk->dw.dof != w0->dw.dof || wk->dw.n_pairs != w0->dw.n_pairs || wk->dw.W != w0->dw.W ||
        wk->blob_bytes != w0->blob_bytes || wk->snapshot_hash != w0->snapshot_hash)
      return set_error(MPG_E_INVALID, "world " + std::to_string(k) + " was not built from world 0's descriptor");
    if (counts[k] > 0 && ((!q[k] && wk->dw.dof > 0) || !flags[k]))
      return set_error(MPG_E_INVALID, "shard " + std::to_string(k) + ": q / flags is NULL");
    if (counts[k] > 0 && gather_masks && !pair_mask[k])
      return set_error(MPG_E_INVALID, "shard " + std::to_string(k) + ": gather_masks needs its pair_mask");
  }
  const int W = w0->dw.W;
  std::vector<int64_t> off(n_worlds + 1, 0);
  for (int k = 0; k < n_worlds; ++k) off[k + 1] = off[k] + counts[k];
  const bool gather = gather_flags || gather_masks;
  if (gather) {  // direct peer copies over xGMI from every other device into device 0
    HIP_TRY(hipSetDevice(w0->device));
    for (int k = 1; k < n_worlds; ++k) {
      if (worlds[k]->device == w0->device) continue;
      int can = 0;
      HIP_TRY(hipDeviceCanAccessPeer(&can, w0->device, worlds[k]->device));
      if (!can) continue;  // hipMemcpyPeerAsync still works, staged by the runtime
      const hipError_t e = hipDeviceEnablePeerAccess(worlds[k]->device, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
        return set_error(MPG_E_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
      (void)hipGetLastError();
    }
  }
  std::vector<int> rc(n_worlds, MPG_OK);
  std::vector<std::string> err(n_worlds);
  auto run = [&](int k) {
    mpg_world* w = worlds[k];
    hipStream_t s = streams ? static_cast<hipStream_t>(streams[k]) : nullptr;
    uint32_t* mk = pair_mask ? pair_mask[k] : nullptr;
    auto fail = [&](int code, const std::string& m) {
      rc[k] = code;
      err[k] = m;
    };
    if (hipSetDevice(w->device) != hipSuccess) return fail(MPG_E_HIP, "hipSetDevice failed");
    if (counts[k] > 0) {
      const int r = mpg_collide_batch(w, q[k], counts[k], flags[k], mk, MPG_MEM_DEVICE, s);
      if (r) return fail(r, g_last_error);
    }
    if (!gather) return;
    hipError_t e = hipSuccess;
    if (counts[k] > 0 && gather_flags)
      e = hipMemcpyPeerAsync(gather_flags + off[k], w0->device, flags[k], w->device, (size_t)counts[k], s);
    if (e == hipSuccess && counts[k] > 0 && gather_masks)
      e = hipMemcpyPeerAsync(gather_masks + off[k] * W, w0->device, mk, w->device,
                             sizeof(uint32_t) * (size_t)counts[k] * W, s);
    if (e == hipSuccess && k > 0) {
      if (!w->gather_ev) e = hipEventCreateWithFlags(&w->gather_ev, hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventRecord(w->gather_ev, s);
    }
    if (e != hipSuccess) return fail(MPG_E_HIP, std::string("gather: ") + hipGetErrorString(e));
  };
  std::vector<std::thread> th;
  for (int k = 1; k < n_worlds; ++k) th.emplace_back(run, k);
  run(0);
  for (auto& t : th) t.join();
  for (int k = 0; k < n_worlds; ++k)
    if (rc[k]) return set_error(rc[k], "world " + std::to_string(k) + ": " + err[k]);
  if (gather) {  // streams[0] orders after every shard's copies
    HIP_TRY(hipSetDevice(w0->device));
    hipStream_t s0 = streams ? static_cast<hipStream_t>(streams[0]) : nullptr;
    for (int k = 1; k < n_worlds; ++k) HIP_TRY(hipStreamWaitEvent(s0, worlds[k]->gather_ev, 0));
  }
  return MPG_OK;
}

int mpg_collide_link_poses(mpg_world* w, const double* link_pose, int64_t n, uint8_t* flags, uint32_t* pair_mask,
                           int mem, void* stream) {
  return collide_common<true>(w, link_pose, n, flags, pair_mask, mem, stream);
}

int mpg_check_motion_batch(mpg_world* w, const double* q_from, const double* q_to, int64_t n, uint32_t so2_mask,
                           double longest_valid_segment, uint8_t* valid, int32_t* first_invalid, int32_t* segments,
                           int mem, void* stream) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  if (n < 0) return set_error(MPG_E_INVALID, "n < 0");
  if (n > 0 && (!q_from || !q_to || !valid)) return set_error(MPG_E_INVALID, "from/to/valid is NULL");
  if (!(longest_valid_segment > 0.0)) return set_error(MPG_E_INVALID, "longest_valid_segment must be > 0");
  if (mem != MPG_MEM_HOST && mem != MPG_MEM_DEVICE) return set_error(MPG_E_INVALID, "bad mem kind");
  if (w->dw.dof > 32) return set_error(MPG_E_UNSUPPORTED, "motion validation supports dof <= 32");
  if (n == 0) return MPG_OK;
  HIP_TRY(hipSetDevice(w->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lk(w->motion_mu);
  const int dof = w->dw.dof;
  const size_t eb = sizeof(double) * (size_t)n * dof;
  auto& M = w->motion;
  auto grow = [&](void** p, size_t& cap, size_t want) { return scratch_grow(M.last, p, cap, want); };
  int rc = scratch_begin(M.last, s);
  if (rc) return rc;
  if ((rc = grow((void**)&M.edges, M.edges_cap, 2 * eb))) return rc;
  if ((rc = grow((void**)&M.segs, M.segs_cap, sizeof(int32_t) * n))) return rc;
  if ((rc = grow((void**)&M.offs, M.offs_cap, sizeof(long long) * n))) return rc;
  if ((rc = grow((void**)&M.out, M.out_cap, (sizeof(int32_t) + 1) * n))) return rc;
  const double* from = q_from;
  const double* to = q_to;
  if (mem == MPG_MEM_HOST) {
    HIP_TRY(hipMemcpyAsync(M.edges, q_from, eb, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(M.edges + (size_t)n * dof, q_to, eb, hipMemcpyHostToDevice, s));
    from = M.edges;
    to = M.edges + (size_t)n * dof;
  }
  const unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(motion_count_kernel, dim3(grid), dim3(256), 0, s, from, to, (long long)n, dof, so2_mask,
                     longest_valid_segment, M.segs);
  HIP_TRY(hipGetLastError());
  // the state count decides the allocation: one synchronisation per call
  std::vector<int32_t> segs((size_t)n);
  HIP_TRY(hipMemcpyAsync(segs.data(), M.segs, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  std::vector<long long> offs((size_t)n);
  long long total = 0;
  for (int64_t e = 0; e < n; ++e) {
    offs[e] = total;
    total += segs[e];
  }
  HIP_TRY(hipMemcpyAsync(M.offs, offs.data(), sizeof(long long) * n, hipMemcpyHostToDevice, s));
  if ((rc = grow((void**)&M.states, M.states_cap, sizeof(double) * (size_t)total * dof))) return rc;
  if ((rc = grow((void**)&M.flags, M.flags_cap, (size_t)total))) return rc;
  hipLaunchKernelGGL(motion_states_kernel, dim3(grid), dim3(256), 0, s, from, to, (long long)n, dof, so2_mask, M.segs,
                     M.offs, M.states);
  HIP_TRY(hipGetLastError());
  rc = launch_collide<false>(w, M.states, total, M.flags, nullptr, s);
  if (rc) return rc;
  uint8_t* d_valid = mem == MPG_MEM_DEVICE ? valid : reinterpret_cast<uint8_t*>(M.out + n);
  int32_t* d_first = first_invalid ? (mem == MPG_MEM_DEVICE ? first_invalid : M.out) : nullptr;
  hipLaunchKernelGGL(motion_reduce_kernel, dim3(grid), dim3(256), 0, s, M.flags, (long long)n, M.segs, M.offs, d_valid,
                     d_first);
  HIP_TRY(hipGetLastError());
  if (mem == MPG_MEM_HOST) {
    HIP_TRY(hipMemcpyAsync(valid, d_valid, n, hipMemcpyDeviceToHost, s));
    if (first_invalid) HIP_TRY(hipMemcpyAsync(first_invalid, d_first, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (segments) std::memcpy(segments, segs.data(), sizeof(int32_t) * n);
  } else if (segments) {
    HIP_TRY(hipMemcpyAsync(segments, M.segs, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
  }
  HIP_TRY(hipEventRecord(M.last, s));
  return MPG_OK;
}

int mpg_distance_batch(mpg_world* w, const double* q, int64_t n, int32_t n_self_pairs, double* d_self,
                       int32_t* p_self, double* d_others, int32_t* p_others, int mem, void* stream) {
  return mpg_distance_batch_ex(w, q, n, n_self_pairs, 0, d_self, p_self, nullptr, d_others, p_others, nullptr, mem,
                               stream);
}

int mpg_distance_batch_ex(mpg_world* w, const double* q, int64_t n, int32_t n_self_pairs, int32_t flags,
                          double* d_self, int32_t* p_self, double* pts_self, double* d_others, int32_t* p_others,
                          double* pts_others, int mem, void* stream) {
  mpg_distance_request req;
  req.flags = flags;
  req.distance_tolerance = 1e-6;
  return mpg_distance_batch_req(w, q, n, n_self_pairs, &req, d_self, p_self, pts_self, d_others, p_others, pts_others,
                                mem, stream);
}

int mpg_distance_batch_req(mpg_world* w, const double* q, int64_t n, int32_t n_self_pairs,
                           const mpg_distance_request* req, double* d_self, int32_t* p_self, double* pts_self,
                           double* d_others, int32_t* p_others, double* pts_others, int mem, void* stream) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  if (!req) return set_error(MPG_E_INVALID, "request is NULL");
  if (n < 0) return set_error(MPG_E_INVALID, "n < 0");
  if (n_self_pairs < 0 || n_self_pairs > w->dw.n_pairs) return set_error(MPG_E_INVALID, "bad n_self_pairs");
  if (n > 0 && ((!q && w->dw.dof > 0) || !d_self || !p_self || !d_others || !p_others))
    return set_error(MPG_E_INVALID, "NULL buffer");
  if (mem != MPG_MEM_HOST && mem != MPG_MEM_DEVICE) return set_error(MPG_E_INVALID, "bad mem kind");
  const int32_t flags = req->flags;
  if (flags & ~(MPG_DISTANCE_SIGNED | MPG_DISTANCE_NEAREST_POINTS | MPG_DISTANCE_GJK_INDEP))
    return set_error(MPG_E_INVALID, "bad flags");
  if (!(req->distance_tolerance >= 0.0)) return set_error(MPG_E_INVALID, "bad distance_tolerance");
  if (w->has_octree2)
    return set_error(MPG_E_UNSUPPORTED, "distance for a pair of two OcTrees (OcTreeDistanceRecurse) is not implemented");
  const bool indep = (flags & MPG_DISTANCE_GJK_INDEP) != 0;
  if (indep && (flags & MPG_DISTANCE_SIGNED))
    return set_error(MPG_E_UNSUPPORTED, "signed distance with GST_INDEP (FCL's EPA) is not implemented");
  if (indep && (w->has_mesh || w->has_octree))
    return set_error(MPG_E_UNSUPPORTED, "distance with GST_INDEP for an OcTree or BVH mesh pair is not implemented");
  const ccd_real tol = (ccd_real)req->distance_tolerance;  // GJKSolver_libccd::distance_tolerance -> ccd.dist_tolerance
  const double dtol = req->distance_tolerance;              // GJKSolver_indep::gjk_tolerance (distance-inl.h)
  const bool want_pts = pts_self || pts_others;
  const int mode = (want_pts || (flags & (MPG_DISTANCE_SIGNED | MPG_DISTANCE_NEAREST_POINTS)) ? MPG_DIST_POINTS : 0) |
                   (flags & MPG_DISTANCE_SIGNED ? MPG_DIST_SIGNED : 0) |
                   (flags & MPG_DISTANCE_NEAREST_POINTS ? MPG_DIST_NP : 0) | (indep ? MPG_DIST_INDEP : 0);
  if (n == 0) return MPG_OK;
  HIP_TRY(hipSetDevice(w->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lk(w->dist_mu);
  auto& D = w->dist;
  auto grow = [&](void** p, size_t& cap, size_t want) { return scratch_grow(D.last, p, cap, want); };
  int rc = scratch_begin(D.last, s);
  if (rc) return rc;
  const size_t nm = std::max(w->dw.n_moving, 1), ns = std::max(w->dw.bp.n_saves, 1);
  if ((rc = grow((void**)&D.poses, D.poses_cap, sizeof(double) * kPoseStride * nm * n))) return rc;
  if ((rc = grow((void**)&D.save64, D.save_cap, sizeof(double) * 12 * ns * n))) return rc;
  const double* qin = q;
  double *ds = d_self, *dd = d_others, *qs = pts_self, *qo = pts_others;
  int32_t *ps = p_self, *po = p_others;
  const size_t out_bytes = (2 * sizeof(double) + 2 * sizeof(int32_t) + (mode ? 12 * sizeof(double) : 0)) * n;
  if (mem == MPG_MEM_HOST) {
    if ((rc = grow((void**)&D.q, D.q_cap, sizeof(double) * std::max(w->dw.dof, 1) * n))) return rc;
    if ((rc = grow((void**)&D.out, D.out_cap, out_bytes))) return rc;
    if (w->dw.dof) HIP_TRY(hipMemcpyAsync(D.q, q, sizeof(double) * w->dw.dof * n, hipMemcpyHostToDevice, s));
    qin = D.q;
    ds = reinterpret_cast<double*>(D.out);
    dd = ds + n;
    qs = dd + n;
    qo = qs + (mode ? 6 * n : 0);
    ps = reinterpret_cast<int32_t*>(qo + (mode ? 6 * n : 0));
    po = ps + n;
  } else if (mode && (!qs || !qo)) {  // device buffers: scratch for the points nobody asked for
    if ((rc = grow((void**)&D.pts, D.pts_cap, 12 * sizeof(double) * n))) return rc;
    if (!qs) qs = D.pts;
    if (!qo) qo = D.pts + 6 * n;
  }
  const unsigned grid = (unsigned)((n + 127) / 128);
  hipLaunchKernelGGL((pose_kernel<false>), dim3(grid), dim3(128), 0, s, w->dw, qin, (long long)n, D.poses, D.save64);
  HIP_TRY(hipGetLastError());
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(128), 0, s, w->dw, D.poses, (long long)n, n_self_pairs, tol, dtol, ds,
                       ps, dd, po, qs, qo);
    return hipGetLastError();
  };
  constexpr int P = MPG_DIST_POINTS, SG = MPG_DIST_SIGNED, NPF = MPG_DIST_NP, IN = MPG_DIST_INDEP;
  switch (mode) {
    case 0: HIP_TRY(launch(distance_kernel<0>)); break;
    case P: HIP_TRY(launch(distance_kernel<P>)); break;
    case P | NPF: HIP_TRY(launch(distance_kernel<P | NPF>)); break;
    case P | SG: HIP_TRY(launch(distance_kernel<P | SG>)); break;
    case P | SG | NPF: HIP_TRY(launch(distance_kernel<P | SG | NPF>)); break;
    case IN: HIP_TRY(launch(distance_kernel<IN>)); break;
    case P | IN: HIP_TRY(launch(distance_kernel<P | IN>)); break;
    default: HIP_TRY(launch(distance_kernel<P | NPF | IN>)); break;
  }
  if (mode & SG) {  // EPAs past the private polytope: again with a big one from the pool
    if ((rc = grow((void**)&D.big, D.big_cap, sizeof(ccdx::BigPolytope) * kBigPool))) return rc;
    if ((rc = grow((void**)&D.list, D.list_cap, sizeof(unsigned) * (n + 1)))) return rc;
    HIP_TRY(hipMemsetAsync(D.list, 0, sizeof(unsigned), s));
    hipLaunchKernelGGL(overflow_list_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ps, (long long)n,
                       D.list);
    HIP_TRY(hipGetLastError());
    auto redo = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(1), dim3(kBigPool), 0, s, w->dw, D.poses, (long long)n, n_self_pairs, tol, dtol,
                         ds, ps, dd, po, qs, qo, D.big, D.list);
      return hipGetLastError();
    };
    if (mode & NPF) HIP_TRY(redo(distance_redo_kernel<P | SG | NPF>));
    else HIP_TRY(redo(distance_redo_kernel<P | SG>));
  }
  HIP_TRY(hipEventRecord(D.last, s));
  if (mem == MPG_MEM_HOST) {
    HIP_TRY(hipMemcpyAsync(d_self, ds, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(d_others, dd, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(p_self, ps, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(p_others, po, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s));
    if (mode && pts_self) HIP_TRY(hipMemcpyAsync(pts_self, qs, sizeof(double) * 6 * n, hipMemcpyDeviceToHost, s));
    if (mode && pts_others) HIP_TRY(hipMemcpyAsync(pts_others, qo, sizeof(double) * 6 * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int64_t i = 0; i < n; ++i) {
      if (p_self[i] == MPG_DISTANCE_FCL_THROWS)
        return set_error(MPG_E_FAILED, "configuration " + std::to_string(i) +
                                           ": FCL's libccd EPA throws here (FCL_THROW_FAILED_AT_THIS_CONFIGURATION)");
      if (p_self[i] == MPG_DISTANCE_EPA_CAPACITY)
        return set_error(MPG_E_UNSUPPORTED, "configuration " + std::to_string(i) +
                                                ": EPA polytope beyond the device capacity (" +
                                                std::to_string(ccdx::kBigPtV) + " vertices)");
    }
  }
  return MPG_OK;
}

int mpg_collide_contacts(mpg_world* w, const double* input, int64_t n, int input_kind, uint8_t* flags,
                         uint32_t* pair_mask, double* depth, double* normal, double* pos, int mem, void* stream) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  if (n < 0) return set_error(MPG_E_INVALID, "n < 0");
  if (input_kind != MPG_INPUT_Q && input_kind != MPG_INPUT_LINK_POSES) return set_error(MPG_E_INVALID, "bad input_kind");
  const bool poses = input_kind == MPG_INPUT_LINK_POSES;
  const size_t row = poses ? (size_t)w->dw.n_links * 7 : (size_t)w->dw.dof;
  if (n > 0 && ((!input && row > 0) || !flags || !pair_mask || !depth || !normal || !pos))
    return set_error(MPG_E_INVALID, "NULL buffer");
  if (mem != MPG_MEM_HOST && mem != MPG_MEM_DEVICE) return set_error(MPG_E_INVALID, "bad mem kind");
  if (w->any_gjk)
    return set_error(MPG_E_UNSUPPORTED, "contacts with gjk_solver MPG_GJK_INDEP (FCL's EPA) are not implemented");
  if (w->has_octree2)
    return set_error(MPG_E_UNSUPPORTED, "contacts for a pair of two OcTrees are not implemented");
  if (w->octree_first)  // contact_kernel reports the (shape, octree) order PlanningWorld uses
    return set_error(MPG_E_UNSUPPORTED, "contacts for a pair whose first object is an OcTree are not implemented");
  if (n == 0) return MPG_OK;
  HIP_TRY(hipSetDevice(w->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t P = (size_t)w->dw.n_pairs, W = (size_t)w->dw.W;
  if (mem == MPG_MEM_DEVICE) {
    ContactOut co{depth, normal, pos};
    return poses ? launch_collide<true>(w, input, n, flags, pair_mask, s, &co)
                 : launch_collide<false>(w, input, n, flags, pair_mask, s, &co);
  }
  // host buffers: grow-only device staging kept by the world (one host call
  // at a time: host_mu), no allocation per call
  std::lock_guard<std::mutex> lk(w->host_mu);
  if (!s && w->own_stream) s = w->own_stream;
  auto grow = [&](void** p, size_t& cap, size_t want) -> bool {
    if (cap >= want) return true;
    if (*p) hipFree(*p);
    *p = nullptr;
    cap = 0;
    if (hipMalloc(p, want) != hipSuccess) return false;
    cap = want;
    return true;
  };
  auto& C = w->contact;
  int rc = MPG_OK;
  do {
    if (!grow((void**)&C.in, C.in_cap, sizeof(double) * std::max<size_t>(1, row * n)) ||
        !grow((void**)&C.out, C.out_cap, sizeof(double) * 7 * P * n) || !grow((void**)&C.fl, C.fl_cap, n) ||
        !grow((void**)&C.mk, C.mk_cap, sizeof(uint32_t) * W * n)) {
      rc = set_error(MPG_E_NOMEM, "contact staging buffers");
      break;
    }
    double *d_in = C.in, *d_out = C.out;
    uint8_t* d_fl = C.fl;
    uint32_t* d_mk = C.mk;
    if (row && hipMemcpyAsync(d_in, input, sizeof(double) * row * n, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = set_error(MPG_E_HIP, "copy input");
      break;
    }
    ContactOut co{d_out, d_out + P * n, d_out + 4 * P * n};
    rc = poses ? launch_collide<true>(w, d_in, n, d_fl, d_mk, s, &co) : launch_collide<false>(w, d_in, n, d_fl, d_mk, s, &co);
    if (rc) break;
    if (hipMemcpyAsync(flags, d_fl, n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(pair_mask, d_mk, sizeof(uint32_t) * W * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(depth, co.depth, sizeof(double) * P * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(normal, co.normal, sizeof(double) * 3 * P * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(pos, co.pos, sizeof(double) * 3 * P * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = set_error(MPG_E_HIP, "copy contact results");
  } while (false);
  return rc;
}

int mpg_fk_batch(mpg_world* w, const double* q, int64_t n, double* link_pose, int mem, void* stream) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  if (n < 0) return set_error(MPG_E_INVALID, "n < 0");
  if (n > 0 && (!q || !link_pose)) return set_error(MPG_E_INVALID, "q/link_pose is NULL");
  HIP_TRY(hipSetDevice(w->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t nout = (size_t)n * w->dw.n_links * 7;
  const unsigned grid = (unsigned)((n + 127) / 128);
  if (mem == MPG_MEM_DEVICE) {
    if (n) hipLaunchKernelGGL(fk_kernel, dim3(grid), dim3(128), 0, s, w->dw, q, (long long)n, link_pose);
    HIP_TRY(hipGetLastError());
    return MPG_OK;
  }
  if (mem != MPG_MEM_HOST) return set_error(MPG_E_INVALID, "bad mem kind");
  std::lock_guard<std::mutex> lk(w->host_mu);
  int rc = ensure_staging(w, (size_t)n, std::max<size_t>(nout, 1));
  if (rc) return rc;
  if (n == 0) return MPG_OK;
  HIP_TRY(hipMemcpyAsync(w->d_q, q, sizeof(double) * n * w->dw.dof, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(fk_kernel, dim3(grid), dim3(128), 0, s, w->dw, w->d_q, (long long)n, w->d_out);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(link_pose, w->d_out, sizeof(double) * nout, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return MPG_OK;
}

int mpg_debug_collide_pairs(mpg_world* w, int32_t geom_a, int32_t geom_b, int64_t n, const double* Ta,
                            const double* Tb, uint8_t* hit) {
  if (!w || n < 0 || (n > 0 && (!Ta || !Tb || !hit))) return set_error(MPG_E_INVALID, "bad arguments");
  if (geom_a < 0 || geom_b < 0 || geom_a >= w->n_geoms || geom_b >= w->n_geoms)
    return set_error(MPG_E_INVALID, "geometry index out of range");
  if (n == 0) return MPG_OK;
  const int ta = w->geom_type_h[geom_a], tb = w->geom_type_h[geom_b];
  int cf = CF_NONE;
  if (ta == MPG_GEOM_MESH || tb == MPG_GEOM_MESH) cf = CF_MESH;
  else if (ta == MPG_GEOM_OCTREE || tb == MPG_GEOM_OCTREE) cf = CF_OCTREE;
  else if (ta == MPG_GEOM_BOX && tb == MPG_GEOM_BOX) cf = CF_BOX_BOX;
  else if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_SPHERE) cf = CF_SPHERE_SPHERE;
  else if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_BOX) cf = CF_SPHERE_BOX;
  else if (ta == MPG_GEOM_BOX && tb == MPG_GEOM_SPHERE) cf = CF_BOX_SPHERE;
  else if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_CAPSULE) cf = CF_SPHERE_CAPSULE;
  else if (ta == MPG_GEOM_CAPSULE && tb == MPG_GEOM_SPHERE) cf = CF_CAPSULE_SPHERE;
  else if (ta == MPG_GEOM_SPHERE && tb == MPG_GEOM_CYLINDER) cf = CF_SPHERE_CYLINDER;
  else if (ta == MPG_GEOM_CYLINDER && tb == MPG_GEOM_SPHERE) cf = CF_CYLINDER_SPHERE;
  if ((cf == CF_OCTREE && ta == tb) || (cf == CF_MESH && (ta == MPG_GEOM_OCTREE || tb == MPG_GEOM_OCTREE)))
    return set_error(MPG_E_UNSUPPORTED, "geometry pair not supported");
  HIP_TRY(hipSetDevice(w->device));
  struct Guard {  // every exit path frees the buffers and the private stream
    double *dA = nullptr, *dB = nullptr;
    uint8_t* dh = nullptr;
    hipStream_t s = nullptr;
    ~Guard() {
      if (s) hipStreamSynchronize(s);
      hipFree(dA);
      hipFree(dB);
      hipFree(dh);
      if (s) hipStreamDestroy(s);
    }
  } g;
  HIP_TRY(hipStreamCreateWithFlags(&g.s, hipStreamNonBlocking));
  HIP_TRY(hipMalloc(&g.dA, sizeof(double) * 12 * n));
  HIP_TRY(hipMalloc(&g.dB, sizeof(double) * 12 * n));
  HIP_TRY(hipMalloc(&g.dh, (size_t)n));
  HIP_TRY(hipMemcpyAsync(g.dA, Ta, sizeof(double) * 12 * n, hipMemcpyHostToDevice, g.s));
  HIP_TRY(hipMemcpyAsync(g.dB, Tb, sizeof(double) * 12 * n, hipMemcpyHostToDevice, g.s));
  // (walk_wave_eval finds the octree / mesh argument itself)
  hipLaunchKernelGGL(debug_pairs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, g.s, w->dw, geom_a, geom_b, cf,
                     (long long)n, g.dA, g.dB, g.dh);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(hit, g.dh, (size_t)n, hipMemcpyDeviceToHost, g.s));
  HIP_TRY(hipStreamSynchronize(g.s));
  return MPG_OK;
}

int mpg_sample_uniform(const double* lower, const double* upper, int32_t dof, int64_t n, uint64_t seed,
                       int64_t row_offset, double* q, int device) {
  if (dof < 0 || dof > kSampleMaxDof) return set_error(MPG_E_INVALID, "dof out of range [0, 64]");
  if (n < 0 || row_offset < 0 || (n > 0 && dof > 0 && (!lower || !upper || !q)))
    return set_error(MPG_E_INVALID, "bad arguments");
  if (n == 0 || dof == 0) return MPG_OK;
  SampleRange r{};
  for (int k = 0; k < dof; ++k) {
    if (!(std::isfinite(lower[k]) && std::isfinite(upper[k]) && lower[k] <= upper[k]))
      return set_error(MPG_E_INVALID, "sampling range must be finite with lower <= upper");
    r.lo[k] = lower[k];
    r.hi[k] = upper[k];
  }
  HIP_TRY(hipSetDevice(device));
  double* d = nullptr;
  HIP_TRY(hipMalloc(&d, sizeof(double) * (size_t)n * dof));
  const long long tot = (long long)n * dof;
  hipLaunchKernelGGL(sample_uniform_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, 0, r, (int)dof,
                     (long long)n, seed, (long long)row_offset, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpy(q, d, sizeof(double) * (size_t)tot, hipMemcpyDeviceToHost);
  hipFree(d);
  if (e != hipSuccess) return set_error(MPG_E_HIP, std::string("mpg_sample_uniform: ") + hipGetErrorString(e));
  return MPG_OK;
}

int mpg_collide_count(mpg_world* w, const double* lower, const double* upper, int64_t n, uint64_t seed,
                      int64_t* counts, void* stream) {
  if (!w) return set_error(MPG_E_INVALID, "world is NULL");
  const int dof = w->dw.dof, P = w->dw.n_pairs, W = w->dw.W;
  if (dof > kSampleMaxDof) return set_error(MPG_E_UNSUPPORTED, "mpg_collide_count supports dof <= 64");
  if (n < 0 || (P > 0 && !counts) || (dof > 0 && (!lower || !upper))) return set_error(MPG_E_INVALID, "bad arguments");
  if ((size_t)P * sizeof(uint32_t) > 64 * 1024) return set_error(MPG_E_UNSUPPORTED, "mpg_collide_count supports <= 16384 pairs");
  for (int p = 0; p < P; ++p) counts[p] = 0;
  if (n == 0 || P == 0) return MPG_OK;
  SampleRange r{};
  for (int k = 0; k < dof; ++k) {
    if (!(std::isfinite(lower[k]) && std::isfinite(upper[k]) && lower[k] <= upper[k]))
      return set_error(MPG_E_INVALID, "sampling range must be finite with lower <= upper");
    r.lo[k] = lower[k];
    r.hi[k] = upper[k];
  }
  HIP_TRY(hipSetDevice(w->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const long long chunk = std::min<long long>(n, w->max_chunk);
  struct Bufs {  // freed on every exit path, after the stream drained
    double* q = nullptr;
    uint8_t* fl = nullptr;
    uint32_t* mk = nullptr;
    unsigned long long* cnt = nullptr;
    hipStream_t s = nullptr;
    ~Bufs() {
      hipStreamSynchronize(s);
      hipFree(q);
      hipFree(fl);
      hipFree(mk);
      hipFree(cnt);
    }
  } b;
  b.s = s;
  HIP_TRY(hipMalloc(&b.q, sizeof(double) * (size_t)chunk * std::max(dof, 1)));
  HIP_TRY(hipMalloc(&b.fl, (size_t)chunk));
  HIP_TRY(hipMalloc(&b.mk, sizeof(uint32_t) * (size_t)chunk * W));
  HIP_TRY(hipMalloc(&b.cnt, sizeof(unsigned long long) * P));
  HIP_TRY(hipMemsetAsync(b.cnt, 0, sizeof(unsigned long long) * P, s));
  for (long long off = 0; off < n; off += chunk) {
    const long long m = std::min(chunk, n - off);
    if (dof > 0) {
      const long long tot = m * dof;
      hipLaunchKernelGGL(sample_uniform_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, r, dof, m, seed,
                         off, b.q);
      HIP_TRY(hipGetLastError());
    }
    const int rc = launch_collide_overlapped<false>(w, b.q, m, b.fl, b.mk, s);
    if (rc) return rc;
    const unsigned grid = (unsigned)std::min<long long>(1024, (m + 255) / 256);
    hipLaunchKernelGGL(pair_count_kernel, dim3(grid), dim3(256), sizeof(uint32_t) * P, s, b.mk, m, W, P, b.cnt);
    HIP_TRY(hipGetLastError());
  }
  std::vector<unsigned long long> h(P);
  HIP_TRY(hipMemcpyAsync(h.data(), b.cnt, sizeof(unsigned long long) * P, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (int p = 0; p < P; ++p) counts[p] = (int64_t)h[p];
  return MPG_OK;
}

int mpg_debug_sincos(const double* x, int64_t n, double* s, double* c, int device) {
  if (n < 0 || (n > 0 && (!x || !s || !c))) return set_error(MPG_E_INVALID, "bad arguments");
  if (n == 0) return MPG_OK;
  HIP_TRY(hipSetDevice(device));
  double *dx = nullptr, *ds = nullptr, *dc = nullptr;
  HIP_TRY(hipMalloc(&dx, sizeof(double) * n));
  HIP_TRY(hipMalloc(&ds, sizeof(double) * n));
  HIP_TRY(hipMalloc(&dc, sizeof(double) * n));
  HIP_TRY(hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(sincos_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dx, (long long)n, ds, dc);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(s, ds, sizeof(double) * n, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(c, dc, sizeof(double) * n, hipMemcpyDeviceToHost));
  hipFree(dx);
  hipFree(ds);
  hipFree(dc);
  return MPG_OK;
}

}  // extern "C"
