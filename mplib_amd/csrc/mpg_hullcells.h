// mpg_hullcells.h -- direction-cell candidate lists for the Convex support
// mapping (FCL 0.7.0 Convex::findExtremeVertex as libccd's supportConvex
// calls it, restated in oracle/collide_oracle.c support_convex: argmax of
// dir . vertex in fp64, first maximum wins).
//
// The sphere of directions is cut into 6 cube faces x K x K cells; each cell
// is a polyhedral cone spanned by its 4 corner rays r_k (widened by kCellWiden).  A
// vertex w is left out of a cell's list only when one other vertex u beats it
// on every corner ray by a margin: r_k.(u - w) > M_k.  Every direction d of
// the cone is a non-negative combination of the r_k, so then
// d.(u - w) > sum a_k M_k >= 1e-9 |d|_1 max|coord|, far more than the
// rounding of the two fp64 dot products (2 * 3.4e-16 |d|_1 max|coord|): the
// rounded dot of w is strictly below that of u and w can never be the first
// maximum.  The list keeps the survivors in vertex order, so a strict '>'
// scan over it returns exactly the vertex the full scan returns.  Directions
// that are zero, non-finite or of extreme magnitude (where the products could
// under/overflow) and hulls of extreme size have no cell: the caller runs the
// full scan.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <array>
#include <vector>
#include "mpg_math.h"

namespace mpg {

constexpr int kCellK = 16;
constexpr int kCellsPerHull = 6 * kCellK * kCellK;
constexpr double kCellMin = 1e-30, kCellMax = 1e30;  // |dir| range with cells
constexpr double kHullMin = 1e-100, kHullMax = 1e100;  // max|coord| range with cells
constexpr double kCellWiden = 1e-5;  // cone widening: covers the fp32 cell arithmetic below
constexpr int kSubK = 8;  // walk hulls: default subcells per axis of a cell that is not trap-free
constexpr int kSub2K = 16;  // walk hulls: fine cells per axis of a trapped subcell (certified endpoints)
constexpr int kSub3K = 4;   // walk hulls: finer cells per axis of a fine cell without a certified endpoint

// cell of direction (x, y, z), or -1 (no cell: full scan).  The range checks
// are exact (fp64); the cell arithmetic is fp32: the ratios u/|m| are off by
// at most a few 1e-7 (|ratio| <= 1), far inside the kCellWiden widening, so the
// direction always lies in the widened cone of the cell returned.
MPG_INLINE int hull_cell(double x, double y, double z) {
  const double ax = std::fabs(x), ay = std::fabs(y), az = std::fabs(z);
  if (!(ax <= kCellMax && ay <= kCellMax && az <= kCellMax)) return -1;  // also NaN
  if (!(ax >= kCellMin || ay >= kCellMin || az >= kCellMin)) return -1;
  int f;
  double m, u, v;
  if (ax >= ay && ax >= az) {
    f = 0; m = x; u = y; v = z;
  } else if (ay >= az) {
    f = 1; m = y; u = z; v = x;
  } else {
    f = 2; m = z; u = x; v = y;
  }
  const float am = (float)std::fabs(m);
#if defined(__HIP_DEVICE_COMPILE__)
  const float inv = __builtin_amdgcn_rcpf(am);
#else
  const float inv = 1.0f / am;
#endif
  const float h = 0.5f * kCellK;
  int iu = (int)(((float)u * inv + 1.0f) * h), iv = (int)(((float)v * inv + 1.0f) * h);
  iu = iu < 0 ? 0 : (iu >= kCellK ? kCellK - 1 : iu);
  iv = iv < 0 ? 0 : (iv >= kCellK ? kCellK - 1 : iv);
  return ((2 * f + (m < 0.0 ? 1 : 0)) * kCellK + iu) * kCellK + iv;
}

// hull_cell plus the subcell (subk x subk per cell) of the direction, its
// fine cell within the subcell (kSub2K x kSub2K) and its finer cell within the
// fine cell (kSub3K x kSub3K): the same fp32 ratios, so the
// direction lies in the widened subcone and fine cone as well (kCellWiden >>
// the ratio error; the scalings by subk * kSub2K are exact for powers of two).
// -1 / sub, fine undefined when there is no cell.
MPG_INLINE int hull_cell_sub(double x, double y, double z, int subk, int* sub, int* fine, int* fine2) {
  const double ax = std::fabs(x), ay = std::fabs(y), az = std::fabs(z);
  if (!(ax <= kCellMax && ay <= kCellMax && az <= kCellMax)) return -1;  // also NaN
  if (!(ax >= kCellMin || ay >= kCellMin || az >= kCellMin)) return -1;
  int f;
  double m, u, v;
  if (ax >= ay && ax >= az) {
    f = 0; m = x; u = y; v = z;
  } else if (ay >= az) {
    f = 1; m = y; u = z; v = x;
  } else {
    f = 2; m = z; u = x; v = y;
  }
  const float am = (float)std::fabs(m);
#if defined(__HIP_DEVICE_COMPILE__)
  const float inv = __builtin_amdgcn_rcpf(am);
#else
  const float inv = 1.0f / am;
#endif
  const float h = 0.5f * kCellK;
  const float fu = ((float)u * inv + 1.0f) * h, fv = ((float)v * inv + 1.0f) * h;
  int iu = (int)fu, iv = (int)fv;
  iu = iu < 0 ? 0 : (iu >= kCellK ? kCellK - 1 : iu);
  iv = iv < 0 ? 0 : (iv >= kCellK ? kCellK - 1 : iv);
  constexpr int kq = kSub2K * kSub3K;
  const int kf = subk * kq;
  int ku = (int)((fu - (float)iu) * (float)kf), kv = (int)((fv - (float)iv) * (float)kf);
  ku = ku < 0 ? 0 : (ku >= kf ? kf - 1 : ku);
  kv = kv < 0 ? 0 : (kv >= kf ? kf - 1 : kv);
  *sub = (ku / kq) * subk + kv / kq;
  *fine = ((ku % kq) / kSub3K) * kSub2K + (kv % kq) / kSub3K;
  *fine2 = (ku % kSub3K) * kSub3K + kv % kSub3K;
  return ((2 * f + (m < 0.0 ? 1 : 0)) * kCellK + iu) * kCellK + iv;
}

// (host) Appends one hull's cell table: kCellsPerHull + 1 entry offsets (absolute
// indices into pts, which gets x, y, z, 0 per entry).  Returns false (nothing
// appended) when the hull's size is outside the range the margin argument
// covers; such hulls use the full scan.
inline bool build_hull_cells(const double* V, int nv, std::vector<uint32_t>& start, std::vector<double>& pts) {
  double X = 0.0;
  for (int i = 0; i < 3 * nv; ++i) X = std::max(X, std::fabs(V[i]));
  if (nv <= 0 || !(X >= kHullMin && X <= kHullMax)) return false;
  const double delta = kCellWiden, rel = 1e-9;
  std::vector<double> P((size_t)nv * 4);
  std::vector<char> keep(nv);
  for (int f = 0; f < 3; ++f)
    for (int s = 0; s < 2; ++s)
      for (int iu = 0; iu < kCellK; ++iu)
        for (int iv = 0; iv < kCellK; ++iv) {
          double r[4][3], M[4];
          const double u0 = -1.0 + 2.0 * iu / kCellK - delta, u1 = -1.0 + 2.0 * (iu + 1) / kCellK + delta;
          const double v0 = -1.0 + 2.0 * iv / kCellK - delta, v1 = -1.0 + 2.0 * (iv + 1) / kCellK + delta;
          for (int k = 0; k < 4; ++k) {
            r[k][f] = s ? -1.0 : 1.0;
            r[k][(f + 1) % 3] = (k & 1) ? u1 : u0;
            r[k][(f + 2) % 3] = (k & 2) ? v1 : v0;
            M[k] = rel * (std::fabs(r[k][0]) + std::fabs(r[k][1]) + std::fabs(r[k][2])) * X;
          }
          int dom[5] = {0, 0, 0, 0, 0};
          for (int i = 0; i < nv; ++i) {
            const double* p = V + 3 * i;
            double c = 0.0;
            for (int k = 0; k < 4; ++k) {
              P[4 * i + k] = r[k][0] * p[0] + r[k][1] * p[1] + r[k][2] * p[2];
              c += P[4 * i + k];
              if (P[4 * i + k] > P[4 * dom[k] + k]) dom[k] = i;
            }
            double cd = 0.0;
            for (int k = 0; k < 4; ++k) cd += P[4 * dom[4] + k];
            if (c > cd) dom[4] = i;
          }
          auto beats = [&](int u, int i) {
            for (int k = 0; k < 4; ++k)
              if (!(P[4 * u + k] - P[4 * i + k] > M[k])) return false;
            return true;
          };
          for (int i = 0; i < nv; ++i) {
            bool k = true;
            for (int j = 0; j < 5 && k; ++j) k = !beats(dom[j], i);
            for (int u = 0; u < nv && k; ++u) k = !beats(u, i);
            keep[i] = k;
          }
          start.push_back((uint32_t)(pts.size() / 4));
          for (int i = 0; i < nv; ++i)
            if (keep[i]) {
              pts.push_back(V[3 * i]);
              pts.push_back(V[3 * i + 1]);
              pts.push_back(V[3 * i + 2]);
              pts.push_back(0.0);
            }
        }
  start.push_back((uint32_t)(pts.size() / 4));
  return true;
}

// Device layout: one 96-byte record per cell holding the first kCellInline
// list entries inline (a short list is padded with its first entry, whose
// equal dot product can never win the strict '>' again), then the entry count
// and the offset of the remaining entries in an overflow array (x, y, z, 0
// each).  A support is then one batch of loads for most cells.
constexpr int kCellInline = 3;
constexpr int kCellRec = 12;  // doubles per record: 3 x (x, y, z), count, offset, pad
#ifndef MPG_OVF_BATCH
#define MPG_OVF_BATCH 4
#endif
constexpr int kOvfBatch = MPG_OVF_BATCH;  // overflow entries loaded per memory round (device)

// (host) converts build_hull_cells lists [start[0], start[kCellsPerHull]) into
// kCellsPerHull records appended to rec, their overflow entries to ovf
inline void pack_cell_records(const uint32_t* start, const double* pts, std::vector<double>& rec,
                              std::vector<double>& ovf) {
  for (int c = 0; c < kCellsPerHull; ++c) {
    const uint32_t s = start[c], n = start[c + 1] - start[c];
    for (int k = 0; k < kCellInline; ++k) {
      const uint32_t e = s + (k < (int)n ? k : 0);
      for (int j = 0; j < 3; ++j) rec.push_back(pts[4 * e + j]);
    }
    const uint32_t off = (uint32_t)(ovf.size() / 4);
    for (uint32_t e = s + kCellInline; e < s + n; ++e)
      for (int j = 0; j < 4; ++j) ovf.push_back(pts[4 * e + j]);
    rec.push_back((double)n);
    rec.push_back((double)off);
    rec.push_back(0.0);
  }
}

// first maximum of dir . p over a cell record (and its overflow entries), in
// the reference's dot order ((x*px + y*py) + z*pz)
template <class PD>
MPG_INLINE void cell_record_support(PD R, PD ovf, double x, double y, double z, double* out) {
  double best = -DBL_MAX, bx = 0.0, by = 0.0, bz = 0.0;
#pragma unroll
  for (int k = 0; k < kCellInline; ++k) {
    const double px = R[3 * k], py = R[3 * k + 1], pz = R[3 * k + 2];
    const double dd = (x * px + y * py) + z * pz;
    if (dd > best) {
      best = dd;
      bx = px;
      by = py;
      bz = pz;
    }
  }
  const int n = (int)R[9];
  if (n > kCellInline) {
    const PD P0 = ovf + 4 * (size_t)R[10];
    const int m = n - kCellInline;
    for (int k0 = 0; k0 < m; k0 += kOvfBatch) {  // loads of a batch together, compares in list order
      double ex[kOvfBatch], ey[kOvfBatch], ez[kOvfBatch];
#pragma unroll
      for (int j = 0; j < kOvfBatch; ++j) {
        const PD P = P0 + 4 * (k0 + j < m ? k0 + j : m - 1);
        ex[j] = P[0];
        ey[j] = P[1];
        ez[j] = P[2];
      }
#pragma unroll
      for (int j = 0; j < kOvfBatch; ++j) {
        if (k0 + j >= m) break;
        const double dd = (x * ex[j] + y * ey[j]) + z * ez[j];
        if (dd > best) {
          best = dd;
          bx = ex[j];
          by = ey[j];
          bz = ez[j];
        }
      }
    }
  }
  out[0] = bx;
  out[1] = by;
  out[2] = bz;
}

// --------------------------------------------------------------------------
// FCL 0.7.0 neighbour-walk hulls [ext: geometry/shape/convex-inl.h]
// --------------------------------------------------------------------------
// Convex::FindVertexNeighbors + ValidateTopology: faces in FCL's layout
// (count, i0 .. i(count-1), count, ...) -> neighbors_ encoding (entry i < nv:
// offset of vertex i's record [count, neighbours in ascending order], std::set
// order), appended to out.  Returns whether FCL walks this hull:
// find_extreme_via_neighbors_ = (nv > kMinVertCountForEdgeWalking = 32) and
// the topology is valid (every vertex in some face, every edge in exactly two
// faces).  Faces must index [0, nv) (the descriptor validation checks).
constexpr int kMinVertCountForEdgeWalking = 32;
// Device visited mask of the climb (wave_walk, one LDS set per wave): walk
// hulls up to kMaxWalkVerts vertices.  Direction tables (build_walk_cells)
// are built for hulls up to kMaxCellWalkVerts (their host build is
// O(cells * nv^2)); larger walk hulls climb from vertex 0 on every support,
// exact and slower.
constexpr int kMaxWalkVerts = 4096;
constexpr int kMaxCellWalkVerts = 512;
// record slot 9 packs the linear list's length n (n <= nv <= kMaxCellWalkVerts)
// and its overflow offset: n + kCellCountMul * offset
constexpr int kCellCountBits = 12;
constexpr double kCellCountMul = (double)(1 << kCellCountBits);
static_assert(kMaxCellWalkVerts < (1 << kCellCountBits), "walk-cell list length must fit its field");
inline bool fcl_convex_neighbors(int nv, const int32_t* faces, int num_faces, std::vector<int>& out) {
  std::vector<std::vector<int>> nb(nv);
  std::vector<std::pair<int, int>> edges;
  int fi = 0;
  for (int f = 0; f < num_faces; ++f) {
    const int cnt = faces[fi];
    int prev = faces[fi + cnt];
    for (int j = fi + 1; j <= fi + cnt; ++j) {
      const int v = faces[j];
      nb[v].push_back(prev);
      nb[prev].push_back(v);
      edges.push_back({std::min(v, prev), std::max(v, prev)});
      prev = v;
    }
    fi += cnt + 1;
  }
  const size_t base = out.size();
  out.resize(base + nv);
  bool connected = true;
  for (int i = 0; i < nv; ++i) {
    std::sort(nb[i].begin(), nb[i].end());
    nb[i].erase(std::unique(nb[i].begin(), nb[i].end()), nb[i].end());
    connected &= !nb[i].empty();
    out[base + i] = (int)(out.size() - base);
    out.push_back((int)nb[i].size());
    out.insert(out.end(), nb[i].begin(), nb[i].end());
  }
  std::sort(edges.begin(), edges.end());
  bool watertight = true;
  for (size_t k = 0; k < edges.size();) {
    size_t e = k;
    while (e < edges.size() && edges[e] == edges[k]) ++e;
    watertight &= (e - k) == 2;
    k = e;
  }
  return nv > kMinVertCountForEdgeWalking && connected && watertight;
}

// Walk-hull cell records (convex_support_local on the device).  Per cell two
// lists: the linear list of build_hull_cells (every vertex that can be the
// global first maximum for a direction of the cell) and the walk list (every
// vertex the walk can END at for some direction of the (widened) cell cone --
// a vertex w is left out only when one of its neighbours u beats it on every
// corner ray by the margin of build_hull_cells, so u's rounded dot product is
// strictly above w's for every direction of the cell and the walk never stops
// at w -- in vertex order).  The walk list contains the linear list, and in a
// trap-free (sub)cell the walk ends at the unique maximum of the walk list,
// which is then the unique global maximum: the linear list's.  So the record,
// read on every support, carries the short linear list; the walk list lives
// with the rarely read data of trapped cells.
// Record layout (kCellRec doubles, like the linear hulls' records): three
// linear-list entries inline (x, y, z; short lists padded with their first
// entry), then
//   slot 9   n + kCellCountMul * (overflow offset, entries of 4 doubles x, y, z, 0),
//   slot 10  0, or k + 1: the trapped cell's data at aux entry k (kWalkAux
//            doubles each): a header (the index of its first endpoint table
//            in ends: one table of kSub2K x kSub2K fine-cell endpoints, vertex
//            index, or -2 - r: finer table r of ends2 (kSub3K x kSub3K
//            endpoints, or -2 - q: climb prefix record q of pres, kWalkPre ints
//            -- see WalkPrefix), per trapped subcell in subcell order; the walk
//            list's length), then per walk-list entry: vertex index, witness
//            neighbour x, y, z -- the neighbour beating it on most of the cell
//            --, the mask of the walk-list entries that are its neighbours,
//            and its x, y, z,
//   slot 11  the bits (uint64) of the trap-free mask: bit s set when subcell s
//            (kSubK x kSubK per cell, hull_cell_sub order) is trap-free
//            (walk_cell_trap_free on the subcell's own list); all ones for a
//            trap-free cell.
constexpr int kWalkAux = 8;
// Clip the convex polygon (u, v) by a*u + b*v + c <= 0 (Sutherland-Hodgman).
inline void clip_poly(std::vector<std::array<double, 2>>& poly, double a, double b, double c) {
  std::vector<std::array<double, 2>> out;
  const size_t n = poly.size();
  for (size_t i = 0; i < n; ++i) {
    const auto& P = poly[i];
    const auto& Q = poly[(i + 1) % n];
    const double fp = a * P[0] + b * P[1] + c, fq = a * Q[0] + b * Q[1] + c;
    if (fp <= 0) out.push_back(P);
    if ((fp < 0 && fq > 0) || (fp > 0 && fq < 0)) {
      const double t = fp / (fp - fq);
      out.push_back({P[0] + t * (Q[0] - P[0]), P[1] + t * (Q[1] - P[1])});
    }
  }
  poly.swap(out);
}

// A cell is trap-free when for every listed vertex w, on the part R_w of
// the (widened) cell where no neighbour beats w (clipped polygon, each
// neighbour half-space loosened by the rounding margin), w beats every
// non-neighbour by the margin.  Then the walk's endpoint e (which lies in the
// list, on R_e) is >= its neighbours and strictly above every other vertex:
// it is the computed maximum, and when that maximum is unique it is the first
// maximum g of the list -- the walk needs not run.  (A tie at the maximum, only
// possible between neighbours, still takes the exact path.)
inline bool walk_cell_trap_free(const double* V, int nv, const int* nbr, const std::vector<int>& list, int f,
                                double sg, double u0, double u1, double v0, double v1, double X) {
  const double rel = 1e-9, m = rel * 3.0 * X;
  std::vector<char> adj(nv);
  for (int w : list) {
    const int* nb = nbr + nbr[w];
    std::vector<std::array<double, 2>> poly = {{u0, v0}, {u1, v0}, {u1, v1}, {u0, v1}};
    std::fill(adj.begin(), adj.end(), 0);
    for (int k = 1; k <= nb[0] && !poly.empty(); ++k) {
      const int u = nb[k];
      adj[u] = 1;
      const double a[3] = {V[3 * u] - V[3 * w], V[3 * u + 1] - V[3 * w + 1], V[3 * u + 2] - V[3 * w + 2]};
      clip_poly(poly, a[(f + 1) % 3], a[(f + 2) % 3], sg * a[f] - m);  // d . a <= m
    }
    for (int k = 1; k <= nb[0]; ++k) adj[nb[k]] = 1;
    for (const auto& pt : poly) {
      double d[3];
      d[f] = sg;
      d[(f + 1) % 3] = pt[0];
      d[(f + 2) % 3] = pt[1];
      const double dw = d[0] * V[3 * w] + d[1] * V[3 * w + 1] + d[2] * V[3 * w + 2];
      const double M = rel * (std::fabs(d[0]) + std::fabs(d[1]) + std::fabs(d[2])) * X;
      for (int v = 0; v < nv; ++v) {
        if (v == w || adj[v]) continue;
        if (!(d[0] * V[3 * v] + d[1] * V[3 * v + 1] + d[2] * V[3 * v + 2] - dw < -M)) return false;
      }
    }
  }
  return true;
}

// The vertices the walk can end at for some direction of the cone spanned by
// face f (sign sg) over u in [u0, u1], v in [v0, v1] (already widened), in
// vertex order, each with its witness neighbour (see above).
inline void walk_cone_list(const double* V, int nv, const int* nbr, int f, double sg, double u0, double u1, double v0,
                           double v1, double X, std::vector<int>& ids, std::vector<int>& wits) {
  const double rel = 1e-9;
  double r[4][3], M[4];
  for (int k = 0; k < 4; ++k) {
    r[k][f] = sg;
    r[k][(f + 1) % 3] = (k & 1) ? u1 : u0;
    r[k][(f + 2) % 3] = (k & 2) ? v1 : v0;
    M[k] = rel * (std::fabs(r[k][0]) + std::fabs(r[k][1]) + std::fabs(r[k][2])) * X;
  }
  std::vector<double> P((size_t)nv * 4);
  for (int i = 0; i < nv; ++i)
    for (int k = 0; k < 4; ++k) P[4 * i + k] = r[k][0] * V[3 * i] + r[k][1] * V[3 * i + 1] + r[k][2] * V[3 * i + 2];
  ids.clear();
  wits.clear();
  for (int i = 0; i < nv; ++i) {
    const int* nb = nbr + nbr[i];
    int wit = -1;
    double best = -DBL_MAX;
    bool dominated = false;
    for (int k = 1; k <= nb[0]; ++k) {
      double m = DBL_MAX;  // > 0: neighbour k beats i on the whole cone
      for (int c = 0; c < 4; ++c) m = std::min(m, P[4 * nb[k] + c] - P[4 * i + c] - M[c]);
      if (m > 0.0) dominated = true;
      if (m > best) {
        best = m;
        wit = nb[k];
      }
    }
    if (dominated) continue;
    ids.push_back(i);
    wits.push_back(wit < 0 ? i : wit);  // wit < 0: isolated vertex (not a walk hull then)
  }
}

// The walk's endpoint for every direction of the cone spanned by face f (sign
// sg) over [u0, u1] x [v0, v1], or -1.  The climb is replayed once; each of its
// comparisons 'value(u) >= value(b)' (b the running maximum) must come out the
// same on the whole cone: (u - b) . r_k beyond the rounding margin on all four
// corner rays (every direction of the cone is a non-negative combination of
// them, so the rounded fp64 dot products then compare the same way), or u and
// b coincide (equal values, '>=' holds).  Then every direction of the cone
// takes the same path and ends at the same vertex.
// Where the climb's replay stopped when a comparison flips inside the cone:
// the running maximum bi, the pass vertex pv whose neighbour list was being
// scanned, the undecided entry's index k in that list, whether the pass had
// moved before it, and the visited set at that point.  The device resumes the
// climb there (wave_walk) instead of from vertex 0.
constexpr int kWalkPre = 4 + 2 * (kMaxCellWalkVerts / 64);  // ints per record
struct WalkPrefix {
  int bi, pv, k, keep;
  uint64_t vis[kMaxCellWalkVerts / 64];
};

inline int walk_cone_endpoint(const double* V, int nv, const int* nbr, int f, double sg, double u0, double u1,
                              double v0, double v1, double X, std::vector<char>& vis, WalkPrefix* pre = nullptr) {
  const double rel = 1e-9;
  double r[4][3], M[4];
  for (int k = 0; k < 4; ++k) {
    r[k][f] = sg;
    r[k][(f + 1) % 3] = (k & 1) ? u1 : u0;
    r[k][(f + 2) % 3] = (k & 2) ? v1 : v0;
    M[k] = rel * (std::fabs(r[k][0]) + std::fabs(r[k][1]) + std::fabs(r[k][2])) * X;
  }
  vis.assign(nv, 0);
  vis[0] = 1;
  int bi = 0;
  bool keep = true;
  while (keep) {
    keep = false;
    const int pv = bi;
    const int* nb = nbr + nbr[pv];
    for (int k = 1; k <= nb[0]; ++k) {
      const int u = nb[k];
      if (vis[u]) continue;
      const double a[3] = {V[3 * u] - V[3 * bi], V[3 * u + 1] - V[3 * bi + 1], V[3 * u + 2] - V[3 * bi + 2]};
      bool ge = a[0] == 0.0 && a[1] == 0.0 && a[2] == 0.0;
      if (!ge) {
        int above = 0, below = 0;
        for (int c = 0; c < 4; ++c) {
          const double t = r[c][0] * a[0] + r[c][1] * a[1] + r[c][2] * a[2];
          above += t > M[c];
          below += t < -M[c];
        }
        if (above != 4 && below != 4) {  // the comparison flips inside the cone
          if (pre) {
            pre->bi = bi;
            pre->pv = pv;
            pre->k = k - 1;
            pre->keep = keep;
            std::memset(pre->vis, 0, sizeof(pre->vis));
            for (int i = 0; i < nv; ++i)
              if (vis[i]) pre->vis[i >> 6] |= 1ull << (i & 63);
          }
          return -1;
        }
        ge = above == 4;
      }
      vis[u] = 1;
      if (ge) {
        keep = true;
        bi = u;
      }
    }
  }
  return bi;
}

// The vertex that beats every other vertex by the rounding margin on the whole
// cone (then it is the unique computed maximum for every direction of the
// cone), or -1.
inline int cone_single_max(const double* V, int nv, int f, double sg, double u0, double u1, double v0, double v1,
                           double X) {
  const double rel = 1e-9;
  double r[4][3], M[4];
  for (int k = 0; k < 4; ++k) {
    r[k][f] = sg;
    r[k][(f + 1) % 3] = (k & 1) ? u1 : u0;
    r[k][(f + 2) % 3] = (k & 2) ? v1 : v0;
    M[k] = rel * (std::fabs(r[k][0]) + std::fabs(r[k][1]) + std::fabs(r[k][2])) * X;
  }
  const double c[3] = {r[0][0] + r[3][0], r[0][1] + r[3][1], r[0][2] + r[3][2]};
  int u = 0;
  for (int i = 1; i < nv; ++i)
    if (c[0] * V[3 * i] + c[1] * V[3 * i + 1] + c[2] * V[3 * i + 2] >
        c[0] * V[3 * u] + c[1] * V[3 * u + 1] + c[2] * V[3 * u + 2])
      u = i;
  for (int i = 0; i < nv; ++i) {
    if (i == u) continue;
    const double a[3] = {V[3 * u] - V[3 * i], V[3 * u + 1] - V[3 * i + 1], V[3 * u + 2] - V[3 * i + 2]};
    for (int k = 0; k < 4; ++k)
      if (!(r[k][0] * a[0] + r[k][1] * a[1] + r[k][2] * a[2] > M[k])) return -1;
  }
  return u;
}

// Certified walk endpoint of a cone: one climb path for the whole cone
// (walk_cone_endpoint), or a trap-free cone (walk_cell_trap_free on its own
// walk list) whose maximum is one vertex by the margin everywhere -- the walk
// ends at the computed maximum there, whatever path it takes.  -1: neither.
inline int cone_endpoint(const double* V, int nv, const int* nbr, int f, double sg, double u0, double u1, double v0,
                         double v1, double X, std::vector<char>& vis, std::vector<int>& ids, std::vector<int>& wits,
                         WalkPrefix* pre = nullptr) {
  const int e = walk_cone_endpoint(V, nv, nbr, f, sg, u0, u1, v0, v1, X, vis, pre);
  if (e >= 0) return e;
  const int u = cone_single_max(V, nv, f, sg, u0, u1, v0, v1, X);
  if (u < 0) return -1;
  walk_cone_list(V, nv, nbr, f, sg, u0, u1, v0, v1, X, ids, wits);
  return walk_cell_trap_free(V, nv, nbr, ids, f, sg, u0, u1, v0, v1, X) ? u : -1;
}

// Walk-hull cell table: kCellsPerHull records in hull_cell order (layout
// above), overflow entries in ovf, trapped cells' walk lists and verification
// data in aux, certified endpoints of the trapped subcells' fine cells in ends.
inline bool build_walk_cells(const double* V, int nv, const int* nbr, int subk, std::vector<double>& rec,
                             std::vector<double>& ovf, std::vector<double>& aux, std::vector<int>& ends,
                             std::vector<int>& ends2, std::vector<int>& pres) {
  double X = 0.0;
  for (int i = 0; i < 3 * nv; ++i) X = std::max(X, std::fabs(V[i]));
  if (nv <= 0 || nv > kMaxCellWalkVerts || !(X >= kHullMin && X <= kHullMax) || subk < 1 || subk * subk > 64)
    return false;
  std::vector<uint32_t> lstart;
  std::vector<double> lpts;
  if (!build_hull_cells(V, nv, lstart, lpts)) return false;
  const double delta = kCellWiden, cw = 2.0 / kCellK, sw = cw / subk, fw = sw / kSub2K, gw = fw / kSub3K;
  std::vector<int> ids, wits, sids, swits, fids, fwits;
  std::vector<char> vis;
  int c = 0;  // hull_cell order: ((2 f + s) K + iu) K + iv
  for (int f = 0; f < 3; ++f)
    for (int s = 0; s < 2; ++s)
      for (int iu = 0; iu < kCellK; ++iu)
        for (int iv = 0; iv < kCellK; ++iv, ++c) {
          const double sg = s ? -1.0 : 1.0;
          const double u0 = -1.0 + cw * iu - delta, u1 = -1.0 + cw * (iu + 1) + delta;
          const double v0 = -1.0 + cw * iv - delta, v1 = -1.0 + cw * (iv + 1) + delta;
          walk_cone_list(V, nv, nbr, f, sg, u0, u1, v0, v1, X, ids, wits);
          uint64_t free_mask = ~0ull;
          if (!walk_cell_trap_free(V, nv, nbr, ids, f, sg, u0, u1, v0, v1, X)) {
            free_mask = 0;
            for (int su = 0; su < subk; ++su)
              for (int sv = 0; sv < subk; ++sv) {
                const double a0 = -1.0 + cw * iu + sw * su - delta, a1 = -1.0 + cw * iu + sw * (su + 1) + delta;
                const double b0 = -1.0 + cw * iv + sw * sv - delta, b1 = -1.0 + cw * iv + sw * (sv + 1) + delta;
                walk_cone_list(V, nv, nbr, f, sg, a0, a1, b0, b1, X, sids, swits);
                if (walk_cell_trap_free(V, nv, nbr, sids, f, sg, a0, a1, b0, b1, X))
                  free_mask |= 1ull << (su * subk + sv);
              }
          }
          // the linear list inline / in the overflow
          const uint32_t l0 = lstart[c], n = lstart[c + 1] - lstart[c];
          const size_t r0 = rec.size();
          rec.resize(r0 + kCellRec, 0.0);
          for (int k = 0; k < kCellInline; ++k) {
            const uint32_t e = l0 + (k < (int)n ? k : 0);
            for (int j = 0; j < 3; ++j) rec[r0 + 3 * k + j] = lpts[4 * e + j];
          }
          if (n > (uint32_t)kMaxCellWalkVerts) return false;  // cannot happen: n <= nv
          rec[r0 + 9] = (double)n + kCellCountMul * (double)(ovf.size() / 4);
          for (uint32_t e = l0 + kCellInline; e < l0 + n; ++e)
            for (int j = 0; j < 4; ++j) ovf.push_back(lpts[4 * e + j]);
          if (free_mask != ~0ull) {
            rec[r0 + 10] = (double)(aux.size() / kWalkAux) + 1.0;
            const size_t nw = ids.size();
            aux.insert(aux.end(), {(double)(ends.size() / (kSub2K * kSub2K)), (double)nw, 0.0, 0.0, 0.0, 0.0, 0.0,
                                   0.0});
            for (int su = 0; su < subk; ++su)
              for (int sv = 0; sv < subk; ++sv) {
                if ((free_mask >> (su * subk + sv)) & 1ull) continue;
                for (int fu = 0; fu < kSub2K; ++fu)
                  for (int fv = 0; fv < kSub2K; ++fv) {
                    const double a0 = -1.0 + cw * iu + sw * su + fw * fu - delta;
                    const double a1 = -1.0 + cw * iu + sw * su + fw * (fu + 1) + delta;
                    const double b0 = -1.0 + cw * iv + sw * sv + fw * fv - delta;
                    const double b1 = -1.0 + cw * iv + sw * sv + fw * (fv + 1) + delta;
                    int e = cone_endpoint(V, nv, nbr, f, sg, a0, a1, b0, b1, X, vis, fids, fwits);
                    if (e < 0) {  // a climb decision flips inside: its kSub3K x kSub3K finer cells
                      e = -2 - (int)(ends2.size() / (kSub3K * kSub3K));
                      for (int gu = 0; gu < kSub3K; ++gu)
                        for (int gv = 0; gv < kSub3K; ++gv) {
                          const double c0 = -1.0 + cw * iu + sw * su + fw * fu + gw * gu - delta;
                          const double c1 = -1.0 + cw * iu + sw * su + fw * fu + gw * (gu + 1) + delta;
                          const double d0 = -1.0 + cw * iv + sw * sv + fw * fv + gw * gv - delta;
                          const double d1 = -1.0 + cw * iv + sw * sv + fw * fv + gw * (gv + 1) + delta;
                          WalkPrefix pre;
                          int e2 = cone_endpoint(V, nv, nbr, f, sg, c0, c1, d0, d1, X, vis, fids, fwits, &pre);
                          if (e2 < 0) {  // still undecided: where the climb can resume
                            e2 = -2 - (int)(pres.size() / kWalkPre);
                            pres.insert(pres.end(), {pre.bi, pre.pv, pre.k, pre.keep});
                            for (int j = 0; j < kMaxCellWalkVerts / 64; ++j) {
                              pres.push_back((int)(uint32_t)pre.vis[j]);
                              pres.push_back((int)(uint32_t)(pre.vis[j] >> 32));
                            }
                          }
                          ends2.push_back(e2);
                        }
                    }
                    ends.push_back(e);
                  }
              }
            for (size_t e = 0; e < nw; ++e) {
              const int* nb = nbr + nbr[ids[e]];
              uint32_t mask = 0;  // bit k: walk-list entry k (k < 32) is a neighbour
              for (size_t k = 0; k < nw && k < 32; ++k)
                for (int j = 1; j <= nb[0]; ++j)
                  if (nb[j] == ids[k]) mask |= 1u << k;
              aux.push_back((double)ids[e]);
              for (int j = 0; j < 3; ++j) aux.push_back(V[3 * wits[e] + j]);
              aux.push_back((double)mask);
              for (int j = 0; j < 3; ++j) aux.push_back(V[3 * ids[e] + j]);
            }
          }
          std::memcpy(&rec[r0 + 11], &free_mask, 8);
        }
  return true;
}

}  // namespace mpg
