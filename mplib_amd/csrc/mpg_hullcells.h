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
    for (int k = 0; k < n - kCellInline; ++k) {
      const PD P = P0 + 4 * k;
      const double px = P[0], py = P[1], pz = P[2];
      const double dd = (x * px + y * py) + z * pz;
      if (dd > best) {
        best = dd;
        bx = px;
        by = py;
        bz = pz;
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
constexpr int kMaxWalkVerts = 512;  // device visited mask (convex_walk)
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

// Walk-hull cell records (convex_support_local on the device): per cell the
// vertices the walk can END at for some direction of the (widened) cell cone
// -- a vertex w is left out only when one of its neighbours u beats it on every
// corner ray by the margin of build_hull_cells, so u's rounded dot product is
// strictly above w's for every direction of the cell and the walk never stops
// at w -- in vertex order, each with the neighbour beating it most often
// (its witness).  The first maximum of the list is the global first maximum
// (the list contains every vertex build_hull_cells keeps).
constexpr int kWalkHead = 4;    // n, overflow offset (entries), pad, pad
constexpr int kWalkEnt = 8;     // x, y, z, vertex index, witness x, y, z, pad
constexpr int kWalkInline = 2;  // entries stored in the record itself
constexpr int kWalkRec = kWalkHead + kWalkInline * kWalkEnt;
inline bool build_walk_cells(const double* V, int nv, const int* nbr, std::vector<double>& rec,
                             std::vector<double>& ovf) {
  double X = 0.0;
  for (int i = 0; i < 3 * nv; ++i) X = std::max(X, std::fabs(V[i]));
  if (nv <= 0 || !(X >= kHullMin && X <= kHullMax)) return false;
  const double delta = kCellWiden, rel = 1e-9;
  std::vector<double> P((size_t)nv * 4);
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
          for (int i = 0; i < nv; ++i)
            for (int k = 0; k < 4; ++k) P[4 * i + k] = r[k][0] * V[3 * i] + r[k][1] * V[3 * i + 1] + r[k][2] * V[3 * i + 2];
          auto margin = [&](int u, int i) {  // > 0: u beats i on the whole cell
            double m = DBL_MAX;
            for (int k = 0; k < 4; ++k) m = std::min(m, P[4 * u + k] - P[4 * i + k] - M[k]);
            return m;
          };
          std::vector<std::array<double, 8>> ents;
          for (int i = 0; i < nv; ++i) {
            const int* nb = nbr + nbr[i];
            int wit = -1;
            double best = -DBL_MAX;
            bool dominated = false;
            for (int k = 1; k <= nb[0]; ++k) {
              const double m = margin(nb[k], i);
              if (m > 0.0) dominated = true;
              if (m > best) {
                best = m;
                wit = nb[k];
              }
            }
            if (dominated) continue;
            if (wit < 0) wit = i;  // isolated vertex (not a walk hull then)
            ents.push_back({V[3 * i], V[3 * i + 1], V[3 * i + 2], (double)i, V[3 * wit], V[3 * wit + 1],
                            V[3 * wit + 2], 0.0});
          }
          const size_t r0 = rec.size();
          rec.resize(r0 + kWalkRec, 0.0);
          rec[r0] = (double)ents.size();
          rec[r0 + 1] = (double)(ovf.size() / kWalkEnt);
          for (size_t e = 0; e < ents.size(); ++e) {
            if ((int)e < kWalkInline) {
              for (int j = 0; j < kWalkEnt; ++j) rec[r0 + kWalkHead + kWalkEnt * e + j] = ents[e][j];
            } else {
              ovf.insert(ovf.end(), ents[e].begin(), ents[e].end());
            }
          }
        }
  return true;
}

}  // namespace mpg
