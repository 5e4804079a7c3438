// mpg_hullcells.h -- direction-cell candidate lists for the Convex support
// mapping (FCL 0.7.0 Convex::findExtremeVertex as libccd's supportConvex
// calls it, restated in oracle/collide_oracle.c support_convex: argmax of
// dir . vertex in fp64, first maximum wins).
//
// The sphere of directions is cut into 6 cube faces x K x K cells; each cell
// is a polyhedral cone spanned by its 4 corner rays r_k (widened by 1e-6).  A
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
#include <cmath>
#include <cstdint>
#include <algorithm>
#include <vector>
#include "mpg_math.h"

namespace mpg {

constexpr int kCellK = 16;
constexpr int kCellsPerHull = 6 * kCellK * kCellK;
constexpr double kCellMin = 1e-100, kCellMax = 1e100;  // |dir| and max|coord| range with cells

// cell of direction (x, y, z), or -1 (no cell: full scan)
MPG_INLINE int hull_cell(double x, double y, double z) {
  const double ax = std::fabs(x), ay = std::fabs(y), az = std::fabs(z);
  if (!(ax <= kCellMax && ay <= kCellMax && az <= kCellMax)) return -1;  // also NaN
  int f;
  double m, u, v;
  if (ax >= ay && ax >= az) {
    f = 0; m = x; u = y; v = z;
  } else if (ay >= az) {
    f = 1; m = y; u = z; v = x;
  } else {
    f = 2; m = z; u = x; v = y;
  }
  const double am = std::fabs(m);
  if (!(am >= kCellMin)) return -1;
  const double inv = 1.0 / am, h = 0.5 * kCellK;
  int iu = (int)((u * inv + 1.0) * h), iv = (int)((v * inv + 1.0) * h);
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
  if (nv <= 0 || !(X >= kCellMin && X <= kCellMax)) return false;
  const double delta = 1e-6, rel = 1e-9;
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

}  // namespace mpg
