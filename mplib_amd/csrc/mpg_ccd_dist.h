// mpg_ccd_dist.h -- FCL 0.7.0's GJK shape distance on float libccd, device
// side (included by mpg_kernels.hip inside its anonymous namespace).
//
//   GJKSolver_libccd::shapeDistance       -> GJKDistance       -> ccdGJKDist2
//   GJKSolver_libccd::shapeSignedDistance -> GJKSignedDistance -> ccdGJKSignedDist
// [ext FCL 0.7.0 fcl/narrowphase/detail/convexity_based_algorithm/
// gjk_libccd-inl.h, namespace libccd_extension; libccd 2.1 vec3.c,
// polytope.[ch]]: __ccdGJK, doSimplex2/3/4, _ccdDist, extractClosestPoints,
// __ccdEPA (simplexToPolytope3/4, validateNearestFeatureOfPolytopeBeingEdge,
// nextSupport, supportEPADirection, faceNormalPointingOutward,
// computeVisiblePatch, expandPolytope), penEPAPosClosest -- the same
// restatement, operation for operation, as oracle/fcl_gjk_dist.h (whose
// header lists the choices made where the published code leaves the order
// to the platform); the two must agree bit for bit (-ffp-contract=off).
//
// One lane runs one query.  libccd's polytope is a set of doubly linked
// lists (vertices, edges, faces) in insertion order with an incrementally
// tracked nearest element; here it is three fixed arrays in private memory,
// edges and faces threaded on index links (slots of deleted elements are
// reused, list order is the link order, as ccdListAppend / ccdListDel keep
// it).  Capacities: kPtV vertices (one per EPA iteration), kPtE edges, kPtF
// faces (the oracle, unbounded, needs at most 29 vertices on the cfg3 / cfg4
// test batches); a query that needs more sets the polytope's overflow flag
// and its configuration is run again with kBigPtV vertices (a global-memory
// pool); past those the call fails loudly (MPG_DISTANCE_EPA_CAPACITY).
#pragma once

namespace ccdx {

constexpr int kPtV = 96;  // the private polytope's vertices (edges 3x, faces 2x)
constexpr ccd_real kEpaTol = ccd_real(0.0001);  // CCD_INIT epa_tolerance
constexpr unsigned kMaxIter = 1000u;            // GJKSolver_libccd::max_distance_iterations
constexpr int kVertex = 1, kEdge = 2, kFace = 3;

struct Sup {
  CV3 v, v1, v2;
};
struct Simplex {
  Sup ps[4];
  int last;
};

enum Status { kOk = 0, kThrow = 1, kOverflow = 2 };

__device__ __forceinline__ bool iszero(ccd_real v) { return std::fabs(v) < kCcdEps; }
__device__ __forceinline__ bool eq(ccd_real _a, ccd_real _b) {
  const ccd_real ab = std::fabs(_a - _b);
  if (std::fabs(ab) < kCcdEps) return true;
  const ccd_real a = std::fabs(_a), b = std::fabs(_b);
  if (b > a) return ab < kCcdEps * b;
  return ab < kCcdEps * a;
}
__device__ __forceinline__ bool veq(const CV3& a, const CV3& b) { return eq(a.x, b.x) && eq(a.y, b.y) && eq(a.z, b.z); }
__device__ __forceinline__ ccd_real len2(const CV3& a) { return vdot(a, a); }
__device__ __forceinline__ ccd_real dist2(const CV3& a, const CV3& b) { return len2(vsub(a, b)); }
__device__ __forceinline__ ccd_real comp(const CV3& a, int i) { return i == 0 ? a.x : i == 1 ? a.y : a.z; }

// vec3.c __ccdVec3PointSegmentDist2
template <bool WIT>
__device__ ccd_real seg_dist2(const CV3& P, const CV3& x0, const CV3& b, CV3* witness) {
  ccd_real dist, t;
  CV3 d = vsub(b, x0);
  const CV3 a = vsub(x0, P);
  t = -ccd_real(1) * vdot(a, d);
  t /= len2(d);
  if (t < ccd_real(0) || iszero(t)) {
    dist = dist2(x0, P);
    if (WIT) *witness = x0;
  } else if (t > ccd_real(1) || eq(t, ccd_real(1))) {
    dist = dist2(b, P);
    if (WIT) *witness = b;
  } else {
    if (WIT) {
      *witness = vadd(vscale(d, t), x0);
      dist = dist2(*witness, P);
    } else {
      d = vadd(vscale(d, t), a);
      dist = len2(d);
    }
  }
  return dist;
}

// vec3.c ccdVec3PointTriDist2
template <bool WIT>
__device__ ccd_real tri_dist2(const CV3& P, const CV3& x0, const CV3& B, const CV3& C, CV3* witness) {
  CV3 d1 = vsub(B, x0), d2 = vsub(C, x0);
  const CV3 a = vsub(x0, P);
  const ccd_real u = vdot(a, a), v = vdot(d1, d1), w = vdot(d2, d2), p = vdot(a, d1), q = vdot(a, d2), r = vdot(d1, d2);
  const ccd_real d = w * v - r * r;
  ccd_real s, t, dist;
  if (iszero(d)) {
    s = t = -ccd_real(1);
  } else {
    s = (q * r - w * p) / d;
    t = (-s * r - q) / w;
  }
  if ((iszero(s) || s > ccd_real(0)) && (eq(s, ccd_real(1)) || s < ccd_real(1)) && (iszero(t) || t > ccd_real(0)) &&
      (eq(t, ccd_real(1)) || t < ccd_real(1)) && (eq(t + s, ccd_real(1)) || t + s < ccd_real(1))) {
    if (WIT) {
      d1 = vscale(d1, s);
      d2 = vscale(d2, t);
      *witness = vadd(vadd(x0, d1), d2);
      dist = dist2(*witness, P);
    } else {
      dist = s * s * v;
      dist += t * t * w;
      dist += ccd_real(2) * s * t * r;
      dist += ccd_real(2) * s * p;
      dist += ccd_real(2) * t * q;
      dist += u;
    }
  } else {
    CV3 w2;
    dist = seg_dist2<WIT>(P, x0, B, witness);
    ccd_real dd = seg_dist2<true>(P, x0, C, &w2);
    if (dd < dist) {
      dist = dd;
      if (WIT) *witness = w2;
    }
    dd = seg_dist2<true>(P, B, C, &w2);
    if (dd < dist) {
      dist = dd;
      if (WIT) *witness = w2;
    }
  }
  return dist;
}

__device__ __forceinline__ int sx_size(const Simplex& s) { return s.last + 1; }
__device__ __forceinline__ void sx_add(Simplex& s, const Sup& v) { s.ps[++s.last] = v; }
__device__ __forceinline__ void sx_set(Simplex& s, int pos, const Sup& a) { s.ps[pos] = a; }
__device__ __forceinline__ void sx_set_size(Simplex& s, int n) { s.last = n - 1; }

__device__ __forceinline__ CV3 triple_cross(const CV3& a, const CV3& b, const CV3& c) { return vcross(vcross(a, b), c); }
__device__ __forceinline__ int sign(ccd_real v) { return iszero(v) ? 0 : (v < ccd_real(0) ? -1 : 1); }
__device__ __forceinline__ bool abs_lt_eps2(ccd_real v) { return std::fabs(v) < kCcdEps * kCcdEps; }

__device__ __forceinline__ bool coincident(const CV3& p, const CV3& q) {
  for (int i = 0; i < 3; ++i) {
    const ccd_real pi = comp(p, i), qi = comp(q, i);
    ccd_real m = ccd_real(1);
    if (std::fabs(pi) > m) m = std::fabs(pi);
    if (std::fabs(qi) > m) m = std::fabs(qi);
    if (std::fabs(pi - qi) > m * kCcdEps) return false;
  }
  return true;
}
__device__ __forceinline__ bool tri_area_zero(const CV3& a, const CV3& b, const CV3& c) {
  if (coincident(a, b) || coincident(a, c) || coincident(b, c)) return true;
  const CV3 n = vcross(vnormalize(vsub(b, a)), vnormalize(vsub(c, a)));
  return std::fabs(n.x) < kCcdEps && std::fabs(n.y) < kCcdEps && std::fabs(n.z) < kCcdEps;
}

__device__ int do_simplex2(Simplex& s, CV3& dir) {
  const Sup &A = s.ps[s.last], &B = s.ps[0];
  const CV3 AB = vsub(B.v, A.v), AO = vscale(A.v, -ccd_real(1));
  const CV3 n = vcross(AB, AO);
  if (len2(n) <= kCcdEps * kCcdEps * len2(AB) * len2(AO)) return 1;
  dir = vcross(n, AB);
  return 0;
}

__device__ int do_simplex3(Simplex& s, CV3& dir) {
  const Sup A = s.ps[s.last], B = s.ps[1], C = s.ps[0];
  CV3 proj;
  const ccd_real d2 = tri_dist2<true>(CV3{0, 0, 0}, A.v, B.v, C.v, &proj);
  if (abs_lt_eps2(d2)) return 1;
  if (tri_area_zero(A.v, B.v, C.v)) return -1;
  const CV3 AO = vscale(A.v, -ccd_real(1)), AB = vsub(B.v, A.v), AC = vsub(C.v, A.v);
  const CV3 ABC = vcross(AB, AC);
  ccd_real dot = vdot(vcross(ABC, AC), AO);
  bool r45 = false;
  if (iszero(dot) || dot > ccd_real(0)) {
    dot = vdot(AC, AO);
    if (iszero(dot) || dot > ccd_real(0)) {
      sx_set(s, 1, A);
      sx_set_size(s, 2);
      dir = triple_cross(AC, AO, AC);
    } else {
      r45 = true;
    }
  } else {
    dot = vdot(vcross(AB, ABC), AO);
    if (iszero(dot) || dot > ccd_real(0)) {
      r45 = true;
    } else {
      dot = vdot(ABC, AO);
      if (iszero(dot) || dot > ccd_real(0)) {
        dir = ABC;
      } else {
        sx_set(s, 0, B);
        sx_set(s, 1, C);
        dir = vscale(ABC, -ccd_real(1));
      }
    }
  }
  if (r45) {
    dot = vdot(AB, AO);
    if (iszero(dot) || dot > ccd_real(0)) {
      sx_set(s, 0, B);
      sx_set(s, 1, A);
      sx_set_size(s, 2);
      dir = triple_cross(AB, AO, AB);
    } else {
      sx_set(s, 0, A);
      sx_set_size(s, 1);
      dir = AO;
    }
  }
  return 0;
}

__device__ int do_simplex4(Simplex& s, CV3& dir) {
  const Sup A = s.ps[s.last], B = s.ps[2], C = s.ps[1], D = s.ps[0];
  const CV3 O{0, 0, 0};
  if (abs_lt_eps2(tri_dist2<false>(A.v, B.v, C.v, D.v, nullptr))) return -1;
  if (abs_lt_eps2(tri_dist2<false>(O, A.v, B.v, C.v, nullptr))) return 1;
  if (abs_lt_eps2(tri_dist2<false>(O, A.v, C.v, D.v, nullptr))) return 1;
  if (abs_lt_eps2(tri_dist2<false>(O, A.v, B.v, D.v, nullptr))) return 1;
  if (abs_lt_eps2(tri_dist2<false>(O, B.v, C.v, D.v, nullptr))) return 1;
  const CV3 AO = vscale(A.v, -ccd_real(1)), AB = vsub(B.v, A.v), AC = vsub(C.v, A.v), AD = vsub(D.v, A.v);
  const CV3 ABC = vcross(AB, AC), ACD = vcross(AC, AD), ADB = vcross(AD, AB);
  const int B_on_ACD = sign(vdot(ACD, AB)), C_on_ADB = sign(vdot(ADB, AC)), D_on_ABC = sign(vdot(ABC, AD));
  const bool AB_O = sign(vdot(ACD, AO)) == B_on_ACD, AC_O = sign(vdot(ADB, AO)) == C_on_ADB,
             AD_O = sign(vdot(ABC, AO)) == D_on_ABC;
  if (AB_O && AC_O && AD_O) return 1;
  if (!AB_O) {
    sx_set(s, 2, A);
  } else if (!AC_O) {
    sx_set(s, 1, D);
    sx_set(s, 0, B);
    sx_set(s, 2, A);
  } else {
    sx_set(s, 0, C);
    sx_set(s, 1, B);
    sx_set(s, 2, A);
  }
  sx_set_size(s, 3);
  return do_simplex3(s, dir);
}

// __ccdGJK: 0 = intersection, -1 = none (the simplex is left for _ccdDist)
template <class SupF>
__device__ int gjk(SupF& sup, Simplex& s) {
  s.last = -1;
  Sup last = sup(CV3{ccd_real(1), ccd_real(0), ccd_real(0)});  // ccdFirstDirDefault
  sx_add(s, last);
  CV3 dir = vscale(last.v, -ccd_real(1));
  for (unsigned it = 0; it < kMaxIter; ++it) {
    last = sup(dir);
    if (vdot(last.v, dir) < ccd_real(0)) return -1;
    sx_add(s, last);
    const int n = sx_size(s);
    const int r = n == 2 ? do_simplex2(s, dir) : n == 3 ? do_simplex3(s, dir) : do_simplex4(s, dir);
    if (r == 1) return 0;
    if (r == -1) return -1;
    if (iszero(len2(dir))) return -1;
  }
  return -1;
}

__device__ ccd_real reduce_to_triangle(Simplex& s, ccd_real dist, CV3& best_witness) {
  int best = -1;
  for (int i = 0; i < 3; ++i) {
    CV3 wit;
    ccd_real nd = tri_dist2<true>(CV3{0, 0, 0}, s.ps[i == 0 ? 3 : 0].v, s.ps[i == 1 ? 3 : 1].v, s.ps[i == 2 ? 3 : 2].v,
                                  &wit);
    nd = std::sqrt(nd);
    if (nd < dist) {
      dist = nd;
      best = i;
      best_witness = wit;
    }
  }
  if (best >= 0) sx_set(s, best, s.ps[3]);
  sx_set_size(s, 3);
  return dist;
}

__device__ __forceinline__ CV3 lerp(const CV3& a, const CV3& b, ccd_real s) { return vadd(a, vscale(vsub(b, a), s)); }

__device__ void points_from_segment(const Sup& a, const Sup& b, CV3& p1, CV3& p2, const CV3& p) {
  const CV3 AB = vsub(b.v, a.v);
  const ccd_real ax = std::fabs(AB.x), ay = std::fabs(AB.y), az = std::fabs(AB.z);
  const int i = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
  const ccd_real A_i = comp(a.v, i), AB_i = comp(AB, i), p_i = comp(p, i);
  if (std::fabs(AB_i) < kCcdEps) {
    p1 = a.v1;
    p2 = a.v2;
    return;
  }
  const ccd_real s = (p_i - A_i) / AB_i;
  p1 = lerp(a.v1, b.v1, s);
  p2 = lerp(a.v2, b.v2, s);
}

// extractClosestPoints(simplex of 1..3 points, p on it)
__device__ void extract_closest(const Sup* ps, int n, CV3& p1, CV3& p2, const CV3& p) {
  if (n == 1) {
    p1 = ps[0].v1;
    p2 = ps[0].v2;
    return;
  }
  if (n == 2) {
    points_from_segment(ps[0], ps[1], p1, p2, p);
    return;
  }
  if (tri_area_zero(ps[0].v, ps[1].v, ps[2].v)) {
    const ccd_real ab = len2(vsub(ps[1].v, ps[0].v)), ac = len2(vsub(ps[2].v, ps[0].v)), bc = len2(vsub(ps[2].v, ps[1].v));
    int ia, ib;
    if (ab >= ac && ab >= bc) {
      ia = 0;
      ib = 1;
    } else if (ac >= ab && ac >= bc) {
      ia = 0;
      ib = 2;
    } else {
      ia = 1;
      ib = 2;
    }
    points_from_segment(ps[ia], ps[ib], p1, p2, p);
    return;
  }
  const CV3 r_AB = vsub(ps[1].v, ps[0].v), r_AC = vsub(ps[2].v, ps[0].v);
  const CV3 nrm = vcross(r_AB, r_AC);
  const ccd_real nn = len2(nrm);
  const CV3 r_Ap = vsub(p, ps[0].v);
  const ccd_real beta = vdot(nrm, vcross(r_Ap, r_AC)) / nn;
  const ccd_real gamma = vdot(nrm, vcross(r_AB, r_Ap)) / nn;
  p1 = vadd(vadd(ps[0].v1, vscale(vsub(ps[1].v1, ps[0].v1), beta)), vscale(vsub(ps[2].v1, ps[0].v1), gamma));
  p2 = vadd(vadd(ps[0].v2, vscale(vsub(ps[1].v2, ps[0].v2), beta)), vscale(vsub(ps[2].v2, ps[0].v2), gamma));
}

// _ccdDist
template <class SupF>
__device__ ccd_real dist(SupF& sup, ccd_real tol, Simplex& s, CV3& p1, CV3& p2) {
  ccd_real d, last_dist = FLT_MAX;
  CV3 dir{0, 0, 0};
  const CV3 O{0, 0, 0};
  for (unsigned it = 0; it < kMaxIter; ++it) {
    const int n = sx_size(s);
    if (n == 1) {
      dir = s.ps[0].v;
      d = std::sqrt(len2(s.ps[0].v));
    } else if (n == 2) {
      d = std::sqrt(seg_dist2<true>(O, s.ps[0].v, s.ps[1].v, &dir));
    } else if (n == 3) {
      d = std::sqrt(tri_dist2<true>(O, s.ps[0].v, s.ps[1].v, s.ps[2].v, &dir));
    } else {
      d = reduce_to_triangle(s, last_dist, dir);
    }
    if (iszero(d)) return -ccd_real(1);
    if ((last_dist - d) < tol) {
      extract_closest(s.ps, sx_size(s), p1, p2, dir);
      return d;
    }
    const Sup last = sup(vnormalize(vscale(dir, -ccd_real(1))));
    last_dist = d;
    d = std::sqrt(len2(last.v));
    if (std::fabs(last_dist - d) < tol) {
      p1 = last.v1;
      p2 = last.v2;
      return last_dist;
    }
    sx_add(s, last);
  }
  return -ccd_real(1);
}

// ------------------------------------------------------------ polytope
struct PtEdge {
  int16_t v[2], f[2], prev, next;
  ccd_real dist;
  CV3 wit;
  uint8_t mark;
};
struct PtFace {
  int16_t e[3], prev, next;
  ccd_real dist;
  CV3 wit;
  uint8_t mark;
};
// V vertices, 3V edges, 2V faces: the kernels' private polytope is
// Polytope (V = kPtV); a query that outgrows it is run again with a
// BigPolytope in a global-memory pool (distance_redo_kernel)
template <int V>
struct PolytopeT {
  static constexpr int kV = V, kE = 3 * V, kF = 2 * V, kStk = 2 * V;
  Sup vs[kV];
  ccd_real vdist[kV];
  int16_t vnew[kV];
  int nv;
  PtEdge es[kE];
  PtFace fs[kF];
  int ehead, etail, efree, fhead, ftail, ffree;
  int near_type, near_idx;  // near_idx < 0: NULL
  ccd_real near_dist;
  bool overflow;
  int16_t stk_f[kStk];
  uint8_t stk_e[kStk];
  int16_t border[kE];
};
using Polytope = PolytopeT<kPtV>;
constexpr int kBigPtV = 2048;
using BigPolytope = PolytopeT<kBigPtV>;

template <class PT>
__device__ void pt_init(PT& pt) {
  pt.nv = 0;
  pt.ehead = pt.etail = -1;
  pt.fhead = pt.ftail = -1;
  for (int i = 0; i < PT::kE; ++i) pt.es[i].next = (int16_t)(i + 1 < PT::kE ? i + 1 : -1);
  for (int i = 0; i < PT::kF; ++i) pt.fs[i].next = (int16_t)(i + 1 < PT::kF ? i + 1 : -1);
  pt.efree = 0;
  pt.ffree = 0;
  pt.near_type = 3;
  pt.near_idx = -1;
  pt.near_dist = FLT_MAX;
  pt.overflow = false;
}

template <class PT>
__device__ __forceinline__ void near_update(PT& pt, int type, int idx, ccd_real d) {
  if (eq(pt.near_dist, d)) {
    if (type < pt.near_type) {
      pt.near_type = type;
      pt.near_idx = idx;
      pt.near_dist = d;
    }
  } else if (d < pt.near_dist) {
    pt.near_type = type;
    pt.near_idx = idx;
    pt.near_dist = d;
  }
}

template <class PT>
__device__ __forceinline__ ccd_real el_dist(const PT& pt, int type, int idx) {
  return type == kVertex ? pt.vdist[idx] : type == kEdge ? pt.es[idx].dist : pt.fs[idx].dist;
}
template <class PT>
__device__ __forceinline__ CV3 el_wit(const PT& pt, int type, int idx) {
  return type == kVertex ? pt.vs[idx].v : type == kEdge ? pt.es[idx].wit : pt.fs[idx].wit;
}

// ccdPtNearest (renew: vertices, edges, faces, each in list order)
template <class PT>
__device__ void pt_nearest(PT& pt) {
  if (pt.near_idx >= 0) return;
  pt.near_dist = FLT_MAX;
  pt.near_type = 3;
  pt.near_idx = -1;
  for (int i = 0; i < pt.nv; ++i) near_update(pt, kVertex, i, pt.vdist[i]);
  for (int e = pt.ehead; e >= 0; e = pt.es[e].next) near_update(pt, kEdge, e, pt.es[e].dist);
  for (int f = pt.fhead; f >= 0; f = pt.fs[f].next) near_update(pt, kFace, f, pt.fs[f].dist);
}

template <class PT>
__device__ int add_vertex(PT& pt, const Sup& v) {
  if (pt.nv >= PT::kV) {
    pt.overflow = true;
    return -1;
  }
  const int i = pt.nv++;
  pt.vs[i] = v;
  pt.vdist[i] = len2(v.v);
  near_update(pt, kVertex, i, pt.vdist[i]);
  return i;
}

template <class PT>
__device__ int add_edge(PT& pt, int v1, int v2) {
  if (pt.efree < 0 || v1 < 0 || v2 < 0) {
    pt.overflow = true;
    return -1;
  }
  const int e = pt.efree;
  PtEdge& E = pt.es[e];
  pt.efree = E.next;
  E.v[0] = (int16_t)v1;
  E.v[1] = (int16_t)v2;
  E.f[0] = E.f[1] = -1;
  E.mark = 0;
  E.dist = seg_dist2<true>(CV3{0, 0, 0}, pt.vs[v1].v, pt.vs[v2].v, &E.wit);
  E.prev = (int16_t)pt.etail;
  E.next = -1;
  if (pt.etail >= 0) pt.es[pt.etail].next = (int16_t)e;
  else pt.ehead = e;
  pt.etail = e;
  near_update(pt, kEdge, e, E.dist);
  return e;
}

// ccdPtFaceVec3 / getFaceVertices order
template <class PT>
__device__ __forceinline__ void face_vertices(const PT& pt, int f, int out[3]) {
  const PtEdge &e0 = pt.es[pt.fs[f].e[0]], &e1 = pt.es[pt.fs[f].e[1]];
  out[0] = e0.v[0];
  out[1] = e0.v[1];
  out[2] = (e1.v[0] != out[0] && e1.v[0] != out[1]) ? e1.v[0] : e1.v[1];
}

template <class PT>
__device__ int add_face(PT& pt, int e1, int e2, int e3) {
  if (pt.ffree < 0 || e1 < 0 || e2 < 0 || e3 < 0) {
    pt.overflow = true;
    return -1;
  }
  const int f = pt.ffree;
  PtFace& F = pt.fs[f];
  pt.ffree = F.next;
  F.e[0] = (int16_t)e1;
  F.e[1] = (int16_t)e2;
  F.e[2] = (int16_t)e3;
  F.mark = 0;
  int vs[3];
  face_vertices(pt, f, vs);
  F.dist = tri_dist2<true>(CV3{0, 0, 0}, pt.vs[vs[0]].v, pt.vs[vs[1]].v, pt.vs[vs[2]].v, &F.wit);
  for (int i = 0; i < 3; ++i) {
    PtEdge& E = pt.es[F.e[i]];
    if (E.f[0] < 0) E.f[0] = (int16_t)f;
    else E.f[1] = (int16_t)f;
  }
  F.prev = (int16_t)pt.ftail;
  F.next = -1;
  if (pt.ftail >= 0) pt.fs[pt.ftail].next = (int16_t)f;
  else pt.fhead = f;
  pt.ftail = f;
  near_update(pt, kFace, f, F.dist);
  return f;
}

template <class PT>
__device__ void del_face(PT& pt, int f) {
  PtFace& F = pt.fs[f];
  for (int i = 0; i < 3; ++i) {
    PtEdge& E = pt.es[F.e[i]];
    if (E.f[0] == f) E.f[0] = E.f[1];
    E.f[1] = -1;
  }
  if (F.prev >= 0) pt.fs[F.prev].next = F.next;
  else pt.fhead = F.next;
  if (F.next >= 0) pt.fs[F.next].prev = F.prev;
  else pt.ftail = F.prev;
  if (pt.near_type == kFace && pt.near_idx == f) pt.near_idx = -1;
  F.next = (int16_t)pt.ffree;
  pt.ffree = f;
}

template <class PT>
__device__ void del_edge(PT& pt, int e) {
  PtEdge& E = pt.es[e];
  if (E.prev >= 0) pt.es[E.prev].next = E.next;
  else pt.ehead = E.next;
  if (E.next >= 0) pt.es[E.next].prev = E.prev;
  else pt.etail = E.prev;
  if (pt.near_type == kEdge && pt.near_idx == e) pt.near_idx = -1;
  E.next = (int16_t)pt.efree;
  pt.efree = e;
}

// simplexToPolytope3: -1 = touching (nearest = the triangle)
template <class SupF, class PT>
__device__ int to_polytope3(SupF& sup, const Simplex& s, PT& pt) {
  const Sup &a = s.ps[0], &b = s.ps[1], &c = s.ps[2];
  CV3 dir = vcross(vsub(b.v, a.v), vsub(c.v, a.v));
  const Sup d = sup(dir);
  const ccd_real dist = tri_dist2<false>(d.v, a.v, b.v, c.v, nullptr);
  dir = vscale(dir, -ccd_real(1));
  const Sup d2 = sup(dir);
  const ccd_real dist2_ = tri_dist2<false>(d2.v, a.v, b.v, c.v, nullptr);
  if (iszero(dist) || iszero(dist2_)) {
    const int v0 = add_vertex(pt, a), v1 = add_vertex(pt, b), v2 = add_vertex(pt, c);
    const int e0 = add_edge(pt, v0, v1), e1 = add_edge(pt, v1, v2), e2 = add_edge(pt, v2, v0);
    const int f = add_face(pt, e0, e1, e2);
    pt.near_type = kFace;  // *nearest = the face (returned through the polytope)
    pt.near_idx = f;
    return -1;
  }
  int v[5], e[9];
  v[0] = add_vertex(pt, a);
  v[1] = add_vertex(pt, b);
  v[2] = add_vertex(pt, c);
  v[3] = add_vertex(pt, d);
  v[4] = add_vertex(pt, d2);
  e[0] = add_edge(pt, v[0], v[1]);
  e[1] = add_edge(pt, v[1], v[2]);
  e[2] = add_edge(pt, v[2], v[0]);
  e[3] = add_edge(pt, v[3], v[0]);
  e[4] = add_edge(pt, v[3], v[1]);
  e[5] = add_edge(pt, v[3], v[2]);
  e[6] = add_edge(pt, v[4], v[0]);
  e[7] = add_edge(pt, v[4], v[1]);
  e[8] = add_edge(pt, v[4], v[2]);
  add_face(pt, e[3], e[4], e[0]);
  add_face(pt, e[4], e[5], e[1]);
  add_face(pt, e[5], e[3], e[2]);
  add_face(pt, e[6], e[7], e[0]);
  add_face(pt, e[7], e[8], e[1]);
  add_face(pt, e[8], e[6], e[2]);
  return 0;
}

// simplexToPolytope4 (the degeneracy checks rewrite the simplex in place,
// as libccd's aliased a..d pointers see it)
template <class SupF, class PT>
__device__ int to_polytope4(SupF& sup, Simplex& s, PT& pt) {
  bool use3 = false;
  if (iszero(tri_dist2<false>(s.ps[0].v, s.ps[1].v, s.ps[2].v, s.ps[3].v, nullptr))) use3 = true;
  if (iszero(tri_dist2<false>(s.ps[0].v, s.ps[2].v, s.ps[3].v, s.ps[1].v, nullptr))) {
    use3 = true;
    sx_set(s, 1, s.ps[2]);
    sx_set(s, 2, s.ps[3]);
  }
  if (iszero(tri_dist2<false>(s.ps[0].v, s.ps[1].v, s.ps[3].v, s.ps[2].v, nullptr))) {
    use3 = true;
    sx_set(s, 2, s.ps[3]);
  }
  if (iszero(tri_dist2<false>(s.ps[1].v, s.ps[2].v, s.ps[3].v, s.ps[0].v, nullptr))) {
    use3 = true;
    sx_set(s, 0, s.ps[1]);
    sx_set(s, 1, s.ps[2]);
    sx_set(s, 2, s.ps[3]);
  }
  if (use3) {
    sx_set_size(s, 3);
    return to_polytope3(sup, s, pt);
  }
  int v[4], e[6];
  for (int i = 0; i < 4; ++i) v[i] = add_vertex(pt, s.ps[i]);
  e[0] = add_edge(pt, v[0], v[1]);
  e[1] = add_edge(pt, v[1], v[2]);
  e[2] = add_edge(pt, v[2], v[0]);
  e[3] = add_edge(pt, v[3], v[0]);
  e[4] = add_edge(pt, v[3], v[1]);
  e[5] = add_edge(pt, v[3], v[2]);
  add_face(pt, e[0], e[1], e[2]);
  add_face(pt, e[3], e[4], e[0]);
  add_face(pt, e[4], e[5], e[1]);
  add_face(pt, e[5], e[3], e[2]);
  return 0;
}

// the 2-simplex (origin on segment AB): a tetrahedron, or -1 (touching:
// nearest = the segment's edge)
template <class SupF, class PT>
__device__ int segment_to_tetrahedron(SupF& sup, Simplex& s, PT& pt) {
  const Sup A = s.ps[0], B = s.ps[1];
  const CV3 AB = vsub(B.v, A.v);
  int k = 0;
  if (std::fabs(AB.y) < std::fabs(comp(AB, k))) k = 1;
  if (std::fabs(AB.z) < std::fabs(comp(AB, k))) k = 2;
  const CV3 axis{k == 0 ? ccd_real(1) : ccd_real(0), k == 1 ? ccd_real(1) : ccd_real(0), k == 2 ? ccd_real(1) : ccd_real(0)};
  CV3 dir = vcross(AB, axis);
  Sup s0 = sup(dir);
  if (veq(s0.v, A.v) || veq(s0.v, B.v)) {
    dir = vscale(dir, -ccd_real(1));
    s0 = sup(dir);
  }
  bool touching = veq(s0.v, A.v) || veq(s0.v, B.v);
  if (!touching) {
    CV3 n = vcross(AB, vsub(s0.v, A.v));
    const Sup s1 = sup(n);
    n = vscale(n, -ccd_real(1));
    const Sup s2 = sup(n);
    n = vscale(n, -ccd_real(1));
    const ccd_real h1 = vdot(vsub(s1.v, A.v), n), h2 = -vdot(vsub(s2.v, A.v), n);
    if (iszero(h1) && iszero(h2)) {
      touching = true;
    } else {
      s.last = -1;
      sx_add(s, A);
      sx_add(s, B);
      sx_add(s, s0);
      sx_add(s, h1 >= h2 ? s1 : s2);
      return 0;
    }
  }
  const int v0 = add_vertex(pt, A), v1 = add_vertex(pt, B);
  pt.near_type = kEdge;
  pt.near_idx = add_edge(pt, v0, v1);
  return -1;
}

// faceNormalPointingOutward (not normalised)
template <class PT>
__device__ CV3 face_normal_out(const PT& pt, int f) {
  const PtEdge &e0 = pt.es[pt.fs[f].e[0]], &e1 = pt.es[pt.fs[f].e[1]];
  const CV3 E1 = vsub(pt.vs[e0.v[1]].v, pt.vs[e0.v[0]].v), E2 = vsub(pt.vs[e1.v[1]].v, pt.vs[e1.v[0]].v);
  CV3 dir = vcross(E1, E2);
  const ccd_real dir_norm = std::sqrt(len2(dir));
  const CV3 unit_dir = vscale(dir, (ccd_real)(1.0 / (double)dir_norm));
  const ccd_real dist_tol = ccd_real(0.01);
  const CV3 f0 = pt.vs[e0.v[0]].v;
  const ccd_real od = vdot(unit_dir, f0);
  if (od < -dist_tol) {
    dir = vscale(dir, -ccd_real(1));
  } else if (-dist_tol <= od && od <= dist_tol) {
    ccd_real max_d = -FLT_MAX, min_d = FLT_MAX;
    for (int i = 0; i < pt.nv; ++i) {
      const ccd_real d = vdot(unit_dir, vsub(pt.vs[i].v, f0));
      if (d > dist_tol) return vscale(dir, -ccd_real(1));
      if (d < -dist_tol) return dir;
      if (d > max_d) max_d = d;
      if (d < min_d) min_d = d;
    }
    if (max_d > std::fabs(min_d)) dir = vscale(dir, -ccd_real(1));
  }
  return dir;
}

template <class PT>
__device__ __forceinline__ bool outside_face(const PT& pt, int f, const CV3& p) {
  const CV3 n = face_normal_out(pt, f);
  return vdot(n, vsub(p, pt.vs[pt.es[pt.fs[f].e[0]].v[0]].v)) > ccd_real(0);
}

// expandPolytope: computeVisiblePatch (its recursion replayed depth first on
// an explicit stack of (face, next edge); re-visiting a face's entry edge is a
// no-op, the parent being marked visible already), border edges kept in the
// order it meets them; delete the visible faces and the internal edges, add
// the vertex, one edge per silhouette vertex and one face per border edge
template <class PT>
__device__ int expand(PT& pt, int el_type, int el_idx, const Sup& newv) {
  int start;
  if (el_type == kVertex) return kThrow;
  if (el_type == kFace) {
    start = el_idx;
  } else {
    const PtEdge& E = pt.es[el_idx];
    if (outside_face(pt, E.f[0], newv.v)) start = E.f[0];
    else if (outside_face(pt, E.f[1], newv.v)) start = E.f[1];
    else return kThrow;
  }
  int nb = 0, sp = 1;
  pt.fs[start].mark = 1;
  pt.stk_f[0] = (int16_t)start;
  pt.stk_e[0] = 0;
  while (sp > 0) {
    const int f = pt.stk_f[sp - 1], ei = pt.stk_e[sp - 1];
    if (ei == 3) {
      --sp;
      continue;
    }
    pt.stk_e[sp - 1] = (uint8_t)(ei + 1);
    const int edge = pt.fs[f].e[ei];
    PtEdge& E = pt.es[edge];
    const int g = E.f[0] == f ? E.f[1] : E.f[0];
    if (!pt.fs[g].mark) {
      if (outside_face(pt, g, newv.v)) {
        pt.fs[g].mark = 1;
        if (!E.mark) E.mark = 1;
        if (sp >= PT::kStk) {
          pt.overflow = true;
          return kOverflow;
        }
        pt.stk_f[sp] = (int16_t)g;
        pt.stk_e[sp] = 0;
        ++sp;
      } else if (!E.mark) {
        E.mark = 2;
        pt.border[nb++] = (int16_t)edge;
      }
    } else if (!E.mark) {
      E.mark = 1;
    }
  }
  for (int f = pt.fhead; f >= 0;) {
    const int nx = pt.fs[f].next;
    if (pt.fs[f].mark) del_face(pt, f);
    f = nx;
  }
  for (int e = pt.ehead; e >= 0;) {
    const int nx = pt.es[e].next;
    if (pt.es[e].mark == 1) del_edge(pt, e);
    e = nx;
  }
  const int nv = add_vertex(pt, newv);
  if (nv < 0) return kOverflow;
  for (int i = 0; i < pt.nv; ++i) pt.vnew[i] = -1;
  for (int b = 0; b < nb; ++b) {
    const int be = pt.border[b];
    pt.es[be].mark = 0;
    int e[2];
    for (int i = 0; i < 2; ++i) {
      const int vi = pt.es[be].v[i];
      if (pt.vnew[vi] < 0) pt.vnew[vi] = (int16_t)add_edge(pt, nv, vi);
      e[i] = pt.vnew[vi];
    }
    add_face(pt, be, e[0], e[1]);
    if (pt.overflow) return kOverflow;
  }
  return kOk;
}

// supportEPADirection
template <class PT>
__device__ int epa_direction(const PT& pt, int type, int idx, CV3& dir) {
  if (iszero(el_dist(pt, type, idx))) {
    if (type != kFace) return kThrow;
    dir = face_normal_out(pt, idx);
  } else {
    dir = el_wit(pt, type, idx);
  }
  dir = vnormalize(dir);
  return kOk;
}

// nextSupport: 0 = expand, 1 = converged, kThrow (as the status, negated)
template <class SupF, class PT>
__device__ int next_support(const PT& pt, SupF& sup, int type, int idx, Sup& out) {
  if (type == kVertex) return 1;
  CV3 dir;
  if (epa_direction(pt, type, idx, dir)) return -kThrow;
  out = sup(dir);
  const ccd_real d = vdot(out.v, dir);
  if (d - std::sqrt(el_dist(pt, type, idx)) < kEpaTol) return 1;
  ccd_real d2;
  if (type == kEdge) {
    d2 = seg_dist2<false>(out.v, pt.vs[pt.es[idx].v[0]].v, pt.vs[pt.es[idx].v[1]].v, nullptr);
  } else {
    int vs[3];
    face_vertices(pt, idx, vs);
    d2 = tri_dist2<false>(out.v, pt.vs[vs[0]].v, pt.vs[vs[1]].v, pt.vs[vs[2]].v, nullptr);
  }
  if (std::sqrt(d2) < kEpaTol) return 1;
  return 0;
}

// validateNearestFeatureOfPolytopeBeingEdge
template <class PT>
__device__ int validate_edge(PT& pt) {
  const PtEdge& E = pt.es[pt.near_idx];
  const ccd_real kEps = ccd_real(2) * kCcdEps;
  const CV3 v0 = pt.vs[E.v[0]].v;
  const ccd_real v0_dist = std::sqrt(len2(v0));
  const ccd_real thr = kEps * (v0_dist > ccd_real(1) ? v0_dist : ccd_real(1));
  double o2f[2];
  for (int i = 0; i < 2; ++i) {
    const CV3 n = vnormalize(face_normal_out(pt, E.f[i]));
    o2f[i] = (double)(-vdot(n, v0));
    if (o2f[i] > (double)thr) return kThrow;
  }
  const int k = o2f[0] > o2f[1] ? 0 : 1;
  pt.near_type = kFace;
  pt.near_idx = E.f[k];
  pt.near_dist = (ccd_real)(o2f[k] * o2f[k]);
  return kOk;
}

// __ccdEPA; on kOk the nearest element is (pt.near_type, pt.near_idx)
template <class SupF, class PT>
__device__ int epa(SupF& sup, Simplex& s, PT& pt) {
  int ret;
  const int size = sx_size(s);
  if (size == 4) {
    ret = to_polytope4(sup, s, pt);
  } else if (size == 3) {
    ret = to_polytope3(sup, s, pt);
  } else {
    ret = segment_to_tetrahedron(sup, s, pt);
    if (ret == 0) ret = to_polytope4(sup, s, pt);
  }
  if (pt.overflow) return kOverflow;
  if (ret == -1) return kOk;  // touching contact
  for (;;) {
    pt_nearest(pt);
    if (pt.near_type == kEdge && validate_edge(pt)) return kThrow;
    Sup supp;
    const int r = next_support(pt, sup, pt.near_type, pt.near_idx, supp);
    if (r < 0) return kThrow;
    if (r != 0) break;
    // convexity guard (oracle/fcl_gjk_dist.h lx_epa): a nearest face the new
    // support point does not see ends the expansion at that face
    if (pt.near_type == kFace && !outside_face(pt, pt.near_idx, supp.v)) break;
    const int er = expand(pt, pt.near_type, pt.near_idx, supp);
    if (er != kOk) return er;
  }
  return kOk;
}

// penEPAPosClosest
template <class PT>
__device__ void pen_epa_pos_closest(const PT& pt, CV3& p1, CV3& p2) {
  const int type = pt.near_type, idx = pt.near_idx;
  if (type == kVertex) {
    p1 = pt.vs[idx].v1;
    p2 = pt.vs[idx].v2;
    return;
  }
  Sup ps[3];
  int n;
  if (type == kEdge) {
    ps[0] = pt.vs[pt.es[idx].v[0]];
    ps[1] = pt.vs[pt.es[idx].v[1]];
    n = 2;
  } else {
    int vs[3];
    face_vertices(pt, idx, vs);
    for (int i = 0; i < 3; ++i) ps[i] = pt.vs[vs[i]];
    n = 3;
  }
  extract_closest(ps, n, p1, p2, el_wit(pt, type, idx));
}

// GJKDistanceImpl with ccdGJKDist2 (SIGNED = false) or ccdGJKSignedDist:
// points start at zero; status kOk / kThrow / kOverflow.  pt: the caller's
// private polytope (signed queries only).
template <bool SIGNED, class SupF, class PT>
__device__ int gjk_distance(SupF& sup, ccd_real tol, PT* pt, ccd_real& d, CV3& p1, CV3& p2) {
  p1 = CV3{0, 0, 0};
  p2 = CV3{0, 0, 0};
  Simplex s;
  if (gjk(sup, s) == 0) {
    if constexpr (!SIGNED) {
      d = -ccd_real(1);
      return kOk;
    } else {
      pt_init(*pt);
      const int r = epa(sup, s, *pt);
      if (r != kOk) return r;
      if (pt->near_idx >= 0) {
        d = -std::sqrt(el_dist(*pt, pt->near_type, pt->near_idx));
        pen_epa_pos_closest(*pt, p1, p2);
      } else {
        d = -ccd_real(1);
      }
      return kOk;
    }
  }
  d = dist(sup, tol, s, p1, p2);
  return kOk;
}

}  // namespace ccdx
