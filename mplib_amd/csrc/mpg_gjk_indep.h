// mpg_gjk_indep.h -- fcl::collide with CollisionRequest(gjk_solver_type =
// GST_INDEP) on a shape pair without a closed form, device side (included by
// mpg_kernels.hip inside its anonymous namespace, after the support mappings).
//
// GJKSolver_indep::shapeIntersect -> details::GJK::evaluate on a
// MinkowskiDiff, double precision [ext FCL 0.7.0 gjk_solver_indep-inl.h,
// convexity_based_algorithm/gjk-inl.h, minkowski_diff-inl.h,
// math/detail/project-inl.h] -- the same restatement, operation for
// operation, as oracle/fcl_gjk_indep.h (test infrastructure), which lists the
// steps.  One lane runs one pair test; the convex support is
// convex_support_local (FCL 0.7.0's findExtremeVertex walk, fp64), whose
// rare wave-cooperative resolution needs the pair's geometry uniform across
// the wave (one pair per wave in every caller).  The simplex keeps copies of
// its support points instead of FCL's pointers into a four-slot store: the
// evaluation only ever reads their w, and the copies carry the same values.
#pragma once

namespace gjki {

struct Proj {
  double p[4];
  unsigned enc;
  double sqd;
};

__device__ __forceinline__ Proj proj0() { return Proj{{0, 0, 0, 0}, 0u, -1.0}; }
__device__ __forceinline__ double triple(const V3& a, const V3& b, const V3& c) { return vdot(a, vcross(b, c)); }

// Project<S>::projectLineOrigin
__device__ __forceinline__ Proj line(const V3& a, const V3& b) {
  Proj r = proj0();
  const V3 d = vsub(b, a);
  const double l = vdot(d, d);
  if (l > 0) {
    const double t = -vdot(a, d);
    r.p[1] = (t >= l) ? 1.0 : ((t <= 0) ? 0.0 : (t / l));
    r.p[0] = 1 - r.p[1];
    if (t >= l) {
      r.sqd = vdot(b, b);
      r.enc = 2;
    } else if (t <= 0) {
      r.sqd = vdot(a, a);
      r.enc = 1;
    } else {
      const V3 x = vadd(a, vscale(d, r.p[1]));
      r.sqd = vdot(x, x);
      r.enc = 3;
    }
  }
  return r;
}

// Project<S>::projectTriangleOrigin
__device__ Proj triangle(const V3& a, const V3& b, const V3& c) {
  Proj r = proj0();
  const V3 vt[3] = {a, b, c};
  const V3 dl[3] = {vsub(a, b), vsub(b, c), vsub(c, a)};
  const V3 n = vcross(dl[0], dl[1]);
  const double l = vdot(n, n);
  if (l > 0) {
    double mindist = -1;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (vdot(vt[i], vcross(dl[i], n)) > 0) {
        const int j = i == 2 ? 0 : i + 1, k = j == 2 ? 0 : j + 1;
        const Proj rl = line(vt[i], vt[j]);
        if (mindist < 0 || rl.sqd < mindist) {
          mindist = rl.sqd;
          r.enc = ((rl.enc & 1) ? 1u << i : 0u) + ((rl.enc & 2) ? 1u << j : 0u);
          r.p[i] = rl.p[0];
          r.p[j] = rl.p[1];
          r.p[k] = 0;
        }
      }
    }
    if (mindist < 0) {
      const double d = vdot(a, n);
      const double s = std::sqrt(l);
      const V3 p = vscale(n, d / l);
      mindist = vdot(p, p);
      r.enc = 7;
      const V3 c0 = vcross(dl[1], vsub(b, p)), c1 = vcross(dl[2], vsub(c, p));
      r.p[0] = std::sqrt(vdot(c0, c0)) / s;
      r.p[1] = std::sqrt(vdot(c1, c1)) / s;
      r.p[2] = 1 - r.p[0] - r.p[1];
    }
    r.sqd = mindist;
  }
  return r;
}

// Project<S>::projectTetrahedraOrigin
__device__ Proj tetrahedron(const V3& a, const V3& b, const V3& c, const V3& d) {
  Proj r = proj0();
  const V3 vt[3] = {a, b, c};
  const V3 dl[3] = {vsub(a, d), vsub(b, d), vsub(c, d)};
  const double vl = triple(dl[0], dl[1], dl[2]);
  const bool ng = (vl * vdot(a, vcross(vsub(b, c), vsub(a, b)))) <= 0;
  if (ng && std::fabs(vl) > 0) {
    double mindist = -1;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int j = i == 2 ? 0 : i + 1, k = j == 2 ? 0 : j + 1;
      const double s = vl * vdot(d, vcross(dl[i], dl[j]));
      if (s > 0) {
        const Proj rt = triangle(vt[i], vt[j], d);
        if (mindist < 0 || rt.sqd < mindist) {
          mindist = rt.sqd;
          r.enc = ((rt.enc & 1) ? 1u << i : 0u) + ((rt.enc & 2) ? 1u << j : 0u) + ((rt.enc & 4) ? 8u : 0u);
          r.p[i] = rt.p[0];
          r.p[j] = rt.p[1];
          r.p[k] = 0;
          r.p[3] = rt.p[2];
        }
      }
    }
    if (mindist < 0) {
      mindist = 0;
      r.enc = 15;
      r.p[0] = triple(c, b, d) / vl;
      r.p[1] = triple(a, c, d) / vl;
      r.p[2] = triple(b, a, d) / vl;
      r.p[3] = 1 - (r.p[0] + r.p[1] + r.p[2]);
    }
    r.sqd = mindist;
  } else if (!ng) {
    r = triangle(a, b, c);
    r.p[3] = 0;
  }
  return r;
}

// getSupport (gjk-inl.h) in the shape's own frame; d is normalised
__device__ __forceinline__ V3 shape_support(const DevWorld& w, cptr<double> HV, int geom, int type, const V3& d) {
  const cptr<double> prm = w.geom_rec + G_STRIDE * geom + G_PARAM;
  if (type == MPG_GEOM_CONVEX) return convex_support_local(w, HV, geom, d);
  if (type == MPG_GEOM_TRIANGLE) {  // the first of the larger dot products a / b / c
    const cptr<double> G = HV + 12 * (size_t)w.geom_gstart[geom];
    const V3 a = v3(G[0], G[4], G[8]), b = v3(G[1], G[5], G[9]), c = v3(G[2], G[6], G[10]);
    const double dota = vdot(d, a), dotb = vdot(d, b), dotc = vdot(d, c);
    if (dota > dotb) return dotc > dota ? c : a;
    return dotc > dotb ? c : b;
  }
  if (type == MPG_GEOM_BOX)
    return v3((d.x > 0) ? (prm[0] / 2) : (-prm[0] / 2), (d.y > 0) ? (prm[1] / 2) : (-prm[1] / 2),
              (d.z > 0) ? (prm[2] / 2) : (-prm[2] / 2));
  if (type == MPG_GEOM_SPHERE) return vscale(d, prm[0]);
  const double half_h = prm[1] * 0.5;
  if (type == MPG_GEOM_CAPSULE) {
    const V3 v = vscale(d, prm[0]);
    const V3 pos1 = vadd(v3(0, 0, half_h), v), pos2 = vadd(v3(0, 0, -half_h), v);
    return vdot(d, pos1) > vdot(d, pos2) ? pos1 : pos2;
  }
  if (type == MPG_GEOM_CONE) {
    double zdist = d.x * d.x + d.y * d.y;
    double len = zdist + d.z * d.z;
    zdist = std::sqrt(zdist);
    len = std::sqrt(len);
    const double radius = prm[0];
    const double sin_a = radius / std::sqrt(radius * radius + 4 * half_h * half_h);
    if (d.z > len * sin_a) return v3(0, 0, half_h);
    if (zdist > 0) {
      const double rad = radius / zdist;
      return v3(rad * d.x, rad * d.y, -half_h);
    }
    return v3(0, 0, -half_h);
  }
  if (type == MPG_GEOM_ELLIPSOID) {  // v / sqrt(v . d), one division per coefficient (Eigen's quotient)
    const V3 v = v3(prm[0] * prm[0] * d.x, prm[1] * prm[1] * d.y, prm[2] * prm[2] * d.z);
    const double dd = std::sqrt(vdot(v, d));
    return v3(v.x / dd, v.y / dd, v.z / dd);
  }
  // cylinder
  const double zdist = std::sqrt(d.x * d.x + d.y * d.y);
  if (zdist == 0.0) return v3(0, 0, (d.z > 0) ? half_h : -half_h);
  const double k = prm[0] / zdist;
  return v3(k * d.x, k * d.y, (d.z > 0) ? half_h : -half_h);
}

struct Mink {
  int ga, ta, gb, tb;
  double ts1[9];  // toshape1 = R2^T R1
  double r0[9];   // toshape0 = tf1^-1 tf2: R1^T R2,
  V3 t0;          //   R1^T t2 + (-(R1^T t1))
};

__device__ __forceinline__ V3 matv(const double* M, const V3& d) {
  return v3((M[0] * d.x + M[1] * d.y) + M[2] * d.z, (M[3] * d.x + M[4] * d.y) + M[5] * d.z,
            (M[6] * d.x + M[7] * d.y) + M[8] * d.z);
}

// GJK::getSupport: d.normalized() (each coefficient over sqrt(|d|^2))
__device__ __forceinline__ V3 normalized(const V3& d_in) {
  const double n2 = vdot(d_in, d_in);
  if (!(n2 > 0)) return d_in;
  const double s = std::sqrt(n2);
  return v3(d_in.x / s, d_in.y / s, d_in.z / s);
}

// MinkowskiDiff::support0(d) / support1(-d) for a normalised d
__device__ __forceinline__ V3 support0(const DevWorld& w, cptr<double> HV, const Mink& m, const V3& d) {
  return shape_support(w, HV, m.ga, m.ta, d);
}
__device__ __forceinline__ V3 support1_neg(const DevWorld& w, cptr<double> HV, const Mink& m, const V3& d) {
  return vadd(matv(m.r0, shape_support(w, HV, m.gb, m.tb, matv(m.ts1, vscale(d, -1.0)))), m.t0);
}

// support0(d) - toshape0 * getSupport(s2, toshape1 * -d), d normalised
__device__ __forceinline__ V3 support_n(const DevWorld& w, cptr<double> HV, const Mink& m, const V3& d) {
  return vsub(support0(w, HV, m, d), support1_neg(w, HV, m, d));
}

enum : int { kGjkValid = 0, kGjkInside = 1, kGjkFailed = 2 };

// the simplex GJK<S>::evaluate leaves (getSimplex()): directions and weights
struct Simplex {
  int rank;
  V3 d[4];
  double p[4];
};

// GJK<S>::evaluate(shape, guess = (-1, 0, 0)) -> status; with SIMPLEX the
// final simplex (simplices[current]) into *out
template <bool SIMPLEX>
__device__ int evaluate(const DevWorld& w, cptr<double> HV, const Mink& m, double tol, Simplex* out) {
  constexpr unsigned kMaxIter = 128u;  // GJKSolver_indep::gjk_max_iterations
  V3 sw[4];  // the current simplex's support points
  V3 sd[4];  // ... their directions (SIMPLEX)
  double sp[4];  // ... and weights (SIMPLEX)
  int rank = 0;
  unsigned iterations = 0;
  double alpha = 0;
  V3 lastw[4];
  unsigned clastw = 0;
  int status = kGjkValid;
  {
    const V3 d0 = normalized(vscale(v3(-1.0, 0.0, 0.0), -1.0));  // -ray, ray = guess = (-1, 0, 0)
    if constexpr (SIMPLEX) {
      sd[0] = d0;
      sp[0] = 1;
    }
    sw[rank++] = support_n(w, HV, m, d0);
  }
  V3 ray = sw[0];
  lastw[0] = lastw[1] = lastw[2] = lastw[3] = ray;
  for (;;) {
    const double rl = std::sqrt(vdot(ray, ray));
    if (rl < tol) {
      status = kGjkInside;
      break;
    }
    {
      const V3 dn = normalized(vscale(ray, -1.0));
      if constexpr (SIMPLEX) sd[rank] = dn;
      sw[rank++] = support_n(w, HV, m, dn);
    }
    const V3 wv = sw[rank - 1];
    bool found = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const V3 e = vsub(wv, lastw[i]);
      if (vdot(e, e) < tol) found = true;
    }
    if (found) {  // removeVertex
      --rank;
      break;
    }
    clastw = (clastw + 1) & 3;
    lastw[clastw] = wv;
    const double omega = vdot(ray, wv) / rl;
    alpha = alpha > omega ? alpha : omega;
    if ((rl - alpha) - tol * rl <= 0) {
      --rank;
      break;
    }
    Proj pr = proj0();
    if (rank == 2) pr = line(sw[0], sw[1]);
    else if (rank == 3) pr = triangle(sw[0], sw[1], sw[2]);
    else pr = tetrahedron(sw[0], sw[1], sw[2], sw[3]);
    if (!(pr.sqd >= 0)) {
      --rank;
      break;
    }
    V3 nw[4], nd[4];
    double np[4];
    int nr = 0;
    ray = v3(0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < rank && (pr.enc & (1u << i))) {
        if constexpr (SIMPLEX) {
          nd[nr] = sd[i];
          np[nr] = pr.p[i];
        }
        nw[nr++] = sw[i];
        ray = vadd(ray, vscale(sw[i], pr.p[i]));
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sw[i] = nw[i];
      if constexpr (SIMPLEX) {
        sd[i] = nd[i];
        sp[i] = np[i];
      }
    }
    rank = nr;
    const bool in15 = pr.enc == 15;
    if (++iterations >= kMaxIter) {  // Failed (an Inside of this very step included)
      status = kGjkFailed;
      break;
    }
    if (in15) {
      status = kGjkInside;
      break;
    }
  }
  if constexpr (SIMPLEX) {
    out->rank = rank;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out->d[i] = sd[i];
      out->p[i] = sp[i];
    }
  }
  return status;
}

}  // namespace gjki

// MinkowskiDiff of (ga at T1, gb at T2) in shape 1's frame: toshape1 =
// R2^T R1, toshape0 = tf1^-1 tf2
__device__ __forceinline__ gjki::Mink gjk_indep_mink(const DevWorld& w, int ga, const SE3& T1, int gb, const SE3& T2) {
  gjki::Mink m;
  m.ga = ga;
  m.gb = gb;
  m.ta = w.geom_type[ga];
  m.tb = w.geom_type[gb];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      m.ts1[3 * i + j] = (T2.R[i] * T1.R[j] + T2.R[3 + i] * T1.R[3 + j]) + T2.R[6 + i] * T1.R[6 + j];
      m.r0[3 * i + j] = (T1.R[i] * T2.R[j] + T1.R[3 + i] * T2.R[3 + j]) + T1.R[6 + i] * T2.R[6 + j];
    }
  double t0[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double inv_t = -((T1.R[i] * T1.p[0] + T1.R[3 + i] * T1.p[1]) + T1.R[6 + i] * T1.p[2]);
    t0[i] = ((T1.R[i] * T2.p[0] + T1.R[3 + i] * T2.p[1]) + T1.R[6 + i] * T2.p[2]) + inv_t;
  }
  m.t0 = v3(t0[0], t0[1], t0[2]);
  return m;
}

// GJKSolver_indep::shapeDistance (generic, ShapeDistanceIndepImpl): GJK with
// gjk_tolerance = the request's distance_tolerance; Valid -> w0 = sum p_i
// support0(d_i), w1 = sum p_i support1(-d_i), distance |w0 - w1|, points
// tf1 * w0 and tf1 * w1; otherwise -1 and zero points
// (oracle/fcl_gjk_indep.h gjk_indep_distance)
__device__ double gjk_indep_distance(const DevWorld& w, cptr<double> HV, int ga, const SE3& T1, int gb, const SE3& T2,
                                     double tol, V3& p1, V3& p2) {
  const gjki::Mink m = gjk_indep_mink(w, ga, T1, gb, T2);
  gjki::Simplex s;
  p1 = p2 = v3(0, 0, 0);
  if (gjki::evaluate<true>(w, HV, m, tol, &s) != gjki::kGjkValid) return -1.0;
  V3 w0 = v3(0, 0, 0), w1 = v3(0, 0, 0);
  for (int i = 0; i < s.rank; ++i) {
    w0 = vadd(w0, vscale(gjki::support0(w, HV, m, s.d[i]), s.p[i]));
    w1 = vadd(w1, vscale(gjki::support1_neg(w, HV, m, s.d[i]), s.p[i]));
  }
  const V3 dv = vsub(w0, w1);
  p1 = v3(((T1.R[0] * w0.x + T1.R[1] * w0.y) + T1.R[2] * w0.z) + T1.p[0],
          ((T1.R[3] * w0.x + T1.R[4] * w0.y) + T1.R[5] * w0.z) + T1.p[1],
          ((T1.R[6] * w0.x + T1.R[7] * w0.y) + T1.R[8] * w0.z) + T1.p[2]);
  p2 = v3(((T1.R[0] * w1.x + T1.R[1] * w1.y) + T1.R[2] * w1.z) + T1.p[0],
          ((T1.R[3] * w1.x + T1.R[4] * w1.y) + T1.R[5] * w1.z) + T1.p[1],
          ((T1.R[6] * w1.x + T1.R[7] * w1.y) + T1.R[8] * w1.z) + T1.p[2]);
  return std::sqrt(vdot(dv, dv));
}

// GJKSolver_indep::shapeIntersect (generic): true = collision
__device__ bool gjk_indep_intersect(const DevWorld& w, int ga, const SE3& T1, int gb, const SE3& T2) {
  const gjki::Mink m = gjk_indep_mink(w, ga, T1, gb, T2);
  return gjki::evaluate<false>(w, w.hull, m, w.mpr_tol, nullptr) == gjki::kGjkInside;
}
