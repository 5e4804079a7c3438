// fcl::CollisionGeometry's local bounding box and mass properties, the
// methods the reference binds on every geometry (python/pybind_fcl.hpp:71-82,
// 128): computeLocalAABB, computeVolume, computeCOM, computeMomentofInertia,
// computeMomentofInertiaRelatedToCOM.  Restated from FCL 0.7.0 [ext, not
// under /root/reference]: the shapes' closed forms (geometry/shape/*-inl.h),
// Convex's and BVHModel's signed-tetrahedron sums about the frame origin
// (convex-inl.h, BVH_model-inl.h), computeBV<AABB>(shape, identity)
// (geometry/shape/utility-inl.h) and OcTree's root box (octree-inl.h).  Host
// only: none of this is on the collision path.
#include <cmath>
#include <limits>

#include "host.hpp"

namespace mpgh {
namespace {

using M3 = std::array<double, 9>;  // row-major

constexpr double kPi = 3.141592653589793238462643383279502884;

M3 diag(double a, double b, double c) { return {a, 0, 0, 0, b, 0, 0, 0, c}; }

Vec3 cross(const Vec3& a, const Vec3& b) {
  return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}
double dot(const Vec3& a, const Vec3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// one signed tetrahedron (v1, v2, v3, origin) of a closed surface
struct TetSum {
  double vol6 = 0.0;  // sum of 6 x signed volumes
  Vec3 com{0, 0, 0};  // sum of (v1 + v2 + v3) * six_vol
  M3 C{};             // sum of A^T C_canonical A six_vol (A rows v1, v2, v3)
  void add(const Vec3& v1, const Vec3& v2, const Vec3& v3) {
    const double d = dot(cross(v1, v2), v3);
    vol6 += d;
    for (int k = 0; k < 3; ++k) com[k] += (v1[k] + v2[k] + v3[k]) * d;
    // C_canonical = 1/120 (J + I): A^T C_c A = (s s^T + sum_i v_i v_i^T) / 120
    const Vec3 s{v1[0] + v2[0] + v3[0], v1[1] + v2[1] + v3[1], v1[2] + v2[2] + v3[2]};
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        C[3 * r + c] += (s[r] * s[c] + v1[r] * v1[c] + v2[r] * v2[c] + v3[r] * v3[c]) / 120.0 * d;
  }
  M3 inertia() const {  // trace(C) I - C
    const double t = C[0] + C[4] + C[8];
    M3 m;
    for (int i = 0; i < 9; ++i) m[i] = -C[i];
    m[0] += t;
    m[4] += t;
    m[8] += t;
    return m;
  }
};

// Convex: a fan of tetrahedra per face around the face's vertex mean
TetSum convex_sum(const Convex& c) {
  TetSum s;
  size_t fi = 0;
  for (int f = 0; f < c.num_faces && fi < c.faces.size(); ++f) {
    const int n = c.faces[fi];
    Vec3 ctr{0, 0, 0};
    for (int j = 1; j <= n; ++j)
      for (int k = 0; k < 3; ++k) ctr[k] += c.vertices[c.faces[fi + j]][k];
    for (int k = 0; k < 3; ++k) ctr[k] = ctr[k] * (1.0 / n);
    for (int j = 1; j <= n; ++j)
      s.add(c.vertices[c.faces[fi + j]], c.vertices[c.faces[fi + (j % n) + 1]], ctr);
    fi += n + 1;
  }
  return s;
}

TetSum mesh_sum(const BVHModel& b) {
  TetSum s;
  for (auto& t : b.triangles) s.add(b.vertices[t[0]], b.vertices[t[1]], b.vertices[t[2]]);
  return s;
}

constexpr int kOctreeDepth = 16;  // octomap's tree depth

}  // namespace

LocalAABB local_aabb(const CollisionGeometry& g) {
  auto sym = [](double x, double y, double z) { return LocalAABB{{-x, -y, -z}, {x, y, z}}; };
  if (auto b = dynamic_cast<const Box*>(&g)) return sym(0.5 * b->side[0], 0.5 * b->side[1], 0.5 * b->side[2]);
  if (auto s = dynamic_cast<const Sphere*>(&g)) return sym(s->radius, s->radius, s->radius);
  if (auto c = dynamic_cast<const Capsule*>(&g)) return sym(c->radius, c->radius, 0.5 * c->lz + c->radius);
  if (auto c = dynamic_cast<const Cylinder*>(&g)) return sym(c->radius, c->radius, 0.5 * c->lz);
  if (auto c = dynamic_cast<const Cone*>(&g)) return sym(c->radius, c->radius, 0.5 * c->lz);
  if (auto e = dynamic_cast<const Ellipsoid*>(&g)) return sym(e->radii[0], e->radii[1], e->radii[2]);
  if (auto o = dynamic_cast<const OcTree*>(&g)) {
    const double d = (double)(1 << kOctreeDepth) * o->resolution / 2;
    return sym(d, d, d);
  }
  if (auto h = dynamic_cast<const PlaneLike*>(&g)) {  // unbounded but along an axis-aligned normal
    const double big = std::numeric_limits<double>::max();
    LocalAABB a{{-big, -big, -big}, {big, big, big}};
    const bool plane = dynamic_cast<const Plane*>(&g) != nullptr;
    for (int k = 0; k < 3; ++k) {
      if (h->n[(k + 1) % 3] != 0.0 || h->n[(k + 2) % 3] != 0.0) continue;
      if (plane) {
        if (h->n[k] != 0.0) a.min[k] = a.max[k] = h->n[k] < 0 ? -h->d : h->d;
      } else if (h->n[k] < 0) {
        a.min[k] = -h->d;
      } else if (h->n[k] > 0) {
        a.max[k] = h->d;
      }
      break;
    }
    return a;
  }
  if (auto t = dynamic_cast<const TriangleP*>(&g)) {  // AABB(a, b, c)
    LocalAABB a;
    for (int k = 0; k < 3; ++k) {
      a.min[k] = std::min(t->a[k], std::min(t->b[k], t->c[k]));
      a.max[k] = std::max(t->a[k], std::max(t->b[k], t->c[k]));
    }
    return a;
  }
  const std::vector<Vec3>* V = nullptr;
  if (auto c = dynamic_cast<const Convex*>(&g)) V = &c->vertices;
  if (auto b = dynamic_cast<const BVHModel*>(&g)) V = &b->vertices;
  const double big = std::numeric_limits<double>::max();
  LocalAABB a{{big, big, big}, {-big, -big, -big}};  // AABB(): empty
  if (V)
    for (auto& v : *V)
      for (int k = 0; k < 3; ++k) {
        a.min[k] = std::min(a.min[k], v[k]);
        a.max[k] = std::max(a.max[k], v[k]);
      }
  return a;
}

void compute_local_aabb(CollisionGeometry& g) {
  const LocalAABB a = local_aabb(g);
  Vec3 c;
  for (int k = 0; k < 3; ++k) c[k] = (a.min[k] + a.max[k]) * 0.5;
  g.aabb_center = c;
  if (auto b = dynamic_cast<const BVHModel*>(&g)) {  // farthest vertex from the centre
    double r2 = 0.0;
    for (auto& v : b->vertices) {
      const Vec3 d{c[0] - v[0], c[1] - v[1], c[2] - v[2]};
      r2 = std::max(r2, dot(d, d));
    }
    g.aabb_radius = std::sqrt(r2);
    return;
  }
  const Vec3 d{a.min[0] - c[0], a.min[1] - c[1], a.min[2] - c[2]};
  g.aabb_radius = std::sqrt(dot(d, d));
}

double compute_volume(const CollisionGeometry& g) {
  if (auto b = dynamic_cast<const Box*>(&g)) return b->side[0] * b->side[1] * b->side[2];
  if (auto s = dynamic_cast<const Sphere*>(&g)) return 4.0 * kPi * s->radius * s->radius * s->radius / 3.0;
  if (auto c = dynamic_cast<const Capsule*>(&g)) return kPi * c->radius * c->radius * (c->lz + c->radius * 4 / 3.0);
  if (auto c = dynamic_cast<const Cylinder*>(&g)) return kPi * c->radius * c->radius * c->lz;
  if (auto c = dynamic_cast<const Cone*>(&g)) return kPi * c->radius * c->radius * c->lz / 3;
  if (auto e = dynamic_cast<const Ellipsoid*>(&g)) return 4.0 * kPi * e->radii[0] * e->radii[1] * e->radii[2] / 3.0;
  if (auto c = dynamic_cast<const Convex*>(&g)) return convex_sum(*c).vol6 / 6;
  if (auto b = dynamic_cast<const BVHModel*>(&g)) return mesh_sum(*b).vol6 / 6;
  return 0.0;  // CollisionGeometry's default (OcTree)
}

Vec3 compute_com(const CollisionGeometry& g) {
  if (auto c = dynamic_cast<const Cone*>(&g)) return {0.0, 0.0, -0.25 * c->lz};
  TetSum s;
  if (auto c = dynamic_cast<const Convex*>(&g))
    s = convex_sum(*c);
  else if (auto b = dynamic_cast<const BVHModel*>(&g))
    s = mesh_sum(*b);
  else
    return {0.0, 0.0, 0.0};
  const double den = s.vol6 * 4;
  return {s.com[0] / den, s.com[1] / den, s.com[2] / den};
}

std::array<double, 9> compute_moment_of_inertia(const CollisionGeometry& g) {
  const double V = compute_volume(g);
  if (auto b = dynamic_cast<const Box*>(&g)) {
    const double a2 = b->side[0] * b->side[0] * V, b2 = b->side[1] * b->side[1] * V, c2 = b->side[2] * b->side[2] * V;
    return diag((b2 + c2) / 12, (a2 + c2) / 12, (a2 + b2) / 12);
  }
  if (auto s = dynamic_cast<const Sphere*>(&g)) {
    const double I = 0.4 * s->radius * s->radius * V;
    return diag(I, I, I);
  }
  if (auto c = dynamic_cast<const Capsule*>(&g)) {
    const double v_cyl = c->radius * c->radius * c->lz * kPi;
    const double v_sph = c->radius * c->radius * c->radius * kPi * 4 / 3.0;
    const double h2 = c->lz * c->lz, r2 = c->radius * c->radius;
    const double ix = v_cyl * (h2 / 12. + r2 / 4.) + v_sph * (0.4 * r2 + h2 * 0.25 + 3. * c->radius * c->lz / 8.);
    const double iz = (0.5 * v_cyl + 0.4 * v_sph) * c->radius * c->radius;
    return diag(ix, ix, iz);
  }
  if (auto c = dynamic_cast<const Cylinder*>(&g)) {
    const double ix = V * (3 * c->radius * c->radius + c->lz * c->lz) / 12, iz = V * c->radius * c->radius / 2;
    return diag(ix, ix, iz);
  }
  if (auto c = dynamic_cast<const Cone*>(&g)) {
    const double ix = V * (0.1 * c->lz * c->lz + 3 * c->radius * c->radius / 20), iz = 0.3 * V * c->radius * c->radius;
    return diag(ix, ix, iz);
  }
  if (auto e = dynamic_cast<const Ellipsoid*>(&g)) {
    const double a2 = e->radii[0] * e->radii[0] * V, b2 = e->radii[1] * e->radii[1] * V,
                 c2 = e->radii[2] * e->radii[2] * V;
    return diag(0.2 * (b2 + c2), 0.2 * (a2 + c2), 0.2 * (a2 + b2));
  }
  if (auto c = dynamic_cast<const Convex*>(&g)) return convex_sum(*c).inertia();
  if (auto b = dynamic_cast<const BVHModel*>(&g)) return mesh_sum(*b).inertia();
  return diag(0, 0, 0);
}

std::array<double, 9> compute_moment_of_inertia_com(const CollisionGeometry& g) {
  M3 C = compute_moment_of_inertia(g);
  const Vec3 m = compute_com(g);
  const double V = compute_volume(g);
  C[0] -= V * (m[1] * m[1] + m[2] * m[2]);
  C[4] -= V * (m[0] * m[0] + m[2] * m[2]);
  C[8] -= V * (m[0] * m[0] + m[1] * m[1]);
  C[1] += V * m[0] * m[1];
  C[2] += V * m[0] * m[2];
  C[3] += V * m[1] * m[0];
  C[5] += V * m[1] * m[2];
  C[6] += V * m[2] * m[0];
  C[7] += V * m[2] * m[1];
  return C;
}

}  // namespace mpgh
