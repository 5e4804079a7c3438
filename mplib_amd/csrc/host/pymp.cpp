// pymp.cpp -- pybind11 module ``mplib_amd.pymp``: the reference's
// ``mplib.pymp`` API surface (python/pybind.cpp:16-27 and the
// python/pybind_*.hpp files it includes) for the components on the
// collision/validity path, plus the batched entry points.  Every evaluation
// goes to the HIP library (include/mpgpu.h); there is no CPU path.
#include <pybind11/numpy.h>
#include <optional>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "host.hpp"
#include "planner.hpp"

namespace py = pybind11;
using namespace mpgh;

namespace {

std::array<double, 4> quat_arg(const std::vector<double>& q) {
  if (q.size() != 4) throw std::invalid_argument("quaternion must have 4 elements (w, x, y, z)");
  return {q[0], q[1], q[2], q[3]};
}
Vec3 vec3_arg(const std::vector<double>& v) {
  if (v.size() != 3) throw std::invalid_argument("expected 3 elements");
  return {v[0], v[1], v[2]};
}
Vec7 vec7_arg(const std::vector<double>& v) {
  if (v.size() != 7) throw std::invalid_argument("pose must have 7 elements (x, y, z, qw, qx, qy, qz)");
  Vec7 o;
  for (int i = 0; i < 7; ++i) o[i] = v[i];
  return o;
}
py::array_t<double> mat3(const SE3& T) {
  py::array_t<double> a({3, 3});
  auto m = a.mutable_unchecked<2>();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) m(i, j) = T.R[3 * i + j];
  return a;
}
py::array_t<double> mat4(const SE3& T) {  // homogeneous matrix of an Isometry3d
  py::array_t<double> a({4, 4});
  auto m = a.mutable_unchecked<2>();
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) m(i, j) = T.R[3 * i + j];
    m(i, 3) = T.p[i];
    m(3, i) = 0.0;
  }
  m(3, 3) = 1.0;
  return a;
}

py::array_t<double> mat33(const std::array<double, 9>& M) {
  py::array_t<double> a({3, 3});
  auto m = a.mutable_unchecked<2>();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) m(i, j) = M[3 * i + j];
  return a;
}

py::array_t<double> mat6x(const std::vector<double>& J) {  // 6 x n row-major -> ndarray
  const ssize_t n = (ssize_t)(J.size() / 6);
  py::array_t<double> a({(ssize_t)6, n});
  auto m = a.mutable_unchecked<2>();
  for (ssize_t r = 0; r < 6; ++r)
    for (ssize_t c = 0; c < n; ++c) m(r, c) = J[(size_t)r * n + c];
  return a;
}

// fcl::Triangle: three vertex indices
struct Triangle {
  std::array<size_t, 3> v{0, 0, 0};
};

py::array_t<double> vec(const double* p, int n) {
  py::array_t<double> a(n);
  auto m = a.mutable_unchecked<1>();
  for (int i = 0; i < n; ++i) m(i) = p[i];
  return a;
}

// NotImplemented-style errors from the host become NotImplementedError.
void translate_exceptions() {
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const std::logic_error& e) {
      std::string m = e.what();
      if (m.rfind("NotImplemented: ", 0) == 0) {
        PyErr_SetString(PyExc_NotImplementedError, m.substr(16).c_str());
        return;
      }
      if (dynamic_cast<const std::invalid_argument*>(&e)) {
        PyErr_SetString(PyExc_ValueError, m.c_str());
        return;
      }
      if (dynamic_cast<const std::out_of_range*>(&e)) {
        PyErr_SetString(PyExc_IndexError, m.c_str());
        return;
      }
      PyErr_SetString(PyExc_RuntimeError, m.c_str());
    }
  });
}

}  // namespace

PYBIND11_MODULE(pymp, m_all) {
  m_all.doc() = "mplib_amd.pymp -- MI355X-native MPlib collision/validity path";
  translate_exceptions();
  m_all.def("set_global_seed", &set_global_seed, py::arg("seed"));
  m_all.def("device_version", []() { return std::string(mpg_version()); });
  auto m_st = m_all.def_submodule("_selftest", "host-only self tests (no device)");
  m_st.def("async_check_shutdown", &async_check_selftest, py::arg("batch_ms"), py::arg("in_flight"),
           py::call_guard<py::gil_scoped_release>(),
           "Destroys the planner's asynchronous validity helper with a fake batch of batch_ms in flight "
           "(or after two completed batches); returns the destructor's wall time in ms.");

  // ------------------------------------------------------------------ fcl
  auto m = m_all.def_submodule("fcl");
  // fcl.Triangle (python/pybind_fcl.hpp:59-65): three vertex indices
  py::class_<Triangle, std::shared_ptr<Triangle>>(m, "Triangle")
      .def(py::init<>())
      .def(py::init([](unsigned long a, unsigned long b, unsigned long c) { return Triangle{{a, b, c}}; }))
      .def("set", [](Triangle& t, int a, int b, int c) { t.v = {(size_t)a, (size_t)b, (size_t)c}; })
      .def("get", [](const Triangle& t, int i) { return t.v.at(i); })
      .def("__getitem__", [](const Triangle& t, int i) { return t.v.at(i); });

  // fcl.CollisionGeometry (python/pybind_fcl.hpp:68-82); the methods are
  // FCL 0.7.0's, restated in geomprops.cpp
  py::class_<CollisionGeometry, std::shared_ptr<CollisionGeometry>>(m, "CollisionGeometry")
      .def_readonly("kind", &CollisionGeometry::kind)
      .def("computeLocalAABB", [](CollisionGeometry& g) { compute_local_aabb(g); })
      .def("isOccupied", [](const CollisionGeometry& g) { return g.cost_density >= g.threshold_occupied; })
      .def("isFree", [](const CollisionGeometry& g) { return g.cost_density <= g.threshold_free; })
      .def("isUncertain",
           [](const CollisionGeometry& g) {
             return !(g.cost_density >= g.threshold_occupied) && !(g.cost_density <= g.threshold_free);
           })
      .def("computeCOM", [](const CollisionGeometry& g) { return compute_com(g); })
      .def("computeMomentofInertia", [](const CollisionGeometry& g) { return mat33(compute_moment_of_inertia(g)); })
      .def("computeVolume", [](const CollisionGeometry& g) { return compute_volume(g); })
      .def("computeMomentofInertiaRelatedToCOM",
           [](const CollisionGeometry& g) { return mat33(compute_moment_of_inertia_com(g)); })
      .def_readwrite("aabb_center", &CollisionGeometry::aabb_center)
      .def_readwrite("aabb_radius", &CollisionGeometry::aabb_radius)
      .def_readwrite("cost_density", &CollisionGeometry::cost_density);
  py::class_<Box, CollisionGeometry, std::shared_ptr<Box>>(m, "Box")
      .def(py::init([](const std::vector<double>& s) { return std::make_shared<Box>(vec3_arg(s)); }), py::arg("side"))
      .def(py::init([](double x, double y, double z) { return std::make_shared<Box>(Vec3{x, y, z}); }), py::arg("x"),
           py::arg("y"), py::arg("z"))
      .def_readwrite("side", &Box::side);
  py::class_<Sphere, CollisionGeometry, std::shared_ptr<Sphere>>(m, "Sphere")
      .def(py::init<double>(), py::arg("radius"))
      .def_readwrite("radius", &Sphere::radius);
  py::class_<Capsule, CollisionGeometry, std::shared_ptr<Capsule>>(m, "Capsule")
      .def(py::init<double, double>(), py::arg("radius"), py::arg("lz"))
      .def_readwrite("radius", &Capsule::radius)
      .def_readwrite("lz", &Capsule::lz);
  py::class_<Cylinder, CollisionGeometry, std::shared_ptr<Cylinder>>(m, "Cylinder")
      .def(py::init<double, double>(), py::arg("radius"), py::arg("lz"))
      .def_readwrite("radius", &Cylinder::radius)
      .def_readwrite("lz", &Cylinder::lz);
  py::class_<Cone, CollisionGeometry, std::shared_ptr<Cone>>(m, "Cone")
      .def(py::init<double, double>(), py::arg("radius"), py::arg("lz"))
      .def_readwrite("radius", &Cone::radius)
      .def_readwrite("lz", &Cone::lz);
  py::class_<Ellipsoid, CollisionGeometry, std::shared_ptr<Ellipsoid>>(m, "Ellipsoid")
      .def(py::init([](double a, double b, double c) { return std::make_shared<Ellipsoid>(Vec3{a, b, c}); }),
           py::arg("a"), py::arg("b"), py::arg("c"))
      .def(py::init([](const std::vector<double>& r) { return std::make_shared<Ellipsoid>(vec3_arg(r)); }),
           py::arg("radii"))
      .def_readwrite("radii", &Ellipsoid::radii);
  py::class_<TriangleP, CollisionGeometry, std::shared_ptr<TriangleP>>(m, "TriangleP")
      .def(py::init([](const std::vector<double>& a, const std::vector<double>& b, const std::vector<double>& c) {
             return std::make_shared<TriangleP>(vec3_arg(a), vec3_arg(b), vec3_arg(c));
           }),
           py::arg("a"), py::arg("b"), py::arg("c"))
      .def_readwrite("a", &TriangleP::a)
      .def_readwrite("b", &TriangleP::b)
      .def_readwrite("c", &TriangleP::c);
  // Halfspace / Plane: the types and their geometry; colliding them raises
  // NotImplementedError (host.hpp PlaneLike)
  auto plane_like = [&](auto cls) {
    using T = typename decltype(cls)::type;
    cls.def(py::init([](const std::vector<double>& n, double d) { return std::make_shared<T>(vec3_arg(n), d); }),
            py::arg("n"), py::arg("d"))
        .def(py::init([](double a, double b, double c, double d) { return std::make_shared<T>(Vec3{a, b, c}, d); }),
             py::arg("a"), py::arg("b"), py::arg("c"), py::arg("d"))
        .def_readwrite("n", &T::n)
        .def_readwrite("d", &T::d)
        .def("signed_distance", [](const T& h, const std::vector<double>& p) { return h.signed_distance(vec3_arg(p)); },
             py::arg("p"))
        .def("distance",
             [](const T& h, const std::vector<double>& p) { return std::fabs(h.signed_distance(vec3_arg(p))); },
             py::arg("p"));
  };
  plane_like(py::class_<Halfspace, CollisionGeometry, std::shared_ptr<Halfspace>>(m, "Halfspace"));
  plane_like(py::class_<Plane, CollisionGeometry, std::shared_ptr<Plane>>(m, "Plane"));
  py::class_<Convex, CollisionGeometry, std::shared_ptr<Convex>>(m, "Convex")
      .def(py::init([](py::array_t<double, py::array::c_style | py::array::forcecast> v,
                       py::array_t<int, py::array::c_style | py::array::forcecast> f, bool throw_if_invalid) {
             (void)throw_if_invalid;
             if (v.ndim() != 2 || v.shape(1) != 3) throw std::invalid_argument("vertices must be [N, 3]");
             if (f.ndim() != 2 || f.shape(1) != 3) throw std::invalid_argument("faces must be [M, 3]");
             std::vector<Vec3> vv;
             auto a = v.unchecked<2>();
             for (ssize_t i = 0; i < v.shape(0); ++i) vv.push_back({a(i, 0), a(i, 1), a(i, 2)});
             std::vector<int> ff;
             auto b = f.unchecked<2>();
             for (ssize_t i = 0; i < f.shape(0); ++i) {
               ff.push_back(3);
               for (int k = 0; k < 3; ++k) {
                 if (b(i, k) < 0 || b(i, k) >= (int)vv.size()) throw std::invalid_argument("face index out of range");
                 ff.push_back(b(i, k));
               }
             }
             return std::make_shared<Convex>(std::move(vv), (int)f.shape(0), std::move(ff));
           }),
           py::arg("vertices"), py::arg("faces"), py::arg("throw_if_invalid") = true)
      .def("get_face_count", [](const Convex& c) { return c.num_faces; })
      .def("get_faces", [](const Convex& c) { return c.faces; })
      .def("get_vertices",
           [](const Convex& c) {
             py::array_t<double> a({(ssize_t)c.vertices.size(), (ssize_t)3});
             auto x = a.mutable_unchecked<2>();
             for (size_t i = 0; i < c.vertices.size(); ++i)
               for (int k = 0; k < 3; ++k) x(i, k) = c.vertices[i][k];
             return a;
           })
      .def("compute_volume", [](const Convex& c) { return compute_volume(c); })
      .def("get_interior_point", [](const Convex& c) {
        auto p = c.interior_point();
        return vec(p.data(), 3);
      });

  // fcl.BVHModel (python/pybind_fcl.hpp:177-219): triangle mesh built with
  // beginModel / addSubModel / endModel
  auto tri_arg = [](py::array_t<int, py::array::c_style | py::array::forcecast> f) {
    if (f.ndim() != 2 || f.shape(1) != 3) throw std::invalid_argument("faces must be [M, 3]");
    std::vector<std::array<int, 3>> t;
    auto b = f.unchecked<2>();
    for (ssize_t i = 0; i < f.shape(0); ++i) t.push_back({b(i, 0), b(i, 1), b(i, 2)});
    return t;
  };
  auto vert_arg = [](py::array_t<double, py::array::c_style | py::array::forcecast> v) {
    if (v.ndim() != 2 || v.shape(1) != 3) throw std::invalid_argument("vertices must be [N, 3]");
    std::vector<Vec3> vv;
    auto a = v.unchecked<2>();
    for (ssize_t i = 0; i < v.shape(0); ++i) vv.push_back({a(i, 0), a(i, 1), a(i, 2)});
    return vv;
  };
  py::class_<BVHModel, CollisionGeometry, std::shared_ptr<BVHModel>>(m, "BVHModel")
      .def(py::init<>())
      .def(
          "beginModel",
          [](BVHModel& b, int num_faces, int num_vertices) {
            (void)num_faces;
            (void)num_vertices;
            b.vertices.clear();
            b.triangles.clear();
            b.building = true;
          },
          py::arg("num_faces") = 0, py::arg("num_vertices") = 0)
      .def("endModel", [](BVHModel& b) { b.building = false; })
      .def(
          "addSubModel", [=](BVHModel& b, py::array_t<double> v) { b.add_sub_model(vert_arg(v), {}); },
          py::arg("vertices"))
      .def(
          "addSubModel", [=](BVHModel& b, py::array_t<double> v, const std::vector<Triangle>& f) {
            std::vector<std::array<int, 3>> t;
            for (auto& x : f) t.push_back({(int)x.v[0], (int)x.v[1], (int)x.v[2]});
            b.add_sub_model(vert_arg(v), t);
          },
          py::arg("vertices"), py::arg("faces"))
      .def(
          "addSubModel", [=](BVHModel& b, py::array_t<double> v, py::array_t<int> f) {
            b.add_sub_model(vert_arg(v), tri_arg(f));
          },
          py::arg("vertices"), py::arg("faces"))
      .def("get_vertices",
           [](const BVHModel& b) {
             py::array_t<double> a({(ssize_t)b.vertices.size(), (ssize_t)3});
             auto x = a.mutable_unchecked<2>();
             for (size_t i = 0; i < b.vertices.size(); ++i)
               for (int k = 0; k < 3; ++k) x(i, k) = b.vertices[i][k];
             return a;
           })
      .def("get_faces",
           [](const BVHModel& b) {
             py::array_t<int> a({(ssize_t)b.triangles.size(), (ssize_t)3});
             auto x = a.mutable_unchecked<2>();
             for (size_t i = 0; i < b.triangles.size(); ++i)
               for (int k = 0; k < 3; ++k) x(i, k) = b.triangles[i][k];
             return a;
           })
      .def_property_readonly("num_faces", [](const BVHModel& b) { return (int)b.triangles.size(); })
      .def_property_readonly("num_vertices", [](const BVHModel& b) { return (int)b.vertices.size(); });

  // fcl.OcTree (python/pybind_fcl.hpp:221-236)
  py::class_<OcTree, CollisionGeometry, std::shared_ptr<OcTree>>(m, "OcTree")
      .def(py::init<double>(), py::arg("resolution"))
      .def(py::init([](py::array_t<double, py::array::c_style | py::array::forcecast> v, double res) {
             if (v.ndim() != 2 || v.shape(1) != 3) throw std::invalid_argument("vertices must be [N, 3]");
             std::vector<Vec3> pts;
             auto a = v.unchecked<2>();
             for (ssize_t i = 0; i < v.shape(0); ++i) pts.push_back({a(i, 0), a(i, 1), a(i, 2)});
             return std::make_shared<OcTree>(pts, res);
           }),
           py::arg("vertices"), py::arg("resolution"))
      .def("get_resolution", [](const OcTree& o) { return o.resolution; })
      .def("get_leaf_boxes",
           [](const OcTree& o) {
             py::array_t<double> a({(ssize_t)o.leaves.size(), (ssize_t)6});
             auto x = a.mutable_unchecked<2>();
             for (size_t i = 0; i < o.leaves.size(); ++i)
               for (int k = 0; k < 6; ++k) x(i, k) = o.leaves[i][k];
             return a;
           },
           "Occupied leaves as [min xyz, max xyz] boxes in the octree frame (FCL traversal order).");

  py::class_<CollisionObject, std::shared_ptr<CollisionObject>>(m, "CollisionObject")
      .def(py::init([](const GeomPtr& g, const std::vector<double>& p, const std::vector<double>& q) {
             return std::make_shared<CollisionObject>(g, se3_from_pq(vec3_arg(p), quat_arg(q)));
           }),
           py::arg("collision_geometry"), py::arg("position") = std::vector<double>{0, 0, 0},
           py::arg("quaternion") = std::vector<double>{1, 0, 0, 0})
      .def("get_collision_geometry", [](const CollisionObject& o) { return o.geom; })
      .def("get_translation", [](const CollisionObject& o) { return vec(o.tf.p, 3); })
      .def("get_rotation", [](const CollisionObject& o) { return mat3(o.tf); })
      .def("set_transformation",
           [](CollisionObject& o, const std::vector<double>& pose) { o.set_transform(se3_from_pose7(vec7_arg(pose))); },
           py::arg("pose"));

  py::enum_<GJKSolverType>(m, "GJKSolverType")
      .value("GST_LIBCCD", GST_LIBCCD)
      .value("GST_INDEP", GST_INDEP)
      .export_values();

  py::class_<CollisionRequest, std::shared_ptr<CollisionRequest>>(m, "CollisionRequest")
      .def(py::init([](size_t nmc, bool ec, size_t nmcs, bool ecost, bool uac, GJKSolverType t, double tol) {
             CollisionRequest r;
             r.num_max_contacts = nmc;
             r.enable_contact = ec;
             r.num_max_cost_sources = nmcs;
             r.enable_cost = ecost;
             r.use_approximate_cost = uac;
             r.gjk_solver_type = t;
             r.gjk_tolerance = tol;
             return r;
           }),
           py::arg("num_max_contacts") = 1, py::arg("enable_contact") = false, py::arg("num_max_cost_sources") = 1,
           py::arg("enable_cost") = false, py::arg("use_approximate_cost") = true,
           py::arg("gjk_solver_type") = GST_LIBCCD, py::arg("gjk_tolerance") = 1e-6)
      .def_readwrite("num_max_contacts", &CollisionRequest::num_max_contacts)
      .def_readwrite("enable_contact", &CollisionRequest::enable_contact)
      .def_readwrite("gjk_solver_type", &CollisionRequest::gjk_solver_type)
      .def_readwrite("gjk_tolerance", &CollisionRequest::gjk_tolerance)
      .def("isSatisfied", [](const CollisionRequest& r, const CollisionResult& res) {
        return !r.enable_cost && res.num_contacts() >= r.num_max_contacts;
      }, py::arg("result"));

  py::class_<Contact, std::shared_ptr<Contact>>(m, "Contact")
      .def(py::init<>())
      .def(py::init([](const GeomPtr& o1, const GeomPtr& o2, int b1, int b2) {
             Contact c;
             c.o1 = o1;
             c.o2 = o2;
             c.b1 = b1;
             c.b2 = b2;
             return c;
           }),
           py::arg("o1"), py::arg("o2"), py::arg("b1"), py::arg("b2"))
      .def(py::init([](const GeomPtr& o1, const GeomPtr& o2, int b1, int b2, const std::vector<double>& pos,
                       const std::vector<double>& normal, double depth) {
             Contact c;
             c.o1 = o1;
             c.o2 = o2;
             c.b1 = b1;
             c.b2 = b2;
             c.pos = vec3_arg(pos);
             c.normal = vec3_arg(normal);
             c.penetration_depth = depth;
             return c;
           }),
           py::arg("o1"), py::arg("o2"), py::arg("b1"), py::arg("b2"), py::arg("pos"), py::arg("normal"),
           py::arg("depth"))
      .def_readonly("normal", &Contact::normal)
      .def_readonly("pos", &Contact::pos)
      .def_readonly("penetration_depth", &Contact::penetration_depth);

  py::class_<ContactPoint, std::shared_ptr<ContactPoint>>(m, "ContactPoint")
      .def(py::init<>())
      .def(py::init([](const std::vector<double>& normal, const std::vector<double>& pos, double depth) {
             return ContactPoint{vec3_arg(normal), vec3_arg(pos), depth};
           }),
           py::arg("normal"), py::arg("pos"), py::arg("penetration_depth"))
      .def_readonly("normal", &ContactPoint::normal)
      .def_readonly("pos", &ContactPoint::pos)
      .def_readonly("penetration_depth", &ContactPoint::penetration_depth);
  py::class_<CostSource, std::shared_ptr<CostSource>>(m, "CostSource")
      .def(py::init<>())
      .def(py::init([](const std::vector<double>& lo, const std::vector<double>& hi, double d) {
             return CostSource(vec3_arg(lo), vec3_arg(hi), d);
           }),
           py::arg("aabb_min"), py::arg("aabb_max"), py::arg("cost_density"))
      .def_readonly("aabb_min", &CostSource::aabb_min)
      .def_readonly("aabb_max", &CostSource::aabb_max)
      .def_readonly("cost_density", &CostSource::cost_density)
      .def_readonly("total_cost", &CostSource::total_cost);

  py::class_<DistanceRequest, std::shared_ptr<DistanceRequest>>(m, "DistanceRequest")
      .def(py::init([](bool np_, bool sd, double rel, double abs_, double tol, GJKSolverType t) {
             DistanceRequest r;
             r.enable_nearest_points = np_;
             r.enable_signed_distance = sd;
             r.rel_err = rel;
             r.abs_err = abs_;
             r.distance_tolerance = tol;
             r.gjk_solver_type = t;
             return r;
           }),
           py::arg("enable_nearest_points") = false, py::arg("enable_signed_distance") = false,
           py::arg("rel_err") = 0.0, py::arg("abs_err") = 0.0, py::arg("distance_tolerance") = 1e-6,
           py::arg("gjk_solver_type") = GST_LIBCCD)
      .def("isSatisfied", [](const DistanceRequest&, const DistanceResult&) { return false; }, py::arg("result"));
  py::class_<DistanceResult, std::shared_ptr<DistanceResult>>(m, "DistanceResult")
      .def(py::init([](double d) {
             DistanceResult r;
             r.min_distance = d;
             return r;
           }),
           py::arg("min_distance") = std::numeric_limits<double>::max())
      .def_readonly("nearest_points", &DistanceResult::nearest_points)
      .def_readonly("min_distance", &DistanceResult::min_distance)
      .def("clear", &DistanceResult::clear);

  py::class_<CollisionResult, std::shared_ptr<CollisionResult>>(m, "CollisionResult")
      .def(py::init<>())
      .def("add_contact", &CollisionResult::add_contact, py::arg("c"))
      .def("add_cost_source", &CollisionResult::add_cost_source, py::arg("c"), py::arg("num_max_cost_sources"))
      .def("num_cost_sources", &CollisionResult::num_cost_sources)
      .def("get_cost_sources", [](const CollisionResult& r) { return r.cost_sources; })
      .def("is_collision", &CollisionResult::is_collision)
      .def("num_contacts", &CollisionResult::num_contacts)
      .def("get_contacts", [](const CollisionResult& r) { return r.contacts; })
      .def("get_contact", [](const CollisionResult& r, size_t i) { return r.contacts.at(i); }, py::arg("i"))
      .def("clear", &CollisionResult::clear);

  py::class_<FCLModel, std::shared_ptr<FCLModel>>(m, "FCLModel")
      .def(py::init([](const std::string& urdf, bool verbose, bool convex) {
             return FCLModel::from_file(urdf, verbose, convex);
           }),
           py::arg("urdf_filename"), py::arg("verbose") = true, py::arg("convex") = false)
      .def_static("create_from_urdf_string", &FCLModel::from_urdf_string, py::arg("urdf_string"),
                  py::arg("collision_links"), py::arg("verbose") = true)
      .def("get_collision_pairs", &FCLModel::get_collision_pairs)
      .def("get_collision_objects", &FCLModel::get_collision_objects)
      .def("get_collision_link_names", &FCLModel::get_collision_link_names)
      .def("set_link_order", &FCLModel::set_link_order, py::arg("names"))
      .def("remove_collision_pairs_from_srdf", &FCLModel::remove_collision_pairs_from_srdf, py::arg("srdf_filename"))
      .def("update_collision_objects",
           [](FCLModel& f, const std::vector<std::vector<double>>& poses) {
             std::vector<Vec7> p;
             for (auto& v : poses) p.push_back(vec7_arg(v));
             f.update_collision_objects(p);
           },
           py::arg("link_poses"))
      .def("collide", &FCLModel::collide, py::arg("request") = CollisionRequest(),
           py::call_guard<py::gil_scoped_release>())
      .def("collide_full", &FCLModel::collide_full, py::arg("request") = CollisionRequest(),
           py::call_guard<py::gil_scoped_release>())
      .def("print_collision_pairs", &FCLModel::print_collision_pairs);

  m.def("load_mesh_as_BVH",
        [](const std::string& path, const std::vector<double>& scale) { return load_mesh_as_bvh(path, vec3_arg(scale)); },
        py::arg("mesh_path"), py::arg("scale"));
  m.def("load_mesh_as_Convex",
        [](const std::string& path, const std::vector<double>& scale) {
          return load_mesh_as_convex(path, vec3_arg(scale));
        },
        py::arg("mesh_path"), py::arg("scale"));
  m.def(
      "collide",
      [](const ObjPtr& o1, const ObjPtr& o2, const CollisionRequest& req) {
        // fcl::collide(o1, o2): a two-object world evaluated on the device
        req.check_supported();
        DescBuilder d;
        d.gjk_tolerance = req.gjk_tolerance;
        d.gjk_solver = req.gjk_solver_type == GST_INDEP ? MPG_GJK_INDEP : MPG_GJK_LIBCCD;
        d.link_parent.push_back(0);
        SE3 I;
        mpg::se3_identity(I);
        push_se3(d.link_placement, I);
        d.moving_link.push_back(0);
        d.moving_geom.push_back(d.add_geometry(o1->geom.get()));
        push_se3(d.moving_offset, o1->tf);
        d.static_geom.push_back(d.add_geometry(o2->geom.get()));
        push_se3(d.static_transform, o2->tf);
        d.pair_a.push_back(0);
        d.pair_b.push_back(1);
        d.pair_allowed.push_back(0);
        DeviceWorld w(d, default_device());
        const double pose[7] = {0, 0, 0, 1, 0, 0, 0};
        uint8_t flag = 0;
        uint32_t mask = 0;
        double depth = 0, normal[3] = {0, 0, 0}, pos[3] = {0, 0, 0};
        if (req.enable_contact)
          check_status(mpg_collide_contacts(w.get(), pose, 1, MPG_INPUT_LINK_POSES, &flag, &mask, &depth, normal, pos,
                                            MPG_MEM_HOST, nullptr),
                       "mpg_collide_contacts");
        else
          check_status(mpg_collide_link_poses(w.get(), pose, 1, &flag, &mask, MPG_MEM_HOST, nullptr),
                       "mpg_collide_link_poses");
        CollisionResult r;
        if (flag) {
          Contact c;
          c.o1 = o1->geom;
          c.o2 = o2->geom;
          if (req.enable_contact) {
            c.penetration_depth = depth;
            for (int k = 0; k < 3; ++k) {
              c.normal[k] = normal[k];
              c.pos[k] = pos[k];
            }
          }
          r.contacts.push_back(c);
        }
        return r;
      },
      py::arg("o1"), py::arg("o2"), py::arg("request") = CollisionRequest());
  m.def(
      "distance",
      [](const ObjPtr& o1, const ObjPtr& o2, const DistanceRequest& req) {
        // fcl::distance(o1, o2): a two-object world evaluated on the device
        req.check_supported();
        DescBuilder d;
        d.link_parent.push_back(0);
        SE3 I;
        mpg::se3_identity(I);
        push_se3(d.link_placement, I);
        d.moving_link.push_back(0);
        d.moving_geom.push_back(d.add_geometry(o1->geom.get()));
        push_se3(d.moving_offset, o1->tf);
        d.static_geom.push_back(d.add_geometry(o2->geom.get()));
        push_se3(d.static_transform, o2->tf);
        d.pair_a.push_back(0);
        d.pair_b.push_back(1);
        d.pair_allowed.push_back(0);
        DeviceWorld w(d, default_device());
        double ds = 0, dd = 0, qs[6], qo[6];
        int32_t ps = -1, po = -1;
        const mpg_distance_request creq = req.to_c();
        check_status(mpg_distance_batch_req(w.get(), nullptr, 1, 0, &creq, &ds, &ps, qs, &dd, &po, qo, MPG_MEM_HOST,
                                            nullptr),
                     "mpg_distance_batch_req");
        DistanceResult r;
        r.min_distance = dd;
        for (int k = 0; k < 3; ++k) {
          r.nearest_points[0][k] = qo[k];
          r.nearest_points[1][k] = qo[3 + k];
        }
        return r;
      },
      py::arg("o1"), py::arg("o2"), py::arg("request") = DistanceRequest());

  // fcl.collide / fcl.distance(articulation, o2, request)
  // (python/pybind_fcl.hpp:371-436): every collision object of the
  // articulation's FCLModel (at its current poses) against o2, as one device
  // world -- the objects ride on one identity link pose, o2 is static
  auto art_world = [](const ArtPtr& art, const ObjPtr& o2, DescBuilder& d) {
    const auto& objs = art->get_fcl_model()->get_collision_objects();
    d.link_parent.push_back(0);
    SE3 I;
    mpg::se3_identity(I);
    push_se3(d.link_placement, I);
    for (auto& o : objs) {
      d.moving_link.push_back(0);
      d.moving_geom.push_back(d.add_geometry(o->geom.get()));
      push_se3(d.moving_offset, o->tf);
    }
    d.static_geom.push_back(d.add_geometry(o2->geom.get()));
    push_se3(d.static_transform, o2->tf);
    for (size_t i = 0; i < objs.size(); ++i) {
      d.pair_a.push_back((int)i);
      d.pair_b.push_back((int)objs.size());
      d.pair_allowed.push_back(0);
    }
    return objs.size();
  };
  m.def(
      "collide",
      [=](const ArtPtr& art, const ObjPtr& o2, const CollisionRequest& req) {
        req.check_supported();
        DescBuilder d;
        d.gjk_tolerance = req.gjk_tolerance;
        d.gjk_solver = req.gjk_solver_type == GST_INDEP ? MPG_GJK_INDEP : MPG_GJK_LIBCCD;
        const size_t n = art_world(art, o2, d);
        std::vector<WorldCollisionResult> ret;
        if (n == 0) return ret;
        DeviceWorld w(d, default_device());
        const double pose[7] = {0, 0, 0, 1, 0, 0, 0};
        uint8_t flag = 0;
        std::vector<uint32_t> mask((n + 31) / 32, 0);
        std::vector<double> depth(n, 0.0), normal(3 * n, 0.0), pos(3 * n, 0.0);
        if (req.enable_contact)
          check_status(mpg_collide_contacts(w.get(), pose, 1, MPG_INPUT_LINK_POSES, &flag, mask.data(), depth.data(),
                                            normal.data(), pos.data(), MPG_MEM_HOST, nullptr),
                       "mpg_collide_contacts");
        else
          check_status(mpg_collide_link_poses(w.get(), pose, 1, &flag, mask.data(), MPG_MEM_HOST, nullptr),
                       "mpg_collide_link_poses");
        const auto& objs = art->get_fcl_model()->get_collision_objects();
        const auto& names = art->get_fcl_model()->get_collision_link_names();
        for (size_t i = 0; i < n; ++i) {
          if (!((mask[i >> 5] >> (i & 31)) & 1u)) continue;
          WorldCollisionResult r;
          Contact c;
          c.o1 = objs[i]->geom;
          c.o2 = o2->geom;
          if (req.enable_contact) fill_contacts(mask.data(), n, depth, normal, pos, i, c);
          r.res.contacts.push_back(c);
          r.collision_type = "articulation_sceneobject";
          r.object_name1 = art->get_name();
          r.object_name2 = "__object__";
          r.link_name1 = names[i];
          r.link_name2 = "__object__";
          ret.push_back(std::move(r));
        }
        return ret;
      },
      py::arg("articulation"), py::arg("o2"), py::arg("request") = CollisionRequest());
  m.def(
      "distance",
      [=](const ArtPtr& art, const ObjPtr& o2, const DistanceRequest& req) {
        req.check_supported();
        DescBuilder d;
        const size_t n = art_world(art, o2, d);
        WorldDistanceResult ret;
        if (n == 0) return ret;
        DeviceWorld w(d, default_device());
        // the pairs are the world's "others" group: minimum and first argmin
        // (FCL's loop keeps the first strictly smaller distance)
        double ds = 0, dd = 0, qs[6], qo[6];
        int32_t ps = -1, po = -1;
        const mpg_distance_request creq = req.to_c();
        check_status(mpg_distance_batch_req(w.get(), nullptr, 1, 0, &creq, &ds, &ps, qs, &dd, &po, qo, MPG_MEM_HOST,
                                            nullptr),
                     "mpg_distance_batch_req");
        if (po < 0) return ret;
        const auto& names = art->get_fcl_model()->get_collision_link_names();
        ret.res.min_distance = dd;
        for (int k = 0; k < 3; ++k) {
          ret.res.nearest_points[0][k] = qo[k];
          ret.res.nearest_points[1][k] = qo[3 + k];
        }
        ret.min_distance = dd;
        ret.distance_type = "articulation_sceneobject";
        ret.object_name1 = art->get_name();
        ret.object_name2 = "__object__";
        ret.link_name1 = names[po];
        ret.link_name2 = "__object__";
        return ret;
      },
      py::arg("articulation"), py::arg("o2"), py::arg("request") = DistanceRequest());

  // ------------------------------------------------------------ pinocchio
  auto mp = m_all.def_submodule("pinocchio");
  py::class_<PinocchioModel, std::shared_ptr<PinocchioModel>>(mp, "PinocchioModel")
      .def(py::init([](const std::string& urdf, const std::vector<double>& g, bool verbose) {
             return PinocchioModel::from_file(urdf, vec3_arg(g), verbose);
           }),
           py::arg("urdf_filename"), py::arg("gravity") = std::vector<double>{0, 0, -9.81}, py::arg("verbose") = true)
      .def_static("create_from_urdf_string",
                  [](const std::string& urdf, const std::vector<double>& g, bool verbose) {
                    return PinocchioModel::from_string(urdf, vec3_arg(g), verbose);
                  },
                  py::arg("urdf_string"), py::arg("gravity") = std::vector<double>{0, 0, -9.81},
                  py::arg("verbose") = true)
      .def("set_joint_order", &PinocchioModel::set_joint_order, py::arg("names"))
      .def("set_link_order", &PinocchioModel::set_link_order, py::arg("names"))
      .def("compute_forward_kinematics", &PinocchioModel::compute_forward_kinematics, py::arg("qpos"))
      .def("get_link_pose",
           [](const PinocchioModel& p, size_t i) {
             auto v = p.get_link_pose(i);
             return vec(v.data(), 7);
           },
           py::arg("index"))
      .def("get_random_configuration", &PinocchioModel::get_random_configuration)
      .def("print_frames", &PinocchioModel::print_frames)
      // Jacobians and CLIK IK (python/pybind_pinocchio.hpp:47-58), host side (kinjac.cpp)
      .def("compute_full_jacobian", &PinocchioModel::compute_full_jacobian, py::arg("qpos"))
      .def("get_link_jacobian",
           [](const PinocchioModel& p, size_t i, bool local) { return mat6x(p.get_link_jacobian(i, local)); },
           py::arg("index"), py::arg("local") = false)
      .def("compute_single_link_local_jacobian",
           [](PinocchioModel& p, const std::vector<double>& q, size_t i) {
             return mat6x(p.compute_single_link_local_jacobian(q, i));
           },
           py::arg("qpos"), py::arg("index"))
      .def("compute_IK_CLIK",
           [](const PinocchioModel& p, size_t i, const std::vector<double>& pose, const std::vector<double>& q_init,
              const std::vector<bool>& mask, double eps, int max_iter, double dt, double damp) {
             const auto r = p.ik_clik(i, vec7_arg(pose), q_init, &mask, nullptr, nullptr, eps, max_iter, dt, damp);
             return py::make_tuple(vec(r.q.data(), (int)r.q.size()), r.success, vec(r.err.data(), 6));
           },
           py::arg("index"), py::arg("pose"), py::arg("q_init"), py::arg("mask") = std::vector<bool>(),
           py::arg("eps") = 1e-5, py::arg("maxIter") = 1000, py::arg("dt") = 1e-1, py::arg("damp") = 1e-12)
      .def("compute_IK_CLIK_JL",
           [](const PinocchioModel& p, size_t i, const std::vector<double>& pose, const std::vector<double>& q_init,
              const std::vector<double>& q_min, const std::vector<double>& q_max, double eps, int max_iter, double dt,
              double damp) {
             const auto r = p.ik_clik(i, vec7_arg(pose), q_init, nullptr, &q_min, &q_max, eps, max_iter, dt, damp);
             return py::make_tuple(vec(r.q.data(), (int)r.q.size()), r.success, vec(r.err.data(), 6));
           },
           py::arg("index"), py::arg("pose"), py::arg("q_init"), py::arg("q_min"), py::arg("q_max"),
           py::arg("eps") = 1e-5, py::arg("maxIter") = 1000, py::arg("dt") = 1e-1, py::arg("damp") = 1e-12)
      .def("get_joint_names", &PinocchioModel::get_joint_names, py::arg("user") = true)
      .def("get_link_names", &PinocchioModel::get_link_names, py::arg("user") = true)
      .def("get_leaf_links", &PinocchioModel::get_leaf_links)
      .def("get_joint_dim", &PinocchioModel::get_joint_dim, py::arg("index"), py::arg("user") = true)
      .def("get_joint_dims", &PinocchioModel::get_joint_dims, py::arg("user") = true)
      .def("get_joint_id", &PinocchioModel::get_joint_id, py::arg("index"), py::arg("user") = true)
      .def("get_joint_ids", &PinocchioModel::get_joint_ids, py::arg("user") = true)
      .def("get_parents", &PinocchioModel::get_parents, py::arg("user") = true)
      .def("get_joint_type", &PinocchioModel::get_joint_type, py::arg("index"), py::arg("user") = true)
      .def("get_joint_types", &PinocchioModel::get_joint_types, py::arg("user") = true)
      .def("get_joint_limit", &PinocchioModel::get_joint_limit, py::arg("index"), py::arg("user") = true)
      .def("get_joint_limits", &PinocchioModel::get_joint_limits, py::arg("user") = true)
      .def("get_chain_joint_name", &PinocchioModel::get_chain_joint_name, py::arg("end_effector"))
      .def("get_chain_joint_index", &PinocchioModel::get_chain_joint_index, py::arg("end_effector"));

  // ------------------------------------------------------------------ kdl
  auto mk = m_all.def_submodule("kdl");
  auto kdl_ret = [](const std::tuple<std::vector<double>, int>& r) {
    const auto& q = std::get<0>(r);
    return py::make_tuple(vec(q.data(), (int)q.size()), std::get<1>(r));
  };
  py::class_<KDLModel, std::shared_ptr<KDLModel>>(mk, "KDLModel")
      .def(py::init<const std::string&, const std::vector<std::string>&, const std::vector<std::string>&, bool>(),
           py::arg("urdf_filename"), py::arg("joint_names"), py::arg("link_names"), py::arg("verbose"))
      .def("get_tree_root_name", &KDLModel::get_tree_root_name)
      .def("chain_IK_LMA",
           [=](const KDLModel& k, size_t i, const std::vector<double>& q0, const std::vector<double>& pose) {
             return kdl_ret(k.chain_ik(i, q0, vec7_arg(pose), 2));
           },
           py::arg("index"), py::arg("q_init"), py::arg("goal_pose"))
      .def("chain_IK_NR",
           [=](const KDLModel& k, size_t i, const std::vector<double>& q0, const std::vector<double>& pose) {
             return kdl_ret(k.chain_ik(i, q0, vec7_arg(pose), 0));
           },
           py::arg("index"), py::arg("q_init"), py::arg("goal_pose"))
      .def("chain_IK_NR_JL",
           [=](const KDLModel& k, size_t i, const std::vector<double>& q0, const std::vector<double>& pose,
               const std::vector<double>& qmin, const std::vector<double>& qmax) {
             return kdl_ret(k.chain_ik(i, q0, vec7_arg(pose), 1, &qmin, &qmax));
           },
           py::arg("index"), py::arg("q_init"), py::arg("goal_pose"), py::arg("q_min"), py::arg("q_max"))
      .def("tree_IK_NR_JL",
           [=](const KDLModel& k, const std::vector<std::string>& ends, const std::vector<double>& q0,
               const std::vector<std::vector<double>>& poses, const std::vector<double>& qmin,
               const std::vector<double>& qmax) {
             std::vector<Vec7> p;
             for (auto& v : poses) p.push_back(vec7_arg(v));
             return kdl_ret(k.tree_ik_nr_jl(ends, q0, p, qmin, qmax));
           },
           py::arg("endpoints"), py::arg("q_init"), py::arg("goal_poses"), py::arg("q_min"), py::arg("q_max"));

  // ---------------------------------------------------------- articulation
  auto ma = m_all.def_submodule("articulation");
  py::class_<ArticulatedModel, std::shared_ptr<ArticulatedModel>>(ma, "ArticulatedModel")
      .def(py::init([](const std::string& urdf, const std::string& srdf, const std::vector<double>& g,
                       const std::vector<std::string>& joints, const std::vector<std::string>& links, bool verbose,
                       bool convex) {
             return ArticulatedModel::create(urdf, srdf, vec3_arg(g), joints, links, verbose, convex);
           }),
           py::arg("urdf_filename"), py::arg("srdf_filename"), py::arg("gravity") = std::vector<double>{0, 0, -9.81},
           py::arg("joint_names") = std::vector<std::string>(), py::arg("link_names") = std::vector<std::string>(),
           py::arg("verbose") = true, py::arg("convex") = false)
      .def_static("create_from_urdf_string",
                  [](const std::string& urdf, const std::string& srdf,
                     const std::vector<std::pair<std::string, std::vector<ObjPtr>>>& links,
                     const std::vector<double>& g, const std::vector<std::string>& joints,
                     const std::vector<std::string>& lnames, bool verbose) {
                    return ArticulatedModel::create_from_urdf_string(urdf, srdf, links, vec3_arg(g), joints, lnames,
                                                                     verbose);
                  },
                  py::arg("urdf_string"), py::arg("srdf_string"), py::arg("collision_links"),
                  py::arg("gravity") = std::vector<double>{0, 0, -9.81},
                  py::arg("joint_names") = std::vector<std::string>(),
                  py::arg("link_names") = std::vector<std::string>(), py::arg("verbose") = true)
      .def("get_pinocchio_model", &ArticulatedModel::get_pinocchio_model)
      .def("get_fcl_model", &ArticulatedModel::get_fcl_model)
      .def("get_user_link_names", &ArticulatedModel::get_user_link_names)
      .def("get_user_joint_names", &ArticulatedModel::get_user_joint_names)
      .def("get_move_group_joint_indices", &ArticulatedModel::get_move_group_joint_indices)
      .def("get_move_group_end_effectors", &ArticulatedModel::get_move_group_end_effectors)
      .def("get_move_group_joint_names", &ArticulatedModel::get_move_group_joint_names)
      .def("set_move_group",
           [](ArticulatedModel& a, const std::string& ee) { a.set_move_group(std::vector<std::string>{ee}); },
           py::arg("end_effector"))
      .def("set_move_group",
           [](ArticulatedModel& a, const std::vector<std::string>& ees) { a.set_move_group(ees); },
           py::arg("end_effectors"))
      .def("get_qpos", [](const ArticulatedModel& a) { return vec(a.get_qpos().data(), (int)a.get_qpos().size()); })
      .def("set_qpos", &ArticulatedModel::set_qpos, py::arg("qpos"), py::arg("full") = false)
      .def("get_qpos_dim", &ArticulatedModel::get_qpos_dim)
      .def("update_SRDF", &ArticulatedModel::update_srdf, py::arg("SRDF"))
      .def("get_name", &ArticulatedModel::get_name);

  // ------------------------------------------------------ collision_matrix
  auto mc = m_all.def_submodule("collision_matrix");
  py::enum_<AllowedCollision>(mc, "AllowedCollision")
      .value("NEVER", AllowedCollision::NEVER)
      .value("ALWAYS", AllowedCollision::ALWAYS)
      .value("CONDITIONAL", AllowedCollision::CONDITIONAL)
      .export_values();
  using ACM = AllowedCollisionMatrix;
  using S = std::string;
  using VS = std::vector<std::string>;
  py::class_<ACM, std::shared_ptr<ACM>>(mc, "AllowedCollisionMatrix")
      .def(py::init<>())
      .def("get_entry", &ACM::get_entry, py::arg("name1"), py::arg("name2"))
      .def("has_entry", py::overload_cast<const S&>(&ACM::has_entry, py::const_), py::arg("name"))
      .def("has_entry", py::overload_cast<const S&, const S&>(&ACM::has_entry, py::const_), py::arg("name1"),
           py::arg("name2"))
      .def("set_entry", py::overload_cast<const S&, const S&, bool>(&ACM::set_entry), py::arg("name1"),
           py::arg("name2"), py::arg("allowed"))
      .def("set_entry", py::overload_cast<const S&, const VS&, bool>(&ACM::set_entry), py::arg("name"),
           py::arg("other_names"), py::arg("allowed"))
      .def("set_entry", py::overload_cast<const VS&, const VS&, bool>(&ACM::set_entry), py::arg("names1"),
           py::arg("names2"), py::arg("allowed"))
      .def("set_entry", py::overload_cast<const S&, bool>(&ACM::set_entry), py::arg("name"), py::arg("allowed"))
      .def("set_entry", py::overload_cast<const VS&, bool>(&ACM::set_entry), py::arg("names"), py::arg("allowed"))
      .def("set_entry", py::overload_cast<bool>(&ACM::set_entry), py::arg("allowed"))
      .def("remove_entry", py::overload_cast<const S&, const S&>(&ACM::remove_entry), py::arg("name1"),
           py::arg("name2"))
      .def("remove_entry", py::overload_cast<const S&, const VS&>(&ACM::remove_entry), py::arg("name"),
           py::arg("other_names"))
      .def("remove_entry", py::overload_cast<const VS&, const VS&>(&ACM::remove_entry), py::arg("names1"),
           py::arg("names2"))
      .def("remove_entry", py::overload_cast<const S&>(&ACM::remove_entry), py::arg("name"))
      .def("remove_entry", py::overload_cast<const VS&>(&ACM::remove_entry), py::arg("names"))
      .def("__len__", &ACM::get_size)
      .def("get_default_entry", &ACM::get_default_entry, py::arg("name"))
      .def("has_default_entry", &ACM::has_default_entry, py::arg("name"))
      .def("set_default_entry", py::overload_cast<const S&, bool>(&ACM::set_default_entry), py::arg("name"),
           py::arg("allowed"))
      .def("set_default_entry", py::overload_cast<const VS&, bool>(&ACM::set_default_entry), py::arg("names"),
           py::arg("allowed"))
      .def("remove_default_entry", py::overload_cast<const S&>(&ACM::remove_default_entry), py::arg("name"))
      .def("remove_default_entry", py::overload_cast<const VS&>(&ACM::remove_default_entry), py::arg("names"))
      .def("get_allowed_collision", &ACM::get_allowed_collision, py::arg("name1"), py::arg("name2"))
      .def("clear", &ACM::clear)
      .def("get_all_entry_names", &ACM::get_all_entry_names)
      .def("__str__", &ACM::print);

  // -------------------------------------------------------- planning_world
  // -------------------------------------------------------- attached_body
  // python/pybind_attached_body.hpp:22-60.  get_pose / get_global_pose return
  // the 4x4 homogeneous matrix (the reference returns an Eigen::Transform,
  // for which its binding registers no converter).
  auto mab = m_all.def_submodule("attached_body");
  auto ab_cls =
      py::class_<AttachedBody, std::shared_ptr<AttachedBody>>(mab, "AttachedBody")
          .def(py::init([](const S& name, const ObjPtr& object, const ArtPtr& art, int link_id,
                           const std::vector<double>& pose, const VS& touch_links) {
                 if (!object || !art) throw std::invalid_argument("object and attached_articulation are required");
                 if (link_id < 0 || link_id >= (int)art->get_user_link_names().size())
                   throw std::out_of_range("attached_link_id out of range");
                 auto b = std::make_shared<AttachedBody>(
                     AttachedBody{name, object, art, link_id, se3_from_pose7(vec7_arg(pose)), touch_links});
                 b->update_pose();  // attached_body.cpp:22
                 return b;
               }),
               py::arg("name"), py::arg("object"), py::arg("attached_articulation"), py::arg("attached_link_id"),
               py::arg("pose"), py::arg("touch_links") = VS())
          .def("get_name", [](const AttachedBody& b) { return b.name; })
          .def("get_object", [](const AttachedBody& b) { return b.object; })
          .def("get_attached_articulation", [](const AttachedBody& b) { return b.articulation; })
          .def("get_attached_link_id", [](const AttachedBody& b) { return b.link_id; })
          .def("get_pose", [](const AttachedBody& b) { return mat4(b.pose); })
          .def(
              "set_pose",
              [](AttachedBody& b, const std::vector<double>& pose) { b.set_pose(se3_from_pose7(vec7_arg(pose))); },
              py::arg("pose"))
          .def("get_global_pose", [](const AttachedBody& b) { return mat4(b.global_pose()); })
          .def("update_pose", &AttachedBody::update_pose)
          .def("get_touch_links", [](const AttachedBody& b) { return b.touch_links; })
          .def("set_touch_links", [](AttachedBody& b, const VS& t) { b.touch_links = t; }, py::arg("touch_links"));

  auto mw = m_all.def_submodule("planning_world");
  mw.attr("AttachedBody") = ab_cls;

  py::class_<WorldCollisionResult, std::shared_ptr<WorldCollisionResult>>(mw, "WorldCollisionResult")
      .def(py::init<>())
      .def_readwrite("res", &WorldCollisionResult::res)
      .def_readwrite("collision_type", &WorldCollisionResult::collision_type)
      .def_readwrite("object_name1", &WorldCollisionResult::object_name1)
      .def_readwrite("object_name2", &WorldCollisionResult::object_name2)
      .def_readwrite("link_name1", &WorldCollisionResult::link_name1)
      .def_readwrite("link_name2", &WorldCollisionResult::link_name2);
  py::class_<WorldDistanceResult, std::shared_ptr<WorldDistanceResult>>(mw, "WorldDistanceResult")
      .def(py::init<>())
      .def_readwrite("res", &WorldDistanceResult::res)
      .def_readwrite("min_distance", &WorldDistanceResult::min_distance)
      .def_readwrite("distance_type", &WorldDistanceResult::distance_type)
      .def_readwrite("object_name1", &WorldDistanceResult::object_name1)
      .def_readwrite("object_name2", &WorldDistanceResult::object_name2)
      .def_readwrite("link_name1", &WorldDistanceResult::link_name1)
      .def_readwrite("link_name2", &WorldDistanceResult::link_name2);

  using PW = PlanningWorld;
  py::class_<PW, std::shared_ptr<PW>>(mw, "PlanningWorld")
      .def(py::init<const std::vector<ArtPtr>&, const VS&, const std::vector<ObjPtr>&, const VS&>(),
           py::arg("articulations"), py::arg("articulation_names"),
           py::arg("normal_objects") = std::vector<ObjPtr>(), py::arg("normal_object_names") = VS())
      .def("get_articulation_names", &PW::get_articulation_names)
      .def("get_planned_articulations", &PW::get_planned_articulations)
      .def("get_articulation", &PW::get_articulation, py::arg("name"))
      .def("has_articulation", &PW::has_articulation, py::arg("name"))
      .def("add_articulation", &PW::add_articulation, py::arg("name"), py::arg("model"), py::arg("planned") = false)
      .def("remove_articulation", &PW::remove_articulation, py::arg("name"))
      .def("is_articulation_planned", &PW::is_articulation_planned, py::arg("name"))
      .def("set_articulation_planned", &PW::set_articulation_planned, py::arg("name"), py::arg("planned"))
      .def("print_attached_body_pose", &PW::print_attached_body_pose)
      .def("get_normal_object_names", &PW::get_normal_object_names)
      .def("get_normal_object", &PW::get_normal_object, py::arg("name"))
      .def("has_normal_object", &PW::has_normal_object, py::arg("name"))
      .def("add_normal_object", &PW::add_normal_object, py::arg("name"), py::arg("collision_object"))
      .def("add_point_cloud",
           [](PW& w, const std::string& name, py::array_t<double, py::array::c_style | py::array::forcecast> v,
              double res) {
             if (v.ndim() != 2 || v.shape(1) != 3) throw std::invalid_argument("vertices must be [N, 3]");
             std::vector<Vec3> pts;
             auto a = v.unchecked<2>();
             for (ssize_t i = 0; i < v.shape(0); ++i) pts.push_back({a(i, 0), a(i, 1), a(i, 2)});
             w.add_point_cloud(name, pts, res);
           },
           py::arg("name"), py::arg("vertices"), py::arg("resolution") = 0.001)
      .def("remove_normal_object", &PW::remove_normal_object, py::arg("name"))
      .def("is_normal_object_attached", &PW::is_normal_object_attached, py::arg("name"))
      .def("get_attached_object", &PW::get_attached_object, py::arg("name"))
      .def("attach_object",
           [](PW& w, const S& n, const S& art, int link, const std::vector<double>& pose, const VS& touch) {
             w.attach_object(n, art, link, vec7_arg(pose), touch);
           },
           py::arg("name"), py::arg("art_name"), py::arg("link_id"), py::arg("pose"), py::arg("touch_links"))
      .def("attach_object",
           [](PW& w, const S& n, const S& art, int link, const std::vector<double>& pose) {
             w.attach_object(n, art, link, vec7_arg(pose));
           },
           py::arg("name"), py::arg("art_name"), py::arg("link_id"), py::arg("pose"))
      .def("attach_object",
           [](PW& w, const S& n, const GeomPtr& g, const S& art, int link, const std::vector<double>& pose,
              const VS& touch) { w.attach_object(n, g, art, link, vec7_arg(pose), touch); },
           py::arg("name"), py::arg("p_geom"), py::arg("art_name"), py::arg("link_id"), py::arg("pose"),
           py::arg("touch_links"))
      .def("attach_object",
           [](PW& w, const S& n, const GeomPtr& g, const S& art, int link, const std::vector<double>& pose) {
             w.attach_object(n, g, art, link, vec7_arg(pose));
           },
           py::arg("name"), py::arg("p_geom"), py::arg("art_name"), py::arg("link_id"), py::arg("pose"))
      .def("attach_sphere",
           [](PW& w, double r, const S& art, int link, const std::vector<double>& pose) {
             w.attach_sphere(r, art, link, vec7_arg(pose));
           },
           py::arg("radius"), py::arg("art_name"), py::arg("link_id"), py::arg("pose"))
      .def("attach_box",
           [](PW& w, const std::vector<double>& size, const S& art, int link, const std::vector<double>& pose) {
             w.attach_box(vec3_arg(size), art, link, vec7_arg(pose));
           },
           py::arg("size"), py::arg("art_name"), py::arg("link_id"), py::arg("pose"))
      .def("attach_mesh",
           [](PW& w, const S& path, const S& art, int link, const std::vector<double>& pose) {
             w.attach_mesh(path, art, link, vec7_arg(pose));
           },
           py::arg("mesh_path"), py::arg("art_name"), py::arg("link_id"), py::arg("pose"))
      .def("detach_object", &PW::detach_object, py::arg("name"), py::arg("also_remove") = false)
      .def("set_qpos", &PW::set_qpos, py::arg("name"), py::arg("qpos"))
      .def("set_qpos_all", &PW::set_qpos_all, py::arg("state"))
      .def("get_allowed_collision_matrix", &PW::get_allowed_collision_matrix)
      .def("collide", &PW::collide, py::arg("request") = CollisionRequest())
      .def("self_collide", &PW::self_collide, py::arg("request") = CollisionRequest())
      .def("collide_with_others", &PW::collide_with_others, py::arg("request") = CollisionRequest())
      .def("collide_full", &PW::collide_full, py::arg("request") = CollisionRequest())
      .def("distance", &PW::distance, py::arg("request") = DistanceRequest())
      .def("self_distance", &PW::self_distance, py::arg("request") = DistanceRequest())
      .def("distance_with_others", &PW::distance_with_others, py::arg("request") = DistanceRequest())
      .def("distance_full", &PW::distance_full, py::arg("request") = DistanceRequest())
      .def("distance_batch",
           [](PW& w, py::array_t<double, py::array::c_style | py::array::forcecast> states, py::object request,
              bool nearest_points) -> py::tuple {
             const int dim = w.state_dim();
             if (states.ndim() != 2 || states.shape(1) != dim)
               throw std::invalid_argument("states must be [N, " + std::to_string(dim) + "] float64");
             DistanceRequest r;
             if (!request.is_none()) r = request.cast<const DistanceRequest&>();
             r.check_supported();
             const int32_t flags = r.flags();
             const int64_t n = states.shape(0);
             py::array_t<double> ds(n), dot(n);
             py::array_t<int32_t> ps(n), po(n);
             const double* q = states.data();
             double *a = ds.mutable_data(), *b = dot.mutable_data();
             int32_t *c = ps.mutable_data(), *d = po.mutable_data();
             if (!nearest_points && flags == 0 && r.distance_tolerance == 1e-6) {
               {
                 py::gil_scoped_release rel;
                 w.distance_batch(q, n, a, c, b, d);
               }
               return py::tuple(py::make_tuple(ds, ps, dot, po));
             }
             py::array_t<double> qs({n, (int64_t)6}), qo({n, (int64_t)6});
             double *e = qs.mutable_data(), *f = qo.mutable_data();
             {
               py::gil_scoped_release rel;
               w.distance_batch_ex(q, n, r, a, c, e, b, d, f);
             }
             return py::tuple(py::make_tuple(ds, ps, dot, po, qs, qo));
           },
           py::arg("states"), py::arg("request") = py::none(), py::arg("nearest_points") = false,
           "Batched self_distance / distance_with_others: (d_self[N], pair_self[N], d_others[N], pair_others[N]); "
           "-1 = a penetrating pair, pair indices into get_collision_pair_info().  With a DistanceRequest "
           "(enable_signed_distance: -penetration depth instead of -1; distance_tolerance) or nearest_points=True, "
           "also DistanceResult.nearest_points of each group's minimum pair: (..., pts_self[N, 6], pts_others[N, 6]) "
           "(include/mpgpu.h mpg_distance_batch_req: which point is which).")
      // ---- batched validity (new; one device launch for N states) ----
      .def("sample_pair_counts",
           [](PW& w, int64_t n, uint64_t seed) {
             std::vector<int64_t> c;
             {
               py::gil_scoped_release rel;
               c = w.sample_pair_counts(n, seed);
             }
             return c;
           },
           py::arg("n"), py::arg("seed") = 0,
           "Planner.generate_collision_pair batched: per pair of get_collision_pair_info(), how many of n random "
           "full configurations (every joint of the planned articulations, uniform in the joint limits, drawn on "
           "the device) report it in collide_full().")
      .def("get_full_state_limits",
           [](PW& w) { return w.full_state_limits(); },
           "(lower, upper) of the full state sample_pair_counts draws from.")
      .def("get_state_dim", &PW::state_dim)
      .def("get_mask_words", &PW::mask_words)
      .def("get_collision_pair_info",
           [](PW& w) {
             py::list out;
             for (auto& p : w.pair_table())
               out.append(py::make_tuple(p.collision_type, p.object_name1, p.object_name2, p.link_name1,
                                         p.link_name2, p.allowed, p.self));
             return out;
           })
      .def("collide_batch",
           [](PW& w, py::array_t<double, py::array::c_style | py::array::forcecast> states) {
             const int dim = w.state_dim();
             if (states.ndim() != 2 || states.shape(1) != dim)
               throw std::invalid_argument("states must be [N, " + std::to_string(dim) + "] float64");
             const int64_t n = states.shape(0);
             const int W = w.mask_words();
             py::array_t<uint8_t> flags(n);
             py::array_t<uint32_t> masks({(ssize_t)n, (ssize_t)W});
             const double* q = states.data();
             uint8_t* f = flags.mutable_data();
             uint32_t* mk = masks.mutable_data();
             {
               py::gil_scoped_release rel;
               w.collide_batch(q, n, f, mk);
             }
             return py::make_tuple(flags, masks);
           },
           py::arg("states"),
           "Batched collide(): flags[i] = collide() at states[i]; bit p of masks[i] = pair p reported by "
           "collide_full() (see get_collision_pair_info()).")
      .def("collide_batch_device",
           [](PW& w, uintptr_t q, int64_t n, uintptr_t flags, uintptr_t masks, uintptr_t stream) {
             w.collide_batch_device(reinterpret_cast<const void*>(q), n, reinterpret_cast<void*>(flags),
                                    reinterpret_cast<void*>(masks), reinterpret_cast<void*>(stream));
           },
           py::arg("states_ptr"), py::arg("n"), py::arg("flags_ptr"), py::arg("masks_ptr") = 0,
           py::arg("stream") = 0,
           "Enqueue the batched check on device buffers (float64 [n, dim], uint8 [n], uint32 [n, W]).")
      .def("distance_batch_device",
           [](PW& w, uintptr_t q, int64_t n, uintptr_t d_self, uintptr_t p_self, uintptr_t d_others,
              uintptr_t p_others, uintptr_t pts_self, uintptr_t pts_others, uintptr_t stream,
              std::optional<DistanceRequest> request) {
             const DistanceRequest r = request ? *request : DistanceRequest();
             w.distance_batch_device(reinterpret_cast<const void*>(q), n, r, reinterpret_cast<void*>(d_self),
                                     reinterpret_cast<void*>(p_self), reinterpret_cast<void*>(pts_self),
                                     reinterpret_cast<void*>(d_others), reinterpret_cast<void*>(p_others),
                                     reinterpret_cast<void*>(pts_others), reinterpret_cast<void*>(stream));
           },
           py::arg("states_ptr"), py::arg("n"), py::arg("d_self_ptr"), py::arg("p_self_ptr"),
           py::arg("d_others_ptr"), py::arg("p_others_ptr"), py::arg("pts_self_ptr") = 0,
           py::arg("pts_others_ptr") = 0, py::arg("stream") = 0, py::arg("request") = py::none(),
           "Enqueue distance_batch on device buffers (float64 [n, dim] -> float64 [n], int32 [n] per group, "
           "optional float64 [n, 6] nearest points).  No error is raised for a configuration where FCL throws: "
           "it gets NaN distances and pair index -2 (MPG_DISTANCE_FCL_THROWS) in both groups, or -3 "
           "(MPG_DISTANCE_EPA_CAPACITY) when the EPA polytope outgrew the device; check p < -1 before indexing "
           "the pair table (mplib_amd.dist.distance_sharded_device does).")
      .def("check_motion_batch",
           [](PW& w, py::array_t<double, py::array::c_style | py::array::forcecast> q_from,
              py::array_t<double, py::array::c_style | py::array::forcecast> q_to, double fraction, double lvs) {
             const int dim = w.state_dim();
             if (q_from.ndim() != 2 || q_from.shape(1) != dim || q_to.ndim() != 2 || q_to.shape(1) != dim ||
                 q_to.shape(0) != q_from.shape(0))
               throw std::invalid_argument("q_from / q_to must both be [N, " + std::to_string(dim) + "] float64");
             if (lvs <= 0.0) lvs = fraction * w.motion_space().max_extent;
             const int64_t n = q_from.shape(0);
             py::array_t<bool> valid(n);
             py::array_t<int32_t> first(n), segs(n);
             const double* a = q_from.data();
             const double* b = q_to.data();
             uint8_t* v = reinterpret_cast<uint8_t*>(valid.mutable_data());
             int32_t* f = first.mutable_data();
             int32_t* sg = segs.mutable_data();
             {
               py::gil_scoped_release rel;
               w.check_motion_batch(a, b, n, lvs, v, f, sg);
             }
             return py::make_tuple(valid, first, segs);
           },
           py::arg("q_from"), py::arg("q_to"), py::arg("longest_valid_segment_fraction") = 0.01,
           py::arg("longest_valid_segment") = 0.0,
           "Batched OMPL DiscreteMotionValidator::checkMotion over the planner's state space: returns (valid[N], "
           "first_invalid[N] (1-based state index along the edge, -1 if valid), segments[N]). The longest valid "
           "segment defaults to fraction * the space's maximum extent, as OMPL's SpaceInformation does.")
      .def("get_motion_space",
           [](PW& w) {
             auto ms = w.motion_space();
             return py::make_tuple(ms.so2_mask, ms.max_extent);
           },
           "(so2_mask, maximum_extent) of the planner state space (src/ompl_planner.cpp:248-293).")
      .def("set_small_batch_max", &PW::set_small_batch_max, py::arg("n"),
           "Host-buffer batches of at most n states run as one launch (latency path, default 1024); 0 always "
           "uses the throughput pipeline. Results are identical.")
      .def("profile_enable", &PW::profile_enable, py::arg("enable") = true,
           "Record HIP events around each device stage of the batched check (diagnostics).")
      .def("profile_read",
           [](PW& w) {
             static const char* names[MPG_NUM_STAGES] = {"cull", "bucket", "narrow"};
             py::dict d;
             auto v = w.profile_read();
             for (int k = 0; k < MPG_NUM_STAGES; ++k) d[names[k]] = py::make_tuple(v[k].ms, v[k].launches, v[k].units);
             return d;
           },
           "{stage: (milliseconds, launches, units)} accumulated since the last read; units are configurations "
           "(cull, bucket) or narrow-phase candidates (narrow).")
      .def("device_handle",
           [](PW& w) { return reinterpret_cast<uintptr_t>(w.device_world()); },
           "The mpg_world* of the current snapshot (include/mpgpu.h), e.g. for mpg_collide_batch_multi_device; valid "
           "until the world changes (a mutation rebuilds the snapshot).  The device is MPLIB_AMD_DEVICE / LOCAL_RANK "
           "(default 0) when the snapshot is built.")
      .def("latency_server_stats",
           [](PW& w) {
             int64_t served = 0, starts = 0, fallbacks = 0;
             int32_t state = 0;
             check_status(mpg_latency_server_stats(w.device_world(), &served, &starts, &fallbacks, &state),
                          "mpg_latency_server_stats");
             static const char* names[3] = {"unused", "in_use", "fallen_back"};
             py::dict d;
             d["served"] = served;
             d["starts"] = starts;
             d["fallbacks"] = fallbacks;
             d["state"] = names[state];
             return d;
           },
           "Latency server accounting of the current snapshot (mpg_latency_server_stats): batches served, "
           "(re)starts, fallbacks to one launch per batch, state.");

  // ---- ompl (reference python/pybind_ompl.hpp:20-33) ----
  auto mo = m_all.def_submodule("ompl");
  // ValidityCheckerTpl (src/ompl_planner.h:54-81): isValid / clearance of one
  // state through the world (which they leave at that state), and batched
  // twins that leave the world alone (one device launch for N states)
  struct ValidityChecker {
    std::shared_ptr<PW> world;
  };
  auto states_arg = [](PW& w, const py::array_t<double, py::array::c_style | py::array::forcecast>& st) {
    const int dim = w.state_dim();
    if (st.ndim() != 2 || st.shape(1) != dim)
      throw std::invalid_argument("states must be [N, " + std::to_string(dim) + "] float64");
    return (int64_t)st.shape(0);
  };
  py::class_<ValidityChecker, std::shared_ptr<ValidityChecker>>(mo, "ValidityChecker")
      .def(py::init([](const std::shared_ptr<PW>& w) { return std::make_shared<ValidityChecker>(ValidityChecker{w}); }),
           py::arg("world"))
      .def("is_valid",
           [](ValidityChecker& v, const std::vector<double>& state) {
             v.world->set_qpos_all(state);
             return !v.world->collide();
           },
           py::arg("state"), "setQposAll(state); !collide()  (ompl_planner.h:59-62)")
      .def("clearance",
           [](ValidityChecker& v, const std::vector<double>& state) {
             v.world->set_qpos_all(state);
             return v.world->distance();
           },
           py::arg("state"),
           "setQposAll(state); distance(): the distance to the nearest invalid state, -1 in collision "
           "(ompl_planner.h:69-72, planning_world.h:271-273)")
      .def("is_valid_batch",
           [states_arg](ValidityChecker& v, py::array_t<double, py::array::c_style | py::array::forcecast> states) {
             const int64_t n = states_arg(*v.world, states);
             std::vector<uint8_t> fl((size_t)n);
             std::vector<uint32_t> mk((size_t)n * (size_t)std::max(v.world->mask_words(), 1));
             {
               py::gil_scoped_release rel;
               v.world->collide_batch(states.data(), n, fl.data(), mk.data());
             }
             py::array_t<bool> out(n);
             for (int64_t i = 0; i < n; ++i) out.mutable_data()[i] = fl[(size_t)i] == 0;
             return out;
           },
           py::arg("states"))
      .def("clearance_batch",
           [states_arg](ValidityChecker& v, py::array_t<double, py::array::c_style | py::array::forcecast> states) {
             const int64_t n = states_arg(*v.world, states);
             std::vector<double> ds((size_t)n), dot((size_t)n);
             std::vector<int32_t> ps((size_t)n), po((size_t)n);
             {
               py::gil_scoped_release rel;
               v.world->distance_batch(states.data(), n, ds.data(), ps.data(), dot.data(), po.data());
             }
             py::array_t<double> out(n);
             for (int64_t i = 0; i < n; ++i)  // distanceFull: the smaller group minimum (planning_world.cpp:718-719)
               out.mutable_data()[i] = ds[(size_t)i] < dot[(size_t)i] ? ds[(size_t)i] : dot[(size_t)i];
             return out;
           },
           py::arg("states"),
           "clearance() of N states in one device launch (MaximizeMinClearanceObjective's query, "
           "ompl_planner.cpp:180-186), world state untouched");
  py::class_<OMPLPlanner, std::shared_ptr<OMPLPlanner>>(mo, "OMPLPlanner")
      .def(py::init([](const std::shared_ptr<PW>& world, py::object checker) {
             auto p = std::make_shared<OMPLPlanner>(world);
             if (!checker.is_none()) {
               // a Python validity checker: f(states[n, dim] float64) -> valid[n]
               auto fn = std::make_shared<py::object>(checker);
               const int dim = (int)p->get_dim();
               p->set_state_validity_checker([fn, dim](const double* st, int64_t n, uint8_t* valid) {
                 py::gil_scoped_acquire acq;
                 py::array_t<double> a({(ssize_t)n, (ssize_t)dim});
                 std::copy(st, st + n * dim, a.mutable_data());
                 auto r = py::array_t<bool, py::array::c_style | py::array::forcecast>((*fn)(a));
                 if (r.size() != n) throw std::runtime_error("state_validity_checker returned a wrong length");
                 const bool* v = r.data();
                 for (int64_t i = 0; i < n; ++i) valid[i] = v[i] ? 1 : 0;
               });
             }
             return p;
           }),
           py::arg("world"), py::arg("state_validity_checker") = py::none(),
           "OMPL planner over the planned articulations' move-group joints. State validity runs as batched "
           "device collide() calls; state_validity_checker (f(states[n, dim]) -> valid[n]) replaces it.")
      .def("set_native_state_validity_checker",
           [](OMPLPlanner& p, uintptr_t fn, uintptr_t ctx) {
             // a C validity checker: int fn(void* ctx, const double* states, int64_t n, uint8_t* valid)
             // (0 = ok), called without Python in the loop, as OMPL calls a C++ StateValidityChecker
             using Fn = int (*)(void*, const double*, int64_t, uint8_t*);
             if (!fn) throw std::invalid_argument("null checker");
             Fn f = reinterpret_cast<Fn>(fn);
             void* c = reinterpret_cast<void*>(ctx);
             p.set_state_validity_checker([f, c](const double* st, int64_t n, uint8_t* valid) {
               if (f(c, st, n, valid) != 0) throw std::runtime_error("native state validity checker failed");
             });
           },
           py::arg("fn_address"), py::arg("ctx_address"),
           "Replace the device checker by a C function int fn(ctx, states[n*dim], n, valid[n]) (0 = ok).")
      .def("get_world", &OMPLPlanner::get_world)
      .def("set_speculative_connect", &OMPLPlanner::set_speculative_connect, py::arg("enable") = true,
           "RRTConnect: validate the blocked motion plus the explored outcome tree of the loop's future in one "
           "batch (default), or one batch per growTree call as OMPL's loop is written (same tree, more round "
           "trips).")
      .def("get_speculative_connect", &OMPLPlanner::get_speculative_connect)
      .def("set_speculation_nodes", &OMPLPlanner::set_speculation_nodes, py::arg("n"),
           "Outcome-tree nodes explored before each validity batch is sent (-1: 16 on the device path, which "
           "keeps exploring while the batch runs, 64 with a custom checker); 0 sends only what is already "
           "explored.")
      .def("get_speculation_nodes", &OMPLPlanner::get_speculation_nodes)
      .def("get_dim", &OMPLPlanner::get_dim)
      .def("random_sample_nearby",
           [](OMPLPlanner& p, const std::vector<double>& s) { auto v = p.random_sample_nearby(s); return vec(v.data(), (int)v.size()); },
           py::arg("start_state"))
      .def("plan",
           [](OMPLPlanner& p, const std::vector<double>& start, const std::vector<std::vector<double>>& goals,
              const std::string& name, double time, double range, double goal_bias, double w, bool only,
              bool verbose) {
             std::pair<std::string, std::vector<std::vector<double>>> r;
             {
               py::gil_scoped_release rel;
               r = p.plan(start, goals, name, time, range, goal_bias, w, only, verbose);
             }
             const ssize_t dim = (ssize_t)p.get_dim();
             py::array_t<double> path({(ssize_t)r.second.size(), dim});
             auto m = path.mutable_unchecked<2>();
             for (ssize_t i = 0; i < (ssize_t)r.second.size(); ++i)
               for (ssize_t j = 0; j < dim; ++j) m(i, j) = r.second[(size_t)i][(size_t)j];
             return py::make_tuple(r.first, path);
           },
           py::arg("start_state"), py::arg("goal_states"), py::arg("planner_name") = "RRTConnect",
           py::arg("time") = 1.0, py::arg("range") = 0.0, py::arg("goal_bias") = 0.05,
           py::arg("pathlen_obj_weight") = 10.0, py::arg("pathlen_obj_only") = false, py::arg("verbose") = false,
           "Plan from start_state to any of goal_states (+-2pi variants of revolute joints are added); returns "
           "(status, path[len, dim]). RRTConnect (speculative batches, see set_speculative_connect) and RRT.")
      .def("get_last_plan_stats",
           [](OMPLPlanner& p) {
             const auto& s = p.last_stats();
             py::dict d;
             d["iterations"] = s.iterations;
             d["ext_trapped"] = s.ext_trapped;
             d["batches"] = s.batches;
             d["states_checked"] = s.states_checked;
             d["start_tree"] = s.start_tree;
             d["goal_tree"] = s.goal_tree;
             d["seconds"] = s.seconds;
             d["check_seconds"] = s.check_seconds;
             d["spec_nodes"] = s.spec_nodes;
             d["spec_wait_nodes"] = s.spec_wait_nodes;
             d["spec_resets"] = s.spec_resets;
             d["t_spec_wait"] = s.t_spec_wait;
             d["t_spec"] = s.t_spec;
             return d;
           },
           "Counters of the last plan(): iterations, validity batches, states checked, tree sizes, seconds.")
      .def("get_state_space",
           [](OMPLPlanner& p) {
             const auto& s = p.space();
             return py::make_tuple(s.lo, s.hi, s.so2, s.revolute, s.max_extent, s.longest_valid_segment);
           },
           "(lower, upper, so2, is_revolute, maximum_extent, longest_valid_segment) of the compound state space.");
}
