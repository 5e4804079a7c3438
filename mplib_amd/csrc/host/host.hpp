// host.hpp -- C++ host side of mplib_amd.  Mirrors the object model of
// MPlib's pybind module ``mplib.pymp`` (reference python/pybind*.hpp) so that
// user code written against the reference keeps working, while every
// kinematics / collision evaluation is executed by the HIP library through
// the C ABI in include/mpgpu.h.  There is no CPU evaluation path: if the
// device library cannot run, calls raise.
#pragma once

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../../include/mpgpu.h"
#include "../mpg_math.h"

namespace mpgh {

using mpg::SE3;
using Vec3 = std::array<double, 3>;
using Vec7 = std::array<double, 7>;  // (px, py, pz, qw, qx, qy, qz)

// ---------------------------------------------------------------------------
// FCL-like geometry and collision objects (reference python/pybind_fcl.hpp)
// ---------------------------------------------------------------------------
struct CollisionGeometry {
  int type = -1;  // MPG_GEOM_*, or -1 for geometry the device does not support
  std::string kind;
  // fcl::CollisionGeometry's bookkeeping (python/pybind_fcl.hpp:67-82):
  // computeLocalAABB sets aabb_center / aabb_radius (CollisionObject's
  // constructor calls it); cost_density against the occupancy thresholds
  Vec3 aabb_center{0, 0, 0};
  double aabb_radius = 0.0;
  double cost_density = 1.0, threshold_occupied = 1.0, threshold_free = 0.0;
  virtual ~CollisionGeometry() = default;
};
struct Box : CollisionGeometry {
  Vec3 side;
  explicit Box(const Vec3& s) : side(s) { type = MPG_GEOM_BOX; kind = "Box"; }
};
struct Sphere : CollisionGeometry {
  double radius;
  explicit Sphere(double r) : radius(r) { type = MPG_GEOM_SPHERE; kind = "Sphere"; }
};
struct Capsule : CollisionGeometry {
  double radius, lz;
  Capsule(double r, double l) : radius(r), lz(l) { type = MPG_GEOM_CAPSULE; kind = "Capsule"; }
};
struct Cylinder : CollisionGeometry {
  double radius, lz;
  Cylinder(double r, double l) : radius(r), lz(l) { type = MPG_GEOM_CYLINDER; kind = "Cylinder"; }
};
struct Ellipsoid : CollisionGeometry {
  Vec3 radii;
  explicit Ellipsoid(const Vec3& r) : radii(r) { type = MPG_GEOM_ELLIPSOID; kind = "Ellipsoid"; }
};
struct Cone : CollisionGeometry {
  double radius, lz;
  Cone(double r, double l) : radius(r), lz(l) { type = MPG_GEOM_CONE; kind = "Cone"; }
};
struct TriangleP : CollisionGeometry {
  Vec3 a, b, c;
  TriangleP(const Vec3& a_, const Vec3& b_, const Vec3& c_) : a(a_), b(b_), c(c_) {
    type = MPG_GEOM_TRIANGLE;
    kind = "TriangleP";
  }
};
// fcl::Halfspace / fcl::Plane (python/pybind_fcl.hpp:143-161): n . x <= d /
// n . x = d, the normal made unit by the constructor (unitNormalTest).  No
// device evaluation (type -1): the reference's own scene conversion leaves
// them out over wrong FCL halfspace checks (mplib/sapien_utils/conversion.py:384-396)
struct PlaneLike : CollisionGeometry {
  Vec3 n;
  double d;
  PlaneLike(const Vec3& n_, double d_, const char* k) : n(n_), d(d_) {
    kind = k;
    const double l = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    if (l > 0) {
      const double inv = 1.0 / l;
      for (double& x : n) x *= inv;
      d *= inv;
    } else {
      n = {1.0, 0.0, 0.0};
      d = 0.0;
    }
  }
  double signed_distance(const Vec3& p) const { return n[0] * p[0] + n[1] * p[1] + n[2] * p[2] - d; }
};
struct Halfspace : PlaneLike {
  Halfspace(const Vec3& n_, double d_) : PlaneLike(n_, d_, "Halfspace") {}
};
struct Plane : PlaneLike {
  Plane(const Vec3& n_, double d_) : PlaneLike(n_, d_, "Plane") {}
};
struct Convex : CollisionGeometry {
  std::vector<Vec3> vertices;
  std::vector<int> faces;  // FCL layout: n, i0..i(n-1), n, ...
  int num_faces = 0;
  Convex(std::vector<Vec3> v, int nf, std::vector<int> f)
      : vertices(std::move(v)), faces(std::move(f)), num_faces(nf) {
    type = MPG_GEOM_CONVEX;
    kind = "Convex";
    if (vertices.empty()) throw std::invalid_argument("Convex needs at least one vertex");
  }
  // FCL 0.7.0 Convex::interior_point_ = (sum of vertices) * (1.0 / n)
  Vec3 interior_point() const {
    double s[3] = {0, 0, 0};
    for (auto& v : vertices) {
      s[0] += v[0];
      s[1] += v[1];
      s[2] += v[2];
    }
    const double inv = 1.0 / (double)vertices.size();
    return {s[0] * inv, s[1] * inv, s[2] * inv};
  }
};
// fcl::OcTree built from a point cloud (octree.cpp): the occupied leaves as
// [min xyz, max xyz] boxes in the octree frame
struct OcTree : CollisionGeometry {
  double resolution;
  std::vector<std::array<double, 6>> leaves;
  explicit OcTree(double res);
  OcTree(const std::vector<Vec3>& points, double res);
};
// fcl::BVHModel<OBBRSS> of a triangle mesh (load_mesh_as_BVH,
// src/urdf_utils.cpp:136-155): vertices and triangles as loaded
struct BVHModel : CollisionGeometry {
  std::vector<Vec3> vertices;
  std::vector<std::array<int, 3>> triangles;
  bool building = false;  // between beginModel and endModel
  BVHModel() {
    type = MPG_GEOM_MESH;
    kind = "BVHModel";
  }
  BVHModel(std::vector<Vec3> v, std::vector<std::array<int, 3>> t) : BVHModel() { add_sub_model(v, t); }
  // fcl BVHModel::addSubModel: vertices appended, triangle indices offset by
  // the vertices already present
  void add_sub_model(const std::vector<Vec3>& v, const std::vector<std::array<int, 3>>& t) {
    const int off = (int)vertices.size();
    for (auto& tr : t)
      for (int k : tr)
        if (k < 0 || k >= (int)v.size()) throw std::invalid_argument("BVHModel: triangle index out of range");
    vertices.insert(vertices.end(), v.begin(), v.end());
    for (auto& tr : t) triangles.push_back({tr[0] + off, tr[1] + off, tr[2] + off});
  }
};
// geometry kinds the reference binds that the device cannot evaluate yet
struct UnsupportedGeometry : CollisionGeometry {
  explicit UnsupportedGeometry(const std::string& k) { kind = k; }
};

using GeomPtr = std::shared_ptr<CollisionGeometry>;

// FCL 0.7.0's mass properties and local bounding box of a geometry
// (geomprops.cpp): computeLocalAABB, computeVolume, computeCOM,
// computeMomentofInertia[RelatedToCOM]
struct LocalAABB {
  Vec3 min, max;
};
LocalAABB local_aabb(const CollisionGeometry& g);
void compute_local_aabb(CollisionGeometry& g);
double compute_volume(const CollisionGeometry& g);
Vec3 compute_com(const CollisionGeometry& g);
std::array<double, 9> compute_moment_of_inertia(const CollisionGeometry& g);
std::array<double, 9> compute_moment_of_inertia_com(const CollisionGeometry& g);

struct CollisionObject {
  GeomPtr geom;
  SE3 tf;
  uint64_t version = 0;
  // fcl::CollisionObject's constructor calls cgeom->computeLocalAABB()
  CollisionObject(GeomPtr g, const SE3& t) : geom(std::move(g)), tf(t) {
    if (geom) compute_local_aabb(*geom);
  }
  void set_transform(const SE3& t) {
    tf = t;
    ++version;
  }
};
using ObjPtr = std::shared_ptr<CollisionObject>;

SE3 se3_from_pose7(const Vec7& pose);  // posevec_to_transform (src/math_utils.cpp:12-18)
SE3 se3_from_pq(const Vec3& p, const std::array<double, 4>& wxyz);

enum GJKSolverType { GST_LIBCCD = 0, GST_INDEP = 1 };

struct CollisionRequest {
  size_t num_max_contacts = 1;
  bool enable_contact = false;
  size_t num_max_cost_sources = 1;
  bool enable_cost = false;
  bool use_approximate_cost = true;
  GJKSolverType gjk_solver_type = GST_LIBCCD;
  double gjk_tolerance = 1e-6;
  // Validates that the device path computes exactly what fcl::collide would.
  void check_supported() const;
};

// fcl::DistanceRequest / DistanceResult (python/pybind_fcl.hpp:306-325)
struct DistanceRequest {
  bool enable_nearest_points = false;
  bool enable_signed_distance = false;
  double rel_err = 0.0, abs_err = 0.0, distance_tolerance = 1e-6;
  GJKSolverType gjk_solver_type = GST_LIBCCD;
  // GST_INDEP: FCL's own GJK, unsigned only (enable_signed_distance raises)
  void check_supported() const;
  // MPG_DISTANCE_* flags of the C ABI
  int32_t flags() const;
  mpg_distance_request to_c() const;
};
struct DistanceResult {
  double min_distance = std::numeric_limits<double>::max();
  std::array<Vec3, 2> nearest_points{};
  void clear() { min_distance = std::numeric_limits<double>::max(); }
};

struct Contact {
  std::shared_ptr<CollisionGeometry> o1, o2;
  int b1 = -1, b2 = -1;
  Vec3 normal{0, 0, 0}, pos{0, 0, 0};
  double penetration_depth = 0;
};

// fcl::ContactPoint / fcl::CostSource (python/pybind_fcl.hpp:340-359)
struct ContactPoint {
  Vec3 normal{0, 0, 0}, pos{0, 0, 0};
  double penetration_depth = 0;
};
struct CostSource {
  Vec3 aabb_min{0, 0, 0}, aabb_max{0, 0, 0};
  double cost_density = 0, total_cost = 0;
  // CostSource(aabb_min, aabb_max, cost_density): total_cost = density x box volume
  CostSource() = default;
  CostSource(const Vec3& lo, const Vec3& hi, double d) : aabb_min(lo), aabb_max(hi), cost_density(d) {
    total_cost = d * (hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]);
  }
  // the std::set order of CollisionResult::cost_sources: larger total cost
  // first, then aabb_min, aabb_max (lexicographic), cost_density
  bool operator<(const CostSource& o) const {
    if (total_cost != o.total_cost) return total_cost > o.total_cost;
    if (aabb_min != o.aabb_min) return aabb_min < o.aabb_min;
    if (aabb_max != o.aabb_max) return aabb_max < o.aabb_max;
    return cost_density < o.cost_density;
  }
};

struct CollisionResult {
  std::vector<Contact> contacts;
  std::vector<CostSource> cost_sources;  // kept sorted (CostSource::operator<), no duplicates
  bool is_collision() const { return !contacts.empty(); }
  size_t num_contacts() const { return contacts.size(); }
  size_t num_cost_sources() const { return cost_sources.size(); }
  void add_contact(const Contact& c) { contacts.push_back(c); }
  // CollisionResult::addCostSource: insert into the ordered set, then drop
  // the last entries beyond num_max
  void add_cost_source(const CostSource& c, size_t num_max) {
    auto it = std::lower_bound(cost_sources.begin(), cost_sources.end(), c);
    if (it == cost_sources.end() || c < *it) cost_sources.insert(it, c);
    while (cost_sources.size() > num_max) cost_sources.pop_back();
  }
  void clear() {
    contacts.clear();
    cost_sources.clear();
  }
};

// ---------------------------------------------------------------------------
// URDF / SRDF / mesh ingestion (urdfdom 4.0.0 + assimp 5.3.1 semantics)
// ---------------------------------------------------------------------------
struct UrdfGeometry {
  enum Kind { MESH, BOX, SPHERE, CYLINDER } kind = BOX;
  std::string filename;
  Vec3 scale{1, 1, 1};
  Vec3 size{0, 0, 0};
  double radius = 0, length = 0;
};
struct UrdfPose {
  Vec3 xyz{0, 0, 0};
  std::array<double, 4> quat{0, 0, 0, 1};  // x y z w (urdf::Rotation)
  SE3 se3() const;
};
struct UrdfLink {
  std::string name;
  std::vector<std::pair<UrdfPose, UrdfGeometry>> collisions;
  std::string parent, parent_joint;
  std::vector<std::string> children;
};
struct UrdfJoint {
  std::string name, type, parent, child;
  UrdfPose origin;
  Vec3 axis{1, 0, 0};
  bool has_limits = false;
  double lower = 0, upper = 0;
};
struct UrdfModel {
  std::string name, root, directory;
  std::map<std::string, UrdfLink> links;
  std::map<std::string, UrdfJoint> joints;
};

UrdfModel parse_urdf_string(const std::string& xml, const std::string& directory = "");
UrdfModel parse_urdf_file(const std::string& path);
std::vector<std::pair<std::string, std::string>> parse_srdf_disabled_pairs(const std::string& xml);
std::string read_file(const std::string& path);

struct MeshData {
  std::vector<Vec3> vertices;             // assimp float values promoted to double
  std::vector<std::array<int, 3>> faces;  // after JoinIdenticalVertices
};
MeshData load_stl(const std::string& path);
std::shared_ptr<Convex> load_mesh_as_convex(const std::string& path, const Vec3& scale);
std::shared_ptr<BVHModel> load_mesh_as_bvh(const std::string& path, const Vec3& scale);

// ---------------------------------------------------------------------------
// device world handle (RAII over mpg_world)
// ---------------------------------------------------------------------------
struct DescBuilder;  // plain arrays -> mpg_world_desc

class DeviceWorld {
 public:
  DeviceWorld(const DescBuilder& d, int device);
  ~DeviceWorld();
  DeviceWorld(const DeviceWorld&) = delete;
  DeviceWorld& operator=(const DeviceWorld&) = delete;
  mpg_world* get() const { return w_; }
  const mpg_world_info& info() const { return info_; }

 private:
  mpg_world* w_ = nullptr;
  mpg_world_info info_{};
};

void check_status(int rc, const char* what);
// copy pair p's contact (mpg_collide_contacts layout) into c
void fill_contacts(const uint32_t* mask, size_t n_pairs, const std::vector<double>& depth,
                   const std::vector<double>& normal, const std::vector<double>& pos, size_t p, Contact& c);
int default_device();

struct DescBuilder {
  std::vector<int32_t> joint_type, joint_parent, joint_q_source;
  std::vector<double> joint_axis, joint_placement, joint_q_const;
  std::vector<double> joint_lower, joint_upper;  // getJointLimit (first coordinate; +-inf for continuous)
  int32_t dof = 0;
  std::vector<int32_t> link_parent;
  std::vector<double> link_placement;
  std::vector<int32_t> geom_type, geom_vertex_start, geom_vertex_count;
  std::vector<double> geom_param, vertices, octree_leaf;
  std::vector<int32_t> mesh_triangle;
  std::vector<int32_t> convex_face;  // FCL layout faces of the convex geometries
  std::vector<int32_t> moving_link, moving_geom;
  std::vector<double> moving_offset;
  std::vector<int32_t> static_geom;
  std::vector<double> static_transform;
  std::vector<int32_t> pair_a, pair_b;
  std::vector<uint8_t> pair_allowed;
  double gjk_tolerance = 1e-6;
  int gjk_solver = MPG_GJK_LIBCCD;  // CollisionRequest::gjk_solver_type
  std::vector<const CollisionGeometry*> geoms;  // identity for geometry dedup

  int add_geometry(const CollisionGeometry* g);
  mpg_world_desc desc() const;
};

void push_se3(std::vector<double>& v, const SE3& T);

// ---------------------------------------------------------------------------
// pinocchio-like kinematic model (reference src/pinocchio_model.{h,cpp})
// ---------------------------------------------------------------------------
struct PinJoint {
  std::string name;
  int type = 0;  // MPG_JOINT_*
  int parent = 0;
  SE3 placement;
  Vec3 axis{0, 0, 1};
  int idx_q = 0, nq = 0, idx_v = 0, nv = 0;
  std::vector<double> lower, upper;
};
struct PinFrame {
  std::string name;
  enum Type { FIXED_JOINT, JOINT, BODY } type;
  int parent;
  SE3 placement;
};

class PinocchioModel {
 public:
  PinocchioModel(const UrdfModel& urdf, const Vec3& gravity, bool verbose);
  static std::shared_ptr<PinocchioModel> from_file(const std::string& urdf, const Vec3& gravity, bool verbose);
  static std::shared_ptr<PinocchioModel> from_string(const std::string& urdf, const Vec3& gravity, bool verbose);

  void set_joint_order(const std::vector<std::string>& names);
  void set_link_order(const std::vector<std::string>& names);
  void compute_forward_kinematics(const std::vector<double>& qpos);  // user order
  Vec7 get_link_pose(size_t index) const;
  std::vector<Vec7> get_link_poses() const;
  std::vector<double> get_random_configuration() const;

  std::vector<std::string> get_link_names(bool user = true) const;
  std::vector<std::string> get_joint_names(bool user = true) const;
  std::vector<std::string> get_leaf_links() const { return leaf_links_; }
  size_t get_joint_dim(size_t i, bool user = true) const;
  std::vector<int> get_joint_dims(bool user = true) const;
  size_t get_joint_id(size_t i, bool user = true) const;
  std::vector<int> get_joint_ids(bool user = true) const;
  std::vector<int> get_parents(bool user = true) const;
  std::string get_joint_type(size_t i, bool user = true) const;
  std::vector<std::string> get_joint_types(bool user = true) const;
  std::vector<std::vector<double>> get_joint_limit(size_t i, bool user = true) const;
  std::vector<std::vector<std::vector<double>>> get_joint_limits(bool user = true) const;
  std::vector<size_t> get_chain_joint_index(const std::string& ee) const;
  std::vector<std::string> get_chain_joint_name(const std::string& ee) const;
  std::vector<size_t> supports(int joint) const;
  int body_frame(const std::string& name) const;

  // PinocchioModelTpl::printFrames (pinocchio_model.cpp:165-185): the model's
  // sizes, then "Frame i name parent_joint TYPE" per frame (kinjac.cpp)
  void print_frames() const;
  // Jacobians and closed-loop IK on the host (kinjac.cpp; pinocchio_model.cpp:335-496)
  std::vector<double> qpos_user2pin(const std::vector<double>& q) const;
  std::vector<double> qpos_pin2user(const std::vector<double>& q) const;
  std::vector<SE3> joint_frames(const std::vector<double>& qpin) const;  // oMi, [0] = universe
  void compute_full_jacobian(const std::vector<double>& qpos);
  std::vector<double> get_link_jacobian(size_t index, bool local) const;  // 6 x nv, row-major
  std::vector<double> compute_single_link_local_jacobian(const std::vector<double>& qpos, size_t index);
  struct IKResult {
    std::vector<double> q;
    bool success = false;
    std::array<double, 6> err{};
  };
  // computeIKCLIK (mask, no limits) / computeIKCLIKJL (q_min / q_max, no mask)
  IKResult ik_clik(size_t index, const Vec7& pose, const std::vector<double>& q_init, const std::vector<bool>* mask,
                   const std::vector<double>* q_min, const std::vector<double>* q_max, double eps, int max_iter,
                   double dt, double damp) const;
  int nq() const { return nq_; }
  int nv() const { return nv_; }

  // kinematic description for the device, user-qpos-driven
  void fill_kinematics(DescBuilder& d, int joint_offset, const std::vector<int>& q_source,
                       const std::vector<double>& q_const) const;
  // per pinocchio joint (1-based index -> [j-1]): user qpos slot, -1 if none
  std::vector<int> pin_joint_user_slot() const;
  const std::vector<PinJoint>& joints() const { return joints_; }
  const std::vector<PinFrame>& frames() const { return frames_; }
  const std::vector<int>& link_frames() const { return link_index_user2pin_; }
  int n_user_joints() const { return (int)user_joint_names_.size(); }
  const std::vector<int>& user_joints() const { return joint_index_user2pin_; }
  const std::vector<int>& user_vidx() const { return vidx_; }

 private:
  void add_fixed(int parent_frame, const SE3& jp, const std::string& jname, const std::string& body);
  void dfs(const UrdfModel& urdf, const std::string& link);
  void ensure_fk_world() const;
  std::vector<size_t> support_columns(int joint) const;
  std::vector<double> user_columns(const std::vector<double>& Jpin) const;
  std::vector<double> joint_local_jacobian(const std::vector<SE3>& oMi, int joint) const;
  std::vector<SE3> jac_oMi_;        // compute_full_jacobian's joint frames
  std::vector<double> jac_world_;   // ... and WORLD Jacobian, pinocchio columns
  bool jac_valid_ = false;

  std::vector<PinJoint> joints_;  // [0] = universe
  std::vector<PinFrame> frames_;
  std::vector<std::string> leaf_links_;
  int nq_ = 0, nv_ = 0;
  Vec3 gravity_;
  bool verbose_;
  std::vector<std::string> user_joint_names_, user_link_names_;
  std::vector<int> joint_index_user2pin_, link_index_user2pin_, vidx_, nvs_;
  // FK state (evaluated on the device, lazily)
  mutable std::unique_ptr<DeviceWorld> fk_world_;
  mutable std::vector<double> qpos_;
  mutable bool fk_dirty_ = false;
  mutable bool fk_valid_ = false;
  mutable std::vector<Vec7> link_poses_;
};

// ---------------------------------------------------------------------------
// FCL model (reference src/fcl_model.{h,cpp})
// ---------------------------------------------------------------------------
// KDLModel (python/pybind_kdl.hpp, src/kdl_model.cpp): chain / tree IK over
// the URDF's kinematic tree (kinjac.cpp); q vectors in joint_names order
class KDLModel {
 public:
  KDLModel(const std::string& urdf, const std::vector<std::string>& joint_names,
           const std::vector<std::string>& link_names, bool verbose);
  const std::string& get_tree_root_name() const { return root_; }
  // kind 0: ChainIkSolverPos_NR, 1: ..._NR_JL (qmin / qmax), 2: ..._LMA
  std::tuple<std::vector<double>, int> chain_ik(size_t index, const std::vector<double>& q0, const Vec7& pose,
                                                int kind, const std::vector<double>* qmin = nullptr,
                                                const std::vector<double>* qmax = nullptr) const;
  std::tuple<std::vector<double>, int> tree_ik_nr_jl(const std::vector<std::string>& endpoints,
                                                     const std::vector<double>& q0, const std::vector<Vec7>& poses,
                                                     const std::vector<double>& qmin,
                                                     const std::vector<double>& qmax) const;

 private:
  std::vector<int> chain(size_t index) const;  // joint ids root -> link
  std::vector<SE3> frames_at(const std::vector<double>& q_user) const;
  SE3 tip(const std::vector<SE3>& oMi, size_t index) const;
  std::vector<double> jacobian(const std::vector<SE3>& oMi, const SE3& T, const std::vector<int>& cols) const;
  std::vector<std::string> user_joint_names_, user_link_names_;
  std::map<std::string, int> user_idx_;
  std::vector<int> pin_user_;  // pinocchio joint -> user slot, -1 if unnamed
  std::shared_ptr<PinocchioModel> pin_;
  std::string root_;
};

class FCLModel {
 public:
  FCLModel(const UrdfModel& urdf, bool verbose, bool convex);
  static std::shared_ptr<FCLModel> from_file(const std::string& urdf, bool verbose, bool convex);
  static std::shared_ptr<FCLModel> from_urdf_string(
      const std::string& urdf, const std::vector<std::pair<std::string, std::vector<ObjPtr>>>& links, bool verbose);

  const std::vector<std::pair<size_t, size_t>>& get_collision_pairs() const { return pairs_; }
  const std::vector<ObjPtr>& get_collision_objects() const;
  const std::vector<ObjPtr>& raw_objects() const { return objects_; }
  const std::vector<std::string>& get_collision_link_names() const { return link_names_; }
  const std::vector<std::string>& get_user_link_names() const { return user_link_names_; }
  const std::vector<size_t>& get_collision_link_user_indices() const { return user_idx_; }
  const std::vector<SE3>& origins() const { return origins_; }
  void set_link_order(const std::vector<std::string>& names);
  void remove_collision_pairs_from_srdf(const std::string& srdf_file);
  void remove_collision_pairs_from_srdf_string(const std::string& srdf);
  void update_collision_objects(const std::vector<Vec7>& link_poses);
  bool collide(const CollisionRequest& req = CollisionRequest()) const;
  std::vector<CollisionResult> collide_full(const CollisionRequest& req = CollisionRequest()) const;
  void print_collision_pairs() const;

  // pose source hook used by ArticulatedModel (lazy FK on the device)
  std::function<std::vector<Vec7>()> pose_provider;
  uint64_t structure_version() const { return structure_version_; }

 private:
  FCLModel() = default;
  void dfs(const UrdfModel& urdf, const std::string& link, const std::string& parent, bool convex);
  void build_pairs_from_parents();
  // pair masks; with req.enable_contact also depth[P], normal[P*3], pos[P*3]
  std::vector<uint32_t> run_pairs(const CollisionRequest& req, std::vector<double>* depth = nullptr,
                                  std::vector<double>* normal = nullptr, std::vector<double>* pos = nullptr) const;
  std::vector<Vec7> current_link_poses() const;

  std::vector<ObjPtr> objects_;
  std::vector<SE3> origins_;
  std::vector<std::string> link_names_, parent_names_, user_link_names_;
  std::vector<size_t> user_idx_;
  std::vector<std::pair<size_t, size_t>> pairs_;
  std::string package_dir_;
  bool verbose_ = false;
  std::vector<Vec7> explicit_poses_;
  bool has_explicit_poses_ = false;
  mutable std::unique_ptr<DeviceWorld> world_;
  mutable uint64_t world_key_ = ~0ull;
  uint64_t structure_version_ = 0;
};

// ---------------------------------------------------------------------------
// ArticulatedModel (reference src/articulated_model.{h,cpp})
// ---------------------------------------------------------------------------
class ArticulatedModel : public std::enable_shared_from_this<ArticulatedModel> {
 public:
  static std::shared_ptr<ArticulatedModel> create(const std::string& urdf, const std::string& srdf, const Vec3& gravity,
                                                  const std::vector<std::string>& joint_names,
                                                  const std::vector<std::string>& link_names, bool verbose,
                                                  bool convex);
  static std::shared_ptr<ArticulatedModel> create_from_urdf_string(
      const std::string& urdf, const std::string& srdf,
      const std::vector<std::pair<std::string, std::vector<ObjPtr>>>& links, const Vec3& gravity,
      const std::vector<std::string>& joint_names, const std::vector<std::string>& link_names, bool verbose);

  std::shared_ptr<PinocchioModel> get_pinocchio_model() const { return pin_; }
  std::shared_ptr<FCLModel> get_fcl_model() const { return fcl_; }
  const std::vector<std::string>& get_user_link_names() const { return user_link_names_; }
  const std::vector<std::string>& get_user_joint_names() const { return user_joint_names_; }
  const std::vector<size_t>& get_move_group_joint_indices() const { return mg_joints_; }
  const std::vector<std::string>& get_move_group_end_effectors() const { return mg_ee_; }
  std::vector<std::string> get_move_group_joint_names() const;
  void set_move_group(const std::vector<std::string>& end_effectors);
  const std::vector<double>& get_qpos() const { return qpos_; }
  void set_qpos(const std::vector<double>& qpos, bool full = false);
  size_t get_qpos_dim() const { return qpos_dim_; }
  void update_srdf(const std::string& srdf);
  const std::string& get_name() const { return name_; }
  void set_name(const std::string& n) { name_ = n; }
  // user-qpos slots of the move group, in setQpos scatter order
  std::vector<int> move_group_slots() const;
  uint64_t structure_version() const { return version_; }

 private:
  ArticulatedModel() = default;
  void init_common(const std::string& srdf_text, bool srdf_is_file);
  std::shared_ptr<PinocchioModel> pin_;
  std::shared_ptr<FCLModel> fcl_;
  std::vector<std::string> user_link_names_, user_joint_names_, mg_ee_;
  std::vector<size_t> mg_joints_;
  size_t qpos_dim_ = 0;
  std::vector<double> qpos_;
  std::string name_;
  bool verbose_ = false;
  uint64_t version_ = 0;
};
using ArtPtr = std::shared_ptr<ArticulatedModel>;

// ---------------------------------------------------------------------------
// AllowedCollisionMatrix (reference src/collision_matrix.{h,cpp})
// ---------------------------------------------------------------------------
enum class AllowedCollision { NEVER = 0, ALWAYS = 1, CONDITIONAL = 2 };

class AllowedCollisionMatrix {
 public:
  std::optional<AllowedCollision> get_entry(const std::string& a, const std::string& b) const;
  bool has_entry(const std::string& a) const { return entries_.count(a) > 0; }
  bool has_entry(const std::string& a, const std::string& b) const;
  void set_entry(const std::string& a, const std::string& b, bool allowed);
  void set_entry(const std::string& a, const std::vector<std::string>& others, bool allowed);
  void set_entry(const std::vector<std::string>& a, const std::vector<std::string>& b, bool allowed);
  void set_entry(const std::string& a, bool allowed);
  void set_entry(const std::vector<std::string>& a, bool allowed);
  void set_entry(bool allowed);
  void remove_entry(const std::string& a, const std::string& b);
  void remove_entry(const std::string& a, const std::vector<std::string>& others);
  void remove_entry(const std::vector<std::string>& a, const std::vector<std::string>& b);
  void remove_entry(const std::string& a);
  void remove_entry(const std::vector<std::string>& a);
  size_t get_size() const { return entries_.size(); }
  std::optional<AllowedCollision> get_default_entry(const std::string& a) const;
  bool has_default_entry(const std::string& a) const { return defaults_.count(a) > 0; }
  void set_default_entry(const std::string& a, bool allowed);
  void set_default_entry(const std::vector<std::string>& a, bool allowed);
  void remove_default_entry(const std::string& a);
  void remove_default_entry(const std::vector<std::string>& a);
  std::optional<AllowedCollision> get_allowed_collision(const std::string& a, const std::string& b) const;
  void clear();
  std::vector<std::string> get_all_entry_names() const;
  std::string print() const;
  uint64_t version() const { return version_; }

 private:
  std::optional<AllowedCollision> default_pair(const std::string& a, const std::string& b) const;
  std::unordered_map<std::string, std::unordered_map<std::string, AllowedCollision>> entries_;
  std::unordered_map<std::string, AllowedCollision> defaults_;
  uint64_t version_ = 0;
};
using AcmPtr = std::shared_ptr<AllowedCollisionMatrix>;

// ---------------------------------------------------------------------------
// AttachedBody + PlanningWorld (reference src/attached_body.h, src/planning_world.{h,cpp})
// ---------------------------------------------------------------------------
// src/attached_body.h:17-73: an object rigidly attached to a link of an
// articulation.  pose = link -> object; the global pose is
// posevec_to_transform(getLinkPose(link)) * pose (attached_body.h:50-53), i.e.
// the link pose goes through its 7-vector (quaternion) form first.
struct AttachedBody {
  std::string name;
  ObjPtr object;
  ArtPtr articulation;
  int link_id;
  SE3 pose;
  std::vector<std::string> touch_links;
  uint64_t version = 0;  // bumped by set_pose: the world's device snapshot bakes `pose` in

  SE3 global_pose() const;
  // attached_body.h:56.  Writes the transform without bumping the object's
  // version: an attached object's own transform is not part of the device
  // snapshot (its pose comes from the link), so no rebuild follows.
  void update_pose() const { object->tf = global_pose(); }
  void set_pose(const SE3& p) {
    pose = p;
    ++version;
  }
};
using AttachedPtr = std::shared_ptr<AttachedBody>;

struct WorldCollisionResult {
  CollisionResult res;
  std::string collision_type, object_name1, object_name2, link_name1, link_name2;
};

struct WorldDistanceResult {  // src/planning_world.h:35-41
  DistanceResult res;
  double min_distance = std::numeric_limits<double>::max();
  std::string distance_type, object_name1, object_name2, link_name1, link_name2;
};

struct PairInfo {
  int a, b;  // device object ids
  std::string collision_type, object_name1, object_name2, link_name1, link_name2;
  bool allowed;
  bool self;  // part of selfCollide() (else collideWithOthers())
};

class PlanningWorld {
 public:
  PlanningWorld(const std::vector<ArtPtr>& arts, const std::vector<std::string>& names,
                const std::vector<ObjPtr>& objs, const std::vector<std::string>& obj_names);

  std::vector<std::string> get_articulation_names() const;
  std::vector<ArtPtr> get_planned_articulations() const;
  ArtPtr get_articulation(const std::string& n) const;
  bool has_articulation(const std::string& n) const { return arts_.count(n) > 0; }
  void add_articulation(const std::string& n, const ArtPtr& a, bool planned = false);
  bool remove_articulation(const std::string& n);
  bool is_articulation_planned(const std::string& n) const { return planned_.count(n) > 0; }
  void set_articulation_planned(const std::string& n, bool planned);
  std::vector<std::string> get_normal_object_names() const;
  ObjPtr get_normal_object(const std::string& n) const;
  bool has_normal_object(const std::string& n) const { return objs_.count(n) > 0; }
  void add_normal_object(const std::string& n, const ObjPtr& o);
  // PlanningWorldTpl::addPointCloud (src/planning_world.cpp:102-110)
  void add_point_cloud(const std::string& n, const std::vector<Vec3>& vertices, double resolution = 0.001);
  bool remove_normal_object(const std::string& n);
  bool is_normal_object_attached(const std::string& n) const { return attached_.count(n) > 0; }
  AttachedPtr get_attached_object(const std::string& n) const;
  void attach_object(const std::string& n, const std::string& art, int link, const Vec7& pose,
                     const std::vector<std::string>& touch_links);
  void attach_object(const std::string& n, const std::string& art, int link, const Vec7& pose);
  void attach_object(const std::string& n, const GeomPtr& g, const std::string& art, int link, const Vec7& pose,
                     const std::vector<std::string>& touch_links);
  void attach_object(const std::string& n, const GeomPtr& g, const std::string& art, int link, const Vec7& pose);
  void attach_sphere(double r, const std::string& art, int link, const Vec7& pose);
  void attach_box(const Vec3& size, const std::string& art, int link, const Vec7& pose);
  void attach_mesh(const std::string& path, const std::string& art, int link, const Vec7& pose);
  bool detach_object(const std::string& n, bool also_remove = false);
  void set_qpos(const std::string& n, const std::vector<double>& q) const;
  void set_qpos_all(const std::vector<double>& state) const;
  AcmPtr get_allowed_collision_matrix() const { return acm_; }
  // PlanningWorldTpl::printAttachedBodyPose (src/planning_world.cpp:237-241)
  void print_attached_body_pose() const;

  bool collide(const CollisionRequest& r = CollisionRequest());
  std::vector<WorldCollisionResult> self_collide(const CollisionRequest& r = CollisionRequest());
  std::vector<WorldCollisionResult> collide_with_others(const CollisionRequest& r = CollisionRequest());
  std::vector<WorldCollisionResult> collide_full(const CollisionRequest& r = CollisionRequest());

  // distance (src/planning_world.cpp:493-720); distance() ignores its
  // request like the reference's (planning_world.h:271-273)
  double distance(const DistanceRequest& r = DistanceRequest());
  WorldDistanceResult self_distance(const DistanceRequest& r = DistanceRequest());
  WorldDistanceResult distance_with_others(const DistanceRequest& r = DistanceRequest());
  WorldDistanceResult distance_full(const DistanceRequest& r = DistanceRequest());
  // per configuration: (self group, others group) minimum and pair index
  void distance_batch(const double* q, int64_t n, double* d_self, int32_t* p_self, double* d_others,
                      int32_t* p_others);
  // with DistanceRequest's flags and the nearest points [n*6] (may be NULL)
  void distance_batch_ex(const double* q, int64_t n, const DistanceRequest& r, double* d_self, int32_t* p_self,
                         double* pts_self, double* d_others, int32_t* p_others, double* pts_others);
  int n_self_pairs();

  // batch API (one launch for N configurations)
  int state_dim();
  const std::vector<PairInfo>& pair_table();
  void collide_batch(const double* q, int64_t n, uint8_t* flags, uint32_t* masks);
  void collide_batch_device(const void* q, int64_t n, void* flags, void* masks, void* stream);
  // distance_batch_ex on device buffers (MPG_MEM_DEVICE, enqueued on stream)
  void distance_batch_device(const void* q, int64_t n, const DistanceRequest& r, void* d_self, void* p_self,
                             void* pts_self, void* d_others, void* p_others, void* pts_others, void* stream);
  int mask_words();
  mpg_world* device_world();  // rebuilds the snapshot if the world changed
  // batched OMPL motion validation over the planner's state space
  // (src/ompl_planner.cpp:248-293): SO2 dofs and the space's maximum extent
  struct MotionSpace {
    uint32_t so2_mask = 0;
    double max_extent = 0.0;
  };
  MotionSpace motion_space();
  void check_motion_batch(const double* from, const double* to, int64_t n, double longest_valid_segment,
                          uint8_t* valid, int32_t* first_invalid, int32_t* segments);
  // Planner.generate_collision_pair (mplib/planner.py:118-163), batched: per
  // pair of pair_table(), how many of n random FULL configurations of the
  // planned articulations (every joint, as set_qpos(q, full=True) sets it)
  // drawn uniformly in the joint limits report it in collide_full()
  std::vector<int64_t> sample_pair_counts(int64_t n, uint64_t seed);
  // the full state those samples range over: limits per value (continuous
  // joints [-pi, pi]), planned articulations in map order
  std::pair<std::vector<double>, std::vector<double>> full_state_limits();
  void profile_enable(bool on);
  // host-buffer batches of at most n states take the one-launch latency path
  void set_small_batch_max(int64_t n);
  struct StageTime { double ms; int64_t launches, units; };
  std::vector<StageTime> profile_read();  // per MPG_STAGE_*

 private:
  std::vector<WorldCollisionResult> run_scalar(const CollisionRequest& r, bool self, bool others);
  void ensure_snapshot(const CollisionRequest& r, bool need_device = true);
  void apply_device_options();
  uint64_t snapshot_key(const CollisionRequest& r) const;
  std::vector<double> current_state() const;
  std::vector<std::string> attached_order() const;
  std::vector<std::string> scene_order() const;

  std::map<std::string, ArtPtr> arts_, planned_;
  std::map<std::string, ObjPtr> objs_;
  std::vector<std::string> obj_insertion_;
  std::map<std::string, AttachedPtr> attached_;
  std::vector<std::string> attached_insertion_;
  AcmPtr acm_;
  uint64_t structure_version_ = 0;
  // snapshot: host description (pairs_, desc_) + lazily created device world
  std::unique_ptr<DescBuilder> desc_;
  uint64_t desc_key_ = ~0ull;
  std::unique_ptr<DeviceWorld> world_;
  uint64_t world_key_ = ~0ull;
  std::vector<PairInfo> pairs_;
  int state_dim_ = 0;
  // the same snapshot with every joint of the planned articulations a state
  // value (sample_pair_counts)
  std::vector<int32_t> full_src_;
  std::vector<double> full_lo_, full_hi_;
  int full_dof_ = 0;
  std::unique_ptr<DeviceWorld> full_world_;
  uint64_t full_key_ = ~0ull;
  double tol_ = 1e-6;
  int64_t small_max_ = -1;  // -1: library default
};

void set_global_seed(unsigned seed);

}  // namespace mpgh
