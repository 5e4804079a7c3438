// ingest.cpp -- URDF/SRDF/STL ingestion and the device-world handle.
//
// urdfdom 4.0.0: Rotation::setFromRPY + normalize, child_links appended while
//   iterating joints in std::map (name-sorted) order (initTree).
// assimp 5.3.1: STL ASCII/binary import, fast_atoreal_move<float>, and
//   JoinIdenticalVertices (unique positions in first-occurrence order);
//   dfs_build_mesh promotes float -> double (reference src/urdf_utils.cpp:82-133).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "host.hpp"
#include "xml.hpp"

namespace mpgh {

// ---------------------------------------------------------------------------
std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::invalid_argument("Cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

SE3 se3_from_pq(const Vec3& p, const std::array<double, 4>& wxyz) {
  SE3 T;
  mpg::quat_to_mat(wxyz[0], wxyz[1], wxyz[2], wxyz[3], T.R);
  T.p[0] = p[0];
  T.p[1] = p[1];
  T.p[2] = p[2];
  return T;
}

SE3 se3_from_pose7(const Vec7& v) { return se3_from_pq({v[0], v[1], v[2]}, {v[3], v[4], v[5], v[6]}); }

SE3 UrdfPose::se3() const { return se3_from_pq(xyz, {quat[3], quat[0], quat[1], quat[2]}); }

void push_se3(std::vector<double>& v, const SE3& T) {
  for (int i = 0; i < 9; ++i) v.push_back(T.R[i]);
  for (int i = 0; i < 3; ++i) v.push_back(T.p[i]);
}

// ---------------------------------------------------------------------------
// URDF
// ---------------------------------------------------------------------------
namespace {

double to_double(const std::string& s) {
  std::istringstream is(s);
  is.imbue(std::locale::classic());
  double v;
  if (!(is >> v)) throw std::invalid_argument("cannot parse number '" + s + "'");
  return v;
}

Vec3 parse_vec3(const std::string* s, const Vec3& def) {
  if (!s) return def;
  std::istringstream is(*s);
  is.imbue(std::locale::classic());
  std::vector<double> v;
  std::string tok;
  while (is >> tok) v.push_back(to_double(tok));
  if (v.size() != 3) throw std::invalid_argument("expected 3 numbers, got '" + *s + "'");
  return {v[0], v[1], v[2]};
}

// urdf::Rotation::setFromRPY + normalize.  sin/cos pairs go through glibc
// sincos(): GCC folds urdfdom's sin(phi)...cos(phi) into it.
std::array<double, 4> rpy_to_quat(double r, double p, double y) {
  const double phi = r / 2.0, the = p / 2.0, psi = y / 2.0;
  double sphi, cphi, sthe, cthe, spsi, cpsi;
  sincos(phi, &sphi, &cphi);
  sincos(the, &sthe, &cthe);
  sincos(psi, &spsi, &cpsi);
  double x = sphi * cthe * cpsi - cphi * sthe * spsi;
  double yy = cphi * sthe * cpsi + sphi * cthe * spsi;
  double z = cphi * cthe * spsi - sphi * sthe * cpsi;
  double w = cphi * cthe * cpsi + sphi * sthe * spsi;
  const double s = std::sqrt(x * x + yy * yy + z * z + w * w);
  if (s == 0.0) return {0.0, 0.0, 0.0, 1.0};
  return {x / s, yy / s, z / s, w / s};
}

UrdfPose parse_origin(const XmlNode* el) {
  UrdfPose p;
  if (!el) return p;
  p.xyz = parse_vec3(el->attr("xyz"), {0, 0, 0});
  if (auto rpy = el->attr("rpy")) {
    Vec3 a = parse_vec3(rpy, {0, 0, 0});
    p.quat = rpy_to_quat(a[0], a[1], a[2]);
  }
  return p;
}

UrdfGeometry parse_geometry(const XmlNode* el) {
  if (!el || el->children.empty()) throw std::invalid_argument("URDF: empty <geometry>");
  const XmlNode* g = el->children[0].get();
  UrdfGeometry out;
  if (g->tag == "mesh") {
    out.kind = UrdfGeometry::MESH;
    out.filename = g->attr_or("filename", "");
    out.scale = parse_vec3(g->attr("scale"), {1, 1, 1});
  } else if (g->tag == "box") {
    out.kind = UrdfGeometry::BOX;
    out.size = parse_vec3(g->attr("size"), {0, 0, 0});
  } else if (g->tag == "sphere") {
    out.kind = UrdfGeometry::SPHERE;
    out.radius = to_double(g->attr_or("radius", "0"));
  } else if (g->tag == "cylinder") {
    out.kind = UrdfGeometry::CYLINDER;
    out.radius = to_double(g->attr_or("radius", "0"));
    out.length = to_double(g->attr_or("length", "0"));
  } else {
    throw std::invalid_argument("Unknown geometry type : " + g->tag);
  }
  return out;
}

}  // namespace

UrdfModel parse_urdf_string(const std::string& xml, const std::string& directory) {
  auto root = XmlParser(xml).parse();
  if (root->tag != "robot") throw std::invalid_argument("The XML stream does not contain a valid URDF model.");
  UrdfModel m;
  m.name = root->attr_or("name", "");
  m.directory = directory;
  for (auto* el : root->children_named("link")) {
    UrdfLink l;
    l.name = el->attr_or("name", "");
    for (auto* c : el->children_named("collision"))
      l.collisions.emplace_back(parse_origin(c->child("origin")), parse_geometry(c->child("geometry")));
    m.links[l.name] = l;
  }
  for (auto* el : root->children_named("joint")) {
    UrdfJoint j;
    j.name = el->attr_or("name", "");
    j.type = el->attr_or("type", "");
    auto pe = el->child("parent");
    auto ce = el->child("child");
    if (!pe || !ce) throw std::invalid_argument("joint " + j.name + " missing parent/child");
    j.parent = pe->attr_or("link", "");
    j.child = ce->attr_or("link", "");
    j.origin = parse_origin(el->child("origin"));
    if (auto ax = el->child("axis")) j.axis = parse_vec3(ax->attr("xyz"), {1, 0, 0});
    if (auto lim = el->child("limit")) {
      j.has_limits = true;
      j.lower = to_double(lim->attr_or("lower", "0"));
      j.upper = to_double(lim->attr_or("upper", "0"));
    }
    m.joints[j.name] = j;
  }
  // initTree: std::map iteration = byte-lexicographic joint names
  for (auto& kv : m.joints) {
    const UrdfJoint& j = kv.second;
    auto pit = m.links.find(j.parent);
    auto cit = m.links.find(j.child);
    if (pit == m.links.end() || cit == m.links.end())
      throw std::invalid_argument("joint " + j.name + " references an unknown link");
    cit->second.parent = j.parent;
    cit->second.parent_joint = j.name;
    pit->second.children.push_back(j.child);
  }
  std::vector<std::string> roots;
  for (auto& kv : m.links)
    if (kv.second.parent.empty()) roots.push_back(kv.first);
  if (roots.size() != 1) throw std::invalid_argument("URDF must have exactly one root link");
  m.root = roots[0];
  return m;
}

UrdfModel parse_urdf_file(const std::string& path) {
  auto slash = path.find_last_of("/\\");
  std::string dir = slash == std::string::npos ? "." : path.substr(0, slash);
  return parse_urdf_string(read_file(path), dir);
}

std::vector<std::pair<std::string, std::string>> parse_srdf_disabled_pairs(const std::string& xml) {
  auto root = XmlParser(xml).parse();
  std::vector<std::pair<std::string, std::string>> out;
  for (auto& c : root->children)
    if (c->tag == "disable_collisions") {
      auto a = c->attr("link1");
      auto b = c->attr("link2");
      if (!a || !b) throw std::invalid_argument("disable_collisions without link1/link2");
      out.emplace_back(*a, *b);
    }
  return out;
}

// ---------------------------------------------------------------------------
// STL (assimp 5.3.1)
// ---------------------------------------------------------------------------
namespace {

const double kFastAtofTable[16] = {0.0,     0.1,      0.01,      0.001,      0.0001,      0.00001,
                                   0.000001, 0.0000001, 0.00000001, 0.000000001, 0.0000000001,
                                   0.00000000001, 0.000000000001, 0.0000000000001,
                                   0.00000000000001, 0.000000000000001};

uint64_t strtoul10_64(const char*& p, unsigned* max_inout) {
  if (*p < '0' || *p > '9') throw std::invalid_argument("STL: cannot parse number");
  unsigned cur = 0;
  uint64_t v = 0;
  for (;;) {
    if (*p < '0' || *p > '9') break;
    v = v * 10 + (uint64_t)(*p - '0');
    ++p;
    ++cur;
    if (max_inout && *max_inout == cur) {
      while (*p >= '0' && *p <= '9') ++p;
      return v;
    }
  }
  if (max_inout) *max_inout = cur;
  return v;
}

// assimp fast_atoreal_move<float>
float fast_atof(const char*& p) {
  float f = 0.0f;
  const bool inv = (*p == '-');
  if (inv || *p == '+') ++p;
  if (*p != '.') f = static_cast<float>(strtoul10_64(p, nullptr));
  if (*p == '.' && p[1] >= '0' && p[1] <= '9') {
    ++p;
    unsigned diff = 15;
    double pl = static_cast<double>(strtoul10_64(p, &diff));
    pl *= kFastAtofTable[diff];
    f += static_cast<float>(pl);
  } else if (*p == '.') {
    ++p;
  }
  if (*p == 'e' || *p == 'E') {
    ++p;
    const bool einv = (*p == '-');
    if (einv || *p == '+') ++p;
    float e = static_cast<float>(strtoul10_64(p, nullptr));
    if (einv) e = -e;
    f *= std::pow(10.0f, e);
  }
  if (inv) f = -f;
  return f;
}

}  // namespace

MeshData load_stl(const std::string& path) {
  const std::string data = read_file(path);
  std::vector<std::array<float, 3>> raw;
  const bool ascii = data.size() >= 5 && strncasecmp(data.c_str(), "solid", 5) == 0 &&
                     data.find("facet", 0) != std::string::npos && data.find("facet", 0) < 4096;
  if (ascii) {
    const char* p = data.c_str();
    const char* end = p + data.size();
    while (p < end) {
      while (p < end && isspace((unsigned char)*p)) ++p;
      const char* tok = p;
      while (p < end && !isspace((unsigned char)*p)) ++p;
      if (p - tok == 6 && std::strncmp(tok, "vertex", 6) == 0) {
        std::array<float, 3> v;
        for (int k = 0; k < 3; ++k) {
          while (p < end && isspace((unsigned char)*p)) ++p;
          v[k] = fast_atof(p);
        }
        raw.push_back(v);
      }
    }
  } else {
    if (data.size() < 84) throw std::invalid_argument("STL too small: " + path);
    uint32_t n;
    std::memcpy(&n, data.data() + 80, 4);
    if (data.size() < 84 + (size_t)n * 50) throw std::invalid_argument("STL truncated: " + path);
    for (uint32_t t = 0; t < n; ++t) {
      const char* rec = data.data() + 84 + (size_t)t * 50;
      for (int k = 0; k < 3; ++k) {
        std::array<float, 3> v;
        std::memcpy(v.data(), rec + 12 + 12 * k, 12);
        raw.push_back(v);
      }
    }
  }
  if (raw.empty() || raw.size() % 3) throw std::invalid_argument("No meshes found in file " + path);
  // JoinIdenticalVertices: first occurrence keeps its slot (+0 == -0)
  MeshData m;
  std::map<std::array<float, 3>, int> index;
  std::vector<int> remap(raw.size());
  for (size_t i = 0; i < raw.size(); ++i) {
    std::array<float, 3> key = {raw[i][0] + 0.0f, raw[i][1] + 0.0f, raw[i][2] + 0.0f};
    auto it = index.find(key);
    if (it == index.end()) {
      index.emplace(key, (int)m.vertices.size());
      remap[i] = (int)m.vertices.size();
      m.vertices.push_back({(double)raw[i][0], (double)raw[i][1], (double)raw[i][2]});
    } else {
      remap[i] = it->second;
    }
  }
  for (size_t t = 0; t < raw.size() / 3; ++t) m.faces.push_back({remap[3 * t], remap[3 * t + 1], remap[3 * t + 2]});
  return m;
}

std::shared_ptr<Convex> load_mesh_as_convex(const std::string& path, const Vec3& scale) {
  MeshData m = load_stl(path);
  std::vector<Vec3> v;
  v.reserve(m.vertices.size());
  for (auto& p : m.vertices) v.push_back({p[0] * scale[0], p[1] * scale[1], p[2] * scale[2]});
  std::vector<int> f;
  for (auto& t : m.faces) {
    f.push_back(3);
    f.push_back(t[0]);
    f.push_back(t[1]);
    f.push_back(t[2]);
  }
  return std::make_shared<Convex>(std::move(v), (int)m.faces.size(), std::move(f));
}

// load_mesh_as_BVH (src/urdf_utils.cpp:136-155): the same vertices
// ((S)p * scale) and triangles, kept as a triangle mesh
std::shared_ptr<BVHModel> load_mesh_as_bvh(const std::string& path, const Vec3& scale) {
  MeshData m = load_stl(path);
  std::vector<Vec3> v;
  v.reserve(m.vertices.size());
  for (auto& p : m.vertices) v.push_back({p[0] * scale[0], p[1] * scale[1], p[2] * scale[2]});
  return std::make_shared<BVHModel>(std::move(v), std::move(m.faces));
}

// ---------------------------------------------------------------------------
// request / device world helpers
// ---------------------------------------------------------------------------
void CollisionRequest::check_supported() const {
  if (num_max_contacts == 0) throw std::invalid_argument("CollisionRequest.num_max_contacts must be >= 1");
  // GST_INDEP: FCL's own GJK on the device for collision; its EPA contacts are
  // not restated
  if (gjk_solver_type == GST_INDEP && enable_contact)
    throw std::logic_error("NotImplemented: enable_contact=True with gjk_solver_type=GST_INDEP (FCL's EPA) is not "
                           "implemented on the device");
  if (enable_cost) throw std::logic_error("NotImplemented: enable_cost=True is not implemented on the device");
  if (!(gjk_tolerance > 0)) throw std::invalid_argument("gjk_tolerance must be > 0");
}

void fill_contacts(const uint32_t* mask, size_t n_pairs, const std::vector<double>& depth,
                   const std::vector<double>& normal, const std::vector<double>& pos, size_t p, Contact& c) {
  (void)mask;
  (void)n_pairs;
  c.penetration_depth = depth[p];
  for (int k = 0; k < 3; ++k) {
    c.normal[k] = normal[3 * p + k];
    c.pos[k] = pos[3 * p + k];
  }
}

void check_status(int rc, const char* what) {
  if (rc == MPG_OK) return;
  std::string msg = std::string(what) + ": " + mpg_last_error();
  if (rc == MPG_E_UNSUPPORTED) throw std::logic_error("NotImplemented: " + msg);
  if (rc == MPG_E_INVALID) throw std::invalid_argument(msg);
  throw std::runtime_error(msg);
}

int default_device() {
  if (const char* e = std::getenv("MPLIB_AMD_DEVICE")) return std::atoi(e);
  if (const char* e = std::getenv("LOCAL_RANK")) return std::atoi(e);
  return 0;
}

int DescBuilder::add_geometry(const CollisionGeometry* g) {
  for (size_t i = 0; i < geoms.size(); ++i)
    if (geoms[i] == g) return (int)i;
  if (g->type < 0)
    throw std::logic_error("NotImplemented: geometry '" + g->kind + "' is not supported by the device collider");
  // FCL's shape traversal reports a pair only when both geometries are
  // occupied (cost_density >= threshold_occupied, ShapeCollisionTraversalNode::
  // leafTesting); the device assumes that (every geometry's default)
  if (!(g->cost_density >= g->threshold_occupied))
    throw std::logic_error("NotImplemented: geometry '" + g->kind +
                           "' with cost_density below its occupancy threshold (FCL's free / uncertain geometry)");
  geoms.push_back(g);
  geom_type.push_back(g->type);
  double prm[4] = {0, 0, 0, 0};
  int vs = 0, nv = 0;
  if (auto b = dynamic_cast<const Box*>(g)) {
    prm[0] = b->side[0];
    prm[1] = b->side[1];
    prm[2] = b->side[2];
  } else if (auto s = dynamic_cast<const Sphere*>(g)) {
    prm[0] = s->radius;
  } else if (auto c = dynamic_cast<const Capsule*>(g)) {
    prm[0] = c->radius;
    prm[1] = c->lz;
  } else if (auto cy = dynamic_cast<const Cylinder*>(g)) {
    prm[0] = cy->radius;
    prm[1] = cy->lz;
  } else if (auto tp = dynamic_cast<const TriangleP*>(g)) {
    vs = (int)(vertices.size() / 3);
    nv = 3;
    for (const Vec3* v : {&tp->a, &tp->b, &tp->c}) vertices.insert(vertices.end(), v->begin(), v->end());
  } else if (auto co = dynamic_cast<const Cone*>(g)) {
    prm[0] = co->radius;
    prm[1] = co->lz;
  } else if (auto el = dynamic_cast<const Ellipsoid*>(g)) {
    prm[0] = el->radii[0];
    prm[1] = el->radii[1];
    prm[2] = el->radii[2];
  } else if (auto oc = dynamic_cast<const OcTree*>(g)) {
    prm[0] = (double)(octree_leaf.size() / 6);
    prm[1] = (double)oc->leaves.size();
    prm[2] = oc->resolution;
    for (auto& l : oc->leaves) octree_leaf.insert(octree_leaf.end(), l.begin(), l.end());
  } else if (auto bm = dynamic_cast<const BVHModel*>(g)) {
    if (bm->building) throw std::invalid_argument("BVHModel used before endModel()");
    vs = (int)(vertices.size() / 3);
    nv = (int)bm->vertices.size();
    for (auto& v : bm->vertices) {
      vertices.push_back(v[0]);
      vertices.push_back(v[1]);
      vertices.push_back(v[2]);
    }
    prm[0] = (double)(mesh_triangle.size() / 3);
    prm[1] = (double)bm->triangles.size();
    for (auto& t : bm->triangles) mesh_triangle.insert(mesh_triangle.end(), t.begin(), t.end());
  } else if (auto cv = dynamic_cast<const Convex*>(g)) {
    vs = (int)(vertices.size() / 3);
    nv = (int)cv->vertices.size();
    for (auto& v : cv->vertices) {
      vertices.push_back(v[0]);
      vertices.push_back(v[1]);
      vertices.push_back(v[2]);
    }
    // the faces decide FCL 0.7.0's support (neighbour walk), include/mpgpu.h
    prm[0] = (double)convex_face.size();
    prm[1] = (double)cv->num_faces;
    convex_face.insert(convex_face.end(), cv->faces.begin(), cv->faces.end());
  }
  geom_vertex_start.push_back(vs);
  geom_vertex_count.push_back(nv);
  for (double x : prm) geom_param.push_back(x);
  return (int)geoms.size() - 1;
}

mpg_world_desc DescBuilder::desc() const {
  mpg_world_desc d{};
  d.n_joints = (int32_t)joint_type.size();
  d.joint_type = joint_type.data();
  d.joint_parent = joint_parent.data();
  d.joint_axis = joint_axis.data();
  d.joint_placement = joint_placement.data();
  d.joint_q_source = joint_q_source.data();
  d.joint_q_const = joint_q_const.data();
  d.dof = dof;
  d.n_links = (int32_t)link_parent.size();
  d.link_parent = link_parent.data();
  d.link_placement = link_placement.data();
  d.n_geoms = (int32_t)geom_type.size();
  d.geom_type = geom_type.data();
  d.geom_vertex_start = geom_vertex_start.data();
  d.geom_vertex_count = geom_vertex_count.data();
  d.geom_param = geom_param.data();
  d.n_vertices = (int64_t)(vertices.size() / 3);
  d.vertices = vertices.data();
  d.n_moving = (int32_t)moving_link.size();
  d.moving_link = moving_link.data();
  d.moving_geom = moving_geom.data();
  d.moving_offset = moving_offset.data();
  d.n_static = (int32_t)static_geom.size();
  d.static_geom = static_geom.data();
  d.static_transform = static_transform.data();
  d.n_pairs = (int32_t)pair_a.size();
  d.pair_a = pair_a.data();
  d.pair_b = pair_b.data();
  d.pair_allowed = pair_allowed.data();
  d.gjk_tolerance = gjk_tolerance;
  d.gjk_solver = gjk_solver;
  d.n_octree_leaves = (int64_t)(octree_leaf.size() / 6);
  d.octree_leaf = octree_leaf.data();
  d.n_mesh_triangles = (int64_t)(mesh_triangle.size() / 3);
  d.mesh_triangle = mesh_triangle.data();
  d.n_convex_face_ints = (int64_t)convex_face.size();
  d.convex_face = convex_face.data();
  const bool lim = joint_lower.size() == joint_type.size() && joint_upper.size() == joint_type.size();
  d.joint_lower = lim ? joint_lower.data() : nullptr;
  d.joint_upper = lim ? joint_upper.data() : nullptr;
  return d;
}

DeviceWorld::DeviceWorld(const DescBuilder& b, int device) {
  mpg_world_desc d = b.desc();
  check_status(mpg_world_create(&d, device, &w_), "mpg_world_create");
  check_status(mpg_world_get_info(w_, &info_), "mpg_world_get_info");
}

DeviceWorld::~DeviceWorld() { mpg_world_destroy(w_); }

}  // namespace mpgh
