// kin.cpp -- PinocchioModel / FCLModel / ArticulatedModel host objects.
//
// Model construction restates MPlib's own tree walks:
//   PinocchioModelTpl::dfs_parse_tree / init  src/pinocchio_model.cpp:559-752
//     (+ pinocchio 2.6.21 UrdfVisitor: joint placements folded with the
//      parent body frame, fixed joints become frames, RX/RY/RZ vs unaligned)
//   FCLModelTpl::dfs_parse_tree / init        src/fcl_model.cpp:196-294
//   ArticulatedModelTpl ctor / setMoveGroup / setQpos
//                                             src/articulated_model.cpp:15-127
// Kinematics and collision queries run on the device (include/mpgpu.h).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <iostream>
#include <limits>

#include "host.hpp"

namespace mpgh {

namespace {

bool is_approx(const Vec3& a, const Vec3& b, double prec = 1e-12) {
  double d = 0, na = 0, nb = 0;
  for (int i = 0; i < 3; ++i) {
    d += (a[i] - b[i]) * (a[i] - b[i]);
    na += a[i] * a[i];
    nb += b[i] * b[i];
  }
  return d <= prec * prec * std::min(na, nb);
}

int cartesian_axis(const Vec3& a) {
  if (is_approx(a, {1, 0, 0})) return 0;
  if (is_approx(a, {0, 1, 0})) return 1;
  if (is_approx(a, {0, 0, 1})) return 2;
  return 3;
}

SE3 identity_se3() {
  SE3 T;
  mpg::se3_identity(T);
  return T;
}

const char* joint_short_name(int t) {
  static const char* names[] = {"JointModelRX",  "JointModelRY", "JointModelRZ",
                                "JointModelRevoluteUnaligned", "JointModelPX", "JointModelPY",
                                "JointModelPZ", "JointModelPrismaticUnaligned", "JointModelRUBX",
                                "JointModelRUBY", "JointModelRUBZ", "JointModelRevoluteUnboundedUnaligned"};
  return names[t];
}

}  // namespace

// ===========================================================================
// PinocchioModel
// ===========================================================================
PinocchioModel::PinocchioModel(const UrdfModel& urdf, const Vec3& gravity, bool verbose)
    : gravity_(gravity), verbose_(verbose) {
  PinJoint universe;
  universe.name = "universe";
  universe.placement = identity_se3();
  joints_.push_back(universe);
  frames_.push_back({"universe", PinFrame::FIXED_JOINT, 0, identity_se3()});
  add_fixed(0, identity_se3(), "root_joint", urdf.root);
  dfs(urdf, urdf.root);
  std::vector<std::string> jn, ln;
  for (auto& j : joints_) jn.push_back(j.name);
  set_joint_order(jn);
  set_link_order(get_link_names(false));
}

std::shared_ptr<PinocchioModel> PinocchioModel::from_file(const std::string& urdf, const Vec3& g, bool verbose) {
  return std::make_shared<PinocchioModel>(parse_urdf_file(urdf), g, verbose);
}
std::shared_ptr<PinocchioModel> PinocchioModel::from_string(const std::string& urdf, const Vec3& g, bool verbose) {
  return std::make_shared<PinocchioModel>(parse_urdf_string(urdf), g, verbose);
}

void PinocchioModel::add_fixed(int parent_frame, const SE3& jp, const std::string& jname, const std::string& body) {
  const PinFrame pf = frames_[parent_frame];
  const SE3 placement = mpg::se3_mul(pf.placement, jp);
  frames_.push_back({jname, PinFrame::FIXED_JOINT, pf.parent, placement});
  frames_.push_back({body, PinFrame::BODY, pf.parent, placement});
}

int PinocchioModel::body_frame(const std::string& name) const {
  for (size_t i = 0; i < frames_.size(); ++i)
    if (frames_[i].type == PinFrame::BODY && frames_[i].name == name) return (int)i;
  return -1;
}

void PinocchioModel::dfs(const UrdfModel& urdf, const std::string& link_name) {
  const UrdfLink& link = urdf.links.at(link_name);
  for (const std::string& child : link.children) {
    const UrdfLink& cl = urdf.links.at(child);
    const UrdfJoint& j = urdf.joints.at(cl.parent_joint);
    const int parent_frame = body_frame(link_name);
    const SE3 jp = j.origin.se3();
    if (verbose_) std::cout << child << " joint " << j.name << " (" << j.type << ")" << std::endl;
    if (j.type == "fixed") {
      add_fixed(parent_frame, jp, j.name, child);
    } else {
      const PinFrame pf = frames_[parent_frame];
      const int ax = cartesian_axis(j.axis);
      PinJoint pj;
      pj.name = j.name;
      pj.parent = pf.parent;
      pj.placement = mpg::se3_mul(pf.placement, jp);
      pj.axis = j.axis;
      if (ax == 3) {  // axis.normalized()
        const double n = std::sqrt(j.axis[0] * j.axis[0] + j.axis[1] * j.axis[1] + j.axis[2] * j.axis[2]);
        pj.axis = {j.axis[0] / n, j.axis[1] / n, j.axis[2] / n};
      }
      if (j.type == "revolute") {
        if (!j.has_limits) throw std::runtime_error("REVOLUTE without limits");
        pj.type = MPG_JOINT_RX + ax;
        pj.nq = pj.nv = 1;
        pj.lower = {j.lower};
        pj.upper = {j.upper};
      } else if (j.type == "continuous") {
        pj.type = MPG_JOINT_RUBX + ax;
        pj.nq = 2;
        pj.nv = 1;
        pj.lower = {-1.01, -1.01};
        pj.upper = {1.01, 1.01};
      } else if (j.type == "prismatic") {
        if (!j.has_limits) throw std::runtime_error("PRISMATIC without limits");
        pj.type = MPG_JOINT_PX + ax;
        pj.nq = pj.nv = 1;
        pj.lower = {j.lower};
        pj.upper = {j.upper};
      } else {
        throw std::invalid_argument("The type of joint " + j.name + " is not supported.");
      }
      pj.idx_q = nq_;
      pj.idx_v = nv_;
      nq_ += pj.nq;
      nv_ += pj.nv;
      const int idx = (int)joints_.size();
      joints_.push_back(pj);
      frames_.push_back({j.name, PinFrame::JOINT, idx, identity_se3()});
      frames_.push_back({child, PinFrame::BODY, idx, mpg::se3_mul(identity_se3(), identity_se3())});
    }
    dfs(urdf, child);
    if (cl.children.empty()) leaf_links_.push_back(child);
  }
}

void PinocchioModel::set_joint_order(const std::vector<std::string>& names) {
  std::vector<int> u2p, vidx, nvs;
  int v = 0;
  for (const auto& n : names) {
    int idx = -1;
    for (size_t j = 0; j < joints_.size(); ++j)
      if (joints_[j].name == n) idx = (int)j;
    if (idx < 0) throw std::invalid_argument(n + " is a invalid name in setJointOrder");
    u2p.push_back(idx);
    vidx.push_back(v);
    nvs.push_back(joints_[idx].nv);
    v += joints_[idx].nv;
  }
  if (v != nv_) throw std::runtime_error("setJointOrder failed");
  user_joint_names_ = names;
  joint_index_user2pin_ = u2p;
  vidx_ = vidx;
  nvs_ = nvs;
  fk_world_.reset();
  fk_valid_ = false;
}

void PinocchioModel::set_link_order(const std::vector<std::string>& names) {
  std::vector<int> fr;
  for (const auto& n : names) {
    int f = body_frame(n);
    if (f < 0) throw std::invalid_argument(n + " is a invalid names in setLinkOrder");
    fr.push_back(f);
  }
  user_link_names_ = names;
  link_index_user2pin_ = fr;
  fk_world_.reset();
  fk_valid_ = false;
}

std::vector<int> PinocchioModel::pin_joint_user_slot() const {
  std::vector<int> slot(joints_.size() > 0 ? joints_.size() - 1 : 0, -1);
  for (size_t u = 0; u < joint_index_user2pin_.size(); ++u) {
    int j = joint_index_user2pin_[u];
    if (j > 0) slot[j - 1] = vidx_[u];
  }
  return slot;
}

void PinocchioModel::fill_kinematics(DescBuilder& d, int joint_offset, const std::vector<int>& q_source,
                                     const std::vector<double>& q_const) const {
  for (size_t j = 1; j < joints_.size(); ++j) {
    const PinJoint& pj = joints_[j];
    d.joint_type.push_back(pj.type);
    d.joint_parent.push_back(pj.parent > 0 ? pj.parent + joint_offset : 0);
    for (int k = 0; k < 3; ++k) d.joint_axis.push_back(pj.axis[k]);
    push_se3(d.joint_placement, pj.placement);
    d.joint_q_source.push_back(q_source[j - 1]);
    d.joint_q_const.push_back(q_const[j - 1]);
    const bool one = pj.nq == 1 && !pj.lower.empty() && !pj.upper.empty();
    d.joint_lower.push_back(one ? pj.lower[0] : -std::numeric_limits<double>::infinity());
    d.joint_upper.push_back(one ? pj.upper[0] : std::numeric_limits<double>::infinity());
  }
  for (int f : link_index_user2pin_) {
    const PinFrame& fr = frames_[f];
    d.link_parent.push_back(fr.parent > 0 ? fr.parent + joint_offset : 0);
    push_se3(d.link_placement, fr.placement);
  }
}

void PinocchioModel::ensure_fk_world() const {
  if (fk_world_) return;
  DescBuilder d;
  std::vector<int> src = pin_joint_user_slot();
  std::vector<double> cst(src.size(), 0.0);
  fill_kinematics(d, 0, src, cst);
  d.dof = nv_;
  fk_world_ = std::make_unique<DeviceWorld>(d, default_device());
}

void PinocchioModel::compute_forward_kinematics(const std::vector<double>& qpos) {
  if ((int)qpos.size() != nv_)
    throw std::runtime_error("Qpos user2pinocchio failed: expected " + std::to_string(nv_) + " values, got " +
                             std::to_string(qpos.size()));
  qpos_ = qpos;
  fk_dirty_ = true;
  fk_valid_ = true;
}

std::vector<Vec7> PinocchioModel::get_link_poses() const {
  if (!fk_valid_) throw std::runtime_error("compute_forward_kinematics has not been called");
  if (fk_dirty_) {
    ensure_fk_world();
    std::vector<double> out(link_index_user2pin_.size() * 7);
    check_status(mpg_fk_batch(fk_world_->get(), qpos_.data(), 1, out.data(), MPG_MEM_HOST, nullptr), "mpg_fk_batch");
    link_poses_.resize(link_index_user2pin_.size());
    for (size_t l = 0; l < link_poses_.size(); ++l)
      for (int k = 0; k < 7; ++k) link_poses_[l][k] = out[7 * l + k];
    fk_dirty_ = false;
  }
  return link_poses_;
}

Vec7 PinocchioModel::get_link_pose(size_t index) const {
  if (index >= link_index_user2pin_.size()) throw std::runtime_error("The link index is out of bound!");
  return get_link_poses()[index];
}

std::vector<double> PinocchioModel::get_random_configuration() const {
  // pinocchio::randomConfiguration: lower + (upper - lower) * rand()/RAND_MAX per
  // coordinate (Eigen::internal::random), continuous joints as a random angle.
  std::vector<double> q(nv_, 0.0);
  for (size_t u = 0; u < joint_index_user2pin_.size(); ++u) {
    int j = joint_index_user2pin_[u];
    if (j <= 0) continue;
    const PinJoint& pj = joints_[j];
    const double r = (double)std::rand() / (double)RAND_MAX;
    if (pj.nq == 2) q[vidx_[u]] = -M_PI + 2 * M_PI * r;
    else q[vidx_[u]] = pj.lower[0] + (pj.upper[0] - pj.lower[0]) * r;
  }
  return q;
}

std::vector<std::string> PinocchioModel::get_link_names(bool user) const {
  if (user) return user_link_names_;
  std::vector<std::string> out;
  for (auto& f : frames_)
    if (f.type == PinFrame::BODY) out.push_back(f.name);
  return out;
}

std::vector<std::string> PinocchioModel::get_joint_names(bool user) const {
  if (user) return user_joint_names_;
  std::vector<std::string> out;
  for (auto& j : joints_) out.push_back(j.name);
  return out;
}

size_t PinocchioModel::get_joint_dim(size_t i, bool user) const {
  if (user) return nvs_.at(i);
  return joints_.at(i).nv;
}
std::vector<int> PinocchioModel::get_joint_dims(bool user) const {
  if (user) return nvs_;
  std::vector<int> out;
  for (auto& j : joints_) out.push_back(j.nv);
  return out;
}
size_t PinocchioModel::get_joint_id(size_t i, bool user) const {
  if (user) return vidx_.at(i);
  return joints_.at(i).idx_v;
}
std::vector<int> PinocchioModel::get_joint_ids(bool user) const {
  if (user) return vidx_;
  std::vector<int> out;
  for (auto& j : joints_) out.push_back(j.idx_v);
  return out;
}
std::vector<int> PinocchioModel::get_parents(bool user) const {
  std::vector<int> out;
  if (user) {
    for (int j : joint_index_user2pin_) out.push_back(j > 0 ? joints_[j].parent : 0);
  } else {
    for (auto& j : joints_) out.push_back(j.parent);
  }
  return out;
}
std::string PinocchioModel::get_joint_type(size_t i, bool user) const {
  int j = user ? joint_index_user2pin_.at(i) : (int)i;
  if (j == 0) return "JointModelFreeFlyer";  // universe placeholder (never a real joint)
  return joint_short_name(joints_.at(j).type);
}
std::vector<std::string> PinocchioModel::get_joint_types(bool user) const {
  std::vector<std::string> out;
  size_t n = user ? user_joint_names_.size() : joints_.size();
  for (size_t i = 0; i < n; ++i) out.push_back(get_joint_type(i, user));
  return out;
}
std::vector<std::vector<double>> PinocchioModel::get_joint_limit(size_t i, bool user) const {
  int j = user ? joint_index_user2pin_.at(i) : (int)i;
  std::vector<std::vector<double>> out;
  if (j == 0) return out;
  const PinJoint& pj = joints_[j];
  const bool unbounded = pj.type >= MPG_JOINT_RUBX;
  if (unbounded) return {{-3.14159265359, 3.14159265359}};
  for (int k = 0; k < pj.nq; ++k) out.push_back({pj.lower[k], pj.upper[k]});
  return out;
}
std::vector<std::vector<std::vector<double>>> PinocchioModel::get_joint_limits(bool user) const {
  std::vector<std::vector<std::vector<double>>> out;
  size_t n = user ? user_joint_names_.size() : joints_.size();
  for (size_t i = 0; i < n; ++i) out.push_back(get_joint_limit(i, user));
  return out;
}
std::vector<size_t> PinocchioModel::supports(int j) const {
  std::vector<size_t> out;
  while (j > 0) {
    out.push_back(j);
    j = joints_[j].parent;
  }
  out.push_back(0);
  std::reverse(out.begin(), out.end());
  return out;
}
std::vector<size_t> PinocchioModel::get_chain_joint_index(const std::string& ee) const {
  int f = body_frame(ee);
  if (f < 0) throw std::invalid_argument("unknown link " + ee);
  std::vector<size_t> out;
  for (size_t j : supports(frames_[f].parent))
    for (size_t u = 0; u < joint_index_user2pin_.size(); ++u)
      if ((size_t)joint_index_user2pin_[u] == j) out.push_back(u);
  return out;
}
std::vector<std::string> PinocchioModel::get_chain_joint_name(const std::string& ee) const {
  std::vector<std::string> out;
  for (size_t u : get_chain_joint_index(ee)) out.push_back(joints_[joint_index_user2pin_[u]].name);
  return out;
}

// ===========================================================================
// FCLModel
// ===========================================================================
FCLModel::FCLModel(const UrdfModel& urdf, bool verbose, bool convex) : verbose_(verbose) {
  package_dir_ = urdf.directory;
  dfs(urdf, urdf.root, "root's parent", convex);
  std::vector<std::string> users = link_names_;
  users.erase(std::unique(users.begin(), users.end()), users.end());
  set_link_order(users);
  build_pairs_from_parents();
}

std::shared_ptr<FCLModel> FCLModel::from_file(const std::string& urdf, bool verbose, bool convex) {
  return std::make_shared<FCLModel>(parse_urdf_file(urdf), verbose, convex);
}

std::shared_ptr<FCLModel> FCLModel::from_urdf_string(
    const std::string& urdf, const std::vector<std::pair<std::string, std::vector<ObjPtr>>>& links, bool verbose) {
  (void)parse_urdf_string(urdf);  // validates the kinematic description
  std::shared_ptr<FCLModel> m(new FCLModel());
  m->verbose_ = verbose;
  for (auto& [name, objs] : links)
    for (auto& o : objs) {
      m->objects_.push_back(o);
      m->link_names_.push_back(name);
      m->origins_.push_back(o->tf);
    }
  std::vector<std::string> users = m->link_names_;
  users.erase(std::unique(users.begin(), users.end()), users.end());
  m->set_link_order(users);
  for (size_t i = 0; i < m->link_names_.size(); ++i)
    for (size_t j = 0; j < i; ++j)
      if (m->link_names_[i] != m->link_names_[j]) m->pairs_.emplace_back(j, i);
  return m;
}

void FCLModel::dfs(const UrdfModel& urdf, const std::string& link_name, const std::string& parent, bool convex) {
  const UrdfLink& link = urdf.links.at(link_name);
  for (const auto& [origin, geom] : link.collisions) {
    GeomPtr g;
    if (geom.kind == UrdfGeometry::MESH) {
      std::string fn = geom.filename;
      if (fn.rfind("package://", 0) == 0) fn = fn.substr(10);
      if (convex && fn.find(".convex.stl") == std::string::npos) fn += ".convex.stl";
      std::string path = package_dir_.empty() ? fn : package_dir_ + "/" + fn;
      if (verbose_) std::cout << "File name " << fn << std::endl;
      if (convex) g = load_mesh_as_convex(path, geom.scale);
      else g = load_mesh_as_bvh(path, geom.scale);
    } else if (geom.kind == UrdfGeometry::CYLINDER) {
      g = std::make_shared<Cylinder>(geom.radius, geom.length);
    } else if (geom.kind == UrdfGeometry::BOX) {
      g = std::make_shared<Box>(geom.size);
    } else {
      g = std::make_shared<Sphere>(geom.radius);
    }
    objects_.push_back(std::make_shared<CollisionObject>(g, identity_se3()));
    link_names_.push_back(link_name);
    parent_names_.push_back(parent);
    origins_.push_back(origin.se3());
  }
  for (const auto& c : link.children) dfs(urdf, c, link_name, convex);
}

void FCLModel::build_pairs_from_parents() {
  pairs_.clear();
  for (size_t i = 0; i < link_names_.size(); ++i)
    for (size_t j = 0; j < i; ++j)
      if (link_names_[i] != link_names_[j] && parent_names_[i] != link_names_[j] && parent_names_[j] != link_names_[i])
        pairs_.emplace_back(j, i);
  ++structure_version_;
}

void FCLModel::set_link_order(const std::vector<std::string>& names) {
  std::vector<size_t> idx;
  for (auto& ln : link_names_) {
    auto it = std::find(names.begin(), names.end(), ln);
    if (it == names.end()) throw std::invalid_argument("The names does not contain link " + ln);
    idx.push_back(it - names.begin());
  }
  user_link_names_ = names;
  user_idx_ = idx;
  ++structure_version_;
}

void FCLModel::remove_collision_pairs_from_srdf_string(const std::string& srdf) {
  for (auto& [l1, l2] : parse_srdf_disabled_pairs(srdf)) {
    if (verbose_) std::cout << "Try to Remove collision parts:" << l1 << " " << l2 << std::endl;
    pairs_.erase(std::remove_if(pairs_.begin(), pairs_.end(),
                                [&](const std::pair<size_t, size_t>& p) {
                                  return (link_names_[p.first] == l1 && link_names_[p.second] == l2) ||
                                         (link_names_[p.first] == l2 && link_names_[p.second] == l1);
                                }),
                 pairs_.end());
  }
  ++structure_version_;
}

void FCLModel::remove_collision_pairs_from_srdf(const std::string& srdf_file) {
  if (srdf_file.empty()) {
    std::cout << "No SRDF file provided!" << std::endl;
    return;
  }
  const std::string ext = srdf_file.substr(srdf_file.find_last_of('.') + 1);
  if (ext != "srdf") throw std::runtime_error(srdf_file + " does not have the right extension.");
  remove_collision_pairs_from_srdf_string(read_file(srdf_file));
}

void FCLModel::update_collision_objects(const std::vector<Vec7>& link_poses) {
  if (link_poses.size() < user_link_names_.size())
    throw std::invalid_argument("update_collision_objects: expected one pose per user link");
  explicit_poses_ = link_poses;
  has_explicit_poses_ = true;
}

std::vector<Vec7> FCLModel::current_link_poses() const {
  if (has_explicit_poses_) return explicit_poses_;
  if (pose_provider) return pose_provider();
  return std::vector<Vec7>(user_link_names_.size(), Vec7{0, 0, 0, 1, 0, 0, 0});
}

const std::vector<ObjPtr>& FCLModel::get_collision_objects() const {
  // refresh the user-visible transforms (FCLModel::updateCollisionObjects)
  std::vector<Vec7> poses;
  if (has_explicit_poses_ || pose_provider) poses = current_link_poses();
  if (!poses.empty())
    for (size_t i = 0; i < objects_.size(); ++i)
      objects_[i]->tf = mpg::se3_mul(se3_from_pose7(poses[user_idx_[i]]), origins_[i]);
  return objects_;
}

std::vector<uint32_t> FCLModel::run_pairs(const CollisionRequest& req, std::vector<double>* depth,
                                          std::vector<double>* normal, std::vector<double>* pos) const {
  req.check_supported();
  const uint64_t key = (structure_version_ * 1000003ull + (uint64_t)std::llround(req.gjk_tolerance * 1e15)) * 2ull +
                       (req.gjk_solver_type == GST_INDEP ? 1ull : 0ull);
  if (!world_ || world_key_ != key) {
    DescBuilder d;
    d.gjk_tolerance = req.gjk_tolerance;
    d.gjk_solver = req.gjk_solver_type == GST_INDEP ? MPG_GJK_INDEP : MPG_GJK_LIBCCD;
    for (size_t l = 0; l < user_link_names_.size(); ++l) {
      d.link_parent.push_back(0);
      push_se3(d.link_placement, identity_se3());
    }
    for (size_t i = 0; i < objects_.size(); ++i) {
      d.moving_link.push_back((int32_t)user_idx_[i]);
      d.moving_geom.push_back(d.add_geometry(objects_[i]->geom.get()));
      push_se3(d.moving_offset, origins_[i]);
    }
    for (auto& p : pairs_) {
      d.pair_a.push_back((int32_t)p.first);
      d.pair_b.push_back((int32_t)p.second);
      d.pair_allowed.push_back(0);
    }
    world_ = std::make_unique<DeviceWorld>(d, default_device());
    world_key_ = key;
  }
  std::vector<Vec7> poses = current_link_poses();
  std::vector<double> flat;
  for (size_t l = 0; l < user_link_names_.size(); ++l)
    for (int k = 0; k < 7; ++k) flat.push_back(poses[l][k]);
  uint8_t flag = 0;
  std::vector<uint32_t> mask(world_->info().mask_words, 0);
  if (req.enable_contact && depth) {
    const size_t P = pairs_.size();
    depth->assign(std::max<size_t>(P, 1), 0.0);
    normal->assign(3 * std::max<size_t>(P, 1), 0.0);
    pos->assign(3 * std::max<size_t>(P, 1), 0.0);
    check_status(mpg_collide_contacts(world_->get(), flat.data(), 1, MPG_INPUT_LINK_POSES, &flag, mask.data(),
                                      depth->data(), normal->data(), pos->data(), MPG_MEM_HOST, nullptr),
                 "mpg_collide_contacts");
    return mask;
  }
  check_status(mpg_collide_link_poses(world_->get(), flat.data(), 1, &flag, mask.data(), MPG_MEM_HOST, nullptr),
               "mpg_collide_link_poses");
  return mask;
}

bool FCLModel::collide(const CollisionRequest& req) const {
  auto m = run_pairs(req);
  for (auto w : m)
    if (w) return true;
  return false;
}

std::vector<CollisionResult> FCLModel::collide_full(const CollisionRequest& req) const {
  std::vector<double> depth, normal, pos;
  auto m = run_pairs(req, &depth, &normal, &pos);
  std::vector<CollisionResult> out(pairs_.size());
  for (size_t p = 0; p < pairs_.size(); ++p)
    if ((m[p >> 5] >> (p & 31)) & 1u) {
      Contact c;
      c.o1 = objects_[pairs_[p].first]->geom;
      c.o2 = objects_[pairs_[p].second]->geom;
      if (req.enable_contact) fill_contacts(m.data(), pairs_.size(), depth, normal, pos, p, c);
      out[p].contacts.push_back(c);
    }
  return out;
}

void FCLModel::print_collision_pairs() const {
  for (auto& p : pairs_) std::cout << link_names_[p.first] << " " << link_names_[p.second] << std::endl;
}

// ===========================================================================
// ArticulatedModel
// ===========================================================================
void ArticulatedModel::init_common(const std::string& srdf, bool srdf_is_file) {
  if (user_link_names_.empty()) user_link_names_ = pin_->get_link_names(false);
  if (user_joint_names_.empty()) user_joint_names_ = pin_->get_joint_names(false);
  pin_->set_link_order(user_link_names_);
  pin_->set_joint_order(user_joint_names_);
  fcl_->set_link_order(user_link_names_);
  if (srdf_is_file) fcl_->remove_collision_pairs_from_srdf(srdf);
  else fcl_->remove_collision_pairs_from_srdf_string(srdf);
  qpos_.assign(pin_->nv(), 0.0);
  std::weak_ptr<PinocchioModel> wp = pin_;
  fcl_->pose_provider = [wp]() {
    auto p = wp.lock();
    if (!p) throw std::runtime_error("pinocchio model expired");
    return p->get_link_poses();
  };
  pin_->compute_forward_kinematics(qpos_);
  set_move_group(user_link_names_);
}

std::shared_ptr<ArticulatedModel> ArticulatedModel::create(const std::string& urdf, const std::string& srdf,
                                                          const Vec3& gravity,
                                                          const std::vector<std::string>& joint_names,
                                                          const std::vector<std::string>& link_names, bool verbose,
                                                          bool convex) {
  std::shared_ptr<ArticulatedModel> a(new ArticulatedModel());
  UrdfModel m = parse_urdf_file(urdf);
  a->verbose_ = verbose;
  a->pin_ = std::make_shared<PinocchioModel>(m, gravity, verbose);
  a->fcl_ = std::make_shared<FCLModel>(m, verbose, convex);
  a->user_link_names_ = link_names;
  a->user_joint_names_ = joint_names;
  a->init_common(srdf, true);
  return a;
}

std::shared_ptr<ArticulatedModel> ArticulatedModel::create_from_urdf_string(
    const std::string& urdf, const std::string& srdf,
    const std::vector<std::pair<std::string, std::vector<ObjPtr>>>& links, const Vec3& gravity,
    const std::vector<std::string>& joint_names, const std::vector<std::string>& link_names, bool verbose) {
  std::shared_ptr<ArticulatedModel> a(new ArticulatedModel());
  a->verbose_ = verbose;
  a->pin_ = PinocchioModel::from_string(urdf, gravity, verbose);
  a->fcl_ = FCLModel::from_urdf_string(urdf, links, verbose);
  a->user_link_names_ = link_names;
  a->user_joint_names_ = joint_names;
  a->init_common(srdf, false);
  return a;
}

std::vector<std::string> ArticulatedModel::get_move_group_joint_names() const {
  std::vector<std::string> out;
  for (auto i : mg_joints_) out.push_back(user_joint_names_[i]);
  return out;
}

void ArticulatedModel::set_move_group(const std::vector<std::string>& ees) {
  mg_ee_ = ees;
  mg_joints_.clear();
  for (auto& ee : ees) {
    auto c = pin_->get_chain_joint_index(ee);
    mg_joints_.insert(mg_joints_.begin(), c.begin(), c.end());
  }
  std::sort(mg_joints_.begin(), mg_joints_.end());
  mg_joints_.erase(std::unique(mg_joints_.begin(), mg_joints_.end()), mg_joints_.end());
  qpos_dim_ = 0;
  for (auto i : mg_joints_) qpos_dim_ += pin_->get_joint_dim(i);
  ++version_;
}

std::vector<int> ArticulatedModel::move_group_slots() const {
  std::vector<int> out;
  for (auto i : mg_joints_) {
    const int start = (int)pin_->get_joint_id(i);
    const int dim = (int)pin_->get_joint_dim(i);
    for (int j = 0; j < dim; ++j) out.push_back(start + j);
  }
  return out;
}

void ArticulatedModel::set_qpos(const std::vector<double>& q, bool full) {
  if (full) {
    if ((int)q.size() != pin_->nv())
      throw std::runtime_error("Length is not correct, Dim of Q: " + std::to_string(pin_->nv()) +
                               " ,Len of qpos: " + std::to_string(q.size()));
    qpos_ = q;
  } else {
    if (q.size() != qpos_dim_)
      throw std::runtime_error("Length is not correct, Dim of Q: " + std::to_string(qpos_dim_) +
                               " ,Len of qpos: " + std::to_string(q.size()));
    auto slots = move_group_slots();
    for (size_t k = 0; k < slots.size(); ++k) qpos_[slots[k]] = q[k];
  }
  pin_->compute_forward_kinematics(qpos_);  // evaluated lazily on the device
}

void ArticulatedModel::update_srdf(const std::string& srdf) {
  fcl_->remove_collision_pairs_from_srdf(srdf);
  ++version_;
}

}  // namespace mpgh
