// world.cpp -- AllowedCollisionMatrix and PlanningWorld.
//
// AllowedCollisionMatrix restates src/collision_matrix.cpp (entries + default
// entries, getAllowedCollision = entry, else combined default entries).
// PlanningWorld restates src/planning_world.cpp: the pair loops of
// selfCollide (:277-369) and collideWithOthers (:372-481) become one pair
// table, in the same (o1, o2) argument order, and filterCollisions (:265-274)
// becomes a per-pair "allowed" bit resolved when the device snapshot is built.
// The snapshot is rebuilt whenever the world, the ACM, an object pose, or a
// constant joint value changes.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <set>
#include <sstream>

#include "host.hpp"
#include "planner.hpp"

namespace mpgh {

// ===========================================================================
// AllowedCollisionMatrix
// ===========================================================================
std::optional<AllowedCollision> AllowedCollisionMatrix::get_entry(const std::string& a, const std::string& b) const {
  auto i = entries_.find(a);
  if (i == entries_.end()) return std::nullopt;
  auto j = i->second.find(b);
  if (j == i->second.end()) return std::nullopt;
  return j->second;
}
bool AllowedCollisionMatrix::has_entry(const std::string& a, const std::string& b) const {
  auto i = entries_.find(a);
  return i != entries_.end() && i->second.count(b) > 0;
}
void AllowedCollisionMatrix::set_entry(const std::string& a, const std::string& b, bool allowed) {
  const auto v = allowed ? AllowedCollision::ALWAYS : AllowedCollision::NEVER;
  entries_[a][b] = entries_[b][a] = v;
  ++version_;
}
void AllowedCollisionMatrix::set_entry(const std::string& a, const std::vector<std::string>& others, bool allowed) {
  for (auto& o : others)
    if (o != a) set_entry(o, a, allowed);
}
void AllowedCollisionMatrix::set_entry(const std::vector<std::string>& a, const std::vector<std::string>& b,
                                       bool allowed) {
  for (auto& x : a) set_entry(x, b, allowed);
}
void AllowedCollisionMatrix::set_entry(const std::string& a, bool allowed) {
  std::vector<std::string> keys;
  for (auto& e : entries_) keys.push_back(e.first);
  for (auto& k : keys)
    if (k != a) set_entry(a, k, allowed);
}
void AllowedCollisionMatrix::set_entry(const std::vector<std::string>& a, bool allowed) {
  for (auto& x : a) set_entry(x, allowed);
}
void AllowedCollisionMatrix::set_entry(bool allowed) {
  const auto v = allowed ? AllowedCollision::ALWAYS : AllowedCollision::NEVER;
  for (auto& e : entries_)
    for (auto& f : e.second) f.second = v;
  ++version_;
}
void AllowedCollisionMatrix::remove_entry(const std::string& a, const std::string& b) {
  if (auto it = entries_.find(a); it != entries_.end())
    if (it->second.erase(b) == 1 && it->second.empty()) entries_.erase(it);
  if (auto it = entries_.find(b); it != entries_.end())
    if (it->second.erase(a) == 1 && it->second.empty()) entries_.erase(it);
  ++version_;
}
void AllowedCollisionMatrix::remove_entry(const std::string& a, const std::vector<std::string>& others) {
  for (auto& o : others)
    if (o != a) remove_entry(o, a);
}
void AllowedCollisionMatrix::remove_entry(const std::vector<std::string>& a, const std::vector<std::string>& b) {
  for (auto& x : a) remove_entry(x, b);
}
void AllowedCollisionMatrix::remove_entry(const std::string& a) {
  entries_.erase(a);
  for (auto it = entries_.begin(); it != entries_.end();)
    if (it->second.erase(a) == 1 && it->second.empty()) it = entries_.erase(it);
    else ++it;
  ++version_;
}
void AllowedCollisionMatrix::remove_entry(const std::vector<std::string>& a) {
  for (auto& x : a) remove_entry(x);
}
std::optional<AllowedCollision> AllowedCollisionMatrix::get_default_entry(const std::string& a) const {
  auto it = defaults_.find(a);
  if (it == defaults_.end()) return std::nullopt;
  return it->second;
}
void AllowedCollisionMatrix::set_default_entry(const std::string& a, bool allowed) {
  defaults_[a] = allowed ? AllowedCollision::ALWAYS : AllowedCollision::NEVER;
  ++version_;
}
void AllowedCollisionMatrix::set_default_entry(const std::vector<std::string>& a, bool allowed) {
  for (auto& x : a) set_default_entry(x, allowed);
}
void AllowedCollisionMatrix::remove_default_entry(const std::string& a) {
  defaults_.erase(a);
  ++version_;
}
void AllowedCollisionMatrix::remove_default_entry(const std::vector<std::string>& a) {
  for (auto& x : a) remove_default_entry(x);
}
std::optional<AllowedCollision> AllowedCollisionMatrix::default_pair(const std::string& a, const std::string& b) const {
  auto t1 = get_default_entry(a), t2 = get_default_entry(b);
  if (!t1 && !t2) return std::nullopt;
  if (t1 && !t2) return t1;
  if (!t1 && t2) return t2;
  if (*t1 == AllowedCollision::NEVER || *t2 == AllowedCollision::NEVER) return AllowedCollision::NEVER;
  if (*t1 == AllowedCollision::CONDITIONAL || *t2 == AllowedCollision::CONDITIONAL) return AllowedCollision::CONDITIONAL;
  return AllowedCollision::ALWAYS;
}
std::optional<AllowedCollision> AllowedCollisionMatrix::get_allowed_collision(const std::string& a,
                                                                              const std::string& b) const {
  auto t = get_entry(a, b);
  return t ? t : default_pair(a, b);
}
void AllowedCollisionMatrix::clear() {
  entries_.clear();
  defaults_.clear();
  ++version_;
}
std::vector<std::string> AllowedCollisionMatrix::get_all_entry_names() const {
  std::set<std::string> s;
  for (auto& e : entries_) s.insert(e.first);
  for (auto& d : defaults_) s.insert(d.first);
  return std::vector<std::string>(s.begin(), s.end());
}
std::string AllowedCollisionMatrix::print() const {
  auto names = get_all_entry_names();
  std::ostringstream os;
  for (auto& a : names) {
    os << a << ": ";
    for (auto& b : names) {
      auto t = get_allowed_collision(a, b);
      os << (!t ? '-' : *t == AllowedCollision::NEVER ? '0' : *t == AllowedCollision::ALWAYS ? '1' : '?');
    }
    os << "\n";
  }
  return os.str();
}

// ===========================================================================
// PlanningWorld
// ===========================================================================
PlanningWorld::PlanningWorld(const std::vector<ArtPtr>& arts, const std::vector<std::string>& names,
                             const std::vector<ObjPtr>& objs, const std::vector<std::string>& obj_names)
    : acm_(std::make_shared<AllowedCollisionMatrix>()) {
  if (arts.size() != names.size())
    throw std::runtime_error("articulations and articulation_names should have the same size");
  if (objs.size() != obj_names.size())
    throw std::runtime_error("normal_objects and normal_object_names should have the same size");
  for (size_t i = 0; i < arts.size(); ++i) {
    arts[i]->set_name(names[i]);
    arts_[names[i]] = arts[i];
    planned_[names[i]] = arts[i];
  }
  for (size_t i = 0; i < objs.size(); ++i) add_normal_object(obj_names[i], objs[i]);
}

std::vector<std::string> PlanningWorld::get_articulation_names() const {
  std::vector<std::string> out;
  for (auto& kv : arts_) out.push_back(kv.first);
  return out;
}
std::vector<ArtPtr> PlanningWorld::get_planned_articulations() const {
  std::vector<ArtPtr> out;
  for (auto& kv : planned_) out.push_back(kv.second);
  return out;
}
ArtPtr PlanningWorld::get_articulation(const std::string& n) const {
  auto it = arts_.find(n);
  return it == arts_.end() ? nullptr : it->second;
}
void PlanningWorld::add_articulation(const std::string& n, const ArtPtr& a, bool planned) {
  a->set_name(n);
  arts_[n] = a;
  set_articulation_planned(n, planned);
  ++structure_version_;
}
bool PlanningWorld::remove_articulation(const std::string& n) {
  auto it = arts_.find(n);
  if (it == arts_.end()) return false;
  auto links = it->second->get_user_link_names();
  arts_.erase(it);
  planned_.erase(n);
  acm_->remove_entry(links);
  acm_->remove_default_entry(links);
  ++structure_version_;
  return true;
}
void PlanningWorld::set_articulation_planned(const std::string& n, bool planned) {
  auto art = arts_.at(n);
  if (planned) planned_[n] = art;
  else planned_.erase(n);
  ++structure_version_;
}
std::vector<std::string> PlanningWorld::get_normal_object_names() const { return obj_insertion_; }
ObjPtr PlanningWorld::get_normal_object(const std::string& n) const {
  auto it = objs_.find(n);
  return it == objs_.end() ? nullptr : it->second;
}
void PlanningWorld::add_normal_object(const std::string& n, const ObjPtr& o) {
  if (!objs_.count(n)) obj_insertion_.push_back(n);
  objs_[n] = o;
  ++structure_version_;
}

void PlanningWorld::add_point_cloud(const std::string& n, const std::vector<Vec3>& vertices, double resolution) {
  SE3 I;
  for (int i = 0; i < 9; ++i) I.R[i] = (i % 4 == 0) ? 1.0 : 0.0;
  I.p[0] = I.p[1] = I.p[2] = 0.0;
  add_normal_object(n, std::make_shared<CollisionObject>(std::make_shared<OcTree>(vertices, resolution), I));
}
bool PlanningWorld::remove_normal_object(const std::string& n) {
  if (!objs_.erase(n)) return false;
  obj_insertion_.erase(std::remove(obj_insertion_.begin(), obj_insertion_.end(), n), obj_insertion_.end());
  if (attached_.erase(n))
    attached_insertion_.erase(std::remove(attached_insertion_.begin(), attached_insertion_.end(), n),
                              attached_insertion_.end());
  acm_->remove_entry(n);
  acm_->remove_default_entry(n);
  ++structure_version_;
  return true;
}
SE3 AttachedBody::global_pose() const {
  return mpg::se3_mul(se3_from_pose7(articulation->get_pinocchio_model()->get_link_pose(link_id)), pose);
}

// Eigen's operator<< for a matrix: the stream's precision, every coefficient
// right-aligned to the widest one, " " between columns, "\n" between rows
void PlanningWorld::print_attached_body_pose() const {
  for (const auto& [name, body] : attached_) {
    const SE3 T = body->global_pose();
    double M[16];
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) M[4 * i + j] = T.R[3 * i + j];
      M[4 * i + 3] = T.p[i];
    }
    M[12] = M[13] = M[14] = 0.0;
    M[15] = 1.0;
    std::string cell[16];
    size_t width = 0;
    for (int k = 0; k < 16; ++k) {
      std::ostringstream o;
      o << M[k];
      cell[k] = o.str();
      width = std::max(width, cell[k].size());
    }
    std::ostringstream out;
    out << name << " global pose:\n";
    for (int i = 0; i < 4; ++i) {
      for (int j = 0; j < 4; ++j) {
        if (j) out << ' ';
        out << std::string(width - cell[4 * i + j].size(), ' ') << cell[4 * i + j];
      }
      if (i < 3) out << '\n';
    }
    std::cout << out.str() << std::endl;
  }
}

AttachedPtr PlanningWorld::get_attached_object(const std::string& n) const {
  auto it = attached_.find(n);
  return it == attached_.end() ? nullptr : it->second;
}

void PlanningWorld::attach_object(const std::string& n, const std::string& art, int link, const Vec7& pose,
                                  const std::vector<std::string>& touch_links) {
  auto obj = objs_.at(n);
  auto a = planned_.at(art);
  if (link < 0 || link >= (int)a->get_user_link_names().size()) throw std::out_of_range("link_id out of range");
  auto body = std::make_shared<AttachedBody>(AttachedBody{n, obj, a, link, se3_from_pose7(pose), touch_links});
  body->update_pose();  // AttachedBody ctor (attached_body.cpp:22)
  auto it = attached_.find(n);
  if (it != attached_.end()) acm_->remove_entry(n, it->second->touch_links);
  else attached_insertion_.push_back(n);
  attached_[n] = body;
  acm_->set_entry(n, touch_links, true);
  ++structure_version_;
}

void PlanningWorld::attach_object(const std::string& n, const std::string& art, int link, const Vec7& pose) {
  auto obj = objs_.at(n);
  auto a = planned_.at(art);
  if (link < 0 || link >= (int)a->get_user_link_names().size()) throw std::out_of_range("link_id out of range");
  auto body = std::make_shared<AttachedBody>(AttachedBody{n, obj, a, link, se3_from_pose7(pose), {}});
  body->update_pose();  // AttachedBody ctor (attached_body.cpp:22)
  auto it = attached_.find(n);
  if (it != attached_.end()) {
    body->touch_links = it->second->touch_links;
    attached_[n] = body;
    ++structure_version_;
    return;
  }
  attached_insertion_.push_back(n);
  attached_[n] = body;
  ++structure_version_;
  // touch_links = self links colliding with the object in the current state
  std::vector<std::string> touch;
  for (auto& c : self_collide())
    if (c.link_name1 == n) touch.push_back(c.link_name2);
    else if (c.link_name2 == n) touch.push_back(c.link_name1);
  body->touch_links = touch;
  acm_->set_entry(n, touch, true);
}

void PlanningWorld::attach_object(const std::string& n, const GeomPtr& g, const std::string& art, int link,
                                  const Vec7& pose, const std::vector<std::string>& touch_links) {
  remove_normal_object(n);
  SE3 I;
  mpg::se3_identity(I);
  add_normal_object(n, std::make_shared<CollisionObject>(g, I));
  attach_object(n, art, link, pose, touch_links);
}
void PlanningWorld::attach_object(const std::string& n, const GeomPtr& g, const std::string& art, int link,
                                  const Vec7& pose) {
  remove_normal_object(n);
  SE3 I;
  mpg::se3_identity(I);
  add_normal_object(n, std::make_shared<CollisionObject>(g, I));
  attach_object(n, art, link, pose);
}
void PlanningWorld::attach_sphere(double r, const std::string& art, int link, const Vec7& pose) {
  attach_object(art + "_" + std::to_string(link) + "_sphere", std::make_shared<Sphere>(r), art, link, pose);
}
void PlanningWorld::attach_box(const Vec3& size, const std::string& art, int link, const Vec7& pose) {
  attach_object(art + "_" + std::to_string(link) + "_box", std::make_shared<Box>(size), art, link, pose);
}
void PlanningWorld::attach_mesh(const std::string& path, const std::string& art, int link, const Vec7& pose) {
  // load_mesh_as_BVH(mesh_path, (1, 1, 1)) (planning_world.cpp:212-218)
  attach_object(art + "_" + std::to_string(link) + "_mesh", load_mesh_as_bvh(path, {1.0, 1.0, 1.0}), art, link, pose);
}
bool PlanningWorld::detach_object(const std::string& n, bool also_remove) {
  if (also_remove) {
    if (objs_.erase(n))
      obj_insertion_.erase(std::remove(obj_insertion_.begin(), obj_insertion_.end(), n), obj_insertion_.end());
    acm_->remove_entry(n);
    acm_->remove_default_entry(n);
  }
  auto it = attached_.find(n);
  ++structure_version_;
  if (it == attached_.end()) return false;
  acm_->remove_entry(n, it->second->touch_links);
  attached_.erase(it);
  attached_insertion_.erase(std::remove(attached_insertion_.begin(), attached_insertion_.end(), n),
                            attached_insertion_.end());
  return true;
}

void PlanningWorld::set_qpos(const std::string& n, const std::vector<double>& q) const { arts_.at(n)->set_qpos(q); }

void PlanningWorld::set_qpos_all(const std::vector<double>& state) const {
  size_t i = 0;
  for (auto& kv : planned_) {
    const size_t n = kv.second->get_qpos_dim();
    if (i + n > state.size()) throw std::runtime_error("State dimension is not correct");
    kv.second->set_qpos(std::vector<double>(state.begin() + i, state.begin() + i + n));
    i += n;
  }
  if (i != state.size()) throw std::runtime_error("State dimension is not correct");
}

std::vector<std::string> PlanningWorld::attached_order() const { return attached_insertion_; }

std::vector<std::string> PlanningWorld::scene_order() const {
  std::vector<std::string> out;
  for (auto& n : obj_insertion_)
    if (!attached_.count(n)) out.push_back(n);
  return out;
}

// state = concatenated move-group qpos of the planned articulations (std::map order)
std::vector<double> PlanningWorld::current_state() const {
  std::vector<double> s;
  for (auto& kv : planned_) {
    auto& q = kv.second->get_qpos();
    for (int slot : kv.second->move_group_slots()) s.push_back(q[slot]);
  }
  return s;
}

uint64_t PlanningWorld::snapshot_key(const CollisionRequest& r) const {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
  auto mixd = [&](double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    mix(u);
  };
  mix(structure_version_);
  mix(acm_->version());
  mixd(r.gjk_tolerance);
  mix((uint64_t)r.gjk_solver_type);
  for (auto& kv : arts_) {
    mix(kv.second->structure_version());
    mix(kv.second->get_fcl_model()->structure_version());
    const bool planned = planned_.count(kv.first) > 0;
    mix(planned);
    // constants baked into the snapshot: non-move-group joints of planned
    // articulations and every joint of unplanned ones
    auto& q = kv.second->get_qpos();
    std::vector<int> slots = planned ? kv.second->move_group_slots() : std::vector<int>();
    for (size_t i = 0; i < q.size(); ++i)
      if (std::find(slots.begin(), slots.end(), (int)i) == slots.end()) mixd(q[i]);
  }
  for (auto& n : obj_insertion_) mix(objs_.at(n)->version);
  for (auto& n : attached_insertion_) {
    mix((uint64_t)(uintptr_t)attached_.at(n).get());
    mix(attached_.at(n)->version);
  }
  return h;
}

void PlanningWorld::ensure_snapshot(const CollisionRequest& r, bool need_device) {
  r.check_supported();
  const uint64_t key = snapshot_key(r);
  if (key == desc_key_) {
    if (need_device && !world_) {
      world_ = std::make_unique<DeviceWorld>(*desc_, default_device());
      world_key_ = key;
      apply_device_options();
    }
    return;
  }
  world_.reset();
  world_key_ = ~0ull;
  desc_ = std::make_unique<DescBuilder>();
  DescBuilder& d = *desc_;
  d.gjk_tolerance = r.gjk_tolerance;
  d.gjk_solver = r.gjk_solver_type == GST_INDEP ? MPG_GJK_INDEP : MPG_GJK_LIBCCD;
  pairs_.clear();
  full_src_.clear();
  full_lo_.clear();
  full_hi_.clear();
  full_dof_ = 0;
  full_world_.reset();
  full_key_ = ~0ull;
  // ---- kinematic forest: planned articulations (map order), then unplanned
  struct ArtInfo {
    ArtPtr art;
    int link_base;   // first user link index in the desc
    int obj_base;    // first moving object id
    bool planned;
  };
  std::vector<ArtInfo> infos;
  int dof = 0;
  auto add_art = [&](const ArtPtr& a, bool planned) {
    auto pin = a->get_pinocchio_model();
    const int joint_offset = (int)d.joint_type.size();
    std::vector<int> user_slot = pin->pin_joint_user_slot();
    auto& q = a->get_qpos();
    std::vector<int> slots = planned ? a->move_group_slots() : std::vector<int>();
    std::vector<int> src(user_slot.size(), -1);
    std::vector<double> cst(user_slot.size(), 0.0);
    for (size_t j = 0; j < user_slot.size(); ++j) {
      const int s = user_slot[j];
      if (s < 0) continue;
      auto it = std::find(slots.begin(), slots.end(), s);
      if (it != slots.end()) src[j] = dof + (int)(it - slots.begin());
      else cst[j] = q[s];
    }
    // full-state variant: every user slot of a planned articulation
    for (size_t j = 0; j < user_slot.size(); ++j)
      full_src_.push_back(planned && user_slot[j] >= 0 ? full_dof_ + user_slot[j] : src[j]);
    if (planned) {
      std::vector<double> lo(pin->nv(), 0.0), hi(pin->nv(), 0.0);
      for (size_t u = 0; u < pin->user_joints().size(); ++u) {
        auto lim = pin->get_joint_limit(u, true);
        if (lim.empty() || u >= pin->user_vidx().size()) continue;
        lo[pin->user_vidx()[u]] = lim[0][0];
        hi[pin->user_vidx()[u]] = lim[0][1];
      }
      full_lo_.insert(full_lo_.end(), lo.begin(), lo.end());
      full_hi_.insert(full_hi_.end(), hi.begin(), hi.end());
      full_dof_ += pin->nv();
    }
    const int link_base = (int)d.link_parent.size();
    pin->fill_kinematics(d, joint_offset, src, cst);
    if (planned) dof += (int)slots.size();
    auto fcl = a->get_fcl_model();
    const int obj_base = (int)d.moving_link.size();
    const auto& objs = fcl->raw_objects();
    for (size_t i = 0; i < objs.size(); ++i) {
      d.moving_link.push_back(link_base + (int)fcl->get_collision_link_user_indices()[i]);
      d.moving_geom.push_back(d.add_geometry(objs[i]->geom.get()));
      push_se3(d.moving_offset, fcl->origins()[i]);
    }
    infos.push_back({a, link_base, obj_base, planned});
  };
  for (auto& kv : planned_) add_art(kv.second, true);
  for (auto& kv : arts_)
    if (!planned_.count(kv.first)) add_art(kv.second, false);
  d.dof = dof;
  state_dim_ = dof;
  // attached bodies (moving objects on a planned articulation's link)
  std::vector<std::string> att = attached_order();
  std::map<std::string, int> att_id;
  for (auto& n : att) {
    auto& b = attached_.at(n);
    int link_base = -1;
    for (auto& inf : infos)
      if (inf.art == b->articulation) link_base = inf.link_base;
    if (link_base < 0) throw std::runtime_error("attached body " + n + " refers to an articulation not in the world");
    att_id[n] = (int)d.moving_link.size();
    d.moving_link.push_back(link_base + b->link_id);
    d.moving_geom.push_back(d.add_geometry(b->object->geom.get()));
    push_se3(d.moving_offset, b->pose);
  }
  const int n_moving = (int)d.moving_link.size();
  // scene objects (static)
  std::vector<std::string> scene = scene_order();
  std::map<std::string, int> scene_id;
  for (auto& n : scene) {
    scene_id[n] = n_moving + (int)d.static_geom.size();
    d.static_geom.push_back(d.add_geometry(objs_.at(n)->geom.get()));
    push_se3(d.static_transform, objs_.at(n)->tf);
  }
  auto add_pair = [&](int a, int b, const char* type, const std::string& on1, const std::string& on2,
                      const std::string& ln1, const std::string& ln2, bool self) {
    auto t = acm_->get_allowed_collision(ln1, ln2);
    const bool allowed = t && *t != AllowedCollision::NEVER;
    pairs_.push_back({a, b, type, on1, on2, ln1, ln2, allowed, self});
    d.pair_a.push_back(a);
    d.pair_b.push_back(b);
    d.pair_allowed.push_back(allowed ? 1 : 0);
  };
  // ---- selfCollide (planning_world.cpp:277-369)
  for (size_t ai = 0; ai < infos.size(); ++ai) {
    if (!infos[ai].planned) continue;
    auto& A = infos[ai];
    auto fcl = A.art->get_fcl_model();
    auto& names = fcl->get_collision_link_names();
    const std::string& an = A.art->get_name();
    for (auto& p : fcl->get_collision_pairs())
      add_pair(A.obj_base + (int)p.first, A.obj_base + (int)p.second, "self", an, an, names[p.first],
               names[p.second], true);
    for (size_t bi = 0; bi < ai; ++bi) {  // planned x planned (earlier in map order)
      auto& B = infos[bi];
      auto fcl2 = B.art->get_fcl_model();
      auto& names2 = fcl2->get_collision_link_names();
      for (size_t i = 0; i < names.size(); ++i)
        for (size_t j = 0; j < names2.size(); ++j)
          add_pair(A.obj_base + (int)i, B.obj_base + (int)j, "self_articulation", an, B.art->get_name(), names[i],
                   names2[j], true);
    }
    for (auto& n : att)
      for (size_t i = 0; i < names.size(); ++i)
        add_pair(att_id[n], A.obj_base + (int)i, "self_attach", an, n, names[i], n, true);
  }
  for (size_t k = 0; k < att.size(); ++k)
    for (size_t k2 = 0; k2 < k; ++k2)
      add_pair(att_id[att[k]], att_id[att[k2]], "attach_attach", att[k], att[k2], att[k], att[k2], true);
  // ---- collideWithOthers (planning_world.cpp:372-481)
  for (auto& A : infos) {
    if (!A.planned) continue;
    auto fcl = A.art->get_fcl_model();
    auto& names = fcl->get_collision_link_names();
    const std::string& an = A.art->get_name();
    for (auto& B : infos) {
      if (B.planned) continue;
      auto& names2 = B.art->get_fcl_model()->get_collision_link_names();
      for (size_t i = 0; i < names.size(); ++i)
        for (size_t j = 0; j < names2.size(); ++j)
          add_pair(A.obj_base + (int)i, B.obj_base + (int)j, "articulation_articulation", an, B.art->get_name(),
                   names[i], names2[j], false);
    }
    for (auto& s : scene)
      for (size_t i = 0; i < names.size(); ++i)
        add_pair(A.obj_base + (int)i, scene_id[s], "articulation_sceneobject", an, s, names[i], s, false);
  }
  for (auto& n : att) {
    for (auto& B : infos) {
      if (B.planned) continue;
      auto& names2 = B.art->get_fcl_model()->get_collision_link_names();
      for (size_t i = 0; i < names2.size(); ++i)
        add_pair(att_id[n], B.obj_base + (int)i, "attach_articulation", n, B.art->get_name(), n, names2[i], false);
    }
    for (auto& s : scene) add_pair(att_id[n], scene_id[s], "attach_sceneobject", n, s, n, s, false);
  }
  desc_key_ = key;
  tol_ = r.gjk_tolerance;
  // validate the descriptor on the host even when no device is needed yet
  if (need_device) {
    world_ = std::make_unique<DeviceWorld>(d, default_device());
    world_key_ = key;
    apply_device_options();
  }
}

void PlanningWorld::apply_device_options() {
  if (world_ && small_max_ >= 0) check_status(mpg_set_small_batch_max(world_->get(), small_max_), "mpg_set_small_batch_max");
}

void PlanningWorld::set_small_batch_max(int64_t n) {
  if (n < 0) throw std::invalid_argument("small_batch_max must be >= 0");
  small_max_ = n;
  apply_device_options();
}

std::vector<WorldCollisionResult> PlanningWorld::run_scalar(const CollisionRequest& r, bool self, bool others) {
  ensure_snapshot(r);
  std::vector<double> s = current_state();
  uint8_t flag = 0;
  std::vector<uint32_t> mask(world_->info().mask_words, 0);
  std::vector<double> depth, normal, pos;
  if (r.enable_contact) {
    const size_t P = std::max<size_t>(pairs_.size(), 1);
    depth.assign(P, 0.0);
    normal.assign(3 * P, 0.0);
    pos.assign(3 * P, 0.0);
    check_status(mpg_collide_contacts(world_->get(), s.data(), 1, MPG_INPUT_Q, &flag, mask.data(), depth.data(),
                                      normal.data(), pos.data(), MPG_MEM_HOST, nullptr),
                 "mpg_collide_contacts");
  } else {
    check_status(mpg_collide_batch(world_->get(), s.data(), 1, &flag, mask.data(), MPG_MEM_HOST, nullptr),
                 "mpg_collide_batch");
  }
  std::vector<WorldCollisionResult> out;
  for (size_t p = 0; p < pairs_.size(); ++p) {
    const PairInfo& pi = pairs_[p];
    if ((pi.self && !self) || (!pi.self && !others)) continue;
    if ((mask[p >> 5] >> (p & 31)) & 1u) {
      WorldCollisionResult w;
      Contact c;
      if (r.enable_contact) fill_contacts(mask.data(), pairs_.size(), depth, normal, pos, p, c);
      w.res.contacts.push_back(c);
      w.collision_type = pi.collision_type;
      w.object_name1 = pi.object_name1;
      w.object_name2 = pi.object_name2;
      w.link_name1 = pi.link_name1;
      w.link_name2 = pi.link_name2;
      out.push_back(w);
    }
  }
  return out;
}

bool PlanningWorld::collide(const CollisionRequest& r) { return !run_scalar(r, true, true).empty(); }
std::vector<WorldCollisionResult> PlanningWorld::self_collide(const CollisionRequest& r) {
  return run_scalar(r, true, false);
}
std::vector<WorldCollisionResult> PlanningWorld::collide_with_others(const CollisionRequest& r) {
  return run_scalar(r, false, true);
}
std::vector<WorldCollisionResult> PlanningWorld::collide_full(const CollisionRequest& r) {
  return run_scalar(r, true, true);
}

int PlanningWorld::state_dim() {
  ensure_snapshot(CollisionRequest(), false);
  return state_dim_;
}
const std::vector<PairInfo>& PlanningWorld::pair_table() {
  ensure_snapshot(CollisionRequest(), false);
  return pairs_;
}
int PlanningWorld::mask_words() {
  ensure_snapshot(CollisionRequest(), false);
  return std::max<int>(1, ((int)pairs_.size() + 31) / 32);
}
mpg_world* PlanningWorld::device_world() {
  ensure_snapshot(CollisionRequest());
  return world_->get();
}
void PlanningWorld::collide_batch(const double* q, int64_t n, uint8_t* flags, uint32_t* masks) {
  ensure_snapshot(CollisionRequest());
  check_status(mpg_collide_batch(world_->get(), q, n, flags, masks, MPG_MEM_HOST, nullptr), "mpg_collide_batch");
}
void PlanningWorld::collide_batch_device(const void* q, int64_t n, void* flags, void* masks, void* stream) {
  ensure_snapshot(CollisionRequest());
  check_status(mpg_collide_batch(world_->get(), static_cast<const double*>(q), n, static_cast<uint8_t*>(flags),
                                 static_cast<uint32_t*>(masks), MPG_MEM_DEVICE, stream),
               "mpg_collide_batch");
}

PlanningWorld::MotionSpace PlanningWorld::motion_space() {
  MotionSpace ms;
  int slot = 0;
  for (auto& kv : planned_) {  // std::map: the state layout of setQposAll
    const auto& pin = kv.second->get_pinocchio_model();
    for (size_t id : kv.second->get_move_group_joint_indices()) {
      const PinJoint& pj = pin->joints()[pin->user_joints().at(id)];
      if (pj.type >= MPG_JOINT_RUBX) {  // continuous joint: SO2StateSpace, extent pi
        if (slot < 32) ms.so2_mask |= 1u << slot;
        ms.max_extent += 1.0 * M_PI;
        slot += 1;
      } else {  // RealVectorStateSpace(nq), extent = |high - low|
        double e2 = 0.0;
        for (int k = 0; k < pj.nq; ++k) e2 += (pj.upper[k] - pj.lower[k]) * (pj.upper[k] - pj.lower[k]);
        ms.max_extent += 1.0 * std::sqrt(e2);
        slot += pj.nq;
      }
    }
  }
  return ms;
}

void PlanningWorld::check_motion_batch(const double* from, const double* to, int64_t n, double lvs, uint8_t* valid,
                                       int32_t* first_invalid, int32_t* segments) {
  ensure_snapshot(CollisionRequest());
  const MotionSpace ms = motion_space();
  check_status(mpg_check_motion_batch(world_->get(), from, to, n, ms.so2_mask, lvs, valid, first_invalid, segments,
                                      MPG_MEM_HOST, nullptr),
               "mpg_check_motion_batch");
}

// GST_INDEP: FCL's own GJK for unsigned distances; its EPA (signed) is not
// restated.  OcTree / BVH mesh pairs with GST_INDEP are refused by the device
// call (MPG_E_UNSUPPORTED -> NotImplementedError).
void DistanceRequest::check_supported() const {
  if (gjk_solver_type == GST_INDEP && enable_signed_distance)
    throw std::logic_error("NotImplemented: enable_signed_distance=True with gjk_solver_type=GST_INDEP (FCL's EPA) "
                           "is not implemented on the device");
}

int32_t DistanceRequest::flags() const {
  return (enable_signed_distance ? MPG_DISTANCE_SIGNED : 0) | (enable_nearest_points ? MPG_DISTANCE_NEAREST_POINTS : 0) |
         (gjk_solver_type == GST_INDEP ? MPG_DISTANCE_GJK_INDEP : 0);
}

mpg_distance_request DistanceRequest::to_c() const {
  mpg_distance_request r;
  r.flags = flags();
  r.distance_tolerance = distance_tolerance;
  return r;
}

int PlanningWorld::n_self_pairs() {
  ensure_snapshot(CollisionRequest(), false);
  int n = 0;
  while (n < (int)pairs_.size() && pairs_[n].self) ++n;
  for (size_t p = n; p < pairs_.size(); ++p)
    if (pairs_[p].self) throw std::logic_error("pair table: self pairs must lead");
  return n;
}

void PlanningWorld::distance_batch(const double* q, int64_t n, double* d_self, int32_t* p_self, double* d_others,
                                   int32_t* p_others) {
  const int ns = n_self_pairs();
  ensure_snapshot(CollisionRequest());
  check_status(mpg_distance_batch(world_->get(), q, n, ns, d_self, p_self, d_others, p_others, MPG_MEM_HOST, nullptr),
               "mpg_distance_batch");
}

void PlanningWorld::distance_batch_ex(const double* q, int64_t n, const DistanceRequest& r, double* d_self,
                                      int32_t* p_self, double* pts_self, double* d_others, int32_t* p_others,
                                      double* pts_others) {
  const int ns = n_self_pairs();
  ensure_snapshot(CollisionRequest());
  const mpg_distance_request req = r.to_c();
  check_status(mpg_distance_batch_req(world_->get(), q, n, ns, &req, d_self, p_self, pts_self, d_others, p_others,
                                      pts_others, MPG_MEM_HOST, nullptr),
               "mpg_distance_batch_req");
}

void PlanningWorld::distance_batch_device(const void* q, int64_t n, const DistanceRequest& r, void* d_self,
                                          void* p_self, void* pts_self, void* d_others, void* p_others,
                                          void* pts_others, void* stream) {
  r.check_supported();
  const int ns = n_self_pairs();
  ensure_snapshot(CollisionRequest());
  const mpg_distance_request req = r.to_c();
  check_status(mpg_distance_batch_req(world_->get(), static_cast<const double*>(q), n, ns, &req,
                                      static_cast<double*>(d_self), static_cast<int32_t*>(p_self),
                                      static_cast<double*>(pts_self), static_cast<double*>(d_others),
                                      static_cast<int32_t*>(p_others), static_cast<double*>(pts_others),
                                      MPG_MEM_DEVICE, stream),
               "mpg_distance_batch_req");
}

namespace {
// the WorldDistanceResult of a group's minimum pair p (DistanceResult with
// its nearest points, planning_world.cpp:512-525)
WorldDistanceResult distance_result(double d, int p, const std::vector<PairInfo>& pairs, const double* pts) {
  WorldDistanceResult r;
  if (p < 0) return r;
  const PairInfo& pi = pairs[p];
  r.min_distance = d;
  r.res.min_distance = d;
  for (int k = 0; k < 3; ++k) {
    r.res.nearest_points[0][k] = pts[k];
    r.res.nearest_points[1][k] = pts[3 + k];
  }
  r.distance_type = pi.collision_type;
  r.object_name1 = pi.object_name1;
  r.object_name2 = pi.object_name2;
  r.link_name1 = pi.link_name1;
  r.link_name2 = pi.link_name2;
  return r;
}
}  // namespace

WorldDistanceResult PlanningWorld::self_distance(const DistanceRequest& r) {
  r.check_supported();
  std::vector<double> s = current_state();
  double ds, dot, qs[6], qo[6];
  int32_t ps, po;
  distance_batch_ex(s.data(), 1, r, &ds, &ps, qs, &dot, &po, qo);
  return distance_result(ds, ps, pairs_, qs);
}
WorldDistanceResult PlanningWorld::distance_with_others(const DistanceRequest& r) {
  r.check_supported();
  std::vector<double> s = current_state();
  double ds, dot, qs[6], qo[6];
  int32_t ps, po;
  distance_batch_ex(s.data(), 1, r, &ds, &ps, qs, &dot, &po, qo);
  return distance_result(dot, po, pairs_, qo);
}
WorldDistanceResult PlanningWorld::distance_full(const DistanceRequest& r) {
  r.check_supported();
  std::vector<double> s = current_state();
  double ds, dot, qs[6], qo[6];
  int32_t ps, po;
  distance_batch_ex(s.data(), 1, r, &ds, &ps, qs, &dot, &po, qo);
  auto r1 = distance_result(ds, ps, pairs_, qs), r2 = distance_result(dot, po, pairs_, qo);
  return r1.min_distance < r2.min_distance ? r1 : r2;  // planning_world.cpp:718-719
}
// the reference ignores the request here (planning_world.h:271-273)
// the reference ignores the request here (planning_world.h:271-273: distanceFull())
double PlanningWorld::distance(const DistanceRequest&) { return distance_full().min_distance; }

void PlanningWorld::profile_enable(bool on) { check_status(mpg_profile_enable(device_world(), on ? 1 : 0), "mpg_profile_enable"); }
std::vector<PlanningWorld::StageTime> PlanningWorld::profile_read() {
  double ms[MPG_NUM_STAGES];
  int64_t n[MPG_NUM_STAGES], u[MPG_NUM_STAGES];
  check_status(mpg_profile_read(device_world(), ms, n, u, MPG_NUM_STAGES), "mpg_profile_read");
  std::vector<StageTime> out;
  for (int k = 0; k < MPG_NUM_STAGES; ++k) out.push_back({ms[k], n[k], u[k]});
  return out;
}

// random_utils.h:10-15: std::srand + OMPL's RNG seed (planner.cpp)
void set_global_seed(unsigned seed) {
  std::srand(seed);
  plan_rng_seed(seed);
}

}  // namespace mpgh

namespace mpgh {

std::pair<std::vector<double>, std::vector<double>> PlanningWorld::full_state_limits() {
  ensure_snapshot(CollisionRequest(), false);
  return {full_lo_, full_hi_};
}

std::vector<int64_t> PlanningWorld::sample_pair_counts(int64_t n, uint64_t seed) {
  if (n < 0) throw std::invalid_argument("sample_pair_counts: n < 0");
  ensure_snapshot(CollisionRequest(), false);
  if (!full_world_ || full_key_ != desc_key_) {
    DescBuilder f = *desc_;
    f.joint_q_source = full_src_;
    f.dof = full_dof_;
    full_world_ = std::make_unique<DeviceWorld>(f, default_device());
    full_key_ = desc_key_;
  }
  std::vector<int64_t> counts(pairs_.size(), 0);
  check_status(mpg_collide_count(full_world_->get(), full_lo_.data(), full_hi_.data(), n, seed, counts.data(), nullptr),
               "mpg_collide_count");
  return counts;
}

}  // namespace mpgh
