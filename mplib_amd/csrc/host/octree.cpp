// octree.cpp -- fcl::OcTree over octomap::OcTree, as PlanningWorld::addPointCloud
// (src/planning_world.cpp:102-110) and fcl.OcTree(vertices, resolution)
// (python/pybind_fcl.hpp:223-236) build it: updateNode(point3d(x, y, z), true)
// per point, lazy_eval = false.  Restated from octomap 1.9.8's published
// algorithm [ext]: float point3d, coordToKeyChecked = floor(coord / res) +
// 32768 on 16 levels, hit log-odds +0.85f clamped to [-2, 3.5], the early
// abort when the found leaf is already clamped, pruned-leaf expansion,
// pruning of 8 equal leaf children, parents holding their max child.
// The device only needs the occupied leaves (log-odds >= occupancy threshold
// 0) as boxes from FCL's getRootBV / computeChildBV recursion [ext FCL 0.7.0].
#include <cmath>
#include <stdexcept>

#include "host.hpp"

namespace mpgh {

namespace {

constexpr int kDepth = 16;
constexpr int kMaxKey = 32768;
constexpr float kHit = 0.85f, kClampMin = -2.0f, kClampMax = 3.5f;

struct Node {
  float v = 0.0f;
  std::unique_ptr<std::array<std::unique_ptr<Node>, 8>> ch;
};

bool has_children(const Node* n) {
  if (!n->ch) return false;
  for (auto& c : *n->ch)
    if (c) return true;
  return false;
}

int child_idx(const int key[3], int bit) {
  return ((key[0] >> bit) & 1) | (((key[1] >> bit) & 1) << 1) | (((key[2] >> bit) & 1) << 2);
}

Node* search(Node* n, const int key[3]) {
  if (!n) return nullptr;
  for (int bit = kDepth - 1; bit >= 0; --bit) {
    const int pos = child_idx(key, bit);
    if (n->ch && (*n->ch)[pos]) {
      n = (*n->ch)[pos].get();
    } else {
      return has_children(n) ? nullptr : n;  // a pruned leaf answers for its subtree
    }
  }
  return n;
}

bool prune(Node* n) {  // isNodeCollapsible + pruneNode
  if (!n->ch || !(*n->ch)[0] || has_children((*n->ch)[0].get())) return false;
  const float v0 = (*n->ch)[0]->v;
  for (int i = 1; i < 8; ++i) {
    const Node* c = (*n->ch)[i].get();
    if (!c || has_children(c) || !(c->v == v0)) return false;
  }
  n->v = v0;
  n->ch.reset();
  return true;
}

void update_recurs(Node* n, bool just_created, const int key[3], int depth) {
  if (depth < kDepth) {
    const int pos = child_idx(key, kDepth - 1 - depth);
    bool created = false;
    if (!n->ch || !(*n->ch)[pos]) {
      if (!has_children(n) && !just_created) {  // expandNode: 8 children with the node's value
        n->ch = std::make_unique<std::array<std::unique_ptr<Node>, 8>>();
        for (auto& c : *n->ch) {
          c = std::make_unique<Node>();
          c->v = n->v;
        }
      } else {
        if (!n->ch) n->ch = std::make_unique<std::array<std::unique_ptr<Node>, 8>>();
        (*n->ch)[pos] = std::make_unique<Node>();
        created = true;
      }
    }
    update_recurs((*n->ch)[pos].get(), created, key, depth + 1);
    if (!prune(n)) {  // updateOccupancyChildren: the max child log-odds
      float m = -std::numeric_limits<float>::max();
      for (auto& c : *n->ch)
        if (c && c->v > m) m = c->v;
      n->v = m;
    }
    return;
  }
  float v = n->v + kHit;  // updateNodeLogOdds
  if (v < kClampMin) v = kClampMin;
  if (v > kClampMax) v = kClampMax;
  n->v = v;
}

void collect(const Node* n, const double lo[3], const double hi[3], std::vector<std::array<double, 6>>& out) {
  if (!has_children(n)) {
    if (n->v >= 0.0f) out.push_back({lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]});
    return;
  }
  for (int i = 0; i < 8; ++i) {
    const Node* c = (*n->ch)[i].get();
    if (!c) continue;
    double clo[3], chi[3];
    for (int a = 0; a < 3; ++a) {  // computeChildBV
      const double mid = (lo[a] + hi[a]) * 0.5;
      clo[a] = ((i >> a) & 1) ? mid : lo[a];
      chi[a] = ((i >> a) & 1) ? hi[a] : mid;
    }
    collect(c, clo, chi, out);
  }
}

}  // namespace

OcTree::OcTree(double res) : resolution(res) {
  type = MPG_GEOM_OCTREE;
  kind = "OcTree";
  if (!(res > 0)) throw std::invalid_argument("OcTree resolution must be > 0");
}

OcTree::OcTree(const std::vector<Vec3>& points, double res) : OcTree(res) {
  std::unique_ptr<Node> root;
  const double inv = 1.0 / res;  // resolution_factor
  for (const auto& p : points) {
    int key[3];
    bool ok = true;
    for (int k = 0; k < 3; ++k) {
      const float c = (float)p[k];  // octomap::point3d is float
      const int s = (int)std::floor(inv * (double)c) + kMaxKey;
      if (s < 0 || s >= 2 * kMaxKey) {
        ok = false;
        break;
      }
      key[k] = s;
    }
    if (!ok) continue;
    Node* leaf = search(root.get(), key);
    if (leaf && leaf->v >= kClampMax) continue;  // no change at the clamping threshold
    bool created_root = false;
    if (!root) {
      root = std::make_unique<Node>();
      created_root = true;
    }
    update_recurs(root.get(), created_root, key, 0);
  }
  if (root) {
    const double delta = (double)(1 << kDepth) * res / 2;  // getRootBV
    const double lo[3] = {-delta, -delta, -delta}, hi[3] = {delta, delta, delta};
    collect(root.get(), lo, hi, leaves);
  }
}

}  // namespace mpgh
