// planner.cpp -- OMPLPlanner with batched device state validity.
// Reference: src/ompl_planner.{h,cpp} (MPlib) over OMPL 1.6.0 RRTConnect / RRT,
// DiscreteMotionValidator, CompoundStateSpace, RealVectorStateSpace,
// SO2StateSpace, GoalStates and PlannerInputStates (restated here; OMPL is not
// in this image).  See planner.hpp for the batching scheme.
#include "planner.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cmath>
#include <cstring>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <queue>
#include <stdexcept>
#include <thread>
#include <tuple>

namespace mpgh {

namespace {
constexpr double kPi = M_PI;                 // boost::math::constants::pi (SO2StateSpace)
constexpr double kRefPi = 3.14159265359;     // #define PI in ompl_planner.cpp:27
constexpr double kEps = std::numeric_limits<double>::epsilon();
using Clock = std::chrono::steady_clock;
double seconds_since(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }
}  // namespace

// ---------------------------------------------------------------------------
// state space (OMPL CompoundStateSpace of RealVector(1) / SO2, weights 1.0)
// ---------------------------------------------------------------------------
double PlanSpace::distance(const double* a, const double* b) const {
  // CompoundStateSpace::distance: sum_i weight_i * d_i; RealVector: sqrt(sum diff^2);
  // SO2: d = |a-b|, d > pi ? 2pi - d : d
  double dist = 0.0;
  for (int i = 0; i < dim; ++i) {
    double di;
    if (so2[i]) {
      const double d = std::fabs(a[i] - b[i]);
      di = d > kPi ? 2.0 * kPi - d : d;
    } else {
      // sqrt(fl(x * x)) == |x| exactly unless x * x underflows
      const double diff = a[i] - b[i];
      di = std::fabs(diff) > 1e-150 ? std::fabs(diff) : std::sqrt(diff * diff);
    }
    dist += 1.0 * di;
  }
  return dist;
}

double PlanSpace::distance_below(const double* a, const double* b, double bound) const {
  // the compound distance if it is < bound, else a value >= bound: partial
  // sums of non-negative terms never decrease, so stopping early is exact
  double dist = 0.0;
  for (int i = 0; i < dim; ++i) {
    double di;
    if (so2[i]) {
      const double d = std::fabs(a[i] - b[i]);
      di = d > kPi ? 2.0 * kPi - d : d;
    } else {
      const double diff = a[i] - b[i];
      di = std::fabs(diff) > 1e-150 ? std::fabs(diff) : std::sqrt(diff * diff);
    }
    dist += 1.0 * di;
    if (dist >= bound) return dist;
  }
  return dist;
}

void PlanSpace::interpolate(const double* a, const double* b, double t, double* out) const {
  for (int i = 0; i < dim; ++i) {
    if (!so2[i]) {  // RealVectorStateSpace::interpolate
      out[i] = a[i] + (b[i] - a[i]) * t;
      continue;
    }
    double diff = b[i] - a[i];  // SO2StateSpace::interpolate
    if (std::fabs(diff) <= kPi) {
      out[i] = a[i] + diff * t;
    } else {
      diff = diff > 0.0 ? 2.0 * kPi - diff : -2.0 * kPi - diff;
      double v = a[i] - diff * t;
      if (v > kPi)
        v -= 2.0 * kPi;
      else if (v < -kPi)
        v += 2.0 * kPi;
      out[i] = v;
    }
  }
}

bool PlanSpace::equal(const double* a, const double* b) const {
  for (int i = 0; i < dim; ++i)  // RealVector / SO2 equalStates: |diff| > 2 eps -> different
    if (so2[i] ? !(std::fabs(a[i] - b[i]) < 2.0 * kEps) : std::fabs(a[i] - b[i]) > 2.0 * kEps) return false;
  return true;
}

unsigned PlanSpace::valid_segment_count(const double* a, const double* b) const {
  // StateSpace::validSegmentCount: factor(1) * ceil(distance / longestValidSegment)
  return 1u * (unsigned)std::ceil(distance(a, b) / longest_valid_segment);
}

bool PlanSpace::satisfies_bounds(const double* s) const {
  for (int i = 0; i < dim; ++i) {
    if (so2[i]) {
      if (s[i] < -kPi || s[i] > kPi) return false;
    } else if (s[i] - kEps > hi[i] || s[i] + kEps < lo[i]) {
      return false;
    }
  }
  return true;
}

// ---------------------------------------------------------------------------
// RNG (ompl/util/RandomNumbers.cpp: RNGSeedGenerator + per-instance mt19937)
// ---------------------------------------------------------------------------
namespace {
struct SeedGenerator {
  bool seeded = false;
  std::mt19937 gen;
  std::uniform_int_distribution<> dist{1, 1000000000};
  unsigned next() {
    if (!seeded) {  // OMPL: first seed from the clock unless setSeed() was called
      gen.seed((unsigned)std::chrono::duration_cast<std::chrono::microseconds>(
                   std::chrono::system_clock::now().time_since_epoch()).count());
      seeded = true;
    }
    return (unsigned)dist(gen);
  }
};
SeedGenerator& seeds() {
  static SeedGenerator g;
  return g;
}
// std::rand() of random_sample_nearby (ompl_planner.cpp:77) as a private glibc
// TYPE_3 generator: the same sequence as rand() after srand(seed), immune to
// other rand() users in the process (the HIP runtime draws from it at init)
struct CRand {
  char buf[128];
  random_data rd{};
  CRand() { seed(1); }
  void seed(unsigned s) {
    rd = random_data{};
    initstate_r(s, buf, sizeof(buf), &rd);
  }
  int next() {
    int32_t r;
    random_r(&rd, &r);
    return (int)r;
  }
};
CRand& crand() {
  static CRand c;
  return c;
}
}  // namespace

PlanRNG::PlanRNG() : gen_(seeds().next()) {}

void plan_rng_seed(unsigned seed) {
  crand().seed(seed);
  auto& g = seeds();
  g.gen.seed(seed);
  g.dist.reset();
  g.seeded = true;
}

// ---------------------------------------------------------------------------
// planner
// ---------------------------------------------------------------------------
OMPLPlanner::OMPLPlanner(const std::shared_ptr<PlanningWorld>& world) : world_(world) {
  if (!world_) throw std::invalid_argument("OMPLPlanner: world is None");
  // build_state_space (ompl_planner.cpp:248-293): planned articulations in
  // std::map name order, move-group joints in move-group order
  PlanSpace& s = space_;
  for (const auto& art : world_->get_planned_articulations()) {
    const auto& pin = art->get_pinocchio_model();
    for (size_t id : art->get_move_group_joint_indices()) {
      const PinJoint& pj = pin->joints()[pin->user_joints().at(id)];
      if (pj.type >= MPG_JOINT_RUBX) {  // JointModelRU*: SO2StateSpace, limits +-PI
        s.so2.push_back(1);
        s.lo.push_back(-kRefPi);
        s.hi.push_back(kRefPi);
        s.revolute.push_back(0);
        s.max_extent += 1.0 * kPi;
        s.dim += 1;
      } else {  // RealVectorStateSpace(nq) with the joint limits
        double e2 = 0.0;
        for (int k = 0; k < pj.nq; ++k) {
          s.so2.push_back(0);
          s.lo.push_back(pj.lower[k]);
          s.hi.push_back(pj.upper[k]);
          e2 += (pj.upper[k] - pj.lower[k]) * (pj.upper[k] - pj.lower[k]);
        }
        s.revolute.push_back(pj.type <= MPG_JOINT_REVOLUTE_UNALIGNED ? 1 : 0);
        s.max_extent += 1.0 * std::sqrt(e2);
        s.dim += pj.nq;
      }
    }
  }
  if (s.dim != world_->state_dim())
    throw std::runtime_error("Dim of bound is different from dim of qpos " + std::to_string(s.dim) + " " +
                             std::to_string(world_->state_dim()));
  // SpaceInformation::setup: longestValidSegment = extent * 0.01
  s.longest_valid_segment = s.max_extent * 0.01;
}

void OMPLPlanner::check(const std::vector<double>& states, std::vector<uint8_t>& valid) {
  const int64_t n = (int64_t)(states.size() / (size_t)space_.dim);
  valid.assign((size_t)n, 0);
  if (n == 0) return;
  const auto t0 = Clock::now();
  if (custom_) {
    custom_(states.data(), n, valid.data());
  } else {
    flags_.resize((size_t)n);
    world_->collide_batch(states.data(), n, flags_.data(), nullptr);
    for (int64_t i = 0; i < n; ++i) valid[(size_t)i] = flags_[(size_t)i] ? 0 : 1;
  }
  stats_.check_seconds += seconds_since(t0);
  stats_.batches += 1;
  stats_.states_checked += n;
}

bool OMPLPlanner::is_valid(const std::vector<double>& s) {
  std::vector<uint8_t> v;
  check(s, v);
  return v[0] != 0;
}

std::vector<double> OMPLPlanner::random_sample_nearby(const std::vector<double>& start) {
  // ompl_planner.cpp:71-95: perturbation ratio (cnt+1)/1000 of the joint
  // range, clipped, first valid sample wins, up to 1001 attempts.  Attempts
  // are generated and validated 16 at a time (one batch each).
  const int d = space_.dim;
  int cnt = 0;
  const int kChunk = 16;
  while (cnt <= 1000) {
    std::vector<double> cand;
    int first = cnt;
    for (; cnt <= 1000 && cnt < first + kChunk; ++cnt) {
      const double ratio = (double)(cnt + 1) / 1000;
      for (int i = 0; i < d; ++i) {
        const double r = (double)crand().next() / RAND_MAX * 2 - 1;
        double v = start[(size_t)i] + (space_.hi[(size_t)i] - space_.lo[(size_t)i]) * ratio * r;
        if (v < space_.lo[(size_t)i])
          v = space_.lo[(size_t)i];
        else if (v > space_.hi[(size_t)i])
          v = space_.hi[(size_t)i];
        cand.push_back(v);
      }
    }
    std::vector<uint8_t> ok;
    check(cand, ok);
    for (size_t k = 0; k < ok.size(); ++k)
      if (ok[k]) {
        std::printf("successfully sampled a new state with a perturbation of %g%% joint limits.\n",
                    (double)(first + (int)k + 1) / 1000 * 100);
        std::fflush(stdout);
        return std::vector<double>(cand.begin() + (ptrdiff_t)(k * d), cand.begin() + (ptrdiff_t)((k + 1) * d));
      }
  }
  return start;
}

namespace {

enum Grow { TRAPPED, ADVANCED, REACHED };

// one RRT tree (OMPL Motion list + exact linear nearest neighbour)
struct Tree {
  int dim;
  std::vector<double> st;
  std::vector<int> parent, root;
  explicit Tree(int d) : dim(d) {}
  int size() const { return (int)parent.size(); }
  const double* state(int i) const { return st.data() + (size_t)i * dim; }
  int add(const double* s, int par) {
    st.insert(st.end(), s, s + dim);
    parent.push_back(par);
    root.push_back(par < 0 ? size() - 1 : root[(size_t)par]);
    return size() - 1;
  }
  // first strict minimum of the space distance (GNAT returns an exact nearest)
  int nearest(const PlanSpace& sp, const double* q, double* dist = nullptr) const {
    int best = -1;
    double bd = std::numeric_limits<double>::infinity();
    for (int i = 0; i < size(); ++i) {
      const double d = sp.distance_below(state(i), q, bd);
      if (d < bd) {
        bd = d;
        best = i;
      }
    }
    if (dist) *dist = bd;
    return best;
  }
};

// states DiscreteMotionValidator::checkMotion(s1, s2) validates: s2, then
// interpolate(s1, s2, j/nd) for j = 1..nd-1 (the bisection order does not
// change the outcome); s1 is assumed valid
void append_motion(const PlanSpace& sp, const double* s1, const double* s2, std::vector<double>& out) {
  out.insert(out.end(), s2, s2 + sp.dim);
  const unsigned nd = sp.valid_segment_count(s1, s2);
  if (nd < 2) return;
  const size_t base = out.size();
  out.resize(base + (size_t)(nd - 1) * sp.dim);
  for (unsigned j = 1; j < nd; ++j) sp.interpolate(s1, s2, (double)j / (double)nd, out.data() + base + (j - 1) * sp.dim);
}

// the states growTree() validates for a motion from `from` (in the tree) to
// `to`: start tree checkMotion(from, to); goal tree isValid(to) &&
// checkMotion(to, from)
void append_grow(const PlanSpace& sp, bool start_tree, const double* from, const double* to,
                 std::vector<double>& out) {
  if (start_tree) {
    append_motion(sp, from, to, out);
  } else {
    out.insert(out.end(), to, to + sp.dim);
    append_motion(sp, to, from, out);
  }
}

bool all_valid(const std::vector<uint8_t>& v, size_t a, size_t b) {
  for (size_t i = a; i < b; ++i)
    if (!v[i]) return false;
  return true;
}

// bits of a state -> 64-bit key (validity cache, hypotheses, nearest memo)
uint64_t hash_state(const double* s, int dim) {
  uint64_t h = 0x9e3779b97f4a7c15ull;
  for (int k = 0; k < dim; ++k) {
    uint64_t x;
    std::memcpy(&x, s + k, 8);
    h ^= x + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
    h *= 0xff51afd7ed558ccdull;
  }
  return h ^ (h >> 33);
}

// state -> validity, open addressing over a pool of the states' bits (no
// per-entry allocation: the planner queries it hundreds of times per iteration)
class ValidityCache {
 public:
  explicit ValidityCache(int dim) : dim_(dim), slots_(1024, -1) {}
  // 1 valid, 0 invalid, -1 unknown
  int find(const double* s) const { return find_h(s, hash_state(s, dim_)); }
  int find_h(const double* s, uint64_t h) const {
    size_t i = h & (slots_.size() - 1);
    for (;; i = (i + 1) & (slots_.size() - 1)) {
      const int e = slots_[i];
      if (e < 0) return -1;
      if (std::memcmp(pool_.data() + (size_t)e * dim_, s, sizeof(double) * dim_) == 0) return val_[(size_t)e];
    }
  }
  void put(const double* s, uint8_t v) {
    const uint64_t h = hash_state(s, dim_);
    if (find_h(s, h) >= 0) return;
    if (2 * (val_.size() + 1) > slots_.size()) grow();
    insert_index(h, (int)val_.size());
    pool_.insert(pool_.end(), s, s + dim_);
    val_.push_back(v);
  }

 private:
  void insert_index(uint64_t h, int e) {
    size_t i = h & (slots_.size() - 1);
    while (slots_[i] >= 0) i = (i + 1) & (slots_.size() - 1);
    slots_[i] = e;
  }
  void grow() {
    slots_.assign(slots_.size() * 2, -1);
    for (size_t e = 0; e < val_.size(); ++e) insert_index(hash_state(pool_.data() + e * dim_, dim_), (int)e);
  }
  int dim_;
  std::vector<int> slots_;
  std::vector<double> pool_;
  std::vector<uint8_t> val_;
};

struct GoalSet {  // ob::GoalStates + PlannerInputStates goal sampling
  const PlanSpace* sp;
  std::vector<double> st;
  std::vector<uint8_t> usable;  // satisfiesBounds && isValid (pure function of the state)
  size_t sample_pos = 0, sampled = 0;
  size_t count() const { return st.size() / (size_t)sp->dim; }
  const double* state(size_t i) const { return st.data() + i * sp->dim; }
  const double* sample_goal() {  // GoalStates::sampleGoal: round robin
    const double* s = state(sample_pos);
    sample_pos = (sample_pos + 1) % count();
    return s;
  }
  double distance_goal(const double* q) const {
    double best = std::numeric_limits<double>::infinity();
    for (size_t i = 0; i < count(); ++i) best = std::min(best, sp->distance(q, state(i)));
    return best;
  }
  // PlannerInputStates::nextGoal(ptc): keep sampling until a usable goal or
  // the goal set is exhausted; nextGoal() (always-terminating ptc): one sample
  const double* next_goal(bool keep_trying) {
    while (sampled < count()) {
      const size_t idx = sample_pos;
      const double* s = sample_goal();
      sampled += 1;
      if (usable[idx]) return s;
      if (!keep_trying) break;
    }
    return nullptr;
  }
};

std::vector<std::vector<double>> path_rows(const PlanSpace& sp, const std::vector<const double*>& states) {
  std::vector<std::vector<double>> out;
  out.reserve(states.size());
  for (const double* s : states) out.emplace_back(s, s + sp.dim);
  return out;
}

// start tree root .. sm, then gm .. goal tree root (RRTConnect's solution path)
template <class T>
std::vector<const double*> connect_path(const T& ts, int sm, const T& tg, int gm) {
  std::vector<const double*> p1, out;
  for (int m = sm; m >= 0; m = ts.parent[(size_t)m]) p1.push_back(ts.state(m));
  for (auto it = p1.rbegin(); it != p1.rend(); ++it) out.push_back(*it);
  for (int m = gm; m >= 0; m = tg.parent[(size_t)m]) out.push_back(tg.state(m));
  return out;
}
template <class T>
std::vector<const double*> root_path(const T& t, int m) {
  std::vector<const double*> rev;
  for (; m >= 0; m = t.parent[(size_t)m]) rev.push_back(t.state(m));
  return std::vector<const double*>(rev.rbegin(), rev.rend());
}

// ---------------------------------------------------------------------------
// RRTConnect with outcome-tree speculation
//
// The serial loop (above, OMPL's as written) asks for one motion's validity
// at a time; each answer decides what is asked next.  Here the loop runs as
// `advance` over a Branch: the two trees (committed nodes plus an overlay of
// nodes added since the last batch), the iteration counter, the goal sampler
// position and the position inside the iteration.  The real branch stops at
// the first motion whose states are not in the validity cache.  From that
// point an outcome tree is explored best first: each explored node is a copy
// of the branch that assumes an outcome (valid / invalid) for every motion on
// its path and stops at the next unknown motion; its probability is the
// product of the outcome rates measured so far in this plan, per motion kind
// and tree: extension, first connect step, later connect steps, each for the
// start and the goal tree (on cfg5 ~0.65, ~0.07 and ~0.77 valid: the first
// step towards the other tree rarely gets through, a chain that has started
// usually continues; splitting by tree saves another ~13 % of the batches).  One device batch carries
// the unknown states of the real motion and of the explored nodes; while it
// runs on the GPU (a helper thread waits on the synchronous C call) the host
// explores deeper.
// When the answers arrive the real branch advances through the cache, the
// explored node it stops at becomes the new root (its subtree is kept,
// everything else dropped), and the unsent states below it form the next
// batch.  Speculation only chooses which states ride in a batch; the real
// branch consults nothing but the cache, so the tree is the serial loop's.
// ---------------------------------------------------------------------------

// committed tree nodes, rows plus columns (the nearest scan reads columns)
struct BaseTree {
  int dim = 0;
  std::vector<double> st;
  std::vector<std::vector<double>> col;
  std::vector<int> parent;
  void init(int d) {
    dim = d;
    col.assign((size_t)d, {});
  }
  int size() const { return (int)parent.size(); }
  const double* state(int i) const { return st.data() + (size_t)i * dim; }
  void add(const double* s, int par) {
    st.insert(st.end(), s, s + dim);
    for (int k = 0; k < dim; ++k) col[(size_t)k].push_back(s[k]);
    parent.push_back(par);
  }
};

// compound distances of nodes i0..i0+n of a column store to q, summed per node
// in subspace order exactly as PlanSpace::distance does (vectorised across nodes)
#pragma GCC push_options
#pragma GCC optimize("O3", "no-math-errno")
__attribute__((target_clones("avx2", "default"))) void l1_columns(const double* const* col, const uint8_t* so2,
                                                                  int dim, const double* q, int64_t i0, int n,
                                                                  double* out) {
  for (int i = 0; i < n; ++i) out[i] = 0.0;
  for (int k = 0; k < dim; ++k) {
    const double* c = col[k] + i0;
    const double qk = q[k];
    if (so2[k]) {
      for (int i = 0; i < n; ++i) {
        const double dd = std::fabs(c[i] - qk);
        out[i] += dd > kPi ? 2.0 * kPi - dd : dd;
      }
    } else {
      for (int i = 0; i < n; ++i) {
        const double diff = c[i] - qk;
        const double a = std::fabs(diff);
        out[i] += a > 1e-150 ? a : std::sqrt(diff * diff);
      }
    }
  }
}
#pragma GCC pop_options

// nearest committed node of tree t to q (first strict minimum in insertion
// order), memoised per (tree, query) and extended when the tree grows
class NearMemo {
 public:
  explicit NearMemo(const PlanSpace& sp) : sp_(sp), slots_(4096, -1) {}
  std::pair<int, double> get(const BaseTree& bt, int t, const double* q) {
    const int d = sp_.dim;
    const uint64_t h = hash_state(q, d) ^ (0x632be59bd9b4e019ull * (uint64_t)(t + 1));
    size_t i = h & (slots_.size() - 1);
    int e = -1;
    for (;; i = (i + 1) & (slots_.size() - 1)) {
      e = slots_[i];
      if (e < 0) break;
      const Ent& x = ents_[(size_t)e];
      if (x.t == t && std::memcmp(qpool_.data() + x.qoff, q, sizeof(double) * d) == 0) break;
    }
    if (e < 0) {
      if (2 * (ents_.size() + 1) > slots_.size()) {
        if (ents_.size() >= (1u << 16)) {  // bound the memory of long runs: start over
          ents_.clear();
          qpool_.clear();
          slots_.assign(4096, -1);
        } else {
          grow();
        }
        return get(bt, t, q);
      }
      e = (int)ents_.size();
      slots_[i] = e;
      ents_.push_back(Ent{t, qpool_.size(), -1, std::numeric_limits<double>::infinity(), 0});
      qpool_.insert(qpool_.end(), q, q + d);
    }
    Ent& x = ents_[(size_t)e];
    extend(bt, qpool_.data() + x.qoff, x);
    return {x.best, x.dist};
  }
  // the same for the uniform sample of iteration `it` (the extension's
  // query): indexed by the iteration, no hashing
  std::pair<int, double> get_sample(const BaseTree& bt, int t, int64_t it, const double* q) {
    std::vector<Ent>& v = by_it_[t];
    if ((int64_t)v.size() <= it) v.resize((size_t)it + 1, Ent{t, 0, -1, std::numeric_limits<double>::infinity(), 0});
    Ent& x = v[(size_t)it];
    extend(bt, q, x);
    return {x.best, x.dist};
  }

 private:
  struct Ent {
    int t;
    size_t qoff;
    int best;
    double dist;
    int upto;
  };
  // fold the tree nodes added since the entry's last query into its minimum
  void extend(const BaseTree& bt, const double* q, Ent& x) {
    if (x.upto >= bt.size()) return;
    const int d = sp_.dim;
    cols_.resize((size_t)d);
    for (int k = 0; k < d; ++k) cols_[(size_t)k] = bt.col[(size_t)k].data();
    double buf[256];
    for (int i0 = x.upto; i0 < bt.size(); i0 += 256) {
      const int n = std::min(256, bt.size() - i0);
      l1_columns(cols_.data(), sp_.so2.data(), d, q, i0, n, buf);
      for (int k = 0; k < n; ++k)
        if (buf[k] < x.dist) {
          x.dist = buf[k];
          x.best = i0 + k;
        }
    }
    x.upto = bt.size();
  }
  std::vector<Ent> by_it_[2];
  void grow() {
    slots_.assign(slots_.size() * 2, -1);
    for (size_t e = 0; e < ents_.size(); ++e) {
      const Ent& x = ents_[e];
      const uint64_t h = hash_state(qpool_.data() + x.qoff, sp_.dim) ^ (0x632be59bd9b4e019ull * (uint64_t)(x.t + 1));
      size_t i = h & (slots_.size() - 1);
      while (slots_[i] >= 0) i = (i + 1) & (slots_.size() - 1);
      slots_[i] = (int)e;
    }
  }
  const PlanSpace& sp_;
  std::vector<int> slots_;
  std::vector<Ent> ents_;
  std::vector<double> qpool_;
  std::vector<const double*> cols_;
};

// one validity batch on the device from a helper thread, so that the planner
// thread keeps exploring while the GPU works (the C call is synchronous).
// Both sides spin for at most kSpin (a batch round trip is ~40 us, and the
// planner submits the next batch right after reading a result), then block
// on a condition variable: between plans and during long host phases no core
// is held.  The destructor lets an in-flight batch finish before it stops the
// helper (a ConnectEngine unwinding between submit() and result()).
class AsyncCheck {
 public:
  using BatchFn = std::function<int(const double*, int64_t, uint8_t*)>;
  explicit AsyncCheck(mpg_world* w)
      : AsyncCheck([w](const double* q, int64_t n, uint8_t* f) {
          return mpg_collide_batch(w, q, n, f, nullptr, MPG_MEM_HOST, nullptr);
        }) {}
  explicit AsyncCheck(BatchFn fn) : fn_(std::move(fn)), th_([this] { loop(); }) {}
  ~AsyncCheck() {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_done_.wait(lk, [&] { return state_.load(std::memory_order_acquire) != kWork; });
      state_.store(kQuit, std::memory_order_release);
    }
    cv_work_.notify_one();
    th_.join();
  }
  void submit(const std::vector<double>& states, int dim) {
    q_ = states;
    n_ = (int64_t)(states.size() / (size_t)dim);
    flags_.assign((size_t)n_, 0);
    {
      std::lock_guard<std::mutex> lk(mu_);
      state_.store(kWork, std::memory_order_release);
    }
    cv_work_.notify_one();
  }
  bool done() const { return state_.load(std::memory_order_acquire) == kDone; }
  // valid[i] for the submitted states; throws on a device error
  void result(std::vector<uint8_t>& valid) {
    if (!spin_until([&] { return done(); })) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_done_.wait(lk, [&] { return done(); });
    }
    state_.store(kIdle, std::memory_order_relaxed);
    check_status(rc_, "mpg_collide_batch");
    valid.resize((size_t)n_);
    for (int64_t i = 0; i < n_; ++i) valid[(size_t)i] = flags_[(size_t)i] ? 0 : 1;
  }

 private:
  static constexpr int kIdle = 0, kWork = 1, kDone = 2, kQuit = 3;
  static constexpr std::chrono::microseconds kSpin{200};
  template <class Pred>
  static bool spin_until(Pred pred) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0;; ++k) {
      if (pred()) return true;
      __builtin_ia32_pause();
      if ((k & 63) == 63 && std::chrono::steady_clock::now() - t0 > kSpin) return pred();
    }
  }
  void loop() {
    for (;;) {
      int s = kIdle;
      auto ready = [&] {
        s = state_.load(std::memory_order_acquire);
        return s == kWork || s == kQuit;
      };
      if (!spin_until(ready)) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_work_.wait(lk, ready);
      }
      if (s == kQuit) return;
      rc_ = fn_(q_.data(), n_, flags_.data());
      {
        std::lock_guard<std::mutex> lk(mu_);
        state_.store(kDone, std::memory_order_release);
      }
      cv_done_.notify_all();
    }
  }
  BatchFn fn_;
  std::vector<double> q_;
  std::vector<uint8_t> flags_;
  int64_t n_ = 0;
  int rc_ = 0;
  std::atomic<int> state_{kIdle};
  std::mutex mu_;
  std::condition_variable cv_work_, cv_done_;
  std::thread th_;  // last: started after every member above exists

};

// CPU self-test of AsyncCheck's shutdown (pymp._selftest): a fake batch that
// takes `batch_ms`; with in_flight the helper is destroyed between submit()
// and result(), as a ConnectEngine that throws there would.  Returns the
// destructor's wall time in ms (it waits for the batch, it never hangs).
double async_check_selftest_impl(double batch_ms, bool in_flight) {
  std::atomic<int> calls{0};
  auto t0 = std::chrono::steady_clock::now();
  {
    AsyncCheck a([&](const double*, int64_t n, uint8_t* f) {
      std::this_thread::sleep_for(std::chrono::duration<double, std::milli>(batch_ms));
      for (int64_t i = 0; i < n; ++i) f[i] = (uint8_t)(i & 1);
      ++calls;
      return 0;
    });
    std::vector<double> st(6, 0.0);
    a.submit(st, 2);
    if (!in_flight) {
      std::vector<uint8_t> v;
      a.result(v);
      if (v.size() != 3 || v[0] != 1 || v[1] != 0) throw std::runtime_error("AsyncCheck selftest: bad result");
      a.submit(st, 3);
      a.result(v);
      if (v.size() != 2) throw std::runtime_error("AsyncCheck selftest: bad result");
    }
    t0 = std::chrono::steady_clock::now();
  }  // destructor
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (calls.load() != (in_flight ? 1 : 2)) throw std::runtime_error("AsyncCheck selftest: batch count");
  return ms;
}

class ConnectEngine {
 public:
  using SampleFn = std::function<void(double*)>;
  using TimeoutFn = std::function<bool()>;
  using CheckFn = std::function<void(const std::vector<double>&, std::vector<uint8_t>&)>;

  ConnectEngine(const PlanSpace& sp, const GoalSet& goals, const std::vector<double>& start, double maxd,
                OMPLPlanner::Stats& stats, SampleFn sample, TimeoutFn timed_out, CheckFn check, mpg_world* dev,
                int spec_nodes)
      : sp_(sp), d_(sp.dim), goals_(goals), maxd_(maxd), stats_(stats), sample_fn_(std::move(sample)),
        timed_out_(std::move(timed_out)), check_(std::move(check)), spec_nodes_(spec_nodes), vc_(sp.dim),
        memo_(sp), rbuf_((size_t)sp.dim), xbuf_((size_t)sp.dim) {
    base_[0].init(d_);
    base_[1].init(d_);
    base_[0].add(start.data(), -1);
    if (dev) async_.reset(new AsyncCheck(dev));
  }

  // (status, path) as the serial loop returns them
  std::pair<std::string, std::vector<const double*>> run() {
    Branch& R = real_;
    Blocked rb;
    for (;;) {
      const Adv a = advance(R, true, 0, rb);
      if (a == A_SOLVED) {
        commit();
        int sm = R.tgi_start ? R.xmotion : R.added;
        int gm = R.tgi_start ? R.added : R.xmotion;
        if (base_[0].parent[(size_t)sm] >= 0)
          sm = base_[0].parent[(size_t)sm];
        else
          gm = base_[1].parent[(size_t)gm];
        sizes();
        return {"Exact solution", connect_path(base_[0], sm, base_[1], gm)};
      }
      if (a != A_BLOCKED) break;  // timeout or no goal
      batch_round(rb);
    }
    commit();
    sizes();
    if (approxsol_ >= 0) return {"Approximate solution", root_path(base_[0], approxsol_)};
    return {"Timeout", {}};
  }

 private:
  enum Adv { A_BLOCKED, A_SOLVED, A_END, A_LIMIT };
  // motion kinds of the outcome model: extension, first connect step, later
  // connect steps; + 3 when the motion grows the goal tree
  enum Kind { K_EXT = 0, K_CONN = 1, K_CONN2 = 2 };
  struct Branch {
    std::vector<double> ost[2];  // overlay: nodes added since the last commit
    std::vector<int> opar[2];    // their parents (global node indices)
    int64_t it = 0;              // iteration (index of its uniform sample)
    bool start_tree = true;      // RRTConnect::startTree_ before iteration `it`
    size_t g_sampled = 0, g_pos = 0;
    int phase = 0;  // 0 iteration start, 1 extension, 2 connect
    int tr = 0;     // tree extended in this iteration (0 start, 1 goal)
    std::vector<double> target;
    int added = -1, xmotion = -1, n_conn = 0;
    bool tgi_start = false;
    std::vector<uint64_t> hv, hinv;  // assumed valid states, assumed invalid motions
  };
  struct Blocked {
    std::vector<double> st;  // the motion's states not known yet
    std::vector<uint64_t> h;
    uint64_t key = 0;
    int kind = K_EXT;
  };
  struct SNode {
    Branch br;  // stopped at `blk`
    Blocked blk;
    double p = 1.0;  // probability of reaching it from the root
    int child[2] = {-1, -1};  // [outcome invalid, valid]: -1 unexplored, -2 ends, else node
    bool sent = false;        // its unknown states went into a batch
  };

  // ---- trees ----
  int tree_size(const Branch& b, int t) const { return base_[t].size() + (int)b.opar[t].size(); }
  const double* node(const Branch& b, int t, int gi) const {
    const int nb = base_[t].size();
    return gi < nb ? base_[t].state(gi) : b.ost[t].data() + (size_t)(gi - nb) * d_;
  }
  int add_node(Branch& b, int t, const double* s, int par) {
    b.ost[t].insert(b.ost[t].end(), s, s + d_);
    b.opar[t].push_back(par);
    return tree_size(b, t) - 1;
  }
  int nearest(const Branch& b, int t, const double* q, int64_t sample_it = -1) {
    auto bn = sample_it >= 0 ? memo_.get_sample(base_[t], t, sample_it, q) : memo_.get(base_[t], t, q);
    int best = bn.first;
    double bd = bn.second;
    const int nb = base_[t].size();
    for (size_t k = 0; k < b.opar[t].size(); ++k) {
      const double dd = sp_.distance_below(b.ost[t].data() + k * d_, q, bd);
      if (dd < bd) {
        bd = dd;
        best = nb + (int)k;
      }
    }
    return best;
  }
  const double* sample(int64_t it) {
    while (samp0_ + (int64_t)(samp_.size() / (size_t)d_) <= it) {
      const size_t o = samp_.size();
      samp_.resize(o + (size_t)d_);
      sample_fn_(samp_.data() + o);
    }
    return samp_.data() + (size_t)(it - samp0_) * d_;
  }
  const double* next_goal(Branch& b, bool keep_trying) const {  // GoalSet::next_goal on the branch's position
    const size_t n = goals_.count();
    while (b.g_sampled < n) {
      const size_t idx = b.g_pos;
      b.g_pos = (b.g_pos + 1) % n;
      b.g_sampled += 1;
      if (goals_.usable[idx]) return goals_.state(idx);
      if (!keep_trying) break;
    }
    return nullptr;
  }

  // ---- validity: 1 valid, 0 invalid, -1 unknown (blk gets the unknown states)
  int status(const Branch& b, const std::vector<double>& mot, Blocked& blk) const {
    const size_t n = mot.size() / (size_t)d_;
    blk.st.clear();
    blk.h.clear();
    uint64_t key = 0x2545f4914f6cdd1dull;
    bool invalid = false;
    for (size_t i = 0; i < n; ++i) {
      const double* s = mot.data() + i * d_;
      const uint64_t h = hash_state(s, d_);
      key = (key ^ h) * 0x9e3779b97f4a7c15ull + (key >> 29);
      const int v = vc_.find_h(s, h);
      if (v == 0) invalid = true;
      if (v < 0 && std::find(b.hv.begin(), b.hv.end(), h) == b.hv.end()) {
        blk.st.insert(blk.st.end(), s, s + d_);
        blk.h.push_back(h);
      }
    }
    if (invalid) return 0;
    if (blk.h.empty()) return 1;
    blk.key = key;
    if (std::find(b.hinv.begin(), b.hinv.end(), key) != b.hinv.end()) return 0;
    return -1;
  }
  void record(int kind, int v) {
    n_out_[kind] += 1;
    n_ok_[kind] += v;
  }
  double prob(int kind, int outcome) const {
    const double pv = (n_ok_[kind] + 1.0) / (n_out_[kind] + 2.0);
    return outcome ? pv : 1.0 - pv;
  }

  // ---- the serial loop, resumable: runs b until a motion's validity is
  // unknown (A_BLOCKED, blk = that motion), a connection (A_SOLVED) or the end
  // (real: timeout / no goal; speculative: max_iters iterations, A_LIMIT)
  Adv advance(Branch& b, bool real, int max_iters, Blocked& blk) {
    int iters = 0;
    for (;;) {
      if (b.phase == 0) {
        if (real) {
          if (timed_out_()) return A_END;
          stats_.iterations += 1;
        } else if (++iters > max_iters) {
          return A_LIMIT;
        }
        b.tr = b.start_tree ? 0 : 1;
        b.start_tree = !b.start_tree;
        const int gsize = tree_size(b, 1);
        if (gsize == 0 || b.g_sampled < (size_t)gsize / 2) {
          const double* g = next_goal(b, gsize == 0);
          if (g) add_node(b, 1, g, -1);
          if (tree_size(b, 1) == 0) return A_END;
        }
        b.phase = 1;
      }
      if (b.phase == 1) {  // extension: growTree(tree, rstate)
        const double* r = sample(b.it);
        std::copy(r, r + d_, rbuf_.begin());
        const int n = nearest(b, b.tr, rbuf_.data(), b.it);
        const double* nst = node(b, b.tr, n);
        const double* ds = rbuf_.data();
        const double dd = sp_.distance(nst, rbuf_.data());
        bool trapped = false;
        if (dd > maxd_) {
          sp_.interpolate(nst, rbuf_.data(), maxd_ / dd, xbuf_.data());
          trapped = sp_.equal(nst, xbuf_.data());
          ds = xbuf_.data();
        }
        if (!trapped) {
          mot_.clear();
          append_grow(sp_, b.tr == 0, nst, ds, mot_);
          const int v = status(b, mot_, blk);
          if (v < 0) {
            blk.kind = K_EXT + 3 * b.tr;
            return A_BLOCKED;
          }
          if (real) record(K_EXT + 3 * b.tr, v);
          trapped = !v;
          if (trapped && real) stats_.ext_trapped += 1;
        }
        if (trapped) {
          b.it += 1;
          b.phase = 0;
          continue;
        }
        b.target.assign(ds, ds + d_);
        b.added = add_node(b, b.tr, ds, n);
        b.xmotion = b.added;
        b.tgi_start = b.tr == 1;  // tgi.start = the connect tree is the start tree
        b.n_conn = 0;
        b.phase = 2;
      }
      // connect: growTree(other, target) while ADVANCED
      const int o = 1 - b.tr;
      const int n = nearest(b, o, b.target.data());
      const double* nst = node(b, o, n);
      const double* ds = b.target.data();
      const double dd = sp_.distance(nst, b.target.data());
      Grow g = REACHED;
      bool need = true;
      if (dd > maxd_) {
        sp_.interpolate(nst, b.target.data(), maxd_ / dd, xbuf_.data());
        ds = xbuf_.data();
        g = ADVANCED;
        if (sp_.equal(nst, xbuf_.data())) {
          g = TRAPPED;
          need = false;
        }
      }
      if (need) {
        mot_.clear();
        append_grow(sp_, o == 0, nst, ds, mot_);
        const int v = status(b, mot_, blk);
        const int kind = (b.n_conn == 0 ? K_CONN : K_CONN2) + 3 * o;
        if (v < 0) {
          blk.kind = kind;
          return A_BLOCKED;
        }
        if (real) record(kind, v);
        if (v)
          b.xmotion = add_node(b, o, ds, n);
        else
          g = TRAPPED;
      }
      if (b.n_conn++ == 0 && g == TRAPPED) b.tgi_start = !b.tgi_start;
      if (g == REACHED) return A_SOLVED;
      if (g == TRAPPED) {
        if (real && b.tgi_start) {  // approximate solution bookkeeping on the start tree
          const double dist = goals_.distance_goal(node(b, 0, b.xmotion));
          if (dist < approxdif_) {
            approxdif_ = dist;
            approxsol_ = b.xmotion;
          }
        }
        b.it += 1;
        b.phase = 0;
      }
    }
  }

  // move the real branch's overlay into the committed trees
  void commit() {
    for (int t = 0; t < 2; ++t) {
      for (size_t k = 0; k < real_.opar[t].size(); ++k) base_[t].add(real_.ost[t].data() + k * d_, real_.opar[t][k]);
      real_.ost[t].clear();
      real_.opar[t].clear();
    }
  }
  void sizes() {
    stats_.start_tree = base_[0].size();
    stats_.goal_tree = base_[1].size();
  }

  // explore outcome `o` of node `pi`'s motion
  void expand(int pi, int o) {
    SNode c;
    c.br = nodes_[(size_t)pi].br;
    const Blocked& pb = nodes_[(size_t)pi].blk;
    if (o)
      c.br.hv.insert(c.br.hv.end(), pb.h.begin(), pb.h.end());
    else
      c.br.hinv.push_back(pb.key);
    c.p = nodes_[(size_t)pi].p * prob(pb.kind, o);
    stats_.spec_nodes += 1;
    if (advance(c.br, false, kMaxSpecIters, c.blk) != A_BLOCKED) {
      nodes_[(size_t)pi].child[o] = -2;
      return;
    }
    const int ci = (int)nodes_.size();
    nodes_[(size_t)pi].child[o] = ci;
    nodes_.push_back(std::move(c));
    push_children(ci);
  }
  void push_children(int i) {
    const SNode& s = nodes_[(size_t)i];
    for (int o = 0; o < 2; ++o)
      if (s.child[o] == -1) frontier_.emplace(s.p * prob(s.blk.kind, o), i, o);
  }
  bool expand_best() {
    while (!frontier_.empty()) {
      const auto top = frontier_.top();
      frontier_.pop();
      if (std::get<0>(top) < kMinProb) {
        frontier_ = {};
        return false;
      }
      if (nodes_[(size_t)std::get<1>(top)].child[std::get<2>(top)] != -1) continue;
      expand(std::get<1>(top), std::get<2>(top));
      return true;
    }
    return false;
  }

  // the real branch is blocked at `rb`: keep the explored subtree the real
  // outcomes lead to (or start a new one), send its unknown states as one
  // batch, explore while the batch runs, store the answers
  void batch_round(const Blocked& rb) {
    const auto t0 = Clock::now();
    // descend along the real outcomes from the previous root
    int cur = nodes_.empty() ? -1 : 0;
    while (cur >= 0) {
      const Blocked& b = nodes_[(size_t)cur].blk;
      int v = 1;
      for (size_t i = 0; i < b.h.size() && v != 0; ++i) {
        const int x = vc_.find_h(b.st.data() + i * d_, b.h[i]);
        if (x == 0) v = 0;
        else if (x < 0) v = -1;
      }
      if (v < 0) break;
      cur = nodes_[(size_t)cur].child[v];
    }
    const size_t n0 = real_.opar[0].size(), n1 = real_.opar[1].size();
    bool keep = cur >= 0 && nodes_[(size_t)cur].blk.key == rb.key && nodes_[(size_t)cur].blk.h == rb.h &&
                nodes_[(size_t)cur].br.it == real_.it && nodes_[(size_t)cur].br.opar[0].size() == n0 &&
                nodes_[(size_t)cur].br.opar[1].size() == n1;
    if (!keep) stats_.spec_resets += 1;
    commit();
    std::vector<SNode> kept;
    frontier_ = {};
    if (keep) {  // re-root: compact the subtree, probabilities relative to it
      std::vector<int> q{cur};
      std::vector<int> idx(nodes_.size(), -1);
      idx[(size_t)cur] = 0;
      kept.push_back(std::move(nodes_[(size_t)cur]));
      kept[0].p = 1.0;
      for (size_t h = 0; h < q.size(); ++h) {
        const int ni = idx[(size_t)q[h]];
        for (int o = 0; o < 2; ++o) {
          const int c = kept[(size_t)ni].child[o];
          if (c < 0) continue;
          idx[(size_t)c] = (int)kept.size();
          kept[(size_t)ni].child[o] = (int)kept.size();
          SNode s = std::move(nodes_[(size_t)c]);
          s.p = kept[(size_t)ni].p * prob(kept[(size_t)ni].blk.kind, o);
          for (int t = 0; t < 2; ++t) {  // drop the committed prefix of the overlay
            const size_t m = t ? n1 : n0;
            s.br.ost[t].erase(s.br.ost[t].begin(), s.br.ost[t].begin() + (ptrdiff_t)(m * d_));
            s.br.opar[t].erase(s.br.opar[t].begin(), s.br.opar[t].begin() + (ptrdiff_t)m);
          }
          kept.push_back(std::move(s));
          q.push_back(c);
        }
      }
      kept[0].br = real_;
      kept[0].blk = rb;
      kept[0].sent = false;
    } else {
      SNode root;
      root.br = real_;
      root.blk = rb;
      kept.push_back(std::move(root));
    }
    nodes_ = std::move(kept);
    for (size_t i = 0; i < nodes_.size(); ++i) push_children((int)i);
    // synchronous exploration when the kept subtree is small (or no GPU wait to hide it)
    const int target_nodes = spec_nodes_ >= 0 ? spec_nodes_ : async_ ? kSyncNodes : kSyncCheckerNodes;
    while ((int)nodes_.size() < target_nodes && (int)nodes_.size() < kMaxNodes && expand_best()) {
    }
    // the batch: unknown states of the nodes not sent yet, by probability
    order_.clear();
    size_t cand = 0;
    for (size_t i = 0; i < nodes_.size(); ++i)
      if (!nodes_[i].sent) {
        order_.push_back((int)i);
        cand += nodes_[i].blk.h.size();
      }
    std::stable_sort(order_.begin(), order_.end(),
                     [&](int a, int b) { return nodes_[(size_t)a].p > nodes_[(size_t)b].p; });
    batch_.clear();
    seen_reset(cand);
    for (int i : order_) {
      if (batch_.size() >= (size_t)kMaxBatch * d_) break;
      SNode& nd = nodes_[(size_t)i];
      const Blocked& b = nd.blk;
      for (size_t k = 0; k < b.h.size(); ++k) {
        const double* s = b.st.data() + k * d_;
        if (vc_.find_h(s, b.h[k]) >= 0 || !mark(b.h[k])) continue;
        batch_.insert(batch_.end(), s, s + d_);
      }
      nd.sent = true;
    }
    stats_.t_spec += seconds_since(t0);
    const auto tc = Clock::now();
    if (async_) {
      async_->submit(batch_, d_);
      const auto tw = Clock::now();
      const int64_t n_before = stats_.spec_nodes;
      while (!async_->done() && (int)nodes_.size() < kMaxNodes && expand_best()) {
      }
      stats_.spec_wait_nodes += stats_.spec_nodes - n_before;
      stats_.t_spec_wait += seconds_since(tw);
      async_->result(valid_);
      stats_.batches += 1;
      stats_.states_checked += (int64_t)valid_.size();
      stats_.check_seconds += seconds_since(tc);
    } else {
      check_(batch_, valid_);
      // MPG_PLAN_EMULATE_WAIT=n: explore n more nodes after the batch is formed, as the device path does
      // while a batch runs (lets CPU runs reproduce the device path's batches)
      static const int emu = std::getenv("MPG_PLAN_EMULATE_WAIT") ? std::atoi(std::getenv("MPG_PLAN_EMULATE_WAIT")) : 0;
      for (int k = 0; k < emu && (int)nodes_.size() < kMaxNodes && expand_best(); ++k) {
      }
    }
    for (size_t i = 0; i < valid_.size(); ++i) vc_.put(batch_.data() + i * d_, valid_[i]);
  }
  // hash set of the batch's states (open addressing on the 64-bit keys, a
  // slot is live when its generation is the current one: no clearing)
  void seen_reset(size_t n) {
    size_t m = 64;
    while (m < 2 * n + 2) m <<= 1;
    if (seen_.size() < m) {
      seen_.assign(m, 0);
      seen_gen_.assign(m, 0);
    }
    gen_ += 1;
  }
  bool mark(uint64_t h) {
    const size_t m = seen_.size() - 1;  // a power of two minus one
    for (size_t i = h & m;; i = (i + 1) & m) {
      if (seen_gen_[i] != gen_) {
        seen_gen_[i] = gen_;
        seen_[i] = h;
        return true;
      }
      if (seen_[i] == h) return false;
    }
  }

  static constexpr int kMaxSpecIters = 64;  // iterations a speculative branch may run without a new unknown
  static constexpr int kMaxNodes = 4096;    // explored nodes kept
  static constexpr int kMaxBatch = 2048;    // states per batch
  static constexpr int kSyncNodes = 16;         // nodes explored before an asynchronous batch is sent
  static constexpr int kSyncCheckerNodes = 64;  // nodes explored before a synchronous checker's batch
  static constexpr double kMinProb = 1e-4;  // outcomes less likely than this are not explored

  const PlanSpace& sp_;
  const int d_;
  const GoalSet& goals_;
  const double maxd_;
  OMPLPlanner::Stats& stats_;
  SampleFn sample_fn_;
  TimeoutFn timed_out_;
  CheckFn check_;
  const int spec_nodes_;
  ValidityCache vc_;
  NearMemo memo_;
  BaseTree base_[2];
  Branch real_;
  std::vector<double> samp_;
  int64_t samp0_ = 0;
  std::vector<SNode> nodes_;
  std::priority_queue<std::tuple<double, int, int>> frontier_;
  std::unique_ptr<AsyncCheck> async_;
  double n_out_[6] = {0, 0, 0, 0, 0, 0}, n_ok_[6] = {0, 0, 0, 0, 0, 0};
  int approxsol_ = -1;
  double approxdif_ = std::numeric_limits<double>::infinity();
  std::vector<double> rbuf_, xbuf_, mot_, batch_;
  std::vector<uint8_t> valid_;
  std::vector<uint64_t> seen_;
  std::vector<uint32_t> seen_gen_;
  uint32_t gen_ = 0;
  std::vector<int> order_;
};

}  // namespace

std::pair<std::string, std::vector<std::vector<double>>> OMPLPlanner::plan(
    const std::vector<double>& start_state, const std::vector<std::vector<double>>& goal_states,
    const std::string& planner_name, double time, double range, double goal_bias, double /*pathlen_obj_weight*/,
    bool /*pathlen_obj_only*/, bool verbose) {
  const PlanSpace& sp = space_;
  const int d = sp.dim;
  if (goal_states.empty()) throw std::invalid_argument("goal_states is empty");
  if (start_state.size() != goal_states[0].size())
    throw std::runtime_error("Length of start state and goal state should be equal");
  if ((int)start_state.size() != d)
    throw std::runtime_error("Length of start state and problem dimension should be equal");
  for (const auto& g : goal_states)
    if ((int)g.size() != d) throw std::runtime_error("Length of start state and goal state should be equal");
  const bool connect = planner_name == "RRTConnect";
  if (!connect && planner_name != "RRT") {
    static const char* known[] = {"PRMstar", "LazyPRMstar", "RRTstar", "RRTsharp", "RRTXstatic", "InformedRRTstar"};
    for (const char* k : known)
      if (planner_name == k)
        throw std::logic_error("NotImplemented: planner '" + planner_name +
                               "' (optimizing planners need the clearance objective); RRTConnect and RRT are "
                               "implemented");
    throw std::runtime_error("Planner Not implemented");
  }
  stats_ = Stats();
  const auto t_begin = Clock::now();

  std::vector<double> start = start_state;
  const bool invalid_start = !is_valid(start);
  if (invalid_start) {
    std::printf("invalid start state!! (collision)\n");
    std::fflush(stdout);
    start = random_sample_nearby(start_state);
  }

  // goal enumeration over +-2pi for revolute joints (ompl_planner.cpp:117-150)
  GoalSet goals;
  goals.sp = &sp;
  int64_t tot_enum_states = 1;
  for (int i = 0; i < d; ++i) tot_enum_states *= 3;
  for (const auto& g : goal_states)
    for (int64_t i = 0; i < tot_enum_states; ++i) {
      std::vector<double> tmp;
      int64_t t = i;
      bool flag = true;
      for (int j = 0; j < d; ++j) {
        tmp.push_back(g[(size_t)j]);
        const int dir = (int)(t % 3);
        t /= 3;
        if (dir != 0 && !sp.revolute[(size_t)j]) {
          flag = false;
          break;
        }
        if (dir == 1) {
          if (tmp[(size_t)j] - 2 * kRefPi > sp.lo[(size_t)j]) {
            tmp[(size_t)j] -= 2 * kRefPi;
          } else {
            flag = false;
            break;
          }
        } else if (dir == 2) {
          if (tmp[(size_t)j] + 2 * kRefPi < sp.hi[(size_t)j]) {
            tmp[(size_t)j] += 2 * kRefPi;
          } else {
            flag = false;
            break;
          }
        }
      }
      if (flag) goals.st.insert(goals.st.end(), tmp.begin(), tmp.end());
    }
  if (verbose) std::printf("number of goal state: %zu\n", goals.count());
  // one batch for every goal's validity (PlannerInputStates checks each
  // sampled goal with satisfiesBounds && isValid)
  {
    std::vector<uint8_t> v;
    check(goals.st, v);
    goals.usable.resize(goals.count());
    for (size_t i = 0; i < goals.count(); ++i) goals.usable[i] = v[i] && sp.satisfies_bounds(goals.state(i));
  }

  const double max_distance = range > 1e-6 ? range : 0.2 * sp.max_extent;  // SelfConfig::configurePlannerRange
  // (status, path): a solved status (exact or approximate) returns the path,
  // prefixed by the original start when it was resampled (ompl_planner.cpp:225-244)
  auto finish = [&](const std::string& status, std::vector<std::vector<double>> path) {
    stats_.seconds = seconds_since(t_begin);
    std::vector<std::vector<double>> ret;
    if (status == "Exact solution" || status == "Approximate solution") {
      if (invalid_start) ret.push_back(start_state);
      for (auto& r : path) ret.push_back(std::move(r));
    }
    return std::make_pair(status, ret);
  };

  // nextStart(): bounds && valid
  const bool start_ok = sp.satisfies_bounds(start.data()) && (start == start_state ? !invalid_start : is_valid(start));
  if (!start_ok) return finish("Invalid start", {});
  if (goals.count() == 0) return finish("Invalid goal", {});

  std::vector<PlanRNG> sampler((size_t)d);  // CompoundStateSampler: one sampler (RNG) per subspace
  auto sample_uniform = [&](double* out) {
    for (int i = 0; i < d; ++i)
      out[i] = sp.so2[(size_t)i] ? sampler[(size_t)i].uniform_real(-kPi, kPi)
                                 : sampler[(size_t)i].uniform_real(sp.lo[(size_t)i], sp.hi[(size_t)i]);
  };
  auto timed_out = [&]() { return seconds_since(t_begin) >= time; };
  std::vector<double> rstate((size_t)d), xstate((size_t)d);
  std::vector<double> batch;
  std::vector<uint8_t> valid;

  if (!connect) {
    // ---------------- RRT (OMPL geometric/planners/rrt/src/RRT.cpp) ----------------
    PlanRNG rng;  // RRT::rng_ (constructed with the planner, before the sampler)
    Tree tree(d);
    tree.add(start.data(), -1);
    int solution = -1, approxsol = -1;
    double approxdif = std::numeric_limits<double>::infinity();
    while (!timed_out()) {
      stats_.iterations += 1;
      if (rng.uniform01() < goal_bias) {
        const double* g = goals.sample_goal();
        std::copy(g, g + d, rstate.begin());
      } else {
        sample_uniform(rstate.data());
      }
      const int nm = tree.nearest(sp, rstate.data());
      const double* dstate = rstate.data();
      const double dd = sp.distance(tree.state(nm), rstate.data());
      if (dd > max_distance) {
        sp.interpolate(tree.state(nm), rstate.data(), max_distance / dd, xstate.data());
        dstate = xstate.data();
      }
      batch.clear();
      append_motion(sp, tree.state(nm), dstate, batch);
      check(batch, valid);
      if (!all_valid(valid, 0, valid.size())) continue;
      const int m = tree.add(dstate, nm);
      const double dist = goals.distance_goal(tree.state(m));
      if (dist < kEps) {  // GoalRegion::isSatisfied: distanceGoal < threshold (epsilon)
        approxdif = dist;
        solution = m;
        break;
      }
      if (dist < approxdif) {
        approxdif = dist;
        approxsol = m;
      }
    }
    stats_.start_tree = tree.size();
    bool approximate = false;
    if (solution < 0) {
      solution = approxsol;
      approximate = true;
    }
    if (solution < 0) return finish("Timeout", {});
    std::vector<const double*> rev;
    for (int m = solution; m >= 0; m = tree.parent[(size_t)m]) rev.push_back(tree.state(m));
    std::vector<const double*> fwd(rev.rbegin(), rev.rend());
    return finish(approximate ? "Approximate solution" : "Exact solution", path_rows(sp, fwd));
  }

  // ---------------- RRTConnect (OMPL geometric/planners/rrt/src/RRTConnect.cpp) ----------------
  if (speculative_) {
    ConnectEngine eng(sp, goals, start, max_distance, stats_, [&](double* out) { sample_uniform(out); }, timed_out,
                      [&](const std::vector<double>& st, std::vector<uint8_t>& v) { check(st, v); },
                      custom_ ? nullptr : world_->device_world(), spec_nodes_);
    auto r = eng.run();
    return finish(r.first, path_rows(sp, r.second));
  }
  // OMPL's loop as written: one validity batch per growTree call
  Tree tstart(d), tgoal(d);
  tstart.add(start.data(), -1);
  bool start_tree = true;  // RRTConnect::startTree_
  int approxsol = -1;
  double approxdif = std::numeric_limits<double>::infinity();
  auto grow_serial = [&](Tree& t, bool is_start, const std::vector<double>& r, int& xm) -> Grow {
    const int n = t.nearest(sp, r.data());
    bool reach = true;
    const double* ds = r.data();
    const double dd = sp.distance(t.state(n), r.data());
    if (dd > max_distance) {
      sp.interpolate(t.state(n), r.data(), max_distance / dd, xstate.data());
      if (sp.equal(t.state(n), xstate.data())) return TRAPPED;
      ds = xstate.data();
      reach = false;
    }
    batch.clear();
    append_grow(sp, is_start, t.state(n), ds, batch);
    check(batch, valid);
    if (!all_valid(valid, 0, valid.size())) return TRAPPED;
    xm = t.add(ds, n);
    return reach ? REACHED : ADVANCED;
  };

  while (!timed_out()) {
    stats_.iterations += 1;
    const bool tree_is_start = start_tree;
    Tree& tree = tree_is_start ? tstart : tgoal;
    start_tree = !start_tree;
    Tree& other = start_tree ? tstart : tgoal;
    const bool other_is_start = start_tree;

    if (tgoal.size() == 0 || goals.sampled < (size_t)tgoal.size() / 2) {
      // the first goal: nextGoal(ptc) keeps sampling; later: nextGoal(), one sample
      const double* g = goals.next_goal(tgoal.size() == 0);
      if (g) tgoal.add(g, -1);
      if (tgoal.size() == 0) {
        if (verbose) std::printf("RRTConnect: Unable to sample any valid states for goal tree\n");
        break;
      }
    }
    sample_uniform(rstate.data());
    int added = -1, xmotion = -1;  // tgi.xmotion
    bool tgi_start = other_is_start;
    if (grow_serial(tree, tree_is_start, rstate, added) == TRAPPED) {
      stats_.ext_trapped += 1;
      continue;
    }
    xmotion = added;
    rstate.assign(tree.state(added), tree.state(added) + d);  // copyState(rstate, tgi.xstate) when not REACHED
    Grow gsc = grow_serial(other, other_is_start, rstate, xmotion);
    if (gsc == TRAPPED) tgi_start = !tgi_start;
    while (gsc == ADVANCED) gsc = grow_serial(other, other_is_start, rstate, xmotion);

    if (gsc == REACHED) {  // isStartGoalPairValid: always true for GoalStates
      int sm = tgi_start ? xmotion : added;
      int gm = tgi_start ? added : xmotion;
      if (tstart.parent[(size_t)sm] >= 0)
        sm = tstart.parent[(size_t)sm];
      else
        gm = tgoal.parent[(size_t)gm];
      stats_.start_tree = tstart.size();
      stats_.goal_tree = tgoal.size();
      return finish("Exact solution", path_rows(sp, connect_path(tstart, sm, tgoal, gm)));
    }
    if (tgi_start) {  // approximate solution bookkeeping on the start tree
      const double dist = goals.distance_goal(tstart.state(xmotion));
      if (dist < approxdif) {
        approxdif = dist;
        approxsol = xmotion;
      }
    }
  }
  stats_.start_tree = tstart.size();
  stats_.goal_tree = tgoal.size();
  if (approxsol >= 0) return finish("Approximate solution", path_rows(sp, root_path(tstart, approxsol)));
  return finish("Timeout", {});
}

double async_check_selftest(double batch_ms, bool in_flight) { return async_check_selftest_impl(batch_ms, in_flight); }

}  // namespace mpgh
