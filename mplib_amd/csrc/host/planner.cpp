// planner.cpp -- OMPLPlanner with batched device state validity.
// Reference: src/ompl_planner.{h,cpp} (MPlib) over OMPL 1.6.0 RRTConnect / RRT,
// DiscreteMotionValidator, CompoundStateSpace, RealVectorStateSpace,
// SO2StateSpace, GoalStates and PlannerInputStates (restated here; OMPL is not
// in this image).  See planner.hpp for the batching scheme.
#include "planner.hpp"

#include <chrono>
#include <cmath>
#include <cstring>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <stdexcept>

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

// state -> validity, open addressing over a pool of the states' bits (no
// per-entry allocation: the planner queries it hundreds of times per iteration)
class ValidityCache {
 public:
  explicit ValidityCache(int dim) : dim_(dim), slots_(1024, -1) {}
  // 1 valid, 0 invalid, -1 unknown
  int find(const double* s) const {
    size_t i = hash(s) & (slots_.size() - 1);
    for (;; i = (i + 1) & (slots_.size() - 1)) {
      const int e = slots_[i];
      if (e < 0) return -1;
      if (std::memcmp(pool_.data() + (size_t)e * dim_, s, sizeof(double) * dim_) == 0) return val_[(size_t)e];
    }
  }
  void put(const double* s, uint8_t v) {
    if (find(s) >= 0) return;
    if (2 * (val_.size() + 1) > slots_.size()) grow();
    insert_index(s, (int)val_.size());
    pool_.insert(pool_.end(), s, s + dim_);
    val_.push_back(v);
  }

 private:
  uint64_t hash(const double* s) const {
    uint64_t h = 0x9e3779b97f4a7c15ull;
    for (int k = 0; k < dim_; ++k) {
      uint64_t x;
      std::memcpy(&x, s + k, 8);
      h ^= x + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
      h *= 0xff51afd7ed558ccdull;
    }
    return h ^ (h >> 33);
  }
  void insert_index(const double* s, int e) {
    size_t i = hash(s) & (slots_.size() - 1);
    while (slots_[i] >= 0) i = (i + 1) & (slots_.size() - 1);
    slots_[i] = e;
  }
  void grow() {
    slots_.assign(slots_.size() * 2, -1);
    for (size_t e = 0; e < val_.size(); ++e) insert_index(pool_.data() + e * dim_, (int)e);
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
  Tree tstart(d), tgoal(d);
  tstart.add(start.data(), -1);
  bool start_tree = true;  // RRTConnect::startTree_
  int approxsol = -1;
  double approxdif = std::numeric_limits<double>::infinity();
  struct Step {
    std::vector<double> state;
    int tree_parent, chain_parent;  // grows from a node of the other tree, or from chain step chain_parent
    bool reach;
    size_t a, b;  // its states in the batch
  };
  std::vector<Step> chain;
  const size_t kMaxChain = 1u << 20;
  // speculative mode: a validity cache (a state's validity is a pure function
  // of the state) and uniform samples drawn ahead of their iteration -- the
  // sampler's draws do not depend on validity, so drawing early keeps the
  // sequence
  ValidityCache vcache(d);
  std::deque<std::vector<double>> ahead;
  auto peek_sample = [&](size_t j) -> const std::vector<double>& {
    while (ahead.size() <= j) {
      std::vector<double> r((size_t)d);
      sample_uniform(r.data());
      ahead.push_back(std::move(r));
    }
    return ahead[j];
  };
  std::vector<double> ext_states, chain_states, spec_states;
  constexpr int kLookahead = 3;
  constexpr size_t kSpecCap = 4096;  // speculated states per batch
  constexpr int kSpecSteps = 8;      // growTree steps of a speculated connect chain
  // the connect chain growTree would run on t (plus `extra`, its newest
  // node) towards x if every motion were valid (as below for the current
  // iteration); its motions' states are appended to out
  auto spec_chain = [&](const Tree& t, bool t_is_start, const double* extra, const double* x, std::vector<double>& out) {
    double best;
    const int n0 = t.nearest(sp, x, &best);
    std::vector<double> cur(t.state(n0), t.state(n0) + d), stt((size_t)d);
    if (extra && sp.distance(extra, x) < best) {
      best = sp.distance(extra, x);
      cur.assign(extra, extra + d);
    }
    for (int k = 0; k < kSpecSteps; ++k) {
      const double dc = sp.distance(cur.data(), x);
      bool reach_k = false;
      if (dc > max_distance) {
        sp.interpolate(cur.data(), x, max_distance / dc, stt.data());
        if (sp.equal(cur.data(), stt.data())) return;
      } else {
        stt.assign(x, x + d);
        reach_k = true;
      }
      append_grow(sp, t_is_start, cur.data(), stt.data(), out);
      if (reach_k) return;
      const double dn = sp.distance(stt.data(), x);
      if (dn < best) {
        best = dn;
        cur = stt;
      }
    }
  };
  // RRTConnect::growTree (serial mode): nearest, step of at most maxDistance,
  // the motion's states in one batch
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
    if (!ahead.empty()) {
      rstate = ahead.front();
      ahead.pop_front();
    } else {
      sample_uniform(rstate.data());
    }

    int added = -1, xmotion = -1;  // tgi.xmotion
    bool tgi_start = other_is_start;
    Grow gsc = TRAPPED;
    if (!speculative_) {
      // OMPL's loop as written: one validity batch per growTree call
      if (grow_serial(tree, tree_is_start, rstate, added) == TRAPPED) {
        stats_.ext_trapped += 1;
        continue;
      }
      xmotion = added;
      rstate.assign(tree.state(added), tree.state(added) + d);  // copyState(rstate, tgi.xstate) when not REACHED
      gsc = grow_serial(other, other_is_start, rstate, xmotion);
      if (gsc == TRAPPED) tgi_start = !tgi_start;
      while (gsc == ADVANCED) gsc = grow_serial(other, other_is_start, rstate, xmotion);
    } else {
    // ---- extension of `tree` towards rstate (growTree)
    const int nm = tree.nearest(sp, rstate.data());
    bool reach = true;
    const double* dstate = rstate.data();
    const double dd = sp.distance(tree.state(nm), rstate.data());
    if (dd > max_distance) {
      sp.interpolate(tree.state(nm), rstate.data(), max_distance / dd, xstate.data());
      if (sp.equal(tree.state(nm), xstate.data())) continue;  // TRAPPED
      dstate = xstate.data();
      reach = false;
    }
    ext_states.clear();
    append_grow(sp, tree_is_start, tree.state(nm), dstate, ext_states);
    const std::vector<double> target(dstate, dstate + d);  // rstate after "copyState(rstate, tgi.xstate)"

    // ---- speculative connect chain of `other` towards target, computed as
    // the serial loop would compute it if every motion were valid: each step
    // grows from the nearest node of other + the chain so far
    const auto tc0 = Clock::now();
    chain.clear();
    chain_states.clear();
    double best_d;
    int tp = other.nearest(sp, target.data(), &best_d), cp = -1;
    std::vector<double> cur(other.state(tp), other.state(tp) + d);
    while (chain.size() < kMaxChain) {
      Step stp;
      stp.tree_parent = tp;
      stp.chain_parent = cp;
      const double dc = sp.distance(cur.data(), target.data());
      if (dc > max_distance) {
        stp.state.resize((size_t)d);
        sp.interpolate(cur.data(), target.data(), max_distance / dc, stp.state.data());
        if (sp.equal(cur.data(), stp.state.data())) break;  // TRAPPED without a motion
        stp.reach = false;
      } else {
        stp.state = target;
        stp.reach = true;
      }
      stp.a = chain_states.size() / (size_t)d;
      append_grow(sp, other_is_start, cur.data(), stp.state.data(), chain_states);
      stp.b = chain_states.size() / (size_t)d;
      chain.push_back(std::move(stp));
      if (chain.back().reach) break;
      // nearest for the next growTree: the first strict minimum over the
      // tree and the chain in insertion order
      const double dn = sp.distance(chain.back().state.data(), target.data());
      if (dn < best_d) {
        best_d = dn;
        tp = -1;
        cp = (int)chain.size() - 1;
      }
      if (tp >= 0)
        cur.assign(other.state(tp), other.state(tp) + d);
      else
        cur = chain[(size_t)cp].state;
    }

    // one batch: the states of this iteration not known yet, plus the
    // extensions the next kLookahead iterations would try for every outcome
    // of this one (assuming the ones in between are trapped)
    auto known = [&](const std::vector<double>& st, size_t a, size_t b, bool& ok) {
      ok = true;
      bool all = true;
      for (size_t i = a; i < b; ++i) {
        const int v = vcache.find(st.data() + i * d);
        if (v < 0) all = false;
        else if (v == 0) ok = false;
      }
      return all;
    };
    auto need = [&](const std::vector<double>& st, size_t a, size_t b) {
      for (size_t i = a; i < b; ++i)
        if (vcache.find(st.data() + i * d) < 0) batch.insert(batch.end(), st.data() + i * d, st.data() + (i + 1) * d);
    };
    // every state goes through the cache: this iteration's extension and
    // connect chain, and the speculated ones (the next iterations'
    // extensions for every outcome of this one, and the connect chains the
    // next iteration would run after them)
    batch.clear();
    bool ext_ok;
    const size_t n_ext = ext_states.size() / (size_t)d;
    const bool ext_known = known(ext_states, 0, n_ext, ext_ok);
    if (!ext_known || ext_ok) {
      need(ext_states, 0, n_ext);
      need(chain_states, 0, chain_states.size() / (size_t)d);
      if (!batch.empty()) {
        stats_.t_chain += seconds_since(tc0);
        const auto ts0 = Clock::now();
        spec_states.clear();
        for (int j = 1; j <= kLookahead; ++j) {
          const bool fut_other = (j & 1) != 0;  // iteration i+1 extends `other`, i+2 `tree`, ...
          Tree& ft = fut_other ? other : tree;
          const bool ft_start = fut_other ? other_is_start : tree_is_start;
          const std::vector<double>& rj = peek_sample((size_t)j - 1);
          std::vector<const double*> cand;
          double be;
          const int ne = ft.nearest(sp, rj.data(), &be);
          cand.push_back(ft.state(ne));
          if (fut_other) {  // prefix minima of the connect chain
            double run = be;
            for (auto& c : chain) {
              const double dc = sp.distance(c.state.data(), rj.data());
              if (dc < run) {
                run = dc;
                cand.push_back(c.state.data());
              }
            }
          } else if (sp.distance(target.data(), rj.data()) < be) {
            cand.push_back(target.data());
          }
          if (&ft == &tgoal && goals.sampled < goals.count() && goals.usable[goals.sample_pos])
            cand.push_back(goals.state(goals.sample_pos));  // a goal root added at that iteration's start
          for (const double* c : cand) {
            const double dj = sp.distance(c, rj.data());
            std::vector<double> x(rj);
            if (dj > max_distance) {
              sp.interpolate(c, rj.data(), max_distance / dj, x.data());
              if (sp.equal(c, x.data())) continue;
            }
            append_grow(sp, ft_start, c, x.data(), spec_states);
            // iteration i+1 connects `tree` (with this iteration's new node)
            // towards x if that extension is valid
            if (j == 1 && c == cand.front() && spec_states.size() < kSpecCap * (size_t)d)
              spec_chain(tree, tree_is_start, target.data(), x.data(), spec_states);
          }
        }
        const size_t spec_off = batch.size() / (size_t)d;
        need(spec_states, 0, spec_states.size() / (size_t)d);
        stats_.t_spec += seconds_since(ts0);
        (void)spec_off;
        check(batch, valid);
        for (size_t i = 0; i < valid.size(); ++i) vcache.put(batch.data() + i * d, valid[i]);
      }
      known(ext_states, 0, n_ext, ext_ok);
    }
    if (!ext_ok) {  // extension TRAPPED
      stats_.ext_trapped += 1;
      continue;
    }
    added = tree.add(target.data(), nm);
    (void)reach;
    // ---- connect: growTree on `other` while ADVANCED
    xmotion = added;
    std::vector<int> node(chain.size(), -1);
    for (size_t k = 0; k < chain.size(); ++k) {
      const Step& s = chain[k];
      bool ok_k = true;
      for (size_t i = s.a; i < s.b && ok_k; ++i) ok_k = vcache.find(chain_states.data() + i * d) == 1;
      if (!ok_k) {
        gsc = TRAPPED;
        break;
      }
      node[k] = other.add(s.state.data(), s.tree_parent >= 0 ? s.tree_parent : node[(size_t)s.chain_parent]);
      xmotion = node[k];
      gsc = s.reach ? REACHED : ADVANCED;
      if (gsc == REACHED) break;
    }
    if (gsc == ADVANCED) gsc = TRAPPED;  // chain ended on a step without progress
    if (node.empty() || node[0] < 0) tgi_start = !tgi_start;  // the first connect growTree was TRAPPED
    }

    if (gsc == REACHED) {  // isStartGoalPairValid: always true for GoalStates
      int sm = tgi_start ? xmotion : added;
      int gm = tgi_start ? added : xmotion;
      Tree& ts = tstart;
      Tree& tg = tgoal;
      if (ts.parent[(size_t)sm] >= 0)
        sm = ts.parent[(size_t)sm];
      else
        gm = tg.parent[(size_t)gm];
      std::vector<const double*> p1, out;
      for (int m = sm; m >= 0; m = ts.parent[(size_t)m]) p1.push_back(ts.state(m));
      for (auto it = p1.rbegin(); it != p1.rend(); ++it) out.push_back(*it);
      for (int m = gm; m >= 0; m = tg.parent[(size_t)m]) out.push_back(tg.state(m));
      stats_.start_tree = tstart.size();
      stats_.goal_tree = tgoal.size();
      return finish("Exact solution", path_rows(sp, out));
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
  if (approxsol >= 0) {
    std::vector<const double*> rev;
    for (int m = approxsol; m >= 0; m = tstart.parent[(size_t)m]) rev.push_back(tstart.state(m));
    std::vector<const double*> fwd(rev.rbegin(), rev.rend());
    return finish("Approximate solution", path_rows(sp, fwd));
  }
  return finish("Timeout", {});
}

}  // namespace mpgh
