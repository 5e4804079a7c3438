// planner.hpp -- OMPL-compatible sampling planners whose state validity runs
// as batched device checks.
//
// Mirrors MPlib's OMPLPlanner (reference src/ompl_planner.{h,cpp}):
//   * the compound state space of the planned articulations' move-group joints
//     (build_state_space, ompl_planner.cpp:248-293): RealVector(1) per bounded
//     revolute / prismatic joint, SO2 per continuous joint, weights 1;
//   * plan(start, goals, planner_name, time, range, ...) (ompl_planner.cpp:97-245)
//     with the invalid-start resampling (random_sample_nearby, :71-95) and the
//     +-2*pi goal enumeration for revolute joints (:117-150);
//   * OMPL 1.6.0's RRTConnect / RRT and DiscreteMotionValidator semantics
//     (restated; OMPL is not in this image).
// OMPL evaluates isValid() one state at a time (ompl_planner.h:59-62).  Here
// RRTConnect runs as a resumable loop that stops at the first motion whose
// validity is not cached; an outcome tree of the loop's future (each motion
// valid or invalid, explored best first by the outcome rates seen so far) is
// explored from that point, and the unknown states of the real motion and of
// the explored ones go to the device as ONE batched collide call.  The host
// explores deeper while the batch runs (a helper thread waits on the device),
// so a plan costs far fewer round trips than growTree calls.  The tree that
// results is the serial algorithm's: the real loop reads nothing but the
// validity cache; speculation only chooses what rides in a batch.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <random>
#include <string>
#include <utility>
#include <vector>

#include "host.hpp"

namespace mpgh {

// Compound state space of the planner (OMPL CompoundStateSpace of RealVector(1)
// and SO2 subspaces with unit weights).
struct PlanSpace {
  int dim = 0;
  std::vector<double> lo, hi;
  std::vector<uint8_t> so2;        // SO2StateSpace component (continuous joint)
  std::vector<uint8_t> revolute;   // is_revolute_ (ompl_planner.cpp:283-289)
  double max_extent = 0.0;         // CompoundStateSpace::getMaximumExtent
  double longest_valid_segment = 0.0;

  double distance(const double* a, const double* b) const;
  double distance_below(const double* a, const double* b, double bound) const;
  void interpolate(const double* a, const double* b, double t, double* out) const;
  bool equal(const double* a, const double* b) const;
  unsigned valid_segment_count(const double* a, const double* b) const;
  bool satisfies_bounds(const double* s) const;
};

// OMPL's RNG (ompl/util/RandomNumbers): std::mt19937 + uniform_real_distribution,
// per-instance seeds drawn from a global seed generator that set_global_seed()
// resets.
class PlanRNG {
 public:
  PlanRNG();
  double uniform01() { return uni_(gen_); }
  double uniform_real(double lo, double hi) { return (hi - lo) * uniform01() + lo; }

 private:
  std::mt19937 gen_;
  std::uniform_real_distribution<> uni_{0.0, 1.0};
};
void plan_rng_seed(unsigned seed);

class OMPLPlanner {
 public:
  // valid[i] = state i (row of a [n, dim] float64 matrix) is collision free
  using Checker = std::function<void(const double* states, int64_t n, uint8_t* valid)>;

  explicit OMPLPlanner(const std::shared_ptr<PlanningWorld>& world);

  const std::shared_ptr<PlanningWorld>& get_world() const { return world_; }
  size_t get_dim() const { return (size_t)space_.dim; }
  const PlanSpace& space() const { return space_; }
  // replace the batched device checker (OMPL's setStateValidityChecker);
  // an empty function restores the device path
  void set_state_validity_checker(Checker c) { custom_ = std::move(c); }
  // RRTConnect: outcome-tree speculation (default), or one batch per growTree
  // call as OMPL's loop is written
  void set_speculative_connect(bool on) { speculative_ = on; }
  bool get_speculative_connect() const { return speculative_; }
  // outcome-tree nodes explored before each batch is sent (-1: 16 on the device
  // path, which also explores while each batch runs; 64 for custom checkers)
  void set_speculation_nodes(int n) { spec_nodes_ = n; }
  int get_speculation_nodes() const { return spec_nodes_; }

  std::vector<double> random_sample_nearby(const std::vector<double>& start);
  std::pair<std::string, std::vector<std::vector<double>>> plan(
      const std::vector<double>& start_state, const std::vector<std::vector<double>>& goal_states,
      const std::string& planner_name = "RRTConnect", double time = 1.0, double range = 0.0,
      double goal_bias = 0.05, double pathlen_obj_weight = 10.0, bool pathlen_obj_only = false,
      bool verbose = false);

  struct Stats {
    int64_t iterations = 0, batches = 0, states_checked = 0, ext_trapped = 0;
    int64_t start_tree = 0, goal_tree = 0, spec_nodes = 0, spec_wait_nodes = 0, spec_resets = 0;
    double seconds = 0.0, check_seconds = 0.0, t_spec = 0.0, t_spec_wait = 0.0;
  };
  const Stats& last_stats() const { return stats_; }

 private:
  void check(const std::vector<double>& states, std::vector<uint8_t>& valid);
  bool is_valid(const std::vector<double>& s);

  std::shared_ptr<PlanningWorld> world_;
  PlanSpace space_;
  Checker custom_;
  bool speculative_ = true;
  int spec_nodes_ = -1;
  Stats stats_;
  std::vector<uint8_t> flags_;
};

// CPU self-test of the planner's asynchronous validity helper (pymp._selftest)
double async_check_selftest(double batch_ms, bool in_flight);

}  // namespace mpgh
