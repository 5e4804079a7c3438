// kinjac.cpp -- PinocchioModel's Jacobians and closed-loop IK on the host
// (python/pybind_pinocchio.hpp:47-58; src/pinocchio_model.cpp:335-496):
// computeFullJacobian / getLinkJacobian / computeSingleLinkLocalJacobian and
// computeIKCLIK / computeIKCLIKJL.  Restated from pinocchio 2.6.21's published
// algorithms [ext, not under /root/reference]: forwardKinematics (oMi =
// oMi[parent] * placement * M(q)), the joint motion subspaces (revolute: w =
// axis, prismatic: v = axis), computeJointJacobians (WORLD: oMi.act(S)),
// computeJointJacobian (LOCAL to the joint), log3 / log6, integrate
// (continuous joints: rotate (cos, sin), first-order renormalisation) and the
// damped least-squares step v = -J^T (J J^T + damp I)^-1 err.  Host only: the
// IK is a caller of the collision path (planner.py:292-326), not part of it;
// the results are floating-point (parity with pinocchio unpinned, tests check
// the Jacobian against finite differences of the oracle FK and the IK
// against its own targets).
//
// KDLModel (python/pybind_kdl.hpp, src/kdl_model.cpp): the chain / tree IK
// entry points with orocos KDL 1.5's solver semantics [ext, not under
// /root/reference]: ChainIkSolverPos_NR (full Newton steps q += J^+ diff(f,
// goal), maxiter 100, eps 1e-6), ..._NR_JL (the same, clamped to the limits
// after each step), ChainIkSolverPos_LMA (Levenberg-Marquardt on the
// L-weighted twist, L = (1, 1, 1, .01, .01, .01), eps 1e-5, maxiter 500,
// eps_joints 1e-15, lambda schedule of KDL's implementation) and
// TreeIkSolverPos_NR_JL (all endpoints' twists stacked, damped least
// squares with lambda 1e-6, maxiter 1000, eps 1e-6).  Twists are KDL's: the
// position error and the base-frame rotation vector of R_cur^T R_goal
// (KDL::diff), Jacobians with the reference point at the tip.  Return codes
// are KDL's (0 ok, -5 max iterations, -100 / -101 LMA's gradient /
// increment too small).  The iteration paths are not KDL's bit for bit (its
// SVD is not restated); answers are checked against their targets.
#include <cmath>
#include <iostream>
#include <sstream>
#include <tuple>

#include "host.hpp"

namespace mpgh {
namespace {

struct Mot {  // pinocchio Motion: linear v, angular w
  double v[3], w[3];
};

void cross3(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
void matv(const double* R, const double* x, double* o) {
  for (int i = 0; i < 3; ++i) o[i] = (R[3 * i] * x[0] + R[3 * i + 1] * x[1]) + R[3 * i + 2] * x[2];
}
void mattv(const double* R, const double* x, double* o) {
  for (int i = 0; i < 3; ++i) o[i] = (R[i] * x[0] + R[3 + i] * x[1]) + R[6 + i] * x[2];
}

// M.act(m): (R v + p x (R w), R w)
Mot act(const SE3& M, const Mot& m) {
  Mot o;
  matv(M.R, m.w, o.w);
  double rv[3], pxw[3];
  matv(M.R, m.v, rv);
  cross3(M.p, o.w, pxw);
  for (int k = 0; k < 3; ++k) o.v[k] = rv[k] + pxw[k];
  return o;
}
// M.actInv(m) = toActionMatrixInverse() * m: (R^T (v - p x w), R^T w)
Mot act_inv(const SE3& M, const Mot& m) {
  Mot o;
  double pxw[3], d[3];
  cross3(M.p, m.w, pxw);
  for (int k = 0; k < 3; ++k) d[k] = m.v[k] - pxw[k];
  mattv(M.R, d, o.v);
  mattv(M.R, m.w, o.w);
  return o;
}

SE3 se3_inverse(const SE3& M) {
  SE3 o;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) o.R[3 * i + j] = M.R[3 * j + i];
  double rp[3];
  mattv(M.R, M.p, rp);
  for (int k = 0; k < 3; ++k) o.p[k] = -rp[k];
  return o;
}

// pinocchio::log3: the rotation vector of R (angle theta in [0, pi])
void log3(const double* R, double* w, double& theta) {
  const double tr = (R[0] + R[4]) + R[8];
  if (tr > 3.0) theta = 0.0;
  else if (tr < -1.0) theta = M_PI;
  else theta = std::acos((tr - 1.0) / 2.0);
  if (theta >= M_PI - 1e-2) {  // near pi: from the diagonal, signs from the skew part
    const double cphi = std::cos(theta - M_PI);
    const double beta = theta * theta / (1.0 + cphi);
    const double t0 = (R[0] + cphi) * beta, t1 = (R[4] + cphi) * beta, t2 = (R[8] + cphi) * beta;
    w[0] = (R[7] > R[5] ? 1.0 : -1.0) * (t0 > 0 ? std::sqrt(t0) : 0.0);
    w[1] = (R[2] > R[6] ? 1.0 : -1.0) * (t1 > 0 ? std::sqrt(t1) : 0.0);
    w[2] = (R[3] > R[1] ? 1.0 : -1.0) * (t2 > 0 ? std::sqrt(t2) : 0.0);
  } else {
    const double t = (theta > 1e-4 ? theta / std::sin(theta) : 1.0) / 2.0;
    w[0] = t * (R[7] - R[5]);
    w[1] = t * (R[2] - R[6]);
    w[2] = t * (R[3] - R[1]);
  }
}

// pinocchio::log6(M).toVector(): (linear, angular)
std::array<double, 6> log6(const SE3& M) {
  double w[3], theta;
  log3(M.R, w, theta);
  const double t = std::sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]), t2 = t * t;
  double alpha, beta;
  if (t < 1e-4) {
    alpha = 1.0 - t2 / 12.0 - t2 * t2 / 720.0;
    beta = 1.0 / 12.0 + t2 / 720.0;
  } else {
    const double st = std::sin(t), ct = std::cos(t);
    alpha = t * st / (2.0 * (1.0 - ct));
    beta = 1.0 / t2 - st / (2.0 * t * (1.0 - ct));
  }
  double wxp[3];
  cross3(w, M.p, wxp);
  const double wp = (w[0] * M.p[0] + w[1] * M.p[1]) + w[2] * M.p[2];
  std::array<double, 6> o;
  for (int k = 0; k < 3; ++k) {
    o[k] = alpha * M.p[k] - 0.5 * wxp[k] + (beta * wp) * w[k];
    o[3 + k] = w[k];
  }
  return o;
}

// solve (A) x = b for a symmetric positive definite 6x6 A (Cholesky)
std::array<double, 6> spd_solve6(std::array<double, 36> A, std::array<double, 6> b) {
  for (int j = 0; j < 6; ++j) {
    double d = A[6 * j + j];
    for (int k = 0; k < j; ++k) d -= A[6 * j + k] * A[6 * j + k];
    if (!(d > 0)) throw std::runtime_error("IK: J J^T + damp I is not positive definite");
    const double l = std::sqrt(d);
    A[6 * j + j] = l;
    for (int i = j + 1; i < 6; ++i) {
      double s = A[6 * i + j];
      for (int k = 0; k < j; ++k) s -= A[6 * i + k] * A[6 * j + k];
      A[6 * i + j] = s / l;
    }
  }
  for (int i = 0; i < 6; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= A[6 * i + k] * b[k];
    b[i] = s / A[6 * i + i];
  }
  for (int i = 5; i >= 0; --i) {
    double s = b[i];
    for (int k = i + 1; k < 6; ++k) s -= A[6 * k + i] * b[k];
    b[i] = s / A[6 * i + i];
  }
  return b;
}

SE3 pose_se3(const Vec7& pose) {  // (x, y, z, qw, qx, qy, qz) -> SE3
  SE3 T;
  mpg::quat_to_mat(pose[3], pose[4], pose[5], pose[6], T.R);
  for (int k = 0; k < 3; ++k) T.p[k] = pose[k];
  return T;
}

}  // namespace

void PinocchioModel::print_frames() const {
  std::ostringstream o;
  const size_t nj = joints_.size();
  o << "Joint dim " << nj << " " << nv_ << " " << nj << " " << nj << "\n";
  o << "Joint Tangent dim " << nq_ << " " << nj << " " << nj << "\n";
  o << "Joint Limit " << nq_ << " " << nq_ << "\n";
  for (size_t i = 0; i < frames_.size(); ++i) {
    const PinFrame& f = frames_[i];
    const char* t = f.type == PinFrame::JOINT ? "JOINT" : f.type == PinFrame::FIXED_JOINT ? "FIXED_JOINT" : "BODY";
    o << "Frame " << i << " " << f.name << " " << f.parent << " " << t << "\n";
  }
  std::cout << o.str() << std::flush;
}

std::vector<double> PinocchioModel::qpos_user2pin(const std::vector<double>& q) const {
  if ((int)q.size() != nv_) throw std::runtime_error("Qpos user2pinocchio failed");
  std::vector<double> out(nq_, 0.0);
  for (size_t u = 0; u < joint_index_user2pin_.size(); ++u) {
    const PinJoint& pj = joints_[joint_index_user2pin_[u]];
    if (pj.nq == 1) out[pj.idx_q] = q[vidx_[u]];
    if (pj.nq == 2) {
      out[pj.idx_q] = std::cos(q[vidx_[u]]);
      out[pj.idx_q + 1] = std::sin(q[vidx_[u]]);
    }
  }
  return out;
}

std::vector<double> PinocchioModel::qpos_pin2user(const std::vector<double>& q) const {
  std::vector<double> out(nv_, 0.0);
  for (size_t u = 0; u < joint_index_user2pin_.size(); ++u) {
    const PinJoint& pj = joints_[joint_index_user2pin_[u]];
    if (pj.nq == 1) out[vidx_[u]] = q[pj.idx_q];
    if (pj.nq == 2) out[vidx_[u]] = std::atan2(q[pj.idx_q + 1], q[pj.idx_q]);
  }
  return out;
}

// forwardKinematics: oMi[j] = oMi[parent] * (placement * M(q)), pinocchio q
std::vector<SE3> PinocchioModel::joint_frames(const std::vector<double>& qpin) const {
  std::vector<SE3> oMi(joints_.size());
  mpg::se3_identity(oMi[0]);
  for (size_t j = 1; j < joints_.size(); ++j) {
    const PinJoint& pj = joints_[j];
    SE3 M;
    mpg::se3_identity(M);
    const int t = pj.type >= MPG_JOINT_RUBX ? pj.type - MPG_JOINT_RUBX : pj.type;
    if (pj.type <= MPG_JOINT_REVOLUTE_UNALIGNED || pj.type >= MPG_JOINT_RUBX) {
      double s, c;
      if (pj.nq == 2) {
        c = qpin[pj.idx_q];
        s = qpin[pj.idx_q + 1];
      } else {
        s = std::sin(qpin[pj.idx_q]);
        c = std::cos(qpin[pj.idx_q]);
      }
      if (t == 0) {
        M.R[4] = c, M.R[5] = -s, M.R[7] = s, M.R[8] = c;
      } else if (t == 1) {
        M.R[0] = c, M.R[2] = s, M.R[6] = -s, M.R[8] = c;
      } else if (t == 2) {
        M.R[0] = c, M.R[1] = -s, M.R[3] = s, M.R[4] = c;
      } else {
        mpg::axis_rot(pj.axis.data(), c, s, M.R);
      }
    } else {
      const double v = qpin[pj.idx_q];
      const Vec3 ax = pj.type == MPG_JOINT_PX ? Vec3{1, 0, 0}
                      : pj.type == MPG_JOINT_PY ? Vec3{0, 1, 0}
                      : pj.type == MPG_JOINT_PZ ? Vec3{0, 0, 1}
                                                : pj.axis;
      for (int k = 0; k < 3; ++k) M.p[k] = ax[k] * v;
    }
    const SE3 li = mpg::se3_mul(pj.placement, M);
    oMi[j] = pj.parent > 0 ? mpg::se3_mul(oMi[pj.parent], li) : li;
  }
  return oMi;
}

// the joint's motion subspace S in its own frame (one column: nv == 1)
static Mot joint_subspace(const PinJoint& pj) {
  Mot S{{0, 0, 0}, {0, 0, 0}};
  const int t = pj.type >= MPG_JOINT_RUBX ? pj.type - MPG_JOINT_RUBX : pj.type;
  const bool rev = pj.type <= MPG_JOINT_REVOLUTE_UNALIGNED || pj.type >= MPG_JOINT_RUBX;
  double* d = rev ? S.w : S.v;
  if (rev ? t < 3 : pj.type != MPG_JOINT_PRISMATIC_UNALIGNED) {
    d[rev ? t : pj.type - MPG_JOINT_PX] = 1.0;
  } else {
    for (int k = 0; k < 3; ++k) d[k] = pj.axis[k];
  }
  return S;
}

// computeJointJacobians: data.J (WORLD) for every joint, columns in pinocchio v order
void PinocchioModel::compute_full_jacobian(const std::vector<double>& qpos) {
  const std::vector<SE3> oMi = joint_frames(qpos_user2pin(qpos));
  jac_oMi_ = oMi;
  jac_world_.assign(6 * (size_t)nv_, 0.0);
  for (size_t j = 1; j < joints_.size(); ++j) {
    const PinJoint& pj = joints_[j];
    if (pj.nv != 1) continue;
    const Mot c = act(oMi[j], joint_subspace(pj));
    for (int k = 0; k < 3; ++k) {
      jac_world_[(size_t)k * nv_ + pj.idx_v] = c.v[k];
      jac_world_[(size_t)(3 + k) * nv_ + pj.idx_v] = c.w[k];
    }
  }
  jac_valid_ = true;
}

// columns of the joints supporting `joint` (getJointJacobian keeps only those)
std::vector<size_t> PinocchioModel::support_columns(int joint) const {
  std::vector<size_t> cols;
  for (int j = joint; j > 0; j = joints_[j].parent)
    if (joints_[j].nv == 1) cols.push_back(joints_[j].idx_v);
  return cols;
}

std::vector<double> PinocchioModel::user_columns(const std::vector<double>& Jpin) const {
  // J * v_map_user2pinocchio_: user column u = pinocchio column of user v u
  std::vector<double> out(6 * (size_t)nv_, 0.0);
  for (size_t u = 0; u < joint_index_user2pin_.size(); ++u) {
    const PinJoint& pj = joints_[joint_index_user2pin_[u]];
    for (int k = 0; k < pj.nv; ++k)
      for (int r = 0; r < 6; ++r) out[(size_t)r * nv_ + vidx_[u] + k] = Jpin[(size_t)r * nv_ + pj.idx_v + k];
  }
  return out;
}

std::vector<double> PinocchioModel::get_link_jacobian(size_t index, bool local) const {
  if (index >= link_index_user2pin_.size()) throw std::runtime_error("The link index is out of bound!");
  if (!jac_valid_) throw std::runtime_error("compute_full_jacobian has not been called");
  const PinFrame& fr = frames_[link_index_user2pin_[index]];
  std::vector<double> J(6 * (size_t)nv_, 0.0);
  for (size_t c : support_columns(fr.parent))
    for (int r = 0; r < 6; ++r) J[(size_t)r * nv_ + c] = jac_world_[(size_t)r * nv_ + c];
  if (local) {
    const SE3 link2world = mpg::se3_mul(jac_oMi_[fr.parent], fr.placement);
    for (int c = 0; c < nv_; ++c) {
      Mot m{{J[c], J[(size_t)nv_ + c], J[2 * (size_t)nv_ + c]},
            {J[3 * (size_t)nv_ + c], J[4 * (size_t)nv_ + c], J[5 * (size_t)nv_ + c]}};
      m = act_inv(link2world, m);
      for (int k = 0; k < 3; ++k) {
        J[(size_t)k * nv_ + c] = m.v[k];
        J[(size_t)(3 + k) * nv_ + c] = m.w[k];
      }
    }
  }
  return user_columns(J);
}

// computeJointJacobian: the supporting joints' columns expressed in the joint's own frame
std::vector<double> PinocchioModel::joint_local_jacobian(const std::vector<SE3>& oMi, int joint) const {
  std::vector<double> J(6 * (size_t)nv_, 0.0);
  for (int j = joint; j > 0; j = joints_[j].parent) {
    const PinJoint& pj = joints_[j];
    if (pj.nv != 1) continue;
    const Mot c = act_inv(oMi[joint], act(oMi[j], joint_subspace(pj)));
    for (int k = 0; k < 3; ++k) {
      J[(size_t)k * nv_ + pj.idx_v] = c.v[k];
      J[(size_t)(3 + k) * nv_ + pj.idx_v] = c.w[k];
    }
  }
  return J;
}

std::vector<double> PinocchioModel::compute_single_link_local_jacobian(const std::vector<double>& qpos,
                                                                      size_t index) {
  if (index >= link_index_user2pin_.size()) throw std::runtime_error("The link index is out of bound!");
  const PinFrame& fr = frames_[link_index_user2pin_[index]];
  std::vector<double> J = joint_local_jacobian(joint_frames(qpos_user2pin(qpos)), fr.parent);
  for (int c = 0; c < nv_; ++c) {  // link2joint.toActionMatrixInverse() * J
    Mot m{{J[c], J[(size_t)nv_ + c], J[2 * (size_t)nv_ + c]},
          {J[3 * (size_t)nv_ + c], J[4 * (size_t)nv_ + c], J[5 * (size_t)nv_ + c]}};
    m = act_inv(fr.placement, m);
    for (int k = 0; k < 3; ++k) {
      J[(size_t)k * nv_ + c] = m.v[k];
      J[(size_t)(3 + k) * nv_ + c] = m.w[k];
    }
  }
  return user_columns(J);
}

// computeIKCLIK / computeIKCLIKJL (src/pinocchio_model.cpp:376-496): damped
// least squares on the joint frame's log6 error, integrate(q, v dt)
PinocchioModel::IKResult PinocchioModel::ik_clik(size_t index, const Vec7& pose, const std::vector<double>& q_init,
                                                 const std::vector<bool>* mask, const std::vector<double>* q_min,
                                                 const std::vector<double>* q_max, double eps, int max_iter, double dt,
                                                 double damp) const {
  if (index >= link_index_user2pin_.size()) throw std::runtime_error("The link index is out of bound!");
  const PinFrame& fr = frames_[link_index_user2pin_[index]];
  const int jid = fr.parent;
  const SE3 joint_pose = mpg::se3_mul(pose_se3(pose), se3_inverse(fr.placement));
  const SE3 joint_pose_inv = se3_inverse(joint_pose);
  std::vector<double> q = qpos_user2pin(q_init), qmin, qmax;
  if (q_min) qmin = qpos_user2pin(*q_min);
  if (q_max) qmax = qpos_user2pin(*q_max);
  IKResult r;
  r.success = false;
  for (int i = 0;; ++i) {
    const std::vector<SE3> oMi = joint_frames(q);
    const std::array<double, 6> err = log6(mpg::se3_mul(joint_pose_inv, oMi[jid]));
    r.err = err;
    double n2 = 0.0;
    for (double e : err) n2 += e * e;
    if (std::sqrt(n2) < eps) {
      r.success = true;
      break;
    }
    if (i >= max_iter) break;
    std::vector<double> J = joint_local_jacobian(oMi, jid);
    if (mask)
      for (size_t j = 0; j < mask->size(); ++j)
        if ((*mask)[j]) {
          const int u = joint_index_user2pin_.at(j) - 1;
          for (int k = 0; k < 6; ++k) J[(size_t)k * nv_ + u] = 0.0;
        }
    std::array<double, 36> JJt{};
    for (int a = 0; a < 6; ++a)
      for (int b = 0; b < 6; ++b) {
        double s = 0.0;
        for (int c = 0; c < nv_; ++c) s += J[(size_t)a * nv_ + c] * J[(size_t)b * nv_ + c];
        JJt[6 * a + b] = s + (a == b ? damp : 0.0);
      }
    const std::array<double, 6> y = spd_solve6(JJt, err);
    std::vector<double> v(nv_, 0.0);
    for (int c = 0; c < nv_; ++c) {
      double s = 0.0;
      for (int a = 0; a < 6; ++a) s += J[(size_t)a * nv_ + c] * y[a];
      v[c] = -s * dt;
    }
    for (size_t j = 1; j < joints_.size(); ++j) {  // pinocchio::integrate
      const PinJoint& pj = joints_[j];
      if (pj.nq == 1) {
        q[pj.idx_q] += v[pj.idx_v];
      } else if (pj.nq == 2) {
        const double ca = q[pj.idx_q], sa = q[pj.idx_q + 1], so = std::sin(v[pj.idx_v]), co = std::cos(v[pj.idx_v]);
        double c2 = co * ca - so * sa, s2 = so * ca + co * sa;
        const double k = (3.0 - (c2 * c2 + s2 * s2)) / 2.0;
        q[pj.idx_q] = c2 * k;
        q[pj.idx_q + 1] = s2 * k;
      }
    }
    if (q_min && q_max)  // computeIKCLIKJL's clamp, in pinocchio coordinates
      for (size_t j = 0; j < q.size(); ++j) {
        if (q[j] < qmin[j]) q[j] = std::fabs(qmin[j] + 3.1415926) < 1e-3 ? 3.1415926 : qmin[j];
        if (q[j] > qmax[j]) q[j] = std::fabs(qmin[j] - 3.1415926) < 1e-3 ? -3.1415926 : qmax[j];
      }
  }
  r.q = qpos_pin2user(q);
  return r;
}


// ------------------------------------------------------------------ KDL
namespace {

// KDL::diff(F_cur, F_goal): (p_goal - p_cur, R_cur * rotvec(R_cur^T R_goal))
std::array<double, 6> kdl_diff(const SE3& cur, const SE3& goal) {
  std::array<double, 6> t;
  for (int k = 0; k < 3; ++k) t[k] = goal.p[k] - cur.p[k];
  double Rr[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      Rr[3 * i + j] = (cur.R[i] * goal.R[j] + cur.R[3 + i] * goal.R[3 + j]) + cur.R[6 + i] * goal.R[6 + j];
  double w[3], th, ww[3];
  log3(Rr, w, th);
  matv(cur.R, w, ww);
  for (int k = 0; k < 3; ++k) t[3 + k] = ww[k];
  return t;
}

// solve A x = b for a symmetric positive definite m x m A (Cholesky, row-major)
std::vector<double> chol_solve(std::vector<double> A, int m, std::vector<double> b) {
  for (int j = 0; j < m; ++j) {
    double d = A[(size_t)j * m + j];
    for (int k = 0; k < j; ++k) d -= A[(size_t)j * m + k] * A[(size_t)j * m + k];
    if (!(d > 0)) throw std::runtime_error("KDL IK: singular system");
    const double l = std::sqrt(d);
    A[(size_t)j * m + j] = l;
    for (int i = j + 1; i < m; ++i) {
      double t = A[(size_t)i * m + j];
      for (int k = 0; k < j; ++k) t -= A[(size_t)i * m + k] * A[(size_t)j * m + k];
      A[(size_t)i * m + j] = t / l;
    }
  }
  for (int i = 0; i < m; ++i) {
    double t = b[i];
    for (int k = 0; k < i; ++k) t -= A[(size_t)i * m + k] * b[k];
    b[i] = t / A[(size_t)i * m + i];
  }
  for (int i = m - 1; i >= 0; --i) {
    double t = b[i];
    for (int k = i + 1; k < m; ++k) t -= A[(size_t)k * m + i] * b[k];
    b[i] = t / A[(size_t)i * m + i];
  }
  return b;
}

// (A^T A + lambda I) x = A^T b, A m x n row-major (Levenberg-Marquardt step)
std::vector<double> damped_ls(const std::vector<double>& A, int m, int n, const std::vector<double>& b, double lambda) {
  std::vector<double> N((size_t)n * n, 0.0), r(n, 0.0);
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int k = 0; k < m; ++k) s += A[(size_t)k * n + i] * A[(size_t)k * n + j];
      N[(size_t)i * n + j] = s + (i == j ? lambda : 0.0);
    }
    for (int k = 0; k < m; ++k) r[i] += A[(size_t)k * n + i] * b[k];
  }
  return chol_solve(std::move(N), n, std::move(r));
}

// J^T (J J^T + l2 I)^-1 b, J m x n row-major: the minimum-norm step
// (ChainIkSolverVel_pinv with l2 -> 0, TreeIkSolverVel_wdls with l2 = lambda^2)
std::vector<double> min_norm_step(const std::vector<double>& J, int m, int n, const std::vector<double>& b, double l2) {
  std::vector<double> G((size_t)m * m, 0.0);
  for (int a = 0; a < m; ++a)
    for (int c = 0; c < m; ++c) {
      double s = 0.0;
      for (int k = 0; k < n; ++k) s += J[(size_t)a * n + k] * J[(size_t)c * n + k];
      G[(size_t)a * m + c] = s + (a == c ? l2 : 0.0);
    }
  const std::vector<double> z = chol_solve(std::move(G), m, b);
  std::vector<double> x(n, 0.0);
  for (int j = 0; j < n; ++j)
    for (int a = 0; a < m; ++a) x[j] += J[(size_t)a * n + j] * z[a];
  return x;
}

}  // namespace

KDLModel::KDLModel(const std::string& urdf, const std::vector<std::string>& joint_names,
                   const std::vector<std::string>& link_names, bool verbose)
    : user_joint_names_(joint_names), user_link_names_(link_names) {
  const UrdfModel m = parse_urdf_file(urdf);
  root_ = m.root;
  pin_ = std::make_shared<PinocchioModel>(m, Vec3{0, 0, -9.81}, verbose);
  for (size_t i = 0; i < joint_names.size(); ++i) user_idx_[joint_names[i]] = (int)i;
  // pinocchio joint -> user slot (by name); joints the user did not name stay at 0
  const auto& J = pin_->joints();
  pin_user_.assign(J.size(), -1);
  for (size_t j = 1; j < J.size(); ++j) {
    auto it = user_idx_.find(J[j].name);
    if (it != user_idx_.end()) pin_user_[j] = it->second;
  }
}

std::vector<int> KDLModel::chain(size_t index) const {
  if (index >= user_link_names_.size()) throw std::runtime_error("link index out of bound");
  const int f = pin_->body_frame(user_link_names_[index]);
  if (f < 0) throw std::runtime_error("unknown link " + user_link_names_[index]);
  std::vector<int> c;
  for (int j = pin_->frames()[f].parent; j > 0; j = pin_->joints()[j].parent) c.push_back(j);
  std::reverse(c.begin(), c.end());
  for (int j : c)
    if (pin_user_[j] < 0) throw std::out_of_range("joint " + pin_->joints()[j].name + " is not in joint_names");
  return c;
}

std::vector<SE3> KDLModel::frames_at(const std::vector<double>& q_user) const {
  const auto& J = pin_->joints();
  std::vector<double> qpin(pin_->nq(), 0.0);
  for (size_t j = 1; j < J.size(); ++j) {
    if (pin_user_[j] < 0 || J[j].nq == 0) continue;
    const double v = q_user.at(pin_user_[j]);
    if (J[j].nq == 1) qpin[J[j].idx_q] = v;
    else {
      qpin[J[j].idx_q] = std::cos(v);
      qpin[J[j].idx_q + 1] = std::sin(v);
    }
  }
  return pin_->joint_frames(qpin);
}

SE3 KDLModel::tip(const std::vector<SE3>& oMi, size_t index) const {
  const PinFrame& fr = pin_->frames()[pin_->body_frame(user_link_names_[index])];
  return mpg::se3_mul(oMi[fr.parent], fr.placement);
}

// KDL's chain Jacobian: reference point at the tip, base-frame axes; columns
// in `cols` order (joint ids)
std::vector<double> KDLModel::jacobian(const std::vector<SE3>& oMi, const SE3& T, const std::vector<int>& cols) const {
  const int n = (int)cols.size();
  std::vector<double> Jm(6 * (size_t)n, 0.0);
  for (int c = 0; c < n; ++c) {
    const PinJoint& pj = pin_->joints()[cols[c]];
    const Mot S = act(oMi[cols[c]], joint_subspace(pj));  // (v at the base origin, w)
    double wxp[3];
    cross3(S.w, T.p, wxp);  // velocity of the tip point: v + w x p
    for (int k = 0; k < 3; ++k) {
      Jm[(size_t)k * n + c] = S.v[k] + wxp[k];
      Jm[(size_t)(3 + k) * n + c] = S.w[k];
    }
  }
  return Jm;
}

std::tuple<std::vector<double>, int> KDLModel::chain_ik(size_t index, const std::vector<double>& q0, const Vec7& pose,
                                                      int kind, const std::vector<double>* qmin,
                                                      const std::vector<double>* qmax) const {
  const std::vector<int> c = chain(index);
  const SE3 goal = pose_se3(pose);
  std::vector<double> q = q0;
  const int n = (int)c.size();
  auto err_of = [&](const std::vector<double>& qq) { return kdl_diff(tip(frames_at(qq), index), goal); };
  if (kind != 2) {  // Newton-Raphson (NR / NR_JL)
    for (int it = 0; it < 100; ++it) {
      const std::vector<SE3> oMi = frames_at(q);
      const auto e = kdl_diff(tip(oMi, index), goal);
      bool zero = true;
      for (double x : e) zero &= std::fabs(x) < 1e-6;  // KDL::Equal(twist, Zero, eps)
      if (zero) return {q, 0};
      const std::vector<double> dq =
          min_norm_step(jacobian(oMi, tip(oMi, index), c), 6, n, std::vector<double>(e.begin(), e.end()), 1e-12);
      for (int k = 0; k < n; ++k) {
        double& v = q[pin_user_[c[k]]];
        v += dq[k];
        if (kind == 1) v = std::min(std::max(v, (*qmin)[pin_user_[c[k]]]), (*qmax)[pin_user_[c[k]]]);
      }
    }
    return {q, -5};
  }
  // Levenberg-Marquardt (ChainIkSolverPos_LMA)
  const double L[6] = {1, 1, 1, 0.01, 0.01, 0.01}, eps = 1e-5, eps_joints = 1e-15;
  auto weighted = [&](const std::array<double, 6>& e) {
    std::vector<double> w(6);
    for (int k = 0; k < 6; ++k) w[k] = L[k] * e[k];
    return w;
  };
  auto norm = [](const std::vector<double>& v) {
    double s = 0.0;
    for (double x : v) s += x * x;
    return std::sqrt(s);
  };
  std::vector<double> dp = weighted(err_of(q));
  double dpn = norm(dp);
  if (dpn < eps) return {q, 0};
  auto wjac = [&](const std::vector<double>& qq) {
    const std::vector<SE3> oMi = frames_at(qq);
    std::vector<double> Jm = jacobian(oMi, tip(oMi, index), c);
    for (int r = 0; r < 6; ++r)
      for (int k = 0; k < n; ++k) Jm[(size_t)r * n + k] *= L[r];
    return Jm;
  };
  std::vector<double> Jw = wjac(q);
  double lambda = 10.0, v = 2.0;
  for (int it = 0; it < 500; ++it) {
    const std::vector<double> diffq = damped_ls(Jw, 6, n, dp, lambda);
    std::vector<double> grad(n, 0.0);
    for (int k = 0; k < n; ++k)
      for (int r = 0; r < 6; ++r) grad[k] += Jw[(size_t)r * n + k] * dp[r];
    if (norm(diffq) < eps_joints) return {q, -101};
    if (norm(grad) * norm(grad) < eps_joints * eps_joints) return {q, -100};
    std::vector<double> qn = q;
    for (int k = 0; k < n; ++k) qn[pin_user_[c[k]]] += diffq[k];
    const std::vector<double> dpnew = weighted(err_of(qn));
    const double dpnn = norm(dpnew);
    double den = 0.0;
    for (int k = 0; k < n; ++k) den += diffq[k] * (lambda * diffq[k] + grad[k]);
    const double rho = (dpn * dpn - dpnn * dpnn) / den;
    if (rho > 0) {
      q = qn;
      dp = dpnew;
      dpn = dpnn;
      if (dpn < eps) return {q, 0};
      Jw = wjac(q);
      const double t = 2 * rho - 1;
      lambda = lambda * std::max(1 / 3.0, 1 - t * t * t);
      v = 2;
    } else {
      lambda = lambda * v;
      v = 2 * v;
    }
  }
  return {q, -5};
}

std::tuple<std::vector<double>, int> KDLModel::tree_ik_nr_jl(const std::vector<std::string>& endpoints,
                                                           const std::vector<double>& q0,
                                                           const std::vector<Vec7>& poses,
                                                           const std::vector<double>& qmin,
                                                           const std::vector<double>& qmax) const {
  if (endpoints.size() != poses.size()) throw std::invalid_argument("endpoints and goal_poses differ in length");
  // the tree's joints: every named pinocchio joint with one dof
  std::vector<int> cols;
  for (size_t j = 1; j < pin_->joints().size(); ++j)
    if (pin_user_[j] >= 0 && pin_->joints()[j].nv == 1) cols.push_back((int)j);
  std::vector<int> ends;
  for (auto& e : endpoints) {
    auto it = std::find(user_link_names_.begin(), user_link_names_.end(), e);
    if (it == user_link_names_.end()) throw std::out_of_range("unknown endpoint " + e);
    ends.push_back((int)(it - user_link_names_.begin()));
  }
  std::vector<SE3> goals;
  for (auto& p : poses) goals.push_back(pose_se3(p));
  const int n = (int)cols.size(), m = 6 * (int)ends.size();
  std::vector<double> q = q0;
  for (int it = 0; it < 1000; ++it) {
    const std::vector<SE3> oMi = frames_at(q);
    std::vector<double> Jall((size_t)m * n, 0.0), e(m, 0.0);
    double en2 = 0.0;
    for (size_t k = 0; k < ends.size(); ++k) {
      const SE3 T = tip(oMi, ends[k]);
      const auto d = kdl_diff(T, goals[k]);
      for (int r = 0; r < 6; ++r) {
        e[6 * k + r] = d[r];
        en2 += d[r] * d[r];
      }
      // only the joints supporting this endpoint move it
      const std::vector<int> sup = chain(ends[k]);
      const std::vector<double> Jk = jacobian(oMi, T, cols);
      for (int c = 0; c < n; ++c) {
        if (std::find(sup.begin(), sup.end(), cols[c]) == sup.end()) continue;
        for (int r = 0; r < 6; ++r) Jall[(size_t)(6 * k + r) * n + c] = Jk[(size_t)r * n + c];
      }
    }
    if (std::sqrt(en2) < 1e-6) return {q, 0};
    // TreeIkSolverVel_wdls, lambda 1e-6: J^T (J J^T + lambda^2 I)^-1 e
    const std::vector<double> dq = min_norm_step(Jall, m, n, e, 1e-12);
    for (int c = 0; c < n; ++c) {
      double& v = q[pin_user_[cols[c]]];
      v = std::min(std::max(v + dq[c], qmin[pin_user_[cols[c]]]), qmax[pin_user_[cols[c]]]);
    }
  }
  return {q, -5};
}

}  // namespace mpgh
