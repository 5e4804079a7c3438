// Test shim: compiles the product's FK/math headers (mplib_amd/csrc/mpg_fk.h)
// for the host with g++ -ffp-contract=off so tests can compare them with the
// oracle on a machine without a GPU.  Not part of the product.
#include "../../mplib_amd/csrc/mpg_fk.h"

extern "C" {
int host_fk(int nj, const int* jt, const int* jp, const int* jqs, const double* jqc, const double* jax,
            const double* jpl, int dof, int n_links, const int* lp, const double* lpl, const double* q, long n,
            double* out) {
  mpg::DevWorld w{};
  w.nj = nj; w.dof = dof; w.n_links = n_links;
  w.joint_type = jt; w.joint_parent = jp; w.joint_q_source = jqs; w.joint_q_const = jqc;
  w.joint_axis = jax; w.joint_place = jpl; w.link_parent = lp; w.link_place = lpl;
  mpg::FkState st;
  for (long i = 0; i < n; ++i) {
    mpg::forward_kinematics(w, q + i * dof, st);
    for (int l = 0; l < n_links; ++l) mpg::link_transform(w, st, l, out + (i * n_links + l) * 7);
  }
  return 0;
}
// fp32 broad-phase FK (mpg_broadphase.h bp_fk): every moving object's world
// transform as float R[9] + p[3], plus the quaternion round trip of R that
// the SAT stage uses (rq[9])
int host_bp_objects(int nj, const int* jt, const int* jp, const int* jqs, const double* jqc, const double* jax,
                    const double* jpl, int dof, int n_links, const int* lp, const double* lpl, int n_moving,
                    const int* mlink, const double* moff, const double* q, long n, float* out, float* rq) {
  std::vector<int> mgeom(n_moving, 0);
  mpg_world_desc d{};
  d.n_joints = nj; d.joint_type = jt; d.joint_parent = jp; d.joint_axis = jax; d.joint_placement = jpl;
  d.joint_q_source = jqs; d.joint_q_const = jqc; d.dof = dof;
  d.n_links = n_links; d.link_parent = lp; d.link_placement = lpl;
  d.n_moving = n_moving; d.moving_link = mlink; d.moving_geom = mgeom.data(); d.moving_offset = moff;
  std::vector<double> obb(7, 0.0);
  mpg::BpProgram P;
  mpg::bp_build(&d, obb, P);
  const mpg::BpView b = mpg::bp_view(&d, P);
  std::vector<float> save(12 * (P.n_saves + 1));
  for (long i = 0; i < n; ++i) {
    mpg::bp_fk(b, q + i * dof, save.data(), 1, [&](int m, const mpg::F34& T) {
      float* o = out + (i * n_moving + m) * 12;
      for (int k = 0; k < 9; ++k) o[k] = T.R[k];
      for (int k = 0; k < 3; ++k) o[9 + k] = T.p[k];
      float qq[4];
      mpg::f_mat_to_quat(T.R, qq);
      mpg::f_quat_to_mat(qq[3], qq[0], qq[1], qq[2], rq + (i * n_moving + m) * 9);
    });
  }
  return 0;
}
void host_sincos(const double* x, long n, double* s, double* c, int fma) {
  for (long i = 0; i < n; ++i) {
    if (fma == 1) { s[i] = mpg::mpg_sin<true>(x[i]); c[i] = mpg::mpg_cos<true>(x[i]); }
    else if (fma == 2) mpg::mpg_sincos(x[i], s + i, c + i);
    else { s[i] = mpg::mpg_sin<false>(x[i]); c[i] = mpg::mpg_cos<false>(x[i]); }
  }
}
}
