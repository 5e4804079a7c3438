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
void host_sincos(const double* x, long n, double* s, double* c, int fma) {
  for (long i = 0; i < n; ++i) {
    if (fma) { s[i] = mpg::mpg_sin<true>(x[i]); c[i] = mpg::mpg_cos<true>(x[i]); }
    else { s[i] = mpg::mpg_sin<false>(x[i]); c[i] = mpg::mpg_cos<false>(x[i]); }
  }
}
}
