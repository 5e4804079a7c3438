// Test shim: compiles the product's FK/math headers (mplib_amd/csrc/mpg_fk.h)
// for the host with g++ -ffp-contract=off so tests can compare them with the
// oracle on a machine without a GPU.  Not part of the product.
#include <algorithm>
#include <cfloat>
#include <cmath>

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
static float g_cen_dev = 0.f;  // largest |J * ocen - T.p| seen by host_bp_objects
float host_bp_cen_dev() { return g_cen_dev; }
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
    mpg::bp_fk(b, q + i * dof, save.data(), 1, [&](int m, const mpg::F34& J, const float* jq) {
      // the object's pose J * oplace (checked against the fp64 FK) and the
      // rotation the SAT stage rebuilds from jq * oquat
      const mpg::F34 T = mpg::f34_mul(J, mpg::f34_load(b.oplace + 12 * m));
      float* o = out + (i * n_moving + m) * 12;
      for (int k = 0; k < 9; ++k) o[k] = T.R[k];
      for (int k = 0; k < 3; ++k) o[9 + k] = T.p[k];
      // the OBB centre the cull stores, J * ocen (here the local centre is 0,
      // so it must be T's position)
      for (int k = 0; k < 3; ++k) {
        const float c = J.R[3 * k] * b.ocen[3 * m] + J.R[3 * k + 1] * b.ocen[3 * m + 1] +
                        J.R[3 * k + 2] * b.ocen[3 * m + 2] + J.p[k];
        g_cen_dev = std::max(g_cen_dev, std::fabs(c - T.p[k]));
      }
      const float oq[4] = {b.oquat[4 * m], b.oquat[4 * m + 1], b.oquat[4 * m + 2], b.oquat[4 * m + 3]};
      float qq[4];
      mpg::f_quat_mul(jq, oq, qq);
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
// Convex support through the direction-cell lists (mpg_hullcells.h) next to
// the full first-maximum scan, for n directions; returns the number of
// directions whose results differ, -1 when the hull has no cell table.
// stats[0] = directions that used a cell, stats[1] = total list entries
// scanned, stats[2] = longest list
long host_hull_support(const double* V, int nv, const double* dirs, long n, double* full, double* cell,
                       long* stats) {
  std::vector<uint32_t> start;
  std::vector<double> pts;
  if (!mpg::build_hull_cells(V, nv, start, pts)) return -1;
  std::vector<double> rec, ovf;
  mpg::pack_cell_records(start.data(), pts.data(), rec, ovf);
  if (ovf.empty()) ovf.assign(4, 0.0);
  long bad = 0;
  stats[0] = stats[1] = stats[2] = 0;
  for (long i = 0; i < n; ++i) {
    const double* d = dirs + 3 * i;
    double best = -DBL_MAX;
    int bi = 0;
    for (int k = 0; k < nv; ++k) {
      const double dd = (d[0] * V[3 * k] + d[1] * V[3 * k + 1]) + d[2] * V[3 * k + 2];
      if (dd > best) {
        best = dd;
        bi = k;
      }
    }
    for (int j = 0; j < 3; ++j) full[3 * i + j] = V[3 * bi + j];
    const int c = mpg::hull_cell(d[0], d[1], d[2]);
    if (c < 0) {
      for (int j = 0; j < 3; ++j) cell[3 * i + j] = full[3 * i + j];
      continue;
    }
    const uint32_t e0 = start[c], e1 = start[c + 1];
    stats[0] += 1;
    stats[1] += e1 - e0;
    stats[2] = std::max<long>(stats[2], e1 - e0);
    mpg::cell_record_support(rec.data() + (size_t)mpg::kCellRec * c, ovf.data(), d[0], d[1], d[2], cell + 3 * i);
    if (cell[3 * i] != full[3 * i] || cell[3 * i + 1] != full[3 * i + 1] || cell[3 * i + 2] != full[3 * i + 2]) ++bad;
  }
  return bad;
}
}
