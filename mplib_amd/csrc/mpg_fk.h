// mpg_fk.h -- device snapshot layout + forward kinematics shared by the HIP
// kernels and the host-side self test (tests/test_host_fk.py compiles this
// header with g++ -ffp-contract=off).
//
//   setQposAll/setQpos   src/planning_world.cpp:250-262, src/articulated_model.cpp:101-127
//   forwardKinematics    [ext pinocchio 2.6.21]: oMi[i] = oMi[parent] * (jointPlacement_i * M_i(q))
//   getLinkPose          src/pinocchio_model.cpp:277-312 (quaternion round trip)
#pragma once
#include "mpg_math.h"
#include "mpg_broadphase.h"
#include "mpg_hullcells.h"
#include "../../include/mpgpu.h"

namespace mpg {

constexpr int kMaxJoints = 32;

// per-geometry double record
// G_OBB_E: local AABB half extents widened for rounding (bounding tests);
// G_AABB_E: the exact half extents (hi - lo) * 0.5 of FCL's computeBV
enum { G_PARAM = 0, G_INTERIOR = 4, G_OBB_C = 7, G_OBB_E = 10, G_RADIUS = 13, G_VMAX = 14, G_AABB_E = 15, G_STRIDE = 18 };
// per-static-object double record
enum { S_ROT = 0, S_ROTINV = 4, S_POS = 8, S_OBBC = 11, S_R = 14, S_STRIDE = 23 };

struct DevWorld {
  int nj, dof, n_links, n_geoms, n_moving, n_static, n_pairs, W;
  double mpr_tol;
  float bp_margin;      // phase-A culling margin (metres), kBpMargin or the libccd false-hit reach
  double small_margin;  // the latency path's bounding-sphere margin, same rule
  int debug_mode;  // diagnostics only: 1 = broad-phase records only, 2 = no SAT stage, 3 = no MPR (latency path: no narrow test), 5 / 6 = no mesh-mesh / mesh-shape walks, 7 = latency path: FK + sphere test only
  unsigned long long* stats;  // diagnostics only (MPG_STATS=1), else NULL
  // the ablation switch as the kernels read it: compiled in only under the
  // MPG_DIAG macro (tools/ablate*.sh build such a library); the product
  // library ignores MPG_DEBUG_CULL entirely, so no result can change
  MPG_INLINE bool dbg(int k) const {
#ifdef MPG_DIAG
    return debug_mode == k;
#else
    (void)k;
    return false;
#endif
  }
  cptr<int> joint_type;      // [nj]
  cptr<int> joint_parent;    // [nj]
  cptr<int> joint_q_source;  // [nj]
  cptr<double> joint_q_const;
  cptr<double> joint_axis;   // [nj*3]
  cptr<double> joint_place;  // [nj*12]
  cptr<int> link_parent;     // [n_links]
  cptr<double> link_place;   // [n_links*12]
  cptr<int> geom_type;       // [n_geoms]
  cptr<int> geom_gstart;     // [n_geoms] first 4-vertex group in `hull`
  cptr<int> geom_ng;         // [n_geoms] number of groups
  cptr<int> geom_nvert;      // [n_geoms] convex vertex count
  cptr<double> geom_rec;     // [n_geoms*G_STRIDE]
  cptr<double> hull;         // AoSoA-4 vertex groups: x0..3 y0..3 z0..3
  int hull_doubles;
  cptr<int> geom_cbase;      // [n_geoms] first cell record of the hull, -1 = none (full scan)
  cptr<double> cell_rec;     // kCellsPerHull records of kCellRec doubles per hull (mpg_hullcells.h)
  cptr<double> cell_ovf;     // list entries beyond the inline ones: x, y, z, 0
  // FCL 0.7.0 neighbour-walk hulls (mpg_hullcells.h): geom_nbr[g] = the
  // hull's first vertex in hull_nbr, -1 = linear support.  hull_nbr holds per
  // vertex (first entry, count) of its sorted neighbour list in nbr_ent, whose
  // entries carry the neighbour's coordinates inline (x, y, z, index): one
  // load per climb step.  Then the hull's cell records (kCellRec doubles,
  // indexed by geom_cbase) and their overflow entries.
  cptr<int> geom_nbr;
  cptr<int> hull_nbr;
  cptr<double> nbr_ent;
  cptr<double> wcell_rec;
  cptr<double> wcell_ovf;
  cptr<double> wcell_aux;  // trapped (sub)cells' verification data (mpg_hullcells.h)
  cptr<int> wcell_end;     // certified walk endpoints of the trapped subcells' fine cells
  cptr<int> wcell_end2;    // ... and of the finer cells of uncertified fine cells
  cptr<int> wcell_pre;     // climb prefix records of still undecided finer cells (WalkPrefix)
  int walk_subk;           // subcells per axis of a trapped cell
  cptr<int> moving_link;     // [n_moving]
  cptr<int> moving_geom;
  cptr<double> moving_offset;  // [n_moving*12]
  cptr<int> static_geom;     // [n_static]
  cptr<double> static_rec;   // [n_static*S_STRIDE]
  cptr<int> pair_a;          // [n_pairs]
  cptr<int> pair_b;
  cptr<int> pair_allowed;
  cptr<int> pair_cf;          // [n_pairs] CF_* closed-form kind (0 = MPR)
  cptr<double> static_T;      // [n_static*12] world transforms as given
  // per user link: the joints from the root to link_parent[l] (1-based,
  // root first) -- lets a thread rebuild one link's oMi without the others
  cptr<int> link_chain_start;  // [n_links]
  cptr<int> link_chain_len;    // [n_links]
  cptr<int> chain_joints;
  BpView bp;  // fp32 broad-phase program (mpg_broadphase.h)
  // phase-A pair schedule (entry e: pair sched_pair[e]).  Moving-moving
  // pairs by their lower object m: entries [sched_start[m], sched_start[m+1])
  // with the partner in sched_other.  Moving-static pairs static-major:
  // entries [st_start[g*(n_static+1) + s], st_start[g*(n_static+1) + s + 1])
  // pair static s with the moving objects st_m (bounding radius st_r); group
  // g = 0 those the object's reach ball can bring near, g = 1 the rest
  // (link-pose input only)
  cptr<int> sched_start;  // [n_moving+1]
  cptr<int> sched_pair;
  cptr<int> sched_other;
  cptr<int> st_start;     // [2 * (n_static + 1)]
  cptr<int> st_m;         // [entries]
  cptr<float> st_r;       // [entries]
  int n_prism;              // prismatic move-group joints with a value bound (a configuration beyond it: every pair)
  cptr<double> prism_bound; // [nj] |q| bound of such a joint, 0 = none
  double pose_bound;        // link-pose input: |position| bound of every link (beyond it: every pair)
  cptr<int> all_mask;       // [W] bits of every non-allowed pair
  // visited sets of walk hulls above kMaxWalkVerts vertices (wave_walk):
  // big_slots slots of big_words words, all zero while free; big_busy[slot]
  unsigned long long* big_vis;
  int* big_busy;
  int big_slots, big_words;
  // octrees: leaf boxes [L][6] (octree frame), per geometry a uniform grid
  // record (OG_*), cell -> leaf lists (CSR)
  cptr<double> oct_leaf;
  cptr<double> oct_grid;   // [n_geoms * OG_STRIDE]
  cptr<int> oct_cells;     // cell start offsets into oct_list
  cptr<int> oct_list;      // leaf indices
  // per leaf its path in FCL's octree (getRootBV halved by computeChildBV):
  // child indices 3 bits per level, the root's first (most significant),
  // and the number of levels (OcTreeMeshIntersectRecurse's gate)
  cptr<uint64_t> oct_path;
  cptr<int> oct_depth;
  // BVH meshes: one record per triangle (TR_*, mesh frame) grouped into
  // spatial clusters (the leaves of a median-split tree): cluster box [6],
  // cluster (first triangle record, triangle count), per geometry (first
  // cluster, cluster count)
  cptr<double> mesh_tri;
  cptr<double> mesh_node;
  cptr<int> mesh_link;  // [clusters * 2]
  cptr<int> mesh_tree;  // [n_geoms * 2]
  // FCL 0.7.0 BVHModel<OBBRSS> of every mesh (OBB half; build_fcl_bvh):
  // nodes [N][FB_STRIDE] (axis row-major, centre, half extents), links [N][3]
  // (first child as a global node index, or -(triangle + 1) for a leaf; first
  // primitive position; primitive count), per geometry its root (-1: none),
  // per triangle (mesh_triangle order) its position in the leaf order; per
  // geometry the OBB FCL's computeBV gives the shape in its own frame
  cptr<double> fb_box;
  cptr<int> fb_link;
  cptr<int> fb_root;   // [n_geoms]
  cptr<int> tri_pos;   // [n_mesh_triangles]
  cptr<double> sobb;   // [n_geoms][FB_STRIDE]
  // latency path: per pair one contiguous record of everything its FK and
  // bounding test read (LR_*; lat_rec_ok = every chain fits kLatChain)
  cptr<double> lat_rec;  // [n_pairs][LR_STRIDE]
  int lat_rec_ok;
};
constexpr int kLatChain = 12;
// latency pair record: header, then per side (0 = pair_a, 1 = pair_b) the
// chain of joints (type, source, constant, axis[3], placement[12] each), the
// link placement, the moving offset (static side: its world transform) and
// the geometry's bounding-sphere centre
enum { LR_ALLOWED = 0, LR_CF = 1, LR_GA = 2, LR_GB = 3, LR_AM = 4, LR_BM = 5, LR_RA = 6, LR_RB = 7, LR_SIDE = 8 };
enum { LS_CL = 0, LS_LINKPL = 1, LS_OFF = 13, LS_OBBC = 25, LS_J = 28, LJ_STRIDE = 18,
       LS_STRIDE = LS_J + kLatChain * LJ_STRIDE };
enum { LR_STRIDE = LR_SIDE + 2 * LS_STRIDE };
enum { FB_AXIS = 0, FB_TO = 9, FB_EXT = 12, FB_STRIDE = 15 };
enum { OG_ORIGIN = 0, OG_INV = 3, OG_DIMS = 4, OG_CELL0 = 7, OG_STRIDE = 8 };
// triangle record: vertices P1 P2 P3, the triangle's AABB, its index in the mesh
enum { TR_P = 0, TR_LO = 9, TR_HI = 12, TR_ID = 15, TR_STRIDE = 16 };

template <class P>
MPG_INLINE SE3 load_se3(P p) {
  SE3 T;
#pragma unroll
  for (int i = 0; i < 9; ++i) T.R[i] = p[i];
  T.p[0] = p[9];
  T.p[1] = p[10];
  T.p[2] = p[11];
  return T;
}

// pinocchio JointModel*::calc as a plain SE3 (see oracle/collide_oracle.c)
MPG_INLINE bool joint_is_revolute(int type) { return type <= MPG_JOINT_REVOLUTE_UNALIGNED || type >= MPG_JOINT_RUBX; }

// sc: optional precomputed (mpg_sin(v), mpg_cos(v)) for revolute joints
template <class P>
MPG_INLINE SE3 joint_motion(int type, P axis, double v, const double* sc = nullptr) {
  SE3 M;
  se3_identity(M);
  if (joint_is_revolute(type)) {
    double s, c;
    if (sc) {
      s = sc[0];
      c = sc[1];
    } else {
      mpg_sincos(v, &s, &c);
    }
    const int t = (type >= MPG_JOINT_RUBX) ? type - MPG_JOINT_RUBX : type;
    if (t == 0) {
      M.R[4] = c; M.R[5] = -s; M.R[7] = s; M.R[8] = c;
    } else if (t == 1) {
      M.R[0] = c; M.R[2] = s; M.R[6] = -s; M.R[8] = c;
    } else if (t == 2) {
      M.R[0] = c; M.R[1] = -s; M.R[3] = s; M.R[4] = c;
    } else {
      axis_rot(axis, c, s, M.R);
    }
  } else if (type == MPG_JOINT_PX) {
    M.p[0] = v;
  } else if (type == MPG_JOINT_PY) {
    M.p[1] = v;
  } else if (type == MPG_JOINT_PZ) {
    M.p[2] = v;
  } else {  // prismatic unaligned: translation = axis * q
    M.p[0] = axis[0] * v;
    M.p[1] = axis[1] * v;
    M.p[2] = axis[2] * v;
  }
  return M;
}

// Forward kinematics for one configuration; oMi in thread-private storage.
struct FkState {
  SE3 oMi[kMaxJoints + 1];
};

MPG_HD inline void forward_kinematics(const DevWorld& w, const double* __restrict__ qrow, FkState& st) {
  se3_identity(st.oMi[0]);
  for (int j = 1; j <= w.nj; ++j) {
    const int src = w.joint_q_source[j - 1];
    const double v = src >= 0 ? qrow[src] : w.joint_q_const[j - 1];
    const SE3 M = joint_motion(w.joint_type[j - 1], w.joint_axis + 3 * (j - 1), v);
    const SE3 li = se3_mul(load_se3(w.joint_place + 12 * (j - 1)), M);
    const int par = w.joint_parent[j - 1];
    st.oMi[j] = par > 0 ? se3_mul(st.oMi[par], li) : li;
  }
}

// oMi[link_parent[l]] by folding liMi along the link's joint chain: the same
// products, in the same order, as forward_kinematics (oMi[j] = oMi[parent] *
// liMi[j], oMi[j] = liMi[j] when the parent is the universe), without storing
// the other joints.
// screw: optional [dof][2] exact (sin, cos) of the row's joint values
// (computed once per configuration by phase A), used for revolute joints
MPG_INLINE SE3 chain_oMi(const DevWorld& w, const double* __restrict__ qrow, int l,
                         const double* __restrict__ screw = nullptr) {
  const int cs = w.link_chain_start[l], cl = w.link_chain_len[l];
  SE3 T;
  se3_identity(T);
  for (int k = 0; k < cl; ++k) {
    const int j = w.chain_joints[cs + k];
    const int src = w.joint_q_source[j - 1];
    const int type = w.joint_type[j - 1];
    const bool pre = screw && src >= 0 && joint_is_revolute(type);
    const double v = pre ? 0.0 : src >= 0 ? qrow[src] : w.joint_q_const[j - 1];
    const SE3 M = joint_motion(type, w.joint_axis + 3 * (j - 1), v, pre ? screw + 2 * src : nullptr);
    const SE3 li = se3_mul(load_se3(w.joint_place + 12 * (j - 1)), M);
    T = k == 0 ? li : se3_mul(T, li);
  }
  return T;
}

// Quaternion round trip of getLinkPose (pinocchio_model.cpp:277-312) then the
// re-matrix of ArticulatedModel::setQpos (articulated_model.cpp:119-124).
MPG_INLINE SE3 link_from_oMi(const DevWorld& w, const SE3& oMi_parent, int l, double* pose7) {
  const SE3 L = se3_mul(oMi_parent, load_se3(w.link_place + 12 * l));
  double qw, qxyz[3];
  mat_to_quat(L.R, &qw, qxyz);
  SE3 T;
  quat_to_mat(qw, qxyz[0], qxyz[1], qxyz[2], T.R);
  T.p[0] = L.p[0];
  T.p[1] = L.p[1];
  T.p[2] = L.p[2];
  if (pose7) {
    pose7[0] = L.p[0]; pose7[1] = L.p[1]; pose7[2] = L.p[2];
    pose7[3] = qw; pose7[4] = qxyz[0]; pose7[5] = qxyz[1]; pose7[6] = qxyz[2];
  }
  return T;
}

// getLinkPose + ArticulatedModel::setQpos re-matrix: returns the link
// Isometry FCL sees, plus the (p, wxyz) pose vector.
MPG_INLINE SE3 link_transform(const DevWorld& w, const FkState& st, int l, double* pose7) {
  return link_from_oMi(w, st.oMi[w.link_parent[l]], l, pose7);
}

}  // namespace mpg
