// mpg_broadphase.h -- phase A of the batched collide(): a conservative fp32
// broad phase that decides, per (configuration, pair), whether the exact fp64
// narrow phase (FCL/libccd MPR, phase B) has to run at all.
//
// The reference has no broad phase for these pairs: PlanningWorld::collideFull
// (src/planning_world.cpp:484-490) calls ::fcl::collide on every pair.  A pair
// culled here is one whose bounding volumes are separated by more than
// kBpMargin, so MPR would report "no intersection" for it; the output bits are
// therefore identical to evaluating every pair.  Soundness budget (DESIGN.md
// "Broad phase"): fp32 FK + record rounding is bounded by ~2e-5 m for a
// 10-joint chain at 1.5 m reach (measured max 1e-6 m, tests/test_broadphase.py),
// MPR's own tolerance is gjk_tolerance = 1e-6 m; kBpMargin = 1e-4 m covers
// both with >= 5x headroom.
//
// Everything here compiles for the host too (tests/native/host_fk.cpp) so the
// fp32-vs-fp64 pose error is checked on the CPU.
#pragma once
#include <cmath>
#include <vector>

#include "mpg_math.h"
#include "../../include/mpgpu.h"

namespace mpg {

constexpr float kBpMargin = 1e-4f;  // metres
// fp32 cull rounding relative to the largest world coordinate it computes
// (~20 dependent fp32 operations along a chain, each 6e-8 relative: 1.2e-6,
// with 3x headroom); world creation keeps the margin above this times the
// coordinate bound, so far-from-origin worlds keep the soundness argument
constexpr double kFp32CullRel = 4e-6;
// travel bound of a prismatic move-group joint without finite limits (metres)
constexpr double kDefaultTravel = 10.0;

// The broad phase is conservative by its margins, not bit-exact: its fp32
// arithmetic may fuse multiply-adds (more accurate, fewer instructions) even
// though the file is built with -ffp-contract=off for the exact fp64 path.
#ifdef __clang__
#define MPG_FP32_CONTRACT _Pragma("clang fp contract(fast)")
#else
#define MPG_FP32_CONTRACT
#endif

// per moving object float record: local OBB centre, half extents, radius
enum { BM_C = 0, BM_E = 3, BM_R = 6, BM_STRIDE = 8 };
// per static object float record: world OBB centre, axes (R columns), extents
enum { BS_C = 0, BS_R = 3, BS_E = 12, BS_STRIDE = 16 };

// Read-only view of the broad-phase program (device snapshot or host vectors).
struct BpView {
  int nj, n_links, n_moving, n_static, n_saves;
  cptr<int> joint_type;      // [nj]
  cptr<int> joint_q_source;  // [nj]
  cptr<double> joint_q_const;
  cptr<int> jsrc;   // [nj] -1: parent is the universe, 0: previous joint, k>0: save slot k-1
  cptr<int> jsave;  // [nj] save slot or -1
  cptr<float> jaxis;   // [nj*3]
  cptr<float> jplace;  // [nj*12]
  cptr<int> link_start;  // [nj+2] links grouped by parent joint
  cptr<int> link_order;  // [n_links]
  cptr<float> lplace;    // [n_links*12]
  cptr<int> obj_start;   // [n_links+1] moving objects grouped by link
  cptr<int> obj_order;   // [n_moving]
  cptr<int> moving_link; // [n_moving]
  cptr<float> moff;      // [n_moving*12]
  cptr<float> mobj;      // [n_moving*BM_STRIDE]
  cptr<float> sobj;      // [n_static*BS_STRIDE]
  // the fp32 FK program (bp_fk): per joint its motion kind (BpKind) and
  // placement with a constant (non-move-group) motion folded in; the moving
  // objects grouped by their link's parent joint (0 = universe) with
  // link placement * moving offset folded into one transform
  cptr<int> jkind;       // [nj]
  cptr<int> jobj_start;  // [nj+2]
  cptr<int> jobj_order;  // [n_moving]
  cptr<float> oplace;    // [n_moving*12]
  cptr<float> oquat;     // [n_moving*4] rotation of oplace as a quaternion (x, y, z, w)
  cptr<float> ocen;      // [n_moving*3] the object's OBB centre in its joint frame (oplace * local centre)
};

// motion kinds of the fp32 FK: a fixed (or constant) joint, a revolute or
// prismatic joint about a principal axis (x, y, z), or about any unit axis
// (BK_SKIP: a constant joint no other joint hangs from, its objects folded
// into its parent's)
enum BpKind { BK_FIXED = 0, BK_REV_X = 1, BK_REV_AXIS = 4, BK_PRI_X = 5, BK_PRI_AXIS = 8, BK_SKIP = 9 };

struct F34 {
  float R[9];  // row-major
  float p[3];
};

template <class P>
MPG_INLINE F34 f34_load(P a) {
  F34 T;
#pragma unroll
  for (int i = 0; i < 9; ++i) T.R[i] = a[i];
  T.p[0] = a[9];
  T.p[1] = a[10];
  T.p[2] = a[11];
  return T;
}

MPG_INLINE F34 f34_mul(const F34& A, const F34& B) {
  MPG_FP32_CONTRACT
  F34 C;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C.R[3 * i + j] = A.R[3 * i] * B.R[j] + A.R[3 * i + 1] * B.R[3 + j] + A.R[3 * i + 2] * B.R[6 + j];
    C.p[i] = A.R[3 * i] * B.p[0] + A.R[3 * i + 1] * B.p[1] + A.R[3 * i + 2] * B.p[2] + A.p[i];
  }
  return C;
}

MPG_INLINE void f_quat_to_mat(float w, float x, float y, float z, float* m) {
  const float tx = 2.f * x, ty = 2.f * y, tz = 2.f * z;
  const float twx = tx * w, twy = ty * w, twz = tz * w;
  const float txx = tx * x, txy = ty * x, txz = tz * x;
  const float tyy = ty * y, tyz = tz * y, tzz = tz * z;
  m[0] = 1.f - (tyy + tzz);
  m[1] = txy - twz;
  m[2] = txz + twy;
  m[3] = txy + twz;
  m[4] = 1.f - (txx + tzz);
  m[5] = tyz - twx;
  m[6] = txz - twy;
  m[7] = tyz + twx;
  m[8] = 1.f - (txx + tyy);
}

// rotation -> unit quaternion (x, y, z, w); Shepperd's method, branch-free selects
MPG_INLINE void f_mat_to_quat(const float* m, float* q) {
  const float t0 = m[0] + m[4] + m[8];
  const float d0 = 1.f + t0, d1 = 1.f + m[0] - m[4] - m[8], d2 = 1.f - m[0] + m[4] - m[8],
              d3 = 1.f - m[0] - m[4] + m[8];
  int k = 0;
  float best = d0;
  if (d1 > best) { best = d1; k = 1; }
  if (d2 > best) { best = d2; k = 2; }
  if (d3 > best) { best = d3; k = 3; }
  const float s = 0.5f / sqrtf(best);
  const float h = 0.5f * sqrtf(best);
  const float a = (m[7] - m[5]) * s, b = (m[2] - m[6]) * s, c = (m[3] - m[1]) * s;  // w*4 components
  const float e = (m[1] + m[3]) * s, f = (m[2] + m[6]) * s, g = (m[5] + m[7]) * s;
  // k = 0: w = h, (a, b, c); k = 1: x = h, w = a, y = e, z = f; ...
  q[0] = k == 0 ? a : k == 1 ? h : k == 2 ? e : f;
  q[1] = k == 0 ? b : k == 1 ? e : k == 2 ? h : g;
  q[2] = k == 0 ? c : k == 1 ? f : k == 2 ? g : h;
  q[3] = k == 0 ? h : k == 1 ? a : k == 2 ? b : c;
}

// Hamilton product a * b of unit quaternions (x, y, z, w): the rotation
// R(a) R(b)
MPG_INLINE void f_quat_mul(const float* a, const float* b, float* q) {
  MPG_FP32_CONTRACT
  q[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
  q[1] = a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0];
  q[2] = a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3];
  q[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
}

// revolute angles are reduced in fp64 before the fp32 sincos so large user
// values (continuous joints) keep full fp32 accuracy
template <class P>
MPG_INLINE F34 f_joint_motion(int type, P axis, double v) {
  F34 M;
#pragma unroll
  for (int i = 0; i < 9; ++i) M.R[i] = (i % 4 == 0) ? 1.f : 0.f;
  M.p[0] = M.p[1] = M.p[2] = 0.f;
  if (type <= MPG_JOINT_REVOLUTE_UNALIGNED || type >= MPG_JOINT_RUBX) {
    const double k = rint(v * 0.15915494309189535);
    const float a = (float)(v - k * 6.283185307179586);
    const float s = sinf(a), c = cosf(a);  // (__sinf / __cosf measured 5 % faster FK, not worth the weaker bound)
    const int t = (type >= MPG_JOINT_RUBX) ? type - MPG_JOINT_RUBX : type;
    if (t == 0) {
      M.R[4] = c; M.R[5] = -s; M.R[7] = s; M.R[8] = c;
    } else if (t == 1) {
      M.R[0] = c; M.R[2] = s; M.R[6] = -s; M.R[8] = c;
    } else if (t == 2) {
      M.R[0] = c; M.R[1] = -s; M.R[3] = s; M.R[4] = c;
    } else {  // Rodrigues about a unit axis
      const float x = axis[0], y = axis[1], z = axis[2], u = 1.f - c;
      M.R[0] = c + x * x * u;     M.R[1] = x * y * u - z * s; M.R[2] = x * z * u + y * s;
      M.R[3] = y * x * u + z * s; M.R[4] = c + y * y * u;     M.R[5] = y * z * u - x * s;
      M.R[6] = z * x * u - y * s; M.R[7] = z * y * u + x * s; M.R[8] = c + z * z * u;
    }
  } else {
    const float f = (float)v;
    if (type == MPG_JOINT_PX) M.p[0] = f;
    else if (type == MPG_JOINT_PY) M.p[1] = f;
    else if (type == MPG_JOINT_PZ) M.p[2] = f;
    else { M.p[0] = axis[0] * f; M.p[1] = axis[1] * f; M.p[2] = axis[2] * f; }
  }
  return M;
}

// fp32 FK over the whole tree; calls sink(m, J, jq) for every moving object
// with its joint's world frame J and J's rotation as a quaternion jq (one
// conversion per joint with objects): the object's pose is J * oplace[m],
// its rotation jq * oquat[m], its OBB centre J * ocen[m].  Per joint: A = parent *
// placement (one 3x4 product), then the motion applied in place -- a
// principal-axis rotation mixes two columns of A.R, a principal-axis
// translation adds one column to A.p, constant joints were folded into the
// placement on the host -- and per moving object one product with its folded
// link placement * offset.  Joint frames that a later non-consecutive child
// needs are kept in registers for the first kRegSaves slots and spilled to
// `save` ([slot - kRegSaves][12] x stride) beyond that.
constexpr int kRegSaves = 2;

// A * R_k(a) for a principal axis k: the columns (U, W) spanning the rotated
// plane become U' = c U + s W, W' = c W - s U
template <int U, int W>
MPG_INLINE void f_rotate_cols(F34& A, float c, float s) {
  MPG_FP32_CONTRACT
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const float u = A.R[3 * r + U], w = A.R[3 * r + W];
    A.R[3 * r + U] = c * u + s * w;
    A.R[3 * r + W] = c * w - s * u;
  }
}

template <class Sink>
MPG_INLINE void bp_fk(const BpView& b, const double* __restrict__ qrow, float* save, int stride, Sink&& sink) {
  MPG_FP32_CONTRACT
  F34 cur, r0, r1;
  if (b.jobj_start[0] < b.jobj_start[1]) {  // objects on the universe
    F34 I;
#pragma unroll
    for (int k = 0; k < 9; ++k) I.R[k] = (k % 4 == 0) ? 1.f : 0.f;
    I.p[0] = I.p[1] = I.p[2] = 0.f;
    const float iq[4] = {0.f, 0.f, 0.f, 1.f};
    for (int o = b.jobj_start[0]; o < b.jobj_start[1]; ++o) sink(b.jobj_order[o], I, iq);
  }
#pragma unroll 1
  for (int jj = 0; jj < b.nj; ++jj) {
    const int kind = b.jkind[jj];
    if (kind == BK_SKIP) continue;
    const F34 Pl = f34_load(b.jplace + 12 * jj);
    const int s = b.jsrc[jj];
    F34 A;
    if (s < 0) {
      A = Pl;
    } else if (s == 0) {
      A = f34_mul(cur, Pl);
    } else if (s == 1) {
      A = f34_mul(r0, Pl);
    } else if (s == 2) {
      A = f34_mul(r1, Pl);
    } else {
      F34 P;
      const float* sp = save + (size_t)(s - 1 - kRegSaves) * 12 * stride;
#pragma unroll
      for (int i = 0; i < 9; ++i) P.R[i] = sp[i * stride];
#pragma unroll
      for (int i = 0; i < 3; ++i) P.p[i] = sp[(9 + i) * stride];
      A = f34_mul(P, Pl);
    }
    if (kind != BK_FIXED) {
      const double v = qrow[b.joint_q_source[jj]];
      if (kind < BK_PRI_X) {
        // revolute angles are reduced in fp64 before the fp32 sincos so large
        // user values (continuous joints) keep full fp32 accuracy
        const double k = rint(v * 0.15915494309189535);
        const float a = (float)(v - k * 6.283185307179586);
        float sn, cs;
        sincosf(a, &sn, &cs);
        if (kind == BK_REV_AXIS) {
          A = f34_mul(A, f_joint_motion(MPG_JOINT_REVOLUTE_UNALIGNED, b.jaxis + 3 * jj, (double)a));
        } else if (kind == BK_REV_X) {
          f_rotate_cols<1, 2>(A, cs, sn);
        } else if (kind == BK_REV_X + 1) {
          f_rotate_cols<2, 0>(A, cs, sn);
        } else {
          f_rotate_cols<0, 1>(A, cs, sn);
        }
      } else {
        const float f = (float)v;
        if (kind == BK_PRI_AXIS) {
          const float ax[3] = {b.jaxis[3 * jj] * f, b.jaxis[3 * jj + 1] * f, b.jaxis[3 * jj + 2] * f};
#pragma unroll
          for (int r = 0; r < 3; ++r) A.p[r] += A.R[3 * r] * ax[0] + A.R[3 * r + 1] * ax[1] + A.R[3 * r + 2] * ax[2];
        } else {
#pragma unroll
          for (int r = 0; r < 3; ++r)
            A.p[r] += (kind == BK_PRI_X ? A.R[3 * r] : kind == BK_PRI_X + 1 ? A.R[3 * r + 1] : A.R[3 * r + 2]) * f;
        }
      }
    }
    cur = A;
    const int sv = b.jsave[jj];
    if (sv == 0) {
      r0 = cur;
    } else if (sv == 1) {
      r1 = cur;
    } else if (sv >= kRegSaves) {
      float* sp = save + (size_t)(sv - kRegSaves) * 12 * stride;
#pragma unroll
      for (int i = 0; i < 9; ++i) sp[i * stride] = cur.R[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) sp[(9 + i) * stride] = cur.p[i];
    }
    const int o0 = b.jobj_start[jj + 1], o1 = b.jobj_start[jj + 2];
    if (o0 < o1) {
      float jq[4];
      f_mat_to_quat(cur.R, jq);
      for (int o = o0; o < o1; ++o) sink(b.jobj_order[o], cur, jq);
    }
  }
}

// moving object transform from a given link pose (px, py, pz, qw, qx, qy, qz)
MPG_INLINE F34 bp_from_pose7(const BpView& b, const double* p7, int m) {
  F34 L;
  f_quat_to_mat((float)p7[3], (float)p7[4], (float)p7[5], (float)p7[6], L.R);
  L.p[0] = (float)p7[0];
  L.p[1] = (float)p7[1];
  L.p[2] = (float)p7[2];
  return f34_mul(L, f34_load(b.moff + 12 * m));
}

struct FObb {
  float c[3];
  float R[9];  // row-major world rotation: column j = box axis j
  float e[3];
};

// 15-axis separating-axis test with every bound widened by `margin`
MPG_INLINE bool fobb_separated(const FObb& A, const FObb& B, float margin) {
  MPG_FP32_CONTRACT
  const float d[3] = {B.c[0] - A.c[0], B.c[1] - A.c[1], B.c[2] - A.c[2]};
  float Rm[3][3], Ab[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      Rm[i][j] = A.R[i] * B.R[j] + A.R[3 + i] * B.R[3 + j] + A.R[6 + i] * B.R[6 + j];
      Ab[i][j] = fabsf(Rm[i][j]) + 1e-6f;
    }
  float t[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = d[0] * A.R[i] + d[1] * A.R[3 + i] + d[2] * A.R[6 + i];
  bool sep = false;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float rb = B.e[0] * Ab[i][0] + B.e[1] * Ab[i][1] + B.e[2] * Ab[i][2];
    sep |= fabsf(t[i]) > A.e[i] + rb + margin;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float ra = A.e[0] * Ab[0][j] + A.e[1] * Ab[1][j] + A.e[2] * Ab[2][j];
    const float tb = t[0] * Rm[0][j] + t[1] * Rm[1][j] + t[2] * Rm[2][j];
    sep |= fabsf(tb) > ra + B.e[j] + margin;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      const float ra = A.e[i1] * Ab[i2][j] + A.e[i2] * Ab[i1][j];
      const float rb = B.e[j1] * Ab[i][j2] + B.e[j2] * Ab[i][j1];
      const float tl = t[i2] * Rm[i1][j] - t[i1] * Rm[i2][j];
      sep |= fabsf(tl) > ra + rb + margin;
    }
  }
  return sep;
}

// moving-object bounding sphere vs static OBB
template <class P>
MPG_INLINE bool fsphere_obb_separated(const float* c, float r, P sobj, float margin) {
  MPG_FP32_CONTRACT
  const float d[3] = {c[0] - sobj[BS_C], c[1] - sobj[BS_C + 1], c[2] - sobj[BS_C + 2]};
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float t = d[0] * sobj[BS_R + j] + d[1] * sobj[BS_R + 3 + j] + d[2] * sobj[BS_R + 6 + j];
    const float ex = fmaxf(fabsf(t) - sobj[BS_E + j], 0.f);
    acc += ex * ex;
  }
  const float rr = r + margin;
  return acc > rr * rr;
}

// Two static OBB records at once (interleaved: field k of record i at
// 2 k + i), packed fp32 math: bit i set when record i's OBB is NOT separated
// from the sphere (c, r) by more than margin (the negation of
// fsphere_obb_separated, same arithmetic per lane and record)
#ifdef __clang__
typedef float mpg_f2 __attribute__((ext_vector_type(2)));
template <class P>
MPG_INLINE uint32_t fsphere_obb_keep2(const float* c, float r, P rec, float margin) {
  MPG_FP32_CONTRACT
  auto ld = [&](int k) { return mpg_f2{rec[2 * k], rec[2 * k + 1]}; };
  const mpg_f2 d0 = c[0] - ld(BS_C), d1 = c[1] - ld(BS_C + 1), d2 = c[2] - ld(BS_C + 2);
  mpg_f2 acc = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const mpg_f2 t = d0 * ld(BS_R + j) + d1 * ld(BS_R + 3 + j) + d2 * ld(BS_R + 6 + j);
    const mpg_f2 a = mpg_f2{fabsf(t.x), fabsf(t.y)} - ld(BS_E + j);
    const mpg_f2 ex = mpg_f2{fmaxf(a.x, 0.f), fmaxf(a.y, 0.f)};
    acc += ex * ex;
  }
  const float rr = r + margin;
  const float r2 = rr * rr;
  return (uint32_t)!(acc.x > r2) | ((uint32_t)!(acc.y > r2) << 1);
}
#else  // host compilers without vector extensions (tests/native): the same per record
template <class P>
inline uint32_t fsphere_obb_keep2(const float* c, float r, P rec, float margin) {
  float a[BS_STRIDE], b[BS_STRIDE];
  for (int k = 0; k < BS_STRIDE; ++k) {
    a[k] = rec[2 * k];
    b[k] = rec[2 * k + 1];
  }
  return (uint32_t)!fsphere_obb_separated(c, r, a, margin) | ((uint32_t)!fsphere_obb_separated(c, r, b, margin) << 1);
}
#endif

// ---------------------------------------------------------------------------
// host: build the program from a world descriptor + the per-geometry local
// OBB records (centre, half extents, bounding radius about that centre)
// ---------------------------------------------------------------------------
struct BpProgram {
  int n_saves = 0;
  std::vector<int> jsrc, jsave, link_start, link_order, obj_start, obj_order, jkind, jobj_start, jobj_order;
  std::vector<float> jaxis, jplace, lplace, moff, mobj, sobj, oplace, oquat, ocen;
};

// row-major 3x4 product in fp64 (host program folding)
inline void se3d_mul(const double* A, const double* B, double* C) {
  double T[12];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    T[9 + i] = A[3 * i] * B[9] + A[3 * i + 1] * B[10] + A[3 * i + 2] * B[11] + A[9 + i];
  }
  for (int k = 0; k < 12; ++k) C[k] = T[k];
}

// unit quaternion (x, y, z, w) of a row-major rotation, fp64 (Shepperd)
inline void mat_to_quat_d(const double* m, double* q) {
  const double d[4] = {1.0 + m[0] + m[4] + m[8], 1.0 + m[0] - m[4] - m[8], 1.0 - m[0] + m[4] - m[8],
                       1.0 - m[0] - m[4] + m[8]};
  int k = 0;
  for (int i = 1; i < 4; ++i)
    if (d[i] > d[k]) k = i;
  const double h = 0.5 * std::sqrt(d[k]), s = 0.25 / h;
  if (k == 0) {
    q[3] = h; q[0] = (m[7] - m[5]) * s; q[1] = (m[2] - m[6]) * s; q[2] = (m[3] - m[1]) * s;
  } else if (k == 1) {
    q[0] = h; q[3] = (m[7] - m[5]) * s; q[1] = (m[1] + m[3]) * s; q[2] = (m[2] + m[6]) * s;
  } else if (k == 2) {
    q[1] = h; q[3] = (m[2] - m[6]) * s; q[0] = (m[1] + m[3]) * s; q[2] = (m[5] + m[7]) * s;
  } else {
    q[2] = h; q[3] = (m[3] - m[1]) * s; q[0] = (m[2] + m[6]) * s; q[1] = (m[5] + m[7]) * s;
  }
}

// a joint's motion at value v in fp64 (pinocchio's joint models)
inline void joint_motion_d(int type, const double* axis, double v, double* M) {
  for (int k = 0; k < 12; ++k) M[k] = (k == 0 || k == 4 || k == 8) ? 1.0 : 0.0;
  if (type <= MPG_JOINT_REVOLUTE_UNALIGNED || type >= MPG_JOINT_RUBX) {
    const double s = std::sin(v), c = std::cos(v);
    const int t = type >= MPG_JOINT_RUBX ? type - MPG_JOINT_RUBX : type;
    const double x = t == 0 ? 1.0 : t == 3 ? axis[0] : 0.0, y = t == 1 ? 1.0 : t == 3 ? axis[1] : 0.0,
                 z = t == 2 ? 1.0 : t == 3 ? axis[2] : 0.0, u = 1.0 - c;
    const double R[9] = {c + x * x * u,     x * y * u - z * s, x * z * u + y * s, y * x * u + z * s, c + y * y * u,
                         y * z * u - x * s, z * x * u - y * s, z * y * u + x * s, c + z * z * u};
    for (int k = 0; k < 9; ++k) M[k] = R[k];
  } else {
    const int t = type - MPG_JOINT_PX;
    for (int k = 0; k < 3; ++k) M[9 + k] = (t == 3 ? axis[k] : (t == k ? 1.0 : 0.0)) * v;
  }
}

inline float widen(double v) {  // |v| rounded away from zero, plus a hair
  const float f = (float)std::fabs(v);
  return std::nextafter(f, INFINITY) * (1.f + 1e-6f) + 1e-7f;
}

// obb[g*7] = local centre (3), half extents (3), radius about the centre
inline void bp_build(const mpg_world_desc* d, const std::vector<double>& obb, BpProgram& P) {
  const int nj = d->n_joints, nl = d->n_links, nm = d->n_moving, ns = d->n_static;
  P.jsrc.assign(std::max(nj, 1), -1);
  P.jsave.assign(std::max(nj, 1), -1);
  std::vector<int> need_save(nj + 1, 0);
  for (int j = 1; j <= nj; ++j) {
    const int par = d->joint_parent[j - 1];
    if (par > 0 && par != j - 1) need_save[par] = 1;
  }
  int slots = 0;
  std::vector<int> slot_of(nj + 1, -1);
  for (int j = 1; j <= nj; ++j)
    if (need_save[j]) slot_of[j] = slots++;
  P.n_saves = slots;
  for (int j = 1; j <= nj; ++j) {
    const int par = d->joint_parent[j - 1];
    P.jsrc[j - 1] = par == 0 ? -1 : par == j - 1 ? 0 : slot_of[par] + 1;
    P.jsave[j - 1] = slot_of[j];
  }
  for (int i = 0; i < 3 * nj; ++i) P.jaxis.push_back((float)d->joint_axis[i]);
  P.jkind.assign(std::max(nj, 1), BK_FIXED);
  std::vector<double> jpl_d((size_t)12 * std::max(nj, 1), 0.0);  // the placements in fp64
  for (int j = 0; j < nj; ++j) {
    const int t = d->joint_type[j];
    double Pl[12];
    for (int k = 0; k < 12; ++k) Pl[k] = d->joint_placement[12 * j + k];
    if (d->joint_q_source[j] < 0) {  // constant motion: folded into the placement
      double M[12];
      joint_motion_d(t, d->joint_axis + 3 * j, d->joint_q_const[j], M);
      se3d_mul(Pl, M, Pl);
    } else if (t <= MPG_JOINT_REVOLUTE_UNALIGNED || t >= MPG_JOINT_RUBX) {
      const int a = t >= MPG_JOINT_RUBX ? t - MPG_JOINT_RUBX : t;
      P.jkind[j] = BK_REV_X + a;
    } else {
      P.jkind[j] = BK_PRI_X + (t - MPG_JOINT_PX);
    }
    for (int k = 0; k < 12; ++k) P.jplace.push_back((float)Pl[k]);
    for (int k = 0; k < 12; ++k) jpl_d[12 * j + k] = Pl[k];
  }
  // constant joints that no joint hangs from (leaves first, so chains of
  // them fold too): skipped, their objects ride on the parent's frame
  std::vector<int> live_children(nj + 1, 0);
  for (int j = 1; j <= nj; ++j) ++live_children[d->joint_parent[j - 1]];
  for (int j = nj; j >= 1; --j)
    if (P.jkind[j - 1] == BK_FIXED && live_children[j] == 0) {
      P.jkind[j - 1] = BK_SKIP;
      --live_children[d->joint_parent[j - 1]];
    }
  for (int i = 0; i < 12 * nl; ++i) P.lplace.push_back((float)d->link_placement[i]);
  for (int i = 0; i < 12 * nm; ++i) P.moff.push_back((float)d->moving_offset[i]);
  P.link_start.assign(nj + 2, 0);
  for (int j = 0; j <= nj; ++j) {
    P.link_start[j] = (int)P.link_order.size();
    for (int l = 0; l < nl; ++l)
      if (d->link_parent[l] == j) P.link_order.push_back(l);
  }
  P.link_start[nj + 1] = (int)P.link_order.size();
  P.obj_start.assign(nl + 1, 0);
  for (int l = 0; l < nl; ++l) {
    P.obj_start[l] = (int)P.obj_order.size();
    for (int m = 0; m < nm; ++m)
      if (d->moving_link[m] == l) P.obj_order.push_back(m);
  }
  P.obj_start[nl] = (int)P.obj_order.size();
  // objects by the joint whose frame carries them (their link's parent joint,
  // or its first ancestor that is not skipped), every placement from there
  // to the collision origin folded into one transform
  std::vector<int> ojoint(std::max(nm, 1), 0);
  std::vector<double> ofold((size_t)12 * std::max(nm, 1), 0.0);
  for (int m = 0; m < nm; ++m) {
    double* O = ofold.data() + 12 * m;
    se3d_mul(d->link_placement + 12 * d->moving_link[m], d->moving_offset + 12 * m, O);
    int j = d->link_parent[d->moving_link[m]];
    while (j > 0 && P.jkind[j - 1] == BK_SKIP) {
      se3d_mul(jpl_d.data() + 12 * (j - 1), O, O);
      j = d->joint_parent[j - 1];
    }
    ojoint[m] = j;
  }
  P.jobj_start.assign(nj + 2, 0);
  P.oplace.assign((size_t)12 * std::max(nm, 1), 0.f);
  for (int j = 0; j <= nj; ++j) {
    P.jobj_start[j] = (int)P.jobj_order.size();
    for (int m = 0; m < nm; ++m)
      if (ojoint[m] == j) P.jobj_order.push_back(m);
  }
  P.jobj_start[nj + 1] = (int)P.jobj_order.size();
  P.oquat.assign((size_t)4 * std::max(nm, 1), 0.f);
  P.ocen.assign((size_t)3 * std::max(nm, 1), 0.f);
  for (int m = 0; m < nm; ++m) {
    const double* O = ofold.data() + 12 * m;
    for (int k = 0; k < 12; ++k) P.oplace[12 * m + k] = (float)O[k];
    double q[4];
    mat_to_quat_d(O, q);
    for (int k = 0; k < 4; ++k) P.oquat[4 * m + k] = (float)q[k];
    const double* g = obb.data() + 7 * d->moving_geom[m];  // local OBB centre
    for (int i = 0; i < 3; ++i)
      P.ocen[3 * m + i] = (float)(O[3 * i] * g[0] + O[3 * i + 1] * g[1] + O[3 * i + 2] * g[2] + O[9 + i]);
  }
  P.mobj.assign((size_t)BM_STRIDE * std::max(nm, 1), 0.f);
  for (int m = 0; m < nm; ++m) {
    const double* g = obb.data() + 7 * d->moving_geom[m];
    float* r = P.mobj.data() + BM_STRIDE * m;
    for (int k = 0; k < 3; ++k) r[BM_C + k] = (float)g[k];
    for (int k = 0; k < 3; ++k) r[BM_E + k] = widen(g[3 + k]);
    r[BM_R] = widen(g[6]);
  }
  P.sobj.assign((size_t)BS_STRIDE * std::max(ns, 1), 0.f);
  for (int s = 0; s < ns; ++s) {
    const double* T = d->static_transform + 12 * s;
    const double* g = obb.data() + 7 * d->static_geom[s];
    float* r = P.sobj.data() + BS_STRIDE * s;
    for (int i = 0; i < 3; ++i)
      r[BS_C + i] = (float)(T[3 * i] * g[0] + T[3 * i + 1] * g[1] + T[3 * i + 2] * g[2] + T[9 + i]);
    for (int k = 0; k < 9; ++k) r[BS_R + k] = (float)T[k];
    for (int k = 0; k < 3; ++k) r[BS_E + k] = widen(g[3 + k]);
  }
}

inline BpView bp_view(const mpg_world_desc* d, const BpProgram& P) {
  BpView b{};
  b.nj = d->n_joints;
  b.n_links = d->n_links;
  b.n_moving = d->n_moving;
  b.n_static = d->n_static;
  b.n_saves = P.n_saves;
  b.joint_type = to_cptr<int>(d->joint_type);
  b.joint_q_source = to_cptr<int>(d->joint_q_source);
  b.joint_q_const = to_cptr<double>(d->joint_q_const);
  b.jsrc = to_cptr<int>(P.jsrc.data());
  b.jsave = to_cptr<int>(P.jsave.data());
  b.jaxis = to_cptr<float>(P.jaxis.data());
  b.jplace = to_cptr<float>(P.jplace.data());
  b.link_start = to_cptr<int>(P.link_start.data());
  b.link_order = to_cptr<int>(P.link_order.data());
  b.lplace = to_cptr<float>(P.lplace.data());
  b.obj_start = to_cptr<int>(P.obj_start.data());
  b.obj_order = to_cptr<int>(P.obj_order.data());
  b.moving_link = to_cptr<int>(d->moving_link);
  b.moff = to_cptr<float>(P.moff.data());
  b.mobj = to_cptr<float>(P.mobj.data());
  b.sobj = to_cptr<float>(P.sobj.data());
  b.jkind = to_cptr<int>(P.jkind.data());
  b.jobj_start = to_cptr<int>(P.jobj_start.data());
  b.jobj_order = to_cptr<int>(P.jobj_order.data());
  b.oplace = to_cptr<float>(P.oplace.data());
  b.oquat = to_cptr<float>(P.oquat.data());
  b.ocen = to_cptr<float>(P.ocen.data());
  return b;
}

}  // namespace mpg
