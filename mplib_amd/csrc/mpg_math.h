// mpg_math.h -- fp64 arithmetic shared by the HIP kernels and the host-side
// snapshot builder.  Every function reproduces the operation ORDER of the
// library the reference calls, with no implicit fused multiply-add (all
// translation units are compiled with -ffp-contract=off; fused steps are
// written explicitly with mpg_fma where the reference's binary fuses them).
//
//   * mpg_sin<kFma> / mpg_cos<kFma>: glibc 2.35 sysdeps/ieee754/dbl-64/s_sin.c.
//     kFma = false is the generic build, which is what glibc's sincos() runs
//     on every x86-64 host (sincos has no FMA ifunc variant).  pinocchio's
//     SINCOS (forwardKinematics, pinocchio_model.cpp:272-274) and
//     qposUser2Pinocchio's cos/sin pair (:515-516) both end in sincos(): GCC
//     folds sin(a);cos(a) into one sincos() call.  kFma = true reproduces the
//     standalone sin()/cos() __sin_fma/__cos_fma variants selected on
//     FMA+AVX2 hosts.  Both verified bit-exact against the host libm by
//     tests/test_sincos.py.
//   * Eigen 3.4 quaternion <-> matrix conversions and lazy 3x3 products
//     (pinocchio_model.cpp:299, articulated_model.cpp:119-124,
//     fcl_model.cpp:139-148, FCL shapeToGJK).
//   * libccd 2.1 ccdQuatRotVec / ccdQuatInvert2 / vec3 helpers.
#pragma once

#include <cstdint>
#include <cstring>
#include <cmath>

#include "mpg_sincostab.h"

#if defined(__HIPCC__)
#define MPG_HD __host__ __device__
#define MPG_INLINE __host__ __device__ __forceinline__
#else
#define MPG_HD
#define MPG_INLINE inline
#endif

// Read-only snapshot arrays live in the constant address space on the device:
// uniform reads of them become scalar (s_load) loads through the scalar cache
// instead of vector loads that wait on the vector memory path.
#if defined(__HIP_DEVICE_COMPILE__)
#define MPG_CONST __attribute__((address_space(4)))
#else
#define MPG_CONST
#endif

namespace mpg {

template <class T>
using cptr = const T MPG_CONST*;
template <class T>
MPG_INLINE cptr<T> to_cptr(const void* p) {
  return (cptr<T>)p;
}

constexpr double kSinCosTab[440] = MPG_SINCOSTAB_INIT;

// glibc's FMA build fuses where GCC -mfma contracts; the generic build rounds
// the product first.
template <bool kFma>
MPG_INLINE double mpg_fma(double a, double b, double c) {
  if constexpr (kFma) return __builtin_fma(a, b, c);
  else return a * b + c;
}

MPG_INLINE uint32_t hi_word(double d) {
  uint64_t u;
  std::memcpy(&u, &d, 8);
  return (uint32_t)(u >> 32);
}
MPG_INLINE int32_t lo_word(double d) {
  uint64_t u;
  std::memcpy(&u, &d, 8);
  return (int32_t)(uint32_t)u;
}

// --------------------------------------------------------------------------
// glibc dbl-64 sin/cos.  Constants: sysdeps/ieee754/dbl-64/usncs.h and
// s_sin.c.  kFma: contraction pattern of GCC -mfma -ffp-contract=fast on that
// code (the __sin_fma/__cos_fma ifunc variants); !kFma: the generic build.
// --------------------------------------------------------------------------
namespace sc {
constexpr double sn3 = -1.66666666666664880952546298448555E-01;
constexpr double sn5 = 8.33333214285722277379541354343671E-03;
constexpr double cs2 = 4.99999999999999999999950396842453E-01;
constexpr double cs4 = -4.16666666666664434524222570944589E-02;
constexpr double cs6 = 1.38888874007937613028114285595617E-03;
constexpr double s1 = -0x1.5555555555555p-3;
constexpr double s2 = 0x1.1111111110ECEp-7;
constexpr double s3 = -0x1.a01a019db08b8p-13;
constexpr double s4 = 0x1.71de27b9a7ed9p-19;
constexpr double s5 = -0x1.addffc2fcdf59p-26;
constexpr double big = 0x1.8p45;
constexpr double hp0 = 0x1.921FB54442D18p0;
constexpr double hp1 = 0x1.1A62633145C07p-54;
constexpr double mp1 = 0x1.921FB58000000p0;
constexpr double mp2 = -0x1.DDE973C000000p-27;
constexpr double pp3 = -0x1.CB3B398000000p-55;
constexpr double pp4 = -0x1.d747f23e32ed7p-83;
constexpr double hpinv = 0x1.45F306DC9C883p-1;
constexpr double toint = 0x1.8p52;
}  // namespace sc

template <bool kFma = false>
MPG_INLINE double taylor_sin(double xx, double a, double da) {
  using namespace sc;
  double p = mpg_fma<kFma>(mpg_fma<kFma>(mpg_fma<kFma>(mpg_fma<kFma>(s5, xx, s4), xx, s3), xx, s2), xx, s1);
  double m2 = 0.5 * da;
  double in = mpg_fma<kFma>(p, a, -m2);
  double t = mpg_fma<kFma>(in, xx, da);
  return a + t;
}

template <bool kFma = false>
MPG_INLINE double do_cos(double x, double dx) {
  using namespace sc;
  if (x < 0) dx = -dx;
  double u = big + std::fabs(x);
  x = std::fabs(x) - (u - big) + dx;
  double xx = x * x;
  double s = mpg_fma<kFma>(x * xx, mpg_fma<kFma>(xx, sn5, sn3), x);
  double c = xx * mpg_fma<kFma>(xx, mpg_fma<kFma>(xx, cs6, cs4), cs2);
  int k = lo_word(u) << 2;
  double sn = kSinCosTab[k], ssn = kSinCosTab[k + 1], cs = kSinCosTab[k + 2], ccs = kSinCosTab[k + 3];
  double cor = mpg_fma<kFma>(-sn, s, mpg_fma<kFma>(-cs, c, mpg_fma<kFma>(-s, ssn, ccs)));
  return cs + cor;
}

template <bool kFma = false>
MPG_INLINE double do_sin(double x, double dx) {
  using namespace sc;
  double xold = x;
  if (std::fabs(x) < 0.126) return taylor_sin<kFma>(x * x, x, dx);
  if (x <= 0) dx = -dx;
  double u = big + std::fabs(x);
  x = std::fabs(x) - (u - big);
  double xx = x * x;
  double s = x + mpg_fma<kFma>(x * xx, mpg_fma<kFma>(xx, sn5, sn3), dx);
  double c = mpg_fma<kFma>(x, dx, xx * mpg_fma<kFma>(xx, mpg_fma<kFma>(xx, cs6, cs4), cs2));
  int k = lo_word(u) << 2;
  double sn = kSinCosTab[k], ssn = kSinCosTab[k + 1], cs = kSinCosTab[k + 2], ccs = kSinCosTab[k + 3];
  double cor = mpg_fma<kFma>(cs, s, mpg_fma<kFma>(-sn, c, mpg_fma<kFma>(s, ccs, ssn)));
  return std::copysign(sn + cor, xold);
}

template <bool kFma = false>
MPG_INLINE int reduce_sincos(double x, double* a, double* da) {
  using namespace sc;
  double t = mpg_fma<kFma>(x, hpinv, toint);
  double xn = t - toint;
  double y = mpg_fma<kFma>(-xn, mp2, mpg_fma<kFma>(-xn, mp1, x));
  int n = lo_word(t) & 3;
  double t2 = mpg_fma<kFma>(-xn, pp3, y);
  double db = mpg_fma<kFma>(-xn, pp3, y - t2);
  double b = mpg_fma<kFma>(-xn, pp4, t2);
  db += mpg_fma<kFma>(-xn, pp4, t2 - b);
  *a = b;
  *da = db;
  return n;
}

template <bool kFma = false>
MPG_INLINE double do_sincos(double a, double da, int n) {
  double r = (n & 1) ? do_cos<kFma>(a, da) : do_sin<kFma>(a, da);
  return (n & 2) ? -r : r;
}

// Valid for |x| < 105414350 (glibc's reduce_sincos range); larger arguments
// return NaN and are rejected by the host before launch.
template <bool kFma = false>
MPG_INLINE double mpg_sin(double x) {
  using namespace sc;
  uint32_t k = hi_word(x) & 0x7fffffffu;
  if (k < 0x3e500000u) return x;
  if (k < 0x3feb6000u) return do_sin<kFma>(x, 0);
  if (k < 0x400368fdu) {
    double t = hp0 - std::fabs(x);
    return std::copysign(do_cos<kFma>(t, hp1), x);
  }
  if (k < 0x419921FBu) {
    double a, da;
    int n = reduce_sincos<kFma>(x, &a, &da);
    return do_sincos<kFma>(a, da, n);
  }
  return x - x + NAN;
}

template <bool kFma = false>
MPG_INLINE double mpg_cos(double x) {
  using namespace sc;
  uint32_t k = hi_word(x) & 0x7fffffffu;
  if (k < 0x3e400000u) return 1.0;
  if (k < 0x3feb6000u) return do_cos<kFma>(x, 0);
  if (k < 0x400368fdu) {
    double y = hp0 - std::fabs(x);
    double a = y + hp1;
    double da = (y - a) + hp1;
    return do_sin<kFma>(a, da);
  }
  if (k < 0x419921FBu) {
    double a, da;
    int n = reduce_sincos<kFma>(x, &a, &da);
    return do_sincos<kFma>(a, da, n + 1);
  }
  return x - x + NAN;
}

// do_sin / do_cos with the table index clamped and do_sin's Taylor branch
// turned into a select, so they can run on arguments of an unselected case
// (the result is discarded) without divergence or out-of-range reads.
MPG_INLINE double do_sin_sel(double x, double dx) {
  using namespace sc;
  const double xold = x;
  const double rt = taylor_sin<false>(x * x, x, dx);
  if (x <= 0) dx = -dx;
  const double u = big + std::fabs(x);
  x = std::fabs(x) - (u - big);
  const double xx = x * x;
  const double s = x + mpg_fma<false>(x * xx, mpg_fma<false>(xx, sn5, sn3), dx);
  const double c = mpg_fma<false>(x, dx, xx * mpg_fma<false>(xx, mpg_fma<false>(xx, cs6, cs4), cs2));
  int k = lo_word(u) << 2;
  k = k < 0 ? 0 : k > 436 ? 436 : k;
  const double sn = kSinCosTab[k], ssn = kSinCosTab[k + 1], cs = kSinCosTab[k + 2], ccs = kSinCosTab[k + 3];
  const double cor = mpg_fma<false>(cs, s, mpg_fma<false>(-sn, c, mpg_fma<false>(s, ccs, ssn)));
  return std::fabs(xold) < 0.126 ? rt : std::copysign(sn + cor, xold);
}

MPG_INLINE double do_cos_sel(double x, double dx) {
  using namespace sc;
  if (x < 0) dx = -dx;
  const double u = big + std::fabs(x);
  x = std::fabs(x) - (u - big) + dx;
  const double xx = x * x;
  const double s = mpg_fma<false>(x * xx, mpg_fma<false>(xx, sn5, sn3), x);
  const double c = xx * mpg_fma<false>(xx, mpg_fma<false>(xx, cs6, cs4), cs2);
  int k = lo_word(u) << 2;
  k = k < 0 ? 0 : k > 436 ? 436 : k;
  const double sn = kSinCosTab[k], ssn = kSinCosTab[k + 1], cs = kSinCosTab[k + 2], ccs = kSinCosTab[k + 3];
  const double cor = mpg_fma<false>(-sn, s, mpg_fma<false>(-cs, c, mpg_fma<false>(-s, ssn, ccs)));
  return cs + cor;
}

// glibc __sincos (generic build) with its case analysis turned into selects.
// Every case of __sin/__cos (s_sin.c) ends in exactly one do_sin-kernel and
// one do_cos-kernel evaluation for the pair, so both run once, on selected
// arguments, and the outputs are picked/negated per case.  Bit-identical to
// mpg_sin<false>/mpg_cos<false> (tests/test_sincos.py), without the per-lane
// branch divergence of calling them separately.
MPG_INLINE void mpg_sincos(double x, double* s_out, double* c_out) {
  using namespace sc;
  const uint32_t k = hi_word(x) & 0x7fffffffu;
  const double ax = std::fabs(x);
  const bool c1 = k < 0x3feb6000u, c2 = !c1 && k < 0x400368fdu, c3 = !c1 && !c2 && k < 0x419921FBu;
  // case 2: sin = copysign(do_cos(t2, hp1), x); cos = do_sin(a2, da2)
  const double t2 = hp0 - ax;
  const double a2 = t2 + hp1;
  const double da2 = (t2 - a2) + hp1;
  // case 3: argument reduction
  double a3, da3;
  const int n = reduce_sincos<false>(c3 ? x : 0.0, &a3, &da3);
  const double sa = c1 ? x : c2 ? a2 : a3, sda = c1 ? 0.0 : c2 ? da2 : da3;
  const double ca = c1 ? x : c2 ? t2 : a3, cda = c1 ? 0.0 : c2 ? hp1 : da3;
  const double rs = do_sin_sel(sa, sda);
  const double rc = do_cos_sel(ca, cda);
  double sv, cv;
  if (c1) {
    sv = k < 0x3e500000u ? x : rs;
    cv = k < 0x3e400000u ? 1.0 : rc;
  } else if (c2) {
    sv = std::copysign(rc, x);
    cv = rs;
  } else if (c3) {
    const double rsin = (n & 1) ? rc : rs, rcos = (n & 1) ? rs : rc;
    sv = (n & 2) ? -rsin : rsin;
    cv = ((n + 1) & 2) ? -rcos : rcos;
  } else {
    sv = cv = x - x + NAN;
  }
  *s_out = sv;
  *c_out = cv;
}

// --------------------------------------------------------------------------
// SE(3) as R[9] (row-major) + p[3]
// --------------------------------------------------------------------------
struct SE3 {
  double R[9];
  double p[3];
};

MPG_INLINE void se3_identity(SE3& T) {
  for (int i = 0; i < 9; ++i) T.R[i] = (i % 4 == 0) ? 1.0 : 0.0;
  T.p[0] = T.p[1] = T.p[2] = 0.0;
}

// pinocchio SE3::__mult__ / Eigen Isometry product: R = A.R B.R entries
// ((a_i0 b_0j + a_i1 b_1j) + a_i2 b_2j); p = A.R B.p + A.p.
MPG_INLINE SE3 se3_mul(const SE3& A, const SE3& B) {
  SE3 C;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C.R[3 * i + j] = (A.R[3 * i] * B.R[j] + A.R[3 * i + 1] * B.R[3 + j]) + A.R[3 * i + 2] * B.R[6 + j];
    C.p[i] = ((A.R[3 * i] * B.p[0] + A.R[3 * i + 1] * B.p[1]) + A.R[3 * i + 2] * B.p[2]) + A.p[i];
  }
  return C;
}

// Eigen QuaternionBase::toRotationMatrix, q = (w, x, y, z)
MPG_INLINE void quat_to_mat(double w, double x, double y, double z, double* m) {
  const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  m[0] = 1.0 - (tyy + tzz);
  m[1] = txy - twz;
  m[2] = txz + twy;
  m[3] = txy + twz;
  m[4] = 1.0 - (txx + tzz);
  m[5] = tyz - twx;
  m[6] = txz - twy;
  m[7] = tyz + twx;
  m[8] = 1.0 - (txx + tyy);
}

// Eigen's non-positive-trace branch for a fixed largest diagonal index I
template <int I>
MPG_INLINE void mat_to_quat_diag(const double* m, double* w_out, double* xyz) {
  constexpr int i = I, j = (I + 1) % 3, k = (j + 1) % 3;
  double t = std::sqrt(((m[3 * i + i] - m[3 * j + j]) - m[3 * k + k]) + 1.0);
  const double qi = 0.5 * t;
  t = 0.5 / t;
  *w_out = (m[3 * k + j] - m[3 * j + k]) * t;
  xyz[i] = qi;
  xyz[j] = (m[3 * j + i] + m[3 * i + j]) * t;
  xyz[k] = (m[3 * k + i] + m[3 * i + k]) * t;
}

// Eigen quaternionbase_assign_impl<Matrix3,3,3>; out (w, x, y, z)
MPG_INLINE void mat_to_quat(const double* m, double* w_out, double* xyz) {
  double t = (m[0] + m[4]) + m[8];
  if (t > 0.0) {
    t = std::sqrt(t + 1.0);
    *w_out = 0.5 * t;
    t = 0.5 / t;
    xyz[0] = (m[7] - m[5]) * t;
    xyz[1] = (m[2] - m[6]) * t;
    xyz[2] = (m[3] - m[1]) * t;
  } else {
    int i = 0;
    if (m[4] > m[0]) i = 1;
    if (m[8] > m[3 * i + i]) i = 2;
    // constant indices per branch keep m[] in registers on the GPU
    if (i == 0) mat_to_quat_diag<0>(m, w_out, xyz);
    else if (i == 1) mat_to_quat_diag<1>(m, w_out, xyz);
    else mat_to_quat_diag<2>(m, w_out, xyz);
  }
}

// pinocchio::toRotationMatrix(axis, cos, sin) for unaligned revolute joints
MPG_INLINE void axis_rot(const double* ax, double c, double s, double* R) {
  double sa0 = s * ax[0], sa1 = s * ax[1], sa2 = s * ax[2];
  double c1 = 1.0 - c;
  double ca0 = c1 * ax[0], ca1 = c1 * ax[1], ca2 = c1 * ax[2];
  double tmp;
  tmp = ca0 * ax[1];
  R[1] = tmp - sa2;
  R[3] = tmp + sa2;
  tmp = ca0 * ax[2];
  R[2] = tmp + sa1;
  R[6] = tmp - sa1;
  tmp = ca1 * ax[2];
  R[5] = tmp - sa0;
  R[7] = tmp + sa0;
  R[0] = ca0 * ax[0] + c;
  R[4] = ca1 * ax[1] + c;
  R[8] = ca2 * ax[2] + c;
}

// --------------------------------------------------------------------------
// libccd 2.1 vec3 / quat (ccd/vec3.h, ccd/quat.h) over its scalar ccd_real_t.
// The reference's libccd is a bare `cmake ..` build of v2.1
// (docker/Dockerfile:16-20), whose ENABLE_DOUBLE_PRECISION option defaults to
// OFF: ccd_real_t = float, CCD_EPS = FLT_EPSILON, and FCL 0.7.0's glue
// converts the doubles it hands over (object poses, support points, the MPR
// tolerance) to float.  MPG_CCD_DOUBLE builds the double-precision variant
// (oracle variant "ccd_double", DESIGN.md "Oracle variants").
// V3T<double> (V3) serves the fp64 code outside libccd.
// --------------------------------------------------------------------------
#ifdef MPG_CCD_DOUBLE
using ccd_real = double;
constexpr ccd_real kCcdEps = 2.220446049250313080847e-16;  // DBL_EPSILON
#else
using ccd_real = float;
constexpr ccd_real kCcdEps = 1.19209289550781250e-7f;  // FLT_EPSILON
#endif

// Reach of libccd's MPR false positives (DESIGN.md "Broad-phase soundness"):
// discoverPortal reports "origin on segment v0-v1" (intersect) when
// |v0 x v1|^2 < CCD_EPS.  v0 (centre difference) and the point x where the
// segment v0-v1 crosses the plane through the origin normal to v0 are both in
// the Minkowski difference, so for shapes separated by D, |v0| >= D, |x| >= D
// and |v0 x v1| >= |v0||x| >= D^2: the exit needs D < CCD_EPS^(1/4).  Every
// other MPR exit reports intersection only within ~CCD_EPS of contact.
// float libccd: 0.0186 m; double: 1.2e-4 m.  Culling tests keep every pair
// within this reach (plus rounding) of touching.
constexpr double kCcdFalseHitReach = sizeof(ccd_real) == 4 ? 0.018581 : 1.2208e-4;

template <class T>
struct V3T {
  T x, y, z;
};
using V3 = V3T<double>;
using CV3 = V3T<ccd_real>;

MPG_INLINE V3 v3(double x, double y, double z) { return V3{x, y, z}; }
// ccdVec3Set: converts to ccd_real_t
MPG_INLINE CV3 cv3(double x, double y, double z) { return CV3{(ccd_real)x, (ccd_real)y, (ccd_real)z}; }
MPG_INLINE V3 to_v3(const CV3& a) { return V3{a.x, a.y, a.z}; }
template <class T>
MPG_INLINE V3T<T> vsub(const V3T<T>& a, const V3T<T>& b) { return V3T<T>{a.x - b.x, a.y - b.y, a.z - b.z}; }
template <class T>
MPG_INLINE V3T<T> vadd(const V3T<T>& a, const V3T<T>& b) { return V3T<T>{a.x + b.x, a.y + b.y, a.z + b.z}; }
template <class T>
MPG_INLINE V3T<T> vscale(const V3T<T>& a, T k) { return V3T<T>{a.x * k, a.y * k, a.z * k}; }
template <class T>
MPG_INLINE T vdot(const V3T<T>& a, const V3T<T>& b) {
  T d = a.x * b.x;
  d += a.y * b.y;
  d += a.z * b.z;
  return d;
}
template <class T>
MPG_INLINE V3T<T> vcross(const V3T<T>& a, const V3T<T>& b) {
  return V3T<T>{(a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)};
}
// ccdVec3Normalize: k = CCD_ONE / CCD_SQRT(len2)
template <class T>
MPG_INLINE V3T<T> vnormalize(const V3T<T>& d) {
  const T k = T(1) / std::sqrt(vdot(d, d));
  return vscale(d, k);
}

// quaternion stored (x, y, z, w) as libccd does
template <class T>
struct Q4T {
  T x, y, z, w;
};
using Q4 = Q4T<double>;
using CQ4 = Q4T<ccd_real>;

template <class T>
MPG_INLINE V3T<T> quat_rot(const V3T<T>& v, const Q4T<T>& q) {
  const T vx = v.x, vy = v.y, vz = v.z;
  const T w = q.w, x = q.x, y = q.y, z = q.z;
  const T c1x = y * vz - z * vy + w * vx;
  const T c1y = z * vx - x * vz + w * vy;
  const T c1z = x * vy - y * vx + w * vz;
  const T c2x = y * c1z - z * c1y;
  const T c2y = z * c1x - x * c1z;
  const T c2z = x * c1y - y * c1x;
  return V3T<T>{vx + T(2) * c2x, vy + T(2) * c2y, vz + T(2) * c2z};
}

template <class T>
MPG_INLINE Q4T<T> quat_invert2(const Q4T<T>& q) {
  T len2 = q.x * q.x;
  len2 += q.y * q.y;
  len2 += q.z * q.z;
  len2 += q.w * q.w;
  // ccdQuatInvert returns -1 (leaving dest = src) when len2 < CCD_EPS; unit
  // quaternions from Eigen never take that branch, kept for fidelity.
  if (len2 < (sizeof(T) == 4 ? (T)1.19209289550781250e-7 : (T)2.220446049250313080847e-16)) return q;
  len2 = T(1) / len2;
  return Q4T<T>{-q.x * len2, -q.y * len2, -q.z * len2, q.w * len2};
}

// FCL shapeToGJK: Quaternion<double> q(tf.linear()), then
// ccdQuatSet(&o->rot, q.x(), q.y(), q.z(), q.w()) -> ccd_real_t
MPG_INLINE CQ4 gjk_rot_from_matrix(const double* R) {
  double w, xyz[3];
  mat_to_quat(R, &w, xyz);
  return CQ4{(ccd_real)xyz[0], (ccd_real)xyz[1], (ccd_real)xyz[2], (ccd_real)w};
}

}  // namespace mpg
