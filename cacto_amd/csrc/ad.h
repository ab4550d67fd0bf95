// Forward-mode derivatives for the DDP backward pass of the non-constant systems:
// hyper-dual numbers f(x + a e1 + b e2 + ab e1 e2), e1^2 = e2^2 = 0. One evaluation of a function
// on hyper-dual inputs yields its value, two directional derivatives and the mixed second
// derivative, each exact up to rounding (no step size). Used for
//   * dtau/dq, dtau/dv of RNEA(q, v, qdd) -> ddq_dq = -M^-1 dtau/dq, ddq_dv = -M^-1 dtau/dv, i.e.
//     Pinocchio's computeABADerivatives (environment.py:111-132) — one RNEA per joint gives the
//     q-direction (a part) and the v-direction (b part) of that joint;
//   * the TO cost's derivatives in a point: the EE position of a chain (environment_TO.py:605-631,
//     :731-758) or a car_park check point (:479-503) — three passes give its gradient and Hessian,
//     which ddp_kernels.hip composes with the kinematics (chain rule); chains with a prismatic joint
//     before the EE fall back to hyper-dual forward kinematics, one pass per (j <= k) joint pair.
// The spatial algebra mirrors env.h (Pinocchio ordering (linear, angular)), templated on the
// scalar; the rigid-body inertias stay float64 constants.
#pragma once
#include "env.h"

namespace cacto {

// the HD overloads below must not hide the float64 math functions from code in this namespace
using ::exp;
using ::log;
using ::sincos;
using ::sqrt;

struct HD {
  double v, a, b, ab;
  __device__ HD() = default;
  __device__ constexpr HD(double x) : v(x), a(0.0), b(0.0), ab(0.0) {}
  __device__ constexpr HD(double x, double da, double db, double dab) : v(x), a(da), b(db), ab(dab) {}
};
__device__ __forceinline__ HD operator+(HD x, HD y) { return HD(x.v + y.v, x.a + y.a, x.b + y.b, x.ab + y.ab); }
__device__ __forceinline__ HD operator-(HD x, HD y) { return HD(x.v - y.v, x.a - y.a, x.b - y.b, x.ab - y.ab); }
__device__ __forceinline__ HD operator-(HD x) { return HD(-x.v, -x.a, -x.b, -x.ab); }
__device__ __forceinline__ HD operator*(HD x, HD y) {
  return HD(x.v * y.v, x.v * y.a + x.a * y.v, x.v * y.b + x.b * y.v, x.v * y.ab + x.a * y.b + x.b * y.a + x.ab * y.v);
}
__device__ __forceinline__ HD operator*(double s, HD x) { return HD(s * x.v, s * x.a, s * x.b, s * x.ab); }
__device__ __forceinline__ HD operator*(HD x, double s) { return s * x; }
__device__ __forceinline__ HD operator+(HD x, double s) { return HD(x.v + s, x.a, x.b, x.ab); }
__device__ __forceinline__ HD operator+(double s, HD x) { return x + s; }
__device__ __forceinline__ HD operator-(HD x, double s) { return HD(x.v - s, x.a, x.b, x.ab); }
__device__ __forceinline__ HD operator-(double s, HD x) { return HD(s - x.v, -x.a, -x.b, -x.ab); }
// f(x) for a scalar f with f' = d1, f'' = d2 at x.v
__device__ __forceinline__ HD chain1(HD x, double f, double d1, double d2) {
  return HD(f, d1 * x.a, d1 * x.b, d1 * x.ab + d2 * x.a * x.b);
}
__device__ __forceinline__ HD recip(HD x) {
  const double r = 1.0 / x.v;
  return chain1(x, r, -r * r, 2.0 * r * r * r);
}
__device__ __forceinline__ HD operator/(HD x, HD y) { return x * recip(y); }
__device__ __forceinline__ HD operator/(HD x, double s) { return (1.0 / s) * x; }
__device__ __forceinline__ HD sqrt(HD x) {
  const double r = ::sqrt(x.v);
  return chain1(x, r, 0.5 / r, -0.25 / (r * x.v));
}
__device__ __forceinline__ HD exp(HD x) {
  const double e = ::exp(x.v);
  return chain1(x, e, e, e);
}
__device__ __forceinline__ HD log(HD x) { return chain1(x, ::log(x.v), 1.0 / x.v, -1.0 / (x.v * x.v)); }
__device__ __forceinline__ void sincos(HD x, HD* s, HD* c) {
  double sv, cv;
  ::sincos(x.v, &sv, &cv);
  *s = chain1(x, sv, cv, -sv);
  *c = chain1(x, cv, -sv, -cv);
}

// ------------------------------------------------------------------ templated spatial algebra
template <typename T>
struct V3T {
  T x, y, z;
};
template <typename T>
__device__ __forceinline__ V3T<T> operator+(const V3T<T>& a, const V3T<T>& b) {
  return {a.x + b.x, a.y + b.y, a.z + b.z};
}
template <typename T>
__device__ __forceinline__ V3T<T> operator-(const V3T<T>& a, const V3T<T>& b) {
  return {a.x - b.x, a.y - b.y, a.z - b.z};
}
template <typename T, typename S>
__device__ __forceinline__ V3T<T> scale3(const S& s, const V3T<T>& a) {
  return {s * a.x, s * a.y, s * a.z};
}
template <typename T>
__device__ __forceinline__ T dot3(const V3T<T>& a, const V3T<T>& b) {
  return a.x * b.x + a.y * b.y + a.z * b.z;
}
template <typename T>
__device__ __forceinline__ V3T<T> cross3(const V3T<T>& a, const V3T<T>& b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
template <typename T>
__device__ __forceinline__ V3T<T> lift(V3 a) {
  return {T(a.x), T(a.y), T(a.z)};
}
template <typename T>
struct M3T {
  T m[9];
};
template <typename T>
__device__ __forceinline__ V3T<T> mulv(const M3T<T>& R, const V3T<T>& v) {
  return {R.m[0] * v.x + R.m[1] * v.y + R.m[2] * v.z, R.m[3] * v.x + R.m[4] * v.y + R.m[5] * v.z,
          R.m[6] * v.x + R.m[7] * v.y + R.m[8] * v.z};
}
template <typename T>
__device__ __forceinline__ V3T<T> mulTv(const M3T<T>& R, const V3T<T>& v) {
  return {R.m[0] * v.x + R.m[3] * v.y + R.m[6] * v.z, R.m[1] * v.x + R.m[4] * v.y + R.m[7] * v.z,
          R.m[2] * v.x + R.m[5] * v.y + R.m[8] * v.z};
}
template <typename T>
__device__ __forceinline__ M3T<T> mulm(const M3T<T>& A, const M3T<T>& B) {
  M3T<T> C;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) C.m[r * 3 + c] = A.m[r * 3] * B.m[c] + A.m[r * 3 + 1] * B.m[3 + c] + A.m[r * 3 + 2] * B.m[6 + c];
  return C;
}
template <typename T>
struct SVT {
  V3T<T> l, a;
};
template <typename T>
struct SE3T {
  M3T<T> R;
  V3T<T> p;
};

// R0 * rot(axis, q) (revolute) or (R0, p0 + R0 axis q) (prismatic): joint_placement of env.h
template <typename T>
__device__ inline SE3T<T> joint_placement_t(const JointView& j, T q) {
  const M3 R0d = j.R0();
  M3T<T> R0;
#pragma unroll
  for (int k = 0; k < 9; ++k) R0.m[k] = T(R0d.m[k]);
  const V3 ax = j.axis();
  SE3T<T> X;
  if (j.kind() == 0) {
    T s, c;
    sincos(q, &s, &c);
    const T t = 1.0 - c;
    M3T<T> R;
    R.m[0] = c + t * (ax.x * ax.x);
    R.m[1] = t * (ax.x * ax.y) - s * ax.z;
    R.m[2] = t * (ax.x * ax.z) + s * ax.y;
    R.m[3] = t * (ax.x * ax.y) + s * ax.z;
    R.m[4] = c + t * (ax.y * ax.y);
    R.m[5] = t * (ax.y * ax.z) - s * ax.x;
    R.m[6] = t * (ax.x * ax.z) - s * ax.y;
    R.m[7] = t * (ax.y * ax.z) + s * ax.x;
    R.m[8] = c + t * (ax.z * ax.z);
    X.R = mulm(R0, R);
    X.p = lift<T>(j.p0());
  } else {
    X.R = R0;
    X.p = lift<T>(j.p0()) + mulv(R0, V3T<T>{q * ax.x, q * ax.y, q * ax.z});
  }
  return X;
}
// parent -> child motion: (R^T (v_l - p x v_a), R^T v_a)
template <typename T>
__device__ __forceinline__ SVT<T> act_motion_inv_t(const SE3T<T>& X, const SVT<T>& v) {
  return {mulTv(X.R, v.l - cross3(X.p, v.a)), mulTv(X.R, v.a)};
}
// child -> parent force: (R f_l, R f_a + p x R f_l)
template <typename T>
__device__ __forceinline__ SVT<T> act_force_t(const SE3T<T>& X, const SVT<T>& f) {
  const V3T<T> Rl = mulv(X.R, f.l);
  return {Rl, mulv(X.R, f.a) + cross3(X.p, Rl)};
}
template <typename T>
__device__ __forceinline__ SVT<T> cross_motion_t(const SVT<T>& v, const SVT<T>& m) {
  return {cross3(v.a, m.l) + cross3(v.l, m.a), cross3(v.a, m.a)};
}
template <typename T>
__device__ __forceinline__ SVT<T> cross_force_t(const SVT<T>& v, const SVT<T>& f) {
  return {cross3(v.a, f.l), cross3(v.a, f.a) + cross3(v.l, f.l)};
}
// I (origin form: m, h = m c, Io) times a motion: (m v_l - h x v_a, Io v_a + h x v_l)
template <typename T>
__device__ __forceinline__ SVT<T> inertia_mul_t(const Inertia& I, const SVT<T>& v) {
  const V3T<T> h = lift<T>(I.h);
  const V3T<T>& w = v.a;
  const V3T<T> Iw{I.Io.xx * w.x + I.Io.xy * w.y + I.Io.xz * w.z, I.Io.xy * w.x + I.Io.yy * w.y + I.Io.yz * w.z,
                  I.Io.xz * w.x + I.Io.yz * w.y + I.Io.zz * w.z};
  return {scale3(I.m, v.l) - cross3(h, v.a), Iw + cross3(h, v.l)};
}

// RNEA tau(q, v, qdd) of a serial chain (Featherstone Table 5.1, a_0 = -gravity).
template <int NJ, typename T>
__device__ inline void rnea_t(const SysDevice& sd, const T* q, const T* v, const double* qdd, T* tau) {
  SE3T<T> X[NJ];
  SVT<T> f[NJ];
  SVT<T> vp{{T(0.0), T(0.0), T(0.0)}, {T(0.0), T(0.0), T(0.0)}};
  SVT<T> ap{{T(-sd.p.gravity[0]), T(-sd.p.gravity[1]), T(-sd.p.gravity[2])}, {T(0.0), T(0.0), T(0.0)}};
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const JointView j{sd.joints + i * CACTO_JOINT_COLS};
    X[i] = joint_placement_t<T>(j, q[i]);
    const SV S = joint_S(j);
    const SVT<T> Sv{scale3(v[i], lift<T>(S.l)), scale3(v[i], lift<T>(S.a))};
    SVT<T> vi = act_motion_inv_t(X[i], vp);
    vi.l = vi.l + Sv.l;
    vi.a = vi.a + Sv.a;
    SVT<T> ai = act_motion_inv_t(X[i], ap);
    const SVT<T> c = cross_motion_t(vi, Sv);
    ai.l = ai.l + c.l + lift<T>(qdd[i] * S.l);
    ai.a = ai.a + c.a + lift<T>(qdd[i] * S.a);
    const Inertia I = j.inertia();
    const SVT<T> Iv = inertia_mul_t(I, vi), Ia = inertia_mul_t(I, ai);
    const SVT<T> vf = cross_force_t(vi, Iv);
    f[i] = {Ia.l + vf.l, Ia.a + vf.a};
    vp = vi;
    ap = ai;
  }
#pragma unroll
  for (int i = NJ - 1; i >= 0; --i) {
    const JointView j{sd.joints + i * CACTO_JOINT_COLS};
    const SV S = joint_S(j);
    tau[i] = dot3(lift<T>(S.l), f[i].l) + dot3(lift<T>(S.a), f[i].a);
    if (i > 0) {
      const SVT<T> fp = act_force_t(X[i], f[i]);
      f[i - 1].l = f[i - 1].l + fp.l;
      f[i - 1].a = f[i - 1].a + fp.a;
    }
  }
}

// Two-tangent numbers (value, d/dq_k, d/dv_k): the a and b parts of HD without the mixed part,
// for the RNEA derivative passes, which read only tau.a and tau.b. Every a / b component is formed
// by HD's formula, so the results are those of the HD pass bit for bit, at 3/4 of the registers.
struct TD {
  double v, a, b;
  __device__ TD() = default;
  __device__ constexpr TD(double x) : v(x), a(0.0), b(0.0) {}
  __device__ constexpr TD(double x, double da, double db) : v(x), a(da), b(db) {}
};
__device__ __forceinline__ TD operator+(TD x, TD y) { return TD(x.v + y.v, x.a + y.a, x.b + y.b); }
__device__ __forceinline__ TD operator-(TD x, TD y) { return TD(x.v - y.v, x.a - y.a, x.b - y.b); }
__device__ __forceinline__ TD operator-(TD x) { return TD(-x.v, -x.a, -x.b); }
__device__ __forceinline__ TD operator*(TD x, TD y) {
  return TD(x.v * y.v, x.v * y.a + x.a * y.v, x.v * y.b + x.b * y.v);
}
__device__ __forceinline__ TD operator*(double s, TD x) { return TD(s * x.v, s * x.a, s * x.b); }
__device__ __forceinline__ TD operator*(TD x, double s) { return s * x; }
__device__ __forceinline__ TD operator+(TD x, double s) { return TD(x.v + s, x.a, x.b); }
__device__ __forceinline__ TD operator+(double s, TD x) { return x + s; }
__device__ __forceinline__ TD operator-(TD x, double s) { return TD(x.v - s, x.a, x.b); }
__device__ __forceinline__ TD operator-(double s, TD x) { return TD(s - x.v, -x.a, -x.b); }
__device__ __forceinline__ void sincos(TD x, TD* s, TD* c) {
  double sv, cv;
  ::sincos(x.v, &sv, &cv);
  *s = TD(sv, cv * x.a, cv * x.b);
  *c = TD(cv, -sv * x.a, -sv * x.b);
}

// Dual numbers (value, one tangent): one direction of the RNEA derivative passes on its own
// thread. The tangent is formed by TD's (and HD's) formula for that component, so it is the same
// value bit for bit.
struct DN {
  double v, a;
  __device__ DN() = default;
  __device__ constexpr DN(double x) : v(x), a(0.0) {}
  __device__ constexpr DN(double x, double da) : v(x), a(da) {}
};
__device__ __forceinline__ DN operator+(DN x, DN y) { return DN(x.v + y.v, x.a + y.a); }
__device__ __forceinline__ DN operator-(DN x, DN y) { return DN(x.v - y.v, x.a - y.a); }
__device__ __forceinline__ DN operator-(DN x) { return DN(-x.v, -x.a); }
__device__ __forceinline__ DN operator*(DN x, DN y) { return DN(x.v * y.v, x.v * y.a + x.a * y.v); }
__device__ __forceinline__ DN operator*(double s, DN x) { return DN(s * x.v, s * x.a); }
__device__ __forceinline__ DN operator*(DN x, double s) { return s * x; }
__device__ __forceinline__ DN operator+(DN x, double s) { return DN(x.v + s, x.a); }
__device__ __forceinline__ DN operator+(double s, DN x) { return x + s; }
__device__ __forceinline__ DN operator-(DN x, double s) { return DN(x.v - s, x.a); }
__device__ __forceinline__ DN operator-(double s, DN x) { return DN(s - x.v, -x.a); }
__device__ __forceinline__ void sincos(DN x, DN* s, DN* c) {
  double sv, cv;
  ::sincos(x.v, &sv, &cv);
  *s = DN(sv, cv * x.a);
  *c = DN(cv, -sv * x.a);
}

// rnea_t for the derivative passes (T = TD, DN) with the joint placements recomputed in the
// backward sweep instead of held from the forward one (NJ SE3 of tangent numbers was most of the
// pass's registers); joint_placement_t is deterministic, so the values are the same.
template <int NJ, typename T>
__device__ inline void rnea_tan(const SysDevice& sd, const T* q, const T* v, const double* qdd, T* tau) {
  SVT<T> f[NJ];
  SVT<T> vp{{T(0.0), T(0.0), T(0.0)}, {T(0.0), T(0.0), T(0.0)}};
  SVT<T> ap{{T(-sd.p.gravity[0]), T(-sd.p.gravity[1]), T(-sd.p.gravity[2])}, {T(0.0), T(0.0), T(0.0)}};
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const JointView j{sd.joints + i * CACTO_JOINT_COLS};
    const SE3T<T> X = joint_placement_t<T>(j, q[i]);
    const SV S = joint_S(j);
    const SVT<T> Sv{scale3(v[i], lift<T>(S.l)), scale3(v[i], lift<T>(S.a))};
    SVT<T> vi = act_motion_inv_t(X, vp);
    vi.l = vi.l + Sv.l;
    vi.a = vi.a + Sv.a;
    SVT<T> ai = act_motion_inv_t(X, ap);
    const SVT<T> c = cross_motion_t(vi, Sv);
    ai.l = ai.l + c.l + lift<T>(qdd[i] * S.l);
    ai.a = ai.a + c.a + lift<T>(qdd[i] * S.a);
    const Inertia I = j.inertia();
    const SVT<T> Iv = inertia_mul_t(I, vi), Ia = inertia_mul_t(I, ai);
    const SVT<T> vf = cross_force_t(vi, Iv);
    f[i] = {Ia.l + vf.l, Ia.a + vf.a};
    vp = vi;
    ap = ai;
  }
#pragma unroll
  for (int i = NJ - 1; i >= 0; --i) {
    const JointView j{sd.joints + i * CACTO_JOINT_COLS};
    const SV S = joint_S(j);
    tau[i] = dot3(lift<T>(S.l), f[i].l) + dot3(lift<T>(S.a), f[i].a);
    if (i > 0) {
      const SVT<T> fp = act_force_t(joint_placement_t<T>(j, q[i]), f[i]);
      f[i - 1].l = f[i - 1].l + fp.l;
      f[i - 1].a = f[i - 1].a + fp.a;
    }
  }
}

// World translation of the EE frame (framesForwardKinematics + oMf['EE'].translation).
template <int NJ, typename T>
__device__ inline V3T<T> chain_ee_t(const SysDevice& sd, const T* q) {
  M3T<T> oR;
  V3T<T> op, ee{T(0.0), T(0.0), T(0.0)};
  const int e = sd.p.ee_parent;
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const JointView j{sd.joints + i * CACTO_JOINT_COLS};
    const SE3T<T> X = joint_placement_t<T>(j, q[i]);
    if (i == 0) {
      oR = X.R;
      op = X.p;
    } else {
      op = mulv(oR, X.p) + op;
      oR = mulm(oR, X.R);
    }
    if (i == e) ee = mulv(oR, V3T<T>{T(sd.p.ee_p[0]), T(sd.p.ee_p[1]), T(sd.p.ee_p[2])}) + op;
  }
  return ee;
}

// ------------------------------------------------------------------ TO cost pieces (reward = -cost)
// log(exp(alpha * -(e - 1)) + 1) / alpha
template <typename T>
__device__ __forceinline__ T soft_ell_t(double alpha, const T& e) {
  return log(exp(alpha * -(e - 1.0)) + 1.0) / alpha;
}
// peak = log(exp(alpha2 * -sum_c(sqrt(d_c^2 + .1) - sqrt(.1) - .1)) + 1) / alpha2 over NC coordinates
template <int NC, typename T>
__device__ __forceinline__ T peak_t(double alpha2, const T* d) {
  T s = T(0.0);
#pragma unroll
  for (int c = 0; c < NC; ++c) s = s + (sqrt(d[c] * d[c] + 0.1) - ::sqrt(0.1) - 0.1);
  return log(exp(alpha2 * -s) + 1.0) / alpha2;
}

// Position part of the reward of the chain systems at EE position p (no velocity / control
// terms): manipulator (planar ellipses, environment_TO.py:605-631) and UR5 (ellipsoids, :731-758).
template <typename T>
__device__ inline T chain_pos_reward_t(const cacto_sys_params& P, const double* w, const V3T<T>& p) {
  const bool ur5 = P.reward_kind == CACTO_REW_UR5;
  T d[3] = {p.x - P.target[0], p.y - P.target[1], p.z - P.target[2]};
  T cost;
  if (ur5) {
    cost = w[0] * (d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) - w[1] * peak_t<3>(P.alpha2, d);
    for (int k = 0; k < 3; ++k) {
      const double* c = P.obs + 3 * k;
      const double* ax = P.obs + 9 + 3 * k;
      const T ex = p.x - c[0], ey = p.y - c[1], ez = p.z - c[2];
      const T e = ex * ex / ((ax[0] / 2) * (ax[0] / 2)) + ey * ey / ((ax[1] / 2) * (ax[1] / 2)) +
                  ez * ez / ((ax[2] / 2) * (ax[2] / 2));
      cost = cost + w[3 + k] * soft_ell_t(P.alpha, e);
    }
  } else {
    cost = w[0] * (d[0] * d[0] + d[1] * d[1]) - w[1] * peak_t<2>(P.alpha2, d);
    for (int k = 0; k < 3; ++k) {
      const T ex = p.x - P.obs[2 * k], ey = p.y - P.obs[2 * k + 1];
      const double A = P.obs[6 + 2 * k], B = P.obs[7 + 2 * k];
      const T e = ex * ex / ((A / 2) * (A / 2)) + ey * ey / ((B / 2) * (B / 2));
      cost = cost + w[3 + k] * soft_ell_t(P.alpha, e);
    }
  }
  return -(P.scale * cost);
}

// obs_cost_fun (environment_TO.py:457-461) at one check point, fv = 1
template <typename T>
__device__ inline T box_cost_t(const T& x, const T& y, double xs, double ys, double Wx, double Wy, double k) {
  const T ay = (y - ys) + Wy / 2, by = (y - ys) - Wy / 2;
  const T ax = (x - xs) + Wx / 2, bx = (x - xs) - Wx / 2;
  const T q1 = sqrt(4.0 + 4.0 * (ay * ay) * (k * k)), q2 = sqrt(4.0 + 4.0 * (by * by) * (k * k));
  const T q3 = sqrt(4.0 + 4.0 * (ax * ax) * (k * k)), q4 = sqrt(4.0 + 4.0 * (bx * bx) * (k * k));
  return (-0.5 * q2 + by * k) / (q1 * q2) * (0.5 * q1 + ay * k) * (0.5 * q3 + ax * k) / (q3 * q4) *
         (-0.5 * q4 + bx * k);
}

}  // namespace cacto
