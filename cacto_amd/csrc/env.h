// Device-side CACTO environments in float64: chain dynamics (Pinocchio computeAllTerms + solve,
// computeABADerivatives.Minv, framePlacement), analytic single-integrator dynamics, rewards and the
// float32 TF pieces of reward_batch. One thread evaluates one sample.
//
// Reference: environment.py (Env :10-163, SingleIntegrator :165-286, DoubleIntegrator :288-362,
// Manipulator :654-734, UR5 :736-816), robot_utils.py:348-432 (RobotSimulator.step/simulate).
#pragma once

#include "common.h"

namespace cacto {

struct SysDevice {
  cacto_sys_params p;
  double joints[CACTO_MAX_JOINTS * CACTO_JOINT_COLS];
  double inv_norm[CACTO_MAX_STATE];  // 1.0 / state_norm (the reference's 1/state_norm_arr, f64)
  // prismatic-only chains (p.const_dyn): the Cholesky factor of M, the bias forces h and the
  // derivative Fu [ns][na] (row-normalised), computed once on the device at system creation
  // (k_const_dyn_init) by the same code the per-sample path runs — M and h do not depend on (q, v)
  double cd_L[CACTO_MAX_JOINTS * CACTO_MAX_JOINTS];
  double cd_h[CACTO_MAX_JOINTS];
  double cd_Fu[CACTO_MAX_STATE * CACTO_MAX_ACTION];
  // 3-joint planar chains (every joint revolute about z, identity placement rotations, no in-plane
  // gravity: the manipulator): the link constants of the closed-form M(q) and h(q, v) the rollout
  // kernels step with (planar3_step below), filled by cacto_sys_create; pl[0] = 1 when they apply
  double pl[20];
};

// ------------------------------------------------------------------ planar 3R closed form
// For a chain of revolute-z joints whose links move in the xy plane (Manipulator,
// environment.py:654-734, conf_manipulator.py's planar_manipulator_3dof.urdf), M(q) and the bias
// forces h(q, v) = C(q, v) v (gravity along z does no work) follow from the link COM positions:
//   M_ij = sum_{k >= max(i,j)} m_k r_ik . r_jk + Izz_k,   h_i = sum_{k >= i} m_k r_ik x a_k,
// with r_ik the vector from joint i to the COM of link k and a_k that COM's acceleration at
// qdd = 0 (every link-fixed vector rotating at w_j = v_0 + ... + v_j contributes -w_j^2 times
// itself). Everything is expressed in link 0's frame, so only q1, q2 enter. Equal to CRBA / RNEA
// to rounding (the rollout tests hold it to 1e-12 of the oracle's Featherstone restatement).
// Layout of SysDevice::pl (host: cacto_sys_create): [0] on, [1,2] joint-1 origin in link 0,
// [3,4] joint-2 origin in link 1, [5..10] COM of links 0..2 in their frames, [11..13] masses,
// [14] Izz_0 + Izz_1 + Izz_2, [15] Izz_1 + Izz_2, [16] Izz_2, [17] m_0 |c_0|^2.
struct Planar3 {
  double P0x, P0y, p2x, p2y, c0x, c0y, c1x, c1y, c2x, c2y, m0, m1, m2, I012, I12, I2, m0cc;
  __device__ __forceinline__ explicit Planar3(const double* pl)
      : P0x(pl[1]), P0y(pl[2]), p2x(pl[3]), p2y(pl[4]), c0x(pl[5]), c0y(pl[6]), c1x(pl[7]), c1y(pl[8]),
        c2x(pl[9]), c2y(pl[10]), m0(pl[11]), m1(pl[12]), m2(pl[13]), I012(pl[14]), I12(pl[15]), I2(pl[16]),
        m0cc(pl[17]) {}
};

// sin and cos of a joint angle: one Cody-Waite reduction by pi/2 (three-part constant, exact
// products in the FMAs) and the FreeBSD k_sin / k_cos minimax kernels on |r| <= pi/4 (within an
// ulp or so), the quadrant by selects — a third of the f64 instructions of the library sincos,
// whose Payne-Hanek branch also cost the one-slot-per-wave rollout its registers. The reduction
// stays accurate while x * 2/pi rounds to the nearest integer, |x| < 2^52 (a joint angle beyond
// that has no meaningful phase); NaN / inf give NaN. Deterministic: every kernel that calls it for
// the same x gets the same bits.
__device__ __forceinline__ void joint_sincos(double x, double* sp, double* cp) {
  const double n = rint(x * 0.63661977236758134308);
  double r = fma(-n, 1.5707963267948966, x);
  r = fma(-n, 6.123233995736766e-17, r);
  r = fma(-n, -1.4973849048591698e-33, r);
  const double z = r * r, w = z * z;
  // k_sin
  const double rs = fma(z, fma(z, 2.75573137070700676789e-06, -1.98412698298579493134e-04), 8.33333333332248946124e-03) +
                    z * w * fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);
  const double sr = fma(z * r, fma(z, rs, -1.66666666666666324348e-01), r);
  // k_cos
  const double rc = z * fma(z, fma(z, 2.48015872894767294178e-05, -1.38888888888741095749e-03), 4.16666666666666019037e-02) +
                    w * w * fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09), -2.75573143513906633035e-07);
  const double hz = 0.5 * z, wc = 1.0 - hz;
  const double cr = wc + (((1.0 - wc) - hz) + z * rc);
  const int q = (int)(n - 4.0 * floor(n * 0.25));  // n mod 4, exact for |n| < 2^53
  const double ss = (q & 1) ? cr : sr, cc = (q & 1) ? sr : cr;
  *sp = (q & 2) ? -ss : ss;
  *cp = ((q + 1) & 2) ? -cc : cc;
}

// M(q), h(q, v) of the planar 3R chain in closed form, returned as the adjugate of M (A, symmetric)
// with r = 1 / det M, so M^-1 = r A and qdd = r A (a - h); sin / cos of q1, q2 given (joint_sincos).
struct Planar3Terms {
  double A00, A01, A02, A11, A12, A22, r, h0, h1, h2;
};
__device__ __forceinline__ Planar3Terms planar3_terms(const Planar3& k, const double* s, double s1, double c1,
                                                      double s2, double c2) {
  const double c12 = fma(c1, c2, -(s1 * s2)), s12 = fma(s1, c2, c1 * s2);
  // link-fixed vectors in link 0's frame: joint 1 -> joint 2 (P1), joint i -> COM i (Ci)
  const double P1x = fma(k.p2x, c1, -(k.p2y * s1)), P1y = fma(k.p2x, s1, k.p2y * c1);
  const double C1x = fma(k.c1x, c1, -(k.c1y * s1)), C1y = fma(k.c1x, s1, k.c1y * c1);
  const double C2x = fma(k.c2x, c12, -(k.c2y * s12)), C2y = fma(k.c2x, s12, k.c2y * c12);
  const double r01x = k.P0x + C1x, r01y = k.P0y + C1y;  // joint 0 -> COM 1
  const double r12x = P1x + C2x, r12y = P1y + C2y;      // joint 1 -> COM 2
  const double r02x = k.P0x + r12x, r02y = k.P0y + r12y;  // joint 0 -> COM 2
  auto dot2 = [](double ax, double ay, double bx, double by) { return fma(ax, bx, ay * by); };
  auto crs2 = [](double ax, double ay, double bx, double by) { return fma(ax, by, -(ay * bx)); };
  const double M00 = fma(k.m2, dot2(r02x, r02y, r02x, r02y), fma(k.m1, dot2(r01x, r01y, r01x, r01y), k.m0cc)) + k.I012;
  const double M01 = fma(k.m2, dot2(r02x, r02y, r12x, r12y), k.m1 * dot2(r01x, r01y, C1x, C1y)) + k.I12;
  const double M02 = fma(k.m2, dot2(r02x, r02y, C2x, C2y), k.I2);
  const double M11 = fma(k.m2, dot2(r12x, r12y, r12x, r12y), k.m1 * dot2(C1x, C1y, C1x, C1y)) + k.I12;
  const double M12 = fma(k.m2, dot2(r12x, r12y, C2x, C2y), k.I2);
  const double M22 = fma(k.m2, dot2(C2x, C2y, C2x, C2y), k.I2);
  // COM accelerations at qdd = 0 (negated): w_j^2 times the link-fixed vectors on the way
  const double w0 = s[3], w1 = w0 + s[4], w2 = w1 + s[5];
  const double q0 = w0 * w0, q1 = w1 * w1, q2 = w2 * w2;
  const double n0x = q0 * k.c0x, n0y = q0 * k.c0y;
  const double b0x = q0 * k.P0x, b0y = q0 * k.P0y;
  const double n1x = fma(q1, C1x, b0x), n1y = fma(q1, C1y, b0y);
  const double n2x = fma(q2, C2x, fma(q1, P1x, b0x)), n2y = fma(q2, C2y, fma(q1, P1y, b0y));
  Planar3Terms T;
  T.h2 = -(k.m2 * crs2(C2x, C2y, n2x, n2y));
  T.h1 = -fma(k.m1, crs2(C1x, C1y, n1x, n1y), k.m2 * crs2(r12x, r12y, n2x, n2y));
  T.h0 = -fma(k.m0, crs2(k.c0x, k.c0y, n0x, n0y), fma(k.m1, crs2(r01x, r01y, n1x, n1y), k.m2 * crs2(r02x, r02y, n2x, n2y)));
  T.A00 = fma(M11, M22, -(M12 * M12));
  T.A01 = fma(M02, M12, -(M01 * M22));
  T.A02 = fma(M01, M12, -(M02 * M11));
  T.A11 = fma(M00, M22, -(M02 * M02));
  T.A12 = fma(M01, M02, -(M00 * M12));
  T.A22 = fma(M00, M11, -(M01 * M01));
  T.r = 1.0 / fma(M00, T.A00, fma(M01, T.A01, M02 * T.A02));
  return T;
}
// qdd = M^-1 (a - h)
__device__ __forceinline__ void planar3_qdd(const Planar3Terms& T, const double* a, double* dv) {
  const double e0 = a[0] - T.h0, e1 = a[1] - T.h1, e2 = a[2] - T.h2;
  dv[0] = fma(T.A00, e0, fma(T.A01, e1, T.A02 * e2)) * T.r;
  dv[1] = fma(T.A01, e0, fma(T.A11, e1, T.A12 * e2)) * T.r;
  dv[2] = fma(T.A02, e0, fma(T.A12, e1, T.A22 * e2)) * T.r;
}

// Explicit Euler step of the planar 3R chain (float64 state and action): qdd = M^-1 (a - h), then
// env_simulate's update q' = q + v dt, v' = v + qdd dt, t' = t + dt — the same operations as the
// chain's generic step (chain_step), so every kernel that steps the manipulator (the rollouts,
// cacto_env_step) gives the same bits. (s1, c1, s2, c2) = joint_sincos of q1, q2.
__device__ __forceinline__ void planar3_step_sc(const Planar3& k, double dt, const double* s, const double* a,
                                                double s1, double c1, double s2, double c2, double* out) {
  const Planar3Terms T = planar3_terms(k, s, s1, c1, s2, c2);
  double dv[3];
  planar3_qdd(T, a, dv);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double v = s[3 + i];
    out[i] = s[i] + v * dt;
    out[3 + i] = v + dv[i] * dt;
  }
  out[6] = s[6] + dt;
}
__device__ __forceinline__ void planar3_step(const Planar3& k, double dt, const double* s, const double* a,
                                             double* out) {
  double s1, c1, s2, c2;
  joint_sincos(s[1], &s1, &c1);
  joint_sincos(s[2], &s2, &c2);
  planar3_step_sc(k, dt, s, a, s1, c1, s2, c2, out);
}

// ------------------------------------------------------------------ small 3-vector algebra
struct V3 {
  double x, y, z;
};
__device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
struct M3 {
  double m[9];  // row-major
};
__device__ __forceinline__ V3 mul(const M3& R, V3 v) {
  return v3(R.m[0] * v.x + R.m[1] * v.y + R.m[2] * v.z, R.m[3] * v.x + R.m[4] * v.y + R.m[5] * v.z,
            R.m[6] * v.x + R.m[7] * v.y + R.m[8] * v.z);
}
__device__ __forceinline__ V3 mulT(const M3& R, V3 v) {
  return v3(R.m[0] * v.x + R.m[3] * v.y + R.m[6] * v.z, R.m[1] * v.x + R.m[4] * v.y + R.m[7] * v.z,
            R.m[2] * v.x + R.m[5] * v.y + R.m[8] * v.z);
}
__device__ __forceinline__ M3 mul(const M3& A, const M3& B) {
  M3 C;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C.m[3 * i + j] = A.m[3 * i] * B.m[j] + A.m[3 * i + 1] * B.m[3 + j] + A.m[3 * i + 2] * B.m[6 + j];
  return C;
}

// Symmetric 3x3 stored xx, xy, xz, yy, yz, zz
struct S3 {
  double xx, xy, xz, yy, yz, zz;
};
__device__ __forceinline__ V3 mul(const S3& I, V3 w) {
  return v3(I.xx * w.x + I.xy * w.y + I.xz * w.z, I.xy * w.x + I.yy * w.y + I.yz * w.z,
            I.xz * w.x + I.yz * w.y + I.zz * w.z);
}

// Spatial motion / force, Pinocchio ordering (linear, angular)
struct SV {
  V3 l, a;
};

// Rigid-body inertia about the body origin: mass, first moment h = m*c, rotational inertia Io
// about the origin (= Ic + m(|c|^2 1 - c c^T)). Linear under summation.
struct Inertia {
  double m;
  V3 h;
  S3 Io;
};
__device__ __forceinline__ SV inertia_mul(const Inertia& I, const SV& v) {
  // f = m v - h x w ; n = Io w + h x v
  SV f;
  f.l = I.m * v.l - cross(I.h, v.a);
  f.a = mul(I.Io, v.a) + cross(I.h, v.l);
  return f;
}
// SE3 (R, p): placement of child frame in parent frame
struct SE3 {
  M3 R;
  V3 p;
};
__device__ __forceinline__ SV act_motion_inv(const SE3& M, const SV& v) {  // parent -> child
  SV o;
  o.a = mulT(M.R, v.a);
  o.l = mulT(M.R, v.l - cross(M.p, v.a));
  return o;
}
__device__ __forceinline__ SV act_force(const SE3& M, const SV& f) {  // child -> parent
  SV o;
  o.l = mul(M.R, f.l);
  o.a = mul(M.R, f.a) + cross(M.p, o.l);
  return o;
}
__device__ __forceinline__ SV cross_motion(const SV& v, const SV& m) {
  SV o;
  o.l = cross(v.a, m.l) + cross(v.l, m.a);
  o.a = cross(v.a, m.a);
  return o;
}
__device__ __forceinline__ SV cross_force(const SV& v, const SV& f) {
  SV o;
  o.l = cross(v.a, f.l);
  o.a = cross(v.a, f.a) + cross(v.l, f.l);
  return o;
}
// Express a child-frame inertia in the parent frame.
__device__ __forceinline__ Inertia act_inertia(const SE3& M, const Inertia& I) {
  Inertia o;
  o.m = I.m;
  V3 hr = mul(M.R, I.h);
  o.h = hr + I.m * M.p;
  // R Io R^T
  M3 A;
  const double io[9] = {I.Io.xx, I.Io.xy, I.Io.xz, I.Io.xy, I.Io.yy, I.Io.yz, I.Io.xz, I.Io.yz, I.Io.zz};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      A.m[3 * i + j] = io[3 * i] * M.R.m[3 * j] + io[3 * i + 1] * M.R.m[3 * j + 1] + io[3 * i + 2] * M.R.m[3 * j + 2];
  M3 RIR = mul(M.R, A);
  const V3 p = M.p;
  const double pp = dot(p, p), ph = 2.0 * dot(p, hr);
  o.Io.xx = RIR.m[0] + I.m * (pp - p.x * p.x) + ph - 2.0 * p.x * hr.x;
  o.Io.yy = RIR.m[4] + I.m * (pp - p.y * p.y) + ph - 2.0 * p.y * hr.y;
  o.Io.zz = RIR.m[8] + I.m * (pp - p.z * p.z) + ph - 2.0 * p.z * hr.z;
  o.Io.xy = RIR.m[1] - I.m * p.x * p.y - p.x * hr.y - hr.x * p.y;
  o.Io.xz = RIR.m[2] - I.m * p.x * p.z - p.x * hr.z - hr.x * p.z;
  o.Io.yz = RIR.m[5] - I.m * p.y * p.z - p.y * hr.z - hr.y * p.z;
  return o;
}
__device__ __forceinline__ void add_inertia(Inertia& a, const Inertia& b) {
  a.m += b.m;
  a.h = a.h + b.h;
  a.Io.xx += b.Io.xx; a.Io.xy += b.Io.xy; a.Io.xz += b.Io.xz;
  a.Io.yy += b.Io.yy; a.Io.yz += b.Io.yz; a.Io.zz += b.Io.zz;
}

// ------------------------------------------------------------------ joint table access
struct JointView {
  const double* r;
  __device__ int parent() const { return (int)r[0]; }
  __device__ int kind() const { return (int)r[1]; }
  __device__ V3 axis() const { return v3(r[2], r[3], r[4]); }
  __device__ M3 R0() const {
    M3 R;
#pragma unroll
    for (int k = 0; k < 9; ++k) R.m[k] = r[5 + k];
    return R;
  }
  __device__ V3 p0() const { return v3(r[14], r[15], r[16]); }
  __device__ Inertia inertia() const {
    // stored: mass, com, Ic (about COM) -> origin form
    Inertia I;
    I.m = r[17];
    V3 c = v3(r[18], r[19], r[20]);
    I.h = I.m * c;
    const double cc = dot(c, c);
    I.Io.xx = r[21] + I.m * (cc - c.x * c.x);
    I.Io.xy = r[22] - I.m * c.x * c.y;
    I.Io.xz = r[23] - I.m * c.x * c.z;
    I.Io.yy = r[24] + I.m * (cc - c.y * c.y);
    I.Io.yz = r[25] - I.m * c.y * c.z;
    I.Io.zz = r[26] + I.m * (cc - c.z * c.z);
    return I;
  }
};

// Joint transform; axis-aligned revolute joints use the closed form (Pinocchio JointModelR{X,Y,Z}),
// others Rodrigues (JointModelRevoluteUnaligned).
__device__ inline M3 joint_rotation(V3 ax, double q) {
  double s, c;
  sincos(q, &s, &c);
  M3 R;
  if (ax.x == 1.0 && ax.y == 0.0 && ax.z == 0.0) {
    R = M3{{1, 0, 0, 0, c, -s, 0, s, c}};
  } else if (ax.x == 0.0 && ax.y == 1.0 && ax.z == 0.0) {
    R = M3{{c, 0, s, 0, 1, 0, -s, 0, c}};
  } else if (ax.x == 0.0 && ax.y == 0.0 && ax.z == 1.0) {
    R = M3{{c, -s, 0, s, c, 0, 0, 0, 1}};
  } else {
    const double t = 1.0 - c;
    R = M3{{c + t * ax.x * ax.x, t * ax.x * ax.y - s * ax.z, t * ax.x * ax.z + s * ax.y,
            t * ax.x * ax.y + s * ax.z, c + t * ax.y * ax.y, t * ax.y * ax.z - s * ax.x,
            t * ax.x * ax.z - s * ax.y, t * ax.y * ax.z + s * ax.x, c + t * ax.z * ax.z}};
  }
  return R;
}

__device__ inline SE3 joint_placement(const JointView& j, double q) {
  SE3 M;
  const M3 R0 = j.R0();
  if (j.kind() == 0) {
    M.R = mul(R0, joint_rotation(j.axis(), q));
    M.p = j.p0();
  } else {
    M.R = R0;
    M.p = j.p0() + mul(R0, q * j.axis());
  }
  return M;
}

__device__ __forceinline__ SV joint_S(const JointView& j) {
  SV S;
  V3 z = v3(0, 0, 0);
  if (j.kind() == 0) {
    S.l = z;
    S.a = j.axis();
  } else {
    S.l = j.axis();
    S.a = z;
  }
  return S;
}
__device__ __forceinline__ double sdot(const SV& S, const SV& f) { return dot(S.l, f.l) + dot(S.a, f.a); }

// M(q) via CRBA and h(q, v) via RNEA (qdd = 0, a_0 = -gravity), Featherstone / Pinocchio, for a
// serial chain of NJ joints (parent(i) = i - 1, validated at cacto_sys_create). NJ is a template
// parameter so every per-joint array lives in registers.
template <int NJ>
__device__ inline void chain_terms(const SysDevice& sd, const double* q, const double* v, double* M, double* h) {
  SE3 X[NJ];
  SV vel[NJ], acc[NJ], f[NJ];
  Inertia Ic[NJ];
  const SV gacc{v3(-sd.p.gravity[0], -sd.p.gravity[1], -sd.p.gravity[2]), v3(0, 0, 0)};
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    JointView j{sd.joints + i * CACTO_JOINT_COLS};
    X[i] = joint_placement(j, q[i]);
    const SV S = joint_S(j);
    const SV vp = i == 0 ? SV{v3(0, 0, 0), v3(0, 0, 0)} : vel[i - 1];
    const SV ap = i == 0 ? gacc : acc[i - 1];
    SV vi = act_motion_inv(X[i], vp);
    const SV Sq{v[i] * S.l, v[i] * S.a};
    vi.l = vi.l + Sq.l;
    vi.a = vi.a + Sq.a;
    SV ai = act_motion_inv(X[i], ap);
    const SV c = cross_motion(vi, Sq);
    ai.l = ai.l + c.l;
    ai.a = ai.a + c.a;
    vel[i] = vi;
    acc[i] = ai;
    Ic[i] = j.inertia();
    const SV Iv = inertia_mul(Ic[i], vi);
    const SV Ia = inertia_mul(Ic[i], ai);
    const SV vf = cross_force(vi, Iv);
    f[i].l = Ia.l + vf.l;
    f[i].a = Ia.a + vf.a;
  }
#pragma unroll
  for (int i = NJ - 1; i >= 0; --i) {
    JointView j{sd.joints + i * CACTO_JOINT_COLS};
    h[i] = sdot(joint_S(j), f[i]);
    if (i > 0) {
      const SV fp = act_force(X[i], f[i]);
      f[i - 1].l = f[i - 1].l + fp.l;
      f[i - 1].a = f[i - 1].a + fp.a;
      add_inertia(Ic[i - 1], act_inertia(X[i], Ic[i]));
    }
  }
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    JointView j{sd.joints + i * CACTO_JOINT_COLS};
    SV F = inertia_mul(Ic[i], joint_S(j));
    M[i * NJ + i] = sdot(joint_S(j), F);
#pragma unroll
    for (int k = i; k > 0; --k) {
      F = act_force(X[k], F);
      JointView jp{sd.joints + (k - 1) * CACTO_JOINT_COLS};
      const double mij = sdot(joint_S(jp), F);
      M[i * NJ + (k - 1)] = mij;
      M[(k - 1) * NJ + i] = mij;
    }
  }
}

// In-place Cholesky of SPD M (NJ x NJ); returns false if not positive definite.
// The two halves of chain_terms with fewer live values (the rollout runs them on different waves):
// nle(q, v) by RNEA, M(q) by CRBA. Same operation order as chain_terms, so results are identical.
template <int NJ>
__device__ inline void chain_nle(const SysDevice& sd, const double* q, const double* v, double* h) {
  SE3 X[NJ];
  SV f[NJ];
  const SV gacc{v3(-sd.p.gravity[0], -sd.p.gravity[1], -sd.p.gravity[2]), v3(0, 0, 0)};
  SV vp{v3(0, 0, 0), v3(0, 0, 0)}, ap = gacc;
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    JointView j{sd.joints + i * CACTO_JOINT_COLS};
    X[i] = joint_placement(j, q[i]);
    const SV S = joint_S(j);
    SV vi = act_motion_inv(X[i], vp);
    const SV Sq{v[i] * S.l, v[i] * S.a};
    vi.l = vi.l + Sq.l;
    vi.a = vi.a + Sq.a;
    SV ai = act_motion_inv(X[i], ap);
    const SV c = cross_motion(vi, Sq);
    ai.l = ai.l + c.l;
    ai.a = ai.a + c.a;
    const Inertia I = j.inertia();
    const SV Iv = inertia_mul(I, vi);
    const SV Ia = inertia_mul(I, ai);
    const SV vf = cross_force(vi, Iv);
    f[i].l = Ia.l + vf.l;
    f[i].a = Ia.a + vf.a;
    vp = vi;
    ap = ai;
  }
#pragma unroll
  for (int i = NJ - 1; i >= 0; --i) {
    JointView j{sd.joints + i * CACTO_JOINT_COLS};
    h[i] = sdot(joint_S(j), f[i]);
    if (i > 0) {
      const SV fp = act_force(X[i], f[i]);
      f[i - 1].l = f[i - 1].l + fp.l;
      f[i - 1].a = f[i - 1].a + fp.a;
    }
  }
}

template <int NJ>
__device__ inline void chain_mass(const SysDevice& sd, const double* q, double* M) {
  SE3 X[NJ];
  Inertia Ic[NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    JointView j{sd.joints + i * CACTO_JOINT_COLS};
    X[i] = joint_placement(j, q[i]);
    Ic[i] = j.inertia();
  }
#pragma unroll
  for (int i = NJ - 1; i > 0; --i) add_inertia(Ic[i - 1], act_inertia(X[i], Ic[i]));
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    JointView j{sd.joints + i * CACTO_JOINT_COLS};
    SV F = inertia_mul(Ic[i], joint_S(j));
    M[i * NJ + i] = sdot(joint_S(j), F);
#pragma unroll
    for (int k = i; k > 0; --k) {
      F = act_force(X[k], F);
      JointView jp{sd.joints + (k - 1) * CACTO_JOINT_COLS};
      const double mij = sdot(joint_S(jp), F);
      M[i * NJ + (k - 1)] = mij;
      M[(k - 1) * NJ + i] = mij;
    }
  }
}

// The factor keeps the reciprocal of its diagonal (1/L_jj on the diagonal): one float64
// division per column instead of one per off-diagonal entry and per solve step (each division is a
// long dependent instruction sequence on the rollout's per-step critical path). Versus dividing,
// results move by at most an ulp per operation; for unit diagonals (prismatic chains such as the
// double integrator) they are identical.
template <int NJ>
__device__ inline bool cholesky(double* L) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    double d = L[j * NJ + j];
#pragma unroll
    for (int k = 0; k < j; ++k) d -= L[j * NJ + k] * L[j * NJ + k];
    ok = ok && d > 0.0;
    const double r = 1.0 / sqrt(d);
    L[j * NJ + j] = r;
#pragma unroll
    for (int i = j + 1; i < NJ; ++i) {
      double s = L[i * NJ + j];
#pragma unroll
      for (int k = 0; k < j; ++k) s -= L[i * NJ + k] * L[j * NJ + k];
      L[i * NJ + j] = s * r;
    }
  }
  return ok;
}
template <int NJ>
__device__ inline void chol_solve(const double* L, double* x) {
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    double s = x[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= L[i * NJ + k] * x[k];
    x[i] = s * L[i * NJ + i];
  }
#pragma unroll
  for (int i = NJ - 1; i >= 0; --i) {
    double s = x[i];
#pragma unroll
    for (int k = i + 1; k < NJ; ++k) s -= L[k * NJ + i] * x[k];
    x[i] = s * L[i * NJ + i];
  }
}

// EE frame translation (forward kinematics to the EE parent joint, then the fixed placement).
// s' from (s, a) given M (Cholesky-factored in place) and h: explicit Euler, float64 path.
template <int NJ>
__device__ inline bool chain_step(const SysDevice& sd, const double* s, const double* a, double* M, const double* h,
                                  double* out) {
  const double dt = sd.p.dt;
  double dv[NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) dv[i] = a[i] - h[i];
  const bool ok = cholesky<NJ>(M);
  chol_solve<NJ>(M, dv);
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const double v = s[NJ + i];
    out[i] = s[i] + v * dt;
    out[NJ + i] = v + dv[i] * dt;
  }
  out[2 * NJ] = s[2 * NJ] + dt;
  return ok;
}

template <int NJ>
__device__ inline V3 chain_ee(const SysDevice& sd, const double* q) {
  M3 oR;
  V3 op, ee = v3(0, 0, 0);
  const int e = sd.p.ee_parent;
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    JointView j{sd.joints + i * CACTO_JOINT_COLS};
    const SE3 X = joint_placement(j, q[i]);
    if (i == 0) {
      oR = X.R;
      op = X.p;
    } else {
      op = mul(oR, X.p) + op;
      oR = mul(oR, X.R);
    }
    if (i == e) ee = mul(oR, v3(sd.p.ee_p[0], sd.p.ee_p[1], sd.p.ee_p[2])) + op;
  }
  return ee;
}

// ------------------------------------------------------------------ environment functions

// Env.simulate. `f32in`: state/action originate from float32 tensors (compute_actor_grad path),
// which makes `v*dt` a float32 product and `self.v += dv*dt` round to float32 (numpy in-place on a
// float32 view, robot_utils.py:403-405); otherwise all float64 (rollouts). environment.py:80-91.
// NJ = 0: single integrator (environment.py:235-243); NJ > 0: Pinocchio chain with NJ joints.
// NJ = -1: Car (environment.py:437-448), NJ = -2: CarPark (environment.py:584-595).
template <int NJ>
__device__ inline bool env_simulate(const SysDevice& sd, const double* s, const double* a, bool f32in, double* out) {
  const double dt = sd.p.dt;
  if constexpr (NJ == 0) {
    out[0] = s[0] + dt * a[0];
    out[1] = s[1] + dt * a[1];
    out[2] = s[2] + dt;
    return true;
  } else if constexpr (NJ == -1) {
    // x' = x + dt*v*tf.cos(th) + dt**2*a*tf.cos(th)/2 (and y with sin). With float32 inputs
    // (simulate_batch in compute_actor_grad) numpy-1.x makes dt*v a float64 scalar, TF casts it to
    // float32 against the float32 tf.cos result, so x', y' are float32 arithmetic; the other
    // components stay float64 scalars.
    const double dt2 = dt * dt;
    if (f32in) {
      const float th = (float)s[2];
      const float c = cosf(th), sn = sinf(th);
      const float x1 = __fadd_rn((float)s[0], __fmul_rn((float)(dt * s[3]), c));
      out[0] = (double)__fadd_rn(x1, __fdiv_rn(__fmul_rn((float)(dt2 * s[4]), c), 2.0f));
      const float y1 = __fadd_rn((float)s[1], __fmul_rn((float)(dt * s[3]), sn));
      out[1] = (double)__fadd_rn(y1, __fdiv_rn(__fmul_rn((float)(dt2 * s[4]), sn), 2.0f));
    } else {
      const double c = cos(s[2]), sn = sin(s[2]);
      out[0] = (s[0] + dt * s[3] * c) + dt2 * s[4] * c / 2.0;
      out[1] = (s[1] + dt * s[3] * sn) + dt2 * s[4] * sn / 2.0;
    }
    out[2] = s[2] + dt * a[0];
    out[3] = s[3] + dt * s[4];
    out[4] = s[4] + dt * a[1];
    out[5] = s[5] + dt;
    return true;
  } else if constexpr (NJ == -2) {
    // math.cos/sin/tan: float64 for any input dtype.
    const double L = sd.p.L_delta, tau = sd.p.tau_delta;
    out[0] = s[0] + dt * s[3] * cos(s[2]);
    out[1] = s[1] + dt * s[3] * sin(s[2]);
    out[2] = s[2] + dt * s[3] * tan(s[4]) / L;
    out[3] = s[3] + dt * a[0];
    out[4] = s[4] + dt * a[1] / tau;
    out[5] = s[5] + dt;
    return true;
  } else {
    double dv[NJ];
    bool ok = true;
    bool planar = false;
    if constexpr (NJ == 3) {
      if (sd.pl[0] != 0.0) {  // the planar 3R chain: closed form (planar3_terms)
        double s1, c1, s2, c2;
        joint_sincos(s[1], &s1, &c1);
        joint_sincos(s[2], &s2, &c2);
        planar3_qdd(planar3_terms(Planar3(sd.pl), s, s1, c1, s2, c2), a, dv);
        planar = true;
      }
    }
    if (!planar) {
      double M[NJ * NJ], h[NJ];
      chain_terms<NJ>(sd, s, s + NJ, M, h);
#pragma unroll
      for (int i = 0; i < NJ; ++i) dv[i] = a[i] - h[i];
      ok = cholesky<NJ>(M);
      chol_solve<NJ>(M, dv);
    }
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const double v = s[NJ + i];
      if (f32in) {
        const float vdt = __fmul_rn((float)v, (float)dt);
        out[i] = s[i] + (double)vdt;
        out[NJ + i] = (double)(float)(v + dv[i] * dt);
      } else {
        out[i] = s[i] + v * dt;
        out[NJ + i] = v + dv[i] * dt;
      }
    }
    out[2 * NJ] = s[2 * NJ] + dt;
    return ok;
  }
}

// Prismatic-only chains (const_dyn): M and nle do not depend on (q, v) (no rotation; see
// DESIGN.md), so the rollout factors M once per episode and reuses it every step.
template <int NJ>
struct ConstDyn {
  double L[NJ > 0 ? NJ * NJ : 1];
  double h[NJ > 0 ? NJ : 1];
};
template <int NJ>
__device__ inline void const_dyn_init(const SysDevice& sd, const double* s, ConstDyn<NJ>& cd) {
  if constexpr (NJ > 0) {
    chain_terms<NJ>(sd, s, s + NJ, cd.L, cd.h);
    cholesky<NJ>(cd.L);
  }
}
template <int NJ>
__device__ inline void env_simulate_const(const SysDevice& sd, const ConstDyn<NJ>& cd, const double* s, const double* a,
                                          double* out) {
  if constexpr (NJ > 0) {
    const double dt = sd.p.dt;
    double dv[NJ];
#pragma unroll
    for (int i = 0; i < NJ; ++i) dv[i] = a[i] - cd.h[i];
    chol_solve<NJ>(cd.L, dv);
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const double v = s[NJ + i];
      out[i] = s[i] + v * dt;
      out[NJ + i] = v + dv[i] * dt;
    }
    out[2 * NJ] = s[2 * NJ] + dt;
  }
}

// env_simulate_derivative for a prismatic-only chain from the factor / Fu tabled in SysDevice:
// the same operations on the same values as the per-sample path (chain_terms -> cholesky ->
// chol_solve), minus the recomputation of the q-independent M and h.
template <int NJ>
__device__ inline bool env_simulate_derivative_const(const SysDevice& sd, const double* s, const double* a, bool f32in,
                                                     double* out, double* Fu) {
  if constexpr (NJ > 0) {
    constexpr int NS = 2 * NJ + 1, NA = NJ;
    const double dt = sd.p.dt;
    double L[NJ * NJ], dv[NJ];
#pragma unroll
    for (int k = 0; k < NJ * NJ; ++k) L[k] = sd.cd_L[k];
#pragma unroll
    for (int i = 0; i < NJ; ++i) dv[i] = a[i] - sd.cd_h[i];
    chol_solve<NJ>(L, dv);
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const double v = s[NJ + i];
      if (f32in) {
        const float vdt = __fmul_rn((float)v, (float)dt);
        out[i] = s[i] + (double)vdt;
        out[NJ + i] = (double)(float)(v + dv[i] * dt);
      } else {
        out[i] = s[i] + v * dt;
        out[NJ + i] = v + dv[i] * dt;
      }
    }
    out[2 * NJ] = s[2 * NJ] + dt;
#pragma unroll
    for (int k = 0; k < NS * NA; ++k) Fu[k] = sd.cd_Fu[k];
  }
  return true;
}

// Env.derivative (environment.py:93-109 / SI :209-219): Fu[ns, na] row-major, rows scaled by
// 1/state_norm when NORMALIZE_INPUTS.
// Car :408-418 (Fu[2,0] = Fu[4,1] = dt), CarPark :555-565 (Fu[3,0] = dt, Fu[4,1] = dt/tau_delta).
template <int NJ>
__device__ inline void env_derivative(const SysDevice& sd, const double* s, double* Fu);

// env_simulate_derivative of the planar 3R chain: the step as env_simulate's, Fu = dt M^-1 (rows
// 3-5) from the same adjugate, row-normalised.
__device__ inline bool env_simulate_derivative_planar3(const SysDevice& sd, const double* s, const double* a,
                                                       bool f32in, double* out, double* Fu) {
  const double dt = sd.p.dt;
  double s1, c1, s2, c2, dv[3];
  joint_sincos(s[1], &s1, &c1);
  joint_sincos(s[2], &s2, &c2);
  const Planar3Terms T = planar3_terms(Planar3(sd.pl), s, s1, c1, s2, c2);
  planar3_qdd(T, a, dv);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double v = s[3 + i];
    if (f32in) {
      const float vdt = __fmul_rn((float)v, (float)dt);
      out[i] = s[i] + (double)vdt;
      out[3 + i] = (double)(float)(v + dv[i] * dt);
    } else {
      out[i] = s[i] + v * dt;
      out[3 + i] = v + dv[i] * dt;
    }
  }
  out[6] = s[6] + dt;
  const double Mi[9] = {T.A00, T.A01, T.A02, T.A01, T.A11, T.A12, T.A02, T.A12, T.A22};
#pragma unroll
  for (int k = 0; k < 7 * 3; ++k) Fu[k] = 0.0;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double v = Mi[3 * i + c] * T.r * dt;
      if (sd.p.normalize) v *= sd.inv_norm[3 + i];
      Fu[(3 + i) * 3 + c] = v;
    }
  return true;
}

// env_simulate(s, a, f32in) and env_derivative(s) together. For a chain, M(q) is factored once and
// serves both the step and the columns of M^-1 (env_derivative would rebuild it with v = 0; M does
// not depend on v, so the factor is the same bits).
template <int NJ>
__device__ inline bool env_simulate_derivative(const SysDevice& sd, const double* s, const double* a, bool f32in,
                                               double* out, double* Fu) {
  if constexpr (NJ > 0) {
    const cacto_sys_params& p = sd.p;
    constexpr int NS = 2 * NJ + 1, NA = NJ;
    const double dt = p.dt;
    if constexpr (NJ == 3)
      if (sd.pl[0] != 0.0) return env_simulate_derivative_planar3(sd, s, a, f32in, out, Fu);
    double M[NJ * NJ], h[NJ], dv[NJ];
    chain_terms<NJ>(sd, s, s + NJ, M, h);
#pragma unroll
    for (int i = 0; i < NJ; ++i) dv[i] = a[i] - h[i];
    const bool ok = cholesky<NJ>(M);
    chol_solve<NJ>(M, dv);
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const double v = s[NJ + i];
      if (f32in) {
        const float vdt = __fmul_rn((float)v, (float)dt);
        out[i] = s[i] + (double)vdt;
        out[NJ + i] = (double)(float)(v + dv[i] * dt);
      } else {
        out[i] = s[i] + v * dt;
        out[NJ + i] = v + dv[i] * dt;
      }
    }
    out[2 * NJ] = s[2 * NJ] + dt;
#pragma unroll
    for (int k = 0; k < NS * NA; ++k) Fu[k] = 0.0;
#pragma unroll
    for (int c = 0; c < NJ; ++c) {  // column c of Minv
      double x[NJ];
#pragma unroll
      for (int i = 0; i < NJ; ++i) x[i] = (i == c) ? 1.0 : 0.0;
      chol_solve<NJ>(M, x);
#pragma unroll
      for (int i = 0; i < NJ; ++i) Fu[(NJ + i) * NA + c] = x[i] * dt;
    }
    if (p.normalize) {
#pragma unroll
      for (int r = 0; r < NS - 1; ++r) {
        const double inv = sd.inv_norm[r];
#pragma unroll
        for (int c = 0; c < NA; ++c) Fu[r * NA + c] *= inv;
      }
    }
    return ok;
  } else {
    const bool ok = env_simulate<NJ>(sd, s, a, f32in, out);
    env_derivative<NJ>(sd, s, Fu);
    return ok;
  }
}

template <int NJ>
__device__ inline void env_derivative(const SysDevice& sd, const double* s, double* Fu) {
  const cacto_sys_params& p = sd.p;
  constexpr int NS = NJ == 0 ? 3 : NJ < 0 ? 6 : 2 * NJ + 1;
  constexpr int NA = NJ > 0 ? NJ : 2;
#pragma unroll
  for (int k = 0; k < NS * NA; ++k) Fu[k] = 0.0;
  if constexpr (NJ == 0) {
    Fu[0 * NA + 0] = p.dt;
    Fu[1 * NA + 1] = p.dt;
  } else if constexpr (NJ == -1) {
    Fu[2 * NA + 0] = p.dt;
    Fu[4 * NA + 1] = p.dt;
  } else if constexpr (NJ == -2) {
    Fu[3 * NA + 0] = p.dt;
    Fu[4 * NA + 1] = p.dt / p.tau_delta;
  } else {
    double M[NJ * NJ], h[NJ], zero[NJ];
#pragma unroll
    for (int i = 0; i < NJ; ++i) zero[i] = 0.0;
    chain_terms<NJ>(sd, s, zero, M, h);
    cholesky<NJ>(M);
#pragma unroll
    for (int c = 0; c < NJ; ++c) {  // column c of Minv
      double x[NJ];
#pragma unroll
      for (int i = 0; i < NJ; ++i) x[i] = (i == c) ? 1.0 : 0.0;
      chol_solve<NJ>(M, x);
#pragma unroll
      for (int i = 0; i < NJ; ++i) Fu[(NJ + i) * NA + c] = x[i] * p.dt;
    }
  }
  if (p.normalize) {
#pragma unroll
    for (int r = 0; r < NS - 1; ++r) {
      const double inv = sd.inv_norm[r];
#pragma unroll
      for (int c = 0; c < NA; ++c) Fu[r * NA + c] *= inv;
    }
  }
}

template <int NJ>
__device__ inline V3 env_ee(const SysDevice& sd, const double* s) {
  if constexpr (NJ == 0 || NJ == -1) {
    return v3(s[0], s[1], 0.0);  // SI / car: environment.py:245-250, :450-455
  } else if constexpr (NJ == -2) {
    // CarPark :597-602: p = s[:2] + [[c, -s], [s, c]] . [L/2, 0]
    const double c = cos(s[2]), sn = sin(s[2]), h = sd.p.L_delta / 2.0;
    return v3(s[0] + (c * h + -sn * 0.0), s[1] + (sn * h + c * 0.0), 0.0);
  } else {
    return chain_ee<NJ>(sd, s);
  }
}

__device__ __forceinline__ double ell_cost(const cacto_sys_params& p, double x, double y, double xc,
                                           double yc, double A, double B) {
  const double e = ((x - xc) * (x - xc)) / ((A / 2) * (A / 2)) + ((y - yc) * (y - yc)) / ((B / 2) * (B / 2));
  return log(exp(p.alpha * -(e - 1.0)) + 1.0) / p.alpha;
}

// One term of bound_control_cost: a^2 + w_b*(a/u_max)^10; x^10 by squaring (within a few ulp of pow).
__device__ __forceinline__ double bound_term(const cacto_sys_params& p, double a, int i) {
  const double x = a / p.u_max[i];
  const double x2 = x * x, x4 = x2 * x2, x8 = x4 * x4;
  return a * a + p.w_b * (x8 * x2);
}
// bound_control_cost (environment.py:158-163), float64: u = 0; u += term_i in action order
template <int NA>
__device__ inline double bound_control_cost(const cacto_sys_params& p, const double* a) {
  double u = 0.0;
#pragma unroll
  for (int i = 0; i < NA; ++i) u += bound_term(p, a[i], i);
  return u;
}

// Env.reward (float64). `f32state`: the state came from a float32 tensor (affects the float32
// numpy dot of the manipulator velocity term). a may be nullptr (reward(w, s) with action=None).
// Reward pieces that the rollout kernel evaluates on different waves (same formulas as env_reward).
__device__ __forceinline__ double peak_cost(const cacto_sys_params& p, double x, double y) {
  const double dx = x - p.target[0], dy = y - p.target[1];
  const double s01 = sqrt(0.1);
  double pk = sqrt(dx * dx + 0.1);
  pk = pk - s01;
  pk = pk - 0.1;
  pk = pk + sqrt(dy * dy + 0.1);
  pk = pk - s01;
  pk = pk - 0.1;
  return log(exp(p.alpha2 * -pk) + 1.0) / p.alpha2;
}
// r = scale*(-w0*dist + w1*peak [- w2*vel] - w3*ell1 - w4*ell2 - w5*ell3 - w6*u_cost + offset),
// evaluated left to right as the reference's Python expression.
__device__ __forceinline__ double combine_reward(const cacto_sys_params& p, const double* w, double x, double y,
                                                 double peak, double vel, bool has_vel, double ell1, double ell2,
                                                 double ell3, double u_cost) {
  const double dx = x - p.target[0], dy = y - p.target[1];
  const double dist = dx * dx + dy * dy;
  double r = -w[0] * dist + w[1] * peak;
  if (has_vel) r = r - w[2] * vel;
  r = r - w[3] * ell1 - w[4] * ell2 - w[5] * ell3 - w[6] * u_cost + p.offset;
  return p.scale * r;
}

// CarPark obs_cost_fun (environment.py:604-613) for one check point, in the Python expression's
// left-to-right order (fv = 1, k = k_db).
__device__ inline double box_cost(double x, double y, double xs, double ys, double Wx, double Wy, double k) {
  const double k2 = k * k;
  const double ay = (y - ys) + Wy / 2, by = (y - ys) - Wy / 2;
  const double ax = (x - xs) + Wx / 2, bx = (x - xs) - Wx / 2;
  const double t1 = 4.0 + 4.0 * (ay * ay) * k2, t2 = 4.0 + 4.0 * (by * by) * k2;
  const double t3 = 4.0 + 4.0 * (ax * ax) * k2, t4 = 4.0 + 4.0 * (bx * bx) * k2;
  // term**(-1/2) as 1/sqrt(term) (<= 1 ulp; numpy's own SIMD pow is not correctly rounded either)
  const double q1 = sqrt(t1), q2 = sqrt(t2), q3 = sqrt(t3), q4 = sqrt(t4);
  double r = 1.0 / q1;
  r = r * (-q2 / 2.0 + by * k);
  r = r * (1.0 / q3);
  r = r * (1.0 / q2);
  r = r * (q1 / 2.0 + ay * k);
  r = r * (1.0 / q4);
  r = r * (q3 / 2.0 + ax * k);
  r = r * (-q4 / 2.0 + bx * k);
  return r;
}

// numpy's pairwise float64 sum of n <= 15 contiguous values (8 partial sums, then the tail).
__device__ inline double np_sum_small(const double* v, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += v[i];
    return r;
  }
  double r = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
  for (int i = 8; i < n; ++i) r += v[i];
  return r;
}

// CarPark.reward (environment.py:615-641): 10 body check points x 3 smooth boxes.
// Pair pr = ob * n_check + k: check point k (rotated by theta, shifted to the EE) against box ob.
__device__ inline double carpark_pair_cost(const cacto_sys_params& p, double x, double y, double c, double sn, int pr) {
  const int ob = pr / p.n_check, k = pr - ob * p.n_check;
  const double bx = p.check_points[2 * k], by = p.check_points[2 * k + 1];
  const double wx = (c * bx + -sn * by) + x, wy = (sn * bx + c * by) + y;
  const double* o = p.obs;
  return box_cost(wx, wy, o[2 * ob], o[2 * ob + 1], o[6 + 2 * ob], o[7 + 2 * ob], p.k_db);
}
// obs_cost = 0; obs_cost += np.sum(box_1); += np.sum(box_2); += np.sum(box_3)
__device__ inline double carpark_sum(const cacto_sys_params& p, const double* v) {
  double tot = 0.0;
  for (int ob = 0; ob < 3; ++ob) tot = tot + np_sum_small(v + ob * p.n_check, p.n_check);
  return tot;
}
// `f32state`: theta came from a float32 tensor, so np.cos/np.sin run in float32.
__device__ inline double carpark_obs_cost(const cacto_sys_params& p, double x, double y, double th, bool f32state) {
  const double c = f32state ? (double)cosf((float)th) : cos(th);
  const double sn = f32state ? (double)sinf((float)th) : sin(th);
  double v[30];
  for (int pr = 0; pr < 3 * p.n_check; ++pr) v[pr] = carpark_pair_cost(p, x, y, c, sn, pr);
  return carpark_sum(p, v);
}

__device__ __forceinline__ double soft_term(double alpha, double e) { return log(exp(alpha * -(e - 1.0)) + 1.0) / alpha; }

// UR5.reward (environment.py:780-805): 3-D ellipsoids, peak over x, y, z, joint-velocity cost and
// u_cost = a.a (the bound term only enters reward_batch's float32 part).
template <int NJ>
__device__ inline double ur5_reward(const SysDevice& sd, const double* w, const double* s, const double* a,
                                    bool f32state, const V3& e) {
  const cacto_sys_params& p = sd.p;
  const double* o = p.obs;
  double ell[3];
  for (int k = 0; k < 3; ++k) {
    const double dx = e.x - o[3 * k], dy = e.y - o[3 * k + 1], dz = e.z - o[3 * k + 2];
    const double A = o[9 + 3 * k] / 2, B = o[10 + 3 * k] / 2, Cc = o[11 + 3 * k] / 2;
    ell[k] = soft_term(p.alpha, (dx * dx) / (A * A) + (dy * dy) / (B * B) + (dz * dz) / (Cc * Cc));
  }
  const double dx = e.x - p.target[0], dy = e.y - p.target[1], dz = e.z - p.target[2];
  const double s01 = sqrt(0.1);
  double pk = sqrt(dx * dx + 0.1);
  pk = pk - s01;
  pk = pk - 0.1;
  pk = pk + sqrt(dy * dy + 0.1);
  pk = pk - s01;
  pk = pk - 0.1;
  pk = pk + sqrt(dz * dz + 0.1);
  pk = pk - s01;
  pk = pk - 0.1;
  const double peak = log(exp(p.alpha2 * -pk) + 1.0) / p.alpha2;
  double u_cost = 0.0;
  if (a) {
    constexpr int NA = NJ > 0 ? NJ : 2;
#pragma unroll
    for (int i = 0; i < NA; ++i) u_cost += a[i] * a[i];
  }
  double vel = 0.0;
  if constexpr (NJ > 0) {
    if (f32state) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < NJ; ++k) acc = __fadd_rn(acc, __fmul_rn((float)s[NJ + k], (float)s[NJ + k]));
      vel = acc;
    } else {
#pragma unroll
      for (int k = 0; k < NJ; ++k) vel += s[NJ + k] * s[NJ + k];
    }
  }
  const double dist = (dx * dx + dy * dy) + dz * dz;
  double r = -w[0] * dist + w[1] * peak;
  r = r - w[2] * vel - w[3] * ell[0] - w[4] * ell[1] - w[5] * ell[2] - w[6] * u_cost + p.offset;
  return p.scale * r;
}

// CarPark.reward with the obstacle cost already summed (rollout path; float64 state).
__device__ inline double carpark_reward(const cacto_sys_params& p, const double* w, double x, double y,
                                        const double* s, const double* a, double obs) {
  const double dx = x - p.target[0], dy = y - p.target[1];
  const double peak = peak_cost(p, x, y);
  const double u_cost = a ? bound_control_cost<2>(p, a) : 0.0;
  const double dist = dx * dx + dy * dy;
  double r = -w[0] * dist + w[1] * peak;
  r = r - w[2] * (s[3] * s[3]) - w[3] * obs - w[6] * u_cost + p.offset;
  return p.scale * r;
}

// Env.reward with the end-effector position e = EE(s) already evaluated (a caller that also
// records EE(s) computes the forward kinematics once).
template <int NJ>
__device__ inline double env_reward_at(const SysDevice& sd, const double* w, const double* s, const double* a,
                                       bool f32state, const V3& e) {
  constexpr int NA = NJ > 0 ? NJ : 2;
  const cacto_sys_params& p = sd.p;
  if (p.reward_kind == CACTO_REW_UR5) return ur5_reward<NJ>(sd, w, s, a, f32state, e);
  const double x = e.x, y = e.y;
  const double* o = p.obs;
  const double ell1 = ell_cost(p, x, y, o[0], o[1], o[6], o[7]);
  const double ell2 = ell_cost(p, x, y, o[2], o[3], o[8], o[9]);
  const double ell3 = ell_cost(p, x, y, o[4], o[5], o[10], o[11]);
  const double dx = x - p.target[0], dy = y - p.target[1];
  const double s01 = sqrt(0.1);
  double pk = sqrt(dx * dx + 0.1);
  pk = pk - s01;
  pk = pk - 0.1;
  pk = pk + sqrt(dy * dy + 0.1);
  pk = pk - s01;
  pk = pk - 0.1;
  const double peak = log(exp(p.alpha2 * -pk) + 1.0) / p.alpha2;
  const double u_cost = a ? bound_control_cost<NA>(p, a) : 0.0;
  const double dist = dx * dx + dy * dy;
  double r = -w[0] * dist + w[1] * peak;
  if (NJ == -2 && p.reward_kind == CACTO_REW_CAR_PARK) {
    // - w2*v^2 - w3*obs_cost (CarPark.reward :638)
    const double v2 = f32state ? (double)__fmul_rn((float)s[3], (float)s[3]) : s[3] * s[3];
    const double obs = carpark_obs_cost(p, x, y, s[2], f32state);
    r = r - w[2] * v2 - w[3] * obs - w[6] * u_cost + p.offset;
    return p.scale * r;
  }
  if (NJ > 0 && p.reward_kind == CACTO_REW_MANIPULATOR) {
    double vel = 0.0;
    if (w[2] != 0.0) {
      if (f32state) {
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < NJ; ++k) acc = __fadd_rn(acc, __fmul_rn((float)s[NJ + k], (float)s[NJ + k]));
        vel = acc;
      } else {
#pragma unroll
        for (int k = 0; k < NJ; ++k) vel += s[NJ + k] * s[NJ + k];
      }
    }
    r = r - w[2] * vel;
  }
  r = r - w[3] * ell1 - w[4] * ell2 - w[5] * ell3 - w[6] * u_cost + p.offset;
  return p.scale * r;
}

template <int NJ>
__device__ inline double env_reward(const SysDevice& sd, const double* w, const double* s, const double* a,
                                    bool f32state) {
  return env_reward_at<NJ>(sd, w, s, a, f32state, env_ee<NJ>(sd, s));
}

// reward_batch's TF float32 part and its tape gradient (environment.py:282-286 and the dr_da tape
// of NeuralNetwork.py:199-204): r = scale*(-w6*u_cost) + f32(partial);
// u_cost = sum(a^2 + w_b*(a/u_max)^10); gradient in TF's op order (Mul/Pow/RealDiv grads).
template <int NA>
__device__ inline float reward_batch_f32(const cacto_sys_params& p, double w6, const float* a, double partial,
                                         float* dr_da) {
  const float scale = (float)p.scale, wb = (float)p.w_b, nw6 = (float)(-w6);
  float u = 0.0f;
  const float g = __fmul_rn(nw6, scale);
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const float umax = (float)p.u_max[i];
    const float D = __fdiv_rn(a[i], umax);
    const float t = __fadd_rn(__fmul_rn(a[i], a[i]), __fmul_rn(wb, powf(D, 10.0f)));
    u = (i == 0) ? t : __fadd_rn(u, t);
    if (dr_da) {
      const float t1 = __fmul_rn(__fmul_rn(g, 2.0f), a[i]);
      const float gD = __fmul_rn(__fmul_rn(__fmul_rn(wb, g), 10.0f), powf(D, 9.0f));
      dr_da[i] = __fadd_rn(t1, __fdiv_rn(gD, umax));
    }
  }
  return __fadd_rn(__fmul_rn(scale, __fmul_rn(nw6, u)), (float)partial);
}

// NJ: 0 single integrator, -1 car, -2 car_park (kinematic, 6 states, 2 controls), > 0 chain joints.
template <int NJ>
struct Dims {
  static constexpr int NS = NJ == 0 ? 3 : NJ < 0 ? 6 : 2 * NJ + 1;
  static constexpr int NA = NJ > 0 ? NJ : 2;
};

// Dispatch a templated launcher on the system's dynamics: F<NJ>::run(args...).
template <template <int> class F, typename... Args>
inline int dispatch_nj(const cacto_sys_params& p, Args&&... args) {
  if (p.dyn_kind == CACTO_DYN_SINGLE_INTEGRATOR) return F<0>::run(args...);
  if (p.dyn_kind == CACTO_DYN_CAR) return F<-1>::run(args...);
  if (p.dyn_kind == CACTO_DYN_CAR_PARK) return F<-2>::run(args...);
  switch (p.n_joints) {
    case 2: return F<2>::run(args...);
    case 3: return F<3>::run(args...);
    case 6: return F<6>::run(args...);
    default: break;
  }
  set_error("unsupported joint count (this build instantiates 2, 3 and 6)");
  return CACTO_EUNSUPPORTED;
}

}  // namespace cacto
