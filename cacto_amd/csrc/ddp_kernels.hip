#include <cstdlib>
// Sobolev labels without CasADi: the DDP backward pass of TO.backward_pass
// (TO.py:119-202) along recorded trajectories, on the GPU.
//
// Per episode (one thread; the recursion is sequential in t, episodes are independent):
//   V_x, V_xx      = d/dx, d2/dx2 of the terminal reward at x_T            (TO.py:166-168)
//   for i = T-1 .. 0:
//     A, B         = augmented_derivative(x_i, u_i)                        (environment.py:111-132,
//                                                                            SI :221-233, Car :420-435)
//     l_x, l_xx, l_u, l_uu of the running reward (l_xu = 0: the cost separates in x and u)
//     Q_x = l_x + A^T V_x   Q_u = l_u + B^T V_x   Q_xx = l_xx + A^T V_xx A
//     Q_uu = l_uu + B^T V_xx B   Q_xu = A^T V_xx B   (TO.py:182-186)
//     V_x = Q_x - Q_xu Qbar^-1 Q_u,  V_xx = Q_xx - Q_xu Qbar^-1 Q_xu^T, Qbar = Q_uu + mu I (:188-194)
// The reference differentiates the TO cost (environment_TO.py, = -reward) symbolically with CasADi;
// here the planar-family derivatives are closed forms of the same expression (ellipses and the
// peak term as softplus of their arguments: d softplus(z)/dz = sigmoid(z)). Qbar is inverted by
// Gauss-Jordan with partial pivoting (np.linalg.pinv in the reference equals the inverse for the
// nonsingular, mu-regularised Qbar): float64 results within 1e-9 relative of the oracle.
//
// Every system: the single integrator (NJ = 0), car (NJ = -1) and prismatic Pinocchio chains (the
// double integrator: M and nle constant, so ddq_dq = ddq_dv = 0 and Fu = dt [0; M^-1]) use closed
// forms; car_park (NJ = -2) closed-form Jacobians (environment.py:567-582) with its smooth-box cost
// differentiated by hyper-dual numbers (ad.h); revolute chains (manipulator NJ = 3, UR5 NJ = 6) take
// ddq_dq, ddq_dv from hyper-dual RNEA (computeABADerivatives) and l_x, l_xx through hyper-dual
// forward kinematics.
#include "ad.h"
#include "internal.h"

namespace cacto {

template <int NJ>
struct DdpDims {
  static constexpr int N = Dims<NJ>::NS - 1, M = Dims<NJ>::NA;
  static constexpr bool ok = NJ >= -2;
};

// Reward derivatives w.r.t. the EE position p = (px, py) of the planar family (environment_TO.py
// :208-234 DI, :90-111 SI, :339-360 Car; reward = -cost), without the scale factor.
struct PosDerivs {
  double g[2];
  double H[3];  // xx, xy, yy
};

__device__ inline void planar_pos_derivs(const cacto_sys_params& p, const double* w, double px, double py, PosDerivs& d) {
  const double dx = px - p.target[0], dy = py - p.target[1];
  // - w0 * dist
  d.g[0] = -w[0] * (2.0 * dx);
  d.g[1] = -w[0] * (2.0 * dy);
  d.H[0] = -w[0] * 2.0;
  d.H[1] = 0.0;
  d.H[2] = -w[0] * 2.0;
  // + w1 * peak, peak = softplus(-alpha2 s) / alpha2, s = sqrt(dx2+.1) - .1 + sqrt(dy2+.1) - .1 - 2 sqrt(.1)
  {
    const double rx = sqrt(dx * dx + 0.1), ry = sqrt(dy * dy + 0.1);
    const double s = rx - 0.1 + ry - 0.1 - 2.0 * sqrt(0.1);
    const double sg = 1.0 / (1.0 + exp(p.alpha2 * s));  // sigmoid(-alpha2 s)
    const double sx = dx / rx, sy = dy / ry;
    const double k2 = p.alpha2 * sg * (1.0 - sg);
    d.g[0] += w[1] * (-sg * sx);
    d.g[1] += w[1] * (-sg * sy);
    d.H[0] += w[1] * (-sg * (0.1 / (rx * rx * rx)) + k2 * sx * sx);
    d.H[1] += w[1] * (k2 * sx * sy);
    d.H[2] += w[1] * (-sg * (0.1 / (ry * ry * ry)) + k2 * sy * sy);
  }
  // - w_{3+k} * ell_k, ell = softplus(alpha (1 - e)) / alpha, e = (dx/a)^2 + (dy/b)^2
  for (int k = 0; k < 3; ++k) {
    const double a = p.obs[6 + 2 * k] / 2, b = p.obs[7 + 2 * k] / 2;
    const double ex = px - p.obs[2 * k], ey = py - p.obs[2 * k + 1];
    const double e = (ex * ex) / (a * a) + (ey * ey) / (b * b);
    const double sg = 1.0 / (1.0 + exp(-(p.alpha * -(e - 1.0))));
    const double gx = 2.0 * ex / (a * a), gy = 2.0 * ey / (b * b);
    const double k2 = p.alpha * sg * (1.0 - sg);
    const double wk = w[3 + k];
    d.g[0] -= wk * (-sg * gx);
    d.g[1] -= wk * (-sg * gy);
    d.H[0] -= wk * (-sg * (2.0 / (a * a)) + k2 * gx * gx);
    d.H[1] -= wk * (k2 * gx * gy);
    d.H[2] -= wk * (-sg * (2.0 / (b * b)) + k2 * gy * gy);
  }
}

// Position terms of a revolute chain's reward: l_q, l_qq by the chain rule through one float64
// forward-kinematics pass. With z_i, o_i joint i's world axis and origin and p the EE position:
// dp/dq_i = z_i x (p - o_i) and d2p/dq_i dq_j = z_i x (z_j x (p - o_j)) for i <= j (0 past the EE's
// parent joint); dr/dp, d2r/dp2 from hyper-dual evaluations of the position reward (6 passes).
// l_q = J^T dr/dp, l_qq = J^T (d2r/dp2) J + sum_c dr/dp_c d2p_c/dq2. Returns false (caller falls back
// to hyper-dual kinematics) if a joint up to the EE is prismatic.
template <int NJ>
__device__ inline bool chain_pos_derivs(const SysDevice& sd, const double* w, const double* q, double* lx,
                                        double* lxx, int ldl) {
  const cacto_sys_params& p = sd.p;
  const int e = p.ee_parent;
  V3 z[NJ], o[NJ];
  M3 oR;
  V3 op;
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const JointView j{sd.joints + i * CACTO_JOINT_COLS};
    if (i <= e && j.kind() != 0) return false;
    const SE3 X = joint_placement(j, q[i]);
    if (i == 0) {
      oR = X.R;
      op = X.p;
    } else {
      op = mul(oR, X.p) + op;
      oR = mul(oR, X.R);
    }
    z[i] = mul(oR, j.axis());
    o[i] = op;
    if (i == e) break;
  }
  // EE: oR, op are joint e's frame when the loop ended
  const V3 pe = mul(oR, v3(p.ee_p[0], p.ee_p[1], p.ee_p[2])) + op;
  double g[3], H[9];
  for (int a = 0; a < 3; ++a)
    for (int b = a; b < 3; ++b) {
      V3T<HD> P{HD(pe.x, a == 0, b == 0, 0.0), HD(pe.y, a == 1, b == 1, 0.0), HD(pe.z, a == 2, b == 2, 0.0)};
      const HD r = chain_pos_reward_t(p, w, P);
      if (a == b) g[a] = r.a;
      H[a * 3 + b] = H[b * 3 + a] = r.ab;
    }
  V3 Jc[NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) Jc[i] = i <= e ? cross(z[i], pe - o[i]) : v3(0, 0, 0);
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    lx[i] = g[0] * Jc[i].x + g[1] * Jc[i].y + g[2] * Jc[i].z;
    const V3 HJi = v3(H[0] * Jc[i].x + H[1] * Jc[i].y + H[2] * Jc[i].z, H[3] * Jc[i].x + H[4] * Jc[i].y + H[5] * Jc[i].z,
                      H[6] * Jc[i].x + H[7] * Jc[i].y + H[8] * Jc[i].z);
#pragma unroll
    for (int k = i; k < NJ; ++k) {
      double v = dot(Jc[k], HJi);
      if (k <= e) {
        const V3 d2 = cross(z[i], cross(z[k], pe - o[k]));
        v += g[0] * d2.x + g[1] * d2.y + g[2] * d2.z;
      }
      lxx[i * ldl + k] = lxx[k * ldl + i] = v;
    }
  }
  return true;
}

// l_x [N], l_xx [N*N] of the reward with weights w at state x (time excluded).
template <int NJ>
__device__ inline void ddp_lx(const SysDevice& sd, const double* w, const double* x, double* lx, double* lxx) {
  constexpr int N = DdpDims<NJ>::N;
  const cacto_sys_params& p = sd.p;
#pragma unroll
  for (int k = 0; k < N * N; ++k) lxx[k] = 0.0;
#pragma unroll
  for (int k = 0; k < N; ++k) lx[k] = 0.0;
  if constexpr (NJ == -2) {
    // car_park (environment_TO.py:479-503): every position term is a function of one planar point
    // Z(x, y, theta) — p_ee for the target terms, p_ee + R(theta) c_k for the 30 (box, check point)
    // pairs. Its gradient / Hessian in Z come from 3 hyper-dual passes; the rigid map Z has
    // dZ/d(x, y) = I, dZ/dtheta = (-(Z_y - y), Z_x - x), d2Z/dtheta2 = -(Z - (x, y)).
    double sn, cs;
    sincos(x[2], &sn, &cs);
    const double h = p.L_delta / 2.0;
    const double pex = x[0] + cs * h, pey = x[1] + sn * h;
    auto add_point = [&](double Zx, double Zy, auto&& f) {
      const HD rxx = f(HD(Zx, 1.0, 1.0, 0.0), HD(Zy));
      const HD rxy = f(HD(Zx, 1.0, 0.0, 0.0), HD(Zy, 0.0, 1.0, 0.0));
      const HD ryy = f(HD(Zx), HD(Zy, 1.0, 1.0, 0.0));
      const double gx = rxy.a, gy = rxy.b, Hxx = rxx.ab, Hxy = rxy.ab, Hyy = ryy.ab;
      const double tx = -(Zy - x[1]), ty = Zx - x[0];   // dZ/dtheta
      lx[0] += gx;
      lx[1] += gy;
      lx[2] += gx * tx + gy * ty;
      lxx[0] += Hxx;
      lxx[1] += Hxy;
      lxx[N + 1] += Hyy;
      lxx[2] += Hxx * tx + Hxy * ty;
      lxx[N + 2] += Hxy * tx + Hyy * ty;
      lxx[2 * N + 2] += tx * (Hxx * tx + Hxy * ty) + ty * (Hxy * tx + Hyy * ty) - gx * (Zx - x[0]) - gy * (Zy - x[1]);
    };
    add_point(pex, pey, [&](HD X, HD Y) {
      HD d[2] = {X - p.target[0], Y - p.target[1]};
      return -(p.scale * (w[0] * (d[0] * d[0] + d[1] * d[1]) - w[1] * peak_t<2>(p.alpha2, d)));
    });
#pragma unroll 1
    for (int k = 0; k < p.n_check; ++k) {
      const double bx = p.check_points[2 * k], by = p.check_points[2 * k + 1];
      add_point(cs * bx - sn * by + pex, sn * bx + cs * by + pey, [&](HD X, HD Y) {
        HD b = HD(0.0);
        for (int ob = 0; ob < 3; ++ob)
          b = b + box_cost_t(X, Y, p.obs[2 * ob], p.obs[2 * ob + 1], p.obs[6 + 2 * ob], p.obs[7 + 2 * ob], p.k_db);
        return -(p.scale * (w[3] * b));
      });
    }
    lxx[N] = lxx[1];
    lxx[2 * N] = lxx[2];
    lxx[2 * N + 1] = lxx[N + 2];
    lx[3] = -(p.scale * (w[2] * (2.0 * x[3])));
    lxx[3 * N + 3] = -(p.scale * (w[2] * 2.0));
    return;
  } else {
    if (NJ > 2 && p.reward_kind != CACTO_REW_PLANAR) {
      // revolute chains: position terms through hyper-dual forward kinematics, one pass per
      // (j <= k) joint pair; the velocity term - scale w2 |v|^2 in closed form
      constexpr int nq = NJ > 0 ? NJ : 1;
      if (!chain_pos_derivs<nq>(sd, w, x, lx, lxx, N)) {
#pragma unroll 1
        for (int j = 0; j < nq; ++j)
#pragma unroll 1
          for (int k = j; k < nq; ++k) {
            HD q[nq];
#pragma unroll
            for (int i = 0; i < nq; ++i) q[i] = HD(x[i], i == j ? 1.0 : 0.0, i == k ? 1.0 : 0.0, 0.0);
            const HD r = chain_pos_reward_t(p, w, chain_ee_t<nq, HD>(sd, q));
            if (k == j) lx[j] = r.a;
            lxx[j * N + k] = lxx[k * N + j] = r.ab;
          }
      }
#pragma unroll
      for (int i = nq; i < N; ++i) {
        lx[i] = -(p.scale * (w[2] * (2.0 * x[i])));
        lxx[i * N + i] = -(p.scale * (w[2] * 2.0));
      }
      return;
    }
    PosDerivs d;
    planar_pos_derivs(p, w, x[0], x[1], d);  // p_ee = (x0, x1): SI / car states, DI q (unit prismatic axes)
    lx[0] = p.scale * d.g[0];
    lx[1] = p.scale * d.g[1];
    lxx[0] = p.scale * d.H[0];
    lxx[1] = lxx[N] = p.scale * d.H[1];
    lxx[N + 1] = p.scale * d.H[2];
    if constexpr (NJ > 0) {
      // DI: - w2 * |v|^2 (environment_TO.py:227-230)
#pragma unroll
      for (int i = NJ; i < N; ++i) {
        lx[i] = p.scale * (-w[2] * (2.0 * x[i]));
        lxx[i * N + i] = p.scale * (-w[2] * 2.0);
      }
    }
  }
}

// Discrete dynamics Jacobians A [N*N], B [N*M] (augmented_derivative).
template <int NJ>
__device__ inline void ddp_jacobians(const SysDevice& sd, const double* x, const double* Minv, double* A, double* B) {
  constexpr int N = DdpDims<NJ>::N, M = DdpDims<NJ>::M;
  const double dt = sd.p.dt;
#pragma unroll
  for (int k = 0; k < N * N; ++k) A[k] = (k % (N + 1) == 0) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < N * M; ++k) B[k] = 0.0;
  if constexpr (NJ == 0) {
    B[0 * M + 0] = dt;
    B[1 * M + 1] = dt;
  } else if constexpr (NJ == -1) {
    const double s2 = sin(x[2]), c2 = cos(x[2]);
    A[0 * N + 2] = -dt * x[3] * s2 - dt * dt * x[4] * s2 / 2;
    A[0 * N + 3] = dt * c2;
    A[0 * N + 4] = dt * dt * c2 / 2;
    A[1 * N + 2] = dt * x[3] * c2 + dt * dt * x[4] * c2 / 2;
    A[1 * N + 3] = dt * s2;
    A[1 * N + 4] = dt * dt * s2 / 2;
    A[3 * N + 4] = dt;
    B[2 * M + 0] = dt;
    B[4 * M + 1] = dt;
  } else if constexpr (NJ == -2) {
    // CarPark.augmented_derivative (environment.py:567-582); sec^2 = 1 / cos^2
    const double s2 = sin(x[2]), c2 = cos(x[2]), L = sd.p.L_delta, cd = cos(x[4]);
    A[0 * N + 2] = -dt * x[3] * s2;
    A[0 * N + 3] = dt * c2;
    A[1 * N + 2] = dt * x[3] * c2;
    A[1 * N + 3] = dt * s2;
    A[2 * N + 3] = dt * tan(x[4]) / L;
    A[2 * N + 4] = dt * x[3] * (1.0 / (cd * cd)) / L;
    B[3 * M + 0] = dt;
    B[4 * M + 1] = dt / sd.p.tau_delta;
  } else {
    constexpr int nv = NJ > 0 ? NJ : 1;
#pragma unroll
    for (int i = 0; i < nv; ++i) A[i * N + nv + i] = dt;  // I + dt [[0, I], [ddq_dq = 0, ddq_dv = 0]]
#pragma unroll
    for (int i = 0; i < nv; ++i)
#pragma unroll
      for (int j = 0; j < M; ++j) B[(nv + i) * M + j] = Minv[i * M + j] * dt;
  }
}

// Structural nonzeros of A, B for the systems of the fused pass (SI, car, prismatic chain). The
// products below skip the terms that are exactly zero: a sum that leaves out 0 * finite terms is the
// same number (the fully unrolled loops fold these tests away), at a third of the f64 instructions.
template <int NJ>
__device__ __forceinline__ constexpr bool a_nz(int k, int c) {
  return k == c || (NJ == -1 && ((k <= 1 && c >= 2) || (k == 3 && c == 4))) || (NJ > 0 && k < NJ && c == k + NJ);
}
template <int NJ>
__device__ __forceinline__ constexpr bool b_nz(int k, int j) {
  return NJ == 0 ? k == j : NJ == -1 ? ((k == 2 && j == 0) || (k == 4 && j == 1)) : k >= NJ;
}

// In-place inverse of a small matrix (Gauss-Jordan, partial pivoting).
template <int M>
__device__ inline void small_inverse(double* a, double* inv) {
#pragma unroll
  for (int i = 0; i < M * M; ++i) inv[i] = (i % (M + 1) == 0) ? 1.0 : 0.0;
#pragma unroll
  for (int c = 0; c < M; ++c) {
    int piv = c;
    double best = fabs(a[c * M + c]);
#pragma unroll
    for (int r = c + 1; r < M; ++r)
      if (fabs(a[r * M + c]) > best) {
        best = fabs(a[r * M + c]);
        piv = r;
      }
#pragma unroll
    for (int r = 0; r < M; ++r)  // swap rows c and piv (branch-free over the fixed row set)
      if (r == piv && r != c)
#pragma unroll
        for (int k = 0; k < M; ++k) {
          double t = a[c * M + k];
          a[c * M + k] = a[r * M + k];
          a[r * M + k] = t;
          t = inv[c * M + k];
          inv[c * M + k] = inv[r * M + k];
          inv[r * M + k] = t;
        }
    const double d = 1.0 / a[c * M + c];
#pragma unroll
    for (int k = 0; k < M; ++k) {
      a[c * M + k] *= d;
      inv[c * M + k] *= d;
    }
#pragma unroll
    for (int r = 0; r < M; ++r)
      if (r != c) {
        const double f = a[r * M + c];
#pragma unroll
        for (int k = 0; k < M; ++k) {
          a[r * M + k] -= f * a[c * M + k];
          inv[r * M + k] -= f * inv[c * M + k];
        }
      }
  }
}

// Revolute chains (computeABADerivatives, environment.py:111-132): M(q)^-1, qdd = M^-1 (u - nle),
// then one hyper-dual RNEA(q + e1 e_k, v + e2 e_k, qdd) per joint k gives column k of dtau/dq (e1
// part) and dtau/dv (e2 part); ddq_dq = -M^-1 dtau/dq, ddq_dv = -M^-1 dtau/dv.
// A = I + dt [[0, I], [ddq_dq, ddq_dv]], B = dt [0; M^-1].
template <int NJ>
__device__ inline void ddp_chain_jacobians(const SysDevice& sd, const double* x, const double* u, double* A,
                                           double* B) {
  if constexpr (NJ > 2) {
    constexpr int N = 2 * NJ;
    const double dt = sd.p.dt;
    double Mm[NJ * NJ], Minv[NJ * NJ], h[NJ], qdd[NJ];
    chain_mass<NJ>(sd, x, Mm);
    small_inverse<NJ>(Mm, Minv);
    chain_nle<NJ>(sd, x, x + NJ, h);
#pragma unroll
    for (int r = 0; r < NJ; ++r) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < NJ; ++k) s += Minv[r * NJ + k] * (u[k] - h[k]);
      qdd[r] = s;
    }
#pragma unroll
    for (int k = 0; k < N * N; ++k) A[k] = (k % (N + 1) == 0) ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < NJ; ++i) A[i * N + NJ + i] = dt;
#pragma unroll 1
    for (int k = 0; k < NJ; ++k) {
      TD q[NJ], v[NJ], tau[NJ];
#pragma unroll
      for (int i = 0; i < NJ; ++i) {
        q[i] = TD(x[i], i == k ? 1.0 : 0.0, 0.0);
        v[i] = TD(x[NJ + i], 0.0, i == k ? 1.0 : 0.0);
      }
      rnea_tan<NJ, TD>(sd, q, v, qdd, tau);
#pragma unroll
      for (int r = 0; r < NJ; ++r) {
        double sq = 0.0, sv = 0.0;
#pragma unroll
        for (int c = 0; c < NJ; ++c) {
          sq += Minv[r * NJ + c] * tau[c].a;
          sv += Minv[r * NJ + c] * tau[c].b;
        }
        A[(NJ + r) * N + k] = -dt * sq;
        A[(NJ + r) * N + NJ + k] += -dt * sv;
      }
    }
#pragma unroll
    for (int k = 0; k < N * NJ; ++k) B[k] = 0.0;
#pragma unroll
    for (int r = 0; r < NJ; ++r)
#pragma unroll
      for (int c = 0; c < NJ; ++c) B[(NJ + r) * NJ + c] = Minv[r * NJ + c] * dt;
  }
}

// Per-step derivative record of the split pass (car_park and the revolute chains, whose
// derivatives cost far more than the recursion): A [N*N], B [N*M], l_x [N], l_xx [N*N] of step t
// (the terminal step: l_x, l_xx of the terminal weights). Workspace layout [t][k][e]: element k of
// episode e's step-t record at ws[(t * R + k) * n_ep + e], so the lanes (episodes) of a wave read
// and write consecutive addresses.
template <int NJ>
struct DdpRec {
  static constexpr int N = DdpDims<NJ>::N, M = DdpDims<NJ>::M;
  static constexpr int A = 0, B = N * N, LX = B + N * M, LXX = LX + N, R = LXX + N * N;
};

// One thread per (episode, step): the steps are independent given the trajectory, so the
// hyper-dual work runs over every step of every episode at once (grid.y = step).
template <int NJ>
__global__ void __launch_bounds__(64) k_ddp_derivs(const SysDevice* __restrict__ sdp, const double* __restrict__ S,
                                                    int64_t ldS, const double* __restrict__ U, int64_t ldU,
                                                    const int32_t* __restrict__ nsteps, int n_ep,
                                                    double* __restrict__ ws) {
  using RC = DdpRec<NJ>;
  constexpr int N = RC::N, M = RC::M, ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = blockIdx.y;
  if (e >= n_ep) return;
  const int Te = nsteps[e];
  if (t > Te) return;  // also Te < 0: a dropped episode (main.py:236), skipped
  const SysDevice& sd = *sdp;
  double x[N], w[7];
#pragma unroll
  for (int k = 0; k < N; ++k) x[k] = S[((size_t)e * ldS + t) * ns + k];
#pragma unroll
  for (int k = 0; k < 7; ++k) w[k] = t == Te ? sd.p.w_terminal[k] : sd.p.w_running[k];
  double* rec = ws + (size_t)t * RC::R * n_ep + e;
  double lx[N], lxx[N * N];
  ddp_lx<NJ>(sd, w, x, lx, lxx);
#pragma unroll
  for (int k = 0; k < N; ++k) rec[(size_t)(RC::LX + k) * n_ep] = lx[k];
#pragma unroll
  for (int k = 0; k < N * N; ++k) rec[(size_t)(RC::LXX + k) * n_ep] = lxx[k];
  if (t == Te) return;
  double u[M], A[N * N], B[N * M];
#pragma unroll
  for (int k = 0; k < M; ++k) u[k] = U[((size_t)e * ldU + t) * na + k];
  if constexpr (NJ > 2)
    ddp_chain_jacobians<NJ>(sd, x, u, A, B);
  else
    ddp_jacobians<NJ>(sd, x, nullptr, A, B);
#pragma unroll
  for (int k = 0; k < N * N; ++k) rec[(size_t)(RC::A + k) * n_ep] = A[k];
#pragma unroll
  for (int k = 0; k < N * M; ++k) rec[(size_t)(RC::B + k) * n_ep] = B[k];
}

// k_ddp_derivs for the revolute chains as three kernels, each with the registers of its own part
// (one thread per (episode, step) carried all of it: A, B, l_xx and NJ hyper-dual RNEA passes
// held at once, 9 KB of scratch per lane for UR5):
//   k_ddp_prim  one thread per step: M^-1 (CRBA, inverse), bias forces, qdd = M^-1 (u - h) ->
//               a [t][k][e] workspace; B = M^-1 dt and A's q rows straight to the record;
//   k_ddp_tan   one thread per (step, direction): direction d < NJ is d/dq_d, d >= NJ d/dv_{d-NJ},
//               one RNEA on dual numbers -> column d of A's v rows;
//   k_ddp_lx    one thread per step (the terminal one included): l_x, l_xx.
// Every value is formed by the same operations in the same order as k_ddp_derivs (the dual
// number's tangent is the hyper-dual's a or b part), so the records are bit-identical.
template <int NJ>
struct DdpPrim {
  static constexpr int MINV = 0, QDD = NJ * NJ, R = NJ * NJ + NJ;
};

template <int NJ>
__global__ void __launch_bounds__(64) k_ddp_prim(const SysDevice* __restrict__ sdp, const double* __restrict__ S,
                                                 int64_t ldS, const double* __restrict__ U, int64_t ldU,
                                                 const int32_t* __restrict__ nsteps, int n_ep, double* __restrict__ ws,
                                                 double* __restrict__ pw) {
  using RC = DdpRec<NJ>;
  using PC = DdpPrim<NJ>;
  constexpr int N = RC::N, ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = blockIdx.y;
  if (e >= n_ep) return;
  const int Te = nsteps[e];
  if (t >= Te) return;  // the terminal step has no A, B; Te < 0: a dropped episode
  const SysDevice& sd = *sdp;
  const double dt = sd.p.dt;
  double x[N], u[NJ], Mm[NJ * NJ], Minv[NJ * NJ], h[NJ];
#pragma unroll
  for (int k = 0; k < N; ++k) x[k] = S[((size_t)e * ldS + t) * ns + k];
#pragma unroll
  for (int k = 0; k < NJ; ++k) u[k] = U[((size_t)e * ldU + t) * na + k];
  chain_mass<NJ>(sd, x, Mm);
  small_inverse<NJ>(Mm, Minv);
  chain_nle<NJ>(sd, x, x + NJ, h);
  double* pr = pw + (size_t)t * PC::R * n_ep + e;
#pragma unroll
  for (int r = 0; r < NJ; ++r) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NJ; ++k) s += Minv[r * NJ + k] * (u[k] - h[k]);
    pr[(size_t)(PC::QDD + r) * n_ep] = s;
  }
#pragma unroll
  for (int k = 0; k < NJ * NJ; ++k) pr[(size_t)(PC::MINV + k) * n_ep] = Minv[k];
  double* rec = ws + (size_t)t * RC::R * n_ep + e;
#pragma unroll
  for (int i = 0; i < NJ; ++i)
#pragma unroll
    for (int c = 0; c < N; ++c) rec[(size_t)(RC::A + i * N + c) * n_ep] = c == i ? 1.0 : (c == NJ + i ? dt : 0.0);
#pragma unroll
  for (int k = 0; k < NJ * NJ; ++k) rec[(size_t)(RC::B + k) * n_ep] = 0.0;
#pragma unroll
  for (int r = 0; r < NJ; ++r)
#pragma unroll
    for (int c = 0; c < NJ; ++c) rec[(size_t)(RC::B + (NJ + r) * NJ + c) * n_ep] = Minv[r * NJ + c] * dt;
}

// A DN spatial vector in LDS, structure of arrays over the 64 lanes of the block
struct SvLds {
  double* b;  // 12 x 64 doubles: (l.x, l.y, l.z, a.x, a.y, a.z) values then tangents
  __device__ __forceinline__ void st(int lane, const SVT<DN>& f) const {
    const DN c[6] = {f.l.x, f.l.y, f.l.z, f.a.x, f.a.y, f.a.z};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      b[k * 64 + lane] = c[k].v;
      b[(6 + k) * 64 + lane] = c[k].a;
    }
  }
  __device__ __forceinline__ SVT<DN> ld(int lane) const {
    DN c[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) c[k] = DN(b[k * 64 + lane], b[(6 + k) * 64 + lane]);
    return {{c[0], c[1], c[2]}, {c[3], c[4], c[5]}};
  }
};

template <int NJ>
__global__ void __launch_bounds__(64) k_ddp_tan(const SysDevice* __restrict__ sdp, const double* __restrict__ S,
                                                int64_t ldS, const int32_t* __restrict__ nsteps, int n_ep,
                                                double* __restrict__ ws, const double* __restrict__ pw) {
  using RC = DdpRec<NJ>;
  using PC = DdpPrim<NJ>;
  constexpr int N = RC::N, ns = Dims<NJ>::NS;
  // rnea_tan<NJ, DN> with the joint loops rolled and the per-joint forces parked in LDS (the fully
  // unrolled pass held every joint's parameters and forces in registers and spilled 4.5 KB per
  // lane); the same operations in the same order
  __shared__ double fl[NJ * 12 * 64];
  __shared__ double taul[NJ * 64];
  const int lane = threadIdx.x;
  const int e = blockIdx.x * blockDim.x + lane;
  const int t = blockIdx.y, d = blockIdx.z;
  if (e >= n_ep) return;
  const int Te = nsteps[e];
  if (t >= Te) return;
  const SysDevice& sd = *sdp;
  const double dt = sd.p.dt;
  const double* pr = pw + (size_t)t * PC::R * n_ep + e;
  const double* xs = S + ((size_t)e * ldS + t) * ns;
  const bool dq = d < NJ;
  const int k = dq ? d : d - NJ;
  SVT<DN> vp{{DN(0.0), DN(0.0), DN(0.0)}, {DN(0.0), DN(0.0), DN(0.0)}};
  SVT<DN> ap{{DN(-sd.p.gravity[0]), DN(-sd.p.gravity[1]), DN(-sd.p.gravity[2])}, {DN(0.0), DN(0.0), DN(0.0)}};
#pragma unroll 1
  for (int i = 0; i < NJ; ++i) {
    const JointView j{sd.joints + i * CACTO_JOINT_COLS};
    const DN qi(xs[i], dq && i == k ? 1.0 : 0.0), vi_(xs[NJ + i], !dq && i == k ? 1.0 : 0.0);
    const double qddi = pr[(size_t)(PC::QDD + i) * n_ep];
    const SE3T<DN> X = joint_placement_t<DN>(j, qi);
    const SV Sj = joint_S(j);
    const SVT<DN> Sv{scale3(vi_, lift<DN>(Sj.l)), scale3(vi_, lift<DN>(Sj.a))};
    SVT<DN> vi = act_motion_inv_t(X, vp);
    vi.l = vi.l + Sv.l;
    vi.a = vi.a + Sv.a;
    SVT<DN> ai = act_motion_inv_t(X, ap);
    const SVT<DN> c = cross_motion_t(vi, Sv);
    ai.l = ai.l + c.l + lift<DN>(qddi * Sj.l);
    ai.a = ai.a + c.a + lift<DN>(qddi * Sj.a);
    const Inertia I = j.inertia();
    const SVT<DN> Iv = inertia_mul_t(I, vi), Ia = inertia_mul_t(I, ai);
    const SVT<DN> vf = cross_force_t(vi, Iv);
    SvLds{fl + i * 12 * 64}.st(lane, {Ia.l + vf.l, Ia.a + vf.a});
    vp = vi;
    ap = ai;
  }
  SVT<DN> f = SvLds{fl + (NJ - 1) * 12 * 64}.ld(lane);
#pragma unroll 1
  for (int i = NJ - 1; i >= 0; --i) {
    const JointView j{sd.joints + i * CACTO_JOINT_COLS};
    const SV Sj = joint_S(j);
    const DN ti = dot3(lift<DN>(Sj.l), f.l) + dot3(lift<DN>(Sj.a), f.a);
    taul[i * 64 + lane] = ti.a;
    if (i > 0) {
      const DN qi(xs[i], dq && i == k ? 1.0 : 0.0);
      const SVT<DN> fp = act_force_t(joint_placement_t<DN>(j, qi), f);
      const SVT<DN> fo = SvLds{fl + (i - 1) * 12 * 64}.ld(lane);
      f.l = fo.l + fp.l;
      f.a = fo.a + fp.a;
    }
  }
  double* rec = ws + (size_t)t * RC::R * n_ep + e;
#pragma unroll
  for (int r = 0; r < NJ; ++r) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < NJ; ++c) s += pr[(size_t)(PC::MINV + r * NJ + c) * n_ep] * taul[c * 64 + lane];
    if (dq)
      rec[(size_t)(RC::A + (NJ + r) * N + k) * n_ep] = -dt * s;
    else
      rec[(size_t)(RC::A + (NJ + r) * N + NJ + k) * n_ep] = (r == k ? 1.0 : 0.0) + -dt * s;
  }
}

template <int NJ>
__global__ void __launch_bounds__(64) k_ddp_lx(const SysDevice* __restrict__ sdp, const double* __restrict__ S,
                                               int64_t ldS, const int32_t* __restrict__ nsteps, int n_ep,
                                               double* __restrict__ ws) {
  using RC = DdpRec<NJ>;
  constexpr int N = RC::N, ns = Dims<NJ>::NS;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = blockIdx.y;
  if (e >= n_ep) return;
  const int Te = nsteps[e];
  if (t > Te) return;
  const SysDevice& sd = *sdp;
  double x[N], w[7], lx[N], lxx[N * N];
#pragma unroll
  for (int k = 0; k < N; ++k) x[k] = S[((size_t)e * ldS + t) * ns + k];
#pragma unroll
  for (int k = 0; k < 7; ++k) w[k] = t == Te ? sd.p.w_terminal[k] : sd.p.w_running[k];
  ddp_lx<NJ>(sd, w, x, lx, lxx);
  double* rec = ws + (size_t)t * RC::R * n_ep + e;
#pragma unroll
  for (int k = 0; k < N; ++k) rec[(size_t)(RC::LX + k) * n_ep] = lx[k];
#pragma unroll
  for (int k = 0; k < N * N; ++k) rec[(size_t)(RC::LXX + k) * n_ep] = lxx[k];
}

// Env.augmented_derivative (environment.py:111-132; SI :221-233, Car :420-435, CarPark :567-582) for
// B independent (state, action) rows: the discrete-time Jacobians Fx [nx, nx], Fu [nx, na] that the
// DDP pass consumes (the same device code), for host-side callers such as TO.backward_pass
// (TO.py:181). Closed-form systems: one thread per row. Revolute chains go through the split DDP
// pass's derivative kernel (k_ddp_derivs: each row as a one-step episode, records extracted by
// k_jac_extract), so their hyper-dual RNEA runs in exactly one kernel.
template <int NJ>
__global__ void __launch_bounds__(64) k_env_jacobians(const SysDevice* __restrict__ sdp, const double* __restrict__ S,
                                                      const double* __restrict__ U, int B, double* __restrict__ Fx,
                                                      double* __restrict__ Fu) {
  constexpr int N = DdpDims<NJ>::N, M = DdpDims<NJ>::M, ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  if constexpr (NJ <= 2) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const SysDevice& sd = *sdp;
    double x[N], A[N * N], Bm[N * M];
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = S[(size_t)b * ns + k];
    if constexpr (NJ > 0) {
      double Mm[M * M], Minv[M * M];
      chain_mass<NJ>(sd, x, Mm);
      small_inverse<M>(Mm, Minv);
      ddp_jacobians<NJ>(sd, x, Minv, A, Bm);
    } else {
      ddp_jacobians<NJ>(sd, x, nullptr, A, Bm);
    }
#pragma unroll
    for (int k = 0; k < N * N; ++k) Fx[(size_t)b * N * N + k] = A[k];
#pragma unroll
    for (int k = 0; k < N * M; ++k) Fu[(size_t)b * N * M + k] = Bm[k];
  }
}

// Rows -> one-step episodes for the derivative kernels: S2 [B, 2, ns] (the state twice), nsteps = 1.
template <int NJ>
__global__ void k_jac_prep(const double* __restrict__ S, int B, double* __restrict__ S2, int32_t* __restrict__ n1) {
  constexpr int ns = Dims<NJ>::NS;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= B * 2 * ns) return;
  const int b = k / (2 * ns), c = k % ns;
  S2[k] = S[(size_t)b * ns + c];
  if (k < B) n1[k] = 1;
}

// Step-0 A, B records ([t][k][e] layout of DdpRec) -> Fx [B, N, N], Fu [B, N, M].
template <int NJ>
__global__ void k_jac_extract(const double* __restrict__ ws, int B, double* __restrict__ Fx, double* __restrict__ Fu) {
  using RC = DdpRec<NJ>;
  constexpr int N = RC::N, M = RC::M;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= B * (N * N + N * M)) return;
  const int b = k % B, r = k / B;
  const double v = ws[(size_t)(RC::A + r) * B + b];
  if (r < N * N)
    Fx[(size_t)b * N * N + r] = v;
  else
    Fu[(size_t)b * N * M + (r - N * N)] = v;
}

// The fused pass for the closed-form systems (SI, car, DI): one thread per episode computes each
// step's A, B, l_x, l_xx inline and runs the Riccati recursion (sequential in t).
template <int NJ>
__global__ void __launch_bounds__(64) k_ddp_backward(const SysDevice* __restrict__ sdp, const double* __restrict__ S,
                                                      int64_t ldS, const double* __restrict__ U, int64_t ldU,
                                                      const int32_t* __restrict__ nsteps, int n_ep, double mu,
                                                      double* __restrict__ dVdx) {
  constexpr int N = DdpDims<NJ>::N, M = DdpDims<NJ>::M, ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_ep) return;
  const SysDevice& sd = *sdp;
  const cacto_sys_params& p = sd.p;
  const int Te = nsteps[e];
  if (Te < 0) return;  // a dropped episode (main.py:236): no labels
  const double* Se = S + (size_t)e * ldS * ns;
  const double* Ue = U + (size_t)e * ldU * na;
  double* Oe = dVdx + (size_t)e * ldS * ns;
  double Minv[NJ > 0 ? M * M : 1];
  if constexpr (NJ > 0) {
    // prismatic chain (the launcher sends only constant-M chains here): M^-1 once per episode
    double Mm[M * M], q[NJ];
#pragma unroll
    for (int i = 0; i < NJ; ++i) q[i] = Se[i];
    chain_mass<NJ>(sd, q, Mm);
    small_inverse<M>(Mm, Minv);
  }
  double w_run[7], w_term[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    w_run[k] = p.w_running[k];
    w_term[k] = p.w_terminal[k];
  }
  double Vx[N], Vxx[N * N], x[N];
#pragma unroll
  for (int k = 0; k < N; ++k) x[k] = Se[(size_t)Te * ns + k];
  ddp_lx<NJ>(sd, w_term, x, Vx, Vxx);
#pragma unroll
  for (int k = 0; k < N; ++k) Oe[(size_t)Te * ns + k] = Vx[k];
  Oe[(size_t)Te * ns + N] = 0.0;
  for (int i = Te - 1; i >= 0; --i) {
    double u[M], A[N * N], B[N * M], lx[N], lxx[N * N];
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = Se[(size_t)i * ns + k];
#pragma unroll
    for (int k = 0; k < M; ++k) u[k] = Ue[(size_t)i * na + k];
    ddp_jacobians<NJ>(sd, x, Minv, A, B);
    ddp_lx<NJ>(sd, w_run, x, lx, lxx);
    // Q_x = l_x + A^T V_x, Q_u = l_u + B^T V_x
    double Qx[N], Qu[M], Qxx[N * N], Quu[M * M], Qxu[N * M], VA[N * N], VB[N * M];
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < N; ++k)
        if (a_nz<NJ>(k, r)) s += A[k * N + r] * Vx[k];
      Qx[r] = lx[r] + s;
    }
#pragma unroll
    for (int j = 0; j < M; ++j) {
      // l_u, l_uu: - w6 * (u^2 + w_b (u / u_max)^10) (bound_control_cost, environment_TO.py:201-206)
      const double um = p.u_max[j];
      const double lu = p.scale * (-w_run[6] * (2.0 * u[j] + p.w_b * 10.0 * pow(u[j] / um, 9.0) / um));
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < N; ++k)
        if (b_nz<NJ>(k, j)) s += B[k * M + j] * Vx[k];
      Qu[j] = lu + s;
    }
    // V_xx A, V_xx B
#pragma unroll
    for (int r = 0; r < N; ++r) {
#pragma unroll
      for (int c = 0; c < N; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (a_nz<NJ>(k, c)) s += Vxx[r * N + k] * A[k * N + c];
        VA[r * N + c] = s;
      }
#pragma unroll
      for (int c = 0; c < M; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (b_nz<NJ>(k, c)) s += Vxx[r * N + k] * B[k * M + c];
        VB[r * M + c] = s;
      }
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
#pragma unroll
      for (int c = 0; c < N; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (a_nz<NJ>(k, r)) s += A[k * N + r] * VA[k * N + c];
        Qxx[r * N + c] = lxx[r * N + c] + s;
      }
#pragma unroll
      for (int c = 0; c < M; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (a_nz<NJ>(k, r)) s += A[k * N + r] * VB[k * M + c];
        Qxu[r * M + c] = s;  // + l_xu = 0
      }
    }
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int c = 0; c < M; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (b_nz<NJ>(k, r)) s += B[k * M + r] * VB[k * M + c];
        const double um = p.u_max[r];
        const double luu = r == c ? p.scale * (-w_run[6] * (2.0 + p.w_b * 90.0 * pow(u[r] / um, 8.0) / (um * um))) : 0.0;
        Quu[r * M + c] = luu + s + (r == c ? mu : 0.0);
      }
    double Qi[M * M];
    small_inverse<M>(Quu, Qi);
    // K = Qbar^-1 Q_xu^T [M x N], k = Qbar^-1 Q_u [M]
    double Kk[M];
#pragma unroll
    for (int r = 0; r < M; ++r) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < M; ++k) s += Qi[r * M + k] * Qu[k];
      Kk[r] = s;
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < M; ++k) s += Qxu[r * M + k] * Kk[k];
      Vx[r] = Qx[r] - s;
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double QK[M];  // row r of Q_xu Qbar^-1
#pragma unroll
      for (int c = 0; c < M; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) s += Qxu[r * M + k] * Qi[k * M + c];
        QK[c] = s;
      }
#pragma unroll
      for (int c = 0; c < N; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) s += QK[k] * Qxu[c * M + k];
        Vxx[r * N + c] = Qxx[r * N + c] - s;
      }
    }
#pragma unroll
    for (int k = 0; k < N; ++k) Oe[(size_t)i * ns + k] = Vx[k];
    Oe[(size_t)i * ns + N] = 0.0;
  }
}

// The Riccati recursion of the split pass with one wavefront per episode: the lanes share each
// step's matrix products (outputs spread over lanes, operands in LDS), so the N = 12 recursion of
// UR5 is ~N^3 / 64 dependent FMAs per product instead of N^3 on one thread. Same products, same
// summation order as k_ddp_backward; Qbar_uu^-1 (M x M) on lane 0.
template <int NJ>
__global__ void __launch_bounds__(64) k_ddp_riccati_wave(const SysDevice* __restrict__ sdp,
                                                         const double* __restrict__ U, int64_t ldU,
                                                         const int32_t* __restrict__ nsteps, int n_ep, double mu,
                                                         const double* __restrict__ ws, int64_t ldS,
                                                         double* __restrict__ dVdx) {
  using RC = DdpRec<NJ>;
  constexpr int N = RC::N, M = RC::M, ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  __shared__ double sA[N * N], sB[N * M], sLx[N], sLxx[N * N], sVx[N], sVxx[N * N], sU[M];
  __shared__ double sVA[N * N], sVB[N * M], sQx[N], sQu[M], sQxx[N * N], sQxu[N * M], sQuu[M * M], sQi[M * M];
  __shared__ double sK[M], sQK[N * M];
  const int e = blockIdx.x, lane = threadIdx.x;
  const cacto_sys_params& p = sdp->p;
  const double w6 = p.w_running[6];
  const int Te = nsteps[e];
  if (Te < 0) return;  // a dropped episode (main.py:236): no labels (uniform over the workgroup)
  double* Oe = dVdx + (size_t)e * ldS * ns;
  const double* Ue = U + (size_t)e * ldU * na;
  {
    const double* rec = ws + (size_t)Te * RC::R * n_ep + e;
    for (int k = lane; k < N; k += 64) sVx[k] = rec[(size_t)(RC::LX + k) * n_ep];
    for (int k = lane; k < N * N; k += 64) sVxx[k] = rec[(size_t)(RC::LXX + k) * n_ep];
  }
  __syncthreads();
  for (int k = lane; k <= N; k += 64) Oe[(size_t)Te * ns + k] = k < N ? sVx[k] : 0.0;
  for (int i = Te - 1; i >= 0; --i) {
    const double* rec = ws + (size_t)i * RC::R * n_ep + e;
    for (int k = lane; k < N * N; k += 64) {
      sA[k] = rec[(size_t)(RC::A + k) * n_ep];
      sLxx[k] = rec[(size_t)(RC::LXX + k) * n_ep];
    }
    for (int k = lane; k < N * M; k += 64) sB[k] = rec[(size_t)(RC::B + k) * n_ep];
    for (int k = lane; k < N; k += 64) sLx[k] = rec[(size_t)(RC::LX + k) * n_ep];
    for (int k = lane; k < M; k += 64) sU[k] = Ue[(size_t)i * na + k];
    __syncthreads();
    // V_xx A, V_xx B, Q_x = l_x + A^T V_x, Q_u = l_u + B^T V_x
    for (int o = lane; o < N * N + N * M + N + M; o += 64) {
      double s = 0.0;
      if (o < N * N) {
        const int r = o / N, c = o - r * N;
#pragma unroll
        for (int k = 0; k < N; ++k) s += sVxx[r * N + k] * sA[k * N + c];
        sVA[o] = s;
      } else if (o < N * N + N * M) {
        const int q = o - N * N, r = q / M, c = q - r * M;
#pragma unroll
        for (int k = 0; k < N; ++k) s += sVxx[r * N + k] * sB[k * M + c];
        sVB[q] = s;
      } else if (o < N * N + N * M + N) {
        const int r = o - N * N - N * M;
#pragma unroll
        for (int k = 0; k < N; ++k) s += sA[k * N + r] * sVx[k];
        sQx[r] = sLx[r] + s;
      } else {
        const int j = o - N * N - N * M - N;
        const double um = p.u_max[j], u = sU[j];
        const double lu = p.scale * (-w6 * (2.0 * u + p.w_b * 10.0 * pow(u / um, 9.0) / um));
#pragma unroll
        for (int k = 0; k < N; ++k) s += sB[k * M + j] * sVx[k];
        sQu[j] = lu + s;
      }
    }
    __syncthreads();
    // Q_xx = l_xx + A^T V_xx A, Q_xu = A^T V_xx B, Qbar_uu = l_uu + B^T V_xx B + mu I
    for (int o = lane; o < N * N + N * M + M * M; o += 64) {
      double s = 0.0;
      if (o < N * N) {
        const int r = o / N, c = o - r * N;
#pragma unroll
        for (int k = 0; k < N; ++k) s += sA[k * N + r] * sVA[k * N + c];
        sQxx[o] = sLxx[o] + s;
      } else if (o < N * N + N * M) {
        const int q = o - N * N, r = q / M, c = q - r * M;
#pragma unroll
        for (int k = 0; k < N; ++k) s += sA[k * N + r] * sVB[k * M + c];
        sQxu[q] = s;
      } else {
        const int q = o - N * N - N * M, r = q / M, c = q - r * M;
#pragma unroll
        for (int k = 0; k < N; ++k) s += sB[k * M + r] * sVB[k * M + c];
        const double um = p.u_max[r];
        const double luu =
            r == c ? p.scale * (-w6 * (2.0 + p.w_b * 90.0 * pow(sU[r] / um, 8.0) / (um * um))) : 0.0;
        sQuu[q] = luu + s + (r == c ? mu : 0.0);
      }
    }
    __syncthreads();
    if (lane == 0) {
      double a[M * M], inv[M * M];
#pragma unroll
      for (int k = 0; k < M * M; ++k) a[k] = sQuu[k];
      small_inverse<M>(a, inv);
#pragma unroll
      for (int r = 0; r < M; ++r) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) s += inv[r * M + k] * sQu[k];
        sK[r] = s;
      }
#pragma unroll
      for (int k = 0; k < M * M; ++k) sQi[k] = inv[k];
    }
    __syncthreads();
    // V_x = Q_x - Q_xu (Qbar^-1 Q_u); row r of Q_xu Qbar^-1
    for (int o = lane; o < N + N * M; o += 64) {
      double s = 0.0;
      if (o < N) {
#pragma unroll
        for (int k = 0; k < M; ++k) s += sQxu[o * M + k] * sK[k];
        sVx[o] = sQx[o] - s;
      } else {
        const int q = o - N, r = q / M, c = q - r * M;
#pragma unroll
        for (int k = 0; k < M; ++k) s += sQxu[r * M + k] * sQi[k * M + c];
        sQK[q] = s;
      }
    }
    __syncthreads();
    // V_xx = Q_xx - (Q_xu Qbar^-1) Q_xu^T
    for (int o = lane; o < N * N; o += 64) {
      const int r = o / N, c = o - r * N;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < M; ++k) s += sQK[r * M + k] * sQxu[c * M + k];
      sVxx[o] = sQxx[o] - s;
    }
    for (int k = lane; k <= N; k += 64) Oe[(size_t)i * ns + k] = k < N ? sVx[k] : 0.0;
    __syncthreads();
  }
}

}  // namespace cacto

using namespace cacto;

namespace {
// Grow-only device workspace of the split pass, owned by the system handle (freed by
// cacto_sys_destroy). Growing frees the old block (hipFree synchronises the device).
int ddp_workspace(cacto_sys* sys, size_t bytes, double** out) {
  if (bytes > sys->ddp_ws_bytes) {
    if (sys->ddp_ws) CACTO_CHECK_HIP(hipFree(sys->ddp_ws));
    sys->ddp_ws = nullptr;
    sys->ddp_ws_bytes = 0;
    CACTO_CHECK_HIP(hipMalloc(&sys->ddp_ws, bytes));
    sys->ddp_ws_bytes = bytes;
  }
  *out = static_cast<double*>(sys->ddp_ws);
  return CACTO_OK;
}

template <int NJ>
struct LaunchDdp {
  static int run(const cacto_sys* sys, const double* S, int64_t ldS, const double* U, int64_t ldU, const int32_t* n,
                 int n_ep, double mu, double* out, hipStream_t st) {
    if constexpr (!DdpDims<NJ>::ok) {
      set_error("cacto_ddp_backward: supported for the single integrator, car and prismatic chains (double integrator)");
      return CACTO_EUNSUPPORTED;
    } else {
      const int rk = sys->host.p.reward_kind;
      const bool rk_ok = NJ == -2 ? rk == CACTO_REW_CAR_PARK
                                  : NJ > 0 ? (sys->host.p.const_dyn ? rk == CACTO_REW_PLANAR
                                                                   : rk == CACTO_REW_MANIPULATOR || rk == CACTO_REW_UR5)
                                           : rk == CACTO_REW_PLANAR;
      // chains: the DI's prismatic pair (constant M) or revolute chains of 3 / 6 joints
      if (!rk_ok || (NJ > 0 && (sys->host.p.const_dyn ? NJ != 2 : NJ == 2))) {
        set_error("cacto_ddp_backward: unsupported (dynamics, reward) combination");
        return CACTO_EUNSUPPORTED;
      }
      if constexpr (NJ > 2 || NJ == -2) {
        // split pass: per-step derivatives over (episode, step), then the recursion
        using RC = DdpRec<NJ>;
        double* ws = nullptr;
        const int rc = ddp_workspace(const_cast<cacto_sys*>(sys), (size_t)ldS * RC::R * n_ep * sizeof(double), &ws);
        if (rc != CACTO_OK) return rc;
        // revolute chains: primal / per-direction tangent / cost-derivative kernels (CACTO_DDP_SPLIT=0:
        // the one-thread-per-step k_ddp_derivs)
        static const char* split_env = std::getenv("CACTO_DDP_SPLIT");
        const bool split = NJ > 2 && !(split_env && split_env[0] == '0');
        if constexpr (NJ > 2) {
          if (split) {
            using PC = DdpPrim<NJ>;
            double* pw = nullptr;
            const size_t rec_bytes = (size_t)ldS * RC::R * n_ep * sizeof(double);
            const int rc2 = ddp_workspace(const_cast<cacto_sys*>(sys), rec_bytes + (size_t)ldS * PC::R * n_ep * sizeof(double),
                                          &ws);
            if (rc2 != CACTO_OK) return rc2;
            pw = ws + (size_t)ldS * RC::R * n_ep;
            const dim3 g(ceil_div(n_ep, 64), (unsigned)ldS);
            hipLaunchKernelGGL(k_ddp_prim<NJ>, g, dim3(64), 0, st, sys->dev, S, ldS, U, ldU, n, n_ep, ws, pw);
            CACTO_CHECK_HIP(hipGetLastError());
            hipLaunchKernelGGL(k_ddp_lx<NJ>, g, dim3(64), 0, st, sys->dev, S, ldS, n, n_ep, ws);
            CACTO_CHECK_HIP(hipGetLastError());
            hipLaunchKernelGGL(k_ddp_tan<NJ>, dim3(g.x, g.y, 2 * NJ), dim3(64), 0, st, sys->dev, S, ldS, n, n_ep, ws, pw);
          }
        }
        if (!split)
          hipLaunchKernelGGL(k_ddp_derivs<NJ>, dim3(ceil_div(n_ep, 64), (unsigned)ldS), dim3(64), 0, st, sys->dev, S,
                             ldS, U, ldU, n, n_ep, ws);
        CACTO_CHECK_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_ddp_riccati_wave<NJ>, dim3(n_ep), dim3(64), 0, st, sys->dev, U, ldU, n, n_ep, mu, ws,
                           ldS, out);
      } else {
        hipLaunchKernelGGL(k_ddp_backward<NJ>, dim3(ceil_div(n_ep, 64)), dim3(64), 0, st, sys->dev, S, ldS, U, ldU,
                           n, n_ep, mu, out);
      }
      CACTO_CHECK_HIP(hipGetLastError());
      return CACTO_OK;
    }
  }
};
template <int NJ>
struct LaunchJac {
  static int run(const cacto_sys* sys, const double* S, const double* U, int B, double* Fx, double* Fu,
                 hipStream_t st) {
    if constexpr (!DdpDims<NJ>::ok) {
      set_error("cacto_env_jacobians: unsupported dynamics");
      return CACTO_EUNSUPPORTED;
    } else {
      if (NJ == 2 && !sys->host.p.const_dyn) {
        set_error("cacto_env_jacobians: 2-joint chains are instantiated for the prismatic pair (double integrator)");
        return CACTO_EUNSUPPORTED;
      }
      if constexpr (NJ > 2) {
        using RC = DdpRec<NJ>;
        using PC = DdpPrim<NJ>;
        constexpr int ns = Dims<NJ>::NS;
        // step 0 of B one-step episodes: only A, B are read, so no l_x kernel
        const size_t rec = (size_t)2 * RC::R * B, pwn = (size_t)PC::R * B, s2 = (size_t)2 * B * ns;
        double* ws = nullptr;
        const int rc = ddp_workspace(const_cast<cacto_sys*>(sys), (rec + pwn + s2 + B) * sizeof(double), &ws);
        if (rc != CACTO_OK) return rc;
        double* pw = ws + rec;
        double* S2 = pw + pwn;
        int32_t* n1 = reinterpret_cast<int32_t*>(S2 + s2);
        hipLaunchKernelGGL(k_jac_prep<NJ>, dim3(ceil_div(B * 2 * ns, 256)), dim3(256), 0, st, S, B, S2, n1);
        CACTO_CHECK_HIP(hipGetLastError());
        const dim3 g(ceil_div(B, 64), 1);
        hipLaunchKernelGGL(k_ddp_prim<NJ>, g, dim3(64), 0, st, sys->dev, S2, (int64_t)2, U, (int64_t)1, n1, B, ws, pw);
        CACTO_CHECK_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_ddp_tan<NJ>, dim3(g.x, 1, 2 * NJ), dim3(64), 0, st, sys->dev, S2, (int64_t)2, n1, B, ws,
                           pw);
        CACTO_CHECK_HIP(hipGetLastError());
        constexpr int per = RC::N * RC::N + RC::N * RC::M;
        hipLaunchKernelGGL(k_jac_extract<NJ>, dim3(ceil_div(B * per, 256)), dim3(256), 0, st, ws, B, Fx, Fu);
      } else {
        hipLaunchKernelGGL(k_env_jacobians<NJ>, dim3(ceil_div(B, 64)), dim3(64), 0, st, sys->dev, S, U, B, Fx, Fu);
      }
      CACTO_CHECK_HIP(hipGetLastError());
      return CACTO_OK;
    }
  }
};
}  // namespace

extern "C" int cacto_ddp_backward(const cacto_sys* sys, const double* S_traj_d, int64_t ldS, const double* U_traj_d,
                                  int64_t ldU, const int32_t* nsteps_d, int n_ep, double mu, double* dVdx_d,
                                  void* stream) {
  CACTO_REQUIRE(sys && S_traj_d && U_traj_d && nsteps_d && dVdx_d && n_ep >= 0 && ldS >= 1 && ldU >= 0,
                "cacto_ddp_backward: bad arguments");
  if (n_ep == 0) return CACTO_OK;
  return dispatch_nj<LaunchDdp>(sys->host.p, sys, S_traj_d, ldS, U_traj_d, ldU, nsteps_d, n_ep, mu, dVdx_d,
                                as_stream(stream));
}

extern "C" int cacto_env_jacobians(const cacto_sys* sys, const double* S_d, const double* A_d, int B, double* Fx_d,
                                   double* Fu_d, void* stream) {
  CACTO_REQUIRE(sys && S_d && A_d && Fx_d && Fu_d && B >= 0, "cacto_env_jacobians: bad arguments");
  if (B == 0) return CACTO_OK;
  return dispatch_nj<LaunchJac>(sys->host.p, sys, S_d, A_d, B, Fx_d, Fu_d, as_stream(stream));
}
