// Batched environment kernels (one thread per sample, float64 dynamics) and replay-buffer
// gather/add (coalesced row copies).
#include "internal.h"

namespace cacto {

// compute_actor_grad's env calls: simulate_batch, derivative_batch, reward_batch, dr/da.
template <int NJ>
__global__ void __launch_bounds__(256) k_env_step_batch(const SysDevice* __restrict__ sdp,
                                                        const float* __restrict__ S, const float* __restrict__ A,
                                                        const double* __restrict__ term,
                                                        const double* __restrict__ Wb, float* __restrict__ Sn,
                                                        float* __restrict__ Fu, float* __restrict__ R,
                                                        float* __restrict__ dR, int B) {
  constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  const SysDevice& sd = *sdp;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double s[ns], a[na], out[ns];
  float af[na];
#pragma unroll
  for (int i = 0; i < ns; ++i) s[i] = (double)S[(size_t)b * ns + i];
#pragma unroll
  for (int i = 0; i < na; ++i) {
    af[i] = A[(size_t)b * na + i];
    a[i] = (double)af[i];
  }
  if (Sn) {
    env_simulate<NJ>(sd, s, a, true, out);
#pragma unroll
    for (int i = 0; i < ns; ++i) Sn[(size_t)b * ns + i] = (float)out[i];
  }
  if (Fu) {
    double F[ns * na];
    env_derivative<NJ>(sd, s, F);
#pragma unroll
    for (int k = 0; k < ns * na; ++k) Fu[(size_t)b * ns * na + k] = (float)F[k];
  }
  if (R || dR) {
    const double t = term ? term[b] : 0.0;
    double w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      w[k] = k >= sd.p.n_weights ? 0.0
             : Wb ? Wb[(size_t)b * sd.p.n_weights + k] : t * sd.p.w_terminal[k] + (1.0 - t) * sd.p.w_running[k];
    const double partial = env_reward<NJ>(sd, w, s, nullptr, true);
    float g[na];
    const float r = reward_batch_f32<na>(sd.p, w[6], af, partial, g);
    if (R) R[b] = r;
    if (dR)
#pragma unroll
      for (int i = 0; i < na; ++i) dR[(size_t)b * na + i] = g[i];
  }
}

// Env.step (float64) + EE of the next state.
template <int NJ>
__global__ void __launch_bounds__(256) k_env_step(const SysDevice* __restrict__ sdp, const double* __restrict__ S,
                                                  const double* __restrict__ A, const double* __restrict__ W,
                                                  double* __restrict__ Sn, double* __restrict__ R,
                                                  double* __restrict__ EE, int B) {
  constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  const SysDevice& sd = *sdp;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double s[ns], a[na], out[ns], w[8];
#pragma unroll
  for (int i = 0; i < ns; ++i) s[i] = S[(size_t)b * ns + i];
#pragma unroll
  for (int i = 0; i < na; ++i) a[i] = A[(size_t)b * na + i];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = k >= sd.p.n_weights ? 0.0 : W ? W[k] : sd.p.w_running[k];
  env_simulate<NJ>(sd, s, a, false, out);
  if (Sn)
#pragma unroll
    for (int i = 0; i < ns; ++i) Sn[(size_t)b * ns + i] = out[i];
  if (R) R[b] = env_reward<NJ>(sd, w, s, a, false);
  if (EE) {
    V3 e = env_ee<NJ>(sd, out);
    EE[(size_t)b * 3 + 0] = e.x;
    EE[(size_t)b * 3 + 1] = e.y;
    EE[(size_t)b * 3 + 2] = e.z;
  }
}

// Env.bound_control_cost (environment.py:158-163) for B action rows (float64, action order).
template <int NJ>
__global__ void __launch_bounds__(256) k_env_bound_cost(const SysDevice* __restrict__ sdp,
                                                        const double* __restrict__ A, double* __restrict__ out,
                                                        int B) {
  constexpr int na = Dims<NJ>::NA;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double a[na];
#pragma unroll
  for (int i = 0; i < na; ++i) a[i] = A[(size_t)b * na + i];
  out[b] = bound_control_cost<na>(sdp->p, a);
}

template <int NJ>
__global__ void __launch_bounds__(256) k_env_ee(const SysDevice* __restrict__ sdp, const double* __restrict__ S,
                                                double* __restrict__ EE, int B) {
  constexpr int ns = Dims<NJ>::NS;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double s[ns];
#pragma unroll
  for (int i = 0; i < ns; ++i) s[i] = S[(size_t)b * ns + i];
  const V3 e = env_ee<NJ>(*sdp, s);
  EE[(size_t)b * 3 + 0] = e.x;
  EE[(size_t)b * 3 + 1] = e.y;
  EE[(size_t)b * 3 + 2] = e.z;
}

__global__ void k_buffer_add(double* __restrict__ storage, int64_t capacity, int64_t next_idx, int cols,
                             const double* __restrict__ rows, int64_t n) {
  const int64_t total = n * cols;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = k / cols, c = k - r * cols;
    storage[((next_idx + r) % capacity) * cols + c] = rows[k];
  }
}

// RL_AC.RL_Solve (RL.py:145-189) for a batch of episodes, fused with the ring write of
// ReplayBuffer.add (replay_buffer.py:25-36) that main.py:240 applies to its output. One workgroup
// per episode. Python's sum() over a float64 slice adds left to right starting from integer 0, so
// acc = 0.0 followed by the same additions reproduces it bit for bit (0 + -0.0 == +0.0 in both);
// the total reward-to-go continues the partial sum's additions before either is rounded to f32.
__global__ void k_rl_solve_add(const double* __restrict__ S, int64_t ldS, const double* __restrict__ R, int64_t ldR,
                               const double* __restrict__ R_term, const double* __restrict__ dVdx,
                               const int64_t* __restrict__ row_off, int ns, int max_T, int nTD, int mc,
                               double* __restrict__ storage, int64_t capacity, int64_t next_idx,
                               double* __restrict__ total_out) {
  extern __shared__ double sm[];
  double* r = sm;                  // rwrd_arr of this episode, [Te+1]
  double* part = sm + max_T + 1;   // partial_reward_to_go_arr, [Te+1]
  const int e = blockIdx.x;
  const int64_t off = row_off[e];
  const int Te = (int)(row_off[e + 1] - off) - 1;  // NSTEPS_SH of this episode
  if (Te < 0 || Te > max_T) return;                // violates the documented precondition: write nothing
  for (int t = threadIdx.x; t <= Te; t += blockDim.x)
    r[t] = (t == Te && R_term) ? R_term[e] : R[e * ldR + t];
  __syncthreads();
  for (int i = threadIdx.x; i <= Te; i += blockDim.x) {
    const int fin = mc ? Te : min(i + nTD, Te);
    double acc = 0.0;
    for (int t = i; t <= fin; ++t) acc += r[t];
    part[i] = (double)(float)acc;
    if (total_out) {
      for (int t = fin + 1; t <= Te; ++t) acc += r[t];
      total_out[e * ldS + i] = (double)(float)acc;
    }
  }
  __syncthreads();
  const double* Se = S + e * ldS * ns;
  const double* De = dVdx ? dVdx + e * ldS * ns : nullptr;
  const int cols = 3 * ns + 3;
  const int64_t n = (int64_t)(Te + 1) * cols;
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
    const int i = (int)(k / cols), c = (int)(k - (int64_t)i * cols);
    const int fin = mc ? Te : min(i + nTD, Te);
    const bool done = mc || fin == Te;
    double v;
    if (c < ns) v = Se[i * ns + c];
    else if (c == ns) v = part[i];
    else if (c <= 2 * ns) v = done ? 0.0 : Se[(fin + 1) * ns + (c - ns - 1)];
    else if (c <= 3 * ns) v = De ? De[i * ns + (c - 2 * ns - 1)] : 0.0;
    else if (c == 3 * ns + 1) v = done ? 1.0 : 0.0;
    else v = i == Te ? 1.0 : 0.0;
    storage[((next_idx + off + i) % capacity) * cols + c] = v;
  }
}

__global__ void k_buffer_gather(const double* __restrict__ storage, int ns, const int32_t* __restrict__ idx, int B,
                                float* __restrict__ S, float* __restrict__ R, float* __restrict__ Sn,
                                float* __restrict__ dVdx, float* __restrict__ d, double* __restrict__ term) {
  const int cols = 3 * ns + 3;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= B * cols) return;
  const int b = k / cols, c = k - b * cols;
  const double v = storage[(size_t)idx[b] * cols + c];
  if (c < ns) {
    if (S) S[b * ns + c] = (float)v;
  } else if (c == ns) {
    if (R) R[b] = (float)v;
  } else if (c < 2 * ns + 1) {
    if (Sn) Sn[b * ns + (c - ns - 1)] = (float)v;
  } else if (c < 3 * ns + 1) {
    if (dVdx) dVdx[b * ns + (c - 2 * ns - 1)] = (float)v;
  } else if (c == 3 * ns + 1) {
    if (d) d[b] = (float)v;
  } else {
    if (term) term[b] = v;
  }
}

// The tabled constants of a prismatic-only chain (SysDevice::cd_*), one thread, at system creation:
// chain_terms / cholesky / the per-sample derivative path evaluated once (at q = v = 0; M and h do
// not depend on them for such chains, which the rollout's per-episode factor relies on as well).
template <int NJ>
__global__ void k_const_dyn_init(SysDevice* sd) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if constexpr (NJ > 0) {
    constexpr int NS = 2 * NJ + 1, NA = NJ;
    double s[NS], a[NA], out[NS], Fu[NS * NA], M[NJ * NJ], h[NJ];
#pragma unroll
    for (int i = 0; i < NS; ++i) s[i] = 0.0;
#pragma unroll
    for (int i = 0; i < NA; ++i) a[i] = 0.0;
    chain_terms<NJ>(*sd, s, s + NJ, M, h);
    cholesky<NJ>(M);
#pragma unroll
    for (int k = 0; k < NJ * NJ; ++k) sd->cd_L[k] = M[k];
#pragma unroll
    for (int i = 0; i < NJ; ++i) sd->cd_h[i] = h[i];
    env_simulate_derivative<NJ>(*sd, s, a, false, out, Fu);
#pragma unroll
    for (int k = 0; k < NS * NA; ++k) sd->cd_Fu[k] = Fu[k];
  }
}

}  // namespace cacto

using namespace cacto;

namespace {
template <int NJ>
struct LaunchStepBatch {
  static int run(const cacto_sys* sys, const float* S, const float* A, const double* term, const double* W, float* Sn,
                 float* Fu, float* R, float* dR, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_env_step_batch<NJ>, dim3(ceil_div(B, 256)), dim3(256), 0, st, sys->dev, S, A, term, W, Sn,
                       Fu, R, dR, B);
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
};
template <int NJ>
struct LaunchStep {
  static int run(const cacto_sys* sys, const double* S, const double* A, const double* W, double* Sn, double* R,
                 double* EE, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_env_step<NJ>, dim3(ceil_div(B, 256)), dim3(256), 0, st, sys->dev, S, A, W, Sn, R, EE, B);
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
};
template <int NJ>
struct LaunchBoundCost {
  static int run(const cacto_sys* sys, const double* A, double* out, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_env_bound_cost<NJ>, dim3(ceil_div(B, 256)), dim3(256), 0, st, sys->dev, A, out, B);
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
};
template <int NJ>
struct LaunchEE {
  static int run(const cacto_sys* sys, const double* S, double* EE, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_env_ee<NJ>, dim3(ceil_div(B, 256)), dim3(256), 0, st, sys->dev, S, EE, B);
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
};
}  // namespace

extern "C" int cacto_env_step_batch(const cacto_sys* sys, const float* S_d, const float* A_d, const double* term_d,
                                    const double* W_d, float* S_next_d, float* Fu_d, float* R_d, float* dR_dA_d, int B,
                                    void* stream) {
  CACTO_REQUIRE(sys && S_d && A_d && B >= 0, "cacto_env_step_batch: bad arguments");
  if (B == 0) return CACTO_OK;
  return dispatch_nj<LaunchStepBatch>(sys->host.p, sys, S_d, A_d, term_d, W_d, S_next_d, Fu_d, R_d, dR_dA_d, B,
                                      as_stream(stream));
}

extern "C" int cacto_env_step(const cacto_sys* sys, const double* S_d, const double* A_d, const double* W_d,
                              double* S_next_d, double* R_d, double* EE_d, int B, void* stream) {
  CACTO_REQUIRE(sys && S_d && A_d && B >= 0, "cacto_env_step: bad arguments");
  if (B == 0) return CACTO_OK;
  return dispatch_nj<LaunchStep>(sys->host.p, sys, S_d, A_d, W_d, S_next_d, R_d, EE_d, B, as_stream(stream));
}

extern "C" int cacto_env_ee(const cacto_sys* sys, const double* S_d, double* EE_d, int B, void* stream) {
  CACTO_REQUIRE(sys && S_d && EE_d && B >= 0, "cacto_env_ee: bad arguments");
  if (B == 0) return CACTO_OK;
  return dispatch_nj<LaunchEE>(sys->host.p, sys, S_d, EE_d, B, as_stream(stream));
}

extern "C" int cacto_env_bound_control_cost(const cacto_sys* sys, const double* A_d, double* out_d, int B,
                                            void* stream) {
  CACTO_REQUIRE(sys && A_d && out_d && B >= 0, "cacto_env_bound_control_cost: bad arguments");
  if (B == 0) return CACTO_OK;
  return dispatch_nj<LaunchBoundCost>(sys->host.p, sys, A_d, out_d, B, as_stream(stream));
}

extern "C" int cacto_buffer_add(const cacto_sys* sys, double* storage_d, int64_t capacity, int64_t next_idx,
                                const double* rows_d, int64_t n, void* stream) {
  CACTO_REQUIRE(sys && storage_d && rows_d && capacity > 0 && n >= 0 && next_idx >= 0 && next_idx < capacity,
                "cacto_buffer_add: bad arguments");
  CACTO_REQUIRE(n <= capacity, "cacto_buffer_add: more rows than capacity");
  if (n == 0) return CACTO_OK;
  const int cols = 3 * sys->host.p.nb_state + 3;
  const int64_t total = n * cols;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(k_buffer_add, dim3(grid), dim3(256), 0, as_stream(stream), storage_d, capacity, next_idx, cols,
                     rows_d, n);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

extern "C" int cacto_rl_solve_add(const cacto_sys* sys, const double* S_traj_d, int64_t ldS, const double* R_d,
                                  int64_t ldR, const double* R_term_d, const double* dVdx_d, const int64_t* row_off_d,
                                  int n_ep, int max_T, int64_t total_rows, int nsteps_td, int mc, double* storage_d,
                                  int64_t capacity, int64_t next_idx, double* total_d, void* stream) {
  CACTO_REQUIRE(sys && S_traj_d && R_d && row_off_d && storage_d && n_ep >= 0 && max_T >= 0 && nsteps_td >= 0 &&
                    capacity > 0 && next_idx >= 0 && next_idx < capacity && total_rows >= 0,
                "cacto_rl_solve_add: bad arguments");
  CACTO_REQUIRE(ldS >= max_T + 1 && ldR >= (R_term_d ? max_T : max_T + 1),
                "cacto_rl_solve_add: trajectory strides shorter than max_T");
  CACTO_REQUIRE(max_T + 1 <= 4096, "cacto_rl_solve_add: episodes longer than 4095 steps");
  CACTO_REQUIRE(total_rows <= capacity, "cacto_rl_solve_add: more rows than capacity");
  if (n_ep == 0 || total_rows == 0) return CACTO_OK;
  const size_t smem = 2 * (size_t)(max_T + 1) * sizeof(double);
  hipLaunchKernelGGL(k_rl_solve_add, dim3(n_ep), dim3(256), smem, as_stream(stream), S_traj_d, ldS, R_d, ldR,
                     R_term_d, dVdx_d, row_off_d, sys->host.p.nb_state, max_T, nsteps_td, mc, storage_d, capacity,
                     next_idx, total_d);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

extern "C" int cacto_buffer_gather(const cacto_sys* sys, const double* storage_d, const int32_t* idx_d, int B,
                                   float* S_d, float* R_d, float* S_next_d, float* dVdx_d, float* d_d, double* term_d,
                                   void* stream) {
  CACTO_REQUIRE(sys && storage_d && idx_d && B >= 0, "cacto_buffer_gather: bad arguments");
  if (B == 0) return CACTO_OK;
  const int ns = sys->host.p.nb_state;
  const int total = B * (3 * ns + 3);
  hipLaunchKernelGGL(k_buffer_gather, dim3(ceil_div(total, 256)), dim3(256), 0, as_stream(stream), storage_d, ns,
                     idx_d, B, S_d, R_d, S_next_d, dVdx_d, d_d, term_d);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

namespace {
template <int NJ>
struct LaunchConstDyn {
  static int run(cacto_sys* sys) {
    hipLaunchKernelGGL(k_const_dyn_init<NJ>, dim3(1), dim3(64), 0, 0, sys->dev);
    CACTO_CHECK_HIP(hipGetLastError());
    CACTO_CHECK_HIP(hipDeviceSynchronize());
    return CACTO_OK;
  }
};
}  // namespace

int cacto_const_dyn_init(cacto_sys* sys) {
  if (!sys->host.p.const_dyn) return CACTO_OK;
  return dispatch_nj<LaunchConstDyn>(sys->host.p, sys);
}
