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
