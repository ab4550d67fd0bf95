// Shared helpers for the CACTO gfx950 kernels: error plumbing, MFMA fragment types, exact-rounding
// float32 arithmetic (the reference's TF ops are separate kernels, so no FMA contraction).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/cacto_hip.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define CACTO_WAVE 64
#define CACTO_NWAVES 4                 // waves per workgroup in the tile kernels
#define CACTO_THREADS (CACTO_WAVE * CACTO_NWAVES)
#define CACTO_TILE 16                  // samples per workgroup tile (MFMA 16x16x4 N dimension)

#ifdef CACTO_STAMPS
__shared__ unsigned long long cacto_stamp_s[32];  // per-workgroup phase stamps (diagnostic builds)
#define PSTAMP(k)                                                                 \
  do {                                                                            \
    if (threadIdx.x == 0) cacto_stamp_s[k] = __builtin_amdgcn_s_memtime();       \
  } while (0)
#else
#define PSTAMP(k) \
  do {            \
  } while (0)
#endif

namespace cacto {

void set_error(const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define CACTO_CHECK_HIP(expr)                                  \
  do {                                                         \
    hipError_t _e = (expr);                                    \
    if (_e != hipSuccess) return ::cacto::hip_fail(_e, #expr); \
  } while (0)

#define CACTO_REQUIRE(cond, msg)          \
  do {                                    \
    if (!(cond)) {                        \
      ::cacto::set_error(msg);            \
      return CACTO_EINVAL;                \
    }                                     \
  } while (0)

// f32 ops that must not be contracted into FMAs (each TF op rounds separately).
__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return __fsub_rn(a, b); }

// The sine-elu critic's elu layers (critic_type 'sine-elu', NeuralNetwork.py:80-93): tf.nn.elu
// (features < 0 ? exp(features) - 1 : features) and the factor EluGrad applies to the upstream
// gradient (activations < 0 ? activations + 1 : 1) — the (h, c) pair a sine layer gives as
// (sin z, cos z).
__device__ __forceinline__ void elu_pair(float z, float* h, float* c) {
  const float y = z < 0.f ? __fsub_rn(expf(z), 1.f) : z;
  *h = y;
  *c = y < 0.f ? __fadd_rn(y, 1.f) : 1.f;
}
// The second derivative of a hidden activation from its stored value h: sine -h (CosGrad's
// -sin), elu h < 0 ? h + 1 (= exp z) : 0.
__device__ __forceinline__ float act_d2(bool elu, float h) { return elu ? (h < 0.f ? __fadd_rn(h, 1.f) : 0.f) : -h; }

// sin and cos of x: Cody-Waite reduction by pi/2 (3-part constant, FMA) and minimax polynomials
// on [-pi/4, pi/4] (max error ~1 ulp for |x| <= 8192, far beyond SIREN pre-activations);
// larger |x| falls back to the library's Payne-Hanek path.
__device__ __forceinline__ void fast_sincos(float x, float* s, float* c) {
  const float j = rintf(x * 0.636619772367581343f);
  float r = fmaf(-j, 1.5703125f, x);
  r = fmaf(-j, 4.837512969970703125e-4f, r);
  r = fmaf(-j, 7.54978995489188216e-8f, r);
  const float r2 = r * r;
  float ps = fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
  ps = fmaf(r2, ps, -1.6666654611e-1f);
  const float sr = fmaf(r * r2, ps, r);
  float pc = fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
  pc = fmaf(r2, pc, 4.166664568298827e-2f);
  const float cr = fmaf(r2 * r2, pc, fmaf(-0.5f, r2, 1.0f));
  const int q = (int)j & 3;
  const float a = (q & 1) ? cr : sr, b = (q & 1) ? sr : cr;
  float so = (q & 2) ? -a : a;
  float co = ((q + 1) & 2) ? -b : b;
  if (__builtin_expect(fabsf(x) > 8192.f, 0)) sincosf(x, &so, &co);
  *s = so;
  *c = co;
}
// fast_sincos on 4 values at once: the four polynomial chains interleave (no per-element branch
// in between), and the large-argument fallback is one branch for the group. Same results as
// fast_sincos element by element.
__device__ __forceinline__ void fast_sincos4(const float x[4], float s[4], float c[4]) {
  bool big = false;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float j = rintf(x[r] * 0.636619772367581343f);
    float t = fmaf(-j, 1.5703125f, x[r]);
    t = fmaf(-j, 4.837512969970703125e-4f, t);
    t = fmaf(-j, 7.54978995489188216e-8f, t);
    const float t2 = t * t;
    float ps = fmaf(t2, -1.9515295891e-4f, 8.3321608736e-3f);
    ps = fmaf(t2, ps, -1.6666654611e-1f);
    const float sr = fmaf(t * t2, ps, t);
    float pc = fmaf(t2, 2.443315711809948e-5f, -1.388731625493765e-3f);
    pc = fmaf(t2, pc, 4.166664568298827e-2f);
    const float cr = fmaf(t2 * t2, pc, fmaf(-0.5f, t2, 1.0f));
    const int q = (int)j & 3;
    const float a = (q & 1) ? cr : sr, b = (q & 1) ? sr : cr;
    s[r] = (q & 2) ? -a : a;
    c[r] = ((q + 1) & 2) ? -b : b;
    big |= fabsf(x[r]) > 8192.f;
  }
  if (__builtin_expect(big, 0)) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (fabsf(x[r]) > 8192.f) sincosf(x[r], &s[r], &c[r]);
  }
}
__device__ __forceinline__ float fdiv(float a, float b) { return __fdiv_rn(a, b); }
__device__ __forceinline__ double dmul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double dadd(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ double dsub(double a, double b) { return __dsub_rn(a, b); }

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// 4 k-steps of one fragment block: a/b carry j = 0..3 (see mlp.h for the layout).
__device__ __forceinline__ floatx4 mfma_block(float4 a, float4 b, floatx4 c) {
  c = mfma4(a.x, b.x, c);
  c = mfma4(a.y, b.y, c);
  c = mfma4(a.z, b.z, c);
  c = mfma4(a.w, b.w, c);
  return c;
}

__device__ __forceinline__ float get4(const float4& v, int r) {
  return r == 0 ? v.x : (r == 1 ? v.y : (r == 2 ? v.z : v.w));
}
__device__ __forceinline__ float get4(const floatx4& v, int r) { return v[r]; }

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace cacto
