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
