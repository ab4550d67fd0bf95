// Semantics check of the q4 machinery (cacto_amd/csrc/q4.h) on gfx950: the 4x4x1 broadcast with
// CBSZ = 2, the permlane swaps, and whole layers (forward image, transposed image, split-K,
// streamed) against a float64 host reference. Prints PASS/FAIL lines; exit status 1 on a failure.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I. tools/mb/q4_check.hip -o /tmp/q4_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../cacto_amd/csrc/q4.h"

using namespace cacto;

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);              \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

__global__ void k_bcast2(float* out) {
  const int l = threadIdx.x;
  floatx4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), 1.0f, c, 2, 1, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

__global__ void k_swaps(float* out) {
  const int l = threadIdx.x;
  const auto r32 = __builtin_amdgcn_permlane32_swap((unsigned)l, (unsigned)(100 + l), false, false);
  const auto r16 = __builtin_amdgcn_permlane16_swap((unsigned)l, (unsigned)(100 + l), false, false);
  out[l * 4 + 0] = (float)r32[0];
  out[l * 4 + 1] = (float)r32[1];
  out[l * 4 + 2] = (float)r16[0];
  out[l * 4 + 3] = (float)r16[1];
}

// one layer in registers: in = 16*KT features, OT out tiles (NT per wave)
template <int KT, int NT, bool BIAS>
__global__ void __launch_bounds__(256) k_layer(const float4* pk, const float* bias, int OT, int nout, const float* X,
                                               float* out) {
  __shared__ float Xs[KT * 64];
  for (int k = threadIdx.x; k < KT * 64; k += 256) Xs[k] = X[k];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Q4Frags<KT, NT> F;
  F.template load<BIAS>(pk, bias, OT, nout, wave, lane);
  F.template run<BIAS>(Xs, OT, wave, lane, [&](int ot, float v) { out[q4e(ot, lane)] = v; });
}

template <int NK>
__global__ void __launch_bounds__(256) k_split(const float4* pk, const float* bias, int KT, int nout, const float* X,
                                               float* out) {
  __shared__ float Xs[16 * 64];
  __shared__ float red[4 * 64];
  for (int k = threadIdx.x; k < KT * 64; k += 256) Xs[k] = X[k];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Q4Split<NK> F;
  F.template load<true>(pk, KT, bias, nout, wave, lane);
  F.template run<true>(KT, Xs, red, wave, lane, [&](int, float v) { out[q4e(0, lane)] = v; });
}

// the 8-wave pair layout (one pair of out tiles per wave), as the q4 chains run it
__global__ void __launch_bounds__(512) k_pairs8(const float4* pk, const float* bias, const float* X, float* out) {
  __shared__ float Xs[16 * 64];
  for (int k = threadIdx.x; k < 16 * 64; k += 512) Xs[k] = X[k];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Q4Pair<16, 8> P0;
  P0.load(pk, 0, wave, lane);
  q4_layer_pairs<16, true, 8>(pk, Xs, wave, lane, [&](int ot, float v) { out[q4e(ot, lane)] = v; }, bias, P0);
}

__global__ void __launch_bounds__(256) k_pairs(const float4* pk, const float* bias, const float* X, float* out) {
  __shared__ float Xs[16 * 64];
  for (int k = threadIdx.x; k < 16 * 64; k += 256) Xs[k] = X[k];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Q4Pair<16, 4> P0;
  P0.load(pk, 0, wave, lane);
  q4_layer_pairs<16, true, 4>(pk, Xs, wave, lane, [&](int ot, float v) { out[q4e(ot, lane)] = v; }, bias, P0);
}

// mlp.h images of W [in][out]
static std::vector<float> pack_fwd(const std::vector<float>& W, int in, int out) {
  const int KT = (in + 15) / 16, OT = (out + 15) / 16;
  std::vector<float> pk((size_t)KT * OT * 256, 0.f);
  for (int ot = 0; ot < OT; ++ot)
    for (int kt = 0; kt < KT; ++kt)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 4; ++j) {
          const int g = l >> 4, c = l & 15, i = 16 * kt + 4 * g + j, o = 16 * ot + c;
          pk[(((size_t)ot * KT + kt) * 64 + l) * 4 + j] = (i < in && o < out) ? W[(size_t)i * out + o] : 0.f;
        }
  return pk;
}
static std::vector<float> pack_bwd(const std::vector<float>& W, int in, int out) {
  const int KT = (in + 15) / 16, OT = (out + 15) / 16;
  std::vector<float> pk((size_t)KT * OT * 256, 0.f);
  for (int it = 0; it < KT; ++it)
    for (int kt = 0; kt < OT; ++kt)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 4; ++j) {
          const int g = l >> 4, c = l & 15, i = 16 * it + c, o = 16 * kt + 4 * g + j;
          pk[(((size_t)it * OT + kt) * 64 + l) * 4 + j] = (i < in && o < out) ? W[(size_t)i * out + o] : 0.f;
        }
  return pk;
}

struct Dev {
  float4* pk;
  float *bias, *X, *out;
};

static int fails = 0;

static void compare(const char* name, const std::vector<float>& got, const std::vector<double>& ref, int nf) {
  // error relative to the largest reference magnitude (f32 sums of O(1) terms)
  double worst = 0, scale = 1e-30;
  for (int k = 0; k < nf * 4; ++k) scale = std::fmax(scale, std::fabs(ref[k]));
  for (int f = 0; f < nf; ++f)
    for (int i = 0; i < 4; ++i) {
      const double r = ref[f * 4 + i], g = got[f * 4 + i];
      const double err = std::fabs(g - r) / scale;
      if (!(err <= worst)) worst = err;
    }
  const bool ok = worst < 2e-6;
  if (!ok) ++fails;
  printf("%s %s (worst rel err %.3g)\n", ok ? "PASS" : "FAIL", name, worst);
}

int main() {
  float* d;
  CK(hipMalloc(&d, 1 << 20));
  std::vector<float> h(256);
  k_bcast2<<<1, 64>>>(d);
  CK(hipMemcpy(h.data(), d, 1024, hipMemcpyDeviceToHost));
  // expected with "block b takes the A operand of block (b & ~3) | 1": D[i] = lane(4*((b&~3)|1)+i) + 1
  bool bok = true;
  for (int l = 0; l < 64; ++l) {
    const int b = l >> 2;
    for (int i = 0; i < 4; ++i) {
      const float want = (float)(4 * ((b & ~3) | 1) + i + 1);
      if (h[l * 4 + i] != want) bok = false;
    }
  }
  printf("%s cbsz=2 abid=1 broadcast within groups of 4 blocks\n", bok ? "PASS" : "FAIL");
  if (!bok) {
    ++fails;
    for (int l = 0; l < 64; ++l) printf("lane %2d: %g %g %g %g\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  }
  k_swaps<<<1, 64>>>(d);
  CK(hipMemcpy(h.data(), d, 1024, hipMemcpyDeviceToHost));
  bool s32 = true, s16 = true;
  for (int l = 0; l < 64; ++l) {
    // permlane32_swap(vdst = l, src = 100 + l): lanes 32-63 of vdst <-> lanes 0-31 of src
    const float v0 = l < 32 ? l : 100 + (l - 32), v1 = l < 32 ? (l + 32) : 100 + l;
    if (h[l * 4] != v0 || h[l * 4 + 1] != v1) s32 = false;
    // permlane16_swap: odd rows of vdst <-> even rows of src
    const int row = l >> 4;
    const float w0 = (row & 1) ? 100 + (l - 16) : l, w1 = (row & 1) ? 100 + l : (l + 16);
    if (h[l * 4 + 2] != w0 || h[l * 4 + 3] != w1) s16 = false;
  }
  printf("%s permlane32_swap semantics\n%s permlane16_swap semantics\n", s32 ? "PASS" : "FAIL", s16 ? "PASS" : "FAIL");
  if (!s32 || !s16) {
    ++fails;
    for (int l = 0; l < 64; ++l) printf("lane %2d: %g %g | %g %g\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  }

  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  Dev D;
  CK(hipMalloc(&D.pk, 1 << 20));
  CK(hipMalloc(&D.bias, 4096));
  CK(hipMalloc(&D.X, 1 << 16));
  CK(hipMalloc(&D.out, 1 << 16));
  auto run_case = [&](const char* name, int in, int out, bool transposed, int kind) -> int {
    std::vector<float> W((size_t)in * out), b(out), X;
    for (auto& w : W) w = U(rng);
    for (auto& v : b) v = U(rng);
    // the op: y[o][i] = sum_k M[k][o] x[k][i] (+ b[o]); M = W (forward) or W^T (transposed)
    const int K = transposed ? out : in, O = transposed ? in : out;
    const int KT = (K + 15) / 16, OT = (O + 15) / 16;
    X.assign((size_t)KT * 64, 0.f);
    for (int k = 0; k < K; ++k)
      for (int i = 0; i < 4; ++i) X[k * 4 + i] = U(rng);
    std::vector<float> pk = transposed ? pack_bwd(W, in, out) : pack_fwd(W, in, out);
    const bool bias = !transposed;
    std::vector<double> ref((size_t)OT * 64, 0.0);
    for (int o = 0; o < O; ++o)
      for (int i = 0; i < 4; ++i) {
        double s = bias ? b[o] : 0.0;
        for (int k = 0; k < K; ++k) s += (double)(transposed ? W[(size_t)o * out + k] : W[(size_t)k * out + o]) * X[k * 4 + i];
        ref[o * 4 + i] = s;
      }
    CK(hipMemcpy(D.pk, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(D.bias, b.data(), b.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(D.X, X.data(), X.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(D.out, 0, 1 << 16));
    const float* bp = bias ? D.bias : nullptr;
    if (kind == 0 && KT == 4 && OT == 8) k_layer<4, 2, true><<<1, 256>>>(D.pk, bp, OT, O, D.X, D.out);
    else if (kind == 0 && KT == 8 && OT == 8) k_layer<8, 2, false><<<1, 256>>>(D.pk, bp, OT, O, D.X, D.out);
    else if (kind == 0 && KT == 1 && OT == 4) k_layer<1, 1, true><<<1, 256>>>(D.pk, bp, OT, O, D.X, D.out);
    else if (kind == 1 && KT == 8) k_split<2><<<1, 256>>>(D.pk, D.bias, KT, O, D.X, D.out);
    else if (kind == 1 && KT == 16) k_split<4><<<1, 256>>>(D.pk, D.bias, KT, O, D.X, D.out);
    else if (kind == 2 && KT == 16 && OT == 16 && bias) k_pairs8<<<1, 512>>>(D.pk, D.bias, D.X, D.out);
    else if (kind == 3 && KT == 16 && OT == 16 && bias) k_pairs<<<1, 256>>>(D.pk, D.bias, D.X, D.out);
    else {
      printf("no kernel for %s\n", name);
      ++fails;
      return 0;
    }
    CK(hipGetLastError());
    std::vector<float> got((size_t)OT * 64);
    CK(hipMemcpy(got.data(), D.out, got.size() * 4, hipMemcpyDeviceToHost));
    compare(name, got, ref, O);
    return 0;
  };
  run_case("layer 64->128 fwd, bias (Q4Frags<4,2>)", 64, 128, false, 0);
  run_case("layer 128->128 transposed (Q4Frags<8,2>)", 128, 128, true, 0);
  run_case("layer 5->64 fwd, bias (Q4Frags<1,1>)", 5, 64, false, 0);
  run_case("split 128->1, bias (Q4Split<2>)", 128, 1, false, 1);
  run_case("split 256->6, bias (Q4Split<4>)", 256, 6, false, 1);
  run_case("paired 256->256, bias, 8 waves (q4_layer_pairs<16, 8>)", 256, 256, false, 2);
  run_case("paired 256->256, bias (q4_layer_pairs<16>)", 256, 256, false, 3);
  printf(fails ? "q4_check: %d FAILED\n" : "q4_check: all passed\n", fails);
  return fails ? 1 : 0;
}
