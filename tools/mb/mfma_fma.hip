// Does a chain of K=1 steps of v_mfma_f32_4x4x1f32 (A broadcast with CBSZ/ABID, as the rollout's
// layer 1 uses it) round like a chain of fmaf, or like separately rounded multiply + add? Counts
// mismatches of both over random operands. Diagnostic only.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/mb/mfma_fma.hip -o tools/mb/bin/mfma_fma
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int Q>
__device__ floatx4 mf(float x, float w, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(x, w, c, 4, Q, 0);
}

// x[t][q][i] (q < 5 features, i < 4 samples), w[t][q][64 lanes]; out: per trial and lane, 4 values
__global__ void k_chain(const float* x, const float* w, int* bad_fma, int* bad_sep, int trials) {
  const int l = threadIdx.x;
  for (int t = blockIdx.x; t < trials; t += gridDim.x) {
    const float* xt = x + t * 20;
    const float* wt = w + t * 5 * 64;
    // lane 4q + i holds x[q][i] (the broadcast block q carries feature q's 4 samples)
    const float xl = l < 20 ? xt[(l >> 2) * 4 + (l & 3)] : 0.f;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = mf<0>(xl, wt[0 * 64 + l], acc);
    acc = mf<1>(xl, wt[1 * 64 + l], acc);
    acc = mf<2>(xl, wt[2 * 64 + l], acc);
    acc = mf<3>(xl, wt[3 * 64 + l], acc);
    acc = mf<4>(xl, wt[4 * 64 + l], acc);
    for (int i = 0; i < 4; ++i) {
      float f = 0.f, s = 0.f;
      for (int q = 0; q < 5; ++q) {
        f = __builtin_fmaf(xt[q * 4 + i], wt[q * 64 + l], f);
        s = __fadd_rn(__fmul_rn(xt[q * 4 + i], wt[q * 64 + l]), s);
      }
      if (__float_as_uint(acc[i]) != __float_as_uint(f)) atomicAdd(bad_fma, 1);
      if (__float_as_uint(acc[i]) != __float_as_uint(s)) atomicAdd(bad_sep, 1);
    }
  }
}

int main() {
  const int trials = 20000;
  std::vector<float> x(trials * 20), w(trials * 5 * 64);
  srand(1);
  auto rnd = [] { return (float)((rand() / (double)RAND_MAX) * 2.0 - 1.0) * (float)(1 << (rand() % 8)); };
  for (auto& v : x) v = rnd();
  for (auto& v : w) v = rnd();
  float *dx, *dw;
  int* dbad;
  hipMalloc(&dx, x.size() * 4);
  hipMalloc(&dw, w.size() * 4);
  hipMalloc(&dbad, 8);
  hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice);
  hipMemset(dbad, 0, 8);
  hipLaunchKernelGGL(k_chain, dim3(256), dim3(64), 0, 0, dx, dw, dbad, dbad + 1, trials);
  int bad[2];
  hipMemcpy(bad, dbad, 8, hipMemcpyDeviceToHost);
  printf("mfma 4x4x1 K=1 chains vs fmaf chains: %d of %d differ; vs separately rounded mul+add: %d differ\n",
         bad[0], trials * 256, bad[1]);
  return 0;
}
