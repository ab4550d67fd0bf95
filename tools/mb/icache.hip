// Microbenchmark: cost of executing straight-line code once (cold instruction cache) vs again
// (warm), for code sizes around the 64 KB instruction cache. Each block is 8 independent
// v_fma_f32 chains; the kernel runs the unrolled body twice (outer loop not unrolled) and stamps
// both passes with s_memtime. Build: hipcc -O3 --offload-arch=gfx950 icache.hip -o icache
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
__global__ void __launch_bounds__(256) k_body(float* out, unsigned long long* t) {
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 0.001f + k;
  unsigned long long s[3];
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    s[pass] = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] = __builtin_fmaf(a[k], 0.999f, 0.001f * (i + 1));
  }
  s[2] = __builtin_amdgcn_s_memtime();
  float r = 0.f;
  for (int k = 0; k < 8; ++k) r += a[k];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) {
    t[blockIdx.x * 2 + 0] = s[1] - s[0];
    t[blockIdx.x * 2 + 1] = s[2] - s[1];
  }
}

template <int N>
void run(int blocks) {
  float* out;
  unsigned long long* t;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&t, blocks * 16);
  unsigned long long h[2 * 256];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_body<N>, dim3(blocks), dim3(256), 0, 0, out, t);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, t, blocks * 16, hipMemcpyDeviceToHost);
  double c0 = 0, c1 = 0;
  for (int b = 0; b < blocks; ++b) c0 += h[2 * b], c1 += h[2 * b + 1];
  c0 /= blocks, c1 /= blocks;
  const double instr = 8.0 * N;
  printf("N=%5d (~%6.0f KB code) blocks=%3d: pass1 %8.0f cyc (%.2f/instr)  pass2 %8.0f cyc (%.2f/instr)\n", N,
         instr * 8 / 1024, blocks, c0, c0 / instr, c1, c1 / instr);
  hipFree(out);
  hipFree(t);
}

int main() {
  for (int blocks : {8, 256}) {
    run<128>(blocks);
    run<512>(blocks);
    run<1024>(blocks);
    run<2048>(blocks);
    run<4096>(blocks);
  }
  return 0;
}
