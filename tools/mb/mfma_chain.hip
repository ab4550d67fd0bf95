// Cycles of a 256-instruction v_mfma_f32_4x4x1f32 (CBSZ 4) sequence in ONE wave per SIMD, with the
// accumulation spread over NACC independent accumulators (the rollout's layer 2 uses 2), and with
// two such waves per SIMD. Tells the per-wave latency floor of layer 2. Diagnostic only.
//   hipcc -O3 --offload-arch=gfx950 tools/mb/mfma_chain.hip -o tools/mb/bin/mfma_chain
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int NACC, int WPS>
__global__ void __launch_bounds__(256 * WPS) k_chain(float* out, unsigned long long* cyc, float seed) {
  __shared__ float pad[40000];  // one workgroup per CU
  floatx4 c[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) c[i] = floatx4{0, 0, 0, 0};
  float a = seed * threadIdx.x, b[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) b[q] = seed + threadIdx.x + q;
  unsigned long long t0 = 0;
  for (int rep = 0; rep < 3; ++rep) {
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
#define Q(q) c[(16 * k + q) % NACC] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b[q], c[(16 * k + q) % NACC], 4, q, 0);
      Q(0) Q(1) Q(2) Q(3) Q(4) Q(5) Q(6) Q(7) Q(8) Q(9) Q(10) Q(11) Q(12) Q(13) Q(14) Q(15)
#undef Q
    }
    floatx4 s = c[0];
#pragma unroll
    for (int i = 1; i < NACC; ++i) s += c[i];
    a = s[0] * 1e-30f + a;  // forces completion before the stamp
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 * WPS + threadIdx.x / 64] = t1 - t0;
  if (a == 1.2345f) out[threadIdx.x] = a + pad[threadIdx.x];
}

template <int NACC, int WPS>
void run(float* d, unsigned long long* dc) {
  hipLaunchKernelGGL((k_chain<NACC, WPS>), dim3(256), dim3(256 * WPS), 0, 0, d, dc, 1.f);
  hipDeviceSynchronize();
  unsigned long long h[256 * 8];
  hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < 256 * 4 * WPS; ++i) s += h[i];
  printf("%d wave(s) per SIMD, %d accumulators: %.0f cycles for 256 MFMAs (+ the reduction)\n", WPS, NACC,
         s / (256 * 4 * WPS));
}

int main() {
  float* d;
  unsigned long long* dc;
  hipMalloc(&d, 1 << 20);
  hipMalloc(&dc, 256 * 8 * 8);
  run<1, 1>(d, dc);
  run<2, 1>(d, dc);
  run<4, 1>(d, dc);
  run<8, 1>(d, dc);
  run<2, 2>(d, dc);
  run<4, 2>(d, dc);
  run<8, 2>(d, dc);
  return 0;
}
