// Microbenchmark: v_mfma_f32_4x4x1f32 (16 blocks) lane layout and issue rate vs 16x16x4f32 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(float* out) {
  const int l = threadIdx.x;
  // A: lane value = 100 + l ; B: lane value = 1 except probe: B = (l==0?1:0) etc.
  floatx4 c = {0, 0, 0, 0};
  float a = (float)(l + 1);
  float b = (float)((l + 1) * 1000);
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

template <int NACC>
__global__ void __launch_bounds__(256) k_rate4(float* out, int iters, float seed) {
  floatx4 c[NACC];
  for (int i = 0; i < NACC; ++i) c[i] = floatx4{0, 0, 0, 0};
  float a = seed * threadIdx.x, b = seed + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#pragma unroll
      for (int i = 0; i < NACC; ++i) c[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[i], 0, 0, 0);
    }
  }
  floatx4 s = c[0];
  for (int i = 1; i < NACC; ++i) s += c[i];
  if (s[0] == 1.2345f) out[threadIdx.x] = s[1];
}

template <int NACC>
__global__ void __launch_bounds__(256) k_rate16(float* out, int iters, float seed) {
  floatx4 c[NACC];
  for (int i = 0; i < NACC; ++i) c[i] = floatx4{0, 0, 0, 0};
  float a = seed * threadIdx.x, b = seed + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int i = 0; i < NACC; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[i], 0, 0, 0);
    }
  }
  floatx4 s = c[0];
  for (int i = 1; i < NACC; ++i) s += c[i];
  if (s[0] == 1.2345f) out[threadIdx.x] = s[1];
}

// 8 waves: waves 0-3 MFMA (4x4x1, 4 acc), waves 4-7 f64 FMA chains (4 independent)
__global__ void __launch_bounds__(512) k_mixed(float* out, double* dout, int iters, float seed, int do_valu) {
  const int w = threadIdx.x >> 6;
  if (w < 4) {
    floatx4 c[4];
    for (int i = 0; i < 4; ++i) c[i] = floatx4{0, 0, 0, 0};
    float a = seed * threadIdx.x, b = seed + threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[i], 0, 0, 0);
      }
    }
    floatx4 s = c[0] + c[1] + c[2] + c[3];
    if (s[0] == 1.2345f) out[threadIdx.x] = s[1];
  } else if (do_valu) {
    double x0 = seed, x1 = seed + 1, x2 = seed + 2, x3 = seed + 3;
    const double m = 0.999999, q = 1e-7;
    for (int it = 0; it < iters * 4; ++it) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        x0 = fma(x0, m, q); x1 = fma(x1, m, q); x2 = fma(x2, m, q); x3 = fma(x3, m, q);
      }
    }
    if (x0 + x1 + x2 + x3 == 1.2345) dout[threadIdx.x] = x0;
  }
}


__global__ void __launch_bounds__(512) k_mix2(float* out, double* dout, int iters, float seed, int mode, int vper) {
  const int w = threadIdx.x >> 6;
  const bool mf = (mode == 0 || mode == 2 || mode == 3 || mode == 5);
  const bool vd = (mode == 1 || mode == 2 || mode == 3);
  const bool vf = (mode == 4 || mode == 5);
  if (w < 4) {
    if (!mf) return;
    floatx4 c[4];
    for (int i = 0; i < 4; ++i) c[i] = floatx4{0, 0, 0, 0};
    float a = seed * threadIdx.x, b = seed + threadIdx.x;
    if (mode == 3) {
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[i], 0, 0, 0);
      }
    } else {
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[i], 0, 0, 0);
      }
    }
    floatx4 s = c[0] + c[1] + c[2] + c[3];
    if (s[0] == 1.2345f) out[threadIdx.x] = s[1];
  } else if (vd) {
    double x0 = seed, x1 = seed + 1, x2 = seed + 2, x3 = seed + 3;
    const double m = 0.999999, q = 1e-7;
    for (int it = 0; it < iters * vper; ++it) {
      x0 = fma(x0, m, q); x1 = fma(x1, m, q); x2 = fma(x2, m, q); x3 = fma(x3, m, q);
    }
    if (x0 + x1 + x2 + x3 == 1.2345) dout[threadIdx.x] = x0;
  } else if (vf) {
    float x0 = seed, x1 = seed + 1, x2 = seed + 2, x3 = seed + 3;
    const float m = 0.999999f, q = 1e-7f;
    for (int it = 0; it < iters * vper; ++it) {
      x0 = fmaf(x0, m, q); x1 = fmaf(x1, m, q); x2 = fmaf(x2, m, q); x3 = fmaf(x3, m, q);
    }
    if (x0 + x1 + x2 + x3 == 1.2345f) out[threadIdx.x] = x0;
  }
}


__global__ void k_bcast(float* out) {
  const int l = threadIdx.x;
  floatx4 c = {0, 0, 0, 0};
  float a = (float)(l + 1);
  float b = (float)((l + 1) * 1000);
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 4, 5, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
__global__ void __launch_bounds__(256) k_rate_bc(float* out, int iters, float seed) {
  floatx4 c[4];
  for (int i = 0; i < 4; ++i) c[i] = floatx4{0, 0, 0, 0};
  float a = seed * threadIdx.x, b = seed + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#define Q(q) c[q & 3] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[q & 3], 4, q, 0);
    Q(0) Q(1) Q(2) Q(3) Q(4) Q(5) Q(6) Q(7) Q(8) Q(9) Q(10) Q(11) Q(12) Q(13) Q(14) Q(15)
    Q(0) Q(1) Q(2) Q(3) Q(4) Q(5) Q(6) Q(7) Q(8) Q(9) Q(10) Q(11) Q(12) Q(13) Q(14) Q(15)
    Q(0) Q(1) Q(2) Q(3) Q(4) Q(5) Q(6) Q(7) Q(8) Q(9) Q(10) Q(11) Q(12) Q(13) Q(14) Q(15)
    Q(0) Q(1) Q(2) Q(3) Q(4) Q(5) Q(6) Q(7) Q(8) Q(9) Q(10) Q(11) Q(12) Q(13) Q(14) Q(15)
  }
  floatx4 s = c[0] + c[1] + c[2] + c[3];
  if (s[0] == 1.2345f) out[threadIdx.x] = s[1];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <typename F>
float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  float* d; double* dd;
  CK(hipMalloc(&d, 1 << 20)); CK(hipMalloc(&dd, 1 << 20));
  k_layout<<<1, 64>>>(d);
  std::vector<float> h(256);
  CK(hipMemcpy(h.data(), d, 1024, hipMemcpyDeviceToHost));
  printf("layout: D[lane][r] = A*B ; A=lane+1, B=(lane+1)*1000\n");
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int r = 0; r < 4; ++r) { float v = h[l * 4 + r]; int ab = (int)(v / 1000.f); printf(" %8.0f", v); (void)ab; }
    printf("\n");
  }
  const int iters = 20000, grid = 256 * 8;
  double fl4 = 512.0 * 16 * iters * 4.0 * grid;  // per-wave flops * waves
  float ms;
  ms = timeit([&] { k_rate4<1><<<grid, 256>>>(d, iters, 1.f); });
  printf("4x4x1 1acc: %.3f ms  %.1f TF/s\n", ms, 512.0 * 16 * iters * 1 * grid * 4 / ms / 1e9);
  ms = timeit([&] { k_rate4<2><<<grid, 256>>>(d, iters, 1.f); });
  printf("4x4x1 2acc: %.3f ms  %.1f TF/s\n", ms, 512.0 * 16 * iters * 2 * grid * 4 / ms / 1e9);
  ms = timeit([&] { k_rate4<4><<<grid, 256>>>(d, iters, 1.f); });
  printf("4x4x1 4acc: %.3f ms  %.1f TF/s\n", ms, 512.0 * 16 * iters * 4 * grid * 4 / ms / 1e9);
  ms = timeit([&] { k_rate16<1><<<grid, 256>>>(d, iters, 1.f); });
  printf("16x16x4 1acc: %.3f ms  %.1f TF/s\n", ms, 2048.0 * 4 * iters * 1 * grid * 4 / ms / 1e9);
  ms = timeit([&] { k_rate16<4><<<grid, 256>>>(d, iters, 1.f); });
  printf("16x16x4 4acc: %.3f ms  %.1f TF/s\n", ms, 2048.0 * 4 * iters * 4 * grid * 4 / ms / 1e9);
  const int g2 = 256;
  ms = timeit([&] { k_mixed<<<g2, 512>>>(d, dd, iters, 1.f, 0); });
  printf("mixed (no valu) : %.3f ms  %.1f TF/s\n", ms, 512.0 * 16 * iters * 4 * g2 * 4 / ms / 1e9);
  ms = timeit([&] { k_mixed<<<g2, 512>>>(d, dd, iters, 1.f, 1); });
  printf("mixed (f64 valu): %.3f ms  %.1f TF/s\n", ms, 512.0 * 16 * iters * 4 * g2 * 4 / ms / 1e9);

  const char* names[] = {"mfma4x4 only", "f64 valu only", "mfma4x4 + f64", "mfma16 + f64", "f32 valu only", "mfma4x4 + f32"};
  for (int vper : {4, 16}) for (int mode = 0; mode < 6; ++mode) {
    ms = timeit([&] { k_mix2<<<g2, 512>>>(d, dd, iters, 1.f, mode, vper); });
    printf("vper %2d %-16s: %.3f ms\n", vper, names[mode], ms);
  }

  k_bcast<<<1, 64>>>(d);
  CK(hipMemcpy(h.data(), d, 1024, hipMemcpyDeviceToHost));
  printf("bcast cbsz=4 abid=5:\n");
  for (int l = 0; l < 64; l += 1) { printf("lane %2d:", l); for (int r = 0; r < 4; ++r) printf(" %8.0f", h[l*4+r]); printf("\n"); }
  ms = timeit([&] { k_rate_bc<<<grid, 256>>>(d, iters / 4, 1.f); });
  printf("4x4x1 bcast 4acc: %.3f ms  %.1f TF/s\n", ms, 512.0 * 64 * (iters / 4) * grid * 4 / ms / 1e9);
  (void)fl4;
  return 0;
}
