// Building blocks shared by the network kernels: tile fills, split-K last layers, critic and
// actor forward passes over a 16-sample tile held in LDS.
#pragma once

#include "internal.h"

namespace cacto {

struct Lane {
  int tid, wave, lane, g, c;
  __device__ Lane() {
    tid = threadIdx.x;
    wave = tid >> 6;
    lane = tid & 63;
    g = lane >> 4;
    c = lane & 15;
  }
};

__device__ __forceinline__ float4 f4(const floatx4& a) { return make_float4(a[0], a[1], a[2], a[3]); }

// Layers whose output is a single 16-row tile (OT == 1): split the K loop over the 4 waves,
// reduce the partial accumulators through LDS `red` (4 x 64 float4) in fixed order, and let
// wave 0 run the epilogue. Contains __syncthreads(): all threads must call it.
template <typename Epi>
__device__ __forceinline__ void mm_single_tile(const float4* __restrict__ A, int KT, const float4* X, float4* red,
                                               const Lane& L, Epi&& epi) {
  float4 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kt = min(L.wave + 4 * i, KT - 1);
    a[i] = A[kt * 64 + L.lane];
    b[i] = X[kt * 64 + L.lane];
  }
  floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (L.wave + 4 * i < KT) {
      c0 = mfma4(a[i].x, b[i].x, c0);
      c1 = mfma4(a[i].y, b[i].y, c1);
      c2 = mfma4(a[i].z, b[i].z, c2);
      c3 = mfma4(a[i].w, b[i].w, c3);
    }
  }
  red[L.wave * 64 + L.lane] = f4((c0 + c1) + (c2 + c3));
  __syncthreads();
  if (L.wave == 0) {
    floatx4 s = {0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < CACTO_NWAVES; ++w) {
      const float4 p = red[w * 64 + L.lane];
      s[0] += p.x;
      s[1] += p.y;
      s[2] += p.z;
      s[3] += p.w;
    }
    epi(0, s);
  }
}

// Generic layer: OT == 1 -> split-K; else out tiles round-robin over waves. Ends with a barrier.
template <typename Epi>
__device__ __forceinline__ void layer(const float4* __restrict__ A, int OT, int KT, const float4* X, float4* red,
                                      const Lane& L, Epi&& epi) {
  if (OT == 1) {
    mm_single_tile(A, KT, X, red, L, epi);
  } else {
    mm_layer(A, OT, KT, X, L.wave, L.lane, epi);
  }
  __syncthreads();
}

constexpr int ZOFF[4] = {0, 4, 8, 16};  // critic hidden-layer tile offsets (64, 64, 128, 128 features)

// Critic forward over the input tile X0. With Hs != nullptr every h_l = sin(z_l) is kept (24 tiles,
// offsets ZOFF); otherwise h tiles alternate in H (2 x 8 tiles). With Cs != nullptr cos(z_l) is
// kept too (24 tiles), so no later pass re-evaluates a transcendental. hook(l, ot, h4) runs for
// every hidden out tile (l = 0..3). V[c] (LDS, 16 floats) receives the output for sample c.
template <typename Hook>
__device__ void critic_forward_tile(const NetView& N, const float4* X0, float4* Cs, float4* Hs, float4* H, float4* red,
                                    float* V, const Lane& L, Hook&& hook) {
  const float4* in = X0;
  for (int l = 0; l < 4; ++l) {
    float4* out = Hs ? Hs + ZOFF[l] * 64 : H + (l & 1) * 8 * 64;
    layer(N.fwd(l), N.t.OT[l], N.t.KT[l], in, red, L, [&](int ot, floatx4 acc) {
      float h[4], c[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) fast_sincos(fadd(acc[r], N.bias(l, 16 * ot + 4 * L.g + r)), &h[r], &c[r]);
      const float4 h4 = make_float4(h[0], h[1], h[2], h[3]);
      if (Cs) Cs[(ZOFF[l] + ot) * 64 + L.lane] = make_float4(c[0], c[1], c[2], c[3]);
      out[ot * 64 + L.lane] = h4;
      hook(l, ot, h4);
    });
    in = out;
  }
  layer(N.fwd(4), 1, N.t.KT[4], in, red, L, [&](int, floatx4 acc) {
    if (L.g == 0) V[L.c] = fadd(acc[0], N.bias(4, 0));
  });
}

// Actor forward; Z1/Z2 (16 tiles each) kept when non-null, h tiles in H (2 x 16 tiles).
// A[c * na + f] (LDS) receives the action.
template <typename Hook>
__device__ void actor_forward_tile(const NetView& N, int na, const float4* X0, float4* Z, float4* H, float4* red,
                                   float* A, const Lane& L, Hook&& hook) {
  const float4* in = X0;
  for (int l = 0; l < 2; ++l) {
    float4* out = H + l * 16 * 64;
    layer(N.fwd(l), N.t.OT[l], N.t.KT[l], in, red, L, [&](int ot, floatx4 acc) {
      float z[4], h[4];
      for (int r = 0; r < 4; ++r) {
        z[r] = fadd(acc[r], N.bias(l, 16 * ot + 4 * L.g + r));
        h[r] = z[r] > 0.f ? z[r] : fmul(z[r], 0.3f);  // LeakyReLU(alpha=0.3)
      }
      const float4 z4 = make_float4(z[0], z[1], z[2], z[3]);
      const float4 h4 = make_float4(h[0], h[1], h[2], h[3]);
      if (Z) Z[(l * 16 + ot) * 64 + L.lane] = z4;
      out[ot * 64 + L.lane] = h4;
      hook(l, ot, z4, h4);
    });
    in = out;
  }
  layer(N.fwd(2), 1, N.t.KT[2], in, red, L, [&](int, floatx4 acc) {
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * L.g + r;
      if (f < na) A[L.c * na + f] = fadd(acc[r], N.bias(2, f));
    }
  });
}

// Fill one input tile (16 features x 16 samples) from per-sample float32 states in LDS
// `st` ([16][16]), normalising. Called by wave 0 (lanes 0..63).
__device__ __forceinline__ void fill_input_tile(const cacto_sys_params& p, const float* st, float4* X, const Lane& L) {
  float v[4];
  for (int r = 0; r < 4; ++r) {
    const int f = 4 * L.g + r;
    v[r] = f < p.nb_state ? normalize_feature(p, f, st[L.c * 16 + f]) : 0.f;
  }
  X[L.lane] = make_float4(v[0], v[1], v[2], v[3]);
}

// Critic input gradient (first backward pass) from the cos tiles Cs: G[4] = W5,
// D[l] = G[l+1] cos z_l, G[l] = D[l] W_l^T. Results: G tiles (G1 at 0, G2 at 4, G3 at 8; 16 tiles)
// when Gs != nullptr, D via hookD(l, ot, lane, d4), and dV/dx0 in G0 (1 tile).
template <typename HookD>
__device__ void critic_first_backward(const NetView& N, const float4* Cs, float4* P /* 2 x 8 tiles */, float4* Gs,
                                      float4* G0, float4* red, const Lane& L, HookD&& hookD) {
  const int goff[4] = {0, 0, 4, 8};  // G[l] tile offsets for l = 1..3
  // D3 = W5[:,0] * cos(z3)
  float4* D = P;
  for (int idx = L.tid; idx < N.t.OT[3] * 64; idx += CACTO_THREADS) {
    const int ot = idx >> 6, lane = idx & 63, g = lane >> 4;
    const float4 c = Cs[(ZOFF[3] + ot) * 64 + lane];
    const int f = 16 * ot + 4 * g;
    const float4 d4 = make_float4(fmul(N.w(4, f, 0), c.x), fmul(N.w(4, f + 1, 0), c.y), fmul(N.w(4, f + 2, 0), c.z),
                                  fmul(N.w(4, f + 3, 0), c.w));
    D[idx] = d4;
    hookD(3, ot, lane, d4);
  }
  __syncthreads();
  for (int l = 3; l >= 1; --l) {
    float4* Dn = P + ((4 - l) & 1) * 8 * 64;  // alternate
    // G[l] = D[l] W_l^T : M tiles = KT[l] (in of layer l), K tiles = OT[l]
    layer(N.bwd(l), N.t.KT[l], N.t.OT[l], D, red, L, [&](int it, floatx4 acc) {
      const float4 gl = f4(acc);
      if (Gs) Gs[(goff[l] + it) * 64 + L.lane] = gl;
      const float4 c = Cs[(ZOFF[l - 1] + it) * 64 + L.lane];
      const float4 d4 = make_float4(fmul(gl.x, c.x), fmul(gl.y, c.y), fmul(gl.z, c.z), fmul(gl.w, c.w));
      Dn[it * 64 + L.lane] = d4;
      hookD(l - 1, it, L.lane, d4);
    });
    D = Dn;
  }
  // G[0] = D0 W_1^T (one tile: ns <= 16)
  layer(N.bwd(0), 1, N.t.OT[0], D, red, L, [&](int, floatx4 acc) { G0[L.lane] = f4(acc); });
}

}  // namespace cacto
