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
                                               const Lane& L, Epi&& epi, const float* __restrict__ bias, int nout) {
  // bias of rows 4g + r < nout, loaded before the MFMAs (wave 0 adds it after the reduction)
  float bq[4] = {0.f, 0.f, 0.f, 0.f};
  if (bias && L.wave == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * L.g + r < nout) bq[r] = bias[4 * L.g + r];
  }
  float4 a[4], b[4];
  const int wave = uniform_wave(L.wave);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kt = min(wave + 4 * i, KT - 1);
    a[i] = ldfrag(A, kt, L.lane);
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
    if (bias)
#pragma unroll
      for (int r = 0; r < 4; ++r) s[r] = fadd(s[r], bq[r]);
    epi(0, s);
  }
}

// Register-held fragments of a single-out-tile layer for split-K (k-tiles wave + 4 i, i < NK),
// with the row biases; run() is mm_single_tile's arithmetic (contains __syncthreads()).
template <int NK>
struct SplitFrag {
  float4 a[NK];
  float bq[4];
  template <bool BIAS>
  __device__ __forceinline__ void load(const float4* __restrict__ A, int KT, const float* __restrict__ bias, int nout,
                                       const Lane& L) {
    const int wave = uniform_wave(L.wave);
#pragma unroll
    for (int i = 0; i < NK; ++i) a[i] = ldfrag(A, min(wave + 4 * i, KT - 1), L.lane);  // branch-free (clamped)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * L.g + r;
      bq[r] = BIAS ? bias[min(f, nout - 1)] : 0.f;
      if (f >= nout) bq[r] = 0.f;
    }
  }
  template <typename Epi>
  __device__ __forceinline__ void run(int KT, const float4* X, float4* red, const Lane& L, const float* bias,
                                      Epi&& epi) const {
    floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
#pragma unroll
    for (int i = 0; i < NK; ++i) {
      const int kt = L.wave + 4 * i;
      if (kt < KT) {
        const float4 b = X[kt * 64 + L.lane];
        c0 = mfma4(a[i].x, b.x, c0);
        c1 = mfma4(a[i].y, b.y, c1);
        c2 = mfma4(a[i].z, b.z, c2);
        c3 = mfma4(a[i].w, b.w, c3);
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
      if (bias)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[r] = fadd(s[r], bq[r]);
      epi(0, s);
    }
  }
};

// The critic's fixed shape (SIREN 64-64-128-128-1 on <= 16 inputs): per wave, forward fragments
// l0: 1 tile x 1 k-tile, l1: 1 x 4, l2: 2 x 4, l3: 2 x 8, l4: split-K 2 of 8 k-tiles; the
// transposed (input-gradient) passes G_l = D_l W_l^T use l3: 2 x 8, l2: 1 x 8, l1: 1 x 4,
// l0: split-K 1 of 4.
struct CriticFwdFrags {
  Frags<1, 1> f0;
  Frags<4, 1> f1;
  Frags<4, 2> f2;
  Frags<8, 2> f3;
  SplitFrag<2> f4;
  template <bool BIAS>
  __device__ __forceinline__ void load(const NetView& N, const Lane& L) {
    f0.load<BIAS>(N.fwd(0), N.biasp(0), 4, L.wave, L.lane);
    f1.load<BIAS>(N.fwd(1), N.biasp(1), 4, L.wave, L.lane);
    f2.load<BIAS>(N.fwd(2), N.biasp(2), 8, L.wave, L.lane);
    f3.load<BIAS>(N.fwd(3), N.biasp(3), 8, L.wave, L.lane);
  }
  __device__ __forceinline__ void load_last(const NetView& N, const Lane& L) {
    f4.load<true>(N.fwd(4), 8, N.biasp(4), 1, L);
  }
};

struct CriticBwdFrags {
  Frags<8, 2> g3;
  Frags<8, 1> g2;
  Frags<4, 1> g1;
  SplitFrag<1> g0;
  float4 w5[2];  // W5[:, 0] at the lane's rows of out tiles wave and wave + 4 of layer 3
  __device__ __forceinline__ void load(const NetView& N, const Lane& L) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float* w = N.flat + N.t.woff[4] + 16 * (L.wave + 4 * t) + 4 * L.g;
      w5[t] = make_float4(w[0], w[1], w[2], w[3]);
    }
    g3.load<false>(N.bwd(3), nullptr, 8, L.wave, L.lane);
    g2.load<false>(N.bwd(2), nullptr, 4, L.wave, L.lane);
    g1.load<false>(N.bwd(1), nullptr, 4, L.wave, L.lane);
    g0.load<false>(N.bwd(0), 4, nullptr, 1, L);
  }
};

// Generic layer: OT == 1 -> split-K; else out tiles round-robin over waves. Ends with a barrier.
// With `bias` (global, nout entries) the epilogue receives acc + bias.
template <typename Epi>
__device__ __forceinline__ void layer(const float4* __restrict__ A, int OT, int KT, const float4* X, float4* red,
                                      const Lane& L, Epi&& epi, const float* __restrict__ bias = nullptr,
                                      int nout = 0) {
  if (OT == 1) {
    mm_single_tile(A, KT, X, red, L, epi, bias, nout);
  } else {
    mm_layer(A, OT, KT, X, L.wave, L.lane, epi, bias);
  }
  __syncthreads();
}

constexpr int ZOFF[4] = {0, 4, 8, 16};  // critic hidden-layer tile offsets (64, 64, 128, 128 features)

// Critic forward over the input tile X0. With Hs != nullptr every h_l = sin(z_l) is kept (24 tiles,
// offsets ZOFF); otherwise h tiles alternate in H (2 x 8 tiles). With Cs != nullptr cos(z_l) is
// kept too (24 tiles), so no later pass re-evaluates a transcendental. hook(l, ot, h4) runs for
// every hidden out tile (l = 0..3). V[c] (LDS, 16 floats) receives the output for sample c.
// The pass with its fragments already in registers (a chain kernel issues the loads of its first
// pass before the row gathers, so their latency overlaps the gathers).
// WANT_V = false: the pass only for its sin / cos tiles (the actor chain needs dV/ds', not V)
template <bool WANT_V = true, typename Hook>
__device__ void critic_forward_tile_f(const CriticFwdFrags& F, const NetView& N, const float4* X0, float4* Cs,
                                      float4* Hs, float4* H, float4* red, float* V, const Lane& L, Hook&& hook);

template <bool WANT_V = true, typename Hook>
__device__ void critic_forward_tile(const NetView& N, const float4* X0, float4* Cs, float4* Hs, float4* H, float4* red,
                                    float* V, const Lane& L, Hook&& hook) {
  CriticFwdFrags F;
  PSTAMP(27);
  F.load<true>(N, L);
  if (WANT_V) F.load_last(N, L);
#ifdef CACTO_STAMPS_LOADWAIT
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PSTAMP(28);
#endif
  critic_forward_tile_f<WANT_V>(F, N, X0, Cs, Hs, H, red, V, L, hook);
}

template <bool WANT_V, typename Hook>
__device__ void critic_forward_tile_f(const CriticFwdFrags& F, const NetView& N, const float4* X0, float4* Cs,
                                      float4* Hs, float4* H, float4* red, float* V, const Lane& L, Hook&& hook) {
  const float4* in = X0;
  auto epi = [&](int l, float4* out) {
    return [&, l, out](int ot, floatx4 acc) {
      float h[4], c[4];
      const float z[4] = {acc[0], acc[1], acc[2], acc[3]};  // x W + b
#ifdef CACTO_CRITIC_ELU
      if ((N.t.act >> l) & 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) elu_pair(z[r], &h[r], &c[r]);
      } else
#endif
      {
        fast_sincos4(z, h, c);
      }
      const float4 h4 = make_float4(h[0], h[1], h[2], h[3]);
      if (Cs) Cs[(ZOFF[l] + ot) * 64 + L.lane] = make_float4(c[0], c[1], c[2], c[3]);
      out[ot * 64 + L.lane] = h4;
      hook(l, ot, h4);
    };
  };
  float4* out = Hs ? Hs + ZOFF[0] * 64 : H;
  PSTAMP(16);
  F.f0.run(in, N.biasp(0), 4, L.wave, L.lane, epi(0, out));
  PSTAMP(17);
  __syncthreads();
  PSTAMP(18);
  in = out;
  out = Hs ? Hs + ZOFF[1] * 64 : H + 8 * 64;
  F.f1.run(in, N.biasp(1), 4, L.wave, L.lane, epi(1, out));
  PSTAMP(19);
  __syncthreads();
  PSTAMP(20);
  in = out;
  out = Hs ? Hs + ZOFF[2] * 64 : H;
  F.f2.run(in, N.biasp(2), 8, L.wave, L.lane, epi(2, out));
  PSTAMP(21);
  __syncthreads();
  PSTAMP(22);
  in = out;
  out = Hs ? Hs + ZOFF[3] * 64 : H + 8 * 64;
  F.f3.run(in, N.biasp(3), 8, L.wave, L.lane, epi(3, out));
  PSTAMP(23);
  __syncthreads();
  PSTAMP(24);
  if (WANT_V) {
    F.f4.run(8, out, red, L, N.biasp(4), [&](int, floatx4 acc) {
      if (L.g == 0) V[L.c] = acc[0];
    });
    PSTAMP(25);
    __syncthreads();
  }
  PSTAMP(26);
}

// Actor forward; Z1/Z2 (16 tiles each) kept when non-null, h tiles in H (2 x 16 tiles).
// A[c * na + f] (LDS) receives the action.
// F1 (optional): layer 1's fragments preloaded (the 256-wide first layer: KT = 1, OT = 16).
template <typename Hook>
__device__ void actor_forward_tile(const NetView& N, int na, const float4* X0, float4* Z, float4* H, float4* red,
                                   float* A, const Lane& L, Hook&& hook, const Frag1<4>* F1 = nullptr) {
  const float4* in = X0;
  for (int l = 0; l < 2; ++l) {
    float4* out = H + l * 16 * 64;
    auto epi = [&](int ot, floatx4 acc) {
      float z[4], h[4];
      for (int r = 0; r < 4; ++r) {
        z[r] = acc[r];  // x W + b
        h[r] = z[r] > 0.f ? z[r] : fmul(z[r], 0.3f);  // LeakyReLU(alpha=0.3)
      }
      const float4 z4 = make_float4(z[0], z[1], z[2], z[3]);
      const float4 h4 = make_float4(h[0], h[1], h[2], h[3]);
      if (Z) Z[(l * 16 + ot) * 64 + L.lane] = z4;
      out[ot * 64 + L.lane] = h4;
      hook(l, ot, z4, h4);
    };
    // the actor's fixed shape (NeuralNetwork.py: ns -> 256 -> 256 -> na, ns <= 16, na <= 16):
    // layer 1 KT = 1, layer 2 KT = 16, 16 out tiles each (4 per wave)
    if (l == 0 && F1)
      mm_layer1_pre<4>(*F1, in, L.wave, L.lane, epi, N.biasp(0));
    else if (l == 0)
      mm_layer_t<1>(N.fwd(0), 4 * CACTO_NWAVES, in, L.wave, L.lane, epi, N.biasp(0));
    else
      mm_layer_t<16>(N.fwd(1), 4 * CACTO_NWAVES, in, L.wave, L.lane, epi, N.biasp(1));
    __syncthreads();
    PSTAMP(10 + l);
    in = out;
  }
  mm_single_tile(N.fwd(2), 4 * CACTO_NWAVES, in, red, L, [&](int, floatx4 acc) {
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * L.g + r;
      if (f < na) A[L.c * na + f] = acc[r];
    }
  }, N.biasp(2), na);
  __syncthreads();
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

// normalize_feature / normalize_backward for this lane's features 4g + r, with the norms loaded
// once into registers (at kernel entry, overlapping the row gathers) instead of from the system
// parameters after each barrier. Same arithmetic as the functions in mlp.h.
struct Norm4 {
  float n[4];
  float nT;
  int ns;
  bool on;
  __device__ __forceinline__ Norm4(const cacto_sys_params& p, const Lane& L) {
    ns = p.nb_state;
    on = p.normalize != 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * L.g + r;
      n[r] = (float)p.state_norm[min(f, ns - 1)];  // branch-free; features >= ns never use it
    }
    nT = (float)p.state_norm[ns - 1];
    f0 = 4 * L.g;
  }
  int f0;
  __device__ __forceinline__ float forward(int r, float s) const {
    if (!on) return s;
    if (f0 + r == ns - 1) return fsub(fmul(fdiv(s, nT), 2.0f), 1.0f);
    return fdiv(s, n[r]);
  }
  __device__ __forceinline__ float backward(int r, float g) const {
    if (!on) return g;
    if (f0 + r == ns - 1) return fdiv(fmul(g, 2.0f), nT);
    return fdiv(g, n[r]);
  }
  // fill_input_tile with the preloaded norms (wave 0)
  __device__ __forceinline__ void fill(const float* st, float4* X, const Lane& L) const {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = f0 + r < ns ? forward(r, st[L.c * 16 + f0 + r]) : 0.f;
    X[L.lane] = make_float4(v[0], v[1], v[2], v[3]);
  }
};

// Critic input gradient (first backward pass) from the cos tiles Cs: G[4] = W5,
// D[l] = G[l+1] cos z_l, G[l] = D[l] W_l^T. Results: G tiles (G1 at 0, G2 at 4, G3 at 8; 16 tiles)
// when Gs != nullptr, D via hookD(l, ot, lane, d4), and dV/dx0 in G0 (1 tile).
template <typename HookD>
__device__ void critic_first_backward(const NetView& N, const float4* Cs, float4* P /* 2 x 8 tiles */, float4* Gs,
                                      float4* G0, float4* red, const Lane& L, HookD&& hookD) {
  const int goff[4] = {0, 0, 4, 8};  // G[l] tile offsets for l = 1..3
  CriticBwdFrags F;
  F.load(N, L);
  // D3 = W5[:,0] * cos(z3): out tiles wave and wave + 4, the lane's 4 rows
  float4* D = P;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ot = L.wave + 4 * t;
    const float4 c = Cs[(ZOFF[3] + ot) * 64 + L.lane];
    const float4 w = F.w5[t];
    const float4 d4 = make_float4(fmul(w.x, c.x), fmul(w.y, c.y), fmul(w.z, c.z), fmul(w.w, c.w));
    D[ot * 64 + L.lane] = d4;
    hookD(3, ot, L.lane, d4);
  }
  __syncthreads();
  auto epi = [&](int l, float4* Dn) {
    return [&, l, Dn](int it, floatx4 acc) {
      const float4 gl = f4(acc);
      if (Gs) Gs[(goff[l] + it) * 64 + L.lane] = gl;
      const float4 c = Cs[(ZOFF[l - 1] + it) * 64 + L.lane];
      const float4 d4 = make_float4(fmul(gl.x, c.x), fmul(gl.y, c.y), fmul(gl.z, c.z), fmul(gl.w, c.w));
      Dn[it * 64 + L.lane] = d4;
      hookD(l - 1, it, L.lane, d4);
    };
  };
  // G[l] = D[l] W_l^T : M tiles = KT[l] (in of layer l), K tiles = OT[l]
  float4* Dn = P + 8 * 64;
  F.g3.run(D, nullptr, 8, L.wave, L.lane, epi(3, Dn));
  __syncthreads();
  D = Dn;
  Dn = P;
  F.g2.run(D, nullptr, 4, L.wave, L.lane, epi(2, Dn));
  __syncthreads();
  D = Dn;
  Dn = P + 8 * 64;
  F.g1.run(D, nullptr, 4, L.wave, L.lane, epi(1, Dn));
  __syncthreads();
  D = Dn;
  // G[0] = D0 W_1^T (one tile: ns <= 16)
  F.g0.run(4, D, red, L, nullptr, [&](int, floatx4 acc) { G0[L.lane] = f4(acc); });
  __syncthreads();
}

}  // namespace cacto
