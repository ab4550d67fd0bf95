// MFMA (v_mfma_f32_16x16x4_f32) tile machinery for the CACTO actor and critic MLPs.
//
// Orientation: features are the MFMA M dimension, samples the N dimension (16 samples per tile),
// so a layer computes out^T[OUT x 16] = W^T[OUT x IN] · in^T[IN x 16].
//
// Activation tile (16 features x 16 samples) = 64 lanes x float4, lane l = g*16 + c holds
// features 4g..4g+3 of sample c. This is exactly the C/D layout of the 16x16 MFMA (row = 4g + r,
// col = c), and — reading component j as k-step j — the B-operand layout for k = 4g + j, so a
// layer's output tile feeds the next layer with no lane movement (one ds_write_b128 /
// ds_read_b128 per lane, conflict-free).
//
// Packed weights ("pk", forward): for out-tile ot and k-tile kt, lane l = (g, c), component j:
//     A[i = c][k = g] of MFMA j  =  W[16kt + 4g + j][16ot + c]      (zero-padded)
// stored at ((pkoff_l + ot*KT + kt) * 64 + l) * 4 + j — one coalesced 1 KiB dwordx4 wave load per
// 4 MFMAs. Transposed ("pkT", input-gradient g_in = W · d_out): block (it, kt):
//     A[i = c][k = g] of MFMA j  =  W[16it + c][16kt + 4g + j]
// at ((pktbase + pkoff_l + it*OT + kt) * 64 + l) * 4 + j.
#pragma once

#include "common.h"

namespace cacto {

constexpr int ACTOR_LAYERS = 3;
constexpr int CRITIC_LAYERS = 5;
constexpr int MAX_LAYERS = 5;

struct NetTopo {
  int L;
  int in[MAX_LAYERS], out[MAX_LAYERS];
  int KT[MAX_LAYERS], OT[MAX_LAYERS];  // k-tiles (= in tiles), out tiles
  int woff[MAX_LAYERS], boff[MAX_LAYERS];
  int pkoff[MAX_LAYERS];  // in blocks
  int blocks;             // pk blocks (pkT region has the same count, starts at `blocks`)
  int params;
  int act;                // critic: bit l set = hidden layer l is elu (critic_type 'sine-elu'), else sine
};

inline NetTopo make_topo(int net, int ns, int na) {
  NetTopo t{};
  const int actor_dims[4] = {ns, 256, 256, na};
  const int critic_dims[6] = {ns, 64, 64, 128, 128, 1};
  const int* d = net == CACTO_NET_ACTOR ? actor_dims : critic_dims;
  t.L = net == CACTO_NET_ACTOR ? ACTOR_LAYERS : CRITIC_LAYERS;
  int off = 0, blk = 0;
  for (int l = 0; l < t.L; ++l) {
    t.in[l] = d[l];
    t.out[l] = d[l + 1];
    t.KT[l] = (d[l] + 15) / 16;
    t.OT[l] = (d[l + 1] + 15) / 16;
    t.woff[l] = off;
    off += d[l] * d[l + 1];
    t.boff[l] = off;
    off += d[l + 1];
    t.pkoff[l] = blk;
    blk += t.KT[l] * t.OT[l];
  }
  t.blocks = blk;
  t.params = off;
  return t;
}

// Device view of one network: flat Keras params (biases, W5 column) + packed fragments.
struct NetView {
  const float* flat;
  const float4* pk;  // base of packed buffer (pk blocks then pkT blocks)
  NetTopo t;
  __device__ __forceinline__ const float4* fwd(int l) const { return pk + (size_t)t.pkoff[l] * 64; }
  __device__ __forceinline__ const float4* bwd(int l) const {
    return pk + (size_t)(t.blocks + t.pkoff[l]) * 64;
  }
  __device__ __forceinline__ float bias(int l, int f) const { return flat[t.boff[l] + f]; }
  __device__ __forceinline__ const float* biasp(int l) const { return flat + t.boff[l]; }
  __device__ __forceinline__ float w(int l, int i, int o) const { return flat[t.woff[l] + i * t.out[l] + o]; }
};

// Fragment block blk (64 lanes x float4, wave-uniform index) of a packed weight image A (a
// kernel-argument pointer, so wave-uniform too) by a buffer load: the block's byte offset goes in
// an SGPR and the lane's in one VGPR shared by every load, so a pass that issues all its fragment
// loads up front holds no 64-bit address per load in VGPRs. Same data as A[blk * 64 + lane].
__device__ __forceinline__ float4 ldfrag(const float4* __restrict__ A, int blk, int lane) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(A), (short)0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, blk * 1024, 0));
}
// the wave index as a value the compiler knows is wave-uniform (SGPR), for fragment indices
__device__ __forceinline__ int uniform_wave(int wave) { return __builtin_amdgcn_readfirstlane(wave); }

// The 4 bias values of out tile ot for this lane (features 16 ot + 4 g + r), or zeros.
__device__ __forceinline__ float4 tile_bias(const float* __restrict__ bias, int ot, int lane) {
  if (!bias) return make_float4(0.f, 0.f, 0.f, 0.f);
  const float* b = bias + 16 * ot + 4 * (lane >> 4);
  return make_float4(b[0], b[1], b[2], b[3]);
}

__device__ __forceinline__ floatx4 add_bias(floatx4 acc, const float* bias, float4 b) {
  if (bias) {
    acc[0] = fadd(acc[0], b.x);
    acc[1] = fadd(acc[1], b.y);
    acc[2] = fadd(acc[2], b.z);
    acc[3] = fadd(acc[3], b.w);
  }
  return acc;
}

// out-tile loop of one layer: each wave takes out tiles ot = wave, wave+4, ...; X = LDS tiles.
// All KT weight fragments of a tile (and its biases, when `bias` is given: the epilogue then
// receives acc + b) are issued before its MFMAs, and the next tile's are in flight while the
// current tile's MFMAs run (A comes from L2: the load latency is paid once per layer, not once
// per k-step, and no epilogue waits on a global load).
template <int KT, typename Epi>
__device__ __forceinline__ void mm_layer_t(const float4* __restrict__ A, int OT, const float4* X, int wave, int lane,
                                           Epi&& epi, const float* __restrict__ bias) {
  int ot = uniform_wave(wave);
  if (ot >= OT) return;
  float4 a[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) a[k] = ldfrag(A, ot * KT + k, lane);
  float4 bv = tile_bias(bias, ot, lane);
  while (true) {
    const int nxt = ot + CACTO_NWAVES;
    float4 an[KT], bn = bv;
    if (nxt < OT) {
#pragma unroll
      for (int k = 0; k < KT; ++k) an[k] = ldfrag(A, nxt * KT + k, lane);
      bn = tile_bias(bias, nxt, lane);
    }
    // the 4 k-steps of a fragment block go to 4 independent accumulators (issue-bound chain)
    floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const float4 b = X[k * 64 + lane];
      c0 = mfma4(a[k].x, b.x, c0);
      c1 = mfma4(a[k].y, b.y, c1);
      c2 = mfma4(a[k].z, b.z, c2);
      c3 = mfma4(a[k].w, b.w, c3);
    }
    epi(ot, add_bias((c0 + c1) + (c2 + c3), bias, bv));
    if (nxt >= OT) break;
    ot = nxt;
    bv = bn;
#pragma unroll
    for (int k = 0; k < KT; ++k) a[k] = an[k];
  }
}

// A whole layer's weight fragments for one wave, held in registers: NT out tiles
// (ot = wave + 4 t) x KT k-tiles, plus their biases. A pass over a fixed-shape network (the
// critic) loads every layer's fragments up front, so the L2/HBM latency is paid once per pass
// instead of once per layer behind each barrier.
//
// The loads are branch-free (tile index clamped, bias presence a template argument): a load
// under a branch makes the compiler's waitcnt tracking fall back to vmcnt(0) at the join, which
// would serialise the prefetch.
template <int KT, int NT>
struct Frags {
  float4 a[NT][KT];
  float4 b[NT];
  template <bool BIAS>
  __device__ __forceinline__ void load(const float4* __restrict__ A, const float* __restrict__ bias, int OT, int wave,
                                       int lane) {
    wave = uniform_wave(wave);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int ot = min(wave + CACTO_NWAVES * t, OT - 1);
#pragma unroll
      for (int k = 0; k < KT; ++k) a[t][k] = ldfrag(A, ot * KT + k, lane);
      if (BIAS) {
        const float* bp = bias + 16 * ot + 4 * (lane >> 4);
        b[t] = make_float4(bp[0], bp[1], bp[2], bp[3]);
      } else {
        b[t] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  // same arithmetic as mm_layer_t: 4 accumulators over the k-steps j, then (c0 + c1) + (c2 + c3)
  // All tiles' MFMAs are issued before the first epilogue, so the epilogue VALU work of tile t
  // overlaps the matrix core's work on tile t + 1.
  template <typename Epi>
  __device__ __forceinline__ void run(const float4* X, const float* bias, int OT, int wave, int lane,
                                      Epi&& epi) const {
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
      if (wave + CACTO_NWAVES * t < OT) {
#pragma unroll
        for (int k = 0; k < KT; ++k) {
          const float4 x = X[k * 64 + lane];
          c0 = mfma4(a[t][k].x, x.x, c0);
          c1 = mfma4(a[t][k].y, x.y, c1);
          c2 = mfma4(a[t][k].z, x.z, c2);
          c3 = mfma4(a[t][k].w, x.w, c3);
        }
      }
      acc[t] = (c0 + c1) + (c2 + c3);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int ot = wave + CACTO_NWAVES * t;
      if (ot < OT) epi(ot, add_bias(acc[t], bias, b[t]));
    }
  }
};

// Preloaded fragments (a caller issues them a phase early, so the L2 latency hides behind other
// work; the in-order vmcnt means they should be issued after any load the intervening phase waits
// for). Same arithmetic as mm_layer_t.
//   KT == 1 layers (OT = 4 * NT): every out tile's single fragment block and bias, no loads inside.
template <int NT>
struct Frag1 {
  float4 a[NT], b[NT];
  __device__ __forceinline__ void load(const float4* __restrict__ A, const float* __restrict__ bias, int wave,
                                       int lane) {
    wave = uniform_wave(wave);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      a[t] = ldfrag(A, wave + CACTO_NWAVES * t, lane);
      b[t] = tile_bias(bias, wave + CACTO_NWAVES * t, lane);
    }
  }
};
template <int NT, typename Epi>
__device__ __forceinline__ void mm_layer1_pre(const Frag1<NT>& F, const float4* X, int wave, int lane, Epi&& epi,
                                              const float* __restrict__ bias) {
  const float4 x = X[lane];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
    c0 = mfma4(F.a[t].x, x.x, c0);
    c1 = mfma4(F.a[t].y, x.y, c1);
    c2 = mfma4(F.a[t].z, x.z, c2);
    c3 = mfma4(F.a[t].w, x.w, c3);
    epi(wave + CACTO_NWAVES * t, add_bias((c0 + c1) + (c2 + c3), bias, F.b[t]));
  }
}
//   the first out tile's KT fragment blocks (no bias), for mm_layer_t_pre below
template <int KT>
struct FragTile {
  float4 a[KT];
  __device__ __forceinline__ void load(const float4* __restrict__ A, int wave, int lane) {
    wave = uniform_wave(wave);
#pragma unroll
    for (int k = 0; k < KT; ++k) a[k] = ldfrag(A, wave * KT + k, lane);
  }
};
// mm_layer_t (no bias) with the first tile's fragments preloaded
template <int KT, typename Epi>
__device__ __forceinline__ void mm_layer_t_pre(const FragTile<KT>& F0, const float4* __restrict__ A, int OT,
                                               const float4* X, int wave, int lane, Epi&& epi) {
  int ot = uniform_wave(wave);
  if (ot >= OT) return;
  float4 a[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) a[k] = F0.a[k];
  while (true) {
    const int nxt = ot + CACTO_NWAVES;
    float4 an[KT];
    if (nxt < OT) {
#pragma unroll
      for (int k = 0; k < KT; ++k) an[k] = ldfrag(A, nxt * KT + k, lane);
    }
    floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const float4 b = X[k * 64 + lane];
      c0 = mfma4(a[k].x, b.x, c0);
      c1 = mfma4(a[k].y, b.y, c1);
      c2 = mfma4(a[k].z, b.z, c2);
      c3 = mfma4(a[k].w, b.w, c3);
    }
    epi(ot, (c0 + c1) + (c2 + c3));
    if (nxt >= OT) break;
    ot = nxt;
#pragma unroll
    for (int k = 0; k < KT; ++k) a[k] = an[k];
  }
}

// mm_layer_t_pre for a layer of exactly 4 NT out tiles (NT per wave), the wave's NT x KT fragments
// streamed through a ring of R registers: fragment f = t KT + k is issued R fragments before its
// MFMAs (the first KT come preloaded), so R, not 2 KT, fragments are live. Same arithmetic.
template <int KT, int NT, int R, typename Epi>
__device__ __forceinline__ void mm_layer_ring(const FragTile<KT>& F0, const float4* __restrict__ A, const float4* X,
                                              int wave, int lane, Epi&& epi) {
  static_assert(R >= KT && R <= NT * KT, "ring size");
  constexpr int NF = NT * KT;
  wave = uniform_wave(wave);
  float4 ring[R];
#pragma unroll
  for (int f = 0; f < R; ++f)
    ring[f] = f < KT ? F0.a[f] : ldfrag(A, (wave + CACTO_NWAVES * (f / KT)) * KT + f % KT, lane);
  floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int k = f % KT;
    if (k == 0) c0 = c1 = c2 = c3 = floatx4{0.f, 0.f, 0.f, 0.f};
    const float4 b = X[k * 64 + lane];
    const float4 a = ring[f % R];
    c0 = mfma4(a.x, b.x, c0);
    c1 = mfma4(a.y, b.y, c1);
    c2 = mfma4(a.z, b.z, c2);
    c3 = mfma4(a.w, b.w, c3);
    if (f + R < NF) ring[f % R] = ldfrag(A, (wave + CACTO_NWAVES * ((f + R) / KT)) * KT + (f + R) % KT, lane);
    if (k == KT - 1) epi(wave + CACTO_NWAVES * (f / KT), (c0 + c1) + (c2 + c3));
  }
}

template <typename Epi>
__device__ __forceinline__ void mm_layer(const float4* __restrict__ A, int OT, int KT, const float4* X, int wave,
                                         int lane, Epi&& epi, const float* __restrict__ bias = nullptr) {
  switch (KT) {
    case 1: mm_layer_t<1>(A, OT, X, wave, lane, epi, bias); break;
    case 4: mm_layer_t<4>(A, OT, X, wave, lane, epi, bias); break;
    case 8: mm_layer_t<8>(A, OT, X, wave, lane, epi, bias); break;
    case 16: mm_layer_t<16>(A, OT, X, wave, lane, epi, bias); break;
    default:
      for (int ot = wave; ot < OT; ot += CACTO_NWAVES) {
        const float4 bv = tile_bias(bias, ot, lane);
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < KT; ++kt) acc = mfma_block(A[((size_t)ot * KT + kt) * 64 + lane], X[kt * 64 + lane], acc);
        epi(ot, add_bias(acc, bias, bv));
      }
  }
}

// utils.py:17-24 in float32 (TF ops: RealDiv, then *2 - 1 for the time column).
__device__ __forceinline__ float normalize_feature(const cacto_sys_params& p, int f, float s) {
  if (!p.normalize) return s;
  const int ns = p.nb_state;
  if (f == ns - 1) return fsub(fmul(fdiv(s, (float)p.state_norm[ns - 1]), 2.0f), 1.0f);
  return fdiv(s, (float)p.state_norm[f]);
}

// d normalize / d s applied to an upstream gradient (RealDiv grad: grad / y; time: (grad*2)/nT).
__device__ __forceinline__ float normalize_backward(const cacto_sys_params& p, int f, float g) {
  if (!p.normalize) return g;
  const int ns = p.nb_state;
  if (f == ns - 1) return fdiv(fmul(g, 2.0f), (float)p.state_norm[ns - 1]);
  return fdiv(g, (float)p.state_norm[f]);
}

// element (f, c) of a tile
__device__ __forceinline__ int tile_lane(int f) { return (f >> 2) * 16; }

}  // namespace cacto
