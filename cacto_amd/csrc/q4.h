// 4-sample tile machinery ("q4") for the learner chains at the batch sizes every reference conf
// trains with (B = 64 / 128): v_mfma_f32_4x4x1_16b_f32 with the A operand broadcast in groups of
// four blocks (CBSZ = 2), so one instruction is 4 samples x 16 output features x 4 k-steps and a
// 16-feature out tile of a layer costs a quarter of the 16x16x4 form's cycles on a quarter of the
// samples. A batch of 128 then runs as 32 + 32 workgroups instead of 8 + 8.
//
// Activation layout in LDS ("F4"): float X[4 f + i] = x[feature f][sample i], i < 4 — one float4
// per feature. The k-tile kt of X (features 16 kt .. 16 kt + 15) is the 64 floats at 64 kt, and
// lane l = 16 g + 4 a + i reading X[64 kt + l] holds x[16 kt + 4 g + a][i]: exactly the A operand
// of the four MFMAs below, so an operand load is one conflict-free ds_read_b32.
//
// Weights: the packed forward / transposed images of mlp.h, unchanged. Block (ot, kt), component
// j, lane (g, c) holds W[16 kt + 4 g + j][16 ot + c]. Read as the B operand of the 4x4x1 form,
// lane 4 b + jj with b = 4 g + (c >> 2), jj = c & 3: block b multiplies k = 16 kt + 4 g + j into
// features 16 ot + 4 (c >> 2) + jj. The four blocks 4 g .. 4 g + 3 share that k, so MFMA j
// broadcasts the A operand of block 4 g + j (CBSZ = 2, ABID = j) to them:
//     acc_j[lane (g, c)][i] += x[16 kt + 4 g + j][i] * W[16 kt + 4 g + j][16 ot + c]
// After all k-tiles, lane (g, c) holds, for feature 16 ot + c and every sample i, the partial sum
// over the k-phase k = 4 g + j (mod 16). q4_reduce sums the four phases across the lane rows and
// leaves each lane ONE element: feature 16 ot + c, sample g (a reduce-scatter: two
// v_permlane32_swap and one v_permlane16_swap, all VALU). Its F4 index is q4e(ot, lane) — the 64
// lanes of a tile write a permutation of 64 consecutive floats (conflict-free).
#pragma once

#include "mlp.h"

namespace cacto {

constexpr int Q4_TILE = 4;  // samples per workgroup tile

// F4 index of the element lane `lane` holds after q4_reduce of out tile ot
__device__ __forceinline__ int q4e(int ot, int lane) { return 64 * ot + 4 * (lane & 15) + (lane >> 4); }

template <int J>
__device__ __forceinline__ floatx4 mfma_q4(float x, float w, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(x, w, c, 2, J, 0);
}

// one k-tile: x = X[64 kt + lane], w = the packed block; the four k-steps go to four accumulators
__device__ __forceinline__ void q4_ktile(float x, const float4& w, floatx4& c0, floatx4& c1, floatx4& c2,
                                         floatx4& c3) {
  c0 = mfma_q4<0>(x, w.x, c0);
  c1 = mfma_q4<1>(x, w.y, c1);
  c2 = mfma_q4<2>(x, w.z, c2);
  c3 = mfma_q4<3>(x, w.w, c3);
}

// Sum the four k-phases (lane rows g = 0..3) of the per-sample partials a[i]; lane (g, c) returns
// sample g's total. Every lane forms (p0 + p2) + (p1 + p3) (up to operand order), so the result
// does not depend on the row.
__device__ __forceinline__ float q4_reduce(const floatx4& a) {
  // lane bit 5: the low half keeps samples 0 / 1 (adding lane + 32), the high half 2 / 3
  const auto r02 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[0]), __float_as_uint(a[2]), false, false);
  const auto r13 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[1]), __float_as_uint(a[3]), false, false);
  const float s02 = __uint_as_float(r02[0]) + __uint_as_float(r02[1]);
  const float s13 = __uint_as_float(r13[0]) + __uint_as_float(r13[1]);
  // lane bit 4: even rows keep samples 0 / 2, odd rows 1 / 3
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s02), __float_as_uint(s13), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// A panel row element: base[(16 ot + c) * ld + row0 + g] (feature-major panels, sample rows)
__device__ __forceinline__ void q4_store_panel(float* base, int ld, int row0, int ot, int lane, float v) {
  base[(size_t)(16 * ot + (lane & 15)) * ld + row0 + (lane >> 4)] = v;
}

__device__ __forceinline__ float q4_bias(const float* __restrict__ bias, int ot, int lane, int nout) {
  const int f = 16 * ot + (lane & 15);
  return (bias && f < nout) ? bias[f] : 0.f;
}

// A team is NW waves working on one pass (the q4 chains run 8 waves per workgroup, as one team of
// 8 or two teams of 4 doing independent passes side by side); wi is the wave's index in its team.

// A whole layer's fragments for one wave, held in registers: NT out tiles (ot = wi + NW t) x KT
// k-tiles, plus the lane's bias. Loads are branch-free (clamped tile index; see mlp.h Frags).
template <int KT, int NT, int NW = CACTO_NWAVES>
struct Q4Frags {
  float4 a[NT][KT];
  float b[NT];
  template <bool BIAS>
  __device__ __forceinline__ void load(const float4* __restrict__ A, const float* __restrict__ bias, int OT, int nout,
                                       int wi, int lane) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int ot = min(wi + NW * t, OT - 1);
#pragma unroll
      for (int k = 0; k < KT; ++k) a[t][k] = A[((size_t)ot * KT + k) * 64 + lane];
      const int f = 16 * ot + (lane & 15);
      b[t] = BIAS ? bias[min(f, nout - 1)] : 0.f;
      if (f >= nout) b[t] = 0.f;
    }
  }
  // every tile's MFMAs, then the reductions, then the epilogues epi(ot, value) (value + bias
  // with BIAS): the epilogue VALU work overlaps the matrix core's tail
  template <bool BIAS, typename Epi>
  __device__ __forceinline__ void run(const float* X, int OT, int wi, int lane, Epi&& epi) const {
    float x[KT];
#pragma unroll
    for (int k = 0; k < KT; ++k) x[k] = X[64 * k + lane];
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
      if (wi + NW * t < OT) {
#pragma unroll
        for (int k = 0; k < KT; ++k) q4_ktile(x[k], a[t][k], c0, c1, c2, c3);
      }
      acc[t] = (c0 + c1) + (c2 + c3);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int ot = wi + NW * t;
      if (ot < OT) {
        const float v = q4_reduce(acc[t]);
        epi(ot, BIAS ? fadd(v, b[t]) : v);
      }
    }
  }
};

// A single-out-tile layer (OT == 1: the critic's output, the actor's action layer, the critic's
// input gradient): wave wi takes k-tiles wi, wi + NW, ...; the team's partials are summed through
// LDS `red` (NW x 64 floats, the team's own) in wave order by the team's wave 0, which runs the
// epilogue. Contains __syncthreads(): every thread of the workgroup must call run() (two teams
// running a split layer at the same time share the barrier).
template <int NK, int NW = CACTO_NWAVES>
struct Q4Split {
  float4 a[NK];
  float b;
  template <bool BIAS>
  __device__ __forceinline__ void load(const float4* __restrict__ A, int KT, const float* __restrict__ bias, int nout,
                                       int wi, int lane) {
#pragma unroll
    for (int i = 0; i < NK; ++i) a[i] = A[min(wi + NW * i, KT - 1) * 64 + lane];
    const int f = lane & 15;
    b = BIAS ? bias[min(f, nout - 1)] : 0.f;
    if (f >= nout) b = 0.f;
  }
  template <bool BIAS, typename Epi>
  __device__ __forceinline__ void run(int KT, const float* X, float* red, int wi, int lane, Epi&& epi) const {
    floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
#pragma unroll
    for (int i = 0; i < NK; ++i) {
      const int kt = wi + NW * i;
      if (kt < KT) q4_ktile(X[64 * kt + lane], a[i], c0, c1, c2, c3);
    }
    red[wi * 64 + lane] = q4_reduce((c0 + c1) + (c2 + c3));
    __syncthreads();
    if (wi == 0) {
      float s = red[lane];
#pragma unroll
      for (int w = 1; w < NW; ++w) s += red[w * 64 + lane];
      epi(0, BIAS ? fadd(s, b) : s);
    }
  }
};

// The actor's 256-wide layers (OT = 16: out tiles wi + NW t) with a wave's tiles taken in pairs:
// both tiles' KT fragment blocks are issued together (branch-free), so a wave waits for one memory
// latency per pair instead of one per tile (the weights come from the memory-side cache after every
// Adam step; a one-tile-ahead prefetch still pays that latency per tile). The first pair is issued
// by the caller a phase early (P0); with 8 waves it is the wave's only pair.
template <int KT, int NW = CACTO_NWAVES>
struct Q4Pair {
  static constexpr int NP = 16 / (2 * NW);  // pairs per wave
  float4 a[2][KT];
  __device__ __forceinline__ void load(const float4* __restrict__ A, int p, int wi, int lane) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ot = wi + NW * (2 * p + u);
#pragma unroll
      for (int k = 0; k < KT; ++k) a[u][k] = A[((size_t)ot * KT + k) * 64 + lane];
    }
  }
};

template <int KT, bool BIAS, int NW, typename Epi>
__device__ __forceinline__ void q4_layer_pairs(const float4* __restrict__ A, const float* X, int wi, int lane,
                                               Epi&& epi, const float* __restrict__ bias, const Q4Pair<KT, NW>& P0) {
  constexpr int NP = Q4Pair<KT, NW>::NP;
  float x[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) x[k] = X[64 * k + lane];
  float bv[2 * NP];
#pragma unroll
  for (int t = 0; t < 2 * NP; ++t) bv[t] = BIAS ? bias[16 * (wi + NW * t) + (lane & 15)] : 0.f;
  Q4Pair<KT, NW> P = P0;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    floatx4 acc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
#pragma unroll
      for (int k = 0; k < KT; ++k) q4_ktile(x[k], P.a[u][k], c0, c1, c2, c3);
      acc[u] = (c0 + c1) + (c2 + c3);
    }
    if (p + 1 < NP) P.load(A, p + 1, wi, lane);  // the next pair, in flight during this pair's epilogue
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const float v = q4_reduce(acc[u]);
      epi(wi + NW * (2 * p + u), BIAS ? fadd(v, bv[2 * p + u]) : v);
    }
  }
}

}  // namespace cacto
