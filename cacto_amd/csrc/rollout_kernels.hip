// Persistent rollout kernel (K18: RL_AC.create_TO_init RL.py:197-233 / PLOT.rollout
// plot_utils.py:245-279): actor MFMA + float64 dynamics / reward / EE per step, all steps in-kernel.
//
// Scheduling. Episode lengths are spread (NSTEPS - int(t/dt), e.g. 1..200 for the double
// integrator), so a workgroup that ran one fixed tile of episodes would idle once its shortest ones
// end and the longest tile would set the launch time. Here a workgroup owns SL = 4*NG episode
// *slots* and a queue of episodes: ranks of the length-sorted order are dealt to the G workgroups
// in snake order (k*G + w for even rounds k, k*G + G-1-w for odd), and a slot whose episode ends
// takes the next queue entry at the step boundary (slots in lane order: deterministic). The host
// picks NG so there are about two episodes per slot; every slot then runs ~T_max steps.
//
// Actor on v_mfma_f32_4x4x1_16b_f32 with A-operand broadcast. The 16x16x4 form needs 16 samples
// per MFMA; the 4x4x1 16-block form runs at the same rate with 4 samples per instruction, so a
// workgroup can hold 8 (or 4, 16) episodes at full MFMA rate. Per instruction: blocks b = 16 groups
// of 4 output features (lane 4b+j <-> feature 64*wave + 4b + j, the B operand = one weight row
// segment W[k][64 wave + lane]), the A operand (4 samples of activation k) broadcast from block q
// (CBSZ = 4, ABID = q), so one VGPR of activations (lane 4q+i = x[sample i][k0 + q]) feeds 16
// consecutive k-steps. The result lands with the feature on the lane and the 4 samples in the
// 4 accumulator registers. Layer-2 rows stay in registers for the whole launch (weight
// stationary) or in LDS (RoSplit); the 256 -> na output layer is a VALU dot product + lane
// reduction. Numerics: every dot product is an f32 FMA chain (MFMA) — F32 tolerance as before.
#include <cstdlib>
#include <utility>

#include "net_common.h"

#ifdef CACTO_STAMPS
__device__ unsigned long long g_rstamps[20];
__device__ unsigned long long g_ttacc[1024 * 2 * 2 * 10];  // [workgroup][team][wave 0/1][phase 0-8, steps]
__device__ unsigned long long g_wsacc[1024 * 8 * 7];  // k_rollout_ks: [workgroup][wave][phase 0-5, steps]
#define RSTAMP(k)                                                                     \
  do {                                                                                \
    if (blockIdx.x == 0 && threadIdx.x == 0 && it == 20) g_rstamps[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define RSTAMP(k) \
  do {            \
  } while (0)
#endif

namespace cacto {

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// D[feature lane][sample r] += x[sample r][k0 + Q] * w[k0 + Q][feature lane]
template <int Q>
__device__ __forceinline__ floatx4 mfma_bc(float x, float w, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(x, w, c, 4, Q, 0);
}

// Layer-2 weight rows by residence: [0, REGK) registers (the whole launch), [REGK, REGK + LDSK)
// LDS, the rest streamed from global memory (L2-resident) at every step. The float64 chain
// dynamics of the manipulator / UR5 need many registers, so those systems keep fewer rows in
// registers (and the UR5 streams some); the LDS share is what fits beside the step buffers.
template <int NJ, int NG>
#ifndef RO_DYN_IN_ACTOR
// 1: the lane RNEA / CRBA inside the actor's layer-2 block (the scheduler keeps them after the MFMA
// stream, and the layer-2 barrier then waits for them): 124.5 M against 132.1 M env-steps/s (UR5,
// 2048 episodes) for the dynamics after the actor, so off
#define RO_DYN_IN_ACTOR 0
#endif
#ifndef RO_STREAM_PF
#define RO_STREAM_PF 2  // ro_layer2's L2-streamed weight rows loaded two 16-row blocks ahead (one at NG > 1)
#endif
#ifndef RO_CHAIN6_LDSK1
#define RO_CHAIN6_LDSK1 128
#endif
struct RoSplit {
#ifndef RO_CHAIN6_REGK1
#define RO_CHAIN6_REGK1 128  // the 6-joint chain at one slot group: W2 wholly resident (128 + 128 rows)
#endif
#ifndef RO_CHAIN6_PF
#define RO_CHAIN6_PF 0
#endif
  static constexpr int REGK = NJ <= 2 ? 192 : NJ == 3 ? (NG == 4 ? 160 : 128) : NG == 4 ? 48 : NG == 1 ? RO_CHAIN6_REGK1 : 64;
  static constexpr int LDSK = NJ <= 2 ? 64 : NJ == 3 ? (NG == 4 ? 96 : 128) : NG == 4 ? 80 : NG == 1 ? RO_CHAIN6_LDSK1 : 112;
  static_assert(REGK % 16 == 0 && LDSK % 16 == 0 && REGK + LDSK <= 256, "row split");
};

template <int NG>
struct RoCfg {
  static constexpr int SL = 4 * NG;     // episode slots per workgroup
  static constexpr int GPW = 64 / SL;   // lane groups of SL lanes per wave (env-term fan-out)
  static constexpr int P = 256 / SL;    // threads per slot in the output layer
  static constexpr int H2S = 256 + P;   // h2 row stride: slots of one wave on distinct banks
  static constexpr int H1B = 320;       // h1 floats per (group, 64-k block): 16 q x 20 (padded)
};

template <int NS, int REGK>
struct RoActorRegs {
  float w2[REGK];     // W2[k][64 wave + lane]
  float w1[NS];       // W1[q][64 wave + lane]
  float b1, b2;
};

template <int NG, int NA, int LDSK>
struct RoActorLds {
  float4 w2[LDSK / 4 * 4 * 64];                 // W2[REGK + 4kq + j][64w + lane] at (kq*4 + w)*64 + lane
  float h1[NG * 4 * RoCfg<NG>::H1B];            // layer-1 output, layer-2 broadcast layout
  float h2[RoCfg<NG>::SL * RoCfg<NG>::H2S];     // layer-2 output [slot][feature]
  float w3[NA * 256];                           // W3^T [a][f]
  float b3[8];
  float x0[NG * 64];                            // normalised input: [g][q][i] = x[slot 4g+i][feature q]
  float a[RoCfg<NG>::SL * NA];                  // actions [slot][a]
};

template <int NG, int NS, int NA, int REGK, int LDSK>
__device__ __forceinline__ void ro_load_actor(const NetView& N, const Lane& L, RoActorRegs<NS, REGK>& R,
                                              RoActorLds<NG, NA, LDSK>& W) {
  const float* W1 = N.flat + N.t.woff[0];
  const float* W2 = N.flat + N.t.woff[1];
  const float* W3 = N.flat + N.t.woff[2];
  const int f = 64 * L.wave + L.lane;
#pragma unroll
  for (int k = 0; k < REGK; ++k) R.w2[k] = W2[k * 256 + f];
#pragma unroll
  for (int q = 0; q < NS; ++q) R.w1[q] = W1[q * 256 + f];
  R.b1 = N.bias(0, f);
  R.b2 = N.bias(1, f);
  for (int e = L.tid; e < LDSK * 64; e += CACTO_THREADS) {
    const int lane = e & 63, w = (e >> 6) & 3, kq = e >> 8;
    const int k = REGK + 4 * kq, col = 64 * w + lane;
    W.w2[e] = make_float4(W2[k * 256 + col], W2[(k + 1) * 256 + col], W2[(k + 2) * 256 + col], W2[(k + 3) * 256 + col]);
  }
  for (int e = L.tid; e < NA * 256; e += CACTO_THREADS) W.w3[e] = W3[(e & 255) * NA + (e >> 8)];
  if (L.tid < 8) W.b3[L.tid] = L.tid < NA ? N.bias(2, L.tid) : 0.f;
}

__device__ __forceinline__ float lrelu(float z) { return z > 0.f ? z : fmul(z, 0.3f); }

// v + (v of the lane `off` above): the butterfly level of layer 3 as seen by the lanes that keep
// the result (lane j < off of a segment adds lane j + off, exactly what __shfl_xor gives those
// lanes, so the sums are bit-identical). Offsets below 16 stay inside a 16-lane DPP row and use a
// row shift (a few cycles) instead of a ds_bpermute round trip through the LDS pipe.
__device__ __forceinline__ float add_from_above(float v, int off) {
  float o;
  switch (off) {
    case 8: o = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x108, 0xF, 0xF, true)); break;
    case 4: o = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x104, 0xF, 0xF, true)); break;
    case 2: o = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x102, 0xF, 0xF, true)); break;
    case 1: o = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x101, 0xF, 0xF, true)); break;
    default: o = __shfl_down(v, off); break;
  }
  return v + o;
}

// Layer 2 of the actor (K = 256) for the NG groups of 4 slots: x = h1 (LDS, broadcast layout) ->
// h2 (LDS, [slot][feature]) for the 64 features of this wave. k = 64 kb + 16 v + q; lane 4q+i
// reads {x[i][64kb + 16v + q], v = 0..3}.
// Summation order (every kernel that can run a system forms the same one, so the schedule never
// changes a result): SPLIT (NJ <= 3: the systems k_rollout_ks runs, the planar 3R chain among
// them) — each half of K (k < 128, k >= 128) as two MFMA chains over its even and odd k in
// increasing k, the half's sum = even + odd, h2 = lrelu((lo + hi) + b2) (k_rollout_ks forms the two
// halves on two waves); otherwise (the 6-joint chain) h2 = lrelu((even + odd) + b2) over all of K.
template <int NG, int NS, int REGK, int LDSK, bool PF, bool SPLIT, typename WT>
__device__ __forceinline__ void ro_layer2(const RoActorRegs<NS, REGK>& R, WT& W, const float* __restrict__ W2g,
                                          const Lane& L) {
  using C = RoCfg<NG>;
  floatx4 acc[NG][2];
  const int f = 64 * L.wave + L.lane;
#pragma unroll
  for (int g = 0; g < NG; ++g) acc[g][0] = acc[g][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int rd = (L.lane >> 2) * 20 + 4 * (L.lane & 3);
  // PF: LDS operands one step ahead (the next 64-k block's activations, the next 16-row block of
  // LDS-resident weights), so their latency hides behind the current block's MFMAs. Measured per
  // system (r03): DI +2.5 %, car_park +2 %, manipulator -3 %, UR5 -20 % (its streamed rows and
  // chain dynamics need the registers), so only the systems without streamed rows take it.
  auto lds_w = [&](int k0, float4* wl) {
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) wl[qq] = W.w2[(((k0 - REGK) / 4 + qq) * 4 + L.wave) * 64 + L.lane];
  };
  auto in_lds = [](int k0) { return k0 >= REGK && k0 < REGK + LDSK; };
  // rows streamed from L2 (the 6-joint chain): each 16-row block's loads issued one block ahead,
  // the first at the layer's start, so their latency overlaps the register / LDS blocks' MFMAs
  constexpr bool SPF = REGK + LDSK < 256 && RO_STREAM_PF > 0;
  constexpr int SD = RO_STREAM_PF > 1 && NG == 1 ? 2 : 1;  // blocks in flight (two need 16 more registers)
  constexpr int S0 = REGK + LDSK;               // the first streamed row
  float wgn[SPF ? SD : 1][16];
  auto g_w = [&](int k0, float* wg) {
#pragma unroll
    for (int q = 0; q < 16; ++q) wg[q] = W2g[(k0 + q) * 256 + 64 * L.wave + L.lane];
  };
  if constexpr (SPF) {
#pragma unroll
    for (int d = 0; d < SD; ++d)
      if (S0 + 16 * d < 256) g_w(S0 + 16 * d, wgn[d]);
    __builtin_amdgcn_sched_barrier(0);  // keep the loads here (the scheduler would sink them to their use)
  }
  float4 xn[NG], wn[4];
  if constexpr (PF) {
#pragma unroll
    for (int g = 0; g < NG; ++g) xn[g] = *reinterpret_cast<const float4*>(&W.h1[(g * 4) * C::H1B + rd]);
    if (in_lds(0)) lds_w(0, wn);
  }
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    float4 xv[NG];
    if constexpr (PF) {
#pragma unroll
      for (int g = 0; g < NG; ++g) xv[g] = xn[g];
      if (kb + 1 < 4)
#pragma unroll
        for (int g = 0; g < NG; ++g) xn[g] = *reinterpret_cast<const float4*>(&W.h1[(g * 4 + kb + 1) * C::H1B + rd]);
    } else {
#pragma unroll
      for (int g = 0; g < NG; ++g) xv[g] = *reinterpret_cast<const float4*>(&W.h1[(g * 4 + kb) * C::H1B + rd]);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int k0 = 64 * kb + 16 * v;  // a 16-row block lies in one residence region
      float4 wl[4];
      float wg[16];
      if (in_lds(k0)) {
        if constexpr (PF) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) wl[qq] = wn[qq];
          if (in_lds(k0 + 16)) lds_w(k0 + 16, wn);
        } else {
          lds_w(k0, wl);
        }
      } else if (k0 >= REGK + LDSK) {
        if constexpr (SPF) {
          const int d = ((k0 - S0) / 16) % SD;  // a constant once the loops unroll
#pragma unroll
          for (int q = 0; q < 16; ++q) wg[q] = wgn[d][q];
          if (k0 + 16 * SD < 256) {
            g_w(k0 + 16 * SD, wgn[d]);
            __builtin_amdgcn_sched_barrier(0);
          }
        } else {
          g_w(k0, wg);
        }
      }
      if constexpr (PF)
        if (!in_lds(k0) && in_lds(k0 + 16)) lds_w(k0 + 16, wn);
      static_for<16>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        const int k = k0 + q;
        const float w = k < REGK ? R.w2[k < REGK ? k : 0] : k < REGK + LDSK ? get4(wl[q >> 2], q & 3) : wg[q];
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[g][q & 1] = mfma_bc<q>(get4(xv[g], v), w, acc[g][q & 1]);
      });
    }
    if (SPLIT && kb == 1) {
      // the k < 128 half done: its sum parked in this lane's own h2 slots (no registers held across
      // the second half), the chains restart for k >= 128
#pragma unroll
      for (int g = 0; g < NG; ++g) {
#pragma unroll
        for (int i = 0; i < 4; ++i) W.h2[(4 * g + i) * C::H2S + f] = fadd(acc[g][0][i], acc[g][1][i]);
        acc[g][0] = acc[g][1] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float& h = W.h2[(4 * g + i) * C::H2S + f];
      const float hi = fadd(acc[g][0][i], acc[g][1][i]);
      h = lrelu(fadd(SPLIT ? fadd(h, hi) : hi, R.b2));
    }
}

// Actor forward of the workgroup's SL slots: x0 -> h1 -> h2 -> a. Contains 3 barriers (the last
// one publishes W.a).
struct RoNoDyn {
  __device__ __forceinline__ void operator()() const {}
};
// dyn: work of this wave that needs nothing layer 2 produces, placed after layer 2's code in the
// same basic block so the scheduler can interleave it with the layer's MFMAs and LDS waits
template <int NG, int NS, int NA, int REGK, int LDSK, bool PF, bool SPLIT, typename WT, typename Bar,
          typename Dyn = RoNoDyn>
__device__ __forceinline__ void ro_actor(const RoActorRegs<NS, REGK>& R, WT& W, const float* __restrict__ W2g,
                                         const Lane& L, int it, Bar&& bar, Dyn dyn = Dyn{}) {
  using C = RoCfg<NG>;
  // ---- layer 1 (K = NS): one activation VGPR per group covers every k
  {
    floatx4 acc[NG];
    float x[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      acc[g] = floatx4{0.f, 0.f, 0.f, 0.f};
      x[g] = W.x0[g * 64 + L.lane];
    }
    static_for<NS>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
#pragma unroll
      for (int g = 0; g < NG; ++g) acc[g] = mfma_bc<q>(x[g], R.w1[q], acc[g]);
    });
    // feature k = 64 wave + lane of sample 4g + i -> h1 block (g, kb = wave), q = lane & 15, v = lane >> 4
    const int q = L.lane & 15, v = L.lane >> 4;
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) W.h1[(g * 4 + L.wave) * C::H1B + q * 20 + 4 * i + v] = lrelu(fadd(acc[g][i], R.b1));
  }
  bar();
  RSTAMP(4);
  // ---- layer 2 (K = 256)
  ro_layer2<NG, NS, REGK, LDSK, PF, SPLIT>(R, W, W2g, L);
  dyn();
  bar();
  RSTAMP(5);
  // ---- layer 3 (256 -> NA): one summation order for every NG (so the schedule never changes a
  //      result): 64 partial chains, chain j = features j, j + 64, j + 128, j + 192 (FMA in that
  //      order), combined by a butterfly over j with offsets 32, 16, ..., 1. Thread (slot s,
  //      segment seg) holds chains seg + P r (r < NG); the offsets >= P are the in-thread steps.
  {
    constexpr int NR = 64 / C::P;  // == NG
    const int s = L.tid / C::P, seg = L.tid % C::P;
    float pa[NA][NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
#pragma unroll
      for (int a = 0; a < NA; ++a) pa[a][r] = 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int f = seg + C::P * r + 64 * m;
        const float h = W.h2[s * C::H2S + f];
#pragma unroll
        for (int a = 0; a < NA; ++a) pa[a][r] = fmaf(W.w3[a * 256 + f], h, pa[a][r]);
      }
    }
#pragma unroll
    for (int half = NR / 2; half >= 1; half >>= 1)
#pragma unroll
      for (int r = 0; r < half; ++r)
#pragma unroll
        for (int a = 0; a < NA; ++a) pa[a][r] = pa[a][r] + pa[a][r + half];
#pragma unroll
    for (int off = C::P / 2; off >= 1; off >>= 1)
#pragma unroll
      for (int a = 0; a < NA; ++a) pa[a][0] = add_from_above(pa[a][0], off);
    if (seg == 0)
#pragma unroll
      for (int a = 0; a < NA; ++a) W.a[s * NA + a] = fadd(pa[a][0], W.b3[a]);
  }
  bar();
}

// Chain dynamics workspace of the rollout, structure of arrays [joint][component][slot] (slot
// fastest: the slot lanes of a wave read consecutive doubles). The joint placements X(q_i) of every
// (slot, joint) are computed in parallel by all threads; the RNEA and CRBA recursions then read
// them (and the RNEA parks its per-joint forces) here instead of holding NJ of each in registers — a 6-joint chain in float64 would otherwise not fit beside the actor.
template <int NJ, int SL>
struct RoChain {
  static constexpr int J = NJ > 0 ? NJ : 1;
  double X[J * 12 * SL];   // SE3: R (9, row-major), p (3)
  double f[J * 6 * SL];    // RNEA forces: l (3), a (3)
};

template <int SL>
__device__ __forceinline__ void se3_st(double* b, const SE3& X) {
#pragma unroll
  for (int k = 0; k < 9; ++k) b[k * SL] = X.R.m[k];
  b[9 * SL] = X.p.x;
  b[10 * SL] = X.p.y;
  b[11 * SL] = X.p.z;
}
template <int SL>
__device__ __forceinline__ SE3 se3_ld(const double* b) {
  SE3 X;
#pragma unroll
  for (int k = 0; k < 9; ++k) X.R.m[k] = b[k * SL];
  X.p = v3(b[9 * SL], b[10 * SL], b[11 * SL]);
  return X;
}
template <int SL>
__device__ __forceinline__ void sv_st(double* b, const SV& v) {
  b[0] = v.l.x, b[SL] = v.l.y, b[2 * SL] = v.l.z;
  b[3 * SL] = v.a.x, b[4 * SL] = v.a.y, b[5 * SL] = v.a.z;
}
template <int SL>
__device__ __forceinline__ SV sv_ld(const double* b) {
  return SV{v3(b[0], b[SL], b[2 * SL]), v3(b[3 * SL], b[4 * SL], b[5 * SL])};
}
// X(q_i) of every active (slot, joint): item e -> slot e % SL, joint e / SL, spread over the waves.
template <int NJ, int SL>
__device__ __forceinline__ void ro_placements(const SysDevice& sd, RoChain<NJ, SL>& C, const double* sS,
                                              const int* sact, const Lane& L) {
  constexpr int ns = Dims<NJ>::NS;
  const int e = (L.tid & 63) * 4 + L.wave;  // consecutive items on different waves
  if (e < SL * NJ) {
    const int c = e % SL, i = e / SL;
    if (sact[c]) se3_st<SL>(C.X + i * 12 * SL + c, joint_placement(JointView{sd.joints + i * CACTO_JOINT_COLS}, sS[c * ns + i]));
  }
}

// Joint loops: unrolled for short chains; a 6-joint chain keeps one joint's values live at a time
// in the CRBA columns, while the RNEA's forward pass (wave 0, the longest per-step chain) is unrolled fully so a
// joint's force terms overlap the next joint's velocity / acceleration recursion (no spills; the
// backward pass unrolled would spill).
#define RO_JU (NJ <= 3 ? NJ : 1)
#ifndef RO_NLE_JU
#define RO_NLE_JU NJ
#endif

// chain_nle (env.h) with X from the workspace and the forces parked there: same operations in the
// same order, so h is bit-identical.
template <int NJ, int SL>
__device__ __forceinline__ void ro_chain_nle(const SysDevice& sd, RoChain<NJ, SL>& C, int c, const double* q,
                                             const double* v, double* hout) {
  const SV gacc{v3(-sd.p.gravity[0], -sd.p.gravity[1], -sd.p.gravity[2]), v3(0, 0, 0)};
  SV vp{v3(0, 0, 0), v3(0, 0, 0)}, ap = gacc, fc;
#pragma unroll RO_NLE_JU
  for (int i = 0; i < NJ; ++i) {
    JointView j{sd.joints + i * CACTO_JOINT_COLS};
    const SE3 X = se3_ld<SL>(C.X + i * 12 * SL + c);
    const SV S = joint_S(j);
    SV vi = act_motion_inv(X, vp);
    const SV Sq{v[i] * S.l, v[i] * S.a};
    vi.l = vi.l + Sq.l;
    vi.a = vi.a + Sq.a;
    SV ai = act_motion_inv(X, ap);
    const SV cm = cross_motion(vi, Sq);
    ai.l = ai.l + cm.l;
    ai.a = ai.a + cm.a;
    const Inertia I = j.inertia();
    const SV Iv = inertia_mul(I, vi);
    const SV Ia = inertia_mul(I, ai);
    const SV vf = cross_force(vi, Iv);
    fc.l = Ia.l + vf.l;
    fc.a = Ia.a + vf.a;
    if (i < NJ - 1) sv_st<SL>(C.f + i * 6 * SL + c, fc);
    vp = vi;
    ap = ai;
  }
#pragma unroll RO_JU
  for (int i = NJ - 1; i >= 0; --i) {
    JointView j{sd.joints + i * CACTO_JOINT_COLS};
    hout[i * SL] = sdot(joint_S(j), fc);
    if (i > 0) {
      const SV fp = act_force(se3_ld<SL>(C.X + i * 12 * SL + c), fc);
      const SV fo = sv_ld<SL>(C.f + (i - 1) * 6 * SL + c);
      fc.l = fo.l + fp.l;
      fc.a = fo.a + fp.a;
    }
  }
}

// A double of the lane below (SHR: row_shr:1) or above (SHL: row_shl:1) in the 16-lane DPP row, two
// 32-bit moves; a row's first / last lane gets zeros (its callers select over those lanes).
constexpr int DPP_SHR1 = 0x111, DPP_SHL1 = 0x101;
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// the same with the lanes whose source lies outside the row keeping `old` (bound_ctrl off)
template <int CTRL>
__device__ __forceinline__ double dpp_d_old(double old, double v) {
  const long long b = __double_as_longlong(v), o = __double_as_longlong(old);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ SV dpp_sv_old(const SV& old, const SV& v) {
  return SV{v3(dpp_d_old<CTRL>(old.l.x, v.l.x), dpp_d_old<CTRL>(old.l.y, v.l.y), dpp_d_old<CTRL>(old.l.z, v.l.z)),
            v3(dpp_d_old<CTRL>(old.a.x, v.a.x), dpp_d_old<CTRL>(old.a.y, v.a.y), dpp_d_old<CTRL>(old.a.z, v.a.z))};
}
template <int CTRL>
__device__ __forceinline__ SV dpp_sv(const SV& v) {
  return SV{v3(dpp_d<CTRL>(v.l.x), dpp_d<CTRL>(v.l.y), dpp_d<CTRL>(v.l.z)),
            v3(dpp_d<CTRL>(v.a.x), dpp_d<CTRL>(v.a.y), dpp_d<CTRL>(v.a.z))};
}
__device__ __forceinline__ SV sv_sel(bool p, const SV& a, const SV& b) {
  return SV{v3(p ? a.l.x : b.l.x, p ? a.l.y : b.l.y, p ? a.l.z : b.l.z),
            v3(p ? a.a.x : b.a.x, p ? a.a.y : b.a.y, p ? a.a.z : b.a.z)};
}

// ro_chain_nle spread over wave 0 by (slot, joint): lane 8 c + j runs joint j of slot c with its
// placement X_j in registers (one LDS read per step instead of one per joint and pass). The
// velocity / acceleration recursion advances one joint per round — each round every lane applies
// its X_j to its parent's (v, a), handed up from the lane below by a DPP row shift, so after round j
// lane j holds v_j, a_j — then the per-joint force terms run on all joints at once, and the force
// recursion hands act_force(X_j, f_j) down one lane per round. Each value is formed by the same
// operations in the same order as chain_nle, so h is bit-identical; only the serial chain of LDS
// round trips is gone. Slots whose lanes hold no episode compute on stale placements; their h is
// not read.
template <int NJ, int SL>
__device__ __forceinline__ void ro_chain_nle_lanes(const SysDevice& sd, const double* jt, RoChain<NJ, SL>& C,
                                                   const double* sS, double* hS, double* dump, int lane,
                                                   bool stamp = false) {
#ifdef CACTO_STAMPS
#define NSTAMP(k)                                                                   \
  do {                                                                              \
    __builtin_amdgcn_s_waitcnt(0);                                                  \
    if (stamp) g_rstamps[k] = __builtin_amdgcn_s_memtime();                         \
  } while (0)
#else
#define NSTAMP(k) \
  do {            \
  } while (0)
#endif
  // lanes per slot: a whole 16-lane DPP row per slot when the slots fit (SL = 4), so the base
  // joint's lane takes (0, a_g) as the shift's out-of-row value instead of a select per round
  constexpr int LPS = SL * 16 <= 64 ? 16 : 8;
  static_assert(NJ <= LPS && SL * LPS <= 64, "one wave");
  constexpr int ns = Dims<NJ>::NS;
  const int cr = lane / LPS, jr = lane % LPS;
  const int c = min(cr, SL - 1), j = min(jr, NJ - 1);
  const bool base = jr == 0, top = jr >= NJ - 1;
  const JointView jv{jt + j * CACTO_JOINT_COLS};  // the LDS copy of the joint table
  const SE3 X = se3_ld<SL>(C.X + j * 12 * SL + c);
  const double qd = sS[c * ns + NJ + j];
  const SV S = joint_S(jv);
  const Inertia I = jv.inertia();
  const SV Sq{qd * S.l, qd * S.a};
  const SV zero{v3(0, 0, 0), v3(0, 0, 0)};
  const SV gacc{v3(-sd.p.gravity[0], -sd.p.gravity[1], -sd.p.gravity[2]), v3(0, 0, 0)};
  SV vp = zero, ap = gacc, vi, ai;
  NSTAMP(17);
#pragma unroll
  for (int r = 0; r < NJ; ++r) {
    vi = act_motion_inv(X, vp);
    vi.l = vi.l + Sq.l;
    vi.a = vi.a + Sq.a;
    ai = act_motion_inv(X, ap);
    const SV cm = cross_motion(vi, Sq);
    ai.l = ai.l + cm.l;
    ai.a = ai.a + cm.a;
    if (r < NJ - 1) {
      if constexpr (LPS == 16) {
        vp = dpp_sv_old<DPP_SHR1>(zero, vi);
        ap = dpp_sv_old<DPP_SHR1>(gacc, ai);
      } else {
        vp = sv_sel(base, zero, dpp_sv<DPP_SHR1>(vi));
        ap = sv_sel(base, gacc, dpp_sv<DPP_SHR1>(ai));
      }
    }
  }
  NSTAMP(18);
  const SV Iv = inertia_mul(I, vi);
  const SV Ia = inertia_mul(I, ai);
  const SV vf = cross_force(vi, Iv);
  SV f;
  f.l = Ia.l + vf.l;
  f.a = Ia.a + vf.a;
  SV fc = f;
  NSTAMP(19);
#pragma unroll
  for (int r = 0; r < NJ - 1; ++r) {
    const SV fp = dpp_sv<DPP_SHL1>(act_force(X, fc));
    SV g;
    g.l = f.l + fp.l;
    g.a = f.a + fp.a;
    fc = sv_sel(top, fc, g);
  }
  const double h = sdot(S, fc);
  // every lane stores (no exec-mask branch in the block): lanes without a value write their dump slot
  const bool own = cr < SL && jr < NJ;
  *(own ? hS + j * SL + c : dump + lane) = h;
#undef NSTAMP
}

template <int CTRL>
__device__ __forceinline__ Inertia dpp_inertia(const Inertia& I) {
  Inertia o;
  o.m = dpp_d<CTRL>(I.m);
  o.h = v3(dpp_d<CTRL>(I.h.x), dpp_d<CTRL>(I.h.y), dpp_d<CTRL>(I.h.z));
  o.Io.xx = dpp_d<CTRL>(I.Io.xx);
  o.Io.xy = dpp_d<CTRL>(I.Io.xy);
  o.Io.xz = dpp_d<CTRL>(I.Io.xz);
  o.Io.yy = dpp_d<CTRL>(I.Io.yy);
  o.Io.yz = dpp_d<CTRL>(I.Io.yz);
  o.Io.zz = dpp_d<CTRL>(I.Io.zz);
  return o;
}

// dpp_inertia with -0.0 in every field of the lanes whose source lies outside the row
template <int CTRL>
__device__ __forceinline__ Inertia dpp_inertia_nz(const Inertia& I) {
  constexpr double nz = -0.0;
  Inertia o;
  o.m = dpp_d_old<CTRL>(nz, I.m);
  o.h = v3(dpp_d_old<CTRL>(nz, I.h.x), dpp_d_old<CTRL>(nz, I.h.y), dpp_d_old<CTRL>(nz, I.h.z));
  o.Io.xx = dpp_d_old<CTRL>(nz, I.Io.xx);
  o.Io.xy = dpp_d_old<CTRL>(nz, I.Io.xy);
  o.Io.xz = dpp_d_old<CTRL>(nz, I.Io.xz);
  o.Io.yy = dpp_d_old<CTRL>(nz, I.Io.yy);
  o.Io.yz = dpp_d_old<CTRL>(nz, I.Io.yz);
  o.Io.zz = dpp_d_old<CTRL>(nz, I.Io.zz);
  return o;
}

// chain_mass spread over one wave by (slot, joint), lane 8 c + j as in ro_chain_nle_lanes: the
// composite inertias Ic_{j-1} = I_{j-1} + X_j^* Ic_j advance one joint per round (each lane
// transports its Ic, the lane below adds its own I), then every column of M at once in a systolic
// sweep — in round t lane k holds column k + t's force in joint k's frame, transports it to its
// parent (act_force with its X_k) and hands it down a lane, where sdot with that joint's S gives
// M[k + t][k - 1]. The same operations in the same order as chain_mass, so M is bit-identical.
template <int NJ, int SL>
__device__ __forceinline__ void ro_chain_mass_lanes(const double* jt, RoChain<NJ, SL>& C, double* MS, double* dump,
                                                    int lane) {
  // a 16-lane row per slot when the slots fit (SL = 4), joints at the row's top lanes: the tip
  // joint's lane then takes -0.0 (x + -0.0 == x for every x) as the shift's out-of-row value
  // instead of a select per round
  constexpr int LPS = SL * 16 <= 64 ? 16 : 8, J0 = LPS == 16 ? 16 - NJ : 0;
  static_assert(NJ <= LPS && SL * LPS <= 64, "one wave");
  const int cr = lane / LPS, jr = lane % LPS - J0;
  const int c = min(cr, SL - 1), j = min(max(jr, 0), NJ - 1);
  const bool top = jr >= NJ - 1, live = cr < SL && jr >= 0 && jr < NJ;
  const JointView jv{jt + j * CACTO_JOINT_COLS};  // the LDS copy of the joint table
  const SE3 X = se3_ld<SL>(C.X + j * 12 * SL + c);
  const SV S = joint_S(jv);
  const Inertia I = jv.inertia();
  Inertia Ic = I;
#pragma unroll
  for (int r = 0; r < NJ - 1; ++r) {
    if constexpr (LPS == 16) {
      const Inertia t = dpp_inertia_nz<DPP_SHL1>(act_inertia(X, Ic));
      Inertia a = I;
      add_inertia(a, t);
      Ic = a;
    } else {
      const Inertia t = dpp_inertia<DPP_SHL1>(act_inertia(X, Ic));
      Inertia a = I;
      add_inertia(a, t);
      if (!top) Ic = a;
    }
  }
  SV F = inertia_mul(Ic, S);
  // every lane stores (no exec-mask branch in the block): lanes without a value write their dump slot
  *(live ? MS + (j * NJ + j) * SL + c : dump + lane) = sdot(S, F);
#pragma unroll
  for (int t = 1; t < NJ; ++t) {
    F = dpp_sv<DPP_SHL1>(act_force(X, F));  // column j + t, in this joint's frame
    const double mij = sdot(S, F);
    const bool w = live && j + t < NJ;
    *(w ? MS + ((j + t) * NJ + j) * SL + c : dump + lane) = mij;
    *(w ? MS + (j * NJ + (j + t)) * SL + c : dump + 64 + lane) = mij;
  }
}

// chain_mass (env.h) from the workspace placements, split by columns over waves 1-3: column i of
// M needs the composite inertia Ic_i = I_i + X_{i+1}^* Ic_{i+1} (tip to base) and then i force
// transports toward the base. Wave 3 takes columns {0, 1} (the whole composite chain), wave 2 the
// lower half of the rest, wave 1 the upper half; each wave runs the composite chain from the tip
// down to its lowest column itself (a few act_inertia recomputed instead of a cross-wave wait).
// Every element is computed by the same operations in the same order as chain_mass, so M is
// bit-identical; row-major M written to Mout[k * SL], each element by exactly one wave.
template <int NJ>
struct RoMassCols {
  static constexpr int rest = NJ > 2 ? NJ - 2 : 0, up = (rest + 1) / 2;
  __device__ static int lo(int w) { return w == 3 ? 0 : (w == 2 ? 2 : 2 + up); }
  __device__ static int hi(int w) { return w == 3 ? (NJ > 1 ? 1 : 0) : (w == 2 ? 1 + up : NJ - 1); }
};

template <int NJ, int SL>
__device__ __forceinline__ void ro_mass_column(const SysDevice& sd, RoChain<NJ, SL>& C, int c, int i,
                                               const Inertia& Ic, double* Mout) {
  JointView j{sd.joints + i * CACTO_JOINT_COLS};
  SV F = inertia_mul(Ic, joint_S(j));
  Mout[(i * NJ + i) * SL] = sdot(joint_S(j), F);
  for (int k = i; k > 0; --k) {
    F = act_force(se3_ld<SL>(C.X + k * 12 * SL + c), F);
    JointView jp{sd.joints + (k - 1) * CACTO_JOINT_COLS};
    const double mij = sdot(joint_S(jp), F);
    Mout[(i * NJ + (k - 1)) * SL] = mij;
    Mout[((k - 1) * NJ + i) * SL] = mij;
  }
}

template <int NJ, int SL>
__device__ __forceinline__ void ro_chain_mass_cols(const SysDevice& sd, RoChain<NJ, SL>& C, int c, double* Mout,
                                                   int lo, int hi) {
  if (lo > hi) return;
  Inertia acc = JointView{sd.joints + (NJ - 1) * CACTO_JOINT_COLS}.inertia();  // Ic_{NJ-1}
  for (int i = NJ - 1;; --i) {
    if (i <= hi) ro_mass_column<NJ, SL>(sd, C, c, i, acc, Mout);
    if (i == lo) break;
    Inertia a = JointView{sd.joints + (i - 1) * CACTO_JOINT_COLS}.inertia();
    add_inertia(a, act_inertia(se3_ld<SL>(C.X + i * 12 * SL + c), acc));
    acc = a;
  }
}

// Per-episode constant dynamics (prismatic chains, ConstDyn) only for short chains: the 6-joint
// chain_terms in one thread would not fit beside the actor, and those chains take the per-step
// RNEA/CRBA path.
template <int NJ>
struct RoConstDyn {
  static constexpr bool ok = NJ > 0 && NJ <= 3;
};

template <int NJ, int NG>
struct RoShared {
  static constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA, SL = RoCfg<NG>::SL;
  RoActorLds<NG, na, RoSplit<NJ, NG>::LDSK> W;
  double sS[SL * ns];                                                 // s_t of every slot
  double MS[NJ > 0 ? SL * NJ * NJ : 1], hS[NJ > 0 ? SL * NJ : 1];    // chain M(q) (or its Cholesky factor), nle: [k][slot]
  RoChain<NJ, SL> ch;
  double jt[NJ > 0 ? NJ * CACTO_JOINT_COLS : 1];  // the joint table (the per-lane recursions' constants)
  double dump[NJ > 0 && NG <= 2 ? 128 : 1];        // the lane recursions' stores of lanes without a value
  int sb[SL], sn[SL], st[SL], sact[SL];
  int anyact;
};

// normalize_feature (mlp.h) with the norms held in registers for the whole launch: the per-step
// input of the next actor pass must not wait on scalar loads of the system parameters (each such
// load's s_waitcnt also drains the LDS queue). Same f32 arithmetic, branch-free.
template <int NS>
struct RoNorm {
  float n[NS];
  bool on;
  __device__ __forceinline__ explicit RoNorm(const cacto_sys_params& p) {
    on = p.normalize != 0;
#pragma unroll
    for (int i = 0; i < NS; ++i) n[i] = (float)p.state_norm[i];
  }
  __device__ __forceinline__ float operator()(int f, float s) const {
    const float q = fdiv(s, n[f]);
    const float v = f == NS - 1 ? fsub(fmul(q, 2.0f), 1.0f) : q;
    return on ? v : s;
  }
};

// The next actor input of one (slot, feature) item per wave-0 lane and round: item e = lane + 64 r
// -> slot e % SL, feature e / SL. The lane's norm is fixed for the launch, so the per-step work is
// one division per item spread over the lanes instead of ns divisions on each slot's lane (the
// same fdiv, so the same bits as RoNorm).
template <int NS, int SL>
struct RoX0Lane {
  static constexpr int R = (SL * NS + 63) / 64;  // rounds
  float n[R];
  bool tcol[R], valid[R];
  __device__ __forceinline__ RoX0Lane(const RoNorm<NS>& nrm, int lane) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = lane + 64 * r, f = e / SL;
      valid[r] = e < SL * NS;
      tcol[r] = f == NS - 1;
      float v = 1.f;
#pragma unroll
      for (int q = 0; q < NS; ++q) v = f == q ? nrm.n[q] : v;  // select chain, no dynamic indexing
      n[r] = v;
    }
  }
  template <typename Sh>
  __device__ __forceinline__ void write(Sh& S, const RoNorm<NS>& nrm, int lane) const {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = lane + 64 * r, c = e % SL, f = e / SL;
      if (valid[r]) {
        const float q = fdiv((float)S.sS[c * NS + f], n[r]);
        const float v = tcol[r] ? fsub(fmul(q, 2.0f), 1.0f) : q;
        S.W.x0[(c >> 2) * 64 + 4 * f + (c & 3)] = nrm.on ? v : (float)S.sS[c * NS + f];
      }
    }
  }
};

// Slot refill (wave 0; every lane calls it, lanes with `need` take the next queue entries in lane
// order). A new episode's s_0 goes to the slot's state and the actor input; episodes of length 0
// are completed on the spot (status 0: RL.py never rolls out NSTEPS_SH == 0).
template <int NJ, int NG, typename ShT, bool INIT_CD = true>
__device__ __forceinline__ void ro_refill(bool need, int c, int& head, ShT& Sh, const SysDevice& sd,
                                          const double* __restrict__ S0,
                                          const int32_t* __restrict__ nsteps, const int32_t* __restrict__ order, int T,
                                          int B, int G, double* __restrict__ Straj, int32_t* __restrict__ status,
                                          const RoNorm<Dims<NJ>::NS>& nrm, const Lane& L, int vb) {
  constexpr int ns = Dims<NJ>::NS, SL = RoCfg<NG>::SL;
  const cacto_sys_params& p = sd.p;
  while (true) {
    const uint64_t m = __ballot(need);
    if (m == 0) break;
    const int rank = __popcll(m & ((1ull << L.lane) - 1ull));
    const int k = head + rank;
    head += __popcll(m);
    if (need) {
      const int r = k * G + ((k & 1) ? G - 1 - vb : vb);
      if (r >= B) {
        need = false;
        Sh.sact[c] = 0;
      } else {
        const int b = order ? order[r] : r;
        const int n = min(nsteps[b], T);
        double s[ns];
#pragma unroll
        for (int i = 0; i < ns; ++i) {
          s[i] = S0[(size_t)b * ns + i];
          if (Straj) Straj[(size_t)b * (T + 1) * ns + i] = s[i];
        }
        if (n == 0) {
          if (status) status[b] = 0;
        } else {
          need = false;
          Sh.sb[c] = b;
          Sh.sn[c] = n;
          Sh.st[c] = 0;
          Sh.sact[c] = 1;
#pragma unroll
          for (int i = 0; i < ns; ++i) Sh.sS[c * ns + i] = s[i];
#pragma unroll
          for (int q = 0; q < ns; ++q) Sh.W.x0[(c >> 2) * 64 + 4 * q + (c & 3)] = nrm(q, (float)s[q]);
          if constexpr (RoConstDyn<NJ>::ok && INIT_CD) {
            if (p.const_dyn) {
              // prismatic chain: M factored once per episode, kept in the slot's MS / hS
              ConstDyn<NJ> cd;
                          const_dyn_init<NJ>(sd, s, cd);
#pragma unroll
              for (int k = 0; k < NJ * NJ; ++k) Sh.MS[k * SL + c] = cd.L[k];
#pragma unroll
              for (int i = 0; i < NJ; ++i) Sh.hS[i * SL + c] = cd.h[i];
            }
          }
        }
      }
    }
  }
}

// A slot's state as wave 0's lane c keeps it in registers: active flag, episode, step, s_t and, for
// prismatic chains, the episode's Cholesky factor and bias forces (loaded from the slot's LDS copy
// after the lane (re)fills it).
template <int NJ, int NG>
struct RoSlotRegs {
  static constexpr int ns = Dims<NJ>::NS, SL = RoCfg<NG>::SL;
  bool act = false;
  int b = 0, t = 0, n = 0;
  double s[ns];
  ConstDyn<NJ> cd;
  template <typename ShT>
  __device__ __forceinline__ void load(const ShT& Sh, int c, bool cdyn) {
    if (c >= SL) return;
    act = Sh.sact[c] != 0;
    b = Sh.sb[c];
    t = Sh.st[c];
    n = Sh.sn[c];
#pragma unroll
    for (int i = 0; i < ns; ++i) s[i] = Sh.sS[c * ns + i];
    if constexpr (NJ > 0) {
      if (cdyn) {
#pragma unroll
        for (int k = 0; k < NJ * NJ; ++k) cd.L[k] = Sh.MS[k * SL + c];
#pragma unroll
        for (int i = 0; i < NJ; ++i) cd.h[i] = Sh.hS[i * SL + c];
      }
    }
  }
};

// Wave 0, lane c (< SL): after s' = f(s, a) of slot c (already in the slot's LDS state): the
// trajectory stores of (a_t, s_{t+1}) and the end of the episode (status; the caller refills).
template <int NJ, int NG>
__device__ __forceinline__ bool ro_advance(int c, int b, int tc, const double* sn, const float* a,
                                           const SysDevice& sd, int T,
                                           double* __restrict__ Straj, float* __restrict__ Atraj,
                                           int32_t* __restrict__ status, const RoNorm<Dims<NJ>::NS>& nrm, int n) {
  constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  const cacto_sys_params& p = sd.p;
  bool bad = false;
#pragma unroll
  for (int i = 0; i < ns; ++i) bad |= isnan(sn[i]);
  if (Atraj)
#pragma unroll
    for (int i = 0; i < na; ++i) Atraj[((size_t)b * T + tc) * na + i] = a[i];
  if (Straj)
#pragma unroll
    for (int i = 0; i < ns; ++i) Straj[((size_t)b * (T + 1) + tc + 1) * ns + i] = sn[i];
  if (bad && Straj) {
    // RL.py:229-231 drops the episode; the rest of its trajectory is NaN (the reward / EE pass
    // skips NaN states)
    for (int t = tc + 2; t <= n; ++t)
#pragma unroll
      for (int i = 0; i < ns; ++i) Straj[((size_t)b * (T + 1) + t) * ns + i] = __builtin_nan("");
  }
  const bool fin = bad || tc + 1 >= n;
  if (fin && status) status[b] = bad ? 1 : 0;
  return fin;
}

// Env.simulate of the rollout (float64 state and action, f32in = false) with the system scalars it
// reads held in registers for the whole launch: env_simulate / env_simulate_const read them from
// the SysDevice parameter block at every call, and in the one-slot-per-wave kernel that scalar
// load's latency sat on every step's dynamics. The same operations in the same order as env_simulate(_const).
struct RoSimScalars {
  double dt, L_delta, tau_delta;
};
template <int NJ>
__device__ __forceinline__ void ro_simulate(const RoSimScalars& k, const ConstDyn<NJ>& cd, const double* s,
                                            const double* a, double* out) {
  const double dt = k.dt;
  if constexpr (NJ == 0) {
    out[0] = s[0] + dt * a[0];
    out[1] = s[1] + dt * a[1];
    out[2] = s[2] + dt;
  } else if constexpr (NJ == -1) {
    const double dt2 = dt * dt;
    const double c = cos(s[2]), sn = sin(s[2]);
    out[0] = (s[0] + dt * s[3] * c) + dt2 * s[4] * c / 2.0;
    out[1] = (s[1] + dt * s[3] * sn) + dt2 * s[4] * sn / 2.0;
    out[2] = s[2] + dt * a[0];
    out[3] = s[3] + dt * s[4];
    out[4] = s[4] + dt * a[1];
    out[5] = s[5] + dt;
  } else if constexpr (NJ == -2) {
    const double L = k.L_delta, tau = k.tau_delta;
    out[0] = s[0] + dt * s[3] * cos(s[2]);
    out[1] = s[1] + dt * s[3] * sin(s[2]);
    out[2] = s[2] + dt * s[3] * tan(s[4]) / L;
    out[3] = s[3] + dt * a[0];
    out[4] = s[4] + dt * a[1] / tau;
    out[5] = s[5] + dt;
  } else {
    double dv[NJ];
#pragma unroll
    for (int i = 0; i < NJ; ++i) dv[i] = a[i] - cd.h[i];
    chol_solve<NJ>(cd.L, dv);
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const double v = s[NJ + i];
      out[i] = s[i] + v * dt;
      out[NJ + i] = v + dv[i] * dt;
    }
    out[2 * NJ] = s[2 * NJ] + dt;
  }
}

// One workgroup = SL episode slots (lane c < SL of wave 0 <-> slot c). Per step:
//   actor (4 waves, MFMA, weights stationary)                                -> a (LDS)
//   wave 0: s' = f(s, a) (chains with configuration-dependent M: RNEA on wave 0 and the CRBA
//   columns on waves 1-3 first, then the Cholesky step), the next actor input, the stores of (a_t, s_{t+1}),
//   finished episodes retired and their slots refilled.
// Rewards and end-effector positions depend only on (s_t, a_t): k_rollout_rewards computes them
// for every recorded step afterwards, fully parallel, so the sequential per-step chain is only
// actor -> dynamics.
template <int NJ, int NG>
__global__ void __launch_bounds__(CACTO_THREADS, 1)
    k_rollout(const SysDevice* __restrict__ sdp, NetView N, const double* __restrict__ S0,
              const int32_t* __restrict__ nsteps, int T, int use_actor, double* __restrict__ Straj,
              float* __restrict__ Atraj, int32_t* __restrict__ status, const int32_t* __restrict__ order, int B) {
  constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  using C = RoCfg<NG>;
  constexpr int SL = C::SL;
  __shared__ RoShared<NJ, NG> Sh;
  const SysDevice& sd = *sdp;
  const cacto_sys_params& p = sd.p;
  const Lane L;
  const int G = gridDim.x;
  // chains with configuration-dependent M: RNEA (wave 0) and CRBA (waves 1-3) run concurrently,
  // except the planar 3R chain, which steps with the closed form (planar3_step, as k_rollout_ks)
  const bool planar = NJ == 3 && sd.pl[0] != 0.0;
  const bool split_dyn = NJ > 0 && !(RoConstDyn<NJ>::ok && p.const_dyn) && !planar;
  constexpr int REGK = RoSplit<NJ, NG>::REGK, LDSK = RoSplit<NJ, NG>::LDSK;
  RoActorRegs<ns, REGK> R;
  if (use_actor) ro_load_actor<NG, ns, na, REGK, LDSK>(N, L, R, Sh.W);
  const float* W2g = N.flat + N.t.woff[1];
  for (int e = L.tid; e < NG * 64; e += CACTO_THREADS) Sh.W.x0[e] = 0.f;
  // slot states too: a slot that is never filled still feeds its (unused) actor input row, which
  // then reads zeros rather than stale LDS
  for (int e = L.tid; e < SL * ns; e += CACTO_THREADS) Sh.sS[e] = 0.0;
  if constexpr (NJ > 0)
    for (int e = L.tid; e < NJ * CACTO_JOINT_COLS; e += CACTO_THREADS) Sh.jt[e] = sd.joints[e];
  if (L.tid < SL) Sh.sact[L.tid] = 0;
  __syncthreads();
  int head = 0;  // queue position (wave 0, uniform)
  const RoNorm<ns> nrm(p);
  const RoSimScalars ks{p.dt, p.L_delta, p.tau_delta};
  if (L.wave == 0) {
    ro_refill<NJ, NG>(L.lane < SL, L.lane, head, Sh, sd, S0, nsteps, order, T, B, G, Straj, status, nrm, L,
                      (int)blockIdx.x);
    const uint64_t m = __ballot(L.lane < SL && Sh.sact[L.lane]);
    if (L.lane == 0) Sh.anyact = m != 0;
  }
  __syncthreads();
  const int c = L.lane % SL;  // slot of this lane
  const RoX0Lane<ns, SL> x0l(nrm, L.lane);
  // wave 0, lane c < SL: its slot's state in registers for the whole launch (the lane is the only
  // writer of the slot's LDS copy: ro_advance and ro_refill run on it), so the dynamics phase waits
  // only for the action, not for LDS reads of s_t and the episode's factored mass matrix
  const bool cdyn = RoConstDyn<NJ>::ok && !split_dyn && NJ > 0;
  RoSlotRegs<NJ, NG> sr;
  if (L.wave == 0) sr.load(Sh, c, cdyn);
  for (int it = 0; Sh.anyact; ++it) {
    RSTAMP(0);
    // joint placements of s_t (published by the actor's first barrier)
    if constexpr (NJ > 0) {
      if (split_dyn) {
        ro_placements<NJ, SL>(sd, Sh.ch, Sh.sS, Sh.sact, L);
        if (!use_actor) __syncthreads();
      }
    }
    // revolute chains on (slot, joint) lanes: M(q) and h(q, v) depend on s_t only, so wave 0's RNEA
    // and wave 1's CRBA run inside the actor, interleaved with their layer-2 MFMAs
    constexpr bool LANE_DYN = NJ > 0 && SL * 8 <= 64;
    constexpr bool APF = NJ <= 2 || (NJ > 3 && NG == 1 && RO_CHAIN6_PF);
    // (one slot group: at two the 8-lane layout's registers beside layer 2 would spill)
    const bool dyn_in_actor = LANE_DYN && SL * 16 <= 64 && split_dyn && use_actor && RO_DYN_IN_ACTOR;
    auto abar = [] { __syncthreads(); };
    if (use_actor) {
      if constexpr (LANE_DYN && SL * 16 <= 64) {
        if (dyn_in_actor) {
          if (L.wave == 0)
            ro_actor<NG, ns, na, REGK, LDSK, APF, (NJ <= 3)>(R, Sh.W, W2g, L, it, abar, [&] {
              ro_chain_nle_lanes<NJ, SL>(sd, Sh.jt, Sh.ch, Sh.sS, Sh.hS, Sh.dump, L.lane);
            });
          else if (L.wave == 1)
            ro_actor<NG, ns, na, REGK, LDSK, APF, (NJ <= 3)>(R, Sh.W, W2g, L, it, abar, [&] {
              ro_chain_mass_lanes<NJ, SL>(Sh.jt, Sh.ch, Sh.MS, Sh.dump, L.lane);
            });
          else
            ro_actor<NG, ns, na, REGK, LDSK, APF, (NJ <= 3)>(R, Sh.W, W2g, L, it, abar);
        } else {
          ro_actor<NG, ns, na, REGK, LDSK, APF, (NJ <= 3)>(R, Sh.W, W2g, L, it, abar);
        }
      } else {
        ro_actor<NG, ns, na, REGK, LDSK, APF, (NJ <= 3)>(R, Sh.W, W2g, L, it, abar);
      }
    }
    RSTAMP(1);
    const bool active = L.lane < SL && (L.wave == 0 ? sr.act : Sh.sact[c] != 0);
    if (split_dyn && !dyn_in_actor) {
      if constexpr (NJ > 0) {
        if (L.wave == 0) {
          if constexpr (SL * 8 <= 64)
            ro_chain_nle_lanes<NJ, SL>(sd, Sh.jt, Sh.ch, Sh.sS, Sh.hS, Sh.dump, L.lane
#ifdef CACTO_STAMPS
                                       , blockIdx.x == 0 && L.lane == 0 && it == 20
#endif
            );
          else if (active)
            ro_chain_nle<NJ, SL>(sd, Sh.ch, c, Sh.sS + c * ns, Sh.sS + c * ns + NJ, Sh.hS + c);
          RSTAMP(9);
        } else if constexpr (SL * 8 <= 64) {
          if (L.wave == 1) {
            ro_chain_mass_lanes<NJ, SL>(Sh.jt, Sh.ch, Sh.MS, Sh.dump, L.lane);
#ifdef CACTO_STAMPS
            if (blockIdx.x == 0 && L.lane == 0 && it == 20) g_rstamps[10] = __builtin_amdgcn_s_memtime();
#endif
          }
        } else if (active) {
          ro_chain_mass_cols<NJ, SL>(sd, Sh.ch, c, Sh.MS + c, RoMassCols<NJ>::lo(L.wave), RoMassCols<NJ>::hi(L.wave));
#ifdef CACTO_STAMPS
          if (blockIdx.x == 0 && L.lane == 0 && it == 20) g_rstamps[9 + L.wave] = __builtin_amdgcn_s_memtime();
#endif
        }
      }
      __syncthreads();
    }
    RSTAMP(2);
    if (L.wave == 0) {
      bool fin = false;
      float a[na];
      if (active) {
        double ad[na], sn[ns];
        const double* s = sr.s;
#pragma unroll
        for (int i = 0; i < na; ++i) {
          a[i] = use_actor ? Sh.W.a[c * na + i] : 0.f;
          ad[i] = (double)a[i];
        }
        if constexpr (NJ > 0) {
          if (split_dyn) {
            double M[NJ * NJ], h[NJ];
#pragma unroll
            for (int k = 0; k < NJ * NJ; ++k) M[k] = Sh.MS[k * SL + c];
#pragma unroll
            for (int i = 0; i < NJ; ++i) h[i] = Sh.hS[i * SL + c];
            chain_step<NJ>(sd, s, ad, M, h, sn);
          } else if (NJ == 3 && planar) {
            planar3_step(Planar3(sd.pl), ks.dt, s, ad, sn);
          } else {
            ro_simulate<NJ>(ks, sr.cd, s, ad, sn);
          }
        } else {
          ro_simulate<NJ>(ks, sr.cd, s, ad, sn);
        }
        RSTAMP(6);
#pragma unroll
        for (int i = 0; i < ns; ++i) {
          Sh.sS[c * ns + i] = sn[i];
          sr.s[i] = sn[i];
        }
      }
      // The next actor input from s_{t+1}: the slots' lanes wrote sS above, and LDS operations of
      // one wave complete in order, so after the wave-scope fence every lane reads them. EARLY
      // (revolute chains): written before the trajectory stores and the bookkeeping, which then
      // overlap its latency; a slot that ends and is refilled gets its new s_0 row from ro_refill
      // afterwards (same wave, later in program order). Measured per system (r03): UR5 +2.7 %,
      // manipulator neutral, car_park -4.5 %, DI neutral — the others write it last.
      constexpr bool EARLY = NJ >= 3;
      if constexpr (EARLY) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        x0l.write(Sh, nrm, L.lane);
      }
      RSTAMP(16);
      if (active) {
        fin = ro_advance<NJ, NG>(c, sr.b, sr.t, sr.s, a, sd, T, Straj, Atraj, status, nrm, sr.n);
        sr.t += 1;
        RSTAMP(7);
      }
      ro_refill<NJ, NG>(fin, c, head, Sh, sd, S0, nsteps, order, T, B, G, Straj, status, nrm, L, (int)blockIdx.x);
      if (fin) sr.load(Sh, c, cdyn);  // the slot's next episode (or none), written by this lane
      if constexpr (!EARLY) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        x0l.write(Sh, nrm, L.lane);
      }
      const uint64_t m = __ballot(L.lane < SL && Sh.sact[c]);
      if (L.lane == 0) Sh.anyact = m != 0;
      RSTAMP(8);
    }
    __syncthreads();
    RSTAMP(3);
  }
}

// ---------------------------------------------------------------- two teams per workgroup
// The same per-step pipeline for the systems whose dynamics need no workgroup (no chain with
// configuration-dependent M: SI, car, car_park, the prismatic DI) run as TWO independent teams of
// 4 waves (4 episode slots each) in one 8-wave workgroup: two waves per SIMD, so while one team is
// in its non-MFMA phases (layer 1's epilogue, layer 3, the dynamics on its wave 0, the stores and
// refill) the other team's layer-2 MFMAs keep the matrix cores busy. The teams share the LDS-resident
// layer-2 weight rows (RoSplitTT: 128 rows in registers — a wave has 256 of them at two waves per
// SIMD — and 128 in LDS) and synchronise with team barriers (an LDS arrival counter), never with
// the workgroup barrier. Each team is a "virtual workgroup" of the snake dealing (vb = 2 b + team,
// G = 2 x workgroups); per-slot arithmetic is the single-team kernel's, so results are identical.
struct RoSplitTT {
  static constexpr int REGK = 128, LDSK = 128;
};

template <int NA>
struct RoTeamActorLds {
  static constexpr int SL = 4;
  float h1[4 * RoCfg<1>::H1B];
  float h2[SL * RoCfg<1>::H2S];
  float x0[64];
  float a[SL * NA];
};

template <int NJ>
struct RoTeamShared {
  static constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA, SL = 4;
  RoTeamActorLds<na> W;
  double sS[SL * ns];
  double MS[NJ > 0 ? SL * NJ * NJ : 1], hS[NJ > 0 ? SL * NJ : 1];
  int sb[SL], sn[SL], st[SL], sact[SL];
  int anyact;
  int bar;  // team barrier: arrivals
};

template <int NJ>
struct RoTTShared {
  static constexpr int na = Dims<NJ>::NA;
  float4 w2[RoSplitTT::LDSK / 4 * 4 * 64];
  float w3[na * 256];
  float b3[8];
  RoTeamShared<NJ> team[2];
};

// ro_actor's view of a team: the shared weights + the team's activations
template <int NA>
struct RoTeamView {
  const float4* w2;
  const float* w3;
  const float* b3;
  float* h1;
  float* h2;
  float* x0;
  float* a;
};

// Barrier of the 4 waves of a team: each wave's lane 0 adds one arrival (release: the wave's LDS
// writes are complete), the wave then waits for 4 arrivals per barrier so far (acquire).
#ifndef RO_TBAR_SLEEP
#define RO_TBAR_SLEEP 1  // s_sleep between polls of a team barrier
#endif
struct RoTeamBar {
  int* ctr;
  int target;
  int lane;
  __device__ __forceinline__ void operator()() {
    target += 4;
    if (lane == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target)
      __builtin_amdgcn_s_sleep(RO_TBAR_SLEEP);
  }
};

template <int NJ>
__global__ void __launch_bounds__(2 * CACTO_THREADS, 1)
    k_rollout_tt(const SysDevice* __restrict__ sdp, NetView N, const double* __restrict__ S0,
                 const int32_t* __restrict__ nsteps, int T, int use_actor, double* __restrict__ Straj,
                 float* __restrict__ Atraj, int32_t* __restrict__ status, const int32_t* __restrict__ order, int B) {
  constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA, NG = 1, SL = 4;
  constexpr int REGK = RoSplitTT::REGK, LDSK = RoSplitTT::LDSK;
  __shared__ RoTTShared<NJ> Sh;
  const SysDevice& sd = *sdp;
  const cacto_sys_params& p = sd.p;
  const int team = threadIdx.x >> 8;
  Lane L;
  // team-local wave (team 1's wave 0 is the workgroup's wave 7: the two teams' dynamics waves sit
  // on different SIMDs) and thread index
  L.wave = (L.wave + team) & 3;
  L.tid = L.wave * 64 + L.lane;
  RoTeamShared<NJ>& S = Sh.team[team];
  RoActorRegs<ns, REGK> R;
  if (use_actor) {
    const float* W1 = N.flat + N.t.woff[0];
    const float* W2 = N.flat + N.t.woff[1];
    const float* W3 = N.flat + N.t.woff[2];
    const int f = 64 * L.wave + L.lane;
#pragma unroll
    for (int k = 0; k < REGK; ++k) R.w2[k] = W2[k * 256 + f];
#pragma unroll
    for (int q = 0; q < ns; ++q) R.w1[q] = W1[q * 256 + f];
    R.b1 = N.bias(0, f);
    R.b2 = N.bias(1, f);
    for (int e = threadIdx.x; e < LDSK * 64; e += 2 * CACTO_THREADS) {
      const int lane = e & 63, w = (e >> 6) & 3, kq = e >> 8;
      const int k = REGK + 4 * kq, col = 64 * w + lane;
      Sh.w2[e] = make_float4(W2[k * 256 + col], W2[(k + 1) * 256 + col], W2[(k + 2) * 256 + col],
                             W2[(k + 3) * 256 + col]);
    }
    for (int e = threadIdx.x; e < na * 256; e += 2 * CACTO_THREADS) Sh.w3[e] = W3[(e & 255) * na + (e >> 8)];
    if (threadIdx.x < 8) Sh.b3[threadIdx.x] = threadIdx.x < na ? N.bias(2, threadIdx.x) : 0.f;
  }
  if (L.tid < 64) S.W.x0[L.tid] = 0.f;
  for (int e = L.tid; e < SL * ns; e += CACTO_THREADS) S.sS[e] = 0.0;
  if (L.tid < SL) S.sact[L.tid] = 0;
  if (L.tid == 0) S.bar = 0;
  __syncthreads();  // the only workgroup barrier: weights and team state in place
  RoTeamBar tbar{&S.bar, 0, L.lane};
  const int vb = 2 * (int)blockIdx.x + team, G = 2 * (int)gridDim.x;
  int head = 0;
  const RoNorm<ns> nrm(p);
  const RoSimScalars ks{p.dt, p.L_delta, p.tau_delta};
  const int c = L.lane % SL;
  // prismatic chains (the host runs this kernel for const_dyn chains only): M's Cholesky factor
  // and h do not depend on (q, v) — the values k_const_dyn_init tabled in SysDevice, computed by
  // the same chain_terms -> cholesky the single-team kernel runs per episode
  ConstDyn<NJ> cd;
  if constexpr (NJ > 0) {
#pragma unroll
    for (int k = 0; k < NJ * NJ; ++k) cd.L[k] = sd.cd_L[k];
#pragma unroll
    for (int i = 0; i < NJ; ++i) cd.h[i] = sd.cd_h[i];
  }
  RoSlotRegs<NJ, NG> sr;
  if (L.wave == 0) {
    ro_refill<NJ, NG, RoTeamShared<NJ>, false>(L.lane < SL, L.lane, head, S, sd, S0, nsteps, order, T, B, G, Straj,
                                                status, nrm, L, vb);
    const uint64_t m = __ballot(L.lane < SL && S.sact[L.lane]);
    if (L.lane == 0) S.anyact = m != 0;
    sr.load(S, c, false);
  }
  tbar();
  const RoX0Lane<ns, SL> x0l(nrm, L.lane);
  RoTeamView<na> V{Sh.w2, Sh.w3, Sh.b3, S.W.h1, S.W.h2, S.W.x0, S.W.a};
  const float* W2g = N.flat + N.t.woff[1];
#ifdef CACTO_STAMPS
#define TSTAMP(k)                                                                                          \
  do {                                                                                                     \
    if (blockIdx.x == 0 && L.wave == 0 && L.lane == 0 && it == 20) g_rstamps[8 * team + k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  // accumulated phase cycles of every step of every team (waves 0 and 1 of the team, lane 0):
  // [0] layer 1 + its barrier, [1] layer 2 + barrier, [2] layer 3 + barrier, [3] dynamics, stores,
  // refill (wave 0; the other waves go straight to the barrier), [4] the end-of-step barrier
  // (wave 0 also splits [3]: [5] action read + s' = f(s, a), [6] trajectory stores, [7] refill,
  // [8] next input + ballot)
  unsigned long long tacc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, tprev = 0, tsub = 0;
  int tbi = 0;
  auto tmark = [&](int ph) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    if (ph == 1) tacc[0] += now - tprev;
    if (ph == 2) tacc[1] += now - tprev;
    if (ph == 3) tacc[2] += now - tprev;
    if (ph == 4) tacc[3] += now - tprev;
    if (ph == 5) tacc[4] += now - tprev;
    tprev = now;
    tsub = now;
  };
  auto tsubmark = [&](int k) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    if (k == 5) tacc[5] += now - tsub;
    if (k == 6) tacc[6] += now - tsub;
    if (k == 7) tacc[7] += now - tsub;
    if (k == 8) tacc[8] += now - tsub;
    tsub = now;
  };
#define TSUB(k) tsubmark(k)
  auto sbar = [&] {
    tbar();
    tmark(++tbi);
  };
  int tsteps = 0;
#else
#define TSTAMP(k) \
  do {            \
  } while (0)
#define TSUB(k) \
  do {          \
  } while (0)
#endif
  for (int it = 0; S.anyact; ++it) {
    TSTAMP(0);
    // Every wave must have read S.anyact (the loop test) before wave 0 rewrites it below. With the
    // actor, its first team barrier orders that; without it (ep == 0, zero controls) this barrier
    // does: a counter barrier, unlike s_barrier, would wait forever for waves that left the loop on
    // an anyact they read too late.
    if (!use_actor) tbar();
#ifdef CACTO_STAMPS
    tbi = 0;
    tmark(0);
    if (use_actor) ro_actor<NG, ns, na, REGK, LDSK, true, true>(R, V, W2g, L, it, sbar);
#else
    if (use_actor) ro_actor<NG, ns, na, REGK, LDSK, true, true>(R, V, W2g, L, it, tbar);
#endif
    TSTAMP(1);
    if (L.wave == 0) {
      const bool active = L.lane < SL && sr.act;
      bool fin = false;
      float a[na];
      if (active) {
        double ad[na], sn[ns];
#pragma unroll
        for (int i = 0; i < na; ++i) {
          a[i] = use_actor ? S.W.a[c * na + i] : 0.f;
          ad[i] = (double)a[i];
        }
        ro_simulate<NJ>(ks, cd, sr.s, ad, sn);
#pragma unroll
        for (int i = 0; i < ns; ++i) {
          S.sS[c * ns + i] = sn[i];
          sr.s[i] = sn[i];
        }
      }
      TSUB(5);
      if (active) {
        fin = ro_advance<NJ, NG>(c, sr.b, sr.t, sr.s, a, sd, T, Straj, Atraj, status, nrm, sr.n);
        sr.t += 1;
      }
      TSUB(6);
      ro_refill<NJ, NG, RoTeamShared<NJ>, false>(fin, c, head, S, sd, S0, nsteps, order, T, B, G, Straj, status, nrm,
                                                  L, vb);
      if (fin) sr.load(S, c, false);
      TSUB(7);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      x0l.write(S, nrm, L.lane);
      const uint64_t m = __ballot(L.lane < SL && S.sact[c]);
      if (L.lane == 0) S.anyact = m != 0;
      TSUB(8);
      TSTAMP(2);
    }
#ifdef CACTO_STAMPS
    tmark(4);
#endif
    tbar();
    TSTAMP(3);
#ifdef CACTO_STAMPS
    tmark(5);
    ++tsteps;
#endif
  }
#ifdef CACTO_STAMPS
  if (L.lane == 0 && L.wave < 2) {
    unsigned long long* o = g_ttacc + ((size_t)(blockIdx.x * 2 + team) * 2 + L.wave) * 10;
    for (int k = 0; k < 9; ++k) o[k] = tacc[k];
    o[9] = tsteps;
  }
#endif
#undef TSTAMP
#undef TSUB
}

// x[lane] for lanes < N (x uniform across the wave) as a select chain kept in VGPRs: without the
// empty asm the optimiser turns the chain into an indexed load from a scratch copy of x.
template <int N, typename V>
__device__ __forceinline__ V lane_pick(const V* x, int lane) {
  V v = x[0];
#pragma unroll
  for (int i = 1; i < N; ++i) {
    v = lane == i ? x[i] : v;
    __asm__ volatile("" : "+v"(v));
  }
  return v;
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// ---------------------------------------------------------------- one slot per wave, K split
// k_rollout_ks: one 8-wave workgroup per CU runs 8 episode slots, wave w owning slot w: after
// layer 2 the wave forms its slot's action (layer 3 — ro_actor's P = 64 lane chains per slot are
// exactly one wave, and the two actions share one permlane butterfly), steps the f64 dynamics,
// writes the trajectory (one component per lane), refills its slot from the workgroup's queue (an
// LDS counter: which slot runs an episode does not change its result) and evaluates layer 1 of its
// slot for all 256 features as fmaf chains straight into the layer-2 operand layout (a K = 1 MFMA
// step rounds exactly like fmaf, tools/mb/mfma_fma.hip). Layer 2 is split over
// the waves by feature quarter AND by half of K: wave (fq, h) = (w & 3, w >> 2) multiplies the
// 128 rows [128 h, 128 h + 128) of W2 for features 64 fq + lane — held in its registers for the
// whole launch, so the 256 KB of layer-2 weights live in the 8 waves' registers and no weight row
// is read from LDS per step — for all 8 slots (two groups of 4 samples, 256 MFMAs), and parks its
// half sum; layer 3 adds the two halves (the SPLIT order of ro_layer2, so results are identical to
// the other rollout kernels). Two hardware barriers per step (one workgroup = one team).
// Systems: SI, DI, car, car_park and the planar 3R chain (the manipulator), whose dynamics are the
// closed form planar3_step (M(q), h(q, v) from the link COM vectors, one 3x3 adjugate solve) —
// short enough for one wave per slot, where the generic chain needs RNEA / CRBA spread over a
// workgroup (k_rollout<3, NG> steps a planar chain with planar3_step too).
template <int NJ>
struct RoKsShared {
  float h1[2 * 4 * RoCfg<1>::H1B];  // layer-1 output of the 8 slots (groups 0, 1), layer-2 operand layout
  float P[2][8 * 256];              // layer-2 half sums [k half][slot][feature]
  int act[8];                       // slot active flags, published by the barrier that ends a step
  int qhead;                        // the workgroup's next queue entry
  // the planar 3R chain keeps W3^T, b2 and its link constants here instead of in registers (its
  // wider input and output layers and the float64 dynamics would otherwise not fit beside the 128
  // layer-2 weight registers); read with layer 3's half sums and during the dynamics' sincos
  static constexpr bool LW = NJ == 3;
  float w3s[LW ? 3 * 256 : 1];  // W3^T [a][f]
  float b2s[LW ? 256 : 1];
  float4 w1s[LW ? 8 * 64 : 1];  // W1 [q][lane][m] = W1[q][lane + 64 m] (q < ns), then b1 [lane][m] at q = 7
  double pls[LW ? 20 : 1];
};

template <int NJ>
__global__ void __launch_bounds__(8 * CACTO_WAVE, 1)
    k_rollout_ks(const SysDevice* __restrict__ sdp, NetView N, const double* __restrict__ S0,
                 const int32_t* __restrict__ nsteps, int T, int use_actor, double* __restrict__ Straj,
                 float* __restrict__ Atraj, int32_t* __restrict__ status, const int32_t* __restrict__ order, int B) {
  constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  constexpr int H1B = RoCfg<1>::H1B;
  __shared__ RoKsShared<NJ> Sh;
  const SysDevice& sd = *sdp;
  const cacto_sys_params& p = sd.p;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fq = w & 3, hk = w >> 2;  // layer 2: features 64 fq + lane, rows [128 hk, 128 hk + 128)
  const int sg = w >> 2, si = w & 3;  // this wave's slot w = 4 sg + si (group, sample)
  constexpr bool LW = RoKsShared<NJ>::LW;
  float w2[128], b2[LW ? 1 : 4], w1[LW ? 1 : ns][4], b1[LW ? 1 : 4], w3[LW ? 1 : na][4], b3[na];
  if (use_actor) {
    const float* W1 = N.flat + N.t.woff[0];
    const float* W2 = N.flat + N.t.woff[1];
    const float* W3 = N.flat + N.t.woff[2];
#pragma unroll
    for (int k = 0; k < 128; ++k) w2[k] = W2[(128 * hk + k) * 256 + 64 * fq + lane];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if constexpr (!LW) {
#pragma unroll
        for (int q = 0; q < ns; ++q) w1[q][m] = W1[q * 256 + lane + 64 * m];
        b1[m] = N.bias(0, lane + 64 * m);
        b2[m] = N.bias(1, lane + 64 * m);
#pragma unroll
        for (int a = 0; a < na; ++a) w3[a][m] = W3[(lane + 64 * m) * na + a];
      }
    }
#pragma unroll
    for (int a = 0; a < na; ++a) b3[a] = N.bias(2, a);
    if constexpr (LW) {
      for (int e = threadIdx.x; e < na * 256; e += 8 * CACTO_WAVE) Sh.w3s[e] = W3[(e & 255) * na + (e >> 8)];
      for (int e = threadIdx.x; e < 256; e += 8 * CACTO_WAVE) Sh.b2s[e] = N.bias(1, e);
      for (int e = threadIdx.x; e < 8 * 64; e += 8 * CACTO_WAVE) {
        const int q = e >> 6, l = e & 63;
        float4 v;
        if (q < ns)
          v = make_float4(W1[q * 256 + l], W1[q * 256 + l + 64], W1[q * 256 + l + 128], W1[q * 256 + l + 192]);
        else
          v = make_float4(N.bias(0, l), N.bias(0, l + 64), N.bias(0, l + 128), N.bias(0, l + 192));
        Sh.w1s[e] = v;
      }
    }
  }
  if constexpr (LW)
    if (threadIdx.x < 20) Sh.pls[threadIdx.x] = sd.pl[threadIdx.x];
  for (int e = threadIdx.x; e < 2 * 4 * H1B; e += 8 * CACTO_WAVE) Sh.h1[e] = 0.f;
  if (threadIdx.x == 0) Sh.qhead = 0;
  __syncthreads();
  const int vb = (int)blockIdx.x, G = (int)gridDim.x;
  const RoNorm<ns> nrm(p);
  float nl = 1.f;
#pragma unroll
  for (int q = 0; q < ns; ++q) nl = lane == q ? nrm.n[q] : nl;
  const bool tl = lane == ns - 1;
  // the prismatic chain's constant Cholesky factor and bias forces; the planar 3R chain's link
  // constants (planar3_step)
  ConstDyn<NJ> cd;
  if constexpr (NJ > 0 && NJ != 3) {
#pragma unroll
    for (int k = 0; k < NJ * NJ; ++k) cd.L[k] = sd.cd_L[k];
#pragma unroll
    for (int i = 0; i < NJ; ++i) cd.h[i] = sd.cd_h[i];
  }
  const RoSimScalars ks{p.dt, p.L_delta, p.tau_delta};
  bool act = false;
  int b = 0, n = 0, t = 0;
  double s[ns];
#pragma unroll
  for (int i = 0; i < ns; ++i) s[i] = 0.0;

  // the next queue entries until one has steps (ro_refill's dealing: snake order over the
  // workgroups; zero-length episodes completed on the spot)
  auto refill = [&]() {
    act = false;
    while (true) {
      int k = 0;
      if (lane == 0) k = __hip_atomic_fetch_add(&Sh.qhead, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      k = __builtin_amdgcn_readfirstlane(k);
      const int r = k * G + ((k & 1) ? G - 1 - vb : vb);
      if (r >= B) return;
      const int bb = __builtin_amdgcn_readfirstlane(order ? order[r] : r);
      const int nn = min(nsteps[bb], T);
#pragma unroll
      for (int i = 0; i < ns; ++i) s[i] = S0[(size_t)bb * ns + i];
      if (Straj && lane < ns) Straj[(size_t)bb * (T + 1) * ns + lane] = lane_pick<ns>(s, lane);
      if (nn == 0) {
        if (status && lane == 0) status[bb] = 0;
        continue;
      }
      b = bb;
      n = nn;
      t = 0;
      act = true;
      return;
    }
  };
  // layer 1 of this wave's slot from s_t: x0[q] = normalise(s_t[q]) on lane q, broadcast through
  // readlane; h1[k] = lrelu(b1[k] + sum_q x0[q] W1[q][k]) for k = lane + 64 m, into the slot's
  // column of the two-group layer-2 operand layout
  auto layer1 = [&]() {
    const double sv = lane_pick<ns>(s, lane);
    const float qv = fdiv((float)sv, nl);
    const float xv = nrm.on ? (tl ? fsub(fmul(qv, 2.0f), 1.0f) : qv) : (float)sv;
    float x0[ns];
#pragma unroll
    for (int q = 0; q < ns; ++q) x0[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv), q));
    if constexpr (LW) {
      float4 wq[ns + 1];  // W1 rows and b1 of this lane's 4 features, from LDS
#pragma unroll
      for (int q = 0; q <= ns; ++q) wq[q] = Sh.w1s[(q < ns ? q : 7) * 64 + lane];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < ns; ++q) acc = __builtin_fmaf(x0[q], get4(wq[q], m), acc);
        Sh.h1[(sg * 4 + m) * H1B + (lane & 15) * 20 + 4 * si + (lane >> 4)] = lrelu(fadd(acc, get4(wq[ns], m)));
      }
    } else {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < ns; ++q) acc = __builtin_fmaf(x0[q], w1[q][m], acc);
        Sh.h1[(sg * 4 + m) * H1B + (lane & 15) * 20 + 4 * si + (lane >> 4)] = lrelu(fadd(acc, b1[m]));
      }
    }
  };

#ifdef CACTO_STAMPS
  // accumulated phase cycles of every step (lane 0 of each wave): [0] loop test + layer 2 + its
  // barrier, [1] layer 3, [2] s' = f(s, a) + trajectory stores, [3] refill, [4] layer 1, [5] the
  // end-of-step barrier
  unsigned long long wacc[6] = {0, 0, 0, 0, 0, 0}, wprev = __builtin_amdgcn_s_memtime();
  int wsteps = 0;
  auto wmark = [&](int ph) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if (k == ph) wacc[k] += now - wprev;
    wprev = now;
  };
#define KMARK(k) wmark(k)
#else
#define KMARK(k) \
  do {           \
  } while (0)
#endif

  refill();
  if (act && use_actor) layer1();
  if (lane == 0) Sh.act[w] = act;
  __syncthreads();
  const int rd = (lane >> 2) * 20 + 4 * (lane & 3);
  for (int it = 0;; ++it) {
    int any = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) any |= Sh.act[k];
    if (any == 0) break;
    // every wave has read the flags (above) before any wave rewrites its own below: the layer-2
    // barrier orders that; without the actor this barrier does
    if (!use_actor) __syncthreads();
    float a[na];
#pragma unroll
    for (int i = 0; i < na; ++i) a[i] = 0.f;
    if (use_actor) {
      // layer 2, this wave's half of K for features 64 fq + lane, both slot groups
      float4 xa[2][2];
#pragma unroll
      for (int gg = 0; gg < 2; ++gg)
#pragma unroll
        for (int kl = 0; kl < 2; ++kl)
          xa[gg][kl] = *reinterpret_cast<const float4*>(&Sh.h1[(gg * 4 + 2 * hk + kl) * H1B + rd]);
      floatx4 acc[2][2];
#pragma unroll
      for (int gg = 0; gg < 2; ++gg) acc[gg][0] = acc[gg][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kl = 0; kl < 2; ++kl)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          static_for<16>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
#pragma unroll
            for (int gg = 0; gg < 2; ++gg)
              acc[gg][q & 1] = mfma_bc<q>(get4(xa[gg][kl], v), w2[64 * kl + 16 * v + q], acc[gg][q & 1]);
          });
#pragma unroll
      for (int gg = 0; gg < 2; ++gg)
#pragma unroll
        for (int i = 0; i < 4; ++i) Sh.P[hk][(4 * gg + i) * 256 + 64 * fq + lane] = fadd(acc[gg][0][i], acc[gg][1][i]);
      __syncthreads();
      KMARK(0);
      if (act) {
        // layer 3 of slot w on the two halves' sums: h2 = lrelu((lo + hi) + b2), then ro_actor's
        // chains and butterfly (both actions in one permlane butterfly for na == 2)
        float pa[na];
#pragma unroll
        for (int i = 0; i < na; ++i) pa[i] = 0.f;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int f = lane + 64 * m;
          const float h = lrelu(fadd(fadd(Sh.P[0][w * 256 + f], Sh.P[1][w * 256 + f]), LW ? Sh.b2s[f] : b2[m % (LW ? 1 : 4)]));
#pragma unroll
          for (int i = 0; i < na; ++i) pa[i] = fmaf(LW ? Sh.w3s[i * 256 + f] : w3[LW ? 0 : i][m], h, pa[i]);
        }
        if constexpr (na == 2) {
          const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(pa[0]), __float_as_uint(pa[1]), false, false);
          float v = __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
          const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
          v = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
#pragma unroll
          for (int off = 8; off >= 1; off >>= 1) v = add_from_above(v, off);
          a[0] = fadd(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)), b3[0]);
          a[1] = fadd(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)), b3[1 % na]);
        } else if constexpr (na == 3) {
          // actions 0 / 1 as above, action 2 through the same levels on its own (lanes 0-31 hold
          // the sums after the first swap); the adds are the butterfly's, so the bits are too
          const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(pa[0]), __float_as_uint(pa[1]), false, false);
          const auto q32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(pa[2]), __float_as_uint(pa[2]), false, false);
          float v = __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
          float v2 = __uint_as_float(q32[0]) + __uint_as_float(q32[1]);
          const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
          const auto q16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v2), __float_as_uint(v2), false, false);
          v = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
          v2 = __uint_as_float(q16[0]) + __uint_as_float(q16[1]);
#pragma unroll
          for (int off = 8; off >= 1; off >>= 1) {
            v = add_from_above(v, off);
            v2 = add_from_above(v2, off);
          }
          a[0] = fadd(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)), b3[0]);
          a[1] = fadd(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)), b3[1 % na]);
          a[2 % na] = fadd(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v2), 0)), b3[2 % na]);
        } else {
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
            for (int i = 0; i < na; ++i) pa[i] = add_from_above(pa[i], off);
#pragma unroll
          for (int i = 0; i < na; ++i)
            a[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(fadd(pa[i], b3[i]))));
        }
      }
      KMARK(1);
    }
    bool fin = false;
    if (act) {
      double ad[na], sn[ns];
#pragma unroll
      for (int i = 0; i < na; ++i) ad[i] = (double)a[i];
      if constexpr (NJ == 3) {
        // sin / cos of q1 on even lanes and of q2 on odd lanes at once (joint_sincos is the
        // function planar3_step calls, so the bits are the same)
        double sv, cv;
        joint_sincos((lane & 1) ? s[2] : s[1], &sv, &cv);
        planar3_step_sc(Planar3(Sh.pls), ks.dt, s, ad, readlane_d(sv, 0), readlane_d(cv, 0), readlane_d(sv, 1),
                        readlane_d(cv, 1), sn);
      } else
        ro_simulate<NJ>(ks, cd, s, ad, sn);
      bool bad = false;
#pragma unroll
      for (int i = 0; i < ns; ++i) bad |= isnan(sn[i]);
      if (Atraj && lane < na) Atraj[((size_t)b * T + t) * na + lane] = lane_pick<na>(a, lane);
      if (Straj && lane < ns) Straj[((size_t)b * (T + 1) + t + 1) * ns + lane] = lane_pick<ns>(sn, lane);
      if (bad && Straj) {
        for (int e = lane; e < (n - t - 1) * ns; e += 64)
          Straj[((size_t)b * (T + 1) + t + 2) * ns + e] = __builtin_nan("");
      }
      fin = bad || t + 1 >= n;
      if (fin && status && lane == 0) status[b] = bad ? 1 : 0;
#pragma unroll
      for (int i = 0; i < ns; ++i) s[i] = sn[i];
      t += 1;
    }
    KMARK(2);
    if (fin) refill();
    KMARK(3);
    if (act && use_actor) layer1();
    if (lane == 0) Sh.act[w] = act;
    KMARK(4);
    __syncthreads();
    KMARK(5);
#ifdef CACTO_STAMPS
    ++wsteps;
#endif
  }
#ifdef CACTO_STAMPS
  if (lane == 0) {
    unsigned long long* o = g_wsacc + ((size_t)blockIdx.x * 8 + w) * 7;
    for (int k = 0; k < 6; ++k) o[k] = wacc[k];
    o[6] = wsteps;
  }
#endif
#undef KMARK
}

// Rewards and end-effector positions of every recorded step (Env.step's reward and
// get_end_effector_position, environment.py:70-78, :146-156): one thread per (episode, t),
// r_t = reward(w, s_t, a_t) for t < n, EE_t = EE(s_t) for t <= n; NaN states (a dropped episode)
// are skipped.
template <int NJ>
__global__ void __launch_bounds__(256, 4) k_rollout_rewards(const SysDevice* __restrict__ sdp, const double* __restrict__ Straj,
                                                         const float* __restrict__ Atraj, const int32_t* __restrict__ nsteps,
                                                         int T, int use_actor, const double* __restrict__ Wext,
                                                         double* __restrict__ Rtraj, double* __restrict__ EEtraj, int B) {
  constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  const SysDevice& sd = *sdp;
  const int64_t total = (int64_t)B * (T + 1);
  double w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = k >= sd.p.n_weights ? 0.0 : Wext ? Wext[k] : sd.p.w_running[k];
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / (T + 1)), t = (int)(e % (T + 1));
    const int n = min(nsteps[b], T);
    if (t > n) continue;
    double s[ns];
    bool bad = false;
#pragma unroll
    for (int i = 0; i < ns; ++i) {
      s[i] = Straj[(size_t)e * ns + i];
      bad |= isnan(s[i]);
    }
    if (bad) continue;
    const V3 v = env_ee<NJ>(sd, s);  // once, for the EE row and the reward
    if (EEtraj) {
      EEtraj[(size_t)e * 3 + 0] = v.x;
      EEtraj[(size_t)e * 3 + 1] = v.y;
      EEtraj[(size_t)e * 3 + 2] = v.z;
    }
    if (Rtraj && t < n) {
      double a[na];
#pragma unroll
      for (int i = 0; i < na; ++i) a[i] = use_actor ? (double)Atraj[((size_t)b * T + t) * na + i] : 0.0;
      Rtraj[(size_t)b * T + t] = env_reward_at<NJ>(sd, w, s, a, false, v);
    }
  }
}

// The same per-element work over the COMPACTED element space: element e of [0, sum_b (n_b + 1))
// is step t = e - off[b] of episode b (off = exclusive prefix of n_b + 1, n_b = min(nsteps[b], T)),
// so every lane of a wave has a recorded step. The per-element code is f64-issue bound (~1.5 k f64
// instructions for DI), and in the [b][t] grid about 40 % of the waves that had any work straddled
// an episode's end with part of their lanes idle. Each workgroup scans the B lengths into LDS
// itself (B <= CACTO_REW_SCAN_MAX; the L2-resident lengths are read once per workgroup) and finds
// an element's episode by binary search there. Same values written (bit-identical).
#define CACTO_REW_SCAN_MAX 16000  // (B + 1) ints within the 64 KiB of dynamic LDS
template <int NJ>
__global__ void __launch_bounds__(256, 4) k_rollout_rewards_c(const SysDevice* __restrict__ sdp,
                                                           const double* __restrict__ Straj,
                                                           const float* __restrict__ Atraj,
                                                           const int32_t* __restrict__ nsteps, int T, int use_actor,
                                                           const double* __restrict__ Wext, double* __restrict__ Rtraj,
                                                           double* __restrict__ EEtraj, int B) {
  constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  extern __shared__ int offs[];  // B + 1
  __shared__ int wsum[4];
  const SysDevice& sd = *sdp;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // block exclusive scan of the element counts: thread tid owns episodes [tid*per, tid*per + per)
  const int per = (B + 255) / 256, b0 = tid * per;
  int loc = 0;
  for (int k = 0; k < per; ++k) {
    const int b = b0 + k;
    if (b < B) {
      const int n = min(nsteps[b], T);
      loc += n >= 0 ? n + 1 : 0;
    }
  }
  int inc = loc;  // inclusive scan over the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(inc, d);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wv; ++w) base += wsum[w];
  int run = base + inc - loc;
  for (int k = 0; k < per; ++k) {
    const int b = b0 + k;
    if (b < B) {
      offs[b] = run;
      const int n = min(nsteps[b], T);
      run += n >= 0 ? n + 1 : 0;
    }
  }
  if (tid == 255) offs[B] = base + inc;
  __syncthreads();
  const int total = offs[B];
  double w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = k >= sd.p.n_weights ? 0.0 : Wext ? Wext[k] : sd.p.w_running[k];
  for (int e = blockIdx.x * 256 + tid; e < total; e += gridDim.x * 256) {
    int lo = 0, hi = B;  // the last b with offs[b] <= e (empty episodes are skipped over)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (offs[mid] <= e) lo = mid;
      else hi = mid;
    }
    const int b = lo, t = e - offs[b];
    const int n = min(nsteps[b], T);
    const size_t row = (size_t)b * (T + 1) + t;
    double s[ns];
    bool bad = false;
#pragma unroll
    for (int i = 0; i < ns; ++i) {
      s[i] = Straj[row * ns + i];
      bad |= isnan(s[i]);
    }
    if (bad) continue;
    const V3 v = env_ee<NJ>(sd, s);
    if (EEtraj) {
      EEtraj[row * 3 + 0] = v.x;
      EEtraj[row * 3 + 1] = v.y;
      EEtraj[row * 3 + 2] = v.z;
    }
    if (Rtraj && t < n) {
      double a[na];
#pragma unroll
      for (int i = 0; i < na; ++i) a[i] = use_actor ? (double)Atraj[((size_t)b * T + t) * na + i] : 0.0;
      Rtraj[(size_t)b * T + t] = env_reward_at<NJ>(sd, w, s, a, false, v);
    }
  }
}

// Episode slots per workgroup and workgroup count for B episodes: about two episodes per slot
// (their lengths pair up long + short), one workgroup per CU.
inline int ro_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      cus = v;
    else
      cus = 256;
  }
  return cus;
}

}  // namespace cacto

using namespace cacto;

namespace {
template <int NJ>
struct LaunchRolloutRewards {
  static int run(const cacto_sys* sys, const double* S, const float* A, const int32_t* n, int T, int use_actor,
                 const double* W, double* R, double* EE, int B, hipStream_t st) {
    const int64_t total = (int64_t)B * (T + 1);
    // compacted elements where the per-element reward is long enough to pay for the per-workgroup
    // scan and the per-element search (measured r03: car_park's 30 smooth boxes 410 -> 428 M
    // env-steps/s; DI's rewards 29.9 -> 34.5 us, the chains unchanged). CACTO_REW_GRID=bt|c forces
    // one (benchmarks).
    static const char* force = std::getenv("CACTO_REW_GRID");
    const bool compact = force ? force[0] == 'c' : NJ == -2;
    if (B <= CACTO_REW_SCAN_MAX && compact) {
      // compacted elements: at most 4 workgroups per CU (each scans the lengths once)
      const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 4 * ro_cus()));
      hipLaunchKernelGGL(k_rollout_rewards_c<NJ>, dim3(grid), dim3(256), (size_t)(B + 1) * sizeof(int), st, sys->dev,
                         S, A, n, T, use_actor, W, R, EE, B);
    } else {
      const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 8 * ro_cus()));
      hipLaunchKernelGGL(k_rollout_rewards<NJ>, dim3(grid), dim3(256), 0, st, sys->dev, S, A, n, T, use_actor, W, R,
                         EE, B);
    }
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
};

template <int NJ>
struct LaunchRollout {
  static int run(const cacto_sys* sys, NetView v, const double* S0, const int32_t* n, int T, int use_actor,
                 const double* W, double* S, float* A, double* R, double* EE, int32_t* status, const int32_t* order,
                 int B, int groups, int wgs, hipStream_t st) {
    const int cus = ro_cus();
    // two teams of 4 slots per workgroup (k_rollout_tt) for the systems whose step needs no
    // workgroup-wide dynamics: automatically where the single-team kernel would take 2 groups,
    // or on request (groups == -1)
    constexpr bool tt_ok = NJ <= 2 && !(NJ > 0 && !RoConstDyn<NJ>::ok);
    const bool tt_sys = tt_ok && (NJ <= 0 || sys->host.p.const_dyn);
    // automatic only where it measured faster: the prismatic chain (DI 0.75 -> 0.72 ms at 4096
    // episodes); car_park's step was slower on two teams (0.42 -> 0.50 ms)
    const bool tt_auto = tt_sys && NJ > 0;
    // planar 3-joint chains (the manipulator): k_rollout_ks with the closed-form planar3_step
    constexpr bool ks_ok = tt_ok || NJ == 3;
    const bool planar = NJ == 3 && sys->host.pl[0] != 0.0;
    const bool ks_sys = tt_sys || planar;
    if ((groups == -1 && !tt_sys) || (groups == -3 && !ks_sys)) {
      set_error("cacto_rollout_sched: groups -1 needs a system without configuration-dependent M, -3 such a system "
                "or a planar 3-joint chain");
      return CACTO_EINVAL;
    }
    // one slot per wave with layer 2 split over K (k_rollout_ks) for every system it can run, up
    // to two episodes per slot. Measured at 4096 episodes (ms per rollout, one MI355X): DI
    // k_rollout_tt 0.750 / one slot per wave in two teams (round 4, removed) 0.630 / k_rollout_ks
    // 0.578; SI single-team 0.519 / ks 0.292; car_park single-team 0.432 / ks 0.405; car 1.865 / 1.768.
    // The planar chain takes it at every batch size.
    const bool ks_auto = (tt_sys && B <= 2 * 8 * cus) || planar;
    if (groups == -3 || (groups == 0 && ks_auto)) {
      // one slot per wave, layer 2 split over K (k_rollout_ks), one 8-wave workgroup per CU
      if (wgs <= 0) wgs = std::min(cus, ceil_div(B, 8));
      wgs = std::max(1, std::min(wgs, ceil_div(B, 8)));
      if constexpr (ks_ok)
        hipLaunchKernelGGL(k_rollout_ks<NJ>, dim3(wgs), dim3(8 * CACTO_WAVE), 0, st, sys->dev, v, S0, n, T,
                           use_actor, S, A, status, order, B);
      CACTO_CHECK_HIP(hipGetLastError());
      if (R || EE) return LaunchRolloutRewards<NJ>::run(sys, S, A, n, T, use_actor, W, R, EE, B, st);
      return CACTO_OK;
    }
    if (tt_sys && (groups == -1 || (tt_auto && groups == 0 && B / (2 * 4 * cus) == 2))) {
      if (wgs <= 0) wgs = std::min(cus, ceil_div(B, 8));
      wgs = std::max(1, std::min(wgs, ceil_div(B, 8)));
      if constexpr (tt_ok)
        hipLaunchKernelGGL(k_rollout_tt<NJ>, dim3(wgs), dim3(2 * CACTO_THREADS), 0, st, sys->dev, v, S0, n, T,
                           use_actor, S, A, status, order, B);
      CACTO_CHECK_HIP(hipGetLastError());
      if (R || EE) return LaunchRolloutRewards<NJ>::run(sys, S, A, n, T, use_actor, W, R, EE, B, st);
      return CACTO_OK;
    }
    // the float64 6-joint chain dynamics need the registers that more slots would take
    constexpr int gmax = 4;
    if (groups <= 0) {
      // about two episodes per slot. (UR5 at 2048 episodes: one group, two episodes per slot,
      // 1.25 ms against 1.28 ms for two groups with one episode per slot, tools/ro_sched.py.)
      const int per = B / (2 * 4 * cus);
      groups = std::min(gmax, per >= 4 ? 4 : per >= 2 ? 2 : 1);
    }
    if (groups > gmax) {
      set_error("cacto_rollout_sched: groups above this system's maximum (1 for 6 joints)");
      return CACTO_EINVAL;
    }
    if (wgs <= 0) wgs = std::min(cus, ceil_div(B, 4 * groups));
    wgs = std::max(1, std::min(wgs, ceil_div(B, 4 * groups)));
    switch (groups) {
      case 1:
        hipLaunchKernelGGL((k_rollout<NJ, 1>), dim3(wgs), dim3(CACTO_THREADS), 0, st, sys->dev, v, S0, n, T, use_actor,
                           S, A, status, order, B);
        break;
      case 2:
        hipLaunchKernelGGL((k_rollout<NJ, (gmax >= 2 ? 2 : 1)>), dim3(wgs), dim3(CACTO_THREADS), 0, st, sys->dev, v, S0,
                           n, T, use_actor, S, A, status, order, B);
        break;
      case 4:
        hipLaunchKernelGGL((k_rollout<NJ, (gmax >= 4 ? 4 : 1)>), dim3(wgs), dim3(CACTO_THREADS), 0, st, sys->dev, v, S0,
                           n, T, use_actor, S, A, status, order, B);
        break;
      default:
        set_error("cacto_rollout_sched: groups must be 1, 2 or 4");
        return CACTO_EINVAL;
    }
    CACTO_CHECK_HIP(hipGetLastError());
    if (R || EE) return LaunchRolloutRewards<NJ>::run(sys, S, A, n, T, use_actor, W, R, EE, B, st);
    return CACTO_OK;
  }
};
}  // namespace

#ifdef CACTO_STAMPS
extern "C" int cacto_debug_rollout_stamps(unsigned long long* out_h) {
  CACTO_CHECK_HIP(hipDeviceSynchronize());
  CACTO_CHECK_HIP(hipMemcpyFromSymbol(out_h, HIP_SYMBOL(g_rstamps), sizeof(unsigned long long) * 20));
  return CACTO_OK;
}
// k_rollout_ks's accumulated phase cycles: 1024 x 8 x 7 values (see the kernel)
extern "C" int cacto_debug_rollout_ws_acc(unsigned long long* out_h) {
  CACTO_CHECK_HIP(hipDeviceSynchronize());
  CACTO_CHECK_HIP(hipMemcpyFromSymbol(out_h, HIP_SYMBOL(g_wsacc), sizeof(unsigned long long) * 1024 * 8 * 7));
  return CACTO_OK;
}
// k_rollout_tt's accumulated phase cycles: 1024 x 2 x 2 x 10 values (see the kernel)
extern "C" int cacto_debug_rollout_tt_acc(unsigned long long* out_h) {
  CACTO_CHECK_HIP(hipDeviceSynchronize());
  CACTO_CHECK_HIP(hipMemcpyFromSymbol(out_h, HIP_SYMBOL(g_ttacc), sizeof(unsigned long long) * 1024 * 2 * 2 * 10));
  return CACTO_OK;
}
#endif

extern "C" int cacto_rollout_sched(const cacto_sys* sys, const float* actor_netbuf_d, const double* S0_d,
                                   const int32_t* nsteps_d, int T, int use_actor, const double* W_d, double* S_traj_d,
                                   float* A_traj_d, double* R_traj_d, double* EE_traj_d, int32_t* status_d,
                                   const int32_t* order_d, int B, int groups, int workgroups, void* stream) {
  CACTO_REQUIRE(sys && S0_d && nsteps_d && T >= 0 && B >= 0, "cacto_rollout: bad arguments");
  CACTO_REQUIRE(!use_actor || actor_netbuf_d, "cacto_rollout: use_actor needs the actor net buffer");
  CACTO_REQUIRE(groups == 0 || groups == 1 || groups == 2 || groups == 4 || groups == -1 || groups == -3,
                "cacto_rollout_sched: groups must be 0, 1, 2, 4, -1 (two teams) or -3 (one slot per wave, layer 2 "
                "split over K)");
  CACTO_REQUIRE(workgroups >= 0, "cacto_rollout_sched: workgroups must be >= 0");
  CACTO_REQUIRE(!(R_traj_d || EE_traj_d) || (S_traj_d && (A_traj_d || !use_actor)),
                "cacto_rollout: R_traj / EE_traj need S_traj (and A_traj when use_actor)");
  if (B == 0) return CACTO_OK;
  NetView v = cacto_make_view(sys, CACTO_NET_ACTOR, actor_netbuf_d);
  return dispatch_nj<LaunchRollout>(sys->host.p, sys, v, S0_d, nsteps_d, T, use_actor, W_d, S_traj_d, A_traj_d,
                                    R_traj_d, EE_traj_d, status_d, order_d, B, groups, workgroups, as_stream(stream));
}

extern "C" int cacto_rollout_rewards(const cacto_sys* sys, const double* S_traj_d, const float* A_traj_d,
                                     const int32_t* nsteps_d, int T, int use_actor, const double* W_d,
                                     double* R_traj_d, double* EE_traj_d, int B, void* stream) {
  CACTO_REQUIRE(sys && S_traj_d && nsteps_d && T >= 0 && B >= 0, "cacto_rollout_rewards: bad arguments");
  CACTO_REQUIRE(!use_actor || A_traj_d, "cacto_rollout_rewards: use_actor needs A_traj");
  if (B == 0 || !(R_traj_d || EE_traj_d)) return CACTO_OK;
  return dispatch_nj<LaunchRolloutRewards>(sys->host.p, sys, S_traj_d, A_traj_d, nsteps_d, T, use_actor, W_d,
                                           R_traj_d, EE_traj_d, B, as_stream(stream));
}

extern "C" int cacto_rollout(const cacto_sys* sys, const float* actor_netbuf_d, const double* S0_d,
                             const int32_t* nsteps_d, int T, int use_actor, const double* W_d, double* S_traj_d,
                             float* A_traj_d, double* R_traj_d, double* EE_traj_d, int32_t* status_d,
                             const int32_t* order_d, int B, void* stream) {
  return cacto_rollout_sched(sys, actor_netbuf_d, S0_d, nsteps_d, T, use_actor, W_d, S_traj_d, A_traj_d, R_traj_d,
                             EE_traj_d, status_d, order_d, B, 0, 0, stream);
}
