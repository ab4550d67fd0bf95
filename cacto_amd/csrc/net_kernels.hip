// Network kernels: weight packing, actor/critic inference, critic input gradient, and the
// persistent rollout kernel (K18: actor MFMA tile + float64 dynamics per step, T steps in-kernel).
#include "net_common.h"

#ifdef CACTO_STAMPS
__device__ unsigned long long g_rstamps[8];
#define RSTAMP(k)                                                                   \
  do {                                                                              \
    if (blockIdx.x == 0 && threadIdx.x == 0 && t == 20) g_rstamps[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define RSTAMP(k) \
  do {            \
  } while (0)
#endif

namespace cacto {

// ---------------------------------------------------------------- packing
__global__ void k_pack(const float* flat, float* packed, NetTopo t) {
  const int64_t total = (int64_t)2 * t.blocks * 256;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(k & 3);
    const int lane = (int)((k >> 2) & 63);
    int blk = (int)(k >> 8);
    const bool tr = blk >= t.blocks;
    if (tr) blk -= t.blocks;
    int l = t.L - 1;
    while (t.pkoff[l] > blk) --l;
    const int local = blk - t.pkoff[l];
    const int g = lane >> 4, c = lane & 15;
    int i, o;
    if (!tr) {  // block (ot, kt): W[16kt + 4g + j][16ot + c]
      const int ot = local / t.KT[l], kt = local % t.KT[l];
      i = 16 * kt + 4 * g + j;
      o = 16 * ot + c;
    } else {  // block (it, kt): W[16it + c][16kt + 4g + j]
      const int it = local / t.OT[l], kt = local % t.OT[l];
      i = 16 * it + c;
      o = 16 * kt + 4 * g + j;
    }
    packed[k] = (i < t.in[l] && o < t.out[l]) ? flat[t.woff[l] + i * t.out[l] + o] : 0.f;
  }
}

// ---------------------------------------------------------------- inference
__global__ void __launch_bounds__(CACTO_THREADS) k_actor_forward(const SysDevice* __restrict__ sdp, NetView N,
                                                                 const float* __restrict__ S, float* __restrict__ Aout,
                                                                 int B) {
  __shared__ float4 X0[64];
  __shared__ float4 H[2 * 16 * 64];
  __shared__ float4 red[4 * 64];
  __shared__ float st[16 * 16];
  __shared__ float A[16 * CACTO_MAX_ACTION];
  const cacto_sys_params& p = sdp->p;
  const Lane L;
  const int ns = p.nb_state, na = p.nb_action, s0 = blockIdx.x * CACTO_TILE;
  if (L.tid < 256) {
    const int c = L.tid >> 4, f = L.tid & 15;
    st[L.tid] = (s0 + c < B && f < ns) ? S[(size_t)(s0 + c) * ns + f] : 0.f;
  }
  __syncthreads();
  if (L.wave == 0) fill_input_tile(p, st, X0, L);
  __syncthreads();
  actor_forward_tile(N, na, X0, nullptr, H, red, A, L, [](int, int, float4, float4) {});
  __syncthreads();
  if (L.tid < 16 * na) {
    const int c = L.tid / na, f = L.tid % na;
    if (s0 + c < B) Aout[(size_t)(s0 + c) * na + f] = A[c * na + f];
  }
}

// V = critic(s); optionally dV/ds (w.r.t. the raw state, through the normalisation).
__global__ void __launch_bounds__(CACTO_THREADS) k_critic_forward(const SysDevice* __restrict__ sdp, NetView N,
                                                                  const float* __restrict__ S, float* __restrict__ Vout,
                                                                  float* __restrict__ dVdS, int B) {
  __shared__ float4 X0[64];
  __shared__ float4 Z[24 * 64];
  __shared__ float4 H[2 * 8 * 64];
  __shared__ float4 G0[64];
  __shared__ float4 red[4 * 64];
  __shared__ float st[16 * 16];
  __shared__ float V[16];
  const cacto_sys_params& p = sdp->p;
  const Lane L;
  const int ns = p.nb_state, s0 = blockIdx.x * CACTO_TILE;
  if (L.tid < 256) {
    const int c = L.tid >> 4, f = L.tid & 15;
    st[L.tid] = (s0 + c < B && f < ns) ? S[(size_t)(s0 + c) * ns + f] : 0.f;
  }
  __syncthreads();
  if (L.wave == 0) fill_input_tile(p, st, X0, L);
  __syncthreads();
  critic_forward_tile(N, X0, dVdS ? Z : nullptr, nullptr, H, red, V, L, [](int, int, float4) {});  // Z: cos tiles
  __syncthreads();
  if (L.tid < 16 && s0 + L.tid < B && Vout) Vout[s0 + L.tid] = V[L.tid];
  if (!dVdS) return;
  critic_first_backward(N, Z, H, nullptr, G0, red, L, [](int, int, int, float4) {});
  __syncthreads();
  if (L.wave == 0) {
    const float4 g = G0[L.lane];
    const float gv[4] = {g.x, g.y, g.z, g.w};
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * L.g + r;
      if (f < ns && s0 + L.c < B) dVdS[(size_t)(s0 + L.c) * ns + f] = normalize_backward(p, f, gv[r]);
    }
  }
}

// ---------------------------------------------------------------- rollout (K18)
// Weight-stationary actor: each wave keeps its share of the actor's MFMA A-fragments in
// registers for the whole rollout (layer 2: out tiles wave, wave+4, wave+8, wave+12 x 16 k-tiles =
// 64 float4; layers 1/3 and biases 12 more), so a step issues only LDS reads and MFMAs.
constexpr int A2_REG_TILES = 3;  // layer-2 out tiles per wave held in registers; the 4th in LDS
struct ActorRegs {
  float4 a2[A2_REG_TILES][16];  // layer 2: out tiles ot = wave + 4i (i < 3), all 16 k-tiles
};
// Layers 1 and 3, the 4th layer-2 out tile of every wave, and all biases live in LDS.
struct ActorLds {
  float4 a1[16 * 64];  // layer-1 blocks (KT = 1)
  float4 a3[16 * 64];  // layer-3 blocks (one out tile, 16 k-tiles)
  float4 a2[4 * 16 * 64];  // layer-2 blocks of out tiles 12..15 (wave + 12), [wave][k][lane]
  float b1[256], b2[256], b3[16];
};

__device__ __forceinline__ void load_actor_regs(const NetView& N, int na, const Lane& L, ActorRegs& R, ActorLds& S) {
  const float4* A1 = N.fwd(0);
  const float4* A2 = N.fwd(1);
  const float4* A3 = N.fwd(2);
#pragma unroll
  for (int i = 0; i < A2_REG_TILES; ++i) {
    const int ot = L.wave + 4 * i;
#pragma unroll
    for (int k = 0; k < 16; ++k) R.a2[i][k] = A2[(ot * 16 + k) * 64 + L.lane];
  }
  for (int k = 0; k < 16; ++k) S.a2[(L.wave * 16 + k) * 64 + L.lane] = A2[((L.wave + 12) * 16 + k) * 64 + L.lane];
  for (int k = L.tid; k < 16 * 64; k += CACTO_THREADS) {
    S.a1[k] = A1[k];
    S.a3[k] = A3[k];
  }
  for (int f = L.tid; f < 256; f += CACTO_THREADS) {
    S.b1[f] = N.bias(0, f);
    S.b2[f] = N.bias(1, f);
  }
  if (L.tid < 16) S.b3[L.tid] = L.tid < na ? N.bias(2, L.tid) : 0.f;
}

__device__ __forceinline__ float4 lrelu_bias(const floatx4& acc, const float* bias, int f) {
  float z[4] = {fadd(acc[0], bias[f]), fadd(acc[1], bias[f + 1]), fadd(acc[2], bias[f + 2]), fadd(acc[3], bias[f + 3])};
#pragma unroll
  for (int r = 0; r < 4; ++r) z[r] = z[r] > 0.f ? z[r] : fmul(z[r], 0.3f);
  return make_float4(z[0], z[1], z[2], z[3]);
}

// Actor forward of one tile with register-resident layer-2 weights. X0 -> H1 -> H2 -> A.
__device__ __forceinline__ void actor_forward_regs(const ActorRegs& R, const ActorLds& W, int na, const float4* X0,
                                                   float4* H1, float4* H2, float4* red, float* A, const Lane& L) {
  // MFMA order: within a k-block, the 4 k-steps (j) outer and the 4 out tiles (i) inner, so
  // consecutive MFMAs hit different accumulators (issue-bound); each accumulator still sums its
  // k-steps in order.
  const float4 x = X0[L.lane];
  {
    float4 a1[4];
    floatx4 acc1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a1[i] = W.a1[(L.wave + 4 * i) * 64 + L.lane];
      acc1[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) acc1[i] = mfma4(a1[i].x, x.x, acc1[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc1[i] = mfma4(a1[i].y, x.y, acc1[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc1[i] = mfma4(a1[i].z, x.z, acc1[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc1[i] = mfma4(a1[i].w, x.w, acc1[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ot = L.wave + 4 * i;
      H1[ot * 64 + L.lane] = lrelu_bias(acc1[i], W.b1, 16 * ot + 4 * L.g);
    }
  }
  __syncthreads();
  floatx4 acc2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc2[i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const float4 b = H1[k * 64 + L.lane];
    const float4 a3 = W.a2[(L.wave * 16 + k) * 64 + L.lane];
#pragma unroll
    for (int i = 0; i < A2_REG_TILES; ++i) acc2[i] = mfma4(R.a2[i][k].x, b.x, acc2[i]);
    acc2[3] = mfma4(a3.x, b.x, acc2[3]);
#pragma unroll
    for (int i = 0; i < A2_REG_TILES; ++i) acc2[i] = mfma4(R.a2[i][k].y, b.y, acc2[i]);
    acc2[3] = mfma4(a3.y, b.y, acc2[3]);
#pragma unroll
    for (int i = 0; i < A2_REG_TILES; ++i) acc2[i] = mfma4(R.a2[i][k].z, b.z, acc2[i]);
    acc2[3] = mfma4(a3.z, b.z, acc2[3]);
#pragma unroll
    for (int i = 0; i < A2_REG_TILES; ++i) acc2[i] = mfma4(R.a2[i][k].w, b.w, acc2[i]);
    acc2[3] = mfma4(a3.w, b.w, acc2[3]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ot = L.wave + 4 * i;
    H2[ot * 64 + L.lane] = lrelu_bias(acc2[i], W.b2, 16 * ot + 4 * L.g);
  }
  __syncthreads();
  floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kt = L.wave + 4 * i;
    const float4 a = W.a3[kt * 64 + L.lane], b = H2[kt * 64 + L.lane];
    c0 = mfma4(a.x, b.x, c0);
    c1 = mfma4(a.y, b.y, c1);
    c2 = mfma4(a.z, b.z, c2);
    c3 = mfma4(a.w, b.w, c3);
  }
  const floatx4 acc3 = (c0 + c1) + (c2 + c3);
  red[L.wave * 64 + L.lane] = make_float4(acc3[0], acc3[1], acc3[2], acc3[3]);
  __syncthreads();
  if (L.wave == 0) {
    float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < CACTO_NWAVES; ++w) {
      const float4 p = red[w * 64 + L.lane];
      sum[0] += p.x;
      sum[1] += p.y;
      sum[2] += p.z;
      sum[3] += p.w;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * L.g + r;
      if (f < na) A[L.c * na + f] = fadd(sum[r], W.b3[f]);
    }
  }
}

// One workgroup = 16 episodes (lane c of a wave <-> episode c of the tile). Per step:
//   actor tile (4 waves, MFMA, weights stationary)                         -> A (LDS)
//   E1: wave 0 integrates the dynamics s -> s'; waves 1-3 evaluate the reward terms of (s, a)
//       (ellipses / peak / control cost) from EE(s) kept in LDS
//   E2: wave 0 combines the reward in the reference's order and writes S/A/R; wave 1 computes
//       EE(s'); wave 2 normalises s' into the next actor input tile.
template <int NJ>
__global__ void __launch_bounds__(CACTO_THREADS, 1)
    k_rollout(const SysDevice* __restrict__ sdp, NetView N, const double* __restrict__ S0,
              const int32_t* __restrict__ nsteps, int T, int use_actor, const double* __restrict__ Wext,
              double* __restrict__ Straj, float* __restrict__ Atraj, double* __restrict__ Rtraj,
              double* __restrict__ EEtraj, int32_t* __restrict__ status, const int32_t* __restrict__ order, int B) {
  constexpr int ns = Dims<NJ>::NS, na = Dims<NJ>::NA;
  __shared__ float4 X0[64];
  __shared__ float4 H1[16 * 64], H2[16 * 64];
  __shared__ float4 red[4 * 64];
  __shared__ float st[16 * 16];
  __shared__ float A[16 * na];
  __shared__ double sS[2 * 16 * ns], sEE[2 * 16 * 3], terms[16 * 6], uterm[16 * 8];
  __shared__ double cpv[NJ == -2 ? 16 * 30 : 1];  // car_park obstacle pair costs
  __shared__ double MS[NJ > 0 ? 16 * NJ * NJ : 1], hS[NJ > 0 ? 16 * NJ : 1];  // chain M(q), nle(q, v)
  __shared__ int sb[16], sn_[16], salive[16];
  __shared__ int tmax;
  __shared__ ActorLds WL;
  const SysDevice& sd = *sdp;
  const cacto_sys_params& p = sd.p;
  const Lane L;
  const int s0 = blockIdx.x * CACTO_TILE;
  const int c = L.c;                      // episode slot handled by this lane (lanes 0..15)
  const bool ep_lane = L.lane < 16 && s0 + c < B;
  double w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = k >= p.n_weights ? 0.0 : Wext ? Wext[k] : p.w_running[k];
  const bool want_R = Rtraj != nullptr, want_EE = EEtraj != nullptr || want_R;
  // planar / manipulator rewards are split over waves 1-3 (terms of EE(s)); others whole on wave 1
  const bool split_R = p.reward_kind == CACTO_REW_PLANAR || p.reward_kind == CACTO_REW_MANIPULATOR;
  // chains with configuration-dependent M: RNEA (wave 0) and CRBA (wave 3) run concurrently
  const bool split_dyn = NJ > 0 && !p.const_dyn;
  ActorRegs R;
  if (use_actor) load_actor_regs(N, na, L, R, WL);
  if (L.tid == 0) tmax = 0;
  __syncthreads();
  ConstDyn<NJ> cd;
  if (L.wave == 0 && L.lane < 16) {
    const bool valid = s0 + c < B;
    const int b = valid ? (order ? order[s0 + c] : s0 + c) : 0;
    const int n = valid ? min(nsteps[b], T) : 0;
    sb[c] = b;
    sn_[c] = n;
    salive[c] = n > 0;
    atomicMax(&tmax, n);
    double s[ns];
#pragma unroll
    for (int i = 0; i < ns; ++i) {
      s[i] = valid ? S0[(size_t)b * ns + i] : 0.0;
      sS[c * ns + i] = s[i];
      st[c * 16 + i] = (float)s[i];
      if (valid && Straj) Straj[(size_t)b * (T + 1) * ns + i] = s[i];
    }
    for (int i = ns; i < 16; ++i) st[c * 16 + i] = 0.f;
    if (NJ > 0 && p.const_dyn && valid) const_dyn_init<NJ>(sd, s, cd);
    if (want_EE) {
      const V3 e = env_ee<NJ>(sd, s);
      sEE[c * 3 + 0] = e.x;
      sEE[c * 3 + 1] = e.y;
      sEE[c * 3 + 2] = e.z;
      if (valid && EEtraj) {
        EEtraj[(size_t)b * (T + 1) * 3 + 0] = e.x;
        EEtraj[(size_t)b * (T + 1) * 3 + 1] = e.y;
        EEtraj[(size_t)b * (T + 1) * 3 + 2] = e.z;
      }
    }
  }
  __syncthreads();
  if (use_actor && L.wave == 0) fill_input_tile(p, st, X0, L);
  __syncthreads();
  const int steps = tmax;
  for (int t = 0; t < steps; ++t) {
    RSTAMP(0);
    if (use_actor) {
      actor_forward_regs(R, WL, na, X0, H1, H2, red, A, L);
      __syncthreads();
    }
    RSTAMP(1);
    // state and EE are double-buffered: step t reads buffer t&1 and writes the other one
    const int cur = t & 1;
    const double* Sc = sS + cur * 16 * ns;
    double* Sn = sS + (cur ^ 1) * 16 * ns;
    const double* Ec = sEE + cur * 48;
    double* En = sEE + (cur ^ 1) * 48;
    const bool act_c = s0 + c < B && salive[c] && t < sn_[c];  // episode c = lane & 15 of any lane group
    const bool active = act_c && L.lane < 16;
    double sn[ns];
    // ---- E1: wave 0 integrates s_t -> s_{t+1}; waves 1-3 evaluate the reward terms of (s_t, a_t)
    if (L.wave == 0) {
      if (active) {
        double s[ns], a[na];
#pragma unroll
        for (int i = 0; i < ns; ++i) s[i] = Sc[c * ns + i];
#pragma unroll
        for (int i = 0; i < na; ++i) a[i] = use_actor ? (double)A[c * na + i] : 0.0;
        if (split_dyn) {
          // chains: nle(q, v) here by RNEA, M(q) on wave 3 by CRBA, Cholesky step after the barrier
          if constexpr (NJ > 0) {
            double h[NJ];
            chain_nle<NJ>(sd, s, s + NJ, h);
#pragma unroll
            for (int i = 0; i < NJ; ++i) hS[c * NJ + i] = h[i];
          }
        } else {
          if (NJ > 0 && p.const_dyn)
            env_simulate_const<NJ>(sd, cd, s, a, sn);
          else
            env_simulate<NJ>(sd, s, a, false, sn);
#pragma unroll
          for (int i = 0; i < ns; ++i) {
            Sn[c * ns + i] = sn[i];
            st[c * 16 + i] = (float)sn[i];
          }
        }
      }
    } else if (split_dyn && L.wave == 3 && active) {
      if constexpr (NJ > 0) {
        double M[NJ * NJ];
        chain_mass<NJ>(sd, Sc + c * ns, M);
#pragma unroll
        for (int k = 0; k < NJ * NJ; ++k) MS[c * NJ * NJ + k] = M[k];
      }
    }
    if (L.wave != 0 && want_R && act_c) {
      const int grp = L.lane >> 4;
      const double x = Ec[c * 3 + 0], y = Ec[c * 3 + 1];
      const double* o = p.obs;
      if (split_R) {
        // the three ellipses share one code path: one lane group each (environment.py:337-339)
        if (L.wave == 1) {
          if (grp < 3) terms[c * 6 + grp] = ell_cost(p, x, y, o[2 * grp], o[2 * grp + 1], o[6 + 2 * grp], o[7 + 2 * grp]);
        } else if (L.wave == 2) {
          if (grp == 0) terms[c * 6 + 3] = peak_cost(p, x, y);
        } else {
          // wave 3: one control-bound term per lane group (summed in action order in E2), velocity cost
          for (int i = grp; i < na; i += 4) uterm[c * 8 + i] = bound_term(p, use_actor ? (double)A[c * na + i] : 0.0, i);
          if (grp == 0) {
            double vel = 0.0;
            if (NJ > 0 && p.reward_kind == CACTO_REW_MANIPULATOR && w[2] != 0.0) {
#pragma unroll
              for (int k = 0; k < (NJ > 0 ? NJ : 1); ++k) vel += Sc[c * ns + NJ + k] * Sc[c * ns + NJ + k];
            }
            terms[c * 6 + 5] = vel;
          }
        }
      } else if constexpr (NJ == -2) {
        // CarPark obstacle cost (environment.py:619-624): 3 x n_check smooth-box terms of EE(s),
        // theta, over 12 lane groups (waves 1-3 x 4 groups of the 16 episode lanes)
        const int g12 = (L.wave - 1) * 4 + grp;
        const double th = Sc[c * ns + 2], ct = cos(th), stt = sin(th);
        for (int pr = g12; pr < 3 * p.n_check; pr += 12) cpv[c * 30 + pr] = carpark_pair_cost(p, x, y, ct, stt, pr);
      } else if (L.wave == 1 && grp == 0) {
        // UR5: the whole Env.step reward of (s, a) (environment.py:780-805)
        double s[ns], a[na];
#pragma unroll
        for (int i = 0; i < ns; ++i) s[i] = Sc[c * ns + i];
#pragma unroll
        for (int i = 0; i < na; ++i) a[i] = use_actor ? (double)A[c * na + i] : 0.0;
        terms[c * 6 + 0] = env_reward<NJ>(sd, w, s, a, false);
      }
    }
    __syncthreads();
    if (split_dyn) {
      if constexpr (NJ > 0) {
        if (L.wave == 0 && active) {
          double s[ns], a[na], M[NJ * NJ], h[NJ];
#pragma unroll
          for (int i = 0; i < ns; ++i) s[i] = Sc[c * ns + i];
#pragma unroll
          for (int i = 0; i < na; ++i) a[i] = use_actor ? (double)A[c * na + i] : 0.0;
#pragma unroll
          for (int k = 0; k < NJ * NJ; ++k) M[k] = MS[c * NJ * NJ + k];
#pragma unroll
          for (int i = 0; i < NJ; ++i) h[i] = hS[c * NJ + i];
          chain_step<NJ>(sd, s, a, M, h, sn);
#pragma unroll
          for (int i = 0; i < ns; ++i) {
            Sn[c * ns + i] = sn[i];
            st[c * 16 + i] = (float)sn[i];
          }
        }
      }
      __syncthreads();
    }
    RSTAMP(2);
    // ---- E2: wave 0 combines the reward (reference order) and writes S/A/R; wave 1 computes
    //          EE(s_{t+1}); wave 2 normalises s_{t+1} into the next actor input tile.
    if (L.wave == 0) {
      if (active) {
        const int b = sb[c];
        if (want_R) {
          double r;
          if constexpr (NJ == -2) {
            double a[na], s[ns];
#pragma unroll
            for (int i = 0; i < na; ++i) a[i] = use_actor ? (double)A[c * na + i] : 0.0;
#pragma unroll
            for (int i = 0; i < ns; ++i) s[i] = Sc[c * ns + i];
            r = carpark_reward(p, w, Ec[c * 3 + 0], Ec[c * 3 + 1], s, a, carpark_sum(p, cpv + c * 30));
          } else {
            const bool has_vel = NJ > 0 && p.reward_kind == CACTO_REW_MANIPULATOR;
            double u_cost = 0.0;
            if (split_R)
#pragma unroll
              for (int i = 0; i < na; ++i) u_cost += uterm[c * 8 + i];
            r = split_R ? combine_reward(p, w, Ec[c * 3 + 0], Ec[c * 3 + 1], terms[c * 6 + 3], terms[c * 6 + 5],
                                         has_vel, terms[c * 6 + 0], terms[c * 6 + 1], terms[c * 6 + 2], u_cost)
                        : terms[c * 6 + 0];
          }
          Rtraj[(size_t)b * T + t] = r;
        }
        if (Atraj)
#pragma unroll
          for (int i = 0; i < na; ++i) Atraj[((size_t)b * T + t) * na + i] = use_actor ? A[c * na + i] : 0.f;
        bool bad = false;
#pragma unroll
        for (int i = 0; i < ns; ++i) {
          bad |= isnan(sn[i]);
          if (Straj) Straj[((size_t)b * (T + 1) + t + 1) * ns + i] = sn[i];
        }
        if (bad) salive[c] = 0;  // RL.py:229-231
      }
    } else if (L.wave == 1) {
      if (active && want_EE) {
        double s[ns];
#pragma unroll
        for (int i = 0; i < ns; ++i) s[i] = Sn[c * ns + i];
        const V3 e = env_ee<NJ>(sd, s);
        En[c * 3 + 0] = e.x;
        En[c * 3 + 1] = e.y;
        En[c * 3 + 2] = e.z;
        if (EEtraj) {
          const int b = sb[c];
          EEtraj[((size_t)b * (T + 1) + t + 1) * 3 + 0] = e.x;
          EEtraj[((size_t)b * (T + 1) + t + 1) * 3 + 1] = e.y;
          EEtraj[((size_t)b * (T + 1) + t + 1) * 3 + 2] = e.z;
        }
      }
    } else if (L.wave == 2 && use_actor) {
      fill_input_tile(p, st, X0, L);
    }
    __syncthreads();
    RSTAMP(3);
  }
  if (L.wave == 0 && ep_lane && status) {
    const int b = sb[c];
    status[b] = (salive[c] || sn_[c] == 0) ? 0 : 1;
  }
}

}  // namespace cacto

using namespace cacto;

namespace {
template <int NJ>
struct LaunchRollout {
  static int run(const cacto_sys* sys, NetView v, const double* S0, const int32_t* n, int T, int use_actor,
                 const double* W, double* S, float* A, double* R, double* EE, int32_t* status, const int32_t* order,
                 int B, hipStream_t st) {
    hipLaunchKernelGGL(k_rollout<NJ>, dim3(ceil_div(B, CACTO_TILE)), dim3(CACTO_THREADS), 0, st, sys->dev, v, S0, n, T,
                       use_actor, W, S, A, R, EE, status, order, B);
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
};
}  // namespace

#ifdef CACTO_STAMPS
extern "C" int cacto_debug_rollout_stamps(unsigned long long* out_h) {
  CACTO_CHECK_HIP(hipDeviceSynchronize());
  CACTO_CHECK_HIP(hipMemcpyFromSymbol(out_h, HIP_SYMBOL(g_rstamps), sizeof(unsigned long long) * 8));
  return CACTO_OK;
}
#endif

NetView cacto_make_view(const cacto_sys* sys, int net, const float* netbuf) {
  NetView v;
  const NetTopo& t = topo(sys, net);
  v.flat = netbuf;
  v.pk = reinterpret_cast<const float4*>(netbuf ? netbuf + flat_span(t) : nullptr);
  v.t = t;
  return v;
}

extern "C" int64_t cacto_mlp_param_count(const cacto_sys* sys, int net) {
  if (!sys || (net != CACTO_NET_ACTOR && net != CACTO_NET_CRITIC)) return -1;
  return topo(sys, net).params;
}

extern "C" int64_t cacto_mlp_netbuf_floats(const cacto_sys* sys, int net) {
  if (!sys || (net != CACTO_NET_ACTOR && net != CACTO_NET_CRITIC)) return -1;
  const NetTopo& t = topo(sys, net);
  return flat_span(t) + (int64_t)2 * t.blocks * 256;
}

extern "C" int cacto_mlp_pack(const cacto_sys* sys, int net, float* netbuf_d, void* stream) {
  CACTO_REQUIRE(sys && netbuf_d && (net == CACTO_NET_ACTOR || net == CACTO_NET_CRITIC), "cacto_mlp_pack: bad arguments");
  const NetTopo& t = topo(sys, net);
  const int64_t total = (int64_t)2 * t.blocks * 256;
  hipLaunchKernelGGL(k_pack, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 2048)), dim3(256), 0,
                     as_stream(stream), netbuf_d, netbuf_d + flat_span(t), t);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

extern "C" int cacto_actor_forward(const cacto_sys* sys, const float* actor_netbuf_d, const float* S_d, float* A_d,
                                   int B, void* stream) {
  CACTO_REQUIRE(sys && actor_netbuf_d && S_d && A_d && B >= 0, "cacto_actor_forward: bad arguments");
  if (B == 0) return CACTO_OK;
  NetView v = cacto_make_view(sys, CACTO_NET_ACTOR, actor_netbuf_d);
  hipLaunchKernelGGL(k_actor_forward, dim3(ceil_div(B, CACTO_TILE)), dim3(CACTO_THREADS), 0, as_stream(stream),
                     sys->dev, v, S_d, A_d, B);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

extern "C" int cacto_critic_forward(const cacto_sys* sys, const float* critic_netbuf_d, const float* S_d, float* V_d,
                                    int B, void* stream) {
  return cacto_critic_input_grad(sys, critic_netbuf_d, S_d, V_d, nullptr, B, stream);
}

extern "C" int cacto_critic_input_grad(const cacto_sys* sys, const float* critic_netbuf_d, const float* S_d,
                                       float* V_d, float* dVdS_d, int B, void* stream) {
  CACTO_REQUIRE(sys && critic_netbuf_d && S_d && B >= 0, "cacto_critic_input_grad: bad arguments");
  if (B == 0) return CACTO_OK;
  NetView v = cacto_make_view(sys, CACTO_NET_CRITIC, critic_netbuf_d);
  hipLaunchKernelGGL(k_critic_forward, dim3(ceil_div(B, CACTO_TILE)), dim3(CACTO_THREADS), 0, as_stream(stream),
                     sys->dev, v, S_d, V_d, dVdS_d, B);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

extern "C" int cacto_rollout(const cacto_sys* sys, const float* actor_netbuf_d, const double* S0_d,
                             const int32_t* nsteps_d, int T, int use_actor, const double* W_d, double* S_traj_d,
                             float* A_traj_d, double* R_traj_d, double* EE_traj_d, int32_t* status_d,
                             const int32_t* order_d, int B, void* stream) {
  CACTO_REQUIRE(sys && S0_d && nsteps_d && T >= 0 && B >= 0, "cacto_rollout: bad arguments");
  CACTO_REQUIRE(!use_actor || actor_netbuf_d, "cacto_rollout: use_actor needs the actor net buffer");
  if (B == 0) return CACTO_OK;
  NetView v = cacto_make_view(sys, CACTO_NET_ACTOR, actor_netbuf_d);
  return dispatch_nj<LaunchRollout>(sys->host.p, sys, v, S0_d, nsteps_d, T, use_actor, W_d, S_traj_d, A_traj_d,
                                    R_traj_d, EE_traj_d, status_d, order_d, B, as_stream(stream));
}
