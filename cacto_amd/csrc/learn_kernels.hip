// Learner kernels: the per-sample chains of NN.compute_critic_grad (Sobolev, double backprop)
// and NN.compute_actor_grad (dynamics Jacobian path), the weight-gradient GEMM (K = samples,
// split-K partial slabs), and the fused slab-reduce + Keras Adam + packed refresh (+ soft update).
//
// Data flow per update (workspace, float32):
//   chain kernel (16 samples / workgroup) -> per-layer operand panels LT_l [in_pad][ld], RT_l
//   [out_pad][ld] (feature-major, sample rows contiguous) such that
//        dW_l = sum_rows LT_l[:, r] (x) RT_l[:, r],  db_l = sum_{rows >= bias_r0} RT_l[:, r]
//   critic rows: [0, Bp) = (Gbar_l, D_l) (Sobolev term), [Bp, 2Bp) = (h_l, zbar_l) (plain backprop)
//   actor rows : [0, Bp) = (h_l, zbar_l)
//   -> k_wgrad: one wave per (layer, 16x16 output tile | bias tile, row chunk) -> slab[chunk][P]
//   -> k_adam : sum chunks in fixed order (deterministic), Adam, packed copies, soft update.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <cstdlib>
#include <vector>

#include "net_common.h"
#include "per_device.h"

#ifdef CACTO_STAMPS
__device__ unsigned long long g_cstamps[32];
__device__ unsigned long long g_astamps[32];  // actor chain, tile 0 (also inside the paired kernel)
#define CSTAMP(k) PSTAMP(k)
#define CSTAMP_DECL
#define CSTAMP_FLUSH                                                                     \
  do {                                                                                   \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                             \
      for (int k_ = 0; k_ < 32; ++k_) g_cstamps[k_] = cacto_stamp_s[k_];                 \
  } while (0)
#else
#define CSTAMP(k) \
  do {            \
  } while (0)
#define CSTAMP_DECL
#define CSTAMP_FLUSH \
  do {               \
  } while (0)
#endif

namespace cacto {

struct GradBufs {
  float* LT[MAX_LAYERS];
  float* RT[MAX_LAYERS];
  int ld;  // row stride of the panels
  int Bp;  // batch rounded up to 16
};

struct ChainScalars {
  float w_S;
  int MC;
  int B_global;
  int want_vt;
  // the two-stream pipeline's device-side ordering (DESIGN §3 "memory-ordering contract"): the actor
  // chain waits, before its critic pass at s', until *wait_p >= wait_v (the critic's Adam of the same
  // update has run) — a relaxed poll, no fence: the Adam wrote the critic through to memory at agent
  // scope and published after its stores completed, and no L2 holds a line of the buffer from before
  // (kernel starts invalidate; nothing reads it in between)
  const unsigned long long* wait_p;
  unsigned long long wait_v;
  // 1 (the PER loops): that wait at the chain's start, before it gathers the sampled rows (the
  // sample of the update precedes the critic's Adam on the other stream)
  int wait_at_start;
  // 1: the 16-sample tiles dealt so that the tiles of one 256-row GEMM chunk run on the XCD that
  // k_wgrad_big runs that chunk on (chain_tile_of)
  int xcd_tiles;
};

// Block b -> tile of a 16-sample chain grid. xcd_tiles (ntiles % 128 == 0): block b runs on XCD
// b % 8 (the dispatcher's round robin), which k_wgrad_big gives the 256-row chunks x, x + 8, ... —
// 16 tiles each — so XCD x takes the tiles of exactly those chunks and their panel rows are written
// into the L2 the GEMM reads them from. Which block runs a tile changes no value.
__device__ __forceinline__ int chain_tile_of(int b, int ntiles, int xcd_tiles) {
  if (!xcd_tiles) return b;
  const int x = b & 7, j = b >> 3;
  return ((j >> 4) * 8 + x) * 16 + (j & 15);
}

// The device-side waits of the pipeline: until *wait_p >= wait_v (normally already true: one load).
// Bounded: after ~2^22 polls (seconds) the wait gives up and latches the timeout word, so an
// ordering bug cannot hang the GPU; the host then fails the call (cacto_pipeline_check). The signal
// words live in cacto_sys::pipe_sig: [0] actor chains finished, [1] timeout latch, [2] critic Adam
// steps finished, [3] k_adam's last-workgroup counter, [4..7] the concurrency probe's words. Relaxed
// polls: the write-after-read order (the critic's Adam may overwrite what an actor chain read once
// that chain has finished) carries no data; for the read-after-write order (the actor chain reads
// what the critic's Adam wrote) the Adam's stores went through to memory before it published (see
// ChainScalars and DESIGN §3's memory-ordering contract).
// ("Memory-ordering contract", sites 2 and 3)
__device__ __forceinline__ void pipe_wait(const unsigned long long* wait_p, unsigned long long wait_v,
                                          unsigned long long* latch) {
  if (!wait_p) return;
  for (int k = 0; k < (1 << 22); ++k) {
    if (__hip_atomic_load(wait_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= wait_v) return;
    __builtin_amdgcn_s_sleep(2);
  }
  __hip_atomic_store(latch, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One-time probe per handle (cacto_update_n[_per]'s first two-stream call): can a kernel on the side
// stream and one on the caller's stream run at the same time? Role 0 (side) raises flag w[4] and
// polls for w[5]; role 1 (caller's stream) polls for w[4], then raises w[5]. Each records in w[6 +
// role] whether its poll succeeded (bounded: ~2^14 polls). When the device serializes kernels
// (AMD_SERIALIZE_KERNEL, HIP_LAUNCH_BLOCKING, counter collection) the first of the two to run cannot
// see the other's flag, so a device-side wait would spin until its bound: the pipeline then orders
// the streams with queue markers.
// ("Memory-ordering contract", site 4)
__global__ void k_pipe_probe(unsigned long long* w, int role) {
  if (threadIdx.x != 0) return;
  unsigned long long* mine = w + 4 + role;
  const unsigned long long* other = w + 5 - role;
  if (role == 0) __hip_atomic_store(mine, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long ok = 0;
  for (int k = 0; k < (1 << 14) && !ok; ++k) {
    ok = __hip_atomic_load(other, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!ok) __builtin_amdgcn_s_sleep(2);
  }
  if (role == 1) __hip_atomic_store(mine, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(w + 6 + role, ok ? 1ull : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void store_panel(float* base, int ld, int row, int t, int g, float4 v) {
  float* p = base + (size_t)(16 * t + 4 * g) * ld + row;
  p[0] = v.x;
  p[ld] = v.y;
  p[2 * (size_t)ld] = v.z;
  p[3 * (size_t)ld] = v.w;
}

// custom_logarithm (NeuralNetwork.py:140-148) and its TF gradient (tf.where / tf.maximum / Log).
__device__ __forceinline__ float clog(float x) {
  const float eps = 1e-7f;
  return x > 0.f ? logf(fadd(fmaxf(x, eps), 1.f)) : -logf(fadd(fmaxf(-x, eps), 1.f));
}
__device__ __forceinline__ float clog_backward(float x, float g) {
  const float eps = 1e-7f;
  const float ax = x > 0.f ? x : -x;
  if (!(ax >= eps)) return 0.f;  // Maximum grad goes to the constant when |x| < eps
  return fmul(g, fdiv(1.f, fadd(ax, 1.f)));
}

// ---------------------------------------------------------------- critic chain (a11)
// 92.7 KB: with the actor chain's 65 KB one critic and one actor workgroup share a CU (the
// pipelined large-batch update runs critic(t+1) and actor(t) side by side)
struct CriticLds {
  float4 X0[64], XT[64], G0[64];
  float4 Cs[24 * 64];  // cos z_l
  float4 Hs[24 * 64];  // h_l = sin z_l; zbar_l from the Sobolev backward on (the same slot: read, then written)
  float4 G[16 * 64];
  float4 GB[16 * 64];
  float4 red[4 * 64];
  float st[256], stn[256], dvdx[256];
  float Rs[16], ds[16], ws[16], Vn[16], V[16], y[16], Vb[16], Vt2[16];
};

// one 16-sample tile of the critic chain (workgroup-wide; S in LDS)
__device__ __forceinline__ void critic_chain(CriticLds& S, const int tile, const SysDevice* __restrict__ sdp,
                                             const NetView& C, const NetView& Tg, const ChainScalars& cs,
                                             const double* __restrict__ storage, const int32_t* __restrict__ idx,
                                             const float* __restrict__ isw, int B, const GradBufs& gb,
                                             float* __restrict__ y_out, float* __restrict__ V_out,
                                             float* __restrict__ Vt_out, int32_t* __restrict__ step) {
  float4 *X0 = S.X0, *XT = S.XT, *G0 = S.G0, *Cs = S.Cs, *Hs = S.Hs, *G = S.G, *ZB = S.Hs, *GB = S.GB, *red = S.red;
  float *st = S.st, *stn = S.stn, *dvdx = S.dvdx, *Rs = S.Rs, *ds = S.ds, *ws = S.ws, *Vn = S.Vn, *V = S.V, *y = S.y,
        *Vb = S.Vb, *Vt2 = S.Vt2;
  CSTAMP_DECL;
  CSTAMP(0);
  const cacto_sys_params& p = sdp->p;
  const Lane L;
  const int ns = p.nb_state, cols = 3 * ns + 3, s0 = tile * CACTO_TILE;
  const int ld = gb.ld, Bp = gb.Bp;
  const bool sob = cs.w_S != 0.f;
  const int zoff[4] = {0, 4, 8, 16};
  const int goff[4] = {0, 0, 4, 8};
  if (tile == 0 && L.tid == 0 && step) step[0] += 1;  // Keras critic optimizer iterations

  // the target network's fragments for the first pass (loaded during the row gathers, below)
  CriticFwdFrags TF;
  float4 w5[2];  // W5[:, 0] at this lane's rows of layer-3 out tiles wave, wave + 4
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float* w = C.flat + C.t.woff[4] + 16 * (L.wave + 4 * t) + 4 * L.g;
    w5[t] = make_float4(w[0], w[1], w[2], w[3]);
  }
  const Norm4 nrm(p, L);  // state_norm of this lane's features, loaded with the rows
  {  // one (sample, feature) per thread: the row gathers overlap
    // branch-free gathers (clamped sample and feature indices, then zeroed): no load sits under
    // a branch, so the waits stay exact
    const int c = L.tid >> 4, f = L.tid & 15;
    const bool valid = s0 + c < B, in = valid && f < ns;
    const int sc = min(s0 + c, B - 1), fc = min(f, ns - 1);
    const int32_t row = idx[sc];
    // issued between the index load and the dependent row loads: the wait for the index (in-order
    // vmcnt) does not cover them, and they have both latencies to land
    TF.load<true>(Tg, L);
    TF.load_last(Tg, L);
    const double* rp = storage + (size_t)row * cols;
    const double x = rp[fc], xn = rp[ns + 1 + fc], xd = rp[2 * ns + 1 + fc];
    const double r = rp[ns], d = rp[3 * ns + 1];
    const float wv = isw ? isw[sc] : 1.f;
    st[c * 16 + f] = in ? (float)x : 0.f;
    stn[c * 16 + f] = in ? (float)xn : 0.f;
    dvdx[c * 16 + f] = in ? (float)xd : 0.f;
    if (f == 0) {
      Rs[c] = valid ? (float)r : 0.f;
      ds[c] = valid ? (float)d : 0.f;
      ws[c] = valid ? wv : 0.f;
    }
  }
  __syncthreads();
  if (L.wave == 0) {
    nrm.fill(st, X0, L);
    nrm.fill(stn, XT, L);
  }
  __syncthreads();
  CSTAMP(1);

  // y = R + (1 - d) * V_tgt(s_next)   (NeuralNetwork.py:153-158)
  if (!cs.MC) critic_forward_tile_f(TF, Tg, XT, nullptr, nullptr, Hs, red, Vn, L, [](int, int, float4) {});
  __syncthreads();
  CSTAMP(2);
  if (L.tid < 16) y[L.tid] = cs.MC ? Rs[L.tid] : fadd(Rs[L.tid], fmul(fsub(1.f, ds[L.tid]), Vn[L.tid]));
  if (cs.want_vt) {  // the extra V_tgt(s) of NeuralNetwork.py:178
    critic_forward_tile_f(TF, Tg, X0, nullptr, nullptr, Hs, red, Vt2, L, [](int, int, float4) {});
    __syncthreads();
  }

  // forward at s, keeping sin z and cos z; h_l -> LT_l second half
  if (L.wave == 0) store_panel(gb.LT[0], ld, Bp + s0 + L.c, 0, L.g, X0[L.lane]);
  critic_forward_tile(C, X0, Cs, Hs, Hs, red, V, L, [&](int l, int ot, float4 h4) {
    store_panel(gb.LT[l + 1], ld, Bp + s0 + L.c, ot, L.g, h4);
  });
  __syncthreads();
  CSTAMP(3);

  CriticFwdFrags SF;
  if (sob) {
    // first backward: D_l -> RT_l first half; G_l kept in LDS; G_0 = dV/dx0
    critic_first_backward(C, Cs, GB, G, G0, red, L, [&](int l, int ot, int lane, float4 d4) {
      store_panel(gb.RT[l], ld, s0 + (lane & 15), ot, lane >> 4, d4);
    });
    __syncthreads();
    CSTAMP(4);
    SF.load<false>(C, L);
    // Sobolev loss gradient w.r.t. dV/ds, then w.r.t. G_0 (NeuralNetwork.py:167-170): one
    // (sample c, feature f) element per thread (the same ops as per lane and feature)
    {
      const int c = L.tid >> 4, f = L.tid & 15;
      float gb0 = 0.f;
      if (f < ns - 1) {
        const float nf = (float)p.state_norm[f];
        auto nback = [&](float g) { return !p.normalize ? g : fdiv(g, nf); };  // f < ns - 1: not the time column
        const float gsq = fdiv(fmul(fdiv(1.f, (float)cs.B_global), ws[c]), (float)(ns - 1));
        const float dvds = nback(reinterpret_cast<const float*>(G0)[((f >> 2) * 16 + c) * 4 + (f & 3)]);
        const float yp = clog(dvds), yt = clog(dvdx[c * 16 + f]);
        const float gyp = fmul(fmul(2.f, gsq), fsub(yp, yt));
        gb0 = nback(clog_backward(dvds, gyp));
      }
      reinterpret_cast<float*>(GB)[((f >> 2) * 16 + c) * 4 + (f & 3)] = gb0;
      gb.LT[0][(size_t)f * ld + s0 + c] = gb0;  // the panel row of feature f (store_panel's layout)
    }
    __syncthreads();
    CSTAMP(5);
    // backward of the first backward, l = 0..3 (see oracle/nn.py compute_critic_grad), on the
    // forward fragments (no bias, loaded before the Sobolev loss above)
    // ZB aliases Hs: each lane reads sin z_l of its element, then writes zbar_l over it (no other
    // reader of that element is left: later passes read other layers' slots)
    auto sp_epi = [&](int l, float4* nxt) {
      return [&, l, nxt](int ot, floatx4 acc) {
        const float4 sz = Hs[(zoff[l] + ot) * 64 + L.lane], cz = Cs[(zoff[l] + ot) * 64 + L.lane];
        const float4 gu = l < 3 ? G[(goff[l + 1] + ot) * 64 + L.lane] : (ot >= 4 ? w5[1] : w5[0]);
        const float sv[4] = {sz.x, sz.y, sz.z, sz.w}, cv[4] = {cz.x, cz.y, cz.z, cz.w};
        const float gg[4] = {gu.x, gu.y, gu.z, gu.w};
        float zb[4], gn[4];
#ifdef CACTO_CRITIC_ELU
        const bool elu = (C.t.act >> l) & 1;
#else
        constexpr bool elu = false;
#endif
        for (int r = 0; r < 4; ++r) {
          // CosGrad: -grad * sin(x) (an elu layer: grad * exp(z) below zero)
          zb[r] = elu ? fmul(fmul(acc[r], gg[r]), act_d2(true, sv[r])) : fmul(-fmul(acc[r], gg[r]), sv[r]);
          gn[r] = fmul(acc[r], cv[r]);                 // MulGrad into the upstream grad
        }
        ZB[(zoff[l] + ot) * 64 + L.lane] = make_float4(zb[0], zb[1], zb[2], zb[3]);
        const float4 g4 = make_float4(gn[0], gn[1], gn[2], gn[3]);
        nxt[ot * 64 + L.lane] = g4;
        store_panel(gb.LT[l + 1], ld, s0 + L.c, ot, L.g, g4);
      };
    };
    float4* nA = GB + 8 * 64;
    SF.f0.run(GB, nullptr, 4, L.wave, L.lane, sp_epi(0, nA));
    __syncthreads();
    CSTAMP(6);
    SF.f1.run(nA, nullptr, 4, L.wave, L.lane, sp_epi(1, GB));
    __syncthreads();
    CSTAMP(7);
    SF.f2.run(GB, nullptr, 8, L.wave, L.lane, sp_epi(2, nA));
    __syncthreads();
    CSTAMP(8);
    SF.f3.run(nA, nullptr, 8, L.wave, L.lane, sp_epi(3, GB));
    __syncthreads();
    CSTAMP(9);
    if (L.tid < 16) gb.RT[4][s0 + L.tid] = 1.f;  // dW5 += Gbar_4 (G_4 = W5[:, 0])
  } else {
    for (int k = L.tid; k < 24 * 64; k += CACTO_THREADS) ZB[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  CSTAMP(10);

  // the transposed fragments of the last backward pass, in flight during the value loss
  CriticBwdFrags HB;
  HB.load(C, L);
  // value loss: Vbar = (2 * ((wS/B) * w)) * (V - y)   (Keras MSE, SUM_OVER_BATCH_SIZE)
  if (L.tid < 16) {
    const int c = L.tid;
    const float wv = sob ? cs.w_S : 1.f;
    const float gl = fmul(fdiv(wv, (float)cs.B_global), ws[c]);
    Vb[c] = fmul(fmul(2.f, gl), fsub(V[c], y[c]));
    gb.RT[4][Bp + s0 + c] = Vb[c];
    if (s0 + c < B) {
      if (y_out) y_out[s0 + c] = y[c];
      if (V_out) V_out[s0 + c] = V[c];
      if (Vt_out && cs.want_vt) Vt_out[s0 + c] = Vt2[c];
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 2; ++t) {  // zbar_3 += (Vbar * W5) * cos(z3): out tiles wave, wave + 4
    const int ot = L.wave + 4 * t;
    const float4 z = Cs[(zoff[3] + ot) * 64 + L.lane];
    float4 zb = ZB[(zoff[3] + ot) * 64 + L.lane];
    const float4 w = w5[t];
    const float vb = Vb[L.c];
    zb.x = fadd(zb.x, fmul(fmul(vb, w.x), z.x));
    zb.y = fadd(zb.y, fmul(fmul(vb, w.y), z.y));
    zb.z = fadd(zb.z, fmul(fmul(vb, w.z), z.z));
    zb.w = fadd(zb.w, fmul(fmul(vb, w.w), z.w));
    ZB[(zoff[3] + ot) * 64 + L.lane] = zb;
  }
  __syncthreads();
  CSTAMP(11);
  // backward through the forward graph: zbar_{l-1} += (zbar_l W_l^T) * cos(z_{l-1})
  auto hb_epi = [&](int l) {
    return [&, l](int it, floatx4 acc) {
      const float4 z = Cs[(zoff[l - 1] + it) * 64 + L.lane];
      float4 zb = ZB[(zoff[l - 1] + it) * 64 + L.lane];
      zb.x = fadd(zb.x, fmul(acc[0], z.x));
      zb.y = fadd(zb.y, fmul(acc[1], z.y));
      zb.z = fadd(zb.z, fmul(acc[2], z.z));
      zb.w = fadd(zb.w, fmul(acc[3], z.w));
      ZB[(zoff[l - 1] + it) * 64 + L.lane] = zb;
    };
  };
  auto store_rt = [&](int l) {
    for (int k = L.tid; k < C.t.OT[l] * 64; k += CACTO_THREADS) {
      const int ot = k >> 6, lane = k & 63;
      store_panel(gb.RT[l], ld, Bp + s0 + (lane & 15), ot, lane >> 4, ZB[(zoff[l] + ot) * 64 + lane]);
    }
  };
  store_rt(3);
  HB.g3.run(ZB + zoff[3] * 64, nullptr, 8, L.wave, L.lane, hb_epi(3));
  __syncthreads();
  CSTAMP(12);
  store_rt(2);
  HB.g2.run(ZB + zoff[2] * 64, nullptr, 4, L.wave, L.lane, hb_epi(2));
  __syncthreads();
  CSTAMP(13);
  store_rt(1);
  HB.g1.run(ZB + zoff[1] * 64, nullptr, 4, L.wave, L.lane, hb_epi(1));
  __syncthreads();
  CSTAMP(14);
  store_rt(0);
  CSTAMP(15);
  __syncthreads();
  CSTAMP_FLUSH;
}

__global__ void __launch_bounds__(CACTO_THREADS)
    k_critic_grad(const SysDevice* __restrict__ sdp, NetView C, NetView Tg, ChainScalars cs,
                  const double* __restrict__ storage, const int32_t* __restrict__ idx, const float* __restrict__ isw,
                  int B, GradBufs gb, float* __restrict__ y_out, float* __restrict__ V_out, float* __restrict__ Vt_out,
                  int32_t* __restrict__ step) {
  __shared__ CriticLds S;
  critic_chain(S, chain_tile_of(blockIdx.x, gridDim.x, cs.xcd_tiles), sdp, C, Tg, cs, storage, idx, isw, B, gb, y_out,
               V_out, Vt_out, step);
}

// env_simulate_derivative (env.h) of a revolute chain for a tile's T samples, spread over threads
// (a tile leaves most of the workgroup idle during the float64 dynamics): M(q) by CRBA (wave 1)
// beside h(q, v) by RNEA (wave 0) — chain_mass / chain_nle, the two halves of chain_terms in its
// operation order — then per sample NJ + 1 threads each factor M and solve one right-hand side:
// a - h (the step) or e_j (column j of M^-1, a column of Fu). The same operations on the same values
// as the one-thread path, so s' and Fu are bit-identical to it. st / stn: [T][16] floats, A: [T][NA],
// Fu: [T][CACTO_MAX_STATE * CACTO_MAX_ACTION], dM / dh: float64 scratch. Contains two barriers.
template <int NJ, int T>
__device__ __forceinline__ void chain_dynamics_spread(const SysDevice& sd, const float* st, const float* A,
                                                      double* dM, double* dh, float* stn, float* Fu, int tid) {
  constexpr int NS = Dims<NJ>::NS, NA = Dims<NJ>::NA;
  const cacto_sys_params& p = sd.p;
  const int wave = tid >> 6, lane = tid & 63;
  if constexpr (NJ == 3) {
    if (sd.pl[0] != 0.0) {
      // the planar 3R chain (the manipulator): the closed form is short, one thread per sample
      // (env_simulate_derivative's planar path, as the 16-sample chain's)
      if (tid < T) {
        const int c = tid;
        double s[NS], a[NA], sn[NS], F[NS * NA];
#pragma unroll
        for (int f = 0; f < NS; ++f) s[f] = (double)st[c * 16 + f];
#pragma unroll
        for (int i = 0; i < NA; ++i) a[i] = (double)A[c * NA + i];
        (void)env_simulate_derivative_planar3(sd, s, a, true, sn, F);
#pragma unroll
        for (int f = 0; f < 16; ++f) stn[c * 16 + f] = f < NS ? (float)sn[f] : 0.f;
#pragma unroll
        for (int k = 0; k < NS * NA; ++k) Fu[c * CACTO_MAX_STATE * CACTO_MAX_ACTION + k] = (float)F[k];
      }
      __syncthreads();
      __syncthreads();
      return;
    }
  }
  if (wave < 2 && lane < T) {
    const int c = lane;
    double q[NJ], v[NJ];
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      q[i] = (double)st[c * 16 + i];
      v[i] = (double)st[c * 16 + NJ + i];
    }
    if (wave == 0) {
      double h[NJ];
      chain_nle<NJ>(sd, q, v, h);
#pragma unroll
      for (int i = 0; i < NJ; ++i) dh[c * NJ + i] = h[i];
    } else {
      double M[NJ * NJ];
      chain_mass<NJ>(sd, q, M);
#pragma unroll
      for (int k = 0; k < NJ * NJ; ++k) dM[c * NJ * NJ + k] = M[k];
    }
  }
  __syncthreads();
  CSTAMP(12);
  if (tid < T * (NJ + 1)) {
    const int c = tid / (NJ + 1), j = tid - c * (NJ + 1);
    const double dt = p.dt;
    double L[NJ * NJ], x[NJ];
#pragma unroll
    for (int k = 0; k < NJ * NJ; ++k) L[k] = dM[c * NJ * NJ + k];
    (void)cholesky<NJ>(L);
    if (j == 0) {
#pragma unroll
      for (int i = 0; i < NJ; ++i) x[i] = (double)A[c * NA + i] - dh[c * NJ + i];
      chol_solve<NJ>(L, x);
      float* sn = stn + c * 16;
#pragma unroll
      for (int i = 0; i < NJ; ++i) {  // env_simulate_derivative's f32in update
        const double s = (double)st[c * 16 + i], vv = (double)st[c * 16 + NJ + i];
        const float vdt = __fmul_rn((float)vv, (float)dt);
        sn[i] = (float)(s + (double)vdt);
        sn[NJ + i] = (float)(double)(float)(vv + x[i] * dt);
      }
      sn[2 * NJ] = (float)((double)st[c * 16 + 2 * NJ] + dt);
#pragma unroll
      for (int f = NS; f < 16; ++f) sn[f] = 0.f;
    } else {
      const int col = j - 1;
#pragma unroll
      for (int i = 0; i < NJ; ++i) x[i] = (i == col) ? 1.0 : 0.0;
      chol_solve<NJ>(L, x);
      float* F = Fu + c * CACTO_MAX_STATE * CACTO_MAX_ACTION;
#pragma unroll
      for (int r = 0; r < NS; ++r) {
        double v = 0.0;
        if (r >= NJ && r < 2 * NJ) {
          v = x[r - NJ] * dt;
          if (p.normalize) v *= sd.inv_norm[r];
        }
        F[r * NA + col] = (float)v;
      }
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------- actor chain (a12)
// Waves per SIMD the large-batch actor chain is compiled for. 2 (<= 256 registers, some spilled)
// lets one actor and one critic workgroup share a CU: manipulator B = 8192 5.86 k -> 7.14 k
// updates/s, car_park 8.78 k -> 8.99 k; the DI (10.84 k -> 10.53 k) and UR5 (10.6 k -> 9.1 k:
// 1.9 KB of spills) keep 1. AG_WPE overrides it for every system (A/B builds).
#ifndef AG_SPREAD_NJ
#define AG_SPREAD_NJ 4  // chains from this many joints take chain_dynamics_spread in the actor chain
#endif
#ifndef AG_RING
#define AG_RING 24  // fragments in flight in the actor's W2^T pass (mm_layer_ring)
#endif
template <int NJ>
constexpr int actor_grad_wpe() {
#ifdef AG_WPE
  return AG_WPE;
#else
  return NJ == 6 ? 1 : 2;
#endif
}
// 65 KB (see CriticLds). The 40-tile region W holds, in turn: the actor's h1, h2 (tiles 0-31); the
// critic pass at s' — its h ping-pong (0-15) and cos z (16-39); the actor's zbar2 (16-31).
struct ActorLds {
  float4 X0[64], XS[64], G0[64], ZB3[64];
  float4 W[40 * 64];
  unsigned char ZS[32 * 64];  // sign bits (z > 0) of the actor's z1, z2: bit r of [(l * 16 + ot) * 64 + lane]
  float4 red[4 * 64];
  float st[256], stn[256], gn[256];
  float A[16 * CACTO_MAX_ACTION];
  float Fu[16 * CACTO_MAX_STATE * CACTO_MAX_ACTION];
  float dra[16 * CACTO_MAX_ACTION];
  float Vn[16];
  double term_s[16];
};

// one 16-sample tile of the actor chain (workgroup-wide; S in LDS)
template <int NJ>
__device__ __forceinline__ void actor_chain(ActorLds& S, const int tile, const SysDevice* __restrict__ sdp,
                                            const NetView& Ac, const NetView& C, const ChainScalars& cs,
                                            const double* __restrict__ storage, const int32_t* __restrict__ idx, int B,
                                            const GradBufs& gb, int32_t* __restrict__ step) {
  float4 *X0 = S.X0, *XS = S.XS, *G0 = S.G0, *ZB3 = S.ZB3, *H = S.W, *ZC = S.W + 16 * 64, *red = S.red;
  unsigned char* ZS = S.ZS;
  float *st = S.st, *stn = S.stn, *gn = S.gn, *A = S.A, *Fu = S.Fu, *dra = S.dra, *Vn = S.Vn;
  double* term_s = S.term_s;
  CSTAMP(0);
  const SysDevice& sd = *sdp;
  const cacto_sys_params& p = sd.p;
  const Lane L;
  const int ns = p.nb_state, na = p.nb_action, cols = 3 * ns + 3, s0 = tile * CACTO_TILE;
  const int ld = gb.ld;
  if (tile == 0 && L.tid == 0 && step) step[1] += 1;  // Keras actor optimizer iterations
  Frag1<4> F1;  // actor layer 1 (ns -> 256), in flight during the row gathers
  F1.load(Ac.fwd(0), Ac.biasp(0), L.wave, L.lane);
  {
    const int c = L.tid >> 4, f = L.tid & 15;
    const bool valid = s0 + c < B;
    const double* rp = storage + (size_t)(valid ? idx[s0 + c] : 0) * cols;
    st[c * 16 + f] = (valid && f < ns) ? (float)rp[f] : 0.f;
    if (f == 0) term_s[c] = valid ? rp[3 * ns + 2] : 0.0;
  }
  __syncthreads();
  if (L.wave == 0) {
    fill_input_tile(p, st, X0, L);
    store_panel(gb.LT[0], ld, s0 + L.c, 0, L.g, X0[L.lane]);  // input of layer 0 (normalised)
  }
  __syncthreads();
  // actor forward; h1 -> LT_1, h2 -> LT_2
  CSTAMP(1);
  actor_forward_tile(Ac, na, X0, nullptr, H, red, A, L, [&](int l, int ot, float4 z4, float4 h4) {
    ZS[(l * 16 + ot) * 64 + L.lane] = (z4.x > 0.f) | (z4.y > 0.f) << 1 | (z4.z > 0.f) << 2 | (z4.w > 0.f) << 3;
    store_panel(gb.LT[l + 1], ld, s0 + L.c, ot, L.g, h4);
  }, &F1);
  __syncthreads();
  CSTAMP(2);
  // dynamics at (s, a) in float64 from float32 tensors (environment.py:134-144, :353-362)
  if constexpr (NJ >= AG_SPREAD_NJ) {
    // revolute chains spread over the workgroup (one thread per sample held all of it; UR5
    // spilled); d reward / d a on wave 2 alongside. Its float64 scratch takes the start of the W
    // region: the actor's h1 / h2 there are dead after the action layer, the critic pass at s'
    // that fills it comes after.
    if (L.tid >= 128 && L.tid < 144) {
      constexpr int NA = Dims<NJ>::NA;
      const int c = L.tid - 128;
      float af[NA], g[NA];
#pragma unroll
      for (int i = 0; i < NA; ++i) af[i] = A[c * na + i];
      const double tc = term_s[c];
      const double w6 = 6 >= p.n_weights ? 0.0 : tc * p.w_terminal[6] + (1.0 - tc) * p.w_running[6];
      (void)reward_batch_f32<NA>(p, w6, af, 0.0, g);
#pragma unroll
      for (int i = 0; i < NA; ++i) dra[c * na + i] = g[i];
    }
    double* dM = reinterpret_cast<double*>(S.W);
    static_assert(sizeof(double) * CACTO_TILE * (NJ * NJ + NJ) <= sizeof(S.W), "chain scratch in W");
    chain_dynamics_spread<NJ, CACTO_TILE>(sd, st, A, dM, dM + CACTO_TILE * NJ * NJ, stn, Fu, L.tid);
  } else if (L.tid < 16) {
    constexpr int NS = Dims<NJ>::NS, NA = Dims<NJ>::NA;
    const int c = L.tid;
    double s[NS], a[NA], sn[NS], F[NS * NA];
    float af[NA];
#pragma unroll
    for (int f = 0; f < NS; ++f) s[f] = (double)st[c * 16 + f];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      af[i] = A[c * na + i];
      a[i] = (double)af[i];
    }
    if constexpr (NJ > 0 && NJ <= 3) {
      if (p.const_dyn) env_simulate_derivative_const<NJ>(sd, s, a, true, sn, F);
      else env_simulate_derivative<NJ>(sd, s, a, true, sn, F);
    } else {
      env_simulate_derivative<NJ>(sd, s, a, true, sn, F);
    }
#pragma unroll
    for (int f = 0; f < 16; ++f) stn[c * 16 + f] = f < NS ? (float)sn[f] : 0.f;
#pragma unroll
    for (int k = 0; k < NS * NA; ++k) Fu[c * CACTO_MAX_STATE * CACTO_MAX_ACTION + k] = (float)F[k];
  } else if (L.tid >= 64 && L.tid < 80) {
    // wave 1, alongside the dynamics: only d reward / d a enters the actor gradient
    // (NeuralNetwork.py:199-204), and only the control cost depends on a, so the state terms of the
    // reward are not evaluated here
    constexpr int NA = Dims<NJ>::NA;
    const int c = L.tid - 64;
    float af[NA], g[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) af[i] = A[c * na + i];
    const double tc = term_s[c];
    const double w6 = 6 >= p.n_weights ? 0.0 : tc * p.w_terminal[6] + (1.0 - tc) * p.w_running[6];
    (void)reward_batch_f32<NA>(p, w6, af, 0.0, g);
#pragma unroll
    for (int i = 0; i < NA; ++i) dra[c * na + i] = g[i];
  }
  __syncthreads();
  CSTAMP(3);
  if (L.wave == 0) fill_input_tile(p, stn, XS, L);
  // pipeline: the critic this pass reads is written by the other stream's Adam
  if (cs.wait_p && L.tid == 0) pipe_wait(cs.wait_p, cs.wait_v, const_cast<unsigned long long*>(cs.wait_p) - 1);
  __syncthreads();
  // critic (already updated) at s': V and dV/dx0 (NeuralNetwork.py:190-195)
  float4* HC = H;            // 16 tiles
  float4* ZB2 = H + 16 * 64;  // 16 tiles
  CSTAMP(4);
  critic_forward_tile<false>(C, XS, ZC, nullptr, HC, red, Vn, L, [](int, int, float4) {});  // V(s') unused
  __syncthreads();
  CSTAMP(5);
  critic_first_backward(C, ZC, HC, nullptr, G0, red, L, [](int, int, int, float4) {});
  __syncthreads();
  CSTAMP(6);
  // dQ/da = dV/ds' Fu + dr/da ; abar = -dQ/da / B  (NeuralNetwork.py:206-231)
  {  // d normalize / d s of every (sample, state) element at once, one per thread
    const int c = L.tid >> 4, i = L.tid & 15;
    if (i < ns) gn[c * 16 + i] = normalize_backward(p, i, reinterpret_cast<const float*>(G0)[((i >> 2) * 16 + c) * 4 + (i & 3)]);
  }
  // the two backward layers' first fragments, in flight during the rest of the dQ/da phase (W3^T:
  // KT = 1, every tile; W2^T: the first tile's 16 blocks); issued after the loads above waited on
  Frag1<4> B2;
  FragTile<16> B1;
  B2.load(Ac.bwd(2), nullptr, L.wave, L.lane);
  B1.load(Ac.bwd(1), L.wave, L.lane);
  __syncthreads();
  if (L.wave == 0) {
    const int c = L.c;
    float abar[4];
    for (int r = 0; r < 4; ++r) {
      const int j = 4 * L.g + r;
      abar[r] = 0.f;
      if (j < na && s0 + c < B) {
        float q = 0.f;
        for (int i = 0; i < ns; ++i) {
          const float t = fmul(gn[c * 16 + i], Fu[c * CACTO_MAX_STATE * CACTO_MAX_ACTION + i * na + j]);
          q = (i == 0) ? t : fadd(q, t);
        }
        q = fadd(q, dra[c * na + j]);
        abar[r] = fmul(-q, fdiv(1.f, (float)cs.B_global));
      }
    }
    const float4 v = make_float4(abar[0], abar[1], abar[2], abar[3]);
    ZB3[L.lane] = v;
    store_panel(gb.RT[2], ld, s0 + c, 0, L.g, v);
  }
  __syncthreads();
  CSTAMP(7);
  // zbar2 = (abar W3^T) * lrelu'(z2) ; zbar1 = (zbar2 W2^T) * lrelu'(z1)
  auto epi2 = [&](int it, floatx4 acc) {
    const unsigned zs = ZS[(16 + it) * 64 + L.lane];
    float o[4];
    for (int r = 0; r < 4; ++r) o[r] = (zs >> r & 1) ? acc[r] : fmul(acc[r], 0.3f);
    const float4 v = make_float4(o[0], o[1], o[2], o[3]);
    ZB2[it * 64 + L.lane] = v;
    store_panel(gb.RT[1], ld, s0 + L.c, it, L.g, v);
  };
  auto epi1 = [&](int it, floatx4 acc) {
    const unsigned zs = ZS[it * 64 + L.lane];
    float o[4];
    for (int r = 0; r < 4; ++r) o[r] = (zs >> r & 1) ? acc[r] : fmul(acc[r], 0.3f);
    store_panel(gb.RT[0], ld, s0 + L.c, it, L.g, make_float4(o[0], o[1], o[2], o[3]));
  };
  // the actor's fixed shape (see actor_forward_tile): W3^T KT = 1, W2^T KT = 16, 16 out tiles each
  mm_layer1_pre<4>(B2, ZB3, L.wave, L.lane, epi2, nullptr);
  __syncthreads();
  CSTAMP(8);
  mm_layer_ring<16, 4, AG_RING>(B1, Ac.bwd(1), ZB2, L.wave, L.lane, epi1);
  __syncthreads();
  CSTAMP(9);
  __syncthreads();
  CSTAMP_FLUSH;
#ifdef CACTO_STAMPS
  if (tile == 0 && L.tid == 0)
    for (int k_ = 0; k_ < 32; ++k_) g_astamps[k_] = cacto_stamp_s[k_];
#endif
}

template <int NJ>
__global__ void __launch_bounds__(CACTO_THREADS) __attribute__((amdgpu_waves_per_eu(actor_grad_wpe<NJ>(), 8)))
    k_actor_grad(const SysDevice* __restrict__ sdp, NetView Ac, NetView C, ChainScalars cs,
                 const double* __restrict__ storage, const int32_t* __restrict__ idx, int B, GradBufs gb,
                 int32_t* __restrict__ step) {
  __shared__ ActorLds S;
  ChainScalars c = cs;
  if (cs.wait_p && cs.wait_at_start) {
    if (threadIdx.x == 0) pipe_wait(cs.wait_p, cs.wait_v, const_cast<unsigned long long*>(cs.wait_p) - 1);
    __syncthreads();
    c.wait_p = nullptr;
  }
  actor_chain<NJ>(S, chain_tile_of(blockIdx.x, gridDim.x, cs.xcd_tiles), sdp, Ac, C, c, storage, idx, B, gb, step);
}

// The critic chain of update t (workgroups [0, nct)) and the actor chain of update t - 1 (the
// rest) in one launch: neither reads what the other writes (the actor reads the critic C_t that
// both chains take; panels and counters are separate), so the single-stream small-batch pipeline
// issues the two as one grid. LDS is the larger of the two layouts, not their sum.
template <int NJ>
__global__ void __launch_bounds__(CACTO_THREADS)
    k_chain_pair(const SysDevice* __restrict__ sdp, NetView C, NetView Tg, NetView Ac, ChainScalars cs,
                 const double* __restrict__ storage, const int32_t* __restrict__ idx_c, const float* __restrict__ isw,
                 const int32_t* __restrict__ idx_a, int B, int nct, GradBufs gbc, GradBufs gba,
                 float* __restrict__ y_out, float* __restrict__ V_out, int32_t* __restrict__ step) {
  constexpr size_t bytes = sizeof(CriticLds) > sizeof(ActorLds) ? sizeof(CriticLds) : sizeof(ActorLds);
  __shared__ __attribute__((aligned(16))) unsigned char smem[bytes];
  if ((int)blockIdx.x < nct) {
    critic_chain(*reinterpret_cast<CriticLds*>(smem), blockIdx.x, sdp, C, Tg, cs, storage, idx_c, isw, B, gbc, y_out,
                 V_out, nullptr, step);
  } else {
    actor_chain<NJ>(*reinterpret_cast<ActorLds*>(smem), blockIdx.x - nct, sdp, Ac, C, cs, storage, idx_a, B, gba,
                    step);
  }
}

}  // namespace cacto

// the same chains on 4-sample tiles (small batches)
#include "chain_q4.h"

namespace cacto {

// ---------------------------------------------------------------- weight-gradient GEMM
struct WgLayer {
  const float* LT;
  const float* RT;
  int in, out, IT, OT, woff, boff;
};
struct WgArgs {
  WgLayer l[MAX_LAYERS];
  int nl, ld, r_begin, r_end, bias_r0, CH, nch, P, tpc;
  int toff[MAX_LAYERS + 1];
  unsigned char perm[64];  // k_wgrad_big: the items of a chunk by decreasing work (full 4 x 4 blocks first)
};

// One workgroup per (row chunk, item). An item is a block of up to 4 x 4 output tiles of one layer
// (the 4 waves split the chunk's rows, each keeping 16 accumulator tiles, then reduce through LDS
// in a fixed order, so the result is deterministic), or up to 4 bias tiles (one per wave). A
// block loads each LT/RT panel slice once for 4 tiles instead of once per tile.
constexpr int WG_BLK = 4;
// 16-row steps of panel slices in flight per wave. Measured (updates/s, DI B = 4096): 1 11.3 k,
// 2 10.5 k, 3 10.3 k — deeper prefetch costs the GEMM its 4 waves per SIMD beside the chains.
#ifndef WG_PF
#define WG_PF 1
#endif

// One workgroup's block of NI x NO output tiles (of a layer) over the rows [lo, hi) of one chunk:
// the 4 waves split the rows, each keeping NI x NO accumulator tiles, then reduce through LDS in a
// fixed order ((p0 + p1) + p2) + p3 (deterministic), in rounds of 8 tiles. ni, no: the tiles that
// exist (<= NI, NO; the generic 4 x 4 instance runs edge blocks on clamped duplicate tiles).
template <int NI, int NO>
__device__ __forceinline__ void wg_block(const WgArgs& a, const WgLayer& Ly, int lo, int hi, int it0, int ot0, int ni,
                                         int no, float* __restrict__ out, float4* part) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int span = ((hi - lo) / 16 + 3) / 4 * 16;  // rows per wave, multiple of 16
  const int r0 = lo + wave * span, r1 = min(hi, r0 + span);
  floatx4 acc[NI][NO];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int o = 0; o < NO; ++o) acc[i][o] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float* ap = Ly.LT + (size_t)(16 * it0 + c) * a.ld + 4 * g;
  const float* bp = Ly.RT + (size_t)(16 * ot0 + c) * a.ld + 4 * g;
  // panel slices of the next WG_PF 16-row steps are in flight while a step's MFMAs run; the steps
  // are summed in row order whatever the depth
  float4 As[WG_PF][NI], Bs[WG_PF][NO];
  auto fetch = [&](float4 (&An)[NI], float4 (&Bn)[NO], int r) {
    const int rr = min(r, r1 - 16);  // clamped (branch-free); a past-the-end fetch is unused
#pragma unroll
    for (int i = 0; i < NI; ++i) An[i] = *reinterpret_cast<const float4*>(ap + (size_t)16 * min(i, ni - 1) * a.ld + rr);
#pragma unroll
    for (int o = 0; o < NO; ++o) Bn[o] = *reinterpret_cast<const float4*>(bp + (size_t)16 * min(o, no - 1) * a.ld + rr);
  };
  auto step = [&](const float4 (&A)[NI], const float4 (&Bv)[NO]) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int o = 0; o < NO; ++o) acc[i][o] = mfma4(A[i].x, Bv[o].x, acc[i][o]);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int o = 0; o < NO; ++o) acc[i][o] = mfma4(A[i].y, Bv[o].y, acc[i][o]);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int o = 0; o < NO; ++o) acc[i][o] = mfma4(A[i].z, Bv[o].z, acc[i][o]);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int o = 0; o < NO; ++o) acc[i][o] = mfma4(A[i].w, Bv[o].w, acc[i][o]);
  };
  if (r0 < r1) {
#pragma unroll
    for (int d = 0; d < WG_PF; ++d) fetch(As[d], Bs[d], r0 + 16 * d);
  }
  for (int r = r0; r < r1; r += 16 * WG_PF) {
#pragma unroll
    for (int d = 0; d < WG_PF; ++d) {
      if (r + 16 * d < r1) {
        float4 A[NI], Bv[NO];
#pragma unroll
        for (int i = 0; i < NI; ++i) A[i] = As[d][i];
#pragma unroll
        for (int o = 0; o < NO; ++o) Bv[o] = Bs[d][o];
        fetch(As[d], Bs[d], r + 16 * (d + WG_PF));
        step(A, Bv);
      }
    }
  }
  constexpr int NT = NI * NO, HT = NT < 8 ? NT : 8;  // tiles, tiles per round
  constexpr int NR = (NT + HT - 1) / HT;
#pragma unroll
  for (int h = 0; h < NR; ++h) {
    if (h) __syncthreads();  // the previous round's partials are consumed
#pragma unroll
    for (int t = h * HT; t < h * HT + HT && t < NT; ++t) part[(wave * HT + (t - h * HT)) * 64 + lane] = f4(acc[t / NO][t % NO]);
    __syncthreads();
    // wave w finishes the round's tiles 2w, 2w + 1: ((p0 + p1) + p2) + p3
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int tl = wave * 2 + k, t = h * HT + tl, i = t / NO, o = t % NO;
      if (tl >= HT || t >= NT || i >= ni || o >= no) continue;
      float4 s4 = part[(0 * HT + tl) * 64 + lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        const float4 q = part[(w * HT + tl) * 64 + lane];
        s4.x += q.x;
        s4.y += q.y;
        s4.z += q.z;
        s4.w += q.w;
      }
      const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
      const int oc = 16 * (ot0 + o) + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ii = 16 * (it0 + i) + 4 * g + q;
        if (ii < Ly.in && oc < Ly.out) out[Ly.woff + ii * Ly.out + oc] = sv[q];
      }
    }
  }
}

//
// xcd = 1: the items of one chunk run on blocks that share an XCD (blocks b and b + 8 are dealt to
// one; observed dealing, so it decides only which L2 serves a re-read): chunk (b / 8 / tpc) * 8 +
// b % 8, item (b / 8) % tpc. The 4 (resp. nbi) blocks that read one LT (RT) slice then read it from
// one L2 instead of up to four; the grid is padded to whole groups of 8 chunks.
//
// sig_p (the pipeline's device-side ordering): this launch follows the actor chain of an iteration
// on its stream, so that chain has finished; block 0 publishes sig_v = (iterations done) for the
// critic stream's Adam, which must not overwrite a critic buffer the chain read (k_adam's wait_p).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) k_wgrad(WgArgs a, float* __restrict__ slab, int xcd,
                                               unsigned long long* sig_p, unsigned long long sig_v) {
  // 32 KiB: the 16 tiles are reduced in two rounds of 8, so a GEMM workgroup fits on a CU beside
  // a chain workgroup — the pipelined update runs the two concurrently
  __shared__ float4 part[4 * (WG_BLK * WG_BLK / 2) * 64];
  if (sig_p && blockIdx.x == 0 && threadIdx.x == 0)  // write-after-read order only: relaxed
    __hip_atomic_store(sig_p, sig_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int chunk, rem;
  if (xcd) {
    const int sl = blockIdx.x >> 3;
    chunk = (sl / a.tpc) * 8 + (blockIdx.x & 7);
    rem = sl % a.tpc;
    if (chunk >= a.nch) return;
  } else {
    chunk = blockIdx.x / a.tpc;
    rem = blockIdx.x - chunk * a.tpc;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  int li = 0;
  while (rem >= a.toff[li + 1]) ++li;
  const WgLayer& Ly = a.l[li];
  rem -= a.toff[li];
  const int lo = a.r_begin + chunk * a.CH, hi = min(a.r_end, lo + a.CH);
  float* out = slab + (size_t)chunk * a.P;
  const int nbi = (Ly.IT + WG_BLK - 1) / WG_BLK, nbo = (Ly.OT + WG_BLK - 1) / WG_BLK;
  if (rem < nbi * nbo) {
    const int it0 = (rem / nbo) * WG_BLK, ot0 = (rem % nbo) * WG_BLK;
    const int ni = min(WG_BLK, Ly.IT - it0), no = min(WG_BLK, Ly.OT - ot0);
    // the block shapes the networks have, compiled for their size (an edge block of the input or
    // output layer loads and multiplies only its own tiles); any other shape runs the 4 x 4 code
    // on clamped duplicate tiles (unused)
    if (ni == WG_BLK && no == WG_BLK) wg_block<WG_BLK, WG_BLK>(a, Ly, lo, hi, it0, ot0, ni, no, out, part);
    else if (ni == 1 && no == WG_BLK) wg_block<1, WG_BLK>(a, Ly, lo, hi, it0, ot0, ni, no, out, part);
    else if (ni == WG_BLK && no == 1) wg_block<WG_BLK, 1>(a, Ly, lo, hi, it0, ot0, ni, no, out, part);
    else wg_block<WG_BLK, WG_BLK>(a, Ly, lo, hi, it0, ot0, ni, no, out, part);
  } else {
    const int ot = (rem - nbi * nbo) * WG_BLK + wave;
    if (ot >= Ly.OT) return;
    const float* bp = Ly.RT + (size_t)(16 * ot + c) * a.ld + 4 * g;
    float s = 0.f;
    int r = max(lo, a.bias_r0);
    for (; r + 64 <= hi; r += 64) {  // 4 loads in flight, summed in row order
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const float4*>(bp + r + 16 * k);
#pragma unroll
      for (int k = 0; k < 4; ++k) s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    }
    for (; r < hi; r += 16) {
      const float4 v = *reinterpret_cast<const float4*>(bp + r);
      s += (v.x + v.y) + (v.z + v.w);
    }
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (g == 0 && 16 * ot + c < Ly.out) out[Ly.boff + 16 * ot + c] = s;
  }
}

// ---------------------------------------------------------------- weight-gradient GEMM, large batches
// k_wgrad_big (rows > 1024: the B >= 1024 updates). The same items as k_wgrad (a block of up to 4 x 4
// output tiles of one layer over one row chunk, or up to 4 bias tiles, slab[chunk][P] out), but the
// 4 waves split the block's TILES instead of its rows: wave w owns A tile w (NI = 4; B tile w when
// NI = 1) and walks every 16-row step of the chunk, so each wave's accumulators cover the whole chunk
// and are written straight to the slab (no cross-wave LDS reduction). The workgroup stages each
// step's panel slices (NI + NO slices of 16 features x 16 rows, 2 float4 per thread) through a
// 2-buffer LDS ring, with the global loads issued AH steps ahead into registers, so the
// latency of a step's loads hides behind AH steps of MFMAs (k_wgrad: one step, and a wave
// covered only 2-4 steps of its chunk, so its time was mostly load latency: 18-21 us per launch at
// B = 4096 alone, 0.17 of the MFMA peak). Each tile's sum runs over the chunk's rows in row order
// (one MFMA accumulator chain; four k-phase chains for the 1-tile waves of edge blocks) — a
// different, fixed order than k_wgrad's four row spans, so the batch sizes that take this kernel
// form their own, schedule-independent, sums.
constexpr int WGB_FS = 20;                    // floats per staged feature row (16 rows + 4 pad: LDS banks)
constexpr int WGB_SLICE = 16 * WGB_FS;        // one 16 x 16 panel slice
constexpr int WGB_STAGE = 8 * WGB_SLICE;      // up to 4 A + 4 B slices

template <int NI, int NO, int AH>
__device__ __forceinline__ void wgb_block(const int ld, const WgLayer Ly, int lo, int hi, int it0, int ot0,
                                          float* __restrict__ out, float* stage) {
  static_assert((NI == 4 && (NO == 4 || NO == 1)) || (NI == 1 && NO == 4), "block shape");
  static_assert(AH == 3 || AH == 6, "the step loop below is unrolled by hand for 3 or 6 landing buffers");
  constexpr int NS = NI + NO;  // staged slices per step
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, c = lane & 15;
  // the loader's part of a step: slice sl = tid >> 5 (if < NS), feature f = (tid >> 1) & 15, rows
  // [8 h, 8 h + 8) of the step, h = tid & 1
  const int sl = tid >> 5, f = (tid >> 1) & 15, h = tid & 1;
  const bool loader = sl < NS;
  const float* src = nullptr;
  if (loader) {
    const int slc = sl < NI ? sl : sl - NI;
    const float* base = sl < NI ? Ly.LT + (size_t)(16 * (it0 + slc)) * ld : Ly.RT + (size_t)(16 * (ot0 + slc)) * ld;
    src = base + (size_t)f * ld + 8 * h;
  }
  const int nsteps = (hi - lo) / 16;  // chunks are multiples of 16 rows
  // landing registers of the next AH steps (named, not an array: an array passed by reference
  // went to scratch)
  float4 r0a, r0b, r1a, r1b, r2a, r2b, r3a, r3b, r4a, r4b, r5a, r5b;
  // clamped, branch-free loads (a past-the-end or non-loader load rereads a valid address; unused)
  const float* src_c = loader ? src : Ly.RT;
  auto load = [&](float4& ra, float4& rb, int s) {
    const float4* p = reinterpret_cast<const float4*>(src_c + lo + 16 * min(s, nsteps - 1));
    ra = p[0];
    rb = p[1];
  };
  load(r0a, r0b, 0);
  load(r1a, r1b, 1);
  load(r2a, r2b, 2);
  if constexpr (AH == 6) {
    load(r3a, r3b, 3);
    load(r4a, r4b, 4);
    load(r5a, r5b, 5);
  }
  // this wave's tiles: NI = 4 -> (w, 0..NO-1); NI = 1 -> (0, w)
  constexpr int NT = NI == 4 ? NO : 1;
  // accumulator chains per tile: one when the wave has 4 tiles (their MFMAs interleave), one per
  // k-phase when it has one
  constexpr int NC = NT == 1 ? 4 : 1;
  floatx4 acc[NT][NC];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int k = 0; k < NC; ++k) acc[t][k] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int ai = NI == 4 ? wave : 0;
  // one step from landing registers r: stage them, refill r with step s + AH, MFMAs
  auto step = [&](float4& ra, float4& rb, int s) {
    float* st = stage + (s & 1) * WGB_STAGE;
    if (loader) {
      float4* q = reinterpret_cast<float4*>(st + sl * WGB_SLICE + f * WGB_FS + 8 * h);
      q[0] = ra;
      q[1] = rb;
    }
    load(ra, rb, s + AH);
    __syncthreads();
    // operands: lane (g, c) = feature c, rows 4g .. 4g + 3 of the step (the k_wgrad layout)
    const float4 av = *reinterpret_cast<const float4*>(st + ai * WGB_SLICE + c * WGB_FS + 4 * g);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int bo = NI == 4 ? t : wave;
      const float4 bv = *reinterpret_cast<const float4*>(st + (NI + bo) * WGB_SLICE + c * WGB_FS + 4 * g);
      acc[t][0] = mfma4(av.x, bv.x, acc[t][0]);
      acc[t][1 % NC] = mfma4(av.y, bv.y, acc[t][1 % NC]);
      acc[t][2 % NC] = mfma4(av.z, bv.z, acc[t][2 % NC]);
      acc[t][3 % NC] = mfma4(av.w, bv.w, acc[t][3 % NC]);
    }
  };
  int s = 0;
  for (; s + AH <= nsteps; s += AH) {
    step(r0a, r0b, s);
    step(r1a, r1b, s + 1);
    step(r2a, r2b, s + 2);
    if constexpr (AH == 6) {
      step(r3a, r3b, s + 3);
      step(r4a, r4b, s + 4);
      step(r5a, r5b, s + 5);
    }
  }
  if (s < nsteps) step(r0a, r0b, s);
  if (s + 1 < nsteps) step(r1a, r1b, s + 1);
  if constexpr (AH == 6) {
    if (s + 2 < nsteps) step(r2a, r2b, s + 2);
    if (s + 3 < nsteps) step(r3a, r3b, s + 3);
    if (s + 4 < nsteps) step(r4a, r4b, s + 4);
  }
  // tile sums (four k-phase chains: (c0 + c1) + (c2 + c3)), straight to the slab
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int i = NI == 4 ? wave : 0, o = NI == 4 ? t : wave;
    floatx4 sm = acc[t][0];
    if constexpr (NC == 4) sm = (acc[t][0] + acc[t][1 % NC]) + (acc[t][2 % NC] + acc[t][3 % NC]);
    const int oc = 16 * (ot0 + o) + c;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ii = 16 * (it0 + i) + 4 * g + q;
      if (ii < Ly.in && oc < Ly.out) out[Ly.woff + ii * Ly.out + oc] = sm[q];
    }
  }
}

//
// Grid order: block b runs on XCD b % 8 (observed dealing), which owns chunks x, x + 8, ...; its j-th
// block (j = b / 8) takes item perm[j / cpx] of its chunk j % cpx — every XCD starts with the full
// 4 x 4 blocks of all its chunks, one per CU, before the lighter items fill in (with the work dealt
// chunk-major, two heavy items could share a CU's matrix cores while others idled).
template <int AH>
__device__ __forceinline__ void wgrad_big_body(const int blk, const WgArgs& a, float* __restrict__ slab, int xcd,
                                               unsigned long long* sig_p, unsigned long long sig_v, float* stage) {
  if (sig_p && blk == 0 && threadIdx.x == 0)  // write-after-read order only: relaxed
    __hip_atomic_store(sig_p, sig_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int chunk, rem;
  if (xcd) {
    const int j = blk >> 3, cpx = (a.nch + 7) >> 3;
    const int pi = j / cpx;
    chunk = (j - pi * cpx) * 8 + (blk & 7);
    if (chunk >= a.nch || pi >= a.tpc) return;
    rem = a.perm[pi];
  } else {
    chunk = blk / a.tpc;
    rem = a.perm[blk - chunk * a.tpc];
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  int li = 0;
  while (rem >= a.toff[li + 1]) ++li;
  const WgLayer& Ly = a.l[li];
  rem -= a.toff[li];
  const int lo = a.r_begin + chunk * a.CH, hi = min(a.r_end, lo + a.CH);
  float* out = slab + (size_t)chunk * a.P;
  const int nbi = (Ly.IT + WG_BLK - 1) / WG_BLK, nbo = (Ly.OT + WG_BLK - 1) / WG_BLK;
  if (rem < nbi * nbo) {
    const int it0 = (rem / nbo) * WG_BLK, ot0 = (rem % nbo) * WG_BLK;
    const int ni = min(WG_BLK, Ly.IT - it0), no = min(WG_BLK, Ly.OT - ot0);
    const WgLayer lv{Ly.LT, Ly.RT, Ly.in, Ly.out, Ly.IT, Ly.OT, Ly.woff, Ly.boff};
    if (ni == 4 && no == 4) wgb_block<4, 4, AH>(a.ld, lv, lo, hi, it0, ot0, out, stage);
    else if (ni == 1 && no == 4) wgb_block<1, 4, AH>(a.ld, lv, lo, hi, it0, ot0, out, stage);
    else if (ni == 4 && no == 1) wgb_block<4, 1, AH>(a.ld, lv, lo, hi, it0, ot0, out, stage);
    // (the host checks that every block of the network has one of these shapes)
  } else {
    const int ot = (rem - nbi * nbo) * WG_BLK + wave;
    if (ot >= Ly.OT) return;
    const float* bp = Ly.RT + (size_t)(16 * ot + c) * a.ld + 4 * g;
    float s = 0.f;
    int r = max(lo, a.bias_r0);
    for (; r + 64 <= hi; r += 64) {  // 4 loads in flight, summed in row order
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const float4*>(bp + r + 16 * k);
#pragma unroll
      for (int k = 0; k < 4; ++k) s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    }
    for (; r < hi; r += 16) {
      const float4 v = *reinterpret_cast<const float4*>(bp + r);
      s += (v.x + v.y) + (v.z + v.w);
    }
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (g == 0 && 16 * ot + c < Ly.out) out[Ly.boff + 16 * ot + c] = s;
  }
}

template <int AH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) k_wgrad_big(WgArgs a, float* __restrict__ slab, int xcd,
                                                   unsigned long long* sig_p, unsigned long long sig_v) {
  __shared__ __attribute__((aligned(16))) float stage[2 * WGB_STAGE];  // 20 KiB
  wgrad_big_body<AH>(blockIdx.x, a, slab, xcd, sig_p, sig_v, stage);
}

// The pipelined PER loop's critic GEMM with the priority update of the same update in one grid:
// blocks [0, nwg) are k_wgrad_big's (the same XCD dealing: nwg is its grid), the next nroot run
// per_update_run_body over the subtrees. Both need only the critic chain before them, and the next
// sample needs both (the trees, and this stream's order). LDS: the GEMM's 20 KiB ring, the priority
// update's 10 KiB in the same bytes.
template <int AH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8)))
k_wgrad_big_per(WgArgs a, float* __restrict__ slab, int xcd, int nwg, PerRunArgs pa, int nroot) {
  static_assert(sizeof(PerRunLds) <= 2 * WGB_STAGE * sizeof(float), "LDS union");
  __shared__ __attribute__((aligned(16))) float stage[2 * WGB_STAGE];  // 20 KiB
  if ((int)blockIdx.x < nwg) wgrad_big_body<AH>(blockIdx.x, a, slab, xcd, nullptr, 0, stage);
  else per_update_run_body(blockIdx.x - nwg, nroot, pa, *reinterpret_cast<PerRunLds*>(stage));
}

// ---------------------------------------------------------------- Adam (+ packed refresh, soft update)
struct AdamArgs {
  double beta1, beta2, eps, tau;
  double lr[5];
  double bounds[4];
  int which;  // 0 critic counter, 1 actor counter
  int soft;
};

// write_packed for a weight W_l[i][o] whose layer and indices are known (no search, no division)
__device__ __forceinline__ void write_packed_w(float4* pk4, const NetTopo& t, int l, int i, int o, float val) {
  float* pk = reinterpret_cast<float*>(pk4);
  pk[((size_t)(t.pkoff[l] + (o >> 4) * t.KT[l] + (i >> 4)) * 64 + ((i & 15) >> 2) * 16 + (o & 15)) * 4 + (i & 3)] = val;
  pk[((size_t)(t.blocks + t.pkoff[l] + (i >> 4) * t.OT[l] + (o >> 4)) * 64 + ((o & 15) >> 2) * 16 + (i & 15)) * 4 +
     (o & 3)] = val;
}

// thru: the store written through to memory at agent scope (a relaxed atomic store), for a reader
// on another stream that orders itself by a device-side flag instead of a kernel boundary
__device__ __forceinline__ void store_f(float* p, float v, bool thru) {
  if (thru) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

__device__ __forceinline__ void write_packed(float4* pk4, const NetTopo& t, int p, float val, bool thru = false) {
  float* pk = reinterpret_cast<float*>(pk4);
  int l = t.L - 1;
  while (t.woff[l] > p) --l;
  if (p >= t.boff[l]) return;
  const int local = p - t.woff[l];
  const int i = local / t.out[l], o = local - (local / t.out[l]) * t.out[l];
  store_f(pk + ((size_t)(t.pkoff[l] + (o >> 4) * t.KT[l] + (i >> 4)) * 64 + ((i & 15) >> 2) * 16 + (o & 15)) * 4 + (i & 3),
          val, thru);
  store_f(pk + ((size_t)(t.blocks + t.pkoff[l] + (i >> 4) * t.OT[l] + (o >> 4)) * 64 + ((o & 15) >> 2) * 16 + (i & 15)) * 4 +
              (o & 3),
          val, thru);
}

struct AdamScalars {
  float alpha, c1, c2, eps, tau, omt;
};

__device__ __forceinline__ AdamScalars adam_scalars(const AdamArgs& a, const int32_t* step) {
  const int it = step[a.which];  // = Keras iterations + 1
  const int iters = it - 1;
  double lr = a.lr[4];
  for (int k = 0; k < 4; ++k)
    if ((double)iters <= a.bounds[k]) {
      lr = a.lr[k];
      break;
    }
  const float tf = (float)it;
  const float b1p = powf((float)a.beta1, tf), b2p = powf((float)a.beta2, tf);
  AdamScalars s;
  s.alpha = fdiv(fmul((float)lr, __fsqrt_rn(fsub(1.f, b2p))), fsub(1.f, b1p));
  s.c1 = (float)(1.0 - a.beta1);
  s.c2 = (float)(1.0 - a.beta2);
  s.eps = (float)a.eps;
  s.tau = (float)a.tau;
  s.omt = (float)(1.0 - a.tau);
  return s;
}

// NCH > 0: every chunk partial of a parameter is loaded at once (clamped, branch-free) together with
// m, v, the weight and the target value, so a thread waits for one memory latency instead of one per
// group of 8 chunks plus one per leftover chunk (B = 4096: 32 chunks, ~11 dependent rounds, 11 us);
// the partials are still summed in chunk order (bit-identical). NCH = 0: any chunk count.
//
// wait_p / wait_v: the pipeline's wait before overwriting a critic buffer an actor chain of the other
// stream read (k_wgrad's sig_p publishes those chains). sig_p / sig_v: after its stores (written
// through to memory, `thru`) the last workgroup to finish publishes sig_p[2] = sig_v (this Adam step
// done) for the actor chain's wait: every thread's stores have completed (waitcnt) before its
// workgroup counts itself; no fence, no L2 write-back.
// nblk: the Adam step's workgroups (the launch's, or the leading part of k_adam_sample's).
// ("Memory-ordering contract", site 2: why no release / acquire is needed here)
__device__ __forceinline__ void adam_publish_thru(unsigned long long* sig_p, unsigned long long sig_v, int nblk) {
  if (!sig_p) return;
  __shared__ int last;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(sig_p + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (unsigned long long)(nblk - 1);
  __syncthreads();
  if (last && threadIdx.x == 0) {
    __hip_atomic_store(sig_p + 3, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sig_p + 2, sig_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int NCH>
__device__ __forceinline__ void adam_nch_body(const int blk, const float* __restrict__ slab, int nch, const NetTopo& t,
                                              const float* src, float* netbuf, float4* packed, float* __restrict__ m,
                                              float* __restrict__ v, const int32_t* __restrict__ step, const AdamArgs& a,
                                              float* target, float4* target_packed, const unsigned long long* wait_p,
                                              unsigned long long wait_v, bool thru = false) {
  const int p0 = blk * 256 + threadIdx.x;
  float q[NCH], mm = 0.f, vv = 0.f, th0 = 0.f, tg0 = 0.f;
  const int pc = min(p0, t.params - 1);
#pragma unroll
  for (int k = 0; k < NCH; ++k) q[k] = slab[(size_t)min(k, nch - 1) * t.params + pc];
  mm = m[pc];
  vv = v[pc];
  th0 = src[pc];
  if (a.soft) tg0 = target[pc];
  const AdamScalars s = adam_scalars(a, step);
  pipe_wait(wait_p, wait_v, const_cast<unsigned long long*>(wait_p) + 1);  // the loads above are in flight
  if (p0 < t.params) {
    float g = q[0];
#pragma unroll
    for (int k = 1; k < NCH; ++k)
      if (k < nch) g += q[k];
    mm = fadd(mm, fmul(fsub(g, mm), s.c1));
    vv = fadd(vv, fmul(fsub(fmul(g, g), vv), s.c2));
    const float th = fsub(th0, fdiv(fmul(mm, s.alpha), fadd(__fsqrt_rn(vv), s.eps)));
    m[p0] = mm;
    v[p0] = vv;
    store_f(netbuf + p0, th, thru);
    write_packed(packed, t, p0, th, thru);
    if (a.soft) {
      const float tg = fadd(fmul(th, s.tau), fmul(tg0, s.omt));
      target[p0] = tg;
      write_packed(target_packed, t, p0, tg);
    }
  }
}

// The pipelined PER loop's critic Adam step with the next update's sample in one grid: blocks
// [0, nadam) are k_adam<NCH>'s, the rest run per_sample_body (4,096-node top, recording the runs for
// the next priority update). The sample needs the trees this update's priority update left (the
// launch before on this stream); the next critic chain needs both.
template <int NCH>
__global__ void __launch_bounds__(256) k_adam_sample(const float* __restrict__ slab, int nch, NetTopo t, const float* src,
                                                     float* netbuf, float4* packed, float* __restrict__ m,
                                                     float* __restrict__ v, const int32_t* __restrict__ step, AdamArgs a,
                                                     float* target, float4* target_packed,
                                                     const unsigned long long* wait_p, unsigned long long wait_v,
                                                     int nadam, PerSampleArgs sa, unsigned long long* sig_p,
                                                     unsigned long long sig_v, int thru) {
  __shared__ double top_s[PER_FUSED_TOP];
  __shared__ double scal_s[4];
  if ((int)blockIdx.x < nadam) {
    adam_nch_body<NCH>(blockIdx.x, slab, nch, t, src, netbuf, packed, m, v, step, a, target, target_packed, wait_p,
                       wait_v, thru != 0);
    adam_publish_thru(sig_p, sig_v, nadam);  // (sig_p only with write-through stores)
  } else
    per_sample_body<PER_FUSED_TOP>(blockIdx.x - nadam, sa, top_s, scal_s);
}

template <int NCH>
__global__ void __launch_bounds__(256) k_adam(const float* __restrict__ slab, int nch, NetTopo t, const float* src,
                                              float* netbuf, float4* packed, float* __restrict__ m, float* __restrict__ v,
                                              const int32_t* __restrict__ step, AdamArgs a, float* target,
                                              float4* target_packed, const unsigned long long* wait_p,
                                              unsigned long long wait_v, unsigned long long* sig_p,
                                              unsigned long long sig_v, int thru) {
  if constexpr (NCH > 0) {
    adam_nch_body<NCH>(blockIdx.x, slab, nch, t, src, netbuf, packed, m, v, step, a, target, target_packed, wait_p,
                       wait_v, thru != 0);
    adam_publish_thru(sig_p, sig_v, gridDim.x);  // (sig_p only with write-through stores)
    return;
  }
  const int it = step[a.which];  // = Keras iterations + 1
  const int iters = it - 1;
  double lr = a.lr[4];
  for (int k = 0; k < 4; ++k)
    if ((double)iters <= a.bounds[k]) {
      lr = a.lr[k];
      break;
    }
  const float tf = (float)it;
  const float b1p = powf((float)a.beta1, tf), b2p = powf((float)a.beta2, tf);
  const float alpha = fdiv(fmul((float)lr, __fsqrt_rn(fsub(1.f, b2p))), fsub(1.f, b1p));
  const float c1 = (float)(1.0 - a.beta1), c2 = (float)(1.0 - a.beta2), eps = (float)a.eps;
  const float tau = (float)a.tau, omt = (float)(1.0 - a.tau);
  pipe_wait(wait_p, wait_v, const_cast<unsigned long long*>(wait_p) + 1);
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < t.params; p += gridDim.x * blockDim.x) {
    // chunk partials summed in chunk order; loads issued 8 at a time so they overlap
    float g = slab[p];
    int ch = 1;
    for (; ch + 8 <= nch; ch += 8) {
      float q[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) q[k] = slab[(size_t)(ch + k) * t.params + p];
#pragma unroll
      for (int k = 0; k < 8; ++k) g += q[k];
    }
    for (; ch < nch; ++ch) g += slab[(size_t)ch * t.params + p];
    float mm = m[p], vv = v[p];
    mm = fadd(mm, fmul(fsub(g, mm), c1));
    vv = fadd(vv, fmul(fsub(fmul(g, g), vv), c2));
    const float th = fsub(src[p], fdiv(fmul(mm, alpha), fadd(__fsqrt_rn(vv), eps)));
    m[p] = mm;
    v[p] = vv;
    store_f(netbuf + p, th, thru != 0);
    write_packed(packed, t, p, th, thru != 0);
    if (a.soft) {
      const float tg = fadd(fmul(th, tau), fmul(target[p], omt));
      target[p] = tg;
      write_packed(target_packed, t, p, tg);
    }
  }
  adam_publish_thru(sig_p, sig_v, gridDim.x);
}

__global__ void __launch_bounds__(256) k_soft(NetTopo t, const float* __restrict__ src, float* target,
                                              float4* target_packed, double tau_d) {
  const float tau = (float)tau_d, omt = (float)(1.0 - tau_d);
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < t.params; p += gridDim.x * blockDim.x) {
    const float tg = fadd(fmul(src[p], tau), fmul(target[p], omt));
    target[p] = tg;
    write_packed(target_packed, t, p, tg);
  }
}

// The data-parallel path's chunk sum (the gradient each rank all-reduces): out[p] = the nch
// partials of parameter p summed in chunk order, as k_adam sums them. NCH > 0: one parameter per
// thread with every partial loaded at once (clamped, branch-free), so a thread waits for one memory
// latency instead of one per chunk (the looped form, NCH = 0, issued one load per add: 16-32
// dependent round trips, 7-8 us per launch at B = 4096).
template <int NCH>
__global__ void __launch_bounds__(256) k_reduce(const float* __restrict__ slab, int nch, int P, float* __restrict__ out) {
  if constexpr (NCH > 0) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    const int pc = min(p, P - 1);
    float q[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) q[k] = slab[(size_t)min(k, nch - 1) * P + pc];
    float g = q[0];
#pragma unroll
    for (int k = 1; k < NCH; ++k)
      if (k < nch) g += q[k];
    if (p < P) out[p] = g;
    return;
  }
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
    float g = slab[p];
    for (int ch = 1; ch < nch; ++ch) g += slab[(size_t)ch * P + p];
    out[p] = g;
  }
}

int launch_reduce(const float* slab, int nch, int P, float* out, hipStream_t st) {
  const int full = (P + 255) / 256;
  if (nch <= 8)
    hipLaunchKernelGGL(k_reduce<8>, dim3(full), dim3(256), 0, st, slab, nch, P, out);
  else if (nch <= 16)
    hipLaunchKernelGGL(k_reduce<16>, dim3(full), dim3(256), 0, st, slab, nch, P, out);
  else if (nch <= 32)
    hipLaunchKernelGGL(k_reduce<32>, dim3(full), dim3(256), 0, st, slab, nch, P, out);
  else if (nch <= 64)
    hipLaunchKernelGGL(k_reduce<64>, dim3(full), dim3(256), 0, st, slab, nch, P, out);
  else
    hipLaunchKernelGGL(k_reduce<0>, dim3(std::min(full, 1024)), dim3(256), 0, st, slab, nch, P, out);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

// ---------------------------------------------------------------- fused weight gradient + Adam (small batches)
// For batches whose weight-gradient rows fit 64-row chunks (rows <= 1024), k_wgrad + k_adam run as
// one launch: one wave per 16 x 16 weight tile or 16-wide bias tile of a layer, over ALL rows,
// then the Adam step (+ packed refresh, + soft update) on the tile's parameters straight from the
// accumulators. No slab round trip and one launch instead of two. The sums are formed in exactly
// the order of k_wgrad (per chunk: the four 16-row wave spans, each a 4-MFMA chain from zero,
// reduced ((p0 + p1) + p2) + p3; bias: 64-row groups, then shuffles over g) followed by k_adam's
// chunk order, so results are bit-identical to the split path.
struct AdamNet {
  WgArgs wg;  // panels, rows, 64-row chunking (as k_wgrad)
  NetTopo t;
  const float* src;  // weights the step starts from (== nb for an in-place step)
  float* nb;
  float4* pk;
  float* m;
  float* v;
  float* target;  // soft update (critic) or nullptr
  float4* tpk;
  AdamArgs ad;
  int items;                    // weight tiles + bias tiles, all layers
  int ioff[MAX_LAYERS + 1];     // first item of layer l: KT*OT weight tiles then OT bias tiles
};

// k_adam's per-parameter arithmetic (same ops, same order), values only
__device__ __forceinline__ void adam_math(const AdamScalars& s, float g, float& mm, float& vv, float& th, float& tg) {
  mm = fadd(mm, fmul(fsub(g, mm), s.c1));
  vv = fadd(vv, fmul(fsub(fmul(g, g), vv), s.c2));
  th = fsub(th, fdiv(fmul(mm, s.alpha), fadd(__fsqrt_rn(vv), s.eps)));
  tg = fadd(fmul(th, s.tau), fmul(tg, s.omt));
}

// k_adam's per-parameter arithmetic (same ops, same order); l >= 0: a weight W_l[i][o] (direct
// packed writes), l < 0: a bias (not packed)
__device__ __forceinline__ void adam_apply(const AdamNet& N, const AdamScalars& s, int p, float g, float mm, float vv,
                                           float th0, float tg0, int l, int i, int o) {
  mm = fadd(mm, fmul(fsub(g, mm), s.c1));
  vv = fadd(vv, fmul(fsub(fmul(g, g), vv), s.c2));
  const float th = fsub(th0, fdiv(fmul(mm, s.alpha), fadd(__fsqrt_rn(vv), s.eps)));
  N.m[p] = mm;
  N.v[p] = vv;
  N.nb[p] = th;
  if (l >= 0) write_packed_w(N.pk, N.t, l, i, o, th);
  if (N.target) {
    const float tg = fadd(fmul(th, s.tau), fmul(tg0, s.omt));
    N.target[p] = tg;
    if (l >= 0) write_packed_w(N.tpk, N.t, l, i, o, tg);
  }
}

// One workgroup per item: the 64-row chunks are dealt to the 4 waves (chunk ch to wave ch % 4),
// each chunk's partial is formed exactly as before and parked in LDS (part[ch]), and wave 0 sums
// them in chunk order and runs the Adam step: the same sums in the same order (bit-identical),
// with a quarter of the chunk loads and MFMAs on each wave.
constexpr int WA_MAXCH = 16;  // fused path: <= 1024 rows of 64
__device__ __forceinline__ void wgrad_adam_item(const AdamNet& N, int item, int l, const int32_t* __restrict__ step,
                                                int wave, int lane, float* tr, float* part) {
  const int g = lane >> 4, c = lane & 15;  // l: the item's layer, from the work list (no search)
  const int rem = item - N.ioff[l];
  const WgLayer& Ly = N.wg.l[l];
  const WgArgs& a = N.wg;
  CSTAMP(1);
  if (rem < Ly.IT * Ly.OT) {
    const int it = rem / Ly.OT, ot = rem - it * Ly.OT;
    const int oc = 16 * ot + c;
    // A full 16 x 16 tile runs Adam in the row layout: lane (g, c) owns W[16 it + c][16 ot + 4g + j],
    // 4 consecutive Keras-flat parameters (float4 loads / stores; the pkT block is this layout and
    // the pk block the MFMA's C layout, one LDS transpose away). Edge tiles: per element.
    const bool full = 16 * it + 16 <= Ly.in && 16 * ot + 16 <= Ly.out;
    const int pT = Ly.woff + (16 * it + c) * Ly.out + 16 * ot + 4 * g;
    // Adam operands of the lane's 4 parameters, in flight during the GEMM
    int p[4];
    float mm[4], vv[4], th[4], tg[4];
    bool ok[4];
    if (wave != 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) ok[q] = false, p[q] = 0, mm[q] = vv[q] = th[q] = tg[q] = 0.f;
    } else if (full) {
      const float4 m4 = *reinterpret_cast<const float4*>(N.m + pT), v4 = *reinterpret_cast<const float4*>(N.v + pT);
      const float4 t4 = *reinterpret_cast<const float4*>(N.src + pT);
      const float4 g4 = N.target ? *reinterpret_cast<const float4*>(N.target + pT) : make_float4(0.f, 0.f, 0.f, 0.f);
      mm[0] = m4.x, mm[1] = m4.y, mm[2] = m4.z, mm[3] = m4.w;
      vv[0] = v4.x, vv[1] = v4.y, vv[2] = v4.z, vv[3] = v4.w;
      th[0] = t4.x, th[1] = t4.y, th[2] = t4.z, th[3] = t4.w;
      tg[0] = g4.x, tg[1] = g4.y, tg[2] = g4.z, tg[3] = g4.w;
#pragma unroll
      for (int q = 0; q < 4; ++q) ok[q] = true, p[q] = pT + q;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ii = 16 * it + 4 * g + q;
        ok[q] = ii < Ly.in && oc < Ly.out;
        p[q] = ok[q] ? Ly.woff + ii * Ly.out + oc : 0;
        mm[q] = N.m[p[q]];
        vv[q] = N.v[p[q]];
        th[q] = N.src[p[q]];
        tg[q] = N.target ? N.target[p[q]] : 0.f;
      }
    }
    const float* ap = Ly.LT + (size_t)(16 * it + c) * a.ld + 4 * g;
    const float* bp = Ly.RT + (size_t)(16 * ot + c) * a.ld + 4 * g;
#ifdef CACTO_STAMPS
    {  // diagnostic: latency of a first touch of this tile's panel rows (chunk 0), then the real loop
      float4 t0 = *reinterpret_cast<const float4*>(ap + a.r_begin);
      float4 t1 = *reinterpret_cast<const float4*>(bp + a.r_begin);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (t0.x == 12345.f && t1.y == 54321.f) N.m[0] = 0.f;
    }
    CSTAMP(5);
#endif
    // this wave's chunks (ch = wave + 4 j), all their panel loads in flight together
    constexpr int CB = WA_MAXCH / 4;
    {
      float4 A[CB][4], Bv[CB][4];
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        const int ch = min(wave + 4 * j, a.nch - 1);
        const int lo = a.r_begin + ch * a.CH, hi = min(a.r_end, lo + a.CH);
        if (wave + 4 * j < a.nch) {
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int r = min(lo + 16 * w, hi - 16);  // clamped (branch-free); unused past hi
            A[j][w] = *reinterpret_cast<const float4*>(ap + r);
            Bv[j][w] = *reinterpret_cast<const float4*>(bp + r);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        const int ch = wave + 4 * j;
        if (ch < a.nch) {
          const int lo = a.r_begin + ch * a.CH, hi = min(a.r_end, lo + a.CH);
          floatx4 part4[4];
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            floatx4 acc = {0.f, 0.f, 0.f, 0.f};
            if (lo + 16 * w < hi) {
              acc = mfma4(A[j][w].x, Bv[j][w].x, acc);
              acc = mfma4(A[j][w].y, Bv[j][w].y, acc);
              acc = mfma4(A[j][w].z, Bv[j][w].z, acc);
              acc = mfma4(A[j][w].w, Bv[j][w].w, acc);
            }
            part4[w] = acc;
          }
          floatx4 s4 = part4[0];
#pragma unroll
          for (int w = 1; w < 4; ++w) {
            s4[0] += part4[w][0];
            s4[1] += part4[w][1];
            s4[2] += part4[w][2];
            s4[3] += part4[w][3];
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) part[ch * 256 + q * 64 + lane] = s4[q];
        }
      }
    }
    __syncthreads();
    if (wave != 0) return;
    floatx4 gs;
#pragma unroll
    for (int q = 0; q < 4; ++q) gs[q] = part[q * 64 + lane];
    for (int ch = 1; ch < a.nch; ++ch)
#pragma unroll
      for (int q = 0; q < 4; ++q) gs[q] += part[ch * 256 + q * 64 + lane];
    CSTAMP(2);
#ifdef CACTO_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // diagnostic: the GEMM's results landed
#endif
    CSTAMP(3);
    const AdamScalars s = adam_scalars(N.ad, step);  // after the loads are in flight
    if (full) {
      // gradient C layout -> row layout through the wave's LDS scratch (LDS operations of one wave
      // complete in order; the wave-scope fence keeps the compiler from reordering across lanes)
#pragma unroll
      for (int q = 0; q < 4; ++q) tr[(4 * g + q) * 16 + c] = gs[q];
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const float4 gT = *reinterpret_cast<const float4*>(tr + c * 16 + 4 * g);
      const float gv[4] = {gT.x, gT.y, gT.z, gT.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) adam_math(s, gv[j], mm[j], vv[j], th[j], tg[j]);
      *reinterpret_cast<float4*>(N.m + pT) = make_float4(mm[0], mm[1], mm[2], mm[3]);
      *reinterpret_cast<float4*>(N.v + pT) = make_float4(vv[0], vv[1], vv[2], vv[3]);
      const float4 th4 = make_float4(th[0], th[1], th[2], th[3]);
      *reinterpret_cast<float4*>(N.nb + pT) = th4;
      const NetTopo& t = N.t;
      const size_t bT = (size_t)(t.blocks + t.pkoff[l] + it * t.OT[l] + ot) * 64 + lane;  // pkT block (it, ot)
      const size_t bF = (size_t)(t.pkoff[l] + ot * t.KT[l] + it) * 64 + lane;             // pk block (ot, it)
      N.pk[bT] = th4;
      auto to_c = [&](const float (&v)[4]) {  // row layout -> C layout (the pk block)
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
        for (int j = 0; j < 4; ++j) tr[c * 16 + 4 * g + j] = v[j];
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = tr[(4 * g + q) * 16 + c];
        return make_float4(o[0], o[1], o[2], o[3]);
      };
      N.pk[bF] = to_c(th);
      if (N.target) {
        const float4 tg4 = make_float4(tg[0], tg[1], tg[2], tg[3]);
        *reinterpret_cast<float4*>(N.target + pT) = tg4;
        N.tpk[bT] = tg4;
        N.tpk[bF] = to_c(tg);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (ok[q]) adam_apply(N, s, p[q], gs[q], mm[q], vv[q], th[q], tg[q], l, 16 * it + 4 * g + q, oc);
    }
  } else {
    const int ot = rem - Ly.IT * Ly.OT;
    const int oc = 16 * ot + c;
    const bool ok = wave == 0 && g == 0 && oc < Ly.out;
    const int pp = ok ? Ly.boff + oc : 0;
    float mm = 0.f, vv = 0.f, th = 0.f, tg = 0.f;
    if (wave == 0) mm = N.m[pp], vv = N.v[pp], th = N.src[pp], tg = N.target ? N.target[pp] : 0.f;
    const float* bp = Ly.RT + (size_t)(16 * min(ot, Ly.OT - 1) + c) * a.ld + 4 * g;
    // per chunk: its (<= 4) 16-row steps from max(lo, bias_r0), summed in row order from 0 — the
    // sequence k_wgrad's 64-row groups and 16-row tail produce — then the shuffles over g; chunks
    // dealt to the waves as for the weight tiles, summed in chunk order by wave 0
    constexpr int CB = WA_MAXCH / 4;
    {
      float4 v4[CB][4];
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        const int ch = min(wave + 4 * j, a.nch - 1);
        const int lo = a.r_begin + ch * a.CH, hi = min(a.r_end, lo + a.CH);
        const int r0 = max(lo, a.bias_r0);
        if (wave + 4 * j < a.nch)
#pragma unroll
          for (int k = 0; k < 4; ++k) v4[j][k] = *reinterpret_cast<const float4*>(bp + max(0, min(r0 + 16 * k, hi - 16)));
      }
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        const int ch = wave + 4 * j;
        if (ch < a.nch) {
          const int lo = a.r_begin + ch * a.CH, hi = min(a.r_end, lo + a.CH);
          const int r0 = max(lo, a.bias_r0);
          float sb = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (r0 + 16 * k < hi) sb += (v4[j][k].x + v4[j][k].y) + (v4[j][k].z + v4[j][k].w);
          sb += __shfl_xor(sb, 16);
          sb += __shfl_xor(sb, 32);
          part[ch * 256 + lane] = sb;
        }
      }
    }
    __syncthreads();
    if (wave != 0) return;
    float gsum = part[lane];
    for (int ch = 1; ch < a.nch; ++ch) gsum = gsum + part[ch * 256 + lane];
    const AdamScalars s = adam_scalars(N.ad, step);
    if (ok) adam_apply(N, s, pp, gsum, mm, vv, th, tg, -1, 0, 0);
  }
}

// One or two networks (the paired update runs the critic of update t and the actor of t - 1).
// Work list: workgroup b runs on XCD b % 8 (the dispatcher's round robin; used for locality only,
// nothing depends on it) and takes one item of that XCD's bin (its 4 waves split the item's row chunks). The bins group the tiles of a layer
// into blocks of in-tiles x out-tiles, so each XCD's L2 fetches a panel slice once for several
// tiles instead of every XCD fetching every slice from the memory-side cache.
__global__ void __launch_bounds__(256) k_wgrad_adam(AdamNet n0, AdamNet n1, const int32_t* __restrict__ items,
                                                    int stride, const int32_t* step) {
  CSTAMP(0);
  // the item is wave-uniform: readfirstlane lets the compiler keep the network descriptor in
  // scalar registers (s_load from the kernel arguments) instead of chasing it through VGPR pointers
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int code = __builtin_amdgcn_readfirstlane(items[(blockIdx.x & 7) * stride + (blockIdx.x >> 3)]);
  __shared__ float tr[256];                    // wave 0: one 16 x 16 transpose
  __shared__ float part[WA_MAXCH * 256];       // per-chunk partial sums
  if (code >= 0) {
    const int l = (code >> 16) & 0xf;
    if (((code >> 15) & 1) == 0) wgrad_adam_item(n0, code & 0x7fff, l, step, wave, lane, tr, part);
    else wgrad_adam_item(n1, code & 0x7fff, l, step, wave, lane, tr, part);
  }
  CSTAMP(4);
#ifdef CACTO_STAMPS
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int k_ = 0; k_ < 6; ++k_) g_cstamps[k_] = cacto_stamp_s[k_];
#endif
}

}  // namespace cacto

#ifdef CACTO_STAMPS
extern "C" int cacto_debug_critic_stamps(unsigned long long* out_h) {
  CACTO_CHECK_HIP(hipDeviceSynchronize());
  CACTO_CHECK_HIP(hipMemcpyFromSymbol(out_h, HIP_SYMBOL(g_cstamps), sizeof(unsigned long long) * 32));
  return CACTO_OK;
}
extern "C" int cacto_debug_actor_stamps(unsigned long long* out_h) {
  CACTO_CHECK_HIP(hipDeviceSynchronize());
  CACTO_CHECK_HIP(hipMemcpyFromSymbol(out_h, HIP_SYMBOL(g_astamps), sizeof(unsigned long long) * 32));
  return CACTO_OK;
}
#endif

using namespace cacto;

namespace {

// Samples per chain workgroup: 4-sample tiles (chain_q4.h) up to a padded batch of Q4_MAX_BP, so a
// reference-size batch (64 / 128) spreads over 4x the workgroups; 16-sample tiles above. A function
// of the batch only, so every update path of one batch size runs the same chain kernels
// (bit-identical results). CACTO_Q4_MAX_BP overrides the bound (read once; benchmarks).
inline int q4_max_bp() {
  static const int v = [] {
    const char* e = std::getenv("CACTO_Q4_MAX_BP");
    return e ? std::atoi(e) : 512;
  }();
  return v;
}
inline int chain_tile(int Bp) { return Bp <= q4_max_bp() ? Q4_TILE : CACTO_TILE; }
inline int cu_count() {
  static const int cus = [] {
    int dev = 0, v = 0;
    return (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
               ? v
               : 256;
  }();
  return cus;
}
template <int NJ>
struct LaunchActorChain {
  static int run(const cacto_sys* sys, NetView Ac, NetView C, ChainScalars cs, const double* storage,
                 const int32_t* idx, int B, GradBufs gb, int32_t* step, hipStream_t st) {
    const int Bp = (B + 15) / 16 * 16;
    if (chain_tile(Bp) == Q4_TILE)
      hipLaunchKernelGGL(k_actor_grad_q4<NJ>, dim3(Bp / Q4_TILE), dim3(Q4_THREADS), 0, st, sys->dev, Ac, C, cs,
                         storage, idx, B, gb, step);
    else
      hipLaunchKernelGGL(k_actor_grad<NJ>, dim3(Bp / 16), dim3(CACTO_THREADS), 0, st, sys->dev, Ac, C, cs, storage, idx,
                         B, gb, step);
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
};

// nct: critic tiles (= actor tiles) of the batch's chain tile size
// XCDs the paired q4 grid of 2 nct tiles runs on (k_chain_pair_q4): about 8 tiles per XCD, at
// most all 8 XCDs. Measured (updates/s, 1 MI355X): manipulator B = 64 (32 tiles) on 8 XCDs 33.4 k,
// on 4 36.2 k; UR5 B = 64 24.3 k / 29.1 k; DI B = 128 (64 tiles) on 8 39.4 k, on 4 38.3 k.
// CACTO_PAIR_XCDS (1, 2, 4 or 8) overrides it (read once; benchmarks).
inline int pair_xcds(int nct) {
  static const int forced = [] {
    const char* e = std::getenv("CACTO_PAIR_XCDS");
    const int v = e ? std::atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4 || v == 8) ? v : 0;
  }();
  if (forced) return forced;
  int nx = 1;
  while (nx < 8 && 2 * nct > 8 * nx) nx *= 2;
  return nx;
}

template <int NJ>
struct LaunchChainPair {
  static int run(const cacto_sys* sys, NetView C, NetView Tg, NetView Ac, ChainScalars cs, const double* storage,
                 const int32_t* idx_c, const float* isw, const int32_t* idx_a, int B, GradBufs gbc, GradBufs gba,
                 float* y, float* V, int32_t* step, hipStream_t st) {
    const int Bp = gbc.Bp;
    if (chain_tile(Bp) == Q4_TILE) {
      const int nct = Bp / Q4_TILE;
      const int nx = pair_xcds(nct);
      hipLaunchKernelGGL(k_chain_pair_q4<NJ>, dim3(8 * ceil_div(2 * nct, nx)), dim3(Q4_THREADS), 0, st, sys->dev, C,
                         Tg, Ac, cs, storage, idx_c, isw, idx_a, B, nct, gbc, gba, y, V, step, nx);
    } else {
      const int nct = Bp / CACTO_TILE;
      hipLaunchKernelGGL(k_chain_pair<NJ>, dim3(2 * nct), dim3(CACTO_THREADS), 0, st, sys->dev, C, Tg, Ac, cs,
                         storage, idx_c, isw, idx_a, B, nct, gbc, gba, y, V, step);
    }
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
};

// Rows per weight-gradient chunk (one slab each): small batches use short chunks so the grid
// still fills the chip; large ones long chunks so Adam sums few slabs.
// Row chunk of the split-K weight-gradient GEMM. CACTO_WG_CHUNK overrides it above 1024 rows
// (read once; benchmarks) — the fused small-batch path always takes 64-row chunks.
inline int wg_chunk_big() {
  static const int v = [] {
    const char* e = std::getenv("CACTO_WG_CHUNK");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}
// Row chunk of the weight-gradient GEMM. From 4096 rows on 256-row chunks: k_wgrad_big walks a whole
// chunk per wave, so longer chunks amortise its pipeline fill (r05, updates/s: DI B = 4096 — the actor's
// 4096 rows — 12.97 k at 128 rows, 13.25 k at 256; car_park PER B = 4096 10.14 k / 9.86 k; 512 rows
// 12.49 k); CACTO_WG_CHUNK overrides it above 1024 rows (read once; benchmarks).
inline int wg_chunk(int rows) {
  if (rows > 1024 && wg_chunk_big() > 0) return wg_chunk_big();
  return rows <= 1024 ? 64 : rows < 4096 ? 128 : 256;
}

struct Workspace {
  GradBufs crit, act;
  float* slab;    // critic weight-gradient slabs
  float* slab_a;  // actor's (a separate region: cacto_update_n overlaps the two steps)
  float* cshadow; // two more critic net buffers (cacto_update_n rotates the critic over three)
  int32_t* pidx;  // cacto_update_n_per: sampled indices, a ring of five buffers of Bp
  float* pisw;    // and the IS weights of the current update
  int32_t* runs;  // the overlapped PER loop's per-subtree sample runs (2 x PER_RUN_SUB ints)
  float* scal;  // y, V, Vt scratch (3 * Bp)
  size_t bytes;
  int Bp;
};

inline size_t align64(size_t n) { return (n + 63) / 64 * 64; }

Workspace plan(const cacto_sys* sys, int B, char* base) {
  Workspace w{};
  const int Bp = (B + 15) / 16 * 16;
  w.Bp = Bp;
  const NetTopo& tc = sys->critic;
  const NetTopo& ta = sys->actor;
  size_t off = 0;
  float* f = reinterpret_cast<float*>(base);
  // critic panels (ld = 2Bp)
  w.crit.ld = 2 * Bp;
  w.crit.Bp = Bp;
  size_t coff = 0;
  for (int l = 0; l < tc.L; ++l) {
    w.crit.LT[l] = f ? f + coff : nullptr;
    coff += (size_t)16 * tc.KT[l] * w.crit.ld;
    w.crit.RT[l] = f ? f + coff : nullptr;
    coff += (size_t)16 * tc.OT[l] * w.crit.ld;
  }
  w.act.ld = Bp;
  w.act.Bp = Bp;
  size_t aoff = align64(coff);  // the actor panels follow the critic's (no aliasing, see slab_a)
  for (int l = 0; l < ta.L; ++l) {
    w.act.LT[l] = f ? f + aoff : nullptr;
    aoff += (size_t)16 * ta.KT[l] * w.act.ld;
    w.act.RT[l] = f ? f + aoff : nullptr;
    aoff += (size_t)16 * ta.OT[l] * w.act.ld;
  }
  off = align64(aoff);
  const int nch_a = ceil_div(Bp, wg_chunk(Bp));
  const int nch_c = ceil_div(2 * Bp, wg_chunk(2 * Bp));  // Sobolev rows, or the plain half
  w.slab = f ? f + off : nullptr;
  off += align64((size_t)nch_c * tc.params);
  w.slab_a = f ? f + off : nullptr;
  off += align64((size_t)nch_a * ta.params);
  w.cshadow = f ? f + off : nullptr;
  off += 2 * align64((size_t)flat_span(tc) + (size_t)2 * tc.blocks * 256);
  w.pidx = f ? reinterpret_cast<int32_t*>(f + off) : nullptr;
  off += align64((size_t)5 * Bp);
  w.pisw = f ? f + off : nullptr;
  off += align64((size_t)Bp);
  w.runs = f ? reinterpret_cast<int32_t*>(f + off) : nullptr;
  off += align64((size_t)2 * PER_RUN_SUB);
  w.scal = f ? f + off : nullptr;
  off += align64((size_t)3 * Bp);
  w.bytes = off * sizeof(float);
  return w;
}

WgArgs wg_args(const NetTopo& t, const GradBufs& gb, int r_begin, int r_end, int bias_r0) {
  WgArgs a{};
  a.nl = t.L;
  a.ld = gb.ld;
  a.r_begin = r_begin;
  a.r_end = r_end;
  a.bias_r0 = bias_r0;
  a.CH = wg_chunk(r_end - r_begin);
  a.nch = ceil_div(r_end - r_begin, a.CH);
  a.P = t.params;
  int tpc = 0;  // workgroups per chunk: 4x4 tile blocks + groups of 4 bias tiles, per layer
  for (int l = 0; l < t.L; ++l) {
    a.l[l] = WgLayer{gb.LT[l], gb.RT[l], t.in[l], t.out[l], t.KT[l], t.OT[l], t.woff[l], t.boff[l]};
    a.toff[l] = tpc;
    tpc += ceil_div(t.KT[l], WG_BLK) * ceil_div(t.OT[l], WG_BLK) + ceil_div(t.OT[l], WG_BLK);
  }
  a.toff[t.L] = tpc;
  a.tpc = tpc;
  // items by decreasing work: 4 x 4 tile blocks, then edge blocks, then bias groups (stable)
  std::vector<std::pair<int, int>> cost;
  for (int l = 0; l < t.L; ++l) {
    const int nbi = ceil_div(t.KT[l], WG_BLK), nbo = ceil_div(t.OT[l], WG_BLK);
    for (int k = 0; k < nbi * nbo; ++k) {
      const int ni = std::min(WG_BLK, t.KT[l] - (k / nbo) * WG_BLK), no = std::min(WG_BLK, t.OT[l] - (k % nbo) * WG_BLK);
      cost.push_back({-ni * no, a.toff[l] + k});
    }
    for (int k = 0; k < nbo; ++k) cost.push_back({0, a.toff[l] + nbi * nbo + k});
  }
  std::stable_sort(cost.begin(), cost.end(), [](const std::pair<int, int>& x, const std::pair<int, int>& y) {
    return x.first < y.first;
  });
  static const bool perm_on = [] {  // CACTO_WG_PERM=0: chunk-major item order (A/B; read once)
    const char* e = std::getenv("CACTO_WG_PERM");
    return !(e && e[0] == '0');
  }();
  for (int k = 0; k < 64; ++k) a.perm[k] = k < tpc ? (unsigned char)(perm_on ? cost[k].second : k) : 0;
  return a;
}

// k_wgrad_big for more than 1024 gradient rows (B > 512 for the actor, the critic's two halves), when
// every 4 x 4 tile block of the network is 4 x 4, 1 x 4 or 4 x 1 tiles (all the configs' networks).
// A function of the network and the row count only, so every path of one batch size takes the same
// kernel. CACTO_WG_BIG=0 keeps k_wgrad (A/B; read once).
bool wgrad_big(const NetTopo& t, int rows) {
  static const bool env_on = [] {
    const char* e = std::getenv("CACTO_WG_BIG");
    return !(e && e[0] == '0');
  }();
  if (!env_on || rows <= 1024) return false;
  for (int l = 0; l < t.L; ++l)
    for (int i0 = 0; i0 < t.KT[l]; i0 += WG_BLK)
      for (int o0 = 0; o0 < t.OT[l]; o0 += WG_BLK) {
        const int ni = std::min(WG_BLK, t.KT[l] - i0), no = std::min(WG_BLK, t.OT[l] - o0);
        if (!((ni == 4 && (no == 4 || no == 1)) || (ni == 1 && no == 4))) return false;
      }
  return true;
}

// the weight-gradient GEMM of one network into its slabs; returns the chunk count k_adam sums
int launch_wgrad(const NetTopo& t, const GradBufs& gb, int r_begin, int r_end, int bias_r0, float* slab,
                 hipStream_t st, int* nch, unsigned long long* sig_p = nullptr, unsigned long long sig_v = 0,
                 const PerRunArgs* per_run = nullptr) {
  const WgArgs a = wg_args(t, gb, r_begin, r_end, bias_r0);
  // chunks grouped by XCD from 8 chunks on (CACTO_WG_XCD=0 / 1 forces it off / on; benchmarks)
  static const int forced = [] {
    const char* e = std::getenv("CACTO_WG_XCD");
    return e ? std::atoi(e) : -1;
  }();
  const int xcd = forced >= 0 ? forced : a.nch >= 8;
  const int grid = xcd ? 8 * ceil_div(a.nch, 8) * a.tpc : a.nch * a.tpc;
  // k_wgrad_big's load lead in 16-row steps: 3, or 6 with CACTO_WGB_AHEAD=6 (same sums). Measured
  // (updates/s, two runs each): DI B = 4096 13.41 / 13.38 k at 6 against 13.33 / 13.37 k at 3,
  // manipulator B = 8192 8.29 / 8.26 k against 8.36 / 8.34 k — inside the pipeline the GEMM is not
  // waiting on its loads, so the lighter form stays.
  static const int ahead = [] {
    const char* e = std::getenv("CACTO_WGB_AHEAD");
    return e && std::atoi(e) == 6 ? 6 : 3;
  }();
  if (per_run) {  // the PER loop's fused form (the caller checked wgrad_big and the tree's shape)
    const int nroot = (int)(per_run->cap / PER_RUN_SUB);
    if (ahead == 3)
      hipLaunchKernelGGL(k_wgrad_big_per<3>, dim3(grid + nroot), dim3(256), 0, st, a, slab, xcd, grid, *per_run, nroot);
    else
      hipLaunchKernelGGL(k_wgrad_big_per<6>, dim3(grid + nroot), dim3(256), 0, st, a, slab, xcd, grid, *per_run, nroot);
  } else if (wgrad_big(t, r_end - r_begin)) {
    if (ahead == 3)
      hipLaunchKernelGGL(k_wgrad_big<3>, dim3(grid), dim3(256), 0, st, a, slab, xcd, sig_p, sig_v);
    else
      hipLaunchKernelGGL(k_wgrad_big<6>, dim3(grid), dim3(256), 0, st, a, slab, xcd, sig_p, sig_v);
  }
  else
    hipLaunchKernelGGL(k_wgrad, dim3(grid), dim3(256), 0, st, a, slab, xcd, sig_p, sig_v);
  CACTO_CHECK_HIP(hipGetLastError());
  *nch = a.nch;
  return CACTO_OK;
}

ChainScalars chain_scalars(const cacto_update_cfg* cfg, int B) {
  ChainScalars cs;
  cs.w_S = (float)cfg->w_S;
  cs.MC = cfg->MC;
  cs.B_global = cfg->B_global > 0 ? cfg->B_global : B;
  cs.want_vt = cfg->want_target_V;
  cs.wait_p = nullptr;
  cs.wait_v = 0;
  cs.wait_at_start = 0;
  // CACTO_CHAIN_XCD=0 keeps the tiles in block order (A/B; read once)
  static const bool xcd_env = [] {
    const char* e = std::getenv("CACTO_CHAIN_XCD");
    return !(e && e[0] == '0');
  }();
  const int Bp = (B + 15) / 16 * 16;
  cs.xcd_tiles = xcd_env && (Bp / CACTO_TILE) % 128 == 0 && wg_chunk(Bp) == 256 && wg_chunk(2 * Bp) == 256;
  return cs;
}

AdamArgs adam_args(const cacto_update_cfg* cfg, int which, int soft) {
  AdamArgs a{};
  a.beta1 = cfg->beta1;
  a.beta2 = cfg->beta2;
  a.eps = cfg->epsilon;
  a.tau = cfg->tau;
  const double* lr = which == CACTO_NET_CRITIC ? cfg->critic_lr : cfg->actor_lr;
  for (int k = 0; k < 5; ++k) a.lr[k] = lr[k];
  for (int k = 0; k < 4; ++k) a.bounds[k] = cfg->lr_bounds[k];
  a.which = which == CACTO_NET_CRITIC ? 0 : 1;
  a.soft = soft;
  return a;
}

int check_nets(const cacto_nets* n) {
  CACTO_REQUIRE(n && n->actor_d && n->actor_m_d && n->actor_v_d && n->critic_d && n->critic_m_d && n->critic_v_d &&
                    n->target_d && n->step_d,
                "cacto_nets: null member");
  return CACTO_OK;
}

int launch_critic_chain(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                        const double* storage, const int32_t* idx, const float* isw, int B, float* y, float* V,
                        float* Vt, const Workspace& w, hipStream_t st) {
  NetView C = cacto_make_view(sys, CACTO_NET_CRITIC, nets->critic_d);
  NetView Tg = cacto_make_view(sys, CACTO_NET_CRITIC, nets->target_d);
  const ChainScalars cs = chain_scalars(cfg, B);
  float* yb = y ? y : w.scal;
  float* Vb = V ? V : w.scal + w.Bp;
  float* Vtb = Vt ? Vt : w.scal + 2 * w.Bp;
  if (chain_tile(w.Bp) == Q4_TILE)
    hipLaunchKernelGGL(k_critic_grad_q4, dim3(w.Bp / Q4_TILE), dim3(Q4_THREADS), 0, st, sys->dev, C, Tg, cs,
                       storage, idx, isw, B, w.crit, yb, Vb, Vtb, nets->step_d);
  else
    hipLaunchKernelGGL(k_critic_grad, dim3(w.Bp / 16), dim3(CACTO_THREADS), 0, st, sys->dev, C, Tg, cs, storage, idx,
                       isw, B, w.crit, yb, Vb, Vtb, nets->step_d);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

int launch_critic_chain_and_wgrad(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                                  const double* storage, const int32_t* idx, const float* isw, int B, float* y,
                                  float* V, float* Vt, const Workspace& w, hipStream_t st, int* nch_out) {
  if (int e = launch_critic_chain(sys, nets, cfg, storage, idx, isw, B, y, V, Vt, w, st)) return e;
  const ChainScalars cs = chain_scalars(cfg, B);
  const bool sob = cs.w_S != 0.f;
  return launch_wgrad(sys->critic, w.crit, sob ? 0 : w.Bp, 2 * w.Bp, w.Bp, w.slab, st, nch_out);
}

int launch_actor_chain(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                       const double* storage, const int32_t* idx, int B, const Workspace& w, hipStream_t st,
                       const unsigned long long* wait_p = nullptr, unsigned long long wait_v = 0,
                       int wait_at_start = 0) {
  NetView Ac = cacto_make_view(sys, CACTO_NET_ACTOR, nets->actor_d);
  NetView C = cacto_make_view(sys, CACTO_NET_CRITIC, nets->critic_d);
  ChainScalars cs = chain_scalars(cfg, B);
  cs.wait_p = wait_p;
  cs.wait_v = wait_v;
  cs.wait_at_start = wait_at_start;
  return dispatch_nj<LaunchActorChain>(sys->host.p, sys, Ac, C, cs, storage, idx, B, w.act, nets->step_d, st);
}

int launch_actor_chain_and_wgrad(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                                 const double* storage, const int32_t* idx, int B, const Workspace& w, hipStream_t st,
                                 int* nch_out) {
  if (int e = launch_actor_chain(sys, nets, cfg, storage, idx, B, w, st)) return e;
  return launch_wgrad(sys->actor, w.act, 0, w.Bp, 0, w.slab_a, st, nch_out);
}

// src: the weights the step starts from (nullptr = in place; cacto_update_n steps the critic from one
// buffer into the other)
int launch_adam(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg, int which,
                const float* slab, int nch, int soft, hipStream_t st, const float* src = nullptr,
                const unsigned long long* wait_p = nullptr, unsigned long long wait_v = 0,
                unsigned long long* sig_p = nullptr, unsigned long long sig_v = 0,
                const PerSampleArgs* sample = nullptr, int thru = 0) {
  const NetTopo& t = topo(sys, which);
  float* nb = which == CACTO_NET_CRITIC ? nets->critic_d : nets->actor_d;
  float* m = which == CACTO_NET_CRITIC ? nets->critic_m_d : nets->actor_m_d;
  float* v = which == CACTO_NET_CRITIC ? nets->critic_v_d : nets->actor_v_d;
  float4* pk = reinterpret_cast<float4*>(nb + flat_span(t));
  float4* tpk = reinterpret_cast<float4*>(nets->target_d + flat_span(t));
  const AdamArgs aa = adam_args(cfg, which, soft && which == CACTO_NET_CRITIC);
  const float* s0 = src ? src : nb;
  // one parameter per thread with all chunk partials in flight (k_adam<NCH>), else the looped kernel
  const int full = (t.params + 255) / 256;
  auto go = [&](auto kern, int grid) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, slab, nch, t, s0, nb, pk, m, v, nets->step_d, aa,
                       nets->target_d, tpk, wait_p, wait_v, sig_p, sig_v, thru);
  };
  if (sample) {  // the PER loop's fused form (the caller checked nch <= 64)
    if ((sig_p && !thru) || nch > 64) {
      set_error("k_adam_sample: a publishing Adam writes through; at most 64 chunks");
      return CACTO_EINVAL;
    }
    const int ns = (sample->B + 255) / 256;
    auto gs = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(full + ns), dim3(256), 0, st, slab, nch, t, s0, nb, pk, m, v, nets->step_d, aa,
                         nets->target_d, tpk, wait_p, wait_v, full, *sample, sig_p, sig_v, thru);
    };
    if (nch <= 8) gs(k_adam_sample<8>);
    else if (nch <= 16) gs(k_adam_sample<16>);
    else if (nch <= 32) gs(k_adam_sample<32>);
    else gs(k_adam_sample<64>);
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
  if (nch <= 8) go(k_adam<8>, full);
  else if (nch <= 16) go(k_adam<16>, full);
  else if (nch <= 32) go(k_adam<32>, full);
  else if (nch <= 64) go(k_adam<64>, full);
  else go(k_adam<0>, std::min(full, 1024));
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

// The fused weight-gradient + Adam launch serves batches whose gradient rows (critic: 2 Bp with the
// Sobolev half, actor: Bp) all fall in 64-row chunks; larger batches keep k_wgrad's split-K slabs
// (many workgroups per tile) and k_adam. A function of B only, so every update path of one batch
// size takes the same kernels (bit-identical results).
inline bool fused_adam(int Bp) { return 2 * Bp <= 1024; }

AdamNet adam_net(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg, int which, const GradBufs& gb,
                 int r_begin, int r_end, int bias_r0, int soft, const float* src, float* nb) {
  AdamNet n{};
  const NetTopo& t = topo(sys, which);
  n.wg = wg_args(t, gb, r_begin, r_end, bias_r0);
  n.t = t;
  n.nb = nb;
  n.src = src ? src : nb;
  n.pk = reinterpret_cast<float4*>(nb + flat_span(t));
  n.m = which == CACTO_NET_CRITIC ? nets->critic_m_d : nets->actor_m_d;
  n.v = which == CACTO_NET_CRITIC ? nets->critic_v_d : nets->actor_v_d;
  const bool sft = soft && which == CACTO_NET_CRITIC;
  n.target = sft ? nets->target_d : nullptr;
  n.tpk = sft ? reinterpret_cast<float4*>(nets->target_d + flat_span(t)) : nullptr;
  n.ad = adam_args(cfg, which, sft);
  int items = 0;
  for (int l = 0; l < t.L; ++l) {
    n.ioff[l] = items;
    items += t.KT[l] * t.OT[l] + t.OT[l];
  }
  n.ioff[t.L] = items;
  for (int l = t.L + 1; l <= MAX_LAYERS; ++l) n.ioff[l] = items;
  n.items = items;
  return n;
}

AdamNet critic_adam_net(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg, const Workspace& w,
                        int soft, const float* src, float* nb) {
  const bool sob = cfg->w_S != 0.0;
  return adam_net(sys, nets, cfg, CACTO_NET_CRITIC, w.crit, sob ? 0 : w.Bp, 2 * w.Bp, w.Bp, soft, src, nb);
}

AdamNet actor_adam_net(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg, const Workspace& w) {
  return adam_net(sys, nets, cfg, CACTO_NET_ACTOR, w.act, 0, w.Bp, 0, 0, nullptr, nets->actor_d);
}

// mode 0: critic alone (n0), 1: actor alone (n0), 2: critic (n0) and actor (n1)
int launch_wgrad_adam(const cacto_sys* sys, int mode, const AdamNet& n0, const AdamNet* n1, const int32_t* step,
                      hipStream_t st) {
  const int stride = sys->wa_stride[mode];
  // one item per workgroup (the 4 waves split its chunks); fused_adam keeps every row set within
  // WA_MAXCH chunks of 64
  if (n0.wg.nch > WA_MAXCH || (n1 && n1->wg.nch > WA_MAXCH)) {
    set_error("k_wgrad_adam: more than WA_MAXCH row chunks");
    return CACTO_EINVAL;
  }
  hipLaunchKernelGGL(k_wgrad_adam, dim3(8 * stride), dim3(256), 0, st, n0, n1 ? *n1 : n0, sys->wa_items[mode],
                     stride, step);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

// critic step after its chain: GEMM + Adam (+ soft update) from src into nb
int critic_step_tail(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg, const Workspace& w,
                     hipStream_t st, const float* src, float* nb, const unsigned long long* wait_p = nullptr,
                     unsigned long long wait_v = 0, unsigned long long* sig_p = nullptr, unsigned long long sig_v = 0,
                     const PerRunArgs* per_run = nullptr, const PerSampleArgs* sample = nullptr, int thru = 0) {
  const int soft = cfg->MC ? 0 : 1;
  if (fused_adam(w.Bp)) return launch_wgrad_adam(sys, 0, critic_adam_net(sys, nets, cfg, w, soft, src, nb), nullptr,
                                                 nets->step_d, st);
  const bool sob = cfg->w_S != 0.0;
  int nch = 0;
  if (int e = launch_wgrad(sys->critic, w.crit, sob ? 0 : w.Bp, 2 * w.Bp, w.Bp, w.slab, st, &nch, nullptr, 0, per_run))
    return e;
  cacto_nets dst = *nets;
  dst.critic_d = nb;
  return launch_adam(sys, &dst, cfg, CACTO_NET_CRITIC, w.slab, nch, soft, st, src, wait_p, wait_v, sig_p, sig_v,
                     sample, thru);
}

// CACTO_PER_OVERLAP (default 1): the pipelined PER loop's priority update and next sample share the
// critic GEMM's and Adam's launches (k_wgrad_big_per, k_adam_sample) instead of following them.
bool per_overlap_on() {
  static const bool v = [] {
    const char* e = std::getenv("CACTO_PER_OVERLAP");
    return !(e && e[0] == '0');
  }();
  return v;
}


int actor_step_tail(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg, const Workspace& w,
                    hipStream_t st, unsigned long long* sig_p = nullptr, unsigned long long sig_v = 0) {
  if (fused_adam(w.Bp)) return launch_wgrad_adam(sys, 1, actor_adam_net(sys, nets, cfg, w), nullptr, nets->step_d, st);
  int nch = 0;
  if (int e = launch_wgrad(sys->actor, w.act, 0, w.Bp, 0, w.slab_a, st, &nch, sig_p, sig_v)) return e;
  return launch_adam(sys, nets, cfg, CACTO_NET_ACTOR, w.slab_a, nch, 0, st);
}

}  // namespace

// k_wgrad_adam's XCD bins (see the kernel). Per layer the IT x OT weight tiles are cut into bi x bo
// = 8 blocks (bi chosen so the blocks are as square as the tile grid allows), block k to bin k; a
// layer's bias tiles go to the bin of their out-tile block. Item numbering is AdamNet's (per layer:
// IT * OT weight tiles, row-major in (it, ot), then OT bias tiles).
// Code: bits 0-14 the item, bit 15 the network (n1 of the paired launch), bits 16-19 the layer
// (so the kernel does not search AdamNet::ioff with dependent scalar loads); -1 = no item.
int cacto_build_wgrad_adam_items(cacto_sys* sys) {
  std::vector<int32_t> bins[3][8];
  const NetTopo* nets[2] = {&sys->critic, &sys->actor};
  for (int mode = 0; mode < 3; ++mode) {
    for (int n = 0; n < 2; ++n) {
      if ((mode == 0 && n == 1) || (mode == 1 && n == 0)) continue;
      const int tag = (mode == 2 && n == 1) ? 1 : 0;  // n1 in the paired launch
      const NetTopo& t = *nets[n];
      int base = 0;
      for (int l = 0; l < t.L; ++l) {
        const int IT = t.KT[l], OT = t.OT[l];
        // bi x bo = 8 with the blocks (IT/bi) x (OT/bo) closest to square; both within the grid
        int bi = 1;
        double best = 1e30;
        for (int c = 1; c <= 8; c *= 2) {
          if (c > IT || 8 / c > OT) continue;
          const double d = std::abs((double)IT / c - (double)OT / (8 / c));
          if (d < best) best = d, bi = c;
        }
        if (best == 1e30) bi = std::max(1, std::min(IT, 8));  // grid smaller than 8 blocks
        const int bo = std::max(1, 8 / bi);
        for (int it = 0; it < IT; ++it)
          for (int ot = 0; ot < OT; ++ot) {
            const int bin = ((it * bi) / IT) * bo + std::min(bo - 1, (ot * bo) / OT);
            bins[mode][bin % 8].push_back((l << 16) | (tag << 15) | (base + it * OT + ot));
          }
        for (int ot = 0; ot < OT; ++ot) {
          const int bin = std::min(bo - 1, (ot * bo) / OT);
          bins[mode][bin % 8].push_back((l << 16) | (tag << 15) | (base + IT * OT + ot));
        }
        base += IT * OT + OT;
      }
    }
    size_t S = 4;
    for (auto& b : bins[mode]) S = std::max(S, (b.size() + 3) / 4 * 4);
    std::vector<int32_t> flat(8 * S, -1);
    for (int x = 0; x < 8; ++x)
      for (size_t k = 0; k < bins[mode][x].size(); ++k) flat[x * S + k] = bins[mode][x][k];
    CACTO_CHECK_HIP(hipMalloc(&sys->wa_items[mode], flat.size() * sizeof(int32_t)));
    CACTO_CHECK_HIP(hipMemcpy(sys->wa_items[mode], flat.data(), flat.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    sys->wa_stride[mode] = (int)S;
  }
  return CACTO_OK;
}

extern "C" size_t cacto_workspace_bytes(const cacto_sys* sys, int B) {
  if (!sys || B <= 0) return 0;
  return plan(sys, B, nullptr).bytes;
}

#define CHECK_WS(ws, nbytes, B)                                                                   \
  CACTO_REQUIRE((ws) != nullptr && (nbytes) >= plan(sys, (B), nullptr).bytes,                     \
                "workspace too small: query cacto_workspace_bytes(sys, B)");                      \
  CACTO_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 255) == 0, "workspace must be 256-byte aligned")

extern "C" int cacto_critic_grad(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                                 const double* storage_d, const int32_t* idx_d, const float* is_w_d, int B,
                                 float* grad_d, float* y_d, float* V_d, float* Vt_d, void* workspace_d,
                                 size_t workspace_bytes, void* stream) {
  CACTO_REQUIRE(sys && cfg && storage_d && idx_d && grad_d && B > 0, "cacto_critic_grad: bad arguments");
  if (int e = check_nets(nets)) return e;
  CHECK_WS(workspace_d, workspace_bytes, B);
  const Workspace w = plan(sys, B, static_cast<char*>(workspace_d));
  hipStream_t st = as_stream(stream);
  int nch = 0;
  if (int e = launch_critic_chain_and_wgrad(sys, nets, cfg, storage_d, idx_d, is_w_d, B, y_d, V_d, Vt_d, w, st, &nch))
    return e;
  const int P = sys->critic.params;
  if (int e = launch_reduce(w.slab, nch, P, grad_d, st)) return e;
  return CACTO_OK;
}

extern "C" int cacto_actor_grad(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                                const double* storage_d, const int32_t* idx_d, int B, float* grad_d, void* workspace_d,
                                size_t workspace_bytes, void* stream) {
  CACTO_REQUIRE(sys && cfg && storage_d && idx_d && grad_d && B > 0, "cacto_actor_grad: bad arguments");
  if (int e = check_nets(nets)) return e;
  CHECK_WS(workspace_d, workspace_bytes, B);
  const Workspace w = plan(sys, B, static_cast<char*>(workspace_d));
  hipStream_t st = as_stream(stream);
  int nch = 0;
  if (int e = launch_actor_chain_and_wgrad(sys, nets, cfg, storage_d, idx_d, B, w, st, &nch)) return e;
  const int P = sys->actor.params;
  if (int e = launch_reduce(w.slab_a, nch, P, grad_d, st)) return e;
  return CACTO_OK;
}

extern "C" int cacto_adam_step(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg, int which,
                               const float* grad_d, int soft_update, void* stream) {
  CACTO_REQUIRE(sys && cfg && grad_d && (which == CACTO_NET_ACTOR || which == CACTO_NET_CRITIC),
                "cacto_adam_step: bad arguments");
  if (int e = check_nets(nets)) return e;
  return launch_adam(sys, nets, cfg, which, grad_d, 1, soft_update, as_stream(stream));
}

extern "C" int cacto_soft_update(const cacto_sys* sys, const cacto_nets* nets, float tau, void* stream) {
  CACTO_REQUIRE(sys, "cacto_soft_update: bad arguments");
  if (int e = check_nets(nets)) return e;
  const NetTopo& t = sys->critic;
  hipLaunchKernelGGL(k_soft, dim3(std::min((t.params + 255) / 256, 1024)), dim3(256), 0, as_stream(stream), t,
                     nets->critic_d, nets->target_d, reinterpret_cast<float4*>(nets->target_d + flat_span(t)),
                     (double)tau);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

extern "C" int cacto_update(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                            const double* storage_d, const int32_t* idx_d, const float* is_w_d, int B, float* y_d,
                            float* V_d, float* Vt_d, void* workspace_d, size_t workspace_bytes, void* stream) {
  CACTO_REQUIRE(sys && cfg && storage_d && idx_d && B > 0, "cacto_update: bad arguments");
  if (int e = check_nets(nets)) return e;
  CHECK_WS(workspace_d, workspace_bytes, B);
  const Workspace w = plan(sys, B, static_cast<char*>(workspace_d));
  hipStream_t st = as_stream(stream);
  if (int e = launch_critic_chain(sys, nets, cfg, storage_d, idx_d, is_w_d, B, y_d, V_d, Vt_d, w, st)) return e;
  if (int e = critic_step_tail(sys, nets, cfg, w, st, nullptr, nets->critic_d)) return e;
  if (int e = launch_actor_chain(sys, nets, cfg, storage_d, idx_d, B, w, st)) return e;
  return actor_step_tail(sys, nets, cfg, w, st);
}

// Data-parallel form of the paired schedule (update_pipeline_pair): per step, the gradients of the
// critic step of update t and of the actor step of update t - 1 (either may be absent) go to one
// flat buffer [critic P | actor P], the caller all-reduces it once (RCCL), then both Adam steps.
namespace {
// stage bit 0: the chain(s) and the critic's weight gradient; bit 1: the actor's weight gradient
// (which reads only the actor chain's panels in the workspace)
int pair_grads(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg, const double* storage_d,
               const int32_t* idx_c_d, const float* is_w_d, const int32_t* idx_a_d, int B, float* grad_d, float* y_d,
               float* V_d, void* workspace_d, size_t workspace_bytes, int stages, hipStream_t st) {
  CHECK_WS(workspace_d, workspace_bytes, B);
  const Workspace w = plan(sys, B, static_cast<char*>(workspace_d));
  const int Pc = sys->critic.params, Pa = sys->actor.params;
  if (stages & 2) {
    if (!idx_a_d) return CACTO_OK;
    int nch = 0;
    if (int e = launch_wgrad(sys->actor, w.act, 0, w.Bp, 0, w.slab_a, st, &nch)) return e;
    return launch_reduce(w.slab_a, nch, Pa, grad_d + Pc, st);
  }
  float* yb = y_d ? y_d : w.scal;
  float* Vb = V_d ? V_d : w.scal + w.Bp;
  if (idx_c_d && idx_a_d) {
    const NetView C = cacto_make_view(sys, CACTO_NET_CRITIC, nets->critic_d);
    const NetView Tg = cacto_make_view(sys, CACTO_NET_CRITIC, nets->target_d);
    const NetView Ac = cacto_make_view(sys, CACTO_NET_ACTOR, nets->actor_d);
    if (int e = dispatch_nj<LaunchChainPair>(sys->host.p, sys, C, Tg, Ac, chain_scalars(cfg, B), storage_d, idx_c_d,
                                             is_w_d, idx_a_d, B, w.crit, w.act, yb, Vb, nets->step_d, st))
      return e;
  } else if (idx_c_d) {
    if (int e = launch_critic_chain(sys, nets, cfg, storage_d, idx_c_d, is_w_d, B, yb, Vb, nullptr, w, st)) return e;
  } else {
    if (int e = launch_actor_chain(sys, nets, cfg, storage_d, idx_a_d, B, w, st)) return e;
  }
  if (idx_c_d) {
    const bool sob = cfg->w_S != 0.0;
    int nch = 0;
    if (int e = launch_wgrad(sys->critic, w.crit, sob ? 0 : w.Bp, 2 * w.Bp, w.Bp, w.slab, st, &nch)) return e;
    if (int e = launch_reduce(w.slab, nch, Pc, grad_d, st)) return e;
  }
  if (stages & 2) return pair_grads(sys, nets, cfg, storage_d, idx_c_d, is_w_d, idx_a_d, B, grad_d, y_d, V_d,
                                    workspace_d, workspace_bytes, 2, st);
  return CACTO_OK;
}
}  // namespace

extern "C" int cacto_update_pair_grads(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                                       const double* storage_d, const int32_t* idx_c_d, const float* is_w_d,
                                       const int32_t* idx_a_d, int B, float* grad_d, float* y_d, float* V_d,
                                       void* workspace_d, size_t workspace_bytes, void* stream) {
  CACTO_REQUIRE(sys && cfg && storage_d && grad_d && B > 0 && (idx_c_d || idx_a_d),
                "cacto_update_pair_grads: bad arguments");
  if (int e = check_nets(nets)) return e;
  return pair_grads(sys, nets, cfg, storage_d, idx_c_d, is_w_d, idx_a_d, B, grad_d, y_d, V_d, workspace_d,
                    workspace_bytes, 1 | 2, as_stream(stream));
}

extern "C" int cacto_update_pair_grads_stage(const cacto_sys* sys, const cacto_nets* nets,
                                             const cacto_update_cfg* cfg, const double* storage_d,
                                             const int32_t* idx_c_d, const float* is_w_d, const int32_t* idx_a_d,
                                             int B, float* grad_d, float* y_d, float* V_d, void* workspace_d,
                                             size_t workspace_bytes, int stage, void* stream) {
  CACTO_REQUIRE(sys && cfg && storage_d && grad_d && B > 0 && (idx_c_d || idx_a_d) && (stage == 0 || stage == 1),
                "cacto_update_pair_grads_stage: bad arguments");
  if (int e = check_nets(nets)) return e;
  return pair_grads(sys, nets, cfg, storage_d, idx_c_d, is_w_d, idx_a_d, B, grad_d, y_d, V_d, workspace_d,
                    workspace_bytes, stage == 0 ? 1 : 2, as_stream(stream));
}

extern "C" int cacto_update_pair_apply(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                                       const float* grad_d, int critic, int actor, int soft_update, void* stream) {
  CACTO_REQUIRE(sys && cfg && grad_d && (critic || actor), "cacto_update_pair_apply: bad arguments");
  if (int e = check_nets(nets)) return e;
  hipStream_t st = as_stream(stream);
  if (critic)
    if (int e = launch_adam(sys, nets, cfg, CACTO_NET_CRITIC, grad_d, 1, soft_update, st)) return e;
  if (actor)
    if (int e = launch_adam(sys, nets, cfg, CACTO_NET_ACTOR, grad_d + sys->critic.params, 1, 0, st)) return e;
  return CACTO_OK;
}

// K consecutive updates (learn_and_update's loop with its minibatches drawn up front, RL.py:120-143)
// as a two-stream pipeline. The critic step of update t+1 reads only the critic, the target and the
// rows — never the actor — so it runs while the actor step of update t is still going:
//   stream : critic chain(t) on C_t, wgrad, Adam(t): C_t -> C_{t+1} (+ soft target update)
//   side   : [wait Adam(t)], actor chain(t) against C_{t+1}, wgrad, Adam(actor), [event]
// The critic rotates over the caller's net buffer and two workspace copies (C_t in buffer t % 3),
// so Adam(t) overwrites the buffer actor chain(t-3) read (and, with PER, the sampler of update t
// the index buffer it read) — the only ordering the stream needs from the side stream: the event
// of side iteration t-3, recorded after that iteration's Adam, normally long signalled. (With two
// buffers the event had to follow the actor chain itself, and its record packet cost the side
// stream — the critical one — a queue gap between the chain and its GEMM.) Every kernel sees the
// same inputs as in K sequential cacto_update calls, so the results are bit-identical; the final
// critic is copied back if it ended in a workspace buffer, and the side stream joins the caller's
// stream before returning.
namespace {
// PER state of cacto_update_n_per (replay_buffer.py:139-218)
struct PerArgs {
  double *sum_tree, *min_tree;
  int64_t cap, max_idx;
  double beta, fresh, eps, alpha;
  const double* uniforms;  // [K][B]
  double *exp_counter, *max_priority;
};

// Whether the PER loop of this batch can take the overlapped form: the count deferred into the
// priority update (large batches), a priority update at all (alpha != 0), 256-leaf subtrees whose
// roots fit one workgroup, the large-batch critic GEMM and an Adam step with all chunks in flight.
bool per_overlap_ok(const cacto_sys* sys, const cacto_update_cfg* cfg, const PerArgs* per, int B, const Workspace& w) {
  if (!per || !per_overlap_on() || B < cacto_per_mw_min() || per->alpha == 0.0) return false;
  if (per->cap < 2 * PER_RUN_SUB || per->cap > (int64_t)PER_RUN_SUB * PER_RUN_SUB || per->cap % PER_RUN_SUB) return false;
  if (fused_adam(w.Bp)) return false;
  const bool sob = cfg->w_S != 0.0;
  const int r0 = sob ? 0 : w.Bp, r1 = 2 * w.Bp;
  return wgrad_big(sys->critic, r1 - r0) && ceil_div(r1 - r0, wg_chunk(r1 - r0)) <= 64;
}

// The priority update of one PER step (RL.py:129-131). late_count: the sampler left its
// exp_counter += 1 to this call (large batches), which applies it first, in the same launch. With
// alpha == 0 the reference skips update_priorities (RL.py:130) — the count still happens.
int per_priority_update(const PerArgs* per, const int32_t* idx, const float* y, const float* V, int B, bool late_count,
                        hipStream_t st) {
  if (per->alpha == 0.0) return late_count ? cacto_per_count_launch(idx, B, per->exp_counter, st) : CACTO_OK;
  if (late_count)
    return cacto_per_update_count(per->sum_tree, per->min_tree, per->cap, idx, y, V, per->exp_counter, per->fresh,
                                  per->eps, per->alpha, per->max_priority, B, st);
  return cacto_per_update(per->sum_tree, per->min_tree, per->cap, idx, y, V, per->exp_counter, per->fresh, per->eps,
                          per->alpha, per->max_priority, B, st);
}

// Small batches (fused_adam): one stream, K + 1 steps. Step t runs the critic chain of update t
// and the actor chain of update t - 1 as one grid (k_chain_pair), then both GEMM + Adam steps as
// one k_wgrad_adam launch:
//   critic(t) reads C_t, T_t (Adam of step t - 1 wrote them); actor(t-1) reads A_{t-1} and C_t —
//   exactly what RL.py:104-109 gives it (the critic after its own update t - 1);
//   Adam: C_t -> C_{t+1} (+ soft T), A_{t-1} -> A_t.
// Every kernel sees the inputs of the sequential loop, so results are bit-identical, with no
// cross-stream events and three launches per update (five with PER).
int update_pipeline_pair(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                         const double* storage_d, const int32_t* idx_d, const PerArgs* per, int K, int B,
                         const Workspace& w, hipStream_t st) {
  float* const y = w.scal;
  float* const V = w.scal + w.Bp;
  const int soft = cfg->MC ? 0 : 1;
  const ChainScalars cs = chain_scalars(cfg, B);
  const NetView C = cacto_make_view(sys, CACTO_NET_CRITIC, nets->critic_d);
  const NetView Tg = cacto_make_view(sys, CACTO_NET_CRITIC, nets->target_d);
  const NetView Ac = cacto_make_view(sys, CACTO_NET_ACTOR, nets->actor_d);
  const AdamNet cn = critic_adam_net(sys, nets, cfg, w, soft, nullptr, nets->critic_d);
  const AdamNet an = actor_adam_net(sys, nets, cfg, w);
  const bool late_count = per && B >= cacto_per_mw_min();  // exp_counter += 1 just before the priority update
  const int32_t* idx_prev = nullptr;
  for (int t = 0; t <= K; ++t) {
    const int32_t* idx = nullptr;
    const float* isw = nullptr;
    if (t < K) {
      idx = idx_d ? idx_d + (size_t)t * B : nullptr;
      if (per) {
        int32_t* pi = w.pidx + (size_t)(t & 1) * w.Bp;
        if (int e = cacto_per_sample(per->sum_tree, per->min_tree, per->cap, per->max_idx, per->beta,
                                     per->uniforms + (size_t)t * B, B, pi, w.pisw, late_count ? nullptr : per->exp_counter, st))
          return e;
        idx = pi;
        isw = w.pisw;
      }
    }
    if (t < K && t > 0) {
      if (int e = dispatch_nj<LaunchChainPair>(sys->host.p, sys, C, Tg, Ac, cs, storage_d, idx, isw, idx_prev, B,
                                               w.crit, w.act, y, V, nets->step_d, st))
        return e;
      if (int e = launch_wgrad_adam(sys, 2, cn, &an, nets->step_d, st)) return e;
    } else if (t < K) {
      if (int e = launch_critic_chain(sys, nets, cfg, storage_d, idx, isw, B, y, V, nullptr, w, st)) return e;
      if (int e = launch_wgrad_adam(sys, 0, cn, nullptr, nets->step_d, st)) return e;
    } else {
      if (int e = launch_actor_chain(sys, nets, cfg, storage_d, idx_prev, B, w, st)) return e;
      if (int e = launch_wgrad_adam(sys, 1, an, nullptr, nets->step_d, st)) return e;
    }
    if (per && t < K)
      if (int e = per_priority_update(per, idx, y, V, B, late_count, st)) return e;
    idx_prev = idx;
  }
  return CACTO_OK;
}

// The side stream and its events, created once per handle and published only when all exist.
int ensure_side_stream(cacto_sys* ms) {
  if (ms->side) return CACTO_OK;
  hipStream_t side = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  hipError_t e = hipStreamCreateWithFlags(&side, hipStreamNonBlocking);
  // device-scope events: every producer and consumer of these dependencies is a kernel on this device
  const unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
  for (int k = 0; k < 4 && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&ev[k], evf);
  unsigned long long* sig = nullptr;
  if (e == hipSuccess) e = hipMalloc(&sig, 8 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(sig, 0, 8 * sizeof(unsigned long long));
  if (e != hipSuccess) {
    if (sig) (void)hipFree(sig);
    for (hipEvent_t x : ev)
      if (x) (void)hipEventDestroy(x);
    if (side) (void)hipStreamDestroy(side);
    return hip_fail(e, "cacto_update_n: side stream / events / pipeline signal");
  }
  ms->pipe_sig = sig;
  ms->pipe_seq = 0;
  ms->ev_critic = ev[0];
  ms->ev_actor[0] = ev[1];
  ms->ev_actor[1] = ev[2];
  ms->ev_actor[2] = ev[3];
  ms->side = side;
  return CACTO_OK;
}

// How the two streams of this call are ordered: true = device-side waits (the default), false = queue
// markers (event record / wait). CACTO_PIPE_DEVWAIT=0 / 1 forces markers / device waits (read once;
// A/B and the timeout test). Otherwise markers when kernels are serialized by the environment
// (AMD_SERIALIZE_KERNEL, HIP_LAUNCH_BLOCKING) or when the handle's one-time concurrency probe failed
// (k_pipe_probe; e.g. counter collection). Always markers while `st` is being captured into a graph:
// the waits compare device counters with absolute targets baked into the launches, and a replayed
// graph would find its targets already reached.
int pipe_devwait(cacto_sys* ms, hipStream_t st, bool* out) {
  static const int env = [] {
    const char* e = std::getenv("CACTO_PIPE_DEVWAIT");
    if (e) return std::atoi(e) != 0 ? 1 : 0;
    const char* s1 = std::getenv("AMD_SERIALIZE_KERNEL");
    const char* s2 = std::getenv("HIP_LAUNCH_BLOCKING");
    if ((s1 && std::atoi(s1) != 0) || (s2 && std::atoi(s2) != 0)) return 0;
    return -1;  // probe
  }();
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  CACTO_CHECK_HIP(hipStreamIsCapturing(st, &cap));
  if (cap != hipStreamCaptureStatusNone) {
    *out = false;
    return CACTO_OK;
  }
  if (env >= 0) {
    *out = env == 1;
    return CACTO_OK;
  }
  if (ms->pipe_probe < 0) {
    // both probe kernels start after everything already queued on `st`; the side one first
    unsigned long long* w = ms->pipe_sig;
    CACTO_CHECK_HIP(hipMemsetAsync(w + 4, 0, 4 * sizeof(unsigned long long), st));
    CACTO_CHECK_HIP(hipEventRecord(ms->ev_critic, st));
    CACTO_CHECK_HIP(hipStreamWaitEvent(ms->side, ms->ev_critic, 0));
    hipLaunchKernelGGL(k_pipe_probe, dim3(1), dim3(64), 0, ms->side, w, 0);
    CACTO_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_pipe_probe, dim3(1), dim3(64), 0, st, w, 1);
    CACTO_CHECK_HIP(hipGetLastError());
    CACTO_CHECK_HIP(hipStreamSynchronize(ms->side));
    CACTO_CHECK_HIP(hipStreamSynchronize(st));
    unsigned long long ok[2] = {0, 0};
    CACTO_CHECK_HIP(hipMemcpy(ok, w + 6, sizeof(ok), hipMemcpyDeviceToHost));
    ms->pipe_probe = ok[0] && ok[1] ? 1 : 0;
  }
  *out = ms->pipe_probe == 1;
  return CACTO_OK;
}

int update_pipeline_body(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                         const double* storage_d, const int32_t* idx_d, const PerArgs* per, int K, int B,
                         const Workspace& w, hipStream_t st, int* cbuf, bool devwait);

int update_pipeline(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg, const double* storage_d,
                    const int32_t* idx_d, const PerArgs* per, int K, int B, const Workspace& w, hipStream_t st) {
  cacto_sys* ms = const_cast<cacto_sys*>(sys);
  std::lock_guard<std::mutex> lock(ms->pipe_mu);
  if (int e = ensure_side_stream(ms)) return e;
  if (!ms->latch_host) {
    CACTO_CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&ms->latch_host), sizeof(unsigned long long),
                                  hipHostMallocDefault));
    *ms->latch_host = 0;
  }
  // a device-side wait of an earlier call timed out and nobody has collected it with
  // cacto_pipeline_check (the Python layer does at the end of every learn_and_update and before
  // every checkpoint save): refuse to build on results whose order cannot be trusted
  if (*reinterpret_cast<volatile unsigned long long*>(ms->latch_host)) {
    set_error("cacto_update_n: a device-side pipeline wait of an earlier call timed out (kernels serialized?); its "
              "results are not trustworthy — collect it with cacto_pipeline_check, or run with CACTO_PIPE_DEVWAIT=0");
    return CACTO_EINVAL;
  }
  bool devwait = false;
  if (int e = pipe_devwait(ms, st, &devwait)) return e;
  const NetTopo& tc = sys->critic;
  const size_t nb_bytes = ((size_t)flat_span(tc) + (size_t)2 * tc.blocks * 256) * sizeof(float);
  const size_t nb_stride = align64((size_t)flat_span(tc) + (size_t)2 * tc.blocks * 256);
  CACTO_CHECK_HIP(hipMemcpyAsync(w.cshadow, nets->critic_d, nb_bytes, hipMemcpyDeviceToDevice, st));
  CACTO_CHECK_HIP(hipMemcpyAsync(w.cshadow + nb_stride, nets->critic_d, nb_bytes, hipMemcpyDeviceToDevice, st));
  CACTO_CHECK_HIP(hipEventRecord(ms->ev_critic, st));  // everything the caller queued before
  CACTO_CHECK_HIP(hipStreamWaitEvent(ms->side, ms->ev_critic, 0));
  // cbuf: the buffer (0 caller's, 1-2 workspace) holding the newest critic; on every exit, error or
  // not, the side stream joins the caller's stream and the newest critic lands in the caller's buffer
  int cbuf = 0;
  const int err = update_pipeline_body(sys, nets, cfg, storage_d, idx_d, per, K, B, w, st, &cbuf, devwait);
  CACTO_CHECK_HIP(hipEventRecord(ms->ev_critic, ms->side));
  CACTO_CHECK_HIP(hipStreamWaitEvent(st, ms->ev_critic, 0));
  // the timeout latch's host copy, read by cacto_pipeline_check after a synchronisation of `st`
  if (devwait)
    CACTO_CHECK_HIP(hipMemcpyAsync(ms->latch_host, ms->pipe_sig + 1, sizeof(unsigned long long),
                                   hipMemcpyDeviceToHost, st));
  if (cbuf)
    CACTO_CHECK_HIP(hipMemcpyAsync(nets->critic_d, w.cshadow + (cbuf - 1) * nb_stride, nb_bytes,
                                   hipMemcpyDeviceToDevice, st));
  return err;
}

int update_pipeline_body(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                         const double* storage_d, const int32_t* idx_d, const PerArgs* per, int K, int B,
                         const Workspace& w, hipStream_t st, int* cbuf, bool devwait) {
  cacto_sys* ms = const_cast<cacto_sys*>(sys);
  hipStream_t side = ms->side;
  const size_t nb_stride = align64((size_t)flat_span(sys->critic) + (size_t)2 * sys->critic.blocks * 256);
  float* const buf[3] = {nets->critic_d, w.cshadow, w.cshadow + nb_stride};
  float* const y = w.scal;
  float* const V = w.scal + w.Bp;
  const bool late_count = per && B >= cacto_per_mw_min();  // exp_counter += 1 just before the priority update
  // queue markers (devwait off): every other iteration with PER (car_park B = 4096: 9.04 k -> 9.36 k
  // updates/s), every iteration without (manipulator B = 8192 lost 8 % to the tighter wait)
  const bool every2 = per != nullptr;
  // devwait: the critic stream's ordering against the side stream without queue markers — the
  // actor's GEMM (the launch after each actor chain) publishes the count of finished actor chains on
  // the device, and the critic's Adam(t) polls it (pipe_wait) before overwriting the buffer actor
  // chain(t-3) read; the PER index ring has four buffers, so the sampler of update t overwrites the
  // one actor chain(t-4) read, which Adam(t-1)'s wait covers. Measured r05 (1 MI355X, updates/s): DI
  // B = 4096 12.3 k -> 12.7 k, car_park PER B = 4096 9.88 k -> 9.98 k, manipulator B = 8192 unchanged.
  // ... and the side stream's wait on the critic's Adam too (devwait_actor): the critic's Adam writes
  // the weights through to memory at agent scope and publishes after its stores completed, the actor
  // chain polls relaxed just before its critic pass at s' (with PER at its start, before it gathers
  // the sampled rows) — where that cannot starve the critic stream of CUs: 16-sample actor tiles (the
  // q4 chains take no wait), at most one actor workgroup per CU (a CU holding one actor workgroup
  // still fits a critic chain, GEMM or Adam workgroup beside it, so the critic stream always
  // progresses). DI B = 4096 13.2-13.3 k -> 14.2-14.4 k updates/s (r05).
  const bool devwait_actor = devwait && chain_tile(w.Bp) == CACTO_TILE && w.Bp / CACTO_TILE <= cu_count();
  const int thru = devwait_actor ? 1 : 0;
  unsigned long long* const sig = ms->pipe_sig;
  // the overlapped PER form (per_overlap_ok): priority update t inside the critic GEMM's launch,
  // sample t + 1 inside its Adam's; the index ring has five buffers (sample t + 1 runs in the launch
  // after the Adam(t - 1) that waited for actor chain t - 4). Otherwise the sample and the priority
  // update run on the critic stream between its launches.
  const bool ovl = per && devwait && per_overlap_ok(sys, cfg, per, B, w);
  const int nring = ovl ? 5 : devwait ? 4 : 3;
  const int nroot = per ? (int)(per->cap / PER_RUN_SUB) : 0;
  const unsigned long long base = ms->pipe_seq;
  ms->pipe_seq = base + K;  // reserved up front: no later call's waits can be satisfied by this call's values
  // test hook (tests/test_gpu_per_pipeline.py): CACTO_PIPE_FAULT_INJECT=1 gives the first device-side
  // wait of the process an unreachable target, so it times out and latches (once per process)
  static std::atomic<int> inject{[] {
    const char* e = std::getenv("CACTO_PIPE_FAULT_INJECT");
    return e && e[0] == '1' ? 1 : 0;
  }()};
  for (int t = 0; t < K; ++t) {
    // actor chain(t-3) read the critic buffer Adam(t) writes and (PER) the index buffer of update t.
    // every2: the side stream records only at even iterations and the critic waits at even t for
    // side iteration t-2 (which covers t-3 here and at t+1) — half the queue markers on each stream
    if (devwait) {
    } else if (every2) {
      if (t >= 2 && (t & 1) == 0) CACTO_CHECK_HIP(hipStreamWaitEvent(st, ms->ev_actor[((t - 2) >> 1) & 1], 0));
    } else if (t >= 3) {
      CACTO_CHECK_HIP(hipStreamWaitEvent(st, ms->ev_actor[t % 3], 0));
    }
    const int32_t* idx = idx_d + (size_t)t * B;
    const float* isw = nullptr;
    if (per) {
      int32_t* pi = w.pidx + (size_t)(t % nring) * w.Bp;
      if (ovl) {
        if (t == 0) {  // the first sample, recording its runs; later ones run inside the Adam launch
          CACTO_CHECK_HIP(hipMemsetAsync(w.runs, 0x7f, (size_t)nroot * sizeof(int32_t), st));
          CACTO_CHECK_HIP(hipMemsetAsync(w.runs + nroot, 0, (size_t)nroot * sizeof(int32_t), st));
          if (int e = cacto_per_sample_runs_launch(per->sum_tree, per->min_tree, per->cap, per->max_idx, per->beta,
                                                   per->uniforms, B, pi, w.pisw, w.runs, st))
            return e;
        }
      } else if (int e = cacto_per_sample(per->sum_tree, per->min_tree, per->cap, per->max_idx, per->beta,
                                          per->uniforms + (size_t)t * B, B, pi, w.pisw,
                                          late_count ? nullptr : per->exp_counter, st)) {
        return e;
      }
      idx = pi;
      isw = w.pisw;
    }
    cacto_nets cur = *nets, nxt = *nets;
    cur.critic_d = buf[t % 3];
    nxt.critic_d = buf[(t + 1) % 3];
    if (int e = launch_critic_chain(sys, &cur, cfg, storage_d, idx, isw, B, y, V, nullptr, w, st)) return e;
    const bool dw = devwait && t >= 3;
    const unsigned long long wait_c = dw && inject.exchange(0) ? ~0ull : base + t - 2;
    PerRunArgs pra{};
    PerSampleArgs psa{};
    if (ovl) {
      pra = PerRunArgs{per->sum_tree, per->min_tree, per->cap, idx, y, V, per->exp_counter, per->max_idx,
                       per->fresh, per->eps, per->alpha, per->max_priority, w.runs, nullptr};
      if (t + 1 < K)
        psa = PerSampleArgs{per->sum_tree, per->min_tree, per->cap, per->max_idx, per->beta,
                            per->uniforms + (size_t)(t + 1) * B, B, w.pidx + (size_t)((t + 1) % nring) * w.Bp,
                            w.pisw, nullptr, 0, w.runs};
    }
    if (int e = critic_step_tail(sys, nets, cfg, w, st, cur.critic_d, nxt.critic_d, dw ? sig : nullptr, wait_c,
                                 devwait_actor ? sig : nullptr, base + t + 1, ovl ? &pra : nullptr,
                                 ovl && t + 1 < K ? &psa : nullptr, thru))
      return e;
    *cbuf = (t + 1) % 3;
    if (!devwait_actor) CACTO_CHECK_HIP(hipEventRecord(ms->ev_critic, st));
    if (per && !ovl)
      if (int e = per_priority_update(per, idx, y, V, B, late_count, st)) return e;
    if (!devwait_actor) CACTO_CHECK_HIP(hipStreamWaitEvent(side, ms->ev_critic, 0));
    if (int e = launch_actor_chain(sys, &nxt, cfg, storage_d, idx, B, w, side, devwait_actor ? sig + 2 : nullptr,
                                   base + t + 1, per ? 1 : 0))
      return e;
    if (int e = actor_step_tail(sys, nets, cfg, w, side, devwait ? sig : nullptr, base + t + 1)) return e;
    if (devwait) {
    } else if (!every2) {
      CACTO_CHECK_HIP(hipEventRecord(ms->ev_actor[t % 3], side));
    } else if ((t & 1) == 0) {
      CACTO_CHECK_HIP(hipEventRecord(ms->ev_actor[(t >> 1) & 1], side));
    }
  }
  return CACTO_OK;
}
}  // namespace

extern "C" int cacto_pipeline_status(const cacto_sys* sys, unsigned long long* out4_h) {
  CACTO_REQUIRE(sys && out4_h, "cacto_pipeline_status: bad arguments");
  for (int k = 0; k < 4; ++k) out4_h[k] = 0;
  if (!sys->pipe_sig) return CACTO_OK;
  CACTO_CHECK_HIP(hipDeviceSynchronize());
  CACTO_CHECK_HIP(hipMemcpy(out4_h, sys->pipe_sig, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  out4_h[3] = sys->pipe_probe < 0 ? 0 : (unsigned long long)sys->pipe_probe + 1;
  return CACTO_OK;
}

extern "C" int cacto_pipeline_check(cacto_sys* sys, void* stream) {
  CACTO_REQUIRE(sys, "cacto_pipeline_check: bad arguments");
  if (!sys->pipe_sig || !sys->latch_host) return CACTO_OK;
  std::lock_guard<std::mutex> lock(sys->pipe_mu);
  CACTO_CHECK_HIP(hipStreamSynchronize(as_stream(stream)));
  volatile unsigned long long* lh = reinterpret_cast<volatile unsigned long long*>(sys->latch_host);
  if (*lh == 0) return CACTO_OK;
  // collected: clear both copies, so the handle's next calls run again
  CACTO_CHECK_HIP(hipMemset(sys->pipe_sig + 1, 0, sizeof(unsigned long long)));
  *lh = 0;
  set_error("cacto_pipeline_check: a device-side wait of the two-stream update pipeline timed out since the last "
            "check (kernels serialized?); the updates of that call ran without their cross-stream order and their "
            "results are not trustworthy — rerun them with CACTO_PIPE_DEVWAIT=0");
  return CACTO_EINVAL;
}

extern "C" int cacto_update_n(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                              const double* storage_d, const int32_t* idx_d, int K, int B, void* workspace_d,
                              size_t workspace_bytes, void* stream) {
  CACTO_REQUIRE(sys && cfg && storage_d && idx_d && B > 0 && K >= 0, "cacto_update_n: bad arguments");
  if (int e = check_nets(nets)) return e;
  CHECK_WS(workspace_d, workspace_bytes, B);
  if (K == 0) return CACTO_OK;
  const Workspace w = plan(sys, B, static_cast<char*>(workspace_d));
  if (fused_adam(w.Bp)) return update_pipeline_pair(sys, nets, cfg, storage_d, idx_d, nullptr, K, B, w, as_stream(stream));
  return update_pipeline(sys, nets, cfg, storage_d, idx_d, nullptr, K, B, w, as_stream(stream));
}

// learn_and_update with PER (RL.py:122-137) for K updates: sample (stratified, IS weights) ->
// update -> priority update per step, the sampling and priority update on the critic's stream
// (the next sample depends on them), pipelined with the actor steps as in cacto_update_n.
extern "C" int cacto_update_n_per(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                                  const double* storage_d, double* sum_tree_d, double* min_tree_d, int64_t capacity,
                                  int64_t max_idx, double beta, const double* uniforms_d, double* exp_counter_d,
                                  double fresh_factor, double eps, double alpha, double* max_priority_d, int K, int B,
                                  void* workspace_d, size_t workspace_bytes, void* stream) {
  CACTO_REQUIRE(sys && cfg && storage_d && sum_tree_d && min_tree_d && uniforms_d && exp_counter_d &&
                    max_priority_d && B > 0 && K >= 0,
                "cacto_update_n_per: bad arguments");
  if (int e = check_nets(nets)) return e;
  CHECK_WS(workspace_d, workspace_bytes, B);
  if (K == 0) return CACTO_OK;
  const Workspace w = plan(sys, B, static_cast<char*>(workspace_d));
  const PerArgs per{sum_tree_d, min_tree_d, capacity, max_idx, beta, fresh_factor, eps, alpha, uniforms_d,
                    exp_counter_d, max_priority_d};
  // small batches: the paired single-stream schedule with the sampling and priority update between
  // steps (car_park B = 64 with the q4 chains: 21.1 k vs 19.8 k updates/s two-stream); larger
  // batches keep the two-stream pipeline (the actor step beside the sampling / priority update)
  if (fused_adam(w.Bp))
    return update_pipeline_pair(sys, nets, cfg, storage_d, nullptr, &per, K, B, w, as_stream(stream));
  return update_pipeline(sys, nets, cfg, storage_d, nullptr, &per, K, B, w, as_stream(stream));
}

// ---------------------------------------------------------------- data-parallel pipeline (RCCL)
// The data-parallel learn_and_update (main.py:219-225 runs the reference's loop on one process; here
// one process per GPU, the gradients all-reduced over xGMI). The K updates of a call run as the
// two-stream pipeline of cacto_update_n with each network's exchange inside its own stream:
//   stream : [PER: shard stats -> all-gather -> stratified sample over the union] critic chain(t) ->
//            weight-gradient GEMM -> slab reduce -> all-reduce (comm 0) -> Adam(t) (+ soft target
//            update) [-> PER priority update]
//   side   : [marker: Adam(t)] actor chain(t) against C_{t+1} -> GEMM -> reduce -> all-reduce (comm 1)
//            -> Adam
// Every rank issues the same collectives in the same order on each communicator, one communicator
// per stream, so neither stream's collectives can interleave with the other's. The streams are
// ordered with queue markers (no device-side polls beside collectives that wait for other ranks).
// The gradients are scaled by 1/B_global inside the chain kernels, so the exchange is a plain sum;
// every rank applies the same Adam to the same sum, so the replicas stay bit-identical. With one
// rank the all-reduce is the identity and the result equals cacto_update_n / the Python
// dp_pipeline bit for bit (tests/test_gpu_dp.py). The host issues ~14 HIP / RCCL calls per update
// (the Python loop of RL_AC issued ~10 ctypes calls and two torch.distributed collectives: ~160 us
// of host time per update, more than the GPU's).
#include <dlfcn.h>
#include <rccl/rccl.h>

namespace {
// RCCL entry points of the copy already in the process (torch.distributed's, found by soname), else
// the ROCm library: no link-time dependency, one RCCL instance per process.
struct Rccl {
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
  bool ok = false;
};
const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
    if (!h) return x;
    x.get_id = reinterpret_cast<decltype(x.get_id)>(dlsym(h, "ncclGetUniqueId"));
    x.init = reinterpret_cast<decltype(x.init)>(dlsym(h, "ncclCommInitRank"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(h, "ncclCommDestroy"));
    x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(dlsym(h, "ncclAllReduce"));
    x.all_gather = reinterpret_cast<decltype(x.all_gather)>(dlsym(h, "ncclAllGather"));
    x.err = reinterpret_cast<decltype(x.err)>(dlsym(h, "ncclGetErrorString"));
    x.ok = x.get_id && x.init && x.destroy && x.all_reduce && x.all_gather && x.err;
    return x;
  }();
  return r;
}

int rccl_fail(ncclResult_t r, const char* what) {
  set_error(std::string(what) + ": " + (rccl().err ? rccl().err(r) : "RCCL error"));
  return CACTO_EHIP;
}
#define CACTO_CHECK_RCCL(call, what)            \
  do {                                          \
    const ncclResult_t r_ = (call);             \
    if (r_ != ncclSuccess) return rccl_fail(r_, what); \
  } while (0)

int update_pipeline_dp_body(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                            const double* storage_d, const int32_t* idx_d, const PerArgs* per, int K, int B,
                            const Workspace& w, hipStream_t st, int* cbuf) {
  cacto_sys* ms = const_cast<cacto_sys*>(sys);
  const Rccl& R = rccl();
  ncclComm_t cc = static_cast<ncclComm_t>(ms->dp_comm[0]), ca = static_cast<ncclComm_t>(ms->dp_comm[1]);
  hipStream_t side = ms->side;
  const int Pc = sys->critic.params, Pa = sys->actor.params;
  const size_t nb_stride = align64((size_t)flat_span(sys->critic) + (size_t)2 * sys->critic.blocks * 256);
  float* const buf[3] = {nets->critic_d, w.cshadow, w.cshadow + nb_stride};
  float* const y = w.scal;
  float* const V = w.scal + w.Bp;
  const bool sob = cfg->w_S != 0.0;
  const int soft = cfg->MC ? 0 : 1;
  // queue markers: every other iteration with PER, every iteration without (update_pipeline_body)
  const bool every2 = per != nullptr;
  // PER in the critic's GEMM and Adam launches (per_overlap_ok, as cacto_update_n_per): the priority
  // update of update t inside the GEMM's launch, then this shard's statistics and their all-gather,
  // and the sample of t + 1 (IS weights over the union) inside the Adam's launch; the index ring has
  // five buffers (sample t + 1 overwrites the one actor chain t - 4 read, which the marker before
  // update t - 1 or t covers). Otherwise the sample and the priority update run between the launches.
  const bool ovl = per && per_overlap_ok(sys, cfg, per, B, w);
  const int nring = ovl ? 5 : 3;
  const int nroot = per ? (int)(per->cap / PER_RUN_SUB) : 0;
  double* const stats = ms->dp_stats;       // [3] this shard
  double* const shards = ms->dp_stats + 3;  // [world][3]
  auto gather_stats = [&]() -> int {
    if (int e = cacto_per_shard_stats(per->sum_tree, per->min_tree, per->max_idx, stats, st)) return e;
    CACTO_CHECK_RCCL(R.all_gather(stats, shards, 3, ncclFloat64, cc, st), "ncclAllGather(PER shards)");
    return CACTO_OK;
  };
  for (int t = 0; t < K; ++t) {
    if (every2) {
      if (t >= 2 && (t & 1) == 0) CACTO_CHECK_HIP(hipStreamWaitEvent(st, ms->ev_actor[((t - 2) >> 1) & 1], 0));
    } else if (t >= 3) {
      CACTO_CHECK_HIP(hipStreamWaitEvent(st, ms->ev_actor[t % 3], 0));
    }
    const int32_t* idx = idx_d + (size_t)t * B;
    const float* isw = nullptr;
    if (per) {
      // replay_buffer.py:139-188 over the union of the ranks' shards: this shard's (sum, min, rows),
      // all-gathered, then the stratified sample with IS weights against the union
      int32_t* pi = w.pidx + (size_t)(t % nring) * w.Bp;
      if (ovl) {
        if (t == 0) {  // the first sample, recording its runs; later ones run inside the Adam launch
          CACTO_CHECK_HIP(hipMemsetAsync(w.runs, 0x7f, (size_t)nroot * sizeof(int32_t), st));
          CACTO_CHECK_HIP(hipMemsetAsync(w.runs + nroot, 0, (size_t)nroot * sizeof(int32_t), st));
          if (int e = gather_stats()) return e;
          if (int e = cacto_per_sample_runs_launch(per->sum_tree, per->min_tree, per->cap, per->max_idx, per->beta,
                                                   per->uniforms, B, pi, w.pisw, w.runs, st, shards, ms->dp_world))
            return e;
        }
      } else {
        if (int e = gather_stats()) return e;
        if (int e = cacto_per_sample_global(per->sum_tree, per->min_tree, per->cap, per->max_idx, per->beta,
                                            per->uniforms + (size_t)t * B, B, shards, ms->dp_world, pi, w.pisw,
                                            per->exp_counter, st))
          return e;
      }
      idx = pi;
      isw = w.pisw;
    }
    cacto_nets cur = *nets, nxt = *nets;
    cur.critic_d = buf[t % 3];
    nxt.critic_d = buf[(t + 1) % 3];
    if (int e = launch_critic_chain(sys, &cur, cfg, storage_d, idx, isw, B, y, V, nullptr, w, st)) return e;
    int nch = 0;
    PerRunArgs pra{};
    PerSampleArgs psa{};
    if (ovl) {
      // the trees after priority update t: the statistics sample t + 1 weighs against, written by the
      // workgroup of the GEMM's launch that rebuilds the top of the trees (with one subtree, a launch)
      pra = PerRunArgs{per->sum_tree, per->min_tree, per->cap, idx, y, V, per->exp_counter, per->max_idx,
                       per->fresh, per->eps, per->alpha, per->max_priority, w.runs,
                       t + 1 < K && nroot > 1 ? shards : nullptr, 3 * ms->dp_rank, 3 * ms->dp_world};
      if (t + 1 < K)
        psa = PerSampleArgs{per->sum_tree, per->min_tree, per->cap, per->max_idx, per->beta,
                            per->uniforms + (size_t)(t + 1) * B, B, w.pidx + (size_t)((t + 1) % nring) * w.Bp,
                            w.pisw, shards, ms->dp_world, w.runs};
    }
    if (int e = launch_wgrad(sys->critic, w.crit, sob ? 0 : w.Bp, 2 * w.Bp, w.Bp, w.slab, st, &nch, nullptr, 0,
                             ovl ? &pra : nullptr))
      return e;
    if (ovl && t + 1 < K) {
      if (nroot > 1)  // the table with this rank's words filled and the others zero: summed = gathered
        CACTO_CHECK_RCCL(R.all_reduce(shards, shards, (size_t)3 * ms->dp_world, ncclFloat64, ncclSum, cc, st),
                         "ncclAllReduce(PER shards)");
      else if (int e = gather_stats())
        return e;
    }
    if (int e = launch_reduce(w.slab, nch, Pc, ms->dp_gc, st)) return e;
    CACTO_CHECK_RCCL(R.all_reduce(ms->dp_gc, ms->dp_gc, (size_t)Pc, ncclFloat32, ncclSum, cc, st),
                     "ncclAllReduce(critic gradient)");
    cacto_nets dst = *nets;
    dst.critic_d = nxt.critic_d;
    if (int e = launch_adam(sys, &dst, cfg, CACTO_NET_CRITIC, ms->dp_gc, 1, soft, st, cur.critic_d, nullptr, 0, nullptr,
                            0, ovl && t + 1 < K ? &psa : nullptr))
      return e;
    *cbuf = (t + 1) % 3;
    CACTO_CHECK_HIP(hipEventRecord(ms->ev_critic, st));
    if (per && !ovl)
      if (int e = per_priority_update(per, idx, y, V, B, false, st)) return e;
    CACTO_CHECK_HIP(hipStreamWaitEvent(side, ms->ev_critic, 0));
    if (int e = launch_actor_chain(sys, &nxt, cfg, storage_d, idx, B, w, side)) return e;
    int ncha = 0;
    if (int e = launch_wgrad(sys->actor, w.act, 0, w.Bp, 0, w.slab_a, side, &ncha)) return e;
    if (int e = launch_reduce(w.slab_a, ncha, Pa, ms->dp_ga, side)) return e;
    CACTO_CHECK_RCCL(R.all_reduce(ms->dp_ga, ms->dp_ga, (size_t)Pa, ncclFloat32, ncclSum, ca, side),
                     "ncclAllReduce(actor gradient)");
    if (int e = launch_adam(sys, nets, cfg, CACTO_NET_ACTOR, ms->dp_ga, 1, 0, side)) return e;
    if (!every2) {
      CACTO_CHECK_HIP(hipEventRecord(ms->ev_actor[t % 3], side));
    } else if ((t & 1) == 0) {
      CACTO_CHECK_HIP(hipEventRecord(ms->ev_actor[(t >> 1) & 1], side));
    }
  }
  return CACTO_OK;
}

int update_pipeline_dp(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                       const double* storage_d, const int32_t* idx_d, const PerArgs* per, int K, int B,
                       const Workspace& w, hipStream_t st) {
  cacto_sys* ms = const_cast<cacto_sys*>(sys);
  std::lock_guard<std::mutex> lock(ms->pipe_mu);
  if (!ms->dp_comm[0] || !ms->dp_comm[1]) {
    set_error("cacto_update_n_dp: no RCCL communicators on this handle (cacto_dp_attach)");
    return CACTO_EINVAL;
  }
  if (int e = ensure_side_stream(ms)) return e;
  const NetTopo& tc = sys->critic;
  const size_t nb_bytes = ((size_t)flat_span(tc) + (size_t)2 * tc.blocks * 256) * sizeof(float);
  const size_t nb_stride = align64((size_t)flat_span(tc) + (size_t)2 * tc.blocks * 256);
  CACTO_CHECK_HIP(hipMemcpyAsync(w.cshadow, nets->critic_d, nb_bytes, hipMemcpyDeviceToDevice, st));
  CACTO_CHECK_HIP(hipMemcpyAsync(w.cshadow + nb_stride, nets->critic_d, nb_bytes, hipMemcpyDeviceToDevice, st));
  CACTO_CHECK_HIP(hipEventRecord(ms->ev_critic, st));
  CACTO_CHECK_HIP(hipStreamWaitEvent(ms->side, ms->ev_critic, 0));
  int cbuf = 0;
  const int err = update_pipeline_dp_body(sys, nets, cfg, storage_d, idx_d, per, K, B, w, st, &cbuf);
  CACTO_CHECK_HIP(hipEventRecord(ms->ev_critic, ms->side));
  CACTO_CHECK_HIP(hipStreamWaitEvent(st, ms->ev_critic, 0));
  if (cbuf)
    CACTO_CHECK_HIP(hipMemcpyAsync(nets->critic_d, w.cshadow + (cbuf - 1) * nb_stride, nb_bytes,
                                   hipMemcpyDeviceToDevice, st));
  return err;
}
}  // namespace

void cacto_dp_release(cacto_sys* sys) {
  for (void*& c : sys->dp_comm) {
    if (c && rccl().ok) (void)rccl().destroy(static_cast<ncclComm_t>(c));
    c = nullptr;
  }
  if (sys->dp_gc) (void)hipFree(sys->dp_gc);
  if (sys->dp_ga) (void)hipFree(sys->dp_ga);
  if (sys->dp_stats) (void)hipFree(sys->dp_stats);
  sys->dp_gc = sys->dp_ga = nullptr;
  sys->dp_stats = nullptr;
  sys->dp_rank = sys->dp_world = 0;
}

extern "C" int cacto_dp_unique_ids(void* out_h, int n) {
  CACTO_REQUIRE(out_h && n >= 1 && n <= 16, "cacto_dp_unique_ids: bad arguments");
  const Rccl& R = rccl();
  CACTO_REQUIRE(R.ok, "cacto_dp_unique_ids: RCCL (librccl.so.1) not found");
  for (int k = 0; k < n; ++k) {
    ncclUniqueId id;
    CACTO_CHECK_RCCL(R.get_id(&id), "ncclGetUniqueId");
    std::memcpy(static_cast<char*>(out_h) + (size_t)k * sizeof(ncclUniqueId), &id, sizeof(ncclUniqueId));
  }
  return CACTO_OK;
}

extern "C" int cacto_dp_attach(cacto_sys* sys, const void* ids_h, int rank, int world) {
  CACTO_REQUIRE(sys && ids_h && world >= 1 && rank >= 0 && rank < world, "cacto_dp_attach: bad arguments");
  const Rccl& R = rccl();
  CACTO_REQUIRE(R.ok, "cacto_dp_attach: RCCL (librccl.so.1) not found");
  std::lock_guard<std::mutex> lock(sys->pipe_mu);
  cacto_dp_release(sys);
  for (int k = 0; k < 2; ++k) {
    ncclUniqueId id;
    std::memcpy(&id, static_cast<const char*>(ids_h) + (size_t)k * sizeof(ncclUniqueId), sizeof(ncclUniqueId));
    ncclComm_t c = nullptr;
    CACTO_CHECK_RCCL(R.init(&c, world, id, rank), "ncclCommInitRank");
    sys->dp_comm[k] = c;
  }
  CACTO_CHECK_HIP(hipMalloc(&sys->dp_gc, sizeof(float) * sys->critic.params));
  CACTO_CHECK_HIP(hipMalloc(&sys->dp_ga, sizeof(float) * sys->actor.params));
  CACTO_CHECK_HIP(hipMalloc(&sys->dp_stats, sizeof(double) * 3 * (world + 1)));
  sys->dp_rank = rank;
  sys->dp_world = world;
  return CACTO_OK;
}

extern "C" int cacto_dp_detach(cacto_sys* sys) {
  CACTO_REQUIRE(sys, "cacto_dp_detach: bad arguments");
  std::lock_guard<std::mutex> lock(sys->pipe_mu);
  if (sys->side) CACTO_CHECK_HIP(hipStreamSynchronize(sys->side));
  cacto_dp_release(sys);
  return CACTO_OK;
}

extern "C" int cacto_update_n_dp(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                                 const double* storage_d, const int32_t* idx_d, int K, int B, void* workspace_d,
                                 size_t workspace_bytes, void* stream) {
  CACTO_REQUIRE(sys && cfg && storage_d && idx_d && B > 0 && K >= 0, "cacto_update_n_dp: bad arguments");
  if (int e = check_nets(nets)) return e;
  CHECK_WS(workspace_d, workspace_bytes, B);
  if (K == 0) return CACTO_OK;
  const Workspace w = plan(sys, B, static_cast<char*>(workspace_d));
  return update_pipeline_dp(sys, nets, cfg, storage_d, idx_d, nullptr, K, B, w, as_stream(stream));
}

extern "C" int cacto_update_n_per_dp(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                                     const double* storage_d, double* sum_tree_d, double* min_tree_d, int64_t capacity,
                                     int64_t max_idx, double beta, const double* uniforms_d, double* exp_counter_d,
                                     double fresh_factor, double eps, double alpha, double* max_priority_d, int K,
                                     int B, void* workspace_d, size_t workspace_bytes, void* stream) {
  CACTO_REQUIRE(sys && cfg && storage_d && sum_tree_d && min_tree_d && uniforms_d && exp_counter_d &&
                    max_priority_d && B > 0 && K >= 0,
                "cacto_update_n_per_dp: bad arguments");
  if (int e = check_nets(nets)) return e;
  CHECK_WS(workspace_d, workspace_bytes, B);
  if (K == 0) return CACTO_OK;
  const Workspace w = plan(sys, B, static_cast<char*>(workspace_d));
  const PerArgs per{sum_tree_d, min_tree_d, capacity, max_idx, beta, fresh_factor, eps, alpha, uniforms_d,
                    exp_counter_d, max_priority_d};
  return update_pipeline_dp(sys, nets, cfg, storage_d, nullptr, &per, K, B, w, as_stream(stream));
}
