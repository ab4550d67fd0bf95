// The learner chains on 4-sample tiles (q4.h): NN.compute_critic_grad (Sobolev double backprop,
// NeuralNetwork.py:150-180) and NN.compute_actor_grad (dynamics Jacobian path,
// NeuralNetwork.py:182-233), the same operations as the 16-sample chains of learn_kernels.hip with
// every activation tile in the F4 layout (one float per lane per 16-feature tile). They write the
// same operand panels (feature-major, sample rows), so k_wgrad / k_wgrad_adam / k_adam are shared.
//
// 8 waves per workgroup. A chain is a sequence of small dependent layer steps (a few hundred MFMA
// cycles each for 4 samples), so what bounds it is latency: the barriers between steps and the
// memory latency of weight fragments that every Adam step has just rewritten (they come from the
// memory-side cache). The 8 waves are used to cut both:
//   * the critic's target forward at s' (waves 4-7) runs beside its forward at s (waves 0-3), two
//     4-wave teams sharing the barriers of one pass;
//   * every other layer runs as one 8-wave team (out tiles wave, wave + 8), so the actor's 256-wide
//     layers are one pair of out tiles per wave, loaded together;
//   * each pass's fragments are issued one phase before the pass (during the previous pass or the
//     dynamics), so no pass starts on a cold load.
// After q4_reduce a wave holds, per out tile, one element per lane: feature 16 ot + (lane & 15) of
// sample lane >> 4 (F4 index q4e(ot, lane)). All elementwise arrays (cos / sin / pre-activation /
// zbar tiles) use the F4 layout, so an epilogue reads its operands at the index it writes.
// Per-sample work (row gathers, input normalisation, dynamics, losses) runs one (sample, feature)
// element per thread.
//
// Included by learn_kernels.hip (uses its GradBufs, ChainScalars, clog, CSTAMP).
#pragma once

#include "q4.h"

namespace cacto {

constexpr int Q4_NW = 8;  // waves per q4 chain workgroup
constexpr int Q4_THREADS = 64 * Q4_NW;

// ---------------------------------------------------------------- critic (fixed 64-64-128-128-1 shape)
// A forward pass's fragments for a team of NW waves (out tiles wi + NW t): layers 0-1 have 4 out
// tiles, layers 2-3 have 8, the output layer is split over the team's k-tiles.
template <int NW>
struct Q4CriticFwd {
  static constexpr int N8 = 8 / NW;
  Q4Frags<1, 1, NW> f0;
  Q4Frags<4, 1, NW> f1;
  Q4Frags<4, N8, NW> f2;
  Q4Frags<8, N8, NW> f3;
  Q4Split<N8, NW> f4;
  int act;  // NetTopo::act (elu layers of the sine-elu critic)
  template <bool BIAS>
  __device__ __forceinline__ void load(const NetView& N, int wi, int lane) {
    act = N.t.act;
    f0.template load<BIAS>(N.fwd(0), N.biasp(0), 4, 64, wi, lane);
    f1.template load<BIAS>(N.fwd(1), N.biasp(1), 4, 64, wi, lane);
    f2.template load<BIAS>(N.fwd(2), N.biasp(2), 8, 128, wi, lane);
    f3.template load<BIAS>(N.fwd(3), N.biasp(3), 8, 128, wi, lane);
  }
  __device__ __forceinline__ void load_last(const NetView& N, int wi, int lane) {
    f4.template load<true>(N.fwd(4), 8, N.biasp(4), 1, wi, lane);
  }
};

// The transposed passes G_l = D_l W_l^T for an 8-wave team: l3 one of 8 out tiles per wave, l2 / l1
// 4 out tiles (waves 0-3), l0 split over the 4 k-tiles. Loaded once per chain and used by both the
// first backward and the backward of the forward graph.
struct Q4CriticBwd {
  Q4Frags<8, 1, Q4_NW> g3;
  Q4Frags<8, 1, Q4_NW> g2;
  Q4Frags<4, 1, Q4_NW> g1;
  Q4Split<1, Q4_NW> g0;
  float w5;  // W5[16 wave + c, 0]: the lane's feature of layer-3 out tile `wave`
  __device__ __forceinline__ void load(const NetView& N, int wave, int lane) {
    load_g3(N, wave, lane);
    load_rest(N, wave, lane);
  }
  // in two parts, so a pass can issue them as its own fragments die
  __device__ __forceinline__ void load_g3(const NetView& N, int wave, int lane) {
    w5 = N.flat[N.t.woff[4] + 16 * wave + (lane & 15)];
    g3.load<false>(N.bwd(3), nullptr, 8, 128, wave, lane);
  }
  __device__ __forceinline__ void load_rest(const NetView& N, int wave, int lane) {
    g2.load<false>(N.bwd(2), nullptr, 4, 64, wave, lane);
    g1.load<false>(N.bwd(1), nullptr, 4, 64, wave, lane);
    g0.load<false>(N.bwd(0), 4, nullptr, 16, wave, lane);
  }
};

// Critic forward over the F4 input tile X0 for a team (net_common.h critic_forward_tile_f): with Hs
// every h_l = sin z_l is kept (24 tiles at ZOFF), else h alternates in H (2 x 8 tiles); with Cs
// cos z_l is kept. hook(l, ot, h, c) per hidden element (h = sin z, c = cos z), mid(l) after layer
// l's epilogues (the caller issues the next pass's fragment loads there); V[i] (LDS) receives sample
// i's value when WANT_V — written by the team's wave 0 after the split's barrier; SYNC_V = false
// leaves out the barrier that would publish it (a caller that reads V only after later barriers).
// `red`: the team's NW x 64 floats.
template <bool WANT_V, int NW, bool SYNC_V = true, typename Hook, typename Mid>
__device__ void q4_critic_forward_f(const Q4CriticFwd<NW>& F, const float* X0, float* Cs, float* Hs, float* H,
                                    float* red, float* V, int wi, int lane, Hook&& hook, Mid&& mid) {
  auto epi = [&](int l, float* out) {
    return [&, l, out](int ot, float z) {
      float h, c;
#ifdef CACTO_CRITIC_ELU
      if ((F.act >> l) & 1) elu_pair(z, &h, &c);
      else
#endif
        fast_sincos(z, &h, &c);
      const int e = q4e(ot, lane);
      if (Cs) Cs[ZOFF[l] * 64 + e] = c;
      out[e] = h;
      hook(l, ot, h, c);
    };
  };
  const float* in = X0;
  float* out = Hs ? Hs + ZOFF[0] * 64 : H;
  F.f0.template run<true>(in, 4, wi, lane, epi(0, out));
  mid(0);
  __syncthreads();
  in = out;
  out = Hs ? Hs + ZOFF[1] * 64 : H + 8 * 64;
  F.f1.template run<true>(in, 4, wi, lane, epi(1, out));
  mid(1);
  __syncthreads();
  in = out;
  out = Hs ? Hs + ZOFF[2] * 64 : H;
  F.f2.template run<true>(in, 8, wi, lane, epi(2, out));
  mid(2);
  __syncthreads();
  in = out;
  out = Hs ? Hs + ZOFF[3] * 64 : H + 8 * 64;
  F.f3.template run<true>(in, 8, wi, lane, epi(3, out));
  mid(3);
  __syncthreads();
  if (WANT_V) {
    F.f4.template run<true>(8, out, red, wi, lane, [&](int, float v) {
      if ((lane & 15) == 0) V[lane >> 4] = v;
    });
    if (SYNC_V) __syncthreads();
  }
}

// Critic input gradient from the cos tiles Cs (net_common.h critic_first_backward), 8 waves:
// G4 = W5, D_l = G_{l+1} cos z_l, G_l = D_l W_l^T. G tiles (G1 at 0, G2 at 4, G3 at 8) when Gs,
// D via hookD(l, ot, d), dV/dx0 = G_0 through g0epi(lane, g) (wave 0; lane's element is feature
// lane & 15 of sample lane >> 4); mid() after the first transposed layer. d3_done: the caller's
// forward already wrote D_3 = W5 cos z3 into P (and its panel), so that step and its barrier go.
template <typename HookD, typename Mid, typename G0Epi>
__device__ void q4_critic_first_backward(const Q4CriticBwd& F, const float* Cs, float* P /* 2 x 8 tiles */,
                                         float* Gs, float* red, int wave, int lane, HookD&& hookD, Mid&& mid,
                                         G0Epi&& g0epi, bool d3_done = false) {
  const int goff[4] = {0, 0, 4, 8};
  float* D = P;
  if (!d3_done) {
    const int e = q4e(wave, lane);
    const float d = fmul(F.w5, Cs[ZOFF[3] * 64 + e]);
    D[e] = d;
    hookD(3, wave, d);
    __syncthreads();
  }
  auto epi = [&](int l, float* Dn) {
    return [&, l, Dn](int it, float g) {
      const int e = q4e(it, lane);
      if (Gs) Gs[goff[l] * 64 + e] = g;
      const float d = fmul(g, Cs[ZOFF[l - 1] * 64 + e]);
      Dn[e] = d;
      hookD(l - 1, it, d);
    };
  };
  float* Dn = P + 8 * 64;
  F.g3.run<false>(D, 8, wave, lane, epi(3, Dn));
  mid();
  __syncthreads();
  D = Dn;
  Dn = P;
  F.g2.run<false>(D, 4, wave, lane, epi(2, Dn));
  __syncthreads();
  D = Dn;
  Dn = P + 8 * 64;
  F.g1.run<false>(D, 4, wave, lane, epi(1, Dn));
  __syncthreads();
  D = Dn;
  F.g0.run<false>(4, D, red, wave, lane, [&](int, float g) { g0epi(lane, g); });
  __syncthreads();
}

// input normalisation of the F4 element e = 4 f + i (utils.py:17-24), norms loaded once
struct Q4Norm {
  float n, nT;
  int f, ns;
  bool on;
  __device__ __forceinline__ Q4Norm(const cacto_sys_params& p, int e) {
    ns = p.nb_state;
    on = p.normalize != 0;
    f = e >> 2;
    n = (float)p.state_norm[min(f, ns - 1)];
    nT = (float)p.state_norm[ns - 1];
  }
  __device__ __forceinline__ float forward(float s) const {
    if (f >= ns) return 0.f;
    if (!on) return s;
    if (f == ns - 1) return fsub(fmul(fdiv(s, nT), 2.0f), 1.0f);
    return fdiv(s, n);
  }
};

struct Q4CriticLds {
  float X0[64], XT[64], G0[64];
  float Cs[24 * 64];  // cos z_l
  float Hs[24 * 64];  // h_l = sin z_l
  float HT[16 * 64];  // the target forward's h ping-pong (waves 4-7)
  float G[16 * 64];
  float ZB[24 * 64];
  float GB[16 * 64];
  float red[Q4_NW * 64];
  float stage[4 * 64];  // gathered rows: [0] s, [1] s_next, [2] dV/dx, [3] (R, d, w) per sample
  float Vn[4], V[4], y[4], Vb[4], Vt2[4], Vx[4];
};

// one 4-sample tile of the critic chain (critic_chain's operations, F4 layout, 8 waves)
__device__ __forceinline__ void q4_critic_chain(Q4CriticLds& S, const int tile, const SysDevice* __restrict__ sdp,
                                                const NetView& C, const NetView& Tg, const ChainScalars& cs,
                                                const double* __restrict__ storage, const int32_t* __restrict__ idx,
                                                const float* __restrict__ isw, int B, const GradBufs& gb,
                                                float* __restrict__ y_out, float* __restrict__ V_out,
                                                float* __restrict__ Vt_out, int32_t* __restrict__ step) {
  float *X0 = S.X0, *XT = S.XT, *G0 = S.G0, *Cs = S.Cs, *Hs = S.Hs, *G = S.G, *ZB = S.ZB, *GB = S.GB, *red = S.red;
  const cacto_sys_params& p = sdp->p;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int team = wave >> 2, wi4 = wave & 3;  // the two 4-wave teams of the forward passes
  const int ns = p.nb_state, cols = 3 * ns + 3, s0 = tile * Q4_TILE;
  const int ld = gb.ld, Bp = gb.Bp;
  const bool sob = cs.w_S != 0.f;
  const int goff[4] = {0, 0, 4, 8};
  CSTAMP(0);
  if (tile == 0 && tid == 0 && step) step[0] += 1;  // Keras critic optimizer iterations

  // the forward passes' fragments, in flight during the row gathers: waves 0-3 the critic (forward
  // at s), waves 4-7 the target network (forward at s')
  Q4CriticFwd<4> F;
  const NetView& FN = team ? Tg : C;
  const float w5 = C.flat[C.t.woff[4] + 16 * wave + (lane & 15)];
  const Q4Norm nrm(p, lane);
  {
    // one (sample c, column) per lane, wave w gathers array w & 3: s, s_next, dV/dx, then (R, d, w)
    // (waves 4-7 repeat the loads of waves 0-3, so every wave runs the same branch-free load
    // sequence: index, row, then the fragments — a load under a wave branch would make the wait
    // for the rows include the fragments)
    const int c = lane >> 4, f = lane & 15, a = wave & 3;
    const bool valid = s0 + c < B;
    const int sc = min(s0 + c, B - 1), fc = min(f, ns - 1);
    const int32_t row = idx[sc];
    const int col = a == 0 ? fc : a < 3 ? a * ns + 1 + fc : (f == 0 ? ns : 3 * ns + 1);
    const double x = storage[(size_t)row * cols + col];
    const float wv = isw ? isw[sc] : 1.f;
    F.load<true>(FN, wi4, lane);
    F.load_last(FN, wi4, lane);
    const bool keep = valid && (a < 3 ? f < ns : f < 2);
    float v = keep ? (float)x : 0.f;
    if (a == 3 && f == 2) v = valid ? wv : 0.f;
    if (wave < 4) S.stage[wave * 64 + c * 16 + f] = v;
  }
  __syncthreads();
  if (wave < 2) {  // wave 0: X0, wave 1: XT (element lane = 4 f + i)
    const int f = lane >> 2, i = lane & 3;
    const float v = nrm.forward(S.stage[wave * 64 + i * 16 + min(f, 15)]);
    (wave == 0 ? X0 : XT)[lane] = v;
    if (wave == 0) gb.LT[0][(size_t)f * ld + Bp + s0 + i] = v;  // LT_0 second half: the input at s
  }
  __syncthreads();
  CSTAMP(1);
  const float* Rs = S.stage + 3 * 64;  // Rs[16 c] = R, [16 c + 1] = d, [16 c + 2] = w

  // forward at s (waves 0-3: sin z, cos z kept, h_l -> LT_l second half) beside the target
  // forward at s' (waves 4-7: V_tgt(s_next) for y = R + (1 - d) * V_tgt(s_next),
  // NeuralNetwork.py:153-158; run even for MC, whose y ignores it). The transposed fragments of the
  // backward passes are issued after layers 2 and 3. With the Sobolev term, D_3 = W5 cos z3 (the
  // first backward's input) is formed in the forward's last epilogue. V and V_tgt are read only
  // after the first backward's barriers, so the pass ends without the barrier that publishes them.
  const bool fuse_d3 = sob && !cs.want_vt;  // want_vt's extra pass reuses GB as scratch
  float w5t[2];                             // W5 at the lane's features of team 0's layer-3 tiles
#pragma unroll
  for (int t = 0; t < 2; ++t) w5t[t] = C.flat[C.t.woff[4] + 16 * (wi4 + 4 * t) + (lane & 15)];
  Q4CriticBwd HB;
  q4_critic_forward_f<true, 4, false>(
      F, team ? XT : X0, team ? nullptr : Cs, team ? nullptr : Hs, team ? S.HT : Hs, red + team * 4 * 64,
      team ? S.Vn : S.V, wi4, lane,
      [&](int l, int ot, float h, float c) {
        if (team == 0) {
          q4_store_panel(gb.LT[l + 1], ld, Bp + s0, ot, lane, h);
          if (l == 3 && fuse_d3) {
            const float d = fmul(w5t[ot >> 2], c);
            GB[q4e(ot, lane)] = d;
            q4_store_panel(gb.RT[3], ld, s0, ot, lane, d);
          }
        }
      },
      [&](int l) {
        if (l == 2) HB.load_g3(C, wave, lane);
        if (l == 3) HB.load_rest(C, wave, lane);
      });
  CSTAMP(2);
  if (cs.want_vt) {  // the extra V_tgt(s) of NeuralNetwork.py:178 (waves 4-7; waves 0-3 repeat into scratch)
    __syncthreads();  // the first pass's split finishers are done with `red`
    q4_critic_forward_f<true, 4>(F, X0, nullptr, nullptr, team ? S.HT : GB, red + team * 4 * 64,
                                 team ? S.Vt2 : S.Vx, wi4, lane, [](int, int, float, float) {}, [](int) {});
  }
  CSTAMP(3);
  // Vbar = (2 * ((wS/B) * w)) * (V - y) of the lane's sample (Keras MSE, SUM_OVER_BATCH_SIZE), every
  // lane for itself: it enters zbar_3 in the layer-3 epilogue below
  auto vbar = [&](int c) {
    const float y = cs.MC ? Rs[16 * c] : fadd(Rs[16 * c], fmul(fsub(1.f, Rs[16 * c + 1]), S.Vn[c]));
    const float wv = sob ? cs.w_S : 1.f;
    const float gl = fmul(fdiv(wv, (float)cs.B_global), Rs[16 * c + 2]);
    return fmul(fmul(2.f, gl), fsub(S.V[c], y));
  };
  auto outputs = [&]() {  // tid < 4: the value loss row of the output layer's panel, y / V / V_tgt outputs
    const int c = tid;
    const float y = cs.MC ? Rs[16 * c] : fadd(Rs[16 * c], fmul(fsub(1.f, Rs[16 * c + 1]), S.Vn[c]));
    gb.RT[4][Bp + s0 + c] = vbar(c);
    if (sob) gb.RT[4][s0 + c] = 1.f;  // dW5 += Gbar_4 (G_4 = W5[:, 0])
    if (s0 + c < B) {
      if (y_out) y_out[s0 + c] = y;
      if (V_out) V_out[s0 + c] = S.V[c];
      if (Vt_out && cs.want_vt) Vt_out[s0 + c] = S.Vt2[c];
    }
  };

  Q4CriticFwd<Q4_NW> SF;  // the forward fragments of the Sobolev passes (8-wave layout, no bias)
  if (sob) {
    // first backward: D_l -> RT_l first half; G_l kept; G_0 = dV/dx0 goes straight into the Sobolev
    // loss gradient w.r.t. dV/ds and then G_0 (NeuralNetwork.py:167-170), in the finisher of its
    // split layer (wave 0, lane = feature f of sample i)
    q4_critic_first_backward(
        HB, Cs, GB, G, red, wave, lane, [&](int l, int ot, float d) { q4_store_panel(gb.RT[l], ld, s0, ot, lane, d); },
        [&]() { SF.load<false>(C, wave, lane); },
        [&](int ln, float g) {
          const int f = ln & 15, i = ln >> 4;
          float gb0 = 0.f;
          if (f < ns - 1) {
            const float nf = (float)p.state_norm[f];
            auto nback = [&](float v) { return !p.normalize ? v : fdiv(v, nf); };  // not the time column
            const float gsq = fdiv(fmul(fdiv(1.f, (float)cs.B_global), Rs[16 * i + 2]), (float)(ns - 1));
            const float dvds = nback(g);
            const float yp = clog(dvds), yt = clog(S.stage[2 * 64 + i * 16 + f]);
            const float gyp = fmul(fmul(2.f, gsq), fsub(yp, yt));
            gb0 = nback(clog_backward(dvds, gyp));
          }
          GB[q4e(0, ln)] = gb0;
          gb.LT[0][(size_t)f * ld + s0 + i] = gb0;
        },
        fuse_d3);
    CSTAMP(4);
    CSTAMP(5);
    const float vb = vbar(lane >> 4);
    // backward of the first backward, l = 0..3, on the forward fragments (no bias); the layer-3
    // epilogue also adds the value loss's zbar_3 += (Vbar * W5) * cos(z3)
    auto sp_epi = [&](int l, float* nxt) {
      return [&, l, nxt](int ot, float acc) {
        const int e = q4e(ot, lane);
        const float sz = Hs[ZOFF[l] * 64 + e], cz = Cs[ZOFF[l] * 64 + e];
        const float gu = l < 3 ? G[goff[l + 1] * 64 + e] : w5;  // layer 3: out tile `wave`
#ifdef CACTO_CRITIC_ELU
        float zb = ((C.t.act >> l) & 1) ? fmul(fmul(acc, gu), act_d2(true, sz))  // elu: grad * exp(z) below 0
                                        : fmul(-fmul(acc, gu), sz);             // CosGrad: -grad * sin(x)
#else
        float zb = fmul(-fmul(acc, gu), sz);
#endif
        if (l == 3) zb = fadd(zb, fmul(fmul(vb, w5), cz));
        ZB[ZOFF[l] * 64 + e] = zb;
        const float gn = fmul(acc, cz);  // MulGrad into the upstream grad
        nxt[e] = gn;
        q4_store_panel(gb.LT[l + 1], ld, s0, ot, lane, gn);
      };
    };
    float* nA = GB + 8 * 64;
    SF.f0.run<false>(GB, 4, wave, lane, sp_epi(0, nA));
    __syncthreads();
    CSTAMP(6);
    SF.f1.run<false>(nA, 4, wave, lane, sp_epi(1, GB));
    __syncthreads();
    CSTAMP(7);
    SF.f2.run<false>(GB, 8, wave, lane, sp_epi(2, nA));
    __syncthreads();
    CSTAMP(8);
    SF.f3.run<false>(nA, 8, wave, lane, sp_epi(3, GB));
    if (tid < 4) outputs();
    __syncthreads();
    CSTAMP(9);
  } else {
    __syncthreads();  // V, V_tgt published
    for (int k = tid; k < ZOFF[3] * 64; k += Q4_THREADS) ZB[k] = 0.f;
    {  // zbar_3 = (Vbar * W5) * cos(z3): out tile `wave`
      const int e = ZOFF[3] * 64 + q4e(wave, lane);
      ZB[e] = fadd(0.f, fmul(fmul(vbar(lane >> 4), w5), Cs[e]));
    }
    if (tid < 4) outputs();
    __syncthreads();
  }
  CSTAMP(10);
  CSTAMP(11);
  // backward through the forward graph: zbar_{l-1} += (zbar_l W_l^T) * cos(z_{l-1})
  auto hb_epi = [&](int l) {
    return [&, l](int it, float acc) {
      const int e = ZOFF[l - 1] * 64 + q4e(it, lane);
      ZB[e] = fadd(ZB[e], fmul(acc, Cs[e]));
    };
  };
  auto store_rt = [&](int l) {
    for (int ot = wave; ot < C.t.OT[l]; ot += Q4_NW)
      q4_store_panel(gb.RT[l], ld, Bp + s0, ot, lane, ZB[ZOFF[l] * 64 + q4e(ot, lane)]);
  };
  store_rt(3);
  HB.g3.run<false>(ZB + ZOFF[3] * 64, 8, wave, lane, hb_epi(3));
  __syncthreads();
  CSTAMP(12);
  store_rt(2);
  HB.g2.run<false>(ZB + ZOFF[2] * 64, 4, wave, lane, hb_epi(2));
  __syncthreads();
  CSTAMP(13);
  store_rt(1);
  HB.g1.run<false>(ZB + ZOFF[1] * 64, 4, wave, lane, hb_epi(1));
  __syncthreads();
  CSTAMP(14);
  store_rt(0);
  CSTAMP(15);
  __syncthreads();
  CSTAMP_FLUSH;
}

__global__ void __launch_bounds__(Q4_THREADS)
    k_critic_grad_q4(const SysDevice* __restrict__ sdp, NetView C, NetView Tg, ChainScalars cs,
                     const double* __restrict__ storage, const int32_t* __restrict__ idx,
                     const float* __restrict__ isw, int B, GradBufs gb, float* __restrict__ y_out,
                     float* __restrict__ V_out, float* __restrict__ Vt_out, int32_t* __restrict__ step) {
  __shared__ Q4CriticLds S;
  q4_critic_chain(S, blockIdx.x, sdp, C, Tg, cs, storage, idx, isw, B, gb, y_out, V_out, Vt_out, step);
}

// ---------------------------------------------------------------- actor chain
struct Q4ActorLds {
  float X0[64], XS[64], G0[64], ZB3[64];
  float ZA[32 * 64];  // actor z1, z2
  float H[32 * 64];   // actor h ping-pong; later critic H (16 tiles) + actor zbar2 (16)
  float ZC[24 * 64];  // critic cos z at s'
  float red[Q4_NW * 64];
  float st[64], stn[64], gn[64];  // [sample][16]
  float A[Q4_TILE * CACTO_MAX_ACTION];
  float Fu[Q4_TILE * CACTO_MAX_STATE * CACTO_MAX_ACTION];
  float dra[Q4_TILE * CACTO_MAX_ACTION];
  double term_s[Q4_TILE];
  double dM[Q4_TILE * CACTO_MAX_JOINTS * CACTO_MAX_JOINTS];  // revolute chains: M(q) and h(q, v) per sample
  double dh[Q4_TILE * CACTO_MAX_JOINTS];
  // the system (joint table, tabled constant dynamics) copied at kernel entry: the float64
  // recursions read a joint's parameters in long dependent sequences, one global load latency each
  SysDevice sys;
};

// the revolute chains' dynamics of the tile's 4 samples spread over threads (chain_dynamics_spread,
// learn_kernels.hip)
template <int NJ>
__device__ __forceinline__ void q4_chain_dynamics(Q4ActorLds& S, const SysDevice& sd, int wave, int lane) {
  chain_dynamics_spread<NJ, Q4_TILE>(sd, S.st, S.A, S.dM, S.dh, S.stn, S.Fu, wave * 64 + lane);
}

// one 4-sample tile of the actor chain (actor_chain's operations, F4 layout, 8 waves). The actor's
// shape is fixed (ns -> 256 -> 256 -> na, ns, na <= 16: KT = 1 / 16 / 16, OT = 16 / 16 / 1).
template <int NJ>
__device__ __forceinline__ void q4_actor_chain(Q4ActorLds& S, const int tile, const SysDevice* __restrict__ sdp,
                                               const NetView& Ac, const NetView& C, const ChainScalars& cs,
                                               const double* __restrict__ storage, const int32_t* __restrict__ idx,
                                               int B, const GradBufs& gb, int32_t* __restrict__ step) {
  float *X0 = S.X0, *XS = S.XS, *G0 = S.G0, *ZB3 = S.ZB3, *ZA = S.ZA, *H = S.H, *ZC = S.ZC, *red = S.red;
  const SysDevice& sd = *sdp;
  const cacto_sys_params& p = sd.p;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int ns = p.nb_state, na = p.nb_action, cols = 3 * ns + 3, s0 = tile * Q4_TILE;
  const int ld = gb.ld;
  CSTAMP(0);
  if (tile == 0 && tid == 0 && step) step[1] += 1;  // Keras actor optimizer iterations
  // layer 1 (ns -> 256) and the wave's pair of layer-2 out tiles, in flight during the row gathers
  // (every wave loads the rows — waves 1-7 the same as wave 0 — so every wave runs one branch-free
  // load sequence: index, row, then the fragments; wave 0's wait for the rows excludes them)
  Q4Frags<1, 2, Q4_NW> F1;
  Q4Pair<16, Q4_NW> W2;
  {
    const int c = lane >> 4, f = lane & 15;
    const bool valid = s0 + c < B;
    const int sc = min(s0 + c, B - 1), fc = min(f, ns - 1);
    const double* rp = storage + (size_t)idx[sc] * cols;
    const double x = rp[fc], term = rp[3 * ns + 2];
    // the system copy (branch-free: clamped index, duplicates write the same value), issued right
    // after the rows so the first barrier's wait covers it and not the fragments
    constexpr int SDW = sizeof(SysDevice) / sizeof(double);
    static_assert(SDW <= 8 * 64 && sizeof(SysDevice) % sizeof(double) == 0, "one double of SysDevice per thread");
    const int k = min(tid, SDW - 1);
    const double sv = reinterpret_cast<const double*>(sdp)[k];
    F1.load<true>(Ac.fwd(0), Ac.biasp(0), 16, 256, wave, lane);
    W2.load(Ac.fwd(1), 0, wave, lane);
    reinterpret_cast<double*>(&S.sys)[k] = sv;
    if (wave == 0) {
      S.st[c * 16 + f] = (valid && f < ns) ? (float)x : 0.f;
      if (f == 0) S.term_s[c] = valid ? term : 0.0;
    }
  }
  __syncthreads();
  if (wave == 0) {  // input of layer 0 (normalised) -> LT_0
    const int f = lane >> 2, i = lane & 3;
    const float v = f < ns ? normalize_feature(p, f, S.st[i * 16 + f]) : 0.f;
    X0[lane] = v;
    gb.LT[0][(size_t)f * ld + s0 + i] = v;
  }
  __syncthreads();
  CSTAMP(1);
  // actor forward; z1, z2 kept; h1 -> LT_1, h2 -> LT_2
  auto lepi = [&](int l) {
    return [&, l](int ot, float z) {
      const float h = z > 0.f ? z : fmul(z, 0.3f);  // LeakyReLU(alpha=0.3)
      const int e = q4e(ot, lane);
      ZA[l * 16 * 64 + e] = z;
      H[l * 16 * 64 + e] = h;
      q4_store_panel(gb.LT[l + 1], ld, s0, ot, lane, h);
    };
  };
  F1.run<true>(X0, 16, wave, lane, lepi(0));
  Q4Split<2, Q4_NW> F3;  // the action layer (256 -> na)
  F3.load<true>(Ac.fwd(2), 16, Ac.biasp(2), na, wave, lane);
  __syncthreads();
  CSTAMP(10);
  q4_layer_pairs<16, true, Q4_NW>(Ac.fwd(1), H, wave, lane, lepi(1), Ac.biasp(1), W2);
  // the critic's forward fragments at s', in flight during the action layer and the dynamics (for
  // the revolute chains after the dynamics: their float64 recursions need the registers)
#ifndef Q4_EARLY_CF_NJ
#define Q4_EARLY_CF_NJ 2
#endif
  constexpr bool early_cf = NJ <= Q4_EARLY_CF_NJ;
  Q4CriticFwd<Q4_NW> CF;
  if (early_cf) CF.load<true>(C, wave, lane);
  __syncthreads();
  CSTAMP(11);
  F3.run<true>(16, H + 16 * 64, red, wave, lane, [&](int, float v) {
    const int f = lane & 15;
    if (f < na) S.A[(lane >> 4) * na + f] = v;
  });
  __syncthreads();
  CSTAMP(2);
  // dynamics at (s, a) in float64 from float32 tensors (environment.py:134-144, :353-362)
  if constexpr (NJ >= 3) {
    // revolute chains: spread over the workgroup; d reward / d a on wave 2 alongside
    if (wave == 2 && lane < Q4_TILE) {
      constexpr int NA = Dims<NJ>::NA;
      const int c = lane;
      float af[NA], g[NA];
#pragma unroll
      for (int i = 0; i < NA; ++i) af[i] = S.A[c * na + i];
      const double tc = S.term_s[c];
      const double w6 = 6 >= p.n_weights ? 0.0 : tc * p.w_terminal[6] + (1.0 - tc) * p.w_running[6];
      (void)reward_batch_f32<NA>(p, w6, af, 0.0, g);
#pragma unroll
      for (int i = 0; i < NA; ++i) S.dra[c * na + i] = g[i];
    }
    // (the 6-joint chain keeps its parameter reads on the scalar path: from LDS the compiler hoists
    // them all and spills)
    q4_chain_dynamics<NJ>(S, NJ <= 3 ? S.sys : sd, wave, lane);
  } else if (tid < Q4_TILE) {
    constexpr int NS = Dims<NJ>::NS, NA = Dims<NJ>::NA;
    const int c = tid;
    double s[NS], a[NA], sn[NS], F[NS * NA];
#pragma unroll
    for (int f = 0; f < NS; ++f) s[f] = (double)S.st[c * 16 + f];
#pragma unroll
    for (int i = 0; i < NA; ++i) a[i] = (double)S.A[c * na + i];
    const SysDevice& sl = S.sys;
    if constexpr (NJ > 0 && NJ <= 3) {
      if (p.const_dyn) env_simulate_derivative_const<NJ>(sl, s, a, true, sn, F);
      else env_simulate_derivative<NJ>(sl, s, a, true, sn, F);
    } else {
      env_simulate_derivative<NJ>(sl, s, a, true, sn, F);
    }
#pragma unroll
    for (int f = 0; f < 16; ++f) S.stn[c * 16 + f] = f < NS ? (float)sn[f] : 0.f;
#pragma unroll
    for (int k = 0; k < NS * NA; ++k) S.Fu[c * CACTO_MAX_STATE * CACTO_MAX_ACTION + k] = (float)F[k];
  } else if (tid >= 64 && tid < 64 + Q4_TILE) {
    // wave 1, alongside the dynamics: only d reward / d a enters the actor gradient
    // (NeuralNetwork.py:199-204), and only the control cost depends on a
    constexpr int NA = Dims<NJ>::NA;
    const int c = tid - 64;
    float af[NA], g[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) af[i] = S.A[c * na + i];
    const double tc = S.term_s[c];
    const double w6 = 6 >= p.n_weights ? 0.0 : tc * p.w_terminal[6] + (1.0 - tc) * p.w_running[6];
    (void)reward_batch_f32<NA>(p, w6, af, 0.0, g);
#pragma unroll
    for (int i = 0; i < NA; ++i) S.dra[c * na + i] = g[i];
  }
  if constexpr (NJ < 3) __syncthreads();
  CSTAMP(3);
  if (!early_cf) CF.load<true>(C, wave, lane);
  if (wave == 0) {
    const int f = lane >> 2, i = lane & 3;
    XS[lane] = f < ns ? normalize_feature(p, f, S.stn[i * 16 + f]) : 0.f;
  }
  __syncthreads();
  CSTAMP(4);
  // critic (already updated) at s': dV/dx0 (NeuralNetwork.py:190-195); V(s') is not used
  float* HC = H;             // 16 tiles
  float* ZB2 = H + 16 * 64;  // 16 tiles
  Q4CriticBwd CB;
  q4_critic_forward_f<false, Q4_NW>(CF, XS, ZC, nullptr, HC, red, nullptr, wave, lane, [](int, int, float, float) {},
                                    [&](int l) {
                                      if (l == 1) CB.load(C, wave, lane);
                                    });
  CSTAMP(5);
  // the backward layers' fragments (W3^T: KT = 1; W2^T: the wave's pair), in flight from the
  // middle of the critic's first backward through the dQ/da phase
  Q4Frags<1, 2, Q4_NW> B2;
  Q4Pair<16, Q4_NW> B1;
  q4_critic_first_backward(
      CB, ZC, HC, nullptr, red, wave, lane, [](int, int, float) {},
      [&]() {
        B2.load<false>(Ac.bwd(2), nullptr, 16, 256, wave, lane);
        B1.load(Ac.bwd(1), 0, wave, lane);
      },
      [&](int ln, float g) { G0[q4e(0, ln)] = g; });
  CSTAMP(6);
  // dQ/da = dV/ds' Fu + dr/da ; abar = -dQ/da / B  (NeuralNetwork.py:206-231)
  if (wave == 0) {  // d normalize / d s of every (state f, sample i) element at once
    const int f = lane >> 2, i = lane & 3;
    if (f < ns) S.gn[i * 16 + f] = normalize_backward(p, f, G0[lane]);
  }
  __syncthreads();
  if (wave == 0) {  // element (action j, sample i) = lane 4 j + i
    const int j = lane >> 2, i = lane & 3;
    float abar = 0.f;
    if (j < na && s0 + i < B) {
      float q = 0.f;
      for (int f = 0; f < ns; ++f) {
        const float t = fmul(S.gn[i * 16 + f], S.Fu[i * CACTO_MAX_STATE * CACTO_MAX_ACTION + f * na + j]);
        q = (f == 0) ? t : fadd(q, t);
      }
      q = fadd(q, S.dra[i * na + j]);
      abar = fmul(-q, fdiv(1.f, (float)cs.B_global));
    }
    ZB3[lane] = abar;
    gb.RT[2][(size_t)j * ld + s0 + i] = abar;
  }
  __syncthreads();
  CSTAMP(7);
  // zbar2 = (abar W3^T) * lrelu'(z2) ; zbar1 = (zbar2 W2^T) * lrelu'(z1)
  auto bepi = [&](int l) {
    return [&, l](int it, float acc) {
      const int e = q4e(it, lane);
      const float z = ZA[l * 16 * 64 + e];
      const float o = z > 0.f ? acc : fmul(acc, 0.3f);
      if (l == 1) ZB2[e] = o;
      q4_store_panel(gb.RT[l], ld, s0, it, lane, o);
    };
  };
  B2.run<false>(ZB3, 16, wave, lane, bepi(1));
  __syncthreads();
  CSTAMP(8);
  q4_layer_pairs<16, false, Q4_NW>(Ac.bwd(1), ZB2, wave, lane, bepi(0), nullptr, B1);
  CSTAMP(9);
  __syncthreads();
  CSTAMP_FLUSH;
#ifdef CACTO_STAMPS
  if (tile == 0 && tid == 0)
    for (int k_ = 0; k_ < 32; ++k_) g_astamps[k_] = cacto_stamp_s[k_];
#endif
}

template <int NJ>
__global__ void __launch_bounds__(Q4_THREADS)
    k_actor_grad_q4(const SysDevice* __restrict__ sdp, NetView Ac, NetView C, ChainScalars cs,
                    const double* __restrict__ storage, const int32_t* __restrict__ idx, int B, GradBufs gb,
                    int32_t* __restrict__ step) {
  __shared__ Q4ActorLds S;
  q4_actor_chain<NJ>(S, blockIdx.x, sdp, Ac, C, cs, storage, idx, B, gb, step);
}

// the critic chain of update t (workgroups [0, nct)) and the actor chain of update t - 1 (the rest)
// in one grid, as k_chain_pair. (Measured and not kept: idle CUs of this grid reading the weight
// images into their XCD's L2 ahead of the chains, +1 %: a CU's fragment stream is bounded by its
// own L2-to-CU rate, ~20-30 B/clk, not by where the lines come from.)
template <int NJ>
__global__ void __launch_bounds__(Q4_THREADS)
    k_chain_pair_q4(const SysDevice* __restrict__ sdp, NetView C, NetView Tg, NetView Ac, ChainScalars cs,
                    const double* __restrict__ storage, const int32_t* __restrict__ idx_c,
                    const float* __restrict__ isw, const int32_t* __restrict__ idx_a, int B, int nct, GradBufs gbc,
                    GradBufs gba, float* __restrict__ y_out, float* __restrict__ V_out, int32_t* __restrict__ step,
                    int nx) {
  constexpr size_t bytes = sizeof(Q4CriticLds) > sizeof(Q4ActorLds) ? sizeof(Q4CriticLds) : sizeof(Q4ActorLds);
  __shared__ __attribute__((aligned(16))) unsigned char smem[bytes];
  // workgroup -> (role, tile): the 2 nct tiles (critic tiles first) on nx of the 8 XCDs. Blocks b
  // and b + 8 are dealt to one XCD (observed dealing: only which XCD's L2 serves a tile depends on
  // it, never a result), so blocks with b % 8 >= nx exit at once and tile sl * nx + b % 8 runs on
  // block b, sl = b / 8: with nx < 8 each weight image is fetched into nx L2s instead of eight.
  const int x = blockIdx.x & 7, j = (blockIdx.x >> 3) * nx + x;
  if (x >= nx || j >= 2 * nct) return;
  if (j < nct) {
    q4_critic_chain(*reinterpret_cast<Q4CriticLds*>(smem), j, sdp, C, Tg, cs, storage, idx_c, isw, B, gbc, y_out,
                    V_out, nullptr, step);
  } else {
    q4_actor_chain<NJ>(*reinterpret_cast<Q4ActorLds*>(smem), j - nct, sdp, Ac, C, cs, storage, idx_a, B, gba, step);
  }
}

}  // namespace cacto
