// Network kernels: weight packing, actor/critic inference, critic input gradient (the rollout
// kernel is in rollout_kernels.hip).
#include "net_common.h"

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

}  // namespace cacto

using namespace cacto;

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
