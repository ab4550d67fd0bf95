// Host-side handle layout shared by the translation units of libcacto_hip.so.
#pragma once

#include <mutex>

#include "env.h"
#include "mlp.h"

struct cacto_sys {
  cacto::SysDevice host;  // host copy (validated)
  cacto::SysDevice* dev;  // device copy read by every kernel
  cacto::NetTopo actor, critic;
  void* ddp_ws = nullptr;  // cacto_ddp_backward's per-step derivative records (grow-only)
  size_t ddp_ws_bytes = 0;
  hipStream_t side = nullptr;  // cacto_update_n's actor-step stream and its events
  hipEvent_t ev_critic = nullptr, ev_actor[3] = {nullptr, nullptr, nullptr};
  std::mutex pipe_mu;  // one two-stream pipeline at a time per handle (they share side / events)
  // pinned host copy of pipe_sig[1] (the device waits' timeout latch), refreshed asynchronously at
  // the end of every pipelined call with device-side waits; read (and cleared) by
  // cacto_pipeline_check after a stream synchronisation, refused on at the start of the next call
  unsigned long long* latch_host = nullptr;
  // device-side ordering of the two-stream pipeline: pipe_sig[0] counts the actor iterations whose
  // chain has finished, [2] the critic Adam steps finished (both monotonic over the handle's life),
  // [1] latches a wait that timed out, [3] is k_adam's last-workgroup counter, [4..7] the one-time
  // concurrency probe's words; pipe_seq is the host's count of pipeline iterations issued before
  // this call; pipe_probe: -1 not run yet, 0 the streams' kernels did not run concurrently (queue
  // markers), 1 they did (device-side waits)
  unsigned long long* pipe_sig = nullptr;
  unsigned long long pipe_seq = 0;
  int pipe_probe = -1;
  // data-parallel updates over RCCL (cacto_dp_attach): one communicator per stream of the pipeline
  // (critic stream, side stream: each orders its own collectives), the all-reduced gradients (one
  // flat buffer per network) and the PER shard statistics ([3] this rank's, [world][3] all ranks')
  void* dp_comm[2] = {nullptr, nullptr};
  int dp_rank = 0, dp_world = 0;
  float *dp_gc = nullptr, *dp_ga = nullptr;
  double* dp_stats = nullptr;
  // k_wgrad_adam work lists, [8 XCD bins][wa_stride] item codes (layer << 16 | net << 15 | item, -1 = none), for
  // the critic alone, the actor alone and both (built at creation, cacto_build_wgrad_adam_items)
  int32_t* wa_items[3] = {nullptr, nullptr, nullptr};
  int wa_stride[3] = {0, 0, 0};
};

namespace cacto {
inline const NetTopo& topo(const cacto_sys* s, int net) { return net == CACTO_NET_ACTOR ? s->actor : s->critic; }
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int64_t flat_span(const NetTopo& t) { return ((int64_t)t.params + 63) / 64 * 64; }
}  // namespace cacto

cacto::NetView cacto_make_view(const cacto_sys* sys, int net, const float* netbuf);
int cacto_const_dyn_init(cacto_sys* sys);  // SysDevice::cd_* of a prismatic-only chain (env_kernels.hip)
int cacto_build_wgrad_adam_items(cacto_sys* sys);  // learn_kernels.hip
void cacto_dp_release(cacto_sys* sys);  // learn_kernels.hip: the RCCL communicators and buffers
// replay_kernels.hip: batches from this size on take the multi-workgroup PER kernels; the update
// pipelines then issue the sample's exp_counter increment just before the priority update (its only
// reader), off the sample -> critic chain path
int cacto_per_mw_min();
int cacto_per_count_launch(const int32_t* idx_d, int B, double* exp_counter_d, hipStream_t st);
int cacto_per_update_count(double* sum_tree_d, double* min_tree_d, int64_t capacity, const int32_t* idx_d,
                           const float* y_d, const float* V_d, double* exp_counter_d, double fresh_factor, double eps,
                           double alpha, double* max_priority_d, int B, hipStream_t st);
int cacto_per_sample_runs_launch(const double* sum_tree_d, const double* min_tree_d, int64_t capacity, int64_t max_idx,
                                 double beta, const double* uniforms_d, int B, int32_t* idx_d, float* is_w_d,
                                 int32_t* runs_d, hipStream_t st, const double* shards_d = nullptr,
                                 int n_shards = 0);
