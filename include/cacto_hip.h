/*
 * cacto_hip.h — C-ABI of libcacto_hip.so, the MI355X (gfx950) hot path of CACTO.
 *
 * Drop-in boundary for the data-parallel hot path of nadimkanazi/cacto (reference paths below are
 * relative to its repository root). Each entry point replaces a Python/TF/Pinocchio call site:
 *
 *   cacto_env_step_batch   Env.simulate_batch + derivative_batch + reward_batch (+ dr/da tape)
 *                          environment.py:134-144, :277-286 (and per-system overrides); as called
 *                          from NN.compute_actor_grad NeuralNetwork.py:188, :199-204
 *   cacto_env_step         Env.step + get_end_effector_position (float64 rollout semantics)
 *                          environment.py:70-78, :146-156; plot_utils.py:262-264
 *   cacto_env_jacobians    Env.augmented_derivative environment.py:111-132 (as called by TO.py:181)
 *   cacto_env_bound_control_cost  Env.bound_control_cost environment.py:158-163
 *   cacto_rollout          RL_AC.create_TO_init loop RL.py:223-231 / PLOT.rollout plot_utils.py:245-279
 *   cacto_rollout_rewards  Env.step reward / get_end_effector_position over recorded trajectories
 *   cacto_ddp_backward     TO.backward_pass TO.py:119-202 (dV/dx Sobolev labels)
 *   cacto_mlp_pack         (layout transform for the kernels; no reference counterpart)
 *   cacto_sys_set_critic_type  RL_AC.setup_model's critic_type choice RL.py:65-76 ('sine' /
 *                          'sine-elu', NeuralNetwork.py:80-108)
 *   cacto_actor_forward    NN.eval(actor, s)  NeuralNetwork.py:130-138 (+ utils.py:17-24)
 *   cacto_critic_forward   NN.eval(critic, s)
 *   cacto_critic_input_grad tape.gradient(V, s)  NeuralNetwork.py:162-165, :190-195
 *   cacto_critic_grad      NN.compute_critic_grad  NeuralNetwork.py:150-178
 *   cacto_actor_grad       NN.compute_actor_grad   NeuralNetwork.py:180-233
 *   cacto_adam_step        optimizer.apply_gradients RL.py:105, :109 (Keras-2.11 Adam, RL.py:79-88)
 *   cacto_soft_update      RL_AC.update_target RL.py:113-118
 *   cacto_update           RL_AC.update + update_target (one learn_and_update iteration, RL.py:122-137)
 *   cacto_update_n[_per]   the learn_and_update loop RL.py:120-143 for K updates (with PER:
 *                          sample -> update -> priority update), pipelined on two streams
 *   cacto_buffer_gather    ReplayBuffer.sample row gather replay_buffer.py:47-61
 *   cacto_buffer_add       ReplayBuffer.add ring write replay_buffer.py:25-36
 *   cacto_rl_solve_add     RL_AC.RL_Solve n-step targets RL.py:145-189 fused with the
 *                          buffer.add of its output (main.py:240)
 *   cacto_per_*            PrioritizedReplayBuffer + segment trees replay_buffer.py:87-218,
 *                          segment_tree.py:4-145
 *
 * Conventions
 *   - Every pointer argument named *_d is DEVICE memory (e.g. torch tensor .data_ptr()), contiguous
 *     row-major. Host pointers are named *_h. The library never frees caller memory.
 *   - Every call is asynchronous on `stream` (a hipStream_t passed as void*; NULL = default stream)
 *     and enqueues no host synchronisation, so sequences can be captured into a hipGraph.
 *     cacto_update_n[_per] also use a side stream owned by the handle, joined back into `stream`
 *     before they return; cacto_ddp_backward (car_park, revolute chains) grows a device workspace
 *     owned by the handle (a hipMalloc, so warm it up before capturing).
 *   - Return 0 on success, <0 on error; cacto_last_error() returns a thread-local message.
 *     No C++ exception crosses the ABI.
 *   - Handles (cacto_sys) are created/destroyed by the caller; concurrent calls on one handle are
 *     undefined (as in the reference's single-threaded loop).
 */
#ifndef CACTO_HIP_H
#define CACTO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CACTO_ABI_VERSION 1

/* error codes */
#define CACTO_OK 0
#define CACTO_EINVAL -1
#define CACTO_EHIP -2
#define CACTO_ENOMEM -3
#define CACTO_EUNSUPPORTED -4

/* dynamics kinds */
#define CACTO_DYN_SINGLE_INTEGRATOR 0 /* environment.py:235-243 */
#define CACTO_DYN_CHAIN 1             /* Pinocchio chain: robot_utils.py:348-432 */
#define CACTO_DYN_CAR 2               /* environment.py:437-448 */
#define CACTO_DYN_CAR_PARK 3          /* environment.py:584-595 */

/* reward kinds */
#define CACTO_REW_PLANAR 0      /* SI / DI / Car: environment.py:252-275, :329-351, :457-480 */
#define CACTO_REW_MANIPULATOR 1 /* planar + w2*|v|^2 when w2 != 0: environment.py:695-723 */
#define CACTO_REW_UR5 2         /* 3-D ellipsoids: environment.py:780-805 */
#define CACTO_REW_CAR_PARK 3    /* smooth-box obstacles: environment.py:604-641 */

#define CACTO_MAX_STATE 16
#define CACTO_MAX_ACTION 8
#define CACTO_MAX_JOINTS 6
#define CACTO_JOINT_COLS 27 /* parent, type, axis[3], R[9], p[3], mass, com[3], I[6] */

/* System description: the numeric content of a conf_*.py module the hot path reads. */
typedef struct {
  int32_t dyn_kind;
  int32_t reward_kind;
  int32_t nb_state;  /* ns = nx + 1 (time last) */
  int32_t nb_action; /* na */
  int32_t nq, nv;    /* chain only */
  int32_t normalize; /* NORMALIZE_INPUTS */
  int32_t n_joints;  /* chain only */
  int32_t ee_parent; /* chain only: joint index of the 'EE' frame's parent */
  int32_t n_check;   /* car_park only */
  int32_t n_weights; /* length of cost_weights_* (7, car_park 8) */
  int32_t const_dyn; /* filled by cacto_sys_create: 1 if every joint is prismatic, so M and nle
                      * do not depend on the state (DI) — input value ignored */
  double dt;
  double state_norm[CACTO_MAX_STATE];
  double u_max[CACTO_MAX_ACTION];
  double w_b;
  double scale, offset;  /* cost_funct_param[1], [0] */
  double alpha, alpha2;  /* soft_max_param */
  double obs[18];        /* obs_param */
  double target[3];      /* TARGET_STATE */
  double w_running[8];   /* cost_weights_running */
  double w_terminal[8];  /* cost_weights_terminal */
  double L_delta, tau_delta, k_db; /* car / car_park */
  double check_points[20];         /* car_park check_points_BF (x, y) pairs */
  double ee_R[9], ee_p[3];         /* chain: EE frame placement in its parent joint frame */
  double gravity[3];               /* chain: model.gravity linear part */
} cacto_sys_params;

typedef struct cacto_sys cacto_sys;

const char* cacto_last_error(void);
int cacto_abi_version(void);

/* joint_table_h: n_joints x CACTO_JOINT_COLS float64 (host), see cacto_amd/robots.py */
int cacto_sys_create(const cacto_sys_params* params_h, const double* joint_table_h, cacto_sys** out);
int cacto_sys_destroy(cacto_sys* sys);
/* The critic's hidden activations (RL.py:65-76 critic_type): 0 = 'sine' (4 SIREN layers, the
 * default, every shipped config), 1 = 'sine-elu' (NeuralNetwork.py:80-93: sine, elu, sine, elu
 * layers of the same widths). Set before creating or updating critic networks of this handle; the
 * 'elu' and 'relu' critics (16, 32, 256, 256 wide) are not built (CACTO_EINVAL). */
int cacto_sys_set_critic_type(cacto_sys* sys, int critic_type);

/* ---------------------------------------------------------------- environment ------------ */

/* compute_actor_grad's environment calls for a batch (float32 tensors in/out, float64 math):
 *   S_next = simulate_batch(S, A); Fu = derivative_batch(S, A);
 *   R = reward_batch(W, S, A); dR_dA = d R / d A  (TF tape over u_cost)
 * W: W_d [B, n_weights] float64 if given, else term*cost_weights_terminal +
 * (1-term)*cost_weights_running from term_d [B] (NeuralNetwork.py:197-201), else running weights.
 * Any output pointer may be NULL. Shapes: S [B,ns], A [B,na], S_next [B,ns], Fu [B,ns,na], R [B],
 * dR_dA [B,na]. */
int cacto_env_step_batch(const cacto_sys* sys, const float* S_d, const float* A_d, const double* term_d,
                         const double* W_d, float* S_next_d, float* Fu_d, float* R_d, float* dR_dA_d, int B,
                         void* stream);

/* get_end_effector_position for B float64 states: EE_d [B,3] (environment.py:146-156). */
int cacto_env_ee(const cacto_sys* sys, const double* S_d, double* EE_d, int B, void* stream);

/* Env.step(W, s, a) in float64 plus the EE position of the next state, for B independent rows.
 * W_d may be NULL (running weights). EE_d [B,3], any output may be NULL. */
int cacto_env_step(const cacto_sys* sys, const double* S_d, const double* A_d, const double* W_d,
                   double* S_next_d, double* R_d, double* EE_d, int B, void* stream);

/* Env.augmented_derivative(s, a) (environment.py:111-132; SI :221-233, Car :420-435, CarPark
 * :567-582) for B float64 rows S_d [B,ns], A_d [B,na]: Fx_d [B,nx,nx] = I + dt*[[0,I],[ddq_dq,ddq_dv]]
 * (closed forms for SI / car / car_park / the prismatic DI pair; hyper-dual RNEA for revolute chains,
 * computeABADerivatives) and Fu_d [B,nx,na] = dt*[0; M^-1] (not normalised), nx = ns-1. Called by the
 * host TO backward pass (TO.py:181); cacto_ddp_backward evaluates the same device code inline. */
int cacto_env_jacobians(const cacto_sys* sys, const double* S_d, const double* A_d, int B, double* Fx_d,
                        double* Fu_d, void* stream);

/* Env.bound_control_cost(a) (environment.py:158-163) for B float64 action rows A_d [B,na]:
 * out_d[b] = sum_i a_i^2 + w_b*(a_i/u_max_i)^10, accumulated in action order. */
int cacto_env_bound_control_cost(const cacto_sys* sys, const double* A_d, double* out_d, int B, void* stream);

/* ---------------------------------------------------------------- networks --------------- */

/* Flat parameter layout = Keras trainable_variables order, kernels [in,out] row-major:
 *   actor : W1[ns,256] b1 W2[256,256] b2 W3[256,na] b3            (NeuralNetwork.py:51-63)
 *   critic: W1[ns,64] b1 W2[64,64] b2 W3[64,128] b3 W4[128,128] b4 W5[128,1] b5  (:95-108)
 * A "net buffer" is one float32 device buffer [flat params | pad to 64 | packed MFMA fragments]
 * of cacto_mlp_netbuf_floats() floats. cacto_mlp_pack() refreshes the packed part from the flat
 * part (the Adam kernels keep both in sync during training). */
#define CACTO_NET_ACTOR 0
#define CACTO_NET_CRITIC 1
int64_t cacto_mlp_param_count(const cacto_sys* sys, int net);
int64_t cacto_mlp_netbuf_floats(const cacto_sys* sys, int net);
int cacto_mlp_pack(const cacto_sys* sys, int net, float* netbuf_d, void* stream);

/* NN.eval: normalisation inside, float32. A [B,na], V [B], dVdS [B,ns] (w.r.t. the raw state). */
int cacto_actor_forward(const cacto_sys* sys, const float* actor_netbuf_d, const float* S_d, float* A_d,
                        int B, void* stream);
int cacto_critic_forward(const cacto_sys* sys, const float* critic_netbuf_d, const float* S_d, float* V_d,
                         int B, void* stream);
int cacto_critic_input_grad(const cacto_sys* sys, const float* critic_netbuf_d, const float* S_d,
                            float* V_d, float* dVdS_d, int B, void* stream);

/* ---------------------------------------------------------------- learner ---------------- */

/* Network state for an update: flat params + Adam moments (+ packed copies maintained by Adam). */
typedef struct {
  float* actor_d;  float* actor_m_d;  float* actor_v_d;   /* net buffer + flat Adam moments */
  float* critic_d; float* critic_m_d; float* critic_v_d;
  float* target_d;                                        /* target critic net buffer */
  int32_t* step_d; /* device counters = Keras optimizer iterations: [0] critic, [1] actor.
                    * cacto_critic_grad / cacto_actor_grad increment their counter; the following
                    * cacto_adam_step uses it as `iterations + 1`. */
} cacto_nets;

typedef struct {
  double w_S;         /* Sobolev weight (main.py --w-S) */
  double tau;         /* UPDATE_RATE */
  double beta1, beta2, epsilon; /* Keras Adam defaults 0.9, 0.999, 1e-7 (python floats) */
  double critic_lr[5]; /* PiecewiseConstantDecay values (all equal when LR_SCHEDULE = 0) */
  double actor_lr[5];
  double lr_bounds[4]; /* boundaries (in iterations) */
  int32_t MC;         /* conf.MC */
  int32_t B_global;   /* batch size the loss means are taken over (= B on one GPU) */
  int32_t want_target_V; /* also compute V_tgt(s) (NeuralNetwork.py:178) */
  int32_t pad;
} cacto_update_cfg;

/* Replay rows are float64 [s | R | s_next | dVdx | d | term] (3ns+3 columns, replay_buffer.py:20). */

/* Bytes of workspace cacto_critic_grad / cacto_actor_grad / cacto_update need for batch B. */
size_t cacto_workspace_bytes(const cacto_sys* sys, int B);

/* Critic gradient (flat, Keras order, summed over the B local rows with 1/B_global scaling).
 * rows: storage_d indexed by idx_d[B] (int32); is_w_d = IS weights [B] or NULL (= 1).
 * Outputs: grad_d [PC]; y_d [B] (reward_to_go), V_d [B], Vt_d [B] (if cfg->want_target_V). */
int cacto_critic_grad(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                      const double* storage_d, const int32_t* idx_d, const float* is_w_d, int B,
                      float* grad_d, float* y_d, float* V_d, float* Vt_d,
                      void* workspace_d, size_t workspace_bytes, void* stream);

/* Actor gradient against the CURRENT critic (call after the critic step, RL.py:104-109). */
int cacto_actor_grad(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                     const double* storage_d, const int32_t* idx_d, int B, float* grad_d,
                     void* workspace_d, size_t workspace_bytes, void* stream);

/* Keras-2.11 Adam on a flat tensor + packed copy refresh; `which` = CACTO_NET_*.
 * The iteration counter nets->step_d[which] is read and incremented on the device.
 * For the critic this also performs the soft target update when soft_update != 0. */
int cacto_adam_step(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg, int which,
                    const float* grad_d, int soft_update, void* stream);

/* target <- tau*critic + (1-tau)*target (and its packed copy) */
int cacto_soft_update(const cacto_sys* sys, const cacto_nets* nets, float tau, void* stream);

/* One full RL_AC.update + update_target (single device): critic grad -> Adam(critic) + soft
 * update -> actor grad (new critic) -> Adam(actor). */
int cacto_update(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                 const double* storage_d, const int32_t* idx_d, const float* is_w_d, int B,
                 float* y_d, float* V_d, float* Vt_d, void* workspace_d, size_t workspace_bytes,
                 void* stream);

/* Diagnostic: the two-stream pipeline's device-side ordering words: out4_h[0] actor chains finished,
 * [1] 1 if a device-side wait timed out since the last cacto_pipeline_check (the waits are bounded
 * so that an ordering fault cannot hang the GPU), [2] critic Adam steps finished, [3] the handle's
 * concurrency probe: 0 not run, 1 the two streams' kernels did not run concurrently (queue markers
 * order them), 2 they did (device-side waits). Synchronizes the device. All zero before the first
 * pipelined call. */
int cacto_pipeline_status(const cacto_sys* sys, unsigned long long* out4_h);
/* Collects the two-stream pipeline's timeout latch: synchronizes `stream` (the stream the pipelined
 * calls were issued on), and if a device-side wait of any cacto_update_n[_per] call since the last
 * check timed out — its updates then ran without their cross-stream order — clears the latch and
 * returns CACTO_EINVAL (the message says so); otherwise CACTO_OK. A set latch also makes the next
 * pipelined call refuse to run until it is collected. The Python layer calls it at the end of every
 * learn_and_update and before every checkpoint save (RL.py:139-143), so no result of a timed-out
 * call leaves unflagged. Ordering: device-side waits are the default; queue markers are used while
 * the stream is being captured into a graph, when the environment serializes kernels
 * (AMD_SERIALIZE_KERNEL, HIP_LAUNCH_BLOCKING) and when a one-time probe per handle finds that the
 * two streams' kernels do not run concurrently (e.g. under counter collection);
 * CACTO_PIPE_DEVWAIT=0 / 1 forces markers / device waits. */
int cacto_pipeline_check(cacto_sys* sys, void* stream);
/* K consecutive updates on minibatch indices idx_d [K][B] (learn_and_update's loop with its
 * minibatches drawn up front, RL.py:120-143; no IS weights). Bit-identical to K cacto_update calls.
 * The critic step of update t+1 overlaps the actor step of update t (the critic step never reads
 * the actor): for batches of at most 512 the two chains run as one grid on `stream` (three launches
 * per update); larger batches use a second stream owned by the system handle, joined back into
 * `stream` before the call returns (also on error). Calls on one handle are serialised internally
 * (a mutex), so two host threads may call it, but their updates are not interleaved. */
int cacto_update_n(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                   const double* storage_d, const int32_t* idx_d, int K, int B, void* workspace_d,
                   size_t workspace_bytes, void* stream);

/* The same pipeline for learn_and_update with PER (RL.py:122-137): per update, the stratified
 * sample (uniforms_d [K][B], as cacto_per_sample) -> update with IS weights -> priority update
 * (as cacto_per_update); bit-identical to the K-step sequential loop. */
int cacto_update_n_per(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                       const double* storage_d, double* sum_tree_d, double* min_tree_d, int64_t capacity,
                       int64_t max_idx, double beta, const double* uniforms_d, double* exp_counter_d,
                       double fresh_factor, double eps, double alpha, double* max_priority_d, int K, int B,
                       void* workspace_d, size_t workspace_bytes, void* stream);

/* Data-parallel K-update loop (RL.py:101-118 per update, replaces the two blocking all-reduces of
 * learn_and_update's DP form with one per update). The host runs K + 1 steps; step t computes the
 * gradient of the critic step of update t (idx_c_d != NULL, with is_w_d / y_d / V_d as in
 * cacto_update) and of the actor step of update t - 1 (idx_a_d != NULL) into
 * grad_d [critic params | actor params] (each scaled by 1/cfg->B_global, so the exchange is a plain
 * sum), the caller all-reduces the present part(s) of grad_d once, then cacto_update_pair_apply runs
 * the Adam steps (critic with the soft target update when soft_update). The actor gradient of
 * update t - 1 is taken against the critic after its update t - 1, as in the sequential loop. */
int cacto_update_pair_grads(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                            const double* storage_d, const int32_t* idx_c_d, const float* is_w_d,
                            const int32_t* idx_a_d, int B, float* grad_d, float* y_d, float* V_d,
                            void* workspace_d, size_t workspace_bytes, void* stream);
/* cacto_update_pair_grads in two stream-ordered stages, so the critic part's all-reduce can be
 * issued while the actor part is still being formed: stage 0 runs the chain(s) and writes the
 * critic gradient (when idx_c_d), stage 1 the actor's weight gradient into grad_d + P_critic (when
 * idx_a_d; a no-op otherwise). Stage 1 reads the panels stage 0 left in the workspace, so the two
 * calls take the same arguments, stage 0 first, on the same stream. Stage 0 + stage 1 = one
 * cacto_update_pair_grads call, bit for bit. */
int cacto_update_pair_grads_stage(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                                  const double* storage_d, const int32_t* idx_c_d, const float* is_w_d,
                                  const int32_t* idx_a_d, int B, float* grad_d, float* y_d, float* V_d,
                                  void* workspace_d, size_t workspace_bytes, int stage, void* stream);
int cacto_update_pair_apply(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                            const float* grad_d, int critic, int actor, int soft_update, void* stream);

/* Data-parallel learn_and_update over RCCL (main.py:219-225's parallelism as one process per GPU,
 * SURVEY §8e). cacto_dp_unique_ids writes n RCCL unique ids (128 bytes each) on one rank; every
 * rank then calls cacto_dp_attach with the same 2 ids (collective: it returns once all `world`
 * ranks have joined), which gives the handle one communicator per stream of the update pipeline.
 * The RCCL library is the one already loaded in the process (torch.distributed's), else
 * librccl.so.1. cacto_dp_detach releases them (cacto_sys_destroy does too). */
int cacto_dp_unique_ids(void* out_h, int n);
int cacto_dp_attach(cacto_sys* sys, const void* ids_h, int rank, int world);
int cacto_dp_detach(cacto_sys* sys);
/* K data-parallel updates (RL.py:101-118 each) on this rank's minibatch indices idx_d [K][B] (B =
 * the local batch; cfg->B_global = B * world, the gradients are scaled by 1 / B_global so the
 * exchange is a plain sum): the two-stream pipeline of cacto_update_n with each network's gradient
 * all-reduced on its own stream's communicator between its GEMM and its Adam step. Every rank
 * applies the same Adam to the same sum, so the replicas stay identical; with one rank the result
 * equals cacto_update_n bit for bit. */
int cacto_update_n_dp(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                      const double* storage_d, const int32_t* idx_d, int K, int B, void* workspace_d,
                      size_t workspace_bytes, void* stream);
/* The same with PER (RL.py:122-137 on every rank's replay shard): per update this shard's (sum,
 * min, rows) exchanged over the critic stream's communicator (its row of a [world][3] table, the
 * other rows zero, sum all-reduced — the all-gather of the statistics), the stratified sample with IS
 * weights against the union (cacto_per_sample_global), the update, then this shard's priority
 * update. Arguments as cacto_update_n_per. */
int cacto_update_n_per_dp(const cacto_sys* sys, const cacto_nets* nets, const cacto_update_cfg* cfg,
                          const double* storage_d, double* sum_tree_d, double* min_tree_d, int64_t capacity,
                          int64_t max_idx, double beta, const double* uniforms_d, double* exp_counter_d,
                          double fresh_factor, double eps, double alpha, double* max_priority_d, int K, int B,
                          void* workspace_d, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- rollouts --------------- */

/* B episodes from S0_d [B,ns] (float64), each for nsteps_d[b] <= T steps:
 *   a_t = actor(s_t) (float32; zeros when use_actor == 0, i.e. ep == 0 in RL.py:224-225),
 *   s_{t+1}, r_t = Env.step(W, s_t, a_t), ee_{t+1} = EE(s_{t+1}).
 * Outputs (any may be NULL): S_traj [B,T+1,ns] f64, A_traj [B,T,na] f32, R_traj [B,T] f64,
 * EE_traj [B,T+1,3] f64. Steps past nsteps_d[b] are not written. W_d: weights [n_weights] or NULL
 * (running). status_d [B] int32 (optional): 0 ok, 1 NaN state encountered (RL.py:229-231).
 * R_traj / EE_traj are evaluated from the recorded trajectory after the sequential pass
 * (cacto_rollout_rewards), so they need S_traj (and A_traj when use_actor).
 * order_d [B] int32 (optional): a permutation of the episodes, longest first (e.g. a stable
 * argsort of -nsteps). Its ranks are dealt to the workgroups in snake order and each workgroup's
 * episode slots take them longest first as earlier episodes end, so every slot runs about the same
 * number of steps. Results do not depend on the order or on the schedule. */
int cacto_rollout(const cacto_sys* sys, const float* actor_netbuf_d, const double* S0_d,
                  const int32_t* nsteps_d, int T, int use_actor, const double* W_d,
                  double* S_traj_d, float* A_traj_d, double* R_traj_d, double* EE_traj_d,
                  int32_t* status_d, const int32_t* order_d, int B, void* stream);

/* cacto_rollout with an explicit schedule: `groups` 4-episode groups per workgroup (1, 2 or 4;
 * 0 = automatic: about two episodes per slot) or, for systems whose step needs no workgroup-wide
 * dynamics (SI, car, car_park and the prismatic DI), an 8-slot workgroup kind: -1 = two
 * independent 4-slot teams (k_rollout_tt), -3 = one slot per wave with layer 2 split over K, the
 * layer-2 weights in registers (k_rollout_ks; automatic for those systems up to two episodes per
 * slot); and `workgroups` (0 = one per CU, capped by B).
 * Same outputs as cacto_rollout for any schedule (tests use it to force slot refills and to
 * compare the kernels). */
int cacto_rollout_sched(const cacto_sys* sys, const float* actor_netbuf_d, const double* S0_d,
                        const int32_t* nsteps_d, int T, int use_actor, const double* W_d,
                        double* S_traj_d, float* A_traj_d, double* R_traj_d, double* EE_traj_d,
                        int32_t* status_d, const int32_t* order_d, int B, int groups, int workgroups,
                        void* stream);

/* Env.step's reward r_t = reward(W, s_t, a_t) (t < nsteps[b]) and EE_t = EE(s_t) (t <= nsteps[b])
 * of recorded trajectories (environment.py:70-78, :146-156): S_traj [B,T+1,ns] f64, A_traj
 * [B,T,na] f32 (ignored, a = 0, when use_actor == 0), outputs R_traj [B,T] / EE_traj [B,T+1,3] f64
 * (either may be NULL). NaN states (a dropped episode) are skipped. Fully parallel over (b, t);
 * cacto_rollout calls it when R_traj or EE_traj is requested. */
int cacto_rollout_rewards(const cacto_sys* sys, const double* S_traj_d, const float* A_traj_d,
                          const int32_t* nsteps_d, int T, int use_actor, const double* W_d,
                          double* R_traj_d, double* EE_traj_d, int B, void* stream);

/* Sobolev labels without CasADi: the DDP backward pass of TO.backward_pass
 * (TO.py:119-202) along n_ep recorded trajectories. Episode e has Te = nsteps_d[e] steps:
 *   S_traj_d [n_ep, ldS, ns] f64 (s_0..s_Te; the time column is ignored), U_traj_d [n_ep, ldU, na]
 *   f64 (u_0..u_{Te-1}), output dVdx_d [n_ep, ldS, ns] f64: V_x(s_t) for t = 0..Te, time column 0 —
 *   the layout cacto_rl_solve_add reads. mu: the Qbar_uu regulariser (1e-9 in the reference).
 *   nsteps_d[e] < 0 skips episode e (a rollout dropped for a NaN state, RL.py:229-231 /
 *   main.py:236): nothing is read or written for it.
 * The reward's derivatives are those of the TO cost (= -reward, environment_TO.py): closed forms
 * for the planar family (SI, DI, car), hyper-dual forward-mode derivatives through the forward
 * kinematics (manipulator, UR5) and the body check points (car_park). Dynamics Jacobians as
 * augmented_derivative (environment.py:111-132, :221-233, :420-435, :567-582); for revolute chains
 * ddq_dq, ddq_dv (computeABADerivatives) come from hyper-dual RNEA. Every system is supported; a
 * (dynamics, reward) combination outside the six systems returns CACTO_EUNSUPPORTED. */
int cacto_ddp_backward(const cacto_sys* sys, const double* S_traj_d, int64_t ldS, const double* U_traj_d,
                       int64_t ldU, const int32_t* nsteps_d, int n_ep, double mu, double* dVdx_d, void* stream);

/* ---------------------------------------------------------------- replay ------------------ */

/* rows_d [n, 3ns+3] f64 written at ring position next_idx (wraps modulo capacity). */
int cacto_buffer_add(const cacto_sys* sys, double* storage_d, int64_t capacity, int64_t next_idx,
                     const double* rows_d, int64_t n, void* stream);

/* RL_Solve (RL.py:145-189) for n_ep episodes, rows written straight into the ring as
 * buffer.add(state_arr, partial_reward_to_go_arr, state_next_rollout_arr, dVdx, done_arr, term_arr)
 * does after it (main.py:240). Episode e has Te = row_off_d[e+1] - row_off_d[e] - 1 steps
 * (NSTEPS_SH), 0 <= Te <= max_T, and its Te+1 rows go to ring slots
 * (next_idx + row_off_d[e] + i) % capacity; total_rows = row_off_d[n_ep] <= capacity.
 *   S_traj_d [n_ep, ldS, ns] f64: s_0..s_Te (ldS >= max_T+1; the cacto_rollout layout with T = max_T)
 *   R_d [n_ep, ldR] f64: rwrd_arr r_0..r_Te, or r_0..r_{Te-1} when R_term_d [n_ep] (f64) gives r_Te
 *     (env_RL: RL.py:160-165); pass -TO_step_cost for env_RL = 0 (RL.py:167)
 *   dVdx_d [n_ep, ldS, ns] f64 or NULL (zeros)
 *   nsteps_td = conf.nsteps_TD_N, mc = conf.MC
 *   total_d [n_ep, ldS] f64 or NULL: total_reward_to_go_arr.
 * Partial/total reward-to-go are Python's left-to-right sums rounded to float32, bit-exact. */
int cacto_rl_solve_add(const cacto_sys* sys, const double* S_traj_d, int64_t ldS, const double* R_d,
                       int64_t ldR, const double* R_term_d, const double* dVdx_d, const int64_t* row_off_d,
                       int n_ep, int max_T, int64_t total_rows, int nsteps_td, int mc, double* storage_d,
                       int64_t capacity, int64_t next_idx, double* total_d, void* stream);

/* replay_buffer.py:47-61: S, R, S_next, dVdx, d as float32, term float64; any may be NULL. */
int cacto_buffer_gather(const cacto_sys* sys, const double* storage_d, const int32_t* idx_d, int B,
                        float* S_d, float* R_d, float* S_next_d, float* dVdx_d, float* d_d, double* term_d,
                        void* stream);

/* Prioritized replay. Trees are float64 arrays of 2*capacity (capacity a power of two), node 1 =
 * root, leaves at [capacity, 2*capacity) — the layout of segment_tree.py:33. */
int cacto_per_init(double* sum_tree_d, double* min_tree_d, int64_t capacity, void* stream);
/* Set leaves [start, start+n) (mod ring_size) to `value` and refresh ancestors (replay_buffer.py:133-135). */
int cacto_per_set_range(double* sum_tree_d, double* min_tree_d, int64_t capacity, int64_t ring_size,
                        int64_t start, int64_t n, double value, void* stream);
/* The same with the value max_priority_d[0] ** alpha read on the device (what ReplayBuffer.add sets new
 * leaves to, replay_buffer.py:133-135), so adding episodes needs no host read of max_priority. The
 * device pow may differ from the host libm pow the reference uses by an ulp; the Python layer
 * computes the power on the host and calls cacto_per_set_range. */
int cacto_per_set_range_max(double* sum_tree_d, double* min_tree_d, int64_t capacity, int64_t ring_size,
                            int64_t start, int64_t n, const double* max_priority_d, double alpha, void* stream);
/* Stratified proportional sampling (replay_buffer.py:139-188). uniforms_d [B] = random.random()
 * draws. Outputs idx_d [B] int32, is_w_d [B] float32 (IS weights), and exp_counter_d (float64
 * [ring]) incremented once per distinct index. */
int cacto_per_sample(const double* sum_tree_d, const double* min_tree_d, int64_t capacity, int64_t max_idx,
                     double beta, const double* uniforms_d, int B, int32_t* idx_d, float* is_w_d,
                     double* exp_counter_d, void* stream);
/* Data-parallel PER: stats_d [3] = (total sum, min leaf, max_idx) of this shard,
 * for an all-gather into shard_stats_d [n_shards, 3]. cacto_per_sample_global then samples B
 * stratified indices from the local tree exactly as cacto_per_sample, with IS weights taken
 * against the union of the shards: w = (N p_i / (G T_g))^-beta / (N min_h(m_h/T_h) / G)^-beta,
 * N = sum of the shards' max_idx, T_g / m_g this shard's sum / min. With one shard the weights
 * equal cacto_per_sample's bit for bit. */
int cacto_per_shard_stats(const double* sum_tree_d, const double* min_tree_d, int64_t max_idx, double* stats_d,
                          void* stream);
int cacto_per_sample_global(const double* sum_tree_d, const double* min_tree_d, int64_t capacity, int64_t max_idx,
                            double beta, const double* uniforms_d, int B, const double* shard_stats_d,
                            int n_shards, int32_t* idx_d, float* is_w_d, double* exp_counter_d, void* stream);
/* update_priorities 'PER' (replay_buffer.py:190-218): p = fresh^count*|y-V| + eps; leaves p^alpha,
 * duplicates last-write-wins; max_priority_d[0] = max(max_priority, p). */
int cacto_per_update(double* sum_tree_d, double* min_tree_d, int64_t capacity, const int32_t* idx_d,
                     const float* y_d, const float* V_d, const double* exp_counter_d, double fresh_factor,
                     double eps, double alpha, double* max_priority_d, int B, void* stream);
/* update_priorities 'ReLO' (replay_buffer.py:193-196): td = (V - y)^2 - (V_tgt - y)^2 in f32 (Keras
 * MeanSquaredError, reduction NONE), clipped as np.clip(td, 0, max(td)); p = fresh^count * td + eps
 * in f64; leaves p^alpha (duplicates last-write-wins), max_priority_d[0] = max(max_priority, p).
 * leaves_ws_d: B doubles of caller workspace. Replaces PrioritizedReplayBuffer.update_priorities
 * with RB_type == 'ReLO'. The reference asserts p > 0 for every sample (replay_buffer.py:212): when
 * some p <= 0 (every td negative) or is NaN (any td NaN), *status_d is set to 1 and the trees,
 * counters and max_priority are left unchanged; a set status makes later calls no-ops until the
 * caller clears it (the host raises the reference's AssertionError). status_d: one device int32. */
int cacto_per_update_relo(double* sum_tree_d, double* min_tree_d, int64_t capacity, const int32_t* idx_d,
                          const float* y_d, const float* V_d, const float* Vt_d, const double* exp_counter_d,
                          double fresh_factor, double eps, double alpha, double* max_priority_d, double* leaves_ws_d,
                          int32_t* status_d, int B, void* stream);
/* Set arbitrary leaves (already raised to alpha) and refresh ancestors; duplicates last-write-wins. */
int cacto_per_set_leaves(double* sum_tree_d, double* min_tree_d, int64_t capacity, const int32_t* idx_d,
                         const double* values_d, int n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CACTO_HIP_H */
