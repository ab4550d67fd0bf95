// Error plumbing and the system handle (cacto_sys_create / destroy).
#include <cstring>
#include <string>

#include "common.h"
#include "env.h"
#include "internal.h"

namespace cacto {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return CACTO_EHIP;
}

}  // namespace cacto

extern "C" const char* cacto_last_error(void) { return cacto::g_last_error.c_str(); }

extern "C" int cacto_abi_version(void) { return CACTO_ABI_VERSION; }

extern "C" int cacto_sys_create(const cacto_sys_params* params_h, const double* joint_table_h, cacto_sys** out) {
  using namespace cacto;
  try {
    CACTO_REQUIRE(params_h && out, "cacto_sys_create: null argument");
    const cacto_sys_params& p = *params_h;
    CACTO_REQUIRE(p.nb_state >= 2 && p.nb_state <= CACTO_MAX_STATE, "cacto_sys_create: nb_state out of range");
    CACTO_REQUIRE(p.nb_action >= 1 && p.nb_action <= CACTO_MAX_ACTION, "cacto_sys_create: nb_action out of range");
    CACTO_REQUIRE(p.nb_state <= 16 && p.nb_action <= 16, "cacto_sys_create: MLP tiles assume ns, na <= 16");
    CACTO_REQUIRE(p.dyn_kind == CACTO_DYN_SINGLE_INTEGRATOR || p.dyn_kind == CACTO_DYN_CHAIN ||
                      p.dyn_kind == CACTO_DYN_CAR || p.dyn_kind == CACTO_DYN_CAR_PARK,
                  "cacto_sys_create: unknown dynamics kind");
    CACTO_REQUIRE(p.reward_kind == CACTO_REW_PLANAR || p.reward_kind == CACTO_REW_MANIPULATOR ||
                      p.reward_kind == CACTO_REW_UR5 || p.reward_kind == CACTO_REW_CAR_PARK,
                  "cacto_sys_create: unknown reward kind");
    if (p.dyn_kind == CACTO_DYN_CAR || p.dyn_kind == CACTO_DYN_CAR_PARK)
      CACTO_REQUIRE(p.nb_state == 6 && p.nb_action == 2, "car / car_park need ns = 6, na = 2");
    if (p.dyn_kind == CACTO_DYN_CAR_PARK)
      CACTO_REQUIRE(p.L_delta > 0.0 && p.tau_delta > 0.0, "car_park needs L_delta > 0 and tau_delta > 0");
    if (p.reward_kind == CACTO_REW_CAR_PARK)
      CACTO_REQUIRE(p.dyn_kind == CACTO_DYN_CAR_PARK && p.n_check >= 1 && p.n_check <= 10,
                    "car_park reward needs car_park dynamics and 1..10 check points");
    if (p.reward_kind == CACTO_REW_UR5)
      CACTO_REQUIRE(p.dyn_kind == CACTO_DYN_CHAIN, "ur5 reward needs chain dynamics");
    if (p.dyn_kind == CACTO_DYN_SINGLE_INTEGRATOR) {
      CACTO_REQUIRE(p.nb_state == 3 && p.nb_action == 2, "single integrator needs ns = 3, na = 2");
    }
    if (p.dyn_kind == CACTO_DYN_CHAIN) {
      CACTO_REQUIRE(joint_table_h != nullptr, "cacto_sys_create: chain dynamics needs a joint table");
      CACTO_REQUIRE(p.n_joints == 2 || p.n_joints == 3 || p.n_joints == 6,
                    "cacto_sys_create: chains of 2, 3 or 6 joints are instantiated in this build");
      CACTO_REQUIRE(p.nq == p.n_joints && p.nv == p.n_joints && p.nb_state == 2 * p.n_joints + 1 &&
                        p.nb_action == p.n_joints,
                    "cacto_sys_create: chain needs nq = nv = na = n_joints, ns = 2n + 1");
      CACTO_REQUIRE(p.ee_parent >= 0 && p.ee_parent < p.n_joints, "cacto_sys_create: bad ee_parent");
      for (int i = 0; i < p.n_joints; ++i) {
        const int parent = (int)joint_table_h[i * CACTO_JOINT_COLS];
        const int kind = (int)joint_table_h[i * CACTO_JOINT_COLS + 1];
        CACTO_REQUIRE(parent == i - 1, "cacto_sys_create: only serial chains (parent = i - 1) are supported");
        CACTO_REQUIRE(kind == 0 || kind == 1, "cacto_sys_create: joint type must be revolute(0)/prismatic(1)");
      }
    }
    CACTO_REQUIRE(p.n_weights >= 7 && p.n_weights <= 8, "cacto_sys_create: n_weights must be 7 or 8");
    SysDevice host{};
    host.p = p;
    host.p.const_dyn = 0;
    if (p.dyn_kind == CACTO_DYN_CHAIN) {
      bool all_prismatic = true;
      for (int i = 0; i < p.n_joints; ++i) all_prismatic = all_prismatic && (int)joint_table_h[i * CACTO_JOINT_COLS + 1] == 1;
      host.p.const_dyn = all_prismatic ? 1 : 0;
    }
    if (joint_table_h && p.dyn_kind == CACTO_DYN_CHAIN)
      std::memcpy(host.joints, joint_table_h, sizeof(double) * p.n_joints * CACTO_JOINT_COLS);
    if (p.dyn_kind == CACTO_DYN_CHAIN && p.n_joints == 3 && p.gravity[0] == 0.0 && p.gravity[1] == 0.0) {
      // planar 3R chain (the manipulator): closed-form M / h constants for the rollout (env.h planar3_step)
      bool planar = true;
      for (int i = 0; i < 3; ++i) {
        const double* r = joint_table_h + i * CACTO_JOINT_COLS;
        planar = planar && (int)r[1] == 0 && r[2] == 0.0 && r[3] == 0.0 && r[4] == 1.0;
        for (int k = 0; k < 9; ++k) planar = planar && r[5 + k] == ((k % 4 == 0) ? 1.0 : 0.0);
      }
      if (planar) {
        const double* J = joint_table_h;
        auto col = [&](int i, int c) { return J[i * CACTO_JOINT_COLS + c]; };
        double* pl = host.pl;
        pl[0] = 1.0;
        pl[1] = col(1, 14), pl[2] = col(1, 15);
        pl[3] = col(2, 14), pl[4] = col(2, 15);
        for (int k = 0; k < 3; ++k) {
          pl[5 + 2 * k] = col(k, 18);
          pl[6 + 2 * k] = col(k, 19);
          pl[11 + k] = col(k, 17);
        }
        pl[14] = col(0, 26) + col(1, 26) + col(2, 26);
        pl[15] = col(1, 26) + col(2, 26);
        pl[16] = col(2, 26);
        pl[17] = col(0, 17) * (col(0, 18) * col(0, 18) + col(0, 19) * col(0, 19));
      }
    }
    for (int r = 0; r < CACTO_MAX_STATE; ++r)  // IEEE double division: the same bits as on the device
      host.inv_norm[r] = r < p.nb_state && p.state_norm[r] != 0.0 ? 1.0 / p.state_norm[r] : 0.0;
    cacto_sys* s = new cacto_sys();
    s->host = host;
    hipError_t e = hipMalloc(&s->dev, sizeof(SysDevice));
    if (e != hipSuccess) {
      delete s;
      return hip_fail(e, "hipMalloc(sys)");
    }
    e = hipMemcpy(s->dev, &host, sizeof(SysDevice), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(s->dev);
      delete s;
      return hip_fail(e, "hipMemcpy(sys)");
    }
    s->actor = make_topo(CACTO_NET_ACTOR, p.nb_state, p.nb_action);
    s->critic = make_topo(CACTO_NET_CRITIC, p.nb_state, p.nb_action);
    if (int rc = cacto_build_wgrad_adam_items(s)) {
      (void)hipFree(s->dev);
      delete s;
      return rc;
    }
    if (int rc = cacto_const_dyn_init(s)) {
      (void)hipFree(s->dev);
      delete s;
      return rc;
    }
    *out = s;
    return CACTO_OK;
  } catch (const std::exception& ex) {
    set_error(std::string("cacto_sys_create: ") + ex.what());
    return CACTO_ENOMEM;
  }
}

extern "C" int cacto_sys_set_critic_type(cacto_sys* sys, int critic_type) {
  CACTO_REQUIRE(sys && (critic_type == 0 || critic_type == 1),
                "cacto_sys_set_critic_type: 0 (sine) or 1 (sine-elu); the elu / relu critics are not built");
#ifndef CACTO_CRITIC_ELU
  // the elu layers are compiled into the kernels only in the CACTO_CRITIC_ELU build
  // (cacto_amd/libcacto_hip_sine_elu.so): a runtime branch in the chain kernels' epilogues cost the
  // sine critic 4-7 % of its B = 4096 update rate
  CACTO_REQUIRE(critic_type == 0, "cacto_sys_set_critic_type: critic_type 'sine-elu' needs the CACTO_CRITIC_ELU build "
                                  "(CACTO_HIP_LIB=cacto_amd/libcacto_hip_sine_elu.so)");
#endif
  sys->critic.act = critic_type == 1 ? 0xA : 0;  // hidden layers 1 and 3 elu
  return CACTO_OK;
}

extern "C" int cacto_sys_destroy(cacto_sys* sys) {
  if (!sys) return CACTO_OK;
  (void)hipFree(sys->dev);
  if (sys->ddp_ws) (void)hipFree(sys->ddp_ws);
  for (int32_t* t : sys->wa_items)
    if (t) (void)hipFree(t);
  if (sys->side) (void)hipStreamSynchronize(sys->side);
  cacto_dp_release(sys);
  if (sys->ev_critic) (void)hipEventDestroy(sys->ev_critic);
  for (hipEvent_t e : sys->ev_actor)
    if (e) (void)hipEventDestroy(e);
  if (sys->side) (void)hipStreamDestroy(sys->side);
  if (sys->latch_host) (void)hipHostFree(sys->latch_host);
  if (sys->pipe_sig) (void)hipFree(sys->pipe_sig);
  delete sys;
  return CACTO_OK;
}
