"""Settings every reference conf_*.py shares, and the derived quantities they compute.

The reference's system configs are flat modules of constants (the plugin surface selected by
`--system-id`, main.py:100-115). Each module here states its system-specific values and then calls
`finalize(globals())`, which fills in the shared defaults (e.g. REPLAY_SIZE = 2**16, MC = 0,
UPDATE_RATE = 1e-3, NH1 = NH2 = 256, NORMALIZE_INPUTS = 1, env_RL = 0, PER α = 0 / β = 0.6 —
conf_double_integrator.py:18-90) and the derived ones (NEPISODES, NLOOPS, LR-schedule lists,
cost_weights_*, obs_param, soft_max_param, cost_funct_param, w_b).
"""
import numpy as np

SHARED = dict(
    REPLAY_SIZE=2 ** 16, MC=0, UPDATE_RATE=0.001, CRITIC_LEARNING_RATE=5e-4,
    ACTOR_LEARNING_RATE=1e-3, critic_type="sine", NH1=256, NH2=256, NORMALIZE_INPUTS=1,
    kreg_l1_A=1e-2, kreg_l2_A=1e-2, breg_l1_A=1e-2, breg_l2_A=1e-2,
    kreg_l1_C=1e-2, kreg_l2_C=1e-2, breg_l1_C=1e-2, breg_l2_C=1e-2,
    prioritized_replay_alpha=0, prioritized_replay_beta=0.6, prioritized_replay_beta_iters=None,
    env_RL=0, EP_UPDATE=200, LR_SCHEDULE=0, save_flag=1, profile=0, offset_cost_fun=0,
    scale_cost_fun=1e-5, simulate_coulomb_friction=0, simulation_type="euler",
    integration_scheme="E-Euler", end_effector_frame_id="EE",
)


def finalize(g):
    for k, v in SHARED.items():
        g.setdefault(k, v)
    g["NEPISODES"] = int(g["EP_UPDATE"] * len(g["UPDATE_LOOPS"]))
    g["NLOOPS"] = len(g["UPDATE_LOOPS"])
    if not g["MC"]:
        g.setdefault("nsteps_TD_N", int(g["NSTEPS"] / g["TD_DIV"]))
    rs, bs = g["REPLAY_SIZE"], g["BATCH_SIZE"]
    bounds = [k * rs / bs for k in (200, 300, 400, 500)]
    g["boundaries_schedule_LR_C"] = list(bounds)
    g["boundaries_schedule_LR_A"] = list(bounds)
    g["values_schedule_LR_C"] = [g["CRITIC_LEARNING_RATE"] / d for d in (1, 2, 4, 8, 16)]
    g["values_schedule_LR_A"] = [g["ACTOR_LEARNING_RATE"] / d for d in (1, 2, 4, 8, 16)]
    g["cost_funct_param"] = np.array([g["offset_cost_fun"], g["scale_cost_fun"]])
    g["soft_max_param"] = np.array([g["alpha"], g["alpha2"]])
    g["weight"] = np.array([g["w_d"], g["w_u"], g["w_peak"], g["w_ob"], g["w_v"]])
    g["w_b"] = 1 / g["w_u"]
    g["u_min"] = np.asarray(g["u_min"], dtype=np.float64)
    g["u_max"] = np.asarray(g["u_max"], dtype=np.float64)
    g["nb_action"] = len(g["u_max"])
    g["TARGET_STATE"] = np.asarray(g["TARGET_STATE"], dtype=np.float64)
    g["save_interval"] = g.get("save_interval", 5000) if g["save_flag"] else np.inf
