"""Oracle: policy rollouts (test infrastructure only — see oracle/__init__).

  * `policy_rollout` restates PLOT.rollout's per-step loop (plot_utils.py:245-279): actor eval at
    batch 1 (float32 in/out, NN.eval NeuralNetwork.py:130-138) -> env.step(running weights, s, a)
    (environment.py:70-78: simulate + reward) -> EE of the new state. This is the env-step of the
    benchmark metric.
  * `to_init_rollout` restates RL_AC.create_TO_init (RL.py:197-233): NSTEPS_SH = NSTEPS -
    int(t/dt), zero controls at ep == 0, NaN check.
States are float64 throughout, as in the reference's numpy arrays.
"""
import numpy as np

from .nn import actor_forward


def actor_eval32(actor, s, norm):
    """NN.eval on one float64 state: float32 input, float32 output (TF Dense in float32)."""
    x = np.asarray(s, dtype=np.float32)[None, :]
    return actor_forward(actor, x.astype(np.float64), norm)[0].astype(np.float32)


def policy_rollout(env, actor, s0, nsteps, weights=None):
    conf = env.conf
    w = conf.cost_weights_running if weights is None else weights
    norm = np.asarray(conf.state_norm_arr, dtype=np.float64)
    S = np.zeros((nsteps + 1, conf.nb_state))
    A = np.zeros((nsteps, conf.nb_action))
    R = np.zeros(nsteps)
    EE = np.zeros((nsteps + 1, 3))
    S[0] = s0
    EE[0] = env.get_end_effector_position(S[0])
    for i in range(nsteps):
        A[i] = actor_eval32(actor, S[i], norm)
        S[i + 1], R[i] = env.step(w, S[i], A[i])
        EE[i + 1] = env.get_end_effector_position(S[i + 1])
    return S, A, R, EE


def nsteps_sh(conf, s0):
    return conf.NSTEPS - int(s0[-1] / conf.dt)


def to_init_rollout(env, actor, s0, ep):
    conf = env.conf
    T = nsteps_sh(conf, s0)
    if T == 0:
        return None
    norm = np.asarray(conf.state_norm_arr, dtype=np.float64)
    S = np.zeros((T + 1, conf.nb_state))
    U = np.zeros((T, conf.nb_action))
    S[0] = s0
    for i in range(T):
        U[i] = 0.0 if ep == 0 else actor_eval32(actor, S[i], norm)
        S[i + 1] = env.simulate(S[i], U[i])
        if np.isnan(S[i + 1]).any():
            return None
    return S, U, T
