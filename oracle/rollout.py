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

from .nn import actor_forward, actor_forward32


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


def batched_policy_rollout_di(env, actor, S0, nsteps, weights=None):
    """The same env-steps as `policy_rollout`, vectorised over episodes with numpy (the CPU
    baseline SURVEY §8d asks for beside the per-sample port, so the GPU/CPU ratio is not inflated
    by Python-loop overhead). Double integrator only: its Pinocchio chain has constant M and zero
    nle (prismatic x, y joints; gravity normal to the plane), so Env.simulate (environment.py:80-91)
    is v' = v + dt M^-1 u, q' = q + dt v for every episode at once. The actor runs in float64
    matmuls (BLAS threads); rewards per environment.py:329-351. Returns (env-steps, final states)."""
    conf = env.conf
    w = np.asarray(conf.cost_weights_running if weights is None else weights, dtype=np.float64)
    norm = np.asarray(conf.state_norm_arr, dtype=np.float64)
    nq = env.chain.n
    Minv = np.linalg.inv(env.chain.mass_matrix(np.zeros(nq)))
    assert np.abs(env.chain.nle(np.zeros(nq), np.ones(nq))).max() == 0.0, "constant-dynamics chains only"
    S = np.array(S0, dtype=np.float64)
    nsteps = np.asarray(nsteps)
    dt = conf.dt
    o, tgt = env.obs, env.target
    steps = 0
    for t in range(int(nsteps.max())):
        act = nsteps > t
        s = S[act]
        a = actor_forward(actor, s.astype(np.float32).astype(np.float64), norm).astype(np.float32).astype(np.float64)
        q, v = s[:, :nq], s[:, nq:2 * nq]
        x, y = q[:, 0], q[:, 1]
        # reward at (s, a): - w0 dist + w1 peak - w3..5 ell - w6 u_cost + offset, times scale
        ell = sum(w[3 + k] * np.log(np.exp(env.alpha * -(((x - o[2 * k]) ** 2) / ((o[6 + 2 * k] / 2) ** 2)
                                                         + ((y - o[2 * k + 1]) ** 2) / ((o[7 + 2 * k] / 2) ** 2)
                                                         - 1.0)) + 1) / env.alpha for k in range(3))
        pk = (np.sqrt((x - tgt[0]) ** 2 + 0.1) - np.sqrt(0.1) - 0.1 + np.sqrt((y - tgt[1]) ** 2 + 0.1)
              - np.sqrt(0.1) - 0.1)
        peak = np.log(np.exp(env.alpha2 * -pk) + 1) / env.alpha2
        u_cost = np.sum(a * a + conf.w_b * (a / conf.u_max) ** 10, axis=1)
        r = env.scale * (-w[0] * ((x - tgt[0]) ** 2 + (y - tgt[1]) ** 2) + w[1] * peak - ell - w[6] * u_cost
                         + env.offset)
        sn = np.empty_like(s)
        sn[:, :nq] = q + dt * v
        sn[:, nq:2 * nq] = v + dt * (a @ Minv.T)
        sn[:, -1] = s[:, -1] + dt
        S[act] = sn
        del r                       # the rewards are produced each step, as in PLOT.rollout
        steps += int(act.sum())
    return steps, S


def nsteps_sh(conf, s0):
    return conf.NSTEPS - int(s0[-1] / conf.dt)


def to_init_rollout(env, actor, s0, ep, f32=False, fail_step=None):
    """RL_AC.create_TO_init (RL.py:197-233). f32: the actor in TF's float32 arithmetic
    (`actor_forward32`: overflow to inf / NaN as the reference's). fail_step (a list) receives the
    step i whose s_{i+1} was NaN when the episode is dropped (RL.py:229-231)."""
    conf = env.conf
    T = nsteps_sh(conf, s0)
    if T == 0:
        return None
    norm = np.asarray(conf.state_norm_arr, dtype=np.float64)
    S = np.zeros((T + 1, conf.nb_state))
    U = np.zeros((T, conf.nb_action))
    S[0] = s0
    for i in range(T):
        if ep == 0:
            U[i] = 0.0
        elif f32:
            U[i] = actor_forward32(actor, np.asarray(S[i])[None, :], norm)[0]
        else:
            U[i] = actor_eval32(actor, S[i], norm)
        with np.errstate(over="ignore", invalid="ignore"):
            S[i + 1] = env.simulate(S[i], U[i])
        if np.isnan(S[i + 1]).any():
            if fail_step is not None:
                fail_step.append(i)
            return None
    return S, U, T
