"""GPU parity: the HIP path (through the C-ABI) against the float64 oracle on the same inputs.

Tolerances (float32 kernels vs float64 oracle):
  * dynamics / Fu / EE in float64 kernels: bit-exact where the arithmetic is exact (SI, DI),
    rel 1e-12 for the manipulator chain (CRBA/RNEA vs 6x6 restatement);
  * float32 outputs of float64 math (S_next, Fu): exact f32 rounding for SI/DI, 2 ulp manipulator;
  * MLP forward: |err| <= 64 * 2^-24 * (forward pass on |W|, |b|, |h|) — the float32 rounding
    scale of the K <= 256 MFMA dot-product chains;
  * gradients: relative L2 error per tensor <= 2e-4 (float32 chains with sin/cos and clog).
"""
import math
import random

import numpy as np
import pytest
import torch

from conftest import load_weights
from oracle import buffer as obuf
from oracle import env as oenv
from oracle import nn as onn
from oracle import rollout as oroll
from cacto_amd.confs import load_conf

pytestmark = pytest.mark.gpu

SYSTEMS = ["single_integrator", "double_integrator", "manipulator", "car", "car_park", "ur5"]
CHAINS = ("manipulator", "ur5")        # float64 CRBA/RNEA vs the 6x6 oracle: few-ulp agreement
TRIG = ("car", "car_park")            # device cos/sin/tan vs libm: <= 1 ulp each


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _env(system):
    from cacto_amd.environment import make_env
    conf = load_conf(system)
    return conf, make_env(conf), oenv.make_env(conf)


def _states(conf, n, rng):
    lo = np.array(conf.x_init_min, dtype=float)
    hi = np.array(conf.x_init_max, dtype=float)
    S = rng.uniform(lo, hi, size=(n, conf.nb_state))
    S[:, :-1] *= 1.3
    flat = np.where(hi[:-1] - lo[:-1] < 1e-12)[0]   # e.g. car_park v, delta start at 0
    S[:, flat] = rng.uniform(-0.5, 0.5, size=(n, len(flat)))
    return S


def _actions(conf, n, rng):
    return rng.uniform(-1.2, 1.2, size=(n, conf.nb_action)) * conf.u_max


def abs_bound(kind, params, S, norm):
    """Forward pass with |W|, |b| and |activations|: the scale of the float32 rounding error of a
    K-term dot-product chain (|err| <= c * 2^-24 * abs_bound)."""
    P = [np.abs(np.asarray(p, dtype=np.float64)) for p in params]
    h = np.abs(onn.normalize(S, norm))
    nl = len(P) // 2
    for l in range(nl):
        h = h @ P[2 * l] + P[2 * l + 1]
        if kind == "critic" and l < nl - 1:
            h = np.ones_like(h)  # |sin| <= 1
    return h


F32_TOL = 64 * 2.0 ** -24


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


# ------------------------------------------------------------------ environment
@pytest.mark.parametrize("system", SYSTEMS)
def test_env_step_batch_f32(system):
    conf, genv, oe = _env(system)
    rng = np.random.default_rng(10)
    B = 333
    S = _states(conf, B, rng).astype(np.float32)
    A = _actions(conf, B, rng).astype(np.float32)
    term = (rng.uniform(size=B) < 0.3).astype(np.float64)
    out = genv.batch_f32(S, A, term=term)
    torch.cuda.synchronize()
    Sn = out["S_next"].cpu().numpy()
    Fu = out["Fu"].cpu().numpy()
    ref_Sn = oe.simulate_batch(S, A)
    ref_Fu = oe.derivative_batch(S, A)
    if system in CHAINS or system in TRIG:
        np.testing.assert_allclose(Sn, ref_Sn, rtol=3e-7, atol=1e-6)
        np.testing.assert_allclose(Fu, ref_Fu, rtol=3e-7, atol=1e-12)
    else:
        np.testing.assert_array_equal(Sn, ref_Sn)
        np.testing.assert_array_equal(Fu, ref_Fu)
    W = term[:, None] * conf.cost_weights_terminal + (1 - term[:, None]) * conf.cost_weights_running
    ref_R = oe.reward_batch(W, S, A)[:, 0]
    if system == "car_park":   # float32 check-point rotation (np.cos f32) under steep box costs
        np.testing.assert_allclose(out["R"].cpu().numpy(), ref_R, rtol=1e-4, atol=1e-6)
    else:
        np.testing.assert_allclose(out["R"].cpu().numpy(), ref_R, rtol=2e-6, atol=1e-9)
    np.testing.assert_allclose(out["dR_dA"].cpu().numpy(), oe.dr_da(W, A), rtol=2e-5, atol=1e-9)


@pytest.mark.parametrize("system", SYSTEMS)
def test_env_step_f64(system):
    conf, genv, oe = _env(system)
    rng = np.random.default_rng(11)
    B = 257
    S = _states(conf, B, rng)
    A = _actions(conf, B, rng)
    Sn, R, EE = genv.step_batch(S, A)
    torch.cuda.synchronize()
    ref = [oe.step(conf.cost_weights_running, s, a) for s, a in zip(S, A)]
    ref_S = np.array([r[0] for r in ref])
    ref_R = np.array([r[1] for r in ref])
    ref_EE = np.array([oe.get_end_effector_position(s) for s in ref_S])
    if system in CHAINS or system in TRIG:
        np.testing.assert_allclose(Sn.cpu().numpy(), ref_S, rtol=1e-12, atol=1e-12)
    else:
        np.testing.assert_array_equal(Sn.cpu().numpy(), ref_S)
    np.testing.assert_allclose(R.cpu().numpy(), ref_R, rtol=1e-11, atol=1e-14)
    np.testing.assert_allclose(EE.cpu().numpy(), ref_EE, rtol=1e-12, atol=1e-12)


# ------------------------------------------------------------------ networks
def _nets(system, tag=None, seed=0):
    from cacto_amd.neural_network import NN
    from cacto_amd.rl import RL_AC
    conf, genv, oe = _env(system)
    nn = NN(genv, conf, w_S=1e-2, seed=seed)
    rl = RL_AC(genv, nn, conf)
    weights = load_weights(tag) if tag else None
    rl.setup_model(weights=weights)
    return conf, genv, oe, nn, rl


@pytest.mark.parametrize("system,tag", [("double_integrator", "di_seed0_final"), ("single_integrator", "si_seed0_0"),
                                        ("manipulator", None)])
def test_forward_and_input_grad(system, tag):
    conf, genv, oe, nn, rl = _nets(system, tag)
    rng = np.random.default_rng(12)
    B = 200
    S = _states(conf, B, rng).astype(np.float32)
    norm = conf.state_norm_arr.astype(np.float64)
    A = nn.eval(rl.actor_model, S).cpu().numpy()
    aw = rl.actor_model.get_weights()
    ref_A = onn.actor_forward(aw, S.astype(np.float64), norm)
    bound = F32_TOL * abs_bound("actor", aw, S.astype(np.float64), norm)
    assert np.all(np.abs(A - ref_A) <= bound), (np.abs(A - ref_A) / bound).max()
    V, g = nn.critic_input_grad(rl.critic_model, S)
    cw = rl.critic_model.get_weights()
    ref_V = onn.critic_forward(cw, S.astype(np.float64), norm)
    ref_g, _ = onn.critic_input_grad(cw, S.astype(np.float64), norm)
    vb = F32_TOL * abs_bound("critic", cw, S.astype(np.float64), norm)
    assert np.all(np.abs(V.cpu().numpy() - ref_V) <= vb), (np.abs(V.cpu().numpy() - ref_V) / vb).max()
    assert rel_l2(g.cpu().numpy(), ref_g) < 2e-5


def _replay_rows(conf, B, rng):
    ns = conf.nb_state
    S = _states(conf, B, rng)
    Sn = _states(conf, B, rng)
    R = rng.normal(size=(B, 1)) * 0.5
    dVdx = rng.normal(size=(B, ns)) * 0.3
    d = (rng.uniform(size=(B, 1)) < 0.3).astype(float)
    term = (rng.uniform(size=(B, 1)) < 0.2).astype(float)
    return np.concatenate([S, R, Sn, dVdx, d, term], axis=1)


@pytest.mark.parametrize("system,tag,w_S,B", [("double_integrator", "di_seed0_0", 1e-2, 128),
                                              ("double_integrator", "di_seed0_final", 1e-2, 100),
                                              ("double_integrator", "di_seed0_0", 0.0, 64),
                                              ("manipulator", None, 1e-2, 64),
                                              ("single_integrator", "si_seed0_0", 0.0, 128),
                                              ("car_park", None, 0.0, 64), ("ur5", None, 1e-2, 64)])
def test_critic_grad(system, tag, w_S, B):
    conf, genv, oe, nn, rl = _nets(system, tag)
    rl.w_S = w_S
    rl.cfg = rl.make_cfg()
    rng = np.random.default_rng(13)
    rows = _replay_rows(conf, B, rng)
    rows_f32 = rows.astype(np.float32).astype(np.float64)  # the reference converts the sample to f32
    ns = conf.nb_state
    g, y, V, Vt = rl.critic_grad_rows(torch.as_tensor(rows, device="cuda"),
                                      torch.arange(B, dtype=torch.int32, device="cuda"))
    norm = conf.state_norm_arr.astype(np.float64)
    ref = onn.compute_critic_grad(rl.critic_model.get_weights(), rl.target_critic.get_weights(),
                                  rows_f32[:, :ns], rows_f32[:, ns + 1:2 * ns + 1], rows_f32[:, ns:ns + 1],
                                  rows_f32[:, 2 * ns + 1:3 * ns + 1], rows_f32[:, 3 * ns + 1:3 * ns + 2],
                                  np.ones((B, 1)), w_S, norm)
    for i, (a, b) in enumerate(zip(g, ref[0])):
        assert rel_l2(a.cpu().numpy(), b) < 2e-4, (i, rel_l2(a.cpu().numpy(), b))
    vb = F32_TOL * abs_bound("critic", rl.critic_model.get_weights(), rows_f32[:, :ns], norm)
    vbn = F32_TOL * abs_bound("critic", rl.target_critic.get_weights(), rows_f32[:, ns + 1:2 * ns + 1], norm)
    assert np.all(np.abs(y.cpu().numpy() - ref[1]) <= vbn + 1e-7 * np.abs(ref[1]))
    assert np.all(np.abs(V.cpu().numpy() - ref[2]) <= vb)
    assert np.all(np.abs(Vt.cpu().numpy() - ref[3]) <= vb)


@pytest.mark.parametrize("system,tag,B", [("double_integrator", "di_seed0_final", 128),
                                          ("manipulator", None, 64), ("single_integrator", "si_seed0_0", 77),
                                          ("car", None, 64), ("car_park", None, 64), ("ur5", None, 64)])
def test_actor_grad(system, tag, B):
    conf, genv, oe, nn, rl = _nets(system, tag)
    rng = np.random.default_rng(14)
    rows = _replay_rows(conf, B, rng)
    ns = conf.nb_state
    g = rl.actor_grad_rows(torch.as_tensor(rows, device="cuda"), torch.arange(B, dtype=torch.int32, device="cuda"))
    S32 = rows[:, :ns].astype(np.float32)
    ref = onn.compute_actor_grad(oe, rl.actor_model.get_weights(), rl.critic_model.get_weights(), S32,
                                 rows[:, 3 * ns + 2:3 * ns + 3], conf.state_norm_arr.astype(np.float64))
    for i, (a, b) in enumerate(zip(g, ref)):
        assert rel_l2(a.cpu().numpy(), b) < 2e-4, (i, rel_l2(a.cpu().numpy(), b))


def test_update_matches_oracle_sequence():
    """Several fused cacto_update steps == the oracle's critic step -> actor step (new critic) ->
    target update sequence with Keras-Adam (RL.py:101-118)."""
    conf, genv, oe, nn, rl = _nets("double_integrator", "di_seed0_0")
    norm = conf.state_norm_arr.astype(np.float64)
    rng = np.random.default_rng(15)
    N, B, steps = 512, 128, 5
    rows = _replay_rows(conf, N, rng)
    storage = torch.as_tensor(rows, device="cuda")
    ns = conf.nb_state
    crit, tgt, act = rl.critic_model.get_weights(), rl.target_critic.get_weights(), rl.actor_model.get_weights()
    oc, oa = onn.KerasAdam(conf.CRITIC_LEARNING_RATE), onn.KerasAdam(conf.ACTOR_LEARNING_RATE)
    for k in range(steps):
        idx = rng.integers(0, N, size=B)
        rl.update_rows(storage, torch.as_tensor(idx.astype(np.int32), device="cuda"))
        r = rows[idx].astype(np.float32).astype(np.float64)
        gc = onn.compute_critic_grad(crit, tgt, r[:, :ns], r[:, ns + 1:2 * ns + 1], r[:, ns:ns + 1],
                                     r[:, 2 * ns + 1:3 * ns + 1], r[:, 3 * ns + 1:3 * ns + 2], np.ones((B, 1)),
                                     1e-2, norm)[0]
        crit = oc.apply(crit, gc)
        ga = onn.compute_actor_grad(oe, act, crit, r[:, :ns].astype(np.float32), rows[idx, 3 * ns + 2:], norm)
        act = oa.apply(act, ga)
        tgt = onn.soft_update(tgt, crit, conf.UPDATE_RATE)
    torch.cuda.synchronize()
    assert rl.steps.cpu().tolist() == [steps, steps]
    for name, got, ref in (("critic", rl.critic_model.get_weights(), crit), ("actor", rl.actor_model.get_weights(), act),
                           ("target", rl.target_critic.get_weights(), tgt)):
        for i, (a, b) in enumerate(zip(got, ref)):
            # Adam normalises the step, so compare the accumulated parameter change
            assert np.abs(a - b).max() < 5e-6 * steps, (name, i, np.abs(a - b).max())
    # packed copies were refreshed: forward with the updated weights matches the oracle
    S = _states(conf, 64, rng).astype(np.float32)
    A = nn.eval(rl.actor_model, S).cpu().numpy()
    aw = rl.actor_model.get_weights()
    refA = onn.actor_forward(aw, S.astype(np.float64), norm)
    assert np.all(np.abs(A - refA) <= F32_TOL * abs_bound("actor", aw, S.astype(np.float64), norm))


# ------------------------------------------------------------------ rollout
def test_rollout_di_known_answer():
    conf, genv, oe, nn, rl = _nets("double_integrator", "di_seed0_final")
    S0 = np.array(conf.init_states_sim)
    T = conf.NSTEPS
    out = rl.rollout_batch(S0, [T] * len(S0), T)
    torch.cuda.synchronize()
    EE = out["EE"].cpu().numpy()
    S = out["S"].cpu().numpy()
    maxy = {(s[0], s[1]): EE[k, :, 1].max() for k, s in enumerate(S0)}
    assert abs(maxy[(2.0, 0.0)] - 3.74) < 0.01
    assert abs(maxy[(10.0, 0.0)] - 7.88) < 0.01
    assert abs(maxy[(10.0, 10.0)] - 10.0) < 0.01
    assert abs(maxy[(12.0, 2.0)] - 8.70) < 0.01
    assert abs(maxy[(15.0, 0.0)] - 9.44) < 0.01
    actor = rl.actor_model.get_weights()
    for k, s0 in enumerate(S0):
        rS, rA, rR, rEE = oroll.policy_rollout(oe, actor, s0, T)
        np.testing.assert_allclose(S[k], rS, rtol=1e-4, atol=2e-4)
        np.testing.assert_allclose(out["R"].cpu().numpy()[k], rR, rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("system", ["double_integrator", "manipulator", "car_park", "ur5"])
@pytest.mark.parametrize("ep,sched", [(1, (0, 0)), (1, (1, 3)), (0, (2, 2)), (1, (-3, 3)), (0, (-3, 2)), (1, (4, 2))])
def test_rollout_rewards_separate_launch(system, ep, sched):
    """cacto_rollout_rewards over a recorded S/A-only rollout gives exactly the R / EE of the
    combined cacto_rollout call (bench.py launches the two kernels apart) — under the automatic
    schedule and a slot-refilling one (1 group, 3 workgroups), with the actor and with zero
    controls (ep == 0), and with an episode of length 0 (EE_0 only)."""
    if sched[0] == -3 and system == "ur5":
        pytest.skip("one slot per wave: systems without configuration-dependent M and the planar 3R chain")
    if sched[0] == 4 and system != "manipulator":
        pytest.skip("4 groups per workgroup: the manipulator's generic-kernel schedule")
    conf, genv, oe, nn, rl = _nets(system, None, seed=2)
    rng = random.Random(5)
    S0 = np.array([oe.reset(rng) for _ in range(37)])
    ns_ = [conf.NSTEPS - int(s[-1] / conf.dt) for s in S0]
    ns_[3] = 0                                   # an episode of length 0: EE_0 only, from the refill
    T = max(ns_)
    ref = rl.rollout_batch(S0, ns_, T, ep=ep, sched=sched)
    got = rl.rollout_batch(S0, ns_, T, ep=ep, want=("S", "A"), sched=sched)
    got["R"] = torch.full_like(ref["R"], float("nan"))
    got["EE"] = torch.full_like(ref["EE"], float("nan"))
    rl.rollout_rewards(got, torch.as_tensor(np.asarray(ns_, dtype=np.int32), device="cuda"), T, ep=ep)
    torch.cuda.synchronize()
    for k, n in enumerate(ns_):
        np.testing.assert_array_equal(got["R"][k, :n].cpu().numpy(), ref["R"][k, :n].cpu().numpy())
        np.testing.assert_array_equal(got["EE"][k, :n + 1].cpu().numpy(), ref["EE"][k, :n + 1].cpu().numpy())
        assert not np.isnan(ref["EE"][k, :n + 1].cpu().numpy()).any()
    if ep == 0:
        return
    w = conf.cost_weights_running
    S, A, R = got["S"].cpu().numpy(), got["A"].cpu().numpy(), got["R"].cpu().numpy()
    for k in range(0, len(S0), 6):
        t = ns_[k] // 2
        np.testing.assert_allclose(R[k, t], oe.reward(w, S[k, t], A[k, t].astype(np.float64)), rtol=1e-10,
                                   atol=1e-14)


@pytest.mark.parametrize("system,tag", [("double_integrator", "di_seed0_final"), ("manipulator", None),
                                        ("car_park", None)])
def test_policy_eval_returns(system, tag):
    """PLOT.rollout (plot_utils.py:245-279): full-NSTEPS rollouts from init_states_sim, returns
    keyed by (x0, y0) = Python sum of the step rewards, p_ee[:, 2] replaced by s[:, 2]."""
    from cacto_amd.plot_utils import PLOT
    conf, genv, oe, nn, rl = _nets(system, tag)
    plot = PLOT(0, genv, nn, conf, learner=rl)
    returns = plot.rollout(0, rl.actor_model, conf.init_states_sim)
    actor = rl.actor_model.get_weights()
    assert len(returns) == len({(s[0], s[1]) for s in conf.init_states_sim})
    for k, s0 in enumerate(conf.init_states_sim):
        rS, rA, rR, rEE = oroll.policy_rollout(oe, actor, s0, conf.NSTEPS)
        ret = 0
        for r in rR:
            ret += r
        assert abs(returns[s0[0], s0[1]] - ret) <= 1e-3 * abs(ret) + 1e-6, (k, returns[s0[0], s0[1]], ret)
        np.testing.assert_array_equal(plot.p_ee_all_sim[k][1:, 2], plot.states_all_sim[k][1:, 2])
        np.testing.assert_allclose(plot.p_ee_all_sim[k][:, :2], rEE[:, :2], rtol=1e-4, atol=2e-4)


@pytest.mark.parametrize("system", ["double_integrator", "manipulator"])
def test_rollout_variable_lengths(system):
    conf, genv, oe, nn, rl = _nets(system, None, seed=3)
    rng = random.Random(5)
    S0 = np.array([oe.reset(rng) for _ in range(37)])
    ns_ = [conf.NSTEPS - int(s[-1] / conf.dt) for s in S0]
    T = max(ns_)
    out = rl.rollout_batch(S0, ns_, T)
    torch.cuda.synchronize()
    S = out["S"].cpu().numpy()
    actor = rl.actor_model.get_weights()
    for k in range(0, 37, 6):
        ref = oroll.to_init_rollout(oe, actor, S0[k], 1)
        rS, rU, rT = ref
        assert rT == ns_[k]
        np.testing.assert_allclose(S[k, :rT + 1], rS, rtol=1e-4, atol=2e-4)
    assert (out["status"].cpu().numpy() == 0).all()


@pytest.mark.parametrize("system", SYSTEMS)
def test_rollout_per_step_consistency(system):
    """Every recorded step of a GPU rollout against the oracle evaluated at the GPU's own (s_t, a_t):
    a_t = actor(s_t) (float32 MFMA), s_{t+1} = simulate(s_t, a_t), r_t = reward(w_run, s_t, a_t),
    EE_t = EE(s_t) — checks the per-step kernels without trajectory divergence."""
    conf, genv, oe, nn, rl = _nets(system, None, seed=4)
    rng = random.Random(8)
    S0 = np.array([oe.reset(rng) for _ in range(40)])
    ns_ = [conf.NSTEPS - int(s[-1] / conf.dt) for s in S0]
    T = max(ns_)
    out = rl.rollout_batch(S0, ns_, T)
    torch.cuda.synchronize()
    S, A, R, EE = (out[k].cpu().numpy() for k in ("S", "A", "R", "EE"))
    actor = rl.actor_model.get_weights()
    norm = conf.state_norm_arr.astype(np.float64)
    w = conf.cost_weights_running
    for k in range(0, 40, 7):
        n = ns_[k]
        ts = sorted(set([0, 1, n // 2, n - 1]))
        a_ref = onn.actor_forward(actor, S[k, ts].astype(np.float32).astype(np.float64), norm)
        bound = F32_TOL * abs_bound("actor", actor, S[k, ts].astype(np.float32).astype(np.float64), norm)
        assert np.all(np.abs(A[k, ts] - a_ref) <= bound)
        for t in ts:
            a = A[k, t].astype(np.float64)
            np.testing.assert_allclose(S[k, t + 1], oe.simulate(S[k, t], a), rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(R[k, t], oe.reward(w, S[k, t], a), rtol=1e-10, atol=1e-14)
            np.testing.assert_allclose(EE[k, t], oe.get_end_effector_position(S[k, t]), rtol=1e-12, atol=1e-12)
    assert (out["status"].cpu().numpy() == 0).all()


@pytest.mark.parametrize("system,sched", [("double_integrator", (1, 3)), ("double_integrator", (2, 2)),
                                          ("manipulator", (4, 1)), ("car_park", (1, 2)), ("ur5", (2, 1)),
                                          ("double_integrator", (-1, 2)), ("double_integrator", (-1, 1)),
                                          ("car_park", (-1, 3)), ("double_integrator", (-3, 3)),
                                          ("double_integrator", (-3, 1)), ("double_integrator", (-3, 6)),
                                          ("single_integrator", (-3, 2)), ("car_park", (-3, 2)),
                                          ("car_park", (-3, 3)), ("car", (-3, 2)), ("manipulator", (-3, 1)),
                                          ("manipulator", (-3, 2)), ("manipulator", (-3, 4)), ("manipulator", (2, 3))])
def test_rollout_slot_refill_matches_one_episode_per_slot(system, sched):
    """Few workgroups force every slot to run several episodes back to back (refill at the step
    boundary, zero-length episodes completed on the spot); every episode must come out exactly as
    in a schedule with one episode per slot, and agree with the oracle's step-by-step semantics.
    groups = -1: the two-team kernel (k_rollout_tt, two 4-slot teams per workgroup on team
    barriers); groups = -3: one slot per wave with layer 2 split over K across the waves
    (k_rollout_ks, queue entries taken through an LDS counter; the manipulator's default, its
    planar closed-form dynamics) — all against the single-team kernel's one-episode-per-slot
    schedule (k_rollout<NJ, 1>, for the manipulator the same planar3_step)."""
    conf, genv, oe, nn, rl = _nets(system, None, seed=4)
    rng = random.Random(11)
    n_ep = 45
    S0 = np.array([oe.reset(rng) for _ in range(n_ep)])
    ns_ = [conf.NSTEPS - int(s[-1] / conf.dt) for s in S0]
    ns_[3] = 0
    ns_[17] = 1
    T = max(ns_)
    ref = rl.rollout_batch(S0, ns_, T, sched=(1, n_ep))
    got = rl.rollout_batch(S0, ns_, T, sched=sched)
    torch.cuda.synchronize()
    for k in range(n_ep):
        n = ns_[k]
        np.testing.assert_array_equal(got["S"][k, :n + 1].cpu().numpy(), ref["S"][k, :n + 1].cpu().numpy())
        np.testing.assert_array_equal(got["A"][k, :n].cpu().numpy(), ref["A"][k, :n].cpu().numpy())
        np.testing.assert_array_equal(got["R"][k, :n].cpu().numpy(), ref["R"][k, :n].cpu().numpy())
        np.testing.assert_array_equal(got["EE"][k, :n + 1].cpu().numpy(), ref["EE"][k, :n + 1].cpu().numpy())
    assert (got["status"].cpu().numpy() == 0).all()
    S, A, R, EE = (got[k].cpu().numpy() for k in ("S", "A", "R", "EE"))
    actor = rl.actor_model.get_weights()
    norm = conf.state_norm_arr.astype(np.float64)
    w = conf.cost_weights_running
    for k in range(0, n_ep, 5):
        n = ns_[k]
        if n == 0:
            np.testing.assert_array_equal(S[k, 0], S0[k])
            continue
        ts = sorted(set([0, n // 2, n - 1]))
        a_ref = onn.actor_forward(actor, S[k, ts].astype(np.float32).astype(np.float64), norm)
        bound = F32_TOL * abs_bound("actor", actor, S[k, ts].astype(np.float32).astype(np.float64), norm)
        assert np.all(np.abs(A[k, ts] - a_ref) <= bound)
        for t in ts:
            a = A[k, t].astype(np.float64)
            np.testing.assert_allclose(S[k, t + 1], oe.simulate(S[k, t], a), rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(R[k, t], oe.reward(w, S[k, t], a), rtol=1e-10, atol=1e-14)
        np.testing.assert_allclose(EE[k, n], oe.get_end_effector_position(S[k, n]), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("sched", [(0, 0), (-1, 2), (-1, 1), (1, 3), (-3, 2), (-3, 1)])
def test_rollout_zero_controls_ep0_exact(sched):
    """ep == 0 (zero warm-start controls, no actor) on the default schedule, on the two-team kernel
    (groups = -1: its loop has no actor barriers, so the team barrier that orders the loop test
    before wave 0 rewrites `anyact` is the only one per step) and on a refilling single-team one."""
    conf, genv, oe, nn, rl = _nets("double_integrator", None)
    rng = random.Random(6)
    S0 = np.array([oe.reset(rng) for _ in range(20)])
    ns_ = [conf.NSTEPS - int(s[-1] / conf.dt) for s in S0]
    out = rl.rollout_batch(S0, ns_, max(ns_), ep=0, sched=sched)
    torch.cuda.synchronize()
    S = out["S"].cpu().numpy()
    for k in range(20):
        rS, rU, rT = oroll.to_init_rollout(oe, None, S0[k], 0)
        np.testing.assert_array_equal(S[k, :rT + 1], rS)
    assert (out["status"].cpu().numpy() == 0).all()


# ------------------------------------------------------------------ replay
def test_buffer_add_gather_bit_exact(ref_vectors):
    from cacto_amd.replay_buffer import ReplayBuffer
    from cacto_amd.system import System
    conf = load_conf("double_integrator")

    class C:
        pass
    c = C()
    c.__dict__.update({k: getattr(conf, k) for k in dir(conf) if not k.startswith("__")})
    c.REPLAY_SIZE, c.BATCH_SIZE = 64, 16
    rb = ReplayBuffer(c, System(conf))
    rows = ref_vectors["rb_adds"]
    off = 0
    for L in ref_vectors["rb_eplens"]:
        rb.add_rows(rows[off:off + L])
        off += L
    np.testing.assert_array_equal(rb.storage.cpu().numpy(), ref_vectors["rb_storage"])
    assert [rb.next_idx, rb.full] == list(ref_vectors["rb_next_full"])
    out = rb.sample(torch.as_tensor(ref_vectors["rb_sidx"].astype(np.int32), device="cuda"))
    for name, got in zip(["s", "r", "sn", "dvdx", "d", "term", "w"], out[:7]):
        np.testing.assert_array_equal(got.cpu().numpy(), ref_vectors["rb_sample_" + name])


def test_per_sampling_bit_exact(ref_vectors):
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    from cacto_amd.system import System
    conf = load_conf("double_integrator")

    class C:
        pass
    c = C()
    c.__dict__.update({k: getattr(conf, k) for k in dir(conf) if not k.startswith("__")})
    c.BATCH_SIZE, c.prioritized_replay_alpha = 64, 0.6
    per = PrioritizedReplayBuffer(c, System(conf))
    leaves = ref_vectors["per_leaves"]
    per.set_leaves(np.arange(len(leaves)), leaves)
    per.next_idx = len(leaves)
    idx, w = per.sample_device(list(ref_vectors["per_u"]))
    np.testing.assert_array_equal(idx.cpu().numpy(), ref_vectors["per_idx"])
    assert per.sum_tree[1].item() == ref_vectors["per_ptotal"][1]
    # IS weights and exp_counter against the oracle
    o = obuf.PrioritizedReplayBuffer(65536, 5, 0.6, 0.6, 1e-2, 0.95, 64)
    for i, v in enumerate(leaves):
        o.it_sum[i] = float(v)
        o.it_min[i] = float(v)
    o.next_idx = len(leaves)
    ow = o.sample_weights(ref_vectors["per_idx"])
    np.testing.assert_allclose(w.cpu().numpy(), ow.astype(np.float32), rtol=1e-6)
    np.testing.assert_array_equal(per.exp_counter.cpu().numpy()[:len(leaves)], o.exp_counter[:len(leaves)])


def test_per_sample_global_matches_oracle(ref_vectors):
    """Sharded PER: local stratified indices, IS weights over the union of shards."""
    from cacto_amd import _lib as L
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    from cacto_amd.system import System, dptr, stream
    conf = load_conf("double_integrator")

    class C:
        pass
    c = C()
    c.__dict__.update({k: getattr(conf, k) for k in dir(conf) if not k.startswith("__")})
    c.BATCH_SIZE, c.prioritized_replay_alpha = 64, 0.6
    per = PrioritizedReplayBuffer(c, System(conf))
    leaves = ref_vectors["per_leaves"]
    per.set_leaves(np.arange(len(leaves)), leaves)
    per.next_idx = len(leaves)
    u = list(ref_vectors["per_u"])
    idx0, w0 = per.sample_device(u)
    stats = torch.empty(3, dtype=torch.float64, device="cuda")
    L.lib().call("cacto_per_shard_stats", dptr(per.sum_tree), dptr(per.min_tree), per.max_idx(), dptr(stats), stream())
    one = stats.reshape(1, 3).contiguous()
    ud = torch.as_tensor(np.asarray(u), device="cuda")
    for shards in (one, torch.cat([one, torch.tensor([[3.5, 1e-3, 700.0], [0.25, 0.2, 40.0]], dtype=torch.float64,
                                                     device="cuda")])):
        idx = torch.empty(len(u), dtype=torch.int32, device="cuda")
        w = torch.empty(len(u), dtype=torch.float32, device="cuda")
        L.lib().call("cacto_per_sample_global", dptr(per.sum_tree), dptr(per.min_tree), per.cap, per.max_idx(),
                     per.beta, dptr(ud), len(u), dptr(shards), shards.shape[0], dptr(idx), dptr(w), None, stream())
        np.testing.assert_array_equal(idx.cpu().numpy(), idx0.cpu().numpy())
        if shards.shape[0] == 1:
            np.testing.assert_array_equal(w.cpu().numpy(), w0.cpu().numpy())
        o = obuf.PrioritizedReplayBuffer(65536, 5, 0.6, 0.6, 1e-2, 0.95, 64)
        for i, v in enumerate(leaves):
            o.it_sum[i] = float(v)
            o.it_min[i] = float(v)
        o.next_idx = len(leaves)
        np.testing.assert_array_equal(shards[0].cpu().numpy(), o.shard_stats())
        ow = o.sample_weights_global(idx0.cpu().numpy(), shards.cpu().numpy())
        np.testing.assert_allclose(w.cpu().numpy(), ow.astype(np.float32), rtol=1e-6)


@pytest.mark.parametrize("cap", [2, 1024, 8192, 16384, 1 << 18, 1 << 20])
def test_per_sample_multi_workgroup_every_depth(cap):
    """The multi-workgroup sampler (B >= 512) at every split of the descent: all levels staged in
    LDS (cap <= 8192), a 1..4-level tail below the staged top, and three-level rounds above the
    tail (2^18, 2^20). Indices bit-exact, IS weights and exp_counter against the oracle."""
    from cacto_amd import _lib as L
    from cacto_amd.system import dptr, stream
    rng = np.random.default_rng(cap)
    leaves = rng.uniform(0.01, 2.0, size=cap) ** 0.6
    leaves[rng.integers(0, cap, size=max(1, cap // 7))] = 0.0  # empty slots (never sampled)
    st, mt = np.zeros(2 * cap), np.full(2 * cap, np.inf)
    st[cap:], mt[cap:] = leaves, np.where(leaves > 0, leaves, np.inf)
    lo = cap // 2
    while lo >= 1:  # parent = op(left, right) level by level, as SegmentTree.__setitem__ leaves it
        k = np.arange(lo, 2 * lo)
        st[k] = st[2 * k] + st[2 * k + 1]
        mt[k] = np.where(mt[2 * k + 1] < mt[2 * k], mt[2 * k + 1], mt[2 * k])
        lo //= 2
    o = obuf.PrioritizedReplayBuffer(cap, 1, 0.6, 0.6, 1e-2, 0.95, 0)
    o.it_sum.value, o.it_min.value = list(st), list(mt)
    max_idx = cap if cap <= 8192 else cap - 5
    o.N, o.next_idx, o.full = cap, max_idx % cap, max_idx == cap
    assert o.max_idx() == max_idx
    for B in (512, 1000):
        o.B = B
        u = rng.uniform(size=B)
        oidx = o.sample_proportional(list(u))
        ow = o.sample_weights(oidx)
        sd, md = torch.as_tensor(st, device="cuda"), torch.as_tensor(mt, device="cuda")
        ud = torch.as_tensor(u, device="cuda")
        idx = torch.empty(B, dtype=torch.int32, device="cuda")
        w = torch.empty(B, dtype=torch.float32, device="cuda")
        cnt = torch.zeros(cap, dtype=torch.float64, device="cuda")
        L.lib().call("cacto_per_sample", dptr(sd), dptr(md), cap, max_idx, 0.6, dptr(ud), B, dptr(idx), dptr(w),
                     dptr(cnt), stream())
        np.testing.assert_array_equal(idx.cpu().numpy(), oidx)
        np.testing.assert_allclose(w.cpu().numpy(), ow.astype(np.float32), rtol=1e-6)
        ref_cnt = np.zeros(cap)
        ref_cnt[oidx] += 1
        np.testing.assert_array_equal(cnt.cpu().numpy(), ref_cnt)


def test_per_update_priorities_matches_oracle():
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    from cacto_amd.system import System
    conf = load_conf("manipulator")
    per = PrioritizedReplayBuffer(conf, System(conf))
    o = obuf.PrioritizedReplayBuffer(conf.REPLAY_SIZE, conf.nb_state, 0.6, 0.6, conf.prioritized_replay_eps,
                                     conf.fresh_factor, conf.BATCH_SIZE)
    per.alpha = 0.6
    rng = np.random.default_rng(16)
    rows = rng.normal(size=(3000, 3 * conf.nb_state + 3))
    per.add_rows(rows)
    o.add_rows(rows)
    for it in range(3):
        u = list(rng.uniform(size=conf.BATCH_SIZE))
        idx, w = per.sample_device(u)
        oidx = o.sample_proportional(u)
        np.testing.assert_array_equal(idx.cpu().numpy(), oidx)
        o.sample_weights(oidx)
        y = rng.normal(size=(conf.BATCH_SIZE, 1)).astype(np.float32)
        V = rng.normal(size=(conf.BATCH_SIZE, 1)).astype(np.float32)
        idx[5] = idx[9]  # duplicates: last write wins
        oidx[5] = oidx[9]
        per.update_priorities_device(idx, torch.as_tensor(y, device="cuda"), torch.as_tensor(V, device="cuda"))
        o.update_priorities(oidx, y, V)
        torch.cuda.synchronize()
        st = per.sum_tree.cpu().numpy()
        np.testing.assert_allclose(st[65536:65536 + 3000], o.it_sum.value[65536:65536 + 3000], rtol=1e-6)
        np.testing.assert_allclose(st[1], o.it_sum.value[1], rtol=1e-6)


def test_per_new_leaves_after_priority_updates_match_host_pow():
    """Rows added after priority updates (max_priority != 1) get leaves max_priority ** alpha
    (replay_buffer.py:133-135, the host Python float power). The device computes the power in
    float64: the leaves must equal the host's bit for bit, and the stratified indices drawn over
    them must equal the oracle's."""
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    from cacto_amd.system import System
    conf = load_conf("car_park")
    per = PrioritizedReplayBuffer(conf, System(conf))
    per.alpha = 0.6
    o = obuf.PrioritizedReplayBuffer(conf.REPLAY_SIZE, conf.nb_state, 0.6, 0.6, conf.prioritized_replay_eps,
                                     conf.fresh_factor, conf.BATCH_SIZE)
    rng = np.random.default_rng(23)
    cols = 3 * conf.nb_state + 3
    rows = rng.normal(size=(2000, cols))
    per.add_rows(rows)
    o.add_rows(rows)
    for it in range(4):
        u = list(rng.uniform(size=conf.BATCH_SIZE))
        idx, _ = per.sample_device(u)
        oidx = o.sample_proportional(u)
        np.testing.assert_array_equal(idx.cpu().numpy(), oidx)
        o.sample_weights(oidx)                     # the IS weights step advances exp_counter
        y = (rng.normal(size=(conf.BATCH_SIZE, 1)) * (3 + it)).astype(np.float32)
        V = rng.normal(size=(conf.BATCH_SIZE, 1)).astype(np.float32)
        per.update_priorities_device(idx, torch.as_tensor(y, device="cuda"), torch.as_tensor(V, device="cuda"))
        o.update_priorities(oidx, y, V)
        more = rng.normal(size=(300, cols))
        n0 = per.next_idx
        per.add_rows(more)
        o.add_rows(more)
        torch.cuda.synchronize()
        maxp = float(per.max_priority.item())
        assert maxp == o.max_priority and maxp != 1.0
        leaves = per.sum_tree.cpu().numpy()[per.cap + n0:per.cap + n0 + 300]
        assert (leaves == maxp ** 0.6).all(), (leaves[0], maxp ** 0.6)
    u = list(rng.uniform(size=conf.BATCH_SIZE))
    np.testing.assert_array_equal(per.sample_device(u)[0].cpu().numpy(), o.sample_proportional(u))
