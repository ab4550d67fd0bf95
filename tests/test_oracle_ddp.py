"""Pinning of the DDP backward-pass oracle (oracle/ddp.py, TO.py:119-202) on CPU.

The sympy TO cost is checked against the oracle reward (itself pinned by the reference's golden
reward vectors: tests/test_oracle_golden.py) and its symbolic derivatives against central
differences of that reward; the recursion against a hand-unrolled one-step case."""
import random

import numpy as np
import pytest

from cacto_amd.confs import load_conf
from oracle import ddp
from oracle import env as oenv

SYSTEMS = list(ddp.SUPPORTED)


def _to_reward(conf, env, w, s, u):
    """The TO cost's reward (-cost) per the oracle env. UR5 is the one system whose Env.reward
    (environment.py:780-805: u.u) and TO cost (environment_TO.py:741-743: bound_control_cost)
    differ in the control term; the state part is the same."""
    if conf.system_id != "ur5":
        return env.reward(w, s, u)
    return env.reward(w, s, None) - conf.cost_funct_param[1] * w[6] * env.bound_control_cost(u)


def _sample(conf, env, rng):
    s = env.reset(rng)
    s[:-1] *= 1.2
    u = np.array([rng.uniform(-1.5, 1.5) * conf.u_max[i] for i in range(conf.nb_action)])
    return s, u


@pytest.mark.parametrize("system", SYSTEMS)
def test_sympy_cost_is_minus_reference_reward(system):
    conf = load_conf(system)
    env = oenv.make_env(conf)
    f = ddp.cost_functions(conf)
    rng = random.Random(3)
    n = conf.nb_state - 1
    for w in (conf.cost_weights_running, conf.cost_weights_terminal):
        for _ in range(20):
            s, u = _sample(conf, env, rng)
            r_sym = float(f["r"](s[:n], u, list(w[:7])))
            r_ref = _to_reward(conf, env, w, s, u)
            assert abs(r_sym - r_ref) <= 1e-12 * max(1.0, abs(r_ref)), (r_sym, r_ref)


@pytest.mark.parametrize("system", SYSTEMS)
def test_symbolic_derivatives_match_central_differences(system):
    conf = load_conf(system)
    env = oenv.make_env(conf)
    f = ddp.cost_functions(conf)
    rng = random.Random(4)
    n, m = conf.nb_state - 1, conf.nb_action
    w = list(conf.cost_weights_running[:7])
    for _ in range(8):
        s, u = _sample(conf, env, rng)
        x = s[:n]
        lx = np.reshape(f["lx"](x, w), n)
        lxx = np.asarray(f["lxx"](x, w), dtype=float)
        lu = np.reshape(f["lu"](u, w), m)
        luu = np.asarray(f["luu"](u, w), dtype=float)
        assert np.allclose(np.asarray(f["lxu"](x, u, w), dtype=float), 0.0)   # separable cost: l_xu = 0
        h = 1e-5

        def R(xx, uu):
            ss = s.copy()
            ss[:n] = xx
            return _to_reward(conf, env, conf.cost_weights_running, ss, uu)

        for i in range(n):
            e = np.zeros(n)
            e[i] = h
            fd = (R(x + e, u) - R(x - e, u)) / (2 * h)
            assert abs(fd - lx[i]) <= 1e-5 * max(1.0, abs(lx[i])), (i, fd, lx[i])
            gp = np.reshape(f["lx"](x + e, w), n)
            gm = np.reshape(f["lx"](x - e, w), n)
            np.testing.assert_allclose((gp - gm) / (2 * h), lxx[i], rtol=1e-4, atol=1e-6 * (1 + abs(lxx).max()))
        for j in range(m):
            e = np.zeros(m)
            e[j] = h
            fd = (R(x, u + e) - R(x, u - e)) / (2 * h)
            assert abs(fd - lu[j]) <= 1e-5 * max(1.0, abs(lu[j]))
            gp = np.reshape(f["lu"](u + e, w), m)
            gm = np.reshape(f["lu"](u - e, w), m)
            np.testing.assert_allclose((gp - gm) / (2 * h), luu[j], rtol=1e-4, atol=1e-9)


@pytest.mark.parametrize("system", SYSTEMS)
def test_augmented_derivative_matches_simulate(system):
    """Fx, Fu are the Jacobians of Env.simulate (float64 path) without the time row/column."""
    conf = load_conf(system)
    env = oenv.make_env(conf)
    rng = random.Random(5)
    n, m = conf.nb_state - 1, conf.nb_action
    for _ in range(5):
        s, u = _sample(conf, env, rng)
        A, B = ddp.augmented_derivative(conf, s[:n], u)
        h = 1e-6
        for i in range(n):
            e = np.zeros(conf.nb_state)
            e[i] = h
            col = (env.simulate(s + e, u) - env.simulate(s - e, u))[:n] / (2 * h)
            np.testing.assert_allclose(col, A[:, i], rtol=1e-6, atol=1e-8)
        for j in range(m):
            e = np.zeros(m)
            e[j] = h
            col = (env.simulate(s, u + e) - env.simulate(s, u - e))[:n] / (2 * h)
            np.testing.assert_allclose(col, B[:, j], rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("system", SYSTEMS)
def test_one_step_recursion(system):
    """T = 2 states: V_x(s_0) = Q_x - Q_xu (Q_uu + mu)^-1 Q_u written out directly."""
    conf = load_conf(system)
    env = oenv.make_env(conf)
    f = ddp.cost_functions(conf)
    rng = random.Random(6)
    n, m = conf.nb_state - 1, conf.nb_action
    s0, u0 = _sample(conf, env, rng)
    s1 = env.simulate(s0, u0)
    V = ddp.backward_pass(conf, np.stack([s0, s1]), u0[None])
    wr, wt = list(conf.cost_weights_running[:7]), list(conf.cost_weights_terminal[:7])
    Vx1 = np.reshape(f["lx"](s1[:n], wt), n)
    Vxx1 = np.asarray(f["lxx"](s1[:n], wt), dtype=float)
    np.testing.assert_allclose(V[1, :n], Vx1, rtol=1e-14, atol=0)
    A, B = ddp.augmented_derivative(conf, s0[:n], u0)
    Qx = np.reshape(f["lx"](s0[:n], wr), n) + A.T @ Vx1
    Qu = np.reshape(f["lu"](u0, wr), m) + B.T @ Vx1
    Quu = np.asarray(f["luu"](u0, wr), dtype=float) + B.T @ Vxx1 @ B + 1e-9 * np.eye(m)
    Qxu = A.T @ Vxx1 @ B
    np.testing.assert_allclose(V[0, :n], Qx - Qxu @ np.linalg.solve(Quu, Qu), rtol=1e-9, atol=1e-12)
    assert V[0, n] == 0.0 and V[1, n] == 0.0
