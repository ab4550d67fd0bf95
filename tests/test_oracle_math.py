"""Internal checks that pin the oracle where no reference executable exists:
finite differences for every gradient (incl. the Sobolev second-order term), an independent
sympy Lagrangian for the planar manipulator, DI M = I / nle = 0, and the DI final-policy
known-answer test against the reference's figure."""
import math
import os

import numpy as np
import pytest

from conftest import load_weights
from oracle import buffer as obuf
from oracle import dynamics as odyn
from oracle import env as oenv
from oracle import nn as onn
from oracle import rollout as oroll
from cacto_amd.confs import load_conf


def _rand_params(rng, shapes, scale=0.3):
    return [rng.normal(scale=scale, size=s) for s in shapes]


def critic_shapes(ns):
    return [(ns, 64), (64,), (64, 64), (64,), (64, 128), (128,), (128, 128), (128,), (128, 1), (1,)]


def actor_shapes(ns, na):
    return [(ns, 256), (256,), (256, 256), (256,), (256, na), (na,)]


@pytest.mark.parametrize("acts", [onn.SINE, onn.SINE_ELU])
@pytest.mark.parametrize("w_S", [0.0, 1e-2])
def test_critic_grad_fd(w_S, acts):
    rng = np.random.default_rng(0)
    ns, B = 5, 6
    norm = np.array([15., 15., 6., 6., 10.])
    crit = _rand_params(rng, critic_shapes(ns))
    tgt = _rand_params(rng, critic_shapes(ns))
    S = rng.uniform(-10, 10, size=(B, ns)); S[:, -1] = rng.uniform(0, 9, size=B)
    Sn = rng.uniform(-10, 10, size=(B, ns))
    R = rng.normal(size=(B, 1)); d = (rng.uniform(size=(B, 1)) < .4) * 1.0
    dVdx = rng.normal(size=(B, ns)); w = rng.uniform(.5, 2, size=(B, 1))
    grads = onn.compute_critic_grad(crit, tgt, S, Sn, R, dVdx, d, w, w_S, norm, acts=acts)[0]
    f = lambda P: onn.critic_loss(P, tgt, S, Sn, R, dVdx, d, w, w_S, norm, acts=acts)
    eps = 1e-6
    for li, (p, g) in enumerate(zip(crit, grads)):
        flat = p.reshape(-1)
        for k in rng.choice(flat.size, size=min(6, flat.size), replace=False):
            old = flat[k]
            flat[k] = old + eps; fp = f(crit)
            flat[k] = old - eps; fm = f(crit)
            flat[k] = old
            fd = (fp - fm) / (2 * eps)
            assert abs(fd - g.reshape(-1)[k]) <= 1e-6 * max(1.0, abs(fd)), (li, k, fd, g.reshape(-1)[k])


@pytest.mark.parametrize("acts", [onn.SINE, onn.SINE_ELU])
def test_critic_input_grad_fd(acts):
    rng = np.random.default_rng(1)
    ns = 7
    norm = np.array([15., 15., 15., 10., 10., 10., 5.])
    crit = _rand_params(rng, critic_shapes(ns))
    S = rng.uniform(-3, 3, size=(4, ns))
    g, _ = onn.critic_input_grad(crit, S, norm, acts=acts)
    eps = 1e-6
    for j in range(ns):
        Sp, Sm = S.copy(), S.copy()
        Sp[:, j] += eps; Sm[:, j] -= eps
        fd = (onn.critic_forward(crit, Sp, norm, acts=acts) - onn.critic_forward(crit, Sm, norm, acts=acts))[:, 0] / (2 * eps)
        np.testing.assert_allclose(g[:, j], fd, rtol=1e-6, atol=1e-8)


def test_actor_grad_fd():
    """Actor grad against FD of mean(-dQ_da . pi(s)) with dQ_da frozen (NeuralNetwork.py:219-231)."""
    conf = load_conf("double_integrator")
    env = oenv.make_env(conf)
    rng = np.random.default_rng(2)
    norm = conf.state_norm_arr.astype(float)
    act = _rand_params(rng, actor_shapes(5, 2), 0.1)
    crit = _rand_params(rng, critic_shapes(5), 0.3)
    S = np.column_stack([rng.uniform(-15, 15, (8, 4)), rng.uniform(0, 9.9, 8)])
    term = (rng.uniform(size=(8, 1)) < .3) * 1.0
    g = onn.compute_actor_grad(env, act, crit, S, term, norm)
    dQ = onn.actor_dq_da(env, act, crit, S, term, norm)[0]
    f = lambda P: np.mean(np.sum(-dQ * onn.actor_forward(P, S, norm), axis=1))
    eps = 1e-6
    for li, (p, gl) in enumerate(zip(act, g)):
        flat = p.reshape(-1)
        for k in rng.choice(flat.size, size=min(5, flat.size), replace=False):
            old = flat[k]
            flat[k] = old + eps; fp = f(act)
            flat[k] = old - eps; fm = f(act)
            flat[k] = old
            fd = (fp - fm) / (2 * eps)
            assert abs(fd - gl.reshape(-1)[k]) <= 1e-6 * max(1e-3, abs(fd)), (li, k, fd, gl.reshape(-1)[k])


def test_dr_da_matches_fd_of_reward_batch():
    conf = load_conf("manipulator")
    env = oenv.make_env(conf)
    rng = np.random.default_rng(3)
    W = np.tile(conf.cost_weights_running, (4, 1))
    S = rng.uniform(-1, 1, size=(4, 7))
    A = rng.uniform(-150, 150, size=(4, 3))
    g = env.dr_da(W, A)
    u = lambda A: -W[:, 6] * env.scale * np.sum(A * A + conf.w_b * (A / conf.u_max) ** 10, axis=1)
    for j in range(3):
        e = np.zeros_like(A); e[:, j] = 1e-4
        np.testing.assert_allclose(g[:, j], (u(A + e) - u(A - e)) / 2e-4, rtol=1e-6)


def test_double_integrator_chain_is_unit_mass():
    conf = load_conf("double_integrator")
    ch = odyn.Chain.from_model(conf.robot)
    rng = np.random.default_rng(4)
    for _ in range(5):
        q, v = rng.normal(size=2) * 10, rng.normal(size=2)
        np.testing.assert_array_equal(ch.mass_matrix(q), np.eye(2))
        np.testing.assert_array_equal(ch.nle(q, v), np.zeros(2))
        np.testing.assert_array_equal(ch.frame_position(q), [q[0], q[1], 0.0])


def _manip_lagrangian():
    """Independent derivation: planar 3-link arm, links of length l, COM at r, mass m,
    inertia izz about the COM; gravity normal to the plane."""
    import sympy as sp
    q = sp.symbols('q0:3'); qd = sp.symbols('qd0:3')
    l, r, m, I = 10, 5, sp.Rational(1, 2), sp.Rational(50, 3)
    T = 0
    th = 0
    px = py = 0
    for k in range(3):
        th = th + q[k]
        cx = px + r * sp.cos(th); cy = py + r * sp.sin(th)
        vx = sum(sp.diff(cx, q[j]) * qd[j] for j in range(3))
        vy = sum(sp.diff(cy, q[j]) * qd[j] for j in range(3))
        w = sum(qd[: k + 1])
        T += m * (vx ** 2 + vy ** 2) / 2 + I * w ** 2 / 2
        px = px + l * sp.cos(th); py = py + l * sp.sin(th)
    M = sp.Matrix(3, 3, lambda i, j: sp.diff(T, qd[i], qd[j]))
    h = sp.Matrix([sum(sp.diff(M[i, j], q[k]) * qd[j] * qd[k] for j in range(3) for k in range(3))
                   - sp.diff(T, q[i]) for i in range(3)])
    ee = (-7 + px, py)
    f = sp.lambdify((q, qd), (M, h, ee), 'numpy')
    return f


def test_manipulator_chain_matches_lagrangian():
    conf = load_conf("manipulator")
    ch = odyn.Chain.from_model(conf.robot)
    f = _manip_lagrangian()
    rng = np.random.default_rng(5)
    for _ in range(6):
        q, v = rng.uniform(-math.pi, math.pi, 3), rng.uniform(-2, 2, 3)
        M, h, ee = f(q, v)
        np.testing.assert_allclose(ch.mass_matrix(q), np.asarray(M, dtype=float), rtol=1e-12, atol=1e-10)
        np.testing.assert_allclose(ch.nle(q, v), np.asarray(h, dtype=float).ravel(), rtol=1e-11, atol=1e-9)
        np.testing.assert_allclose(ch.frame_position(q)[:2], np.asarray(ee, dtype=float), atol=1e-12)


def test_di_final_policy_known_answer():
    """KAT: roll out actor_final.h5 from init_states_sim with DI dynamics; the
    per-trajectory max y and end points reproduce Figures/N_try_6/PolicyEvaluationSingleInit_6_51000.png."""
    conf = load_conf("double_integrator")
    env = oenv.make_env(conf)
    actor = load_weights("di_seed0_final")["actor"]
    maxy, ends = {}, {}
    for s0 in conf.init_states_sim:
        S, A, R, EE = oroll.policy_rollout(env, actor, s0, conf.NSTEPS)
        maxy[(s0[0], s0[1])] = EE[:, 1].max()
        ends[(s0[0], s0[1])] = EE[-1, :2]
    assert abs(maxy[(2.0, 0.0)] - 3.74) < 0.01
    assert abs(maxy[(10.0, 0.0)] - 7.88) < 0.01
    assert abs(maxy[(10.0, 10.0)] - 10.0) < 0.01
    assert abs(maxy[(12.0, 2.0)] - 8.70) < 0.01
    assert abs(maxy[(15.0, 0.0)] - 9.44) < 0.01
    assert abs(ends[(10.0, 10.0)][0] + 19.3) < 0.2
    near = [np.hypot(e[0] + 8, e[1] + 0.9) < 1.5 for e in ends.values()]
    assert sum(near) >= 5


def _fk_links(model, q):
    """Independent forward kinematics (4x4 homogeneous transforms + Rodrigues), per link:
    world rotation R_i and COM position c_i (robots.py model conventions: joint frame placed in
    the parent joint frame by (R, p), then rotated about `axis` by q_i)."""
    def rod(axis, th):
        a = np.asarray(axis, float) / np.linalg.norm(axis)
        K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
        return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    Ts, out = [], []
    for i, j in enumerate(model.joints):
        T = np.eye(4)
        T[:3, :3], T[:3, 3] = j.R, j.p
        J = np.eye(4)
        J[:3, :3] = rod(j.axis, q[i])
        Tw = (Ts[j.parent] if j.parent >= 0 else np.eye(4)) @ T @ J
        Ts.append(Tw)
        out.append((Tw[:3, :3], Tw[:3, :3] @ j.com + Tw[:3, 3]))
    return out


def _lagrangian_terms(model, q, v, eps=1e-6):
    """M(q) from link Jacobians (finite differences of the independent FK) and
    h(q, v) = Mdot v - 1/2 d(v'Mv)/dq + dV/dq (Lagrange's equations), by central differences."""
    n = len(q)
    g = np.asarray(model.gravity, float)

    def mass(qq):
        links = _fk_links(model, qq)
        M = np.zeros((n, n))
        for i, j in enumerate(model.joints):
            Jv, Jw = np.zeros((3, n)), np.zeros((3, n))
            for k in range(n):
                dq = np.zeros(n)
                dq[k] = eps
                Rp, cp = _fk_links(model, qq + dq)[i]
                Rm, cm = _fk_links(model, qq - dq)[i]
                Jv[:, k] = (cp - cm) / (2 * eps)
                W = (Rp - Rm) / (2 * eps) @ links[i][0].T   # skew(omega_k)
                Jw[:, k] = [W[2, 1], W[0, 2], W[1, 0]]
            R = links[i][0]
            M += j.mass * Jv.T @ Jv + Jw.T @ (R @ j.inertia @ R.T) @ Jw
        return M

    def potential(qq):
        return -sum(j.mass * g @ c for j, (_, c) in zip(model.joints, _fk_links(model, qq)))

    M = mass(q)
    h = np.zeros(n)
    e2 = 1e-4
    Mdot = (mass(q + e2 * v) - mass(q - e2 * v)) / (2 * e2)
    h += Mdot @ v
    for k in range(n):
        dq = np.zeros(n)
        dq[k] = e2
        h[k] -= 0.5 * (v @ mass(q + dq) @ v - v @ mass(q - dq) @ v) / (2 * e2)
        h[k] += (potential(q + dq) - potential(q - dq)) / (2 * e2)
    return M, h


def test_ur5_chain_matches_lagrangian():
    """UR5 (6-DoF, 3-D, gravity) oracle CRBA/RNEA vs an independent Lagrangian evaluation. Pinocchio
    (the reference's dynamics, pin 2.9.2) is absent: UR5 parity is pinned by this internal
    consistency only."""
    from cacto_amd.robots import builtin_model
    from oracle.dynamics import Chain
    model = builtin_model("ur5")
    chain = Chain.from_model(model)
    rng = np.random.default_rng(5)
    for _ in range(3):
        q = rng.uniform(-np.pi, np.pi, 6)
        v = rng.uniform(-1, 1, 6)
        M_ref, h_ref = _lagrangian_terms(model, q, v)
        np.testing.assert_allclose(chain.mass_matrix(q), M_ref, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(chain.nle(q, v), h_ref, rtol=1e-5, atol=1e-5)
        # EE frame: wrist_3 placement composed with the fixed EE offset
        ee = chain.frame_position(q)
        Tw = np.eye(4)
        for i, j in enumerate(model.joints):
            A = np.eye(4)
            A[:3, :3], A[:3, 3] = j.R, j.p
            Jr = np.eye(4)
            a = j.axis / np.linalg.norm(j.axis)
            K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
            Jr[:3, :3] = np.eye(3) + np.sin(q[i]) * K + (1 - np.cos(q[i])) * K @ K
            Tw = Tw @ A @ Jr
        np.testing.assert_allclose(ee, Tw[:3, :3] @ model.ee_p + Tw[:3, 3], atol=1e-12)


def test_vectorised_di_rollout_matches_per_sample_port():
    """bench.py's vectorised CPU baseline computes the same trajectories as the per-sample port."""
    import random
    from cacto_amd.confs import load_conf
    from oracle import env as oenv
    from oracle import rollout as oroll
    conf = load_conf("double_integrator")
    oe = oenv.make_env(conf)
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "weights", "di_seed0_0.npz"))
    actor = [z["actor_%d" % i] for i in range(6)]
    rng = random.Random(4)
    S0 = np.array([oe.reset(rng) for _ in range(12)])
    n = np.array([oroll.nsteps_sh(conf, s) for s in S0])
    steps, S = oroll.batched_policy_rollout_di(oe, actor, S0, n)
    assert steps == int(n.sum())
    for e in range(len(S0)):
        ref = oroll.policy_rollout(oe, actor, S0[e], int(n[e]))[0][-1]
        np.testing.assert_allclose(S[e], ref, rtol=1e-12, atol=1e-12)


def test_prefix_terms_closed_form_matches_reduce_walk():
    """The multi-workgroup sampler (cacto_amd/csrc/per_device.h) forms prefix_reduce's terms of
    sum(0, end) in closed form: the walk stops at depth d* = L - min(trailing ones of end, L) with
    that node itself as the last term, and above it a right step at depth k (bit L-1-k of end set)
    adds the node's left child. Same nodes, same order, as the recursion of SegmentTree._reduce
    (segment_tree.py:76-98) — checked here for every end of every capacity up to 2^10 and sampled
    ends up to 2^20."""
    def walk(cap, end):  # the recursion's path (reduce(0, end) with end inclusive)
        terms, node, ns, ne = [], 1, 0, cap - 1
        while True:
            if end == ne:
                terms.append(node)
                return terms
            mid = (ns + ne) // 2
            if end <= mid:
                node, ne = 2 * node, mid
            else:
                terms.append(2 * node)
                node, ns = 2 * node + 1, mid + 1

    def closed(cap, end):
        L = cap.bit_length() - 1
        ones = 0
        while ones < L and (end >> ones) & 1:
            ones += 1
        dstar = L - ones
        out = []
        for k in range(dstar + 1):
            if k == dstar:
                out.append((1 << k) | (end >> (L - k)))
            elif (end >> (L - 1 - k)) & 1:
                out.append(((1 << k) | (end >> (L - k))) * 2)
        return out

    rng = np.random.default_rng(0)
    for L in range(0, 21):
        cap = 1 << L
        ends = range(cap) if cap <= 1024 else rng.integers(0, cap, size=2000)
        for end in ends:
            assert closed(cap, int(end)) == walk(cap, int(end)), (cap, end)
    # and the sums agree with SegmentTree.sum on a random tree (the right-nested combination)
    t = obuf.SumSegmentTree(1 << 12)
    vals = rng.uniform(0, 1, size=1 << 12)
    for i, v in enumerate(vals):
        t[i] = float(v)
    for end in rng.integers(1, 1 << 12, size=200):
        terms = closed(1 << 12, int(end) - 1)
        r = t.value[terms[-1]]
        for node in reversed(terms[:-1]):
            r = t.value[node] + r
        assert r == t.sum(0, int(end))
