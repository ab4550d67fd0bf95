"""Oracle: the DDP backward pass that gives the Sobolev labels dV/dx — test infrastructure only
(see oracle/__init__).

Restates `TO.backward_pass` (TO.py:119-202) for every system: the TO costs of SI / DI / Car (the
planar family, environment_TO.py:90-111, :208-234, :339-360), car_park (:450-503), manipulator
(:605-631) and UR5 (:731-758); `augmented_derivative` of SI (environment.py:221-233), Car
(:420-435), CarPark (:567-582) and the Pinocchio chains (environment.py:111-132): for the
prismatic double integrator ddq_dq = ddq_dv = 0 (M and nle do not depend on (q, v)); for the
revolute chains computeABADerivatives is restated by complex-step differentiation of the oracle's
forward dynamics (oracle/dynamics.py, itself pinned by the reference's golden vectors).

The cost derivatives are taken the way the reference takes them — symbolically (for the chains
through the chain rule over the sympy forward kinematics): the TO cost is
rebuilt in sympy from the same formulas (CasADi's `cost_fun`) and differentiated with
`sympy.hessian` / `sympy.diff` (the reference: `casadi.hessian`, `casadi.jacobian`, TO.py:145-149),
then lambdified to numpy. `running_cost = -cost` (TO.py:142-143): the DDP works on the reward.
The recursion keeps the reference's operation order, with `np.linalg.pinv` (TO.py:189-190).

Pinning: the sympy cost equals -reward of oracle/env.py (pinned by the reference's golden reward
vectors) at sample points, and its derivatives agree with central differences of that reward
(tests/test_oracle_ddp.py).
"""
import functools

import numpy as np
import sympy as sp

SUPPORTED = ("single_integrator", "double_integrator", "car", "car_park", "manipulator", "ur5")
CHAINS = ("manipulator", "ur5")


def system_of(conf):
    """System id of a conf module (cacto_amd.confs.conf_<system_id>)."""
    return conf.__name__.rsplit(".", 1)[-1][len("conf_"):]


def _n_m(conf):
    return conf.nb_state - 1, conf.nb_action


@functools.lru_cache(maxsize=None)
def _cost_functions(system, key):
    """Lambdified reward derivatives of one system's TO cost: l_x(x, w), l_xx(x, w), l_u(u, w),
    l_uu(u, w), l_xu(x, u, w) and the reward itself. `key` carries the conf numbers (hashable)."""
    (n, m, offset, scale, alpha, alpha2, obs, target, w_b, u_max, nq, vel_cost) = key
    x = sp.symbols("x0:%d" % n, real=True)
    u = sp.symbols("u0:%d" % m, real=True)
    w = sp.symbols("w0:7", real=True)
    px, py = x[0], x[1]          # p_ee: SI / Car states (environment_TO.py:76-81), DI q (prismatic x, y)

    def ell(xc, yc, A, B):       # environment_TO.py:211-213
        return sp.log(sp.exp(alpha * -(((px - xc) ** 2) / ((A / 2) ** 2) + ((py - yc) ** 2) / ((B / 2) ** 2) - 1.0))
                      + 1) / alpha

    o = obs
    ell1, ell2, ell3 = ell(o[0], o[1], o[6], o[7]), ell(o[2], o[3], o[8], o[9]), ell(o[4], o[5], o[10], o[11])
    u_cost = sum(u[i] * u[i] + w_b * (u[i] / u_max[i]) ** 10 for i in range(m))       # :201-206
    dist = (px - target[0]) ** 2 + (py - target[1]) ** 2
    peak = sp.log(sp.exp(alpha2 * -(sp.sqrt((px - target[0]) ** 2 + 0.1) - 0.1 + sp.sqrt((py - target[1]) ** 2 + 0.1)
                                    - 0.1 - 2 * sp.sqrt(0.1))) + 1) / alpha2
    cost = w[0] * dist - w[1] * peak
    if vel_cost:                                                                        # DI :227-230
        cost = cost + w[2] * sum(x[nq + i] ** 2 for i in range(n - nq))
    cost = scale * (cost + w[3] * ell1 + w[4] * ell2 + w[5] * ell3 + w[6] * u_cost - offset)
    r = -cost                                                                           # TO.py:142
    X, U = sp.Matrix(x), sp.Matrix(u)
    args_x, args_u, args_xu = (x, w), (u, w), (x, u, w)
    lx = sp.Matrix([r]).jacobian(X).T
    lxx = sp.hessian(r, X)
    lu = sp.Matrix([r]).jacobian(U).T
    luu = sp.hessian(r, U)
    lxu = lx.jacobian(U)
    f = lambda args, e: sp.lambdify(args, e, "numpy")  # noqa: E731
    return dict(r=f(args_xu, r), lx=f(args_x, lx), lxx=f(args_x, lxx), lu=f(args_u, lu), luu=f(args_u, luu),
                lxu=f(args_xu, lxu))


def _u_cost_sym(u, m, w_b, u_max):
    return sum(u[i] * u[i] + w_b * (u[i] / u_max[i]) ** 10 for i in range(m))    # bound_control_cost


def _peak_sym(alpha2, d):
    s = sum(sp.sqrt(dk ** 2 + 0.1) - sp.sqrt(0.1) - 0.1 for dk in d)
    return sp.log(sp.exp(alpha2 * -s) + 1) / alpha2


@functools.lru_cache(maxsize=None)
def _car_park_functions(key):
    """car_park TO cost (environment_TO.py:450-503) over x = (x, y, theta, v, delta). sympy
    differentiates the smooth box obs_cost_fun (:457-461) in the check-point coordinates (X, Y) and
    the target terms in the EE position; both are composed with the rigid maps
    Z_k(x, y, theta) = p_ee + R(theta) c_k (:482-486) by the chain rule (their derivatives in theta are
    closed forms: dZ/dtheta = (-(Z_y - y), Z_x - x), d2Z/dtheta2 = -(Z - (x, y)))."""
    (n, m, offset, scale, alpha2, obs, target, w_b, u_max, L_delta, k_db, checks) = key
    X, Y, xs, ys, Wx, Wy = sp.symbols("X Y xs ys Wx Wy", real=True)
    k = k_db
    t1 = 4 + 4 * (Y - ys + Wy / 2) ** 2 * k ** 2
    t2 = 4 + 4 * (Y - ys - Wy / 2) ** 2 * k ** 2
    t3 = 4 + 4 * (X - xs + Wx / 2) ** 2 * k ** 2
    t4 = 4 + 4 * (X - xs - Wx / 2) ** 2 * k ** 2
    box = (t1 ** sp.Rational(-1, 2) * (-sp.sqrt(t2) / 2 + (Y - ys - Wy / 2) * k) * t3 ** sp.Rational(-1, 2)
           * t2 ** sp.Rational(-1, 2) * (sp.sqrt(t1) / 2 + (Y - ys + Wy / 2) * k) * t4 ** sp.Rational(-1, 2)
           * (sp.sqrt(t3) / 2 + (X - xs + Wx / 2) * k) * (-sp.sqrt(t4) / 2 + (X - xs - Wx / 2) * k))
    Zs = sp.Matrix([X, Y])
    bargs = (X, Y, xs, ys, Wx, Wy)
    f_box = sp.lambdify(bargs, box, "numpy")
    f_bg = sp.lambdify(bargs, sp.Matrix([box]).jacobian(Zs).T, "numpy", cse=True)
    f_bH = sp.lambdify(bargs, sp.hessian(box, Zs), "numpy", cse=True)
    P = sp.symbols("p0:2", real=True)
    w = sp.symbols("w0:7", real=True)
    u = sp.symbols("u0:%d" % m, real=True)
    d = (P[0] - target[0], P[1] - target[1])
    pos = w[0] * (d[0] ** 2 + d[1] ** 2) - w[1] * _peak_sym(alpha2, d)
    Pm = sp.Matrix(P)
    f_pos = sp.lambdify((P, w), pos, "numpy")
    f_pg = sp.lambdify((P, w), sp.Matrix([pos]).jacobian(Pm).T, "numpy", cse=True)
    f_pH = sp.lambdify((P, w), sp.hessian(pos, Pm), "numpy", cse=True)
    r_u = -scale * w[6] * _u_cost_sym(u, m, w_b, u_max)
    U = sp.Matrix(u)
    lu = sp.lambdify((u, w), sp.Matrix([r_u]).jacobian(U).T, "numpy")
    luu = sp.lambdify((u, w), sp.hessian(r_u, U), "numpy")
    f_ru = sp.lambdify((u, w), r_u, "numpy")
    boxes = [(obs[2 * ob], obs[2 * ob + 1], obs[6 + 2 * ob], obs[7 + 2 * ob]) for ob in range(3)]

    def points(x):
        c, s_ = np.cos(x[2]), np.sin(x[2])
        pe = np.array([x[0] + c * (L_delta / 2), x[1] + s_ * (L_delta / 2)])
        return pe, [np.array([c * bx - s_ * by, s_ * bx + c * by]) + pe for (bx, by) in checks]

    def terms(x):
        """(value, gradient, Hessian) of each position term as a function of a planar point Z,
        together with Z itself: the target terms at p_ee, then every (box, check point) pair."""
        pe, Zk = points(x)
        out = [(f_pos(pe, w_), np.reshape(f_pg(pe, w_), 2), np.asarray(f_pH(pe, w_), dtype=float), pe, wsc)
               for (w_, wsc) in [(W[0], 1.0)]]
        for (bxs, bys, bwx, bwy) in boxes:
            for Z in Zk:
                a = (Z[0], Z[1], bxs, bys, bwx, bwy)
                out.append((f_box(*a), np.reshape(f_bg(*a), 2), np.asarray(f_bH(*a), dtype=float), Z, W[0][3]))
        return out

    W = [None]

    def lx_lxx(x, wv):
        x = np.asarray(x, dtype=np.float64)
        W[0] = list(wv)
        lx, lxx = np.zeros(n), np.zeros((n, n))
        for (_, g, H, Z, wsc) in terms(x):
            dth = np.array([-(Z[1] - x[1]), Z[0] - x[0]])        # dZ/dtheta
            J = np.array([[1.0, 0.0, dth[0]], [0.0, 1.0, dth[1]]])
            lx[:3] += -scale * wsc * (J.T @ g)
            Hx = J.T @ H @ J
            Hx[2, 2] += g @ -(Z - x[:2])                           # d2Z/dtheta2
            lxx[:3, :3] += -scale * wsc * Hx
        lx[3] = -scale * wv[2] * 2.0 * x[3]
        lxx[3, 3] = -scale * wv[2] * 2.0
        return lx, lxx

    def r(x, uu, wv):
        x = np.asarray(x, dtype=np.float64)
        W[0] = list(wv)
        t = terms(x)
        obs_cost = sum(v for (v, _, _, _, _) in t[1:])
        return (-scale * (t[0][0] + wv[2] * x[3] ** 2 + wv[3] * obs_cost - offset)) + f_ru(uu, wv)

    return dict(r=r, lx=lambda x, wv: lx_lxx(x, wv)[0], lxx=lambda x, wv: lx_lxx(x, wv)[1], lu=lu, luu=luu,
                lxu=lambda x, uu, wv: np.zeros((n, m)))


def _lambdify_all(r, x, u, w):
    X, U = sp.Matrix(x), sp.Matrix(u)
    lx = sp.Matrix([r]).jacobian(X).T
    f = lambda args, e: sp.lambdify(args, e, "numpy", cse=True)  # noqa: E731
    return dict(r=f((x, u, w), r), lx=f((x, w), lx), lxx=f((x, w), sp.hessian(r, X)),
                lu=f((u, w), sp.Matrix([r]).jacobian(U).T), luu=f((u, w), sp.hessian(r, U)),
                lxu=f((x, u, w), lx.jacobian(U)))


def _fk_sym(chain, q):
    """EE translation of the chain (Pinocchio framesForwardKinematics + oMf['EE'].translation, the
    p_ee CasADi function of environment_TO.py:584-585 / :716-717) as a sympy 3-vector."""
    oR, op = [None] * chain.n, [None] * chain.n
    for i in range(chain.n):
        R0 = sp.Matrix(chain.R0[i])
        if chain.kind[i] == 0:
            ax = chain.axis[i]
            K = sp.Matrix([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
            R = R0 * (sp.eye(3) + sp.sin(q[i]) * K + (1 - sp.cos(q[i])) * K * K)
            p = sp.Matrix(chain.p0[i])
        else:
            R = R0
            p = sp.Matrix(chain.p0[i]) + R0 * sp.Matrix(chain.axis[i]) * q[i]
        if chain.parent[i] < 0:
            oR[i], op[i] = R, p
        else:
            pr = chain.parent[i]
            oR[i], op[i] = oR[pr] * R, oR[pr] * p + op[pr]
    j = chain.ee_parent
    return oR[j] * sp.Matrix(chain.ee_p) + op[j]


_CHAIN_CACHE = {}


def _chain_functions(conf, key):
    """Manipulator / UR5 TO cost (environment_TO.py:605-631 / :731-758): reward r(p_ee(q), v, u).
    sympy differentiates the cost in the EE position P and the forward kinematics p(q) separately;
    l_q = J^T dr/dP, l_qq = J^T d2r/dP2 J + sum_c dr/dP_c d2p_c/dq2 (chain rule)."""
    if key in _CHAIN_CACHE:
        return _CHAIN_CACHE[key]
    from .env import make_env
    (name, n, m, offset, scale, alpha, alpha2, obs, target, w_b, u_max) = key
    chain = make_env(conf).chain
    nq = chain.n
    q = sp.symbols("q0:%d" % nq, real=True)
    v = sp.symbols("v0:%d" % (n - nq), real=True)
    u = sp.symbols("u0:%d" % m, real=True)
    w = sp.symbols("w0:7", real=True)
    P = sp.symbols("p0:3", real=True)
    ur5 = name == "ur5"
    nc = 3 if ur5 else 2
    d = [P[c] - target[c] for c in range(nc)]
    if ur5:
        ell = [sp.log(sp.exp(alpha * -(sum((P[c] - obs[3 * kk + c]) ** 2 / (obs[9 + 3 * kk + c] / 2) ** 2
                                           for c in range(3)) - 1.0)) + 1) / alpha for kk in range(3)]
    else:
        ell = [sp.log(sp.exp(alpha * -((P[0] - obs[2 * kk]) ** 2 / (obs[6 + 2 * kk] / 2) ** 2
                                       + (P[1] - obs[2 * kk + 1]) ** 2 / (obs[7 + 2 * kk] / 2) ** 2 - 1.0)) + 1) / alpha
               for kk in range(3)]
    pos_cost = w[0] * sum(dk ** 2 for dk in d) - w[1] * _peak_sym(alpha2, d) + sum(w[3 + kk] * ell[kk] for kk in range(3))
    v_cost = sum(vi ** 2 for vi in v)
    u_cost = _u_cost_sym(u, m, w_b, u_max)
    r_pos = -scale * pos_cost
    Pm = sp.Matrix(P)
    lam = lambda args, e: sp.lambdify(args, e, "numpy", cse=True)  # noqa: E731
    p_sym = _fk_sym(chain, q)
    Qm = sp.Matrix(q)
    fk = lam((q,), p_sym)
    J = lam((q,), p_sym.jacobian(Qm))
    Hc = [lam((q,), sp.hessian(p_sym[c], Qm)) for c in range(3)]
    gP = lam((P, w), sp.Matrix([r_pos]).jacobian(Pm).T)
    HP = lam((P, w), sp.hessian(r_pos, Pm))
    r_all = lam((P, v, u, w), -scale * (pos_cost + w[2] * v_cost + w[6] * u_cost - offset))
    U = sp.Matrix(u)
    r_u = -scale * w[6] * u_cost
    lu = lam((u, w), sp.Matrix([r_u]).jacobian(U).T)
    luu = lam((u, w), sp.hessian(r_u, U))

    def lx_lxx(x, wv):
        x = np.asarray(x, dtype=np.float64)
        qq, vv = x[:nq], x[nq:n]
        Pv = np.reshape(fk(qq), 3)
        Jv = np.asarray(J(qq), dtype=np.float64).reshape(3, nq)
        g = np.reshape(gP(Pv, wv), 3)
        H = np.asarray(HP(Pv, wv), dtype=np.float64)
        lx = np.zeros(n)
        lxx = np.zeros((n, n))
        lx[:nq] = Jv.T @ g
        lxx[:nq, :nq] = Jv.T @ H @ Jv + sum(g[c] * np.asarray(Hc[c](qq), dtype=np.float64) for c in range(3))
        lx[nq:] = -scale * wv[2] * 2.0 * vv
        lxx[nq:, nq:] = -scale * wv[2] * 2.0 * np.identity(n - nq)
        return lx, lxx

    out = dict(r=lambda x, uu, wv: r_all(np.reshape(fk(np.asarray(x)[:nq]), 3), np.asarray(x)[nq:n], uu, wv),
               lx=lambda x, wv: lx_lxx(x, wv)[0], lxx=lambda x, wv: lx_lxx(x, wv)[1],
               lu=lu, luu=luu, lxu=lambda x, uu, wv: np.zeros((n, m)))
    _CHAIN_CACHE[key] = out
    return out


def cost_functions(conf):
    name = system_of(conf)
    if name not in SUPPORTED:
        raise NotImplementedError("DDP backward pass oracle: %s" % name)
    n, m = _n_m(conf)
    if name == "car_park":
        return _car_park_functions((n, m, float(conf.cost_funct_param[0]), float(conf.cost_funct_param[1]),
                                    float(conf.soft_max_param[1]), tuple(float(v) for v in conf.obs_param),
                                    tuple(float(v) for v in conf.TARGET_STATE), float(conf.w_b),
                                    tuple(float(v) for v in conf.u_max), float(conf.L_delta), float(conf.k_db),
                                    tuple((float(a), float(b)) for a, b in np.asarray(conf.check_points_BF))))
    if name in CHAINS:
        return _chain_functions(conf, (name, n, m, float(conf.cost_funct_param[0]), float(conf.cost_funct_param[1]),
                                       float(conf.soft_max_param[0]), float(conf.soft_max_param[1]),
                                       tuple(float(v) for v in conf.obs_param),
                                       tuple(float(v) for v in conf.TARGET_STATE), float(conf.w_b),
                                       tuple(float(v) for v in conf.u_max)))
    nq = int(conf.nq) if name == "double_integrator" else n
    key = (n, m, float(conf.cost_funct_param[0]), float(conf.cost_funct_param[1]), float(conf.soft_max_param[0]),
           float(conf.soft_max_param[1]), tuple(float(v) for v in conf.obs_param),
           tuple(float(v) for v in conf.TARGET_STATE), float(conf.w_b), tuple(float(v) for v in conf.u_max), nq,
           name == "double_integrator")
    return _cost_functions(name, key)


def augmented_derivative(conf, state, action):
    """Discrete-time (Fx, Fu) without the time row/column: environment.py:111-132 (DI chain),
    :221-233 (SI), :420-435 (Car)."""
    n, m = _n_m(conf)
    dt = conf.dt
    name = system_of(conf)
    if name == "single_integrator":
        Fx = np.array([[1.0, 0.0], [0.0, 1.0]])
        Fu = np.zeros((n, m))
        Fu[0, 0] = dt
        Fu[1, 1] = dt
        return Fx, Fu
    if name == "car":
        s = state
        Fx = np.array([[1, 0, -dt * s[3] * np.sin(s[2]) - dt ** 2 * s[4] * np.sin(s[2]) / 2, dt * np.cos(s[2]),
                        dt ** 2 * np.cos(s[2]) / 2],
                       [0, 1, dt * s[3] * np.cos(s[2]) + dt ** 2 * s[4] * np.cos(s[2]) / 2, dt * np.sin(s[2]),
                        dt ** 2 * np.sin(s[2]) / 2],
                       [0, 0, 1, 0, 0], [0, 0, 0, 1, dt], [0, 0, 0, 0, 1]], dtype=np.float64)
        Fu = np.zeros((n, m))
        Fu[2, 0] = dt
        Fu[4, 1] = dt
        return Fx, Fu
    if name == "car_park":                                                  # environment.py:567-582
        s = state
        L = conf.L_delta
        Fx = np.array([[1, 0, -dt * s[3] * np.sin(s[2]), dt * np.cos(s[2]), 0],
                       [0, 1, dt * s[3] * np.cos(s[2]), dt * np.sin(s[2]), 0],
                       [0, 0, 1, dt * np.tan(s[4]) / L, dt * s[3] / np.cos(s[4]) ** 2 / L],
                       [0, 0, 0, 1, 0], [0, 0, 0, 0, 1]], dtype=np.float64)
        Fu = np.zeros((n, m))
        Fu[3, 0] = dt
        Fu[4, 1] = dt / conf.tau_delta
        return Fx, Fu
    if name in CHAINS:
        return _chain_augmented_derivative(conf, state, action)
    # double integrator: prismatic chain, M(q) = I (constant), nle = 0 -> ddq_dq = ddq_dv = 0
    nq, nv = conf.nq, conf.nv
    from .env import make_env
    Minv = np.linalg.inv(make_env(conf).chain.mass_matrix(np.asarray(state[:nq], dtype=np.float64)))
    Fx = np.zeros((n, n))
    Fx[:nv, nv:n] = np.identity(nv)
    Fx = np.identity(n) + dt * Fx
    Fu = np.zeros((n, m))
    Fu[nv:n, :] = Minv
    Fu *= dt
    return Fx, Fu


def _chain_augmented_derivative(conf, state, action, h=1e-20):
    """computeABADerivatives (environment.py:111-132) by complex-step differentiation of the
    oracle's forward dynamics ddq = M(q)^-1 (u - nle(q, v)) (oracle/dynamics.py): column k is
    Im(ddq(x + i h e_k)) / h, exact to rounding for these analytic functions (no subtraction)."""
    from .env import make_env
    chain = make_env(conf).chain
    nq = chain.n
    n, m = _n_m(conf)
    dt = conf.dt
    q0 = np.asarray(state[:nq], dtype=np.float64)
    v0 = np.asarray(state[nq:n], dtype=np.float64)
    u = np.asarray(action, dtype=np.float64)

    def ddq(q, v):
        return np.linalg.solve(chain.mass_matrix(q), u - chain.nle(q, v))

    Fx = np.zeros((n, n))
    Fx[:nq, nq:n] = np.identity(nq)
    for k in range(nq):
        e = np.zeros(nq, dtype=complex)
        e[k] = 1j * h
        Fx[nq:n, k] = np.imag(ddq(q0 + e, v0.astype(complex))) / h
        Fx[nq:n, nq + k] = np.imag(ddq(q0.astype(complex), v0 + e)) / h
    Fx = np.identity(n) + dt * Fx
    Fu = np.zeros((n, m))
    Fu[nq:n, :] = np.linalg.inv(chain.mass_matrix(q0))
    Fu *= dt
    return Fx, Fu


def backward_pass(conf, states, controls, mu=1e-9, inverse="pinv"):
    """TO.py:119-202. states [T, >= n] (s_0..s_{T-1}; a time column, if present, is ignored),
    controls [T-1, m]. Returns V_x [T, n+1] (the last, time, column stays 0).
    inverse="inv" evaluates Qbar_uu^-1 with np.linalg.inv instead of the reference's pinv: the two
    agree to rounding when Qbar_uu is well conditioned, and their difference measures how strongly
    the recursion amplifies rounding for that trajectory (Q_uu passes near zero where the reward's
    curvature in u, -2 scale w6, is cancelled by dt^2 V_xx)."""
    n, m = _n_m(conf)
    T = states.shape[0]
    X_bar = np.asarray(states, dtype=np.float64)[:, :n]
    U_bar = np.asarray(controls, dtype=np.float64)[:T - 1, :m]
    f = cost_functions(conf)
    w_run = [float(v) for v in conf.cost_weights_running[:7]]
    w_term = [float(v) for v in conf.cost_weights_terminal[:7]]
    V_x = np.zeros((T, n + 1))
    V_xx = np.zeros((T, n, n))
    V_x[T - 1, :-1] = np.reshape(f["lx"](X_bar[-1], w_term), n)                           # :166-168
    V_xx[T - 1] = f["lxx"](X_bar[-1], w_term)
    for i in range(T - 2, -1, -1):
        A, B = augmented_derivative(conf, X_bar[i], U_bar[i])
        l_x = np.reshape(f["lx"](X_bar[i], w_run), n)
        l_xx = np.asarray(f["lxx"](X_bar[i], w_run), dtype=np.float64)
        l_u = np.reshape(f["lu"](U_bar[i], w_run), m)
        l_uu = np.asarray(f["luu"](U_bar[i], w_run), dtype=np.float64)
        l_xu = np.asarray(f["lxu"](X_bar[i], U_bar[i], w_run), dtype=np.float64).reshape(n, m)
        Q_x = l_x + A.T @ V_x[i + 1, :-1]                                                  # :182-186
        Q_u = l_u + B.T @ V_x[i + 1, :-1]
        Q_xx = l_xx + A.T @ V_xx[i + 1] @ A
        Q_uu = l_uu + B.T @ V_xx[i + 1] @ B
        Q_xu = l_xu + A.T @ V_xx[i + 1] @ B
        Qbar_uu = Q_uu + mu * np.identity(m)                                               # :188-189
        Qbar_uu_pinv = np.linalg.pinv(Qbar_uu) if inverse == "pinv" else np.linalg.inv(Qbar_uu)
        V_x[i, :-1] = Q_x - Q_xu @ Qbar_uu_pinv @ Q_u                                      # :192-193
        V_xx[i] = Q_xx - Q_xu @ Qbar_uu_pinv @ Q_xu.T
    return V_x
