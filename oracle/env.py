"""Oracle: CACTO environments (test infrastructure only — see oracle/__init__).

Restates `environment.py` (reference) per sample, with the reference's dtype semantics under
numpy 1.24 (requirements.txt:205): inputs may be float32 (batch paths: `state_batch.numpy()`,
NeuralNetwork.py:188, :201) or float64 (rollout paths: RL.py:223-231, plot_utils.py:262-267);
scalar arithmetic promotes to float64 (numpy-1.x scalar promotion), array*python-float keeps the
array dtype. numpy >= 2 changed scalar promotion (NEP 50), so every such promotion is explicit here.
"""
import math

import numpy as np

from .dynamics import Chain

F32, F64 = np.float32, np.float64


class Env:
    """Base class: environment.py:10-163."""

    def __init__(self, conf):
        self.conf = conf
        self.nb_state = conf.nb_state
        self.nb_action = conf.nb_action
        self.nx = conf.nx
        self.nu = conf.na
        self.offset = float(conf.cost_funct_param[0])    # environment.py:43
        self.scale = float(conf.cost_funct_param[1])     # environment.py:44
        self.alpha = float(conf.soft_max_param[0])
        self.alpha2 = float(conf.soft_max_param[1])
        self.obs = [float(v) for v in conf.obs_param]
        self.target = [float(v) for v in conf.TARGET_STATE]
        robot = getattr(conf, 'robot', None)
        self.chain = Chain.from_model(robot) if robot is not None else None
        self.nq = conf.nq
        self.nv = conf.nv

    # ---- reset: environment.py:46-55 ----
    def reset(self, rng):
        """`rng` is a `random.Random` (the reference uses the module-level `random`)."""
        c = self.conf
        state = np.zeros(c.nb_state)
        time = rng.uniform(c.x_init_min[-1], c.x_init_max[-1])
        for i in range(c.nb_state - 1):
            state[i] = rng.uniform(c.x_init_min[i], c.x_init_max[i])
        state[-1] = c.dt * round(time / c.dt)
        return state

    # ---- robot simulate: environment.py:80-91 -> robot_utils.py:415-432, :348-410 ----
    def simulate(self, state, action):
        c = self.conf
        state = np.asarray(state)
        nq, nx = self.nq, self.nx
        q = np.copy(state[:nq])
        v = np.copy(state[nq:nx])
        qd, vd = q.astype(F64), v.astype(F64)
        M = self.chain.mass_matrix(qd)
        h = self.chain.nle(qd, vd)
        u = np.asarray(action).astype(F64)                         # u - tau_c (tau_c = 0, f64)
        dv = np.linalg.solve(M, u - h)                             # robot_utils.py:401
        q_new = qd + (v * v.dtype.type(c.dt)).astype(F64)          # pin.integrate(q, v*dt), :403
        v_new = (vd + dv * c.dt).astype(v.dtype)                   # self.v += self.dv*dt, :405
        out = np.zeros(nx + 1)
        out[:nq] = q_new
        out[nq:nx] = v_new
        out[-1] = F64(state[-1]) + c.dt                            # environment.py:89
        return out

    # ---- derivative: environment.py:93-109 ----
    def derivative(self, state, action):
        c = self.conf
        q = np.asarray(state[:self.nq]).astype(F64)
        Minv = np.linalg.inv(self.chain.mass_matrix(q))
        Fu = np.zeros((self.nx + 1, self.nu))
        Fu[self.nv:-1, :] = Minv
        Fu[:self.nx, :] *= c.dt
        if c.NORMALIZE_INPUTS:
            Fu[:-1] *= (1 / c.state_norm_arr[:-1, None])
        return Fu

    # ---- batch wrappers: environment.py:134-144 (outputs cast to float32) ----
    def simulate_batch(self, S, A):
        return np.array([self.simulate(s, a) for s, a in zip(S, A)]).astype(F32)

    def derivative_batch(self, S, A):
        return np.array([self.derivative(s, a) for s, a in zip(S, A)]).astype(F32)

    def get_end_effector_position(self, state):
        q = np.asarray(state[:self.nq]).astype(F64)
        return self.chain.frame_position(q)

    # ---- bound_control_cost: environment.py:158-163 ----
    def bound_control_cost(self, action):
        c = self.conf
        u_cost = 0
        for i in range(c.nb_action):
            a = F64(action[i])
            u_cost += a * a + c.w_b * (a / c.u_max[i]) ** 10
        return u_cost

    # ---- step: environment.py:70-78 ----
    def step(self, weights, state, action):
        return self.simulate(state, action), self.reward(weights, state, action)

    # ---- shared reward pieces (the ellipse / peak formulas are identical across systems) ----
    def _ell(self, x, y, xc, yc, A, B):
        # log(exp(alpha * -(e - 1)) + 1) / alpha, e = ((x-xc)/(A/2))^2 + ((y-yc)/(B/2))^2
        e = ((x - xc) ** 2) / ((A / 2) ** 2) + ((y - yc) ** 2) / ((B / 2) ** 2)
        return math.log(math.exp(self.alpha * -(e - 1.0)) + 1) / self.alpha

    def _peak(self, *d):
        # sqrt(dx²+.1) - sqrt(.1) - .1 + sqrt(dy²+.1) - sqrt(.1) - .1, evaluated left to right
        s = None
        for dk in d:
            r = math.sqrt(dk ** 2 + 0.1)
            s = r if s is None else s + r
            s = s - math.sqrt(0.1)
            s = s - 0.1
        return math.log(math.exp(self.alpha2 * -s) + 1) / self.alpha2

    def _planar_reward(self, weights, state, action, vel_cost):
        """Reward of SI/DI/Car/Manipulator: environment.py:252-275 / :329-351 / :695-723."""
        p = self.get_end_effector_position(state)
        x, y = F64(p[0]), F64(p[1])
        o = self.obs
        ell1 = self._ell(x, y, o[0], o[1], o[6], o[7])
        ell2 = self._ell(x, y, o[2], o[3], o[8], o[9])
        ell3 = self._ell(x, y, o[4], o[5], o[10], o[11])
        peak = self._peak(x - self.target[0], y - self.target[1])
        u_cost = self.bound_control_cost(action) if action is not None else 0
        dist = (x - self.target[0]) ** 2 + (y - self.target[1]) ** 2
        w = [F64(v) for v in weights]
        r = - w[0] * dist + w[1] * peak
        if vel_cost is not None:
            r = r - w[2] * vel_cost
        r = r - w[3] * ell1 - w[4] * ell2 - w[5] * ell3 - w[6] * u_cost + self.offset
        return self.scale * r

    def reward(self, weights, state, action=None):
        return self._planar_reward(weights, state, action, None)

    # ---- reward_batch: environment.py:277-286 (float32 TF part for u_cost) ----
    def reward_batch(self, W, S, A):
        c = self.conf
        W = np.asarray(W, dtype=F64)
        partial = np.array([self.reward(w, s) for w, s in zip(W, S)]).astype(F32)
        A = np.asarray(A, dtype=F32)
        umax = c.u_max.astype(F32)
        u_cost = np.sum(A * A + F32(c.w_b) * (A / umax) ** F32(10), axis=1, dtype=F32)
        r = F32(self.scale) * ((-W[:, 6]).astype(F32) * u_cost) + partial
        return r.reshape(-1, 1).astype(F32)

    def dr_da(self, W, A):
        """d reward_batch / d action (only the TF u_cost term depends on the action)."""
        c = self.conf
        W = np.asarray(W, dtype=F64)
        A = np.asarray(A, dtype=F64)
        g = -W[:, 6:7] * self.scale
        return g * (2 * A + c.w_b * 10 * (A / c.u_max) ** 9 / c.u_max)


class SingleIntegrator(Env):
    """environment.py:165-286."""

    def simulate(self, state, action):
        dt = self.conf.dt
        out = np.zeros(self.nx + 1)
        out[0] = F64(state[0]) + dt * F64(action[0])
        out[1] = F64(state[1]) + dt * F64(action[1])
        out[2] = F64(state[2]) + dt
        return out

    def derivative(self, state, action):
        c = self.conf
        Fu = np.zeros((self.nx + 1, self.nu))
        Fu[0, 0] = c.dt
        Fu[1, 1] = c.dt
        if c.NORMALIZE_INPUTS:
            Fu[:-1] *= (1 / c.state_norm_arr[:-1, None])
        return Fu

    def get_end_effector_position(self, state):
        p = np.zeros(3)
        p[:2] = np.asarray(state[:2]).astype(F64)
        return p


class DoubleIntegrator(Env):
    """environment.py:288-362 (dynamics through the Pinocchio chain: M = I, nle = 0)."""


class Manipulator(Env):
    """environment.py:654-734."""

    def reward(self, weights, state, action=None):
        vel = None
        if F64(weights[2]) != 0:
            v = np.asarray(state[self.nq:self.nx])
            if v.dtype == F32:   # numpy f32 dot (reference state_batch.numpy() is float32)
                acc = F32(0)
                for k in range(len(v)):
                    acc = F32(acc + v[k] * v[k])
                vel = F64(acc)
            else:
                vel = F64(v.dot(v))
        else:
            vel = 0
        return self._planar_reward(weights, state, action, vel)


class Car(Env):
    """environment.py:364-491. Car.simulate (:437-448) uses tf.cos/tf.sin: with float32 inputs the
    numpy-1.x scalar dt*v is float64, TF casts it to float32 against the float32 tf.cos, so x' and y'
    are float32 arithmetic; with float64 inputs everything is float64."""

    def simulate(self, state, action):
        dt = self.conf.dt
        s = np.asarray(state)
        out = np.zeros(self.nx + 1)
        if s.dtype == F32:
            c, sn = F32(math.cos(F64(s[2]))), F32(math.sin(F64(s[2])))   # tf.cos(float32 scalar)
            x1 = F32(s[0]) + F32(F64(dt) * F64(s[3])) * c
            out[0] = F64(x1 + F32(F32(F64(dt) ** 2 * F64(s[4])) * c) / F32(2))
            y1 = F32(s[1]) + F32(F64(dt) * F64(s[3])) * sn
            out[1] = F64(y1 + F32(F32(F64(dt) ** 2 * F64(s[4])) * sn) / F32(2))
        else:
            c, sn = math.cos(F64(s[2])), math.sin(F64(s[2]))
            out[0] = F64(s[0]) + dt * F64(s[3]) * c + dt ** 2 * F64(s[4]) * c / 2
            out[1] = F64(s[1]) + dt * F64(s[3]) * sn + dt ** 2 * F64(s[4]) * sn / 2
        out[2] = F64(s[2]) + dt * F64(action[0])
        out[3] = F64(s[3]) + dt * F64(s[4])
        out[4] = F64(s[4]) + dt * F64(action[1])
        out[5] = F64(s[5]) + dt
        return out

    def derivative(self, state, action):
        c = self.conf
        Fu = np.zeros((self.nx + 1, self.nu))
        Fu[2, 0] = c.dt
        Fu[4, 1] = c.dt
        if c.NORMALIZE_INPUTS:
            Fu[:-1] *= (1 / c.state_norm_arr[:-1, None])
        return Fu

    def get_end_effector_position(self, state):
        p = np.zeros(3)
        p[:2] = np.asarray(state[:2]).astype(F64)
        return p


class CarPark(Car):
    """environment.py:493-652 (math.cos/sin/tan: float64 dynamics for any input dtype)."""

    def simulate(self, state, action):
        c = self.conf
        dt = c.dt
        s = [F64(v) for v in state]
        out = np.zeros(self.nx + 1)
        out[0] = s[0] + dt * s[3] * math.cos(s[2])
        out[1] = s[1] + dt * s[3] * math.sin(s[2])
        out[2] = s[2] + dt * s[3] * math.tan(s[4]) / c.L_delta
        out[3] = s[3] + dt * F64(action[0])
        out[4] = s[4] + dt * F64(action[1]) / c.tau_delta
        out[5] = s[5] + dt
        return out

    def derivative(self, state, action):
        c = self.conf
        Fu = np.zeros((self.nx + 1, self.nu))
        Fu[3, 0] = c.dt
        Fu[4, 1] = c.dt / c.tau_delta
        if c.NORMALIZE_INPUTS:
            Fu[:-1] *= (1 / c.state_norm_arr[:-1, None])
        return Fu

    def get_end_effector_position(self, state):
        th = F64(state[2])
        R = np.array([[math.cos(th), -math.sin(th)], [math.sin(th), math.cos(th)]])
        p = np.zeros(3)
        p[:2] = np.asarray(state[:2]).astype(F64) + R.dot(np.array([self.conf.L_delta / 2, 0]))
        return p

    def obs_cost_fun(self, x, y, x_step, y_step, Wx, Wy, fv=1):
        k = self.conf.k_db
        term1 = 4 + 4 * (y - y_step + Wy / 2) ** 2 * k ** 2
        term2 = 4 + 4 * (y - y_step - Wy / 2) ** 2 * k ** 2
        term3 = 4 + 4 * (x - x_step + Wx / 2) ** 2 * k ** 2
        term4 = 4 + 4 * (x - x_step - Wx / 2) ** 2 * k ** 2
        return ((term1) ** (-1 / 2) * fv * (-np.sqrt(term2) / 2 + (y - y_step - Wy / 2) * k) * (term3) ** (-1 / 2)
                * (term2) ** (-1 / 2) * (np.sqrt(term1) / 2 + (y - y_step + Wy / 2) * k) * (term4) ** (-1 / 2)
                * (np.sqrt(term3) / 2 + (x - x_step + Wx / 2) * k) * (-np.sqrt(term4) / 2 + (x - x_step - Wx / 2) * k))

    def reward(self, weights, state, action=None):
        c = self.conf
        p = self.get_end_effector_position(state)
        x, y = F64(p[0]), F64(p[1])
        th = state[2]   # float32 state -> np.cos/np.sin in float32
        R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
        wf = np.dot(R, c.check_points_BF.T).T + np.array([x, y])
        o = self.obs
        obs_cost = 0
        for k in range(3):
            obs_cost += np.sum(self.obs_cost_fun(wf[:, 0], wf[:, 1], o[2 * k], o[2 * k + 1], o[6 + 2 * k], o[7 + 2 * k]))
        peak = self._peak(x - self.target[0], y - self.target[1])
        u_cost = self.bound_control_cost(action) if action is not None else 0
        dist = (x - self.target[0]) ** 2 + (y - self.target[1]) ** 2
        w = [F64(v) for v in weights]
        v2 = state[3] ** 2   # float32 scalar square for a float32 state
        r = - w[0] * dist + w[1] * peak - w[2] * F64(v2) - w[3] * obs_cost - w[6] * u_cost + self.offset
        return self.scale * r


class UR5(Env):
    """environment.py:736-816."""

    def reward(self, weights, state, action=None):
        e = self.get_end_effector_position(state)
        x, y, z = F64(e[0]), F64(e[1]), F64(e[2])
        o = self.obs
        ells = []
        for k in range(3):
            xc, yc, zc = o[3 * k], o[3 * k + 1], o[3 * k + 2]
            A, B, C = o[9 + 3 * k], o[10 + 3 * k], o[11 + 3 * k]
            ex = ((x - xc) ** 2) / ((A / 2) ** 2) + ((y - yc) ** 2) / ((B / 2) ** 2) + ((z - zc) ** 2) / ((C / 2) ** 2)
            ells.append(math.log(math.exp(self.alpha * -(ex - 1.0)) + 1) / self.alpha)
        peak = self._peak(x - self.target[0], y - self.target[1], z - self.target[2])
        u_cost = F64(np.asarray(action, dtype=F64).dot(np.asarray(action, dtype=F64))) if action is not None else 0
        v = np.asarray(state[self.nq:self.nx])
        if v.dtype == F32:
            acc = F32(0)
            for k in range(len(v)):
                acc = F32(acc + v[k] * v[k])
            vel = F64(acc)
        else:
            vel = F64(v.dot(v))
        dist = (x - self.target[0]) ** 2 + (y - self.target[1]) ** 2 + (z - self.target[2]) ** 2
        w = [F64(v_) for v_ in weights]
        r = (- w[0] * dist + w[1] * peak - w[2] * vel - w[3] * ells[0] - w[4] * ells[1] - w[5] * ells[2]
             - w[6] * u_cost + self.offset)
        return self.scale * r


ENV_CLASSES = {
    'single_integrator': SingleIntegrator,
    'double_integrator': DoubleIntegrator,
    'car': Car,
    'car_park': CarPark,
    'manipulator': Manipulator,
    'ur5': UR5,
}


def make_env(conf):
    return ENV_CLASSES[conf.system_id](conf)
