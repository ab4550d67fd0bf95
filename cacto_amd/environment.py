"""Environment plugins with the reference surface (environment.py:10-816), backed by the HIP
kernels. Every numeric method runs on the GPU through libcacto_hip.so; `reset` keeps the
reference's host-side CPython `random` draws (bit-exact initial states, environment.py:46-55).

Batch methods take/return torch CUDA tensors (float32, as the reference's TF tensors);
per-sample methods take/return numpy float64 arrays (as the reference's numpy arrays).
"""
import random

import numpy as np
import torch

from .system import DEVICE, dptr, shared_system, stream
from . import _lib as L


def _as_dev(x, dtype):
    if isinstance(x, torch.Tensor):
        return x.to(device=DEVICE, dtype=dtype).contiguous()
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=DEVICE).contiguous()


class Env:
    """Base class: environment.py:10-163."""

    def __init__(self, conf):
        self.conf = conf
        self.sys = shared_system(conf)
        self.nq, self.nv = conf.nq, conf.nv
        self.nx, self.nu = conf.nx, conf.na
        self.offset = conf.cost_funct_param[0]
        self.scale = conf.cost_funct_param[1]
        self.ns, self.na = conf.nb_state, conf.nb_action

    # ---- environment.py:46-55 (host CPython random, as the reference) ----
    def reset(self):
        c = self.conf
        state = np.zeros(c.nb_state)
        time = random.uniform(c.x_init_min[-1], c.x_init_max[-1])
        for i in range(c.nb_state - 1):
            state[i] = random.uniform(c.x_init_min[i], c.x_init_max[i])
        state[-1] = c.dt * round(time / c.dt)
        return state

    # ---- batched GPU primitives ----
    def step_batch(self, S, A, W=None):
        """Env.step over rows in float64: returns (S_next [B,ns], R [B], EE(S_next) [B,3])."""
        S = _as_dev(S, torch.float64)
        A = _as_dev(A, torch.float64)
        B = S.shape[0]
        Sn = torch.empty_like(S)
        R = torch.empty(B, dtype=torch.float64, device=DEVICE)
        EE = torch.empty(B, 3, dtype=torch.float64, device=DEVICE)
        Wt = None if W is None else _as_dev(np.asarray(W, dtype=np.float64).reshape(-1), torch.float64)
        L.lib().call("cacto_env_step", self.sys.handle, dptr(S, torch.float64, (B, self.ns)),
                     dptr(A, torch.float64, (B, self.na)), dptr(Wt), dptr(Sn), dptr(R), dptr(EE), B, stream())
        return Sn, R, EE

    def batch_f32(self, S, A, term=None, W=None, want=("S_next", "Fu", "R", "dR_dA")):
        """compute_actor_grad's env calls (float32 tensors, float64 math)."""
        S = _as_dev(S, torch.float32)
        A = _as_dev(A, torch.float32)
        B = S.shape[0]
        out = {}
        if "S_next" in want:
            out["S_next"] = torch.empty(B, self.ns, dtype=torch.float32, device=DEVICE)
        if "Fu" in want:
            out["Fu"] = torch.empty(B, self.ns, self.na, dtype=torch.float32, device=DEVICE)
        if "R" in want:
            out["R"] = torch.empty(B, dtype=torch.float32, device=DEVICE)
        if "dR_dA" in want:
            out["dR_dA"] = torch.empty(B, self.na, dtype=torch.float32, device=DEVICE)
        t = None if term is None else _as_dev(np.asarray(term, dtype=np.float64).reshape(-1), torch.float64)
        Wt = None if W is None else _as_dev(np.asarray(W, dtype=np.float64), torch.float64)
        L.lib().call("cacto_env_step_batch", self.sys.handle, dptr(S, torch.float32, (B, self.ns)),
                     dptr(A, torch.float32, (B, self.na)), dptr(t), dptr(Wt), dptr(out.get("S_next")),
                     dptr(out.get("Fu")), dptr(out.get("R")), dptr(out.get("dR_dA")), B, stream())
        return out

    # ---- reference surface ----
    def step(self, weights, state, action):
        """environment.py:70-78."""
        Sn, R, _ = self.step_batch(np.asarray(state, dtype=np.float64)[None],
                                   np.asarray(action, dtype=np.float64)[None], weights)
        return Sn[0].cpu().numpy(), float(R[0].item())

    def simulate(self, state, action):
        """environment.py:80-91 (float64 semantics)."""
        return self.step(self.conf.cost_weights_running, state, action)[0]

    def derivative(self, state, action):
        """environment.py:93-109, returned as float64 of the float32 kernel result."""
        Fu = self.batch_f32(np.asarray(state, dtype=np.float32)[None], np.asarray(action, dtype=np.float32)[None],
                            want=("Fu",))["Fu"]
        return Fu[0].double().cpu().numpy()

    def simulate_batch(self, state, action):
        """environment.py:134-138: float32 tensor [B, ns]."""
        return self.batch_f32(state, action, want=("S_next",))["S_next"]

    def derivative_batch(self, state, action):
        """environment.py:140-144: float32 tensor [B, ns, na]."""
        return self.batch_f32(state, action, want=("Fu",))["Fu"]

    def get_end_effector_position(self, state, recompute=True):
        """environment.py:146-156."""
        S = _as_dev(np.asarray(state, dtype=np.float64)[None], torch.float64)
        EE = torch.empty(1, 3, dtype=torch.float64, device=DEVICE)
        L.lib().call("cacto_env_ee", self.sys.handle, dptr(S), dptr(EE), 1, stream())
        return EE[0].cpu().numpy()

    def augmented_derivative(self, state, action):
        """environment.py:111-132 (SI :221-233, Car :420-435, CarPark :567-582): discrete-time
        (Fx [nx, nx], Fu [nx, na]) float64, as TO.backward_pass consumes them (TO.py:181)."""
        Fx, Fu = self.augmented_derivative_batch(np.asarray(state, dtype=np.float64)[None],
                                                 np.asarray(action, dtype=np.float64)[None])
        return Fx[0].cpu().numpy(), Fu[0].cpu().numpy()

    def augmented_derivative_batch(self, S, A):
        """augmented_derivative over rows on the device: (Fx [B, nx, nx], Fu [B, nx, na]) float64."""
        S = _as_dev(S, torch.float64)
        A = _as_dev(A, torch.float64)
        B, nx = S.shape[0], self.ns - 1
        Fx = torch.empty(B, nx, nx, dtype=torch.float64, device=DEVICE)
        Fu = torch.empty(B, nx, self.na, dtype=torch.float64, device=DEVICE)
        L.lib().call("cacto_env_jacobians", self.sys.handle, dptr(S, torch.float64, (B, self.ns)),
                     dptr(A, torch.float64, (B, self.na)), B, dptr(Fx), dptr(Fu), stream())
        return Fx, Fu

    def bound_control_cost(self, action):
        """environment.py:158-163: sum_i a_i^2 + w_b (a_i / u_max_i)^10 (float64)."""
        return float(self.bound_control_cost_batch(np.asarray(action, dtype=np.float64)[None])[0].item())

    def bound_control_cost_batch(self, A):
        A = _as_dev(A, torch.float64)
        B = A.shape[0]
        out = torch.empty(B, dtype=torch.float64, device=DEVICE)
        L.lib().call("cacto_env_bound_control_cost", self.sys.handle, dptr(A, torch.float64, (B, self.na)), dptr(out),
                     B, stream())
        return out

    def reward(self, weights, state, action=None):
        """Per-system reward (environment.py:252-275, :329-351, :695-723); action=None -> u_cost 0."""
        a = np.zeros(self.na) if action is None else action
        return self.step(weights, state, a)[1]

    def reward_batch(self, weights, state, action):
        """environment.py:277-286 etc.: float32 tensor [B, 1]."""
        return self.batch_f32(state, action, W=weights, want=("R",))["R"].reshape(-1, 1)

    def dr_da_batch(self, weights, state, action):
        """The tape gradient of reward_batch w.r.t. the action (NeuralNetwork.py:199-204)."""
        return self.batch_f32(state, action, W=weights, want=("dR_dA",))["dR_dA"]


class SingleIntegrator(Env):
    """environment.py:165-286."""


class DoubleIntegrator(Env):
    """environment.py:288-362."""


class Car(Env):
    """environment.py:364-491 (kinematic car: x, y, theta, v, a)."""


class CarPark(Car):
    """environment.py:493-652 (kinematic bicycle, smooth-box obstacles over body check points)."""


class Manipulator(Env):
    """environment.py:654-734."""


class UR5(Env):
    """environment.py:736-816 (6-DoF arm, 3-D ellipsoids)."""


ENV_CLASSES = {
    "single_integrator": SingleIntegrator,
    "double_integrator": DoubleIntegrator,
    "car": Car,
    "car_park": CarPark,
    "manipulator": Manipulator,
    "ur5": UR5,
}


def make_env(conf):
    return ENV_CLASSES[conf.system_id](conf)
