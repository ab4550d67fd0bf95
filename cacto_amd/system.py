"""System handle: packs a conf_*.py module into `cacto_sys_params` (include/cacto_hip.h) and owns
the `cacto_sys` handle every HIP entry point takes. Also the tensor-contract helpers of the
ctypes boundary (device, dtype, contiguity, shape checks)."""
import ctypes as C

import numpy as np
import torch

from . import _lib as L

DEVICE = "cuda"


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("cacto_amd needs an MI355X (HIP device); none is visible — there is no CPU path")


def dptr(t, dtype=None, shape=None, name="tensor"):
    """Device pointer of a contiguous CUDA tensor after checking the contract."""
    if t is None:
        return None
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError("%s must be a CUDA (HIP) tensor" % name)
    if dtype is not None and t.dtype != dtype:
        raise TypeError("%s must be %s, got %s" % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError("%s must have shape %s, got %s" % (name, tuple(shape), tuple(t.shape)))
    return C.c_void_p(t.data_ptr())


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _fill(arr, values):
    for i, v in enumerate(values):
        arr[i] = float(v)


_SHARED = {}


def shared_system(conf):
    """The System of a conf module: the reference constructs `Environment(conf)`,
    `ReplayBuffer(conf)`, `NN(env, conf)` ... from the same conf (main.py:145-150), and they all
    address one device copy of it (one `cacto_sys` handle). The cache holds the System weakly (its
    handle is destroyed once no Env / buffer / net uses it) and keys it by the conf's packed
    numeric content as well as its identity: a conf module changed after a System was made from it
    (dt, weights, norms, ...) gets a new System instead of silently reusing the stale one."""
    import weakref
    key = id(conf)
    fp = fingerprint(conf)
    hit = _SHARED.get(key)
    sysobj = hit[1]() if hit is not None and hit[0] is conf and hit[2] == fp else None
    if sysobj is None:
        sysobj = System(conf)
        _SHARED[key] = (conf, weakref.ref(sysobj), fp)
    return sysobj


def fingerprint(conf):
    """The bytes System(conf) hands the device: the packed parameters and the joint table."""
    p, table = pack_params(conf)
    return bytes(p) + (table.tobytes() if table is not None else b"")


def pack_params(conf):
    """conf module -> (cacto_sys_params, joint table or None), host only."""
    p = L.SysParams()
    sid = conf.system_id
    robot = getattr(conf, "robot", None)
    if sid == "single_integrator":
        p.dyn_kind, p.reward_kind = L.CACTO_DYN_SINGLE_INTEGRATOR, L.CACTO_REW_PLANAR
    elif sid == "car":
        p.dyn_kind, p.reward_kind = L.CACTO_DYN_CAR, L.CACTO_REW_PLANAR
    elif sid == "car_park":
        p.dyn_kind, p.reward_kind = L.CACTO_DYN_CAR_PARK, L.CACTO_REW_CAR_PARK
        p.L_delta, p.tau_delta, p.k_db = float(conf.L_delta), float(conf.tau_delta), float(conf.k_db)
        cp = np.asarray(conf.check_points_BF, dtype=np.float64)
        p.n_check = cp.shape[0]
        _fill(p.check_points, cp.reshape(-1))
    elif robot is not None and sid in ("double_integrator", "manipulator", "ur5"):
        p.dyn_kind = L.CACTO_DYN_CHAIN
        p.reward_kind = {"manipulator": L.CACTO_REW_MANIPULATOR, "ur5": L.CACTO_REW_UR5}.get(sid, L.CACTO_REW_PLANAR)
    else:
        raise NotImplementedError("system %r is not in this build's hot path" % sid)
    p.nb_state, p.nb_action = conf.nb_state, conf.nb_action
    p.nq = conf.nq or 0
    p.nv = conf.nv or 0
    p.normalize = int(conf.NORMALIZE_INPUTS)
    p.n_weights = len(conf.cost_weights_running)
    p.dt = conf.dt
    _fill(p.state_norm, conf.state_norm_arr)
    _fill(p.u_max, conf.u_max)
    p.w_b = conf.w_b
    p.offset, p.scale = float(conf.cost_funct_param[0]), float(conf.cost_funct_param[1])
    p.alpha, p.alpha2 = float(conf.soft_max_param[0]), float(conf.soft_max_param[1])
    _fill(p.obs, conf.obs_param)
    _fill(p.target, conf.TARGET_STATE)
    _fill(p.w_running, conf.cost_weights_running)
    _fill(p.w_terminal, conf.cost_weights_terminal)
    table = None
    if robot is not None:
        p.n_joints = robot.nq
        p.ee_parent = robot.ee_parent
        _fill(p.ee_R, np.asarray(robot.ee_R).reshape(-1))
        _fill(p.ee_p, robot.ee_p)
        _fill(p.gravity, robot.gravity)
        table = np.ascontiguousarray(robot.table(), dtype=np.float64)
    return p, table


class System:
    """Numeric content of a conf module + the device copy the kernels read."""

    def __init__(self, conf):
        require_gpu()
        self.conf = conf
        p, table = pack_params(conf)
        self.params = p
        self._table = table
        h = C.c_void_p()
        L.lib().call("cacto_sys_create", C.byref(p),
                     table.ctypes.data_as(C.c_void_p) if table is not None else None, C.byref(h))
        self.handle = h
        self.ns, self.na = conf.nb_state, conf.nb_action

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                L.lib().raw("cacto_sys_destroy")(h)
            except Exception:
                pass
            self.handle = None

    def param_count(self, net):
        return int(L.lib().raw("cacto_mlp_param_count")(self.handle, net))

    def set_critic_type(self, critic_type):
        """RL.py:65-76 critic_type of this system's critics: 'sine' or 'sine-elu'. The activations are
        a property of the handle, read by every critic kernel: once a critic net exists on it (the
        learner's critic and target), a different type is refused instead of silently changing
        those nets' activations."""
        cur = getattr(self, "critic_type", "sine")
        live = len(getattr(self, "critic_nets", None) or ())
        if critic_type != cur and live > 0:
            raise ValueError("critic_type %r requested on a system whose %d critic net(s) are %r: the activations "
                             "belong to the system handle (make the other critic type from its own conf / system)"
                             % (critic_type, live, cur))
        L.lib().call("cacto_sys_set_critic_type", self.handle, {"sine": 0, "sine-elu": 1}[critic_type])
        self.critic_type = critic_type

    def netbuf_floats(self, net):
        return int(L.lib().raw("cacto_mlp_netbuf_floats")(self.handle, net))

    def workspace_bytes(self, B):
        return int(L.lib().raw("cacto_workspace_bytes")(self.handle, int(B)))
