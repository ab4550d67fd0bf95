"""ctypes binding of libcacto_hip.so (include/cacto_hip.h).

This is the thin boundary layer: structs mirror the C header, every call checks the return code
and raises with `cacto_last_error()`. There is no fallback: if the library is missing or fails to
load, importing anything that needs it raises (the product path is the HIP path only).
"""
import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CACTO_HIP_LIB", os.path.join(HERE, "libcacto_hip.so"))
HEADER = os.path.join(HERE, "..", "include", "cacto_hip.h")

CACTO_DYN_SINGLE_INTEGRATOR, CACTO_DYN_CHAIN, CACTO_DYN_CAR, CACTO_DYN_CAR_PARK = 0, 1, 2, 3
CACTO_REW_PLANAR, CACTO_REW_MANIPULATOR, CACTO_REW_UR5, CACTO_REW_CAR_PARK = 0, 1, 2, 3
CACTO_NET_ACTOR, CACTO_NET_CRITIC = 0, 1
MAX_STATE, MAX_ACTION, MAX_JOINTS, JOINT_COLS = 16, 8, 6, 27


class SysParams(C.Structure):
    _fields_ = [
        ("dyn_kind", C.c_int32), ("reward_kind", C.c_int32), ("nb_state", C.c_int32),
        ("nb_action", C.c_int32), ("nq", C.c_int32), ("nv", C.c_int32), ("normalize", C.c_int32),
        ("n_joints", C.c_int32), ("ee_parent", C.c_int32), ("n_check", C.c_int32),
        ("n_weights", C.c_int32), ("const_dyn", C.c_int32),
        ("dt", C.c_double), ("state_norm", C.c_double * MAX_STATE), ("u_max", C.c_double * MAX_ACTION),
        ("w_b", C.c_double), ("scale", C.c_double), ("offset", C.c_double), ("alpha", C.c_double),
        ("alpha2", C.c_double), ("obs", C.c_double * 18), ("target", C.c_double * 3),
        ("w_running", C.c_double * 8), ("w_terminal", C.c_double * 8), ("L_delta", C.c_double),
        ("tau_delta", C.c_double), ("k_db", C.c_double), ("check_points", C.c_double * 20),
        ("ee_R", C.c_double * 9), ("ee_p", C.c_double * 3), ("gravity", C.c_double * 3),
    ]


class Nets(C.Structure):
    _fields_ = [
        ("actor_d", C.c_void_p), ("actor_m_d", C.c_void_p), ("actor_v_d", C.c_void_p),
        ("critic_d", C.c_void_p), ("critic_m_d", C.c_void_p), ("critic_v_d", C.c_void_p),
        ("target_d", C.c_void_p), ("step_d", C.c_void_p),
    ]


class UpdateCfg(C.Structure):
    _fields_ = [
        ("w_S", C.c_double), ("tau", C.c_double), ("beta1", C.c_double), ("beta2", C.c_double),
        ("epsilon", C.c_double), ("critic_lr", C.c_double * 5), ("actor_lr", C.c_double * 5),
        ("lr_bounds", C.c_double * 4), ("MC", C.c_int32), ("B_global", C.c_int32),
        ("want_target_V", C.c_int32), ("pad", C.c_int32),
    ]


vp, i32, i64, dbl, flt, sz = C.c_void_p, C.c_int32, C.c_int64, C.c_double, C.c_float, C.c_size_t
_SIGS = {
    "cacto_last_error": (C.c_char_p, []),
    "cacto_abi_version": (C.c_int, []),
    "cacto_sys_create": (C.c_int, [C.POINTER(SysParams), vp, C.POINTER(vp)]),
    "cacto_sys_destroy": (C.c_int, [vp]),
    "cacto_sys_set_critic_type": (C.c_int, [vp, C.c_int]),
    "cacto_env_step_batch": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, C.c_int, vp]),
    "cacto_env_ee": (C.c_int, [vp, vp, vp, C.c_int, vp]),
    "cacto_env_step": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, C.c_int, vp]),
    "cacto_env_jacobians": (C.c_int, [vp, vp, vp, C.c_int, vp, vp, vp]),
    "cacto_env_bound_control_cost": (C.c_int, [vp, vp, vp, C.c_int, vp]),
    "cacto_mlp_param_count": (i64, [vp, C.c_int]),
    "cacto_mlp_netbuf_floats": (i64, [vp, C.c_int]),
    "cacto_mlp_pack": (C.c_int, [vp, C.c_int, vp, vp]),
    "cacto_actor_forward": (C.c_int, [vp, vp, vp, vp, C.c_int, vp]),
    "cacto_critic_forward": (C.c_int, [vp, vp, vp, vp, C.c_int, vp]),
    "cacto_critic_input_grad": (C.c_int, [vp, vp, vp, vp, vp, C.c_int, vp]),
    "cacto_workspace_bytes": (sz, [vp, C.c_int]),
    "cacto_critic_grad": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), vp, vp, vp, C.c_int, vp, vp,
                                    vp, vp, vp, sz, vp]),
    "cacto_actor_grad": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), vp, vp, C.c_int, vp, vp, sz, vp]),
    "cacto_adam_step": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), C.c_int, vp, C.c_int, vp]),
    "cacto_soft_update": (C.c_int, [vp, C.POINTER(Nets), flt, vp]),
    "cacto_update": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), vp, vp, vp, C.c_int, vp, vp, vp,
                               vp, sz, vp]),
    "cacto_pipeline_status": (C.c_int, [vp, vp]),
    "cacto_pipeline_check": (C.c_int, [vp, vp]),
    "cacto_update_n": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), vp, vp, C.c_int, C.c_int, vp, sz, vp]),
    "cacto_update_n_per": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), vp, vp, vp, i64, i64, C.c_double, vp,
                                     vp, C.c_double, C.c_double, C.c_double, vp, C.c_int, C.c_int, vp, sz, vp]),
    "cacto_dp_unique_ids": (C.c_int, [vp, C.c_int]),
    "cacto_dp_attach": (C.c_int, [vp, vp, C.c_int, C.c_int]),
    "cacto_dp_detach": (C.c_int, [vp]),
    "cacto_update_n_dp": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), vp, vp, C.c_int, C.c_int, vp, sz,
                                    vp]),
    "cacto_update_n_per_dp": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), vp, vp, vp, i64, i64, C.c_double,
                                        vp, vp, C.c_double, C.c_double, C.c_double, vp, C.c_int, C.c_int, vp, sz,
                                        vp]),
    "cacto_update_pair_grads": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), vp, vp, vp, vp, C.c_int, vp, vp,
                                          vp, vp, sz, vp]),
    "cacto_update_pair_grads_stage": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), vp, vp, vp, vp, C.c_int,
                                                vp, vp, vp, vp, sz, C.c_int, vp]),
    "cacto_update_pair_apply": (C.c_int, [vp, C.POINTER(Nets), C.POINTER(UpdateCfg), vp, C.c_int, C.c_int, C.c_int,
                                          vp]),
    "cacto_rollout": (C.c_int, [vp, vp, vp, vp, C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_int, vp]),
    "cacto_rollout_sched": (C.c_int, [vp, vp, vp, vp, C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_int,
                                      C.c_int, C.c_int, vp]),
    "cacto_rollout_rewards": (C.c_int, [vp, vp, vp, vp, C.c_int, C.c_int, vp, vp, vp, C.c_int, vp]),
    "cacto_ddp_backward": (C.c_int, [vp, vp, i64, vp, i64, vp, C.c_int, C.c_double, vp, vp]),
    "cacto_buffer_add": (C.c_int, [vp, vp, i64, i64, vp, i64, vp]),
    "cacto_rl_solve_add": (C.c_int, [vp, vp, i64, vp, i64, vp, vp, vp, C.c_int, C.c_int, i64, C.c_int, C.c_int, vp,
                                     i64, i64, vp, vp]),
    "cacto_buffer_gather": (C.c_int, [vp, vp, vp, C.c_int, vp, vp, vp, vp, vp, vp, vp]),
    "cacto_per_init": (C.c_int, [vp, vp, i64, vp]),
    "cacto_per_set_range": (C.c_int, [vp, vp, i64, i64, i64, i64, dbl, vp]),
    "cacto_per_set_range_max": (C.c_int, [vp, vp, i64, i64, i64, i64, vp, dbl, vp]),
    "cacto_per_sample": (C.c_int, [vp, vp, i64, i64, dbl, vp, C.c_int, vp, vp, vp, vp]),
    "cacto_per_shard_stats": (C.c_int, [vp, vp, i64, vp, vp]),
    "cacto_per_sample_global": (C.c_int, [vp, vp, i64, i64, dbl, vp, C.c_int, vp, C.c_int, vp, vp, vp, vp]),
    "cacto_per_update": (C.c_int, [vp, vp, i64, vp, vp, vp, vp, dbl, dbl, dbl, vp, C.c_int, vp]),
    "cacto_per_set_leaves": (C.c_int, [vp, vp, i64, vp, vp, C.c_int, vp]),
    "cacto_per_update_relo": (C.c_int, [vp, vp, i64, vp, vp, vp, vp, vp, dbl, dbl, dbl, vp, vp, vp, C.c_int, vp]),
}


def header_exports():
    """Names of every function declared in include/cacto_hip.h."""
    with open(HEADER) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cacto_[a-z0-9_]+)\s*\(", text)))


class _Lib:
    def __init__(self, path=LIB_PATH):
        if not os.path.exists(path):
            raise RuntimeError("libcacto_hip.so not found at %s — build it with `python -m cacto_amd.build` "
                               "(there is no CPU fallback)" % path)
        self.path = path
        self.dll = C.CDLL(path)
        # CACTO_LIB_PARTIAL=1 (diagnostics only: A/B runs against libraries of older revisions)
        # binds the symbols the library has and skips the rest
        partial = os.environ.get("CACTO_LIB_PARTIAL") == "1"
        for name, (res, args) in _SIGS.items():
            if partial and not hasattr(self.dll, name):
                continue
            fn = getattr(self.dll, name)
            fn.restype = res
            fn.argtypes = args
        if self.dll.cacto_abi_version() != 1:
            raise RuntimeError("libcacto_hip.so ABI mismatch")

    def call(self, name, *args):
        rc = getattr(self.dll, name)(*args)
        if rc != 0:
            msg = self.dll.cacto_last_error().decode(errors="replace")
            raise RuntimeError("%s failed (%d): %s" % (name, rc, msg))
        return rc

    def raw(self, name):
        return getattr(self.dll, name)


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _Lib()
    return _LIB
