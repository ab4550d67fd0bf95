"""Diagnostic: accumulated per-phase cycles of k_rollout_sw (the manipulator's actor waves beside
dynamics waves), averaged over the workgroups, per half-step (CACTO_STAMPS build). Not part of the
product path.
    CACTO_HIP_LIB=cacto_amd/libcacto_diag.so python tools/sw_stamps.py [system [R]]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cacto_amd import _lib as L  # noqa: E402
import bench  # noqa: E402


def main():
    system = sys.argv[1] if len(sys.argv) > 1 else "manipulator"
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    conf, env, rl = bench.make_learner(system)
    S0, n = bench.initial_states(env, conf, R, seed=0)
    T = int(n.max())
    inputs = rl.rollout_inputs(S0, n)
    for _ in range(3):
        rl.rollout_batch(None, None, T, inputs=inputs, want=("S", "A"), sched=(-4, 0))
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (1024 * 2 * 6))()
    L.lib().dll.cacto_debug_rollout_sw_acc(buf)
    v = np.array(buf[:], dtype=np.float64).reshape(1024, 2, 6)
    used = v[:, 0, 5] > 0
    a, d = v[used, 0], v[used, 1]
    hs = a[:, 5].sum()
    print("%s %d k_rollout_sw, %d workgroups, %.0f half-steps each" % (system, R, used.sum(), a[:, 5].mean()))
    print("   actor waves per half-step: actor + placements %.0f, end barrier %.0f" % (a[:, 0].sum() / hs,
                                                                                  a[:, 1].sum() / hs))
    print("   dynamics waves per half-step: loop test %.0f, RNEA / CRBA + bar %.0f, step + stores + refill "
          "+ next input %.0f, end barrier %.0f" % tuple(d[:, k].sum() / hs for k in range(4)))


if __name__ == "__main__":
    main()
