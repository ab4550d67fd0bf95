"""Diagnostic: per-phase cycles of one step (step 20, workgroup 0) of each team of k_rollout_tt,
or ('ks') per-phase cycles of every step of k_rollout_ks (CACTO_STAMPS build). Not part of the
product path.
    CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so python tools/tt_stamps.py [system] [ks]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cacto_amd import _lib as L  # noqa: E402
import bench  # noqa: E402


def main():
    system = sys.argv[1] if len(sys.argv) > 1 else "double_integrator"
    conf, env, rl = bench.make_learner(system)
    S0, n = bench.initial_states(env, conf, 4096, seed=0)
    T = int(n.max())
    inputs = rl.rollout_inputs(S0, n)
    for _ in range(3):
        rl.rollout_batch(None, None, T, inputs=inputs, want=("S", "A"), sched=(-1, 0))
    torch.cuda.synchronize()
    st = (ctypes.c_ulonglong * 20)()
    L.lib().dll.cacto_debug_rollout_stamps(st)
    v = np.array(st[:16], dtype=np.float64)
    for team in (0, 1):
        t = v[8 * team: 8 * team + 4]
        print(system, "team", team, "step %.0f: actor %.0f, dynamics+stores+refill %.0f, barrier %.0f"
              % (t[3] - t[0], t[1] - t[0], t[2] - t[1], t[3] - t[2]), "(start offset vs team 0: %.0f)" % (t[0] - v[0]))
    print("   team 0 actor: layer 1 %.0f, layer 2 %.0f, layer 3 %.0f" % (v[4] - v[0], v[5] - v[4], v[1] - v[5]))
    # every step of every team of the last launch, accumulated in-kernel (wave 0 and wave 1 of each team)
    acc = (ctypes.c_ulonglong * (1024 * 2 * 2 * 10))()
    L.lib().dll.cacto_debug_rollout_tt_acc(acc)
    a = np.array(acc[:], dtype=np.float64).reshape(1024, 2, 2, 10)
    names = ["layer 1 + bar", "layer 2 + bar", "layer 3 + bar", "dynamics/stores/refill", "end barrier",
             "(wave 0: a + s'=f(s,a)", "stores", "refill", "next input + ballot)"]
    for w in (0, 1):
        steps = a[:, :, w, 9].sum()
        tot = a[:, :, w, :9].sum(axis=(0, 1))
        per = tot / max(steps, 1)
        print("   all teams, wave %d, %d team-steps: cycles per step %.0f = " % (w, steps, per[:5].sum()) +
              ", ".join("%s %.0f" % (n, x) for n, x in zip(names, per)))


def ks(system):
    """k_rollout_ks (groups -3): per-phase cycles per step, every wave."""
    conf, env, rl = bench.make_learner(system)
    S0, n = bench.initial_states(env, conf, 4096, seed=0)
    T = int(n.max())
    inputs = rl.rollout_inputs(S0, n)
    for _ in range(3):
        rl.rollout_batch(None, None, T, inputs=inputs, want=("S", "A"), sched=(-3, 0))
    torch.cuda.synchronize()
    acc = (ctypes.c_ulonglong * (1024 * 8 * 7))()
    L.lib().dll.cacto_debug_rollout_ws_acc(acc)
    a = np.array(acc[:], dtype=np.float64).reshape(1024, 8, 7)
    names = ["loop test + layer 2 + bar", "layer 3", "s'=f(s,a) + stores", "refill", "layer 1", "end barrier"]
    steps = a[..., 6].sum()
    per = a[..., :6].sum(axis=(0, 1)) / max(steps, 1)
    print(system, "k_rollout_ks, %d wave-steps: cycles per step %.0f = " % (steps, per.sum()) +
          ", ".join("%s %.0f" % (nm, x) for nm, x in zip(names, per)))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "ks":
        ks(sys.argv[1])
        sys.exit(0)
    main()
