"""Diagnostic: per-phase cycle counts of one k_rollout step (workgroup 0, step 20) from the
CACTO_STAMPS build. Not part of the product path.

    python -c "from cacto_amd.build import build_variant; build_variant('libcacto_hip_stamps', ['CACTO_STAMPS'])"
    CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so python tools/rollout_stamps.py [system [R [groups,workgroups]]]
"""
import ctypes
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv += [] if len(sys.argv) > 1 else ["double_integrator"]

from cacto_amd import _lib as L  # noqa: E402
import bench  # noqa: E402


def main():
    system = sys.argv[1]
    conf, env, rl = bench.make_learner(system)
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    S0, n = bench.initial_states(env, conf, R, seed=0)
    T = int(n.max())
    inputs = rl.rollout_inputs(S0, n)
    sched = tuple(int(x) for x in sys.argv[3].split(",")) if len(sys.argv) > 3 else None
    for _ in range(3):
        out = rl.rollout_batch(None, None, T, inputs=inputs, sched=sched or (0, 0))
    torch.cuda.synchronize()
    st = (ctypes.c_ulonglong * 20)()
    L.lib().dll.cacto_debug_rollout_stamps(st)
    t = np.array(st[:4], dtype=np.float64)
    a1, a2 = float(st[4]) - t[0], float(st[5]) - float(st[4])
    names = ["actor", "E1 (dynamics | reward terms)", "E2 (reward combine + stores + refill | EE(s'))"]
    print(system, R, "step cycles %.0f: " % (t[3] - t[0]) + ", ".join("%s %.0f" % (nm, d) for nm, d in zip(names, np.diff(t))))
    print("   actor: layer 1 (+ placements) %.0f, layer 2 %.0f, layer 3 %.0f" % (a1, a2, t[1] - float(st[5])))
    if st[9] > st[1]:
        print("   chain dynamics after the actor: RNEA (wave 0) %.0f, CRBA columns (waves 1-3) %s"
              % (float(st[9]) - t[1], ", ".join("%.0f" % (float(st[9 + w]) - t[1]) if st[9 + w] > st[1] else "-"
                                                   for w in (1, 2, 3))))
    if st[17] > st[1] and st[18] > st[17]:
        print("   RNEA by lanes: loads %.0f, v / a rounds %.0f, force terms %.0f, force rounds %.0f"
              % (float(st[17]) - t[1], float(st[18]) - float(st[17]), float(st[19]) - float(st[18]),
                 float(st[9]) - float(st[19])))
    if st[13] > st[2] or st[14] > st[2]:
        print("   reward waves after the actor / dynamics phase: r_t (wave 1) %s, EE(s_t) (wave 2) %s, EE(s_n) (wave 3) %s"
              % tuple("%.0f" % (float(st[k]) - t[2]) if st[k] > st[2] else "-" for k in (13, 14, 15)))
    print("   wave 0 after the dynamics phase: s' %.0f, advance/stores %.0f, refill+ballot %.0f, barrier %.0f"
          % (float(st[6]) - t[2], float(st[7]) - float(st[6]), float(st[8]) - float(st[7]), t[3] - float(st[8])))
    if st[16] >= st[6]:
        print("      (of advance/stores: next input (revolute chains: before the stores) %.0f, stores %.0f)"
              % (float(st[16]) - float(st[6]), float(st[7]) - float(st[16])))


if __name__ == "__main__":
    main()
