"""Diagnostic: phase stamps (s_memtime) of k_wgrad_adam, workgroup 0 / wave 0 (the actor's layer-0
tile after an update_rows call), from the CACTO_STAMPS build. Not part of the product path.

    CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so python tools/fused_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cacto_amd import _lib as L  # noqa: E402
import bench  # noqa: E402


def main():
    conf, env, rl = bench.make_learner("double_integrator")
    rows = torch.randn(8192, 3 * conf.nb_state + 3, dtype=torch.float64, device="cuda")
    for B in (64, 128, 256):
        idx = torch.randint(0, 8192, (B,), dtype=torch.int32, device="cuda")
        for _ in range(3):
            rl.update_rows(rows, idx)
        torch.cuda.synchronize()
        st = (ctypes.c_ulonglong * 32)()
        L.lib().dll.cacto_debug_critic_stamps(st)
        t = np.array(st[:6], dtype=np.float64)
        print("fused B=%d total %.0f: scalars %.0f, first touch %.0f, gemm %.0f, land %.0f, adam %.0f" %
              (B, t[4] - t[0], t[1] - t[0], t[5] - t[1], t[2] - t[5], t[3] - t[2], t[4] - t[3]))


if __name__ == "__main__":
    main()
