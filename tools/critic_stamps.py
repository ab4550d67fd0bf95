"""Diagnostic: per-phase cycle counts (s_memtime) of k_critic_grad, workgroup 0, from the
CACTO_STAMPS build. Not part of the product path.

    python -c "from cacto_amd.build import build_variant; build_variant('libcacto_hip_stamps', ['CACTO_STAMPS'])"
    CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so python tools/critic_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cacto_amd import _lib as L  # noqa: E402
import bench  # noqa: E402

NAMES = ["load", "tgt_fwd", "vt_fwd+fwd", "first_bwd", "sob_g0", "sp_l0", "sp_l1", "sp_l2", "sp_l3", "vloss",
         "zb3", "hb_l3", "hb_l2", "hb_l1", "tail"]
IDS = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15]


def main():
    conf, env, rl = bench.make_learner("double_integrator")
    rows = torch.randn(8192, 3 * conf.nb_state + 3, dtype=torch.float64, device="cuda")
    for B in (128, 4096):
        idx = torch.randint(0, 8192, (B,), dtype=torch.int32, device="cuda")
        for _ in range(3):
            rl.critic_grad_flat(rows, idx)
        torch.cuda.synchronize()
        st = (ctypes.c_ulonglong * 32)()
        L.lib().dll.cacto_debug_critic_stamps(st)
        t = np.array(st[:16], dtype=np.float64)
        d = np.diff(t[IDS])
        print("B=%d total %.0f cycles: " % (B, t[15] - t[0]) + ", ".join("%s %.0f" % (n, x) for n, x in zip(NAMES, d)))
        f = np.array(st[16:27], dtype=np.float64)
        if st[28] > st[27]:
            print("   forward fragment loads (wave 0, issue -> all landed): %d cycles" % (st[28] - st[27]))
        fn = ["l0 mfma+epi", "l0 barrier", "l1", "l1 bar", "l2", "l2 bar", "l3", "l3 bar", "l4", "l4 bar"]
        print("   last critic forward (thread 0): start->l0 %.0f after fwd start; " % (f[0] - t[2]) +
              ", ".join("%s %.0f" % (n, x) for n, x in zip(fn, np.diff(f))))


def actor():
    conf, env, rl = bench.make_learner(sys.argv[2] if len(sys.argv) > 2 else "double_integrator")
    rows = torch.randn(8192, 3 * conf.nb_state + 3, dtype=torch.float64, device="cuda") * 0.5
    names = ["load", "actor_fwd", "dynamics", "fill", "critic_fwd", "critic_bwd1", "dQda", "actor_bwd_l2",
             "actor_bwd_l1"]
    for B in (128, 4096):
        idx = torch.randint(0, 8192, (B,), dtype=torch.int32, device="cuda")
        for _ in range(3):
            rl.actor_grad_flat(rows, idx)
        torch.cuda.synchronize()
        st = (ctypes.c_ulonglong * 32)()
        L.lib().dll.cacto_debug_critic_stamps(st)
        t = np.array(st[:10], dtype=np.float64)
        print("actor B=%d total %.0f cycles: " % (B, t[9] - t[0]) + ", ".join("%s %.0f" % (n, x) for n, x in zip(names, np.diff(t))))
        if st[10] > st[1] and st[11] > st[10]:
            print("   actor forward: layer 1 %.0f, layer 2 %.0f, layer 3 %.0f" % (st[10] - st[1], st[11] - st[10], st[2] - st[11]))
        if st[2] < st[12] < st[3]:
            print("   dynamics: M / h %.0f, factor + solves %.0f" % (st[12] - st[2], st[3] - st[12]))


def pair():
    """The actor chain inside the paired kernel (cacto_update_n at B <= 512), tile 0."""
    conf, env, rl = bench.make_learner(sys.argv[2] if len(sys.argv) > 2 else "double_integrator")
    rows = torch.randn(8192, 3 * conf.nb_state + 3, dtype=torch.float64, device="cuda") * 0.5
    names = ["load", "actor_fwd", "dynamics", "fill", "critic_fwd", "critic_bwd1", "dQda", "actor_bwd_l2",
             "actor_bwd_l1"]
    for B in (64, 128):
        idx = torch.randint(0, 8192, (3, B), dtype=torch.int32, device="cuda")
        for _ in range(2):
            rl.update_rows_n(rows, idx)
        torch.cuda.synchronize()
        st = (ctypes.c_ulonglong * 32)()
        L.lib().dll.cacto_debug_actor_stamps(st)
        t = np.array(st[:10], dtype=np.float64)
        print("paired actor B=%d total %.0f cycles: " % (B, t[9] - t[0]) +
              ", ".join("%s %.0f" % (n, x) for n, x in zip(names, np.diff(t))))
        print("   actor forward: layer 1 %.0f, layer 2 %.0f, layer 3 %.0f" % (st[10] - st[1], st[11] - st[10], st[2] - st[11]))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "pair":
        pair()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "actor":
        actor()
        sys.exit(0)
    main()
