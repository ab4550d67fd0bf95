"""Diagnostic: one full-size rollout batch of a system (bench.py's initial states and weights), S and A
saved to an .npz, for bit-for-bit comparison of two library builds (CACTO_HIP_LIB). Not part of the
product path.

    CACTO_HIP_LIB=cacto_amd/libA.so python tools/ro_bits.py ur5 2048 a.npz
    CACTO_HIP_LIB=cacto_amd/libB.so python tools/ro_bits.py ur5 2048 b.npz
    python tools/ro_bits.py --compare a.npz b.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        n = a["n"]
        bad = 0
        for e in range(len(n)):
            k = int(n[e])
            if not (np.array_equal(a["S"][e, :k + 1], b["S"][e, :k + 1]) and np.array_equal(a["A"][e, :k], b["A"][e, :k])):
                bad += 1
        print("episodes differing: %d of %d" % (bad, len(n)))
        sys.exit(1 if bad else 0)
    import torch
    import bench
    system, R, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    conf, env, rl = bench.make_learner(system)
    S0, n = bench.initial_states(env, conf, R, seed=0)
    T = int(n.max())
    res = rl.rollout_batch(S0, n, T, want=("S", "A"))
    torch.cuda.synchronize()
    np.savez(out, S=res["S"].cpu().numpy(), A=res["A"].cpu().numpy(), n=np.asarray(n))
    print("saved", out)


if __name__ == "__main__":
    main()
