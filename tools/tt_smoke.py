"""Two-team rollout kernel (k_rollout_tt) against the single-team kernel on a small DI batch:
the trajectories must be identical. Prints OK and the two kernels' times at 4096 episodes."""
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import bench  # noqa: E402


def main():
    system = sys.argv[1] if len(sys.argv) > 1 else "double_integrator"
    conf, env, rl = bench.make_learner(system)
    rng = random.Random(2)
    S0 = np.array([env.reset() for _ in range(40)])
    ns_ = [conf.NSTEPS - int(s[-1] / conf.dt) for s in S0]
    T = max(ns_)
    a = rl.rollout_batch(S0, ns_, T, sched=(1, 40))
    b = rl.rollout_batch(S0, ns_, T, sched=(-1, 2))
    torch.cuda.synchronize()
    for k, n in enumerate(ns_):
        for key, m in (("S", n + 1), ("A", n)):
            assert np.array_equal(a[key][k, :m].cpu().numpy(), b[key][k, :m].cpu().numpy()), (key, k)
    assert (b["status"].cpu().numpy() == 0).all()
    print("small batch identical")
    S0, n = bench.initial_states(env, conf, 4096, seed=0)
    T = int(n.max())
    inputs = rl.rollout_inputs(S0, n)
    out = {"S": torch.zeros(4096, T + 1, conf.nb_state, dtype=torch.float64, device="cuda"),
           "A": torch.zeros(4096, T, conf.nb_action, dtype=torch.float32, device="cuda"),
           "status": torch.zeros(4096, dtype=torch.int32, device="cuda")}
    for sched in ((2, 0), (-1, 0), (2, 0), (-1, 0)):
        for _ in range(3):
            rl.rollout_batch(None, None, T, inputs=inputs, out=out, sched=sched)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            rl.rollout_batch(None, None, T, inputs=inputs, out=out, sched=sched)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 50
        print(system, "sched", sched, "%.4f ms  %.1f M env-steps/s" % (dt * 1e3, n.sum() / dt / 1e6))


if __name__ == "__main__":
    main()
