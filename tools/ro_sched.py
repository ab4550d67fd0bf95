"""Diagnostic: k_rollout time (HIP events) per schedule for one system's bench rollout batch.
Not part of the product path.

    python tools/ro_sched.py SYSTEM R "g,w g,w ..."     # (groups, workgroups); 0 = automatic
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    system, R = sys.argv[1], int(sys.argv[2])
    scheds = [tuple(int(x) for x in t.split(",")) for t in (sys.argv[3] if len(sys.argv) > 3 else "0,0").split()]
    conf, env, rl = bench.make_learner(system)
    S0, n = bench.initial_states(env, conf, R, seed=0)
    T = int(n.max())
    inputs = rl.rollout_inputs(S0, n)
    f64 = dict(dtype=torch.float64, device="cuda")
    out = {"S": torch.empty(R, T + 1, conf.nb_state, **f64),
           "A": torch.empty(R, T, conf.nb_action, dtype=torch.float32, device="cuda"),
           "status": torch.empty(R, dtype=torch.int32, device="cuda")}
    steps = int(n.sum())
    for sc in scheds:
        for _ in range(2):
            rl.rollout_batch(None, None, T, inputs=inputs, out=out, sched=sc)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        reps = int(os.environ.get("RO_REPS", "50"))
        for _ in range(reps):
            rl.rollout_batch(None, None, T, inputs=inputs, out=out, sched=sc)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print("%s R=%d sched=%s: %.3f ms  %.1fM env-steps/s" % (system, R, sc, ms, steps / ms / 1e3), flush=True)


if __name__ == "__main__":
    main()
