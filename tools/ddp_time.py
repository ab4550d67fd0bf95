"""Diagnostic: cacto_ddp_backward time for a system's bench rollout batch (the bench's ddp_labels).
    python tools/ddp_time.py SYSTEM R"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    system, R = sys.argv[1], int(sys.argv[2])
    conf, env, rl = bench.make_learner(system)
    roll = bench.rollout_phase(rl, conf, env, R, 3, 1, 1, 0)
    _, d = bench.ddp_labels(rl, conf, env, roll, K=10)
    print("%s R=%d ddp labels: %.3f ms (%d Riccati steps, %.1f M steps/s)" % (system, R, d["ms_per_call"],
                                                                          d["riccati_steps"], d["steps_per_s"] / 1e6))


if __name__ == "__main__":
    bench.LONG_STEPS = 0
    main()
