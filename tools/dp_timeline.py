"""Diagnostic: the data-parallel update loop over a one-rank RCCL group (cacto_update_n_dp /
cacto_update_n_per_dp) on synthetic replay rows, for a kernel trace. Not part of the product path.

    rocprofv3 --kernel-trace -d D -o run -- python tools/dp_timeline.py [car_park|ur5] [B] [K]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch.distributed as dist
    system = sys.argv[1] if len(sys.argv) > 1 else "car_park"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 300
    cfg = bench.EXTRA[system]
    conf, env, rl = bench.make_learner(system, w_S=cfg["w_S"])
    group = bench.init_dp1_group()
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer, ReplayBuffer
    ns = conf.nb_state
    rng = np.random.default_rng(0)
    N = 60000
    lo, hi = np.array(conf.x_init_min, dtype=float), np.array(conf.x_init_max, dtype=float)
    S = rng.uniform(lo, hi, size=(N, ns))
    rows = np.concatenate([S, rng.normal(size=(N, 1)), S + 0.01, rng.normal(size=(N, ns)) * 0.3,
                           np.zeros((N, 1)), np.zeros((N, 1))], axis=1)
    conf.BATCH_SIZE = B
    if cfg["per"]:
        conf.prioritized_replay_alpha = 0.6
        buf = PrioritizedReplayBuffer(conf, env.sys)
    else:
        buf = ReplayBuffer(conf, env.sys)
    buf.add_rows(rows)
    for mode in ("single", "dp"):
        rl.set_data_parallel(1, group if mode == "dp" else None)
        if cfg["per"]:
            buf.set_data_parallel(1, group if mode == "dp" else None)
            U = torch.as_tensor(rng.random((K, B)), device="cuda")
            loop = rl.update_rows_n_per_dp if mode == "dp" else rl.update_rows_n_per
            loop(buf, U[:50])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            loop(buf, U)
        else:
            idx = torch.as_tensor(rng.integers(0, N, size=(K, B)).astype(np.int32), device="cuda")
            rl.update_rows_n(buf.storage, idx[:50])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rl.update_rows_n(buf.storage, idx)
        torch.cuda.synchronize()
        print("%s %s B=%d: %.1f updates/s" % (system, mode, B, K / (time.perf_counter() - t0)), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
