"""Diagnostic: host enqueue time vs GPU completion time of the update loop (sequential update_rows
calls vs the pipelined update_rows_n), to tell a launch-bound loop from a GPU-bound one.

    python tools/update_host_cost.py [B]          # GRAPH_OF_PIPELINE=1: also the pipelined loop as a HIP graph

Measured (B = 128, DI): sequential 92.6 us/update (host 22.9), pipelined 61.3 (host 35.5),
pipelined replayed as a HIP graph 56.4 (host 27.8: ROCm enqueues graph nodes from the host).
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    conf, env, rl = bench.make_learner("double_integrator")
    N, K = 65536, 200
    ns = conf.nb_state
    rng = np.random.default_rng(0)
    S = np.column_stack([rng.uniform(-15, 15, (N, ns - 1)), rng.uniform(0, 9.9, N)])
    rows = np.concatenate([S, rng.normal(size=(N, 1)), S + 0.05, rng.normal(size=(N, ns)) * 0.3,
                           np.zeros((N, 2))], axis=1)
    storage = torch.as_tensor(rows, device="cuda")
    idx = torch.as_tensor(rng.integers(0, N, size=(K, B)).astype(np.int32), device="cuda")
    for _ in range(2):
        rl.update_rows_n(storage, idx[:10])
        for k in range(10):
            rl.update_rows(storage, idx[k])
    torch.cuda.synchronize()
    for name, fn in (("sequential", lambda: [rl.update_rows(storage, idx[k]) for k in range(K)]),
                     ("pipelined", lambda: rl.update_rows_n(storage, idx))):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("%-10s B=%d: host enqueue %.1f us/update, completion %.1f us/update"
              % (name, B, 1e6 * (t1 - t0) / K, 1e6 * (t2 - t0) / K))


def graph_of_pipeline(B=128):
    """The pipelined K-update call captured into one HIP graph and replayed."""
    conf, env, rl = bench.make_learner("double_integrator")
    N, K = 65536, 200
    ns = conf.nb_state
    rng = np.random.default_rng(0)
    S = np.column_stack([rng.uniform(-15, 15, (N, ns - 1)), rng.uniform(0, 9.9, N)])
    rows = np.concatenate([S, rng.normal(size=(N, 1)), S + 0.05, rng.normal(size=(N, ns)) * 0.3,
                           np.zeros((N, 2))], axis=1)
    storage = torch.as_tensor(rows, device="cuda")
    idx = torch.as_tensor(rng.integers(0, N, size=(K, B)).astype(np.int32), device="cuda")
    rl.update_rows_n(storage, idx[:10])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        rl.update_rows_n(storage, idx)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("graph(pipelined) B=%d: host %.1f us/update, completion %.1f us/update"
          % (B, 1e6 * (t1 - t0) / K, 1e6 * (t2 - t0) / K))


if __name__ == "__main__":
    main()
    if os.environ.get("GRAPH_OF_PIPELINE"):
        graph_of_pipeline(int(sys.argv[1]) if len(sys.argv) > 1 else 128)
