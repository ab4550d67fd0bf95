#!/usr/bin/env python
"""CACTO hot-path benchmark on MI355X (BASELINE.json metric: env-steps/sec + critic-updates/sec).

Workload (BASELINE.json configs[1]): double_integrator, w_S = 1e-2, 4096 rollouts per GPU.
  * step = one batched rollout of the 4096 episodes (RL_AC.create_TO_init / PLOT.rollout loop:
    actor MFMA tile + float64 dynamics + reward + EE per env-step, all in one persistent kernel);
    initial states from Env.reset (CPython random seeded per rank), NSTEPS_SH = NSTEPS - int(t/dt).
    `value` = env-steps/s summed over ranks (weak scaling: every rank rolls out its own episodes).
  * critic_updates: the learn_and_update loop (RL_AC.update + update_target) at the reference
    minibatch (128) and a scaled one (4096), on a 65,536-row replay buffer filled from the
    rollouts; with N > 1 ranks each rank takes the minibatch locally and the gradients are
    all-reduced over RCCL (data parallel, one global update per iteration).
Inputs are resident in HBM before timing. Weights: the reference's DI seed-0 initial weights
(tests/golden/weights/di_seed0_0.npz); dVdx labels come from the DDP backward pass along the
rollouts (cacto_ddp_backward, every system; the TO NLP solve itself is host-side CasADi, absent).

    python bench.py [--gpus N --steps K --warmup W]
"""
import argparse
import ctypes
import json
import os
import random
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec + critic-updates/sec per node, double_integrator & manipulator"
FP32_MFMA_PEAK = 157.3e12   # MI355X_MICROARCH.md: FP32 matrix 157.3 TF spec (dense)


def fa_flops(ns, na):
    return 2 * (ns * 256 + 256 * 256 + 256 * na)


def fc_flops(ns):
    return 2 * (ns * 64 + 64 * 64 + 64 * 128 + 128 * 128 + 128)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--system", default="double_integrator")
    p.add_argument("--rollouts", type=int, default=4096)
    p.add_argument("--update-steps", type=int, default=1000)
    p.add_argument("--batches", default="128,4096")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--graph", action="store_true",
                   help="replay the update loop as one HIP graph (RL_AC.capture_updates) instead of launching "
                        "it eagerly; measured equal on MI355X (the update is bound by its kernels, not launches)")
    p.add_argument("--extra-systems", default="manipulator,car_park,ur5")
    p.add_argument("--no-dp1", action="store_true",
                   help="skip the one-rank RCCL data-parallel update leg (N = 1 only)")
    p.add_argument("--no-config0", action="store_true",
                   help="skip BASELINE configs[0] (single integrator, one main.py training iteration, GPU vs CPU)")
    p.add_argument("--no-diagnostics", action="store_true",
                   help="skip the rollout variants (profiling runs: every k_rollout dispatch is a full rollout)")
    p.add_argument("--long-steps", type=int, default=1000,
                   help="rollout batches of the long robustness region reported beside the K-step value")
    p.add_argument("--dry-run", action="store_true",
                   help="rank plumbing only: launch / rendezvous (gloo on the CPU) and print each rank's "
                        "RANK / LOCAL_RANK / WORLD_SIZE and the device it would use; no GPU call")
    p.add_argument("--launch-timeout", type=float, default=1800.0,
                   help="seconds the --gpus N launcher waits for its ranks before killing them")
    return p.parse_args()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) run directly, without a torch.distributed launcher: start N
    fresh rank processes of this script — one per GPU, RANK = LOCAL_RANK = r, WORLD_SIZE = N,
    rendezvous on 127.0.0.1 — before this process makes any GPU call (it makes none), wait for
    them, and exit with the first failing rank's code. Rank 0 writes the JSON line to this
    process's stdout; the other ranks' stdout goes to stderr. Replaces the reference's
    multiprocessing.Pool (main.py:219-225) as the node-level parallelism: one process per GPU."""
    import signal
    import subprocess
    n = args.gpus
    port = os.environ.get("MASTER_PORT") or str(free_port())
    procs = []

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.kill()
        raise SystemExit(143)
    signal.signal(signal.SIGTERM, stop)
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                          stdout=None if r == 0 else sys.stderr.fileno()))
        t0, last = time.time(), time.time()
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print("bench launcher: rank %d exited with %d; stopping the other ranks" % (r, c), file=sys.stderr)
                return c
            if all(c == 0 for c in codes):
                return 0
            if time.time() - t0 > args.launch_timeout:
                print("bench launcher: ranks still running after %.0f s; killing them" % args.launch_timeout,
                      file=sys.stderr)
                return 124
            if time.time() - last > 60:
                last = time.time()
                print("bench launcher: %d of %d ranks running, %.0f s" % (sum(c is None for c in codes), n,
                                                                          last - t0), file=sys.stderr, flush=True)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()


def dry_run(args):
    """The rank plumbing without the GPU: rendezvous over gloo (CPU) as the real run would over
    RCCL, all-gather what every rank sees, rank 0 prints one JSON line."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # launcher tests: a rank that fails or hangs before the rendezvous
    if os.environ.get("CACTO_DRYRUN_FAIL_RANK") == str(rank):
        sys.exit(3)
    if os.environ.get("CACTO_DRYRUN_HANG_RANK") == str(rank):
        time.sleep(3600)
    me = dict(rank=rank, local_rank=local, world_size=world, device="cuda:%d" % local,
              master="%s:%s" % (os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")))
    ranks = [me]
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
        dist.destroy_process_group()
    if rank == 0:
        # the PER loop a real run of this world size times (per_loop against the RL_AC method names)
        from cacto_amd.rl import RL_AC
        loop = per_loop(RL_AC.__new__(RL_AC), world)
        print(json.dumps({"dry_run": True, "n_gpus": world, "gpus_requested": args.gpus, "ranks": ranks,
                          "backend": os.environ.get("CACTO_DIST_BACKEND", "nccl"),
                          "per_loop": None if loop is None else loop.__name__}))


def pmc_traffic(kernel=("k_rollout_ks<2", "k_rollout_tt<2", "k_rollout<2,")):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summaries
    (profiles/rNN_pmc_{fetch,write}.csv, made by tools/prof_summary.py from separate --pmc
    FETCH_SIZE / WRITE_SIZE passes). gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE
    counts half of the bytes of 16-B-per-lane reads -> x2; WRITE_SIZE is exact. Values are KiB."""
    import csv
    import glob
    prof = os.path.join(ROOT, "profiles")
    fetch = sorted(glob.glob(os.path.join(prof, "r*_pmc_fetch.csv")))
    write = sorted(glob.glob(os.path.join(prof, "r*_pmc_write.csv")))
    if not fetch or not write:
        return None, None

    kernels = (kernel,) if isinstance(kernel, str) else kernel

    def mean(path, counter):
        # the first of `kernels` the summary holds: the double integrator's sequential pass at its
        # bench schedule (k_rollout_ks<2> since round 4, k_rollout_tt<2> in round 3, k_rollout<2, 2>
        # before)
        with open(path) as f:
            rows = list(csv.DictReader(f))
        for k in kernels:
            for row in rows:
                if row["kernel"].replace(" ", "").startswith(k) and row["counter"] == counter:
                    return float(row["mean"])
        return None
    fk, wk = mean(fetch[-1], "FETCH_SIZE"), mean(write[-1], "WRITE_SIZE")
    if fk is None or wk is None:
        return None, None
    return (2.0 * fk + wk) * 1024.0, os.path.basename(fetch[-1]) + " + " + os.path.basename(write[-1])


def pmc_update_traffic(B):
    """HBM bytes per DI update at batch B from the committed learner PMC summaries
    (profiles/rNN_pmc_learn_{fetch,write}_b<B>.csv: separate FETCH_SIZE / WRITE_SIZE passes over
    the update kernels of a DI-only run). Bytes of every learner dispatch in the run ÷ the number of
    updates (one critic gradient per update: the paired chain grid, or the standalone critic chain
    that opens and the classic k_critic_grad). Same gfx950 corrections as pmc_traffic (FETCH_SIZE
    x2, KiB). Returns (bytes, per-kernel bytes per update, source) or (None, None, None)."""
    import csv
    import glob
    prof = os.path.join(ROOT, "profiles")
    fetch = sorted(glob.glob(os.path.join(prof, "r*_pmc_learn_fetch_b%d.csv" % B)))
    write = sorted(glob.glob(os.path.join(prof, "r*_pmc_learn_write_b%d.csv" % B)))
    if not fetch or not write:
        return None, None, None
    tot, updates = {}, {}
    for path, counter, scale in ((fetch[-1], "FETCH_SIZE", 2.0), (write[-1], "WRITE_SIZE", 1.0)):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["counter"] != counter:
                    continue
                k, n = row["kernel"], int(row["dispatches"])
                tot[k] = tot.get(k, 0.0) + scale * float(row["mean"]) * 1024.0 * n
                if k.startswith(("k_chain_pair", "k_critic_grad")):
                    updates[(counter, k)] = n
    nup = sum(n for (c, _), n in updates.items() if c == "FETCH_SIZE")
    if not tot or nup == 0:
        return None, None, None
    per = {k: v / nup for k, v in tot.items()}
    return sum(per.values()), per, os.path.basename(fetch[-1]) + " + " + os.path.basename(write[-1])


def init_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CACTO_DIST_BACKEND=gloo: rehearsal of the multi-rank path on fewer GPUs than ranks (ranks
    # share devices round-robin); the default is RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("CACTO_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    DIST["backend"] = backend if world > 1 else None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
        DIST["ranks"] = dist.get_world_size()
        # the physical devices the ranks run on (a gloo rehearsal may put several ranks on one GPU)
        devs = [None] * world
        props = torch.cuda.get_device_properties(local)
        dist.all_gather_object(devs, str(getattr(props, "uuid", local)))
        DIST["devices"] = len(set(devs))
    return world, rank


DIST = {"backend": None, "ranks": 1, "devices": 1}


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def make_learner(system, w_S=1e-2):
    from cacto_amd.confs import load_conf
    from cacto_amd.environment import make_env
    from cacto_amd.neural_network import NN
    from cacto_amd.rl import RL_AC
    conf = load_conf(system)
    env = make_env(conf)
    nn = NN(env, conf, w_S=w_S, seed=0)
    rl = RL_AC(env, nn, conf)
    weights = None
    if system == "double_integrator":
        z = np.load(os.path.join(ROOT, "tests", "golden", "weights", "di_seed0_0.npz"))
        weights = {k: [z["%s_%d" % (k, i)] for i in range(6 if k == "actor" else 10)]
                   for k in ("actor", "critic", "target")}
    rl.setup_model(weights=weights)
    return conf, env, rl


def initial_states(env, conf, R, seed):
    random.seed(seed)
    S0, n = [], []
    while len(S0) < R:
        s = env.reset()
        k = conf.NSTEPS - int(s[-1] / conf.dt)
        if k > 0:                      # NSTEPS_SH == 0 episodes are dropped (RL.py:202-203)
            S0.append(s)
            n.append(k)
    return np.array(S0), np.array(n, dtype=np.int32)


def rollout_phase(rl, conf, env, R, K, W, world, rank):
    S0, nsteps = initial_states(env, conf, R, seed=rank)
    T = int(nsteps.max())
    inputs = rl.rollout_inputs(S0, nsteps)
    f64 = dict(dtype=torch.float64, device="cuda")
    out = {"S": torch.zeros(R, T + 1, conf.nb_state, **f64), "A": torch.zeros(R, T, conf.nb_action,
                                                                              dtype=torch.float32, device="cuda"),
           "R": torch.zeros(R, T, **f64), "EE": torch.zeros(R, T + 1, 3, **f64),
           "status": torch.zeros(R, dtype=torch.int32, device="cuda")}
    seq = {k: out[k] for k in ("S", "A", "status")}
    n_d = inputs[1]

    def step(mid=None):
        # one rollout batch = the sequential pass (k_rollout: actor + dynamics, S/A) and the parallel
        # reward / EE pass over the recorded steps (k_rollout_rewards), launched apart (a HIP event
        # between them on the sampled steps gives each kernel its own time); both run on torch's
        # current stream. (Rewards on the rollout's idle waves beside the dynamics measured slower: one
        # f64 reward per lane is a 7.6 k-cycle chain on DI against wave 0's 2 k-cycle dynamics phase —
        # DESIGN.md §3.)
        rl.rollout_batch(None, None, T, inputs=inputs, out=seq)
        if mid is not None:
            mid.record()
        rl.rollout_rewards(out, n_d, T)

    # robustness check beside the contract's K-step region (the driver runs K = 20, ~16 ms): a long
    # region of max(K, LONG_STEPS) rollout batches, as 5 consecutive segments, median reported. It runs
    # BEFORE the contract's W warmup + K timed batches, so those are taken at settled GPU clocks (the
    # first ~100 batches of a fresh process ran 5-10 % slower while the clocks ramped, r02 / r03).
    steps_per_call = int(nsteps.sum())
    long_k = max(K, LONG_STEPS) if LONG_STEPS > 0 else 0
    long_region = None
    if long_k >= 5:
        lev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        cuts_l = [j * long_k // 5 for j in range(6)]
        barrier(world)
        lev[0].record()
        for j in range(5):
            for _ in range(cuts_l[j + 1] - cuts_l[j]):
                rl.rollout_batch(None, None, T, inputs=inputs, out=seq)
                rl.rollout_rewards(out, n_d, T)
            lev[j + 1].record()
    # the W warmup steps follow the long region on the queue with no host synchronisation between
    # them (its rates are read after the timed region), so the GPU does not idle before the timed
    # region's own barrier
    for _ in range(W):
        step()
    # HIP events in the timed region: the 5 segment boundaries, and around the rollout kernel and the
    # rewards kernel of the last step of each segment (every step when K < 5), where the kernel
    # times (roofline.kernel_ms) are taken. An event is a queue marker with a cost of its own (≈5 µs
    # on this stack, §6), so the K steps are not bracketed one by one.
    nseg = 5 if K >= 5 else 0
    cuts = [j * K // 5 for j in range(6)] if nseg else []
    sampled = sorted({cuts[j + 1] - 1 for j in range(5)}) if nseg else list(range(K))
    smp = {k: [torch.cuda.Event(enable_timing=True) for _ in range(3)] for k in sampled}
    seg_ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)] if nseg else []
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        if nseg and k in cuts[:5]:
            seg_ev[cuts.index(k)].record()
        e = smp.get(k)
        if e is not None:
            e[0].record()
        step(e[1] if e is not None else None)
        if e is not None:
            e[2].record()
    if nseg:
        seg_ev[5].record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    wall = max_over_ranks(t1 - t0, world)
    if long_k >= 5:
        rates = [steps_per_call * (cuts_l[j + 1] - cuts_l[j]) / (lev[j].elapsed_time(lev[j + 1]) * 1e-3)
                 for j in range(5)]
        long_region = dict(batches=long_k, seconds=lev[0].elapsed_time(lev[5]) * 1e-3, segment_rates=rates,
                           median=sum_over_ranks(float(np.median(rates)), world),
                           spread=float((max(rates) - min(rates)) / np.median(rates)))
    evs = [smp[k] for k in sampled]
    kern_ms = sum(e[0].elapsed_time(e[2]) for e in evs) / len(evs)
    seq_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs)
    # the timed region in 5 consecutive segments (HIP events at their boundaries): per-segment rate
    # and the median of the 5, beside the whole-region value
    seg = None
    if nseg:
        rates = [steps_per_call * (cuts[j + 1] - cuts[j]) / (seg_ev[j].elapsed_time(seg_ev[j + 1]) * 1e-3)
                 for j in range(5)]
        seg = dict(n=5, items_per_segment=K // 5, rates=rates, median=float(np.median(rates)),
                   spread=float((max(rates) - min(rates)) / np.median(rates)))
    return dict(out=out, S0=S0, nsteps=nsteps, T=T, wall=wall, kernel_ms=kern_ms, seq_kernel_ms=seq_ms,
                seq_kernel_ms_median=float(np.median([e[0].elapsed_time(e[1]) for e in evs])),
                kernel_ms_samples=len(evs), rewards_kernel_ms=kern_ms - seq_ms, steps_per_call=steps_per_call,
                total_steps=sum_over_ranks(steps_per_call * K, world), segments=seg, long_region=long_region)


def rollout_diagnostics(rl, conf, roll, K=5):
    """Kernel time of variants of the same rollout batch: states+actions only (create_TO_init
    outputs), zero controls (ep == 0: dynamics/reward/EE only)."""
    T = roll["T"]
    inputs = rl.rollout_inputs(roll["S0"], roll["nsteps"])
    out = roll["out"]
    res = {}
    for name, o, ep in (("states_actions_only", {"S": out["S"], "A": out["A"]}, 1),
                        ("ep0_zero_controls", out, 0)):
        rl.rollout_batch(None, None, T, ep=ep, inputs=inputs, out=o)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            rl.rollout_batch(None, None, T, ep=ep, inputs=inputs, out=o)
        e1.record()
        torch.cuda.synchronize()
        res[name + "_kernel_ms"] = e0.elapsed_time(e1) / K
    return res


def terminal_rewards(env, conf, roll):
    """rwrd_arr[-1] = env.reward(cost_weights_terminal, s_T) per episode (RL.py:165), on the device."""
    S, n = roll["out"]["S"], torch.as_tensor(roll["nsteps"].astype(np.int64), device="cuda")
    s_T = S[torch.arange(S.shape[0], device="cuda"), n]
    return env.step_batch(s_T, torch.zeros(S.shape[0], conf.nb_action, dtype=torch.float64, device="cuda"),
                          conf.cost_weights_terminal)[1]


def episode_groups(nsteps, max_rows):
    """Consecutive episode ranges of at most max_rows replay rows each."""
    groups, lo, rows = [], 0, 0
    for e, T in enumerate(nsteps):
        if rows + T + 1 > max_rows:
            groups.append((lo, e))
            lo, rows = e, 0
        rows += int(T) + 1
    groups.append((lo, len(nsteps)))
    return groups


def ddp_labels(rl, conf, env, roll, K=5):
    """Sobolev labels dV/dx of every rollout episode by the DDP backward pass (TO.backward_pass,
    TO.py:119-202, cacto_ddp_backward) along the rollout trajectory — the stand-in for the TO
    solution the reference labels (the NLP solve is host-side CasADi, out of scope). Returns the
    labels [R, T+1, ns] f64 and its timing."""
    from cacto_amd.to import TO
    to = TO(env, conf, w_S=rl.w_S)
    S, A = roll["out"]["S"], roll["out"]["A"].double()
    n = torch.as_tensor(roll["nsteps"].astype(np.int32), device="cuda")
    out = to.backward_pass_batch(S, A, n)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K):
        to.backward_pass_batch(S, A, n, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / K
    steps = int(roll["nsteps"].sum())
    return out, dict(kernel="k_ddp_backward", ms_per_call=ms, episodes=len(roll["nsteps"]), riccati_steps=steps,
                     steps_per_s=steps / (ms * 1e-3), source="rollout trajectories (TO NLP solve is host-side)")


def fill_buffer(rl, conf, roll, env, seed, per=False, dVdx=None):
    """Replay rows from the rollouts on the device: RL_Solve n-step targets fused with the ring add
    (cacto_rl_solve_add), rewards = the rollout rewards + terminal reward, dVdx = the DDP labels
    when given, else synthetic N(0,1). Episodes go in groups of <= 8192 rows until the ring has
    wrapped once, so `full` latches."""
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer, ReplayBuffer
    buf = PrioritizedReplayBuffer(conf, rl.sys) if per else ReplayBuffer(conf, rl.sys)
    S, R, nsteps = roll["out"]["S"], roll["out"]["R"], roll["nsteps"]
    R_term = terminal_rewards(env, conf, roll)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(seed)
    added = 0
    while added < conf.REPLAY_SIZE + 8192:
        for lo, hi in episode_groups(nsteps, 8192):
            dV = dVdx[lo:hi] if dVdx is not None else torch.randn(hi - lo, S.shape[1], S.shape[2],
                                                                  dtype=torch.float64, device="cuda", generator=gen)
            buf.add_episodes(S[lo:hi], R[lo:hi], nsteps[lo:hi], R_term=R_term[lo:hi], dVdx=dV)
            added += int((nsteps[lo:hi] + 1).sum())
            if added >= conf.REPLAY_SIZE + 8192:
                break
    return buf


def episode_to_buffer_phase(rl, conf, roll, env, K, dVdx=None):
    """The whole rollout batch through cacto_rl_solve_add into one ring that holds it (RL_Solve +
    buffer.add for every episode of a create_TO_init batch). Returns rows/s and the kernel's
    algorithmic bandwidth: per row it reads s and dVdx (8*ns each) and r (8), writes 8*(3ns+3)."""
    from cacto_amd.replay_buffer import ReplayBuffer
    nsteps = roll["nsteps"]
    rows = int((nsteps + 1).sum())
    c = types.SimpleNamespace(**{k: getattr(conf, k) for k in dir(conf) if not k.startswith("__")})
    c.REPLAY_SIZE = rows
    buf = ReplayBuffer(c, rl.sys)
    S, R = roll["out"]["S"], roll["out"]["R"]
    R_term = terminal_rewards(env, conf, roll)
    dV = dVdx if dVdx is not None else torch.randn(S.shape, dtype=torch.float64, device="cuda")
    buf.add_episodes(S, R, nsteps, R_term=R_term, dVdx=dV)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K):
        buf.add_episodes(S, R, nsteps, R_term=R_term, dVdx=dV)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / K
    ns = conf.nb_state
    row_bytes = 8 * (2 * ns + 1) + 8 * (3 * ns + 3)
    return dict(rows_per_s=rows / (ms * 1e-3), rows_per_call=rows, ms_per_call=ms, episodes=len(nsteps),
                algorithmic_bytes_per_row=row_bytes, achieved_GBps=rows * row_bytes / (ms * 1e-3) / 1e9)


# untimed updates before each update phase's timed region, queued right before its barrier: the host
# work between phases (buffer fills, index draws) idles the GPU, and a few warm-up updates left the
# timed region's first segment below the settled rate (the rollout's timed region showed the same,
# DESIGN.md §6)
UPDATE_WARMUP = 200


def update_phase(rl, buf, B, K, W, world, seed):
    """K learn_and_update iterations (RL.py:101-118 each) on pre-drawn minibatch indices, as the
    package's learn_and_update runs them: one RL_AC.update_rows_n call (the critic step of update
    t+1 overlaps the actor step of update t; bit-identical to K sequential updates). With --graph
    (one rank) the K updates replay as one HIP graph of the sequential loop instead. With N > 1
    ranks each update is the data-parallel one (RCCL all-reduce of both gradients)."""
    W = max(W, UPDATE_WARMUP)
    gen = np.random.Generator(np.random.PCG64(seed))
    idx = torch.as_tensor(gen.integers(0, buf.max_idx(), size=(K + W, B)).astype(np.int32), device="cuda")
    if (world == 1 and not USE_GRAPH) or rl._dp:
        rl.update_rows_n(buf.storage, idx[:W])     # warm-up on the timed path (creates its stream)
    else:
        for i in range(W):
            rl.update_rows(buf.storage, idx[i])
    graph = rl.capture_updates(buf.storage, idx[W:]) if world == 1 and USE_GRAPH and not rl._dp else None
    cuts = [W + j * K // 5 for j in range(6)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    if graph is not None:
        graph.replay()
    else:
        # K updates, critic(t+1) overlapping actor(t), as 5 consecutive calls (segments for the median)
        for j in range(5):
            rl.update_rows_n(buf.storage, idx[cuts[j]:cuts[j + 1]])
            ev[j + 1].record()
    HOST["enqueue_s"] = time.perf_counter() - t0
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    wall = max_over_ranks(t1 - t0, world)
    seg = None if graph is not None else update_segments(ev, cuts)
    return wall, seg


def update_segments(ev, cuts):
    rates = [(cuts[j + 1] - cuts[j]) / (ev[j].elapsed_time(ev[j + 1]) * 1e-3) for j in range(5)]
    return dict(n=5, rates=rates, median=float(np.median(rates)),
                spread=float((max(rates) - min(rates)) / np.median(rates)))


# BASELINE.json configs[2..4] (per GPU): rollouts, minibatches, Sobolev weight, PER.
EXTRA = {
    "manipulator": dict(R=8192, batches=(64, 8192), w_S=0.0, per=False,
                        config="configs[2]: manipulator (3-DoF planar), batch 8192"),
    "car_park": dict(R=4096, batches=(64, 4096), w_S=0.0, per=True,
                     config="configs[3]: car_park, PER (alpha 0.6, beta 0.6), 4096 rollouts and B=4096 per GPU"),
    "ur5": dict(R=2048, batches=(64, 2048), w_S=1e-2, per=False,
                config="configs[4]: ur5 (6-DoF), Sobolev w-S=1e-2, 16384 rollouts / global batch over 8 GPUs "
                       "(2048 per GPU)"),
}


def per_loop(rl, world):
    """The PER update loop learn_and_update runs (RL.py:122-137 between checkpoint saves): one rank
    calls RL_AC.update_rows_n_per (cacto_update_n_per: sample -> update -> priorities, pipelined on
    two streams); N ranks (or one rank with an explicit RCCL group, the dp1 leg) call
    RL_AC.update_rows_n_per_dp (rl.py learn_and_update: each rank samples its shard against the
    union's (sum, min, rows), the paired critic/actor gradients all-reduced in two stages). None with
    --graph (the sequential loop replayed as one HIP graph)."""
    dp = world > 1 or rl._dp
    if USE_GRAPH and not dp:
        return None
    return rl.update_rows_n_per_dp if dp else rl.update_rows_n_per


def per_update_phase(rl, buf, B, K, W, world, seed):
    """learn_and_update with PER (RL.py:122-137): sample (stratified, IS weights) -> update ->
    priority update, with the per-step uniforms pre-drawn on the device, through the loop the
    product runs at this rank count (per_loop)."""
    W = max(W, UPDATE_WARMUP)
    gen = np.random.Generator(np.random.PCG64(seed))
    U = torch.as_tensor(gen.random((K + W, B)), device="cuda")
    loop = per_loop(rl, world)
    if loop is not None:
        loop(buf, U[:W])                    # warm-up on the timed path
    graph = rl.capture_updates(None, None, per_buffer=buf, uniforms=U[W:]) if loop is None else None
    cuts = [W + j * K // 5 for j in range(6)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    if graph is not None:
        graph.replay()
    else:
        for j in range(5):
            loop(buf, U[cuts[j]:cuts[j + 1]])       # sample -> update -> priorities, K/5 updates per call
            ev[j + 1].record()
    HOST["enqueue_s"] = time.perf_counter() - t0
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    seg = None if graph is not None else update_segments(ev, cuts)
    return max_over_ranks(t1 - t0, world), seg, ("graph" if loop is None else loop.__name__)


def extra_system(name, args, world, rank):
    cfg = EXTRA[name]
    conf, env, rl = make_learner(name, w_S=cfg["w_S"])
    if world > 1:
        rl.set_data_parallel(world)
    if cfg["per"]:
        conf.prioritized_replay_alpha = 0.6
    r = rollout_phase(rl, conf, env, cfg["R"], args.steps, args.warmup, world, rank)
    labels, ddp = ddp_labels(rl, conf, env, r)
    buf = fill_buffer(rl, conf, r, env, seed=rank, per=cfg["per"], dVdx=labels)
    if cfg["per"] and world > 1:
        buf.set_data_parallel(world)        # IS weights over the union of the ranks' shards
    ups = {}
    ns, na = conf.nb_state, conf.nb_action
    for B in cfg["batches"]:
        loop = None
        if cfg["per"]:
            conf.BATCH_SIZE = B
            wall, seg, loop = per_update_phase(rl, buf, B, args.update_steps, 3, world, seed=300 + rank)
        else:
            wall, seg = update_phase(rl, buf, B, args.update_steps, 3, world, seed=200 + rank)
        flop = B * world * ((9 if cfg["w_S"] else 6) * fc_flops(ns) + 3 * fa_flops(ns, na))
        ups["B=%d" % B] = dict(value=args.update_steps / wall, unit="critic-updates/s", global_batch=B * world, loop=loop,
                               ms_per_update=1e3 * wall / args.update_steps, segments=seg,
                               tflops=flop * args.update_steps / wall / 1e12,
                               mfma_frac=flop * args.update_steps / wall / (FP32_MFMA_PEAK * world))
    dp1 = None
    if DP1_GROUP is not None and name in ("car_park", "ur5"):
        dp1 = dp1_phase(rl, buf, cfg, args, ups["B=%d" % cfg["batches"][-1]])
    return dict(config=cfg["config"], env_steps_per_s=r["total_steps"] / r["wall"], rollouts_per_gpu=cfg["R"],
                rollout_kernel_ms=r["kernel_ms"], env_steps_per_launch=r["steps_per_call"], segments=r["segments"],
                long_region=r["long_region"],
                rollout_mfma_frac=r["steps_per_call"] * fa_flops(ns, na) / (r["seq_kernel_ms"] * 1e-3) /
                FP32_MFMA_PEAK,
                w_S=cfg["w_S"], per=cfg["per"], critic_updates=ups, ddp_labels=ddp, dp1_rccl=dp1)


# host time of the last timed update region's issue (before its closing synchronize)
HOST = {"enqueue_s": None}
# a one-rank RCCL process group (N = 1 runs, unless --no-dp1): the data-parallel update loops of
# configs[3] / configs[4] timed on one GPU
DP1_GROUP = None


def init_dp1_group():
    """One-rank 'nccl' (RCCL) group on this GPU, the setup of tests/test_gpu_dp.py's RCCL tests: with an
    explicit group RL_AC takes its data-parallel path (set_data_parallel) at world size 1."""
    import torch.distributed as dist
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % free_port(), rank=0, world_size=1,
                            device_id=torch.device("cuda", torch.cuda.current_device()))
    return dist.group.WORLD


def dp1_phase(rl, buf, cfg, args, pipelined):
    """The data-parallel update loop learn_and_update runs at N > 1 (RL_AC._update_rows_n_dp /
    update_rows_n_per_dp: per update the paired [critic t | actor t-1] gradient stages, two async
    RCCL all-reduces, the Adam steps; with PER the shard statistics all-gathered per sample) over a
    one-rank RCCL group, at the configuration's per-GPU batch, beside the single-rank pipelined rate
    of the same batch: the cost of the exchange path itself (host issue + collectives) without
    other ranks, and its host issue time per update. (Its HIP-graph form, RL_AC.capture_updates over
    RCCL, is not timed here: a capture as long as this loop trips the RCCL process group's watchdog,
    which polls an event recorded inside the capture.)"""
    B = cfg["batches"][-1]
    K = args.update_steps
    rl.set_data_parallel(1, DP1_GROUP)
    if cfg["per"]:
        buf.set_data_parallel(1, DP1_GROUP)     # the shard statistics all-gathered per sample
    try:
        if cfg["per"]:
            wall, seg, loop = per_update_phase(rl, buf, B, K, 3, 1, seed=400)
        else:
            wall, seg = update_phase(rl, buf, B, K, 3, 1, seed=400)
            loop = "_update_rows_n_dp"
        enq = HOST["enqueue_s"]
    finally:
        rl.set_data_parallel(1, None)
        if cfg["per"]:
            buf.set_data_parallel(1, None)
    rate = K / wall
    return dict(batch=B, loop=loop, updates_per_s=rate, ms_per_update=1e3 * wall / K, segments=seg,
                host_enqueue_us_per_update=1e6 * enq / K, pipelined_single_rank_updates_per_s=pipelined["value"],
                vs_pipelined=rate / pipelined["value"])


def cpu_baseline_rollout(conf, rl, roll, seconds):
    """The oracle's per-sample port (PLOT.rollout loop: float32 actor at batch 1 + float64 env.step),
    single core, on the first episodes of the same workload until `seconds` elapse."""
    from oracle import env as oenv
    from oracle import rollout as oroll
    oe = oenv.make_env(conf)
    actor = rl.actor_model.get_weights()
    steps, t0, e = 0, time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds and e < len(roll["S0"]):
        oroll.policy_rollout(oe, actor, roll["S0"][e], int(roll["nsteps"][e]))
        steps += int(roll["nsteps"][e])
        e += 1
    dt = time.perf_counter() - t0
    return dict(value=steps / dt, unit="env-steps/s", cores=1, kind="port",
                sample="%d of the %d episodes (%d env-steps, %.1f s), oracle/rollout.py policy_rollout"
                       % (e, len(roll["S0"]), steps, dt))


def cpu_baseline_rollout_vectorized(conf, rl, roll, seconds):
    """The same rollouts vectorised over episodes (oracle/rollout.py batched_policy_rollout_di):
    numpy float64 with its BLAS threads, on growing episode prefixes until `seconds` elapse."""
    from oracle import env as oenv
    from oracle import rollout as oroll
    oe = oenv.make_env(conf)
    actor = rl.actor_model.get_weights()
    S0, n = np.asarray(roll["S0"]), np.asarray(roll["nsteps"])
    steps, e, t0 = 0, 64, time.perf_counter()
    while True:
        steps += oroll.batched_policy_rollout_di(oe, actor, S0[:e], n[:e])[0]
        el = time.perf_counter() - t0
        if el >= seconds or e >= len(S0):
            break
        e = min(2 * e, len(S0))
    threads = None
    try:
        from threadpoolctl import threadpool_info
        threads = max((i.get("num_threads", 1) for i in threadpool_info()), default=1)
    except Exception:
        pass
    return dict(value=steps / el, unit="env-steps/s", cores=threads or 1, kind="port",
                sample="%d env-steps over episode prefixes up to %d of %d, %.1f s, numpy vectorised over episodes"
                       % (steps, e, len(S0), el))


def cpu_baseline_update(conf, rl, buf, B, seconds):
    from oracle import env as oenv
    from oracle import nn as onn
    oe = oenv.make_env(conf)
    norm = conf.state_norm_arr.astype(np.float64)
    rows = buf.storage[:4096].cpu().numpy()
    ns = conf.nb_state
    crit, tgt, act = rl.critic_model.get_weights(), rl.target_critic.get_weights(), rl.actor_model.get_weights()
    oc, oa = onn.KerasAdam(conf.CRITIC_LEARNING_RATE), onn.KerasAdam(conf.ACTOR_LEARNING_RATE)
    gen = np.random.default_rng(0)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        r = rows[gen.integers(0, len(rows), B)].astype(np.float32).astype(np.float64)
        g = onn.compute_critic_grad(crit, tgt, r[:, :ns], r[:, ns + 1:2 * ns + 1], r[:, ns:ns + 1],
                                    r[:, 2 * ns + 1:3 * ns + 1], r[:, 3 * ns + 1:3 * ns + 2], np.ones((B, 1)),
                                    rl.w_S, norm)[0]
        crit = oc.apply(crit, g)
        ga = onn.compute_actor_grad(oe, act, crit, r[:, :ns].astype(np.float32), r[:, 3 * ns + 2:], norm)
        act = oa.apply(act, ga)
        tgt = onn.soft_update(tgt, crit, conf.UPDATE_RATE)
        n += 1
    dt = time.perf_counter() - t0
    return dict(value=n / dt, unit="critic-updates/s", cores=1, kind="port", batch=B,
                sample="%d updates at B=%d in %.1f s (oracle/nn.py, numpy float64)" % (n, B, dt))


def host_info():
    """The host the CPU baselines ran on: CPU model, the cores this process may use, BLAS threads."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    blas = None
    try:
        from threadpoolctl import threadpool_info
        blas = [dict(api=i.get("internal_api"), threads=i.get("num_threads")) for i in threadpool_info()]
    except Exception:
        pass
    return dict(cpu_model=model, cores_available=len(os.sched_getaffinity(0)), blas=blas,
                omp_num_threads=os.environ.get("OMP_NUM_THREADS"))


def config0(args, rank, cpu_updates):
    """BASELINE configs[0]: single_integrator, seed 0, w_S = 0 — one main.py training iteration
    (main.py:216-243, ep = 0: EP_UPDATE = 200 episodes with zero warm-start controls, RL_Solve,
    buffer.add, learn_and_update of UPDATE_LOOPS[0] = 1000 updates at B = 128), from the reference's
    SI seed-0 initial weights. GPU: the package's path (one rollout launch, device labels and
    RL_Solve + ring add, pipelined update loop), timed whole. CPU (rank 0): oracle/cpu_ref.py with
    Pool(2) as main.py:219-225 runs it — episodes in full, `cpu_updates` updates measured and
    projected to 1000. TO_Solve (CasADi) is absent on both sides: the warm start stands in for it."""
    from cacto_amd.confs import load_conf
    from cacto_amd.environment import make_env
    from cacto_amd.neural_network import NN
    from cacto_amd.replay_buffer import ReplayBuffer
    from cacto_amd.rl import RL_AC
    conf = load_conf("single_integrator", fresh=True)
    conf.NNs_path = None
    env = make_env(conf)
    rl = RL_AC(env, NN(env, conf, w_S=0.0), conf)
    z = np.load(os.path.join(ROOT, "tests", "golden", "weights", "si_seed0_0.npz"))
    w = {k: [z["%s_%d" % (k, i)] for i in range(6 if k == "actor" else 10)] for k in ("actor", "critic")}
    res = {}
    for rep in range(2):            # the first pass warms the kernels / allocations up
        rl.setup_model(weights=w)
        random.seed(0)
        np.random.seed(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        S0 = np.array([env.reset() for _ in range(conf.EP_UPDATE)])
        n = np.array([conf.NSTEPS - int(s[-1] / conf.dt) for s in S0])
        keep = n > 0
        S0, n = S0[keep], n[keep]
        T = int(n.max())
        out = rl.rollout_batch(S0, n, T, ep=0, weights=conf.cost_weights_running)
        roll = dict(out=out, nsteps=n)
        R_term = terminal_rewards(env, conf, roll)
        buf = ReplayBuffer(conf)
        buf.add_episodes(out["S"], out["R"], n, R_term=R_term)      # w_S = 0: no labels needed
        counter = rl.learn_and_update(0, buf, 0)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        res = dict(iteration_s=t1 - t0, episodes=int(len(n)), env_steps=int(n.sum()), updates=int(counter),
                   batch=conf.BATCH_SIZE)
    out = {"config": "configs[0]: single_integrator, seed 0, w-S 0, nb-cpus 2 — one main.py iteration "
                     "(200 episodes + 1000 updates at B=128)", "gpu": res}
    if rank == 0 and not args.no_cpu_baseline:
        from oracle import cpu_ref
        c = cpu_ref.training_iteration("single_integrator", w, seed=0, nb_cpus=2, ep=0, update_sample=cpu_updates)
        c.update(kind="port", cores=2, sample="episodes in full on Pool(2); %d of the %d updates measured, "
                                               "projected" % (c["updates_measured"], c["update_loops"]))
        out["cpu"] = c
        out["speedup_vs_cpu"] = c["projected_iteration_s"] / res["iteration_s"]
    return out


def flat_summary(updates, upd_roof, extra, world):
    """Top-level scalar copies of the nested results (a record that keeps only the line's
    top-level scalars still carries the update rates, the update roofline and the configs[2..4]
    figures), plus what the distributed run actually was."""
    out = {"rccl_ranks": DIST["ranks"] if DIST["backend"] == "nccl" else None,
           "dist_backend": DIST["backend"], "devices": DIST["devices"] if world > 1 else 1}
    for k, u in (updates or {}).items():
        b = k.split("=")[1]
        out["di_updates_per_s_b%s" % b] = u["value"]
        out["di_update_mfma_frac_b%s" % b] = u["mfma_frac"]
    if upd_roof:
        out["update_mfma_frac"] = upd_roof["mfma_frac"]
        out["update_counter_over_algorithmic"] = upd_roof["counter_over_algorithmic"]
    for name, e in (extra or {}).items():
        out["%s_env_steps_per_s" % name] = e["env_steps_per_s"]
        out["%s_rollout_mfma_frac" % name] = e["rollout_mfma_frac"]
        for k, u in e["critic_updates"].items():
            b = k.split("=")[1]
            out["%s_updates_per_s_b%s" % (name, b)] = u["value"]
            out["%s_update_mfma_frac_b%s" % (name, b)] = u["mfma_frac"]
        d = e.get("dp1_rccl")
        if d:
            pre = "dp1_rccl_%s_b%d_" % (name, d["batch"])
            out[pre + "updates_per_s"] = d["updates_per_s"]
            out[pre + "host_us_per_update"] = d["host_enqueue_us_per_update"]
            out[pre + "vs_pipelined"] = d["vs_pipelined"]
    return out


USE_GRAPH = False
LONG_STEPS = 1000


def main():
    global USE_GRAPH, LONG_STEPS
    args = parse()
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args))       # N rank processes of this script, one per GPU
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%s (a launcher started a different number of ranks)"
                 % (args.gpus, os.environ["WORLD_SIZE"]))
    if args.dry_run:
        return dry_run(args)
    USE_GRAPH = args.graph
    LONG_STEPS = args.long_steps
    world, rank = init_dist()
    torch.backends.cuda.matmul.allow_tf32 = False
    conf, env, rl = make_learner(args.system)
    if world > 1:
        rl.set_data_parallel(world)
    ns, na = conf.nb_state, conf.nb_action
    roll = rollout_phase(rl, conf, env, args.rollouts, args.steps, args.warmup, world, rank)
    value = roll["total_steps"] / roll["wall"]
    # the dominant kernel is the sequential pass (k_rollout); its own HIP-event time
    achieved = roll["steps_per_call"] * fa_flops(ns, na) / (roll["seq_kernel_ms"] * 1e-3)
    diag = None if args.no_diagnostics else rollout_diagnostics(rl, conf, roll)
    labels, ddp = ddp_labels(rl, conf, env, roll)
    buf = fill_buffer(rl, conf, roll, env, seed=rank, dVdx=labels)
    e2b = episode_to_buffer_phase(rl, conf, roll, env, 5, dVdx=labels)
    updates = {}
    for B in [int(b) for b in args.batches.split(",") if b]:
        K = args.update_steps
        wall, seg = update_phase(rl, buf, B, K, max(3, args.warmup), world, seed=100 + rank)
        flop = B * world * (9 * fc_flops(ns) + 3 * fa_flops(ns, na))
        updates["B=%d" % B] = dict(value=K / wall, unit="critic-updates/s", global_batch=B * world,
                                   ms_per_update=1e3 * wall / K, tflops=flop * K / wall / 1e12,
                                   mfma_frac=flop * K / wall / (FP32_MFMA_PEAK * world), segments=seg)
    # the two-stream update pipeline's ordering on this box (cacto_pipeline_status: the handle's
    # one-time concurrency probe) and its timeout latch, collected (a latched wait fails the run)
    from cacto_amd import _lib as L
    rl.check_pipeline()
    st = (ctypes.c_ulonglong * 4)()
    L.lib().call("cacto_pipeline_status", rl.sys.handle, st)
    pipe = {"ordering": {0: "not run", 1: "queue markers (probe: streams not concurrent)",
                         2: "device-side waits (probe: streams concurrent)"}[int(st[3])],
            "forced": os.environ.get("CACTO_PIPE_DEVWAIT")}
    extra = {}
    global DP1_GROUP
    if world == 1 and not args.no_dp1 and ("car_park" in args.extra_systems or "ur5" in args.extra_systems):
        DP1_GROUP = init_dp1_group()
    for sysname in [s for s in args.extra_systems.split(",") if s and s != args.system]:
        extra[sysname] = extra_system(sysname, args, world, rank)
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline_rollout(conf, rl, roll, args.cpu_seconds)
        cpu["update"] = cpu_baseline_update(conf, rl, buf, 128, args.cpu_seconds / 2)
        if args.system == "double_integrator":
            cpu["vectorized"] = cpu_baseline_rollout_vectorized(conf, rl, roll, args.cpu_seconds / 2)
    c0 = None if args.no_config0 else config0(args, rank, max(20, int(args.cpu_seconds * 20)))
    if cpu is not None:
        cpu["host"] = host_info()
    traffic, traffic_src = pmc_traffic()
    rw_traffic, _ = pmc_traffic("k_rollout_rewards<2>")
    n_ep = len(roll["nsteps"])
    roll_bytes = (roll["steps_per_call"] * (8 * ns + 4 * na + 8 + 24) + n_ep * (8 * ns + 24 + 8 * ns + 4)
                  + 4 * rl.actor_model.P)
    upd_roof = None
    upd_roofs = {}
    if updates:
        # per batch: SURVEY §8(d) algorithmic FLOP and bytes per update, against the measured rate and
        # the PMC counter bytes of its kernels; `update` (in the roofline object) is the first batch's
        # (the reference's B = 128)
        PA, PC = rl.actor_model.P, rl.critic_model.P
        for Bu in [int(b) for b in args.batches.split(",") if b]:
            u = updates["B=%d" % Bu]
            fl = Bu * world * (9 * fc_flops(ns) + 3 * fa_flops(ns, na)) + 12 * (PA + PC) + 3 * PC
            by = Bu * world * ((3 * ns + 3) * 4 + 8) + 36 * (PA + PC) + 12 * PC
            ctr, per, src = pmc_update_traffic(Bu)
            upd_roofs[Bu] = {"batch": Bu, "flop_per_update": fl, "algorithmic_bytes_per_update": by,
                             "ms_per_update": u["ms_per_update"],
                             "achieved_tflops": fl / (u["ms_per_update"] * 1e-3) / 1e12,
                             "mfma_frac": fl / (u["ms_per_update"] * 1e-3) / (FP32_MFMA_PEAK * world),
                             "counter_bytes_per_update": ctr, "counter_bytes_by_kernel": per,
                             "counter_over_algorithmic": (ctr / by) if ctr else None, "traffic_source": src}
        upd_roof = upd_roofs[[int(b) for b in args.batches.split(",") if b][0]]
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * roll["wall"] / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (MLP, MFMA) / f64 (dynamics)",
            "data": "synthetic: Env.reset initial states (random.seed(rank)), reference DI seed-0 weights, "
                    "dVdx labels from the DDP backward pass along the rollouts (cacto_ddp_backward)",
            "config": {"workload": "double_integrator, w-S=1e-2, %d rollouts per GPU (BASELINE configs[1])"
                                   % args.rollouts,
                       "system": args.system, "rollouts_per_gpu": args.rollouts,
                       "env_steps_per_rollout_batch": roll["steps_per_call"], "T_max": roll["T"],
                       "parallelism": "dp%d" % world},
            "segments": roll["segments"],
            "long_region": roll["long_region"],
            "roofline": {"kernel": "k_rollout (k_rollout_ks<2>: one slot per wave, layer 2 split over K, at this "
                                   "schedule)",
                         "bound": "mfma", "achieved": achieved / 1e12,
                         "peak": FP32_MFMA_PEAK / 1e12, "unit": "TFLOP/s", "frac": achieved / FP32_MFMA_PEAK,
                         "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                         "kernel_ms": roll["seq_kernel_ms"], "kernel_ms_samples": roll["kernel_ms_samples"],
                         "flop_per_env_step": fa_flops(ns, na),
                         "rollout_batch_ms": roll["kernel_ms"], "rewards_kernel_ms": roll["rewards_kernel_ms"],
                         "env_steps_per_launch": roll["steps_per_call"],
                         # bytes the batch (k_rollout + k_rollout_rewards) must move: per env step
                         # s_{t+1} (8 ns), a_t (4 na), r_t (8), EE (24) written; per episode s_0 read
                         # and written, EE_0, the length; the actor weights read once
                         "batch_algorithmic_bytes": roll_bytes,
                         "batch_traffic": (traffic + rw_traffic) if traffic and rw_traffic else None,
                         "batch_traffic_over_algorithmic": ((traffic + rw_traffic) / roll_bytes
                                                            if traffic and rw_traffic else None),
                         "update": upd_roof,
                         "update_by_batch": {str(k): v for k, v in upd_roofs.items()}},
            "critic_updates": updates,
            "update_pipeline": pipe,
            "episode_to_buffer": e2b,
            "ddp_labels": ddp,
            "rollout_diagnostics": diag,
            "cpu_baseline": cpu,
            "extra_systems": extra,
            "config0": c0,
        }
        line.update(flat_summary(updates, upd_roof, extra, world))
        for Bu, r in upd_roofs.items():     # flat per-batch copies (a record that keeps only scalars)
            line["di_update_counter_over_algorithmic_b%d" % Bu] = r["counter_over_algorithmic"]
            line["di_update_counter_bytes_b%d" % Bu] = r["counter_bytes_per_update"]
        print(json.dumps(line))
    if world > 1 or DP1_GROUP is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
