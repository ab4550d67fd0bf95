"""Data-parallel update logic on CPU (gloo, world size 2).

cacto_amd.rl.dp_update_step is the exchange/ordering logic RL_AC uses with RCCL on the GPUs. Here it
drives oracle gradients over two gloo ranks, each holding half of a global minibatch with losses
normalised by the GLOBAL batch. The result must equal one single-process update on the whole
batch (RL.py:101-118), and the two ranks must end with identical weights.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import env as oenv
from oracle import nn as onn
from tests.conftest import load_weights

B_GLOBAL = 16


def _rows(conf, rng):
    ns = conf.nb_state
    lo = np.asarray(conf.x_init_min, dtype=np.float64)
    hi = np.asarray(conf.x_init_max, dtype=np.float64)
    S = lo + (hi - lo) * rng.uniform(size=(B_GLOBAL, ns))
    Sn = lo + (hi - lo) * rng.uniform(size=(B_GLOBAL, ns))
    R = rng.normal(size=(B_GLOBAL, 1)) * 0.5
    dVdx = rng.normal(size=(B_GLOBAL, ns)) * 0.3
    d = (rng.uniform(size=(B_GLOBAL, 1)) < 0.3).astype(float)
    term = (rng.uniform(size=(B_GLOBAL, 1)) < 0.2).astype(float)
    return np.concatenate([S, R, Sn, dVdx, d, term], axis=1)


def _flat(ps):
    return torch.from_numpy(np.concatenate([np.asarray(p, dtype=np.float64).ravel() for p in ps]))


def _unflat(t, like):
    out, off = [], 0
    for p in like:
        n = int(np.prod(np.shape(p)))
        out.append(t[off:off + n].numpy().reshape(np.shape(p)))
        off += n
    return out


def _run_update(rows, world, all_reduce, n_steps=3, pipelined=True):
    """n_steps data-parallel updates on `rows` (this rank's shard), returning final weights.
    pipelined: RL_AC's schedule (cacto_amd.rl.dp_pipeline: one exchange per update, the critic step
    of update t beside the actor step of update t-1); else one update after the other
    (dp_update_step, RL.py:104-109 literally)."""
    from cacto_amd.confs import load_conf
    from cacto_amd.rl import dp_pipeline, dp_update_step
    conf = load_conf("double_integrator")
    oe = oenv.make_env(conf)
    w = load_weights("di_seed0_0")
    st = {"actor": [np.asarray(p, np.float64) for p in w["actor"]],
          "critic": [np.asarray(p, np.float64) for p in w["critic"]],
          "target": [np.asarray(p, np.float64) for p in w["target"]]}
    adam = {"critic": onn.KerasAdam(conf.CRITIC_LEARNING_RATE), "actor": onn.KerasAdam(conf.ACTOR_LEARNING_RATE)}
    norm = conf.state_norm_arr.astype(np.float64)
    ns = conf.nb_state
    S, R, Sn = rows[:, :ns], rows[:, ns:ns + 1], rows[:, ns + 1:2 * ns + 1]
    dVdx, d, term = rows[:, 2 * ns + 1:3 * ns + 1], rows[:, 3 * ns + 1:3 * ns + 2], rows[:, 3 * ns + 2:]
    scale = rows.shape[0] / float(B_GLOBAL)  # local-mean gradient -> share of the global mean

    def critic_grad():
        g = onn.compute_critic_grad(st["critic"], st["target"], S, Sn, R, dVdx, d, np.ones((S.shape[0], 1)), 1e-2,
                                    norm)[0]
        return _flat(g) * scale

    def actor_grad():
        g = onn.compute_actor_grad(oe, st["actor"], st["critic"], S.astype(np.float32), term, norm)
        return _flat(g) * scale

    def apply(which, g, soft):
        st[which] = adam[which].apply(st[which], _unflat(g, st[which]))
        if soft:
            st["target"] = onn.soft_update(st["target"], st["critic"], conf.UPDATE_RATE)

    if not pipelined:
        for _ in range(n_steps):
            dp_update_step(critic_grad, actor_grad, apply, all_reduce, soft_update=True)
        return {k: _flat(v).numpy() for k, v in st.items()}

    def stages(c, a):
        # each part is exchanged as soon as it is formed (dp_pipeline issues the all-reduce at the
        # yield), so the critic's exchange is in flight while the actor gradient is computed
        if c is not None:
            yield "critic", critic_grad()
        if a is not None:
            yield "actor", actor_grad()

    order = []

    def apply_part(which, step, g):
        order.append((which, step))
        apply(which, g, which == "critic")
    dp_pipeline(n_steps, stages, all_reduce, apply_part)
    # RL.py:104-109 per update: critic(t) before actor(t); actor(t-1) after critic(t-1)
    assert order == [("critic", 0)] + [x for t in range(1, n_steps) for x in (("critic", t), ("actor", t - 1))] + \
        [("actor", n_steps - 1)]
    return {k: _flat(v).numpy() for k, v in st.items()}


def _worker(rank, world, port, rows, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = rows.shape[0] // world
        out = _run_update(rows[rank * n:(rank + 1) * n], world, lambda t: dist.all_reduce(t, async_op=True))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_dp_update_equals_single_process():
    from cacto_amd.confs import load_conf
    rows = _rows(load_conf("double_integrator"), np.random.default_rng(7))
    ref = _run_update(rows, 1, lambda t: None, pipelined=False)   # the sequential reference order
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, rows, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in ("actor", "critic", "target"):
        assert np.array_equal(res[0][k], res[1][k]), k          # replicas stay identical
        np.testing.assert_allclose(res[0][k], ref[k], rtol=1e-9, atol=1e-12, err_msg=k)
    # and the update did move the weights
    w0 = load_weights("di_seed0_0")
    assert not np.allclose(ref["critic"], _flat(w0["critic"]).numpy())


# ------------------------------------------------------------------ PER over replay shards
def _per_shard(rank):
    from oracle import buffer as obuf
    rng = np.random.default_rng(100 + rank)
    o = obuf.PrioritizedReplayBuffer(1024, 5, 0.6, 0.6, 1e-2, 0.95, 32)
    n = 300 + 200 * rank                                   # shards of different fill
    for i, v in enumerate(rng.uniform(0.05, 3.0, size=n) ** 0.6):
        o.it_sum[i] = float(v)
        o.it_min[i] = float(v)
    o.next_idx = n
    u = rng.uniform(size=32)
    return o, o.sample_proportional(u)


def _per_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cacto_amd.replay_buffer import exchange_shard_stats
        o, idx = _per_shard(rank)
        stats = exchange_shard_stats(torch.from_numpy(o.shard_stats()), world, lambda out, t: dist.all_gather(out, t))
        w = o.sample_weights_global(idx, stats.numpy())
        q.put((rank, stats.numpy(), np.asarray(idx), w))
    finally:
        dist.destroy_process_group()


def test_per_shard_exchange_gives_union_weights():
    from oracle import buffer as obuf
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_per_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (st, idx, w)) for r, st, idx, w in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = [_per_shard(r)[0] for r in range(2)]
    expect = np.stack([s.shard_stats() for s in shards])
    for r in range(2):
        np.testing.assert_array_equal(res[r][0], expect)          # rank order, exact values
    # the union: each shard draws the same count, so P(i) = p_i / (G T_g) over N = N_0 + N_1 rows
    N = sum(s.max_idx() for s in shards)
    P = [np.array([s.it_sum[i] for i in range(s.max_idx())]) / (2 * s.it_sum.sum()) for s in shards]
    wmax = (N * min(p.min() for p in P)) ** -0.6
    for r in range(2):
        idx, w = res[r][1], res[r][2]
        np.testing.assert_allclose(w, (N * P[r][idx]) ** -0.6 / wmax, rtol=1e-12)
        assert np.all(w <= 1.0 + 1e-12)
    # one shard: exactly the single-buffer weights
    o, idx = _per_shard(0)
    o2, _ = _per_shard(0)
    np.testing.assert_array_equal(o.sample_weights_global(idx, o.shard_stats()[None]), o2.sample_weights(idx))


# ------------------------------------------------------------------ the configs' rank counts
# configs[3]: car_park with PER on 4 ranks (a replay shard per rank, IS weights over the union of
# the shards); configs[4]: UR5 with the Sobolev term (w_S = 1e-2) on 8 ranks at a global batch of
# 16,384 (2,048 per rank). Each rank runs the schedule RL_AC runs over RCCL (dp_pipeline: the
# critic gradient of update t beside the actor gradient of update t-1, each part all-reduced as
# soon as it is formed; with PER the stratified sample of update t after the priority update of
# t-1, as update_rows_n_per_dp orders it) on oracle gradients; a single process running the
# sequential loop (RL.py:101-137) at the global batch over all the shards is the reference.
CP_B, CP_K, CP_WORLD = 8, 3, 4
UR5_B, UR5_K, UR5_WORLD = 2048, 2, 8


def _init_params(conf, seed):
    rng = np.random.default_rng(seed)
    ns, na = conf.nb_state, conf.nb_action

    def lin(i, o, s):
        return [rng.uniform(-s, s, (i, o)), rng.uniform(-0.05, 0.05, o)]
    actor = lin(ns, 256, np.sqrt(6.0 / ns)) + lin(256, 256, np.sqrt(6.0 / 256)) + lin(256, na, 0.1 * np.sqrt(6.0 / 256))
    critic = (lin(ns, 64, 1.0 / ns) + lin(64, 64, np.sqrt(6.0 / 64)) + lin(64, 128, np.sqrt(6.0 / 64)) +
              lin(128, 128, np.sqrt(6.0 / 128)) + lin(128, 1, np.sqrt(6.0 / 128)))
    return actor, critic


class _Learner:
    """Replicated actor / critic / target on oracle gradients and the Keras Adam restatement."""

    def __init__(self, system, w_S, B_global):
        from cacto_amd.confs import load_conf
        self.conf = conf = load_conf(system)
        self.oe = oenv.make_env(conf)
        a, c = _init_params(conf, 5)
        self.st = {"actor": a, "critic": c, "target": [p.copy() for p in c]}
        self.adam = {"critic": onn.KerasAdam(conf.CRITIC_LEARNING_RATE), "actor": onn.KerasAdam(conf.ACTOR_LEARNING_RATE)}
        self.norm = conf.state_norm_arr.astype(np.float64)
        self.w_S, self.Bg = w_S, B_global

    def _split(self, rows):
        ns = self.conf.nb_state
        return (rows[:, :ns], rows[:, ns:ns + 1], rows[:, ns + 1:2 * ns + 1], rows[:, 2 * ns + 1:3 * ns + 1],
                rows[:, 3 * ns + 1:3 * ns + 2], rows[:, 3 * ns + 2:])

    def critic_grad(self, rows, w):
        S, R, Sn, dVdx, d, _ = self._split(rows)
        g, y, V, _, _ = onn.compute_critic_grad(self.st["critic"], self.st["target"], S, Sn, R, dVdx, d,
                                                np.asarray(w).reshape(-1, 1), self.w_S, self.norm)
        return _flat(g) * (rows.shape[0] / self.Bg), y, V       # local mean -> share of the global mean

    def actor_grad(self, rows):
        S, _, _, _, _, term = self._split(rows)
        g = onn.compute_actor_grad(self.oe, self.st["actor"], self.st["critic"], S.astype(np.float32), term, self.norm)
        return _flat(g) * (rows.shape[0] / self.Bg)

    def apply(self, which, g):
        self.st[which] = self.adam[which].apply(self.st[which], _unflat(g, self.st[which]))
        if which == "critic":
            self.st["target"] = onn.soft_update(self.st["target"], self.st["critic"], self.conf.UPDATE_RATE)

    def weights(self):
        return {k: _flat(v).numpy() for k, v in self.st.items()}


def _shard_rows(conf, n, seed):
    ns = conf.nb_state
    rng = np.random.default_rng(seed)
    lo = np.asarray(conf.x_init_min, dtype=np.float64)
    hi = np.asarray(conf.x_init_max, dtype=np.float64)
    S = lo + (hi - lo) * rng.uniform(size=(n, ns))
    Sn = lo + (hi - lo) * rng.uniform(size=(n, ns))
    return np.concatenate([S, rng.normal(size=(n, 1)) * 0.5, Sn, rng.normal(size=(n, ns)) * 0.3,
                           (rng.uniform(size=(n, 1)) < 0.3).astype(float),
                           (rng.uniform(size=(n, 1)) < 0.2).astype(float)], axis=1)


def _cp_shard(conf, rank):
    """Rank `rank`'s car_park replay shard: rows of a different fill per rank, leaves of assorted
    priorities (as after some updates), and the rank's own random.random() draws."""
    from oracle import buffer as obuf
    o = obuf.PrioritizedReplayBuffer(256, conf.nb_state, 0.6, 0.6, 1e-2, 0.95, CP_B)
    n = 90 + 40 * rank
    o.add_rows(_shard_rows(conf, n, 300 + rank))
    rng = np.random.default_rng(400 + rank)
    for i, p in enumerate(rng.uniform(0.05, 3.0, size=n)):
        o.it_sum[i] = float(p) ** 0.6
        o.it_min[i] = float(p) ** 0.6
    o.max_priority = 3.0
    return o, rng.uniform(size=(CP_K, CP_B))


def _shard_state(o):
    cap = o.it_sum.cap
    return dict(sum=np.array(o.it_sum.value[cap:]), min=np.array(o.it_min.value[cap:]),
                exp=o.exp_counter.copy(), maxp=o.max_priority)


def _per_rank(rank, world, all_gather, all_reduce):
    """update_rows_n_per_dp's schedule on one rank (car_park, PER)."""
    from cacto_amd.rl import dp_pipeline
    from cacto_amd.replay_buffer import exchange_shard_stats
    L = _Learner("car_park", 0.0, CP_B * world)
    o, U = _cp_shard(L.conf, rank)
    drawn, yv, idxs = {}, {}, []

    def stages(c, a):
        if c is not None:
            stats = exchange_shard_stats(torch.from_numpy(o.shard_stats()), world, all_gather).numpy()
            idx = o.sample_proportional(U[c])
            w = o.sample_weights_global(idx, stats)
            drawn[c] = idx
            idxs.append(idx.copy())
            g, y, V = L.critic_grad(o.storage[idx], w)
            yv[c] = (y, V)
            yield "critic", g
        if a is not None:
            yield "actor", L.actor_grad(o.storage[drawn[a]])

    def apply(which, step, g):
        L.apply(which, g)
        if which == "critic":                      # the priority update after the critic's Adam
            o.update_priorities(drawn[step], *yv[step])
    dp_pipeline(CP_K, stages, all_reduce, apply)
    return dict(weights=L.weights(), shard=_shard_state(o), idx=np.array(idxs))


def _per_reference(world):
    """One process, the sequential loop: per update every shard samples its B_local from its own
    tree with weights against the union, one update at the global batch, then the priorities."""
    L = _Learner("car_park", 0.0, CP_B * world)
    sh = [_cp_shard(L.conf, r) for r in range(world)]
    idxs = [[] for _ in range(world)]
    for t in range(CP_K):
        stats = np.stack([o.shard_stats() for o, _ in sh])
        parts = []
        for r, (o, U) in enumerate(sh):
            idx = o.sample_proportional(U[t])
            parts.append((idx, o.sample_weights_global(idx, stats)))
            idxs[r].append(idx.copy())
        rows = np.concatenate([o.storage[idx] for (o, _), (idx, _) in zip(sh, parts)])
        g, y, V = L.critic_grad(rows, np.concatenate([w for _, w in parts]))
        L.apply("critic", g)
        L.apply("actor", L.actor_grad(rows))
        for r, ((o, _), (idx, _)) in enumerate(zip(sh, parts)):
            o.update_priorities(idx, y[r * CP_B:(r + 1) * CP_B], V[r * CP_B:(r + 1) * CP_B])
    return L.weights(), [_shard_state(o) for o, _ in sh], [np.array(i) for i in idxs]


def _ur5_rank(rank, world, all_gather, all_reduce):
    """update_rows_n's data-parallel schedule on one rank (UR5, w_S = 1e-2, no PER)."""
    from cacto_amd.rl import dp_pipeline
    L = _Learner("ur5", 1e-2, UR5_B * world)
    rows = _shard_rows(L.conf, UR5_B * world, 77)[rank * UR5_B:(rank + 1) * UR5_B]
    w = np.ones(UR5_B)

    def stages(c, a):
        if c is not None:
            yield "critic", L.critic_grad(rows, w)[0]
        if a is not None:
            yield "actor", L.actor_grad(rows)
    dp_pipeline(UR5_K, stages, all_reduce, lambda which, step, g: L.apply(which, g))
    return dict(weights=L.weights())


def _ur5_reference(world):
    L = _Learner("ur5", 1e-2, UR5_B * world)
    rows = _shard_rows(L.conf, UR5_B * world, 77)
    for _ in range(UR5_K):
        L.apply("critic", L.critic_grad(rows, np.ones(len(rows)))[0])
        L.apply("actor", L.actor_grad(rows))
    return L.weights()


_RANK_FNS = {"per": _per_rank, "ur5": _ur5_rank}


def _generic_worker(rank, world, port, kind, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = _RANK_FNS[kind](rank, world, lambda out, t: dist.all_gather(out, t),
                              lambda t: dist.all_reduce(t, async_op=True))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _spawn(kind, world):
    """Start `world` gloo ranks of `kind`; returns a function that collects their results (the
    caller computes its reference meanwhile)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    old = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    os.environ.update(OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    try:
        procs = [ctx.Process(target=_generic_worker, args=(r, world, port, kind, q)) for r in range(world)]
        for p in procs:
            p.start()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v

    def collect():
        try:
            res = dict(q.get(timeout=600) for _ in procs)
            for p in procs:
                p.join(timeout=60)
                assert p.exitcode == 0
            return res
        finally:
            for p in procs:
                if p.is_alive():
                    p.kill()
    return collect


def _assert_weights(res, ref, world):
    for k in ("actor", "critic", "target"):
        for r in range(1, world):
            assert np.array_equal(res[r]["weights"][k], res[0]["weights"][k]), (k, r)   # replicas identical
        np.testing.assert_allclose(res[0]["weights"][k], ref[k], rtol=1e-9, atol=1e-12, err_msg=k)


def test_dp_per_car_park_ws4_equals_global_sampler():
    """configs[3] at its rank count: 4 ranks, one PER shard each (different fills), union IS
    weights, the pipelined DP schedule. Against the single-process global sampler: the same indices
    on every shard, the same exp_counter, trees and max_priority, and the same weights."""
    collect = _spawn("per", CP_WORLD)
    ref_w, ref_sh, ref_idx = _per_reference(CP_WORLD)
    res = collect()
    _assert_weights(res, ref_w, CP_WORLD)
    for r in range(CP_WORLD):
        np.testing.assert_array_equal(res[r]["idx"], ref_idx[r])
        got, exp = res[r]["shard"], ref_sh[r]
        np.testing.assert_array_equal(got["exp"], exp["exp"])
        # leaves float(p)**alpha of p = f32(fresh^n |y - V|) + eps: y, V differ from the reference
        # by the reassociated all-reduce sums only
        np.testing.assert_allclose(got["sum"], exp["sum"], rtol=1e-6)
        np.testing.assert_allclose(got["min"], exp["min"], rtol=1e-6)
        assert abs(got["maxp"] - exp["maxp"]) <= 1e-6 * exp["maxp"]
    # the priorities did move away from the initial leaves, and the shards drew different rows
    assert not np.allclose(ref_sh[0]["sum"], _shard_state(_cp_shard(_Learner("car_park", 0.0, 1).conf, 0)[0])["sum"])
    assert sum(s["exp"].sum() for s in ref_sh) == CP_WORLD * CP_K * CP_B - sum(
        len(i) - len(np.unique(i)) for idx in ref_idx for i in idx)


def test_dp_ur5_ws8_global_16384_equals_single_process():
    """configs[4] at its rank count: 8 ranks x 2,048 rows = the global batch of 16,384, UR5 with the
    Sobolev term, two pipelined DP updates against the single-process sequential loop."""
    collect = _spawn("ur5", UR5_WORLD)
    ref = _ur5_reference(UR5_WORLD)
    res = collect()
    _assert_weights(res, ref, UR5_WORLD)
