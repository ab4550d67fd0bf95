"""The HIP data-parallel update on the GPU (the ordering it keeps is RL.py:104-109):
two spawned ranks, both on cuda:0, exchanging over gloo (the driver's multi-GPU runs use RCCL, one
rank per GPU; the exchange code path — RL_AC.set_data_parallel + update_rows, the all-reduce of
the critic gradient before its Adam step and of the actor gradient after it — is the same).

  * RL_AC.update_rows with set_data_parallel(2), each rank on its half of the global minibatch,
    equals a single-rank update_rows at the global batch (the split only reassociates the sum over
    samples: float32 rounding of the gradient, so weights within Adam's 5e-6/step), and the two
    replicas end bit-identical.
  * PrioritizedReplayBuffer.sample_device with two replay shards: indices bit-exact against the
    oracle's per-shard sampler, IS weights against oracle.sample_weights_global over the union of
    the shards (the all-gathered (sum, min, rows) of both ranks).
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

K, B_LOCAL, WORLD = 4, 64, 2


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rows(n, seed):
    from cacto_amd.confs import load_conf
    conf = load_conf("double_integrator")
    rng = np.random.default_rng(seed)
    ns = conf.nb_state
    S = np.column_stack([rng.uniform(-15, 15, (n, ns - 1)), rng.uniform(0, 9.9, n)])
    Sn = np.column_stack([rng.uniform(-15, 15, (n, ns - 1)), rng.uniform(0, 9.9, n)])
    return np.concatenate([S, rng.normal(size=(n, 1)) * 0.5, Sn, rng.normal(size=(n, ns)) * 0.3,
                           (rng.uniform(size=(n, 1)) < 0.3).astype(float),
                           (rng.uniform(size=(n, 1)) < 0.2).astype(float)], axis=1)


def _sys_rows(conf, n, rng):
    """Replay rows [s | R | s' | dVdx | d | term] with states in the system's Env.reset box."""
    ns = conf.nb_state
    lo, hi = np.array(conf.x_init_min, dtype=float), np.array(conf.x_init_max, dtype=float)

    def states():
        S = rng.uniform(lo, hi, size=(n, ns))
        flat = np.where(hi[:-1] - lo[:-1] < 1e-12)[0]
        S[:, flat] = rng.uniform(-0.5, 0.5, size=(n, len(flat)))
        return S
    S, Sn = states(), states()
    return np.concatenate([S, rng.normal(size=(n, 1)) * 0.5, Sn, rng.normal(size=(n, ns)) * 0.3,
                           (rng.uniform(size=(n, 1)) < 0.3).astype(float),
                           (rng.uniform(size=(n, 1)) < 0.2).astype(float)], axis=1)


def _learner(world, system="double_integrator", w_S=1e-2):
    from conftest import load_weights
    from cacto_amd.confs import load_conf
    from cacto_amd.environment import make_env
    from cacto_amd.neural_network import NN
    from cacto_amd.rl import RL_AC
    conf = load_conf(system)
    env = make_env(conf)
    rl = RL_AC(env, NN(env, conf, w_S=w_S, seed=3), conf)
    rl.setup_model(weights=load_weights("di_seed0_0") if system == "double_integrator" else None)
    if world > 1:
        rl.set_data_parallel(world)
    return rl


def _state(rl):
    return [t.cpu().numpy().copy() for t in (rl.actor_model.buf, rl.critic_model.buf, rl.target_critic.buf,
                                             rl.actor_m, rl.actor_v, rl.critic_m, rl.critic_v)]


def _init(rank, port):
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=WORLD)
    return dist


def _update_worker(rank, port, rows, idx, q):
    dist = _init(rank, port)
    try:
        rl = _learner(WORLD)
        storage = torch.as_tensor(rows, device="cuda")
        for k in range(K):
            loc = idx[k, rank * B_LOCAL:(rank + 1) * B_LOCAL].astype(np.int32)
            rl.update_rows(storage, torch.as_tensor(loc, device="cuda"))
        torch.cuda.synchronize()
        # the K updates again as one pipelined call (one exchange per update: critic of t with actor of t-1)
        rp = _learner(WORLD)
        loc = np.ascontiguousarray(idx[:, rank * B_LOCAL:(rank + 1) * B_LOCAL].astype(np.int32))
        rp.update_rows_n(storage, torch.as_tensor(loc, device="cuda"))
        torch.cuda.synchronize()
        q.put((rank, _state(rl), rl.steps.cpu().tolist(), _state(rp), rp.steps.cpu().tolist()))
    finally:
        dist.destroy_process_group()


def _isw_worker(rank, port, rows, idx, wts, q):
    dist = _init(rank, port)
    try:
        rl = _learner(WORLD)
        storage = torch.as_tensor(rows, device="cuda")
        y = torch.empty(B_LOCAL, dtype=torch.float32, device="cuda")
        V = torch.empty_like(y)
        for k in range(K):
            sl = slice(rank * B_LOCAL, (rank + 1) * B_LOCAL)
            rl.update_rows(storage, torch.as_tensor(idx[k, sl].astype(np.int32), device="cuda"),
                           torch.as_tensor(wts[k, sl], device="cuda"), y, V)
        torch.cuda.synchronize()
        q.put((rank, _state(rl), y.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def _cfg_worker(rank, port, system, w_S, rows, idx, wts, q):
    dist = _init(rank, port)
    try:
        rl = _learner(WORLD, system, w_S)
        storage = torch.as_tensor(rows, device="cuda")
        b = idx.shape[1] // WORLD
        sl = slice(rank * b, (rank + 1) * b)
        y = torch.empty(b, dtype=torch.float32, device="cuda")
        V = torch.empty_like(y)
        for k in range(idx.shape[0]):
            w = torch.as_tensor(wts[k, sl], device="cuda") if wts is not None else None
            rl.update_rows(storage, torch.as_tensor(idx[k, sl].astype(np.int32), device="cuda"), w, y, V)
        torch.cuda.synchronize()
        q.put((rank, _state(rl), y.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def _per_worker(rank, port, q):
    dist = _init(rank, port)
    try:
        from cacto_amd.confs import load_conf
        from cacto_amd.replay_buffer import PrioritizedReplayBuffer
        conf = load_conf("double_integrator", fresh=True)
        conf.prioritized_replay_alpha = 0.6
        conf.BATCH_SIZE = B_LOCAL
        buf = PrioritizedReplayBuffer(conf)
        buf.set_data_parallel(WORLD)
        n_rows, leaves, u = _per_shard(rank)
        buf.add_rows(_rows(n_rows, 50 + rank))
        buf.set_leaves(np.arange(n_rows), leaves)
        idx, w = buf.sample_device(torch.as_tensor(u, device="cuda"))
        torch.cuda.synchronize()
        q.put((rank, idx.cpu().numpy(), w.cpu().numpy(), buf.exp_counter[:n_rows].cpu().numpy()))
    finally:
        dist.destroy_process_group()


def _per_loop_worker(rank, port, q):
    """The data-parallel PER loop two ways on this rank's shard: K sequential (sample -> update ->
    priorities) steps, and RL_AC.update_rows_n_per_dp (the paired, pipelined form)."""
    dist = _init(rank, port)
    try:
        from cacto_amd.confs import load_conf
        from cacto_amd.replay_buffer import PrioritizedReplayBuffer
        conf = load_conf("double_integrator", fresh=True)
        conf.prioritized_replay_alpha = 0.6
        conf.BATCH_SIZE = B_LOCAL
        rows = _rows(900 + 300 * rank, 90 + rank)
        U = np.random.default_rng(300 + rank).uniform(size=(K + 1, B_LOCAL))
        out = []
        for pipelined in (False, True):
            rl = _learner(WORLD)
            buf = PrioritizedReplayBuffer(conf, rl.sys)
            buf.set_data_parallel(WORLD)
            buf.add_rows(rows)
            if pipelined:
                rl.update_rows_n_per_dp(buf, torch.as_tensor(U, device="cuda"))
            else:
                y = torch.empty(B_LOCAL, dtype=torch.float32, device="cuda")
                V = torch.empty_like(y)
                for k in range(K + 1):
                    idx, w = buf.sample_device(torch.as_tensor(U[k], device="cuda"))
                    rl.update_rows(buf.storage, idx, w, y, V)
                    buf.update_priorities_device(idx, y, V)
            torch.cuda.synchronize()
            out.append((_state(rl), rl.steps.cpu().tolist(), buf.sum_tree.cpu().numpy(), buf.min_tree.cpu().numpy(),
                        buf.exp_counter.cpu().numpy(), float(buf.max_priority.item())))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _per_shard(rank):
    rng = np.random.default_rng(200 + rank)
    n_rows = 700 + 500 * rank                                # shards of different fill
    return n_rows, rng.uniform(0.05, 3.0, size=n_rows) ** 0.6, rng.uniform(size=B_LOCAL)


def _spawn(target, args_of_rank):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, port) + args_of_rank(r) + (q,)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        res = {}
        for _ in procs:
            item = q.get(timeout=240)
            res[item[0]] = item[1:]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    return res


def test_dp_update_on_gpu_equals_single_rank():
    rng = np.random.default_rng(61)
    N = 4096
    rows = _rows(N, 60)
    idx = rng.integers(0, N, size=(K, WORLD * B_LOCAL))
    res = _spawn(_update_worker, lambda r: (rows, idx))
    s0, s1 = res[0][0], res[1][0]
    for a, b in zip(s0, s1):
        assert np.array_equal(a, b)                          # replicas stay bit-identical
    assert res[0][1] == [K, K]
    for r in range(WORLD):                                   # pipelined DP loop == K single DP updates
        assert res[r][3] == [K, K]
        for a, b in zip(res[r][0], res[r][2]):
            assert np.array_equal(a, b)
    single = _learner(1)
    storage = torch.as_tensor(rows, device="cuda")
    for k in range(K):
        single.update_rows(storage, torch.as_tensor(idx[k].astype(np.int32), device="cuda"))
    torch.cuda.synchronize()
    ref = _state(single)
    for name, a, b in zip(("actor", "critic", "target"), s0[:3], ref[:3]):
        P = single.actor_model.P if name == "actor" else single.critic_model.P
        err = np.abs(a[:P] - b[:P]).max()
        assert err < 5e-6 * K, (name, err)
    # the exchange mattered: a rank's update on its half alone is measurably different
    alone = _learner(1)
    for k in range(K):
        alone.update_rows(storage, torch.as_tensor(idx[k, :B_LOCAL].astype(np.int32), device="cuda"))
    P = alone.critic_model.P
    assert np.abs(alone.critic_model.buf.cpu().numpy()[:P] - s0[1][:P]).max() > 20 * 5e-6 * K


def test_dp_per_shards_on_gpu_match_oracle():
    from oracle import buffer as obuf
    res = _spawn(_per_worker, lambda r: ())
    shards = []
    for r in range(WORLD):
        n_rows, leaves, u = _per_shard(r)
        o = obuf.PrioritizedReplayBuffer(65536, 5, 0.6, 0.6, 1e-2, 0.95, B_LOCAL)
        for i, v in enumerate(leaves):
            o.it_sum[i] = float(v)
            o.it_min[i] = float(v)
        o.next_idx = n_rows
        shards.append((o, u))
    stats = np.stack([o.shard_stats() for o, _ in shards])
    for r, (o, u) in enumerate(shards):
        idx, w, cnt = res[r]
        oidx = o.sample_proportional(u)
        np.testing.assert_array_equal(idx, oidx)
        ow = o.sample_weights_global(oidx, stats)
        np.testing.assert_allclose(w, ow.astype(np.float32), rtol=1e-6)
        np.testing.assert_array_equal(cnt, o.exp_counter[:len(cnt)])


def test_dp_update_with_is_weights_on_gpu():
    """The data-parallel update with per-sample IS weights (the PER path of learn_and_update,
    replay_buffer.py:159-188 weights into NeuralNetwork.py:167-173): equals a single-rank weighted
    update at the global batch, replicas bit-identical, and each rank's y / V outputs are its own
    samples' (the priority update reads them)."""
    rng = np.random.default_rng(71)
    N = 4096
    rows = _rows(N, 70)
    idx = rng.integers(0, N, size=(K, WORLD * B_LOCAL))
    wts = rng.uniform(0.2, 1.0, size=(K, WORLD * B_LOCAL)).astype(np.float32)
    res = _spawn(_isw_worker, lambda r: (rows, idx, wts))
    for a, b in zip(res[0][0], res[1][0]):
        assert np.array_equal(a, b)
    single = _learner(1)
    storage = torch.as_tensor(rows, device="cuda")
    y = torch.empty(WORLD * B_LOCAL, dtype=torch.float32, device="cuda")
    V = torch.empty_like(y)
    for k in range(K):
        single.update_rows(storage, torch.as_tensor(idx[k].astype(np.int32), device="cuda"),
                           torch.as_tensor(wts[k], device="cuda"), y, V)
    torch.cuda.synchronize()
    ref = _state(single)
    for name, a, b in zip(("actor", "critic", "target"), res[0][0][:3], ref[:3]):
        P = single.actor_model.P if name == "actor" else single.critic_model.P
        assert np.abs(a[:P] - b[:P]).max() < 5e-6 * K, name
    # y of the last update: rank r's half of the global batch (y depends only on the target critic
    # and the rows, identical on every rank and in the single-rank run up to the target's rounding)
    yg = y.cpu().numpy()
    for r in range(WORLD):
        np.testing.assert_allclose(res[r][1], yg[r * B_LOCAL:(r + 1) * B_LOCAL], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("system,w_S,B,weighted", [("car_park", 0.0, 4096, True),
                                                  ("ur5", 1e-2, 2048, False)])
def test_dp_baseline_configs_on_gpu(system, w_S, B, weighted):
    """configs[3] (car_park, PER IS weights, global batch 4096) and configs[4] (UR5, Sobolev
    w-S=1e-2, batch 2048 per GPU) through the data-parallel exchange: two ranks on their halves
    equal one rank at the global batch (float32 reassociation of the sample sum only), replicas end
    bit-identical, and each rank's y / V are its own samples'."""
    from cacto_amd.confs import load_conf
    K2 = 2
    conf = load_conf(system)
    rng = np.random.default_rng(81)
    N = 2 * B
    rows = _sys_rows(conf, N, rng)
    idx = rng.integers(0, N, size=(K2, B))
    wts = rng.uniform(0.2, 1.0, size=(K2, B)).astype(np.float32) if weighted else None
    res = _spawn(_cfg_worker, lambda r: (system, w_S, rows, idx, wts))
    for a, b in zip(res[0][0], res[1][0]):
        assert np.array_equal(a, b)
    single = _learner(1, system, w_S)
    storage = torch.as_tensor(rows, device="cuda")
    y = torch.empty(B, dtype=torch.float32, device="cuda")
    V = torch.empty_like(y)
    for k in range(K2):
        w = torch.as_tensor(wts[k], device="cuda") if weighted else None
        single.update_rows(storage, torch.as_tensor(idx[k].astype(np.int32), device="cuda"), w, y, V)
    torch.cuda.synchronize()
    ref = _state(single)
    for name, a, b in zip(("actor", "critic", "target"), res[0][0][:3], ref[:3]):
        P = single.actor_model.P if name == "actor" else single.critic_model.P
        assert np.abs(a[:P] - b[:P]).max() < 5e-6 * K2, name
    yg = y.cpu().numpy()
    h = B // WORLD
    for r in range(WORLD):
        np.testing.assert_allclose(res[r][1], yg[r * h:(r + 1) * h], rtol=1e-5, atol=1e-5)


def test_dp_per_loop_pipelined_equals_sequential():
    """learn_and_update's data-parallel PER branch (RL.py:122-137, replay_buffer.py:139-218 on
    each rank's shard): the paired pipeline (one shard-stats all-gather and one gradient all-reduce
    per update, uniforms pre-drawn and copied once) equals the sequential sample -> update ->
    priority-update loop bit for bit on every rank — weights, moments, counters, both trees,
    exp_counter, max_priority — and the replicas' weights stay identical."""
    res = _spawn(_per_loop_worker, lambda r: ())
    for r in range(WORLD):
        seq, pip = res[r][0]
        for a, b in zip(seq[0], pip[0]):
            assert np.array_equal(a, b)
        assert seq[1] == pip[1] == [K + 1, K + 1]
        for a, b in zip(seq[2:5], pip[2:5]):
            assert np.array_equal(a, b)
        assert seq[5] == pip[5]
    for a, b in zip(res[0][0][1][0], res[1][0][1][0]):
        assert np.array_equal(a, b)
    # the shards differ (each rank's own rows and priorities)
    assert not np.array_equal(res[0][0][1][2], res[1][0][1][2])


def _host_loop_learner(group):
    """A learner whose data-parallel updates run the host loop dp_pipeline (torch.distributed
    collectives) instead of the library's RCCL pipeline."""
    rl = _learner(1)
    os.environ["CACTO_DP_NATIVE"] = "0"
    try:
        rl.set_data_parallel(1, group)
    finally:
        del os.environ["CACTO_DP_NATIVE"]
    assert not rl._dp_native
    return rl


def _rccl_worker(rank, port, rows, idx, q):
    """One rank over RCCL (backend 'nccl'): the exchange path of RL_AC (an explicit process group
    selects it at world size 1) — the library's pipeline (cacto_update_n_dp) eager and captured into
    a HIP graph, and the host loop dp_pipeline."""
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    try:
        storage = torch.as_tensor(rows, device="cuda")
        ix = torch.as_tensor(idx.astype(np.int32), device="cuda")
        single = _learner(1)
        single.update_rows_n(storage, ix)                     # the one-rank pipeline (no exchange)
        eager = _learner(1)
        eager.set_data_parallel(1, dist.group.WORLD)
        assert eager._dp_native
        eager.update_rows_n(storage, ix)                      # cacto_update_n_dp, RCCL all-reduces
        host = _host_loop_learner(dist.group.WORLD)
        host.update_rows_n(storage, ix)                       # dp_pipeline, torch.distributed all-reduces
        graphed = _learner(1)
        graphed.set_data_parallel(1, dist.group.WORLD)
        g = graphed.capture_updates(storage, ix)
        g.replay()
        torch.cuda.synchronize()
        first = (_state(single), _state(eager), _state(graphed), _state(host), graphed.steps.cpu().tolist())
        eager.update_rows_n(storage, ix)                      # a second replay continues from the new state
        g.replay()
        torch.cuda.synchronize()
        q.put((0, first, _state(eager), _state(graphed), graphed.steps.cpu().tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [128, 1024])
def test_dp_loop_over_rccl_is_graph_capturable(B):
    """The data-parallel K-step loop over RCCL — the library's pipeline (cacto_update_n_dp: the
    two-stream pipeline, each network's gradient all-reduced on its stream's communicator between
    its GEMM and its Adam step) and the host loop dp_pipeline (staged gradients, torch.distributed
    all-reduces) — captured into one HIP graph: replays equal the eager loop bit for bit, and at
    one rank (the exchange is the identity) both loops equal the single-rank pipeline. B = 128: the
    4-sample-tile chains; 1024: the 16-sample ones. The multi-GPU driver runs the same code with
    world size N."""
    import torch.multiprocessing as mp
    rng = np.random.default_rng(91)
    N = 4096
    rows = _rows(N, 92)
    idx = rng.integers(0, N, size=(6, B))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(0, _free_port(), rows, idx, q))
    p.start()
    try:
        _, first, eager2, graphed2, steps2 = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert p.exitcode == 0
    single, eager, graphed, host, steps = first
    assert steps == [6, 6] and steps2 == [12, 12]
    for a, b, c, d in zip(single, eager, graphed, host):
        assert np.array_equal(a, b) and np.array_equal(b, c) and np.array_equal(c, d)
    for a, b in zip(eager2, graphed2):
        assert np.array_equal(a, b)


def _rccl_per_worker(rank, port, rows, U, q):
    """One rank over RCCL: the data-parallel PER loop (update_rows_n_per_dp: shard-stats
    all-gather, stratified sample, gradients, priority updates) in the library (eager and
    captured), the host loop, and the single-rank pipelined PER loop."""
    import torch.distributed as dist
    from cacto_amd.confs import load_conf
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    try:
        conf = load_conf("double_integrator", fresh=True)
        conf.prioritized_replay_alpha = 0.6
        conf.BATCH_SIZE = U.shape[1]
        out = []
        for mode in ("eager", "graphed", "host", "single"):
            rl = _host_loop_learner(dist.group.WORLD) if mode == "host" else _learner(1)
            if mode in ("eager", "graphed"):
                rl.set_data_parallel(1, dist.group.WORLD)
            buf = PrioritizedReplayBuffer(conf, rl.sys)
            if mode != "single":
                buf.set_data_parallel(1, dist.group.WORLD)
            buf.add_rows(rows)
            Ud = torch.as_tensor(U, device="cuda")
            if mode == "graphed":
                g = rl.capture_updates(None, None, per_buffer=buf, uniforms=Ud)
                g.replay()
            elif mode == "single":
                rl.update_rows_n_per(buf, Ud)
            else:
                rl.update_rows_n_per_dp(buf, Ud)
            torch.cuda.synchronize()
            out.append((_state(rl), rl.steps.cpu().tolist(), buf.sum_tree.cpu().numpy(), buf.min_tree.cpu().numpy(),
                        buf.exp_counter.cpu().numpy(), float(buf.max_priority.item())))
        q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [64, 1024])
def test_dp_per_loop_over_rccl_is_graph_capturable(B):
    """capture_updates(per_buffer=...) of the data-parallel PER loop over RCCL (one rank): the
    replayed graph equals the eager update_rows_n_per_dp bit for bit — weights, moments, counters,
    both trees, exp_counter, max_priority — and so do the host loop and, at one rank, the
    single-rank pipelined PER loop (cacto_update_n_per)."""
    import torch.multiprocessing as mp
    rows = _rows(3000, 93)
    U = np.random.default_rng(94).uniform(size=(5, B))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_per_worker, args=(0, _free_port(), rows, U, q))
    p.start()
    try:
        runs = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert p.exitcode == 0
    eager = runs[0]
    for other in runs[1:]:
        assert eager[1] == other[1] == [5, 5]
        for a, b in zip(eager[0], other[0]):
            assert np.array_equal(a, b)
        for a, b in zip(eager[2:5], other[2:5]):
            assert np.array_equal(a, b)
        assert eager[5] == other[5]
