"""The update loop replayed as one HIP graph (RL_AC.capture_updates), and the pipelined K-update
call (RL_AC.update_rows_n / cacto_update_n), do exactly what the eager loop does: bit-identical
weights, Adam moments and optimiser counters after K updates."""
import os

import numpy as np
import pytest
import torch

from cacto_amd.confs import load_conf
from cacto_amd.environment import make_env
from cacto_amd.neural_network import NN
from cacto_amd.rl import RL_AC

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "weights")


def _learner(conf, env):
    z = np.load(os.path.join(GOLD, "di_seed0_0.npz"))
    w = {k: [z["%s_%d" % (k, i)] for i in range(6 if k == "actor" else 10)] for k in ("actor", "critic", "target")}
    rl = RL_AC(env, NN(env, conf, w_S=1e-2), conf)
    rl.setup_model(weights=w)
    return rl


def _state(rl):
    return [t.clone() for t in (rl.actor_model.buf, rl.critic_model.buf, rl.target_critic.buf, rl.actor_m,
                                rl.actor_v, rl.critic_m, rl.critic_v, rl.steps)]


def test_graph_replay_equals_eager_updates():
    conf = load_conf("double_integrator", fresh=True)
    env = make_env(conf)
    ns = conf.nb_state
    rng = np.random.default_rng(5)
    N, B, K = 2048, 128, 6
    S = np.column_stack([rng.uniform(-15, 15, (N, 4)), rng.uniform(0, 9.9, N)])
    rows = np.concatenate([S, rng.normal(size=(N, 1)), S + 0.05, rng.normal(size=(N, ns)) * 0.3,
                           (rng.uniform(size=(N, 1)) < 0.1).astype(float), (rng.uniform(size=(N, 1)) < 0.1)
                           .astype(float)], axis=1)
    storage = torch.as_tensor(rows, device="cuda")
    idx = torch.as_tensor(rng.integers(0, N, size=(K, B)).astype(np.int32), device="cuda")
    eager = _learner(conf, env)
    for k in range(K):
        eager.update_rows(storage, idx[k])
    graphed = _learner(conf, env)
    g = graphed.capture_updates(storage, idx)
    before = _state(graphed)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(before, _state(_learner(conf, env))))  # capture ran nothing
    g.replay()
    torch.cuda.synchronize()
    for a, b in zip(_state(eager), _state(graphed)):
        assert torch.equal(a, b)
    assert int(graphed.steps[0]) == K and int(graphed.steps[1]) == K


def test_graph_replay_equals_eager_updates_with_per():
    """learn_and_update with PER (RL.py:122-137): sample -> update -> priority update, replayed as one
    graph, leaves the weights, the sum / min trees and the experience counters as the eager loop."""
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    conf = load_conf("double_integrator", fresh=True)
    conf.prioritized_replay_alpha = 0.6
    env = make_env(conf)
    ns = conf.nb_state
    rng = np.random.default_rng(9)
    N, B, K = 3000, 64, 5
    S = np.column_stack([rng.uniform(-15, 15, (N, 4)), rng.uniform(0, 9.9, N)])
    rows = np.concatenate([S, rng.normal(size=(N, 1)), S + 0.05, rng.normal(size=(N, ns)) * 0.3,
                           np.zeros((N, 1)), np.zeros((N, 1))], axis=1)
    U = torch.as_tensor(rng.uniform(size=(K, B)), device="cuda")

    def setup():
        rl = _learner(conf, env)
        buf = PrioritizedReplayBuffer(conf, env.sys)
        buf.add_rows(rows)
        return rl, buf
    eager, ebuf = setup()
    y = torch.empty(B, dtype=torch.float32, device="cuda")
    V = torch.empty_like(y)
    for k in range(K):
        idx, w = ebuf.sample_device(U[k])
        eager.update_rows(ebuf.storage, idx, w, y, V)
        ebuf.update_priorities_device(idx, y, V)
    graphed, gbuf = setup()
    g = graphed.capture_updates(None, None, per_buffer=gbuf, uniforms=U)
    g.replay()
    torch.cuda.synchronize()
    for a, b in zip(_state(eager), _state(graphed)):
        assert torch.equal(a, b)
    for name in ("sum_tree", "min_tree", "exp_counter"):
        assert torch.equal(getattr(ebuf, name), getattr(gbuf, name)), name


def test_captured_two_stream_pipeline_replays_equal_eager_calls():
    """cacto_update_n above the paired threshold (B = 1024: the two-stream pipeline) captured into a
    graph and replayed twice equals two eager calls bit for bit. The device-side waits compare device
    counters with absolute targets baked into the launches, so a replay would find its targets
    already reached: while the stream is being captured the pipeline orders its streams
    with queue markers instead."""
    conf = load_conf("double_integrator", fresh=True)
    env = make_env(conf)
    ns = conf.nb_state
    rng = np.random.default_rng(21)
    N, B, K = 6000, 1024, 5
    S = np.column_stack([rng.uniform(-15, 15, (N, 4)), rng.uniform(0, 9.9, N)])
    rows = np.concatenate([S, rng.normal(size=(N, 1)), S + 0.05, rng.normal(size=(N, ns)) * 0.3,
                           (rng.uniform(size=(N, 1)) < 0.1).astype(float), np.zeros((N, 1))], axis=1)
    storage = torch.as_tensor(rows, device="cuda")
    idx = torch.as_tensor(rng.integers(0, N, size=(K, B)).astype(np.int32), device="cuda")
    graphed = _learner(conf, env)
    graphed.update_rows_n(storage, idx[:1])        # the handle's side stream, probe and workspace first
    torch.cuda.synchronize()
    ref = _learner(conf, env)
    ref.update_rows_n(storage, idx[:1])
    ref.update_rows_n(storage, idx)
    ref.update_rows_n(storage, idx)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            graphed.update_rows_n(storage, idx)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    for a, b in zip(_state(ref), _state(graphed)):
        assert torch.equal(a, b)
    assert int(graphed.steps[0]) == 2 * K + 1
    graphed.check_pipeline()
    ref.check_pipeline()


@pytest.mark.parametrize("system,B,K,MC", [("double_integrator", 128, 7, 0), ("double_integrator", 1000, 7, 0),
                                         ("manipulator", 64, 7, 0), ("double_integrator", 128, 1, 0),
                                         ("double_integrator", 128, 2, 0), ("double_integrator", 128, 8, 0),
                                         ("double_integrator", 128, 8, 1), ("double_integrator", 256, 3, 1),
                                         ("car_park", 200, 5, 0), ("double_integrator", 512, 3, 0),
                                         ("double_integrator", 520, 2, 0), ("ur5", 48, 3, 0)])
def test_pipelined_updates_equal_sequential(system, B, K, MC):
    """cacto_update_n overlaps critic(t+1) with actor(t): for B <= 512 as one paired grid per step on
    one stream, above on two streams; either way the result is the same bits. Two streams: odd K
    ends with the critic in the workspace copy (copied back), even K in the caller's buffer; K = 1, 2
    finish before the first two-updates-old wait. MC = 1 has no soft target update. B = 200 and 48
    leave a partial last tile; 512 / 520 sit either side of the paired / two-stream threshold."""
    conf = load_conf(system, fresh=True)
    conf.MC = MC
    env = make_env(conf)
    ns = conf.nb_state
    rng = np.random.default_rng(11)
    N = 4096
    S = np.column_stack([rng.uniform(-3, 3, (N, ns - 1)), rng.uniform(0, 4.9, N)])
    rows = np.concatenate([S, rng.normal(size=(N, 1)), S + 0.01, rng.normal(size=(N, ns)) * 0.3,
                           (rng.uniform(size=(N, 1)) < 0.1).astype(float), (rng.uniform(size=(N, 1)) < 0.1)
                           .astype(float)], axis=1)
    storage = torch.as_tensor(rows, device="cuda")
    idx = torch.as_tensor(rng.integers(0, N, size=(K, B)).astype(np.int32), device="cuda")

    def learner():
        rl = RL_AC(env, NN(env, conf, w_S=1e-2 if system in ("double_integrator", "ur5") else 0.0, seed=3), conf)
        rl.setup_model()
        return rl
    seq = learner()
    for k in range(K):
        seq.update_rows(storage, idx[k])
    pipe = learner()
    pipe.update_rows_n(storage, idx)
    torch.cuda.synchronize()
    for a, b in zip(_state(seq), _state(pipe)):
        assert torch.equal(a, b)
    assert int(pipe.steps[0]) == K and int(pipe.steps[1]) == K


def test_pipelined_per_updates_equal_sequential():
    """cacto_update_n_per: sample -> update -> priority update per step, pipelined, equals the
    sequential PER loop bit for bit (weights, moments, counters, trees, experience counters)."""
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    conf = load_conf("car_park", fresh=True)
    conf.prioritized_replay_alpha = 0.6
    env = make_env(conf)
    ns = conf.nb_state
    rng = np.random.default_rng(13)
    N, B, K = 5000, 64, 7
    S = np.column_stack([rng.uniform(-3, 3, (N, ns - 1)), rng.uniform(0, 4.9, N)])
    rows = np.concatenate([S, rng.normal(size=(N, 1)), S + 0.01, rng.normal(size=(N, ns)) * 0.3,
                           np.zeros((N, 1)), np.zeros((N, 1))], axis=1)
    U = torch.as_tensor(rng.uniform(size=(K, B)), device="cuda")

    def setup():
        rl = RL_AC(env, NN(env, conf, w_S=0.0, seed=5), conf)
        rl.setup_model()
        buf = PrioritizedReplayBuffer(conf, env.sys)
        buf.add_rows(rows)
        return rl, buf
    seq, sbuf = setup()
    y = torch.empty(B, dtype=torch.float32, device="cuda")
    V = torch.empty_like(y)
    for k in range(K):
        idx, w = sbuf.sample_device(U[k])
        seq.update_rows(sbuf.storage, idx, w, y, V)
        sbuf.update_priorities_device(idx, y, V)
    pipe, pbuf = setup()
    pipe.update_rows_n_per(pbuf, U)
    torch.cuda.synchronize()
    for a, b in zip(_state(seq), _state(pipe)):
        assert torch.equal(a, b)
    for name in ("sum_tree", "min_tree", "exp_counter", "max_priority"):
        assert torch.equal(getattr(sbuf, name), getattr(pbuf, name)), name


@pytest.mark.parametrize("system,B,w_S,MC", [("double_integrator", 128, 1e-2, 0), ("double_integrator", 200, 1e-2, 1),
                                            ("double_integrator", 512, 1e-2, 0), ("manipulator", 64, 0.0, 0),
                                            ("car_park", 96, 0.0, 1)])
def test_fused_gemm_adam_equals_split_path(system, B, w_S, MC):
    """Small batches (gradient rows <= 1024) run the weight-gradient GEMM and Adam as one launch
    (k_wgrad_adam); its sums are formed in k_wgrad's order, so an update equals the split path
    (cacto_critic_grad -> slabs -> reduce, cacto_adam_step; the same for the actor) bit for bit."""
    from cacto_amd.rl import ACTOR, CRITIC
    conf = load_conf(system, fresh=True)
    conf.MC = MC
    env = make_env(conf)
    ns = conf.nb_state
    rng = np.random.default_rng(17)
    N = 3000
    S = np.column_stack([rng.uniform(-3, 3, (N, ns - 1)), rng.uniform(0, 4.9, N)])
    rows = np.concatenate([S, rng.normal(size=(N, 1)), S + 0.01, rng.normal(size=(N, ns)) * 0.3,
                           (rng.uniform(size=(N, 1)) < 0.1).astype(float), (rng.uniform(size=(N, 1)) < 0.1)
                           .astype(float)], axis=1)
    storage = torch.as_tensor(rows, device="cuda")
    idx = torch.as_tensor(rng.integers(0, N, size=(3, B)).astype(np.int32), device="cuda")
    wts = torch.as_tensor(rng.uniform(0.2, 1.0, size=(3, B)).astype(np.float32), device="cuda")

    def learner():
        rl = RL_AC(env, NN(env, conf, w_S=w_S, seed=4), conf)
        rl.setup_model()
        return rl
    fused, split = learner(), learner()
    for k in range(3):
        fused.update_rows(storage, idx[k], wts[k])
        gc = split.critic_grad_flat(storage, idx[k], wts[k])
        split.apply_gradients(CRITIC, gc, soft_update=not MC)
        ga = split.actor_grad_flat(storage, idx[k])
        split.apply_gradients(ACTOR, ga)
    torch.cuda.synchronize()
    for a, b in zip(_state(fused), _state(split)):
        assert torch.equal(a, b)
