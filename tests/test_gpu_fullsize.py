"""Parity at BASELINE.json's full sizes (configs[1..3]), through properties that do not need the
oracle to redo the whole workload: exact time columns, per-step consistency with the oracle's
Env.simulate / actor on sampled episodes, schedule invariance, the pipelined update against the
sequential one, DDP labels of sampled episodes, and PER sampling / priority updates on a full
65,536-row buffer (SURVEY §8d inputs)."""
import random

import numpy as np
import pytest
import torch

from oracle import buffer as obuf
from oracle import ddp as oddp
from oracle import nn as onn
from test_gpu_parity import F32_TOL, _nets, abs_bound

pytestmark = pytest.mark.gpu


def _rollout(system, R):
    conf, genv, oe, nn, rl = _nets(system, None, seed=2)
    rng = random.Random(0)
    S0 = np.array([oe.reset(rng) for _ in range(R)])
    n = np.array([conf.NSTEPS - int(s[-1] / conf.dt) for s in S0])
    return conf, oe, rl, S0, n


@pytest.mark.parametrize("system,R", [("double_integrator", 4096), ("manipulator", 8192), ("car_park", 4096),
                                      ("ur5", 2048)])
def test_fullsize_rollout_properties(system, R):
    conf, oe, rl, S0, n = _rollout(system, R)
    T = int(n.max())
    out = rl.rollout_batch(S0, n, T)
    torch.cuda.synchronize()
    S, A = out["S"].cpu().numpy(), out["A"].cpu().numpy()
    assert (out["status"].cpu().numpy() == 0).all()
    # the time column: t_{k+1} = t_k + dt, the same float64 additions as Env.simulate
    t = S0[:, -1].copy()
    for k in range(T):
        live = n > k
        t = np.where(live, t + conf.dt, t)
        np.testing.assert_array_equal(S[live, k + 1, -1], t[live])
    # sampled episodes: actor within the float32 bound, dynamics exact, at three steps each
    actor = rl.actor_model.get_weights()
    norm = conf.state_norm_arr.astype(np.float64)
    pick = np.random.default_rng(1).choice(R, 48, replace=False)
    for e in pick:
        ts = sorted({0, int(n[e]) // 2, int(n[e]) - 1})
        x = S[e, ts].astype(np.float32).astype(np.float64)
        a_ref = onn.actor_forward(actor, x, norm)
        assert np.all(np.abs(A[e, ts] - a_ref) <= F32_TOL * abs_bound("actor", actor, x, norm))
        for k in ts:
            np.testing.assert_allclose(S[e, k + 1], oe.simulate(S[e, k], A[e, k].astype(np.float64)), rtol=1e-12,
                                       atol=1e-12)
    # schedule invariance at full size: another (groups, workgroups) split gives the same bits (the
    # manipulator, whose default is the one-slot-per-wave kernel, also on the generic kernel's
    # 16-slot workgroups, groups = 4)
    for sched in [(1, 512)] + ([(4, 0)] if system == "manipulator" else []):
        other = rl.rollout_batch(S0, n, T, want=("S", "A"), sched=sched)
        torch.cuda.synchronize()
        oS, oA = other["S"].cpu().numpy(), other["A"].cpu().numpy()
        for e in range(R):
            k = int(n[e])
            assert np.array_equal(oS[e, :k + 1], S[e, :k + 1]), (sched, e)
            assert np.array_equal(oA[e, :k], A[e, :k]), (sched, e)


def test_fullsize_pipelined_updates_equal_sequential():
    """configs[1] at the scaled batch B = 4096 on a 65,536-row buffer."""
    from test_gpu_graph import _state
    from cacto_amd.confs import load_conf
    from cacto_amd.environment import make_env
    from cacto_amd.neural_network import NN
    from cacto_amd.rl import RL_AC
    conf = load_conf("double_integrator")
    env = make_env(conf)
    ns = conf.nb_state
    rng = np.random.default_rng(21)
    N, B, K = 65536, 4096, 3
    S = np.column_stack([rng.uniform(-15, 15, (N, ns - 1)), rng.uniform(0, 9.9, N)])
    rows = np.concatenate([S, rng.normal(size=(N, 1)), S + 0.05, rng.normal(size=(N, ns)) * 0.3,
                           (rng.uniform(size=(N, 1)) < 0.05).astype(float), np.zeros((N, 1))], axis=1)
    storage = torch.as_tensor(rows, device="cuda")
    idx = torch.as_tensor(rng.integers(0, N, size=(K, B)).astype(np.int32), device="cuda")

    def learner():
        rl = RL_AC(env, NN(env, conf, w_S=1e-2, seed=4), conf)
        rl.setup_model()
        return rl
    seq, pipe = learner(), learner()
    for k in range(K):
        seq.update_rows(storage, idx[k])
    pipe.update_rows_n(storage, idx)
    torch.cuda.synchronize()
    for a, b in zip(_state(seq), _state(pipe)):
        assert torch.equal(a, b)


def test_fullsize_ddp_labels_sampled_episodes():
    """DDP labels of all 4096 configs[1] rollouts; 6 sampled episodes against the oracle."""
    from cacto_amd.to import TO
    conf, oe, rl, S0, n = _rollout("double_integrator", 4096)
    T = int(n.max())
    out = rl.rollout_batch(S0, n, T, want=("S", "A"))
    to = TO(rl.env, conf, w_S=1e-2)
    lab = to.backward_pass_batch(out["S"], out["A"].double(), torch.as_tensor(n.astype(np.int32), device="cuda"))
    torch.cuda.synchronize()
    S, A, L = out["S"].cpu().numpy(), out["A"].cpu().numpy().astype(np.float64), lab.cpu().numpy()
    m = conf.nb_state - 1
    for e in np.random.default_rng(3).choice(4096, 6, replace=False):
        k = int(n[e])
        ref = oddp.backward_pass(conf, S[e, :k + 1], A[e, :k])
        alt = oddp.backward_pass(conf, S[e, :k + 1], A[e, :k], inverse="inv")
        tol = 1e-9 * (np.abs(ref[:, :m]).max() + 1e-12) + 100.0 * np.abs(alt[:, :m] - ref[:, :m]).max(axis=1,
                                                                                                   keepdims=True)
        assert (np.abs(L[e, :k + 1, :m] - ref[:, :m]) <= tol).all()


def test_fullsize_per_sample_and_update():
    """configs[3] PER at B = 4096 on a full 65,536-row shard: stratified indices bit-exact against the
    oracle sampler, IS weights, and the priority update."""
    from cacto_amd.confs import load_conf
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    from cacto_amd.system import System
    conf = load_conf("car_park")
    B = 4096
    per = PrioritizedReplayBuffer(conf, System(conf))
    per.alpha = 0.6
    o = obuf.PrioritizedReplayBuffer(conf.REPLAY_SIZE, conf.nb_state, 0.6, 0.6, conf.prioritized_replay_eps,
                                     conf.fresh_factor, B)
    rng = np.random.default_rng(31)
    # REPLAY_SIZE - 1 rows: an add that ends exactly at the ring's end leaves `full` unset and
    # next_idx at 0 (the reference's latch quirk, replay_buffer.py:25-36), i.e. an empty-looking buffer
    N = conf.REPLAY_SIZE - 1
    rows = rng.normal(size=(N, 3 * conf.nb_state + 3))
    per.add_rows(rows)
    o.add_rows(rows)
    for it in range(2):
        u = list(rng.uniform(size=B))
        idx, w = per.sample_device(torch.as_tensor(np.asarray(u), device="cuda"))
        oidx = o.sample_proportional(u)
        np.testing.assert_array_equal(idx.cpu().numpy(), oidx)
        ow = o.sample_weights(oidx)
        np.testing.assert_allclose(w.cpu().numpy(), np.asarray(ow, dtype=np.float32).reshape(-1), rtol=1e-6)
        y = rng.normal(size=(B, 1)).astype(np.float32)
        V = rng.normal(size=(B, 1)).astype(np.float32)
        per.update_priorities_device(idx, torch.as_tensor(y, device="cuda"), torch.as_tensor(V, device="cuda"))
        o.update_priorities(oidx, y, V)
        torch.cuda.synchronize()
        st = per.sum_tree.cpu().numpy()
        cap = st.shape[0] // 2
        np.testing.assert_allclose(st[cap:cap + N], o.it_sum.value[cap:cap + N], rtol=1e-6)
        np.testing.assert_allclose(st[1], o.it_sum.value[1], rtol=1e-6)
