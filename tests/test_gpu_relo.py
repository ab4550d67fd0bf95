"""The 'ReLO' priority rule of PrioritizedReplayBuffer.update_priorities (replay_buffer.py:193-196,
:200-218). The shipped reference never selects it (RB_type is commented out, :118), so this is the
reference's alternative rule, restated: td = MSE(y, V) - MSE(y, V_tgt) per sample (Keras
MeanSquaredError, reduction NONE), np.clip(td, 0, max td), p = fresh^count * td + eps in f64.
Device (cacto_per_update_relo) against oracle/buffer.py update_priorities_relo; leaves p^alpha
agree to 2 ulp (device pow vs libm pow, as for the 'PER' leaves), everything else exactly."""
import random

import numpy as np
import pytest
import torch

from oracle import buffer as obuf
from cacto_amd.confs import load_conf

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _pair(conf, rows):
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    from cacto_amd.system import System
    per = PrioritizedReplayBuffer(conf, System(conf))
    per.RB_type = "ReLO"
    o = obuf.PrioritizedReplayBuffer(conf.REPLAY_SIZE, conf.nb_state, per.alpha, per.beta, per.eps, per.fresh,
                                     conf.BATCH_SIZE)
    per.add_rows(rows)
    o.add_rows(rows)
    return per, o


def _state(per, o, n):
    cap = per.cap
    return (per.sum_tree[cap:cap + n].cpu().numpy(), np.array(o.it_sum.value[cap:cap + n]),
            per.min_tree[cap:cap + n].cpu().numpy(), np.array(o.it_min.value[cap:cap + n]))


@pytest.mark.parametrize("B", [64, 700])
def test_relo_priorities_match_oracle(B):
    conf = load_conf("car_park", fresh=True)
    conf.prioritized_replay_alpha = 0.6
    conf.BATCH_SIZE = B
    rng = np.random.default_rng(21 + B)
    rows = rng.normal(size=(3000, 3 * conf.nb_state + 3))
    per, o = _pair(conf, rows)
    for it in range(3):
        u = list(rng.uniform(size=B))
        idx, _ = per.sample_device(u)
        oidx = o.sample_proportional(u)
        np.testing.assert_array_equal(idx.cpu().numpy(), oidx)
        o.sample_weights(oidx)                       # exp_counter, as the device sampler
        y = rng.normal(size=(B, 1)).astype(np.float32)
        V = (y + rng.normal(size=(B, 1)) * 0.5).astype(np.float32)
        Vt = (y + rng.normal(size=(B, 1)) * 0.3).astype(np.float32)
        if it == 2:
            Vt[: B // 2] = V[: B // 2]              # td == 0 -> p = eps exactly
        per.update_priorities(idx, y, V, Vt)
        o.update_priorities_relo(oidx, y, V, Vt)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(per.exp_counter.cpu().numpy(), o.exp_counter)
        assert per.max_priority.item() == pytest.approx(o.max_priority, rel=1e-15)
        for got, exp in zip(*[iter(_state(per, o, 3000))] * 2):
            np.testing.assert_allclose(got, exp, rtol=4.5e-16, atol=0)


def test_relo_needs_target_value():
    conf = load_conf("double_integrator", fresh=True)
    conf.prioritized_replay_alpha = 0.6
    per, _ = _pair(conf, np.random.default_rng(3).normal(size=(200, 3 * conf.nb_state + 3)))
    idx, _ = per.sample_device(list(np.random.default_rng(4).uniform(size=conf.BATCH_SIZE)))
    y = torch.zeros(conf.BATCH_SIZE, dtype=torch.float32, device="cuda")
    with pytest.raises(ValueError):
        per.update_priorities_device(idx, y, y)


def test_learn_and_update_relo_equals_manual_loop():
    """learn_and_update with RB_type 'ReLO' (RL.py:120-143): sample -> update (y, V, V_tgt) ->
    ReLO priorities per update, equal bit for bit to the same loop spelled out."""
    from cacto_amd.environment import make_env
    from cacto_amd.neural_network import NN
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    from cacto_amd.rl import RL_AC
    from conftest import load_weights
    conf = load_conf("double_integrator", fresh=True)
    conf.prioritized_replay_alpha = 0.6
    conf.BATCH_SIZE = 64
    conf.UPDATE_LOOPS = [4]
    conf.NNs_path = None
    rows = np.random.default_rng(8).normal(size=(2000, 3 * conf.nb_state + 3))
    rows[:, 3 * conf.nb_state + 1:] = (rows[:, 3 * conf.nb_state + 1:] > 0.5).astype(float)
    res = []
    for manual in (False, True):
        env = make_env(conf)
        rl = RL_AC(env, NN(env, conf, w_S=1e-2, seed=3), conf)
        rl.setup_model(weights=load_weights("di_seed0_0"))
        buf = PrioritizedReplayBuffer(conf, rl.sys, py_random=random.Random(5))
        buf.RB_type = "ReLO"
        buf.add_rows(rows)
        if manual:
            B = conf.BATCH_SIZE
            y = torch.empty(B, dtype=torch.float32, device="cuda")
            V, Vt = torch.empty_like(y), torch.empty_like(y)
            for _ in range(4):
                u = [buf.random.random() for _ in range(B)]
                idx, w = buf.sample_device(u)
                rl.update_rows(buf.storage, idx, w, y, V, Vt)
                buf.update_priorities_device(idx, y, V, Vt)
        else:
            assert rl.learn_and_update(0, buf, 0) == 4
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in (rl.critic_model.buf, rl.actor_model.buf, buf.sum_tree, buf.min_tree,
                                              buf.exp_counter, buf.max_priority)])
    for a, b in zip(*res):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("case", ["all_negative", "nan"])
def test_relo_failed_assert_raises_and_leaves_trees(case):
    """replay_buffer.py:212 asserts every new priority > 0. With V closer to y than V_tgt for every
    sample, td < 0 everywhere, np.clip's bound max(td) is negative and p = fresh^c max(td) + eps < 0;
    a NaN td makes np.max NaN and every p NaN. The device flags the batch instead of writing NaN
    leaves: update_priorities raises AssertionError, and the trees, counters and max_priority are
    exactly as before the call (the next, valid, update then proceeds as usual)."""
    conf = load_conf("car_park", fresh=True)
    conf.prioritized_replay_alpha = 0.6
    B = 64
    conf.BATCH_SIZE = B
    rng = np.random.default_rng(31)
    per, o = _pair(conf, rng.normal(size=(1500, 3 * conf.nb_state + 3)))
    idx, _ = per.sample_device(list(rng.uniform(size=B)))
    y = rng.normal(size=(B, 1)).astype(np.float32)
    V = (y + rng.normal(size=(B, 1)) * 0.01).astype(np.float32)
    Vt = (y + 1.0 + np.abs(rng.normal(size=(B, 1)))).astype(np.float32)
    if case == "nan":
        Vt = (y + rng.normal(size=(B, 1)) * 0.3).astype(np.float32)
        V[5, 0] = np.nan
    torch.cuda.synchronize()
    before = [t.clone() for t in (per.sum_tree, per.min_tree, per.exp_counter, per.max_priority)]
    with pytest.raises(AssertionError):
        per.update_priorities(idx, y, V, Vt)
    for a, b in zip(before, (per.sum_tree, per.min_tree, per.exp_counter, per.max_priority)):
        assert torch.equal(a, b)
    # the flag was cleared: a valid update goes through and matches the oracle
    o.sample_weights(idx.cpu().numpy())             # the device sampler's exp_counter side effect
    V2 = (y + rng.normal(size=(B, 1)) * 0.5).astype(np.float32)
    Vt2 = (y + rng.normal(size=(B, 1)) * 0.3).astype(np.float32)
    per.update_priorities(idx, y, V2, Vt2)
    o.update_priorities_relo(idx.cpu().numpy(), y, V2, Vt2)
    torch.cuda.synchronize()
    for got, exp in zip(*[iter(_state(per, o, 1500))] * 2):
        np.testing.assert_allclose(got, exp, rtol=4.5e-16, atol=0)


def test_learn_and_update_alpha_zero_skips_priorities():
    """RL.py:130: with prioritized_replay_alpha == 0 learn_and_update never calls update_priorities
    (a PrioritizedReplayBuffer built directly; main.py:150 would pick the plain buffer). The ReLO
    loop and the pipelined 'PER' loop both leave the trees as the adds set them, and the weights
    equal the manual sample -> update loop without priority updates."""
    from cacto_amd.environment import make_env
    from cacto_amd.neural_network import NN
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer
    from cacto_amd.rl import RL_AC
    from conftest import load_weights
    for rb_type in ("ReLO", "PER"):
        conf = load_conf("double_integrator", fresh=True)
        conf.prioritized_replay_alpha = 0.0
        conf.BATCH_SIZE = 64
        conf.UPDATE_LOOPS = [3]
        conf.NNs_path = None
        rows = np.random.default_rng(9).normal(size=(1500, 3 * conf.nb_state + 3))
        rows[:, 3 * conf.nb_state + 1:] = (rows[:, 3 * conf.nb_state + 1:] > 0.5).astype(float)
        res = []
        for manual in (False, True):
            env = make_env(conf)
            rl = RL_AC(env, NN(env, conf, w_S=1e-2, seed=3), conf)
            rl.setup_model(weights=load_weights("di_seed0_0"))
            buf = PrioritizedReplayBuffer(conf, rl.sys, py_random=random.Random(7))
            buf.RB_type = rb_type
            buf.add_rows(rows)
            torch.cuda.synchronize()
            trees0 = [buf.sum_tree.clone(), buf.min_tree.clone(), buf.max_priority.clone()]
            if manual:
                B = conf.BATCH_SIZE
                y = torch.empty(B, dtype=torch.float32, device="cuda")
                V, Vt = torch.empty_like(y), torch.empty_like(y)
                for _ in range(3):
                    u = [buf.random.random() for _ in range(B)]
                    idx, w = buf.sample_device(u)
                    rl.update_rows(buf.storage, idx, w, y, V, Vt if rb_type == "ReLO" else None)
            else:
                assert rl.learn_and_update(0, buf, 0) == 3
            torch.cuda.synchronize()
            for a, b in zip(trees0, (buf.sum_tree, buf.min_tree, buf.max_priority)):
                assert torch.equal(a, b), rb_type
            res.append([t.cpu().numpy() for t in (rl.critic_model.buf, rl.actor_model.buf, buf.exp_counter)])
        for a, b in zip(*res):
            np.testing.assert_array_equal(a, b)
