"""One main.py training loop (main.py:145-262) through the drop-in shims, with the reference's
call sequence and argument order, checked against the oracle:

    env = Environment(conf); NN_inst = NN(env, conf, w_S); RLAC = RL_AC(env, NN_inst, conf, N_try)
    buffer = ReplayBuffer(conf)                                          (main.py:145-150)
    RLAC.setup_model(); RLAC.RL_save_weights(update_step_counter)        (main.py:153-165)
    for ep: init_rand_state = [env.reset() ...]                          (main.py:225-230, GPU_flag)
            compute_sample: create_TO_init -> TO_Solve -> RL_Solve       (main.py:174-195)
            buffer.add(state_arr, partial_reward_to_go_arr, ...)         (main.py:240)
            update_step_counter = RLAC.learn_and_update(counter, buffer, ep)   (main.py:243)

TO_Solve (CasADi + ipopt, TO.py:37-106) is host-side and out of scope: the test stands in for it
with the warm start itself (TO_states / TO_controls = create_TO_init's rollout), a seeded step
cost, and the Sobolev labels from the GPU DDP backward pass (TO.backward_pass, TO.py:119-202, the
part of TO_Solve this build implements; parity-tested in test_gpu_ddp.py).

Checked: Env.reset against the reference's own draws (ref_vectors di_reset, random.seed(0)); the
warm-start rollouts against oracle/rollout.py; every replay row bit-exact against oracle RL_Solve
+ ReplayBuffer.add; learn_and_update (UPDATE_LOOPS = [7, 9]) with save_interval = 1 (every update
its own call) and 5 (pipelined chunks that end at the checkpoint saves 5, 10, 15): every call's
minibatch indices equal the reference's np.random draws, and the oracle, RE-SEEDED from the device
weights, target and Adam moments / iterations at the start of each call, repeats the call's K
updates to within STEP_TOL * K per element (STEP_TOL = 5e-6, the per-step bound of
test_gpu_update_parity.py) — so with save_interval = 1 every single update is checked at 5e-6; the
.h5 checkpoints written at the save steps equal the device weights after the call that reached them.
"""
import os
import random

import numpy as np
import pytest
import torch

from conftest import load_weights
from oracle import buffer as obuf
from oracle import env as oenv
from oracle import nn as onn
from oracle import rollout as oroll
from cacto_amd.confs import load_conf

pytestmark = pytest.mark.gpu
STEP_TOL = 5e-6


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _device_state(rl):
    """Weights (critic, target, actor) and Adam (m, v, iterations) per optimizer, as float64 lists."""
    def split(model, t):
        return [a.astype(np.float64) for a in model.split(t.detach().cpu().numpy())]
    it = rl.steps.cpu().numpy()
    return dict(nets=(rl.critic_model.get_weights(), rl.target_critic.get_weights(), rl.actor_model.get_weights()),
                critic=(split(rl.critic_model, rl.critic_m), split(rl.critic_model, rl.critic_v), int(it[0])),
                actor=(split(rl.actor_model, rl.actor_m), split(rl.actor_model, rl.actor_v), int(it[1])))


@pytest.mark.parametrize("save_interval", [1, 5])
def test_main_loop_double_integrator(tmp_path, ref_vectors, save_interval):
    from cacto_amd import h5
    from cacto_amd.environment import DoubleIntegrator
    from cacto_amd.neural_network import NN
    from cacto_amd.replay_buffer import PrioritizedReplayBuffer, ReplayBuffer
    from cacto_amd.rl import RL_AC
    from cacto_amd.to import TO

    conf = load_conf("double_integrator", fresh=True)
    conf.EP_UPDATE = 8
    conf.UPDATE_LOOPS = np.array([7, 9])
    conf.save_interval = save_interval
    conf.NNs_path = str(tmp_path)
    N_try, w_S = 0, 1e-2
    os.makedirs(os.path.join(conf.NNs_path, "N_try_%d" % N_try), exist_ok=True)

    # ---- main.py:145-165 ----
    env = DoubleIntegrator(conf)
    NN_inst = NN(env, conf, w_S)
    TrOp = TO(env, conf, w_S)
    RLAC = RL_AC(env, NN_inst, conf, N_try)
    buffer = ReplayBuffer(conf) if conf.prioritized_replay_alpha == 0 else PrioritizedReplayBuffer(conf)
    RLAC.setup_model(weights=load_weights("di_seed0_0"))    # the reference's seed-0 initial .h5 weights
    update_step_counter = 0
    RLAC.RL_save_weights(update_step_counter)

    # ---- the oracle's replica ----
    oe = oenv.make_env(conf)
    ns, B = conf.nb_state, conf.BATCH_SIZE
    norm = conf.state_norm_arr.astype(np.float64)
    obuffer = obuf.ReplayBuffer(conf.REPLAY_SIZE, ns)
    o_rng = np.random.RandomState(1234)
    # every learn_and_update call of the device (a chunk of K updates): the state it started from,
    # its indices, the state it ended in
    calls = []
    update_rows_n = RLAC.update_rows_n

    def spy(storage, idx_steps):
        torch.cuda.synchronize()
        pre = _device_state(RLAC)
        update_rows_n(storage, idx_steps)
        torch.cuda.synchronize()
        calls.append((pre, idx_steps.cpu().numpy(), _device_state(RLAC)))
    RLAC.update_rows_n = spy

    random.seed(0)                      # Env.reset draws from the module-level `random`
    np.random.seed(1234)                # ReplayBuffer.sample draws from the global numpy RNG
    cost_rng = np.random.default_rng(7)
    o_counter = 0
    for ep in range(len(conf.UPDATE_LOOPS)):
        init_rand_state = [env.reset() for _ in range(conf.EP_UPDATE)]
        if ep == 0:
            np.testing.assert_array_equal(np.array(init_rand_state), ref_vectors["di_reset"][:conf.EP_UPDATE])
        actor_now = RLAC.actor_model.get_weights()
        tmp = []
        for ICS in init_rand_state:
            # compute_sample (main.py:174-195)
            init_state, init_TO_states, init_TO_controls, NSTEPS_SH, ok = RLAC.create_TO_init(ep, ICS)
            if ok == 0:
                continue
            ref = oroll.to_init_rollout(oe, actor_now, ICS, ep)
            assert ref is not None and ref[2] == NSTEPS_SH
            np.testing.assert_allclose(init_TO_states, ref[0], rtol=0, atol=1e-5 * (1 + np.abs(ref[0]).max()))
            if ep == 0:
                np.testing.assert_array_equal(init_TO_states, ref[0])
                assert not init_TO_controls.any()
            np.testing.assert_allclose(RLAC.ee_pos_arr[0], oe.get_end_effector_position(np.asarray(ICS)), rtol=0,
                                       atol=1e-12)
            TO_states, TO_controls = init_TO_states, init_TO_controls          # TO_Solve stand-in
            TO_step_cost = cost_rng.normal(size=NSTEPS_SH + 1)
            dVdx = TrOp.backward_pass(NSTEPS_SH + 1, TO_states, TO_controls)
            (state_arr, partial, total, s_next, done, rwrd, term, ep_return,
             RL_ee_pos_arr) = RLAC.RL_Solve(TO_controls, TO_states, TO_step_cost)
            o_partial, o_total, o_snext, o_done, o_term = obuf.rl_solve(TO_states, TO_step_cost, conf.nsteps_TD_N)
            np.testing.assert_array_equal(partial, o_partial)
            np.testing.assert_array_equal(total, o_total)
            np.testing.assert_array_equal(s_next, o_snext)
            assert RL_ee_pos_arr.shape == (NSTEPS_SH + 1, 3)
            tmp.append((NSTEPS_SH, TO_controls, None, dVdx, state_arr.tolist(), partial, s_next, done, rwrd, term,
                        ep_return, RL_ee_pos_arr))
        (NSTEPS_SH, TO_controls, ee_pos_arr_TO, dVdx, state_arr, partial_reward_to_go_arr, state_next_rollout_arr,
         done_arr, rwrd_arr, term_arr, ep_return, ee_pos_arr_RL) = zip(*tmp)
        buffer.add(state_arr, partial_reward_to_go_arr, state_next_rollout_arr, dVdx, done_arr, term_arr)
        obuffer.add_rows(obuffer.concatenate(state_arr, partial_reward_to_go_arr, state_next_rollout_arr, dVdx,
                                             done_arr, term_arr))
        np.testing.assert_array_equal(buffer.storage.cpu().numpy(), obuffer.storage)
        assert buffer.next_idx == obuffer.next_idx

        n_calls = len(calls)
        update_step_counter = RLAC.learn_and_update(update_step_counter, buffer, ep)
        K_ep = int(conf.UPDATE_LOOPS[ep])
        ep_calls = calls[n_calls:]
        assert sum(len(c[1]) for c in ep_calls) == K_ep
        # the reference's loop (RL.py:120-143): one np.random.randint(0, max_idx, B) per update
        draws = np.stack([o_rng.randint(0, obuffer.max_idx(), size=B) for _ in range(K_ep)])
        np.testing.assert_array_equal(np.concatenate([c[1] for c in ep_calls]), draws)
        for pre, idx, post in ep_calls:
            # the oracle re-seeded from the device state at the start of the call
            crit, tgt, act = pre["nets"]
            oc, oa = onn.KerasAdam(conf.CRITIC_LEARNING_RATE), onn.KerasAdam(conf.ACTOR_LEARNING_RATE)
            for opt, st in ((oc, pre["critic"]), (oa, pre["actor"])):
                opt.m, opt.v, opt.iterations = list(st[0]), list(st[1]), st[2]
            for row in idx:
                r = obuffer.storage[row].astype(np.float32).astype(np.float64)
                gc = onn.compute_critic_grad(crit, tgt, r[:, :ns], r[:, ns + 1:2 * ns + 1], r[:, ns:ns + 1],
                                             r[:, 2 * ns + 1:3 * ns + 1], r[:, 3 * ns + 1:3 * ns + 2],
                                             np.ones((B, 1)), w_S, norm)[0]
                crit = oc.apply(crit, gc)
                ga = onn.compute_actor_grad(oe, act, crit, r[:, :ns].astype(np.float32),
                                            obuffer.storage[row, 3 * ns + 2:3 * ns + 3], norm)
                act = oa.apply(act, ga)
                tgt = onn.soft_update(tgt, crit, conf.UPDATE_RATE)
                o_counter += 1
            K = len(idx)
            for name, got, ref in zip(("critic", "target", "actor"), post["nets"], (crit, tgt, act)):
                for i, (a, b) in enumerate(zip(got, ref)):
                    err = np.abs(a - b).max()
                    assert err < STEP_TOL * K, (name, i, o_counter, K, err)
            assert post["critic"][2] == pre["critic"][2] + K and post["actor"][2] == pre["actor"][2] + K
            # the checkpoint a call ends on (RL.py:139-141) holds exactly the device weights
            if o_counter % conf.save_interval == 0:
                for name, got in zip(("critic", "target_critic", "actor"), post["nets"]):
                    path = os.path.join(conf.NNs_path, "N_try_%d" % N_try, "%s_%d.h5" % (name, o_counter))
                    for a, b in zip(h5.read_keras_weights(path), got):
                        np.testing.assert_array_equal(a, b)
        assert update_step_counter == o_counter
    # every call ends at a checkpoint or at the end of an episode's loop
    assert len(calls) == (16 if save_interval == 1 else 5)
    torch.cuda.synchronize()
    assert os.path.exists(os.path.join(conf.NNs_path, "N_try_0", "actor_0.h5"))


def test_reference_signature_grads_and_optimizer():
    """NN.compute_critic_grad(critic_model, target_critic, ...) / compute_actor_grad(actor_model,
    critic_model, state, term, batch_size) and optimizer.apply_gradients(zip(grads,
    model.trainable_variables)) exactly as RL_AC.update calls them (RL.py:101-111), against the
    fused update on the same minibatch (same kernels: bit-identical weights and counters)."""
    from cacto_amd.environment import make_env
    from cacto_amd.neural_network import NN
    from cacto_amd.rl import RL_AC
    from cacto_amd.replay_buffer import ReplayBuffer
    conf = load_conf("double_integrator", fresh=True)
    env = make_env(conf)
    rng = np.random.default_rng(31)
    B, ns = conf.BATCH_SIZE, conf.nb_state

    def learner():
        rl = RL_AC(env, NN(env, conf, 1e-2), conf, 0)
        rl.setup_model(weights=load_weights("di_seed0_0"))
        return rl
    S = np.column_stack([rng.uniform(-15, 15, (B, 4)), rng.uniform(0, 9.9, B)])
    rows = np.concatenate([S, rng.normal(size=(B, 1)), S + 0.05, rng.normal(size=(B, ns)) * 0.3,
                           (rng.uniform(size=(B, 1)) < 0.2).astype(float), (rng.uniform(size=(B, 1)) < 0.2)
                           .astype(float)], axis=1)
    buf = ReplayBuffer(conf)
    buf.add_rows(rows)
    idx = torch.arange(B, dtype=torch.int32, device="cuda")
    s, r, sn, dv, d, term, w, _ = buf.sample(idx)

    ref = learner()
    ref.update_rows(buf.storage, idx)
    rl = learner()
    NN_ = rl.NN
    critic_grad, y, V, Vt = NN_.compute_critic_grad(rl.critic_model, rl.target_critic, s, sn, r, dv, d, w)
    rl.critic_optimizer.apply_gradients(zip(critic_grad, rl.critic_model.trainable_variables))
    actor_grad = NN_.compute_actor_grad(rl.actor_model, rl.critic_model, s, term.cpu().numpy(), None)
    rl.actor_optimizer.apply_gradients(zip(actor_grad, rl.actor_model.trainable_variables))
    rl.update_target(rl.target_critic.variables, rl.critic_model.variables)
    torch.cuda.synchronize()
    assert rl.critic_optimizer.iterations == 1 and rl.actor_optimizer.iterations == 1
    for a, b in zip((ref.actor_model.buf, ref.critic_model.buf, ref.target_critic.buf, ref.actor_m, ref.critic_v),
                    (rl.actor_model.buf, rl.critic_model.buf, rl.target_critic.buf, rl.actor_m, rl.critic_v)):
        assert torch.equal(a, b)
    assert y.shape == (B, 1) and V.shape == (B, 1) and Vt.shape == (B, 1)
