"""critic_type 'sine-elu' (NeuralNetwork.py:80-93: sine, elu, sine, elu hidden layers, same widths as
the sine critic) on the CACTO_CRITIC_ELU build of the library (cacto_amd/libcacto_hip_sine_elu.so; the
default build compiles the sine critic only), in a child process that loads that
library: forward, dV/ds, the Sobolev critic gradient and the actor gradient against the oracle
(acts=SINE_ELU, pinned by finite differences in test_oracle_math.py) at B = 128 (4-sample tiles) and
1024 (16-sample tiles) for the double integrator and the manipulator (revolute-chain actor path), the
pipelined update loop against the sequential one, bit for bit, the .h5 checkpoints' Keras layer names
(the reference's sine-elu models) and that a 'sine' critic is refused on a handle whose sine-elu
critics exist. The default library refuses the critic type (CACTO_EINVAL)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANT = os.path.join(ROOT, "cacto_amd", "libcacto_hip_sine_elu.so")


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _nets(system, seed=0):
    from oracle import env as oenv
    from cacto_amd.confs import load_conf
    from cacto_amd.environment import make_env
    from cacto_amd.neural_network import NN
    from cacto_amd.rl import RL_AC
    conf = load_conf(system, fresh=True)
    conf.critic_type = "sine-elu"
    genv = make_env(conf)
    nn = NN(genv, conf, w_S=1e-2, seed=seed)
    rl = RL_AC(genv, nn, conf)
    rl.setup_model()
    assert genv.sys.critic_type == "sine-elu"
    return conf, genv, oenv.make_env(conf), nn, rl


def _rows(conf, B, rng):
    ns = conf.nb_state
    lo, hi = np.array(conf.x_init_min, dtype=float), np.array(conf.x_init_max, dtype=float)
    S = rng.uniform(lo, hi, size=(B, ns))
    Sn = rng.uniform(lo, hi, size=(B, ns))
    return np.concatenate([S, rng.normal(size=(B, 1)) * 0.5, Sn, rng.normal(size=(B, ns)) * 0.3,
                           (rng.uniform(size=(B, 1)) < 0.3).astype(float),
                           (rng.uniform(size=(B, 1)) < 0.2).astype(float)], axis=1)


def _child():
    import torch
    sys.path.insert(0, ROOT)
    from oracle import nn as onn
    out = {}
    for B in (128, 1024):
        conf, genv, oe, nn, rl = _nets("double_integrator")
        ns = conf.nb_state
        norm = conf.state_norm_arr.astype(np.float64)
        rng = np.random.default_rng(21)
        S = _rows(conf, 200, rng)[:, :ns].astype(np.float32)
        cw = rl.critic_model.get_weights()
        V, g = nn.critic_input_grad(rl.critic_model, S)
        ref_V = onn.critic_forward(cw, S.astype(np.float64), norm, acts=onn.SINE_ELU)
        ref_g, _ = onn.critic_input_grad(cw, S.astype(np.float64), norm, acts=onn.SINE_ELU)
        out["V_err_%d" % B] = float(np.abs(V.cpu().numpy() - ref_V).max() / max(1.0, np.abs(ref_V).max()))
        out["dVds_rel_%d" % B] = float(rel_l2(g.cpu().numpy(), ref_g))
        Ve = nn.eval(rl.critic_model, S).cpu().numpy()
        out["eval_err_%d" % B] = float(np.abs(Ve - ref_V).max() / max(1.0, np.abs(ref_V).max()))
        rows = _rows(conf, B, rng)
        r32 = rows.astype(np.float32).astype(np.float64)
        idx = torch.arange(B, dtype=torch.int32, device="cuda")
        gc, y, Vr, Vt = rl.critic_grad_rows(torch.as_tensor(rows, device="cuda"), idx)
        ref = onn.compute_critic_grad(cw, rl.target_critic.get_weights(), r32[:, :ns], r32[:, ns + 1:2 * ns + 1],
                                      r32[:, ns:ns + 1], r32[:, 2 * ns + 1:3 * ns + 1], r32[:, 3 * ns + 1:3 * ns + 2],
                                      np.ones((B, 1)), 1e-2, norm, acts=onn.SINE_ELU)
        out["critic_grad_rel_%d" % B] = max(float(rel_l2(a.cpu().numpy(), b)) for a, b in zip(gc, ref[0]))
        ga = rl.actor_grad_rows(torch.as_tensor(rows, device="cuda"), idx)
        refa = onn.compute_actor_grad(oe, rl.actor_model.get_weights(), cw, rows[:, :ns].astype(np.float32),
                                      rows[:, 3 * ns + 2:3 * ns + 3], norm, acts=onn.SINE_ELU)
        out["actor_grad_rel_%d" % B] = max(float(rel_l2(a.cpu().numpy(), b)) for a, b in zip(ga, refa))
    runs = []
    for pipelined in (False, True):
        conf, genv, oe, nn, rl = _nets("double_integrator", seed=3)
        rng = np.random.default_rng(22)
        storage = torch.as_tensor(_rows(conf, 4000, rng), device="cuda")
        idx = torch.as_tensor(rng.integers(0, 4000, size=(4, 1024)).astype(np.int32), device="cuda")
        if pipelined:
            rl.update_rows_n(storage, idx)
        else:
            for k in range(4):
                rl.update_rows(storage, idx[k])
        torch.cuda.synchronize()
        runs.append([t.cpu().numpy() for t in (rl.actor_model.buf, rl.critic_model.buf, rl.target_critic.buf)])
    out["pipelined_equal"] = all(bool(np.array_equal(a, b)) for a, b in zip(*runs))
    # the revolute-chain actor path (the manipulator: CRBA / RNEA dynamics Jacobian) at both tile sizes
    for B in (128, 1024):
        conf, genv, oe, nn, rl = _nets("manipulator", seed=1)
        ns = conf.nb_state
        norm = conf.state_norm_arr.astype(np.float64)
        rng = np.random.default_rng(23)
        rows = _rows(conf, B, rng)
        r32 = rows.astype(np.float32).astype(np.float64)
        cw = rl.critic_model.get_weights()
        idx = torch.arange(B, dtype=torch.int32, device="cuda")
        gc, y, Vr, Vt = rl.critic_grad_rows(torch.as_tensor(rows, device="cuda"), idx)
        ref = onn.compute_critic_grad(cw, rl.target_critic.get_weights(), r32[:, :ns], r32[:, ns + 1:2 * ns + 1],
                                      r32[:, ns:ns + 1], r32[:, 2 * ns + 1:3 * ns + 1], r32[:, 3 * ns + 1:3 * ns + 2],
                                      np.ones((B, 1)), 1e-2, norm, acts=onn.SINE_ELU)
        out["man_critic_grad_rel_%d" % B] = max(float(rel_l2(a.cpu().numpy(), b)) for a, b in zip(gc, ref[0]))
        ga = rl.actor_grad_rows(torch.as_tensor(rows, device="cuda"), idx)
        refa = onn.compute_actor_grad(oe, rl.actor_model.get_weights(), cw, rows[:, :ns].astype(np.float32),
                                      rows[:, 3 * ns + 2:3 * ns + 3], norm, acts=onn.SINE_ELU)
        out["man_actor_grad_rel_%d" % B] = max(float(rel_l2(a.cpu().numpy(), b)) for a, b in zip(ga, refa))
    # checkpoints in the reference's layout: the sine-elu models' Keras layer names (NeuralNetwork.py:80-93,
    # created after the actor, RL.py:52-76), read back bit for bit
    import tempfile
    from cacto_amd import h5
    names = {}
    with tempfile.TemporaryDirectory() as d:
        for role, net in (("critic", rl.critic_model), ("target", rl.target_critic)):
            path = os.path.join(d, role + ".h5")
            net.save_weights(path)
            with open(path, "rb") as f:
                hf = h5.H5File(f.read())
            names[role] = h5._strings(hf.attributes(hf.object(hf.root))["layer_names"])
            out["h5_%s_equal" % role] = all(bool(np.array_equal(a, b)) for a, b in
                                            zip(h5.read_keras_weights(path), net.get_weights()))
    out["h5_names"] = names
    # the activations belong to the handle: a 'sine' critic on it is refused while sine-elu nets live
    try:
        nn.create_critic_sine()
        out["sine_refused"] = False
    except ValueError:
        out["sine_refused"] = True
    print("RESULT " + json.dumps(out), flush=True)


@pytest.mark.gpu
def test_sine_elu_critic_on_its_build():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert os.path.exists(VARIANT), "build it: python -m cacto_amd.build"
    env = dict(os.environ, CACTO_HIP_LIB=VARIANT)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1][len("RESULT "):])
    for B in (128, 1024):
        assert res["V_err_%d" % B] <= 1e-5 and res["eval_err_%d" % B] <= 1e-5, res
        assert res["dVds_rel_%d" % B] < 2e-5, res
        assert res["critic_grad_rel_%d" % B] < 2e-4, res
        assert res["actor_grad_rel_%d" % B] < 2e-4, res
    assert res["pipelined_equal"], res
    for B in (128, 1024):
        assert res["man_critic_grad_rel_%d" % B] < 2e-4 and res["man_actor_grad_rel_%d" % B] < 2e-4, res
    assert res["h5_names"] == {
        "critic": ["sinusodial_representation_dense", "dense_3", "sinusodial_representation_dense_1", "dense_4",
                   "dense_5"],
        "target": ["sinusodial_representation_dense_2", "dense_6", "sinusodial_representation_dense_3", "dense_7",
                   "dense_8"]}, res
    assert res["h5_critic_equal"] and res["h5_target_equal"] and res["sine_refused"], res


@pytest.mark.gpu
def test_default_build_refuses_sine_elu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cacto_amd import _lib as L
    if os.path.abspath(L.LIB_PATH) == os.path.abspath(VARIANT):
        pytest.skip("running on the sine-elu build")
    with pytest.raises(RuntimeError, match="CACTO_CRITIC_ELU"):
        _nets("double_integrator")


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    _child()
