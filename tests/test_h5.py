"""Keras-2.11 .h5 checkpoint interop (cacto_amd/h5.py).

* Reading: the reference's own checkpoints (`Results */NNs/N_try_*/{actor,critic,target_critic}_*.h5`,
  RL.py:191-195) against the .npz fixtures tests/golden/make_h5_fixtures.py extracted from them with
  h5py — skipped where /root/reference is absent (the GPU box).
* Writing: round trip through the native reader, and — where an interpreter with h5py exists in
  this container (/opt/conda/bin/python3.9) — the written file opened by h5py itself, the library
  Keras' load_weights uses.
* GPU: RL_AC.RL_save_weights writes .h5 files that setup_model(recover_training=...) restores.
"""
import os
import subprocess

import numpy as np
import pytest

from cacto_amd import h5

REF = "/root/reference"
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "weights")
DI = os.path.join(REF, "Results Double Integrator/Results set test/NNs/N_try_6")
SI = os.path.join(REF, "Results Single Integrator/Results set test/NNs")
H5PY_PYTHON = "/opt/conda/bin/python3.9"

CASES = [
    ("di_seed0_0", "actor", os.path.join(DI, "actor_0.h5")),
    ("di_seed0_0", "critic", os.path.join(DI, "critic_0.h5")),
    ("di_seed0_0", "target", os.path.join(DI, "target_critic_0.h5")),
    ("di_seed0_final", "actor", os.path.join(DI, "actor_final.h5")),
    ("di_seed0_final", "critic", os.path.join(DI, "critic_final.h5")),
    ("di_seed0_final", "target", os.path.join(DI, "target_critic_final.h5")),
    ("si_seed0_0", "actor", os.path.join(SI, "N_try_0/actor_0.h5")),
    ("si_seed10_0", "critic", os.path.join(SI, "N_try_5/critic_0.h5")),
]


@pytest.mark.parametrize("tag,key,path", CASES)
def test_read_reference_checkpoints(tag, key, path):
    if not os.path.exists(path):
        pytest.skip("reference checkpoints are not present on this machine")
    z = np.load(os.path.join(GOLD, tag + ".npz"))
    got = h5.read_keras_weights(path)
    n = len([k for k in z.files if k.startswith(key + "_")])
    assert len(got) == n
    for i, a in enumerate(got):
        ref = z["%s_%d" % (key, i)]
        assert a.dtype == np.float32 and a.shape == ref.shape
        assert np.array_equal(a, ref)


def test_reference_attributes():
    path = os.path.join(DI, "target_critic_0.h5")
    if not os.path.exists(path):
        pytest.skip("reference checkpoints are not present on this machine")
    f = h5.H5File(open(path, "rb").read())
    attrs = f.attributes(f.object(f.root))
    assert attrs["keras_version"] == b"2.11.0" and attrs["backend"] == b"tensorflow"
    names = [n.decode() for n in attrs["layer_names"]]
    assert names[1:] == ["sinusodial_representation_dense_%d" % k for k in range(4, 8)] + ["dense_4"]


def _layers(ws, names):
    return [(n, [(n + "/kernel:0", ws[2 * i]), (n + "/bias:0", ws[2 * i + 1])]) for i, n in enumerate(names)]


ACTOR = ["dense", "dense_1", "dense_2"]
CRITIC = ["sinusodial_representation_dense", "sinusodial_representation_dense_1",
          "sinusodial_representation_dense_2", "sinusodial_representation_dense_3", "dense_3"]


def test_write_read_round_trip(tmp_path):
    z = np.load(os.path.join(GOLD, "di_seed0_0.npz"))
    ws = [z["critic_%d" % i] for i in range(10)]
    p = str(tmp_path / "critic.h5")
    h5.write_keras_weights(p, _layers(ws, CRITIC))
    got = h5.read_keras_weights(p)
    assert len(got) == 10 and all(np.array_equal(a, b) for a, b in zip(got, ws))
    f = h5.H5File(open(p, "rb").read())
    attrs = f.attributes(f.object(f.root))
    assert [s.decode() for s in attrs["layer_names"]] == CRITIC
    assert attrs["keras_version"] == b"2.11.0"


def test_written_file_opens_in_h5py(tmp_path):
    if not os.path.exists(H5PY_PYTHON):
        pytest.skip("no interpreter with h5py here")
    if subprocess.run([H5PY_PYTHON, "-c", "import h5py"], capture_output=True).returncode != 0:
        pytest.skip("h5py not importable")
    rng = np.random.default_rng(0)
    ws = [rng.standard_normal(s).astype(np.float32) for s in [(5, 256), (256,), (256, 256), (256,), (256, 2), (2,)]]
    p = str(tmp_path / "actor.h5")
    h5.write_keras_weights(p, _layers(ws, ACTOR))
    np.savez(str(tmp_path / "expect.npz"), *ws)
    script = (
        "import sys, h5py, numpy as np\n"
        "f = h5py.File(sys.argv[1], 'r')\n"
        "z = np.load(sys.argv[2])\n"
        "names = [n.decode() for n in f.attrs['layer_names']]\n"
        "got = []\n"
        "for n in names:\n"
        "    for w in f[n].attrs['weight_names']:\n"
        "        got.append(np.asarray(f[n][w.decode()]))\n"
        "assert len(got) == len(z.files)\n"
        "for i, a in enumerate(got):\n"
        "    assert a.dtype == np.float32 and np.array_equal(a, z['arr_%d' % i]), i\n"
        "print('ok', names, f.attrs['keras_version'])\n")
    r = subprocess.run([H5PY_PYTHON, "-B", "-c", script, p, str(tmp_path / "expect.npz")], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok")


def test_rejects_non_hdf5(tmp_path):
    p = tmp_path / "x.h5"
    p.write_bytes(b"not hdf5 at all" * 10)
    with pytest.raises(h5.H5Error):
        h5.read_keras_weights(str(p))


@pytest.mark.gpu
def test_rl_save_and_recover_h5(tmp_path):
    """RL_save_weights -> .h5 (RL.py:191-195); setup_model(recover_training) reads them back."""
    import torch  # noqa: F401
    from cacto_amd.confs import load_conf
    from cacto_amd.environment import make_env
    from cacto_amd.neural_network import NN
    from cacto_amd.rl import RL_AC
    conf = load_conf("double_integrator", fresh=True)
    env = make_env(conf)
    z = np.load(os.path.join(GOLD, "di_seed0_final.npz"))
    w = {k: [z["%s_%d" % (k, i)] for i in range(6 if k == "actor" else 10)] for k in ("actor", "critic", "target")}
    rl = RL_AC(env, NN(env, conf, w_S=1e-2), conf, N_try=3)
    rl.setup_model(weights=w)
    conf.NNs_path = str(tmp_path)
    os.makedirs(os.path.join(str(tmp_path), "N_try_3"))
    rl.RL_save_weights(7)
    for name in ("actor", "critic", "target_critic"):
        assert os.path.exists(os.path.join(str(tmp_path), "N_try_3", "%s_7.h5" % name))
    rl2 = RL_AC(env, NN(env, conf, w_S=1e-2), conf)
    rl2.setup_model(recover_training=(str(tmp_path), 3, 7))
    for net, key in ((rl2.actor_model, "actor"), (rl2.critic_model, "critic"), (rl2.target_critic, "target")):
        assert all(np.array_equal(a, b) for a, b in zip(net.get_weights(), w[key]))
