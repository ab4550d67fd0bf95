"""GPU parity of cacto_ddp_backward (TO.backward_pass, TO.py:119-202) against the oracle."""
import random

import numpy as np
import pytest
import torch

from cacto_amd.confs import load_conf
from oracle import ddp as oddp
from oracle import env as oenv

pytestmark = pytest.mark.gpu

# float64 closed forms vs the oracle's sympy derivatives + numpy pinv: a few ulps per operation,
# compounded over <= 200 Riccati steps
RTOL = 1e-9


def _setup(system):
    from cacto_amd.environment import make_env
    from cacto_amd.to import TO
    conf = load_conf(system)
    genv = make_env(conf)
    return conf, oenv.make_env(conf), TO(genv, conf, w_S=1e-2)


def _episodes(conf, oe, n_ep, rng, zero_len=()):
    """Trajectories of Env.simulate under random controls, lengths NSTEPS - int(t/dt)."""
    ns, na = conf.nb_state, conf.nb_action
    S0 = [oe.reset(rng) for _ in range(n_ep)]
    T = [conf.NSTEPS - int(s[-1] / conf.dt) for s in S0]
    for k in zero_len:
        T[k] = 0
    L = max(T) + 1
    S = np.zeros((n_ep, L, ns))
    U = np.zeros((n_ep, L, na))
    for e in range(n_ep):
        S[e, 0] = S0[e]
        for t in range(T[e]):
            U[e, t] = [rng.uniform(-1.2, 1.2) * conf.u_max[i] for i in range(na)]
            S[e, t + 1] = oe.simulate(S[e, t], U[e, t])
    return S, U, np.asarray(T, dtype=np.int32)


@pytest.mark.parametrize("system", list(oddp.SUPPORTED))
def test_ddp_backward_matches_oracle(system):
    conf, oe, to = _setup(system)
    rng = random.Random(21)
    S, U, T = _episodes(conf, oe, 9, rng, zero_len=(4,))
    out = to.backward_pass_batch(torch.as_tensor(S, device="cuda"), torch.as_tensor(U, device="cuda"),
                                 torch.as_tensor(T, device="cuda"))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    n = conf.nb_state - 1
    for e in range(len(T)):
        ref = oddp.backward_pass(conf, S[e, :T[e] + 1], U[e, :T[e]])
        # rounding amplification of this trajectory's recursion: the oracle against itself with
        # an equivalent inverse (see oracle/ddp.py); the GPU may differ by a multiple of it
        alt = oddp.backward_pass(conf, S[e, :T[e] + 1], U[e, :T[e]], inverse="inv")
        scale = np.abs(ref[:, :n]).max() + 1e-12
        tol = RTOL * scale + 100.0 * np.abs(alt[:, :n] - ref[:, :n]).max(axis=1, keepdims=True)
        assert (np.abs(got[e, :T[e] + 1, :n] - ref[:, :n]) <= tol).all(), (system, e)
        assert (got[e, :T[e] + 1, n] == 0).all()
        assert (got[e, T[e] + 1:] == 0).all()   # rows past Te untouched


def test_ddp_backward_single_episode_api():
    """TO.backward_pass(T, TO_states, TO_controls) — the reference's per-episode signature."""
    conf, oe, to = _setup("double_integrator")
    rng = random.Random(8)
    S, U, T = _episodes(conf, oe, 1, rng)
    Te = int(T[0])
    got = to.backward_pass(Te + 1, S[0, :Te + 1, :-1], U[0, :Te])
    ref = oddp.backward_pass(conf, S[0, :Te + 1], U[0, :Te])
    alt = oddp.backward_pass(conf, S[0, :Te + 1], U[0, :Te], inverse="inv")
    tol = RTOL * np.abs(ref).max() + 100.0 * np.abs(alt - ref).max(axis=1, keepdims=True)
    assert (np.abs(got - ref) <= tol).all()


def test_ddp_backward_bad_arguments_fail_loudly():
    conf, oe, to = _setup("manipulator")
    S = torch.zeros(1, 3, conf.nb_state, dtype=torch.float64, device="cuda")
    U = torch.zeros(1, 3, conf.nb_action, dtype=torch.float64, device="cuda")
    from cacto_amd import _lib as L
    from cacto_amd.system import dptr, stream
    with pytest.raises(RuntimeError, match="cacto_ddp_backward"):
        L.lib().call("cacto_ddp_backward", to.sys.handle, dptr(S, torch.float64), 0, dptr(U, torch.float64), 3,
                     dptr(torch.tensor([2], dtype=torch.int32, device="cuda"), torch.int32), 1, 1e-9,
                     dptr(S, torch.float64), stream())


def _labels_in_subprocess(system, split, S, U, T):
    import os
    import subprocess
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as d:
        np.savez(os.path.join(d, "in.npz"), S=S, U=U, T=T)
        code = ("import sys, numpy as np, torch; sys.path.insert(0, %r)\n"
                "from cacto_amd.confs import load_conf\nfrom cacto_amd.environment import make_env\n"
                "from cacto_amd.to import TO\nz = np.load(%r)\nconf = load_conf(%r)\n"
                "to = TO(make_env(conf), conf, w_S=1e-2)\n"
                "out = to.backward_pass_batch(*(torch.as_tensor(z[k], device='cuda') for k in ('S', 'U', 'T')))\n"
                "np.save(%r, out.cpu().numpy())\n") % (root, os.path.join(d, "in.npz"), system,
                                                       os.path.join(d, "out.npy"))
        env = dict(os.environ, CACTO_DDP_SPLIT="1" if split else "0")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        return np.load(os.path.join(d, "out.npy"))


@pytest.mark.parametrize("system", ["manipulator", "ur5"])
def test_ddp_split_derivative_kernels_equal_the_fused_one(system):
    """The revolute chains' derivative records from the three split kernels (primal, one dual-number
    RNEA per direction with the forces in LDS, cost derivatives) are the fused k_ddp_derivs' bit
    for bit, and so are the labels."""
    conf, oe, _ = _setup(system)
    S, U, T = _episodes(conf, oe, 70, random.Random(33), zero_len=(5,))
    T[7] = -1                                  # a dropped episode: skipped by both
    a = _labels_in_subprocess(system, True, S, U, T)
    b = _labels_in_subprocess(system, False, S, U, T)
    assert np.array_equal(a, b)
