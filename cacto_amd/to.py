"""TO — the value-gradient half of the reference's trajectory optimisation (TO.py:9-202).

The NLP solve itself (TO_System_Solve, TO.py:37-100: CasADi + ipopt) stays on the host CPU and is
not part of this package. What the learner consumes from it besides the trajectory is the Sobolev
label dV/dx, which the reference computes with a DDP backward pass (TO.backward_pass,
TO.py:119-202). That pass runs here on the GPU (`cacto_ddp_backward`), one thread per episode,
along any recorded trajectory — a TO solution handed over from the host, or the policy rollouts
of `RL_AC.rollout_batch` (the TO warm start, RL.py:197-233).
"""
import numpy as np
import torch

from . import _lib as L
from .system import DEVICE, dptr, stream


class TO:
    def __init__(self, env, conf, w_S=0):
        self.env = env
        self.conf = conf
        self.w_S = w_S
        self.sys = env.sys

    def backward_pass(self, T, TO_states, TO_controls, mu=1e-9):
        """TO.py:119-202 for one episode: T states s_0..s_{T-1} ([T, >= ns-1]; a time column is
        ignored), T-1 controls. Returns V_x [T, ns] (numpy float64, last column 0)."""
        ns, na = self.conf.nb_state, self.conf.nb_action
        S = np.zeros((1, T, ns))
        S[0, :, :ns - 1] = np.asarray(TO_states, dtype=np.float64)[:T, :ns - 1]
        U = np.zeros((1, max(T - 1, 1), na))
        U[0, :T - 1] = np.asarray(TO_controls, dtype=np.float64)[:T - 1, :na]
        out = self.backward_pass_batch(torch.as_tensor(S, device=DEVICE), torch.as_tensor(U, device=DEVICE),
                                       torch.tensor([T - 1], dtype=torch.int32, device=DEVICE), mu=mu)
        return out[0].cpu().numpy()

    def backward_pass_batch(self, S_traj, U_traj, nsteps, mu=1e-9, out=None, status=None):
        """Device batch: S_traj [E, ldS, ns] f64, U_traj [E, ldU, na] f64, nsteps [E] int32 (Te per
        episode: Te + 1 states). Returns dVdx [E, ldS, ns] f64 (rows past Te untouched).
        status [E] int32 (device, a rollout's): episodes with status != 0 were dropped for a NaN
        state (RL.py:229-231, main.py:236) and get no labels (their rows stay untouched)."""
        E, ldS = S_traj.shape[0], S_traj.shape[1]
        if out is None:
            out = torch.zeros_like(S_traj)
        if status is not None:
            nsteps = torch.where(status.to(device=DEVICE) == 0, nsteps.to(device=DEVICE, dtype=torch.int32),
                                 torch.full_like(nsteps, -1, dtype=torch.int32, device=DEVICE)).contiguous()
        L.lib().call("cacto_ddp_backward", self.sys.handle, dptr(S_traj, torch.float64), ldS,
                     dptr(U_traj, torch.float64), U_traj.shape[1], dptr(nsteps, torch.int32), E, float(mu),
                     dptr(out, torch.float64), stream())
        return out
