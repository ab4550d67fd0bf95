"""Actor/critic networks with the reference surface (NeuralNetwork.py:10-233), on the HIP kernels.

A model is a `Net`: one device "net buffer" [flat Keras-order params | MFMA-packed fragments]
(include/cacto_hip.h). NN.eval / compute_critic_grad / compute_actor_grad call the fused kernels;
the training loop (cacto_amd.rl.RL_AC) uses the fused `cacto_update` directly on replay rows.
"""
import ctypes as C

import numpy as np
import torch

from . import _lib as L
from . import h5
from .system import DEVICE, dptr, stream

ACTOR, CRITIC = L.CACTO_NET_ACTOR, L.CACTO_NET_CRITIC
SINE_ELU = ("sine", "elu", "sine", "elu")  # critic_type 'sine-elu' hidden layers (NeuralNetwork.py:80-93)


def layer_shapes(kind, ns, na):
    if kind == ACTOR:  # NeuralNetwork.py:51-63
        dims = [ns, 256, 256, na]
    else:              # NeuralNetwork.py:95-108 (critic_type 'sine', every shipped config)
        dims = [ns, 64, 64, 128, 128, 1]
    shapes = []
    for i, o in zip(dims[:-1], dims[1:]):
        shapes += [(i, o), (o,)]
    return shapes


# Keras layer names of the reference's three models in one process (the .h5 files it writes,
# e.g. Results Double Integrator/.../N_try_6/{actor,critic,target_critic}_0.h5): Keras numbers each
# layer class separately in creation order (actor, critic, target critic, RL.py:52-76), so the
# sine-elu critic's Dense elu layers continue the actor's dense_* count (NeuralNetwork.py:80-93)
LAYER_NAMES = {
    "actor": ["dense", "dense_1", "dense_2"],
    "critic": ["sinusodial_representation_dense", "sinusodial_representation_dense_1",
               "sinusodial_representation_dense_2", "sinusodial_representation_dense_3", "dense_3"],
    "target": ["sinusodial_representation_dense_4", "sinusodial_representation_dense_5",
               "sinusodial_representation_dense_6", "sinusodial_representation_dense_7", "dense_4"],
}
LAYER_NAMES_SINE_ELU = {
    "actor": LAYER_NAMES["actor"],
    "critic": ["sinusodial_representation_dense", "dense_3", "sinusodial_representation_dense_1", "dense_4",
               "dense_5"],
    "target": ["sinusodial_representation_dense_2", "dense_6", "sinusodial_representation_dense_3", "dense_7",
               "dense_8"],
}


class Net:
    """Keras-model stand-in: weights live on the device in the net-buffer layout."""

    def __init__(self, sys, kind, role=None):
        self.sys = sys
        self.kind = kind
        self.role = role or ("actor" if kind == ACTOR else "critic")
        self.shapes = layer_shapes(kind, sys.ns, sys.na)
        self.P = sys.param_count(kind)
        assert self.P == sum(int(np.prod(s)) for s in self.shapes)
        self.buf = torch.zeros(sys.netbuf_floats(kind), dtype=torch.float32, device=DEVICE)
        # the critic activations belong to the system handle: a critic net fixes them (System.set_critic_type)
        self.critic_type = getattr(sys, "critic_type", "sine") if kind == CRITIC else None
        if kind == CRITIC:
            if getattr(sys, "critic_nets", None) is None:
                import weakref
                sys.critic_nets = weakref.WeakSet()
            sys.critic_nets.add(self)

    @property
    def flat(self):
        return self.buf[:self.P]

    def pack(self):
        L.lib().call("cacto_mlp_pack", self.sys.handle, self.kind, dptr(self.buf), stream())

    def set_weights(self, weights):
        flat = np.concatenate([np.asarray(w, dtype=np.float32).reshape(-1) for w in weights])
        if flat.size != self.P:
            raise ValueError("expected %d parameters, got %d" % (self.P, flat.size))
        self.flat.copy_(torch.from_numpy(flat))
        self.pack()

    def get_weights(self):
        flat = self.flat.detach().cpu().numpy()
        out, off = [], 0
        for s in self.shapes:
            n = int(np.prod(s))
            out.append(flat[off:off + n].reshape(s).copy())
            off += n
        return out

    def split(self, flat):
        """Views of a flat Keras-order vector (parameters or gradients) per trainable variable."""
        out, off = [], 0
        for sh in self.shapes:
            n = int(np.prod(sh))
            out.append(flat[off:off + n].reshape(sh))
            off += n
        return out

    @property
    def trainable_variables(self):
        """Keras `model.trainable_variables`: device views of the flat parameters (kernels [in,out])."""
        return self.split(self.flat)

    variables = trainable_variables

    def copy_from(self, other):
        self.buf.copy_(other.buf)

    def save_weights(self, path):
        """Keras `save_weights` (RL.py:191-195): a Keras-2.11 .h5 file for a `.h5` path (native
        writer, cacto_amd/h5.py), else an .npz of the Keras-order arrays."""
        ws = self.get_weights()
        if str(path).endswith(".h5"):
            names = (LAYER_NAMES_SINE_ELU if self.critic_type == "sine-elu" else LAYER_NAMES)[self.role]
            h5.write_keras_weights(path, [(n, [(n + "/kernel:0", ws[2 * i]), (n + "/bias:0", ws[2 * i + 1])])
                                          for i, n in enumerate(names)])
        else:
            np.savez(path, *ws)

    def load_weights(self, path):
        """Keras `load_weights` (main.py:154-158, RL.py:52-62): a reference .h5 checkpoint or .npz."""
        if str(path).endswith(".h5"):
            self.set_weights(h5.read_keras_weights(path))
            return
        z = np.load(path)
        self.set_weights([z["arr_%d" % i] for i in range(len(self.shapes))])


def init_weights(kind, ns, na, rng, critic_acts=("sine",) * 4):
    """Keras initialisers: Glorot-uniform kernels / zero biases for Dense; tf_siren
    SinusodialRepresentationDense (w0 = 1, c = 6): kernel U(+-sqrt(6/fan_in)), bias he_uniform
    U(+-sqrt(6/units)). `critic_acts`: the critic's hidden layers ('sine' SIREN layers, 'elu' Dense
    layers: NeuralNetwork.py:80-93)."""
    ws = []
    shapes = layer_shapes(kind, ns, na)
    for li in range(0, len(shapes), 2):
        fi, fo = shapes[li]
        siren = kind == CRITIC and li < 8 and critic_acts[li // 2] == "sine"
        lim = np.sqrt(6.0 / fi) if siren else np.sqrt(6.0 / (fi + fo))
        ws.append(rng.uniform(-lim, lim, size=(fi, fo)).astype(np.float32))
        b = rng.uniform(-np.sqrt(6.0 / fo), np.sqrt(6.0 / fo), size=fo) if siren else np.zeros(fo)
        ws.append(b.astype(np.float32))
    return ws


class NN:
    """NeuralNetwork.py:10-233 surface."""

    def __init__(self, env, conf, w_S=0, seed=0):
        self.env = env
        self.conf = conf
        self.w_S = w_S
        self.sys = env.sys
        self.rng = np.random.default_rng(seed)

    def create_actor(self):
        net = Net(self.sys, ACTOR)
        net.set_weights(init_weights(ACTOR, self.sys.ns, self.sys.na, self.rng))
        return net

    def create_critic_sine(self):
        self.sys.set_critic_type("sine")
        net = Net(self.sys, CRITIC)
        net.set_weights(init_weights(CRITIC, self.sys.ns, self.sys.na, self.rng))
        return net

    def create_critic_sine_elu(self):
        """NeuralNetwork.py:80-93: sine (64), elu (64), sine (128), elu (128) hidden layers + Dense(1).
        The activation is a property of the system handle (cacto_sys_set_critic_type), so every
        critic of this system — the target too — takes it."""
        self.sys.set_critic_type("sine-elu")
        net = Net(self.sys, CRITIC)
        net.set_weights(init_weights(CRITIC, self.sys.ns, self.sys.na, self.rng, critic_acts=SINE_ELU))
        return net

    def create_critic_elu(self):
        raise NotImplementedError("critic_type 'elu' (16, 32, 256, 256 wide) is not built; every shipped conf "
                                  "uses 'sine' ('sine-elu' is built)")

    create_critic_relu = create_critic_elu

    # ---- NeuralNetwork.py:130-138 ----
    def eval(self, model, x):
        S = torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x,
                            dtype=torch.float32, device=DEVICE).contiguous()
        if S.dim() == 1:
            S = S[None]
        B = S.shape[0]
        if model.kind == ACTOR:
            out = torch.empty(B, self.sys.na, dtype=torch.float32, device=DEVICE)
            L.lib().call("cacto_actor_forward", self.sys.handle, dptr(model.buf), dptr(S), dptr(out), B, stream())
            return out
        out = torch.empty(B, dtype=torch.float32, device=DEVICE)
        L.lib().call("cacto_critic_forward", self.sys.handle, dptr(model.buf), dptr(S), dptr(out), B, stream())
        return out.reshape(B, 1)

    def critic_input_grad(self, model, x):
        """tape.gradient(V(s), s) for a batch (NeuralNetwork.py:162-165, :190-195)."""
        S = torch.as_tensor(x, dtype=torch.float32, device=DEVICE).contiguous()
        B = S.shape[0]
        V = torch.empty(B, dtype=torch.float32, device=DEVICE)
        g = torch.empty(B, self.sys.ns, dtype=torch.float32, device=DEVICE)
        L.lib().call("cacto_critic_input_grad", self.sys.handle, dptr(model.buf), dptr(S), dptr(V), dptr(g), B,
                     stream())
        return V.reshape(B, 1), g

    # ---- NeuralNetwork.py:150-233 with the reference's signatures ----
    @staticmethod
    def _rows(state, R, state_next, dVdx, d, term):
        f = lambda x: torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x,
                                      device=DEVICE).to(torch.float64).reshape(len(state), -1)
        return torch.cat([f(state), f(R), f(state_next), f(dVdx), f(d), f(term)], dim=1).contiguous()

    def _cfg(self, B):
        cfg = L.UpdateCfg()
        cfg.w_S = float(self.w_S)
        cfg.MC = int(self.conf.MC)
        cfg.B_global = int(B)
        cfg.want_target_V = 1
        return cfg

    def _scratch(self, B):
        """Workspace and a private optimizer-counter pair for the standalone gradient calls: the
        device gradient kernels advance `step_d` (the fused update's Keras iterations), which a
        bare compute_*_grad must not do to the learner's counters."""
        if getattr(self, "_ws_B", 0) < B:
            self._ws = torch.empty(self.sys.workspace_bytes(B) // 4 + 64, dtype=torch.float32, device=DEVICE)
            self._ws_B = B
            self._steps = torch.zeros(2, dtype=torch.int32, device=DEVICE)
        return self._ws, self._steps

    def _nets(self, actor=None, critic=None, target=None):
        ws, steps = self._scratch(1)
        fill = (critic or actor).buf
        p = lambda n: (n.buf if n is not None else fill).data_ptr()
        scratch = ws.data_ptr()   # Adam moments are never touched by the gradient kernels
        return L.Nets(p(actor), scratch, scratch, p(critic), scratch, scratch, p(target), steps.data_ptr())

    def compute_critic_grad(self, critic_model, target_critic, state_batch, state_next_rollout_batch,
                            partial_reward_to_go_batch, dVdx_batch, d_batch, weights_batch):
        """NeuralNetwork.py:150-178. Returns (critic_grad [Keras trainable_variables order],
        reward_to_go_batch [B,1], critic_value [B,1], V_target(state_batch) [B,1])."""
        B = len(state_batch)
        rows = self._rows(state_batch, partial_reward_to_go_batch, state_next_rollout_batch, dVdx_batch, d_batch,
                          np.zeros(B))
        ws, _ = self._scratch(B)
        nets = self._nets(critic=critic_model, target=target_critic)
        idx = torch.arange(B, dtype=torch.int32, device=DEVICE)
        w = torch.as_tensor(np.asarray(weights_batch) if not isinstance(weights_batch, torch.Tensor) else weights_batch,
                            dtype=torch.float32, device=DEVICE).reshape(B).contiguous()
        grad = torch.empty(critic_model.P, dtype=torch.float32, device=DEVICE)
        y = torch.empty(B, dtype=torch.float32, device=DEVICE)
        V, Vt = torch.empty_like(y), torch.empty_like(y)
        L.lib().call("cacto_critic_grad", self.sys.handle, C.byref(nets), C.byref(self._cfg(B)),
                     dptr(rows, torch.float64), dptr(idx, torch.int32), dptr(w), B, dptr(grad), dptr(y), dptr(V),
                     dptr(Vt), dptr(ws), ws.numel() * 4, stream())
        return critic_model.split(grad), y.reshape(B, 1), V.reshape(B, 1), Vt.reshape(B, 1)

    def compute_actor_grad(self, actor_model, critic_model, state_batch, term_batch, batch_size=None):
        """NeuralNetwork.py:180-233: grads of mean_b(-dQ/da_b . pi(s_b)) against `critic_model`.
        `batch_size` only shapes the reference's reshapes; the mean is over len(state_batch)."""
        B = len(state_batch)
        if batch_size is not None and int(batch_size) != B:
            raise ValueError("compute_actor_grad: batch_size %d != len(state_batch) %d" % (batch_size, B))
        z = np.zeros((B, self.sys.ns))
        rows = self._rows(state_batch, np.zeros(B), z, z, np.zeros(B), term_batch)
        ws, _ = self._scratch(B)
        nets = self._nets(actor=actor_model, critic=critic_model, target=critic_model)
        idx = torch.arange(B, dtype=torch.int32, device=DEVICE)
        grad = torch.empty(actor_model.P, dtype=torch.float32, device=DEVICE)
        L.lib().call("cacto_actor_grad", self.sys.handle, C.byref(nets), C.byref(self._cfg(B)),
                     dptr(rows, torch.float64), dptr(idx, torch.int32), B, dptr(grad), dptr(ws), ws.numel() * 4,
                     stream())
        return actor_model.split(grad)
