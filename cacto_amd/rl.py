"""RL_AC with the reference surface (RL.py:6-233) on the HIP kernels.

The update hot loop (learn_and_update, RL.py:120-143) runs entirely on the device: per iteration
one `cacto_update` (critic chain -> weight-grad GEMM -> Adam + soft target update -> actor chain
-> weight-grad GEMM -> Adam), reading replay rows in place by index. Indices for the whole loop
are drawn up front (the reference draws them with the unseeded global numpy RNG,
replay_buffer.py:45) and copied once, so the loop enqueues work with no host synchronisation.
"""
import ctypes as C
import os
import math

import numpy as np
import torch

from . import _lib as L
from .neural_network import ACTOR, CRITIC, Net
from .system import DEVICE, dptr, stream


def dp_update_step(critic_grad, actor_grad, apply, all_reduce, soft_update):
    """One data-parallel RL_AC.update (RL.py:101-111) + update_target (RL.py:113-118).

    Every rank holds replicated weights and a local minibatch; the gradient callables return flat
    gradients whose losses are already normalised by the GLOBAL batch, so the exchange is a plain
    sum. Order (the reference's): critic gradient -> all-reduce -> critic Adam (+ soft target
    update) -> actor gradient against the UPDATED critic -> all-reduce -> actor Adam.
    """
    gc = critic_grad()
    all_reduce(gc)
    apply("critic", gc, soft_update)
    ga = actor_grad()
    all_reduce(ga)
    apply("actor", ga, False)


class _Done:
    """The handle of an exchange that completed when it was issued (a synchronous all-reduce)."""

    def wait(self):
        return True


def dp_pipeline(K, stages, all_reduce, apply):
    """K data-parallel updates (RL.py:101-118 each) with the gradient exchange off the critical path.

    Step t = 0..K forms the gradient of the critic step of update t (c = t, absent at t = K) and of
    the actor step of update t - 1 (a = t - 1, absent at t = 0), then applies both Adam steps. The
    critic step of update t never reads the actor, and the actor step of update t - 1 sees the
    critic after its update t - 1 — the ordering RL.py:104-109 prescribes — so the K updates equal
    the sequential loop. Gradients are normalised by the GLOBAL batch, so the exchange is a plain
    sum.

    stages(c, a) is a generator that yields ("critic", g) / ("actor", g) as each part is formed
    (critic first); each part's all-reduce is issued the moment it is yielded — all_reduce(g)
    returns a handle with wait() (torch.distributed async work; RCCL runs it on its own stream
    after the work already queued) — so the critic's exchange overlaps the forming of the actor
    gradient, and the actor's exchange overlaps the critic Adam step. apply(which, step, g) runs
    after that part's wait(), critic before actor, as the sequential loop has them.
    """
    for t in range(K + 1):
        c = t if t < K else None
        a = t - 1 if t > 0 else None
        pending = []
        for which, g in stages(c, a):
            h = all_reduce(g)
            pending.append((which, g, h if h is not None else _Done()))
        for which, g, h in pending:
            h.wait()
            apply(which, c if which == "critic" else a, g)


class Adam:
    """tf.keras.optimizers.Adam surface (RL.py:79-88) over the device Keras-2.11 Adam step
    (`cacto_adam_step`, with the learner's PiecewiseConstantDecay schedule when LR_SCHEDULE)."""

    def __init__(self, learner, which):
        self.learner = learner
        self.which = which

    @property
    def iterations(self):
        return int(self.learner.steps[0 if self.which == CRITIC else 1].item())

    def apply_gradients(self, grads_and_vars):
        """optimizer.apply_gradients(zip(grads, model.trainable_variables)) (RL.py:105, :109)."""
        grads = [g for g, _ in grads_and_vars]
        flat = torch.cat([torch.as_tensor(g, dtype=torch.float32, device=DEVICE).reshape(-1) for g in grads])
        model = self.learner.critic_model if self.which == CRITIC else self.learner.actor_model
        if flat.numel() != model.P:
            raise ValueError("apply_gradients: %d gradient values for a model of %d parameters" % (flat.numel(), model.P))
        # the device Adam reads the counter as Keras `iterations + 1` (the fused update's gradient
        # kernels advance it; a standalone apply_gradients advances it here)
        self.learner.steps[0 if self.which == CRITIC else 1] += 1
        self.learner.apply_gradients(self.which, flat)


class RL_AC:
    def __init__(self, env, NN, conf, N_try=0, w_S=None):
        self.env = env
        self.NN = NN
        self.conf = conf
        self.N_try = N_try
        self.sys = env.sys
        self.w_S = NN.w_S if w_S is None else w_S
        self.actor_model = None
        self.critic_model = None
        self.target_critic = None
        self.NSTEPS_SH = 0
        self._ws = None
        self._ws_B = 0

    # ---- RL.py:61-99 ----
    def setup_model(self, recover_training=None, weights=None):
        """`weights`: optional dict {'actor', 'critic', 'target'} of Keras-order arrays (e.g. the
        .h5-derived fixtures) instead of fresh initialisers."""
        self.actor_model = self.NN.create_actor()
        # RL.py:65-76 (critic_type: 'sine' in every shipped config; 'sine-elu' built; 'elu' / 'relu'
        # raise NotImplementedError)
        ctype = getattr(self.conf, "critic_type", "sine")
        create = {"sine": self.NN.create_critic_sine, "sine-elu": self.NN.create_critic_sine_elu,
                  "elu": self.NN.create_critic_elu}.get(ctype, self.NN.create_critic_relu)
        self.critic_model = create()
        self.target_critic = Net(self.sys, CRITIC, role="target")
        if weights is not None:
            self.actor_model.set_weights(weights["actor"])
            self.critic_model.set_weights(weights["critic"])
            self.target_critic.set_weights(weights.get("target", weights["critic"]))
        elif recover_training is not None:
            # RL.py:88-92: <path>/N_try_<n>/{actor,critic,target_critic}_<step>.h5 (the reference's
            # checkpoints load directly); .npz files of an earlier run of this package also work
            path, n_try, step = recover_training
            for net, name in ((self.actor_model, "actor"), (self.critic_model, "critic"),
                              (self.target_critic, "target_critic")):
                base = "%s/N_try_%s/%s_%s" % (path, n_try, name, step)
                net.load_weights(base + ".h5" if os.path.exists(base + ".h5") else base + ".npz")
        else:
            self.target_critic.copy_from(self.critic_model)       # RL.py:99
        f32 = dict(dtype=torch.float32, device=DEVICE)
        self.actor_m = torch.zeros(self.actor_model.P, **f32)
        self.actor_v = torch.zeros(self.actor_model.P, **f32)
        self.critic_m = torch.zeros(self.critic_model.P, **f32)
        self.critic_v = torch.zeros(self.critic_model.P, **f32)
        self.steps = torch.zeros(2, dtype=torch.int32, device=DEVICE)  # Keras optimizer iterations
        self.nets = L.Nets(self.actor_model.buf.data_ptr(), self.actor_m.data_ptr(), self.actor_v.data_ptr(),
                           self.critic_model.buf.data_ptr(), self.critic_m.data_ptr(), self.critic_v.data_ptr(),
                           self.target_critic.buf.data_ptr(), self.steps.data_ptr())
        self.cfg = self.make_cfg()
        self.critic_optimizer = Adam(self, CRITIC)
        self.actor_optimizer = Adam(self, ACTOR)

    def make_cfg(self, B_global=None):
        c = self.conf
        cfg = L.UpdateCfg()
        cfg.w_S = float(self.w_S)
        cfg.tau = float(c.UPDATE_RATE)
        cfg.beta1, cfg.beta2, cfg.epsilon = 0.9, 0.999, 1e-7        # Keras Adam defaults
        if c.LR_SCHEDULE:                                          # PiecewiseConstantDecay, RL.py:80-85
            for k in range(5):
                cfg.critic_lr[k] = c.values_schedule_LR_C[k]
                cfg.actor_lr[k] = c.values_schedule_LR_A[k]
            for k in range(4):
                cfg.lr_bounds[k] = c.boundaries_schedule_LR_C[k]
        else:
            for k in range(5):
                cfg.critic_lr[k] = c.CRITIC_LEARNING_RATE
                cfg.actor_lr[k] = c.ACTOR_LEARNING_RATE
            for k in range(4):
                cfg.lr_bounds[k] = float("inf")
        cfg.MC = int(c.MC)
        cfg.B_global = int(B_global or c.BATCH_SIZE)
        cfg.want_target_V = 0
        return cfg

    def workspace(self, B):
        if self._ws is None or self._ws_B < B:
            nbytes = self.sys.workspace_bytes(B)
            self._ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=DEVICE)
            self._ws_B = B
        return self._ws

    def _cfg_for(self, B, want_vt=False):
        """Loss means are over the global batch: B per rank times the data-parallel world."""
        cfg = L.UpdateCfg.from_buffer_copy(self.cfg)
        cfg.B_global = B * self.dp_world
        cfg.want_target_V = int(want_vt)
        return cfg

    dp_world = 1
    dp_group = None
    _dp_native = False

    def set_data_parallel(self, world_size, group=None):
        """Replicated weights, local minibatch per rank, all-reduce of the gradients. An explicit
        `group` selects the exchange path even for world_size 1 (a one-rank RCCL group: the path
        the one-GPU box can run).

        Over RCCL (a process group of backend 'nccl') the K updates of a call run in the library
        (cacto_update_n_dp / cacto_update_n_per_dp): the two-stream pipeline of cacto_update_n
        with each network's gradient all-reduced on its own stream's RCCL communicator, created
        here (cacto_dp_attach; rank 0's unique ids broadcast over the group). Otherwise (gloo: the
        CPU tests and the one-GPU multi-rank rehearsal), or with CACTO_DP_NATIVE=0, the host loop
        dp_pipeline: per update [critic gradient of update t | actor gradient of update t-1], the
        critic part's all-reduce issued as soon as it is formed. Both keep RL.py:104-109's order
        (the actor gradient is taken against the critic after its own update)."""
        self.dp_world = int(world_size)
        self.dp_group = group
        self._dp_native = False
        if not self._dp or os.environ.get("CACTO_DP_NATIVE", "1") == "0":
            return
        import torch.distributed as dist
        if not dist.is_initialized() or dist.get_backend(group) != "nccl":
            return
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        if world != self.dp_world and group is None:
            raise ValueError("set_data_parallel(%d): the default process group has %d ranks" % (self.dp_world, world))
        ids = C.create_string_buffer(2 * 128)
        if rank == 0:
            L.lib().call("cacto_dp_unique_ids", ids, 2)
        obj = [ids.raw]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        ids = C.create_string_buffer(obj[0], 2 * 128)
        L.lib().call("cacto_dp_attach", self.sys.handle, ids, rank, world)
        self._dp_native = True

    @property
    def _dp(self):
        return self.dp_world > 1 or self.dp_group is not None

    # ---- gradient pieces (explicit rows; used by the DP path and the parity tests) ----
    def critic_grad_flat(self, rows, idx, w=None, y=None, V=None, Vt=None):
        B = idx.shape[0]
        ws = self.workspace(B)
        grad = torch.empty(self.critic_model.P, dtype=torch.float32, device=DEVICE)
        cfg = self._cfg_for(B, Vt is not None)
        L.lib().call("cacto_critic_grad", self.sys.handle, C.byref(self.nets), C.byref(cfg),
                     dptr(rows, torch.float64), dptr(idx, torch.int32), dptr(w), B, dptr(grad), dptr(y), dptr(V),
                     dptr(Vt), dptr(ws), ws.numel() * 4, stream())
        return grad

    def actor_grad_flat(self, rows, idx):
        B = idx.shape[0]
        ws = self.workspace(B)
        grad = torch.empty(self.actor_model.P, dtype=torch.float32, device=DEVICE)
        cfg = self._cfg_for(B)
        L.lib().call("cacto_actor_grad", self.sys.handle, C.byref(self.nets), C.byref(cfg), dptr(rows, torch.float64),
                     dptr(idx, torch.int32), B, dptr(grad), dptr(ws), ws.numel() * 4, stream())
        return grad

    def critic_grad_rows(self, rows, idx, w=None, want_vt=True):
        B = idx.shape[0]
        y = torch.empty(B, dtype=torch.float32, device=DEVICE)
        V, Vt = torch.empty_like(y), torch.empty_like(y)
        grad = self.critic_grad_flat(rows, idx, w, y, V, Vt if want_vt else None)
        return self.critic_model.split(grad), y.reshape(B, 1), V.reshape(B, 1), Vt.reshape(B, 1)

    def actor_grad_rows(self, rows, idx, batch_size=None):
        return self.actor_model.split(self.actor_grad_flat(rows, idx))

    def apply_gradients(self, which, flat_grad, soft_update=False):
        """optimizer.apply_gradients (RL.py:105/:109) for a flat gradient (after the grad call that
        advanced the iteration counter)."""
        L.lib().call("cacto_adam_step", self.sys.handle, C.byref(self.nets), C.byref(self.cfg), which,
                     dptr(flat_grad.contiguous(), torch.float32), int(soft_update), stream())

    # ---- RL.py:101-111 on replay rows ----
    def update_rows(self, storage, idx, is_w=None, y=None, V=None, Vt=None):
        if self._dp:
            return self._update_rows_dp(storage, idx, is_w, y, V, Vt)
        B = idx.shape[0]
        ws = self.workspace(B)
        cfg = self._cfg_for(B, Vt is not None)
        L.lib().call("cacto_update", self.sys.handle, C.byref(self.nets), C.byref(cfg), dptr(storage, torch.float64),
                     dptr(idx, torch.int32), dptr(is_w), B, dptr(y), dptr(V), dptr(Vt), dptr(ws), ws.numel() * 4,
                     stream())

    def update_rows_n(self, storage, idx_steps):
        """len(idx_steps) consecutive RL.py:101-118 updates on the minibatch indices idx_steps [K, B]
        (int32, device) in one call: `cacto_update_n` overlaps the critic step of update t+1 with the
        actor step of update t on a second stream (the critic step never reads the actor), with
        results bit-identical to K update_rows calls. Single rank (the data-parallel update
        all-reduces between the two steps)."""
        if self._dp:
            return self._update_rows_n_dp(storage, idx_steps)
        K, B = int(idx_steps.shape[0]), int(idx_steps.shape[1])
        ws = self.workspace(B)
        cfg = self._cfg_for(B)
        L.lib().call("cacto_update_n", self.sys.handle, C.byref(self.nets), C.byref(cfg), dptr(storage, torch.float64),
                     dptr(idx_steps.contiguous(), torch.int32), K, B, dptr(ws), ws.numel() * 4, stream())

    def update_rows_n_per(self, buffer, uniforms):
        """learn_and_update's PER loop (RL.py:122-137) for K = len(uniforms) updates in one call
        (`cacto_update_n_per`): per update the stratified sample from uniforms[k] ([K, B] f64 on the
        device, the reference's random.random() draws in order), the update with IS weights and the
        priority update, pipelined with the actor steps; bit-identical to the sequential loop.
        Single rank (the data-parallel PER exchange runs per sample call)."""
        K, B = int(uniforms.shape[0]), int(uniforms.shape[1])
        ws = self.workspace(B)
        cfg = self._cfg_for(B)
        u = uniforms.to(device=DEVICE, dtype=torch.float64).contiguous()
        b = buffer
        L.lib().call("cacto_update_n_per", self.sys.handle, C.byref(self.nets), C.byref(cfg),
                     dptr(b.storage, torch.float64), dptr(b.sum_tree), dptr(b.min_tree), b.cap, b.max_idx(), b.beta,
                     dptr(u), dptr(b.exp_counter), b.fresh, b.eps, b.alpha, dptr(b.max_priority), K, B, dptr(ws),
                     ws.numel() * 4, stream())

    def capture_updates(self, storage, idx_steps, per_buffer=None, uniforms=None):
        """One HIP graph of len(idx_steps) consecutive RL.py:101-118 updates (critic chain ->
        weight-gradient GEMM -> Adam + soft update -> actor chain -> GEMM -> Adam per step), captured
        without running; `graph.replay()` runs them in order. Every launch of the loop is a kernel
        on the current stream and the optimiser counters live on the device, so replaying the graph
        is the same work as calling update_rows per step, without the per-launch host cost.
        idx_steps [K, B] int32 (device, kept alive by the caller). With `per_buffer` (a
        PrioritizedReplayBuffer) each step instead samples from `uniforms[k]` ([K, B] f64) and
        updates the priorities (learn_and_update with PER, RL.py:122-137).
        Data parallel (RCCL process group): the graph holds the dp_pipeline loop — stage kernels,
        the all-reduces on RCCL's stream and the Adam steps joined by stream waits — since nothing
        in it waits on the host (gloo's collectives run on the host and cannot be captured)."""
        K = (uniforms if per_buffer is not None else idx_steps).shape[0]
        B = (uniforms if per_buffer is not None else idx_steps).shape[1]
        self.workspace(B)                       # allocated before the capture
        if self._dp:
            import torch.distributed as dist
            if dist.get_backend(self.dp_group) != "nccl":
                raise RuntimeError("capture_updates: a data-parallel loop is captured only over RCCL (backend "
                                   "'nccl'), not %r" % dist.get_backend(self.dp_group))
            self._dp_grad_buf(self.critic_model.P + self.actor_model.P)
            keep = None
            if per_buffer is not None:
                # the uniforms on the device before the capture (a host tensor cannot be copied inside
                # it), and the loop's y / V allocated here and kept alive with the graph
                uniforms = uniforms.to(device=DEVICE, dtype=torch.float64).contiguous()
                keep = (uniforms, torch.empty(B, dtype=torch.float32, device=DEVICE),
                        torch.empty(B, dtype=torch.float32, device=DEVICE))
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                if per_buffer is None:
                    self._update_rows_n_dp(storage, idx_steps)
                else:
                    self.update_rows_n_per_dp(per_buffer, keep[0], y=keep[1], V=keep[2])
            g.keep = keep
            return g
        y = torch.empty(B, dtype=torch.float32, device=DEVICE)
        V = torch.empty_like(y)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for k in range(K):
                if per_buffer is None:
                    self.update_rows(storage, idx_steps[k])
                else:
                    idx, w = per_buffer.sample_device(uniforms[k])
                    self.update_rows(per_buffer.storage, idx, w, y, V)
                    if per_buffer.alpha != 0:       # RL.py:130
                        per_buffer.update_priorities_device(idx, y, V)
        g.keep = (y, V)
        return g

    def _update_rows_dp(self, storage, idx, is_w=None, y=None, V=None, Vt=None):
        if Vt is not None:      # the extra V_tgt(s) output: the two-exchange form
            import torch.distributed as dist
            dp_update_step(lambda: self.critic_grad_flat(storage, idx, is_w, y, V, Vt),
                           lambda: self.actor_grad_flat(storage, idx),
                           lambda which, g, soft: self.apply_gradients(CRITIC if which == "critic" else ACTOR, g,
                                                                       soft_update=soft),
                           lambda t: dist.all_reduce(t, group=self.dp_group),
                           soft_update=not self.conf.MC)
            return
        self._update_rows_n_dp(storage, idx.reshape(1, -1), is_w, y, V)

    def _update_rows_n_dp(self, storage, idx_steps, is_w=None, y=None, V=None):
        """K data-parallel updates. Over RCCL: one cacto_update_n_dp call (the two-stream pipeline,
        each network's gradient all-reduced on its stream's communicator). Otherwise dp_pipeline:
        per step one C-ABI call for the paired gradients (critic of update t, actor of update t-1)
        into one buffer, the all-reduces through torch.distributed, one call for the Adam steps.
        is_w / y / V only with K = 1 (PER)."""
        import torch.distributed as dist
        K, B = int(idx_steps.shape[0]), int(idx_steps.shape[1])
        if K != 1 and (is_w is not None or y is not None or V is not None):
            raise ValueError("_update_rows_n_dp: IS weights / y / V belong to one update (K == 1); "
                             "K PER updates go through update_rows_n_per_dp")
        ws = self.workspace(B)
        cfg = self._cfg_for(B)
        if self._dp_native and is_w is None and y is None and V is None:
            L.lib().call("cacto_update_n_dp", self.sys.handle, C.byref(self.nets), C.byref(cfg),
                         dptr(storage, torch.float64), dptr(idx_steps.contiguous(), torch.int32), K, B, dptr(ws),
                         ws.numel() * 4, stream())
            return
        Pc, Pa = self.critic_model.P, self.actor_model.P
        g = self._dp_grad_buf(Pc + Pa)
        idx_steps = idx_steps.contiguous()

        def stages(c, a):
            ic = idx_steps[c] if c is not None else None
            ia = idx_steps[a] if a is not None else None
            args = (self.sys.handle, C.byref(self.nets), C.byref(cfg), dptr(storage, torch.float64),
                    dptr(ic, torch.int32), dptr(is_w if c is not None else None), dptr(ia, torch.int32), B, dptr(g),
                    dptr(y if c is not None else None), dptr(V if c is not None else None), dptr(ws), ws.numel() * 4)
            L.lib().call("cacto_update_pair_grads_stage", *args, 0, stream())
            if c is not None:
                yield "critic", g[:Pc]
            if a is not None:
                L.lib().call("cacto_update_pair_grads_stage", *args, 1, stream())
                yield "actor", g[Pc:]
        dp_pipeline(K, stages, self._all_reduce_async, self._dp_apply(g, cfg))

    def _all_reduce_async(self, t):
        import torch.distributed as dist
        return dist.all_reduce(t, group=self.dp_group, async_op=True)

    def _dp_apply(self, g, cfg, after_critic=None):
        def apply(which, step, _):
            crit = which == "critic"
            L.lib().call("cacto_update_pair_apply", self.sys.handle, C.byref(self.nets), C.byref(cfg), dptr(g),
                         int(crit), int(not crit), int(crit and not self.conf.MC), stream())
            if crit and after_critic is not None:
                after_critic(step)
        return apply

    def update_rows_n_per_dp(self, buffer, uniforms, y=None, V=None):
        """K data-parallel PER updates (RL.py:122-137 on every rank's replay shard, the sampling of
        replay_buffer.py:139-188 over the union of the shards) in the paired schedule of
        dp_pipeline: step t samples update t (one all-gather of the shards' (sum, min, rows), then
        the stratified sample and IS weights, all on the device), computes [critic gradient of
        update t | actor gradient of update t - 1] into one buffer in two stages — the critic part's
        async all-reduce is issued before the actor part is formed, the actor part's after it —
        applies the critic's Adam step once its exchange is done (then the local priorities of
        update t), and the actor's once its own is. uniforms [K, B] (this
        rank's random.random() draws, in order) go to the device in one copy. Every kernel sees the
        inputs of the sequential loop (sample -> update -> priorities), so the result equals K
        update_rows + update_priorities_device calls (bit for bit when the collective's sums are
        order-independent, e.g. two ranks). Over RCCL the whole loop is one cacto_update_n_per_dp
        call (the shard statistics exchanged on the device per sample, the two-stream pipeline
        with in-stream all-reduces)."""
        import torch.distributed as dist
        K, B = int(uniforms.shape[0]), int(uniforms.shape[1])
        u = uniforms.to(device=DEVICE, dtype=torch.float64).contiguous()
        ws = self.workspace(B)
        cfg = self._cfg_for(B)
        if self._dp_native and buffer.dp_group is self.dp_group:
            # (y / V: the caller's scratch of the host loop; the library keeps its own)
            b = buffer
            L.lib().call("cacto_update_n_per_dp", self.sys.handle, C.byref(self.nets), C.byref(cfg),
                         dptr(b.storage, torch.float64), dptr(b.sum_tree), dptr(b.min_tree), b.cap, b.max_idx(),
                         b.beta, dptr(u), dptr(b.exp_counter), b.fresh, b.eps, b.alpha, dptr(b.max_priority), K, B,
                         dptr(ws), ws.numel() * 4, stream())
            return
        Pc, Pa = self.critic_model.P, self.actor_model.P
        g = self._dp_grad_buf(Pc + Pa)
        y = torch.empty(B, dtype=torch.float32, device=DEVICE) if y is None else y
        V = torch.empty_like(y) if V is None else V
        drawn = {}

        def stages(c, a):
            if c is not None:
                drawn[c] = buffer.sample_device(u[c])
                drawn.pop(c - 2, None)
            ic, wc = drawn[c] if c is not None else (None, None)
            ia = drawn[a][0] if a is not None else None
            args = (self.sys.handle, C.byref(self.nets), C.byref(cfg), dptr(buffer.storage, torch.float64),
                    dptr(ic, torch.int32), dptr(wc), dptr(ia, torch.int32), B, dptr(g),
                    dptr(y if c is not None else None), dptr(V if c is not None else None), dptr(ws), ws.numel() * 4)
            L.lib().call("cacto_update_pair_grads_stage", *args, 0, stream())
            if c is not None:
                yield "critic", g[:Pc]
            if a is not None:
                L.lib().call("cacto_update_pair_grads_stage", *args, 1, stream())
                yield "actor", g[Pc:]
        # RL.py:130: no priority update with alpha == 0 (the sampler's count still happens)
        prio = (lambda c: buffer.update_priorities_device(drawn[c][0], y, V)) if buffer.alpha != 0 else None
        dp_pipeline(K, stages, self._all_reduce_async, self._dp_apply(g, cfg, prio))

    def _dp_grad_buf(self, n):
        if getattr(self, "_dp_g", None) is None or self._dp_g.numel() < n:
            self._dp_g = torch.empty(n, dtype=torch.float32, device=DEVICE)
        return self._dp_g

    def update(self, state_batch, state_next_rollout_batch, partial_reward_to_go_batch, dVdx_batch, d_batch,
               term_batch, weights_batch, batch_size=None):
        """RL.py:101-111 surface on explicit tensors (+ update_target, which learn_and_update would
        call next). Returns (reward_to_go, critic_value, target_critic_value)."""
        B = len(state_batch)
        rows = self.NN._rows(state_batch, partial_reward_to_go_batch, state_next_rollout_batch, dVdx_batch, d_batch,
                             term_batch)
        idx = torch.arange(B, dtype=torch.int32, device=DEVICE)
        y = torch.empty(B, dtype=torch.float32, device=DEVICE)
        V, Vt = torch.empty_like(y), torch.empty_like(y)
        w = torch.as_tensor(weights_batch, dtype=torch.float32, device=DEVICE).reshape(B).contiguous()
        self.update_rows(rows, idx, w, y, V, Vt)
        return y.reshape(B, 1), V.reshape(B, 1), Vt.reshape(B, 1)

    def update_target(self, target_weights=None, weights=None):
        """RL.py:113-118 (standalone; cacto_update already fuses it into the critic Adam step)."""
        L.lib().call("cacto_soft_update", self.sys.handle, C.byref(self.nets), float(self.conf.UPDATE_RATE), stream())

    # ---- RL.py:120-143 ----
    def learn_and_update(self, update_step_counter, buffer, ep, rng=None):
        n = int(self.conf.UPDATE_LOOPS[ep])
        B = self.conf.BATCH_SIZE
        per = getattr(buffer, "prioritized", False)
        if per and getattr(buffer, "RB_type", "PER") == "ReLO":
            return self._learn_and_update_relo(update_step_counter, buffer, n, B)
        if per:
            if self._dp and (buffer.dp_world, buffer.dp_group) != (self.dp_world, self.dp_group):
                buffer.set_data_parallel(self.dp_world, self.dp_group)
            # the updates between two checkpoint saves as one pipelined call; the uniforms are the
            # per-step random.random() draws of the sequential loop, in the same order
            i = 0
            while i < n:
                k = min(n - i, self.conf.save_interval - update_step_counter % self.conf.save_interval)
                U = np.array([[buffer.random.random() for _ in range(B)] for _ in range(k)], dtype=np.float64)
                if not self._dp:
                    self.update_rows_n_per(buffer, torch.as_tensor(U, device=DEVICE))
                else:
                    self.update_rows_n_per_dp(buffer, torch.as_tensor(U, device=DEVICE))
                for _ in range(k):
                    update_step_counter = self._after_step(update_step_counter)
                i += k
            self.check_pipeline()
            return update_step_counter
        idx_all = buffer.sample_indices(n, rng)                  # [n, B] int32 on device
        # the updates between two checkpoint saves (RL.py:139-141) run as one pipelined call
        i = 0
        while i < n:
            k = min(n - i, self.conf.save_interval - update_step_counter % self.conf.save_interval)
            self.update_rows_n(buffer.storage, idx_all[i:i + k])
            for _ in range(k):
                update_step_counter = self._after_step(update_step_counter)
            i += k
        self.check_pipeline()
        return update_step_counter

    def check_pipeline(self):
        """Raise if a device-side wait of the two-stream update pipeline timed out since the last
        check (cacto_pipeline_check: synchronizes the current stream, clears the latch): the
        updates of that call ran without their cross-stream order (RL.py:104-109 orders critic(t)
        before actor(t)), so their weights must not be used. learn_and_update calls it before it
        returns, RL_save_weights before it writes a checkpoint."""
        L.lib().call("cacto_pipeline_check", self.sys.handle, stream())

    def _learn_and_update_relo(self, update_step_counter, buffer, n, B):
        """RL.py:120-143 with RB_type 'ReLO' (replay_buffer.py:193-196): the priority rule needs
        V_tgt(s) from the update (want_target_V), so the loop runs update by update — sample,
        update (with y, V, V_tgt), priorities — instead of the pipelined PER call."""
        if self._dp and (buffer.dp_world, buffer.dp_group) != (self.dp_world, self.dp_group):
            buffer.set_data_parallel(self.dp_world, self.dp_group)
        y = torch.empty(B, dtype=torch.float32, device=DEVICE)
        V, Vt = torch.empty_like(y), torch.empty_like(y)
        for _ in range(n):
            U = torch.as_tensor(np.array([buffer.random.random() for _ in range(B)], dtype=np.float64), device=DEVICE)
            idx, w = buffer.sample_device(U)
            self.update_rows(buffer.storage, idx, w, y, V, Vt)
            if buffer.alpha != 0:                   # RL.py:130
                buffer.update_priorities_device(idx, y, V, Vt)
                buffer.check_priorities()           # replay_buffer.py:212 assert priority > 0
            update_step_counter = self._after_step(update_step_counter)
        return update_step_counter

    def _after_step(self, counter):
        counter += 1
        if counter % self.conf.save_interval == 0 and getattr(self.conf, "NNs_path", None):
            self.RL_save_weights(counter)
        return counter

    # ---- RL.py:145-189 (host, float64 as the reference) ----
    def RL_Solve(self, TO_controls, TO_states, TO_step_cost):
        """One episode's n-step targets. Returns (state_arr, partial_reward_to_go_arr,
        total_reward_to_go_arr, state_next_rollout_arr, done_arr, rwrd_arr, term_arr, ep_return,
        ee_pos_arr). With env_RL the episode is re-simulated from TO_controls on the device
        (RL.py:157-165: Env.step with the running weights, EE of every state, terminal reward);
        otherwise states and rewards are the TO's (RL.py:166-167) and ee_pos_arr is the array
        create_TO_init started (row 0 = EE(s_0); the reference leaves the other rows unset —
        np.empty — and main.py:192-193 replaces it with the TO's EE positions)."""
        T = self.NSTEPS_SH
        ns = self.conf.nb_state
        self.control_arr = TO_controls
        if self.conf.env_RL:
            S, rwrd, EE = self._env_rl_episode(np.asarray(TO_controls, dtype=np.float64), T)
            self.state_arr, self.ee_pos_arr = S, EE
        else:
            self.state_arr = TO_states
            rwrd = -np.asarray(TO_step_cost, dtype=np.float64)
        s_next = np.zeros((T + 1, ns))
        partial = np.empty(T + 1)
        total = np.empty(T + 1)
        term = np.zeros(T + 1)
        term[-1] = 1
        done = np.zeros(T + 1)
        for i in range(T + 1):
            if self.conf.MC:
                final = T
                done[i] = 1
            else:
                final = min(i + self.conf.nsteps_TD_N, T)
                if final == T:
                    done[i] = 1
                else:
                    s_next[i, :] = self.state_arr[final + 1, :]
            partial[i] = np.float32(sum(rwrd[i:final + 1]))
            total[i] = np.float32(sum(rwrd[i:T + 1]))
        ep_return = sum(rwrd)
        return self.state_arr, partial, total, s_next, done, rwrd, term, ep_return, self.ee_pos_arr

    def _env_rl_episode(self, controls, T):
        """RL.py:157-165 on the device: s_{i+1}, r_i = Env.step(w_running, s_i, u_i),
        ee_{i+1} = EE(s_{i+1}); r_T = reward(w_terminal, s_T). One launch per step, no host sync."""
        ns = self.conf.nb_state
        S = torch.empty(T + 1, ns, dtype=torch.float64, device=DEVICE)
        S[0] = torch.as_tensor(np.asarray(self.state_arr[0], dtype=np.float64), device=DEVICE)
        R = torch.empty(T + 1, dtype=torch.float64, device=DEVICE)
        EE = torch.empty(T + 1, 3, dtype=torch.float64, device=DEVICE)
        U = torch.as_tensor(controls, device=DEVICE)
        W = torch.as_tensor(np.asarray(self.conf.cost_weights_running, dtype=np.float64), device=DEVICE)
        h = self.sys.handle
        for i in range(T):
            L.lib().call("cacto_env_step", h, dptr(S[i:i + 1]), dptr(U[i:i + 1].contiguous()), dptr(W),
                         dptr(S[i + 1:i + 2]), dptr(R[i:i + 1]), dptr(EE[i + 1:i + 2]), 1, stream())
        Wt = torch.as_tensor(np.asarray(self.conf.cost_weights_terminal, dtype=np.float64), device=DEVICE)
        zero = torch.zeros(1, self.conf.nb_action, dtype=torch.float64, device=DEVICE)
        L.lib().call("cacto_env_step", h, dptr(S[T:T + 1]), dptr(zero), dptr(Wt), None, dptr(R[T:T + 1]), None, 1,
                     stream())
        L.lib().call("cacto_env_ee", h, dptr(S[0:1]), dptr(EE[0:1]), 1, stream())
        return S.cpu().numpy(), R.cpu().numpy(), EE.cpu().numpy()

    def RL_save_weights(self, update_step_counter='final'):
        """RL.py:191-195: Keras-2.11 .h5 files the reference can load."""
        self.check_pipeline()
        base = "%s/N_try_%s/" % (self.conf.NNs_path, self.N_try)
        self.actor_model.save_weights(base + "actor_%s.h5" % update_step_counter)
        self.critic_model.save_weights(base + "critic_%s.h5" % update_step_counter)
        self.target_critic.save_weights(base + "target_critic_%s.h5" % update_step_counter)

    # ---- RL.py:197-233, batched over episodes on the GPU ----
    def rollout_inputs(self, S0, nsteps):
        """Device copies of the start states, lengths and the length-sorted episode order."""
        nsteps = np.asarray(nsteps, dtype=np.int32)
        order = np.argsort(-nsteps, kind="stable").astype(np.int32)
        return (torch.as_tensor(np.asarray(S0, dtype=np.float64), device=DEVICE).contiguous(),
                torch.as_tensor(nsteps, device=DEVICE).contiguous(), torch.as_tensor(order, device=DEVICE))

    def rollout_batch(self, S0, nsteps, T, ep=1, weights=None, want=("S", "A", "R", "EE"), inputs=None, out=None,
                      actor=None, sched=(0, 0)):
        """Roll out len(S0) episodes in one persistent kernel (K18); episode slots are refilled
        longest-first as episodes end. `actor` (an NN-held network, default self.actor_model) gives
        the policy; `sched` = (groups, workgroups) of cacto_rollout_sched (0 = automatic)."""
        S0, n, order = inputs if inputs is not None else self.rollout_inputs(S0, nsteps)
        R = S0.shape[0]
        ns, na = self.conf.nb_state, self.conf.nb_action
        if out is not None:
            return self._launch_rollout(S0, n, order, T, ep, weights, out, actor, sched)
        f64 = dict(dtype=torch.float64, device=DEVICE)
        out = {}
        # rewards and EE positions are evaluated from the recorded (s_t, a_t) after the rollout.
        # Zero-filled: the rows of an episode past its NSTEPS_SH are never written, and consumers
        # that take whole [R, T+1, .] blocks (DDP labels, RL_Solve, host copies) must not see junk.
        need_sa = "R" in want or "EE" in want
        if "S" in want or need_sa:
            out["S"] = torch.zeros(R, T + 1, ns, **f64)
        if "A" in want or (need_sa and ep != 0):
            out["A"] = torch.zeros(R, T, na, dtype=torch.float32, device=DEVICE)
        if "R" in want:
            out["R"] = torch.zeros(R, T, **f64)
        if "EE" in want:
            out["EE"] = torch.zeros(R, T + 1, 3, **f64)
        out["status"] = torch.empty(R, dtype=torch.int32, device=DEVICE)
        return self._launch_rollout(S0, n, order, T, ep, weights, out, actor, sched)

    def _launch_rollout(self, S0, n, order, T, ep, weights, out, actor=None, sched=(0, 0)):
        W = None if weights is None else torch.as_tensor(np.asarray(weights, dtype=np.float64), device=DEVICE)
        actor = self.actor_model if actor is None else actor
        L.lib().call("cacto_rollout_sched", self.sys.handle, dptr(actor.buf), dptr(S0), dptr(n), T,
                     int(ep != 0), dptr(W), dptr(out.get("S")), dptr(out.get("A")), dptr(out.get("R")),
                     dptr(out.get("EE")), dptr(out.get("status")), dptr(order), S0.shape[0], int(sched[0]),
                     int(sched[1]), stream())
        return out

    def rollout_rewards(self, out, n, T, ep=1, weights=None):
        """Rewards / EE positions of a recorded rollout (cacto_rollout_rewards) into out["R"] /
        out["EE"]: the second kernel of a rollout, launched on its own (bench times it apart)."""
        W = None if weights is None else torch.as_tensor(np.asarray(weights, dtype=np.float64), device=DEVICE)
        L.lib().call("cacto_rollout_rewards", self.sys.handle, dptr(out["S"]), dptr(out.get("A")), dptr(n), T,
                     int(ep != 0), dptr(W), dptr(out.get("R")), dptr(out.get("EE")), out["S"].shape[0], stream())
        return out

    def nsteps_sh(self, s0):
        return self.conf.NSTEPS - int(s0[-1] / self.conf.dt)

    def create_TO_init(self, ep, ICS):
        """RL.py:197-233 for one episode (one cacto_rollout launch). Returns (init_rand_state,
        init_TO_states, init_TO_controls, NSTEPS_SH, success_init_flag); leaves state_arr,
        control_arr and ee_pos_arr (row 0 = EE(ICS)) for RL_Solve as the reference does."""
        self.init_rand_state = ICS
        self.NSTEPS_SH = self.nsteps_sh(ICS)
        if self.NSTEPS_SH == 0:
            return None, None, None, None, 0
        T = self.NSTEPS_SH
        ns, na = self.conf.nb_state, self.conf.nb_action
        self.control_arr = np.empty((T, na))
        self.state_arr = np.empty((T + 1, ns))
        self.ee_pos_arr = np.zeros((T + 1, 3))
        self.state_arr[0, :] = ICS
        self.ee_pos_arr[0, :] = self.env.get_end_effector_position(self.state_arr[0, :])
        out = self.rollout_batch(np.asarray(ICS)[None], [T], T, ep=ep, want=("S", "A"))
        if int(out["status"][0].item()) != 0:
            return None, None, None, None, 0
        states = out["S"][0].cpu().numpy()
        controls = out["A"][0].double().cpu().numpy() if "A" in out else np.zeros((T, na))
        return self.init_rand_state, states, controls, self.NSTEPS_SH, 1

    def create_TO_init_batch(self, ep, ICS_list):
        """create_TO_init for every initial state of a main.py iteration (main.py:174-224 calls it
        once per episode) in ONE rollout launch and one device->host copy: returns the list of
        tuples create_TO_init returns, in order — (None, None, None, None, 0) for NSTEPS_SH == 0 or
        an episode dropped for a NaN state (RL.py:229-231). The per-episode attributes create_TO_init
        leaves for RL_Solve (state_arr, ee_pos_arr) are not set; batched callers take the device
        path (rollout_batch -> TO.backward_pass_batch -> ReplayBuffer.add_episodes)."""
        ICS = np.asarray(ICS_list, dtype=np.float64).reshape(len(ICS_list), -1)
        ns_ = [self.nsteps_sh(s) for s in ICS]
        fail = (None, None, None, None, 0)
        T = max(ns_) if ns_ else 0
        if T <= 0:
            return [fail for _ in ns_]
        na = self.conf.nb_action
        out = self.rollout_batch(ICS, ns_, T, ep=ep, want=("S", "A"))
        S, A, st = out["S"].cpu().numpy(), out["A"].double().cpu().numpy(), out["status"].cpu().numpy()
        res = []
        for k, n in enumerate(ns_):
            if n <= 0 or st[k] != 0:
                res.append(fail)
            else:
                res.append((ICS[k].copy(), S[k, :n + 1].copy(), A[k, :n].copy() if ep != 0 else np.zeros((n, na)),
                            n, 1))
        return res
