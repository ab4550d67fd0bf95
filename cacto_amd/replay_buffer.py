"""Replay buffers with the reference surface (replay_buffer.py:9-240), device-resident.

Storage is the reference's float64 row layout [s | R | s_next | dVdx | d | term] (3ns+3 columns,
replay_buffer.py:20) in HBM; sampling gathers rows on the GPU (or the update kernels read them in
place by index). The prioritized buffer keeps float64 sum/min segment trees on the GPU with the
reference's node layout and combination order (segment_tree.py) so sampled indices are bit-exact.
"""
import random

import numpy as np
import torch

from . import _lib as L
from .system import DEVICE, dptr, shared_system, stream


class ReplayBuffer:
    prioritized = False

    def __init__(self, conf, sys=None):
        """replay_buffer.py:10 `ReplayBuffer(conf)`; `sys` defaults to the conf's shared System."""
        self.conf = conf
        self.sys = sys if sys is not None else shared_system(conf)
        self.N = conf.REPLAY_SIZE
        self.ns = conf.nb_state
        self.cols = 3 * self.ns + 3
        self.storage = torch.zeros(self.N, self.cols, dtype=torch.float64, device=DEVICE)
        self.next_idx = 0
        self.full = 0
        self.np_rng = np.random  # the reference draws from the global numpy RNG (unseeded)

    @staticmethod
    def concatenate_sample(obses_t, rewards, obses_t1, dVdxs, dones, terms):
        """replay_buffer.py:63-72."""
        cat = lambda xs: np.concatenate(xs, axis=0)
        return np.concatenate((cat(obses_t), cat(rewards).reshape(-1, 1), cat(obses_t1), cat(dVdxs),
                               cat(dones).reshape(-1, 1), cat(terms).reshape(-1, 1)), axis=1)

    def add_rows(self, rows):
        rows = torch.as_tensor(rows, dtype=torch.float64, device=DEVICE).contiguous()
        n = rows.shape[0]
        if n == 0:
            return
        if n > self.N:
            raise ValueError("cannot add more rows than REPLAY_SIZE at once")
        L.lib().call("cacto_buffer_add", self.sys.handle, dptr(self.storage), self.N, self.next_idx, dptr(rows), n,
                     stream())
        self._advance(n)

    def _advance(self, n):
        start = self.next_idx
        if n + self.next_idx > self.N:
            self.full = 1
        self.next_idx = (self.next_idx + n) % self.N
        self._rows_added(start, n)

    def _rows_added(self, start, n):
        pass

    def _row_offsets(self, rows):
        """Exclusive prefix sum of the episode row counts on the device; the last batch's copy is
        reused when the counts repeat (one create_TO_init batch is added many times in a bench)."""
        key = rows.tobytes()
        if getattr(self, "_off_key", None) != key:
            off = np.zeros(len(rows) + 1, dtype=np.int64)
            np.cumsum(rows, out=off[1:])
            self._off_key, self._off = key, (torch.as_tensor(off, device=DEVICE), int(off[-1]))
        return self._off

    def add_episodes(self, S_traj, rewards, nsteps, R_term=None, dVdx=None, want_total=False, status=None):
        """RL_AC.RL_Solve (RL.py:145-189) for a batch of episodes, with the rows of each episode
        added in order as main.py:240 adds them, all on the device (cacto_rl_solve_add).

        S_traj [E, ldS, ns] f64 device (s_0..s_T per episode, e.g. cacto_rollout's S_traj);
        rewards [E, ldR] f64 device: r_0..r_T, or r_0..r_{T-1} with R_term [E] giving r_T;
        nsteps: host ints (NSTEPS_SH per episode); dVdx [E, ldS, ns] f64 device or None (zeros).
        status [E] (a rollout's, host or device): episodes with status != 0 hit a NaN state and are
        dropped as main.py:236 drops them (no rows; the kept episodes' rows stay contiguous, in
        order). Returns total_reward_to_go [E, ldS] (device) when want_total, else None."""
        nsteps = np.asarray(nsteps, dtype=np.int64)
        E = len(nsteps)
        if E == 0:
            return None
        rows = nsteps + 1
        if status is not None:
            st = status.cpu().numpy() if torch.is_tensor(status) else np.asarray(status)
            rows = np.where(st.reshape(-1) == 0, rows, 0)
            if not rows.any():
                return None
        off_d, n = self._row_offsets(rows)
        if n > self.N:
            raise ValueError("cannot add more rows than REPLAY_SIZE at once")
        f64 = lambda t: t.to(device=DEVICE, dtype=torch.float64).contiguous()
        S_traj, rewards = f64(S_traj), f64(rewards)
        if S_traj.dim() != 3 or S_traj.shape[0] != E or S_traj.shape[2] != self.ns or rewards.shape[0] != E:
            raise ValueError("add_episodes: S_traj must be [E, T+1, ns] and rewards [E, *]")
        R_term = None if R_term is None else f64(R_term)
        dVdx = None if dVdx is None else f64(dVdx)
        if dVdx is not None and dVdx.shape != S_traj.shape:
            raise ValueError("add_episodes: dVdx must have the shape of S_traj")
        total = torch.empty(E, S_traj.shape[1], dtype=torch.float64, device=DEVICE) if want_total else None
        L.lib().call("cacto_rl_solve_add", self.sys.handle, dptr(S_traj), S_traj.shape[1], dptr(rewards),
                     rewards.shape[1], dptr(R_term), dptr(dVdx), dptr(off_d), E, int(nsteps.max()), n,
                     int(getattr(self.conf, "nsteps_TD_N", 0)), int(bool(self.conf.MC)), dptr(self.storage), self.N,
                     self.next_idx, dptr(total), stream())
        self._advance(n)
        return total

    def add(self, obses_t, rewards, obses_t1, dVdxs, dones, terms):
        """replay_buffer.py:25-36."""
        self.add_rows(self.concatenate_sample(obses_t, rewards, obses_t1, dVdxs, dones, terms))

    def max_idx(self):
        return self.N if self.full else self.next_idx

    def sample_indices(self, n, rng=None):
        """n batches of indices in one draw (int32, device)."""
        r = self.np_rng if rng is None else rng
        idx = r.randint(0, self.max_idx(), size=(n, self.conf.BATCH_SIZE)) if hasattr(r, "randint") else \
            r.integers(0, self.max_idx(), size=(n, self.conf.BATCH_SIZE))
        return torch.as_tensor(idx.astype(np.int32), device=DEVICE)

    def gather(self, idx):
        B = idx.shape[0]
        ns = self.ns
        f32 = dict(dtype=torch.float32, device=DEVICE)
        s, r, sn, dv, d = (torch.empty(B, ns, **f32), torch.empty(B, 1, **f32), torch.empty(B, ns, **f32),
                           torch.empty(B, ns, **f32), torch.empty(B, 1, **f32))
        term = torch.empty(B, 1, dtype=torch.float64, device=DEVICE)
        L.lib().call("cacto_buffer_gather", self.sys.handle, dptr(self.storage), dptr(idx, torch.int32), B, dptr(s),
                     dptr(r), dptr(sn), dptr(dv), dptr(d), dptr(term), stream())
        return s, r, sn, dv, d, term

    def sample(self, idx=None):
        """replay_buffer.py:38-61: (s, R, s_next, dVdx, d, term, weights, None)."""
        if idx is None:
            idx = self.sample_indices(1)[0]
        s, r, sn, dv, d, term = self.gather(idx)
        w = torch.ones(idx.shape[0], 1, dtype=torch.float32, device=DEVICE)
        return s, r, sn, dv, d, term, w, None


def exchange_shard_stats(local, world, all_gather):
    """Gather every rank's 3-vector (sum, min, max_idx) into one contiguous [world, 3] tensor in
    rank order; `all_gather(list_out, tensor)` is torch.distributed.all_gather (RCCL or gloo)."""
    parts = [torch.empty_like(local) for _ in range(world)]
    all_gather(parts, local)
    return torch.stack(parts).contiguous()


class PrioritizedReplayBuffer(ReplayBuffer):
    """replay_buffer.py:87-218 (with the three shipped crash bugs fixed — DESIGN.md §PER)."""
    prioritized = True

    def __init__(self, conf, sys=None, py_random=None):
        """replay_buffer.py:88 `PrioritizedReplayBuffer(conf)`."""
        super().__init__(conf, sys)
        cap = 1
        while cap < self.N:
            cap *= 2
        self.cap = cap
        self.sum_tree = torch.empty(2 * cap, dtype=torch.float64, device=DEVICE)
        self.min_tree = torch.empty(2 * cap, dtype=torch.float64, device=DEVICE)
        L.lib().call("cacto_per_init", dptr(self.sum_tree), dptr(self.min_tree), cap, stream())
        self.max_priority = torch.ones(1, dtype=torch.float64, device=DEVICE)
        self.exp_counter = torch.zeros(self.N, dtype=torch.float64, device=DEVICE)
        self.alpha = float(conf.prioritized_replay_alpha)
        self.beta = float(conf.prioritized_replay_beta)
        self.eps = float(conf.prioritized_replay_eps)
        self.fresh = float(conf.fresh_factor)
        self.random = py_random or random  # replay_buffer.py:150 uses the global `random`
        # replay_buffer.py:118 (commented out there, so 'PER'); 'ReLO' selects the other priority
        # rule of update_priorities (replay_buffer.py:193-196)
        self.RB_type = getattr(conf, "RB_type", "PER")
        self._relo_ws = None
        self._relo_status = None    # device int32: the ReLO rule's failed `assert priority > 0`

    def _rows_added(self, start, n):
        # leaves = max_priority ** alpha (replay_buffer.py:133-135) with the host's Python float
        # power, as the reference: the device pow can differ from libm's by an ulp once max_priority
        # != 1, and the leaves feed the stratified sampling. One 8-byte read per add (adds happen
        # once per episode batch, outside the update loop); cacto_per_set_range_max is the
        # sync-free variant.
        leaf = float(self.max_priority.item()) ** self.alpha
        L.lib().call("cacto_per_set_range", dptr(self.sum_tree), dptr(self.min_tree), self.cap, self.N, start, n,
                     leaf, stream())

    def sample_device(self, uniforms=None):
        """_sample_proportional + IS weights + exp_counter (replay_buffer.py:139-188)."""
        if isinstance(uniforms, torch.Tensor):      # device uniforms (e.g. pre-drawn for many steps)
            u = uniforms.to(device=DEVICE, dtype=torch.float64).contiguous()
            B = u.shape[0]
        else:
            B = self.conf.BATCH_SIZE
            if uniforms is None:
                uniforms = [self.random.random() for _ in range(B)]
            u = torch.as_tensor(np.asarray(uniforms, dtype=np.float64), device=DEVICE)
        idx = torch.empty(B, dtype=torch.int32, device=DEVICE)
        w = torch.empty(B, dtype=torch.float32, device=DEVICE)
        if self.dp_world > 1 or self.dp_group is not None:
            stats = self.shard_stats()
            L.lib().call("cacto_per_sample_global", dptr(self.sum_tree), dptr(self.min_tree), self.cap,
                         self.max_idx(), self.beta, dptr(u), B, dptr(stats), self.dp_world, dptr(idx), dptr(w),
                         dptr(self.exp_counter), stream())
            return idx, w
        L.lib().call("cacto_per_sample", dptr(self.sum_tree), dptr(self.min_tree), self.cap, self.max_idx(),
                     self.beta, dptr(u), B, dptr(idx), dptr(w), dptr(self.exp_counter), stream())
        return idx, w

    # ---- data parallel: one replay shard per rank, IS weights over the union ----
    dp_world = 1
    dp_group = None

    def set_data_parallel(self, world_size, group=None):
        self.dp_world = int(world_size)
        self.dp_group = group

    def shard_stats(self):
        """All ranks' (sum, min, max_idx), [G, 3] f64 on the device, via one all-gather (RCCL)."""
        import torch.distributed as dist
        local = torch.empty(3, dtype=torch.float64, device=DEVICE)
        L.lib().call("cacto_per_shard_stats", dptr(self.sum_tree), dptr(self.min_tree), self.max_idx(), dptr(local),
                     stream())
        return exchange_shard_stats(local, self.dp_world, lambda out, t: dist.all_gather(out, t, group=self.dp_group))

    def sample(self, uniforms=None):
        idx, w = self.sample_device(uniforms)
        s, r, sn, dv, d, term = self.gather(idx)
        return s, r, sn, dv, d, term, w.reshape(-1, 1), idx

    def update_priorities_device(self, idx, y, V, Vt=None):
        B = idx.shape[0]
        if self.RB_type == "ReLO":
            if Vt is None:
                raise ValueError("update_priorities with RB_type 'ReLO' needs target_critic_value")
            if self._relo_ws is None or self._relo_ws.numel() < B:
                self._relo_ws = torch.empty(B, dtype=torch.float64, device=DEVICE)
            if self._relo_status is None:
                self._relo_status = torch.zeros(1, dtype=torch.int32, device=DEVICE)
            L.lib().call("cacto_per_update_relo", dptr(self.sum_tree), dptr(self.min_tree), self.cap,
                         dptr(idx, torch.int32), dptr(y.reshape(-1).contiguous(), torch.float32),
                         dptr(V.reshape(-1).contiguous(), torch.float32),
                         dptr(Vt.reshape(-1).contiguous(), torch.float32), dptr(self.exp_counter), self.fresh,
                         self.eps, self.alpha, dptr(self.max_priority), dptr(self._relo_ws), dptr(self._relo_status),
                         B, stream())
            return
        L.lib().call("cacto_per_update", dptr(self.sum_tree), dptr(self.min_tree), self.cap, dptr(idx, torch.int32),
                     dptr(y.reshape(-1).contiguous(), torch.float32), dptr(V.reshape(-1).contiguous(), torch.float32),
                     dptr(self.exp_counter), self.fresh, self.eps, self.alpha, dptr(self.max_priority), B, stream())

    def check_priorities(self):
        """The reference's `assert priority > 0` (replay_buffer.py:212) for the ReLO rule: the device
        flags a batch with some p <= 0 or NaN and leaves the trees unchanged; this raises
        AssertionError once per flagged update (one 4-byte read) and clears the flag."""
        if self._relo_status is not None and int(self._relo_status.item()):
            self._relo_status.zero_()
            raise AssertionError("update_priorities (ReLO): a new priority is not > 0 (every td error negative, "
                                 "or a NaN td error); the trees were left unchanged")

    def update_priorities(self, idxes, reward_to_go_batch, critic_value, target_critic_value=None):
        """replay_buffer.py:190-218 (RB_type 'PER', or 'ReLO' with target_critic_value)."""
        idx = torch.as_tensor(np.asarray(idxes, dtype=np.int32) if not isinstance(idxes, torch.Tensor) else idxes,
                              dtype=torch.int32, device=DEVICE).contiguous()
        f32 = lambda x: torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x, dtype=torch.float32,
                                        device=DEVICE).reshape(-1).contiguous()
        self.update_priorities_device(idx, f32(reward_to_go_batch), f32(critic_value),
                                      None if target_critic_value is None else f32(target_critic_value))
        if self.RB_type == "ReLO":
            self.check_priorities()

    def set_leaves(self, idx, values):
        idx = torch.as_tensor(np.asarray(idx, dtype=np.int32), device=DEVICE)
        v = torch.as_tensor(np.asarray(values, dtype=np.float64), device=DEVICE)
        L.lib().call("cacto_per_set_leaves", dptr(self.sum_tree), dptr(self.min_tree), self.cap, dptr(idx), dptr(v),
                     len(idx), stream())
