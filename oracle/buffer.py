"""Oracle: replay buffers, segment trees, PER, n-step TD targets (test infrastructure only).

Restated:
  * ReplayBuffer.add / sample                      replay_buffer.py:9-83
  * SumSegmentTree / MinSegmentTree                segment_tree.py:4-145 (OpenAI baselines)
  * PrioritizedReplayBuffer add / _sample_proportional / sample / update_priorities
                                                   replay_buffer.py:87-218, with the three shipped
    crash bugs fixed as documented in DESIGN.md (unqualified tree class names :114-115; tree
    fancy-indexing :175 read element-wise; RB_type defaulting to 'PER' :193) and every other
    semantic kept: tail-excluding p_total (:148), duplicate-once exp_counter (:174),
    last-write-wins leaf updates (:209-218).
  * RL_AC.RL_Solve n-step targets                  RL.py:145-189
The reference's numpy RNG is never seeded (replay_buffer.py:45), so sampled indices/uniforms are
explicit inputs here and on the GPU.
"""
import operator

import numpy as np


class ReplayBuffer:
    def __init__(self, replay_size, nb_state):
        self.N = replay_size
        self.ns = nb_state
        self.storage = np.zeros((replay_size, 3 * nb_state + 3))
        self.next_idx = 0
        self.full = 0

    @staticmethod
    def concatenate(obses_t, rewards, obses_t1, dVdxs, dones, terms):
        cat = lambda xs: np.concatenate(xs, axis=0)
        return np.concatenate((cat(obses_t), cat(rewards).reshape(-1, 1), cat(obses_t1), cat(dVdxs),
                               cat(dones).reshape(-1, 1), cat(terms).reshape(-1, 1)), axis=1)

    def add_rows(self, data):
        """replay_buffer.py:25-36 (ring wrap; `full` latches)."""
        n, N = len(data), self.N
        if n + self.next_idx > N:
            self.storage[self.next_idx:, :] = data[:N - self.next_idx, :]
            self.storage[:self.next_idx + n - N, :] = data[N - self.next_idx:, :]
            self.full = 1
        else:
            self.storage[self.next_idx:self.next_idx + n, :] = data
        self.next_idx = (self.next_idx + n) % N

    def max_idx(self):
        return self.N if self.full else self.next_idx

    def gather(self, idxes):
        """replay_buffer.py:47-61 with `idxes` supplied: returns the f32 tensors and f64 `terms`."""
        ns, st = self.ns, self.storage[np.asarray(idxes, dtype=np.int64)]
        f = lambda a: a.astype(np.float32)
        return (f(st[:, :ns]), f(st[:, ns:ns + 1]), f(st[:, ns + 1:2 * ns + 1]),
                f(st[:, 2 * ns + 1:3 * ns + 1]), f(st[:, 3 * ns + 1:3 * ns + 2]),
                st[:, 3 * ns + 2:3 * ns + 3].copy())


class SegmentTree:
    def __init__(self, capacity, operation, neutral):
        assert capacity > 0 and capacity & (capacity - 1) == 0
        self.cap = capacity
        self.value = [neutral for _ in range(2 * capacity)]
        self.op = operation

    def _reduce(self, start, end, node, ns, ne):
        if start == ns and end == ne:
            return self.value[node]
        mid = (ns + ne) // 2
        if end <= mid:
            return self._reduce(start, end, 2 * node, ns, mid)
        if mid + 1 <= start:
            return self._reduce(start, end, 2 * node + 1, mid + 1, ne)
        return self.op(self._reduce(start, mid, 2 * node, ns, mid),
                       self._reduce(mid + 1, end, 2 * node + 1, mid + 1, ne))

    def reduce(self, start=0, end=None):
        if end is None:
            end = self.cap
        if end < 0:
            end += self.cap
        end -= 1
        return self._reduce(start, end, 1, 0, self.cap - 1)

    def __setitem__(self, idx, val):
        idx += self.cap
        self.value[idx] = val
        idx //= 2
        while idx >= 1:
            self.value[idx] = self.op(self.value[2 * idx], self.value[2 * idx + 1])
            idx //= 2

    def __getitem__(self, idx):
        return self.value[self.cap + idx]


class SumSegmentTree(SegmentTree):
    def __init__(self, capacity):
        super().__init__(capacity, operator.add, 0.0)

    def sum(self, start=0, end=None):
        return self.reduce(start, end)

    def find_prefixsum_idx(self, prefixsum):
        idx = 1
        while idx < self.cap:
            if self.value[2 * idx] > prefixsum:
                idx = 2 * idx
            else:
                prefixsum -= self.value[2 * idx]
                idx = 2 * idx + 1
        return idx - self.cap


class MinSegmentTree(SegmentTree):
    def __init__(self, capacity):
        super().__init__(capacity, min, float('inf'))

    def min(self, start=0, end=None):
        return self.reduce(start, end)


class PrioritizedReplayBuffer(ReplayBuffer):
    def __init__(self, replay_size, nb_state, alpha, beta, eps, fresh_factor, batch_size):
        super().__init__(replay_size, nb_state)
        cap = 1
        while cap < replay_size:
            cap *= 2
        self.it_sum = SumSegmentTree(cap)
        self.it_min = MinSegmentTree(cap)
        self.max_priority = 1.0
        self.alpha, self.beta, self.eps, self.fresh = alpha, beta, eps, fresh_factor
        self.B = batch_size
        self.exp_counter = np.zeros(replay_size)

    def add_rows(self, data):
        """replay_buffer.py:124-137."""
        start = self.next_idx
        super().add_rows(data)
        leaf = self.max_priority ** self.alpha
        for i in range(len(data)):
            self.it_sum[(start + i) % self.N] = leaf
            self.it_min[(start + i) % self.N] = leaf

    def sample_proportional(self, uniforms):
        """replay_buffer.py:139-157 with the B draws of random.random() supplied."""
        p_total = self.it_sum.sum(0, self.max_idx() - 1)
        segment = p_total / self.B
        return np.array([self.it_sum.find_prefixsum_idx(u * segment + i * segment)
                         for i, u in enumerate(uniforms)], dtype=np.int64)

    def sample_weights(self, idxes):
        """replay_buffer.py:167-176: IS weights and the exp_counter side effect."""
        max_idx = self.max_idx()
        total = self.it_sum.sum()
        p_min = self.it_min.min() / total
        max_weight = (p_min * max_idx) ** (-self.beta)
        self.exp_counter[idxes] += 1
        pr = np.array([self.it_sum[int(i)] for i in idxes]) / total
        return (pr * max_idx) ** (-self.beta) / max_weight

    def shard_stats(self):
        """(sum, min, max_idx) of this shard, the 3-vector the data-parallel ranks all-gather."""
        return np.array([self.it_sum.sum(), self.it_min.min(), float(self.max_idx())])

    def sample_weights_global(self, idxes, shard_stats):
        """IS weights when G shards each draw the same number of stratified samples (a
        build extension; the reference is single-process): P(i) = p_i / (G * T_g) over N = sum N_h
        rows, w = (N P(i))^-beta / max over the union. G = 1 reduces to sample_weights."""
        st = np.asarray(shard_stats, dtype=np.float64).reshape(-1, 3)
        G = st.shape[0]
        n_all = 0.0
        ratio_min = float("inf")
        for T, m, n in st:
            n_all += n
            ratio_min = min(ratio_min, m / T)
        scale = n_all / G
        max_weight = (ratio_min * scale) ** (-self.beta)
        self.exp_counter[idxes] += 1
        pr = np.array([self.it_sum[int(i)] for i in idxes]) / self.it_sum.sum()
        return (pr * scale) ** (-self.beta) / max_weight

    def update_priorities_relo(self, idxes, y, V, Vt):
        """replay_buffer.py:193-196 + :200-218 ('ReLO' branch): Keras MeanSquaredError with reduction
        NONE gives the per-sample f32 (V - y)^2; td = MSE(y, V) - MSE(y, V_tgt) (numpy f32);
        td_norm = np.clip(td, 0, np.max(td)); p = fresh^count (f64) * td_norm (f32, promoted) + eps
        — numpy arithmetic, so p is f64 here (the 'PER' branch multiplies a TF f32 tensor)."""
        f32 = np.float32
        y, V, Vt = (np.asarray(a, dtype=f32).reshape(-1) for a in (y, V, Vt))
        td = (V - y) * (V - y) - (Vt - y) * (Vt - y)
        td_norm = np.clip(td, 0, np.max(td))
        new_p = self.fresh ** self.exp_counter[np.asarray(idxes)] * td_norm + self.eps
        for idx, p in zip(idxes, new_p):
            assert p > 0
            leaf = p ** self.alpha
            self.it_sum[int(idx)] = float(leaf)
            self.it_min[int(idx)] = float(leaf)
            self.max_priority = max(self.max_priority, float(p))
        return new_p

    def update_priorities(self, idxes, y, V):
        """replay_buffer.py:190-218 ('PER' branch): p = fresh^count * |y - V| + eps.
        The reference multiplies a float64 numpy array by float32 TF tensors, so p is a float32
        tensor (TF converts the numpy operand to the tensor dtype); leaves are float(p) ** alpha
        as Python floats (the fixed semantics)."""
        f32 = np.float32
        td = np.abs(np.asarray(y, dtype=f32) - np.asarray(V, dtype=f32))[:, 0]
        fresh = (self.fresh ** self.exp_counter[np.asarray(idxes)]).astype(f32)
        new_p = (fresh * td).astype(f32) + f32(self.eps)
        for idx, p in zip(idxes, new_p):
            assert p > 0
            leaf = float(p) ** self.alpha
            self.it_sum[int(idx)] = leaf
            self.it_min[int(idx)] = leaf
            self.max_priority = max(self.max_priority, float(p))
        return new_p


def rl_solve(states, step_cost, nsteps_td, MC=False):
    """RL.py:145-189 with env_RL = 0: rewards = -TO_step_cost, states = TO_states.
    Returns (partial_reward_to_go, total_reward_to_go, state_next_rollout, done, term)."""
    T = len(step_cost) - 1
    rwrd = -np.asarray(step_cost, dtype=np.float64)
    ns = states.shape[1]
    s_next = np.zeros((T + 1, ns))
    partial = np.empty(T + 1)
    total = np.empty(T + 1)
    term = np.zeros(T + 1)
    term[-1] = 1
    done = np.zeros(T + 1)
    for i in range(T + 1):
        if MC:
            final = T
            done[i] = 1
        else:
            final = min(i + nsteps_td, T)
            if final == T:
                done[i] = 1
            else:
                s_next[i, :] = states[final + 1, :]
        partial[i] = np.float32(sum(rwrd[i:final + 1]))
        total[i] = np.float32(sum(rwrd[i:T + 1]))
    return partial, total, s_next, done, term
