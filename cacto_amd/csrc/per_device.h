// Device bodies of the prioritized-replay kernels shared by two translation units: the stratified
// sampler (replay_kernels.hip's k_per_sample_mw / k_per_sample_runs, and learn_kernels.hip's
// k_adam_sample, which runs it beside the critic's Adam step) and the per-subtree priority update of
// the pipelined PER loop (learn_kernels.hip's k_wgrad_big_per, beside the critic's weight-gradient
// GEMM). Node layout and arithmetic of segment_tree.py / replay_buffer.py:139-218.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace cacto {

__device__ __forceinline__ double tree_min(double a, double b) { return b < a ? b : a; }  // Python min(a, b)

constexpr int PER_MW_TOP = 8192;     // k_per_sample_mw: staged top nodes (64 KiB of LDS)
constexpr int PER_FUSED_TOP = 4096;  // the sampler beside the Adam step (32 KiB)
constexpr int PER_RUN_SUB = 256;     // leaves per workgroup of per_update_run_body
constexpr int PER_RUN_EMPTY = 0x7f7f7f7f;  // runs[s] before any sample landed in subtree s (memset 0x7f)

// Select a[j] (j in [0, N)) from a register array without dynamic indexing (no scratch).
// A tournament of selects on j's bits (a chain of j == q selects gets folded back into an indexed
// load, which moves the array to scratch).
template <int N>
__device__ __forceinline__ double reg_pick(const double (&a)[N], int j) {
  static_assert((N & (N - 1)) == 0, "power of two");
  double w[N];
#pragma unroll
  for (int q = 0; q < N; ++q) w[q] = a[q];
#pragma unroll
  for (int h = N / 2, b = 0; h >= 1; h /= 2, ++b)
#pragma unroll
    for (int q = 0; q < h; ++q) w[q] = ((j >> b) & 1) ? w[2 * q + 1] : w[2 * q];
  return w[0];
}

// The last R levels of find_prefixsum_idx below node n (whose descendants R levels down are the
// leaves): the left child of every internal node and all 2^R leaves are loaded together, so the R
// comparisons and the sampled leaf's own value (P(i) of the IS weight) cost one memory latency.
// Same comparisons and subtractions as the reference's loop (segment_tree.py:103-114), in order.
// One internal level D (1-based) of per_tail: its left children are lv[2^(D-1) - 1 + q].
template <int D, int NLV>
__device__ __forceinline__ void tail_step(const double (&lv)[NLV], int& j, double& p) {
  double row[1 << (D - 1)];
#pragma unroll
  for (int q = 0; q < (1 << (D - 1)); ++q) row[q] = lv[(1 << (D - 1)) - 1 + q];
  const double left = reg_pick(row, j);
  if (left > p) {
    j = 2 * j;
  } else {
    p -= left;
    j = 2 * j + 1;
  }
}

template <int R>
__device__ __forceinline__ void per_tail(const double* __restrict__ tree, int64_t n, double& p, int64_t& node,
                                         double& val) {
  static_assert(R >= 1 && R <= 5, "per_tail covers up to five levels");
  constexpr int NL = 1 << R;
  double lf[NL];
  double lv[R > 1 ? (1 << (R - 1)) - 1 : 1];
#pragma unroll
  for (int d = 1; d < R; ++d)
#pragma unroll
    for (int j = 0; j < (1 << (d - 1)); ++j) lv[(1 << (d - 1)) - 1 + j] = tree[(n << d) + 2 * j];
#pragma unroll
  for (int k = 0; k < NL; ++k) lf[k] = tree[(n << R) + k];
  int j = 0;  // position within the current level below n
  if constexpr (R > 1) tail_step<1>(lv, j, p);
  if constexpr (R > 2) tail_step<2>(lv, j, p);
  if constexpr (R > 3) tail_step<3>(lv, j, p);
  if constexpr (R > 4) tail_step<4>(lv, j, p);
  const double left = reg_pick(lf, 2 * j);
  if (left > p) {
    j = 2 * j;
  } else {
    p -= left;
    j = 2 * j + 1;
  }
  node = (n << R) + j;
  val = reg_pick(lf, j);
}

struct PerSampleArgs {
  const double* sum_tree;
  const double* min_tree;
  int64_t cap, max_idx;
  double beta;
  const double* uniforms;  // [B]
  int B;
  int32_t* idx_out;
  float* w_out;
  const double* shards;  // data-parallel shard statistics [n_shards][3] (nullptr: one buffer)
  int n_shards;
  // optional (the pipelined loop's fused priority update): runs[s] = min sample index and
  // runs[cap / PER_RUN_SUB + s] = sample count of subtree s, by relaxed atomics (the indices are
  // sorted, so each subtree's samples are one contiguous run)
  int32_t* runs;
};

// One sample per thread, 256 per workgroup (workgroup blk takes samples [256 blk, 256 blk + 256)).
// Each workgroup stages the top TOPN nodes of the sum tree in LDS with every thread's loads in flight
// at once while wave 0 gathers the batch scalars' terms (lane k the k-th term of prefix_reduce's
// sum(0, max_idx - 1)) in the same latency; the descent walks the staged levels in LDS, then rounds
// of three levels until at most five remain, then per_tail (one more memory latency for the
// remaining levels and the leaf value). For the 2^16-row buffer: two dependent global latencies per
// sample at TOPN = 8192 (four levels below the top) and at 4096 (five).
#ifdef CACTO_STAMPS
// diagnostic builds: s_memtime of thread 0 of each sampler workgroup at its phase boundaries (start,
// staged top + scalars, LDS descent done, tail done, end), [blk][8]; read by cacto_debug_per_stamps
__device__ unsigned long long g_per_stamps[64 * 8];
#define PER_STAMP(blk, k)                                                                        \
  do {                                                                                           \
    if (threadIdx.x == 0 && (blk) < 64) g_per_stamps[(blk) * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define PER_STAMP(blk, k) \
  do {                    \
  } while (0)
#endif

template <int TOPN>
__device__ __forceinline__ void per_sample_body(int blk, const PerSampleArgs& a, double* top_s, double* scal_s) {
  PER_STAMP(blk, 0);
  const int64_t cap = a.cap, max_idx = a.max_idx;
  const double* __restrict__ sum_tree = a.sum_tree;
  const int B = a.B;
  const int64_t ntop = cap < TOPN ? cap : TOPN;
  const int tid = threadIdx.x;
  const int i = blk * 256 + tid;
  const double u = i < B ? a.uniforms[i] : 0.0;  // in flight with the loads below
  // the staging loads first (ntop / 2 double2 pairs over 256 threads), then, while they are in
  // flight: wave 0 walks prefix_reduce's path (lane k loads its k-th term) and wave 1 loads the roots
  // and forms the IS-weight normaliser (a pow) beside wave 0's sum
  constexpr int PAIRS = TOPN / 2 / 256;
  double2 st[PAIRS];
  {
    const double2* src = reinterpret_cast<const double2*>(sum_tree);
#pragma unroll
    for (int r = 0; r < PAIRS; ++r) {
      const int64_t q = tid + r * 256;
      st[r] = 2 * q < ntop ? src[q] : make_double2(0.0, 0.0);
    }
  }
  // lane k's term in closed form (cap = 2^L; [0, cap - 1] halves at every level, so the path to
  // `end` is end's bits from the top): the walk stops at depth d* = L - (trailing ones of end, at
  // most L) with the node itself as the last term; above it, a step right at depth k (bit L - 1 - k
  // of end set) adds that node's left child
  double term = 0.0;
  bool has_term = false;
  int dstar = -1;  // deepest term's depth (no term when end < 0)
  const int64_t end = max_idx - 2;
  if (end >= 0) {
    const int L = 63 - __builtin_clzll((unsigned long long)cap);
    const int ones = __builtin_ctzll(~(unsigned long long)end);
    dstar = L - (ones < L ? ones : L);
  }
  if (tid < 64) {
    const int k = tid;
    if (end >= 0) {
      const int L = 63 - __builtin_clzll((unsigned long long)cap);
      int64_t at = -1;
      if (k == dstar) at = ((int64_t)1 << k) | (end >> (L - k));
      else if (k < dstar && ((end >> (L - 1 - k)) & 1)) at = (((int64_t)1 << k) | (end >> (L - k))) * 2;
      has_term = at >= 0;
      PER_STAMP(blk, 5);
      if (has_term) term = sum_tree[at];
    }
  } else if (tid == 64) {
    const double root_sum = sum_tree[1];
    scal_s[1] = root_sum;
    if (a.shards) {  // data parallel: IS weights over the union of the shards (see k_per_sample)
      double n_all = 0.0, ratio_min = __builtin_inf();
      for (int g = 0; g < a.n_shards; ++g) {
        n_all += a.shards[3 * g + 2];
        ratio_min = tree_min(ratio_min, a.shards[3 * g + 1] / a.shards[3 * g + 0]);
      }
      scal_s[3] = n_all / a.n_shards;
      scal_s[2] = pow(ratio_min * (n_all / a.n_shards), -a.beta);
    } else {
      const double p_min = a.min_tree[1] / root_sum;
      scal_s[3] = (double)max_idx;
      scal_s[2] = pow(p_min * (double)max_idx, -a.beta);
    }
  }
#pragma unroll
  for (int r = 0; r < PAIRS; ++r) {
    const int64_t q = tid + r * 256;
    if (2 * q < ntop) reinterpret_cast<double2*>(top_s)[q] = st[r];
  }
  PER_STAMP(blk, 6);
  if (tid < 64) {
    // the right-nested sum, deepest term first, as prefix_reduce combines them
    const unsigned long long mask = __ballot(has_term);
    double r = 0.0;
    bool have = false;
    for (int k = dstar; k >= 0; --k)
      if ((mask >> k) & 1ull) {  // k is uniform: read the lane's term into scalar registers
        const long long tb = __double_as_longlong(term);
        const int lo = __builtin_amdgcn_readlane((int)(tb & 0xffffffffll), k);
        const int hi = __builtin_amdgcn_readlane((int)(tb >> 32), k);
        const double tk = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
        r = have ? tk + r : tk;
        have = true;
      }
    if (tid == 0) scal_s[0] = r / B;  // segment
    PER_STAMP(blk, 7);
  }
  __syncthreads();
  PER_STAMP(blk, 1);
  if (i >= B) return;
  const double seg = scal_s[0];
  double p = u * seg + i * seg;
  int64_t nd = 1;
  while (4 * nd < ntop) {  // two staged levels per LDS latency: the left child and both left grandchildren
    const double a0 = top_s[2 * nd], b0 = top_s[4 * nd], b1 = top_s[4 * nd + 2];
    int64_t m;
    if (a0 > p) {
      m = 2 * nd;
    } else {
      p -= a0;
      m = 2 * nd + 1;
    }
    const double bl = (m & 1) ? b1 : b0;
    if (bl > p) {
      nd = 2 * m;
    } else {
      p -= bl;
      nd = 2 * m + 1;
    }
  }
  if (2 * nd < ntop) {
    const double left = top_s[2 * nd];
    if (left > p) {
      nd = 2 * nd;
    } else {
      p -= left;
      nd = 2 * nd + 1;
    }
  }
  PER_STAMP(blk, 2);
  // levels below the staged top, three at a time, until at most five remain
  int rem = 0;
  for (int64_t s = nd; s < cap; s *= 2) ++rem;  // levels from nd down to the leaves
  while (rem > 5) {
    const double a0 = sum_tree[2 * nd], b0 = sum_tree[4 * nd], b1 = sum_tree[4 * nd + 2];
    double c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = sum_tree[8 * nd + 2 * q];
    int64_t m;
    if (a0 > p) {
      m = 2 * nd;
    } else {
      p -= a0;
      m = 2 * nd + 1;
    }
    const double bl = (m & 1) ? b1 : b0;
    if (bl > p) {
      m = 2 * m;
    } else {
      p -= bl;
      m = 2 * m + 1;
    }
    const double cl = reg_pick(c, (int)(m - 4 * nd));
    if (cl > p) {
      m = 2 * m;
    } else {
      p -= cl;
      m = 2 * m + 1;
    }
    nd = m;
    rem -= 3;
  }
  int64_t leaf;
  double val;
  switch (rem) {
    case 5: per_tail<5>(sum_tree, nd, p, leaf, val); break;
    case 4: per_tail<4>(sum_tree, nd, p, leaf, val); break;
    case 3: per_tail<3>(sum_tree, nd, p, leaf, val); break;
    case 2: per_tail<2>(sum_tree, nd, p, leaf, val); break;
    case 1: per_tail<1>(sum_tree, nd, p, leaf, val); break;
    default: leaf = nd; val = sum_tree[nd]; break;  // capacity 1: the root is the leaf
  }
  PER_STAMP(blk, 3);
  const int32_t id = (int32_t)(leaf - cap);
  a.idx_out[i] = id;
  a.w_out[i] = (float)(pow(val / scal_s[1] * scal_s[3], -a.beta) / scal_s[2]);
  PER_STAMP(blk, 4);
  if (a.runs) {
    const int64_t nroot = cap / PER_RUN_SUB, s = id / PER_RUN_SUB;
    __hip_atomic_fetch_min(a.runs + s, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(a.runs + nroot + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

struct PerRunArgs {
  double* sum_tree;
  double* min_tree;
  int64_t cap;
  const int32_t* idx;  // the sampler's (sorted) indices of this update
  const float* y;
  const float* V;
  double* exp_counter;
  int64_t rows;  // exp_counter's length (the replay size)
  double fresh, eps, alpha;
  double* max_priority;
  int32_t* runs;  // the sampler's per-subtree runs, reset here for the next sample
  // data parallel (cacto_update_n_per_dp): the ranks' (sum, min, rows) table [world][3], or nullptr.
  // The workgroup that rebuilds the top writes this shard's values (k_per_shard_stats') at
  // stats_off and zeros in the other ranks' words, so a sum all-reduce of the table is the
  // all-gather (x + 0.0 == x for the non-negative statistics)
  double* stats;
  int stats_off = 0, stats_words = 3;
};

struct PerRunLds {
  double ts[2 * PER_RUN_SUB], tm[2 * PER_RUN_SUB];  // local node j (1-based heap of the subtree)
  double cnt[PER_RUN_SUB];                          // exp_counter of the subtree's rows before this update
  int run[2];
  int last;
};

// update_priorities 'PER' for the samples in subtree blk (leaves [cap + 256 blk, cap + 256 blk + 256))
// of one stratified sample, with the sampler's deferred exp_counter += 1 — k_per_update_sub's
// arithmetic, for sorted indices whose run the sampler recorded, so nothing is searched:
//   1. one memory latency: the subtree's leaves of both trees, its rows' exp_counter values and the
//      run (runs[] reset for the next sample);
//   2. one more: the run's indices (and neighbours, for the duplicate tests), y and V; every
//      occurrence of a row reads the row's count from LDS (numpy's fancy-index increment reads the
//      old count once per distinct index), the first occurrence writes old + 1, the last one the leaf;
//   3. the subtree rebuilt in LDS and written back, its root at agent scope; the last of the nroot
//      workgroups to finish (counter in the unused word sum_tree[0]) rebuilds the nodes above the
//      roots (nroot <= PER_RUN_SUB).
// Values, last-write-wins and max_priority as k_per_update_sub (bit-identical trees and counters).
__device__ __forceinline__ void per_update_run_body(int blk, int nroot, const PerRunArgs& a, PerRunLds& L) {
  const int tid = threadIdx.x;
  constexpr int SUB = PER_RUN_SUB;
  const int64_t cap = a.cap;
  const int64_t id_lo = (int64_t)blk * SUB;
  const int64_t leaf0 = cap + id_lo;
  {
    const double sv = a.sum_tree[leaf0 + tid], mv = a.min_tree[leaf0 + tid];
    const double cv = id_lo + tid < a.rows ? a.exp_counter[id_lo + tid] : 0.0;
    if (tid == 0) {
      L.run[0] = a.runs[blk];
      L.run[1] = a.runs[nroot + blk];
      a.runs[blk] = PER_RUN_EMPTY;
      a.runs[nroot + blk] = 0;
    }
    L.ts[SUB + tid] = sv;
    L.tm[SUB + tid] = mv;
    L.cnt[tid] = cv;
  }
  __syncthreads();
  const int r0 = L.run[0], rn = L.run[1];
  if (rn > 0) {
    double my_max = -__builtin_inf();
    for (int i = r0 + tid; i < r0 + rn; i += SUB) {
      const int32_t id = a.idx[i];
      const bool first = i == r0 || a.idx[i - 1] != id;
      const bool last = i + 1 == r0 + rn || a.idx[i + 1] != id;
      const float td = fabsf(__fsub_rn(a.y[i], a.V[i]));
      const double old = L.cnt[id - id_lo];
      const float fd = (float)pow(a.fresh, old + 1.0);
      const float p = __fadd_rn(__fmul_rn(fd, td), (float)a.eps);
      my_max = fmax(my_max, (double)p);
      const double leaf = pow((double)p, a.alpha);
      if (last) {
        L.ts[SUB + (id - id_lo)] = leaf;
        L.tm[SUB + (id - id_lo)] = leaf;
        a.sum_tree[cap + id] = leaf;
        a.min_tree[cap + id] = leaf;
      }
      if (first) a.exp_counter[id] = old + 1.0;
    }
    if (a.max_priority) {
      double m = my_max;
      for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off));
      if ((tid & 63) == 0 && m > 0.0)  // false for -inf (no leaf) and NaN
        atomicMax(reinterpret_cast<unsigned long long*>(a.max_priority), (unsigned long long)__double_as_longlong(m));
    }
    __syncthreads();  // the leaves are in LDS
    int lvl = 0;
    for (int lo = SUB / 2; lo >= 1; lo /= 2) {
      ++lvl;
      if (tid < lo) {
        const int k = lo + tid;
        L.ts[k] = L.ts[2 * k] + L.ts[2 * k + 1];
        L.tm[k] = tree_min(L.tm[2 * k], L.tm[2 * k + 1]);
        const int64_t g = (leaf0 >> lvl) + (k - lo);
        if (k == 1 && nroot > 1) {  // the root, read by the last workgroup: at agent scope
          __hip_atomic_store(a.sum_tree + g, L.ts[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.min_tree + g, L.tm[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          a.sum_tree[g] = L.ts[k];
          a.min_tree[g] = L.tm[k];
        }
      }
      __syncthreads();
    }
  }
  if (nroot == 1) return;
  // last workgroup done: the root stores have completed (vmcnt 0) before the count (agent-scope
  // publication without a fence: DESIGN.md §3, "Memory-ordering contract", site 1)
  unsigned long long* done = reinterpret_cast<unsigned long long*>(a.sum_tree);
  if (tid == 0) {
    __builtin_amdgcn_s_waitcnt(0);
    L.last = __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (unsigned long long)(nroot - 1);
  }
  __syncthreads();
  if (!L.last) return;
  if (tid < nroot) {
    L.ts[nroot + tid] = __hip_atomic_load(a.sum_tree + nroot + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    L.tm[nroot + tid] = __hip_atomic_load(a.min_tree + nroot + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  for (int lo = nroot / 2; lo >= 1; lo /= 2) {
    if (tid < lo) {
      const int k = lo + tid;
      L.ts[k] = L.ts[2 * k] + L.ts[2 * k + 1];
      L.tm[k] = tree_min(L.tm[2 * k], L.tm[2 * k + 1]);
      a.sum_tree[k] = L.ts[k];
      a.min_tree[k] = L.tm[k];
    }
    __syncthreads();
  }
  if (tid == 0) {
    __hip_atomic_store(done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // +0.0, node 0
    if (a.stats) {
      for (int k = 0; k < a.stats_words; ++k) a.stats[k] = 0.0;
      a.stats[a.stats_off + 0] = L.ts[1];
      a.stats[a.stats_off + 1] = L.tm[1];
      a.stats[a.stats_off + 2] = (double)a.rows;
    }
  }
}

}  // namespace cacto
