// Prioritized replay on the GPU: float64 sum/min segment trees in the exact node layout and
// combination order of segment_tree.py (so sampled indices are bit-exact), stratified proportional
// sampling, IS weights, the duplicate-once exp_counter update and last-write-wins priority updates
// (replay_buffer.py:87-218).
#include <cstdlib>

#include "internal.h"
#include "per_device.h"

namespace cacto {

constexpr int PER_THREADS = 1024;
constexpr int PER_MAX_B = 8192;


__global__ void k_per_init(double* sum_tree, double* min_tree, int64_t n2) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n2; k += (int64_t)gridDim.x * blockDim.x) {
    sum_tree[k] = 0.0;
    min_tree[k] = __builtin_inf();
  }
}

// Leaves [start, start+n) mod ring get `value`; then every ancestor is recomputed bottom-up.
// Recomputing an ancestor from final children yields the value the sequential Python updates
// leave behind (each node's last recomputation follows its subtree's last leaf write).
__global__ void k_per_fill_leaves(double* sum_tree, double* min_tree, int64_t cap, int64_t ring, int64_t start, int64_t n,
                                  double value, const double* __restrict__ max_priority, double alpha) {
  // replay_buffer.py:133-135: new leaves = max_priority ** alpha, read on the device (no host sync)
  if (max_priority) value = pow(max_priority[0], alpha);
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t leaf = cap + (start + k) % ring;
    sum_tree[leaf] = value;
    min_tree[leaf] = value;
  }
}

// One level of ancestors of the leaf range: nodes [lo, hi] at this level.
__global__ void k_per_level(double* sum_tree, double* min_tree, int64_t lo, int64_t hi) {
  for (int64_t k = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k <= hi; k += (int64_t)gridDim.x * blockDim.x) {
    sum_tree[k] = sum_tree[2 * k] + sum_tree[2 * k + 1];
    min_tree[k] = tree_min(min_tree[2 * k], min_tree[2 * k + 1]);
  }
}

// Top of the sum tree staged in LDS by the PER kernels: nodes [1, TOP_NODES).
constexpr int TOP_NODES = 1024;

__device__ __forceinline__ double tree_at(const double* tree, const double* top, int64_t ntop, int64_t node) {
  return node < ntop ? top[node] : tree[node];
}

// _reduce_helper(0, end, 1, 0, cap-1) for the sum tree (end inclusive): right-nested sum of the
// maximal left-aligned nodes, exactly as the recursion combines them. The path depends on `end`
// only, so every term is loaded independently (one memory latency, not one per level).
__device__ double prefix_reduce(const double* tree, const double* top, int64_t ntop, int64_t cap, int64_t end) {
  constexpr int MAXD = 32;  // capacity <= 2^31 (int32 indices)
  double t[MAXD];
  bool v[MAXD];
  int64_t node = 1, ns = 0, ne = cap - 1;
  bool done = false;
#pragma unroll
  for (int k = 0; k < MAXD; ++k) {
    v[k] = false;
    t[k] = 0.0;
    if (!done) {
      if (end == ne) {
        t[k] = tree_at(tree, top, ntop, node);
        v[k] = true;
        done = true;
      } else {
        const int64_t mid = (ns + ne) / 2;
        if (end <= mid) {
          node = 2 * node;
          ne = mid;
        } else {
          t[k] = tree_at(tree, top, ntop, 2 * node);
          v[k] = true;
          node = 2 * node + 1;
          ns = mid + 1;
        }
      }
    }
  }
  double r = 0.0;
  bool have = false;
#pragma unroll
  for (int k = MAXD - 1; k >= 0; --k)
    if (v[k]) {
      r = have ? t[k] + r : t[k];
      have = true;
    }
  return r;
}

// SPT samples per thread, PG of them in lock-step: the one-workgroup launch (1024 threads) takes
// SPT = 8, PG = 4; the multi-workgroup launch one sample per thread (256-thread workgroups), so
// each thread's serial work is one descent and one IS-weight pow
template <int SPT, int PG>
__global__ void __launch_bounds__(SPT == 1 ? 256 : PER_THREADS) k_per_sample(const double* __restrict__ sum_tree,
                                                           const double* __restrict__ min_tree, int64_t cap,
                                                           int64_t max_idx, double beta,
                                                           const double* __restrict__ uniforms, int B,
                                                           int32_t* __restrict__ idx_out, float* __restrict__ w_out,
                                                           double* __restrict__ exp_counter,
                                                           const double* __restrict__ shards, int n_shards) {
  __shared__ double seg_s, total_s, maxw_s, scale_s;
  // the multi-workgroup launch (SPT = 1) stages a deeper top (4,096 nodes: two rounds of global
  // levels instead of three below it) and needs no index copy
  constexpr int TOPN = SPT == 1 ? 4 * TOP_NODES : TOP_NODES;
  __shared__ int32_t idx_s[SPT == 1 ? 1 : PER_MAX_B];
  __shared__ double top_s[TOPN];
  const int64_t ntop = cap < TOPN ? cap : TOPN;
  // multi-workgroup launches (SPT = 1): workgroup b takes samples [b * blockDim.x, (b + 1) * blockDim.x)
  // (each stages the top and forms the batch scalars itself; exp_counter then goes to k_per_count)
  const int base = blockIdx.x * SPT * blockDim.x;
  // thread 0 forms the batch scalars from global memory while the others stage the top (the same
  // node values either way), so the two memory latencies overlap
  if (threadIdx.x > 0)  // threads 1.. stage the top
    for (int k = threadIdx.x - 1; k < ntop; k += blockDim.x - 1) top_s[k] = k ? sum_tree[k] : 0.0;
  if (threadIdx.x == 0) {
    const double p_total = prefix_reduce(sum_tree, top_s, 0, cap, max_idx - 2);  // sum(0, max_idx - 1)
    seg_s = p_total / B;
    total_s = sum_tree[1];
    if (shards) {
      // Data parallel: every shard draws B stratified samples from its own tree, so sample i of
      // shard g has probability p_i / (G * total_g) in the union of N = sum N_g rows. The IS
      // weight (N * P(i))^-beta is normalised by its maximum over all shards. For one shard this
      // is exactly the single-buffer formula below.
      double n_all = 0.0, ratio_min = __builtin_inf();
      for (int g = 0; g < n_shards; ++g) {
        n_all += shards[3 * g + 2];
        ratio_min = tree_min(ratio_min, shards[3 * g + 1] / shards[3 * g + 0]);
      }
      scale_s = n_all / n_shards;
      maxw_s = pow(ratio_min * scale_s, -beta);
    } else {
      const double p_min = min_tree[1] / total_s;
      scale_s = (double)max_idx;
      maxw_s = pow(p_min * scale_s, -beta);
    }
  }
  __syncthreads();
  const double seg = seg_s, total = total_s, maxw = maxw_s, scale = scale_s;
  // find_prefixsum_idx for every sample: the top levels from LDS, the rest in rounds of up to three
  // levels whose seven candidate left children are loaded together (one memory latency per round
  // instead of per level). The comparisons and subtractions are the reference's, in its order. The
  // (up to 8) descents of a thread advance in lock-step so their loads overlap too.
  constexpr int PT = SPT;
  int64_t node[PT];
#pragma unroll
  for (int g = 0; g < PT; g += PG) {
    if (base + threadIdx.x + g * blockDim.x >= (unsigned)B) {
#pragma unroll
      for (int j = g; j < g + PG; ++j) node[j] = cap;
      continue;
    }
    double p[PG];
    int64_t nd[PG];
#pragma unroll
    for (int jj = 0; jj < PG; ++jj) {
      const int i = base + threadIdx.x + (g + jj) * blockDim.x;
      p[jj] = i < B ? uniforms[i] * seg + i * seg : 0.0;
      nd[jj] = 1;
      if (i < B) {
        while (2 * nd[jj] < ntop) {
          const double left = top_s[2 * nd[jj]];
          if (left > p[jj]) {
            nd[jj] = 2 * nd[jj];
          } else {
            p[jj] -= left;
            nd[jj] = 2 * nd[jj] + 1;
          }
        }
      }
    }
    while (true) {
      bool any = false;
#pragma unroll
      for (int jj = 0; jj < PG; ++jj) any |= (base + threadIdx.x + (g + jj) * blockDim.x < (unsigned)B) && nd[jj] < cap;
      if (!any) break;
      double a[PG], b0[PG], b1[PG], c[PG][4];
#pragma unroll
      for (int jj = 0; jj < PG; ++jj) {
        const int64_t n = nd[jj];
        const bool live = base + threadIdx.x + (g + jj) * blockDim.x < (unsigned)B && n < cap;
        a[jj] = live ? tree_at(sum_tree, top_s, ntop, 2 * n) : 0.0;
        const bool two = live && 2 * n < cap, three = live && 4 * n < cap;
        b0[jj] = two ? sum_tree[4 * n] : 0.0;
        b1[jj] = two ? sum_tree[4 * n + 2] : 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) c[jj][q] = three ? sum_tree[8 * n + 2 * q] : 0.0;
      }
#pragma unroll
      for (int jj = 0; jj < PG; ++jj) {
        const int64_t n = nd[jj];
        if (base + threadIdx.x + (g + jj) * blockDim.x >= (unsigned)B || n >= cap) continue;
        int64_t m;
        if (a[jj] > p[jj]) {
          m = 2 * n;
        } else {
          p[jj] -= a[jj];
          m = 2 * n + 1;
        }
        if (2 * n < cap) {
          const double bl = (m & 1) ? b1[jj] : b0[jj];
          if (bl > p[jj]) {
            m = 2 * m;
          } else {
            p[jj] -= bl;
            m = 2 * m + 1;
          }
          if (4 * n < cap) {
            const int q = (int)(m - 4 * n);
            const double cl = q == 0 ? c[jj][0] : q == 1 ? c[jj][1] : q == 2 ? c[jj][2] : c[jj][3];
            if (cl > p[jj]) {
              m = 2 * m;
            } else {
              p[jj] -= cl;
              m = 2 * m + 1;
            }
          }
        }
        nd[jj] = m;
      }
    }
#pragma unroll
    for (int jj = 0; jj < PG; ++jj) node[g + jj] = nd[jj];
  }
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    const int i = base + threadIdx.x + j * blockDim.x;
    if (i < B) {
      const int32_t id = (int32_t)(node[j] - cap);
      if constexpr (SPT > 1) idx_s[i - base] = id;
      idx_out[i] = id;
      const double pr = sum_tree[node[j]] / total;
      w_out[i] = (float)(pow(pr * scale, -beta) / maxw);
    }
  }
  if (SPT == 1 || gridDim.x > 1) return;  // the multi-workgroup launch: k_per_count follows
  __syncthreads();
  // exp_counter[idxes] += 1: numpy fancy-index increment counts each distinct index once.
  double old[PER_MAX_B / PER_THREADS];
  int k = 0;
  for (int i = threadIdx.x; i < B; i += blockDim.x) old[k++] = exp_counter ? exp_counter[idx_s[i]] : 0.0;
  __syncthreads();
  k = 0;
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    if (exp_counter) exp_counter[idx_s[i]] = old[k] + 1.0;
    ++k;
  }
}

// The multi-workgroup sampler (B >= CACTO_PER_MW_MIN, default 512): per_sample_body (per_device.h)
// with an 8,192-node top, one sample per thread, 256 per workgroup. exp_counter follows in k_per_count.
__global__ void __launch_bounds__(256) k_per_sample_mw(PerSampleArgs a) {
  __shared__ double top_s[PER_MW_TOP];
  __shared__ double scal_s[4];
  per_sample_body<PER_MW_TOP>(blockIdx.x, a, top_s, scal_s);
}

// The pipelined PER loop's first sample (the later ones run inside k_adam_sample): the 4,096-node top
// of the fused form, with the per-subtree runs for per_update_run_body.
__global__ void __launch_bounds__(256) k_per_sample_runs(PerSampleArgs a) {
  __shared__ double top_s[PER_FUSED_TOP];
  __shared__ double scal_s[4];
  per_sample_body<PER_FUSED_TOP>(blockIdx.x, a, top_s, scal_s);
}

// The leaf writes of k_per_set over many workgroups, one leaf per thread (the two f64 pows of a
// priority are the serial work): every workgroup checks the whole index list for order itself (so
// "last occurrence" is the neighbour test for sorted lists, a scan otherwise, as in k_per_set), and
// max_priority = max(max_priority, max p) by an atomic max on the bit pattern — the priorities are
// positive (p >= eps > 0), where the IEEE order and the integer order agree; NaN is skipped as fmax
// skips it. Same leaf values, same last-write-wins, same max (bit-identical).
__global__ void __launch_bounds__(256) k_per_leaves_mw(double* sum_tree, double* min_tree, int64_t cap,
                                                      const int32_t* __restrict__ idx, const double* __restrict__ vals,
                                                      int n, const float* __restrict__ y, const float* __restrict__ V,
                                                      const double* __restrict__ exp_counter, double fresh, double eps,
                                                      double alpha, double* max_priority,
                                                      const int32_t* __restrict__ skip) {
  if (skip && *skip) return;
  bool unsorted = false;
  for (int i = threadIdx.x; i + 1 < n; i += blockDim.x) unsorted |= idx[i + 1] < idx[i];
  const bool sorted = !__syncthreads_or(unsorted);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  double my_max = -__builtin_inf();
  if (i < n) {
    const int32_t id = idx[i];
    double leaf;
    if (vals) {
      leaf = vals[i];
    } else {
      const float td = fabsf(__fsub_rn(y[i], V[i]));
      const float fd = (float)pow(fresh, exp_counter[id]);
      const float p = __fadd_rn(__fmul_rn(fd, td), (float)eps);
      my_max = fmax(my_max, (double)p);
      leaf = pow((double)p, alpha);
    }
    bool last = true;
    if (sorted) {
      last = i + 1 == n || idx[i + 1] != id;
    } else {
      for (int j = i + 1; j < n; ++j)
        if (idx[j] == id) {
          last = false;
          break;
        }
    }
    if (last) {
      sum_tree[cap + id] = leaf;
      min_tree[cap + id] = leaf;
    }
  }
  if (max_priority) {
    double m = my_max;
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off));
    if ((threadIdx.x & 63) == 0 && m > 0.0)  // false for -inf (no leaf) and NaN
      atomicMax(reinterpret_cast<unsigned long long*>(max_priority), (unsigned long long)__double_as_longlong(m));
  }
}

// exp_counter[idxes] += 1 after a multi-workgroup k_per_sample (numpy's fancy-index increment counts
// each distinct index once). With a sorted index list (the stratified sampler's output) each distinct
// index is incremented by the thread of its first occurrence alone, so no thread reads a counter
// another one writes; an unsorted list (checked by every workgroup) is counted by workgroup 0 with
// every read before any write. Same counters either way.
__global__ void __launch_bounds__(256) k_per_count(const int32_t* __restrict__ idx, int B,
                                                     double* __restrict__ exp_counter) {
  bool unsorted = false;
  for (int i = threadIdx.x; i + 1 < B; i += blockDim.x) unsorted |= idx[i + 1] < idx[i];
  const bool sorted = !__syncthreads_or(unsorted);
  if (sorted) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < B && (i == 0 || idx[i - 1] != idx[i])) exp_counter[idx[i]] += 1.0;
    return;
  }
  if (blockIdx.x != 0) return;
  double old[PER_MAX_B / 256];
  int k = 0;
  for (int i = threadIdx.x; i < B; i += blockDim.x) old[k++] = exp_counter[idx[i]];
  __syncthreads();
  k = 0;
  for (int i = threadIdx.x; i < B; i += blockDim.x) exp_counter[idx[i]] = old[k++] + 1.0;
}

// Ancestor refresh of a priority update as whole subtrees in LDS: workgroup s loads the SUB leaves
// [cap + s SUB, cap + (s + 1) SUB) of both trees, rebuilds the subtree's levels in LDS and writes
// every internal node back. The tree is consistent (each node = op(children), set by these kernels
// and k_per_level), so nodes over untouched leaves come out unchanged and the touched ones get
// op(final children) — the value the reference's leaf-by-leaf updates leave (see k_per_fill_leaves).
// One memory latency per workgroup instead of one barrier-separated global round per level.
constexpr int PER_SUB = 1024;
__global__ void __launch_bounds__(256) k_per_subtrees(double* __restrict__ sum_tree, double* __restrict__ min_tree,
                                                     int64_t cap, int sub) {
  __shared__ double ts[2 * PER_SUB], tm[2 * PER_SUB];  // local node j (1-based heap of the subtree)
  const int64_t leaf0 = cap + (int64_t)blockIdx.x * sub;
  for (int k = threadIdx.x; k < sub; k += blockDim.x) {
    ts[sub + k] = sum_tree[leaf0 + k];
    tm[sub + k] = min_tree[leaf0 + k];
  }
  __syncthreads();
  int lvl = 0;
  for (int lo = sub / 2; lo >= 1; lo /= 2) {
    ++lvl;
    for (int k = lo + threadIdx.x; k < 2 * lo; k += blockDim.x) {
      ts[k] = ts[2 * k] + ts[2 * k + 1];
      tm[k] = tree_min(tm[2 * k], tm[2 * k + 1]);
      // local node k of level lvl is global node (leaf0 >> lvl) + (k - lo)
      const int64_t g = (leaf0 >> lvl) + (k - lo);
      sum_tree[g] = ts[k];
      min_tree[g] = tm[k];
    }
    __syncthreads();
  }
}

// A whole priority update as one launch over the subtrees of `sub` leaves (large batches): workgroup s
// owns leaves [cap + s sub, cap + (s + 1) sub), so every sample whose index falls there — every write
// of those leaves, of their exp_counter entries and of the subtree's internal nodes — belongs to one
// workgroup, and no two workgroups write the same word. Per workgroup:
//   1. its samples: with a sorted index list (the stratified sampler's output) the contiguous run
//      [lower_bound(s sub), lower_bound((s + 1) sub)), two binary searches; otherwise a filter over
//      the whole list (every workgroup checks the order itself, so all take the same branch);
//   2. the leaves as k_per_set forms them (p = fresh^count |y - V| + eps in f32, p^alpha; or given
//      values), duplicates last-write-wins, into the subtree staged in LDS and into the trees;
//      count = 1 also applies the sampler's exp_counter += 1 first (numpy's fancy-index increment:
//      once per distinct index; every occurrence reads the old count, the first one then writes
//      old + 1 after a barrier), so the pipelined update needs no separate counting launch;
//   3. the subtree's levels rebuilt in LDS and written back (as k_per_subtrees);
//   4. the last workgroup to finish (a counter in the unused word sum_tree[0], reset to 0 = +0.0
//      afterwards) rebuilds the nodes above the subtree roots (as k_per_top); the roots are stored
//      at agent scope and counted after their stores completed, so no L2-wide fence is needed.
// max_priority by the atomic bit-pattern max of k_per_leaves_mw. A set `skip` flag (the ReLO
// priority rule's error status) leaves the trees, counters and max_priority unchanged. Every value
// is formed as on the k_per_leaves_mw + k_per_count + k_per_subtrees + k_per_top path, so the
// results are bit-identical to it (and to k_per_set).
constexpr int PER_FUSED_MAX_ROOTS = PER_SUB;  // the top fits the subtree's LDS arrays
__global__ void __launch_bounds__(256) k_per_update_sub(double* __restrict__ sum_tree, double* __restrict__ min_tree,
                                                       int64_t cap, int sub, const int32_t* __restrict__ idx,
                                                       const double* __restrict__ vals, int n,
                                                       const float* __restrict__ y, const float* __restrict__ V,
                                                       double* __restrict__ exp_counter, int count, double fresh,
                                                       double eps, double alpha, double* max_priority,
                                                       const int32_t* __restrict__ skip) {
  // 64 KiB: both subtrees and the index list (binary searches and neighbour tests in LDS); the
  // unused heap slots ts[0] / tm[0] hold the run bounds and the last-workgroup flag
  __shared__ double ts[2 * PER_SUB], tm[2 * PER_SUB];  // local node j (1-based heap of the subtree)
  __shared__ int32_t id_s[PER_MAX_B];
  int* run_s = reinterpret_cast<int*>(&ts[0]);
  int* last_s = reinterpret_cast<int*>(&tm[0]);
  if (skip && *skip) return;  // uniform: every workgroup returns, the counter stays 0
  const int tid = threadIdx.x;
  const int64_t id_lo = (int64_t)blockIdx.x * sub, id_hi = id_lo + sub;
  const int64_t leaf0 = cap + id_lo;
  // the index list and both subtrees' leaves: every load in flight before the first LDS write (a
  // plain staging loop waited for each load in turn: 16 + 4 dependent memory latencies at B = 4096)
  {
    constexpr int NI = PER_MAX_B / 256, NL = PER_SUB / 256;
    int iv[NI];
    double sv[NL], mv[NL];
#pragma unroll
    for (int j = 0; j < NI; ++j) iv[j] = tid + 256 * j < n ? idx[tid + 256 * j] : 0;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int k = tid + 256 * j;
      sv[j] = k < sub ? sum_tree[leaf0 + k] : 0.0;
      mv[j] = k < sub ? min_tree[leaf0 + k] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < NI; ++j)
      if (tid + 256 * j < n) id_s[tid + 256 * j] = iv[j];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int k = tid + 256 * j;
      if (k < sub) {
        ts[sub + k] = sv[j];
        tm[sub + k] = mv[j];
      }
    }
  }
  __syncthreads();
  bool unsorted = false;
  for (int i = tid; i + 1 < n; i += 256) unsorted |= id_s[i + 1] < id_s[i];
  const bool sorted = !__syncthreads_or(unsorted);
  if (sorted && tid < 2) {  // lower_bound of id_lo (thread 0) and id_hi (thread 1)
    const int64_t key = tid ? id_hi : id_lo;
    int lo = 0, hi = n;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((int64_t)id_s[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    run_s[tid] = lo;
  }
  __syncthreads();
  const int a = sorted ? run_s[0] : 0, b = sorted ? run_s[1] : n;
  auto mine = [&](int i) {
    if (sorted) return true;
    const int64_t id = id_s[i];
    return id >= id_lo && id < id_hi;
  };
  auto first_occ = [&](int i, int32_t id) {
    if (sorted) return i == 0 || id_s[i - 1] != id;
    for (int j = 0; j < i; ++j)
      if (id_s[j] == id) return false;
    return true;
  };
  auto last_occ = [&](int i, int32_t id) {
    if (sorted) return i + 1 == n || id_s[i + 1] != id;
    for (int j = i + 1; j < n; ++j)
      if (id_s[j] == id) return false;
    return true;
  };
  double my_max = -__builtin_inf();
  for (int i = a + tid; i < b; i += 256) {
    if (!mine(i)) continue;
    const int32_t id = id_s[i];
    double leaf;
    if (vals) {
      leaf = vals[i];
    } else {
      const double cnt = exp_counter[id] + (count ? 1.0 : 0.0);
      const float td = fabsf(__fsub_rn(y[i], V[i]));
      const float fd = (float)pow(fresh, cnt);
      const float p = __fadd_rn(__fmul_rn(fd, td), (float)eps);
      my_max = fmax(my_max, (double)p);
      leaf = pow((double)p, alpha);
    }
    if (last_occ(i, id)) {
      ts[sub + (id - id_lo)] = leaf;
      tm[sub + (id - id_lo)] = leaf;
      sum_tree[cap + id] = leaf;
      min_tree[cap + id] = leaf;
    }
  }
  if (max_priority) {
    double m = my_max;
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off));
    if ((tid & 63) == 0 && m > 0.0)  // false for -inf (no leaf) and NaN
      atomicMax(reinterpret_cast<unsigned long long*>(max_priority), (unsigned long long)__double_as_longlong(m));
  }
  __syncthreads();  // every occurrence has read its old count; the leaves are in LDS
  if (count && exp_counter && !vals)
    for (int i = a + tid; i < b; i += 256) {
      if (!mine(i)) continue;
      const int32_t id = id_s[i];
      if (first_occ(i, id)) exp_counter[id] += 1.0;
    }
  const int64_t nroot = cap / sub;
  int lvl = 0;
  for (int lo = sub / 2; lo >= 1; lo /= 2) {
    ++lvl;
    for (int k = lo + tid; k < 2 * lo; k += 256) {
      ts[k] = ts[2 * k] + ts[2 * k + 1];
      tm[k] = tree_min(tm[2 * k], tm[2 * k + 1]);
      const int64_t g = (leaf0 >> lvl) + (k - lo);
      if (k == 1 && nroot > 1) {
        // the subtree root, read by the last workgroup below: stored at agent scope (coherent
        // across the XCDs' L2s) instead of releasing the whole L2 with a fence — a fence's L2
        // write-back here also flushed the concurrent chains' panel writes (29 us per launch)
        __hip_atomic_store(sum_tree + g, ts[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(min_tree + g, tm[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        sum_tree[g] = ts[k];
        min_tree[g] = tm[k];
      }
    }
    __syncthreads();
  }
  if (nroot == 1) return;
  // last workgroup done: the root stores have completed (vmcnt 0) before the count (agent-scope
  // publication without a fence: DESIGN.md §3, "Memory-ordering contract", site 1)
  unsigned long long* done = reinterpret_cast<unsigned long long*>(sum_tree);
  if (tid == 0) {
    __builtin_amdgcn_s_waitcnt(0);
    *last_s = __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
              (unsigned long long)(nroot - 1);
  }
  __syncthreads();
  if (!*last_s) return;
  for (int64_t k = nroot + tid; k < 2 * nroot; k += 256) {
    ts[k] = __hip_atomic_load(sum_tree + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tm[k] = __hip_atomic_load(min_tree + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  for (int64_t lo = nroot / 2; lo >= 1; lo /= 2) {
    for (int64_t k = lo + tid; k < 2 * lo; k += 256) {
      ts[k] = ts[2 * k] + ts[2 * k + 1];
      tm[k] = tree_min(tm[2 * k], tm[2 * k + 1]);
      sum_tree[k] = ts[k];
      min_tree[k] = tm[k];
    }
    __syncthreads();
  }
  if (tid == 0) __hip_atomic_store(done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // +0.0, node 0
}

// The nodes above the subtree roots, [1, cap / sub), from the roots (one workgroup, LDS).
__global__ void __launch_bounds__(PER_THREADS) k_per_top(double* __restrict__ sum_tree, double* __restrict__ min_tree,
                                                        int64_t nroot) {
  extern __shared__ double sh[];  // 2 nroot sums, then 2 nroot mins
  double* ts = sh;
  double* tm = sh + 2 * nroot;
  for (int64_t k = nroot + threadIdx.x; k < 2 * nroot; k += blockDim.x) {
    ts[k] = sum_tree[k];
    tm[k] = min_tree[k];
  }
  __syncthreads();
  for (int64_t lo = nroot / 2; lo >= 1; lo /= 2) {
    for (int64_t k = lo + threadIdx.x; k < 2 * lo; k += blockDim.x) {
      ts[k] = ts[2 * k] + ts[2 * k + 1];
      tm[k] = tree_min(tm[2 * k], tm[2 * k + 1]);
      sum_tree[k] = ts[k];
      min_tree[k] = tm[k];
    }
    __syncthreads();
  }
}

// This shard's (sum, min, row count) for the data-parallel exchange of cacto_per_sample_global.
__global__ void k_per_shard_stats(const double* __restrict__ sum_tree, const double* __restrict__ min_tree,
                                  int64_t max_idx, double* __restrict__ stats) {
  if (threadIdx.x == 0) {
    stats[0] = sum_tree[1];
    stats[1] = min_tree[1];
    stats[2] = (double)max_idx;
  }
}

// Leaf writes with last-write-wins among duplicates, then ancestor refresh level by level.
__global__ void __launch_bounds__(PER_THREADS) k_per_set(double* sum_tree, double* min_tree, int64_t cap,
                                                        const int32_t* __restrict__ idx, const double* __restrict__ vals,
                                                        int n, const float* __restrict__ y, const float* __restrict__ V,
                                                        const double* __restrict__ exp_counter, double fresh, double eps,
                                                        double alpha, double* max_priority, int leaves_only,
                                                        const int32_t* __restrict__ skip) {
  __shared__ int32_t id_s[PER_MAX_B];
  if (skip && *skip) return;
  __shared__ double maxp_s[PER_THREADS / 64];
  __shared__ double top_sum[TOP_NODES], top_min[TOP_NODES];
  double my_max = -__builtin_inf();
  bool unsorted = false;
  for (int i = threadIdx.x; i < n; i += blockDim.x) id_s[i] = idx[i];
  __syncthreads();
  // Stratified samples come out non-decreasing in i (monotone prefix-sum search), so duplicates are
  // adjacent and "last occurrence" is a neighbour test; arbitrary index lists take the O(n^2) scan.
  for (int i = threadIdx.x; i + 1 < n; i += blockDim.x) unsorted |= id_s[i + 1] < id_s[i];
  const bool sorted = !__syncthreads_or(unsorted);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    double leaf;
    if (vals) {
      leaf = vals[i];
    } else {
      // p = fresh^count * |y - V| + eps evaluated as TF would (float32 tensors), leaf = p^alpha
      const float td = fabsf(__fsub_rn(y[i], V[i]));
      const float fd = (float)pow(fresh, exp_counter[id_s[i]]);
      const float p = __fadd_rn(__fmul_rn(fd, td), (float)eps);
      my_max = fmax(my_max, (double)p);
      leaf = pow((double)p, alpha);
    }
    bool last = true;
    if (sorted) {
      last = i + 1 == n || id_s[i + 1] != id_s[i];
    } else {
      for (int j = i + 1; j < n; ++j)
        if (id_s[j] == id_s[i]) {
          last = false;
          break;
        }
    }
    if (last) {
      sum_tree[cap + id_s[i]] = leaf;
      min_tree[cap + id_s[i]] = leaf;
    }
  }
  if (max_priority) {  // max is order-independent: wave reduction, then across the waves
    double m = my_max;
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off));
    if ((threadIdx.x & 63) == 0) maxp_s[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      double mm = maxp_s[0];
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w) mm = fmax(mm, maxp_s[w]);
      max_priority[0] = fmax(max_priority[0], mm);
    }
  }
  if (leaves_only) return;  // k_per_subtrees + k_per_top refresh the ancestors
  __syncthreads();
  // Ancestors below the LDS-staged top, one level per barrier. With sorted indices a node is
  // refreshed only by the first sample below it (the others would rewrite the same value). Each
  // thread loads the children of all its nodes before storing any parent, so the loads overlap.
  constexpr int PT = PER_MAX_B / PER_THREADS;
  int log2cap = 0;
  while (((int64_t)1 << log2cap) < cap) ++log2cap;
  const int64_t ntop = cap < TOP_NODES / 2 ? cap : TOP_NODES / 2;  // rows [ntop, 2 ntop) fit the LDS arrays
  int log2top = 0;
  while (((int64_t)1 << log2top) < ntop) ++log2top;
  for (int shift = 1; shift <= log2cap - log2top; ++shift) {
    int64_t nd[PT];
    double s0[PT], s1[PT], m0[PT], m1[PT];
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = threadIdx.x + j * blockDim.x;
      nd[j] = 0;
      if (i < n) {
        const int64_t x = (cap + id_s[i]) >> shift;
        if (!(sorted && i > 0 && ((cap + id_s[i - 1]) >> shift) == x)) nd[j] = x;
      }
      if (nd[j]) {
        s0[j] = sum_tree[2 * nd[j]];
        s1[j] = sum_tree[2 * nd[j] + 1];
        m0[j] = min_tree[2 * nd[j]];
        m1[j] = min_tree[2 * nd[j] + 1];
      }
    }
#pragma unroll
    for (int j = 0; j < PT; ++j)
      if (nd[j]) {
        sum_tree[nd[j]] = s0[j] + s1[j];
        min_tree[nd[j]] = tree_min(m0[j], m1[j]);
      }
    __syncthreads();
  }
  // The top: its bottom row [ntop, 2 ntop) is current now; rebuild nodes [1, ntop) in LDS. Nodes
  // no sample touched come out unchanged (the tree is consistent, the op is deterministic).
  double* ts = top_sum;
  double* tm = top_min;
  for (int64_t k = ntop + threadIdx.x; k < 2 * ntop; k += blockDim.x) {
    ts[k] = sum_tree[k];
    tm[k] = min_tree[k];
  }
  __syncthreads();
  for (int64_t lo = ntop / 2; lo >= 1; lo /= 2) {
    for (int64_t k = lo + threadIdx.x; k < 2 * lo; k += blockDim.x) {
      ts[k] = ts[2 * k] + ts[2 * k + 1];
      tm[k] = tree_min(tm[2 * k], tm[2 * k + 1]);
    }
    __syncthreads();
  }
  for (int64_t k = 1 + threadIdx.x; k < ntop; k += blockDim.x) {
    sum_tree[k] = ts[k];
    min_tree[k] = tm[k];
  }
}

}  // namespace cacto

using namespace cacto;

static bool pow2(int64_t c) { return c > 0 && (c & (c - 1)) == 0; }

extern "C" int cacto_per_init(double* sum_tree_d, double* min_tree_d, int64_t capacity, void* stream) {
  CACTO_REQUIRE(sum_tree_d && min_tree_d && pow2(capacity), "cacto_per_init: capacity must be a power of two");
  hipLaunchKernelGGL(k_per_init, dim3((unsigned)std::min<int64_t>((2 * capacity + 255) / 256, 4096)), dim3(256), 0,
                     as_stream(stream), sum_tree_d, min_tree_d, 2 * capacity);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

namespace {
int per_set_range(double* sum_tree_d, double* min_tree_d, int64_t capacity, int64_t ring_size, int64_t start,
                  int64_t n, double value, const double* max_priority_d, double alpha, hipStream_t st) {
  CACTO_REQUIRE(sum_tree_d && min_tree_d && pow2(capacity) && ring_size > 0 && ring_size <= capacity && n >= 0 &&
                    start >= 0 && start < ring_size,
                "cacto_per_set_range: bad arguments");
  if (n == 0) return CACTO_OK;
  n = std::min(n, ring_size);
  hipLaunchKernelGGL(k_per_fill_leaves, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0, st,
                     sum_tree_d, min_tree_d, capacity, ring_size, start, n, value, max_priority_d, alpha);
  CACTO_CHECK_HIP(hipGetLastError());
  // affected leaf interval(s); refresh the covering node interval per level (superset is harmless)
  const int64_t a = start, b = start + n - 1;
  int64_t lo = capacity + (b < ring_size ? a : 0), hi = capacity + (b < ring_size ? b : ring_size - 1);
  while (lo > 1) {
    lo >>= 1;
    hi >>= 1;
    const int64_t cnt = hi - lo + 1;
    hipLaunchKernelGGL(k_per_level, dim3((unsigned)std::min<int64_t>((cnt + 255) / 256, 4096)), dim3(256), 0, st,
                       sum_tree_d, min_tree_d, lo, hi);
    CACTO_CHECK_HIP(hipGetLastError());
  }
  return CACTO_OK;
}
}  // namespace

namespace {
// Batches of at least PER_MW_MIN samples take the multi-workgroup paths: the descents one sample per
// thread over 256-thread workgroups (+ k_per_count, or the count deferred into the priority update
// of the pipelined loop), and the priority update as one launch over the subtrees (k_per_update_sub:
// leaves, count, subtree rebuild in LDS, the top by the last workgroup). Smaller batches keep the
// one-workgroup kernels (fewer launches). Every path forms the same values (bit-identical indices, weights, trees).
// CACTO_PER_MW_MIN overrides the bound (read once; benchmarks).
int per_mw_min() {
  static const int v = [] {
    const char* e = std::getenv("CACTO_PER_MW_MIN");
    return e ? std::atoi(e) : 512;
  }();
  return v;
}

int launch_per_sample(const double* sum_tree_d, const double* min_tree_d, int64_t capacity, int64_t max_idx,
                      double beta, const double* uniforms_d, int B, int32_t* idx_d, float* is_w_d,
                      double* exp_counter_d, const double* shards_d, int n_shards, hipStream_t st) {
  if (B >= per_mw_min()) {
    constexpr int TPB = 256;  // one sample per thread
    static const bool deep = [] {
      const char* e = std::getenv("CACTO_PER_DEEP_TOP");  // 0: the round-4 sampler (A/B)
      return !(e && e[0] == '0');
    }();
    // CACTO_PER_TOP=4096: the fused loop's 4,096-node form standalone (its parity tests; read once)
    static const bool top4k = [] {
      const char* e = std::getenv("CACTO_PER_TOP");
      return e && std::atoi(e) == 4096;
    }();
    const PerSampleArgs sa{sum_tree_d, min_tree_d, capacity, max_idx, beta, uniforms_d, B, idx_d, is_w_d,
                           shards_d, n_shards, nullptr};
    if (deep && top4k)
      hipLaunchKernelGGL(k_per_sample_runs, dim3((B + TPB - 1) / TPB), dim3(TPB), 0, st, sa);
    else if (deep)
      hipLaunchKernelGGL(k_per_sample_mw, dim3((B + TPB - 1) / TPB), dim3(TPB), 0, st, sa);
    else
      hipLaunchKernelGGL((k_per_sample<1, 1>), dim3((B + TPB - 1) / TPB), dim3(TPB), 0, st, sum_tree_d, min_tree_d, capacity,
                         max_idx, beta, uniforms_d, B, idx_d, is_w_d, nullptr, shards_d, n_shards);
    CACTO_CHECK_HIP(hipGetLastError());
    if (exp_counter_d) {
      hipLaunchKernelGGL(k_per_count, dim3((B + 255) / 256), dim3(256), 0, st, idx_d, B, exp_counter_d);
      CACTO_CHECK_HIP(hipGetLastError());
    }
    return CACTO_OK;
  }
  hipLaunchKernelGGL((k_per_sample<PER_MAX_B / PER_THREADS, 4>), dim3(1), dim3(PER_THREADS), 0, st, sum_tree_d, min_tree_d, capacity, max_idx, beta,
                     uniforms_d, B, idx_d, is_w_d, exp_counter_d, shards_d, n_shards);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

}  // namespace

#ifdef CACTO_STAMPS
extern "C" int cacto_debug_per_stamps(unsigned long long* out_h) {  // [64][8], this TU's samplers
  CACTO_CHECK_HIP(hipDeviceSynchronize());
  CACTO_CHECK_HIP(hipMemcpyFromSymbol(out_h, HIP_SYMBOL(cacto::g_per_stamps), sizeof(unsigned long long) * 64 * 8));
  return CACTO_OK;
}
#endif

// The fused PER loop's first sample (learn_kernels.hip): k_per_sample_runs, recording the per-subtree
// runs (runs_d: 2 cap / PER_RUN_SUB ints, PER_RUN_EMPTY / 0 on entry).
int cacto_per_sample_runs_launch(const double* sum_tree_d, const double* min_tree_d, int64_t capacity, int64_t max_idx,
                                 double beta, const double* uniforms_d, int B, int32_t* idx_d, float* is_w_d,
                                 int32_t* runs_d, hipStream_t st, const double* shards_d, int n_shards) {
  using namespace cacto;
  const PerSampleArgs sa{sum_tree_d, min_tree_d, capacity, max_idx, beta, uniforms_d, B, idx_d, is_w_d,
                         shards_d, n_shards, runs_d};
  hipLaunchKernelGGL(k_per_sample_runs, dim3((B + 255) / 256), dim3(256), 0, st, sa);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

namespace {

// count = 1: exp_counter += 1 (the sampler's count, deferred) applied inside the priority update;
// skip_d: an int status that, when set, leaves everything unchanged (the ReLO rule's error flag)
int launch_per_set(double* sum_tree_d, double* min_tree_d, int64_t capacity, const int32_t* idx_d,
                   const double* values_d, int n, const float* y_d, const float* V_d, double* exp_counter_d,
                   double fresh, double eps, double alpha, double* max_priority_d, hipStream_t st, int count = 0,
                   const int32_t* skip_d = nullptr) {
  const int64_t sub = std::min<int64_t>(PER_SUB, capacity), nroot = capacity / sub;
  const bool mw = n >= per_mw_min();
  // CACTO_PER_FUSED=0 selects the round-3 multi-workgroup chain (leaves, count, subtrees, top;
  // read once; A/B and the bit-identity test)
  static const bool fused_env = [] {
    const char* e = std::getenv("CACTO_PER_FUSED");
    return !(e && e[0] == '0');
  }();
  if (mw && fused_env && nroot <= PER_FUSED_MAX_ROOTS) {
    hipLaunchKernelGGL(k_per_update_sub, dim3((unsigned)nroot), dim3(256), 0, st, sum_tree_d, min_tree_d, capacity,
                       (int)sub, idx_d, values_d, n, y_d, V_d, exp_counter_d, count, fresh, eps, alpha, max_priority_d,
                       skip_d);
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
  if (count) {
    hipLaunchKernelGGL(k_per_count, dim3((n + 255) / 256), dim3(256), 0, st, idx_d, n, exp_counter_d);
    CACTO_CHECK_HIP(hipGetLastError());
  }
  // k_per_top stages both trees' nroot subtree roots and their parents (4 nroot doubles) in
  // dynamic LDS, which is 64 KiB per workgroup without an opt-in attribute
  constexpr int64_t MW_MAX_ROOTS = 2048;
  static_assert(4 * MW_MAX_ROOTS * sizeof(double) <= 65536, "k_per_top: dynamic LDS above 64 KiB");
  if (!mw || nroot > MW_MAX_ROOTS) {
    hipLaunchKernelGGL(k_per_set, dim3(1), dim3(PER_THREADS), 0, st, sum_tree_d, min_tree_d, capacity, idx_d, values_d,
                       n, y_d, V_d, exp_counter_d, fresh, eps, alpha, max_priority_d, 0, skip_d);
    CACTO_CHECK_HIP(hipGetLastError());
    return CACTO_OK;
  }
  hipLaunchKernelGGL(k_per_leaves_mw, dim3((n + 255) / 256), dim3(256), 0, st, sum_tree_d, min_tree_d, capacity, idx_d,
                     values_d, n, y_d, V_d, exp_counter_d, fresh, eps, alpha, max_priority_d, skip_d);
  CACTO_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_per_subtrees, dim3((unsigned)nroot), dim3(256), 0, st, sum_tree_d, min_tree_d, capacity, (int)sub);
  CACTO_CHECK_HIP(hipGetLastError());
  if (nroot > 1) {
    hipLaunchKernelGGL(k_per_top, dim3(1), dim3(PER_THREADS), (size_t)4 * nroot * sizeof(double), st, sum_tree_d,
                       min_tree_d, nroot);
    CACTO_CHECK_HIP(hipGetLastError());
  }
  return CACTO_OK;
}
}  // namespace

int cacto_per_mw_min() { return per_mw_min(); }
int cacto_per_count_launch(const int32_t* idx_d, int B, double* exp_counter_d, hipStream_t st) {
  hipLaunchKernelGGL(k_per_count, dim3((B + 255) / 256), dim3(256), 0, st, idx_d, B, exp_counter_d);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

// The pipelined PER loop's priority update with the sampler's deferred exp_counter += 1 applied
// first (the count's only reader is this update): one launch from PER_MW_MIN samples on.
int cacto_per_update_count(double* sum_tree_d, double* min_tree_d, int64_t capacity, const int32_t* idx_d,
                           const float* y_d, const float* V_d, double* exp_counter_d, double fresh_factor, double eps,
                           double alpha, double* max_priority_d, int B, hipStream_t st) {
  return launch_per_set(sum_tree_d, min_tree_d, capacity, idx_d, nullptr, B, y_d, V_d, exp_counter_d, fresh_factor, eps,
                        alpha, max_priority_d, st, 1);
}

extern "C" int cacto_per_set_range(double* sum_tree_d, double* min_tree_d, int64_t capacity, int64_t ring_size,
                                   int64_t start, int64_t n, double value, void* stream) {
  return per_set_range(sum_tree_d, min_tree_d, capacity, ring_size, start, n, value, nullptr, 0.0, as_stream(stream));
}

extern "C" int cacto_per_set_range_max(double* sum_tree_d, double* min_tree_d, int64_t capacity, int64_t ring_size,
                                       int64_t start, int64_t n, const double* max_priority_d, double alpha,
                                       void* stream) {
  CACTO_REQUIRE(max_priority_d, "cacto_per_set_range_max: null max_priority_d");
  return per_set_range(sum_tree_d, min_tree_d, capacity, ring_size, start, n, 0.0, max_priority_d, alpha,
                       as_stream(stream));
}

extern "C" int cacto_per_sample(const double* sum_tree_d, const double* min_tree_d, int64_t capacity, int64_t max_idx,
                                double beta, const double* uniforms_d, int B, int32_t* idx_d, float* is_w_d,
                                double* exp_counter_d, void* stream) {
  CACTO_REQUIRE(sum_tree_d && min_tree_d && uniforms_d && idx_d && is_w_d && pow2(capacity),
                "cacto_per_sample: bad arguments");
  CACTO_REQUIRE(B > 0 && B <= PER_MAX_B, "cacto_per_sample: 0 < B <= 8192");
  // max_idx <= 1 makes the reference's sum(0, max_idx - 1) recurse past the leaves (segment_tree.py:36-49)
  CACTO_REQUIRE(max_idx >= 2 && max_idx <= capacity, "cacto_per_sample: need 2 <= max_idx <= capacity");
  return launch_per_sample(sum_tree_d, min_tree_d, capacity, max_idx, beta, uniforms_d, B, idx_d, is_w_d, exp_counter_d,
                           nullptr, 0, as_stream(stream));
}

extern "C" int cacto_per_shard_stats(const double* sum_tree_d, const double* min_tree_d, int64_t max_idx,
                                     double* stats_d, void* stream) {
  CACTO_REQUIRE(sum_tree_d && min_tree_d && stats_d && max_idx >= 0, "cacto_per_shard_stats: bad arguments");
  hipLaunchKernelGGL(k_per_shard_stats, dim3(1), dim3(64), 0, as_stream(stream), sum_tree_d, min_tree_d, max_idx,
                     stats_d);
  CACTO_CHECK_HIP(hipGetLastError());
  return CACTO_OK;
}

extern "C" int cacto_per_sample_global(const double* sum_tree_d, const double* min_tree_d, int64_t capacity,
                                       int64_t max_idx, double beta, const double* uniforms_d, int B,
                                       const double* shard_stats_d, int n_shards, int32_t* idx_d, float* is_w_d,
                                       double* exp_counter_d, void* stream) {
  CACTO_REQUIRE(sum_tree_d && min_tree_d && uniforms_d && idx_d && is_w_d && shard_stats_d && n_shards > 0 &&
                    pow2(capacity),
                "cacto_per_sample_global: bad arguments");
  CACTO_REQUIRE(B > 0 && B <= PER_MAX_B, "cacto_per_sample_global: 0 < B <= 8192");
  CACTO_REQUIRE(max_idx >= 2 && max_idx <= capacity, "cacto_per_sample_global: need 2 <= max_idx <= capacity");
  return launch_per_sample(sum_tree_d, min_tree_d, capacity, max_idx, beta, uniforms_d, B, idx_d, is_w_d, exp_counter_d,
                           shard_stats_d, n_shards, as_stream(stream));
}

extern "C" int cacto_per_update(double* sum_tree_d, double* min_tree_d, int64_t capacity, const int32_t* idx_d,
                                const float* y_d, const float* V_d, const double* exp_counter_d, double fresh_factor,
                                double eps, double alpha, double* max_priority_d, int B, void* stream) {
  CACTO_REQUIRE(sum_tree_d && min_tree_d && idx_d && y_d && V_d && exp_counter_d && max_priority_d && pow2(capacity),
                "cacto_per_update: bad arguments");
  CACTO_REQUIRE(B > 0 && B <= PER_MAX_B, "cacto_per_update: 0 < B <= 8192");
  return launch_per_set(sum_tree_d, min_tree_d, capacity, idx_d, nullptr, B, y_d, V_d,
                        const_cast<double*>(exp_counter_d), fresh_factor, eps, alpha, max_priority_d, as_stream(stream));
}

// update_priorities 'ReLO' (replay_buffer.py:193-196, :200-218; dead in the shipped reference,
// RB_type is never set): td_i = MSE(y, V)_i - MSE(y, V_tgt)_i with Keras MeanSquaredError
// (reduction NONE, so per sample: f32 (V - y)^2 over the size-1 last axis), clipped as numpy clips
// it, np.minimum(np.maximum(td, 0), max(td)); then p = fresh^count (f64) * td_norm (f32 -> f64, numpy
// promotion) + eps in f64 — unlike the 'PER' branch, whose TF tensor keeps p in f32. One workgroup
// (B <= PER_MAX_B): the per-sample leaves p^alpha go to leaves[], max_priority takes the batch max.
// The reference asserts p > 0 for every sample (replay_buffer.py:212). It fails when every td is
// negative (np.clip's upper bound max(td) < 0 then gives p = fresh^c max(td) + eps, possibly <= 0) or
// when any td is NaN (np.max propagates it, so every p is NaN): then *status = 1 and nothing is
// written — no leaf, no max_priority — and the leaf pass that follows skips on the flag, so the
// trees are unchanged. A set status (sticky until the host clears it) makes later calls no-ops too.
__global__ void __launch_bounds__(PER_THREADS) k_per_relo(const int32_t* __restrict__ idx, const float* __restrict__ y,
                                                         const float* __restrict__ V, const float* __restrict__ Vt,
                                                         const double* __restrict__ exp_counter, double fresh,
                                                         double eps, double alpha, int B, double* __restrict__ leaves,
                                                         double* __restrict__ max_priority, int32_t* status) {
  __shared__ float red_f[PER_THREADS / 64];
  __shared__ double red_d[PER_THREADS / 64];
  if (*status) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  auto td_of = [&](int i) {
    const float d1 = __fsub_rn(V[i], y[i]), d2 = __fsub_rn(Vt[i], y[i]);
    return __fsub_rn(__fmul_rn(d1, d1), __fmul_rn(d2, d2));
  };
  float mx = -__builtin_inff();
  bool nan_td = false;
  for (int i = tid; i < B; i += blockDim.x) {
    const float td = td_of(i);
    nan_td |= td != td;
    mx = fmaxf(mx, td);
  }
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  if (lane == 0) red_f[wv] = mx;
  __syncthreads();
  mx = red_f[0];
  for (int k = 1; k < (int)(blockDim.x / 64); ++k) mx = fmaxf(mx, red_f[k]);
  double pm = -__builtin_inf();
  bool bad = nan_td;
  double leaf[PER_MAX_B / PER_THREADS];
  int k = 0;
  for (int i = tid; i < B; i += blockDim.x, ++k) {
    const float tn = fminf(fmaxf(td_of(i), 0.f), mx);
    const double p = pow(fresh, exp_counter[idx[i]]) * (double)tn + eps;
    bad |= !(p > 0.0);
    leaf[k] = pow(p, alpha);
    pm = fmax(pm, p);
  }
  if (__syncthreads_or(bad)) {
    if (tid == 0) *status = 1;
    return;
  }
  k = 0;
  for (int i = tid; i < B; i += blockDim.x, ++k) leaves[i] = leaf[k];
  for (int off = 32; off > 0; off >>= 1) pm = fmax(pm, __shfl_xor(pm, off));
  if (lane == 0) red_d[wv] = pm;
  __syncthreads();
  if (tid == 0) {
    double m = max_priority[0];
    for (int q = 0; q < (int)(blockDim.x / 64); ++q) m = fmax(m, red_d[q]);
    max_priority[0] = m;
  }
}

extern "C" int cacto_per_update_relo(double* sum_tree_d, double* min_tree_d, int64_t capacity, const int32_t* idx_d,
                                     const float* y_d, const float* V_d, const float* Vt_d,
                                     const double* exp_counter_d, double fresh_factor, double eps, double alpha,
                                     double* max_priority_d, double* leaves_ws_d, int32_t* status_d, int B,
                                     void* stream) {
  CACTO_REQUIRE(sum_tree_d && min_tree_d && idx_d && y_d && V_d && Vt_d && exp_counter_d && max_priority_d &&
                    leaves_ws_d && status_d && pow2(capacity),
                "cacto_per_update_relo: bad arguments");
  CACTO_REQUIRE(B > 0 && B <= PER_MAX_B, "cacto_per_update_relo: 0 < B <= 8192");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_per_relo, dim3(1), dim3(PER_THREADS), 0, st, idx_d, y_d, V_d, Vt_d, exp_counter_d, fresh_factor,
                     eps, alpha, B, leaves_ws_d, max_priority_d, status_d);
  CACTO_CHECK_HIP(hipGetLastError());
  return launch_per_set(sum_tree_d, min_tree_d, capacity, idx_d, leaves_ws_d, B, nullptr, nullptr, nullptr, 0.0, 0.0,
                        0.0, nullptr, st, 0, status_d);
}

extern "C" int cacto_per_set_leaves(double* sum_tree_d, double* min_tree_d, int64_t capacity, const int32_t* idx_d,
                                    const double* values_d, int n, void* stream) {
  CACTO_REQUIRE(sum_tree_d && min_tree_d && idx_d && values_d && pow2(capacity), "cacto_per_set_leaves: bad arguments");
  CACTO_REQUIRE(n > 0 && n <= PER_MAX_B, "cacto_per_set_leaves: 0 < n <= 8192");
  return launch_per_set(sum_tree_d, min_tree_d, capacity, idx_d, values_d, n, nullptr, nullptr, nullptr, 0.0, 0.0, 0.0,
                        nullptr, as_stream(stream));
}
