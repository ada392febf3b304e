// Device-resident chunk-level prioritized replay (sum tree) for gfx950.
//
// Replaces Prioritized_Experience_Replay + SumTree (vdn/replay_buffer/buffer.py:10-90,
// vdn/replay_buffer/sumtree.py:8-66; qmix/replay_buffer/per.py:10-81,
// qmix/replay_buffer/sumtree.py:8-72). Same heap layout (2*cap-1 f64 nodes,
// leaves at [cap-1, 2cap-2], children 2i+1/2i+2, "s <= left -> go left"),
// same priority (td+eps)^alpha, same stratified sampling and IS weights, VDN's
// whole-tree step-weight decay after every sample. The tree never leaves HBM.
//
// Batched insert (K chunks from K envs at once — the reference inserts one
// chunk per call): free slots first in order; the remaining inserts replace the
// K' smallest existing leaves (ties -> lower slot), assigned in ascending slot
// order. Equal to the reference's sequential min-eviction whenever no new chunk
// would itself be evicted within the batch (oracle/sumtree.py add_batch).
//
// Every op is ONE single-workgroup launch (1024 threads): K-smallest selection
// by an 8-pass radix select on the f64 bit patterns with LDS histograms, slot
// compaction by block prefix sums, then a level-by-level rebuild of the internal
// nodes. Row indirection: slot_row[slot] is the chunk-store row holding that
// slot's data; an insert swaps the staging row in and hands the freed row back,
// so chunk data is never copied.
#pragma clang fp contract(off)
#include <vector>

#include "common.h"
#include "minimarl.h"
#include "per_small.h"
#include "rollout_fold.h"

namespace mm {

// two consecutive doubles of the sum tree's leaf row: leaves = tree + (cap - 1) is only 8-byte aligned for a
// power-of-two capacity, so the pair is copied (well-defined at 8-byte alignment; still one 16-byte load)
__device__ __forceinline__ double2 ld_double2(const double* p) {
  double2 v;
  __builtin_memcpy(&v, p, sizeof(v));
  return v;
}

}  // namespace mm

struct mm_per {
  mm::PerDev* st;
  int64_t cap;
  int32_t flavor;
  double alpha, beta, eps, step_weight, alpha_inc, beta_inc;
  int32_t use_step_weight;
  int64_t n_data;
  double* tree;       // [2cap-1]
  int64_t* slot_row;  // [cap]
  void* alloc;
  void* mb;           // multi-block insert scratch (MbScratch), power-of-two cap >= MB_MIN_CAP
  int32_t* last;      // [cap] per_update scratch: last sample index per leaf (-1 between calls)
};

namespace mm {
static constexpr int PT = 1024;

__device__ void rebuild_tree(double* tree, int64_t cap) {
  // internal nodes [0, cap-2]; depth(i) = floor(log2(i+1)); deepest internal level first
  if (cap <= 1) return;
  int maxd = 63 - __clzll((unsigned long long)(cap - 1));  // depth of node cap-2
  for (int dpt = maxd; dpt >= 0; --dpt) {
    const int64_t lo = (1ll << dpt) - 1, hi = min((1ll << (dpt + 1)) - 2, cap - 2);
    for (int64_t i = lo + threadIdx.x; i <= hi; i += PT) tree[i] = tree[2 * i + 1] + tree[2 * i + 2];
    __syncthreads();
  }
}

__device__ __forceinline__ uint64_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  // exclusive scan of one value per thread over PT threads (Hillis-Steele in LDS)
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int off = 1; off < PT; off <<= 1) {
    uint32_t t = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : 0;
    __syncthreads();
    sh[threadIdx.x] += t;
    __syncthreads();
  }
  uint32_t incl = sh[threadIdx.x];
  *total = sh[PT - 1];
  __syncthreads();
  return incl - v;
}

// Exclusive scan / total of one value per thread over the PT threads: wave prefix by shuffles,
// the 16 wave totals through LDS (two barriers instead of Hillis-Steele's 2 log2(PT)).
__device__ __forceinline__ uint32_t block_excl_scan_w(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < PT / 64; ++w) {
    const uint32_t x = wsum[w];
    before += w < wave ? x : 0u;
    tot += x;
  }
  *total = tot;
  __syncthreads();
  return before + incl - v;
}
__device__ __forceinline__ uint32_t block_sum_w(uint32_t v, uint32_t* wsum) {
  uint32_t tot;
  (void)block_excl_scan_w(v, wsum, &tot);
  return tot;
}

__global__ __launch_bounds__(PT) void per_add_kernel(double* tree, int64_t* slot_row, int64_t cap, PerDev* st,
                                                     const float* td, int64_t K, double eps,
                                                     int64_t* rows_inout, int64_t* slots_out, int64_t* scratch) {
  const int64_t n_data = st->n_data;
  const double alpha = st->alpha;
  __shared__ uint32_t hist[256];
  __shared__ uint32_t scan_sh[PT];
  __shared__ uint64_t s_prefix;
  __shared__ int64_t s_need;
  __shared__ uint32_t s_tot;
  double* leaves = tree + (cap - 1);
  const int64_t free_n = min(K, cap - n_data);
  const int64_t rest = K - free_n;
  int64_t* victims = scratch;  // [rest]
  if (rest > 0) {
    // candidates: leaves [0, n_data) (slots filled in this batch are never victims)
    const int64_t M = n_data;
    if (threadIdx.x == 0) {
      s_prefix = 0;
      s_need = rest;
    }
    __syncthreads();
    // radix select (MSB first, 8 bits per pass) of the rest-th smallest key
    for (int pass = 7; pass >= 0; --pass) {
      for (int i = threadIdx.x; i < 256; i += PT) hist[i] = 0;
      __syncthreads();
      const int shift = pass * 8;
      const uint64_t hi_mask = (pass == 7) ? 0ull : (~0ull << (shift + 8));
      for (int64_t i = threadIdx.x; i < M; i += PT) {
        const uint64_t key = (uint64_t)__double_as_longlong(leaves[i]);
        if ((key & hi_mask) == (s_prefix & hi_mask)) atomicAdd(&hist[(key >> shift) & 255], 1u);
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        int64_t need = s_need;
        int b = 0;
        for (; b < 256; ++b) {
          if ((int64_t)hist[b] >= need) break;
          need -= hist[b];
        }
        s_prefix |= ((uint64_t)b << shift);
        s_need = need;  // how many with key == threshold are taken (after all passes)
      }
      __syncthreads();
    }
    const uint64_t T = s_prefix;
    const int64_t take_eq = s_need;
    // compaction in ascending slot order: key < T, plus the first take_eq slots with key == T
    int64_t base_lt = 0, base_eq = 0;
    for (int64_t c0 = 0; c0 < M; c0 += PT) {
      const int64_t i = c0 + threadIdx.x;
      uint64_t key = i < M ? (uint64_t)__double_as_longlong(leaves[i]) : ~0ull;
      const uint32_t lt = (i < M && key < T) ? 1u : 0u;
      const uint32_t eq = (i < M && key == T) ? 1u : 0u;
      uint32_t tot_lt, tot_eq;
      const uint64_t pre_lt = block_excl_scan(lt, scan_sh, &tot_lt);
      const uint64_t pre_eq = block_excl_scan(eq, scan_sh, &tot_eq);
      // the final victim list is sorted by slot: position = (#lt before) + (#eq taken before)
      const int64_t eq_rank = base_eq + (int64_t)pre_eq;
      const int64_t lt_rank = base_lt + (int64_t)pre_lt;
      if (lt || (eq && eq_rank < take_eq)) {
        const int64_t pos = lt_rank + min(eq_rank, take_eq);
        victims[pos] = i;
      }
      base_lt += tot_lt;
      base_eq += tot_eq;
    }
    (void)s_tot;
    __syncthreads();
  }
  // write priorities, slot assignment, row swap
  for (int64_t j = threadIdx.x; j < K; j += PT) {
    const int64_t slot = j < free_n ? n_data + j : victims[j - free_n];
    const double p = pow((double)td[j] + eps, alpha);
    leaves[slot] = p;
    if (slots_out) slots_out[j] = slot;
    if (rows_inout) {
      const int64_t old = slot_row[slot];
      slot_row[slot] = rows_inout[j];
      rows_inout[j] = old;
    }
  }
  __syncthreads();
  rebuild_tree(tree, cap);
  if (threadIdx.x == 0) st->n_data = min(cap, n_data + K);
}

// Fast insert for a power-of-two capacity cap = PT * VPT (VPT <= 64): thread t keeps the 16-bit
// tops (sign, exponent, 4 mantissa bits) of its VPT contiguous leaves [t*VPT, (t+1)*VPT) in
// registers. Selection of the rest-th smallest key without contended histograms: a 16-step binary
// search on count(top <= mid) (every thread counts its registers, wave-shuffle block sums), then
// the keys sharing the threshold's top (usually a few hundred) are staged in LDS and an 8-bit
// radix select over their low 48 bits finds the exact key. Slot-ordered compaction is one block
// scan of per-thread counts, and the tree rebuild is a register subtree per thread plus a
// 1024-leaf LDS top tree (same pairwise f64 sums as rebuild_tree, hence identical trees).
constexpr int FAST_MAX_VICTIMS = 8192;
constexpr int FAST_MAX_CAND = 4096;   // keys sharing the threshold's 16-bit top staged in LDS

template <int VPT>
__global__ __launch_bounds__(PT) void per_add_fast_kernel(double* tree, int64_t* slot_row, int64_t cap, PerDev* st,
                                                          const float* td, int64_t K, double eps,
                                                          int64_t* rows_inout, int64_t* slots_out) {
  __shared__ uint32_t binsum[256];
  __shared__ uint32_t wsum[PT / 64];
  __shared__ int32_t victims[FAST_MAX_VICTIMS];
  __shared__ uint64_t cand[FAST_MAX_CAND];
  __shared__ double top[PT];
  __shared__ uint64_t s_prefix;
  __shared__ int64_t s_need;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int64_t n_data = st->n_data;
  const double alpha = st->alpha;
  double* leaves = tree + (cap - 1);
  const int64_t free_n = min(K, cap - n_data);
  const int64_t rest = K - free_n;
  const int64_t s0 = (int64_t)t * VPT;
  if (rest > 0) {
    // candidates: slots [0, n_data) (this batch's free slots are never victims). Registers hold
    // only the top 16 bits of each key (sign, exponent, 4 mantissa bits; two per VGPR); the full
    // key is re-read from the leaf only when those bits tie the selected prefix.
    uint32_t kp[VPT / 2];
#pragma unroll
    for (int i = 0; i < VPT; i += 2) {
      const double2 v = ld_double2(leaves + s0 + i);
      const uint32_t a = (s0 + i < n_data) ? (uint32_t)((uint64_t)__double_as_longlong(v.x) >> 48) : 0xffffu;
      const uint32_t b = (s0 + i + 1 < n_data) ? (uint32_t)((uint64_t)__double_as_longlong(v.y) >> 48) : 0xffffu;
      kp[i / 2] = a | (b << 16);
      if ((i & 15) == 14) asm volatile("" ::: "memory");  // bound the loads in flight (VGPRs)
    }
    auto top16 = [&](int i) -> uint32_t { return (kp[i >> 1] >> ((i & 1) * 16)) & 0xffffu; };
    const double* lv = leaves + s0;
    auto full = [&](int i) -> uint64_t { return (uint64_t)__double_as_longlong(lv[i]); };
    auto valid = [&](int i) -> bool { return s0 + i < n_data; };
    // (1) the 16-bit top b of the rest-th smallest key: binary search on count(top16 <= mid), every
    //     thread counting its VPT register keys (contention-free; 16 block sums)
    uint32_t lo = 0, hi = 0xffffu;   // invariant: cnt_le(hi) >= rest
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      uint32_t c = 0;
#pragma unroll
      for (int i = 0; i < VPT; ++i) c += (valid(i) && top16(i) <= mid) ? 1u : 0u;
      if ((int64_t)block_sum_w(c, wsum) >= rest) hi = mid;
      else lo = mid + 1;
    }
    const uint32_t b16 = lo;
    uint32_t clt = 0, ceq = 0;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      clt += (valid(i) && top16(i) < b16) ? 1u : 0u;
      ceq += (valid(i) && top16(i) == b16) ? 1u : 0u;
    }
    const int64_t n_lt16 = block_sum_w(clt, wsum);
    uint32_t m;
    const uint32_t cpos = block_excl_scan_w(ceq, wsum, &m);
    int64_t need = rest - n_lt16;     // 1 <= need <= m among the keys whose top is b16
    uint64_t prefix = (uint64_t)b16 << 48;
    if (m <= (uint32_t)FAST_MAX_CAND) {
      // (2) candidates' full keys into LDS, then an 8-bit radix select over their low 48 bits
      uint32_t pos = cpos;
#pragma unroll
      for (int i = 0; i < VPT; ++i)
        if (valid(i) && top16(i) == b16) cand[pos++] = full(i);
      __syncthreads();
      for (int shift = 40; shift >= 0; shift -= 8) {
        for (int i = t; i < 256; i += PT) binsum[i] = 0;
        __syncthreads();
        const uint64_t hmask = ~0ull << (shift + 8);
        for (uint32_t i = t; i < m; i += PT) {
          const uint64_t k = cand[i];
          if ((k & hmask) == prefix) atomicAdd(&binsum[(k >> shift) & 255], 1u);
        }
        __syncthreads();
        if (wave == 0) {
          uint32_t b4[4], loc = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            b4[q] = binsum[lane * 4 + q];
            loc += b4[q];
          }
          uint32_t incl = loc;
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
          }
          const uint32_t excl = incl - loc;
          if ((int64_t)excl < need && (int64_t)incl >= need) {
            int64_t n2 = need - excl;
            int found = -1;
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (found < 0) {
                if ((int64_t)b4[q] >= n2) found = lane * 4 + q;
                else n2 -= b4[q];
              }
            s_prefix = prefix | ((uint64_t)found << shift);
            s_need = n2;
          }
        }
        __syncthreads();
        prefix = s_prefix;
        need = s_need;
        __syncthreads();
      }
    } else {
      // many equal tops (e.g. near-identical priorities): the same radix passes on the full keys
      // re-read from the leaves
      for (int shift = 40; shift >= 0; shift -= 8) {
        for (int i = t; i < 256; i += PT) binsum[i] = 0;
        asm volatile("" : "+v"(lv));
        __syncthreads();
        const uint64_t hmask = ~0ull << (shift + 8);
#pragma unroll
        for (int i = 0; i < VPT; ++i)
          if (valid(i) && top16(i) == b16) {
            const uint64_t k = full(i);
            if ((k & hmask) == prefix) atomicAdd(&binsum[(k >> shift) & 255], 1u);
          }
        __syncthreads();
        if (t == 0) {
          int64_t n2 = need;
          int bb = 0;
          for (; bb < 256; ++bb) {
            if ((int64_t)binsum[bb] >= n2) break;
            n2 -= binsum[bb];
          }
          s_prefix = prefix | ((uint64_t)bb << shift);
          s_need = n2;
        }
        __syncthreads();
        prefix = s_prefix;
        need = s_need;
        __syncthreads();
      }
    }
    if (t == 0) {
      s_prefix = prefix;
      s_need = need;
    }
    __syncthreads();
    const uint64_t T = s_prefix;
    const uint32_t T16 = (uint32_t)(T >> 48);
    asm volatile("" : "+v"(lv));
    const int64_t take_eq = s_need;
    // 0: key < T, 1: key == T, 2: key > T
    auto cmp = [&](int i) -> int {
      const uint32_t k = top16(i);
      if (k != T16) return k < T16 ? 0 : 2;
      if (s0 + i >= n_data) return 2;
      const uint64_t f = full(i);
      return f < T ? 0 : (f == T ? 1 : 2);
    };
    uint64_t mlt = 0, meq = 0;  // classification bitmasks of the thread's VPT keys
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = cmp(i);
      mlt |= (c == 0 ? 1ull : 0ull) << i;
      meq |= (c == 1 ? 1ull : 0ull) << i;
    }
    const uint32_t nlt = (uint32_t)__popcll(mlt), neq = (uint32_t)__popcll(meq);
    uint32_t tot;
    const uint32_t lt0 = block_excl_scan_w(nlt, wsum, &tot);
    const uint32_t eq0 = block_excl_scan_w(neq, wsum, &tot);
    int64_t lt_rank = lt0, eq_rank = eq0;
    for (uint64_t m = mlt | meq; m; m &= m - 1) {
      const int i = __ffsll((unsigned long long)m) - 1;
      const bool lt = (mlt >> i) & 1ull;
      if (lt) {
        victims[lt_rank + min(eq_rank, take_eq)] = (int32_t)(s0 + i);
        ++lt_rank;
      } else {
        if (eq_rank < take_eq) victims[lt_rank + eq_rank] = (int32_t)(s0 + i);
        ++eq_rank;
      }
    }
    __syncthreads();
  }
  // priorities, slot assignment, row swap
  for (int64_t j = t; j < K; j += PT) {
    const int64_t slot = j < free_n ? n_data + j : (int64_t)victims[j - free_n];
    leaves[slot] = pow((double)td[j] + eps, alpha);
    if (slots_out) slots_out[j] = slot;
    if (rows_inout) {
      const int64_t old = slot_row[slot];
      slot_row[slot] = rows_inout[j];
      rows_inout[j] = old;
    }
  }
  __syncthreads();
  // rebuild: register subtree of the thread's VPT leaves, then the PT-leaf top tree in LDS
  double v[VPT / 2];
  int64_t lvl_nodes = cap >> 1;  // nodes on the current level (first: the leaves' parents)
  {
    const int64_t base = lvl_nodes - 1 + (int64_t)t * (VPT / 2);
#pragma unroll
    for (int i = 0; i < VPT / 2; ++i) {
      const double2 x = ld_double2(leaves + s0 + 2 * i);
      v[i] = x.x + x.y;
      tree[base + i] = v[i];
      if ((i & 7) == 7) asm volatile("" ::: "memory");  // bound the loads in flight (VGPRs)
    }
  }
#pragma unroll
  for (int w = VPT / 2; w > 1; w >>= 1) {
    lvl_nodes >>= 1;
    const int64_t base = lvl_nodes - 1 + (int64_t)t * (w / 2);
#pragma unroll
    for (int i = 0; i < w / 2; ++i) {
      v[i] = v[2 * i] + v[2 * i + 1];
      tree[base + i] = v[i];
    }
  }
  top[t] = v[0];
  __syncthreads();
  for (int n = PT / 2; n >= 1; n >>= 1) {
    double x = 0.0;
    if (t < n) x = top[2 * t] + top[2 * t + 1];
    __syncthreads();
    if (t < n) {
      top[t] = x;
      tree[n - 1 + t] = x;
    }
    __syncthreads();
  }
  if (t == 0) st->n_data = min(cap, n_data + K);
}

// Uniform chunk replay (qmix/qmix.py:12-50 ReplayBuffer.sample_chunk draws start indices uniformly;
// here whole stored chunks): B slots uniform over the filled slots [0, n_data), device counter RNG
// (fresh stream per call via st->n_samples), unit IS weights; nodes_out = the slots' leaf nodes.
__global__ __launch_bounds__(1024) void per_uniform_kernel(int64_t cap, int B, uint64_t seed, uint64_t counter,
                                                          PerDev* st, int64_t* nodes_out, int64_t* slots_out,
                                                          float* is_w) {
  // ONE workgroup: every lane reads the draw counter before the single bump below (a multi-block grid
  // would race the bump against other blocks' reads; __syncthreads orders only this block)
  const uint64_t ctr = counter + st->n_samples;
  const int64_t n = st->n_data;
  __syncthreads();
  if (threadIdx.x == 0) st->n_samples += 1;
  for (int k = threadIdx.x; k < B; k += blockDim.x) {
    const double u = (double)(rng_draw(seed, ctr, (uint64_t)k, 91) >> 11) * (1.0 / 9007199254740992.0);
    const int64_t slot = min(n - 1, (int64_t)(u * (double)n));
    if (slots_out) slots_out[k] = slot;
    if (nodes_out) nodes_out[k] = slot + cap - 1;
    if (is_w) is_w[k] = 1.0f;
  }
}

__global__ __launch_bounds__(PT) void per_sample_kernel(double* tree, int64_t cap, int B, const double* fracs,
                                                        uint64_t seed, uint64_t counter, PerDev* st, double decay,
                                                        int64_t* nodes_out, int64_t* slots_out, float* is_w) {
  per_sample_body(tree, cap, B, fracs, seed, counter, st, decay, nodes_out, slots_out, is_w);
}

__global__ __launch_bounds__(1024) void per_update_small_kernel(double* tree, int64_t cap, const int64_t* nodes,
                                                                const float* td, int B, PerDev* st, float eps) {
  per_update_small_body(tree, cap, nodes, td, B, st, eps);
}

// Duplicate nodes: the LAST sample index wins (sequential tree[idx] = p semantics). One workgroup;
// the per-leaf winner is found with atomicMax into the leaf scratch `last` (all -1 between calls,
// restored before the rebuild), O(B) instead of comparing every pair.
__global__ __launch_bounds__(PT) void per_update_kernel(double* tree, int64_t cap, const int64_t* nodes, const float* td,
                                                        int B, const PerDev* st, float eps, int32_t* last) {
  const float alpha = (float)st->alpha;
  bool bad = false;
  for (int k = threadIdx.x; k < B; k += PT) {
    const int64_t nd = nodes[k];
    if (nd >= cap - 1 && nd < 2 * cap - 1)
      atomicMax(&last[nd - (cap - 1)], k);
    else
      bad = true;
  }
  // out-of-range nodes are skipped (the reference's tree[idx] = p would raise or write an internal node)
  // and flagged in the sticky error word, read by mm_per_error_word
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(&const_cast<PerDev*>(st)->err, 1);
  __syncthreads();
  for (int k = threadIdx.x; k < B; k += PT) {
    const int64_t nd = nodes[k];
    // the reference computes (td + eps) ** alpha on a float32 tensor (vdn/_train.py:230-233)
    if (nd >= cap - 1 && nd < 2 * cap - 1 && last[nd - (cap - 1)] == k) tree[nd] = (double)powf(td[k] + eps, alpha);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < B; k += PT) {
    const int64_t nd = nodes[k];
    if (nd >= cap - 1 && nd < 2 * cap - 1) last[nd - (cap - 1)] = -1;
  }
  __syncthreads();
  if ((cap & (cap - 1)) == 0 && B <= PT) {
    // power-of-two capacity: every leaf is at depth log2(cap), so only the changed leaves' paths are
    // recomputed, 4 levels per barrier: each thread re-sums the height-4 subtree above its node from
    // the (complete) level below, bottom-up (the same pairwise f64 sums as rebuild_tree, so identical
    // trees; nodes off the changed paths are recomputed from unchanged children, i.e. unchanged)
    int64_t nd = -1;
    if ((int)threadIdx.x < B) {
      nd = nodes[threadIdx.x];
      if (nd < cap - 1 || nd >= 2 * cap - 1) nd = -1;
    }
    int d = 63 - __clzll((unsigned long long)cap);   // depth of the leaves
    while (d > 0) {
      const int h = d < 4 ? d : 4, da = d - h;
      if (nd >= 0) {
        const int64_t a = ((nd + 1) >> h) - 1;        // ancestor at depth da
        double v[16];
        const int64_t base = ((a + 1) << h) - 1;      // first node of a's subtree at depth d
        for (int i = 0; i < (1 << h); ++i) v[i] = tree[base + i];
        for (int l = h - 1; l >= 0; --l) {           // depth da + l, 2^l nodes
          const int64_t lb = ((a + 1) << l) - 1;
          for (int i = 0; i < (1 << l); ++i) {
            v[i] = v[2 * i] + v[2 * i + 1];
            tree[lb + i] = v[i];
          }
        }
        nd = a;
      }
      d = da;
      __syncthreads();
    }
  } else {
    rebuild_tree(tree, cap);
  }
}


// ---------------------------------------------------------------- multi-block batched insert
// For large power-of-two capacities the single-workgroup insert is bound by one CU's memory
// bandwidth over the whole tree. This path spreads every pass over G = cap/1024 workgroups in THREE
// stream-ordered launches (graph-capturable, same results as per_add_fast_kernel). A pass's decision is
// re-derived by EVERY workgroup of the next launch from the finished global counts (the launch boundary
// orders it after the previous pass's atomics), so only the last pass needs an arrival ticket:
//   A sel1    [the chunk's last rollout TD / store and the new chunks' priorities, folded in]
//             first-level histogram of the keys: 7 binades around the previous insert's threshold x 512
//             mantissa steps (mb_bin1), two edge bins for the keys outside the window (the priorities
//             (td + eps)^alpha span a few binades and drift slowly: a fixed 12-bit sign + exponent histogram
//             resolves ~2 bits of them)
//   B sel2    each block picks the threshold's bin b1; the keys in b1 listed with their slots, histogram of
//             their next 12 bits (31..42), per-block counts of the keys below b1
//   C apply   each block picks b2 (an interior b1: the candidates share a 33-bit prefix; an edge b1: all
//             listed keys are candidates), radix-selects the exact key T among the candidates (8-bit digits
//             over the bits below their common prefix; ties — equal priorities are common: envs that stayed
//             greedy since an episode start repeat each other's chunks — cost no passes) and its own victim
//             offsets, writes its victims / free slots (the fold's priorities, row swaps) and rebuilds its
//             1024-leaf subtree from LDS; the last block (ticket) builds the top levels and updates n_data
constexpr int MB_T = 256, MB_VPT = 4, MB_SLOTS = MB_T * MB_VPT;   // 1024 slots per block
constexpr int64_t MB_MIN_CAP = 16384;
constexpr int MB_CAND_LDS = 12288;   // candidate keys compacted into the apply block's LDS
constexpr int MB_MAX_BLOCKS = 1024;
struct MbScratch {
  uint32_t hist1[4096];               // first level (mb_bin1), built by sel1, read by sel2
  uint32_t hist2[4096];               // bits 44..33 of the keys in bin b1 (sel2), read by apply
  uint32_t blk[2 * MB_MAX_BLOCKS];   // per block #keys below bin b1 (sel2)
  uint32_t cand_n;
  uint32_t ticket;
  int32_t ewin;                       // the first level's lowest biased exponent (apply's last block: T's - 3)
  int32_t pad_;
  uint64_t sel[4];                    // b1, the remaining rank inside it (sel2 block 0, for the record)
  uint64_t cand[1];                   // [2 cap] the listed (key, slot) pairs: keys at cand, slots at cand + cap;
                                      // then [cap] f64: the new chunks' priorities from the fold (mm_per_insert_fold)
};
static size_t mb_bytes(int64_t cap) { return sizeof(MbScratch) + (size_t)cap * 24; }
__host__ __device__ inline double* mb_prio(MbScratch* mb, int64_t cap) {
  return reinterpret_cast<double*>(mb->cand + 2 * cap);
}

// phase stamps of the multi-block insert (s_memrealtime, 100 MHz) per launch k and workgroup, tools/mb_per_trace.py;
// trace builds only (-DMM_PER_TRACE=1), never the product
#if MM_PER_TRACE
__device__ uint64_t g_per_trace[4][64][16];
#define PER_STAMP(k, i)                                   \
  if (threadIdx.x == 0 && blockIdx.x < 64) g_per_trace[k][blockIdx.x][i] = __builtin_amdgcn_s_memrealtime();
#define PER_NOTE(i, v) \
  if (threadIdx.x == 0 && blockIdx.x == 0) g_per_trace[0][0][i] = (uint64_t)(v);
#else
#define PER_STAMP(k, i)
#define PER_NOTE(i, v)
#endif

__device__ __forceinline__ uint64_t leaf_key(const double* leaves, int64_t s) {
  return (uint64_t)__double_as_longlong(leaves[s]);
}
// the insert of a chunk folded from a timed-out chunk-persistent launch (error bit 1 of the rollout's word, sticky
// until the host reads it): every pass returns at once, block-uniformly, so nothing of it enters the tree
__device__ __forceinline__ bool mb_skip(const uint32_t* err) {
  return err && (*reinterpret_cast<const volatile uint32_t*>(err) & 2u);
}
// first-level bin of a key (monotone in the key) in the window of 7 binades from biased exponent e0: 0 below it (and
// +0), 4095 above it, else 1 + (binade - e0) * 512 + the top 9 mantissa bits — an interior bin is the class of keys
// sharing their top 21 bits (sign 0, exponent, 9 mantissa bits). The window follows the threshold from insert to
// insert (MbScratch::ewin); one that misses it only costs speed (an edge bin lists all its keys).
constexpr int MB_WIN = 7, MB_EWIN0 = 1023 - 3;
__device__ __forceinline__ uint32_t mb_bin1(uint64_t k, int e0) {
  const int e = (int)(k >> 52);
  if (e < e0) return 0u;
  if (e >= e0 + MB_WIN) return 4095u;
  return 1u + (((uint32_t)(e - e0) << 9) | (uint32_t)((k >> 43) & 511u));
}

// block-wide exclusive scan of one u32 per thread (MB_T threads) + total
__device__ __forceinline__ uint32_t mb_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < MB_T / 64; ++w) {
    const uint32_t x = wsum[w];
    before += w < wave ? x : 0u;
    tot += x;
  }
  *total = tot;
  __syncthreads();
  return before + incl - v;
}

// Find the bin holding the need-th key of a 4096-bin global histogram written by the previous launch's
// atomics (complete at the launch boundary; this launch starts with invalidated vector caches, so plain
// 16-byte loads read the L2 copies): returns bin, updates need to the rank inside it. Every thread gets the result.
__device__ __forceinline__ int mb_pick(const uint32_t* h, int64_t& need, uint32_t* wsum, int64_t* sh) {
  uint32_t loc[16], sum = 0;
  const uint4* h4 = reinterpret_cast<const uint4*>(h + threadIdx.x * 16);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint4 v = h4[i];
    loc[4 * i] = v.x;
    loc[4 * i + 1] = v.y;
    loc[4 * i + 2] = v.z;
    loc[4 * i + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) sum += loc[i];
  uint32_t tot;
  const uint32_t before = mb_scan(sum, wsum, &tot);
  if ((int64_t)before < need && (int64_t)(before + sum) >= need) {
    int64_t n2 = need - before;
    int bin = -1;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (bin < 0) {
        if ((int64_t)loc[i] >= n2) bin = threadIdx.x * 16 + i;
        else n2 -= loc[i];
      }
    sh[0] = bin;
    sh[1] = n2;
  }
  __syncthreads();
  const int bin = (int)sh[0];
  need = sh[1];
  __syncthreads();
  return bin;
}

// arrival ticket of a pass: true in the workgroup that finishes last (its earlier writes and every other
// workgroup's are then visible to it at device scope). One lane fences: the workgroup barrier orders every wave's
// stores before thread 0's agent-scope release (an L2 write-back, not per-lane state), and thread 0's acquire before
// the barrier that releases the other waves of the last workgroup (MI355X_MICROARCH.md: a fence by every lane of a
// 1024-thread workgroup costs several times one lane's)
#ifndef MM_PER_ONE_FENCE
#define MM_PER_ONE_FENCE 1
#endif
__device__ __forceinline__ bool mb_last(uint32_t* ticket, uint32_t* s_last) {
#if MM_PER_ONE_FENCE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores are in L2 before the barrier
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const bool l = atomicAdd(ticket, 1u) == gridDim.x - 1;
    if (l) __threadfence();
    *s_last = l ? 1u : 0u;
  }
  __syncthreads();
  return *s_last != 0;
#else
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) *s_last = atomicAdd(ticket, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  const bool last = *s_last != 0;
  if (last) __threadfence();
  return last;
#endif
}

// The chunk's last TD / store step (td_chunk_kernel, rollout.hip; cal_td_error + the chunk lists,
// vdn/_utils.py:44-52, vdn/main.py:140-167): thread per (env, agent), agent-order sums per env.
__device__ void mb_td_fold(TdFuse t, int64_t E, int N, float (*sh)[MB_T]) {
  const int epb = MB_T / N;
  const int le = threadIdx.x / N, k = threadIdx.x % N;
  if (t.counter && blockIdx.x == 0 && threadIdx.x == 0) *t.counter += 1;   // RNG stream of the next step
  for (int64_t g0 = blockIdx.x; g0 * epb < E; g0 += gridDim.x) {
    const int64_t e = g0 * epb + le;
    const bool on = le < epb && e < E;
    float r = 0.f, q = 0.f, m = 0.f;
    if (on) {
      const int64_t o = e * N + k;
      const int64_t row = t.rows[e];
      r = t.rew[o];
      q = t.q_taken[o];
      m = t.maxq[o];
      t.s_act[(row * t.C + t.slot) * N + k] = (uint8_t)t.act[o];
      t.s_rew[(row * t.C + t.slot) * N + k] = r;
      if (k == 0) t.s_done[row * t.C + t.slot] = t.done[e];
    }
    sh[0][threadIdx.x] = r;
    sh[1][threadIdx.x] = q;
    sh[2][threadIdx.x] = m;
    __syncthreads();
    if (on && k == 0) {
      float sr = 0.f, sq = 0.f, sm = 0.f;
      for (int j = 0; j < N; ++j) {
        sr += sh[0][threadIdx.x + j];
        sq += sh[1][threadIdx.x + j];
        sm += sh[2][threadIdx.x + j];
      }
      const float d = t.done[e] ? 1.0f : 0.0f;
      const float td = rollout_td(sr, sq, sm, d, t.gamma);
      t.chunk_td[e] = (t.slot == 0 ? 0.0f : t.chunk_td[e]) + td;
    }
    __syncthreads();
  }
}

// pass A's histogram part, run by workgroup b of the nb histogram workgroups
__device__ __forceinline__ void mb_sel1_hist(const double* __restrict__ tree, int64_t cap, const PerDev* st, int64_t K,
                                             MbScratch* mb, int b, int nb) {
  __shared__ uint32_t h[4096];
  // the candidate list of the previous insert was last read by its apply launch, which has finished
  if (b == 0 && threadIdx.x == 0) mb->cand_n = 0;
  for (int i = b * MB_T + threadIdx.x; i < 4096; i += nb * MB_T) mb->hist2[i] = 0;   // (last read by apply)
  const int64_t n_data = st->n_data;
  if (K - min(K, cap - n_data) <= 0) return;
  const int e0 = mb->ewin;
  const double* leaves = tree + (cap - 1);
  for (int i = threadIdx.x; i < 4096; i += MB_T) h[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)b * MB_SLOTS;
#pragma unroll
  for (int i = 0; i < MB_VPT; ++i) {
    const int64_t sl = base + threadIdx.x + i * MB_T;
    if (sl < n_data) atomicAdd(&h[mb_bin1(leaf_key(leaves, sl), e0)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 4096; i += MB_T)
    if (h[i]) atomicAdd(&mb->hist1[i], h[i]);
}

__global__ __launch_bounds__(MB_T) void per_mb_sel1(const double* __restrict__ tree, int64_t cap, const PerDev* st,
                                                    int64_t K, MbScratch* mb, TdFuse tdf, int32_t td_n) {
  __shared__ float shtd[3][MB_T];
  if (tdf.on) mb_td_fold(tdf, K, td_n, shtd);
  mb_sel1_hist(tree, cap, st, K, mb, blockIdx.x, gridDim.x);
}

// pass A with the chunk-persistent rollout's TD / store fold of the chunk's last span (rollout_fold.h) in the same
// grid: workgroups [0, nh) build the histogram of the existing leaves, the rest fold 16 envs each. Independent work
// (the histogram reads only leaves, the fold writes chunk_td and the store rows that only apply reads), one launch
// instead of two.
template <bool VEC>
__global__ __launch_bounds__(MB_T) void per_mb_sel1_fold(const double* __restrict__ tree, int64_t cap,
                                                         const PerDev* st, int64_t K, MbScratch* mb, int nh,
                                                         FoldArgs fa) {
  if (mb_skip(fa.err)) return;
  if ((int)blockIdx.x < nh) {
    PER_STAMP(0, 0);
    mb_sel1_hist(tree, cap, st, K, mb, blockIdx.x, nh);
    PER_STAMP(0, 1);
  } else {
    td_fold_group<VEC>(fa, (int)blockIdx.x - nh);
  }
}

// Every workgroup of sel2 / apply re-derives the previous pass's decision itself from the finished global
// histogram (the launch boundary orders it after every atomic of the previous pass), so no pass needs an arrival
// ticket and its device-scope fences.
// bins[bin] += 1 for this lane when on: one LDS atomic per wave when every active lane has the same bin (the
// common case inside a tie-heavy candidate list), per-lane atomics otherwise
__device__ __forceinline__ void mb_bin_add(uint32_t* bins, bool on, uint32_t bin) {
  const uint64_t act = __ballot(on);
  if (!act) return;
  const int first = __builtin_ctzll(act);
  const uint32_t b0 = __shfl(bin, first);
  if (__ballot(on && bin == b0) == act) {
    if ((threadIdx.x & 63) == first) atomicAdd(&bins[b0], (uint32_t)__popcll(act));
  } else if (on) {
    atomicAdd(&bins[bin], 1u);
  }
}

__global__ __launch_bounds__(MB_T) void per_mb_sel2(const double* __restrict__ tree, int64_t cap, const PerDev* st,
                                                    int64_t K, MbScratch* mb, const uint32_t* skip_err) {
  __shared__ uint32_t h[4096];
  __shared__ uint32_t wsum[MB_T / 64];
  __shared__ int64_t sh[2];
  if (mb_skip(skip_err)) return;
  const int64_t n_data = st->n_data;
  int64_t need = K - min(K, cap - n_data);
  if (need <= 0) return;
  PER_STAMP(1, 0);
  // this block's keys first: their loads overlap the pick's round trip
  const double* leaves = tree + (cap - 1);
  const int64_t base = (int64_t)blockIdx.x * MB_SLOTS;
  uint64_t kk[MB_VPT];
#pragma unroll
  for (int i = 0; i < MB_VPT; ++i) {
    const int64_t sl = base + threadIdx.x + i * MB_T;
    kk[i] = sl < n_data ? leaf_key(leaves, sl) : ~0ull;
  }
  const uint32_t b1 = (uint32_t)mb_pick(mb->hist1, need, wsum, sh);
  PER_STAMP(1, 1);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    mb->sel[0] = b1;
    mb->sel[1] = (uint64_t)need;
  }
  for (int i = threadIdx.x; i < 4096; i += MB_T) h[i] = 0;
  __syncthreads();
  uint64_t* ckey = mb->cand;
  uint64_t* cslot = mb->cand + cap;
  uint32_t below = 0, nc = 0;
  bool isc[MB_VPT];
  const int e0 = mb->ewin;
#pragma unroll
  for (int i = 0; i < MB_VPT; ++i) {
    const int64_t sl = base + threadIdx.x + i * MB_T;
    const uint32_t bb = mb_bin1(kk[i], e0);
    below += (sl < n_data && bb < b1) ? 1u : 0u;
    isc[i] = sl < n_data && bb == b1;
    nc += isc[i] ? 1u : 0u;
    mb_bin_add(h, isc[i], (uint32_t)(kk[i] >> 31) & 4095u);   // wave-aggregated: a tie bin is one atomic per wave
  }
  // the keys in b1 listed with ONE cand_n reservation per block (per-wave atomics on one counter serialize): a block
  // scan of (below, listed) packed in 16-bit halves (each <= 1024)
  uint32_t tb;
  const uint32_t ex = mb_scan((below << 16) | nc, wsum, &tb);   // (its barriers also order the h atomics)
  if (threadIdx.x == 0) {
    mb->blk[blockIdx.x] = tb >> 16;
    sh[0] = (tb & 0xFFFFu) ? (int64_t)atomicAdd(&mb->cand_n, tb & 0xFFFFu) : 0;
  }
  __syncthreads();
  uint32_t at = (uint32_t)sh[0] + (ex & 0xFFFFu);
#pragma unroll
  for (int i = 0; i < MB_VPT; ++i)
    if (isc[i]) {
      ckey[at] = kk[i];
      cslot[at] = (uint64_t)(base + threadIdx.x + i * MB_T);
      ++at;
    }
  for (int i = threadIdx.x; i < 4096; i += MB_T)
    if (h[i]) atomicAdd(&mb->hist2[i], h[i]);
  PER_STAMP(1, 2);
}

// Block-wide min / max of a u64 (MB_T threads); every thread gets both.
__device__ __forceinline__ void mb_minmax(uint64_t& lo, uint64_t& hi, uint64_t* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[2 * wave] = lo;
    red[2 * wave + 1] = hi;
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < MB_T / 64; ++w) {
    lo = red[2 * w] < lo ? red[2 * w] : lo;
    hi = red[2 * w + 1] > hi ? red[2 * w + 1] : hi;
  }
  __syncthreads();
}


// The exact threshold key T (radix select) and this workgroup's victim offsets: lt_off = keys < T in the
// workgroups before it, eq_off = keys == T in them. Run by every workgroup. The second histogram (sel2) narrows an
// interior first-level bin (19-bit prefix) to a 31-bit prefix, so ONE pass over the listed keys (coalesced loads
// issued ahead, no global atomics) counts the earlier workgroups' keys below the prefix and compacts those with it
// into LDS (key, workgroup); the radix digits then run over that short list, from its highest differing bit (a list
// of equal keys — ties are common: envs that stay greedy from an episode start repeat each other's chunks — needs no
// pass at all). An edge bin (keys outside the first level's binades) takes every listed key as a candidate.
__device__ void mb_threshold(const MbScratch* mb, int64_t cap, uint64_t* cl, uint16_t* cb, uint32_t* bins,
                             uint32_t* wsum, int64_t* sh, uint32_t* s_n, uint64_t& T, int64_t& take_eq,
                             int64_t& lt_off, int64_t& eq_off) {
  const uint32_t b1 = (uint32_t)mb->sel[0];
  int64_t need = (int64_t)mb->sel[1];
  const bool edge = b1 == 0u || b1 == 4095u;
  const uint64_t* ckey = mb->cand;
  const uint64_t* cslot = mb->cand + cap;
  // the listed keys' first PF * MB_T entries are loaded before the pick (their latency overlaps its round trip)
  constexpr int PF = 4;
  const uint32_t m = mb->cand_n;
  uint64_t kf[PF], sf[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    const uint32_t i = q * MB_T + threadIdx.x;
    kf[q] = i < m ? ckey[i] : 0;
    sf[q] = i < m ? cslot[i] : 0;
  }
  uint64_t pre = 0;   // interior b1: the candidates' 33-bit prefix (sign, exponent, 21 mantissa bits)
  if (!edge) {
    const uint64_t p21 = ((uint64_t)(((b1 - 1u) >> 9) + (uint32_t)mb->ewin) << 9) | ((b1 - 1u) & 511u);
    pre = (p21 << 12) | (uint64_t)mb_pick(mb->hist2, need, wsum, sh);
  }
  PER_STAMP(3, 1);
  auto is_cand = [&](uint64_t k) { return edge || (k >> 31) == pre; };
  const uint32_t me = blockIdx.x;
  if (threadIdx.x == 0) *s_n = 0;
  __syncthreads();
  uint32_t lt = 0;
  uint64_t lo = ~0ull, hi = 0;
  for (uint32_t i00 = 0; i00 < m; i00 += PF * MB_T) {
    uint64_t kq[PF], sq[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {   // this round's keys (loaded last round), the next round's loads issued
      const uint32_t i = i00 + (PF + q) * MB_T + threadIdx.x;
      kq[q] = kf[q];
      sq[q] = sf[q];
      kf[q] = i < m ? ckey[i] : 0;
      sf[q] = i < m ? cslot[i] : 0;
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const uint32_t i = i00 + q * MB_T + threadIdx.x;
      const uint64_t k = kq[q], blk = sq[q] / MB_SLOTS;
      lt += (i < m && !edge && (k >> 31) < pre && blk < me) ? 1u : 0u;
      const bool in = i < m && is_cand(k);
      if (in) {
        lo = k < lo ? k : lo;
        hi = k > hi ? k : hi;
      }
      const uint64_t w = __ballot(in);
      if (w) {
        const int lane = threadIdx.x & 63, first = __builtin_ctzll(w);
        uint32_t at0 = 0;
        if (lane == first) at0 = atomicAdd(s_n, (uint32_t)__popcll(w));
        at0 = __shfl(at0, first);
        const uint32_t at = at0 + (uint32_t)__popcll(w & ((1ull << lane) - 1ull));
        if (in && at < (uint32_t)MB_CAND_LDS) {
          cl[at] = k;
          cb[at] = (uint16_t)blk;
        }
      }
    }
  }
  mb_minmax(lo, hi, reinterpret_cast<uint64_t*>(bins));   // (its barriers publish the compacted list)
  const uint32_t n = *s_n;
  PER_STAMP(3, 2);
  PER_NOTE(6, m);
  PER_NOTE(7, n);
  const bool in_lds = n <= (uint32_t)MB_CAND_LDS;
  // candidate j: from LDS, or (overflow: tens of thousands of exactly equal keys, or an edge bin's list) filtered
  // from the global list on every pass
  uint64_t prefix = lo & (lo == hi ? ~0ull : (~0ull << (64 - __clzll(lo ^ hi))));
  int top = (n == 0 || lo == hi) ? -1 : 63 - __clzll(lo ^ hi);
  if (top >= 0 && in_lds && n <= (uint32_t)MB_T) {
    // a short list of distinct keys: candidate i's rank among the n by direct comparison (no radix passes)
    if (threadIdx.x < n) {
      const uint64_t k = cl[threadIdx.x];
      uint32_t less = 0, eq = 0;
      for (uint32_t j = 0; j < n; ++j) {
        less += cl[j] < k ? 1u : 0u;
        eq += cl[j] == k ? 1u : 0u;
      }
      if ((int64_t)less < need && need <= (int64_t)(less + eq)) {   // (equal keys write the same values)
        sh[0] = (int64_t)k;
        sh[1] = need - less;
      }
    }
    __syncthreads();
    prefix = (uint64_t)sh[0];
    need = sh[1];
    top = -1;
    __syncthreads();
  }
  for (int shift = top - 7; top >= 0; shift -= 8) {
    const int sft = shift < 0 ? 0 : shift;
    const int width = shift < 0 ? shift + 8 : 8;
    for (int i = threadIdx.x; i < 256; i += MB_T) bins[i] = 0;
    __syncthreads();
    const uint64_t hmask = ~0ull << (sft + width);
    const uint32_t dmask = (1u << width) - 1u;
    const uint32_t cnt = in_lds ? n : m;
    for (uint32_t i0 = 0; i0 < cnt; i0 += MB_T) {
      const uint32_t i = i0 + threadIdx.x;
      const uint64_t k = i < cnt ? (in_lds ? cl[i] : ckey[i]) : 0;
      const bool on = i < cnt && is_cand(k) && (k & hmask) == prefix;
      mb_bin_add(bins, on, (uint32_t)(k >> sft) & dmask);
    }
    __syncthreads();
    const uint32_t v = bins[threadIdx.x];
    uint32_t tot;
    const uint32_t before = mb_scan(v, wsum, &tot);
    if ((int64_t)before < need && (int64_t)(before + v) >= need) {
      sh[0] = threadIdx.x;
      sh[1] = need - before;
    }
    __syncthreads();
    prefix |= (uint64_t)sh[0] << sft;
    need = sh[1];
    __syncthreads();
    if (shift <= 0) break;
  }
  PER_STAMP(3, 3);
  T = prefix;        // the rest-th smallest key; the first `need` slots equal to it are taken
  take_eq = need;
  uint32_t eq = 0;
  for (uint32_t b = threadIdx.x; b < me; b += MB_T) lt += mb->blk[b];
  if (in_lds) {
    for (uint32_t i = threadIdx.x; i < n; i += MB_T)
      if (cb[i] < me) {
        lt += cl[i] < T ? 1u : 0u;
        eq += cl[i] == T ? 1u : 0u;
      }
  } else {
    for (uint32_t i = threadIdx.x; i < m; i += MB_T) {
      const uint64_t k = ckey[i];
      if (!is_cand(k) || (uint32_t)(cslot[i] / MB_SLOTS) >= me) continue;
      lt += k < T ? 1u : 0u;
      eq += k == T ? 1u : 0u;
    }
  }
  uint32_t tl, te;
  (void)mb_scan(lt, wsum, &tl);
  (void)mb_scan(eq, wsum, &te);
  lt_off = tl;
  eq_off = te;
  PER_STAMP(3, 4);
}

// prio (the fold path): the new chunks' priorities, computed by the fold; else (td + eps)^alpha here
__global__ __launch_bounds__(MB_T) void per_mb_apply(double* tree, int64_t* slot_row, int64_t cap, PerDev* st,
                                                     const float* td, const double* prio, int64_t K, double eps,
                                                     int64_t* rows_inout, int64_t* slots_out, MbScratch* mb,
                                                     const uint32_t* skip_err) {
  __shared__ double lv[MB_SLOTS];
  __shared__ double v[2][MB_SLOTS / 2];
  __shared__ uint64_t cl[MB_CAND_LDS];
  __shared__ uint16_t cb[MB_CAND_LDS];
  __shared__ uint32_t s_n;
  __shared__ __attribute__((aligned(16))) uint32_t bins[256];   // mb_minmax reuses it as uint64_t
  __shared__ uint32_t wsum[MB_T / 64];
  __shared__ int64_t sh[2];
  __shared__ uint32_t s_last;
  if (mb_skip(skip_err)) return;
  const int L = 63 - __clzll((unsigned long long)cap);      // leaves at level L
  const int64_t n_data = st->n_data;
  const double alpha = st->alpha;
  const int64_t free_n = min(K, cap - n_data);
  const bool evict = K - free_n > 0;
  double* leaves = tree + (cap - 1);
  PER_STAMP(3, 0);
  const int64_t base = (int64_t)blockIdx.x * MB_SLOTS;
  // this block's 1024 leaves: 4 contiguous per thread (keys for the victim test, LDS copy for the
  // rebuild) and their store rows, loaded first so the latency overlaps the threshold selection
  const int64_t s0 = base + threadIdx.x * MB_VPT;
  double x[MB_VPT];
  int64_t srow[MB_VPT] = {0, 0, 0, 0};
  {
    const double2 a = ld_double2(leaves + s0);
    const double2 b = ld_double2(leaves + s0 + 2);
    x[0] = a.x;
    x[1] = a.y;
    x[2] = b.x;
    x[3] = b.y;
    if (rows_inout) {
      const longlong2 ra = *reinterpret_cast<const longlong2*>(slot_row + s0);
      const longlong2 rb = *reinterpret_cast<const longlong2*>(slot_row + s0 + 2);
      srow[0] = ra.x;
      srow[1] = ra.y;
      srow[2] = rb.x;
      srow[3] = rb.y;
    }
  }
  uint64_t T = 0;
  int64_t take_eq = 0, lt_off = 0, eq_off = 0;
  if (evict) {
    mb_threshold(mb, cap, cl, cb, bins, wsum, sh, &s_n, T, take_eq, lt_off, eq_off);
    // hist1 was last read by sel2 (finished): cleared here for the next insert
    for (int i = blockIdx.x * MB_T + threadIdx.x; i < 4096; i += gridDim.x * MB_T) mb->hist1[i] = 0;
  }
  uint32_t lt = 0, eq = 0;
  if (evict) {
#pragma unroll
    for (int i = 0; i < MB_VPT; ++i) {
      const uint64_t k = s0 + i < n_data ? (uint64_t)__double_as_longlong(x[i]) : ~0ull;
      lt += k < T ? 1u : 0u;
      eq += k == T ? 1u : 0u;
    }
  }
  uint32_t tot;
  int64_t lt_rank = mb_scan(lt, wsum, &tot);
  int64_t eq_rank = mb_scan(eq, wsum, &tot);
  lt_rank += lt_off;
  eq_rank += eq_off;
  PER_STAMP(3, 8);
  // the insert index j of each of the thread's slots (-1: kept), then every load of the new chunks' data at once,
  // then the stores (one global round trip per thread, not one per slot behind the previous slot's stores)
  int64_t jj[MB_VPT];
#pragma unroll
  for (int i = 0; i < MB_VPT; ++i) {
    const int64_t sl = s0 + i;
    int64_t j = -1;
    if (sl >= n_data && sl < n_data + free_n) {
      j = sl - n_data;                                   // a free slot, filled in order
    } else if (evict && sl < n_data) {
      const uint64_t k = (uint64_t)__double_as_longlong(x[i]);
      if (k < T) {
        j = free_n + lt_rank + min(eq_rank, take_eq);    // victims in ascending slot order
        ++lt_rank;
      } else if (k == T) {
        if (eq_rank < take_eq) j = free_n + lt_rank + eq_rank;
        ++eq_rank;
      }
    }
    jj[i] = j;
  }
  double pv[MB_VPT];
  int64_t rin[MB_VPT];
#pragma unroll
  for (int i = 0; i < MB_VPT; ++i) {
    pv[i] = jj[i] < 0 ? 0.0 : (prio ? prio[jj[i]] : (double)td[jj[i]]);
    rin[i] = (jj[i] >= 0 && rows_inout) ? rows_inout[jj[i]] : 0;
  }
  PER_STAMP(3, 9);
#pragma unroll
  for (int i = 0; i < MB_VPT; ++i) {
    const int64_t sl = s0 + i, j = jj[i];
    if (j >= 0) {
      x[i] = prio ? pv[i] : pow(pv[i] + eps, alpha);
      leaves[sl] = x[i];
      if (slots_out) slots_out[j] = sl;
      if (rows_inout) {
        slot_row[sl] = rin[i];
        rows_inout[j] = srow[i];
      }
    }
    lv[threadIdx.x * MB_VPT + i] = x[i];
  }
  PER_STAMP(3, 10);
  __syncthreads();
  PER_STAMP(3, 5);
  // levels L-1 .. L-10 of this block's subtree from the LDS leaves (pairwise f64 sums = rebuild_tree)
  {
    const int64_t o = ((int64_t)1 << (L - 1)) - 1 + (int64_t)blockIdx.x * (MB_SLOTS / 2);
    for (int i = threadIdx.x; i < MB_SLOTS / 2; i += MB_T) {
      v[0][i] = lv[2 * i] + lv[2 * i + 1];
      tree[o + i] = v[0][i];
    }
  }
  __syncthreads();
  int cur = 0;
  for (int n = MB_SLOTS / 4, l = L - 2; n >= 1; n >>= 1, --l) {
    const int64_t o = ((int64_t)1 << l) - 1 + (int64_t)blockIdx.x * n;
    for (int i = threadIdx.x; i < n; i += MB_T) {
      const double y = v[cur][2 * i] + v[cur][2 * i + 1];
      v[cur ^ 1][i] = y;
      tree[o + i] = y;
    }
    cur ^= 1;
    __syncthreads();
  }
  PER_STAMP(3, 6);
  if (!mb_last(&mb->ticket, &s_last)) return;
  // the last block: the levels above the per-block roots
  const int G = gridDim.x, lg = L - 10;                     // G = 2^lg roots at level lg (G <= 1024)
  if (G <= 64) {   // one wave: root i in lane i, each level's pairwise sums by lane shuffles (no block barriers)
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    double y = lane < G ? __hip_atomic_load(&tree[((int64_t)1 << lg) - 1 + lane], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT)
                        : 0.0;
    for (int n = G / 2, l = lg - 1; n >= 1; n >>= 1, --l) {
      const double a = __shfl(y, (2 * lane) & 63), b = __shfl(y, (2 * lane + 1) & 63);
      y = a + b;
      if (lane < n) tree[((int64_t)1 << l) - 1 + lane] = y;
    }
    if (lane == 0) {
      mb->ticket = 0;
      st->n_data = min(cap, n_data + K);
      if (evict) mb->ewin = min(max((int)(T >> 52) - 3, 0), 2047 - MB_WIN);   // the next insert's window
    }
    PER_STAMP(3, 7);
    return;
  }
  double* w = &lv[0];
  for (int i = threadIdx.x; i < G; i += MB_T)
    w[i] = __hip_atomic_load(&tree[((int64_t)1 << lg) - 1 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  for (int n = G / 2, l = lg - 1; n >= 1; n >>= 1, --l) {
    double y[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = threadIdx.x + q * MB_T;
      y[q] = i < n ? w[2 * i] + w[2 * i + 1] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = threadIdx.x + q * MB_T;
      if (i < n) {
        w[i] = y[q];
        tree[((int64_t)1 << l) - 1 + i] = y[q];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    mb->ticket = 0;
    st->n_data = min(cap, n_data + K);
    if (evict) mb->ewin = min(max((int)(T >> 52) - 3, 0), 2047 - MB_WIN);   // the next insert's window
  }  PER_STAMP(3, 7);
}

// the chunk's last TD / store on its own (the single-workgroup insert paths)
__global__ __launch_bounds__(MB_T) void per_td_fold_kernel(TdFuse tdf, int64_t E, int N) {
  __shared__ float shtd[3][MB_T];
  mb_td_fold(tdf, E, N, shtd);
}

static int per_insert_mb(mm_per* per, const float* td, int64_t k, int64_t* rows_inout, int64_t* slots_out,
                         const TdFuse* tdf, int32_t td_n, hipStream_t s, const FoldArgs* fold = nullptr) {
  const int64_t cap = per->cap;
  const int G = (int)(cap / MB_SLOTS);
  MbScratch* mb = static_cast<MbScratch*>(per->mb);
  TdFuse t{};
  if (tdf) t = *tdf;
  double* prio = nullptr;
  if (fold) {
    FoldArgs fa = *fold;
    fa.prio = prio = mb_prio(mb, cap);
    fa.alpha = &per->st->alpha;
    fa.eps = per->eps;
    const int fb = (fold->E + 15) / 16;
    auto kern = fold_vec_ok(fa) ? per_mb_sel1_fold<true> : per_mb_sel1_fold<false>;
    hipLaunchKernelGGL(kern, dim3(G + fb), dim3(MB_T), 0, s, per->tree, cap, per->st, k, mb, G, fa);
  } else {
    hipLaunchKernelGGL(per_mb_sel1, dim3(G), dim3(MB_T), 0, s, per->tree, cap, per->st, k, mb, t, td_n);
  }
  const uint32_t* skip_err = fold ? fold->err : nullptr;
  hipLaunchKernelGGL(per_mb_sel2, dim3(G), dim3(MB_T), 0, s, per->tree, cap, per->st, k, mb, skip_err);
  hipLaunchKernelGGL(per_mb_apply, dim3(G), dim3(MB_T), 0, s, per->tree, per->slot_row, cap, per->st, td, prio, k,
                     per->eps, rows_inout, slots_out, mb, skip_err);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}
}  // namespace mm

#if MM_PER_TRACE
extern "C" int mm_per_trace_copy(uint64_t* out) {   // trace builds only: [4][64][8] stamps
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mm::g_per_trace), sizeof(mm::g_per_trace)) == hipSuccess ? 0 : -1;   // [4][64][16]
}
#endif

extern "C" {

int mm_per_create(int64_t capacity, int32_t flavor, double alpha, double beta, double eps, double step_weight,
                  int32_t use_step_weight, double alpha_inc, double beta_inc, mm_per** out) {
  MM_REQUIRE(out && capacity >= 1 && capacity < (1ll << 30), "per_create: bad capacity");
  mm_per* p = new mm_per;
  p->cap = capacity;
  p->flavor = flavor;
  p->alpha = alpha;
  p->beta = beta;
  p->eps = eps;
  p->step_weight = step_weight;
  p->use_step_weight = use_step_weight && flavor == MM_PER_VDN;
  p->alpha_inc = alpha_inc;
  p->beta_inc = beta_inc;
  p->n_data = 0;
  const size_t tree_b = ((size_t)(2 * capacity - 1) * 8 + 255) & ~size_t(255);
  const size_t row_b = ((size_t)capacity * 8 + 255) & ~size_t(255);
  const size_t scr_b = (size_t)capacity * 8;
  const size_t last_b = ((size_t)capacity * 4 + 255) & ~size_t(255);
  void* base = nullptr;
  if (hipMalloc(&base, tree_b + row_b + scr_b + 256 + last_b) != hipSuccess) {
    delete p;
    mm::set_error("per_create: hipMalloc failed");
    return MM_ENOMEM;
  }
  p->alloc = base;
  p->tree = static_cast<double*>(base);
  p->st = reinterpret_cast<mm::PerDev*>(static_cast<char*>(base) + tree_b + row_b + scr_b);
  const mm::PerDev st0 = {0, alpha, beta, alpha_inc, beta_inc, 0};
  p->slot_row = reinterpret_cast<int64_t*>(static_cast<char*>(base) + tree_b);
  p->last = reinterpret_cast<int32_t*>(static_cast<char*>(base) + tree_b + row_b + scr_b + 256);
  std::vector<int64_t> rows(capacity);
  for (int64_t i = 0; i < capacity; ++i) rows[i] = i;  // slot s reserves row s until first filled
  if (hipMemset(p->tree, 0, tree_b) != hipSuccess || hipMemset(p->last, 0xFF, last_b) != hipSuccess ||
      hipMemcpy(p->slot_row, rows.data(), capacity * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(p->st, &st0, sizeof(st0), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(base);
    delete p;
    mm::set_error("per_create: init failed");
    return MM_EHIP;
  }
  p->mb = nullptr;
  if ((capacity & (capacity - 1)) == 0 && capacity >= mm::MB_MIN_CAP && capacity <= (1ll << 20)) {
    const int32_t ewin0 = mm::MB_EWIN0;   // the first-level window of the first insert: 2^-3 .. 2^4
    if (hipMalloc(&p->mb, mm::mb_bytes(capacity)) != hipSuccess || hipMemset(p->mb, 0, mm::mb_bytes(capacity)) != hipSuccess ||
        hipMemcpy(&static_cast<mm::MbScratch*>(p->mb)->ewin, &ewin0, 4, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(base);
      delete p;
      mm::set_error("per_create: scratch allocation failed");
      return MM_ENOMEM;
    }
  }
  *out = p;
  return MM_OK;
}

void mm_per_destroy(mm_per* per) {
  if (!per) return;
  (void)hipFree(per->alloc);
  if (per->mb) (void)hipFree(per->mb);
  delete per;
}

static int64_t* per_scratch(mm_per* p) {
  const size_t tree_b = ((size_t)(2 * p->cap - 1) * 8 + 255) & ~size_t(255);
  const size_t row_b = ((size_t)p->cap * 8 + 255) & ~size_t(255);
  return reinterpret_cast<int64_t*>(static_cast<char*>(p->alloc) + tree_b + row_b);
}

static int per_insert_impl(mm_per* per, const float* td, int64_t k, int64_t* rows_inout, int64_t* slots_out,
                           const mm::TdFuse* tdf, int32_t td_n, hipStream_t s) {
  MM_REQUIRE(per && (td || k == 0), "per_add: null argument");
  MM_REQUIRE(k >= 0 && k <= per->cap, "per_add: batch %lld larger than capacity", (long long)k);
  if (k == 0) return MM_OK;
  const int64_t cap = per->cap;
  const bool pow2 = (cap & (cap - 1)) == 0;
  const int64_t vpt = cap / mm::PT;
  if (per->mb) {
    const int rc = mm::per_insert_mb(per, td, k, rows_inout, slots_out, tdf, td_n, s);
    if (rc) return rc;
    per->n_data = std::min(per->cap, per->n_data + k);
    return MM_OK;
  }
  if (tdf) {   // the other insert paths run the chunk's last TD / store as its own launch first
    const int64_t epb = mm::MB_T / td_n;
    const int g = (int)std::min<int64_t>((k + epb - 1) / epb, 1024);
    hipLaunchKernelGGL(mm::per_td_fold_kernel, dim3(g), dim3(mm::MB_T), 0, s, *tdf, k, td_n);
    MM_HIP_CHECK(hipGetLastError());
  }
  if (pow2 && cap >= 2 * mm::PT && vpt <= 64 && k <= mm::FAST_MAX_VICTIMS) {
#define MM_PER_FAST(V)                                                                                        \
  case V:                                                                                                     \
    hipLaunchKernelGGL(mm::per_add_fast_kernel<V>, dim3(1), dim3(mm::PT), 0, s, per->tree, per->slot_row, cap, \
                       per->st, td, k, per->eps, rows_inout, slots_out);                                      \
    break;
    switch (vpt) {
      MM_PER_FAST(2)
      MM_PER_FAST(4)
      MM_PER_FAST(8)
      MM_PER_FAST(16)
      MM_PER_FAST(32)
      MM_PER_FAST(64)
    }
#undef MM_PER_FAST
  } else {
    hipLaunchKernelGGL(mm::per_add_kernel, dim3(1), dim3(mm::PT), 0, s, per->tree, per->slot_row, cap, per->st, td, k,
                       per->eps, rows_inout, slots_out, per_scratch(per));
  }
  MM_HIP_CHECK(hipGetLastError());
  per->n_data = std::min(per->cap, per->n_data + k);
  return MM_OK;
}

int mm_per_insert(mm_per* per, const float* td, int64_t k, int64_t* rows_inout, int64_t* slots_out, mm_stream_t s) {
  return per_insert_impl(per, td, k, rows_inout, slots_out, nullptr, 0, (hipStream_t)s);
}

int mm_per_insert_fold(mm_per* per, int64_t k, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                       const float* q_taken, const float* max_q_next, const int32_t* act, int64_t ring_se,
                       int32_t slot0, int32_t n_slots, int32_t chunk_len, float* chunk_td, uint8_t* store_act,
                       float* store_rew, uint8_t* store_done, int64_t* rows_inout, int64_t n_rows, int32_t* err,
                       int64_t* slots_out, mm_stream_t s) {
  MM_REQUIRE(per && rew && done && q_taken && max_q_next && act && chunk_td && store_act && store_rew && store_done &&
                 rows_inout, "per_insert_fold: null argument");
  MM_REQUIRE(n_slots >= 1 && slot0 >= 0 && slot0 + n_slots == chunk_len,
             "per_insert_fold: the slots [slot0, slot0 + n) must end the chunk");
  MM_REQUIRE(n_agents >= 1 && n_agents <= 256 && ring_se >= k * n_agents, "per_insert_fold: bad agents / ring");
  MM_REQUIRE(k >= 1 && k <= per->cap, "per_insert_fold: batch %lld outside [1, capacity]", (long long)k);
  if (!per->mb) {   // (the single-workgroup insert paths: the fold as its own launch, then the insert)
    const int rc = mm_td_fold_range(k, n_agents, gamma, rew, done, q_taken, max_q_next, act, ring_se, slot0, n_slots,
                                    chunk_len, chunk_td, store_act, store_rew, store_done, rows_inout, n_rows, err, s);
    if (rc) return rc;
    return per_insert_impl(per, chunk_td, k, rows_inout, slots_out, nullptr, 0, (hipStream_t)s);
  }
  const mm::FoldArgs fa{rew, done, q_taken, max_q_next, act, chunk_td, store_act, store_rew, store_done, rows_inout,
                        reinterpret_cast<uint32_t*>(err), ring_se, n_rows, (int)k, n_agents, slot0, n_slots,
                        chunk_len, gamma};
  const int rc = mm::per_insert_mb(per, chunk_td, k, rows_inout, slots_out, nullptr, 0, (hipStream_t)s, &fa);
  if (rc) return rc;
  per->n_data = std::min(per->cap, per->n_data + k);
  return MM_OK;
}

int mm_per_insert_td(mm_per* per, int64_t k, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                     const float* q_taken, const float* max_q_next, const int32_t* act, float* chunk_td,
                     int32_t step_in_chunk, int32_t chunk_len, uint8_t* store_act, float* store_rew,
                     uint8_t* store_done, uint64_t* counter, int64_t* rows_inout, int64_t* slots_out, mm_stream_t s) {
  MM_REQUIRE(rew && done && q_taken && max_q_next && act && chunk_td && store_act && store_rew && store_done &&
                 rows_inout, "per_insert_td: null argument");
  MM_REQUIRE(step_in_chunk >= 0 && step_in_chunk < chunk_len, "per_insert_td: bad step");
  MM_REQUIRE(n_agents >= 1 && n_agents <= 256, "per_insert_td: n_agents must be in [1,256]");
  const mm::TdFuse t{rew, done, q_taken, max_q_next, act, chunk_td, store_act, store_rew, store_done, rows_inout,
                     counter, gamma, step_in_chunk, chunk_len, 1};
  return per_insert_impl(per, chunk_td, k, rows_inout, slots_out, &t, n_agents, (hipStream_t)s);
}

int mm_per_add_batch(mm_per* per, const float* td, int64_t k, int64_t* slots_out, mm_stream_t s) {
  return mm_per_insert(per, td, k, nullptr, slots_out, s);
}

int mm_per_sample_uniform(mm_per* per, int32_t batch, uint64_t seed, uint64_t counter, int64_t* slots_out,
                          float* is_w, mm_stream_t s) {
  MM_REQUIRE(per && slots_out && batch >= 1, "per_sample_uniform: bad argument");
  MM_REQUIRE(per->n_data > 0, "per_sample_uniform: empty buffer");
  hipLaunchKernelGGL(mm::per_uniform_kernel, dim3(1), dim3(1024), 0, (hipStream_t)s, per->cap, batch,
                     seed, counter, per->st, (int64_t*)nullptr, slots_out, is_w);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

// the host mirror of a sample call's annealing (buffer.py:53-56); returns the tree decay of the call
static double per_sample_prep(mm_per* per) {
  per->alpha = std::min(1.0, per->alpha + per->alpha_inc);
  per->beta = std::min(1.0, per->beta + per->beta_inc);
  return per->use_step_weight ? per->step_weight : 1.0;
}

static int per_sample_impl(mm_per* per, int32_t batch, const double* fracs, uint64_t seed, uint64_t counter,
                           int64_t* nodes_out, int64_t* slots_out, float* is_w, mm_stream_t s) {
  MM_REQUIRE(per && nodes_out && is_w, "per_sample: null argument");
  MM_REQUIRE(batch >= 1 && batch <= mm::PT * mm::PER_SAMPLE_MAXJ, "per_sample: batch must be in [1, %d]",
             mm::PT * mm::PER_SAMPLE_MAXJ);
  MM_REQUIRE(per->n_data > 0, "per_sample: empty buffer");
  const double decay = per_sample_prep(per);
  hipLaunchKernelGGL(mm::per_sample_kernel, dim3(1), dim3(mm::PT), 0, (hipStream_t)s, per->tree, per->cap, batch,
                     fracs, seed, counter, per->st, decay, nodes_out, slots_out, is_w);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_per_sample(mm_per* per, int32_t batch, const double* fracs, int64_t* nodes_out, int64_t* slots_out,
                  float* is_w, mm_stream_t s) {
  MM_REQUIRE(fracs, "per_sample: fracs required");
  return per_sample_impl(per, batch, fracs, 0, 0, nodes_out, slots_out, is_w, s);
}

int mm_per_sample_rng(mm_per* per, int32_t batch, uint64_t seed, uint64_t counter, int64_t* nodes_out,
                      int64_t* slots_out, float* is_w, mm_stream_t s) {
  return per_sample_impl(per, batch, nullptr, seed, counter, nodes_out, slots_out, is_w, s);
}

int mm_per_update(mm_per* per, const int64_t* nodes, const float* td, int32_t batch, mm_stream_t s) {
  MM_REQUIRE(per && nodes && td, "per_update: null argument");
  MM_REQUIRE(batch >= 1 && batch <= 65536, "per_update: bad batch");
  if ((per->cap & (per->cap - 1)) == 0 && batch <= mm::PU_B)
    hipLaunchKernelGGL(mm::per_update_small_kernel, dim3(1), dim3(1024), 0, (hipStream_t)s, per->tree, per->cap, nodes,
                       td, batch, per->st, (float)per->eps);
  else
    hipLaunchKernelGGL(mm::per_update_kernel, dim3(1), dim3(mm::PT), 0, (hipStream_t)s, per->tree, per->cap, nodes, td,
                       batch, per->st, (float)per->eps, per->last);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

double* mm_per_tree_ptr(mm_per* per) { return per ? per->tree : nullptr; }
int64_t* mm_per_slot_rows(mm_per* per) { return per ? per->slot_row : nullptr; }
int64_t mm_per_size(const mm_per* per) { return per ? per->n_data : -1; }
int64_t mm_per_capacity(const mm_per* per) { return per ? per->cap : -1; }
double mm_per_alpha(const mm_per* per) { return per ? per->alpha : 0.0; }
double mm_per_beta(const mm_per* per) { return per ? per->beta : 0.0; }
void mm_per_set_size_host(mm_per* per, int64_t n) {
  if (per) per->n_data = n;  // host mirror only (device state advanced by graph-replayed inserts)
}
void mm_per_set_size(mm_per* per, int64_t n) {
  if (!per) return;
  per->n_data = n;
  (void)hipMemcpy(&per->st->n_data, &n, sizeof(n), hipMemcpyHostToDevice);
}
int mm_per_error_word(mm_per* per, int32_t* host_out, int32_t clear, mm_stream_t s) {
  MM_REQUIRE(per && host_out, "per_error_word: null argument");
  MM_HIP_CHECK(hipMemcpyAsync(host_out, &per->st->err, sizeof(int32_t), hipMemcpyDeviceToHost, (hipStream_t)s));
  if (clear) MM_HIP_CHECK(hipMemsetAsync(&per->st->err, 0, sizeof(int32_t), (hipStream_t)s));
  MM_HIP_CHECK(hipStreamSynchronize((hipStream_t)s));
  return MM_OK;
}
int mm_per_copy_tree(mm_per* per, double* dst, mm_stream_t s) {
  MM_REQUIRE(per && dst, "per_copy_tree: null argument");
  MM_HIP_CHECK(hipMemcpyAsync(dst, per->tree, (size_t)(2 * per->cap - 1) * 8, hipMemcpyDeviceToDevice, (hipStream_t)s));
  return MM_OK;
}
int mm_per_copy_slot_rows(mm_per* per, int64_t* dst, mm_stream_t s) {
  MM_REQUIRE(per && dst, "per_copy_slot_rows: null argument");
  MM_HIP_CHECK(hipMemcpyAsync(dst, per->slot_row, (size_t)per->cap * 8, hipMemcpyDeviceToDevice, (hipStream_t)s));
  return MM_OK;
}

int mm_per_save_state(mm_per* per, double* tree_dst, int64_t* rows_dst, double* scalars, mm_stream_t s) {
  MM_REQUIRE(per && tree_dst && rows_dst && scalars, "per_save_state: null argument");
  MM_HIP_CHECK(hipMemcpyAsync(tree_dst, per->tree, (size_t)(2 * per->cap - 1) * 8, hipMemcpyDeviceToDevice,
                              (hipStream_t)s));
  MM_HIP_CHECK(hipMemcpyAsync(rows_dst, per->slot_row, (size_t)per->cap * 8, hipMemcpyDeviceToDevice, (hipStream_t)s));
  mm::PerDev h;
  MM_HIP_CHECK(hipMemcpyAsync(&h, per->st, sizeof(h), hipMemcpyDeviceToHost, (hipStream_t)s));
  MM_HIP_CHECK(hipStreamSynchronize((hipStream_t)s));
  scalars[0] = (double)h.n_data;
  scalars[1] = h.alpha;
  scalars[2] = h.beta;
  scalars[3] = h.alpha_inc;
  scalars[4] = h.beta_inc;
  scalars[5] = (double)h.n_samples;
  return MM_OK;
}

int mm_per_load_state(mm_per* per, const double* tree_src, const int64_t* rows_src, const double* scalars,
                      mm_stream_t s) {
  MM_REQUIRE(per && tree_src && rows_src && scalars, "per_load_state: null argument");
  MM_REQUIRE(scalars[0] >= 0 && scalars[0] <= (double)per->cap, "per_load_state: fill count out of range");
  MM_HIP_CHECK(hipMemcpyAsync(per->tree, tree_src, (size_t)(2 * per->cap - 1) * 8, hipMemcpyDeviceToDevice,
                              (hipStream_t)s));
  MM_HIP_CHECK(hipMemcpyAsync(per->slot_row, rows_src, (size_t)per->cap * 8, hipMemcpyDeviceToDevice, (hipStream_t)s));
  mm::PerDev h;
  h.n_data = (int64_t)scalars[0];
  h.alpha = scalars[1];
  h.beta = scalars[2];
  h.alpha_inc = scalars[3];
  h.beta_inc = scalars[4];
  h.n_samples = (uint64_t)scalars[5];
  h.err = 0;
  h.pad = 0;
  MM_HIP_CHECK(hipMemcpyAsync(per->st, &h, sizeof(h), hipMemcpyHostToDevice, (hipStream_t)s));
  MM_HIP_CHECK(hipStreamSynchronize((hipStream_t)s));
  per->n_data = h.n_data;
  per->alpha = h.alpha;
  per->beta = h.beta;
  return MM_OK;
}
}
