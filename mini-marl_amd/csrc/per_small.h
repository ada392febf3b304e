// PER pieces shared by per.hip and the learner's launches (learner.hip / qmix_unit.hip): the device scalars and the
// small-batch priority update body, which the learner runs as one extra block of an update launch.
#pragma once
#include <cstdint>

#include "common.h"

namespace mm {

// Mutable PER scalars live in HBM so that inserts / samples / updates are graph-replayable
// (the host keeps an identical mirror for queries).
struct PerDev {
  int64_t n_data;
  double alpha, beta, alpha_inc, beta_inc;
  uint64_t n_samples;
  int32_t err;   // sticky error bits: 1 = a priority update named a node outside the leaves (skipped)
  int32_t pad;
};

// Small batches (B <= PU_B, power-of-two capacity: every leaf at depth L): one round trip for the sample
// nodes / TDs, one for every sibling along the changed root paths, then the paths re-summed bottom-up in
// LDS — each changed node = left child + right child, the changed child from LDS, the unchanged one as
// loaded — the same f64 pairwise sums as rebuild_tree, so identical trees; duplicate nodes: the LAST
// sample index wins. (per.hip's general kernel pays a global round trip per 4 levels plus the duplicate
// scratch passes: 13.8 us at B = 32 on a 65536-leaf tree.)
constexpr int PU_B = 64, PU_L = 30;
// static LDS of the body below (34.5 KB), rounded up: what a launch carrying it has left for dynamic LDS
constexpr size_t kPerSmallLds = 36 * 1024;
// (any block of >= B threads: per_update_small_kernel's, or one extra block of a learner launch)
__device__ __forceinline__ void per_update_small_body(double* tree, int64_t cap, const int64_t* nodes, const float* td,
                                                      int B, PerDev* st, float eps) {
  __shared__ int64_t snd[PU_B];
  __shared__ float stv[PU_B];
  __shared__ double sval[PU_L + 1][PU_B];   // [depth][sample]: new value of the sample's ancestor
  __shared__ double ssib[PU_L + 1][PU_B];   // [depth][sample]: stored value of that ancestor's sibling
  __shared__ int8_t spart[PU_L + 1][PU_B];  // [depth][sample]: a sample whose path holds that sibling, or -1
  const int L = 63 - __clzll((unsigned long long)cap);
  const int t = threadIdx.x;
  const float alpha = (float)st->alpha;
  if (t < B) {
    const int64_t nd = nodes[t];
    const bool ok = nd >= cap - 1 && nd < 2 * cap - 1;
    snd[t] = ok ? nd : -1;
    stv[t] = td[t];
    if (!ok) atomicOr(&st->err, 1);
  }
  __syncthreads();
  // per (sample, depth): the sibling's stored value (one round trip for all) and whether the sibling lies on
  // another changed path (then its new value is taken instead); scans without early exit, so the LDS reads
  // of a scan are all in flight together
  for (int i = t; i < B * L; i += blockDim.x) {
    const int k = i / L, d = 1 + i % L;
    const int64_t nd = snd[k];
    if (nd >= 0) {
      const int64_t a = ((nd + 1) >> (L - d)) - 1;   // ancestor at depth d
      const int64_t sib = ((a + 1) ^ 1) - 1;
      ssib[d][k] = tree[sib];
      int part = -1;
#pragma unroll 8
      for (int k2 = B - 1; k2 >= 0; --k2) {
        const int64_t n2 = snd[k2];
        part = (n2 >= 0 && ((n2 + 1) >> (L - d)) - 1 == sib) ? k2 : part;
      }
      spart[d][k] = (int8_t)part;
    }
  }
  if (t < B && snd[t] >= 0) {
    int w = t;   // the last sample naming the same leaf
#pragma unroll 8
    for (int k2 = 0; k2 < B; ++k2) w = (k2 > t && snd[k2] == snd[t]) ? k2 : w;
    // the reference computes (td + eps) ** alpha on a float32 tensor (vdn/_train.py:230-233)
    sval[L][t] = (double)powf(stv[w] + eps, alpha);
  }
  __syncthreads();
  for (int d = L - 1; d >= 0; --d) {
    if (t < B && snd[t] >= 0) {
      const int64_t c = ((snd[t] + 1) >> (L - d - 1)) - 1;   // the path's child at depth d + 1
      const int part = spart[d + 1][t];
      const double sv = part >= 0 ? sval[d + 1][part] : ssib[d + 1][t];
      const double cv = sval[d + 1][t];
      sval[d][t] = (c & 1) ? cv + sv : sv + cv;   // odd index = left child
    }
    __syncthreads();
  }
  // every changed node written once the paths are done; nodes shared by several paths get identical values
  for (int i = t; i < B * (L + 1); i += blockDim.x) {
    const int k = i / (L + 1), d = i % (L + 1);
    const int64_t nd = snd[k];
    if (nd >= 0) tree[((nd + 1) >> (L - d)) - 1] = sval[d][k];
  }
}

// Stratified PER sampling (one 1024-thread block; per_sample_kernel's, or one extra block of the learner's Adam
// launch sampling the NEXT update's batch): B draws, the sampled nodes / slots, IS weights, alpha / beta annealing
// and the VDN step-weight decay (vdn/replay_buffer/buffer.py:50-81, qmix/replay_buffer/per.py:36-59).
constexpr int PS_T = 1024;            // the block size
constexpr int PER_SAMPLE_MAXJ = 8;    // batch <= PS_T * 8
__device__ __forceinline__ void per_sample_body(double* tree, int64_t cap, int B, const double* fracs, uint64_t seed,
                                                uint64_t counter, PerDev* st, double decay, int64_t* nodes_out,
                                                int64_t* slots_out, float* is_w) {
  // anneal alpha / beta before the draws (buffer.py:53-56)
  const double alpha = fmin(1.0, st->alpha + st->alpha_inc);
  const double beta = fmin(1.0, st->beta + st->beta_inc);
  // device-side draw counter: every (graph-replayed) sample call gets a fresh RNG stream
  const uint64_t ctr = counter + st->n_samples;
  // the tree's top 11 levels (2047 nodes) staged in LDS in one round trip: a draw's descent then pays a
  // global round trip only below depth 10 (6 instead of 16 dependent loads at 65536 leaves); same nodes,
  // same comparisons
  __shared__ double top[2047];
  const int64_t n_nodes = 2 * cap - 1;
  const int64_t ntop = n_nodes < 2047 ? n_nodes : 2047;
  for (int64_t i = threadIdx.x; i < ntop; i += PS_T) top[i] = tree[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    st->alpha = alpha;
    st->beta = beta;
    st->n_samples += 1;
  }
  // each thread owns samples k = threadIdx.x + j * PS_T (B <= PS_T * PER_SAMPLE_MAXJ), leaf priorities and
  // IS weights kept in registers
  double pk[PER_SAMPLE_MAXJ], wk[PER_SAMPLE_MAXJ];
  const double total = top[0];
  const double seg = total / (double)B;
#pragma unroll
  for (int j = 0; j < PER_SAMPLE_MAXJ; ++j) {
    const int k = threadIdx.x + j * PS_T;
    pk[j] = 0.0;
    if (k >= B) continue;
    double f = fracs ? fracs[k] : (double)(rng_draw(seed, ctr, (uint64_t)k, 77) >> 11) * (1.0 / 9007199254740992.0);
    const double a = seg * (double)k;
    const double b = seg * (double)(k + 1);
    double s = a + (b - a) * f;
    int64_t idx = 0;
    while (true) {
      const int64_t left = 2 * idx + 1;
      if (left >= n_nodes) break;
      const double lv = left < ntop ? top[left] : tree[left];
      if (s <= lv) {
        idx = left;
      } else {
        s = s - lv;
        idx = left + 1;
      }
    }
    nodes_out[k] = idx;
    if (slots_out) slots_out[k] = idx - (cap - 1);
    pk[j] = tree[idx];
  }
  __syncthreads();
  // VDN: whole tree x step_weight after sampling (buffer.py:72-73)
  if (decay != 1.0) {
    for (int64_t i = threadIdx.x; i < n_nodes; i += PS_T) tree[i] = decay * tree[i];
    __syncthreads();
  }
  const double total2 = tree[0];
  double mx = 0.0;
#pragma unroll
  for (int j = 0; j < PER_SAMPLE_MAXJ; ++j) {
    const int k = threadIdx.x + j * PS_T;
    wk[j] = 0.0;
    if (k >= B) continue;
    wk[j] = pow((double)cap * (pk[j] / total2), -beta);
    mx = fmax(mx, wk[j]);
  }
  // block max (exact in any order)
  __shared__ double s_mx[PS_T / 64];
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  if ((threadIdx.x & 63) == 0) s_mx[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = s_mx[0];
  for (int w = 1; w < PS_T / 64; ++w) mx = fmax(mx, s_mx[w]);
#pragma unroll
  for (int j = 0; j < PER_SAMPLE_MAXJ; ++j) {
    const int k = threadIdx.x + j * PS_T;
    if (k < B) is_w[k] = (float)(wk[j] / mx);
  }
}

// the small update's arguments as one extra block of another launch (tree == nullptr: none)
struct PerUpd {
  double* tree;
  int64_t cap;
  const int64_t* nodes;
  const float* td;
  PerDev* st;
  int B;
  float eps;
};
__device__ __forceinline__ void per_update_small_block(const PerUpd& pu) {
  per_update_small_body(pu.tree, pu.cap, pu.nodes, pu.td, pu.B, pu.st, pu.eps);
}
// a sample's arguments as one extra block of another launch (tree == nullptr: none)
struct PerSmp {
  double* tree;
  int64_t cap;
  PerDev* st;
  uint64_t seed, counter;
  double decay;
  int64_t *nodes, *slots;
  float* isw;
  int B;
};
__device__ __forceinline__ void per_sample_block(const PerSmp& ps) {
  per_sample_body(ps.tree, ps.cap, ps.B, nullptr, ps.seed, ps.counter, ps.st, ps.decay, ps.nodes, ps.slots, ps.isw);
}

}  // namespace mm
