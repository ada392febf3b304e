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

}  // namespace mm
