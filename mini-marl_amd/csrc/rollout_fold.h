// The TD / chunk-store fold of n consecutive rollout steps of a chunk (cal_td_error + the chunk lists,
// vdn/_utils.py:44-52, vdn/main.py:140-167, qmix/main.py:183-233), shared by td_fold_range_kernel (rollout.hip) and
// the PER insert's first pass (per.hip, per_mb_sel1_fold: the fold's blocks beside the histogram's in one grid).
// Thread (slot j, env) of a 16-env group computes td_chunk_kernel's per-step value (agent-order sums, rollout_td's
// fixed rounding) and stores the step's act / rew / done into its store row; then one thread per env accumulates the
// chunk priority over the slots in order (the same float additions as n consecutive td_chunk_kernel launches).
// VEC (N % 4 == 0, 16-byte aligned rings / store rows): float4 / int4 loads and float4 / packed-byte row stores.
#pragma once
#include "common.h"

namespace mm {

struct FoldArgs {
  const float* rew;        // [n][E][N] (ring_se apart per step)
  const uint8_t* done;     // [n][E]
  const float* q_taken;
  const float* maxq_next;
  const int32_t* act;
  float* chunk_td;         // [E]
  uint8_t* s_act;          // store [rows][C][N]
  float* s_rew;
  uint8_t* s_done;         // store [rows][C]
  const int64_t* rows;     // [E] staging rows
  uint32_t* err;           // sticky bit 0: a staging row outside the store; bit 1 set (a chunk-persistent launch whose
                           // hand-off wait expired): nothing is folded — its steps' data never reach the chunk store
  int64_t ring_se, n_rows;
  int E, N, slot0, n, C;
  float gamma;
  // the PER insert's fold (per_mb_sel1_fold) only: the chunk priorities (td + eps)^alpha of the finished chunks,
  // computed here beside the histogram instead of on the insert's critical path (per_mb_apply reads them)
  double* prio = nullptr;        // [E]
  const double* alpha = nullptr; // the PER's device alpha (PerDev::alpha)
  double eps = 0.0;
};

// one 16-env group (block-local index blk) of the fold; blockDim.x >= 16 min(n, 16). Spans longer than 16 slots
// (chunk lengths > 16) run in slot groups of 16: each group's per-step values go through tdv, then the env's thread
// adds them to its running priority in slot order, so the float additions are those of n td_chunk_kernel launches.
template <bool VEC>
__device__ __forceinline__ void td_fold_group(const FoldArgs& a, int blk) {
  __shared__ float tdv[16][16];
  if (a.err && (*reinterpret_cast<const volatile uint32_t*>(a.err) & 2u)) return;   // (block-uniform)
  const int jl = threadIdx.x >> 4, le = threadIdx.x & 15;
  const int e = blk * 16 + le;
  const int N = a.N;
  float ctd = 0.0f;
  if (jl == 0 && e < a.E && a.slot0 != 0) ctd = a.chunk_td[e];
  for (int j0 = 0; j0 < a.n; j0 += 16) {
    const int j = j0 + jl;
    const bool on = e < a.E && jl < 16 && j < a.n;
    if (on) {
      const int t = a.slot0 + j;
      const int64_t o = (int64_t)j * a.ring_se + (int64_t)e * N;
      const int64_t row = a.rows[e];
      const uint8_t d8 = a.done[(int64_t)j * a.E + e];
      const bool rok = row >= 0 && row < a.n_rows;
      const int64_t so = (row * a.C + t) * N;
      float sr = 0.f, sq = 0.f, st = 0.f;   // agent order, like the reference's sum over dim 1
      if constexpr (VEC) {
        for (int k = 0; k < N; k += 4) {
          const float4 r4 = *reinterpret_cast<const float4*>(a.rew + o + k);
          const float4 q4 = *reinterpret_cast<const float4*>(a.q_taken + o + k);
          const float4 m4 = *reinterpret_cast<const float4*>(a.maxq_next + o + k);
          const int4 a4 = *reinterpret_cast<const int4*>(a.act + o + k);
          sr += r4.x; sr += r4.y; sr += r4.z; sr += r4.w;
          sq += q4.x; sq += q4.y; sq += q4.z; sq += q4.w;
          st += m4.x; st += m4.y; st += m4.z; st += m4.w;
          if (rok) {
            *reinterpret_cast<float4*>(a.s_rew + so + k) = r4;
            *reinterpret_cast<uint32_t*>(a.s_act + so + k) = (uint32_t)(a4.x & 255) | ((uint32_t)(a4.y & 255) << 8) |
                                                              ((uint32_t)(a4.z & 255) << 16) | ((uint32_t)a4.w << 24);
          }
        }
      } else {
        for (int k = 0; k < N; ++k) {
          const float r = a.rew[o + k];
          sr += r;
          sq += a.q_taken[o + k];
          st += a.maxq_next[o + k];
          if (rok) {
            a.s_act[so + k] = (uint8_t)a.act[o + k];
            a.s_rew[so + k] = r;
          }
        }
      }
      const float d = d8 ? 1.0f : 0.0f;
      tdv[jl][le] = rollout_td(sr, sq, st, d, a.gamma);
      if (rok) {
        a.s_done[row * a.C + t] = d8;
      } else if (a.err) {
        atomicOr(a.err, 1u);
      }
    }
    __syncthreads();
    if (jl == 0 && e < a.E) {
      const int m = a.n - j0 < 16 ? a.n - j0 : 16;
      for (int jj = 0; jj < m; ++jj) ctd = (a.slot0 + j0 + jj == 0 ? 0.0f : ctd) + tdv[jj][le];
    }
    __syncthreads();
  }
  if (jl == 0 && e < a.E) {
    a.chunk_td[e] = ctd;
    if (a.prio) a.prio[e] = pow((double)ctd + a.eps, *a.alpha);   // = per_mb_apply's pow of chunk_td[e]
  }
}

// VEC applies: N % 4 == 0 and every ring / store base 16-byte aligned (4-byte for the act bytes)
inline bool fold_vec_ok(const FoldArgs& a) {
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return a.N % 4 == 0 && a.ring_se % 4 == 0 && a16(a.rew) && a16(a.q_taken) && a16(a.maxq_next) && a16(a.act) &&
         a16(a.s_rew) && ((uintptr_t)a.s_act & 3) == 0;
}

}  // namespace mm
