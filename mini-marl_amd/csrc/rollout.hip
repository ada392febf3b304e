// Rollout bookkeeping kernels: per-step TD error into the chunk priority and the
// transition store, plus the chunk-begin obs copy (gfx950).
//
// Replaces cal_td_error + the python chunk lists (vdn/_utils.py:44-52,
// vdn/main.py:140-167, qmix/main.py:183-233): per env e at rollout step t
//   td = |sum_i r_i + (1-d)*gamma*sum_i max_a Q'_i - sum_i Q_{i,a_i}|   (no xN here)
//   chunk_td[e] += td; store act/rew/done at slot t of the env's staging row.
// Chunks span episode boundaries exactly like the reference's global count_step.
// HBM-bound, one thread per env; sums over agents in registers.
#include "common.h"
#include "minimarl.h"
#include "rollout_fold.h"

namespace mm {

// One thread per (env, agent): coalesced loads/stores; per-env sums over agents through LDS.
__global__ __launch_bounds__(256) void td_chunk_kernel(int E, int N, float gamma, const float* __restrict__ rew,
                                                       const uint8_t* __restrict__ done,
                                                       const float* __restrict__ q_taken,
                                                       const float* __restrict__ maxq_next,
                                                       const int32_t* __restrict__ act, float* __restrict__ chunk_td,
                                                       int t, int C, uint8_t* __restrict__ s_act,
                                                       float* __restrict__ s_rew, uint8_t* __restrict__ s_done,
                                                       const int64_t* __restrict__ rows,
                                                       uint64_t* __restrict__ counter) {
  __shared__ float sh[3][256];
  const int epb = blockDim.x / N;                    // envs per block
  const int le = threadIdx.x / N, k = threadIdx.x % N;
  const int e = blockIdx.x * epb + le;
  if (counter && blockIdx.x == 0 && threadIdx.x == 0) *counter += 1;  // RNG stream of the next step
  const bool on = le < epb && e < E;
  float r = 0.f, q = 0.f, m = 0.f;
  if (on) {
    const int64_t o = (int64_t)e * N + k;
    const int64_t row = rows ? rows[e] : (int64_t)e;
    r = rew[o];
    q = q_taken[o];
    m = maxq_next[o];
    if (s_act) s_act[(row * C + t) * N + k] = (uint8_t)act[o];
    if (s_rew) s_rew[(row * C + t) * N + k] = r;
    if (k == 0 && s_done) s_done[row * C + t] = done[e];
  }
  sh[0][threadIdx.x] = r;
  sh[1][threadIdx.x] = q;
  sh[2][threadIdx.x] = m;
  __syncthreads();
  if (on && k == 0) {
    float sr = 0.f, sq = 0.f, st = 0.f;   // agent order, like the reference's sum over dim 1
    for (int j = 0; j < N; ++j) {
      sr += sh[0][threadIdx.x + j];
      sq += sh[1][threadIdx.x + j];
      st += sh[2][threadIdx.x + j];
    }
    const float d = done[e] ? 1.0f : 0.0f;
    const float td = rollout_td(sr, sq, st, d, gamma);
    chunk_td[e] = (t == 0 ? 0.0f : chunk_td[e]) + td;
  }
}

// The TD / store of n consecutive steps of a chunk (the chunk-persistent rollout's fold, mm_td_fold_range): one
// 16-env group per block (rollout_fold.h), E / 16 blocks
template <bool VEC>
__global__ __launch_bounds__(256) void td_fold_range_kernel(FoldArgs a) {
  td_fold_group<VEC>(a, blockIdx.x);
}

// Diagnostic (mm_hold_cus): one 1024-thread workgroup per CU (16 waves holding VGPRs + 64 KiB of dynamic LDS, so no
// chunk-kernel block, which needs every VGPR of the CU's SIMDs, can share the CU) that spins on the 100 MHz clock for `ticks`; *seen |= 2 if a watched hand-off word already carries `tag` when
// the block starts, |= 1 if one carries it when the block ends (1 alone: a chunk-persistent launch ran beside it).
// tests/test_gpu_chunk.py uses it to break the chunk kernel's co-residency contract on purpose (bounded: the waits
// expire, the grid drains).
__device__ __forceinline__ int hold_scan(const uint64_t* watch, int64_t n_watch, uint32_t tag) {
  int saw = 0;
  for (int64_t i = threadIdx.x; i < n_watch; i += blockDim.x)
    saw |= (uint32_t)(__hip_atomic_load(watch + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) == tag ? 1 : 0;
  return __syncthreads_or(saw) ? 1 : 0;
}
__global__ __launch_bounds__(1024) void hold_cus_kernel(int64_t ticks, const uint64_t* watch, int64_t n_watch,
                                                      uint32_t tag, int32_t* seen) {
  extern __shared__ float hold_lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  hold_lds[threadIdx.x] = 0.0f;
  const int pre = hold_scan(watch, n_watch, tag);
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)ticks) __builtin_amdgcn_s_sleep(64);
  const int post = hold_scan(watch, n_watch, tag);
  if (threadIdx.x == 0 && (pre || post)) atomicOr(seen, (pre ? 2 : 0) | (post ? 1 : 0));
}

// chunk begin: obs_cur [E][ND] -> store slot 0 of each env's staging row
__global__ __launch_bounds__(256) void chunk_begin_kernel(int E, int ND, const float* __restrict__ obs_cur,
                                                          float* __restrict__ s_obs, int64_t row_stride,
                                                          const int64_t* __restrict__ rows) {
  const int64_t total = (int64_t)E * ND;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i / ND, r = i % ND;
    const int64_t row = rows ? rows[e] : e;
    s_obs[row * row_stride + r] = obs_cur[i];
  }
}

// Chunk start from the store itself: slot 0 of row dst_rows[e] = slot src_off of row src_rows[e]
// (the previous step's next obs), or the env's reset obs where src_rows[e] < 0 (env just reset).
__global__ __launch_bounds__(256) void chunk_begin_rows_kernel(int E, int ND, float* __restrict__ s_obs,
                                                               int64_t row_stride,
                                                               const int64_t* __restrict__ src_rows, int64_t src_off,
                                                               const float* __restrict__ reset_obs,
                                                               const int64_t* __restrict__ dst_rows) {
  const int64_t total = (int64_t)E * ND;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i / ND, r = i % ND;
    const int64_t src = src_rows[e];
    const float v = src >= 0 ? s_obs[src * row_stride + src_off + r] : reset_obs[r];
    s_obs[dst_rows[e] * row_stride + r] = v;
  }
}

// Greedy evaluation episode accumulators (vdn/_test.py:22-50, qmix/_test.py:19-36,
// magym_runner.py:198-241): while env e is still in its episode, score[e] += sum_i r_i and, given
// Q(a) and max Q', loss[e] += td^2 with td as cal_td_error (vdn/_utils.py:44-52); done ends it.
__global__ __launch_bounds__(256) void eval_accum_kernel(int E, int N, float gamma, const float* __restrict__ rew,
                                                         const uint8_t* __restrict__ done,
                                                         const float* __restrict__ q_taken,
                                                         const float* __restrict__ maxq_next,
                                                         uint8_t* __restrict__ active, float* __restrict__ score,
                                                         float* __restrict__ loss) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E || !active[e]) return;
  float sr = 0.f, sq = 0.f, st = 0.f;
  for (int j = 0; j < N; ++j) {
    sr += rew[(int64_t)e * N + j];
    if (q_taken) sq += q_taken[(int64_t)e * N + j];
    if (maxq_next) st += maxq_next[(int64_t)e * N + j];
  }
  score[e] += sr;
  const bool dn = done[e] != 0;
  if (q_taken && maxq_next && loss) {
    const float td = rollout_td(sr, sq, st, dn ? 1.0f : 0.0f, gamma);
    loss[e] += td * td;
  }
  if (dn) active[e] = 0;
}

// Training score of the rollout (vdn/main.py:173 train_score += sum(reward); qmix/main.py:247): one
// thread per env walks the C steps of the chunk it just stored (row rows[e]), adds the agents' rewards
// to the env's running episode return and, at each episode end, moves the return into acc[0] (sum of
// finished episodes' returns) and acc[1] (their count). f64 accumulators, atomics per finished episode.
__global__ __launch_bounds__(256) void chunk_score_kernel(int E, int C, int N, const float* __restrict__ store_rew,
                                                          const uint8_t* __restrict__ store_done,
                                                          const int64_t* __restrict__ rows,
                                                          float* __restrict__ ep_ret, double* __restrict__ acc) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int64_t r = rows[e];
  float ret = ep_ret[e];
  double fin = 0.0, cnt = 0.0;
  for (int c = 0; c < C; ++c) {
    const float* rw = store_rew + (r * C + c) * N;
    float sr = 0.f;
    for (int j = 0; j < N; ++j) sr += rw[j];
    ret += sr;
    if (store_done[r * C + c]) {
      fin += (double)ret;
      cnt += 1.0;
      ret = 0.f;
    }
  }
  ep_ret[e] = ret;
  if (cnt > 0.0) {
    atomicAdd(&acc[0], fin);
    atomicAdd(&acc[1], cnt);
  }
}

// VDN mixing of one step (vdn/_train.py:23-47: q.gather(2, action).squeeze().sum(1); the target side
// max(2)[0].sum(1), vdn/_train.py:68-71): out[b] = sum_i q[b, i, act[b, i]] (or max_a q[b, i, a] when act
// is NULL), agents summed in id order. One thread per row; q rows at b * q_se + i * q_sa.
__global__ __launch_bounds__(256) void vdn_sum_kernel(int64_t B, int N, int A, const float* __restrict__ q, int64_t q_se,
                                                      int64_t q_sa, const int32_t* __restrict__ act,
                                                      float* __restrict__ out, int32_t* __restrict__ err) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  float acc = 0.f;
  for (int i = 0; i < N; ++i) {
    const float* qr = q + b * q_se + (int64_t)i * q_sa;
    float v;
    if (act) {
      const int a = act[b * N + i];
      const bool ok = a >= 0 && a < A;
      if (!ok && err) atomicOr(err, 1);
      v = ok ? qr[a] : 0.f;
    } else {
      v = qr[0];
      for (int a = 1; a < A; ++a) v = fmaxf(v, qr[a]);
    }
    acc += v;
  }
  out[b] = acc;
}

}  // namespace mm

extern "C" {
int mm_chunk_score(int64_t n_envs, int32_t chunk, int32_t n_agents, const float* store_rew,
                   const uint8_t* store_done, const int64_t* rows, float* ep_ret, double* acc, mm_stream_t s) {
  MM_REQUIRE(store_rew && store_done && rows && ep_ret && acc && chunk >= 1 && n_agents >= 1,
             "chunk_score: bad args");
  if (n_envs <= 0) return MM_OK;
  hipLaunchKernelGGL(mm::chunk_score_kernel, dim3((int)((n_envs + 255) / 256)), dim3(256), 0, (hipStream_t)s,
                     (int)n_envs, chunk, n_agents, store_rew, store_done, rows, ep_ret, acc);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_eval_accum(int64_t n_envs, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                  const float* q_taken, const float* max_q_next, uint8_t* active, float* score, float* loss,
                  mm_stream_t s) {
  MM_REQUIRE(rew && done && active && score && n_agents >= 1, "eval_accum: bad args");
  if (n_envs <= 0) return MM_OK;
  hipLaunchKernelGGL(mm::eval_accum_kernel, dim3((int)((n_envs + 255) / 256)), dim3(256), 0, (hipStream_t)s,
                     (int)n_envs, n_agents, gamma, rew, done, q_taken, max_q_next, active, score, loss);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_chunk_begin_rows(int64_t n_envs, int32_t nd, float* store_obs, int64_t row_stride, const int64_t* src_rows,
                        int64_t src_off, const float* reset_obs, const int64_t* dst_rows, mm_stream_t s) {
  MM_REQUIRE(store_obs && src_rows && reset_obs && dst_rows, "chunk_begin_rows: null argument");
  if (n_envs <= 0) return MM_OK;
  const int threads = 256;
  const int64_t total = n_envs * nd;
  const int blocks = (int)std::min<int64_t>((total + threads - 1) / threads, 8192);
  hipLaunchKernelGGL(mm::chunk_begin_rows_kernel, dim3(blocks), dim3(threads), 0, (hipStream_t)s, (int)n_envs, nd,
                     store_obs, row_stride, src_rows, src_off, reset_obs, dst_rows);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_td_fold_range(int64_t n_envs, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                     const float* q_taken, const float* max_q_next, const int32_t* act, int64_t ring_se,
                     int32_t slot0, int32_t n_slots, int32_t chunk_len, float* chunk_td, uint8_t* store_act,
                     float* store_rew, uint8_t* store_done, const int64_t* rows, int64_t n_rows, int32_t* err,
                     mm_stream_t s) {
  MM_REQUIRE(rew && done && q_taken && max_q_next && act && chunk_td && store_act && store_rew && store_done && rows,
             "td_fold_range: null argument");
  MM_REQUIRE(n_slots >= 1 && slot0 >= 0 && slot0 + n_slots <= chunk_len,
             "td_fold_range: slots [slot0, slot0 + n) must lie in one chunk");
  MM_REQUIRE(n_agents >= 1 && n_agents <= 256 && ring_se >= n_envs * n_agents, "td_fold_range: bad agents / ring");
  if (n_envs <= 0) return MM_OK;
  mm::FoldArgs a{rew, done, q_taken, max_q_next, act, chunk_td, store_act, store_rew, store_done, rows,
                 reinterpret_cast<uint32_t*>(err), ring_se, n_rows, (int)n_envs, n_agents, slot0, n_slots, chunk_len,
                 gamma};
  const int blocks = (int)((n_envs + 15) / 16);
  auto kern = mm::fold_vec_ok(a) ? mm::td_fold_range_kernel<true> : mm::td_fold_range_kernel<false>;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(16 * std::min(n_slots, 16)), 0, (hipStream_t)s, a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_td_chunk_step_rows(int64_t n_envs, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                          const float* q_taken, const float* max_q_next, const int32_t* act, float* chunk_td,
                          int32_t step_in_chunk, int32_t chunk_len, uint8_t* store_act, float* store_rew,
                          uint8_t* store_done, const int64_t* rows, uint64_t* counter, mm_stream_t s) {
  MM_REQUIRE(rew && done && q_taken && max_q_next && (act || !store_act) && chunk_td, "td_chunk_step: null argument");
  MM_REQUIRE(step_in_chunk >= 0 && step_in_chunk < chunk_len, "td_chunk_step: bad step");
  if (n_envs <= 0) return MM_OK;
  MM_REQUIRE(n_agents >= 1 && n_agents <= 256, "td_chunk_step: n_agents must be in [1,256]");
  const int epb = 256 / n_agents;
  const int threads = epb * n_agents;
  const int blocks = (int)((n_envs + epb - 1) / epb);
  hipLaunchKernelGGL(mm::td_chunk_kernel, dim3(blocks), dim3(threads), 0, (hipStream_t)s, (int)n_envs, n_agents,
                     gamma, rew, done, q_taken, max_q_next, act, chunk_td, step_in_chunk, chunk_len, store_act,
                     store_rew, store_done, rows, counter);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_td_chunk_step(int64_t n_envs, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                     const float* q_taken, const float* max_q_next, const int32_t* act, float* chunk_td,
                     int32_t step_in_chunk, int32_t chunk_len, uint8_t* store_act, float* store_rew,
                     uint8_t* store_done, int64_t store_row0, mm_stream_t s) {
  (void)store_row0;
  return mm_td_chunk_step_rows(n_envs, n_agents, gamma, rew, done, q_taken, max_q_next, act, chunk_td,
                               step_in_chunk, chunk_len, store_act, store_rew, store_done, nullptr, nullptr, s);
}

int mm_chunk_begin(int64_t n_envs, int32_t nd, const float* obs_cur, float* store_obs, int64_t row_stride,
                   const int64_t* rows, mm_stream_t s) {
  MM_REQUIRE(obs_cur && store_obs, "chunk_begin: null argument");
  if (n_envs <= 0) return MM_OK;
  const int threads = 256;
  const int64_t total = n_envs * nd;
  const int blocks = (int)std::min<int64_t>((total + threads - 1) / threads, 8192);
  hipLaunchKernelGGL(mm::chunk_begin_kernel, dim3(blocks), dim3(threads), 0, (hipStream_t)s, (int)n_envs, nd,
                     obs_cur, store_obs, row_stride, rows);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_vdn_sum(int64_t B, int32_t N, int32_t A, const float* q, int64_t q_se, int64_t q_sa, const int32_t* act,
               float* out, int32_t* err, mm_stream_t s) {
  MM_REQUIRE(q && out && N >= 1 && A >= 1 && B >= 0, "vdn_sum: bad args");
  if (B == 0) return MM_OK;
  hipLaunchKernelGGL(mm::vdn_sum_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)s, B, N, A, q,
                     q_se, q_sa, act, out, err);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_hold_cus(int32_t n_blocks, int64_t ticks, const int64_t* watch, int64_t n_watch, uint32_t tag, int32_t* seen,
                mm_stream_t s) {
  MM_REQUIRE(n_blocks >= 1 && n_blocks <= 4096 && ticks >= 0 && ticks <= 200000000ll && seen && (watch || !n_watch),
             "hold_cus: bad args (at most 2 s)");
  hipLaunchKernelGGL(mm::hold_cus_kernel, dim3(n_blocks), dim3(1024), 64 * 1024, (hipStream_t)s, ticks,
                     reinterpret_cast<const uint64_t*>(watch), n_watch, tag, seen);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}
}
