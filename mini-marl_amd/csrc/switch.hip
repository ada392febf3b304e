// The ma_gym Switch corridor env (QMIX's default "ma_gym:Switch2-v0", qmix/_config.py:14-19,
// qmix/main.py:66-71), E envs in lockstep. Dynamics spec: oracle/switch.py (ma-gym is absent, so
// parity with it is unpinned). The whole state of an env is 4 agent cells, 4 done bits and a step
// count (16 bytes); the step kernel runs one lane per (env, agent) and forms each env's termination
// from a wave ballot of its agents' done bits. The same kernel serves the plain step, the rollout
// engine's chunk-store row step and the row step fused with the previous step's TD / store.
#include <math.h>

#include <vector>

#include "common.h"
#include "minimarl.h"

namespace mm {

struct SwitchState {
  int8_t pos[4][2];
  uint8_t adone[4];
  int32_t steps;
};

// obs feature tables round(c / 6, 2), round(r / 2, 2) (Python floats -> float32), passed by value in
// the kernel arguments (no per-device constant-memory state to initialise)
struct SwitchTab {
  float col[7];
  float row[3];
};

static SwitchTab switch_tables() {
  SwitchTab t;
  for (int c = 0; c < 7; ++c) t.col[c] = (float)(std::round(c / 6.0 * 100.0) / 100.0);
  for (int r = 0; r < 3; ++r) t.row[r] = (float)(r / 2.0);
  return t;
}

// open cells of the 3 x 7 grid: the middle row and columns 0, 1, 5, 6
__device__ __forceinline__ bool sw_open(int r, int c) {
  return r >= 0 && r < 3 && c >= 0 && c < 7 && (r == 1 || c <= 1 || c >= 5);
}

__device__ __forceinline__ void sw_init(SwitchState& s, int N) {
  const int8_t ir[4] = {0, 0, 2, 2}, ic[4] = {1, 5, 1, 5};
  for (int k = 0; k < 4; ++k) {
    s.pos[k][0] = k < N ? ir[k] : -1;
    s.pos[k][1] = k < N ? ic[k] : -1;
    s.adone[k] = 0;
  }
  s.steps = 0;
}

__device__ __forceinline__ void sw_obs(const SwitchTab& tab, const SwitchState& s, int N, int max_steps, int full,
                                       int clock, float* __restrict__ out) {
  const int ld = 2 + clock;
  const int D = full ? ld * N : ld;
  const float clk = (float)((double)s.steps / (double)max_steps);
  for (int k = 0; k < N; ++k) {
    float loc[3] = {tab.row[s.pos[k][0]], tab.col[s.pos[k][1]], clk};
    if (full) {
      for (int j = 0; j < N; ++j)
        for (int f = 0; f < ld; ++f) out[j * D + k * ld + f] = loc[f];
    } else {
      for (int f = 0; f < ld; ++f) out[k * D + f] = loc[f];
    }
  }
}

__global__ __launch_bounds__(256) void switch_reset_kernel(SwitchTab tab, SwitchState* __restrict__ st, int64_t E, int N,
                                                           int max_steps, int full, int clock, float* __restrict__ obs,
                                                           float* __restrict__ reset_table) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  SwitchState s;
  sw_init(s, N);
  st[e] = s;
  const int D = (2 + clock) * (full ? N : 1);
  if (obs) sw_obs(tab, s, N, max_steps, full, clock, obs + e * N * D);
  if (reset_table && e == 0) sw_obs(tab, s, N, max_steps, full, clock, reset_table);
}

// One lockstep step. Lane = (env, agent): NP = 2 or 4 lanes per env (N <= NP; N = 3 leaves one lane
// idle), 256 / NP envs per block. Phase 0 issues every global read of the step (state, actions, the
// fused TD inputs of the previous step). The agent-ordered moves (a move sees the positions updated so
// far this step) cost N <= 4 iterations, so every lane of an env runs them on its own register copy of
// the 16-byte state (the env's actions come in by lane shuffles) and keeps only its own agent's
// reward and done bit. The env's termination — all(done), the reference's `while not all(done)` /
// `done = int(all(done))` (qmix/main.py:109,199,215) — is a wave ballot of the agent-done bits: the
// NP-bit group of the env's lanes must be full. Lane k then writes agent k's obs floats (partial: its
// D-float run; full observable: its local part into every agent's row), reward and done bit; lane 0
// of the env writes the env's done, cur_row and the state (the initial state where the env finished
// and auto-reset is on). With next_row the next obs of env e goes to next_obs + next_row[e] * next_se
// (the engine's chunk-store staging row); cur_row[e] = that row, or -1 where the env reset (the
// current obs is then the reset table).
template <int NP>
__global__ __launch_bounds__(256) void switch_step_kernel(SwitchTab tab, SwitchState* __restrict__ st, int64_t E, int N,
                                                          int max_steps, int full, int clock, float step_cost,
                                                          const int32_t* __restrict__ act, float* __restrict__ next_obs,
                                                          int64_t next_se, const int64_t* __restrict__ next_row,
                                                          float* __restrict__ obs_cur, int64_t* __restrict__ cur_row,
                                                          float* rew, uint8_t* __restrict__ agent_done,
                                                          uint8_t* __restrict__ done_out, TdFuse tdf, BeginCopy bc) {
  const int64_t gl = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t e = gl / NP;
  const int k = (int)(gl % NP);
  const int lane = threadIdx.x & 63;
  const int base = lane & ~(NP - 1);   // first lane of this env in the wave
  const bool env_ok = e < E;
  const bool ag = env_ok && k < N;
  // ---- phase 0: all global reads
  SwitchState s;
  if (env_ok) {
    s = st[e];
  } else {
    sw_init(s, N);
  }
  const int a_own = ag ? act[e * N + k] : 4;
  float trew = 0.f, tq = 0.f, tm = 0.f;
  int32_t tact = 0;
  int64_t trow = 0;
  uint8_t tdone = 0;
  if (tdf.on && env_ok) {
    trow = tdf.rows[e];
    tdone = tdf.done[e];
    if (ag) {
      trew = tdf.rew[e * N + k];
      tq = tdf.q_taken[e * N + k];
      tm = tdf.maxq[e * N + k];
      tact = tdf.act[e * N + k];
    }
  }
  const int64_t srow = env_ok ? (next_row ? next_row[e] : e) : 0;
  const int64_t bsrc = (bc.on && env_ok) ? cur_row[e] : -1;   // read before lane 0 overwrites it below
  int a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = __shfl(a_own, base + (j < NP ? j : 0));

  // ---- fused TD / store of the previous step (td_chunk_kernel's arithmetic: agent-order sums)
  if (tdf.on) {
    if (ag) {
      tdf.s_act[(trow * tdf.C + tdf.slot) * N + k] = (uint8_t)tact;
      tdf.s_rew[(trow * tdf.C + tdf.slot) * N + k] = trew;
    }
    float sr = 0.f, sq = 0.f, sm = 0.f;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const float r_j = __shfl(trew, base + j), q_j = __shfl(tq, base + j), m_j = __shfl(tm, base + j);
      if (j < N) {
        sr += r_j;
        sq += q_j;
        sm += m_j;
      }
    }
    if (env_ok && k == 0) {
      const float dn = tdone ? 1.0f : 0.0f;
      const float td = rollout_td(sr, sq, sm, dn, tdf.gamma);
      tdf.chunk_td[e] = (tdf.slot == 0 ? 0.0f : tdf.chunk_td[e]) + td;
      tdf.s_done[trow * tdf.C + tdf.slot] = tdone;
    }
    if (tdf.counter && gl == 0) *tdf.counter += 1;
  }

  // ---- dynamics (oracle/switch.py SwitchOracle.step): agents in id order on the lane's state copy
  s.steps += 1;
  bool reached = false;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    if (j >= N || s.adone[j]) continue;
    const int aj = a[j];
    if (aj >= 0 && aj < 4) {   // 0 down, 1 left, 2 up, 3 right
      const int r = s.pos[j][0] + (aj == 0) - (aj == 2), c = s.pos[j][1] + (aj == 3) - (aj == 1);
      bool ok = sw_open(r, c);
#pragma unroll
      for (int i = 0; i < NP; ++i) ok = ok && (i >= N || i == j || s.pos[i][0] != r || s.pos[i][1] != c);
      if (ok) {
        s.pos[j][0] = (int8_t)r;
        s.pos[j][1] = (int8_t)c;
      }
    }
    if (s.pos[j][0] == (j < 2 ? 0 : 2) && s.pos[j][1] == ((j & 1) ? 0 : 6)) {   // targets (0,6) (0,0) (2,6) (2,0)
      s.adone[j] = 1;
      if (j == k) reached = true;
    }
  }
  const bool timeout = s.steps >= max_steps;
  // this lane's agent (register selects, no dynamically indexed state array)
  int my_r = 0, my_c = 0;
  bool my_ad = false;
#pragma unroll
  for (int j = 0; j < NP; ++j)
    if (j == k) {
      my_r = s.pos[j][0];
      my_c = s.pos[j][1];
      my_ad = s.adone[j] != 0;
    }
  const bool my_done = ag && (timeout || my_ad);
  // termination mask: one ballot per wave, each env's NP-bit group must hold all N agents
  const uint64_t dm = __ballot(my_done);
  const uint64_t full_grp = (1ull << N) - 1;
  const bool all = env_ok && ((dm >> base) & full_grp) == full_grp;
  if (timeout) {
#pragma unroll
    for (int j = 0; j < 4; ++j) s.adone[j] = j < N ? 1 : 0;
  }

  // ---- outputs
  const int ld = 2 + clock;
  const int D = full ? ld * N : ld;
  if (bc.on && ag) {   // chunk start (mm_chunk_begin_rows folded in): this agent's D floats of slot 0
    const float* sp = bsrc >= 0 ? bc.store + bsrc * bc.row_stride + bc.src_off : bc.reset_obs;
    float* dp = bc.store + srow * bc.row_stride;
    for (int f = 0; f < D; ++f) dp[k * D + f] = sp[k * D + f];
  }
  if (ag) {
    rew[e * N + k] = reached ? 5.0f : step_cost;
    if (agent_done) agent_done[e * N + k] = my_done ? 1 : 0;
    const float clk = (float)((double)s.steps / (double)max_steps);
    const float loc[3] = {tab.row[my_r], tab.col[my_c], clk};
    if (next_obs) {
      float* o = next_obs + srow * next_se;
      if (full) {
        for (int j = 0; j < N; ++j)
          for (int f = 0; f < ld; ++f) o[j * D + k * ld + f] = loc[f];
      } else {
        for (int f = 0; f < ld; ++f) o[k * D + f] = loc[f];
      }
    }
  }
  const bool autoreset = obs_cur || cur_row;
  if (env_ok && k == 0) {
    done_out[e] = all ? 1 : 0;
    if (cur_row) cur_row[e] = all ? -1 : srow;
    if (autoreset && all) sw_init(s, N);
    st[e] = s;
  }
  if (obs_cur && ag) {          // the next current obs: the reset obs where the env finished
    // a finished env restarts at the agents' initial cells, step 0: (0,1) (0,5) (2,1) (2,5)
    const int r0 = all ? (k < 2 ? 0 : 2) : my_r, c0 = all ? ((k & 1) ? 5 : 1) : my_c;
    const float clk = all ? 0.0f : (float)((double)s.steps / (double)max_steps);
    const float loc[3] = {tab.row[r0], tab.col[c0], clk};
    float* o = obs_cur + e * N * D;
    if (full) {
      for (int j = 0; j < N; ++j)
        for (int f = 0; f < ld; ++f) o[j * D + k * ld + f] = loc[f];
    } else {
      for (int f = 0; f < ld; ++f) o[k * D + f] = loc[f];
    }
  }
}

}  // namespace mm

struct mm_switch {
  mm_switch_cfg cfg;
  mm::SwitchTab tab;
  int64_t E;
  mm::SwitchState* st;
  float* reset_obs;   // [N, D] the (deterministic) reset obs
};

namespace mm {
static int switch_step(mm_switch* w, const int32_t* act, float* next_obs, int64_t next_se, const int64_t* next_row,
                       float* obs_cur, int64_t* cur_row, float* rew, uint8_t* agent_done, uint8_t* done,
                       const TdFuse* tdf, hipStream_t s, const BeginCopy* bcp = nullptr) {
  MM_REQUIRE(w && act && rew && done, "switch_step: bad arguments");
  MM_REQUIRE(next_obs || obs_cur, "switch_step: no obs output");
  const mm_switch_cfg& c = w->cfg;
  const int D = (2 + c.clock) * (c.full_observable ? c.n_agents : 1);
  TdFuse t{};
  if (tdf) t = *tdf;
  BeginCopy bc{};
  if (bcp) bc = *bcp;
  MM_REQUIRE(!bc.on || (cur_row && next_row), "switch_step: the chunk-begin copy needs cur_row and the staging rows");
  const int64_t se = next_se > 0 ? next_se : (int64_t)c.n_agents * D;
  if (c.n_agents == 2) {
    hipLaunchKernelGGL(switch_step_kernel<2>, dim3((w->E * 2 + 255) / 256), dim3(256), 0, s, w->tab, w->st, w->E,
                       c.n_agents, c.max_steps, c.full_observable, c.clock, c.step_cost, act, next_obs, se, next_row,
                       obs_cur, cur_row, rew, agent_done, done, t, bc);
  } else {
    hipLaunchKernelGGL(switch_step_kernel<4>, dim3((w->E * 4 + 255) / 256), dim3(256), 0, s, w->tab, w->st, w->E,
                       c.n_agents, c.max_steps, c.full_observable, c.clock, c.step_cost, act, next_obs, se, next_row,
                       obs_cur, cur_row, rew, agent_done, done, t, bc);
  }
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}
}  // namespace mm

extern "C" {

int mm_switch_create(const mm_switch_cfg* cfg, int64_t n_envs, mm_switch** out) {
  MM_REQUIRE(cfg && out && n_envs >= 1 && n_envs < (1ll << 40), "switch_create: bad arguments");
  MM_REQUIRE(cfg->n_agents >= 2 && cfg->n_agents <= 4, "switch_create: n_agents must be 2..4 (got %d)", cfg->n_agents);
  MM_REQUIRE(cfg->max_steps >= 1, "switch_create: max_steps must be >= 1");
  mm_switch* w = new mm_switch;
  w->cfg = *cfg;
  w->cfg.full_observable = cfg->full_observable ? 1 : 0;
  w->cfg.clock = cfg->clock ? 1 : 0;
  w->tab = mm::switch_tables();
  w->E = n_envs;
  const int nd = w->cfg.n_agents * (2 + w->cfg.clock) * (w->cfg.full_observable ? w->cfg.n_agents : 1);
  const size_t st_bytes = (sizeof(mm::SwitchState) * n_envs + 255) & ~size_t(255);
  void* base = nullptr;
  if (hipMalloc(&base, st_bytes + nd * sizeof(float)) != hipSuccess) {
    delete w;
    mm::set_error("switch_create: hipMalloc failed");
    return MM_ENOMEM;
  }
  w->st = static_cast<mm::SwitchState*>(base);
  w->reset_obs = reinterpret_cast<float*>(static_cast<char*>(base) + st_bytes);
  const mm_switch_cfg& c = w->cfg;
  hipLaunchKernelGGL(mm::switch_reset_kernel, dim3((n_envs + 255) / 256), dim3(256), 0, 0, w->tab, w->st, n_envs,
                     c.n_agents, c.max_steps, c.full_observable, c.clock, (float*)nullptr, w->reset_obs);
  if (hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(base);
    delete w;
    mm::set_error("switch_create: init failed");
    return MM_EHIP;
  }
  *out = w;
  return MM_OK;
}

void mm_switch_destroy(mm_switch* w) {
  if (!w) return;
  (void)hipFree(w->st);
  delete w;
}

int mm_switch_obs_dim(const mm_switch* w) {
  return w ? (2 + w->cfg.clock) * (w->cfg.full_observable ? w->cfg.n_agents : 1) : -1;
}

const float* mm_switch_reset_obs(const mm_switch* w) { return w ? w->reset_obs : nullptr; }

int mm_switch_reset(mm_switch* w, float* obs, mm_stream_t s) {
  MM_REQUIRE(w, "switch_reset: NULL handle");
  const mm_switch_cfg& c = w->cfg;
  hipLaunchKernelGGL(mm::switch_reset_kernel, dim3((w->E + 255) / 256), dim3(256), 0, (hipStream_t)s, w->tab, w->st,
                     w->E, c.n_agents, c.max_steps, c.full_observable, c.clock, obs, (float*)nullptr);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_switch_step(mm_switch* w, const int32_t* act, float* next_obs, float* obs_cur, float* rew,
                   uint8_t* agent_done, uint8_t* done, mm_stream_t s) {
  return mm::switch_step(w, act, next_obs, 0, nullptr, obs_cur, nullptr, rew, agent_done, done, nullptr,
                         (hipStream_t)s);
}

int mm_switch_step_rows(mm_switch* w, const int32_t* act, float* next_obs, int64_t next_se, const int64_t* next_row,
                        float* obs_cur, int64_t* cur_row, float* rew, uint8_t* done, mm_stream_t s) {
  return mm::switch_step(w, act, next_obs, next_se, next_row, obs_cur, cur_row, rew, nullptr, done, nullptr,
                         (hipStream_t)s);
}

int mm_switch_step_rows_begin(mm_switch* w, const int32_t* act, float* store_obs, int64_t row_stride,
                              int32_t chunk_len, const int64_t* staging, int64_t* cur_row, float* rew, uint8_t* done,
                              mm_stream_t s) {
  MM_REQUIRE(w && store_obs && staging && cur_row && chunk_len >= 1, "switch_step_rows_begin: bad arguments");
  const int64_t nd = (int64_t)w->cfg.n_agents * mm_switch_obs_dim(w);
  MM_REQUIRE(row_stride >= (chunk_len + 1) * nd, "switch_step_rows_begin: row_stride < (chunk_len + 1) * N * D");
  const mm::BeginCopy bc{store_obs, row_stride, chunk_len * nd, w->reset_obs, 1};
  return mm::switch_step(w, act, store_obs + nd, row_stride, staging, nullptr, cur_row, rew, nullptr, done, nullptr,
                         (hipStream_t)s, &bc);
}

int mm_switch_step_rows_td(mm_switch* w, const int32_t* act, float* next_obs, int64_t next_se,
                           const int64_t* next_row, int64_t* cur_row, float* rew, uint8_t* done, float gamma,
                           const float* td_rew, const uint8_t* td_done, const float* q_taken, const float* max_q_next,
                           const int32_t* td_act, float* chunk_td, int32_t step_in_chunk, int32_t chunk_len,
                           uint8_t* store_act, float* store_rew, uint8_t* store_done, const int64_t* td_rows,
                           uint64_t* counter, mm_stream_t s) {
  MM_REQUIRE(td_rew && td_done && q_taken && max_q_next && td_act && chunk_td && store_act && store_rew &&
                 store_done && td_rows, "switch_step_rows_td: null TD argument");
  MM_REQUIRE(step_in_chunk >= 0 && step_in_chunk < chunk_len, "switch_step_rows_td: bad step");
  mm::TdFuse t{td_rew, td_done, q_taken, max_q_next, td_act, chunk_td, store_act, store_rew, store_done, td_rows,
               counter, gamma, step_in_chunk, chunk_len, 1};
  return mm::switch_step(w, act, next_obs, next_se, next_row, nullptr, cur_row, rew, nullptr, done, &t,
                         (hipStream_t)s);
}

int mm_switch_get_state(mm_switch* w, int32_t* pos, uint8_t* agent_done, int32_t* steps) {
  MM_REQUIRE(w && pos && agent_done && steps, "switch_get_state: bad arguments");
  std::vector<mm::SwitchState> h(w->E);
  MM_HIP_CHECK(hipDeviceSynchronize());
  MM_HIP_CHECK(hipMemcpy(h.data(), w->st, sizeof(mm::SwitchState) * w->E, hipMemcpyDeviceToHost));
  const int N = w->cfg.n_agents;
  for (int64_t e = 0; e < w->E; ++e) {
    for (int k = 0; k < N; ++k) {
      pos[(e * N + k) * 2] = h[e].pos[k][0];
      pos[(e * N + k) * 2 + 1] = h[e].pos[k][1];
      agent_done[e * N + k] = h[e].adone[k];
    }
    steps[e] = h[e].steps;
  }
  return MM_OK;
}

int mm_switch_set_state(mm_switch* w, const int32_t* pos, const uint8_t* agent_done, const int32_t* steps) {
  MM_REQUIRE(w && pos && agent_done && steps, "switch_set_state: bad arguments");
  const int N = w->cfg.n_agents;
  std::vector<mm::SwitchState> h(w->E);
  for (int64_t e = 0; e < w->E; ++e) {
    mm::SwitchState& s = h[e];
    for (int k = 0; k < 4; ++k) {
      const bool on = k < N;
      const int r = on ? pos[(e * N + k) * 2] : -1, c = on ? pos[(e * N + k) * 2 + 1] : -1;
      MM_REQUIRE(!on || (r >= 0 && r < 3 && c >= 0 && c < 7), "switch_set_state: position off the grid");
      s.pos[k][0] = (int8_t)r;
      s.pos[k][1] = (int8_t)c;
      s.adone[k] = on ? (agent_done[e * N + k] ? 1 : 0) : 0;
    }
    s.steps = steps[e];
  }
  MM_HIP_CHECK(hipDeviceSynchronize());
  MM_HIP_CHECK(hipMemcpy(w->st, h.data(), sizeof(mm::SwitchState) * w->E, hipMemcpyHostToDevice));
  return MM_OK;
}

}  // extern "C"
