// The ma_gym Switch corridor env (QMIX's default "ma_gym:Switch2-v0", qmix/_config.py:14-19,
// qmix/main.py:66-71), E envs in lockstep. Dynamics spec: oracle/switch.py (ma-gym is absent, so
// parity with it is unpinned). The whole state of an env is 4 agent cells, 4 done bits and a step
// count — one thread per env keeps it in registers for the agent-ordered move loop; the obs rows
// (3 or 3N floats per agent) are written as the thread's contiguous [N, D] run.
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

__constant__ float kSwitchCol[7];
__constant__ float kSwitchRow[3];

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

__device__ __forceinline__ void sw_obs(const SwitchState& s, int N, int max_steps, int full, int clock,
                                       float* __restrict__ out) {
  const int ld = 2 + clock;
  const int D = full ? ld * N : ld;
  const float clk = (float)((double)s.steps / (double)max_steps);
  for (int k = 0; k < N; ++k) {
    float loc[3] = {kSwitchRow[s.pos[k][0]], kSwitchCol[s.pos[k][1]], clk};
    if (full) {
      for (int j = 0; j < N; ++j)
        for (int f = 0; f < ld; ++f) out[j * D + k * ld + f] = loc[f];
    } else {
      for (int f = 0; f < ld; ++f) out[k * D + f] = loc[f];
    }
  }
}

__global__ __launch_bounds__(256) void switch_reset_kernel(SwitchState* __restrict__ st, int64_t E, int N,
                                                           int max_steps, int full, int clock, float* __restrict__ obs) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  SwitchState s;
  sw_init(s, N);
  st[e] = s;
  const int D = (2 + clock) * (full ? N : 1);
  if (obs) sw_obs(s, N, max_steps, full, clock, obs + e * N * D);
}

__global__ __launch_bounds__(256) void switch_step_kernel(SwitchState* __restrict__ st, int64_t E, int N, int max_steps,
                                                          int full, int clock, float step_cost,
                                                          const int32_t* __restrict__ act, float* __restrict__ next_obs,
                                                          float* __restrict__ obs_cur, float* __restrict__ rew,
                                                          uint8_t* __restrict__ agent_done, uint8_t* __restrict__ done) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  const int dr[5] = {1, 0, -1, 0, 0}, dc[5] = {0, -1, 0, 1, 0};
  const int fr[4] = {0, 0, 2, 2}, fc[4] = {6, 0, 6, 0};
  SwitchState s = st[e];
  s.steps += 1;
  float r_out[4];
  for (int k = 0; k < N; ++k) {
    r_out[k] = step_cost;
    if (s.adone[k]) continue;
    const int a = act[e * N + k];
    if (a >= 0 && a < 4) {
      const int r = s.pos[k][0] + dr[a], c = s.pos[k][1] + dc[a];
      bool ok = sw_open(r, c);
      for (int j = 0; j < N; ++j) ok = ok && (j == k || s.pos[j][0] != r || s.pos[j][1] != c);
      if (ok) {
        s.pos[k][0] = (int8_t)r;
        s.pos[k][1] = (int8_t)c;
      }
    }
    if (s.pos[k][0] == fr[k] && s.pos[k][1] == fc[k]) {
      s.adone[k] = 1;
      r_out[k] = 5.0f;
    }
  }
  bool all = true;
  for (int k = 0; k < N; ++k) {
    if (s.steps >= max_steps) s.adone[k] = 1;
    all = all && s.adone[k];
  }
  const int D = (2 + clock) * (full ? N : 1);
  sw_obs(s, N, max_steps, full, clock, next_obs + e * N * D);
  for (int k = 0; k < N; ++k) {
    rew[e * N + k] = r_out[k];
    if (agent_done) agent_done[e * N + k] = s.adone[k];
  }
  done[e] = all ? 1 : 0;
  if (obs_cur) {                         // auto-reset: the next current obs is the reset obs of a done env
    if (all) sw_init(s, N);
    sw_obs(s, N, max_steps, full, clock, obs_cur + e * N * D);
  }
  st[e] = s;
}

}  // namespace mm

struct mm_switch {
  mm_switch_cfg cfg;
  int64_t E;
  mm::SwitchState* st;
};

extern "C" {

int mm_switch_create(const mm_switch_cfg* cfg, int64_t n_envs, mm_switch** out) {
  MM_REQUIRE(cfg && out && n_envs >= 1, "switch_create: bad arguments");
  MM_REQUIRE(cfg->n_agents >= 2 && cfg->n_agents <= 4, "switch_create: n_agents must be 2..4 (got %d)", cfg->n_agents);
  MM_REQUIRE(cfg->max_steps >= 1, "switch_create: max_steps must be >= 1");
  static bool tables = false;
  if (!tables) {   // round(c / 6, 2), round(r / 2, 2) as Python floats -> float32
    float col[7], row[3];
    for (int c = 0; c < 7; ++c) col[c] = (float)(std::round(c / 6.0 * 100.0) / 100.0);
    for (int r = 0; r < 3; ++r) row[r] = (float)(r / 2.0);
    MM_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(mm::kSwitchCol), col, sizeof(col)));
    MM_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(mm::kSwitchRow), row, sizeof(row)));
    tables = true;
  }
  mm_switch* w = new mm_switch;
  w->cfg = *cfg;
  w->E = n_envs;
  if (hipMalloc(&w->st, sizeof(mm::SwitchState) * n_envs) != hipSuccess) {
    delete w;
    mm::set_error("switch_create: hipMalloc failed");
    return MM_ENOMEM;
  }
  const mm_switch_cfg& c = w->cfg;
  hipLaunchKernelGGL(mm::switch_reset_kernel, dim3((n_envs + 255) / 256), dim3(256), 0, 0, w->st, n_envs, c.n_agents,
                     c.max_steps, c.full_observable, c.clock, (float*)nullptr);
  if (hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(w->st);
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

int mm_switch_reset(mm_switch* w, float* obs, mm_stream_t s) {
  MM_REQUIRE(w, "switch_reset: NULL handle");
  const mm_switch_cfg& c = w->cfg;
  hipLaunchKernelGGL(mm::switch_reset_kernel, dim3((w->E + 255) / 256), dim3(256), 0, (hipStream_t)s, w->st, w->E,
                     c.n_agents, c.max_steps, c.full_observable, c.clock, obs);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_switch_step(mm_switch* w, const int32_t* act, float* next_obs, float* obs_cur, float* rew,
                   uint8_t* agent_done, uint8_t* done, mm_stream_t s) {
  MM_REQUIRE(w && act && next_obs && rew && done, "switch_step: bad arguments");
  const mm_switch_cfg& c = w->cfg;
  hipLaunchKernelGGL(mm::switch_step_kernel, dim3((w->E + 255) / 256), dim3(256), 0, (hipStream_t)s, w->st, w->E,
                     c.n_agents, c.max_steps, c.full_observable, c.clock, c.step_cost, act, next_obs, obs_cur, rew,
                     agent_done, done);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
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

}  // extern "C"
