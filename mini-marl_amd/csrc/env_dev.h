// Device view of the restated ma_gym Checkers-v0 env (oracle/env.py), shared by the env kernels (env.hip) and
// the fused rollout step (agent_fwd.hip, rollout_step_kernel).
#pragma once
#include <stdint.h>

namespace mm {
static constexpr int OBS_LOCAL = 47;

struct EnvDev {
  int E, N, R, C, D, max_steps, full_obs, init_apples;
  int eb;  // envs per block of the step kernel
  float step_cost;
  // live state (the env kernels read and write these). The fused rollout step double-buffers it: it reads
  // buffer t % 2 (0 = these, 1 = the *_alt arrays) and writes the other.
  int32_t* pos;     // [E][N] prev_r << 24 | prev_c << 16 | r << 8 | c
  int8_t* grid;     // [E][R*C] _full_obs codes
  int32_t* steps;   // [E]
  int32_t* apples;  // [E]
  int32_t* pos_alt;
  int8_t* grid_alt;
  int32_t* steps_alt;
  int32_t* apples_alt;
  const int8_t* init_grid;  // [R*C] (agent markers at their start cells, then the fruit)
  const int32_t* init_pos;  // [N] (prev = pos)
  const float* rtab;        // [R] round(r / (R - 1), 2) as f32
  const float* ctab;        // [C] round(c / (C - 1), 2) as f32
  float* reset_obs;         // [N][D]
};

__host__ __device__ __forceinline__ int pos_r(int32_t w) { return (w >> 8) & 255; }
__host__ __device__ __forceinline__ int pos_c(int32_t w) { return w & 255; }
}  // namespace mm

struct mm_env {
  mm::EnvDev d;
  void* alloc;
};
