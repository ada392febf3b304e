// Device view of the Checkers gridworld (env.hip) for the fused rollout step (agent_fwd.hip): the
// env's integer state double-buffered by step parity (the fused kernel's blocks all read buffer t & 1
// while one block per env tile writes buffer (t + 1) & 1, so no block reads a half-updated state).
#pragma once
#include "common.h"
#include "minimarl.h"

namespace mm {
struct FusedEnv {
  int E, N, R, C, D, max_steps, full_obs, init_apples;
  float step_cost, inv_r, inv_c;
  int32_t* pos[2];          // [E][N] r * 256 + c
  int8_t* grid[2];          // [E][R * C] 0 empty, 1 lemon, 2 apple
  int32_t* steps[2];        // [E]
  int32_t* apples[2];       // [E]
  const int8_t* init_grid;  // [R * C]
  const int32_t* init_pos;  // [N]
  const float* reset_obs;   // [N][D]
};
// fills v (buffer 0 = the env's live state, buffer 1 its second copy); MM_EINVAL for a shape the fused
// step does not support
int env_fused_view(mm_env* env, FusedEnv* v);
}  // namespace mm
