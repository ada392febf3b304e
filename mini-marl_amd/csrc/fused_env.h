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

// ---- per-env pieces of the fused step (agent_fwd.hip rollout_step_h3_kernel), host+device so the CPU
// suite checks them against oracle/env.py (tests/native/fused_env_check.cpp)
constexpr int FS_ENVS = 256;   // envs per workgroup (16 waves x 16 envs)
constexpr int FS_PW = 8;       // packed grid words per env (16 cells each: R * C <= 128)
struct FusedSmem {              // after the weight image (bytes)
  static constexpr int pos = 0;                            // u16 [8][256]: r * 256 + c
  static constexpr int grid = pos + 8 * FS_ENVS * 2;       // u32 [8][256]: 2-bit cells
  static constexpr int mask = grid + FS_PW * FS_ENVS * 4;  // u64 [4][256]: obs masks of the observed agents
  static constexpr int row = mask + 4 * FS_ENVS * 8;       // i32 [256]: the env's staging row
  static constexpr int imask = row + FS_ENVS * 4;          // u64 [4]: obs masks of the initial state
  static constexpr int igrid = imask + 4 * 8;              // u32 [8]: initial grid, packed
  static constexpr int ipos = igrid + FS_PW * 4;           // u16 [8]: initial positions
  static constexpr int done = ipos + 8 * 2;                // u8 [256]
  static constexpr int total = done + FS_ENVS;
};

// cell i of a packed grid whose words are `stride` u32 apart
__host__ __device__ __forceinline__ int fs_cell(const uint32_t* g, int stride, int i) {
  return (int)((g[(i >> 4) * stride] >> ((i & 15) * 2)) & 3u);
}

// 2-bit cells of 4 grid bytes (values 0..2) packed into 8 bits
__host__ __device__ __forceinline__ uint32_t fs_pack4(uint32_t v) {
  return (v & 3u) | ((v >> 6) & 0xCu) | ((v >> 12) & 0x30u) | ((v >> 18) & 0xC0u);
}
// ... and back: 8 bits -> 4 bytes
__host__ __device__ __forceinline__ uint32_t fs_unpack4(uint32_t b) {
  return (b & 3u) | ((b & 0xCu) << 6) | ((b & 0x30u) << 12) | ((b & 0xC0u) << 18);
}

// packed word pw (cells 16 pw .. 16 pw + 15) of a row of RC grid bytes; loads clamped inside the row (no
// branches: every load of the caller is in flight at once)
__host__ __device__ __forceinline__ uint32_t fs_load_word(const int8_t* rowp, int RC, int pw) {
  uint32_t w = 0;
  if ((RC & 3) == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int off = 16 * pw + 4 * q;
      const uint32_t v = *reinterpret_cast<const uint32_t*>(rowp + (off < RC ? off : RC - 4));
      w |= (off < RC ? fs_pack4(v) : 0u) << (8 * q);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int off = 16 * pw + i;
      const uint32_t v = (uint32_t)(uint8_t)rowp[off < RC ? off : RC - 1];
      w |= (off < RC ? (v & 3u) : 0u) << (2 * i);
    }
  }
  return w;
}

// 45-bit local observation mask of the agent at (ar, ac): cell-major 3x3 (row-major, centre = own cell) x 5
// channels {lemon, apple, even agent, odd agent, wall} (oracle/env.py observe)
__host__ __device__ __forceinline__ uint64_t fs_obs_mask(const uint32_t* g, int stride, const int (&pr)[8], const int (&pc)[8],
                                                int N, int R, int C, int ar, int ac) {
  uint64_t m = 0;
#pragma unroll
  for (int cell = 0; cell < 9; ++cell) {
    const int rr = ar + cell / 3 - 1, cc = ac + cell % 3 - 1;
    uint32_t bits;
    if (rr < 0 || rr >= R || cc < 0 || cc >= C) {
      bits = 16u;
    } else {
      const int item = fs_cell(g, stride, rr * C + cc);
      int who = -1;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < N && pr[j] == rr && pc[j] == cc) who = j;
      bits = (item == 1 ? 1u : 0u) | (item == 2 ? 2u : 0u) | ((item == 0 && who >= 0) ? ((who & 1) ? 8u : 4u) : 0u);
    }
    m |= (uint64_t)bits << (5 * cell);
  }
  return m;
}

// positions and obs masks of the observed agent(s) of one state into LDS (item stride `stride`)
__host__ __device__ __forceinline__ void fs_publish(const FusedEnv& ev, const int (&pr)[8], const int (&pc)[8], const uint32_t* g,
                                           int gstride, int agent, uint16_t* sp, uint64_t* sm, int stride) {
#pragma unroll
  for (int j = 0; j < 8; ++j) sp[j * stride] = (uint16_t)(j < ev.N ? ((pr[j] << 8) | pc[j]) : 0);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int aq = ev.full_obs ? q : agent;
    if (q < (ev.full_obs ? ev.N : 1)) {
      int ar = 0, ac = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j == aq) {
          ar = pr[j];
          ac = pc[j];
        }
      sm[q * stride] = fs_obs_mask(g, gstride, pr, pc, ev.N, ev.R, ev.C, ar, ac);
    }
  }
}

// obs feature f of agent `agent` (partial: its 47 local features; full: agent f / 47's) of env le, or of the
// initial state (the reset obs) where `init`
__host__ __device__ __forceinline__ float fs_feature(const FusedEnv& ev, const uint16_t* s_pos, const uint64_t* s_mask,
                                            const uint16_t* s_ipos, const uint64_t* s_imask, int le, bool init,
                                            int agent, int f) {
  int q = 0, lf = f, a = agent;
  if (ev.full_obs) {
    q = f / 47;
    lf = f - 47 * q;
    a = q;
  }
  if (lf < 2) {
    const int p = init ? s_ipos[a] : s_pos[a * FS_ENVS + le];
    return lf == 0 ? (float)(p >> 8) * ev.inv_r : (float)(p & 255) * ev.inv_c;
  }
  const uint64_t m = init ? s_imask[q] : s_mask[q * FS_ENVS + le];
  return ((m >> (lf - 2)) & 1ull) ? 1.0f : 0.0f;
}

// one env's transition (oracle/env.py VecEnvOracle.step, env.hip phase 1): agents in id order, a move blocked
// by the border or a cell held by another agent, the fruit of the destination cell eaten; positions in pr / pc,
// the packed grid at g (words `stride` apart) updated in place. Returns done (max steps or no apple left).
__host__ __device__ __forceinline__ bool fs_dynamics(const FusedEnv& ev, int (&pr)[8], int (&pc)[8], const int (&ak)[8],
                                                     uint32_t* g, int stride, int& steps, int& apples, float (&rw)[8]) {
  steps += 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    rw[k] = 0.f;
    if (k < ev.N) {
      const int a = ak[k];
      const int nr = pr[k] + (a == 0 ? 1 : (a == 2 ? -1 : 0));
      const int nc = pc[k] + (a == 1 ? -1 : (a == 3 ? 1 : 0));
      bool okm = nr >= 0 && nr < ev.R && nc >= 0 && nc < ev.C;
#pragma unroll
      for (int j = 0; j < 8; ++j) okm = okm && (j == k || pr[j] != nr || pc[j] != nc);
      if (okm) {
        pr[k] = nr;
        pc[k] = nc;
      }
      const int cell = pr[k] * ev.C + pc[k];
      const int item = fs_cell(g, stride, cell);
      const bool big = (k & 1) == 0;
      rw[k] = ev.step_cost + (item == 2 ? (big ? 10.0f : 1.0f) : (item == 1 ? (big ? -10.0f : -1.0f) : 0.0f));
      apples -= item == 2 ? 1 : 0;
      g[(cell >> 4) * stride] &= ~(3u << ((cell & 15) * 2));
    }
  }
  return steps >= ev.max_steps || apples == 0;
}
}  // namespace mm
