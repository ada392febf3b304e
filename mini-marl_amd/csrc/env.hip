// ma_gym Checkers-v0, restated (oracle/env.py): E envs x N agents stepped by one kernel (gfx950).
//
// Replaces the per-step gym env call (vdn/main.py:93,143; qmix/main.py:115,189;
// mappo/runner/shared/magym_runner.py:53-57). ma-gym 0.0.14 itself is absent, so the dynamics follow the
// rule-by-rule restatement of ma_gym's published envs/checkers/checkers.py in oracle/env.py (parity with
// ma_gym: UNPINNED; parity with oracle/env.py: bit-exact, integer state). The state mirrors ma_gym's:
// _full_obs as one byte per cell (0 empty, 1 lemon, 2 apple, 3 + k agent k's marker), agent_pos and
// agent_prev_pos packed in one word per agent (prev_r << 24 | prev_c << 16 | r << 8 | c), _step_count and
// _food_count['apple'] per env.
//
// One wave per env tile (256-thread blocks, the extra waves stream the obs out): phase 0 stages every global
// input of the step (grids as bytes [E][R*C], one contiguous coalesced run; positions, actions, counters,
// coordinate tables) in LDS in ONE round trip; phase 1 runs the sequential-in-agent-order dynamics one lane
// per env on the LDS grid; phase 2 builds each (env, agent)'s 47 local features into an LDS tile from the
// grid; phase 3 streams the tile out as 16-byte stores and writes the state back (or the initial state for
// envs that auto-reset).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"
#include "env_dev.h"
#include "minimarl.h"

namespace mm {

// feature f in [0, 47) of agent k's local obs (get_agent_obs): coords from the tables, then the 3x3 cells x
// {lemon, apple, even agent, odd agent, wall} read from the grid; off-grid cells stay all zero
__device__ __forceinline__ float obs_value(const EnvDev& d, const int32_t* pos, const int8_t* grid, int k, int f) {
  const int r = pos_r(pos[k]), c = pos_c(pos[k]);
  if (f == 0) return d.rtab[r];
  if (f == 1) return d.ctab[c];
  const int cell = (f - 2) / 5, ch = (f - 2) % 5;
  const int rr = r + cell / 3 - 1, cc = c + cell % 3 - 1;
  if (rr < 0 || rr >= d.R || cc < 0 || cc >= d.C || ch == 4) return 0.0f;
  const int item = grid[rr * d.C + cc];
  if (ch < 2) return item == ch + 1 ? 1.0f : 0.0f;
  return (item >= 3 && ((item - 3) & 1) == ch - 2) ? 1.0f : 0.0f;
}

// Writes obs of one env (N x D) from the given state into out (+ optional 2nd copy).
__device__ __forceinline__ float obs_elem(const EnvDev& d, const int32_t* pos, const int8_t* grid, int k, int f) {
  if (d.full_obs) return obs_value(d, pos, grid, f / OBS_LOCAL, f % OBS_LOCAL);
  (void)k;
  return obs_value(d, pos, grid, k, f);
}

__global__ __launch_bounds__(256) void env_reset_kernel(EnvDev d, float* obs, int write_table) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int32_t* spos = reinterpret_cast<int32_t*>(smem);
  int8_t* sgrid = reinterpret_cast<int8_t*>(smem + ((d.N * 4 + 15) & ~15));
  const int RC = d.R * d.C;
  for (int i = threadIdx.x; i < d.N; i += blockDim.x) spos[i] = d.init_pos[i];
  for (int i = threadIdx.x; i < RC; i += blockDim.x) sgrid[i] = d.init_grid[i];
  __syncthreads();
  if (write_table && blockIdx.x == 0) {
    for (int i = threadIdx.x; i < d.N * d.D; i += blockDim.x)
      d.reset_obs[i] = obs_elem(d, spos, sgrid, i / d.D, i % d.D);
  }
  const int e0 = blockIdx.x * d.eb;
  const int ne = min(d.eb, d.E - e0);
  for (int i = threadIdx.x; i < ne * RC; i += blockDim.x) d.grid[(int64_t)e0 * RC + i] = sgrid[i % RC];
  for (int i = threadIdx.x; i < ne * d.N; i += blockDim.x) d.pos[(int64_t)e0 * d.N + i] = spos[i % d.N];
  for (int i = threadIdx.x; i < ne; i += blockDim.x) {
    d.steps[e0 + i] = 0;
    d.apples[e0 + i] = d.init_apples;
  }
  if (obs) {
    const int ND = d.N * d.D;
    for (int i = threadIdx.x; i < ne * ND; i += blockDim.x) {
      const int k = (i % ND) / d.D, f = i % d.D;
      obs[(int64_t)e0 * ND + i] = obs_elem(d, spos, sgrid, k, f);
    }
  }
}

// One wave of (env, agent) lanes per block, EPW = 64 / N envs (lane = env-slot * N + agent). Phase 0 issues
// every global read of the step at once (positions, actions, grid words, counters, destination rows, the fused
// TD inputs, the coordinate tables); phase 1 runs ma_gym's sequential-in-agent-order dynamics, one lane per env
// on the env's LDS grid; phase 2 every (env, agent) lane writes its 47 local features into an LDS tile; phase 3
// streams the tile out as 16-byte stores (one contiguous N*D run per env, coalesced across the wave) and writes
// the state back.
static constexpr int WT = 64;     // lanes of the (env, agent) work: one wave
static constexpr int TB = 256;    // threads per block: the extra waves only help stream the obs / state out

// LDS layout of the step kernel (byte offsets, 16-byte aligned pieces), shared by the kernel and the host
struct EnvSmem {
  int sloc, srow, sbsrc, std3, spos, sact, sdm, stab, sgrid, total;
};
__host__ __device__ __forceinline__ int al16(int x) { return (x + 15) & ~15; }
__host__ __device__ __forceinline__ EnvSmem env_smem(int EPW, int N, int R, int C) {
  EnvSmem m;
  int o = 0;
  m.sloc = o;  o = al16(o + EPW * N * OBS_LOCAL * 4);   // [EPW][N][47] f32 obs tile
  m.srow = o;  o = al16(o + EPW * 8);                   // [EPW] i64 destination rows
  m.sbsrc = o; o = al16(o + EPW * 8);                   // [EPW] i64 chunk-begin source rows
  m.std3 = o;  o = al16(o + 3 * EPW * N * 4);           // [3][EPW*N] fused TD inputs
  m.spos = o;  o = al16(o + EPW * N * 4);               // [EPW*N] position words
  m.sact = o;  o = al16(o + EPW * N * 4);               // [EPW*N] actions
  m.sdm = o;   o = al16(o + 8);                         // termination mask (wave ballot)
  m.stab = o;  o = al16(o + (R + C) * 4);               // [R] row + [C] column coordinate features
  m.sgrid = o; o = al16(o + EPW * R * C);               // [EPW][RC] grids (_full_obs)
  m.total = o;
  return m;
}

__global__ __launch_bounds__(TB) void env_step_wave_kernel(EnvDev d, const int32_t* __restrict__ act,
                                                           float* __restrict__ next_obs, int64_t next_se,
                                                           const int64_t* __restrict__ next_row,
                                                           float* __restrict__ obs_cur,
                                                           int64_t* __restrict__ cur_row, float* rew,  // rew may alias tdf.rew
                                                           uint8_t* __restrict__ done_out, TdFuse tdf, BeginCopy bc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int RC = d.R * d.C;
  const int N = d.N;
  const int EPW = d.eb;  // envs per wave (<= 64 / N)
  const int lane = threadIdx.x;
  const bool autoreset = obs_cur || cur_row;
  const int ND = N * d.D;
  const int LD = N * OBS_LOCAL;                                              // local tile per env
  const EnvSmem lay = env_smem(EPW, N, d.R, d.C);
  float* sloc = reinterpret_cast<float*>(smem + lay.sloc);
  int64_t* srow = reinterpret_cast<int64_t*>(smem + lay.srow);
  int64_t* sbsrc = reinterpret_cast<int64_t*>(smem + lay.sbsrc);
  float* std3 = reinterpret_cast<float*>(smem + lay.std3);
  int32_t* spos = reinterpret_cast<int32_t*>(smem + lay.spos);
  int32_t* sact = reinterpret_cast<int32_t*>(smem + lay.sact);
  uint64_t* sdm = reinterpret_cast<uint64_t*>(smem + lay.sdm);
  float* stab = reinterpret_cast<float*>(smem + lay.stab);
  int8_t* sgrid = reinterpret_cast<int8_t*>(smem + lay.sgrid);
  const int e0 = blockIdx.x * EPW;
  const int ne = min(EPW, d.E - e0);
  const int nl = ne * N;                   // active (env, agent) lanes
  const int le_l = lane / N, k_l = lane % N;
  const int e_l = e0 + le_l;

  // ---- phase 0: every global read of the step issued into registers first (one memory round
  // trip for the wave), then staged in LDS
  constexpr int GWR = 4;                   // grid dwords per lane held in registers
  const bool g32ok = (RC & 3) == 0;
  const int nw = g32ok ? ne * RC / 4 : 0;
  const uint32_t* g32 = reinterpret_cast<const uint32_t*>(d.grid + (int64_t)e0 * RC);
  uint32_t gr[GWR];
#pragma unroll
  for (int w = 0; w < GWR; ++w) gr[w] = (lane + w * TB < nw) ? g32[lane + w * TB] : 0u;
  int32_t pos_w = 0, act_r = 0, tact_r = 0;
  float trew = 0.f, tq = 0.f, tm = 0.f, tab = 0.f;
  int64_t trow = 0;
  if (lane < nl) {
    const int64_t o = (int64_t)e0 * N + lane;
    pos_w = d.pos[o];
    act_r = act[o];
    if (tdf.on) {
      trew = tdf.rew[o];
      tq = tdf.q_taken[o];
      tm = tdf.maxq[o];
      tact_r = tdf.act[o];
      trow = tdf.rows[e_l];
    }
  }
  if (lane < d.R + d.C) tab = lane < d.R ? d.rtab[lane] : d.ctab[lane - d.R];
  int apples0 = 0, steps0 = 0;
  int64_t srow_r = 0, bsrc_r = -1;
  uint8_t tdone = 0;
  if (lane < ne) {
    srow_r = next_row ? next_row[e0 + lane] : (int64_t)(e0 + lane);
    apples0 = d.apples[e0 + lane];
    steps0 = d.steps[e0 + lane];
    if (tdf.on) tdone = tdf.done[e0 + lane];
    if (bc.on) bsrc_r = cur_row[e0 + lane];     // read before this step overwrites it
  }
#pragma unroll
  for (int w = 0; w < GWR; ++w)
    if (lane + w * TB < nw) reinterpret_cast<uint32_t*>(sgrid)[lane + w * TB] = gr[w];
  for (int i = lane + GWR * TB; i < nw; i += TB) reinterpret_cast<uint32_t*>(sgrid)[i] = g32[i];
  if (!g32ok)
    for (int i = lane; i < ne * RC; i += TB) sgrid[i] = d.grid[(int64_t)e0 * RC + i];
  for (int i = lane + TB; i < d.R + d.C; i += TB) stab[i] = i < d.R ? d.rtab[i] : d.ctab[i - d.R];
  if (lane < d.R + d.C) stab[lane] = tab;
  if (lane < nl) {
    spos[lane] = pos_w;
    sact[lane] = act_r;
    if (tdf.on) {
      std3[lane] = trew;
      std3[EPW * N + lane] = tq;
      std3[2 * EPW * N + lane] = tm;
      tdf.s_act[(trow * tdf.C + tdf.slot) * N + k_l] = (uint8_t)tact_r;
      tdf.s_rew[(trow * tdf.C + tdf.slot) * N + k_l] = trew;
    }
  }
  if (lane < ne) {
    srow[lane] = srow_r;
    sbsrc[lane] = bsrc_r;
  }
  __syncthreads();

  // fused TD of the previous step: agent-order sums per env (one lane per env)
  if (tdf.on && lane < ne) {
    const int e = e0 + lane;
    float sr = 0.f, sq = 0.f, st = 0.f;
    for (int j = 0; j < N; ++j) {
      sr += std3[lane * N + j];
      sq += std3[EPW * N + lane * N + j];
      st += std3[2 * EPW * N + lane * N + j];
    }
    const float dn = tdone ? 1.0f : 0.0f;
    const float td = rollout_td(sr, sq, st, dn, tdf.gamma);
    tdf.chunk_td[e] = (tdf.slot == 0 ? 0.0f : tdf.chunk_td[e]) + td;
    const int64_t row = tdf.rows[e];
    tdf.s_done[row * tdf.C + tdf.slot] = tdone;
    if (tdf.counter && blockIdx.x == 0 && lane == 0) *tdf.counter += 1;
  }

  // ---- phase 1: ma_gym Checkers.step, one lane per env, agents in id order (oracle/env.py
  // VecEnvOracle.step): move when the next cell is on the grid and holds no agent marker (agent_prev_pos <-
  // old position only then); if agent_pos != agent_prev_pos (possibly stale) the fruit at the agent's cell is
  // eaten (lemon / apple reward, apple count) and the view update writes empty at agent_prev_pos and the
  // marker at agent_pos. Two dependent LDS round trips per agent (the target cell, then the agent's cell).
  if (lane < ne) {
    const int le = lane, e = e0 + lane;
    int8_t* g = sgrid + le * RC;
    int32_t* p = spos + le * N;
    int apples = apples0;
    const int steps = steps0 + 1;
#pragma unroll 1
    for (int k = 0; k < N; ++k) {
      const int a = sact[le * N + k];
      const int32_t w = p[k];
      int r = pos_r(w), c = pos_c(w), pr = (w >> 24) & 255, pc = (w >> 16) & 255;
      const int nr = r + (a == 0 ? 1 : (a == 2 ? -1 : 0));
      const int nc = c + (a == 1 ? -1 : (a == 3 ? 1 : 0));
      const bool inside = a != 4 && nr >= 0 && nr < d.R && nc >= 0 && nc < d.C;
      if (inside && g[nr * d.C + nc] < 3) {
        pr = r;
        pc = c;
        r = nr;
        c = nc;
      }
      float rk = d.step_cost;
      if (r != pr || c != pc) {
        const int cell = r * d.C + c;
        const int item = g[cell];
        const bool big = (k & 1) == 0;
        if (item == 1) rk += big ? -10.0f : -1.0f;
        if (item == 2) {
          rk += big ? 10.0f : 1.0f;
          apples -= 1;
        }
        g[pr * d.C + pc] = 0;
        g[cell] = (int8_t)(3 + k);
      }
      p[k] = (pr << 24) | (pc << 16) | (r << 8) | c;
      rew[(int64_t)e * N + k] = rk;
    }
    const bool dn = steps >= d.max_steps || apples == 0;
    // termination mask of the block's envs: one wave ballot (lanes < ne are wave 0's first lanes)
    const uint64_t dm = __ballot(dn);
    if (lane == 0) *sdm = dm;
    done_out[e] = dn ? 1 : 0;
    if (cur_row) cur_row[e] = dn ? -1 : srow_r;
    d.steps[e] = dn && autoreset ? 0 : steps;
    d.apples[e] = dn && autoreset ? d.init_apples : apples;
  }
  __syncthreads();
  // ---- phase 2: local obs of (env, agent) ea = lane % 64 into the LDS tile; the block's TB / 64 waves
  // split the 9 neighbourhood cells (wave w: cells w, w + TB/64, ...), wave 0 also writes the coords
  const int ea = lane & (WT - 1), part = lane / WT;
  int mypos = 0;
  if (ea < nl) mypos = spos[ea];
  if (ea < nl) {
    const int le2 = ea / N, k2 = ea % N;
    float* o = sloc + le2 * LD + k2 * OBS_LOCAL;
    const int pr = pos_r(mypos), pc = pos_c(mypos);
    if (part == 0) {
      o[0] = stab[pr];
      o[1] = stab[d.R + pc];
    }
    const int8_t* g = sgrid + le2 * RC;
    for (int cell = part; cell < 9; cell += TB / WT) {
      const int rr = pr + cell / 3 - 1, cc = pc + cell % 3 - 1;
      const bool inside = rr >= 0 && rr < d.R && cc >= 0 && cc < d.C;
      const int item = inside ? g[rr * d.C + cc] : 0;
      float* q = o + 2 + 5 * cell;
      q[0] = item == 1 ? 1.f : 0.f;
      q[1] = item == 2 ? 1.f : 0.f;
      q[2] = (item >= 3 && ((item - 3) & 1) == 0) ? 1.f : 0.f;
      q[3] = (item >= 3 && ((item - 3) & 1) == 1) ? 1.f : 0.f;
      q[4] = 0.f;
    }
  }
  __syncthreads();

  // ---- phase 3: stream the obs out (env le's N*D run from its local tile) and write state back
  const uint64_t dmask = *sdm;
  auto env_done = [&](int le) { return ((dmask >> le) & 1ull) != 0; };
  const bool full = d.full_obs != 0;
  const float* robs = d.reset_obs;
  const bool vec = (ND & 3) == 0 && (next_se & 3) == 0 && ((uintptr_t)next_obs & 15) == 0 &&
                   ((uintptr_t)obs_cur & 15) == 0;
  if (vec) {
    // flat float4 index i = lane + TB*it over the block's ne x ND4 outputs, walked with a running
    // (env, offset) pair instead of a division per element
    const int ND4 = ND >> 2;
    int le = 0, r4 = lane;
    while (r4 >= ND4 && le < ne) {
      r4 -= ND4;
      ++le;
    }
    for (; le < ne;) {
      const int r = r4 * 4;
      const float* t = sloc + le * LD;
      float4 v;
      if (!full) {
        v = *reinterpret_cast<const float4*>(t + r);
      } else {
        v.x = t[(r + 0) % LD];  // full obs: every agent sees the whole [N][47] tile
        v.y = t[(r + 1) % LD];
        v.z = t[(r + 2) % LD];
        v.w = t[(r + 3) % LD];
      }
      if (next_obs) *reinterpret_cast<float4*>(next_obs + srow[le] * next_se + r) = v;
      if (obs_cur) {
        if (env_done(le)) v = *reinterpret_cast<const float4*>(robs + r);
        *reinterpret_cast<float4*>(obs_cur + (int64_t)(e0 + le) * ND + r) = v;
      }
      r4 += TB;
      while (r4 >= ND4 && le < ne) {
        r4 -= ND4;
        ++le;
      }
    }
  } else {
    for (int i = lane; i < ne * ND; i += TB) {
      const int le = i / ND, r = i - le * ND;
      const float v = sloc[le * LD + (full ? r % LD : r)];
      if (next_obs) next_obs[srow[le] * next_se + r] = v;
      if (obs_cur) obs_cur[(int64_t)(e0 + le) * ND + r] = env_done(le) ? robs[r] : v;
    }
  }
  if (bc.on) {
    // chunk start (mm_chunk_begin_rows folded in): slot 0 of the new staging row <- slot C of the env's
    // previous row (its last next obs), or the reset obs where the env had just reset
    const bool bvec = (ND & 3) == 0 && (bc.row_stride & 3) == 0 && (bc.src_off & 3) == 0 &&
                      ((uintptr_t)bc.store & 15) == 0 && ((uintptr_t)robs & 15) == 0;
    if (bvec) {
      const int ND4 = ND >> 2;
      for (int i = lane; i < ne * ND4; i += TB) {
        const int le = i / ND4, r = (i - le * ND4) * 4;
        const int64_t src = sbsrc[le];
        const float* sp = src >= 0 ? bc.store + src * bc.row_stride + bc.src_off : robs;
        *reinterpret_cast<float4*>(bc.store + srow[le] * bc.row_stride + r) = *reinterpret_cast<const float4*>(sp + r);
      }
    } else {
      for (int i = lane; i < ne * ND; i += TB) {
        const int le = i / ND, r = i - le * ND;
        const int64_t src = sbsrc[le];
        bc.store[srow[le] * bc.row_stride + r] = src >= 0 ? bc.store[src * bc.row_stride + bc.src_off + r] : robs[r];
      }
    }
  }
  if ((RC & 3) == 0) {
    uint32_t* g32w = reinterpret_cast<uint32_t*>(d.grid + (int64_t)e0 * RC);
    const uint32_t* ig32 = reinterpret_cast<const uint32_t*>(d.init_grid);
    const int RC4 = RC >> 2;
    for (int i = lane; i < ne * RC4; i += TB) {
      const int le = i / RC4;
      g32w[i] = (autoreset && env_done(le)) ? ig32[i - le * RC4] : reinterpret_cast<const uint32_t*>(sgrid)[i];
    }
  } else {
    for (int i = lane; i < ne * RC; i += TB) {
      const int le = i / RC;
      d.grid[(int64_t)e0 * RC + i] = (autoreset && env_done(le)) ? d.init_grid[i % RC] : sgrid[i];
    }
  }
  if (lane < nl) d.pos[(int64_t)e0 * N + lane] = (autoreset && env_done(le_l)) ? d.init_pos[k_l] : mypos;
}

static size_t step_smem(const EnvDev& d) { return (size_t)env_smem(d.eb, d.N, d.R, d.C).total; }

// round(i / (n - 1), 2) as Python computes it (the correctly rounded 2-decimal value of the double quotient,
// ties to even), then float32: printf's %.2f rounds the exact binary value the same way
static float coord_feature(int i, int n) {
  if (n <= 1) return 0.0f;
  char buf[32];
  snprintf(buf, sizeof(buf), "%.2f", (double)i / (double)(n - 1));
  return (float)strtod(buf, nullptr);
}

int env_create(const mm_env_cfg* cfg, int64_t n_envs, uint64_t seed, mm_env** out) {
  (void)seed;  // the layout is deterministic (ma_gym Checkers resets to a fixed layout)
  MM_REQUIRE(cfg && out, "env_create: null argument");
  MM_REQUIRE(n_envs >= 1 && n_envs < (1ll << 31), "env_create: bad n_envs");
  MM_REQUIRE(cfg->n_agents >= 1 && cfg->n_agents <= 64, "env_create: n_agents must be in [1,64]");
  const int cols = cfg->cols > 0 ? cfg->cols : 8;
  MM_REQUIRE(cols >= 3 && cols <= 255, "env_create: cols must be in [3,255]");
  EnvDev d;
  d.E = (int)n_envs;
  d.N = cfg->n_agents;
  d.eb = WT / d.N;
  MM_REQUIRE(d.eb >= 1 && d.eb * d.N <= WT, "env_create: bad envs-per-block");
  d.R = 3 * ((d.N + 1) / 2);
  d.C = cols;
  MM_REQUIRE(d.R <= 255, "env_create: too many agents for the grid");
  d.full_obs = cfg->full_observable ? 1 : 0;
  d.D = OBS_LOCAL * (d.full_obs ? d.N : 1);
  d.max_steps = cfg->max_steps;
  d.step_cost = cfg->step_cost;
  const int RC = d.R * d.C;
  // __init_full_obs: agent markers first, then the fruit of every 3-row band (lemon flag first, flipped
  // after every cell of the column-major walk over columns 0..C-3)
  std::vector<int8_t> grid(RC, 0);
  std::vector<int32_t> pos(d.N);
  for (int k = 0; k < d.N; ++k) {
    const int r = 3 * (k / 2) + 2 * (k % 2), c = d.C - 2;
    pos[k] = (r << 24) | (c << 16) | (r << 8) | c;
    grid[r * d.C + c] = (int8_t)(3 + k);
  }
  int apples = 0;
  for (int b = 0; b < d.R / 3; ++b) {
    bool lemon = true;
    for (int c = 0; c < d.C - 2; ++c)
      for (int lr = 0; lr < 3; ++lr) {
        grid[(3 * b + lr) * d.C + c] = lemon ? 1 : 2;
        apples += lemon ? 0 : 1;
        lemon = !lemon;
      }
  }
  d.init_apples = apples;
  std::vector<float> tab(d.R + d.C);
  for (int r = 0; r < d.R; ++r) tab[r] = coord_feature(r, d.R);
  for (int c = 0; c < d.C; ++c) tab[d.R + c] = coord_feature(c, d.C);
  MM_REQUIRE(step_smem(d) <= 64 * 1024, "env_create: grid too large for LDS staging");

  const size_t E = (size_t)d.E;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  const size_t o_pos = take(E * d.N * 4), o_grid = take(E * RC), o_steps = take(E * 4), o_apples = take(E * 4),
               o_pos2 = take(E * d.N * 4), o_grid2 = take(E * RC), o_steps2 = take(E * 4), o_apples2 = take(E * 4),
               o_igrid = take(RC), o_ipos = take(d.N * 4), o_tab = take((d.R + d.C) * 4),
               o_robs = take((size_t)d.N * d.D * 4);
  void* base = nullptr;
  MM_HIP_CHECK(hipMalloc(&base, off));
  char* b = static_cast<char*>(base);
  d.pos = reinterpret_cast<int32_t*>(b + o_pos);
  d.grid = reinterpret_cast<int8_t*>(b + o_grid);
  d.steps = reinterpret_cast<int32_t*>(b + o_steps);
  d.apples = reinterpret_cast<int32_t*>(b + o_apples);
  d.pos_alt = reinterpret_cast<int32_t*>(b + o_pos2);
  d.grid_alt = reinterpret_cast<int8_t*>(b + o_grid2);
  d.steps_alt = reinterpret_cast<int32_t*>(b + o_steps2);
  d.apples_alt = reinterpret_cast<int32_t*>(b + o_apples2);
  d.init_grid = reinterpret_cast<int8_t*>(b + o_igrid);
  d.init_pos = reinterpret_cast<int32_t*>(b + o_ipos);
  d.rtab = reinterpret_cast<float*>(b + o_tab);
  d.ctab = d.rtab + d.R;
  d.reset_obs = reinterpret_cast<float*>(b + o_robs);
  hipError_t e = hipMemcpy(b + o_igrid, grid.data(), RC, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(b + o_ipos, pos.data(), d.N * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(b + o_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
  mm_env* env = new mm_env;
  env->d = d;
  env->alloc = base;
  const int blocks = (d.E + d.eb - 1) / d.eb;
  const size_t sm = ((d.N * 4 + 15) & ~15) + RC;
  if (e == hipSuccess) {
    hipLaunchKernelGGL(env_reset_kernel, dim3(blocks), dim3(256), sm, 0, d, (float*)nullptr, 1);
    e = hipDeviceSynchronize();
  }
  if (e != hipSuccess) {
    set_error("env_create: reset failed: %s", hipGetErrorString(e));
    (void)hipFree(base);
    delete env;
    return MM_EHIP;
  }
  *out = env;
  return MM_OK;
}

int env_reset(mm_env* env, float* obs, hipStream_t s) {
  MM_REQUIRE(env, "env_reset: null env");
  const EnvDev& d = env->d;
  const int blocks = (d.E + d.eb - 1) / d.eb;
  const size_t sm = ((d.N * 4 + 15) & ~15) + d.R * d.C;
  hipLaunchKernelGGL(env_reset_kernel, dim3(blocks), dim3(256), sm, s, d, obs, 0);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int env_step(mm_env* env, const int32_t* act, float* next_obs, int64_t next_se, const int64_t* next_row,
             float* obs_cur, int64_t* cur_row, float* rew, uint8_t* done, const TdFuse* tdf, hipStream_t s,
             const BeginCopy* bcp = nullptr) {
  MM_REQUIRE(env && act && rew && done, "env_step: null argument");
  MM_REQUIRE(next_obs || obs_cur, "env_step: no obs output");
  const EnvDev& d = env->d;
  const int blocks = (d.E + d.eb - 1) / d.eb;
  TdFuse t{};
  if (tdf) t = *tdf;
  BeginCopy bc{};
  if (bcp) bc = *bcp;
  MM_REQUIRE(!bc.on || (cur_row && next_row), "env_step: the chunk-begin copy needs cur_row and the staging rows");
  hipLaunchKernelGGL(env_step_wave_kernel, dim3(blocks), dim3(TB), step_smem(d), s, d, act, next_obs,
                     next_se > 0 ? next_se : (int64_t)d.N * d.D, next_row, obs_cur, cur_row, rew, done, t, bc);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

const float* env_reset_obs(const mm_env* env) { return env->d.reset_obs; }

}  // namespace mm

extern "C" {
int mm_env_create(const mm_env_cfg* cfg, int64_t n_envs, uint64_t seed, mm_env** out) {
  return mm::env_create(cfg, n_envs, seed, out);
}
void mm_env_destroy(mm_env* env) {
  if (!env) return;
  (void)hipFree(env->alloc);
  delete env;
}
int mm_env_obs_dim(const mm_env* env) { return env ? env->d.D : -1; }
int mm_env_grid_shape(const mm_env* env, int32_t* rows, int32_t* cols) {
  if (!env) return MM_EINVAL;
  *rows = env->d.R;
  *cols = env->d.C;
  return MM_OK;
}
int mm_env_reset(mm_env* env, float* obs, mm_stream_t s) { return mm::env_reset(env, obs, (hipStream_t)s); }
int mm_env_step(mm_env* env, const int32_t* act, float* next_obs, float* obs_cur, float* rew, uint8_t* done,
                mm_stream_t s) {
  return mm::env_step(env, act, next_obs, 0, nullptr, obs_cur, nullptr, rew, done, nullptr, (hipStream_t)s);
}
int mm_env_step_rows(mm_env* env, const int32_t* act, float* next_obs, int64_t next_se, const int64_t* next_row,
                     float* obs_cur, int64_t* cur_row, float* rew, uint8_t* done, mm_stream_t s) {
  return mm::env_step(env, act, next_obs, next_se, next_row, obs_cur, cur_row, rew, done, nullptr, (hipStream_t)s);
}
int mm_env_step_rows_td(mm_env* env, const int32_t* act, float* next_obs, int64_t next_se, const int64_t* next_row,
                        int64_t* cur_row, float* rew, uint8_t* done, float gamma, const float* td_rew,
                        const uint8_t* td_done, const float* q_taken, const float* max_q_next, const int32_t* td_act,
                        float* chunk_td, int32_t step_in_chunk, int32_t chunk_len, uint8_t* store_act,
                        float* store_rew, uint8_t* store_done, const int64_t* td_rows, uint64_t* counter,
                        mm_stream_t s) {
  MM_REQUIRE(td_rew && td_done && q_taken && max_q_next && td_act && chunk_td && store_act && store_rew &&
                 store_done && td_rows, "env_step_rows_td: null TD argument");
  MM_REQUIRE(step_in_chunk >= 0 && step_in_chunk < chunk_len, "env_step_rows_td: bad step");
  mm::TdFuse t{td_rew, td_done, q_taken, max_q_next, td_act, chunk_td, store_act, store_rew, store_done, td_rows,
               counter, gamma, step_in_chunk, chunk_len, 1};
  return mm::env_step(env, act, next_obs, next_se, next_row, nullptr, cur_row, rew, done, &t, (hipStream_t)s);
}
const float* mm_env_reset_obs(const mm_env* env) { return env ? env->d.reset_obs : nullptr; }
int mm_env_step_rows_begin(mm_env* env, const int32_t* act, float* store_obs, int64_t row_stride, int32_t chunk_len,
                           const int64_t* staging, int64_t* cur_row, float* rew, uint8_t* done, mm_stream_t s) {
  MM_REQUIRE(env && store_obs && staging && cur_row && chunk_len >= 1, "env_step_rows_begin: bad arguments");
  const int64_t nd = (int64_t)env->d.N * env->d.D;
  MM_REQUIRE(row_stride >= (chunk_len + 1) * nd, "env_step_rows_begin: row_stride < (chunk_len + 1) * N * D");
  const mm::BeginCopy bc{store_obs, row_stride, chunk_len * nd, env->d.reset_obs, 1};
  return mm::env_step(env, act, store_obs + nd, row_stride, staging, nullptr, cur_row, rew, done, nullptr,
                      (hipStream_t)s, &bc);
}
int mm_env_get_state_buf(mm_env* env, int32_t which, int32_t* pos, int32_t* prev, int8_t* grid, int32_t* steps,
                         int32_t* apples) {
  if (!env || which < 0 || which > 1) return MM_EINVAL;
  const mm::EnvDev& d = env->d;
  const int32_t* dpos = which ? d.pos_alt : d.pos;
  const int8_t* dgrid = which ? d.grid_alt : d.grid;
  if (hipDeviceSynchronize() != hipSuccess) return MM_EHIP;
  std::vector<int32_t> p((size_t)d.E * d.N);
  if (hipMemcpy(p.data(), dpos, p.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return MM_EHIP;
  for (size_t i = 0; i < p.size(); ++i) {
    if (pos) {
      pos[2 * i] = (p[i] >> 8) & 255;
      pos[2 * i + 1] = p[i] & 255;
    }
    if (prev) {
      prev[2 * i] = (p[i] >> 24) & 255;
      prev[2 * i + 1] = (p[i] >> 16) & 255;
    }
  }
  if (grid && hipMemcpy(grid, dgrid, (size_t)d.E * d.R * d.C, hipMemcpyDeviceToHost) != hipSuccess) return MM_EHIP;
  if (steps && hipMemcpy(steps, which ? d.steps_alt : d.steps, (size_t)d.E * 4, hipMemcpyDeviceToHost) != hipSuccess)
    return MM_EHIP;
  if (apples && hipMemcpy(apples, which ? d.apples_alt : d.apples, (size_t)d.E * 4, hipMemcpyDeviceToHost) != hipSuccess)
    return MM_EHIP;
  return MM_OK;
}
int mm_env_get_state(mm_env* env, int32_t* pos, int32_t* prev, int8_t* grid, int32_t* steps, int32_t* apples) {
  return mm_env_get_state_buf(env, 0, pos, prev, grid, steps, apples);
}

int mm_env_set_state_buf(mm_env* env, int32_t which, const int32_t* pos, const int32_t* prev, const int8_t* grid,
                         const int32_t* steps, const int32_t* apples) {
  MM_REQUIRE(env && pos && prev && grid && steps && apples, "env_set_state: null argument");
  MM_REQUIRE(which == 0 || which == 1, "env_set_state: state buffer must be 0 or 1");
  const mm::EnvDev& d = env->d;
  std::vector<int32_t> p((size_t)d.E * d.N);
  for (size_t i = 0; i < p.size(); ++i) {
    MM_REQUIRE(pos[2 * i] >= 0 && pos[2 * i] < d.R && pos[2 * i + 1] >= 0 && pos[2 * i + 1] < d.C &&
                   prev[2 * i] >= 0 && prev[2 * i] < d.R && prev[2 * i + 1] >= 0 && prev[2 * i + 1] < d.C,
               "env_set_state: position out of the grid");
    p[i] = (prev[2 * i] << 24) | (prev[2 * i + 1] << 16) | (pos[2 * i] << 8) | pos[2 * i + 1];
  }
  const size_t RC = (size_t)d.R * d.C;
  for (size_t i = 0; i < (size_t)d.E * RC; ++i)
    MM_REQUIRE(grid[i] >= 0 && grid[i] < 3 + d.N, "env_set_state: grid code out of range");
  MM_HIP_CHECK(hipDeviceSynchronize());
  MM_HIP_CHECK(hipMemcpy(which ? d.pos_alt : d.pos, p.data(), p.size() * 4, hipMemcpyHostToDevice));
  MM_HIP_CHECK(hipMemcpy(which ? d.grid_alt : d.grid, grid, (size_t)d.E * RC, hipMemcpyHostToDevice));
  MM_HIP_CHECK(hipMemcpy(which ? d.steps_alt : d.steps, steps, (size_t)d.E * 4, hipMemcpyHostToDevice));
  MM_HIP_CHECK(hipMemcpy(which ? d.apples_alt : d.apples, apples, (size_t)d.E * 4, hipMemcpyHostToDevice));
  return MM_OK;
}
int mm_env_set_state(mm_env* env, const int32_t* pos, const int32_t* prev, const int8_t* grid, const int32_t* steps,
                     const int32_t* apples) {
  return mm_env_set_state_buf(env, 0, pos, prev, grid, steps, apples);
}
}
