/*
 * minimarl — MI355X-native C ABI for the QMIX / VDN rollout-and-learn hot path.
 *
 * Plain C: raw device pointers, sizes, strides and a hipStream_t passed as
 * void*. Every call enqueues work on that stream and returns immediately (no
 * host synchronisation) unless documented otherwise. Return value: 0 on
 * success, a negative errno-style code otherwise; mm_last_error() gives the
 * message (thread-local). Handles are opaque, created/destroyed in pairs,
 * stream-ordered and not thread-safe per handle.
 *
 * Which reference interface each entry point replaces (reference @ /root/reference):
 *   mm_env_*             gym.make("ma_gym:Checkers-v0") reset/step   vdn/main.py:61-64,83,93,143; qmix/main.py:66-71,189
 *                        (ma_gym checkers.py restated in oracle/env.py)
 *   mm_switch_*          gym.make("ma_gym:Switch2-v0") reset/step    qmix/_config.py:14-19; qmix/main.py:66-71,103-115
 *   mm_agent_q_fwd       Q_Net.forward / sample_action               qmix/_network.py:44-74; vdn/_network.py:52-58,71-88
 *   mm_qnet_*            Q_Net parameters (per-agent Linear/GRUCell)  qmix/_network.py:15-42; vdn/_network.py:32-42,61-69
 *   mm_td_chunk_step     cal_td_error + chunk assembly               vdn/_utils.py:44-52; vdn/main.py:140-167
 *   mm_per_*             Prioritized_Experience_Replay + SumTree     vdn/replay_buffer/{buffer,sumtree}.py; qmix/replay_buffer/{per,sumtree}.py
 *   mm_mixer_fwd         Mix_Net.forward                             qmix/_network.py:199-217
 *   mm_lrn_, mm_..._bwd  Train_dqn.train / Target_Dqn.train          qmix/_train.py:19-121; vdn/_train.py:184-235
 *   mm_mappo_fwd         R_MAPPOPolicy.get_actions/get_values/evaluate_actions  mappo/algorithms/rmappo_policy.py:57-136
 *   mm_mappo_bwd, wgrad  R_MAPPO.ppo_update/cal_value_loss/train     mappo/algorithms/ramppo_network.py:56-287
 *   mm_mappo_grad        (fused: forward recompute + BPTT + weight grads of one epoch, same lines)
 *   mm_mappo_gae, insert SharedReplayBuffer.compute_returns/insert   mappo/runner/shared/shared_buffer.py:82-157
 *   mm_offq_*            offpolicy QMix.train_policy_on_batch etc.   offpolicy/algorithms/qmix/qmix.py:80-226
 *   mm_erb_*             PrioritizedRecReplayBuffer / RecReplayBuffer offpolicy/utils/rec_buffer.py:10-324; segment_tree.py:18-165
 *   mm_eval_accum        greedy test loops                           vdn/_test.py:22-50; magym_runner.py:198-241
 */
#ifndef MINIMARL_H
#define MINIMARL_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* mm_stream_t; /* hipStream_t */

const char* mm_last_error(void);
int mm_version(void);

/* ------------------------------------------------------------------ Q-network */
/* Per-agent (non-shared) Q_Net: Linear(D,F1)+ReLU, Linear(F1,G)+ReLU, GRUCell(G,H), Linear(H,A).
 * Reference sizes: F1=64, G=H=32 (qmix/_network.py:11-13). Supported (F1,G,H):
 * (64,32,32) (64,64,64) (128,32,32) (64,32,64); A <= 64; any D >= 1. */
typedef struct mm_qnet_dims {
  int32_t n_agents, obs_dim, f1, g, h, n_actions;
} mm_qnet_dims;

/* Canonical flat parameter layout (float32): the 10 tensors
 *   W1[N,F1,D] b1[N,F1] W2[N,G,F1] b2[N,G] Wih[N,3H,G] Whh[N,3H,H] bih[N,3H] bhh[N,3H] Wq[N,A,H] bq[N,A]
 * concatenated in that order. offs[0..9] = element offsets, offs[10] = total. */
int mm_qnet_param_offsets(const mm_qnet_dims* d, int64_t offs[11]);
/* Size (floats) of the MFMA-fragment-packed weight images used by mm_agent_q_fwd: the exact-f32
 * fragment image followed by the fp16x3-split image of the large-E (LDS-staged) forward
 * (v_mfma_f32_32x32x16_f16 x3 per product; set MM_FWD_F32=1 to use the f32 MFMA kernel instead). */
int64_t mm_qnet_packed_count(const mm_qnet_dims* d);
/* Repack flat params into the fragment image (call after every optimizer step). */
int mm_qnet_pack(const mm_qnet_dims* d, const float* params, float* packed, mm_stream_t s);
/* Repack only the exact-f32 fragment image (the learner's own forward after an Adam step; ~1/4 of the
 * full pack's time). The fp16x3 image and its safety flags are left stale: call mm_qnet_pack before the
 * next large-E (fp16x3) forward. */
int mm_qnet_pack_f32(const mm_qnet_dims* d, const float* params, float* packed, mm_stream_t s);

enum { MM_Q_NONE = 0, MM_Q_ACT = 1, MM_Q_MAX = 2, MM_Q_GATHER = 3 };

typedef struct mm_qfwd_io {
  /* obs(e, agent, f) = obs[r(e)*obs_se + obs_off + agent*obs_sa + f] with r(e) = e, or r(e) = obs_row[e]
   * when obs_row != NULL (a gather); obs_row[e] < 0 selects reset_obs[agent*obs_sa + f] instead. */
  const float* obs; int64_t obs_se, obs_sa, obs_off;
  const int64_t* obs_row; const float* reset_obs;
  /* hidden in/out: h(e, agent, f) = h[e*se + agent*sa + f*sf]; reset[e] != 0 => h_in treated as 0 */
  const float* h_in; int64_t hin_se, hin_sa, hin_sf;
  float* h_out; int64_t hout_se, hout_sa, hout_sf;
  const uint8_t* reset;
  float* q_out; int64_t q_se, q_sa;                 /* optional Q values [.., A] (unit stride) */
  int32_t mode;                                       /* MM_Q_* */
  /* MM_Q_ACT: epsilon-greedy, one uniform per env row (vdn/_network.py:53). Injected draws if
   * u != NULL (u[E], rand_act[E*N]) else counter RNG(seed, counter, env[, agent]). */
  float epsilon; const float* u; const int32_t* rand_act; uint64_t seed; uint64_t counter;
  int32_t* act_out;                                   /* [E,N] chosen actions (ACT) */
  const int32_t* act_in; int64_t act_se;              /* GATHER: act_in[e*act_se + agent] */
  float* qsel_out;                                    /* [E,N]: Q(a_chosen) (ACT/GATHER) or max_a Q (MAX) */
  /* optional device scalars overriding epsilon / counter (graph-replayable rollouts) */
  const float* eps_ptr; const uint64_t* counter_ptr;
  /* optional training save: per (e, agent) row of SD = F1+G+6H floats
   * [x1 | x2 | h_in | r | z | n | W_hn h + b_hn | h_out] at save + (e*N + agent)*SD */
  float* save;
  /* split forward (mm_agent_q_pre2 / mm_agent_q_rec2): the GRU input projection per (e, agent),
   * [e][agent][3H] = (b_ih + b_hh for r, z | b_ih for n) + W_ih x2 */
  float* gi;
} mm_qfwd_io;

int mm_agent_q_fwd(const mm_qnet_dims* d, const float* packed, const mm_qfwd_io* io, int64_t n_envs,
                   mm_stream_t s);

/* Two nets of the same dims in ONE launch (e.g. target fwd of step t + behavior fwd of step t+1). */
int mm_agent_q_fwd2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t n_envs0,
                    const float* packed1, const mm_qfwd_io* io1, int64_t n_envs1, mm_stream_t s);

/* Split forward for training over a whole chunk batch: PRE runs the non-recurrent part (layers 1-2
 * and W_ih x2, writing io.gi and the x1|x2 save columns) for all E = C*B rows of two nets in one
 * launch; REC runs one recurrent step (W_hh h, gates, Q head, epilogue) reading io.gi. Together
 * bit-identical to mm_agent_q_fwd2 (same MFMA accumulation order). io1 == NULL or n_envs1 == 0: one net. */
int mm_agent_q_pre2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t n_envs0,
                    const float* packed1, const mm_qfwd_io* io1, int64_t n_envs1, mm_stream_t s);
int mm_agent_q_rec2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t n_envs0,
                    const float* packed1, const mm_qfwd_io* io1, int64_t n_envs1, mm_stream_t s);
/* PRE on the fp16x3-split fragment image (the fast mode of large learner batches, QLearner(mixer_fp16=True)):
 * same outputs as mm_agent_q_pre2 within the fp16x3 forward's rtol 1e-5 (not bit-identical); agents flagged by
 * the pack-time range guard run on the exact-f32 image. Reference: qmix/_network.py:44-64 (Q_Net.forward). */
int mm_agent_q_pre2_h3(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t n_envs0,
                       const float* packed1, const mm_qfwd_io* io1, int64_t n_envs1, mm_stream_t s);
/* REC for all `steps` chunk steps in one launch (the W_hh fragments stay in registers, the hidden
 * state in LDS): step t reads io.gi / writes io.save, io.qsel_out and reads io.act_in at the step-0
 * pointers + t * (E*N*3H / E*N*SD / E*N / E*act_se); h_in/h_out are not used (zero start, resets
 * where reset[(t-1)*E + e] for t >= 1). Bit-identical to `steps` mm_agent_q_rec2 launches. */
int mm_agent_q_rec_seq2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t n_envs0,
                        const float* packed1, const mm_qfwd_io* io1, int64_t n_envs1, int32_t steps,
                        const uint8_t* reset, mm_stream_t s);

/* Survey-style convenience entry: contiguous obs [E,N,D], hidden [E,N,H] -> q [E,N,A], h_out [E,N,H]. */
int mm_agent_q_fwd_simple(const mm_qnet_dims* d, const float* packed, const float* obs, const float* h,
                          float* q, float* h_out, int64_t n_envs, mm_stream_t s);

/* ------------------------------------------------------------------ environment */
typedef struct mm_env_cfg {
  int32_t n_agents, max_steps, full_observable, cols;
  float step_cost;
} mm_env_cfg;
typedef struct mm_env mm_env;

int mm_env_create(const mm_env_cfg* cfg, int64_t n_envs, uint64_t seed, mm_env** out);
void mm_env_destroy(mm_env* env);
int mm_env_obs_dim(const mm_env* env);
/* Reset every env; writes obs [E,N,D]. */
int mm_env_reset(mm_env* env, float* obs, mm_stream_t s);
/* Step every env with act [E,N] (int32): writes the (terminal) next obs [E,N,D], rew [E,N],
 * done [E] (env-level, 1 byte). If obs_cur != NULL the env also auto-resets done envs and writes
 * the next CURRENT obs (reset obs where done) into obs_cur; otherwise done envs stay terminal. */
int mm_env_step(mm_env* env, const int32_t* act, float* next_obs, float* obs_cur, float* rew,
                uint8_t* done, mm_stream_t s);
/* Copy out the integer state (for parity tests): pos / prev [E,N,2] int32 (ma_gym's agent_pos /
 * agent_prev_pos), grid [E,R,C] int8 (_full_obs: 0 empty, 1 lemon, 2 apple, 3 + k agent k's marker),
 * steps [E], apples [E]; host pointers, synchronous. */
int mm_env_get_state(mm_env* env, int32_t* pos, int32_t* prev, int8_t* grid, int32_t* steps, int32_t* apples);
/* Restore the integer state written by mm_env_get_state (checkpoint resume; host pointers, synchronous). */
int mm_env_set_state(mm_env* env, const int32_t* pos, const int32_t* prev, const int8_t* grid, const int32_t* steps,
                     const int32_t* apples);
int mm_env_grid_shape(const mm_env* env, int32_t* rows, int32_t* cols);
/* The same for one of the two state buffers of the fused rollout step (mm_rollout_step reads buffer
 * state_in = t % 2 and writes the other): which = 0 is the buffer the env kernels use. */
int mm_env_get_state_buf(mm_env* env, int32_t which, int32_t* pos, int32_t* prev, int8_t* grid, int32_t* steps,
                         int32_t* apples);
int mm_env_set_state_buf(mm_env* env, int32_t which, const int32_t* pos, const int32_t* prev, const int8_t* grid,
                         const int32_t* steps, const int32_t* apples);

/* ------------------------------------------------------------------ TD error + chunk store */
/* One rollout step for E envs: td = |sum_i r_i + (1-done)*gamma*sum_i maxq'_i - sum_i q_taken_i|
 * (vdn/_utils.py:44-52), accumulated into chunk_td[E]; and the transition is written into the
 * device chunk store at slot t = step_in_chunk of chunk row chunk_base+e:
 *   act8[row, t, N] (uint8), rew[row, t, N] (f32), done[row, t] (uint8)
 * obs are written by the env kernel directly into the store. */
int mm_td_chunk_step(int64_t n_envs, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                     const float* q_taken, const float* max_q_next, const int32_t* act, float* chunk_td,
                     int32_t step_in_chunk, int32_t chunk_len, uint8_t* store_act, float* store_rew,
                     uint8_t* store_done, int64_t store_row0, mm_stream_t s);

/* Greedy-evaluation episode accumulators (vdn/_test.py:22-50, qmix/_test.py:19-36): for envs still
 * active, score[e] += sum_i rew; if q_taken and max_q_next are given, loss[e] += td^2 (cal_td_error);
 * done[e] deactivates the env. */
int mm_eval_accum(int64_t n_envs, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                  const float* q_taken, const float* max_q_next, uint8_t* active, float* score, float* loss,
                  mm_stream_t s);
/* Training score of the rollout (vdn/main.py:173, qmix/main.py:247 train score = the episode's summed
 * reward): walks the chunk just stored in rows[e] (store rew [rows, C, N], done [rows, C]), carries the
 * running episode return ep_ret[e] and adds each finished episode's return / count to acc[0] / acc[1]
 * (f64). Replaces the reference's per-step Python ``score += sum(reward)``. */
int mm_chunk_score(int64_t n_envs, int32_t chunk, int32_t n_agents, const float* store_rew,
                   const uint8_t* store_done, const int64_t* rows, float* ep_ret, double* acc, mm_stream_t s);

/* ------------------------------------------------------------------ prioritized replay */
enum { MM_PER_VDN = 0, MM_PER_QMIX = 1 };
typedef struct mm_per mm_per;
int mm_per_create(int64_t capacity, int32_t flavor, double alpha, double beta, double eps, double step_weight,
                  int32_t use_step_weight, double alpha_inc, double beta_inc, mm_per** out);
void mm_per_destroy(mm_per* per);
/* Insert K chunks with rollout td sums td[K] (device f32): free slots first, then the K lowest
 * leaves are replaced; slots_out[K] (device int64) receives the data slot of each insert. */
int mm_per_add_batch(mm_per* per, const float* td, int64_t k, int64_t* slots_out, mm_stream_t s);
/* Stratified sample of B leaves with injected fractions fracs[B] (device f64, in [0,1)):
 * nodes_out / slots_out (device int64), is_w (device f32). Anneals alpha/beta first. */
int mm_per_sample(mm_per* per, int32_t batch, const double* fracs, int64_t* nodes_out, int64_t* slots_out,
                  float* is_w, mm_stream_t s);
/* Same with device-generated fractions from a counter RNG. */
int mm_per_sample_rng(mm_per* per, int32_t batch, uint64_t seed, uint64_t counter, int64_t* nodes_out,
                      int64_t* slots_out, float* is_w, mm_stream_t s);
/* Uniform replay of whole stored chunks (the minimal QMIX's ReplayBuffer.sample_chunk,
 * qmix/qmix.py:19-46, draws uniformly): B slots uniform over the filled slots (device counter RNG,
 * a fresh stream per call), is_w (may be NULL) = 1. Priorities are not read. */
int mm_per_sample_uniform(mm_per* per, int32_t batch, uint64_t seed, uint64_t counter, int64_t* slots_out,
                          float* is_w, mm_stream_t s);
/* Priority update leaf(nodes[b]) = (td[b]+eps)^alpha; duplicate nodes: last sample index wins. */
int mm_per_update(mm_per* per, const int64_t* nodes, const float* td, int32_t batch, mm_stream_t s);
double* mm_per_tree_ptr(mm_per* per);               /* device f64 [2*cap-1] */
int64_t mm_per_size(const mm_per* per);
double mm_per_alpha(const mm_per* per);
double mm_per_beta(const mm_per* per);

/* ------------------------------------------------------------------ rollout engine plumbing
 * (the device chunk store of mini-marl_amd/minimarl/engine.py; replaces the per-step Python chunk
 *  lists of vdn/main.py:140-167 / qmix/main.py:186-237) */
/* Step with destination rows: the terminal next obs of env e goes to next_obs + next_row[e]*next_se
 * (NULL next_obs: not written); obs_cur (may be NULL) gets the auto-reset current obs; cur_row (may be
 * NULL) gets next_row[e], or -1 where the env finished and was reset. Auto-reset happens when either
 * obs_cur or cur_row is given. */
int mm_env_step_rows(mm_env* env, const int32_t* act, float* next_obs, int64_t next_se, const int64_t* next_row,
                     float* obs_cur, int64_t* cur_row, float* rew, uint8_t* done, mm_stream_t s);
const float* mm_env_reset_obs(const mm_env* env); /* device [N, D]: the (deterministic) reset obs */
/* The rollout engine's chunk-start step: mm_chunk_begin_rows + mm_env_step_rows in ONE launch. Store rows
 * are row_stride floats, chunk_len + 1 obs slots of N*D floats. Slot 0 of row staging[e] <- slot chunk_len
 * of row cur_row[e] (the previous chunk's last next obs), or the reset obs where cur_row[e] < 0; then the
 * step: next obs into slot 1 of row staging[e], cur_row[e] <- staging[e] (or -1 where the env finished). */
int mm_env_step_rows_begin(mm_env* env, const int32_t* act, float* store_obs, int64_t row_stride, int32_t chunk_len,
                           const int64_t* staging, int64_t* cur_row, float* rew, uint8_t* done, mm_stream_t s);
/* mm_env_step_rows (auto-reset via cur_row, no obs_cur) fused with mm_td_chunk_step_rows of the
 * PREVIOUS step (td_* inputs, slot step_in_chunk of store rows td_rows): one launch instead of two
 * for every in-chunk step of the rollout engine (cal_td_error + chunk lists, vdn/_utils.py:44-52,
 * vdn/main.py:140-167). Identical results to the two separate calls. */
int mm_env_step_rows_td(mm_env* env, const int32_t* act, float* next_obs, int64_t next_se, const int64_t* next_row,
                        int64_t* cur_row, float* rew, uint8_t* done, float gamma, const float* td_rew,
                        const uint8_t* td_done, const float* q_taken, const float* max_q_next, const int32_t* td_act,
                        float* chunk_td, int32_t step_in_chunk, int32_t chunk_len, uint8_t* store_act,
                        float* store_rew, uint8_t* store_done, const int64_t* td_rows, uint64_t* counter,
                        mm_stream_t s);
/* ONE launch per rollout step (replaces the per-step loop body of vdn/main.py:93-167 / qmix/main.py:186-233:
 * env.step, the chunk-list append, the target max_a Q' of the next obs and sample_action of the next step):
 * the env step of step t (mm_env_step_rows_td / _begin semantics) fused into the dual forward of
 * mm_agent_q_fwd2 (target net io_t on s'_t, mode MAX; behavior net io_b on s_{t+1}, mode ACT). Results are
 * bit-identical to the two-launch step. The observations never touch HBM on the way in: every block steps
 * its env tile itself and builds its agent's obs from the grid in LDS. Double-buffered state: the env state
 * buffer state_in (= t % 2, see mm_env_get_state_buf) is read and the other written; counter[state_in] is
 * the behavior net's RNG step counter and counter[1 - state_in] = counter[state_in] + 1 is written; rew /
 * done / io_t.qsel_out must not alias the td_* inputs of the previous step, nor io_b.act_out / qsel_out
 * the act of this step or td_act / td_qsel (a ring of 3). io_b.reset must be NULL (the behavior hidden
 * state resets where this step's env finished). Supported when mm_rollout_step_supported() != 0. */
typedef struct mm_rollout_step_io {
  const int32_t* act;                 /* [E,N] actions of step t */
  float* store_obs; int64_t row_stride; int32_t slot, chunk_len;   /* s'_t -> slot (= step_in_chunk + 1) of row staging[e] */
  int32_t begin;                      /* chunk start: also s_t -> slot 0 of row staging[e] */
  const int64_t* staging; int64_t* cur_row;
  float* rew; uint8_t* done;          /* [E,N] rewards, [E] done of step t */
  int32_t state_in;                   /* env state buffer read (0 / 1) */
  uint64_t* counter;                  /* [2] device RNG step counter */
  /* TD / store of the previous step (mm_td_chunk_step_rows semantics, slot td_slot of rows staging[e]; the
   * RNG counter is not touched) when td_on */
  int32_t td_on, td_slot; float gamma;
  const float* td_rew; const uint8_t* td_done; const float* td_qsel; const float* td_maxq; const int32_t* td_act;
  float* chunk_td; uint8_t* store_act; float* store_rew; uint8_t* store_done;
  /* guard rail: rows of the chunk store; a staging row outside [0, n_rows) is never written through (its env's
   * stores are skipped) and sets bit 0 of *err (device int32, sticky; may be NULL) */
  int64_t n_rows; int32_t* err;
} mm_rollout_step_io;
/* 1 when the fused step fits: local obs, 8 grid columns and an even row count (4 or 8 agents), E >= 2048, one of
 * the compiled layer widths, LDS budget; 0 otherwise (use the two-launch step). */
int mm_rollout_step_supported(const mm_env* env, const mm_qnet_dims* d, int64_t n_envs);
int mm_rollout_step(mm_env* env, const mm_qnet_dims* d, const float* packed_t, const mm_qfwd_io* io_t,
                    const float* packed_b, const mm_qfwd_io* io_b, int64_t n_envs, const mm_rollout_step_io* x,
                    mm_stream_t s);
/* The rollout steps t0 .. t0 + n_steps - 1 (chunk position c0 = t0 % chunk_len) in ONE launch (chunk-persistent; replaces
 * n_steps iterations of the reference's per-step loop body, vdn/main.py:93-167 / qmix/main.py:186-233, like n_steps
 * mm_rollout_step calls, with bit-identical results): every (net, agent, 256-env tile) block stays resident for all
 * the steps, keeps its weight image and its copy of the tile's env state in LDS, and waits only for the tile's
 * behavior actions of each step (a tile-local hand-off through tagged handoff words), never for a launch boundary.
 * A launch may cross chunk boundaries: its k-th chunk (k = 0 .. n_sets - 1) writes staging row set (set0 + k) %
 * n_sets of staging [n_sets][E] (s'_t into slot c + 1 and, at a chunk start, s_t into slot 0 of row staging[set][e]),
 * so the chunks' PER inserts can all run after the launch (each insert swaps its own set's rows). Per-step outputs
 * live in rings of ring_len steps, launch step i at ring position p = (ring_pos + i) % ring_len: rewards at rew +
 * p E N, dones at done + p E, the target's max Q' at io_t->qsel_out + p E N, the behavior's act / Q(a) of the NEXT
 * step at io_b->act_out / qsel_out + ((p + 1) % ring_len) E N (so n_steps < ring_len); cur_row per env. act0 holds
 * the actions of step t0, done_prev the dones of step t0 - 1. Hidden states are updated in place (h_in == h_out,
 * io.reset NULL). The TD / chunk-store fold of the steps is mm_td_fold_range / mm_per_insert_fold per chunk. ctl =
 * device int64 [3]: launch sequence, env state buffer (low int32 of ctl[1], read; flipped by each launch: see
 * mm_env_get_state_buf), arrival ticket — zero-initialised once, then owned by these launches.
 * handoff = int64 [T][handoff_len][N][32], T = ceil(E / 256), handoff_len >= n_steps, zero-initialised: word w of
 * (tile, launch step, agent) = (low 32 bits of the launch sequence + 1) << 32 | the 4-bit actions of the tile's envs
 * 8 w .. 8 w + 7. Supported when mm_rollout_chunk_supported() != 0 (the fused step's geometry and 2 N T blocks <= the
 * device's CUs: all blocks must be co-resident; a hand-off wait longer than 20 ms sets bit 1 of *err and proceeds). */
typedef struct mm_rollout_chunk_io {
  float* store_obs; int64_t row_stride; int64_t n_rows;
  const int64_t* staging; int64_t* cur_row;
  int32_t c0, n_steps, chunk_len, n_sets;
  int32_t set0, ring_len, ring_pos, handoff_len;
  const int32_t* act0; const uint8_t* done_prev;
  float* rew; uint8_t* done;
  int64_t* counter;      /* device RNG step counter: step t0 + i draws with *counter + i; += n_steps */
  int64_t* ctl;          /* device int64 [3]: launch sequence, env state buffer (low int32), arrival ticket */
  int64_t* handoff;
  int32_t* err;
} mm_rollout_chunk_io;
int mm_rollout_chunk_supported(const mm_env* env, const mm_qnet_dims* d, int64_t n_envs);
int mm_rollout_chunk(mm_env* env, const mm_qnet_dims* d, const float* packed_t, const mm_qfwd_io* io_t,
                     const float* packed_b, const mm_qfwd_io* io_b, int64_t n_envs, const mm_rollout_chunk_io* x,
                     mm_stream_t s);
/* Co-residency contract of mm_rollout_chunk: NOTHING else may run on the device while it runs (no kernel on another
 * stream, no collective, no other process's work), because its blocks wait for each other's hand-off words. A launch
 * that was not fully co-resident completes (every wait expires after 20 ms) with bit 1 of *err set: its rollout data
 * is then invalid and the caller must stop (RolloutEngine.check_errors raises); while the bit is set, mm_td_fold_range
 * and mm_per_insert_fold (multi-block insert, power-of-two capacity >= 16384) fold and insert nothing, so no data of
 * such a launch reaches the chunk store's act / rew / done rows or the PER. Keep collectives stream-ordered on the
 * rollout stream, or outside the rollout's graph launches.
 * Diagnostic for that path: mm_hold_cus occupies n_blocks CUs (one 1024-thread workgroup with 64 KiB of LDS each) for
 * `ticks` of the 100 MHz clock; *seen (device int32) |= 2 if one of the n_watch handoff words carries `tag` in its
 * high 32 bits when a workgroup starts, |= 1 if one does when it ends (1 alone: a chunk launch ran beside it). */
int mm_hold_cus(int32_t n_blocks, int64_t ticks, const int64_t* watch, int64_t n_watch, uint32_t tag, int32_t* seen,
                mm_stream_t s);
/* Large-batch learner kernel shapes (process-wide, default 1 / 1): at B >= 512 the mixer forward and its recurrence
 * backward run 8 samples per block and the agent backward 8 samples per wave; 0 selects the one-sample kernels
 * (identical results, slower). */
int mm_learner_set_multi_sample(int32_t mixer, int32_t agent_bwd);
/* The TD / chunk-store fold of n_slots consecutive rollout steps slot0 .. slot0 + n_slots - 1 of a chunk (what
 * n_slots mm_td_chunk_step_rows calls do, identical results; cal_td_error + the chunk lists, vdn/_utils.py:44-52,
 * vdn/main.py:140-167): step j's rew / q_taken / max_q_next / act at + j ring_se elements, done at + j n_envs; rows
 * outside [0, n_rows) are skipped and set bit 0 of *err (may be NULL). Any span length (groups of 16 slots). */
int mm_td_fold_range(int64_t n_envs, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                     const float* q_taken, const float* max_q_next, const int32_t* act, int64_t ring_se,
                     int32_t slot0, int32_t n_slots, int32_t chunk_len, float* chunk_td, uint8_t* store_act,
                     float* store_rew, uint8_t* store_done, const int64_t* rows, int64_t n_rows, int32_t* err,
                     mm_stream_t s);
/* TD step writing into store rows rows[e]; increments the device RNG step counter (may be NULL). */
int mm_td_chunk_step_rows(int64_t n_envs, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                          const float* q_taken, const float* max_q_next, const int32_t* act, float* chunk_td,
                          int32_t step_in_chunk, int32_t chunk_len, uint8_t* store_act, float* store_rew,
                          uint8_t* store_done, const int64_t* rows, uint64_t* counter, mm_stream_t s);
/* Slot 0 of each staging row: obs_cur[e] (mm_chunk_begin) or, without materialising the current obs,
 * slot src_off of row src_rows[e] / the reset obs where src_rows[e] < 0 (mm_chunk_begin_rows). */
int mm_chunk_begin(int64_t n_envs, int32_t nd, const float* obs_cur, float* store_obs, int64_t row_stride,
                   const int64_t* rows, mm_stream_t s);
int mm_chunk_begin_rows(int64_t n_envs, int32_t nd, float* store_obs, int64_t row_stride, const int64_t* src_rows,
                        int64_t src_off, const float* reset_obs, const int64_t* dst_rows, mm_stream_t s);
/* PER insert with store-row indirection: slot_row[slot] <-> rows_inout[j] (the evicted row is handed
 * back as the next staging row; chunk data is never copied). */
int mm_per_insert(mm_per* per, const float* td, int64_t k, int64_t* rows_inout, int64_t* slots_out, mm_stream_t s);
/* mm_td_fold_range of the chunk's last span (slot0 + n_slots == chunk_len) followed by mm_per_insert(per, chunk_td, k,
 * rows_inout = the staging rows, slots_out), with the fold's workgroups beside the insert's first histogram pass in ONE
 * launch (the chunk-persistent rollout's chunk end; same results as the two calls). */
int mm_per_insert_fold(mm_per* per, int64_t k, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                       const float* q_taken, const float* max_q_next, const int32_t* act, int64_t ring_se,
                       int32_t slot0, int32_t n_slots, int32_t chunk_len, float* chunk_td, uint8_t* store_act,
                       float* store_rew, uint8_t* store_done, int64_t* rows_inout, int64_t n_rows, int32_t* err,
                       int64_t* slots_out, mm_stream_t s);
/* The chunk's last rollout step: mm_td_chunk_step_rows of the k envs (slot step_in_chunk of store rows
 * rows_inout, before the swap) followed by mm_per_insert(per, chunk_td, k, rows_inout, slots_out). For the
 * multi-block insert (power-of-two capacity >= 16384) the TD / store runs inside the insert's first launch
 * (one launch fewer); results identical to the two separate calls. */
int mm_per_insert_td(mm_per* per, int64_t k, int32_t n_agents, float gamma, const float* rew, const uint8_t* done,
                     const float* q_taken, const float* max_q_next, const int32_t* act, float* chunk_td,
                     int32_t step_in_chunk, int32_t chunk_len, uint8_t* store_act, float* store_rew,
                     uint8_t* store_done, uint64_t* counter, int64_t* rows_inout, int64_t* slots_out, mm_stream_t s);
int64_t* mm_per_slot_rows(mm_per* per);             /* device int64 [cap] */
int64_t mm_per_capacity(const mm_per* per);
void mm_per_set_size(mm_per* per, int64_t n);      /* host + device fill count (synchronous) */
void mm_per_set_size_host(mm_per* per, int64_t n); /* host mirror only (graph-replayed inserts) */
int mm_per_copy_tree(mm_per* per, double* dst, mm_stream_t s);
int mm_per_copy_slot_rows(mm_per* per, int64_t* dst, mm_stream_t s);
/* Sticky device error bits of the PER (1 = an mm_per_update node outside the leaf range was skipped);
 * synchronous; clear != 0 resets them. Replaces the IndexError / silent internal-node write of the
 * reference's `self.tree[idx] = p` (vdn/replay_buffer/sumtree.py update) for bad indices. */
int mm_per_error_word(mm_per* per, int32_t* host_out, int32_t clear, mm_stream_t s);
/* Checkpoint state of the replay: tree (device f64 [2cap-1]) and slot -> row map (device i64 [cap])
 * copied stream-ordered; scalars[6] (host) = fill count, alpha, beta, alpha_inc, beta_inc, sample-call
 * counter (the device RNG stream index). Both calls synchronise the stream (the scalars cross PCIe). */
int mm_per_save_state(mm_per* per, double* tree_dst, int64_t* rows_dst, double* scalars, mm_stream_t s);
int mm_per_load_state(mm_per* per, const double* tree_src, const int64_t* rows_src, const double* scalars,
                      mm_stream_t s);

/* ------------------------------------------------------------------ QMIX / VDN learner
 * (Train_dqn.train qmix/_train.py:19-121, Target_Dqn.train vdn/_train.py:184-235; orchestrated by
 *  mini-marl_amd/minimarl/learner.py). Mixer = Mix_Net (qmix/_network.py:172-217). */
int mm_mixer_param_count(int32_t state_dim, int32_t hm, int32_t k1, int32_t n_agents, int64_t* count);
int mm_mixer_save_dim(int32_t hm, int32_t k1, int32_t n_agents);
int mm_mixer_delta_dim(int32_t hm, int32_t k1, int32_t n_agents);
/* Gather B sampled chunks (PER slots -> store rows): obs offsets, acts, rewards, dones. */
int mm_lrn_gather(int32_t B, int32_t C, int32_t N, int64_t row_stride, int64_t nd, const int64_t* slots,
                  const int64_t* slot_row, const uint8_t* s_done, const uint8_t* s_act, const float* s_rew,
                  int64_t* s_off, int64_t* s2_off, int32_t* acts, float* rew, float* done, uint8_t* done8,
                  mm_stream_t s);
typedef struct mm_mix_net {
  const float* P;
  const float* gi;  /* [B, 3Hm] precomputed input projection of this step (mm_mixer_gi) or NULL */
  const float* q; const int64_t* s_off; const float* h_in; const uint8_t* reset;
  float* h_out; float* qtot; float* save;
} mm_mix_net;
/* Mixer GRU input projection W_ih s + b_ih for all R = C*B gathered states of 1-2 nets at once. */
int mm_mixer_gi(int32_t R, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* obs, const float* reset_obs,
                const float* P0, const int64_t* s_off0, float* gi0, const float* P1, const int64_t* s_off1, float* gi1,
                mm_stream_t s);
/* cfg5 fp16 mode of mm_mixer_gi (rtol 2e-3 on Q_tot, stated apart from the fp32 parity): the
 * same projection on v_mfma_f32_32x32x16_f16 (state and W_ih rounded to f16, fp32 accumulate and bias);
 * Hm in {32, 64}. */
int mm_mixer_gi_f16(int32_t R, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* obs, const float* reset_obs,
                    const float* P0, const int64_t* s_off0, float* gi0, const float* P1, const int64_t* s_off1,
                    float* gi1, mm_stream_t s);
/* One mixer time step for 1-2 nets (behavior / target) in one launch. */
/* Chunk-sequence mixer backward: all C steps (t = C-1 .. 0) in one launch, a block per sample
 * carrying dhm. Step t reads save [C][B][MSD], qa [C][B][N], dq [C][B] and writes dqa [C][B][N],
 * delta [C][B][MDD] at the step-0 pointers + t * (per-step size); the future gradient is dropped at
 * t = C-1 (ones) and where done[t*B + b]. Bit-identical to C mm_mixer_bwd launches.
 * ws: [C][B][4][Hm] floats of workspace (B < 512: the hypernet input gradients of every step are
 * computed for all rows at once, then one block per sample runs the serial GRU chain); may be NULL
 * (then the single-launch LDS kernel runs). */
/* All C steps of the mixer forward for both nets (B < 512): a serial launch with block = (sample, net),
 * the net's W_hh staged once into LDS and the mixer hidden carried in LDS, then the hypernets. Step t's arrays
 * are at the step-0 pointers of nets[] + t * (B x width): gi [B][3Hm] (required, mm_mixer_gi), q [B][N],
 * qtot [B], save [B][mm_mixer_save_dim]; h_out [C][B][Hm] receives the hidden sequence (required: the
 * serial GRU kernel writes it, then one launch runs the hypernets of all C*B rows); step 0 starts
 * from nets[].h_in / reset, step t >= 1 resets where reset_steps[(t-1)*B + b]. Results are
 * bit-identical to C per-step mm_mixer_fwd launches. mm_mixer_fwd_seq_fits tells whether it applies. */
int mm_mixer_fwd_seq_fits(int32_t B, int32_t N, int32_t Hm, int32_t K1);
int mm_mixer_fwd_seq(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const mm_mix_net* nets,
                     int32_t n_nets, int32_t steps, const uint8_t* reset_steps, mm_stream_t s);
/* The split halves of mm_mixer_fwd_seq / mm_mixer_bwd_seq (same arguments), so the mixer's own recurrence can
 * run on a second stream beside the agent chain (Train_dqn.train, qmix/_train.py:55-116: the Mix_Net GRU over
 * the state needs no agent Q; its backward needs only the hypernet pass's dhm): fwd_seq_rec -> [join with the
 * agent forward] -> fwd_seq_hyper; bwd_seq_hyper -> {bwd_seq_rec || agent BPTT}. Only where
 * mm_mixer_seq_split(B, N, S, Hm, K1, P, ws, steps) != 0 (else MM_EINVAL). */
int mm_mixer_fwd_seq_rec(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const mm_mix_net* nets,
                         int32_t n_nets, int32_t steps, const uint8_t* reset_steps, mm_stream_t s);
int mm_mixer_fwd_seq_hyper(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const mm_mix_net* nets,
                           int32_t n_nets, int32_t steps, const uint8_t* reset_steps, mm_stream_t s);
int mm_mixer_bwd_seq_hyper(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* save,
                           const float* qa, const float* dq, const float* done, const float* ones, float* dhm,
                           float* dqa, float* delta, float* ws, int32_t steps, mm_stream_t s);
/* mm_mixer_bwd_seq_hyper, then mm_per_update(per, nodes, td, batch): the small priority update rides as one more
 * block of the hypernet launch (its TDs come from the loss before it; Train_dqn's priority update,
 * qmix/main.py:240-244). Results identical to the two calls. */
int mm_mixer_bwd_seq_hyper_per(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P,
                               const float* save, const float* qa, const float* dq, const float* done,
                               const float* ones, float* dhm, float* dqa, float* delta, float* ws, int32_t steps,
                               mm_per* per, const int64_t* nodes, const float* td, int32_t batch, mm_stream_t s);
int mm_mixer_bwd_seq_rec(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* save,
                         const float* qa, const float* dq, const float* done, const float* ones, float* dhm, float* dqa,
                         float* delta, float* ws, int32_t steps, mm_stream_t s);
int mm_mixer_seq_split(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* ws,
                       int32_t steps);
/* The learner forward's two independent chains in shared grids (no stream fork / join in the update graph), each
 * block running the separate kernel's body, so results are identical to the separate calls:
 *   mm_agent_mixer_pre     = mm_mixer_gi(R = rows, both mixers) + mm_agent_q_pre2(both nets, rows rows each)
 *   mm_agent_mixer_rec_seq = mm_mixer_fwd_seq_rec(B, nets[2], steps, reset_steps)
 *                            + mm_agent_q_rec_seq2(both nets, B envs each, steps, reset)
 * (Train_dqn.train's forward, qmix/_train.py:55-77). mm_agent_mixer_pair_supported returns bit 0 when the pre pair
 * applies to (dims, B x steps rows), bit 1 when the recurrence pair does; outside them both return MM_EINVAL. */
int mm_agent_mixer_pair_supported(const mm_qnet_dims* d, int32_t B, int32_t steps, int32_t N, int32_t S, int32_t Hm,
                                  int32_t K1);
int mm_agent_mixer_pre(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, const float* packed1,
                       const mm_qfwd_io* io1, int64_t rows, int32_t N, int32_t S, int32_t Hm, int32_t K1,
                       const float* obs, const float* reset_obs, const float* mP0, const int64_t* s_off0, float* gi0,
                       const float* mP1, const int64_t* s_off1, float* gi1, mm_stream_t s);
int mm_agent_mixer_rec_seq(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, const float* packed1,
                           const mm_qfwd_io* io1, int32_t B, int32_t steps, const uint8_t* reset, int32_t N,
                           int32_t S, int32_t Hm, int32_t K1, const mm_mix_net* nets, int32_t n_nets,
                           const uint8_t* reset_steps, mm_stream_t s);
int mm_mixer_bwd_seq(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* save,
                     const float* qa, const float* dq, const float* done, const float* ones, float* dhm, float* dqa,
                     float* delta, float* ws, int32_t steps, mm_stream_t s);
int mm_mixer_fwd(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* obs, const float* reset_obs,
                 const mm_mix_net* nets, int32_t n_nets, mm_stream_t s);
/* TD loss terms and their gradient seeds (reference quirks: bootstrap x N, IS weight on the target). */
/* Loss variants for mm_lrn_loss_ex (flags, OR-ed):
 *   MM_LOSS_MIX_SUM     Q_tot = sum_i Q_i (VDN, vdn/_train.py:23-47)
 *   MM_LOSS_HUBER       smooth_l1 (beta 1) instead of MSE (qmix/qmix.py:218)
 *   MM_LOSS_TARGET_SUM  y = sum_i r_i + gamma*(1-d)*Q'_tot, no IS weight (qmix/qmix.py:215-217)
 * (0 = Train_dqn: y = w * sum_i (r_i + gamma*(1-d)*Q'_tot), MSE, qmix/_train.py:80-82). */
enum { MM_LOSS_MIX_SUM = 1, MM_LOSS_HUBER = 2, MM_LOSS_TARGET_SUM = 4 };
int mm_lrn_loss_ex(int32_t B, int32_t C, int32_t N, float gamma, const float* rew, const float* done,
                   const float* isw, const float* qtot, const float* qtot_t, int32_t flags, const float* qa,
                   const float* maxq, float* dq, float* dqa, float* loss_parts, float* td_last, float* loss,
                   mm_stream_t s);
int mm_lrn_loss(int32_t B, int32_t C, int32_t N, float gamma, const float* rew, const float* done, const float* isw,
                const float* qtot, const float* qtot_t, int32_t mix_sum, const float* qa, const float* maxq,
                float* dq, float* dqa, float* loss_parts, float* td_last, float* loss, mm_stream_t s);
int mm_mixer_bwd(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* save,
                 const float* qa, const float* dq, const float* done, float* dhm, float* dqa, float* delta,
                 mm_stream_t s);
/* Mixer weight gradients of R rows from the backward's delta [R][mm_mixer_delta_dim] and the forward's save
 * [R][mm_mixer_save_dim]: every Mix_Net parameter's gradient written into dP (the mixer's flat gradient, MIX_KEYS
 * order) by one batched outer-reduce launch + a fixed-order partial sum. States: rows gathered through s_off
 * (reset_obs for -1), or contiguous [R][S] when s_off is NULL. partial: mm_mixer_wgrad_partial_count floats. */
int64_t mm_mixer_wgrad_partial_count(int32_t R, int32_t N, int32_t S, int32_t Hm, int32_t K1);
int mm_mixer_wgrad(int32_t R, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* state, const int64_t* s_off,
                   const float* reset_obs, const float* save, const float* delta, float* dP, float* partial,
                   int64_t partial_count, mm_stream_t s);
/* VDN mixing (vdn/_train.py:23-47, 68-71): out[b] = sum_i q[b,i,act[b,i]], or sum_i max_a q[b,i,a] when act is
 * NULL; q rows at b*q_se + i*q_sa (unit action stride). An action outside [0, A) adds 0 and sets bit 0 of *err
 * (err may be NULL). */
int mm_vdn_sum(int64_t B, int32_t N, int32_t A, const float* q, int64_t q_se, int64_t q_sa, const int32_t* act,
               float* out, int32_t* err, mm_stream_t s);
/* All C steps of the agent BPTT chain in one launch (small batches): step t's arrays at the step-0 pointers
 * + t x (B x N x width) (save, acts, dqa, dgi, dgh, dq); done of step t < C-1 at done + t*B, step C-1
 * uses ones; dh carries the hidden gradient (in: zero, out: grad wrt the chunk-start hidden).
 * Bit-identical to C per-step mm_agent_bwd launches. */
/* mm_agent_bwd_seq and the mixer recurrence's backward (mm_mixer_bwd_seq_rec with the same B, done, ones, dqa and
 * steps; S, Hm, K1, mP .. ws its mixer arguments) in ONE launch: the two chains are independent and share the grid
 * (agent blocks first); results identical to the two calls. Needs the split mixer path (mm_mixer_seq_split). */
int mm_agent_mixer_bwd_seq(const mm_qnet_dims* d, const float* P, int64_t oWq, int64_t oWhh, int32_t B,
                           const float* save, const int32_t* acts, const float* dqa, const float* done,
                           const float* ones, float* dh, float* dgi, float* dgh, float* dq, int32_t steps, int32_t S,
                           int32_t Hm, int32_t K1, const float* mP, const float* msave, const float* qa,
                           const float* mdq, float* dhm, float* mdelta, float* ws, mm_stream_t s);
int mm_agent_bwd_seq(const mm_qnet_dims* d, const float* P, int64_t oWq, int64_t oWhh, int32_t B, const float* save,
                     const int32_t* acts, const float* dqa, const float* done, const float* ones, float* dh,
                     float* dgi, float* dgh, float* dq, int32_t steps, mm_stream_t s);
int mm_agent_bwd(const mm_qnet_dims* d, const float* P, int64_t oWq, int64_t oWhh, int32_t B, const float* save,
                 const int32_t* acts, const float* dqa, const float* done, float* dh, float* dgi, float* dgh,
                 float* dq, mm_stream_t s);
/* Batched outer-product weight gradients dW[g] (+)= sum_r U[g,r,:]^T V[g,r,:] (+ db). */
typedef struct mm_outer_args {
  const float* U; int64_t u_g, u_m;
  const float* V; int64_t v_g, v_m; const int64_t* v_off; const float* v_reset;
  float* dW; int64_t w_g;
  float* db; int64_t b_g;
  int32_t M, R, Cc, accumulate, groups;
} mm_outer_args;
int mm_outer_reduce(const mm_outer_args* x, mm_stream_t s);
/* Up to 16 independent outer-reduce jobs in one launch (M split into 32-row slices, partials summed
 * in fixed order by a second launch: deterministic). partial: device floats, size from
 * mm_outer_reduce_batch_partial(jobs, n). */
int64_t mm_outer_reduce_batch_partial(const mm_outer_args* x, int32_t n_jobs);
int mm_outer_reduce_batch(const mm_outer_args* x, int32_t n_jobs, float* partial, int64_t partial_count,
                          mm_stream_t s);
/* The same reduction with every product as a bf16x3 split on v_mfma_f32_32x32x16_bf16 (~2^-16 relative per
 * product, fp32 exponent range): the learner's fast mode (QLearner(mixer_fp16=True) at C*B >= 2048). */
int mm_outer_reduce_batch_bf3(const mm_outer_args* x, int32_t n_jobs, float* partial, int64_t partial_count,
                              mm_stream_t s);
/* Batched (gated) transposed mat-vec Y[g] = (W[g]^T X[g]) * Z[g]. */
typedef struct mm_tmv_args {
  const float* W; int64_t w_g;
  const float* X; int64_t x_g, x_m;
  const float* Z; int64_t z_g, z_m;
  float* Y; int64_t y_g, y_m;
  int32_t M, R, Cc, groups;
} mm_tmv_args;
int mm_tmv(const mm_tmv_args* x, mm_stream_t s);
/* Global-norm clip (torch clip_grad_norm_ over G[0:n_clip]) scaled by grad_scale (1/world after an
 * all-reduce), then Adam on P[0:n]; step is a device counter, norm_out receives the pre-clip norm. */
/* mm_clip_adam (two_groups = 0, clip group G[0:n_clip]) or mm_clip2_adam (two_groups != 0, split = n_clip), then the
 * behavior net's exact-f32 image written from the new parameters (what mm_qnet_pack_f32(d, P, packed) writes after
 * the step; the agent net's d->n_agents nets lead P), and, when per != NULL, mm_per_update(per, nodes, td, batch):
 * two launches instead of four (the Adam step and the image in one grid, the priority update one more block of it).
 * next_per != NULL (per == NULL: the priorities already updated): that block runs mm_per_sample_rng(next_per, batch,
 * next_seed, next_counter, next_nodes, next_slots, next_isw) instead — the NEXT update's draws, one launch fewer.
 * Results identical to the separate calls (Train_dqn.train's step + priority update, qmix/_train.py:86-96,
 * qmix/main.py:240-244). */
int mm_clip_adam_pack(float* P, float* G, float* m, float* v, int64_t n, int64_t n_clip, int32_t two_groups,
                      float max_norm, float lr, float beta1, float beta2, float eps, float* step, float* partials,
                      float* norm_out, float grad_scale, const mm_qnet_dims* d, float* packed, mm_per* per,
                      const int64_t* nodes, const float* td, int32_t batch, mm_per* next_per, uint64_t next_seed,
                      uint64_t next_counter, int64_t* next_nodes, int64_t* next_slots, float* next_isw,
                      mm_stream_t s);
/* clip_grad_norm_ on G[0:split] and on G[split:n] separately (qmix/qmix.py:235-238), then Adam. */
int mm_clip2_adam(float* P, float* G, float* m, float* v, int64_t n, int64_t split, float max_norm, float lr,
                  float beta1, float beta2, float eps, float* step, float* partials, float* norm_out, float grad_scale,
                  mm_stream_t s);
int mm_clip_adam(float* P, float* G, float* m, float* v, int64_t n, int64_t n_clip, float max_norm, float lr,
                 float beta1, float beta2, float eps, float* step, float* partials, float* norm_out, float grad_scale,
                 mm_stream_t s);

/* ------------------------------------------------------------------ MAPPO (rmappo, shared policy)
 * Replaces R_MAPPOPolicy.get_actions / get_values / evaluate_actions
 * (mappo/algorithms/rmappo_policy.py:57-136), SharedReplayBuffer.compute_returns + insert
 * (mappo/runner/shared/shared_buffer.py:82-157, magym_runner.py:138-195) and R_MAPPO.train /
 * ppo_update / cal_value_loss (mappo/algorithms/ramppo_network.py:56-287).
 * Net 0 = actor (head: A logits), net 1 = critic (head: 1 value). Per-net flat parameters in the
 * layout of mm_mappo_param_offsets (18 tensors: ln0_w ln0_b W1 b1 ln1_w ln1_b W2 b2 ln2_w ln2_b
 * Wih Whh bih bhh lnr_w lnr_b Wo bo + total; W1 rows padded to Dp = ceil4(D), Wo/bo to ceil4(O)).
 * Buffer arrays are [T(+1), EN] row-major with EN = envs*agents (row = t*EN + en); obs rows [.., D],
 * hiddens [.., H]. Supported: H = 32, A = 5, D in {47, 94}. */
typedef struct mm_mappo_dims {
  int32_t obs_dim, hidden, n_actions;
} mm_mappo_dims;
enum { MM_MAPPO_ROLLOUT = 0, MM_MAPPO_VALUES = 1, MM_MAPPO_TRAIN = 2 };
enum { MM_MAPPO_MAX_JOBS = 16 };
/* device scalar slots of the stats vector (float[8]) */
enum { MM_MST_ADV_MEAN = 0, MM_MST_ADV_STD = 1, MM_MST_ACTIVE_SUM = 2, MM_MST_RET_MEAN = 3, MM_MST_RET_SQ_MEAN = 4,
       MM_MST_VN_MEAN = 5, MM_MST_VN_STD = 6 };
/* loss accumulator slots (float[4], logging only): masked means as in train_info */
enum { MM_MLOSS_POLICY = 0, MM_MLOSS_ENTROPY = 1, MM_MLOSS_VALUE = 2, MM_MLOSS_RATIO = 3 };
typedef struct mm_mappo_net_io {
  const float* P;     /* flat parameters */
  const float* h_in;  /* rollout: [rows, H]; train: stored hiddens [T+1, EN, H] */
  float* h_out;       /* rollout: [rows, H] (may alias the next buffer slot) */
  float* out;         /* rollout: actor log-prob of the action / critic value, [rows] */
  float* save;        /* train: SoA scratch [mm_mappo_save_fields][rs] */
} mm_mappo_net_io;
typedef struct mm_mappo_fwd_args {
  mm_mappo_net_io net[2];
  const float* obs;      /* rollout [rows, D]; train [T+1, EN, D] */
  const float* mask;     /* rollout [rows] (NULL = ones); train masks [T+1, EN] */
  const int32_t* act_in; /* rollout: evaluate given actions instead of sampling */
  int32_t* act_out;      /* rollout: sampled actions [rows] */
  const float* u;        /* rollout: injected uniforms [rows] (NULL = counter RNG) */
  uint64_t seed;
  const uint64_t* counter_ptr; /* device RNG step counter (NULL = counter) */
  uint64_t counter;
  int64_t rows;
  int64_t en;
  int32_t T, L;
  int64_t rs;            /* SoA row stride (>= T*EN, multiple of 64; tail rows must stay zero) */
  int32_t mode;
  int32_t deterministic; /* rollout: take the mode (first argmax) instead of sampling (policy.act,
                            rmappo_policy.py:140-153 with deterministic=True) */
} mm_mappo_fwd_args;
typedef struct mm_mappo_bwd_args {
  const float* P[2];
  const float* save[2];  /* forward SoA scratch of each net */
  float* gsoa[2];        /* out: SoA operands of the weight gradients [mm_mappo_grad_fields][rs] */
  const float* obs;      /* [T+1, EN, D] */
  const float* mask;     /* masks [T+1, EN] */
  const float* active;   /* active masks [T+1, EN] */
  const int32_t* act;    /* actions [T, EN] */
  const float* adv;      /* raw advantages [T, EN] (normalised with stats) */
  const float* old_logp; /* action_log_probs [T, EN] */
  const float* old_value;/* value_preds [T+1, EN] */
  const float* returns;  /* [T+1, EN] */
  const float* stats;    /* float[8], see MM_MST_* */
  float* loss_acc;       /* float[4] or NULL */
  float clip, huber_delta, entropy_coef, value_coef;
  int64_t en;
  int32_t T, L;
  int64_t rs;
} mm_mappo_bwd_args;
int64_t mm_mappo_param_count(const mm_mappo_dims* d, int32_t net);
int mm_mappo_param_offsets(const mm_mappo_dims* d, int32_t net, int64_t offs[19]);
int mm_mappo_save_fields(const mm_mappo_dims* d, int32_t net);
int mm_mappo_grad_fields(const mm_mappo_dims* d, int32_t net);
/* Actor + critic forward: ROLLOUT (sample or evaluate act_in; new hiddens), VALUES (critic only),
 * TRAIN (every L-step chunk from its stored hidden, h <- h*mask each step; saves activations). */
int mm_mappo_fwd(const mm_mappo_dims* d, const mm_mappo_fwd_args* a, mm_stream_t s);
/* Loss seeds + chunked BPTT of both nets (after a TRAIN forward of the same data). */
int mm_mappo_bwd(const mm_mappo_dims* d, const mm_mappo_bwd_args* a, mm_stream_t s);
/* Weight gradients of one net from mm_mappo_bwd's SoA operands into its flat gradient vector. */
/* One PPO epoch's gradients of both nets (mappo_grad.hip; replaces mm_mappo_fwd TRAIN + mm_mappo_bwd +
 * mm_mappo_wgrad, ramppo_network.py:56-209) in two passes: the recurrent pass runs, per tile of 32 L-step
 * chunks, the forward from the stored chunk-start hiddens (h_actor / h_critic = rnn_states /
 * rnn_states_critic [T+1, EN, H], 16-byte aligned), recomputes it step by step in reverse for the BPTT and
 * writes d loss / d x2 (the GRU input) of every row-step; the row-parallel MLP pass backpropagates those
 * through the LN-MLP. Weight gradients are reduced on MFMA inside both. Uses a's P, obs, mask, active, act,
 * adv, old_logp, old_value, returns, stats, loss_acc, coefficients, en, T, L (save / gsoa / rs ignored).
 * Writes the full flat gradient vectors. scratch: mm_mappo_grad_scratch_count(d, L, T, en) floats, 16-byte
 * aligned. H 32, A 5, D 47 | 94. */
int64_t mm_mappo_grad_scratch_count(const mm_mappo_dims* d, int32_t L, int32_t T, int64_t en);
int mm_mappo_grad(const mm_mappo_dims* d, const mm_mappo_bwd_args* a, const float* h_actor, const float* h_critic,
                  float* grad_actor, float* grad_critic, float* scratch, mm_stream_t s);
/* R_MAPPOPolicy.evaluate_actions (rmappo_policy.py:101-136; RNNLayer's masked segments, rnn.py:24-80; the
 * Categorical head, distributions.py:55-68): a TRAIN-mode forward of both nets (a: T = L steps of EN chunks, rows
 * t*EN + en, chunk-start hiddens at h_in slot 0, masks [T, EN], save buffers), then per row the value, the log-prob
 * of act[row] and the entropy (ent_rows [T*EN]), and *entropy = the mean of ent_rows weighted by active [T*EN]
 * (NULL: plain mean). H 32, A 5. An action outside [0, A) sets bit 0 of *err (may be NULL). */
int mm_mappo_evaluate_actions(const mm_mappo_dims* d, const mm_mappo_fwd_args* a, const int32_t* act,
                              const float* active, float* values, float* logp, float* ent_rows, float* entropy,
                              int32_t* err, mm_stream_t s);
int64_t mm_mappo_wgrad_partial_count(const mm_mappo_dims* d, int64_t rs);
int mm_mappo_wgrad(const mm_mappo_dims* d, int32_t net, const float* gsoa, int64_t rs, float* grad, float* partial,
                   mm_stream_t s);
/* GAE with ValueNorm denormalisation (vn = float[3]: running mean, mean sq, debias): returns[t<T]. */
int mm_mappo_gae(const float* rew, const float* value_preds, const float* masks, float* returns, const float* vn,
                 int32_t T, int64_t en, float gamma, float gae_lambda, mm_stream_t s);
/* adv = returns - denorm(value_preds) over rows = T*EN; masked mean/std (two-pass, as np.nanstd),
 * active count, return moments into stats. partial: device double[7 * 256 + 5]; its last 5
 * entries (partial + 1792) receive the raw sums (adv, count, ret, ret^2, adv^2) for a
 * data-parallel all-reduce followed by mm_mappo_stats_from_sums (rows = global row count). */
int mm_mappo_adv_stats(const float* returns, const float* value_preds, const float* active, const float* vn,
                       float* adv, int64_t rows, double* partial, float* stats, mm_stream_t s);
int mm_mappo_stats_from_sums(const double* sums, int64_t rows, float* stats, mm_stream_t s);
/* One ValueNorm.update with the batch moments in stats, then stats[VN_MEAN/VN_STD]. */
int mm_mappo_vn_update(float* vn, float* stats, double beta, mm_stream_t s);
/* After env.step: masks/active of slot t+1, zero hiddens of done envs (done [E] u8); increments
 * the device RNG step counter (u64, may be NULL). */
int mm_mappo_insert(const uint8_t* done, int32_t n_agents, int32_t hidden, int64_t n_envs, float* mask_next,
                    float* active_next, float* h_actor, float* h_critic, uint64_t* counter, mm_stream_t s);

/* ------------------------------------------------------------------ offpolicy episode QMix / VDN
 * Replaces QMix.train_policy_on_batch (offpolicy/algorithms/qmix/qmix.py:80-210) with the shared
 * QMixPolicy (algorithm/QMixPolicy.py:51-195; AgentQFunction = LN(D) -> [Linear, ReLU, LN] x 2 ->
 * GRU(H) -> LN -> Linear(A), agent_q_function.py) and QMixer (2-layer hypernets, ELU,
 * algorithm/q_mixer.py:6-94) or VDNMixer (vdn/algorithm/vdn_mixer.py), plus soft_update
 * (utils/util.py:123-134). Agent parameters: the trunk layout of mm_mappo_param_offsets (net 0) with
 * hidden H; mixer parameters: the 14 QMixer tensors in named_parameters() order (mm_offq_mixer_offsets).
 * One flat vector [agent | mixer] per net (behavior P, target PT) and for the gradient.
 * Batch = PrioritizedRecReplayBuffer.sample layout (rec_buffer.py:192-240): obs [N, T+1, B, D],
 * share_obs [T+1, B, S], acts one-hot [N, T, B, A], rewards [N, T, B] (agent 0's are used,
 * qmix.py:169), dones_env [T, B], is_weight [B] (NULL: no PER). Supported: H = 64, A = 5,
 * D in {47, 94}; QMIX: hypernet_layers = 2, any S, N*K <= 4096. */
enum { MM_OFFQ_VDN = 0, MM_OFFQ_QMIX = 1 };
typedef struct mm_offq_dims {
  int32_t n_agents, obs_dim, hidden, n_actions;
  int32_t mixer;                                   /* MM_OFFQ_VDN / MM_OFFQ_QMIX */
  int32_t state_dim, mixer_hidden, hyper_hidden;   /* QMIX: S, K (mixer_hidden_dim), hypernet_hidden_dim */
} mm_offq_dims;
typedef struct mm_offq_batch {
  const float* obs; const float* share_obs; const float* acts; const float* rewards; const float* dones_env;
  const float* is_weight;
  int32_t T, B;
  int32_t double_q, huber;
  float gamma, huber_delta, per_nu, per_eps;
} mm_offq_batch;
int mm_offq_param_counts(const mm_offq_dims* d, int64_t* agent, int64_t* mixer);
int mm_offq_mixer_offsets(const mm_offq_dims* d, int64_t offs[15]);
int64_t mm_offq_workspace_bytes(const mm_offq_dims* d, int32_t T, int32_t B);
/* Forward (behavior + target over all T+1 steps), loss, R2D2 priorities and the gradient of the
 * loss w.r.t. P (written to grad; zero-initialised pads stay zero). stats: float[2] = loss, Q_tot
 * mean (train_info); priorities [B] (PER only, may be NULL). ws: zero-initialised device scratch of
 * mm_offq_workspace_bytes for these (T, B), reused across calls. Follow with mm_clip_adam over the
 * whole [agent | mixer] vector (max_grad_norm, lr, opti_eps) to complete the update. */
int mm_offq_loss_grad(const mm_offq_dims* d, const mm_offq_batch* b, const float* P, const float* PT, float* grad,
                      void* ws, int64_t ws_bytes, float* stats, float* priorities, mm_stream_t s);
/* get_q_values over a sequence: obs [L, R, D] (stacked rows), h0 [R, H] (NULL = zeros) ->
 * q [L, R, A], h_out [R, H] (may be NULL). ws: mm_offq_qvals_workspace_bytes(d, L, R). */
int64_t mm_offq_qvals_workspace_bytes(const mm_offq_dims* d, int32_t L, int64_t R);
int mm_offq_q_values(const mm_offq_dims* d, const float* P, const float* obs, const float* h0, float* q, float* h_out,
                     int32_t L, int64_t R, void* ws, int64_t ws_bytes, mm_stream_t s);
/* soft_update: target <- target * (1 - tau) + source * tau over n floats (tau = 1: hard update). */
int mm_offq_soft_update(float* target, const float* source, int64_t n, double tau, mm_stream_t s);

/* ------------------------------------------------------- ma_gym Switch corridor env (mm_switch_*) */
/* gym.make("ma_gym:Switch2-v0", max_steps, step_cost) (qmix/_config.py:14-19, qmix/main.py:66-71,
 * 103-115): E envs in lockstep, n_agents 2..4 on the 3 x 7 two-room grid. Dynamics spec (ma-gym is
 * absent: parity unpinned): oracle/switch.py. Obs per agent [row/2, round(col/6, 2)(, step/max_steps)],
 * D = 2 + clock, or N x that when full_observable; actions 0 down 1 left 2 up 3 right 4 noop. */
typedef struct mm_switch_cfg {
  int32_t n_agents, max_steps, full_observable, clock;
  float step_cost;
} mm_switch_cfg;
typedef struct mm_switch mm_switch;
int mm_switch_create(const mm_switch_cfg* cfg, int64_t n_envs, mm_switch** out);
void mm_switch_destroy(mm_switch* w);
int mm_switch_obs_dim(const mm_switch* w);
/* reset every env; obs [E, N, D] (may be NULL) */
int mm_switch_reset(mm_switch* w, float* obs, mm_stream_t s);
/* step with act [E, N] int32: next_obs [E, N, D] (terminal), rew [E, N], agent_done [E, N] u8 (may be
 * NULL; the env's per-agent done list), done [E] u8 (all agents done). obs_cur != NULL: done envs
 * auto-reset and obs_cur gets the next current obs. */
int mm_switch_step(mm_switch* w, const int32_t* act, float* next_obs, float* obs_cur, float* rew,
                   uint8_t* agent_done, uint8_t* done, mm_stream_t s);
/* host copies of the state (synchronous): pos [E, N, 2], agent_done [E, N], steps [E] */
int mm_switch_get_state(mm_switch* w, int32_t* pos, uint8_t* agent_done, int32_t* steps);
/* restore a state returned by mm_switch_get_state (checkpoint resume; synchronous) */
int mm_switch_set_state(mm_switch* w, const int32_t* pos, const uint8_t* agent_done, const int32_t* steps);
const float* mm_switch_reset_obs(const mm_switch* w); /* device [N, D]: the (deterministic) reset obs */
/* The rollout engine's row steps, same contract as mm_env_step_rows / mm_env_step_rows_td (the env's
 * done written is all(agent done), what qmix/main.py:199,215 stores): the Switch env behind the same
 * chunk-store engine as the Checkers env. */
int mm_switch_step_rows(mm_switch* w, const int32_t* act, float* next_obs, int64_t next_se, const int64_t* next_row,
                        float* obs_cur, int64_t* cur_row, float* rew, uint8_t* done, mm_stream_t s);
int mm_switch_step_rows_begin(mm_switch* w, const int32_t* act, float* store_obs, int64_t row_stride,
                              int32_t chunk_len, const int64_t* staging, int64_t* cur_row, float* rew, uint8_t* done,
                              mm_stream_t s);
int mm_switch_step_rows_td(mm_switch* w, const int32_t* act, float* next_obs, int64_t next_se,
                           const int64_t* next_row, int64_t* cur_row, float* rew, uint8_t* done, float gamma,
                           const float* td_rew, const uint8_t* td_done, const float* q_taken, const float* max_q_next,
                           const int32_t* td_act, float* chunk_td, int32_t step_in_chunk, int32_t chunk_len,
                           uint8_t* store_act, float* store_rew, uint8_t* store_done, const int64_t* td_rows,
                           uint64_t* counter, mm_stream_t s);

/* ------------------------------------------------------- offpolicy episode replay (mm_erb_*) */
/* RecReplayBuffer / PrioritizedRecReplayBuffer of one policy (offpolicy/utils/rec_buffer.py:10-324)
 * with its SumSegmentTree / MinSegmentTree (offpolicy/utils/segment_tree.py:18-165), resident in HBM.
 * Episode store: one ring of buffer_size episodes, each field [slot][L][row] (L = T + 1 for obs /
 * share_obs, T for the rest). Trees: f64 heaps [2 * itcap], root 1, leaves at itcap + i (itcap = the
 * next power of two >= buffer_size). The ring cursor (current_i / filled_i) is host state; the trees
 * and max_priority live on the device, so insert -> sample -> train -> update_priorities never syncs.
 * leaf_mode 0 = the reference's insert, which writes max_priority ** alpha into leaves 0..n-1
 * (rec_buffer.py:265-268); 1 = write the inserted slots' leaves instead. */
typedef struct mm_erb mm_erb;
typedef struct mm_erb_dims {
  int32_t T, N, D, S, A;     /* episode_length, agents, obs dim, share_obs dim, act dim (one-hot width) */
  int32_t same_share;        /* use_same_share_obs: share_obs stored once per step ([L, B, S] samples) */
  int32_t prioritized;       /* PrioritizedRecReplayBuffer (trees + max_priority) */
  int32_t leaf_mode;         /* 0 reference (leaves 0..n-1), 1 slots */
} mm_erb_dims;
/* Episode fields, device pointers. insert: the reference's insert layout obs [T+1, n, N, D],
 * share_obs [T+1, n, N, S] (agent 0 is kept when same_share), acts [T, n, N, A], rewards / dones
 * [T, n, N, 1], dones_env [T, n, 1]. gather (sample_inds, rec_buffer.py:192-240): obs [N, T+1, B, D],
 * share_obs [T+1, B, S] (same_share) or [N, T+1, B, S], acts [N, T, B, A], rewards / dones
 * [N, T, B, 1], dones_env [T, B, 1]. Any field may be NULL in a gather (not written). */
typedef struct mm_erb_fields {
  float* obs; float* share_obs; float* acts; float* rewards; float* dones; float* dones_env;
} mm_erb_fields;
int mm_erb_create(const mm_erb_dims* d, int64_t buffer_size, double alpha, mm_erb** out);
void mm_erb_destroy(mm_erb* b);
/* RecPolicyBuffer.insert + the prioritized leaf writes (rec_buffer.py:146-190, 262-270); n <= size.
 * idx_range_host (may be NULL): int64 [n], the ring slots written (host memory, filled at once). */
int mm_erb_insert(mm_erb* b, int32_t n, const mm_erb_fields* src, int64_t* idx_range_host, mm_stream_t s);
int64_t mm_erb_len(const mm_erb* b);          /* filled_i */
int64_t mm_erb_current(const mm_erb* b);      /* current_i */
int64_t mm_erb_it_capacity(const mm_erb* b);
/* Prioritized sample indices + IS weights (rec_buffer.py:272-296): mass_b = u_b * sum(0, len-1),
 * prefix-sum descent, w_b = (p_b len)^-beta / (p_min len)^-beta. u_b = fracs[b] (device f64 [B],
 * the injected np.random.random draws) or, when fracs is NULL, the device counter RNG (seed,
 * counter). idx_out: device int64 [B]; w_out: device f64 [B] (may be NULL); w32_out: device f32 [B]
 * (may be NULL; the trainer's importance_weights). Requires len > B, beta > 0 (reference asserts). */
int mm_erb_sample_prioritized(mm_erb* b, int32_t B, double beta, const double* fracs, uint64_t seed,
                              uint64_t counter, int64_t* idx_out, double* w_out, float* w32_out, mm_stream_t s);
/* Uniform indices (RecReplayBuffer.sample, rec_buffer.py:76): idx_b = floor(u_b len), device RNG. */
int mm_erb_sample_uniform(mm_erb* b, int32_t B, uint64_t seed, uint64_t counter, int64_t* idx_out, mm_stream_t s);
/* sample_inds: gather the B episodes idx [B] (device int64) into the sample layout above (an index
 * outside [0, buffer_size) gathers zeros and sets bit 2 of the error word). */
int mm_erb_gather(mm_erb* b, int32_t B, const int64_t* idx, const mm_erb_fields* dst, mm_stream_t s);
/* update_priorities (rec_buffer.py:306-324): leaves[idx] = prio ** alpha (f32 pow, last duplicate
 * wins), ancestors re-derived, max_priority = max(max_priority, max prio). idx, prio: device [B]. An
 * index outside [0, len) or a priority <= 0 (the reference's asserts) skips that entry and sets the
 * error word (mm_erb_error_word). */
int mm_erb_update_priorities(mm_erb* b, const int64_t* idx, const float* prio, int32_t B, mm_stream_t s);
double* mm_erb_sum_tree(mm_erb* b);           /* device f64 [2 * itcap] */
double* mm_erb_min_tree(mm_erb* b);           /* device f64 [2 * itcap] */
float* mm_erb_max_priority(mm_erb* b);        /* device f32 [1] */
int32_t* mm_erb_error_word(mm_erb* b);        /* device i32 [1]: bit 0 bad update index, bit 1 priority <= 0,
                                                 bit 2 bad gather index */
/* Stream-ordered device copies of the trees, max_priority and the error word (any may be NULL). */
int mm_erb_copy_state(mm_erb* b, double* sum_dst, double* min_dst, float* maxp_dst, int32_t* err_dst, mm_stream_t s);

/* Debug: copy the first n (<= 4096) u64 slots of the timing trace buffer that kernels fill when
 * MM_REC_TRACE=1 is set in the environment (clock64 stamps per phase; tools/trace_rec.py). mm_debug_trace(NULL, 0) allocates the buffer
 * (call it before any graph capture). */
int mm_debug_trace(uint64_t* host_out, int32_t n);

#ifdef __cplusplus
}
#endif
#endif
