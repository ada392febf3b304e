// One translation unit for the agent-network kernels (agent_fwd.hip) and the QMIX learner kernels (learner.hip):
// the learner's forward runs an agent body and a mixer body in ONE grid (two independent chains sharing the GPU),
// which needs both in one TU. On ROCm's graph executor every stream fork / join edge of the captured update cost
// 5-10 us (profiles/r05_learner_b32_timeline.txt): a shared grid has none.
//   mm_agent_mixer_pre     = mm_mixer_gi (Mix_Net W_ih s of every (t, b)) || mm_agent_q_pre2 (layers 1-2 and
//                            W_ih x2 of every (t, b) row, both nets)
//   mm_agent_mixer_rec_seq = mm_mixer_fwd_seq_rec (the Mix_Net GRU over the state) || mm_agent_q_rec_seq2 (the
//                            agent GRU + Q head over the C steps, both nets)
//   mm_clip_adam_pack      = mm_clip_adam + mm_qnet_pack_f32 of the behavior net (+ mm_per_update, or + the next
//                            update's mm_per_sample_rng): the Adam step writes the exact-f32 image from the new
//                            values (one more block: the priorities, or the next batch's draws)
//   mm_mixer_bwd_seq_hyper_per = mm_mixer_bwd_seq_hyper + mm_per_update (one more block of the hypernet pass)
// (Train_dqn.train's forward over the chunk, qmix/_train.py:55-77: Q_Net per step, then Mix_Net per step; the
// Mix_Net's GRU depends on the state only, so it runs beside the agent chain; the step / priority update,
// qmix/_train.py:86-96 and main.py:240-244.) Each block runs the same body as the separate kernel, so the results
// are bit-identical to the separate launches (test_paired_fwd_launches_bit_identical, test_clip_adam_pack_*).
#include "agent_fwd.hip"
#include "learner.hip"
#include "per.hip"

namespace mm {

template <int F1, int G, int H>
struct PairGeo {
  // (the kernels' __launch_bounds__ spell these out: a template argument list inside the macro would split it)
  static constexpr int NW = 3 * (H / 32) > F1 / 32 ? 3 * (H / 32) : F1 / 32;   // agent_pre_rb_kernel's waves
  static constexpr int PRE_THREADS = 64 * NW;
  static constexpr int REC_THREADS = 64 * (3 * (H / 32) + 1);                  // agent_rec_seq_gp_kernel's
};

// blocks [0, n_gi): mixer_gi tile (bid % gx, (bid / gx) % gy) of net bid / (gx gy); the rest: agent_pre_rb
template <int F1, int G, int H, int AB>
__global__ __launch_bounds__(64 * (3 * (H / 32) > F1 / 32 ? 3 * (H / 32) : F1 / 32)) void agent_mixer_pre_kernel(
    QFwdParams p0, QFwdParams p1, MixGiArgs ga, int n_gi, int gx, int gy) {
  const int bid = (int)blockIdx.x;
  if (bid < n_gi) {
    mixer_gi_body(ga, bid % gx, (bid / gx) % gy, bid / (gx * gy));
    return;
  }
  const int b = bid - n_gi;
  if (b >= p0.nblocks)
    agent_pre_rb_body<F1, G, H, AB>(p1, (b - p0.nblocks) % p1.N, (b - p0.nblocks) / p1.N);
  else
    agent_pre_rb_body<F1, G, H, AB>(p0, b % p0.N, b / p0.N);
}

// blocks [0, n_agent): rec_seq_gp (net 0's tiles, then net 1's); the rest: the mixer recurrence of sample j % B of
// net j / B, j = bid - n_agent. The dynamic LDS holds whichever body the block runs.
template <int F1, int G, int H, int AB, int HM>
__global__ __launch_bounds__(64 * (3 * (H / 32) + 1)) void agent_mixer_rec_kernel(QFwdParams p0, QFwdParams p1,
                                                                                   RecSeq s0, RecSeq s1, MixFwdArgs ma,
                                                                                   MixRecFwd mq, int n_agent) {
  extern __shared__ __attribute__((aligned(16))) char plds[];
  const int bid = (int)blockIdx.x;
  if (bid < n_agent) {
    if (bid >= p0.nblocks)
      rec_seq_gp_body<F1, G, H, AB>(p1, s1, bid - p0.nblocks, plds);
    else
      rec_seq_gp_body<F1, G, H, AB>(p0, s0, bid, plds);
    return;
  }
  const int j = bid - n_agent;
  if (j < ma.B)
    mixer_rec_fwd_body<HM>(ma, ma.net[0], mq, j, 0, reinterpret_cast<float*>(plds));
  else
    mixer_rec_fwd_body<HM>(ma, ma.net[1], mq, j - ma.B, 1, reinterpret_cast<float*>(plds));
}

static bool pair_dims_ok(const mm_qnet_dims* d) {
  return d && d->f1 == 64 && d->g == 64 && d->h == 64 && d->n_actions <= 32;   // the B = 32 learner's agent net
}

// the pre pair: the small-batch row-block PRE and the split-K state projection, agent block wide enough for the
// projection's 4 waves
static bool pre_pair_ok(const mm_qnet_dims* d, int64_t rows, int32_t N) {
  if (!pair_dims_ok(d) || d->n_agents != N || d->obs_dim > 32 * kPreRbMaxKD) return false;
  const int64_t tiles = (rows + 31) / 32 * N;
  return 2 * tiles <= 2048 && rows < 2048 && PairGeo<64, 64, 64>::PRE_THREADS >= 256;
}

static size_t rec_pair_lds(int32_t Hm, int32_t steps) {
  return std::max(RecGpLds<64>::bytes, mix_rec_fwd_floats(Hm, mix_rec_win(steps, Hm, false)) * 4);
}

static bool rec_pair_ok(const mm_qnet_dims* d, int32_t B, int32_t N, int32_t Hm, int32_t K1, int32_t steps) {
  if (!pair_dims_ok(d) || d->n_agents != N) return false;
  const int64_t agent_blocks = 2 * ((B + 31) / 32) * (int64_t)N;
  return agent_blocks < 512 && mix_split_enabled() && mix_rec_supported(Hm) && mm_mixer_fwd_seq_fits(B, N, Hm, K1) &&
         rec_pair_lds(Hm, steps) <= 160 * 1024;
}

// Blocks [0, nA): image elements (grid-stride): the Adam step of the element's parameter(s), the image element
// from the new values (qnet_pack_value: what qnet_pack_kernel writes after adam_kernel); blocks [nA, nA + nB): the
// Adam step of the parameters outside the agent image ([n_agent, n): the mixer's); block nA + nB (when pu.tree):
// per_update_small_block. Every parameter's step runs exactly once (qnet_pack_src: each agent parameter lies in one
// image element). (A parameter-centric order — coalesced Adam, each image element written through the inverse
// mapping — measured 16.0 vs 13.2 us at the B = 32 shapes.)
// (ps.tree: the extra block samples the NEXT update's batch instead, once this update's priorities are in)
__global__ __launch_bounds__(1024) void adam_pack_kernel(AdamArgs a, float* packed, QnetGeo g, int N, int D, int F1,
                                                         int G, int H, int A, QnetOffsets o, int nA, int nB, PerUpd pu,
                                                         PerSmp ps) {
  const int bid = (int)blockIdx.x;
  if (bid >= nA + nB) {
    if (ps.tree)
      per_sample_block(ps);
    else
      per_update_small_block(pu);
    return;
  }
  const AdamConst c = adam_const(a);
  if (bid < nA) {
    const int64_t per_agent = g.agent_stride, total = per_agent * N;
    for (int64_t idx = bid * 1024ll + threadIdx.x; idx < total; idx += (int64_t)nA * 1024) {
      const PackSrc ps = qnet_pack_src(g, (int)(idx / per_agent), idx % per_agent, D, F1, G, H, A, o);
      const float v0 = ps.j0 >= 0 ? adam_elem(a, c, ps.j0) : 0.0f;
      const float v1 = ps.j1 >= 0 ? adam_elem(a, c, ps.j1) : 0.0f;
      packed[idx] = qnet_pack_value(ps, v0, v1);
    }
  } else {
    for (int64_t i = o.total + (int64_t)(bid - nA) * 1024 + threadIdx.x; i < a.n; i += (int64_t)nB * 1024)
      adam_elem(a, c, i);
  }
}

}  // namespace mm

extern "C" {

int mm_mixer_bwd_seq_hyper_per(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P,
                               const float* save, const float* qa, const float* dq, const float* done,
                               const float* ones, float* dhm, float* dqa, float* delta, float* ws, int32_t steps,
                               mm_per* per, const int64_t* nodes, const float* td, int32_t batch, mm_stream_t s) {
  MM_REQUIRE(per && nodes && td, "mixer_bwd_seq_hyper_per: null PER argument");
  const bool small = (per->cap & (per->cap - 1)) == 0 && batch >= 1 && batch <= mm::PU_B &&
                     mm::mix_hyper_bwd_floats(Hm, K1, N) * 4 + mm::kPerSmallLds <= mm::kMixSeqLds;
  if (small) {
    const mm::PerUpd pu = {per->tree, per->cap, nodes, td, per->st, batch, (float)per->eps};
    return mixer_bwd_seq_part(1, B, N, S, Hm, K1, P, save, qa, dq, done, ones, dhm, dqa, delta, ws, steps, s, &pu);
  }
  const int rc = mixer_bwd_seq_part(1, B, N, S, Hm, K1, P, save, qa, dq, done, ones, dhm, dqa, delta, ws, steps, s);
  if (rc) return rc;
  return mm_per_update(per, nodes, td, batch, s);
}

int mm_clip_adam_pack(float* P, float* G, float* m, float* v, int64_t n, int64_t n_clip, int32_t two_groups,
                      float max_norm, float lr, float beta1, float beta2, float eps, float* step, float* partials,
                      float* norm_out, float grad_scale, const mm_qnet_dims* d, float* packed, mm_per* per,
                      const int64_t* nodes, const float* td, int32_t batch, mm_per* next_per, uint64_t next_seed,
                      uint64_t next_counter, int64_t* next_nodes, int64_t* next_slots, float* next_isw,
                      mm_stream_t s) {
  MM_REQUIRE(P && G && m && v && step && partials && packed && d && n > 0 && n_clip >= 0 && n_clip <= n,
             "clip_adam_pack: bad args");
  mm::QnetGeo g;
  mm::QnetOffsets o;
  int rc = mm::qnet_geometry(d, &g, &o);
  if (rc) return rc;
  MM_REQUIRE(o.total <= n, "clip_adam_pack: the agent net (%lld params) must lead P (%lld)", (long long)o.total,
             (long long)n);
  const int nb = 256;
  hipLaunchKernelGGL(mm::sumsq_kernel, dim3(nb), dim3(256), 0, (hipStream_t)s, G, n_clip, partials, step);
  MM_HIP_CHECK(hipGetLastError());
  if (two_groups) {
    hipLaunchKernelGGL(mm::sumsq_kernel, dim3(nb), dim3(256), 0, (hipStream_t)s, G + n_clip, n - n_clip,
                       partials + nb, (float*)nullptr);
    MM_HIP_CHECK(hipGetLastError());
  }
  const mm::AdamArgs a = {P, G, m, v, n, n_clip, partials, nb, max_norm, lr, beta1, beta2, eps, step, norm_out,
                          grad_scale, two_groups ? partials + nb : nullptr};
  const int64_t total = g.agent_stride * d->n_agents;
  const int nA = (int)std::min<int64_t>((total + 1023) / 1024, 1024);
  const int nB = (int)std::min<int64_t>((n - o.total + 1023) / 1024, 512);
  mm::PerUpd pu = {};
  mm::PerSmp ps = {};
  const bool per_block = per && nodes && td && (per->cap & (per->cap - 1)) == 0 && batch >= 1 && batch <= mm::PU_B;
  if (next_per) {   // sample the next update's batch (this update's priorities must be in already)
    MM_REQUIRE(!per && next_nodes && next_slots && next_isw && batch >= 1 && batch <= mm::PS_T * mm::PER_SAMPLE_MAXJ,
               "clip_adam_pack: the next sample needs its outputs and no priority update in the same launch");
    MM_REQUIRE(next_per->n_data > 0, "per_sample: empty buffer");
    const double decay = per_sample_prep(next_per);
    ps = {next_per->tree, next_per->cap, next_per->st, next_seed, next_counter, decay, next_nodes, next_slots,
          next_isw, batch};
  } else if (per_block) {
    pu = {per->tree, per->cap, nodes, td, per->st, batch, (float)per->eps};
  }
  const int extra = (next_per || per_block) ? 1 : 0;
  hipLaunchKernelGGL(mm::adam_pack_kernel, dim3(nA + nB + extra), dim3(1024), 0, (hipStream_t)s, a, packed, g,
                     d->n_agents, d->obs_dim, d->f1, d->g, d->h, d->n_actions, o, nA, nB, pu, ps);
  MM_HIP_CHECK(hipGetLastError());
  if (per && !per_block) return mm_per_update(per, nodes, td, batch, s);
  return MM_OK;
}

int mm_agent_mixer_pair_supported(const mm_qnet_dims* d, int32_t B, int32_t steps, int32_t N, int32_t S, int32_t Hm,
                                  int32_t K1) {
  (void)S;
  int m = 0;
  if (mm::pre_pair_ok(d, (int64_t)B * steps, N)) m |= 1;
  if (mm::rec_pair_ok(d, B, N, Hm, K1, steps)) m |= 2;
  return m;
}

int mm_agent_mixer_pre(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, const float* packed1,
                       const mm_qfwd_io* io1, int64_t rows, int32_t N, int32_t S, int32_t Hm, int32_t K1,
                       const float* obs, const float* reset_obs, const float* mP0, const int64_t* s_off0, float* gi0,
                       const float* mP1, const int64_t* s_off1, float* gi1, mm_stream_t s) {
  MM_REQUIRE(mm::pre_pair_ok(d, rows, N), "agent_mixer_pre: shapes outside the paired launch (see "
                                          "mm_agent_mixer_pair_supported)");
  MM_REQUIRE(io0 && io1 && mP0 && mP1 && gi0 && gi1 && s_off0 && s_off1 && obs, "agent_mixer_pre: null argument");
  MM_REQUIRE(io0->gi && io1->gi, "agent_pre: io.gi required");
  MM_REQUIRE((((uintptr_t)io0->gi | (uintptr_t)io0->save | (uintptr_t)io1->gi | (uintptr_t)io1->save) & 15) == 0,
             "agent_pre: gi / save bases must be 16-byte aligned");
  mm::QFwdParams p0, p1;
  int rc = mm::make_params(d, packed0, io0, rows, &p0);
  if (rc) return rc;
  rc = mm::make_params(d, packed1, io1, rows, &p1);
  if (rc) return rc;
  p0.nblocks = (int)((rows + 31) / 32) * N;
  p1.nblocks = p0.nblocks;
  mm::MixGiArgs a;
  a.net[0] = {mP0, s_off0, gi0};
  a.net[1] = {mP1, s_off1, gi1};
  a.obs = obs;
  a.reset_obs = reset_obs;
  a.R = (int)rows;
  a.S = S;
  a.Hm = Hm;
  a.K1 = K1;
  a.N = N;
  const int gx = (int)((rows + 31) / 32), gy = (3 * Hm + 31) / 32, n_gi = gx * gy * 2;
  using PG = mm::PairGeo<64, 64, 64>;
  if ((d->n_actions + 31) / 32 == 1)
    hipLaunchKernelGGL((mm::agent_mixer_pre_kernel<64, 64, 64, 1>), dim3(n_gi + p0.nblocks + p1.nblocks),
                       dim3(PG::PRE_THREADS), 0, (hipStream_t)s, p0, p1, a, n_gi, gx, gy);
  else
    return MM_EINVAL;
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_agent_mixer_rec_seq(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, const float* packed1,
                           const mm_qfwd_io* io1, int32_t B, int32_t steps, const uint8_t* reset, int32_t N,
                           int32_t S, int32_t Hm, int32_t K1, const mm_mix_net* nets, int32_t n_nets,
                           const uint8_t* reset_steps, mm_stream_t s) {
  MM_REQUIRE(mm::rec_pair_ok(d, B, N, Hm, K1, steps), "agent_mixer_rec_seq: shapes outside the paired launch (see "
                                                       "mm_agent_mixer_pair_supported)");
  MM_REQUIRE(io0 && io1 && nets && n_nets == 2, "agent_mixer_rec_seq: both nets of each side required");
  mm::QFwdParams p0, p1;
  mm::RecSeq s0, s1;
  bool single;
  int rc = mm::rec_seq_args(d, packed0, io0, B, packed1, io1, B, steps, reset, p0, p1, s0, s1, single);
  if (rc) return rc;
  p0.nblocks = (p0.E + 31) / 32 * p0.N;
  p1.nblocks = (p1.E + 31) / 32 * p1.N;
  mm::MixFwdArgs ma;
  mm::MixRecFwd mq;
  rc = mixer_fwd_seq_part(3, B, N, S, Hm, K1, nets, n_nets, steps, reset_steps, s, &ma, &mq);
  if (rc) return rc;
  const size_t sm = mm::rec_pair_lds(Hm, steps);
  const int n_agent = p0.nblocks + p1.nblocks;
  using PG = mm::PairGeo<64, 64, 64>;
#define MM_RPAIR(HM_)                                                                                              \
  do {                                                                                                             \
    static const hipError_t attr = hipFuncSetAttribute((const void*)mm::agent_mixer_rec_kernel<64, 64, 64, 1, HM_>, \
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);    \
    MM_HIP_CHECK(attr);                                                                                            \
    hipLaunchKernelGGL((mm::agent_mixer_rec_kernel<64, 64, 64, 1, HM_>), dim3(n_agent + 2 * B),                    \
                       dim3(PG::REC_THREADS), sm, (hipStream_t)s, p0, p1, s0, s1, ma, mq, n_agent);               \
  } while (0)
  if ((d->n_actions + 31) / 32 != 1) return MM_EINVAL;
  if (Hm == 32)
    MM_RPAIR(32);
  else
    MM_RPAIR(64);
#undef MM_RPAIR
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

}  // extern "C"
