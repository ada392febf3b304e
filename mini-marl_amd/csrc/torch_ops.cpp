// PyTorch custom-op registry of the minimarl hot path: TORCH_LIBRARY(minimarl, ...).
//
// Every op is a thin, checked wrapper over the C ABI of libminimarl.so (include/minimarl.h): tensors
// are caller-allocated (torch caching allocator), outputs are the ops' mutable arguments (no hidden
// allocation in a hot op), work is enqueued on the CURRENT HIP stream of the tensors' device with no
// host sync, and argument errors raise RuntimeError (TORCH_CHECK) with the library's message.
// Stateful pieces of the reference (the env object, the prioritized replay) are TorchScript custom
// classes holding the C ABI handles: torch.classes.minimarl.Env / torch.classes.minimarl.PER.
//
// Reference interfaces replaced (reference @ /root/reference):
//   qnet_pack / agent_q_fwd      Q_Net.forward                        qmix/_network.py:44-64, vdn/_network.py:71-83
//   agent_q_act                  Q_Net.sample_action / epsilon_greedy  qmix/_network.py:66-74, vdn/_network.py:52-58
//   agent_q_max                  target_network(next_state) -> max     qmix/main.py:191-193
//   td_error                     cal_td_error                         vdn/_utils.py:44-52, qmix/_utils.py:86-97
//   gae_scan                     SharedReplayBuffer.compute_returns   mappo/runner/shared/shared_buffer.py:131-157
//   qmix_mixer_fwd               Mix_Net.forward (one step)           qmix/_network.py:199-217
//   qmix_mixer_bwd               its backward: dQ_i, dh, every Mix_Net parameter gradient
//   td_target_loss               Train_dqn / Target_Dqn TD target + MSE (or Huber), dQ_tot seeds, priorities
//                                                                     qmix/_train.py:75-84,118-121; vdn/_train.py:73-79
//   vdn_sum                      VDN mixing sum_i Q_i(a_i) / sum_i max_a Q_i   vdn/_train.py:23-47,68-71
//   mappo_get_actions            R_MAPPOPolicy.get_actions / act: MLPBase -> masked GRU step -> LayerNorm ->
//                                Categorical sample + log-prob, critic value   rmappo_policy.py:57-99,
//                                rnn.py:26-29, distributions.py:55-68
//   mappo_evaluate_actions       R_MAPPOPolicy.evaluate_actions: masked GRU scan over L-step chunks (RNNLayer's
//                                segments, rnn.py:30-80) + Categorical log-prob / entropy + values
//                                rmappo_policy.py:101-136
//   Env.reset / Env.step         gym.make("ma_gym:Checkers-v0")       vdn/main.py:61-64,143
//   PER.insert / sample / update Prioritized_Experience_Replay        vdn/replay_buffer/buffer.py:34-90
#include <ATen/ATen.h>
// PyTorch-ROCm reports GPU tensors as DeviceType::CUDA; its HIP guard / stream types for such
// devices are the "MasqueradingAsCUDA" ones
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <string>
#include <vector>

#include "minimarl.h"

namespace {

mm_stream_t stream_of(const at::Tensor& t) {
  return (mm_stream_t)c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void ok(int rc, const char* what) { TORCH_CHECK(rc == 0, "minimarl::", what, ": ", mm_last_error()); }

void need(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " must be ", c10::toString(dt), ", got ", c10::toString(t.scalar_type()));
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void same_device(const at::Tensor& a, const at::Tensor& b, const char* name) {
  TORCH_CHECK(a.device() == b.device(), name, " is on ", b.device(), " but the op runs on ", a.device());
}

mm_qnet_dims dims_of(const std::vector<int64_t>& d) {
  TORCH_CHECK(d.size() == 6, "dims must be [n_agents, obs_dim, f1, g, h, n_actions]");
  mm_qnet_dims q;
  q.n_agents = (int32_t)d[0];
  q.obs_dim = (int32_t)d[1];
  q.f1 = (int32_t)d[2];
  q.g = (int32_t)d[3];
  q.h = (int32_t)d[4];
  q.n_actions = (int32_t)d[5];
  return q;
}

// ------------------------------------------------------------------ Q-network
void qnet_pack(const at::Tensor& params, std::vector<int64_t> dims, at::Tensor packed) {
  const mm_qnet_dims d = dims_of(dims);
  need(params, at::kFloat, "params");
  need(packed, at::kFloat, "packed");
  same_device(params, packed, "packed");
  int64_t offs[11];
  ok(mm_qnet_param_offsets(&d, offs), "qnet_pack");
  TORCH_CHECK(params.numel() == offs[10], "params has ", params.numel(), " elements, the layout needs ", offs[10]);
  TORCH_CHECK(packed.numel() == mm_qnet_packed_count(&d), "packed has ", packed.numel(), " elements, needs ",
              mm_qnet_packed_count(&d));
  const c10::hip::HIPGuardMasqueradingAsCUDA g(params.device());
  ok(mm_qnet_pack(&d, params.data_ptr<float>(), packed.data_ptr<float>(), stream_of(params)), "qnet_pack");
}

// obs [E,N,D], hidden [E,N,H] (any strides, feature stride 1 for obs) -> io
mm_qfwd_io base_io(const mm_qnet_dims& d, const at::Tensor& packed, const at::Tensor& obs, const at::Tensor& hidden,
                   at::Tensor& hidden_out) {
  need(packed, at::kFloat, "packed");
  TORCH_CHECK(obs.is_cuda() && obs.scalar_type() == at::kFloat && obs.dim() == 3 && obs.stride(2) == 1,
              "obs must be a float GPU tensor [E, N, D] with unit feature stride");
  const int64_t E = obs.size(0);
  TORCH_CHECK(obs.size(1) == d.n_agents && obs.size(2) == d.obs_dim, "obs shape ", obs.sizes(), " != [E, ",
              d.n_agents, ", ", d.obs_dim, "]");
  for (const at::Tensor* h : std::initializer_list<const at::Tensor*>{&hidden, &hidden_out}) {
    TORCH_CHECK(h->is_cuda() && h->scalar_type() == at::kFloat && h->dim() == 3, "hidden tensors must be float [E,N,H]");
    TORCH_CHECK(h->size(0) == E && h->size(1) == d.n_agents && h->size(2) == d.h, "hidden shape ", h->sizes(),
                " != [", E, ", ", d.n_agents, ", ", d.h, "]");
    same_device(obs, *h, "hidden");
  }
  same_device(obs, packed, "packed");
  TORCH_CHECK(packed.numel() == mm_qnet_packed_count(&d), "packed image size mismatch (run qnet_pack first)");
  mm_qfwd_io io{};
  io.obs = obs.data_ptr<float>();
  io.obs_se = obs.stride(0);
  io.obs_sa = obs.stride(1);
  io.h_in = hidden.data_ptr<float>();
  io.hin_se = hidden.stride(0);
  io.hin_sa = hidden.stride(1);
  io.hin_sf = hidden.stride(2);
  io.h_out = hidden_out.data_ptr<float>();
  io.hout_se = hidden_out.stride(0);
  io.hout_sa = hidden_out.stride(1);
  io.hout_sf = hidden_out.stride(2);
  return io;
}

void en_out(const at::Tensor& t, int64_t E, int64_t N, at::ScalarType dt, const at::Tensor& like, const char* name) {
  need(t, dt, name);
  same_device(like, t, name);
  TORCH_CHECK(t.numel() == E * N, name, " must hold [E, N] = ", E * N, " elements");
}

void agent_q_fwd(const at::Tensor& packed, std::vector<int64_t> dims, const at::Tensor& obs, const at::Tensor& hidden,
                 at::Tensor hidden_out, at::Tensor q) {
  const mm_qnet_dims d = dims_of(dims);
  mm_qfwd_io io = base_io(d, packed, obs, hidden, hidden_out);
  const int64_t E = obs.size(0);
  TORCH_CHECK(q.is_cuda() && q.scalar_type() == at::kFloat && q.dim() == 3 && q.size(0) == E &&
                  q.size(1) == d.n_agents && q.size(2) == d.n_actions && q.stride(2) == 1,
              "q must be float [E, N, A] with unit action stride");
  same_device(obs, q, "q");
  io.q_out = q.data_ptr<float>();
  io.q_se = q.stride(0);
  io.q_sa = q.stride(1);
  io.mode = MM_Q_NONE;
  const c10::hip::HIPGuardMasqueradingAsCUDA g(obs.device());
  ok(mm_agent_q_fwd(&d, packed.data_ptr<float>(), &io, E, stream_of(obs)), "agent_q_fwd");
}

void agent_q_act(const at::Tensor& packed, std::vector<int64_t> dims, const at::Tensor& obs, const at::Tensor& hidden,
                 double epsilon, const c10::optional<at::Tensor>& u, const c10::optional<at::Tensor>& rand_act,
                 int64_t seed, int64_t counter, at::Tensor hidden_out, at::Tensor act, at::Tensor q_taken,
                 const c10::optional<at::Tensor>& q) {
  const mm_qnet_dims d = dims_of(dims);
  mm_qfwd_io io = base_io(d, packed, obs, hidden, hidden_out);
  const int64_t E = obs.size(0);
  en_out(act, E, d.n_agents, at::kInt, obs, "act");
  en_out(q_taken, E, d.n_agents, at::kFloat, obs, "q_taken");
  TORCH_CHECK(u.has_value() == rand_act.has_value(), "u and rand_act are injected together");
  if (u.has_value()) {
    need(*u, at::kFloat, "u");
    need(*rand_act, at::kInt, "rand_act");
    TORCH_CHECK(u->numel() == E && rand_act->numel() == E * d.n_agents, "u [E] / rand_act [E, N] size mismatch");
    io.u = u->data_ptr<float>();
    io.rand_act = rand_act->data_ptr<int32_t>();
  }
  if (q.has_value()) {
    TORCH_CHECK(q->is_cuda() && q->scalar_type() == at::kFloat && q->dim() == 3 && q->size(0) == E &&
                    q->size(1) == d.n_agents && q->size(2) == d.n_actions && q->stride(2) == 1,
                "q must be float [E, N, A] with unit action stride");
    same_device(obs, *q, "q");
    io.q_out = q->data_ptr<float>();
    io.q_se = q->stride(0);
    io.q_sa = q->stride(1);
  }
  io.mode = MM_Q_ACT;
  io.epsilon = (float)epsilon;
  io.seed = (uint64_t)seed;
  io.counter = (uint64_t)counter;
  io.act_out = act.data_ptr<int32_t>();
  io.qsel_out = q_taken.data_ptr<float>();
  const c10::hip::HIPGuardMasqueradingAsCUDA g(obs.device());
  ok(mm_agent_q_fwd(&d, packed.data_ptr<float>(), &io, E, stream_of(obs)), "agent_q_act");
}

void agent_q_max(const at::Tensor& packed, std::vector<int64_t> dims, const at::Tensor& obs, const at::Tensor& hidden,
                 at::Tensor hidden_out, at::Tensor max_q) {
  const mm_qnet_dims d = dims_of(dims);
  mm_qfwd_io io = base_io(d, packed, obs, hidden, hidden_out);
  const int64_t E = obs.size(0);
  en_out(max_q, E, d.n_agents, at::kFloat, obs, "max_q");
  io.mode = MM_Q_MAX;
  io.qsel_out = max_q.data_ptr<float>();
  const c10::hip::HIPGuardMasqueradingAsCUDA g(obs.device());
  ok(mm_agent_q_fwd(&d, packed.data_ptr<float>(), &io, E, stream_of(obs)), "agent_q_max");
}

// ------------------------------------------------------------------ TD error, GAE
void td_error(const at::Tensor& rew, const at::Tensor& done, const at::Tensor& q_taken, const at::Tensor& max_q_next,
              double gamma, at::Tensor td) {
  need(rew, at::kFloat, "rew");
  TORCH_CHECK(rew.dim() == 2, "rew must be [E, N]");
  const int64_t E = rew.size(0), N = rew.size(1);
  need(done, at::kByte, "done");
  TORCH_CHECK(done.numel() == E, "done must be uint8 [E]");
  en_out(q_taken, E, N, at::kFloat, rew, "q_taken");
  en_out(max_q_next, E, N, at::kFloat, rew, "max_q_next");
  need(td, at::kFloat, "td");
  TORCH_CHECK(td.numel() == E, "td must be [E]");
  same_device(rew, done, "done");
  same_device(rew, td, "td");
  // cal_td_error of one step = the chunk-TD kernel at step 0 of a 1-step chunk with no store writes
  const c10::hip::HIPGuardMasqueradingAsCUDA g(rew.device());
  ok(mm_td_chunk_step(E, (int32_t)N, (float)gamma, rew.data_ptr<float>(), done.data_ptr<uint8_t>(),
                      q_taken.data_ptr<float>(), max_q_next.data_ptr<float>(), nullptr, td.data_ptr<float>(), 0, 1,
                      nullptr, nullptr, nullptr, 0, stream_of(rew)),
     "td_error");
}

void gae_scan(const at::Tensor& rewards, const at::Tensor& value_preds, const at::Tensor& masks,
              const at::Tensor& value_norm, double gamma, double gae_lambda, at::Tensor returns) {
  need(rewards, at::kFloat, "rewards");
  TORCH_CHECK(rewards.dim() == 2, "rewards must be [T, EN]");
  const int64_t T = rewards.size(0), EN = rewards.size(1);
  const at::Tensor* ts[3] = {&value_preds, &masks, &returns};
  const char* names[3] = {"value_preds", "masks", "returns"};
  for (int i = 0; i < 3; ++i) {
    need(*ts[i], at::kFloat, names[i]);
    same_device(rewards, *ts[i], names[i]);
    TORCH_CHECK(ts[i]->numel() == (T + 1) * EN, names[i], " must be [T+1, EN]");
  }
  need(value_norm, at::kFloat, "value_norm");
  TORCH_CHECK(value_norm.numel() == 3, "value_norm = [running_mean, running_mean_sq, debiasing_term]");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(rewards.device());
  ok(mm_mappo_gae(rewards.data_ptr<float>(), value_preds.data_ptr<float>(), masks.data_ptr<float>(),
                  returns.data_ptr<float>(), value_norm.data_ptr<float>(), (int32_t)T, EN, (float)gamma,
                  (float)gae_lambda, stream_of(rewards)),
     "gae_scan");
}

// ------------------------------------------------------------------ QMIX mixer, TD loss, VDN sum
struct MixDims {
  int32_t N, S, Hm, K1;
  int64_t n_params, save_dim, delta_dim;
};
MixDims mix_dims(const std::vector<int64_t>& d) {
  TORCH_CHECK(d.size() == 4, "mixer dims must be [n_agents, state_dim, mixer_hidden, hypernet_k1]");
  MixDims m{(int32_t)d[0], (int32_t)d[1], (int32_t)d[2], (int32_t)d[3], 0, 0, 0};
  ok(mm_mixer_param_count(m.S, m.Hm, m.K1, m.N, &m.n_params), "mixer dims");
  m.save_dim = mm_mixer_save_dim(m.Hm, m.K1, m.N);
  m.delta_dim = mm_mixer_delta_dim(m.Hm, m.K1, m.N);
  return m;
}

void rows_of(const at::Tensor& t, int64_t B, int64_t width, at::ScalarType dt, const at::Tensor& like, const char* name) {
  need(t, dt, name);
  same_device(like, t, name);
  TORCH_CHECK(t.numel() == B * width, name, " must hold [", B, ", ", width, "] elements, got ", t.sizes());
}

// Mix_Net.forward of one step: Q_tot[b] = mix(q[b], state[b]) with the GRU hidden h -> h_out (rows where
// reset[b] != 0 start from zeros); save [B, mixer_save_dim] keeps what qmix_mixer_bwd needs.
void qmix_mixer_fwd(const at::Tensor& P, std::vector<int64_t> dims, const at::Tensor& q, const at::Tensor& state,
                    const at::Tensor& h, const c10::optional<at::Tensor>& reset, at::Tensor qtot, at::Tensor h_out,
                    const c10::optional<at::Tensor>& save) {
  const MixDims m = mix_dims(dims);
  need(P, at::kFloat, "P");
  TORCH_CHECK(P.numel() == m.n_params, "P has ", P.numel(), " elements, the mixer needs ", m.n_params);
  need(state, at::kFloat, "state");
  TORCH_CHECK(state.dim() >= 1 && state.numel() % m.S == 0, "state must be [B, state_dim]");
  const int64_t B = state.numel() / m.S;
  TORCH_CHECK(B >= 1, "empty batch");
  rows_of(q, B, m.N, at::kFloat, state, "q");
  rows_of(h, B, m.Hm, at::kFloat, state, "h");
  rows_of(h_out, B, m.Hm, at::kFloat, state, "h_out");
  rows_of(qtot, B, 1, at::kFloat, state, "qtot");
  same_device(state, P, "P");
  if (reset.has_value()) rows_of(*reset, B, 1, at::kByte, state, "reset");
  if (save.has_value()) rows_of(*save, B, m.save_dim, at::kFloat, state, "save");
  mm_mix_net n{};
  n.P = P.data_ptr<float>();
  n.gi = nullptr;
  n.q = q.data_ptr<float>();
  n.s_off = nullptr;                         // contiguous state rows
  n.h_in = h.data_ptr<float>();
  n.reset = reset.has_value() ? reset->data_ptr<uint8_t>() : nullptr;
  n.h_out = h_out.data_ptr<float>();
  n.qtot = qtot.data_ptr<float>();
  n.save = save.has_value() ? save->data_ptr<float>() : nullptr;
  const c10::hip::HIPGuardMasqueradingAsCUDA g(state.device());
  ok(mm_mixer_fwd((int32_t)B, m.N, m.S, m.Hm, m.K1, state.data_ptr<float>(), state.data_ptr<float>(), &n, 1,
                  stream_of(state)),
     "qmix_mixer_fwd");
}

int64_t qmix_mixer_workspace(std::vector<int64_t> dims, int64_t B) {
  const MixDims m = mix_dims(dims);
  TORCH_CHECK(B >= 1, "B must be >= 1");
  const int64_t part = mm_mixer_wgrad_partial_count((int32_t)B, m.N, m.S, m.Hm, m.K1);
  TORCH_CHECK(part >= 0, "mixer workspace: bad dims");
  return ((B * m.delta_dim + 3) & ~int64_t(3)) + part;
}

// Backward of one qmix_mixer_fwd step: dqtot [B] -> dq [B, N] (dQ_tot/dq_i), dh (in: the gradient w.r.t. h_out,
// dropped where drop[b] > 0.5 — the next step restarted from zeros; out: the gradient w.r.t. h), dP [n_params]
// (every Mix_Net parameter gradient, MIX_KEYS order, overwritten). workspace: qmix_mixer_workspace(dims, B) floats.
void qmix_mixer_bwd(const at::Tensor& P, std::vector<int64_t> dims, const at::Tensor& state, const at::Tensor& save,
                    const at::Tensor& q, const at::Tensor& dqtot, const at::Tensor& drop, at::Tensor dh, at::Tensor dq,
                    at::Tensor dP, at::Tensor workspace) {
  const MixDims m = mix_dims(dims);
  need(P, at::kFloat, "P");
  TORCH_CHECK(P.numel() == m.n_params, "P has ", P.numel(), " elements, the mixer needs ", m.n_params);
  need(state, at::kFloat, "state");
  const int64_t B = state.numel() / m.S;
  TORCH_CHECK(B >= 1 && B * m.S == state.numel(), "state must be [B, state_dim]");
  rows_of(save, B, m.save_dim, at::kFloat, state, "save");
  rows_of(q, B, m.N, at::kFloat, state, "q");
  rows_of(dqtot, B, 1, at::kFloat, state, "dqtot");
  rows_of(drop, B, 1, at::kFloat, state, "drop");
  rows_of(dh, B, m.Hm, at::kFloat, state, "dh");
  rows_of(dq, B, m.N, at::kFloat, state, "dq");
  need(dP, at::kFloat, "dP");
  TORCH_CHECK(dP.numel() == m.n_params, "dP must hold the mixer's ", m.n_params, " parameters");
  need(workspace, at::kFloat, "workspace");
  const int64_t need_ws = qmix_mixer_workspace(dims, B);
  TORCH_CHECK(workspace.numel() >= need_ws, "workspace has ", workspace.numel(), " floats, needs ", need_ws,
              " (qmix_mixer_workspace)");
  same_device(state, P, "P");
  same_device(state, dP, "dP");
  same_device(state, workspace, "workspace");
  float* delta = workspace.data_ptr<float>();
  const int64_t doff = (B * m.delta_dim + 3) & ~int64_t(3);
  const c10::hip::HIPGuardMasqueradingAsCUDA g(state.device());
  const mm_stream_t st = stream_of(state);
  ok(mm_mixer_bwd((int32_t)B, m.N, m.S, m.Hm, m.K1, P.data_ptr<float>(), save.data_ptr<float>(), q.data_ptr<float>(),
                  dqtot.data_ptr<float>(), drop.data_ptr<float>(), dh.data_ptr<float>(), dq.data_ptr<float>(), delta,
                  st),
     "qmix_mixer_bwd");
  ok(mm_mixer_wgrad((int32_t)B, m.N, m.S, m.Hm, m.K1, state.data_ptr<float>(), nullptr, nullptr,
                    save.data_ptr<float>(), delta, dP.data_ptr<float>(), delta + doff, workspace.numel() - doff, st),
     "qmix_mixer_bwd (weight gradients)");
}

// TD targets + loss over a chunk (rows t*B + b): y = w_b * sum_i (r_i + gamma (1-d) Q'_tot) (the reference,
// flags 0) or sum_i r_i + gamma (1-d) Q'_tot (flag 4 = MM_LOSS_TARGET_SUM, no IS weight); MSE (or smooth-L1,
// flag 2) mean over B summed over C; dqtot = dLoss/dQ_tot; td_last = |y - Q_tot| of the last step (priorities).
void td_target_loss(const at::Tensor& rew, const at::Tensor& done, const c10::optional<at::Tensor>& is_weight,
                    const at::Tensor& qtot, const at::Tensor& qtot_target, double gamma, int64_t flags,
                    at::Tensor dqtot, at::Tensor td_last, at::Tensor loss, at::Tensor loss_parts) {
  TORCH_CHECK((flags & ~(int64_t)(MM_LOSS_HUBER | MM_LOSS_TARGET_SUM)) == 0,
              "flags: MM_LOSS_HUBER (2) | MM_LOSS_TARGET_SUM (4); VDN sums Q with vdn_sum first");
  need(rew, at::kFloat, "rew");
  TORCH_CHECK(rew.dim() == 3, "rew must be [C, B, N]");
  const int64_t C = rew.size(0), B = rew.size(1), N = rew.size(2);
  rows_of(done, C * B, 1, at::kFloat, rew, "done");
  rows_of(qtot, C * B, 1, at::kFloat, rew, "qtot");
  rows_of(qtot_target, C * B, 1, at::kFloat, rew, "qtot_target");
  rows_of(dqtot, C * B, 1, at::kFloat, rew, "dqtot");
  rows_of(loss_parts, C * B, 1, at::kFloat, rew, "loss_parts");
  rows_of(td_last, B, 1, at::kFloat, rew, "td_last");
  rows_of(loss, 1, 1, at::kFloat, rew, "loss");
  TORCH_CHECK((flags & MM_LOSS_TARGET_SUM) || is_weight.has_value(), "is_weight required (reference target)");
  if (is_weight.has_value()) rows_of(*is_weight, B, 1, at::kFloat, rew, "is_weight");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(rew.device());
  ok(mm_lrn_loss_ex((int32_t)B, (int32_t)C, (int32_t)N, (float)gamma, rew.data_ptr<float>(), done.data_ptr<float>(),
                    is_weight.has_value() ? is_weight->data_ptr<float>() : nullptr, qtot.data_ptr<float>(),
                    qtot_target.data_ptr<float>(), (int32_t)flags, nullptr, nullptr, dqtot.data_ptr<float>(), nullptr,
                    loss_parts.data_ptr<float>(), td_last.data_ptr<float>(), loss.data_ptr<float>(), stream_of(rew)),
     "td_target_loss");
}

void vdn_sum(const at::Tensor& q, const c10::optional<at::Tensor>& act, at::Tensor out) {
  TORCH_CHECK(q.is_cuda() && q.scalar_type() == at::kFloat && q.dim() == 3 && q.stride(2) == 1,
              "q must be a float GPU tensor [B, N, A] with unit action stride");
  const int64_t B = q.size(0), N = q.size(1), A = q.size(2);
  rows_of(out, B, 1, at::kFloat, q, "out");
  if (act.has_value()) rows_of(*act, B, N, at::kInt, q, "act");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  ok(mm_vdn_sum(B, (int32_t)N, (int32_t)A, q.data_ptr<float>(), q.stride(0), q.stride(1),
                act.has_value() ? act->data_ptr<int32_t>() : nullptr, out.data_ptr<float>(), nullptr, stream_of(q)),
     "vdn_sum");
}

// ------------------------------------------------------------------ MAPPO actor / critic
mm_mappo_dims mappo_dims(const std::vector<int64_t>& d, const at::Tensor& actor_P, const at::Tensor& critic_P) {
  TORCH_CHECK(d.size() == 3, "MAPPO dims must be [obs_dim, hidden, n_actions]");
  mm_mappo_dims m{(int32_t)d[0], (int32_t)d[1], (int32_t)d[2]};
  need(actor_P, at::kFloat, "actor_P");
  need(critic_P, at::kFloat, "critic_P");
  same_device(actor_P, critic_P, "critic_P");
  TORCH_CHECK(actor_P.numel() == mm_mappo_param_count(&m, 0), "actor_P has ", actor_P.numel(),
              " elements, the actor needs ", mm_mappo_param_count(&m, 0));
  TORCH_CHECK(critic_P.numel() == mm_mappo_param_count(&m, 1), "critic_P has ", critic_P.numel(),
              " elements, the critic needs ", mm_mappo_param_count(&m, 1));
  return m;
}

// get_actions: rows R = E*N, one recurrent step (h <- h * mask), sample (device counter RNG or injected
// uniforms u [R]) or, deterministic, the mode; writes both nets' new hiddens, actions, log-probs, values.
void mappo_get_actions(const at::Tensor& actor_P, const at::Tensor& critic_P, std::vector<int64_t> dims,
                       const at::Tensor& obs, const at::Tensor& h_actor, const at::Tensor& h_critic,
                       const c10::optional<at::Tensor>& masks, const c10::optional<at::Tensor>& u, int64_t seed,
                       int64_t counter, bool deterministic, at::Tensor h_actor_out, at::Tensor h_critic_out,
                       at::Tensor actions, at::Tensor logp, at::Tensor values) {
  const mm_mappo_dims m = mappo_dims(dims, actor_P, critic_P);
  need(obs, at::kFloat, "obs");
  TORCH_CHECK(obs.numel() % m.obs_dim == 0, "obs must be [R, obs_dim]");
  const int64_t R = obs.numel() / m.obs_dim;
  TORCH_CHECK(R >= 1, "empty batch");
  same_device(obs, actor_P, "actor_P");
  rows_of(h_actor, R, m.hidden, at::kFloat, obs, "h_actor");
  rows_of(h_critic, R, m.hidden, at::kFloat, obs, "h_critic");
  rows_of(h_actor_out, R, m.hidden, at::kFloat, obs, "h_actor_out");
  rows_of(h_critic_out, R, m.hidden, at::kFloat, obs, "h_critic_out");
  rows_of(actions, R, 1, at::kInt, obs, "actions");
  rows_of(logp, R, 1, at::kFloat, obs, "logp");
  rows_of(values, R, 1, at::kFloat, obs, "values");
  if (masks.has_value()) rows_of(*masks, R, 1, at::kFloat, obs, "masks");
  if (u.has_value()) rows_of(*u, R, 1, at::kFloat, obs, "u");
  mm_mappo_fwd_args a{};
  a.net[0] = {actor_P.data_ptr<float>(), h_actor.data_ptr<float>(), h_actor_out.data_ptr<float>(),
              logp.data_ptr<float>(), nullptr};
  a.net[1] = {critic_P.data_ptr<float>(), h_critic.data_ptr<float>(), h_critic_out.data_ptr<float>(),
              values.data_ptr<float>(), nullptr};
  a.obs = obs.data_ptr<float>();
  a.mask = masks.has_value() ? masks->data_ptr<float>() : nullptr;
  a.act_out = actions.data_ptr<int32_t>();
  a.u = u.has_value() ? u->data_ptr<float>() : nullptr;
  a.seed = (uint64_t)seed;
  a.counter = (uint64_t)counter;
  a.rows = R;
  a.mode = MM_MAPPO_ROLLOUT;
  a.deterministic = deterministic ? 1 : 0;
  const c10::hip::HIPGuardMasqueradingAsCUDA g(obs.device());
  ok(mm_mappo_fwd(&m, &a, stream_of(obs)), "mappo_get_actions");
}

int64_t mappo_eval_rs(int64_t rows) { return (rows + 63) / 64 * 64; }

int64_t mappo_evaluate_workspace(std::vector<int64_t> dims, int64_t rows) {
  TORCH_CHECK(dims.size() == 3 && rows >= 1, "dims [obs_dim, hidden, n_actions], rows >= 1");
  mm_mappo_dims m{(int32_t)dims[0], (int32_t)dims[1], (int32_t)dims[2]};
  const int64_t rs = mappo_eval_rs(rows);
  return (int64_t)(mm_mappo_save_fields(&m, 0) + mm_mappo_save_fields(&m, 1)) * rs + rs;
}

// evaluate_actions over n recurrent chunks of L steps (rows l*n + j, shared_buffer.py:318-427 order):
// chunk-start hiddens h_actor0 / h_critic0 [n, H], masks [L*n] (h <- h * mask every step) -> values, log-probs of
// actions [L*n], entropy [1] = the active-masked mean of the Categorical entropies.
void mappo_evaluate_actions(const at::Tensor& actor_P, const at::Tensor& critic_P, std::vector<int64_t> dims,
                            const at::Tensor& obs, const at::Tensor& h_actor0, const at::Tensor& h_critic0,
                            const at::Tensor& actions, const at::Tensor& masks,
                            const c10::optional<at::Tensor>& active_masks, int64_t L, at::Tensor values,
                            at::Tensor logp, at::Tensor entropy, at::Tensor workspace) {
  const mm_mappo_dims m = mappo_dims(dims, actor_P, critic_P);
  need(obs, at::kFloat, "obs");
  TORCH_CHECK(L >= 1 && obs.numel() % (m.obs_dim * L) == 0, "obs must be [L * n, obs_dim]");
  const int64_t rows = obs.numel() / m.obs_dim, n = rows / L;
  same_device(obs, actor_P, "actor_P");
  rows_of(h_actor0, n, m.hidden, at::kFloat, obs, "h_actor0");
  rows_of(h_critic0, n, m.hidden, at::kFloat, obs, "h_critic0");
  rows_of(actions, rows, 1, at::kInt, obs, "actions");
  rows_of(masks, rows, 1, at::kFloat, obs, "masks");
  if (active_masks.has_value()) rows_of(*active_masks, rows, 1, at::kFloat, obs, "active_masks");
  rows_of(values, rows, 1, at::kFloat, obs, "values");
  rows_of(logp, rows, 1, at::kFloat, obs, "logp");
  rows_of(entropy, 1, 1, at::kFloat, obs, "entropy");
  need(workspace, at::kFloat, "workspace");
  same_device(obs, workspace, "workspace");
  TORCH_CHECK(workspace.numel() >= mappo_evaluate_workspace(dims, rows), "workspace too small (mappo_evaluate_workspace)");
  const int64_t rs = mappo_eval_rs(rows);
  float* ws = workspace.data_ptr<float>();
  mm_mappo_fwd_args a{};
  a.net[0] = {actor_P.data_ptr<float>(), h_actor0.data_ptr<float>(), nullptr, nullptr, ws};
  a.net[1] = {critic_P.data_ptr<float>(), h_critic0.data_ptr<float>(), nullptr, nullptr,
              ws + (int64_t)mm_mappo_save_fields(&m, 0) * rs};
  a.obs = obs.data_ptr<float>();
  a.mask = masks.data_ptr<float>();
  a.en = n;
  a.T = (int32_t)L;
  a.L = (int32_t)L;
  a.rs = rs;
  a.mode = MM_MAPPO_TRAIN;
  float* ent_rows = ws + (int64_t)(mm_mappo_save_fields(&m, 0) + mm_mappo_save_fields(&m, 1)) * rs;
  const c10::hip::HIPGuardMasqueradingAsCUDA g(obs.device());
  ok(mm_mappo_evaluate_actions(&m, &a, actions.data_ptr<int32_t>(),
                               active_masks.has_value() ? active_masks->data_ptr<float>() : nullptr,
                               values.data_ptr<float>(), logp.data_ptr<float>(), ent_rows, entropy.data_ptr<float>(),
                               nullptr, stream_of(obs)),
     "mappo_evaluate_actions");
}

// ------------------------------------------------------------------ env (custom class)
struct Env : torch::CustomClassHolder {
  mm_env* h = nullptr;
  int64_t E, N, D;
  c10::Device dev;
  Env(int64_t n_envs, int64_t n_agents, int64_t max_steps, double step_cost, bool full_observable, int64_t device)
      : E(n_envs), N(n_agents), dev(c10::DeviceType::CUDA, (c10::DeviceIndex)device) {
    const c10::hip::HIPGuardMasqueradingAsCUDA g(dev);
    mm_env_cfg cfg{(int32_t)n_agents, (int32_t)max_steps, full_observable ? 1 : 0, 8, (float)step_cost};
    ok(mm_env_create(&cfg, n_envs, 0, &h), "Env");
    D = mm_env_obs_dim(h);
  }
  ~Env() override {
    if (h) mm_env_destroy(h);
  }
  int64_t obs_dim() const { return D; }
  void check_obs(const at::Tensor& t, const char* name) const {
    need(t, at::kFloat, name);
    TORCH_CHECK(t.device() == dev, name, " must be on ", dev);
    TORCH_CHECK(t.numel() == E * N * D, name, " must hold [E, N, D] = [", E, ", ", N, ", ", D, "]");
  }
  void reset(at::Tensor obs) {
    check_obs(obs, "obs");
    const c10::hip::HIPGuardMasqueradingAsCUDA g(dev);
    ok(mm_env_reset(h, obs.data_ptr<float>(), stream_of(obs)), "Env.reset");
  }
  // next_obs: terminal next obs; obs_cur: auto-reset current obs (undefined tensor = not written)
  void step(const at::Tensor& act, at::Tensor next_obs, c10::optional<at::Tensor> obs_cur, at::Tensor rew,
            at::Tensor done) {
    need(act, at::kInt, "act");
    TORCH_CHECK(act.device() == dev && act.numel() == E * N, "act must be int32 [E, N] on ", dev);
    check_obs(next_obs, "next_obs");
    if (obs_cur.has_value()) check_obs(*obs_cur, "obs_cur");
    need(rew, at::kFloat, "rew");
    TORCH_CHECK(rew.device() == dev && rew.numel() == E * N, "rew must be float [E, N] on ", dev);
    need(done, at::kByte, "done");
    TORCH_CHECK(done.device() == dev && done.numel() == E, "done must be uint8 [E] on ", dev);
    const c10::hip::HIPGuardMasqueradingAsCUDA g(dev);
    ok(mm_env_step(h, act.data_ptr<int32_t>(), next_obs.data_ptr<float>(),
                   obs_cur.has_value() ? obs_cur->data_ptr<float>() : nullptr, rew.data_ptr<float>(),
                   done.data_ptr<uint8_t>(), stream_of(act)),
       "Env.step");
  }
};

// ------------------------------------------------------------------ prioritized replay (custom class)
struct PER : torch::CustomClassHolder {
  mm_per* h = nullptr;
  c10::Device dev;
  PER(int64_t capacity, std::string flavor, double alpha, double beta, double eps, double step_weight,
      bool use_step_weight, double alpha_inc, double beta_inc, int64_t device)
      : dev(c10::DeviceType::CUDA, (c10::DeviceIndex)device) {
    TORCH_CHECK(flavor == "vdn" || flavor == "qmix", "flavor must be 'vdn' or 'qmix'");
    const c10::hip::HIPGuardMasqueradingAsCUDA g(dev);
    ok(mm_per_create(capacity, flavor == "vdn" ? MM_PER_VDN : MM_PER_QMIX, alpha, beta, eps, step_weight,
                     use_step_weight ? 1 : 0, alpha_inc, beta_inc, &h),
       "PER");
  }
  ~PER() override {
    if (h) mm_per_destroy(h);
  }
  int64_t size() const { return mm_per_size(h); }
  int64_t capacity() const { return mm_per_capacity(h); }
  double alpha() const { return mm_per_alpha(h); }
  double beta() const { return mm_per_beta(h); }
  // collect_sample of K chunks at once: td [K] f32 -> slots [K] int64
  void insert(const at::Tensor& td, at::Tensor slots) {
    need(td, at::kFloat, "td");
    need(slots, at::kLong, "slots");
    TORCH_CHECK(td.device() == dev && slots.device() == dev && slots.numel() == td.numel(), "td / slots mismatch");
    const c10::hip::HIPGuardMasqueradingAsCUDA g(dev);
    ok(mm_per_insert(h, td.data_ptr<float>(), td.numel(), nullptr, slots.data_ptr<int64_t>(), stream_of(td)),
       "PER.insert");
  }
  // sample(B): injected stratum fractions (f64 [B]) or the device counter RNG (fracs undefined)
  void sample(c10::optional<at::Tensor> fracs, int64_t seed, int64_t counter, at::Tensor nodes, at::Tensor slots,
              at::Tensor is_weight) {
    need(nodes, at::kLong, "nodes");
    need(slots, at::kLong, "slots");
    need(is_weight, at::kFloat, "is_weight");
    const int64_t B = nodes.numel();
    TORCH_CHECK(slots.numel() == B && is_weight.numel() == B && nodes.device() == dev, "sample outputs mismatch");
    TORCH_CHECK(size() > 0, "PER.sample: empty replay");
    const c10::hip::HIPGuardMasqueradingAsCUDA g(dev);
    if (fracs.has_value()) {
      need(*fracs, at::kDouble, "fracs");
      TORCH_CHECK(fracs->numel() == B && fracs->device() == dev, "fracs must be f64 [B] on ", dev);
      ok(mm_per_sample(h, (int32_t)B, fracs->data_ptr<double>(), nodes.data_ptr<int64_t>(), slots.data_ptr<int64_t>(),
                       is_weight.data_ptr<float>(), stream_of(nodes)),
         "PER.sample");
    } else {
      ok(mm_per_sample_rng(h, (int32_t)B, (uint64_t)seed, (uint64_t)counter, nodes.data_ptr<int64_t>(),
                           slots.data_ptr<int64_t>(), is_weight.data_ptr<float>(), stream_of(nodes)),
         "PER.sample");
    }
  }
  void update(const at::Tensor& nodes, const at::Tensor& td) {
    need(nodes, at::kLong, "nodes");
    need(td, at::kFloat, "td");
    TORCH_CHECK(nodes.numel() == td.numel() && nodes.device() == dev && td.device() == dev, "nodes / td mismatch");
    const c10::hip::HIPGuardMasqueradingAsCUDA g(dev);
    ok(mm_per_update(h, nodes.data_ptr<int64_t>(), td.data_ptr<float>(), (int32_t)nodes.numel(), stream_of(td)),
       "PER.update");
  }
  at::Tensor tree() const {
    auto out = at::empty({2 * capacity() - 1}, at::TensorOptions().dtype(at::kDouble).device(dev));
    const c10::hip::HIPGuardMasqueradingAsCUDA g(dev);
    ok(mm_per_copy_tree(h, out.data_ptr<double>(), stream_of(out)), "PER.tree");
    return out;
  }
};

}  // namespace

TORCH_LIBRARY(minimarl, m) {
  m.def("qnet_pack(Tensor params, int[] dims, Tensor(a!) packed) -> ()");
  m.def("agent_q_fwd(Tensor packed, int[] dims, Tensor obs, Tensor hidden, Tensor(a!) hidden_out, "
        "Tensor(b!) q) -> ()");
  m.def("agent_q_act(Tensor packed, int[] dims, Tensor obs, Tensor hidden, float epsilon, Tensor? u, "
        "Tensor? rand_act, int seed, int counter, Tensor(a!) hidden_out, Tensor(b!) act, Tensor(c!) q_taken, "
        "Tensor(d!)? q=None) -> ()");
  m.def("agent_q_max(Tensor packed, int[] dims, Tensor obs, Tensor hidden, Tensor(a!) hidden_out, "
        "Tensor(b!) max_q) -> ()");
  m.def("td_error(Tensor rew, Tensor done, Tensor q_taken, Tensor max_q_next, float gamma, Tensor(a!) td) -> ()");
  m.def("gae_scan(Tensor rewards, Tensor value_preds, Tensor masks, Tensor value_norm, float gamma, "
        "float gae_lambda, Tensor(a!) returns) -> ()");
  m.def("qmix_mixer_fwd(Tensor P, int[] dims, Tensor q, Tensor state, Tensor h, Tensor? reset, Tensor(a!) qtot, "
        "Tensor(b!) h_out, Tensor(c!)? save=None) -> ()");
  m.def("qmix_mixer_workspace(int[] dims, int B) -> int");
  m.def("qmix_mixer_bwd(Tensor P, int[] dims, Tensor state, Tensor save, Tensor q, Tensor dqtot, Tensor drop, "
        "Tensor(a!) dh, Tensor(b!) dq, Tensor(c!) dP, Tensor(d!) workspace) -> ()");
  m.def("td_target_loss(Tensor rew, Tensor done, Tensor? is_weight, Tensor qtot, Tensor qtot_target, float gamma, "
        "int flags, Tensor(a!) dqtot, Tensor(b!) td_last, Tensor(c!) loss, Tensor(d!) loss_parts) -> ()");
  m.def("vdn_sum(Tensor q, Tensor? act, Tensor(a!) out) -> ()");
  m.def("mappo_get_actions(Tensor actor_P, Tensor critic_P, int[] dims, Tensor obs, Tensor h_actor, Tensor h_critic, "
        "Tensor? masks, Tensor? u, int seed, int counter, bool deterministic, Tensor(a!) h_actor_out, "
        "Tensor(b!) h_critic_out, Tensor(c!) actions, Tensor(d!) logp, Tensor(e!) values) -> ()");
  m.def("mappo_evaluate_workspace(int[] dims, int rows) -> int");
  m.def("mappo_evaluate_actions(Tensor actor_P, Tensor critic_P, int[] dims, Tensor obs, Tensor h_actor0, "
        "Tensor h_critic0, Tensor actions, Tensor masks, Tensor? active_masks, int L, Tensor(a!) values, "
        "Tensor(b!) logp, Tensor(c!) entropy, Tensor(d!) workspace) -> ()");
  m.class_<Env>("Env")
      .def(torch::init<int64_t, int64_t, int64_t, double, bool, int64_t>())
      .def("obs_dim", &Env::obs_dim)
      .def("reset", &Env::reset)
      .def("step", &Env::step);
  m.class_<PER>("PER")
      .def(torch::init<int64_t, std::string, double, double, double, double, bool, double, double, int64_t>())
      .def("size", &PER::size)
      .def("capacity", &PER::capacity)
      .def("alpha", &PER::alpha)
      .def("beta", &PER::beta)
      .def("insert", &PER::insert)
      .def("sample", &PER::sample)
      .def("update", &PER::update)
      .def("tree", &PER::tree);
}

TORCH_LIBRARY_IMPL(minimarl, CUDA, m) {
  m.impl("qnet_pack", qnet_pack);
  m.impl("agent_q_fwd", agent_q_fwd);
  m.impl("agent_q_act", agent_q_act);
  m.impl("agent_q_max", agent_q_max);
  m.impl("td_error", td_error);
  m.impl("gae_scan", gae_scan);
  m.impl("qmix_mixer_fwd", qmix_mixer_fwd);
  m.impl("qmix_mixer_bwd", qmix_mixer_bwd);
  m.impl("td_target_loss", td_target_loss);
  m.impl("vdn_sum", vdn_sum);
  m.impl("mappo_get_actions", mappo_get_actions);
  m.impl("mappo_evaluate_actions", mappo_evaluate_actions);
}

// size queries: no tensor arguments, so they dispatch on the catch-all kernel
TORCH_LIBRARY_IMPL(minimarl, CompositeExplicitAutograd, m) {
  m.impl("qmix_mixer_workspace", qmix_mixer_workspace);
  m.impl("mappo_evaluate_workspace", mappo_evaluate_workspace);
}
