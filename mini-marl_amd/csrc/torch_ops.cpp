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
}
