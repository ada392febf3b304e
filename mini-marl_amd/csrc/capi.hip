// extern "C" surface of libminimarl (see include/minimarl.h) + error plumbing.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "minimarl.h"
#include "qnet_geo.h"

namespace mm {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int qnet_pack(const mm_qnet_dims* d, const float* params, float* packed, hipStream_t s, int f32_only);
int agent_q_rec_seq2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t e0,
                     const float* packed1, const mm_qfwd_io* io1, int64_t e1, int32_t steps, const uint8_t* reset,
                     hipStream_t s);
int agent_q_fwd(const mm_qnet_dims* d, const float* packed, const mm_qfwd_io* io, int64_t n_envs, hipStream_t s);
int agent_q_fwd2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t e0,
                 const float* packed1, const mm_qfwd_io* io1, int64_t e1, hipStream_t s);
int agent_q_split2(int phase, const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t e0,
                   const float* packed1, const mm_qfwd_io* io1, int64_t e1, hipStream_t s);
size_t rollout_step_lds(const mm_env* env, const mm_qnet_dims* d, int64_t n_envs);
size_t rollout_chunk_lds(const mm_env* env, const mm_qnet_dims* d, int64_t n_envs);
int rollout_chunk(mm_env* env, const mm_qnet_dims* d, const float* packed_t, const mm_qfwd_io* io_t,
                  const float* packed_b, const mm_qfwd_io* io_b, int64_t n_envs, const mm_rollout_chunk_io* x,
                  hipStream_t s);
int rollout_step(mm_env* env, const mm_qnet_dims* d, const float* packed_t, const mm_qfwd_io* io_t,
                 const float* packed_b, const mm_qfwd_io* io_b, int64_t n_envs, const mm_rollout_step_io* x,
                 hipStream_t s);
}  // namespace mm

extern "C" {

const char* mm_last_error(void) { return mm::g_err; }
int mm_version(void) { return 100; }

int mm_qnet_param_offsets(const mm_qnet_dims* d, int64_t offs[11]) {
  mm::QnetOffsets o;
  int rc = mm::qnet_offsets(d, &o);
  if (rc) return rc;
  const int64_t v[11] = {o.W1, o.b1, o.W2, o.b2, o.Wih, o.Whh, o.bih, o.bhh, o.Wq, o.bq, o.total};
  for (int i = 0; i < 11; ++i) offs[i] = v[i];
  return MM_OK;
}

int64_t mm_qnet_packed_count(const mm_qnet_dims* d) {
  mm::QnetGeo g;
  mm::QnetOffsets o;
  if (mm::qnet_geometry(d, &g, &o)) return -1;
  // [fp32 fragment image | fp16x3-split image | per-agent fp16x3 safety flags (int, padded to 64)]
  return 2 * g.agent_stride * d->n_agents + ((d->n_agents + 63) & ~63);
}

int mm_qnet_pack(const mm_qnet_dims* d, const float* params, float* packed, mm_stream_t s) {
  MM_REQUIRE(params && packed, "qnet_pack: null pointer");
  return mm::qnet_pack(d, params, packed, (hipStream_t)s, 0);
}

int mm_qnet_pack_f32(const mm_qnet_dims* d, const float* params, float* packed, mm_stream_t s) {
  MM_REQUIRE(params && packed, "qnet_pack_f32: null pointer");
  return mm::qnet_pack(d, params, packed, (hipStream_t)s, 1);
}

int mm_agent_q_fwd(const mm_qnet_dims* d, const float* packed, const mm_qfwd_io* io, int64_t n_envs,
                   mm_stream_t s) {
  return mm::agent_q_fwd(d, packed, io, n_envs, (hipStream_t)s);
}

int mm_agent_q_fwd2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t n_envs0,
                    const float* packed1, const mm_qfwd_io* io1, int64_t n_envs1, mm_stream_t s) {
  return mm::agent_q_fwd2(d, packed0, io0, n_envs0, packed1, io1, n_envs1, (hipStream_t)s);
}

int mm_rollout_step_supported(const mm_env* env, const mm_qnet_dims* d, int64_t n_envs) {
  return mm::rollout_step_lds(env, d, n_envs) > 0 ? 1 : 0;
}

int mm_rollout_chunk_supported(const mm_env* env, const mm_qnet_dims* d, int64_t n_envs) {
  return mm::rollout_chunk_lds(env, d, n_envs) > 0 ? 1 : 0;
}

int mm_rollout_chunk(mm_env* env, const mm_qnet_dims* d, const float* packed_t, const mm_qfwd_io* io_t,
                     const float* packed_b, const mm_qfwd_io* io_b, int64_t n_envs, const mm_rollout_chunk_io* x,
                     mm_stream_t s) {
  return mm::rollout_chunk(env, d, packed_t, io_t, packed_b, io_b, n_envs, x, (hipStream_t)s);
}

int mm_rollout_step(mm_env* env, const mm_qnet_dims* d, const float* packed_t, const mm_qfwd_io* io_t,
                    const float* packed_b, const mm_qfwd_io* io_b, int64_t n_envs, const mm_rollout_step_io* x,
                    mm_stream_t s) {
  return mm::rollout_step(env, d, packed_t, io_t, packed_b, io_b, n_envs, x, (hipStream_t)s);
}

int mm_agent_q_pre2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t n_envs0,
                    const float* packed1, const mm_qfwd_io* io1, int64_t n_envs1, mm_stream_t s) {
  return mm::agent_q_split2(1, d, packed0, io0, n_envs0, packed1, io1, n_envs1, (hipStream_t)s);
}

int mm_agent_q_pre2_h3(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t n_envs0,
                       const float* packed1, const mm_qfwd_io* io1, int64_t n_envs1, mm_stream_t s) {
  return mm::agent_q_split2(3, d, packed0, io0, n_envs0, packed1, io1, n_envs1, (hipStream_t)s);
}

int mm_agent_q_rec_seq2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t n_envs0,
                        const float* packed1, const mm_qfwd_io* io1, int64_t n_envs1, int32_t steps,
                        const uint8_t* reset, mm_stream_t s) {
  return mm::agent_q_rec_seq2(d, packed0, io0, n_envs0, packed1, io1, n_envs1, steps, reset, (hipStream_t)s);
}

int mm_agent_q_rec2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t n_envs0,
                    const float* packed1, const mm_qfwd_io* io1, int64_t n_envs1, mm_stream_t s) {
  return mm::agent_q_split2(2, d, packed0, io0, n_envs0, packed1, io1, n_envs1, (hipStream_t)s);
}

int mm_agent_q_fwd_simple(const mm_qnet_dims* d, const float* packed, const float* obs, const float* h, float* q,
                          float* h_out, int64_t n_envs, mm_stream_t s) {
  MM_REQUIRE(d, "agent_q_fwd_simple: null dims");
  mm_qfwd_io io = {};
  io.obs = obs;
  io.obs_se = (int64_t)d->n_agents * d->obs_dim;
  io.obs_sa = d->obs_dim;
  io.h_in = h;
  io.hin_se = (int64_t)d->n_agents * d->h;
  io.hin_sa = d->h;
  io.hin_sf = 1;
  io.h_out = h_out;
  io.hout_se = io.hin_se;
  io.hout_sa = io.hin_sa;
  io.hout_sf = 1;
  io.q_out = q;
  io.q_se = (int64_t)d->n_agents * d->n_actions;
  io.q_sa = d->n_actions;
  io.mode = MM_Q_NONE;
  return mm::agent_q_fwd(d, packed, &io, n_envs, (hipStream_t)s);
}
}

// ---- debug timing traces (not part of the hot path; see common.h) ----
namespace mm {
static uint64_t* g_trace = nullptr;
int debug_trace_alloc() {
  if (g_trace) return 0;
  if (hipMalloc(&g_trace, 65536 * sizeof(uint64_t)) != hipSuccess) return -1;
  return hipMemset(g_trace, 0, 65536 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
uint64_t* debug_trace_buffer(const char* env_name) {
  const char* v = getenv(env_name);
  if (!v || v[0] == '0') return nullptr;
  return g_trace;   // allocated by mm_debug_trace(NULL, 0) beforehand
}
}  // namespace mm

extern "C" int mm_debug_trace(uint64_t* host_out, int32_t n) {
  if (!host_out && n == 0) return mm::debug_trace_alloc();  // allocate up front (not legal inside graph capture)
  if (!mm::g_trace || n <= 0 || n > 65536) { mm::set_error("mm_debug_trace: no trace buffer (set the trace env var) or bad n"); return -1; }
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpy(host_out, mm::g_trace, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess ? 0
                                                                                                          : -1;
}
