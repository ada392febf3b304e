// MAPPO (rmappo, shared policy) hot path on gfx950: actor/critic trunk forward (rollout and
// chunked training), PPO + clipped-Huber value loss fused into the chunked BPTT backward,
// weight-gradient reduction on MFMA, GAE scan, advantage statistics, ValueNorm.
//
// Reference (behaviour restated in oracle/mappo.py, pinned by tests/golden/mappo_*.npz):
//   trunk  mappo/utils/algorithm_utils/mlp.py:31-55 (LN(D); [Linear, ReLU, LN] x 2),
//          rnn.py:24-29,79 (GRU on h*mask, LayerNorm on the output), act.py/distributions.py
//          (Categorical), r_actor_critic.py:189-208 (v_out)
//   train  mappo/algorithms/ramppo_network.py:56-209 (ppo_update, cal_value_loss),
//          shared_buffer.py:318-427 (chunks of L steps; start hidden = stored hidden)
//   GAE    shared_buffer.py:131-153 (+ valuenorm.py denormalize), f64 accumulator
//
// Design: hidden = 32, so one thread owns one row (rollout) or one L-step chunk (training):
// LayerNorm / softmax / GRU gates are plain per-thread code, every weight read is an LDS
// broadcast (the net's whole parameter vector, ~38 KB, is staged per block). The canonical
// flat parameter layout (MGeo) is 16-byte aligned with W1 rows padded to Dp, so it IS the LDS
// image (no pack step) and the Adam state shares it (pads stay exactly zero).
#include "common.h"
#include "minimarl.h"
#include "trunk.h"

namespace mm {


// One trunk step; fills the save slots if sv != nullptr.
template <int D, int H, int O>
struct Trunk {
  using G = MGeo<D, H, O>;
  using S = SF<H, O>;
  // sv: this row's column of a tiled SoA array (field stride 64, see soa_col)
  __device__ static __forceinline__ void step(const float* W, const float (&x)[D], float (&h)[H], float (&out)[O],
                                              float* sv) {
    float mu, rs;
    ln_stats<D>(x, mu, rs);
    float f0[D];
    ln_apply<D>(x, mu, rs, W + G::ln0_w, W + G::ln0_b, f0);
    if (sv) {
      sv[S::MU0 * 64] = mu;
      sv[S::RS0 * 64] = rs;
    }
    float a[H], f[H];
    matvec<H, D, G::Dp>(W + G::W1, W + G::b1, f0, a);
#pragma unroll
    for (int i = 0; i < H; ++i) a[i] = fmaxf(a[i], 0.0f);
    ln_stats<H>(a, mu, rs);
    if (sv) {
#pragma unroll
      for (int i = 0; i < H; ++i) sv[(S::A1 + i) * 64] = a[i];
      sv[S::MU1 * 64] = mu;
      sv[S::RS1 * 64] = rs;
    }
    ln_apply<H>(a, mu, rs, W + G::ln1_w, W + G::ln1_b, f);
    matvec<H, H, H>(W + G::W2, W + G::b2, f, a);
#pragma unroll
    for (int i = 0; i < H; ++i) a[i] = fmaxf(a[i], 0.0f);
    ln_stats<H>(a, mu, rs);
    if (sv) {
#pragma unroll
      for (int i = 0; i < H; ++i) sv[(S::A2 + i) * 64] = a[i];
      sv[S::MU2 * 64] = mu;
      sv[S::RS2 * 64] = rs;
    }
    ln_apply<H>(a, mu, rs, W + G::ln2_w, W + G::ln2_b, f);
    // GRU (torch gate order r, z, n; h' = n + z * (h - n))
#pragma unroll
    for (int j = 0; j < H; ++j) {
      float gir = W[G::bih + j], giz = W[G::bih + H + j], gin = W[G::bih + 2 * H + j];
      float ghr = W[G::bhh + j], ghz = W[G::bhh + H + j], ghn = W[G::bhh + 2 * H + j];
#pragma unroll
      for (int i = 0; i < H; ++i) {
        gir = fmaf(W[G::Wih + j * H + i], f[i], gir);
        giz = fmaf(W[G::Wih + (H + j) * H + i], f[i], giz);
        gin = fmaf(W[G::Wih + (2 * H + j) * H + i], f[i], gin);
        ghr = fmaf(W[G::Whh + j * H + i], h[i], ghr);
        ghz = fmaf(W[G::Whh + (H + j) * H + i], h[i], ghz);
        ghn = fmaf(W[G::Whh + (2 * H + j) * H + i], h[i], ghn);
      }
      const float r = sigmoidf_(gir + ghr);
      const float z = sigmoidf_(giz + ghz);
      const float n = tanhf_(gin + r * ghn);
      a[j] = n + z * (h[j] - n);  // new hidden (h still needed by later j)
      if (sv) {
        sv[(S::HIN + j) * 64] = h[j];
        sv[(S::R + j) * 64] = r;
        sv[(S::Z + j) * 64] = z;
        sv[(S::N + j) * 64] = n;
        sv[(S::GHN + j) * 64] = ghn;
      }
    }
#pragma unroll
    for (int j = 0; j < H; ++j) h[j] = a[j];
    ln_stats<H>(h, mu, rs);
    if (sv) {
#pragma unroll
      for (int j = 0; j < H; ++j) sv[(S::H2 + j) * 64] = h[j];
      sv[S::MUR * 64] = mu;
      sv[S::RSR * 64] = rs;
    }
    ln_apply<H>(h, mu, rs, W + G::lnr_w, W + G::lnr_b, f);
    matvec<O, H, H>(W + G::Wo, W + G::bo, f, out);
  }
};

// log-softmax in place (logits -> logp), returns entropy
template <int A>
__device__ __forceinline__ float log_softmax(float (&l)[A]) {
  float mx = l[0];
#pragma unroll
  for (int a = 1; a < A; ++a) mx = fmaxf(mx, l[a]);
  float s = 0.0f;
#pragma unroll
  for (int a = 0; a < A; ++a) s += expf(l[a] - mx);
  const float lse = mx + logf(s);
  float ent = 0.0f;
#pragma unroll
  for (int a = 0; a < A; ++a) {
    l[a] -= lse;
    ent -= expf(l[a]) * l[a];
  }
  return ent;
}

// ------------------------------------------------------------------ forward kernel
template <int D, int H, int A>
__device__ __forceinline__ void fwd_body(const mm_mappo_fwd_args& a, int net, float* sm) {
  using TA = Trunk<D, H, A>;
  using TC = Trunk<D, H, 1>;
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const mm_mappo_net_io& io = a.net[net];
  if (a.mode != MM_MAPPO_TRAIN) {
    // rollout / get_values: one row per thread
    if (tid >= a.rows) return;
    float x[D], h[H];
    load_row<D>(a.obs + tid * D, x);
    const float m = a.mask ? a.mask[tid] : 1.0f;
    load_row<H>(io.h_in + tid * H, h);
#pragma unroll
    for (int i = 0; i < H; ++i) h[i] *= m;
    if (net == 0) {
      float l[A];
      TA::step(sm, x, h, l, nullptr);
      log_softmax<A>(l);
      int act;
      if (a.act_in) {
        act = a.act_in[tid];
      } else if (a.deterministic) {
        // Categorical.mode() = first argmax of the probabilities (distributions.py:61-62)
        act = 0;
#pragma unroll
        for (int q = 1; q < A; ++q)
          if (l[q] > l[act]) act = q;
        if (a.act_out) a.act_out[tid] = act;
      } else {
        float u;
        if (a.u) {
          u = a.u[tid];
        } else {
          const uint64_t ctr = a.counter_ptr ? *a.counter_ptr : a.counter;
          u = rng_uniform(rng_draw(a.seed, ctr, (uint64_t)tid, 0x9E37ull));
        }
        // inverse CDF: first k with u < cumsum(p)[k], the last action if rounding leaves none
        act = A - 1;
        bool found = false;
        float cs = 0.0f;
#pragma unroll
        for (int q = 0; q < A; ++q) {
          cs += expf(l[q]);
          if (!found && u < cs) {
            act = q;
            found = true;
          }
        }
        if (a.act_out) a.act_out[tid] = act;
      }
      float lp = l[0];
#pragma unroll
      for (int k = 1; k < A; ++k)
        if (k == act) lp = l[k];
      if (io.out) io.out[tid] = lp;
    } else {
      float v[1];
      TC::step(sm, x, h, v, nullptr);
      if (io.out) io.out[tid] = v[0];
    }
    if (io.h_out) {
#pragma unroll
      for (int i = 0; i < H; ++i) io.h_out[tid * H + i] = h[i];
    }
    return;
  }
  // training: one L-step chunk per thread; chunk c = k * EN + en covers t = k*L .. k*L+L-1
  const int64_t EN = a.en, n_chunks = (int64_t)(a.T / a.L) * EN;
  if (tid >= n_chunks) return;
  const int64_t k = tid / EN, en = tid - k * EN;
  float h[H];
  load_row<H>(io.h_in + ((k * a.L) * EN + en) * H, h);
  for (int l = 0; l < a.L; ++l) {
    const int64_t row = (k * a.L + l) * EN + en;
    float x[D];
    load_row<D>(a.obs + row * D, x);
    const float m = a.mask[row];
#pragma unroll
    for (int i = 0; i < H; ++i) h[i] *= m;
    if (net == 0) {
      float* sv = soa_col(io.save, row, SF<H, A>::NS);
      float lg[A];
      TA::step(sm, x, h, lg, sv);
      log_softmax<A>(lg);
#pragma unroll
      for (int q = 0; q < A; ++q) sv[(SF<H, A>::OUT + q) * 64] = lg[q];
    } else {
      float* sv = soa_col(io.save, row, SF<H, 1>::NS);
      float v[1];
      TC::step(sm, x, h, v, sv);
      sv[SF<H, 1>::OUT * 64] = v[0];
    }
  }
}

template <int D, int H, int A>
__global__ __launch_bounds__(256) void mappo_fwd_kernel(mm_mappo_fwd_args a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int net = (int)blockIdx.y + (a.mode == MM_MAPPO_VALUES ? 1 : 0);
  const int n = net == 0 ? MGeo<D, H, A>::total : MGeo<D, H, 1>::total;
  stage_params(sm, a.net[net].P, n);
  if (net == 0)
    fwd_body<D, H, A>(a, 0, sm);
  else
    fwd_body<D, H, A>(a, 1, sm);
}

// ------------------------------------------------------------------ backward kernel
// Per chunk, reverse over its L steps: loss seed (PPO clipped surrogate + entropy for the
// actor, ValueNorm-targeted clipped Huber for the critic), then BPTT through head, LN_r, GRU,
// LN2/L2, LN1/L1, LN0. Writes the (delta, input) operand pairs of every weight gradient.
struct LossSeed {
  float clip, huber_delta, entropy_coef, value_coef;
};

__device__ __forceinline__ float huber_d(float e, float d) { return fabsf(e) <= d ? e : (e > 0.f ? d : -d); }
__device__ __forceinline__ float huber_f(float e, float d) {
  return fabsf(e) <= d ? e * e * 0.5f : d * (fabsf(e) - d * 0.5f);
}


template <int D, int H, int A, int O>
__device__ __forceinline__ void bwd_body(const mm_mappo_bwd_args& a, int net, const float* W) {
  using G = MGeo<D, H, O>;
  using S = SF<H, O>;
  using GF_ = GF<D, H, O>;
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t EN = a.en, n_chunks = (int64_t)(a.T / a.L) * EN;
  if (tid >= n_chunks) return;
  const int64_t k = tid / EN, en = tid - k * EN;
  const float* sv0 = a.save[net];
  float* go0 = a.gsoa[net];
  const float inv_m = 1.0f / a.stats[MM_MST_ACTIVE_SUM];
  float dh_next[H];
#pragma unroll
  for (int i = 0; i < H; ++i) dh_next[i] = 0.0f;
  float lsum0 = 0.f, lsum1 = 0.f, lsum2 = 0.f;
  for (int l = a.L - 1; l >= 0; --l) {
    const int64_t row = (k * a.L + l) * EN + en;
    const float* sv = soa_col(sv0, row, S::NS);
    float* go = soa_col(go0, row, GF_::NG);
    const float m = a.active[row];
    // ---- loss seed d(out)
    float dout[O];
    if constexpr (O == A) {
      float lp[A];
      soa_ld<A>(sv, S::OUT, lp);
      float ent = 0.0f;
#pragma unroll
      for (int q = 0; q < A; ++q) ent -= expf(lp[q]) * lp[q];
      const int act = a.act[row];
      float lpa = lp[0];
#pragma unroll
      for (int q = 1; q < A; ++q)
        if (q == act) lpa = lp[q];
      const float adv = (a.adv[row] - a.stats[MM_MST_ADV_MEAN]) / (a.stats[MM_MST_ADV_STD] + 1e-5f);
      const float ratio = expf(lpa - a.old_logp[row]);
      const float s1 = ratio * adv;
      const float rc = fminf(fmaxf(ratio, 1.0f - a.clip), 1.0f + a.clip);
      const float s2 = rc * adv;
      const float inr = (ratio >= 1.0f - a.clip && ratio <= 1.0f + a.clip) ? 1.0f : 0.0f;
      // torch.min backward: the smaller side gets the gradient, ties split it in half
      const float g = s1 < s2 ? 1.0f : (s1 > s2 ? inr : 0.5f + 0.5f * inr);
      const float dlpa = -m * inv_m * adv * ratio * g;
      const float dent = -a.entropy_coef * m * inv_m;
      lsum0 += -fminf(s1, s2) * m;
      lsum1 += ent * m;
      lsum2 += ratio;
#pragma unroll
      for (int q = 0; q < A; ++q) {
        const float p = expf(lp[q]);
        dout[q] = dlpa * ((q == act ? 1.0f : 0.0f) - p) + dent * (-p * (lp[q] + ent));
      }
    } else {
      const float v = soa_ld1(sv, S::OUT);
      const float old = a.old_value[row];
      const float tgt = (a.returns[row] - a.stats[MM_MST_VN_MEAN]) / a.stats[MM_MST_VN_STD];
      const float dv = v - old;
      const float vc = old + fminf(fmaxf(dv, -a.clip), a.clip);
      const float eo = tgt - v, ec = tgt - vc;
      const float lo = huber_f(eo, a.huber_delta), lc = huber_f(ec, a.huber_delta);
      const float go_ = -huber_d(eo, a.huber_delta);
      const float gc = -huber_d(ec, a.huber_delta) * ((dv >= -a.clip && dv <= a.clip) ? 1.0f : 0.0f);
      const float d = lo > lc ? go_ : (lc > lo ? gc : 0.5f * (go_ + gc));
      dout[0] = a.value_coef * m * inv_m * d;
      lsum0 += fmaxf(lo, lc) * m;
    }
    // ---- head: y = LN_r(h2); out = Wo y + bo
    float xr[H], t[H];
    soa_ld<H>(sv, S::H2, t);
    {
      const float mur = soa_ld1(sv, S::MUR), rsr = soa_ld1(sv, S::RSR);
      float y[H];
#pragma unroll
      for (int i = 0; i < H; ++i) {
        xr[i] = (t[i] - mur) * rsr;
        y[i] = xr[i] * W[G::lnr_w + i] + W[G::lnr_b + i];
      }
      soa_st<O>(go, GF_::DOUT, dout);
      soa_st<H>(go, GF_::Y, y);
      float dy[H], dh[H];
      matvec_t<O, H, H>(W + G::Wo, dout, dy);
      ln_bwd<H>(dy, xr, rsr, W + G::lnr_w, dh);
      soa_st<H>(go, GF_::DY, dy);
#pragma unroll
      for (int i = 0; i < H; ++i) {
        t[i] = dy[i] * xr[i];
        xr[i] = dh[i] + dh_next[i];  // xr now holds d(h2)
      }
      soa_st<H>(go, GF_::PY, t);
    }
    // ---- GRU (h2 = n + z (h - n), gates r, z, n), streamed over hidden units j so that only the
    // accumulators Wih^T dgi (-> dx2) and Whh^T dgh (-> dh_prev) stay live
    float dx[H], dhh[H];
#pragma unroll
    for (int i = 0; i < H; ++i) {
      dx[i] = 0.0f;
      dhh[i] = 0.0f;
    }
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const float r = soa_ld1(sv, S::R + j), z = soa_ld1(sv, S::Z + j), n = soa_ld1(sv, S::N + j);
      const float ghn = soa_ld1(sv, S::GHN + j), hin = soa_ld1(sv, S::HIN + j);
      const float dh = xr[j];
      const float dn = dh * (1.0f - z);
      const float dz = dh * (hin - n);
      const float dpn = dn * (1.0f - n * n);
      const float dgr = dpn * ghn * r * (1.0f - r);
      const float dgz = dz * z * (1.0f - z);
      const float dghn = dpn * r;
      dh_next[j] = dh * z;  // direct path; Whh^T dgh added below
      soa_st1(go, GF_::DGI + j, dgr);
      soa_st1(go, GF_::DGI + H + j, dgz);
      soa_st1(go, GF_::DGI + 2 * H + j, dpn);
      soa_st1(go, GF_::DGH + j, dgr);
      soa_st1(go, GF_::DGH + H + j, dgz);
      soa_st1(go, GF_::DGH + 2 * H + j, dghn);
      soa_st1(go, GF_::HIN + j, hin);
#pragma unroll
      for (int i = 0; i < H; ++i) {
        dx[i] = fmaf(W[G::Wih + j * H + i], dgr, dx[i]);
        dx[i] = fmaf(W[G::Wih + (H + j) * H + i], dgz, dx[i]);
        dx[i] = fmaf(W[G::Wih + (2 * H + j) * H + i], dpn, dx[i]);
        dhh[i] = fmaf(W[G::Whh + j * H + i], dgr, dhh[i]);
        dhh[i] = fmaf(W[G::Whh + (H + j) * H + i], dgz, dhh[i]);
        dhh[i] = fmaf(W[G::Whh + (2 * H + j) * H + i], dghn, dhh[i]);
      }
    }
    {
      const float mk = a.mask[row];
#pragma unroll
      for (int i = 0; i < H; ++i) dh_next[i] = (dh_next[i] + dhh[i]) * mk;
    }
    // ---- x2 = LN2(a2) (input of the GRU); dx = d x2 from the GRU
    float ah[H], xh[H], da[H];
    {
      soa_ld<H>(sv, S::A2, ah);
      const float mu = soa_ld1(sv, S::MU2), rs = soa_ld1(sv, S::RS2);
#pragma unroll
      for (int i = 0; i < H; ++i) {
        xh[i] = (ah[i] - mu) * rs;
        t[i] = xh[i] * W[G::ln2_w + i] + W[G::ln2_b + i];
      }
      soa_st<H>(go, GF_::X2, t);
      ln_bwd<H>(dx, xh, rs, W + G::ln2_w, da);
#pragma unroll
      for (int i = 0; i < H; ++i) {
        t[i] = dx[i] * xh[i];
        da[i] = ah[i] > 0.0f ? da[i] : 0.0f;
      }
      soa_st<H>(go, GF_::DX2, dx);
      soa_st<H>(go, GF_::P2, t);
      soa_st<H>(go, GF_::DPRE2, da);
    }
    // ---- x1 = LN1(a1) (input of L2)
    {
      soa_ld<H>(sv, S::A1, ah);
      const float mu = soa_ld1(sv, S::MU1), rs = soa_ld1(sv, S::RS1);
#pragma unroll
      for (int i = 0; i < H; ++i) {
        xh[i] = (ah[i] - mu) * rs;
        t[i] = xh[i] * W[G::ln1_w + i] + W[G::ln1_b + i];
      }
      soa_st<H>(go, GF_::F1, t);
      matvec_t<H, H, H>(W + G::W2, da, dx);
      ln_bwd<H>(dx, xh, rs, W + G::ln1_w, da);
#pragma unroll
      for (int i = 0; i < H; ++i) {
        t[i] = dx[i] * xh[i];
        da[i] = ah[i] > 0.0f ? da[i] : 0.0f;
      }
      soa_st<H>(go, GF_::DX1, dx);
      soa_st<H>(go, GF_::P1, t);
      soa_st<H>(go, GF_::DPRE1, da);
    }
    // ---- f0 = LN0(obs) (input of L1)
    {
      float x0[D], df0[D];
      load_row<D>(a.obs + row * D, x0);
      const float mu = soa_ld1(sv, S::MU0), rs = soa_ld1(sv, S::RS0);
      matvec_t<H, D, G::Dp>(W + G::W1, da, df0);
      soa_st<D>(go, GF_::DF0, df0);
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const float xh0 = (x0[i] - mu) * rs;
        df0[i] *= xh0;
        x0[i] = xh0 * W[G::ln0_w + i] + W[G::ln0_b + i];
      }
      soa_st<D>(go, GF_::P0, df0);
      soa_st<D>(go, GF_::F0, x0);
    }
  }
  if (a.loss_acc) {
    // logging only (train_info): wave-level sums, one atomic per wave
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lsum0 += __shfl_xor(lsum0, o);
      lsum1 += __shfl_xor(lsum1, o);
      lsum2 += __shfl_xor(lsum2, o);
    }
    if ((threadIdx.x & 63) == 0) {
      if constexpr (O == A) {
        atomicAdd(&a.loss_acc[MM_MLOSS_POLICY], lsum0 * inv_m);
        atomicAdd(&a.loss_acc[MM_MLOSS_ENTROPY], lsum1 * inv_m);
        atomicAdd(&a.loss_acc[MM_MLOSS_RATIO], lsum2);
      } else {
        atomicAdd(&a.loss_acc[MM_MLOSS_VALUE], lsum0 * inv_m);
      }
    }
  }
}

template <int D, int H, int A>
__global__ __launch_bounds__(256, 2) void mappo_bwd_kernel(mm_mappo_bwd_args a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int net = blockIdx.y;
  const int n = net == 0 ? MGeo<D, H, A>::total : MGeo<D, H, 1>::total;
  stage_params(sm, a.P[net], n);
  if (net == 0)
    bwd_body<D, H, A, A>(a, 0, sm);
  else
    bwd_body<D, H, A, 1>(a, 1, sm);
}


// ------------------------------------------------------------------ GAE, advantages, ValueNorm
// ValueNorm state (f32, valuenorm.py): vn[0] running_mean, vn[1] running_mean_sq, vn[2] debias.
__device__ __forceinline__ void vn_mean_var(const float* vn, float& mean, float& var) {
  const float d = fmaxf(vn[2], 1e-5f);
  mean = vn[0] / d;
  const float msq = vn[1] / d;
  var = fmaxf(msq - mean * mean, 1e-2f);
}

// returns[t] for t < T, one thread per (env, agent) column; delta in f32, gae in f64 (shared_buffer.py:141-148)
__global__ __launch_bounds__(256) void mappo_gae_kernel(const float* __restrict__ rew, const float* __restrict__ vp,
                                                        const float* __restrict__ masks, float* __restrict__ ret,
                                                        const float* __restrict__ vn, int T, int64_t EN, float gamma,
                                                        float gl) {
#pragma clang fp contract(off)
  const int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (c >= EN) return;
  float mean, var;
  vn_mean_var(vn, mean, var);
  const float sd = sqrtf(var);
  double gae = 0.0;
  float dn1 = vp[(int64_t)T * EN + c] * sd + mean;
  for (int t = T - 1; t >= 0; --t) {
    const float dn0 = vp[(int64_t)t * EN + c] * sd + mean;
    const float m1 = masks[(int64_t)(t + 1) * EN + c];
    const float delta = (rew[(int64_t)t * EN + c] + (gamma * dn1) * m1) - dn0;
    gae = (double)delta + (double)(gl * m1) * gae;
    ret[(int64_t)t * EN + c] = (float)(gae + (double)dn0);
    dn1 = dn0;
  }
}

// adv = returns - denorm(value_preds) over t < T; block partials [5] of (sum, count, sum of squares)
// over active rows plus (sum ret, sum ret^2) over all rows (the ValueNorm batch moments).
__global__ __launch_bounds__(256) void mappo_adv_kernel(const float* __restrict__ ret, const float* __restrict__ vp,
                                                        const float* __restrict__ active, const float* __restrict__ vn,
                                                        float* __restrict__ adv, int64_t R, double* __restrict__ part) {
#pragma clang fp contract(off)
  __shared__ double sh[5][256];
  float mean, var;
  vn_mean_var(vn, mean, var);
  const float sd = sqrtf(var);
  double s = 0, n = 0, sr = 0, sr2 = 0, s2 = 0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < R; i += (int64_t)gridDim.x * 256) {
    const float v = ret[i] - (vp[i] * sd + mean);
    adv[i] = v;
    if (active[i] != 0.0f) {
      s += v;
      n += 1.0;
      s2 += (double)v * v;
    }
    sr += ret[i];
    sr2 += (double)ret[i] * ret[i];
  }
  sh[0][threadIdx.x] = s;
  sh[1][threadIdx.x] = n;
  sh[2][threadIdx.x] = sr;
  sh[3][threadIdx.x] = sr2;
  sh[4][threadIdx.x] = s2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int q = 0; q < 5; ++q) sh[q][threadIdx.x] += sh[q][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 5) part[blockIdx.x * 5 + threadIdx.x] = sh[threadIdx.x][0];
}

// second pass (np.nanstd is two-pass): sum of squared deviations from the masked mean
__global__ __launch_bounds__(256) void mappo_adv_var_kernel(const float* __restrict__ adv,
                                                            const float* __restrict__ active, int64_t R,
                                                            const double* __restrict__ part, int nb,
                                                            double* __restrict__ part2) {
  __shared__ double sh[256];
  __shared__ double s_mean;
  if (threadIdx.x == 0) {
    double s = 0, n = 0;
    for (int b = 0; b < nb; ++b) {
      s += part[b * 5];
      n += part[b * 5 + 1];
    }
    s_mean = n > 0 ? s / n : 0.0;
  }
  __syncthreads();
  const double mu = s_mean;
  double q = 0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < R; i += (int64_t)gridDim.x * 256)
    if (active[i] != 0.0f) q += ((double)adv[i] - mu) * ((double)adv[i] - mu);
  sh[threadIdx.x] = q;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part2[blockIdx.x] = sh[0];
}

// stats[]: adv mean/std, active count, ValueNorm batch moments; sums[5] = the raw sums
// (sum adv, count, sum ret, sum ret^2, sum adv^2) for a data-parallel all-reduce.
__global__ void mappo_stats_kernel(const double* part, const double* part2, int nb, int64_t R, float* stats,
                                   double* sums) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0, n = 0, sr = 0, sr2 = 0, s2 = 0, q = 0;
  for (int b = 0; b < nb; ++b) {
    s += part[b * 5];
    n += part[b * 5 + 1];
    sr += part[b * 5 + 2];
    sr2 += part[b * 5 + 3];
    s2 += part[b * 5 + 4];
    q += part2[b];
  }
  stats[MM_MST_ADV_MEAN] = (float)(n > 0 ? s / n : 0.0);
  stats[MM_MST_ADV_STD] = (float)(n > 0 ? sqrt(q / n) : 0.0);
  stats[MM_MST_ACTIVE_SUM] = (float)n;
  stats[MM_MST_RET_MEAN] = (float)(sr / (double)R);
  stats[MM_MST_RET_SQ_MEAN] = (float)(sr2 / (double)R);
  sums[0] = s;
  sums[1] = n;
  sums[2] = sr;
  sums[3] = sr2;
  sums[4] = s2;
}

// stats from all-reduced sums (replicas of a data-parallel job see the global statistics)
__global__ void mappo_stats_from_sums_kernel(const double* sums, int64_t R, float* stats) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double s = sums[0], n = sums[1], sr = sums[2], sr2 = sums[3], s2 = sums[4];
  const double mu = n > 0 ? s / n : 0.0;
  stats[MM_MST_ADV_MEAN] = (float)mu;
  stats[MM_MST_ADV_STD] = (float)(n > 0 ? sqrt(fmax(s2 / n - mu * mu, 0.0)) : 0.0);
  stats[MM_MST_ACTIVE_SUM] = (float)n;
  stats[MM_MST_RET_MEAN] = (float)(sr / (double)R);
  stats[MM_MST_RET_SQ_MEAN] = (float)(sr2 / (double)R);
}

// One ValueNorm.update(returns) (valuenorm.py:37-54, f32, weight = beta) followed by the
// normalisation constants for this epoch's value loss.
__global__ void mappo_vn_update_kernel(float* vn, float* stats, float w, float omw) {
#pragma clang fp contract(off)
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  vn[0] = vn[0] * w + stats[MM_MST_RET_MEAN] * omw;
  vn[1] = vn[1] * w + stats[MM_MST_RET_SQ_MEAN] * omw;
  vn[2] = vn[2] * w + omw;
  float mean, var;
  vn_mean_var(vn, mean, var);
  stats[MM_MST_VN_MEAN] = mean;
  stats[MM_MST_VN_STD] = sqrtf(var);
}

// Rollout insert after env.step (magym_runner.py:151-195): masks[t+1] = 0 and zero hiddens for
// done envs, active masks 1 (env-level done: every agent finishes together).
__global__ __launch_bounds__(256) void mappo_insert_kernel(const uint8_t* __restrict__ done, int N, int H, int64_t E,
                                                           float* __restrict__ mask_next, float* __restrict__ active_next,
                                                           float* __restrict__ ha, float* __restrict__ hc,
                                                           uint64_t* counter) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;  // (env, agent, feature) over E*N*H
  if (i == 0 && counter) *counter += 1;  // device RNG step counter of the next rollout step
  if (i >= E * N * H) return;
  const int64_t row = i / H, e = row / N;
  const bool d = done[e] != 0;
  if (d) {
    ha[i] = 0.0f;
    hc[i] = 0.0f;
  }
  if (i % H == 0) {
    mask_next[row] = d ? 0.0f : 1.0f;
    active_next[row] = 1.0f;
  }
}

// ------------------------------------------------------------------ host dispatch
int mappo_roll_fwd(const mm_mappo_dims* d, const mm_mappo_fwd_args* a, hipStream_t s);   // mappo_grad.hip

template <int D, int H, int A>
struct MappoShape {
  using GA = MGeo<D, H, A>;
  using GC = MGeo<D, H, 1>;
  static int fwd(const mm_mappo_fwd_args* a, hipStream_t s) {
    if (a->mode != MM_MAPPO_TRAIN && H == 32) {   // rollout / get_values: the MFMA forward (mappo_grad.hip)
      const mm_mappo_dims d{D, H, A};
      return mappo_roll_fwd(&d, a, s);
    }
    const int64_t n = a->mode == MM_MAPPO_TRAIN ? (int64_t)(a->T / a->L) * a->en : a->rows;
    if (n <= 0) return MM_OK;
    const int nets = a->mode == MM_MAPPO_VALUES ? 1 : 2;
    hipLaunchKernelGGL((mappo_fwd_kernel<D, H, A>), dim3((unsigned)((n + 255) / 256), nets), dim3(256),
                       (size_t)GA::total * 4, s, *a);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  static int bwd(const mm_mappo_bwd_args* a, hipStream_t s) {
    const int64_t n = (int64_t)(a->T / a->L) * a->en;
    if (n <= 0) return MM_OK;
    hipLaunchKernelGGL((mappo_bwd_kernel<D, H, A>), dim3((unsigned)((n + 255) / 256), 2), dim3(256),
                       (size_t)GA::total * 4, s, *a);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  using TW = TrunkWgrad<D, H>;
  static int64_t partial_count(int64_t Rs) {
    WgJobDev jv[2 * MM_MAPPO_MAX_JOBS];
    const int64_t nblk = (Rs + TW::rows_per_block(Rs) - 1) / TW::rows_per_block(Rs);
    int64_t tot = 0;
    for (int net = 0; net < 2; ++net) {
      const int nj = net == 0 ? TW::template jobs<A>(nullptr, Rs, nullptr, jv) : TW::template jobs<1>(nullptr, Rs, nullptr, jv);
      for (int q = 0; q < nj; ++q) tot += nblk * (int64_t)(jv[q].M * jv[q].K + jv[q].M);
    }
    return tot;
  }
  static int wgrad(int net, const float* gsoa, int64_t Rs, float* grad, float* partial, hipStream_t s) {
    return net == 0 ? TW::template wgrad<A>(gsoa, Rs, grad, partial, s) : TW::template wgrad<1>(gsoa, Rs, grad, partial, s);
  }
};

// evaluate_actions epilogue (r_actor_critic.py:95-140, act.py:40-82, distributions.py:55-68) after a
// TRAIN-mode forward: per row the critic value, the log-prob of the given action from the actor's
// log-softmax save fields, and the Categorical entropy -sum_a p_a log p_a; then the masked mean of the
// entropies over active_masks (or the plain mean) in one workgroup, fixed order (deterministic).
template <int H, int A>
__global__ __launch_bounds__(256) void mappo_eval_rows_kernel(const float* __restrict__ save0,
                                                              const float* __restrict__ save1, int64_t rows,
                                                              const int32_t* __restrict__ act,
                                                              float* __restrict__ values, float* __restrict__ logp,
                                                              float* __restrict__ ent_rows, int32_t* __restrict__ err) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  using S0 = SF<H, A>;
  using S1 = SF<H, 1>;
  const float* c0 = soa_col(save0, r, S0::NS);
  float lp[A];
  soa_ld<A>(c0, S0::OUT, lp);
  float ent = 0.0f;
#pragma unroll
  for (int q = 0; q < A; ++q) ent -= expf(lp[q]) * lp[q];
  const int a = act[r];
  if ((a < 0 || a >= A) && err) atomicOr(err, 1);
  float lpa = 0.0f;
#pragma unroll
  for (int q = 0; q < A; ++q)
    if (q == a) lpa = lp[q];
  values[r] = soa_ld1(soa_col(save1, r, S1::NS), S1::OUT);
  logp[r] = lpa;
  ent_rows[r] = ent;
}

__global__ __launch_bounds__(1024) void masked_mean_kernel(const float* __restrict__ x, const float* __restrict__ m,
                                                           int64_t rows, float* __restrict__ out) {
  __shared__ float sx[1024], sm[1024];
  float ax = 0.f, am = 0.f;
  for (int64_t r = threadIdx.x; r < rows; r += 1024) {
    const float w = m ? m[r] : 1.0f;
    ax += x[r] * w;
    am += w;
  }
  sx[threadIdx.x] = ax;
  sm[threadIdx.x] = am;
  __syncthreads();
  for (int st = 512; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) {
      sx[threadIdx.x] += sx[threadIdx.x + st];
      sm[threadIdx.x] += sm[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = sx[0] / sm[0];
}

template <int H, int A>
static int mappo_eval_launch(const mm_mappo_fwd_args* a, const int32_t* act, const float* active, float* values,
                             float* logp, float* ent_rows, float* entropy, int32_t* err, hipStream_t s) {
  const int64_t rows = (int64_t)a->T * a->en;
  hipLaunchKernelGGL((mappo_eval_rows_kernel<H, A>), dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s,
                     a->net[0].save, a->net[1].save, rows, act, values, logp, ent_rows, err);
  MM_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(masked_mean_kernel, dim3(1), dim3(1024), 0, s, ent_rows, active, rows, entropy);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

#define MM_MAPPO_DISPATCH(d, CALL)                                                  \
  do {                                                                              \
    if ((d)->hidden == 32 && (d)->n_actions == 5 && (d)->obs_dim == 47) {           \
      using SH = mm::MappoShape<47, 32, 5>;                                           \
      return CALL;                                                                  \
    }                                                                               \
    if ((d)->hidden == 32 && (d)->n_actions == 5 && (d)->obs_dim == 94) {           \
      using SH = mm::MappoShape<94, 32, 5>;                                           \
      return CALL;                                                                  \
    }                                                                               \
    mm::set_error("mappo: unsupported dims D=%d H=%d A=%d (supported: D 47|94, H 32, A 5)", (d)->obs_dim, \
              (d)->hidden, (d)->n_actions);                                         \
    return MM_EINVAL;                                                               \
  } while (0)

static int64_t param_count(const mm_mappo_dims* d, int net) {
  if (d->hidden == 32 && d->n_actions == 5 && d->obs_dim == 47)
    return net == 0 ? MGeo<47, 32, 5>::total : MGeo<47, 32, 1>::total;
  if (d->hidden == 32 && d->n_actions == 5 && d->obs_dim == 94)
    return net == 0 ? MGeo<94, 32, 5>::total : MGeo<94, 32, 1>::total;
  return -1;
}

}  // namespace mm

// ------------------------------------------------------------------ C ABI
extern "C" {

int64_t mm_mappo_param_count(const mm_mappo_dims* d, int32_t net) {
  if (!d || net < 0 || net > 1) return -1;
  return mm::param_count(d, net);
}

int mm_mappo_param_offsets(const mm_mappo_dims* d, int32_t net, int64_t offs[19]) {
  MM_REQUIRE(d && offs && (net == 0 || net == 1), "mappo_param_offsets: bad args");
  MM_REQUIRE(mm::param_count(d, net) > 0, "mappo: unsupported dims D=%d H=%d A=%d", d->obs_dim, d->hidden,
             d->n_actions);
  const int H = d->hidden, O = net == 0 ? d->n_actions : 1;
  const int Dp = (d->obs_dim + 3) & ~3, Op = (O + 3) & ~3;
  int64_t c = 0;
  const int64_t sz[18] = {Dp, Dp, (int64_t)H * Dp, H, H, H, (int64_t)H * H, H, H, H, 3ll * H * H, 3ll * H * H,
                          3 * H, 3 * H, H, H, (int64_t)Op * H, Op};
  for (int i = 0; i < 18; ++i) {
    offs[i] = c;
    c += sz[i];
  }
  offs[18] = c;
  return MM_OK;
}

int mm_mappo_save_fields(const mm_mappo_dims* d, int32_t net) {
  if (!d) return -1;
  return 8 + 8 * d->hidden + (net == 0 ? d->n_actions : 1);
}

int mm_mappo_grad_fields(const mm_mappo_dims* d, int32_t net) {
  if (!d) return -1;
  return (net == 0 ? d->n_actions : 1) + 18 * d->hidden + 3 * d->obs_dim;
}

int mm_mappo_fwd(const mm_mappo_dims* d, const mm_mappo_fwd_args* a, mm_stream_t s) {
  MM_REQUIRE(d && a, "mappo_fwd: null argument");
  MM_REQUIRE(a->obs && a->net[1].P && a->net[1].h_in, "mappo_fwd: obs / critic params / hiddens required");
  MM_REQUIRE(a->mode == MM_MAPPO_VALUES || (a->net[0].P && a->net[0].h_in), "mappo_fwd: actor params required");
  MM_REQUIRE(a->mode != MM_MAPPO_TRAIN ||
                 (a->L > 0 && a->T % a->L == 0 && a->mask && a->net[0].save && a->net[1].save && a->rs >= a->T * a->en),
             "mappo_fwd: train mode needs L | T, masks, save buffers and rs >= T*EN");
  MM_MAPPO_DISPATCH(d, SH::fwd(a, (hipStream_t)s));
}

int mm_mappo_bwd(const mm_mappo_dims* d, const mm_mappo_bwd_args* a, mm_stream_t s) {
  MM_REQUIRE(d && a, "mappo_bwd: null argument");
  MM_REQUIRE(a->L > 0 && a->T % a->L == 0 && a->rs >= a->T * a->en && a->rs % 64 == 0,
             "mappo_bwd: need L | T and rs >= T*EN, rs % 64 == 0");
  MM_REQUIRE(a->P[0] && a->P[1] && a->save[0] && a->save[1] && a->gsoa[0] && a->gsoa[1] && a->obs && a->mask &&
                 a->active && a->act && a->adv && a->old_logp && a->old_value && a->returns && a->stats,
             "mappo_bwd: null pointer");
  MM_MAPPO_DISPATCH(d, SH::bwd(a, (hipStream_t)s));
}

int mm_mappo_evaluate_actions(const mm_mappo_dims* d, const mm_mappo_fwd_args* a, const int32_t* act,
                              const float* active, float* values, float* logp, float* ent_rows, float* entropy,
                              int32_t* err, mm_stream_t s) {
  MM_REQUIRE(d && a && act && values && logp && ent_rows && entropy, "mappo_evaluate_actions: null argument");
  MM_REQUIRE(a->mode == MM_MAPPO_TRAIN, "mappo_evaluate_actions: TRAIN-mode forward arguments required");
  MM_REQUIRE(d->hidden == 32 && d->n_actions == 5, "mappo_evaluate_actions: H 32, A 5");
  const int rc = mm_mappo_fwd(d, a, s);
  if (rc) return rc;
  return mm::mappo_eval_launch<32, 5>(a, act, active, values, logp, ent_rows, entropy, err, (hipStream_t)s);
}

int64_t mm_mappo_wgrad_partial_count(const mm_mappo_dims* d, int64_t rs) {
  if (!d || mm::param_count(d, 0) < 0) return -1;
  if (d->obs_dim == 47) return mm::MappoShape<47, 32, 5>::partial_count(rs);
  return mm::MappoShape<94, 32, 5>::partial_count(rs);
}

int mm_mappo_wgrad(const mm_mappo_dims* d, int32_t net, const float* gsoa, int64_t rs, float* grad, float* partial,
                   mm_stream_t s) {
  MM_REQUIRE(d && gsoa && grad && partial && (net == 0 || net == 1) && rs % 64 == 0, "mappo_wgrad: bad args");
  MM_MAPPO_DISPATCH(d, SH::wgrad(net, gsoa, rs, grad, partial, (hipStream_t)s));
}

int mm_mappo_gae(const float* rew, const float* value_preds, const float* masks, float* returns, const float* vn,
                 int32_t T, int64_t en, float gamma, float gae_lambda, mm_stream_t s) {
  MM_REQUIRE(rew && value_preds && masks && returns && vn && T > 0 && en > 0, "mappo_gae: bad args");
  const float gl = (float)((double)gamma * (double)gae_lambda);
  hipLaunchKernelGGL(mm::mappo_gae_kernel, dim3((unsigned)((en + 255) / 256)), dim3(256), 0, (hipStream_t)s, rew,
                     value_preds, masks, returns, vn, T, en, gamma, gl);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_mappo_adv_stats(const float* returns, const float* value_preds, const float* active, const float* vn,
                       float* adv, int64_t rows, double* partial, float* stats, mm_stream_t s) {
  MM_REQUIRE(returns && value_preds && active && vn && adv && partial && stats && rows > 0, "mappo_adv_stats: bad args");
  const int nb = 256;
  hipLaunchKernelGGL(mm::mappo_adv_kernel, dim3(nb), dim3(256), 0, (hipStream_t)s, returns, value_preds, active, vn,
                     adv, rows, partial);
  MM_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(mm::mappo_adv_var_kernel, dim3(nb), dim3(256), 0, (hipStream_t)s, adv, active, rows, partial, nb,
                     partial + 5 * nb);
  MM_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(mm::mappo_stats_kernel, dim3(1), dim3(64), 0, (hipStream_t)s, partial, partial + 5 * nb, nb, rows,
                     stats, partial + 7 * nb);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_mappo_stats_from_sums(const double* sums, int64_t rows, float* stats, mm_stream_t s) {
  MM_REQUIRE(sums && stats && rows > 0, "mappo_stats_from_sums: bad args");
  hipLaunchKernelGGL(mm::mappo_stats_from_sums_kernel, dim3(1), dim3(64), 0, (hipStream_t)s, sums, rows, stats);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_mappo_vn_update(float* vn, float* stats, double beta, mm_stream_t s) {
  MM_REQUIRE(vn && stats, "mappo_vn_update: null pointer");
  // torch: running.mul_(beta) casts the double beta to f32; (1.0 - beta) is formed in double first
  hipLaunchKernelGGL(mm::mappo_vn_update_kernel, dim3(1), dim3(64), 0, (hipStream_t)s, vn, stats, (float)beta,
                     (float)(1.0 - beta));
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_mappo_insert(const uint8_t* done, int32_t n_agents, int32_t hidden, int64_t n_envs, float* mask_next,
                    float* active_next, float* h_actor, float* h_critic, uint64_t* counter, mm_stream_t s) {
  MM_REQUIRE(done && mask_next && active_next && h_actor && h_critic, "mappo_insert: null pointer");
  const int64_t n = n_envs * n_agents * hidden;
  hipLaunchKernelGGL(mm::mappo_insert_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)s, done,
                     n_agents, hidden, n_envs, mask_next, active_next, h_actor, h_critic, counter);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

}  // extern "C"
