// Fused per-agent Q-network forward for E lockstep envs x N agents (gfx950).
//
// Replaces Q_Net.forward + sample_action (qmix/_network.py:44-74,
// vdn/_network.py:52-58,71-88): per agent i (own weights)
//   x1 = ReLU(W1 o + b1) (D->F1), x2 = ReLU(W2 x1 + b2) (F1->G),
//   h' = GRUCell(x2, h) (torch gate order r, z, n; h' = n + z*(h-n)),
//   q  = Wq h' + bq, then epsilon-greedy / max / gather epilogue.
//
// Mapping: one wave = 32 envs of one agent; features on MFMA rows, envs on
// columns, so every layer's D registers are directly the next layer's B
// operand (see common.h kperm) — no LDS, no transposes. Weights are the A
// operand, read from the packed fragment image (4 x dwordx4 wave-instructions of
// 1 KiB each per 16 MFMAs), L2/L1-resident: block b serves agent b % N, so
// with N = 8 each XCD's L2 only ever holds one agent's weights.
// Arithmetic: exact-f32 MFMA v_mfma_f32_32x32x2_f32 (fp32 in, fp32 accumulate).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "env_dev.h"
#include "minimarl.h"
#include "qnet_geo.h"

namespace mm {

struct QFwdParams {
  mm_qfwd_io io;
  QnetGeo g;
  const float* packed;
  int E, N, D, A;
  int nblocks;  // blocks of this net inside a (possibly dual) launch
  int stagger;  // fp16x3 kernel: waves 8-15 start stagger x s_sleep(8) late
  int dbg;      // unused (kept for the kernarg layout)
  int pad_;
};

// Fragment image of one 32x32 k-block: [q = s>>2][lane][s&3] floats, so each of the 4 dwordx4
// wave-instructions reads 1 KiB contiguous (and an LDS copy would be conflict-free).
__device__ __forceinline__ void load_frag(const float* __restrict__ base, int lane, float (&a)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4 v = *reinterpret_cast<const float4*>(base + q * 256 + lane * 4);
    a[4 * q + 0] = v.x;
    a[4 * q + 1] = v.y;
    a[4 * q + 2] = v.z;
    a[4 * q + 3] = v.w;
  }
}

__device__ __forceinline__ f32x16 load_bias(const float* __restrict__ base, int hh) {
  const float4* p = reinterpret_cast<const float4*>(base + hh * 16);
  f32x16 r;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4 v = p[q];
    r[4 * q + 0] = v.x;
    r[4 * q + 1] = v.y;
    r[4 * q + 2] = v.z;
    r[4 * q + 3] = v.w;
  }
  return r;
}

// Post-layer-1 weight fragments in consumption order (compile-time index -> packed offset):
//   L2 (rb < RB2, kb < RB1); per hidden block hb: Wih r,z,n (kb < RB2), Whh r,z,n (kb < HB); Q (ab, kb < HB).
template <int F1, int G, int H, int AB>
struct Sched {
  static constexpr int RB1 = F1 / 32, RB2 = G / 32, HB = H / 32;
  static constexpr int NF2 = RB2 * RB1, PERHB = 3 * RB2 + 3 * HB, NFG = HB * PERHB, NFQ = AB * HB;
  static constexpr int NF = NF2 + NFG + NFQ;
  using CG = QnetCGeo<F1, G, H, AB>;
  __device__ static constexpr int off(int i) {
    if (i < NF2) return CG::off_l2 + ((i / RB1) * RB1 + i % RB1) * 1024;
    i -= NF2;
    if (i < NFG) {
      const int hb = i / PERHB;
      int r = i % PERHB;
      if (r < 3 * RB2) return CG::off_ih + (((r / RB2) * HB + hb) * RB2 + r % RB2) * 1024;
      r -= 3 * RB2;
      return CG::off_hh + (((r / HB) * HB + hb) * HB + r % HB) * 1024;
    }
    i -= NFG;
    return CG::off_q + ((i / HB) * HB + i % HB) * 1024;
  }
};

// Observation row of (env e, agent): the chunk-store row (or the reset obs when obs_row < 0).
__device__ __forceinline__ const float* obs_row_ptr(const QFwdParams& p, int agent, int e) {
  if (e >= p.E) return nullptr;
  const mm_qfwd_io& io = p.io;
  const int64_t r = io.obs_row ? io.obs_row[e] : (int64_t)e;
  return (r >= 0) ? io.obs + r * io.obs_se + io.obs_off + (int64_t)agent * io.obs_sa
                  : io.reset_obs + (int64_t)agent * io.obs_sa;
}

// B operand of layer-1 k-block kb: lane (j, hh) holds obs features 32 kb + kperm(s, hh).
__device__ __forceinline__ void load_obs_kblock(const float* orow, int kb, int D, float (&x)[16]) {
  const int hh = (threadIdx.x & 63) >> 5;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int k = kb * 32 + kperm(s, hh);
    x[s] = (orow && k < D) ? orow[k] : 0.0f;
  }
}

// Q output / argmax / eps-greedy / gather epilogue shared by the fused and the split forward.
template <int AB>
__device__ __forceinline__ int q_epilogue_v(const QFwdParams& p, const mm_qfwd_io& io, int agent, int e, bool valid,
                                            const f32x16 (&qa)[AB], float eps, uint64_t ctr, int act_pre = -1,
                                            int64_t out_off = 0);
template <int AB>
__device__ __forceinline__ void q_epilogue(const QFwdParams& p, int agent, int e, bool valid, const f32x16 (&qa)[AB]) {
  const mm_qfwd_io& io = p.io;
  const float eps = (io.mode == MM_Q_ACT && io.eps_ptr) ? *io.eps_ptr : io.epsilon;
  const uint64_t ctr = (io.mode == MM_Q_ACT && io.counter_ptr) ? *io.counter_ptr : io.counter;
  q_epilogue_v<AB>(p, io, agent, e, valid, qa, eps, ctr);
}
// returns the selected action (every lane); out_off: element offset of the act / qsel outputs (a ring slot)
template <int AB>
__device__ __forceinline__ int q_epilogue_v(const QFwdParams& p, const mm_qfwd_io& io, int agent, int e, bool valid,
                                            const f32x16 (&qa)[AB], float eps, uint64_t ctr, int act_pre,
                                            int64_t out_off) {
  const int hh = (threadIdx.x & 63) >> 5;
  if (valid && io.q_out) {
    float* qrow = io.q_out + (int64_t)e * io.q_se + (int64_t)agent * io.q_sa;
#pragma unroll
    for (int ab = 0; ab < AB; ++ab)
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int row = ab * 32 + kperm(s, hh);
        if (row < p.A) qrow[row] = qa[ab][s];
      }
  }
  if (io.mode == MM_Q_NONE) return 0;

  // ---- epilogue: first-index argmax over A rows spread across the two lane halves
  float best = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int ab = 0; ab < AB; ++ab)
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int row = ab * 32 + kperm(s, hh);
      const float v = qa[ab][s];
      if (row < p.A && (v > best || (v == best && row < bi))) {
        best = v;
        bi = row;
      }
    }
  const float ob = __shfl_xor(best, 32);
  const int oi = __shfl_xor(bi, 32);
  if (ob > best || (ob == best && oi < bi)) {
    best = ob;
    bi = oi;
  }
  int act = bi;
  if (io.mode == MM_Q_ACT) {
    float u;
    if (io.u) {
      u = valid ? io.u[e] : 1.0f;
    } else {
      u = rng_uniform(rng_draw(io.seed, ctr, (uint64_t)e, 0xFFFFFFFFull));
    }
    if (u <= eps) {
      if (io.rand_act) {
        act = valid ? io.rand_act[(int64_t)e * p.N + agent] : 0;
      } else {
        act = (int)(rng_draw(io.seed ^ 0x5bd1e995ull, ctr, (uint64_t)e, (uint64_t)agent) % (uint64_t)p.A);
      }
    }
  } else if (io.mode == MM_Q_GATHER) {
    act = act_pre >= 0 ? act_pre : (valid ? io.act_in[(int64_t)e * io.act_se + agent] : 0);
  }
  float mine = 0.0f;
#pragma unroll
  for (int ab = 0; ab < AB; ++ab)
#pragma unroll
    for (int s = 0; s < 16; ++s)
      if (ab * 32 + kperm(s, hh) == act) mine = qa[ab][s];
  const float qsel = (io.mode == MM_Q_MAX) ? best : mine + __shfl_xor(mine, 32);
  if (valid && hh == 0) {
    const int64_t o = out_off + (int64_t)e * p.N + agent;
    if (io.act_out && io.mode == MM_Q_ACT) io.act_out[o] = act;
    if (io.qsel_out) io.qsel_out[o] = qsel;
  }
  return act;
}

// xn: layer-1 k-block 0 of the observation, loaded by the caller (before weight staging).
// ol(kb, x) loads observation k-block kb (lane (i, hh) holds features 32 kb + kperm(s, hh) of env e);
// zero_h: start the GRU from zeros (invalid env or reset flag)
// ovr: the epilogue's epsilon / RNG step counter / output offset are eps_o / ctr_o / off_o instead of read from
// p.io (the chunk-persistent rollout); returns the selected action (ACT mode)
template <int F1, int G, int H, int AB, class OL>
__device__ __forceinline__ int agent_q_fwd_body(const QFwdParams& p, int agent, int e,
                                                const float* __restrict__ W, const OL& ol,
                                                float (&xn)[16], bool zero_h, bool ovr = false, float eps_o = 0.f,
                                                uint64_t ctr_o = 0, int64_t off_o = 0) {
  using S = Sched<F1, G, H, AB>;
  using CG = typename S::CG;
  constexpr int RB1 = S::RB1, RB2 = S::RB2, HB = S::HB, NF = S::NF;
  const int lane = threadIdx.x & 63;
  const int hh = lane >> 5;
  const bool valid = e < p.E;
  const mm_qfwd_io& io = p.io;

  // fragment pipeline (prefetch distance 1): nxt holds the next fragment of the schedule
  float cur[16], nxt[16];
  load_frag(W + S::off(0), lane, nxt);
  auto consume = [&](int i, const f32x16& x, f32x16& acc) {
#pragma unroll
    for (int s = 0; s < 16; ++s) cur[s] = nxt[s];
    if (i + 1 < NF) load_frag(W + S::off(i + 1), lane, nxt);
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = mfma32(cur[s], x[s], acc);
  };

  // ---- layer 1: x1 = ReLU(W1 o + b1), K = D streamed in 32-wide k-blocks (next k-block prefetched)
  f32x16 x1[RB1];
#pragma unroll
  for (int rb = 0; rb < RB1; ++rb) x1[rb] = load_bias(W + CG::off_b1 + rb * 32, hh);
  float xb[16];
  float fa[RB1][16], fn[RB1][16];
#pragma unroll
  for (int rb = 0; rb < RB1; ++rb) load_frag(W + CG::off_l1 + (int64_t)(rb * p.g.KD) * 1024, lane, fn[rb]);
  for (int kb = 0; kb < p.g.KD; ++kb) {
#pragma unroll
    for (int s = 0; s < 16; ++s) xb[s] = xn[s];
#pragma unroll
    for (int rb = 0; rb < RB1; ++rb)
#pragma unroll
      for (int s = 0; s < 16; ++s) fa[rb][s] = fn[rb][s];
    if (kb + 1 < p.g.KD) {
      ol(kb + 1, xn);
#pragma unroll
      for (int rb = 0; rb < RB1; ++rb)
        load_frag(W + CG::off_l1 + (int64_t)(rb * p.g.KD + kb + 1) * 1024, lane, fn[rb]);
    }
#pragma unroll
    for (int rb = 0; rb < RB1; ++rb)
#pragma unroll
      for (int s = 0; s < 16; ++s) x1[rb] = mfma32(fa[rb][s], xb[s], x1[rb]);
  }
#pragma unroll
  for (int rb = 0; rb < RB1; ++rb)
#pragma unroll
    for (int s = 0; s < 16; ++s) x1[rb][s] = fmaxf(x1[rb][s], 0.0f);
  // training save row (see mm_qfwd_io.save): [x1 | x2 | h_in | r | z | n | anh | h_out]
  float* sv = (io.save && valid) ? io.save + ((int64_t)e * p.N + agent) * (F1 + G + 6 * H) : nullptr;
  if (sv) {
#pragma unroll
    for (int rb = 0; rb < RB1; ++rb)
#pragma unroll
      for (int s = 0; s < 16; ++s) sv[rb * 32 + kperm(s, hh)] = x1[rb][s];
  }

  // ---- layer 2: x2 = ReLU(W2 x1 + b2)
  f32x16 x2[RB2];
#pragma unroll
  for (int rb = 0; rb < RB2; ++rb) {
    x2[rb] = load_bias(W + CG::off_b2 + rb * 32, hh);
#pragma unroll
    for (int kb = 0; kb < RB1; ++kb) consume(rb * RB1 + kb, x1[kb], x2[rb]);
#pragma unroll
    for (int s = 0; s < 16; ++s) x2[rb][s] = fmaxf(x2[rb][s], 0.0f);
    if (sv) {
#pragma unroll
      for (int s = 0; s < 16; ++s) sv[F1 + rb * 32 + kperm(s, hh)] = x2[rb][s];
    }
  }

  // ---- GRU cell
  f32x16 h0[HB];
#pragma unroll
  for (int hb = 0; hb < HB; ++hb) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int f = hb * 32 + kperm(s, hh);
      h0[hb][s] = zero_h ? 0.0f
                         : io.h_in[(int64_t)e * io.hin_se + (int64_t)agent * io.hin_sa + (int64_t)f * io.hin_sf];
    }
  }
  f32x16 h1[HB];
#pragma unroll
  for (int hb = 0; hb < HB; ++hb) {
    const int base = S::NF2 + hb * S::PERHB;
    f32x16 ar = load_bias(W + CG::off_brz + hb * 32, hh);
    f32x16 az = load_bias(W + CG::off_brz + (HB + hb) * 32, hh);
    f32x16 anx = load_bias(W + CG::off_bin + hb * 32, hh);
    f32x16 anh = load_bias(W + CG::off_bhn + hb * 32, hh);
#pragma unroll
    for (int kb = 0; kb < RB2; ++kb) consume(base + kb, x2[kb], ar);
#pragma unroll
    for (int kb = 0; kb < RB2; ++kb) consume(base + RB2 + kb, x2[kb], az);
#pragma unroll
    for (int kb = 0; kb < RB2; ++kb) consume(base + 2 * RB2 + kb, x2[kb], anx);
#pragma unroll
    for (int kb = 0; kb < HB; ++kb) consume(base + 3 * RB2 + kb, h0[kb], ar);
#pragma unroll
    for (int kb = 0; kb < HB; ++kb) consume(base + 3 * RB2 + HB + kb, h0[kb], az);
#pragma unroll
    for (int kb = 0; kb < HB; ++kb) consume(base + 3 * RB2 + 2 * HB + kb, h0[kb], anh);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const float r = sigmoidf_(ar[s]);
      const float z = sigmoidf_(az[s]);
      const float n = tanhf_(anx[s] + r * anh[s]);
      h1[hb][s] = n + z * (h0[hb][s] - n);
      if (sv) {
        float* o = sv + F1 + G + hb * 32 + kperm(s, hh);
        o[0] = h0[hb][s];
        o[H] = r;
        o[2 * H] = z;
        o[3 * H] = n;
        o[4 * H] = anh[s];
        o[5 * H] = h1[hb][s];
      }
    }
  }
  if (valid && io.h_out) {
#pragma unroll
    for (int hb = 0; hb < HB; ++hb)
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int f = hb * 32 + kperm(s, hh);
        io.h_out[(int64_t)e * io.hout_se + (int64_t)agent * io.hout_sa + (int64_t)f * io.hout_sf] = h1[hb][s];
      }
  }

  // ---- Q head
  f32x16 qa[AB];
#pragma unroll
  for (int ab = 0; ab < AB; ++ab) {
    qa[ab] = load_bias(W + CG::off_bq + ab * 32, hh);
#pragma unroll
    for (int kb = 0; kb < HB; ++kb) consume(S::NF2 + S::NFG + ab * HB + kb, h1[kb], qa[ab]);
  }
  if (ovr) return q_epilogue_v<AB>(p, io, agent, e, valid, qa, eps_o, ctr_o, -1, off_o);
  q_epilogue<AB>(p, agent, e, valid, qa);
  return 0;
}

// ---------------------------------------------------------------- split forward (training)
// PRE: layers 1-2 and the GRU input projection for every (row, agent) of a chunk batch; REC: one
// recurrent step from those projections. Same MFMA accumulation order as the fused body (biases,
// then W_ih x2, then W_hh h), so PRE + REC reproduce agent_q_fwd_body bit for bit.
// a 32-wide act-frag vector (lane half hh holds features kperm(s, hh)) stored as 4 runs of 4 floats:
// features 8j + 4hh + 0..3 are v[4j..4j+3]. dst must be 16-byte aligned (row strides of saves / gi are
// multiples of 4 floats; the bases are torch allocations).
__device__ __forceinline__ void store_kperm16(float* dst, int hh, const f32x16& v) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    *reinterpret_cast<float4*>(dst + 8 * j + 4 * hh) = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
}

template <int F1, int G, int H, int AB>
__device__ __forceinline__ void agent_pre_body(const QFwdParams& p, int agent, int e, const float* __restrict__ W,
                                               const float* orow) {
  using S = Sched<F1, G, H, AB>;
  using CG = typename S::CG;
  constexpr int RB1 = S::RB1, RB2 = S::RB2, HB = S::HB;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const bool valid = e < p.E;
  const mm_qfwd_io& io = p.io;
  float fr[16], xk[16], xn[16];
  f32x16 x1[RB1];
#pragma unroll
  for (int rb = 0; rb < RB1; ++rb) x1[rb] = load_bias(W + CG::off_b1 + rb * 32, hh);
  load_obs_kblock(orow, 0, p.D, xn);
  for (int kb = 0; kb < p.g.KD; ++kb) {
#pragma unroll
    for (int s = 0; s < 16; ++s) xk[s] = xn[s];
    if (kb + 1 < p.g.KD) load_obs_kblock(orow, kb + 1, p.D, xn);   // next k-block in flight
#pragma unroll
    for (int rb = 0; rb < RB1; ++rb) {
      load_frag(W + CG::off_l1 + (int64_t)(rb * p.g.KD + kb) * 1024, lane, fr);
#pragma unroll
      for (int s = 0; s < 16; ++s) x1[rb] = mfma32(fr[s], xk[s], x1[rb]);
    }
  }
  float* sv = (io.save && valid) ? io.save + ((int64_t)e * p.N + agent) * (F1 + G + 6 * H) : nullptr;
#pragma unroll
  for (int rb = 0; rb < RB1; ++rb) {
#pragma unroll
    for (int s = 0; s < 16; ++s) x1[rb][s] = fmaxf(x1[rb][s], 0.0f);
    if (sv) store_kperm16(sv + rb * 32, hh, x1[rb]);
  }
  f32x16 x2[RB2];
#pragma unroll
  for (int rb = 0; rb < RB2; ++rb) {
    x2[rb] = load_bias(W + CG::off_b2 + rb * 32, hh);
#pragma unroll
    for (int kb = 0; kb < RB1; ++kb) {
      load_frag(W + S::off(rb * RB1 + kb), lane, fr);
#pragma unroll
      for (int s = 0; s < 16; ++s) x2[rb] = mfma32(fr[s], x1[kb][s], x2[rb]);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) x2[rb][s] = fmaxf(x2[rb][s], 0.0f);
    if (sv) store_kperm16(sv + F1 + rb * 32, hh, x2[rb]);
  }
  float* gi = valid ? io.gi + ((int64_t)e * p.N + agent) * 3 * H : nullptr;
#pragma unroll
  for (int hb = 0; hb < HB; ++hb) {
#pragma unroll
    for (int gte = 0; gte < 3; ++gte) {
      f32x16 acc = gte < 2 ? load_bias(W + CG::off_brz + (gte * HB + hb) * 32, hh)
                           : load_bias(W + CG::off_bin + hb * 32, hh);
#pragma unroll
      for (int kb = 0; kb < RB2; ++kb) {
        load_frag(W + S::off(S::NF2 + hb * S::PERHB + gte * RB2 + kb), lane, fr);
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = mfma32(fr[s], x2[kb][s], acc);
      }
      if (gi) store_kperm16(gi + gte * H + hb * 32, hh, acc);
    }
  }
}

// PRE for small batches: one block = one 32-env tile of one agent, the row blocks of each layer on
// separate waves (layer 1: RB1 waves, layer 2: RB2 waves, W_ih: 3 HB waves), activations handed over
// through LDS. Every wave issues ALL its loads (weight fragments of the layers it computes, the
// observation k-blocks, biases) before its first MFMA: one memory round trip per launch instead of one
// per fragment, and a critical path of KD + RB1 + RB2 k-blocks of MFMAs instead of the whole network
// on one wave. Per output the accumulation order is agent_pre_body's (bit-identical).
constexpr int kPreRbMaxKD = 2;   // observation k-blocks (D <= 64) supported by the row-block PRE
template <int F1, int G, int H, int AB>
__device__ __forceinline__ void agent_pre_rb_body(const QFwdParams& p, int agent, int tile) {
  using S = Sched<F1, G, H, AB>;
  using CG = typename S::CG;
  constexpr int RB1 = S::RB1, RB2 = S::RB2, HB = S::HB;
  __shared__ float x1s[RB1][16][64];
  __shared__ float x2s[RB2][16][64];
  const float* W = p.packed + (int64_t)agent * p.g.agent_stride;
  const int lane = threadIdx.x & 63, hh = lane >> 5, wv = threadIdx.x >> 6;
  const int e = tile * 32 + (lane & 31);
  const bool valid = e < p.E;
  const mm_qfwd_io& io = p.io;
  const float* orow = obs_row_ptr(p, agent, e);
  const int KD = p.g.KD;
  // ---- every load of this wave first
  float f1[kPreRbMaxKD][16], xo[kPreRbMaxKD][16], f2[RB1][16], f3[RB2][16];
  f32x16 b1, b2, b3;
  const int hb3 = wv % HB, gte = wv / HB;
  if (wv < RB1) {
    b1 = load_bias(W + CG::off_b1 + wv * 32, hh);
#pragma unroll
    for (int kb = 0; kb < kPreRbMaxKD; ++kb)
      if (kb < KD) {
        load_frag(W + CG::off_l1 + (int64_t)(wv * KD + kb) * 1024, lane, f1[kb]);
        load_obs_kblock(orow, kb, p.D, xo[kb]);
      }
  }
  if (wv < RB2) {
    b2 = load_bias(W + CG::off_b2 + wv * 32, hh);
#pragma unroll
    for (int kb = 0; kb < RB1; ++kb) load_frag(W + S::off(wv * RB1 + kb), lane, f2[kb]);
  }
  if (wv < 3 * HB) {
    b3 = gte < 2 ? load_bias(W + CG::off_brz + (gte * HB + hb3) * 32, hh) : load_bias(W + CG::off_bin + hb3 * 32, hh);
#pragma unroll
    for (int kb = 0; kb < RB2; ++kb) load_frag(W + S::off(S::NF2 + hb3 * S::PERHB + gte * RB2 + kb), lane, f3[kb]);
  }
  float* sv = (io.save && valid) ? io.save + ((int64_t)e * p.N + agent) * (F1 + G + 6 * H) : nullptr;
  // ---- layer 1 (row block wv)
  if (wv < RB1) {
    f32x16 acc = b1;
#pragma unroll
    for (int kb = 0; kb < kPreRbMaxKD; ++kb)
      if (kb < KD) {
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = mfma32(f1[kb][s], xo[kb][s], acc);
      }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      acc[s] = fmaxf(acc[s], 0.0f);
      x1s[wv][s][lane] = acc[s];
    }
    if (sv) store_kperm16(sv + wv * 32, hh, acc);
  }
  __syncthreads();
  // ---- layer 2 (row block wv)
  if (wv < RB2) {
    f32x16 acc = b2;
#pragma unroll
    for (int kb = 0; kb < RB1; ++kb)
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = mfma32(f2[kb][s], x1s[kb][s][lane], acc);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      acc[s] = fmaxf(acc[s], 0.0f);
      x2s[wv][s][lane] = acc[s];
    }
    if (sv) store_kperm16(sv + F1 + wv * 32, hh, acc);
  }
  __syncthreads();
  // ---- GRU input projection (gate gte, hidden block hb3)
  if (wv < 3 * HB) {
    f32x16 acc = b3;
#pragma unroll
    for (int kb = 0; kb < RB2; ++kb)
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = mfma32(f3[kb][s], x2s[kb][s][lane], acc);
    if (valid) {
      float* gi = io.gi + ((int64_t)e * p.N + agent) * 3 * H;
      store_kperm16(gi + gte * H + hb3 * 32, hh, acc);
    }
  }
}

template <int F1, int G, int H, int AB>
__global__ __launch_bounds__(64 * (3 * (H / 32) > F1 / 32 ? 3 * (H / 32) : F1 / 32)) void agent_pre_rb_kernel(
    QFwdParams p0, QFwdParams p1) {
  if ((int)blockIdx.x >= p0.nblocks) {
    const int bid = (int)blockIdx.x - p0.nblocks;
    agent_pre_rb_body<F1, G, H, AB>(p1, bid % p1.N, bid / p1.N);
  } else {
    const int bid = (int)blockIdx.x;
    agent_pre_rb_body<F1, G, H, AB>(p0, bid % p0.N, bid / p0.N);
  }
}

// REC for small batches: the HB hidden blocks of one 32-env tile run on HB waves of the block (each
// loads all its W_hh fragments, gi and h up front: one memory latency per step instead of one per
// fragment); the Q head + epilogue run on wave 0 after an LDS exchange of the new hidden blocks.
template <int F1, int G, int H, int AB>
__device__ __forceinline__ void agent_rec_body(const QFwdParams& p, int agent, int tile, const float* __restrict__ W) {
  using S = Sched<F1, G, H, AB>;
  using CG = typename S::CG;
  constexpr int RB2 = S::RB2, HB = S::HB;
  __shared__ float hx[HB][16][64];
  const int lane = threadIdx.x & 63, hh = lane >> 5, hb = threadIdx.x >> 6;
  const int e = tile * 32 + (lane & 31);
  const bool valid = e < p.E;
  const mm_qfwd_io& io = p.io;
  const bool zero_h = !valid || (io.reset && io.reset[e]);
  float fz[3][HB][16];
  const int base = S::NF2 + hb * S::PERHB + 3 * RB2;
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int kb = 0; kb < HB; ++kb) load_frag(W + S::off(base + g * HB + kb), lane, fz[g][kb]);
  f32x16 h0[HB];
#pragma unroll
  for (int kb = 0; kb < HB; ++kb)
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int f = kb * 32 + kperm(s, hh);
      h0[kb][s] = zero_h ? 0.0f
                         : io.h_in[(int64_t)e * io.hin_se + (int64_t)agent * io.hin_sa + (int64_t)f * io.hin_sf];
    }
  const float* gi = io.gi + ((int64_t)(valid ? e : 0) * p.N + agent) * 3 * H;
  f32x16 ar, az, anx;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int f = hb * 32 + kperm(s, hh);
    ar[s] = gi[f];
    az[s] = gi[H + f];
    anx[s] = gi[2 * H + f];
  }
  f32x16 anh = load_bias(W + CG::off_bhn + hb * 32, hh);
#pragma unroll
  for (int kb = 0; kb < HB; ++kb)
#pragma unroll
    for (int s = 0; s < 16; ++s) ar = mfma32(fz[0][kb][s], h0[kb][s], ar);
#pragma unroll
  for (int kb = 0; kb < HB; ++kb)
#pragma unroll
    for (int s = 0; s < 16; ++s) az = mfma32(fz[1][kb][s], h0[kb][s], az);
#pragma unroll
  for (int kb = 0; kb < HB; ++kb)
#pragma unroll
    for (int s = 0; s < 16; ++s) anh = mfma32(fz[2][kb][s], h0[kb][s], anh);
  float* sv = (io.save && valid) ? io.save + ((int64_t)e * p.N + agent) * (F1 + G + 6 * H) : nullptr;
  float h1v[16];
  float h0v[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    // h0 of this wave's hidden block (compile-time register selection)
    float v = h0[0][s];
#pragma unroll
    for (int kb = 1; kb < HB; ++kb)
      if (kb == hb) v = h0[kb][s];
    h0v[s] = v;
  }
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const float r = sigmoidf_(ar[s]);
    const float z = sigmoidf_(az[s]);
    const float n = tanhf_(anx[s] + r * anh[s]);
    h1v[s] = n + z * (h0v[s] - n);
    hx[hb][s][lane] = h1v[s];
    if (sv) {
      float* o = sv + F1 + G + hb * 32 + kperm(s, hh);
      o[0] = h0v[s];
      o[H] = r;
      o[2 * H] = z;
      o[3 * H] = n;
      o[4 * H] = anh[s];
      o[5 * H] = h1v[s];
    }
  }
  if (valid && io.h_out) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int f = hb * 32 + kperm(s, hh);
      io.h_out[(int64_t)e * io.hout_se + (int64_t)agent * io.hout_sa + (int64_t)f * io.hout_sf] = h1v[s];
    }
  }
  __syncthreads();
  if (hb != 0) return;
  f32x16 h1[HB];
#pragma unroll
  for (int kb = 0; kb < HB; ++kb)
#pragma unroll
    for (int s = 0; s < 16; ++s) h1[kb][s] = hx[kb][s][lane];
  f32x16 qa[AB];
  float fr[16];
#pragma unroll
  for (int ab = 0; ab < AB; ++ab) {
    qa[ab] = load_bias(W + CG::off_bq + ab * 32, hh);
#pragma unroll
    for (int kb = 0; kb < HB; ++kb) {
      load_frag(W + S::off(S::NF2 + S::NFG + ab * HB + kb), lane, fr);
#pragma unroll
      for (int s = 0; s < 16; ++s) qa[ab] = mfma32(fr[s], h1[kb][s], qa[ab]);
    }
  }
  q_epilogue<AB>(p, agent, e, valid, qa);
}

// PHASE 1 = PRE: 128 rows of one agent per block (4 waves x 32). PHASE 2 = REC: one 32-env tile of
// one agent per block (H/32 waves). Block b serves agent b % N.
template <int F1, int G, int H, int AB, int PHASE>
__global__ __launch_bounds__(256, 2) void agent_split_kernel(QFwdParams p0, QFwdParams p1) {
  const bool second = (int)blockIdx.x >= p0.nblocks;
  const QFwdParams& p = second ? p1 : p0;
  const int bid = second ? (int)blockIdx.x - p0.nblocks : (int)blockIdx.x;
  const int agent = bid % p.N, tile = bid / p.N;
  const float* W = p.packed + (int64_t)agent * p.g.agent_stride;
  if constexpr (PHASE == 1) {
    const int e = tile * 128 + (threadIdx.x >> 6) * 32 + (threadIdx.x & 31);
    agent_pre_body<F1, G, H, AB>(p, agent, e, W, obs_row_ptr(p, agent, e));
  } else {
    agent_rec_body<F1, G, H, AB>(p, agent, tile, W);
  }
}

// REC over all C steps of a learner chunk in one launch (one block = one 32-env tile of one agent
// for the whole sequence): the W_hh fragments stay in registers, the hidden state stays in LDS
// between steps (hx exchange), and step t's pointers are the step-0 ones + t * stride. Same
// arithmetic as C launches of agent_rec_body (bit-identical results).
struct RecSeq {
  int C;
  int64_t gi_st, save_st, act_st, qsel_st;   // elements per step
  const uint8_t* reset;                        // step t >= 1 resets where reset[(t-1)*reset_st + e]
  int64_t reset_st;
  uint64_t* trace;                             // timing trace (MM_REC_TRACE), nullptr normally
};

template <int F1, int G, int H, int AB>
__global__ __launch_bounds__(256, 2) void agent_rec_seq_kernel(QFwdParams p0, QFwdParams p1, RecSeq s0,
                                                               RecSeq s1) {
  using S = Sched<F1, G, H, AB>;
  using CG = typename S::CG;
  constexpr int RB2 = S::RB2, HB = S::HB;
  __shared__ float hx[HB][16][64];
  const bool second = (int)blockIdx.x >= p0.nblocks;
  const QFwdParams& p = second ? p1 : p0;
  const RecSeq& sq = second ? s1 : s0;
  const int bid = second ? (int)blockIdx.x - p0.nblocks : (int)blockIdx.x;
  const int agent = bid % p.N, tile = bid / p.N;
  const float* W = p.packed + (int64_t)agent * p.g.agent_stride;
  const int lane = threadIdx.x & 63, hh = lane >> 5, hb = threadIdx.x >> 6;
  const int e = tile * 32 + (lane & 31);
  const bool valid = e < p.E;
  float fz[3][HB][16];
  const int base = S::NF2 + hb * S::PERHB + 3 * RB2;
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int kb = 0; kb < HB; ++kb) load_frag(W + S::off(base + g * HB + kb), lane, fz[g][kb]);
  const f32x16 bhn = load_bias(W + CG::off_bhn + hb * 32, hh);
  mm_qfwd_io io = p.io;
  const float eps = (io.mode == MM_Q_ACT && io.eps_ptr) ? *io.eps_ptr : io.epsilon;
  const uint64_t ctr = (io.mode == MM_Q_ACT && io.counter_ptr) ? *io.counter_ptr : io.counter;
  for (int t = 0; t < sq.C; ++t) {
    f32x16 h0[HB];
    const bool zero_h = !valid || t == 0 || sq.reset[(int64_t)(t - 1) * sq.reset_st + e];
    if (t > 0) __syncthreads();   // previous step's hx writes visible
#pragma unroll
    for (int kb = 0; kb < HB; ++kb)
#pragma unroll
      for (int s = 0; s < 16; ++s) h0[kb][s] = zero_h ? 0.0f : hx[kb][s][lane];
    const float* gi = io.gi + t * sq.gi_st + ((int64_t)(valid ? e : 0) * p.N + agent) * 3 * H;
    f32x16 ar, az, anx;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int f = hb * 32 + kperm(s, hh);
      ar[s] = gi[f];
      az[s] = gi[H + f];
      anx[s] = gi[2 * H + f];
    }
    f32x16 anh = bhn;
#pragma unroll
    for (int kb = 0; kb < HB; ++kb)
#pragma unroll
      for (int s = 0; s < 16; ++s) ar = mfma32(fz[0][kb][s], h0[kb][s], ar);
#pragma unroll
    for (int kb = 0; kb < HB; ++kb)
#pragma unroll
      for (int s = 0; s < 16; ++s) az = mfma32(fz[1][kb][s], h0[kb][s], az);
#pragma unroll
    for (int kb = 0; kb < HB; ++kb)
#pragma unroll
      for (int s = 0; s < 16; ++s) anh = mfma32(fz[2][kb][s], h0[kb][s], anh);
    float* sv = (io.save && valid) ? io.save + t * sq.save_st + ((int64_t)e * p.N + agent) * (F1 + G + 6 * H)
                                   : nullptr;
    float h1v[16], h0v[16], rv[16], zv[16], nv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      h0v[s] = h0[0][s];
#pragma unroll
      for (int kb = 1; kb < HB; ++kb)
        if (kb == hb) h0v[s] = h0[kb][s];
      rv[s] = sigmoidf_(ar[s]);
      zv[s] = sigmoidf_(az[s]);
      nv[s] = tanhf_(anx[s] + rv[s] * anh[s]);
      h1v[s] = nv[s] + zv[s] * (h0v[s] - nv[s]);
    }
    if (sv) {
      // the save row's 6 fields: lane (e, hh) holds features 8j + 4hh + 0..3 of each, so every field goes
      // out as 4 16-byte stores (sv + F1 + G and the field strides are multiples of 4 floats; the host
      // requires a 16-byte aligned save base) instead of 16 scattered 4-byte stores
      float* o = sv + F1 + G + hb * 32 + 4 * hh;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = 4 * j;
        float* oj = o + 8 * j;
        *reinterpret_cast<float4*>(oj) = make_float4(h0v[q], h0v[q + 1], h0v[q + 2], h0v[q + 3]);
        *reinterpret_cast<float4*>(oj + H) = make_float4(rv[q], rv[q + 1], rv[q + 2], rv[q + 3]);
        *reinterpret_cast<float4*>(oj + 2 * H) = make_float4(zv[q], zv[q + 1], zv[q + 2], zv[q + 3]);
        *reinterpret_cast<float4*>(oj + 3 * H) = make_float4(nv[q], nv[q + 1], nv[q + 2], nv[q + 3]);
        *reinterpret_cast<float4*>(oj + 4 * H) = make_float4(anh[q], anh[q + 1], anh[q + 2], anh[q + 3]);
        *reinterpret_cast<float4*>(oj + 5 * H) = make_float4(h1v[q], h1v[q + 1], h1v[q + 2], h1v[q + 3]);
      }
    }
    __syncthreads();   // every wave has read hx (its h0) before it is overwritten
#pragma unroll
    for (int s = 0; s < 16; ++s) hx[hb][s][lane] = h1v[s];
    __syncthreads();
    if (hb == 0) {
      f32x16 h1[HB];
#pragma unroll
      for (int kb = 0; kb < HB; ++kb)
#pragma unroll
        for (int s = 0; s < 16; ++s) h1[kb][s] = hx[kb][s][lane];
      f32x16 qa[AB];
      float fr[16];
#pragma unroll
      for (int ab = 0; ab < AB; ++ab) {
        qa[ab] = load_bias(W + CG::off_bq + ab * 32, hh);
#pragma unroll
        for (int kb = 0; kb < HB; ++kb) {
          load_frag(W + S::off(S::NF2 + S::NFG + ab * HB + kb), lane, fr);
#pragma unroll
          for (int s = 0; s < 16; ++s) qa[ab] = mfma32(fr[s], h1[kb][s], qa[ab]);
        }
      }
      mm_qfwd_io it = io;
      if (it.act_in) it.act_in += t * sq.act_st;
      if (it.qsel_out) it.qsel_out += t * sq.qsel_st;
      q_epilogue_v<AB>(p, it, agent, e, valid, qa, eps, ctr);
    }
  }
}

// Gate-parallel REC sequence (small batches): one block = one 32-env tile of one agent for all C steps,
// 3 * HB + 1 waves: wave (g, hb) (g = r, z, n) runs only its gate's MFMA chain for hidden block hb
// (32 MFMAs at HB = 2 instead of 96 on one wave), the r-wave of each hb combines the gates, and the
// last wave computes the Q head + epilogue of step t while the gate waves already run step t + 1.
// Every accumulator starts from the same value and accumulates in the same (kb, s) order as
// agent_rec_body, so the results are bit-identical to the per-step launches.
//
// Memory-counter discipline (gfx9 counts stores in vmcnt, so any load wait also drains every store
// issued before it): the r- and z-waves only LOAD (next step's gate inputs, one step ahead), the
// n-wave only STORES (the training save rows of step t - 1, staged in LDS by the r-wave and written
// out while the r-wave computes step t's gates), and the Q wave loads its gathered action before
// issuing its stores. No wave on the recurrence's critical path ever waits for a store.
// LDS of one gate-parallel REC block (dynamic, so a paired launch can carve the same space for another body)
template <int H>
struct RecGpLds {
  static constexpr int HB = H / 32;
  static constexpr size_t hx = 0;                                  // float [2][HB][16][64]
  static constexpr size_t gx = hx + 2 * HB * 16 * 64 * 4;          // float [2][HB][16][64]
  static constexpr size_t svs = gx + 2 * HB * 16 * 64 * 4;         // float [2][HB][6][32][33]
  static constexpr size_t zreset = svs + 2 * HB * 6 * 32 * 33 * 4; // int [64]
  static constexpr size_t bytes = zreset + 64 * 4;
};

template <int F1, int G, int H, int AB>
__device__ __forceinline__ void rec_seq_gp_body(const QFwdParams& p, const RecSeq& sq, int bid, char* lds) {
  const uint64_t t_entry = clock64();
  using S = Sched<F1, G, H, AB>;
  using CG = typename S::CG;
  using LY = RecGpLds<H>;
  constexpr int RB2 = S::RB2, HB = S::HB;
  constexpr int SROW = F1 + G + 6 * H;   // training save row of one (env, agent)
  // new hidden blocks, double-buffered by step parity
  float(*hx)[HB][16][64] = reinterpret_cast<float(*)[HB][16][64]>(lds + LY::hx);
  // z / n-hidden gate accumulators handed to the r-wave
  float(*gx)[HB][16][64] = reinterpret_cast<float(*)[HB][16][64]>(lds + LY::gx);
  // save-row staging [step parity][hb][field][feature][env] (env stride 33: conflict-free both ways), so
  // the save rows go out as 128-byte runs (one env's 32 features of one field)
  float(*svs)[HB][6][32][33] = reinterpret_cast<float(*)[HB][6][32][33]>(lds + LY::svs);
  int* zreset = reinterpret_cast<int*>(lds + LY::zreset);   // reset flag of the next step (r-wave of hb 0)
  const int agent = bid % p.N, tile = bid / p.N;
  const float* W = p.packed + (int64_t)agent * p.g.agent_stride;
  const int lane = threadIdx.x & 63, hh = lane >> 5, wv = threadIdx.x >> 6;
  const bool qwave = wv == 3 * HB;
  const int g = qwave ? 0 : wv / HB, hb = qwave ? 0 : wv % HB;
  const int e = tile * 32 + (lane & 31);
  const bool valid = e < p.E;
  const mm_qfwd_io io = p.io;
  const float eps = (io.mode == MM_Q_ACT && io.eps_ptr) ? *io.eps_ptr : io.epsilon;
  const uint64_t ctr = (io.mode == MM_Q_ACT && io.counter_ptr) ? *io.counter_ptr : io.counter;
  uint64_t* tr = (sq.trace && bid == 0 && lane == 0 && (wv == 0 || qwave)) ? sq.trace : nullptr;
  if (tr && wv == 0) {
    tr[0] = clock64();
    tr[3] = t_entry;
  }
  // The Q wave and the gate waves run separate loops, so the register allocator sees their
  // loop-carried state (W_q fragments vs. gate fragments + prefetched inputs) as disjoint.
  if (qwave) {
    // Q-head wave: W_q fragments and bias loaded once for the whole sequence
    float fq[AB][HB][16];
    f32x16 bq[AB];
#pragma unroll
    for (int ab = 0; ab < AB; ++ab) {
      bq[ab] = load_bias(W + CG::off_bq + ab * 32, hh);
#pragma unroll
      for (int kb = 0; kb < HB; ++kb) load_frag(W + S::off(S::NF2 + S::NFG + ab * HB + kb), lane, fq[ab][kb]);
    }
    for (int t = 0; t < sq.C; ++t) {
      uint64_t* ts = tr ? tr + 4 + t * 8 : nullptr;
      // gathered action of step t, loaded before this wave's stores of step t (see above)
      const int act_t =
          (io.mode == MM_Q_GATHER && valid) ? io.act_in[t * sq.act_st + (int64_t)e * io.act_se + agent] : 0;
      lds_sync();   // A
      lds_sync();   // B
      if (ts) ts[5] = clock64();
      f32x16 h1[HB];
#pragma unroll
      for (int kb = 0; kb < HB; ++kb)
#pragma unroll
        for (int s = 0; s < 16; ++s) h1[kb][s] = hx[(t + 1) & 1][kb][s][lane];
      f32x16 qa[AB];
#pragma unroll
      for (int ab = 0; ab < AB; ++ab) {
        qa[ab] = bq[ab];
#pragma unroll
        for (int kb = 0; kb < HB; ++kb)
#pragma unroll
          for (int s = 0; s < 16; ++s) qa[ab] = mfma32(fq[ab][kb][s], h1[kb][s], qa[ab]);
      }
      mm_qfwd_io it = io;
      if (it.act_in) it.act_in += t * sq.act_st;
      if (it.qsel_out) it.qsel_out += t * sq.qsel_st;
      if (ts) ts[6] = clock64() + (uint64_t)qa[0][0] * 0;
      q_epilogue_v<AB>(p, it, agent, e, valid, qa, eps, ctr, act_t);
      if (ts) ts[7] = clock64();
    }
    if (tr) tr[2] = clock64();
    return;
  }

  // ---- gate waves
  float fz[HB][16];
  {
    const int base = S::NF2 + hb * S::PERHB + 3 * RB2;
#pragma unroll
    for (int kb = 0; kb < HB; ++kb) load_frag(W + S::off(base + g * HB + kb), lane, fz[kb]);
  }
  // gate inputs of this wave: r-wave gi_r (+ gi_n at +2H), z-wave gi_z; the n-wave's accumulator
  // starts from b_hn (held in gin0, never replaced)
  const float* gsrc =
      io.gi ? io.gi + ((int64_t)(valid ? e : 0) * p.N + agent) * 3 * H + hb * 32 + (g == 1 ? H : 0) : nullptr;
  auto load_gi = [&](int t, float (&a0)[16], float (&a1)[16]) {
    const float* src = gsrc + (int64_t)t * sq.gi_st;
#pragma unroll
    for (int s = 0; s < 16; ++s) a0[s] = src[kperm(s, hh)];
    if (g == 0) {
#pragma unroll
      for (int s = 0; s < 16; ++s) a1[s] = src[2 * H + kperm(s, hh)];
    }
  };
  float gin0[16], gin1[16], nxt0[16], nxt1[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) gin1[s] = nxt1[s] = 0.0f;
  if (g < 2) {
    load_gi(0, gin0, gin1);
  } else {
    const f32x16 bhn = load_bias(W + CG::off_bhn + hb * 32, hh);
#pragma unroll
    for (int s = 0; s < 16; ++s) gin0[s] = bhn[s];
  }
  // reset flag of the next step: loaded one step ahead by the r-wave of hb 0 (a loader wave), handed to
  // all gate waves through LDS (zreset) so the n-wave never waits on a load
  int rst_raw = 0;
  const bool rst_loader = g == 0 && hb == 0;
  // n-wave: write the save rows of step ts (staged in svs[ts & 1][hb]) as 128-byte runs
  auto write_saves = [&](int ts) {
    const int fl = lane & 31;   // lanes 0-31: env 2q, lanes 32-63: env 2q + 1
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int el = 2 * q + hh, ee = tile * 32 + el;
      float v[6];
#pragma unroll
      for (int fld = 0; fld < 6; ++fld) v[fld] = svs[ts & 1][hb][fld][fl][el];
      if (ee < p.E) {
        float* row = io.save + ts * sq.save_st + ((int64_t)ee * p.N + agent) * SROW + F1 + G + hb * 32 + fl;
#pragma unroll
        for (int fld = 0; fld < 6; ++fld) row[fld * H] = v[fld];
      }
    }
  };
  const bool saver = g == 2 && io.save != nullptr;
  // drain the prologue loads here, so the loop's wait analysis starts from an empty counter (otherwise
  // it waits for the whole next-step prefetch before the first MFMA of every step)
  __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0) (builtin, so the compiler's wait analysis sees it)
  for (int t = 0; t < sq.C; ++t) {
    uint64_t* ts = tr ? tr + 4 + t * 8 : nullptr;
    if (ts) ts[0] = clock64();
    const bool zero_h = !valid || t == 0 || zreset[lane] != 0;
    if (g < 2 && t + 1 < sq.C) load_gi(t + 1, nxt0, nxt1);   // prefetch next step's inputs
    if (rst_loader && t + 1 < sq.C && valid) rst_raw = sq.reset[(int64_t)t * sq.reset_st + e];
    // h_{t-1} (+0.0 after a reset): unconditional LDS reads masked bitwise, no per-element branches
    const uint32_t keep = zero_h ? 0u : 0xFFFFFFFFu;
    f32x16 h0[HB];
#pragma unroll
    for (int kb = 0; kb < HB; ++kb)
#pragma unroll
      for (int s = 0; s < 16; ++s) h0[kb][s] = __uint_as_float(__float_as_uint(hx[t & 1][kb][s][lane]) & keep);
    f32x16 acc;
#pragma unroll
    for (int s = 0; s < 16; ++s) acc[s] = gin0[s];
#pragma unroll
    for (int kb = 0; kb < HB; ++kb)
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = mfma32(fz[kb][s], h0[kb][s], acc);
    if (ts) ts[1] = clock64() + (uint64_t)acc[0] * 0;
    // each gate wave finishes its own gate before the hand-over (the r-wave's critical section after
    // barrier A is then only n and h'): z-wave z = sigmoid, n-wave the raw W_hn h + b_hn; both stage
    // their save field
    const int el0 = lane & 31;
    if (g == 0) {
#pragma unroll
      for (int s = 0; s < 16; ++s) acc[s] = sigmoidf_(acc[s]);   // r
    } else {
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const float v = g == 1 ? sigmoidf_(acc[s]) : acc[s];
        gx[g - 1][hb][s][lane] = v;
        if (io.save) svs[t & 1][hb][g == 1 ? 2 : 4][kperm(s, hh)][el0] = v;
      }
    }
    lds_sync();   // A: gate values visible
    if (ts) ts[2] = clock64();
    if (g == 0) {
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        float h0v = h0[0][s];
#pragma unroll
        for (int kb = 1; kb < HB; ++kb)
          if (kb == hb) h0v = h0[kb][s];
        const float r = acc[s];
        const float z = gx[0][hb][s][lane];
        const float anh = gx[1][hb][s][lane];
        const float n = tanhf_(gin1[s] + r * anh);
        const float h1v = n + z * (h0v - n);
        hx[(t + 1) & 1][hb][s][lane] = h1v;
        if (s == 0 && rst_loader) zreset[lane] = rst_raw;   // read by every gate wave after barrier B
        if (io.save) {
          const int fs = kperm(s, hh);
          svs[t & 1][hb][0][fs][el0] = h0v;
          svs[t & 1][hb][1][fs][el0] = r;
          svs[t & 1][hb][3][fs][el0] = n;
          svs[t & 1][hb][5][fs][el0] = h1v;
        }
      }
    } else if (saver && t > 0) {
      write_saves(t - 1);   // step t-1 rows, complete since barrier B of step t-1
    }
    if (ts) ts[3] = clock64();
    lds_sync();   // B: new hidden of step t complete
    if (ts) ts[4] = clock64();
    if (g < 2) {
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        gin0[s] = nxt0[s];
        gin1[s] = nxt1[s];
      }
    }
  }
  if (saver) write_saves(sq.C - 1);
  if (tr) tr[1] = clock64();
}

// The two nets take separate (inlined) copies of the body: each copy reads its own kernel arguments
// directly (scalar loads), where a reference selected at run time between the two would be read
// through a generic pointer, one vector-memory round trip per field use inside the step loop.
template <int F1, int G, int H, int AB>
__global__ __launch_bounds__(64 * (3 * (H / 32) + 1)) void agent_rec_seq_gp_kernel(QFwdParams p0, QFwdParams p1,
                                                                                   RecSeq s0, RecSeq s1) {
  extern __shared__ __attribute__((aligned(16))) char rlds[];
  if ((int)blockIdx.x >= p0.nblocks)
    rec_seq_gp_body<F1, G, H, AB>(p1, s1, (int)blockIdx.x - p0.nblocks, rlds);
  else
    rec_seq_gp_body<F1, G, H, AB>(p0, s0, (int)blockIdx.x, rlds);
}

// One launch serves one or two nets (e.g. the target net on s'_t and the behavior net on
// s_{t+1} of the next rollout step): blocks [0, p0.nblocks) run net 0, the rest net 1.
// Two waves per SIMD (launch_bounds 256 x 2 blocks/CU) so one wave's fragment loads hide
// under the other's MFMAs.
template <int F1, int G, int H, int AB>
__global__ __launch_bounds__(256, (F1 > 64 ? 1 : 2)) void agent_q_fwd_kernel(QFwdParams p0, QFwdParams p1) {
  const bool second = (int)blockIdx.x >= p0.nblocks;
  const QFwdParams& p = second ? p1 : p0;
  const int bid = second ? (int)blockIdx.x - p0.nblocks : (int)blockIdx.x;
  const int agent = bid % p.N, tile = bid / p.N;
  const int e = tile * 128 + (threadIdx.x >> 6) * 32 + (threadIdx.x & 31);
  const float* orow = obs_row_ptr(p, agent, e);
  float xn[16];
  load_obs_kblock(orow, 0, p.D, xn);
  const bool zero_h = e >= p.E || (p.io.reset && p.io.reset[e]);
  agent_q_fwd_body<F1, G, H, AB>(p, agent, e, p.packed + (int64_t)agent * p.g.agent_stride,
                                 [&](int kb, float (&x)[16]) { load_obs_kblock(orow, kb, p.D, x); }, xn, zero_h);
}

// ---------------------------------------------------------------- fp16x3-split forward (large E)
// Same network, but every fp32 product W*x runs as three f16 MFMAs with fp32 accumulation:
//   W*x ~= Wh*xh + Wh*xl + Wl*xh,  Wh = f16(W), Wl = f16(W - Wh) (same split for x).
// Each f16 x f16 product is exact in fp32; the dropped Wl*xl and the split residuals are ~2^-22
// relative (fp16 subnormals bound the absolute error of small parts by 2^-25), so results agree
// with the fp32 network to ~1e-6 relative (tests: rtol 1e-5 vs the oracle). Per 32-deep k-step:
// 3 x v_mfma_f32_16x16x32_f16 (16 cycles each) per 16 output rows instead of 16 x 64-cycle f32
// MFMAs per 32 rows: 5.3x less MFMA time.
// Mapping: one wave = 16 envs of one agent (16x16 tiles: feature rows x env columns), 16 waves
// (256 envs of one agent) per 1024-thread block sharing the agent's LDS image: 4 waves per SIMD
// to hide the per-wave dependency chain. A 16x16 D tile gives lane (c = l&15, g = l>>4) rows
// 4g..4g+3; two consecutive tiles are directly the next layer's 32-deep k-step B fragment with
// element j <-> feature 16(j>>2) + 4g + (j&3) (kperm16), so layers chain through registers.
// Weight image (packed + N*agent_stride, same 32x32-block geometry as the f32 image): per block
// [16-row half q][part hi|lo][lane][8 halves] = 4 KiB, every A fragment one conflict-free
// ds_read_b128 (lane (i, g) of half q holds W[32rb + 16q + i][32kb + kperm16(j, g)]); biases in
// natural order.
#ifndef MM_H3_LB
#define MM_H3_LB 1
#endif
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__host__ __device__ __forceinline__ int kperm16(int j, int g) { return 16 * (j >> 2) + 4 * g + (j & 3); }

__device__ __forceinline__ f32x4 mfma16x16(const f16x8& a, const f16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// one 32-deep k-step of B: hi / lo parts
struct KS {
  f16x8 h, l;
};
#ifndef MM_SPLIT_MIX
#define MM_SPLIT_MIX 1
#endif
typedef _Float16 f16x2_ __attribute__((ext_vector_type(2)));
typedef float f32x2_ __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split8(const float (&x)[8], KS& t, int lo_pairs = 4) {
#if MM_SPLIT_MIX
  // per pair: hi = v_cvt_pk_f16_f32 (round to nearest even, as (_Float16)x), lo = f16(x - hi) by v_fma_mixlo / mixhi
  // (fma(hi, -1, x) with hi read as f16 and x as f32: the residual x - hi is exact in f32, rounded once to f16 — the
  // same bits as (_Float16)(x - (float)hi)); 3 VALU per pair instead of ~5.5
  uint32_t hw[4], lw[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x2_ v = {x[2 * j], x[2 * j + 1]};
    hw[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2_));
    uint32_t lo;
    if (j >= lo_pairs) {
      lw[j] = 0u;   // (pairs known to be exact in f16: lo = +0, what the fma_mix pair would give)
    } else {
      asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hw[j]), "v"(v.x));
      asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hw[j]), "v"(v.y));
      lw[j] = lo;
    }
  }
  t.h = __builtin_bit_cast(f16x8, hw);
  t.l = __builtin_bit_cast(f16x8, lw);
#else
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 hv = (_Float16)x[j];
    t.h[j] = hv;
    t.l[j] = (_Float16)(x[j] - (float)hv);
  }
#endif
}
// two consecutive 16-row D tiles -> one k-step
__device__ __forceinline__ void split_pair(const f32x4& a, const f32x4& b, KS& t) {
  float x[8];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    x[r] = a[r];
    x[4 + r] = b[r];
  }
  split8(x, t);
}
// acc (16 rows: half q of block blk) += W * X(k-step)
__device__ __forceinline__ void mm16(const float* __restrict__ blk, int q, const KS& x, int lane, f32x4& acc) {
  const f16x8 ah = *reinterpret_cast<const f16x8*>(blk + (q * 2) * 256 + lane * 4);
  const f16x8 al = *reinterpret_cast<const f16x8*>(blk + (q * 2 + 1) * 256 + lane * 4);
  acc = mfma16x16(al, x.h, acc);
  acc = mfma16x16(ah, x.l, acc);
  acc = mfma16x16(ah, x.h, acc);
}
// the same for a k-step whose X is exactly f16 (x.l == 0: {0, 1} observation bits): Wl·xh + Wh·xh, same sum
// (the skipped Wh·xl term is exactly 0; the accumulation order of the other two is unchanged)
__device__ __forceinline__ void mm16_x16(const float* __restrict__ blk, int q, const KS& x, int lane, f32x4& acc) {
  const f16x8 ah = *reinterpret_cast<const f16x8*>(blk + (q * 2) * 256 + lane * 4);
  const f16x8 al = *reinterpret_cast<const f16x8*>(blk + (q * 2 + 1) * 256 + lane * 4);
  acc = mfma16x16(al, x.h, acc);
  acc = mfma16x16(ah, x.h, acc);
}
struct Frag {
  f16x8 h, l;
};
__device__ __forceinline__ Frag ldfrag(const float* __restrict__ blk, int q, int lane) {
  Frag f;
  f.h = *reinterpret_cast<const f16x8*>(blk + (q * 2) * 256 + lane * 4);
  f.l = *reinterpret_cast<const f16x8*>(blk + (q * 2 + 1) * 256 + lane * 4);
  return f;
}
__device__ __forceinline__ void mmf(const Frag& a, const KS& x, f32x4& acc) {
  acc = mfma16x16(a.l, x.h, acc);
  acc = mfma16x16(a.h, x.l, acc);
  acc = mfma16x16(a.h, x.h, acc);
}
__device__ __forceinline__ f32x4 bias4(const float* __restrict__ b, int t, int g) {
  return *reinterpret_cast<const f32x4*>(b + 16 * t + 4 * g);
}
// obs k-step kb: lane (c, g) holds obs features 32 kb + kperm16(j, g)
__device__ __forceinline__ void load_obs_ks(const float* orow, int kb, int D, float (&x)[8]) {
  const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = kb * 32 + kperm16(j, g);
    x[j] = (orow && k < D) ? orow[k] : 0.0f;
  }
}

// Q output / argmax / eps-greedy / gather epilogue for 16-row Q tiles (rows 16t + 4g + r).
// out_off: element offset of the act / qsel outputs (the fused rollout step's ring slot)
template <int AT>
__device__ __forceinline__ int q_epilogue16(const QFwdParams& p, int agent, int e, bool valid,
                                            const f32x4 (&qa)[AT], float eps, uint64_t ctr, int64_t out_off = 0,
                                            const uint64_t* rng_in = nullptr) {
  const int g = (threadIdx.x & 63) >> 4;
  const mm_qfwd_io& io = p.io;
  if (valid && io.q_out) {
    float* qrow = io.q_out + (int64_t)e * io.q_se + (int64_t)agent * io.q_sa;
#pragma unroll
    for (int t = 0; t < AT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * t + 4 * g + r;
        if (row < p.A) qrow[row] = qa[t][r];
      }
  }
  if (io.mode == MM_Q_NONE) return 0;
  float best = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int t = 0; t < AT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * t + 4 * g + r;
      const float v = qa[t][r];
      if (row < p.A && (v > best || (v == best && row < bi))) {
        best = v;
        bi = row;
      }
    }
#pragma unroll
  for (int o = 16; o <= 32; o <<= 1) {
    const float ob = __shfl_xor(best, o);
    const int oi = __shfl_xor(bi, o);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  int act = bi;
  if (io.mode == MM_Q_ACT) {
#ifndef MM_RNG_SPLIT
#define MM_RNG_SPLIT 1
#endif
    if (MM_RNG_SPLIT && !io.u && !io.rand_act) {
      // both device draws of env c in ONE rng_draw sequence: lanes of even g draw the uniform, odd g the random
      // action (the same (seed, counter, e, b) streams as two calls), exchanged across g by an xor-16 shuffle
      const bool ra_lane = (g & 1) != 0;
      // (rng_in: this lane's rng_inner(e, b), computed once per launch by the chunk-persistent rollout)
      const uint64_t sd = ra_lane ? io.seed ^ 0x5bd1e995ull : io.seed;
      const uint64_t r = rng_in ? rng_draw_inner(sd, ctr, *rng_in)
                                : rng_draw(sd, ctr, (uint64_t)e, ra_lane ? (uint64_t)agent : 0xFFFFFFFFull);
      const float uu = rng_uniform(r);
      const uint32_t Au = (uint32_t)p.A;
      const int ra = (int)rng_mod_small_u(r, Au, 0xFFFFFFFFu / Au, (0xFFFFFFFFu % Au + 1u) % Au);
      const float uo = __shfl_xor(uu, 16);
      const int rao = __shfl_xor(ra, 16);
      if ((ra_lane ? uo : uu) <= eps) act = ra_lane ? ra : rao;
    } else {
      float u;
      if (io.u) {
        u = valid ? io.u[e] : 1.0f;
      } else {
        u = rng_uniform(rng_draw(io.seed, ctr, (uint64_t)e, 0xFFFFFFFFull));
      }
      if (u <= eps) {
        if (io.rand_act) {
          act = valid ? io.rand_act[(int64_t)e * p.N + agent] : 0;
        } else {
          act = (int)(rng_draw(io.seed ^ 0x5bd1e995ull, ctr, (uint64_t)e, (uint64_t)agent) % (uint64_t)p.A);
        }
      }
    }
  } else if (io.mode == MM_Q_GATHER) {
    act = valid ? io.act_in[(int64_t)e * io.act_se + agent] : 0;
  }
  float mine = 0.0f;
#pragma unroll
  for (int t = 0; t < AT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (16 * t + 4 * g + r == act) mine = qa[t][r];
  mine += __shfl_xor(mine, 16);
  mine += __shfl_xor(mine, 32);
  const float qsel = (io.mode == MM_Q_MAX) ? best : mine;
  if (valid && g == 0) {
    const int64_t o = out_off + (int64_t)e * p.N + agent;
    if (io.act_out && io.mode == MM_Q_ACT) io.act_out[o] = act;
    if (io.qsel_out) io.qsel_out[o] = qsel;
  }
  return act;
}

// ol(kb, x) loads observation k-step kb (lane (c, g) holds features 32 kb + kperm16(j, g) of env e)
template <int F1, int G, int H, int AB, class OL>
__device__ __forceinline__ int agent_q_fwd_body_h3(const QFwdParams& p, int agent, int e,
                                                    const float* __restrict__ W, const OL& ol,
                                                    float (&xn)[8], const f32x4 (&h0)[H / 16], float eps,
                                                    uint64_t ctr, int64_t out_off = 0, int x16_from_kb = 1 << 30,
                                                    f32x4 (*h1_keep)[H / 16] = nullptr, bool store_h = true,
                                                    const uint64_t* rng_in = nullptr) {
  using CG = QnetCGeo<F1, G, H, AB>;
  constexpr int T1 = F1 / 16, T2 = G / 16, TH = H / 16, AT = (AB * 32 + 15) / 16;
  constexpr int RB1 = F1 / 32, RB2 = G / 32, HB = H / 32;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const bool valid = e < p.E;
  const mm_qfwd_io& io = p.io;
  const int ATr = (p.A + 15) / 16;   // Q tiles that hold real actions
#ifndef MM_LDS_REBASE
#define MM_LDS_REBASE 1
#endif
  // LDS image addressing of the post-layer-1 fragments and the biases: per-lane base pointers every 15360 floats (each
  // 4 KiB block then lies within the 64 KiB immediate offset of its base) and one for the biases (+ 4 g), made opaque in
  // the LDS address space, so each ds_read_b128 is base + immediate (no v_add per fragment beyond the first 64 KiB)
  constexpr int NWB = (CG::off_b1 + 15359) / 15360;
  auto lds_opaque = [](const float* q) {
    auto l = (const __attribute__((address_space(3))) float*)q;
    if (MM_LDS_REBASE) asm volatile("" : "+v"(l));
    return (const float*)l;
  };
  const float* WL[NWB];
#pragma unroll
  for (int k = 0; k < NWB; ++k) WL[k] = lds_opaque(W + 15360 * k + lane * 4);
  const float* WBias = lds_opaque(W + CG::off_b1 + 4 * g);
  // fragment block at image offset off (compile-time), lane part included / bias tile t of the vector at offset off
  auto wblk = [&](int off) { return WL[off / 15360] + (off % 15360); };
  auto wbias = [&](int off, int t) { return *reinterpret_cast<const f32x4*>(WBias + (off - CG::off_b1) + 16 * t); };
  auto mmb = [&](int off, int q, const KS& x, f32x4& acc) {
    const f16x8 ah = *reinterpret_cast<const f16x8*>(wblk(off) + (q * 2) * 256);
    const f16x8 al = *reinterpret_cast<const f16x8*>(wblk(off) + (q * 2 + 1) * 256);
    acc = mfma16x16(al, x.h, acc);
    acc = mfma16x16(ah, x.l, acc);
    acc = mfma16x16(ah, x.h, acc);
  };
  auto frag = [&](int off, int q) {
    Frag f;
    f.h = *reinterpret_cast<const f16x8*>(wblk(off) + (q * 2) * 256);
    f.l = *reinterpret_cast<const f16x8*>(wblk(off) + (q * 2 + 1) * 256);
    return f;
  };

  // ---- layer 1 (K = D in 32-deep k-steps, next obs k-step prefetched)
  f32x4 x1[T1];
#pragma unroll
  for (int t = 0; t < T1; ++t) x1[t] = wbias(CG::off_b1, t);
  for (int kb = 0; kb < p.g.KD; ++kb) {
    KS ob;
    // observation k-steps from x16_from_kb on are exact in f16 (the rollout's 0/1 bits: no lo part at all); in the
    // rollout's k-step 0 only pair 0 (features 0, 1 of lane group 0: the two coordinates) can have one
    split8(xn, ob, kb >= x16_from_kb ? 0 : (x16_from_kb == 1 ? 1 : 4));
    if (kb + 1 < p.g.KD) ol(kb + 1, xn);
    if (kb >= x16_from_kb) {   // observation k-steps known to be exact in f16 (the fused rollout step's bits)
#pragma unroll
      for (int t = 0; t < T1; ++t)
        mm16_x16(W + CG::off_l1 + (int64_t)((t >> 1) * p.g.KD + kb) * 1024, t & 1, ob, lane, x1[t]);
    } else {
#pragma unroll
      for (int t = 0; t < T1; ++t)
        mm16(W + CG::off_l1 + (int64_t)((t >> 1) * p.g.KD + kb) * 1024, t & 1, ob, lane, x1[t]);
    }
  }
  KS x1s[RB1];
#pragma unroll
  for (int t = 0; t < T1; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) x1[t][r] = relu_bits(x1[t][r]);
#pragma unroll
  for (int kb = 0; kb < RB1; ++kb) split_pair(x1[2 * kb], x1[2 * kb + 1], x1s[kb]);
  float* sv = (io.save && valid) ? io.save + ((int64_t)e * p.N + agent) * (F1 + G + 6 * H) : nullptr;
  if (sv) {
#pragma unroll
    for (int t = 0; t < T1; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) sv[16 * t + 4 * g + r] = x1[t][r];
  }

  // ---- layer 2
  f32x4 x2[T2];
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    x2[t] = wbias(CG::off_b2, t);
#pragma unroll
    for (int kb = 0; kb < RB1; ++kb) mmb(CG::off_l2 + ((t >> 1) * RB1 + kb) * 1024, t & 1, x1s[kb], x2[t]);
#pragma unroll
    for (int r = 0; r < 4; ++r) x2[t][r] = relu_bits(x2[t][r]);
    if (sv) {
#pragma unroll
      for (int r = 0; r < 4; ++r) sv[F1 + 16 * t + 4 * g + r] = x2[t][r];
    }
  }
  KS x2s[RB2];
#pragma unroll
  for (int kb = 0; kb < RB2; ++kb) split_pair(x2[2 * kb], x2[2 * kb + 1], x2s[kb]);

  // ---- GRU cell (h0 loaded by the caller at kernel start)
  KS h0s[HB];
#pragma unroll
  for (int kb = 0; kb < HB; ++kb) split_pair(h0[2 * kb], h0[2 * kb + 1], h0s[kb]);
  float* hop = (valid && io.h_out && store_h) ? io.h_out + (int64_t)e * io.hout_se + (int64_t)agent * io.hout_sa +
                                         (int64_t)(4 * g) * io.hout_sf
                                   : nullptr;
  // GRU: per hidden tile t and k-step, the three gates' fragments are read together and their
  // 9 MFMAs interleaved (gate r, z, n, r, z, n, ...): consecutive MFMAs are independent, so no
  // accumulator read-after-write stall between them.
  f32x4 h1[TH];
#pragma unroll
  for (int t = 0; t < TH; ++t) {
    const int rb = t >> 1, q = t & 1;
    f32x4 ar = wbias(CG::off_brz, t);
    f32x4 az = wbias(CG::off_brz + H, t);
    f32x4 anx = wbias(CG::off_bin, t);
    f32x4 anh = wbias(CG::off_bhn, t);
    auto tri = [&](int base, int gstride, const KS& x, f32x4& a0, f32x4& a1, f32x4& a2) {
      const Frag f0 = frag(base, q);
      const Frag f1 = frag(base + gstride, q);
      const Frag f2 = frag(base + 2 * gstride, q);
      a0 = mfma16x16(f0.l, x.h, a0);
      a1 = mfma16x16(f1.l, x.h, a1);
      a2 = mfma16x16(f2.l, x.h, a2);
      a0 = mfma16x16(f0.h, x.l, a0);
      a1 = mfma16x16(f1.h, x.l, a1);
      a2 = mfma16x16(f2.h, x.l, a2);
      a0 = mfma16x16(f0.h, x.h, a0);
      a1 = mfma16x16(f1.h, x.h, a1);
      a2 = mfma16x16(f2.h, x.h, a2);
    };
#pragma unroll
    for (int kb = 0; kb < RB2; ++kb) tri(CG::off_ih + (rb * RB2 + kb) * 1024, HB * RB2 * 1024, x2s[kb], ar, az, anx);
#pragma unroll
    for (int kb = 0; kb < HB; ++kb) tri(CG::off_hh + (rb * HB + kb) * 1024, HB * HB * 1024, h0s[kb], ar, az, anh);
#ifndef MM_H3_PK
#define MM_H3_PK 1
#endif
#if MM_H3_PK
    // gates two rows at a time on packed f32 (v_pk_mul / v_pk_add / v_pk_fma: two values per VALU
    // issue); the transcendentals stay scalar. Same operations as sigmoidf_ / tanhf_.
    float rrs[4], zs[4], ns[4];
#pragma unroll
    for (int rp = 0; rp < 4; rp += 2) {
      const f32x2 vr = {ar[rp], ar[rp + 1]}, vz = {az[rp], az[rp + 1]};
      const f32x2 vx = {anx[rp], anx[rp + 1]}, vh = {anh[rp], anh[rp + 1]}, v0 = {h0[t][rp], h0[t][rp + 1]};
      f32x2 er = vr * -1.4426950408889634f, ez = vz * -1.4426950408889634f;
      er.x = __builtin_amdgcn_exp2f(er.x);
      er.y = __builtin_amdgcn_exp2f(er.y);
      ez.x = __builtin_amdgcn_exp2f(ez.x);
      ez.y = __builtin_amdgcn_exp2f(ez.y);
      er = er + 1.0f;
      ez = ez + 1.0f;
      f32x2 rr, z;
      rr.x = __builtin_amdgcn_rcpf(er.x);
      rr.y = __builtin_amdgcn_rcpf(er.y);
      z.x = __builtin_amdgcn_rcpf(ez.x);
      z.y = __builtin_amdgcn_rcpf(ez.y);
      f32x2 en = (vx + rr * vh) * 2.8853900817779268f;
      en.x = __builtin_amdgcn_exp2f(en.x);
      en.y = __builtin_amdgcn_exp2f(en.y);
      en = en + 1.0f;
      f32x2 n;
      n.x = __builtin_amdgcn_rcpf(en.x);
      n.y = __builtin_amdgcn_rcpf(en.y);
      n = 1.0f - 2.0f * n;
      const f32x2 hn = n + z * (v0 - n);
      h1[t][rp] = hn.x;
      h1[t][rp + 1] = hn.y;
      rrs[rp] = rr.x;
      rrs[rp + 1] = rr.y;
      zs[rp] = z.x;
      zs[rp + 1] = z.y;
      ns[rp] = n.x;
      ns[rp + 1] = n.y;
    }
    if (sv) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* o = sv + F1 + G + 16 * t + 4 * g + r;
        o[0] = h0[t][r];
        o[H] = rrs[r];
        o[2 * H] = zs[r];
        o[3 * H] = ns[r];
        o[4 * H] = anh[r];
        o[5 * H] = h1[t][r];
      }
    }
#else
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float rr = sigmoidf_(ar[r]);
      const float z = sigmoidf_(az[r]);
      const float n = tanhf_(anx[r] + rr * anh[r]);
      h1[t][r] = n + z * (h0[t][r] - n);
      if (sv) {
        float* o = sv + F1 + G + 16 * t + 4 * g + r;
        o[0] = h0[t][r];
        o[H] = rr;
        o[2 * H] = z;
        o[3 * H] = n;
        o[4 * H] = anh[r];
        o[5 * H] = h1[t][r];
      }
    }
#endif
    if (hop) {
#pragma unroll
      for (int r = 0; r < 4; ++r) hop[(int64_t)(16 * t + r) * io.hout_sf] = h1[t][r];
    }
  }
  if (h1_keep) {
#pragma unroll
    for (int t = 0; t < TH; ++t) (*h1_keep)[t] = h1[t];
  }
  KS h1s[HB];
#pragma unroll
  for (int kb = 0; kb < HB; ++kb) split_pair(h1[2 * kb], h1[2 * kb + 1], h1s[kb]);

  // ---- Q head (only the 16-row tiles that hold real actions)
  f32x4 qa[AT];
#pragma unroll
  for (int t = 0; t < AT; ++t) {
    qa[t] = wbias(CG::off_bq, t);
    if (t < ATr) {
#pragma unroll
      for (int kb = 0; kb < HB; ++kb) mmb(CG::off_q + ((t >> 1) * HB + kb) * 1024, t & 1, h1s[kb], qa[t]);
    }
  }
  return q_epilogue16<AT>(p, agent, e, valid, qa, eps, ctr, out_off, rng_in);
}

// The LDS-staged large-E kernel on the fp16x3 image: a 1024-thread block (16 waves x 16 envs = 256
// envs of one agent) first DMAs the agent's image into LDS (global_load_lds_dwordx4, issued after
// every global read of the wave so the latencies overlap), then runs the body. One block per CU.
template <int F1, int G, int H, int AB>
__global__ __launch_bounds__(1024, MM_H3_LB) void agent_q_fwd_h3_kernel(QFwdParams p0, QFwdParams p1) {
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  const bool second = (int)blockIdx.x >= p0.nblocks;
  // the selected net's parameters read straight from the kernarg segment (p0, p1 back to back):
  // uniform scalar loads on demand instead of both structs held (and spilled) in SGPRs
  const QFwdParams* kargs = (const QFwdParams*)__builtin_amdgcn_kernarg_segment_ptr();
  static_assert(sizeof(QFwdParams) % 8 == 0, "kernarg layout");
  const QFwdParams& p = kargs[second ? 1 : 0];
  (void)p1;
  const int bid = second ? (int)blockIdx.x - p0.nblocks : (int)blockIdx.x;
  const int agent = bid % p.N, tile = bid / p.N;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // range guard (qnet_h3_bound_block): an agent whose split operands could leave the f16 range runs
  // this block on the exact-f32 image (8 waves x 32 envs = the same 256 envs), the rest idle
  if (reinterpret_cast<const int*>(p.packed + 2 * p.g.agent_stride * p.N)[agent]) {
    const int e32 = tile * 256 + wave * 32 + (lane & 31);
    const float* src32 = p.packed + (int64_t)agent * p.g.agent_stride;
    const int nch = (int)(p.g.agent_stride >> 8);
    for (int c = wave; c < nch; c += 16)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src32 + c * 256 + lane * 4),
                                       (__attribute__((address_space(3))) void*)(wsm + c * 256), 16, 0, 0);
    const float* orow32 = obs_row_ptr(p, agent, e32);
    float x32[16];
    load_obs_kblock(orow32, 0, p.D, x32);
    const bool zero_h = e32 >= p.E || (p.io.reset && p.io.reset[e32]);
    __syncthreads();
    if (wave < 8)
      agent_q_fwd_body<F1, G, H, AB>(p, agent, e32, wsm,
                                     [&](int kb, float (&x)[16]) { load_obs_kblock(orow32, kb, p.D, x); }, x32,
                                     zero_h);
    return;
  }
  const int e = tile * 256 + wave * 16 + (lane & 15);
  const int g = lane >> 4;
  // weight image DMA first (no dependencies), then the wave's own global reads: the hidden state
  // (independent of the reset flag: loaded unconditionally, zeroed after), the obs row index and
  // the obs k-step 0 that depends on it. All latencies overlap before the barrier.
  const float* src = p.packed + (int64_t)p.N * p.g.agent_stride + (int64_t)agent * p.g.agent_stride;
  const int nchunk = (int)(p.g.agent_stride >> 8);
  for (int c = wave; c < nchunk; c += 16)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c * 256 + lane * 4),
                                     (__attribute__((address_space(3))) void*)(wsm + c * 256), 16, 0, 0);
  const mm_qfwd_io& io = p.io;
  const int ec = min(e, p.E - 1);
  f32x4 h0[H / 16];
  if (io.h_in) {
    const float* hp = io.h_in + (int64_t)ec * io.hin_se + (int64_t)agent * io.hin_sa + (int64_t)(4 * g) * io.hin_sf;
#pragma unroll
    for (int t = 0; t < H / 16; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) h0[t][r] = hp[(int64_t)(16 * t + r) * io.hin_sf];
  } else {
#pragma unroll
    for (int t = 0; t < H / 16; ++t) h0[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool reset = io.reset && io.reset[ec];
  const float* orow = obs_row_ptr(p, agent, e);
  float xn[8];
  load_obs_ks(orow, 0, p.D, xn);
  const float eps = (io.mode == MM_Q_ACT && io.eps_ptr) ? *io.eps_ptr : io.epsilon;
  const uint64_t ctr = (io.mode == MM_Q_ACT && io.counter_ptr) ? *io.counter_ptr : io.counter;
  if (e >= p.E || reset) {
#pragma unroll
    for (int t = 0; t < H / 16; ++t) h0[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  if (wave >= 8)
    for (int i = 0; i < p.stagger; ++i) __builtin_amdgcn_s_sleep(8);
  agent_q_fwd_body_h3<F1, G, H, AB>(p, agent, e, wsm,
                                    [&](int kb, float (&x)[8]) { load_obs_ks(orow, kb, p.D, x); }, xn, h0, eps, ctr);
}

// ---------------------------------------------------------------- fused rollout step
// ONE launch per rollout step for the LDS-staged geometry (E >= 2048, the image in LDS): the env step of
// step t (the restated Checkers dynamics of env.hip, oracle/env.py) inside the dual forward of
// agent_q_fwd_h3_kernel (target net on s'_t, behavior net on s_{t+1}). It replaces the env launch + the
// forward launch of the two-launch engine step (vdn/main.py:93-143: sample_action -> env.step -> store ->
// target max_a Q'), with identical results.
//
// Every block (256 envs x one agent x one net) runs the env dynamics of its 256 envs itself: the 16 blocks of
// an env tile compute the same transitions redundantly and each builds its own agent's observation k-steps
// straight from the grid in LDS, so no observation is read from HBM and no block waits for another. Block
// timeline (tools/roll_trace.py): (1) all 16 waves stage the tile's env inputs (grids, positions, actions,
// counters; the writer block also step t-1's TD inputs) as contiguous 1 KiB LDS-DMA pieces into the region the
// weight image later occupies; (2) waves 0-3 unpack them (one lane per env: nibble rows, packed positions /
// actions) while the writer's waves 4-15 fold the TD / chunk-store write of step t-1; (3) waves 4-15 issue the
// image DMA while waves 0-3 run the dynamics (env_step_wave_kernel's phase 1, one LDS round trip per agent);
// (4) after the barrier every wave runs agent_q_fwd_body_h3 with its obs k-steps built from the LDS grid
// (target blocks store s'_t into the chunk store on the way). Cross-block hazards are avoided by buffering
// instead of synchronisation: the env state is double-buffered (read buffer par = t % 2, the tile's writer
// block — target net, agent 0 — writes buffer 1 - par), the RNG step counter too (counter[1 - par] =
// counter[par] + 1), rewards / max Q' by step parity and the actions / Q(a) of the behavior net in a ring of
// 3, so the writer can fold in step t - 1's TD while other blocks of the same launch already write step
// t + 1's actions. At a chunk start target blocks also store s_t into slot 0.
struct RollStep {   // kernarg right after the two QFwdParams (read through the kernarg pointer)
  EnvDev env;
  const int32_t* act;      // [E][N] actions of step t
  float* store_obs;        // chunk-store obs; s'_t of (e, agent) at staging[e] * row_stride + next_off + agent * D
  int64_t row_stride, next_off;
  const int64_t* staging;  // [E] store rows of this chunk
  int64_t* cur_row;        // [E] staging[e], or -1 where the env finished (written by the writer blocks)
  float* rew;              // [E][N] rewards of step t
  uint8_t* done;           // [E]
  uint64_t* counter;       // [2] RNG step counter, double-buffered
  TdFuse td;               // step t - 1's TD / store (td.on), td.counter unused
  uint64_t* trace;         // timing trace (MM_ROLL_TRACE builds only; tools/roll_trace.py), nullptr normally
  int64_t n_rows;          // chunk-store rows: a staging row outside [0, n_rows) is never written through
  uint32_t* err;           // sticky error bits (bit 0: a corrupt staging row was skipped)
  int par, begin, lds_env, pad_;   // state buffer read; chunk start (also write s_t to slot 0); env LDS offset
};
// a store row the kernel may write through; otherwise the sticky error bit 0 is set and the row's stores skipped
__device__ __forceinline__ bool roll_row_ok(int64_t row, int64_t n_rows, uint32_t* err) {
  const bool ok = row >= 0 && row < n_rows;
  if (!ok && err) atomicOr(err, 1u);
  return ok;
}
// timing stamps (s_memrealtime, 100 MHz) of block b at trace[8 b + i] when tracing (builds with -DMM_ROLL_DEBUG=1
// only: tools/roll_trace.py, tools/roll_probe.py); compiled out of the product kernel
#ifndef MM_ROLL_DEBUG
#define MM_ROLL_DEBUG 0
#endif
#if MM_ROLL_DEBUG
#define MM_RSTAMP(i, cond)                                                                             \
  do {                                                                                                 \
    if (rs.trace && (cond) && blockIdx.x < 512) rs.trace[8 * blockIdx.x + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define MM_RSTAMP(i, cond) \
  do {                     \
  } while (0)
#endif

static_assert(sizeof(QFwdParams) % 8 == 0 && alignof(RollStep) == 8, "rollout_step kernarg layout");
#if MM_ROLL_DEBUG && defined(MM_ROLL_PROBE_BITS)
#define MM_ROLL_PROBE MM_ROLL_PROBE_BITS   // timing probes only (tools/roll_probe.py): 1 skip the env step, 2 skip the obs build, 4 skip obs stores
#else
#define MM_ROLL_PROBE 0
#endif
static constexpr int kRollMaxN = 10;    // 3 ceil(N / 2) <= 16 rows and agent markers 3 + k in a nibble
static constexpr int kRollMaxR = 16;    // rows of 8 cells: one 32-bit nibble word per row

// LDS staging of the env step (after the weight image): coordinate features, the tile's grids as nibble rows
// (row r of env l = cells (r, 0..7) at bits 4c of word l * roll_gbw(R) + r), agent cells r << 4 | c, done flags
struct RollLds {
  int stab, sgrid, spos, sdone, total;
};
__host__ __device__ __forceinline__ int roll_gbw(int R) { return R | 1; }   // odd word stride: fewer bank conflicts
__host__ __device__ __forceinline__ RollLds roll_lds(int R, int C, int N) {
  auto a16 = [](int x) { return (x + 15) & ~15; };
  RollLds m;
  int o = 0;
  m.stab = o;  o = a16(o + (R + C) * 4);
  m.sgrid = o; o = a16(o + 256 * roll_gbw(R) * 4);
  m.spos = o;  o = a16(o + 256 * N);
  m.sdone = o; o = a16(o + 256);
  m.total = o;
  return m;
}
// 4 grid bytes (codes < 16) -> 4 nibbles, and back
__device__ __forceinline__ uint32_t nib_pack4(uint32_t x) {
  return (x & 0xFu) | ((x >> 4) & 0xF0u) | ((x >> 8) & 0xF00u) | ((x >> 12) & 0xF000u);
}
__device__ __forceinline__ uint32_t nib_unpack4(uint32_t x) {
  return (x & 0xFu) | ((x & 0xF0u) << 4) | ((x & 0xF00u) << 8) | ((x & 0xF000u) << 12);
}
// position word of the global state (prev_r << 24 | prev_c << 16 | r << 8 | c) -> 16 bits (4 per field)
__device__ __forceinline__ uint32_t pos16(int32_t w) {
  return (uint32_t)((((w >> 24) & 15) << 12) | (((w >> 16) & 15) << 8) | (((w >> 8) & 15) << 4) | (w & 15));
}

// The local observation of an agent at (r, c) as a bit word: bit f = feature f (>= 2) of get_agent_obs, i.e. bit
// 2 + 5 cell + ch for the 3 x 3 cells (row-major) x {lemon, apple, even agent, odd agent, wall}; off-grid cells
// are 0 (env.hip obs_value). Item code -> channel bits by a nibble table: 1 lemon, 2 apple, 3 + k agent k.
__device__ __forceinline__ uint64_t roll_obs_word(const uint32_t* rows, int R, int r, int c) {
  const uint32_t wm = r > 0 ? rows[r - 1] : 0u, w0 = rows[r], wp = r + 1 < R ? rows[r + 1] : 0u;
  auto nb3 = [c](uint32_t w) { return (c > 0 ? (w >> (4 * c - 4)) : (w << 4)) & 0xFFFu; };   // cells c-1, c, c+1
  const uint64_t items = (uint64_t)nb3(wm) | ((uint64_t)nb3(w0) << 12) | ((uint64_t)nb3(wp) << 24);
  constexpr uint64_t kLut = 0x4848484848484210ull;   // item -> {lemon 1, apple 2, even agent 4, odd agent 8}
  uint64_t word = 0;
#pragma unroll
  for (int cell = 0; cell < 9; ++cell) {
    const uint32_t it = (uint32_t)(items >> (4 * cell)) & 15u;
    word |= ((kLut >> (4 * it)) & 15ull) << (2 + 5 * cell);
  }
  return word;
}
// roll_obs_word shared by the 4 lanes (c, g = 0..3) of one env in the fp16x3 layout: lane group g < 3 builds the 3 cells
// of grid row r - 1 + g (bits 2 + 15 g .. 16 + 15 g of the word), and two v_permlane16/32_swap ORs per dword combine
// the groups (the 4 lanes of an env differ in lane bits 4 and 5) — the same word, one row read and ~1/3 of the ALU
// per lane. Every lane of the wave must be active.
__device__ __forceinline__ uint64_t roll_obs_word_g(const uint32_t* rows, int R, int r, int c, int g) {
  const int rr = r - 1 + g;
  const uint32_t w = (g < 3 && rr >= 0 && rr < R) ? rows[rr] : 0u;
  const uint32_t f12 = (c > 0 ? (w >> (4 * c - 4)) : (w << 4)) & 0xFFFu;   // cells c-1, c, c+1
  constexpr uint64_t kLut = 0x4848484848484210ull;   // item -> {lemon 1, apple 2, even agent 4, odd agent 8}
  uint32_t f15 = 0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const uint32_t it = (f12 >> (4 * j)) & 15u;
    f15 |= (uint32_t)((kLut >> (4 * it)) & 15ull) << (5 * j);
  }
  uint32_t lo = g < 2 ? f15 << (2 + 15 * g) : 0u, hi = g == 2 ? f15 : 0u;
  auto or16 = [](uint32_t v) {
    const auto x = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return x[0] | x[1];
  };
  auto or32 = [](uint32_t v) {
    const auto x = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return x[0] | x[1];
  };
  lo = or32(or16(lo));
  hi = or32(or16(hi));
  return ((uint64_t)hi << 32) | lo;
}
// features f0 .. f0 + 3 of the word into x[0..3] (the coordinates for f < 2)
__device__ __forceinline__ void roll_feat4(uint64_t word, int f0, float cr, float cc, float* x) {
  const uint32_t fld = f0 < 64 ? (uint32_t)(word >> f0) : 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = (float)((fld >> i) & 1u);
  if (f0 == 0) {
    x[0] = cr;
    x[1] = cc;
  }
}
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
// store features f0 .. f0 + 3 (< D) of one (env, agent) row
__device__ __forceinline__ void roll_store4(float* dst, int f0, int D, const float* x) {
  if (f0 + 3 < D) {
    *reinterpret_cast<f32x4u*>(dst + f0) = f32x4u{x[0], x[1], x[2], x[3]};
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (f0 + i < D) dst[f0 + i] = x[i];
  }
}

template <int F1, int G, int H, int AB>
__global__ __launch_bounds__(1024, 1) void rollout_step_kernel(QFwdParams p0, QFwdParams p1, RollStep rs_) {
  extern __shared__ __attribute__((aligned(16))) float wsm[];
#if MM_ROLL_DEBUG
  const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();   // (timing trace only)
#endif
  const bool second = (int)blockIdx.x >= p0.nblocks;     // p0: target net on s'_t, p1: behavior net on s_{t+1}
  // parameters read from the kernarg segment on demand (uniform scalar loads) instead of held in SGPRs
  const QFwdParams* kargs = (const QFwdParams*)__builtin_amdgcn_kernarg_segment_ptr();
  const QFwdParams& p = kargs[second ? 1 : 0];
  const RollStep& rs = *reinterpret_cast<const RollStep*>(kargs + 2);
  (void)p1;
  (void)rs_;
  const int bid = second ? (int)blockIdx.x - p0.nblocks : (int)blockIdx.x;
  const int agent = bid % p.N, tile = bid / p.N;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const EnvDev& ev = rs.env;
  const int N = p.N, D = p.D, R = ev.R, C = ev.C, RC = R * C, E = p.E;
  const RollLds lay = roll_lds(R, C, N);
  char* envl = reinterpret_cast<char*>(wsm) + rs.lds_env;
  float* stab = reinterpret_cast<float*>(envl + lay.stab);
  uint8_t* sgrid = reinterpret_cast<uint8_t*>(envl + lay.sgrid);
  uint8_t* spos = reinterpret_cast<uint8_t*>(envl + lay.spos);
  uint8_t* sdone = reinterpret_cast<uint8_t*>(envl + lay.sdone);
  const bool writer = !second && agent == 0;
  const int e0 = tile * 256;
  const int par = rs.par;
  const mm_qfwd_io& io = p.io;
  const bool exact = reinterpret_cast<const int*>(p.packed + 2 * p.g.agent_stride * p.N)[agent] != 0;
  MM_RSTAMP(0, threadIdx.x == 0);

  if (threadIdx.x >= 256 && threadIdx.x < 256 + R + C) {
    const int i = threadIdx.x - 256;
    stab[i] = i < R ? ev.rtab[i] : ev.ctab[i - R];
  }

  // ---- waves 0-3: the env step of the tile, one lane per env (env_step_wave_kernel's phase 1 on nibble rows:
  // one LDS round trip per agent, the agents in a rolled loop over packed position / action registers)
  const int le_d = threadIdx.x;
  const int de = e0 + le_d;
  const bool dvalid = threadIdx.x < 256 && de < E && !(MM_ROLL_PROBE & 1);
  uint32_t pq[kRollMaxN / 2];   // 16-bit position words, agent k in half k & 1 of pq[k >> 1]
  uint32_t aq[2];               // 4-bit actions, agent k at bits 4 (k & 7) of aq[k >> 3]
  int steps0 = 0, apples0 = 0;
  int64_t myrow = 0;   // writer: this env's store row (cur_row after the step)
  uint32_t* rows = reinterpret_cast<uint32_t*>(sgrid) + le_d * roll_gbw(R);
  // the tile's env inputs are contiguous in HBM (grids [E][RC], positions / actions [E][N], counters [E]): staged
  // by all 16 waves as 1 KiB LDS-DMA pieces into the image region (free until the image DMA below), so a
  // dynamics lane then reads its env with a few ds_read_b128 instead of ~24 strided global loads
  const int ne = min(256, E - e0);
  const int st_grid = 0, st_pos = (256 * RC + 15) & ~15, st_act = st_pos + 256 * N * 4, st_steps = st_act + 256 * N * 4,
            st_apples = st_steps + 1024;
  // the writer block also stages the TD / store inputs of step t - 1 (same contiguous layout)
  const bool tdw = writer && rs.td.on;
  const int st_srow = st_apples + 1024 + 4 * 256 * N * 4 + 2048 + 1024 + 256;   // the tile's staging rows (writer)
  const int st_trew = st_apples + 1024, st_tq = st_trew + 256 * N * 4, st_tm = st_tq + 256 * N * 4,
            st_tact = st_tm + 256 * N * 4, st_trow = st_tact + 256 * N * 4, st_ctd = st_trow + 2048,
            st_tdone = st_ctd + 1024;
  {
    char* stg = reinterpret_cast<char*>(wsm);
    auto piece16 = [&](const void* src, int off, int bytes) {   // bytes of src -> stg + off, 16 B per lane
      for (int c = wave; c * 1024 < bytes; c += 16)
        if (c * 1024 + lane * 16 < bytes)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(static_cast<const char*>(src) + c * 1024 + lane * 16),
              (__attribute__((address_space(3))) void*)(stg + off + c * 1024), 16, 0, 0);
    };
    if (!(MM_ROLL_PROBE & 1)) {
      piece16((par ? ev.grid_alt : ev.grid) + (int64_t)e0 * RC, st_grid, ne * RC);
      piece16((par ? ev.pos_alt : ev.pos) + (int64_t)e0 * N, st_pos, ne * N * 4);
      piece16(rs.act + (int64_t)e0 * N, st_act, ne * N * 4);
      piece16((par ? ev.steps_alt : ev.steps) + e0, st_steps, (ne * 4 + 15) & ~15);
      piece16((par ? ev.apples_alt : ev.apples) + e0, st_apples, (ne * 4 + 15) & ~15);
    }
    if (!second) piece16(rs.staging + e0, st_srow, (ne * 8 + 15) & ~15);   // target blocks: the store rows
    if (tdw) {
      const TdFuse& td = rs.td;
      piece16(td.rew + (int64_t)e0 * N, st_trew, ne * N * 4);
      piece16(td.q_taken + (int64_t)e0 * N, st_tq, ne * N * 4);
      piece16(td.maxq + (int64_t)e0 * N, st_tm, ne * N * 4);
      piece16(td.act + (int64_t)e0 * N, st_tact, ne * N * 4);
      piece16(td.rows + e0, st_trow, (ne * 8 + 15) & ~15);
      piece16(td.chunk_td + e0, st_ctd, (ne * 4 + 15) & ~15);
      if (threadIdx.x < ne) reinterpret_cast<uint8_t*>(wsm)[st_tdone + threadIdx.x] = td.done[e0 + threadIdx.x];
    }
  }
  __syncthreads();
  if (tdw && wave >= 4) {
    // the TD / store of step t - 1 (td_chunk_kernel's arithmetic: agent-order sums per env), from the staging
    const TdFuse& td = rs.td;
    const char* stg = reinterpret_cast<const char*>(wsm);
    const float* trew = reinterpret_cast<const float*>(stg + st_trew);
    const float* tq = reinterpret_cast<const float*>(stg + st_tq);
    const float* tm = reinterpret_cast<const float*>(stg + st_tm);
    const int32_t* tact = reinterpret_cast<const int32_t*>(stg + st_tact);
    const int64_t* trow = reinterpret_cast<const int64_t*>(stg + st_trow);
    const float* ctd = reinterpret_cast<const float*>(stg + st_ctd);
    const uint8_t* tdone = reinterpret_cast<const uint8_t*>(stg + st_tdone);
    const int i = threadIdx.x - 256;   // 768 threads
    if (i < ne) {
      float sr = 0.f, sq = 0.f, st = 0.f;
      for (int j = 0; j < N; ++j) {
        sr += trew[i * N + j];
        sq += tq[i * N + j];
        st += tm[i * N + j];
      }
      const uint8_t dd = tdone[i];
      const float dn = dd ? 1.0f : 0.0f;
      const float v = rollout_td(sr, sq, st, dn, td.gamma);
      td.chunk_td[e0 + i] = (td.slot == 0 ? 0.0f : ctd[i]) + v;
      if (roll_row_ok(trow[i], rs.n_rows, rs.err)) td.s_done[trow[i] * td.C + td.slot] = dd;
    }
    for (int q = i; q < ne * N; q += 768) {
      const int l = q / N, k = q - l * N;
      if (trow[l] < 0 || trow[l] >= rs.n_rows) continue;   // (flagged above)
      const int64_t o = (trow[l] * td.C + td.slot) * N + k;
      td.s_act[o] = (uint8_t)tact[q];
      td.s_rew[o] = trew[q];
    }
  }
  if (dvalid) {
    const char* stg = reinterpret_cast<const char*>(wsm);
    const int32_t* pw = reinterpret_cast<const int32_t*>(stg + st_pos) + le_d * N;
    const int32_t* ac = reinterpret_cast<const int32_t*>(stg + st_act) + le_d * N;
    const uint4* gin = reinterpret_cast<const uint4*>(stg + st_grid + le_d * RC);
    if (writer) {
      myrow = reinterpret_cast<const int64_t*>(stg + st_srow)[le_d];
      if (!roll_row_ok(myrow, rs.n_rows, rs.err)) myrow = -1;   // a corrupt row is never handed on as cur_row
    }
    steps0 = reinterpret_cast<const int32_t*>(stg + st_steps)[le_d];
    apples0 = reinterpret_cast<const int32_t*>(stg + st_apples)[le_d];
#pragma unroll
    for (int j = 0; j < kRollMaxN / 2; ++j) pq[j] = 0u;
    aq[0] = aq[1] = 0u;
#pragma unroll
    for (int k = 0; k < kRollMaxN; ++k)
      if (k < N) {
        const int32_t w = pw[k];
        pq[k >> 1] |= pos16(w) << (16 * (k & 1));
        aq[k >> 3] |= (uint32_t)(ac[k] & 15) << (4 * (k & 7));
        spos[le_d * N + k] = (uint8_t)((pos_r(w) << 4) | pos_c(w));
      }
#pragma unroll
    for (int j = 0; j < kRollMaxR / 2; ++j)
      if (2 * j < R) {   // 16 bytes = 2 rows of 8 cells (RC = 8 R)
        const uint4 g = gin[j];
        rows[2 * j] = nib_pack4(g.x) | (nib_pack4(g.y) << 16);
        if (2 * j + 1 < R) rows[2 * j + 1] = nib_pack4(g.z) | (nib_pack4(g.w) << 16);
      }
  }
  // the store rows of this wave's envs (h3 lane mapping, and the exact path's 32-env mapping), read from the
  // staging before the image DMA overwrites it: no global round trip in front of the first obs store
  int64_t srow_h3 = 0, srow_ex = 0;
  if (!second) {
    const int64_t* st_rows = reinterpret_cast<const int64_t*>(reinterpret_cast<const char*>(wsm) + st_srow);
    const int l16 = wave * 16 + (lane & 15), l32 = wave * 32 + (lane & 31);
    // out-of-range rows -> -1 (sticky error bit 0): no store of this env goes through them
    if (e0 + l16 < E) srow_h3 = st_rows[l16];
    if (l32 < 256 && e0 + l32 < E) srow_ex = st_rows[l32];
    if (e0 + l16 < E && !roll_row_ok(srow_h3, rs.n_rows, rs.err)) srow_h3 = -1;
    if (l32 < 256 && e0 + l32 < E && !roll_row_ok(srow_ex, rs.n_rows, rs.err)) srow_ex = -1;
  }
  MM_RSTAMP(1, threadIdx.x == 0);
  __syncthreads();
#if MM_ROLL_DEBUG
  if (rs.trace && threadIdx.x == 0 && blockIdx.x < 512) rs.trace[8 * blockIdx.x + 2] = t_entry;
#endif
  // ---- waves 4-15, once the env inputs have been consumed: the weight image DMA into the staging region
  // (range-guarded agents: the exact-f32 image) while waves 0-3 run the env step
  if (wave >= 4) {
    const float* src = p.packed + (exact ? 0 : (int64_t)p.N * p.g.agent_stride) + (int64_t)agent * p.g.agent_stride;
    const int nchunk = (int)(p.g.agent_stride >> 8);
    for (int c = wave - 4; c < nchunk; c += 12)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c * 256 + lane * 4),
                                       (__attribute__((address_space(3))) void*)(wsm + c * 256), 16, 0, 0);
  }
  const int le = wave * 16 + (lane & 15), e = e0 + le;
  if (rs.begin) {
    // chunk start: slot 0 of the staging rows <- s_t, the observation of the state before this step; lane
    // (env, g) writes features 16 q + 4 g .. + 3 of its env
    __syncthreads();
    if (!second && e < E && srow_h3 >= 0) {
      const int rc = spos[le * N + agent];
      const uint64_t wd =
          roll_obs_word(reinterpret_cast<const uint32_t*>(sgrid) + le * roll_gbw(R), R, rc >> 4, rc & 15);
      const float cr = stab[rc >> 4], cc = stab[R + (rc & 15)];
      float* d0 = rs.store_obs + srow_h3 * rs.row_stride + (int64_t)agent * D;
      for (int f0 = 4 * (lane >> 4); f0 < D; f0 += 16) {
        float x[4];
        roll_feat4(wd, f0, cr, cc, x);
        roll_store4(d0, f0, D, x);
      }
    }
    __syncthreads();
  }
  if (dvalid) {
    int apples = apples0;
    const int steps = steps0 + 1;
    int32_t* pout = (par ? ev.pos : ev.pos_alt) + (int64_t)de * N;
    float* rout = rs.rew + (int64_t)de * N;
#pragma unroll 1
    for (int k = 0; k < N; ++k) {
      const uint32_t w = pq[0] & 0xFFFFu;
      const int a = (int)(aq[0] & 15u);
#pragma unroll
      for (int j = 0; j < kRollMaxN / 2 - 1; ++j) pq[j] = __builtin_amdgcn_alignbit(pq[j + 1], pq[j], 16);
      pq[kRollMaxN / 2 - 1] >>= 16;
      aq[0] = __builtin_amdgcn_alignbit(aq[1], aq[0], 4);
      aq[1] >>= 4;
      int r = (w >> 4) & 15, c = w & 15, pr = (w >> 12) & 15, pc = (w >> 8) & 15;
      const int nr = r + (a == 0 ? 1 : (a == 2 ? -1 : 0));
      const int nc = c + (a == 1 ? -1 : (a == 3 ? 1 : 0));
      const bool inside = a != 4 && nr >= 0 && nr < R && nc >= 0 && nc < C;
      // every row this agent may read or write, in one round trip: the target row, its own row, its stale prev row
      const uint32_t w_n = rows[inside ? nr : r], w_r = rows[r], w_p = rows[pr];
      asm volatile("" ::"v"(w_n), "v"(w_r), "v"(w_p));   // all three reads in flight together (not sunk into branches)
      const bool moved = inside && ((w_n >> (4 * nc)) & 15u) < 3u;
      if (moved) {
        pr = r;
        pc = c;
        r = nr;
        c = nc;
      }
      // view update (ma_gym __update_agent_view) when agent_pos != agent_prev_pos: empty at agent_prev_pos, the
      // marker at agent_pos; the fruit under a moving agent is eaten. Branch-free: both rows are written back
      // every agent (unchanged when there is no update; the (r, c) row last, so a shared row gets both edits).
      const bool upd = r != pr || c != pc;
      const uint32_t A = moved ? w_n : w_r;   // row of (r, c)
      const uint32_t B = moved ? w_r : w_p;   // row of (pr, pc)
      const uint32_t item = upd ? (A >> (4 * c)) & 15u : 0u;
      const bool big = (k & 1) == 0;
      const float rk = ev.step_cost + (item == 1u ? (big ? -10.0f : -1.0f) : (item == 2u ? (big ? 10.0f : 1.0f) : 0.0f));
      apples -= item == 2u ? 1 : 0;
      const uint32_t clr = upd ? ~(15u << (4 * pc)) : ~0u;
      const uint32_t A1 = pr == r ? (A & clr) : A;
      rows[pr] = B & clr;
      rows[r] = upd ? ((A1 & ~(15u << (4 * c))) | ((uint32_t)(3 + k) << (4 * c))) : A1;
      spos[le_d * N + k] = (uint8_t)((r << 4) | c);
      if (writer) {
        pout[k] = (pr << 24) | (pc << 16) | (r << 8) | c;
        rout[k] = rk;
      }
    }
    const bool dn = steps >= ev.max_steps || apples == 0;
    sdone[le_d] = dn ? 1 : 0;
    if (writer) {
      // the step's outputs and the next state (auto-reset where the episode ended)
      rs.done[de] = dn ? 1 : 0;
      rs.cur_row[de] = dn ? -1 : myrow;
      (par ? ev.steps : ev.steps_alt)[de] = dn ? 0 : steps;
      (par ? ev.apples : ev.apples_alt)[de] = dn ? ev.init_apples : apples;
      uint4* gout = reinterpret_cast<uint4*>((par ? ev.grid : ev.grid_alt) + (int64_t)de * RC);
      const uint4* ig = reinterpret_cast<const uint4*>(ev.init_grid);
#pragma unroll
      for (int j = 0; j < kRollMaxR / 2; ++j)
        if (2 * j < R) {
          uint4 v;
          if (dn) {
            v = ig[j];
          } else {
            const uint32_t a0 = rows[2 * j], a1 = 2 * j + 1 < R ? rows[2 * j + 1] : 0u;
            v = make_uint4(nib_unpack4(a0 & 0xFFFFu), nib_unpack4(a0 >> 16), nib_unpack4(a1 & 0xFFFFu),
                           nib_unpack4(a1 >> 16));
          }
          gout[j] = v;
        }
      if (dn)
        for (int k = 0; k < N; ++k) pout[k] = ev.init_pos[k];
    }
  }
  if (writer && tile == 0 && threadIdx.x == 0) rs.counter[1 - par] = rs.counter[par] + 1;
  MM_RSTAMP(3, threadIdx.x == 0);

  if (exact) {
    // range-guarded agent: the exact-f32 body, 8 waves x 32 envs (agent_q_fwd_h3_kernel's fallback)
    const int l32 = wave * 32 + (lane & 31), e32 = e0 + l32, hh = (lane & 63) >> 5;
    const int64_t srow32 = srow_ex;
    const bool r32 = !second && io.reset && e32 < E && io.reset[e32];
    __syncthreads();
    const bool bd = second && e32 < E && sdone[l32];
    float* dst = (!second && e32 < E && srow32 >= 0) ? rs.store_obs + srow32 * rs.row_stride + rs.next_off + (int64_t)agent * D
                                                      : nullptr;
    const int rc32 = spos[l32 * N + agent];
    const uint64_t wd32 =
        roll_obs_word(reinterpret_cast<const uint32_t*>(sgrid) + l32 * roll_gbw(R), R, rc32 >> 4, rc32 & 15);
    const float cr32 = stab[rc32 >> 4], cc32 = stab[R + (rc32 & 15)];
    // k-block kb: element s = 4 i + j holds feature 32 kb + 8 i + 4 hh + j (kperm)
    auto ol32 = [&](int kb, float (&x)[16]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int f0 = kb * 32 + 8 * i + 4 * hh;
        roll_feat4(wd32, f0, cr32, cc32, x + 4 * i);
        if (bd || e32 >= E)
#pragma unroll
          for (int j = 0; j < 4; ++j) x[4 * i + j] = (e32 < E && f0 + j < D) ? ev.reset_obs[agent * D + f0 + j] : 0.0f;
        if (dst) roll_store4(dst, f0, D, x + 4 * i);
      }
    };
    float x32[16];
    if (wave < 8) {
      ol32(0, x32);
      agent_q_fwd_body<F1, G, H, AB>(p, agent, e32, wsm, ol32, x32, e32 >= E || r32 || bd);
    }
    return;
  }
  // hidden state of this wave's 16 envs (target: reset where step t - 1 ended; behavior: where step t ended)
  const int ec = min(e, E - 1);
  const int g = lane >> 4;
  f32x4 h0[H / 16];
  {
    const float* hp = io.h_in + (int64_t)ec * io.hin_se + (int64_t)agent * io.hin_sa + (int64_t)(4 * g) * io.hin_sf;
#pragma unroll
    for (int t = 0; t < H / 16; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) h0[t][r] = hp[(int64_t)(16 * t + r) * io.hin_sf];
  }
  const bool rt = !second && io.reset && io.reset[ec];
  const float eps = (io.mode == MM_Q_ACT && io.eps_ptr) ? *io.eps_ptr : io.epsilon;
  const uint64_t ctr = (io.mode == MM_Q_ACT && io.counter_ptr) ? *io.counter_ptr : io.counter;
  __syncthreads();
  MM_RSTAMP(4, threadIdx.x == 0);
  const bool bd = second && e < E && sdone[le];
  if (e >= E || rt || bd) {
#pragma unroll
    for (int t = 0; t < H / 16; ++t) h0[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // the store destination of s'_t (target blocks), loaded after the env step (a global load before it would be
  // waited on inside the dynamics loop by the spill reloads' vmcnt)
  const int64_t srow = srow_h3;
  float* dst = (!second && e < E && srow >= 0) ? rs.store_obs + srow * rs.row_stride + rs.next_off + (int64_t)agent * D
                                               : nullptr;
  const int rc = spos[le * N + agent];
  const uint64_t wd = roll_obs_word(reinterpret_cast<const uint32_t*>(sgrid) + le * roll_gbw(R), R, rc >> 4, rc & 15);
  const float cr = stab[rc >> 4], cc = stab[R + (rc & 15)];
  // k-step kb: element 4 q + j holds feature 32 kb + 16 q + 4 g + j (kperm16)
  auto ol = [&](int kb, float (&x)[8]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int f0 = kb * 32 + 16 * q + 4 * g;
      if (MM_ROLL_PROBE & 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) x[4 * q + j] = 0.25f;
      } else {
        roll_feat4(wd, f0, cr, cc, x + 4 * q);
      }
      if (bd || e >= E)
#pragma unroll
        for (int j = 0; j < 4; ++j) x[4 * q + j] = (e < E && f0 + j < D) ? ev.reset_obs[agent * D + f0 + j] : 0.0f;
      if (dst && !(MM_ROLL_PROBE & 4)) roll_store4(dst, f0, D, x + 4 * q);
    }
  };
  float xn[8];
  ol(0, xn);
  MM_RSTAMP(5, threadIdx.x == 0);
  if (wave >= 8)
    for (int i = 0; i < p.stagger; ++i) __builtin_amdgcn_s_sleep(8);
  // observation features 32.. are {0, 1} bits of the grid (only features 0, 1, the coordinates, are not
  // exact in f16): layer-1 k-steps from 1 on skip the Wh·xl MFMA (exactly 0); behavior blocks of envs that
  // reset read the reset obs, which are the same kind of values
  agent_q_fwd_body_h3<F1, G, H, AB>(p, agent, e, wsm, ol, xn, h0, eps, ctr, 0, 1);
  MM_RSTAMP(6, threadIdx.x == 0);
  MM_RSTAMP(7, threadIdx.x == 64 * 15);
}

// ---------------------------------------------------------------- chunk-persistent rollout
// The rollout steps of (part of) one chunk in ONE launch (mm_rollout_chunk): each (net, agent, 256-env tile) block
// of rollout_step_kernel stays resident for all n steps, so its weight image is DMA'd into LDS once per launch
// instead of once per step, its copy of the tile's env state (grids, positions, dones) lives in LDS across the
// steps, and the only cross-block dependency of a step — the N behavior blocks' actions of the tile, which every
// block of the tile needs for its (redundant) env dynamics — is a tile-local hand-off through HBM (per-step
// slots, written write-through `sc1` + `s_waitcnt vmcnt(0)` + an `sc1` flag store, polled with `sc1` loads:
// MI355X_MICROARCH.md's inter-workgroup hand-off, row 1), not a launch boundary. Per step t = c0 + i (same
// arithmetic as rollout_step_kernel, results bit-identical):
//   (1) i > 0: wave 0 polls the N behavior flags of the tile; the dynamics lanes load the actions of step t;
//   (2) envs that ended at step t - 1 are reset in LDS (the launch's initial state is already post-reset);
//   (3) chunk start (c == 0): target blocks store s_t into slot 0 of their rows;
//   (4) waves 0-3: the env dynamics of step t (one lane per env, one LDS round trip per agent); the tile's
//       writer block (target net, agent 0) writes rew / done of step t into their ring positions and cur_row;
//   (5) every wave: the forward (target on s'_t -> max Q'_t, storing s'_t into slot c + 1; behavior on s_{t+1}
//       -> act / Q(a) of step t + 1 into their ring positions); behavior blocks then publish their actions.
// The TD / chunk-store fold of the launch's steps runs afterwards (mm_td_fold_range). Blocks are mapped so that a
// tile's 2N blocks share an XCD (blocks b, b + 8, ... share one: MI355X_MICROARCH.md "Workgroup dispatch"), which
// keeps the hand-off in one L2 — a speed choice only, correctness never depends on placement. All blocks must be
// co-resident (one per CU, the host checks the grid against the CU count); every wait has a time limit (sticky
// error bit 1 on expiry, the block then proceeds) so the grid always drains. The last block to finish advances
// the launch state (RNG step counter += n, env state buffer flipped, launch sequence + 1).
// the dynamic LDS of the rollout kernels (one extern array per kernel; helper for device functions)
__device__ __forceinline__ float* wsm_ptr() {
  extern __shared__ __attribute__((aligned(16))) float wsm_dyn[];
  return wsm_dyn;
}
struct RollChunk {   // kernarg right after the two QFwdParams
  EnvDev env;
  float* store_obs;
  int64_t row_stride;
  const int64_t* staging;    // [S][E] staging row sets: the launch's k-th chunk writes set (set0 + k) % S
  int64_t* cur_row;
  int64_t n_rows;
  const int32_t* act0;       // [E][N] actions of the launch's first step
  const uint8_t* done_prev;  // [E] dones of the step before the launch (the target's hidden reset of step c0)
  float* rew;                // ring [RL][E][N]: rewards of launch step i at ring position (pos0 + i) % RL
  uint8_t* done;             // ring [RL][E]
  uint64_t* counter;         // RNG step counter (step c0 + i draws with *counter + i)
  uint64_t* seq;             // launch sequence number (hand-off flag epoch)
  int32_t* envpar;           // env state buffer read (0 / 1)
  uint32_t* ticket;          // blocks finished
  uint64_t* hx;              // [T][C][N][32] hand-off words, one slot per step: (seq + 1) << 32 | 8 envs' 4-bit actions
  uint32_t* err;             // sticky error bits: 1 staging row outside the store, 2 hand-off wait expired
  uint64_t* trace;           // per-step timing stamps (MM_ROLL_DEBUG builds, tools/chunk_trace.py), else nullptr
  int c0, n, CL, lds_env;   // first step's chunk position, steps, chunk length, LDS offset of the env state
  int S, set0, RL, pos0;     // staging sets, the first chunk's set, ring length (steps), the first step's ring position
  int hxl;                   // hand-off word slots per tile (steps): launch step i's words at slot i
};
static_assert(alignof(RollChunk) == 8, "rollout_chunk kernarg layout");
static constexpr uint64_t kHandoffTimeout = 2000000;   // s_memrealtime ticks (100 MHz): 20 ms

// LDS after the weight image: coordinate features, nibble-row grids, 16-bit position words (prev_r, prev_c, r, c),
// dones by step parity, the behavior block's outgoing actions
struct RollChunkLds {
  int stab, sgrid, spq, ssa, sdone, shx, total;
};
__host__ __device__ __forceinline__ RollChunkLds roll_chunk_lds(int R, int C, int N) {
  auto a16 = [](int x) { return (x + 15) & ~15; };
  RollChunkLds m;
  int o = 0;
  m.stab = o;  o = a16(o + (R + C) * 4);
  m.sgrid = o; o = a16(o + 256 * roll_gbw(R) * 4);
  m.spq = o;   o = a16(o + 256 * N * 2);
  m.ssa = o;   o = a16(o + 2 * 256 * 2);
  m.sdone = o; o = a16(o + 2 * 256);
  m.shx = o;   o = a16(o + N * 32 * 4);   // (exact body: the outgoing actions, 256 B; every block: the step's hand-off words)
  m.total = o;
  return m;
}

// per-launch constants of a chunk-kernel block (computed once, read by the step loop)
struct ChunkCtx {
  float* stab;
  uint32_t* sgrid;
  uint16_t* spq;      // [256][N] position words prev_r << 12 | prev_c << 8 | r << 4 | c
  uint16_t* ssa;      // [2][256] steps, apples of the env
  uint8_t* sdone;     // [2][256] dones by step parity
  uint8_t* shx;       // [256] the exact-body behavior block's outgoing actions; at the loop top [N][32] u32 hand-off words
  uint64_t ctr0, seq;
  float eps;
  int tile, agent, e0;
  bool second, writer;
};

// The n steps of a chunk-kernel block; EXACT: the range-guarded agent's exact-f32 body (8 waves x 32 envs), else the
// fp16x3 body (16 waves x 16 envs). One instantiation per body keeps each loop's live registers those of one body.
template <int F1, int G, int H, int AB>
__device__ __forceinline__ ChunkCtx chunk_ctx(const QFwdParams* kargs) {
  const RollChunk& rc = *reinterpret_cast<const RollChunk*>(kargs + 2);
  const int nb = (int)gridDim.x, b = (int)blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;   // a tile's 2N blocks: b, b + 8, ... (one XCD)
  const int N = kargs[0].N;
  ChunkCtx cx;
  cx.tile = lb / (2 * N);
  const int role = lb % (2 * N);
  cx.second = role >= N;                          // false: target net on s'_t, true: behavior on s_{t+1}
  cx.agent = cx.second ? role - N : role;
  cx.writer = !cx.second && cx.agent == 0;
  cx.e0 = cx.tile * 256;
  const RollChunkLds lay = roll_chunk_lds(rc.env.R, rc.env.C, N);
  char* envl = reinterpret_cast<char*>(wsm_ptr()) + rc.lds_env;
  cx.stab = reinterpret_cast<float*>(envl + lay.stab);
  cx.sgrid = reinterpret_cast<uint32_t*>(envl + lay.sgrid);
  cx.spq = reinterpret_cast<uint16_t*>(envl + lay.spq);
  cx.ssa = reinterpret_cast<uint16_t*>(envl + lay.ssa);
  cx.sdone = reinterpret_cast<uint8_t*>(envl + lay.sdone);
  cx.shx = reinterpret_cast<uint8_t*>(envl + lay.shx);
  // (the last block rewrites these only after every block has finished: constant for the launch)
  cx.ctr0 = *rc.counter;
  cx.seq = *rc.seq;
  cx.eps = cx.second ? *kargs[1].io.eps_ptr : 0.0f;
  return cx;
}

// timing stamp k of step i of waves 0 and 15 (lane 0; MM_ROLL_DEBUG builds only)
#if MM_ROLL_DEBUG
#define MM_CSTAMP(k)                                                                                          \
  do {                                                                                                        \
    if (rc.trace && lane == 0 && i < 16 && (wave == 0 || wave == 15)) {                                       \
      const int lbk = cx.tile * 2 * N + (second ? N : 0) + agent;                                             \
      rc.trace[(((int64_t)lbk * 2 + (wave ? 1 : 0)) * 16 + i) * 4 + (k)] = __builtin_amdgcn_s_memrealtime();  \
    }                                                                                                         \
  } while (0)
#else
#define MM_CSTAMP(k) \
  do {               \
  } while (0)
#endif

template <int F1, int G, int H, int AB, bool EXACT>
__device__ __forceinline__ void roll_chunk_steps() {
  const QFwdParams* kargs0 = (const QFwdParams*)__builtin_amdgcn_kernarg_segment_ptr();
  const int nsteps = reinterpret_cast<const RollChunk*>(kargs0 + 2)->n;
  // fp16x3 body: each lane's hidden state stays in registers from one step to the next (the same lane owns the same
  // (env, agent, features) every step); read from h_in at the launch's first step, written to h_out at its last
  f32x4 hkeep[H / 16];
#pragma unroll
  for (int t = 0; t < H / 16; ++t) hkeep[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // behavior lanes: the (env, agent) part of the eps-greedy draws (rng_inner) is the same every step
  uint64_t rin = 0;
  if (!EXACT) {
    const ChunkCtx c0x = chunk_ctx<F1, G, H, AB>(kargs0);
    const int l0 = (int)threadIdx.x & 63;
    const int e_r = c0x.e0 + ((int)threadIdx.x >> 6) * 16 + (l0 & 15);
    rin = rng_inner((uint64_t)e_r, ((l0 >> 4) & 1) ? (uint64_t)c0x.agent : 0xFFFFFFFFull);
  }
  for (int i = 0; i < nsteps; ++i) {
  // every per-launch constant is re-derived from the kernarg segment in each step (scalar loads, K$ hits) through
  // a pointer the compiler cannot prove invariant, and every lane index from a thread id it cannot hoist: nothing
  // stays live across the step's forward body (the body's registers are those of rollout_step_kernel's)
  // (the opaque offset is added in the kernarg address space, so the parameter reads stay scalar loads: a laundered
  // generic pointer would turn every one of them into a vector flat load)
  int tz = 0;
  asm volatile("" : "+s"(tz));
  const QFwdParams* kargs =
      (const QFwdParams*)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() + tz);
  (void)kargs0;
  const int tx = (int)threadIdx.x + tz;
  const int wave = tx >> 6, lane = tx & 63;
  const ChunkCtx cx = chunk_ctx<F1, G, H, AB>(kargs);
  const QFwdParams& p = kargs[cx.second ? 1 : 0];
  const RollChunk& rc = *reinterpret_cast<const RollChunk*>(kargs + 2);
  const int CL = rc.CL;   // chunk length (C below is the env grid's column count)
  const EnvDev& ev = rc.env;
  const int N = p.N, D = p.D, R = ev.R, C = ev.C, E = p.E;
  const int64_t EN = (int64_t)E * N, nd = (int64_t)N * D;
  const mm_qfwd_io& io = p.io;
  const int tile = cx.tile, agent = cx.agent, e0 = cx.e0;
  const bool second = cx.second, writer = cx.writer;
  const int le_d = tx, de = e0 + le_d;
  const bool dvalid = tx < 256 && de < E;
  uint32_t* rows = cx.sgrid + le_d * roll_gbw(R);
  const int le = wave * 16 + (lane & 15), e = e0 + le;           // fp16x3 body / begin-store lane mapping
  const int l32 = wave * 32 + (lane & 31), e32 = e0 + l32;       // exact body lane mapping (waves 0-7)
    // chunk position c of launch step i, the chunk's staging set (a launch may cross chunk boundaries: its k-th chunk
    // writes staging set (set0 + k) % S), ring position of the step (rings of RL steps hold rewards / dones / max Q' /
    // actions / Q(a) by step)
    int c = rc.c0 + i, kset = rc.set0;
    while (c >= CL) {
      c -= CL;
      kset = kset + 1 == rc.S ? 0 : kset + 1;
    }
    const int64_t* stg = rc.staging + (int64_t)kset * E;
    const int pos = rc.pos0 + i >= rc.RL ? rc.pos0 + i - rc.RL : rc.pos0 + i;
    const int posn = pos + 1 == rc.RL ? 0 : pos + 1;
    const uint64_t ctr = cx.ctr0 + (uint64_t)i;
    const int cur = i & 1, prv = cur ^ 1;
    MM_CSTAMP(0);
    // (1) the actions of step t (i > 0: published by the tile's N behavior blocks at the end of their step t - 1)
    uint32_t aq[2] = {0u, 0u};   // 4-bit actions, agent k at bits 4 (k & 7) of aq[k >> 3]
    if (i > 0) {
      __syncthreads();   // every wave is past its reads of the LDS env state of step i - 1
      if (wave == 0) {
        // the tile's N x 32 hand-off words of step i, polled by wave 0 until each carries this launch's tag (tag and
        // actions are one 64-bit word: a word that matches holds this step's actions, no flag / fence needed), their
        // action halves into LDS
        const uint64_t* hs = rc.hx + ((int64_t)tile * rc.hxl + i) * N * 32;
        uint32_t* hl = reinterpret_cast<uint32_t*>(cx.shx);
        const uint32_t tag = (uint32_t)cx.seq + 1u;
        const int nw = N * 32;
        uint32_t got = 0u;   // bit q: word q * 64 + lane received (or outside the N x 32 words)
#pragma unroll
        for (int q = 0; q < (kRollMaxN * 32 + 63) / 64; ++q)
          if (q * 64 + lane >= nw) got |= 1u << q;
        const uint32_t need = (1u << ((kRollMaxN * 32 + 63) / 64)) - 1u;
        const uint64_t tw = __builtin_amdgcn_s_memrealtime();
        while (true) {
          uint64_t w[(kRollMaxN * 32 + 63) / 64];
#pragma unroll
          for (int q = 0; q < (kRollMaxN * 32 + 63) / 64; ++q)
            if (!((got >> q) & 1u)) w[q] = __hip_atomic_load(hs + q * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int q = 0; q < (kRollMaxN * 32 + 63) / 64; ++q)
            if (!((got >> q) & 1u) && (uint32_t)(w[q] >> 32) == tag) {
              hl[q * 64 + lane] = (uint32_t)w[q];
              got |= 1u << q;
            }
          if (__all(got == need)) break;
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - tw > kHandoffTimeout) {
            if (lane == 0) atomicOr(rc.err, 2u);
            break;
          }
        }
      }
      __syncthreads();
      MM_CSTAMP(1);
      if (dvalid) {
        const uint32_t* hl = reinterpret_cast<const uint32_t*>(cx.shx) + (le_d >> 3);
        const uint32_t sh = 4u * (uint32_t)(le_d & 7);
#pragma unroll
        for (int k = 0; k < kRollMaxN; ++k)
          if (k < N) aq[k >> 3] |= ((hl[k * 32] >> sh) & 15u) << (4 * (k & 7));
        // (2) auto-reset of an env that ended at step t - 1 (the initial grid / positions / counters)
        if (cx.sdone[prv * 256 + le_d]) {
          const uint4* ig = reinterpret_cast<const uint4*>(ev.init_grid);
#pragma unroll
          for (int j = 0; j < kRollMaxR / 2; ++j)
            if (2 * j < R) {
              const uint4 g = ig[j];
              rows[2 * j] = nib_pack4(g.x) | (nib_pack4(g.y) << 16);
              if (2 * j + 1 < R) rows[2 * j + 1] = nib_pack4(g.z) | (nib_pack4(g.w) << 16);
            }
          for (int k = 0; k < N; ++k) cx.spq[le_d * N + k] = (uint16_t)pos16(ev.init_pos[k]);
          cx.ssa[le_d] = 0;
          cx.ssa[256 + le_d] = (uint16_t)ev.init_apples;
        }
      }
    } else if (dvalid) {
      for (int k = 0; k < N; ++k) aq[k >> 3] |= (uint32_t)(rc.act0[(int64_t)de * N + k] & 15) << (4 * (k & 7));
    }
    // the store rows of the target's obs stores (re-read per step: not live across the body); out of range -> -1
    int64_t srow = -1;
    if (!second) {
      const int el = EXACT ? e32 : e;
      if ((EXACT ? (wave < 8) : true) && el < E) {
        srow = stg[el];
        if (srow < 0 || srow >= rc.n_rows) srow = -1;   // (flagged once per launch by the prologue)
      }
    }
    // (3) chunk start: slot 0 of the staging rows <- s_t (lane (env, g) writes features 16 q + 4 g .. + 3)
    if (c == 0) {
      __syncthreads();
      if (!second && e < E) {
        const int64_t srb = stg[e];
        if (srb >= 0 && srb < rc.n_rows) {
          const int rcw = cx.spq[le * N + agent] & 0xFF;
          const uint64_t wd = roll_obs_word(cx.sgrid + le * roll_gbw(R), R, rcw >> 4, rcw & 15);
          const float cr = cx.stab[rcw >> 4], cc = cx.stab[R + (rcw & 15)];
          float* d0 = rc.store_obs + srb * rc.row_stride + (int64_t)agent * D;
          for (int f0 = 4 * (lane >> 4); f0 < D; f0 += 16) {
            float x[4];
            roll_feat4(wd, f0, cr, cc, x);
            roll_store4(d0, f0, D, x);
          }
        }
      }
      __syncthreads();
    }
    // (4) the env dynamics of step t (rollout_step_kernel's loop; positions / counters from LDS)
    if (dvalid) {
      int64_t myrow = -1;
      if (writer) {
        myrow = stg[de];
        if (myrow < 0 || myrow >= rc.n_rows) myrow = -1;   // never handed on as cur_row
      }
      uint32_t pq[kRollMaxN / 2];
#pragma unroll
      for (int j = 0; j < kRollMaxN / 2; ++j) pq[j] = 0u;
#pragma unroll
      for (int k = 0; k < kRollMaxN; ++k)
        if (k < N) pq[k >> 1] |= (uint32_t)cx.spq[le_d * N + k] << (16 * (k & 1));
      const int st = (int)cx.ssa[le_d] + 1;
      int apples = cx.ssa[256 + le_d];
      float* rout = rc.rew + (int64_t)pos * EN + (int64_t)de * N;
      // (unrolled over the compile-time agent bound: each agent's own target cell is independent of the others, so
      // the compiler can compute it ahead of the previous agent's LDS round trip; only the grid rows chain them)
#pragma unroll
      for (int k = 0; k < kRollMaxN; ++k) {
        if (k < N) {
        const uint32_t w = pq[0] & 0xFFFFu;
        const int a = (int)(aq[0] & 15u);
#pragma unroll
        for (int j = 0; j < kRollMaxN / 2 - 1; ++j) pq[j] = __builtin_amdgcn_alignbit(pq[j + 1], pq[j], 16);
        pq[kRollMaxN / 2 - 1] >>= 16;
        aq[0] = __builtin_amdgcn_alignbit(aq[1], aq[0], 4);
        aq[1] >>= 4;
        int r = (w >> 4) & 15, cc = w & 15, pr = (w >> 12) & 15, pc = (w >> 8) & 15;
        const int nr = r + (a == 0 ? 1 : (a == 2 ? -1 : 0));
        const int nc = cc + (a == 1 ? -1 : (a == 3 ? 1 : 0));
        const bool inside = a != 4 && nr >= 0 && nr < R && nc >= 0 && nc < C;
        const uint32_t w_n = rows[inside ? nr : r], w_r = rows[r], w_p = rows[pr];
        asm volatile("" ::"v"(w_n), "v"(w_r), "v"(w_p));
        const bool moved = inside && ((w_n >> (4 * nc)) & 15u) < 3u;
        if (moved) {
          pr = r;
          pc = cc;
          r = nr;
          cc = nc;
        }
        const bool upd = r != pr || cc != pc;
        const uint32_t A = moved ? w_n : w_r;
        const uint32_t B = moved ? w_r : w_p;
        const uint32_t item = upd ? (A >> (4 * cc)) & 15u : 0u;
        const bool big = (k & 1) == 0;
        const float mag = big ? 10.0f : 1.0f;   // (selects, no branch: item 1 lemon -mag, 2 apple +mag)
        const float rk = ev.step_cost + (item == 2u ? mag : (item == 1u ? -mag : 0.0f));
        apples -= item == 2u ? 1 : 0;
        const uint32_t clr = upd ? ~(15u << (4 * pc)) : ~0u;
        const uint32_t A1 = pr == r ? (A & clr) : A;
        rows[pr] = B & clr;
        rows[r] = upd ? ((A1 & ~(15u << (4 * cc))) | ((uint32_t)(3 + k) << (4 * cc))) : A1;
        cx.spq[le_d * N + k] = (uint16_t)((pr << 12) | (pc << 8) | (r << 4) | cc);
        if (writer) rout[k] = rk;
        }
      }
      const bool dn = st >= ev.max_steps || apples == 0;
      cx.ssa[le_d] = (uint16_t)st;
      cx.ssa[256 + le_d] = (uint16_t)apples;
      cx.sdone[cur * 256 + le_d] = dn ? 1 : 0;
      if (writer) {
        rc.done[(int64_t)pos * E + de] = dn ? 1 : 0;
        rc.cur_row[de] = dn ? -1 : myrow;
      }
    }
    __syncthreads();
    MM_CSTAMP(2);
    // (5) the forward: target on s'_t (max Q'_t, s'_t stored into slot c + 1), behavior on s_{t+1} (act / Q(a))
    const int64_t off = (int64_t)(second ? posn : pos) * EN;
    const int64_t nxt_off = (int64_t)(c + 1) * nd;
    if constexpr (EXACT) {
      const int hh = lane >> 5;
      if (wave < 8) {
        const bool ok32 = e32 < E;
        const bool r32 = !second && ok32 && cx.sdone[prv * 256 + l32];
        const bool bd = second && ok32 && cx.sdone[cur * 256 + l32];
        float* dst = (!second && srow >= 0) ? rc.store_obs + srow * rc.row_stride + nxt_off + (int64_t)agent * D : nullptr;
        const int ls = ok32 ? l32 : 0;
        const int rc32 = cx.spq[ls * N + agent] & 0xFF;
        const uint64_t wd32 = roll_obs_word(cx.sgrid + ls * roll_gbw(R), R, rc32 >> 4, rc32 & 15);
        const float cr32 = cx.stab[rc32 >> 4], cc32 = cx.stab[R + (rc32 & 15)];
        auto ol32 = [&](int kb, float (&x)[16]) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int f0 = kb * 32 + 8 * q + 4 * hh;
            roll_feat4(wd32, f0, cr32, cc32, x + 4 * q);
            if (bd || !ok32)
#pragma unroll
              for (int j = 0; j < 4; ++j) x[4 * q + j] = (ok32 && f0 + j < D) ? ev.reset_obs[agent * D + f0 + j] : 0.0f;
            if (dst) roll_store4(dst, f0, D, x + 4 * q);
          }
        };
        float x32[16];
        ol32(0, x32);
        const int a = agent_q_fwd_body<F1, G, H, AB>(p, agent, ok32 ? e32 : E, wsm_ptr() + tz, ol32, x32,
                                                     !ok32 || r32 || bd, true, cx.eps, ctr, off);
        if (second && hh == 0 && ok32) cx.shx[l32] = (uint8_t)a;
      }
    } else {
      const int ec = min(e, E - 1);
      const int g = lane >> 4;
      f32x4 h0[H / 16];
      if (i == 0) {
        const float* hp = io.h_in + (int64_t)ec * io.hin_se + (int64_t)agent * io.hin_sa + (int64_t)(4 * g) * io.hin_sf;
#pragma unroll
        for (int t = 0; t < H / 16; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) h0[t][r] = hp[(int64_t)(16 * t + r) * io.hin_sf];
      } else {
#pragma unroll
        for (int t = 0; t < H / 16; ++t) h0[t] = hkeep[t];
      }
      const bool rt = !second && e < E && cx.sdone[prv * 256 + le];
      const bool bd = second && e < E && cx.sdone[cur * 256 + le];
      if (e >= E || rt || bd) {
#pragma unroll
        for (int t = 0; t < H / 16; ++t) h0[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      float* dst = (!second && srow >= 0) ? rc.store_obs + srow * rc.row_stride + nxt_off + (int64_t)agent * D : nullptr;
      const int ls = e < E ? le : 0;
      const int rcw = cx.spq[ls * N + agent] & 0xFF;
      const uint64_t wd = roll_obs_word_g(cx.sgrid + ls * roll_gbw(R), R, rcw >> 4, rcw & 15, g);
      const float cr = cx.stab[rcw >> 4], cc = cx.stab[R + (rcw & 15)];
      auto ol = [&](int kb, float (&x)[8]) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int f0 = kb * 32 + 16 * q + 4 * g;
          roll_feat4(wd, f0, cr, cc, x + 4 * q);
          if (bd || e >= E)
#pragma unroll
            for (int j = 0; j < 4; ++j) x[4 * q + j] = (e < E && f0 + j < D) ? ev.reset_obs[agent * D + f0 + j] : 0.0f;
          if (dst) roll_store4(dst, f0, D, x + 4 * q);
        }
      };
      float xn[8];
      ol(0, xn);
      if (wave >= 8)
        for (int s = 0; s < p.stagger; ++s) __builtin_amdgcn_s_sleep(8);
      // (the image base offset by the per-step opaque zero: the fragment addresses are formed inside the step,
      // not hoisted out of the loop into registers that then spill)
      const int a = agent_q_fwd_body_h3<F1, G, H, AB>(p, agent, e, wsm_ptr() + tz, ol, xn, h0, cx.eps, ctr, off, 1,
                                                      &hkeep, i + 1 == nsteps, &rin);
      // behavior blocks: each wave publishes its 16 envs' actions of step t + 1 as soon as its forward is done (every
      // lane (c, g) holds env c's action): lanes 0-7 / 8-15 OR their nibbles into the two hand-off words of the wave
      if (second && i + 1 < rc.n) {
        uint32_t v = ((uint32_t)a & 15u) << (4 * (lane & 7));
        v |= __shfl_xor(v, 1);
        v |= __shfl_xor(v, 2);
        v |= __shfl_xor(v, 4);
        if (lane == 0 || lane == 8) {
          uint64_t* hd = rc.hx + (((int64_t)tile * rc.hxl + i + 1) * N + agent) * 32 + wave * 2 + (lane >> 3);
          __hip_atomic_store(hd, ((uint64_t)((uint32_t)cx.seq + 1u) << 32) | v, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    MM_CSTAMP(3);
    // exact-f32 body (8 waves x 32 envs): the actions gathered in LDS, then wave 0 publishes the 32 words
    if (EXACT && second && i + 1 < rc.n) {
      __syncthreads();
      if (wave == 0 && lane < 32) {
        const uint2 b = reinterpret_cast<const uint2*>(cx.shx)[lane];   // envs 8 lane .. 8 lane + 7
        uint64_t* hd = rc.hx + (((int64_t)tile * rc.hxl + i + 1) * N + agent) * 32 + lane;
        __hip_atomic_store(hd, ((uint64_t)((uint32_t)cx.seq + 1u) << 32) | nib_pack4(b.x) | (nib_pack4(b.y) << 16),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

template <int F1, int G, int H, int AB>
__global__ __launch_bounds__(1024, 1) void rollout_chunk_kernel(QFwdParams p0, QFwdParams p1, RollChunk rc_) {
  float* wsm = wsm_ptr();
  const QFwdParams* kargs = (const QFwdParams*)__builtin_amdgcn_kernarg_segment_ptr();
  const RollChunk& rc = *reinterpret_cast<const RollChunk*>(kargs + 2);
  (void)p0;
  (void)p1;
  (void)rc_;
  const int N = kargs[0].N;
  const ChunkCtx cx = chunk_ctx<F1, G, H, AB>(kargs);
  const int nb = (int)gridDim.x;
  const QFwdParams& p = kargs[cx.second ? 1 : 0];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const EnvDev& ev = rc.env;
  const int R = ev.R, C = ev.C, RC = R * C, E = p.E;
  const int agent = cx.agent, e0 = cx.e0;
  const bool exact = reinterpret_cast<const int*>(p.packed + 2 * p.g.agent_stride * N)[agent] != 0;
  const int par = *rc.envpar;

  // ---- once per launch: the weight image (the exact-f32 one for a range-guarded agent) into LDS
  {
    const float* src = p.packed + (exact ? 0 : (int64_t)N * p.g.agent_stride) + (int64_t)agent * p.g.agent_stride;
    const int nchunk = (int)(p.g.agent_stride >> 8);
    for (int c = wave; c < nchunk; c += 16)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c * 256 + lane * 4),
                                       (__attribute__((address_space(3))) void*)(wsm + c * 256), 16, 0, 0);
  }
  if (threadIdx.x >= 256 && threadIdx.x < 256 + R + C) {
    const int i = threadIdx.x - 256;
    cx.stab[i] = i < R ? ev.rtab[i] : ev.ctab[i - R];
  }
  // ---- the tile's env state into LDS (one lane per env); staging rows checked once (sticky bit 0)
  const int le_d = threadIdx.x, de = e0 + le_d;
  const bool dvalid = threadIdx.x < 256 && de < E;
  if (dvalid) {
    const int32_t* pw = (par ? ev.pos_alt : ev.pos) + (int64_t)de * N;
    const uint4* gin = reinterpret_cast<const uint4*>((par ? ev.grid_alt : ev.grid) + (int64_t)de * RC);
    uint32_t* rows = cx.sgrid + le_d * roll_gbw(R);
    cx.ssa[le_d] = (uint16_t)(par ? ev.steps_alt : ev.steps)[de];
    cx.ssa[256 + le_d] = (uint16_t)(par ? ev.apples_alt : ev.apples)[de];
    for (int k = 0; k < N; ++k) cx.spq[le_d * N + k] = (uint16_t)pos16(pw[k]);
#pragma unroll
    for (int j = 0; j < kRollMaxR / 2; ++j)
      if (2 * j < R) {
        const uint4 g = gin[j];
        rows[2 * j] = nib_pack4(g.x) | (nib_pack4(g.y) << 16);
        if (2 * j + 1 < R) rows[2 * j + 1] = nib_pack4(g.z) | (nib_pack4(g.w) << 16);
      }
    cx.sdone[256 + le_d] = rc.done_prev[de];   // "previous step" slot of step 0 (parity 1)
    if (cx.writer) {   // every staging set the launch writes
      int ks = rc.set0;
      for (int k = 0; k < rc.S && k * rc.CL < rc.c0 + rc.n; ++k) {
        roll_row_ok(rc.staging[(int64_t)ks * E + de], rc.n_rows, rc.err);
        ks = ks + 1 == rc.S ? 0 : ks + 1;
      }
    }
  } else if (threadIdx.x < 256) {
    cx.sdone[256 + le_d] = 0;
  }
  __syncthreads();

  // (two loops, one per body: the exact-f32 loop's spills stay in that rare path — the fp16x3 loop's spill code is
  // the same as with no exact path at all, checked in the ISA)
#if MM_ROLL_DEBUG
  // in-kernel clock (MI355X_MICROARCH.md DVFS check 6): shader-clock and 100 MHz stamps around the step loop of
  // every block, trace[60000 + 4 b ..] (tools/chunk_trace.py: delta memtime / delta memrealtime x 100 MHz)
  uint64_t* clk = (rc.trace && threadIdx.x == 0) ? rc.trace + 60000 + 4 * (int)blockIdx.x : nullptr;
  if (clk) {
    clk[0] = __builtin_amdgcn_s_memtime();
    clk[1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  if (exact)
    roll_chunk_steps<F1, G, H, AB, true>();
  else
    roll_chunk_steps<F1, G, H, AB, false>();
#if MM_ROLL_DEBUG
  if (clk) {
    clk[2] = __builtin_amdgcn_s_memtime();
    clk[3] = __builtin_amdgcn_s_memrealtime();
  }
#endif

  // ---- the tile's final env state into buffer 1 - par (reset where the last step ended), by the writer block
  const int lastp = (rc.n - 1) & 1;
  if (cx.writer && dvalid) {
    const bool dn = cx.sdone[lastp * 256 + le_d] != 0;
    int32_t* pout = (par ? ev.pos : ev.pos_alt) + (int64_t)de * N;
    for (int k = 0; k < N; ++k) {
      const uint32_t w = cx.spq[le_d * N + k];
      pout[k] = dn ? ev.init_pos[k]
                   : (int32_t)((((w >> 12) & 15) << 24) | (((w >> 8) & 15) << 16) | (((w >> 4) & 15) << 8) | (w & 15));
    }
    (par ? ev.steps : ev.steps_alt)[de] = dn ? 0 : (int32_t)cx.ssa[le_d];
    (par ? ev.apples : ev.apples_alt)[de] = dn ? ev.init_apples : (int32_t)cx.ssa[256 + le_d];
    uint4* gout = reinterpret_cast<uint4*>((par ? ev.grid : ev.grid_alt) + (int64_t)de * RC);
    const uint4* ig = reinterpret_cast<const uint4*>(ev.init_grid);
    const uint32_t* rows = cx.sgrid + le_d * roll_gbw(R);
#pragma unroll
    for (int j = 0; j < kRollMaxR / 2; ++j)
      if (2 * j < R) {
        uint4 v;
        if (dn) {
          v = ig[j];
        } else {
          const uint32_t a0 = rows[2 * j], a1 = 2 * j + 1 < R ? rows[2 * j + 1] : 0u;
          v = make_uint4(nib_unpack4(a0 & 0xFFFFu), nib_unpack4(a0 >> 16), nib_unpack4(a1 & 0xFFFFu),
                         nib_unpack4(a1 >> 16));
        }
        gout[j] = v;
      }
  }
  // ---- the last block to finish advances the launch state (every block has read it by then)
  __syncthreads();
  if (threadIdx.x == 0) {
    if (atomicAdd(rc.ticket, 1u) == (uint32_t)nb - 1) {
      *rc.counter = cx.ctr0 + (uint64_t)rc.n;
      *rc.envpar = 1 - par;
      *rc.seq = cx.seq + 1;
      *rc.ticket = 0u;
    }
  }
}

// ---------------------------------------------------------------- learner PRE on the fp16x3 image
// The learner's non-recurrent part (layers 1-2 with their training saves, and gi = W_ih x2 + b_ih) of large
// batches in the fast (cfg5) mode, QLearner(mixer_fp16=True): agent_q_fwd_body_h3's layers 1-2 and its
// W_ih gate products (fp16x3 split, fp32 accumulate: ~2^-22 relative per product, the forward's rtol 1e-5
// parity) instead of agent_pre_body's exact-f32 MFMAs, at ~5x less MFMA time per product. Same outputs /
// layouts as agent_pre_body: saves [x1 | x2] by feature, gi [r | z | n] by feature.
template <int F1, int G, int H, int AB>
__device__ __forceinline__ void agent_pre_body_h3(const QFwdParams& p, int agent, int e, const float* __restrict__ W,
                                                  const float* orow) {
  using CG = QnetCGeo<F1, G, H, AB>;
  constexpr int T1 = F1 / 16, T2 = G / 16, TH = H / 16;
  constexpr int RB1 = F1 / 32, RB2 = G / 32, HB = H / 32;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const bool valid = e < p.E;
  const mm_qfwd_io& io = p.io;
  // obs k-steps as 16-byte loads where the row is 16-byte aligned (the cfg5 store rows of D = 300 are): lane
  // (c, g) reads features 32 kb + 16 q + 4 g + 0..3 for q = 0, 1 — 2 loads instead of 8 guarded dword loads
  const bool o16 = orow && (reinterpret_cast<uintptr_t>(orow) & 15) == 0;
  auto ld_obs = [&](int kb, float (&x)[8]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int k0 = kb * 32 + 16 * q + 4 * g;
      if (o16 && k0 + 3 < p.D) {
        const float4 v = *reinterpret_cast<const float4*>(orow + k0);
        x[4 * q] = v.x;
        x[4 * q + 1] = v.y;
        x[4 * q + 2] = v.z;
        x[4 * q + 3] = v.w;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) x[4 * q + r] = (orow && k0 + r < p.D) ? orow[k0 + r] : 0.0f;
      }
    }
  };
  float xn[8];
  ld_obs(0, xn);
  // ---- layer 1 (next obs k-step prefetched)
  f32x4 x1[T1];
#pragma unroll
  for (int t = 0; t < T1; ++t) x1[t] = bias4(W + CG::off_b1, t, g);
  for (int kb = 0; kb < p.g.KD; ++kb) {
    KS ob;
    split8(xn, ob);
    if (kb + 1 < p.g.KD) ld_obs(kb + 1, xn);
#pragma unroll
    for (int t = 0; t < T1; ++t) mm16(W + CG::off_l1 + (int64_t)((t >> 1) * p.g.KD + kb) * 1024, t & 1, ob, lane, x1[t]);
  }
  float* sv = (io.save && valid) ? io.save + ((int64_t)e * p.N + agent) * (F1 + G + 6 * H) : nullptr;
  KS x1s[RB1];
#pragma unroll
  for (int t = 0; t < T1; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) x1[t][r] = relu_bits(x1[t][r]);
    if (sv) *reinterpret_cast<f32x4*>(sv + 16 * t + 4 * g) = x1[t];
  }
#pragma unroll
  for (int kb = 0; kb < RB1; ++kb) split_pair(x1[2 * kb], x1[2 * kb + 1], x1s[kb]);
  // ---- layer 2
  f32x4 x2[T2];
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    x2[t] = bias4(W + CG::off_b2, t, g);
#pragma unroll
    for (int kb = 0; kb < RB1; ++kb) mm16(W + CG::off_l2 + ((t >> 1) * RB1 + kb) * 1024, t & 1, x1s[kb], lane, x2[t]);
#pragma unroll
    for (int r = 0; r < 4; ++r) x2[t][r] = relu_bits(x2[t][r]);
    if (sv) *reinterpret_cast<f32x4*>(sv + F1 + 16 * t + 4 * g) = x2[t];
  }
  KS x2s[RB2];
#pragma unroll
  for (int kb = 0; kb < RB2; ++kb) split_pair(x2[2 * kb], x2[2 * kb + 1], x2s[kb]);
  // ---- gi = W_ih x2 + b_ih (gates r, z, n), three gates' fragments per k-step interleaved
  float* gi = valid ? io.gi + ((int64_t)e * p.N + agent) * 3 * H : nullptr;
#pragma unroll
  for (int t = 0; t < TH; ++t) {
    const int rb = t >> 1, q = t & 1;
    f32x4 ar = bias4(W + CG::off_brz, t, g);
    f32x4 az = bias4(W + CG::off_brz + H, t, g);
    f32x4 an = bias4(W + CG::off_bin, t, g);
#pragma unroll
    for (int kb = 0; kb < RB2; ++kb) {
      const int base = CG::off_ih + (rb * RB2 + kb) * 1024, gs = HB * RB2 * 1024;
      const Frag f0 = ldfrag(W + base, q, lane);
      const Frag f1 = ldfrag(W + base + gs, q, lane);
      const Frag f2 = ldfrag(W + base + 2 * gs, q, lane);
      mmf(f0, x2s[kb], ar);
      mmf(f1, x2s[kb], az);
      mmf(f2, x2s[kb], an);
    }
    if (gi) {
      float* o = gi + 16 * t + 4 * g;
      *reinterpret_cast<f32x4*>(o) = ar;
      *reinterpret_cast<f32x4*>(o + H) = az;
      *reinterpret_cast<f32x4*>(o + 2 * H) = an;
    }
  }
}

// 1024-thread block = 16 waves x 16 rows of one agent (the dual forward's geometry); an agent flagged by
// the pack-time range guard runs its 256 rows on the exact-f32 image (agent_pre_body, 8 waves x 32 rows).
template <int F1, int G, int H, int AB>
__global__ __launch_bounds__(1024, 1) void agent_pre_h3_kernel(QFwdParams p0, QFwdParams p1) {
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  const bool second = (int)blockIdx.x >= p0.nblocks;
  const QFwdParams* kargs = (const QFwdParams*)__builtin_amdgcn_kernarg_segment_ptr();
  const QFwdParams& p = kargs[second ? 1 : 0];
  (void)p1;
  const int bid = second ? (int)blockIdx.x - p0.nblocks : (int)blockIdx.x;
  const int agent = bid % p.N, tile = bid / p.N;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool exact = reinterpret_cast<const int*>(p.packed + 2 * p.g.agent_stride * p.N)[agent] != 0;
  const float* src = p.packed + (exact ? 0 : (int64_t)p.N * p.g.agent_stride) + (int64_t)agent * p.g.agent_stride;
  const int nchunk = (int)(p.g.agent_stride >> 8);
  for (int c = wave; c < nchunk; c += 16)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c * 256 + lane * 4),
                                     (__attribute__((address_space(3))) void*)(wsm + c * 256), 16, 0, 0);
  __syncthreads();
  if (exact) {
    const int e32 = tile * 256 + wave * 32 + (lane & 31);
    if (wave < 8) agent_pre_body<F1, G, H, AB>(p, agent, e32, wsm, obs_row_ptr(p, agent, e32));
    return;
  }
  const int e = tile * 256 + wave * 16 + (lane & 15);
  agent_pre_body_h3<F1, G, H, AB>(p, agent, e, wsm, obs_row_ptr(p, agent, e));
}

// ---------------------------------------------------------------- learner PRE, weights in LDS
// Layers 1-2 and the GRU input projection of large learner batches: agent_pre_body (exact f32, one wave
// = 32 rows) with the agent's f32 fragment image staged ONCE per 1024-thread block by LDS-DMA and shared
// by its 16 waves (512 rows), instead of every wave streaming the ~100 KB of fragments (cfg5) from L2 per
// 32 rows. Same arithmetic as agent_split_kernel<.., 1>: bit-identical results.
template <int F1, int G, int H, int AB>
__global__ __launch_bounds__(1024, 1) void agent_pre_lds_kernel(QFwdParams p0, QFwdParams p1) {
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  const bool second = (int)blockIdx.x >= p0.nblocks;
  const QFwdParams* kargs = (const QFwdParams*)__builtin_amdgcn_kernarg_segment_ptr();
  const QFwdParams& p = kargs[second ? 1 : 0];
  (void)p1;
  const int bid = second ? (int)blockIdx.x - p0.nblocks : (int)blockIdx.x;
  const int agent = bid % p.N, tile = bid / p.N;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float* src = p.packed + (int64_t)agent * p.g.agent_stride;
  const int nchunk = (int)(p.g.agent_stride >> 8);
  for (int c = wave; c < nchunk; c += 16)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c * 256 + lane * 4),
                                     (__attribute__((address_space(3))) void*)(wsm + c * 256), 16, 0, 0);
  const int e = tile * 512 + wave * 32 + (lane & 31);
  const float* orow = obs_row_ptr(p, agent, e);
  __syncthreads();
  agent_pre_body<F1, G, H, AB>(p, agent, e, wsm, orow);
}

// ---------------------------------------------------------------- packing
// The canonical flat parameters behind f32 image element r of one agent (r < agent_stride): j0 (and, for the
// combined b_ih + b_hh rows of the r / z gates, j1) as indices into the flat parameters, bias = a bias image
// element (value j0 + j1, or j0 + 0.0f). j0 = -1: zero padding. Every parameter of the agent net appears in
// exactly one image element.
struct PackSrc {
  int64_t j0, j1;
  bool bias;
};
__device__ __forceinline__ PackSrc qnet_pack_src(const QnetGeo& g, int agent, int64_t r, int D, int F1, int G, int H,
                                                 int A, const QnetOffsets& o) {
  PackSrc ps{-1, -1, false};
  bool hit = false;
  // weight images: [rb][kb][q][lane][s & 3] (see load_frag)
  auto wimg = [&](int64_t off, int KB, int rows, int cols, int64_t src) {
    const int64_t sz = (int64_t)((rows + 31) / 32) * KB * 1024;
    if (r >= off && r < off + sz) {
      const int64_t t = r - off;
      const int lane = (int)((t >> 2) & 63), s = (int)(((t >> 8) & 3) * 4 + (t & 3));
      const int64_t blk = t >> 10;
      const int kb = (int)(blk % KB), rb = (int)(blk / KB);
      const int row = rb * 32 + (lane & 31), col = kb * 32 + kperm(s, lane >> 5);
      if (row < rows && col < cols) ps.j0 = src + (int64_t)row * cols + col;
      hit = true;
    }
  };
  // bias images: [rb][h][s] -> b[32 rb + kperm(s, h)]
  auto bimg = [&](int64_t off, int rows, int64_t src, int64_t src2) {
    const int64_t sz = (int64_t)((rows + 31) / 32) * 32;
    if (r >= off && r < off + sz) {
      const int64_t t = r - off;
      const int s = (int)(t & 15), h = (int)((t >> 4) & 1), rb = (int)(t >> 5);
      const int row = rb * 32 + kperm(s, h);
      if (row < rows) {
        ps.j0 = src + row;
        ps.j1 = src2 >= 0 ? src2 + row : -1;
        ps.bias = true;
      }
      hit = true;
    }
  };
  wimg(g.off_l1, g.KD, F1, D, o.W1 + (int64_t)agent * F1 * D);
  if (!hit) wimg(g.off_l2, F1 / 32, G, F1, o.W2 + (int64_t)agent * G * F1);
  if (!hit) wimg(g.off_ih, G / 32, 3 * H, G, o.Wih + (int64_t)agent * 3 * H * G);
  if (!hit) wimg(g.off_hh, H / 32, 3 * H, H, o.Whh + (int64_t)agent * 3 * H * H);
  if (!hit) wimg(g.off_q, H / 32, A, H, o.Wq + (int64_t)agent * A * H);
  if (!hit) bimg(g.off_b1, F1, o.b1 + (int64_t)agent * F1, -1);
  if (!hit) bimg(g.off_b2, G, o.b2 + (int64_t)agent * G, -1);
  if (!hit) bimg(g.off_brz, 2 * H, o.bih + (int64_t)agent * 3 * H, o.bhh + (int64_t)agent * 3 * H);
  if (!hit) bimg(g.off_bin, H, o.bih + (int64_t)agent * 3 * H + 2 * H, -1);
  if (!hit) bimg(g.off_bhn, H, o.bhh + (int64_t)agent * 3 * H + 2 * H, -1);
  if (!hit) bimg(g.off_bq, A, o.bq + (int64_t)agent * A, -1);
  return ps;
}
__device__ __forceinline__ float qnet_pack_value(const PackSrc& ps, float v0, float v1) {
  if (ps.j0 < 0) return 0.0f;
  return ps.bias ? v0 + (ps.j1 >= 0 ? v1 : 0.0f) : v0;
}

// One thread per packed element: gathers the canonical flat parameters into
// the per-lane MFMA fragment image (zero padding outside the real shape).
__device__ __forceinline__ void qnet_pack_body(const float* __restrict__ params, float* __restrict__ packed, QnetGeo g,
                                               int N, int D, int F1, int G, int H, int A, QnetOffsets o, int nblk) {
  const int64_t per_agent = g.agent_stride;
  const int64_t total = per_agent * N;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)nblk * blockDim.x) {
    const int agent = (int)(idx / per_agent);
    const PackSrc ps = qnet_pack_src(g, agent, idx % per_agent, D, F1, G, H, A, o);
    const float v0 = ps.j0 >= 0 ? params[ps.j0] : 0.0f;
    const float v1 = ps.j1 >= 0 ? params[ps.j1] : 0.0f;
    packed[idx] = qnet_pack_value(ps, v0, v1);
  }
}

// fp16x3 image (packed + N*agent_stride): weight blocks as [16-row half q][part][lane][8 halves]
// (see agent_q_fwd_body_h3); bias vectors in natural order.
__device__ __forceinline__ void qnet_pack_h3_body(const float* __restrict__ params, float* __restrict__ packed,
                                                  QnetGeo g, int N, int D, int F1, int G, int H, int A, QnetOffsets o,
                                                  int nblk) {
  const int64_t per_agent = g.agent_stride;
  const int64_t total = per_agent * N;
  uint32_t* out = reinterpret_cast<uint32_t*>(packed + total);
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)nblk * blockDim.x) {
    const int agent = (int)(idx / per_agent);
    const int64_t r = idx % per_agent;
    uint32_t v = 0u;
    bool hit = false;
    auto wimg = [&](int64_t off, int KB, int rows, int cols, int64_t src) {
      const int64_t sz = (int64_t)((rows + 31) / 32) * KB * 1024;
      if (!hit && r >= off && r < off + sz) {
        const int64_t t = r - off;
        const int blk = (int)(t >> 10), w = (int)(t & 1023);
        const int kb = blk % KB, rb = blk / KB;
        const int q = w >> 9, part = (w >> 8) & 1, lane = (w >> 2) & 63, dw = w & 3;
        const int row = rb * 32 + 16 * q + (lane & 15);
        uint32_t bits = 0u;
        for (int jj = 0; jj < 2; ++jj) {
          const int j = 2 * dw + jj;
          const int col = kb * 32 + kperm16(j, lane >> 4);
          const float x = (row < rows && col < cols) ? params[src + (int64_t)row * cols + col] : 0.0f;
          const _Float16 hv = (_Float16)x;
          const _Float16 pv = part == 0 ? hv : (_Float16)(x - (float)hv);
          bits |= (uint32_t)__builtin_bit_cast(uint16_t, pv) << (16 * jj);
        }
        v = bits;
        hit = true;
      }
    };
    auto bnat = [&](int64_t off, int rows, int64_t src, int64_t src2) {
      const int64_t sz = (int64_t)((rows + 31) / 32) * 32;
      if (!hit && r >= off && r < off + sz) {
        const int row = (int)(r - off);
        const float x = row < rows ? params[src + row] + (src2 >= 0 ? params[src2 + row] : 0.0f) : 0.0f;
        v = __float_as_uint(x);
        hit = true;
      }
    };
    wimg(g.off_l1, g.KD, F1, D, o.W1 + (int64_t)agent * F1 * D);
    wimg(g.off_l2, F1 / 32, G, F1, o.W2 + (int64_t)agent * G * F1);
    wimg(g.off_ih, G / 32, 3 * H, G, o.Wih + (int64_t)agent * 3 * H * G);
    wimg(g.off_hh, H / 32, 3 * H, H, o.Whh + (int64_t)agent * 3 * H * H);
    wimg(g.off_q, H / 32, A, H, o.Wq + (int64_t)agent * A * H);
    bnat(g.off_b1, F1, o.b1 + (int64_t)agent * F1, -1);
    bnat(g.off_b2, G, o.b2 + (int64_t)agent * G, -1);
    bnat(g.off_brz, 2 * H, o.bih + (int64_t)agent * 3 * H, o.bhh + (int64_t)agent * 3 * H);
    bnat(g.off_bin, H, o.bih + (int64_t)agent * 3 * H + 2 * H, -1);
    bnat(g.off_bhn, H, o.bhh + (int64_t)agent * 3 * H + 2 * H, -1);
    bnat(g.off_bq, A, o.bq + (int64_t)agent * A, -1);
    out[idx] = v;
  }
}

// Range guard of the fp16x3 forward, decided once per pack: a split operand must stay below 65504 in
// magnitude (the largest finite f16). With |obs| <= kH3ObsBound and the GRU state |h| <= 1, the
// layer outputs are bounded by m1 = max_r sum_k |W1[r,k]| kH3ObsBound + |b1[r]| and
// m2 = max_r sum_k |W2[r,k]| m1 + |b2[r]|, and every weight is split as well. Agent a whose bounds
// or largest weight reach kH3Limit gets flag[a] = 1 (tail of the packed buffer), and the fp16x3
// kernel runs that agent's blocks on the exact-f32 image instead: a per-block branch, no per-value
// check in the hot path.
constexpr float kH3ObsBound = 1.0f, kH3Limit = 32768.0f;
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// max_r (|b[r]| + scale * sum_k |W[r][k]|) over rows r of W [rows][cols]: one wave per row, lanes over k
// (coalesced, every row's loads independent), 4 rows in flight per wave
__device__ __forceinline__ float row_abs_bound(const float* __restrict__ W, const float* __restrict__ b, int rows,
                                               int cols, float scale) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  float m = 0.f;
#pragma unroll 4
  for (int r = w; r < rows; r += nw) {
    float acc = 0.f;
    for (int k = lane; k < cols; k += 64) acc += fabsf(W[(int64_t)r * cols + k]);
    acc = fabsf(b[r]) + wave_sum(acc) * scale;
    m = fmaxf(m, acc);
  }
  return m;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
// block max (any blockDim <= 1024): wave maxima through LDS, then one wave reduces them
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float m = lane < nw ? red[lane] : 0.f;
  return wave_max(m);
}
// max |p[i]| over i < n with 8 independent loads per thread in flight (addresses clamped, so every
// load is unconditional and the compiler issues them back to back: the scan costs ~n / (8 blockDim)
// memory round trips instead of n / (4 blockDim))
__device__ __forceinline__ float abs_max_scan(const float* __restrict__ p, int64_t n, float m) {
  const int64_t bd = blockDim.x;
  for (int64_t i = threadIdx.x; i < n; i += 8 * bd) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p[min(i + j * bd, n - 1)];
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
  }
  return m;
}
__device__ void qnet_h3_bound_block(const float* __restrict__ params, int* flags, int agent, int D, int F1, int G,
                                    int H, int A, QnetOffsets o) {
  __shared__ float red[16];
  // largest |weight| of the agent (every weight matrix is split)
  float wmax = 0.f;
  wmax = abs_max_scan(params + o.W1 + (int64_t)agent * F1 * D, (int64_t)F1 * D, wmax);
  wmax = abs_max_scan(params + o.W2 + (int64_t)agent * G * F1, (int64_t)G * F1, wmax);
  wmax = abs_max_scan(params + o.Wih + (int64_t)agent * 3 * H * G, (int64_t)3 * H * G, wmax);
  wmax = abs_max_scan(params + o.Whh + (int64_t)agent * 3 * H * H, (int64_t)3 * H * H, wmax);
  wmax = abs_max_scan(params + o.Wq + (int64_t)agent * A * H, (int64_t)A * H, wmax);
  // layer-1 output bound, then layer 2 scaled by it
  const float m1 = block_max(row_abs_bound(params + o.W1 + (int64_t)agent * F1 * D, params + o.b1 + (int64_t)agent * F1,
                                           F1, D, kH3ObsBound), red);
  const float m2 = row_abs_bound(params + o.W2 + (int64_t)agent * G * F1, params + o.b2 + (int64_t)agent * G, G, F1, m1);
  const float m = block_max(fmaxf(fmaxf(m2, wmax), m1), red);
  if (threadIdx.x == 0) flags[agent] = !(m < kH3Limit);   // NaN weights: unsafe as well
}

// both images (f32 fragments, fp16x3 split) from the canonical parameters in ONE launch; the last N
// blocks compute the per-agent fp16x3 safety flags
// f32_only: the exact-f32 image alone (no fp16x3 image, no flag blocks) — what the learner's own exact forward
// reads after each Adam step; the rollout's fp16x3 image is refreshed lazily by a full pack before its next use
__global__ __launch_bounds__(1024) void qnet_pack_kernel(const float* __restrict__ params, float* __restrict__ packed, QnetGeo g, int N,
                                 int D, int F1, int G, int H, int A, QnetOffsets o, int f32_only) {
  const int nb = (int)gridDim.x - (f32_only ? 0 : N);
  if ((int)blockIdx.x >= nb) {
    qnet_h3_bound_block(params, reinterpret_cast<int*>(packed + 2 * g.agent_stride * N), (int)blockIdx.x - nb, D,
                        F1, G, H, A, o);
    return;
  }
  qnet_pack_body(params, packed, g, N, D, F1, G, H, A, o, nb);
  if (!f32_only) qnet_pack_h3_body(params, packed, g, N, D, F1, G, H, A, o, nb);
}

int qnet_pack(const mm_qnet_dims* d, const float* params, float* packed, hipStream_t s, int f32_only) {
  QnetGeo g;
  QnetOffsets o;
  int rc = qnet_geometry(d, &g, &o);
  if (rc) return rc;
  const int64_t total = g.agent_stride * d->n_agents;
  // 1024-thread blocks: the N flag blocks' scans and row bounds are latency chains, 16 waves each
  const int threads = 1024;
  const int blocks = (int)std::min<int64_t>((total + threads - 1) / threads, 1024) + (f32_only ? 0 : d->n_agents);
  hipLaunchKernelGGL(qnet_pack_kernel, dim3(blocks), dim3(threads), 0, s, params, packed, g, d->n_agents,
                     d->obs_dim, d->f1, d->g, d->h, d->n_actions, o, f32_only);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

// LDS-staged variant when every net of the launch has >= 2048 envs and the image fits in LDS.
static bool use_lds(const QFwdParams& p0, const QFwdParams* p1) {
  const size_t bytes = (size_t)p0.g.agent_stride * 4;
  return bytes <= 160 * 1024 && p0.E >= 2048 && (!p1 || p1->E >= 2048);
}

template <int F1, int G, int H, int AB>
static int launch_fwd(QFwdParams p0, const QFwdParams* p1in, hipStream_t s) {
  QFwdParams p1 = p1in ? *p1in : p0;
  if (use_lds(p0, p1in)) {
    p0.nblocks = (p0.E + 255) / 256 * p0.N;
    p1.nblocks = (p1.E + 255) / 256 * p1.N;
    const int nb = p0.nblocks + (p1in ? p1.nblocks : 0);
    const size_t sm = (size_t)p0.g.agent_stride * 4;
    hipLaunchKernelGGL((agent_q_fwd_h3_kernel<F1, G, H, AB>), dim3(nb), dim3(1024), sm, s, p0, p1);
  } else {
    const int nb = p0.nblocks + (p1in ? p1.nblocks : 0);
    hipLaunchKernelGGL((agent_q_fwd_kernel<F1, G, H, AB>), dim3(nb), dim3(256), 0, s, p0, p1);
  }
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

template <int F1, int G, int H, int AB>
static int launch_roll(QFwdParams p0, QFwdParams p1, const RollStep& rs, size_t sm, hipStream_t s) {
  p0.nblocks = (p0.E + 255) / 256 * p0.N;
  p1.nblocks = (p1.E + 255) / 256 * p1.N;
  hipLaunchKernelGGL((rollout_step_kernel<F1, G, H, AB>), dim3(p0.nblocks + p1.nblocks), dim3(1024), sm, s, p0, p1,
                     rs);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

template <int F1, int G, int H, int AB>
static int launch_chunk(QFwdParams p0, QFwdParams p1, const RollChunk& rc, int nb, size_t sm, hipStream_t s) {
  hipLaunchKernelGGL((rollout_chunk_kernel<F1, G, H, AB>), dim3(nb), dim3(1024), sm, s, p0, p1, rc);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

static int make_params(const mm_qnet_dims* d, const float* packed, const mm_qfwd_io* io, int64_t n_envs,
                       QFwdParams* p) {
  MM_REQUIRE(d && packed && io, "agent_q_fwd: null argument");
  MM_REQUIRE(n_envs >= 1 && n_envs < (1ll << 31), "agent_q_fwd: bad n_envs %lld", (long long)n_envs);
  p->io = *io;
  QnetOffsets o;
  int rc = qnet_geometry(d, &p->g, &o);
  if (rc) return rc;
  p->packed = packed;
  p->E = (int)n_envs;
  p->N = d->n_agents;
  p->D = d->obs_dim;
  p->A = d->n_actions;
  p->nblocks = (int)((n_envs + 127) / 128) * d->n_agents;
  p->stagger = 4;   // fp16x3 kernel: waves 8-15 start 4 x s_sleep(8) late (VALU phases under the others' MFMAs)
  p->dbg = 0;
  MM_REQUIRE(io->obs, "agent_q_fwd: obs required");
  MM_REQUIRE(io->h_in || io->reset == nullptr, "agent_q_fwd: h_in required");
  MM_REQUIRE(io->mode != MM_Q_GATHER || io->act_in, "agent_q_fwd: GATHER needs act_in");
  MM_REQUIRE(io->obs_row == nullptr || io->reset_obs, "agent_q_fwd: obs_row needs reset_obs");
  return MM_OK;
}

static int dispatch(const mm_qnet_dims* d, const QFwdParams& p0, const QFwdParams* p1, hipStream_t s) {
  const int AB = (d->n_actions + 31) / 32;
  if (d->f1 == 64 && d->g == 32 && d->h == 32) return AB == 1 ? launch_fwd<64, 32, 32, 1>(p0, p1, s) : launch_fwd<64, 32, 32, 2>(p0, p1, s);
  if (d->f1 == 64 && d->g == 64 && d->h == 64) return AB == 1 ? launch_fwd<64, 64, 64, 1>(p0, p1, s) : launch_fwd<64, 64, 64, 2>(p0, p1, s);
  if (d->f1 == 128 && d->g == 32 && d->h == 32) return AB == 1 ? launch_fwd<128, 32, 32, 1>(p0, p1, s) : launch_fwd<128, 32, 32, 2>(p0, p1, s);
  if (d->f1 == 64 && d->g == 32 && d->h == 64) return AB == 1 ? launch_fwd<64, 32, 64, 1>(p0, p1, s) : launch_fwd<64, 32, 64, 2>(p0, p1, s);
  set_error("agent_q_fwd: unsupported (F1,G,H)=(%d,%d,%d)", d->f1, d->g, d->h);
  return MM_EINVAL;
}

template <int F1, int G, int H, int AB>
static int launch_split(int phase, QFwdParams p0, QFwdParams p1, hipStream_t s) {
  const bool single = p1.nblocks == 0;   // one net only (agent_q_split2 with io1 == NULL)
  if (phase == 1) {
    const int t0 = (p0.E + 31) / 32 * p0.N, t1 = single ? 0 : (p1.E + 31) / 32 * p1.N;
    if (t0 + t1 <= 2048 && p0.g.KD <= kPreRbMaxKD) {
      // small batches: row blocks of each layer on separate waves (latency-bound regime)
      p0.nblocks = t0;
      p1.nblocks = t1;
      constexpr int NW = 3 * (H / 32) > F1 / 32 ? 3 * (H / 32) : F1 / 32;
      static_assert(NW >= G / 32, "layer-2 row blocks need a wave each");
      hipLaunchKernelGGL((agent_pre_rb_kernel<F1, G, H, AB>), dim3(t0 + t1), dim3(64 * NW), 0, s, p0, p1);
      MM_HIP_CHECK(hipGetLastError());
      return MM_OK;
    }
    const size_t sm = (size_t)p0.g.agent_stride * 4;
    if (sm <= 160 * 1024) {
      // many row tiles: the f32 image staged once per 512 rows
      p0.nblocks = (p0.E + 511) / 512 * p0.N;
      p1.nblocks = single ? 0 : (p1.E + 511) / 512 * p1.N;
      hipLaunchKernelGGL((agent_pre_lds_kernel<F1, G, H, AB>), dim3(p0.nblocks + p1.nblocks), dim3(1024), sm, s, p0,
                         p1);
      MM_HIP_CHECK(hipGetLastError());
      return MM_OK;
    }
    const int nb = p0.nblocks + p1.nblocks;
    hipLaunchKernelGGL((agent_split_kernel<F1, G, H, AB, 1>), dim3(nb), dim3(256), 0, s, p0, p1);
  } else {
    p0.nblocks = (p0.E + 31) / 32 * p0.N;
    p1.nblocks = single ? 0 : (p1.E + 31) / 32 * p1.N;
    const int nb = p0.nblocks + p1.nblocks;
    hipLaunchKernelGGL((agent_split_kernel<F1, G, H, AB, 2>), dim3(nb), dim3(64 * (H / 32)), 0, s, p0, p1);
  }
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

template <int F1, int G, int H, int AB>
static int launch_pre_h3(QFwdParams p0, QFwdParams p1, hipStream_t s) {
  const bool single = p1.nblocks == 0;
  p0.nblocks = (p0.E + 255) / 256 * p0.N;
  p1.nblocks = single ? 0 : (p1.E + 255) / 256 * p1.N;
  const size_t sm = (size_t)p0.g.agent_stride * 4;
  // an image too large to stage in LDS (large obs_dim): the exact-f32 PRE of phase 1 instead (same outputs at
  // the f32 bar), so a configuration that runs in exact mode never fails in fast mode
  if (sm > 160 * 1024) return launch_split<F1, G, H, AB>(1, p0, p1, s);
  hipLaunchKernelGGL((agent_pre_h3_kernel<F1, G, H, AB>), dim3(p0.nblocks + p1.nblocks), dim3(1024), sm, s, p0, p1);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

static int dispatch_split(const mm_qnet_dims* d, int phase, const QFwdParams& p0, const QFwdParams& p1,
                          hipStream_t s) {
  const int AB = (d->n_actions + 31) / 32;
#define MM_SPLIT(F1_, G_, H_)                                                                               \
  if (d->f1 == F1_ && d->g == G_ && d->h == H_) {                                                           \
    if (phase == 3)                                                                                         \
      return AB == 1 ? launch_pre_h3<F1_, G_, H_, 1>(p0, p1, s) : launch_pre_h3<F1_, G_, H_, 2>(p0, p1, s); \
    return AB == 1 ? launch_split<F1_, G_, H_, 1>(phase, p0, p1, s) : launch_split<F1_, G_, H_, 2>(phase, p0, p1, s); \
  }
  MM_SPLIT(64, 32, 32)
  MM_SPLIT(64, 64, 64)
  MM_SPLIT(128, 32, 32)
  MM_SPLIT(64, 32, 64)
#undef MM_SPLIT
  set_error("agent_q_split: unsupported (F1,G,H)=(%d,%d,%d)", d->f1, d->g, d->h);
  return MM_EINVAL;
}

template <int F1, int G, int H, int AB>
static int launch_rec_seq(QFwdParams p0, QFwdParams p1, const RecSeq& s0, const RecSeq& s1, bool single,
                          hipStream_t s) {
  p0.nblocks = (p0.E + 31) / 32 * p0.N;
  p1.nblocks = single ? 0 : (p1.E + 31) / 32 * p1.N;
  // few tiles (small learner batches): gate-parallel waves shorten each step's dependent MFMA chain 3x;
  // many tiles: the 2-wave kernel keeps more blocks per CU
  const bool gp = (p0.nblocks + p1.nblocks) < 512;
  if (gp) {
    static const hipError_t attr = hipFuncSetAttribute((const void*)agent_rec_seq_gp_kernel<F1, G, H, AB>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)RecGpLds<H>::bytes);
    MM_HIP_CHECK(attr);
    hipLaunchKernelGGL((agent_rec_seq_gp_kernel<F1, G, H, AB>), dim3(p0.nblocks + p1.nblocks),
                       dim3(64 * (3 * (H / 32) + 1)), RecGpLds<H>::bytes, s, p0, p1, s0, s1);
  } else {
    hipLaunchKernelGGL((agent_rec_seq_kernel<F1, G, H, AB>), dim3(p0.nblocks + p1.nblocks), dim3(64 * (H / 32)), 0,
                       s, p0, p1, s0, s1);
  }
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

// the two nets' launch parameters and sequence arguments of agent_q_rec_seq2 (also the paired launch's)
static int rec_seq_args(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t e0,
                        const float* packed1, const mm_qfwd_io* io1, int64_t e1, int32_t steps, const uint8_t* reset,
                        QFwdParams& p0, QFwdParams& p1, RecSeq& s0, RecSeq& s1, bool& single) {
  int rc = make_params(d, packed0, io0, e0, &p0);
  if (rc) return rc;
  single = !io1 || e1 <= 0;
  if (single) {
    p1 = p0;
  } else {
    rc = make_params(d, packed1, io1, e1, &p1);
    if (rc) return rc;
  }
  MM_REQUIRE(steps >= 1 && (steps == 1 || reset), "agent_q_rec_seq: steps >= 1 and reset flags required");
  MM_REQUIRE(io0->gi && (single || io1->gi), "agent_q_rec_seq: io.gi required");
  MM_REQUIRE(((uintptr_t)io0->save & 15) == 0 && (single || ((uintptr_t)io1->save & 15) == 0),
             "agent_q_rec_seq: the training save base must be 16-byte aligned");
  auto mk = [&](const QFwdParams& p) {
    RecSeq q;
    q.C = steps;
    q.gi_st = (int64_t)p.E * p.N * 3 * d->h;
    q.save_st = (int64_t)p.E * p.N * (d->f1 + d->g + 6 * d->h);
    q.act_st = (int64_t)p.E * p.io.act_se;
    q.qsel_st = (int64_t)p.E * p.N;
    q.reset = reset;
    q.reset_st = p.E;
    q.trace = nullptr;
    return q;
  };
  s0 = mk(p0);
  s1 = mk(p1);
  s0.trace = debug_trace_buffer("MM_REC_TRACE");
  return MM_OK;
}

int agent_q_rec_seq2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t e0,
                     const float* packed1, const mm_qfwd_io* io1, int64_t e1, int32_t steps, const uint8_t* reset,
                     hipStream_t s) {
  QFwdParams p0, p1;
  RecSeq s0, s1;
  bool single;
  const int rc = rec_seq_args(d, packed0, io0, e0, packed1, io1, e1, steps, reset, p0, p1, s0, s1, single);
  if (rc) return rc;
  const int AB = (d->n_actions + 31) / 32;
#define MM_RSEQ(F1_, G_, H_)                                                                                    \
  if (d->f1 == F1_ && d->g == G_ && d->h == H_)                                                                 \
    return AB == 1 ? launch_rec_seq<F1_, G_, H_, 1>(p0, p1, s0, s1, single, s)                                  \
                   : launch_rec_seq<F1_, G_, H_, 2>(p0, p1, s0, s1, single, s);
  MM_RSEQ(64, 32, 32)
  MM_RSEQ(64, 64, 64)
  MM_RSEQ(128, 32, 32)
  MM_RSEQ(64, 32, 64)
#undef MM_RSEQ
  set_error("agent_q_rec_seq: unsupported (F1,G,H)=(%d,%d,%d)", d->f1, d->g, d->h);
  return MM_EINVAL;
}

int agent_q_split2(int phase, const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t e0,
                   const float* packed1, const mm_qfwd_io* io1, int64_t e1, hipStream_t s) {
  QFwdParams p0, p1;
  int rc = make_params(d, packed0, io0, e0, &p0);
  if (rc) return rc;
  if (!io1 || e1 <= 0) {   // single net
    MM_REQUIRE(io0->gi, "agent_q_split: io.gi required");
    MM_REQUIRE(phase == 2 || (((uintptr_t)io0->gi | (uintptr_t)io0->save) & 15) == 0,
               "agent_q_pre: gi / save bases must be 16-byte aligned");
    p1 = p0;
    p1.nblocks = 0;
    return dispatch_split(d, phase, p0, p1, s);
  }
  rc = make_params(d, packed1, io1, e1, &p1);
  if (rc) return rc;
  MM_REQUIRE(io0->gi && io1->gi, "agent_q_split: io.gi required");
  MM_REQUIRE(phase == 2 || (((uintptr_t)io0->gi | (uintptr_t)io1->gi | (uintptr_t)io0->save | (uintptr_t)io1->save) & 15) == 0,
             "agent_q_pre: gi / save bases must be 16-byte aligned");
  MM_REQUIRE(phase == 2 || (io0->obs && io1->obs), "agent_q_pre: obs required");   // phase 3: PRE on fp16x3
  return dispatch_split(d, phase, p0, p1, s);
}

int agent_q_fwd(const mm_qnet_dims* d, const float* packed, const mm_qfwd_io* io, int64_t n_envs, hipStream_t s) {
  if (n_envs == 0) return MM_OK;
  QFwdParams p;
  int rc = make_params(d, packed, io, n_envs, &p);
  if (rc) return rc;
  return dispatch(d, p, nullptr, s);
}

int agent_q_fwd2(const mm_qnet_dims* d, const float* packed0, const mm_qfwd_io* io0, int64_t e0,
                 const float* packed1, const mm_qfwd_io* io1, int64_t e1, hipStream_t s) {
  QFwdParams p0, p1;
  int rc = make_params(d, packed0, io0, e0, &p0);
  if (rc) return rc;
  rc = make_params(d, packed1, io1, e1, &p1);
  if (rc) return rc;
  return dispatch(d, p0, &p1, s);
}

// LDS bytes of the fused rollout step for this env / net, or 0 when the fused step does not apply (the
// two-launch path is used instead): local obs (D = 47), agent markers in a nibble, a grid of <= 128 cells
// in 16-byte rows, E >= 2048 and image + env staging within the CU's 160 KiB.
// bytes of the region that first stages the env (and TD) inputs and then holds the weight image
static size_t roll_region(const EnvDev& ev, const QnetGeo& g) {
  // grids | positions | actions | steps | apples | TD: rew, Q(a), max Q', act | TD rows | chunk_td | dones | rows
  const size_t staging = ((256 * (size_t)ev.R * ev.C + 15) & ~size_t(15)) + 6 * 256 * (size_t)ev.N * 4 + 7424;
  return (std::max((size_t)g.agent_stride * 4, staging) + 15) & ~size_t(15);
}

size_t rollout_step_lds(const mm_env* env, const mm_qnet_dims* d, int64_t n_envs) {
  if (!env || !d) return 0;
  const EnvDev& ev = env->d;
  QnetGeo g;
  QnetOffsets o;
  if (qnet_geometry(d, &g, &o)) return 0;
  if (ev.full_obs || ev.D != OBS_LOCAL || d->obs_dim != ev.D || d->n_agents != ev.N) return 0;
  // 8 columns: one nibble word per row; an even row count: whole 16-byte grid pieces per env (staging reads and the
  // writer's grid stores)
  if (ev.N > kRollMaxN || ev.R > kRollMaxR || ev.C != 8 || (ev.R & 1)) return 0;
  if (n_envs < 2048 || n_envs != ev.E) return 0;
  const bool known = (d->f1 == 64 && d->g == 32 && d->h == 32) || (d->f1 == 64 && d->g == 64 && d->h == 64) ||
                     (d->f1 == 128 && d->g == 32 && d->h == 32) || (d->f1 == 64 && d->g == 32 && d->h == 64);
  if (!known) return 0;
  const size_t sm = roll_region(ev, g) + (size_t)roll_lds(ev.R, ev.C, ev.N).total;
  return sm <= 160 * 1024 ? sm : 0;
}

int rollout_step(mm_env* env, const mm_qnet_dims* d, const float* packed_t, const mm_qfwd_io* io_t,
                 const float* packed_b, const mm_qfwd_io* io_b, int64_t n_envs, const mm_rollout_step_io* x,
                 hipStream_t s) {
  MM_REQUIRE(env && d && x, "rollout_step: null argument");
  const size_t sm = rollout_step_lds(env, d, n_envs);
  MM_REQUIRE(sm > 0, "rollout_step: configuration not supported by the fused step (mm_rollout_step_supported)");
  MM_REQUIRE(x->act && x->store_obs && x->staging && x->cur_row && x->rew && x->done && x->counter,
             "rollout_step: null step buffer");
  MM_REQUIRE(x->state_in == 0 || x->state_in == 1, "rollout_step: state_in must be 0 or 1");
  MM_REQUIRE(io_t->mode == MM_Q_MAX && io_b->mode == MM_Q_ACT, "rollout_step: target io must be MAX, behavior io ACT");
  MM_REQUIRE(io_t->h_in && io_b->h_in && io_t->h_out && io_b->h_out, "rollout_step: hidden states required");
  MM_REQUIRE(io_b->reset == nullptr, "rollout_step: the behavior reset flags are the step's own dones (pass NULL)");
  const int64_t nd = (int64_t)d->n_agents * d->obs_dim;
  MM_REQUIRE(x->slot >= 1 && x->chunk_len >= x->slot && x->row_stride >= (x->chunk_len + 1) * nd,
             "rollout_step: bad store slot / row stride");
  QFwdParams p0, p1;
  int rc = make_params(d, packed_t, io_t, n_envs, &p0);
  if (rc) return rc;
  rc = make_params(d, packed_b, io_b, n_envs, &p1);
  if (rc) return rc;
  RollStep rs;
  rs.env = env->d;
  rs.act = x->act;
  rs.store_obs = x->store_obs;
  rs.row_stride = x->row_stride;
  rs.next_off = (int64_t)x->slot * nd;
  rs.staging = x->staging;
  rs.cur_row = x->cur_row;
  rs.rew = x->rew;
  rs.done = x->done;
  rs.counter = x->counter;
  rs.td = TdFuse{};
  if (x->td_on) {
    MM_REQUIRE(x->td_rew && x->td_done && x->td_qsel && x->td_maxq && x->td_act && x->chunk_td && x->store_act &&
                   x->store_rew && x->store_done, "rollout_step: null TD argument");
    MM_REQUIRE(x->td_slot >= 0 && x->td_slot < x->chunk_len, "rollout_step: bad TD slot");
    rs.td = TdFuse{x->td_rew, x->td_done, x->td_qsel, x->td_maxq, x->td_act, x->chunk_td, x->store_act,
                   x->store_rew, x->store_done, x->staging, nullptr, x->gamma, x->td_slot, x->chunk_len, 1};
  }
  rs.par = x->state_in;
#if MM_ROLL_DEBUG
  rs.trace = debug_trace_buffer("MM_ROLL_TRACE");
#else
  rs.trace = nullptr;
#endif
  MM_REQUIRE(x->n_rows >= 1 && x->n_rows < (1ll << 40), "rollout_step: n_rows must be the chunk store's row count");
  rs.n_rows = x->n_rows;
  rs.err = reinterpret_cast<uint32_t*>(x->err);
  rs.begin = x->begin ? 1 : 0;
  rs.lds_env = (int)roll_region(env->d, p0.g);
  const int AB = (d->n_actions + 31) / 32;
#define MM_ROLL(F1_, G_, H_)                                                                             \
  if (d->f1 == F1_ && d->g == G_ && d->h == H_)                                                          \
    return AB == 1 ? launch_roll<F1_, G_, H_, 1>(p0, p1, rs, sm, s) : launch_roll<F1_, G_, H_, 2>(p0, p1, rs, sm, s);
  MM_ROLL(64, 32, 32)
  MM_ROLL(64, 64, 64)
  MM_ROLL(128, 32, 32)
  MM_ROLL(64, 32, 64)
#undef MM_ROLL
  set_error("rollout_step: unsupported (F1,G,H)");
  return MM_EINVAL;
}

// LDS bytes of the chunk-persistent rollout (image + the env state it keeps across steps), or 0 when it does not
// apply: the fused step's geometry, and a grid of 2 N ceil(E / 256) blocks that fits the device's CUs one block per
// CU (every block must be co-resident: the hand-off waits need all of a tile's blocks running).
size_t rollout_chunk_lds(const mm_env* env, const mm_qnet_dims* d, int64_t n_envs) {
  if (rollout_step_lds(env, d, n_envs) == 0) return 0;
  const EnvDev& ev = env->d;
  QnetGeo g;
  QnetOffsets o;
  if (qnet_geometry(d, &g, &o)) return 0;
  const size_t img = ((size_t)g.agent_stride * 4 + 15) & ~size_t(15);
  const size_t sm = img + (size_t)roll_chunk_lds(ev.R, ev.C, ev.N).total;
  if (sm > 160 * 1024) return 0;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  const int64_t nb = 2 * (int64_t)ev.N * ((n_envs + 255) / 256);
  return nb <= cus ? sm : 0;
}

int rollout_chunk(mm_env* env, const mm_qnet_dims* d, const float* packed_t, const mm_qfwd_io* io_t,
                  const float* packed_b, const mm_qfwd_io* io_b, int64_t n_envs, const mm_rollout_chunk_io* x,
                  hipStream_t s) {
  MM_REQUIRE(env && d && x && io_t && io_b, "rollout_chunk: null argument");
  const size_t sm = rollout_chunk_lds(env, d, n_envs);
  MM_REQUIRE(sm > 0, "rollout_chunk: configuration not supported (mm_rollout_chunk_supported)");
  const EnvDev& ev = env->d;
  MM_REQUIRE(x->store_obs && x->staging && x->cur_row && x->act0 && x->done_prev && x->rew && x->done && x->counter &&
                 x->ctl && x->handoff, "rollout_chunk: null buffer");
  MM_REQUIRE(x->chunk_len >= 1 && x->chunk_len <= 4096 && x->c0 >= 0 && x->c0 < x->chunk_len && x->n_steps >= 1,
             "rollout_chunk: bad chunk position / step count");
  MM_REQUIRE(x->n_sets >= 1 && x->n_sets <= 64 && x->set0 >= 0 && x->set0 < x->n_sets &&
                 x->c0 + x->n_steps <= (int64_t)x->n_sets * x->chunk_len,
             "rollout_chunk: the launch's steps span more chunks than staging sets (%d)", x->n_sets);
  MM_REQUIRE(x->ring_len >= 2 && x->ring_pos >= 0 && x->ring_pos < x->ring_len && x->n_steps < x->ring_len,
             "rollout_chunk: the rings must hold the launch's steps plus the next step's actions (n_steps < ring_len)");
  MM_REQUIRE(x->handoff_len >= x->n_steps, "rollout_chunk: handoff_len < n_steps");
  MM_REQUIRE(x->n_rows >= 1 && x->n_rows < (1ll << 40), "rollout_chunk: n_rows must be the chunk store's row count");
  MM_REQUIRE(io_t->mode == MM_Q_MAX && io_b->mode == MM_Q_ACT, "rollout_chunk: target io must be MAX, behavior io ACT");
  MM_REQUIRE(io_t->h_in && io_b->h_in && io_t->h_in == io_t->h_out && io_b->h_in == io_b->h_out,
             "rollout_chunk: hidden states required, updated in place");
  MM_REQUIRE(io_b->eps_ptr && io_b->act_out && io_b->qsel_out && io_t->qsel_out,
             "rollout_chunk: behavior eps_ptr / act_out / qsel_out and target qsel_out required");
  MM_REQUIRE(io_b->reset == nullptr && io_t->reset == nullptr, "rollout_chunk: reset flags come from the env (pass NULL)");
  const int64_t nd = (int64_t)d->n_agents * d->obs_dim;
  MM_REQUIRE(x->row_stride >= (x->chunk_len + 1) * nd, "rollout_chunk: row stride too small");
  QFwdParams p0, p1;
  mm_qfwd_io i0 = *io_t, i1 = *io_b;
  i0.obs = i1.obs = ev.reset_obs;   // unused (the obs come from the env state); make_params wants a pointer
  int rc = make_params(d, packed_t, &i0, n_envs, &p0);
  if (rc) return rc;
  rc = make_params(d, packed_b, &i1, n_envs, &p1);
  if (rc) return rc;
  const int tiles = (int)((n_envs + 255) / 256);
  p0.nblocks = p1.nblocks = tiles * d->n_agents;
  RollChunk r;
  r.env = ev;
  r.store_obs = x->store_obs;
  r.row_stride = x->row_stride;
  r.staging = x->staging;
  r.cur_row = x->cur_row;
  r.n_rows = x->n_rows;
  r.act0 = x->act0;
  r.done_prev = x->done_prev;
  r.rew = x->rew;
  r.done = x->done;
  r.counter = reinterpret_cast<uint64_t*>(x->counter);
  r.seq = reinterpret_cast<uint64_t*>(x->ctl);
  r.envpar = reinterpret_cast<int32_t*>(x->ctl + 1);
  r.ticket = reinterpret_cast<uint32_t*>(x->ctl + 2);
  r.hx = reinterpret_cast<uint64_t*>(x->handoff);
  r.err = reinterpret_cast<uint32_t*>(x->err);
#if MM_ROLL_DEBUG
  r.trace = debug_trace_buffer("MM_ROLL_TRACE");
#else
  r.trace = nullptr;
#endif
  r.c0 = x->c0;
  r.n = x->n_steps;
  r.CL = x->chunk_len;
  r.S = x->n_sets;
  r.set0 = x->set0;
  r.RL = x->ring_len;
  r.pos0 = x->ring_pos;
  r.hxl = x->handoff_len;
  QnetGeo g;
  QnetOffsets o;
  qnet_geometry(d, &g, &o);
  r.lds_env = (int)(((size_t)g.agent_stride * 4 + 15) & ~size_t(15));
  const int nb = 2 * tiles * d->n_agents;
  const int AB = (d->n_actions + 31) / 32;
#define MM_ROLLC(F1_, G_, H_)                                                                       \
  if (d->f1 == F1_ && d->g == G_ && d->h == H_)                                                     \
    return AB == 1 ? launch_chunk<F1_, G_, H_, 1>(p0, p1, r, nb, sm, s)                             \
                   : launch_chunk<F1_, G_, H_, 2>(p0, p1, r, nb, sm, s);
  MM_ROLLC(64, 32, 32)
  MM_ROLLC(64, 64, 64)
  MM_ROLLC(128, 32, 32)
  MM_ROLLC(64, 32, 64)
#undef MM_ROLLC
  set_error("rollout_chunk: unsupported (F1,G,H)");
  return MM_EINVAL;
}

}  // namespace mm
