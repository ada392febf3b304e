// Episode-level recurrent QMix / VDN trainer of the reference's offpolicy fork on gfx950
// (SURVEY §8f rank 3): QMix.train_policy_on_batch (offpolicy/algorithms/qmix/qmix.py:80-210).
//
//   agent  QMixPolicy / AgentQFunction (QMixPolicy.py:51-111, agent_q_function.py:24-57): one
//          LN-MLP-GRU-LN net shared by all agents, run over whole episodes (T+1 steps) from h = 0.
//          Same trunk as the MAPPO actor (trunk.h: MGeo layout, SF / GF fields, MFMA wgrad).
//   mixer  QMixer (q_mixer.py:20-94): hypernets Linear(S,Hh) -> ReLU -> Linear(Hh, N*K | K | 1),
//          hyper_b1 Linear(S,K); hidden = elu(q . |w1| + b1), Q_tot = hidden . |w2| + b2. VDN: sum.
//   loss   targets r^(agent 0) + (1 - d_env) gamma Q'_tot (target nets, double Q at the behavior
//          net's greedy actions), error masked by the previous step's d_env, PER-weighted MSE or
//          Huber / sum(mask), R2D2 priorities (1 - nu) mean_t |err| + nu max_t |err| + eps.
//
// Work split (T+1 = 101 steps x N*B = 256 rows at the reference shapes; everything is latency):
//   * the non-recurrent layers (LN0, L1, LN1, L2, LN2, W_ih x) and the heads (LN_r, W_o) run over
//     ALL (T+1)*N*B row-steps at once, one thread per row-step, weights LDS-staged;
//   * only the GRU recurrence is sequential: one wave per row, lane j = hidden unit j, its three
//     W_hh rows (forward) / W_hh column (BPTT) held in 192 VGPRs for the whole episode, h (or
//     dgh) broadcast lane-to-SGPR with v_readlane - no LDS, no barriers inside the time loop;
//   * the hypernet layers are GEMMs (LDS-tiled fp32, batched job list, deterministic split-K);
//   * agent weight gradients: the MFMA row reduction of trunk.h over GF operands.
#include "common.h"
#include "minimarl.h"
#include "trunk.h"

namespace mm {

constexpr int OQ_MAX_GEMM = 16;

// ------------------------------------------------------------------ workspace layout
struct OqWs {
  int64_t a1, a2, st, gi, hs, gates, act, qa, nqa, z1, w1o, w2o, b2o, qtot, dqtot, dqa, dw1o, dw2o, db2o, dz1, dh2, dg, gsoa,
      wpart, gpart, red, aerr, ones, total;  // float offsets
  int64_t NB, R1, Rb, rs1, rsb, TB;
  int NS, NG, ZW, NK;
};

static inline int64_t al64(int64_t x) { return (x + 63) / 64 * 64; }

__device__ __forceinline__ float rl(float v, int i) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), i));
}

// ------------------------------------------------------------------ forward: non-recurrent layers
// Saves of the behavior net (plain row-major): a1 / a2 [R][H] (post-ReLU), st [R][8] =
// mu0, rs0, mu1, rs1, mu2, rs2, mu_r, rs_r.
enum { ST_MU0 = 0, ST_RS0, ST_MU1, ST_RS1, ST_MU2, ST_RS2, ST_MUR, ST_RSR, ST_N };

struct OqPreArgs {
  const float* P[2];
  const float* obs;
  float* gi[2];
  float* a1; float* a2; float* st;   // behavior saves or NULL
  int64_t R1, NB;
  int T1, B;        // steps (T+1) and episodes; stacked = 1: obs is [L][R][D] already
  int stacked;
};

// full-wave sum broadcast to every lane: DPP inside each 16-lane row (quad_perm 1032 / 2301,
// row_ror 4 / 8), then the four row sums via v_readlane (no LDS round trips)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x124>(v);
  v += dpp<0x128>(v);
  return (rl(v, 0) + rl(v, 16)) + (rl(v, 32) + rl(v, 48));
}

// Per-wave LDS broadcast of a 64-vector held one element per lane: lane j stores v, every lane then
// reads the whole vector with 16 ds_read_b128 (same address in all lanes = broadcast). A wave's
// LDS operations execute in order, so no barrier is needed inside the wave-private slot.
template <int NV>
__device__ __forceinline__ void bcast_put(float* slot, int j, const float (&v)[NV]) {
#pragma unroll
  for (int c = 0; c < NV; ++c) slot[c * 64 + j] = v[c];
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ float4 bcast_get4(const float* slot, int i4) {
  return reinterpret_cast<const float4*>(slot)[i4];
}

__device__ __forceinline__ const float* obs_row(const float* obs, int stacked, int64_t r, int64_t NB, int B, int T1,
                                                int D) {
  if (stacked) return obs + r * D;
  const int64_t t = r / NB, q = r - t * NB;
  const int64_t i = q / B, b = q - i * B;
  return obs + ((i * T1 + t) * B + b) * D;
}

// One wave per row at a time, lane j = feature j (H == 64; D <= 128 as two lane halves). The net's
// W1 / W2 / W_ih rows are staged once per 1024-thread block into LDS with row strides of 4 x odd
// floats (a wave's ds_read_b128 of 64 different rows is conflict-free), so 16 waves per CU share one
// copy; activations are broadcast through a wave-private LDS slot, LayerNorm sums are DPP wave sums.
template <int D> struct PreLds {
  static constexpr int Dp = (D + 3) & ~3;
  static constexpr int S1 = ((Dp / 4) & 1) ? Dp : Dp + 4;    // W1 row stride (4 x odd)
  static constexpr int S2 = 68;                              // W2 / W_ih row stride
  static constexpr int oW2 = 64 * S1, oWih = oW2 + 64 * S2, oSlot = oWih + 192 * S2, total = oSlot + 16 * 128;
};

template <int D, int H, int A>
__global__ __launch_bounds__(1024) void offq_pre_kernel(OqPreArgs a) {
  static_assert(H == 64 && D <= 128, "lane-per-feature layout");
  using G = MGeo<D, H, A>;
  using L = PreLds<D>;
  constexpr int D0 = D < 64 ? D : 64, D1 = D - D0;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int y = blockIdx.y;
  const float* P = a.P[y];
  // stage W1 (Dp-wide rows), W2, W_ih as float4 rows
  for (int i = threadIdx.x; i < 64 * (G::Dp / 4); i += blockDim.x) {
    const int rj = i / (G::Dp / 4), c = i % (G::Dp / 4);
    *reinterpret_cast<float4*>(sm + rj * L::S1 + 4 * c) = *reinterpret_cast<const float4*>(P + G::W1 + rj * G::Dp + 4 * c);
  }
  for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) {
    const int rj = i >> 4, c = i & 15;
    *reinterpret_cast<float4*>(sm + L::oW2 + rj * L::S2 + 4 * c) = *reinterpret_cast<const float4*>(P + G::W2 + rj * H + 4 * c);
  }
  for (int i = threadIdx.x; i < 192 * 16; i += blockDim.x) {
    const int rj = i >> 4, c = i & 15;
    *reinterpret_cast<float4*>(sm + L::oWih + rj * L::S2 + 4 * c) = *reinterpret_cast<const float4*>(P + G::Wih + rj * H + 4 * c);
  }
  __syncthreads();
  const int j = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t wid = blockIdx.x * 16 + wv, nw = (int64_t)gridDim.x * 16;
  const float* w1 = sm + j * L::S1;
  const float* w2 = sm + L::oW2 + j * L::S2;
  const float* wr = sm + L::oWih + j * L::S2;
  const float* wz = sm + L::oWih + (H + j) * L::S2;
  const float* wn = sm + L::oWih + (2 * H + j) * L::S2;
  float* slot = sm + L::oSlot + wv * 128;
  const float g0a = j < D0 ? P[G::ln0_w + j] : 0.f, b0a = j < D0 ? P[G::ln0_b + j] : 0.f;
  const float g0b = j < D1 ? P[G::ln0_w + 64 + j] : 0.f, b0b = j < D1 ? P[G::ln0_b + 64 + j] : 0.f;
  const float b1 = P[G::b1 + j], g1 = P[G::ln1_w + j], c1 = P[G::ln1_b + j];
  const float b2 = P[G::b2 + j], g2 = P[G::ln2_w + j], c2 = P[G::ln2_b + j];
  const float bir = P[G::bih + j], biz = P[G::bih + H + j], bin = P[G::bih + 2 * H + j];
  const bool save = y == 0 && a.a1;
  // the next row's observation is loaded one row ahead
  float xa_n = 0.f, xb_n = 0.f;
  if (wid < a.R1) {
    const float* xp = obs_row(a.obs, a.stacked, wid, a.NB, a.B, a.T1, D);
    xa_n = j < D0 ? xp[j] : 0.f;
    xb_n = j < D1 ? xp[64 + j] : 0.f;
  }
  for (int64_t r = wid; r < a.R1; r += nw) {
    const float xa = xa_n, xb = xb_n;
    if (r + nw < a.R1) {
      const float* xp = obs_row(a.obs, a.stacked, r + nw, a.NB, a.B, a.T1, D);
      xa_n = j < D0 ? xp[j] : 0.f;
      xb_n = j < D1 ? xp[64 + j] : 0.f;
    }
    // LN0
    const float mu0 = wave_sum(xa + xb) / (float)D;
    const float da = j < D0 ? xa - mu0 : 0.f, db = j < D1 ? xb - mu0 : 0.f;
    const float rs0 = 1.0f / sqrtf(wave_sum(da * da + db * db) / (float)D + kLnEps);
    const float fa = da * rs0 * g0a + b0a, fb = db * rs0 * g0b + b0b;
    // L1 + ReLU + LN1 (W1 pad columns are zero)
    {
      const float fv[2] = {fa, fb};
      bcast_put<2>(slot, j, fv);
    }
    float s0 = b1, s1 = 0.f;
#pragma unroll
    for (int c = 0; c < G::Dp / 4; ++c) {
      const float4 t4 = bcast_get4(slot, c), w4 = *reinterpret_cast<const float4*>(w1 + 4 * c);
      s0 = fmaf(w4.x, t4.x, s0);
      s1 = fmaf(w4.y, t4.y, s1);
      s0 = fmaf(w4.z, t4.z, s0);
      s1 = fmaf(w4.w, t4.w, s1);
    }
    const float a1 = fmaxf(s0 + s1, 0.0f);
    const float mu1 = wave_sum(a1) * (1.0f / H);
    const float e1 = a1 - mu1;
    const float rs1 = 1.0f / sqrtf(wave_sum(e1 * e1) * (1.0f / H) + kLnEps);
    const float f1 = e1 * rs1 * g1 + c1;
    // L2 + ReLU + LN2
    {
      const float fv[1] = {f1};
      bcast_put<1>(slot, j, fv);
    }
    s0 = b2;
    s1 = 0.f;
#pragma unroll
    for (int c = 0; c < H / 4; ++c) {
      const float4 t4 = bcast_get4(slot, c), w4 = *reinterpret_cast<const float4*>(w2 + 4 * c);
      s0 = fmaf(w4.x, t4.x, s0);
      s1 = fmaf(w4.y, t4.y, s1);
      s0 = fmaf(w4.z, t4.z, s0);
      s1 = fmaf(w4.w, t4.w, s1);
    }
    const float a2 = fmaxf(s0 + s1, 0.0f);
    const float mu2 = wave_sum(a2) * (1.0f / H);
    const float e2 = a2 - mu2;
    const float rs2 = 1.0f / sqrtf(wave_sum(e2 * e2) * (1.0f / H) + kLnEps);
    const float x2 = e2 * rs2 * g2 + c2;
    // GRU input projection
    {
      const float fv[1] = {x2};
      bcast_put<1>(slot, j, fv);
    }
    float gr = bir, gz = biz, gn = bin;
#pragma unroll
    for (int c = 0; c < H / 4; ++c) {
      const float4 t4 = bcast_get4(slot, c);
      const float4 r4 = *reinterpret_cast<const float4*>(wr + 4 * c);
      const float4 z4 = *reinterpret_cast<const float4*>(wz + 4 * c);
      const float4 n4 = *reinterpret_cast<const float4*>(wn + 4 * c);
      gr = fmaf(r4.x, t4.x, gr);
      gz = fmaf(z4.x, t4.x, gz);
      gn = fmaf(n4.x, t4.x, gn);
      gr = fmaf(r4.y, t4.y, gr);
      gz = fmaf(z4.y, t4.y, gz);
      gn = fmaf(n4.y, t4.y, gn);
      gr = fmaf(r4.z, t4.z, gr);
      gz = fmaf(z4.z, t4.z, gz);
      gn = fmaf(n4.z, t4.z, gn);
      gr = fmaf(r4.w, t4.w, gr);
      gz = fmaf(z4.w, t4.w, gz);
      gn = fmaf(n4.w, t4.w, gn);
    }
    float* go = a.gi[y] + r * (3 * H);
    go[j] = gr;
    go[H + j] = gz;
    go[2 * H + j] = gn;
    if (save) {
      a.a1[r * H + j] = a1;
      a.a2[r * H + j] = a2;
      if (j < 6) {
        const float sv = j == 0 ? mu0 : j == 1 ? rs0 : j == 2 ? mu1 : j == 3 ? rs1 : j == 4 ? mu2 : rs2;
        a.st[r * ST_N + j] = sv;
      }
    }
  }
}

// ------------------------------------------------------------------ forward: GRU recurrence
struct OqRecArgs {
  const float* P[2];
  const float* gi[2];
  float* hs[2];     // [L][NB][H]
  float* gates;     // behavior [L][NB][4][H] (r, z, n, W_hn h + b_hn) or NULL
  const float* h0;  // [NB][H] or NULL (zeros)
  float* hout;      // [NB][H] or NULL (net 0)
  int64_t NB;
  int L, whh, bhh;
};


// one wave per row q; lane j owns hidden unit j (H == 64)
template <int H>
__global__ __launch_bounds__(256) void offq_rec_kernel(OqRecArgs a) {
  static_assert(H == 64, "one lane per hidden unit");
  const int y = blockIdx.y;
  const int64_t q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= a.NB) return;
  const int j = threadIdx.x & 63;
  const float* P = a.P[y];
  float wr[H], wz[H], wn[H];
#pragma unroll
  for (int i = 0; i < H; ++i) {
    wr[i] = P[a.whh + j * H + i];
    wz[i] = P[a.whh + (H + j) * H + i];
    wn[i] = P[a.whh + (2 * H + j) * H + i];
  }
  const float br = P[a.bhh + j], bz = P[a.bhh + H + j], bn = P[a.bhh + 2 * H + j];
  float h = (a.h0 && y == 0) ? a.h0[q * H + j] : 0.0f;
  __shared__ __attribute__((aligned(16))) float sm[4][64];
  float* slot = sm[threadIdx.x >> 6];
  const float* gi = a.gi[y];
  float* hs = a.hs[y];
  float* gates = y == 0 ? a.gates : nullptr;
  // next step's input projections are loaded one step ahead (off the recurrence's critical path)
  const float* gp = gi + q * 3 * H + j;
  float gr = gp[0], gz = gp[H], gn = gp[2 * H];
  for (int t = 0; t < a.L; ++t) {
    const int64_t r = (int64_t)t * a.NB + q;
    float gr1 = 0.f, gz1 = 0.f, gn1 = 0.f;
    if (t + 1 < a.L) {
      const float* np_ = gp + (int64_t)(t + 1) * a.NB * 3 * H;
      gr1 = np_[0];
      gz1 = np_[H];
      gn1 = np_[2 * H];
    }
    // two partial sums per gate halve the dependent FMA chain; h is broadcast through LDS
    {
      const float fv[1] = {h};
      bcast_put<1>(slot, j, fv);
    }
    float ar0 = br, az0 = bz, an0 = bn, ar1 = 0.f, az1 = 0.f, an1 = 0.f;
#pragma unroll
    for (int c = 0; c < H / 4; ++c) {
      const float4 t4 = bcast_get4(slot, c);
      ar0 = fmaf(wr[4 * c], t4.x, ar0);
      az0 = fmaf(wz[4 * c], t4.x, az0);
      an0 = fmaf(wn[4 * c], t4.x, an0);
      ar1 = fmaf(wr[4 * c + 1], t4.y, ar1);
      az1 = fmaf(wz[4 * c + 1], t4.y, az1);
      an1 = fmaf(wn[4 * c + 1], t4.y, an1);
      ar0 = fmaf(wr[4 * c + 2], t4.z, ar0);
      az0 = fmaf(wz[4 * c + 2], t4.z, az0);
      an0 = fmaf(wn[4 * c + 2], t4.z, an0);
      ar1 = fmaf(wr[4 * c + 3], t4.w, ar1);
      az1 = fmaf(wz[4 * c + 3], t4.w, az1);
      an1 = fmaf(wn[4 * c + 3], t4.w, an1);
    }
    const float an = an0 + an1;
    const float rr = sigmoidf_(gr + (ar0 + ar1));
    const float zz = sigmoidf_(gz + (az0 + az1));
    const float nn = tanhf_(gn + rr * an);
    h = nn + zz * (h - nn);
    hs[r * H + j] = h;
    if (gates) {
      float* g = gates + r * 4 * H;
      g[j] = rr;
      g[H + j] = zz;
      g[2 * H + j] = nn;
      g[3 * H + j] = an;
    }
    gr = gr1;
    gz = gz1;
    gn = gn1;
  }
  if (a.hout && y == 0) a.hout[q * H + j] = h;
}

// ------------------------------------------------------------------ forward: heads + Q selection
struct OqPostArgs {
  const float* P[2];
  const float* hs[2];
  float* st;            // behavior mu_r / rs_r into st[r][6..7] (or NULL)
  float* q_out;         // [R1][A] of net 0 (or NULL)
  const float* acts;    // one-hot [N][T][B][A] (or NULL: no selection)
  int32_t* act;         // [Rb] chosen action index of the behavior row
  float* qa;            // [T][B][N] Q(s_t, a_t)
  float* nqa;           // [T][B][N] target Q at t+1
  int64_t R1, NB;
  int T, B, N, nets, double_q;
};

template <int D, int H, int A>
__global__ __launch_bounds__(256) void offq_post_kernel(OqPostArgs a) {
  using G = MGeo<D, H, A>;
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r >= a.R1) return;
  float qv[2][A];
  for (int y = 0; y < a.nets; ++y) {
    const float* P = a.P[y];
    float h[H], yv[H];
    load_row<H>(a.hs[y] + r * H, h);
    float mu, rs;
    ln_stats<H>(h, mu, rs);
    if (y == 0 && a.st) {
      a.st[r * ST_N + ST_MUR] = mu;
      a.st[r * ST_N + ST_RSR] = rs;
    }
    ln_apply<H>(h, mu, rs, P + G::lnr_w, P + G::lnr_b, yv);
    float o[A];
    matvec<A, H, H>(P + G::Wo, P + G::bo, yv, o);
#pragma unroll
    for (int k = 0; k < A; ++k) qv[y][k] = o[k];
  }
  if (a.q_out) {
#pragma unroll
    for (int k = 0; k < A; ++k) a.q_out[r * A + k] = qv[0][k];
  }
  if (!a.acts) return;
  const int64_t t = r / a.NB, qq = r - t * a.NB;
  const int64_t i = qq / a.B, b = qq - i * a.B;
  if (t < a.T) {
    // action index = first max of the one-hot row (q_values_from_actions, QMixPolicy.py:103)
    const float* oh = a.acts + ((i * a.T + t) * a.B + b) * A;
    int ai = 0;
    float best = oh[0];
#pragma unroll
    for (int k = 1; k < A; ++k)
      if (oh[k] > best) {
        best = oh[k];
        ai = k;
      }
    a.act[r] = ai;
    float sel = qv[0][0];
#pragma unroll
    for (int k = 1; k < A; ++k)
      if (k == ai) sel = qv[0][k];
    a.qa[(t * a.B + b) * a.N + i] = sel;
  }
  if (t >= 1) {
    float nq;
    if (a.double_q) {
      int g = 0;
#pragma unroll
      for (int k = 1; k < A; ++k)
        if (qv[0][k] > qv[0][g]) g = k;
      nq = qv[1][0];
#pragma unroll
      for (int k = 1; k < A; ++k)
        if (k == g) nq = qv[1][k];
    } else {
      nq = qv[1][0];
#pragma unroll
      for (int k = 1; k < A; ++k) nq = fmaxf(nq, qv[1][k]);
    }
    a.nqa[((t - 1) * a.B + b) * a.N + i] = nq;
  }
}

// ------------------------------------------------------------------ batched fp32 GEMM jobs
// C(m, n) = sum_k A(m, k) B(k, n) [+ bias(n)] [* (mask(m, n) > 0)], with
//   A(m, k) = ta ? A[k*lda + m] : A[m*lda + k],  B(k, n) = tb ? B[n*ldb + k] : B[k*ldb + n],
// optional ReLU applied to A / B elements on load. 64x64 tiles, BK = 16, LDS-staged, 4x4 per
// thread. ksplit > 1: per-slice partials summed by offq_gemm_sum_kernel in slice order.
struct GemmJob {
  const float* A; const float* B; float* C; const float* bias; const float* mask;
  int64_t lda, ldb, ldc, ldm;
  int M, N, K, ta, tb, relu_a, relu_b, ksplit, kchunk, tiles_m, tiles_n, blk0;
  int64_t part;
};
struct GemmArgs {
  GemmJob job[OQ_MAX_GEMM];
  int njobs;
  float* partial;
};

__global__ __launch_bounds__(256) void offq_gemm_kernel(GemmArgs g) {
  int jx = 0;
  while (jx + 1 < g.njobs && (int)blockIdx.x >= g.job[jx + 1].blk0) ++jx;
  const GemmJob& j = g.job[jx];
  const int b = blockIdx.x - j.blk0;
  const int tiles = j.tiles_m * j.tiles_n;
  const int ks = b / tiles, tile = b - ks * tiles;
  const int m0 = (tile / j.tiles_n) * 64, n0 = (tile % j.tiles_n) * 64;
  const int k_begin = ks * j.kchunk, k_end = min(j.K, k_begin + j.kchunk);
  __shared__ float As[16][68], Bs[16][68];
  const int tid = threadIdx.x, tm = tid >> 4, tn = tid & 15;
  float c[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) c[u][v] = 0.0f;
  for (int k0 = k_begin; k0 < k_end; k0 += 16) {
    // A tile 64 (m) x 16 (k)
    if (!j.ta) {
      const int m = tid >> 2, kk = (tid & 3) * 4;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int gm = m0 + m, gk = k0 + kk + u;
        float v = (gm < j.M && gk < k_end) ? j.A[(int64_t)gm * j.lda + gk] : 0.0f;
        As[kk + u][m] = j.relu_a ? fmaxf(v, 0.0f) : v;
      }
    } else {
      const int kk = tid >> 4, m = (tid & 15) * 4;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int gm = m0 + m + u, gk = k0 + kk;
        float v = (gm < j.M && gk < k_end) ? j.A[(int64_t)gk * j.lda + gm] : 0.0f;
        As[kk][m + u] = j.relu_a ? fmaxf(v, 0.0f) : v;
      }
    }
    // B tile 16 (k) x 64 (n)
    if (j.tb) {
      const int n = tid >> 2, kk = (tid & 3) * 4;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int gn = n0 + n, gk = k0 + kk + u;
        float v = (gn < j.N && gk < k_end) ? j.B[(int64_t)gn * j.ldb + gk] : 0.0f;
        Bs[kk + u][n] = j.relu_b ? fmaxf(v, 0.0f) : v;
      }
    } else {
      const int kk = tid >> 4, n = (tid & 15) * 4;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int gn = n0 + n + u, gk = k0 + kk;
        float v = (gn < j.N && gk < k_end) ? j.B[(int64_t)gk * j.ldb + gn] : 0.0f;
        Bs[kk][n + u] = j.relu_b ? fmaxf(v, 0.0f) : v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        av[u] = As[kk][tm * 4 + u];
        bv[u] = Bs[kk][tn * 4 + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) c[u][v] = fmaf(av[u], bv[v], c[u][v]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int m = m0 + tm * 4 + u;
    if (m >= j.M) continue;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int n = n0 + tn * 4 + v;
      if (n >= j.N) continue;
      if (j.ksplit > 1) {
        g.partial[j.part + ((int64_t)ks * j.M + m) * j.N + n] = c[u][v];
      } else {
        float val = c[u][v] + (j.bias ? j.bias[n] : 0.0f);
        if (j.mask && !(j.mask[(int64_t)m * j.ldm + n] > 0.0f)) val = 0.0f;
        j.C[(int64_t)m * j.ldc + n] = val;
      }
    }
  }
}

__global__ __launch_bounds__(256) void offq_gemm_sum_kernel(GemmArgs g) {
  const GemmJob& j = g.job[blockIdx.y];
  if (j.ksplit <= 1) return;
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t MN = (int64_t)j.M * j.N;
  if (e >= MN) return;
  const int m = (int)(e / j.N), n = (int)(e % j.N);
  float s = 0.0f;
  for (int k = 0; k < j.ksplit; ++k) s += g.partial[j.part + k * MN + e];
  if (j.bias) s += j.bias[n];
  if (j.mask && !(j.mask[(int64_t)m * j.ldm + n] > 0.0f)) s = 0.0f;
  j.C[(int64_t)m * j.ldc + n] = s;
}

struct GemmList {
  GemmArgs g = {};
  int blocks = 0, max_mn = 0, nsplit = 0;
  int64_t part = 0;
  void add(const float* A, int64_t lda, int ta, int relu_a, const float* B, int64_t ldb, int tb, int relu_b, float* C,
           int64_t ldc, int M, int N, int K, const float* bias = nullptr, const float* mask = nullptr,
           int64_t ldm = 0, int rows_per_split = 0) {
    GemmJob& j = g.job[g.njobs++];
    j.A = A; j.B = B; j.C = C; j.bias = bias; j.mask = mask;
    j.lda = lda; j.ldb = ldb; j.ldc = ldc; j.ldm = ldm;
    j.M = M; j.N = N; j.K = K; j.ta = ta; j.tb = tb; j.relu_a = relu_a; j.relu_b = relu_b;
    j.ksplit = rows_per_split > 0 ? (K + rows_per_split - 1) / rows_per_split : 1;
    if (j.ksplit < 1) j.ksplit = 1;
    j.kchunk = (K + j.ksplit - 1) / j.ksplit;
    j.kchunk = (j.kchunk + 15) / 16 * 16;
    j.ksplit = j.kchunk > 0 ? (K + j.kchunk - 1) / j.kchunk : 1;
    if (j.ksplit < 1) j.ksplit = 1;
    j.tiles_m = (M + 63) / 64;
    j.tiles_n = (N + 63) / 64;
    j.blk0 = blocks;
    blocks += j.tiles_m * j.tiles_n * j.ksplit;
    j.part = part;
    if (j.ksplit > 1) {
      part += (int64_t)j.ksplit * M * N;
      nsplit++;
    }
    max_mn = std::max(max_mn, M * N);
  }
  int launch(float* partial, hipStream_t s) {
    if (g.njobs == 0) return MM_OK;
    g.partial = partial;
    hipLaunchKernelGGL(offq_gemm_kernel, dim3(blocks), dim3(256), 0, s, g);
    MM_HIP_CHECK(hipGetLastError());
    if (nsplit) {
      hipLaunchKernelGGL(offq_gemm_sum_kernel, dim3((max_mn + 255) / 256, g.njobs), dim3(256), 0, s, g);
      MM_HIP_CHECK(hipGetLastError());
    }
    return MM_OK;
  }
};

// ------------------------------------------------------------------ mixer forward combine
struct OqMixArgs {
  const float* z1[2]; const float* w1o[2]; const float* w2o[2]; const float* b2o[2];
  const float* q[2];     // qa / nqa [TB][N]
  float* qtot[2];
  int64_t TB;
  int N, K, Hh, ZW, nets, vdn;
};

__device__ __forceinline__ float elu1(float x) { return x > 0.0f ? x : expm1f(x); }

// KP = pow2 >= K lanes per mixer row (K <= 64): lane k owns mixing unit k; sums over k by shuffles
__device__ __forceinline__ float lanes_sum(float v, int kp) {
  for (int o = kp >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(256) void offq_mix_fwd_kernel(OqMixArgs a) {
  const int y = blockIdx.y;
  if (y >= a.nets) return;
  if (a.vdn) {
    const int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (m >= a.TB) return;
    const float* q = a.q[y] + m * a.N;
    float s = 0.0f;
    for (int i = 0; i < a.N; ++i) s += q[i];
    a.qtot[y][m] = s;
    return;
  }
  int kp = 1;
  while (kp < a.K) kp <<= 1;
  const int k = threadIdx.x & (kp - 1);
  const int64_t m = blockIdx.x * (int64_t)(blockDim.x / kp) + threadIdx.x / kp;
  const bool on = m < a.TB;
  const int64_t mm_ = on ? m : 0;
  const float* q = a.q[y] + mm_ * a.N;
  const float* w1 = a.w1o[y] + mm_ * (int64_t)a.N * a.K;
  float c = 0.0f;
  if (on && k < a.K) {
    float s = 0.0f;
    for (int i = 0; i < a.N; ++i) s = fmaf(q[i], fabsf(w1[i * a.K + k]), s);
    const float hid = elu1(s + a.z1[y][mm_ * a.ZW + 2 * a.Hh + k]);
    c = hid * fabsf(a.w2o[y][mm_ * a.K + k]);
  }
  c = lanes_sum(c, kp);
  if (on && k == 0) a.qtot[y][m] = c + a.b2o[y][m];
}

// ------------------------------------------------------------------ loss, priorities, dQ_tot
struct OqLossArgs {
  const float* qtot; const float* qtot_t;   // [T][B]
  const float* rew;                          // [N][T][B] (agent 0 slice used)
  const float* dn;                           // [T][B]
  const float* isw;                          // [B] or NULL
  float* dqtot;                              // [T][B]
  float* stats;                              // [2]
  float* prio;                               // [B] or NULL
  float* ones;
  float* aerr;                               // [T][B] scratch |err|
  int T, B, huber;
  float gamma, delta, nu, eps;
};

__device__ float block_sum1024(float v, float* sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = 0.0f;
  for (int w = 0; w < 16; ++w) r += sh[w];
  __syncthreads();
  return r;
}

// one block of 1024 threads: elementwise over the T*B (t, b) entries, then per-episode priorities
__global__ __launch_bounds__(1024) void offq_loss_kernel(OqLossArgs a) {
  __shared__ float sh[16];
  if (threadIdx.x == 0) a.ones[0] = 1.0f;
  const int T = a.T, B = a.B, TB = T * B;
  float cnt = 0.0f, qs = 0.0f;
  for (int e = threadIdx.x; e < TB; e += 1024) {
    const float keep = 1.0f - (e >= B ? a.dn[e - B] : 0.0f);
    cnt += keep;
    qs += a.qtot[e] * keep;
  }
  const float denom = block_sum1024(cnt, sh);
  const float qsum = block_sum1024(qs, sh);
  float lsum = 0.0f;
  for (int e = threadIdx.x; e < TB; e += 1024) {
    const int b = e % B;
    const float w = a.isw ? a.isw[b] : 1.0f;
    const float keep = 1.0f - (e >= B ? a.dn[e - B] : 0.0f);
    const float y = a.rew[e] + (1.0f - a.dn[e]) * a.gamma * a.qtot_t[e];
    const float er = (a.qtot[e] - y) * keep;
    const float ae = fabsf(er);
    float le, dle;
    if (a.huber) {
      const bool in = ae <= a.delta;
      le = in ? er * er / 2.0f : a.delta * (ae - a.delta / 2.0f);
      dle = in ? er : a.delta * (er > 0.0f ? 1.0f : (er < 0.0f ? -1.0f : 0.0f));
    } else {
      le = er * er;
      dle = 2.0f * er;
    }
    a.dqtot[e] = (w / denom) * dle * keep;
    a.aerr[e] = ae;
    lsum += le * w;
  }
  const float loss = block_sum1024(lsum, sh);  // (its barriers also order the aerr writes)
  if (a.prio) {
    for (int b = threadIdx.x; b < B; b += 1024) {
      float s = 0.0f, mx = 0.0f;
      for (int t = 0; t < T; ++t) {
        const float v = a.aerr[t * B + b];
        s += v;
        mx = fmaxf(mx, v);
      }
      a.prio[b] = (1.0f - a.nu) * (s / (float)T) + a.nu * mx + a.eps;
    }
  }
  if (threadIdx.x == 0) {
    a.stats[0] = loss / denom;
    a.stats[1] = qsum / (float)TB;
  }
}

// ------------------------------------------------------------------ mixer backward (per row)
struct OqMixBwdArgs {
  const float* z1; const float* w1o; const float* w2o; const float* q; const float* dqtot;
  float* dw1o; float* dw2o; float* db2o; float* dz1; float* dqa;
  int64_t TB;
  int N, K, Hh, ZW, vdn;
};

__global__ __launch_bounds__(256) void offq_mix_bwd_kernel(OqMixBwdArgs a) {
  if (a.vdn) {
    const int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (m >= a.TB) return;
    const float g = a.dqtot[m];
    for (int i = 0; i < a.N; ++i) a.dqa[m * a.N + i] = g;
    return;
  }
  int kp = 1;
  while (kp < a.K) kp <<= 1;
  const int k = threadIdx.x & (kp - 1);
  const int64_t m = blockIdx.x * (int64_t)(blockDim.x / kp) + threadIdx.x / kp;
  const bool on = m < a.TB && k < a.K;
  const int64_t mm_ = m < a.TB ? m : 0;
  const float g = a.dqtot[mm_];
  const float* q = a.q + mm_ * a.N;
  const float* w1 = a.w1o + mm_ * (int64_t)a.N * a.K;
  float dpre = 0.0f;
  if (on) {
    float s = 0.0f;
    for (int i = 0; i < a.N; ++i) s = fmaf(q[i], fabsf(w1[i * a.K + k]), s);
    const float pre = s + a.z1[mm_ * a.ZW + 2 * a.Hh + k];
    const float hid = elu1(pre);
    const float w2k = a.w2o[mm_ * a.K + k];
    // |w2|' = sign(w2) (0 at 0); elu' = 1 (x > 0) or exp(x) = elu(x) + 1
    a.dw2o[mm_ * a.K + k] = g * hid * (w2k > 0.0f ? 1.0f : (w2k < 0.0f ? -1.0f : 0.0f));
    dpre = g * fabsf(w2k) * (pre > 0.0f ? 1.0f : hid + 1.0f);
    a.dz1[mm_ * a.ZW + 2 * a.Hh + k] = dpre;
    if (k == 0) a.db2o[mm_] = g;
  }
  for (int i = 0; i < a.N; ++i) {
    float c = 0.0f;
    if (on) {
      const float wv = w1[i * a.K + k];
      a.dw1o[mm_ * (int64_t)a.N * a.K + i * a.K + k] = q[i] * dpre * (wv > 0.0f ? 1.0f : (wv < 0.0f ? -1.0f : 0.0f));
      c = fabsf(wv) * dpre;
    }
    c = lanes_sum(c, kp);
    if (m < a.TB && k == 0) a.dqa[m * a.N + i] = c;
  }
}

// ------------------------------------------------------------------ agent backward: heads
struct OqHeadBwdArgs {
  const float* P; const float* hs; const float* st; const int32_t* act; const float* dqa;
  float* gsoa; float* dh2;
  int64_t Rb, NB;
  int B, N;
};

template <int D, int H, int A>
__global__ __launch_bounds__(256) void offq_head_bwd_kernel(OqHeadBwdArgs a) {
  using G = MGeo<D, H, A>;
  using F = GF<D, H, A>;
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r >= a.Rb) return;
  const int64_t t = r / a.NB, qq = r - t * a.NB;
  const int64_t i = qq / a.B, b = qq - i * a.B;
  const float dq = a.dqa[(t * a.B + b) * a.N + i];
  const int ai = a.act[r];
  float dout[A];
#pragma unroll
  for (int k = 0; k < A; ++k) dout[k] = k == ai ? dq : 0.0f;
  float* go = soa_col(a.gsoa, r, F::NG);
  const float* W = a.P;
  float h[H], xr[H], yv[H];
  load_row<H>(a.hs + r * H, h);
  const float mur = a.st[r * ST_N + ST_MUR], rsr = a.st[r * ST_N + ST_RSR];
#pragma unroll
  for (int k = 0; k < H; ++k) {
    xr[k] = (h[k] - mur) * rsr;
    yv[k] = xr[k] * W[G::lnr_w + k] + W[G::lnr_b + k];
  }
  soa_st<A>(go, F::DOUT, dout);
  soa_st<H>(go, F::Y, yv);
  float dy[H], dh[H];
  matvec_t<A, H, H>(W + G::Wo, dout, dy);
  ln_bwd<H>(dy, xr, rsr, W + G::lnr_w, dh);
  soa_st<H>(go, F::DY, dy);
#pragma unroll
  for (int k = 0; k < H; ++k) yv[k] = dy[k] * xr[k];
  soa_st<H>(go, F::PY, yv);
  float* o = a.dh2 + r * H;
#pragma unroll
  for (int k = 0; k < H; k += 4) *reinterpret_cast<float4*>(o + k) = make_float4(dh[k], dh[k + 1], dh[k + 2], dh[k + 3]);
}

// ------------------------------------------------------------------ agent backward: BPTT
struct OqRecBwdArgs {
  const float* P; const float* hs; const float* gates; const float* dh2;
  float* dg;  // [Rb][6][H]: dgi (r, z, n) then dgh (r, z, n)
  int64_t NB;
  int T, whh;
};

template <int H>
__global__ __launch_bounds__(256) void offq_rec_bwd_kernel(OqRecBwdArgs a) {
  static_assert(H == 64, "one lane per hidden unit");
  const int64_t q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= a.NB) return;
  const int j = threadIdx.x & 63;
  // column j of W_hh: wr[k] = W_hr[k][j], ...
  float wr[H], wz[H], wn[H];
#pragma unroll
  for (int k = 0; k < H; ++k) {
    wr[k] = a.P[a.whh + k * H + j];
    wz[k] = a.P[a.whh + (H + k) * H + j];
    wn[k] = a.P[a.whh + (2 * H + k) * H + j];
  }
  float dnext = 0.0f;
  __shared__ __attribute__((aligned(16))) float sm[4][3 * 64];
  float* slot = sm[threadIdx.x >> 6];
  // operands of step t-1 are loaded one step ahead
  auto load = [&](int t, float& d2, float& rr, float& zz, float& nn, float& ghn, float& hin) {
    const int64_t r = (int64_t)t * a.NB + q;
    d2 = a.dh2[r * H + j];
    const float* g = a.gates + r * 4 * H;
    rr = g[j];
    zz = g[H + j];
    nn = g[2 * H + j];
    ghn = g[3 * H + j];
    hin = t > 0 ? a.hs[(r - a.NB) * H + j] : 0.0f;
  };
  float d2, rr, zz, nn, ghn, hin;
  load(a.T - 1, d2, rr, zz, nn, ghn, hin);
  for (int t = a.T - 1; t >= 0; --t) {
    const int64_t r = (int64_t)t * a.NB + q;
    float d2n = 0.f, rrn = 0.f, zzn = 0.f, nnn = 0.f, ghnn = 0.f, hinn = 0.f;
    if (t > 0) load(t - 1, d2n, rrn, zzn, nnn, ghnn, hinn);
    const float dh = d2 + dnext;
    const float dn = dh * (1.0f - zz);
    const float dz = dh * (hin - nn);
    const float dpn = dn * (1.0f - nn * nn);
    const float dgr = dpn * ghn * rr * (1.0f - rr);
    const float dgz = dz * zz * (1.0f - zz);
    const float dghn = dpn * rr;
    float* o = a.dg + r * 6 * H;
    o[j] = dgr;
    o[H + j] = dgz;
    o[2 * H + j] = dpn;
    o[3 * H + j] = dgr;
    o[4 * H + j] = dgz;
    o[5 * H + j] = dghn;
    {
      const float fv[3] = {dgr, dgz, dghn};
      bcast_put<3>(slot, j, fv);
    }
    float acc0 = dh * zz, acc1 = 0.0f, acc2 = 0.0f;
#pragma unroll
    for (int c = 0; c < H / 4; ++c) {
      const float4 tr = bcast_get4(slot, c), tz = bcast_get4(slot, 16 + c), tn = bcast_get4(slot, 32 + c);
      const float vr[4] = {tr.x, tr.y, tr.z, tr.w}, vz[4] = {tz.x, tz.y, tz.z, tz.w}, vn[4] = {tn.x, tn.y, tn.z, tn.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc0 = fmaf(wr[4 * c + u], vr[u], acc0);
        acc1 = fmaf(wz[4 * c + u], vz[u], acc1);
        acc2 = fmaf(wn[4 * c + u], vn[u], acc2);
      }
    }
    dnext = acc0 + acc1 + acc2;
    d2 = d2n;
    rr = rrn;
    zz = zzn;
    nn = nnn;
    ghn = ghnn;
    hin = hinn;
  }
}

// ------------------------------------------------------------------ agent backward: MLP / LN layers
// Lane-per-feature like the forward: lane k keeps column k of W_ih (3 gates), W2 and W1 in VGPRs,
// so every transposed mat-vec is 64 readlane broadcasts + FMAs; the LayerNorm backward sums are
// wave reductions. Writes the GF operands of the weight-gradient reduction (tiled SoA).
struct OqPreBwdArgs {
  const float* P; const float* obs; const float* a1; const float* a2; const float* st; const float* hs;
  const float* dg;
  float* gsoa;
  int64_t Rb, NB;
  int T1, B;
};

template <int D, int H, int A>
__global__ __launch_bounds__(256) void offq_pre_bwd_kernel(OqPreBwdArgs a) {
  static_assert(H == 64 && D <= 128, "lane-per-feature layout");
  using G = MGeo<D, H, A>;
  using F = GF<D, H, A>;
  constexpr int D0 = D < 64 ? D : 64, D1 = D - D0;
  const float* P = a.P;
  const int k = threadIdx.x & 63;
  const int64_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  constexpr int HB = D1 > 0 ? H : 1;  // second W1 column half only when D > 64
  float cr[H], cz[H], cn[H], c2[H], c1a[H], c1bb[HB];
#pragma unroll
  for (int jj = 0; jj < H; ++jj) {
    cr[jj] = P[G::Wih + jj * H + k];
    cz[jj] = P[G::Wih + (H + jj) * H + k];
    cn[jj] = P[G::Wih + (2 * H + jj) * H + k];
    c2[jj] = P[G::W2 + jj * H + k];
    c1a[jj] = k < D0 ? P[G::W1 + jj * G::Dp + k] : 0.f;
  }
#pragma unroll
  for (int jj = 0; jj < HB; ++jj) c1bb[jj] = (D1 > 0 && k < D1) ? P[G::W1 + jj * G::Dp + 64 + k] : 0.f;
  const float g2 = P[G::ln2_w + k], c2b = P[G::ln2_b + k], g1 = P[G::ln1_w + k], c1 = P[G::ln1_b + k];
  const float g0a = k < D0 ? P[G::ln0_w + k] : 0.f, b0a = k < D0 ? P[G::ln0_b + k] : 0.f;
  const float g0b = k < D1 ? P[G::ln0_w + 64 + k] : 0.f, b0b = k < D1 ? P[G::ln0_b + 64 + k] : 0.f;
  __shared__ __attribute__((aligned(16))) float sm[4][3 * 64];
  float* slot = sm[threadIdx.x >> 6];
  // the GF operands of RG consecutive rows are gathered in LDS (the two field ranges this kernel writes: [DGI, DY) and
  // [DX2, NG)) and leave as one 16-byte store per field and lane: the rows of a 64-row SoA tile are contiguous per
  // field, where per-row stores wrote 64 separate 4-byte pieces per instruction
  constexpr int NA = F::DY - F::DGI, NR = NA + (F::NG - F::DX2);
  constexpr int RG = 4;   // rows per group (8: 144 KB of LDS, measured slower than 4: 0.809 vs 0.79 ms per update)
  __shared__ __attribute__((aligned(16))) float rbuf[4][RG][NR];
  const int64_t ngroups = (a.Rb + RG - 1) / RG;
  for (int64_t gq = wid; gq < ngroups; gq += nw) {
  for (int j = 0; j < RG; ++j) {
    const int64_t r = gq * RG + j;
    if (r >= a.Rb) break;
    float* lo = rbuf[threadIdx.x >> 6][j];
    auto put = [&](int f, float v) { lo[f < F::DY ? f - F::DGI : NA + (f - F::DX2)] = v; };
    const float* dgp = a.dg + r * 6 * H;
    const float dr = dgp[k], dz = dgp[H + k], dn = dgp[2 * H + k];
    put(F::DGI + k, dr);
    put(F::DGI + H + k, dz);
    put(F::DGI + 2 * H + k, dn);
    put(F::DGH + k, dgp[3 * H + k]);
    put(F::DGH + H + k, dgp[4 * H + k]);
    put(F::DGH + 2 * H + k, dgp[5 * H + k]);
    put(F::HIN + k, r >= a.NB ? a.hs[(r - a.NB) * H + k] : 0.0f);
    // dx2 = W_ih^T dgi
    {
      const float fv[3] = {dr, dz, dn};
      bcast_put<3>(slot, k, fv);
    }
    float x0 = 0.f, x1 = 0.f, x2 = 0.f;
#pragma unroll
    for (int c = 0; c < H / 4; ++c) {
      const float4 tr = bcast_get4(slot, c), tz = bcast_get4(slot, 16 + c), tn = bcast_get4(slot, 32 + c);
      const float vr[4] = {tr.x, tr.y, tr.z, tr.w}, vz[4] = {tz.x, tz.y, tz.z, tz.w}, vn[4] = {tn.x, tn.y, tn.z, tn.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        x0 = fmaf(cr[4 * c + u], vr[u], x0);
        x1 = fmaf(cz[4 * c + u], vz[u], x1);
        x2 = fmaf(cn[4 * c + u], vn[u], x2);
      }
    }
    const float* sp = a.st + r * ST_N;
    // LN2 backward (x2 = LN2(a2)), ReLU
    float dx = x0 + x1 + x2;
    float av = a.a2[r * H + k];
    float xh = (av - sp[ST_MU2]) * sp[ST_RS2];
    put(F::X2 + k, xh * g2 + c2b);
    float gg = dx * g2;
    float sg = wave_sum(gg) * (1.0f / H), sgx = wave_sum(gg * xh) * (1.0f / H);
    float dpre = sp[ST_RS2] * (gg - sg - xh * sgx);
    dpre = av > 0.0f ? dpre : 0.0f;
    put(F::DX2 + k, dx);
    put(F::P2 + k, dx * xh);
    put(F::DPRE2 + k, dpre);
    // dx1 = W2^T dpre2, LN1 backward, ReLU
    {
      const float fv[1] = {dpre};
      bcast_put<1>(slot, k, fv);
    }
    x0 = 0.f;
    x1 = 0.f;
#pragma unroll
    for (int c = 0; c < H / 4; ++c) {
      const float4 t4 = bcast_get4(slot, c);
      x0 = fmaf(c2[4 * c], t4.x, x0);
      x1 = fmaf(c2[4 * c + 1], t4.y, x1);
      x0 = fmaf(c2[4 * c + 2], t4.z, x0);
      x1 = fmaf(c2[4 * c + 3], t4.w, x1);
    }
    dx = x0 + x1;
    av = a.a1[r * H + k];
    xh = (av - sp[ST_MU1]) * sp[ST_RS1];
    put(F::F1 + k, xh * g1 + c1);
    gg = dx * g1;
    sg = wave_sum(gg) * (1.0f / H);
    sgx = wave_sum(gg * xh) * (1.0f / H);
    dpre = sp[ST_RS1] * (gg - sg - xh * sgx);
    dpre = av > 0.0f ? dpre : 0.0f;
    put(F::DX1 + k, dx);
    put(F::P1 + k, dx * xh);
    put(F::DPRE1 + k, dpre);
    // df0 = W1^T dpre1 (lanes k < D0, and 64 + k < D), LN0 operands
    {
      const float fv[1] = {dpre};
      bcast_put<1>(slot, k, fv);
    }
    x0 = 0.f;
    x1 = 0.f;
#pragma unroll
    for (int c = 0; c < H / 4; ++c) {
      const float4 t4 = bcast_get4(slot, c);
      const float tv[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        x0 = fmaf(c1a[4 * c + u], tv[u], x0);
        if constexpr (D1 > 0) x1 = fmaf(c1bb[4 * c + u], tv[u], x1);
      }
    }
    const float* xp = obs_row(a.obs, 0, r, a.NB, a.B, a.T1, D);
    const float mu0 = sp[ST_MU0], rs0 = sp[ST_RS0];
    if (k < D0) {
      const float xh0 = (xp[k] - mu0) * rs0;
      put(F::DF0 + k, x0);
      put(F::P0 + k, x0 * xh0);
      put(F::F0 + k, xh0 * g0a + b0a);
    }
    if (k < D1) {
      const float xh0 = (xp[64 + k] - mu0) * rs0;
      put(F::DF0 + 64 + k, x1);
      put(F::P0 + 64 + k, x1 * xh0);
      put(F::F0 + 64 + k, xh0 * g0b + b0b);
    }
  }
  __builtin_amdgcn_wave_barrier();
  {
    const int64_t r0 = gq * RG;
    const int nv = (int)std::min<int64_t>(RG, a.Rb - r0);
    float* go0 = soa_col(a.gsoa, r0, F::NG);
    const float (*rb)[NR] = rbuf[threadIdx.x >> 6];
    for (int i = k; i < NR; i += 64) {
      const int f = i < NA ? F::DGI + i : F::DX2 + (i - NA);
      if (nv == RG) {
#pragma unroll
        for (int q = 0; q < RG; q += 4)
          *reinterpret_cast<float4*>(go0 + (int64_t)f * 64 + q) =
              make_float4(rb[q][i], rb[q + 1][i], rb[q + 2][i], rb[q + 3][i]);
      } else {
        for (int jj = 0; jj < nv; ++jj) go0[(int64_t)f * 64 + jj] = rb[jj][i];
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------ soft update
__global__ __launch_bounds__(256) void offq_soft_update_kernel(float* __restrict__ tgt, const float* __restrict__ src,
                                                               int64_t n, float c1, float c2) {
#pragma clang fp contract(off)
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    tgt[e] = tgt[e] * c1 + src[e] * c2;
}

// ------------------------------------------------------------------ host side
// register-weight lane-per-feature backward: >= 8 rows per wave (amortises the per-wave weight
// loads), <= 2048 waves
static inline unsigned wave_blocks(int64_t rows) {
  int64_t waves = (rows + 7) / 8;
  if (waves > 2048) waves = 2048;
  if (waves < 1) waves = 1;
  return (unsigned)((waves + 3) / 4);
}

// LDS-weight lane-per-feature kernels (16 waves per block, one block per CU): >= 4 rows per wave,
// at most one block per CU over all nets of the launch
static inline unsigned lds_blocks(int64_t rows, int nets) {
  int64_t b = (rows + 63) / 64;
  const int64_t cap = 256 / nets;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (unsigned)b;
}

static inline int mix_rows_per_block(int K, bool qm) {
  if (!qm) return 256;
  int kp = 1;
  while (kp < K) kp <<= 1;
  return 256 / kp;
}
static int64_t mixer_offsets(const mm_offq_dims* d, int64_t o[15]) {
  const int64_t S = d->state_dim, K = d->mixer_hidden, Hh = d->hyper_hidden, NK = (int64_t)d->n_agents * K;
  const int64_t sz[14] = {Hh * S, Hh, NK * Hh, NK, Hh * S, Hh, K * Hh, K, K * S, K, Hh * S, Hh, Hh, 1};
  int64_t c = 0;
  for (int i = 0; i < 14; ++i) {
    o[i] = c;
    c += d->mixer == MM_OFFQ_QMIX ? sz[i] : 0;
  }
  o[14] = c;
  return c;
}

template <int D, int H, int A>
struct OffqShape {
  using G = MGeo<D, H, A>;
  using TW = TrunkWgrad<D, H>;

  static OqWs layout(const mm_offq_dims* d, int T, int B) {
    OqWs w = {};
    w.NB = (int64_t)d->n_agents * B;
    w.R1 = (int64_t)(T + 1) * w.NB;
    w.Rb = (int64_t)T * w.NB;
    w.rs1 = al64(w.R1);
    w.rsb = al64(w.Rb);
    w.TB = (int64_t)T * B;
    w.NS = SF<H, A>::NS;
    w.NG = GF<D, H, A>::NG;
    const bool qm = d->mixer == MM_OFFQ_QMIX;
    w.ZW = qm ? 3 * d->hyper_hidden + d->mixer_hidden : 0;
    w.NK = qm ? d->n_agents * d->mixer_hidden : 0;
    const int K = qm ? d->mixer_hidden : 0;
    int64_t c = 0;
    auto take = [&](int64_t n) {
      const int64_t o = c;
      c += al64(n);
      return o;
    };
    w.a1 = take(w.R1 * H);
    w.a2 = take(w.R1 * H);
    w.st = take(w.R1 * ST_N);
    w.gi = take(2 * w.R1 * 3 * H);
    w.hs = take(2 * w.R1 * H);
    w.gates = take(w.R1 * 4 * H);
    w.act = take(w.Rb);
    w.qa = take(w.TB * d->n_agents);
    w.nqa = take(w.TB * d->n_agents);
    w.z1 = take(2 * w.TB * w.ZW);
    w.w1o = take(2 * w.TB * w.NK);
    w.w2o = take(2 * w.TB * K);
    w.b2o = take(2 * w.TB);
    w.qtot = take(2 * w.TB);
    w.dqtot = take(w.TB);
    w.dqa = take(w.TB * d->n_agents);
    w.dw1o = take(w.TB * w.NK);
    w.dw2o = take(w.TB * K);
    w.db2o = take(w.TB);
    w.dz1 = take(w.TB * w.ZW);
    w.dh2 = take(w.Rb * H);
    w.dg = take(w.Rb * 6 * H);
    w.gsoa = take(w.rsb * w.NG);
    {
      WgJobDev jv[MM_MAPPO_MAX_JOBS * 2];
      const int nj = TW::template jobs<A>(nullptr, w.rsb, nullptr, jv);
      const int64_t nblk = (w.rsb + TW::rows_per_block(w.rsb) - 1) / TW::rows_per_block(w.rsb);
      int64_t tot = 0;
      for (int q = 0; q < nj; ++q) tot += nblk * (int64_t)(jv[q].M * jv[q].K + jv[q].M);
      w.wpart = take(tot);
    }
    {
      GemmList gl;
      mixer_bwd_jobs(d, w, nullptr, nullptr, nullptr, nullptr, gl, true);
      w.gpart = take(gl.part > 0 ? gl.part : 1);
    }
    w.red = take(1024);
    w.aerr = take(w.TB);
    w.ones = take(1);
    w.total = c;
    return w;
  }

  // rows per split-K slice of the mixer weight-gradient reductions
  static constexpr int kRowsPerSplit = 256;

  static void mixer_bwd_jobs(const mm_offq_dims* d, const OqWs& w, float* ws, const float* P, float* grad,
                             const float* states, GemmList& gl, bool sizing) {
    if (d->mixer != MM_OFFQ_QMIX) return;
    int64_t o[15];
    mixer_offsets(d, o);
    const int K = d->mixer_hidden, Hh = d->hyper_hidden, S = d->state_dim, NK = w.NK, ZW = w.ZW;
    const int TB = (int)w.TB;
    const float* Pm = P ? P + G::total : nullptr;
    float* gm = grad ? grad + G::total : nullptr;
    auto f = [&](int64_t off) { return ws ? ws + off : nullptr; };
    auto gp = [&](int i) { return gm ? gm + o[i] : nullptr; };
    const float* ones = f(w.ones);
    // second layers: dW = D^T relu(Z1 part), db = colsum D
    gl.add(f(w.dw1o), NK, 1, 0, f(w.z1), ZW, 0, 1, gp(2), Hh, NK, Hh, TB, nullptr, nullptr, 0, kRowsPerSplit);
    gl.add(f(w.dw1o), NK, 1, 0, ones, 0, 0, 0, gp(3), 1, NK, 1, TB, nullptr, nullptr, 0, kRowsPerSplit);
    gl.add(f(w.dw2o), K, 1, 0, f(w.z1) ? f(w.z1) + Hh : nullptr, ZW, 0, 1, gp(6), Hh, K, Hh, TB, nullptr, nullptr, 0,
           kRowsPerSplit);
    gl.add(f(w.dw2o), K, 1, 0, ones, 0, 0, 0, gp(7), 1, K, 1, TB, nullptr, nullptr, 0, kRowsPerSplit);
    gl.add(f(w.db2o), 1, 1, 0, f(w.z1) ? f(w.z1) + 2 * Hh + K : nullptr, ZW, 0, 1, gp(12), Hh, 1, Hh, TB, nullptr,
           nullptr, 0, kRowsPerSplit);
    gl.add(f(w.db2o), 1, 1, 0, ones, 0, 0, 0, gp(13), 1, 1, 1, TB, nullptr, nullptr, 0, kRowsPerSplit);
    // first layers: dW = dZ1 part^T states, db = colsum
    const int col[4] = {0, Hh, 2 * Hh, 2 * Hh + K};
    const int rows[4] = {Hh, Hh, K, Hh};
    const int wi[4] = {0, 4, 8, 10};
    for (int s = 0; s < 4; ++s) {
      const float* dz = f(w.dz1) ? f(w.dz1) + col[s] : nullptr;
      gl.add(dz, ZW, 1, 0, states, S, 0, 0, gp(wi[s]), S, rows[s], S, TB, nullptr, nullptr, 0, kRowsPerSplit);
      gl.add(dz, ZW, 1, 0, ones, 0, 0, 0, gp(wi[s] + 1), 1, rows[s], 1, TB, nullptr, nullptr, 0, kRowsPerSplit);
    }
    (void)Pm;
    (void)sizing;
  }

  static int loss_grad(const mm_offq_dims* d, const mm_offq_batch* bt, const float* P, const float* PT, float* grad,
                       float* ws, float* stats, float* prio, hipStream_t s) {
    const int T = bt->T, B = bt->B, N = d->n_agents;
    const OqWs w = layout(d, T, B);
    const bool qm = d->mixer == MM_OFFQ_QMIX;
    const int K = qm ? d->mixer_hidden : 0, Hh = qm ? d->hyper_hidden : 0, S = d->state_dim;
    int64_t mo[15];
    mixer_offsets(d, mo);
    // ---- agent forward (behavior + target) over all T+1 steps
    OqPreArgs pa = {};
    pa.P[0] = P;
    pa.P[1] = PT;
    pa.obs = bt->obs;
    pa.gi[0] = ws + w.gi;
    pa.gi[1] = ws + w.gi + w.R1 * 3 * H;
    pa.a1 = ws + w.a1;
    pa.a2 = ws + w.a2;
    pa.st = ws + w.st;
    pa.R1 = w.R1;
    pa.NB = w.NB;
    pa.T1 = T + 1;
    pa.B = B;
    hipLaunchKernelGGL((offq_pre_kernel<D, H, A>), dim3(lds_blocks(w.R1, 2), 2), dim3(1024),
                       (size_t)PreLds<D>::total * 4, s, pa);
    MM_HIP_CHECK(hipGetLastError());
    OqRecArgs ra = {};
    ra.P[0] = P;
    ra.P[1] = PT;
    ra.gi[0] = pa.gi[0];
    ra.gi[1] = pa.gi[1];
    ra.hs[0] = ws + w.hs;
    ra.hs[1] = ws + w.hs + w.R1 * H;
    ra.gates = ws + w.gates;
    ra.NB = w.NB;
    ra.L = T + 1;
    ra.whh = G::Whh;
    ra.bhh = G::bhh;
    hipLaunchKernelGGL((offq_rec_kernel<H>), dim3((unsigned)((w.NB + 3) / 4), 2), dim3(256), 0, s, ra);
    MM_HIP_CHECK(hipGetLastError());
    OqPostArgs po = {};
    po.P[0] = P;
    po.P[1] = PT;
    po.hs[0] = ra.hs[0];
    po.hs[1] = ra.hs[1];
    po.st = ws + w.st;
    po.acts = bt->acts;
    po.act = reinterpret_cast<int32_t*>(ws + w.act);
    po.qa = ws + w.qa;
    po.nqa = ws + w.nqa;
    po.R1 = w.R1;
    po.NB = w.NB;
    po.T = T;
    po.B = B;
    po.N = N;
    po.nets = 2;
    po.double_q = bt->double_q;
    hipLaunchKernelGGL((offq_post_kernel<D, H, A>), dim3((unsigned)((w.R1 + 255) / 256)), dim3(256), 0, s, po);
    MM_HIP_CHECK(hipGetLastError());
    // ---- mixer forward (behavior on s_0..s_{T-1}, target on s_1..s_T)
    const float* st[2] = {bt->share_obs, bt->share_obs + (int64_t)B * S};
    if (qm) {
      GemmList g1, g2;
      for (int y = 0; y < 2; ++y) {
        const float* Pm = (y == 0 ? P : PT) + G::total;
        float* z1 = ws + w.z1 + y * w.TB * w.ZW;
        g1.add(st[y], S, 0, 0, Pm + mo[0], S, 1, 0, z1, w.ZW, (int)w.TB, Hh, S, Pm + mo[1]);
        g1.add(st[y], S, 0, 0, Pm + mo[4], S, 1, 0, z1 + Hh, w.ZW, (int)w.TB, Hh, S, Pm + mo[5]);
        g1.add(st[y], S, 0, 0, Pm + mo[8], S, 1, 0, z1 + 2 * Hh, w.ZW, (int)w.TB, K, S, Pm + mo[9]);
        g1.add(st[y], S, 0, 0, Pm + mo[10], S, 1, 0, z1 + 2 * Hh + K, w.ZW, (int)w.TB, Hh, S, Pm + mo[11]);
        g2.add(z1, w.ZW, 0, 1, Pm + mo[2], Hh, 1, 0, ws + w.w1o + y * w.TB * w.NK, w.NK, (int)w.TB, w.NK, Hh,
               Pm + mo[3]);
        g2.add(z1 + Hh, w.ZW, 0, 1, Pm + mo[6], Hh, 1, 0, ws + w.w2o + y * w.TB * K, K, (int)w.TB, K, Hh, Pm + mo[7]);
        g2.add(z1 + 2 * Hh + K, w.ZW, 0, 1, Pm + mo[12], Hh, 1, 0, ws + w.b2o + y * w.TB, 1, (int)w.TB, 1, Hh,
               Pm + mo[13]);
      }
      int rc = g1.launch(ws + w.gpart, s);
      if (rc) return rc;
      rc = g2.launch(ws + w.gpart, s);
      if (rc) return rc;
    }
    OqMixArgs ma = {};
    for (int y = 0; y < 2; ++y) {
      ma.z1[y] = ws + w.z1 + y * w.TB * w.ZW;
      ma.w1o[y] = ws + w.w1o + y * w.TB * w.NK;
      ma.w2o[y] = ws + w.w2o + y * w.TB * K;
      ma.b2o[y] = ws + w.b2o + y * w.TB;
      ma.qtot[y] = ws + w.qtot + y * w.TB;
    }
    ma.q[0] = ws + w.qa;
    ma.q[1] = ws + w.nqa;
    ma.TB = w.TB;
    ma.N = N;
    ma.K = K;
    ma.Hh = Hh;
    ma.ZW = w.ZW;
    ma.nets = 2;
    ma.vdn = !qm;
    hipLaunchKernelGGL(offq_mix_fwd_kernel, dim3((unsigned)((w.TB + mix_rows_per_block(K, qm) - 1) / mix_rows_per_block(K, qm)), 2),
                       dim3(256), 0, s, ma);
    MM_HIP_CHECK(hipGetLastError());
    // ---- loss, priorities, dQ_tot
    OqLossArgs la = {};
    la.qtot = ws + w.qtot;
    la.qtot_t = ws + w.qtot + w.TB;
    la.rew = bt->rewards;
    la.dn = bt->dones_env;
    la.isw = bt->is_weight;
    la.dqtot = ws + w.dqtot;
    la.stats = stats;
    la.prio = bt->is_weight ? prio : nullptr;
    la.ones = ws + w.ones;
    la.T = T;
    la.B = B;
    la.huber = bt->huber;
    la.gamma = bt->gamma;
    la.delta = bt->huber_delta;
    la.nu = bt->per_nu;
    la.eps = bt->per_eps;
    la.aerr = ws + w.aerr;
    hipLaunchKernelGGL(offq_loss_kernel, dim3(1), dim3(1024), 0, s, la);
    MM_HIP_CHECK(hipGetLastError());
    // ---- mixer backward
    OqMixBwdArgs mb = {};
    mb.z1 = ws + w.z1;
    mb.w1o = ws + w.w1o;
    mb.w2o = ws + w.w2o;
    mb.q = ws + w.qa;
    mb.dqtot = ws + w.dqtot;
    mb.dw1o = ws + w.dw1o;
    mb.dw2o = ws + w.dw2o;
    mb.db2o = ws + w.db2o;
    mb.dz1 = ws + w.dz1;
    mb.dqa = ws + w.dqa;
    mb.TB = w.TB;
    mb.N = N;
    mb.K = K;
    mb.Hh = Hh;
    mb.ZW = w.ZW;
    mb.vdn = !qm;
    hipLaunchKernelGGL(offq_mix_bwd_kernel, dim3((unsigned)((w.TB + mix_rows_per_block(K, qm) - 1) / mix_rows_per_block(K, qm))),
                       dim3(256), 0, s, mb);
    MM_HIP_CHECK(hipGetLastError());
    if (qm) {
      const float* Pm = P + G::total;
      float* z1 = ws + w.z1;
      float* dz1 = ws + w.dz1;
      GemmList g3, g4;
      // hypernet hidden deltas: dZ1 part = (D . W_second) * (Z1 part > 0)
      g3.add(ws + w.dw1o, w.NK, 0, 0, Pm + mo[2], Hh, 0, 0, dz1, w.ZW, (int)w.TB, Hh, w.NK, nullptr, z1, w.ZW);
      g3.add(ws + w.dw2o, K, 0, 0, Pm + mo[6], Hh, 0, 0, dz1 + Hh, w.ZW, (int)w.TB, Hh, K, nullptr, z1 + Hh, w.ZW);
      g3.add(ws + w.db2o, 1, 0, 0, Pm + mo[12], Hh, 0, 0, dz1 + 2 * Hh + K, w.ZW, (int)w.TB, Hh, 1, nullptr,
             z1 + 2 * Hh + K, w.ZW);
      int rc = g3.launch(ws + w.gpart, s);
      if (rc) return rc;
      mixer_bwd_jobs(d, w, ws, P, grad, st[0], g4, false);
      rc = g4.launch(ws + w.gpart, s);
      if (rc) return rc;
    }
    // ---- agent backward (behavior rows t < T)
    OqHeadBwdArgs hb = {};
    hb.P = P;
    hb.hs = ws + w.hs;
    hb.st = ws + w.st;
    hb.act = reinterpret_cast<const int32_t*>(ws + w.act);
    hb.dqa = ws + w.dqa;
    hb.gsoa = ws + w.gsoa;
    hb.dh2 = ws + w.dh2;
    hb.Rb = w.Rb;
    hb.NB = w.NB;
    hb.B = B;
    hb.N = N;
    hipLaunchKernelGGL((offq_head_bwd_kernel<D, H, A>), dim3((unsigned)((w.Rb + 255) / 256)), dim3(256), 0, s, hb);
    MM_HIP_CHECK(hipGetLastError());
    OqRecBwdArgs rb = {};
    rb.P = P;
    rb.hs = ws + w.hs;
    rb.gates = ws + w.gates;
    rb.dh2 = ws + w.dh2;
    rb.dg = ws + w.dg;
    rb.NB = w.NB;
    rb.T = T;
    rb.whh = G::Whh;
    hipLaunchKernelGGL((offq_rec_bwd_kernel<H>), dim3((unsigned)((w.NB + 3) / 4)), dim3(256), 0, s, rb);
    MM_HIP_CHECK(hipGetLastError());
    OqPreBwdArgs pb = {};
    pb.P = P;
    pb.obs = bt->obs;
    pb.a1 = ws + w.a1;
    pb.a2 = ws + w.a2;
    pb.st = ws + w.st;
    pb.hs = ws + w.hs;
    pb.dg = ws + w.dg;
    pb.gsoa = ws + w.gsoa;
    pb.Rb = w.Rb;
    pb.NB = w.NB;
    pb.T1 = T + 1;
    pb.B = B;
    hipLaunchKernelGGL((offq_pre_bwd_kernel<D, H, A>), dim3(wave_blocks(w.Rb)), dim3(256), 0, s, pb);
    MM_HIP_CHECK(hipGetLastError());
    return TW::template wgrad<A>(ws + w.gsoa, w.rsb, grad, ws + w.wpart, s);
  }

  static int64_t qvals_ws(int L, int64_t R) { return al64((int64_t)L * R * 3 * H) + al64((int64_t)L * R * H); }

  static int q_values(const float* P, const float* obs, const float* h0, float* q, float* hout, int L, int64_t R,
                      float* ws, hipStream_t s) {
    const int64_t R1 = (int64_t)L * R;
    OqPreArgs pa = {};
    pa.P[0] = P;
    pa.obs = obs;
    pa.gi[0] = ws;
    pa.R1 = R1;
    pa.NB = R;
    pa.T1 = L;
    pa.B = 1;
    pa.stacked = 1;
    hipLaunchKernelGGL((offq_pre_kernel<D, H, A>), dim3(lds_blocks(R1, 1), 1), dim3(1024),
                       (size_t)PreLds<D>::total * 4, s, pa);
    MM_HIP_CHECK(hipGetLastError());
    OqRecArgs ra = {};
    ra.P[0] = P;
    ra.gi[0] = ws;
    ra.hs[0] = ws + al64(R1 * 3 * H);
    ra.h0 = h0;
    ra.hout = hout;
    ra.NB = R;
    ra.L = L;
    ra.whh = G::Whh;
    ra.bhh = G::bhh;
    hipLaunchKernelGGL((offq_rec_kernel<H>), dim3((unsigned)((R + 3) / 4), 1), dim3(256), 0, s, ra);
    MM_HIP_CHECK(hipGetLastError());
    OqPostArgs po = {};
    po.P[0] = P;
    po.hs[0] = ra.hs[0];
    po.q_out = q;
    po.R1 = R1;
    po.NB = R;
    po.nets = 1;
    hipLaunchKernelGGL((offq_post_kernel<D, H, A>), dim3((unsigned)((R1 + 255) / 256)), dim3(256), 0, s, po);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }

  static int set_lds() {
    static bool done = false;
    if (done) return MM_OK;
    MM_HIP_CHECK(hipFuncSetAttribute((const void*)offq_pre_kernel<D, H, A>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, PreLds<D>::total * 4));
    done = true;
    return MM_OK;
  }
};

#define MM_OFFQ_DISPATCH(d, CALL)                                                                  \
  do {                                                                                             \
    if ((d)->hidden == 64 && (d)->n_actions == 5 && (d)->obs_dim == 47) {                          \
      using SH = mm::OffqShape<47, 64, 5>;                                                          \
      return CALL;                                                                                 \
    }                                                                                              \
    if ((d)->hidden == 64 && (d)->n_actions == 5 && (d)->obs_dim == 94) {                          \
      using SH = mm::OffqShape<94, 64, 5>;                                                          \
      return CALL;                                                                                 \
    }                                                                                              \
    mm::set_error("offq: unsupported dims D=%d H=%d A=%d (supported: D 47|94, H 64, A 5)", (d)->obs_dim, \
                  (d)->hidden, (d)->n_actions);                                                    \
    return MM_EINVAL;                                                                              \
  } while (0)

static int check_dims(const mm_offq_dims* d) {
  MM_REQUIRE(d && d->n_agents >= 1, "offq: bad dims");
  MM_REQUIRE(d->mixer == MM_OFFQ_VDN || d->mixer == MM_OFFQ_QMIX, "offq: mixer must be MM_OFFQ_VDN or MM_OFFQ_QMIX");
  MM_REQUIRE(d->mixer == MM_OFFQ_VDN ||
                 (d->state_dim >= 1 && d->mixer_hidden >= 1 && d->hyper_hidden >= 1 &&
                  (int64_t)d->n_agents * d->mixer_hidden <= 4096),
             "offq: QMIX needs state_dim, mixer_hidden, hyper_hidden >= 1 and N*K <= 4096");
  return MM_OK;
}

}  // namespace mm

// ------------------------------------------------------------------ C ABI
extern "C" {

int mm_offq_param_counts(const mm_offq_dims* d, int64_t* agent, int64_t* mixer) {
  int rc = mm::check_dims(d);
  if (rc) return rc;
  MM_REQUIRE(agent && mixer, "offq_param_counts: null output");
  int64_t o[15];
  *mixer = mm::mixer_offsets(d, o);
  MM_OFFQ_DISPATCH(d, (*agent = SH::G::total, MM_OK));
}

int mm_offq_mixer_offsets(const mm_offq_dims* d, int64_t offs[15]) {
  int rc = mm::check_dims(d);
  if (rc) return rc;
  MM_REQUIRE(offs, "offq_mixer_offsets: null output");
  mm::mixer_offsets(d, offs);
  return MM_OK;
}

int64_t mm_offq_workspace_bytes(const mm_offq_dims* d, int32_t T, int32_t B) {
  if (mm::check_dims(d) || T < 1 || B < 1) return -1;
  if (d->hidden == 64 && d->n_actions == 5 && d->obs_dim == 47) return mm::OffqShape<47, 64, 5>::layout(d, T, B).total * 4;
  if (d->hidden == 64 && d->n_actions == 5 && d->obs_dim == 94) return mm::OffqShape<94, 64, 5>::layout(d, T, B).total * 4;
  return -1;
}

int mm_offq_loss_grad(const mm_offq_dims* d, const mm_offq_batch* b, const float* P, const float* PT, float* grad,
                      void* ws, int64_t ws_bytes, float* stats, float* priorities, mm_stream_t s) {
  int rc = mm::check_dims(d);
  if (rc) return rc;
  MM_REQUIRE(b && P && PT && grad && ws && stats, "offq_loss_grad: null argument");
  MM_REQUIRE(b->obs && b->acts && b->rewards && b->dones_env && (d->mixer == MM_OFFQ_VDN || b->share_obs),
             "offq_loss_grad: batch arrays missing");
  MM_REQUIRE(b->T >= 1 && b->B >= 1, "offq_loss_grad: T, B must be >= 1");
  MM_REQUIRE(!b->is_weight || priorities, "offq_loss_grad: PER (is_weight) needs a priorities output");
  const int64_t need = mm_offq_workspace_bytes(d, b->T, b->B);
  MM_REQUIRE(need > 0 && ws_bytes >= need, "offq_loss_grad: workspace %lld bytes < %lld", (long long)ws_bytes,
             (long long)need);
  MM_OFFQ_DISPATCH(d, (SH::set_lds() ? MM_EHIP
                                     : SH::loss_grad(d, b, P, PT, grad, (float*)ws, stats, priorities, (hipStream_t)s)));
}

int64_t mm_offq_qvals_workspace_bytes(const mm_offq_dims* d, int32_t L, int64_t R) {
  if (!d || L < 1 || R < 1 || d->hidden != 64) return -1;
  return mm::OffqShape<47, 64, 5>::qvals_ws(L, R) * 4;
}

int mm_offq_q_values(const mm_offq_dims* d, const float* P, const float* obs, const float* h0, float* q, float* h_out,
                     int32_t L, int64_t R, void* ws, int64_t ws_bytes, mm_stream_t s) {
  MM_REQUIRE(d && P && obs && q && ws && L >= 1 && R >= 1, "offq_q_values: bad args");
  const int64_t need = mm_offq_qvals_workspace_bytes(d, L, R);
  MM_REQUIRE(need > 0 && ws_bytes >= need, "offq_q_values: workspace too small");
  MM_OFFQ_DISPATCH(d, (SH::set_lds() ? MM_EHIP : SH::q_values(P, obs, h0, q, h_out, L, R, (float*)ws, (hipStream_t)s)));
}

int mm_offq_soft_update(float* target, const float* source, int64_t n, double tau, mm_stream_t s) {
  MM_REQUIRE(target && source && n >= 0, "offq_soft_update: bad args");
  if (n == 0) return MM_OK;
  // torch: target * (1.0 - tau) + source * tau with the python-float scalars cast to f32
  const float c1 = (float)(1.0 - tau), c2 = (float)tau;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(mm::offq_soft_update_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)s, target, source, n, c1,
                     c2);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

}  // extern "C"
