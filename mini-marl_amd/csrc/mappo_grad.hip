// MAPPO training gradients on MFMA, one PPO epoch in two row passes (replaces the per-thread TRAIN forward
// + saves, the BPTT backward writing per-row gradient operands and the separate weight-gradient reduction).
//
// Reference (restated in oracle/mappo.py, pinned by tests/golden/mappo_*.npz):
//   trunk  mappo/utils/algorithm_utils/mlp.py:31-55, rnn.py:24-29,79, act.py / distributions.py,
//          r_actor_critic.py:189-208
//   loss   mappo/algorithms/ramppo_network.py:56-209 (ppo_update, cal_value_loss)
//   chunks mappo/runner/shared/shared_buffer.py:318-427 (L steps, start hidden = stored hidden)
//
// Layout: one wave = one tile of 32 rows (chunks in the recurrent pass, row-steps in the MLP pass).
// Activations live in the MFMA "act-frag" layout: lane (c, h) = (lane & 31, lane >> 5) holds, for row c,
// the 16 features kperm(q, h) of a 32-wide vector (q = 0..15), which is exactly the D layout of
// v_mfma_f32_32x32x2_f32 with features on M and rows on N and, with the same k permutation, the B operand of
// the next layer — forward and backward layer chains need no data movement. Weight gradients
// dW[m][n] = sum_c delta[m][c] x[n][c] put the row index on the MFMA k dimension: delta and x tiles are
// transposed through a per-wave LDS tile (4 x ds_write_b128 + 16 x ds_read_b32 per lane), and the same
// transposed reads give the bias and LayerNorm column sums. Each wave keeps its weight-gradient
// accumulators in registers across all its tiles; a block reduces its waves in LDS in a fixed order and
// writes one partial; a third kernel sums every partial of both passes in a fixed order (deterministic).
//
// Pass G (mappo_grad_gru_kernel, per tile of 32 L-step chunks): step 1 runs the trunk forward over the L
// steps from the stored chunk-start hidden and parks the L input hiddens and GRU inputs x2 in a per-wave
// global scratch (reused across the wave's tiles); step 2 walks the steps backwards, recomputes each step's
// GRU gates from its parked input hidden and x2, seeds the PPO / Huber loss, runs the head, LN_r and GRU
// backward, accumulates dW_ih, dW_hh, dWo and their biases / LN_r parameters, and writes the step's
// gradient w.r.t. the GRU input x2 (dx2 = W_ih^T dgates, 32 floats per row-step) to HBM.
// Pass M (mappo_grad_mlp_kernel, row-parallel, no recurrence): per tile of 32 row-steps it recomputes the
// LN-MLP forward from the obs and backpropagates dx2 through LN2, L2, LN1, L1 and LN0, accumulating dW2,
// dW1, b1, b2 and the three LayerNorms' parameters. Splitting the MLP backward out of the recurrent pass
// keeps pass G's registers to its 7 accumulator tiles + the step's GRU state (no spills, 2 waves per SIMD)
// and drops the parking of the MLP activations the single-pass kernel needed.
#include <algorithm>

#include "common.h"
#include "minimarl.h"
#include "trunk.h"

namespace mm {
namespace mgr {

constexpr int H = 32;          // hidden width this kernel is written for
constexpr int TP = 36;         // pitch of a transpose tile row (one chunk)
constexpr int TILE = 32 * TP;  // floats per transpose tile
constexpr int GW = 4;          // pass G: waves per block (1 per SIMD), one block per CU
constexpr int GT = 2;          // pass G: transpose tiles per wave
constexpr int MT = 3;          // pass M: transpose tiles per wave
constexpr int NB = 128;        // blocks per net and pass

// LDS image of a net (padded rows; transposed W_ih / W_hh for the backward data chain). Pass G stages all
// of it (the recomputed forward needs the MLP too); pass M stages the leading MLP part only (up to W2) plus
// the LayerNorm / bias vectors it reads, relocated right after W2 (MLP layout Geo::M*).
template <int D, int O>
struct Geo {
  static constexpr int DT = (D + 31) / 32, DPT = 32 * DT, P1 = DPT + 4, PW = 36, PT = 100;
  static constexpr int W1 = 0, W2 = W1 + 32 * P1, Wih = W2 + 32 * PW, Whh = Wih + 96 * PW, WihT = Whh + 96 * PW,
                       WhhT = WihT + 32 * PT, ln0w = WhhT + 32 * PT, ln0b = ln0w + DPT, b1 = ln0b + DPT,
                       ln1w = b1 + 32, ln1b = ln1w + 32, b2 = ln1b + 32, ln2w = b2 + 32, ln2b = ln2w + 32,
                       bih = ln2b + 32, bhh = bih + 96, lnrw = bhh + 96, lnrb = lnrw + 32, Wo = lnrb + 32,
                       bo = Wo + 8 * 32, scr = bo + 8;
  static_assert(O <= 8, "head wider than 8 outputs");
};

// v(lane) + v(lane ^ 32) with one v_permlane32_swap (no LDS round trip of ds_bpermute)
__device__ __forceinline__ float xsum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __builtin_amdgcn_sched_barrier(0);   // measured: without it the transposes' LDS traffic interleaves worse
}
// a zero the compiler cannot see through: LDS bases offset by it are re-derived per step, so the
// loop-invariant weight / LayerNorm reads are not hoisted out of the tile loop into hundreds of VGPRs
__device__ __forceinline__ int opaque0() {
  int z = 0;
  asm volatile("" : "+s"(z));
  return z;
}
__device__ __forceinline__ int lane_c() { return (int)(threadIdx.x & 31); }
__device__ __forceinline__ int lane_h() { return (int)((threadIdx.x >> 5) & 1); }

// acc += W[(lane & 31)][kperm(s, h)] * v[s] over s < 16 (row-major LDS W, pitch P): W v in act-frag
// k-groups of 8 features (4 per lane half) holding any of the first n features of a 32-wide block
constexpr int kgroups(int n) { return n >= 32 ? 4 : (n + 7) / 8; }
template <int P>
__device__ __forceinline__ void mm_rows(const float* W, const float (&v)[16], f32x16& acc, int ng = 4) {
  const float* wr = W + lane_c() * P + 4 * lane_h();
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    if (g >= ng) break;
    const float4 a4 = *reinterpret_cast<const float4*>(wr + 8 * g);
    acc = mfma32(a4.x, v[4 * g], acc);
    acc = mfma32(a4.y, v[4 * g + 1], acc);
    acc = mfma32(a4.z, v[4 * g + 2], acc);
    acc = mfma32(a4.w, v[4 * g + 3], acc);
  }
}
// acc += W[kperm(s, h)][(lane & 31)] * v[s]: W^T v in act-frag (column reads of row-major W, pitch P)
template <int P>
__device__ __forceinline__ void mm_cols(const float* W, const float (&v)[16], f32x16& acc) {
  const float* wc = W + 4 * lane_h() * P + lane_c();
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma32(wc[kperm(s, 0) * P], v[s], acc);
}

// transpose tile: lane (c, h) stores its act-frag vector as row c; reads give lane (i, h) feature i of
// chunk 2 s + h at k-step s
__device__ __forceinline__ void tput(float* T, const float (&v)[16]) {
  float* p = T + lane_c() * TP + 4 * lane_h();
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<float4*>(p + 8 * g) = make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
}
__device__ __forceinline__ void tget(const float* T, float (&o)[16]) {
  const float* p = T + lane_h() * TP + lane_c();
#pragma unroll
  for (int s = 0; s < 16; ++s) o[s] = p[2 * s * TP];
}
__device__ __forceinline__ float tsum(const float* T) {
  const float* p = T + lane_h() * TP + lane_c();
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += p[2 * k * TP];
  return s;
}

// weight-gradient accumulation (chunks on k)
__device__ __forceinline__ void acc_mfma(f32x16& acc, float a, float b) { acc = mfma32(a, b, acc); }

__device__ __forceinline__ void ld16(const float* p, float (&v)[16]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 t = reinterpret_cast<const float4*>(p)[g];
    v[4 * g] = t.x;
    v[4 * g + 1] = t.y;
    v[4 * g + 2] = t.z;
    v[4 * g + 3] = t.w;
  }
}
__device__ __forceinline__ void st16(float* p, const float (&v)[16]) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    reinterpret_cast<float4*>(p)[g] = make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
}
// a pointer the compiler cannot see through (no store-to-load forwarding of parked registers), laundered in the global
// address space: the loads through it stay global_load (a laundered generic pointer makes them flat loads, which
// also count on lgkmcnt, so every LDS wait after them would wait for their HBM round trip)
__device__ __forceinline__ const float* opaque_ptr(const float* p) {
  auto g = (const __attribute__((address_space(1))) float*)p;
  asm volatile("" : "+v"(g));
  return (const float*)g;
}

__device__ __forceinline__ void zero16(f32x16& a) {
#pragma unroll
  for (int q = 0; q < 16; ++q) a[q] = 0.f;
}

// LayerNorm statistics of a 32-wide act-frag vector (both lane halves get them)
__device__ __forceinline__ void ln32(const float (&v)[16], float& mu, float& rs) {
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) s += v[q];
  mu = xsum(s) / 32.f;
  float d2 = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) d2 = fmaf(v[q] - mu, v[q] - mu, d2);
  rs = 1.0f / sqrtf(xsum(d2) / 32.f + kLnEps);
}
// LayerNorm backward (trunk.h ln_bwd) of act-frag dy with normalised input xh, LN weight w (LDS)
__device__ __forceinline__ void ln32_bwd(const float (&dy)[16], const float (&xh)[16], float rs, const float* w,
                                         float (&dx)[16]) {
  const int h = lane_h();
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float g = dy[q] * w[kperm(q, h)];
    sg += g;
    sgx = fmaf(g, xh[q], sgx);
  }
  sg = xsum(sg) / 32.f;
  sgx = xsum(sgx) / 32.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) dx[q] = rs * (dy[q] * w[kperm(q, h)] - sg - xh[q] * sgx);
}

// value of LDS image offset e (< Geo::scr) from the net's flat MGeo parameters
template <int D, int O>
__device__ __forceinline__ float stage_value(const float* __restrict__ P, int e) {
  using G = Geo<D, O>;
  using F = MGeo<D, H, O>;
  float v = 0.f;
  if (e < G::W2) {
    const int m = e / G::P1, k = e - m * G::P1;
    if (k < D) v = P[F::W1 + m * F::Dp + k];
  } else if (e < G::Wih) {
    const int r = e - G::W2, m = r / G::PW, k = r - m * G::PW;
    if (k < H) v = P[F::W2 + m * H + k];
  } else if (e < G::Whh) {
    const int r = e - G::Wih, m = r / G::PW, k = r - m * G::PW;
    if (k < H) v = P[F::Wih + m * H + k];
  } else if (e < G::WihT) {
    const int r = e - G::Whh, m = r / G::PW, k = r - m * G::PW;
    if (k < H) v = P[F::Whh + m * H + k];
  } else if (e < G::WhhT) {
    const int r = e - G::WihT, i = r / G::PT, j = r - i * G::PT;
    if (j < 3 * H) v = P[F::Wih + j * H + i];
  } else if (e < G::ln0w) {
    const int r = e - G::WhhT, i = r / G::PT, j = r - i * G::PT;
    if (j < 3 * H) v = P[F::Whh + j * H + i];
  } else if (e < G::ln0b) {
    const int k = e - G::ln0w;
    if (k < D) v = P[F::ln0_w + k];
  } else if (e < G::b1) {
    const int k = e - G::ln0b;
    if (k < D) v = P[F::ln0_b + k];
  } else if (e < G::bih) {
    const int r = e - G::b1, seg = r >> 5, i = r & 31;
    const int src[6] = {F::b1, F::ln1_w, F::ln1_b, F::b2, F::ln2_w, F::ln2_b};
    v = P[src[seg] + i];
  } else if (e < G::lnrw) {
    const int r = e - G::bih;
    v = r < 96 ? P[F::bih + r] : P[F::bhh + r - 96];
  } else if (e < G::Wo) {
    const int r = e - G::lnrw;
    v = r < 32 ? P[F::lnr_w + r] : P[F::lnr_b + r - 32];
  } else if (e < G::bo) {
    const int r = e - G::Wo, o = r >> 5, i = r & 31;
    if (o < O) v = P[F::Wo + o * H + i];
  } else {
    const int o = e - G::bo;
    if (o < O) v = P[F::bo + o];
  }
  return v;
}

// obs row -> DT act-frag tiles (feature 32 t + kperm(q, h); zero beyond D)
template <int D, int DT>
__device__ __forceinline__ void load_obs(const float* __restrict__ orow, float (&x)[DT][16]) {
  const int h = lane_h();
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int f = 32 * t + kperm(q, h);
      const float v = orow[f < D ? f : D - 1];
      x[t][q] = f < D ? v : 0.f;
    }
}

template <int D, int DT>
__device__ __forceinline__ void ln0_stats(const float (&x)[DT][16], float& mu, float& rs) {
  const int h = lane_h();
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) s += x[t][q];
  mu = xsum(s) / (float)D;
  float d2 = 0.f;
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float d = 32 * t + kperm(q, h) < D ? x[t][q] - mu : 0.f;
      d2 = fmaf(d, d, d2);
    }
  rs = 1.0f / sqrtf(xsum(d2) / (float)D + kLnEps);
}

// Offsets of the MLP's LayerNorm / bias vectors relative to ln0w (the same in both LDS images)
template <int D>
struct LnOff {
  static constexpr int DPT = 32 * ((D + 31) / 32);
  static constexpr int ln0w = 0, ln0b = DPT, b1 = 2 * DPT, ln1w = b1 + 32, ln1b = ln1w + 32, b2 = ln1b + 32,
                       ln2w = b2 + 32, ln2b = ln2w + 32;
};

// LN0 -> L1 -> ReLU -> LN1 -> L2 -> ReLU (-> LN2 statistics) of one row tile in act-frag. W1 / W2: the padded
// LDS rows (pitches P1 / PW); lv: the LayerNorm / bias vectors (LnOff).
template <int D, int O>
struct Mlp {
  using G = Geo<D, O>;
  using LO = LnOff<D>;
  static constexpr int DT = G::DT;
  float mu0, rs0, a1[16], mu1, rs1, a2[16], mu2, rs2;

  __device__ __forceinline__ void run(const float* W1, const float* W2, const float* lv, const float* __restrict__ orow) {
    const int h = lane_h();
    float x[DT][16];
    load_obs<D, DT>(orow, x);
    ln0_stats<D, DT>(x, mu0, rs0);
    f32x16 acc;
    zero16(acc);
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      float f0[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int f = 32 * t + kperm(q, h);
        f0[q] = (x[t][q] - mu0) * rs0 * lv[LO::ln0w + f] + lv[LO::ln0b + f];
      }
      mm_rows<G::P1>(W1 + 32 * t, f0, acc, kgroups(D - 32 * t));
    }
    float f[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) a1[q] = fmaxf(acc[q] + lv[LO::b1 + kperm(q, h)], 0.f);
    ln32(a1, mu1, rs1);
#pragma unroll
    for (int q = 0; q < 16; ++q) f[q] = (a1[q] - mu1) * rs1 * lv[LO::ln1w + kperm(q, h)] + lv[LO::ln1b + kperm(q, h)];
    zero16(acc);
    mm_rows<G::PW>(W2, f, acc);
#pragma unroll
    for (int q = 0; q < 16; ++q) a2[q] = fmaxf(acc[q] + lv[LO::b2 + kperm(q, h)], 0.f);
    ln32(a2, mu2, rs2);
  }
  // x2 = LN2(a2)
  __device__ __forceinline__ void x2(const float* lv, float (&o)[16]) const {
    const int h = lane_h();
#pragma unroll
    for (int q = 0; q < 16; ++q) o[q] = (a2[q] - mu2) * rs2 * lv[LO::ln2w + kperm(q, h)] + lv[LO::ln2b + kperm(q, h)];
  }
};

// GRU cell (torch gate order r, z, n; h' = n + z (h - n)) of one row tile from x2 and the input hidden
template <int D, int O>
struct Gru {
  using G = Geo<D, O>;
  float r[16], z[16], n[16], ghn[16], h2[16];

  __device__ __forceinline__ void run(const float* sm, const float (&x2)[16], const float (&hin)[16]) {
    const int h = lane_h();
    f32x16 ai, ah;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      zero16(ai);
      zero16(ah);
      mm_rows<G::PW>(sm + G::Wih + 32 * g * G::PW, x2, ai);
      mm_rows<G::PW>(sm + G::Whh + 32 * g * G::PW, hin, ah);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int j = 32 * g + kperm(q, h);
        const float gi = ai[q] + sm[G::bih + j], gh = ah[q] + sm[G::bhh + j];
        if (g == 0) r[q] = sigmoidf_(gi + gh);
        if (g == 1) z[q] = sigmoidf_(gi + gh);
        if (g == 2) {
          ghn[q] = gh;
          n[q] = tanhf_(gi + r[q] * gh);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) h2[q] = n[q] + z[q] * (hin[q] - n[q]);
  }
};

struct GradArgs {
  mm_mappo_bwd_args a;
  const float* h_in[2];
  float* hseq;      // [2][NB * GW][2][L][64 * 16]: input hidden and GRU input x2 of every step of the wave's tile
  float* dx2;       // [2][T * EN][32]: d loss / d x2 of every row-step (pass G -> pass M)
  float* partial;   // [2][2 NB][pstride]: pass G blocks, then pass M blocks
  int64_t pstride;
};

// store an act-frag vector as row `row` of a [rows][32] array: features 8 j + 4 h + 0..3 are 4 consecutive floats
__device__ __forceinline__ void st_row32(float* base, int64_t row, const float (&v)[16]) {
  float* p = base + row * 32 + 4 * lane_h();
#pragma unroll
  for (int j = 0; j < 4; ++j)
    *reinterpret_cast<float4*>(p + 8 * j) = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
}
__device__ __forceinline__ void ld_row32(const float* base, int64_t row, float (&v)[16]) {
  const float* p = base + row * 32 + 4 * lane_h();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 t = *reinterpret_cast<const float4*>(p + 8 * j);
    v[4 * j] = t.x;
    v[4 * j + 1] = t.y;
    v[4 * j + 2] = t.z;
    v[4 * j + 3] = t.w;
  }
}

// ---------------------------------------------------------------- fp16x3 products of pass G
// Every fp32 product of pass G runs as three v_mfma_f32_32x32x16_f16 (Wl·xh + Wh·xl + Wh·xh, fp32 accumulate; Wh =
// f16(W), Wl = f16(W - Wh), the same for x): 6 MFMAs of 32 cycles for a 32 x 32 x 32 block instead of 16
// v_mfma_f32_32x32x2_f32 of 64 cycles (5.3x less matrix-pipe time). Both operands are scaled by powers of two
// before the split so that their largest magnitude lies in [2^13, 2^14): the weight image by one factor per image (its
// max |W|), the vector operand of a W x product by one factor per column (a column of the MFMA's result depends on
// that column's operand only: the max over the row's two lanes, unscaled per lane), the operands of a weight gradient
// (rows summed over the k dimension) by one factor per wave tile. Then every operand within 2^-16 of its scale's max
// has normal f16 hi and lo parts, hi + lo represents it to 2^-24 relative, and the
// dropped Wl·xl term is ~2^-24 relative: fp32-level products relative to the tile's largest terms (smaller operands
// carry an absolute error below 2^-38 of the max). Results are unscaled by the exact inverse powers of two;
// weight-gradient blocks, whose operand scales change from tile to tile, accumulate into a temporary tile that is
// unscaled into the running accumulator (running scales that are only lowered measured both slower — the rescale
// paths spill — and, where a late tile's values sit far below the running max, outside the fp32 bars).
// The act-frag layout carries over: MFMA block j (k-steps s in [8 j, 8 j + 8)) takes lane (c, h)'s v[8 j .. 8 j + 7]
// as its B operand (features kperm(s, h)), and the weight images hold, per 32 x 32 block, lane (i, h)'s A operand
// W[i][kperm(8 j + e, h)] for e < 8 as f16 hi / lo pieces ([j][hi | lo][lane][8 halves], one ds_read_b128 each).
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef _Float16 h2v_ __attribute__((ext_vector_type(2)));
typedef float f2v_ __attribute__((ext_vector_type(2)));
struct S16 {
  h8v h[2], l[2];
};
__device__ __forceinline__ void split16(const float (&v)[16], S16& o) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const f2v_ x = {v[8 * j + 2 * p], v[8 * j + 2 * p + 1]};
      hw[p] = __builtin_bit_cast(uint32_t, __builtin_convertvector(x, h2v_));
      uint32_t lo;   // lo = f16(x - hi): the residual is exact in f32, rounded once (v_fma_mixlo / mixhi)
      asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hw[p]), "v"(x.x));
      asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hw[p]), "v"(x.y));
      lw[p] = lo;
    }
    o.h[j] = __builtin_bit_cast(h8v, hw);
    o.l[j] = __builtin_bit_cast(h8v, lw);
  }
}
__device__ __forceinline__ f32x16 mf16(const h8v& a, const h8v& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
constexpr int HBLK = 1024;   // floats per split 32 x 32 block
// acc += W v over the first nj 16-deep k blocks (W: the split block at LDS float offset blk)
__device__ __forceinline__ void mmh(const float* blk, const S16& v, f32x16& acc, int nj = 2) {
  const int lane = (int)(threadIdx.x & 63);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j >= nj) break;
    const h8v ah = *reinterpret_cast<const h8v*>(blk + (2 * j * 64 + lane) * 4);
    const h8v al = *reinterpret_cast<const h8v*>(blk + ((2 * j + 1) * 64 + lane) * 4);
    acc = mf16(al, v.h[j], acc);
    acc = mf16(ah, v.l[j], acc);
    acc = mf16(ah, v.h[j], acc);
  }
}
// weight-gradient accumulation, chunks on k: acc[i][n] += sum_k a[i][k] b[n][k] (a, b: transposed tiles, tget)
__device__ __forceinline__ void accg(f32x16& acc, const S16& a, const S16& b) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    acc = mf16(a.l[j], b.h[j], acc);
    acc = mf16(a.h[j], b.l[j], acc);
    acc = mf16(a.h[j], b.h[j], acc);
  }
}
// the power of two that brings a max magnitude m into [2^13, 2^14) (1 for m = 0)
__device__ __forceinline__ float scale_for(float m) {
  int e = 0;
  (void)frexpf(m, &e);
  return m > 0.f ? ldexpf(1.0f, 14 - e) : 1.0f;
}
__device__ __forceinline__ float absmax16(const float (&v)[16], float m = 0.f) {
#pragma unroll
  for (int q = 0; q < 16; ++q) m = fmaxf(m, fabsf(v[q]));
  return m;
}
// the wave-wide max of per-lane values >= 0 (DPP within each row of 16, then v_permlane16 / 32 swaps; no LDS)
template <int CTRL>
__device__ __forceinline__ float dpp_max(float m) {
  const int o = __builtin_amdgcn_update_dpp(0, __float_as_int(m), CTRL, 0xF, 0xF, false);
  return fmaxf(m, __int_as_float(o));
}
__device__ __forceinline__ float wave_max(float m) {
  m = dpp_max<0xB1>(m);    // quad_perm [1, 0, 3, 2]
  m = dpp_max<0x4E>(m);    // quad_perm [2, 3, 0, 1]
  m = dpp_max<0x141>(m);   // row_half_mirror
  m = dpp_max<0x140>(m);   // row_mirror
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  m = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// the max over the two lanes of one act-frag column (chunk c: lanes c and c + 32)
__device__ __forceinline__ float col_max(float m) {
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// split of x * s (s: a power of two)
__device__ __forceinline__ void split16s(const float (&v)[16], float s, S16& o) {
  float x[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) x[q] = v[q] * s;
  split16(x, o);
}
// running += tmp * inv (a weight-gradient block unscaled into its accumulator)
__device__ __forceinline__ void acc_unscale(f32x16& run, const f32x16& tmp, float inv) {
#pragma unroll
  for (int q = 0; q < 16; ++q) run[q] = fmaf(tmp[q], inv, run[q]);
}

// Pass G's LDS image: the split blocks of W1 (DT blocks), W2, W_ih (3 gate blocks), W_hh (3), W_ih^T (3: block g = the
// gate-g columns), W_hh^T (3), then the f32 LayerNorm / bias / head vectors (Geo's ln0w .. bo block, same relative
// offsets), then the wave transpose tiles (offsets in floats)
template <int D, int O>
struct GeoH {
  using G = Geo<D, O>;
  static constexpr int DT = G::DT;
  static constexpr int W1 = 0, W2 = W1 + DT * HBLK, Wih = W2 + HBLK, Whh = Wih + 3 * HBLK, WihT = Whh + 3 * HBLK,
                       WhhT = WihT + 3 * HBLK, vec = WhhT + 3 * HBLK, nblk = vec / HBLK;
  static constexpr int v(int g_off) { return vec + (g_off - G::ln0w); }   // a Geo vector offset in this image
  static constexpr int ln0w = vec, bih = vec + (G::bih - G::ln0w), bhh = vec + (G::bhh - G::ln0w),
                       lnrw = vec + (G::lnrw - G::ln0w), lnrb = vec + (G::lnrb - G::ln0w),
                       Wo = vec + (G::Wo - G::ln0w), bo = vec + (G::bo - G::ln0w);
  // scales (f32): [0] the weight image's, then the static scales of the LayerNorm outputs the products read, from
  // their bounds |LN(x) w + b| <= sqrt(n - 1) max|w| + max|b| (a normalised n-vector has no entry beyond
  // sqrt(n - 1)): [1] f0 = LN0, [2] f1 = LN1, [3] x2 = LN2, [4] y = LN_r; the GRU hidden states (|h| < 1) use 2^14
  static constexpr int wsc = vec + (G::scr - G::ln0w);
  static constexpr int scr = wsc + 8, total = scr + GW * GT * TILE;
};
// Pass M's LDS image: the split blocks of W1 (DT), W2, W2^T, W1^T (DT: block t = the columns 32 t .. 32 t + 31 of W1),
// the f32 LayerNorm / bias vectors of the MLP (ln0w .. ln2b, LnOff offsets), the scales (GeoH's wsc slots), then the
// wave transpose tiles. W1 / W2 / the vectors sit at GeoH's offsets, so the forward (MlpH) reads either image.
template <int D, int O>
struct GeoM {
  using G = Geo<D, O>;
  static constexpr int DT = G::DT;
  static constexpr int W1 = 0, W2 = W1 + DT * HBLK, W2T = W2 + HBLK, W1T = W2T + HBLK, vec = W1T + DT * HBLK,
                       nblk = vec / HBLK, ln0w = vec, wsc = vec + (G::bih - G::ln0w), scr = wsc + 8;
  // waves per block: 8 (2 per SIMD) where the registers allow it (DT <= 2) and the tiles fit the 160 KB of LDS
  static constexpr int MW = (DT <= 2 && (scr + 8 * MT * TILE) * 4 <= 160 * 1024) ? 8 : 4;
  static constexpr int total = scr + MW * MT * TILE;
};
static_assert(GeoH<47, 5>::W2 == GeoM<47, 5>::W2 && GeoH<94, 5>::W2 == GeoM<94, 5>::W2, "W1 / W2 offsets");

// W of split block b at (row i, column k) from the flat MGeo parameters (MI: pass M's image, else pass G's)
template <int D, int O, bool MI>
__device__ __forceinline__ float hblk_value(const float* __restrict__ P, int b, int i, int k) {
  using GH = GeoH<D, O>;
  using F = MGeo<D, H, O>;
  constexpr int DT = GH::DT;
  if (b < DT) {
    const int kk = 32 * b + k;
    return kk < D ? P[F::W1 + i * F::Dp + kk] : 0.f;
  }
  b -= DT;
  if (b == 0) return P[F::W2 + i * H + k];
  b -= 1;
  if constexpr (MI) {
    if (b == 0) return P[F::W2 + k * H + i];   // W2^T
    b -= 1;
    const int kk = 32 * b + i;                 // W1^T, columns 32 b ..
    return kk < D ? P[F::W1 + k * F::Dp + kk] : 0.f;
  }
  if (b < 3) return P[F::Wih + (32 * b + i) * H + k];
  b -= 3;
  if (b < 3) return P[F::Whh + (32 * b + i) * H + k];
  b -= 3;
  if (b < 3) return P[F::Wih + (32 * b + k) * H + i];   // W_ih^T, gate-b columns
  b -= 3;
  return P[F::Whh + (32 * b + k) * H + i];              // W_hh^T
}
// stage a split image (MI: pass M's GeoM, else pass G's GeoH) and its scales
template <int D, int O, bool MI>
__device__ void stage_h(float* sm, const float* __restrict__ P) {
  using GH = std::conditional_t<MI, GeoM<D, O>, GeoH<D, O>>;
  // the image's weight scale: max |W| over the staged matrices (every entry of a block is one (b, i, k))
  float m = 0.f;
  for (int x = threadIdx.x; x < GH::nblk * 1024; x += blockDim.x)
    m = fmaxf(m, fabsf(hblk_value<D, O, MI>(P, x >> 10, (x >> 5) & 31, x & 31)));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) sm[GH::wsc + (threadIdx.x >> 6)] = m;   // (<= 8 waves: the 8 scale slots)
  __syncthreads();
  float mw = 0.f;
  for (int ww = 0; ww < (int)(blockDim.x >> 6); ++ww) mw = fmaxf(mw, sm[GH::wsc + ww]);
  const float sw = scale_for(mw);
  __syncthreads();
  if (threadIdx.x == 0) sm[GH::wsc] = sw;
  if (threadIdx.x < 64) {   // the LayerNorm output bounds (wave 0)
    using F = MGeo<D, H, O>;
    const int l = threadIdx.x;
    float w0 = 0.f, b0 = 0.f;
    for (int k = l; k < D; k += 64) {
      w0 = fmaxf(w0, fabsf(P[F::ln0_w + k]));
      b0 = fmaxf(b0, fabsf(P[F::ln0_b + k]));
    }
    const float w1 = l < 32 ? fabsf(P[F::ln1_w + l]) : 0.f, b1 = l < 32 ? fabsf(P[F::ln1_b + l]) : 0.f;
    const float w2 = l < 32 ? fabsf(P[F::ln2_w + l]) : 0.f, b2 = l < 32 ? fabsf(P[F::ln2_b + l]) : 0.f;
    const float wr = l < 32 ? fabsf(P[F::lnr_w + l]) : 0.f, br = l < 32 ? fabsf(P[F::lnr_b + l]) : 0.f;
    const float s31 = sqrtf(31.f);
    const float B0 = sqrtf((float)(D - 1)) * wave_max(w0) + wave_max(b0), B1 = s31 * wave_max(w1) + wave_max(b1);
    const float B2 = s31 * wave_max(w2) + wave_max(b2), Br = s31 * wave_max(wr) + wave_max(br);
    if (l == 0) {
      sm[GH::wsc + 1] = scale_for(B0 * 1.0001f);   // (headroom for the bound's own rounding)
      sm[GH::wsc + 2] = scale_for(B1 * 1.0001f);
      sm[GH::wsc + 3] = scale_for(B2 * 1.0001f);
      sm[GH::wsc + 4] = scale_for(Br * 1.0001f);
    }
  }
  _Float16* hs = reinterpret_cast<_Float16*>(sm);
  for (int x = threadIdx.x; x < GH::nblk * 2 * HBLK; x += blockDim.x) {   // halves
    const int b = x / (2 * HBLK), r = x % (2 * HBLK);
    const int jp = r / 512, l = (r % 512) / 8, e8 = r % 8;
    const int j = jp >> 1, part = jp & 1, i = l & 31, hh = l >> 5;
    const float w = hblk_value<D, O, MI>(P, b, i, kperm(8 * j + e8, hh)) * sw;
    const _Float16 hi = (_Float16)w;
    hs[x] = part ? (_Float16)(w - (float)hi) : hi;
  }
  for (int e = threadIdx.x; e < GH::wsc - GH::vec; e += blockDim.x)
    sm[GH::vec + e] = stage_value<D, O>(P, Geo<D, O>::ln0w + e);
  __syncthreads();
}

// LN0 -> L1 -> ReLU -> LN1 -> L2 -> ReLU (-> LN2 statistics) of one row tile on a split image (GI: GeoH or GeoM; both
// hold W1 / W2 / the MLP vectors / the scales at the same places): Mlp's arithmetic with fp16x3 products
template <int D, class GI>
struct MlpH {
  using LO = LnOff<D>;
  static constexpr int DT = GI::DT;
  float mu0, rs0, a1[16], mu1, rs1, a2[16], mu2, rs2;

  __device__ __forceinline__ void run(const float* sm, const float* __restrict__ orow) {
    const int h = lane_h();
    const float* lv = sm + GI::ln0w;
    const float sw = sm[GI::wsc];
    float x[DT][16];
    load_obs<D, DT>(orow, x);
    ln0_stats<D, DT>(x, mu0, rs0);
    f32x16 acc;
    zero16(acc);
    const float s0 = sm[GI::wsc + 1];
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      float f0[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int f = 32 * t + kperm(q, h);
        f0[q] = (x[t][q] - mu0) * rs0 * lv[LO::ln0w + f] + lv[LO::ln0b + f];
      }
      S16 sf;
      split16s(f0, s0, sf);
      mmh(sm + GI::W1 + t * HBLK, sf, acc, kgroups(D - 32 * t) > 2 ? 2 : 1);
    }
    float f[16];
    const float u0 = 1.0f / (sw * s0);
#pragma unroll
    for (int q = 0; q < 16; ++q) a1[q] = fmaxf(acc[q] * u0 + lv[LO::b1 + kperm(q, h)], 0.f);
    ln32(a1, mu1, rs1);
#pragma unroll
    for (int q = 0; q < 16; ++q) f[q] = (a1[q] - mu1) * rs1 * lv[LO::ln1w + kperm(q, h)] + lv[LO::ln1b + kperm(q, h)];
    zero16(acc);
    const float s1 = sm[GI::wsc + 2];
    {
      S16 sf;
      split16s(f, s1, sf);
      mmh(sm + GI::W2, sf, acc);
    }
    const float u1 = 1.0f / (sw * s1);
#pragma unroll
    for (int q = 0; q < 16; ++q) a2[q] = fmaxf(acc[q] * u1 + lv[LO::b2 + kperm(q, h)], 0.f);
    ln32(a2, mu2, rs2);
  }
};
// x2 = LN2(a2) of one row tile on pass G's image (pass G's step 1)
template <int D, int O>
__device__ __forceinline__ void mlp_x2_h(const float* sm, const float* __restrict__ orow, float (&x2)[16]) {
  using LO = LnOff<D>;
  const int h = lane_h();
  const float* lv = sm + GeoH<D, O>::ln0w;
  MlpH<D, GeoH<D, O>> mp;
  mp.run(sm, orow);
#pragma unroll
  for (int q = 0; q < 16; ++q)
    x2[q] = (mp.a2[q] - mp.mu2) * mp.rs2 * lv[LO::ln2w + kperm(q, h)] + lv[LO::ln2b + kperm(q, h)];
}

// GRU cell on the split image (Gru's arithmetic with fp16x3 products)
template <int D, int O>
struct GruH {
  using GH = GeoH<D, O>;
  float r[16], z[16], n[16], ghn[16], h2[16];

  // sx2 / shin: x2 and hin split at their wave scales; ux / uh = 1 / (weight scale x that scale)
  __device__ __forceinline__ void run(const float* sm, const S16& sx2, float ux, const S16& shin, float uh,
                                      const float (&hin)[16]) {
    const int h = lane_h();
    f32x16 ai, ah;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      zero16(ai);
      zero16(ah);
      mmh(sm + GH::Wih + g * HBLK, sx2, ai);
      mmh(sm + GH::Whh + g * HBLK, shin, ah);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int j = 32 * g + kperm(q, h);
        const float gi = ai[q] * ux + sm[GH::bih + j], gh = ah[q] * uh + sm[GH::bhh + j];
        if (g == 0) r[q] = sigmoidf_(gi + gh);
        if (g == 1) z[q] = sigmoidf_(gi + gh);
        if (g == 2) {
          ghn[q] = gh;
          n[q] = tanhf_(gi + r[q] * gh);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) h2[q] = n[q] + z[q] * (hin[q] - n[q]);
  }
};

// ---------------------------------------------------------------- pass G: recurrent part
template <int D, int A, int O>
__device__ void gru_body(const GradArgs& k, int net, float* sm) {
  using GH = GeoH<D, O>;
  using F = MGeo<D, H, O>;
  const mm_mappo_bwd_args& a = k.a;
  stage_h<D, O, false>(sm, a.P[net]);
  const int lane = (int)(threadIdx.x & 63), ci = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // wave-uniform: scalar loop control
  float* S0 = sm + GH::scr + w * GT * TILE;
  float* S1 = S0 + TILE;
  const int L = a.L;
  const int64_t EN = a.en, nch = (int64_t)(a.T / L) * EN, ntile = (nch + 31) / 32;
  const int wg = blockIdx.x * GW + w, nwg = gridDim.x * GW;
  float* hs = k.hseq + ((int64_t)net * nwg + wg) * 2 * L * 1024 + lane * 16;   // input hiddens, then x2
  float* xs = hs + L * 1024;
  float* dx2o = k.dx2 + (int64_t)net * a.T * EN * 32;
  const float* __restrict__ hin0 = k.h_in[net];
  const float inv_m = 1.0f / a.stats[MM_MST_ACTIVE_SUM];

  f32x16 aWih[3], aWhh[3], aWo;
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    zero16(aWih[g]);
    zero16(aWhh[g]);
  }
  zero16(aWo);
  float sbr = 0.f, sbz = 0.f, sbn = 0.f, sbhn = 0.f, sbo = 0.f, slrw = 0.f, slrb = 0.f;
  float lsum0 = 0.f, lsum1 = 0.f, lsum2 = 0.f;

  for (int64_t tile = wg; tile < ntile; tile += nwg) {
    const int64_t c = tile * 32 + ci;
    const bool valid = c < nch;
    const int64_t cc = valid ? c : 0, kc = cc / EN, en = cc - kc * EN;
    // ---- step 1: forward over the chunk, input hidden of every step kept in the wave scratch
    float hc[16];
    {
      const float* hp = hin0 + ((kc * L) * EN + en) * H + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 v = *reinterpret_cast<const float4*>(hp + 8 * g);
        hc[4 * g] = v.x;
        hc[4 * g + 1] = v.y;
        hc[4 * g + 2] = v.z;
        hc[4 * g + 3] = v.w;
      }
    }
    for (int l = 0; l < L; ++l) {
      const int64_t row = (kc * L + l) * EN + en;
      const float m = a.mask[row];
#pragma unroll
      for (int q = 0; q < 16; ++q) hc[q] *= m;
      st16(hs + l * 1024, hc);
      const float* smo = sm + opaque0();
      float x2[16];
      mlp_x2_h<D, O>(smo, a.obs + row * D, x2);
      st16(xs + l * 1024, x2);         // the GRU input of every step, for step 2 (no MLP recompute there)
      if (l + 1 < L) {
        GruH<D, O> gr;
        S16 sx, sh;
        const float sw = smo[GH::wsc], s_x = smo[GH::wsc + 3], s_h = 0x1p14f;
        split16s(x2, s_x, sx);
        split16s(hc, s_h, sh);
        gr.run(smo, sx, 1.0f / (sw * s_x), sh, 1.0f / (sw * s_h), hc);
#pragma unroll
        for (int q = 0; q < 16; ++q) hc[q] = gr.h2[q];
      }
    }
    // ---- step 2: backward over the steps, each step's forward recomputed from its input hidden
    float dhn[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) dhn[q] = 0.f;
    for (int l = L - 1; l >= 0; --l) {
      const int64_t row = (kc * L + l) * EN + en;
      const float* smb = sm + opaque0();
      float hin[16], x2[16];
      ld16(opaque_ptr(hs + l * 1024), hin);
      ld16(opaque_ptr(xs + l * 1024), x2);
      __builtin_amdgcn_sched_barrier(0);
      GruH<D, O> st;
      const float sw = smb[GH::wsc];
      const float s_x = smb[GH::wsc + 3], s_h = 0x1p14f;   // (the static scales of x2 and the hidden state)
      {
        S16 sx, sh;
        split16s(x2, s_x, sx);
        split16s(hin, s_h, sh);
        st.run(smb, sx, 1.0f / (sw * s_x), sh, 1.0f / (sw * s_h), hin);
      }
      // head: y = LN_r(h2); out = Wo y + bo
      float mur, rsr, xr[16], y[16];
      ln32(st.h2, mur, rsr);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        xr[q] = (st.h2[q] - mur) * rsr;
        y[q] = xr[q] * smb[GH::lnrw + kperm(q, h)] + smb[GH::lnrb + kperm(q, h)];
      }
      float out[O];
#pragma unroll
      for (int o = 0; o < O; ++o) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) s = fmaf(smb[GH::Wo + o * 32 + kperm(q, h)], y[q], s);
        out[o] = smb[GH::bo + o] + xsum(s);
      }
      // ---- loss seed d(out) (mappo.hip bwd_body; ramppo_network.py:56-209)
      const float m = valid ? a.active[row] : 0.f;
      float dout[O];
      if constexpr (O == A) {
        float mx = out[0];
#pragma unroll
        for (int q = 1; q < A; ++q) mx = fmaxf(mx, out[q]);
        float se = 0.f;
#pragma unroll
        for (int q = 0; q < A; ++q) se += expf(out[q] - mx);
        const float lse = mx + logf(se);
        float lp[A], ent = 0.f;
#pragma unroll
        for (int q = 0; q < A; ++q) {
          lp[q] = out[q] - lse;
          ent -= expf(lp[q]) * lp[q];
        }
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
        if (h == 0 && valid) {
          lsum0 += -fminf(s1, s2) * m;
          lsum1 += ent * m;
          lsum2 += ratio;
        }
#pragma unroll
        for (int q = 0; q < A; ++q) {
          const float p = expf(lp[q]);
          dout[q] = dlpa * ((q == act ? 1.0f : 0.0f) - p) + dent * (-p * (lp[q] + ent));
        }
      } else {
        const float v = out[0];
        const float old = a.old_value[row];
        const float tgt = (a.returns[row] - a.stats[MM_MST_VN_MEAN]) / a.stats[MM_MST_VN_STD];
        const float dv = v - old;
        const float vc = old + fminf(fmaxf(dv, -a.clip), a.clip);
        const float eo = tgt - v, ec = tgt - vc;
        const float hd = a.huber_delta;
        const float lo = fabsf(eo) <= hd ? eo * eo * 0.5f : hd * (fabsf(eo) - hd * 0.5f);
        const float lc = fabsf(ec) <= hd ? ec * ec * 0.5f : hd * (fabsf(ec) - hd * 0.5f);
        const float go = -(fabsf(eo) <= hd ? eo : (eo > 0.f ? hd : -hd));
        const float gc =
            -(fabsf(ec) <= hd ? ec : (ec > 0.f ? hd : -hd)) * ((dv >= -a.clip && dv <= a.clip) ? 1.0f : 0.0f);
        const float d = lo > lc ? go : (lc > lo ? gc : 0.5f * (go + gc));
        dout[0] = a.value_coef * m * inv_m * d;
        if (h == 0 && valid) lsum0 += fmaxf(lo, lc) * m;
      }
      // ---- head gradients: dWo = dout y^T, dbo = dout (MFMA with chunks on k); dy = Wo^T dout
      float dy[16];
      {
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int o = kperm(q, h);
          float d = 0.f, s = 0.f;
#pragma unroll
          for (int oo = 0; oo < O; ++oo) {
            if (oo == o) d = dout[oo];
            s = fmaf(smb[GH::Wo + oo * 32 + o], dout[oo], s);
          }
          v[q] = d;
          dy[q] = s;
        }
        tput(S0, v);
        tput(S1, y);
        wave_fence();
        float At[16], Bt[16];
        tget(S0, At);
        tget(S1, Bt);
        {
          const float s_a = scale_for(wave_max(absmax16(At))), s_b = smb[GH::wsc + 4];
          S16 sa, sb;
          split16s(At, s_a, sa);
          split16s(Bt, s_b, sb);
          f32x16 tmp;
          zero16(tmp);
          accg(tmp, sa, sb);
          acc_unscale(aWo, tmp, 1.0f / (s_a * s_b));
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) sbo += At[s];
        wave_fence();
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = dy[q] * xr[q];
        tput(S0, v);
        tput(S1, dy);
        wave_fence();
        slrw += tsum(S0);
        slrb += tsum(S1);
        wave_fence();
      }
      // LN_r backward -> d h2 (+ the gradient carried from the next step)
      float dh[16];
      ln32_bwd(dy, xr, rsr, smb + GH::lnrw, dh);
      // ---- GRU backward (h2 = n + z (hin - n); gates r, z, n)
      float dgr[16], dgz[16], dpn[16], dghn[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float d = dh[q] + dhn[q];
        const float r = st.r[q], z = st.z[q], n = st.n[q];
        const float dn = d * (1.0f - z);
        const float dz = d * (hin[q] - n);
        dpn[q] = dn * (1.0f - n * n);
        dgr[q] = dpn[q] * st.ghn[q] * r * (1.0f - r);
        dgz[q] = dz * z * (1.0f - z);
        dghn[q] = dpn[q] * r;
        dhn[q] = d * z;
      }
      // one column scale for the four gate deltas (the dx2 / dhh products), their wave scale for the weight gradients
      const float md = absmax16(dghn, absmax16(dpn, absmax16(dgz, absmax16(dgr))));
      const float c_d = scale_for(col_max(md)), s_d = scale_for(wave_max(md));
      const float u_d = 1.0f / (sw * c_d);
      S16 sgr, sgz;
      split16s(dgr, c_d, sgr);
      split16s(dgz, c_d, sgz);
      {
        // d x2 = W_ih^T dgates -> the MLP pass
        f32x16 dx2;
        zero16(dx2);
        S16 spn;
        split16s(dpn, c_d, spn);
        mmh(smb + GH::WihT, sgr, dx2);
        mmh(smb + GH::WihT + HBLK, sgz, dx2);
        mmh(smb + GH::WihT + 2 * HBLK, spn, dx2);
        if (valid) {
          float v[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] = dx2[q] * u_d;
          st_row32(dx2o, row, v);
        }
      }
      {
        f32x16 dhh;
        zero16(dhh);
        S16 shn;
        split16s(dghn, c_d, shn);
        mmh(smb + GH::WhhT, sgr, dhh);
        mmh(smb + GH::WhhT + HBLK, sgz, dhh);
        mmh(smb + GH::WhhT + 2 * HBLK, shn, dhh);
        const float mk = a.mask[row];
#pragma unroll
        for (int q = 0; q < 16; ++q) dhn[q] = (dhn[q] + dhh[q] * u_d) * mk;
      }
      // GRU weight gradients: dW_ih += dg x2^T, dW_hh += dgh hin^T, gate biases (two transpose tiles)
      {
        float XT[16], HT[16];
        tput(S0, x2);
        tput(S1, hin);
        wave_fence();
        tget(S0, XT);
        tget(S1, HT);
        wave_fence();
        // (XT / HT hold x2 / hin transposed: the same values, the same wave scales)
        S16 sXT, sHT;
        split16s(XT, s_x, sXT);
        split16s(HT, s_h, sHT);
        const float u_dx = 1.0f / (s_d * s_x), u_dh = 1.0f / (s_d * s_h);
        f32x16 tmp;
        tput(S0, dgr);
        tput(S1, dgz);
        wave_fence();
        {
          float R[16], Z[16];
          tget(S0, R);
          tget(S1, Z);
          S16 sR, sZ;
          split16s(R, s_d, sR);
          split16s(Z, s_d, sZ);
          zero16(tmp);
          accg(tmp, sR, sXT);
          acc_unscale(aWih[0], tmp, u_dx);
          zero16(tmp);
          accg(tmp, sR, sHT);
          acc_unscale(aWhh[0], tmp, u_dh);
          zero16(tmp);
          accg(tmp, sZ, sXT);
          acc_unscale(aWih[1], tmp, u_dx);
          zero16(tmp);
          accg(tmp, sZ, sHT);
          acc_unscale(aWhh[1], tmp, u_dh);
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            sbr += R[s];
            sbz += Z[s];
          }
        }
        wave_fence();
        tput(S0, dpn);
        tput(S1, dghn);
        wave_fence();
        {
          float Nn[16], Nh[16];
          tget(S0, Nn);
          tget(S1, Nh);
          S16 sN, sH2;
          split16s(Nn, s_d, sN);
          split16s(Nh, s_d, sH2);
          zero16(tmp);
          accg(tmp, sN, sXT);
          acc_unscale(aWih[2], tmp, u_dx);
          zero16(tmp);
          accg(tmp, sH2, sHT);
          acc_unscale(aWhh[2], tmp, u_dh);
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            sbn += Nn[s];
            sbhn += Nh[s];
          }
        }
        wave_fence();
      }
    }
  }

  // ---- loss sums (logging only, train_info): one atomic per wave
  if (a.loss_acc) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lsum0 += __shfl_xor(lsum0, o);
      lsum1 += __shfl_xor(lsum1, o);
      lsum2 += __shfl_xor(lsum2, o);
    }
    if (lane == 0) {
      if constexpr (O == A) {
        atomicAdd(&a.loss_acc[MM_MLOSS_POLICY], lsum0 * inv_m);
        atomicAdd(&a.loss_acc[MM_MLOSS_ENTROPY], lsum1 * inv_m);
        atomicAdd(&a.loss_acc[MM_MLOSS_RATIO], lsum2);
      } else {
        atomicAdd(&a.loss_acc[MM_MLOSS_VALUE], lsum0 * inv_m);
      }
    }
  }

  // ---- block reduction of the waves (fixed order) into the flat gradient layout, one partial
  __syncthreads();
  float* red = sm;
  for (int e = threadIdx.x; e < F::total; e += blockDim.x) red[e] = 0.f;
  sbr = xsum(sbr);
  sbz = xsum(sbz);
  sbn = xsum(sbn);
  sbhn = xsum(sbhn);
  sbo = xsum(sbo);
  slrw = xsum(slrw);
  slrb = xsum(slrb);
  __syncthreads();
  for (int ww = 0; ww < GW; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int mm = kperm(q, h);
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          red[F::Wih + (32 * g + mm) * H + ci] += aWih[g][q];
          red[F::Whh + (32 * g + mm) * H + ci] += aWhh[g][q];
        }
        if (mm < O) red[F::Wo + mm * H + ci] += aWo[q];
      }
      if (h == 0) {
        red[F::bih + ci] += sbr;
        red[F::bih + 32 + ci] += sbz;
        red[F::bih + 64 + ci] += sbn;
        red[F::bhh + ci] += sbr;
        red[F::bhh + 32 + ci] += sbz;
        red[F::bhh + 64 + ci] += sbhn;
        red[F::lnr_w + ci] += slrw;
        red[F::lnr_b + ci] += slrb;
        if (ci < O) red[F::bo + ci] += sbo;
      }
    }
    __syncthreads();
  }
  float* outp = k.partial + ((int64_t)net * 2 * NB + blockIdx.x) * k.pstride;
  for (int e = threadIdx.x; e < F::total; e += blockDim.x) outp[e] = red[e];
}

// ---------------------------------------------------------------- pass M: LN-MLP backward, row-parallel
// One wave = 32 row-steps (rows on the MFMA's N), fp16x3 products on pass M's split image: the forward (MlpH), then
// dW2 / db2 / LN2 parameters from d x2 (pass G's output), dx1 = W2^T da2 -> LN1 backward, dW1 / db1, df0 = W1^T da1 ->
// LN0 parameters. Weight-gradient operands are transposed through 3 LDS tiles per wave (chunks on k); the vector
// operands of the W^T products take one scale per column (row), those of the weight gradients one per wave tile.
template <int D, int O>
__device__ void mlp_body(const GradArgs& k, int net, float* sm) {
  using GM = GeoM<D, O>;
  using F = MGeo<D, H, O>;
  using LO = LnOff<D>;
  constexpr int DT = GM::DT;
  const mm_mappo_bwd_args& a = k.a;
  stage_h<D, O, true>(sm, a.P[net]);
  const int lane = (int)(threadIdx.x & 63), ci = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  float* S0 = sm + GM::scr + w * MT * TILE;
  float* S1 = S0 + TILE;
  float* S2 = S1 + TILE;
  const int64_t R = (int64_t)a.T * a.en, ntile = (R + 31) / 32;
  constexpr int MWV = GM::MW;
  const int wg = blockIdx.x * MWV + w, nwg = gridDim.x * MWV;
  const float* dx2i = k.dx2 + (int64_t)net * R * 32;

  f32x16 aW2, aW1[DT];
  zero16(aW2);
#pragma unroll
  for (int t = 0; t < DT; ++t) zero16(aW1[t]);
  float sb2 = 0.f, sb1 = 0.f, sl2w = 0.f, sl2b = 0.f, sl1w = 0.f, sl1b = 0.f, sl0w[DT], sl0b[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) sl0w[t] = sl0b[t] = 0.f;

  for (int64_t tile = wg; tile < ntile; tile += nwg) {
    const int64_t r = tile * 32 + ci;
    const bool valid = r < R;
    const int64_t row = valid ? r : R - 1;
    const float* smb = sm + opaque0();
    const float* lv = smb + GM::ln0w;
    const float sw = smb[GM::wsc], s_f0 = smb[GM::wsc + 1], s_f1 = smb[GM::wsc + 2];
    float dxv[16];
    ld_row32(dx2i, row, dxv);
    if (!valid) {
#pragma unroll
      for (int q = 0; q < 16; ++q) dxv[q] = 0.f;
    }
    MlpH<D, GM> mp;
    mp.run(smb, a.obs + row * D);
    // ---- LN2 backward (x2 = LN2(a2), a2 = relu(W2 f1 + b2)); f1 = LN1(a1)
    float da[16], xh[16], tt[16], f1[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) xh[q] = (mp.a2[q] - mp.mu2) * mp.rs2;
    ln32_bwd(dxv, xh, mp.rs2, lv + LO::ln2w, da);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      tt[q] = dxv[q] * xh[q];
      da[q] = mp.a2[q] > 0.f ? da[q] : 0.f;
      xh[q] = (mp.a1[q] - mp.mu1) * mp.rs1;
      f1[q] = xh[q] * lv[LO::ln1w + kperm(q, h)] + lv[LO::ln1b + kperm(q, h)];
    }
    tput(S0, da);
    tput(S1, f1);
    tput(S2, tt);
    const float s_a2 = scale_for(wave_max(absmax16(da)));
    // ---- LN1 backward: dx1 = W2^T da2 (one scale per column), then da1
    float dx1[16], da1[16];
    {
      const float c_a = scale_for(col_max(absmax16(da)));
      S16 sa;
      split16s(da, c_a, sa);
      f32x16 acc;
      zero16(acc);
      mmh(smb + GM::W2T, sa, acc);
      const float u = 1.0f / (sw * c_a);
#pragma unroll
      for (int q = 0; q < 16; ++q) dx1[q] = acc[q] * u;
      ln32_bwd(dx1, xh, mp.rs1, lv + LO::ln1w, da1);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        tt[q] = dx1[q] * xh[q];
        da1[q] = mp.a1[q] > 0.f ? da1[q] : 0.f;
      }
    }
    wave_fence();
    // dW2 += da2 f1^T, db2
    float At[16];
    {
      float Bt[16];
      tget(S0, At);
      tget(S1, Bt);
      sl2w += tsum(S2);
      wave_fence();
      tput(S0, da1);
      tput(S1, dxv);
      tput(S2, tt);
      S16 sa, sb;
      split16s(At, s_a2, sa);
      split16s(Bt, s_f1, sb);
      f32x16 tmp;
      zero16(tmp);
      accg(tmp, sa, sb);
      acc_unscale(aW2, tmp, 1.0f / (s_a2 * s_f1));
#pragma unroll
      for (int s = 0; s < 16; ++s) sb2 += At[s];
    }
    const float s_a1 = scale_for(wave_max(absmax16(da1)));
    wave_fence();
    sl2b += tsum(S1);
    sl1w += tsum(S2);
    tget(S0, At);   // da1 transposed
    wave_fence();
    tput(S1, dx1);
    wave_fence();
    sl1b += tsum(S1);
    wave_fence();
    // ---- L1 / LN0: dW1 += da1 f0^T, db1, df0 = W1^T da1 -> LN0 parameter gradients
    {
      S16 sa;
      split16s(At, s_a1, sa);
#pragma unroll
      for (int s = 0; s < 16; ++s) sb1 += At[s];
      const float c_b = scale_for(col_max(absmax16(da1)));
      S16 sd;
      split16s(da1, c_b, sd);
      const float u_b = 1.0f / (sw * c_b), u_w = 1.0f / (s_a1 * s_f0);
      float x[DT][16];
      load_obs<D, DT>(a.obs + row * D, x);
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        float x0[16], f0[16], dfv[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int f = 32 * t + kperm(q, h);
          x0[q] = (x[t][q] - mp.mu0) * mp.rs0;
          f0[q] = x0[q] * lv[LO::ln0w + f] + lv[LO::ln0b + f];
        }
        tput(S0, f0);
        f32x16 acc;
        zero16(acc);
        mmh(smb + GM::W1T + t * HBLK, sd, acc);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          dfv[q] = acc[q] * u_b;
          tt[q] = dfv[q] * x0[q];
        }
        tput(S1, tt);
        tput(S2, dfv);
        wave_fence();
        float Bt[16];
        tget(S0, Bt);
        sl0w[t] += tsum(S1);
        sl0b[t] += tsum(S2);
        S16 sb;
        split16s(Bt, s_f0, sb);
        f32x16 tmp;
        zero16(tmp);
        accg(tmp, sa, sb);
        acc_unscale(aW1[t], tmp, u_w);
        wave_fence();
      }
    }
  }

  // ---- block reduction (fixed order), one partial per block
  __syncthreads();
  float* red = sm;
  for (int e = threadIdx.x; e < F::total; e += blockDim.x) red[e] = 0.f;
  sb2 = xsum(sb2);
  sb1 = xsum(sb1);
  sl2w = xsum(sl2w);
  sl2b = xsum(sl2b);
  sl1w = xsum(sl1w);
  sl1b = xsum(sl1b);
#pragma unroll
  for (int t = 0; t < DT; ++t) {
    sl0w[t] = xsum(sl0w[t]);
    sl0b[t] = xsum(sl0b[t]);
  }
  __syncthreads();
  for (int ww = 0; ww < MWV; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int mm = kperm(q, h);
        red[F::W2 + mm * H + ci] += aW2[q];
#pragma unroll
        for (int t = 0; t < DT; ++t)
          if (32 * t + ci < D) red[F::W1 + mm * F::Dp + 32 * t + ci] += aW1[t][q];
      }
      if (h == 0) {
        red[F::b2 + ci] += sb2;
        red[F::b1 + ci] += sb1;
        red[F::ln2_w + ci] += sl2w;
        red[F::ln2_b + ci] += sl2b;
        red[F::ln1_w + ci] += sl1w;
        red[F::ln1_b + ci] += sl1b;
#pragma unroll
        for (int t = 0; t < DT; ++t)
          if (32 * t + ci < D) {
            red[F::ln0_w + 32 * t + ci] += sl0w[t];
            red[F::ln0_b + 32 * t + ci] += sl0b[t];
          }
      }
    }
    __syncthreads();
  }
  float* outp = k.partial + ((int64_t)net * 2 * NB + NB + blockIdx.x) * k.pstride;
  for (int e = threadIdx.x; e < F::total; e += blockDim.x) outp[e] = red[e];
}

// ---------------------------------------------------------------- rollout forward on MFMA
// get_actions / get_values (rmappo_policy.py:57-99; r_actor_critic.py:60-93, 189-208) for one step of every row: the
// actor and critic trunks (LN0 -> L1 -> LN1 -> L2 -> LN2 -> GRU on h * mask -> LN_r -> head) with the same act-frag
// MFMA building blocks as the training passes (Mlp / Gru above: one wave = 32 rows, features on M, rows on N,
// v_mfma_f32_32x32x2_f32 exact-f32 products), then per row (lane half h = 0) the Categorical sample / log-prob
// (inverse CDF of the softmax with the injected or counter-RNG uniform, mappo.hip fwd_body's arithmetic) or the
// value, and the new hidden state as 16-byte stores. Block = 4 waves, 2 blocks per CU (the forward part of the
// LDS image only); blockIdx.y = net (0 actor, 1 critic; VALUES mode: critic only).
template <int D, int O>
__device__ void stage_fwd(float* sm, const float* __restrict__ P) {
  using G = Geo<D, O>;
  constexpr int gap = G::ln0w - G::WihT;   // the transposed W_ih / W_hh of the backward: not staged
  for (int e = threadIdx.x; e < G::scr - gap; e += blockDim.x) {
    const int src = e < G::WihT ? e : e + gap;
    sm[src] = stage_value<D, O>(P, src);
  }
  __syncthreads();
}

template <int D, int A, int O>
__device__ void roll_body(const mm_mappo_fwd_args& a, int net, float* sm) {
  using G = Geo<D, O>;
  stage_fwd<D, O>(sm, a.net[net].P);
  const mm_mappo_net_io& io = a.net[net];
  const int lane = (int)(threadIdx.x & 63), ci = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t R = a.rows, ntile = (R + 31) / 32;
  const uint64_t ctr = a.counter_ptr ? *a.counter_ptr : a.counter;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + w; tile < ntile; tile += (int64_t)gridDim.x * 4) {
    const int64_t r0 = tile * 32 + ci;
    const bool valid = r0 < R;
    const int64_t row = valid ? r0 : R - 1;
    const float* smo = sm + opaque0();
    float x2[16], hc[16];
    {
      Mlp<D, O> mp;
      mp.run(smo + G::W1, smo + G::W2, smo + G::ln0w, a.obs + row * D);
      mp.x2(smo + G::ln0w, x2);
    }
    ld_row32(io.h_in, row, hc);
    const float m = a.mask ? a.mask[row] : 1.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) hc[q] *= m;
    Gru<D, O> gr;
    gr.run(smo, x2, hc);
    if (valid && io.h_out) st_row32(io.h_out, row, gr.h2);
    // head: LN_r(h2) -> Wo y + bo
    float mur, rsr, y[16];
    ln32(gr.h2, mur, rsr);
#pragma unroll
    for (int q = 0; q < 16; ++q) y[q] = (gr.h2[q] - mur) * rsr * smo[G::lnrw + kperm(q, h)] + smo[G::lnrb + kperm(q, h)];
    float l[O];
#pragma unroll
    for (int o = 0; o < O; ++o) {
      float sacc = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) sacc = fmaf(smo[G::Wo + o * 32 + kperm(q, h)], y[q], sacc);
      l[o] = smo[G::bo + o] + xsum(sacc);
    }
    if (!valid || h != 0) continue;
    if constexpr (O == 1) {
      if (io.out) io.out[row] = l[0];
    } else {
      // log-softmax (mappo.hip log_softmax)
      float mx = l[0];
#pragma unroll
      for (int q = 1; q < O; ++q) mx = fmaxf(mx, l[q]);
      float se = 0.0f;
#pragma unroll
      for (int q = 0; q < O; ++q) se += expf(l[q] - mx);
      const float lse = mx + logf(se);
#pragma unroll
      for (int q = 0; q < O; ++q) l[q] -= lse;
      int act;
      if (a.act_in) {
        act = a.act_in[row];
      } else if (a.deterministic) {
        act = 0;   // Categorical.mode() = first argmax (distributions.py:61-62)
#pragma unroll
        for (int q = 1; q < O; ++q)
          if (l[q] > l[act]) act = q;
        if (a.act_out) a.act_out[row] = act;
      } else {
        const float u = a.u ? a.u[row] : rng_uniform(rng_draw(a.seed, ctr, (uint64_t)row, 0x9E37ull));
        act = O - 1;   // inverse CDF: first k with u < cumsum(p)[k], the last action if rounding leaves none
        bool found = false;
        float cs = 0.0f;
#pragma unroll
        for (int q = 0; q < O; ++q) {
          cs += expf(l[q]);
          if (!found && u < cs) {
            act = q;
            found = true;
          }
        }
        if (a.act_out) a.act_out[row] = act;
      }
      float lp = l[0];
#pragma unroll
      for (int q = 1; q < O; ++q)
        if (q == act) lp = l[q];
      if (io.out) io.out[row] = lp;
    }
  }
}

template <int D, int A>
__global__ __launch_bounds__(256, 2) void mappo_roll_kernel(mm_mappo_fwd_args a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int net = (int)blockIdx.y + (a.mode == MM_MAPPO_VALUES ? 1 : 0);
  if (net == 0)
    roll_body<D, A, A>(a, 0, sm);
  else
    roll_body<D, A, 1>(a, 1, sm);
}

template <int D, int A>
static int roll_fwd(const mm_mappo_fwd_args* a, hipStream_t s) {
  constexpr size_t lds = (size_t)Geo<D, A>::scr * 4;
  static_assert(Geo<D, A>::scr == Geo<D, 1>::scr, "actor / critic LDS images differ");
  static const int attr_rc = [&]() -> int {
    MM_HIP_CHECK(hipFuncSetAttribute((const void*)mappo_roll_kernel<D, A>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
    return MM_OK;
  }();
  if (attr_rc != MM_OK) return attr_rc;
  if (a->rows <= 0) return MM_OK;
  const int64_t ntile = (a->rows + 31) / 32;
  const int nets = a->mode == MM_MAPPO_VALUES ? 1 : 2;
  const unsigned nb = (unsigned)std::min<int64_t>((ntile + 3) / 4, 1024);
  hipLaunchKernelGGL((mappo_roll_kernel<D, A>), dim3(nb, nets), dim3(256), lds, s, *a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

template <int D, int A>
__global__ __launch_bounds__(64 * GW, 1) void mappo_grad_gru_kernel(GradArgs k) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  if (blockIdx.y == 0)
    gru_body<D, A, A>(k, 0, sm);
  else
    gru_body<D, A, 1>(k, 1, sm);
}

template <int D, int A>
__global__ __launch_bounds__((64 * GeoM<D, A>::MW), 1) void mappo_grad_mlp_kernel(GradArgs k) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  if (blockIdx.y == 0)
    mlp_body<D, A>(k, 0, sm);
  else
    mlp_body<D, 1>(k, 1, sm);
}

// grad[p] = sum over the partials of both passes [b][p], fixed order
__global__ __launch_bounds__(256) void mappo_grad_sum_kernel(const float* __restrict__ partial, int nb,
                                                             int64_t pstride, int n0, int n1, float* g0, float* g1) {
  const int net = blockIdx.y;
  const int n = net == 0 ? n0 : n1;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  const float* src = partial + (int64_t)net * nb * pstride + p;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += src[(int64_t)b * pstride];
  (net == 0 ? g0 : g1)[p] = s;
}

template <int D, int A>
struct GradShape {
  static int64_t pstride() { return ((int64_t)MGeo<D, H, A>::total + 3) & ~3ll; }
  static int64_t hseq_count(int L) { return 2ll * NB * GW * 2 * L * 1024; }
  static int64_t scratch(int L, int T, int64_t en) {
    return hseq_count(L) + 2ll * T * en * 32 + 2ll * 2 * NB * pstride();
  }
  static int run(const mm_mappo_bwd_args* a, const float* ha, const float* hc, float* ga, float* gc, float* scratch,
                 hipStream_t s) {
    constexpr size_t lds_g = (size_t)GeoH<D, A>::total * 4, lds_m = (size_t)GeoM<D, A>::total * 4;
    static_assert(GeoH<D, A>::total == GeoH<D, 1>::total && GeoM<D, A>::total == GeoM<D, 1>::total,
                  "actor / critic LDS images differ");
    static_assert(GeoH<D, A>::total * 4 <= 160 * 1024 && GeoM<D, A>::total * 4 <= 160 * 1024, "LDS budget");
    // thread-safe one-time setup (a function-local static's initialiser runs once); the sizes are compile-time
    static const int attr_rc = [&]() -> int {
      MM_HIP_CHECK(hipFuncSetAttribute((const void*)mappo_grad_gru_kernel<D, A>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_g));
      MM_HIP_CHECK(hipFuncSetAttribute((const void*)mappo_grad_mlp_kernel<D, A>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_m));
      return MM_OK;
    }();
    if (attr_rc != MM_OK) return attr_rc;
    GradArgs k = {};
    k.a = *a;
    k.h_in[0] = ha;
    k.h_in[1] = hc;
    k.hseq = scratch;
    k.dx2 = scratch + hseq_count(a->L);
    k.partial = k.dx2 + 2ll * a->T * a->en * 32;
    k.pstride = pstride();
    hipLaunchKernelGGL((mappo_grad_gru_kernel<D, A>), dim3(NB, 2), dim3(64 * GW), lds_g, s, k);
    MM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL((mappo_grad_mlp_kernel<D, A>), dim3(NB, 2), dim3(64 * GeoM<D, A>::MW), lds_m, s, k);
    MM_HIP_CHECK(hipGetLastError());
    const int n0 = MGeo<D, H, A>::total, n1 = MGeo<D, H, 1>::total;
    hipLaunchKernelGGL(mappo_grad_sum_kernel, dim3((n0 + 255) / 256, 2), dim3(256), 0, s, k.partial, 2 * NB,
                       k.pstride, n0, n1, ga, gc);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
};

}  // namespace mgr

// the rollout / get_values forward on MFMA (mappo.hip routes MM_MAPPO_ROLLOUT / VALUES here for H 32, D 47 | 94, A 5)
int mappo_roll_fwd(const mm_mappo_dims* d, const mm_mappo_fwd_args* a, hipStream_t s) {
  if (d->obs_dim == 47) return mgr::roll_fwd<47, 5>(a, s);
  return mgr::roll_fwd<94, 5>(a, s);
}
}  // namespace mm

extern "C" {

int64_t mm_mappo_grad_scratch_count(const mm_mappo_dims* d, int32_t L, int32_t T, int64_t en) {
  if (!d || L <= 0 || T <= 0 || en <= 0 || d->hidden != 32 || d->n_actions != 5) return -1;
  if (d->obs_dim == 47) return mm::mgr::GradShape<47, 5>::scratch(L, T, en);
  if (d->obs_dim == 94) return mm::mgr::GradShape<94, 5>::scratch(L, T, en);
  return -1;
}

int mm_mappo_grad(const mm_mappo_dims* d, const mm_mappo_bwd_args* a, const float* h_actor, const float* h_critic,
                  float* grad_actor, float* grad_critic, float* scratch, mm_stream_t s) {
  MM_REQUIRE(d && a && h_actor && h_critic && grad_actor && grad_critic && scratch, "mappo_grad: null argument");
  MM_REQUIRE(a->L > 0 && a->T % a->L == 0 && a->en > 0, "mappo_grad: need L | T");
  MM_REQUIRE(a->P[0] && a->P[1] && a->obs && a->mask && a->active && a->act && a->adv && a->old_logp &&
                 a->old_value && a->returns && a->stats,
             "mappo_grad: null pointer");
  MM_REQUIRE(((uintptr_t)h_actor & 15) == 0 && ((uintptr_t)h_critic & 15) == 0 && ((uintptr_t)scratch & 15) == 0,
             "mappo_grad: hiddens and scratch must be 16-byte aligned");
  MM_REQUIRE(d->hidden == 32 && d->n_actions == 5 && (d->obs_dim == 47 || d->obs_dim == 94),
             "mappo_grad: unsupported dims D=%d H=%d A=%d (supported: D 47|94, H 32, A 5)", d->obs_dim, d->hidden,
             d->n_actions);
  if (d->obs_dim == 47)
    return mm::mgr::GradShape<47, 5>::run(a, h_actor, h_critic, grad_actor, grad_critic, scratch, (hipStream_t)s);
  return mm::mgr::GradShape<94, 5>::run(a, h_actor, h_critic, grad_actor, grad_critic, scratch, (hipStream_t)s);
}

}  // extern "C"
