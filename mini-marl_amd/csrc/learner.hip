// Learner kernels for the chunked-BPTT QMIX / VDN update (gfx950).
//
// Replaces Train_dqn.train (qmix/_train.py:19-121) and Target_Dqn.train
// (vdn/_train.py:184-235): one update = sample B chunks of C steps from the
// device PER, forward the behavior and target agent nets (mm_agent_q_fwd with
// the training save) and mixers over the C steps, loss, backward through time,
// clip_grad_norm_, Adam, priority update. Reference quirks reproduced
// (SURVEY App. A): target = w * sum_i(r_i + gamma*(1-d)*Q'_tot) (bootstrap x N,
// IS weight on the target), MSE mean over B summed over C, hidden states zero at
// the chunk start and reset on done, priorities from the LAST step's |y - Q_tot|,
// QMIX clips the agent params only.
//
// Structure: the C-step recurrences (forward, mixer backward, agent backward
// chain) are small dependent launches; every weight gradient is deferred and
// computed at the end as ONE batched outer-product reduction over all C*B
// (step, sample) rows — so the sequential part only carries the data-gradient
// chain. All reductions use a fixed order (bit-reproducible run to run).
#pragma clang fp contract(off)
#include "common.h"
#include "minimarl.h"
#include "per_small.h"

namespace mm {
// large-batch kernel shape (mm_learner_set_multi_sample): B >= 512 runs the mixer forward / recurrence backward with
// MIX_SPB samples per block and the agent backward with BWD_SPW samples per wave (shared weight reads); 0 selects the
// one-sample kernels, whose results are identical (tests/test_gpu_learner.py pins the equality)
static int g_mix_multi = 1, g_bwd_multi = 1;

// Element offset of state row i in the obs array: the gathered chunk-store offsets (-1: the env's reset
// obs), or, without offsets (the torch ops' contiguous [rows, S] state), row i itself.
__device__ __forceinline__ int64_t state_off(const int64_t* s_off, int64_t i, int S) {
  return s_off ? s_off[i] : i * (int64_t)S;
}

// ------------------------------------------------------------------ gather
// For sample b (PER slot -> chunk-store row) and step t:
//   s_off[t][b]  = element offset of s_t in store.obs  (-1 => the env's reset obs)
//   s2_off[t][b] = element offset of s'_t
//   acts[t][b][i] (int32), rew[t][b][i] (f32), done[t][b] (f32), done8[t][b] (u8)
// The learner's chunk-store gather of the sampled slots (lrn_gather_kernel): row i = (t, b) of the [C][B] batch from chunk-store row
// slot_row[slots[b]] — state offsets (s_t: -1 after an earlier done in the chunk, i.e. the reset obs; s'_t), the
// agents' actions and rewards, the done flag (f32 and u8). qmix/replay_buffer/per.py:61-81 (Replay_buffer.sample
// over chunk lists), vdn/replay_buffer/buffer.py:58-70.
struct SampleGather {
  int C, N;
  int64_t row_stride, nd;
  const int64_t* slot_row;
  const uint8_t* s_done;
  const uint8_t* s_act;
  const float* s_rew;
  int64_t *s_off, *s2_off;
  int32_t* acts;
  float *rew, *done;
  uint8_t* done8;
};
// row: the chunk-store row of sample b = i % B
__device__ __forceinline__ void sample_gather_row(const SampleGather& g, int B, int64_t row, int i) {
  const int C = g.C, N = g.N;
  const int t = i / B;
  const uint8_t dprev = t > 0 ? g.s_done[row * C + t - 1] : 0;
  g.s_off[i] = (t > 0 && dprev) ? -1 : row * g.row_stride + (int64_t)t * g.nd;
  g.s2_off[i] = row * g.row_stride + (int64_t)(t + 1) * g.nd;
  const uint8_t dn = g.s_done[row * C + t];
  g.done[i] = dn ? 1.0f : 0.0f;
  g.done8[i] = dn;
  for (int k = 0; k < N; ++k) {
    g.acts[(int64_t)i * N + k] = g.s_act[(row * C + t) * N + k];
    g.rew[(int64_t)i * N + k] = g.s_rew[(row * C + t) * N + k];
  }
}

__global__ void lrn_gather_kernel(SampleGather g, int B, const int64_t* slots) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * g.C) sample_gather_row(g, B, g.slot_row[slots[i % B]], i);
}

// ------------------------------------------------------------------ block helpers
// out[r] = (bias ? bias[r] : 0) + sum_k W[r*K + k] * x[k]   for r < rows (x in LDS). fixed-order sums.
__device__ void block_matvec(const float* __restrict__ W, const float* __restrict__ bias, int rows, int K,
                             const float* x, float* out) {
  if (K >= 128) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int r = w; r < rows; r += nw) {
      float acc = 0.f;
      for (int k = lane; k < K; k += 64) acc += W[(int64_t)r * K + k] * x[k];
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
      if (lane == 0) out[r] = acc + (bias ? bias[r] : 0.f);
    }
  } else {
    for (int r = threadIdx.x; r < rows; r += blockDim.x) {
      float acc = 0.f;
      for (int k = 0; k < K; ++k) acc += W[(int64_t)r * K + k] * x[k];
      out[r] = acc + (bias ? bias[r] : 0.f);
    }
  }
}

// out[c] (+)= sum_r W[r*K + c] * d[r]   for c < K (transpose matvec, coalesced over c). The rows are
// split over the block's waves (wave w takes r = w mod nw, unrolled by 4 so loads overlap) and the
// per-wave partials are combined in a fixed order through LDS (red: >= nw*K floats of scratch).
// Ends with __syncthreads.
__device__ void block_matvec_t(const float* __restrict__ W, int rows, int K, const float* d, float* out,
                               bool accumulate, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int c = lane; c < K; c += 64) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int r = w;
    for (; r + 3 * nw < rows; r += 4 * nw) {
      a0 += W[(int64_t)r * K + c] * d[r];
      a1 += W[(int64_t)(r + nw) * K + c] * d[r + nw];
      a2 += W[(int64_t)(r + 2 * nw) * K + c] * d[r + 2 * nw];
      a3 += W[(int64_t)(r + 3 * nw) * K + c] * d[r + 3 * nw];
    }
    for (; r < rows; r += nw) a0 += W[(int64_t)r * K + c] * d[r];
    red[w * K + c] = (a0 + a1) + (a2 + a3);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < K; c += blockDim.x) {
    float acc = 0.f;
    for (int q = 0; q < nw; ++q) acc += red[q * K + c];
    out[c] = accumulate ? out[c] + acc : acc;
  }
  __syncthreads();
}

// ------------------------------------------------------------------ mixer
// Canonical mixer layout (qmix/_network.py:172-197), oracle/nets.py MIXER_KEYS order.
struct MixOff {
  int64_t gWih, gWhh, gbih, gbhh, w1W, w1b, w2W, w2b, b1W, b1b, b2aW, b2ab, b2bW, b2bb, total;
};

__host__ __device__ inline MixOff mix_offsets(int S, int Hm, int K1, int N) {
  MixOff o;
  int64_t c = 0;
  o.gWih = c; c += (int64_t)3 * Hm * S;
  o.gWhh = c; c += (int64_t)3 * Hm * Hm;
  o.gbih = c; c += 3 * Hm;
  o.gbhh = c; c += 3 * Hm;
  o.w1W = c; c += (int64_t)N * K1 * Hm;
  o.w1b = c; c += N * K1;
  o.w2W = c; c += (int64_t)K1 * Hm;
  o.w2b = c; c += K1;
  o.b1W = c; c += (int64_t)K1 * Hm;
  o.b1b = c; c += K1;
  o.b2aW = c; c += (int64_t)K1 * Hm;
  o.b2ab = c; c += K1;
  o.b2bW = c; c += K1;
  o.b2bb = c; c += 1;
  o.total = c;
  return o;
}

// per-(t,b) mixer save row: [hm0 | r | z | n | anh | hm1 | w1raw (N*K1) | b1 | w2raw | b2pre | ypre | b2]
__host__ __device__ inline int mix_save_dim(int Hm, int K1, int N) { return 6 * Hm + N * K1 + 4 * K1 + 1; }

struct MixFwdNet {
  const float* P;        // mixer params (canonical)
  const float* gi;       // [B][3Hm] precomputed W_ih s + b_ih of this step (mixer_gi_kernel) or nullptr
  const float* q;        // [B][N] agent values fed to the mixer (Q(a) or max Q')
  const int64_t* s_off;  // [B] state offsets into obs (-1: reset obs)
  const float* h_in;     // [B][Hm] (nullptr => zero)
  const uint8_t* reset;  // [B] (nullptr => none)
  float* h_out;          // [B][Hm]
  float* qtot;           // [B]
  float* save;           // [B][MSD] or nullptr
};

struct MixFwdArgs {
  MixFwdNet net[2];
  const float* obs;
  const float* reset_obs;  // [N*D]
  int B, N, S, Hm, K1;
};

// Mixer GRU input projection for every (t, b) of the chunk batch at once (the state input does
// not depend on the recurrence): gi[r][m] = b_ih[m] + sum_k W_ih[m][k] s_r[k] with s_r gathered
// through the state offsets (reset obs where off < 0). v_mfma_f32_32x32x2_f32, features of W_ih
// on rows, samples on columns; block = 4 waves splitting K, reduced through LDS.
struct MixGiNet {
  const float* P;
  const int64_t* s_off;  // [R]
  float* gi;             // [R][3Hm]
};
struct MixGiArgs {
  MixGiNet net[2];
  const float* obs;
  const float* reset_obs;
  int R, S, Hm, K1, N;
};

// one 32-sample x 32-row tile (bx, by) of net bz, by the block's first 4 waves (a paired launch's wider block
// lets its other waves pass: every thread reaches the barrier)
__device__ __forceinline__ void mixer_gi_body(const MixGiArgs& a, int bx, int by, int bz) {
  __shared__ float red[4][1024];
  const MixGiNet& nt = a.net[bz];
  const int S = a.S, M3 = 3 * a.Hm;
  const MixOff o = mix_offsets(S, a.Hm, a.K1, a.N);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 31, hh = lane >> 5;
  const int rb = by, col = bx * 32 + i;
  const int row = rb * 32 + i;
  if (wave < 4) {
    const float* W = nt.P + o.gWih + (int64_t)(row < M3 ? row : 0) * S;
    const int64_t off = col < a.R ? state_off(nt.s_off, col, a.S) : -1;
    const float* x = off >= 0 ? a.obs + off : a.reset_obs;
    const int KD = (S + 31) / 32;
    f32x16 acc = {0};
    for (int kb = wave; kb < KD; kb += 4) {
      float av[16], bv[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int k = kb * 32 + kperm(s, hh);
        const bool ok = k < S;
        av[s] = (ok && row < M3) ? W[k] : 0.0f;
        bv[s] = (ok && col < a.R) ? x[k] : 0.0f;
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = mfma32(av[s], bv[s], acc);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) red[wave][kperm(s, hh) * 32 + i] = acc[s];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 1024; e += blockDim.x) {
    const int m = rb * 32 + (e >> 5), c = bx * 32 + (e & 31);
    if (m < M3 && c < a.R)
      nt.gi[(int64_t)c * M3 + m] = nt.P[o.gbih + m] + ((red[0][e] + red[1][e]) + (red[2][e] + red[3][e]));
  }
}
__global__ __launch_bounds__(256) void mixer_gi_kernel(MixGiArgs a) {
  mixer_gi_body(a, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z);
}

// LDS-tiled form of the same projection: block = 4 waves = 64 samples x 64 gate rows, per 32-deep
// k chunk the gathered state rows and the W_ih rows are staged in LDS ([k][sample], [k][row];
// both loads coalesced along k), every wave accumulates a 32 x 32 sub-tile with 16 exact-f32
// MFMAs in fixed k order.
__global__ __launch_bounds__(256) void mixer_gi_tiled_kernel(MixGiArgs a) {
  __shared__ float sx[32][65];
  __shared__ float sw[32][65];
  const MixGiNet& nt = a.net[blockIdx.z];
  const int S = a.S, M3 = 3 * a.Hm;
  const MixOff o = mix_offsets(S, a.Hm, a.K1, a.N);
  const int c0 = blockIdx.y * 64, m0 = blockIdx.x * 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  const int cw = wave >> 1, mw = wave & 1;
  const float* Wih = nt.P + o.gWih;
  // the 8 sample rows (c0 + (tid >> 5) + 8p) and 8 weight rows (m0 + ...) this thread stages
  const float* xr[8];
  const float* wr[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int rr = (threadIdx.x >> 5) + 8 * p;
    const int c = c0 + rr;
    const int64_t off = c < a.R ? state_off(nt.s_off, c, a.S) : -1;
    xr[p] = c < a.R ? (off >= 0 ? a.obs + off : a.reset_obs) : nullptr;
    wr[p] = m0 + rr < M3 ? Wih + (int64_t)(m0 + rr) * S : nullptr;
  }
  const int x = threadIdx.x & 31;
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
  // chunk k0 + 32 is loaded into registers while chunk k0 is reduced (one memory latency per launch instead of one
  // per 32-deep chunk; same values, same MFMA order)
  float px[8], pw[8];
  auto fetch = [&](int k0) {
    const bool ok = k0 + x < S;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      px[p] = (ok && xr[p]) ? xr[p][k0 + x] : 0.f;
      pw[p] = (ok && wr[p]) ? wr[p][k0 + x] : 0.f;
    }
  };
  fetch(0);
  for (int k0 = 0; k0 < S; k0 += 32) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int rr = (threadIdx.x >> 5) + 8 * p;
      sx[x][rr] = px[p];
      sw[x][rr] = pw[p];
    }
    __syncthreads();
    if (k0 + 32 < S) fetch(k0 + 32);
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
      acc = mfma32(sx[2 * s2 + lh][cw * 32 + li], sw[2 * s2 + lh][mw * 32 + li], acc);
    __syncthreads();
  }
  const int m = m0 + mw * 32 + li;
  if (m < M3) {
    const float bias = nt.P[o.gbih + m];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int c = c0 + cw * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
      if (c < a.R) nt.gi[(int64_t)c * M3 + m] = bias + acc[q];
    }
  }
}

// cfg5 fp16 mode (rtol 2e-3 on Q_tot, stated separately from the fp32 parity): the same
// state projection gi = W_ih s + b_ih on v_mfma_f32_32x32x16_f16 (inputs rounded to f16, fp32
// accumulate). Block = 64 samples x all 3Hm gate rows (RBK = 3Hm / 32 row blocks; 2 RBK waves, each one
// 32 x 32 tile), the K = S state width in 64-deep chunks staged as f16 in LDS (row pitch 72 halves:
// conflict-free 16-byte fragment reads), the next chunk's global loads in flight during the MFMAs.
// Loads are 16-byte (4 consecutive k of one state / weight row per item; a row whose start is not
// 16-byte aligned takes 4 scalar loads), the 64 samples' state offsets read once into LDS.
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
template <int RBK>
__global__ __launch_bounds__(64 * 2 * RBK) void mixer_gi_f16_kernel(MixGiArgs a) {
  constexpr int NT = 64 * 2 * RBK, ROWS = 32 * RBK, PITCH = 72, KC = 64;
  constexpr int NX4 = 64 * KC / 4, NW4 = ROWS * KC / 4;    // 4-float items per chunk: state, weights
  constexpr int NI = (NX4 + NW4 + NT - 1) / NT;            // items per thread per chunk
  __shared__ __attribute__((aligned(16))) _Float16 sx[2][64 * PITCH];
  __shared__ __attribute__((aligned(16))) _Float16 sw[2][ROWS * PITCH];
  __shared__ const float* srow[64];
  const MixGiNet& nt = a.net[blockIdx.y];
  const int S = a.S, M3 = 3 * a.Hm;
  const MixOff o = mix_offsets(S, a.Hm, a.K1, a.N);
  const int c0 = blockIdx.x * 64;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, li = lane & 31, lh = lane >> 5;
  const int cw = wave & 1, rw = wave >> 1;   // this wave's 32 samples / 32 gate rows
  if (tid < 64) {
    const int c = min(c0 + tid, a.R - 1);
    const int64_t off = state_off(nt.s_off, c, a.S);
    srow[tid] = off >= 0 ? a.obs + off : a.reset_obs;
  }
  const float* Wih = nt.P + o.gWih;
  __syncthreads();
  float4 v[NI];
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int idx = tid + j * NT;
      if (idx >= NX4 + NW4) break;
      const int i2 = idx < NX4 ? idx : idx - NX4;
      const int r = i2 >> 4, k = k0 + 4 * (i2 & 15);
      const float* row = idx < NX4 ? srow[r] : Wih + (int64_t)min(r, M3 - 1) * S;
      if (k + 3 < S && ((reinterpret_cast<uintptr_t>(row) & 15) == 0)) {
        v[j] = *reinterpret_cast<const float4*>(row + k);
      } else {
        v[j].x = k < S ? row[k] : 0.f;
        v[j].y = k + 1 < S ? row[k + 1] : 0.f;
        v[j].z = k + 2 < S ? row[k + 2] : 0.f;
        v[j].w = k + 3 < S ? row[k + 3] : 0.f;
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int idx = tid + j * NT;
      if (idx >= NX4 + NW4) break;
      const int i2 = idx < NX4 ? idx : idx - NX4;
      const int r = i2 >> 4, x = 4 * (i2 & 15);
      const h16x4 hv = {(_Float16)v[j].x, (_Float16)v[j].y, (_Float16)v[j].z, (_Float16)v[j].w};
      _Float16* dst = idx < NX4 ? &sx[buf][r * PITCH + x] : &sw[buf][r * PITCH + x];
      *reinterpret_cast<h16x4*>(dst) = hv;
    }
  };
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  const int nch = (S + KC - 1) / KC;
  load(0);
  store(0);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nch) load((ch + 1) * KC);   // next chunk in flight during the MFMAs
#pragma unroll
    for (int ks = 0; ks < KC / 16; ++ks) {
      const h16x8 av = *reinterpret_cast<const h16x8*>(&sw[buf][(rw * 32 + li) * PITCH + ks * 16 + 8 * lh]);
      const h16x8 bv = *reinterpret_cast<const h16x8*>(&sx[buf][(cw * 32 + li) * PITCH + ks * 16 + 8 * lh]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv, acc, 0, 0, 0);
    }
    if (ch + 1 < nch) store(buf ^ 1);
    __syncthreads();
  }
  // D: col = sample li, row = (q & 3) + 8 (q >> 2) + 4 lh
  // gate rows rw*32 + 8j + 4lh + 0..3 of sample c are acc[4j..4j+3]: 16-byte stores (M3 = 96 / 192 and the
  // gi base keep every run 16-byte aligned), not 16 scattered dword stores per lane
  const int c = c0 + cw * 32 + li;
  if (c < a.R) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = rw * 32 + 8 * j + 4 * lh;
      const float* bb = nt.P + o.gbih + m;
      *reinterpret_cast<float4*>(nt.gi + (int64_t)c * M3 + m) =
          make_float4(bb[0] + acc[4 * j], bb[1] + acc[4 * j + 1], bb[2] + acc[4 * j + 2], bb[3] + acc[4 * j + 3]);
    }
  }
}

// One block per (sample, net): blockIdx.y selects behavior / target.
__device__ __forceinline__ void mixer_fwd_body(const MixFwdArgs& a, const MixFwdNet& nt, int b);

__global__ __launch_bounds__(256) void mixer_fwd_kernel(MixFwdArgs a) {
  mixer_fwd_body(a, a.net[blockIdx.y], blockIdx.x);
}

__device__ __forceinline__ void mixer_fwd_body(const MixFwdArgs& a, const MixFwdNet& nt, int b) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int S = a.S, Hm = a.Hm, K1 = a.K1, N = a.N;
  const MixOff o = mix_offsets(S, Hm, K1, N);
  float* xs = sm;                  // [S]
  float* h0 = xs + S;              // [Hm]
  float* gi = h0 + Hm;             // [3Hm]
  float* gh = gi + 3 * Hm;         // [3Hm]
  float* h1 = gh + 3 * Hm;         // [Hm]
  float* hyp = h1 + Hm;            // [N*K1 + 3*K1]: w1raw | b1 | w2raw | b2pre
  float* yp = hyp + N * K1 + 3 * K1;  // [K1]
  const bool rz = !nt.h_in || (nt.reset && nt.reset[b]);
  for (int i = threadIdx.x; i < Hm; i += blockDim.x) h0[i] = rz ? 0.f : nt.h_in[(int64_t)b * Hm + i];
  if (nt.gi) {
    for (int i = threadIdx.x; i < 3 * Hm; i += blockDim.x) gi[i] = nt.gi[(int64_t)b * 3 * Hm + i];
    __syncthreads();
  } else {
    const int64_t off = state_off(nt.s_off, b, a.S);
    const float* src = off >= 0 ? a.obs + off : a.reset_obs;
    for (int i = threadIdx.x; i < S; i += blockDim.x) xs[i] = src[i];
    __syncthreads();
    block_matvec(nt.P + o.gWih, nt.P + o.gbih, 3 * Hm, S, xs, gi);
  }
  block_matvec(nt.P + o.gWhh, nt.P + o.gbhh, 3 * Hm, Hm, h0, gh);
  __syncthreads();
  float* sv = nt.save ? nt.save + (int64_t)b * mix_save_dim(Hm, K1, N) : nullptr;
  for (int i = threadIdx.x; i < Hm; i += blockDim.x) {
    const float r = sigmoidf_(gi[i] + gh[i]);
    const float z = sigmoidf_(gi[Hm + i] + gh[Hm + i]);
    const float n = tanhf_(gi[2 * Hm + i] + r * gh[2 * Hm + i]);
    const float hv = n + z * (h0[i] - n);
    h1[i] = hv;
    nt.h_out[(int64_t)b * Hm + i] = hv;
    if (sv) {
      sv[i] = h0[i];
      sv[Hm + i] = r;
      sv[2 * Hm + i] = z;
      sv[3 * Hm + i] = n;
      sv[4 * Hm + i] = gh[2 * Hm + i];
      sv[5 * Hm + i] = hv;
    }
  }
  __syncthreads();
  // hypernets on h1: w1raw [N*K1], b1 [K1], w2raw [K1], b2 hidden pre-ReLU [K1]
  block_matvec(nt.P + o.w1W, nt.P + o.w1b, N * K1, Hm, h1, hyp);
  block_matvec(nt.P + o.b1W, nt.P + o.b1b, K1, Hm, h1, hyp + N * K1);
  block_matvec(nt.P + o.w2W, nt.P + o.w2b, K1, Hm, h1, hyp + N * K1 + K1);
  block_matvec(nt.P + o.b2aW, nt.P + o.b2ab, K1, Hm, h1, hyp + N * K1 + 2 * K1);
  __syncthreads();
  // y_pre[k] = sum_i |w1raw[k*N + i]| q_i + b1[k]   (bmm(W1 [K1,N], q [N,1]) + b1)
  for (int k = threadIdx.x; k < K1; k += blockDim.x) {
    float acc = 0.f;
    for (int i = 0; i < N; ++i) acc += fabsf(hyp[k * N + i]) * nt.q[(int64_t)b * N + i];
    yp[k] = acc + hyp[N * K1 + k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float* w2raw = hyp + N * K1 + K1;
    const float* b2pre = hyp + N * K1 + 2 * K1;
    float b2 = 0.f;
    for (int k = 0; k < K1; ++k) b2 += nt.P[o.b2bW + k] * fmaxf(b2pre[k], 0.f);
    b2 += nt.P[o.b2bb];
    float acc = 0.f;
    for (int k = 0; k < K1; ++k) acc += fabsf(w2raw[k]) * fmaxf(yp[k], 0.f);
    nt.qtot[b] = acc + b2;
    if (sv) sv[6 * Hm + N * K1 + 4 * K1] = b2;
  }
  if (sv) {
    // [w1raw | b1 | w2raw | relu(b2 hidden)] (relu'd: the b2 weight gradient needs it, and its
    // mask relu(x) > 0 equals x > 0)
    for (int i = threadIdx.x; i < N * K1 + 3 * K1; i += blockDim.x)
      sv[6 * Hm + i] = i >= N * K1 + 2 * K1 ? fmaxf(hyp[i], 0.f) : hyp[i];
    for (int k = threadIdx.x; k < K1; k += blockDim.x) sv[6 * Hm + N * K1 + 3 * K1 + k] = yp[k];
  }
}

constexpr int MIX_SPB = 8;
// Hypernets + mixing of MIX_SPB rows b0 .. b0 + ns - 1 whose new mixer hidden is in h1 [SPB][Hm]
// (LDS; rows >= ns zero): hyp = W_hyp h1 + b (sequential k, bias last), y_pre, Q_tot, the save-row tail.
// hyp [SPB][RW], yp [SPB][K1] LDS scratch. Rows index nt.q / qtot / save directly (a flat row range).
__device__ __forceinline__ void mixer_hyper_rows(const MixFwdArgs& a, const MixFwdNet& nt, int b0, int ns,
                                                 const float* h1, float* hyp, float* yp) {
  const int Hm = a.Hm, K1 = a.K1, N = a.N, NK = N * K1, RW = NK + 3 * K1;
  const MixOff o = mix_offsets(a.S, Hm, K1, N);
  // hypernets on h1 (rows: w1 [NK], b1 [K1], w2 [K1], b2 hidden [K1])
  for (int r = threadIdx.x; r < RW; r += blockDim.x) {
    const float* w;
    float bb;
    if (r < NK) {
      w = nt.P + o.w1W + (int64_t)r * Hm;
      bb = nt.P[o.w1b + r];
    } else if (r < NK + K1) {
      w = nt.P + o.b1W + (int64_t)(r - NK) * Hm;
      bb = nt.P[o.b1b + r - NK];
    } else if (r < NK + 2 * K1) {
      w = nt.P + o.w2W + (int64_t)(r - NK - K1) * Hm;
      bb = nt.P[o.w2b + r - NK - K1];
    } else {
      w = nt.P + o.b2aW + (int64_t)(r - NK - 2 * K1) * Hm;
      bb = nt.P[o.b2ab + r - NK - 2 * K1];
    }
    float acc[MIX_SPB];
#pragma unroll
    for (int q = 0; q < MIX_SPB; ++q) acc[q] = 0.f;
#pragma unroll 8
    for (int k = 0; k < Hm; ++k) {   // (weight loads issued ahead; per-sample adds in k order)
      const float wk = w[k];
#pragma unroll
      for (int q = 0; q < MIX_SPB; ++q) acc[q] += wk * h1[q * Hm + k];
    }
#pragma unroll
    for (int q = 0; q < MIX_SPB; ++q) hyp[q * RW + r] = acc[q] + bb;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < ns * K1; idx += blockDim.x) {
    const int sI = idx / K1, k = idx % K1, b = b0 + sI;
    const float* hp = hyp + sI * RW;
    float acc = 0.f;
    for (int i = 0; i < N; ++i) acc += fabsf(hp[k * N + i]) * nt.q[(int64_t)b * N + i];
    yp[sI * K1 + k] = acc + hp[NK + k];
  }
  __syncthreads();
  if ((int)threadIdx.x < ns) {
    const int sI = threadIdx.x, b = b0 + sI;
    const float* hp = hyp + sI * RW;
    const float* w2raw = hp + NK + K1;
    const float* b2pre = hp + NK + 2 * K1;
    float b2 = 0.f;
    for (int k = 0; k < K1; ++k) b2 += nt.P[o.b2bW + k] * fmaxf(b2pre[k], 0.f);
    b2 += nt.P[o.b2bb];
    float acc = 0.f;
    for (int k = 0; k < K1; ++k) acc += fabsf(w2raw[k]) * fmaxf(yp[sI * K1 + k], 0.f);
    nt.qtot[b] = acc + b2;
    if (nt.save) nt.save[(int64_t)b * mix_save_dim(Hm, K1, N) + 6 * Hm + NK + 4 * K1] = b2;
  }
  if (nt.save) {
    for (int idx = threadIdx.x; idx < ns * RW; idx += blockDim.x) {
      const int sI = idx / RW, i = idx % RW;
      float* sv = nt.save + (int64_t)(b0 + sI) * mix_save_dim(Hm, K1, N);
      const float v = hyp[sI * RW + i];
      sv[6 * Hm + i] = i >= NK + 2 * K1 ? fmaxf(v, 0.f) : v;
    }
    for (int idx = threadIdx.x; idx < ns * K1; idx += blockDim.x) {
      const int sI = idx / K1, k = idx % K1;
      nt.save[(int64_t)(b0 + sI) * mix_save_dim(Hm, K1, N) + 6 * Hm + NK + 3 * K1 + k] = yp[sI * K1 + k];
    }
  }
}

// Large batches: MIX_SPB samples per block share every weight read (the single-sample block re-reads
// ~140 KB of W_hh + hypernet weights from L2 per sample). Same per-sample arithmetic and order as
// mixer_fwd_body (bit-identical); needs the precomputed input projection (nt.gi).
__global__ __launch_bounds__(256) void mixer_fwd_multi_kernel(MixFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const MixFwdNet& nt = a.net[blockIdx.y];
  const int Hm = a.Hm, K1 = a.K1, N = a.N, NK = N * K1, RW = NK + 3 * K1;
  const MixOff o = mix_offsets(a.S, Hm, K1, N);
  const int b0 = blockIdx.x * MIX_SPB;
  const int ns = min(MIX_SPB, a.B - b0);
  float* h0 = sm;                        // [SPB][Hm]
  float* gi = h0 + MIX_SPB * Hm;         // [SPB][3Hm]
  float* gh = gi + MIX_SPB * 3 * Hm;     // [SPB][3Hm]
  float* h1 = gh + MIX_SPB * 3 * Hm;     // [SPB][Hm]
  float* hyp = h1 + MIX_SPB * Hm;        // [SPB][RW]: w1raw | b1 | w2raw | b2pre
  float* yp = hyp + MIX_SPB * RW;        // [SPB][K1]
  for (int idx = threadIdx.x; idx < MIX_SPB * Hm; idx += blockDim.x) {
    const int sI = idx / Hm, i = idx % Hm, b = b0 + sI;
    float v = 0.f;
    if (sI < ns) {
      const bool rz = !nt.h_in || (nt.reset && nt.reset[b]);
      v = rz ? 0.f : nt.h_in[(int64_t)b * Hm + i];
    }
    h0[idx] = v;
  }
  for (int idx = threadIdx.x; idx < MIX_SPB * 3 * Hm; idx += blockDim.x) {
    const int sI = idx / (3 * Hm);
    gi[idx] = sI < ns ? nt.gi[(int64_t)b0 * 3 * Hm + idx] : 0.f;
  }
  __syncthreads();
  // gh = W_hh h + b_hh (block_matvec order: sequential k, bias last)
  for (int r = threadIdx.x; r < 3 * Hm; r += blockDim.x) {
    float acc[MIX_SPB];
#pragma unroll
    for (int q = 0; q < MIX_SPB; ++q) acc[q] = 0.f;
    const float* w = nt.P + o.gWhh + (int64_t)r * Hm;
#pragma unroll 8
    for (int k = 0; k < Hm; ++k) {   // (weight loads issued ahead; per-sample adds in k order)
      const float wk = w[k];
#pragma unroll
      for (int q = 0; q < MIX_SPB; ++q) acc[q] += wk * h0[q * Hm + k];
    }
    const float bb = nt.P[o.gbhh + r];
#pragma unroll
    for (int q = 0; q < MIX_SPB; ++q) gh[q * 3 * Hm + r] = acc[q] + bb;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < ns * Hm; idx += blockDim.x) {
    const int sI = idx / Hm, i = idx % Hm, b = b0 + sI;
    const float* gI = gi + sI * 3 * Hm;
    const float* gH = gh + sI * 3 * Hm;
    const float r = sigmoidf_(gI[i] + gH[i]);
    const float z = sigmoidf_(gI[Hm + i] + gH[Hm + i]);
    const float n = tanhf_(gI[2 * Hm + i] + r * gH[2 * Hm + i]);
    const float h0v = h0[sI * Hm + i];
    const float hv = n + z * (h0v - n);
    h1[sI * Hm + i] = hv;
    nt.h_out[(int64_t)b * Hm + i] = hv;
    if (nt.save) {
      float* sv = nt.save + (int64_t)b * mix_save_dim(Hm, K1, N);
      sv[i] = h0v;
      sv[Hm + i] = r;
      sv[2 * Hm + i] = z;
      sv[3 * Hm + i] = n;
      sv[4 * Hm + i] = gH[2 * Hm + i];
      sv[5 * Hm + i] = hv;
    }
  }
  __syncthreads();
  mixer_hyper_rows(a, nt, b0, ns, h1, hyp, yp);
}

// ------------------------------------------------------------------ mixer sequences with LDS-resident weights
// Small batches (B < 512): one block per (sample, net) runs ALL C steps of the mixer forward (or
// backward) in one launch, with the net's W_hh and hypernet weights staged ONCE into LDS (row
// stride Hm + 1: conflict-free for both the row-per-lane forward and the column-per-lane transposed
// backward) and the recurrent state carried in LDS between steps. Per-step arithmetic and summation
// order are exactly mixer_fwd_body / mixer_bwd_body's (bit-identical to the per-step launches).
// Image rows: [W_hh (3Hm) | w1W (N*K1) | b1W (K1) | w2W (K1) | b2aW (K1)] = the forward's hypernet
// row order after W_hh.
struct MixSeqGeo {
  int Hm, K1, N, NK, RW, ld, rows;
  __host__ __device__ MixSeqGeo(int Hm_, int K1_, int N_)
      : Hm(Hm_), K1(K1_), N(N_), NK(N_ * K1_), RW(N_ * K1_ + 3 * K1_), ld(Hm_ + 1), rows(3 * Hm_ + N_ * K1_ + 3 * K1_) {}
  __host__ __device__ size_t img() const { return (size_t)rows * ld; }
  // biases staged with the image: b_hh [3Hm] | hypernet biases [RW] | b2 output weights [K1] + bias [1]
  __host__ __device__ size_t bias() const { return (size_t)3 * Hm + RW + K1 + 1; }
  // forward scratch: h0, gi, gh, h1, hyp, yp, q (N), reset flag
  __host__ __device__ size_t fwd_floats() const { return img() + bias() + 8 * Hm + RW + K1 + N + 4; }
  // backward scratch: dhm, dhm1, dgh, shd, red, 2 x prefetched step inputs (save row + qa + dq + done)
  __host__ __device__ size_t step_in() const { return (size_t)mix_save_dim(Hm, K1, N) + N + 2; }
  __host__ __device__ size_t bwd_floats() const { return img() + bias() + 5 * Hm + RW + 4 * Hm + 2 * step_in(); }
};

__device__ __forceinline__ const float* mixer_image_row(const float* __restrict__ P, const MixOff& o, const MixSeqGeo& g,
                                                        int r) {
  const int M3 = 3 * g.Hm;
  if (r < M3) return P + o.gWhh + (int64_t)r * g.Hm;
  if (r < M3 + g.NK) return P + o.w1W + (int64_t)(r - M3) * g.Hm;
  if (r < M3 + g.NK + g.K1) return P + o.b1W + (int64_t)(r - M3 - g.NK) * g.Hm;
  if (r < M3 + g.NK + 2 * g.K1) return P + o.w2W + (int64_t)(r - M3 - g.NK - g.K1) * g.Hm;
  return P + o.b2aW + (int64_t)(r - M3 - g.NK - 2 * g.K1) * g.Hm;
}

// One wave copies one row at a time (lane = column): every wave keeps 32 rows' loads in flight before
// the LDS stores, so the staging costs ~rows / (32 * waves) memory round trips, not one per element.
__device__ void stage_mixer_image(const float* __restrict__ P, const MixOff& o, const MixSeqGeo& g, float* img) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const bool on = lane < g.Hm;
  for (int r0 = w * 32; r0 < g.rows; r0 += nw * 32) {
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const int r = r0 + j;
      v[j] = (on && r < g.rows) ? mixer_image_row(P, o, g, r)[lane] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 32; ++j)
      if (on && r0 + j < g.rows) img[(r0 + j) * g.ld + lane] = v[j];
  }
  __syncthreads();
}

__device__ void stage_mixer_bias(const float* __restrict__ P, const MixOff& o, const MixSeqGeo& g, float* bs) {
  const int M3 = 3 * g.Hm, NK = g.NK, K1 = g.K1;
  for (int i = threadIdx.x; i < (int)g.bias(); i += blockDim.x) {
    float v;
    if (i < M3) v = P[o.gbhh + i];
    else if (i < M3 + NK) v = P[o.w1b + i - M3];
    else if (i < M3 + NK + K1) v = P[o.b1b + i - M3 - NK];
    else if (i < M3 + NK + 2 * K1) v = P[o.w2b + i - M3 - NK - K1];
    else if (i < M3 + NK + 3 * K1) v = P[o.b2ab + i - M3 - NK - 2 * K1];
    else if (i < M3 + NK + 4 * K1) v = P[o.b2bW + i - M3 - NK - 3 * K1];
    else v = P[o.b2bb];
    bs[i] = v;
  }
}

struct MixFwdSeq {
  int C;
  int64_t gi_st, q_st, qtot_st, save_st, hout_st;
  const uint8_t* reset_steps;  // [C-1][B]: reset flags of steps t >= 1 (step 0 uses net.reset / h_in)
};

__device__ __forceinline__ void mixer_fwd_seq_body(const MixFwdArgs& a, const MixFwdNet& nt, const MixFwdSeq& sq) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x;
  const int S = a.S, Hm = a.Hm, K1 = a.K1, N = a.N;
  const MixOff o = mix_offsets(S, Hm, K1, N);
  const MixSeqGeo g(Hm, K1, N);
  const int NK = g.NK, RW = g.RW, ld = g.ld, M3 = 3 * Hm;
  float* img = sm;
  float* bs = img + g.img();   // biases (stage_mixer_bias)
  float* h0 = bs + g.bias();   // [Hm]
  float* gi = h0 + Hm;         // [3Hm] this step's input projection
  float* gh = gi + 3 * Hm;     // [3Hm]
  float* h1 = gh + 3 * Hm;     // [Hm]
  float* hyp = h1 + Hm;        // [RW]
  float* yp = hyp + RW;        // [K1]
  float* qs = yp + K1;         // [N] this step's agent values
  float* rst = qs + N;         // [1] reset flag of the next step
  stage_mixer_image(nt.P, o, g, img);
  stage_mixer_bias(nt.P, o, g, bs);
  const float* b_hh = bs;
  const float* b_hy = bs + M3;
  const float* b2w = bs + M3 + RW;
  const int svd = mix_save_dim(Hm, K1, N);
  {
    const bool rz = !nt.h_in || (nt.reset && nt.reset[b]);
    for (int i = threadIdx.x; i < Hm; i += blockDim.x) h0[i] = rz ? 0.f : nt.h_in[(int64_t)b * Hm + i];
    for (int i = threadIdx.x; i < M3; i += blockDim.x) gi[i] = nt.gi[(int64_t)b * M3 + i];
    for (int i = threadIdx.x; i < N; i += blockDim.x) qs[i] = nt.q[(int64_t)b * N + i];
  }
  __syncthreads();
  for (int t = 0; t < sq.C; ++t) {
    // prefetch step t+1's inputs into registers (written to LDS after their last use in step t)
    const bool more = t + 1 < sq.C;
    const int ti = (int)threadIdx.x;
    const float g_nx = (more && ti < M3) ? nt.gi[(t + 1) * sq.gi_st + (int64_t)b * M3 + ti] : 0.f;
    const float q_nx = (more && ti < N) ? nt.q[(t + 1) * sq.q_st + (int64_t)b * N + ti] : 0.f;
    const float r_nx = (more && ti == 0) ? (sq.reset_steps[(int64_t)t * a.B + b] != 0 ? 1.f : 0.f) : 0.f;
    // gh = W_hh h0 + b_hh (block_matvec order: sequential k, bias last)
    for (int r = threadIdx.x; r < M3; r += blockDim.x) gh[r] = dot_seq_n(img + r * ld, h0, Hm, 0.f) + b_hh[r];
    lds_sync();
    float* sv = nt.save ? nt.save + t * sq.save_st + (int64_t)b * svd : nullptr;
    float* hout = nt.h_out ? nt.h_out + t * sq.hout_st : nullptr;
    for (int i = threadIdx.x; i < Hm; i += blockDim.x) {
      const float r = sigmoidf_(gi[i] + gh[i]);
      const float z = sigmoidf_(gi[Hm + i] + gh[Hm + i]);
      const float n = tanhf_(gi[2 * Hm + i] + r * gh[2 * Hm + i]);
      const float hv = n + z * (h0[i] - n);
      h1[i] = hv;
      if (hout) hout[(int64_t)b * Hm + i] = hv;
      if (sv) {
        sv[i] = h0[i];
        sv[Hm + i] = r;
        sv[2 * Hm + i] = z;
        sv[3 * Hm + i] = n;
        sv[4 * Hm + i] = gh[2 * Hm + i];
        sv[5 * Hm + i] = hv;
      }
    }
    lds_sync();
    // hypernets on h1 (rows w1 [NK] | b1 [K1] | w2 [K1] | b2 hidden [K1]), each row's bias last
    for (int r = threadIdx.x; r < RW; r += blockDim.x) hyp[r] = dot_seq_n(img + (M3 + r) * ld, h1, Hm, 0.f) + b_hy[r];
    lds_sync();
    for (int k = threadIdx.x; k < K1; k += blockDim.x) {
      float acc = 0.f;
      for (int i = 0; i < N; ++i) acc += fabsf(hyp[k * N + i]) * qs[i];
      yp[k] = acc + hyp[NK + k];
    }
    lds_sync();
    if (threadIdx.x == 0) {
      const float* w2raw = hyp + NK + K1;
      const float* b2pre = hyp + NK + 2 * K1;
      float b2 = 0.f;
      for (int k = 0; k < K1; ++k) b2 += b2w[k] * fmaxf(b2pre[k], 0.f);
      b2 += b2w[K1];
      float acc = 0.f;
      for (int k = 0; k < K1; ++k) acc += fabsf(w2raw[k]) * fmaxf(yp[k], 0.f);
      nt.qtot[t * sq.qtot_st + b] = acc + b2;
      if (sv) sv[6 * Hm + NK + 4 * K1] = b2;
    }
    if (sv) {
      for (int i = threadIdx.x; i < RW; i += blockDim.x) sv[6 * Hm + i] = i >= NK + 2 * K1 ? fmaxf(hyp[i], 0.f) : hyp[i];
      for (int k = threadIdx.x; k < K1; k += blockDim.x) sv[6 * Hm + NK + 3 * K1 + k] = yp[k];
    }
    // next step's inputs (gi / q were last read above); h0 <- h1 unless the next step resets
    if (more) {
      if (ti < M3) gi[ti] = g_nx;
      if (ti < N) qs[ti] = q_nx;
      if (ti == 0) rst[0] = r_nx;
    }
    lds_sync();
    if (more) {
      const bool rz = rst[0] != 0.f;
      for (int i = threadIdx.x; i < Hm; i += blockDim.x) h0[i] = rz ? 0.f : h1[i];
    }
    lds_sync();
  }
}

// one inlined body per net: each reads its own kernel-argument fields with scalar loads
__global__ __launch_bounds__(256) void mixer_fwd_seq_lds_kernel(MixFwdArgs a, MixFwdSeq sq) {
  if (blockIdx.y == 0)
    mixer_fwd_seq_body(a, a.net[0], sq);
  else
    mixer_fwd_seq_body(a, a.net[1], sq);
}

// ------------------------------------------------------------------ loss (all steps at once)
// y = w * sum_i (r_i + gamma*(1-d)*Q'tot)   (qmix/_train.py:80-82, vdn/_train.py:76-77)
// dQtot = 2 (Qtot - y) / B ;  loss = sum_t mean_b (y - Qtot)^2 ;  td = |y - Qtot| at t = C-1.
// VDN (mix_sum): Qtot = sum_i qa_i, Q'tot = sum_i maxq'_i, dqa_i = dQtot.
// flags: MM_LOSS_MIX_SUM (VDN), MM_LOSS_HUBER (smooth_l1, beta 1: qmix/qmix.py:218),
// MM_LOSS_TARGET_SUM (y = sum_i r_i + gamma*(1-d)*Q'tot: qmix/qmix.py:215-217, no xN, no IS weight).
__device__ __forceinline__ void lrn_loss_elem(int i, int B, int C, int N, float gamma, const float* rew,
                                              const float* done, const float* isw, const float* qtot,
                                              const float* qtot_t, int flags, const float* qa, const float* maxq,
                                              float* dq, float* dqa, float* loss_parts, float* td_last) {
  const int mix_sum = flags & MM_LOSS_MIX_SUM;
  const int b = i % B, t = i / B;
  float qt, qn;
  if (mix_sum) {
    qt = 0.f;
    qn = 0.f;
    for (int k = 0; k < N; ++k) {
      qt += qa[(int64_t)i * N + k];
      qn += maxq[(int64_t)i * N + k];
    }
  } else {
    qt = qtot[i];
    qn = qtot_t[i];
  }
  float y;
  if (flags & MM_LOSS_TARGET_SUM) {
    float rs = 0.f;
    for (int k = 0; k < N; ++k) rs += rew[(int64_t)i * N + k];
    y = rs + gamma * qn * (1.0f - done[i]);
  } else {
    const float boot = gamma * (1.0f - done[i]) * qn;
    float acc = 0.f;
    for (int k = 0; k < N; ++k) acc += rew[(int64_t)i * N + k] + boot;
    y = isw[b] * acc;
  }
  const float diff = qt - y;
  float g, part;
  if (flags & MM_LOSS_HUBER) {
    const float ad = fabsf(diff);
    g = (ad < 1.0f ? diff : copysignf(1.0f, diff)) / (float)B;
    part = ad < 1.0f ? 0.5f * diff * diff : ad - 0.5f;
  } else {
    g = 2.0f * diff / (float)B;
    part = diff * diff;
  }
  dq[i] = g;
  if (mix_sum)
    for (int k = 0; k < N; ++k) dqa[(int64_t)i * N + k] = g;
  loss_parts[i] = part;
  if (t == C - 1) td_last[b] = fabsf(diff);
}
__global__ void lrn_loss_kernel(int B, int C, int N, float gamma, const float* rew, const float* done,
                                const float* isw, const float* qtot, const float* qtot_t, int flags,
                                const float* qa, const float* maxq, float* dq, float* dqa, float* loss_parts,
                                float* td_last) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * C) lrn_loss_elem(i, B, C, N, gamma, rew, done, isw, qtot, qtot_t, flags, qa, maxq, dq, dqa, loss_parts, td_last);
}

// loss = sum_t (1/B) sum_b parts (logging value): small batches one thread per step t summing its
// B parts in order; large batches (B > 256) a strided per-thread sum + fixed-shape tree per step.
// Steps accumulated in order by thread 0 (deterministic either way).
__global__ __launch_bounds__(256) void lrn_loss_reduce_kernel(int B, int C, const float* parts, float* loss) {
  __shared__ float sh[256];
  if (B <= 256) {
    for (int t = threadIdx.x; t < C; t += 256) {
      float s = 0.f;
      for (int b = 0; b < B; ++b) s += parts[(int64_t)t * B + b];
      if (t < 256) sh[t] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float tot = 0.f;
      for (int t = 0; t < C && t < 256; ++t) tot += sh[t] / (float)B;
      for (int t = 256; t < C; ++t) {
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += parts[(int64_t)t * B + b];
        tot += s / (float)B;
      }
      *loss = tot;
    }
    return;
  }
  float tot = 0.f;
  for (int t = 0; t < C; ++t) {
    float s = 0.f;
#pragma unroll 16
    for (int b = threadIdx.x; b < B; b += 256) s += parts[(int64_t)t * B + b];   // (loads issued ahead, adds in order)
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
      __syncthreads();
    }
    tot += sh[0] / (float)B;
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = tot;
}

// Small batches (B * C <= 1024, B <= 256): the loss terms and the per-step in-order reduction in ONE
// workgroup (the parts go through global memory inside the block: same values, same summation order as
// lrn_loss_kernel + lrn_loss_reduce_kernel, one launch fewer per update).
struct LossArgs {
  int B, C, N;
  float gamma;
  const float *rew, *done, *isw, *qtot, *qtot_t;
  int flags;
  const float *qa, *maxq;
  float *dq, *dqa, *loss_parts, *td_last, *loss;
};
// one block, any size (B <= 256, C <= 256, B * C rows grid-strided over the block)
__device__ __forceinline__ void lrn_loss_small_body(const LossArgs& a) {
  __shared__ float sh[256];
  for (int i = threadIdx.x; i < a.B * a.C; i += blockDim.x)
    lrn_loss_elem(i, a.B, a.C, a.N, a.gamma, a.rew, a.done, a.isw, a.qtot, a.qtot_t, a.flags, a.qa, a.maxq, a.dq,
                  a.dqa, a.loss_parts, a.td_last);
  __syncthreads();
  for (int t = threadIdx.x; t < a.C; t += blockDim.x) {
    float sacc = 0.f;
    for (int b = 0; b < a.B; ++b) sacc += a.loss_parts[(int64_t)t * a.B + b];
    sh[t] = sacc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int t = 0; t < a.C; ++t) tot += sh[t] / (float)a.B;
    *a.loss = tot;
  }
}
__global__ __launch_bounds__(1024) void lrn_loss_small_kernel(LossArgs a) { lrn_loss_small_body(a); }

// ------------------------------------------------------------------ mixer backward (one step)
struct MixBwdArgs {
  const float* P;        // behavior mixer params
  const float* save;     // [B][MSD] of this step
  const float* qa;       // [B][N] of this step
  const float* dq;       // [B] dQtot of this step
  const float* done;     // [B] done of THIS step (1 => drop the future gradient)
  float* dhm;            // [B][Hm] in: grad wrt hm1 from step t+1 ; out: grad wrt hm0 (for step t-1)
  float* dqa;            // [B][N] out
  float* delta;          // [B][MDD] out: [dgi 3Hm | dgh 3Hm | dw1raw N*K1 | db1 K1 | dw2raw K1 | db2pre K1 | dQ 1]
  int B, N, S, Hm, K1;
};
__host__ __device__ inline int mix_delta_dim(int Hm, int K1, int N) { return 6 * Hm + N * K1 + 3 * K1 + 1; }

__device__ __forceinline__ void mixer_bwd_body(const MixBwdArgs& a, int b);

__global__ __launch_bounds__(256) void mixer_bwd_kernel(MixBwdArgs a) { mixer_bwd_body(a, blockIdx.x); }

// Chunk-sequence launch: all C steps backwards in one launch (block = one sample; dhm carried by
// the same threads), step t's pointers = step-0 ones + t * stride.
// done of step t: ones at t = C-1 (no future), else done + t * done_st.
struct MixBwdSeq {
  int C;
  int64_t save_st, qa_st, dq_st, done_st, dqa_st, delta_st;
  const float* ones;
};
__global__ __launch_bounds__(256) void mixer_bwd_seq_kernel(MixBwdArgs a, MixBwdSeq sq) {
  for (int t = sq.C - 1; t >= 0; --t) {
    MixBwdArgs x = a;
    x.save += t * sq.save_st;
    x.qa += t * sq.qa_st;
    x.dq += t * sq.dq_st;
    x.done = t == sq.C - 1 ? sq.ones : a.done + t * sq.done_st;
    x.dqa += t * sq.dqa_st;
    x.delta += t * sq.delta_st;
    mixer_bwd_body(x, blockIdx.x);
    __syncthreads();
  }
}

__device__ __forceinline__ void mixer_bwd_body(const MixBwdArgs& a, int b) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Hm = a.Hm, K1 = a.K1, N = a.N;
  const MixOff o = mix_offsets(a.S, Hm, K1, N);
  const float* sv = a.save + (int64_t)b * mix_save_dim(Hm, K1, N);
  const float* hm0 = sv;
  const float* rg = sv + Hm;
  const float* zg = sv + 2 * Hm;
  const float* ng = sv + 3 * Hm;
  const float* anh = sv + 4 * Hm;
  const float* w1raw = sv + 6 * Hm;
  const float* w2raw = w1raw + N * K1 + K1;
  const float* b2pre = w2raw + K1;
  const float* ypre = b2pre + K1;
  float* dl = a.delta + (int64_t)b * mix_delta_dim(Hm, K1, N);
  float* d_w1 = dl + 6 * Hm;         // [N*K1]
  float* d_b1 = d_w1 + N * K1;       // [K1]
  float* d_w2 = d_b1 + K1;           // [K1]
  float* d_b2pre = d_w2 + K1;        // [K1]
  float* dhm1 = sm;                  // [Hm]
  float* dgh = dhm1 + Hm;            // [3Hm]
  float* shd = dgh + 3 * Hm;         // [N*K1 + 3*K1] local copy of the hypernet deltas
  float* red = shd + N * K1 + 3 * K1;  // [4*Hm] wave partials of the transposed mat-vecs
  const float dQ = a.dq[b];
  // hypernet / mixing deltas
  for (int k = threadIdx.x; k < K1; k += blockDim.x) {
    const float y = fmaxf(ypre[k], 0.f);
    const float w2 = w2raw[k];
    const float dw2 = dQ * y * (w2 > 0.f ? 1.f : (w2 < 0.f ? -1.f : 0.f));
    const float dyp = ypre[k] > 0.f ? dQ * fabsf(w2) : 0.f;
    const float db2p = b2pre[k] > 0.f ? dQ * a.P[o.b2bW + k] : 0.f;
    d_b1[k] = dyp;
    d_w2[k] = dw2;
    d_b2pre[k] = db2p;
    shd[N * K1 + k] = dyp;
    shd[N * K1 + K1 + k] = dw2;
    shd[N * K1 + 2 * K1 + k] = db2p;
    for (int i = 0; i < N; ++i) {
      const float w = w1raw[k * N + i];
      const float dw1 = dyp * a.qa[(int64_t)b * N + i] * (w > 0.f ? 1.f : (w < 0.f ? -1.f : 0.f));
      d_w1[k * N + i] = dw1;
      shd[k * N + i] = dw1;
    }
  }
  if (threadIdx.x == 0) dl[6 * Hm + N * K1 + 3 * K1] = dQ;
  __syncthreads();
  // dqa_i = sum_k dy_pre_k |W1[k,i]|
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    float acc = 0.f;
    for (int k = 0; k < K1; ++k) acc += shd[N * K1 + k] * fabsf(w1raw[k * N + i]);
    a.dqa[(int64_t)b * N + i] = acc;
  }
  // dhm1 = (future grad unless done) + hypernet input grads
  const bool drop = a.done[b] > 0.5f;
  for (int c = threadIdx.x; c < Hm; c += blockDim.x) dhm1[c] = drop ? 0.f : a.dhm[(int64_t)b * Hm + c];
  __syncthreads();
  block_matvec_t(a.P + o.w1W, N * K1, Hm, shd, dhm1, true, red);
  block_matvec_t(a.P + o.b1W, K1, Hm, shd + N * K1, dhm1, true, red);
  block_matvec_t(a.P + o.w2W, K1, Hm, shd + N * K1 + K1, dhm1, true, red);
  block_matvec_t(a.P + o.b2aW, K1, Hm, shd + N * K1 + 2 * K1, dhm1, true, red);
  // GRU backward (h' = n + z (h - n))
  for (int i = threadIdx.x; i < Hm; i += blockDim.x) {
    const float dh = dhm1[i];
    const float r = rg[i], z = zg[i], n = ng[i];
    const float dn = dh * (1.f - z);
    const float dz = dh * (hm0[i] - n);
    const float dpn = dn * (1.f - n * n);
    const float dr = dpn * anh[i];
    const float dar = dr * r * (1.f - r);
    const float daz = dz * z * (1.f - z);
    dl[i] = dar;
    dl[Hm + i] = daz;
    dl[2 * Hm + i] = dpn;
    dl[3 * Hm + i] = dar;
    dl[4 * Hm + i] = daz;
    dl[5 * Hm + i] = dpn * r;
    dgh[i] = dar;
    dgh[Hm + i] = daz;
    dgh[2 * Hm + i] = dpn * r;
  }
  __syncthreads();
  // dhm0 = z * dhm1 + W_hh^T dgh
  for (int c = threadIdx.x; c < Hm; c += blockDim.x) shd[c] = dhm1[c] * zg[c];
  __syncthreads();
  block_matvec_t(a.P + o.gWhh, 3 * Hm, Hm, dgh, shd, true, red);
  for (int c = threadIdx.x; c < Hm; c += blockDim.x) a.dhm[(int64_t)b * Hm + c] = shd[c];
}

// block_matvec_t for MIX_SPB samples at once: out[q][c] += sum_r W[r][c] d[q][r]; every W element
// read serves all samples. Per sample the partial-sum order is block_matvec_t's (bit-identical).
// red: [MIX_SPB][nw][K] floats.
template <bool ACC = true>
__device__ __forceinline__ void block_matvec_t_multi(const float* __restrict__ W, int rows, int K, const float* d, int ds,
                                     float* out, int os, float* red) {
  constexpr int Q = MIX_SPB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int c = lane; c < K; c += 64) {
    float a0[Q], a1[Q], a2[Q], a3[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) a0[q] = a1[q] = a2[q] = a3[q] = 0.f;
    int r = w;
    for (; r + 3 * nw < rows; r += 4 * nw) {
      const float w0 = W[(int64_t)r * K + c], w1 = W[(int64_t)(r + nw) * K + c];
      const float w2 = W[(int64_t)(r + 2 * nw) * K + c], w3 = W[(int64_t)(r + 3 * nw) * K + c];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const float* dq = d + q * ds;
        a0[q] += w0 * dq[r];
        a1[q] += w1 * dq[r + nw];
        a2[q] += w2 * dq[r + 2 * nw];
        a3[q] += w3 * dq[r + 3 * nw];
      }
    }
    for (; r < rows; r += nw) {
      const float w0 = W[(int64_t)r * K + c];
#pragma unroll
      for (int q = 0; q < Q; ++q) a0[q] += w0 * d[q * ds + r];
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) red[(q * nw + w) * K + c] = (a0[q] + a1[q]) + (a2[q] + a3[q]);
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < Q * K; idx += blockDim.x) {
    const int q = idx / K, c = idx % K;
    float acc = 0.f;
    for (int v = 0; v < nw; ++v) acc += red[(q * nw + v) * K + c];
    if (ACC)
      out[q * os + c] += acc;
    else
      out[q * os + c] = acc;
  }
  __syncthreads();
}

// Chunk-sequence mixer backward with MIX_SPB samples per block (B >= 512): the per-sample math of
// mixer_bwd_body in the same order, the transposed mat-vecs shared over the block's samples.
__global__ __launch_bounds__(256) void mixer_bwd_seq_multi_kernel(MixBwdArgs a0, MixBwdSeq sq) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int Q = MIX_SPB;
  const int Hm = a0.Hm, K1 = a0.K1, N = a0.N, NK = N * K1, SH = NK + 3 * K1;
  const MixOff o = mix_offsets(a0.S, Hm, K1, N);
  const int b0 = blockIdx.x * Q;
  const int ns = min(Q, a0.B - b0);
  float* dhm1 = sm;                 // [Q][Hm]
  float* dgh = dhm1 + Q * Hm;       // [Q][3Hm]
  float* shd = dgh + Q * 3 * Hm;    // [Q][SH]
  float* red = shd + Q * SH;        // [Q][nw][Hm]
  const int svd = mix_save_dim(Hm, K1, N), dld = mix_delta_dim(Hm, K1, N);
  for (int t = sq.C - 1; t >= 0; --t) {
    const float* save = a0.save + t * sq.save_st;
    const float* qa = a0.qa + t * sq.qa_st;
    const float* dqv = a0.dq + t * sq.dq_st;
    const float* done = t == sq.C - 1 ? sq.ones : a0.done + t * sq.done_st;
    float* dqa = a0.dqa + t * sq.dqa_st;
    float* delta = a0.delta + t * sq.delta_st;
    // hypernet / mixing deltas
    for (int idx = threadIdx.x; idx < ns * K1; idx += blockDim.x) {
      const int s = idx / K1, k = idx % K1, b = b0 + s;
      const float* w1raw = save + (int64_t)b * svd + 6 * Hm;
      const float* w2raw = w1raw + NK + K1;
      const float* b2pre = w2raw + K1;
      const float* ypre = b2pre + K1;
      float* dl = delta + (int64_t)b * dld;
      float* sh = shd + s * SH;
      const float dQ = dqv[b];
      const float y = fmaxf(ypre[k], 0.f);
      const float w2 = w2raw[k];
      const float dw2 = dQ * y * (w2 > 0.f ? 1.f : (w2 < 0.f ? -1.f : 0.f));
      const float dyp = ypre[k] > 0.f ? dQ * fabsf(w2) : 0.f;
      const float db2p = b2pre[k] > 0.f ? dQ * a0.P[o.b2bW + k] : 0.f;
      dl[6 * Hm + NK + k] = dyp;
      dl[6 * Hm + NK + K1 + k] = dw2;
      dl[6 * Hm + NK + 2 * K1 + k] = db2p;
      sh[NK + k] = dyp;
      sh[NK + K1 + k] = dw2;
      sh[NK + 2 * K1 + k] = db2p;
      for (int i = 0; i < N; ++i) {
        const float wv = w1raw[k * N + i];
        const float dw1 = dyp * qa[(int64_t)b * N + i] * (wv > 0.f ? 1.f : (wv < 0.f ? -1.f : 0.f));
        dl[6 * Hm + k * N + i] = dw1;
        sh[k * N + i] = dw1;
      }
    }
    if ((int)threadIdx.x < ns) {
      const int b = b0 + threadIdx.x;
      delta[(int64_t)b * dld + 6 * Hm + NK + 3 * K1] = dqv[b];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < ns * N; idx += blockDim.x) {
      const int s = idx / N, i = idx % N, b = b0 + s;
      const float* w1raw = save + (int64_t)b * svd + 6 * Hm;
      float acc = 0.f;
      for (int k = 0; k < K1; ++k) acc += shd[s * SH + NK + k] * fabsf(w1raw[k * N + i]);
      dqa[(int64_t)b * N + i] = acc;
    }
    for (int idx = threadIdx.x; idx < Q * Hm; idx += blockDim.x) {
      const int s = idx / Hm, c = idx % Hm, b = b0 + s;
      dhm1[idx] = (s >= ns || done[b] > 0.5f) ? 0.f : a0.dhm[(int64_t)b * Hm + c];
    }
    __syncthreads();
    block_matvec_t_multi(a0.P + o.w1W, NK, Hm, shd, SH, dhm1, Hm, red);
    block_matvec_t_multi(a0.P + o.b1W, K1, Hm, shd + NK, SH, dhm1, Hm, red);
    block_matvec_t_multi(a0.P + o.w2W, K1, Hm, shd + NK + K1, SH, dhm1, Hm, red);
    block_matvec_t_multi(a0.P + o.b2aW, K1, Hm, shd + NK + 2 * K1, SH, dhm1, Hm, red);
    // GRU backward (h' = n + z (h - n))
    for (int idx = threadIdx.x; idx < Q * Hm; idx += blockDim.x) {
      const int s = idx / Hm, i = idx % Hm, b = b0 + s;
      if (s >= ns) {
        dgh[s * 3 * Hm + i] = dgh[s * 3 * Hm + Hm + i] = dgh[s * 3 * Hm + 2 * Hm + i] = 0.f;
        continue;
      }
      const float* sv = save + (int64_t)b * svd;
      const float dh = dhm1[idx];
      const float r = sv[Hm + i], z = sv[2 * Hm + i], n = sv[3 * Hm + i];
      const float dn = dh * (1.f - z);
      const float dz = dh * (sv[i] - n);
      const float dpn = dn * (1.f - n * n);
      const float dr = dpn * sv[4 * Hm + i];
      const float dar = dr * r * (1.f - r);
      const float daz = dz * z * (1.f - z);
      float* dl = delta + (int64_t)b * dld;
      dl[i] = dar;
      dl[Hm + i] = daz;
      dl[2 * Hm + i] = dpn;
      dl[3 * Hm + i] = dar;
      dl[4 * Hm + i] = daz;
      dl[5 * Hm + i] = dpn * r;
      dgh[s * 3 * Hm + i] = dar;
      dgh[s * 3 * Hm + Hm + i] = daz;
      dgh[s * 3 * Hm + 2 * Hm + i] = dpn * r;
      shd[s * SH + i] = dh * z;   // dhm0 direct path (hypernet deltas are consumed)
    }
    __syncthreads();
    block_matvec_t_multi(a0.P + o.gWhh, 3 * Hm, Hm, dgh, 3 * Hm, shd, SH, red);
    for (int idx = threadIdx.x; idx < ns * Hm; idx += blockDim.x) {
      const int s = idx / Hm, c = idx % Hm;
      a0.dhm[(int64_t)(b0 + s) * Hm + c] = shd[s * SH + c];
    }
    __syncthreads();
  }
}

// block_matvec_t over an LDS row-major image with row stride ld (same partial-sum order).
__device__ void block_matvec_t_ld(const float* W, int ld, int rows, int K, const float* d, float* out, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int c = lane; c < K; c += 64) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int r = w;
#pragma unroll 4
    for (; r + 3 * nw < rows; r += 4 * nw) {
      a0 += W[r * ld + c] * d[r];
      a1 += W[(r + nw) * ld + c] * d[r + nw];
      a2 += W[(r + 2 * nw) * ld + c] * d[r + 2 * nw];
      a3 += W[(r + 3 * nw) * ld + c] * d[r + 3 * nw];
    }
    for (; r < rows; r += nw) a0 += W[r * ld + c] * d[r];
    red[w * K + c] = (a0 + a1) + (a2 + a3);
  }
  lds_sync();
  for (int c = threadIdx.x; c < K; c += blockDim.x) {
    float acc = 0.f;
    for (int q = 0; q < nw; ++q) acc += red[q * K + c];
    out[c] = out[c] + acc;
  }
  lds_sync();
}

__global__ __launch_bounds__(256) void mixer_bwd_seq_lds_kernel(MixBwdArgs a, MixBwdSeq sq) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x;
  const int Hm = a.Hm, K1 = a.K1, N = a.N;
  const MixOff o = mix_offsets(a.S, Hm, K1, N);
  const MixSeqGeo g(Hm, K1, N);
  const int NK = g.NK, ld = g.ld, M3 = 3 * Hm;
  const int svd = mix_save_dim(Hm, K1, N), dld = mix_delta_dim(Hm, K1, N), SI = (int)g.step_in();
  float* img = sm;
  float* bs = img + g.img();
  float* dhm = bs + g.bias();   // [Hm] carried: grad wrt hm1 of step t (from step t+1)
  float* dhm1 = dhm + Hm;       // [Hm]
  float* dgh = dhm1 + Hm;       // [3Hm]
  float* shd = dgh + 3 * Hm;    // [RW]
  float* red = shd + g.RW;      // [4][Hm]
  float* inb = red + 4 * Hm;    // [2][SI]: step inputs (save row | qa [N] | dQ | done), double-buffered
  const float* b2w = bs + M3 + g.RW;
  stage_mixer_image(a.P, o, g, img);
  stage_mixer_bias(a.P, o, g, bs);
  const int ti = (int)threadIdx.x;
  auto step_ptr = [&](int t, int i) -> float {   // element i of step t's input block (global)
    if (i < svd) return a.save[t * sq.save_st + (int64_t)b * svd + i];
    i -= svd;
    if (i < N) return a.qa[t * sq.qa_st + (int64_t)b * N + i];
    if (i == N) return a.dq[t * sq.dq_st + b];
    const float* done = t == sq.C - 1 ? sq.ones : a.done + t * sq.done_st;
    return done[b];
  };
  for (int i = ti; i < SI; i += blockDim.x) inb[((sq.C - 1) & 1) * SI + i] = step_ptr(sq.C - 1, i);
  for (int c = ti; c < Hm; c += blockDim.x) dhm[c] = a.dhm[(int64_t)b * Hm + c];
  __syncthreads();
  for (int t = sq.C - 1; t >= 0; --t) {
    // prefetch step t-1's inputs into registers (stored to the other buffer at the end of the step)
    float nx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = ti + j * 256;
      nx[j] = (t > 0 && i < SI) ? step_ptr(t - 1, i) : 0.f;
    }
    const float* sv = inb + (t & 1) * SI;
    const float* qa = sv + svd;
    const float dQ = qa[N];
    const float done_b = qa[N + 1];
    float* dqa = a.dqa + t * sq.dqa_st;
    float* dl = a.delta + t * sq.delta_st + (int64_t)b * dld;
    const float* hm0 = sv;
    const float* rg = sv + Hm;
    const float* zg = sv + 2 * Hm;
    const float* ng = sv + 3 * Hm;
    const float* anh = sv + 4 * Hm;
    const float* w1raw = sv + 6 * Hm;
    const float* w2raw = w1raw + NK + K1;
    const float* b2pre = w2raw + K1;
    const float* ypre = b2pre + K1;
    float* d_w1 = dl + 6 * Hm;
    float* d_b1 = d_w1 + NK;
    float* d_w2 = d_b1 + K1;
    float* d_b2pre = d_w2 + K1;
    for (int k = ti; k < K1; k += blockDim.x) {
      const float y = fmaxf(ypre[k], 0.f);
      const float w2 = w2raw[k];
      const float dw2 = dQ * y * (w2 > 0.f ? 1.f : (w2 < 0.f ? -1.f : 0.f));
      const float dyp = ypre[k] > 0.f ? dQ * fabsf(w2) : 0.f;
      const float db2p = b2pre[k] > 0.f ? dQ * b2w[k] : 0.f;
      d_b1[k] = dyp;
      d_w2[k] = dw2;
      d_b2pre[k] = db2p;
      shd[NK + k] = dyp;
      shd[NK + K1 + k] = dw2;
      shd[NK + 2 * K1 + k] = db2p;
      for (int i = 0; i < N; ++i) {
        const float w = w1raw[k * N + i];
        const float dw1 = dyp * qa[i] * (w > 0.f ? 1.f : (w < 0.f ? -1.f : 0.f));
        d_w1[k * N + i] = dw1;
        shd[k * N + i] = dw1;
      }
    }
    if (ti == 0) dl[6 * Hm + NK + 3 * K1] = dQ;
    lds_sync();
    for (int i = ti; i < N; i += blockDim.x) {
      float acc = 0.f;
      for (int k = 0; k < K1; ++k) acc += shd[NK + k] * fabsf(w1raw[k * N + i]);
      dqa[(int64_t)b * N + i] = acc;
    }
    const bool drop = done_b > 0.5f;
    for (int c = ti; c < Hm; c += blockDim.x) dhm1[c] = drop ? 0.f : dhm[c];
    lds_sync();
    block_matvec_t_ld(img + M3 * ld, ld, NK, Hm, shd, dhm1, red);
    block_matvec_t_ld(img + (M3 + NK) * ld, ld, K1, Hm, shd + NK, dhm1, red);
    block_matvec_t_ld(img + (M3 + NK + K1) * ld, ld, K1, Hm, shd + NK + K1, dhm1, red);
    block_matvec_t_ld(img + (M3 + NK + 2 * K1) * ld, ld, K1, Hm, shd + NK + 2 * K1, dhm1, red);
    for (int i = ti; i < Hm; i += blockDim.x) {
      const float dh = dhm1[i];
      const float r = rg[i], z = zg[i], n = ng[i];
      const float dn = dh * (1.f - z);
      const float dz = dh * (hm0[i] - n);
      const float dpn = dn * (1.f - n * n);
      const float dr = dpn * anh[i];
      const float dar = dr * r * (1.f - r);
      const float daz = dz * z * (1.f - z);
      dl[i] = dar;
      dl[Hm + i] = daz;
      dl[2 * Hm + i] = dpn;
      dl[3 * Hm + i] = dar;
      dl[4 * Hm + i] = daz;
      dl[5 * Hm + i] = dpn * r;
      dgh[i] = dar;
      dgh[Hm + i] = daz;
      dgh[2 * Hm + i] = dpn * r;
    }
    lds_sync();
    for (int c = ti; c < Hm; c += blockDim.x) shd[c] = dhm1[c] * zg[c];
    lds_sync();
    block_matvec_t_ld(img, ld, M3, Hm, dgh, shd, red);
    for (int c = ti; c < Hm; c += blockDim.x) dhm[c] = shd[c];
    if (t > 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = ti + j * 256;
        if (i < SI) inb[((t - 1) & 1) * SI + i] = nx[j];
      }
    }
    lds_sync();
  }
  for (int c = ti; c < Hm; c += blockDim.x) a.dhm[(int64_t)b * Hm + c] = dhm[c];
}

// ------------------------------------------------------------------ split mixer sequences (B < 512)
// The mixer GRU over Hm is the only serial part of a chunk: the hypernets and the mixing read a step's
// new hidden but feed nothing back into the recurrence. So each direction runs as two launches:
//   forward : mixer_rec_fwd_kernel  (block per (sample, net): W_hh in LDS, C steps of gh + gates,
//                                    writes the hidden sequence) ->
//             mixer_hyper_fwd_kernel (all C*B rows at once, MIX_SPB rows per block: mixer_hyper_rows)
//   backward: mixer_hyper_bwd_kernel (all rows at once: hypernet deltas, dqa and the four hypernet
//                                    input-gradient mat-vecs X_j = W_j^T d_j, kept apart) ->
//             mixer_rec_bwd_kernel  (block per sample: dh = ((((future + X_0) + X_1) + X_2) + X_3),
//                                    GRU backward, dh_prev = dh z + W_hh^T dgh)
// Each value keeps mixer_fwd_body / mixer_bwd_body's arithmetic and summation order (bit-identical to
// the per-step launches). The serial kernels load a window of steps' inputs into LDS with one round
// of loads, so their step loops issue only stores (on gfx9 every load wait also drains the stores
// issued before it) and synchronise with two LDS-only barriers per step.
struct MixRecFwd {
  int C, win;
  int64_t gi_st, hout_st, save_st;
  const uint8_t* reset_steps;   // [C-1][B]: step t >= 1 starts from zero hidden where set
  uint64_t* trace;              // clock64 stamps of block 0 (MM_MIX_TRACE), nullptr normally
};
struct MixRecBwd {
  int C, win;
  int64_t save_st, delta_st, done_st;
  const float* done;   // [C][B] done of step t (t = C-1: no future, always dropped)
  const float* xws;    // [C][B][4][Hm] hypernet input gradients (mixer_hyper_bwd_kernel)
  const float* ones;   // [B] of 1.0 (done of the last step)
  uint64_t* trace;     // clock64 stamps of block 0 (MM_MIX_TRACE), nullptr normally
};

// rows x K row-major global matrix -> LDS image with row stride ld; each wave keeps 32 rows' loads in
// flight (lane = column, K <= 64 per pass). No trailing barrier.
__device__ void stage_rows(const float* __restrict__ src, int rows, int K, int ld, float* img) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int c0 = 0; c0 < K; c0 += 64) {
    const int c = c0 + lane;
    const bool on = c < K;
    for (int r0 = w * 32; r0 < rows; r0 += nw * 32) {
      float v[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = (on && r0 + j < rows) ? src[(int64_t)(r0 + j) * K + c] : 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j)
        if (on && r0 + j < rows) img[(r0 + j) * ld + c] = v[j];
    }
  }
}

// Prologue gathers. The address lambdas return a pointer to the 32-bit word to load; the loads are
// issued UNCONDITIONALLY (out-of-range lanes load the last valid element and discard it): a load
// under a branch becomes a copy at the join, and copying a pending load result forces the wave to wait
// for it, serialising one memory round trip per element.
//
// dst[row * rowlen + j] = *addr(row, j) for row < nrows, j < rowlen, by the whole block, 16 loads in
// flight per thread before their LDS stores, (row, j) stepped incrementally (no integer division).
// No trailing barrier.
template <typename A>
__device__ __forceinline__ void block_gather_rows(float* dst, int nrows, int rowlen, A addr) {
  constexpr int U = 16;
  const int bd = blockDim.x, n = nrows * rowlen;
  if (n <= 0) return;
  int row = 0, j = threadIdx.x;
  while (j >= rowlen) {
    j -= rowlen;
    ++row;
  }
  for (int base = threadIdx.x; base < n; base += U * bd) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = base + u * bd < n;
      v[u] = *addr(ok ? row : nrows - 1, ok ? j : rowlen - 1);
      j += bd;
      while (j >= rowlen) {
        j -= rowlen;
        ++row;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * bd < n) dst[base + u * bd] = v[u];
  }
}

// Register-staged gathers: every load of a prologue is issued (gather_issue: v[u] = *addr(i) for
// i = tid + u * blockDim, clamped to n - 1) before the first LDS store that consumes one
// (gather_commit: put(i, v) for i < n), so the prologue costs one memory round trip, not one per
// gather (a store waits for its load and, vmcnt being in order, for all loads issued before it).
template <int U, typename A>
__device__ __forceinline__ void gather_issue(float (&v)[U], int n, A addr) {
  if (n <= 0) return;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = min((int)(threadIdx.x + u * blockDim.x), n - 1);
    v[u] = *addr(i);
  }
}
template <int U, typename D>
__device__ __forceinline__ void gather_commit(const float (&v)[U], int n, D put) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = threadIdx.x + u * blockDim.x;
    if (i < n) put(i, v[u]);
  }
}

// LDS row strides of the W_hh images: forward rows are read along k by one lane (b128 reads: stride
// HM + 4 keeps 16-byte alignment and spreads 16 lanes over all 64 banks); backward columns are read
// along r by 64 lanes (b32 reads: stride HM + 1 is conflict-free)
template <int HM>
struct MixRecGeo {
  static constexpr int M3 = 3 * HM, LDF = HM + 4, LDB = HM + 1;
  static constexpr size_t fwd_floats(int win) {
    return (size_t)M3 * LDF + 2 * HM + 2 * M3 + (size_t)win * M3 + win + 1;
  }
  static constexpr size_t bwd_floats(int win) {
    return (((size_t)M3 * LDB + M3 + 4 * HM + 3) & ~(size_t)3) + (size_t)win * (9 * HM + 1);
  }
};
__host__ __device__ inline size_t mix_rec_fwd_floats(int Hm, int win) {
  return Hm == 32 ? MixRecGeo<32>::fwd_floats(win) : MixRecGeo<64>::fwd_floats(win);
}
__host__ __device__ inline size_t mix_rec_bwd_floats(int Hm, int win) {
  return Hm == 32 ? MixRecGeo<32>::bwd_floats(win) : MixRecGeo<64>::bwd_floats(win);
}
inline bool mix_rec_supported(int Hm) { return Hm == 32 || Hm == 64; }

// sample b of net `net` (block (b, net) of mixer_rec_fwd_kernel); sm: the block's dynamic LDS
template <int HM>
__device__ __forceinline__ void mixer_rec_fwd_body(const MixFwdArgs& a, const MixFwdNet& nt, const MixRecFwd& sq, int b,
                                                   int net, float* sm) {
  using Geo = MixRecGeo<HM>;
  constexpr int M3 = Geo::M3, LD = Geo::LDF;
  const int ti = (int)threadIdx.x;
  const MixOff o = mix_offsets(a.S, HM, a.K1, a.N);
  float* img = sm;                 // W_hh [M3][LD]
  float* hb = img + M3 * LD;       // [2][HM] hidden by step parity (already zero where the step resets)
  float* gh = hb + 2 * HM;         // [M3]
  float* bhh = gh + M3;            // [M3]
  float* gin = bhh + M3;           // [win][M3] input projections of the window's steps
  float* rs = gin + sq.win * M3;   // [win + 1] 1: step w0 + tt starts from zero hidden
  uint64_t* tr = (sq.trace && b == 0 && net == 0 && ti == 0) ? sq.trace : nullptr;
  if (tr) tr[0] = clock64();
  // prologue: W_hh image, b_hh, h_in and the first window's input projections by LDS-DMA (one round
  // trip, compact code); the reset flags by a plain load issued first
  const int nr0 = min(sq.win, sq.C) + 1;
  const int tr0 = min(max(ti, 1), sq.C - 1);
  const uint8_t* rp = sq.C > 1 ? sq.reset_steps + (int64_t)(tr0 - 1) * a.B + b : (const uint8_t*)nt.P;
  const uint8_t rflag = *rp;   // (unused when C == 1)
  glds_rows(img, M3, HM, LD, [&](int r, int j) { return nt.P + o.gWhh + r * HM + j; });
  glds_gather(bhh, M3, [&](int i) { return nt.P + o.gbhh + i; });
  const bool rz = !nt.h_in || (nt.reset && nt.reset[b]);
  if (rz) {
    for (int i = ti; i < HM; i += blockDim.x) hb[i] = 0.f;
  } else {
    glds_gather(hb, HM, [&](int i) { return nt.h_in + (int64_t)b * HM + i; });
  }
  glds_rows16(gin, min(sq.win, sq.C), M3, M3, [&](int tt) { return nt.gi + tt * sq.gi_st + (int64_t)b * M3; });
  if (ti < nr0) rs[ti] = (ti >= 1 && ti < sq.C && rflag != 0) ? 1.f : 0.f;
  const int svd = mix_save_dim(HM, a.K1, a.N);
  for (int w0 = 0; w0 < sq.C; w0 += sq.win) {
    const int wn = min(sq.win, sq.C - w0);
    if (w0 > 0) {   // later windows (the first one came with the prologue)
      __syncthreads();
      glds_rows16(gin, wn, M3, M3, [&](int tt) { return nt.gi + (w0 + tt) * sq.gi_st + (int64_t)b * M3; });
    }
    if (w0 > 0 || nr0 > (int)blockDim.x)
      for (int tt = ti; tt <= wn; tt += blockDim.x) {
        const int t = w0 + tt;
        rs[tt] = (t >= 1 && t < sq.C && sq.reset_steps[(int64_t)(t - 1) * a.B + b] != 0) ? 1.f : 0.f;
      }
    __syncthreads();
    if (tr) tr[1] = clock64();
    for (int tt = 0; tt < wn; ++tt) {
      const int t = w0 + tt;
      uint64_t* ts = tr ? tr + 4 + 4 * t : nullptr;
      const float* h0 = hb + (t & 1) * HM;
      float* h1 = hb + ((t + 1) & 1) * HM;
      if (ts) ts[0] = clock64();
      // gh = W_hh h0 + b_hh (block_matvec order: sequential k from 0, bias last), 4 k per LDS read
      for (int r = ti; r < M3; r += blockDim.x) {
        const float* wr = img + r * LD;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < HM; k += 4) {
          const float4 w4 = *reinterpret_cast<const float4*>(wr + k);
          const float4 x4 = *reinterpret_cast<const float4*>(h0 + k);
          acc += w4.x * x4.x;
          acc += w4.y * x4.y;
          acc += w4.z * x4.z;
          acc += w4.w * x4.w;
        }
        gh[r] = acc + bhh[r];
      }
      if (ts) ts[1] = clock64() + (uint64_t)gh[0] * 0;
      lds_sync();
      if (ts) ts[2] = clock64();
      const float* gI = gin + tt * M3;
      const bool zero_next = rs[tt + 1] != 0.f;
      float* sv = nt.save ? nt.save + t * sq.save_st + (int64_t)b * svd : nullptr;
      for (int i = ti; i < HM; i += blockDim.x) {
        const float r = sigmoidf_(gI[i] + gh[i]);
        const float z = sigmoidf_(gI[HM + i] + gh[HM + i]);
        const float n = tanhf_(gI[2 * HM + i] + r * gh[2 * HM + i]);
        const float h0v = h0[i];
        const float hv = n + z * (h0v - n);
        h1[i] = zero_next ? 0.f : hv;
        nt.h_out[t * sq.hout_st + (int64_t)b * HM + i] = hv;
        if (sv) {
          sv[i] = h0v;
          sv[HM + i] = r;
          sv[2 * HM + i] = z;
          sv[3 * HM + i] = n;
          sv[4 * HM + i] = gh[2 * HM + i];
          sv[5 * HM + i] = hv;
        }
      }
      if (ts) ts[3] = clock64();
      lds_sync();
    }
  }
  if (tr) tr[2] = clock64();
}

// one inlined body per net: each reads its own kernel-argument fields with scalar loads
template <int HM>
__global__ __launch_bounds__(256) void mixer_rec_fwd_kernel(MixFwdArgs a, MixRecFwd sq) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  if (blockIdx.y == 0)
    mixer_rec_fwd_body<HM>(a, a.net[0], sq, (int)blockIdx.x, 0, sm);
  else
    mixer_rec_fwd_body<HM>(a, a.net[1], sq, (int)blockIdx.x, 1, sm);
}

// all R = C*B rows of one net: the hidden sequence (h_out) -> hypernets, Q_tot, save-row tail
__device__ __forceinline__ void mixer_hyper_fwd_body(const MixFwdArgs& a, const MixFwdNet& nt, int R) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Hm = a.Hm, K1 = a.K1, RW = a.N * K1 + 3 * K1;
  const int b0 = blockIdx.x * MIX_SPB;
  const int ns = min(MIX_SPB, R - b0);
  float* h1 = sm;                    // [SPB][Hm]
  float* hyp = h1 + MIX_SPB * Hm;    // [SPB][RW]
  float* yp = hyp + MIX_SPB * RW;    // [SPB][K1]
  for (int idx = threadIdx.x; idx < MIX_SPB * Hm; idx += blockDim.x)
    h1[idx] = idx / Hm < ns ? nt.h_out[(int64_t)b0 * Hm + idx] : 0.f;
  __syncthreads();
  mixer_hyper_rows(a, nt, b0, ns, h1, hyp, yp);
}
__global__ __launch_bounds__(256) void mixer_hyper_fwd_kernel(MixFwdArgs a, int R) {
  if (blockIdx.y == 0)
    mixer_hyper_fwd_body(a, a.net[0], R);
  else
    mixer_hyper_fwd_body(a, a.net[1], R);
}
__host__ __device__ inline size_t mix_hyper_fwd_floats(int Hm, int K1, int N) {
  return (size_t)MIX_SPB * (Hm + N * K1 + 3 * K1 + K1);
}

// all R = C*B rows at once (flat row arrays: save [R][MSD], qa [R][N], dq [R], dqa [R][N],
// delta [R][MDD]): mixer_bwd_body's hypernet deltas + dqa, and X_j = W_j^T d_j (j = w1, b1, w2, b2a)
// stored apart in xws [R][4][Hm] (the serial kernel adds them to the future gradient in order).
// PER: one more block (the last) runs the small priority update (its inputs, the loss's TDs, are final here)
template <bool PER>
__global__ __launch_bounds__(256) void mixer_hyper_bwd_kernel(MixBwdArgs a, int R, float* xws, uint64_t* trace,
                                                              PerUpd pu) {
  if constexpr (PER) {
    if ((int)blockIdx.x == (int)gridDim.x - 1) {
      per_update_small_block(pu);
      return;
    }
  }
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int Q = MIX_SPB;
  const int Hm = a.Hm, K1 = a.K1, N = a.N, NK = N * K1, SH = NK + 3 * K1;
  const MixOff o = mix_offsets(a.S, Hm, K1, N);
  const int b0 = blockIdx.x * Q;
  const int ns = min(Q, R - b0);
  // the four hypernet weight matrices (w1 [NK][Hm] | b1, w2, b2a [K1][Hm]) staged in LDS by 16-byte
  // LDS-DMA (row-major: the transposed mat-vecs read a row with lane = column, conflict-free)
  float* wim = sm;                          // [SH][Hm]
  float* shd = wim + SH * Hm;               // [Q][SH]
  float* xo = shd + Q * SH;                 // [Q][4][Hm]
  float* red = xo + Q * 4 * Hm;             // [Q][4 waves][Hm]
  const int svd = mix_save_dim(Hm, K1, N), dld = mix_delta_dim(Hm, K1, N);
  uint64_t* tr = (trace && blockIdx.x == 0 && threadIdx.x == 0) ? trace : nullptr;
  if (tr) tr[0] = clock64();
  {
    const int n1 = NK * Hm / 4, n2 = K1 * Hm / 4;
    glds16_gather(wim, n1, [&](int i) { return a.P + o.w1W + 4 * i; });
    glds16_gather(wim + NK * Hm, n2, [&](int i) { return a.P + o.b1W + 4 * i; });
    glds16_gather(wim + (NK + K1) * Hm, n2, [&](int i) { return a.P + o.w2W + 4 * i; });
    glds16_gather(wim + (NK + 2 * K1) * Hm, n2, [&](int i) { return a.P + o.b2aW + 4 * i; });
  }
  for (int idx = threadIdx.x; idx < Q * SH; idx += blockDim.x) shd[idx] = 0.f;
  __syncthreads();
  if (tr) tr[1] = clock64();
  for (int idx = threadIdx.x; idx < ns * K1; idx += blockDim.x) {
    const int s = idx / K1, k = idx % K1, b = b0 + s;
    const float* w1raw = a.save + (int64_t)b * svd + 6 * Hm;
    const float* w2raw = w1raw + NK + K1;
    const float* b2pre = w2raw + K1;
    const float* ypre = b2pre + K1;
    float* dl = a.delta + (int64_t)b * dld;
    float* sh = shd + s * SH;
    const float dQ = a.dq[b];
    const float y = fmaxf(ypre[k], 0.f);
    const float w2 = w2raw[k];
    const float dw2 = dQ * y * (w2 > 0.f ? 1.f : (w2 < 0.f ? -1.f : 0.f));
    const float dyp = ypre[k] > 0.f ? dQ * fabsf(w2) : 0.f;
    const float db2p = b2pre[k] > 0.f ? dQ * a.P[o.b2bW + k] : 0.f;
    dl[6 * Hm + NK + k] = dyp;
    dl[6 * Hm + NK + K1 + k] = dw2;
    dl[6 * Hm + NK + 2 * K1 + k] = db2p;
    sh[NK + k] = dyp;
    sh[NK + K1 + k] = dw2;
    sh[NK + 2 * K1 + k] = db2p;
    for (int i = 0; i < N; ++i) {
      const float wv = w1raw[k * N + i];
      const float dw1 = dyp * a.qa[(int64_t)b * N + i] * (wv > 0.f ? 1.f : (wv < 0.f ? -1.f : 0.f));
      dl[6 * Hm + k * N + i] = dw1;
      sh[k * N + i] = dw1;
    }
  }
  if ((int)threadIdx.x < ns) {
    const int b = b0 + threadIdx.x;
    a.delta[(int64_t)b * dld + 6 * Hm + NK + 3 * K1] = a.dq[b];
  }
  if (tr) tr[2] = clock64();
  __syncthreads();
  if (tr) tr[3] = clock64();
  for (int idx = threadIdx.x; idx < ns * N; idx += blockDim.x) {
    const int s = idx / N, i = idx % N, b = b0 + s;
    const float* w1raw = a.save + (int64_t)b * svd + 6 * Hm;
    float acc = 0.f;
    for (int k = 0; k < K1; ++k) acc += shd[s * SH + NK + k] * fabsf(w1raw[k * N + i]);
    a.dqa[(int64_t)b * N + i] = acc;
  }
  if (tr) tr[4] = clock64();
  block_matvec_t_multi<false>(wim, NK, Hm, shd, SH, xo, 4 * Hm, red);
  if (tr) tr[5] = clock64();
  block_matvec_t_multi<false>(wim + NK * Hm, K1, Hm, shd + NK, SH, xo + Hm, 4 * Hm, red);
  block_matvec_t_multi<false>(wim + (NK + K1) * Hm, K1, Hm, shd + NK + K1, SH, xo + 2 * Hm, 4 * Hm, red);
  block_matvec_t_multi<false>(wim + (NK + 2 * K1) * Hm, K1, Hm, shd + NK + 2 * K1, SH, xo + 3 * Hm, 4 * Hm, red);
  if (tr) tr[6] = clock64();
  for (int idx = threadIdx.x; idx < ns * 4 * Hm; idx += blockDim.x) xws[(int64_t)b0 * 4 * Hm + idx] = xo[idx];
  if (tr) tr[7] = clock64();
}
__host__ __device__ inline size_t mix_hyper_bwd_floats(int Hm, int K1, int N) {
  return (size_t)(N * K1 + 3 * K1) * Hm + (size_t)MIX_SPB * (N * K1 + 3 * K1 + 4 * Hm + 4 * Hm);
}

// bid: the sample (block) index; sm: the block's dynamic LDS (mixer_rec_bwd_kernel, agent_mixer_bwd_kernel)
template <int HM>
__device__ __forceinline__ void mixer_rec_bwd_body(const MixBwdArgs& a, const MixRecBwd& sq, int bid, float* sm) {
  using Geo = MixRecGeo<HM>;
  constexpr int M3 = Geo::M3, LD = Geo::LDB, NW = 4;   // 256 threads = 4 waves
  static_assert(M3 % (4 * NW) == 0, "W_hh^T partial loop assumes 16 | 3 Hm");
  const int b = bid, ti = (int)threadIdx.x;
  const MixOff o = mix_offsets(a.S, HM, a.K1, a.N);
  const int svd = mix_save_dim(HM, a.K1, a.N), dld = mix_delta_dim(HM, a.K1, a.N);
  constexpr int SI = 9 * HM;       // per-step inputs: hm0 r z n anh (5Hm) | X_0..X_3 (4Hm); done apart
  float* img = sm;                 // W_hh [M3][LD]
  float* dgh = img + M3 * LD;      // [M3]
  float* red = dgh + M3;           // [4][HM] wave partials of W_hh^T dgh
  static_assert(SI % 4 == 0, "16-byte rows");
  float* inw = sm + ((M3 * LD + M3 + 4 * HM + 3) & ~3);   // [win][SI] (16-byte aligned)
  float* dnw = inw + sq.win * SI;  // [win] done flags
  uint64_t* tr = (sq.trace && b == 0 && ti == 0) ? sq.trace : nullptr;
  if (tr) tr[0] = clock64();
  const int lane = ti & 63, w = ti >> 6;
  // a window of step inputs: save rows (word pieces: rows are not 16-byte aligned), the X rows
  // (16-byte pieces) and the done flags
  auto load_window = [&](int w0, int wn) {
    glds_rows(inw, wn, 5 * HM, SI, [&](int tt, int j) { return a.save + (w0 + tt) * sq.save_st + (int64_t)b * svd + j; });
    glds_rows16(inw + 5 * HM, wn, 4 * HM, SI, [&](int tt) { return sq.xws + ((int64_t)(w0 + tt) * a.B + b) * 4 * HM; });
    glds_gather(dnw, wn, [&](int tt) {
      const int t = w0 + tt;
      return t == sq.C - 1 ? sq.ones + b : sq.done + t * sq.done_st + b;
    });
  };
  // prologue: W_hh image + the last window's step inputs by LDS-DMA (one round trip, compact code)
  const int wfirst = min(sq.win, sq.C);
  glds_rows(img, M3, HM, LD, [&](int r, int j) { return a.P + o.gWhh + r * HM + j; });
  load_window(sq.C - wfirst, wfirst);
  float dhm_c = a.dhm[(int64_t)b * HM + min(ti, HM - 1)];   // carried by thread c = ti (>= HM: unused)
  for (int w1 = sq.C; w1 > 0; w1 -= sq.win) {
    const int w0 = max(0, w1 - sq.win), wn = w1 - w0;
    if (w1 != sq.C) {   // later windows (the first one came with the prologue)
      __syncthreads();
      load_window(w0, wn);
    }
    __syncthreads();
    if (tr) tr[1] = clock64();
    for (int tt = wn - 1; tt >= 0; --tt) {
      const int t = w0 + tt;
      uint64_t* ts = tr ? tr + 4 + 4 * t : nullptr;
      if (ts) ts[0] = clock64();
      const float* in = inw + tt * SI;
      float shd_c = 0.f;
      if (ti < HM) {
        const int i = ti;
        float dh = dnw[tt] > 0.5f ? 0.f : dhm_c;
#pragma unroll
        for (int j = 0; j < 4; ++j) dh = dh + in[(5 + j) * HM + i];
        const float r = in[HM + i], z = in[2 * HM + i], n = in[3 * HM + i];
        const float dn = dh * (1.f - z);
        const float dz = dh * (in[i] - n);
        const float dpn = dn * (1.f - n * n);
        const float dr = dpn * in[4 * HM + i];
        const float dar = dr * r * (1.f - r);
        const float daz = dz * z * (1.f - z);
        float* dl = a.delta + t * sq.delta_st + (int64_t)b * dld;
        dl[i] = dar;
        dl[HM + i] = daz;
        dl[2 * HM + i] = dpn;
        dl[3 * HM + i] = dar;
        dl[4 * HM + i] = daz;
        dl[5 * HM + i] = dpn * r;
        dgh[i] = dar;
        dgh[HM + i] = daz;
        dgh[2 * HM + i] = dpn * r;
        shd_c = dh * z;
      }
      if (ts) ts[1] = clock64();
      lds_sync();
      // W_hh^T dgh: block_matvec_t_ld's per-wave partials (rows r = w mod 4, 4 interleaved sums)
      if (lane < HM) {
        const int c = lane;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
        for (int q = 0; q < M3 / (4 * NW); ++q) {
          const int r = w + 4 * NW * q;
          a0 += img[r * LD + c] * dgh[r];
          a1 += img[(r + NW) * LD + c] * dgh[r + NW];
          a2 += img[(r + 2 * NW) * LD + c] * dgh[r + 2 * NW];
          a3 += img[(r + 3 * NW) * LD + c] * dgh[r + 3 * NW];
        }
        red[w * HM + c] = (a0 + a1) + (a2 + a3);
      }
      if (ts) ts[2] = clock64();
      lds_sync();
      if (ti < HM) {
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) acc += red[q * HM + ti];
        dhm_c = shd_c + acc;
      }
      if (ts) ts[3] = clock64() + (uint64_t)dhm_c * 0;
    }
  }
  if (tr) tr[2] = clock64();
  if (ti < HM) a.dhm[(int64_t)b * HM + ti] = dhm_c;
}

template <int HM>
__global__ __launch_bounds__(256) void mixer_rec_bwd_kernel(MixBwdArgs a, MixRecBwd sq) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  mixer_rec_bwd_body<HM>(a, sq, (int)blockIdx.x, sm);
}

// dynamic-LDS limit of the sequence kernels (MI355X: 160 KB per CU, one block per CU)
constexpr size_t kMixSeqLds = 160 * 1024;
static int mix_seq_lds_setup() {
  static bool done = false;
  if (done) return MM_OK;
  MM_HIP_CHECK(hipFuncSetAttribute((const void*)mixer_fwd_seq_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)kMixSeqLds));
  MM_HIP_CHECK(hipFuncSetAttribute((const void*)mixer_bwd_seq_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)kMixSeqLds));
  const void* serial[] = {(const void*)mixer_rec_fwd_kernel<32>, (const void*)mixer_rec_fwd_kernel<64>,
                          (const void*)mixer_rec_bwd_kernel<32>, (const void*)mixer_rec_bwd_kernel<64>,
                          (const void*)mixer_hyper_bwd_kernel<false>};
  for (const void* k : serial)
    MM_HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMixSeqLds));
  // (the PER block's static LDS comes off the dynamic limit)
  MM_HIP_CHECK(hipFuncSetAttribute((const void*)mixer_hyper_bwd_kernel<true>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kMixSeqLds - kPerSmallLds)));
  done = true;
  return MM_OK;
}
// ------------------------------------------------------------------ agent backward chain (one step)
struct AgentBwdArgs {
  const float* P;            // behavior agent params (canonical flat)
  int64_t oWq, oWhh;         // element offsets of Wq / Whh in P
  const float* save;         // [B][N][SD] of this step
  const int32_t* acts;       // [B][N]
  const float* dqa;          // [B][N]
  const float* done;         // [B] done of THIS step (drop the future gradient)
  float* dh;                 // [B][N][H] in: grad wrt h_out from step t+1 ; out: grad wrt h_in
  float* dgi;                // [B][N][3H] out (also the dgh rows via dgh pointer)
  float* dgh;                // [B][N][3H] out
  float* dq;                 // [B][N][A] out (dense one-hot dQ for the Wq gradient)
  int B, N, F1, G, H, A;
};

// one wave per (sample, agent); lane = hidden feature
__device__ __forceinline__ void agent_bwd_body(const AgentBwdArgs& a);

__global__ __launch_bounds__(256) void agent_bwd_kernel(AgentBwdArgs a) { agent_bwd_body(a); }

__device__ __forceinline__ void agent_bwd_body(const AgentBwdArgs& a) {
  __shared__ float sdg[4][3 * 256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pair0 = blockIdx.x * 4 + w;
  const bool on = pair0 < a.B * a.N;
  const int pair = on ? pair0 : 0;
  const int b = pair / a.N, i = pair % a.N;
  const int H = a.H, A = a.A;
  const int SD = a.F1 + a.G + 6 * H;
  const float* sv = a.save + (int64_t)pair * SD;
  const float* h0 = sv + a.F1 + a.G;
  const int act = a.acts[pair];
  const float dqa = a.dqa[pair];
  const float* Wq = a.P + a.oWq + (int64_t)i * A * H;
  const float* Whh = a.P + a.oWhh + (int64_t)i * 3 * H * H;
  const bool drop = a.done[b] > 0.5f;
  if (on)
    for (int c = lane; c < A; c += 64) a.dq[(int64_t)pair * A + c] = (c == act) ? dqa : 0.f;
  for (int f = lane; f < H && on; f += 64) {
    const float dh1 = Wq[(int64_t)act * H + f] * dqa + (drop ? 0.f : a.dh[(int64_t)pair * H + f]);
    const float r = h0[H + f], z = h0[2 * H + f], n = h0[3 * H + f], anh = h0[4 * H + f];
    const float dn = dh1 * (1.f - z);
    const float dz = dh1 * (h0[f] - n);
    const float dpn = dn * (1.f - n * n);
    const float dar = dpn * anh * r * (1.f - r);
    const float daz = dz * z * (1.f - z);
    float* gi = a.dgi + (int64_t)pair * 3 * H;
    float* gh = a.dgh + (int64_t)pair * 3 * H;
    gi[f] = dar;
    gi[H + f] = daz;
    gi[2 * H + f] = dpn;
    gh[f] = dar;
    gh[H + f] = daz;
    gh[2 * H + f] = dpn * r;
    sdg[w][f] = dar;
    sdg[w][H + f] = daz;
    sdg[w][2 * H + f] = dpn * r;
    // stash dh1*z for the direct path
    a.dh[(int64_t)pair * H + f] = dh1 * z;
  }
  __syncthreads();
  for (int f = lane; f < H && on; f += 64) {
    float acc = a.dh[(int64_t)pair * H + f];
    for (int r = 0; r < 3 * H; ++r) acc += Whh[(int64_t)r * H + f] * sdg[w][r];
    a.dh[(int64_t)pair * H + f] = acc;
  }
}

// Chunk-sequence agent backward (small batches): block = one agent x 4 samples (one wave each, lane =
// hidden feature) for ALL C steps. The agent's W_hh is staged once into LDS TRANSPOSED ([f][r], row
// stride 3H + 4: a lane's 4 consecutive r are one conflict-free ds_read_b128), the step inputs of a
// window of steps are loaded into LDS with one round of loads (the step loop then issues only stores,
// so no load wait ever drains them), and the hidden-state gradient is carried in registers. The waves
// never exchange data, so the step loop has no block barrier. Per-step arithmetic and the sequential
// r order of the W_hh^T mat-vec are agent_bwd_body's (bit-identical to the per-step launches).
struct AgentBwdSeq {
  int C, win;
  int64_t save_st, acts_st, dqa_st, dgi_st, dq_st, done_st;
  const float* ones;
  uint64_t* trace;     // clock64 stamps of block 0 wave 0 (MM_ABWD_TRACE), nullptr normally
};
__host__ __device__ inline size_t agent_bwd_seq_floats(int H, int A, int win) {
  return (size_t)H * (3 * H + 4) + 3 * (size_t)H * H + 4 * 3 * (size_t)H + (size_t)A * H + 4 +
         4 * (size_t)win * (5 * H + 3);
}
// (bx, by) = (batch group of 4 samples, agent); sm: the block's dynamic LDS (agent_bwd_seq_kernel,
// agent_mixer_bwd_kernel)
template <int H>
__device__ __forceinline__ void agent_bwd_seq_body(const AgentBwdArgs& a, const AgentBwdSeq& sq, int bx, int by,
                                                   float* sm) {
  constexpr int H3 = 3 * H, LDT = H3 + 4, SI = 5 * H;   // input rows: 16-byte aligned (H % 4 == 0)
  const int A = a.A;
  float* whT = sm;                 // [H][LDT]: whT[f * LDT + r] = W_hh[r][f]
  float* whr = whT + H * LDT;      // [3H][H] W_hh as loaded (row-major), transposed into whT
  float* sdg = whr + H3 * H;       // [4][3H] this wave's gate gradients
  float* wq = sdg + 4 * H3;        // [A][H]
  float* inw = wq + ((A * H + 3) & ~3);   // [win][4][5H]: h0 r z n anh of (step, wave)
  float* scw = inw + sq.win * 4 * SI;      // [win][4][3]: act (int bits) | dQ(a) | done
  const int w = threadIdx.x >> 6, f = threadIdx.x & 63;
  const int i = by;
  const int b = bx * 4 + w;
  const bool on = b < a.B && f < H;
  const int64_t pair = (int64_t)(b < a.B ? b : 0) * a.N + i;
  const int SD = a.F1 + a.G + 6 * H;
  uint64_t* tr = (sq.trace && bx == 0 && by == 0 && threadIdx.x == 0) ? sq.trace : nullptr;
  if (tr) tr[0] = clock64();
  const float* Wq_g = a.P + a.oWq + (int64_t)i * A * H;
  const float* Whh = a.P + a.oWhh + (int64_t)i * H3 * H;
  // input row (step w0 + row / 4, wave row % 4): the 5H saved GRU values (16-byte pieces), then the
  // action (raw int bits), dQ(a) and the done flag (one word each)
  auto save_row = [&](int w0, int row) -> const float* {
    const int t = w0 + (row >> 2), bb = min(bx * 4 + (row & 3), a.B - 1);
    return a.save + t * sq.save_st + ((int64_t)bb * a.N + i) * SD + a.F1 + a.G;
  };
  auto scalar_in = [&](int w0, int row, int j) -> const float* {   // j = 0 act, 1 dQ(a), 2 done
    const int t = w0 + (row >> 2), bb = min(bx * 4 + (row & 3), a.B - 1);
    const int64_t pr = (int64_t)bb * a.N + i;
    if (j == 0) return reinterpret_cast<const float*>(a.acts + t * sq.acts_st + pr);
    if (j == 1) return a.dqa + t * sq.dqa_st + pr;
    return t == sq.C - 1 ? sq.ones + bb : a.done + t * sq.done_st + bb;
  };
  auto load_window = [&](int w0, int wn) {
    glds_rows16(inw, 4 * wn, SI, SI, [&](int row) { return save_row(w0, row); });
    glds_gather(scw, 3 * 4 * wn, [&](int e) {
      const int row = e / 3;
      return scalar_in(w0, row, e - 3 * row);
    });
  };
  // prologue: W_hh (row-major image, transposed in LDS below), W_q and the last window's step inputs
  // by LDS-DMA (one round trip, compact code)
  const int wfirst = min(sq.win, sq.C);
  glds_rows16(whr, 1, H3 * H, H3 * H, [&](int) { return Whh; });
  if (tr) tr[103] = clock64();
  glds_gather(wq, A * H, [&](int idx) { return Wq_g + idx; });
  if (tr) tr[104] = clock64();
  load_window(sq.C - wfirst, wfirst);
  float dh = a.dh[pair * H + min(f, H - 1)];   // (lanes f >= H: unused)
  if (tr) tr[100] = clock64();
  __syncthreads();
  if (tr) tr[101] = clock64();
#pragma unroll 4
  for (int q = threadIdx.x; q < H3 * H / 4; q += blockDim.x) {
    const int r = (4 * q) / H, c = (4 * q) % H;
    const float4 v = *reinterpret_cast<const float4*>(whr + 4 * q);
    whT[(c + 0) * LDT + r] = v.x;
    whT[(c + 1) * LDT + r] = v.y;
    whT[(c + 2) * LDT + r] = v.z;
    whT[(c + 3) * LDT + r] = v.w;
  }
  if (tr) tr[102] = clock64();
  const float* whrow = whT + f * LDT;
  float* sdw = sdg + w * H3;
  for (int w1 = sq.C; w1 > 0; w1 -= sq.win) {
    const int w0 = max(0, w1 - sq.win), wn = w1 - w0;
    if (w1 != sq.C) {   // later windows (the first one came with the prologue)
      __syncthreads();
      load_window(w0, wn);
    }
    __syncthreads();   // window (and, first pass, the transposed W_hh) visible
    if (tr) tr[1] = clock64();
    for (int tt = wn - 1; tt >= 0; --tt) {
      const int t = w0 + tt;
      uint64_t* ts = tr ? tr + 4 + 4 * t : nullptr;
      if (ts) ts[0] = clock64();
      const float* in = inw + (tt * 4 + w) * SI;
      const float* sc = scw + (tt * 4 + w) * 3;
      float stash = 0.f;
      if (b < a.B) {
        const int act = __float_as_int(sc[0]);
        const float dqa = sc[1];
        if (f < A) a.dq[t * sq.dq_st + pair * A + f] = (f == act) ? dqa : 0.f;
        if (f < H) {
          const bool drop = sc[2] > 0.5f;
          const float dh1 = wq[act * H + f] * dqa + (drop ? 0.f : dh);
          const float r = in[H + f], z = in[2 * H + f], n = in[3 * H + f], anh = in[4 * H + f];
          const float dn = dh1 * (1.f - z);
          const float dz = dh1 * (in[f] - n);
          const float dpn = dn * (1.f - n * n);
          const float dar = dpn * anh * r * (1.f - r);
          const float daz = dz * z * (1.f - z);
          float* gi = a.dgi + t * sq.dgi_st + pair * H3;
          float* gh = a.dgh + t * sq.dgi_st + pair * H3;
          gi[f] = dar;
          gi[H + f] = daz;
          gi[2 * H + f] = dpn;
          gh[f] = dar;
          gh[H + f] = daz;
          gh[2 * H + f] = dpn * r;
          sdw[f] = dar;
          sdw[H + f] = daz;
          sdw[2 * H + f] = dpn * r;
          stash = dh1 * z;
        }
      }
      if (ts) ts[1] = clock64();
      // sdw is written and read by this wave only: LDS ops of one wave complete in order, so a
      // compiler fence is all the hand-over needs
      __builtin_amdgcn_wave_barrier();
      if (on) {
        float acc = stash;
#pragma unroll
        for (int r4 = 0; r4 < H3; r4 += 4) {
          const float4 wv = *reinterpret_cast<const float4*>(whrow + r4);
          const float4 dv = *reinterpret_cast<const float4*>(sdw + r4);
          acc += wv.x * dv.x;
          acc += wv.y * dv.y;
          acc += wv.z * dv.z;
          acc += wv.w * dv.w;
        }
        dh = acc;
      }
      if (ts) ts[2] = clock64() + (uint64_t)dh * 0;
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (tr) tr[2] = clock64();
  if (on) a.dh[pair * H + f] = dh;
}

template <int H>
__global__ __launch_bounds__(256) void agent_bwd_seq_kernel(AgentBwdArgs a, AgentBwdSeq sq) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  agent_bwd_seq_body<H>(a, sq, (int)blockIdx.x, (int)blockIdx.y, sm);
}

// The agent BPTT (blocks [0, n_agent_blocks), (batch group, agent) = (bid % gx, bid / gx)) and the mixer
// recurrence's backward (the remaining B blocks, one per sample) in ONE launch: the two chains are independent
// (both read the hypernet pass's outputs), so they share the grid instead of a stream fork / join in the update
// graph. Same bodies as the two kernels, so the same results.
template <int H, int HM>
__global__ __launch_bounds__(256) void agent_mixer_bwd_kernel(AgentBwdArgs a, AgentBwdSeq q, MixBwdArgs ma,
                                                              MixRecBwd mq, int gx, int n_agent_blocks) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int bid = (int)blockIdx.x;
  if (bid < n_agent_blocks)
    agent_bwd_seq_body<H>(a, q, bid % gx, bid / gx, sm);
  else
    mixer_rec_bwd_body<HM>(ma, mq, bid - n_agent_blocks, sm);
}

// Large-batch variant (H <= 64): one block = one agent x 32 samples, one wave = 8 samples of that
// agent, lane = hidden feature. Every W_hh element the transposed mat-vec reads serves the wave's
// 8 samples (the one-pair-per-wave kernel re-reads the agent's 48 KB W_hh per pair, which bounds
// it on L2 bandwidth at large B). Per-sample arithmetic and summation order are those of
// agent_bwd_body, so the results are bit-identical (tested).
constexpr int BWD_SPW = 8;   // samples per wave
__global__ __launch_bounds__(256) void agent_bwd_multi_kernel(AgentBwdArgs a) {
  __shared__ float4 sdg[4][3 * 64][BWD_SPW / 4];   // [wave][gate row][sample]
  const int w = threadIdx.x >> 6, f = threadIdx.x & 63;
  const int i = blockIdx.y;
  const int b0 = (blockIdx.x * 4 + w) * BWD_SPW;
  const int H = a.H, A = a.A;
  const int SD = a.F1 + a.G + 6 * H;
  const float* Wq = a.P + a.oWq + (int64_t)i * A * H;
  const float* Whh = a.P + a.oWhh + (int64_t)i * 3 * H * H;
  float* sd = reinterpret_cast<float*>(&sdg[w][0][0]);
  float acc[BWD_SPW];
#pragma unroll
  for (int s = 0; s < BWD_SPW; ++s) {
    const int b = b0 + s;
    acc[s] = 0.f;
    if (b >= a.B) continue;
    const int64_t pair = (int64_t)b * a.N + i;
    const float* h0 = a.save + pair * SD + a.F1 + a.G;
    const int act = a.acts[pair];
    const float dqa = a.dqa[pair];
    if (f < A) a.dq[pair * A + f] = (f == act) ? dqa : 0.f;
    if (f < H) {
      const bool drop = a.done[b] > 0.5f;
      const float dh1 = Wq[(int64_t)act * H + f] * dqa + (drop ? 0.f : a.dh[pair * H + f]);
      const float r = h0[H + f], z = h0[2 * H + f], n = h0[3 * H + f], anh = h0[4 * H + f];
      const float dn = dh1 * (1.f - z);
      const float dz = dh1 * (h0[f] - n);
      const float dpn = dn * (1.f - n * n);
      const float dar = dpn * anh * r * (1.f - r);
      const float daz = dz * z * (1.f - z);
      float* gi = a.dgi + pair * 3 * H;
      float* gh = a.dgh + pair * 3 * H;
      gi[f] = dar;
      gi[H + f] = daz;
      gi[2 * H + f] = dpn;
      gh[f] = dar;
      gh[H + f] = daz;
      gh[2 * H + f] = dpn * r;
      sd[f * BWD_SPW + s] = dar;
      sd[(H + f) * BWD_SPW + s] = daz;
      sd[(2 * H + f) * BWD_SPW + s] = dpn * r;
      acc[s] = dh1 * z;
    }
  }
  // each wave reads only its own rows of sdg: LDS is in order within a wave
  __builtin_amdgcn_wave_barrier();
  if (f >= H) return;
#pragma unroll 8
  for (int r = 0; r < 3 * H; ++r) {
    const float wv = Whh[(int64_t)r * H + f];
#pragma unroll
    for (int q = 0; q < BWD_SPW / 4; ++q) {
      const float4 x = sdg[w][r][q];
      acc[4 * q + 0] += wv * x.x;
      acc[4 * q + 1] += wv * x.y;
      acc[4 * q + 2] += wv * x.z;
      acc[4 * q + 3] += wv * x.w;
    }
  }
#pragma unroll
  for (int s = 0; s < BWD_SPW; ++s)
    if (b0 + s < a.B) a.dh[((int64_t)(b0 + s) * a.N + i) * H + f] = acc[s];
}

// ------------------------------------------------------------------ batched reductions
// dW[g][r][c] (+)= sum_m U[g](m, r) * V[g](m, c) ;  db[g][r] (+)= sum_m U[g](m, r)
//   U(m, r) = U[g*u_g + m*u_m + r];  V(m, c) = V[g*v_g + m*v_m + c], or, if v_off != nullptr,
//   V(m, c) = (v_off[m] >= 0 ? V + v_off[m] : v_reset) [g*v_g + c]   (gathered obs rows)
// Fixed summation order over m (deterministic). Block = 256 threads -> 32 x 32 tile.
struct OuterArgs {
  const float* U; int64_t u_g, u_m;
  const float* V; int64_t v_g, v_m; const int64_t* v_off; const float* v_reset;
  float* dW; int64_t w_g;   // dW[g*w_g + r*Cc + c]
  float* db; int64_t b_g;   // db[g*b_g + r] (nullptr: none)
  int M, R, Cc, accumulate;
};

__global__ __launch_bounds__(256) void outer_reduce_kernel(OuterArgs a) {
  // LDS double buffer + register prefetch: chunk m0+32 is loaded while chunk m0 is reduced, so
  // the M/32 sequential steps pay one memory latency instead of one each.
  __shared__ float su[2][32][33];
  __shared__ float svv[2][32][33];
  const int g = blockIdx.z;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tr = threadIdx.x / 32, tc = threadIdx.x % 32;  // tr in [0,8): rows tr, tr+8, tr+16, tr+24
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float accb = 0.f;
  float pu[4], pv[4];
  auto fetch = [&](int m0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = threadIdx.x + 256 * q;
      const int mm = k / 32, x = k % 32;
      const int m = m0 + mm;
      float u = 0.f, v = 0.f;
      if (m < a.M) {
        if (r0 + x < a.R) u = a.U[g * a.u_g + (int64_t)m * a.u_m + r0 + x];
        if (c0 + x < a.Cc) {
          if (a.v_off) {
            const int64_t off = a.v_off[m];
            const float* base = off >= 0 ? a.V + off : a.v_reset;
            v = base[g * a.v_g + c0 + x];
          } else {
            v = a.V[g * a.v_g + (int64_t)m * a.v_m + c0 + x];
          }
        }
      }
      pu[q] = u;
      pv[q] = v;
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = threadIdx.x + 256 * q;
      su[buf][k / 32][k % 32] = pu[q];
      svv[buf][k / 32][k % 32] = pv[q];
    }
  };
  fetch(0);
  stash(0);
  __syncthreads();
  int buf = 0;
  for (int m0 = 0; m0 < a.M; m0 += 32) {
    const bool more = m0 + 32 < a.M;
    if (more) fetch(m0 + 32);
    for (int mm = 0; mm < 32; ++mm) {
      const float v = svv[buf][mm][tc];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += su[buf][mm][tr + 8 * q] * v;
    }
    if (a.db && blockIdx.x == 0 && threadIdx.x < 32)
      for (int mm = 0; mm < 32; ++mm) accb += su[buf][mm][threadIdx.x];
    if (more) stash(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = r0 + tr + 8 * q, c = c0 + tc;
    if (r < a.R && c < a.Cc) {
      float* o = a.dW + g * a.w_g + (int64_t)r * a.Cc + c;
      *o = a.accumulate ? *o + acc[q] : acc[q];
    }
  }
  if (a.db && blockIdx.x == 0 && threadIdx.x < 32 && r0 + threadIdx.x < a.R) {
    float* o = a.db + g * a.b_g + r0 + threadIdx.x;
    *o = a.accumulate ? *o + accb : accb;
  }
}

// Batched split-M outer reduce: many independent OuterArgs jobs in ONE launch, each job's M rows
// split into slices of 32-row chunks; block (job, tile, group, slice) reduces one tile over one slice
// into a partial, outer_sum_kernel adds the slices in fixed order (deterministic).
constexpr int OB_MAX = 16;
struct OuterBatch {
  OuterArgs job[OB_MAX];
  int tiles_c[OB_MAX], tiles_r[OB_MAX], groups[OB_MAX], slices[OB_MAX], rps[OB_MAX];
  int tr_shift[OB_MAX];  // block tile TR x TC = (32 << s) x (128 >> s): 32x128, 64x64 or 128x32 (least padding)
  int blk0[OB_MAX + 1];
  int64_t part[OB_MAX];  // partial offset: [slice][group][R*Cc + R]
  int njobs;
  int bf3;   // fast mode: the MFMA products as bf16x3 splits (outer_tile_bf3)
  float* partial;
};

// Block = 4 waves = one TR x TC tile of (R, Cc), each wave a 32 x 32 sub-tile accumulated with 16
// exact-f32 MFMAs per 32-row chunk (v_mfma_f32_32x32x2_f32, the reduction index m on the MFMA k
// dimension). Per chunk the U [32][TR] and V [32][TC] slabs (NL = (TR + TC) / 8 floats per thread,
// coalesced rows) are staged in LDS while the next chunk's slabs are already in flight; gathered V rows
// (v_off) take their row offsets from LDS, loaded one chunk further ahead, so no load waits behind
// another. Bias sums (U^T 1) come from the U values each thread loads (its column is fixed:
// 256 % TR == 0), combined over the 256 / TR threads of a column in fixed order at the end.
struct ObSmem {
  float su[32][132];
  float svv[32][132];
  int64_t soff[2][32];
  float sbias[256];
};

// bf16x3 split (the learner's fast mode): x = hi + lo + O(2^-16 x) with hi = bf16(x), lo = bf16(x - hi), both
// round-to-nearest-even; hi_a hi_b + hi_a lo_b + lo_a hi_b in fp32 accumulation carries ~2^-16 relative error
// per product at fp32's exponent range (no f16 underflow of small gradients), on v_mfma_f32_32x32x16_bf16:
// 3 x 32 cycles per 32 x 32 x 16 block instead of 8 x 64 cycles of the exact-f32 MFMA.
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint32_t bf16_rne_bits(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ void bf3_split(const float (&x)[8], bf16x8& hi, bf16x8& lo) {
  s16x8 h, l;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t hb = bf16_rne_bits(x[i]);
    h[i] = (short)hb;
    l[i] = (short)bf16_rne_bits(x[i] - __uint_as_float(hb << 16));
  }
  hi = __builtin_bit_cast(bf16x8, h);
  lo = __builtin_bit_cast(bf16x8, l);
}

template <int TS, bool BF3 = false>
__device__ __forceinline__ void outer_tile(const OuterBatch& ob, int j, int t, ObSmem& sm) {
  constexpr int TR = 32 << TS, TC = 128 >> TS, NU = TR / 8, NL = NU + TC / 8;
  constexpr int MU = 256 / TR, MV = 256 / TC;   // rows between a thread's consecutive U / V elements
  const OuterArgs& a = ob.job[j];
  const int tc_ = t % ob.tiles_c[j];
  t /= ob.tiles_c[j];
  const int tr_ = t % ob.tiles_r[j];
  t /= ob.tiles_r[j];
  const int g = t % ob.groups[j];
  const int sl = t / ob.groups[j];
  const int r0 = tr_ * TR, c0 = tc_ * TC;
  const int m_begin = sl * ob.rps[j], m_end = min(a.M, m_begin + ob.rps[j]);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, li = lane & 31, lh = lane >> 5;
  constexpr int NRW = TR / 32;
  const int rw = wave % NRW, cw = wave / NRW;
  const bool gather = a.v_off != nullptr;
  // this thread's U column xu / first row mu0, V column xv / first row mv0
  const int xu = tid % TR, mu0 = tid / TR, xv = tid % TC, mv0 = tid / TC;
  const bool uok = r0 + xu < a.R, vok = c0 + xv < a.Cc;
  const float* Ub = a.U + g * a.u_g + r0 + xu;
  const float* Vb = a.V + g * a.v_g + c0 + xv;
  const float* Vr = gather ? a.v_reset + g * a.v_g + c0 + xv : nullptr;
  const int64_t u_m = a.u_m, v_m = a.v_m;
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
  float sb = 0.f;
  float pv[NL];
  auto load = [&](int m0, int buf) {
    const float* up = Ub + (int64_t)(m0 + mu0) * u_m;
#pragma unroll
    for (int p = 0; p < NU; ++p) {
      const int m = m0 + mu0 + MU * p;
      pv[p] = (uok && m < m_end) ? up[0] : 0.f;
      up += MU * u_m;
    }
    if (gather) {
#pragma unroll
      for (int p = 0; p < NL - NU; ++p) {
        const int mm = mv0 + MV * p, m = m0 + mm;
        const int64_t off = sm.soff[buf][mm];
        pv[NU + p] = (vok && m < m_end) ? (off >= 0 ? Vb + off : Vr)[0] : 0.f;
      }
    } else {
      const float* vp = Vb + (int64_t)(m0 + mv0) * v_m;
#pragma unroll
      for (int p = 0; p < NL - NU; ++p) {
        const int m = m0 + mv0 + MV * p;
        pv[NU + p] = (vok && m < m_end) ? vp[0] : 0.f;
        vp += MV * v_m;
      }
    }
  };
  int64_t off_next = -1;
  if (gather && tid < 32) {
    const int m = m_begin + tid;
    sm.soff[0][tid] = m < m_end ? a.v_off[m] : -1;
    off_next = m + 32 < m_end ? a.v_off[m + 32] : -1;
  }
  __syncthreads();
  if (m_begin < m_end) load(m_begin, 0);
  int buf = 0;
  for (int m0 = m_begin; m0 < m_end; m0 += 32) {
#pragma unroll
    for (int p = 0; p < NU; ++p) {
      sm.su[mu0 + MU * p][xu] = pv[p];
      sb += pv[p];
    }
#pragma unroll
    for (int p = 0; p < NL - NU; ++p) sm.svv[mv0 + MV * p][xv] = pv[NU + p];
    if (gather && tid < 32) {   // offsets of chunk m0 + 32 for the loads below; the next ones in flight
      sm.soff[buf ^ 1][tid] = off_next;
      const int m = m0 + 64 + tid;
      off_next = m < m_end ? a.v_off[m] : -1;
    }
    __syncthreads();
    if (m0 + 32 < m_end) load(m0 + 32, buf ^ 1);
    if constexpr (BF3) {
      // two 16-deep k-steps over the chunk's 32 rows m: lane (li, lh) holds rows m = 16 ks + 8 lh + 0..7
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float av[8], bv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          av[i] = sm.su[16 * ks + 8 * lh + i][rw * 32 + li];
          bv[i] = sm.svv[16 * ks + 8 * lh + i][cw * 32 + li];
        }
        bf16x8 ah, al, bh, bl;
        bf3_split(av, ah, al);
        bf3_split(bv, bh, bl);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2)
        acc = mfma32(sm.su[2 * s2 + lh][rw * 32 + li], sm.svv[2 * s2 + lh][cw * 32 + li], acc);
    }
    __syncthreads();
    buf ^= 1;
  }
  const int64_t per = (int64_t)a.R * a.Cc + a.R;
  float* out = ob.partial + ob.part[j] + ((int64_t)sl * ob.groups[j] + g) * per;
  const int c = c0 + cw * 32 + li;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int r = r0 + rw * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
    if (r < a.R && c < a.Cc) out[(int64_t)r * a.Cc + c] = acc[q];
  }
  if (a.db && tc_ == 0) {
    sm.sbias[tid] = sb;
    __syncthreads();
    if (tid < TR && r0 + tid < a.R) {
      float s = 0.f;
      for (int k = tid; k < 256; k += TR) s += sm.sbias[k];
      out[(int64_t)a.R * a.Cc + r0 + tid] = s;
    }
  }
}

__global__ __launch_bounds__(256) void outer_batch_kernel(OuterBatch ob) {
  __shared__ ObSmem sm;
  int j = 0;
  while (j + 1 < ob.njobs && (int)blockIdx.x >= ob.blk0[j + 1]) ++j;
  const int t = blockIdx.x - ob.blk0[j];
  if (ob.bf3) {
    switch (ob.tr_shift[j]) {
      case 0: outer_tile<0, true>(ob, j, t, sm); break;
      case 1: outer_tile<1, true>(ob, j, t, sm); break;
      default: outer_tile<2, true>(ob, j, t, sm); break;
    }
    return;
  }
  switch (ob.tr_shift[j]) {
    case 0: outer_tile<0>(ob, j, t, sm); break;
    case 1: outer_tile<1>(ob, j, t, sm); break;
    default: outer_tile<2>(ob, j, t, sm); break;
  }
}

__global__ __launch_bounds__(256) void outer_sum_kernel(OuterBatch ob) {
  const int j = blockIdx.y;
  const OuterArgs& a = ob.job[j];
  const int64_t per = (int64_t)a.R * a.Cc + a.R;
  const int64_t total = per * ob.groups[j];
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int g = (int)(e / per);
    const int64_t w = e % per;
    if (w >= (int64_t)a.R * a.Cc && !a.db) continue;
    float s = 0.f;
    const float* p = ob.partial + ob.part[j] + e;
    for (int sl = 0; sl < ob.slices[j]; ++sl) s += p[(int64_t)sl * total];
    float* o = w < (int64_t)a.R * a.Cc ? a.dW + g * a.w_g + w : a.db + g * a.b_g + (w - (int64_t)a.R * a.Cc);
    *o = a.accumulate ? *o + s : s;
  }
}

// Y[g](m, c) = gate(m, c) * sum_r W[g][r][c] * X[g](m, r)      (batched transpose matvec, gated by x > 0)
//   W[g*w_g + r*Cc + c], X[g*x_g + m*x_m + r], gate = Z[g*z_g + m*z_m + c] > 0 (if Z), Y[g*y_g + m*y_m + c]
struct TmvArgs {
  const float* W; int64_t w_g;
  const float* X; int64_t x_g, x_m;
  const float* Z; int64_t z_g, z_m;
  float* Y; int64_t y_g, y_m;
  int M, R, Cc;
  int aligned16;   // tmv_full_kernel: 16-byte LDS-DMA staging allowed
};

__global__ __launch_bounds__(256) void tmv_kernel(TmvArgs a) {
  __shared__ float sx[32][33];
  __shared__ float sw[32][33];
  const int g = blockIdx.z;
  const int m0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tm = threadIdx.x / 32, tc = threadIdx.x % 32;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int rr = 0; rr < a.R; rr += 32) {
    for (int k = threadIdx.x; k < 32 * 32; k += 256) {
      const int p = k / 32, x = k % 32;
      const int m = m0 + p, r = rr + x;
      sx[p][x] = (m < a.M && r < a.R) ? a.X[g * a.x_g + (int64_t)m * a.x_m + r] : 0.f;
      const int r2 = rr + p, c = c0 + x;
      sw[p][x] = (r2 < a.R && c < a.Cc) ? a.W[g * a.w_g + (int64_t)r2 * a.Cc + c] : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < 32; ++r) {
      const float w = sw[r][tc];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += sx[tm + 8 * q][r] * w;
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = m0 + tm + 8 * q, c = c0 + tc;
    if (m < a.M && c < a.Cc) {
      float v = acc[q];
      if (a.Z && !(a.Z[g * a.z_g + (int64_t)m * a.z_m + c] > 0.f)) v = 0.f;
      a.Y[g * a.y_g + (int64_t)m * a.y_m + c] = v;
    }
  }
}

// Same op and summation order, with the whole r range of the block's X rows and W columns staged in
// ONE round of loads (R <= 256: sx [32][R], sw [R][32] in dynamic LDS) instead of one memory round
// trip per 32-deep chunk.
__global__ __launch_bounds__(256) void tmv_full_kernel(TmvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int R = a.R;
  float* sx = sm;             // [32][R] (a wave reads 2 rows: broadcasts)
  float* sw = sx + 32 * R;    // [R][32]
  const int g = blockIdx.z;
  const int m0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tm = threadIdx.x / 32, tc = threadIdx.x % 32;
  // rows m >= M / columns c >= Cc load a valid neighbour; their results are never stored
  if (a.aligned16) {   // 16-byte LDS-DMA (R, x_m, Cc, c0 multiples of 4; 16-byte aligned bases)
    const int R4 = R >> 2;
    glds16_gather(sx, 32 * R4, [&](int i) {
      const int p = i / R4;
      return a.X + g * a.x_g + (int64_t)min(m0 + p, a.M - 1) * a.x_m + 4 * (i - p * R4);
    });
    glds16_gather(sw, R * 8, [&](int i) {
      const int r = i >> 3;
      return a.W + g * a.w_g + (int64_t)r * a.Cc + min(c0 + 4 * (i & 7), a.Cc - 4);
    });
  } else {
    block_gather_rows(sx, 32, R, [&](int p, int r) {
      return a.X + g * a.x_g + (int64_t)min(m0 + p, a.M - 1) * a.x_m + r;
    });
    block_gather_rows(sw, R, 32, [&](int r, int x) {
      return a.W + g * a.w_g + (int64_t)r * a.Cc + min(c0 + x, a.Cc - 1);
    });
  }
  __syncthreads();
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < R; ++r) {
    const float w = sw[r * 32 + tc];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] += sx[(tm + 8 * q) * R + r] * w;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = m0 + tm + 8 * q, c = c0 + tc;
    if (m < a.M && c < a.Cc) {
      float v = acc[q];
      if (a.Z && !(a.Z[g * a.z_g + (int64_t)m * a.z_m + c] > 0.f)) v = 0.f;
      a.Y[g * a.y_g + (int64_t)m * a.y_m + c] = v;
    }
  }
}

// Same op on exact-f32 MFMA (v_mfma_f32_32x32x2_f32): block = 4 waves = one 64 (m) x 64 (c) tile,
// per 32-deep r chunk the X / W slabs are staged in LDS (X transposed to [r][m]) and every wave
// accumulates its 32 x 32 sub-tile with 16 MFMAs (r on the MFMA k dimension; fixed order).
__global__ __launch_bounds__(256) void tmv_mfma_kernel(TmvArgs a) {
  __shared__ float sx[32][65];
  __shared__ float sw[32][65];
  const int g = blockIdx.z;
  const int m0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  const int mw = wave >> 1, cw = wave & 1;
  const float* X = a.X + g * a.x_g;
  const float* W = a.W + g * a.w_g;
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
  // chunk rr + 32's slabs are loaded into registers while chunk rr is reduced (one memory latency per launch
  // instead of one per 32-deep chunk; same values, same MFMA order)
  float px[8], pw[8];
  auto fetch = [&](int rr) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = threadIdx.x + 256 * q;
      const int mm = k >> 5, x = k & 31;          // X: 32 consecutive r of one row per 32 lanes
      const int m = m0 + mm, r = rr + x;
      px[q] = (m < a.M && r < a.R) ? X[(int64_t)m * a.x_m + r] : 0.f;
      const int kk = k >> 6, y = k & 63;          // W: 64 consecutive c of one r
      const int r2 = rr + kk, c = c0 + y;
      pw[q] = (r2 < a.R && c < a.Cc) ? W[(int64_t)r2 * a.Cc + c] : 0.f;
    }
  };
  fetch(0);
  for (int rr = 0; rr < a.R; rr += 32) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = threadIdx.x + 256 * q;
      sx[k & 31][k >> 5] = px[q];
      sw[k >> 6][k & 63] = pw[q];
    }
    __syncthreads();
    if (rr + 32 < a.R) fetch(rr + 32);
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
      acc = mfma32(sx[2 * s2 + lh][mw * 32 + li], sw[2 * s2 + lh][cw * 32 + li], acc);
    __syncthreads();
  }
  const int c = c0 + cw * 32 + li;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int m = m0 + mw * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
    if (m < a.M && c < a.Cc) {
      float v = acc[q];
      if (a.Z && !(a.Z[g * a.z_g + (int64_t)m * a.z_m + c] > 0.f)) v = 0.f;
      a.Y[g * a.y_g + (int64_t)m * a.y_m + c] = v;
    }
  }
}

// tmv_mfma_kernel's op and MFMA order for R <= TMV_FULL_RMAX with 16-byte aligned rows (aligned16): the block's whole r range of
// X (64 rows) and W (64 columns) staged in ONE round of 16-byte loads (issued 4 deep) into dynamic LDS ([R][65] each,
// X transposed) instead of a round of scalar loads per 32-deep chunk
constexpr int TMV_FULL_RMAX = 64;   // (R = 192, 100 KB of LDS, one block per CU: slower than the chunked kernel)
__global__ __launch_bounds__(256) void tmv_mfma_full_kernel(TmvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smt[];
  const int R = a.R, R4 = R >> 2, Rp = (R + 31) & ~31;   // (the last 32-deep chunk's rows r >= R read zeros)
  float (*sx)[65] = reinterpret_cast<float (*)[65]>(smt);             // [Rp][65]: [r][m]
  float (*sw)[65] = reinterpret_cast<float (*)[65]>(smt + Rp * 65);   // [Rp][65]: [r][c]
  const int g = blockIdx.z;
  const int m0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  const int mw = wave >> 1, cw = wave & 1;
  const float* X = a.X + g * a.x_g;
  const float* W = a.W + g * a.w_g;
#pragma unroll 4
  for (int i = threadIdx.x; i < 64 * R4; i += 256) {   // X: 64 rows x R4 float4
    const int mm = i / R4, r4 = i - mm * R4;
    const float4 v = *reinterpret_cast<const float4*>(X + (int64_t)min(m0 + mm, a.M - 1) * a.x_m + 4 * r4);
    sx[4 * r4][mm] = v.x;
    sx[4 * r4 + 1][mm] = v.y;
    sx[4 * r4 + 2][mm] = v.z;
    sx[4 * r4 + 3][mm] = v.w;
  }
#pragma unroll 4
  for (int i = threadIdx.x; i < 16 * R; i += 256) {    // W: R rows x 16 float4 (64 columns)
    const int r = i >> 4, c4 = i & 15;
    const float4 v = *reinterpret_cast<const float4*>(W + (int64_t)r * a.Cc + min(c0 + 4 * c4, a.Cc - 4));
    sw[r][4 * c4] = v.x;
    sw[r][4 * c4 + 1] = v.y;
    sw[r][4 * c4 + 2] = v.z;
    sw[r][4 * c4 + 3] = v.w;
  }
  for (int i = R * 64 + threadIdx.x; i < Rp * 64; i += 256) {
    sx[i >> 6][i & 63] = 0.f;
    sw[i >> 6][i & 63] = 0.f;
  }
  __syncthreads();
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
  for (int rr = 0; rr < R; rr += 32) {
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
      acc = mfma32(sx[rr + 2 * s2 + lh][mw * 32 + li], sw[rr + 2 * s2 + lh][cw * 32 + li], acc);
  }
  const int c = c0 + cw * 32 + li;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int m = m0 + mw * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
    if (m < a.M && c < a.Cc) {
      float v = acc[q];
      if (a.Z && !(a.Z[g * a.z_g + (int64_t)m * a.z_m + c] > 0.f)) v = 0.f;
      a.Y[g * a.y_g + (int64_t)m * a.y_m + c] = v;
    }
  }
}

// ------------------------------------------------------------------ clip + Adam
// partial sums of squares of G[0:n_clip] ; also advances the Adam step counter
__global__ __launch_bounds__(256) void sumsq_kernel(const float* G, int64_t n, float* partials, float* step) {
  __shared__ float sh[256];
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc += G[i] * G[i];
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) partials[blockIdx.x] = sh[0];
  if (step && blockIdx.x == 0 && threadIdx.x == 0) *step += 1.0f;
}

// torch.optim.Adam (no amsgrad / weight decay) with clip_grad_norm_ applied to G[0:n_clip]
// With partials2 != null a second clip group [n_clip, n) uses its own norm (partials2) and coefficient
// (qmix/qmix.py:235-238 clips the agent net and the mixer separately).
struct AdamArgs {
  float *P, *G, *m, *v;
  int64_t n, n_clip;
  const float* partials;   // [n_part] sumsq partials of G[0:n_clip] (sumsq_kernel)
  int n_part;              // <= 256
  float max_norm, lr, b1, b2, eps;
  const float* step;
  float* norm_out;
  float grad_scale;
  const float* partials2;  // second clip group [n_clip, n) or nullptr
};
// per-launch Adam constants of the block: clip coefficients of both groups from the sumsq partials (threads 0-255:
// one partial each, a fixed-order tree — the same sums whatever the block size) and the bias corrections
struct AdamConst {
  float coef, coef2, step_size, bc2s;
};
__device__ __forceinline__ AdamConst adam_const(const AdamArgs& a) {
  __shared__ float s_coef[2];
  __shared__ float red[2][256];
  const int tid = (int)threadIdx.x;
  if (tid < 256) {
    float p1 = 0.f, p2 = 0.f;
    for (int i = tid; i < a.n_part; i += 256) {
      p1 += a.partials[i];
      if (a.partials2) p2 += a.partials2[i];
    }
    red[0][tid] = p1;
    red[1][tid] = p2;
  }
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) {
      red[0][tid] += red[0][tid + st];
      red[1][tid] += red[1][tid + st];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const float tot = red[0][0], tot2 = red[1][0];
    const float norm = sqrtf(tot) * a.grad_scale;
    const float norm2 = sqrtf(tot2) * a.grad_scale;
    s_coef[0] = a.max_norm > 0.f ? fminf(1.0f, a.max_norm / (norm + 1e-6f)) : 1.0f;
    s_coef[1] = (a.partials2 && a.max_norm > 0.f) ? fminf(1.0f, a.max_norm / (norm2 + 1e-6f)) : 1.0f;
    if (a.norm_out && blockIdx.x == 0) {
      a.norm_out[0] = norm;
      if (a.partials2) a.norm_out[1] = norm2;
    }
  }
  __syncthreads();
  AdamConst c;
  c.coef = s_coef[0];
  c.coef2 = s_coef[1];
  const float t = *a.step;
  const float bc1 = 1.0f - powf(a.b1, t);
  const float bc2 = 1.0f - powf(a.b2, t);
  c.step_size = a.lr / bc1;
  c.bc2s = sqrtf(bc2);
  return c;
}
// one parameter's Adam step; returns the new value
__device__ __forceinline__ float adam_elem(const AdamArgs& a, const AdamConst& c, int64_t i) {
  float g = a.G[i] * a.grad_scale;
  g *= i < a.n_clip ? c.coef : c.coef2;
  const float mi = a.m[i] + (g - a.m[i]) * (1.0f - a.b1);
  const float vi = a.v[i] * a.b2 + g * g * (1.0f - a.b2);
  a.m[i] = mi;
  a.v[i] = vi;
  const float denom = sqrtf(vi) / c.bc2s + a.eps;
  const float p = a.P[i] - c.step_size * (mi / denom);
  a.P[i] = p;
  return p;
}
__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  const AdamConst c = adam_const(a);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x)
    adam_elem(a, c, i);
}

}  // namespace mm

// ------------------------------------------------------------------ C ABI
extern "C" {

int mm_learner_set_multi_sample(int32_t mixer, int32_t agent_bwd) {
  mm::g_mix_multi = mixer != 0;
  mm::g_bwd_multi = agent_bwd != 0;
  return MM_OK;
}

int mm_mixer_param_count(int32_t state_dim, int32_t hm, int32_t k1, int32_t n_agents, int64_t* count) {
  MM_REQUIRE(count && state_dim > 0 && hm > 0 && k1 > 0 && n_agents > 0, "mixer_param_count: bad dims");
  *count = mm::mix_offsets(state_dim, hm, k1, n_agents).total;
  return MM_OK;
}
int mm_mixer_save_dim(int32_t hm, int32_t k1, int32_t n_agents) { return mm::mix_save_dim(hm, k1, n_agents); }
int mm_mixer_delta_dim(int32_t hm, int32_t k1, int32_t n_agents) { return mm::mix_delta_dim(hm, k1, n_agents); }

int mm_lrn_gather(int32_t B, int32_t C, int32_t N, int64_t row_stride, int64_t nd, const int64_t* slots,
                  const int64_t* slot_row, const uint8_t* s_done, const uint8_t* s_act, const float* s_rew,
                  int64_t* s_off, int64_t* s2_off, int32_t* acts, float* rew, float* done, uint8_t* done8,
                  mm_stream_t s) {
  MM_REQUIRE(B > 0 && C > 0 && N > 0, "lrn_gather: bad dims");
  const int n = B * C;
  const mm::SampleGather g = {C, N, row_stride, nd, slot_row, s_done, s_act, s_rew, s_off, s2_off, acts, rew, done,
                              done8};
  hipLaunchKernelGGL(mm::lrn_gather_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s, g, B, slots);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_mixer_fwd(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* obs, const float* reset_obs,
                 const mm_mix_net* nets, int32_t n_nets, mm_stream_t s) {
  MM_REQUIRE(nets && n_nets >= 1 && n_nets <= 2 && B > 0, "mixer_fwd: bad args");
  MM_REQUIRE(3 * Hm <= 4096 && N * K1 <= 4096, "mixer_fwd: dims too large");
  mm::MixFwdArgs a;
  for (int i = 0; i < 2; ++i) {
    const mm_mix_net& n = nets[i < n_nets ? i : 0];
    a.net[i] = {n.P, n.gi, n.q, n.s_off, n.h_in, n.reset, n.h_out, n.qtot, n.save};
  }
  a.obs = obs;
  a.reset_obs = reset_obs;
  a.B = B;
  a.N = N;
  a.S = S;
  a.Hm = Hm;
  a.K1 = K1;
  const size_t sm = sizeof(float) * ((size_t)S + 9 * Hm + N * K1 + 4 * K1);
  MM_REQUIRE(sm <= 64 * 1024, "mixer_fwd: state too large for LDS (%zu B)", sm);
  bool all_gi = true;
  for (int i = 0; i < n_nets; ++i) all_gi = all_gi && nets[i].gi;
  const size_t smm = sizeof(float) * (size_t)mm::MIX_SPB * (9 * Hm + N * K1 + 4 * K1);
  if (B >= 512 && all_gi && smm <= 64 * 1024 && mm::g_mix_multi) {
    hipLaunchKernelGGL(mm::mixer_fwd_multi_kernel, dim3((B + mm::MIX_SPB - 1) / mm::MIX_SPB, n_nets), dim3(256), smm,
                       (hipStream_t)s, a);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  hipLaunchKernelGGL(mm::mixer_fwd_kernel, dim3(B, n_nets), dim3(256), sm, (hipStream_t)s, a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_mixer_gi(int32_t R, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* obs, const float* reset_obs,
                const float* P0, const int64_t* s_off0, float* gi0, const float* P1, const int64_t* s_off1, float* gi1,
                mm_stream_t s) {
  MM_REQUIRE(R > 0 && P0 && gi0 && obs && (s_off0 || !P1), "mixer_gi: bad args");
  mm::MixGiArgs a;
  a.net[0] = {P0, s_off0, gi0};
  a.net[1] = {P1 ? P1 : P0, P1 ? s_off1 : s_off0, P1 ? gi1 : gi0};
  a.obs = obs;
  a.reset_obs = reset_obs;
  a.R = R;
  a.S = S;
  a.Hm = Hm;
  a.K1 = K1;
  a.N = N;
  // small R (B = 32 updates): the split-K register kernel gives more blocks and wins
  if (R >= 2048) {
    dim3 grid((3 * Hm + 63) / 64, (R + 63) / 64, P1 ? 2 : 1);
    hipLaunchKernelGGL(mm::mixer_gi_tiled_kernel, grid, dim3(256), 0, (hipStream_t)s, a);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  dim3 grid((R + 31) / 32, (3 * Hm + 31) / 32, P1 ? 2 : 1);
  hipLaunchKernelGGL(mm::mixer_gi_kernel, grid, dim3(256), 0, (hipStream_t)s, a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_mixer_gi_f16(int32_t R, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* obs, const float* reset_obs,
                    const float* P0, const int64_t* s_off0, float* gi0, const float* P1, const int64_t* s_off1,
                    float* gi1, mm_stream_t s) {
  MM_REQUIRE(R > 0 && P0 && gi0 && obs && (s_off0 || !P1), "mixer_gi_f16: bad args");
  MM_REQUIRE(Hm == 32 || Hm == 64, "mixer_gi_f16: Hm must be 32 or 64");
  MM_REQUIRE((((uintptr_t)gi0 | (uintptr_t)gi1) & 15) == 0, "mixer_gi_f16: gi must be 16-byte aligned");
  mm::MixGiArgs a;
  a.net[0] = {P0, s_off0, gi0};
  a.net[1] = {P1 ? P1 : P0, P1 ? s_off1 : s_off0, P1 ? gi1 : gi0};
  a.obs = obs;
  a.reset_obs = reset_obs;
  a.R = R;
  a.S = S;
  a.Hm = Hm;
  a.K1 = K1;
  a.N = N;
  dim3 grid((R + 63) / 64, P1 ? 2 : 1);
  if (Hm == 32)
    hipLaunchKernelGGL(mm::mixer_gi_f16_kernel<3>, grid, dim3(384), 0, (hipStream_t)s, a);
  else
    hipLaunchKernelGGL(mm::mixer_gi_f16_kernel<6>, grid, dim3(768), 0, (hipStream_t)s, a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_lrn_loss_ex(int32_t B, int32_t C, int32_t N, float gamma, const float* rew, const float* done,
                   const float* isw, const float* qtot, const float* qtot_t, int32_t flags, const float* qa,
                   const float* maxq, float* dq, float* dqa, float* loss_parts, float* td_last, float* loss,
                   mm_stream_t s) {
  MM_REQUIRE(B > 0 && C > 0 && N > 0 && rew && done && dq && loss_parts && td_last && loss, "lrn_loss: bad args");
  MM_REQUIRE((flags & MM_LOSS_MIX_SUM) ? (qa && maxq && dqa) : (qtot && qtot_t), "lrn_loss: missing Q inputs");
  MM_REQUIRE((flags & MM_LOSS_TARGET_SUM) || isw, "lrn_loss: isw required");
  const int n = B * C;
  if (n <= 1024 && B <= 256 && C <= 256) {
    const mm::LossArgs a = {B, C, N, gamma, rew, done, isw, qtot, qtot_t, flags, qa, maxq, dq, dqa, loss_parts,
                            td_last, loss};
    hipLaunchKernelGGL(mm::lrn_loss_small_kernel, dim3(1), dim3(1024), 0, (hipStream_t)s, a);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  hipLaunchKernelGGL(mm::lrn_loss_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s, B, C, N, gamma, rew,
                     done, isw, qtot, qtot_t, flags, qa, maxq, dq, dqa, loss_parts, td_last);
  MM_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(mm::lrn_loss_reduce_kernel, dim3(1), dim3(256), 0, (hipStream_t)s, B, C, loss_parts, loss);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_lrn_loss(int32_t B, int32_t C, int32_t N, float gamma, const float* rew, const float* done, const float* isw,
                const float* qtot, const float* qtot_t, int32_t mix_sum, const float* qa, const float* maxq,
                float* dq, float* dqa, float* loss_parts, float* td_last, float* loss, mm_stream_t s) {
  const int n = B * C;
  hipLaunchKernelGGL(mm::lrn_loss_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s, B, C, N, gamma, rew,
                     done, isw, qtot, qtot_t, mix_sum ? MM_LOSS_MIX_SUM : 0, qa, maxq, dq, dqa, loss_parts, td_last);
  MM_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(mm::lrn_loss_reduce_kernel, dim3(1), dim3(256), 0, (hipStream_t)s, B, C, loss_parts, loss);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

static bool mix_split_enabled() { return true; }   // split recurrence / hypernet launches (the LDS sequence kernels
                                                    // remain the fallback for shapes the split path does not take)
// steps per LDS window of the serial mixer kernels
static int mix_rec_win(int C, int Hm, bool bwd) {
  int win = C;
  while (win > 1 && (bwd ? mm::mix_rec_bwd_floats(Hm, win) : mm::mix_rec_fwd_floats(Hm, win)) * 4 > mm::kMixSeqLds)
    win = (win + 1) / 2;
  return win;
}

// the split (hypernet + recurrence) mixer backward applies: one launch each, so a caller may run the recurrence
// beside the agent BPTT (it reads only the mixer's own saves and the hypernet pass's dhm / delta)
static bool mix_bwd_split_ok(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* ws,
                             int32_t steps) {
  const int win = mix_rec_win(steps, Hm, true);
  return B < 512 && ws && mix_split_enabled() && mm::mix_rec_supported(Hm) &&
         mm::mix_rec_bwd_floats(Hm, win) * 4 <= mm::kMixSeqLds && mm::mix_hyper_bwd_floats(Hm, K1, N) * 4 <= mm::kMixSeqLds &&
         Hm % 4 == 0 && K1 % 4 == 0 && mm::mix_offsets(S, Hm, K1, N).w1W % 4 == 0 && (uintptr_t)P % 16 == 0 &&
         (uintptr_t)ws % 16 == 0;
}

// part 0: the whole backward; 1: the hypernet pass only (dq -> dqa, dhm, delta); 2: the recurrence only
// pu (part 1, may be null): the PER priority update as one more block of the hypernet launch
static int mixer_bwd_seq_part(int part, int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P,
                              const float* save, const float* qa, const float* dq, const float* done, const float* ones,
                              float* dhm, float* dqa, float* delta, float* ws, int32_t steps, mm_stream_t s,
                              const mm::PerUpd* pu = nullptr) {
  MM_REQUIRE(P && save && qa && dq && done && ones && dhm && dqa && delta && steps >= 1, "mixer_bwd_seq: bad args");
  MM_REQUIRE(part == 0 || mix_bwd_split_ok(B, N, S, Hm, K1, P, ws, steps),
             "mixer_bwd_seq: the hypernet / recurrence parts need the split path (mm_mixer_seq_split)");
  mm::MixBwdArgs a = {P, save, qa, dq, done, dhm, dqa, delta, B, N, S, Hm, K1};
  mm::MixBwdSeq q;
  q.C = steps;
  q.save_st = (int64_t)B * mm::mix_save_dim(Hm, K1, N);
  q.qa_st = (int64_t)B * N;
  q.dq_st = B;
  q.done_st = B;
  q.dqa_st = (int64_t)B * N;
  q.delta_st = (int64_t)B * mm::mix_delta_dim(Hm, K1, N);
  q.ones = ones;
  const size_t smm = sizeof(float) * (size_t)mm::MIX_SPB * (4 * Hm + N * K1 + 3 * K1 + 4 * Hm);
  if (B >= 512 && smm <= 64 * 1024 && mm::g_mix_multi) {
    hipLaunchKernelGGL(mm::mixer_bwd_seq_multi_kernel, dim3((B + mm::MIX_SPB - 1) / mm::MIX_SPB), dim3(256), smm,
                       (hipStream_t)s, a, q);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  const int win = mix_rec_win(steps, Hm, true);
  MM_REQUIRE(!ws || (uintptr_t)ws % 16 == 0, "mixer_bwd_seq: ws must be 16-byte aligned");
  if (ws && mix_split_enabled() && mm::mix_rec_supported(Hm) && mm::mix_rec_bwd_floats(Hm, win) * 4 <= mm::kMixSeqLds &&
      mm::mix_hyper_bwd_floats(Hm, K1, N) * 4 <= mm::kMixSeqLds && Hm % 4 == 0 && K1 % 4 == 0 &&
      mm::mix_offsets(S, Hm, K1, N).w1W % 4 == 0 && (uintptr_t)P % 16 == 0) {
    const int rc = mm::mix_seq_lds_setup();
    if (rc) return rc;
    const int R = B * steps;
    if (part != 2) {
      const int nbh = (R + mm::MIX_SPB - 1) / mm::MIX_SPB;
      if (pu)
        hipLaunchKernelGGL(mm::mixer_hyper_bwd_kernel<true>, dim3(nbh + 1), dim3(256),
                           mm::mix_hyper_bwd_floats(Hm, K1, N) * 4, (hipStream_t)s, a, R, ws,
                           mm::debug_trace_buffer("MM_HYB_TRACE"), *pu);
      else
        hipLaunchKernelGGL(mm::mixer_hyper_bwd_kernel<false>, dim3(nbh), dim3(256),
                           mm::mix_hyper_bwd_floats(Hm, K1, N) * 4, (hipStream_t)s, a, R, ws,
                           mm::debug_trace_buffer("MM_HYB_TRACE"), mm::PerUpd{});
      MM_HIP_CHECK(hipGetLastError());
    }
    if (part == 1) return MM_OK;
    mm::MixRecBwd rq;
    rq.C = steps;
    rq.win = win;
    rq.save_st = q.save_st;
    rq.delta_st = q.delta_st;
    rq.done_st = B;
    rq.done = done;
    rq.xws = ws;
    rq.ones = ones;
    rq.trace = mm::debug_trace_buffer("MM_MIX_TRACE_BWD");
    if (Hm == 32)
      hipLaunchKernelGGL(mm::mixer_rec_bwd_kernel<32>, dim3(B), dim3(256), mm::mix_rec_bwd_floats(Hm, win) * 4,
                         (hipStream_t)s, a, rq);
    else
      hipLaunchKernelGGL(mm::mixer_rec_bwd_kernel<64>, dim3(B), dim3(256), mm::mix_rec_bwd_floats(Hm, win) * 4,
                         (hipStream_t)s, a, rq);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  MM_REQUIRE(part == 0, "mixer_bwd_seq: split path not taken");
  const mm::MixSeqGeo g(Hm, K1, N);
  if (g.bwd_floats() * 4 <= mm::kMixSeqLds && g.step_in() <= 1024) {
    const int rc = mm::mix_seq_lds_setup();
    if (rc) return rc;
    hipLaunchKernelGGL(mm::mixer_bwd_seq_lds_kernel, dim3(B), dim3(256), g.bwd_floats() * 4, (hipStream_t)s, a, q);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  const size_t sm = sizeof(float) * ((size_t)8 * Hm + N * K1 + 3 * K1);
  hipLaunchKernelGGL(mm::mixer_bwd_seq_kernel, dim3(B), dim3(256), sm, (hipStream_t)s, a, q);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_mixer_bwd_seq(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* save,
                     const float* qa, const float* dq, const float* done, const float* ones, float* dhm, float* dqa,
                     float* delta, float* ws, int32_t steps, mm_stream_t s) {
  return mixer_bwd_seq_part(0, B, N, S, Hm, K1, P, save, qa, dq, done, ones, dhm, dqa, delta, ws, steps, s);
}
int mm_mixer_bwd_seq_hyper(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* save,
                           const float* qa, const float* dq, const float* done, const float* ones, float* dhm,
                           float* dqa, float* delta, float* ws, int32_t steps, mm_stream_t s) {
  return mixer_bwd_seq_part(1, B, N, S, Hm, K1, P, save, qa, dq, done, ones, dhm, dqa, delta, ws, steps, s);
}
int mm_mixer_bwd_seq_rec(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* save,
                         const float* qa, const float* dq, const float* done, const float* ones, float* dhm, float* dqa,
                         float* delta, float* ws, int32_t steps, mm_stream_t s) {
  return mixer_bwd_seq_part(2, B, N, S, Hm, K1, P, save, qa, dq, done, ones, dhm, dqa, delta, ws, steps, s);
}

int mm_mixer_fwd_seq_fits(int32_t B, int32_t N, int32_t Hm, int32_t K1) {
  const mm::MixSeqGeo g(Hm, K1, N);
  if (mix_split_enabled())
    return B < 512 && mm::mix_rec_supported(Hm) && mm::mix_rec_fwd_floats(Hm, 1) * 4 <= mm::kMixSeqLds &&
           mm::mix_hyper_fwd_floats(Hm, K1, N) * 4 <= 64 * 1024;
  return B < 512 && g.fwd_floats() * 4 <= mm::kMixSeqLds && 3 * Hm <= 256 && N <= 256;
}

// part 0: the whole forward; 1: the mixer recurrence only (reads gi, not the agents' Q: a caller may run it
// beside the agent forward); 2: the hypernet pass only (after both)
// part 3: no launch, the recurrence's arguments into *a_out / *rq_out (a paired launch, mm_agent_mixer_rec_seq)
static int mixer_fwd_seq_part(int part, int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const mm_mix_net* nets,
                              int32_t n_nets, int32_t steps, const uint8_t* reset_steps, mm_stream_t s,
                              mm::MixFwdArgs* a_out = nullptr, mm::MixRecFwd* rq_out = nullptr) {
  MM_REQUIRE(nets && n_nets >= 1 && n_nets <= 2 && B > 0 && steps >= 1, "mixer_fwd_seq: bad args");
  MM_REQUIRE(part == 0 || mix_split_enabled(), "mixer_fwd_seq: the parts need the split path");
  MM_REQUIRE(steps == 1 || reset_steps, "mixer_fwd_seq: reset_steps required for steps > 1");
  MM_REQUIRE(mm_mixer_fwd_seq_fits(B, N, Hm, K1), "mixer_fwd_seq: B >= 512 or the weights exceed the LDS");
  for (int i = 0; i < n_nets; ++i)
    MM_REQUIRE(nets[i].gi && nets[i].q && nets[i].qtot, "mixer_fwd_seq: gi / q / qtot required");
  mm::MixFwdArgs a;
  for (int i = 0; i < 2; ++i) {
    const mm_mix_net& n = nets[i < n_nets ? i : 0];
    a.net[i] = {n.P, n.gi, n.q, n.s_off, n.h_in, n.reset, n.h_out, n.qtot, n.save};
  }
  a.obs = nullptr;
  a.reset_obs = nullptr;
  a.B = B;
  a.N = N;
  a.S = S;
  a.Hm = Hm;
  a.K1 = K1;
  mm::MixFwdSeq q;
  q.C = steps;
  q.gi_st = (int64_t)B * 3 * Hm;
  q.q_st = (int64_t)B * N;
  q.qtot_st = B;
  q.save_st = (int64_t)B * mm::mix_save_dim(Hm, K1, N);
  q.hout_st = 0;
  q.reset_steps = reset_steps;
  const int rc = mm::mix_seq_lds_setup();
  if (rc) return rc;
  if (mix_split_enabled()) {
    for (int i = 0; i < n_nets; ++i) {
      MM_REQUIRE(nets[i].h_out, "mixer_fwd_seq: h_out [C][B][Hm] required");
      MM_REQUIRE((uintptr_t)nets[i].gi % 16 == 0, "mixer_fwd_seq: gi must be 16-byte aligned");
    }
    mm::MixRecFwd rq;
    rq.C = steps;
    rq.win = mix_rec_win(steps, Hm, false);
    rq.gi_st = q.gi_st;
    rq.hout_st = (int64_t)B * Hm;
    rq.save_st = q.save_st;
    rq.reset_steps = reset_steps;
    rq.trace = mm::debug_trace_buffer("MM_MIX_TRACE_FWD");
    if (part == 3) {
      *a_out = a;
      *rq_out = rq;
      return MM_OK;
    }
    if (part != 2) {
      if (Hm == 32)
        hipLaunchKernelGGL(mm::mixer_rec_fwd_kernel<32>, dim3(B, n_nets), dim3(256),
                           mm::mix_rec_fwd_floats(Hm, rq.win) * 4, (hipStream_t)s, a, rq);
      else
        hipLaunchKernelGGL(mm::mixer_rec_fwd_kernel<64>, dim3(B, n_nets), dim3(256),
                           mm::mix_rec_fwd_floats(Hm, rq.win) * 4, (hipStream_t)s, a, rq);
      MM_HIP_CHECK(hipGetLastError());
    }
    if (part == 1) return MM_OK;
    const int R = B * steps;
    hipLaunchKernelGGL(mm::mixer_hyper_fwd_kernel, dim3((R + mm::MIX_SPB - 1) / mm::MIX_SPB, n_nets), dim3(256),
                       mm::mix_hyper_fwd_floats(Hm, K1, N) * 4, (hipStream_t)s, a, R);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  const mm::MixSeqGeo g(Hm, K1, N);
  hipLaunchKernelGGL(mm::mixer_fwd_seq_lds_kernel, dim3(B, n_nets), dim3(256), g.fwd_floats() * 4, (hipStream_t)s, a,
                     q);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_mixer_fwd_seq(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const mm_mix_net* nets,
                     int32_t n_nets, int32_t steps, const uint8_t* reset_steps, mm_stream_t s) {
  return mixer_fwd_seq_part(0, B, N, S, Hm, K1, nets, n_nets, steps, reset_steps, s);
}
int mm_mixer_fwd_seq_rec(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const mm_mix_net* nets,
                         int32_t n_nets, int32_t steps, const uint8_t* reset_steps, mm_stream_t s) {
  return mixer_fwd_seq_part(1, B, N, S, Hm, K1, nets, n_nets, steps, reset_steps, s);
}
int mm_mixer_fwd_seq_hyper(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const mm_mix_net* nets,
                           int32_t n_nets, int32_t steps, const uint8_t* reset_steps, mm_stream_t s) {
  return mixer_fwd_seq_part(2, B, N, S, Hm, K1, nets, n_nets, steps, reset_steps, s);
}

int mm_mixer_seq_split(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* ws,
                       int32_t steps) {
  return (mm_mixer_fwd_seq_fits(B, N, Hm, K1) && mix_split_enabled() &&
          mix_bwd_split_ok(B, N, S, Hm, K1, P, ws, steps)) ? 1 : 0;
}

int mm_mixer_bwd(int32_t B, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* P, const float* save,
                 const float* qa, const float* dq, const float* done, float* dhm, float* dqa, float* delta,
                 mm_stream_t s) {
  mm::MixBwdArgs a = {P, save, qa, dq, done, dhm, dqa, delta, B, N, S, Hm, K1};
  const size_t sm = sizeof(float) * ((size_t)8 * Hm + N * K1 + 3 * K1);
  hipLaunchKernelGGL(mm::mixer_bwd_kernel, dim3(B), dim3(256), sm, (hipStream_t)s, a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

// The agent BPTT's kernel arguments and dynamic LDS size (mm_agent_bwd_seq, mm_agent_mixer_bwd_seq)
static int agent_bwd_seq_prep(const mm_qnet_dims* d, const float* P, int64_t oWq, int64_t oWhh, int32_t B,
                              const float* save, const int32_t* acts, const float* dqa, const float* done,
                              const float* ones, float* dh, float* dgi, float* dgh, float* dq, int32_t steps,
                              mm::AgentBwdArgs* a, mm::AgentBwdSeq* q, size_t* smem) {
  MM_REQUIRE(d && P && save && acts && dqa && done && ones && dh && dgi && dgh && dq && steps >= 1 && B > 0,
             "agent_bwd_seq: bad args");
  MM_REQUIRE((d->h == 32 || d->h == 64) && d->n_actions <= 64, "agent_bwd_seq: needs H in {32, 64} and A <= 64");
  MM_REQUIRE(oWhh % 4 == 0 && (uintptr_t)P % 16 == 0 && (uintptr_t)save % 16 == 0 && (d->f1 + d->g) % 4 == 0,
             "agent_bwd_seq: W_hh / save rows must be 16-byte aligned (16-byte LDS-DMA)");
  int win = steps;
  while (win > 1 && mm::agent_bwd_seq_floats(d->h, d->n_actions, win) * 4 > mm::kMixSeqLds) win = (win + 1) / 2;
  *smem = sizeof(float) * mm::agent_bwd_seq_floats(d->h, d->n_actions, win);
  MM_REQUIRE(*smem <= mm::kMixSeqLds, "agent_bwd_seq: W_hh too large for LDS");
  {
    // thread-safe one-time setup (a function-local static's initialiser runs once); the sizes are compile-time
    static const int attr_rc = [&]() -> int {
      const void* k[] = {(const void*)mm::agent_bwd_seq_kernel<32>, (const void*)mm::agent_bwd_seq_kernel<64>,
                         (const void*)mm::agent_mixer_bwd_kernel<32, 32>, (const void*)mm::agent_mixer_bwd_kernel<32, 64>,
                         (const void*)mm::agent_mixer_bwd_kernel<64, 32>, (const void*)mm::agent_mixer_bwd_kernel<64, 64>};
      for (const void* f : k)
        MM_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mm::kMixSeqLds));
      return MM_OK;
    }();
    if (attr_rc != MM_OK) return attr_rc;
  }
  *a = {P, oWq, oWhh, save, acts, dqa, done, dh, dgi, dgh, dq, B, d->n_agents, d->f1, d->g, d->h, d->n_actions};
  const int64_t BN = (int64_t)B * d->n_agents;
  q->C = steps;
  q->save_st = BN * (d->f1 + d->g + 6 * d->h);
  q->acts_st = BN;
  q->dqa_st = BN;
  q->dgi_st = BN * 3 * d->h;
  q->dq_st = BN * d->n_actions;
  q->done_st = B;
  q->ones = ones;
  q->win = win;
  q->trace = mm::debug_trace_buffer("MM_ABWD_TRACE");
  return MM_OK;
}

int mm_agent_bwd_seq(const mm_qnet_dims* d, const float* P, int64_t oWq, int64_t oWhh, int32_t B, const float* save,
                     const int32_t* acts, const float* dqa, const float* done, const float* ones, float* dh,
                     float* dgi, float* dgh, float* dq, int32_t steps, mm_stream_t s) {
  mm::AgentBwdArgs a;
  mm::AgentBwdSeq q;
  size_t smem = 0;
  const int rc = agent_bwd_seq_prep(d, P, oWq, oWhh, B, save, acts, dqa, done, ones, dh, dgi, dgh, dq, steps, &a, &q,
                                    &smem);
  if (rc) return rc;
  if (d->h == 32)
    hipLaunchKernelGGL(mm::agent_bwd_seq_kernel<32>, dim3((B + 3) / 4, d->n_agents), dim3(256), smem, (hipStream_t)s,
                       a, q);
  else
    hipLaunchKernelGGL(mm::agent_bwd_seq_kernel<64>, dim3((B + 3) / 4, d->n_agents), dim3(256), smem, (hipStream_t)s,
                       a, q);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_agent_mixer_bwd_seq(const mm_qnet_dims* d, const float* P, int64_t oWq, int64_t oWhh, int32_t B,
                           const float* save, const int32_t* acts, const float* dqa, const float* done,
                           const float* ones, float* dh, float* dgi, float* dgh, float* dq, int32_t steps, int32_t S,
                           int32_t Hm, int32_t K1, const float* mP, const float* msave, const float* qa,
                           const float* mdq, float* dhm, float* mdelta, float* ws, mm_stream_t s) {
  mm::AgentBwdArgs a;
  mm::AgentBwdSeq q;
  size_t smem = 0;
  int rc = agent_bwd_seq_prep(d, P, oWq, oWhh, B, save, acts, dqa, done, ones, dh, dgi, dgh, dq, steps, &a, &q, &smem);
  if (rc) return rc;
  MM_REQUIRE(mP && msave && qa && mdq && dhm && mdelta && (Hm == 32 || Hm == 64) &&
                 mix_bwd_split_ok(B, d->n_agents, S, Hm, K1, mP, ws, steps),
             "agent_mixer_bwd_seq: the mixer recurrence needs the split path (mm_mixer_seq_split)");
  rc = mm::mix_seq_lds_setup();
  if (rc) return rc;
  const int N = d->n_agents;
  const mm::MixBwdArgs ma = {mP, msave, qa, mdq, done, dhm, const_cast<float*>(dqa), mdelta, B, N, S, Hm, K1};
  mm::MixRecBwd mq;
  mq.C = steps;
  mq.win = mix_rec_win(steps, Hm, true);
  mq.save_st = (int64_t)B * mm::mix_save_dim(Hm, K1, N);
  mq.delta_st = (int64_t)B * mm::mix_delta_dim(Hm, K1, N);
  mq.done_st = B;
  mq.done = done;
  mq.xws = ws;
  mq.ones = ones;
  mq.trace = mm::debug_trace_buffer("MM_MIX_TRACE_BWD");
  const size_t sm = std::max(smem, mm::mix_rec_bwd_floats(Hm, mq.win) * 4);
  const int gx = (B + 3) / 4, na = gx * N;
#define MM_PAIR(HA, HMX)                                                                                          \
  hipLaunchKernelGGL((mm::agent_mixer_bwd_kernel<HA, HMX>), dim3(na + B), dim3(256), sm, (hipStream_t)s, a, q, ma, \
                     mq, gx, na)
  if (d->h == 32 && Hm == 32) MM_PAIR(32, 32);
  else if (d->h == 32) MM_PAIR(32, 64);
  else if (Hm == 32) MM_PAIR(64, 32);
  else MM_PAIR(64, 64);
#undef MM_PAIR
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_agent_bwd(const mm_qnet_dims* d, const float* P, int64_t oWq, int64_t oWhh, int32_t B, const float* save,
                 const int32_t* acts, const float* dqa, const float* done, float* dh, float* dgi, float* dgh,
                 float* dq, mm_stream_t s) {
  MM_REQUIRE(d && d->h <= 256, "agent_bwd: H must be <= 256");
  mm::AgentBwdArgs a = {P, oWq, oWhh, save, acts, dqa, done, dh, dgi, dgh, dq,
                        B, d->n_agents, d->f1, d->g, d->h, d->n_actions};
  const int pairs = B * d->n_agents;
  if (B >= 512 && d->h <= 64 && mm::g_bwd_multi) {
    hipLaunchKernelGGL(mm::agent_bwd_multi_kernel, dim3((B + 4 * mm::BWD_SPW - 1) / (4 * mm::BWD_SPW), d->n_agents),
                       dim3(256), 0, (hipStream_t)s, a);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  hipLaunchKernelGGL(mm::agent_bwd_kernel, dim3((pairs + 3) / 4), dim3(256), 0, (hipStream_t)s, a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

int mm_outer_reduce(const mm_outer_args* x, mm_stream_t s) {
  MM_REQUIRE(x && x->M >= 0 && x->R > 0 && x->Cc > 0 && x->groups > 0, "outer_reduce: bad args");
  mm::OuterArgs a = {x->U, x->u_g, x->u_m, x->V, x->v_g, x->v_m, x->v_off, x->v_reset, x->dW, x->w_g,
                     x->db, x->b_g, x->M, x->R, x->Cc, x->accumulate};
  dim3 grid((x->Cc + 31) / 32, (x->R + 31) / 32, x->groups);
  hipLaunchKernelGGL(mm::outer_reduce_kernel, grid, dim3(256), 0, (hipStream_t)s, a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

static int64_t outer_batch_layout(const mm_outer_args* x, int n, mm::OuterBatch* ob) {
  int blk = 0;
  int64_t part = 0;
  for (int j = 0; j < n; ++j) {
    const mm_outer_args& q = x[j];
    ob->job[j] = {q.U, q.u_g, q.u_m, q.V, q.v_g, q.v_m, q.v_off, q.v_reset, q.dW, q.w_g, q.db, q.b_g, q.M, q.R,
                  q.Cc, q.accumulate};
    // tile shape with the least padded area (ties: fewer row tiles)
    int best = 0;
    int64_t best_area = -1;
    for (int sh = 2; sh >= 0; --sh) {
      const int TR = 32 << sh, TC = 128 >> sh;
      const int64_t area = (int64_t)((q.R + TR - 1) / TR) * TR * ((q.Cc + TC - 1) / TC) * TC;
      if (best_area < 0 || area < best_area) {
        best_area = area;
        best = sh;
      }
    }
    ob->tr_shift[j] = best;
    ob->tiles_r[j] = (q.R + (32 << best) - 1) / (32 << best);
    ob->tiles_c[j] = (q.Cc + (128 >> best) - 1) / (128 >> best);
    ob->groups[j] = q.groups;
    // slices of 32-row chunks: about 4096 blocks per job (long-lived blocks, bounded partials), at most 64
    const int chunks = (q.M + 31) / 32;
    const int64_t tiles = (int64_t)ob->tiles_r[j] * ob->tiles_c[j] * q.groups;
    int want = (int)std::min<int64_t>(64, std::max<int64_t>(1, (4096 + tiles - 1) / tiles));
    want = std::min(want, chunks);
    ob->rps[j] = 32 * ((chunks + want - 1) / want);
    ob->slices[j] = (q.M + ob->rps[j] - 1) / ob->rps[j];
    ob->blk0[j] = blk;
    ob->part[j] = part;
    blk += (int)(tiles * ob->slices[j]);
    part += (int64_t)ob->slices[j] * q.groups * ((int64_t)q.R * q.Cc + q.R);
  }
  ob->blk0[n] = blk;
  ob->njobs = n;
  return part;
}

int64_t mm_outer_reduce_batch_partial(const mm_outer_args* x, int32_t n_jobs) {
  if (!x || n_jobs < 1 || n_jobs > mm::OB_MAX) return -1;
  mm::OuterBatch ob;
  return outer_batch_layout(x, n_jobs, &ob);
}

static int outer_reduce_batch_impl(const mm_outer_args* x, int32_t n_jobs, float* partial, int64_t partial_count,
                                   int bf3, mm_stream_t s);
int mm_outer_reduce_batch(const mm_outer_args* x, int32_t n_jobs, float* partial, int64_t partial_count,
                          mm_stream_t s) {
  return outer_reduce_batch_impl(x, n_jobs, partial, partial_count, 0, s);
}
int mm_outer_reduce_batch_bf3(const mm_outer_args* x, int32_t n_jobs, float* partial, int64_t partial_count,
                              mm_stream_t s) {
  return outer_reduce_batch_impl(x, n_jobs, partial, partial_count, 1, s);
}
static int outer_reduce_batch_impl(const mm_outer_args* x, int32_t n_jobs, float* partial, int64_t partial_count,
                                   int bf3, mm_stream_t s) {
  MM_REQUIRE(x && partial && n_jobs >= 1 && n_jobs <= mm::OB_MAX, "outer_reduce_batch: bad args");
  mm::OuterBatch ob;
  int64_t maxper = 0;
  for (int j = 0; j < n_jobs; ++j) {
    MM_REQUIRE(x[j].M > 0 && x[j].R > 0 && x[j].Cc > 0 && x[j].groups > 0, "outer_reduce_batch: bad job %d", j);
    maxper = std::max<int64_t>(maxper, ((int64_t)x[j].R * x[j].Cc + x[j].R) * x[j].groups);
  }
  const int64_t need = outer_batch_layout(x, n_jobs, &ob);
  MM_REQUIRE(need <= partial_count, "outer_reduce_batch: partial buffer too small (%lld < %lld)",
             (long long)partial_count, (long long)need);
  ob.partial = partial;
  ob.bf3 = bf3;
  hipLaunchKernelGGL(mm::outer_batch_kernel, dim3(ob.blk0[n_jobs]), dim3(256), 0, (hipStream_t)s, ob);
  MM_HIP_CHECK(hipGetLastError());
  const int gx = (int)std::min<int64_t>((maxper + 255) / 256, 1024);
  hipLaunchKernelGGL(mm::outer_sum_kernel, dim3(gx, n_jobs), dim3(256), 0, (hipStream_t)s, ob);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

// Mixer weight gradients of R = rows samples from the backward's per-row operands (mm_mixer_bwd /
// mm_mixer_bwd_seq delta [R][mm_mixer_delta_dim], the forward's save [R][mm_mixer_save_dim]) and the
// states (state rows through s_off with reset_obs for -1 offsets, or contiguous [R][S] rows when s_off
// is NULL), as ONE batched outer-reduce launch + its fixed-order partial sum (deterministic):
//   gWih/gbih <- d_gi x s,  gWhh/gbhh <- d_gh x h_in,  hypernets <- their deltas x h_out,
//   b2 output layer <- dQ_tot x relu(b2 hidden)          (Mix_Net, qmix/_network.py:172-217)
// dP: the mixer's flat gradient (overwritten).
static int mixer_wgrad_jobs(int32_t R, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* state,
                            const int64_t* s_off, const float* reset_obs, const float* save, const float* delta,
                            float* dP, mm_outer_args* j) {
  const mm::MixOff o = mm::mix_offsets(S, Hm, K1, N);
  const int64_t MSD = mm::mix_save_dim(Hm, K1, N), MDD = mm::mix_delta_dim(Hm, K1, N);
  const float* hm1 = save + 5 * Hm;
  auto job = [&](int i, const float* U, const float* V, int64_t v_m, const int64_t* voff, int64_t w, int64_t b,
                 int32_t rows, int32_t cols) {
    mm_outer_args& a = j[i];
    a.U = U;
    a.u_g = 0;
    a.u_m = MDD;
    a.V = V;
    a.v_g = 0;
    a.v_m = v_m;
    a.v_off = voff;
    a.v_reset = voff ? reset_obs : nullptr;
    a.dW = dP + w;
    a.w_g = 0;
    a.db = dP + b;
    a.b_g = 0;
    a.M = R;
    a.R = rows;
    a.Cc = cols;
    a.accumulate = 0;
    a.groups = 1;
  };
  job(0, delta, state, s_off ? 0 : S, s_off, o.gWih, o.gbih, 3 * Hm, S);
  job(1, delta + 3 * Hm, save, MSD, nullptr, o.gWhh, o.gbhh, 3 * Hm, Hm);
  job(2, delta + 6 * Hm, hm1, MSD, nullptr, o.w1W, o.w1b, N * K1, Hm);
  job(3, delta + 6 * Hm + N * K1, hm1, MSD, nullptr, o.b1W, o.b1b, K1, Hm);
  job(4, delta + 6 * Hm + N * K1 + K1, hm1, MSD, nullptr, o.w2W, o.w2b, K1, Hm);
  job(5, delta + 6 * Hm + N * K1 + 2 * K1, hm1, MSD, nullptr, o.b2aW, o.b2ab, K1, Hm);
  job(6, delta + 6 * Hm + N * K1 + 3 * K1, save + 6 * Hm + N * K1 + 2 * K1, MSD, nullptr, o.b2bW, o.b2bb, 1, K1);
  return 7;
}

int64_t mm_mixer_wgrad_partial_count(int32_t R, int32_t N, int32_t S, int32_t Hm, int32_t K1) {
  if (R < 1 || N < 1 || S < 1 || Hm < 1 || K1 < 1) return -1;
  mm_outer_args j[7];
  const float* f = reinterpret_cast<const float*>(16);
  const int n = mixer_wgrad_jobs(R, N, S, Hm, K1, f, nullptr, nullptr, f, f, const_cast<float*>(f), j);
  return mm_outer_reduce_batch_partial(j, n);
}

int mm_mixer_wgrad(int32_t R, int32_t N, int32_t S, int32_t Hm, int32_t K1, const float* state, const int64_t* s_off,
                   const float* reset_obs, const float* save, const float* delta, float* dP, float* partial,
                   int64_t partial_count, mm_stream_t s) {
  MM_REQUIRE(R > 0 && state && save && delta && dP && partial, "mixer_wgrad: bad args");
  MM_REQUIRE(!s_off || reset_obs, "mixer_wgrad: s_off needs reset_obs");
  mm_outer_args j[7];
  const int n = mixer_wgrad_jobs(R, N, S, Hm, K1, state, s_off, reset_obs, save, delta, dP, j);
  return mm_outer_reduce_batch(j, n, partial, partial_count, s);
}

int mm_tmv(const mm_tmv_args* x, mm_stream_t s) {
  MM_REQUIRE(x && x->M > 0 && x->R > 0 && x->Cc > 0 && x->groups > 0, "tmv: bad args");
  mm::TmvArgs a = {x->W, x->w_g, x->X, x->x_g, x->x_m, x->Z, x->z_g, x->z_m, x->Y, x->y_g, x->y_m,
                   x->M, x->R, x->Cc, 0};
  a.aligned16 = (x->R % 4 == 0 && x->x_m % 4 == 0 && x->x_g % 4 == 0 && x->Cc % 4 == 0 && x->w_g % 4 == 0 &&
                 (uintptr_t)x->X % 16 == 0 && (uintptr_t)x->W % 16 == 0);
  // small M (B = 32 updates): the 32 x 32 scalar tiles give more blocks and win
  if (x->M >= 2048) {
    dim3 grid((x->Cc + 63) / 64, (x->M + 63) / 64, x->groups);
    if (a.aligned16 && x->R <= mm::TMV_FULL_RMAX) {
      const int Rp = (x->R + 31) & ~31;
      const size_t lds = sizeof(float) * 2 * 65 * (size_t)Rp;
      static const int attr_rc = [] {
        MM_HIP_CHECK(hipFuncSetAttribute((const void*)mm::tmv_mfma_full_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)(sizeof(float) * 2 * 65 * mm::TMV_FULL_RMAX)));
        return MM_OK;
      }();
      if (attr_rc != MM_OK) return attr_rc;
      hipLaunchKernelGGL(mm::tmv_mfma_full_kernel, grid, dim3(256), lds, (hipStream_t)s, a);
    } else
      hipLaunchKernelGGL(mm::tmv_mfma_kernel, grid, dim3(256), 0, (hipStream_t)s, a);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  dim3 grid((x->Cc + 31) / 32, (x->M + 31) / 32, x->groups);
  if (x->R <= 256) {   // whole r range staged at once
    hipLaunchKernelGGL(mm::tmv_full_kernel, grid, dim3(256), sizeof(float) * (64 * (size_t)x->R),
                       (hipStream_t)s, a);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
  hipLaunchKernelGGL(mm::tmv_kernel, grid, dim3(256), 0, (hipStream_t)s, a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

// G *= grad_scale (e.g. 1/world after the RCCL sum), clip_grad_norm_(G[0:n_clip], max_norm), then Adam
// over P[0:n]; partials: >= 256 floats scratch
int mm_clip_adam(float* P, float* G, float* m, float* v, int64_t n, int64_t n_clip, float max_norm, float lr,
                 float beta1, float beta2, float eps, float* step, float* partials, float* norm_out, float grad_scale,
                 mm_stream_t s) {
  MM_REQUIRE(P && G && m && v && step && partials && n > 0 && n_clip >= 0 && n_clip <= n, "clip_adam: bad args");
  const int nb = 256;
  hipLaunchKernelGGL(mm::sumsq_kernel, dim3(nb), dim3(256), 0, (hipStream_t)s, G, n_clip, partials, step);
  MM_HIP_CHECK(hipGetLastError());
  const int nb2 = (int)std::min<int64_t>((n + 255) / 256, 2048);
  const mm::AdamArgs a = {P, G, m, v, n, n_clip, partials, nb, max_norm, lr, beta1, beta2, eps, step, norm_out,
                          grad_scale, nullptr};
  hipLaunchKernelGGL(mm::adam_kernel, dim3(nb2), dim3(256), 0, (hipStream_t)s, a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}

// Two clip groups: clip_grad_norm_(G[0:split]) and clip_grad_norm_(G[split:n]) separately (same
// max_norm), then Adam over P[0:n]; partials: >= 512 floats scratch; norm_out (may be null) gets
// both norms.
int mm_clip2_adam(float* P, float* G, float* m, float* v, int64_t n, int64_t split, float max_norm, float lr,
                  float beta1, float beta2, float eps, float* step, float* partials, float* norm_out, float grad_scale,
                  mm_stream_t s) {
  MM_REQUIRE(P && G && m && v && step && partials && n > 0 && split >= 0 && split <= n, "clip2_adam: bad args");
  const int nb = 256;
  hipLaunchKernelGGL(mm::sumsq_kernel, dim3(nb), dim3(256), 0, (hipStream_t)s, G, split, partials, step);
  MM_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(mm::sumsq_kernel, dim3(nb), dim3(256), 0, (hipStream_t)s, G + split, n - split, partials + nb,
                     (float*)nullptr);
  MM_HIP_CHECK(hipGetLastError());
  const int nb2 = (int)std::min<int64_t>((n + 255) / 256, 2048);
  const mm::AdamArgs a = {P, G, m, v, n, split, partials, nb, max_norm, lr, beta1, beta2, eps, step, norm_out,
                          grad_scale, partials + nb};
  hipLaunchKernelGGL(mm::adam_kernel, dim3(nb2), dim3(256), 0, (hipStream_t)s, a);
  MM_HIP_CHECK(hipGetLastError());
  return MM_OK;
}
}
