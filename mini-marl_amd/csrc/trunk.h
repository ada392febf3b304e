// Shared building blocks of the LN-MLP-GRU-LN "trunk" nets (MAPPO R_Actor / R_Critic,
// mappo/utils/algorithm_utils/{mlp,rnn}.py; the offpolicy AgentQFunction has the same shape,
// offpolicy/algorithms/qmix/algorithm/agent_q_function.py): flat parameter geometry, tiled-SoA
// save / gradient-operand fields, per-thread LayerNorm / mat-vec helpers and the MFMA
// weight-gradient reduction over rows.
#pragma once
#include "common.h"
#include "minimarl.h"

namespace mm {

constexpr float kLnEps = 1e-5f;

template <int D, int H, int O>
struct MGeo {
  static constexpr int Dp = (D + 3) & ~3, Op = (O + 3) & ~3;
  static constexpr int ln0_w = 0, ln0_b = Dp, W1 = 2 * Dp, b1 = W1 + H * Dp, ln1_w = b1 + H, ln1_b = ln1_w + H;
  static constexpr int W2 = ln1_b + H, b2 = W2 + H * H, ln2_w = b2 + H, ln2_b = ln2_w + H;
  static constexpr int Wih = ln2_b + H, Whh = Wih + 3 * H * H, bih = Whh + 3 * H * H, bhh = bih + 3 * H;
  static constexpr int lnr_w = bhh + 3 * H, lnr_b = lnr_w + H, Wo = lnr_b + H, bo = Wo + Op * H;
  static constexpr int total = bo + Op;
};

// forward save fields (tiled SoA, see soa_col; row = t*EN + en), per net
template <int H, int O>
struct SF {
  static constexpr int MU0 = 0, RS0 = 1, A1 = 2, MU1 = A1 + H, RS1 = MU1 + 1, A2 = RS1 + 1, MU2 = A2 + H,
                       RS2 = MU2 + 1, HIN = RS2 + 1, R = HIN + H, Z = R + H, N = Z + H, GHN = N + H, H2 = GHN + H,
                       MUR = H2 + H, RSR = MUR + 1, OUT = RSR + 1, NS = OUT + O;
};
// backward output fields (SoA), operands of the weight-gradient reduction
template <int D, int H, int O>
struct GF {
  static constexpr int DOUT = 0, Y = DOUT + O, DGI = Y + H, X2 = DGI + 3 * H, DGH = X2 + H, HIN = DGH + 3 * H,
                       DPRE2 = HIN + H, F1 = DPRE2 + H, DPRE1 = F1 + H, F0 = DPRE1 + H, DY = F0 + D, PY = DY + H,
                       DX2 = PY + H, P2 = DX2 + H, DX1 = P2 + H, P1 = DX1 + H, DF0 = P1 + H, P0 = DF0 + D,
                       NG = P0 + D;
};

// ------------------------------------------------------------------ per-thread building blocks
template <int OUT, int IN, int LD>
__device__ __forceinline__ void matvec(const float* __restrict__ W, const float* __restrict__ b, const float (&x)[IN],
                                       float (&y)[OUT]) {
#pragma unroll
  for (int o = 0; o < OUT; ++o) {
    float acc = b[o];
#pragma unroll
    for (int i = 0; i < IN; ++i) acc = fmaf(W[o * LD + i], x[i], acc);
    y[o] = acc;
  }
}

template <int OUT, int IN, int LD>
__device__ __forceinline__ void matvec_t(const float* __restrict__ W, const float (&d)[OUT], float (&dx)[IN]) {
#pragma unroll
  for (int i = 0; i < IN; ++i) dx[i] = 0.0f;
#pragma unroll
  for (int o = 0; o < OUT; ++o)
#pragma unroll
    for (int i = 0; i < IN; ++i) dx[i] = fmaf(W[o * LD + i], d[o], dx[i]);
}

template <int N>
__device__ __forceinline__ void ln_stats(const float (&x)[N], float& mu, float& rs) {
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < N; ++i) s += x[i];
  mu = s / (float)N;
  float v = 0.0f;
#pragma unroll
  for (int i = 0; i < N; ++i) v = fmaf(x[i] - mu, x[i] - mu, v);
  rs = 1.0f / sqrtf(v / (float)N + kLnEps);
}

template <int N>
__device__ __forceinline__ void ln_apply(const float (&x)[N], float mu, float rs, const float* w, const float* b,
                                         float (&y)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) y[i] = (x[i] - mu) * rs * w[i] + b[i];
}

// dx = rs * (g - mean(g) - xhat * mean(g * xhat)), g = dy * w
template <int N>
__device__ __forceinline__ void ln_bwd(const float (&dy)[N], const float (&xh)[N], float rs, const float* w,
                                       float (&dx)[N]) {
  float sg = 0.0f, sgx = 0.0f;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float g = dy[i] * w[i];
    sg += g;
    sgx = fmaf(g, xh[i], sgx);
  }
  sg /= (float)N;
  sgx /= (float)N;
#pragma unroll
  for (int i = 0; i < N; ++i) dx[i] = rs * (dy[i] * w[i] - sg - xh[i] * sgx);
}

// Tiled SoA arrays: rows in tiles of 64, [tile][field][64] -> a field's 64 rows are contiguous
// (coalesced per wave) and the field stride is the compile-time 64 floats.
__device__ __forceinline__ float* soa_col(float* base, int64_t row, int nf) {
  return base + (row >> 6) * (int64_t)nf * 64 + (row & 63);
}
__device__ __forceinline__ const float* soa_col(const float* base, int64_t row, int nf) {
  return base + (row >> 6) * (int64_t)nf * 64 + (row & 63);
}

template <int D>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&x)[D]) {
#pragma unroll
  for (int i = 0; i < D; ++i) x[i] = p[i];
}

// Stage a net's flat parameters (multiple of 4 floats) into LDS.
__device__ __forceinline__ void stage_params(float* sm, const float* __restrict__ P, int n) {
  const float4* s = reinterpret_cast<const float4*>(P);
  float4* d = reinterpret_cast<float4*>(sm);
  for (int i = threadIdx.x; i < n / 4; i += blockDim.x) d[i] = s[i];
  __syncthreads();
}

// SoA column access with the address kept in VGPRs: every 16-field window starts from an
// opaque pointer (asm barrier) and uses immediate offsets, so the compiler cannot hoist ~1000
// uniform field offsets into SGPRs (which spilled thousands of SGPRs).
template <int N>
__device__ __forceinline__ void soa_st(float* col, int f0, const float (&v)[N]) {
#pragma unroll
  for (int c = 0; c < N; c += 16) {
    float* q = col + (f0 + c) * 64;
    asm volatile("" : "+v"(q));
#pragma unroll
    for (int i = c; i < (N < c + 16 ? N : c + 16); ++i) q[(i - c) * 64] = v[i];
  }
}
template <int N>
__device__ __forceinline__ void soa_ld(const float* col, int f0, float (&v)[N]) {
#pragma unroll
  for (int c = 0; c < N; c += 16) {
    const float* q = col + (f0 + c) * 64;
    asm volatile("" : "+v"(q));
#pragma unroll
    for (int i = c; i < (N < c + 16 ? N : c + 16); ++i) v[i] = q[(i - c) * 64];
  }
}
__device__ __forceinline__ void soa_st1(float* col, int f, float v) {
  float* q = col + f * 64;
  asm volatile("" : "+v"(q));
  *q = v;
}
__device__ __forceinline__ float soa_ld1(const float* col, int f) {
  const float* q = col + f * 64;
  asm volatile("" : "+v"(q));
  return *q;
}

// ------------------------------------------------------------------ weight-gradient reduction
// dW[M][K] = sum_r A[m][r] * B[k][r], db[m] = sum_r A[m][r] over tiled SoA operands (soa_col),
// on v_mfma_f32_32x32x2_f32 with the reduction (row) index on the MFMA k dimension: lane (i, h)
// of k-step s supplies row r0 + 16 h + s of feature i, so each lane streams 64 contiguous bytes
// per operand per 32 rows. Every block reduces one job over one row range for all (m, k) tiles
// of the job (operands read from HBM once) and writes a partial; a second kernel sums partials.
struct WgJobDev {
  const float* A;
  const float* B;
  float* dW;
  float* db;
  int M, K, ldw, blk0, nblk;
  int64_t part;  // offset of this job's partials: nblk x (M*K + M)
};
struct WgArgsDev {
  WgJobDev job[MM_MAPPO_MAX_JOBS];
  int njobs;
  int nf;  // fields of the tiled SoA operand array (tile stride nf * 64)
  int64_t Rs, rows_per_block;
  float* partial;
};

__device__ __forceinline__ void load16(const float* p, bool ok, float (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4 t = ok ? *reinterpret_cast<const float4*>(p + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    v[4 * q] = t.x;
    v[4 * q + 1] = t.y;
    v[4 * q + 2] = t.z;
    v[4 * q + 3] = t.w;
  }
}

// Jobs are split on the host so that M <= 96 (3 m-tiles) and K <= 64 (2 k-tiles).
static __global__ __launch_bounds__(256) void mappo_wgrad_kernel(WgArgsDev a) {
  int j = 0;
  while (j + 1 < a.njobs && (int)blockIdx.x >= a.job[j + 1].blk0) ++j;
  const WgJobDev& jb = a.job[j];
  const int b = blockIdx.x - jb.blk0;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 31, hh = lane >> 5;
  const int MT = (jb.M + 31) / 32, KT = (jb.K + 31) / 32;
  const int64_t r_begin = (int64_t)b * a.rows_per_block;
  const int64_t r_end = min(r_begin + a.rows_per_block, a.Rs);
  const int64_t tile = (int64_t)a.nf * 64;
  f32x16 acc[3][2];
  float cs[3];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) {
    cs[mt] = 0.0f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 16; ++s) acc[mt][kt][s] = 0.0f;
  }
  for (int64_t r = r_begin + wave * 32; r < r_end; r += 128) {
    float av[3][16], bv[2][16];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
      const int m = mt * 32 + i;
      const bool ok = mt < MT && m < jb.M;
      load16(jb.A + (ok ? (r >> 6) * tile + m * 64 + (r & 63) + 16 * hh : 0), ok, av[mt]);
#pragma unroll
      for (int s = 0; s < 16; ++s) cs[mt] += av[mt][s];
    }
    if (KT > 0) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const int kk = kt * 32 + i;
        const bool ok = kt < KT && kk < jb.K;
        load16(jb.B + (ok ? (r >> 6) * tile + kk * 64 + (r & 63) + 16 * hh : 0), ok, bv[kt]);
      }
#pragma unroll
      for (int s = 0; s < 16; ++s)
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
            if (mt < MT && kt < KT) acc[mt][kt] = mfma32(av[mt][s], bv[kt][s], acc[mt][kt]);
    }
  }
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) cs[mt] += __shfl_xor(cs[mt], 32);
  // combine the 4 waves in LDS (waves add in turn), then one partial per block
  __shared__ float red[3 * 2 * 1024 + 3 * 32];
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            const int idx = (mt * 2 + kt) * 1024 + kperm(s, hh) * 32 + i;
            red[idx] = (w == 0 ? 0.0f : red[idx]) + acc[mt][kt][s];
          }
        if (hh == 0) red[6 * 1024 + mt * 32 + i] = (w == 0 ? 0.0f : red[6 * 1024 + mt * 32 + i]) + cs[mt];
      }
    }
    __syncthreads();
  }
  float* out = a.partial + jb.part + (int64_t)b * (jb.M * jb.K + jb.M);
  const int nW = jb.M * jb.K;
  for (int e = threadIdx.x; e < nW + jb.M; e += 256) {
    int idx;
    if (e < nW) {
      const int m = e / jb.K, kk = e % jb.K;
      idx = ((m >> 5) * 2 + (kk >> 5)) * 1024 + (m & 31) * 32 + (kk & 31);
    } else {
      idx = 6 * 1024 + (e - nW);
    }
    out[e] = red[idx];
  }
}

// Sum the per-block partials: block = 64 outputs x 4 waves, each wave a quarter of the partials.
static __global__ __launch_bounds__(256) void mappo_wgrad_sum_kernel(WgArgsDev a) {
  __shared__ float sh[4][64];
  const WgJobDev& jb = a.job[blockIdx.y];
  const int per = jb.M * jb.K + jb.M;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int e = blockIdx.x * 64 + lane;
  float s = 0.0f;
  if (e < per) {
    const float* p = a.partial + jb.part + e;
    for (int b = wave; b < jb.nblk; b += 4) s += p[(int64_t)b * per];
  }
  sh[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && e < per) {
    s = sh[0][lane] + sh[1][lane] + sh[2][lane] + sh[3][lane];
    if (e < jb.M * jb.K) {
      if (jb.dW) jb.dW[(e / jb.K) * jb.ldw + e % jb.K] = s;
    } else if (jb.db) {
      jb.db[e - jb.M * jb.K] = s;
    }
  }
}

// Weight gradients of one trunk net (MGeo<D,H,O> flat layout) from its GF<D,H,O> operands.
template <int D, int H>
struct TrunkWgrad {
  // job list of one net's weight gradients (outputs in the net's flat gradient vector)
  template <int O>
  static int jobs(const float* gsoa, int64_t Rs, float* grad, WgJobDev* jv) {
    using G = MGeo<D, H, O>;
    using F = GF<D, H, O>;
    int nj = 0;
    auto add = [&](int fa, int M, int fb, int K, int wofs, int ld, int bofs) {
      for (int m0 = 0; m0 < M; m0 += 96)
        for (int k0 = 0; k0 < (K > 0 ? K : 1); k0 += 64) {
          WgJobDev& j = jv[nj++];
          j.M = M - m0 < 96 ? M - m0 : 96;
          j.K = K > 0 ? (K - k0 < 64 ? K - k0 : 64) : 0;
          j.A = gsoa + (int64_t)(fa + m0) * 64;
          j.B = K > 0 ? gsoa + (int64_t)(fb + k0) * 64 : nullptr;
          j.dW = K > 0 ? grad + wofs + m0 * ld + k0 : nullptr;
          j.ldw = ld;
          j.db = (k0 == 0 && bofs >= 0) ? grad + bofs + m0 : nullptr;
        }
    };
    add(F::DOUT, O, F::Y, H, G::Wo, H, G::bo);
    add(F::DGI, 3 * H, F::X2, H, G::Wih, H, G::bih);
    add(F::DGH, 3 * H, F::HIN, H, G::Whh, H, G::bhh);
    add(F::DPRE2, H, F::F1, H, G::W2, H, G::b2);
    add(F::DPRE1, H, F::F0, D, G::W1, G::Dp, G::b1);
    add(F::DY, H, 0, 0, 0, 0, G::lnr_b);
    add(F::PY, H, 0, 0, 0, 0, G::lnr_w);
    add(F::DX2, H, 0, 0, 0, 0, G::ln2_b);
    add(F::P2, H, 0, 0, 0, 0, G::ln2_w);
    add(F::DX1, H, 0, 0, 0, 0, G::ln1_b);
    add(F::P1, H, 0, 0, 0, 0, G::ln1_w);
    add(F::DF0, D, 0, 0, 0, 0, G::ln0_b);
    add(F::P0, D, 0, 0, 0, 0, G::ln0_w);
    return nj;
  }
  static int64_t rows_per_block(int64_t Rs) {
    int64_t rpb = (Rs + 399) / 400;
    rpb = (rpb + 127) / 128 * 128;
    return rpb < 128 ? 128 : rpb;
  }
  template <int O>
  static int wgrad(const float* gsoa, int64_t Rs, float* grad, float* partial, hipStream_t s) {
    WgArgsDev w = {};
    w.Rs = Rs;
    w.rows_per_block = rows_per_block(Rs);
    w.partial = partial;
    w.njobs = jobs<O>(gsoa, Rs, grad, w.job);
    w.nf = GF<D, H, O>::NG;
    const int nblk = (int)((Rs + w.rows_per_block - 1) / w.rows_per_block);
    int64_t part = 0;
    int blk = 0, maxper = 0;
    for (int q = 0; q < w.njobs; ++q) {
      w.job[q].blk0 = blk;
      w.job[q].nblk = nblk;
      w.job[q].part = part;
      const int per = w.job[q].M * w.job[q].K + w.job[q].M;
      part += (int64_t)nblk * per;
      blk += nblk;
      maxper = per > maxper ? per : maxper;
    }
    hipLaunchKernelGGL(mappo_wgrad_kernel, dim3(blk), dim3(256), 0, s, w);
    MM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(mappo_wgrad_sum_kernel, dim3((maxper + 63) / 64, w.njobs), dim3(256), 0, s, w);
    MM_HIP_CHECK(hipGetLastError());
    return MM_OK;
  }
};

}  // namespace mm
