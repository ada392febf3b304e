// Shared helpers for the minimarl HIP/CDNA4 kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MM_OK 0
#define MM_EINVAL (-22)
#define MM_EHIP (-5)
#define MM_ENOMEM (-12)

namespace mm {

void set_error(const char* fmt, ...);

// A wave (64 lanes) computes a 32-env x (feature rows) tile with the exact-f32
// MFMA v_mfma_f32_32x32x2_f32. Fragment maps (gfx950):
//   A[i = lane&31][k = lane>>5], B[k = lane>>5][j = lane&31],
//   D reg r of lane (j, h=lane>>5): row (r&3) + 8*(r>>2) + 4*h, col j.
// Chaining layers through registers: k-step s of a 32-deep k-block uses, in
// lane half h, the input feature kperm(s, h) = (s&3) + 8*(s>>2) + 4*h, i.e.
// exactly D register s of the producing layer. Weights are pre-packed so that
// lane (i, h) of k-step s reads W[32*rb + i][32*kb + kperm(s, h)].
typedef float f32x16 __attribute__((ext_vector_type(16)));

__host__ __device__ __forceinline__ int kperm(int s, int h) { return (s & 3) + 8 * (s >> 2) + 4 * h; }

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Hardware transcendental forms (v_exp_f32 + v_rcp_f32, ~1 ulp each): 4-5 VALU ops instead of the
// ~25 of libm expf + IEEE division. Relative error <= ~1e-6 for |x| < 30, far inside the
// parity tolerances (rtol 1e-5); saturate correctly (exp2 -> inf / 0, rcp(inf) = 0).
__device__ __forceinline__ float sigmoidf_(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
__device__ __forceinline__ float tanhf_(float x) {
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * 2.8853900817779268f));
}

// splitmix64-based counter RNG (stateless; one draw per (seed, counter, a, b)).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rng_draw(uint64_t seed, uint64_t counter, uint64_t a, uint64_t b) {
  return mix64(seed ^ mix64(counter * 0xD1B54A32D192ED03ull ^ mix64(a * 0x8CB92BA72F3D8DD7ull + b)));
}
// rng_draw split at its (a, b) part: rng_draw(seed, counter, a, b) == rng_draw_inner(seed, counter, rng_inner(a, b)),
// so a lane that draws with the same (a, b) every step computes rng_inner once
__device__ __forceinline__ uint64_t rng_inner(uint64_t a, uint64_t b) { return mix64(a * 0x8CB92BA72F3D8DD7ull + b); }
__device__ __forceinline__ uint64_t rng_draw_inner(uint64_t seed, uint64_t counter, uint64_t inner) {
  return mix64(seed ^ mix64(counter * 0xD1B54A32D192ED03ull ^ inner));
}
// x % m for a wave-uniform 1 <= m <= 65536 without a division: q0 = umulhi(x, floor((2^32 - 1) / m)) is floor(x / m)
// or up to 2 below it, so x - q0 m lies in [0, 3 m) and two conditional subtractions make it exact
__device__ __forceinline__ uint32_t umod_small(uint32_t x, uint32_t m, uint32_t minv) {
  uint32_t r = x - __umulhi(x, minv) * m;
  r = r >= m ? r - m : r;
  return r >= m ? r - m : r;
}
// the rollout priority term |sum_i r_i + (1 - d) gamma sum_i max Q'_i - sum_i Q_i(a_i)| (cal_td_error,
// vdn/_utils.py:44-52) with ONE fixed rounding sequence (no FMA contraction): every kernel that folds a rollout TD
// (two-launch, fused, chunk-persistent, PER insert) produces the same bits
__device__ __forceinline__ float rollout_td(float sr, float sq, float st, float d, float gamma) {
  const float boot = __fmul_rn(__fmul_rn(1.0f - d, gamma), st);
  return fabsf(__fsub_rn(__fadd_rn(sr, boot), sq));
}
__device__ __forceinline__ float rng_uniform(uint64_t r) { return (float)(r >> 40) * (1.0f / 16777216.0f); }
// r % m for 1 <= m <= 65536 in 32-bit arithmetic (exact: r = hi 2^32 + lo, (hi % m)(2^32 % m) + lo % m < 2^32)
__device__ __forceinline__ uint32_t rng_mod_small(uint64_t r, uint32_t m) {
  const uint32_t p32 = (0xFFFFFFFFu % m + 1u) % m;   // 2^32 mod m
  return ((uint32_t)(r >> 32) % m * p32 + (uint32_t)r % m) % m;
}
// the same value with the wave-uniform constants hoisted: minv = 0xFFFFFFFF / m, p32 = 2^32 mod m
__device__ __forceinline__ uint32_t rng_mod_small_u(uint64_t r, uint32_t m, uint32_t minv, uint32_t p32) {
  return umod_small(umod_small((uint32_t)(r >> 32), m, minv) * p32 + umod_small((uint32_t)r, m, minv), m, minv);
}
// max(x, 0) on the bit pattern: one v_max_i32 (negative floats are negative integers; no canonicalising v_max_f32
// pair), equal to fmaxf(x, 0) for every non-NaN x but -0 -> +0
#ifndef MM_RELU_BITS
#define MM_RELU_BITS 1
#endif
__device__ __forceinline__ float relu_bits(float x) {
  return MM_RELU_BITS ? __int_as_float(max(__float_as_int(x), 0)) : fmaxf(x, 0.0f);
}

// Debug timing traces: a static device buffer of 4096 u64 slots, allocated when the named
// environment variable is set (kernels record clock64() into it); mm_debug_trace copies it out.
uint64_t* debug_trace_buffer(const char* env_name);

// ---- LDS-DMA (global_load_lds_dword): loads that write LDS directly, no VGPR destination. The LDS
// address of lane L is (wave-uniform base) + 4 L; the global address is per lane, so a rolled loop of
// these is a compact gather (no unrolled register staging: the code of a one-pass prologue costs
// instruction-cache misses) whose loads are all in flight at once. Completion: vmcnt, so a
// __syncthreads() (whose fence waits vmcnt(0) while an LDS-DMA is pending) before the data is read.
typedef __attribute__((address_space(3))) void lds_void_t;
__device__ __forceinline__ void glds_dword(const void* g, float* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)lds_base, 4, 0, 0);
}
// dst[i] = *addr(i) for i < n (dst contiguous in LDS)
template <typename A>
__device__ __forceinline__ void glds_gather(float* dst, int n, A addr) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  for (int c0 = (int)(threadIdx.x >> 6) * 64; c0 < n; c0 += nw * 64)
    if (c0 + lane < n) glds_dword(addr(c0 + lane), dst + c0);
}
// dst[r * ld + j] = *addr(r, j) for r < rows, j < rowlen (a padded LDS image: one wave-instruction
// per 64-word piece of a row, so no instruction's words cross a row)
template <typename A>
__device__ __forceinline__ void glds_rows(float* dst, int rows, int rowlen, int ld, A addr) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int pr = (rowlen + 63) >> 6;   // pieces per row
  for (int q = (int)(threadIdx.x >> 6); q < rows * pr; q += nw) {
    const int r = q / pr, c0 = (q - r * pr) * 64;
    if (c0 + lane < rowlen) glds_dword(addr(r, c0 + lane), dst + r * ld + c0);
  }
}

// 16-byte LDS-DMA: LDS[base + 16 L .. +15] = 16 bytes at g (16-byte aligned on both sides)
__device__ __forceinline__ void glds_dwordx4(const void* g, float* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)lds_base, 16, 0, 0);
}
// dst[r * ld + j] = src(r)[j] for r < rows, j < rowlen: contiguous source rows, 16-byte pieces (rowlen,
// ld multiples of 4 floats; src(r) and dst 16-byte aligned); one wave-instruction per 256-float piece
template <typename S>
__device__ __forceinline__ void glds_rows16(float* dst, int rows, int rowlen, int ld, S src) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int pr = (rowlen + 255) >> 8;   // pieces per row
  for (int q = (int)(threadIdx.x >> 6); q < rows * pr; q += nw) {
    const int r = q / pr, c0 = (q - r * pr) * 256;
    if (c0 + 4 * lane < rowlen) glds_dwordx4(src(r) + c0 + 4 * lane, dst + r * ld + c0);
  }
}

// dst[4 i .. 4 i + 3] = 16 bytes at addr(i) for i < n4 (dst contiguous and 16-byte aligned; each
// source 16-byte aligned): 64 float4 per wave-instruction, the source address per lane
template <typename A>
__device__ __forceinline__ void glds16_gather(float* dst, int n4, A addr) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  for (int c0 = (int)(threadIdx.x >> 6) * 64; c0 < n4; c0 += nw * 64)
    if (c0 + lane < n4) glds_dwordx4(addr(c0 + lane), dst + 4 * c0);
}

// Workgroup barrier that orders LDS only: waits for this wave's outstanding LDS operations, then
// s_barrier. Unlike __syncthreads() it does not wait for outstanding global stores, so a sequence
// kernel whose waves communicate through LDS does not stall every step on its own result writes.
// Only for kernels that never read, within the launch, global data written by another wave.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// acc = sum_k w[k * ws] * x[k] in sequential k order (fma chain), fully unrolled for the common widths
// so every load is in flight before the chain starts; same result as the plain loop.
template <int K>
__device__ __forceinline__ float dot_seq(const float* w, const float* x, float acc) {
#pragma unroll
  for (int k = 0; k < K; ++k) acc += w[k] * x[k];
  return acc;
}
__device__ __forceinline__ float dot_seq_n(const float* w, const float* x, int K, float acc) {
  if (K == 64) return dot_seq<64>(w, x, acc);
  if (K == 32) return dot_seq<32>(w, x, acc);
  for (int k = 0; k < K; ++k) acc += w[k] * x[k];
  return acc;
}

// Fused TD/store of the PREVIOUS rollout step (td_chunk_kernel's work, rollout.hip) done by the
// env kernels (env.hip, switch.hip) of the next step: its inputs (rew, done, Q(a), max Q') are final once the dual forward
// of that step has run, and the env kernel of step t+1 is the next launch on the stream. Saves one
// launch per in-chunk step. Same arithmetic and agent-order sums as td_chunk_kernel.
struct TdFuse {
  const float* rew;       // [E][N] rewards of the previous step (overwritten by this step later)
  const uint8_t* done;    // [E]
  const float* q_taken;   // [E][N]
  const float* maxq;      // [E][N]
  const int32_t* act;     // [E][N]
  float* chunk_td;        // [E]
  uint8_t* s_act;         // store [rows][C][N]
  float* s_rew;           // store [rows][C][N]
  uint8_t* s_done;        // store [rows][C]
  const int64_t* rows;    // [E] store rows of the previous step
  uint64_t* counter;      // RNG step counter (may be null)
  float gamma;
  int slot, C, on;
};


// Chunk start folded into the env kernels (mm_chunk_begin_rows, rollout.hip): slot 0 of the env's new
// staging row <- slot src_off of its previous row (cur_row before this step), or the reset obs.
struct BeginCopy {
  float* store;           // chunk-store obs base
  int64_t row_stride;     // floats per store row
  int64_t src_off;        // C * N * D: the previous chunk's last next obs
  const float* reset_obs; // [N * D]
  int on;
};

}  // namespace mm

#define MM_HIP_CHECK(expr)                                                     \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      mm::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),     \
                    __FILE__, __LINE__);                                       \
      return MM_EHIP;                                                          \
    }                                                                          \
  } while (0)

#define MM_REQUIRE(cond, ...)        \
  do {                               \
    if (!(cond)) {                   \
      mm::set_error(__VA_ARGS__);    \
      return MM_EINVAL;              \
    }                                \
  } while (0)
