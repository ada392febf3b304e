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
__device__ __forceinline__ float rng_uniform(uint64_t r) { return (float)(r >> 40) * (1.0f / 16777216.0f); }

// Debug timing traces: a static device buffer of 4096 u64 slots, allocated when the named
// environment variable is set (kernels record clock64() into it); mm_debug_trace copies it out.
uint64_t* debug_trace_buffer(const char* env_name);

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
