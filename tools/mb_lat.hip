// Latency microbenchmarks of the sequence-kernel building blocks on one CU (one block):
//   chain   : 32 dependent v_mfma_f32_32x32x2_f32 (one wave)
//   chain16 : 32 dependent v_mfma_f32_16x16x4_f32 (one wave)
//   sync    : __syncthreads (7 waves)
//   ldssync : s_waitcnt lgkmcnt(0) + s_barrier (7 waves)
//   ldrt    : one dependent global load (pointer chase over 64 MiB)
//   st+sync : 96 scattered global stores per lane, then __syncthreads (7 waves)
// Build: hipcc -O3 --offload-arch=gfx950 tools/mb_lat.hip -o /tmp/mb_lat
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ void k_chain(float* out, int R) {
  f32x16 acc = {0};
  float a = threadIdx.x, b = 1.0f;
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int s = 0; s < 32; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    a += 1.0f;
  }
  float x = 0;
  for (int i = 0; i < 16; ++i) x += acc[i];
  out[threadIdx.x] = x;
}
__global__ void k_chain16(float* out, int R) {
  f32x4 acc = {0};
  float a = threadIdx.x, b = 1.0f;
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int s = 0; s < 32; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    a += 1.0f;
  }
  out[threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}
__global__ void k_sync(float* out, int R) {
  __shared__ float sh[512];
  float v = threadIdx.x;
  for (int r = 0; r < R; ++r) {
    sh[threadIdx.x] = v;
    __syncthreads();
    v += sh[(threadIdx.x + 64) % blockDim.x];
    __syncthreads();
  }
  out[threadIdx.x] = v;
}
__global__ void k_ldssync(float* out, int R) {
  __shared__ float sh[512];
  float v = threadIdx.x;
  for (int r = 0; r < R; ++r) {
    sh[threadIdx.x] = v;
    lds_sync();
    v += sh[(threadIdx.x + 64) % blockDim.x];
    lds_sync();
  }
  out[threadIdx.x] = v;
}
__global__ void k_ldrt(const int* next, int* out, int R) {
  int p = threadIdx.x * 4099;
  for (int r = 0; r < R; ++r) p = next[p];
  out[threadIdx.x] = p;
}
__global__ void k_stsync(float* buf, float* out, int R) {
  float v = threadIdx.x;
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int s = 0; s < 96; ++s) buf[((int64_t)(threadIdx.x & 31) * 4096 + s * 64 + (threadIdx.x >> 5)) % (1 << 24)] = v + s;
    __syncthreads();
    v += 1.0f;
  }
  out[threadIdx.x] = v;
}
__global__ void k_stldsync(float* buf, float* out, int R) {
  float v = threadIdx.x;
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int s = 0; s < 96; ++s) buf[((int64_t)(threadIdx.x & 31) * 4096 + s * 64 + (threadIdx.x >> 5)) % (1 << 24)] = v + s;
    lds_sync();
    v += 1.0f;
  }
  out[threadIdx.x] = v;
}

template <typename F>
static double timeit(F f, int R) {
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  f();
  hipDeviceSynchronize();
  hipEventRecord(s, 0);
  f();
  hipEventRecord(e, 0);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  return ms * 1e3 / R;  // us per iteration
}

int main() {
  const int R = 2000;
  float *out, *buf;
  int *next, *iout;
  hipMalloc(&out, 4096 * 4);
  hipMalloc(&buf, (1 << 24) * 4);
  const int n = 1 << 24;
  hipMalloc(&next, (size_t)n * 4);
  int* h = (int*)malloc((size_t)n * 4);
  for (int i = 0; i < n; ++i) h[i] = (int)(((long long)i * 2654435761ll + 977) % n);
  hipMemcpy(next, h, (size_t)n * 4, hipMemcpyHostToDevice);
  hipMalloc(&iout, 4096 * 4);
  printf("{\"chain32x32x2_us\": %.3f, ", timeit([&] { hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, out, R); }, R));
  printf("\"chain16x16x4_us\": %.3f, ", timeit([&] { hipLaunchKernelGGL(k_chain16, dim3(1), dim3(64), 0, 0, out, R); }, R));
  printf("\"syncthreads_pair_us\": %.3f, ", timeit([&] { hipLaunchKernelGGL(k_sync, dim3(1), dim3(448), 0, 0, out, R); }, R));
  printf("\"ldssync_pair_us\": %.3f, ", timeit([&] { hipLaunchKernelGGL(k_ldssync, dim3(1), dim3(448), 0, 0, out, R); }, R));
  printf("\"load_roundtrip_us\": %.3f, ", timeit([&] { hipLaunchKernelGGL(k_ldrt, dim3(1), dim3(64), 0, 0, next, iout, R); }, R));
  printf("\"stores96_syncthreads_us\": %.3f, ", timeit([&] { hipLaunchKernelGGL(k_stsync, dim3(1), dim3(448), 0, 0, buf, out, R); }, R));
  printf("\"stores96_ldssync_us\": %.3f}\n", timeit([&] { hipLaunchKernelGGL(k_stldsync, dim3(1), dim3(448), 0, 0, buf, out, R); }, R));
  return 0;
}
