// Floor of the agent forward's MFMA work on this chip: 256 blocks x 512 threads (two waves per
// SIMD), each wave issuing 512 v_mfma_f32_32x32x2_f32 in 32-long dependent chains (the forward's
// shape), no memory traffic. Build: hipcc -O3 --offload-arch=gfx950 tools/mb_mfma.hip -o /tmp/mb_mfma
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(512, 1) void chain(float* out, float a0, float b0, int nchain) {
  f32x16 acc = {0};
  float a = a0 + threadIdx.x, b = b0;
  for (int c = 0; c < nchain; ++c) {
#pragma unroll
    for (int s = 0; s < 32; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    a += 1.0f;
  }
  float r = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) r += acc[i];
  out[blockIdx.x * 512 + threadIdx.x] = r;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 512 * 4);
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(chain, dim3(256), dim3(512), 0, 0, out, 1.0f, 2.0f, 16);
    hipDeviceSynchronize();
    hipEventRecord(s, 0);
    const int it = 200;
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL(chain, dim3(256), dim3(512), 0, 0, out, 1.0f, 2.0f, 16);
    hipEventRecord(e, 0);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    const double us = ms * 1e3 / it;
    const double flop = 256.0 * 8 * 512 * 4096;  // blocks x waves x mfma x flop/mfma
    printf("{\"mfma_floor_us\": %.2f, \"tflops\": %.1f, \"implied_ghz\": %.3f}\n", us, flop / us * 1e-6,
           (8.0 * 512 * 64 / 4) / (us * 1e3));
  }
  return 0;
}
