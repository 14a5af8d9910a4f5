// mfma_peak.hip -- diagnostic: sustained v_mfma_f32_32x32x2_f32 rate with operands in registers
// (no memory traffic), 4 independent accumulators per wave, one or two waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float seed) {
  f32x16 acc[NACC];
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
  float x = seed + threadIdx.x * 1e-3f, y = seed * 0.5f - threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[a], 0, 0, 0);
  }
  float s = 0.f;
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 16; ++r) s += acc[a][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void mfma16_loop(float* out, int iters, float seed) {
  f32x4 acc[NACC];
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 4; ++r) acc[a][r] = 0.f;
  float x = seed + threadIdx.x * 1e-3f, y = seed * 0.5f - threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, acc[a], 0, 0, 0);
  }
  float s = 0.f;
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 4; ++r) s += acc[a][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 20000;
  for (int nacc = 1; nacc <= 4; nacc *= 2)
  for (int blocks_per_cu = 1; blocks_per_cu <= 2; ++blocks_per_cu) {
    int grid = 256 * blocks_per_cu;
    auto run = [&](int it) {
      if (nacc == 1) mfma_loop<1><<<grid, 256>>>(out, it * 4, 1.f);
      if (nacc == 2) mfma_loop<2><<<grid, 256>>>(out, it * 2, 1.f);
      if (nacc == 4) mfma_loop<4><<<grid, 256>>>(out, it, 1.f);
    };
    run(100);
    hipDeviceSynchronize();
    hipEventRecord(a);
    run(iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double flops = (double)grid * 4 /*waves*/ * iters * 4 /*mfma per iter-equiv*/ * 32 * 32 * 2 * 2;
    printf("mfma_f32_32x32x2 %d acc, %d wave/SIMD: %.3f ms  %.1f TFLOP/s\n", nacc, blocks_per_cu, ms, flops / ms / 1e9);
  }
  // 16x16x4 f32: 1024 MACs per instruction (half the work of 32x32x2)
  for (int nacc = 1; nacc <= 8; nacc *= 2)
  for (int blocks_per_cu = 1; blocks_per_cu <= 2; ++blocks_per_cu) {
    int grid = 256 * blocks_per_cu;
    auto run = [&](int it) {
      if (nacc == 1) mfma16_loop<1><<<grid, 256>>>(out, it * 8, 1.f);
      if (nacc == 2) mfma16_loop<2><<<grid, 256>>>(out, it * 4, 1.f);
      if (nacc == 4) mfma16_loop<4><<<grid, 256>>>(out, it * 2, 1.f);
      if (nacc == 8) mfma16_loop<8><<<grid, 256>>>(out, it, 1.f);
    };
    run(100);
    hipDeviceSynchronize();
    hipEventRecord(a);
    run(iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double flops = (double)grid * 4 * iters * 8 * 16 * 16 * 4 * 2;
    printf("mfma_f32_16x16x4 %d acc, %d wave/SIMD: %.3f ms  %.1f TFLOP/s\n", nacc, blocks_per_cu, ms, flops / ms / 1e9);
  }
  return 0;
}
