// cohab_probe.hip -- do the data-parallel step's GEMMs still get every CU while RCCL runs beside them?
//
// RCCL's collective kernel on gfx950 (ncclDevKernel_Generic_*, metadata of the librccl.so code object
// in this image) takes 37,664 B of LDS and 248-256 VGPRs per lane, launch bounds 512 threads, and each
// channel's workgroup stays resident on its CU for the whole collective.  A GEMM workgroup co-resides
// on such a CU only if LDS (160 KB per CU) and the VGPR file (512 per SIMD lane) hold both.  This probe
// parks an "occupier" with RCCL's footprint (37,664 B LDS, 256 VGPRs, 256 or 512 threads) on `nocc`
// CUs for the duration of a run of data-parallel gradient GEMMs (tnet_affine_grad, 1024 x 2048 ->
// 2048 x 2048) and times them against the same run alone, per tile configuration.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/cohab_probe tools/cohab_probe.hip -Innet-asr_amd/../include \
//         -Lnnet-asr_amd/lib -ltnet_amd -Wl,-rpath,'$ORIGIN/../nnet-asr_amd/lib'
//   ./tools/cohab_probe [nocc]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "tnet_kernels.h"
#include "tnet_train.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)
#define CT(x)                                                    \
  do {                                                           \
    int r_ = (x);                                                \
    if (r_ != 0) {                                               \
      fprintf(stderr, "%s:%d tnet status %d\n", __FILE__, __LINE__, r_); \
      exit(1);                                                   \
    }                                                            \
  } while (0)

// RCCL's footprint: 37,664 B of LDS, 256 VGPRs (the clobber of v255), NT threads; every wave leaves
// after `ticks` of the 100 MHz real-time counter (an exit every wave reaches)
template <int NT, int LDSB = 37664, int NV = 256>
__global__ __launch_bounds__(NT) void occupier(float* out, long ticks) {
  __shared__ float lds[LDSB / 4];
  const long t0 = (long)__builtin_amdgcn_s_memrealtime();
  float acc = 0.f;
  for (int i = threadIdx.x; i < LDSB / 4; i += NT) lds[i] = (float)i;
  __syncthreads();
  while ((long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    acc += lds[(threadIdx.x * 7 + (int)acc) & (LDSB / 4 - 1 < 1023 ? 255 : 1023)];
    __builtin_amdgcn_s_sleep(8);
  }
  if constexpr (NV == 280) asm volatile("" ::: "v255", "a23");  // torch's librccl: 261-280 (VGPR + AGPR)
  if constexpr (NV == 256) asm volatile("" ::: "v255");
  if constexpr (NV == 192) asm volatile("" ::: "v191");
  if constexpr (NV == 128) asm volatile("" ::: "v127");
  if constexpr (NV == 248) asm volatile("" ::: "v247");
  if constexpr (NV == 224) asm volatile("" ::: "v223");
  if (acc == -1.f) out[threadIdx.x] = acc;
}

// ./tools/cohab_probe steal [nocc]: the step's backward-pass GEMM shapes (gradient 128x128, backward
// 64x128 + diff-sigmoid + slab sums, forward 64x128 + bias + sigmoid) alone and beside nocc RCCL-footprint
// occupiers (512 threads, 37.6 KB LDS, 256 VGPRs), on the plain tile grid and as stream-K over CUs - R
// workgroups (tnet_gemm_config "+rsv<R>", gemm16_sk_kernel)
static int steal_probe(int nocc) {
  const int M = 1024, K = 2048, N = 2048, reps = 20;
  CT(tnet_select_gpu(0));
  std::vector<float> h((size_t)K * N);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
  float *X, *E, *G, *W, *Y, *bias, *P, *gb, *junk;
  CK(hipMalloc(&X, (size_t)M * K * 4));
  CK(hipMalloc(&E, (size_t)M * N * 4));
  CK(hipMalloc(&G, (size_t)K * N * 4));
  CK(hipMalloc(&W, (size_t)K * N * 4));
  CK(hipMalloc(&Y, (size_t)M * K * 4));
  CK(hipMalloc(&bias, N * 4));
  CK(hipMalloc(&P, 64 * N * 4));
  CK(hipMalloc(&gb, N * 4));
  CK(hipMalloc(&junk, 4096));
  CK(hipMemcpy(X, h.data(), (size_t)M * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(E, h.data(), (size_t)M * N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(W, h.data(), (size_t)K * N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(Y, h.data(), (size_t)M * K * 4, hipMemcpyHostToDevice));
  CK(hipMemset(bias, 0, N * 4));
  CK(hipMemset(P, 0, 64 * N * 4));
  const TnetMatrixDim dX = {M, K, K}, dE = {M, N, N}, dG = {K, N, N}, dW = {K, N, N}, dY = {M, K, K};
  hipStream_t s1 = (hipStream_t)tnet_stream(), s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[] = {"grad+bias 1024x2048 -> 2048x2048 (128x128)", "bwd+dsig+slabs 1024x2048 x 2048x2048^T (64x128)",
                         "fwd+bias+sigmoid 1024x2048 x 2048x2048 (64x128)"};
  auto run = [&](int which) {
    for (int i = 0; i < reps; ++i) {
      if (which == 0) CT(tnet_affine_grad_bias(X, dX, E, dE, G, dG, P, N, gb, s1));
      else if (which == 1) CT(tnet_affine_bwd_colsum(E, dE, W, dW, Y, K, X, dX, P, K, s1));
      else CT(tnet_affine_fwd(X, dX, W, dW, bias, Y, dY, 1, s1));
    }
  };
  auto timed = [&](int which) {
    float ms = 0.f;
    CK(hipEventRecord(a, s1));
    run(which);
    CK(hipEventRecord(b, s1));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
  };
  // the two RCCL builds this image carries (profiles/r04_rccl_footprint.json): /opt/rocm's
  // ncclDevKernel_Generic (512 threads, 37,664 B LDS, 248-256 VGPRs) and torch's bundled rcclGenericKernel,
  // the one a Python process maps (256 threads, 19,744 B LDS, 261-280 VGPRs)
  const char* modes[] = {"auto+rsv0", "auto+rsv8", "auto+rsv16"};
  for (int fp = 0; fp < 2; ++fp)
    for (int which = 0; which < 3; ++which)
      for (const char* mode : modes) {
        CT(tnet_gemm_config(mode));
        run(which);
        CK(hipStreamSynchronize(s1));
        const float alone = timed(which);
        const long ticks = (long)(alone * 4.0f * 1e5f) + 20000;
        if (fp == 0) occupier<512><<<nocc, 512, 0, s2>>>(junk, ticks);
        else occupier<256, 19744, 280><<<nocc, 256, 0, s2>>>(junk, ticks);
        CK(hipGetLastError());
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        const float occ = timed(which);
        CK(hipStreamSynchronize(s2));
        printf("%-50s %-9s: alone %.1f us; beside %d %s occupiers: %.1f us (x%.2f)\n", names[which], mode,
               1e3f * alone / reps, nocc,
               fp == 0 ? "/opt/rocm RCCL-footprint (512 thr, 37.6 KB, 256 VGPR)"
                       : "torch RCCL-footprint (256 thr, 19.7 KB, 280 VGPR)",
               1e3f * occ / reps, occ / alone);
        fflush(stdout);
      }
  CT(tnet_gemm_config("auto+rsv0"));
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "steal")) return steal_probe(argc > 2 ? atoi(argv[2]) : 8);
  const int nocc = argc > 1 ? atoi(argv[1]) : 32;
  const int M = 1024, K = 2048, N = 2048, reps = 20;
  CT(tnet_select_gpu(0));
  std::vector<float> h((size_t)M * K);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
  float *X, *E, *G, *junk;
  CK(hipMalloc(&X, (size_t)M * K * 4));
  CK(hipMalloc(&E, (size_t)M * N * 4));
  CK(hipMalloc(&G, (size_t)K * N * 4));
  CK(hipMalloc(&junk, 4096));
  CK(hipMemcpy(X, h.data(), (size_t)M * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(E, h.data(), (size_t)M * N * 4, hipMemcpyHostToDevice));
  const TnetMatrixDim dX = {M, K, K}, dE = {M, N, N}, dG = {K, N, N};
  hipStream_t s1 = (hipStream_t)tnet_stream(), s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* cfgs[] = {"auto", "m128x128k32s3", "m128x128k64s2", "m64x128k64s2"};
  for (const char* cfg : cfgs) {
    CT(tnet_gemm_config(cfg));
    for (int i = 0; i < 5; ++i) CT(tnet_affine_grad(X, dX, E, dE, G, dG, s1));
    CK(hipStreamSynchronize(s1));
    float ms_alone = 0.f, ms_occ[2] = {0.f, 0.f};
    CK(hipEventRecord(a, s1));
    for (int i = 0; i < reps; ++i) CT(tnet_affine_grad(X, dX, E, dE, G, dG, s1));
    CK(hipEventRecord(b, s1));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms_alone, a, b));
    for (int v = 0; v < 2; ++v) {
      // occupier for the run's expected length x 3 (ticks of 10 ns), launched first on its own stream
      const long ticks = (long)(ms_alone * 3.0f * 1e5f) + 20000;
      if (v == 0) occupier<256><<<nocc, 256, 0, s2>>>(junk, ticks);
      else occupier<512><<<nocc, 512, 0, s2>>>(junk, ticks);
      CK(hipGetLastError());
      std::this_thread::sleep_for(std::chrono::microseconds(200));
      CK(hipEventRecord(a, s1));
      for (int i = 0; i < reps; ++i) CT(tnet_affine_grad(X, dX, E, dE, G, dG, s1));
      CK(hipEventRecord(b, s1));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms_occ[v], a, b));
      CK(hipStreamSynchronize(s2));
    }
    printf("grad 1024x2048 -> 2048x2048, cfg %-14s: alone %.1f us; beside %d occupier WGs (37.6 KB LDS, 256 VGPR): "
           "256 threads %.1f us (x%.2f), 512 threads %.1f us (x%.2f)\n",
           cfg, 1e3f * ms_alone / reps, nocc, 1e3f * ms_occ[0] / reps, ms_occ[0] / ms_alone, 1e3f * ms_occ[1] / reps,
           ms_occ[1] / ms_alone);
    fflush(stdout);
  }
  // which resource keeps the GEMM's workgroup off an occupied CU: occupiers with less LDS / fewer VGPRs
  CT(tnet_gemm_config("m128x128k32s3"));
  float ms0 = 0.f;
  CK(hipEventRecord(a, s1));
  for (int i = 0; i < reps; ++i) CT(tnet_affine_grad(X, dX, E, dE, G, dG, s1));
  CK(hipEventRecord(b, s1));
  CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms0, a, b));
  const long ticks = (long)(ms0 * 3.0f * 1e5f) + 20000;
  for (int v = 0; v < 4; ++v) {
    const char* what[] = {"4 KB LDS, few VGPRs", "4 KB LDS, 256 VGPRs", "37.6 KB LDS, few VGPRs", "64 threads, 4 KB, few"};
    if (v == 0) occupier<256, 4096, 0><<<nocc, 256, 0, s2>>>(junk, ticks);
    if (v == 1) occupier<256, 4096, 256><<<nocc, 256, 0, s2>>>(junk, ticks);
    if (v == 2) occupier<256, 37664, 0><<<nocc, 256, 0, s2>>>(junk, ticks);
    if (v == 3) occupier<64, 4096, 0><<<nocc, 64, 0, s2>>>(junk, ticks);
    CK(hipGetLastError());
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    float ms = 0.f;
    CK(hipEventRecord(a, s1));
    for (int i = 0; i < reps; ++i) CT(tnet_affine_grad(X, dX, E, dE, G, dG, s1));
    CK(hipEventRecord(b, s1));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipStreamSynchronize(s2));
    printf("  m128x128k32s3 (96 KB LDS, 210 VGPRs) beside %d occupiers of %s: %.1f us (x%.2f)\n", nocc, what[v],
           1e3f * ms / reps, ms / ms0);
  }
  // the VGPR budget a SIMD shares: occupiers of 128 / 192 VGPRs beside the 210-VGPR gradient GEMM,
  // and the 256-VGPR occupier beside the hidden forward GEMM (64x128 + bias + sigmoid, 132 VGPRs)
  for (int v = 0; v < 2; ++v) {
    if (v == 0) occupier<256, 4096, 128><<<nocc, 256, 0, s2>>>(junk, ticks);
    else occupier<256, 4096, 192><<<nocc, 256, 0, s2>>>(junk, ticks);
    CK(hipGetLastError());
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    float ms = 0.f;
    CK(hipEventRecord(a, s1));
    for (int i = 0; i < reps; ++i) CT(tnet_affine_grad(X, dX, E, dE, G, dG, s1));
    CK(hipEventRecord(b, s1));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipStreamSynchronize(s2));
    printf("  m128x128k32s3 (210 VGPRs) beside %d occupiers of 4 KB LDS, %d VGPRs: %.1f us (x%.2f)\n", nocc,
           v == 0 ? 128 : 192, 1e3f * ms / reps, ms / ms0);
  }
  CT(tnet_gemm_config("auto"));
  float* bias;
  float* Y;
  CK(hipMalloc(&bias, N * 4));
  CK(hipMemset(bias, 0, N * 4));
  CK(hipMalloc(&Y, (size_t)M * N * 4));
  const TnetMatrixDim dW = {K, N, N}, dY = {M, N, N};
  for (int v = 0; v < 5; ++v) {
    if (v == 1) occupier<256, 37664, 256><<<nocc, 256, 0, s2>>>(junk, ticks);
    if (v == 2) occupier<512, 37664, 256><<<nocc, 512, 0, s2>>>(junk, ticks);
    if (v == 3) occupier<256, 37664, 248><<<nocc, 256, 0, s2>>>(junk, ticks);
    if (v == 4) occupier<256, 37664, 224><<<nocc, 256, 0, s2>>>(junk, ticks);
    CK(hipGetLastError());
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    float ms = 0.f;
    CK(hipEventRecord(a, s1));
    for (int i = 0; i < reps; ++i) CT(tnet_affine_fwd(X, dX, G, dW, bias, Y, dY, 1, s1));
    CK(hipEventRecord(b, s1));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipStreamSynchronize(s2));
    if (v == 0) ms0 = ms;
    printf("  fwd 1024x2048 x 2048x2048 + bias + sigmoid (64x128, 96 KB, 132 VGPRs)%s: %.1f us (x%.2f)\n",
           v == 0 ? " alone" : v == 1 ? " beside RCCL-footprint occupiers (256 thr)" : v == 2 ? " beside RCCL-footprint occupiers (512 thr)"
           : v == 3 ? " beside 248-VGPR occupiers (256 thr)" : " beside 224-VGPR occupiers (256 thr)",
           1e3f * ms / reps, ms / ms0);
  }
  return 0;
}
