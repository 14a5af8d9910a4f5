// issue_cost.hip -- diagnostic: what one 1-KiB global->LDS piece costs a SIMD that is otherwise busy
// issuing v_mfma_f32_16x16x4_f32 (the GEMM main loop's question).
// One workgroup per CU, 4 waves (one per SIMD); every iteration issues 8 independent MFMAs (256 cycles
// of MFMA issue) plus the variant's memory instructions, from an L2-resident source:
//   0: nothing                          1: one global_load_lds_dwordx4 (LDS-DMA piece)
//   2: one global_load_dwordx4 into registers + one ds_write_b128 of the previous iteration's registers
//   3: the global_load_dwordx4 alone    4: the ds_write_b128 alone (of loop-carried registers)
// Prints ns per iteration; the excess over variant 0 is the SIMD cost of that variant's instructions.
#include <hip/hip_runtime.h>

#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int V, int PER>
__global__ __launch_bounds__(256) void issue_loop(const float* __restrict__ src, float* out, int iters) {
  __shared__ __attribute__((aligned(16))) float lds[4 * 2048];  // per wave: eight 1-KiB pieces
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  f32x4 acc[8];
  for (int a = 0; a < 8; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
  float x = lane * 1e-3f, y = 0.5f - lane * 1e-3f;
  // a 256-KiB window per workgroup, read in 1-KiB wave pieces (L2-resident after the first pass)
  const char* base = (const char*)src + (size_t)(blockIdx.x % 64) * 262144;
  // register ring for variants 2 / 3: piece p loads into rr[p % 8] and consumes rr[(p + 1) % 8], the
  // registers loaded 7 pieces (= 7 / PER iterations) earlier, so the wait rarely stalls on latency
  f32x4 rr[8];
  for (int k = 0; k < 8; ++k) rr[k] = f32x4{1.f, 2.f, 3.f, (float)k};
  f32x4 sink = {0.f, 0.f, 0.f, 0.f};
  float* wl = lds + wid * 2048;
  // LDS byte offset of this lane's 16 B in the wave's first piece (lds is the kernel's only LDS object)
  const unsigned lds_off = (unsigned)(wid * 2048 + lane * 4) * 4u;
  constexpr int U = 8 / PER;  // iterations per outer step (8 pieces)
  for (int i = 0; i < iters; i += U) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
#pragma unroll
      for (int a = 0; a < 8; ++a) acc[a] = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, acc[a], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int pc = j * PER + q;  // piece index in the outer step: 0..7
        const unsigned off = (unsigned)(((i + j) * 8 + q * 4 + wid) & 255) * 1024u + lane * 16u;
        if constexpr (V == 1) {
          __builtin_amdgcn_global_load_lds((const void*)(base + off), (void*)(wl + pc * 256), 16, 0, 0);
        } else if constexpr (V == 2) {
          // the store in asm: the compiler may neither drop it (dead-store) nor hoist it out of the loop
          rr[pc] = *reinterpret_cast<const f32x4*>(base + off);
          asm volatile("ds_write_b128 %0, %1" ::"v"(lds_off + ((pc + 1) & 7) * 1024u), "v"(rr[(pc + 1) & 7])
                       : "memory");
        } else if constexpr (V == 3) {
          rr[pc] = *reinterpret_cast<const f32x4*>(base + off);
          asm volatile("" ::"v"(rr[(pc + 1) & 7]));
        } else if constexpr (V == 4) {
          asm volatile("ds_write_b128 %0, %1" ::"v"(lds_off + pc * 1024u), "v"(sink) : "memory");
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float s = wl[lane] + sink[0];
  for (int k = 0; k < 8; ++k) s += rr[k][1];
  for (int a = 0; a < 8; ++a) s += acc[a][0] + acc[a][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int V, int PER>
static void run(const float* src, float* out, int iters, const char* name) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  issue_loop<V, PER><<<256, 256>>>(src, out, 200);
  hipDeviceSynchronize();
  hipEventRecord(a);
  issue_loop<V, PER><<<256, 256>>>(src, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("%-44s %d per 8 MFMA: %.2f ns/iter\n", name, PER, 1e6 * ms / iters);
}

int main() {
  float *src, *out;
  hipMalloc(&src, 64 * 262144 + 4096);
  hipMemset(src, 0, 64 * 262144 + 4096);
  hipMalloc(&out, 256 * 256 * 4);
  const int iters = 200000;
  run<0, 1>(src, out, iters, "8 MFMA only");
  run<0, 8>(src, out, iters, "8 MFMA only");
  run<1, 1>(src, out, iters, "global_load_lds_dwordx4");
  run<1, 2>(src, out, iters, "global_load_lds_dwordx4");
  run<1, 4>(src, out, iters, "global_load_lds_dwordx4");
  run<2, 1>(src, out, iters, "global_load_dwordx4 + ds_write_b128");
  run<2, 2>(src, out, iters, "global_load_dwordx4 + ds_write_b128");
  run<2, 4>(src, out, iters, "global_load_dwordx4 + ds_write_b128");
  run<3, 2>(src, out, iters, "global_load_dwordx4 alone");
  run<4, 2>(src, out, iters, "ds_write_b128 alone");
  return 0;
}
