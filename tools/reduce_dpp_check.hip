// reduce_dpp_check.hip -- the wave reductions of kcommon.h (permlane-swap / DPP butterflies) against the
// ds_bpermute butterflies they replaced, bit for bit, on random data (values with ties and with mixed signs
// and magnitudes), every lane's result.  Prints "reduce_dpp_check ok <n>" or the first mismatch; exit 1 on
// a mismatch.
//   hipcc --offload-arch=gfx950 -O3 -I include -I nnet-asr_amd/csrc/kernels -o tools/reduce_dpp_check \
//         tools/reduce_dpp_check.hip && ./tools/reduce_dpp_check
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <vector>

#include "kcommon.h"

using namespace tnetk;

// out per lane: [sum, sum_shfl, max, max_shfl, argmax.v, argmax_shfl.v, argmax.i, argmax_shfl.i] as bits,
// then the double sums as two words each
__global__ __launch_bounds__(256) void check_kernel(const float* in, const int* ties, unsigned* out) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const float v = in[g];
  // many equal values (argmax ties) and NaNs (never the maximum; ordered by index among themselves)
  const float t = ties[g] == 1 ? 1.0f : ties[g] == 2 ? __int_as_float(0x7fc00000) : v;
  unsigned* o = out + (long)g * 12;
  const float s0 = wave_sum(v), s1 = wave_sum_shfl(v);
  const float m0 = wave_max(v), m1 = wave_max_shfl(v);
  const ArgMax a0 = wave_argmax(ArgMax{t, (int)(threadIdx.x & 63) * 3}), a1 = wave_argmax_shfl(ArgMax{t, (int)(threadIdx.x & 63) * 3});
  const double d = (double)v * 1.000000119 + 1e-9 * g;
  const double d0 = wave_sum_d(d), d1 = wave_sum_d_shfl(d);
  o[0] = __float_as_uint(s0);
  o[1] = __float_as_uint(s1);
  o[2] = __float_as_uint(m0);
  o[3] = __float_as_uint(m1);
  o[4] = __float_as_uint(a0.v);
  o[5] = __float_as_uint(a1.v);
  o[6] = (unsigned)a0.i;
  o[7] = (unsigned)a1.i;
  const unsigned long long u0 = __double_as_longlong(d0), u1 = __double_as_longlong(d1);
  o[8] = (unsigned)u0;
  o[9] = (unsigned)(u0 >> 32);
  o[10] = (unsigned)u1;
  o[11] = (unsigned)(u1 >> 32);
}

int main() {
  const int blocks = 4096, n = blocks * 256;
  std::vector<float> h(n);
  std::vector<int> ties(n);
  unsigned s = 12345u;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    const float u = (float)(s >> 8) / 16777216.0f - 0.5f;
    const int e = (int)((s >> 3) % 40) - 20;
    h[i] = ldexpf(u, e);
    const unsigned k = (s >> 13) % 10;
    ties[i] = k < 2 ? 1 : k == 2 ? 2 : 0;
    if (i % (64 * 7) < 64) ties[i] = 2;  // some waves all NaN
  }
  float* din;
  int* dt;
  unsigned* dout;
  if (hipMalloc(&din, n * 4) || hipMalloc(&dt, n * 4) || hipMalloc(&dout, (size_t)n * 48)) return 2;
  if (hipMemcpy(din, h.data(), n * 4, hipMemcpyHostToDevice) ||
      hipMemcpy(dt, ties.data(), n * 4, hipMemcpyHostToDevice))
    return 2;
  check_kernel<<<blocks, 256>>>(din, dt, dout);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<unsigned> o((size_t)n * 12);
  if (hipMemcpy(o.data(), dout, (size_t)n * 48, hipMemcpyDeviceToHost)) return 2;
  const char* what[] = {"wave_sum", "wave_max", "wave_argmax.v", "wave_argmax.i"};
  for (int i = 0; i < n; ++i) {
    const unsigned* r = &o[(size_t)i * 12];
    for (int k = 0; k < 4; ++k)
      if (r[2 * k] != r[2 * k + 1]) {
        printf("MISMATCH %s lane %d: %08x vs %08x\n", what[k], i, r[2 * k], r[2 * k + 1]);
        return 1;
      }
    if (i % 64 == 0) {  // the first maximum of the wave's argmax inputs, NaN never taken unless all are NaN
      int best = -1;
      float bv = 0.0f;
      for (int l = 0; l < 64; ++l) {
        const float t = ties[i + l] == 1 ? 1.0f : ties[i + l] == 2 ? NAN : h[i + l];
        if (t == t && (best < 0 || t > bv || bv != bv)) best = l, bv = t;
        if (best < 0 && t != t) best = l, bv = t;
      }
      if ((int)r[6] != best * 3) {
        printf("MISMATCH wave_argmax.i vs the sequential scan, wave at lane %d: %d vs %d\n", i, (int)r[6], best * 3);
        return 1;
      }
    }
    if (r[8] != r[10] || r[9] != r[11]) {
      printf("MISMATCH wave_sum_d lane %d\n", i);
      return 1;
    }
  }
  printf("reduce_dpp_check ok %d lanes (sum, max, argmax with ties and NaNs, double sum bit-identical; argmax = the sequential scan)\n", n);
  return 0;
}
