// kcommon.h -- shared device-side helpers for the gfx950 kernels of the TNet SGD path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tnet_kernels.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define TNET_WAVE 64

namespace tnetk {

// Wave-wide butterfly reductions, partner lane i ^ o for o = 32, 16, 8, 4, 2, 1 (every lane ends with the
// result).  The exchanges are VALU cross-lane moves instead of ds_bpermute (an LDS round trip and an lgkmcnt
// wait per step): o = 32 / 16 by v_permlane32_swap / v_permlane16_swap (gfx950), o = 8 by the DPP row
// rotation by 8 (= xor 8 inside a 16-lane row), o = 4 by the DPP row rotation by 4 -- lane j gets j + 4
// mod 16, which is j ^ 4 or (j ^ 4) ^ 8, and after the o = 8 step lanes j and j ^ 8 hold the same value --
// and o = 2 / 1 by DPP quad permutations.  Each step combines a lane with exactly the value the
// __shfl_xor butterfly would give it, and fp addition is commutative, so the results are bit-identical to
// the shfl form (tools/reduce_dpp_check.hip checks all four reductions bit for bit on MI355X).
__device__ __forceinline__ unsigned xlane32(unsigned x) {  // lane i ^ 32's x
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (__lane_id() & 32) ? r[0] : r[1];
}
__device__ __forceinline__ unsigned xlane16(unsigned x) {  // lane i ^ 16's x
  const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return (__lane_id() & 16) ? r[0] : r[1];
}
template <int CTRL>
__device__ __forceinline__ unsigned xdpp(unsigned x) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
constexpr int kDppRor8 = 0x128, kDppRor4 = 0x124, kDppXor2 = 0x4E, kDppXor1 = 0xB1;
// the partner's 32-bit word at butterfly step S (0: xor 32 .. 5: xor 1; step 3 relies on step 2's symmetry)
template <int S>
__device__ __forceinline__ unsigned xstep(unsigned x) {
  if constexpr (S == 0) return xlane32(x);
  else if constexpr (S == 1) return xlane16(x);
  else if constexpr (S == 2) return xdpp<kDppRor8>(x);
  else if constexpr (S == 3) return xdpp<kDppRor4>(x);
  else if constexpr (S == 4) return xdpp<kDppXor2>(x);
  else return xdpp<kDppXor1>(x);
}
template <int S>
__device__ __forceinline__ float xstep_f(float v) {
  return __uint_as_float(xstep<S>(__float_as_uint(v)));
}
template <int S>
__device__ __forceinline__ double xstep_d(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = xstep<S>((unsigned)u), hi = xstep<S>((unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += xstep_f<0>(v);
  v += xstep_f<1>(v);
  v += xstep_f<2>(v);
  v += xstep_f<3>(v);
  v += xstep_f<4>(v);
  v += xstep_f<5>(v);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
  v += xstep_d<0>(v);
  v += xstep_d<1>(v);
  v += xstep_d<2>(v);
  v += xstep_d<3>(v);
  v += xstep_d<4>(v);
  v += xstep_d<5>(v);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, xstep_f<0>(v));
  v = fmaxf(v, xstep_f<1>(v));
  v = fmaxf(v, xstep_f<2>(v));
  v = fmaxf(v, xstep_f<3>(v));
  v = fmaxf(v, xstep_f<4>(v));
  v = fmaxf(v, xstep_f<5>(v));
  return v;
}
// the ds_bpermute butterflies these replace (tools/reduce_dpp_check.hip compares the two)
__device__ __forceinline__ float wave_sum_shfl(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d_shfl(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max_shfl(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// sigmoid 1/(1+exp(-x)) (cukernels.cu:192-206) on the hardware transcendentals: v_exp_f32 of
// -x*log2(e) and v_rcp_f32 -- 3 VALU instead of ocml expf + an IEEE division (~25), which made the
// sigmoid the largest part of the fused forward GEMM's epilogue.  Error <= ~3e-7 absolute for
// |x| <= 16 (the scaled exponent's rounding, damped by sigma(1-sigma) <= 1/4), well inside the
// kernel tests' 2e-6; exp overflow / underflow give exactly 0 / 1.
#ifdef TNET_PRECISE_TRANSCENDENTALS
// diagnostics build (make precise): the reference's double-precision formula, and libm-accurate exp
__device__ __forceinline__ float sigmoidf_ref(float x) { return (float)(1.0 / (1.0 + exp(-(double)x))); }
#else
__device__ __forceinline__ float sigmoidf_ref(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}
#endif

// Write-through (sc1) 16-B output stores through a buffer descriptor of the workgroup's output tile (or row).  A
// plain store leaves its line dirty in the XCD's L2 and the kernel-end release writes every dirty line
// back AFTER the last workgroup has finished (MI355X_MICROARCH.md price list, 'boundary': + B / 6 TB/s
// for B dirty bytes); an sc1 store sends the line out as it is written, overlapped with the other
// workgroups' main loops.  Nothing is lost by dropping the line: the next kernel reads the output on
// other XCDs (L2s are not coherent across XCDs; a kernel boundary invalidates them).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7FFFFFF0, 0x00020000);
}
__device__ __forceinline__ void st_wt(__amdgpu_buffer_rsrc_t r, long elem_off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)(elem_off * 4), 0, 16);
}
// the matching sc1 load: reads what another workgroup stored with st_wt without an acquire fence
// (cdna_hip_programming.md, in-launch split-K reduction, sc1 form)
__device__ __forceinline__ f32x4 ld_sc1(__amdgpu_buffer_rsrc_t r, long elem_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(elem_off * 4), 0, 16));
}

struct ArgMax {
  float v;
  int i;
};
__device__ __forceinline__ ArgMax argmax_merge(ArgMax a, ArgMax b) {
  // first maximum wins: larger value, or equal value with smaller index.  A NaN never wins over a number (the
  // reference's scan `val > max` never takes one, cukernels.cu:408-411) and two NaNs go by index, so the merge
  // is symmetric for every input -- what the butterfly below relies on
  const bool a_nan = a.v != a.v, b_nan = b.v != b.v;
  if (a_nan != b_nan) return a_nan ? b : a;
  if (b.v > a.v || (!(b.v < a.v) && b.i < a.i)) return b;
  return a;
}
template <int S>
__device__ __forceinline__ ArgMax xstep_am(ArgMax a) {
  return ArgMax{xstep_f<S>(a.v), (int)xstep<S>((unsigned)a.i)};
}
// argmax_merge is symmetric (the larger value, the smaller index on ties, NaN ordered below every number), so the
// butterfly steps above apply
__device__ __forceinline__ ArgMax wave_argmax(ArgMax a) {
  a = argmax_merge(a, xstep_am<0>(a));
  a = argmax_merge(a, xstep_am<1>(a));
  a = argmax_merge(a, xstep_am<2>(a));
  a = argmax_merge(a, xstep_am<3>(a));
  a = argmax_merge(a, xstep_am<4>(a));
  a = argmax_merge(a, xstep_am<5>(a));
  return a;
}
__device__ __forceinline__ ArgMax wave_argmax_shfl(ArgMax a) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = argmax_merge(a, b);
  }
  return a;
}

// exp(x) for x <= 0 on v_exp_f32: exp2(x*log2 e); relative error ~|x|*6e-8 (the rounding of the
// scaled argument), i.e. <= 1e-6 over the 16 nats that carry any probability mass
#ifdef TNET_PRECISE_TRANSCENDENTALS
__device__ __forceinline__ float fast_exp(float x) { return (float)exp((double)x); }
#else
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(1.44269504088896341f * x); }
#endif

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// HybridTaus uniform of the RBM sampling (CuRand, curandkernels.cu:14-44): three Tausworthe steps +
// one LCG step on an element's four states, u = 2^-32-scaled xor in double rounded to float, redrawn
// unless 0 < u < 1 (rand.hip: generator notes)
__device__ __forceinline__ unsigned taus_step(unsigned& z, int s1, int s2, int s3, unsigned m) {
  const unsigned b = ((z << s1) ^ z) >> s2;
  return z = ((z & m) << s3) ^ b;
}
__device__ __forceinline__ unsigned lcg_step(unsigned& z) { return z = 1664525u * z + 1013904223u; }

__device__ __forceinline__ float hybrid_taus(unsigned& z1, unsigned& z2, unsigned& z3, unsigned& z4) {
  float r;
  do {
    const unsigned x = taus_step(z1, 13, 19, 12, 4294967294u) ^ taus_step(z2, 2, 25, 4, 4294967288u) ^
                       taus_step(z3, 3, 11, 17, 4294967280u) ^ lcg_step(z4);
    r = (float)(2.3283064365387e-10 * (double)x);
  } while (!(r > 0.0f && r < 1.0f));
  return r;
}

}  // namespace tnetk

#define TNET_LAUNCH_CHECK()                                   \
  do {                                                        \
    hipError_t _e = hipGetLastError();                        \
    if (_e != hipSuccess) return TNET_ERR_LAUNCH;             \
  } while (0)
