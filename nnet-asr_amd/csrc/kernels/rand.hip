// rand.hip -- the per-element random number generators of the RBM path (CuRand,
// src/CuBaseLib/curand.h:11-32, curandkernels.cu:14-107) on gfx950.
//
// Same generator as the reference: every matrix element owns four 32-bit states (three Tausworthe
// steps + one LCG step, "HybridTaus", period ~2^121), seeded on the host from lrand48 (> 128,
// curand.tcc:36-45) and kept in HBM between calls; uniform = 2.3283064365387e-10 * (t1^t2^t3^lcg)
// computed in double and rounded to float, redrawn unless 0 < u < 1 (curandkernels.cu:30-44);
// Gaussian = Box-Muller r*sin(theta) from two uniforms (:55-67).  The integer recurrences are
// exact, so uniforms and binarised states are bit-identical to the reference's for the same
// seeds.  The state arrays share the stride of the target matrix (index = col + row*stride, as
// the reference indexes them with the target's MatrixDim).
//
// MI355X: one lane per element, rows along blockIdx.y (coalesced state loads/stores), and the
// binarisation fused with the draw (the reference writes the uniforms to a temporary matrix and
// reads them back, curand.tcc:121-134).  HBM-bound: 32 B of state traffic per element.
#include "kcommon.h"

namespace tnetk {

__device__ __forceinline__ float box_muller(unsigned& z1, unsigned& z2, unsigned& z3, unsigned& z4) {
  const float two_pi = 6.283185307179586476925286766558f;
  const float u0 = hybrid_taus(z1, z2, z3, z4), u1 = hybrid_taus(z1, z2, z3, z4);
  // the reference's float instantiation: T r = sqrt(-2.0*log(u0)) (double sqrt of a float log,
  // rounded to float), T theta = M_2PI*u1, return r*sin(theta) in float
  const float r = (float)sqrt(-2.0 * (double)logf(u0));
  const float theta = two_pi * u1;
  return r * sinf(theta);
}

// MODE 0: dst = U ; 1: dst = N(0,1) ; 2: dst = (src > U) ; 3: dst += scale * N(0,1)
template <int MODE>
__global__ __launch_bounds__(256) void rand_kernel(float* __restrict__ dst, int ldd, const float* __restrict__ src,
                                                   int lds, TnetMatrixDim d, unsigned* __restrict__ z1,
                                                   unsigned* __restrict__ z2, unsigned* __restrict__ z3,
                                                   unsigned* __restrict__ z4, float scale) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  const int row = blockIdx.y;
  if (col >= d.cols || row >= d.rows) return;
  const long s = (long)row * d.stride + col;  // state index (reference: i + j*d.stride)
  unsigned a = z1[s], b = z2[s], c = z3[s], e = z4[s];
  float* o = dst + (long)row * ldd + col;
  if (MODE == 0) {
    *o = hybrid_taus(a, b, c, e);
  } else if (MODE == 1) {
    *o = box_muller(a, b, c, e);
  } else if (MODE == 2) {
    const float u = hybrid_taus(a, b, c, e);
    *o = src[(long)row * lds + col] > u ? 1.0f : 0.0f;
  } else {
    *o = *o + scale * box_muller(a, b, c, e);
  }
  z1[s] = a; z2[s] = b; z3[s] = c; z4[s] = e;
}

template <int MODE>
static int rand_run(float* dst, int ldd, const float* src, int lds, TnetMatrixDim d, unsigned* z1, unsigned* z2,
                    unsigned* z3, unsigned* z4, float scale, void* stream) {
  if (d.rows < 0 || d.cols < 0 || d.stride < d.cols || !dst || !z1 || !z2 || !z3 || !z4) return TNET_ERR_ARG;
  if (!d.rows || !d.cols) return TNET_OK;
  rand_kernel<MODE><<<dim3(cdiv(d.cols, 256), d.rows), 256, 0, (hipStream_t)stream>>>(dst, ldd, src, lds, d, z1, z2, z3,
                                                                                       z4, scale);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

}  // namespace tnetk

using namespace tnetk;

extern "C" int tnetF_rand(float* mat, TnetMatrixDim d, unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4,
                          void* stream) {
  return rand_run<0>(mat, d.stride, nullptr, 0, d, z1, z2, z3, z4, 0.f, stream);
}

extern "C" int tnetF_gauss_rand(float* mat, TnetMatrixDim d, unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4,
                                void* stream) {
  return rand_run<1>(mat, d.stride, nullptr, 0, d, z1, z2, z3, z4, 0.f, stream);
}

extern "C" int tnet_rand_binarize(float* states, int ld_states, const float* probs, TnetMatrixDim d, unsigned* z1,
                                  unsigned* z2, unsigned* z3, unsigned* z4, void* stream) {
  if (!probs) return TNET_ERR_ARG;
  return rand_run<2>(states, ld_states, probs, d.stride, d, z1, z2, z3, z4, 0.f, stream);
}

extern "C" int tnet_add_gauss_noise(float* mat, TnetMatrixDim d, float scale, unsigned* z1, unsigned* z2,
                                    unsigned* z3, unsigned* z4, void* stream) {
  return rand_run<3>(mat, d.stride, nullptr, 0, d, z1, z2, z3, z4, scale, stream);
}

namespace tnetk {
__global__ __launch_bounds__(256) void binarize_kernel(float* __restrict__ states, const float* __restrict__ probs,
                                                       const float* __restrict__ rnd, TnetMatrixDim d) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  const int row = blockIdx.y;
  if (col >= d.cols || row >= d.rows) return;
  const long i = (long)row * d.stride + col;
  states[i] = probs[i] > rnd[i] ? 1.0f : 0.0f;
}
}  // namespace tnetk

extern "C" int tnetF_binarize_probs(float* states, const float* probs, const float* rnd, TnetMatrixDim d,
                                    void* stream) {
  if (d.rows < 0 || d.cols < 0 || d.stride < d.cols || !states || !probs || !rnd) return TNET_ERR_ARG;
  if (!d.rows || !d.cols) return TNET_OK;
  binarize_kernel<<<dim3(cdiv(d.cols, 256), d.rows), 256, 0, (hipStream_t)stream>>>(states, probs, rnd, d);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}
