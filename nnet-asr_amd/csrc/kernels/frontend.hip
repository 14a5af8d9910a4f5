// frontend.hip -- the block-diagonal linear transform of the feature front end (<blocklinearity>,
// src/CuTNetLib/cuCRBEDctFeat.h:175-235, CuMath::BlockLinearity, src/CuBaseLib/cumath.cc:76-113).
//
// The reference issues one cublasSgemm per block (23 blocks of 51 -> 26 in the examples/01
// Hamm_dct_norm transform), each a skinny GEMM at an odd column offset.  Here the whole
// block-diagonal product is ONE launch: the [bi x bo] block matrix is staged in LDS once per
// workgroup, every lane owns one output column of a run of rows (coalesced stores; the bi inputs
// of its block are shared by the bo lanes of that block through L1/L2).  The work is tiny next to
// the network (bi*bo MACs per block per frame), HBM-bound on X and Y; arbitrary strides and
// offsets, no alignment requirement.  Summation order: i = 0 .. bi-1, one fma per term.
#include "kcommon.h"

namespace tnetk {

constexpr int BL_THREADS = 256;
constexpr int BL_ROWS = 8;              // rows per workgroup (the block matrix is loaded once)
constexpr int BL_LDS_FLOATS = 16384;    // 64 KiB of block matrix in LDS; larger -> read from L2

template <bool LDS>
__global__ __launch_bounds__(BL_THREADS) void block_linearity_kernel(float* __restrict__ y, TnetMatrixDim dy,
                                                                     const float* __restrict__ x, TnetMatrixDim dx,
                                                                     const float* __restrict__ t, TnetMatrixDim dt) {
  extern __shared__ float st[];
  const int bi = dt.rows, bo = dt.cols;
  const float* tm = t;
  int ldt = dt.stride;
  if (LDS) {
    for (int e = threadIdx.x; e < bi * bo; e += BL_THREADS) st[e] = t[(long)(e / bo) * dt.stride + e % bo];
    __syncthreads();
    tm = st;
    ldt = bo;
  }
  for (int r0 = blockIdx.y * BL_ROWS; r0 < dy.rows; r0 += gridDim.y * BL_ROWS) {
    const int r1 = min(dy.rows, r0 + BL_ROWS);
    for (int c = blockIdx.x * BL_THREADS + threadIdx.x; c < dy.cols; c += gridDim.x * BL_THREADS) {
      const int b = c / bo, o = c - b * bo;
      const float* tc = tm + o;
      for (int r = r0; r < r1; ++r) {
        const float* xr = x + (long)r * dx.stride + (long)b * bi;
        float acc = 0.f;
        for (int i = 0; i < bi; ++i) acc = fmaf(xr[i], tc[(long)i * ldt], acc);
        y[(long)r * dy.stride + c] = acc;
      }
    }
  }
}

}  // namespace tnetk

using namespace tnetk;

extern "C" int tnet_block_linearity(float* y, TnetMatrixDim dy, const float* x, TnetMatrixDim dx, const float* t,
                                    TnetMatrixDim dt, void* stream) {
  if (!y || !x || !t || dt.rows <= 0 || dt.cols <= 0 || dt.stride < dt.cols || dx.stride < dx.cols ||
      dy.stride < dy.cols || dx.rows != dy.rows || dx.cols % dt.rows != 0 || dy.cols % dt.cols != 0 ||
      dx.cols / dt.rows != dy.cols / dt.cols)
    return TNET_ERR_ARG;
  if (!dy.rows || !dy.cols) return TNET_OK;
  const dim3 grid(cdiv(dy.cols, BL_THREADS), min(cdiv(dy.rows, BL_ROWS), 16384));
  hipStream_t st = (hipStream_t)stream;
  const long tsz = (long)dt.rows * dt.cols;
  if (tsz <= BL_LDS_FLOATS)
    block_linearity_kernel<true><<<grid, BL_THREADS, tsz * sizeof(float), st>>>(y, dy, x, dx, t, dt);
  else
    block_linearity_kernel<false><<<grid, BL_THREADS, 0, st>>>(y, dy, x, dx, t, dt);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}
