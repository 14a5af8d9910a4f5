// gemv.hip -- single-frame (one-row) kernels: the recurrent layer and the per-frame SGD of the
// TRecurrentCu loop (src/CuTNetLib/cuRecurrent.cc:16-153, CuMath::OffsetGemv / BlasGer,
// src/CuBaseLib/cumath.cc:292-362), where every GEMM has one row and the reference issues
// cublasSgemv / cublasSger calls.
//
//   * row vector x matrix  (y = act(b + v W), W [K x N] row-major): split-K over many workgroups
//     (lane = column, coalesced 256-B rows of W), fixed-order partials, one finishing kernel --
//     enough workgroups to fill the chip for K ~ 1000, deterministic;
//   * matrix x vector rows (y_r = W[r0 + r, :] . x, optionally times s(1-s) and plus beta*y):
//     one wavefront per row, float4 loads, butterfly reduction;
//   * recurrent weight update: all BPTT outer products + weight decay + the weight write in ONE
//     pass over W (the reference: bptt+1 cublasSger calls, AddScaled, AddScaled).
#include "kcommon.h"

namespace tnetk {

constexpr int GV_KSLICE = 64;  // k rows per split-K slice

// partial[s][c] = sum_{k in slice s} v[k] * W[k][c]
__global__ __launch_bounds__(256) void gemv_rowvec_partial(const float* __restrict__ v, int K,
                                                           const float* __restrict__ W, long ldw, int N,
                                                           float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int k0 = blockIdx.y * GV_KSLICE, k1 = min(K, k0 + GV_KSLICE);
  float acc = 0.f;
  if (c < N) {
#pragma unroll 4
    for (int k = k0 + w; k < k1; k += 4) acc += v[k] * W[(long)k * ldw + c];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && c < N) partial[(long)blockIdx.y * N + c] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// y[c] = act(b[c] + sum_s partial[s][c]) ; act: 0 none, 1 sigmoid
__global__ __launch_bounds__(256) void gemv_rowvec_final(const float* __restrict__ partial, int slices, int N,
                                                         const float* __restrict__ b, float* __restrict__ y, int act) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  float s = 0.f;
  for (int k = 0; k < slices; ++k) s += partial[(long)k * N + c];
  const float a = (b ? b[c] : 0.f) + s;
  y[c] = act == 1 ? sigmoidf_ref(a) : a;
}

// y[r] = beta*y[r] + dot(W[r0 + r, 0:n], x) ; then if s != NULL: y[r] *= s[r] (1 - s[r])
__global__ __launch_bounds__(256) void gemv_rows_kernel(const float* __restrict__ W, long ldw, int r0, int nrows,
                                                        int n, const float* __restrict__ x, float* __restrict__ y,
                                                        float beta, const float* __restrict__ s) {
  const int lane = threadIdx.x & 63;
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= nrows) return;
  const float* row = W + (long)(r0 + r) * ldw;
  float acc = 0.f;
  if ((n & 3) == 0 && (ldw & 3) == 0 && (((uintptr_t)row | (uintptr_t)x) & 15) == 0) {
    for (int c = lane * 4; c < n; c += 256) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(row + c), b = *reinterpret_cast<const f32x4*>(x + c);
      acc += a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
    }
  } else {
    for (int c = lane; c < n; c += 64) acc += row[c] * x[c];
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    float o = beta == 0.f ? acc : beta * y[r] + acc;
    if (s) o = o * (s[r] * (1.f - s[r]));
    y[r] = o;
  }
}

// Recurrent update (cuRecurrent.cc:88-153).  Per element of W [rows x nout]:
//   acc = sum_{i < steps} (-lr h_i[k]) d_i[c]       (the BlasGer accumulations, corr reset to 0)
//   c   = (-lr wc) W + acc ; W = c + W
// h_i = history row i (physical row (head + i) % R of hist), d_i = row i of D.
// Block row gridDim.y-1 updates the bias: cb = -lr d_0 + mmt cb ; cb = -lr d_i + cb ; b += cb.
__global__ __launch_bounds__(256) void rnn_update_kernel(float* __restrict__ W, long ldw, int rows, int nout,
                                                         const float* __restrict__ hist, long ldh, int head, int R,
                                                         const float* __restrict__ D, long ldd, int steps,
                                                         float* __restrict__ b, float* __restrict__ cb, float lr,
                                                         float mmt, float wc) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (c >= nout) return;
  if (k == rows) {  // bias
    float g = -lr * D[c] + mmt * cb[c];
    for (int i = 1; i < steps; ++i) g = -lr * D[(long)i * ldd + c] + g;
    cb[c] = g;
    b[c] = g + b[c];
    return;
  }
  float acc = 0.f;
  for (int i = 0; i < steps; ++i) {
    const float h = hist[(long)((head + i) % R) * ldh + k];
    acc += (-lr * h) * D[(long)i * ldd + c];
  }
  float* wp = W + (long)k * ldw + c;
  const float w = *wp;
  const float corr = (-lr * wc) * w + acc;
  *wp = corr + w;
}

}  // namespace tnetk

using namespace tnetk;

extern "C" long tnet_gemv_workspace(int K, int N) { return (long)cdiv(K, GV_KSLICE) * (N > 0 ? N : 1) * 4; }

extern "C" int tnet_gemv_rowvec(const float* v, int K, const float* W, int ldw, const float* b, float* y, int N,
                                int act, void* workspace, void* stream) {
  if (K <= 0 || N <= 0 || ldw < N || !v || !W || !y || !workspace || act < 0 || act > 1) return TNET_ERR_ARG;
  const int slices = cdiv(K, GV_KSLICE);
  float* part = (float*)workspace;
  hipStream_t st = (hipStream_t)stream;
  gemv_rowvec_partial<<<dim3(cdiv(N, 64), slices), 256, 0, st>>>(v, K, W, ldw, N, part);
  TNET_LAUNCH_CHECK();
  gemv_rowvec_final<<<cdiv(N, 256), 256, 0, st>>>(part, slices, N, b, y, act);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_gemv_rows(const float* W, int ldw, int r0, int nrows, int n, const float* x, float* y,
                              float beta, const float* s, void* stream) {
  if (nrows < 0 || n < 0 || ldw < n || r0 < 0 || !W || !x || !y) return TNET_ERR_ARG;
  if (!nrows) return TNET_OK;
  gemv_rows_kernel<<<cdiv((long)nrows * 64, 256), 256, 0, (hipStream_t)stream>>>(W, ldw, r0, nrows, n, x, y, beta, s);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_rnn_update(float* W, int ldw, int rows, int nout, const float* hist, int ldh, int head, int R,
                               const float* D, int ldd, int steps, float* b, float* corr_b, float lr, float mmt,
                               float wc, void* stream) {
  if (rows <= 0 || nout <= 0 || steps <= 0 || steps > R || head < 0 || head >= R || !W || !hist || !D || !b ||
      !corr_b || ldw < nout || ldh < rows || ldd < nout)
    return TNET_ERR_ARG;
  rnn_update_kernel<<<dim3(cdiv(nout, 256), rows + 1), 256, 0, (hipStream_t)stream>>>(
      W, ldw, rows, nout, hist, ldh, head, R, D, ldd, steps, b, corr_b, lr, mmt, wc);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}
