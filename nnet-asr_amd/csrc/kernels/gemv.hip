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
#include <float.h>

#include "kcommon.h"

namespace tnetk {

constexpr int GV_KSLICE = 64;  // k rows per split-K slice

// The recurrent update of the previous frame (rnn_update_kernel's arithmetic) carried into the next
// frame's forward: every W element is updated by the workgroup that reads it next (below)
struct RnnPendingUpdate {
  const float* hist;  // the history ring [R x ldh] at the update's head
  long ldh;
  int head, R;
  const float* D;  // [steps x ldd] back-propagated errors d_0..d_{steps-1}
  long ldd;
  int steps;       // = the kernel's ST
  float* b;
  float* cb;
  float lr, mmt, wc;
};
constexpr int GV_UPD_MAX = 9;  // steps = bptt + 1 of the folded form (deeper: the update's own launch)

// The look-ahead form of the frame chain (CuRecurrentTrainer, TNET_RNN_AHEAD).  The next frame's recurrent forward
// v_{t+1} W_{t+1}, v_{t+1} = [x_{t+1}, y_t], needs the frame's update W_{t+1} = W_t + corr (cuRecurrent.cc:88-153:
// corr = (-lr wc) W_t + sum_i (-lr h_i) (x) d_i), which exists only after the frame's BPTT.  Since
//   v W_{t+1} = (1 - lr wc) (v W_t) + sum_i (-lr (v . h_i)) d_i,
// the product with the OLD weights and the dots v . h_i are taken as soon as y_t exists -- beside the output layer's
// backprop (RnnAhead blocks of rnn_out_bwd_kernel) -- and the next frame's first launch only adds the rank-(bptt+1)
// correction while it finishes the sigmoid (rnn_out_full_kernel with RnnCorr), the weight update itself running in
// that launch's extra workgroups.  One launch less a frame on the dependent chain; the recurrent output differs from
// the materialised product by fp32 reassociation only.
struct RnnAhead {
  // bias blocks: the previous frame's recurrent bias update, computed by the forward that used it into bnext /
  // cbnext, copied to b / cb here (the forward's other workgroups were reading the old values)
  int nbias, H;
  const float* bnext;
  const float* cbnext;
  float* b;
  float* cb;
  // look-ahead blocks: partial[s][c] = sum_{k in slice s} v[k] W[k][c] over cdiv(H, 64) x slices blocks, the
  // column-block-0 ones also the dots dpart[s][i] = sum_{k in slice s} v[k] h_i[k] (h_i = ring row (head + i) % R,
  // i < steps) and the push of v into the ring row vout
  int nlook;
  const float* v0;
  int K0;
  const float* v1;
  int K;
  const float* W;
  long ldw;
  float* partial;
  float* dpart;
  float* vout;
  const float* hist;
  long ldh;
  int head, R, steps;
};
constexpr int GV_DOTS = 16;  // dpart row stride (steps <= GV_UPD_MAX)

// the next frame's first launch: the correction of the look-ahead product and the pending update
struct RnnCorr {
  int on;
  const float* dpart;  // [slices x GV_DOTS]
  const float* D;      // [steps x ldd] d_0 .. d_{steps-1} of the pending update
  long ldd;
  int steps;
  float lr, mmt, wc;
  const float* cb;  // the bias' momentum (old); the old bias is rnn_out_full_kernel's hb
  float* bnext;     // new bias / momentum (written by workgroup 0; copied by the next RnnAhead bias blocks)
  float* cbnext;
  // update blocks: W [rows x H] (rnn_update_kernel's arithmetic, no bias), 4 elements a thread
  int nupd;
  float* W;
  long ldw;
  int rows;
  const float* hist;
  long ldh;
  int head, R;
};

// partial[s][c] = sum_{k in slice s} v[k] * W[k][c], v = [v0[0:K0], v1[0:K-K0]] (the recurrent
// layer's [x_t, y_{t-1}], read in place); the column-block-0 workgroups also store v to vout (the
// history row, cuRecurrent.cc:31-35), so the two row copies need no launches of their own.
// UPD: the previous frame's recurrent update first (cuRecurrent.cc:88-153; per element exactly
// rnn_update_kernel's sum in step order, corr = (-lr wc) w + acc, w = corr + w), written back and used
// for this frame's product -- the update needs no launch of its own (every element of W is read by
// exactly one workgroup here); the k-slice-0 workgroups update the bias.  The ring must not hand vout
// a row the update reads (R >= steps + 1: CuRecurrent keeps bptt + 2 rows).
template <bool UPD, int ST = 1>
__global__ __launch_bounds__(256) void gemv_rowvec_partial_k(const float* __restrict__ v0, int K0,
                                                             const float* __restrict__ v1, int K,
                                                             float* __restrict__ W, long ldw, int N,
                                                             float* __restrict__ partial, float* __restrict__ vout,
                                                             RnnPendingUpdate u) {
  __shared__ float red[4][64];
  __shared__ float hsl[UPD ? ST * GV_KSLICE : 1];  // the update's history values of this k-slice
  constexpr int KPW = GV_KSLICE / 4;                       // k rows per wave
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, cc = min(c, N - 1);
  const int k0 = blockIdx.y * GV_KSLICE, k1 = min(K, k0 + GV_KSLICE);
  auto vk = [&](int k) { return k < K0 ? v0[k] : v1[k - K0]; };
  // every load of the workgroup in one round: the wave's KPW rows of W, the row vector, (UPD) the
  // errors of column c and the slice's history rows
  float wv[KPW], xv[KPW];
#pragma unroll
  for (int q = 0; q < KPW; ++q) {
    const int k = min(k0 + w + 4 * q, K - 1);
    wv[q] = W[(long)k * ldw + cc];
    xv[q] = vk(k);
  }
  float acc = 0.f;
  if constexpr (UPD) {
    // (one round of loads: every value the update needs is requested before the first is used --
    // the bias operands too, whose pointers the compiler cannot prove apart from W / cb)
    // unconditional loads at clamped indices (a predicated load is a branch here, and the branches
    // serialise the round); ST steps at compile time: straight-line code, the LDS reads batched
    float dv[ST];
#pragma unroll
    for (int i = 0; i < ST; ++i) dv[i] = u.D[(long)i * u.ldd + cc];
    constexpr int HPT = (ST * GV_KSLICE + 255) / 256;  // history values per thread
    float hl[HPT];
#pragma unroll
    for (int q = 0; q < HPT; ++q) {
      const int j = min((int)threadIdx.x + 256 * q, ST * GV_KSLICE - 1), i = j / GV_KSLICE;
      const int k = min(k0 + j % GV_KSLICE, K - 1);
      int r = u.head + i;
      r = r >= u.R ? r - u.R : r;
      hl[q] = u.hist[(long)r * u.ldh + k];
    }
    const bool bias = blockIdx.y == 0 && w == 0 && c < N;  // rnn_update_kernel's bias row
    const float cbv = u.cb[cc], bv = u.b[cc];
#pragma unroll
    for (int q = 0; q < HPT; ++q)
      if (threadIdx.x + 256 * q < ST * GV_KSLICE) hsl[threadIdx.x + 256 * q] = hl[q];
    if (bias) {
      float g = __fmaf_rn(-u.lr, dv[0], u.mmt * cbv);
#pragma unroll
      for (int i = 1; i < ST; ++i) g = __fmaf_rn(-u.lr, dv[i], g);
      u.cb[c] = g;
      u.b[c] = g + bv;
    }
    __syncthreads();
    float hv[KPW][ST];
#pragma unroll
    for (int q = 0; q < KPW; ++q)
#pragma unroll
      for (int i = 0; i < ST; ++i) hv[q][i] = hsl[i * GV_KSLICE + w + 4 * q];
#pragma unroll
    for (int q = 0; q < KPW; ++q) {
      const int k = k0 + w + 4 * q;
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < ST; ++i) a = __fmaf_rn(-u.lr * hv[q][i], dv[i], a);
      const float corr = __fmaf_rn(-u.lr * u.wc, wv[q], a);
      const float wn = corr + wv[q];
      if (k < k1 && c < N) {
        W[(long)k * ldw + c] = wn;
        acc += xv[q] * wn;
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < KPW; ++q)
      if (k0 + w + 4 * q < k1) acc += xv[q] * wv[q];
  }
  // the history push after the update's reads of the ring (a different row: R >= steps + 1)
  if (vout && blockIdx.x == 0)
    for (int k = k0 + threadIdx.x; k < k1; k += blockDim.x) vout[k] = vk(k);
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && c < N) partial[(long)blockIdx.y * N + c] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// One block of the look-ahead product (gemv_rowvec_partial_k<false>'s arithmetic and k order) at block coordinates
// (bx, by), its dots (bx == 0) and the push; 256 threads.
__device__ __forceinline__ void rnn_ahead_block(const RnnAhead& a, const int bx, const int by) {
  __shared__ float red[4][64];
  constexpr int KPW = GV_KSLICE / 4;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int N = a.H, K = a.K;
  const int c = bx * 64 + lane, cc = min(c, N - 1);
  const int k0 = by * GV_KSLICE, k1 = min(K, k0 + GV_KSLICE);
  auto vk = [&](int k) { return k < a.K0 ? a.v0[k] : a.v1[k - a.K0]; };
  float wv[KPW], xv[KPW];
#pragma unroll
  for (int q = 0; q < KPW; ++q) {
    const int k = min(k0 + w + 4 * q, K - 1);
    wv[q] = a.W[(long)k * a.ldw + cc];
    xv[q] = vk(k);
  }
  float acc = 0.f;
#pragma unroll
  for (int q = 0; q < KPW; ++q)
    if (k0 + w + 4 * q < k1) acc += xv[q] * wv[q];
  if (bx == 0) {
    // the dots of this k-slice, wave i over steps i, i + 4, ...: lane l takes k0 + l (the ring rows are read before
    // the push below replaces row vout: a different row, R >= steps + 1)
    const int k = k0 + lane;
    const float x = k < k1 ? vk(k) : 0.f;
    for (int i = w; i < a.steps; i += 4) {
      int r = a.head + i;
      r = r >= a.R ? r - a.R : r;
      const float h = k < k1 ? a.hist[(long)r * a.ldh + k] : 0.f;
      const float d = wave_sum(x * h);
      if (lane == 0) a.dpart[(long)by * GV_DOTS + i] = d;
    }
    __syncthreads();  // every wave's ring reads done before the push
    for (int kk = k0 + threadIdx.x; kk < k1; kk += blockDim.x) a.vout[kk] = vk(kk);
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && c < N) a.partial[(long)by * N + c] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// y[c] = act(b[c] + sum_s partial[s][c]) ; act: 0 none, 1 sigmoid
__global__ __launch_bounds__(256) void gemv_rowvec_final(const float* __restrict__ partial, int slices, int N,
                                                         const float* __restrict__ b, float* __restrict__ y, int act) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  float s = 0.f;
#pragma unroll 8
  for (int k = 0; k < slices; ++k) s += partial[(long)k * N + c];
  const float a = (b ? b[c] : 0.f) + s;
  y[c] = act == 1 ? sigmoidf_ref(a) : a;
}

// the output layer + <softmax> + cross-entropy of one frame (TRecurrentCu's
// CuBiasedLinearity::Propagate -> CuSoftmax::Propagate -> CuCrossEntropy::EvaluateLabels, with the
// network-output and error copies): z = b + sum_s partial[s] (the order of gemv_rowvec_final),
// y = softmax(z), e = y - onehot(t), xent / argmax-correct into the stats slots.  One workgroup,
// N <= GV_SMX_MAX columns held in registers (16 per thread).
constexpr int GV_SMX_PER = 16, GV_SMX_MAX = 256 * GV_SMX_PER;
__global__ __launch_bounds__(256) void gemv_softmax_xent_final(const float* __restrict__ partial, int slices, int N,
                                                               const float* __restrict__ b, float* __restrict__ z,
                                                               float* __restrict__ y, float* __restrict__ e,
                                                               const int* __restrict__ label,
                                                               double* __restrict__ stats) {
  __shared__ float smax[4];
  __shared__ double ssum[4];
  __shared__ ArgMax sarg[4];
  __shared__ float syt;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float rv[GV_SMX_PER];
  // slice-outer: each slice's 16 loads per thread are independent (a column-outer loop serialises
  // slices x 16 load latencies, 37 us at N = 4000); per column the sum order is unchanged
#pragma unroll
  for (int q = 0; q < GV_SMX_PER; ++q) rv[q] = 0.f;
  // loads are unconditional at a clamped column (no per-column branch + wait), masked afterwards
  const int nq = min(GV_SMX_PER, (N + 255) / 256);  // wave-uniform
  for (int k = 0; k < slices; ++k) {
    const float* pk = partial + (long)k * N;
    float p[GV_SMX_PER];
#pragma unroll
    for (int q = 0; q < GV_SMX_PER; ++q)
      if (q < nq) p[q] = pk[min((int)threadIdx.x + 256 * q, N - 1)];
#pragma unroll
    for (int q = 0; q < GV_SMX_PER; ++q)
      if (q < nq) rv[q] += p[q];
  }
  float bb[GV_SMX_PER];
#pragma unroll
  for (int q = 0; q < GV_SMX_PER; ++q) bb[q] = (b && q < nq) ? b[min((int)threadIdx.x + 256 * q, N - 1)] : 0.f;
  float m = -1e20f;
#pragma unroll
  for (int q = 0; q < GV_SMX_PER; ++q) {
    const int c = threadIdx.x + 256 * q;
    const float a = c < N ? bb[q] + rv[q] : -1e30f;
    if (z && c < N) z[c] = a;
    rv[q] = a;
    m = fmaxf(m, a);
  }
  m = wave_max(m);
  if (lane == 0) smax[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < GV_SMX_PER; ++q) {
    if (threadIdx.x + 256 * q < N) {
      rv[q] = fast_exp(rv[q] - m);
      s += rv[q];
    }
  }
  const double ws = wave_sum_d((double)s);
  if (lane == 0) ssum[wv] = ws;
  __syncthreads();
  const float rsum = 1.f / (float)(ssum[0] + ssum[1] + ssum[2] + ssum[3]);
  const int t = label[0] < N ? label[0] : -1;  // out of range: an unlabeled frame, as the batched kernels
  ArgMax ay{-1e20f, 0x7fffffff};
#pragma unroll
  for (int q = 0; q < GV_SMX_PER; ++q) {
    const int c = threadIdx.x + 256 * q;
    if (c < N) {
      const float yc = rv[q] * rsum;
      if (yc > ay.v) { ay.v = yc; ay.i = c; }
      if (y) y[c] = yc;
      if (e) e[c] = yc - (c == t ? 1.f : 0.f);
      if (c == t) syt = yc;
    }
  }
  ay = wave_argmax(ay);
  if (lane == 0) sarg[wv] = ay;
  __syncthreads();
  if (threadIdx.x == 0 && stats) {
    ArgMax a = sarg[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) a = argmax_merge(a, sarg[w]);
    const double xent = (t >= 0 && t < N) ? -(double)logf(fmaxf(syt, FLT_MIN)) : 0.0;
    atomicAdd(stats, xent);
    atomicAdd(stats + 1, (a.i == (t >= 0 ? t : 0)) ? 1.0 : 0.0);
  }
}

// a[0] b[0] + a[1] b[1] + a[2] b[2] + a[3] b[3] with every product rounded and the sums taken left to right
// (no contraction): the vectoriser may turn the products into v_pk_mul_f32 in one kernel and leave them for
// v_fmac in another, so gemv_rows_kernel and the BPTT chain pin the arithmetic here to stay bit-identical.
__device__ __forceinline__ float dot4_rounded(const f32x4 a, const f32x4 b) {
#pragma clang fp contract(off)
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
}

// y[r] = beta*y[r] + dot(W[r0 + r, 0:n], x) ; then if s != NULL: y[r] *= s[r] (1 - s[r]).
// Rows of <= 1024 aligned floats: every load of the wave (the row, x, s[r], y[r]) issued in one round
// at clamped addresses, the products then added in the loop form's order (c = 4 lane + 256 q)
__global__ __launch_bounds__(256) void gemv_rows_kernel(const float* __restrict__ W, long ldw, int r0, int nrows,
                                                        int n, const float* __restrict__ x, float* __restrict__ y,
                                                        float beta, const float* __restrict__ s) {
  const int lane = threadIdx.x & 63;
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= nrows) return;
  const float* row = W + (long)(r0 + r) * ldw;
  const float sv = s ? s[r] : 0.f;
  const float yv = beta != 0.f ? y[r] : 0.f;
  float acc = 0.f;
  if ((n & 3) == 0 && (ldw & 3) == 0 && (((uintptr_t)row | (uintptr_t)x) & 15) == 0) {
    if (n <= 1024) {
      f32x4 a[4], b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = min(lane * 4 + 256 * q, n - 4);
        a[q] = *reinterpret_cast<const f32x4*>(row + c);
        b[q] = *reinterpret_cast<const f32x4*>(x + c);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (lane * 4 + 256 * q < n) acc += dot4_rounded(a[q], b[q]);
    } else {
      for (int c = lane * 4; c < n; c += 256) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(row + c), b = *reinterpret_cast<const f32x4*>(x + c);
        acc += a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
      }
    }
  } else {
    for (int c = lane; c < n; c += 64) acc += row[c] * x[c];
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    float o = beta == 0.f ? acc : beta * yv + acc;
    if (s) o = o * (sv * (1.f - sv));
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
  if (k == rows) {  // bias (explicit fused multiply-adds: the same rounding in the folded form below)
    float g = __fmaf_rn(-lr, D[c], mmt * cb[c]);
    for (int i = 1; i < steps; ++i) g = __fmaf_rn(-lr, D[(long)i * ldd + c], g);
    cb[c] = g;
    b[c] = g + b[c];
    return;
  }
  float acc = 0.f;
  float* wp = W + (long)k * ldw + c;
  const float w = *wp;
  for (int i0 = 0; i0 < steps; i0 += 8) {  // up to 8 steps' loads in flight, accumulated in step order
    float hv[8], dv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = i0 + q;
      hv[q] = i < steps ? hist[(long)((head + i) % R) * ldh + k] : 0.f;
      dv[q] = i < steps ? D[(long)i * ldd + c] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (i0 + q < steps) acc = __fmaf_rn(-lr * hv[q], dv[q], acc);
  }
  const float corr = __fmaf_rn(-lr * wc, w, acc);
  *wp = corr + w;
}

// single-frame CuBiasedLinearity::Backpropagate + Update (cuBiasedLinearity.cc:32-64) in one pass
// over W, one wavefront per weight row i: eo[i] = W[i,:] . e with the OLD row (the order of
// gemv_rows_kernel), then the row's SGD exactly as affine_update_row_kernel; with s: d[i] =
// eo[i] s_i (1 - s_i) -- the diff-sigmoid of the recurrent layer below (cuRecurrent.cc:88-92).
// Workgroups past the weight rows update the bias.
__global__ __launch_bounds__(256) void affine_bwd_update_row_kernel(
    const float* __restrict__ x, int n_in, const float* __restrict__ e, int n_out, float* __restrict__ W, long ldw,
    float* __restrict__ corrW, long ldc, float* __restrict__ b, float* __restrict__ cb, float scale, float mmt,
    float l2, float* __restrict__ eo, const float* __restrict__ s, float* __restrict__ d, int row_blocks) {
  if ((int)blockIdx.x >= row_blocks) {  // bias
    const int j = (blockIdx.x - row_blocks) * blockDim.x + threadIdx.x;
    if (j >= n_out) return;
    float g = e[j];
    if (cb) {
      g = g + mmt * cb[j];
      cb[j] = g;
    }
    b[j] = b[j] + scale * g;
    return;
  }
  const int lane = threadIdx.x & 63;
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (i >= n_in) return;
  const float xi = x[i];
  float* row = W + (long)i * ldw;
  float* qrow = corrW ? corrW + (long)i * ldc : nullptr;
  auto upd = [&](float w, float ej, float* q) {
    float c = xi * ej;
    if (qrow) {
      c = c + mmt * *q;
      *q = c;
    }
    w = w + scale * c;
    return w + l2 * w;
  };
  float acc = 0.f;
  if ((n_out & 3) == 0 && (ldw & 3) == 0 && (!qrow || (ldc & 3) == 0) &&
      (((uintptr_t)row | (uintptr_t)e | (uintptr_t)qrow) & 15) == 0) {
    for (int c = lane * 4; c < n_out; c += 256) {
      f32x4 a = *reinterpret_cast<const f32x4*>(row + c);
      const f32x4 ev = *reinterpret_cast<const f32x4*>(e + c);
      acc += a[0] * ev[0] + a[1] * ev[1] + a[2] * ev[2] + a[3] * ev[3];
      f32x4 qv = qrow ? *reinterpret_cast<const f32x4*>(qrow + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      float q[4] = {qv[0], qv[1], qv[2], qv[3]};
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = upd(a[k], ev[k], &q[k]);
      *reinterpret_cast<f32x4*>(row + c) = a;
      if (qrow) *reinterpret_cast<f32x4*>(qrow + c) = f32x4{q[0], q[1], q[2], q[3]};
    }
  } else {
    for (int c = lane; c < n_out; c += 64) {
      const float w = row[c], ej = e[c];
      acc += w * ej;
      row[c] = upd(w, ej, qrow ? qrow + c : nullptr);
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    if (eo) eo[i] = acc;
    if (d) d[i] = acc * (s[i] * (1.f - s[i]));
  }
}

// single-frame CuBiasedLinearity::Update (cuBiasedLinearity.cc:46-64) as one rank-1 kernel: the
// GEMM's acc = x_i e_j (one exact fp32 product), the SGD epilogue of tnet_affine_update and the bias
// SGD of tnet_bias_update (the column sum of one row is the row) -- three launches in one
__global__ __launch_bounds__(256) void affine_update_row_kernel(const float* __restrict__ x, int n_in,
                                                                const float* __restrict__ e, int n_out,
                                                                float* __restrict__ W, long ldw,
                                                                float* __restrict__ corrW, long ldc,
                                                                float* __restrict__ b, float* __restrict__ cb,
                                                                float scale, float mmt, float l2) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = blockIdx.y;
  if (j >= n_out) return;
  const float ej = e[j];
  if (i == n_in) {  // bias
    float g = ej;
    if (cb) {
      g = g + mmt * cb[j];
      cb[j] = g;
    }
    b[j] = b[j] + scale * g;
    return;
  }
  float c = x[i] * ej;
  if (corrW) {
    float* qp = corrW + (long)i * ldc + j;
    c = c + mmt * *qp;
    *qp = c;
  }
  float* wp = W + (long)i * ldw + j;
  float w = *wp;
  w = w + scale * c;
  w = w + l2 * w;
  *wp = w;
}

// ---------------------------------------------------------------------------------------------
// TRecurrentCu frame chain, output side, in three launches instead of four (the recurrent layer's
// sigmoid finish, the output GEMV, the one-workgroup softmax and the output-layer backprop + update):
//   rnn_out_partial_kernel : h = sigmoid(b + sum of the recurrent split-K partials) for the
//                            workgroup's 64-row slice (gemv_rowvec_final's order, computed where it is
//                            consumed; column block 0 stores it), then the output split-K partials
//                            (gemv_rowvec_partial's order)
//   rnn_out_stats_kernel   : z = b + sum of the output partials (gemv_softmax_xent_final's order) for
//                            256 columns per workgroup, the workgroup's max m_g and sum of exp(z - m_g)
//   rnn_out_bwd_kernel     : every workgroup combines the (m_g, s_g) pairs into the softmax normaliser,
//                            forms e = softmax(z) - onehot(t) where it reads it, and runs
//                            affine_bwd_update_row_kernel's arithmetic; the bias workgroups add the
//                            cross-entropy and fold their argmax into the frame's 64-bit argmax key
//                            (atomicMax of {y bits, ~column}: largest y, first column on ties)
//   argmax_correct_kernel  : at the end of the utterance, frame accuracy from the keys
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rnn_out_partial_kernel(const float* __restrict__ hpart, int hslices,
                                                              const float* __restrict__ hb, float* __restrict__ h,
                                                              int H, const float* __restrict__ Wo, long ldw, int N,
                                                              float* __restrict__ opart) {
  __shared__ float red[4][64];
  __shared__ float hs[GV_KSLICE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int k0 = blockIdx.y * GV_KSLICE, k1 = min(H, k0 + GV_KSLICE);
  if ((int)threadIdx.x < k1 - k0) {
    const int k = k0 + threadIdx.x;
    float sacc = 0.f;
    for (int q0 = 0; q0 < hslices; q0 += 16) {  // 16 slices' loads in flight, added in slice order
      float p[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) p[q] = q0 + q < hslices ? hpart[(long)(q0 + q) * H + k] : 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (q0 + q < hslices) sacc += p[q];
    }
    const float hv = sigmoidf_ref((hb ? hb[k] : 0.f) + sacc);
    hs[threadIdx.x] = hv;
    if (blockIdx.x == 0) h[k] = hv;
  }
  __syncthreads();
  float acc = 0.f;
  if (c < N) {
#pragma unroll 4
    for (int k = k0 + w; k < k1; k += 4) acc += hs[k - k0] * Wo[(long)k * ldw + c];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && c < N) opart[(long)blockIdx.y * N + c] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

__global__ __launch_bounds__(256) void rnn_out_stats_kernel(const float* __restrict__ opart, int slices, int N,
                                                            const float* __restrict__ b, float* __restrict__ z,
                                                            double* __restrict__ smx) {
  __shared__ float smax[4];
  __shared__ double ssum[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int cc = min(c, N - 1);
  float p[8];
  float sacc = 0.f;
  for (int k0 = 0; k0 < slices; k0 += 8) {  // 8 slices' loads in flight, added in slice order
#pragma unroll
    for (int q = 0; q < 8; ++q) p[q] = k0 + q < slices ? opart[(long)(k0 + q) * N + cc] : 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (k0 + q < slices) sacc += p[q];
  }
  const float a = c < N ? (b ? b[c] : 0.f) + sacc : -1e30f;
  if (z && c < N) z[c] = a;
  float m = wave_max(a);
  if (lane == 0) smax[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
  const double ws = wave_sum_d(c < N ? (double)fast_exp(a - m) : 0.0);
  if (lane == 0) ssum[wv] = ws;
  __syncthreads();
  if (threadIdx.x == 0) {
    smx[2 * blockIdx.x] = (double)m;
    smx[2 * blockIdx.x + 1] = ssum[0] + ssum[1] + ssum[2] + ssum[3];
  }
}

// The output side's first two launches in one: every workgroup finishes ALL of h (the recurrent
// sigmoid from the split-K partials, rnn_out_partial_kernel's order; workgroup 0 stores it), then the
// complete z of its 64 columns -- 16 waves over interleaved k (wave w: k = w, w + 16, ...; 32 loads
// of Wo in flight per lane at H = 512), wave sums added in wave order -- and the pair {max z, sum
// exp(z - max)} of those columns (rnn_out_stats_kernel's arithmetic per 64 instead of 256 columns).
// No output partials, no stats launch: ceil(N / 64) <= 64 pairs for rnn_out_bwd_kernel.
constexpr int GV_FULL_MAXH = 2048;
__global__ __launch_bounds__(1024) void rnn_out_full_kernel(const float* __restrict__ hpart, int hslices,
                                                            const float* __restrict__ hb, float* __restrict__ h,
                                                            int H, const float* __restrict__ Wo, long ldw, int N,
                                                            const float* __restrict__ bo, float* __restrict__ z,
                                                            double* __restrict__ smx, const RnnCorr cr) {
  __shared__ float hs[GV_FULL_MAXH];
  __shared__ float red[16][64];
  __shared__ float sdot[GV_DOTS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nout_blocks = (N + 63) / 64;
  if (cr.on && (int)blockIdx.x >= nout_blocks) {
    // ---- the pending recurrent update (rnn_update_kernel's per-element arithmetic and step order; the bias is
    // the output blocks' business below), 4 consecutive elements of a row a thread.  Every load is issued before
    // the first is used -- the row's history values and the 4 columns' d_i at clamped step indices (unconditional:
    // a predicated load is a branch, and branches serialise the round trips), W's 4 elements -- then the sums.
    const long e0 = ((long)(blockIdx.x - nout_blocks) * 1024 + threadIdx.x) * 4;
    const int k = (int)(e0 / H), c0 = (int)(e0 % H);
    if (k >= cr.rows) return;
    float hk[GV_UPD_MAX];
    f32x4 dv[GV_UPD_MAX];
#pragma unroll
    for (int i = 0; i < GV_UPD_MAX; ++i) {
      const int ii = min(i, cr.steps - 1);
      int r = cr.head + ii;
      r = r >= cr.R ? r - cr.R : r;
      hk[i] = cr.hist[(long)r * cr.ldh + k];
      dv[i] = *reinterpret_cast<const f32x4*>(cr.D + (long)ii * cr.ldd + c0);
    }
    float* wrow = cr.W + (long)k * cr.ldw;
    const f32x4 wv = *reinterpret_cast<const f32x4*>(wrow + c0);
    f32x4 out;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < GV_UPD_MAX; ++i)
        if (i < cr.steps) acc = __fmaf_rn(-cr.lr * hk[i], dv[i][j], acc);
      const float corr = __fmaf_rn(-cr.lr * cr.wc, wv[j], acc);
      out[j] = corr + wv[j];
    }
    st_wt(tile_rsrc(wrow), c0, out);  // write-through: no dirty W lines left for the kernel-end release
    return;
  }
  const int c = blockIdx.x * 64 + lane, cc = min(c, N - 1);
  // ONE round of loads before anything waits: the first 32 rows per lane of the column block's Wo, (cr.on, threads
  // < GV_DOTS) the first 16 slices' partial dots, then per unit k the pending update's d_i at clamped step indices,
  // the bias operands and the recurrent partial sums.  The dots are summed and shared only after the units' sums,
  // so their round trip overlaps the others instead of preceding them.
  float wv[32];
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const int k = w + 16 * q;
    wv[q] = k < H ? Wo[(long)k * ldw + cc] : 0.f;
  }
  const bool dots = cr.on && threadIdx.x < GV_DOTS;
  float pd[16];
  if (dots) {
#pragma unroll
    for (int q = 0; q < 16; ++q) pd[q] = cr.dpart[(long)min(q, hslices - 1) * GV_DOTS + threadIdx.x];
  }
  constexpr int KPT = GV_FULL_MAXH / 1024;  // units per thread
  float sacc[KPT], g[KPT], dk[KPT][GV_UPD_MAX], hbk[KPT];
#pragma unroll
  for (int u = 0; u < KPT; ++u) {
    const int k = threadIdx.x + 1024 * u;
    if (k >= H) break;
    float cbk = 0.f;
    if (cr.on) {
#pragma unroll
      for (int i = 0; i < GV_UPD_MAX; ++i) dk[u][i] = cr.D[(long)min(i, cr.steps - 1) * cr.ldd + k];
      cbk = cr.cb[k];
    }
    hbk[u] = hb ? hb[k] : 0.f;
    sacc[u] = 0.f;
    for (int q0 = 0; q0 < hslices; q0 += 16) {  // 16 slices' loads in flight, added in slice order
      float p[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) p[q] = q0 + q < hslices ? hpart[(long)(q0 + q) * H + k] : 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (q0 + q < hslices) sacc[u] += p[q];
    }
    if (cr.on) {
      // the pending bias update (rnn_update_kernel's chain)
      g[u] = __fmaf_rn(-cr.lr, dk[u][0], cr.mmt * cbk);
#pragma unroll
      for (int i = 1; i < GV_UPD_MAX; ++i)
        if (i < cr.steps) g[u] = __fmaf_rn(-cr.lr, dk[u][i], g[u]);
    }
  }
  if (cr.on) {
    if (dots) {  // the dots, summed over the slices in slice order
      float d = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (q < hslices) d += pd[q];
      for (int q0 = 16; q0 < hslices; ++q0) d += cr.dpart[(long)q0 * GV_DOTS + threadIdx.x];
      sdot[threadIdx.x] = d;
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < KPT; ++u) {
    const int k = threadIdx.x + 1024 * u;
    if (k >= H) break;
    float hv;
    if (cr.on) {
      // the correction of the look-ahead product
      float a = 0.f;
      a = __fmaf_rn(-cr.lr * sdot[0], dk[u][0], a);
#pragma unroll
      for (int i = 1; i < GV_UPD_MAX; ++i)
        if (i < cr.steps) a = __fmaf_rn(-cr.lr * sdot[i], dk[u][i], a);
      const float bn = g[u] + hbk[u];
      if (blockIdx.x == 0) {
        cr.cbnext[k] = g[u];
        cr.bnext[k] = bn;
      }
      hv = sigmoidf_ref(bn + (__fmaf_rn(-cr.lr * cr.wc, sacc[u], sacc[u]) + a));
    } else {
      hv = sigmoidf_ref(hbk[u] + sacc[u]);
    }
    hs[k] = hv;
    if (blockIdx.x == 0) h[k] = hv;
  }
  __syncthreads();
  float acc = 0.f;
  for (int k0 = w; k0 < H; k0 += 16 * 32) {  // 32 rows of Wo per lane in flight
    if (k0 != w) {
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const int k = k0 + 16 * q;
        wv[q] = k < H ? Wo[(long)k * ldw + cc] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int k = k0 + 16 * q;
      if (k < H) acc += hs[k] * wv[q];
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0) {
    float t = red[0][lane];
#pragma unroll
    for (int q = 1; q < 16; ++q) t += red[q][lane];
    const float a = c < N ? (bo ? bo[c] : 0.f) + t : -1e30f;
    if (z && c < N) z[c] = a;
    const float m = wave_max(a);
    const double ws = wave_sum_d(c < N ? (double)fast_exp(a - m) : 0.0);
    if (lane == 0) {
      smx[2 * blockIdx.x] = (double)m;
      smx[2 * blockIdx.x + 1] = ws;
    }
  }
}

// WPR waves per weight row (1: rows of <= 1024 columns, a wave each; 4: a workgroup per row, so a
// 4000-column row has its 16 KB of W in flight at once and the row sums meet in LDS in wave order).
// Every load of a workgroup goes out in one round before the first is used -- the softmax pairs, the
// label, h_i, and (rows of <= 4 passes) the whole row of W, z and the momentum row at clamped addresses
// -- then the arithmetic in the per-pass order of the loop form.
template <int WPR>
__global__ __launch_bounds__(256) void rnn_out_bwd_kernel(
    const float* __restrict__ z, const double* __restrict__ smx, int G, const int* __restrict__ label,
    const float* __restrict__ h, int n_in, int n_out, float* __restrict__ W, long ldw, float* __restrict__ corrW,
    long ldc, float* __restrict__ b, float* __restrict__ cb, float scale, float mmt, float l2,
    float* __restrict__ yout, float* __restrict__ eout, float* __restrict__ eo, float* __restrict__ d,
    double* __restrict__ stats, unsigned long long* __restrict__ argkey, int row_blocks, int train,
    const RnnAhead ah) {
  __shared__ ArgMax sarg[4];
  __shared__ float racc[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int stat_blocks = (n_out + 255) / 256, xb = (int)blockIdx.x - row_blocks - stat_blocks;
  if (xb >= 0) {  // ---- RnnAhead: the recurrent bias copy, then the next frame's look-ahead blocks
    if (xb < ah.nbias) {
      const int k = xb * 256 + threadIdx.x;
      if (k < ah.H) {
        ah.cb[k] = ah.cbnext[k];
        ah.b[k] = ah.bnext[k];
      }
      return;
    }
    const int lb = xb - ah.nbias, nbx = (ah.H + 63) / 64;
    rnn_ahead_block(ah, lb % nbx, lb / nbx);
    return;
  }
  // the softmax normaliser from the pairs {m_g, s_g}: M = max m_g, S = sum s_g exp(m_g - M), every wave
  // reducing the G <= 64 pairs itself (lane g); their loads and the label's go out with the rest
  const int gl = min(lane, G - 1);  // clamped, unconditional: no branch between the loads
  const double mg_raw = smx[2 * gl], sg_raw = smx[2 * gl + 1];
  const int t0 = label[0];
  const float mg = lane < G ? (float)mg_raw : -1e30f;
  const double sg = lane < G ? sg_raw : 0.0;
  if ((int)blockIdx.x >= row_blocks) {  // bias / statistics workgroups: 256 columns each
    const int j = (blockIdx.x - row_blocks) * blockDim.x + threadIdx.x;
    const int jj = min(j, n_out - 1);
    const float zj = z[jj];
    const float cbj = (train && cb) ? cb[jj] : 0.f, bj = train ? b[jj] : 0.f;
    const float M = wave_max(mg);
    const float rsum = 1.f / (float)wave_sum_d(lane < G ? sg * (double)fast_exp(mg - M) : 0.0);
    const int t = t0 < n_out ? t0 : -1;  // out of range: an unlabeled frame, as the batched kernels
    ArgMax ay{-1e20f, 0x7fffffff};
    if (j < n_out) {
      const float yj = fast_exp(zj - M) * rsum;
      const float ej = yj - (j == t ? 1.f : 0.f);
      ay.v = yj;
      ay.i = j;
      if (yout) yout[j] = yj;
      if (eout) eout[j] = ej;
      if (j == t && stats) atomicAdd(stats, -(double)logf(fmaxf(yj, FLT_MIN)));
      if (train) {
        float g = ej;
        if (cb) {
          g = g + mmt * cbj;
          cb[j] = g;
        }
        b[j] = bj + scale * g;
      }
    }
    ay = wave_argmax(ay);
    if (lane == 0) sarg[wv] = ay;
    __syncthreads();
    if (threadIdx.x == 0 && argkey) {
      ArgMax a = sarg[0];
#pragma unroll
      for (int q = 1; q < 4; ++q) a = argmax_merge(a, sarg[q]);
      if (a.i < n_out) {
        const unsigned long long key =
            ((unsigned long long)__float_as_uint(fmaxf(a.v, 0.f)) << 32) | (unsigned long long)(0xffffffffu - (unsigned)a.i);
        atomicMax(argkey, key);
      }
    }
    return;
  }
  if (!train) return;
  constexpr int RPB = 4 / WPR;  // rows per workgroup
  const int i = blockIdx.x * RPB + wv / WPR, sub = wv % WPR;
  const bool live = i < n_in;
  const float xi = live ? h[i] : 0.f;
  float* row = W + (long)(live ? i : 0) * ldw;
  float* qrow = corrW ? corrW + (long)(live ? i : 0) * ldc : nullptr;
  auto upd = [&](float w, float ej, float* q) {
    float c = xi * ej;
    if (qrow) {
      c = c + mmt * *q;
      *q = c;
    }
    w = w + scale * c;
    return w + l2 * w;
  };
  constexpr int STEP = 256 * WPR;  // floats per pass of the row's waves
  constexpr int NP = 4;            // passes held in registers (n_out <= 4 STEP)
  const bool vec = (n_out & 3) == 0 && (ldw & 3) == 0 && (!qrow || (ldc & 3) == 0) &&
                   (((uintptr_t)row | (uintptr_t)z | (uintptr_t)qrow) & 15) == 0;
  float acc = 0.f;
  if (vec && n_out <= NP * STEP) {
    // the updated row (and momentum row) stored write-through: at 4000 outputs the launch rewrites 8-16 MB, which
    // plain stores would leave dirty for the kernel-end release to write back after the last workgroup
    const __amdgpu_buffer_rsrc_t wr = tile_rsrc(row), qr = tile_rsrc(qrow ? qrow : row);
    f32x4 a[NP], zv[NP], qv[NP];
    const float* qsrc = qrow ? qrow : row;  // unconditional (no branch in the round); unused without momentum
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int c = min((sub * 64 + lane) * 4 + p * STEP, n_out - 4);
      a[p] = *reinterpret_cast<const f32x4*>(row + c);
      zv[p] = *reinterpret_cast<const f32x4*>(z + c);
      qv[p] = *reinterpret_cast<const f32x4*>(qsrc + c);
    }
    const float M = wave_max(mg);
    const float rsum = 1.f / (float)wave_sum_d(lane < G ? sg * (double)fast_exp(mg - M) : 0.0);
    const int t = t0 < n_out ? t0 : -1;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int c = (sub * 64 + lane) * 4 + p * STEP;
      if (!live || c >= n_out) continue;
      float ev[4], q[4] = {qv[p][0], qv[p][1], qv[p][2], qv[p][3]};
#pragma unroll
      for (int k = 0; k < 4; ++k) ev[k] = fast_exp(zv[p][k] - M) * rsum - (c + k == t ? 1.f : 0.f);
      f32x4 w4 = a[p];
      acc += w4[0] * ev[0] + w4[1] * ev[1] + w4[2] * ev[2] + w4[3] * ev[3];
#pragma unroll
      for (int k = 0; k < 4; ++k) w4[k] = upd(w4[k], ev[k], &q[k]);
      st_wt(wr, c, w4);
      if (qrow) st_wt(qr, c, f32x4{q[0], q[1], q[2], q[3]});
    }
  } else {
    const float M = wave_max(mg);
    const float rsum = 1.f / (float)wave_sum_d(lane < G ? sg * (double)fast_exp(mg - M) : 0.0);
    const int t = t0 < n_out ? t0 : -1;
    auto err = [&](int c, float zc) { return fast_exp(zc - M) * rsum - (c == t ? 1.f : 0.f); };
    if (live && vec) {
#pragma unroll 2
      for (int c = (sub * 64 + lane) * 4; c < n_out; c += STEP) {
        f32x4 a = *reinterpret_cast<const f32x4*>(row + c);
        const f32x4 z4 = *reinterpret_cast<const f32x4*>(z + c);
        f32x4 q4 = qrow ? *reinterpret_cast<const f32x4*>(qrow + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        float ev[4], q[4] = {q4[0], q4[1], q4[2], q4[3]};
#pragma unroll
        for (int k = 0; k < 4; ++k) ev[k] = err(c + k, z4[k]);
        acc += a[0] * ev[0] + a[1] * ev[1] + a[2] * ev[2] + a[3] * ev[3];
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = upd(a[k], ev[k], &q[k]);
        *reinterpret_cast<f32x4*>(row + c) = a;
        if (qrow) *reinterpret_cast<f32x4*>(qrow + c) = f32x4{q[0], q[1], q[2], q[3]};
      }
    } else if (live) {
      for (int c = sub * 64 + lane; c < n_out; c += 64 * WPR) {
        const float w = row[c], ej = err(c, z[c]);
        acc += w * ej;
        row[c] = upd(w, ej, qrow ? qrow + c : nullptr);
      }
    }
  }
  acc = wave_sum(acc);
  if constexpr (WPR > 1) {
    if (lane == 0) racc[wv] = acc;
    __syncthreads();
    acc = ((racc[0] + racc[1]) + racc[2]) + racc[3];
  }
  if (live && sub == 0 && lane == 0) {
    if (eo) eo[i] = acc;
    if (d) d[i] = acc * (xi * (1.f - xi));
  }
}

__global__ __launch_bounds__(256) void argmax_correct_kernel(const unsigned long long* __restrict__ keys,
                                                             const int* __restrict__ labels, int T, int N,
                                                             double* __restrict__ stats) {
  __shared__ double red[4];
  double n = 0.0;
  for (int f = threadIdx.x; f < T; f += 256) {
    const int t = labels[f];
    const int des = (t >= 0 && t < N) ? t : 0;
    const unsigned idx = 0xffffffffu - (unsigned)(keys[f] & 0xffffffffull);
    n += (keys[f] != 0ull && idx == (unsigned)des) ? 1.0 : 0.0;
  }
  n = wave_sum_d(n);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(stats + 1, red[0] + red[1] + red[2] + red[3]);
}

}  // namespace tnetk

using namespace tnetk;

extern "C" int tnet_gemv_rowvec_partial(const float* v0, int K0, const float* v1, int K1, float* vout,
                                        const float* W, int ldw, int N, float* partial, void* stream) {
  const int K = K0 + K1;
  if (K0 < 0 || K1 < 0 || K <= 0 || N <= 0 || ldw < N || (K0 && !v0) || (K1 && !v1) || !W || !partial)
    return TNET_ERR_ARG;
  gemv_rowvec_partial_k<false><<<dim3(cdiv(N, 64), cdiv(K, GV_KSLICE)), 256, 0, (hipStream_t)stream>>>(
      v0, K0, v1, K, const_cast<float*>(W), ldw, N, partial, vout, RnnPendingUpdate{});
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_rnn_out_partial(const float* hpart, int hslices, const float* hb, float* h, int H,
                                    const float* Wo, int ldwo, int N, float* opart, void* stream) {
  if (hslices <= 0 || H <= 0 || N <= 0 || ldwo < N || !hpart || !h || !Wo || !opart) return TNET_ERR_ARG;
  rnn_out_partial_kernel<<<dim3(cdiv(N, 64), cdiv(H, GV_KSLICE)), 256, 0, (hipStream_t)stream>>>(
      hpart, hslices, hb, h, H, Wo, ldwo, N, opart);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_rnn_out_full(const float* hpart, int hslices, const float* hb, float* h, int H, const float* Wo,
                                 int ldwo, int N, const float* bo, float* z, double* smx, void* stream) {
  if (hslices <= 0 || H <= 0 || N <= 0 || ldwo < N || !hpart || !h || !Wo || !smx) return TNET_ERR_ARG;
  if (H > GV_FULL_MAXH || cdiv(N, 64) > 64) return TNET_ERR_UNSUPPORTED;
  rnn_out_full_kernel<<<cdiv(N, 64), 1024, 0, (hipStream_t)stream>>>(hpart, hslices, hb, h, H, Wo, ldwo, N, bo, z, smx,
                                                                      RnnCorr{});
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_gemv_rowvec_partial_update(const float* v0, int K0, const float* v1, int K1, float* vout,
                                               float* W, int ldw, int N, float* partial, const float* hist, int ldh,
                                               int head, int R, const float* D, int ldd, int steps, float* b,
                                               float* corr_b, float lr, float mmt, float wc, void* stream) {
  const int K = K0 + K1;
  if (K0 < 0 || K1 < 0 || K <= 0 || N <= 0 || ldw < N || (K0 && !v0) || (K1 && !v1) || !W || !partial || !hist ||
      !D || !b || !corr_b || steps <= 0 || head < 0 || head >= R || ldh < K || ldd < N)
    return TNET_ERR_ARG;
  if (steps > GV_UPD_MAX || steps >= R) return TNET_ERR_UNSUPPORTED;  // the push must not hit a row the update reads
  const RnnPendingUpdate u{hist, ldh, head, R, D, ldd, steps, b, corr_b, lr, mmt, wc};
  const dim3 grid(cdiv(N, 64), cdiv(K, GV_KSLICE));
  hipStream_t st = (hipStream_t)stream;
  switch (steps) {
#define TNET_UPD_CASE(n) \
  case n: gemv_rowvec_partial_k<true, n><<<grid, 256, 0, st>>>(v0, K0, v1, K, W, ldw, N, partial, vout, u); break;
    TNET_UPD_CASE(1) TNET_UPD_CASE(2) TNET_UPD_CASE(3) TNET_UPD_CASE(4) TNET_UPD_CASE(5) TNET_UPD_CASE(6)
    TNET_UPD_CASE(7) TNET_UPD_CASE(8) TNET_UPD_CASE(9)
#undef TNET_UPD_CASE
    default: return TNET_ERR_UNSUPPORTED;
  }
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_rnn_out_stats(const float* opart, int H, int N, const float* bo, float* z, double* smx,
                                  void* stream) {
  if (H <= 0 || N <= 0 || !opart || !smx) return TNET_ERR_ARG;
  rnn_out_stats_kernel<<<cdiv(N, 256), 256, 0, (hipStream_t)stream>>>(opart, cdiv(H, GV_KSLICE), N, bo, z, smx);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_rnn_out_bwd_update(const float* z, const double* smx, int pairs, int N, const int* label,
                                       const float* h, int H, float* Wo, int ldwo, float* corrWo, int ldc, float* bo,
                                       float* corr_bo, float scale, float mmt, float l2, float* y, float* e, float* eo,
                                       float* d, double* stats, unsigned long long* argkey, int train, void* stream) {
  if (N <= 0 || H <= 0 || !z || !smx || !label || !h || (train && (!Wo || !bo || ldwo < N)) ||
      (train && mmt != 0.f && (!corrWo || !corr_bo || ldc < N)) || pairs < 1)
    return TNET_ERR_ARG;
  if (pairs > 64) return TNET_ERR_UNSUPPORTED;  // one pair per lane in rnn_out_bwd_kernel's normaliser
  const bool wide = N > 1024;  // a workgroup per weight row
  const int row_blocks = train ? (wide ? H : cdiv(H, 4)) : 0;
  const dim3 grid(row_blocks + cdiv(N, 256));
  hipStream_t st = (hipStream_t)stream;
  if (wide)
    rnn_out_bwd_kernel<4><<<grid, 256, 0, st>>>(z, smx, pairs, label, h, H, N, Wo, ldwo,
                                                mmt != 0.f ? corrWo : nullptr, ldc, bo, mmt != 0.f ? corr_bo : nullptr,
                                                scale, mmt, l2, y, e, eo, d, stats, argkey, row_blocks, train,
                                                RnnAhead{});
  else
    rnn_out_bwd_kernel<1><<<grid, 256, 0, st>>>(z, smx, pairs, label, h, H, N, Wo, ldwo,
                                                mmt != 0.f ? corrWo : nullptr, ldc, bo, mmt != 0.f ? corr_bo : nullptr,
                                                scale, mmt, l2, y, e, eo, d, stats, argkey, row_blocks, train,
                                                RnnAhead{});
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

// the look-ahead frame chain (RnnAhead / RnnCorr above; CuRecurrentTrainer::TrainFrameFused)
extern "C" int tnet_rnn_out_full_ahead(const float* hpart, int hslices, const float* hb, float* h, int H,
                                       const float* Wo, int ldwo, int N, const float* bo, float* z, double* smx,
                                       const float* dpart, const float* D, int ldd, int steps, float lr, float mmt,
                                       float wc, const float* cb, float* bnext, float* cbnext, float* W, int ldw,
                                       int rows, const float* hist, int ldh, int head, int R, void* stream) {
  if (hslices <= 0 || H <= 0 || N <= 0 || ldwo < N || !hpart || !hb || !h || !Wo || !smx || !dpart || !D || !cb ||
      !bnext || !cbnext || !W || !hist || steps <= 0 || ldd < H || ldw < H || ldh < rows || head < 0 || head >= R ||
      rows <= 0)
    return TNET_ERR_ARG;
  if (H > GV_FULL_MAXH || cdiv(N, 64) > 64 || steps > GV_UPD_MAX || steps >= R || (H & 3) ||
      hslices != cdiv(rows, GV_KSLICE) || (ldw & 3) || (ldd & 3) || ((uintptr_t)W & 15) || ((uintptr_t)D & 15))
    return TNET_ERR_UNSUPPORTED;
  RnnCorr cr{};
  cr.on = 1;
  cr.dpart = dpart; cr.D = D; cr.ldd = ldd; cr.steps = steps; cr.lr = lr; cr.mmt = mmt; cr.wc = wc;
  cr.cb = cb; cr.bnext = bnext; cr.cbnext = cbnext;
  cr.nupd = (int)cdiv((long)rows * H, 4096);
  cr.W = W; cr.ldw = ldw; cr.rows = rows; cr.hist = hist; cr.ldh = ldh; cr.head = head; cr.R = R;
  rnn_out_full_kernel<<<cdiv(N, 64) + cr.nupd, 1024, 0, (hipStream_t)stream>>>(hpart, hslices, hb, h, H, Wo, ldwo, N,
                                                                               bo, z, smx, cr);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_rnn_out_bwd_update_ahead(const float* z, const double* smx, int pairs, int N, const int* label,
                                             const float* h, int H, float* Wo, int ldwo, float* corrWo, int ldc,
                                             float* bo, float* corr_bo, float scale, float mmt, float l2, float* e,
                                             float* eo, float* d, double* stats, unsigned long long* argkey,
                                             const float* bnext, const float* cbnext, float* b, float* cb,
                                             const float* x_next, int nIn, const float* W, int ldw, float* partial,
                                             float* dpart, float* vout, const float* hist, int ldh, int head, int R,
                                             int steps, void* stream) {
  // tnet_rnn_out_bwd_update (train) + the recurrent bias copy (bnext != NULL) + the next frame's look-ahead
  // (x_next != NULL: v = [x_next, h], K = nIn + H)
  if (N <= 0 || H <= 0 || !z || !smx || !label || !h || !Wo || !bo || ldwo < N ||
      (mmt != 0.f && (!corrWo || !corr_bo || ldc < N)) || pairs < 1)
    return TNET_ERR_ARG;
  if (bnext && (!cbnext || !b || !cb)) return TNET_ERR_ARG;
  const int K = nIn + H;
  if (x_next && (!W || !partial || !dpart || !vout || !hist || nIn <= 0 || ldw < H || ldh < K || head < 0 ||
                 head >= R || steps <= 0))
    return TNET_ERR_ARG;
  if (pairs > 64 || (x_next && (steps > GV_UPD_MAX || steps >= R))) return TNET_ERR_UNSUPPORTED;
  RnnAhead ah{};
  ah.H = H;
  if (bnext) {
    ah.nbias = cdiv(H, 256);
    ah.bnext = bnext; ah.cbnext = cbnext; ah.b = b; ah.cb = cb;
  }
  if (x_next) {
    ah.nlook = cdiv(H, 64) * cdiv(K, GV_KSLICE);
    ah.v0 = x_next; ah.K0 = nIn; ah.v1 = h; ah.K = K; ah.W = W; ah.ldw = ldw; ah.partial = partial;
    ah.dpart = dpart; ah.vout = vout; ah.hist = hist; ah.ldh = ldh; ah.head = head; ah.R = R; ah.steps = steps;
  }
  const bool wide = N > 1024;
  const int row_blocks = wide ? H : cdiv(H, 4);
  const dim3 grid(row_blocks + cdiv(N, 256) + ah.nbias + ah.nlook);
  hipStream_t st = (hipStream_t)stream;
  float* cw = mmt != 0.f ? corrWo : nullptr;
  float* cbo = mmt != 0.f ? corr_bo : nullptr;
  if (wide)
    rnn_out_bwd_kernel<4><<<grid, 256, 0, st>>>(z, smx, pairs, label, h, H, N, Wo, ldwo, cw, ldc, bo, cbo, scale, mmt,
                                                l2, nullptr, e, eo, d, stats, argkey, row_blocks, 1, ah);
  else
    rnn_out_bwd_kernel<1><<<grid, 256, 0, st>>>(z, smx, pairs, label, h, H, N, Wo, ldwo, cw, ldc, bo, cbo, scale, mmt,
                                                l2, nullptr, e, eo, d, stats, argkey, row_blocks, 1, ah);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_argmax_correct(const unsigned long long* keys, const int* labels, int T, int N, double* stats,
                                   void* stream) {
  if (T < 0 || N <= 0 || (T && (!keys || !labels || !stats))) return TNET_ERR_ARG;
  if (!T) return TNET_OK;
  argmax_correct_kernel<<<1, 256, 0, (hipStream_t)stream>>>(keys, labels, T, N, stats);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_affine_update_row(const float* x, int n_in, const float* e, int n_out, float* W, int ldw,
                                      float* corrW, int ldc, float* b, float* corr_b, float scale, float mmt,
                                      float l2, void* stream) {
  if (n_in <= 0 || n_out <= 0 || !x || !e || !W || !b || ldw < n_out || (corrW && ldc < n_out) ||
      (mmt != 0.f && (!corrW || !corr_b)))
    return TNET_ERR_ARG;
  affine_update_row_kernel<<<dim3(cdiv(n_out, 256), n_in + 1), 256, 0, (hipStream_t)stream>>>(
      x, n_in, e, n_out, W, ldw, corrW, ldc, b, mmt != 0.f ? corr_b : nullptr, scale, mmt, l2);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_affine_bwd_update_row(const float* x, int n_in, const float* e, int n_out, float* W, int ldw,
                                          float* corrW, int ldc, float* b, float* corr_b, float scale, float mmt,
                                          float l2, float* e_out, const float* s, float* d_out, void* stream) {
  if (n_in <= 0 || n_out <= 0 || !x || !e || !W || !b || ldw < n_out || (corrW && ldc < n_out) ||
      (mmt != 0.f && (!corrW || !corr_b)) || (d_out && !s))
    return TNET_ERR_ARG;
  const int row_blocks = cdiv((long)n_in * 64, 256);
  affine_bwd_update_row_kernel<<<row_blocks + cdiv(n_out, 256), 256, 0, (hipStream_t)stream>>>(
      x, n_in, e, n_out, W, ldw, mmt != 0.f ? corrW : nullptr, ldc, b, mmt != 0.f ? corr_b : nullptr, scale, mmt,
      l2, e_out, s, d_out, row_blocks);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" long tnet_gemv_workspace(int K, int N) { return (long)cdiv(K, GV_KSLICE) * (N > 0 ? N : 1) * 4; }

extern "C" int tnet_gemv_rowvec(const float* v, int K, const float* W, int ldw, const float* b, float* y, int N,
                                int act, void* workspace, void* stream) {
  if (K <= 0 || N <= 0 || ldw < N || !v || !W || !y || !workspace || act < 0 || act > 1) return TNET_ERR_ARG;
  return tnet_gemv_rowvec_cat(v, K, nullptr, 0, nullptr, W, ldw, b, y, N, act, workspace, stream);
}

extern "C" int tnet_gemv_rowvec_cat(const float* v0, int K0, const float* v1, int K1, float* vout, const float* W,
                                    int ldw, const float* b, float* y, int N, int act, void* workspace,
                                    void* stream) {
  const int K = K0 + K1;
  if (K0 < 0 || K1 < 0 || K <= 0 || N <= 0 || ldw < N || (K0 && !v0) || (K1 && !v1) || !W || !y || !workspace ||
      act < 0 || act > 1)
    return TNET_ERR_ARG;
  const int slices = cdiv(K, GV_KSLICE);
  float* part = (float*)workspace;
  hipStream_t st = (hipStream_t)stream;
  gemv_rowvec_partial_k<false><<<dim3(cdiv(N, 64), slices), 256, 0, st>>>(v0, K0, v1, K, const_cast<float*>(W), ldw,
                                                                          N, part, vout, RnnPendingUpdate{});
  TNET_LAUNCH_CHECK();
  gemv_rowvec_final<<<cdiv(N, 256), 256, 0, st>>>(part, slices, N, b, y, act);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_gemv_rowvec_softmax_xent(const float* v, int K, const float* W, int ldw, const float* b,
                                             float* z, float* y, float* e, int N, const int* label, double* stats,
                                             void* workspace, void* stream) {
  if (K <= 0 || N <= 0 || ldw < N || !v || !W || !label || !workspace) return TNET_ERR_ARG;
  if (N > GV_SMX_MAX) return TNET_ERR_UNSUPPORTED;
  const int slices = cdiv(K, GV_KSLICE);
  float* part = (float*)workspace;
  hipStream_t st = (hipStream_t)stream;
  gemv_rowvec_partial_k<false><<<dim3(cdiv(N, 64), slices), 256, 0, st>>>(v, K, nullptr, K, const_cast<float*>(W), ldw,
                                                                          N, part, nullptr, RnnPendingUpdate{});
  TNET_LAUNCH_CHECK();
  gemv_softmax_xent_final<<<1, 256, 0, st>>>(part, slices, N, b, z, y, e, label, stats);
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
