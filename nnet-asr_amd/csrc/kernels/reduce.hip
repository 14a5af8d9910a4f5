// reduce.hip -- row / column reductions of the TNet path on gfx950:
//   * column sums (bias gradient; _add_col_sum / _add_col_sum_reduce, cukernels.cu:147-187) as a
//     deterministic two-stage reduction: fp32 partials over fixed row slabs, combined in fp64;
//   * fused softmax + cross-entropy + error + frame accuracy, one wavefront per row
//     (_softmax / _softmax_reduce / _check_class / _log_elem / _mul_elem, cukernels.cu:131-483,
//     driven by CuCrossEntropy::Evaluate, cuObjectiveFunction.cc:50-83).  The reference runs
//     one THREAD per row with three serial passes for rows > 256 columns; here the row is held
//     in registers (16 B per lane per step) and every reduction is a 64-lane butterfly.
#include <float.h>

#include "kcommon.h"
#include "rbm_stats.h"

namespace tnetk {

// partial[s][c] = sum of rows of slab s in column c (fixed order: row sub-group w takes rows
// r0+w, r0+w+4, ...; the 4 sub-group sums are added in order)
template <bool V4>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ M, TnetMatrixDim d,
                                                             float* __restrict__ partial, int slabs, int neg_from,
                                                             long ldp) {
  __shared__ float red[CS_WAVES * CS_COLS * (V4 ? 4 : 1)];
  colsum_partial_block<V4>(M, d, partial, slabs, neg_from, ldp, blockIdx.x, blockIdx.y, red);
}

// mode 0: v = alpha*sum + beta*v ; mode 1: bias update (c = sum + mmt*corr; b += scale*c; corr=c)
// mode 2: grad_out = sum ; mode 3: RBM bias update (c = mmt*corr + scale*sum; corr = c; b += c)
__global__ __launch_bounds__(64) void colsum_final_kernel(const float* __restrict__ partial, int slabs, int cols,
                                                           int mode, float alpha, float beta, float* __restrict__ v,
                                                           float* __restrict__ corr, float scale, float mmt) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < cols; c += gridDim.x * blockDim.x) {
    double s = 0.0;
#pragma unroll 8
    for (int k = 0; k < slabs; ++k) s += (double)partial[(long)k * cols + c];
    if (mode == 0) {
      v[c] = (float)(alpha * s + (beta == 0.f ? 0.0 : (double)beta * v[c]));
    } else if (mode == 1) {
      float g = (float)s;
      if (corr) {
        g = g + mmt * corr[c];
        corr[c] = g;
      }
      v[c] = v[c] + scale * g;
    } else if (mode == 3) {
      const float g = mmt * corr[c] + scale * (float)s;
      corr[c] = g;
      v[c] = v[c] + g;
    } else {
      v[c] = (float)s;
    }
  }
}

// internal fallback workspace (single device, not thread-safe; the C++ layer always passes one)
static float* g_ws = nullptr;
static long g_ws_bytes = 0;
static float* get_ws(long bytes) {
  if (bytes > g_ws_bytes) {
    if (g_ws) (void)hipFree(g_ws);
    if (hipMalloc(&g_ws, bytes) != hipSuccess) { g_ws = nullptr; g_ws_bytes = 0; return nullptr; }
    g_ws_bytes = bytes;
  }
  return g_ws;
}

static int colsum_run(const float* M, TnetMatrixDim d, void* workspace, hipStream_t st, int mode, float alpha,
                      float beta, float* v, float* corr, float scale, float mmt, int neg_from = 0x7fffffff) {
  if (d.rows < 0 || d.cols < 0 || d.stride < d.cols) return TNET_ERR_ARG;
  if (d.cols == 0) return TNET_OK;
  const int slabs = cs_slabs(d.rows);
  float* ws = workspace ? (float*)workspace : get_ws((long)slabs * d.cols * 4);
  if (!ws) return TNET_ERR_RUNTIME;
  if (d.rows > 0) {
    const bool v4 = (d.cols & 3) == 0 && (d.stride & 3) == 0 && ((uintptr_t)M & 15) == 0;
    if (v4)
      colsum_partial_kernel<true><<<dim3(cdiv(d.cols, CS_COLS * 4), slabs), 256, 0, st>>>(M, d, ws, slabs,
                                                                                         neg_from, d.cols);
    else
      colsum_partial_kernel<false><<<dim3(cdiv(d.cols, CS_COLS), slabs), 256, 0, st>>>(M, d, ws, slabs, neg_from,
                                                                                      d.cols);
    TNET_LAUNCH_CHECK();
  } else {
    if (hipMemsetAsync(ws, 0, (size_t)slabs * d.cols * 4, st) != hipSuccess) return TNET_ERR_RUNTIME;
  }
  // one 64-lane wave per 64 columns: enough workgroups to spread the slab reads over many CUs
  colsum_final_kernel<<<cdiv(d.cols, 64), 64, 0, st>>>(ws, slabs, d.cols, mode, alpha, beta, v, corr, scale, mmt);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

// ---------------------------------------------------------------------------------------------
// softmax / cross-entropy, one wave per row
// ---------------------------------------------------------------------------------------------
constexpr int SX_MAXV4 = 16;  // row held in registers up to 16 float4 per lane = 4096 columns



// KIND 0: class-id labels; KIND 1: dense targets D.  Z == nullptr: Y already holds softmax output.
template <int KIND>
__global__ __launch_bounds__(256) void softmax_xent_kernel(const float* __restrict__ Z, TnetMatrixDim d,
                                                           const int* __restrict__ labels,
                                                           const float* __restrict__ D, int strideD,
                                                           float* __restrict__ Y, int strideY,
                                                           float* __restrict__ E, int strideE,
                                                           double* __restrict__ stats, int vec4) {
  __shared__ double red[2][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= d.rows) {
    if (lane == 0) { red[0][wv] = 0.0; red[1][wv] = 0.0; }
    __syncthreads();
    return;
  }
  const int N = d.cols;
  const float* src = Z ? Z + (long)row * d.stride : Y + (long)row * strideY;
  const bool cached = vec4 && N <= SX_MAXV4 * 256;
  // a class id outside [0, N) is treated as an unlabeled row (the host intake rejects one, CheckLabels);
  // loaded first, in flight with the row's values instead of a dependent trip after the reductions
  int t = (KIND == 0) ? labels[row] : -1;
  if (t >= N) t = -1;

  // ---- pass 1: max
  f32x4 rv[SX_MAXV4];
  float m = -1e20f;
  if (cached) {
#pragma unroll
    for (int j = 0; j < SX_MAXV4; ++j) {
      const int c = j * 256 + lane * 4;
      f32x4 x = {-1e30f, -1e30f, -1e30f, -1e30f};
      if (c < N) x = *reinterpret_cast<const f32x4*>(src + c);
      rv[j] = x;
      m = fmaxf(m, fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])));
    }
  } else {
    for (int c = lane; c < N; c += 64) m = fmaxf(m, src[c]);
  }
  m = wave_max(m);

  // ---- pass 2: sum of exp (only when normalising logits)
  float inv = 1.f;
  double dsum = 0.0;
  if (Z) {
    float s = 0.f;
    if (cached) {
#pragma unroll
      for (int j = 0; j < SX_MAXV4; ++j) {
        const int c = j * 256 + lane * 4;
        if (c < N) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float e = fast_exp(rv[j][k] - m);
            rv[j][k] = e;
            s += e;
          }
        }
      }
    } else {
      for (int c = lane; c < N; c += 64) s += fast_exp(src[c] - m);
    }
    dsum = wave_sum_d((double)s);
  }
  const float sum = (float)dsum;
  const float rsum = 1.f / sum;  // one division per row; y = e * (1/sum)

  // ---- pass 3: y, error, argmax, xent
  ArgMax ay{-1e20f, 0x7fffffff}, ad{-1e20f, 0x7fffffff};
  double xent = 0.0;
  float ytl = 0.f;  // KIND 0: the y written for column t, on the lane that owns t
  float* yrow = Y ? Y + (long)row * strideY : nullptr;
  float* erow = E ? E + (long)row * strideE : nullptr;
  const float* drow = (KIND == 1) ? D + (long)row * strideD : nullptr;
  auto visit = [&](int c, float y) {
    float dv;
    if (KIND == 0) {
      dv = (c == t) ? 1.f : 0.f;
      if (c == t) ytl = y;
    } else {
      dv = drow[c];
    }
    if (y > ay.v) { ay.v = y; ay.i = c; }
    if (KIND == 1 && dv > ad.v) { ad.v = dv; ad.i = c; }
    if (KIND == 1 && dv != 0.f) xent -= (double)dv * (double)logf(fmaxf(y, FLT_MIN));
    return dv;
  };
  if (cached) {
#pragma unroll
    for (int j = 0; j < SX_MAXV4; ++j) {
      const int c = j * 256 + lane * 4;
      if (c < N) {
        f32x4 y, e;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          y[k] = Z ? rv[j][k] * rsum : rv[j][k];
          e[k] = y[k] - visit(c + k, y[k]);
        }
        if (yrow && Z) *reinterpret_cast<f32x4*>(yrow + c) = y;
        if (erow) *reinterpret_cast<f32x4*>(erow + c) = e;
      }
    }
  } else {
    for (int c = lane; c < N; c += 64) {
      const float y = Z ? fast_exp(src[c] - m) * rsum : src[c];
      const float dv = visit(c, y);
      if (yrow && Z) yrow[c] = y;
      if (erow) erow[c] = y - dv;
    }
  }
  ay = wave_argmax(ay);
  int des;
  if (KIND == 0) {
    des = t >= 0 ? t : 0;  // all-zero target row: first max of zeros is column 0
  } else {
    ad = wave_argmax(ad);
    des = ad.i;
  }
  if (KIND == 1) xent = wave_sum_d(xent);
  // the label column's y from its owner lane's registers (the value a re-read of the row recomputes:
  // fast_exp(z_t - m) * rsum, or y_t itself) -- no dependent load at the row's end
  float yt = 0.f;
  if (KIND == 0) yt = __shfl(ytl, t < 0 ? 0 : cached ? (t & 255) >> 2 : t & 63, 64);
  if (lane == 0) {
    if (KIND == 0 && t >= 0) xent = -(double)logf(fmaxf(yt, FLT_MIN));
    red[0][wv] = xent;
    red[1][wv] = (ay.i == des) ? 1.0 : 0.0;
  }
  __syncthreads();
  if (threadIdx.x == 0 && stats) {
    const int slot = blockIdx.x % TNET_STATS_SLOTS;
    atomicAdd(stats + 2 * slot, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    atomicAdd(stats + 2 * slot + 1, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

__global__ __launch_bounds__(256) void mse_kernel(const float* __restrict__ Y, TnetMatrixDim d,
                                                  const float* __restrict__ D, int strideD, float* __restrict__ E,
                                                  int strideE, double* __restrict__ stats) {
  __shared__ double red[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  double s = 0.0;
  if (row < d.rows) {
    for (int c = lane; c < d.cols; c += 64) {
      const float e = Y[(long)row * d.stride + c] - D[(long)row * strideD + c];
      if (E) E[(long)row * strideE + c] = e;
      s += (double)(e * e);
    }
    s = wave_sum_d(s);
  }
  if (lane == 0) red[wv] = s;
  __syncthreads();
  if (threadIdx.x == 0 && stats)
    atomicAdd(stats + 2 * (blockIdx.x % TNET_STATS_SLOTS), red[0] + red[1] + red[2] + red[3]);
}

__global__ __launch_bounds__(256) void check_class_kernel(const float* __restrict__ out,
                                                          const float* __restrict__ des, int* __restrict__ match,
                                                          TnetMatrixDim d) {
  const int lane = threadIdx.x & 63;
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= d.rows) return;
  ArgMax a{-1e20f, 0x7fffffff}, b{-1e20f, 0x7fffffff};
  for (int c = lane; c < d.cols; c += 64) {
    const float x = out[(long)row * d.stride + c], y = des[(long)row * d.stride + c];
    if (x > a.v) { a.v = x; a.i = c; }
    if (y > b.v) { b.v = y; b.i = c; }
  }
  a = wave_argmax(a);
  b = wave_argmax(b);
  if (lane == 0) match[row] = (a.i == b.i) ? 1 : 0;
}

}  // namespace tnetk

using namespace tnetk;

extern "C" long tnet_col_sum_workspace(TnetMatrixDim d) { return (long)cs_slabs(d.rows) * (d.cols > 0 ? d.cols : 1) * 4; }

extern "C" int tnetF_add_col_sum(float alpha, const float* mat, float beta, float* vec, TnetMatrixDim d,
                                 void* workspace, void* stream) {
  return colsum_run(mat, d, workspace, (hipStream_t)stream, 0, alpha, beta, vec, nullptr, 0.f, 0.f);
}

extern "C" int tnet_colsum_slab_sums(const float* E, TnetMatrixDim dE, float* colpart, int ldcolpart, void* stream) {
  // the 32-row slab sums tnet_affine_bwd_colsum writes, for an E no backward GEMM produced (the top
  // layer's error from the softmax): same slab count (tnet_colsum_slabs), fp32 sums in row order
  if (dE.rows < 0 || dE.cols < 0 || dE.stride < dE.cols || !colpart || ldcolpart < dE.cols) return TNET_ERR_ARG;
  if (!dE.rows || !dE.cols) return TNET_OK;
  const int slabs = cs_slabs(dE.rows);
  if (slabs != cdiv(dE.rows, CS_ROWS)) return TNET_ERR_UNSUPPORTED;  // > 8192 rows: capped slab count
  const bool v4 = (dE.cols & 3) == 0 && (dE.stride & 3) == 0 && ((uintptr_t)E & 15) == 0;
  if (v4)
    colsum_partial_kernel<true><<<dim3(cdiv(dE.cols, CS_COLS * 4), slabs), 256, 0, (hipStream_t)stream>>>(
        E, dE, colpart, slabs, 0x7fffffff, ldcolpart);
  else
    colsum_partial_kernel<false><<<dim3(cdiv(dE.cols, CS_COLS), slabs), 256, 0, (hipStream_t)stream>>>(
        E, dE, colpart, slabs, 0x7fffffff, ldcolpart);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_bias_update(const float* E, TnetMatrixDim dE, float* b, float* corr_b, float* grad_out,
                                float scale, float mmt, void* workspace, void* stream) {
  if (mmt != 0.f && !corr_b && !grad_out) return TNET_ERR_ARG;
  if (grad_out) return colsum_run(E, dE, workspace, (hipStream_t)stream, 2, 1.f, 0.f, grad_out, nullptr, 0.f, 0.f);
  return colsum_run(E, dE, workspace, (hipStream_t)stream, 1, 1.f, 0.f, b, corr_b, scale, mmt);
}

extern "C" int tnet_rbm_bias_update(const float* M, TnetMatrixDim d, int neg_from, float* b, float* corr_b,
                                    float scale, float mmt, void* workspace, void* stream) {
  if (!b || !corr_b || neg_from < 0) return TNET_ERR_ARG;
  return colsum_run(M, d, workspace, (hipStream_t)stream, 3, 1.f, 0.f, b, corr_b, scale, mmt, neg_from);
}

// CD-1 statistics of one RBM step in ONE launch: rbm_stats.h (rbm_stats_block)
__global__ __launch_bounds__(256) void rbm_stats_kernel(const float* __restrict__ Vs, TnetMatrixDim dV,
                                                        const float* __restrict__ Hs, TnetMatrixDim dH, int B,
                                                        int nvb, float* __restrict__ vb, float* __restrict__ cvb,
                                                        float* __restrict__ hb, float* __restrict__ chb, float scale,
                                                        float mmt, double* __restrict__ stats, int nhb) {
  __shared__ __attribute__((aligned(16))) float smem[RS_SMEM_FLOATS];
  rbm_stats_block((int)blockIdx.x, smem, Vs, dV, Hs, dH, B, nvb, vb, cvb, hb, chb, scale, mmt, stats, nhb);
}

// Wide rows (1025..4096 columns, 16-B aligned), class-id targets, logits in Z: one 256-thread block
// per ROW, wave w holding 256-column chunks w, w+4, w+8, w+12 in registers; the row max / sum /
// argmax meet through LDS.  Four waves per row keep four times the loads in flight per row and a
// quarter of the exp / compare work per wave of the one-wave-per-row kernel (latency-bound there).
__device__ __forceinline__ void softmax_xent_row4(const float* __restrict__ Z, TnetMatrixDim d,
                                                  const int* __restrict__ labels, float* __restrict__ Y, int strideY,
                                                  float* __restrict__ E, int strideE, double* __restrict__ stats,
                                                  const int row) {
  constexpr int CPW = SX_MAXV4 / 4;  // chunks per wave
  __shared__ float smax[4];
  __shared__ double ssum[4];
  __shared__ ArgMax sarg[4];
  __shared__ float syt;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int N = d.cols;
  const float* src = Z + (long)row * d.stride;
  // the label first: its load is in flight with the row's, not a dependent trip after the reductions
  int t = labels[row];
  if (t >= N) t = -1;  // out of range: an unlabeled row (the host intake rejects one, CheckLabels)
  f32x4 rv[CPW];
  float m = -1e20f;
#pragma unroll
  for (int q = 0; q < CPW; ++q) {
    const int c = (wv + 4 * q) * 256 + lane * 4;
    f32x4 x = {-1e30f, -1e30f, -1e30f, -1e30f};
    if (c < N) x = *reinterpret_cast<const f32x4*>(src + c);
    rv[q] = x;
    m = fmaxf(m, fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])));
  }
  m = wave_max(m);
  if (lane == 0) smax[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < CPW; ++q) {
    const int c = (wv + 4 * q) * 256 + lane * 4;
    if (c < N) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float e = fast_exp(rv[q][k] - m);
        rv[q][k] = e;
        s += e;
      }
    }
  }
  const double ws = wave_sum_d((double)s);
  if (lane == 0) ssum[wv] = ws;
  __syncthreads();
  const float sum = (float)(ssum[0] + ssum[1] + ssum[2] + ssum[3]);
  const float rsum = 1.f / sum;
  float* yrow = Y ? Y + (long)row * strideY : nullptr;
  float* erow = E ? E + (long)row * strideE : nullptr;
  // write-through row stores (kcommon.h st_wt): E is 16 MB at 4000 senones, read next on other XCDs
  const __amdgpu_buffer_rsrc_t ry = tile_rsrc(yrow ? yrow : Z), re = tile_rsrc(erow ? erow : Z);
  ArgMax ay{-1e20f, 0x7fffffff};
#pragma unroll
  for (int q = 0; q < CPW; ++q) {
    const int c = (wv + 4 * q) * 256 + lane * 4;
    if (c < N) {
      f32x4 y, e;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        y[k] = rv[q][k] * rsum;
        if (y[k] > ay.v) { ay.v = y[k]; ay.i = c + k; }
        e[k] = y[k] - ((c + k == t) ? 1.f : 0.f);
        // the y written for column t, handed to thread 0 from the owning lane's registers (the same value
        // a re-read of the logit recomputes: fast_exp(z_t - m) * rsum, without that dependent load)
        if (c + k == t) syt = y[k];
      }
      if (yrow) st_wt(ry, c, y);
      if (erow) st_wt(re, c, e);
    }
  }
  ay = wave_argmax(ay);
  if (lane == 0) sarg[wv] = ay;
  __syncthreads();
  if (threadIdx.x == 0) {
    ArgMax a = sarg[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) a = argmax_merge(a, sarg[w]);
    const int des = t >= 0 ? t : 0;  // all-zero target row: first max of zeros is column 0
    double xent = 0.0;
    if (t >= 0) xent = -(double)logf(fmaxf(syt, FLT_MIN));
    if (stats) {
      const int slot = row % TNET_STATS_SLOTS;
      atomicAdd(stats + 2 * slot, xent);
      atomicAdd(stats + 2 * slot + 1, (a.i == des) ? 1.0 : 0.0);
    }
  }
}
__global__ __launch_bounds__(256) void softmax_xent_row4_kernel(const float* __restrict__ Z, TnetMatrixDim d,
                                                                const int* __restrict__ labels,
                                                                float* __restrict__ Y, int strideY,
                                                                float* __restrict__ E, int strideE,
                                                                double* __restrict__ stats) {
  softmax_xent_row4(Z, d, labels, Y, strideY, E, strideE, stats, (int)blockIdx.x);
}
static bool v4ok(const void* p, int stride) { return ((uintptr_t)p & 15) == 0 && (stride & 3) == 0; }

extern "C" int tnet_softmax_xent(const float* Z, TnetMatrixDim dZ, const int* labels, float* Y, int strideY, float* E,
                                 int strideE, double* stats, void* stream) {
  if (dZ.rows < 0 || dZ.cols <= 0 || !labels || (!Z && !Y)) return TNET_ERR_ARG;
  if (!dZ.rows) return TNET_OK;
  const int v4 = (dZ.cols & 3) == 0 && (!Z || v4ok(Z, dZ.stride)) && (!Y || v4ok(Y, strideY)) &&
                 (!E || v4ok(E, strideE));
  // when Z == NULL, Y already holds the softmax output (read through strideY)
  TnetMatrixDim dd = dZ;
  if (!Z) dd.stride = strideY;
  // (one row a workgroup: pipelined R-rows-a-workgroup forms measured slower in the dnn4 step, 9.8 / 11.8 vs
  // 9.0 us, profiles/r04_softmax_rows_ab.json, and the one-pass softmax + slab sums 36.7 vs 9.8 + 6.7 us,
  // profiles/r02_softmax_slabs_ab.txt -- both removed in round 6)
  if (Z && v4 && dZ.cols > 1024 && dZ.cols <= SX_MAXV4 * 256)
    softmax_xent_row4_kernel<<<dZ.rows, 256, 0, (hipStream_t)stream>>>(Z, dd, labels, Y, strideY, E, strideE, stats);
  else
    softmax_xent_kernel<0><<<cdiv((long)dZ.rows * 64, 256), 256, 0, (hipStream_t)stream>>>(
        Z, dd, labels, nullptr, 0, Y, strideY, E, strideE, stats, v4);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_softmax_xent_dense(const float* Z, TnetMatrixDim dZ, const float* D, int strideD, float* Y,
                                       int strideY, float* E, int strideE, double* stats, void* stream) {
  if (dZ.rows < 0 || dZ.cols <= 0 || !D || (!Z && !Y)) return TNET_ERR_ARG;
  if (!dZ.rows) return TNET_OK;
  const float* z = Z;
  const int v4 = (dZ.cols & 3) == 0 && (!z || v4ok(z, dZ.stride)) && (!Y || v4ok(Y, strideY)) &&
                 (!E || v4ok(E, strideE));
  // when Z == NULL the kernel reads Y rows through the stride of dZ
  TnetMatrixDim dd = dZ;
  if (!z) dd.stride = strideY;
  softmax_xent_kernel<1><<<cdiv((long)dZ.rows * 64, 256), 256, 0, (hipStream_t)stream>>>(
      z, dd, nullptr, D, strideD, Y, strideY, E, strideE, stats, v4);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnetF_softmax(float* y, const float* x, TnetMatrixDim d, void* stream) {
  if (d.rows < 0 || d.cols <= 0) return TNET_ERR_ARG;
  if (!d.rows) return TNET_OK;
  // softmax only: no labels/targets -> reuse the class-id kernel with label -1 semantics disabled
  const int v4 = (d.cols & 3) == 0 && v4ok(x, d.stride) && v4ok(y, d.stride);
  softmax_xent_kernel<1><<<cdiv((long)d.rows * 64, 256), 256, 0, (hipStream_t)stream>>>(
      x, d, nullptr, x /*unused targets*/, d.stride, y, d.stride, nullptr, 0, nullptr, v4);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_rbm_stats_update(const float* Vs, TnetMatrixDim dV, const float* Hs, TnetMatrixDim dH, int B,
                                     float* vb, float* cvb, float* hb, float* chb, float scale, float mmt,
                                     double* mse_stats, void* stream) {
  if (B < 0 || dV.rows != 2 * B || dH.rows != 2 * B || dV.cols <= 0 || dH.cols <= 0 || dV.stride < dV.cols ||
      dH.stride < dH.cols || !Vs || !Hs || !vb || !cvb || !hb || !chb)
    return TNET_ERR_ARG;
  if (!B) return TNET_OK;
  if (2 * B > CS_ROWS * RS_MAX_SLABS) return TNET_ERR_UNSUPPORTED;  // slabs of more than 32 rows
  const int nvb = cdiv(dV.cols, RS_COLS), nhb = cdiv(dH.cols, RS_COLS), nmb = mse_stats ? cdiv(B, RS_MROWS) : 0;
  rbm_stats_kernel<<<nvb + nhb + nmb, 256, 0, (hipStream_t)stream>>>(Vs, dV, Hs, dH, B, nvb, vb, cvb, hb, chb, scale,
                                                                     mmt, mse_stats, nhb);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_mse(const float* Y, TnetMatrixDim dY, const float* D, int strideD, float* E, int strideE,
                        double* stats, void* stream) {
  if (dY.rows < 0 || dY.cols <= 0) return TNET_ERR_ARG;
  if (!dY.rows) return TNET_OK;
  mse_kernel<<<cdiv((long)dY.rows * 64, 256), 256, 0, (hipStream_t)stream>>>(Y, dY, D, strideD, E, strideE, stats);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_stats_fetch(const double* stats, double* error, double* correct, void* stream) {
  static double h[TNET_STATS_WORDS];
  if (!stats) return TNET_ERR_ARG;
  if (hipMemcpyAsync(h, stats, sizeof h, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess)
    return TNET_ERR_RUNTIME;
  if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return TNET_ERR_RUNTIME;
  double e = 0.0, c = 0.0;
  for (int i = 0; i < TNET_STATS_SLOTS; i++) {
    e += h[2 * i];
    c += h[2 * i + 1];
  }
  if (error) *error = e;
  if (correct) *correct = c;
  return TNET_OK;
}

extern "C" int tnetF_check_class(const float* out, const float* des, int* match, TnetMatrixDim d, void* stream) {
  if (d.rows < 0 || d.cols <= 0) return TNET_ERR_ARG;
  if (!d.rows) return TNET_OK;
  check_class_kernel<<<cdiv((long)d.rows * 64, 256), 256, 0, (hipStream_t)stream>>>(out, des, match, d);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}
