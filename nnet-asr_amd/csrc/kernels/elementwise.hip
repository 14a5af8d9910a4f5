// elementwise.hip -- HBM-bound element-wise / gather kernels of CuBaseLib on gfx950.
//
// Reference semantics: src/CuBaseLib/cukernels.cu:11-141 (matrix ops), :192-217 (sigmoid),
// :347-393 (expand / rearrange / randomize).  The reference launches 16x16 thread blocks per
// element with a device sync after each call; here every op is a flat grid-stride kernel over
// rows x (cols/4) float4 columns (16 B per lane, 1 KiB per wave instruction) whenever the
// stride and width allow it, and a scalar tail otherwise; no sync, caller's stream.
#include <float.h>

#include <algorithm>
#include <cstdlib>

#include "kcommon.h"

namespace tnetk {

constexpr int EW_THREADS = 256;

inline unsigned ew_grid(long work) {
  long g = (work + EW_THREADS - 1) / EW_THREADS;
  if (g > 2048 * 4) g = 2048 * 4;  // grid-stride beyond ~32 waves/CU
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Generic 2-D map: f(row, col) over d.rows x d.cols, scalar form (handles any stride).
template <typename F>
__global__ __launch_bounds__(EW_THREADS) void map2d_kernel(TnetMatrixDim d, F f) {
  const long n = (long)d.rows * d.cols;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
    const int r = (int)(idx / d.cols), c = (int)(idx % d.cols);
    f(r, c);
  }
}

template <typename F>
static int map2d(TnetMatrixDim d, hipStream_t s, F f) {
  if (d.rows < 0 || d.cols < 0 || d.stride < d.cols) return TNET_ERR_ARG;
  if (d.rows == 0 || d.cols == 0) return TNET_OK;
  map2d_kernel<<<ew_grid((long)d.rows * d.cols), EW_THREADS, 0, s>>>(d, f);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

__global__ __launch_bounds__(EW_THREADS) void sigmoid_kernel(float* __restrict__ y, const float* __restrict__ x,
                                                             TnetMatrixDim d, int vec4) {
  if (vec4) {
    const int c4 = d.cols >> 2;
    const long n = (long)d.rows * c4;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
      const long off = (idx / c4) * d.stride + (idx % c4) * 4;
      f32x4 v = *reinterpret_cast<const f32x4*>(x + off);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = sigmoidf_ref(v[k]);
      *reinterpret_cast<f32x4*>(y + off) = v;
    }
  } else {
    const long n = (long)d.rows * d.cols;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
      const long off = (idx / d.cols) * d.stride + idx % d.cols;
      y[off] = sigmoidf_ref(x[off]);
    }
  }
}

__global__ __launch_bounds__(EW_THREADS) void diff_sigmoid_kernel(float* __restrict__ eo,
                                                                  const float* __restrict__ e,
                                                                  const float* __restrict__ y, TnetMatrixDim d,
                                                                  int vec4) {
  if (vec4) {
    const int c4 = d.cols >> 2;
    const long n = (long)d.rows * c4;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
      const long off = (idx / c4) * d.stride + (idx % c4) * 4;
      const f32x4 ev = *reinterpret_cast<const f32x4*>(e + off);
      const f32x4 yv = *reinterpret_cast<const f32x4*>(y + off);
      f32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = yv[k] * (1.f - yv[k]) * ev[k];
      *reinterpret_cast<f32x4*>(eo + off) = o;
    }
  } else {
    const long n = (long)d.rows * d.cols;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
      const long off = (idx / d.cols) * d.stride + idx % d.cols;
      eo[off] = y[off] * (1.f - y[off]) * e[off];
    }
  }
}

// Row gather: y[i,:] = x[idx[i],:]   (cache shuffle / bunch fetch; one wave per row, float4)
__global__ __launch_bounds__(EW_THREADS) void gather_rows_kernel(float* __restrict__ y, const float* __restrict__ x,
                                                                 const int* __restrict__ idx, TnetMatrixDim dout,
                                                                 TnetMatrixDim din, int vec4,
                                                                 int* __restrict__ lab_out = nullptr,
                                                                 const int* __restrict__ lab_in = nullptr) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int r = wave; r < dout.rows; r += nwaves) {
    const int ir = idx[r];
    if (lab_out && lane == 0) lab_out[r] = lab_in[ir];  // the bunch's class ids ride along
    const long src = (long)ir * din.stride;
    const long dst = (long)r * dout.stride;
    if (vec4) {
      // the bunch row written through (kcommon.h st_wt): the step's first GEMM reads it on every XCD
      const __amdgpu_buffer_rsrc_t ry = tile_rsrc(y + dst);
      for (int c = lane * 4; c < dout.cols; c += 256) st_wt(ry, c, *reinterpret_cast<const f32x4*>(x + src + c));
    } else {
      for (int c = lane; c < dout.cols; c += 64) y[dst + c] = x[src + c];
    }
  }
}

__global__ __launch_bounds__(EW_THREADS) void gather_i32_kernel(int* __restrict__ out, const int* __restrict__ in,
                                                                const int* __restrict__ idx, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = in[idx[i]];
}

// SGD on flat arrays: c = g + mmt*corr; p += scale*c; p += l2*p; corr = c
__global__ __launch_bounds__(EW_THREADS) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ corr, long n, float scale, float mmt,
                                                         float l2) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float c = g[i];
    if (corr) {
      c = c + mmt * corr[i];
      corr[i] = c;
    }
    float w = p[i];
    w = w + scale * c;
    w = w + l2 * w;
    p[i] = w;
  }
}

// several SGD segments (a layer's W and b, ...) in one launch: block b serves the segment whose
// [first, first + nblk) block range holds it (uniform per block), 16-B accesses where aligned
constexpr int SGD_MAXSEG = 8;
struct SgdSegs {
  TnetSgdSeg s[SGD_MAXSEG];
  int first[SGD_MAXSEG + 1];
  int nseg;
};
__global__ __launch_bounds__(EW_THREADS) void sgd_multi_kernel(const SgdSegs segs, float scale, float mmt) {
  int k = 0;
  while (k + 1 < segs.nseg && (int)blockIdx.x >= segs.first[k + 1]) ++k;
  const TnetSgdSeg sg = segs.s[k];
  const long nb = segs.first[k + 1] - segs.first[k];
  const long t0 = (long)(blockIdx.x - segs.first[k]) * blockDim.x + threadIdx.x, step = nb * blockDim.x;
  const bool v4 = ((sg.n & 3) == 0) && (((uintptr_t)sg.p | (uintptr_t)sg.g | (uintptr_t)sg.corr) & 15) == 0;
  if (v4) {
    // U vectors per thread per pass, every load of the pass issued before the first store: the launch is
    // a few hundred fat workgroups (not one 16-B vector per thread), so beside the GEMMs of the step it
    // takes few wave launches and issue slots for its bytes
    constexpr int U = 4;
    const f32x4* g = reinterpret_cast<const f32x4*>(sg.g);
    const f32x4* p = reinterpret_cast<const f32x4*>(sg.p);
    const f32x4* q = reinterpret_cast<const f32x4*>(sg.corr);
    // parameters and momentum written through (kcommon.h st_wt): read next by the all-gather / the
    // next step's forward, from any XCD -- nothing is gained by leaving them dirty in this XCD's L2
    const bool wt = sg.n < (1L << 29);  // byte offsets of the descriptor stay below 2^31
    const __amdgpu_buffer_rsrc_t rp = tile_rsrc(sg.p), rq = tile_rsrc(q ? sg.corr : sg.p);
    const long n4 = sg.n / 4;
    for (long i0 = t0; i0 < n4; i0 += U * step) {
      f32x4 c[U], w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long i = i0 + u * step;
        if (i < n4) {
          c[u] = g[i];
          w[u] = p[i];
          if (q) c[u] = c[u] + mmt * q[i];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long i = i0 + u * step;
        if (i >= n4) break;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          w[u][e] = w[u][e] + scale * c[u][e];
          w[u][e] = w[u][e] + sg.l2 * w[u][e];
        }
        if (q) {
          if (wt) st_wt(rq, 4 * i, c[u]);
          else reinterpret_cast<f32x4*>(sg.corr)[i] = c[u];
        }
        if (wt) st_wt(rp, 4 * i, w[u]);
        else reinterpret_cast<f32x4*>(sg.p)[i] = w[u];
      }
    }
  } else {
    for (long i = t0; i < sg.n; i += step) {
      float c = sg.g[i];
      if (sg.corr) {
        c = c + mmt * sg.corr[i];
        sg.corr[i] = c;
      }
      float w = sg.p[i];
      w = w + scale * c;
      w = w + sg.l2 * w;
      sg.p[i] = w;
    }
  }
}

static bool vec4_ok(const void* a, TnetMatrixDim d) {
  return ((uintptr_t)a & 15) == 0 && (d.cols & 3) == 0 && (d.stride & 3) == 0;
}

}  // namespace tnetk

using namespace tnetk;

#define STREAM ((hipStream_t)stream)

extern "C" int tnetF_set_const(float* mat, float value, TnetMatrixDim d, void* stream) {
  return map2d(d, STREAM, [=] __device__(int r, int c) { mat[(long)r * d.stride + c] = value; });
}

extern "C" int tnetF_apply_log(float* mat, TnetMatrixDim d, void* stream) {
  return map2d(d, STREAM, [=] __device__(int r, int c) {
    float* q = mat + (long)r * d.stride + c;
    *q = logf(*q);
  });
}

extern "C" int tnetF_apply_mask(float* mat, const float* mask, TnetMatrixDim dmat, TnetMatrixDim dmask,
                                void* stream) {
  return map2d(dmat, STREAM, [=] __device__(int r, int c) {
    if (mask[(long)r * dmask.stride + c] == 0.f) mat[(long)r * dmat.stride + c] = 0.f;
  });
}

extern "C" int tnetF_apply_l1(float* mat, float l1, TnetMatrixDim d, void* stream) {
  return map2d(d, STREAM, [=] __device__(int r, int c) {
    float* q = mat + (long)r * d.stride + c;
    const float v = *q;
    *q = (fabsf(v) < l1) ? 0.f : (v > 0.f ? v - l1 : v + l1);
  });
}

extern "C" int tnetF_scale_cols(float* mat, const float* scale, TnetMatrixDim d, void* stream) {
  return map2d(d, STREAM, [=] __device__(int r, int c) { mat[(long)r * d.stride + c] *= scale[c]; });
}

extern "C" int tnetF_scale_rows(float* mat, const float* scale, TnetMatrixDim d, void* stream) {
  return map2d(d, STREAM, [=] __device__(int r, int c) { mat[(long)r * d.stride + c] *= scale[r]; });
}

extern "C" int tnetF_add_scaled(float alpha, const float* A, int strideA, float beta, float* dst, TnetMatrixDim d,
                                void* stream) {
  return map2d(d, STREAM, [=] __device__(int r, int c) {
    float* q = dst + (long)r * d.stride + c;
    *q = alpha * A[(long)r * strideA + c] + beta * *q;
  });
}

extern "C" int tnetF_add_scaled_row(float alpha, const float* row, float beta, float* dst, TnetMatrixDim d,
                                    void* stream) {
  return map2d(d, STREAM, [=] __device__(int r, int c) {
    float* q = dst + (long)r * d.stride + c;
    *q = (beta == 0.f) ? alpha * row[c] : alpha * row[c] + beta * *q;
  });
}

extern "C" int tnetF_mul_elem(float* mat, const float* A, int strideA, TnetMatrixDim d, void* stream) {
  return map2d(d, STREAM, [=] __device__(int r, int c) { mat[(long)r * d.stride + c] *= A[(long)r * strideA + c]; });
}

extern "C" int tnetF_log_elem(float* mat, TnetMatrixDim d, void* stream) {
  return map2d(d, STREAM, [=] __device__(int r, int c) {
    float* q = mat + (long)r * d.stride + c;
    float v = *q;
    if (v < FLT_MIN) v = FLT_MIN;
    *q = logf(v);
  });
}

extern "C" int tnetF_sigmoid(float* y, const float* x, TnetMatrixDim d, void* stream) {
  if (d.rows < 0 || d.cols < 0 || d.stride < d.cols) return TNET_ERR_ARG;
  if (!d.rows || !d.cols) return TNET_OK;
  const int v4 = vec4_ok(x, d) && vec4_ok(y, d);
  sigmoid_kernel<<<ew_grid((long)d.rows * d.cols / (v4 ? 4 : 1)), EW_THREADS, 0, STREAM>>>(y, x, d, v4);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnetF_diff_sigmoid(float* eout, const float* e, const float* y, TnetMatrixDim d, void* stream) {
  if (d.rows < 0 || d.cols < 0 || d.stride < d.cols) return TNET_ERR_ARG;
  if (!d.rows || !d.cols) return TNET_OK;
  const int v4 = vec4_ok(e, d) && vec4_ok(y, d) && vec4_ok(eout, d);
  diff_sigmoid_kernel<<<ew_grid((long)d.rows * d.cols / (v4 ? 4 : 1)), EW_THREADS, 0, STREAM>>>(eout, e, y, d, v4);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnetF_expand(float* y, const float* x, const int* off, TnetMatrixDim dout, TnetMatrixDim din,
                            void* stream) {
  if (din.cols <= 0) return TNET_ERR_ARG;
  return map2d(dout, STREAM, [=] __device__(int r, int c) {
    const int src_col = c % din.cols;
    int src_row = r + off[c / din.cols];
    if (src_row < 0) src_row = 0;
    if (src_row >= din.rows) src_row = din.rows - 1;
    y[(long)r * dout.stride + c] = x[(long)src_row * din.stride + src_col];
  });
}

extern "C" int tnetF_rearrange(float* y, const float* x, const int* copy_from, TnetMatrixDim dout,
                               TnetMatrixDim din, void* stream) {
  return map2d(dout, STREAM, [=] __device__(int r, int c) {
    const int src_col = copy_from[c];
    y[(long)r * dout.stride + c] =
        (src_col >= 0 && src_col < din.cols) ? x[(long)r * din.stride + src_col] : __builtin_inff();
  });
}

extern "C" int tnetF_randomize(float* y, const float* x, const int* copy_from, TnetMatrixDim dout,
                               TnetMatrixDim din, void* stream) {
  if (dout.cols != din.cols || dout.rows < 0) return TNET_ERR_ARG;
  if (!dout.rows || !dout.cols) return TNET_OK;
  const int v4 = vec4_ok(x, din) && vec4_ok(y, dout);
  long waves = dout.rows;
  unsigned grid = (unsigned)((waves * 64 + EW_THREADS - 1) / EW_THREADS);
  if (grid > 4096) grid = 4096;
  gather_rows_kernel<<<grid, EW_THREADS, 0, STREAM>>>(y, x, copy_from, dout, din, v4);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_gather_bunch(float* y, const float* x, int* labels_out, const int* labels_in,
                                 const int* copy_from, TnetMatrixDim dout, TnetMatrixDim din, void* stream) {
  if (dout.cols != din.cols || dout.rows < 0 || !labels_out || !labels_in) return TNET_ERR_ARG;
  if (!dout.rows) return TNET_OK;
  const int v4 = vec4_ok(x, din) && vec4_ok(y, dout);
  unsigned grid = (unsigned)(((long)dout.rows * 64 + EW_THREADS - 1) / EW_THREADS);
  if (grid > 4096) grid = 4096;
  gather_rows_kernel<<<grid, EW_THREADS, 0, STREAM>>>(y, x, copy_from, dout, din, v4, labels_out, labels_in);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_gather_i32(int* out, const int* in, const int* copy_from, int n, void* stream) {
  if (n < 0) return TNET_ERR_ARG;
  if (!n) return TNET_OK;
  gather_i32_kernel<<<ew_grid(n), EW_THREADS, 0, STREAM>>>(out, in, copy_from, n);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_sgd_update(float* p, const float* g, float* corr, long n, float scale, float mmt, float l2,
                               void* stream) {
  if (n < 0 || (mmt != 0.f && !corr)) return TNET_ERR_ARG;
  if (!n) return TNET_OK;
  sgd_kernel<<<ew_grid(n), EW_THREADS, 0, STREAM>>>(p, g, corr, n, scale, mmt, l2);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_sgd_update_multi(const TnetSgdSeg* segs, int nseg, float scale, float mmt, void* stream) {
  if (nseg < 0 || (nseg && !segs)) return TNET_ERR_ARG;
  for (int k0 = 0; k0 < nseg; k0 += SGD_MAXSEG) {
    SgdSegs a{};
    long total = 0;
    int blocks = 0;
    a.nseg = 0;
    for (int k = k0; k < nseg && k < k0 + SGD_MAXSEG; ++k) {
      const TnetSgdSeg& sg = segs[k];
      if (sg.n < 0 || (sg.n && (!sg.p || !sg.g)) || (mmt != 0.f && sg.n && !sg.corr)) return TNET_ERR_ARG;
      if (!sg.n) continue;
      total += sg.n;
      a.s[a.nseg++] = sg;
    }
    if (!a.nseg) continue;
    // blocks proportional to the segment sizes (at least one each), the whole launch capped at
    // TNET_SGD_BLOCKS (default 1024: 4 per CU; grid-stride beyond, 4 vectors per thread per pass).  Beside
    // the data-parallel step's backward GEMMs: 893 k frames/s at 1024 against 882 k at 512, 881 k at 256
    // and 876 k at 8192 (one vector per thread, the round-3 form) -- profiles/r04_dp_apply_ab.json
    static const long cap = getenv("TNET_SGD_BLOCKS") ? std::max(1L, atol(getenv("TNET_SGD_BLOCKS"))) : 1024L;
    const long want = std::min(cap, (total / 4 + EW_THREADS - 1) / EW_THREADS);
    for (int k = 0; k < a.nseg; ++k) {
      a.first[k] = blocks;
      blocks += (int)std::max(1L, (long)((double)want * a.s[k].n / total + 0.5));
    }
    a.first[a.nseg] = blocks;
    sgd_multi_kernel<<<blocks, EW_THREADS, 0, STREAM>>>(a, scale, mmt);
    TNET_LAUNCH_CHECK();
  }
  return TNET_OK;
}
