// top_rows.hip -- a narrow top layer (n_out <= 144 classes: BASELINE config 2's 135 monophone states) in ONE launch:
// Z = X W + b, and -- unless logits_only -- Y = softmax(Z), E = Y - onehot, the cross-entropy / accuracy statistics
// and E's 32-row slab column sums (CuBiasedLinearity::PropagateFnc + CuSoftmax::PropagateFnc +
// CuCrossEntropy::Evaluate, cuBiasedLinearity.cc:11-16, cuActivation.cc:28-31, cuObjectiveFunction.cc:50-83).
//
// Why a kernel of its own: 1024 x 135 over K = 1024 is 283 MFLOP -- 1.8 us of the chip's fp32 MFMA rate -- but only
// 48 64x64 output tiles, so the general GEMM took it as split-K slices plus a combine-and-softmax launch of 32
// workgroups (one per 32-row slab): 19.6 us, 0.085 of peak.  Here the work is cut into 16-row
// blocks x 4 K slices = 256 workgroups (one per CU at M = 1024), each 3 waves x 3 16x16 tiles over its K slice with
// every fragment loaded up front (W, 552 KB, is L2-resident: a slice's 147 KB is shared by the row blocks on the two
// XCDs that run that slice); the slices' partial tiles are handed over write-through (sc1) and the row block's LAST
// slice to finish (a ticket counter, cdna_hip_programming.md section 5 'In-launch split-K reduction', sc1 form) adds
// them in slice order, adds the bias and runs the softmax / cross-entropy / error of its 16 rows; the slab sums
// of a 32-row slab meet the same way between its two row blocks (fixed order: rows 0-15 + rows 16-31).
//
// The same kernel in logits-only mode is what tnet_affine_fwd runs for these shapes, so the fused and the
// three-call forms give the same Z bit for bit (and the same Y / E: the softmax arithmetic and lane map are
// softmax_xent_kernel's, reduce.hip).
#include <hip/hip_runtime.h>

#include <float.h>

#include <map>
#include <mutex>

#include "kcommon.h"

namespace tnetk {

namespace {
constexpr int kRows = 16;    // rows per block (one MFMA row tile)
constexpr int kSlices = 4;   // K slices
constexpr int kWaves = 3;    // waves per block
constexpr int kMaxCols = 144;

struct TopRowsP {
  const float* X;
  long ldx;
  const float* W;
  long ldw;
  const float* b;
  int M, N, K, NT;      // NT: 16-column tiles
  const int* labels;
  float* Z;
  long ldz;
  float* Y;
  long ldy;
  float* E;
  long lde;
  double* stats;
  float* cpart;
  long ldcp;
  int v4, logits_only;
  float* ws;            // [kSlices][16 NT][Mpad] partial tiles, column-major per slice
  float* ws2;           // [row blocks][16 NT] row-block column sums of E
  unsigned* cnt;        // [row blocks] slice tickets, then [slabs] half-slab tickets
  int Mpad, nrb;
};
}  // namespace

template <int TPW, int NCH>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void top_rows_kernel(const TopRowsP q) {
  __shared__ __attribute__((aligned(16))) float zs[kRows * kMaxCols];
  __shared__ double red[2][kWaves];
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int lg = lane >> 4, li = lane & 15;
  // block b: row block b / 4, slice b % 4 -- the blocks of one slice (the same 147 KB of W) run on two XCDs
  const int rb = blockIdx.x / kSlices, sl = blockIdx.x % kSlices;
  const int M = q.M, N = q.N;
  const int ksl = NCH * 16, k0 = sl * ksl;

  // ---- this wave's TPW tiles of the row block over the slice: every fragment loaded before the first MFMA
  // (lane (lg, li) supplies A[li][k], B[k][li] with k = 16 c + 4 lg + s at the chunk's step s: the 16x16x4 kernels'
  // lane map, gemm_f32.hip)
  const int arow = min(rb * kRows + li, M - 1);
  const float* xa = q.X + (long)arow * q.ldx + k0 + 4 * lg;
  f32x4 a[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) a[c] = *reinterpret_cast<const f32x4*>(xa + 16 * c);
  float bf[TPW][NCH][4];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int col = min((wv * TPW + t) * 16 + li, N - 1);  // padding columns: a real column, never stored
    const float* wb = q.W + (long)(k0 + 4 * lg) * q.ldw + col;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int s = 0; s < 4; ++s) bf[t][c][s] = wb[(long)(16 * c + s) * q.ldw];
  }
  f32x4 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c][s], bf[t][c][s], acc[t], 0, 0, 0);

  // ---- the partial tiles, written through: slice sl, column n, rows 4 lg .. 4 lg + 3 as one 16-B vector
  const long cspan = 16L * q.NT;
  const __amdgpu_buffer_rsrc_t rw = tile_rsrc(q.ws + (long)sl * cspan * q.Mpad + (long)rb * kRows);
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tile = wv * TPW + t;
    if (tile < q.NT) st_wt(rw, (long)(tile * 16 + li) * q.Mpad + 4 * lg, acc[t]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __attribute__((address_space(1))) unsigned* c =
        (__attribute__((address_space(1))) unsigned*)(q.cnt + rb);
    const unsigned ticket = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == (unsigned)(kSlices - 1);
    if (last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
    s_flag = last;
  }
  __syncthreads();
  if (!s_flag) return;

  // ---- the row block's last slice: Z = ((s0 + s1) + s2) + s3 + b into LDS (and Z), 4 rows of a column a thread
  const int nr = min(kRows, M - rb * kRows);
  const __amdgpu_buffer_rsrc_t rr = tile_rsrc(q.ws + (long)rb * kRows);
  for (int u = tid; u < 4 * (int)cspan; u += kWaves * 64) {
    const int n = u >> 2, r4 = (u & 3) * 4;
    f32x4 v = ld_sc1(rr, (long)n * q.Mpad + r4);
#pragma unroll
    for (int s = 1; s < kSlices; ++s) {
      const f32x4 w = ld_sc1(rr, (long)s * cspan * q.Mpad + (long)n * q.Mpad + r4);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = v[e] + w[e];
    }
    if (n < N) {
      const float bb = q.b[n];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = v[e] + bb;
        zs[(r4 + e) * kMaxCols + n] = y;
        if (q.Z && r4 + e < nr) q.Z[(long)(rb * kRows + r4 + e) * q.ldz + n] = y;
      }
    }
  }
  if (q.logits_only) return;
  __syncthreads();

  // ---- softmax / cross-entropy / error of the block's rows, a wave per row (softmax_xent_kernel's arithmetic and
  // lane map: Y, E and the statistics identical to the separate launch's)
  double wx = 0.0, wc = 0.0;
  for (int r = wv; r < nr; r += kWaves) {
    float* zr = zs + r * kMaxCols;
    const long row = (long)rb * kRows + r;
    int t = q.labels[row];
    if (t >= N) t = -1;  // unlabeled (the host intake rejects such a label, CheckLabels)
    float x[4];
    int cl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cl[j] = q.v4 ? 4 * lane + j : lane + 64 * j;
      x[j] = cl[j] < N ? zr[cl[j]] : -1e30f;
    }
    const float zt = t >= 0 ? zr[t] : 0.f;
    float m = -1e20f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (cl[j] < N) m = fmaxf(m, x[j]);
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (cl[j] < N) {
        x[j] = fast_exp(x[j] - m);
        s += x[j];
      }
    const float rsum = 1.f / (float)wave_sum_d((double)s);
    ArgMax ay{-1e20f, 0x7fffffff};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (cl[j] < N) {
        const float y = x[j] * rsum;
        if (y > ay.v) { ay.v = y; ay.i = cl[j]; }
        const float e = y - (cl[j] == t ? 1.f : 0.f);
        if (q.Y) q.Y[row * q.ldy + cl[j]] = y;
        q.E[row * q.lde + cl[j]] = e;
        zr[cl[j]] = e;  // every lane has read its logits and zt above
      }
    ay = wave_argmax(ay);
    if (lane == 0) {
      if (t >= 0) wx += -(double)logf(fmaxf(fast_exp(zt - m) * rsum, FLT_MIN));
      wc += ay.i == (t >= 0 ? t : 0) ? 1.0 : 0.0;
    }
  }
  if (lane == 0) {
    red[0][wv] = wx;
    red[1][wv] = wc;
  }
  __syncthreads();
  if (tid == 0 && q.stats) {
    double sx = 0.0, sc = 0.0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      sx += red[0][w];
      sc += red[1][w];
    }
    const int slot = rb % TNET_STATS_SLOTS;
    atomicAdd(q.stats + 2 * slot, sx);
    atomicAdd(q.stats + 2 * slot + 1, sc);
  }
  if (!q.cpart) return;

  // ---- E's column sums over the block's rows (fp32, row order), then the 32-row slab's two halves in fixed order
  const int slab = rb / 2, first = slab * 2, halves = min(2, q.nrb - first);
  float* half = q.ws2 + (long)rb * cspan;
  const __amdgpu_buffer_rsrc_t rh = tile_rsrc(q.ws2);
  for (int n = tid; n < N; n += kWaves * 64) {
    float sum = 0.f;
    for (int r = 0; r < nr; ++r) sum += zs[r * kMaxCols + n];
    if (halves == 1) q.cpart[(long)slab * q.ldcp + n] = sum;
    else half[n] = sum;
  }
  if (halves == 1) return;
  // the halves go through ws2 (plain stores + one agent-scope release: only 144 floats)
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __attribute__((address_space(1))) unsigned* c =
        (__attribute__((address_space(1))) unsigned*)(q.cnt + q.nrb + slab);
    const unsigned ticket = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == 1u;
    if (last) {
      __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_flag = last;
  }
  __syncthreads();
  if (!s_flag) return;
  (void)rh;
  const float* h0 = q.ws2 + (long)first * cspan;
  const float* h1 = h0 + cspan;
  for (int n = tid; n < N; n += kWaves * 64) q.cpart[(long)slab * q.ldcp + n] = h0[n] + h1[n];
}

namespace {
// per-stream workspace (partial tiles, half-slab sums) and ticket counters (zeroed once, reset by the last arrivers)
struct TopWs {
  float* ws = nullptr;
  size_t ws_bytes = 0;
  unsigned* cnt = nullptr;
  size_t ncnt = 0;
};
std::mutex g_top_mu;
std::map<hipStream_t, TopWs> g_top;
TopWs* top_ws(hipStream_t st, size_t bytes, size_t ncnt) {
  std::lock_guard<std::mutex> lk(g_top_mu);
  TopWs& w = g_top[st];
  if (bytes > w.ws_bytes) {
    if (w.ws) {
      if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
      (void)hipFree(w.ws);
      w.ws = nullptr;
      w.ws_bytes = 0;
    }
    if (hipMalloc(&w.ws, bytes) != hipSuccess) return nullptr;
    w.ws_bytes = bytes;
  }
  if (ncnt > w.ncnt) {
    if (w.cnt) {
      if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
      (void)hipFree(w.cnt);
      w.cnt = nullptr;
      w.ncnt = 0;
    }
    const size_t cap = (ncnt + 1023) & ~(size_t)1023;
    if (hipMalloc(&w.cnt, cap * sizeof(unsigned)) != hipSuccess) return nullptr;
    if (hipMemsetAsync(w.cnt, 0, cap * sizeof(unsigned), st) != hipSuccess) return nullptr;
    w.ncnt = cap;
  }
  return &w;
}
}  // namespace

}  // namespace tnetk

using namespace tnetk;

// Which shapes the kernel takes (TNET_TOP_ROWS=0: none): n_out <= 144, K a multiple of 64 in [512, 1024] (3 waves x
// 3 tiles of up to 16 chunks of 16 k held in registers), at least 64 rows, 16-B aligned k-contiguous X.
extern "C" __attribute__((visibility("hidden"))) int tnetk_top_rows_ok(const float* X, long ldx, int M, int N, int K) {
  static const bool on = !(getenv("TNET_TOP_ROWS") && getenv("TNET_TOP_ROWS")[0] == '0');
  return on && N >= 1 && N <= kMaxCols && K >= 512 && K <= 1024 && K % 64 == 0 && M >= 64 &&
         ((uintptr_t)X & 15) == 0 && (ldx & 3) == 0 && (long)M * ldx * 4 < (1L << 31);
}

extern "C" __attribute__((visibility("hidden"))) int tnetk_top_rows(
    const float* X, long ldx, const float* W, long ldw, const float* b, int M, int N, int K, const int* labels,
    float* Z, long ldz, float* Y, long ldy, float* E, long lde, double* stats, float* cpart, long ldcp, int v4,
    int logits_only, void* stream) {
  if (!tnetk_top_rows_ok(X, ldx, M, N, K)) return TNET_ERR_UNSUPPORTED;
  const hipStream_t st = (hipStream_t)stream;
  TopRowsP q{};
  q.X = X; q.ldx = ldx; q.W = W; q.ldw = ldw; q.b = b; q.M = M; q.N = N; q.K = K;
  q.NT = (N + 15) / 16;
  q.labels = labels; q.Z = Z; q.ldz = ldz; q.Y = Y; q.ldy = ldy; q.E = E; q.lde = lde; q.stats = stats;
  q.cpart = cpart; q.ldcp = ldcp; q.v4 = v4; q.logits_only = logits_only;
  q.nrb = (M + kRows - 1) / kRows;
  q.Mpad = q.nrb * kRows;
  const long cspan = 16L * q.NT;
  const size_t wsf = (size_t)kSlices * cspan * q.Mpad, ws2f = (size_t)q.nrb * cspan;
  if (4 * (long)wsf >= (1L << 31)) return TNET_ERR_UNSUPPORTED;
  TopWs* w = top_ws(st, (wsf + ws2f) * sizeof(float), (size_t)q.nrb + (q.nrb + 1) / 2);
  if (!w) return TNET_ERR_RUNTIME;
  q.ws = w->ws;
  q.ws2 = w->ws + wsf;
  q.cnt = w->cnt;
  const int tpw = (q.NT + kWaves - 1) / kWaves, nch = K / 64;
  const dim3 grid((unsigned)(q.nrb * kSlices));
#define TOP_GO(T, C) top_rows_kernel<T, C><<<grid, kWaves * 64, 0, st>>>(q)
  if (tpw == 1) { if (nch == 8) TOP_GO(1, 8); else if (nch == 12) TOP_GO(1, 12); else TOP_GO(1, 16); }
  else if (tpw == 2) { if (nch == 8) TOP_GO(2, 8); else if (nch == 12) TOP_GO(2, 12); else TOP_GO(2, 16); }
  else { if (nch == 8) TOP_GO(3, 8); else if (nch == 12) TOP_GO(3, 12); else TOP_GO(3, 16); }
#undef TOP_GO
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}
