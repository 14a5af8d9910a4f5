// top_rows.hip -- a narrow top layer (n_out <= 144 classes: BASELINE config 2's 135 monophone states) in ONE launch:
// Z = X W + b, and -- unless logits_only -- Y = softmax(Z), E = Y - onehot, the cross-entropy / accuracy statistics
// and E's 32-row slab column sums (CuBiasedLinearity::PropagateFnc + CuSoftmax::PropagateFnc +
// CuCrossEntropy::Evaluate, cuBiasedLinearity.cc:11-16, cuActivation.cc:28-31, cuObjectiveFunction.cc:50-83).
//
// Why a kernel of its own: 1024 x 135 over K = 1024 is 283 MFLOP -- 1.8 us of the chip's fp32 MFMA rate -- but only
// 48 64x64 output tiles, so the general GEMM took it as split-K slices plus a combine-and-softmax launch of 32
// workgroups (one per 32-row slab): 19.6 us, 0.085 of peak.  Here the work is cut into 16-row
// blocks x 4 K slices = 256 workgroups (one per CU at M = 1024), each 4 waves over up to 9 16x16 tiles of its K slice:
// the slice of W (147 KB at K = 1024; W, 552 KB, stays L2-resident, a slice shared by the row blocks on the two XCDs
// that run it) is staged in LDS with 16-B loads and the MFMA B fragments are read from there, the A fragments are
// loaded straight into registers; the slices' partial tiles are handed over write-through (sc1) and the row block's
// LAST slice to finish (a ticket counter, cdna_hip_programming.md section 5 'In-launch split-K reduction', sc1 form) adds
// them in slice order, adds the bias and runs the softmax / cross-entropy / error of its 16 rows; the slab sums
// of a 32-row slab meet the same way between its two row blocks (fixed order: rows 0-15 + rows 16-31).
//
// The same kernel in logits-only mode is what tnet_affine_fwd runs for these shapes, so the fused and the
// three-call forms give the same Z bit for bit (and the same Y / E: the softmax arithmetic and lane map are
// softmax_xent_kernel's, reduce.hip).
//
// Status: OPT-IN (tnet_top_rows_config / TNET_TOP_ROWS=1), parity-tested, not the default.  Measured at 1024 x 1024
// -> 135 on MI355X (tools/top_rows_bench.py, profiles/r05_top_rows.json): logits 13.1 us and fused 19.7 us against
// 12.2 / 17.8 us for the two-launch form.  Phase stamps show why the 9 us target is out of reach in this shape: the
// MFMAs alone are 6.2k cycles (144 padded columns x 1024 rows x 1024 k on every SIMD of the chip = 2.6 us at the fp32
// MFMA rate), every block pulls its 147 KB W slice through its CU's L1 (8.5k cycles with the operand loads), and the
// two write-through hand-offs (slices -> last slice, half slabs -> slab) each cost a store-drain + ticket round
// trip of ~2 us on the critical path, ahead of a softmax tail that runs on 64 of the 256 CUs.
#include <hip/hip_runtime.h>

#include <float.h>

#include <map>
#include <mutex>

#include "kcommon.h"

namespace tnetk {

namespace {
constexpr int kRows = 16;    // rows per block (one MFMA row tile)
constexpr int kSlices = 4;   // K slices
constexpr int kWaves = 4;    // waves per block
constexpr int kMaxCols = 144;
constexpr int kPitch = 148;  // LDS row pitch of the W slice (floats): 4 rows apart = 16 banks apart

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
  int v4, logits_only;  // 2: the K slices' partial products only (row-major into part), no combine
  float* part;          // [kSlices][M][ldpart] (logits_only 2)
  long ldpart;
  float* ws;            // [kSlices][16 NT][Mpad] partial tiles, column-major per slice
  float* ws2;           // [row blocks][16 NT] row-block column sums of E
  unsigned* cnt;        // [row blocks] slice tickets, then [slabs] half-slab tickets
  int Mpad, nrb;
  long long* stamps;    // diagnostics (tnet_top_rows_stamps): thread 0's s_memtime per phase, 8 words a block
};
}  // namespace

// V: how the B fragments reach the MFMAs -- 1: straight from global memory into registers, all before the first MFMA;
// 3: the slice of W staged in LDS with 16-B loads, then every fragment read into registers before the first MFMA
// (tnet_top_rows_config; default 1.  A variant reading the fragments from LDS inside the MFMA loop measured slower
// than both, 18.7 us for the logits at 1024 x 1024 -> 135, and was dropped)
template <int NCH, int V>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void top_rows_kernel(const TopRowsP q) {
  // LDS: the slice of W [16 NCH k][kPitch] during the GEMM (V 3), then the block's logits / errors [kRows][kMaxCols]
  constexpr int LDS_F = V == 1 ? kRows * kMaxCols : 16 * NCH * kPitch;
  __shared__ __attribute__((aligned(16))) float lds[LDS_F];
  __shared__ double red[2][kWaves];
  __shared__ int s_flag;
  __shared__ int s_lab[kRows];
  float* const zs = lds;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int lg = lane >> 4, li = lane & 15;
  // block b: row block b / 4, slice b % 4 -- the blocks of one slice (the same 147 KB of W) run on two XCDs
  const int rb = blockIdx.x / kSlices, sl = blockIdx.x % kSlices;
  const int M = q.M, N = q.N;
  const int ksl = NCH * 16, k0 = sl * ksl;
  auto stamp = [&](int i) {
    if (q.stamps && tid == 0) q.stamps[(long)blockIdx.x * 8 + i] = (long long)__builtin_amdgcn_s_memtime();
  };
  stamp(0);
  // this block's class ids (read by the softmax of the row block's last slice; loaded now, off its critical path)
  const int my_label = (q.logits_only == 0 && tid < kRows && rb * kRows + tid < M) ? q.labels[rb * kRows + tid] : -1;

  // ---- the A fragments straight into registers (lane (lg, li) supplies A[li][k], B[k][li] with k = 16 c + 4 lg + s
  // at the chunk's step s: the 16x16x4 kernels' lane map, gemm_f32.hip); tiles wv, wv + 4, wv + 8 (N <= 144)
  const int arow = min(rb * kRows + li, M - 1);
  const float* xa = q.X + (long)arow * q.ldx + k0 + 4 * lg;
  f32x4 a[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) a[c] = *reinterpret_cast<const f32x4*>(xa + 16 * c);
  f32x4 acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (V == 1) {
    float bf[3][NCH][4];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int col = min((wv + 4 * t) * 16 + li, N - 1);  // padding columns: a real column, never stored
      const float* wb = q.W + (long)(k0 + 4 * lg) * q.ldw + col;
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int s = 0; s < 4; ++s) bf[t][c][s] = wb[(long)(16 * c + s) * q.ldw];
    }
    if (q.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(1);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c][s], bf[t][c][s], acc[t], 0, 0, 0);
  } else {
    // the slice of W into LDS with 16-B loads, every load of a thread issued before its first LDS write (row pitch
    // kPitch: the fragment reads hit 64 distinct banks; the padding columns up to 16 NT are read, q.ldw >= 16 NT)
    // (u / c4 as a float product: u < 9216, the rounding error of (u + 0.5) / c4 is far below 0.5 / c4)
    const int c4 = 4 * q.NT, tot = ksl * c4;
    const float rc4 = 1.f / (float)c4;
    constexpr int IT = (16 * NCH * (kMaxCols / 4) + kWaves * 64 - 1) / (kWaves * 64);
    f32x4 wv4[IT];
    int kk[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int u = min(tid + kWaves * 64 * i, tot - 1), k = (int)(((float)u + 0.5f) * rc4), j = u - k * c4;
      kk[i] = k * kPitch + 4 * j;
      wv4[i] = *reinterpret_cast<const f32x4*>(q.W + (long)(k0 + k) * q.ldw + 4 * j);
    }
#pragma unroll
    for (int i = 0; i < IT; ++i)
      if (tid + kWaves * 64 * i < tot) *reinterpret_cast<f32x4*>(lds + kk[i]) = wv4[i];
    __syncthreads();
    if (q.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(1);
    const float* wl = lds + (4 * lg) * kPitch + li + wv * 16;
    {
      float bf[3][NCH][4];
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int s = 0; s < 4; ++s) bf[t][c][s] = wl[(16 * c + s) * kPitch + 64 * t];
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c][s], bf[t][c][s], acc[t], 0, 0, 0);
    }
  }
  stamp(2);

  if (q.logits_only == 2) {
    // ---- partials only: slice sl's rows 4 lg .. 4 lg + 3 of column (tile, li), row-major at part[sl][row][col]
    // (every column of the 16 NT is written, the padding ones from the clamped W column; the next launch combines)
    float* pp = q.part + (long)sl * M * q.ldpart;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int tile = wv + 4 * t;
      if (tile >= q.NT) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rb * kRows + 4 * lg + r;
        if (row < M) pp[(long)row * q.ldpart + tile * 16 + li] = acc[t][r];
      }
    }
    return;
  }

  // ---- the partial tiles, written through: slice sl, column n, rows 4 lg .. 4 lg + 3 as one 16-B vector
  const long cspan = 16L * q.NT;
  const __amdgpu_buffer_rsrc_t rw = tile_rsrc(q.ws + (long)sl * cspan * q.Mpad + (long)rb * kRows);
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int tile = wv + 4 * t;
    if (tile < q.NT) st_wt(rw, (long)(tile * 16 + li) * q.Mpad + 4 * lg, acc[t]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // (also: every wave is done with the W slice in LDS before zs overwrites it)
  if (tid == 0) {
    __attribute__((address_space(1))) unsigned* c =
        (__attribute__((address_space(1))) unsigned*)(q.cnt + rb);
    const unsigned ticket = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == (unsigned)(kSlices - 1);
    if (last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
    s_flag = last;
  }
  __syncthreads();
  stamp(3);
  if (!s_flag) return;
  if (tid < kRows) s_lab[tid] = my_label;

  // ---- the row block's last slice: Z = ((s0 + s1) + s2) + s3 + b into LDS (and Z), 4 rows of a column a thread
  const int nr = min(kRows, M - rb * kRows);
  const __amdgpu_buffer_rsrc_t rr = tile_rsrc(q.ws + (long)rb * kRows);
  constexpr int CI = (4 * kMaxCols + kWaves * 64 - 1) / (kWaves * 64);
  f32x4 pv[CI][kSlices];  // every partial of the thread requested before the first add
#pragma unroll
  for (int i = 0; i < CI; ++i) {
    const int u = min(tid + kWaves * 64 * i, 4 * (int)cspan - 1), n = u >> 2, r4 = (u & 3) * 4;
#pragma unroll
    for (int s = 0; s < kSlices; ++s) pv[i][s] = ld_sc1(rr, (long)s * cspan * q.Mpad + (long)n * q.Mpad + r4);
  }
#pragma unroll
  for (int i = 0; i < CI; ++i) {
    const int u = tid + kWaves * 64 * i, n = u >> 2, r4 = (u & 3) * 4;
    if (u >= 4 * (int)cspan) break;
    f32x4 v = pv[i][0];
#pragma unroll
    for (int s = 1; s < kSlices; ++s)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = v[e] + pv[i][s][e];
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
  if (q.logits_only) {
    stamp(4);
    return;
  }
  __syncthreads();

  // ---- softmax / cross-entropy / error of the block's rows, a wave per row (softmax_xent_kernel's arithmetic and
  // lane map: Y, E and the statistics identical to the separate launch's), two rows at a time per wave so that the
  // two rows' reduction chains overlap
  double wx = 0.0, wc = 0.0;
  auto row_softmax = [&](int r, bool live, float (&x)[4], int (&cl)[4], int& t, float& zt, float& m, float& rsum) {
    t = live ? s_lab[r] : -1;
    if (t >= N) t = -1;  // unlabeled (the host intake rejects such a label, CheckLabels)
    const float* zr = zs + (live ? r : 0) * kMaxCols;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cl[j] = q.v4 ? 4 * lane + j : lane + 64 * j;
      x[j] = cl[j] < N ? zr[cl[j]] : -1e30f;
    }
    zt = t >= 0 ? zr[t] : 0.f;
    m = -1e20f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (cl[j] < N) m = fmaxf(m, x[j]);
  };
  for (int r = wv; r < nr; r += 2 * kWaves) {
    const int r2 = r + kWaves;
    const bool live2 = r2 < nr;
    float x[2][4], zt[2], m[2], rsum[2];
    int cl[2][4], t[2];
    row_softmax(r, true, x[0], cl[0], t[0], zt[0], m[0], rsum[0]);
    row_softmax(r2, live2, x[1], cl[1], t[1], zt[1], m[1], rsum[1]);
    m[0] = wave_max(m[0]);
    m[1] = wave_max(m[1]);
    float s[2] = {0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (cl[h][j] < N) {
          x[h][j] = fast_exp(x[h][j] - m[h]);
          s[h] += x[h][j];
        }
    const double d0 = wave_sum_d((double)s[0]), d1 = wave_sum_d((double)s[1]);
    rsum[0] = 1.f / (float)d0;
    rsum[1] = 1.f / (float)d1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !live2) break;
      const int rr = h ? r2 : r;
      float* zr = zs + rr * kMaxCols;
      const long row = (long)rb * kRows + rr;
      ArgMax ay{-1e20f, 0x7fffffff};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (cl[h][j] < N) {
          const float y = x[h][j] * rsum[h];
          if (y > ay.v) { ay.v = y; ay.i = cl[h][j]; }
          const float e = y - (cl[h][j] == t[h] ? 1.f : 0.f);
          if (q.Y) q.Y[row * q.ldy + cl[h][j]] = y;
          q.E[row * q.lde + cl[h][j]] = e;
          zr[cl[h][j]] = e;  // every lane has read its logits and zt above
        }
      ay = wave_argmax(ay);
      if (lane == 0) {
        if (t[h] >= 0) wx += -(double)logf(fmaxf(fast_exp(zt[h] - m[h]) * rsum[h], FLT_MIN));
        wc += ay.i == (t[h] >= 0 ? t[h] : 0) ? 1.0 : 0.0;
      }
    }
  }
  if (lane == 0) {
    red[0][wv] = wx;
    red[1][wv] = wc;
  }
  __syncthreads();
  stamp(5);
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
  // (rows 0-15 + rows 16-31); the halves are handed over write-through (sc1 16-B stores drained before the ticket,
  // sc1 loads in the last arriver: no fences)
  const int slab = rb / 2, first = slab * 2, halves = min(2, q.nrb - first);
  const int N4 = (N + 3) / 4;
  const __amdgpu_buffer_rsrc_t rh = tile_rsrc(q.ws2 + (long)first * cspan);
  for (int u = tid; u < N4; u += kWaves * 64) {
    f32x4 sum = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < nr; ++r)
#pragma unroll
      for (int e = 0; e < 4; ++e) sum[e] += zs[r * kMaxCols + 4 * u + e];
    if (halves == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * u + e < N) q.cpart[(long)slab * q.ldcp + 4 * u + e] = sum[e];
    } else {
      st_wt(rh, (long)(rb - first) * cspan + 4 * u, sum);
    }
  }
  if (halves == 1) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __attribute__((address_space(1))) unsigned* c =
        (__attribute__((address_space(1))) unsigned*)(q.cnt + q.nrb + slab);
    const unsigned ticket = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == 1u;
    if (last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_flag = last;
  }
  __syncthreads();
  if (!s_flag) return;
  for (int u = tid; u < N4; u += kWaves * 64) {
    const f32x4 h0 = ld_sc1(rh, 4 * u), h1 = ld_sc1(rh, cspan + 4 * u);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (4 * u + e < N) q.cpart[(long)slab * q.ldcp + 4 * u + e] = h0[e] + h1[e];
  }
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
long long* g_top_stamps = nullptr;  // tnet_top_rows_stamps
struct TopMode {
  bool on;
  int v;
};
TopMode& top_rows_mode() {  // tnet_top_rows_config; initial state from TNET_TOP_ROWS / TNET_TOP_ROWS_V (default off)
  static TopMode m{getenv("TNET_TOP_ROWS") && getenv("TNET_TOP_ROWS")[0] == '1',
                   getenv("TNET_TOP_ROWS_V") ? atoi(getenv("TNET_TOP_ROWS_V")) : 1};
  return m;
}
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

// Which shapes the kernel takes (TNET_TOP_ROWS=0: none): n_out <= 144, K = 512, 768 or 1024 (4 slices of 8, 12 or 16
// chunks of 16 k, the chunks of A held in registers), at least 64 rows, 16-B aligned k-contiguous X.
extern "C" __attribute__((visibility("hidden"))) int tnetk_top_rows_shape_ok(const float* X, long ldx, const float* W,
                                                                            long ldw, int M, int N, int K) {
  // (W is read in 16-B pieces up to column 16 ceil(N / 16): inside its padded rows)
  return N >= 1 && N <= kMaxCols && (K == 512 || K == 768 || K == 1024) && M >= 64 &&
         ((uintptr_t)X & 15) == 0 && (ldx & 3) == 0 && (long)M * ldx * 4 < (1L << 31) && ((uintptr_t)W & 15) == 0 &&
         (ldw & 3) == 0 && ldw >= 16L * ((N + 15) / 16);
}
extern "C" __attribute__((visibility("hidden"))) int tnetk_top_rows_ok(const float* X, long ldx, const float* W,
                                                                      long ldw, int M, int N, int K) {
  return top_rows_mode().on && tnetk_top_rows_shape_ok(X, ldx, W, ldw, M, N, K);
}

extern "C" __attribute__((visibility("hidden"))) int tnetk_top_rows(
    const float* X, long ldx, const float* W, long ldw, const float* b, int M, int N, int K, const int* labels,
    float* Z, long ldz, float* Y, long ldy, float* E, long lde, double* stats, float* cpart, long ldcp, int v4,
    int logits_only, float* part, long ldpart, void* stream) {
  if (logits_only == 2 ? !tnetk_top_rows_shape_ok(X, ldx, W, ldw, M, N, K) || !part || ldpart < 16L * ((N + 15) / 16)
                       : !tnetk_top_rows_ok(X, ldx, W, ldw, M, N, K))
    return TNET_ERR_UNSUPPORTED;
  const hipStream_t st = (hipStream_t)stream;
  TopRowsP q{};
  q.X = X; q.ldx = ldx; q.W = W; q.ldw = ldw; q.b = b; q.M = M; q.N = N; q.K = K;
  q.NT = (N + 15) / 16;
  q.labels = labels; q.Z = Z; q.ldz = ldz; q.Y = Y; q.ldy = ldy; q.E = E; q.lde = lde; q.stats = stats;
  q.cpart = cpart; q.ldcp = ldcp; q.v4 = v4; q.logits_only = logits_only;
  q.part = part; q.ldpart = ldpart;
  q.nrb = (M + kRows - 1) / kRows;
  q.Mpad = q.nrb * kRows;
  const long cspan = 16L * q.NT;
  const size_t wsf = (size_t)kSlices * cspan * q.Mpad, ws2f = (size_t)q.nrb * cspan;
  if (4 * (long)wsf >= (1L << 31)) return TNET_ERR_UNSUPPORTED;
  if (logits_only != 2) {  // the in-launch combine's partial tiles, half-slab sums and tickets
    TopWs* w = top_ws(st, (wsf + ws2f) * sizeof(float), (size_t)q.nrb + (q.nrb + 1) / 2);
    if (!w) return TNET_ERR_RUNTIME;
    q.ws = w->ws;
    q.ws2 = w->ws + wsf;
    q.cnt = w->cnt;
  }
  const int nch = K / 64;
  const dim3 grid((unsigned)(q.nrb * kSlices));
  q.stamps = g_top_stamps;
  const int v = top_rows_mode().v;
#define TOP_GO(V)                                                              \
  do {                                                                         \
    if (nch == 8) top_rows_kernel<8, V><<<grid, kWaves * 64, 0, st>>>(q);      \
    else if (nch == 12) top_rows_kernel<12, V><<<grid, kWaves * 64, 0, st>>>(q); \
    else top_rows_kernel<16, V><<<grid, kWaves * 64, 0, st>>>(q);              \
  } while (0)
  if (v == 3) TOP_GO(3);
  else TOP_GO(1);
#undef TOP_GO
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_top_rows_config(int on, int variant) {
  if (variant != 1 && variant != 3) return TNET_ERR_ARG;
  top_rows_mode() = TopMode{on != 0, variant};
  return TNET_OK;
}

// diagnostics: the next launches record thread 0's s_memtime per phase into buf[block * 8 + i] (i: 0 entry, 1 operands
// in registers / LDS, 2 MFMAs issued, 3 partial tiles stored and the ticket drawn, 4 the last slice's end); NULL: off
extern "C" int tnet_top_rows_stamps(long long* buf) {
  g_top_stamps = buf;
  return TNET_OK;
}
