// top_rows.hip -- the K slices of a narrow top layer's GEMM (n_out <= 144 classes: BASELINE config 2's 135 monophone
// states) for the split-K combine launch behind it: Z = X W + b of CuBiasedLinearity::PropagateFnc
// (cuBiasedLinearity.cc:11-16), whose combine is either affine_softmax_xent_kernel (with CuSoftmax::PropagateFnc +
// CuCrossEntropy::Evaluate, cuActivation.cc:28-31, cuObjectiveFunction.cc:50-83) or splitk_reduce_kernel
// (tnet_affine_fwd) -- the same slices, so both give the same Z bit for bit.
//
// Why a kernel of its own: 1024 x 135 over K = 1024 is 283 MFLOP -- 1.8 us of the chip's fp32 MFMA rate -- but only
// 48 64x64 output tiles, so the general GEMM's split-K tiles leave most CUs idle.  Here the work is cut into 16-row
// blocks x 4 K slices = 256 workgroups (one per CU at M = 1024), each 4 waves over up to 9 16x16 tiles of its K
// slice, both operands loaded straight into registers before the first MFMA; each writes its partial tile row-major
// into the split-K workspace [4][M][ldpart].
//
// (Round 5's full one-launch form -- the slices combined in the launch by the row block's last slice, softmax and
// slab sums there too -- measured slower than this + the combine launch, 19.7 vs 17.8 us, profiles/r05_top_rows.json,
// and is gone since round 6.)
#include <hip/hip_runtime.h>

#include <float.h>

#include "kcommon.h"

namespace tnetk {

namespace {
constexpr int kRows = 16;    // rows per block (one MFMA row tile)
constexpr int kSlices = 4;   // K slices
constexpr int kWaves = 4;    // waves per block
constexpr int kMaxCols = 144;

struct TopRowsP {
  const float* X;
  long ldx;
  const float* W;
  long ldw;
  int M, N, K, NT;  // NT: 16-column tiles
  float* part;      // [kSlices][M][ldpart]
  long ldpart;
};
}  // namespace

// block b: row block b / 4, slice b % 4 -- the blocks of one slice (the same 147 KB of W) run on two XCDs.
// Lane (lg, li) supplies A[li][k], B[k][li] with k = 16 c + 4 lg + s at the chunk's step s (the 16x16x4 kernels'
// lane map, gemm_f32.hip); wave wv takes 16-column tiles wv, wv + 4, wv + 8 (N <= 144).
template <int NCH>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void top_rows_kernel(const TopRowsP q) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int lg = lane >> 4, li = lane & 15;
  const int rb = blockIdx.x / kSlices, sl = blockIdx.x % kSlices;
  const int M = q.M, N = q.N;
  const int k0 = sl * NCH * 16;
  const int arow = min(rb * kRows + li, M - 1);
  const float* xa = q.X + (long)arow * q.ldx + k0 + 4 * lg;
  f32x4 a[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) a[c] = *reinterpret_cast<const f32x4*>(xa + 16 * c);
  f32x4 acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bf[3][NCH][4];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int col = min((wv + 4 * t) * 16 + li, N - 1);  // padding columns: a real column, never combined
    const float* wb = q.W + (long)(k0 + 4 * lg) * q.ldw + col;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int s = 0; s < 4; ++s) bf[t][c][s] = wb[(long)(16 * c + s) * q.ldw];
  }
  // Every load of the block issued before the first MFMA, and the MFMA chain free of anything else (only its
  // counted waits).  Without a fence the scheduler interleaves loads and MFMAs to save registers (60 instead of 275
  // VGPRs: 30.5 us for the top layer in the step); a sched_barrier alone keeps the loads ahead but lets spill reloads
  // and the stores' address arithmetic into the chain (12.4 us a launch).  What gives round 5's clean chain (8.6 us,
  // rocprofv3 in the MLP3 step, profiles/r06_top_rows_schedule.json): a memory-clobbering asm in its own basic block --
  // the branch is never taken (ldpart >= 16, checked by the launch) -- plus a sched_barrier behind the chain.
  if (q.ldpart < 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c][s], bf[t][c][s], acc[t], 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  // slice sl's rows 4 lg .. 4 lg + 3 of column (tile, li), row-major at part[sl][row][col] (every column of the
  // 16 NT is written, the padding ones from the clamped W column)
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
}

}  // namespace tnetk

using namespace tnetk;

// Which shapes the kernel takes: n_out <= 144, K = 512, 768 or 1024 (4 slices of 8, 12 or 16 chunks of 16 k, the
// chunks of A held in registers), at least 64 rows, 16-B aligned k-contiguous X.
extern "C" __attribute__((visibility("hidden"))) int tnetk_top_rows_shape_ok(const float* X, long ldx, const float* W,
                                                                            long ldw, int M, int N, int K) {
  // (W is read up to column 16 ceil(N / 16) - 1 clamped to N - 1: inside its rows)
  return N >= 1 && N <= kMaxCols && (K == 512 || K == 768 || K == 1024) && M >= 64 &&
         ((uintptr_t)X & 15) == 0 && (ldx & 3) == 0 && (long)M * ldx * 4 < (1L << 31) && ((uintptr_t)W & 15) == 0 &&
         (ldw & 3) == 0 && ldw >= 16L * ((N + 15) / 16);
}

// the 4 K slices' partial products into part [4][M][ldpart] (ldpart >= 16 ceil(N / 16))
extern "C" __attribute__((visibility("hidden"))) int tnetk_top_rows_partials(const float* X, long ldx, const float* W,
                                                                            long ldw, int M, int N, int K, float* part,
                                                                            long ldpart, void* stream) {
  if (!tnetk_top_rows_shape_ok(X, ldx, W, ldw, M, N, K) || !part || ldpart < 16L * ((N + 15) / 16))
    return TNET_ERR_UNSUPPORTED;
  if (4L * kSlices * M * ldpart >= (1L << 31)) return TNET_ERR_UNSUPPORTED;
  const hipStream_t st = (hipStream_t)stream;
  TopRowsP q{};
  q.X = X; q.ldx = ldx; q.W = W; q.ldw = ldw; q.M = M; q.N = N; q.K = K;
  q.NT = (N + 15) / 16;
  q.part = part; q.ldpart = ldpart;
  const int nrb = (M + kRows - 1) / kRows, nch = K / 64;
  const dim3 grid((unsigned)(nrb * kSlices));
  if (nch == 8) top_rows_kernel<8><<<grid, kWaves * 64, 0, st>>>(q);
  else if (nch == 12) top_rows_kernel<12><<<grid, kWaves * 64, 0, st>>>(q);
  else top_rows_kernel<16><<<grid, kWaves * 64, 0, st>>>(q);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}
