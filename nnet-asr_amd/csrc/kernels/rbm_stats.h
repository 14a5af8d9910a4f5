// rbm_stats.h -- the CD-1 statistics block of one RBM step (device code shared by reduce.hip's
// rbm_stats_kernel and gemm_f32.hip's weight-update + statistics launch).
#pragma once
#include "kcommon.h"

namespace tnetk {

constexpr int CS_COLS = 64;     // scalar path: columns per block (one per lane)
constexpr int CS_WAVES = 4;     // row sub-groups per block
constexpr int CS_ROWS = 32;     // rows per slab (8 per row sub-group: 8 loads in flight per lane)

__host__ __device__ static inline int cs_slabs(int rows) {
  int s = (rows + CS_ROWS - 1) / CS_ROWS;
  if (s > 256) s = 256;
  if (s < 1) s = 1;
  return s;
}

// One block of the slab column sums (reduce.hip colsum_partial_kernel; gemm_f32.hip's backward GEMM +
// slab-sum launch): partial[s][c] = sum of the rows of slab s in column c, row sub-group w (wave w) taking
// rows r0+w, r0+w+4, ..., the CS_WAVES sub-group sums added in order.  Block (bx, s): CS_COLS * CW columns
// from bx * CS_COLS * CW; `red`: CS_WAVES * CS_COLS * CW floats of the caller's LDS.
template <bool V4>
__device__ __forceinline__ void colsum_partial_block(const float* __restrict__ M, TnetMatrixDim d,
                                                     float* __restrict__ partial, int slabs, int neg_from, long ldp,
                                                     const int bx, const int s, float* __restrict__ red) {
  constexpr int CW = V4 ? 4 : 1;  // columns per lane
  constexpr int RW = CS_COLS * CW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = (bx * CS_COLS + lane) * CW;
  const int rows_per = (d.rows + slabs - 1) / slabs;
  const int r0 = s * rows_per, r1 = min(d.rows, r0 + rows_per);
  float acc[CW];
#pragma unroll
  for (int k = 0; k < CW; ++k) acc[k] = 0.f;
  if (c0 < d.cols) {
#pragma unroll 8
    for (int r = r0 + w; r < r1; r += CS_WAVES) {
      // rows from neg_from on enter negated (RBM: positive minus negative phase statistics)
      const float sg = r < neg_from ? 1.f : -1.f;
      if (V4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(M + (long)r * d.stride + c0);
#pragma unroll
        for (int k = 0; k < CW; ++k) acc[k] += sg * v[k];
      } else {
        acc[0] += sg * M[(long)r * d.stride + c0];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < CW; ++k) red[w * RW + lane * CW + k] = acc[k];
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int k = 0; k < CW; ++k) {
      const int c = c0 + k;
      if (c < d.cols) {
        float t = red[lane * CW + k];
#pragma unroll
        for (int q = 1; q < CS_WAVES; ++q) t += red[q * RW + lane * CW + k];
        partial[(long)s * ldp + c] = t;
      }
    }
  }
}

// CD-1 statistics of one RBM step in ONE launch (cuRbm.cc:148-164 bias updates + the TRbmCu
// reconstruction MSE, TRbmCu.cc:350), replacing two colsum_partial/colsum_final pairs and mse_kernel.
// Blocks [0, nvb) take 16 visible columns of Vs = [pos_vis; neg_vis] (rows from B on enter negated),
// the rest 16 hidden columns of Hs = [pos_hid; -neg_hid] (stored negated: every row adds).  Per column
// the sum runs exactly as colsum_partial + colsum_final do it: fp32 over the cs_slabs(rows) slabs (row
// sub-group g takes rows r0+g, r0+g+4, ...; the four sub-group sums added in order g = 0..3), slabs
// combined in fp64 in slab order -- bit-identical bias updates.  Lane 16g + j of a wave holds
// sub-group g of column j; the 4 waves take slabs round-robin; the slab sums meet in LDS.  The last
// blocks (from nvb + nhb on) add sum (neg_vis - pos_vis)^2 over RS_MROWS rows each to the MSE
// statistics (a row range per block: every load of a block in flight at once).
constexpr int RS_COLS = 16;
constexpr int RS_MAX_SLABS = 256;  // cs_slabs() cap
constexpr int RS_MROWS = 8;        // MSE rows per block
// LDS of one block: ts [RS_MAX_SLABS][RS_COLS] floats, then 4 doubles
constexpr int RS_SMEM_FLOATS = RS_MAX_SLABS * RS_COLS + 8;

// block `blk` of the statistics grid (256 threads) over the caller's LDS (RS_SMEM_FLOATS, 8-B aligned)
__device__ __forceinline__ void rbm_stats_block(const int blk, float* __restrict__ smem, const float* __restrict__ Vs,
                                                TnetMatrixDim dV, const float* __restrict__ Hs, TnetMatrixDim dH,
                                                int B, int nvb, float* __restrict__ vb, float* __restrict__ cvb,
                                                float* __restrict__ hb, float* __restrict__ chb, float scale,
                                                float mmt, double* __restrict__ stats, int nhb) {
  float (*ts)[RS_COLS] = reinterpret_cast<float (*)[RS_COLS]>(smem);
  double* dred = reinterpret_cast<double*>(smem + RS_MAX_SLABS * RS_COLS);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  if (blk >= nvb + nhb) {
    // ---- reconstruction MSE over rows [r0, r0 + RS_MROWS) of the visible statistics
    const int r0 = (blk - nvb - nhb) * RS_MROWS, nr = min(RS_MROWS, B - r0), C = dV.cols;
    constexpr int PER = 16;  // elements per thread per batch
    double e2 = 0.0;
    for (int i0 = 0; i0 < nr * C; i0 += 256 * PER) {
      float a[PER], b[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = min(i0 + (int)threadIdx.x + 256 * k, nr * C - 1), r = r0 + i / C, c = i % C;
        a[k] = Vs[(long)(B + r) * dV.stride + c];
        b[k] = Vs[(long)r * dV.stride + c];
      }
#pragma unroll
      for (int k = 0; k < PER; ++k)
        if (i0 + (int)threadIdx.x + 256 * k < nr * C) {
          const float e = a[k] - b[k];
          e2 += (double)(e * e);
        }
    }
    e2 = wave_sum_d(e2);
    if (lane == 0) dred[w] = e2;
    __syncthreads();
    if (threadIdx.x == 0)
      atomicAdd(stats + 2 * (blk % TNET_STATS_SLOTS), dred[0] + dred[1] + dred[2] + dred[3]);
    return;
  }
  const bool vis = blk < nvb;
  const float* M = vis ? Vs : Hs;
  const TnetMatrixDim d = vis ? dV : dH;
  const int neg_from = vis ? B : 0x7fffffff;
  const int c = (vis ? blk : blk - nvb) * RS_COLS + j;
  const bool cok = c < d.cols;
  const int slabs = cs_slabs(d.rows), rows_per = (d.rows + slabs - 1) / slabs;
  // a wave takes slabs w, w+4, ..., w+28 together (64 loads per lane in flight at 32-row slabs), then
  // the next eight; each slab's rows are still added in row order
  constexpr int SG = 8, RMAX = CS_ROWS / CS_WAVES;  // slabs per group, rows per sub-group at full slabs
  for (int s0 = w; s0 < slabs; s0 += 4 * SG) {
    float x[SG][RMAX];
#pragma unroll
    for (int q = 0; q < SG; ++q) {
      const int sl = s0 + 4 * q, r0 = sl * rows_per, r1 = min(d.rows, r0 + rows_per);
#pragma unroll
      for (int k = 0; k < RMAX; ++k) {
        const int r = r0 + g + CS_WAVES * k;
        x[q][k] = (cok && sl < slabs && r < r1 && k * CS_WAVES < rows_per) ? M[(long)r * d.stride + c] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < SG; ++q) {
      const int sl = s0 + 4 * q, r0 = sl * rows_per;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < RMAX; ++k) {
        const int r = r0 + g + CS_WAVES * k;
        acc += (r < neg_from ? 1.f : -1.f) * x[q][k];
      }
      // rows past the slab (k*4 >= rows_per or r >= r1) were loaded as 0: +-0 leaves acc unchanged
      // except the sign of a zero sum, which the +0 start already fixes as colsum_partial's
      const float a1 = __shfl(acc, j + 16, 64), a2 = __shfl(acc, j + 32, 64), a3 = __shfl(acc, j + 48, 64);
      if (g == 0 && sl < slabs) ts[sl][j] = ((acc + a1) + a2) + a3;
    }
  }
  __syncthreads();
  if (w == 0 && g == 0 && cok) {  // colsum_final_kernel mode 3
    double sum = 0.0;
    for (int sl = 0; sl < slabs; ++sl) sum += (double)ts[sl][j];
    float* bv = vis ? vb : hb;
    float* cv = vis ? cvb : chb;
    const float gr = mmt * cv[c] + scale * (float)sum;
    cv[c] = gr;
    bv[c] = bv[c] + gr;
  }
}

}  // namespace tnetk
