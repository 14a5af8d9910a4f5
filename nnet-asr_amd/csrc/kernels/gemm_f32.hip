// gemm_f32.hip -- fp32 GEMM on the gfx950 matrix cores (v_mfma_f32_32x32x2_f32) with fused
// epilogues for the TNet affine layer (CuBiasedLinearity, src/CuTNetLib/cuBiasedLinearity.cc).
//
// Replaces cublasSgemm (src/CuBaseLib/cumatrix.tcc:336-370) plus the element-wise kernels the
// reference runs around it (_add_scaled_row, _sigmoid, _diff_sigmoid, _add_scaled;
// src/CuBaseLib/cukernels.cu:87-217).
//
// Design (MI355X-first):
//  * f32-in / f32-acc MFMA 32x32x2: lane l supplies A[i=l&31][kh=l>>5], B[kh][j=l&31]; the two
//    k-slots of one MFMA are mapped to real k = kk + 4*kh + s for step s = 0..3 of an 8-deep k
//    chunk, which lets a k-contiguous operand feed 4 MFMAs from one ds_read_b128 while an
//    m/n-contiguous operand feeds them with conflict-free ds_read_b32 -- so every operand layout
//    (NN forward, NT backward, TN weight gradient) is staged straight from coalesced 16-B global
//    loads, no transposes.
//  * operand k-tiles stream global -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR staging)
//    into an S-slot ring with S-1 tiles in flight and ONE raw s_barrier per k-tile behind a
//    counted vmcnt (cdna_hip_programming.md section 5, "Pipelining across barriers");
//  * k-contiguous operand images are [rows][BK] with the 16-B chunk index XOR-swizzled per row
//    (the DMA image is lane-linear, so the swizzle goes on the per-lane SOURCE address and is
//    undone on the ds_read_b128, rule 21): every 16-lane group of ds_read_b128 hits 16 distinct
//    4-bank slots.  Row-contiguous images are plain [BK][cols] read with conflict-free b32;
//  * blockIdx -> tile: bijective XCD-contiguous remap (T1) followed by a grouped order (GROUP
//    tile-rows, column-major inside a group), so the ~64 workgroups resident on one XCD cover a
//    square-ish block of C and its L2 holds few A and B panels;
//  * the whole epilogue (bias, sigmoid, diff-sigmoid, momentum-SGD) is fused into the stores.
#include <float.h>

#include <cstdlib>
#include <array>
#include <cstring>
#include <initializer_list>
#include <map>
#include <mutex>
#include <unordered_map>
#include <type_traits>

#include "kcommon.h"
#include "rbm_stats.h"
#include "gather.h"

namespace tnetk {

// EPI_BIAS_NSIG / EPI_BIAS_NEG store the negated activation (the RBM negative phase enters the
// stacked statistics with a minus sign); EPI_RBM is the CD-1 weight update of CuRbm::RbmUpdate
// (cuRbm.cc:133-174): c = mmt*corr + scale*acc + l2*W ; corr = c ; W += c
enum { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_SIG = 2, EPI_DSIG = 3, EPI_SGD = 4, EPI_BIAS_NSIG = 5,
       EPI_BIAS_NEG = 6, EPI_RBM = 7,
       // fused bias gradient (16x16 kernel): EPI_DSIG_CS = EPI_DSIG + per-32-row-slab column sums of the
       // output (the bias gradient of the layer below); EPI_SGD_B = EPI_SGD + that layer's bias SGD from
       // the slab sums, done by the first tile-row's workgroups in the prologue
       EPI_DSIG_CS = 8, EPI_SGD_B = 9,
       // data-parallel gradient: EPI_STORE of X^T E plus the raw bias gradient from the slab sums
       EPI_STORE_BG = 10,
       // RBM positive phase: EPI_BIAS_SIG, then the workgroup samples its tile (states = y > U, U the
       // elements' HybridTaus draws) -- CuRand::BinarizeProbs fused into the launch
       EPI_BIAS_SIG_BIN = 11 };
constexpr int kColsumSlabRows = 32;
constexpr int kMaxSplit = 8;  // split-K slices at most
// base epilogue of a fused one
constexpr int epi_base(int e) {
  return e == EPI_DSIG_CS ? EPI_DSIG : e == EPI_SGD_B ? EPI_SGD : e == EPI_STORE_BG ? EPI_STORE
       : e == EPI_BIAS_SIG_BIN ? EPI_BIAS_SIG : e;
}
// epilogues that also produce the bias (SGD update or raw gradient) from slab sums
constexpr bool epi_bias_slabs(int e) { return e == EPI_SGD_B || e == EPI_STORE_BG; }

struct GemmP {
  int M, N, K;
  const float* A; long lda;
  const float* B; long ldb;
  float* C; long ldc;
  float alpha, beta;
  const float* bias;            // EPI_BIAS*: [N]
  const float* aux; long ldaux; // EPI_DSIG: y of the layer below [M x N]
  float* corr; long ldcorr;     // EPI_SGD: momentum buffer (nullable)
  float scale, mmt, l2;         // EPI_SGD
  float* cpart; long ldcpart;   // EPI_DSIG_CS: [cdiv(M,32)][N] column sums of the output per 32-row slab
  const float* bpart; long ldbpart; int bslabs;  // EPI_SGD_B: bias-gradient slab sums [bslabs][N]
  float* bvec; float* bcorr;    // EPI_SGD_B: bias [N] and its momentum buffer (nullable); EPI_STORE_BG: gradient out
  float bscale, bmmt;           // EPI_SGD_B
  int group;                    // tile-rows per group of the blockIdx -> tile order
  int diag_noload;              // diagnostics only: skip the k-loop's global loads (wrong results)
  // split-K (gemm16_kernel, blockIdx.y = split z): the split reads A + z*kstepA, B + z*kstepB over
  // K = its own depth and stores its partial product to C + z*slabC (EPI_STORE, alpha 1, beta 0)
  int ksplit;
  long kstepA, kstepB, slabC;
  int early_issue;  // gemm16_kernel prologue: issue all S ring slots before the first wait (TNET_GEMM_EARLY)
  int wt;           // gemm16_kernel epilogue: 16-B output stores write-through (sc1) (TNET_GEMM_WT)
  // per-tile counters (stream-K pieces, split2): see those kernels
  unsigned* tile_cnt;
  // EPI_BIAS_SIG_BIN: sampled states [M x N] (row stride ldbin) and the four HybridTaus state arrays,
  // indexed row * ldc + col like the probabilities C (the reference indexes them with C's MatrixDim)
  float* bin; long ldbin;
  unsigned* rz[4];
  // stream-K piece (gemm16_body EPI_T >= kEpiStreamK, gemm16_sk_kernel): ksplit = the tile's piece count
  // (1 or 2); the first of a split tile's pieces to finish stores its accumulators to skws + tile * BM * BN
  // (fragment order), the second adds them to its own and runs the tile's epilogue (tile_cnt[tile])
  float* skws;
  // EPI_SGD / EPI_SGD_B (gemm16_body only): the updated W also stored transposed, Ct[col][row] (row stride ldct):
  // the weight's shadow that the next step's backward GEMM reads n-contiguous (tnet_weight_shadow)
  float* Ct; long ldct;
};


// ---- epilogue: C/D map of 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
template <int TM, int TN, int EPI>
__device__ __forceinline__ void epilogue(const GemmP& p, f32x16 (&acc)[TM][TN], int bm, int bn, int wm0, int wn0,
                                         int li, int lh) {
  const int M = p.M, N = p.N;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = bn + wn0 + b * 32 + li;
      if (col >= N) continue;
      float bias_v = 0.f;
      if (EPI == EPI_BIAS || EPI == EPI_BIAS_SIG || EPI == EPI_BIAS_NSIG || EPI == EPI_BIAS_NEG) bias_v = p.bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = bm + wm0 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row >= M) continue;
        float* cp = p.C + (long)row * p.ldc + col;
        const float v = acc[a][b][r];
        if (EPI == EPI_STORE) {
          *cp = (p.beta == 0.f) ? p.alpha * v : p.alpha * v + p.beta * *cp;
        } else if (EPI == EPI_BIAS) {
          *cp = v + bias_v;
        } else if (EPI == EPI_BIAS_SIG) {
          *cp = sigmoidf_ref(v + bias_v);
        } else if (EPI == EPI_BIAS_NSIG) {
          *cp = -sigmoidf_ref(v + bias_v);
        } else if (EPI == EPI_BIAS_NEG) {
          *cp = -(v + bias_v);
        } else if (EPI == EPI_DSIG) {
          const float y = p.aux[(long)row * p.ldaux + col];
          *cp = y * (1.f - y) * v;
        } else if (EPI == EPI_RBM) {
          float* qp = p.corr + (long)row * p.ldcorr + col;
          const float w = *cp;
          const float c = p.mmt * *qp + p.scale * v + p.l2 * w;
          *qp = c;
          *cp = w + c;
        } else {  // EPI_SGD
          float c = v;
          if (p.corr) {
            float* qp = p.corr + (long)row * p.ldcorr + col;
            c = v + p.mmt * *qp;
            *qp = c;
          }
          float w = *cp;
          w = w + p.scale * c;
          w = w + p.l2 * w;
          *cp = w;
        }
      }
    }
  }
}


// ---- EPI_SGD_B: the workgroups of the first tile-row (bm == 0) also update the bias of their BN
// columns.  g = the fp32 slab sums added in fp64, in slab order (the reference accumulates the column
// sum in double, _add_col_sum cukernels.cu:147-164); then corr = g + mmt*corr ; b += scale*corr
// (cuBiasedLinearity.cc:46-64).  The first 32 slab sums, b and corr are loaded into registers right
// after the prologue (bias_pre_load) so their latency hides under the main loop; the sum and the
// stores happen at the epilogue (bias_pre_finish).  Column c of the WG is thread c (BN <= NT).
constexpr int kBiasPreSlabs = 32;
struct BiasPre {
  float v[kBiasPreSlabs];
  float b, q;
};
template <int BN, bool GRAD>
__device__ __forceinline__ void bias_pre_load(const GemmP& p, int bn, BiasPre& bp) {
  const int col = bn + (int)threadIdx.x;
  if ((int)threadIdx.x >= BN || col >= p.N) return;
#pragma unroll
  for (int k = 0; k < kBiasPreSlabs; ++k) bp.v[k] = k < p.bslabs ? p.bpart[(long)k * p.ldbpart + col] : 0.f;
  if (GRAD) return;  // EPI_STORE_BG: the raw gradient, no bias read
  bp.b = p.bvec[col];
  bp.q = p.bcorr ? p.bcorr[col] : 0.f;
}
template <int BN, bool GRAD>
__device__ __forceinline__ void bias_pre_finish(const GemmP& p, int bn, const BiasPre& bp) {
  const int col = bn + (int)threadIdx.x;
  if ((int)threadIdx.x >= BN || col >= p.N) return;
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < kBiasPreSlabs; ++k) s += (double)bp.v[k];
  for (int k = kBiasPreSlabs; k < p.bslabs; ++k) s += (double)p.bpart[(long)k * p.ldbpart + col];
  float g = (float)s;
  if (GRAD) {
    p.bvec[col] = g;
    return;
  }
  if (p.bcorr) {
    g = g + p.bmmt * bp.q;
    p.bcorr[col] = g;
  }
  p.bvec[col] = bp.b + p.bscale * g;
}

// ---- split-K combine of 4 columns of one row: C = epilogue(P[0] + ... + P[splits-1]) summed in
// slice order (fixed: deterministic), with gemm16_kernel's epilogue arithmetic (EPI = a base epilogue)
template <int EPI>
__device__ __forceinline__ void combine4(const GemmP& p, const float* __restrict__ P, long slab, int splits, int ldp,
                                         int row, int col) {
  const float* q = P + (long)row * ldp + col;
  float* cp = p.C + (long)row * p.ldc + col;
  const int nv = min(4, p.N - col);
  const bool full = nv == 4;
  // the epilogue's operands first (W / corr, Y below, C, bias): independent of the slices, so every
  // load of the thread is in flight before the first add -- 16-byte where the 4 columns are live
  constexpr bool BIAS = EPI == EPI_BIAS || EPI == EPI_BIAS_SIG || EPI == EPI_BIAS_NSIG || EPI == EPI_BIAS_NEG;
  const float* asrc = nullptr;
  if constexpr (EPI == EPI_DSIG) asrc = p.aux + (long)row * p.ldaux + col;
  else if constexpr (EPI == EPI_STORE) asrc = p.beta != 0.f ? cp : nullptr;
  else if constexpr (EPI == EPI_SGD || EPI == EPI_RBM) asrc = cp;
  float* qsrc = (EPI == EPI_SGD || EPI == EPI_RBM) && p.corr ? p.corr + (long)row * p.ldcorr + col : nullptr;
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, qv = {0.f, 0.f, 0.f, 0.f}, bb = {0.f, 0.f, 0.f, 0.f};
  auto ld4 = [&](const float* src, f32x4& d) {
    if (full) {
      d = *reinterpret_cast<const f32x4*>(src);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (e < nv) d[e] = src[e];
    }
  };
  if (asrc) ld4(asrc, a);
  if (qsrc) ld4(qsrc, qv);
  if constexpr (BIAS)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (e < nv) bb[e] = p.bias[col + e];
  // every slice's load in flight before the first add (splits <= kMaxSplit)
  f32x4 t[kMaxSplit];
#pragma unroll
  for (int z = 0; z < kMaxSplit; ++z)
    if (z < splits) t[z] = *reinterpret_cast<const f32x4*>(q + z * slab);
  f32x4 v = t[0];
#pragma unroll
  for (int z = 1; z < kMaxSplit; ++z)
    if (z < splits)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = v[e] + t[z][e];
  f32x4 o = {0.f, 0.f, 0.f, 0.f}, qn = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x = v[e];
    if constexpr (EPI == EPI_STORE) {
      o[e] = (p.beta == 0.f) ? p.alpha * x : p.alpha * x + p.beta * a[e];
    } else if constexpr (BIAS) {
      const float y = x + bb[e];
      o[e] = EPI == EPI_BIAS ? y : EPI == EPI_BIAS_SIG ? sigmoidf_ref(y) : EPI == EPI_BIAS_NSIG ? -sigmoidf_ref(y) : -y;
    } else if constexpr (EPI == EPI_DSIG) {
      const float y = a[e];
      o[e] = y * (1.f - y) * x;
    } else if constexpr (EPI == EPI_RBM) {
      const float w = a[e];
      const float c = p.mmt * qv[e] + p.scale * x + p.l2 * w;
      qn[e] = c;
      o[e] = w + c;
    } else if constexpr (EPI == EPI_SGD) {
      float c = x;
      if (qsrc) c = x + p.mmt * qv[e];
      qn[e] = c;
      float w = a[e];
      w = w + p.scale * c;
      w = w + p.l2 * w;
      o[e] = w;
    }
  }
  if (full && p.wt) {  // write-through (kcommon.h st_wt); launch_splitk checks the 2^31-byte offsets
    st_wt(tile_rsrc(p.C), (long)row * p.ldc + col, o);
    if (qsrc) st_wt(tile_rsrc(p.corr), (long)row * p.ldcorr + col, qn);
  } else if (full) {
    *reinterpret_cast<f32x4*>(cp) = o;
    if (qsrc) *reinterpret_cast<f32x4*>(qsrc) = qn;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (e < nv) {
        cp[e] = o[e];
        if (qsrc) qsrc[e] = qn[e];
      }
  }
}

// EPI_BIAS_SIG_BIN: after the tile's probabilities are stored, the workgroup reads them back (its own
// stores: drained + barrier) with every element's four generator states, draws U and writes the
// sampled state and the advanced generator states (rand.hip rand_kernel<2>'s arithmetic per element)
template <int BM, int BN, int NT>
__device__ __forceinline__ void binarize_tile(const GemmP& p, int bm, int bn) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // elements per thread per batch (5 loads each in flight): the whole tile in one batch up to 64x128
  constexpr int PER = (BM * BN / NT) < 32 ? (BM * BN / NT > 0 ? BM * BN / NT : 1) : 32;
  for (int u0 = 0; u0 < BM * BN; u0 += NT * PER) {
    float pr[PER];
    unsigned z[4][PER];
    long si[PER];
    bool ok[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int u = u0 + (int)threadIdx.x + NT * k, row = bm + u / BN, col = bn + u % BN;
      ok[k] = u < BM * BN && row < p.M && col < p.N;
      const int rr = ok[k] ? row : 0, cc = ok[k] ? col : 0;
      si[k] = (long)rr * p.ldc + cc;
      pr[k] = p.C[si[k]];
#pragma unroll
      for (int q = 0; q < 4; ++q) z[q][k] = p.rz[q][si[k]];
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (!ok[k]) continue;
      const int u = u0 + (int)threadIdx.x + NT * k, row = bm + u / BN, col = bn + u % BN;
      unsigned a = z[0][k], b = z[1][k], c = z[2][k], e = z[3][k];
      const float x = hybrid_taus(a, b, c, e);
      p.bin[(long)row * p.ldbin + col] = pr[k] > x ? 1.0f : 0.0f;
      p.rz[0][si[k]] = a;
      p.rz[1][si[k]] = b;
      p.rz[2][si[k]] = c;
      p.rz[3][si[k]] = e;
    }
  }
}

// =============================================================================================
// LDS-DMA pipelined GEMM.  BMxBN workgroup tile, BK k-depth per ring slot, WMxWN waves each
// owning (BM/WM)x(BN/WN) = TMxTN blocks of 32x32 MFMA accumulators.
//   * rows / columns beyond M / N are clamped to valid memory (their products only reach outputs
//     that are never stored); a partial last k-tile (K % BK) goes through a masked register path.
// =============================================================================================
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  // gfx9 s_waitcnt simm16: vmcnt[3:0], expcnt[6:4], lgkmcnt[11:8], vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | (((N >> 4) & 0x3) << 14));
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n <= N (the immediate must be a constant)
template <int N>
__device__ __forceinline__ void wait_vmcnt_le(int n) {
  if constexpr (N <= 0) {
    wait_vmcnt<0>();
  } else {
    if (n >= N) wait_vmcnt<N>();
    else wait_vmcnt_le<N - 1>(n);
  }
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n in [LO, HI] (binary search over the immediates)
template <int LO, int HI>
__device__ __forceinline__ void wait_vmcnt_bin(int n) {
  if constexpr (LO >= HI) {
    wait_vmcnt<LO>();
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (n <= MID) wait_vmcnt_bin<LO, MID>(n);
    else wait_vmcnt_bin<MID + 1, HI>(n);
  }
}

// XOR swizzle of the 16-B chunk index of row r of a k-contiguous [rows][BK] image.
//   BK = 32: rows are 128 B, two per 256-B bank row -> ((r >> 1) & 7) over the 8 chunks;
//   BK = 64: rows are 256 B, one per bank row        -> (r & 15) over the 16 chunks.
template <int BK>
__device__ __forceinline__ int swz(int r) {
  return BK == 32 ? ((r >> 1) & 7) : (r & 15);
}

template <int BM, int BN, int BK, int WM, int WN, int S, int IL, bool A_KC, bool B_KC, int EPI>
__global__ __launch_bounds__(WM * WN * 64) void gemm_f32_glds_kernel(const GemmP p) {
  constexpr int NT = WM * WN * 64, NW = WM * WN;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1 && BM == TM * WM * 32 && BN == TN * WN * 32, "32x32 MFMA blocks per wave");
  static_assert(BK == 32 || BK == 64, "BK");
  constexpr int CH = BK / 4;  // 16-B chunks per k-contiguous row
  constexpr int A_SZ = BM * BK, B_SZ = BN * BK, ST_SZ = A_SZ + B_SZ;
  constexpr int GA = A_SZ / 4 / NT, GB = B_SZ / 4 / NT, G = GA + GB;  // DMA instructions per thread per tile
  static_assert(A_SZ % (4 * NT) == 0 && B_SZ % (4 * NT) == 0, "tile splits into 1-KiB wave pieces");
  static_assert(2 * G < 64, "vmcnt range");
  __shared__ __attribute__((aligned(16))) float smem[S * ST_SZ];

  const int M = p.M, N = p.N, K = p.K;
  const int nbn = (N + BN - 1) / BN, nbm = (M + BM - 1) / BM;
  const int nwg = nbm * nbn;
  // bijective XCD remap: the blocks one XCD receives (bid % 8) take a contiguous range of L ...
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int L = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  // ... and that range is walked in groups of `group` tile-rows, column-major inside a group
  const int grp = p.group, per_group = grp * nbn;
  const int first_m = (L / per_group) * grp;
  const int gsz = min(nbm - first_m, grp);
  const int bm = (first_m + (L % per_group) % gsz) * BM, bn = ((L % per_group) / gsz) * BN;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm0 = (wid / WN) * (BM / WM), wn0 = (wid % WN) * (BN / WN);
  const int li = lane & 31, lh = lane >> 5;

  // per-lane source offsets (elements) of each DMA piece, relative to the k-tile origin
  long srcA[GA], srcB[GB];
#pragma unroll
  for (int g = 0; g < GA; ++g) {
    const int u = (g * NW + wid) * 64 + lane;  // 16-B unit index inside the image
    if (A_KC) {
      const int r = u / CH, j = u % CH;
      srcA[g] = (long)min(bm + r, M - 1) * p.lda + 4 * (j ^ swz<BK>(r));
    } else {
      const int k = u / (BM / 4), c = (u % (BM / 4)) * 4;
      srcA[g] = (long)k * p.lda + (bm + c < M ? bm + c : 0);
    }
  }
#pragma unroll
  for (int g = 0; g < GB; ++g) {
    const int u = (g * NW + wid) * 64 + lane;
    if (B_KC) {
      const int r = u / CH, j = u % CH;
      srcB[g] = (long)min(bn + r, N - 1) * p.ldb + 4 * (j ^ swz<BK>(r));
    } else {
      const int k = u / (BN / 4), c = (u % (BN / 4)) * 4;
      srcB[g] = (long)k * p.ldb + (bn + c < N ? bn + c : 0);
    }
  }

  auto issue_piece = [&](int t, int g) {  // DMA piece g (A pieces first) of k-tile t into slot t % S
    float* st = smem + (t % S) * ST_SZ;
    if (g < GA) {
      const long ka = A_KC ? (long)t * BK : (long)t * BK * p.lda;
      __builtin_amdgcn_global_load_lds((const void*)(p.A + ka + srcA[g]), (void*)(st + (g * NW + wid) * 256), 16, 0,
                                       0);
    } else {
      const int h = g - GA;
      const long kb = B_KC ? (long)t * BK : (long)t * BK * p.ldb;
      __builtin_amdgcn_global_load_lds((const void*)(p.B + kb + srcB[h]), (void*)(st + A_SZ + (h * NW + wid) * 256),
                                       16, 0, 0);
    }
  };
  auto issue = [&](int t) {  // DMA of full k-tile t into ring slot t % S
    float* st = smem + (t % S) * ST_SZ;
    const long ka = A_KC ? (long)t * BK : (long)t * BK * p.lda;
    const long kb = B_KC ? (long)t * BK : (long)t * BK * p.ldb;
#pragma unroll
    for (int g = 0; g < GA; ++g)
      __builtin_amdgcn_global_load_lds((const void*)(p.A + ka + srcA[g]), (void*)(st + (g * NW + wid) * 256), 16, 0,
                                       0);
#pragma unroll
    for (int g = 0; g < GB; ++g)
      __builtin_amdgcn_global_load_lds((const void*)(p.B + kb + srcB[g]), (void*)(st + A_SZ + (g * NW + wid) * 256),
                                       16, 0, 0);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  // k of MFMA step s (0..3) of 8-deep chunk kc is 8kc + 4*kh + s (kh = lane >> 5), so a
  // k-contiguous operand feeds 4 MFMAs from one ds_read_b128.  Fragments live in a 4-deep
  // register ring (chunk c -> buffer c % 4) and are read TWO chunks ahead of their MFMAs --
  // across k-tile boundaries too -- so an MFMA never waits on an LDS read issued just before it,
  // even where the compiler's waitcnt is a conservative lgkmcnt(0).
  constexpr int KC = BK / 8, NB = 4;
  static_assert(KC % NB == 0, "chunk -> buffer mapping is per tile");
  float av[NB][TM][4], bv[NB][TN][4];
  auto read_frags = [&](const float* st, int kc, int buf) {  // chunk kc of the slot at st
    const float* As = st;
    const float* Bs = st + A_SZ;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int row = wm0 + a * 32 + li;
      if (A_KC) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(As + row * BK + 4 * ((2 * kc + lh) ^ swz<BK>(row)));
        av[buf][a][0] = x[0]; av[buf][a][1] = x[1]; av[buf][a][2] = x[2]; av[buf][a][3] = x[3];
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) av[buf][a][s] = As[(8 * kc + 4 * lh + s) * BM + row];
      }
    }
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = wn0 + b * 32 + li;
      if (B_KC) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(Bs + col * BK + 4 * ((2 * kc + lh) ^ swz<BK>(col)));
        bv[buf][b][0] = x[0]; bv[buf][b][1] = x[1]; bv[buf][b][2] = x[2]; bv[buf][b][3] = x[3];
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) bv[buf][b][s] = Bs[(8 * kc + 4 * lh + s) * BN + col];
      }
    }
  };
  auto mfmas = [&](int buf) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[buf][a][s], bv[buf][b][s], acc[a][b], 0, 0, 0);
  };
  // diagnostics only (wrong results): bit 0 no global loads in the k-loop, bit 1 no barriers,
  // bit 2 no LDS fragment reads after the first
  const bool noload = (p.diag_noload & 1) != 0, nobar = (p.diag_noload & 2) != 0,
             noread = (p.diag_noload & 4) != 0;
  auto slot = [&](int t) { return smem + ((noload ? 0 : t) % S) * ST_SZ; };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    if (!nobar) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  const int nfull = K / BK;
  // IL = 0: the DMA of k-tile t+S is issued in one burst right after the hand-over barrier.
  // IL = 1: its G pieces are spread over the next KC chunks (piece group c = (kc + 2) % KC), one
  //         group per MFMA chunk, so each wave's DMA issue hides under MFMAs (T3 interleave).
  //         The prologue then issues tiles 0..S-2 plus the first half of tile S-1's pieces.
  constexpr int GH = IL ? (2 * G) / KC : 0;  // pieces of the newest tile issued before its hand-over
  auto pieces_of = [&](int c, int& g0, int& g1) { g0 = c * G / KC; g1 = (c + 1) * G / KC; };
#pragma unroll
  for (int t = 0; t < S - 1; ++t)
    if (t < nfull) issue(t);
  if (IL && S - 1 < nfull)
#pragma unroll
    for (int g = 0; g < GH; ++g) issue_piece(S - 1, g);
  static_assert(EPI != EPI_DSIG_CS, "column sums: 16x16 kernel only");
  static_assert(!epi_bias_slabs(EPI) || BN <= NT, "one thread per bias column");
  BiasPre bpre;
  if constexpr (epi_bias_slabs(EPI))
    if (bm == 0) bias_pre_load<BN, EPI == EPI_STORE_BG>(p, bn, bpre);
  if (nfull > 0) {
    // tile 0 must land; younger DMAs in flight: full tiles 1..S-2 (+ GH pieces of tile S-1)
    int younger = (min(S - 2, nfull - 1)) * G + ((IL && S - 1 < nfull) ? GH : 0);
    wait_vmcnt_le<3 * G + GH>(younger);
    barrier();  // tile 0 landed in every wave's pieces
    if (!IL && S - 1 < nfull && !noload) issue(S - 1);
    read_frags(slot(0), 0, 0);
    read_frags(slot(0), 1, 1);
    if (noread) {
      read_frags(slot(0), 2, 2);
      read_frags(slot(0), 3, 3);
    }
  }
  for (int t = 0; t < nfull; ++t) {
    const float* st = slot(t);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int nk = kc + 2;  // chunk whose fragments are read under this chunk's MFMAs
      if (noread) {
      } else if (nk < KC) {
        read_frags(st, nk, nk % NB);
      } else if (t + 1 < nfull) {
        if (nk == KC) {
          // hand over to tile t+1: this wave's reads of tile t are done (lgkmcnt 0), tile t+1
          // has landed (vmcnt: only tiles t+2..t+S-1 may stay in flight), and after the barrier
          // no wave reads tile t any more, so its slot takes the DMA of tile t+S
          __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
          wait_vmcnt_le<3 * G + GH>(min(S - 2, nfull - 2 - t) * G);
          barrier();
          if (!IL && t + S < nfull && !noload) issue(t + S);
        }
        read_frags(slot(t + 1), nk - KC, nk % NB);
      }
      if (IL && !noload) {
        const int T = (kc >= KC - 2) ? t + S : t + S - 1;  // tile whose pieces this chunk issues
        if (T < nfull && (kc < KC - 2 || t + 1 < nfull)) {
          int g0, g1;
          pieces_of((kc + 2) % KC, g0, g1);
#pragma unroll
          for (int g = 0; g < G; ++g)
            if (g >= g0 && g < g1) issue_piece(T, g);
        }
      }
      mfmas(kc % NB);
    }
  }
  if (K % BK) {
    // masked tail k-tile through registers, same swizzled image, in slot nfull % S
    __builtin_amdgcn_s_barrier();
    float* st = smem + (nfull % S) * ST_SZ;
    const int k0 = nfull * BK;
    for (int u = threadIdx.x; u < A_SZ / 4; u += NT) {
      int gr, gc;
      if (A_KC) { const int r = u / CH, j = u % CH; gr = bm + r; gc = k0 + 4 * (j ^ swz<BK>(r)); }
      else { const int k = u / (BM / 4); gr = k0 + k; gc = bm + (u % (BM / 4)) * 4; }
      const int rmax = A_KC ? M : K, cmax = A_KC ? K : M;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (gr < rmax) {
        const float* q = p.A + (long)gr * p.lda + gc;
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = (gc + e < cmax) ? q[e] : 0.f;
      }
      *reinterpret_cast<f32x4*>(st + u * 4) = x;
    }
    for (int u = threadIdx.x; u < B_SZ / 4; u += NT) {
      int gr, gc;
      if (B_KC) { const int r = u / CH, j = u % CH; gr = bn + r; gc = k0 + 4 * (j ^ swz<BK>(r)); }
      else { const int k = u / (BN / 4); gr = k0 + k; gc = bn + (u % (BN / 4)) * 4; }
      const int rmax = B_KC ? N : K, cmax = B_KC ? K : N;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (gr < rmax) {
        const float* q = p.B + (long)gr * p.ldb + gc;
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = (gc + e < cmax) ? q[e] : 0.f;
      }
      *reinterpret_cast<f32x4*>(st + A_SZ + u * 4) = x;
    }
    __syncthreads();
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      read_frags(st, kc, kc % NB);
      mfmas(kc % NB);
    }
  }
  if constexpr (epi_bias_slabs(EPI))
    if (bm == 0) bias_pre_finish<BN, EPI == EPI_STORE_BG>(p, bn, bpre);
  epilogue<TM, TN, epi_base(EPI)>(p, acc, bm, bn, wm0, wn0, li, lh);
  if constexpr (EPI == EPI_BIAS_SIG_BIN) binarize_tile<BM, BN, WM * WN * 64>(p, bm, bn);
}


// ---- diagnostic clock stamps (separate build: make stamp -> lib/libtnet_amd_stamp.so; the product
// library has none; the stamp build's ablations TNET_GEMM_DIAG_NODMA / _NOREAD / _NOBAR drop the
// main loop's LDS-DMA pieces / fragment reads / seam barriers -- wrong results, timing only).  Wave 0 of every workgroup records s_memtime (shader clock) at kernel entry,
// after the prologue, after the main loop and after the epilogue, and s_memrealtime (100 MHz) at
// entry and exit, into a buffer no other code reads (MI355X_MICROARCH.md 'DVFS give-back' item 6).
#ifdef TNET_GEMM_STAMP
__device__ unsigned long long g_tnet_stamps[8192 * 6];
#define TNET_STAMP(i)                                                                   \
  do {                                                                                  \
    const unsigned long long tt_ = __builtin_amdgcn_s_memtime();                        \
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_tnet_stamps[blockIdx.x * 6 + (i)] = tt_; \
  } while (0)
#define TNET_STAMP_RT(i)                                                                \
  do {                                                                                  \
    const unsigned long long tt_ = __builtin_amdgcn_s_memrealtime();                    \
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_tnet_stamps[blockIdx.x * 6 + (i)] = tt_; \
  } while (0)
#else
#define TNET_STAMP(i) do { } while (0)
#define TNET_STAMP_RT(i) do { } while (0)
#endif

// V consecutive floats from LDS (ds_read_b128 / b64 / b32) into x[0..V)
template <int V>
__device__ __forceinline__ void lds_vec(const float* p, float (&x)[4]) {
  if constexpr (V == 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p);
    x[0] = v[0]; x[1] = v[1]; x[2] = v[2]; x[3] = v[3];
  } else if constexpr (V == 2) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    x[0] = v.x; x[1] = v.y;
  } else {
    x[0] = *p;
  }
}

// =============================================================================================
// 16x16x4 variant (v_mfma_f32_16x16x4_f32: 32 cycles per 1024 MACs; on this part it sustains a
// higher clock than the 32x32x2 form -- tools/mfma_peak.hip: ~155 vs ~137-145 TFLOP/s).
//   * lane l = 16*g + i supplies A[i][k] / B[k][i] with k = 16c + 4g + s for step s = 0..3 of a
//     16-deep chunk c; D row = 4g + r (reg r), col = i.
//   * k-contiguous operand: one ds_read_b128 per 16x16 tile per chunk = the 4 steps' k values
//     (swizzled image as above).
//   * m/n-contiguous operand: one ds_read_b128 per step per FOUR tiles -- the 4 consecutive floats
//     feed 4 interleaved tiles (tile 4q+e holds rows/cols 64q + 4i + e), so every LDS read is a
//     conflict-free b128 and, for an n-contiguous B, the epilogue stores 4 consecutive columns
//     per lane as one 16-B store.
// =============================================================================================
//   * SP = 1 (S >= 3): the G LDS-DMA pieces of tile t+S-1 are issued spread over tile t's chunks
//     (about G/KCH per chunk, between the fragment reads and the chunk's MFMAs) instead of all at
//     the tile seam, and the MFMA block runs at s_setprio 1 (an 8-wave workgroup's partner wave
//     then fills the other wave's seams).
//   * SP = 2: one extra LOADER wave issues every LDS-DMA piece; the WMxWN compute waves only read
//     fragments and issue MFMAs.  An LDS-DMA instruction holds its issuing wave for ~20-30 cycles
//     (tools/gemm_clock.py ablation: dropping the compute waves' pieces cut the 2048^2 main loop by
//     8 %), which the loader now absorbs on its own wave slot.  Same ring protocol: the loader waits
//     for tile t+1 (counted vmcnt), meets the compute waves at the seam barrier, then refills the
//     slot of tile t.  MEASURED SLOWER (2048^2 main loop 185k vs 149k cycles): the issue cost is paid
//     by the loader's SIMD, whose compute wave then trails the other three at every seam barrier --
//     kept as one config (m64x128k64s2L) for the record, not chosen by the heuristic.
// EPI_T >= kEpiStreamK: a stream-K piece (gemm16_sk_kernel) whose tile epilogue is EPI_T - kEpiStreamK
constexpr int kEpiStreamK = 64;
// PX (exact prefetch): the tile grid covers M x N exactly and the epilogue operands are 16-B aligned
// (launch_cfg checks), so the epilogue-operand prefetch is a known number of unconditional loads per
// wave and the first seam waits for the ring only, not for them (TNET_GEMM_PRE0=0: off)
// The body of one workgroup (tile bid_x of the grid) over the caller's LDS array (gemm16_smem_floats
// floats): gemm16_kernel runs one GEMM, gemm16_pair_kernel two independent ones in one launch.
// (exactly the ring: 128 KB for 128x128 tiles -- one float more and the grid's start-up spread grew from
// ~1.1 to 2.9-3.9 us, in-kernel stamps; the PX bias slab sums reuse the ring after the main loop)
template <int BM, int BN, int BK, int S, int EPI_T, bool PX>
constexpr int gemm16_smem_floats() {
  return S * (BM + BN) * BK;
}
// SKM (EPI_T >= kEpiStreamK): a stream-K piece; bid_x is the tile's index in the grouped order itself
// (gemm16_sk_kernel gives each XCD a contiguous range of it)
template <int BM, int BN, int BK, int WM, int WN, int S, int SP, bool A_KC, bool B_KC, int EPI_T, bool PX>
__device__ __forceinline__ void gemm16_body(const GemmP& p_in, float* __restrict__ smem, const int bid_x) {
  constexpr bool SKM = EPI_T >= kEpiStreamK;
  constexpr int EPI = SKM ? EPI_T - kEpiStreamK : EPI_T;  // the tile epilogue
  GemmP p = p_in;
  if (!SKM && p.ksplit > 1) {
    const long z = blockIdx.y;
    p.A += z * p.kstepA;
    p.B += z * p.kstepB;
    p.C += z * p.slabC;
  }
  constexpr int NT = WM * WN * 64, NW = WM * WN;
  constexpr bool LDR = SP == 2;
  // SP >= 3: the direct form (no LDS ring; see the main loop), DD chunks of 16 k in flight per wave
  constexpr bool DIR = SP >= 3;
  constexpr int DD = (SP == 3 || SP == 5 || SP == 9) ? 4 : SP == 7 ? 2 : 8;
  static_assert(SP != 1 || S >= 3, "spread DMA needs a 3-slot ring");
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "16x16 tiles per wave");
  // an m/n-contiguous operand is read VM/VN consecutive floats per lane (ds_read_b128/b64/b32), which
  // feed VM/VN interleaved 16x16 tiles: tile V*q + e holds rows (cols) 16*V*q + V*i + e
  constexpr int VM = A_KC ? 1 : (TM % 4 == 0 ? 4 : TM % 2 == 0 ? 2 : 1);
  constexpr int VN = B_KC ? 1 : (TN % 4 == 0 ? 4 : TN % 2 == 0 ? 2 : 1);
  constexpr int NRA = A_KC ? TM : 4 * TM / VM, NRB = B_KC ? TN : 4 * TN / VN;  // fragment reads per chunk
  static_assert(BK == 32 || BK == 64, "BK");
  constexpr int CH = BK / 4, KCH = BK / 16;
  constexpr int A_SZ = BM * BK, B_SZ = BN * BK, ST_SZ = A_SZ + B_SZ;
  constexpr int GA = A_SZ / 4 / NT, GB = B_SZ / 4 / NT, G = GA + GB;
  static_assert(A_SZ % (4 * NT) == 0 && B_SZ % (4 * NT) == 0, "tile splits into 1-KiB wave pieces");
  static_assert(3 * G < 64, "vmcnt range");
  // smem: the ring (S slots of ST_SZ floats; after the main loop the PX bias slab sums, see PXB below)
  TNET_STAMP_RT(4);
  TNET_STAMP(0);

  const int M = p.M, N = p.N, K = p.K;
  const int nbn = (N + BN - 1) / BN, nbm = (M + BM - 1) / BM;
  const int nwg = nbm * nbn;
  const int bid = bid_x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int L = SKM ? bid : (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int grp = p.group, per_group = grp * nbn;
  const int first_m = (L / per_group) * grp;
  const int gsz = min(nbm - first_m, grp);
  const int bm = (first_m + (L % per_group) % gsz) * BM, bn = ((L % per_group) / gsz) * BN;

  // wave index in an SGPR: every LDS-DMA destination (M0) is then scalar arithmetic
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm0 = (wid / WN) * WTM, wn0 = (wid % WN) * WTN;
  const int lg = lane >> 4, li = lane & 15;

  if constexpr (LDR) {
    if (wid == NW) {  // ---- loader wave: all G_L pieces of every k-tile, nothing else
      constexpr int GAL = A_SZ / 256, GBL = B_SZ / 256, GL = GAL + GBL;
      static_assert((S - 2) * GL < 64, "loader vmcnt range");
      unsigned offA[GAL], offB[GBL];
#pragma unroll
      for (int g = 0; g < GAL; ++g) {
        const int u = g * 64 + lane;
        if (A_KC) {
          const int r = u / CH, j = u % CH;
          offA[g] = 4u * (unsigned)(min(bm + r, M - 1) * p.lda + 4 * (j ^ swz<BK>(r)));
        } else {
          const int k = u / (BM / 4), c = (u % (BM / 4)) * 4;
          offA[g] = 4u * (unsigned)(k * p.lda + (bm + c < M ? bm + c : 0));
        }
      }
#pragma unroll
      for (int g = 0; g < GBL; ++g) {
        const int u = g * 64 + lane;
        if (B_KC) {
          const int r = u / CH, j = u % CH;
          offB[g] = 4u * (unsigned)(min(bn + r, N - 1) * p.ldb + 4 * (j ^ swz<BK>(r)));
        } else {
          const int k = u / (BN / 4), c = (u % (BN / 4)) * 4;
          offB[g] = 4u * (unsigned)(k * p.ldb + (bn + c < N ? bn + c : 0));
        }
      }
      auto issue_l = [&](int t, int sl) {
        float* st = smem + sl * ST_SZ;
        const char* ab = (const char*)(p.A + (A_KC ? (long)t * BK : (long)t * BK * p.lda));
        const char* bb = (const char*)(p.B + (B_KC ? (long)t * BK : (long)t * BK * p.ldb));
#pragma unroll
        for (int g = 0; g < GAL; ++g) {
          unsigned o = offA[g];
          asm volatile("" : "+v"(o));
          __builtin_amdgcn_global_load_lds((const void*)(ab + o), (void*)(st + g * 256), 16, 0, 0);
        }
#pragma unroll
        for (int g = 0; g < GBL; ++g) {
          unsigned o = offB[g];
          asm volatile("" : "+v"(o));
          __builtin_amdgcn_global_load_lds((const void*)(bb + o), (void*)(st + A_SZ + g * 256), 16, 0, 0);
        }
      };
      const int nfull = K / BK, tlast = max(nfull - 1, 0);
      if (nfull > 0) {
#pragma unroll
        for (int t = 0; t < S - 1; ++t) issue_l(min(t, tlast), t);
        wait_vmcnt<(S - 2) * GL>();
        __builtin_amdgcn_s_barrier();  // tile 0 landed
        issue_l(min(S - 1, tlast), S - 1);
      }
      int sl = 0;
      for (int t = 0; t < nfull; ++t) {
        wait_vmcnt<(S - 2) * GL>();    // tile t+1 landed
        __builtin_amdgcn_s_barrier();  // seam t: every compute wave is done with tile t's slot
        issue_l(min(t + S, tlast), sl);
        sl = sl + 1 == S ? 0 : sl + 1;
      }
      wait_vmcnt<0>();  // no DMA may outlive the workgroup's LDS
      if (K % BK) {     // the masked tail's two barriers
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_barrier();
      }
      return;
    }
  }

  // per-lane BYTE offsets from the tile's base (32-bit: the launcher checks the operand extent), so
  // each DMA is global_load_lds with a scalar base (advanced per tile) + one VGPR offset
  unsigned srcA[GA], srcB[GB];
#pragma unroll
  for (int g = 0; g < GA; ++g) {
    const int u = (g * NW + wid) * 64 + lane;
    if (A_KC) {
      const int r = u / CH, j = u % CH;
      srcA[g] = 4u * (unsigned)(min(bm + r, M - 1) * p.lda + 4 * (j ^ swz<BK>(r)));
    } else {
      const int k = u / (BM / 4), c = (u % (BM / 4)) * 4;
      srcA[g] = 4u * (unsigned)(k * p.lda + (bm + c < M ? bm + c : 0));
    }
  }
#pragma unroll
  for (int g = 0; g < GB; ++g) {
    const int u = (g * NW + wid) * 64 + lane;
    if (B_KC) {
      const int r = u / CH, j = u % CH;
      srcB[g] = 4u * (unsigned)(min(bn + r, N - 1) * p.ldb + 4 * (j ^ swz<BK>(r)));
    } else {
      const int k = u / (BN / 4), c = (u % (BN / 4)) * 4;
      srcB[g] = 4u * (unsigned)(k * p.ldb + (bn + c < N ? bn + c : 0));
    }
  }
  // DMA of k-tile t into ring slot sl (t may be a clamped repeat of the last tile: see the loop)
  auto issue = [&](int t, int sl) {
    float* st = smem + sl * ST_SZ;
    const char* ab = (const char*)(p.A + (A_KC ? (long)t * BK : (long)t * BK * p.lda));
    const char* bb = (const char*)(p.B + (B_KC ? (long)t * BK : (long)t * BK * p.ldb));
#pragma unroll
    for (int g = 0; g < GA; ++g)
      __builtin_amdgcn_global_load_lds((const void*)(ab + srcA[g]), (void*)(st + (g * NW + wid) * 256), 16, 0, 0);
#pragma unroll
    for (int g = 0; g < GB; ++g)
      __builtin_amdgcn_global_load_lds((const void*)(bb + srcB[g]), (void*)(st + A_SZ + (g * NW + wid) * 256), 16, 0,
                                       0);
  };
  // pieces [g0, g1) of tile t (piece g < GA: A piece g, else B piece g - GA)
  constexpr int PPC = (G + KCH - 1) / KCH;
  auto issue_part = [&](int t, int sl, int c) {
    float* st = smem + sl * ST_SZ;
    const char* ab = (const char*)(p.A + (A_KC ? (long)t * BK : (long)t * BK * p.lda));
    const char* bb = (const char*)(p.B + (B_KC ? (long)t * BK : (long)t * BK * p.ldb));
#pragma unroll
    for (int g = c * PPC; g < (c + 1) * PPC && g < G; ++g) {
      if (g < GA)
        __builtin_amdgcn_global_load_lds((const void*)(ab + srcA[g]), (void*)(st + (g * NW + wid) * 256), 16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds((const void*)(bb + srcB[g - GA]),
                                         (void*)(st + A_SZ + ((g - GA) * NW + wid) * 256), 16, 0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  float av[2][TM][4], bv[2][TN][4];
  auto read_frags = [&](const float* st, int c, int buf) {  // chunk c (16 k) of the slot at st
    const float* As = st;
    const float* Bs = st + A_SZ;
    if (A_KC) {
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = wm0 + 16 * a + li;
        const f32x4 x = *reinterpret_cast<const f32x4*>(As + row * BK + 4 * ((4 * c + lg) ^ swz<BK>(row)));
#pragma unroll
        for (int s = 0; s < 4; ++s) av[buf][a][s] = x[s];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int q = 0; q < TM / VM; ++q) {
          float x[4];
          lds_vec<VM>(As + (16 * c + 4 * lg + s) * BM + wm0 + 16 * VM * q + VM * li, x);
#pragma unroll
          for (int e = 0; e < VM; ++e) av[buf][VM * q + e][s] = x[e];
        }
    }
    if (B_KC) {
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = wn0 + 16 * b + li;
        const f32x4 x = *reinterpret_cast<const f32x4*>(Bs + col * BK + 4 * ((4 * c + lg) ^ swz<BK>(col)));
#pragma unroll
        for (int s = 0; s < 4; ++s) bv[buf][b][s] = x[s];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int q = 0; q < TN / VN; ++q) {
          float x[4];
          lds_vec<VN>(Bs + (16 * c + 4 * lg + s) * BN + wn0 + 16 * VN * q + VN * li, x);
#pragma unroll
          for (int e = 0; e < VN; ++e) bv[buf][VN * q + e][s] = x[e];
        }
    }
  };
  auto mfmas = [&](int buf) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[buf][a][s], bv[buf][b][s], acc[a][b], 0, 0, 0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int NRD = NRA + NRB;    // fragment reads per chunk
  constexpr int NMF = 4 * TM * TN;  // MFMAs per chunk
  // fillers (fragment reads, DMA pieces) pinned after each MFMA: one, or more on small wave tiles
  constexpr int FPM = (NRD + (SP == 1 ? PPC : LDR ? 0 : G) + NMF - 1) / NMF;
  static_assert(PPC * KCH >= G, "pieces per chunk");
  // vmcnt at a seam: everything younger than tile t+1 may stay in flight -- tiles t+2..t+S-1 without
  // SP; with SP tiles t+2..t+S-2 plus the pieces of tile t+S-1 issued in the chunks before the seam
  // (the seam chunk issues its share after the wait)
  constexpr int SEAM_VM = SP == 1 ? (S - 3) * G + (G < (KCH - 1) * PPC ? G : (KCH - 1) * PPC) : (S - 2) * G;

  // Branch-free main loop: every tile ends with the seam (wait for tile t+1, barrier, first
  // fragments of t+1) and every tile issues exactly G pieces, so the counted vmcnt is the constant
  // (S-2)*G.  Tiles past the end are re-loads of the last tile into a slot no later tile reads
  // (harmless); the fragments read at the final seam are discarded.  Straight-line code lets the
  // compiler count lgkmcnt exactly instead of draining at every block join.
  const int nfull = K / BK;
  const int tlast = max(nfull - 1, 0);
  // Prologue.  early: every slot's tile is issued before the first wait (tile S-1 lands while tile 0
  // computes) -- else tile S-1 goes out only after tile 0 has landed (SP spreads it over tile 0)
  const bool early = !SP && !LDR && p.early_issue;
  if constexpr (!LDR && !DIR) {
    if (nfull > 0) {
#pragma unroll
      for (int t = 0; t < S - 1; ++t) issue(min(t, tlast), t);
      if (early) issue(min(S - 1, tlast), S - 1);
    }
  }
  if (!DIR && nfull > 0) {
    if constexpr (!LDR) {
      if (early) wait_vmcnt<(S - 1) * G>();
      else wait_vmcnt<(S - 2) * G>();
    }
    barrier();  // tile 0 landed in every wave's pieces
    if (!SP && !early) issue(min(S - 1, tlast), S - 1);
    read_frags(smem, 0, 0);
  }
  asm volatile("" ::: "memory");  // the prefetch loads below stay younger than every prologue DMA piece
  // Epilogue operands (bias / y of the layer below / W and the momentum buffer) are loaded into
  // registers HERE, right after the prologue (issued inside the main loop at tile 1 instead, they
  // shortened the prologue by 3-4k cycles but stretched the main loop by 4-7k): the main loop hides their latency (a seam's counted
  // vmcnt wait may also wait for them: they are older than every DMA piece still in flight -- safe)
  // and the epilogue is pure arithmetic + stores.  (Loaded at the end, each load waits behind the
  // stores issued before it -- vmcnt is in order -- one full round trip per row of the tile.)
  constexpr int EB = epi_base(EPI);
  constexpr bool EV = !B_KC;  // output columns in VN-vectors (n-contiguous B) or scalars (k-contiguous B)
  constexpr int NE = EV ? VN : 1;
  constexpr int NJ = TN / NE;
  // TRE: k-contiguous A and B (NT: the backward GEMM) leave each lane 4 ROWS of one column per tile;
  // the epilogue then goes through LDS (the ring is free after the main loop) so that every lane
  // holds 4 consecutive COLUMNS of a row: 16-B loads of the diff-sigmoid operand and 16-B stores
  // instead of one 4-B access per element
  constexpr bool TRE = A_KC && B_KC && !LDR && (epi_base(EPI) == EPI_DSIG || epi_base(EPI) == EPI_STORE);
  constexpr int LDT = WTN + 4, QPR = WTN / 4, RPP = 64 / QPR, TP = WTM / RPP;
  static_assert(!TRE || (QPR <= 64 && 64 % QPR == 0 && WTM % RPP == 0 && NW * WTM * LDT <= S * ST_SZ),
                "transposed epilogue");
  const int tcq = lane % QPR, tr0 = lane / QPR;
  constexpr bool PRE_BIAS = EB == EPI_BIAS || EB == EPI_BIAS_SIG || EB == EPI_BIAS_NSIG || EB == EPI_BIAS_NEG;
  constexpr bool PRE_C = EB == EPI_SGD || EB == EPI_RBM;
  constexpr bool PRE_AUX = EB == EPI_DSIG;
  constexpr bool PRE_Q = EB == EPI_SGD || EB == EPI_RBM;
  auto erow = [&](int a, int r) {
    return A_KC ? bm + wm0 + 16 * a + 4 * lg + r : bm + wm0 + 16 * VM * (a / VM) + VM * (4 * lg + r) + (a % VM);
  };
  auto ecol = [&](int j) { return bn + wn0 + 16 * NE * j + NE * li; };
  auto ld_tile = [&](const float* base, long ld, int row, int col) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < M) {
      const float* q = base + (long)row * ld + col;
      if (NE == 4 && col + 3 < N) {
        v = *reinterpret_cast<const f32x4*>(q);
      } else if (NE == 2 && col + 1 < N) {
        const float2 t = *reinterpret_cast<const float2*>(q);
        v[0] = t.x;
        v[1] = t.y;
      } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) v[e] = col + e < N ? q[e] : 0.f;
      }
    }
    return v;
  };
  f32x4 pre_bias[PRE_BIAS ? NJ : 1];
  f32x4 pre_a[PRE_C || PRE_AUX ? TM : 1][4][PRE_C || PRE_AUX ? NJ : 1];
  f32x4 pre_q[PRE_Q ? TM : 1][4][PRE_Q ? NJ : 1];
  f32x4 pre_t[TRE ? TP : 1];
  auto ld_row4 = [&](const float* base, long ld, int row, int col) {  // 4 columns of one row, masked
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < M) {
      const float* q = base + (long)row * ld + col;
      if (col + 3 < N) v = *reinterpret_cast<const f32x4*>(q);
      else
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = col + e < N ? q[e] : 0.f;
    }
    return v;
  };
  const bool has_q = PRE_Q && p.corr != nullptr;
  // exact prefetch (PX): every epilogue-operand load below is one unconditional
  // 16-B load (or one 4-B slab-sum load), npre counts this wave's, and the first seam lets them stay
  // in flight (vmcnt is in order: the npre youngest operations are exactly these loads)
  constexpr bool PEX = (!SP || DIR) && !LDR && (!PRE_BIAS || NE == 4) && (TRE || !(PRE_C || PRE_AUX || PRE_Q) || NE == 4);
  constexpr bool pex = PEX && PX;
  int npre = 0;
  if constexpr (PRE_BIAS) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = ecol(j);
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (pex) {
        v = *reinterpret_cast<const f32x4*>(p.bias + col);
      } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) v[e] = col + e < N ? p.bias[col + e] : 0.f;
      }
      pre_bias[j] = v;
    }
    npre += NJ;
  }
  // tiles of more than 128 prefetched floats per lane (128x256 tiles) are loaded at the epilogue
  // instead, all at once (one round trip): held across the main loop they would spill
  constexpr int PRE_TILE = TM * 4 * NJ * NE;
  constexpr bool EARLY = ((PRE_C || PRE_AUX) ? PRE_TILE : 0) + (PRE_Q ? PRE_TILE : 0) <= 128;
  auto prefetch_tiles = [&]() {
    auto ld16 = [&](const float* base, long ld, int row, int col) {
      return *reinterpret_cast<const f32x4*>(base + (long)row * ld + col);
    };
    // one branch on pex around each operand's whole tile (not one per load)
    if constexpr (TRE) {
      if constexpr (PRE_AUX) {
        if (pex) {
#pragma unroll
          for (int q = 0; q < TP; ++q) pre_t[q] = ld16(p.aux, p.ldaux, bm + wm0 + tr0 + RPP * q, bn + wn0 + 4 * tcq);
        } else {
#pragma unroll
          for (int q = 0; q < TP; ++q)
            pre_t[q] = ld_row4(p.aux, p.ldaux, bm + wm0 + tr0 + RPP * q, bn + wn0 + 4 * tcq);
        }
        npre += TP;
      }
    } else if constexpr (PRE_C || PRE_AUX) {
      const float* base = PRE_AUX ? p.aux : p.C;
      const long ld = PRE_AUX ? p.ldaux : p.ldc;
      if (pex) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < NJ; ++j) pre_a[a][r][j] = ld16(base, ld, erow(a, r), ecol(j));
      } else {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < NJ; ++j) pre_a[a][r][j] = ld_tile(base, ld, erow(a, r), ecol(j));
      }
      npre += TM * 4 * NJ;
    }
    if constexpr (PRE_Q) {
      if (has_q) {
        if (pex) {
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int j = 0; j < NJ; ++j) pre_q[a][r][j] = ld16(p.corr, p.ldcorr, erow(a, r), ecol(j));
        } else {
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int j = 0; j < NJ; ++j) pre_q[a][r][j] = ld_tile(p.corr, p.ldcorr, erow(a, r), ecol(j));
        }
        npre += TM * 4 * NJ;
      }
    }
  };
  if constexpr (EARLY) prefetch_tiles();

  static_assert(!epi_bias_slabs(EPI) || BN <= NT, "one thread per bias column");
  // The bias of the tile's BN columns (EPI_SGD_B / EPI_STORE_BG).  Without PX the first tile-row's
  // workgroups do it all (bias_pre_load / _finish).  With PX (PXB) it is spread over the tile-rows:
  // tile-row i owns columns [i*cpw, (i+1)*cpw) of the tile (cpw <= 8, launch_cfg checks), thread u loads
  // slab u/8 of column u%8 -- ONE straight-line load per lane (+ b, + corr) issued with the prefetch
  // above, so every workgroup carries the same small share and no seam waits for it; the slab sums
  // meet in LDS after the main loop and thread u < cpw adds its column's 32 slab sums in fp64 in slab
  // order (bias_pre_finish's arithmetic)
  constexpr bool PXB = pex && epi_bias_slabs(EPI);
  BiasPre bpre;
  if constexpr (epi_bias_slabs(EPI) && !pex)
    if (bm == 0) bias_pre_load<BN, EPI == EPI_STORE_BG>(p, bn, bpre);
  float pxb_v = 0.f, pxb_b = 0.f, pxb_q = 0.f;
  int pxb_col = 0, pxb_cpw = 0;
  if constexpr (PXB) {
    const int nbm_ = M / BM, tr = bm / BM;
    pxb_cpw = (BN + nbm_ - 1) / nbm_;
    const int u = threadIdx.x, slab = u >> 3, cl = u & 7;
    pxb_col = bn + min(tr * pxb_cpw + min(cl, pxb_cpw - 1), BN - 1);
    pxb_v = p.bpart[(long)min(slab, p.bslabs - 1) * p.ldbpart + pxb_col];
    npre += 1;
    if constexpr (EPI != EPI_STORE_BG) {
      pxb_b = p.bvec[pxb_col];
      npre += 1;
      if (p.bcorr) {
        pxb_q = p.bcorr[pxb_col];
        npre += 1;
      }
    }
  }

  TNET_STAMP(1);
  // one fragment read (r < TM: operand A, else B) of chunk c of the slot at st into buffer buf
  auto read_one = [&](const float* st, int c, int buf, int r) {
    const float* As = st;
    const float* Bs = st + A_SZ;
    if (r < NRA) {
      if (A_KC) {
        const int a = r, row = wm0 + 16 * a + li;
        const f32x4 x = *reinterpret_cast<const f32x4*>(As + row * BK + 4 * ((4 * c + lg) ^ swz<BK>(row)));
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) av[buf][a][s2] = x[s2];
      } else {
        const int s2 = r % 4, q = r / 4;
        float x[4];
        lds_vec<VM>(As + (16 * c + 4 * lg + s2) * BM + wm0 + 16 * VM * q + VM * li, x);
#pragma unroll
        for (int e = 0; e < VM; ++e) av[buf][VM * q + e][s2] = x[e];
      }
    } else {
      const int rb = r - NRA;
      if (B_KC) {
        const int b = rb, col = wn0 + 16 * b + li;
        const f32x4 x = *reinterpret_cast<const f32x4*>(Bs + col * BK + 4 * ((4 * c + lg) ^ swz<BK>(col)));
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) bv[buf][b][s2] = x[s2];
      } else {
        const int s2 = rb % 4, q = rb / 4;
        float x[4];
        lds_vec<VN>(Bs + (16 * c + 4 * lg + s2) * BN + wn0 + 16 * VN * q + VN * li, x);
#pragma unroll
        for (int e = 0; e < VN; ++e) bv[buf][VN * q + e][s2] = x[e];
      }
    }
  };
  // one DMA piece g of tile t into slot sl
  // (the 32-bit offset is made opaque per use so its zero-extension stays next to the load and the
  // instruction selects the SGPR-base + 32-bit VGPR-offset form: no 64-bit VALU add per piece)
  auto issue_one = [&](int t, int sl, int g) {
    float* st = smem + sl * ST_SZ;
    if (g < GA) {
      const char* ab = (const char*)(p.A + (A_KC ? (long)t * BK : (long)t * BK * p.lda));
      unsigned o = srcA[g];
      asm volatile("" : "+v"(o));
      __builtin_amdgcn_global_load_lds((const void*)(ab + o), (void*)(st + (g * NW + wid) * 256), 16, 0, 0);
    } else {
      const char* bb = (const char*)(p.B + (B_KC ? (long)t * BK : (long)t * BK * p.ldb));
      unsigned o = srcB[g - GA];
      asm volatile("" : "+v"(o));
      __builtin_amdgcn_global_load_lds((const void*)(bb + o), (void*)(st + A_SZ + ((g - GA) * NW + wid) * 256), 16,
                                       0, 0);
    }
  };

  // Each chunk is written out as its MFMA sequence with one filler instruction pinned after each
  // of the first MFMAs (sched_barrier fences): first the NRD fragment reads of the next chunk,
  // then the chunk's DMA pieces (SP: PPC of tile t+S-1; seam without SP: all G of tile t+S).
  // Left to itself the scheduler sinks every read to just before its first use and waits
  // lgkmcnt(0) there, and bunches the DMA pieces behind the barrier with the MFMA pipe idle.
  if constexpr (DIR) {
    // ---- the direct form: every wave loads its own fragments from global memory straight into registers
    // (16-B buffer loads in read_frags' lane map; the two waves that share an A row block or a B column
    // block read the same lines, L1 / L2-served), DD chunks of 16 k in a register ring: chunk c's MFMAs
    // run while chunks c+1..c+DD-2 are in flight and the loads of chunk c+DD-1 go out between them, into
    // the slot chunk c-1 used.  No LDS, no LDS-DMA issue cost on the MFMA waves, no seam barrier.
    constexpr int NR = NRA + NRB;
    // SP >= 5 (a<D> configurations): the ring's loads are inline-asm buffer loads the compiler does not
    // track, waited for by one counted vmcnt per chunk that also ties the chunk's registers (the compiler's
    // own waits drain the whole ring at every loop back edge); 16-B loads and 6, 8 or 12 per chunk only
    constexpr bool ASM = SP >= 5 && (A_KC || VM == 4) && (B_KC || VN == 4) && (NR == 6 || NR == 8 || NR == 12);
    // SP 8 / 9 (c<D> configurations) with a k-contiguous operand: in read_frags' lane map lane (li, lg) reads
    // 16 B of row li, so the four lanes of a quad hit four rows and every lane is a request of its own (the
    // backward's B: 101 vs 78 us direct vs ring).  Here the four lanes of a quad read one row's 64-B chunk
    // piece (lane 4a + b: row a, k 4b..4b+3) and each lane then takes its fragment from the lane that loaded
    // it (ds_bpermute, one per dword, issued a chunk ahead between the MFMAs): the same values in the same
    // registers, so bit-identical to the ring and to the a<D> forms
    constexpr bool CKC = ASM && (SP == 8 || SP == 9) && (A_KC || B_KC);
    constexpr int NKC = (A_KC ? NRA : 0) + (B_KC ? NRB : 0);  // k-contiguous fragment registers per chunk
    const int rq = CKC ? lane >> 2 : li, kq = CKC ? lane & 3 : lg;  // the row and 16-B piece a lane loads
    const __amdgpu_buffer_rsrc_t rA = tile_rsrc(p.A), rB = tile_rsrc(p.B);
    unsigned oA[NRA], oB[NRB];
#pragma unroll
    for (int r = 0; r < NRA; ++r) {
      // rows / columns past the matrix edge read the last valid ones (their outputs are never stored)
      if (A_KC) {
        oA[r] = 4u * (unsigned)(min(bm + wm0 + 16 * r + rq, M - 1) * p.lda + 4 * kq);
      } else {
        const int s2 = r % 4, q = r / 4;
        oA[r] = 4u * (unsigned)((4 * lg + s2) * p.lda + max(min(bm + wm0 + 16 * VM * q + VM * li, M - VM), 0));
      }
    }
#pragma unroll
    for (int r = 0; r < NRB; ++r) {
      if (B_KC) {
        oB[r] = 4u * (unsigned)(min(bn + wn0 + 16 * r + rq, N - 1) * p.ldb + 4 * kq);
      } else {
        const int s2 = r % 4, q = r / 4;
        oB[r] = 4u * (unsigned)((4 * lg + s2) * p.ldb + max(min(bn + wn0 + 16 * VN * q + VN * li, N - VN), 0));
      }
    }
    const int cA = A_KC ? 64 : 64 * p.lda, cB = B_KC ? 64 : 64 * p.ldb;  // bytes per chunk
    const int nch = nfull * KCH;
    if constexpr (ASM) {
      const unsigned long long ba = (unsigned long long)(uintptr_t)p.A, bb = (unsigned long long)(uintptr_t)p.B;
      const u32x4 dA = {(unsigned)ba, (unsigned)(ba >> 32), 0x7FFFFFF0u, 0x00020000u};
      const u32x4 dB = {(unsigned)bb, (unsigned)(bb >> 32), 0x7FFFFFF0u, 0x00020000u};
      f32x4 ring[DD][NR];
      auto ld = [&](int c, int r) {
        f32x4 v;
        if (r < NRA)
          asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(v) : "v"(oA[r]), "s"(dA), "s"(c * cA));
        else
          asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(v) : "v"(oB[r - NRA]), "s"(dB), "s"(c * cB));
        return v;
      };
      constexpr int WV = (DD - 2) * NR;  // loads younger than a chunk's when it is consumed
      auto wait_slot = [&](f32x4 (&q)[NR]) {
        if constexpr (NR == 6)
          asm volatile("s_waitcnt vmcnt(%6)" : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]), "+v"(q[4]), "+v"(q[5])
                       : "n"(WV));
        else if constexpr (NR == 8)
          asm volatile("s_waitcnt vmcnt(%8)"
                       : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]), "+v"(q[4]), "+v"(q[5]), "+v"(q[6]), "+v"(q[7])
                       : "n"(WV));
        else
          asm volatile("s_waitcnt vmcnt(%12)"
                       : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]), "+v"(q[4]), "+v"(q[5]), "+v"(q[6]), "+v"(q[7]),
                         "+v"(q[8]), "+v"(q[9]), "+v"(q[10]), "+v"(q[11])
                       : "n"(WV));
      };
      // CKC: lane (li, lg) takes its fragment from lane 4 li + lg; the t-th k-contiguous register of a slot
      const int pperm = 4 * (4 * li + lg);
      auto perm = [&](f32x4& v) {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[e] = __int_as_float(__builtin_amdgcn_ds_bpermute(pperm, __float_as_int(v[e])));
        v = o;
      };
      auto kc_reg = [](int t) { return A_KC ? t : NRA + t; };
      static_assert(!CKC || 4 * TM * TN >= NR + NKC, "a chunk's MFMAs cover its loads and the next one's permutes");
#pragma unroll
      for (int j = 0; j < DD - 1; ++j)
#pragma unroll
        for (int r = 0; r < NR; ++r) ring[j][r] = ld(min(j, nch - 1), r);
      if constexpr (CKC) {
        wait_slot(ring[0]);
#pragma unroll
        for (int t = 0; t < NKC; ++t) perm(ring[0][kc_reg(t)]);
      }
      for (int c0 = 0; c0 < nch; c0 += DD) {
#pragma unroll
        for (int j = 0; j < DD; ++j) {
          const int cn = min(c0 + j + DD - 1, nch - 1);  // past the end: a repeat of the last chunk, never used
          if constexpr (!CKC) {
            __builtin_amdgcn_sched_barrier(0);  // the wait stays after the previous chunk's MFMAs
            wait_slot(ring[j]);
            __builtin_amdgcn_sched_barrier(0);
          }
          int mi = 0;
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
              for (int b = 0; b < TN; ++b) {
                const float av_ = A_KC ? ring[j][a][s2] : ring[j][(a / 4) * 4 + s2][a % 4];
                const float bv_ = B_KC ? ring[j][NRA + b][s2] : ring[j][NRA + (b / 4) * 4 + s2][b % 4];
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av_, bv_, acc[a][b], 0, 0, 0);
                if (mi < NR) {
                  __builtin_amdgcn_sched_barrier(0);
                  ring[(j + DD - 1) % DD][mi] = ld(cn, mi);
                  __builtin_amdgcn_sched_barrier(0);
                }
                if constexpr (CKC) {
                  // the next chunk: its loads are DD - 2 chunks old once this chunk's are out (the same
                  // count the a<D> forms wait for at the chunk's head); then its permutes between the MFMAs
                  if (mi == NR - 1) {
                    __builtin_amdgcn_sched_barrier(0);
                    wait_slot(ring[(j + 1) % DD]);
                    __builtin_amdgcn_sched_barrier(0);
                  } else if (mi >= NR && mi < NR + NKC) {
                    __builtin_amdgcn_sched_barrier(0);
                    perm(ring[(j + 1) % DD][kc_reg(mi - NR)]);
                    __builtin_amdgcn_sched_barrier(0);
                  }
                }
                ++mi;
              }
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the repeat loads of the last chunk
    } else {
    float fa[DD][TM][4], fb[DD][TN][4];
    auto gld = [&](__amdgpu_buffer_rsrc_t rs, unsigned off, int soff, float (&x)[4], auto vtag) {
      constexpr int V = decltype(vtag)::value;
      if constexpr (V == 4) {
        const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, soff, 0));
        x[0] = v[0]; x[1] = v[1]; x[2] = v[2]; x[3] = v[3];
      } else if constexpr (V == 2) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)off, soff, 0);
        x[0] = __uint_as_float(v[0]); x[1] = __uint_as_float(v[1]);
      } else {
        x[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, soff, 0));
      }
    };
    auto load_one = [&](int c, float (&ra)[TM][4], float (&rb)[TN][4], int r) {
      if (r < NRA) {
        if (A_KC) {
          gld(rA, oA[r], c * cA, ra[r], std::integral_constant<int, 4>{});
        } else {
          const int s2 = r % 4, q = r / 4;
          float x[4];
          gld(rA, oA[r], c * cA, x, std::integral_constant<int, VM>{});
#pragma unroll
          for (int e = 0; e < VM; ++e) ra[VM * q + e][s2] = x[e];
        }
      } else {
        const int rb_ = r - NRA;
        if (B_KC) {
          gld(rB, oB[rb_], c * cB, rb[rb_], std::integral_constant<int, 4>{});
        } else {
          const int s2 = rb_ % 4, q = rb_ / 4;
          float x[4];
          gld(rB, oB[rb_], c * cB, x, std::integral_constant<int, VN>{});
#pragma unroll
          for (int e = 0; e < VN; ++e) rb[VN * q + e][s2] = x[e];
        }
      }
    };
#pragma unroll
    for (int j = 0; j < DD - 1; ++j)
#pragma unroll
      for (int r = 0; r < NR; ++r) load_one(min(j, nch - 1), fa[j], fb[j], r);
    for (int c0 = 0; c0 < nch; c0 += DD) {
#pragma unroll
      for (int j = 0; j < DD; ++j) {
        const int cn = min(c0 + j + DD - 1, nch - 1);  // past the end: a repeat of the last chunk, never used
        int mi = 0;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) {
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[j][a][s2], fb[j][b][s2], acc[a][b], 0, 0, 0);
              if (mi < NR) {
                __builtin_amdgcn_sched_barrier(0);
                load_one(cn, fa[(j + DD - 1) % DD], fb[(j + DD - 1) % DD], mi);
                __builtin_amdgcn_sched_barrier(0);
              }
              ++mi;
            }
      }
    }
    }
  } else {
  int sl = 0;  // slot of tile t
  for (int t = 0; t < nfull; ++t) {
    const float* st = smem + sl * ST_SZ;
    const int sl1 = sl + 1 == S ? 0 : sl + 1;          // slot of tile t+1
    const int slp = sl == 0 ? S - 1 : sl - 1;          // slot of tile t+S-1 (= t-1, released at the last seam)
    const int tsp = min(t + S - 1, tlast), tns = min(t + S, tlast);
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      const int buf = c & 1;  // KCH is even: chunk 0 of every tile uses buffer 0
      const bool seam = c + 1 == KCH;
      const float* rst = seam ? smem + sl1 * ST_SZ : st;
      const int rc = seam ? 0 : c + 1;
      if (seam) {
        // hand over to tile t+1: own reads of tile t retired, tile t+1 landed, everyone past
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        if constexpr (!LDR) {
          // seam 0 under PX: tile 1 only, the prefetch loads behind it may still be in flight
          // (more than 63 - SEAM_VM of them: vmcnt saturates, the wait for 63 is still exact)
          if (pex && t == 0) wait_vmcnt_bin<SEAM_VM, 63>(min(SEAM_VM + npre, 63));
          else wait_vmcnt<SEAM_VM>();
        }
#ifdef TNET_GEMM_DIAG_NOBAR
        if constexpr (LDR) barrier();  // the loader wave meets the compute waves at every seam barrier
#else
        barrier();
#endif
      }
      if (SP == 1) __builtin_amdgcn_s_setprio(1);
      constexpr int NP = SP == 1 ? PPC : LDR ? 0 : G;
      int mi = 0;
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[buf][a][s], bv[buf][b][s], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < FPM; ++f) {
            const int idx = mi * FPM + f;
            if (idx < NRD) {
              __builtin_amdgcn_sched_barrier(0);
#ifndef TNET_GEMM_DIAG_NOREAD
              read_one(rst, rc, buf ^ 1, idx);
#endif
              __builtin_amdgcn_sched_barrier(0);
            } else if (idx < NRD + NP) {
              const int g = SP == 1 ? c * PPC + (idx - NRD) : idx - NRD;
              if (SP == 1 && g < G) {
                __builtin_amdgcn_sched_barrier(0);
#ifndef TNET_GEMM_DIAG_NODMA
                issue_one(tsp, slp, g);
#endif
                __builtin_amdgcn_sched_barrier(0);
              } else if (SP == 0 && seam) {
                __builtin_amdgcn_sched_barrier(0);
#ifndef TNET_GEMM_DIAG_NODMA
                issue_one(tns, sl, g);
#endif
                __builtin_amdgcn_sched_barrier(0);
              }
            }
            }
            ++mi;
          }
      if (SP == 1) __builtin_amdgcn_s_setprio(0);
    }
    sl = sl1;
  }
  }
  wait_vmcnt<0>();  // repeat loads of the last tile still land in LDS
  TNET_STAMP(2);

  if (!LDR && K % BK && K % 4 == 0) {
    // partial last k-tile (Kt = K % BK deep) through the same LDS-DMA images, in slot nfull % S (the
    // final seam read it: every wave's reads retire before the barrier).  Sources past K are clamped
    // to valid memory (last k column / row) and the fragments with k >= Kt are zeroed in registers.
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    float* st = smem + (nfull % S) * ST_SZ;
    const int k0 = nfull * BK, Kt = K - k0;
#pragma unroll
    for (int g = 0; g < GA; ++g) {
      const int u = (g * NW + wid) * 64 + lane;
      long off;
      if (A_KC) {
        const int r = u / CH, j = u % CH, kc = k0 + 4 * (j ^ swz<BK>(r));
        off = (long)min(bm + r, M - 1) * p.lda + (kc < K ? kc : K - 4);
      } else {
        const int k = u / (BM / 4), c = (u % (BM / 4)) * 4;
        off = (long)min(k0 + k, K - 1) * p.lda + (bm + c < M ? bm + c : 0);
      }
      __builtin_amdgcn_global_load_lds((const void*)(p.A + off), (void*)(st + (g * NW + wid) * 256), 16, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < GB; ++g) {
      const int u = (g * NW + wid) * 64 + lane;
      long off;
      if (B_KC) {
        const int r = u / CH, j = u % CH, kc = k0 + 4 * (j ^ swz<BK>(r));
        off = (long)min(bn + r, N - 1) * p.ldb + (kc < K ? kc : K - 4);
      } else {
        const int k = u / (BN / 4), c = (u % (BN / 4)) * 4;
        off = (long)min(k0 + k, K - 1) * p.ldb + (bn + c < N ? bn + c : 0);
      }
      __builtin_amdgcn_global_load_lds((const void*)(p.B + off), (void*)(st + A_SZ + (g * NW + wid) * 256), 16, 0,
                                       0);
    }
    wait_vmcnt<0>();
    barrier();
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      if (16 * c >= Kt) break;
      read_frags(st, c, 0);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const bool ok = 16 * c + 4 * lg + s2 < Kt;  // k of this lane's operand elements in MFMA step s2
#pragma unroll
        for (int a = 0; a < TM; ++a) av[0][a][s2] = ok ? av[0][a][s2] : 0.f;
#pragma unroll
        for (int b = 0; b < TN; ++b) bv[0][b][s2] = ok ? bv[0][b][s2] : 0.f;
      }
      mfmas(0);
    }
  } else if (K % BK) {
    // K not a multiple of 4 (or the loader-wave variant): masked tail k-tile through registers,
    // same images, in slot nfull % S
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    float* st = smem + (nfull % S) * ST_SZ;
    const int k0 = nfull * BK;
    for (int u = threadIdx.x; u < A_SZ / 4; u += NT) {
      int gr, gc;
      if (A_KC) { const int r = u / CH, j = u % CH; gr = bm + r; gc = k0 + 4 * (j ^ swz<BK>(r)); }
      else { const int k = u / (BM / 4); gr = k0 + k; gc = bm + (u % (BM / 4)) * 4; }
      const int rmax = A_KC ? M : K, cmax = A_KC ? K : M;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (gr < rmax) {
        const float* q = p.A + (long)gr * p.lda + gc;
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = (gc + e < cmax) ? q[e] : 0.f;
      }
      *reinterpret_cast<f32x4*>(st + u * 4) = x;
    }
    for (int u = threadIdx.x; u < B_SZ / 4; u += NT) {
      int gr, gc;
      if (B_KC) { const int r = u / CH, j = u % CH; gr = bn + r; gc = k0 + 4 * (j ^ swz<BK>(r)); }
      else { const int k = u / (BN / 4); gr = k0 + k; gc = bn + (u % (BN / 4)) * 4; }
      const int rmax = B_KC ? N : K, cmax = B_KC ? K : N;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (gr < rmax) {
        const float* q = p.B + (long)gr * p.ldb + gc;
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = (gc + e < cmax) ? q[e] : 0.f;
      }
      *reinterpret_cast<f32x4*>(st + A_SZ + u * 4) = x;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      read_frags(st, c, 0);
      mfmas(0);
    }
  }

  if constexpr (SKM) {
    // ---- stream-K fixup: a split tile has exactly two pieces (gemm16_sk_kernel's ranges are at least
    // a tile long).  Each draws a ticket as it finishes its k-range; the first stores its accumulators
    // and flags them stored, the second waits for that flag -- the first piece is running by then (it
    // drew its ticket), so the wait is bounded by one tile store whatever else holds the CUs -- and adds
    // the stored partial to its own accumulators, then runs the tile's epilogue.  Two-term fp32 sums
    // commute exactly: the result is the same whichever piece finishes last.  The hand-off is the sc1
    // form of cdna_hip_programming.md's in-launch reduction (placement-independent, no L2 writeback or
    // invalidate): sc1 (write-through) stores in fragment order (lane-contiguous 16 B), drained before
    // the relaxed agent-scope flag; sc1 loads of every stored word.  tile_cnt[tile]: tickets in the low
    // half, the stored flag in the high half; the second piece resets it for the next launch.
    if (p.ksplit > 1) {
      constexpr int SLICE = BM * BN;
      const __amdgpu_buffer_rsrc_t rw = tile_rsrc(p.skws + (long)bid_x * SLICE);
      __attribute__((address_space(1))) unsigned* cnt =
          (__attribute__((address_space(1))) unsigned*)(p.tile_cnt + bid_x);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // every wave's ring reads retired (smem[0] below is in slot 0)
      if (threadIdx.x == 0) {
        const unsigned ticket = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        smem[0] = (ticket & 0xFFFFu) == 0 ? 0.f : 1.f;
      }
      __syncthreads();
      if (smem[0] == 0.f) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) st_wt(rw, ((long)(a * TN + b) * NT + threadIdx.x) * 4, acc[a][b]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 0x10000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;  // uniform: the workgroup's next piece (after the caller's barrier)
      }
      if (threadIdx.x == 0) {
        while ((__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 16) == 0u)
          __builtin_amdgcn_s_sleep(2);
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
      }
      __syncthreads();
      f32x4 t[TM][TN];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) t[a][b] = ld_sc1(rw, ((long)(a * TN + b) * NT + threadIdx.x) * 4);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = acc[a][b] + t[a][b];
    }
  }
  if constexpr (epi_bias_slabs(EPI) && !PXB)
    if (bm == 0) bias_pre_finish<BN, EPI == EPI_STORE_BG>(p, bn, bpre);
  if constexpr (PXB) {
    static_assert(S * ST_SZ >= kBiasPreSlabs * 8 && WM * WN * 64 == kBiasPreSlabs * 8, "PX bias layout");
    float* bsm = smem;  // the ring's first 1 KB, once every wave's last fragment reads have retired
    const int u = threadIdx.x;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __syncthreads();
    bsm[u] = (u >> 3) < p.bslabs ? pxb_v : 0.f;
    __syncthreads();
    if (u < pxb_cpw && (bm / BM) * pxb_cpw + u < BN) {
      double sum = 0.0;
#pragma unroll
      for (int k = 0; k < kBiasPreSlabs; ++k) sum += (double)bsm[k * 8 + u];
      float g = (float)sum;
      if constexpr (EPI == EPI_STORE_BG) {
        p.bvec[pxb_col] = g;
      } else {
        if (p.bcorr) {
          g = g + p.bmmt * pxb_q;
          p.bcorr[pxb_col] = g;
        }
        p.bvec[pxb_col] = pxb_b + p.bscale * g;
      }
    }
  }

  if constexpr (!EARLY) prefetch_tiles();
  const __amdgpu_buffer_rsrc_t rs_c = tile_rsrc(p.C + (long)bm * p.ldc + bn);
  const __amdgpu_buffer_rsrc_t rs_q = tile_rsrc(p.corr ? p.corr + (long)bm * p.ldcorr + bn : p.C);
  constexpr bool CS = EPI == EPI_DSIG_CS;
  static_assert(!CS || (A_KC && WTM == kColsumSlabRows), "column sums: k-contiguous A, 32-row wave tiles");
  if constexpr (TRE) {
    // ---- transposed epilogue (see TRE)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's last fragment reads retired
    __builtin_amdgcn_s_barrier();         // every wave is done with the ring
    float* wl = smem + wid * WTM * LDT;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) wl[(16 * a + 4 * lg + r) * LDT + 16 * b + li] = acc[a][b][r];
    // EPI_DSIG_CS: the wave's 32 rows are one slab; a lane sums its rows of 4 columns in order, the
    // lanes of a column quad meet by xor-shuffles
    float cs4[4] = {0.f, 0.f, 0.f, 0.f};
    const int col = bn + wn0 + 4 * tcq;
#pragma unroll
    for (int q = 0; q < TP; ++q) {
      const int rl = tr0 + RPP * q, row = bm + wm0 + rl;
      const f32x4 v = *reinterpret_cast<const f32x4*>(wl + rl * LDT + 4 * tcq);
      if (row >= M) continue;
      f32x4 o;
      if constexpr (EB == EPI_STORE) {
        if (p.beta == 0.f) {
          o = p.alpha * v;
        } else {
          o = p.alpha * v + p.beta * ld_row4(p.C, p.ldc, row, col);
        }
      } else {  // EPI_DSIG
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = pre_t[q][e] * (1.f - pre_t[q][e]) * v[e];
      }
      float* cp = p.C + (long)row * p.ldc + col;
      if (col + 3 < N) {
        if (p.wt) st_wt(rs_c, (long)(row - bm) * p.ldc + (col - bn), o);
        else *reinterpret_cast<f32x4*>(cp) = o;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (col + e < N) cp[e] = o[e];
      }
      if constexpr (CS)
#pragma unroll
        for (int e = 0; e < 4; ++e) cs4[e] += o[e];
    }
    if constexpr (CS) {
#pragma unroll
      for (int k = QPR; k < 64; k <<= 1)
#pragma unroll
        for (int e = 0; e < 4; ++e) cs4[e] += __shfl_xor(cs4[e], k, 64);
      const int slab_row = bm + wm0;
      if (tr0 == 0 && slab_row < M) {
        float* cp = p.cpart + (long)(slab_row / kColsumSlabRows) * p.ldcpart + col;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (col + e < N) cp[e] = cs4[e];
      }
    }
  } else {
  // ---- epilogue: arithmetic on the prefetched operands, then 16-B (n-contiguous) or 4-B stores
  // EPI_DSIG_CS: each wave owns 32 output rows (one slab) x its columns; a lane sums its 8 rows of
  // a column in order, the 4 lane groups of a column meet by two xor-shuffles
  float csum[CS ? TN : 1];
#pragma unroll
  for (int j = 0; j < (CS ? TN : 1); ++j) csum[j] = 0.f;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = erow(a, r);
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = ecol(j);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < NE; ++e) v[e] = acc[a][NE * j + e][r];
        f32x4 o = v, qn = v;
        if constexpr (EB == EPI_STORE) {
          if (p.beta == 0.f) {
#pragma unroll
            for (int e = 0; e < NE; ++e) o[e] = p.alpha * v[e];
          } else {
            const f32x4 c0 = ld_tile(p.C, p.ldc, row, col);
#pragma unroll
            for (int e = 0; e < NE; ++e) o[e] = p.alpha * v[e] + p.beta * c0[e];
          }
        } else if constexpr (PRE_BIAS) {
#pragma unroll
          for (int e = 0; e < NE; ++e) {
            const float x = v[e] + pre_bias[j][e];
            o[e] = EB == EPI_BIAS ? x : EB == EPI_BIAS_SIG ? sigmoidf_ref(x)
                 : EB == EPI_BIAS_NSIG ? -sigmoidf_ref(x) : -x;
          }
        } else if constexpr (EB == EPI_DSIG) {
#pragma unroll
          for (int e = 0; e < NE; ++e) {
            const float y = pre_a[a][r][j][e];
            o[e] = y * (1.f - y) * v[e];
          }
          if constexpr (CS)
#pragma unroll
            for (int e = 0; e < NE; ++e) csum[NE * j + e] += o[e];
        } else if constexpr (EB == EPI_RBM) {
          // c = mmt*corr + scale*acc + l2*W ; corr = c ; W += c   (cuRbm.cc:133-174)
#pragma unroll
          for (int e = 0; e < NE; ++e) {
            const float w = pre_a[a][r][j][e];
            const float c = p.mmt * pre_q[a][r][j][e] + p.scale * v[e] + p.l2 * w;
            qn[e] = c;
            o[e] = w + c;
          }
        } else {  // EPI_SGD: corr = acc + mmt*corr ; W += scale*corr ; W += l2*W   (cuBiasedLinearity.cc:46-64)
#pragma unroll
          for (int e = 0; e < NE; ++e) {
            const float c = has_q ? v[e] + p.mmt * pre_q[a][r][j][e] : v[e];
            qn[e] = c;
            float w = pre_a[a][r][j][e];
            w = w + p.scale * c;
            w = w + p.l2 * w;
            o[e] = w;
          }
          if (p.Ct)  // the updated values stay in the accumulators for the transposed stores below
#pragma unroll
            for (int e = 0; e < NE; ++e) acc[a][NE * j + e][r] = o[e];
        }
        float* cp = p.C + (long)row * p.ldc + col;
        float* qp = has_q ? p.corr + (long)row * p.ldcorr + col : nullptr;
        if (NE == 4 && col + 3 < N) {
          if (p.wt) {
            const long eo = (long)(row - bm) * p.ldc + (col - bn);
            st_wt(rs_c, eo, o);
            if (has_q) st_wt(rs_q, (long)(row - bm) * p.ldcorr + (col - bn), qn);
          } else {
            *reinterpret_cast<f32x4*>(cp) = o;
            if (has_q) *reinterpret_cast<f32x4*>(qp) = qn;
          }
        } else if (NE == 2 && col + 1 < N) {
          *reinterpret_cast<float2*>(cp) = float2{o[0], o[1]};
          if (has_q) *reinterpret_cast<float2*>(qp) = float2{qn[0], qn[1]};
        } else {
#pragma unroll
          for (int e = 0; e < NE; ++e)
            if (col + e < N) {
              cp[e] = o[e];
              if (has_q) qp[e] = qn[e];
            }
        }
      }
    }
  }
  if constexpr (CS) {
    // lane (lg, li) summed its rows of each column it holds; the four lane groups of a column meet by two xor
    // shuffles (NE consecutive columns per lane where B is n-contiguous: the backward from the transposed weight)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      csum[j] += __shfl_xor(csum[j], 16, 64);
      csum[j] += __shfl_xor(csum[j], 32, 64);
    }
    const int slab_row = bm + wm0;
    if (lg == 0 && slab_row < M) {
      float* cp = p.cpart + (long)(slab_row / kColsumSlabRows) * p.ldcpart;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = ecol(j);
        if (NE == 4 && col + 3 < N) {
          *reinterpret_cast<f32x4*>(cp + col) = f32x4{csum[4 * j], csum[4 * j + 1], csum[4 * j + 2], csum[4 * j + 3]};
        } else {
#pragma unroll
          for (int e = 0; e < NE; ++e)
            if (col + e < N) cp[col + e] = csum[NE * j + e];
        }
      }
    }
  }
  if constexpr (EB == EPI_SGD) {
    // the transposed shadow Ct[col][row] of the updated W (tnet_weight_shadow), staged through LDS so that the
    // global stores are whole lines: each lane holds its rows of a column as VM-row vectors (erow), which go into
    // an LDS image of the tile's columns [BN][BM + 4]; then every thread writes 16-B pieces of the image's rows,
    // consecutive threads consecutive pieces of one Ct row (BM floats), written through (sc1) like W
    if (p.Ct) {
      constexpr int LDP = BM + 4, Q = BM / 4;
      static_assert(BN * LDP <= S * ST_SZ, "shadow image fits the ring");
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS reads retired
      __syncthreads();
      float* ts = smem;
#pragma unroll
      for (int aq = 0; aq < TM / VM; ++aq)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl0 = erow(VM * aq, r) - bm;
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int e = 0; e < NE; ++e) {
              const int cl = ecol(j) + e - bn;
              if constexpr (VM == 4) {
                *reinterpret_cast<f32x4*>(ts + cl * LDP + rl0) =
                    f32x4{acc[4 * aq][NE * j + e][r], acc[4 * aq + 1][NE * j + e][r], acc[4 * aq + 2][NE * j + e][r],
                          acc[4 * aq + 3][NE * j + e][r]};
              } else {
#pragma unroll
                for (int m = 0; m < VM; ++m) ts[cl * LDP + rl0 + m] = acc[VM * aq + m][NE * j + e][r];
              }
            }
        }
      __syncthreads();
      const __amdgpu_buffer_rsrc_t rs_t = tile_rsrc(p.Ct + (long)bn * p.ldct + bm);
      for (int u = threadIdx.x; u < BN * Q; u += NT) {
        const int cl = u / Q, q4 = u % Q, col = bn + cl, row0 = bm + 4 * q4;
        if (col >= N || row0 >= M) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(ts + cl * LDP + 4 * q4);
        if (row0 + 3 < M) {
          st_wt(rs_t, (long)cl * p.ldct + 4 * q4, v);
        } else {
#pragma unroll
          for (int m = 0; m < 4; ++m)
            if (row0 + m < M) p.Ct[(long)col * p.ldct + row0 + m] = v[m];
        }
      }
    }
  }
  }
  if constexpr (EPI == EPI_BIAS_SIG_BIN) binarize_tile<BM, BN, NT>(p, bm, bn);
  TNET_STAMP(3);
  TNET_STAMP_RT(5);
}

// Stream-K over G workgroups (the GEMMs beside RCCL).  A tile grid of one
// workgroup per CU loses a whole second round when R CUs are held by another kernel (RCCL's channel
// workgroups keep 37.6 KB LDS and 248-256 VGPRs per lane for the whole collective:
// tools/cohab_probe.hip), so while collectives are in flight the data-parallel step's GEMMs run on
// G = CUs - R workgroups: the T tiles' T * KT k-tiles (tiles in the grouped order) are cut into G equal
// contiguous ranges, and the ranges go to the workgroups XCD by XCD (workgroup b runs on XCD b % 8: each
// XCD gets a contiguous run of ranges, so a tile's pieces meet in one L2 and its neighbours share
// operands there, as in the plain grid).  T >= G: a range is at least a tile long, so it covers whole
// tiles and at most a piece at either end, and a split tile has exactly two pieces; they combine through
// gemm16_body's stream-K fixup and the second to finish runs the tile's own epilogue.  Static and
// deterministic: no claims, no queues.
// SPK: the pieces' form (0: the LDS ring, 5: the direct form -- TNET_GEMM_DIRECT, n-contiguous B only)
template <int BM, int BN, int BK, int WM, int WN, int S, bool A_KC, bool B_KC, int EPI, int SPK = 0>
__global__ __launch_bounds__(WM * WN * 64)
__attribute__((amdgpu_waves_per_eu((WM * WN + 3) / 4, (WM * WN + 3) / 4)))
void gemm16_sk_kernel(const GemmP p, const int G) {
  __shared__ __attribute__((aligned(16))) float smem[gemm16_smem_floats<BM, BN, BK, S, EPI, true>()];
  const int T = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN), KT = p.K / BK;
  const long I = (long)T * KT;
  const int b = blockIdx.x, xcd = b & 7, q8 = G >> 3, r8 = G & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const long s = (long)v * I / G, e = (long)(v + 1) * I / G;
  for (long k0 = s; k0 < e;) {
    const int t = (int)(k0 / KT);
    const long tb = (long)t * KT, te = tb + KT, k1 = e < te ? e : te;
    if (k0 != s) __syncthreads();  // the previous piece is done with the ring
    // the ranges holding the tile's first and last k-tile: w(k) = ((k + 1) G - 1) / I
    const int w0 = (int)(((tb + 1) * G - 1) / I), w1 = (int)((te * G - 1) / I);
    GemmP q = p;
    q.ksplit = w1 - w0 + 1;
    const long kk = (k0 - tb) * BK;
    q.A = p.A + (A_KC ? kk : kk * p.lda);
    q.B = p.B + (B_KC ? kk : kk * p.ldb);
    q.K = (int)((k1 - k0) * BK);
    gemm16_body<BM, BN, BK, WM, WN, S, SPK, A_KC, B_KC, kEpiStreamK + EPI, true>(q, smem, t);
    k0 = k1;
  }
}

// Split-K in two over 2T workgroups (tiles too few for the CUs, K long): the two k-halves of a tile are
// two pieces of gemm16_body's stream-K fixup -- the first to finish stores its accumulators, the second
// adds them and runs the tile's own fused epilogue (no second launch, no slice workspace pass over the
// whole output).  Workgroups b are mapped XCD by XCD (the body's bijective remap over 2T), so a tile's
// two pieces are neighbours on one XCD and start together.
template <int BM, int BN, bool A_KC, bool B_KC, int EPI, bool PX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm16_split2_kernel(const GemmP p) {
  __shared__ __attribute__((aligned(16))) float smem[gemm16_smem_floats<BM, BN, 64, 2, EPI, PX>()];
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  GemmP q = p;
  const long kk = (long)(v & 1) * (p.K / 2);
  q.A = p.A + (A_KC ? kk : kk * p.lda);
  q.B = p.B + (B_KC ? kk : kk * p.ldb);
  q.K = p.K / 2;
  q.ksplit = 2;
  gemm16_body<BM, BN, 64, 2, 2, 2, 0, A_KC, B_KC, kEpiStreamK + EPI, PX>(q, smem, v >> 1);
}

template <int BM, int BN, int BK, int WM, int WN, int S, int SP, bool A_KC, bool B_KC, int EPI_T, bool PX = false>
__global__ __launch_bounds__((WM * WN + (SP == 2)) * 64)
__attribute__((amdgpu_waves_per_eu((WM * WN + (SP == 2) + 3) / 4, (WM * WN + (SP == 2) + 3) / 4)))
void gemm16_kernel(const GemmP p_in) {
  __shared__ __attribute__((aligned(16))) float smem[gemm16_smem_floats<BM, BN, BK, S, EPI_T, PX>()];
  gemm16_body<BM, BN, BK, WM, WN, S, SP, A_KC, B_KC, EPI_T, PX>(p_in, smem, blockIdx.x);
}

// Two independent GEMMs in ONE launch: blocks [0, na) are GEMM A's tiles, the rest GEMM B's (2x2-wave
// BK-64 two-slot configurations; one LDS array of the larger size, one workgroup per CU).  The training
// step pairs the weight update of layer l with the backward GEMM of layer l-1 (disjoint operands: the
// update writes W_l, the backward reads W_{l-1}): the blocks are dispatched in index order, so B's
// workgroups start on the CUs A's finish on -- B's operand fill overlaps A's epilogue stores and tail
// instead of waiting for a kernel boundary, A's end-of-kernel drain and B's start-up spread.
// SPA: GEMM A's form (0: the LDS ring, 5: the direct form -- TNET_GEMM_DIRECT); SPB: GEMM B's (0, or 8: the
// direct form with coalesced k-contiguous loads -- TNET_GEMM_KC); KTA / STA: GEMM A's k-tile and slot count (the
// top layer's 128x256 update: 32 / 3, its m128x256a2 form)
template <int BMA, int BNA, bool AKA, bool BKA, int EPIA, bool PXA, int BMB, int BNB, bool AKB, bool BKB, int EPIB,
          bool PXB, int SPA = 0, int SPB = 0, int KTA = 64, int STA = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm16_pair_kernel(const GemmP pa, const GemmP pb, const int na) {
  constexpr int SA = gemm16_smem_floats<BMA, BNA, KTA, STA, EPIA, PXA>(), SB = gemm16_smem_floats<BMB, BNB, 64, 2, EPIB, PXB>();
  __shared__ __attribute__((aligned(16))) float smem[SA > SB ? SA : SB];
  if ((int)blockIdx.x < na) gemm16_body<BMA, BNA, KTA, 2, 2, STA, SPA, AKA, BKA, EPIA, PXA>(pa, smem, blockIdx.x);
  else gemm16_body<BMB, BNB, 64, 2, 2, 2, SPB, AKB, BKB, EPIB, PXB>(pb, smem, (int)blockIdx.x - na);
}

// Two independent SMALL weight updates (fused SGD + bias SGD, TN) in ONE launch, same tile
// configuration for both (64x64, BK 32, four slots, 4x1 waves), blocks [0, na) update A, the rest B.
// For the step's last two updates when neither fills the chip (the MLP3's 1024x135 and 598x1024: 48 +
// 160 tiles): both grids run side by side in one round instead of back to back (and the 1024x135 one
// without its split-K combine launch).  A second HIP stream for the same overlap was measured slower
// (the cross-stream fork / join costs more than the overlap saves at this size).
template <int BM, int BN, int BK, int WM, int WN, int S>
__global__ __launch_bounds__(WM * WN * 64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm16_upd_pair_kernel(const GemmP pa, const GemmP pb, const int na) {
  __shared__ __attribute__((aligned(16))) float smem[gemm16_smem_floats<BM, BN, BK, S, EPI_SGD_B, false>()];
  if ((int)blockIdx.x < na) gemm16_body<BM, BN, BK, WM, WN, S, 0, false, false, EPI_SGD_B, false>(pa, smem, blockIdx.x);
  else gemm16_body<BM, BN, BK, WM, WN, S, 0, false, false, EPI_SGD_B, false>(pb, smem, (int)blockIdx.x - na);
}

// tnet_affine_update_bias_gather: the update pair kernel's tiles (nb = 0: one update) and ng gather blocks
// after them.  Blocks are dispatched in index order, so the gather blocks take the CUs the update's tiles
// leave free (one workgroup per CU: the ring's LDS and 1 wave per SIMD) and run beside the tiles.
// EPI_STORE_BG: the data-parallel step's last gradient GEMM(s) (tnet_affine_grad_bias_gather).
template <int BM, int BN, int BK, int WM, int WN, int S, int EPI = EPI_SGD_B>
__global__ __launch_bounds__(WM * WN * 64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm16_upd_gather_kernel(const GemmP pa, const GemmP pb, const int na, const int nb, const BunchGatherP g) {
  __shared__ __attribute__((aligned(16))) float smem[gemm16_smem_floats<BM, BN, BK, S, EPI, false>()];
  const int b = blockIdx.x;
  if (b < na) gemm16_body<BM, BN, BK, WM, WN, S, 0, false, false, EPI, false>(pa, smem, b);
  else if (b < na + nb) gemm16_body<BM, BN, BK, WM, WN, S, 0, false, false, EPI, false>(pb, smem, b - na);
  else bunch_gather_block(g, b - na - nb, (int)gridDim.x - na - nb);
}

// The fused step's last two weight updates when they take different tile configurations -- a 2048-wide layer's
// (128x128 direct form, exact prefetch: what tnet_affine_update_bias runs for it) and the first layer's (64x64,
// BK 32, four slots, 4x1 waves) -- and the next bunch's gather, in ONE launch: blocks [0, na) the big update's
// tiles (one round over the CUs), then the small update's tiles and the gather blocks, which take the CUs as the
// big grid's tail drains instead of after a kernel boundary.  Each half runs its separate launch's body: the
// results are bit-identical to the two calls.
// BD: B's tiles in the 64x64 direct form (m64x64a4, what tnet_affine_update_bias runs for B's shape then), else the
// 64x64 ring form with 16x64 wave tiles (m64x64k32s4w41)
template <bool BD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm16_upd_mixed_gather_kernel(const GemmP pa, const GemmP pb, const int na, const int nb, const BunchGatherP g) {
  constexpr int SA = gemm16_smem_floats<128, 128, 64, 2, EPI_SGD_B, true>();
  constexpr int SB = BD ? gemm16_smem_floats<64, 64, 64, 2, EPI_SGD_B, false>()
                        : gemm16_smem_floats<64, 64, 32, 4, EPI_SGD_B, false>();
  __shared__ __attribute__((aligned(16))) float smem[SA > SB ? SA : SB];
  const int b = blockIdx.x;
  if (b < na) {
    gemm16_body<128, 128, 64, 2, 2, 2, 5, false, false, EPI_SGD_B, true>(pa, smem, b);
  } else if (b < na + nb) {
    if constexpr (BD) gemm16_body<64, 64, 64, 2, 2, 2, 5, false, false, EPI_SGD_B, false>(pb, smem, b - na);
    else gemm16_body<64, 64, 32, 4, 1, 4, 0, false, false, EPI_SGD_B, false>(pb, smem, b - na);
  } else {
    bunch_gather_block(g, b - na - nb, (int)gridDim.x - na - nb);
  }
}

// tnet_affine_bwd_colsum_slabs: the top layer's backward GEMM (64x128 NT + diff-sigmoid + Eo's slab sums,
// na tiles) and the slab sums of its OWN input error E (the softmax error: the top layer's bias gradient,
// colsum_partial blocks after the tiles).  Independent (the GEMM reads E, the blocks read E); the blocks
// take the CUs as the tiles finish instead of a launch of their own before the GEMM.
// BKC false: the GEMM from the weight's transposed shadow (NN, tnet_affine_bwd_colsum_slabs_t)
template <bool PX, int SP = 0, bool BKC = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm16_bwd_slabs_kernel(const GemmP p, const int na, const float* __restrict__ Et, const TnetMatrixDim dEt,
                             float* __restrict__ cpt, const long ldcpt, const int slabs, const int ncb) {
  __shared__ __attribute__((aligned(16))) float smem[gemm16_smem_floats<64, 128, 64, 2, EPI_DSIG_CS, PX>()];
  const int b = blockIdx.x;
  if (b < na) {
    gemm16_body<64, 128, 64, 2, 2, 2, SP, true, BKC, EPI_DSIG_CS, PX>(p, smem, b);
  } else {
    const int c = b - na;
    colsum_partial_block<true>(Et, dEt, cpt, slabs, 0x7fffffff, ldcpt, c % ncb, c / ncb, smem);
  }
}

// One RBM step's CD-1 weight update (tnet_rbm_update: 64x64 TN tiles + EPI_RBM) and its statistics
// (tnet_rbm_stats_update: both bias updates + the reconstruction MSE, rbm_stats.h) in ONE launch: blocks
// [0, na) the GEMM's tiles, the rest the statistics blocks.  Independent: both read the stacked V and H;
// the GEMM writes W and its momentum, the statistics the biases, their momentum and the MSE slots.  The
// statistics blocks run beside the GEMM's tiles instead of after them.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm16_rbm_update_stats_kernel(const GemmP p, const int na, const float* __restrict__ Vs, TnetMatrixDim dV,
                                    const float* __restrict__ Hs, TnetMatrixDim dH, int B, int nvb,
                                    float* __restrict__ vb, float* __restrict__ cvb, float* __restrict__ hb,
                                    float* __restrict__ chb, float scale, float mmt, double* __restrict__ stats,
                                    int nhb, const BunchGatherP g, const int ng) {
  // blocks [na, na + ng): the next bunch's gather (tnet_rbm_update_stats_gather; ng = 0 without one)
  constexpr int SG = gemm16_smem_floats<64, 64, 32, 4, EPI_RBM, false>();
  __shared__ __attribute__((aligned(16))) float smem[SG > RS_SMEM_FLOATS ? SG : RS_SMEM_FLOATS];
  const int b = blockIdx.x;
  if (b < na) gemm16_body<64, 64, 32, 4, 1, 4, 0, false, false, EPI_RBM, false>(p, smem, b);
  else if (b < na + ng) bunch_gather_block(g, b - na, ng);
  else rbm_stats_block(b - na - ng, smem, Vs, dV, Hs, dH, B, nvb, vb, cvb, hb, chb, scale, mmt, stats, nhb);
}

// ---------------------------------------------------------------------------------------------
// split-K combine: C = epilogue(P[0] + P[1] + ... + P[splits-1]) summed in split order (fixed, so the
// result is deterministic), then the same epilogue arithmetic as gemm16_kernel; 4 columns / thread
// ---------------------------------------------------------------------------------------------
constexpr bool epi_splittable(int e) { return e != EPI_DSIG_CS && e != EPI_BIAS_SIG_BIN; }

template <int EPI_FULL>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmP p, const float* __restrict__ P, long slab,
                                                            int splits, int ldp, unsigned main_blocks) {
  if constexpr (epi_bias_slabs(EPI_FULL)) {
    // EPI_SGD_B / EPI_STORE_BG: the trailing workgroups update (or store) the bias, a column per
    // thread, with the fused epilogue's own arithmetic (bias_pre_load / bias_pre_finish)
    if (blockIdx.x >= main_blocks) {
      constexpr bool GRAD = EPI_FULL == EPI_STORE_BG;
      const int bn = (int)(blockIdx.x - main_blocks) * 256;
      BiasPre bp;
      bias_pre_load<256, GRAD>(p, bn, bp);
      bias_pre_finish<256, GRAD>(p, bn, bp);
      return;
    }
  }
  constexpr int EPI = epi_base(EPI_FULL);
  const int N4 = (p.N + 3) >> 2;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)p.M * N4) return;
  const int row = (int)(i / N4), col = (int)(i % N4) * 4;
  combine4<EPI>(p, P, slab, splits, ldp, row, col);
}

// ---------------------------------------------------------------------------------------------
// The top layer of a TNet MLP for at most 256 classes (BASELINE config 2's 135 senones): the
// GEMM's slices combined with the bias into the logits, softmax + cross-entropy + error + frame
// accuracy per row, and the error's 32-row slab column sums (the top layer's bias gradient), in ONE
// workgroup per slab -- replacing splitk_reduce_kernel<EPI_BIAS> + softmax_xent_kernel +
// colsum_partial_kernel (tnet_affine_fwd, tnet_softmax_xent, tnet_colsum_slab_sums).
//   * logits: the slices added in slice order, then + bias (splitk_reduce_kernel's arithmetic);
//   * softmax row: softmax_xent_kernel's arithmetic and lane-to-column map (4 contiguous columns a
//     lane when v4, else columns lane + 64 j), so Y / E / the statistics per row are its values;
//   * slab sums: fp32 over the slab's rows in row order (a thread per column).
// ---------------------------------------------------------------------------------------------
constexpr int kSxMaxN = TNET_AFFINE_SOFTMAX_MAX_N;
constexpr int kSxThreads = 1024;  // 16 waves, 2 rows each
constexpr int kSxPer = kColsumSlabRows * (kSxMaxN / 4) / kSxThreads;  // float4 logits per thread
__global__ __launch_bounds__(kSxThreads) void affine_softmax_xent_kernel(
    const GemmP p, const float* __restrict__ P, long slab, int splits, int ldp, const int* __restrict__ labels,
    float* __restrict__ Z, long ldz, float* __restrict__ Y, long ldy, float* __restrict__ E, long lde,
    double* __restrict__ stats, float* __restrict__ cpart, long ldcpart, int v4) {
  constexpr int NW = kSxThreads / 64;
  __shared__ __attribute__((aligned(16))) float zs[kColsumSlabRows * kSxMaxN];
  __shared__ int s_lab[kColsumSlabRows];
  __shared__ double red[2][NW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int N = p.N, r0 = blockIdx.x * kColsumSlabRows, nr = min(kColsumSlabRows, p.M - r0);
  if (tid < nr) s_lab[tid] = labels[r0 + tid];
  // ---- logits of the slab into LDS (and Z): every slice's loads of a thread in flight together
  const int N4 = (N + 3) >> 2, n = nr * N4;
  f32x4 v[kSxPer], bv[kSxPer];
#pragma unroll
  for (int k = 0; k < kSxPer; ++k) {
    const int i = min(tid + kSxThreads * k, n - 1), r = i / N4, c = (i % N4) * 4;
    v[k] = *reinterpret_cast<const f32x4*>(P + (long)(r0 + r) * ldp + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[k][e] = c + e < N ? p.bias[c + e] : 0.f;
  }
  // the other slices: up to kSxBatch of them requested before the first add (one memory round trip instead of
  // one per slice: the planner gives this kernel 2 slices at MLP3's 1024 x 1024 -> 135), added in slice order
  constexpr int kSxBatch = 4;
  for (int z0 = 1; z0 < splits; z0 += kSxBatch) {
    f32x4 t[kSxBatch][kSxPer];
#pragma unroll
    for (int b = 0; b < kSxBatch; ++b) {
      const int z = min(z0 + b, splits - 1);
#pragma unroll
      for (int k = 0; k < kSxPer; ++k) {
        const int i = min(tid + kSxThreads * k, n - 1), r = i / N4, c = (i % N4) * 4;
        t[b][k] = *reinterpret_cast<const f32x4*>(P + (long)z * slab + (long)(r0 + r) * ldp + c);
      }
    }
#pragma unroll
    for (int b = 0; b < kSxBatch; ++b) {
      if (z0 + b >= splits) break;
#pragma unroll
      for (int k = 0; k < kSxPer; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[k][e] = v[k][e] + t[b][k][e];
    }
  }
#pragma unroll
  for (int k = 0; k < kSxPer; ++k) {
    const int i = tid + kSxThreads * k;
    if (i >= n) break;
    const int r = i / N4, c = (i % N4) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (c + e >= N) break;
      const float y = v[k][e] + bv[k][e];
      zs[r * kSxMaxN + c + e] = y;
      if (Z) Z[(long)(r0 + r) * ldz + c + e] = y;
    }
  }
  __syncthreads();
  // ---- softmax / xent / error, a wave per row (rows wv, wv + NW, ...)
  double wx = 0.0, wc = 0.0;
  for (int r = wv; r < nr; r += NW) {
    float* zr = zs + r * kSxMaxN;
    const long row = r0 + r;
    int t = s_lab[r];
    if (t >= N) t = -1;  // unlabeled (the host intake rejects such a label, CheckLabels)
    float x[4];
    int cl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cl[j] = v4 ? 4 * lane + j : lane + 64 * j;
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
        if (Y) Y[row * ldy + cl[j]] = y;
        E[row * lde + cl[j]] = e;
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
  if (tid == 0 && stats) {
    double sx = 0.0, sc = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      sx += red[0][w];
      sc += red[1][w];
    }
    const int slot = blockIdx.x % TNET_STATS_SLOTS;
    atomicAdd(stats + 2 * slot, sx);
    atomicAdd(stats + 2 * slot + 1, sc);
  }
  // ---- the slab's column sums of the error
  if (cpart)
    for (int c = tid; c < N; c += kSxThreads) {
      float a = 0.f;
      for (int r = 0; r < nr; ++r) a += zs[r * kSxMaxN + c];
      cpart[(long)blockIdx.x * ldcpart + c] = a;
    }
}

// per-stream partial-product workspace of the split-K path (grown on demand; the library enqueues
// a stream's GEMMs in order, so one buffer per stream is reused launch after launch)
static std::mutex g_skws_mu;
static std::map<hipStream_t, std::pair<void*, size_t>> g_skws;
static float* splitk_workspace(size_t bytes, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_skws_mu);
  auto& w = g_skws[st];
  if (bytes > w.second) {
    if (w.first) {
      if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
      (void)hipFree(w.first);
      w = {nullptr, 0};
    }
    void* q = nullptr;
    if (hipMalloc(&q, bytes) != hipSuccess) return nullptr;
    w = {q, bytes};
  }
  return (float*)w.first;
}

// per-stream tile counters of the in-launch combine: zeroed at allocation, and every tile's last
// slice puts its counter back to 0, so a stream's next launch finds them zero
static std::map<hipStream_t, std::pair<unsigned*, size_t>> g_skcnt;
static unsigned* splitk_counters(size_t n, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_skws_mu);
  auto& w = g_skcnt[st];
  if (n > w.second) {
    if (w.first) {
      if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
      (void)hipFree(w.first);
      w = {nullptr, 0};
    }
    const size_t cap = (n + 1023) & ~(size_t)1023;
    void* q = nullptr;
    if (hipMalloc(&q, cap * sizeof(unsigned)) != hipSuccess) return nullptr;
    if (hipMemsetAsync(q, 0, cap * sizeof(unsigned), st) != hipSuccess) return nullptr;
    w = {(unsigned*)q, cap};
  }
  return w.first;
}

// ---------------------------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------------------------
// name: g<BM>x<BN>k<BK>s<S>w<waves>[i]: 32x32x2 kernel (waves laid out WMxWN; i = DMA pieces
//       interleaved); m<BM>x<BN>k<BK>s<S>[w<WM><WN>][p|L]: 16x16x4 kernel (default 2x2 waves; p = DMA
//       pieces spread over the chunks + MFMA at setprio 1; L = one extra loader wave issues all DMA);
//       m<BM>x<BN>d<D>: the 16x16x4 kernel's direct form (fragments loaded from global memory into a
//       D-chunk register ring, no LDS ring)
#define TNET_GEMM_CFGS(X)                         \
  X(g64x64k32s4w4, 0, 64, 64, 32, 2, 2, 4, 0)           \
  X(m64x64k32s4w41, 1, 64, 64, 32, 4, 1, 4, 0)          \
  X(m128x128k64s2, 1, 128, 128, 64, 2, 2, 2, 0)         \
  X(m64x128k64s2, 1, 64, 128, 64, 2, 2, 2, 0)           \
  X(m64x128a4, 1, 64, 128, 64, 2, 2, 2, 5)              \
  X(m64x128a8, 1, 64, 128, 64, 2, 2, 2, 6)              \
  X(m128x128a4, 1, 128, 128, 64, 2, 2, 2, 5)            \
  X(m128x256a2, 1, 128, 256, 32, 2, 2, 3, 7)            \
  X(m64x128c8, 1, 64, 128, 64, 2, 2, 2, 8)              \
  X(m128x256k32s3, 1, 128, 256, 32, 2, 2, 3, 0)         \
  X(m64x64k64s2, 1, 64, 64, 64, 2, 2, 2, 0)             \
  X(m64x64k32s4, 1, 64, 64, 32, 2, 2, 4, 0)             \
  X(m32x64k64s2, 1, 32, 64, 64, 2, 2, 2, 0)             \
  X(m64x64a4, 1, 64, 64, 64, 2, 2, 2, 5)

enum GemmCfg {
#define X(name, ...) CFG_##name,
  TNET_GEMM_CFGS(X)
#undef X
  CFG_COUNT
};
static const char* kCfgNames[CFG_COUNT] = {
#define X(name, ...) #name,
    TNET_GEMM_CFGS(X)
#undef X
};

static int g_cfg = -2;  // -2: not initialised, -1: automatic
static int g_group = -1;
static int g_split = -1;  // TNET_GEMM_SPLITK: forced split-K count (diagnostics / sweeps), -1 automatic
static int g_early = 1;   // TNET_GEMM_EARLY=0: prologue issues S-1 slots before the first wait (round-1 form)
// (the split-K combine is a second launch: round 2's in-launch combine by each tile's last slice was measured
// SLOWER on every MLP3 / RBM shape -- the 1024 x 135 update 19.0 vs 14.6 us, MLP3 10.45 M vs 10.96 M frames/s, the
// agent-scope release + acquire costing more than the launch boundary -- and is gone since round 6)
static int g_pair = 1;  // TNET_GEMM_PAIR=0: tnet_affine_update_bwd_pair never pairs (A/B measurements)
static int g_pre0 = 1;  // TNET_GEMM_PRE0=0: the first seam also waits for the epilogue-operand prefetch
// CUs reserved for another kernel (RCCL's channel workgroups) while the data-parallel step's collectives
// are in flight (tnet_gemm_reserve, set by the gradient exchange; tnet_gemm_config "+rsv<R>" for tests):
// the 64x128 backward / forward and the 128x128 gradient then run as stream-K over CUs - R workgroups
// (gemm16_sk_kernel).  0: the plain tile grid.
static int g_reserve = 0, g_cus = 0;
// TNET_GEMM_DIRECT: the planner's m64x128k64s2 / m128x128k64s2 choices with an n-contiguous B (the forward
// and update GEMMs; the backward's k-contiguous B reads 64-B row pieces, slower direct: 99 vs 78 us) run in
// the direct form -- 1: m64x128a8 / m128x128a4, also the update half of the update + backward pair kernel
// (dnn4 969.9 k -> 1006.2 k frames/s, the 2048^2 set 69.1 -> 65.6 us a launch, roofline 0.790 -> 0.832,
// profiles/r04_gemm_direct_ab.json); 4 (default): 1 + the 128x256 update (the top layer's) as m128x256a2
// (134.6 -> 126.3 us, dnn4 1005 k -> 1015 k, profiles/r04_gemm_direct_128x256_ab.jsonl); 3: m64x128a4 /
// m128x128a4; 0: the LDS ring everywhere.  (Round 6 removed the configurations measured never faster: the
// compiler-tracked direct forms d4 / d8, the loader-wave and spread-DMA rings, the 8-wave 64x128, the 3-slot /
// 32-deep ring variants and c4 -- profiles/r02_*, r04_gemm_direct_variants.jsonl keep the sweeps)
static int g_direct = -1;
// TNET_GEMM_KC: the backward GEMMs (k-contiguous A and B, 64x128 tiles) in the direct form with coalesced loads,
// m64x128c8, instead of the LDS ring -- 1 (default): the top layer's (1024 x 2048 over K = 4000, with its own
// slab sums, tnet_affine_bwd_colsum_slabs): 135.1 -> 133.0 us in the SGD step; 2: also the 2048^2 backward
// alone (71.3 -> 72.5 us, slower) and in the update + backward pair (67.2 -> 67.1 us); 0: the ring everywhere
// (profiles/r04_gemm_kc_ab.json)
static int g_kc = -1;
static int g_wt = 1;  // TNET_GEMM_WT=0: plain 16-B epilogue stores instead of write-through (sc1; measured +1.4 % frames/s)
// Transposed weight shadows (tnet_weight_shadow): W -> Wt registered by the host; an update launch of W attaches
// Wt as GemmP::Ct (shadow_attach) and the launch paths whose kernel does not run gemm16_body's SGD epilogue (the
// 32x32 kernel, the split-K combine, split2) drop it (shadow_drop); the entry point then records whether this
// update of W kept its shadow (shadow_done), which tnet_weight_shadow_kept reports
// the narrow top layer's K-slice kernel (top_rows.hip): the shapes it takes, and the slices
extern "C" int tnetk_top_rows_shape_ok(const float* X, long ldx, const float* W, long ldw, int M, int N, int K);
extern "C" int tnetk_top_rows_partials(const float* X, long ldx, const float* W, long ldw, int M, int N, int K,
                                       float* part, long ldpart, void* stream);
static int forced_cfg();
static bool upd64_direct(const GemmP& p);
// The narrow top layer's K slices from top_rows.hip's row-block kernel (16-row blocks x 4 K slices = 256
// workgroups, operands straight into registers) into the split-K workspace [4][M][ldp], for
// the second launch that combines them -- affine_softmax_xent_kernel (tnet_affine_softmax_xent) or
// splitk_reduce_kernel (tnet_affine_fwd: the same slices, so both give the same Z) -- instead of the 32x64 split-K
// tiles (TNET_TOP_SPLIT=0: those)
constexpr int kTopSlices = 4;
static float* splitk_workspace(size_t bytes, hipStream_t st);
static bool top_split_ok(const GemmP& p) {
  static const bool on = !(getenv("TNET_TOP_SPLIT") && getenv("TNET_TOP_SPLIT")[0] == '0');
  return on && forced_cfg() < 0 && g_split <= 0 && tnetk_top_rows_shape_ok(p.A, p.lda, p.B, p.ldb, p.M, p.N, p.K);
}
static float* top_split_partials(const GemmP& p, hipStream_t st, int* ldp_out) {
  const int ldp = 16 * ((p.N + 15) / 16);
  float* ws = splitk_workspace(sizeof(float) * kTopSlices * (size_t)p.M * ldp, st);
  if (!ws) return nullptr;
  if (tnetk_top_rows_partials(p.A, p.lda, p.B, p.ldb, p.M, p.N, p.K, ws, ldp, st) != TNET_OK) return nullptr;
  *ldp_out = ldp;
  return ws;
}
struct WeightShadow {
  float* t;
  long ld;
  int rows, cols;
  int kept;
};
static std::mutex g_shadow_mu;
static std::unordered_map<const float*, WeightShadow> g_shadow;
static thread_local int g_shadow_dropped = 0;
static void shadow_attach(GemmP& p) {
  p.Ct = nullptr;
  p.ldct = 0;
  g_shadow_dropped = 0;
  std::lock_guard<std::mutex> g(g_shadow_mu);
  auto it = g_shadow.find(p.C);
  if (it != g_shadow.end() && it->second.rows == p.M && it->second.cols == p.N) {
    p.Ct = it->second.t;
    p.ldct = it->second.ld;
  }
}
static void shadow_drop(const GemmP& p) {
  if (p.Ct) g_shadow_dropped = 1;
}
static int shadow_done(const GemmP& p, int st) {
  std::lock_guard<std::mutex> g(g_shadow_mu);
  auto it = g_shadow.find(p.C);
  if (it != g_shadow.end()) it->second.kept = (st == TNET_OK && p.Ct && !g_shadow_dropped) ? 1 : 0;
  return st;
}
static int forced_cfg() {
  if (g_cfg == -2) {
    g_cfg = -1;
    const char* e = getenv("TNET_GEMM_CFG");
    if (e)
      for (int i = 0; i < CFG_COUNT; i++)
        if (!strcmp(e, kCfgNames[i])) g_cfg = i;
    const char* gg = getenv("TNET_GEMM_GROUP");
    if (gg) g_group = atoi(gg);
    const char* sk = getenv("TNET_GEMM_SPLITK");
    if (sk) g_split = atoi(sk);
    const char* ea = getenv("TNET_GEMM_EARLY");
    if (ea) g_early = atoi(ea);
    const char* pr = getenv("TNET_GEMM_PAIR");
    if (pr) g_pair = atoi(pr);
    const char* p0 = getenv("TNET_GEMM_PRE0");
    if (p0) g_pre0 = atoi(p0);
    const char* wt = getenv("TNET_GEMM_WT");
    if (wt) g_wt = atoi(wt);
    const char* dr = getenv("TNET_GEMM_DIRECT");
    g_direct = dr ? atoi(dr) : 4;
    const char* kc = getenv("TNET_GEMM_KC");
    g_kc = kc ? atoi(kc) : 1;

  }
  return g_cfg;
}

// the exact-prefetch instantiation (PX) may run this launch: the grid covers M x N exactly, the epilogue
// operands are 16-B aligned, and (bias epilogues) every column's slab sums fit one workgroup's 256 lanes
// (32 slabs x 8 columns of the tile per tile-row)
template <int BM, int BN, int EPI>
static bool px_exact(const GemmP& p) {
  auto a16 = [](const void* v) { return ((uintptr_t)v & 15) == 0; };
  return g_pre0 && p.ksplit <= 1 && p.M % BM == 0 && p.N % BN == 0 && (p.ldc & 3) == 0 && a16(p.C) &&
         (!p.bias || a16(p.bias)) && (!p.aux || (a16(p.aux) && (p.ldaux & 3) == 0)) &&
         (!p.corr || (a16(p.corr) && (p.ldcorr & 3) == 0)) &&
         (!epi_bias_slabs(EPI) ||
          (p.bslabs >= 1 && p.bslabs <= kBiasPreSlabs && (BN + p.M / BM - 1) / (p.M / BM) <= 8));
}

template <int KIND, int BM, int BN, int BK, int WM, int WN, int S, int IL, bool A_KC, bool B_KC, int EPI>
static bool launch_cfg(const GemmP& p, hipStream_t st) {
  const unsigned tiles = (unsigned)((long)cdiv(p.M, BM) * cdiv(p.N, BN));
  if constexpr (KIND == 0) {
    shadow_drop(p);  // the 32x32 kernel's epilogue writes no transposed shadow
    gemm_f32_glds_kernel<BM, BN, BK, WM, WN, S, IL, A_KC, B_KC, EPI><<<tiles, WM * WN * 64, 0, st>>>(p);
    return true;
  } else {
    constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
    // the 16x16 kernel addresses a k-tile with 32-bit byte offsets from a per-tile base
    const long extA = A_KC ? (long)p.M * p.lda : (long)BK * p.lda + p.M;
    const long extB = B_KC ? (long)p.N * p.ldb : (long)BK * p.ldb + p.N;
    if (4 * extA >= (1L << 32) || 4 * extB >= (1L << 32)) return false;
    const dim3 grid(tiles, p.ksplit > 1 ? p.ksplit : 1);
    GemmP q = p;
    q.early_issue = g_early;
    // write-through epilogue stores: not where the workgroup reads its own stores back (RBM sampling)
    q.wt = EPI == EPI_BIAS_SIG_BIN ? 0 : g_wt;
    // the exact-prefetch instantiation (PX) only for the training step's large-layer kernels: the
    // hidden forward (64x128 NN + bias + sigmoid), backward (64x128 NT + diff-sigmoid + slab sums)
    // and update (128x128 TN + SGD / the data-parallel gradient)
    constexpr bool PXK = (IL == 0 || IL >= 3) && BK == 64 && S == 2 &&
                         ((BM == 64 && BN == 128 && A_KC && !B_KC && EPI == EPI_BIAS_SIG) ||
                          (BM == 64 && BN == 128 && A_KC && EPI == EPI_DSIG_CS) ||
                          (BM == 128 && BN == 128 && !A_KC && !B_KC &&
                           (EPI == EPI_SGD_B || EPI == EPI_SGD || EPI == EPI_STORE_BG)));
    const bool exact = px_exact<BM, BN, EPI>(p);
    if constexpr (IL >= 3) {
      // the direct form loads 16-B fragments (clamped at the M / N edges) over the full k-tiles: 16-B
      // aligned operands, at least one full k-tile (DD = 8: an even count); otherwise the ring form
      const int nfull = p.K / BK;
      auto a16p = [](const void* v) { return ((uintptr_t)v & 15) == 0; };
      // (an m / n-contiguous operand's 16-B vectors are either wholly inside or wholly past the edge:
      // M / N a multiple of 4 there)
      if (p.ksplit > 1 || nfull < 1 || (!A_KC && p.M % 4) || (!B_KC && p.N % 4) || ((IL == 4 || IL == 6 || IL == 8) && nfull % 2) ||
          (p.lda & 3) || (p.ldb & 3) || !a16p(p.A) ||
          !a16p(p.B) || 4 * (A_KC ? (long)p.M * p.lda : (long)p.K * p.lda) >= (1L << 31) ||
          4 * (B_KC ? (long)p.N * p.ldb : (long)p.K * p.ldb) >= (1L << 31))
        return launch_cfg<KIND, BM, BN, BK, WM, WN, S, 0, A_KC, B_KC, EPI>(p, st);
    }
    if constexpr (PXK) {
      if (exact) {
        gemm16_kernel<BM, BN, BK, WM, WN, S, IL, A_KC, B_KC, EPI, true><<<grid, WM * WN * 64, 0, st>>>(q);
        return true;
      }
    }
    gemm16_kernel<BM, BN, BK, WM, WN, S, IL, A_KC, B_KC, EPI><<<grid, (WM * WN + (IL == 2)) * 64, 0, st>>>(q);
    return true;
  }
}

// a 64x128 backward grid (k-contiguous A and B) may run m64x128c8 (TNET_GEMM_KC; launch_cfg's direct-form
// conditions: whole k-tiles in an even count, 16-B aligned operands, 31-bit offsets)
static bool kc_direct(const GemmP& p) {
  forced_cfg();
  auto a16p = [](const void* v) { return ((uintptr_t)v & 15) == 0; };
  const int nfull = p.K / 64;
  return g_kc > 0 && p.ksplit <= 1 && nfull >= 1 && nfull % 2 == 0 && !(p.lda & 3) && !(p.ldb & 3) && a16p(p.A) &&
         a16p(p.B) && 4L * p.M * p.lda < (1L << 31) && 4L * p.N * p.ldb < (1L << 31);
}

static void cfg_shape(int cfg, int* bm, int* bn, int* kind) {
  switch (cfg) {
#define X(name, KIND, BM, BN, BK, WM, WN, S, IL) \
  case CFG_##name: *bm = BM; *bn = BN; *kind = KIND; return;
    TNET_GEMM_CFGS(X)
#undef X
    default: *bm = 64; *bn = 64; *kind = 0;
  }
}

// gemm16_sk_kernel launch of a PX-exact 64x128 / 128x128 BK-64 two-slot shape over CUs - g_reserve
// workgroups; false: not applicable (no reservation, other shapes)
template <int BM, int BN, bool A_KC, bool B_KC, int EPI>
static bool launch_sk(const GemmP& p, hipStream_t st) {
  forced_cfg();
  if (g_reserve <= 0) return false;
  constexpr bool OK = (BM == 64 && BN == 128 && A_KC && B_KC && EPI == EPI_DSIG_CS) ||
                      (BM == 64 && BN == 128 && A_KC && !B_KC && EPI == EPI_BIAS_SIG) ||
                      (BM == 128 && BN == 128 && !A_KC && !B_KC && (EPI == EPI_STORE_BG || EPI == EPI_STORE));
  if constexpr (!OK) {
    return false;
  } else {
    if (!g_cus) {
      int dev = 0;
      hipDeviceProp_t prop;
      if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
      g_cus = prop.multiProcessorCount;
    }
    const long T = (long)cdiv(p.M, BM) * cdiv(p.N, BN);
    const int G = g_cus - g_reserve;
    if (G < 1 || T < G || T > 8L * G || p.K % 64 || p.K < 128 || !px_exact<BM, BN, EPI>(p)) return false;
    const long extA = A_KC ? (long)p.M * p.lda : 64L * p.lda + p.M;
    const long extB = B_KC ? (long)p.N * p.ldb : 64L * p.ldb + p.N;
    if (4 * extA >= (1L << 32) || 4 * extB >= (1L << 32)) return false;
    // T >= G: every range is at least KT k-tiles long, so a tile is cut into at most two pieces
    float* ws = splitk_workspace(sizeof(float) * (size_t)T * BM * BN, st);
    unsigned* cnt = ws ? splitk_counters((size_t)T, st) : nullptr;
    if (!cnt) return false;
    GemmP q = p;
    q.group = g_group > 0 ? g_group : 8;
    q.early_issue = g_early;
    q.wt = g_wt;
    q.skws = ws;
    q.tile_cnt = cnt;
    // the pieces in the direct form where the plain grid would run it (n-contiguous B, aligned operands)
    auto a16p = [](const void* v) { return ((uintptr_t)v & 15) == 0; };
    const bool dir = g_direct > 0 && !B_KC && !(p.lda & 3) && !(p.ldb & 3) && a16p(p.A) && a16p(p.B) &&
                     (A_KC || p.M % 4 == 0) && p.N % 4 == 0 &&
                     4 * (A_KC ? (long)p.M * p.lda : (long)p.K * p.lda) < (1L << 31) &&
                     4 * (B_KC ? (long)p.N * p.ldb : (long)p.K * p.ldb) < (1L << 31);
    if constexpr (!B_KC) {
      if (dir) {
        gemm16_sk_kernel<BM, BN, 64, 2, 2, 2, A_KC, B_KC, EPI, 5><<<(unsigned)G, 256, 0, st>>>(q, G);
        return true;
      }
    }
    gemm16_sk_kernel<BM, BN, 64, 2, 2, 2, A_KC, B_KC, EPI><<<(unsigned)G, 256, 0, st>>>(q, G);
    return true;
  }
}

// gemm16_split2_kernel for the update GEMMs whose 64x128 tiles are too few for the CUs (the first
// layer's 440 x 2048 over K = 1024: 112 tiles -> 224 pieces of K = 512).  Opt-in (TNET_GEMM_SPLIT2=1):
// MEASURED SLOWER on MI355X (tools/gemm_sweep.py, round 3): 28.3 vs 24.5 us with the bias SGD, 27.4 vs
// 22.8 us without -- the update's m-contiguous A in 64-row tiles reads its fragments 8 B per lane, and
// 8 k-tiles per piece leave the prologue / epilogue unamortised.  false: not applicable
static int g_split2 = -1;
template <bool A_KC, bool B_KC, int EPI>
static bool launch_split2(const GemmP& p, hipStream_t st) {
  if (g_split2 < 0) g_split2 = getenv("TNET_GEMM_SPLIT2") ? atoi(getenv("TNET_GEMM_SPLIT2")) : 0;
  constexpr bool OK = !A_KC && !B_KC && (EPI == EPI_SGD_B || EPI == EPI_SGD || EPI == EPI_STORE_BG || EPI == EPI_STORE);
  if constexpr (!OK) {
    return false;
  } else {
    if (!g_split2 || forced_cfg() >= 0 || g_split > 0) return false;
    const long T = (long)cdiv(p.M, 64) * cdiv(p.N, 128);
    if (T < 90 || T > 160 || p.K % 128 || p.K < 512 || p.N % 128) return false;
    const long extA = 64L * p.lda + p.M, extB = 64L * p.ldb + p.N;
    if (4 * extA >= (1L << 32) || 4 * extB >= (1L << 32)) return false;
    float* ws = splitk_workspace(sizeof(float) * (size_t)T * 64 * 128, st);
    unsigned* cnt = ws ? splitk_counters((size_t)T, st) : nullptr;
    if (!cnt) return false;
    GemmP q = p;
    q.group = g_group > 0 ? g_group : 8;
    q.early_issue = g_early;
    q.wt = g_wt;
    q.skws = ws;
    q.tile_cnt = cnt;
    shadow_drop(p);
    gemm16_split2_kernel<64, 128, A_KC, B_KC, EPI, false><<<(unsigned)(2 * T), 256, 0, st>>>(q);
    return true;
  }
}

// split-K: the K range is cut into ks slices (blockIdx.y) whose raw products A B go to the stream's
// workspace (slice z at ws + z * slab, rows of ldp = N rounded up to 4 floats); then
// splitk_reduce_kernel combines them, in slice order, with the epilogue
struct Partials {
  float* ws;
  long slab;
  int ldp;
};
template <bool A_KC, bool B_KC>
static int launch_partials(const GemmP& p, int cfg, int ks, hipStream_t st, Partials* out) {
  const int ldp = (p.N + 3) & ~3;
  const long slab = (long)p.M * ldp;
  float* ws = splitk_workspace(sizeof(float) * (size_t)slab * ks, st);
  if (!ws) return TNET_ERR_RUNTIME;
  GemmP q = p;
  q.K = p.K / ks;
  q.ksplit = ks;
  q.kstepA = A_KC ? (long)q.K : (long)q.K * p.lda;
  q.kstepB = B_KC ? (long)q.K : (long)q.K * p.ldb;
  q.C = ws;
  q.ldc = ldp;
  q.slabC = slab;
  q.alpha = 1.f;
  q.beta = 0.f;
  bool ok = false;
  switch (cfg) {
#define X(name, KIND, BM, BN, BK, WM, WN, S, IL) \
  case CFG_##name: if (KIND == 1) ok = launch_cfg<KIND, BM, BN, BK, WM, WN, S, IL, A_KC, B_KC, EPI_STORE>(q, st); break;
    TNET_GEMM_CFGS(X)
#undef X
    default: break;
  }
  if (!ok) return TNET_ERR_UNSUPPORTED;
  TNET_LAUNCH_CHECK();
  *out = Partials{ws, slab, ldp};
  return TNET_OK;
}

template <bool A_KC, bool B_KC, int EPI>
static int launch_splitk(const GemmP& p, int cfg, int ks, hipStream_t st) {
  shadow_drop(p);  // the combine writes no transposed shadow
  Partials pt;
  const int rc = launch_partials<A_KC, B_KC>(p, cfg, ks, st, &pt);
  if (rc) return rc;
  float* ws = pt.ws;
  const long slab = pt.slab;
  const int ldp = pt.ldp;
  const long n = (long)p.M * ((p.N + 3) >> 2);
  const unsigned main_blocks = (unsigned)cdiv(n, 256);
  GemmP pc = p;  // the combine's output stores write-through where the byte offsets fit the descriptor
  pc.wt = g_wt && (long)p.M * p.ldc < (1L << 29) && (!p.corr || (long)p.M * p.ldcorr < (1L << 29));
  const unsigned bias_blocks = epi_bias_slabs(EPI) ? (unsigned)cdiv(p.N, 256) : 0u;
  splitk_reduce_kernel<EPI><<<main_blocks + bias_blocks, 256, 0, st>>>(pc, ws, slab, ks, ldp, main_blocks);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

// bwd GEMM + diff-sigmoid + column sums: 16x16 configs with 32-row wave tiles (= slabs); 64x128 where
// that gives ~one workgroup per CU, else 64x64 (MLP3's 1024 x 1024 over K = 135: 128 tiles of 64x128)
static int launch_colsum_bwd(const GemmP& p_in, hipStream_t st) {
  if (p_in.M <= 0 || p_in.N <= 0) return TNET_OK;
  int cfg = forced_cfg();
  const bool autocfg = cfg < 0;
  GemmP p = p_in;
  p.group = g_group > 0 ? g_group : 8;
  if (cfg != CFG_m64x128k64s2 && cfg != CFG_m64x64k32s4 && cfg != CFG_m64x64k64s2)
    cfg = (long)cdiv(p.M, 64) * cdiv(p.N, 128) >= 200 ? CFG_m64x128k64s2 : CFG_m64x64k32s4;
  if (cfg == CFG_m64x128k64s2 && launch_sk<64, 128, true, true, EPI_DSIG_CS>(p, st)) {
    TNET_LAUNCH_CHECK();
    return TNET_OK;
  }
  bool ok = false;
  if (cfg == CFG_m64x128k64s2 && autocfg && g_kc >= 2)
    ok = launch_cfg<1, 64, 128, 64, 2, 2, 2, 8, true, true, EPI_DSIG_CS>(p, st);  // (the ring where it must)
  else if (cfg == CFG_m64x128k64s2) ok = launch_cfg<1, 64, 128, 64, 2, 2, 2, 0, true, true, EPI_DSIG_CS>(p, st);
  else if (cfg == CFG_m64x64k64s2) ok = launch_cfg<1, 64, 64, 64, 2, 2, 2, 0, true, true, EPI_DSIG_CS>(p, st);
  else ok = launch_cfg<1, 64, 64, 32, 2, 2, 4, 0, true, true, EPI_DSIG_CS>(p, st);
  if (!ok) return TNET_ERR_UNSUPPORTED;
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

// The same backward from the weight's transposed shadow Wt (B n-contiguous, the forward's NN layout): the 64x128
// grid in the forward's direct form (m64x128a8) where it gives ~one workgroup per CU, else 64x64 tiles (32-row
// wave tiles = slabs either way).  Per output element the MFMA operands and their order are the NT kernel's
// (the lane -> k map is layout-independent): Eo is bit-identical to launch_colsum_bwd's; the slab sums add the
// same rows in another order.  Not while CUs are reserved for RCCL (the caller takes the NT stream-K form).
static int launch_colsum_bwd_t(const GemmP& p_in, hipStream_t st) {
  if (p_in.M <= 0 || p_in.N <= 0) return TNET_OK;
  if (g_reserve > 0 || forced_cfg() >= 0) return TNET_ERR_UNSUPPORTED;
  GemmP p = p_in;
  p.group = g_group > 0 ? g_group : 8;
  bool ok;
  if ((long)cdiv(p.M, 64) * cdiv(p.N, 128) >= 200)
    ok = g_direct > 0 ? launch_cfg<1, 64, 128, 64, 2, 2, 2, 6, true, false, EPI_DSIG_CS>(p, st)
                      : launch_cfg<1, 64, 128, 64, 2, 2, 2, 0, true, false, EPI_DSIG_CS>(p, st);
  else
    ok = launch_cfg<1, 64, 64, 32, 2, 2, 4, 0, true, false, EPI_DSIG_CS>(p, st);
  if (!ok) return TNET_ERR_UNSUPPORTED;
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

// the configuration and split-K count of a GEMM: the forced ones (TNET_GEMM_CFG / _SPLITK,
// tnet_gemm_config) or the measured per-shape choice
struct GemmPlan {
  int cfg, ks;
};
template <bool A_KC>
static GemmPlan plan_gemm(const GemmP& p, bool splittable) {
  int cfg = forced_cfg();
  if (cfg < 0) {
    // measured per-shape choice (tools/gemm_sweep.py on MI355X, round 1): the largest tile that
    // still gives ~one workgroup per CU (256 CUs), the 16x16x4 kernel where the layout allows
    const long t128 = (long)cdiv(p.M, 128) * cdiv(p.N, 128), t64x128 = (long)cdiv(p.M, 64) * cdiv(p.N, 128);
    const long t128x256 = (long)cdiv(p.M, 128) * cdiv(p.N, 256);
    // round 2 (tools/gemm_sweep.py): 16x64 wave tiles (w41) for 64x64 tiles in every layout (the
    // 440-row update 24.4 -> 23.4 us), 32x64 tiles where 64x64 leaves most CUs idle (RBM phases,
    // 256 x 2048 over K = 440: 11.8 -> 9.7 us); fewer tiles than that: split-K below
    const long t64 = (long)cdiv(p.M, 64) * cdiv(p.N, 64), t32x64 = (long)cdiv(p.M, 32) * cdiv(p.N, 64);
    if (!A_KC && t128x256 >= 240) cfg = CFG_m128x256k32s3;  // one round where 128x128 needs two
    else if (t128 >= 240) cfg = CFG_m128x128k64s2;
    else if (A_KC && t64x128 >= 200) cfg = CFG_m64x128k64s2;  // incl. the K = 440 first layer (one round)
    else if (t64 >= 200) cfg = CFG_m64x64k32s4w41;
    // 32x64 tiles only in the K-contiguous A layout: over the update's [K][M] A they ran 35.5 us where
    // 64x64 ran 22.4 (MLP3's 598 x 1024 update over K = 1024, round 2)
    else if (A_KC && t32x64 >= 128) cfg = CFG_m32x64k64s2;
    else cfg = CFG_m64x64k32s4w41;
  }
  int ks = 1;
  if (splittable) {
    // split-K where few output tiles meet a long K (the RBM reconstruction 256 x 440 over K = 2048:
    // 28 tiles of 64x64 for 256 CUs)
    int tbm, tbn, kind;
    cfg_shape(cfg, &tbm, &tbn, &kind);
    const long tiles = (long)cdiv(p.M, tbm) * cdiv(p.N, tbn);
    if (g_split > 0) {
      ks = g_split < kMaxSplit ? g_split : kMaxSplit;
    } else if (tiles < 100 && p.K >= 1024) {
      while (ks < kMaxSplit && tiles * ks * 2 <= 288) ks *= 2;
      // 32x64 tiles need half the slices of 64x64 ones for the same workgroup count: less combine traffic
      const long t32 = (long)cdiv(p.M, 32) * cdiv(p.N, 64);
      if (cfg == CFG_m64x64k32s4w41 && ks >= 4 && t32 * (ks / 2) <= 288) {
        cfg = CFG_m32x64k64s2;
        kind = 1;
        ks /= 2;
      }
    }
    while (ks > 1 && (p.K % (4 * ks) != 0 || p.K / ks < 64)) ks /= 2;
    if (ks > 1 && kind != 1) cfg = CFG_m64x64k32s4w41;  // slices: 16x16 kernel only
  }
  return GemmPlan{cfg, ks};
}

template <bool A_KC, bool B_KC, int EPI>
static int launch_gemm(const GemmP& p_in, hipStream_t st) {
  if constexpr (EPI == EPI_DSIG_CS) {
    if constexpr (B_KC) return launch_colsum_bwd(p_in, st);
    else return launch_colsum_bwd_t(p_in, st);
  } else {
  if (p_in.M <= 0 || p_in.N <= 0) return TNET_OK;
  static const int noload = getenv("TNET_GEMM_DIAG") ? atoi(getenv("TNET_GEMM_DIAG")) : 0;
  GemmP p = p_in;
  p.diag_noload = noload;
  p.group = g_group > 0 ? g_group : 8;
  if (launch_split2<A_KC, B_KC, EPI>(p, st)) {
    TNET_LAUNCH_CHECK();
    return TNET_OK;
  }
  const GemmPlan pl = plan_gemm<A_KC>(p, epi_splittable(EPI));
  const int cfg = pl.cfg;
  if (pl.ks > 1) return launch_splitk<A_KC, B_KC, EPI>(p, cfg, pl.ks, st);
  bool sk_done = false;
  if (cfg == CFG_m64x128k64s2) sk_done = launch_sk<64, 128, A_KC, B_KC, EPI>(p, st);
  else if (cfg == CFG_m128x128k64s2) sk_done = launch_sk<128, 128, A_KC, B_KC, EPI>(p, st);
  if (sk_done) {
    TNET_LAUNCH_CHECK();
    return TNET_OK;
  }
  int rcfg = cfg;
  if (g_direct > 0 && forced_cfg() < 0 && !B_KC) {
    // (short K -- the first layer's 440: the 4-chunk ring's shorter prologue, 19.6 vs 20.9 us, tools/gemm_sweep.py r5o)
    if (cfg == CFG_m64x128k64s2)
      rcfg = (g_direct == 3 || p.K <= 512) ? CFG_m64x128a4 : CFG_m64x128a8;
    else if (cfg == CFG_m128x128k64s2) rcfg = CFG_m128x128a4;
    else if (cfg == CFG_m128x256k32s3 && g_direct == 4) rcfg = CFG_m128x256a2;  // 4: 1 + the 128x256 update
  }
  if (g_kc >= 2 && forced_cfg() < 0 && A_KC && B_KC && cfg == CFG_m64x128k64s2) rcfg = CFG_m64x128c8;
  if constexpr (!A_KC && !B_KC && (EPI == EPI_SGD_B || EPI == EPI_SGD))
    if (forced_cfg() < 0 && cfg == CFG_m64x64k32s4w41 && upd64_direct(p)) rcfg = CFG_m64x64a4;
  bool ok = false;
  switch (rcfg) {
#define X(name, KIND, BM, BN, BK, WM, WN, S, IL) \
  case CFG_##name: ok = launch_cfg<KIND, BM, BN, BK, WM, WN, S, IL, A_KC, B_KC, EPI>(p, st); break;
    TNET_GEMM_CFGS(X)
#undef X
    default: return TNET_ERR_ARG;
  }
  if (!ok) launch_cfg<0, 64, 64, 32, 2, 2, 4, 0, A_KC, B_KC, EPI>(p, st);  // layout not supported by cfg
  TNET_LAUNCH_CHECK();
  return TNET_OK;
  }
}

// tnet_affine_update_bwd_pair: the update GEMM (A: fused SGD + bias SGD, the 128x128 configuration the
// planner gives it) and an independent backward GEMM (B: diff-sigmoid + slab sums, 64x128) as one
// gemm16_pair_kernel launch; TNET_ERR_UNSUPPORTED where either would run another configuration (the
// caller then makes the two calls)
template <int EPIA, bool PXA, int SPA>
static void pair_go(const GemmP& pu, const GemmP& pb, int na, int nb, bool kc, int bt, hipStream_t st) {
  // bt: the backward half reads the weight's transposed shadow (NN; 1: the direct form m64x128a8, 2: the ring)
  if (bt == 1)
    gemm16_pair_kernel<128, 128, false, false, EPIA, PXA, 64, 128, true, false, EPI_DSIG_CS, true, SPA, 6>
        <<<na + nb, 256, 0, st>>>(pu, pb, na);
  else if (bt == 2)
    gemm16_pair_kernel<128, 128, false, false, EPIA, PXA, 64, 128, true, false, EPI_DSIG_CS, true, SPA, 0>
        <<<na + nb, 256, 0, st>>>(pu, pb, na);
  else if (kc)
    gemm16_pair_kernel<128, 128, false, false, EPIA, PXA, 64, 128, true, true, EPI_DSIG_CS, true, SPA, 8>
        <<<na + nb, 256, 0, st>>>(pu, pb, na);
  else
    gemm16_pair_kernel<128, 128, false, false, EPIA, PXA, 64, 128, true, true, EPI_DSIG_CS, true, SPA>
        <<<na + nb, 256, 0, st>>>(pu, pb, na);
}

// The top layer's update (128x256 tiles, the m128x256a2 direct form tnet_affine_update_bias runs for it) with the
// backward of the layer below from its transposed shadow (64x128 NN, m64x128a8) as ONE launch: the backward's
// workgroups start on the CUs the update's tiles leave instead of after a kernel boundary (TNET_PAIR_WIDE=0: the
// two launches).  Only where both run those direct forms alone; otherwise TNET_ERR_UNSUPPORTED.
static int launch_pair_wide_bwd_t(GemmP pu, GemmP pb, hipStream_t st) {
  static const bool on = !(getenv("TNET_PAIR_WIDE") && getenv("TNET_PAIR_WIDE")[0] == '0');
  if (!on || g_direct != 4 || g_reserve > 0) return TNET_ERR_UNSUPPORTED;
  if ((long)cdiv(pb.M, 64) * cdiv(pb.N, 128) < 200) return TNET_ERR_UNSUPPORTED;  // launch_colsum_bwd_t's 64x128 rule
  auto a16p = [](const void* v) { return ((uintptr_t)v & 15) == 0; };
  // A: launch_cfg's direct-form conditions for m128x256a2 (BK 32) and its 32-bit tile offsets
  const bool dir_a = pu.K / 32 >= 1 && pu.M % 4 == 0 && pu.N % 4 == 0 && !(pu.lda & 3) && !(pu.ldb & 3) &&
                     a16p(pu.A) && a16p(pu.B) && 4 * ((long)pu.K * pu.lda) < (1L << 31) &&
                     4 * ((long)pu.K * pu.ldb) < (1L << 31) && 4 * (32L * pu.lda + pu.M) < (1L << 32) &&
                     4 * (32L * pu.ldb + pu.N) < (1L << 32);
  // B: the NN backward's direct form (launch_colsum_bwd_t's m64x128a8: an even count of whole 64-k tiles)
  const bool dir_b = pb.K / 64 >= 1 && (pb.K / 64) % 2 == 0 && pb.N % 4 == 0 && !(pb.lda & 3) && !(pb.ldb & 3) &&
                     a16p(pb.A) && a16p(pb.B) && 4 * ((long)pb.M * pb.lda) < (1L << 31) &&
                     4 * ((long)pb.K * pb.ldb) < (1L << 31) && 4 * (64L * pb.ldb + pb.N) < (1L << 32);
  if (!dir_a || !dir_b || !px_exact<64, 128, EPI_DSIG_CS>(pb)) return TNET_ERR_UNSUPPORTED;
  pu.group = pb.group = g_group > 0 ? g_group : 8;
  pu.early_issue = pb.early_issue = g_early;
  pu.wt = pb.wt = g_wt;
  const int na = cdiv(pu.M, 128) * cdiv(pu.N, 256), nb = cdiv(pb.M, 64) * cdiv(pb.N, 128);
  gemm16_pair_kernel<128, 256, false, false, EPI_SGD_B, false, 64, 128, true, false, EPI_DSIG_CS, true, 7, 6, 32, 3>
      <<<na + nb, 256, 0, st>>>(pu, pb, na);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

template <int EPIA>
static int launch_pair_a_bwd(GemmP pu, GemmP pb, hipStream_t st, bool bwd_t = false) {
  // EPI_STORE_BG (the data-parallel gradient): not while CUs are reserved for RCCL (the exchange window runs the
  // stream-K forms; a 512-workgroup pair would lose a second round on the held CUs)
  if (EPIA == EPI_STORE_BG && g_reserve > 0) return TNET_ERR_UNSUPPORTED;
  if (forced_cfg() >= 0 || !g_pair) return TNET_ERR_UNSUPPORTED;
  if (pu.M <= 0 || pu.N <= 0 || pb.M <= 0 || pb.N <= 0) return TNET_ERR_UNSUPPORTED;
  const GemmPlan pl = plan_gemm<false>(pu, true);
  if (EPIA == EPI_SGD_B && bwd_t && pl.cfg == CFG_m128x256k32s3 && pl.ks == 1)
    return launch_pair_wide_bwd_t(pu, pb, st);
  if (pl.cfg != CFG_m128x128k64s2 || pl.ks != 1) return TNET_ERR_UNSUPPORTED;
  if ((long)cdiv(pb.M, 64) * cdiv(pb.N, 128) < 200) return TNET_ERR_UNSUPPORTED;  // launch_colsum_bwd's 64x128 rule
  pu.group = pb.group = g_group > 0 ? g_group : 8;
  pu.early_issue = pb.early_issue = g_early;
  pu.wt = pb.wt = g_wt;
  // the 16x16 kernel's 32-bit tile offsets (launch_cfg's check)
  const long extA_u = 64L * pu.lda + pu.M, extB_u = 64L * pu.ldb + pu.N;
  const long extA_b = (long)pb.M * pb.lda, extB_b = bwd_t ? 64L * pb.ldb + pb.N : (long)pb.N * pb.ldb;
  if (4 * extA_u >= (1L << 32) || 4 * extB_u >= (1L << 32) || 4 * extA_b >= (1L << 32) || 4 * extB_b >= (1L << 32))
    return TNET_ERR_UNSUPPORTED;
  if (!px_exact<64, 128, EPI_DSIG_CS>(pb)) return TNET_ERR_UNSUPPORTED;
  const int na = cdiv(pu.M, 128) * cdiv(pu.N, 128), nb = cdiv(pb.M, 64) * cdiv(pb.N, 128);
  // the update half in the direct form (launch_cfg's direct-form conditions)
  auto a16p = [](const void* v) { return ((uintptr_t)v & 15) == 0; };
  const bool dir = g_direct > 0 && pu.K / 64 >= 1 && !(pu.lda & 3) && !(pu.ldb & 3) && a16p(pu.A) && a16p(pu.B) &&
                   pu.M % 4 == 0 && pu.N % 4 == 0 &&
                   4 * ((long)pu.K * pu.lda) < (1L << 31) && 4 * ((long)pu.K * pu.ldb) < (1L << 31);
  const bool px = px_exact<128, 128, EPIA>(pu);
  const bool kc = !bwd_t && g_kc >= 2 && kc_direct(pb);  // the backward half in the coalesced k-contiguous direct form
  int bt = 0;
  if (bwd_t) {
    // the NN backward half (from the transposed shadow) in the direct form where launch_cfg would run it so
    const bool dir_b = g_direct > 0 && pb.K / 64 >= 1 && (pb.K / 64) % 2 == 0 && pb.N % 4 == 0 && !(pb.lda & 3) &&
                       !(pb.ldb & 3) && a16p(pb.A) && a16p(pb.B) && 4 * ((long)pb.M * pb.lda) < (1L << 31) &&
                       4 * ((long)pb.K * pb.ldb) < (1L << 31);
    bt = dir_b ? 1 : 2;
  }
  if (dir && px) pair_go<EPIA, true, 5>(pu, pb, na, nb, kc, bt, st);
  else if (dir) pair_go<EPIA, false, 5>(pu, pb, na, nb, kc, bt, st);
  else if (px) pair_go<EPIA, true, 0>(pu, pb, na, nb, kc, bt, st);
  else pair_go<EPIA, false, 0>(pu, pb, na, nb, kc, bt, st);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

static int launch_pair_upd_bwd(GemmP pu, GemmP pb, hipStream_t st) { return launch_pair_a_bwd<EPI_SGD_B>(pu, pb, st); }

static int cu_count() {
  if (!g_cus) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
    g_cus = prop.multiProcessorCount;
  }
  return g_cus;
}
static bool split2_on() {
  if (g_split2 < 0) g_split2 = getenv("TNET_GEMM_SPLIT2") ? atoi(getenv("TNET_GEMM_SPLIT2")) : 0;
  return g_split2 != 0;
}

// tnet_affine_update_bias_pair: both updates in one gemm16_upd_pair_kernel launch when their 64x64 grids
// together fit one round over the CUs; TNET_ERR_UNSUPPORTED otherwise (the caller makes the two calls)
static int launch_upd_pair(GemmP pa, GemmP pb, hipStream_t st) {
  if (forced_cfg() >= 0 || !g_pair) return TNET_ERR_UNSUPPORTED;
  if (pa.M <= 0 || pa.N <= 0 || pb.M <= 0 || pb.N <= 0) return TNET_ERR_UNSUPPORTED;
  if (!g_cus) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
      return TNET_ERR_UNSUPPORTED;
    g_cus = prop.multiProcessorCount;
  }
  const int na = cdiv(pa.M, 64) * cdiv(pa.N, 64), nb = cdiv(pb.M, 64) * cdiv(pb.N, 64);
  if (na + nb > g_cus - g_reserve) return TNET_ERR_UNSUPPORTED;
  // the 16x16 kernel's 32-bit k-tile offsets (launch_cfg's check, BK 32, m- / n-contiguous operands)
  for (const GemmP* q : {&pa, &pb})
    if (4 * (32L * q->lda + q->M) >= (1L << 32) || 4 * (32L * q->ldb + q->N) >= (1L << 32)) return TNET_ERR_UNSUPPORTED;
  pa.group = pb.group = g_group > 0 ? g_group : 8;
  pa.early_issue = pb.early_issue = g_early;
  pa.wt = pb.wt = g_wt;
  gemm16_upd_pair_kernel<64, 64, 32, 4, 1, 4><<<na + nb, 256, 0, st>>>(pa, pb, na);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

static bool aligned16(const void* q) { return ((uintptr_t)q & 15) == 0; }

static int check_common(const GemmP& p) {
  if (p.M < 0 || p.N < 0 || p.K < 0) return TNET_ERR_ARG;
  if ((p.lda & 3) || (p.ldb & 3) || (p.ldc & 3)) return TNET_ERR_ARG;
  if (!aligned16(p.A) || !aligned16(p.B) || !aligned16(p.C)) return TNET_ERR_ARG;
  return TNET_OK;
}

}  // namespace tnetk

using namespace tnetk;

extern "C" int tnet_sgemm(char transa, char transb, int m, int n, int k, float alpha, const float* A, int lda,
                          const float* B, int ldb, float beta, float* C, int ldc, void* stream) {
  GemmP p{};
  p.M = m; p.N = n; p.K = k;
  p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.C = C; p.ldc = ldc;
  p.alpha = alpha; p.beta = beta;
  int st = check_common(p);
  if (st) return st;
  const bool ta = (transa == 'T' || transa == 't'), tb = (transb == 'T' || transb == 't');
  hipStream_t s = (hipStream_t)stream;
  if (k == 0) {  // C = beta*C
    if (beta == 1.f) return TNET_OK;
    TnetMatrixDim d{m, n, ldc};
    return tnetF_add_scaled(0.f, C, ldc, beta, C, d, stream);
  }
  if (!ta && !tb) return launch_gemm<true, false, EPI_STORE>(p, s);
  if (!ta && tb) return launch_gemm<true, true, EPI_STORE>(p, s);
  if (ta && !tb) return launch_gemm<false, false, EPI_STORE>(p, s);
  return launch_gemm<false, true, EPI_STORE>(p, s);
}

extern "C" int tnet_affine_fwd(const float* X, TnetMatrixDim dX, const float* W, TnetMatrixDim dW, const float* b,
                               float* Y, TnetMatrixDim dY, int act, void* stream) {
  if (dX.cols != dW.rows || dY.rows != dX.rows || dY.cols != dW.cols || !b || act < 0 || act > 3) return TNET_ERR_ARG;
  GemmP p{};
  p.M = dX.rows; p.N = dW.cols; p.K = dX.cols;
  p.A = X; p.lda = dX.stride; p.B = W; p.ldb = dW.stride; p.C = Y; p.ldc = dY.stride;
  p.bias = b;
  int st = check_common(p);
  if (st) return st;
  if (act == 0 && top_split_ok(p)) {  // the same slices as tnet_affine_softmax_xent, combined by splitk_reduce_kernel
    int ldp = 0;
    if (float* ws = top_split_partials(p, (hipStream_t)stream, &ldp)) {
      const unsigned g = (unsigned)cdiv((long)p.M * ((p.N + 3) / 4), 256);
      splitk_reduce_kernel<EPI_BIAS><<<g, 256, 0, (hipStream_t)stream>>>(p, ws, (long)p.M * ldp, kTopSlices, ldp, g);
      TNET_LAUNCH_CHECK();
      return TNET_OK;
    }
  }
  switch (act) {
    case 1: return launch_gemm<true, false, EPI_BIAS_SIG>(p, (hipStream_t)stream);
    case 2: return launch_gemm<true, false, EPI_BIAS_NEG>(p, (hipStream_t)stream);
    case 3: return launch_gemm<true, false, EPI_BIAS_NSIG>(p, (hipStream_t)stream);
    default: return launch_gemm<true, false, EPI_BIAS>(p, (hipStream_t)stream);
  }
}

extern "C" int tnet_affine_fwd_sample(const float* X, TnetMatrixDim dX, const float* W, TnetMatrixDim dW,
                                      const float* b, float* Y, TnetMatrixDim dY, float* states, int ld_states,
                                      unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4, void* stream) {
  // Y = sigmoid(X W + b), states = (Y > U) with U the HybridTaus draws of states z1..z4 (indexed with Y's
  // stride) -- tnet_affine_fwd(act 1) + tnet_rand_binarize in one launch
  if (dX.cols != dW.rows || dY.rows != dX.rows || dY.cols != dW.cols || !b || !states || ld_states < dY.cols ||
      !z1 || !z2 || !z3 || !z4)
    return TNET_ERR_ARG;
  GemmP p{};
  p.M = dX.rows; p.N = dW.cols; p.K = dX.cols;
  p.A = X; p.lda = dX.stride; p.B = W; p.ldb = dW.stride; p.C = Y; p.ldc = dY.stride;
  p.bias = b;
  p.bin = states; p.ldbin = ld_states;
  p.rz[0] = z1; p.rz[1] = z2; p.rz[2] = z3; p.rz[3] = z4;
  int st = check_common(p);
  if (st) return st;
  return launch_gemm<true, false, EPI_BIAS_SIG_BIN>(p, (hipStream_t)stream);
}

extern "C" int tnet_affine_fwd_t(const float* X, TnetMatrixDim dX, const float* W, TnetMatrixDim dW, const float* b,
                                 float* Y, TnetMatrixDim dY, int act, void* stream) {
  // Y[rows x n_in] = act(X[rows x n_out] W^T + b) with W stored [n_in x n_out] (CuRbm::Reconstruct)
  if (dX.cols != dW.cols || dY.rows != dX.rows || dY.cols != dW.rows || !b || act < 0 || act > 1) return TNET_ERR_ARG;
  GemmP p{};
  p.M = dX.rows; p.N = dW.rows; p.K = dX.cols;
  p.A = X; p.lda = dX.stride; p.B = W; p.ldb = dW.stride; p.C = Y; p.ldc = dY.stride;
  p.bias = b;
  int st = check_common(p);
  if (st) return st;
  if (act == 1) return launch_gemm<true, true, EPI_BIAS_SIG>(p, (hipStream_t)stream);
  return launch_gemm<true, true, EPI_BIAS>(p, (hipStream_t)stream);
}

extern "C" int tnet_affine_softmax_xent(const float* X, TnetMatrixDim dX, const float* W, TnetMatrixDim dW,
                                        const float* b, const int* labels, float* Z, int strideZ, float* Y,
                                        int strideY, float* E, int strideE, double* stats, float* colpart,
                                        int ldcolpart, void* stream) {
  // the top <biasedlinearity> + <softmax> + cross-entropy for n_out <= 256: Z = X W + b (nullable),
  // Y = softmax(Z) (nullable), E = Y - onehot(labels), stats, and (colpart non-null) E's 32-row slab
  // column sums -- tnet_affine_fwd(act 0) + tnet_softmax_xent + tnet_colsum_slab_sums in two launches
  if (dX.cols != dW.rows || !b || !labels || !E || dX.rows < 0 || strideE < dW.cols || (Z && strideZ < dW.cols) ||
      (Y && strideY < dW.cols) || (colpart && ldcolpart < dW.cols))
    return TNET_ERR_ARG;
  if (dW.cols > kSxMaxN) return TNET_ERR_UNSUPPORTED;
  if (dX.rows == 0 || dW.cols == 0) return TNET_OK;
  GemmP p{};
  p.M = dX.rows; p.N = dW.cols; p.K = dX.cols;
  p.A = X; p.lda = dX.stride; p.B = W; p.ldb = dW.stride;  // C: the slices' workspace
  p.bias = b;
  int st = check_common(p);
  if (st) return st;
  hipStream_t s = (hipStream_t)stream;
  // softmax_xent_kernel's lane-to-column map: the 16-byte one where its launch would use it
  const int v4 = (p.N & 3) == 0 && (!Z || (aligned16(Z) && (strideZ & 3) == 0)) &&
                 (!Y || (aligned16(Y) && (strideY & 3) == 0)) && aligned16(E) && (strideE & 3) == 0;
  if (top_split_ok(p)) {  // the row-block kernel's 4 K slices, then this kernel's combine + softmax launch
    int ldp = 0;
    if (float* ws = top_split_partials(p, s, &ldp)) {
      affine_softmax_xent_kernel<<<(unsigned)cdiv(p.M, kColsumSlabRows), kSxThreads, 0, s>>>(
          p, ws, (long)p.M * ldp, kTopSlices, ldp, labels, Z, strideZ, Y, strideY, E, strideE, stats, colpart,
          ldcolpart, v4);
      TNET_LAUNCH_CHECK();
      return TNET_OK;
    }
  }
  const GemmPlan pl = plan_gemm<true>(p, true);
  int cfg = pl.cfg, bm, bn, kind;
  cfg_shape(cfg, &bm, &bn, &kind);
  if (kind != 1) cfg = CFG_m64x64k32s4w41;  // slices: 16x16 kernel only
  p.group = g_group > 0 ? g_group : 8;
  Partials pt;
  st = launch_partials<true, false>(p, cfg, pl.ks, s, &pt);
  if (st) return st;
  affine_softmax_xent_kernel<<<(unsigned)cdiv(p.M, kColsumSlabRows), kSxThreads, 0, s>>>(
      p, pt.ws, pt.slab, pl.ks, pt.ldp, labels, Z, strideZ, Y, strideY, E, strideE, stats, colpart, ldcolpart, v4);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_rbm_update(const float* V, TnetMatrixDim dV, const float* H, TnetMatrixDim dH, float* W,
                               TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                               void* stream) {
  // corr = mmt*corr + scale*(V^T H) + l2*W ; W += corr, with V / H the row-stacked positive and
  // (sign-flipped) negative phase statistics
  if (dV.rows != dH.rows || dW.rows != dV.cols || dW.cols != dH.cols || !corrW || (strideCorr & 3))
    return TNET_ERR_ARG;
  GemmP p{};
  p.M = dV.cols; p.N = dH.cols; p.K = dV.rows;
  p.A = V; p.lda = dV.stride; p.B = H; p.ldb = dH.stride; p.C = W; p.ldc = dW.stride;
  p.corr = corrW; p.ldcorr = strideCorr;
  p.scale = scale; p.mmt = mmt; p.l2 = l2;
  int st = check_common(p);
  if (st) return st;
  return launch_gemm<false, false, EPI_RBM>(p, (hipStream_t)stream);
}

static int rbm_update_stats_run(const float* V, TnetMatrixDim dV, const float* H, TnetMatrixDim dH, float* W,
                                TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2, int B,
                                float* vb, float* cvb, float* hb, float* chb, double* mse_stats, const BunchGatherP& g,
                                int ng, void* stream);

// byte ranges one launch touches: a gather riding on an update launch must be independent of it -- nothing
// the gather writes (y, labels_out) may be read or written by the update, nothing the update writes may be
// read by the gather (x, labels_in, copy_from) -- or the combined launch is a race the separate calls are not
struct ByteSpan {
  const void* p;
  size_t n;
};
static ByteSpan span_of(const void* p, long rows, long stride, size_t elem) {
  return ByteSpan{p, p && rows > 0 && stride > 0 ? (size_t)rows * (size_t)stride * elem : 0};
}
static bool spans_overlap(ByteSpan a, ByteSpan b) {
  if (!a.p || !b.p || !a.n || !b.n) return false;
  const char *a0 = (const char*)a.p, *b0 = (const char*)b.p;
  return a0 < b0 + b.n && b0 < a0 + a.n;
}
static bool any_overlap(std::initializer_list<ByteSpan> xs, std::initializer_list<ByteSpan> ys) {
  for (const ByteSpan& x : xs)
    for (const ByteSpan& y : ys)
      if (spans_overlap(x, y)) return true;
  return false;
}
// the gather's writes / reads (tnet_gather_bunch: y[dy.rows x dy.stride], labels_out[dy.rows] written;
// x[dx.rows x dx.stride], labels_in[dx.rows], copy_from[dy.rows] read)
static bool gather_independent(float* y, const float* x, int* labels_out, const int* labels_in, const int* copy_from,
                               TnetMatrixDim dy, TnetMatrixDim dx, std::initializer_list<ByteSpan> upd_reads,
                               std::initializer_list<ByteSpan> upd_writes) {
  const ByteSpan gw[] = {span_of(y, dy.rows, dy.stride, 4), span_of(labels_out, dy.rows, 1, 4)};
  const ByteSpan gr[] = {span_of(x, dx.rows, dx.stride, 4), span_of(labels_in, dx.rows, 1, 4),
                         span_of(copy_from, dy.rows, 1, 4)};
  for (const ByteSpan& w : gw) {
    if (any_overlap({w}, upd_reads) || any_overlap({w}, upd_writes)) return false;
    for (const ByteSpan& r : gr)
      if (spans_overlap(w, r)) return false;
  }
  for (const ByteSpan& r : gr)
    if (any_overlap({r}, upd_writes)) return false;
  return true;
}

extern "C" int tnet_rbm_update_stats(const float* V, TnetMatrixDim dV, const float* H, TnetMatrixDim dH, float* W,
                                     TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                                     int B, float* vb, float* cvb, float* hb, float* chb, double* mse_stats,
                                     void* stream) {
  return rbm_update_stats_run(V, dV, H, dH, W, dW, corrW, strideCorr, scale, mmt, l2, B, vb, cvb, hb, chb, mse_stats,
                              BunchGatherP{}, 0, stream);
}

extern "C" int tnet_rbm_update_stats_gather(const float* V, TnetMatrixDim dV, const float* H, TnetMatrixDim dH,
                                            float* W, TnetMatrixDim dW, float* corrW, int strideCorr, float scale,
                                            float mmt, float l2, int B, float* vb, float* cvb, float* hb, float* chb,
                                            double* mse_stats, float* y, const float* x, int* labels_out,
                                            const int* labels_in, const int* copy_from, TnetMatrixDim dy,
                                            TnetMatrixDim dx, void* stream) {
  // tnet_rbm_update_stats + tnet_gather_bunch (the next bunch's visible rows) in one launch
  if (!y || !x || !labels_out || !labels_in || !copy_from || dy.cols != dx.cols || dy.rows < 0 || dy.stride < dy.cols ||
      dx.stride < dx.cols)
    return TNET_ERR_ARG;
  const int c4 = (dy.cols + 3) & ~3;
  if (((uintptr_t)y & 15) || ((uintptr_t)x & 15) || (dy.stride & 3) || (dx.stride & 3) || c4 > dy.stride ||
      c4 > dx.stride)
    return TNET_ERR_UNSUPPORTED;
  // the gather independent of the update + statistics (they read V, H; write W, its momentum, both biases and
  // their momentum, the MSE slots)
  if (!gather_independent(y, x, labels_out, labels_in, copy_from, dy, dx,
                          {span_of(V, dV.rows, dV.stride, 4), span_of(H, dH.rows, dH.stride, 4)},
                          {span_of(W, dW.rows, dW.stride, 4), span_of(corrW, dW.rows, strideCorr, 4),
                           span_of(vb, dV.cols, 1, 4), span_of(cvb, dV.cols, 1, 4), span_of(hb, dH.cols, 1, 4),
                           span_of(chb, dH.cols, 1, 4), span_of(mse_stats, TNET_STATS_WORDS, 1, 8)}))
    return TNET_ERR_ARG;
  return rbm_update_stats_run(V, dV, H, dH, W, dW, corrW, strideCorr, scale, mmt, l2, B, vb, cvb, hb, chb, mse_stats,
                              BunchGatherP{y, x, labels_out, labels_in, copy_from, dy.rows, c4, dy.stride, dx.stride},
                              16, stream);
}

static int rbm_update_stats_run(const float* V, TnetMatrixDim dV, const float* H, TnetMatrixDim dH, float* W,
                                TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2, int B,
                                float* vb, float* cvb, float* hb, float* chb, double* mse_stats, const BunchGatherP& g,
                                int ng, void* stream) {
  // tnet_rbm_update(V, H, W, corrW, scale, mmt, l2) + tnet_rbm_stats_update(V, H, B, vb, cvb, hb, chb, scale, mmt,
  // mse_stats) as one launch where the update runs the 64x64 configuration unsplit (what it runs alone,
  // so the results are those of the two calls); TNET_ERR_UNSUPPORTED otherwise
  if (dV.rows != dH.rows || dW.rows != dV.cols || dW.cols != dH.cols || !corrW || (strideCorr & 3))
    return TNET_ERR_ARG;
  if (B < 0 || dV.rows != 2 * B || dV.cols <= 0 || dH.cols <= 0 || dV.stride < dV.cols || dH.stride < dH.cols || !vb ||
      !cvb || !hb || !chb)
    return TNET_ERR_ARG;
  if (!B || 2 * B > CS_ROWS * RS_MAX_SLABS || forced_cfg() >= 0 || !g_pair) return TNET_ERR_UNSUPPORTED;
  GemmP p{};
  p.M = dV.cols; p.N = dH.cols; p.K = dV.rows;
  p.A = V; p.lda = dV.stride; p.B = H; p.ldb = dH.stride; p.C = W; p.ldc = dW.stride;
  p.corr = corrW; p.ldcorr = strideCorr;
  p.scale = scale; p.mmt = mmt; p.l2 = l2;
  int st = check_common(p);
  if (st) return st;
  const GemmPlan pl = plan_gemm<false>(p, epi_splittable(EPI_RBM));
  if (pl.cfg != CFG_m64x64k32s4w41 || pl.ks != 1) return TNET_ERR_UNSUPPORTED;
  if (4 * (32L * p.lda + p.M) >= (1L << 32) || 4 * (32L * p.ldb + p.N) >= (1L << 32)) return TNET_ERR_UNSUPPORTED;
  p.group = g_group > 0 ? g_group : 8;
  p.early_issue = g_early;
  p.wt = g_wt;
  const int na = cdiv(p.M, 64) * cdiv(p.N, 64);
  const int nvb = cdiv(dV.cols, RS_COLS), nhb = cdiv(dH.cols, RS_COLS), nmb = mse_stats ? cdiv(B, RS_MROWS) : 0;
  if (ng && cu_count() - g_reserve - na < ng) return TNET_ERR_UNSUPPORTED;  // the gather's CUs beside the tiles
  gemm16_rbm_update_stats_kernel<<<na + ng + nvb + nhb + nmb, 256, 0, (hipStream_t)stream>>>(
      p, na, V, dV, H, dH, B, nvb, vb, cvb, hb, chb, scale, mmt, mse_stats, nhb, g, ng);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_affine_bwd(const float* E, TnetMatrixDim dE, const float* W, TnetMatrixDim dW,
                               const float* Ybelow, int strideYbelow, float* Eo, TnetMatrixDim dEo, int dsig,
                               void* stream) {
  // Eo[rows x n_in] = E[rows x n_out] * W^T, W stored [n_in x n_out] == B stored [N][K]
  if (dE.cols != dW.cols || dEo.rows != dE.rows || dEo.cols != dW.rows) return TNET_ERR_ARG;
  GemmP p{};
  p.M = dE.rows; p.N = dW.rows; p.K = dE.cols;
  p.A = E; p.lda = dE.stride; p.B = W; p.ldb = dW.stride; p.C = Eo; p.ldc = dEo.stride;
  p.alpha = 1.f; p.beta = 0.f;
  p.aux = Ybelow; p.ldaux = strideYbelow;
  int st = check_common(p);
  if (st) return st;
  if (dsig) {
    if (!Ybelow || !aligned16(Ybelow) || (strideYbelow & 3)) return TNET_ERR_ARG;
    return launch_gemm<true, true, EPI_DSIG>(p, (hipStream_t)stream);
  }
  return launch_gemm<true, true, EPI_STORE>(p, (hipStream_t)stream);
}

extern "C" int tnet_affine_update(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* W,
                                  TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt,
                                  float l2, void* stream) {
  // W[n_in x n_out] += scale * (X^T E + mmt*corr): A = X stored [K=rows][M=n_in], B = E [K][N]
  if (dX.rows != dE.rows || dW.rows != dX.cols || dW.cols != dE.cols) return TNET_ERR_ARG;
  GemmP p{};
  p.M = dX.cols; p.N = dE.cols; p.K = dX.rows;
  p.A = X; p.lda = dX.stride; p.B = E; p.ldb = dE.stride; p.C = W; p.ldc = dW.stride;
  p.corr = (mmt != 0.f || corrW) ? corrW : nullptr; p.ldcorr = strideCorr;
  if (mmt != 0.f && !corrW) return TNET_ERR_ARG;
  if (p.corr && (p.ldcorr & 3)) return TNET_ERR_ARG;
  p.scale = scale; p.mmt = mmt; p.l2 = l2;
  int st = check_common(p);
  if (st) return st;
  shadow_attach(p);
  return shadow_done(p, launch_gemm<false, false, EPI_SGD>(p, (hipStream_t)stream));
}

extern "C" int tnet_colsum_slabs(int rows) { return rows > 0 ? (rows + kColsumSlabRows - 1) / kColsumSlabRows : 0; }

extern "C" int tnet_affine_bwd_colsum(const float* E, TnetMatrixDim dE, const float* W, TnetMatrixDim dW,
                                      const float* Ybelow, int strideYbelow, float* Eo, TnetMatrixDim dEo,
                                      float* colpart, int ldcolpart, void* stream) {
  // tnet_affine_bwd with dsig, plus colpart[s][c] = sum of Eo[r][c] over the 32-row slab s (fp32, in row order)
  if (dE.cols != dW.cols || dEo.rows != dE.rows || dEo.cols != dW.rows || !Ybelow || !colpart ||
      ldcolpart < dEo.cols || !aligned16(Ybelow) || (strideYbelow & 3))
    return TNET_ERR_ARG;
  GemmP p{};
  p.M = dE.rows; p.N = dW.rows; p.K = dE.cols;
  p.A = E; p.lda = dE.stride; p.B = W; p.ldb = dW.stride; p.C = Eo; p.ldc = dEo.stride;
  p.alpha = 1.f; p.beta = 0.f;
  p.aux = Ybelow; p.ldaux = strideYbelow;
  p.cpart = colpart; p.ldcpart = ldcolpart;
  int st = check_common(p);
  if (st) return st;
  return launch_gemm<true, true, EPI_DSIG_CS>(p, (hipStream_t)stream);
}

static int bwd_colsum_slabs(const float* E, TnetMatrixDim dE, const float* W, TnetMatrixDim dW, const float* Ybelow,
                            int strideYbelow, float* Eo, TnetMatrixDim dEo, float* colpart, int ldcolpart,
                            float* colpartE, int ldcolpartE, void* stream, bool bt) {
  // tnet_affine_bwd_colsum(E, W, Ybelow, Eo, colpart) + tnet_colsum_slab_sums(E, colpartE) in one launch
  // (bt: W is the transposed shadow [n_out x n_in], the NN form)
  const int w_k = bt ? dW.rows : dW.cols, w_n = bt ? dW.cols : dW.rows;
  if (dE.cols != w_k || dEo.rows != dE.rows || dEo.cols != w_n || !Ybelow || !colpart ||
      ldcolpart < dEo.cols || !aligned16(Ybelow) || (strideYbelow & 3) || !colpartE || ldcolpartE < dE.cols)
    return TNET_ERR_ARG;
  GemmP p{};
  p.M = dE.rows; p.N = w_n; p.K = dE.cols;
  p.A = E; p.lda = dE.stride; p.B = W; p.ldb = dW.stride; p.C = Eo; p.ldc = dEo.stride;
  p.alpha = 1.f; p.beta = 0.f;
  p.aux = Ybelow; p.ldaux = strideYbelow;
  p.cpart = colpart; p.ldcpart = ldcolpart;
  int st = check_common(p);
  if (st) return st;
  // what launch_colsum_bwd runs alone: the plain 64x128 grid (no forced configuration, no stream-K)
  if (p.M <= 0 || p.N <= 0 || forced_cfg() >= 0 || g_reserve > 0) return TNET_ERR_UNSUPPORTED;
  if ((long)cdiv(p.M, 64) * cdiv(p.N, 128) < 200) return TNET_ERR_UNSUPPORTED;
  if (4L * p.M * p.lda >= (1L << 32) || 4L * (bt ? (long)p.K : (long)p.N) * p.ldb >= (1L << 32))
    return TNET_ERR_UNSUPPORTED;
  // tnet_colsum_slab_sums's 16-B form
  const int slabs = cs_slabs(dE.rows);
  if (slabs != cdiv(dE.rows, CS_ROWS) || (dE.cols & 3) || (dE.stride & 3) || !aligned16(E)) return TNET_ERR_UNSUPPORTED;
  p.group = g_group > 0 ? g_group : 8;
  p.early_issue = g_early;
  p.wt = g_wt;
  const int na = cdiv(p.M, 64) * cdiv(p.N, 128), ncb = cdiv(dE.cols, CS_COLS * 4);
  const unsigned grid = (unsigned)(na + ncb * slabs);
  if (bt) {
    // the forward's direct form (m64x128a8: whole k-tiles in an even count, 16-B aligned, 31-bit offsets; the
    // k tail through the DMA images) where the exact prefetch holds, else the ring
    const int nfull = p.K / 64;
    const bool dir = g_direct > 0 && nfull >= 1 && nfull % 2 == 0 && p.N % 4 == 0 && !(p.lda & 3) && !(p.ldb & 3) &&
                     aligned16(p.A) && aligned16(p.B) && 4L * p.M * p.lda < (1L << 31) &&
                     4L * p.K * p.ldb < (1L << 31);
    if (px_exact<64, 128, EPI_DSIG_CS>(p) && dir)
      gemm16_bwd_slabs_kernel<true, 6, false><<<grid, 256, 0, (hipStream_t)stream>>>(p, na, E, dE, colpartE, ldcolpartE, slabs, ncb);
    else if (px_exact<64, 128, EPI_DSIG_CS>(p))
      gemm16_bwd_slabs_kernel<true, 0, false><<<grid, 256, 0, (hipStream_t)stream>>>(p, na, E, dE, colpartE, ldcolpartE, slabs, ncb);
    else
      gemm16_bwd_slabs_kernel<false, 0, false><<<grid, 256, 0, (hipStream_t)stream>>>(p, na, E, dE, colpartE, ldcolpartE, slabs, ncb);
  } else if (px_exact<64, 128, EPI_DSIG_CS>(p) && kc_direct(p))
    gemm16_bwd_slabs_kernel<true, 8><<<grid, 256, 0, (hipStream_t)stream>>>(p, na, E, dE, colpartE, ldcolpartE, slabs, ncb);
  else if (px_exact<64, 128, EPI_DSIG_CS>(p))
    gemm16_bwd_slabs_kernel<true><<<grid, 256, 0, (hipStream_t)stream>>>(p, na, E, dE, colpartE, ldcolpartE, slabs, ncb);
  else
    gemm16_bwd_slabs_kernel<false><<<grid, 256, 0, (hipStream_t)stream>>>(p, na, E, dE, colpartE, ldcolpartE, slabs, ncb);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_affine_bwd_colsum_slabs(const float* E, TnetMatrixDim dE, const float* W, TnetMatrixDim dW,
                                            const float* Ybelow, int strideYbelow, float* Eo, TnetMatrixDim dEo,
                                            float* colpart, int ldcolpart, float* colpartE, int ldcolpartE,
                                            void* stream) {
  return bwd_colsum_slabs(E, dE, W, dW, Ybelow, strideYbelow, Eo, dEo, colpart, ldcolpart, colpartE, ldcolpartE,
                          stream, false);
}

extern "C" int tnet_affine_bwd_colsum_slabs_t(const float* E, TnetMatrixDim dE, const float* Wt, TnetMatrixDim dWt,
                                              const float* Ybelow, int strideYbelow, float* Eo, TnetMatrixDim dEo,
                                              float* colpart, int ldcolpart, float* colpartE, int ldcolpartE,
                                              void* stream) {
  return bwd_colsum_slabs(E, dE, Wt, dWt, Ybelow, strideYbelow, Eo, dEo, colpart, ldcolpart, colpartE, ldcolpartE,
                          stream, true);
}

extern "C" int tnet_affine_bwd_colsum_t(const float* E, TnetMatrixDim dE, const float* Wt, TnetMatrixDim dWt,
                                        const float* Ybelow, int strideYbelow, float* Eo, TnetMatrixDim dEo,
                                        float* colpart, int ldcolpart, void* stream) {
  // tnet_affine_bwd_colsum from the transposed shadow Wt [n_out x n_in]: Eo = (E Wt) .* y (1 - y), NN
  if (dE.cols != dWt.rows || dEo.rows != dE.rows || dEo.cols != dWt.cols || !Ybelow || !colpart ||
      ldcolpart < dEo.cols || !aligned16(Ybelow) || (strideYbelow & 3))
    return TNET_ERR_ARG;
  GemmP p{};
  p.M = dE.rows; p.N = dWt.cols; p.K = dE.cols;
  p.A = E; p.lda = dE.stride; p.B = Wt; p.ldb = dWt.stride; p.C = Eo; p.ldc = dEo.stride;
  p.alpha = 1.f; p.beta = 0.f;
  p.aux = Ybelow; p.ldaux = strideYbelow;
  p.cpart = colpart; p.ldcpart = ldcolpart;
  int st = check_common(p);
  if (st) return st;
  return launch_colsum_bwd_t(p, (hipStream_t)stream);
}

// ---- transposed weight shadows
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ A, TnetMatrixDim d,
                                                        float* __restrict__ T, long ldt) {
  __shared__ float tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int r = r0 + ty + 4 * k, c = c0 + tx;
    tile[ty + 4 * k][tx] = (r < (int)d.rows && c < (int)d.cols) ? A[(long)r * d.stride + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = c0 + ty + 4 * k, r = r0 + tx;
    if (c < (int)d.cols && r < (int)d.rows) T[(long)c * ldt + r] = tile[tx][ty + 4 * k];
  }
}

extern "C" int tnet_transpose(const float* A, TnetMatrixDim dA, float* T, int ldt, void* stream) {
  if (!A || !T || ldt < (int)dA.rows || dA.stride < dA.cols) return TNET_ERR_ARG;
  if (!dA.rows || !dA.cols) return TNET_OK;
  transpose_kernel<<<dim3(cdiv(dA.cols, 64), cdiv(dA.rows, 64)), 256, 0, (hipStream_t)stream>>>(A, dA, T, ldt);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_weight_shadow(const float* W, TnetMatrixDim dW, float* Wt, int ldwt) {
  if (!W) return TNET_ERR_ARG;
  std::lock_guard<std::mutex> g(g_shadow_mu);
  if (!Wt) {
    g_shadow.erase(W);
    return TNET_OK;
  }
  if (ldwt < (int)dW.rows || (ldwt & 3) || ((uintptr_t)Wt & 15)) return TNET_ERR_ARG;
  g_shadow[W] = WeightShadow{Wt, (long)ldwt, (int)dW.rows, (int)dW.cols, 0};
  return TNET_OK;
}

extern "C" int tnet_weight_shadow_kept(const float* W) {
  std::lock_guard<std::mutex> g(g_shadow_mu);
  auto it = g_shadow.find(W);
  return it == g_shadow.end() ? TNET_ERR_ARG : it->second.kept;
}

extern "C" int tnet_affine_update_bias(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* W,
                                       TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt,
                                       float l2, const float* colpart, int ldcolpart, float* b, float* corr_b,
                                       void* stream) {
  // tnet_affine_update + the bias SGD of tnet_bias_update(E, b, corr_b, scale, mmt), the column sum of E
  // taken from the slab sums tnet_affine_bwd_colsum wrote for E
  if (dX.rows != dE.rows || dW.rows != dX.cols || dW.cols != dE.cols || !colpart || !b || ldcolpart < dE.cols)
    return TNET_ERR_ARG;
  if (mmt != 0.f && (!corrW || !corr_b)) return TNET_ERR_ARG;
  GemmP p{};
  p.M = dX.cols; p.N = dE.cols; p.K = dX.rows;
  p.A = X; p.lda = dX.stride; p.B = E; p.ldb = dE.stride; p.C = W; p.ldc = dW.stride;
  p.corr = (mmt != 0.f || corrW) ? corrW : nullptr; p.ldcorr = strideCorr;
  if (p.corr && (p.ldcorr & 3)) return TNET_ERR_ARG;
  p.scale = scale; p.mmt = mmt; p.l2 = l2;
  p.bpart = colpart; p.ldbpart = ldcolpart; p.bslabs = tnet_colsum_slabs(dE.rows);
  p.bvec = b; p.bcorr = mmt != 0.f ? corr_b : nullptr; p.bscale = scale; p.bmmt = mmt;
  int st = check_common(p);
  if (st) return st;
  if (p.M <= 0 || p.N <= 0) return TNET_OK;
  shadow_attach(p);
  return shadow_done(p, launch_gemm<false, false, EPI_SGD_B>(p, (hipStream_t)stream));
}

// the GemmP of tnet_affine_update_bias's launch (TNET_ERR_ARG on bad arguments)
static int update_bias_params(GemmP& p, const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* W,
                              TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                              const float* colpart, int ldcolpart, float* b, float* corr_b) {
  if (dX.rows != dE.rows || dW.rows != dX.cols || dW.cols != dE.cols || !colpart || !b || ldcolpart < dE.cols)
    return TNET_ERR_ARG;
  if (mmt != 0.f && (!corrW || !corr_b)) return TNET_ERR_ARG;
  p = GemmP{};
  p.M = dX.cols; p.N = dE.cols; p.K = dX.rows;
  p.A = X; p.lda = dX.stride; p.B = E; p.ldb = dE.stride; p.C = W; p.ldc = dW.stride;
  p.corr = (mmt != 0.f || corrW) ? corrW : nullptr; p.ldcorr = strideCorr;
  if (p.corr && (p.ldcorr & 3)) return TNET_ERR_ARG;
  p.scale = scale; p.mmt = mmt; p.l2 = l2;
  p.bpart = colpart; p.ldbpart = ldcolpart; p.bslabs = tnet_colsum_slabs(dE.rows);
  p.bvec = b; p.bcorr = mmt != 0.f ? corr_b : nullptr; p.bscale = scale; p.bmmt = mmt;
  return check_common(p);
}

extern "C" int tnet_affine_update_bias_pair(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE,
                                           float* W, TnetMatrixDim dW, float* corrW, int strideCorr, float scale,
                                           float mmt, float l2, const float* colpart, int ldcolpart, float* b,
                                           float* corr_b, const float* X2, TnetMatrixDim dX2, const float* E2,
                                           TnetMatrixDim dE2, float* W2, TnetMatrixDim dW2, float* corrW2,
                                           int strideCorr2, float scale2, float mmt2, float l22,
                                           const float* colpart2, int ldcolpart2, float* b2, float* corr_b2,
                                           void* stream) {
  // two tnet_affine_update_bias calls in one launch; they must be independent (distinct W, b, momentum
  // buffers; neither reads what the other writes)
  GemmP pa, pb;
  int st = update_bias_params(pa, X, dX, E, dE, W, dW, corrW, strideCorr, scale, mmt, l2, colpart, ldcolpart, b,
                              corr_b);
  if (st) return st;
  st = update_bias_params(pb, X2, dX2, E2, dE2, W2, dW2, corrW2, strideCorr2, scale2, mmt2, l22, colpart2, ldcolpart2,
                          b2, corr_b2);
  if (st) return st;
  if (W == W2 || b == b2 || (corrW && corrW == corrW2)) return TNET_ERR_ARG;
  shadow_attach(pb);
  shadow_attach(pa);
  const int rc = launch_upd_pair(pa, pb, (hipStream_t)stream);
  shadow_done(pa, rc);
  return shadow_done(pb, rc);
}

// An update GEMM (TN, SGD epilogue) the planner gives 64x64 tiles runs in the 64x64 direct form where those tiles
// fill ~a round of the CUs (the first layer's 440x2048 over K = 1024, 224 tiles: 21.9 vs 24.3 us; MLP3's 598x1024,
// 160 tiles, is slower direct: 26.6 vs 23.5 -- tools/gemm_sweep.py, profiles/r05_gemm_sweep_small_k.txt) and the
// direct-form conditions hold (launch_cfg's; TNET_UPD64_DIRECT=0: never)
namespace tnetk {
static bool upd64_direct(const GemmP& p) {
  static const bool on = !(getenv("TNET_UPD64_DIRECT") && getenv("TNET_UPD64_DIRECT")[0] == '0');
  auto a16p = [](const void* v) { return ((uintptr_t)v & 15) == 0; };
  return on && g_direct > 0 && p.ksplit <= 1 && (long)cdiv(p.M, 64) * cdiv(p.N, 64) >= 200 && p.K / 64 >= 1 &&
         p.M % 4 == 0 && p.N % 4 == 0 && !(p.lda & 3) && !(p.ldb & 3) && a16p(p.A) && a16p(p.B) &&
         4 * ((long)p.K * p.lda) < (1L << 31) && 4 * ((long)p.K * p.ldb) < (1L << 31);
}

// gemm16_upd_mixed_gather_kernel's conditions (TNET_UPD_MIXED=0: never): A is what tnet_affine_update_bias runs as
// m128x128a4 with the exact prefetch (the planner's m128x128k64s2, unsplit, the direct-form conditions, PX), B what
// it runs as m64x64k32s4w41 unsplit; no CUs reserved
static bool upd_mixed_ok(const GemmP& pa, const GemmP& pb) {
  static const bool on = !(getenv("TNET_UPD_MIXED") && getenv("TNET_UPD_MIXED")[0] == '0');
  if (!on || !g_pair || g_reserve > 0 || g_direct <= 0 || forced_cfg() >= 0) return false;
  const GemmPlan la = plan_gemm<false>(pa, true), lb = plan_gemm<false>(pb, true);
  if (la.cfg != CFG_m128x128k64s2 || la.ks != 1 || lb.cfg != CFG_m64x64k32s4w41 || lb.ks != 1) return false;
  auto a16p = [](const void* v) { return ((uintptr_t)v & 15) == 0; };
  const bool dir = pa.K / 64 >= 1 && !(pa.lda & 3) && !(pa.ldb & 3) && a16p(pa.A) && a16p(pa.B) && pa.M % 4 == 0 &&
                   pa.N % 4 == 0 && 4 * ((long)pa.K * pa.lda) < (1L << 31) && 4 * ((long)pa.K * pa.ldb) < (1L << 31);
  if (!dir || !px_exact<128, 128, EPI_SGD_B>(pa)) return false;
  // the 16x16 kernel's 32-bit tile offsets (launch_cfg's checks)
  if (4 * (64L * pa.lda + pa.M) >= (1L << 32) || 4 * (64L * pa.ldb + pa.N) >= (1L << 32)) return false;
  if (4 * (32L * pb.lda + pb.M) >= (1L << 32) || 4 * (32L * pb.ldb + pb.N) >= (1L << 32)) return false;
  return true;
}
}  // namespace tnetk

extern "C" int tnet_affine_update_bias_gather(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE,
                                              float* W, TnetMatrixDim dW, float* corrW, int strideCorr, float scale,
                                              float mmt, float l2, const float* colpart, int ldcolpart, float* b,
                                              float* corr_b, const float* X2, TnetMatrixDim dX2, const float* E2,
                                              TnetMatrixDim dE2, float* W2, TnetMatrixDim dW2, float* corrW2,
                                              int strideCorr2, float scale2, float mmt2, float l22,
                                              const float* colpart2, int ldcolpart2, float* b2, float* corr_b2,
                                              float* y, const float* x, int* labels_out, const int* labels_in,
                                              const int* copy_from, TnetMatrixDim dy, TnetMatrixDim dx,
                                              void* stream) {
  // tnet_affine_update_bias (X2 NULL) or tnet_affine_update_bias_pair, and tnet_gather_bunch, in one launch
  GemmP pa, pb{};
  int st = update_bias_params(pa, X, dX, E, dE, W, dW, corrW, strideCorr, scale, mmt, l2, colpart, ldcolpart, b,
                              corr_b);
  if (st) return st;
  const bool two = X2 != nullptr;
  if (two) {
    st = update_bias_params(pb, X2, dX2, E2, dE2, W2, dW2, corrW2, strideCorr2, scale2, mmt2, l22, colpart2,
                            ldcolpart2, b2, corr_b2);
    if (st) return st;
    if (W == W2 || b == b2 || (corrW && corrW == corrW2)) return TNET_ERR_ARG;
  }
  if (!y || !x || !labels_out || !labels_in || !copy_from || dy.cols != dx.cols || dy.rows < 0 || dy.stride < dy.cols ||
      dx.stride < dx.cols)
    return TNET_ERR_ARG;
  // the gather independent of the update(s): they read X, E and the slab sums, read and write W, its momentum,
  // b and its momentum
  auto reads = [](const GemmP& q) {
    return std::array<ByteSpan, 3>{span_of(q.A, q.K, q.lda, 4), span_of(q.B, q.K, q.ldb, 4),
                                    span_of(q.bpart, q.bslabs, q.ldbpart, 4)};
  };
  auto writes = [](const GemmP& q) {
    return std::array<ByteSpan, 4>{span_of(q.C, q.M, q.ldc, 4), span_of(q.corr, q.M, q.ldcorr, 4),
                                   span_of(q.bvec, q.N, 1, 4), span_of(q.bcorr, q.N, 1, 4)};
  };
  // the registered transposed shadows (written in the same pass as W) are writes of this launch too
  shadow_attach(pa);  // every form below runs gemm16_body's epilogue: the shadows are kept
  if (two) shadow_attach(pb);
  const ByteSpan cta = span_of(pa.Ct, pa.N, pa.ldct, 4), ctb = span_of(two ? pb.Ct : nullptr, pb.N, pb.ldct, 4);
  const auto ra = reads(pa), rb = reads(pb);
  const auto wa = writes(pa), wb = writes(pb);
  if (!gather_independent(y, x, labels_out, labels_in, copy_from, dy, dx, {ra[0], ra[1], ra[2], rb[0], rb[1], rb[2]},
                          {wa[0], wa[1], wa[2], wa[3], wb[0], wb[1], wb[2], wb[3], cta, ctb}))
    return TNET_ERR_ARG;
  // a shadow may alias nothing else either update reads or writes (it is written while they run)
  if (any_overlap({cta, ctb}, {ra[0], ra[1], ra[2], rb[0], rb[1], rb[2], wa[0], wa[1], wa[2], wa[3], wb[0], wb[1],
                               wb[2], wb[3]}) ||
      spans_overlap(cta, ctb))
    return TNET_ERR_ARG;
  const int c4 = (dy.cols + 3) & ~3;
  if (((uintptr_t)y & 15) || ((uintptr_t)x & 15) || (dy.stride & 3) || (dx.stride & 3) || c4 > dy.stride ||
      c4 > dx.stride)
    return TNET_ERR_UNSUPPORTED;
  if (forced_cfg() >= 0 || split2_on() || g_split > 0) return TNET_ERR_UNSUPPORTED;
  if (pa.M <= 0 || pa.N <= 0 || (two && (pb.M <= 0 || pb.N <= 0))) return TNET_ERR_UNSUPPORTED;
  int na, nb = 0;
  if (two && upd_mixed_ok(pa, pb)) {
    // a 2048-wide layer's update (128x128 direct) + the first layer's (64x64) + the gather
    na = cdiv(pa.M, 128) * cdiv(pa.N, 128);
    nb = cdiv(pb.M, 64) * cdiv(pb.N, 64);
    const int cus = cu_count();
    if (cus <= 0) return TNET_ERR_UNSUPPORTED;
    const int spare = cus - nb;
    const int ng = spare < 8 ? 8 : spare > 64 ? 64 : spare;
    pa.group = pb.group = g_group > 0 ? g_group : 8;
    pa.early_issue = pb.early_issue = g_early;
    pa.wt = pb.wt = g_wt;
    BunchGatherP g{y, x, labels_out, labels_in, copy_from, dy.rows, c4, dy.stride, dx.stride};
    if (upd64_direct(pb)) gemm16_upd_mixed_gather_kernel<true><<<na + nb + ng, 256, 0, (hipStream_t)stream>>>(pa, pb, na, nb, g);
    else gemm16_upd_mixed_gather_kernel<false><<<na + nb + ng, 256, 0, (hipStream_t)stream>>>(pa, pb, na, nb, g);
    TNET_LAUNCH_CHECK();
    shadow_done(pa, TNET_OK);
    return shadow_done(pb, TNET_OK);
  }
  if (two) {
    // the pair kernel's conditions (launch_upd_pair): both 64x64 grids in one round over the CUs
    if (!g_pair) return TNET_ERR_UNSUPPORTED;
    na = cdiv(pa.M, 64) * cdiv(pa.N, 64);
    nb = cdiv(pb.M, 64) * cdiv(pb.N, 64);
  } else {
    // what tnet_affine_update_bias runs alone: the 64x64 configuration, unsplit
    const GemmPlan pl = plan_gemm<false>(pa, epi_splittable(EPI_SGD_B));
    if (pl.cfg != CFG_m64x64k32s4w41 || pl.ks != 1) return TNET_ERR_UNSUPPORTED;
    na = cdiv(pa.M, 64) * cdiv(pa.N, 64);
  }
  for (const GemmP* q : {&pa, &pb}) {
    if (q == &pb && !two) break;
    if (4 * (32L * q->lda + q->M) >= (1L << 32) || 4 * (32L * q->ldb + q->N) >= (1L << 32)) return TNET_ERR_UNSUPPORTED;
  }
  const int cus = cu_count();
  if (cus <= 0) return TNET_ERR_UNSUPPORTED;
  const int spare = cus - g_reserve - na - nb;
  if (two && na + nb > cus - g_reserve) return TNET_ERR_UNSUPPORTED;
  if (spare < 8) return TNET_ERR_UNSUPPORTED;
  const int ng = spare < 64 ? spare : 64;
  pa.group = pb.group = g_group > 0 ? g_group : 8;
  pa.early_issue = pb.early_issue = g_early;
  pa.wt = pb.wt = g_wt;
  BunchGatherP g{y, x, labels_out, labels_in, copy_from, dy.rows, c4, dy.stride, dx.stride};
  gemm16_upd_gather_kernel<64, 64, 32, 4, 1, 4><<<na + nb + ng, 256, 0, (hipStream_t)stream>>>(pa, pb, na, nb, g);
  TNET_LAUNCH_CHECK();
  shadow_done(pa, TNET_OK);
  if (two) shadow_done(pb, TNET_OK);
  return TNET_OK;
}

static int update_bwd_pair(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* W,
                           TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                           const float* colpart, int ldcolpart, float* b, float* corr_b, const float* E2,
                           TnetMatrixDim dE2, const float* W2, TnetMatrixDim dW2, const float* Ybelow, int strideYbelow,
                           float* Eo, TnetMatrixDim dEo, float* colpart2, int ldcolpart2, void* stream, bool bwd_t) {
  // tnet_affine_update_bias(X, E, W, ...) and tnet_affine_bwd_colsum(E2, W2, Ybelow, Eo, colpart2) in one
  // launch; the two must be independent (W is not W2, Eo / colpart2 overlap none of the update's operands).
  // bwd_t: W2 is the lower layer's transposed shadow [n_out x n_in] (tnet_affine_bwd_colsum_t's operand)
  if (dX.rows != dE.rows || dW.rows != dX.cols || dW.cols != dE.cols || !colpart || !b || ldcolpart < dE.cols)
    return TNET_ERR_ARG;
  if (mmt != 0.f && (!corrW || !corr_b)) return TNET_ERR_ARG;
  const int w2_k = bwd_t ? dW2.rows : dW2.cols, w2_n = bwd_t ? dW2.cols : dW2.rows;
  if (dE2.cols != w2_k || dEo.rows != dE2.rows || dEo.cols != w2_n || !Ybelow || !colpart2 ||
      ldcolpart2 < dEo.cols || !aligned16(Ybelow) || (strideYbelow & 3))
    return TNET_ERR_ARG;
  if (W == W2) return TNET_ERR_ARG;
  GemmP pu{};
  pu.M = dX.cols; pu.N = dE.cols; pu.K = dX.rows;
  pu.A = X; pu.lda = dX.stride; pu.B = E; pu.ldb = dE.stride; pu.C = W; pu.ldc = dW.stride;
  pu.corr = (mmt != 0.f || corrW) ? corrW : nullptr; pu.ldcorr = strideCorr;
  if (pu.corr && (pu.ldcorr & 3)) return TNET_ERR_ARG;
  pu.scale = scale; pu.mmt = mmt; pu.l2 = l2;
  pu.bpart = colpart; pu.ldbpart = ldcolpart; pu.bslabs = tnet_colsum_slabs(dE.rows);
  pu.bvec = b; pu.bcorr = mmt != 0.f ? corr_b : nullptr; pu.bscale = scale; pu.bmmt = mmt;
  int st = check_common(pu);
  if (st) return st;
  GemmP pb{};
  pb.M = dE2.rows; pb.N = w2_n; pb.K = dE2.cols;
  pb.A = E2; pb.lda = dE2.stride; pb.B = W2; pb.ldb = dW2.stride; pb.C = Eo; pb.ldc = dEo.stride;
  pb.alpha = 1.f; pb.beta = 0.f;
  pb.aux = Ybelow; pb.ldaux = strideYbelow;
  pb.cpart = colpart2; pb.ldcpart = ldcolpart2;
  st = check_common(pb);
  if (st) return st;
  if (bwd_t && g_reserve > 0) return TNET_ERR_UNSUPPORTED;
  shadow_attach(pu);
  // the update's own shadow is written in this launch: the backward may neither read it (a W2t that is the
  // updated layer's shadow would be read while it changes) nor write into it
  if (any_overlap({span_of(pu.Ct, pu.N, pu.ldct, 4)},
                  {span_of(pb.A, pb.M, pb.lda, 4), span_of(pb.B, bwd_t ? pb.K : pb.N, pb.ldb, 4),
                   span_of(pb.aux, pb.M, pb.ldaux, 4), span_of(pb.C, pb.M, pb.ldc, 4),
                   span_of(pb.cpart, tnet_colsum_slabs(pb.M), pb.ldcpart, 4)}))
    return TNET_ERR_ARG;
  return shadow_done(pu, launch_pair_a_bwd<EPI_SGD_B>(pu, pb, (hipStream_t)stream, bwd_t));
}

extern "C" int tnet_affine_update_bwd_pair(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE,
                                          float* W, TnetMatrixDim dW, float* corrW, int strideCorr, float scale,
                                          float mmt, float l2, const float* colpart, int ldcolpart, float* b,
                                          float* corr_b, const float* E2, TnetMatrixDim dE2, const float* W2,
                                          TnetMatrixDim dW2, const float* Ybelow, int strideYbelow, float* Eo,
                                          TnetMatrixDim dEo, float* colpart2, int ldcolpart2, void* stream) {
  return update_bwd_pair(X, dX, E, dE, W, dW, corrW, strideCorr, scale, mmt, l2, colpart, ldcolpart, b, corr_b, E2,
                         dE2, W2, dW2, Ybelow, strideYbelow, Eo, dEo, colpart2, ldcolpart2, stream, false);
}

extern "C" int tnet_affine_update_bwd_pair_t(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE,
                                            float* W, TnetMatrixDim dW, float* corrW, int strideCorr, float scale,
                                            float mmt, float l2, const float* colpart, int ldcolpart, float* b,
                                            float* corr_b, const float* E2, TnetMatrixDim dE2, const float* W2t,
                                            TnetMatrixDim dW2t, const float* Ybelow, int strideYbelow, float* Eo,
                                            TnetMatrixDim dEo, float* colpart2, int ldcolpart2, void* stream) {
  return update_bwd_pair(X, dX, E, dE, W, dW, corrW, strideCorr, scale, mmt, l2, colpart, ldcolpart, b, corr_b, E2,
                         dE2, W2t, dW2t, Ybelow, strideYbelow, Eo, dEo, colpart2, ldcolpart2, stream, true);
}

extern "C" int tnet_affine_grad_bwd_pair(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* G,
                                        TnetMatrixDim dG, const float* colpart, int ldcolpart, float* gradB,
                                        const float* E2, TnetMatrixDim dE2, const float* W2, TnetMatrixDim dW2,
                                        const float* Ybelow, int strideYbelow, float* Eo, TnetMatrixDim dEo,
                                        float* colpart2, int ldcolpart2, void* stream) {
  // tnet_affine_grad_bias(X, E, G, colpart, gradB) and tnet_affine_bwd_colsum(E2, W2, Ybelow, Eo, colpart2) in one
  // launch (the data-parallel step's gradient of layer l and the backward GEMM of layer l-1); independent: G / gradB
  // / Eo / colpart2 overlap none of the other's operands
  if (dX.rows != dE.rows || dG.rows != dX.cols || dG.cols != dE.cols || !colpart || !gradB || ldcolpart < dE.cols)
    return TNET_ERR_ARG;
  if (dE2.cols != dW2.cols || dEo.rows != dE2.rows || dEo.cols != dW2.rows || !Ybelow || !colpart2 ||
      ldcolpart2 < dEo.cols || !aligned16(Ybelow) || (strideYbelow & 3))
    return TNET_ERR_ARG;
  GemmP pu{};
  pu.M = dX.cols; pu.N = dE.cols; pu.K = dX.rows;
  pu.A = X; pu.lda = dX.stride; pu.B = E; pu.ldb = dE.stride; pu.C = G; pu.ldc = dG.stride;
  pu.alpha = 1.f; pu.beta = 0.f;
  pu.bpart = colpart; pu.ldbpart = ldcolpart; pu.bslabs = tnet_colsum_slabs(dE.rows);
  pu.bvec = gradB;
  int st = check_common(pu);
  if (st) return st;
  GemmP pb{};
  pb.M = dE2.rows; pb.N = dW2.rows; pb.K = dE2.cols;
  pb.A = E2; pb.lda = dE2.stride; pb.B = W2; pb.ldb = dW2.stride; pb.C = Eo; pb.ldc = dEo.stride;
  pb.alpha = 1.f; pb.beta = 0.f;
  pb.aux = Ybelow; pb.ldaux = strideYbelow;
  pb.cpart = colpart2; pb.ldcpart = ldcolpart2;
  st = check_common(pb);
  if (st) return st;
  // the two launches' outputs must not feed the other launch
  const std::array<ByteSpan, 2> wu{span_of(G, dG.rows, dG.stride, 4), span_of(gradB, dG.cols, 1, 4)};
  const std::array<ByteSpan, 2> wb{span_of(Eo, dEo.rows, dEo.stride, 4), span_of(colpart2, tnet_colsum_slabs(dE2.rows), ldcolpart2, 4)};
  if (any_overlap({wu[0], wu[1]}, {span_of(E2, dE2.rows, dE2.stride, 4), span_of(W2, dW2.rows, dW2.stride, 4),
                                   span_of(Ybelow, dEo.rows, strideYbelow, 4), wb[0], wb[1]}) ||
      any_overlap({wb[0], wb[1]}, {span_of(X, dX.rows, dX.stride, 4), span_of(E, dE.rows, dE.stride, 4),
                                   span_of(colpart, tnet_colsum_slabs(dE.rows), ldcolpart, 4)}))
    return TNET_ERR_ARG;
  return launch_pair_a_bwd<EPI_STORE_BG>(pu, pb, (hipStream_t)stream);
}

extern "C" int tnet_affine_grad_bias(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* G,
                                     TnetMatrixDim dG, const float* colpart, int ldcolpart, float* gradB,
                                     void* stream) {
  // tnet_affine_grad + gradB = colsum(E) from the slab sums tnet_affine_bwd_colsum wrote for E
  if (dX.rows != dE.rows || dG.rows != dX.cols || dG.cols != dE.cols || !colpart || !gradB || ldcolpart < dE.cols)
    return TNET_ERR_ARG;
  GemmP p{};
  p.M = dX.cols; p.N = dE.cols; p.K = dX.rows;
  p.A = X; p.lda = dX.stride; p.B = E; p.ldb = dE.stride; p.C = G; p.ldc = dG.stride;
  p.alpha = 1.f; p.beta = 0.f;
  p.bpart = colpart; p.ldbpart = ldcolpart; p.bslabs = tnet_colsum_slabs(dE.rows);
  p.bvec = gradB;
  int st = check_common(p);
  if (st) return st;
  if (p.M <= 0 || p.N <= 0) return TNET_OK;
  return launch_gemm<false, false, EPI_STORE_BG>(p, (hipStream_t)stream);
}

static int grad_bias_params(GemmP& p, const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* G,
                            TnetMatrixDim dG, const float* colpart, int ldcolpart, float* gradB) {
  if (dX.rows != dE.rows || dG.rows != dX.cols || dG.cols != dE.cols || !colpart || !gradB || ldcolpart < dE.cols)
    return TNET_ERR_ARG;
  p = GemmP{};
  p.M = dX.cols; p.N = dE.cols; p.K = dX.rows;
  p.A = X; p.lda = dX.stride; p.B = E; p.ldb = dE.stride; p.C = G; p.ldc = dG.stride;
  p.alpha = 1.f; p.beta = 0.f;
  p.bpart = colpart; p.ldbpart = ldcolpart; p.bslabs = tnet_colsum_slabs(dE.rows);
  p.bvec = gradB;
  return check_common(p);
}

extern "C" int tnet_affine_grad_bias_gather(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE,
                                            float* G, TnetMatrixDim dG, const float* colpart, int ldcolpart,
                                            float* gradB, const float* X2, TnetMatrixDim dX2, const float* E2,
                                            TnetMatrixDim dE2, float* G2, TnetMatrixDim dG2, const float* colpart2,
                                            int ldcolpart2, float* gradB2, float* y, const float* x, int* labels_out,
                                            const int* labels_in, const int* copy_from, TnetMatrixDim dy,
                                            TnetMatrixDim dx, void* stream) {
  // tnet_affine_grad_bias (X2 NULL) or two of them, and tnet_gather_bunch, in one launch (the data-parallel step's
  // last gradient GEMM(s) with the next bunch's gather on the CUs their tiles leave free:
  // tnet_affine_update_bias_gather's form)
  GemmP pa, pb{};
  int st = grad_bias_params(pa, X, dX, E, dE, G, dG, colpart, ldcolpart, gradB);
  if (st) return st;
  const bool two = X2 != nullptr;
  if (two) {
    st = grad_bias_params(pb, X2, dX2, E2, dE2, G2, dG2, colpart2, ldcolpart2, gradB2);
    if (st) return st;
    // the two gradients must not feed each other
    if (any_overlap({span_of(G, dG.rows, dG.stride, 4), span_of(gradB, dG.cols, 1, 4)},
                    {span_of(X2, dX2.rows, dX2.stride, 4), span_of(E2, dE2.rows, dE2.stride, 4),
                     span_of(colpart2, pb.bslabs, ldcolpart2, 4), span_of(G2, dG2.rows, dG2.stride, 4),
                     span_of(gradB2, dG2.cols, 1, 4)}) ||
        any_overlap({span_of(G2, dG2.rows, dG2.stride, 4), span_of(gradB2, dG2.cols, 1, 4)},
                    {span_of(X, dX.rows, dX.stride, 4), span_of(E, dE.rows, dE.stride, 4),
                     span_of(colpart, pa.bslabs, ldcolpart, 4)}))
      return TNET_ERR_ARG;
  }
  if (!y || !x || !labels_out || !labels_in || !copy_from || dy.cols != dx.cols || dy.rows < 0 || dy.stride < dy.cols ||
      dx.stride < dx.cols)
    return TNET_ERR_ARG;
  // the gather independent of the GEMM(s): they read X, E and the slab sums, write G and gradB
  auto reads = [](const GemmP& q) {
    return std::array<ByteSpan, 3>{span_of(q.A, q.K, q.lda, 4), span_of(q.B, q.K, q.ldb, 4),
                                    span_of(q.bpart, q.bslabs, q.ldbpart, 4)};
  };
  auto writes = [](const GemmP& q) {
    return std::array<ByteSpan, 2>{span_of(q.C, q.M, q.ldc, 4), span_of(q.bvec, q.N, 1, 4)};
  };
  const auto ra = reads(pa), rb = reads(pb);
  const auto wa = writes(pa), wb = writes(pb);
  if (!gather_independent(y, x, labels_out, labels_in, copy_from, dy, dx, {ra[0], ra[1], ra[2], rb[0], rb[1], rb[2]},
                          {wa[0], wa[1], wb[0], wb[1]}))
    return TNET_ERR_ARG;
  const int c4 = (dy.cols + 3) & ~3;
  if (((uintptr_t)y & 15) || ((uintptr_t)x & 15) || (dy.stride & 3) || (dx.stride & 3) || c4 > dy.stride ||
      c4 > dx.stride)
    return TNET_ERR_UNSUPPORTED;
  if (forced_cfg() >= 0 || split2_on() || g_split > 0) return TNET_ERR_UNSUPPORTED;
  if (pa.M <= 0 || pa.N <= 0 || (two && (pb.M <= 0 || pb.N <= 0))) return TNET_ERR_UNSUPPORTED;
  int na, nb = 0;
  if (two) {
    // both 64x64 grids in one round over the CUs (the update pair's rule)
    if (!g_pair) return TNET_ERR_UNSUPPORTED;
    na = cdiv(pa.M, 64) * cdiv(pa.N, 64);
    nb = cdiv(pb.M, 64) * cdiv(pb.N, 64);
  } else {
    // what tnet_affine_grad_bias runs alone: the 64x64 configuration, unsplit
    const GemmPlan pl = plan_gemm<false>(pa, epi_splittable(EPI_STORE_BG));
    if (pl.cfg != CFG_m64x64k32s4w41 || pl.ks != 1) return TNET_ERR_UNSUPPORTED;
    na = cdiv(pa.M, 64) * cdiv(pa.N, 64);
  }
  for (const GemmP* q : {&pa, &pb}) {
    if (q == &pb && !two) break;
    if (4 * (32L * q->lda + q->M) >= (1L << 32) || 4 * (32L * q->ldb + q->N) >= (1L << 32)) return TNET_ERR_UNSUPPORTED;
  }
  const int cus = cu_count();
  if (cus <= 0) return TNET_ERR_UNSUPPORTED;
  if (two && na + nb > cus - g_reserve) return TNET_ERR_UNSUPPORTED;
  const int spare = cus - g_reserve - na - nb;
  if (spare < 8) return TNET_ERR_UNSUPPORTED;
  const int ng = spare < 64 ? spare : 64;
  pa.group = pb.group = g_group > 0 ? g_group : 8;
  pa.early_issue = pb.early_issue = g_early;
  pa.wt = pb.wt = g_wt;
  BunchGatherP g{y, x, labels_out, labels_in, copy_from, dy.rows, c4, dy.stride, dx.stride};
  gemm16_upd_gather_kernel<64, 64, 32, 4, 1, 4, EPI_STORE_BG><<<na + nb + ng, 256, 0, (hipStream_t)stream>>>(
      pa, pb, na, nb, g);
  TNET_LAUNCH_CHECK();
  return TNET_OK;
}

extern "C" int tnet_affine_grad(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* G,
                                TnetMatrixDim dG, void* stream) {
  if (dX.rows != dE.rows || dG.rows != dX.cols || dG.cols != dE.cols) return TNET_ERR_ARG;
  GemmP p{};
  p.M = dX.cols; p.N = dE.cols; p.K = dX.rows;
  p.A = X; p.lda = dX.stride; p.B = E; p.ldb = dE.stride; p.C = G; p.ldc = dG.stride;
  p.alpha = 1.f; p.beta = 0.f;
  int st = check_common(p);
  if (st) return st;
  return launch_gemm<false, false, EPI_STORE>(p, (hipStream_t)stream);
}

extern "C" int tnet_gemm_config(const char* name) {
  forced_cfg();  // read the environment once, before it could override this call
  // "<cfg>[+sk<n>]": a tile configuration (or "auto"), optionally a forced split-K count.
  // "+rsv<R>": R CUs reserved (gemm16_sk_kernel over CUs - R workgroups for the data-parallel shapes),
  // 0 none -- as tnet_gemm_reserve, stays as set until changed; "+s2<0|1>": gemm16_split2_kernel for the
  // few-tile updates off / on (TNET_GEMM_SPLIT2), stays as set
  char base[64] = "auto";
  int split = -1, rsv = -1, s2 = -1;
  if (name) {
    const char* plus = strchr(name, '+');
    const size_t n = plus ? (size_t)(plus - name) : strlen(name);
    if (n >= sizeof(base)) return TNET_ERR_ARG;
    memcpy(base, name, n);
    base[n] = 0;
    while (plus) {
      if (!strncmp(plus, "+sk", 3) && atoi(plus + 3) >= 1) split = atoi(plus + 3);
      else if (!strncmp(plus, "+rsv", 4) && plus[4] >= '0' && plus[4] <= '9') rsv = atoi(plus + 4);
      else if (!strncmp(plus, "+s2", 3) && (plus[3] == '0' || plus[3] == '1')) s2 = plus[3] - '0';
      else return TNET_ERR_ARG;
      plus = strchr(plus + 1, '+');
    }
  }
  int cfg = -2;
  if (!strcmp(base, "auto")) cfg = -1;
  for (int i = 0; i < CFG_COUNT; i++)
    if (!strcmp(base, kCfgNames[i])) cfg = i;
  if (cfg == -2) return TNET_ERR_ARG;
  g_cfg = cfg;
  g_split = split;
  if (rsv >= 0) g_reserve = rsv;
  if (s2 >= 0) g_split2 = s2;
  return TNET_OK;
}

extern "C" int tnet_gemm_reserve(int cus) {
  if (cus < 0) return TNET_ERR_ARG;
  forced_cfg();
  g_reserve = cus;
  return TNET_OK;
}

#ifdef TNET_GEMM_STAMP
extern "C" int tnet_diag_stamps(unsigned long long* host, int n_wg) {
  if (n_wg > 8192) n_wg = 8192;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tnet_stamps), sizeof(unsigned long long) * 6 * n_wg, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? TNET_OK : TNET_ERR_LAUNCH;
}
extern "C" int tnet_diag_stamps_clear() {
  void* a = nullptr;
  if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_tnet_stamps)) != hipSuccess) return TNET_ERR_RUNTIME;
  // hipMemset is queued on the null stream, which does not order the library's non-blocking stream: without
  // the device-wide wait the next stamped launch could start under the clear and lose its first stamps
  return hipMemset(a, 0, sizeof(g_tnet_stamps)) == hipSuccess && hipDeviceSynchronize() == hipSuccess
             ? TNET_OK : TNET_ERR_RUNTIME;
}
#endif
