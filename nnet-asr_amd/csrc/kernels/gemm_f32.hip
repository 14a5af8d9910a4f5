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
//  * 256-thread workgroups (4 waves, one per SIMD), BK = 32, LDS double buffer filled from a
//    register prefetch of the next k-tile issued before the MFMAs of the current one: one
//    barrier per k-tile; the global latency hides under 16-32 MFMAs per wave.
//  * k-contiguous tiles live in LDS as [rows][BK+4] (the +4 pad makes the 16-lane groups of
//    ds_read_b128 hit 16 distinct 4-bank slots); row-contiguous tiles as [BK][cols].
//  * tile shape chosen per GEMM shape so one launch has >= 256 workgroups where possible
//    (256 CUs); blockIdx is remapped so that consecutive tiles (which share operand panels)
//    run on one XCD (bijective remap, cdna_hip_programming.md T1).
#include <cstdlib>
#include <cstring>

#include "kcommon.h"

namespace tnetk {

enum { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_SIG = 2, EPI_DSIG = 3, EPI_SGD = 4 };

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
  int diag_noload;              // diagnostics only: skip the k-loop's global loads (wrong results)
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
      if (EPI == EPI_BIAS || EPI == EPI_BIAS_SIG) bias_v = p.bias[col];
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
        } else if (EPI == EPI_DSIG) {
          const float y = p.aux[(long)row * p.ldaux + col];
          *cp = y * (1.f - y) * v;
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

// A tile of R rows x CF floats (row-major in global memory, leading dimension ld), held in
// registers between its global load and its LDS store ([R][LDS_S] image).
template <int R, int CF, int LDS_S, int NT>
struct TileLoader {
  static constexpr int C4 = CF / 4;
  static constexpr int NV = R * C4 / NT;
  static_assert(R * C4 % NT == 0, "tile must split evenly over the workgroup");
  static_assert(NV <= 10, "3 validity bits per float4");
  f32x4 v[NV];
  unsigned valid;

  // Branch-free bounded load: every lane issues its dwordx4 loads unconditionally (so hipcc keeps
  // them all in flight and waits once, at the LDS store); out-of-range rows are clamped to the last
  // valid row and out-of-range columns to column 0, then zeroed by select.  A column start
  // gc < cmax <= ld (ld % 4 == 0) keeps the 16-byte read inside the row's allocation.
  __device__ __forceinline__ void load(const float* __restrict__ g, long ld, int r0, int c0, int rmax, int cmax) {
    const int t = threadIdx.x;
    valid = 0;
#pragma unroll
    for (int p = 0; p < NV; ++p) {
      const int idx = t + p * NT;
      const int r = idx / C4, c = (idx % C4) * 4;
      const int gr = r0 + r, gc = c0 + c;
      const int grc = gr < rmax ? gr : rmax - 1;
      const int gcc = gc < cmax ? gc : 0;
      v[p] = *reinterpret_cast<const f32x4*>(g + (long)grc * ld + gcc);
      // validity of the 4 elements, applied at store time so the loads stay in flight
      const int nvalid = gr < rmax ? (cmax - gc < 0 ? 0 : (cmax - gc > 4 ? 4 : cmax - gc)) : 0;
      valid |= (unsigned)nvalid << (3 * p);
    }
  }
  __device__ __forceinline__ void store(float* s) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < NV; ++p) {
      const int idx = t + p * NT;
      const int r = idx / C4, c = (idx % C4) * 4;
      const int nv = (valid >> (3 * p)) & 7;
      f32x4 x = v[p];
#pragma unroll
      for (int k = 0; k < 4; ++k) x[k] = (k < nv) ? x[k] : 0.f;
      *reinterpret_cast<f32x4*>(s + r * LDS_S + c) = x;
    }
  }
};

template <int BM, int BN, int BK, int WM, int WN, int PF, bool A_KC, bool B_KC, int EPI>
__global__ __launch_bounds__(WM * WN * 64) void gemm_f32_kernel(const GemmP p) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1 && BM == TM * WM * 32 && BN == TN * WN * 32, "32x32 MFMA blocks per wave");
  static_assert(BK % 8 == 0, "k chunks of 8");
  constexpr int A_S = A_KC ? (BK + 4) : BM;
  constexpr int B_S = B_KC ? (BK + 4) : BN;
  constexpr int A_SZ = A_KC ? BM * A_S : BK * A_S;
  constexpr int B_SZ = B_KC ? BN * B_S : BK * B_S;
  __shared__ __attribute__((aligned(16))) float smem[2 * (A_SZ + B_SZ)];

  const int M = p.M, N = p.N, K = p.K;
  const int nbn = (N + BN - 1) / BN, nbm = (M + BM - 1) / BM;
  const int nwg = nbm * nbn;
  // bijective XCD-aware remap: blocks b, b+8, ... (one XCD) take a contiguous range of tiles
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int L = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  const int bm = (L / nbn) * BM, bn = (L % nbn) * BN;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm0 = (wid / WN) * (BM / WM), wn0 = (wid % WN) * (BN / WN);
  const int li = lane & 31, lh = lane >> 5;

  using LA = TileLoader<A_KC ? BM : BK, A_KC ? BK : BM, A_S, NT>;
  using LB = TileLoader<B_KC ? BN : BK, B_KC ? BK : BN, B_S, NT>;
  LA la[PF];
  LB lb[PF];

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  auto load_stage = [&](LA& l_a, LB& l_b, int k0) {
    if (p.diag_noload && k0 > 0) return;
    if (A_KC) l_a.load(p.A, p.lda, bm, k0, M, K);
    else      l_a.load(p.A, p.lda, k0, bm, K, M);
    if (B_KC) l_b.load(p.B, p.ldb, bn, k0, N, K);
    else      l_b.load(p.B, p.ldb, k0, bn, K, N);
  };
  auto store_stage = [&](const LA& l_a, const LB& l_b, int t) {
    if (p.diag_noload) return;
    float* An = smem + (t & 1) * (A_SZ + B_SZ);
    l_a.store(An);
    l_b.store(An + A_SZ);
  };

  // MFMAs over one LDS stage; fragments of k-chunk kk+8 are read while the MFMAs of chunk kk issue
  auto compute = [&](int t) {
    const float* As = smem + (t & 1) * (A_SZ + B_SZ);
    const float* Bs = As + A_SZ;
    float av[2][TM][4], bv[2][TN][4];
    auto read_frags = [&](int kk, float (&a_)[TM][4], float (&b_)[TN][4]) {
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = wm0 + a * 32 + li;
        if (A_KC) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(As + row * A_S + kk + 4 * lh);
          a_[a][0] = x[0]; a_[a][1] = x[1]; a_[a][2] = x[2]; a_[a][3] = x[3];
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) a_[a][s] = As[(kk + 4 * lh + s) * A_S + row];
        }
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = wn0 + b * 32 + li;
        if (B_KC) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(Bs + col * B_S + kk + 4 * lh);
          b_[b][0] = x[0]; b_[b][1] = x[1]; b_[b][2] = x[2]; b_[b][3] = x[3];
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) b_[b][s] = Bs[(kk + 4 * lh + s) * B_S + col];
        }
      }
    };
    read_frags(0, av[0], bv[0]);
#pragma unroll
    for (int kc = 0; kc < BK / 8; ++kc) {
      const int cur = kc & 1;
      if (kc + 1 < BK / 8) read_frags((kc + 1) * 8, av[cur ^ 1], bv[cur ^ 1]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[cur][a][s], bv[cur][b][s], acc[a][b], 0, 0, 0);
    }
  };

  const int nk = (K + BK - 1) / BK;
  if constexpr (PF == 1) {
    // one k-tile in flight: load t+1 to registers under the MFMAs of t, store after them
    load_stage(la[0], lb[0], 0);
    la[0].store(smem);
    lb[0].store(smem + A_SZ);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      if (t + 1 < nk) load_stage(la[0], lb[0], (t + 1) * BK);
      compute(t);
      if (t + 1 < nk) store_stage(la[0], lb[0], t + 1);
      __syncthreads();
    }
  } else {
    // two k-tiles in flight: register set (s % 2) holds k-tile s from its load (issued two
    // tiles ahead) until its LDS store (one tile ahead); plain loads survive the barriers
    load_stage(la[0], lb[0], 0);
    if (nk > 1) load_stage(la[1], lb[1], BK);
    la[0].store(smem);
    lb[0].store(smem + A_SZ);
    __syncthreads();
    for (int t = 0; t < nk; t += 2) {
      if (t + 2 < nk) load_stage(la[0], lb[0], (t + 2) * BK);
      compute(t);
      if (t + 1 < nk) store_stage(la[1], lb[1], t + 1);
      __syncthreads();
      if (t + 1 < nk) {
        if (t + 3 < nk) load_stage(la[1], lb[1], (t + 3) * BK);
        compute(t + 1);
        if (t + 2 < nk) store_stage(la[0], lb[0], t + 2);
        __syncthreads();
      }
    }
  }

  epilogue<TM, TN, EPI>(p, acc, bm, bn, wm0, wn0, li, lh);
}

// =============================================================================================
// LDS-DMA pipelined variant: k-tiles of 32 are streamed global -> LDS by global_load_lds_dwordx4
// (no VGPR staging) into an S-slot ring, S-1 tiles in flight, one raw s_barrier per k-tile behind
// a COUNTED vmcnt (cdna_hip_programming.md section 5 "Pipelining across barriers").
//   * k-contiguous operand images are [rows][32] with the 16-B chunk index XOR-swizzled by
//     ((row >> 1) & 7): the DMA image is lane-linear, so the swizzle is applied to the per-lane
//     SOURCE address and undone on the ds_read_b128 (rule 21); the 16-lane groups of ds_read_b128
//     then hit 16 distinct 4-bank slots.  Row-contiguous images are plain [32][cols].
//   * rows / columns beyond M / N are clamped to valid memory (their products only reach outputs
//     that are never stored); a partial last k-tile (K % 32) goes through the masked register path.
// =============================================================================================
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  // gfx9 s_waitcnt simm16: vmcnt[3:0], expcnt[6:4], lgkmcnt[11:8], vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | (((N >> 4) & 0x3) << 14));
}

__device__ __forceinline__ int swz8(int r) { return (r >> 1) & 7; }

template <int BM, int BN, int WM, int WN, int S, bool SB, bool A_KC, bool B_KC, int EPI>
__global__ __launch_bounds__(256) void gemm_f32_glds_kernel(const GemmP p) {
  constexpr int BK = 32, NT = 256;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "4 waves of 32x32 MFMA blocks");
  constexpr int A_SZ = BM * BK, B_SZ = BN * BK, ST_SZ = A_SZ + B_SZ;
  constexpr int GA = A_SZ / 4 / NT, GB = B_SZ / 4 / NT, G = GA + GB;  // DMA instructions per thread per tile
  static_assert(A_SZ % (4 * NT) == 0 && B_SZ % (4 * NT) == 0, "tile splits into 1-KiB wave pieces");
  __shared__ __attribute__((aligned(16))) float smem[S * ST_SZ];

  const int M = p.M, N = p.N, K = p.K;
  const int nbn = (N + BN - 1) / BN, nbm = (M + BM - 1) / BM;
  const int nwg = nbm * nbn;
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int L = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  const int bm = (L / nbn) * BM, bn = (L % nbn) * BN;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm0 = (wid / WN) * (BM / WM), wn0 = (wid % WN) * (BN / WN);
  const int li = lane & 31, lh = lane >> 5;

  // per-lane source offsets (elements) of each DMA piece, relative to the k-tile origin
  long srcA[GA], srcB[GB];
#pragma unroll
  for (int g = 0; g < GA; ++g) {
    const int u = (g * 4 + wid) * 64 + lane;  // 16-B unit index inside the image
    if (A_KC) {
      const int r = u >> 3, j = u & 7;
      const int gr = min(bm + r, M - 1);
      srcA[g] = (long)gr * p.lda + 4 * (j ^ swz8(r));
    } else {
      const int k = u / (BM / 4), c = (u % (BM / 4)) * 4;
      srcA[g] = (long)k * p.lda + (bm + c < M ? bm + c : 0);
    }
  }
#pragma unroll
  for (int g = 0; g < GB; ++g) {
    const int u = (g * 4 + wid) * 64 + lane;
    if (B_KC) {
      const int r = u >> 3, j = u & 7;
      const int gr = min(bn + r, N - 1);
      srcB[g] = (long)gr * p.ldb + 4 * (j ^ swz8(r));
    } else {
      const int k = u / (BN / 4), c = (u % (BN / 4)) * 4;
      srcB[g] = (long)k * p.ldb + (bn + c < N ? bn + c : 0);
    }
  }

  auto issue = [&](int t) {  // DMA of full k-tile t into ring slot t % S
    float* st = smem + (t % S) * ST_SZ;
    const long ka = A_KC ? (long)t * BK : (long)t * BK * p.lda;
    const long kb = B_KC ? (long)t * BK : (long)t * BK * p.ldb;
#pragma unroll
    for (int g = 0; g < GA; ++g)
      __builtin_amdgcn_global_load_lds((const void*)(p.A + ka + srcA[g]), (void*)(st + (g * 4 + wid) * 256), 16, 0, 0);
#pragma unroll
    for (int g = 0; g < GB; ++g)
      __builtin_amdgcn_global_load_lds((const void*)(p.B + kb + srcB[g]), (void*)(st + A_SZ + (g * 4 + wid) * 256), 16,
                                       0, 0);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  auto compute = [&](const float* st) {
    const float* As = st;
    const float* Bs = st + A_SZ;
    float av[2][TM][4], bv[2][TN][4];
    auto read_frags = [&](int kc, float (&a_)[TM][4], float (&b_)[TN][4]) {
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = wm0 + a * 32 + li;
        if (A_KC) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(As + row * BK + 4 * ((2 * kc + lh) ^ swz8(row)));
          a_[a][0] = x[0]; a_[a][1] = x[1]; a_[a][2] = x[2]; a_[a][3] = x[3];
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) a_[a][s] = As[(8 * kc + 4 * lh + s) * BM + row];
        }
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = wn0 + b * 32 + li;
        if (B_KC) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(Bs + col * BK + 4 * ((2 * kc + lh) ^ swz8(col)));
          b_[b][0] = x[0]; b_[b][1] = x[1]; b_[b][2] = x[2]; b_[b][3] = x[3];
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) b_[b][s] = Bs[(8 * kc + 4 * lh + s) * BN + col];
        }
      }
    };
    read_frags(0, av[0], bv[0]);
#pragma unroll
    for (int kc = 0; kc < BK / 8; ++kc) {
      const int cur = kc & 1;
      if (kc + 1 < BK / 8) read_frags(kc + 1, av[cur ^ 1], bv[cur ^ 1]);
      if (SB) __builtin_amdgcn_sched_barrier(0);  // keep the next chunk's ds_reads ahead of these MFMAs
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[cur][a][s], bv[cur][b][s], acc[a][b], 0, 0, 0);
    }
  };

  const int nfull = K / BK;
  // prologue: S-1 tiles in flight
#pragma unroll
  for (int t = 0; t < S - 1; ++t)
    if (t < nfull) issue(t);
  for (int t = 0; t < nfull; ++t) {
    // retire tile t: at most min(S-2, nfull-1-t) younger tiles may stay in flight
    const int younger = min(S - 2, nfull - 1 - t);
    if (younger >= 2) wait_vmcnt<2 * G>();
    else if (younger == 1) wait_vmcnt<G>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // every wave's pieces of tile t have landed; slot (t-1)%S is free
    if (t + S - 1 < nfull && !p.diag_noload) issue(t + S - 1);
    compute(smem + ((p.diag_noload ? 0 : t) % S) * ST_SZ);
  }
  if (K % BK) {
    // masked tail k-tile through registers, same swizzled image, in slot nfull % S
    __builtin_amdgcn_s_barrier();
    float* st = smem + (nfull % S) * ST_SZ;
    const int k0 = nfull * BK;
    for (int u = threadIdx.x; u < A_SZ / 4; u += NT) {
      int gr, gc, lds;
      if (A_KC) { const int r = u >> 3, j = u & 7; gr = bm + r; gc = k0 + 4 * (j ^ swz8(r)); }
      else { const int k = u / (BM / 4); gr = k0 + k; gc = bm + (u % (BM / 4)) * 4; }
      lds = u * 4;
      const int rmax = A_KC ? M : K, cmax = A_KC ? K : M;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (gr < rmax) {
        const float* q = p.A + (long)gr * p.lda + gc;
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = (gc + e < cmax) ? q[e] : 0.f;
      }
      *reinterpret_cast<f32x4*>(st + lds) = x;
    }
    for (int u = threadIdx.x; u < B_SZ / 4; u += NT) {
      int gr, gc;
      if (B_KC) { const int r = u >> 3, j = u & 7; gr = bn + r; gc = k0 + 4 * (j ^ swz8(r)); }
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
    compute(st);
  }
  epilogue<TM, TN, EPI>(p, acc, bm, bn, wm0, wn0, li, lh);
}

// ---------------------------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------------------------
// Tile configurations: BMxBN tile, BK k-depth per LDS stage, WMxWN waves (each wave owns a
// (BM/WM)x(BN/WN) sub-tile of 32x32 MFMA blocks).
enum GemmCfg { CFG_128x64_W4, CFG_64x64_W4, CFG_128x64_W8, CFG_G128x64_S3, CFG_G64x64_S3, CFG_G64x64_S4,
               CFG_G128x64_S3B, CFG_G64x64_S3B, CFG_G64x64_S4B, CFG_COUNT };
static const char* kCfgNames[CFG_COUNT] = {"128x64w4", "64x64w4", "128x64w8", "g128x64s3", "g64x64s3", "g64x64s4",
                                           "g128x64s3b", "g64x64s3b", "g64x64s4b"};

static int g_cfg = -2;  // -2: not initialised, -1: automatic
static int forced_cfg() {
  if (g_cfg == -2) {
    g_cfg = -1;
    const char* e = getenv("TNET_GEMM_CFG");
    if (e)
      for (int i = 0; i < CFG_COUNT; i++)
        if (!strcmp(e, kCfgNames[i])) g_cfg = i;
  }
  return g_cfg;
}

template <int BM, int BN, int BK, int WM, int WN, int PF, bool A_KC, bool B_KC, int EPI>
static void launch_cfg(const GemmP& p, hipStream_t st) {
  const unsigned tiles = (unsigned)((long)cdiv(p.M, BM) * cdiv(p.N, BN));
  gemm_f32_kernel<BM, BN, BK, WM, WN, PF, A_KC, B_KC, EPI><<<tiles, WM * WN * 64, 0, st>>>(p);
}

template <int BM, int BN, int WM, int WN, int S, bool SB, bool A_KC, bool B_KC, int EPI>
static void launch_glds(const GemmP& p, hipStream_t st) {
  const unsigned tiles = (unsigned)((long)cdiv(p.M, BM) * cdiv(p.N, BN));
  gemm_f32_glds_kernel<BM, BN, WM, WN, S, SB, A_KC, B_KC, EPI><<<tiles, 256, 0, st>>>(p);
}

template <bool A_KC, bool B_KC, int EPI>
static int launch_gemm(const GemmP& p_in, hipStream_t st) {
  if (p_in.M <= 0 || p_in.N <= 0) return TNET_OK;
  static const int noload = getenv("TNET_GEMM_DIAG_NOLOAD") ? 1 : 0;
  GemmP p = p_in;
  p.diag_noload = noload;
  auto tiles = [&](int bm, int bn) { return (long)cdiv(p.M, bm) * cdiv(p.N, bn); };
  int cfg = forced_cfg();
  if (cfg < 0) {
    // the largest tile that still gives ~one workgroup per CU (256 CUs)
    cfg = CFG_G64x64_S4;
  }
  switch (cfg) {
    case CFG_128x64_W4: launch_cfg<128, 64, 32, 2, 2, 1, A_KC, B_KC, EPI>(p, st); break;
    case CFG_64x64_W4: launch_cfg<64, 64, 32, 2, 2, 1, A_KC, B_KC, EPI>(p, st); break;
    case CFG_128x64_W8: launch_cfg<128, 64, 32, 4, 2, 1, A_KC, B_KC, EPI>(p, st); break;
    case CFG_G128x64_S3: launch_glds<128, 64, 2, 2, 3, false, A_KC, B_KC, EPI>(p, st); break;
    case CFG_G64x64_S3: launch_glds<64, 64, 2, 2, 3, false, A_KC, B_KC, EPI>(p, st); break;
    case CFG_G64x64_S4: launch_glds<64, 64, 2, 2, 4, false, A_KC, B_KC, EPI>(p, st); break;
    case CFG_G128x64_S3B: launch_glds<128, 64, 2, 2, 3, true, A_KC, B_KC, EPI>(p, st); break;
    case CFG_G64x64_S3B: launch_glds<64, 64, 2, 2, 3, true, A_KC, B_KC, EPI>(p, st); break;
    case CFG_G64x64_S4B: launch_glds<64, 64, 2, 2, 4, true, A_KC, B_KC, EPI>(p, st); break;
    default: return TNET_ERR_ARG;
  }
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
  if (dX.cols != dW.rows || dY.rows != dX.rows || dY.cols != dW.cols || !b) return TNET_ERR_ARG;
  GemmP p{};
  p.M = dX.rows; p.N = dW.cols; p.K = dX.cols;
  p.A = X; p.lda = dX.stride; p.B = W; p.ldb = dW.stride; p.C = Y; p.ldc = dY.stride;
  p.bias = b;
  int st = check_common(p);
  if (st) return st;
  if (act == 1) return launch_gemm<true, false, EPI_BIAS_SIG>(p, (hipStream_t)stream);
  return launch_gemm<true, false, EPI_BIAS>(p, (hipStream_t)stream);
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
    if (!Ybelow) return TNET_ERR_ARG;
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
  p.scale = scale; p.mmt = mmt; p.l2 = l2;
  int st = check_common(p);
  if (st) return st;
  return launch_gemm<false, false, EPI_SGD>(p, (hipStream_t)stream);
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
  if (!name || !strcmp(name, "auto")) {
    g_cfg = -1;
    return TNET_OK;
  }
  for (int i = 0; i < CFG_COUNT; i++)
    if (!strcmp(name, kCfgNames[i])) {
      g_cfg = i;
      return TNET_OK;
    }
  return TNET_ERR_ARG;
}
