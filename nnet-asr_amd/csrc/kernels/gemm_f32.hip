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
  int group;                    // tile-rows per group of the blockIdx -> tile order
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

// XOR swizzle of the 16-B chunk index of row r of a k-contiguous [rows][BK] image.
//   BK = 32: rows are 128 B, two per 256-B bank row -> ((r >> 1) & 7) over the 8 chunks;
//   BK = 64: rows are 256 B, one per bank row        -> (r & 15) over the 16 chunks.
template <int BK>
__device__ __forceinline__ int swz(int r) {
  return BK == 32 ? ((r >> 1) & 7) : (r & 15);
}

template <int BM, int BN, int BK, int WM, int WN, int S, bool A_KC, bool B_KC, int EPI>
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

  // MFMAs over one ring slot.  k of MFMA step s (0..3) of 8-deep chunk kc is 8kc + 4*kh + s
  // (kh = lane >> 5), so a k-contiguous operand feeds 4 MFMAs from one ds_read_b128.
  auto compute = [&](const float* st) {
    const float* As = st;
    const float* Bs = st + A_SZ;
    float av[2][TM][4], bv[2][TN][4];
    auto read_frags = [&](int kc, float (&a_)[TM][4], float (&b_)[TN][4]) {
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = wm0 + a * 32 + li;
        if (A_KC) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(As + row * BK + 4 * ((2 * kc + lh) ^ swz<BK>(row)));
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
          const f32x4 x = *reinterpret_cast<const f32x4*>(Bs + col * BK + 4 * ((2 * kc + lh) ^ swz<BK>(col)));
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
    compute(st);
  }
  epilogue<TM, TN, EPI>(p, acc, bm, bn, wm0, wn0, li, lh);
}

// ---------------------------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------------------------
// name: g<BM>x<BN>k<BK>s<S>w<waves>  (waves laid out WMxWN)
#define TNET_GEMM_CFGS(X)                   \
  X(g64x64k32s4w4, 64, 64, 32, 2, 2, 4)     \
  X(g64x64k64s2w4, 64, 64, 64, 2, 2, 2)     \
  X(g64x64k32s4w2, 64, 64, 32, 2, 1, 4)     \
  X(g64x64k64s2w2, 64, 64, 64, 2, 1, 2)     \
  X(g128x64k32s3w4, 128, 64, 32, 2, 2, 3)   \
  X(g64x128k32s3w4, 64, 128, 32, 2, 2, 3)   \
  X(g128x128k32s2w4, 128, 128, 32, 2, 2, 2) \
  X(g128x128k32s3w8, 128, 128, 32, 2, 4, 3)

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
static int forced_cfg() {
  if (g_cfg == -2) {
    g_cfg = -1;
    const char* e = getenv("TNET_GEMM_CFG");
    if (e)
      for (int i = 0; i < CFG_COUNT; i++)
        if (!strcmp(e, kCfgNames[i])) g_cfg = i;
    const char* gg = getenv("TNET_GEMM_GROUP");
    if (gg) g_group = atoi(gg);
  }
  return g_cfg;
}

template <int BM, int BN, int BK, int WM, int WN, int S, bool A_KC, bool B_KC, int EPI>
static void launch_glds(const GemmP& p, hipStream_t st) {
  const unsigned tiles = (unsigned)((long)cdiv(p.M, BM) * cdiv(p.N, BN));
  gemm_f32_glds_kernel<BM, BN, BK, WM, WN, S, A_KC, B_KC, EPI><<<tiles, WM * WN * 64, 0, st>>>(p);
}

template <bool A_KC, bool B_KC, int EPI>
static int launch_gemm(const GemmP& p_in, hipStream_t st) {
  if (p_in.M <= 0 || p_in.N <= 0) return TNET_OK;
  static const int noload = getenv("TNET_GEMM_DIAG_NOLOAD") ? 1 : 0;
  GemmP p = p_in;
  p.diag_noload = noload;
  int cfg = forced_cfg();
  if (cfg < 0) cfg = CFG_g64x64k32s4w4;
  p.group = g_group > 0 ? g_group : 8;
  switch (cfg) {
#define X(name, BM, BN, BK, WM, WN, S) \
  case CFG_##name: launch_glds<BM, BN, BK, WM, WN, S, A_KC, B_KC, EPI>(p, st); break;
    TNET_GEMM_CFGS(X)
#undef X
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
  forced_cfg();  // read the environment once, before it could override this call
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
