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
};

constexpr int BK = 32;

// A tile of R rows x CF floats (row-major in global memory, leading dimension ld), held in
// registers between its global load and its LDS store ([R][LDS_S] image).
template <int R, int CF, int LDS_S>
struct TileLoader {
  static constexpr int C4 = CF / 4;
  static constexpr int NV = R * C4 / 256;
  static_assert(R * C4 % 256 == 0, "tile must split evenly over 256 threads");
  f32x4 v[NV];

  __device__ __forceinline__ void load(const float* __restrict__ g, long ld, int r0, int c0, int rmax, int cmax,
                                       bool interior) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < NV; ++p) {
      const int idx = t + p * 256;
      const int r = idx / C4, c = (idx % C4) * 4;
      const int gr = r0 + r, gc = c0 + c;
      if (interior) {
        v[p] = *reinterpret_cast<const f32x4*>(g + (long)gr * ld + gc);
      } else {
        f32x4 x = {0.f, 0.f, 0.f, 0.f};
        if (gr < rmax) {
          const float* q = g + (long)gr * ld + gc;
          if (gc + 3 < cmax) {
            x = *reinterpret_cast<const f32x4*>(q);
          } else {
            if (gc < cmax) x[0] = q[0];
            if (gc + 1 < cmax) x[1] = q[1];
            if (gc + 2 < cmax) x[2] = q[2];
          }
        }
        v[p] = x;
      }
    }
  }
  __device__ __forceinline__ void store(float* s) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < NV; ++p) {
      const int idx = t + p * 256;
      const int r = idx / C4, c = (idx % C4) * 4;
      *reinterpret_cast<f32x4*>(s + r * LDS_S + c) = v[p];
    }
  }
};

template <int BM, int BN, int WM, int WN, bool A_KC, bool B_KC, int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const GemmP p) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1 && WM * WN == 4, "4 waves, 32x32 MFMA blocks");
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

  using LA = TileLoader<A_KC ? BM : BK, A_KC ? BK : BM, A_S>;
  using LB = TileLoader<B_KC ? BN : BK, B_KC ? BK : BN, B_S>;
  LA la;
  LB lb;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const bool rowsA_in = bm + BM <= M, colsB_in = bn + BN <= N;
  auto load_stage = [&](int k0) {
    const bool kin = k0 + BK <= K;
    if (A_KC) la.load(p.A, p.lda, bm, k0, M, K, rowsA_in && kin);
    else      la.load(p.A, p.lda, k0, bm, K, M, rowsA_in && kin);
    if (B_KC) lb.load(p.B, p.ldb, bn, k0, N, K, colsB_in && kin);
    else      lb.load(p.B, p.ldb, k0, bn, K, N, colsB_in && kin);
  };

  const int nk = (K + BK - 1) / BK;
  load_stage(0);
  la.store(smem);
  lb.store(smem + A_SZ);
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const float* As = smem + (t & 1) * (A_SZ + B_SZ);
    const float* Bs = As + A_SZ;
    if (t + 1 < nk) load_stage((t + 1) * BK);

#pragma unroll
    for (int kk = 0; kk < BK; kk += 8) {
      float av[TM][4], bv[TN][4];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = wm0 + a * 32 + li;
        if (A_KC) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(As + row * A_S + kk + 4 * lh);
          av[a][0] = x[0]; av[a][1] = x[1]; av[a][2] = x[2]; av[a][3] = x[3];
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) av[a][s] = As[(kk + 4 * lh + s) * A_S + row];
        }
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = wn0 + b * 32 + li;
        if (B_KC) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(Bs + col * B_S + kk + 4 * lh);
          bv[b][0] = x[0]; bv[b][1] = x[1]; bv[b][2] = x[2]; bv[b][3] = x[3];
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) bv[b][s] = Bs[(kk + 4 * lh + s) * B_S + col];
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a][s], bv[b][s], acc[a][b], 0, 0, 0);
    }

    if (t + 1 < nk) {
      float* An = smem + ((t + 1) & 1) * (A_SZ + B_SZ);
      la.store(An);
      lb.store(An + A_SZ);
    }
    __syncthreads();
  }

  // ---- epilogue: C/D map of 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
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

// ---------------------------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------------------------
template <bool A_KC, bool B_KC, int EPI>
static int launch_gemm(const GemmP& p, hipStream_t st) {
  if (p.M <= 0 || p.N <= 0) return TNET_OK;
  auto tiles = [&](int bm, int bn) { return (long)cdiv(p.M, bm) * cdiv(p.N, bn); };
  // choose the largest tile that still gives ~one workgroup per CU
  if (tiles(128, 128) >= 240) {
    gemm_f32_kernel<128, 128, 2, 2, A_KC, B_KC, EPI><<<(unsigned)tiles(128, 128), 256, 0, st>>>(p);
  } else if (tiles(128, 64) >= 200) {
    gemm_f32_kernel<128, 64, 2, 2, A_KC, B_KC, EPI><<<(unsigned)tiles(128, 64), 256, 0, st>>>(p);
  } else {
    gemm_f32_kernel<64, 64, 2, 2, A_KC, B_KC, EPI><<<(unsigned)tiles(64, 64), 256, 0, st>>>(p);
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
