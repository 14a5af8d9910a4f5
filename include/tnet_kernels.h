/*
 * tnet_kernels.h -- C ABI of the MI355X (gfx950) device kernels of the TNet frame-batched
 * forward / backward / SGD-update path.
 *
 * This is the drop-in replacement for the two device-side ABIs the reference CuBaseLib uses:
 *   (1) the extern "C" cudaF_* kernel wrappers of src/CuBaseLib/cukernels.h:5-79 and
 *       src/CuBaseLib/curandkernels.h:8-31, and
 *   (2) the legacy cuBLAS calls cublasSgemm / cublasSgemv / cublasSger
 *       (src/CuBaseLib/cumatrix.tcc:363,384, src/CuBaseLib/cumath.cc:105,237,334,358).
 * plus the fused kernels the MI355X path is built from.
 *
 * Conventions (all functions):
 *   - row-major matrices described by TnetMatrixDim {rows, cols, stride} (== MatrixDim,
 *     cukernels.h:11-15); stride is in elements;
 *   - raw device pointers, never owned, never freed here; no allocation inside except in the
 *     documented workspaces the caller passes in;
 *   - launch geometry is a kernel-internal detail (no dim3 in the ABI, unlike cukernels.h);
 *   - every launch goes on the caller's stream (hipStream_t passed as void*; NULL = default);
 *     no device synchronisation inside (the reference synchronised after every call,
 *     cucommon.h:13-22);
 *   - return 0 (TNET_OK) or a negative TNET_ERR_* status; the C++ layer maps a status to an
 *     exception exactly like cuSafeCall (cucommon.h:13-22) minus the sync;
 *   - thread-safe per stream.
 */
#ifndef TNET_KERNELS_H_
#define TNET_KERNELS_H_

#ifdef __cplusplus
extern "C" {
#endif

typedef struct TnetMatrixDim_ {
  int rows;
  int cols;
  int stride;
} TnetMatrixDim;

/* objective statistics accumulator: TNET_STATS_SLOTS pairs {error, correct} of doubles */
#define TNET_STATS_SLOTS 512
#define TNET_STATS_WORDS (2 * TNET_STATS_SLOTS)

enum {
  TNET_OK = 0,
  TNET_ERR_ARG = -1,       /* bad dimension / stride / pointer alignment */
  TNET_ERR_LAUNCH = -2,    /* hipGetLastError after launch */
  TNET_ERR_RUNTIME = -3,   /* other HIP runtime failure */
  TNET_ERR_UNSUPPORTED = -4
};

/* Returns a static string for a status code. */
const char* tnet_status_str(int status);
/* Build / device description ("gfx950 tnet_amd <version>"). */
const char* tnet_version(void);

/* ------------------------------------------------------------------------------------
 * Element-wise matrix ops  (cukernels.h:21-31 -> cukernels.cu:11-141)
 * ---------------------------------------------------------------------------------- */
/* M[i,j] = v                                  -- cudaF_set_const (cukernels.cu:11-19) */
int tnetF_set_const(float* mat, float value, TnetMatrixDim d, void* stream);
/* M = log(M)                                  -- cudaF_apply_log (cukernels.cu:23-31) */
int tnetF_apply_log(float* mat, TnetMatrixDim d, void* stream);
/* M[mask==0] = 0                              -- cudaF_apply_mask (cukernels.cu:34-43) */
int tnetF_apply_mask(float* mat, const float* mask, TnetMatrixDim dmat, TnetMatrixDim dmask, void* stream);
/* soft threshold |x|<l1 -> 0, else x -+ l1    -- cudaF_apply_l1 (cukernels.cu:46-62) */
int tnetF_apply_l1(float* mat, float l1, TnetMatrixDim d, void* stream);
/* M[i,j] *= s[j]                              -- cudaF_scale_cols (cukernels.cu:65-73) */
int tnetF_scale_cols(float* mat, const float* scale, TnetMatrixDim d, void* stream);
/* M[i,j] *= s[i]                              -- cudaF_scale_rows (cukernels.cu:76-84) */
int tnetF_scale_rows(float* mat, const float* scale, TnetMatrixDim d, void* stream);
/* D = alpha*A + beta*D                        -- cudaF_add_scaled (cukernels.cu:87-95);
 * A and D share dimensions d but may have different strides (strideA). */
int tnetF_add_scaled(float alpha, const float* A, int strideA, float beta, float* dst, TnetMatrixDim d,
                     void* stream);
/* D[i,j] = alpha*row[j] + beta*D[i,j]         -- cudaF_add_scaled_row (cukernels.cu:98-117) */
int tnetF_add_scaled_row(float alpha, const float* row, float beta, float* dst, TnetMatrixDim d, void* stream);
/* M = M .* A                                  -- cudaF_mul_elem (cukernels.cu:120-128) */
int tnetF_mul_elem(float* mat, const float* A, int strideA, TnetMatrixDim d, void* stream);
/* M = log(max(M, FLT_MIN))                    -- cudaF_log_elem (cukernels.cu:131-141) */
int tnetF_log_elem(float* mat, TnetMatrixDim d, void* stream);

/* ------------------------------------------------------------------------------------
 * Vector reductions  (cukernels.h:33-35)
 * ---------------------------------------------------------------------------------- */
/* v[j] = alpha * sum_i M[i,j] + beta * v[j]   -- cudaF_add_col_sum / _add_col_sum_reduce
 * (cukernels.cu:147-187).  Deterministic: fixed-order partial sums in fp32, combined in fp64.
 * `workspace` needs tnet_col_sum_workspace(d) bytes of device memory (or NULL to use an
 * internal per-device buffer, not thread-safe). */
long tnet_col_sum_workspace(TnetMatrixDim d);
int tnetF_add_col_sum(float alpha, const float* mat, float beta, float* vec, TnetMatrixDim d, void* workspace,
                      void* stream);

/* ------------------------------------------------------------------------------------
 * Activations / objective  (cukernels.h:38-41, 51-52)
 * ---------------------------------------------------------------------------------- */
/* y = 1/(1+exp(-x))                           -- cudaF_sigmoid (cukernels.cu:192-206) */
int tnetF_sigmoid(float* y, const float* x, TnetMatrixDim d, void* stream);
/* eout = y (1-y) e                            -- cudaF_diff_sigmoid (cukernels.cu:209-217) */
int tnetF_diff_sigmoid(float* eout, const float* e, const float* y, TnetMatrixDim d, void* stream);
/* row softmax, y = exp(x - max) / sum         -- cudaF_softmax / _softmax_reduce (cukernels.cu:220-343);
 * one wavefront per row, any number of columns. */
int tnetF_softmax(float* y, const float* x, TnetMatrixDim d, void* stream);
/* match[i] = argmax(out[i,:]) == argmax(des[i,:]) (first max wins)
 *                                             -- cudaF_check_class[_reduce] (cukernels.cu:396-483) */
int tnetF_check_class(const float* out, const float* des, int* match, TnetMatrixDim d, void* stream);

/* ------------------------------------------------------------------------------------
 * Gathers / front-end transforms  (cukernels.h:43-45)
 * ---------------------------------------------------------------------------------- */
/* y[i,j] = x[i + off[j / in.cols], j % in.cols] with edge clamp  -- cudaF_expand (cukernels.cu:347-361) */
int tnetF_expand(float* y, const float* x, const int* off, TnetMatrixDim dout, TnetMatrixDim din, void* stream);
/* y[i,j] = x[i, copy_from[j]] (out of range -> +inf)            -- cudaF_rearrange (cukernels.cu:364-379) */
int tnetF_rearrange(float* y, const float* x, const int* copy_from, TnetMatrixDim dout, TnetMatrixDim din,
                    void* stream);
/* y[:, b*bo:(b+1)*bo] = x[:, b*bi:(b+1)*bi] . t for every block b, t = [bi x bo], one launch
 * -- CuMath::BlockLinearity (cumath.cc:76-113: one cublasSgemm per block), <blocklinearity>
 * (cuCRBEDctFeat.h:146-197); any strides/offsets */
int tnet_block_linearity(float* y, TnetMatrixDim dy, const float* x, TnetMatrixDim dx, const float* t,
                         TnetMatrixDim dt, void* stream);
/* y[i,:] = x[copy_from[i], :]                                    -- cudaF_randomize (cukernels.cu:382-393) */
int tnetF_randomize(float* y, const float* x, const int* copy_from, TnetMatrixDim dout, TnetMatrixDim din,
                    void* stream);
/* labels_out[i] = labels_in[copy_from[i]]  (class-id twin of randomize for one-hot targets) */
int tnet_gather_i32(int* out, const int* in, const int* copy_from, int n, void* stream);
/* both in one launch: y = rows copy_from[] of x, labels_out[i] = labels_in[copy_from[i]]
 * (CuCache::GetBunch's two _randomize calls, cuCache.cc:155-200, for a class-id target cache) */
int tnet_gather_bunch(float* y, const float* x, int* labels_out, const int* labels_in, const int* copy_from,
                      TnetMatrixDim dout, TnetMatrixDim din, void* stream);

/* ------------------------------------------------------------------------------------
 * GEMM (replaces cublasSgemm at cumatrix.tcc:336-370, row-major semantics)
 *   C[m x n] = alpha * op(A) * op(B) + beta * C,  op(X) = X or X^T ('N' / 'T')
 * fp32 in / fp32 accumulate on the f32 MFMA (v_mfma_f32_16x16x4_f32; exact f32 FMA chain per k).
 * Shapes with few output tiles and a long K (fewer than ~100 tiles, K >= 1024) are split over K:
 * the slices' partial products are added in slice order (deterministic) before the epilogue, by a
 * second launch.
 * Requirements: lda/ldb/ldc multiples of 4 elements, pointers 16-byte aligned.
 * ---------------------------------------------------------------------------------- */
int tnet_sgemm(char transa, char transb, int m, int n, int k, float alpha, const float* A, int lda,
               const float* B, int ldb, float beta, float* C, int ldc, void* stream);
/* Tuning knob: force one GEMM tile configuration for every later launch in this process
 * ("auto" = per-shape heuristic; names as in gemm_f32.hip, e.g. "m64x128k64s2"), optionally with a
 * forced split-K count ("m64x64k32s4w41+sk8") and a CU reservation ("+rsv<R>", as tnet_gemm_reserve;
 * sticky).  Not thread-safe. */
int tnet_gemm_config(const char* name);
/* R CUs held by another kernel while the caller's next GEMMs run (the data-parallel exchange sets it
 * while RCCL's collectives are in flight, 0 when they are done): the step's 64x128 backward / forward
 * and 128x128 gradient shapes then run as stream-K over CUs - R workgroups (gemm16_sk_kernel) instead of
 * a one-tile-per-CU grid whose last tiles would wait for a second round.  No reference counterpart
 * (the reference has no multi-GPU path).  Not thread-safe. */
int tnet_gemm_reserve(int cus);

/* ------------------------------------------------------------------------------------
 * Fused kernels of the MI355X SGD path (no reference counterpart: each replaces a chain of
 * reference calls, cited per function).
 * ---------------------------------------------------------------------------------- */
/* Y = act(X W + b), act = 0 none | 1 sigmoid | 2 negated (-(XW+b)) | 3 negated sigmoid.
 * X [rows x n_in], W [n_in x n_out] (memory layout of CuBiasedLinearity::mLinearity), b [n_out].
 * Replaces AddScaledRow + Gemm('N','N') + CuMath::Sigmoid (cuBiasedLinearity.cc:11-16,
 * cuActivation.cc:11-14; CuRbm::PropagateFnc cuRbm.cc:15-23). The negated forms write the RBM
 * negative-phase hidden statistics with the sign the fused update needs (tnet_rbm_update). */
int tnet_affine_fwd(const float* X, TnetMatrixDim dX, const float* W, TnetMatrixDim dW, const float* b,
                    float* Y, TnetMatrixDim dY, int act, void* stream);
/* Y = sigmoid(X W + b) and states = (Y > U), U the HybridTaus uniforms of the per-element generator
 * states z1..z4 (advanced in place; indexed row * dY.stride + col, as CuRand indexes them with the
 * probabilities' MatrixDim): the RBM positive phase + CuRand::BinarizeProbs (cuRbm.cc:15-23,
 * curand.tcc:121-134, curandkernels.cu:14-44, TRbmCu.cc:336-341) in one launch; the states are
 * bit-identical to tnet_affine_fwd(act 1) + tnet_rand_binarize. */
int tnet_affine_fwd_sample(const float* X, TnetMatrixDim dX, const float* W, TnetMatrixDim dW, const float* b,
                           float* Y, TnetMatrixDim dY, float* states, int ld_states, unsigned* z1, unsigned* z2,
                           unsigned* z3, unsigned* z4, void* stream);
/* Y = act(X W^T + b), act = 0 none | 1 sigmoid; X [rows x n_out], W [n_in x n_out], b [n_in].
 * Replaces CuRbm::Reconstruct (cuRbm.cc:117-128: AddScaledRow + Gemm('N','T') + Sigmoid). */
int tnet_affine_fwd_t(const float* X, TnetMatrixDim dX, const float* W, TnetMatrixDim dW, const float* b,
                      float* Y, TnetMatrixDim dY, int act, void* stream);
/* Eo = (E W^T) .* Ybelow (1 - Ybelow)  (dsig=1)  or  Eo = E W^T (dsig=0); Ybelow 16-byte aligned with a
 * stride that is a multiple of 4 (as the other operands).
 * Replaces Gemm('N','T') + CuMath::DiffSigmoid (cuBiasedLinearity.cc:21-25, cuActivation.cc:19-22). */
int tnet_affine_bwd(const float* E, TnetMatrixDim dE, const float* W, TnetMatrixDim dW, const float* Ybelow,
                    int strideYbelow, float* Eo, TnetMatrixDim dEo, int dsig, void* stream);
/* Fused weight update of CuBiasedLinearity::Update (cuBiasedLinearity.cc:46-64):
 *   G  = X^T E                       (X [rows x n_in], E [rows x n_out])
 *   C  = G + mmt * corrW             (corrW may be NULL when mmt == 0; then C = G)
 *   W  = W + scale * C ; W = W + l2 * W
 *   corrW = C                        (if corrW != NULL)
 * scale = -lr/N, l2 = -lr*wc*(gdf?1:rows) are computed by the caller. */
int tnet_affine_update(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* W,
                       TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                       void* stream);
/* ---- bias gradient fused into the GEMMs (removes the AddColSum pass over E and its two launches)
 * The error E_l of a hidden layer is produced by the backward GEMM of the layer above; that GEMM also
 * writes the column sums of E_l per 32-row slab.  The update GEMM of layer l then applies the bias SGD
 * of tnet_bias_update from those slab sums (fp32 within a slab, fp64 across slabs) in its prologue. */
/* number of 32-row slabs of a [rows x n] error matrix (rows of the colpart buffer) */
int tnet_colsum_slabs(int rows);
/* tnet_affine_bwd(..., dsig=1) plus colpart[s * ldcolpart + c] = sum_{r in slab s} Eo[r][c]
 * (cuBiasedLinearity.cc:21-25 + cuActivation.cc:19-22 + the AddColSum half of cuBiasedLinearity.cc:56). */
int tnet_affine_bwd_colsum(const float* E, TnetMatrixDim dE, const float* W, TnetMatrixDim dW,
                           const float* Ybelow, int strideYbelow, float* Eo, TnetMatrixDim dEo, float* colpart,
                           int ldcolpart, void* stream);
/* slab sums for an E that no backward GEMM produced (the top layer's softmax error): the same slab
 * count; the slabs are disjoint row ranges (32 rows when rows % 32 == 0) whose sum is colsum(E), which
 * is all tnet_affine_update_bias / tnet_affine_grad_bias use.  TNET_ERR_UNSUPPORTED above 8192 rows. */
int tnet_colsum_slab_sums(const float* E, TnetMatrixDim dE, float* colpart, int ldcolpart, void* stream);
/* The top layer for n_out <= TNET_AFFINE_SOFTMAX_MAX_N classes in two launches (the GEMM's K slices, then one workgroup per
 * 32-row slab): Z = X W + b (written when Z != NULL), Y = softmax(Z) (when Y != NULL), E = Y - onehot,
 * the statistics of tnet_softmax_xent, and (colpart != NULL) E's slab column sums for
 * tnet_affine_update_bias -- tnet_affine_fwd(act 0) + tnet_softmax_xent + tnet_colsum_slab_sums with
 * the same Z, Y, E per element (CuBiasedLinearity::PropagateFnc + CuSoftmax::PropagateFnc +
 * CuCrossEntropy::Evaluate, cuBiasedLinearity.cc:11-16, cuActivation.cc:28-31,
 * cuObjectiveFunction.cc:50-83).  TNET_ERR_UNSUPPORTED for more classes (use the three calls). */
#define TNET_AFFINE_SOFTMAX_MAX_N 256
int tnet_affine_softmax_xent(const float* X, TnetMatrixDim dX, const float* W, TnetMatrixDim dW, const float* b,
                             const int* labels, float* Z, int strideZ, float* Y, int strideY, float* E, int strideE,
                             double* stats, float* colpart, int ldcolpart, void* stream);
/* tnet_affine_update + tnet_bias_update(E, b, corr_b, scale, mmt) in one launch, colsum(E) taken from
 * colpart (written for E by tnet_affine_bwd_colsum); corr_b is required when mmt != 0
 * (cuBiasedLinearity.cc:46-64). */
int tnet_affine_update_bias(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* W,
                            TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                            const float* colpart, int ldcolpart, float* b, float* corr_b, void* stream);
/* tnet_affine_update_bias(X, E, W, ...) of layer l and tnet_affine_bwd_colsum(E2, W2, Ybelow, Eo,
 * colpart2) of layer l-1 in ONE launch (the two GEMMs are independent: CuNetwork::Backpropagate,
 * cuNetwork.h:170-194, runs layer l's Update after its backprop, and layer l-1's backprop reads only
 * W_{l-1}); same results as the two calls.  TNET_ERR_UNSUPPORTED when either GEMM would run another
 * tile configuration than the pair kernel's (the caller then makes the two calls). */
int tnet_affine_update_bwd_pair(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* W,
                                TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                                const float* colpart, int ldcolpart, float* b, float* corr_b, const float* E2,
                                TnetMatrixDim dE2, const float* W2, TnetMatrixDim dW2, const float* Ybelow,
                                int strideYbelow, float* Eo, TnetMatrixDim dEo, float* colpart2, int ldcolpart2,
                                void* stream);
/* Two tnet_affine_update_bias calls -- the updates of two layers (cuBiasedLinearity.cc:46-64) -- in ONE
 * launch; the two must be independent (distinct W, b and momentum buffers).  For small layers whose
 * tile grids together fit the CUs (CuNetwork runs the last two updates of a step this way, e.g. the
 * MLP3's 1024x135 and 598x1024): results identical to the two calls made with the same tile
 * configuration; TNET_ERR_UNSUPPORTED when the two grids do not fit one round (make the two calls). */
int tnet_affine_update_bias_pair(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* W,
                                 TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                                 const float* colpart, int ldcolpart, float* b, float* corr_b, const float* X2,
                                 TnetMatrixDim dX2, const float* E2, TnetMatrixDim dE2, float* W2, TnetMatrixDim dW2,
                                 float* corrW2, int strideCorr2, float scale2, float mmt2, float l22,
                                 const float* colpart2, int ldcolpart2, float* b2, float* corr_b2, void* stream);
/* tnet_affine_bwd_colsum(E, W, Ybelow, Eo, colpart) and tnet_colsum_slab_sums(E, colpartE) -- the top layer's
 * backward GEMM and the slab sums of its own input error (the softmax error: the top layer's bias gradient,
 * cuBiasedLinearity.cc:46-64 AddColSum) -- in ONE launch, the slab-sum blocks on the CUs the GEMM tiles free.
 * Results identical to the two calls; TNET_ERR_UNSUPPORTED where the backward would run another tile
 * configuration or the slab sums another form (make the two calls). */
int tnet_affine_bwd_colsum_slabs(const float* E, TnetMatrixDim dE, const float* W, TnetMatrixDim dW,
                                 const float* Ybelow, int strideYbelow, float* Eo, TnetMatrixDim dEo, float* colpart,
                                 int ldcolpart, float* colpartE, int ldcolpartE, void* stream);
/* ---- the backward GEMM from a transposed weight shadow (the same CuBiasedLinearity::BackpropagateFnc,
 * cuBiasedLinearity.cc:21-25, E_in = E W^T, read from Wt = W^T [n_out x n_in] so that the weight operand is
 * n-contiguous: the forward GEMM's NN layout and direct form instead of the NT one).  Eo is bit-identical to the
 * W forms (the same MFMA operands in the same order per element); the slab sums add the same rows in another
 * order (fp32, within the tests' slab-sum tolerance).  TNET_ERR_UNSUPPORTED while CUs are reserved for RCCL.
 *   tnet_weight_shadow(W, dW, Wt, ldwt): register Wt [dW.cols x dW.rows] (row stride ldwt, 16-B aligned) as the
 *     transposed shadow of W (Wt NULL: unregister).  Every update launch of W through tnet_affine_update[_bias],
 *     tnet_affine_update_bias_pair / _gather and tnet_affine_update_bwd_pair[_t] whose form runs the 16x16 kernel's
 *     SGD epilogue writes the updated W into Wt as well, in the same pass (16-B stores, written through);
 *     tnet_weight_shadow_kept(W) = 1 when the last such update of W did (0: it ran a form without the shadow
 *     store -- refresh Wt with tnet_transpose before reading it; < 0: W not registered).  W changed by any other
 *     means leaves Wt stale: the caller tracks that.
 *   tnet_transpose(A, dA, T, ldt): T[c][r] = A[r][c] (T [dA.cols x dA.rows], row stride ldt). */
int tnet_affine_bwd_colsum_t(const float* E, TnetMatrixDim dE, const float* Wt, TnetMatrixDim dWt, const float* Ybelow,
                             int strideYbelow, float* Eo, TnetMatrixDim dEo, float* colpart, int ldcolpart,
                             void* stream);
int tnet_affine_bwd_colsum_slabs_t(const float* E, TnetMatrixDim dE, const float* Wt, TnetMatrixDim dWt,
                                   const float* Ybelow, int strideYbelow, float* Eo, TnetMatrixDim dEo, float* colpart,
                                   int ldcolpart, float* colpartE, int ldcolpartE, void* stream);
int tnet_affine_update_bwd_pair_t(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* W,
                                  TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                                  const float* colpart, int ldcolpart, float* b, float* corr_b, const float* E2,
                                  TnetMatrixDim dE2, const float* W2t, TnetMatrixDim dW2t, const float* Ybelow,
                                  int strideYbelow, float* Eo, TnetMatrixDim dEo, float* colpart2, int ldcolpart2,
                                  void* stream);
int tnet_weight_shadow(const float* W, TnetMatrixDim dW, float* Wt, int ldwt);
int tnet_weight_shadow_kept(const float* W);
int tnet_transpose(const float* A, TnetMatrixDim dA, float* T, int ldt, void* stream);
/* The step's last weight update(s) and the NEXT bunch's gather in ONE launch: tnet_affine_update_bias(X, E,
 * W, ...) -- and, when X2 is not NULL, tnet_affine_update_bias(X2, E2, W2, ...) as in
 * tnet_affine_update_bias_pair -- plus tnet_gather_bunch(y, x, labels_out, labels_in, copy_from, dy, dx)
 * (CuCache::GetBunch of the bunch after this one, cuCache.cc:155-200) as extra workgroups on the CUs the
 * update's tiles leave free.  The gather must be independent of the updates (y / labels_out overlap none of
 * their operands -- TNET_ERR_ARG where y overlaps X, E, X2 or E2: the trainer gathers into the other half of a
 * double-buffered bunch).  Results identical
 * to the separate calls (the gather may also fill y's row padding up to the next multiple of 4 columns);
 * TNET_ERR_UNSUPPORTED when the updates would run another tile configuration alone, fewer than 8 CUs are
 * left for the gather, or the strides are not 16-B multiples (make the separate calls). */
int tnet_affine_update_bias_gather(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* W,
                                   TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                                   const float* colpart, int ldcolpart, float* b, float* corr_b, const float* X2,
                                   TnetMatrixDim dX2, const float* E2, TnetMatrixDim dE2, float* W2,
                                   TnetMatrixDim dW2, float* corrW2, int strideCorr2, float scale2, float mmt2,
                                   float l22, const float* colpart2, int ldcolpart2, float* b2, float* corr_b2,
                                   float* y, const float* x, int* labels_out, const int* labels_in,
                                   const int* copy_from, TnetMatrixDim dy, TnetMatrixDim dx, void* stream);
/* G = X^T E into a gradient buffer (data-parallel path: all-reduced before tnet_sgd_update). */
int tnet_affine_grad(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* G,
                     TnetMatrixDim dG, void* stream);
/* tnet_affine_grad + gradB = colsum(E) from the 32-row slab sums tnet_affine_bwd_colsum wrote for E
 * (data-parallel path: both gradients are all-reduced, then applied by tnet_sgd_update_multi). */
int tnet_affine_grad_bias(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* G,
                          TnetMatrixDim dG, const float* colpart, int ldcolpart, float* gradB, void* stream);
/* tnet_affine_grad_bias(X, E, G, colpart, gradB) and tnet_affine_bwd_colsum(E2, W2, Ybelow, Eo, colpart2) in ONE
 * launch (the data-parallel step's gradient of layer l -- cuBiasedLinearity.cc:46-64's GEMM and AddColSum written
 * to a buffer for the all-reduce -- and the backward GEMM of layer l-1, cuBiasedLinearity.cc:21-25, which reads
 * W_{l-1} only), tnet_affine_update_bwd_pair's form; results identical to the two calls.  TNET_ERR_ARG when an
 * output of one overlaps an operand of the other; TNET_ERR_UNSUPPORTED where either would run another
 * configuration alone, or while CUs are reserved for RCCL (tnet_gemm_reserve: make the two calls). */
int tnet_affine_grad_bwd_pair(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* G,
                              TnetMatrixDim dG, const float* colpart, int ldcolpart, float* gradB, const float* E2,
                              TnetMatrixDim dE2, const float* W2, TnetMatrixDim dW2, const float* Ybelow,
                              int strideYbelow, float* Eo, TnetMatrixDim dEo, float* colpart2, int ldcolpart2,
                              void* stream);
/* tnet_affine_grad_bias (X2 NULL) or two of them (X2, E2, G2, colpart2, gradB2: the step's last two gradients when
 * both 64x64 grids fit one round over the CUs) plus tnet_gather_bunch (the next bunch's CuCache::GetBunch,
 * cuCache.cc:155-200) on the CUs the gradient GEMMs' tiles leave free -- the data-parallel step's last gradient
 * launch, tnet_affine_update_bias_gather's form and rules: the gather independent of the GEMMs and the two GEMMs of
 * each other (TNET_ERR_ARG otherwise), TNET_ERR_UNSUPPORTED when the single GEMM would run another tile
 * configuration alone, the pair does not fit one round, or fewer than 8 CUs are left.  The two-GEMM form runs both
 * as unsplit 64x64 grids (sums in k order), also where the planner would split one of them over K alone: then
 * that gradient differs from tnet_affine_grad_bias's in fp32 summation order only (the fused step's update pair,
 * tnet_affine_update_bias_pair, has the same rule). */
int tnet_affine_grad_bias_gather(const float* X, TnetMatrixDim dX, const float* E, TnetMatrixDim dE, float* G,
                                 TnetMatrixDim dG, const float* colpart, int ldcolpart, float* gradB, const float* X2,
                                 TnetMatrixDim dX2, const float* E2, TnetMatrixDim dE2, float* G2, TnetMatrixDim dG2,
                                 const float* colpart2, int ldcolpart2, float* gradB2, float* y, const float* x,
                                 int* labels_out, const int* labels_in, const int* copy_from, TnetMatrixDim dy,
                                 TnetMatrixDim dx, void* stream);
/* Element-wise SGD of the same formula on flat arrays:  c = g + mmt*corr; p += scale*c; p += l2*p;
 * corr = c (corr may be NULL when mmt == 0). */
int tnet_sgd_update(float* p, const float* g, float* corr, long n, float scale, float mmt, float l2,
                    void* stream);
/* The same SGD over several flat segments in ONE launch (a layer's W and b after the all-reduce):
 * per segment k: c = g + mmt*corr; p += scale*c; p += l2_k*p; corr = c. */
typedef struct TnetSgdSeg_ {
  float* p;
  const float* g;
  float* corr; /* NULL when mmt == 0 */
  long n;
  float l2;
} TnetSgdSeg;
int tnet_sgd_update_multi(const TnetSgdSeg* segs, int nseg, float scale, float mmt, void* stream);
/* Bias update from the error matrix E (CuVector::AddColSum + AddScaled, cuBiasedLinearity.cc:56-59):
 *   c = colsum(E) + mmt*corr_b ; b += scale * c ; corr_b = c   (corr_b may be NULL if mmt == 0)
 * If grad_out != NULL the raw colsum is written there instead and b is not touched (DP path). */
int tnet_bias_update(const float* E, TnetMatrixDim dE, float* b, float* corr_b, float* grad_out, float scale,
                     float mmt, void* workspace, void* stream);
/* ---- RBM contrastive divergence (CuRbm::RbmUpdate, cuRbm.cc:133-174) ----------------------
 * V [2B x n_vis] = [pos_vis ; neg_vis] and H [2B x n_hid] = [pos_hid ; -neg_hid] row-stacked:
 *   corr = mmt*corr + scale*(V^T H) + l2*W ; W += corr
 * with scale = lr/B and l2 = -lr*wc.  One GEMM over K = 2B replaces the reference's two
 * Gemm('T','N') calls + AddScaled(-lr*wc) + AddScaled into W. */
int tnet_rbm_update(const float* V, TnetMatrixDim dV, const float* H, TnetMatrixDim dH, float* W,
                    TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                    void* stream);
/* RBM bias update (cuRbm.cc:148-164): rows from neg_from on enter negated,
 *   corr_b = mmt*corr_b + scale*(sum_{r<neg_from} M[r] - sum_{r>=neg_from} M[r]) ; b += corr_b. */
int tnet_rbm_bias_update(const float* M, TnetMatrixDim d, int neg_from, float* b, float* corr_b, float scale,
                         float mmt, void* workspace, void* stream);
/* tnet_rbm_update(V, H, W, corrW, scale, mmt, l2) and tnet_rbm_stats_update(V, H, B, vb, cvb, hb, chb, scale,
 * mmt, mse_stats) -- one TRbmCu step's CD-1 weight update and its bias updates + reconstruction MSE
 * (cuRbm.cc:133-174, TRbmCu.cc:350) -- in ONE launch (independent: both read the stacked statistics).
 * Results identical to the two calls; TNET_ERR_UNSUPPORTED where the update would not run the 64x64
 * configuration unsplit or the statistics kernel declines (make the two calls). */
int tnet_rbm_update_stats(const float* V, TnetMatrixDim dV, const float* H, TnetMatrixDim dH, float* W,
                          TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2, int B,
                          float* vb, float* cvb, float* hb, float* chb, double* mse_stats, void* stream);
/* tnet_rbm_update_stats and tnet_gather_bunch(y, x, labels_out, labels_in, copy_from, dy, dx) -- the NEXT
 * bunch's visible rows (CuCache::GetBunch, cuCache.cc:155-200) -- in ONE launch, the gather on CUs beside the
 * update's tiles.  y must lie outside V (TNET_ERR_ARG; the trainer double-buffers the visible statistics).
 * Results identical to the separate calls (y's row padding up to 4 columns may be written too);
 * TNET_ERR_UNSUPPORTED where tnet_rbm_update_stats declines, fewer than 16 CUs are left beside the tiles,
 * or the strides are not 16-B multiples (make the separate calls). */
int tnet_rbm_update_stats_gather(const float* V, TnetMatrixDim dV, const float* H, TnetMatrixDim dH, float* W,
                                 TnetMatrixDim dW, float* corrW, int strideCorr, float scale, float mmt, float l2,
                                 int B, float* vb, float* cvb, float* hb, float* chb, double* mse_stats, float* y,
                                 const float* x, int* labels_out, const int* labels_in, const int* copy_from,
                                 TnetMatrixDim dy, TnetMatrixDim dx, void* stream);
/* The CD-1 bias updates and reconstruction error of one RBM step in one launch (replaces the
 * AddColSum / AddScaled pairs of cuRbm.cc:148-164 and CuMeanSquareError::Evaluate of TRbmCu.cc:350):
 * Vs = [pos_vis; neg_vis] (2B x V), Hs = [pos_hid; -neg_hid] (2B x H, negative phase stored negated);
 *   c_v = mmt*c_v + scale*(sum pos_vis - sum neg_vis) ; vb += c_v
 *   c_h = mmt*c_h + scale*(sum of all rows of Hs)      ; hb += c_h
 *   mse_stats (nullable, stats layout as tnet_mse) += sum (neg_vis - pos_vis)^2.
 * Column sums bit-identical to tnet_rbm_bias_update; no workspace.  TNET_ERR_UNSUPPORTED for B > 4096. */
int tnet_rbm_stats_update(const float* Vs, TnetMatrixDim dV, const float* Hs, TnetMatrixDim dH, int B, float* vb,
                          float* cvb, float* hb, float* chb, float scale, float mmt, double* mse_stats, void* stream);

/* ---- single-frame kernels (TRecurrentCu: CuMath::OffsetGemv / BlasGer, cumath.cc:292-362) ---- */
/* single-frame forward of the recurrent layer: y = act(b + [v0, v1] W) for the row [v0 (K0), v1 (K1)]
 * read in place, also stored to vout (K0+K1 floats, NULL: not stored) -- CuRecurrent::Propagate's
 * history push + OffsetGemv (cuRecurrent.cc:26-47) in two launches; v1 may alias y. */
int tnet_gemv_rowvec_cat(const float* v0, int K0, const float* v1, int K1, float* vout, const float* W, int ldw,
                         const float* b, float* y, int N, int act, void* workspace, void* stream);
/* single-frame output layer + softmax + cross-entropy (CuBiasedLinearity::Propagate, CuSoftmax::
 * Propagate, CuCrossEntropy::EvaluateLabels for one row; TRecurrentCu.cc:360-368): z = b + v W,
 * y = softmax(z), e = y - onehot(*label), xent / correct added to stats slot 0.  z / y / e may be NULL.
 * N <= 4096 (else TNET_ERR_UNSUPPORTED); workspace: tnet_gemv_workspace(K, N) bytes. */
int tnet_gemv_rowvec_softmax_xent(const float* v, int K, const float* W, int ldw, const float* b, float* z, float* y,
                                  float* e, int N, const int* label, double* stats, void* workspace, void* stream);
/* ---- the TRecurrentCu frame chain (CuRecurrentTrainer's fused path) ----
 * [<recurrent> nIn->H, <biasedlinearity> H->N, <softmax>] + cross-entropy, one frame
 * (TRecurrentCu.cc:360-368 over cuRecurrent.cc:16-53 and cuBiasedLinearity.cc:11-64):
 *   tnet_gemv_rowvec_partial : split-K partials of [v0, v1] W (ceil(K/64) x N floats; vout: the
 *                              history row [v0, v1], NULL: not stored) -- CuRecurrent's forward,
 *                              without the sigmoid finish
 *   tnet_rnn_out_partial     : h = sigmoid(hb + sum of the hslices partials [hslices x H]) stored to h,
 *                              and the split-K partials of h Wo (ceil(H/64) x N floats)
 *   tnet_rnn_out_stats       : z = bo + sum of those partials (z may be NULL: not stored) and per 256
 *                              columns the pair {max z, sum exp(z - max)} into smx (2*ceil(N/256) doubles)
 *   tnet_rnn_out_full        : tnet_rnn_out_partial + tnet_rnn_out_stats in one launch without output
 *                              partials: every workgroup finishes all of h, then the complete z of 64
 *                              columns and their pair (2*ceil(N/64) doubles; H <= 2048, N <= 4096, else
 *                              TNET_ERR_UNSUPPORTED) -- the trainer's path
 *   tnet_gemv_rowvec_partial_update : tnet_gemv_rowvec_partial with the previous frame's recurrent
 *                              update (tnet_rnn_update's arguments and arithmetic per element) applied
 *                              to W as it is read -- the update's own launch folded into the next
 *                              frame's forward; needs steps < R (the history push must not overwrite a
 *                              row the update reads) and steps <= 9 (else TNET_ERR_UNSUPPORTED)
 *   tnet_rnn_out_bwd_update  : e = softmax(z) - onehot(*label) formed in place from z and the `pairs`
 *                              softmax pairs in smx (<= 64: ceil(N/256) from tnet_rnn_out_stats,
 *                              ceil(N/64) from tnet_rnn_out_full); with
 *                              train: the output layer's backprop + SGD of tnet_affine_bwd_update_row
 *                              (e_out = Wo e, d = e_out .* h (1 - h)); cross-entropy into stats slot 0;
 *                              the frame's argmax folded into *argkey (zero it first) by atomicMax of
 *                              {y bits << 32 | ~column}; y / e / e_out / d may be NULL
 *   tnet_argmax_correct      : frame accuracy of T frames from their argmax keys into stats slot 0 */
int tnet_gemv_rowvec_partial(const float* v0, int K0, const float* v1, int K1, float* vout, const float* W, int ldw,
                             int N, float* partial, void* stream);
int tnet_rnn_out_partial(const float* hpart, int hslices, const float* hb, float* h, int H, const float* Wo, int ldwo,
                         int N, float* opart, void* stream);
int tnet_rnn_out_stats(const float* opart, int H, int N, const float* bo, float* z, double* smx, void* stream);
int tnet_rnn_out_full(const float* hpart, int hslices, const float* hb, float* h, int H, const float* Wo, int ldwo,
                      int N, const float* bo, float* z, double* smx, void* stream);
int tnet_gemv_rowvec_partial_update(const float* v0, int K0, const float* v1, int K1, float* vout, float* W, int ldw,
                                    int N, float* partial, const float* hist, int ldh, int head, int R, const float* D,
                                    int ldd, int steps, float* b, float* corr_b, float lr, float mmt, float wc,
                                    void* stream);
int tnet_rnn_out_bwd_update(const float* z, const double* smx, int pairs, int N, const int* label, const float* h,
                            int H, float* Wo, int ldwo, float* corrWo, int ldc, float* bo, float* corr_bo, float scale,
                            float mmt, float l2, float* y, float* e, float* e_out, float* d, double* stats,
                            unsigned long long* argkey, int train, void* stream);
int tnet_argmax_correct(const unsigned long long* keys, const int* labels, int T, int N, double* stats,
                        void* stream);
/* The look-ahead form of the chain (frames after an utterance's first; TNET_RNN_AHEAD=0: off).  The next frame's
 * recurrent forward needs W_{t+1} = W_t + corr (cuRecurrent.cc:88-153), which exists only after this frame's BPTT;
 * with v = [x_{t+1}, y_t], v W_{t+1} = (1 - lr wc) (v W_t) + sum_i (-lr (v . h_i)) d_i, so:
 *   tnet_rnn_out_bwd_update_ahead : tnet_rnn_out_bwd_update (train) plus, in the same launch, the copy of the
 *                              recurrent bias / momentum computed by the previous tnet_rnn_out_full_ahead (bnext,
 *                              cbnext -> b, cb; bnext NULL: none) and (x_next != NULL) the next frame's look-ahead:
 *                              the split-K partials of [x_next, h] W_t (tnet_gemv_rowvec_partial's), the dots
 *                              [x_next, h] . h_i with the history rows (head + i) % R, i < steps, as
 *                              dpart [ceil(K/64) x 16] partials, and the push of [x_next, h] into vout
 *   tnet_rnn_out_full_ahead  : tnet_rnn_out_full with h = sigmoid(b' + (1 - lr wc) sum(hpart) + sum_i (-lr dot_i)
 *                              d_i) -- b' the bias after the pending update (bnext / cbnext written, the
 *                              tnet_rnn_update chain) -- and that update of W (rows x H, tnet_rnn_update's
 *                              per-element arithmetic with history head / R and d_i = D rows) in extra workgroups
 * The recurrent output differs from the materialised product by fp32 reassociation only (test_gpu_rnn.py). */
int tnet_rnn_out_full_ahead(const float* hpart, int hslices, const float* hb, float* h, int H, const float* Wo,
                            int ldwo, int N, const float* bo, float* z, double* smx, const float* dpart, const float* D,
                            int ldd, int steps, float lr, float mmt, float wc, const float* cb, float* bnext,
                            float* cbnext, float* W, int ldw, int rows, const float* hist, int ldh, int head, int R,
                            void* stream);
int tnet_rnn_out_bwd_update_ahead(const float* z, const double* smx, int pairs, int N, const int* label,
                                  const float* h, int H, float* Wo, int ldwo, float* corrWo, int ldc, float* bo,
                                  float* corr_bo, float scale, float mmt, float l2, float* e, float* eo, float* d,
                                  double* stats, unsigned long long* argkey, const float* bnext, const float* cbnext,
                                  float* b, float* cb, const float* x_next, int nIn, const float* W, int ldw,
                                  float* partial, float* dpart, float* vout, const float* hist, int ldh, int head,
                                  int R, int steps, void* stream);
/* single-frame CuBiasedLinearity::Backpropagate + Update (cuBiasedLinearity.cc:32-64) in one pass
 * over W: e_out = W e (with the weights before the update), then the update of
 * tnet_affine_update_row; with s != NULL also d_out = e_out .* s (1 - s) (the diff-sigmoid of a
 * recurrent layer below).  e_out / d_out may be NULL. */
int tnet_affine_bwd_update_row(const float* x, int n_in, const float* e, int n_out, float* W, int ldw, float* corrW,
                               int ldc, float* b, float* corr_b, float scale, float mmt, float l2, float* e_out,
                               const float* s, float* d_out, void* stream);
/* one frame's tnet_affine_update + tnet_bias_update in one launch (the output layer of TRecurrentCu,
 * cuBiasedLinearity.cc:46-64 with one row): c = x_i e_j (+ mmt corrW); W += scale c; W += l2 W;
 * b += scale (e_j + mmt corr_b). corrW / corr_b may be NULL when mmt == 0. */
int tnet_affine_update_row(const float* x, int n_in, const float* e, int n_out, float* W, int ldw, float* corrW,
                           int ldc, float* b, float* corr_b, float scale, float mmt, float l2, void* stream);
/* workspace bytes for tnet_gemv_rowvec */
long tnet_gemv_workspace(int K, int N);
/* y[0:N] = act(b + v[0:K] W), W [K x N] row-major (ld ldw), act 0 none | 1 sigmoid; b may be NULL.
 * Split-K over many workgroups, fixed-order partials in `workspace`. */
int tnet_gemv_rowvec(const float* v, int K, const float* W, int ldw, const float* b, float* y, int N, int act,
                     void* workspace, void* stream);
/* y[r] = beta*y[r] + W[r0 + r, 0:n] . x  for r < nrows, then y[r] *= s[r](1 - s[r]) if s != NULL
 * (OffsetGemv('N') with the row offset, and the fused diff-sigmoid of the BPTT step). */
int tnet_gemv_rows(const float* W, int ldw, int r0, int nrows, int n, const float* x, float* y, float beta,
                   const float* s, void* stream);
/* CuRecurrent::Update weight/bias step (cuRecurrent.cc:88-153) in one pass over W [rows x nout]:
 *   corr = sum_{i<steps} (-lr h_i) (x) d_i ; corr += -lr*wc*W ; W += corr
 *   cb = -lr d_0 + mmt*cb ; cb = -lr d_i + cb (i >= 1) ; b += cb
 * h_i = row (head + i) % R of the history ring hist [R x rows], d_i = row i of D. */
int tnet_rnn_update(float* W, int ldw, int rows, int nout, const float* hist, int ldh, int head, int R,
                    const float* D, int ldd, int steps, float* b, float* corr_b, float lr, float mmt, float wc,
                    void* stream);

/* ---- per-element HybridTaus random numbers (CuRand, curand.tcc / curandkernels.cu) ----------
 * z1..z4: four uint32 state arrays with the element layout of the target matrix (index =
 * col + row*stride), seeded by the caller with lrand48() values > 128 (curand.tcc:36-45) and
 * advanced in place. */
/* mat = U(0,1) (cudaF_rand, curandkernels.cu:46-52) */
int tnetF_rand(float* mat, TnetMatrixDim d, unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4, void* stream);
/* mat = N(0,1) by Box-Muller (cudaF_gauss_rand, curandkernels.cu:69-77) */
int tnetF_gauss_rand(float* mat, TnetMatrixDim d, unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4,
                     void* stream);
/* states = probs > rnd ? 1 : 0 (cudaF_binarize_probs, curandkernels.cu:80-88) */
int tnetF_binarize_probs(float* states, const float* probs, const float* rnd, TnetMatrixDim d, void* stream);
/* states = probs > U(0,1) ? 1 : 0 in one pass (CuRand::BinarizeProbs = Rand + binarize,
 * curand.tcc:121-134); d describes probs and the state arrays. */
int tnet_rand_binarize(float* states, int ld_states, const float* probs, TnetMatrixDim d, unsigned* z1,
                       unsigned* z2, unsigned* z3, unsigned* z4, void* stream);
/* mat += scale * N(0,1) (CuRand::AddGaussNoise, curand.tcc:55-60) */
int tnet_add_gauss_noise(float* mat, TnetMatrixDim d, float scale, unsigned* z1, unsigned* z2, unsigned* z3,
                         unsigned* z4, void* stream);

/* Fused softmax + cross-entropy + error + accuracy for class-id targets
 * (CuSoftmax::PropagateFnc + CuCrossEntropy::Evaluate, cuActivation.cc:28-31,
 *  cuObjectiveFunction.cc:50-83; kernels _softmax, _add_scaled, _check_class, _log_elem,
 *  _mul_elem, _add_col_sum):
 *   y = softmax(Z row)          -> written to Y if Y != NULL
 *   E = y - onehot(label)       (label < 0: all-zero target row)
 *   xent += -log(max(y[label], FLT_MIN)), correct += #(argmax y == argmax target)
 *   stats: device array of TNET_STATS_WORDS doubles (or NULL), accumulated without contention:
 *   workgroup w adds its rows into slot (w % TNET_STATS_SLOTS); totals are
 *   xent = sum_i stats[2i], correct = sum_i stats[2i+1] (tnet_stats_fetch).
 * Z == NULL: Y already holds the network output (softmax not recomputed). */
int tnet_softmax_xent(const float* Z, TnetMatrixDim dZ, const int* labels, float* Y, int strideY, float* E,
                      int strideE, double* stats, void* stream);
/* Same objective for dense desired matrices D (any soft targets; cuObjectiveFunction.cc:50-83):
 * Y = softmax(Z) (if Z != NULL, else Y already holds the network output), E = Y - D, stats as above
 * with xent = -sum D log(max(Y, FLT_MIN)). */
int tnet_softmax_xent_dense(const float* Z, TnetMatrixDim dZ, const float* D, int strideD, float* Y,
                            int strideY, float* E, int strideE, double* stats, void* stream);
/* Mean-square-error objective (CuMeanSquareError::Evaluate, cuObjectiveFunction.cc:28-45):
 * E = Y - D, error += sum E^2 (stats layout as above). */
int tnet_mse(const float* Y, TnetMatrixDim dY, const float* D, int strideD, float* E, int strideE,
             double* stats, void* stream);
/* Synchronous read-back of a stats accumulator: totals of the error and correct slots. */
int tnet_stats_fetch(const double* stats, double* error, double* correct, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TNET_KERNELS_H_ */
