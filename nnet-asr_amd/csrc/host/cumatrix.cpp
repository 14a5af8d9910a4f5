// cumatrix.cpp -- float math of CuMatrix / CuVector and the CuMath statics, all on the HIP kernels
// of include/tnet_kernels.h (reference: src/CuBaseLib/cumatrix.tcc:193-423, cuvector.tcc:129-191,
// cumath.cc:13-206).
#include "cumath.h"

namespace TNet {

#define PROF(name) CuProfileScope _prof(name)
#define S ((void*)CuDevice::Instantiate().Stream())

template <>
void CuMatrix<BaseFloat>::SetConst(BaseFloat value) {
  PROF("CuMatrix::SetConst");
  TNET_SAFE_CALL(tnetF_set_const(mpCUData, value, Dim(), S));
}
template <>
void CuMatrix<BaseFloat>::ApplyLog() {
  PROF("CuMatrix::ApplyLog");
  TNET_SAFE_CALL(tnetF_apply_log(mpCUData, Dim(), S));
}
template <>
void CuMatrix<BaseFloat>::ApplyMask(const CuMatrix<BaseFloat>& mask) {
  PROF("CuMatrix::ApplyMask");
  assert(mask.Rows() == Rows() && mask.Cols() == Cols());
  TNET_SAFE_CALL(tnetF_apply_mask(mpCUData, mask.pCUData(), Dim(), mask.Dim(), S));
}
template <>
void CuMatrix<BaseFloat>::ApplyL1(BaseFloat l1) {
  PROF("CuMatrix::ApplyL1");
  TNET_SAFE_CALL(tnetF_apply_l1(mpCUData, l1, Dim(), S));
}
template <>
void CuMatrix<BaseFloat>::ScaleCols(const CuVector<BaseFloat>& scale) {
  PROF("CuMatrix::ScaleCols");
  assert(scale.Dim() == Cols());
  TNET_SAFE_CALL(tnetF_scale_cols(mpCUData, scale.pCUData(), Dim(), S));
}
template <>
void CuMatrix<BaseFloat>::ScaleRows(const CuVector<BaseFloat>& scale) {
  PROF("CuMatrix::ScaleRows");
  assert(scale.Dim() == Rows());
  TNET_SAFE_CALL(tnetF_scale_rows(mpCUData, scale.pCUData(), Dim(), S));
}
template <>
void CuMatrix<BaseFloat>::AddScaled(BaseFloat alpha, const CuMatrix<BaseFloat>& A, BaseFloat beta) {
  PROF("CuMatrix::AddScaled");
  assert(A.Rows() == Rows() && A.Cols() == Cols());
  TNET_SAFE_CALL(tnetF_add_scaled(alpha, A.pCUData(), (int)A.Stride(), beta, mpCUData, Dim(), S));
}
template <>
void CuMatrix<BaseFloat>::AddScaledRow(BaseFloat alpha, const CuVector<BaseFloat>& row, BaseFloat beta) {
  PROF("CuMatrix::AddScaledRow");
  if (row.Dim() != Cols()) Error("CuMatrix::AddScaledRow: non matching dimensions");
  TNET_SAFE_CALL(tnetF_add_scaled_row(alpha, row.pCUData(), beta, mpCUData, Dim(), S));
}
template <>
void CuMatrix<BaseFloat>::Gemm(char transa, char transb, BaseFloat alpha, const CuMatrix<BaseFloat>& A,
                               const CuMatrix<BaseFloat>& B, BaseFloat beta) {
  PROF("CuMatrix::Gemm");
  // C[m x n] = alpha op(A) op(B) + beta C   (cumatrix.tcc:336-370)
  const bool ta = (transa == 'T' || transa == 't'), tb = (transb == 'T' || transb == 't');
  const size_t m = ta ? A.Cols() : A.Rows(), k = ta ? A.Rows() : A.Cols();
  const size_t kb = tb ? B.Cols() : B.Rows(), n = tb ? B.Rows() : B.Cols();
  if (k != kb || m != Rows() || n != Cols()) Error("CuMatrix::Gemm: non matching dimensions");
  TNET_SAFE_CALL(tnet_sgemm(transa, transb, (int)m, (int)n, (int)k, alpha, A.pCUData(), (int)A.Stride(),
                            B.pCUData(), (int)B.Stride(), beta, mpCUData, (int)mStride, S));
}
template <>
void CuMatrix<BaseFloat>::MulElem(const CuMatrix<BaseFloat>& A) {
  PROF("CuMatrix::MulElem");
  assert(A.Rows() == Rows() && A.Cols() == Cols());
  TNET_SAFE_CALL(tnetF_mul_elem(mpCUData, A.pCUData(), (int)A.Stride(), Dim(), S));
}
template <>
void CuMatrix<BaseFloat>::LogElem() {
  PROF("CuMatrix::LogElem");
  TNET_SAFE_CALL(tnetF_log_elem(mpCUData, Dim(), S));
}

template <>
void CuVector<BaseFloat>::SetConst(BaseFloat value) {
  TNET_SAFE_CALL(tnetF_set_const(mpCUData, value, MatDim(), S));
}
template <>
void CuVector<BaseFloat>::AddScaled(BaseFloat alpha, const CuVector<BaseFloat>& vec, BaseFloat beta) {
  PROF("CuVector::AddScaled");
  assert(vec.Dim() == Dim());
  TNET_SAFE_CALL(tnetF_add_scaled(alpha, vec.pCUData(), (int)Dim(), beta, mpCUData, MatDim(), S));
}
template <>
void CuVector<BaseFloat>::AddColSum(BaseFloat alpha, const CuMatrix<BaseFloat>& mat, BaseFloat beta) {
  PROF("CuVector::AddColSum");
  if (mat.Cols() != Dim()) Error("CuVector::AddColSum: non matching dimensions");
  TnetMatrixDim d = mat.Dim();
  void* ws = CuDevice::Instantiate().Workspace((size_t)tnet_col_sum_workspace(d));
  TNET_SAFE_CALL(tnetF_add_col_sum(alpha, mat.pCUData(), beta, mpCUData, d, ws, S));
}

// ---------------------------------------------------------------------------------- CuMath
void CuMath<BaseFloat>::Sigmoid(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X) {
  PROF("CuMath::Sigmoid");
  assert(Y.Rows() == X.Rows() && Y.Cols() == X.Cols() && Y.Stride() == X.Stride());
  TNET_SAFE_CALL(tnetF_sigmoid(Y.pCUData(), X.pCUData(), X.Dim(), S));
}
void CuMath<BaseFloat>::DiffSigmoid(CuMatrix<BaseFloat>& Eout, const CuMatrix<BaseFloat>& Ein,
                                    const CuMatrix<BaseFloat>& Y) {
  PROF("CuMath::DiffSigmoid");
  assert(Eout.Rows() == Ein.Rows() && Ein.Rows() == Y.Rows() && Eout.Cols() == Y.Cols());
  TNET_SAFE_CALL(tnetF_diff_sigmoid(Eout.pCUData(), Ein.pCUData(), Y.pCUData(), Y.Dim(), S));
}
void CuMath<BaseFloat>::Softmax(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X) {
  PROF("CuMath::Softmax");
  assert(Y.Rows() == X.Rows() && Y.Cols() == X.Cols() && Y.Stride() == X.Stride());
  TNET_SAFE_CALL(tnetF_softmax(Y.pCUData(), X.pCUData(), X.Dim(), S));
}
void CuMath<BaseFloat>::BlockLinearity(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X,
                                       const CuMatrix<BaseFloat>& block_transf) {
  PROF("CuMath::BlockLinearity");
  // Y[:, b*bo:(b+1)*bo] = X[:, b*bi:(b+1)*bi] * T  for every block b (cumath.cc:78-113)
  const size_t bi = block_transf.Rows(), bo = block_transf.Cols();
  if (X.Cols() % bi != 0 || Y.Cols() != X.Cols() / bi * bo || X.Rows() != Y.Rows())
    Error("CuMath::BlockLinearity: non matching dimensions");
  // all blocks in one launch (the reference: one cublasSgemm per block)
  TNET_SAFE_CALL(tnet_block_linearity(Y.pCUData(), Y.Dim(), X.pCUData(), X.Dim(), block_transf.pCUData(),
                                      block_transf.Dim(), S));
}
void CuMath<BaseFloat>::Expand(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X,
                               const CuVector<int>& frameOffsets) {
  PROF("CuMath::Expand");
  assert(Y.Cols() == X.Cols() * frameOffsets.Dim() && Y.Rows() == X.Rows());
  TNET_SAFE_CALL(tnetF_expand(Y.pCUData(), X.pCUData(), frameOffsets.pCUData(), Y.Dim(), X.Dim(), S));
}
void CuMath<BaseFloat>::Rearrange(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X,
                                  const CuVector<int>& copyFrom) {
  PROF("CuMath::Rearrange");
  assert(copyFrom.Dim() == Y.Cols() && Y.Rows() == X.Rows());
  TNET_SAFE_CALL(tnetF_rearrange(Y.pCUData(), X.pCUData(), copyFrom.pCUData(), Y.Dim(), X.Dim(), S));
}
void CuMath<BaseFloat>::Randomize(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X,
                                  const CuVector<int>& copyFrom) {
  PROF("CuMath::Randomize");
  assert(X.Cols() == Y.Cols() && copyFrom.Dim() <= Y.Rows());
  TnetMatrixDim dout = Y.Dim();
  dout.rows = (int)copyFrom.Dim();
  TNET_SAFE_CALL(tnetF_randomize(Y.pCUData(), X.pCUData(), copyFrom.pCUData(), dout, X.Dim(), S));
}
void CuMath<BaseFloat>::CheckClass(const CuMatrix<BaseFloat>& out, const CuMatrix<BaseFloat>& des,
                                   CuVector<int>& match) {
  PROF("CuMath::CheckClass");
  assert(out.Rows() == des.Rows() && out.Cols() == des.Cols() && out.Stride() == des.Stride());
  match.Init(out.Rows());
  TNET_SAFE_CALL(tnetF_check_class(out.pCUData(), des.pCUData(), match.pCUData(), out.Dim(), S));
}

}  // namespace TNet
