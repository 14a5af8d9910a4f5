// cumatrix.h -- CuMatrix / CuVector: owning pitched device containers of the MI355X TNet library.
//
// Source-compatible counterpart of src/CuBaseLib/cumatrix.h:18-181 and cuvector.h:13-85:
// same method names and semantics (Init is a no-op when the dimensions are unchanged and zeroes
// new memory, cumatrix.tcc:15-35; row-major, stride padded).  Every operation is enqueued on the
// CuDevice stream and calls the HIP kernels through the C ABI (include/tnet_kernels.h); nothing
// synchronises except the explicit host copies (CopyTo / CopyFrom(host)).
//
// Layout for MI355X: stride padded to a multiple of 64 elements (256 B), so every row starts
// 256-B aligned (float4 / dwordx4 accesses, whole 128-B lines) -- the reference's
// cudaMallocPitch pitch is 512 B.  Copying a CuMatrix would double-free, so copies are deleted.
#pragma once

#include <cassert>
#include <cmath>
#include <cstdint>
#include <iostream>
#include <sstream>
#include <type_traits>

#include "cudevice.h"
#include "hostmatrix.h"

namespace TNet {

template <typename T>
class CuVector;

inline size_t tnet_pad_stride(size_t cols) { return cols == 0 ? 0 : ((cols + 63) / 64) * 64; }

template <typename T>
class CuMatrix {
 public:
  CuMatrix() {}
  CuMatrix(size_t rows, size_t cols) { Init(rows, cols); }
  ~CuMatrix() { Destroy(); }
  CuMatrix(const CuMatrix&) = delete;
  CuMatrix& operator=(const CuMatrix&) = delete;

  size_t Rows() const { return mRows; }
  size_t Cols() const { return mCols; }
  size_t Stride() const { return mStride; }
  TnetMatrixDim Dim() const { return TnetMatrixDim{(int)mRows, (int)mCols, (int)mStride}; }
  const T* pCUData() const { return mpCUData; }
  T* pCUData() { return mpCUData; }
  const T* pCURowData(size_t r) const { return mpCUData + r * mStride; }
  T* pCURowData(size_t r) { return mpCUData + r * mStride; }
  size_t MSize() const { return mRows * mStride * sizeof(T); }
  size_t MRowSize() const { return mStride * sizeof(T); }

  /// Non-owning view of caller memory (C ABI / FFI boundary); stride in elements.
  static void MakeView(CuMatrix& m, T* data, size_t rows, size_t cols, size_t stride) {
    m.Destroy();
    m.mpCUData = data;
    m.mRows = rows;
    m.mCols = cols;
    m.mStride = stride;
    m.mBytes = 0;
    m.mView = true;
  }
  bool IsView() const { return mView; }

  /// (Re)allocate; no-op if the dimensions are unchanged (cumatrix.tcc:20-23); new memory zeroed.
  CuMatrix& Init(size_t rows, size_t cols) {
    if (mRows == rows && mCols == cols && (mpCUData || rows * cols == 0)) return *this;
    if (mView) Error("CuMatrix::Init: cannot resize a view of external memory");
    Destroy();
    if (rows * cols == 0) {
      mRows = rows; mCols = cols; mStride = tnet_pad_stride(cols);
      return *this;
    }
    CuDevice& dev = CuDevice::Instantiate();
    mStride = tnet_pad_stride(cols);
    mBytes = rows * mStride * sizeof(T);
    mpCUData = (T*)dev.Alloc(mBytes);
    TNET_HIP_CALL(hipMemsetAsync(mpCUData, 0, mBytes, dev.Stream()));
    mRows = rows;
    mCols = cols;
    return *this;
  }
  void Destroy() {
    if (mpCUData && !mView) CuDevice::Instantiate().Free(mpCUData, mBytes);
    mpCUData = nullptr;
    mRows = mCols = mStride = 0;
    mBytes = 0;
    mView = false;
  }

  CuMatrix& CopyFrom(const CuMatrix<T>& src) {
    Init(src.Rows(), src.Cols());
    if (mRows * mCols)
      TNET_HIP_CALL(hipMemcpy2DAsync(mpCUData, mStride * sizeof(T), src.pCUData(), src.Stride() * sizeof(T),
                                     mCols * sizeof(T), mRows, hipMemcpyDeviceToDevice, Stream()));
    return *this;
  }
  CuMatrix& CopyFrom(const Matrix<T>& src) {
    Init(src.Rows(), src.Cols());
    if (mRows * mCols) {
      TNET_HIP_CALL(hipMemcpy2DAsync(mpCUData, mStride * sizeof(T), src.pData(), src.Stride() * sizeof(T),
                                     mCols * sizeof(T), mRows, hipMemcpyHostToDevice, Stream()));
      TNET_HIP_CALL(hipStreamSynchronize(Stream()));  // host buffer may go away
    }
    return *this;
  }
  /// Host -> device from a raw row-major buffer (rows x cols, leading dimension ld).
  CuMatrix& CopyFromHost(const T* src, size_t rows, size_t cols, size_t ld, bool sync = true) {
    Init(rows, cols);
    if (rows * cols) {
      TNET_HIP_CALL(hipMemcpy2DAsync(mpCUData, mStride * sizeof(T), src, ld * sizeof(T), cols * sizeof(T), rows,
                                     hipMemcpyHostToDevice, Stream()));
      if (sync) TNET_HIP_CALL(hipStreamSynchronize(Stream()));
    }
    return *this;
  }
  Matrix<T>& CopyTo(Matrix<T>& dst) const {
    if (dst.Rows() != mRows || dst.Cols() != mCols) dst.Init(mRows, mCols);
    CopyToHost(dst.pData(), dst.Stride());
    return dst;
  }
  void CopyToHost(T* dst, size_t ld) const {
    if (mRows * mCols) {
      TNET_HIP_CALL(hipMemcpy2DAsync(dst, ld * sizeof(T), mpCUData, mStride * sizeof(T), mCols * sizeof(T), mRows,
                                     hipMemcpyDeviceToHost, Stream()));
      TNET_HIP_CALL(hipStreamSynchronize(Stream()));
    }
  }
  /// rows [srcOri, srcOri+rowCnt) of src -> rows [dstOri, ...) of this (cumatrix.tcc:120-150)
  void CopyRows(size_t rowCnt, size_t srcOri, const CuMatrix<T>& src, size_t dstOri) {
    assert(rowCnt + srcOri <= src.Rows() && rowCnt + dstOri <= Rows() && Cols() == src.Cols());
    if (!rowCnt || !mCols) return;
    TNET_HIP_CALL(hipMemcpy2DAsync(pCURowData(dstOri), mStride * sizeof(T), src.pCURowData(srcOri),
                                   src.Stride() * sizeof(T), mCols * sizeof(T), rowCnt, hipMemcpyDeviceToDevice,
                                   Stream()));
  }
  /// cols [srcOri, srcOri+colCnt) of src -> cols [dstOri, ...) of this (cumatrix.tcc:153-183)
  void CopyCols(size_t colCnt, size_t srcOri, const CuMatrix<T>& src, size_t dstOri) {
    assert(colCnt + srcOri <= src.Cols() && colCnt + dstOri <= Cols() && Rows() == src.Rows());
    if (!colCnt || !mRows) return;
    TNET_HIP_CALL(hipMemcpy2DAsync(mpCUData + dstOri, mStride * sizeof(T), src.pCUData() + srcOri,
                                   src.Stride() * sizeof(T), colCnt * sizeof(T), mRows, hipMemcpyDeviceToDevice,
                                   Stream()));
  }
  void SetZero() {
    if (mpCUData) TNET_HIP_CALL(hipMemsetAsync(mpCUData, 0, mBytes, Stream()));
  }

  // ---- float math (cumatrix.tcc:193-423)
  void SetConst(T value);
  void ApplyLog();
  void ApplyMask(const CuMatrix<BaseFloat>& mask);
  void ApplyL1(BaseFloat l1);
  void ScaleCols(const CuVector<T>& scale);
  void ScaleRows(const CuVector<T>& scale);
  void AddScaled(T alpha, const CuMatrix<T>& A, T beta);
  void AddScaledRow(T alpha, const CuVector<T>& row, T beta);
  void Gemm(char transa, char transb, T alpha, const CuMatrix<T>& A, const CuMatrix<T>& B, T beta);
  void MulElem(const CuMatrix<T>& A);
  void LogElem();

  void Print() const {
    Matrix<T> m;
    CopyTo(m);
    std::cout << m;
  }
  void CheckData() const {
    Matrix<T> m;
    CopyTo(m);
    for (size_t i = 0; i < Rows(); i++)
      for (size_t j = 0; j < Cols(); j++)
        if (std::isnan((double)m(i, j)) || std::isinf((double)m(i, j))) {
          std::ostringstream os;
          os << "Invalid value:" << m(i, j) << "at row" << i << " col" << j << "\n";
          Error(os.str());
        }
  }

  static hipStream_t Stream() { return CuDevice::Instantiate().Stream(); }

 private:
  size_t mRows = 0, mCols = 0, mStride = 0, mBytes = 0;
  T* mpCUData = nullptr;
  bool mView = false;

 public:
  /// exchange the storage of two matrices (double buffers)
  void Swap(CuMatrix& o) {
    std::swap(mRows, o.mRows);
    std::swap(mCols, o.mCols);
    std::swap(mStride, o.mStride);
    std::swap(mBytes, o.mBytes);
    std::swap(mpCUData, o.mpCUData);
    std::swap(mView, o.mView);
  }
};

template <typename T>
class CuVector {
 public:
  CuVector() {}
  explicit CuVector(size_t dim) { Init(dim); }
  ~CuVector() { Destroy(); }
  CuVector(const CuVector&) = delete;
  CuVector& operator=(const CuVector&) = delete;

  size_t Dim() const { return mDim; }
  TnetMatrixDim MatDim() const { return TnetMatrixDim{1, (int)mDim, (int)mDim}; }
  const T* pCUData() const { return mpCUData; }
  T* pCUData() { return mpCUData; }

  static void MakeView(CuVector& v, T* data, size_t dim) {
    v.Destroy();
    v.mpCUData = data;
    v.mDim = dim;
    v.mView = true;
  }

  CuVector& Init(size_t dim) {
    if (mDim == dim && (mpCUData || dim == 0)) return *this;
    if (mView) Error("CuVector::Init: cannot resize a view of external memory");
    Destroy();
    if (!dim) return *this;
    CuDevice& dev = CuDevice::Instantiate();
    mBytes = ((dim + 63) / 64) * 64 * sizeof(T);
    mpCUData = (T*)dev.Alloc(mBytes);
    TNET_HIP_CALL(hipMemsetAsync(mpCUData, 0, mBytes, dev.Stream()));
    mDim = dim;
    return *this;
  }
  void Destroy() {
    if (mpCUData && !mView) CuDevice::Instantiate().Free(mpCUData, mBytes);
    mpCUData = nullptr;
    mDim = 0;
    mBytes = 0;
    mView = false;
  }
  CuVector& CopyFrom(const CuVector<T>& src) {
    Init(src.Dim());
    if (mDim)
      TNET_HIP_CALL(hipMemcpyAsync(mpCUData, src.pCUData(), mDim * sizeof(T), hipMemcpyDeviceToDevice, Stream()));
    return *this;
  }
  CuVector& CopyFrom(const Vector<T>& src) { return CopyFromHost(src.pData(), src.Dim()); }
  CuVector& CopyFromHost(const T* src, size_t n, bool sync = true) {
    Init(n);
    if (n) {
      TNET_HIP_CALL(hipMemcpyAsync(mpCUData, src, n * sizeof(T), hipMemcpyHostToDevice, Stream()));
      if (sync) TNET_HIP_CALL(hipStreamSynchronize(Stream()));
    }
    return *this;
  }
  Vector<T>& CopyTo(Vector<T>& dst) const {
    if (dst.Dim() != mDim) dst.Init(mDim);
    CopyToHost(dst.pData());
    return dst;
  }
  void CopyToHost(T* dst) const {
    if (mDim) {
      TNET_HIP_CALL(hipMemcpyAsync(dst, mpCUData, mDim * sizeof(T), hipMemcpyDeviceToHost, Stream()));
      TNET_HIP_CALL(hipStreamSynchronize(Stream()));
    }
  }
  void SetZero() {
    if (mpCUData) TNET_HIP_CALL(hipMemsetAsync(mpCUData, 0, mBytes, Stream()));
  }
  void SetConst(T value);
  void AddScaled(T alpha, const CuVector<T>& vec, T beta);
  void AddColSum(T alpha, const CuMatrix<T>& mat, T beta);

  static hipStream_t Stream() { return CuDevice::Instantiate().Stream(); }

 private:
  size_t mDim = 0, mBytes = 0;
  T* mpCUData = nullptr;
  bool mView = false;

 public:
  void Swap(CuVector& o) {
    std::swap(mDim, o.mDim);
    std::swap(mBytes, o.mBytes);
    std::swap(mpCUData, o.mpCUData);
    std::swap(mView, o.mView);
  }
};

/// The arguments of one bunch gather (tnet_gather_bunch): bunch row r = cache row copy_from[r], its class
/// id alongside.  CuCache hands them out for the NEXT bunch so the step's last weight-update launch can
/// carry the gather (tnet_affine_update_bias_gather).
struct BunchGather {
  float* y = nullptr;
  const float* x = nullptr;
  int* labels_out = nullptr;
  const int* labels_in = nullptr;
  const int* copy_from = nullptr;
  TnetMatrixDim dy{}, dx{};
};

}  // namespace TNet
