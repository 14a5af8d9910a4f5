// hostmatrix.h -- minimal host-side Matrix/Vector (the KaldiLib boundary types the CuTNetLib API
// exchanges with the drivers: src/KaldiLib/Matrix.h, Vector.h) and their text format
// (src/KaldiLib/Matrix.tcc:521-600 "m R C" + rows; Vector.tcc:525-571 "v N" + values).
#pragma once

#include <cmath>
#include <cstring>
#include <istream>
#include <ostream>
#include <string>
#include <vector>

#include "tnet_common.h"

#ifdef TNET_HOST_KALDILIB
// drop-in build: the reference's host containers and their text I/O (src/KaldiLib/Matrix.h,
// Vector.h, Matrix.tcc:521-600, Vector.tcc:525-571)
#include "Matrix.h"
#include "Vector.h"
#else
namespace TNet {

enum MatrixTrasposeType { NO_TRANS = 'N', TRANS = 'T' };

template <typename T>
class Matrix {
 public:
  Matrix() {}
  Matrix(size_t r, size_t c) { Init(r, c); }
  Matrix(const Matrix& m, MatrixTrasposeType t) {
    if (t == NO_TRANS) {
      *this = m;
    } else {
      Init(m.Cols(), m.Rows());
      for (size_t i = 0; i < m.Rows(); i++)
        for (size_t j = 0; j < m.Cols(); j++) (*this)(j, i) = m(i, j);
    }
  }
  void Init(size_t r, size_t c) {
    mRows = r;
    mCols = c;
    mData.assign(r * c, T(0));
  }
  size_t Rows() const { return mRows; }
  size_t Cols() const { return mCols; }
  size_t Stride() const { return mCols; }
  T* pData() { return mData.data(); }
  const T* pData() const { return mData.data(); }
  T* pRowData(size_t r) { return mData.data() + r * mCols; }
  const T* pRowData(size_t r) const { return mData.data() + r * mCols; }
  T& operator()(size_t r, size_t c) { return mData[r * mCols + c]; }
  const T& operator()(size_t r, size_t c) const { return mData[r * mCols + c]; }
  void Zero() { std::fill(mData.begin(), mData.end(), T(0)); }
  /// NaN / Inf check (Matrix::CheckData, used at TNetCu.cc:386)
  bool CheckData(const std::string& file = "") const {
    for (size_t i = 0; i < mData.size(); i++)
      if (std::isnan((double)mData[i]) || std::isinf((double)mData[i]))
        Error("Matrix::CheckData: NaN or Inf in " + file);
    return true;
  }

 private:
  size_t mRows = 0, mCols = 0;
  std::vector<T> mData;
};

template <typename T>
class Vector {
 public:
  Vector() {}
  explicit Vector(size_t n) { Init(n); }
  void Init(size_t n) { mData.assign(n, T(0)); }
  size_t Dim() const { return mData.size(); }
  T* pData() { return mData.data(); }
  const T* pData() const { return mData.data(); }
  T& operator[](size_t i) { return mData[i]; }
  const T& operator[](size_t i) const { return mData[i]; }
  double Sum() const {
    double s = 0;
    for (auto v : mData) s += v;
    return s;
  }

 private:
  std::vector<T> mData;
};

// ---- text I/O ("new" format only: the one the .nnet writer emits)
template <typename T>
std::istream& operator>>(std::istream& in, Matrix<T>& m) {
  in >> std::ws;
  if (in.peek() != 'm') Error("Failed to read matrix from stream: expected 'm R C'");
  in.get();
  long long r = -1, c = -1;
  in >> r >> c;
  if (in.fail() || r < 0 || c < 0) Error("Failed to read matrix from stream: no size");
  m.Init((size_t)r, (size_t)c);
  for (long long i = 0; i < r; i++)
    for (long long j = 0; j < c; j++) {
      in >> m((size_t)i, (size_t)j);
      if (in.fail()) Error("Failed to read matrix from stream");
    }
  return in;
}

template <typename T>
std::ostream& operator<<(std::ostream& out, const Matrix<T>& m) {
  out << "m " << m.Rows() << ' ' << m.Cols() << '\n';
  for (size_t i = 0; i < m.Rows(); i++) {
    for (size_t j = 0; j < m.Cols(); j++) out << m(i, j) << ' ';
    out << '\n';
  }
  return out;
}

template <typename T>
std::istream& operator>>(std::istream& in, Vector<T>& v) {
  in >> std::ws;
  if (in.peek() != 'v') Error("Failed to read vector from stream: expected 'v N'");
  in.get();
  long long n = -1;
  in >> n;
  if (in.fail() || n < 0) Error("Failed to read vector from stream: no size");
  v.Init((size_t)n);
  for (long long i = 0; i < n; i++) {
    in >> v[(size_t)i];
    if (in.fail()) Error("Failed to read vector from stream");
  }
  return in;
}

template <typename T>
std::ostream& operator<<(std::ostream& out, const Vector<T>& v) {
  out << "v " << v.Dim() << "  ";
  for (size_t i = 0; i < v.Dim(); i++) out << v[i] << ' ';
  return out;
}

typedef Matrix<BaseFloat> BfMatrix;
typedef Vector<BaseFloat> BfVector;

}  // namespace TNet
#endif  // TNET_HOST_KALDILIB
