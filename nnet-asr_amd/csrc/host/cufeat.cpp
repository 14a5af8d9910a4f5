// cufeat.cpp -- see cufeat.h.  Each component is one gfx950 launch (the gathers and the
// column scale are flat float4 kernels, the block transform one LDS-staged kernel), on the
// library's stream, no host sync.
#include "cufeat.h"

#include <sstream>

#include "culayers.h"

namespace TNet {

#define S ((void*)CuDevice::Instantiate().Stream())

void ReadIntVector(std::istream& in, std::vector<int>& v) {
  in >> std::ws;
  if (in.peek() != 'v') Error("Failed to read vector from stream: expected 'v N'");
  in.get();
  long long n = -1;
  in >> n;
  if (in.fail() || n < 0) Error("Failed to read vector from stream: no size");
  v.assign((size_t)n, 0);
  for (long long i = 0; i < n; i++) {
    in >> v[(size_t)i];
    if (in.fail()) Error("Failed to read vector from stream");
  }
}

void WriteIntVector(std::ostream& out, const std::vector<int>& v) {
  out << "v " << v.size() << "  ";
  for (int x : v) out << x << ' ';
}

static void NonsenseBackprop(const char* name) { Error(std::string(name) + " : backpropagation is nonsense"); }

// ------------------------------------------------------------------------------ <expand>
void CuExpand::ReadFromStream(std::istream& rIn) {
  ReadIntVector(rIn, mHostOffsets);
  if (mHostOffsets.empty() || GetNInputs() * mHostOffsets.size() != GetNOutputs()) {
    std::ostringstream os;
    os << "<expand>: " << mHostOffsets.size() << " frame offsets do not map " << GetNInputs() << " inputs to "
       << GetNOutputs() << " outputs";
    Error(os.str());
  }
  mFrameOffset.CopyFromHost(mHostOffsets.data(), mHostOffsets.size());
}
void CuExpand::WriteToStream(std::ostream& rOut) { WriteIntVector(rOut, mHostOffsets); }
void CuExpand::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuMath<BaseFloat>::Expand(Y, X, mFrameOffset);
}
void CuExpand::BackpropagateFnc(const CuMatrix<BaseFloat>&, CuMatrix<BaseFloat>&) { NonsenseBackprop(GetName()); }

// ------------------------------------------------------------------------------ <copy>
void CuCopy::ReadFromStream(std::istream& rIn) {
  ReadIntVector(rIn, mHostIndices);
  for (int& i : mHostIndices) i -= 1;  // the file is 1-based (vec.Add(-1), cuCRBEDctFeat.h:71)
  if (mHostIndices.size() != GetNOutputs()) Error("<copy>: number of indices must equal the output dim");
  mCopyFromIndices.CopyFromHost(mHostIndices.data(), mHostIndices.size());
}
void CuCopy::WriteToStream(std::ostream& rOut) {
  std::vector<int> one_based(mHostIndices);
  for (int& i : one_based) i += 1;
  WriteIntVector(rOut, one_based);
}
void CuCopy::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuMath<BaseFloat>::Rearrange(Y, X, mCopyFromIndices);
}
void CuCopy::BackpropagateFnc(const CuMatrix<BaseFloat>&, CuMatrix<BaseFloat>&) { NonsenseBackprop(GetName()); }

// ------------------------------------------------------------------------------ <transpose>
void CuTranspose::ReadFromStream(std::istream& rIn) {
  rIn >> std::ws >> mContext;
  if (rIn.fail() || mContext <= 0) Error("<transpose>: missing context length");
  if (GetNInputs() != GetNOutputs()) Error("Input dim must be same as output dim");
  if (GetNInputs() % mContext != 0) Error("Number of inputs must be divisible by context length");
  // output i = channel ch of frame f  <-  input f*channels + ch, channel-major (cuCRBEDctFeat.h:109-123)
  const int n = (int)GetNInputs(), channels = n / mContext;
  std::vector<int> idx((size_t)n);
  for (int i = 0, ch = 0; ch < channels; ch++)
    for (int src = ch; src < n; src += channels, i++) idx[(size_t)i] = src;
  mCopyFromIndices.CopyFromHost(idx.data(), idx.size());
}
void CuTranspose::WriteToStream(std::ostream& rOut) { rOut << " " << mContext << "\n"; }
void CuTranspose::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuMath<BaseFloat>::Rearrange(Y, X, mCopyFromIndices);
}
void CuTranspose::BackpropagateFnc(const CuMatrix<BaseFloat>&, CuMatrix<BaseFloat>&) { NonsenseBackprop(GetName()); }

// ------------------------------------------------------------------------------ <blocklinearity>
void CuBlockLinearity::ReadFromStream(std::istream& rIn) {
  BfMatrix stored;  // [bo x bi]
  ReadMatrixFast(rIn, stored);
  if (stored.Rows() * stored.Cols() == 0) Error("Missing block matrix in network file");
  mBlockLinearity.CopyFrom(BfMatrix(stored, TRANS));
  if (GetNOutputs() % mBlockLinearity.Cols() != 0 || GetNInputs() % mBlockLinearity.Rows() != 0 ||
      GetNOutputs() / mBlockLinearity.Cols() != GetNInputs() / mBlockLinearity.Rows())
    Error("BlockLinearity matrix dimensions must divide IO dims");
}
void CuBlockLinearity::WriteToStream(std::ostream& rOut) {
  BfMatrix tmp;
  mBlockLinearity.CopyTo(tmp);
  rOut << BfMatrix(tmp, TRANS);
}
void CuBlockLinearity::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuMath<BaseFloat>::BlockLinearity(Y, X, mBlockLinearity);
}
void CuBlockLinearity::BackpropagateFnc(const CuMatrix<BaseFloat>&, CuMatrix<BaseFloat>&) {
  Error("<blocklinearity> : backpropagation not implemented");
}

// ------------------------------------------------------------------------------ <bias>
void CuBias::ReadFromStream(std::istream& rIn) {
  BfVector vec;
  ReadVectorFast(rIn, vec);
  if (vec.Dim() != GetNOutputs()) Error("<bias>: vector dim must equal the output dim");
  mBias.CopyFrom(vec);
}
void CuBias::WriteToStream(std::ostream& rOut) {
  BfVector vec;
  mBias.CopyTo(vec);
  rOut << vec;
}
void CuBias::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  Y.CopyFrom(X);
  Y.AddScaledRow(1.0f, mBias, 1.0f);
}
void CuBias::BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) { Y.CopyFrom(X); }

// ------------------------------------------------------------------------------ <window>
void CuWindow::ReadFromStream(std::istream& rIn) {
  BfVector vec;
  ReadVectorFast(rIn, vec);
  if (vec.Dim() != GetNOutputs()) Error("<window>: vector dim must equal the output dim");
  mWindow.CopyFrom(vec);
}
void CuWindow::WriteToStream(std::ostream& rOut) {
  BfVector vec;
  mWindow.CopyTo(vec);
  rOut << vec;
}
void CuWindow::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  Y.CopyFrom(X);
  Y.ScaleCols(mWindow);
}
void CuWindow::BackpropagateFnc(const CuMatrix<BaseFloat>&, CuMatrix<BaseFloat>&) {
  Error("<window> : backpropagation not implemented");
}

// ------------------------------------------------------------------------------ <log>
void CuLog::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  Y.CopyFrom(X);
  Y.ApplyLog();
}
void CuLog::BackpropagateFnc(const CuMatrix<BaseFloat>&, CuMatrix<BaseFloat>&) {
  Error("<log> : backpropagation not implemented");
}

}  // namespace TNet
