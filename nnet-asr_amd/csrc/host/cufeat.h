// cufeat.h -- the feature front-end components of a --FEATURETRANSFORM network
// (src/CuTNetLib/cuCRBEDctFeat.h:16-304): <expand>, <copy>, <transpose>, <blocklinearity>,
// <bias>, <window>, <log>.
//
// TNetCu / TFeaCatCu push every utterance through such a network before the cache
// (TNetCu.cc:384-393): e.g. examples/01's Hamm_dct_norm = <expand> 23 -> 51 frames x 23,
// <transpose> to band-major, <window> (Hamming), <blocklinearity> (DCT 51 -> 26 per band),
// <bias> + <window> (global mean / variance normalisation).  Forward only, like the reference:
// only <bias> backpropagates (a copy).  File formats, index conventions (<copy> stores 1-based
// indices) and errors as the reference.
#pragma once

#include <vector>

#include "cucomponent.h"

namespace TNet {

/// "v N i1 .. iN" integer vector (the KaldiLib Vector<int> text format, Vector.tcc:525-571)
void ReadIntVector(std::istream& in, std::vector<int>& v);
void WriteIntVector(std::ostream& out, const std::vector<int>& v);

/// frame-context splice: out = [x(t+o_1) .. x(t+o_k)], edge frames repeated (cuCRBEDctFeat.h:16-47)
class CuExpand : public CuComponent {
 public:
  CuExpand(size_t nInputs, size_t nOutputs, CuComponent* pPred) : CuComponent(nInputs, nOutputs, pPred) {}
  ComponentType GetType() const override { return EXPAND; }
  const char* GetName() const override { return "<expand>"; }
  void ReadFromStream(std::istream& rIn) override;
  void WriteToStream(std::ostream& rOut) override;
  const std::vector<int>& FrameOffsets() const { return mHostOffsets; }

 protected:
  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  std::vector<int> mHostOffsets;
  CuVector<int> mFrameOffset;
};

/// column gather by (file: 1-based) indices (cuCRBEDctFeat.h:54-85)
class CuCopy : public CuComponent {
 public:
  CuCopy(size_t nInputs, size_t nOutputs, CuComponent* pPred) : CuComponent(nInputs, nOutputs, pPred) {}
  ComponentType GetType() const override { return COPY; }
  const char* GetName() const override { return "<copy>"; }
  void ReadFromStream(std::istream& rIn) override;
  void WriteToStream(std::ostream& rOut) override;

 protected:
  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  std::vector<int> mHostIndices;  // 0-based
  CuVector<int> mCopyFromIndices;
};

/// frame-major -> channel-major reorder of a spliced vector (cuCRBEDctFeat.h:87-139)
class CuTranspose : public CuComponent {
 public:
  CuTranspose(size_t nInputs, size_t nOutputs, CuComponent* pPred)
      : CuComponent(nInputs, nOutputs, pPred), mContext(0) {}
  ComponentType GetType() const override { return TRANSPOSE; }
  const char* GetName() const override { return "<transpose>"; }
  void ReadFromStream(std::istream& rIn) override;
  void WriteToStream(std::ostream& rOut) override;

 protected:
  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  int mContext;
  CuVector<int> mCopyFromIndices;
};

/// block-diagonal linear transform, file stores the [bo x bi] block transposed (cuCRBEDctFeat.h:146-197)
class CuBlockLinearity : public CuComponent {
 public:
  CuBlockLinearity(size_t nInputs, size_t nOutputs, CuComponent* pPred) : CuComponent(nInputs, nOutputs, pPred) {}
  ComponentType GetType() const override { return BLOCK_LINEARITY; }
  const char* GetName() const override { return "<blocklinearity>"; }
  void ReadFromStream(std::istream& rIn) override;
  void WriteToStream(std::ostream& rOut) override;

 protected:
  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  CuMatrix<BaseFloat> mBlockLinearity;  // [bi x bo]
};

/// Y = X + b (cuCRBEDctFeat.h:201-234)
class CuBias : public CuComponent {
 public:
  CuBias(size_t nInputs, size_t nOutputs, CuComponent* pPred) : CuComponent(nInputs, nOutputs, pPred) {}
  ComponentType GetType() const override { return BIAS; }
  const char* GetName() const override { return "<bias>"; }
  void ReadFromStream(std::istream& rIn) override;
  void WriteToStream(std::ostream& rOut) override;

 protected:
  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  CuVector<BaseFloat> mBias;
};

/// Y = X .* w per column (cuCRBEDctFeat.h:238-271)
class CuWindow : public CuComponent {
 public:
  CuWindow(size_t nInputs, size_t nOutputs, CuComponent* pPred) : CuComponent(nInputs, nOutputs, pPred) {}
  ComponentType GetType() const override { return WINDOW; }
  const char* GetName() const override { return "<window>"; }
  void ReadFromStream(std::istream& rIn) override;
  void WriteToStream(std::ostream& rOut) override;

 protected:
  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  CuVector<BaseFloat> mWindow;
};

/// Y = log(X) (cuCRBEDctFeat.h:273-304)
class CuLog : public CuComponent {
 public:
  CuLog(size_t nInputs, size_t nOutputs, CuComponent* pPred) : CuComponent(nInputs, nOutputs, pPred) {}
  ComponentType GetType() const override { return LOG; }
  const char* GetName() const override { return "<log>"; }

 protected:
  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
};

}  // namespace TNet
