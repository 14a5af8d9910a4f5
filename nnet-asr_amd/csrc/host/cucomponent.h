// cucomponent.h -- the CuComponent plugin API (the drop-in boundary of the hot path).
//
// Same class names, virtuals, ownership and wiring as src/CuTNetLib/cuComponent.h:27-175:
// a component OWNS its output and error-output matrices and BORROWS its input and error-input
// (double-linked with its predecessor at construction, cuComponent.h:183-195); Propagate()
// (re)initialises the output and calls PropagateFnc, Backpropagate() the error output and
// BackpropagateFnc (cuComponent.h:205-235).  Updatable components carry the learn rate,
// momentum, weight cost and GradDivFrm flag and implement Update().
//
// MI355X addition (no reference counterpart): updatable components can split Update() into
// ComputeGradient() + ApplyGradient() around a data-parallel gradient exchange (RCCL all-reduce,
// see trainer.h), and expose their gradient buffers for it.
#pragma once

#include <string>
#include <vector>

#include "cumath.h"

namespace TNet {

class CuComponent {
 public:
  typedef enum {
    UPDATABLE_COMPONENT = 0x0100,
    BIASED_LINEARITY,
    DISCRETE_LINEARITY,
    SHARED_LINEARITY,
    SPARSE_LINEARITY,
    RBM,
    RBM_SPARSE,
    RECURRENT,

    ACT_FUN = 0x0200,
    SOFTMAX,
    SIGMOID,

    OTHER = 0x0400,
    EXPAND,
    COPY,
    TRANSPOSE,
    BLOCK_LINEARITY,
    WINDOW,
    BIAS,
    LOG,

    BLOCK_ARRAY,

    CLUSTER_LINEARITY,
  } ComponentType;

  CuComponent(size_t nInputs, size_t nOutputs, CuComponent* pPred)
      : mNInputs(nInputs), mNOutputs(nOutputs), mpInput(nullptr), mpErrorInput(nullptr) {
    if (pPred != nullptr) {
      SetInput(pPred->GetOutput());
      pPred->SetErrorInput(GetErrorOutput());
    }
  }
  virtual ~CuComponent() {}

  virtual ComponentType GetType() const = 0;
  virtual const char* GetName() const = 0;
  virtual bool IsUpdatable() const { return false; }

  size_t GetNInputs() const { return mNInputs; }
  size_t GetNOutputs() const { return mNOutputs; }

  const CuMatrix<BaseFloat>& GetInput() const {
    if (!mpInput) Error("mpInput is NULL");
    return *mpInput;
  }
  const CuMatrix<BaseFloat>& GetOutput() const { return mOutput; }
  const CuMatrix<BaseFloat>& GetErrorInput() const {
    if (!mpErrorInput) Error("mpErrorInput is NULL");
    return *mpErrorInput;
  }
  const CuMatrix<BaseFloat>& GetErrorOutput() const { return mErrorOutput; }
  /// Mutable access used by fused network-level kernels (MI355X fast path).
  CuMatrix<BaseFloat>& Output() { return mOutput; }
  CuMatrix<BaseFloat>& ErrorOutput() { return mErrorOutput; }

  void SetInput(const CuMatrix<BaseFloat>& rInput) { mpInput = &rInput; }
  void SetErrorInput(const CuMatrix<BaseFloat>& rErrorInput) { mpErrorInput = &rErrorInput; }

  void Propagate() {
    mOutput.Init(GetInput().Rows(), GetNOutputs());
    if (GetNInputs() != GetInput().Cols()) {
      std::ostringstream os;
      os << "Non-matching INPUT dim!!! Network dim: " << GetNInputs() << " Data dim: " << GetInput().Cols();
      Error(os.str());
    }
    PropagateFnc(GetInput(), mOutput);
  }
  void Backpropagate() {
    mErrorOutput.Init(GetErrorInput().Rows(), GetNInputs());
    if (GetErrorInput().Cols() != mNOutputs) Error("Backpropagate: non-matching error-input dim");
    BackpropagateFnc(GetErrorInput(), mErrorOutput);
  }

  virtual void ReadFromStream(std::istream& rIn) {}
  virtual void WriteToStream(std::ostream& rOut) {}

 protected:
  virtual void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) = 0;
  virtual void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) = 0;

  size_t mNInputs;
  size_t mNOutputs;
  const CuMatrix<BaseFloat>* mpInput;
  const CuMatrix<BaseFloat>* mpErrorInput;
  CuMatrix<BaseFloat> mOutput;
  CuMatrix<BaseFloat> mErrorOutput;
};

/// A contiguous device parameter block taking part in the gradient exchange.
struct CuParamBlock {
  float* grad;   // gradient buffer (device), n elements
  long n;
  float* param;  // the parameters it updates, same n-element layout (sharded apply: all-gathered)
};

class GradExchange;

class CuUpdatableComponent : public CuComponent {
 public:
  CuUpdatableComponent(size_t nInputs, size_t nOutputs, CuComponent* pPred)
      : CuComponent(nInputs, nOutputs, pPred),
        mLearningRate(0.0f), mMomentum(0.0f), mWeightcost(0.0f), mGradDivFrm(true) {}
  virtual ~CuUpdatableComponent() {}
  bool IsUpdatable() const override { return true; }

  /// get gradient and update the parameters in one step (fused on MI355X)
  virtual void Update() = 0;

  // ---- data-parallel split of Update() (MI355X addition)
  /// Compute the local gradient into the component's gradient buffers (no parameter change).
  virtual void ComputeGradient() { Error(std::string(GetName()) + ": ComputeGradient not supported"); }
  /// Apply the (already reduced) gradient; `frames` = global rows contributing.
  /// stream: where to enqueue the update (nullptr: the library stream); ex: the exchange whose
  /// ApplyRanges pick the elements this rank updates (nullptr: all of them)
  virtual void ApplyGradient(size_t frames, void* stream = nullptr, const GradExchange* ex = nullptr) {
    (void)frames;
    (void)stream;
    (void)ex;
    Error(std::string(GetName()) + ": ApplyGradient not supported");
  }
  /// Gradient buffers of this component (valid after ComputeGradient()).
  virtual std::vector<CuParamBlock> GradientBlocks() { return {}; }
  /// Zero the gradient buffers (a data-parallel rank without a bunch contributes nothing).
  void ZeroGradient();

  void LearnRate(BaseFloat rate) { mLearningRate = rate; }
  BaseFloat LearnRate() const { return mLearningRate; }
  void Momentum(BaseFloat mmt) { mMomentum = mmt; }
  BaseFloat Momentum() const { return mMomentum; }
  void Weightcost(BaseFloat cost) { mWeightcost = cost; }
  BaseFloat Weightcost() const { return mWeightcost; }
  void GradDivFrm(bool div) { mGradDivFrm = div; }
  bool GradDivFrm() const { return mGradDivFrm; }

 protected:
  BaseFloat mLearningRate;
  BaseFloat mMomentum;
  BaseFloat mWeightcost;
  bool mGradDivFrm;
};

}  // namespace TNet
