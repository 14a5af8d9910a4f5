// culayers.h -- the hot-path components: <biasedlinearity>, <sigmoid>, <softmax>.
//
// CuBiasedLinearity : src/CuTNetLib/cuBiasedLinearity.h:15-85, .cc:11-119
// CuSigmoid/CuSoftmax: src/CuTNetLib/cuActivation.h:16-56, .cc:11-41
#pragma once

#include "cucomponent.h"

namespace TNet {

class CuBiasedLinearity : public CuUpdatableComponent {
 public:
  CuBiasedLinearity(size_t nInputs, size_t nOutputs, CuComponent* pPred)
      : CuUpdatableComponent(nInputs, nOutputs, pPred),
        mLinearity(nInputs, nOutputs), mBias(nOutputs),
        mLinearityCorrection(nInputs, nOutputs), mBiasCorrection(nOutputs) {}
  ~CuBiasedLinearity() {
    // the shadow's registration is keyed by W's address (the one registered, which is W's current storage unless
    // W was re-initialised since): gone before that storage can serve another matrix
    if (mShadowKey) (void)tnet_weight_shadow(mShadowKey, TnetMatrixDim{}, nullptr, 0);
  }

  ComponentType GetType() const override { return BIASED_LINEARITY; }
  const char* GetName() const override { return "<biasedlinearity>"; }

  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void Update() override;
  void ComputeGradient() override;
  // ComputeGradient with the bias gradient from the slab column sums of E (tnet_affine_grad_bias)
  void ComputeGradientColsum(const CuMatrix<BaseFloat>& colpart);
  // ComputeGradientColsum -- and with `other` (its inputs set by SetInput / SetErrorInput) also
  // other->ComputeGradientColsum(*colpart2) -- with the next bunch's gather `g` on the CUs the GEMMs' tiles leave
  // free, in ONE launch (tnet_affine_grad_bias_gather); false: nothing enqueued (make the separate calls)
  bool ComputeGradientColsumGather(const CuMatrix<BaseFloat>& colpart, const BunchGather& g,
                                   CuBiasedLinearity* other = nullptr, const CuMatrix<BaseFloat>* colpart2 = nullptr);
  // ComputeGradientColsum(colpart) of THIS layer (inputs as set by SetInput / SetErrorInput) and below's backward
  // Eo = (E2 W_below^T) .* Ybelow (1 - Ybelow) + Eo's slab sums in ONE launch (tnet_affine_grad_bwd_pair); false:
  // nothing enqueued (make the two calls)
  bool ComputeGradientColsumWithBwd(const CuMatrix<BaseFloat>& colpart, const CuBiasedLinearity& below,
                                    const CuMatrix<BaseFloat>& E2, const CuMatrix<BaseFloat>& Ybelow,
                                    CuMatrix<BaseFloat>& Eo, CuMatrix<BaseFloat>& colpart2);
  void ApplyGradient(size_t frames, void* stream = nullptr, const GradExchange* ex = nullptr) override;
  /// the applies of n (<= 2) layers on the compute stream in ONE launch when their SGD constants agree (the
  /// data-parallel step's inline exchange, GradExchange::SubmitInline); else ApplyGradient per layer
  static void ApplyGradients(CuBiasedLinearity* const* ls, int n, size_t frames, const GradExchange* ex);
  std::vector<CuParamBlock> GradientBlocks() override;

  void ReadFromStream(std::istream& rIn) override;
  void WriteToStream(std::ostream& rOut) override;

  // ---- access for the fused network-level kernels and the C ABI (the mutable accessor marks the transposed
  // shadow stale: the caller may change W through it)
  CuMatrix<BaseFloat>& Linearity() {
    mShadowValid = false;
    return mLinearity;
  }
  const CuMatrix<BaseFloat>& Linearity() const { return mLinearity; }
  const CuMatrix<BaseFloat>& LinearityRO() const { return mLinearity; }
  /// The transposed shadow Wt = W^T [nOut x nIn] the backward GEMM reads n-contiguous
  /// (tnet_affine_bwd_colsum_t): UseShadow registers it (tnet_weight_shadow), so that every fused update launch
  /// of W that supports it also writes Wt; ShadowForBwd refreshes it first when an update did not (or W changed
  /// by other means since) and returns it.
  void UseShadow();
  const CuMatrix<BaseFloat>& ShadowForBwd();
  bool HasShadow() const { return mShadowOn; }
  CuVector<BaseFloat>& Bias() { return mBias; }
  CuMatrix<BaseFloat>& LinearityCorrection() { return mLinearityCorrection; }
  CuVector<BaseFloat>& BiasCorrection() { return mBiasCorrection; }
  /// SGD constants of CuBiasedLinearity::Update (cuBiasedLinearity.cc:46-64) for `rows` frames
  void UpdateConstants(size_t rows, float* scale, float* l2) const;
  /// Update from explicit input/error matrices (fused GEMM + SGD epilogue, + bias kernel)
  void UpdateFrom(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E);
  /// single frame: Backpropagate (E -> Eout, old weights) + Update in one pass over W; with s != NULL
  /// also d = Eout .* s (1 - s) (tnet_affine_bwd_update_row)
  void BackpropUpdateRow(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E, CuMatrix<BaseFloat>& Eout,
                         const float* s, float* d);
  // same update with the bias gradient taken from the 32-row slab column sums of E that the backward
  // GEMM of the layer above wrote (tnet_affine_bwd_colsum): one launch instead of three
  void UpdateFromColsum(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E, const CuMatrix<BaseFloat>& colpart);
  /// This layer's UpdateFromColsum(X, E, colpart) and other's UpdateFromColsum(X2, E2, colpart2) in ONE
  /// launch (tnet_affine_update_bias_pair) when the two small grids fit one round over the CUs; false:
  /// nothing enqueued (make the two calls).
  bool UpdatePairFromColsum(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E,
                            const CuMatrix<BaseFloat>& colpart, CuBiasedLinearity& other, const CuMatrix<BaseFloat>& X2,
                            const CuMatrix<BaseFloat>& E2, const CuMatrix<BaseFloat>& colpart2);
  /// UpdateFromColsum (other == nullptr) or UpdatePairFromColsum, with the next bunch's gather `g` on the
  /// CUs the update's tiles leave free, all in ONE launch (tnet_affine_update_bias_gather); false: nothing
  /// enqueued (make the separate calls).
  bool UpdateFromColsumGather(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E,
                              const CuMatrix<BaseFloat>& colpart, CuBiasedLinearity* other,
                              const CuMatrix<BaseFloat>* X2, const CuMatrix<BaseFloat>* E2,
                              const CuMatrix<BaseFloat>* colpart2, const BunchGather& g);
  /// UpdateFromColsum and, in the same launch, the backward GEMM of the layer below
  /// (tnet_affine_update_bwd_pair): Eo = (E2 below.W^T) .* Ybelow (1 - Ybelow) + Eo's slab sums into
  /// colpart2.  False (nothing enqueued) when the pair kernel does not take these shapes.
  bool UpdateFromColsumWithBwd(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E,
                               const CuMatrix<BaseFloat>& colpart, const CuBiasedLinearity& below,
                               const CuMatrix<BaseFloat>& E2, const CuMatrix<BaseFloat>& Ybelow,
                               CuMatrix<BaseFloat>& Eo, CuMatrix<BaseFloat>& colpart2, bool use_shadow);

 protected:
  CuMatrix<BaseFloat> mLinearity;            ///< [nIn x nOut] (file stores the transpose)
  CuVector<BaseFloat> mBias;                 ///< [nOut]
  CuMatrix<BaseFloat> mLinearityCorrection;  ///< momentum buffer
  CuVector<BaseFloat> mBiasCorrection;       ///< momentum buffer
  CuMatrix<BaseFloat> mGradW;                ///< data-parallel gradient buffers (lazy)
  CuVector<BaseFloat> mGradB;
  CuMatrix<BaseFloat> mLinearityT;           ///< transposed shadow of mLinearity [nOut x nIn] (UseShadow)
  bool mShadowOn = false, mShadowValid = false;
  const float* mShadowKey = nullptr;         ///< the W address the shadow is registered under
  /// unregister the shadow under an address W no longer has (no-op while the registration is current)
  void DropShadowKey();
  /// after an update launch of W: the shadow is current iff that launch wrote it (tnet_weight_shadow_kept)
  void NoteUpdate() { mShadowValid = mShadowOn && tnet_weight_shadow_kept(mLinearity.pCUData()) == 1; }
  /// the SGD segments (W, b: this rank's ranges) of the data-parallel apply into seg (<= 4), their scale
  int ApplySegments(size_t frames, const GradExchange* ex, TnetSgdSeg* seg, float* scale);
};

class CuSigmoid : public CuComponent {
 public:
  CuSigmoid(size_t nInputs, size_t nOutputs, CuComponent* pPred) : CuComponent(nInputs, nOutputs, pPred) {}
  ComponentType GetType() const override { return SIGMOID; }
  const char* GetName() const override { return "<sigmoid>"; }

 protected:
  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
};

class CuSoftmax : public CuComponent {
 public:
  CuSoftmax(size_t nInputs, size_t nOutputs, CuComponent* pPred) : CuComponent(nInputs, nOutputs, pPred) {}
  ComponentType GetType() const override { return SOFTMAX; }
  const char* GetName() const override { return "<softmax>"; }

 protected:
  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
};

/// Fast text parsing of "m R C ..." / "v N ..." blocks (strtof on a buffered stream).
void ReadMatrixFast(std::istream& in, Matrix<BaseFloat>& m);
void ReadVectorFast(std::istream& in, Vector<BaseFloat>& v);

}  // namespace TNet
