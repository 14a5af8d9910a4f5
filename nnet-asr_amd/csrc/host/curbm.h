// curbm.h -- Gauss/Bernoulli RBM layer, its per-element random numbers, and the CD-1
// pre-training loop (BASELINE config 4).
//
//   CuRbm        : src/CuTNetLib/cuRbm.h:15-95, cuRbm.cc:15-241 (<rbm> component: fine-tuning
//                  Propagate/Backpropagate/Update, plus the RBM API Propagate / Reconstruct /
//                  RbmUpdate and the "bern|gauss bern|gauss" text format)
//   CuRand       : src/CuBaseLib/curand.h:11-32, curand.tcc:13-154 (HybridTaus state per element,
//                  seeded from the lrand48 stream)
//   CuRbmTrainer : the TRbmCu loop, src/TRbmCu.cc:291-357 (cache -> positive phase -> sample ->
//                  reconstruct -> negative phase -> update -> reconstruction MSE)
//
// MI355X: the trainer keeps the positive and negative phase statistics row-stacked in one
// [2B x n_vis] and one [2B x n_hid] buffer (negative hidden probabilities stored negated by the
// GEMM epilogue), so the whole weight update is ONE K = 2B GEMM with the momentum/weight-cost
// epilogue and each bias update one signed column sum; sampling is fused with the draw.
#pragma once

#include "cucache.h"
#include "culayers.h"
#include "cuobjective.h"
#include "rng48.h"

namespace TNet {

/// The RBM training interface the drivers program against (cuRbm.h:15-45).
class CuRbmBase : public CuBiasedLinearity {
 public:
  typedef enum { BERNOULLI, GAUSSIAN } RbmUnitType;
  CuRbmBase(size_t nInputs, size_t nOutputs, CuComponent* pPred) : CuBiasedLinearity(nInputs, nOutputs, pPred) {}
  virtual void Propagate(const CuMatrix<BaseFloat>& visProbs, CuMatrix<BaseFloat>& hidProbs) = 0;
  virtual void Reconstruct(const CuMatrix<BaseFloat>& hidState, CuMatrix<BaseFloat>& visProbs) = 0;
  virtual void RbmUpdate(const CuMatrix<BaseFloat>& pos_vis, const CuMatrix<BaseFloat>& pos_hid,
                         const CuMatrix<BaseFloat>& neg_vis, const CuMatrix<BaseFloat>& neg_hid) = 0;
  virtual RbmUnitType VisType() const = 0;
  virtual RbmUnitType HidType() const = 0;
  using CuComponent::Propagate;
};

class CuRbm : public CuRbmBase {
 public:
  CuRbm(size_t nInputs, size_t nOutputs, CuComponent* pPred)
      : CuRbmBase(nInputs, nOutputs, pPred), mVisBias(nInputs), mVisBiasCorrection(nInputs) {}

  ComponentType GetType() const override { return RBM; }
  const char* GetName() const override { return "<rbm>"; }

  // CuUpdatableComponent API (fine-tuning as a feed-forward layer)
  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void Update() override;

  // RBM training API (cuRbm.h:27-45)
  void Propagate(const CuMatrix<BaseFloat>& visProbs, CuMatrix<BaseFloat>& hidProbs) override;
  void Reconstruct(const CuMatrix<BaseFloat>& hidState, CuMatrix<BaseFloat>& visProbs) override;
  void RbmUpdate(const CuMatrix<BaseFloat>& pos_vis, const CuMatrix<BaseFloat>& pos_hid,
                 const CuMatrix<BaseFloat>& neg_vis, const CuMatrix<BaseFloat>& neg_hid) override;
  RbmUnitType VisType() const override { return mVisType; }
  RbmUnitType HidType() const override { return mHidType; }
  using CuComponent::Propagate;
  void SetUnitTypes(RbmUnitType vis, RbmUnitType hid) { mVisType = vis; mHidType = hid; }

  void ReadFromStream(std::istream& rIn) override;
  void WriteToStream(std::ostream& rOut) override;

  CuMatrix<BaseFloat>& VisHid() { return mLinearity; }  ///< [n_vis x n_hid]
  CuVector<BaseFloat>& HidBias() { return mBias; }
  CuVector<BaseFloat>& VisBias() { return mVisBias; }
  CuVector<BaseFloat>& VisBiasCorrection() { return mVisBiasCorrection; }
  CuVector<BaseFloat>& HidBiasCorrection() { return mBiasCorrection; }
  CuMatrix<BaseFloat>& VisHidCorrection() { return mLinearityCorrection; }

 private:
  CuVector<BaseFloat> mVisBias, mVisBiasCorrection;
  CuMatrix<BaseFloat> mBackpropErrBuf;
  RbmUnitType mVisType = GAUSSIAN, mHidType = BERNOULLI;
};

/// Per-element HybridTaus generator state for a rows x cols target (curand.h:11-32).
class CuRandState {
 public:
  CuRandState() {}
  CuRandState(size_t rows, size_t cols, Rng48& rng) { SeedGpu(rows, cols, rng); }
  /// Four state matrices filled row by row with lrand48() values > 128, z1 first
  /// (curand.tcc:13-45: the draws come from the process lrand48 stream, here `rng`).
  void SeedGpu(size_t rows, size_t cols, Rng48& rng);
  void Rand(CuMatrix<BaseFloat>& tgt);
  void GaussRand(CuMatrix<BaseFloat>& tgt);
  void BinarizeProbs(const CuMatrix<BaseFloat>& probs, CuMatrix<BaseFloat>& states);
  /// probs = sigmoid(X W + b) and BinarizeProbs(probs, states) in one launch (tnet_affine_fwd_sample);
  /// probs already sized like the generator
  void AffineSigmoidSample(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& W, const CuVector<BaseFloat>& b,
                           CuMatrix<BaseFloat>& probs, CuMatrix<BaseFloat>& states);
  void AddGaussNoise(CuMatrix<BaseFloat>& tgt, BaseFloat gscale = 1.0f);
  size_t Rows() const { return z[0].Rows(); }
  size_t Cols() const { return z[0].Cols(); }
  CuMatrix<unsigned>& State(int i) { return z[i]; }

 private:
  void Check(const CuMatrix<BaseFloat>& m) const;
  CuMatrix<unsigned> z[4];
};

/// The reference's CuRand<T>(rows, cols) (curand.h:11-32): seeded from the process lrand48
/// stream (GlobalRng: libc's srand48/lrand48 in the drop-in build).
template <typename T>
class CuRand : public CuRandState {
  static_assert(std::is_same<T, BaseFloat>::value, "CuRand: BaseFloat only");

 public:
  CuRand(size_t rows, size_t cols) : CuRandState(rows, cols, GlobalRng()) {}
};

struct RbmTrainerOptions {
  size_t bunchsize = 256;    // TRbmCu.cc:173 --BUNCHSIZE
  size_t cachesize = 12800;  // --CACHESIZE
  long seed = 0;             // --SEED (0 = time seeded)
  bool randomize = true;
  int trace = 0;
};

class CuRbmTrainer {
 public:
  CuRbmTrainer(CuRbm* rbm, const RbmTrainerOptions& opt);
  void AddUtterance(const float* feats, size_t rows, size_t cols, size_t ld);
  void Finish();
  long Steps() const { return mSteps; }
  CuMeanSquareError& Mse() { return mMse; }
  size_t Prefill(const float* feats, size_t rows, size_t cols, size_t ld);
  void Replay(long n);
  Rng48& Rng() { return mRng; }

 private:
  void DrainCache();
  void Step();

  CuRbm* mRbm;
  RbmTrainerOptions mOpt;
  Rng48 mRng;
  CuRandState mRand;
  CuCache mCache;
  CuMeanSquareError mMse;
  // the stacked visible statistics twice: the step trains mVB[mCurV] while its last launch gathers the next
  // bunch into the positive half of the other (tnet_rbm_update_stats_gather)
  CuMatrix<BaseFloat> mVB[2], mH, mStates;           // [2B x vis] x 2, [2B x hid], [B x hid]
  CuMatrix<BaseFloat> mPosVis, mNegVis, mPosHid, mNegHid;  // row views into mVB[mCurV] / mH
  CuMatrix<BaseFloat> mNextPosVis;                   // the positive half of mVB[mCurV ^ 1]
  int mCurV = 0;
  bool mAheadV = false;  // mVB[mCurV ^ 1] holds the next bunch
  void ViewV();
  CuVector<int> mDummyLabels;
  std::vector<int> mZeroLabels;
  long mSteps = 0;
  bool mTrainedSinceFill = false;
};

}  // namespace TNet
