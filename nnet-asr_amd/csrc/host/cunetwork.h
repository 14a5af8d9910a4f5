// cunetwork.h -- CuNetwork (src/CuTNetLib/cuNetwork.h:22-194, .cc:27-387).
//
// Same API: ReadNetwork/WriteNetwork (.nnet text, tags case-insensitive, <endblock> terminates),
// Propagate (component by component), Backpropagate (backprop with the PRE-update weights, then
// Update, stop at the "stopper" = first updatable component with learn rate > 0), SetLearnRate
// with per-layer factors "f1:f2:..." and the stopper rule (cuNetwork.cc:80-134), SetMomentum /
// SetWeightcost / SetL1 / SetGradDivFrm.
//
// MI355X fast path (TrainBunch): for the plain sigmoid-MLP topology
//   (<biasedlinearity> <sigmoid>)* <biasedlinearity> <softmax>  + cross-entropy
// one SGD step is  gather -> per layer one GEMM with bias+sigmoid epilogue -> one
// softmax+xent+error kernel -> per layer one GEMM with diff-sigmoid epilogue + one GEMM with the
// SGD update in its epilogue + one bias kernel.  Numerically it is the same sequence of float
// operations as Propagate + CuCrossEntropy::Evaluate + Backpropagate (checked against the oracle
// in tests/), minus the intermediate HBM round trips.
#pragma once

#include <memory>
#include <vector>

#include "culayers.h"
#include "cuobjective.h"

namespace TNet {

class GradExchange;  // trainer.h (data-parallel all-reduce)

class CuNetwork {
  typedef std::vector<CuComponent*> LayeredType;

 public:
  CuNetwork() {}
  explicit CuNetwork(std::istream& rIn) { ReadNetwork(rIn); }
  ~CuNetwork();
  CuNetwork(const CuNetwork&) = delete;
  CuNetwork& operator=(const CuNetwork&) = delete;

  void AddLayer(CuComponent* layer);
  int Layers() { return (int)mNetComponents.size(); }
  CuComponent& Layer(int i) { return *mNetComponents[i]; }

  /// forward the data to the output
  void Propagate(const CuMatrix<BaseFloat>& in, CuMatrix<BaseFloat>& out);
  /// backpropagate the error while updating weights
  void Backpropagate(const CuMatrix<BaseFloat>& globerr);

  void ReadNetwork(const char* pSrc);
  void WriteNetwork(const char* pDst);
  void ReadNetwork(std::istream& rIn);
  void WriteNetwork(std::ostream& rOut);

  size_t GetNInputs() const;
  size_t GetNOutputs() const;

  void SetLearnRate(BaseFloat learnRate, const char* pLearnRateFactors = NULL);
  BaseFloat GetLearnRate() { return mGlobLearnRate; }
  void PrintLearnRate();
  void SetMomentum(BaseFloat momentum);
  void SetWeightcost(BaseFloat weightcost);
  void SetL1(BaseFloat l1);
  void SetGradDivFrm(bool div);
  /// Directory for the cluster-transform bases of the TROY components (TNetCu.cc:245-248); no
  /// component of this build uses it, the value is only kept.
  void SetTempBasisDir(const char* dir) { mTempBasisDir = dir ? dir : ""; }

  // ---- MI355X fused training path -------------------------------------------------------
  /// true if the topology is the plain sigmoid MLP with a softmax output
  bool IsFusableMLP() const;
  /// One SGD step on a bunch (class-id targets). `obj` accumulates the statistics.
  /// With `exchange` set, gradients are all-reduced over data-parallel ranks before the update
  /// and `global_rows` frames enter the GRADDIVFRM normalisation.
  /// `train` = false: cross-validation (forward + objective only).
  /// Data-parallel step of a rank without a bunch: zero gradients into the exchange, then the
  /// same update as the ranks that trained (GradExchange::GlobalRows).
  void TrainEmpty(GradExchange& exchange);
  void TrainBunch(const CuMatrix<BaseFloat>& X, const CuVector<int>& labels, CuObjectiveFunction& obj,
                  bool train = true, GradExchange* exchange = nullptr);
  /// Keep the softmax output in the <softmax> component after TrainBunch (costs one extra
  /// [rows x classes] write per step; off by default).
  void KeepOutput(bool keep) { mKeepOutput = keep; }
  /// The NEXT bunch's gather, carried by the last weight-update launch of the next TrainBunch where the
  /// library takes it (tnet_affine_update_bias_gather: the update's tiles leave CUs free); TailGatherDone()
  /// says whether it went out -- if not, the caller launches it.  The descriptor is copied (the network
  /// never holds a pointer into the caller's frame); nullptr clears it.
  void SetTailGather(const BunchGather* g) {
    mHasTailGather = g != nullptr;
    if (g) mTailGather = *g;
    mTailDone = false;
  }
  bool TailGatherDone() const { return mTailDone; }
  /// Fault injection for the recovery tests: the n-th next TrainBunch (any network) throws before it
  /// enqueues anything; 0 disarms.
  static void DebugFailTrainBunch(long n);

 private:
  CuComponent* ComponentFactory(std::istream& In);
  void ComponentDumper(std::ostream& rOut, CuComponent& rComp);
  void TrainBunchGeneric(const CuMatrix<BaseFloat>& X, const CuVector<int>& labels, CuObjectiveFunction& obj,
                         bool train);

  LayeredType mNetComponents;
  std::string mTempBasisDir;
  CuComponent* mpPropagErrorStopper = nullptr;
  BaseFloat mGlobLearnRate = 0.0f;
  std::string mLearnRateFactors;
  bool mKeepOutput = false;
  BunchGather mTailGather;
  bool mHasTailGather = false;
  bool mTailDone = false;
  // fused-path buffers: activations of sigmoid layers are the components' own outputs;
  // errors live here (one per affine layer input)
  std::vector<std::unique_ptr<CuMatrix<BaseFloat>>> mErr;
  std::vector<std::unique_ptr<CuMatrix<BaseFloat>>> mColPart;  // per layer: 32-row slab column sums of its error
  CuMatrix<BaseFloat> mGlobErr;
};

}  // namespace TNet
