// curecurrent.h -- Elman recurrent layer trained frame by frame with truncated BPTT, and the
// TRecurrentCu loop (BASELINE config 5).
//
//   CuRecurrent        : src/CuTNetLib/cuRecurrent.h:15-57, cuRecurrent.cc:16-183 -- input row
//                        [x_t, y_{t-1}] pushed into a (bptt+1)-row history, y_t = sigmoid(b + row W),
//                        per-frame update from the present row plus bptt back-propagated rows
//   CuRecurrentTrainer : src/TRecurrentCu.cc:319-375 -- per utterance: clear the history, then for
//                        every frame propagate, cross-entropy, backpropagate + update
//
// MI355X: the history is a ring (no row shifting), every one-row GEMM/GEMV runs on the single-
// frame kernels of gemv.hip (split-K row-vector x matrix, wave-per-row matrix x vector), and the
// whole recurrent weight update -- all bptt+1 outer products, weight decay and the write of W --
// is one pass over W.
#pragma once

#include <cstdint>
#include <map>
#include <vector>

#include "cuobjective.h"
#include "culayers.h"

namespace TNet {

class CuNetwork;

class CuRecurrent : public CuUpdatableComponent {
 public:
  CuRecurrent(size_t nInputs, size_t nOutputs, CuComponent* pPred)
      : CuUpdatableComponent(nInputs, nOutputs, pPred), mLinearity(nInputs + nOutputs, nOutputs), mBias(nOutputs),
        mBiasCorrection(nOutputs) {}

  ComponentType GetType() const override { return RECURRENT; }
  const char* GetName() const override { return "<recurrent>"; }

  void PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) override;
  void Update() override;
  /// Update with d_0 = e .* y(1-y) already in DiffRow0() (written by the fused output-layer kernel).
  /// defer: the BPTT now, the weight update carried into the next PropagatePartial (its launch folded
  /// into the next frame's forward, tnet_gemv_rowvec_partial_update); any other use of the layer
  /// first runs it on its own (FlushPendingUpdate)
  void UpdateFromDiff0(bool defer = false);
  void FlushPendingUpdate();
  /// Fused-chain forward, first half: push the history row [x_t, y_{t-1}] and write the split-K
  /// partials of row W to `part` (tnet_gemv_rowvec_partial, with a deferred update applied); the bias
  /// + sigmoid finish is done by the output layer's kernel, which stores y_t into GetOutput().
  void PropagatePartial(const CuMatrix<BaseFloat>& X, float* part);
  float* DiffRow0() { return mDiff.pCURowData(0); }

  /// BPTT order; allocates the input history (cuRecurrent.h:30-33: ord+1 rows; here a ring of ord+2,
  /// so the next frame's push never lands on a row a deferred update still reads)
  void BpttOrder(int ord);
  int GetBpttOrder() const { return mBpttOrder; }
  /// zero the history and the previous output (cuRecurrent.h:34-39)
  void ClearHistory();

  void ReadFromStream(std::istream& rIn) override;
  void WriteToStream(std::ostream& rOut) override;

  CuMatrix<BaseFloat>& Linearity() { return mLinearity; }  ///< [(nIn + nOut) x nOut]
  CuVector<BaseFloat>& Bias() { return mBias; }
  CuVector<BaseFloat>& BiasCorrection() { return mBiasCorrection; }

  // ---- the look-ahead chain (CuRecurrentTrainer::TrainFrameFused; tnet_rnn_out_full_ahead / _bwd_update_ahead)
  /// the shapes it takes: bptt + 1 <= 9 steps (one fewer than the ring's rows), nOut a multiple of 4
  bool AheadOk() const {
    return mBpttOrder >= 0 && mBpttOrder + 1 <= 9 && mBpttOrder + 1 < (int)mInputHistory.Rows() && GetNOutputs() % 4 == 0;
  }
  int Steps() const { return mBpttOrder + 1; }
  float* HistoryData() { return mInputHistory.pCUData(); }
  int HistoryStride() const { return (int)mInputHistory.Stride(); }
  int HistoryRows() const { return (int)mInputHistory.Rows(); }
  float* DiffData() { return mDiff.pCUData(); }
  int DiffStride() const { return (int)mDiff.Stride(); }
  /// the ring row the next frame's history row goes to (the look-ahead pushes it)
  int NextHead() const { return (mHead + (int)mInputHistory.Rows() - 1) % (int)mInputHistory.Rows(); }
  /// a frame whose history row the previous frame's look-ahead already pushed: advance the ring head and hand the
  /// deferred update (its ring head; the caller's launch applies it) over -- -1 when none is pending
  int AheadAdvance();

  /// ring head (host state the per-frame chain advances; a graph replay sets it as the capture left it)
  int Head() const { return mHead; }
  void SetHead(int h) { mHead = h; }
  /// everything the fused frame chain's launches take from this layer (device pointers, ring shape,
  /// hyper-parameters): a recorded chain replays only while all of it is unchanged
  void ChainKey(std::vector<uint64_t>& k) const;

 private:
  const float* HistRow(int i) const {  // logical history row i (0 = present)
    return mInputHistory.pCURowData((size_t)((mHead + i) % (int)mInputHistory.Rows()));
  }
  CuMatrix<BaseFloat> mLinearity;
  CuVector<BaseFloat> mBias, mBiasCorrection;
  CuMatrix<BaseFloat> mInputHistory;  // ring of bptt+2 rows [x, y_prev] (the update reads bptt+1)
  CuMatrix<BaseFloat> mDiff;          // [bptt+1 x nOut] back-propagated errors of the present update
  CuMatrix<BaseFloat> mDiffTmp;       // [1 x nOut]
  int mBpttOrder = -1;
  int mHead = 0;
  bool mPending = false;  // UpdateFromDiff0(defer): the update of the ring at mPendHead not yet applied
  int mPendHead = 0;
  void RunUpdate(int head);
};

/// The TRecurrentCu loop over a network containing <recurrent> layers.
class CuRecurrentTrainer {
 public:
  CuRecurrentTrainer(CuNetwork* net, CuObjectiveFunction* obj, int bptt, bool crossval);
  /// One utterance: features [rows x cols] (host, leading dim ld) and class ids.
  void TrainUtterance(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels);
  long Frames() const { return mFrames; }

 private:
  CuNetwork* mNet;
  CuObjectiveFunction* mObj;
  bool mCrossval;
  // [<recurrent>, <biasedlinearity>, <softmax>] + cross-entropy: the per-frame chain on the fused
  // single-frame kernels (4 launches + the BPTT a frame instead of 18)
  bool FusedFrameOk() const;
  void TrainFrameFused(size_t f);
  CuMatrix<BaseFloat> mFeats, mOut, mErr, mRow;
  CuVector<int> mLabels, mLabelRow;
  long mFrames = 0;
  size_t mUttRows = 0;  // frames of the utterance on the fused chain (the last one's update is not deferred)
  // fused-chain scratch: recurrent / output split-K partials, softmax pairs, per-frame argmax keys
  CuMatrix<BaseFloat> mRecPart, mOutPart;
  // the look-ahead chain (TNET_RNN_AHEAD=0: off): the dots' partials, the recurrent bias / momentum after the
  // pending update (written by the frame's first launch, copied by its second); mAheadNext: the previous frame's
  // second launch took this frame's look-ahead
  CuMatrix<BaseFloat> mDotPart;
  CuVector<BaseFloat> mBnext, mCbnext;
  bool mAheadNext = false;
  bool AheadOn() const;
  void* mSmx = nullptr;
  size_t mSmxBytes = 0;
  void* mArgKey = nullptr;
  size_t mArgKeyBytes = 0;
  void* Scratch(void*& p, size_t& have, size_t bytes);
  // the utterance's fused frame chain recorded as hipGraphs and replayed (TNET_RNN_GRAPH=0: off):
  // one entry per utterance length; a key is recorded the second time it is seen (a length seen once
  // runs eagerly) and replayed from the third on.  The chain is cut into segments of at most
  // TNET_RNN_GRAPH_FRAMES frames (default 96, ~870 kernel nodes): rocprofiler-sdk (ROCm 7.2) faults
  // inside hipGraphLaunch on graphs of a few thousand kernel nodes (tools/graph_probe.hip: 1000 nodes
  // fine, 3000 SIGSEGV, profiles/r03_graph_probe_rocprof.txt), and a segment launch costs ~2 us
  struct ChainGraph {
    std::vector<uint64_t> key;
    int seen = 0;
    std::vector<hipGraphExec_t> execs;
    int head_after = 0;
  };
  void DestroyExecs(ChainGraph& g);
  std::map<size_t, ChainGraph> mGraphs;
  std::vector<uint64_t> ChainKey(size_t rows);
  bool GraphsEnabled() const;
  void RunFrames(size_t rows);

 public:
  ~CuRecurrentTrainer();
};

}  // namespace TNet
