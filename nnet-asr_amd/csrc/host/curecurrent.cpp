// curecurrent.cpp -- see curecurrent.h.
#include "curecurrent.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "cunetwork.h"

namespace TNet {

#define S ((void*)CuDevice::Instantiate().Stream())

void CuRecurrent::BpttOrder(int ord) {
  if (ord < 0) Error("CuRecurrent::BpttOrder: negative order");
  FlushPendingUpdate();
  mBpttOrder = ord;
  mInputHistory.Init((size_t)ord + 2, GetNInputs() + GetNOutputs());
  mDiff.Init((size_t)ord + 1, GetNOutputs());
  mDiffTmp.Init(1, GetNOutputs());
  mHead = 0;
}

int CuRecurrent::AheadAdvance() {
  if (mInputHistory.Rows() == 0) Error("Bptt order was not set");
  mOutput.Init(1, GetNOutputs());
  mHead = NextHead();
  if (!mPending) return -1;
  mPending = false;
  return mPendHead;
}

void CuRecurrent::ClearHistory() {
  FlushPendingUpdate();
  mInputHistory.SetZero();
  if (mOutput.MSize() > 0) mOutput.SetZero();
  mHead = 0;
}

void CuRecurrent::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuProfileScope p("CuRecurrent::Propagate");
  if (X.Rows() != 1 || Y.Rows() != 1) Error("CuRecurrent: frame-by-frame (one row) propagation only");
  if (mInputHistory.Rows() == 0) Error("Bptt order was not set");
  FlushPendingUpdate();
  // push back the history: the ring head moves to the row of the oldest entry (cuRecurrent.cc:26-29)
  const int R = (int)mInputHistory.Rows();
  mHead = (mHead + R - 1) % R;
  float* row = mInputHistory.pCURowData((size_t)mHead);
  // row 0 = [x_t, y_{t-1}]: Y still holds the previous frame's output (cuRecurrent.cc:31-35);
  // y_t = sigmoid(b + row W) (AddScaledRow + OffsetGemv('T') + Sigmoid, cuRecurrent.cc:41-47).  The
  // row-vector kernel reads [x_t, y_{t-1}] in place and stores the history row itself.
  const int K = (int)(GetNInputs() + GetNOutputs()), N = (int)GetNOutputs();
  void* ws = CuDevice::Instantiate().Workspace((size_t)tnet_gemv_workspace(K, N));
  TNET_SAFE_CALL(tnet_gemv_rowvec_cat(X.pCUData(), (int)X.Cols(), Y.pCUData(), (int)Y.Cols(), row,
                                      mLinearity.pCUData(), (int)mLinearity.Stride(), mBias.pCUData(), Y.pCUData(),
                                      N, 1, ws, S));
}

void CuRecurrent::PropagatePartial(const CuMatrix<BaseFloat>& X, float* part) {
  if (X.Rows() != 1 || X.Cols() != GetNInputs()) Error("CuRecurrent::PropagatePartial: one input row");
  if (mInputHistory.Rows() == 0) Error("Bptt order was not set");
  mOutput.Init(1, GetNOutputs());  // y_{t-1}: kept across frames (no-op when allocated, cumatrix.tcc:20-23)
  const int R = (int)mInputHistory.Rows();
  mHead = (mHead + R - 1) % R;
  if (mPending) {
    mPending = false;
    const int st = tnet_gemv_rowvec_partial_update(
        X.pCUData(), (int)X.Cols(), mOutput.pCUData(), (int)mOutput.Cols(), mInputHistory.pCURowData((size_t)mHead),
        mLinearity.pCUData(), (int)mLinearity.Stride(), (int)GetNOutputs(), part, mInputHistory.pCUData(),
        (int)mInputHistory.Stride(), mPendHead, R, mDiff.pCUData(), (int)mDiff.Stride(), mBpttOrder + 1,
        mBias.pCUData(), mBiasCorrection.pCUData(), mLearningRate, mMomentum, mWeightcost, S);
    if (st != TNET_ERR_UNSUPPORTED) {
      TNET_SAFE_CALL(st);
      return;
    }
    RunUpdate(mPendHead);  // (bptt > 8) on its own, before the forward reads W
  }
  TNET_SAFE_CALL(tnet_gemv_rowvec_partial(X.pCUData(), (int)X.Cols(), mOutput.pCUData(), (int)mOutput.Cols(),
                                          mInputHistory.pCURowData((size_t)mHead), mLinearity.pCUData(),
                                          (int)mLinearity.Stride(), (int)GetNOutputs(), part, S));
}

void CuRecurrent::BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuProfileScope p("CuRecurrent::Backpropagate");
  FlushPendingUpdate();
  // diff = e .* y(1-y) ; Y += W[0:nIn] diff  (OffsetGemv('N', beta = 1.0), cuRecurrent.cc:58-83:
  // the reference accumulates into the persistent error buffer; kept as is)
  mDiffTmp.Init(1, GetNOutputs());
  CuMath<BaseFloat>::DiffSigmoid(mDiffTmp, X, GetOutput());
  TNET_SAFE_CALL(tnet_gemv_rows(mLinearity.pCUData(), (int)mLinearity.Stride(), 0, (int)GetNInputs(),
                                (int)GetNOutputs(), mDiffTmp.pCUData(), Y.pCUData(), 1.0f, nullptr, S));
}

void CuRecurrent::Update() {
  CuProfileScope p("CuRecurrent::Update");
  FlushPendingUpdate();
  const int nIn = (int)GetNInputs(), nOut = (int)GetNOutputs(), R = (int)mInputHistory.Rows();
  // d_0 = e .* y(1-y) (present frame)
  CuMatrix<BaseFloat> d0;
  CuMatrix<BaseFloat>::MakeView(d0, mDiff.pCURowData(0), 1, (size_t)nOut, mDiff.Stride());
  CuMath<BaseFloat>::DiffSigmoid(d0, GetErrorInput(), GetOutput());
  UpdateFromDiff0();
}

void CuRecurrent::UpdateFromDiff0(bool defer) {
  FlushPendingUpdate();
  const int nIn = (int)GetNInputs(), nOut = (int)GetNOutputs();
  // BPTT: d_i = (W[nIn:nIn+nOut] d_{i-1}) .* y_{t-i}(1 - y_{t-i}), y_{t-i} = y part of history row i-1 --
  // one tnet_gemv_rows launch per step.  (Round 4's one-launch chain of the `order` steps, epoch-tagged granule
  // hand-offs, was measured slower -- 35.7 k vs 45.4 k frames/s at 135 senones, profiles/r04_rnn_chain_ab.json:
  // each step's all-to-all hand-off costs more than the launch boundary -- and is gone since round 6.)
  for (int i = 1; i <= mBpttOrder; i++)
    TNET_SAFE_CALL(tnet_gemv_rows(mLinearity.pCUData(), (int)mLinearity.Stride(), nIn, nOut, nOut,
                                  mDiff.pCURowData((size_t)i - 1), mDiff.pCURowData((size_t)i), 0.0f,
                                  HistRow(i - 1) + nIn, S));
  if (defer) {
    mPending = true;
    mPendHead = mHead;
    return;
  }
  RunUpdate(mHead);
}

// corr = sum_i -lr h_i (x) d_i ; corr += -lr wc W ; W += corr ; bias with momentum (cuRecurrent.cc:88-153)
void CuRecurrent::RunUpdate(int head) {
  const int nIn = (int)GetNInputs(), nOut = (int)GetNOutputs(), R = (int)mInputHistory.Rows();
  TNET_SAFE_CALL(tnet_rnn_update(mLinearity.pCUData(), (int)mLinearity.Stride(), nIn + nOut, nOut,
                                 mInputHistory.pCUData(), (int)mInputHistory.Stride(), head, R, mDiff.pCUData(),
                                 (int)mDiff.Stride(), mBpttOrder + 1, mBias.pCUData(), mBiasCorrection.pCUData(),
                                 mLearningRate, mMomentum, mWeightcost, S));
}

void CuRecurrent::FlushPendingUpdate() {
  if (!mPending) return;
  mPending = false;
  RunUpdate(mPendHead);
}

static uint64_t fbits(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  return u;
}

void CuRecurrent::ChainKey(std::vector<uint64_t>& k) const {
  for (const void* p : {(const void*)mLinearity.pCUData(), (const void*)mBias.pCUData(),
                        (const void*)mBiasCorrection.pCUData(), (const void*)mOutput.pCUData(),
                        (const void*)mInputHistory.pCUData(), (const void*)mDiff.pCUData()})
    k.push_back((uint64_t)(uintptr_t)p);
  k.insert(k.end(), {(uint64_t)mLinearity.Stride(), (uint64_t)mInputHistory.Rows(), (uint64_t)mInputHistory.Stride(),
                     (uint64_t)mDiff.Stride(), (uint64_t)mBpttOrder, (uint64_t)mHead, fbits(mLearningRate),
                     fbits(mMomentum), fbits(mWeightcost)});
}

void CuRecurrent::ReadFromStream(std::istream& rIn) {
  // W^T [nOut x (nIn + nOut)] then the bias (cuRecurrent.cc:158-168)
  BfMatrix transpose;
  ReadMatrixFast(rIn, transpose);
  if (transpose.Rows() != GetNOutputs() || transpose.Cols() != GetNInputs() + GetNOutputs())
    Error("Wrong dimensionalities of the <recurrent> matrix in network file");
  mLinearity.CopyFrom(BfMatrix(transpose, TRANS));
  BfVector bias;
  ReadVectorFast(rIn, bias);
  if (bias.Dim() != GetNOutputs()) Error("Wrong dimensionality of the <recurrent> bias");
  mBias.CopyFrom(bias);
}

void CuRecurrent::WriteToStream(std::ostream& rOut) {
  FlushPendingUpdate();
  BfMatrix tmp;
  mLinearity.CopyTo(tmp);
  rOut << BfMatrix(tmp, TRANS);
  BfVector vec;
  mBias.CopyTo(vec);
  rOut << vec << std::endl;
}

// ============================================================================ trainer
CuRecurrentTrainer::CuRecurrentTrainer(CuNetwork* net, CuObjectiveFunction* obj, int bptt, bool crossval)
    : mNet(net), mObj(obj), mCrossval(crossval) {
  // TRecurrentCu.cc:290-295
  for (int i = 0; i < net->Layers(); i++)
    if (net->Layer(i).GetType() == CuComponent::RECURRENT) dynamic_cast<CuRecurrent&>(net->Layer(i)).BpttOrder(bptt);
}

CuRecurrentTrainer::~CuRecurrentTrainer() {
  (void)hipStreamSynchronize(CuDevice::Instantiate().Stream());
  if (mSmx) (void)hipFree(mSmx);
  if (mArgKey) (void)hipFree(mArgKey);
  for (auto& kv : mGraphs) DestroyExecs(kv.second);
}

void CuRecurrentTrainer::DestroyExecs(ChainGraph& g) {
  for (auto e : g.execs) (void)hipGraphExecDestroy(e);
  g.execs.clear();
}

void* CuRecurrentTrainer::Scratch(void*& p, size_t& have, size_t bytes) {
  if (bytes > have) {
    if (p) {
      TNET_HIP_CALL(hipStreamSynchronize(CuDevice::Instantiate().Stream()));
      TNET_HIP_CALL(hipFree(p));
      p = nullptr;
      have = 0;
    }
    TNET_HIP_CALL(hipMalloc(&p, bytes));
    have = bytes;
  }
  return p;
}

void CuRecurrentTrainer::TrainUtterance(const float* feats, size_t rows, size_t cols, size_t ld,
                                        const int* labels) {
  if (cols != mNet->GetNInputs()) Error("CuRecurrentTrainer: feature dim != network input dim");
  if (rows == 0) return;
  CheckLabels(labels, rows, mNet->GetNOutputs(), "CuRecurrentTrainer::TrainUtterance");
  mFeats.Init(rows, cols);
  mFeats.CopyFromHost(feats, rows, cols, ld);
  mLabels.Init(rows);
  mLabels.CopyFromHost(labels, rows);
  // reset the history context (TRecurrentCu.cc:351-356)
  for (int i = 0; i < mNet->Layers(); i++)
    if (mNet->Layer(i).GetType() == CuComponent::RECURRENT) dynamic_cast<CuRecurrent&>(mNet->Layer(i)).ClearHistory();
  if (FusedFrameOk()) {
    // per-frame argmax keys of this utterance, read by tnet_argmax_correct at its end
    Scratch(mArgKey, mArgKeyBytes, rows * sizeof(unsigned long long));
    TNET_HIP_CALL(hipMemsetAsync(mArgKey, 0, rows * sizeof(unsigned long long), CuDevice::Instantiate().Stream()));
    RunFrames(rows);
    TNET_SAFE_CALL(tnet_argmax_correct((const unsigned long long*)mArgKey, mLabels.pCUData(), (int)rows,
                                       (int)mNet->GetNOutputs(), mObj->DeviceStats(), S));
    mFrames += (long)rows;
    return;
  }
  for (size_t f = 0; f < rows; f++) {
    CuMatrix<BaseFloat>::MakeView(mRow, mFeats.pCURowData(f), 1, cols, mFeats.Stride());
    CuVector<int>::MakeView(mLabelRow, mLabels.pCUData() + f, 1);
    mNet->Propagate(mRow, mOut);
    mObj->EvaluateLabels(mOut, mLabelRow, mErr);
    if (!mCrossval) mNet->Backpropagate(mErr);
  }
  mFrames += (long)rows;
}

bool CuRecurrentTrainer::GraphsEnabled() const {
  const char* e = getenv("TNET_RNN_GRAPH");
  if (e && e[0] == '0') return false;
  CuDevice& dev = CuDevice::Instantiate();
  // event records do not belong in a recorded chain; the legacy null stream cannot be captured
  return !dev.KernelTiming() && !dev.Profile() && dev.Stream() != nullptr;
}

// Every value the fused chain's launches take for an utterance of `rows` frames: the buffers (the
// features, labels, argmax keys, scratch, both layers' parameters, outputs and history), their
// strides, the ring head at the start and the hyper-parameters.  Equal keys => identical launches.
std::vector<uint64_t> CuRecurrentTrainer::ChainKey(size_t rows) {
  auto& rec = dynamic_cast<CuRecurrent&>(mNet->Layer(0));
  auto& lin = dynamic_cast<CuBiasedLinearity&>(mNet->Layer(1));
  std::vector<uint64_t> k = {(uint64_t)rows, (uint64_t)mCrossval};
  for (const void* p : {(const void*)mFeats.pCUData(), (const void*)mLabels.pCUData(), (const void*)mArgKey,
                        (const void*)mSmx, (const void*)mRecPart.pCUData(), (const void*)mOutPart.pCUData(),
                        (const void*)lin.Linearity().pCUData(), (const void*)lin.Bias().pCUData(),
                        (const void*)lin.LinearityCorrection().pCUData(), (const void*)lin.BiasCorrection().pCUData(),
                        (const void*)lin.Output().pCUData(), (const void*)lin.ErrorOutput().pCUData(),
                        (const void*)mObj->DeviceStats(), (const void*)mDotPart.pCUData(),
                        (const void*)mBnext.pCUData(), (const void*)mCbnext.pCUData()})
    k.push_back((uint64_t)(uintptr_t)p);
  k.push_back((uint64_t)AheadOn());
  float scale, l2;
  lin.UpdateConstants(1, &scale, &l2);
  k.insert(k.end(), {(uint64_t)mFeats.Stride(), (uint64_t)lin.Linearity().Stride(),
                     (uint64_t)lin.LinearityCorrection().Stride(), fbits(scale), fbits(l2), fbits(lin.Momentum())});
  rec.ChainKey(k);
  return k;
}

// The utterance's frames on the fused chain.  Per-frame launches are short (4-9 us), so the chain is
// recorded once per utterance length (stream capture of exactly the eager launches) and replayed as
// one hipGraph: the host submits one graph instead of ~9 launches a frame.  The host state the frames
// advance (ring head, frame count) is set as the recorded run left it.
void CuRecurrentTrainer::RunFrames(size_t rows) {
  const size_t cols = mFeats.Cols();
  mUttRows = rows;
  auto eager = [&](size_t f0, size_t f1) {
    for (size_t f = f0; f < f1; f++) {
      CuMatrix<BaseFloat>::MakeView(mRow, mFeats.pCURowData(f), 1, cols, mFeats.Stride());
      TrainFrameFused(f);
    }
  };
  if (!GraphsEnabled()) {
    eager(0, rows);
    return;
  }
  auto& rec = dynamic_cast<CuRecurrent&>(mNet->Layer(0));
  hipStream_t st = CuDevice::Instantiate().Stream();
  const std::vector<uint64_t> key = ChainKey(rows);
  auto it = mGraphs.find(rows);
  if (it == mGraphs.end()) {
    if (mGraphs.size() >= 64) {  // bounded: lengths beyond the first 64 distinct ones run eagerly
      eager(0, rows);
      return;
    }
    it = mGraphs.emplace(rows, ChainGraph()).first;
  }
  ChainGraph& g = it->second;
  if (!g.execs.empty() && g.key == key) {
    for (auto e : g.execs) TNET_HIP_CALL(hipGraphLaunch(e, st));
    rec.SetHead(g.head_after);
    mObj->AddFrames(rows);
    return;
  }
  if (g.key != key) {
    DestroyExecs(g);
    g.key = key;
    g.seen = 0;
  }
  if (++g.seen < 2) {  // first sighting: every buffer the chain touches gets allocated eagerly
    eager(0, rows);
    return;
  }
  static const size_t seg = [] {
    const char* e = getenv("TNET_RNN_GRAPH_FRAMES");
    const long v = e ? atol(e) : 96;
    return (size_t)(v > 0 ? v : 96);
  }();
  // record segment by segment, each launched right after its recording: the host state the frames
  // advance (ring head, frame count) moves exactly as in an eager run
  for (size_t f0 = 0; f0 < rows; f0 += seg) {
    const size_t f1 = std::min(rows, f0 + seg);
    hipGraph_t graph = nullptr;
    TNET_HIP_CALL(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    try {
      eager(f0, f1);  // recorded, not run
    } catch (...) {
      (void)hipStreamEndCapture(st, &graph);
      if (graph) (void)hipGraphDestroy(graph);
      DestroyExecs(g);
      g.seen = 0;
      throw;
    }
    TNET_HIP_CALL(hipStreamEndCapture(st, &graph));
    hipGraphExec_t exec = nullptr;
    const hipError_t e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) DestroyExecs(g);
    TNET_HIP_CALL(e);
    g.execs.push_back(exec);
    TNET_HIP_CALL(hipGraphLaunch(exec, st));
  }
  g.head_after = rec.Head();
}

// (Round 2's whole utterance as ONE persistent launch, rnn_persistent.hip, weights in LDS and in-launch granule
// hand-offs, was measured slower than the per-frame launch chain -- 61-62 us a frame vs ~35 us, the hand-offs
// 2.5-6.6 us each -- and is gone since round 6.)
bool CuRecurrentTrainer::FusedFrameOk() const {
  const char* generic = getenv("TNET_RNN_GENERIC");  // 1: the component-by-component chain (tests)
  if (generic && generic[0] == '1') return false;
  if (mNet->Layers() != 3 || mNet->Layer(0).GetType() != CuComponent::RECURRENT ||
      mNet->Layer(1).GetType() != CuComponent::BIASED_LINEARITY || mNet->Layer(2).GetType() != CuComponent::SOFTMAX ||
      !dynamic_cast<CuCrossEntropy*>(mObj) || mNet->Layer(2).GetNOutputs() > 4096 ||
      mNet->Layer(1).GetNInputs() > 2048)  // tnet_rnn_out_full's limits
    return false;
  if (mCrossval) return true;
  // both layers trained: the stopper is the recurrent layer (its error output is never formed)
  auto& rec = dynamic_cast<CuUpdatableComponent&>(mNet->Layer(0));
  auto& lin = dynamic_cast<CuUpdatableComponent&>(mNet->Layer(1));
  return rec.LearnRate() > 0.0f && lin.LearnRate() > 0.0f;
}

// One frame of TRecurrentCu.cc:360-368 on the fused kernels, the arithmetic of the generic
// Propagate / EvaluateLabels / Backpropagate chain: the recurrent split-K partials (+ the history
// push), the sigmoid finish fused with the output layer's split-K partials, z + the softmax pairs,
// the output layer's softmax error + backprop + update + the recurrent diff-sigmoid (+ xent and the
// frame's argmax key), then the BPTT GEMVs (bptt) and the recurrent update (1).  The network-output
// / softmax copies of the generic chain have no reader here and are not made.
bool CuRecurrentTrainer::AheadOn() const {
  static const bool on = !(getenv("TNET_RNN_AHEAD") && getenv("TNET_RNN_AHEAD")[0] == '0');
  return on && !mCrossval && dynamic_cast<const CuRecurrent&>(mNet->Layer(0)).AheadOk();
}

void CuRecurrentTrainer::TrainFrameFused(size_t f) {
  auto& rec = dynamic_cast<CuRecurrent&>(mNet->Layer(0));
  auto& lin = dynamic_cast<CuBiasedLinearity&>(mNet->Layer(1));
  const int nIn = (int)rec.GetNInputs(), H = (int)lin.GetNInputs(), N = (int)lin.GetNOutputs();
  const int hs = (nIn + H + 63) / 64, G = (N + 63) / 64;
  mRecPart.Init((size_t)hs, (size_t)H);
  double* smx = (double*)Scratch(mSmx, mSmxBytes, sizeof(double) * 2 * (size_t)G);
  lin.Output().Init(1, (size_t)N);
  // the look-ahead chain: this frame's forward product was taken by the previous frame's second launch (with the
  // weights before that frame's update; corrected here) -- one launch less a frame on the dependent chain
  const bool ahead = AheadOn();
  if (ahead) {
    mDotPart.Init((size_t)hs, 16);
    mBnext.Init((size_t)H);
    mCbnext.Init((size_t)H);
  }
  const bool corrected = ahead && f > 0 && mAheadNext;
  if (corrected) {
    const int pend = rec.AheadAdvance();
    if (pend < 0) Error("CuRecurrentTrainer: look-ahead frame without a pending update");
    TNET_SAFE_CALL(tnet_rnn_out_full_ahead(
        mRecPart.pCUData(), hs, rec.Bias().pCUData(), rec.Output().pCUData(), H, lin.Linearity().pCUData(),
        (int)lin.Linearity().Stride(), N, lin.Bias().pCUData(), lin.Output().pCUData(), smx, mDotPart.pCUData(),
        rec.DiffData(), rec.DiffStride(), rec.Steps(), rec.LearnRate(), rec.Momentum(), rec.Weightcost(),
        rec.BiasCorrection().pCUData(), mBnext.pCUData(), mCbnext.pCUData(), rec.Linearity().pCUData(),
        (int)rec.Linearity().Stride(), nIn + H, rec.HistoryData(), rec.HistoryStride(), pend, rec.HistoryRows(), S));
  } else {
    rec.PropagatePartial(mRow, mRecPart.pCUData());
    // (the partial kernel addresses [slices x cols] densely inside this allocation)
    TNET_SAFE_CALL(tnet_rnn_out_full(mRecPart.pCUData(), hs, rec.Bias().pCUData(), rec.Output().pCUData(), H,
                                     lin.Linearity().pCUData(), (int)lin.Linearity().Stride(), N, lin.Bias().pCUData(),
                                     lin.Output().pCUData(), smx, S));
  }
  float scale, l2;
  lin.UpdateConstants(1, &scale, &l2);
  const bool mmt = lin.Momentum() != 0.0f;
  lin.ErrorOutput().Init(1, (size_t)H);
  const bool next = f + 1 < mUttRows;
  mAheadNext = false;
  if (ahead) {
    // the output layer's backprop + update, the recurrent bias of the update applied above, and the next frame's
    // look-ahead product / dots / history push
    TNET_SAFE_CALL(tnet_rnn_out_bwd_update_ahead(
        lin.Output().pCUData(), smx, G, N, mLabels.pCUData() + f, rec.Output().pCUData(), H,
        lin.Linearity().pCUData(), (int)lin.Linearity().Stride(), mmt ? lin.LinearityCorrection().pCUData() : nullptr,
        (int)lin.LinearityCorrection().Stride(), lin.Bias().pCUData(), mmt ? lin.BiasCorrection().pCUData() : nullptr,
        scale, lin.Momentum(), l2, nullptr, lin.ErrorOutput().pCUData(), rec.DiffRow0(), mObj->DeviceStats(),
        (unsigned long long*)mArgKey + f, corrected ? mBnext.pCUData() : nullptr,
        corrected ? mCbnext.pCUData() : nullptr, rec.Bias().pCUData(), rec.BiasCorrection().pCUData(),
        next ? mFeats.pCURowData(f + 1) : nullptr, nIn, rec.Linearity().pCUData(), (int)rec.Linearity().Stride(),
        mRecPart.pCUData(), mDotPart.pCUData(),
        rec.HistoryData() + (long)rec.NextHead() * rec.HistoryStride(), rec.HistoryData(), rec.HistoryStride(),
        rec.Head(), rec.HistoryRows(), rec.Steps(), S));
    mAheadNext = next;
  } else {
    TNET_SAFE_CALL(tnet_rnn_out_bwd_update(
        lin.Output().pCUData(), smx, G, N, mLabels.pCUData() + f, rec.Output().pCUData(), H, lin.Linearity().pCUData(),
        (int)lin.Linearity().Stride(), mmt ? lin.LinearityCorrection().pCUData() : nullptr,
        (int)lin.LinearityCorrection().Stride(), lin.Bias().pCUData(), mmt ? lin.BiasCorrection().pCUData() : nullptr,
        scale, lin.Momentum(), l2, nullptr, nullptr, lin.ErrorOutput().pCUData(), rec.DiffRow0(), mObj->DeviceStats(),
        (unsigned long long*)mArgKey + f, mCrossval ? 0 : 1, S));
  }
  mObj->AddFrames(1);
  if (mCrossval) return;
  rec.UpdateFromDiff0(next);  // the last frame's update runs on its own: no state leaves the utterance
}

}  // namespace TNet
