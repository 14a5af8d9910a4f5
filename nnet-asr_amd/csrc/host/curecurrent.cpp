// curecurrent.cpp -- see curecurrent.h.
#include "curecurrent.h"

#include <cstdlib>

#include "cunetwork.h"

namespace TNet {

#define S ((void*)CuDevice::Instantiate().Stream())

void CuRecurrent::BpttOrder(int ord) {
  if (ord < 0) Error("CuRecurrent::BpttOrder: negative order");
  mBpttOrder = ord;
  mInputHistory.Init((size_t)ord + 1, GetNInputs() + GetNOutputs());
  mDiff.Init((size_t)ord + 1, GetNOutputs());
  mDiffTmp.Init(1, GetNOutputs());
  mHead = 0;
}

void CuRecurrent::ClearHistory() {
  mInputHistory.SetZero();
  if (mOutput.MSize() > 0) mOutput.SetZero();
  mHead = 0;
}

void CuRecurrent::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuProfileScope p("CuRecurrent::Propagate");
  if (X.Rows() != 1 || Y.Rows() != 1) Error("CuRecurrent: frame-by-frame (one row) propagation only");
  if (mInputHistory.Rows() == 0) Error("Bptt order was not set");
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

void CuRecurrent::BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuProfileScope p("CuRecurrent::Backpropagate");
  // diff = e .* y(1-y) ; Y += W[0:nIn] diff  (OffsetGemv('N', beta = 1.0), cuRecurrent.cc:58-83:
  // the reference accumulates into the persistent error buffer; kept as is)
  mDiffTmp.Init(1, GetNOutputs());
  CuMath<BaseFloat>::DiffSigmoid(mDiffTmp, X, GetOutput());
  TNET_SAFE_CALL(tnet_gemv_rows(mLinearity.pCUData(), (int)mLinearity.Stride(), 0, (int)GetNInputs(),
                                (int)GetNOutputs(), mDiffTmp.pCUData(), Y.pCUData(), 1.0f, nullptr, S));
}

void CuRecurrent::Update() {
  CuProfileScope p("CuRecurrent::Update");
  const int nIn = (int)GetNInputs(), nOut = (int)GetNOutputs(), R = (int)mInputHistory.Rows();
  // d_0 = e .* y(1-y) (present frame)
  CuMatrix<BaseFloat> d0;
  CuMatrix<BaseFloat>::MakeView(d0, mDiff.pCURowData(0), 1, (size_t)nOut, mDiff.Stride());
  CuMath<BaseFloat>::DiffSigmoid(d0, GetErrorInput(), GetOutput());
  UpdateFromDiff0();
}

void CuRecurrent::UpdateFromDiff0() {
  const int nIn = (int)GetNInputs(), nOut = (int)GetNOutputs(), R = (int)mInputHistory.Rows();
  // BPTT: d_i = (W[nIn:nIn+nOut] d_{i-1}) .* y_{t-i}(1 - y_{t-i}), y_{t-i} = y part of history row i-1
  for (int i = 1; i <= mBpttOrder; i++)
    TNET_SAFE_CALL(tnet_gemv_rows(mLinearity.pCUData(), (int)mLinearity.Stride(), nIn, nOut, nOut,
                                  mDiff.pCURowData((size_t)i - 1), mDiff.pCURowData((size_t)i), 0.0f,
                                  HistRow(i - 1) + nIn, S));
  // corr = sum_i -lr h_i (x) d_i ; corr += -lr wc W ; W += corr ; bias with momentum (cuRecurrent.cc:88-153)
  TNET_SAFE_CALL(tnet_rnn_update(mLinearity.pCUData(), (int)mLinearity.Stride(), nIn + nOut, nOut,
                                 mInputHistory.pCUData(), (int)mInputHistory.Stride(), mHead, R, mDiff.pCUData(),
                                 (int)mDiff.Stride(), mBpttOrder + 1, mBias.pCUData(), mBiasCorrection.pCUData(),
                                 mLearningRate, mMomentum, mWeightcost, S));
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
  const bool fused = FusedFrameOk();
  for (size_t f = 0; f < rows; f++) {
    CuMatrix<BaseFloat>::MakeView(mRow, mFeats.pCURowData(f), 1, cols, mFeats.Stride());
    if (fused) {
      TrainFrameFused(f);
      continue;
    }
    CuVector<int>::MakeView(mLabelRow, mLabels.pCUData() + f, 1);
    mNet->Propagate(mRow, mOut);
    mObj->EvaluateLabels(mOut, mLabelRow, mErr);
    if (!mCrossval) mNet->Backpropagate(mErr);
  }
  mFrames += (long)rows;
}

bool CuRecurrentTrainer::FusedFrameOk() const {
  const char* generic = getenv("TNET_RNN_GENERIC");  // 1: the component-by-component chain (tests)
  if (generic && generic[0] == '1') return false;
  if (mNet->Layers() != 3 || mNet->Layer(0).GetType() != CuComponent::RECURRENT ||
      mNet->Layer(1).GetType() != CuComponent::BIASED_LINEARITY || mNet->Layer(2).GetType() != CuComponent::SOFTMAX ||
      !dynamic_cast<CuCrossEntropy*>(mObj) || mNet->Layer(2).GetNOutputs() > 4096)
    return false;
  if (mCrossval) return true;
  // both layers trained: the stopper is the recurrent layer (its error output is never formed)
  auto& rec = dynamic_cast<CuUpdatableComponent&>(mNet->Layer(0));
  auto& lin = dynamic_cast<CuUpdatableComponent&>(mNet->Layer(1));
  return rec.LearnRate() > 0.0f && lin.LearnRate() > 0.0f;
}

// One frame of TRecurrentCu.cc:360-368 on the fused kernels, the same arithmetic as the generic
// Propagate / EvaluateLabels / Backpropagate chain: the recurrent forward (2 launches: split-K
// partials that also push the history row, + the sigmoid finish), output layer + softmax +
// cross-entropy (2), output-layer backprop + update + the recurrent diff-sigmoid (1), the BPTT
// GEMVs (bptt) and the recurrent update (1).  The network-output / softmax-error copies of the
// generic chain have no reader here and are not made.
void CuRecurrentTrainer::TrainFrameFused(size_t f) {
  auto& rec = dynamic_cast<CuRecurrent&>(mNet->Layer(0));
  auto& lin = dynamic_cast<CuBiasedLinearity&>(mNet->Layer(1));
  CuComponent& sm = mNet->Layer(2);
  rec.SetInput(mRow);
  rec.Propagate();
  const int H = (int)lin.GetNInputs(), N = (int)lin.GetNOutputs();
  lin.Output().Init(1, (size_t)N);
  sm.Output().Init(1, (size_t)N);
  mErr.Init(1, (size_t)N);
  void* ws = CuDevice::Instantiate().Workspace((size_t)tnet_gemv_workspace(H, N));
  TNET_SAFE_CALL(tnet_gemv_rowvec_softmax_xent(rec.GetOutput().pCUData(), H, lin.Linearity().pCUData(),
                                               (int)lin.Linearity().Stride(), lin.Bias().pCUData(),
                                               lin.Output().pCUData(), sm.Output().pCUData(),
                                               mCrossval ? nullptr : mErr.pCUData(), N, mLabels.pCUData() + f,
                                               mObj->DeviceStats(), ws, S));
  mObj->AddFrames(1);
  if (mCrossval) return;
  lin.BackpropUpdateRow(rec.GetOutput(), mErr, lin.ErrorOutput(), rec.GetOutput().pCUData(), rec.DiffRow0());
  rec.UpdateFromDiff0();
}

}  // namespace TNet
