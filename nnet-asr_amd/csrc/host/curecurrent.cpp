// curecurrent.cpp -- see curecurrent.h.
#include "curecurrent.h"

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
  hipStream_t st = CuDevice::Instantiate().Stream();
  // row 0 = [x_t, y_{t-1}]: Y still holds the previous frame's output (cuRecurrent.cc:31-35)
  TNET_HIP_CALL(hipMemcpyAsync(row, X.pCUData(), sizeof(float) * X.Cols(), hipMemcpyDeviceToDevice, st));
  TNET_HIP_CALL(hipMemcpyAsync(row + X.Cols(), Y.pCUData(), sizeof(float) * Y.Cols(), hipMemcpyDeviceToDevice, st));
  // y_t = sigmoid(b + row W) (AddScaledRow + OffsetGemv('T') + Sigmoid, cuRecurrent.cc:41-47)
  const int K = (int)(GetNInputs() + GetNOutputs()), N = (int)GetNOutputs();
  void* ws = CuDevice::Instantiate().Workspace((size_t)tnet_gemv_workspace(K, N));
  TNET_SAFE_CALL(tnet_gemv_rowvec(row, K, mLinearity.pCUData(), (int)mLinearity.Stride(), mBias.pCUData(),
                                  Y.pCUData(), N, 1, ws, S));
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
  mFeats.Init(rows, cols);
  mFeats.CopyFromHost(feats, rows, cols, ld);
  mLabels.Init(rows);
  mLabels.CopyFromHost(labels, rows);
  // reset the history context (TRecurrentCu.cc:351-356)
  for (int i = 0; i < mNet->Layers(); i++)
    if (mNet->Layer(i).GetType() == CuComponent::RECURRENT) dynamic_cast<CuRecurrent&>(mNet->Layer(i)).ClearHistory();
  for (size_t f = 0; f < rows; f++) {
    CuMatrix<BaseFloat>::MakeView(mRow, mFeats.pCURowData(f), 1, cols, mFeats.Stride());
    CuVector<int>::MakeView(mLabelRow, mLabels.pCUData() + f, 1);
    mNet->Propagate(mRow, mOut);
    mObj->EvaluateLabels(mOut, mLabelRow, mErr);
    if (!mCrossval) mNet->Backpropagate(mErr);
  }
  mFrames += (long)rows;
}

}  // namespace TNet
