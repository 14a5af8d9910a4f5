// cuobjective.cpp -- see cuobjective.h.
#include "cuobjective.h"

namespace TNet {

#define S ((void*)CuDevice::Instantiate().Stream())

CuObjectiveFunction* CuObjectiveFunction::Factory(ObjFunType type) {
  switch (type) {
    case MEAN_SQUARE_ERROR: return new CuMeanSquareError;
    case CROSS_ENTROPY: return new CuCrossEntropy;
    default: Error("Unknown ObjFun type");
  }
}

CuObjectiveFunction::CuObjectiveFunction() {
  CuDevice& d = CuDevice::Instantiate();
  mDevStats = (double*)d.Alloc(TNET_STATS_WORDS * sizeof(double));
  TNET_HIP_CALL(hipMemsetAsync(mDevStats, 0, TNET_STATS_WORDS * sizeof(double), d.Stream()));
}

CuObjectiveFunction::~CuObjectiveFunction() {
  if (mDevStats) CuDevice::Instantiate().Free(mDevStats, TNET_STATS_WORDS * sizeof(double));
}

void CuObjectiveFunction::Sync() {
  CuDevice& d = CuDevice::Instantiate();
  double e = 0.0, c = 0.0;
  TNET_SAFE_CALL(tnet_stats_fetch(mDevStats, &e, &c, d.Stream()));
  TNET_HIP_CALL(hipMemsetAsync(mDevStats, 0, TNET_STATS_WORDS * sizeof(double), d.Stream()));
  mError += e;
  mCorrect += c;
}

double CuObjectiveFunction::GetError() {
  Sync();
  return mError;
}
double CuObjectiveFunction::GetCorrect() {
  Sync();
  return mCorrect;
}

void CuObjectiveFunction::MergeTotals(double err, size_t frames, double correct) {
  mError += err;
  mFrames += frames;
  mCorrect += correct;
}

void CuObjectiveFunction::Reset() {
  Sync();
  mError = 0;
  mCorrect = 0;
  mFrames = 0;
}

void CuObjectiveFunction::EvaluateLabels(const CuMatrix<BaseFloat>&, const CuVector<int>&, CuMatrix<BaseFloat>&) {
  Error(std::string(GetTypeLabel()) + ": class-id targets not supported");
}

// ---------------------------------------------------------------------------- MSE
void CuMeanSquareError::Evaluate(const CuMatrix<BaseFloat>& out, const CuMatrix<BaseFloat>& des,
                                 CuMatrix<BaseFloat>& err) {
  CuProfileScope p("CuMeanSquareError::Evaluate");
  // err = out - des ; mError += sum err^2   (cuObjectiveFunction.cc:28-45)
  if (out.Rows() != des.Rows() || out.Cols() != des.Cols()) Error("CuMeanSquareError: non-matching dims");
  err.Init(out.Rows(), out.Cols());
  TNET_SAFE_CALL(tnet_mse(out.pCUData(), out.Dim(), des.pCUData(), (int)des.Stride(), err.pCUData(), (int)err.Stride(),
                          mDevStats, S));
  mFrames += out.Rows();
}

void CuMeanSquareError::EvaluateStats(const CuMatrix<BaseFloat>& out, const CuMatrix<BaseFloat>& des) {
  if (out.Rows() != des.Rows() || out.Cols() != des.Cols()) Error("CuMeanSquareError: non-matching dims");
  TNET_SAFE_CALL(tnet_mse(out.pCUData(), out.Dim(), des.pCUData(), (int)des.Stride(), nullptr, 0, mDevStats, S));
  mFrames += out.Rows();
}

std::string CuMeanSquareError::Report() {
  Sync();
  std::ostringstream ss;
  ss << "Mse:" << mError << " frames:" << mFrames << " err/frm:" << mError / mFrames << "\n";
  return ss.str();
}

// ---------------------------------------------------------------------------- Xent
void CuCrossEntropy::Evaluate(const CuMatrix<BaseFloat>& out, const CuMatrix<BaseFloat>& des,
                              CuMatrix<BaseFloat>& err) {
  CuProfileScope p("CuCrossEntropy::Evaluate");
  if (des.Cols() != out.Cols() || des.Rows() != out.Rows()) {
    std::ostringstream os;
    os << "Non-matching dimensions of network output with training targets!!!"
       << " Netoutput:" << out.Cols() << " Targets:" << des.Cols();
    Error(os.str());
  }
  // err = y - d; correct += argmax match; xent += -sum d log(max(y, FLT_MIN))  (one kernel)
  err.Init(out.Rows(), out.Cols());
  TnetMatrixDim d = out.Dim();
  TNET_SAFE_CALL(tnet_softmax_xent_dense(nullptr, d, des.pCUData(), (int)des.Stride(), const_cast<float*>(out.pCUData()),
                                         (int)out.Stride(), err.pCUData(), (int)err.Stride(), mDevStats, S));
  mFrames += out.Rows();
}

void CuCrossEntropy::EvaluateLabels(const CuMatrix<BaseFloat>& out, const CuVector<int>& labels,
                                    CuMatrix<BaseFloat>& err) {
  CuProfileScope p("CuCrossEntropy::Evaluate");
  if (labels.Dim() != out.Rows()) Error("CuCrossEntropy: number of labels != rows");
  err.Init(out.Rows(), out.Cols());
  TNET_SAFE_CALL(tnet_softmax_xent(nullptr, out.Dim(), labels.pCUData(), const_cast<float*>(out.pCUData()),
                                   (int)out.Stride(), err.pCUData(), (int)err.Stride(), mDevStats, S));
  mFrames += out.Rows();
}

std::string CuCrossEntropy::Report() {
  Sync();
  std::ostringstream ss;
  // cuObjectiveFunction.h:132-144 (same fields, same default 6-digit precision)
  ss << "Xent:" << mError << " frames:" << mFrames << " err/frm:" << mError / mFrames << " correct["
     << 100.0 * mCorrect / mFrames << "%]"
     << "\n";
  return ss.str();
}

}  // namespace TNet
