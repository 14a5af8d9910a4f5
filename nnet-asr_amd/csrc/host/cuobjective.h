// cuobjective.h -- CuObjectiveFunction / CuCrossEntropy / CuMeanSquareError
// (src/CuTNetLib/cuObjectiveFunction.h:20-157, .cc:28-83).
//
// MI355X changes: the per-bunch statistics are accumulated ON THE DEVICE (two fp64 words updated
// by the objective kernel) and copied back only when GetError()/Report() asks -- the reference
// does two D2H copies + host sums per bunch (cuObjectiveFunction.cc:68,78).  One-hot targets can
// be passed as class ids (4 B/frame) instead of a dense [rows x classes] matrix.
#pragma once

#include "cumatrix.h"

namespace TNet {

class CuObjectiveFunction {
 public:
  typedef enum { OBJ_FUN_I = 0x0300, MEAN_SQUARE_ERROR, CROSS_ENTROPY } ObjFunType;
  static CuObjectiveFunction* Factory(ObjFunType type);

  CuObjectiveFunction();
  virtual ~CuObjectiveFunction();
  virtual ObjFunType GetTypeId() = 0;
  virtual const char* GetTypeLabel() = 0;

  /// evaluates the data (dense desired matrix), computes the global error
  virtual void Evaluate(const CuMatrix<BaseFloat>& rNetOutput, const CuMatrix<BaseFloat>& rDesired,
                        CuMatrix<BaseFloat>& rNetError) = 0;
  /// class-id targets (label < 0 = unlabeled frame, all-zero target row)
  virtual void EvaluateLabels(const CuMatrix<BaseFloat>& rNetOutput, const CuVector<int>& rLabels,
                              CuMatrix<BaseFloat>& rNetError);

  virtual double GetError();
  virtual size_t GetFrames() { return mFrames; }
  virtual std::string Report() = 0;

  /// device accumulator words {error, correct} (for the fused kernels and DP merging)
  double* DeviceStats() { return mDevStats; }
  void AddFrames(size_t n) { mFrames += n; }
  /// Pull device statistics to host (synchronises the stream).
  void Sync();
  /// MergeStats (src/TNetLib/ObjFun.cc:214-230) -- adds another instance's totals
  void MergeTotals(double err, size_t frames, double correct);
  double GetCorrect();
  void Reset();

 protected:
  double* mDevStats = nullptr;  // [0]=error sum, [1]=correct count
  double mError = 0.0;           // host totals already pulled
  double mCorrect = 0.0;
  size_t mFrames = 0;
};

class CuMeanSquareError : public CuObjectiveFunction {
 public:
  ObjFunType GetTypeId() override { return MEAN_SQUARE_ERROR; }
  const char* GetTypeLabel() override { return "<mean_square_error>"; }
  void Evaluate(const CuMatrix<BaseFloat>& rNetOutput, const CuMatrix<BaseFloat>& rDesired,
                CuMatrix<BaseFloat>& rNetError) override;
  /// statistics only (the error matrix is not needed, e.g. the RBM reconstruction error)
  void EvaluateStats(const CuMatrix<BaseFloat>& rNetOutput, const CuMatrix<BaseFloat>& rDesired);
  std::string Report() override;
};

class CuCrossEntropy : public CuObjectiveFunction {
 public:
  ObjFunType GetTypeId() override { return CROSS_ENTROPY; }
  const char* GetTypeLabel() override { return "<cross_entropy>"; }
  void Evaluate(const CuMatrix<BaseFloat>& rNetOutput, const CuMatrix<BaseFloat>& rDesired,
                CuMatrix<BaseFloat>& rNetError) override;
  void EvaluateLabels(const CuMatrix<BaseFloat>& rNetOutput, const CuVector<int>& rLabels,
                      CuMatrix<BaseFloat>& rNetError) override;
  std::string Report() override;
};

}  // namespace TNet
