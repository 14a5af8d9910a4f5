// cumath.h -- CuMath statics (src/CuBaseLib/cumath.h:15-142) on the gfx950 kernels.
#pragma once

#include "cumatrix.h"

namespace TNet {

template <typename T>
class CuMath;

template <>
class CuMath<BaseFloat> {
 public:
  /// Y = 1/(1+exp(-X))                                    (cumath.cc:13-25)
  static void Sigmoid(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X);
  /// Eout = Y(1-Y) Ein                                     (cumath.cc:27-39)
  static void DiffSigmoid(CuMatrix<BaseFloat>& Eout, const CuMatrix<BaseFloat>& Ein, const CuMatrix<BaseFloat>& Y);
  /// row softmax                                            (cumath.cc:42-74)
  static void Softmax(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X);
  /// per-block linear transform (front end <blocklinearity>) (cumath.cc:78-113)
  static void BlockLinearity(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X,
                             const CuMatrix<BaseFloat>& block_transf);
  /// frame-context splice with edge clamp                   (cumath.cc:118-133)
  static void Expand(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X, const CuVector<int>& frameOffsets);
  /// column gather                                          (cumath.cc:136-151)
  static void Rearrange(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X, const CuVector<int>& copyFrom);
  /// row gather                                             (cumath.cc:155-174)
  static void Randomize(CuMatrix<BaseFloat>& Y, const CuMatrix<BaseFloat>& X, const CuVector<int>& copyFrom);
  /// argmax(out)==argmax(des) per row                       (cumath.cc:178-206)
  static void CheckClass(const CuMatrix<BaseFloat>& out, const CuMatrix<BaseFloat>& des, CuVector<int>& match);
};

}  // namespace TNet
