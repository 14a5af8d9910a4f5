// tnet_common.h -- host-side error model and basic types of the MI355X TNet library.
//
// Mirrors the reference's error handling: every device call returns a status that is turned
// into a TNet::MyException with file/line/call text, as cuSafeCall does
// (src/CuBaseLib/cucommon.h:13-22) -- but WITHOUT the device synchronisation after each call.
#pragma once

#include <hip/hip_runtime_api.h>

#include <sstream>
#include <stdexcept>
#include <string>

#include "tnet_kernels.h"

#ifdef TNET_HOST_KALDILIB
// Drop-in build: the library is compiled against the reference's own KaldiLib
// (src/KaldiLib/Error.h, Types.h), so drivers such as TNetCu.cc exchange its Matrix / Vector /
// MyException types with the CuTNetLib API unchanged.
#include "Error.h"
#include "Types.h"
#else
namespace TNet {

typedef float BaseFloat;  // src/KaldiLib/Types.h:15-18 (DOUBLEPRECISION off)

class MyException : public std::runtime_error {
 public:
  explicit MyException(const std::string& s) : std::runtime_error(s) {}
};

[[noreturn]] inline void Error(const std::string& msg) { throw MyException(msg); }

inline void Warning(const std::string& msg);

}  // namespace TNet
#endif

#define TNET_SAFE_CALL(fun)                                                                       \
  do {                                                                                            \
    int _st = (fun);                                                                              \
    if (_st != 0) {                                                                               \
      std::ostringstream _os;                                                                     \
      _os << "TNET DEVICE ERROR #" << _st << " (" << tnet_status_str(_st) << ") " << __FILE__     \
          << ":" << __LINE__ << " " << __func__ << "() '" #fun "'";                               \
      throw TNet::MyException(_os.str());                                                         \
    }                                                                                             \
  } while (0)

#define TNET_HIP_CALL(fun)                                                                        \
  do {                                                                                            \
    hipError_t _e = (fun);                                                                        \
    if (_e != hipSuccess) {                                                                       \
      std::ostringstream _os;                                                                     \
      _os << "HIP ERROR #" << (int)_e << " " << __FILE__ << ":" << __LINE__ << " " << __func__    \
          << "() '" #fun "' " << hipGetErrorString(_e);                                           \
      throw TNet::MyException(_os.str());                                                         \
    }                                                                                             \
  } while (0)

#ifndef TNET_HOST_KALDILIB
#include <iostream>
inline void TNet::Warning(const std::string& msg) { std::cerr << "WARNING " << msg << std::endl; }
#endif

namespace TNet {
// Class-id targets at intake: each label names an output column, or is < 0 (an unlabeled row, the
// all-zero target row of the reference's one-hot matrix).  The reference cannot hold an
// out-of-range id (LabelRepository::GenDesiredMatrix builds [T x n_out] one-hot rows,
// src/KaldiLib/Labels.cc:44-187); here a label >= n_out would index past the softmax row.
inline void CheckLabels(const int* labels, size_t rows, size_t n_out, const char* who) {
  if (rows && !labels) Error(std::string(who) + ": labels pointer is null");
  for (size_t r = 0; r < rows; r++) {
    if (labels[r] >= 0 && (size_t)labels[r] >= n_out) {
      std::ostringstream os;
      os << who << ": label " << labels[r] << " of frame " << r << " is outside [0, " << n_out << ")";
      Error(os.str());
    }
  }
}
}  // namespace TNet
