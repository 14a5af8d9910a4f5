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
