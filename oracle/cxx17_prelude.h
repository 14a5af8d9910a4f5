// cxx17_prelude.h -- forced include (-include) when the reference's C++98 sources (TNetCu.cc,
// KaldiLib headers) are compiled in the drop-in build next to our C++17 headers: C++98's <math.h>
// put isnan / isinf in the global namespace, <cmath> since C++11 only in std.  Test
// infrastructure only (oracle/Makefile.dropin).
#pragma once
#include <cmath>
using std::isinf;
using std::isnan;
