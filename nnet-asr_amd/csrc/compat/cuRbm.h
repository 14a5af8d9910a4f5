// cuRbm.h -- drop-in header name of the reference (src/CuTNetLib/cuRbm.h): the MI355X CuTNetLib API lives in curbm.h.
#pragma once
#include "../host/curbm.h"
