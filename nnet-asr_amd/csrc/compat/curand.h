// curand.h -- drop-in header name of the reference (src/CuBaseLib/curand.h): the MI355X CuTNetLib API lives in curbm.h.
#pragma once
#include "../host/curbm.h"
