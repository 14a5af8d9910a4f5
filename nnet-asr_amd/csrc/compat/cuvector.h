// cuvector.h -- drop-in header name of the reference (src/CuBaseLib/cuvector.h): the MI355X CuTNetLib API lives in cumatrix.h.
#pragma once
#include "../host/cumatrix.h"
