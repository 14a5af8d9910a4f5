// cuObjectiveFunction.h -- drop-in header name of the reference (src/CuTNetLib/cuObjectiveFunction.h): the MI355X CuTNetLib API lives in cuobjective.h.
#pragma once
#include "../host/cuobjective.h"
