// cuNetwork.h -- drop-in header name of the reference (src/CuTNetLib/cuNetwork.h): the MI355X CuTNetLib API lives in cunetwork.h.
#pragma once
#include "../host/cunetwork.h"
