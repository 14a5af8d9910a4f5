// cuRecurrent.h -- drop-in header name of the reference (src/CuTNetLib/cuRecurrent.h): the MI355X CuTNetLib API lives in curecurrent.h.
#pragma once
#include "../host/curecurrent.h"
