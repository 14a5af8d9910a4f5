// cuCache.h -- drop-in header name of the reference (src/CuTNetLib/cuCache.h): the MI355X CuTNetLib API lives in cucache.h.
#pragma once
#include "../host/cucache.h"
