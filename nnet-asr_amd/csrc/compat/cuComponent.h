// cuComponent.h -- drop-in header name of the reference (src/CuTNetLib/cuComponent.h): the MI355X CuTNetLib API lives in cucomponent.h.
#pragma once
#include "../host/cucomponent.h"
