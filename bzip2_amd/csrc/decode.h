// decode.h -- CPU decoder behind BZ2_bzDecompress* (the reference's decoder, decompress.c, is
// outside the accelerated path).  Declared for bzlib_api.cpp.
#pragma once
#include "../../include/bzlib.h"
