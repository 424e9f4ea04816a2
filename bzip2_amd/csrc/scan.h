// scan.h -- device-wide prefix scans over u32 arrays (sum or max): up to 64 tiles of 4096 one
// launch with decoupled look-back, above that three passes (scan.hip).
#pragma once
#include "common.h"

namespace bzg {

enum class ScanOp { Sum, Max };

// Scratch requirement (in u32 words) for scan_u32 over n elements.
size_t scan_scratch_words(size_t n);

// out[i] = op(in[0..i)) (exclusive, identity 0) or op(in[0..i]) (inclusive).
// `total` (device pointer, may be null) receives op over all n elements.
// in and out may alias.  `scratch` needs scan_scratch_words(n) words, zero when first used
// (Workspace::u32z); every scan leaves it zero again.  Scans on one scratch must be ordered
// (one stream).
void scan_u32(ScanOp op, bool exclusive, const uint32_t* in, uint32_t* out, size_t n,
              uint32_t* total, uint32_t* scratch, hipStream_t st);

}  // namespace bzg
