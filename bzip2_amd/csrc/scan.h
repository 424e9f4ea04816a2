// scan.h -- device-wide prefix scans over u32 arrays (sum or max), tile-reduce /
// scan-of-aggregates / tile-apply with recursion on the aggregates.
#pragma once
#include "common.h"

namespace bzg {

enum class ScanOp { Sum, Max };

// Scratch requirement (in u32 words) for scan_u32 over n elements.
size_t scan_scratch_words(size_t n);

// out[i] = op(in[0..i)) (exclusive, identity 0) or op(in[0..i]) (inclusive).
// `total` (device pointer, may be null) receives op over all n elements.
// in and out may alias.  `scratch` needs scan_scratch_words(n) words.
void scan_u32(ScanOp op, bool exclusive, const uint32_t* in, uint32_t* out, size_t n,
              uint32_t* total, uint32_t* scratch, hipStream_t st);

}  // namespace bzg
