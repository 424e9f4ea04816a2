// resolver.h -- origPtr of exactly periodic blocks.
//
// For a block w^k (k >= 2, |w| >= 2) the k copies of rotation 0 are identical; the
// reference's choice among them is an emergent property of its divsufsort internals
// (blocksort.c:946-956, 1050-1122).  The device sort returns rank0 = rank of rotation 0 among
// the |w| distinct rotations of w; this resolver turns it into the reference's origPtr.
#pragma once
#include <cstdint>
#include <vector>

namespace bzg {

struct ResolverFailure {};

// d_blk: device block bytes; boff/period/rank: host arrays for nb blocks.  On return
// rank[b] holds origPtr for every block.
void resolve_origptrs(const uint8_t* d_blk, const std::vector<uint32_t>& boff, const std::vector<uint32_t>& period,
                      std::vector<uint32_t>& rank);

// origPtr of one periodic block computed on the host (reference tie order).
int32_t periodic_origptr(const uint8_t* blk, int32_t n);

}  // namespace bzg
