// tieorder.h -- origPtr of exactly periodic blocks.
//
// For a block w^k (k >= 2, |w| >= 2) the k copies of every rotation are identical; the
// reference's choice among the copies of rotation 0 follows from the exchange sequence of its
// block sort (blocksort.c).  The device sort returns rank0 = the rank of rotation 0 among the
// |w| distinct rotations of w; tieorder.cpp adds the copy index (see the analysis there).
#pragma once
#include <cstdint>
#include <vector>

namespace bzg {

struct ResolverFailure {};

// d_blk: device block bytes; boff/period/rank: host arrays for nb blocks.  On entry rank[b] is
// the device sort's rank of rotation 0 among the period's rotations; on return the origPtr.
void resolve_origptrs(const uint8_t* d_blk, const std::vector<uint32_t>& boff, const std::vector<uint32_t>& period,
                      std::vector<uint32_t>& rank);

// Copy index of rotation 0 of the block w^(n/p) (p = primitive period, p < n).
int32_t periodic_copy_rank(const uint8_t* blk, int32_t n, int32_t p);

// origPtr of one periodic block computed on the host alone (test entry; needs no GPU).
int32_t periodic_origptr(const uint8_t* blk, int32_t n);

}  // namespace bzg
