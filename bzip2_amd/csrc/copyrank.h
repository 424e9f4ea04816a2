// copyrank.h -- A5: which of the k identical copies of rotation 0 the reference ranks first
// in a block w^k.  copy_rank is derived from
// divsufsort as modified in the reference's blocksort.c (MIT notice and citations at the top
// of copyrank.cpp); the one-B*-per-period closed form is original and also runs on the device
// (origptr.hip).
#pragma once
#include <cstdint>

namespace bzg {

struct CopyRankFailure {};

// Largest number of B* offsets per root the device closed form (origptr.hip k_copyrank_cf)
// evaluates; copy_rank_distinct applies the same cap so that it reports what the device does.
constexpr int32_t kCopyRankQMax = 1024;
// ... and the bound on its class comparisons: a root of at most kCopyRankPMax bytes with
// q * p <= kCopyRankCmpMax (a thread compares one class with the others, at most p bytes; a
// workgroup at most q * p), longer roots go to the host model
constexpr int32_t kCopyRankPMax = 16384;
constexpr int64_t kCopyRankCmpMax = 1ll << 22;

// B* structure of the cyclic root w (|w| = p >= 2, primitive): number of B* offsets q.
int32_t root_bstar_count(const uint8_t* w, int32_t p);

// Closed form for q == 1 (copyrank.cpp section 4); -1 when q != 1.
int32_t copy_rank_single(const uint8_t* w, int32_t p, int32_t k);

// Closed form for q >= 2 whose B* classes have pairwise different keys, the first class alone in
// its (c0, c1) bucket, when the reference's rank-stage budget lasts (copyrank_cf.cpp); -1 when
// the rule does not apply.
int32_t copy_rank_distinct(const uint8_t* w, int32_t p, int32_t k);

// Copy index r of rotation 0 of the block w^k (k >= 2, w primitive, |w| >= 2).
int32_t copy_rank(const uint8_t* w, int32_t p, int32_t k);

// Rank of rotation 0 among the p distinct rotations of w.
int32_t root_rotation_rank(const uint8_t* w, int32_t p);

// Smallest period p dividing n with t = t[0,p)^(n/p); n when aperiodic.
int32_t primitive_period(const uint8_t* t, int32_t n);

}  // namespace bzg
