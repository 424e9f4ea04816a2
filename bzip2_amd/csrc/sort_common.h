// sort_common.h -- shared types of the A4 block sorter (sort.hip: text-key string sort;
// sortdbl.hip: prefix-doubling fallback for groups that stay unresolved to a large depth).
#pragma once
#include "stages.h"

namespace bzg {

// One unit per block: the block's primitive root (the whole block when aperiodic).
// Slots [sbase, sbase + len) hold the unit's sorted rotations; k = copies of the root.
struct Unit {
  uint32_t sbase, len, toff, k;
};

// A group of slots whose rotations are known equal to some depth.
// flags: bit0 = data lives in the alternate buffers (sa2/sk2), bit1 = identity (slot e holds
// rotation e; nothing stored yet), bits 2-4 = valid bytes of the members' key caches (S1),
// bits 5.. = depth (characters known equal).
struct Grp {
  uint32_t start, size, unit, flags;
};
constexpr uint32_t kGrpAlt = 1u, kGrpIdent = 2u;
constexpr uint32_t kGrpDepthShift = 5;
__host__ __device__ inline uint32_t grp_depth(const Grp& g) { return g.flags >> kGrpDepthShift; }
__host__ __device__ inline uint32_t grp_cache(const Grp& g) { return (g.flags >> 2) & 7u; }
__host__ __device__ inline uint32_t grp_flags(uint32_t alt, uint32_t depth, uint32_t cache) {
  return alt | (cache << 2) | (depth << kGrpDepthShift);
}

struct SortBufs {
  uint32_t *sa, *isa, *key, *sa2, *key2;
  uint32_t *sk, *sk2;  // S1 key caches beside sa / sa2: the next characters, most significant first
  const uint8_t* text;
  const Unit* units;
  uint32_t dwave;  // S2 gives a tied group to the doubling fallback (S3) at this depth
  uint32_t dwave_tiny;  // the same for groups of <= 8 rotations (k_tiny)
};

// Largest g with P[g] <= x (P is an exclusive prefix, P[0] = 0).
__device__ __forceinline__ uint32_t upper_idx(const uint32_t* __restrict__ P, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Prefix doubling (Manber-Myers / Larsson-Sadakane) over the groups in L, all of which are
// known equal to depth >= h, with B.isa holding for every slot of every affected unit the
// first slot of its group.  On return every group is resolved: SA and ISA are final.
void doubling_sort(Workspace& ws, const SortBufs& B, const Grp* L0, uint32_t nL0, uint32_t h,
                   int* iterations, uint64_t* revisited, hipStream_t st);

}  // namespace bzg
