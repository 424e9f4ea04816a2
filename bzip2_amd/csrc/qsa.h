// qsa.h -- sorted rotations of a quasi-periodic block (the pathological
// inputs of 8b config 4): a block t = w^k w' of length n whose smallest period p (t[i] ==
// t[i + p] for all i < n - p) does not divide n, with the block cyclically aperiodic.  The
// single-repeated-byte input ends in such a block ((aaaa\xfb)^k a after RLE1), which the
// general string sort only resolves after ~30 passes.  See qsa.cpp for the derivation.
#pragma once
#include <cstdint>
#include <vector>

namespace bzg {

constexpr uint32_t kQsaMaxPeriod = 256;  // periods handled analytically (blocks with n >= 2p)

// Smallest period p <= kQsaMaxPeriod with 2p <= n, of a block that is not a power of a shorter
// word (primitive_period(t, n) == n); 0 when there is none.  The device test (k_qperiod) follows
// the same rule.
uint32_t quasi_period(const uint8_t* t, uint32_t n);

// The order of the rotations of t = w^k w' (|w| = p, n = |t|) as a merge of two sorted lists:
// the "normal" rotations i <= n - p, which sort by the phase i mod p (phases in the order of
// the rotations of the cyclic word w) and, within a phase, by position (descending when desc),
// and the p - 1 "special" rotations i > n - p.
struct QsaPlan {
  uint32_t n = 0, p = 0;
  bool desc = false;
  std::vector<uint32_t> cum;   // p + 1: normals in the phases ord[0 .. k)
  std::vector<uint32_t> ord;   // p: phases in sorted order
  std::vector<uint32_t> lo;    // p - 1, ascending: normals before each special (specials in order)
  std::vector<uint32_t> srot;  // p - 1: the special rotations in sorted order
};

// w = t[0, p); requires p >= 2, n >= 2p, n % p != 0 and t cyclically aperiodic.
void qsa_plan(const uint8_t* w, uint32_t p, uint32_t n, QsaPlan& plan);

// Rotation at normal index y (0 <= y < n - p + 1) of the plan.
uint32_t qsa_normal_at(const QsaPlan& plan, uint32_t y);

// BWT (last column) and origPtr of the block from the plan (host; the device kernel k_qsa in
// sort.hip writes the same bytes).
uint32_t qsa_bwt(const QsaPlan& plan, const uint8_t* t, uint8_t* bwt);

}  // namespace bzg
