// copyrank_cf.cpp -- A5 closed forms for periodic roots with several B* offsets (SURVEY.md
// section 8a row A5, section 8f row 4).  Original: these are derived from the behaviour of the
// reference's block sort on k identical copies (checked against the reference build and the
// copy-rank model), not from divsufsort code.  origptr.hip evaluates the same rules on the
// device; this host version is their specification and the parity tests' mirror.
//
// Setting (copyrank.cpp sections 1-2): a block T = w^k, w primitive, |w| = p, with q >= 2 B*
// offsets off[0] < ... < off[q-1] in w; B* item x = j q + c is copy j of class c.  We need r, the
// rank of copy 0 of class 0 among the k copies of class 0.
//
// Distinct classes.  When the q classes have pairwise different full keys (first two
// characters, then the B* substring: copyrank.cpp's class rank), every group of the rank stage
// is one class; and when the class f with the smallest key is alone in its (c0, c1) bucket, the
// substring stage leaves f's copies in a simple order:
//  a. substring stage: f's bucket holds copies 0 .. k-1 in order (class q-1: copy k-1, the
//     item whose substring wraps round the text end, first, then 0 .. k-2).  All of them tie at
//     every character, so the radix sort of the bucket's first block of s0 = min(items, 1024)
//     items (the wrapped item excluded) only exchanges the block's first item with its middle
//     one (the pivot rules all pick the middle of equal keys), once per character of the class's
//     substring: gap = distance to the next B* offset times.  Merges of later blocks keep the
//     first block in place.  So copy 0 ends at bucket position g0 = (s0 > 8 and gap odd) ? s0/2 : 0
//     (+1 after the wrapped item for class q-1).
//     (The buckets of the other classes may mix classes: their substring-stage order does not
//     matter, below.)
//  b. rank stage: groups are refined in key order.  The first group, class f, compares the
//     ranks of the items h = 1, 2, ... places further on; those belong to
//     other, unrefined groups (all equal) until h = q, where the group repeats itself and is
//     final in slot order.  Each of those q levels of a group of more than 8 items exchanges its
//     first slot with its middle one (slot k/2).
//     Every later class c meets, at the smallest h with class (c + h) mod q already refined, keys
//     that are all different: it is sorted by them, i.e. it takes the copy order of that class.
//     Following these links from class 0 forward ends at class f without passing the end of the
//     text (f is refined before every other class), so class 0 has class f's copy order with no
//     copy shift: r = the final slot of copy 0 in class f's group.
//  c. the reference's rank stage stops refining group by group once a work budget
//     (lg(m) * 2/3 + 1) * m, m = q k, is spent, and finishes by rank doubling instead; the rule
//     holds only when the budget lasts to the last group.  Work charged per group: q k for the
//     first group (q levels); for any other group c, (h_c - 1) k for the levels before its keys
//     differ, then at most k (lg k + 1) for the sort (at most lg k + 1 partition levels of at most k
//     items each).  The rule is used when the sum over every group but the last is < the budget.
#include <algorithm>
#include <vector>

#include "copyrank.h"

namespace bzg {
namespace {

int lg32(uint32_t v) { return v == 0 ? -1 : 31 - __builtin_clz(v); }

}  // namespace

int32_t copy_rank_distinct(const uint8_t* w, int32_t p, int32_t k) {
  if (!w || p < 2 || k < 2) return -1;
  // B* offsets: w[i] < w[i+1] and the first symbol after the run starting at i+1 is smaller
  std::vector<int32_t> off;
  for (int32_t i = 0; i < p; i++) {
    const int32_t j = i + 1 == p ? 0 : i + 1;
    const uint8_t c = w[j];
    if (w[i] >= c) continue;
    int32_t t = j;
    do t = t + 1 == p ? 0 : t + 1;
    while (w[t] == c);
    if (w[t] < c) off.push_back(i);
  }
  const int32_t q = (int32_t)off.size();
  if (q < 2 || q > kCopyRankQMax) return -1;  // (the device's caps, origptr.hip)
  if (p > kCopyRankPMax || (int64_t)q * p > kCopyRankCmpMax) return -1;
  const uint64_t m = (uint64_t)q * (uint64_t)k;
  if (m > 0x7fffffffull) return -1;
  std::vector<int32_t> bk(q), gap(q), ord(q), rk(q);
  for (int32_t c = 0; c < q; c++) {
    bk[c] = (w[off[c]] << 8) | w[off[c] + 1 == p ? 0 : off[c] + 1];
    gap[c] = (c + 1 < q ? off[c + 1] : off[0] + p) - off[c];
  }
  // full key: bucket, then the substring characters 2 .. gap + 1, a shorter equal prefix first
  auto cmp = [&](int32_t x, int32_t y) {
    if (bk[x] != bk[y]) return bk[x] < bk[y] ? -1 : 1;
    const int32_t n = std::min(gap[x], gap[y]);
    for (int32_t d = 0, a = (off[x] + 2) % p, b = (off[y] + 2) % p; d < n; d++) {
      if (w[a] != w[b]) return w[a] < w[b] ? -1 : 1;
      a = a + 1 == p ? 0 : a + 1;
      b = b + 1 == p ? 0 : b + 1;
    }
    return gap[x] == gap[y] ? 0 : gap[x] < gap[y] ? -1 : 1;
  };
  for (int32_t c = 0; c < q; c++) ord[c] = c;
  std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return cmp(a, b) < 0; });
  for (int32_t i = 1; i < q; i++)
    if (cmp(ord[i - 1], ord[i]) == 0) return -1;  // two classes in one group: not this rule
  for (int32_t i = 0; i < q; i++) rk[ord[i]] = i;
  const int32_t f = ord[0];
  for (int32_t c = 0; c < q; c++)
    if (c != f && bk[c] == bk[f]) return -1;  // f shares its bucket: its substring order is not simple
  // budget (c): every group but the last in key order
  const int64_t budget = (int64_t)(lg32((uint32_t)m) * 2 / 3 + 1) * (int64_t)m;
  int64_t work = (int64_t)q * k;
  const int64_t sort_work = (int64_t)k * (lg32((uint32_t)k) + 1);
  for (int32_t c = 0; c < q; c++) {
    if (rk[c] == 0 || rk[c] == q - 1) continue;
    int32_t h = 1;
    while (rk[(c + h) % q] > rk[c]) h++;
    work += (int64_t)(h - 1) * k + sort_work;
  }
  if (work >= budget) return -1;
  // (a) and (b) on the first group, class f
  const bool wrapped = f == q - 1;
  const int32_t s0 = std::min(wrapped ? k - 1 : k, 1024);
  int32_t g = (wrapped ? 1 : 0) + ((s0 > 8 && (gap[f] & 1)) ? s0 / 2 : 0);
  if (k > 8 && (q & 1)) g = g == 0 ? k / 2 : g == k / 2 ? 0 : g;
  return g;
}

}  // namespace bzg
