// qsa.cpp -- sorted rotations of a quasi-periodic block (see qsa.h).
//
// The reference sorts every block with divsufsort (blocksort.c:1503-1545); for an aperiodic
// block all rotations are distinct, so any correct sort of the rotations gives its BWT and
// origPtr.  For t = w^k w' (|t| = n, smallest period p, r = n mod p != 0, w primitive) the
// cyclic text is w^infinity read from phase 0 up to position n, where it restarts at phase 0
// instead of continuing at phase r: one defect.  Write W(c) for w^infinity read from phase c.
//   * Two rotations a < b of the same phase agree until b reaches the defect; then b reads
//     W(0) while a reads W(r) for b - a >= p characters (then a reaches the defect and both are
//     in phase again).  W(0) != W(r) within p characters (w is primitive and r != 0), so
//     rotation b sorts before rotation a iff W(0) < W(r), whatever a and b: within a phase the
//     rotations sort by position, descending iff W(0) < W(r).
//   * A rotation i <= n - p reads at least p characters of W(i mod p) before the defect, and
//     two different phases differ within p - 1 characters: such "normal" rotations of
//     different phases sort by the order of the rotations of the cyclic word w.
// So the normal rotations are the phases in w's rotation order, each phase's positions
// ascending or descending.  The p - 1 rotations i > n - p ("special") are placed by binary
// search among the normal ones and sorted among themselves, comparing the actual cyclic text
// (same-phase pairs by the rule above); their comparisons end within about 2p characters.
#include "qsa.h"

#include <algorithm>

#include "copyrank.h"

namespace bzg {

uint32_t quasi_period(const uint8_t* t, uint32_t n) {
  if (n < 4) return 0;
  const uint32_t pmax = std::min<uint32_t>(kQsaMaxPeriod, n / 2);
  for (uint32_t p = 1; p <= pmax; p++) {
    uint32_t i = 0;
    while (i < n - p && t[i] == t[i + p]) i++;
    if (i < n - p) continue;
    if (n % p == 0) return 0;  // a power of t[0, p): the periodic path (A5)
    return primitive_period(t, (int32_t)n) == (int32_t)n ? p : 0;
  }
  return 0;
}

namespace {

struct Ctx {
  const uint8_t* w;
  uint32_t p, n;
  bool desc;
  // rotation a < rotation b of the cyclic text t[x] = w[x mod p], x < n
  bool less(uint32_t a, uint32_t b) const {
    if (a % p == b % p) return desc ? a > b : a < b;
    uint32_t ia = a, ib = b, pa = a % p, pb = b % p;
    for (uint32_t d = 0; d < n; d++) {
      const uint8_t ca = w[pa], cb = w[pb];
      if (ca != cb) return ca < cb;
      if (++ia == n) ia = 0, pa = 0;
      else if (++pa == p) pa = 0;
      if (++ib == n) ib = 0, pb = 0;
      else if (++pb == p) pb = 0;
    }
    return false;  // equal rotations: the block would be periodic
  }
};

// W(a) < W(b) over one period (a != b phases of the primitive word w)
bool phase_less(const uint8_t* w, uint32_t p, uint32_t a, uint32_t b) {
  for (uint32_t d = 0; d < p; d++) {
    const uint8_t ca = w[(a + d) % p], cb = w[(b + d) % p];
    if (ca != cb) return ca < cb;
  }
  return false;
}

}  // namespace

uint32_t qsa_normal_at(const QsaPlan& P, uint32_t y) {
  const uint32_t k = (uint32_t)(std::upper_bound(P.cum.begin(), P.cum.begin() + P.p, y) - P.cum.begin()) - 1;
  const uint32_t c = P.ord[k], o = y - P.cum[k], cnt = P.cum[k + 1] - P.cum[k];
  return c + (P.desc ? cnt - 1 - o : o) * P.p;
}

void qsa_plan(const uint8_t* w, uint32_t p, uint32_t n, QsaPlan& P) {
  P.n = n;
  P.p = p;
  P.desc = phase_less(w, p, 0, n % p);
  P.ord.resize(p);
  for (uint32_t c = 0; c < p; c++) P.ord[c] = c;
  std::sort(P.ord.begin(), P.ord.end(), [&](uint32_t a, uint32_t b) { return phase_less(w, p, a, b); });
  // normals of phase c: c, c + p, ... <= n - p
  P.cum.assign(p + 1, 0);
  for (uint32_t k = 0; k < p; k++) P.cum[k + 1] = P.cum[k] + (n - p - P.ord[k]) / p + 1;
  const Ctx C{w, p, n, P.desc};
  const uint32_t nn = n - p + 1;
  P.srot.resize(p - 1);
  for (uint32_t j = 0; j + 1 < p; j++) P.srot[j] = n - p + 1 + j;
  std::sort(P.srot.begin(), P.srot.end(), [&](uint32_t a, uint32_t b) { return C.less(a, b); });
  P.lo.resize(p - 1);
  for (uint32_t j = 0; j + 1 < p; j++) {  // normals before special j (binary search)
    uint32_t lo = j ? P.lo[j - 1] : 0, hi = nn;
    const uint32_t s = P.srot[j];
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (C.less(qsa_normal_at(P, mid), s)) lo = mid + 1;
      else hi = mid;
    }
    P.lo[j] = lo;
  }
}

uint32_t qsa_bwt(const QsaPlan& P, const uint8_t* t, uint8_t* bwt) {
  const uint32_t n = P.n, nn = n - P.p + 1;
  uint32_t orig = 0, j = 0, x = 0;
  auto put = [&](uint32_t rot) {
    bwt[x] = t[rot == 0 ? n - 1 : rot - 1];
    if (rot == 0) orig = x;
    x++;
  };
  for (uint32_t y = 0; y < nn; y++) {
    while (j < P.lo.size() && P.lo[j] == y) put(P.srot[j++]);
    put(qsa_normal_at(P, y));
  }
  while (j < P.lo.size()) put(P.srot[j++]);
  return orig;
}

}  // namespace bzg

// C-ABI (include/bzg.h): host reference of the analytic path, for the parity tests.
extern "C" uint32_t bzg_qperiodic_bwt(const uint8_t* block, uint32_t n, uint8_t* bwt, uint32_t* origptr) {
  const uint32_t p = bzg::quasi_period(block, n);
  if (p == 0) return 0;
  bzg::QsaPlan plan;
  bzg::qsa_plan(block, p, n, plan);
  *origptr = bzg::qsa_bwt(plan, block, bwt);
  return p;
}
