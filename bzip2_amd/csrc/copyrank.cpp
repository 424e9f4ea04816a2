// copyrank.cpp -- A5: origPtr of an exactly periodic block.
//
// DERIVED WORK NOTICE.  Sections 3a/3b below model, on class labels, the exchange sequence of
// divsufsort as modified in the reference's blocksort.c: the B* substring sort (ss_pivot /
// ss_median3 / ss_median5 blocksort.c:211-262, ss_fixdown / ss_heapsort 168-209,
// ss_multikey_introsort 300-424, ss_merge_forward / ss_merge_backward / ss_merge 436-622,
// substringsort 625-664) and the rank refinement (tr_partition / tr_copy / tr_introsort
// 964-1122, lssort / ls_introsort 833-959, trsort 1285-1309).  For q > 1 periodic roots the
// tie order IS those exchanges, so this model mirrors their structure; it is a derived
// component of divsufsort, used under its licence:
//
//   divsufsort
//   Copyright (c) 2003-2007 Yuta Mori All Rights Reserved.
//
//   Permission is hereby granted, free of charge, to any person obtaining a copy of this
//   software and associated documentation files (the "Software"), to deal in the Software
//   without restriction, including without limitation the rights to use, copy, modify,
//   merge, publish, distribute, sublicense, and/or sell copies of the Software, and to
//   permit persons to whom the Software is furnished to do so, subject to the following
//   conditions:
//
//   The above copyright notice and this permission notice shall be included in all copies
//   or substantial portions of the Software.
//
//   THE SOFTWARE IS PROVIDED "AS IS", WITHOUT WARRANTY OF ANY KIND, EXPRESS OR IMPLIED,
//   INCLUDING BUT NOT LIMITED TO THE WARRANTIES OF MERCHANTABILITY, FITNESS FOR A
//   PARTICULAR PURPOSE AND NONINFRINGEMENT. IN NO EVENT SHALL THE AUTHORS OR COPYRIGHT
//   HOLDERS BE LIABLE FOR ANY CLAIM, DAMAGES OR OTHER LIABILITY, WHETHER IN AN ACTION OF
//   CONTRACT, TORT OR OTHERWISE, ARISING FROM, OUT OF OR IN CONNECTION WITH THE SOFTWARE
//   OR THE USE OR OTHER DEALINGS IN THE SOFTWARE.
//
// The q = 1 closed form (section 4, evaluated on the device in origptr.hip) and the
// quasi-periodic ordering (qsa.cpp) are not derived from divsufsort code.
//
// A block T = w^k (w primitive, |w| = p >= 2, k >= 2) has k identical copies of each of its p
// distinct rotations.  The last column does not depend on how the copies are ordered, but
// origPtr does: the reference reports the slot of rotation 0, which sits somewhere inside the
// run of its k copies.  The device sort gives rank0, the rank of rotation 0 among the p
// distinct rotations of w, so origPtr = rank0 * k + r, and this file computes r.
//
// 1. Where r comes from.  The reference sorts the B* rotations (cyclic types: B = smaller
//    than the next rotation, A = larger, B* = a B position followed by an A position) and
//    places every other rotation by induction (blocksort.c:1439-1501): a rotation is placed
//    when its successor is met in a left-to-right (type A) or right-to-left (type B) scan, at
//    the next free slot of its bucket.  The k copies of one rotation are met in the order of
//    their successors and fill adjacent slots in that order, so induction keeps copy order.
//    Rotation 0 is induced, through non-B* positions, from the first B* position b0 of the
//    text; hence r = the rank of the copy at b0 among the k copies of that B* rotation.
// 2. The B* level.  With q B* offsets off[0] < ... < off[q-1] in w, the text has m = k q B*
//    items; item x has class x mod q, copy x div q and position (x div q) p + off[x mod q].
//    The reference orders them in two stages, and among copies of a class every comparison
//    ties, so each stage acts on the copies only through the positions its exchanges touch:
//    a. the substring stage (blocksort.c:1314-1385, 302-664): items are bucketed by their
//       first two characters, in ascending item order except that the last item m - 1 is
//       placed first; a bucket is sorted by the B* substring (characters 2 .. gap + 1) in
//       blocks of 1024 items with a ternary radix quicksort, the blocks are then merged
//       stably, and item m - 1, whose substring wraps around the text end, is put in front
//       of the items equal to it;
//    b. the rank stage (blocksort.c:1283-1309, 669-959): groups of equal substrings are
//       refined by the rank of the B* item h places further on (h = 1, 2, 3, ... with
//       tandem-repeat induction), group by group from the left, against a work budget;
//       when the budget is spent the remaining groups are refined by rank doubling.
//    Section 3 restates both stages on class labels; section 4 gives the closed form for
//    q = 1, the case of every block cut from a long run of one byte (config 4), which the
//    device evaluates on its own (origptr.hip).
// 3. Facts the restatement uses instead of the reference's control flow:
//    * substring stage: the sorted runs are disjoint and their keys are fixed text
//      characters, so the order in which sub-ranges are finished does not matter (plain
//      recursion); merging sorted blocks stably equals one stable sort of their
//      concatenation by the full substring, so the merge is a std::stable_sort; insertion
//      sorts of <= 8 items are stable sorts;
//    * a run of items that are all equal under the current key is not reordered by the
//      three-way split except for the pivot exchange: one step swaps the first item with the
//      middle one (all three pivot rules return the middle position on equal keys);
//    * rank stage: keys are ranks of other items, which change as groups are finished, so the
//      order of work matters.  After a split, the reference works on the three parts in
//      ascending size (ties: smaller keys, larger keys, equal keys), skipping parts of one
//      item; a rank-stage task also reports whether it ended inside the small-range loop or
//      in the main loop, because a pending remainder of a small range is resumed by the
//      small-range rules in the first case and by the sorted-run rules in the second;
//    * the budget is checked only between top-level groups;
//    * the final doubling round may read ranks past the rank array (slots of the B* position
//      list and zero scratch); they are modelled as the reference's work array lays them out.
// Checked against the reference build: tests/test_abi.py (SURVEY.md 8a KATs, random periodic
// blocks, a 5,000-block fuzz across short/long roots, 2..180,000 copies, budget exhaustion).
#include "copyrank.h"

#include <algorithm>
#include <vector>

namespace bzg {
namespace {

using i32 = int32_t;
using i64 = int64_t;

int floor_lg(uint32_t v) { return v == 0 ? -1 : 31 - __builtin_clz(v); }
// depth limits: the substring stage takes lg of the low 16 bits, the rank stage of 32
int lg16(i32 v) { return floor_lg((uint32_t)v & 0xffffu); }
int lg32(i32 v) { return floor_lg((uint32_t)v); }

// ---------------------------------------------------------------- shared split machinery
// Pivot position for a[lo, hi) under key K: median of 3 up to 32 items, of 5 up to 512, of
// 3 medians of 3 above.
template <class K>
i32 median3(const i32* a, i32 i, i32 j, i32 l, K key) {
  if (key(a[i]) > key(a[j])) std::swap(i, j);
  if (key(a[j]) > key(a[l])) return key(a[i]) > key(a[l]) ? i : l;
  return j;
}

template <class K>
i32 median5(const i32* a, i32 v1, i32 v2, i32 v3, i32 v4, i32 v5, K key) {
  if (key(a[v2]) > key(a[v3])) std::swap(v2, v3);
  if (key(a[v4]) > key(a[v5])) std::swap(v4, v5);
  if (key(a[v2]) > key(a[v4])) {
    std::swap(v2, v4);
    std::swap(v3, v5);
  }
  if (key(a[v1]) > key(a[v3])) std::swap(v1, v3);
  if (key(a[v1]) > key(a[v4])) {
    std::swap(v1, v4);
    std::swap(v3, v5);
  }
  return key(a[v3]) > key(a[v4]) ? v4 : v3;
}

template <class K>
i32 pick_pivot(const i32* a, i32 lo, i32 hi, K key) {
  i32 t = hi - lo;
  const i32 mid = lo + t / 2;
  if (t <= 32) return median3(a, lo, mid, hi - 1, key);
  if (t <= 512) {
    t >>= 2;
    return median5(a, lo, lo + t, mid, hi - 1 - t, hi - 1, key);
  }
  t >>= 3;
  return median3(a, median3(a, lo, lo + t, lo + 2 * t, key), median3(a, mid - t, mid, mid + t, key),
                 median3(a, hi - 1 - 2 * t, hi - 1 - t, hi - 1, key), key);
}

// Split-end three-way partition of a[lo, hi) around value v (Bentley & McIlroy): scanning
// starts at `from` (lo + 1 when the pivot was moved to a[lo], lo when only v is given); equal
// items are parked at both ends and then swapped into the middle.  Returns false when every
// scanned item equals v (nothing moves); otherwise [lt, gt) is the run of items equal to v.
template <class K>
bool split3(i32* a, i32 lo, i32 hi, i32 from, int v, K key, i32* lt, i32* gt) {
  i32 b = from;
  while (b < hi && key(a[b]) == v) ++b;
  i32 el = b;  // next slot for an equal item at the left end
  if (b < hi && key(a[b]) < v) {
    for (++b; b < hi; ++b) {
      const int x = key(a[b]);
      if (x > v) break;
      if (x == v) std::swap(a[b], a[el++]);
    }
  }
  i32 c = hi - 1;
  while (b < c && key(a[c]) == v) --c;
  i32 er = c;  // next slot for an equal item at the right end
  if (b < c && key(a[c]) > v) {
    for (--c; b < c; --c) {
      const int x = key(a[c]);
      if (x < v) break;
      if (x == v) std::swap(a[c], a[er--]);
    }
  }
  while (b < c) {
    std::swap(a[b], a[c]);
    for (++b; b < c; ++b) {
      const int x = key(a[b]);
      if (x > v) break;
      if (x == v) std::swap(a[b], a[el++]);
    }
    for (--c; b < c; --c) {
      const int x = key(a[c]);
      if (x < v) break;
      if (x == v) std::swap(a[c], a[er--]);
    }
  }
  if (el > er) return false;
  // the left equals [lo, el) move next to the smaller items, the right ones next to the larger
  const i32 nl = el - lo, ns = b - el;
  for (i32 s = std::min(nl, ns), e = lo, f = b - s; s > 0; --s) std::swap(a[e++], a[f++]);
  const i32 nr = er - (b - 1), ng = hi - er - 1;
  for (i32 s = std::min(nr, ng), e = b, f = hi - s; s > 0; --s) std::swap(a[e++], a[f++]);
  *lt = lo + ns;
  *gt = hi - nr;
  return true;
}

// In-place heap sort of a[0, n) by key, with the reference's even-size preamble (the extra
// last item is set aside and compared with its parent first).
template <class K>
void sift(i32* a, i32 i, i32 size, K key) {
  const i32 v = a[i];
  const int c = key(v);
  for (i32 j; (j = 2 * i + 1) < size;) {
    i32 k = j;
    int d = key(a[j]);
    if (j + 1 < size && key(a[j + 1]) > d) {
      k = j + 1;
      d = key(a[k]);
    }
    if (d <= c) break;
    a[i] = a[k];
    i = k;
  }
  a[i] = v;
}

template <class K>
void heap_sort(i32* a, i32 n, K key) {
  i32 m = n;
  if (n % 2 == 0) {
    --m;
    if (key(a[m / 2]) < key(a[m])) std::swap(a[m], a[m / 2]);
  }
  for (i32 i = m / 2 - 1; i >= 0; --i) sift(a, i, m, key);
  if (n % 2 == 0) {
    std::swap(a[0], a[m]);
    sift(a, 0, m, key);
  }
  for (i32 i = m - 1; i > 0; --i) {
    const i32 t = a[0];
    a[0] = a[i];
    sift(a, 0, i, key);
    a[i] = t;
  }
}

// ---------------------------------------------------------------- the root and its B* items
struct Root {
  const uint8_t* w;
  i32 p, k, q, m;
  std::vector<i32> off, gap;  // B* offsets in w, distance to the next B* offset
  std::vector<i32> crank;     // class rank by (first two characters, B* substring), ties equal
  int at(i64 i) const { return w[i % p]; }
  i32 pos(i32 x) const { return (x / q) * p + off[x % q]; }

  Root(const uint8_t* w_, i32 p_, i32 k_) : w(w_), p(p_), k(k_) {
    // cyclic types, decided backwards from a strict comparison
    std::vector<uint8_t> isB(p);
    i32 s0 = -1;
    for (i32 i = 0; i < p && s0 < 0; i++)
      if (w[i] != at(i + 1)) s0 = i;
    if (s0 < 0) throw CopyRankFailure();
    isB[s0] = w[s0] < at(s0 + 1);
    for (i32 t = 1; t < p; t++) {
      const i32 i = (s0 - t + p) % p, nx = (i + 1) % p;
      isB[i] = w[i] < w[nx] || (w[i] == w[nx] && isB[nx]);
    }
    for (i32 i = 0; i < p; i++)
      if (isB[i] && !isB[(i + 1) % p]) off.push_back(i);
    q = (i32)off.size();
    m = q * k;
    gap.resize(q);
    for (i32 c = 0; c < q; c++) gap[c] = (c + 1 < q ? off[c + 1] : off[0] + p) - off[c];
    // full key of a class: bucket characters, then the substring at depths 0 .. gap - 1
    std::vector<i32> order(q);
    for (i32 c = 0; c < q; c++) order[c] = c;
    auto less = [&](i32 x, i32 y) {
      const int bx = (at(off[x]) << 8) | at(off[x] + 1), by = (at(off[y]) << 8) | at(off[y] + 1);
      if (bx != by) return bx < by;
      const i32 n = std::min(gap[x], gap[y]);
      for (i32 d = 0; d < n; d++) {
        const int cx = at(off[x] + 2 + d), cy = at(off[y] + 2 + d);
        if (cx != cy) return cx < cy;
      }
      return gap[x] < gap[y];
    };
    std::stable_sort(order.begin(), order.end(), less);
    crank.assign(q, 0);
    for (i32 i = 1; i < q; i++) crank[order[i]] = crank[order[i - 1]] + (less(order[i - 1], order[i]) ? 1 : 0);
  }
  int bucket(i32 c) const { return (at(off[c]) << 8) | at(off[c] + 1); }
};

// ---------------------------------------------------------------- stage a: B* substrings
class SubstringStage {
 public:
  SubstringStage(const Root& r, std::vector<i32>& sa) : R(r), sa_(sa) {}

  // Sort one bucket sa[lo, hi) laid out as the reference lays it out.  Blocks of 1024 items
  // are radix-sorted and merged pairwise like a binary counter.  The merges are stable, but a
  // merge that borrows the bucket's still-unsorted rest as its scratch leaves that rest
  // permuted, which changes how later blocks break their ties; so the merges are modelled
  // with their element moves (section 3), tie chains marked as ~item ("equals the previous").
  void bucket(i32 lo, i32 hi, i32 bufsize, i32* scratch) {
    const bool wraps = sa_[lo] == R.m - 1;
    i32* const first = sa_.data() + lo + (wraps ? 1 : 0);
    i32* const last = sa_.data() + hi;
    i32* a = first;
    i32 nblk = 0;
    for (; a + 1024 < last; a += 1024, ++nblk) {
      sort_block(a, a + 1024);
      i32* cur = a + 1024;
      i32 cursize = (i32)(last - cur);
      if (cursize <= bufsize) cur = scratch, cursize = bufsize;
      i32* b = a;
      for (i32 k = 1024, j = nblk; j & 1; b -= k, k <<= 1, j >>= 1) merge(b - k, b, b + k, cur, cursize);
    }
    sort_block(a, last);
    for (i32 k = 1024, j = nblk; j != 0; k <<= 1, j >>= 1)
      if (j & 1) {
        merge(a - k, a, last, scratch, bufsize);
        a -= k;
      }
    for (i32* x = first; x < last; ++x)
      if (*x < 0) *x = ~*x;
    if (wraps) {  // item m - 1 goes in front of the items equal to it
      const i32 key = full(R.m - 1);
      i32* t = first;
      while (t < last && full(*t) < key) {
        t[-1] = *t;
        ++t;
      }
      t[-1] = R.m - 1;
    }
  }
  i32 full(i32 x) const { return R.crank[x % R.q]; }

 private:
  int fkey(i32 v) const { return full(v < 0 ? ~v : v); }

  void sort_block(i32* lo, i32* hi) {
    const i32 b = (i32)(lo - sa_.data()), e = (i32)(hi - sa_.data());
    radix(b, e, 0, lg16(e - b));
    for (i32 x = e - 1; x > b; x--)
      if (full(sa_[x]) == full(sa_[x - 1])) sa_[x] = ~sa_[x];
  }
  // a chain head at a that equals its left neighbour joins its chain
  void join_left(i32* a) {
    if (*a >= 0 && fkey(a[-1]) == fkey(*a)) *a = ~*a;
  }

  // Merge with the right run parked in the scratch: output is written from the top down, and
  // each slot written passes its old content to the slot just read (the scratch keeps a
  // permutation of its content).  Ties: the left chain ends up before the right one.
  void merge_back(i32* buf, i32* first, i32* middle, i32* last) {
    std::swap_ranges(middle, last, buf);
    const i32 t = last[-1];
    i32 *i = last - 1, *j = buf + (last - middle) - 1, *k = middle - 1;
    auto take_j = [&] { *i-- = *j; *j-- = *i; };
    auto take_k = [&] { *i-- = *k; *k-- = *i; };
    auto drain = [&] {
      while (buf <= j) take_j();
      *buf = t;
    };
    for (;;) {
      const int vj = fkey(*j), vk = fkey(*k);
      if (vj >= vk) {
        if (*j < 0) do take_j(); while (*j < 0);
        if (vj > vk) {
          take_j();
        } else {  // equal: the right head now follows the left chain
          *i-- = ~*j;
          *j-- = *i;
        }
        if (j < buf) {
          *buf = t;
          return;
        }
        if (vj > vk) continue;
      }
      if (*k < 0) do take_k(); while (*k < 0);
      take_k();
      if (k < first) return drain();
    }
  }

  // Merge with the left run parked in the scratch, output written from the bottom up.
  void merge_front(i32* buf, i32* first, i32* middle, i32* last) {
    const i32 n = (i32)(middle - first);
    std::swap_ranges(first, middle, buf);
    i32* const bend = buf + n;
    const i32 t = *first;
    i32 *i = first, *j = buf, *k = middle;
    for (;;) {
      const int vj = fkey(*j), vk = fkey(*k);
      if (vj == vk) *k = ~*k;
      if (vj <= vk) {
        do {
          *i++ = *j;
          *j++ = *i;
          if (bend <= j) {
            bend[-1] = t;
            return;
          }
        } while (*j < 0);
      }
      if (vj >= vk) {
        do {
          *i++ = *k;
          *k++ = *i;
          if (last <= k) {
            do {
              *i++ = *j;
              *j++ = *i;
            } while (j < bend);
            bend[-1] = t;
            return;
          }
        } while (*k < 0);
      }
    }
  }

  // Merge of two adjacent sorted runs with a scratch of bufsize slots; when neither run fits,
  // the runs exchange the blocks that are out of order (a symmetric rotation merge) and the two
  // halves are merged in turn, the smaller span first, without cutting a tie chain.
  void merge(i32* first, i32* middle, i32* last, i32* buf, i32 bufsize) {
    struct Job {
      i32 *a, *b, *c;
      int check;
    };
    std::vector<Job> todo;
    int check = 0;
    for (;;) {
      bool done = true;
      if (last - middle <= bufsize) {
        if (first < middle && middle < last) merge_back(buf, first, middle, last);
      } else if (middle - first <= bufsize) {
        if (first < middle) merge_front(buf, first, middle, last);
      } else {
        // the count m of right items that belong before the left run's last m items
        i32 lo = 0, hi = (i32)std::min(middle - first, last - middle);
        while (lo < hi) {
          const i32 mid = (lo + hi + 1) / 2;
          if (fkey(middle[mid - 1]) < fkey(middle[-mid])) lo = mid;
          else hi = mid - 1;
        }
        const i32 m = lo;
        if (m > 0) {
          std::swap_ranges(middle - m, middle, middle);
          i32 *i = middle, *j = middle;
          int next = 0;
          if (middle + m < last) {
            if (middle[m] < 0) {
              while (i[-1] < 0) --i;
              middle[m] = ~middle[m];
            }
            while (*j < 0) ++j;
            next = 1;
          }
          if (i - first <= last - j) {
            todo.push_back({j, middle + m, last, (check & 2) | (next & 1)});
            middle -= m, last = i, check &= 1;
          } else {
            if (i == middle && middle == j) next <<= 1;
            todo.push_back({first, middle - m, i, (check & 1) | (next & 2)});
            first = j, middle += m, check = (check & 2) | (next & 1);
          }
          done = false;
        } else {
          if (check & 1) join_left(first);
          join_left(middle);
          if (check & 2) join_left(last);
          check = 0;
        }
      }
      if (done) {
        if (check & 1) join_left(first);
        if (check & 2) join_left(last);
        if (todo.empty()) return;
        first = todo.back().a, middle = todo.back().b, last = todo.back().c, check = todo.back().check;
        todo.pop_back();
      }
    }
  }
  int chr(i32 x, i32 d) const { return R.at(R.off[x % R.q] + 2 + d); }
  int prev(i32 x, i32 d) const { return R.at(R.off[x % R.q] + 1 + d); }
  bool ended(i32 x, i32 d) const { return d >= R.gap[x % R.q] - 1; }

  // items whose substring ends at depth d move to the front (they all tie); returns the
  // first slot of the rest
  i32 drop_ended(i32 lo, i32 hi, i32 d) {
    i32 a = lo - 1, b = hi;
    for (;;) {
      while (++a < b && ended(sa_[a], d)) {
      }
      while (a < --b && !ended(sa_[b], d)) {
      }
      if (b <= a) break;
      std::swap(sa_[a], sa_[b]);
    }
    return a;
  }

  void radix(i32 lo, i32 hi, i32 d, int limit) {
    i32* a = sa_.data();
    for (;;) {
      const i32 n = hi - lo;
      if (n <= 8) {
        if (n > 1) std::stable_sort(a + lo, a + hi, [&](i32 x, i32 y) { return full(x) < full(y); });
        return;
      }
      auto key = [&](i32 x) { return chr(x, d); };
      if (limit-- == 0) {
        // depth limit: heap sort on this character, then each run of equal characters
        // (two items or more) continues one character deeper
        heap_sort(a + lo, n, key);
        for (i32 s = lo; s < hi;) {
          const int v = key(a[s]);
          i32 e = s + 1;
          while (e < hi && key(a[e]) == v) ++e;
          if (e - s > 1) {
            const i32 s2 = prev(a[s], d) < v ? drop_ended(s, e, d) : s;
            radix(s2, e, d + 1, lg16(e - s2));
          }
          s = e;
        }
        return;
      }
      const i32 pv = pick_pivot(a, lo, hi, key);
      std::swap(a[lo], a[pv]);
      const int v = key(a[lo]);
      i32 lt, gt;
      if (split3(a, lo, hi, lo + 1, v, key, &lt, &gt)) {
        const i32 e2 = v <= prev(a[lt], d) ? lt : drop_ended(lt, gt, d);
        radix(lo, lt, d, limit);
        radix(gt, hi, d, limit);
        radix(e2, gt, d + 1, lg16(gt - e2));
        return;
      }
      // every item has this character: one step deeper (after the pivot exchange)
      limit += 1;
      if (prev(a[lo], d) < v) {
        lo = drop_ended(lo, hi, d);
        limit = lg16(hi - lo);
      }
      d += 1;
    }
  }

  const Root& R;
  std::vector<i32>& sa_;
};

// ---------------------------------------------------------------- stage b: ranks
class RankStage {
 public:
  enum Exit { kLoop, kMain };

  RankStage(const Root& r, std::vector<i32>& sa) : R(r), m(r.m), sa_(sa), isa(r.m), tie(r.m), done(r.m) {}

  // groups of equal substring: rank = last slot of the group; single items are final
  void init_groups(const SubstringStage& ss) {
    for (i32 i = 0; i < m;) {
      i32 j = i + 1;
      while (j < m && R.bucket(sa_[j] % R.q) == R.bucket(sa_[i] % R.q) && ss.full(sa_[j]) == ss.full(sa_[i])) ++j;
      for (i32 t = i; t < j; t++) isa[sa_[t]] = j - 1;
      if (j - i == 1) done[i] = 1;
      i = j;
    }
  }

  void run() {
    budget = (i64)(lg32(m) * 2 / 3 + 1) * m;
    for (i32 i = 0; i < m;) {
      if (done[i]) {
        ++i;
        continue;
      }
      const i32 last = isa[sa_[i]] + 1;
      work(i, last, 1, lg32(last - i));
      std::fill(done.begin() + i, done.begin() + last, 1);
      i = last;
      if (budget <= 0) {
        doubling();
        break;
      }
    }
  }

  i32 rank(i32 x) const { return isa[x]; }

 private:
  int key(i32 x, i64 h) const {
    i64 j = x + h;
    if (j >= m) j -= m;
    return j < m ? isa[j] : beyond(j);
  }
  // a rank read past the array (only the last doubling round can), as the reference's work
  // array holds it: ranks occupy slots [m, 2m) of an n-slot array whose last m slots list
  // the B* positions; other slots are zero
  int beyond(i64 j) const {
    const i64 n = (i64)R.p * R.k, slot = m + j;
    return slot >= n - m && slot < n ? R.pos((i32)(slot - (n - m))) : 0;
  }
  void set_rank(i32 lo, i32 hi, i32 v) {
    for (i32 i = lo; i < hi; i++) isa[sa_[i]] = v;
  }
  void finalize(i32 lo, i32 hi) {
    for (i32 i = lo; i < hi; i++) isa[sa_[i]] = i;
  }
  bool repeats(i32 x, i64 h) const { return isa[x] == key(x, h); }
  // the first tied run at lo (ties are marked on all but the run's last slot); clears marks
  i32 run_end(i32 lo) {
    i32 a = lo;
    while (tie[a]) tie[a++] = 0;
    return a + 1;
  }
  void stable_by_key(i32 lo, i32 hi, i64 h) {
    std::vector<std::pair<int, i32>> kv(hi - lo);
    for (i32 i = lo; i < hi; i++) kv[i - lo] = {key(sa_[i], h), sa_[i]};
    std::stable_sort(kv.begin(), kv.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    for (i32 i = lo; i < hi; i++) {
      sa_[i] = kv[i - lo].second;
      tie[i] = i + 1 < hi && kv[i - lo].first == kv[i + 1 - lo].first;
    }
  }
  void heap_by_key(i32 lo, i32 hi, i64 h) {
    heap_sort(sa_.data() + lo, hi - lo, [&](i32 x) { return key(x, h); });
    for (i32 i = lo; i < hi; i++) tie[i] = i + 1 < hi && key(sa_[i], h) == key(sa_[i + 1], h);
  }

  // A group whose items repeat with period h (some item h places on lies in the group
  // itself): the items compared at depth h split into smaller / repeating / larger; the
  // outer parts are refined one level deeper, and the repeating items then take their order
  // from the items h places further on (induction from both ends).
  Exit tandem(i32 lo, i32 hi, i64 h) {
    const i32 v = hi - 1;
    i32 a = lo, b = hi;
    auto k = [&](i32 x) { return key(x, h); };
    if (!split3(sa_.data(), lo, hi, lo, v, k, &a, &b)) a = lo, b = hi;
    if (lo == a && b == hi) {
      finalize(lo, hi);
      return kMain;
    }
    if (a < hi) set_rank(lo, a, a - 1);
    if (b < hi) set_rank(a, b, b - 1);
    Exit e = kMain;
    const i32 sl = a - lo, sg = hi - b;
    if (sl <= sg) {
      if (sl > 1) {
        e = work(lo, a, h + 1, lg32(sl));
        e = work(b, hi, h + 1, lg32(sg));
      } else if (sg > 1) {
        e = work(b, hi, h + 1, lg32(sg));
      }
    } else {
      if (sg > 1) {
        e = work(b, hi, h + 1, lg32(sg));
        e = work(lo, a, h + 1, lg32(sl));
      } else if (sl > 1) {
        e = work(lo, a, h + 1, lg32(sl));
      }
    }
    if (b - a > 1) {
      induce(lo, a, b, hi, h);
      e = kMain;
    }
    return e;
  }

  void induce(i32 lo, i32 a, i32 b, i32 hi, i64 h) {
    const i32 v = b - 1;
    auto back = [&](i32 x) {
      i64 s = x - h;
      if (s < 0) s += m;
      return (i32)s;
    };
    i32 d = a - 1;
    for (i32 c = lo; c <= d; ++c) {
      const i32 s = back(sa_[c]);
      if (isa[s] == v) {
        sa_[++d] = s;
        isa[s] = d;
      }
    }
    const i32 e = d + 1;
    d = b;
    for (i32 c = hi - 1; e < d; --c) {
      const i32 s = back(sa_[c]);
      if (isa[s] == v) {
        sa_[--d] = s;
        isa[s] = d;
      }
    }
  }

  // a range of <= 8 items just sorted at depth h: finish its tied runs left to right, each
  // one level deeper; a remainder is resumed here unless the last run ended in the main loop
  Exit small_runs(i32 lo, i32 hi, i64 h) {
    for (;;) {
      while (lo < hi && !tie[lo]) {
        isa[sa_[lo]] = lo;
        ++lo;
      }
      if (lo >= hi) return kLoop;
      const i32 a = run_end(lo);
      const bool rep = repeats(sa_[a - 1], h);
      if (a < hi) set_rank(lo, a, a - 1);
      if (!rep && hi - a <= 1) {  // nothing waits behind the run: go one level deeper
        budget -= a - lo;
        stable_by_key(lo, a, h + 1);
        hi = a;
        h += 1;
        continue;
      }
      Exit e;
      if (rep) {
        e = tandem(lo, a, h);
      } else {
        budget -= a - lo;
        stable_by_key(lo, a, h + 1);
        e = small_runs(lo, a, h + 1);
      }
      if (hi - a <= 1) return e;
      if (e == kMain) return sorted_runs(a, hi, h);
      lo = a;
    }
  }

  // a range sorted at depth h with its tied runs marked (after a heap sort, or a remainder
  // resumed from the main loop): the smaller of the first run and the rest goes first
  Exit sorted_runs(i32 lo, i32 hi, i64 h) {
    for (;;) {
      while (lo < hi && !tie[lo]) {
        isa[sa_[lo]] = lo;
        ++lo;
      }
      if (lo >= hi) return kMain;
      const i32 a = run_end(lo);
      const int next = repeats(sa_[a - 1], h) ? -1 : lg32(a - lo);
      if (a < hi) set_rank(lo, a, a - 1);
      if (a - lo <= hi - a) {
        work(lo, a, h + 1, next);
        lo = a;
      } else if (hi - a > 1) {
        sorted_runs(a, hi, h);
        return work(lo, a, h + 1, next);
      } else {
        return work(lo, a, h + 1, next);
      }
    }
  }

  // refine the group sa[lo, hi) at depth h; limit < 0 selects the repeat (-1) or sorted-run
  // (-3) rules
  Exit work(i32 lo, i32 hi, i64 h, int limit) {
    for (;;) {
      if (limit == -1) return tandem(lo, hi, h - 1);
      if (limit < -1) return sorted_runs(lo, hi, h);
      const i32 n = hi - lo;
      if (n <= 8) {
        budget -= n;
        stable_by_key(lo, hi, h);
        return small_runs(lo, hi, h);
      }
      if (limit-- == 0) {
        budget -= n;
        heap_by_key(lo, hi, h);
        limit = -3;
        continue;
      }
      auto k = [&](i32 x) { return key(x, h); };
      const i32 pv = pick_pivot(sa_.data(), lo, hi, k);
      std::swap(sa_[lo], sa_[pv]);
      const int v = k(sa_[lo]);
      i32 a, b;
      if (split3(sa_.data(), lo, hi, lo + 1, v, k, &a, &b)) {
        const int next = repeats(sa_[a], h) ? -1 : lg32(b - a);
        set_rank(lo, a, a - 1);
        if (b < hi) set_rank(a, b, b - 1);
        budget -= n;
        struct Part {
          i32 lo, hi;
          i64 h;
          int limit;
        } parts[3] = {{lo, a, h, limit}, {b, hi, h, limit}, {a, b, h + 1, next}};
        std::stable_sort(parts, parts + 3, [](const Part& x, const Part& y) { return x.hi - x.lo < y.hi - y.lo; });
        int last = -1;
        for (int i = 0; i < 3; i++)
          if (parts[i].hi - parts[i].lo > 1) last = i;
        if (last < 0) return kMain;
        for (int i = 0; i < last; i++)
          if (parts[i].hi - parts[i].lo > 1) work(parts[i].lo, parts[i].hi, parts[i].h, parts[i].limit);
        lo = parts[last].lo, hi = parts[last].hi, h = parts[last].h, limit = parts[last].limit;
        continue;
      }
      // all items tie at this depth: one level deeper (a repeat ends the descent)
      limit = repeats(sa_[lo], h) ? -1 : limit + 1;
      h += 1;
      budget -= n;
    }
  }

  // ---- budget spent: rank doubling over the remaining groups
  void doubling() {
    for (i64 h = 1;; h += h) {
      if (std::find(done.begin(), done.end(), 0) == done.end()) return;
      for (i32 i = 0; i < m;) {
        if (done[i]) {
          ++i;
          continue;
        }
        const i32 last = isa[sa_[i]] + 1;
        refine(i, last, h, lg32(last - i));
        i = last;
      }
      if (h > m) {  // past the string length: remaining ties are final in slot order
        for (i32 i = 0; i < m;) {
          if (done[i]) {
            ++i;
            continue;
          }
          const i32 last = isa[sa_[i]] + 1;
          finalize(i, last);
          i = last;
        }
        return;
      }
    }
  }

  void regroup(i32 lo, i32 hi) {
    for (i32 i = lo; i < hi;) {
      if (!tie[i]) {
        isa[sa_[i]] = i;
        done[i] = 1;
        ++i;
        continue;
      }
      const i32 a = run_end(i);
      set_rank(i, a, a - 1);
      i = a;
    }
  }

  void refine(i32 lo, i32 hi, i64 h, int limit) {
    for (;;) {
      const i32 n = hi - lo;
      if (n <= 8) {
        if (n > 1) {
          stable_by_key(lo, hi, h);
          regroup(lo, hi);
        } else if (n == 1) {
          done[lo] = 1;
        }
        return;
      }
      if (limit-- == 0) {
        heap_by_key(lo, hi, h);
        regroup(lo, hi);
        return;
      }
      auto k = [&](i32 x) { return key(x, h); };
      const i32 pv = pick_pivot(sa_.data(), lo, hi, k);
      std::swap(sa_[lo], sa_[pv]);
      const int v = k(sa_[lo]);
      i32 a, b;
      if (!split3(sa_.data(), lo, hi, lo + 1, v, k, &a, &b)) return;  // all tie: next round
      set_rank(lo, a, a - 1);
      if (b < hi) set_rank(a, b, b - 1);
      if (b - a == 1) done[a] = 1;
      if (a - lo <= hi - b) {  // the equal part waits for the next round
        if (lo < a) refine(lo, a, h, limit);
        lo = b;
      } else {
        if (b < hi) refine(b, hi, h, limit);
        hi = a;
      }
    }
  }

  const Root& R;
  const i32 m;
  std::vector<i32>& sa_;
  std::vector<i32> isa;
  std::vector<uint8_t> tie, done;
  i64 budget = 0;
};

}  // namespace

int32_t root_bstar_count(const uint8_t* w, int32_t p) {
  if (!w || p < 2) throw CopyRankFailure();
  return Root(w, p, 1).q;
}

// Section 4: one B* offset per period (q = 1).  The bucket holds all k items: k - 1 first,
// then 0 .. k - 2.  Its first 1024-block (s0 items, item 0 at its front) ties at every one
// of the p characters of the substring stage, and each of those radix steps swaps the
// block's first item with its middle one; the merge keeps blocks in order.  The rank stage
// sees one group of k items that repeats at depth 1: a group of more than 8 swaps its first
// and middle slots once before the repeat ends it, and slot order is final.
int32_t copy_rank_single(const uint8_t* w, int32_t p, int32_t k) {
  if (root_bstar_count(w, p) != 1) return -1;
  const i32 s0 = std::min(k - 1, 1024);
  const i32 g = 1 + ((s0 > 8 && (p & 1)) ? s0 / 2 : 0);
  return (k > 8 && g == k / 2) ? 0 : g;
}

int32_t copy_rank(const uint8_t* w, int32_t p, int32_t k) {
  if (!w || p < 2 || k < 2) throw CopyRankFailure();
  const Root R(w, p, k);
  const i32 m = R.m;
  // bucket layout: buckets in (c0, c1) order, ascending items, item m - 1 first in its bucket
  std::vector<i32> cls(R.q);
  for (i32 c = 0; c < R.q; c++) cls[c] = c;
  std::stable_sort(cls.begin(), cls.end(), [&](i32 x, i32 y) { return R.bucket(x) < R.bucket(y); });
  std::vector<i32> sa;
  sa.reserve(m);
  std::vector<std::pair<i32, i32>> buckets;
  for (i32 i = 0; i < R.q;) {
    i32 j = i;
    while (j < R.q && R.bucket(cls[j]) == R.bucket(cls[i])) ++j;
    const i32 lo = (i32)sa.size();
    std::vector<uint8_t> in(R.q, 0);
    for (i32 t = i; t < j; t++) in[cls[t]] = 1;
    if (in[R.q - 1]) sa.push_back(m - 1);
    for (i32 x = 0; x < m - 1; x++)
      if (in[x % R.q]) sa.push_back(x);
    buckets.push_back({lo, (i32)sa.size()});
    i = j;
  }
  SubstringStage ss(R, sa);
  // merge scratch: the reference's work array beyond the buckets (n - 2m slots) or a
  // 256-slot array; its content never reaches the order, only its size matters
  const i64 n = (i64)p * k;
  const i32 bufsize = n - 2 * (i64)m > 256 ? (i32)(n - 2 * (i64)m) : 256;
  std::vector<i32> scratch(std::min<i64>(bufsize, m) + 1, 0);
  for (auto& b : buckets)
    if (b.second - b.first > 1) ss.bucket(b.first, b.second, bufsize, scratch.data());
  RankStage rs(R, sa);
  rs.init_groups(ss);
  rs.run();
  // r = rank of copy 0 of class 0 among its k copies (items 0, q, 2q, ...)
  i32 r = 0;
  for (i32 c = 1; c < R.k; c++) r += rs.rank(c * R.q) < rs.rank(0);
  return r;
}

int32_t root_rotation_rank(const uint8_t* w, int32_t p) {
  i32 r = 0;
  for (i32 i = 1; i < p; i++) {
    i32 x = 0;
    while (x < p && w[(i + x) % p] == w[x]) x++;
    if (x < p && w[(i + x) % p] < w[x]) r++;
  }
  return r;
}

int32_t primitive_period(const uint8_t* t, int32_t n) {
  // smallest p | n with t[i] = t[i - p]: from the prefix function of t
  if (n <= 1) return n;
  std::vector<i32> pi(n, 0);
  for (i32 i = 1; i < n; i++) {
    i32 j = pi[i - 1];
    while (j > 0 && t[i] != t[j]) j = pi[j - 1];
    if (t[i] == t[j]) ++j;
    pi[i] = j;
  }
  const i32 p = n - pi[n - 1];
  return n % p == 0 ? p : n;
}

}  // namespace bzg
